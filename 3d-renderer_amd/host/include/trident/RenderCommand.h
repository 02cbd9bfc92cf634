// RenderCommand.h — the static facade Trident-Forge drives the renderer through
// (Trident/src/Renderer/RenderCommand.h:11-84), restricted to the draw path. Each call forwards to
// the process-wide renderer (Startup::GetRenderer(), Application/Startup.h:38) — here
// RenderCommand::GetRenderer(). AI / recording / text / gizmo entry points are outside the path.
#pragma once

#include <string>
#include <vector>

#include "Renderer.h"

namespace Trident {

class RenderCommand {
public:
    static Renderer& GetRenderer();  // stands in for Startup::GetRenderer()

    static void Init() { GetRenderer().Init(); }
    static void Shutdown() { GetRenderer().Shutdown(); }
    static void DrawFrame() { GetRenderer().DrawFrame(); }
    static void SetViewport(uint32_t viewportId, const ViewportInfo& info) { GetRenderer().SetViewport(viewportId, info); }
    static void SetClearColor(const glm::vec4& color) { GetRenderer().SetClearColor(color); }
    static void AppendMeshes(std::vector<Geometry::Mesh> meshes, std::vector<Geometry::Material> materials,
                             std::vector<std::string> textures) {
        GetRenderer().AppendMeshes(std::move(meshes), std::move(materials), std::move(textures));
    }
    static void UploadMesh(const std::vector<Geometry::Mesh>& meshes, const std::vector<Geometry::Material>& materials,
                           const std::vector<std::string>& textures) {
        GetRenderer().UploadMesh(meshes, materials, textures);
    }
    static void SetEditorCamera(Camera* camera) { GetRenderer().SetEditorCamera(camera); }
    static void SetRuntimeCamera(Camera* camera) { GetRenderer().SetRuntimeCamera(camera); }
    static void SetRuntimeCameraReady(bool ready) { GetRenderer().SetRuntimeCameraReady(ready); }
    static void SetActiveRegistry(ECS::Registry* registry) { GetRenderer().SetActiveRegistry(registry); }
    static bool HasRuntimeCamera() { return GetRenderer().HasRuntimeCamera(); }
    static ViewportInfo GetViewport() { return GetRenderer().GetViewport(); }
    static void* GetViewportTexture(uint32_t viewportId) { return GetRenderer().GetViewportTexture(viewportId); }
    static glm::mat4 GetViewportViewMatrix(uint32_t id) { return GetRenderer().GetViewportViewMatrix(id); }
    static glm::mat4 GetViewportProjectionMatrix(uint32_t id) { return GetRenderer().GetViewportProjectionMatrix(id); }
    static glm::vec4 GetClearColor() { return GetRenderer().GetClearColor(); }
    static FrameTimingStats GetFrameTimingStats() { return GetRenderer().GetFrameTimingStats(); }
    static size_t GetModelCount() { return GetRenderer().GetModelCount(); }
    static int32_t ResolveTextureSlot(const std::string& texturePath) { return GetRenderer().ResolveTextureSlot(texturePath); }
    static size_t GetOrCreatePrimitiveMeshIndex(MeshComponent::PrimitiveType primitiveType) {
        return GetRenderer().GetOrCreatePrimitiveMeshIndex(primitiveType);
    }
};

}  // namespace Trident
