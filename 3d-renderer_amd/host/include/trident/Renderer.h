// Renderer.h — Trident::Renderer, the reference's renderer API (Trident/src/Renderer/Renderer.h:77-598)
// for the draw path, backed by the HIP software rasterizer through the C-ABI (include/tri_raster.h)
// instead of Vulkan. Same names, argument meaning and error behaviour (no exceptions on the frame
// path; failures are logged and the frame is skipped, Renderer.cpp:779-824). Vulkan-typed getters
// become opaque device pointers (GetViewportTexture).
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../../include/tri_raster.h"
#include "Camera.h"
#include "Scene.h"

namespace Trident {

struct ViewportInfo {
    uint32_t ViewportID = 0;
    glm::vec2 Position{0.0f};
    glm::vec2 Size{0.0f};
};

struct FrameTimingSample {
    double FrameMilliseconds = 0.0;
    double FramesPerSecond = 0.0;
    std::chrono::system_clock::time_point CaptureTime{};
};

struct FrameTimingStats {  // Renderer.h:472-479
    double MinimumMilliseconds = 0.0;
    double MaximumMilliseconds = 0.0;
    double AverageMilliseconds = 0.0;
    double MinimumFPS = 0.0;
    double MaximumFPS = 0.0;
    double AverageFPS = 0.0;  // mean of per-frame 1000/ms (Renderer.cpp:6335-6342)
};

class Renderer {
public:
    Renderer();
    ~Renderer();

    void Init();
    void Shutdown();
    void DrawFrame();

    void UploadMesh(const std::vector<Geometry::Mesh>& meshes, const std::vector<Geometry::Material>& materials,
                    const std::vector<std::string>& textures);
    void AppendMeshes(std::vector<Geometry::Mesh> meshes, std::vector<Geometry::Material> materials,
                      std::vector<std::string> textures);
    void UploadTexture(const std::string& texturePath, const Loader::TextureData& texture);
    void SetEditorCamera(Camera* camera) { m_EditorCamera = camera; }
    void SetRuntimeCamera(Camera* camera) { m_RuntimeCamera = camera; }
    void SetRuntimeCameraReady(bool ready) { m_RuntimeCameraReady = ready; }
    void SetActiveRegistry(ECS::Registry* registry) { m_Registry = registry; }
    bool HasRuntimeCamera() const { return m_RuntimeCamera != nullptr && m_RuntimeCameraReady; }

    int32_t ResolveTextureSlot(const std::string& texturePath);
    size_t GetOrCreatePrimitiveMeshIndex(MeshComponent::PrimitiveType primitiveType);

    void SetClearColor(const glm::vec4& color) { m_ClearColor = color; }
    // The AI frame blend of Default.frag (:182-191). SetAiBlendStrength clamps to [0, 1] (Renderer.cpp:2533-2538,
    // default 0.35, Renderer.h:508). SubmitAiInterpolation takes a generated frame the way UploadAiInterpolationToGpu
    // does (Renderer.cpp:1560-1700): width * height * channels floats, each clamped to [0, 1] and rounded to a UNORM8
    // byte, alpha 1 when the frame has fewer than four channels; every viewport then blends with it (UpdateUniformBuffer
    // packs AiBlendConfig = (strength, 1 / width, 1 / height, 1) while a frame is held, :5916-5921). nullptr or an
    // empty frame drops it (the blend is off again). The frame generator (ONNX Runtime) itself stays outside.
    void SetAiBlendStrength(float blendStrength) { m_AiBlendStrength = std::min(std::max(blendStrength, 0.0f), 1.0f); }
    float GetAiBlendStrength() const { return m_AiBlendStrength; }
    bool SubmitAiInterpolation(const float* pixels, uint32_t width, uint32_t height, uint32_t channels);
    bool HasAiFrame() const { return m_AiWidth != 0 && m_AiHeight != 0; }
    // Replaces the skybox cubemap (CreateSkyboxCubemap, Renderer.cpp:3818-4110). Init installs the
    // reference's fallback, a solid 0x808080 cubemap (:3925-3926). An invalid cubemap is rejected
    // and logged; returns false in that case.
    bool SetSkyboxCubemap(const Loader::CubemapTextureData& cubemap);
    // Where CreateSkyboxCubemap looks for Skyboxes/ (the reference: "Assets", next to the executable,
    // Renderer.cpp:3830). Changing it re-runs the discovery; GetSkyboxSource names what was loaded
    // ("PNG fallback", "Default directory", ... or "solid 0x808080").
    void SetAssetsDirectory(const std::string& directory);
    const std::string& GetSkyboxSource() const { return m_SkyboxSource; }
    glm::vec4 GetClearColor() const { return m_ClearColor; }

    size_t GetModelCount() const { return m_ModelCount; }
    size_t GetTriangleCount() const { return m_TriangleCount; }
    const FrameTimingStats& GetFrameTimingStats() const { return m_PerformanceStats; }
    size_t GetFrameTimingHistoryCount() const { return m_PerformanceSampleCount; }

    void SetViewport(uint32_t viewportId, const ViewportInfo& info);  // also makes it the active viewport
    // Swapchain extent stand-in (Swapchain.cpp): when set, DrawFrame ends by blitting the active
    // viewport onto a present image of this size with linear filtering (Renderer.cpp:5346-5361). With no
    // active viewport rendered this frame (none registered, or the active one has no target), it renders
    // the skybox, meshes and sprites straight into the present image at this extent instead — the legacy
    // direct-to-swapchain path (Renderer.cpp:5233, :5498-5590), camera from GetActiveCamera().
    void SetPresentExtent(uint32_t width, uint32_t height) { m_PresentWidth = width; m_PresentHeight = height; }
    // The last presented image (RGBA8 rows, BGRA reordered) and its size; false before a present.
    bool ReadPresentPixels(std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height);
    // Wait for the frame the last DrawFrame submitted (its viewport passes and present blit), re-rendering a pass
    // that outgrew the internal queues. DrawFrame itself calls it first, for the previous frame — the reference waits
    // for the previous frame's timeline value at the start of DrawFrame (Renderer.cpp:752-772) — so the caller's host
    // work between frames overlaps the GPU. The readers (ReadViewportPixels, ReadPresentPixels, GetViewportTexture)
    // call it on demand.
    void FinishFrame();
    // Frames in flight (1..4; default 1, the reference's pacing: DrawFrame waits for the previous frame's timeline
    // value). With n > 1 every single-device viewport keeps n render targets and frame k renders into target k mod n,
    // so DrawFrame waits only for frame k - n + 1 and the next frames' vertex and set-up work overlaps this frame's
    // raster (the C-ABI bench's contexts in flight, through the engine API). GetViewportTexture / ReadViewportPixels
    // return the latest frame's target. Multi-device viewports (SetDeviceCount > 1) keep 1 (tri_group double-buffers
    // its own frame). Changing it waits for every frame in flight and rebuilds the targets at the next DrawFrame.
    void SetFramesInFlight(uint32_t n);
    uint32_t GetFramesInFlight() const { return m_FramesInFlight; }
    uint32_t GetActiveViewportId() const { return m_ActiveViewportId; }
    ViewportInfo GetViewport() const;
    // Vulkan returned a VkDescriptorSet for ImGui (Renderer.h:235); here: an opaque handle, a pointer to
    // the viewport's tri_image (device pointer, size, pitch, B8G8R8A8_UNORM, device ordinal) that an ImGui
    // HIP/GL-interop backend can display. nullptr before the viewport's first frame; valid until its next
    // resize or Shutdown.
    void* GetViewportTexture(uint32_t viewportId) const;
    // Shadow-map pre-pass (BASELINE config 5): the reference reserves LightComponent::m_ShadowCaster
    // (LightComponent.h:33) without rendering shadows; here, when the directional light UpdateUniformBuffer
    // picks (the first enabled one) is a shadow caster, every viewport renders a size x size map fitted
    // to the visible draws' world box (tri_shadow_fit_ortho) first. 0 disables the pass entirely.
    void SetShadowMapSize(uint32_t size) { m_ShadowMapSize = size; }
    // The pre-pass configuration DrawFrame uses this frame (false: no shadow-casting sun).
    bool BuildShadowConfig(tri_shadow_config& out);
    // How many times the concatenated geometry went to the device: once per UploadMeshFromCache
    // generation, shared by every viewport (the reference binds one vertex/index buffer for all).
    uint64_t GetGeometryUploadCount() const { return m_GeometryUploads; }
    const Camera* GetActiveCamera() const;
    glm::mat4 GetViewportViewMatrix(uint32_t viewportId) const;
    glm::mat4 GetViewportProjectionMatrix(uint32_t viewportId) const;

    std::vector<Geometry::Material>& GetMaterials() { return m_Materials; }
    const std::vector<Geometry::Material>& GetMaterials() const { return m_Materials; }

    // Frame readback (ResolvePendingReadback, Renderer.cpp:1299-1389): RGBA8 rows of the viewport
    // (BGRA reordered to RGBA), optionally the D32 depth.
    bool ReadViewportPixels(uint32_t viewportId, std::vector<uint8_t>& rgba, std::vector<float>* depth = nullptr);
    // The exact uniform block + draw list DrawFrame submits for a viewport (GatherMeshDraws +
    // UpdateUniformBuffer + the push-constant loop): host-only, used to test frame preparation. Id 0 with
    // no viewport registered: the legacy present pass's inputs (GetActiveCamera()).
    bool BuildFrameInputs(uint32_t viewportId, tri_global_ubo& ubo, std::vector<tri_draw>& draws);
    // Rasterizer flags (TRI_FLAG_*) used for viewports created from now on.
    void SetRasterFlags(uint32_t flags) { m_RasterFlags = flags; }
    // Multi-device viewports (SURVEY 8(b) tri_config.device_count, 8(e)): with count > 1 every viewport
    // renders as a tri_group of `count` row bands on `devices` (default 0 .. count-1; an ordinal may
    // repeat), the frame assembled on the first band's device over RCCL; count <= 1 is one context per
    // viewport (the default). Existing viewport targets are rebuilt at the next DrawFrame. The geometry
    // goes to each distinct device once per generation and is shared by every viewport there. Returns
    // false (and changes nothing) for an invalid device list.
    bool SetDeviceCount(uint32_t count, const std::vector<int32_t>& devices = {});
    uint32_t GetDeviceCount() const { return (uint32_t)std::max<size_t>(m_Devices.size(), 1); }
    bool IsShutdown() const { return m_Shutdown; }
    // The concatenated buffers UploadMeshFromCache builds (the device copy of these is what
    // tri_upload_geometry receives).
    const std::vector<tri_vertex>& GetVertexBuffer() const { return m_VertexBuffer; }
    const std::vector<uint32_t>& GetIndexBuffer() const { return m_IndexBuffer; }
    std::vector<tri_mesh_range> GetMeshRanges() const;

private:
    struct MeshDrawInfo {  // Renderer.h:293-299
        uint32_t m_FirstIndex = 0;
        uint32_t m_IndexCount = 0;
        int32_t m_BaseVertex = 0;
        int32_t m_MaterialIndex = -1;
    };
    struct MeshDrawCommand {
        glm::mat4 m_ModelMatrix{1.0f};
        const MeshComponent* m_Component = nullptr;
        const TextureComponent* m_TextureComponent = nullptr;
        const AnimationComponent* m_AnimationComponent = nullptr;
        uint32_t m_BoneOffset = 0;
        uint32_t m_BoneCount = 0;
        ECS::Entity m_Entity = 0;
    };
    struct SpriteDrawCommand {  // Renderer.h SpriteDrawCommand: one visible SpriteComponent per frame
        glm::mat4 m_ModelMatrix{1.0f};
        const SpriteComponent* m_Component = nullptr;
        const TextureComponent* m_TextureComponent = nullptr;
        ECS::Entity m_Entity = 0;
    };
    struct ViewportContext {
        ViewportInfo m_Info{};
        tri_ctx* m_Ctx = nullptr;      // one-device viewport
        tri_group* m_Group = nullptr;  // multi-device viewport (SetDeviceCount > 1)
        uint32_t m_Width = 0, m_Height = 0;
        uint64_t m_GeometryGeneration = 0, m_TextureGeneration = 0, m_MaterialGeneration = 0, m_SkyboxGeneration = 0;
        uint64_t m_AiGeneration = 0;
        std::vector<float> m_BonePalette;  // the palette last uploaded to this viewport's context
        tri_shadow_config m_Shadow{};      // the pre-pass configuration last set on this context
        tri_image m_Image{};               // GetViewportTexture's handle (after the first frame)
        bool m_HasImage = false;
    };

    void CreateSkyboxCubemap();
    void UploadMeshFromCache();
    void EnsurePrimitiveMeshesInCache();
    size_t CreatePrimitiveMeshInCache(MeshComponent::PrimitiveType primitiveType);
    void ResolveMaterialTextureSlots(const std::vector<std::string>& textures, size_t offset, size_t count);
    void GatherMeshDraws();
    void GatherSpriteDraws();
    void GatherDraws();  // GatherMeshDraws + GatherSpriteDraws (adds the sprite quad to the geometry once)
    void PrepareBonePaletteBuffer();
    void UpdateUniformBuffer(const Camera* camera, tri_global_ubo& out) const;
    void BuildDrawList(std::vector<tri_draw>& out) const;
    const Camera* GetActiveCamera(const ViewportContext& context) const;
    bool PrepareViewport(ViewportContext& context);
    // One viewport pass: pre-pass / palette / UBO / draws, then tri_render (asynchronous); false on error.
    bool SubmitTarget(ViewportContext& context, const tri_global_ubo& ubo, const std::vector<tri_draw>& draws,
                      const tri_shadow_config& shadow, bool shadowOn);
    void RecordFrameTiming(double milliseconds);

    Camera* m_EditorCamera = nullptr;
    Camera* m_RuntimeCamera = nullptr;
    bool m_RuntimeCameraReady = false;
    ECS::Registry* m_Registry = nullptr;

    std::vector<Geometry::Mesh> m_GeometryCache;
    std::vector<Geometry::Material> m_Materials;
    std::vector<MeshDrawInfo> m_MeshDrawInfo;
    std::vector<MeshDrawCommand> m_MeshDrawCommands;
    std::vector<SpriteDrawCommand> m_SpriteDrawList;
    // The sprite quad (BuildSpriteGeometry, Renderer.cpp:2853-2890): the reference keeps it in its own
    // vertex/index buffer; here it is one more mesh range after the cached meshes, appended to the
    // device geometry the first time a sprite is drawn (mesh index m_MeshDrawInfo.size()).
    bool m_HasSpriteGeometry = false;
    MeshDrawInfo m_SpriteDrawInfo{};
    static constexpr uint32_t s_MaxBonesPerSkeleton = 128;  // Renderer.h:291
    std::vector<float> m_BonePalette;  // PrepareBonePaletteBuffer's scratch: per-draw palettes, back to back
    size_t m_PrimitiveMeshIndices[3] = {SIZE_MAX, SIZE_MAX, SIZE_MAX};
    bool m_IsUploadingMeshes = false;
    tri_geometry* m_SharedGeometry = nullptr;  // the device copy every viewport context binds
    uint64_t m_SharedGeometryGeneration = 0;
    std::vector<int32_t> m_Devices;                 // SetDeviceCount's bands (empty: one context per viewport)
    std::vector<tri_geometry*> m_DeviceGeometry;    // multi-device: one shared copy per distinct device
    std::vector<uint64_t> m_DeviceGeometryGeneration;
    bool UploadSharedGeometry(std::vector<tri_geometry*>& out);
    void DestroyViewportTargets();
    uint64_t m_GeometryUploads = 0;
    std::vector<glm::vec3> m_MeshBoundsMin, m_MeshBoundsMax;  // object-space box per cached mesh
    uint32_t m_ShadowMapSize = 2048;
    std::vector<tri_vertex> m_VertexBuffer;
    std::vector<uint32_t> m_IndexBuffer;
    uint64_t m_GeometryGeneration = 1, m_TextureGeneration = 1, m_MaterialGeneration = 1;
    Loader::CubemapTextureData m_SkyboxCubemap;
    std::string m_AssetsDirectory = "Assets";
    std::string m_SkyboxSource;
    uint64_t m_SkyboxGeneration = 1;
    std::vector<uint8_t> m_AiFrame;  // the AI frame's R8G8B8A8_UNORM bytes (SubmitAiInterpolation)
    uint32_t m_AiWidth = 0, m_AiHeight = 0;
    float m_AiBlendStrength = 0.35f;
    uint64_t m_AiGeneration = 1;

    struct TextureSlot {
        std::string m_SourcePath;
        Loader::TextureData m_Data;
    };
    std::vector<TextureSlot> m_TextureSlots;
    std::unordered_map<std::string, uint32_t> m_TextureSlotLookup;

    std::map<uint32_t, ViewportContext> m_Viewports;
    ViewportInfo m_LastViewport{};
    uint32_t m_ActiveViewportId = 0;
    uint32_t m_PresentWidth = 0, m_PresentHeight = 0;
    tri_ctx* m_PresentSource = nullptr;    // viewport context the last present was blitted from
    tri_group* m_PresentGroup = nullptr;   // ... or multi-device viewport
    ViewportContext m_LegacyTarget;        // the legacy path's present-extent target (no active viewport)
    bool m_PresentLegacy = false;          // the last present was rendered directly (legacy path), not blitted
    // the extent the last present was produced at (SetPresentExtent may change before ReadPresentPixels)
    uint32_t m_PresentedWidth = 0, m_PresentedHeight = 0;
    uint32_t m_RasterFlags = 0;
    struct PendingFrame {  // what a DrawFrame submitted and no fence has waited for yet
        std::vector<ViewportContext*> m_Targets;
        ViewportContext* m_Legacy = nullptr;  // the legacy present target among them
        ViewportContext* m_Blit = nullptr;    // the primary viewport target whose present blit was enqueued
        uint32_t m_BlitWidth = 0, m_BlitHeight = 0;
    };
    std::deque<PendingFrame> m_Pending;  // oldest first; at most m_FramesInFlight
    void FinishOldestFrame();
    // frames in flight: viewport id -> its targets 1 .. n-1 (target 0 is the m_Viewports entry), and the target of its
    // latest frame
    uint32_t m_FramesInFlight = 1;
    uint64_t m_FrameCount = 0;
    std::map<uint32_t, std::vector<ViewportContext>> m_RingTargets;
    std::map<uint32_t, uint32_t> m_LatestTarget;
    ViewportContext& TargetOf(uint32_t viewportId, ViewportContext& primary, uint32_t index);
    const ViewportContext* LatestTarget(uint32_t viewportId) const;

    glm::vec3 m_AmbientColor{0.03f};
    float m_AmbientIntensity = 1.0f;
    glm::vec4 m_ClearColor{0.005f, 0.005f, 0.005f, 1.0f};
    size_t m_ModelCount = 0;
    size_t m_TriangleCount = 0;

    static constexpr size_t s_PerformanceHistorySize = 240;
    std::vector<FrameTimingSample> m_PerformanceHistory;
    size_t m_PerformanceHistoryNextIndex = 0;
    size_t m_PerformanceSampleCount = 0;
    FrameTimingStats m_PerformanceStats{};
    bool m_Initialised = false;
    bool m_Shutdown = false;
};

}  // namespace Trident
