// SceneFile.h — the `.trident` scene text format (Trident/src/ECS/Scene.cpp:80-151 save/load,
// :288-430 SerializeEntity, :432-961 DeserializeEntity, :963-1081 RebuildMeshAssetsFromComponents)
// and Forge's model import (ApplicationLayer::ImportDroppedAssets, ApplicationLayer.cpp:815-1031),
// restricted to the components the draw path reads: Tag, UUID, Transform, Camera, Mesh (with the
// SourceAsset provenance that rebuilds geometry on load), Sprite (Scene.cpp:343-367, :549-779), Texture
// and Light. Animation and Script lines are recognised and skipped (their subsystems are outside the hot
// path), including an Animation component's trailing AnimationBones line.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "Camera.h"
#include "Renderer.h"
#include "Scene.h"

namespace Trident {

struct UUIDComponent {
    uint64_t m_ID = 0;
};

struct CameraComponent {  // ECS/Components/CameraComponent.h:16-26
    Camera::ProjectionType m_ProjectionType{Camera::ProjectionType::Perspective};
    float m_FieldOfView{60.0f};
    float m_OrthographicSize{20.0f};
    float m_NearClip{0.1f};
    float m_FarClip{1000.0f};
    bool m_Primary{false};
    bool m_FixedAspectRatio{false};
    float m_AspectRatio{16.0f / 9.0f};
};

class Scene {
public:
    // `renderer` receives the rebuilt geometry on Load (Startup::GetRenderer() in the reference);
    // null skips the upload, as the reference does without a Startup instance (Scene.cpp:1074-1077).
    Scene(ECS::Registry& registry, Renderer* renderer, std::string name = "Untitled");

    void Save(const std::string& path) const;
    // Clears the registry, reads the entities, rebuilds imported meshes. False if the file cannot be
    // opened (the registry is left untouched then).
    bool Load(const std::string& path);
    void RebuildMeshAssetsFromComponents();

    const std::string& GetName() const { return m_SceneName; }
    void SetName(const std::string& name) { m_SceneName = name; }
    size_t GetLoadedEntityCount() const { return m_LoadedEntityCount; }

    static std::string EscapeString(const std::string& value);
    static std::string UnescapeString(const std::string& value);

private:
    void SerializeEntity(std::ostream& stream, ECS::Entity entity) const;
    void DeserializeEntity(std::istream& stream);

    ECS::Registry& m_Registry;
    Renderer* m_Renderer;
    std::string m_SceneName;
    size_t m_LoadedEntityCount = 0;
};

// Forge's drop import for one model file: ModelLoader, entities per mesh instance (or one per mesh at
// identity) with decomposed Transform + MeshComponent{SourceAsset, SourceMeshIndex} + Tag, then
// Renderer::AppendMeshes. Returns false when nothing was imported.
bool ImportModel(Renderer& renderer, ECS::Registry& registry, const std::string& path,
                 std::vector<ECS::Entity>* spawned = nullptr);

}  // namespace Trident
