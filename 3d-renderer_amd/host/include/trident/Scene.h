// Scene.h — the data Trident's renderer pulls each frame, with the reference's names and defaults:
// Vertex (Trident/src/Renderer/Vertex.h:9-78), Geometry::Mesh / Material (Geometry/Mesh.h:12-17,
// Material.h:10-19), the ECS components (ECS/Components/*.h) and the unordered_map-per-type
// ECS::Registry (ECS/Registry.h:27-205).
#pragma once

#include <algorithm>
#include <cstdint>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <typeindex>
#include <unordered_map>
#include <vector>

#include "glm_subset.h"

struct Vertex {
    static constexpr uint32_t MaxBoneInfluences = 4;
    glm::vec3 Position;
    glm::vec3 Normal;
    glm::vec3 Tangent;
    glm::vec3 Bitangent;
    glm::vec3 Color;
    glm::vec2 TexCoord;
    glm::ivec4 m_BoneIndices{0};
    glm::vec4 m_BoneWeights{0.0f};
};
static_assert(sizeof(Vertex) == 100, "Vertex must keep Trident's 100-byte stride");

namespace Trident {

namespace Geometry {
struct Material {
    glm::vec4 BaseColorFactor{1.0f, 1.0f, 1.0f, 1.0f};
    float MetallicFactor = 1.0f;
    float RoughnessFactor = 1.0f;
    int BaseColorTextureIndex = -1;
    int BaseColorTextureSlot = 0;
    int MetallicRoughnessTextureIndex = -1;
    int NormalTextureIndex = -1;
};

struct Mesh {
    std::vector<Vertex> Vertices;
    std::vector<uint32_t> Indices;
    int MaterialIndex = -1;
};
}  // namespace Geometry

namespace Loader {
struct TextureData {  // TextureLoader output: RGBA8 (forced 4 channels), rows already flipped
    int Width = 0;
    int Height = 0;
    int Channels = 4;
    std::vector<uint8_t> Pixels;
};
// CubemapTextureData (Loader/TextureLoader.h:30-48), LDR subset: 6 faces +X,-X,+Y,-Y,+Z,-Z of
// m_Width x m_Height RGBA8 sRGB texels, one mip, stored face after face.
struct CubemapTextureData {
    uint32_t m_Width = 0;
    uint32_t m_Height = 0;
    uint32_t m_MipCount = 1;
    std::vector<uint8_t> m_PixelData;
    bool IsValid() const {
        return m_Width > 0 && m_Width == m_Height && m_PixelData.size() >= 6ull * m_Width * m_Height * 4;
    }
    static CubemapTextureData CreateSolidColor(uint32_t rgba8888) {  // TextureLoader.cpp:309-330
        CubemapTextureData d;
        d.m_Width = d.m_Height = 1;
        d.m_PixelData.resize(24);
        for (int f = 0; f < 6; ++f)
            for (int b = 0; b < 4; ++b) d.m_PixelData[4 * f + b] = (uint8_t)(rgba8888 >> (8 * b));  // little-endian memcpy
        return d;
    }
};
}  // namespace Loader

struct Transform {
    glm::vec3 Position{0.0f};
    glm::vec3 Rotation{0.0f};  // Euler degrees
    glm::vec3 Scale{1.0f};
};

struct MeshComponent {
    enum class PrimitiveType { None, Cube, Sphere, Quad };
    size_t m_MeshIndex{std::numeric_limits<size_t>::max()};
    int32_t m_MaterialIndex{-1};
    uint32_t m_FirstIndex{0};
    uint32_t m_IndexCount{0};
    int32_t m_BaseVertex{0};
    bool m_Visible{true};
    PrimitiveType m_Primitive{PrimitiveType::None};
    std::string m_SourceAssetPath{};
    size_t m_SourceMeshIndex{0};
};

struct TextureComponent {
    std::string m_TexturePath{};
    int32_t m_TextureSlot{-1};
    bool m_IsDirty{true};
};

struct LightComponent {
    enum class Type : uint32_t { Directional = 0, Point = 1 };
    Type m_Type = Type::Directional;
    glm::vec3 m_Color{1.0f, 0.98f, 0.92f};
    float m_Intensity = 5.0f;
    glm::vec3 m_Direction{-0.5f, -1.0f, -0.3f};
    float m_Range = 10.0f;
    bool m_Enabled = true;
    bool m_ShadowCaster = false;
    bool m_Reserved0 = false;
    bool m_Reserved1 = false;
};

// SpriteComponent (ECS/Components/SpriteComponent.h:17-43): a camera-independent unit quad drawn with the
// Default pipeline after the meshes (Renderer.cpp:2996-3089, :5154-5157). The atlas / animation fields are
// authoring data the renderer does not read yet (the reference's DrawSprites ignores them too).
struct SpriteComponent {
    std::string m_TextureId{};
    glm::vec4 m_TintColor{1.0f};
    glm::vec2 m_UVScale{1.0f};
    glm::vec2 m_UVOffset{0.0f};
    float m_TilingFactor{1.0f};
    bool m_Visible{true};
    bool m_UseMaterialOverride{false};
    std::string m_MaterialOverrideId{};
    int32_t m_AtlasTiles[2]{1, 1};
    int m_AtlasIndex{0};
    float m_AnimationSpeed{0.0f};
    float m_SortOffset{0.0f};
};

// AnimationComponent (ECS/Components/AnimationComponent.h:29-73), the part the renderer reads: the
// skinning palette the CPU animation system writes each frame (m_BoneMatrices, column-major mat4s).
// Clip/skeleton bookkeeping stays with the animation system, which is outside the hot path.
struct AnimationComponent {
    std::vector<glm::mat4> m_BoneMatrices{};
};

struct TagComponent {
    std::string m_Tag;
};

namespace ECS {
using Entity = uint32_t;

class Registry {
public:
    Entity CreateEntity() {
        const Entity e = m_Next++;
        m_ActiveEntities.push_back(e);
        return e;
    }
    void DestroyEntity(Entity entity) {
        for (auto& it : m_Storages) it.second->Remove(entity);
        m_ActiveEntities.erase(std::remove(m_ActiveEntities.begin(), m_ActiveEntities.end(), entity),
                               m_ActiveEntities.end());
    }
    void Clear() {
        for (auto& it : m_Storages) it.second->Clear();
        m_ActiveEntities.clear();
    }
    template <typename T, typename... Args>
    T& AddComponent(Entity entity, Args&&... args) {
        return Storage<T>().Emplace(entity, T{std::forward<Args>(args)...});
    }
    template <typename T>
    bool HasComponent(Entity entity) const {
        auto it = m_Storages.find(std::type_index(typeid(T)));
        return it != m_Storages.end() && static_cast<const ComponentStorage<T>*>(it->second.get())->Has(entity);
    }
    template <typename T>
    T& GetComponent(Entity entity) {
        return Storage<T>().Get(entity);
    }
    template <typename T>
    const T& GetComponent(Entity entity) const {
        auto it = m_Storages.find(std::type_index(typeid(T)));
        if (it == m_Storages.end()) throw std::out_of_range("component not present");
        return static_cast<const ComponentStorage<T>*>(it->second.get())->Get(entity);
    }
    template <typename T>
    void RemoveComponent(Entity entity) {
        Storage<T>().Remove(entity);
    }
    const std::vector<Entity>& GetEntities() const { return m_ActiveEntities; }

private:
    struct IComponentStorage {
        virtual ~IComponentStorage() = default;
        virtual void Remove(Entity) = 0;
        virtual void Clear() = 0;
    };
    template <typename T>
    struct ComponentStorage : IComponentStorage {
        std::unordered_map<Entity, T> m_Components;
        T& Emplace(Entity e, T value) {
            auto r = m_Components.emplace(e, value);
            if (!r.second) r.first->second = std::move(value);
            return r.first->second;
        }
        bool Has(Entity e) const { return m_Components.find(e) != m_Components.end(); }
        T& Get(Entity e) { return m_Components.at(e); }
        const T& Get(Entity e) const { return m_Components.at(e); }
        void Remove(Entity e) override { m_Components.erase(e); }
        void Clear() override { m_Components.clear(); }
    };
    template <typename T>
    ComponentStorage<T>& Storage() {
        auto& p = m_Storages[std::type_index(typeid(T))];
        if (!p) p = std::make_unique<ComponentStorage<T>>();
        return *static_cast<ComponentStorage<T>*>(p.get());
    }
    std::unordered_map<std::type_index, std::unique_ptr<IComponentStorage>> m_Storages;
    std::vector<Entity> m_ActiveEntities;
    Entity m_Next = 0;
};
}  // namespace ECS

}  // namespace Trident
