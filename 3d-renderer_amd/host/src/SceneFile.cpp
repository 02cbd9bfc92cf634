// SceneFile.cpp — `.trident` save / load and model import (see SceneFile.h).
#include "trident/SceneFile.h"

#include <cstdio>
#include <filesystem>
#include <fstream>
#include <iomanip>
#include <limits>
#include <sstream>
#include <unordered_map>

#include "trident/ModelLoader.h"

namespace Trident {

namespace {

constexpr size_t kInvalidMesh = std::numeric_limits<size_t>::max();

void Warn(const std::string& what) { std::fprintf(stderr, "[Trident][Scene] %s\n", what.c_str()); }

std::string NormalizePath(const std::string& path) {  // Utilities.cpp:390-394
    return std::filesystem::path(path).lexically_normal().generic_string();
}

// Scene::ExtractQuotedToken (Scene.cpp:1160-1171): between the FIRST and the LAST quote of the line.
std::string ExtractQuotedToken(const std::string& line) {
    const size_t a = line.find('"'), b = line.find_last_of('"');
    if (a == std::string::npos || b == std::string::npos || b <= a) return {};
    return Scene::UnescapeString(line.substr(a + 1, b - a - 1));
}

bool StartsWith(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

// Scene.cpp:549-779: each "Key=" token runs to the next space; an absent token keeps the default, a
// malformed one warns and keeps what was parsed before the failure (istream semantics).
std::string SpriteToken(const std::string& line, const std::string& key) {
    const size_t k = line.find(key);
    if (k == std::string::npos) return {};
    const size_t a = k + key.size();
    size_t b = line.find(' ', a);
    if (b == std::string::npos) b = line.size();
    return line.substr(a, b - a);
}

template <typename T>
bool ParseList(const std::string& v, T* out, int n) {  // "x,y[,z,w]"
    if (v.empty()) return true;
    std::istringstream ts(v);
    for (int i = 0; i < n; ++i) {
        char comma = ',';
        if (i > 0 && (!(ts >> comma) || comma != ',')) return false;
        if (!(ts >> out[i])) return false;
    }
    return true;
}

bool ParseBoolToken(const std::string& v, bool& out) {
    if (v.empty()) return true;
    std::istringstream ts(v);
    if (ts >> std::boolalpha >> out) return true;
    std::istringstream ti(v);
    int x = 0;
    if (ti >> x) {
        out = x != 0;
        return true;
    }
    return false;
}

SpriteComponent ParseSprite(const std::string& line) {
    SpriteComponent sp{};
    sp.m_TextureId = ExtractQuotedToken(line);
    auto warn = [](const char* what, const std::string& tok) { Warn(std::string("failed to parse sprite ") + what + " token '" + tok + "'"); };
    std::string t;
    if (!ParseList(t = SpriteToken(line, "Tint="), &sp.m_TintColor.x, 4)) warn("tint", t);
    if (!ParseList(t = SpriteToken(line, "UVScale="), &sp.m_UVScale.x, 2)) warn("UVScale", t);
    if (!ParseList(t = SpriteToken(line, "UVOffset="), &sp.m_UVOffset.x, 2)) warn("UVOffset", t);
    if (!ParseList(t = SpriteToken(line, "Tiling="), &sp.m_TilingFactor, 1)) warn("tiling", t);
    if (!ParseBoolToken(t = SpriteToken(line, "Visible="), sp.m_Visible)) warn("visibility", t);
    if (!ParseBoolToken(t = SpriteToken(line, "UseMaterialOverride="), sp.m_UseMaterialOverride)) warn("material override", t);
    const size_t m = line.find("Material=");
    if (m != std::string::npos) sp.m_MaterialOverrideId = ExtractQuotedToken(line.substr(m));
    if (!ParseList(t = SpriteToken(line, "AtlasTiles="), sp.m_AtlasTiles, 2)) warn("atlas tiles", t);
    if (!ParseList(t = SpriteToken(line, "AtlasIndex="), &sp.m_AtlasIndex, 1)) warn("atlas index", t);
    if (!ParseList(t = SpriteToken(line, "AnimationSpeed="), &sp.m_AnimationSpeed, 1)) warn("animation speed", t);
    if (!ParseList(t = SpriteToken(line, "SortOffset="), &sp.m_SortOffset, 1)) warn("sort offset", t);
    return sp;
}

}  // namespace

Scene::Scene(ECS::Registry& registry, Renderer* renderer, std::string name)
    : m_Registry(registry), m_Renderer(renderer), m_SceneName(std::move(name)) {}

std::string Scene::EscapeString(const std::string& value) {  // Scene.cpp:1083-1112
    std::string r;
    r.reserve(value.size());
    for (char c : value) {
        switch (c) {
            case '\\': r += "\\\\"; break;
            case '"': r += "\\\""; break;
            case '\n': r += "\\n"; break;
            case '\r': r += "\\r"; break;
            case '\t': r += "\\t"; break;
            default: r += c;
        }
    }
    return r;
}

std::string Scene::UnescapeString(const std::string& value) {  // Scene.cpp:1114-1158
    std::string r;
    r.reserve(value.size());
    for (size_t i = 0; i < value.size(); ++i) {
        const char c = value[i];
        if (c == '\\' && i + 1 < value.size()) {
            const char n = value[++i];
            switch (n) {
                case 'n': r += '\n'; break;
                case 'r': r += '\r'; break;
                case 't': r += '\t'; break;
                default: r += n;  // '\\', '"' and anything else: the character itself
            }
        } else {
            r += c;
        }
    }
    return r;
}

void Scene::Save(const std::string& path) const {  // Scene.cpp:80-103
    std::ofstream s(path, std::ios::trunc);
    if (!s.is_open()) {
        Warn("failed to open scene file '" + path + "' for writing");
        return;
    }
    s << "# Trident Scene\n";
    s << "Scene \"" << EscapeString(m_SceneName) << "\"\n";
    s << std::boolalpha;
    for (ECS::Entity e : m_Registry.GetEntities()) SerializeEntity(s, e);
}

void Scene::SerializeEntity(std::ostream& s, ECS::Entity e) const {  // Scene.cpp:288-430
    s << "Entity " << e << "\n";
    if (m_Registry.HasComponent<UUIDComponent>(e)) s << "UUID " << m_Registry.GetComponent<UUIDComponent>(e).m_ID << "\n";
    if (m_Registry.HasComponent<TagComponent>(e))
        s << "Tag \"" << EscapeString(m_Registry.GetComponent<TagComponent>(e).m_Tag) << "\"\n";
    if (m_Registry.HasComponent<Transform>(e)) {
        const Transform& t = m_Registry.GetComponent<Transform>(e);
        s << std::setprecision(6) << "Transform " << t.Position.x << ' ' << t.Position.y << ' ' << t.Position.z << ' '
          << t.Rotation.x << ' ' << t.Rotation.y << ' ' << t.Rotation.z << ' ' << t.Scale.x << ' ' << t.Scale.y << ' '
          << t.Scale.z << "\n";
    }
    if (m_Registry.HasComponent<CameraComponent>(e)) {
        const CameraComponent& c = m_Registry.GetComponent<CameraComponent>(e);
        s << "Camera " << static_cast<uint32_t>(c.m_ProjectionType) << ' ' << c.m_FieldOfView << ' ' << c.m_OrthographicSize
          << ' ' << c.m_NearClip << ' ' << c.m_FarClip << ' ' << c.m_Primary << ' ' << c.m_FixedAspectRatio << ' '
          << c.m_AspectRatio << "\n";
    }
    if (m_Registry.HasComponent<MeshComponent>(e)) {
        const MeshComponent& m = m_Registry.GetComponent<MeshComponent>(e);
        s << "Mesh " << m.m_MeshIndex << ' ' << m.m_MaterialIndex << ' ' << m.m_FirstIndex << ' ' << m.m_IndexCount << ' '
          << m.m_BaseVertex << ' ' << m.m_Visible << ' ' << static_cast<int>(m.m_Primitive);
        if (!m.m_SourceAssetPath.empty())
            s << ' ' << "SourceAsset=\"" << EscapeString(m.m_SourceAssetPath) << "\"" << ' ' << "SourceMeshIndex="
              << m.m_SourceMeshIndex;
        s << "\n";
    }
    if (m_Registry.HasComponent<SpriteComponent>(e)) {  // Scene.cpp:343-367
        const SpriteComponent& sp = m_Registry.GetComponent<SpriteComponent>(e);
        s << "Sprite " << "Texture=\"" << EscapeString(sp.m_TextureId) << "\" " << "Tint=" << sp.m_TintColor.x << ','
          << sp.m_TintColor.y << ',' << sp.m_TintColor.z << ',' << sp.m_TintColor.w << ' ' << "UVScale=" << sp.m_UVScale.x
          << ',' << sp.m_UVScale.y << ' ' << "UVOffset=" << sp.m_UVOffset.x << ',' << sp.m_UVOffset.y << ' '
          << "Tiling=" << sp.m_TilingFactor << ' ' << "Visible=" << sp.m_Visible << ' '
          << "UseMaterialOverride=" << sp.m_UseMaterialOverride << ' ';
        if (!sp.m_MaterialOverrideId.empty()) s << "Material=\"" << EscapeString(sp.m_MaterialOverrideId) << "\" ";
        s << "AtlasTiles=" << sp.m_AtlasTiles[0] << ',' << sp.m_AtlasTiles[1] << ' ' << "AtlasIndex=" << sp.m_AtlasIndex
          << ' ' << "AnimationSpeed=" << sp.m_AnimationSpeed << ' ' << "SortOffset=" << sp.m_SortOffset << "\n";
    }
    if (m_Registry.HasComponent<TextureComponent>(e)) {
        const TextureComponent& t = m_Registry.GetComponent<TextureComponent>(e);
        s << "Texture \"" << EscapeString(t.m_TexturePath) << "\" Slot=" << t.m_TextureSlot << " Dirty=" << t.m_IsDirty
          << "\n";
    }
    if (m_Registry.HasComponent<LightComponent>(e)) {
        const LightComponent& l = m_Registry.GetComponent<LightComponent>(e);
        s << "Light " << static_cast<uint32_t>(l.m_Type) << ' ' << l.m_Color.x << ' ' << l.m_Color.y << ' ' << l.m_Color.z
          << ' ' << l.m_Intensity << ' ' << l.m_Direction.x << ' ' << l.m_Direction.y << ' ' << l.m_Direction.z << ' '
          << l.m_Range << ' ' << l.m_Enabled << ' ' << l.m_ShadowCaster << ' ' << l.m_Reserved0 << ' ' << l.m_Reserved1
          << "\n";
    }
    s << "EndEntity\n";
}

bool Scene::Load(const std::string& path) {  // Scene.cpp:105-151
    std::ifstream s(path);
    if (!s.is_open()) {
        Warn("failed to open scene file '" + path + "' for reading");
        return false;
    }
    m_Registry.Clear();
    m_LoadedEntityCount = 0;
    std::string line;
    while (std::getline(s, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty() || line.front() == '#') continue;
        if (StartsWith(line, "Scene ")) {
            const std::string name = ExtractQuotedToken(line);
            if (!name.empty()) m_SceneName = name;
            continue;
        }
        if (StartsWith(line, "Entity")) DeserializeEntity(s);
    }
    RebuildMeshAssetsFromComponents();
    return true;
}

void Scene::DeserializeEntity(std::istream& s) {  // Scene.cpp:432-961 (ids in the file are ignored)
    const ECS::Entity e = m_Registry.CreateEntity();
    ++m_LoadedEntityCount;
    std::string line;
    while (std::getline(s, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty() || line.front() == '#') continue;
        if (StartsWith(line, "UUID ")) {
            UUIDComponent u;
            std::istringstream(line.substr(5)) >> u.m_ID;
            m_Registry.AddComponent<UUIDComponent>(e, u);
            continue;
        }
        if (line == "EndEntity") break;
        if (StartsWith(line, "Tag ")) {
            m_Registry.AddComponent<TagComponent>(e, TagComponent{ExtractQuotedToken(line)});
            continue;
        }
        if (StartsWith(line, "Transform ")) {
            Transform t{};
            std::istringstream ts(line.substr(10));
            ts >> t.Position.x >> t.Position.y >> t.Position.z >> t.Rotation.x >> t.Rotation.y >> t.Rotation.z >>
                t.Scale.x >> t.Scale.y >> t.Scale.z;
            m_Registry.AddComponent<Transform>(e, t);
            continue;
        }
        if (StartsWith(line, "Camera ")) {
            CameraComponent c{};
            std::istringstream ts(line.substr(7));
            uint32_t type = 0;
            ts >> type;
            c.m_ProjectionType = static_cast<Camera::ProjectionType>(type);
            ts >> c.m_FieldOfView >> c.m_OrthographicSize >> c.m_NearClip >> c.m_FarClip;
            ts >> std::boolalpha >> c.m_Primary >> c.m_FixedAspectRatio;
            ts >> c.m_AspectRatio;
            m_Registry.AddComponent<CameraComponent>(e, c);
            continue;
        }
        if (StartsWith(line, "Mesh ")) {
            MeshComponent m{};
            std::istringstream ts(line.substr(5));
            ts >> m.m_MeshIndex >> m.m_MaterialIndex >> m.m_FirstIndex >> m.m_IndexCount >> m.m_BaseVertex;
            ts >> std::boolalpha >> m.m_Visible;
            int prim = 0;
            if (ts >> prim)  // unknown values clamp to None (Scene.cpp:507-520)
                m.m_Primitive = (prim >= 0 && prim <= 3) ? static_cast<MeshComponent::PrimitiveType>(prim)
                                                          : MeshComponent::PrimitiveType::None;
            const size_t sa = line.find("SourceAsset=");
            if (sa != std::string::npos) {
                m.m_SourceAssetPath = ExtractQuotedToken(line.substr(sa));
                if (!m.m_SourceAssetPath.empty()) m.m_SourceAssetPath = NormalizePath(m.m_SourceAssetPath);
            }
            const size_t sm = line.find("SourceMeshIndex=");
            if (sm != std::string::npos) {
                std::istringstream ss(line.substr(sm + 16));
                size_t v = 0;
                if (ss >> v) m.m_SourceMeshIndex = v;
            }
            m_Registry.AddComponent<MeshComponent>(e, m);
            continue;
        }
        if (StartsWith(line, "Texture ")) {
            TextureComponent t{};
            t.m_TexturePath = ExtractQuotedToken(line);
            const size_t sl = line.find("Slot=");
            if (sl != std::string::npos) std::istringstream(line.substr(sl + 5)) >> t.m_TextureSlot;
            const size_t di = line.find("Dirty=");
            if (di != std::string::npos) std::istringstream(line.substr(di + 6)) >> std::boolalpha >> t.m_IsDirty;
            m_Registry.AddComponent<TextureComponent>(e, t);
            continue;
        }
        if (StartsWith(line, "Light ")) {
            LightComponent l{};
            std::istringstream ts(line.substr(6));
            uint32_t type = 0;
            ts >> type;
            l.m_Type = static_cast<LightComponent::Type>(type);
            ts >> l.m_Color.x >> l.m_Color.y >> l.m_Color.z >> l.m_Intensity;
            ts >> l.m_Direction.x >> l.m_Direction.y >> l.m_Direction.z >> l.m_Range;
            ts >> std::boolalpha >> l.m_Enabled >> l.m_ShadowCaster >> l.m_Reserved0 >> l.m_Reserved1;
            m_Registry.AddComponent<LightComponent>(e, l);
            continue;
        }
        if (StartsWith(line, "Animation ")) {  // skipped; consume its AnimationBones line
            const size_t bc = line.find("BoneCount=");
            size_t bones = 0;
            if (bc != std::string::npos) std::istringstream(line.substr(bc + 10)) >> bones;
            if (bones > 0) std::getline(s, line);
            continue;
        }
        if (StartsWith(line, "Sprite ")) {
            m_Registry.AddComponent<SpriteComponent>(e, ParseSprite(line));
            continue;
        }
        if (StartsWith(line, "Script ")) continue;  // outside the draw path
        Warn("unknown token while deserialising entity: '" + line + "'");
    }
}

void Scene::RebuildMeshAssetsFromComponents() {  // Scene.cpp:963-1081
    struct Binding {
        MeshComponent* m_Component;
        size_t m_LocalMeshIndex;
    };
    std::vector<std::string> order;  // first-seen asset order (the reference iterates an unordered_map)
    std::unordered_map<std::string, std::vector<Binding>> bindings;
    bool warned = false;
    for (ECS::Entity e : m_Registry.GetEntities()) {
        if (!m_Registry.HasComponent<MeshComponent>(e)) continue;
        MeshComponent& c = m_Registry.GetComponent<MeshComponent>(e);
        if (!c.m_SourceAssetPath.empty()) {
            if (!bindings.count(c.m_SourceAssetPath)) order.push_back(c.m_SourceAssetPath);
            bindings[c.m_SourceAssetPath].push_back(Binding{&c, c.m_SourceMeshIndex});
        } else if (c.m_Primitive == MeshComponent::PrimitiveType::None) {
            c.m_MeshIndex = kInvalidMesh;
            if (!warned) Warn("mesh components without source asset metadata are skipped");
            warned = true;
        }
    }
    std::vector<Geometry::Mesh> meshes;
    std::vector<Geometry::Material> materials;
    std::vector<std::string> textures;
    for (const std::string& asset : order) {
        std::vector<Binding>& bs = bindings[asset];
        Loader::ModelData d = Loader::ModelLoader::Load(asset);
        if (d.m_Meshes.empty()) {
            Warn("failed to reload mesh asset '" + asset + "'");
            for (Binding& b : bs) b.m_Component->m_MeshIndex = kInvalidMesh;
            continue;
        }
        const size_t baseMesh = meshes.size(), meshCount = d.m_Meshes.size(), baseMaterial = materials.size();
        const int texOffset = static_cast<int>(textures.size());
        for (std::string& t : d.m_Textures) textures.push_back(std::move(t));
        for (Geometry::Material& m : d.m_Materials) {
            if (m.BaseColorTextureIndex >= 0) m.BaseColorTextureIndex += texOffset;
            if (m.MetallicRoughnessTextureIndex >= 0) m.MetallicRoughnessTextureIndex += texOffset;
            if (m.NormalTextureIndex >= 0) m.NormalTextureIndex += texOffset;
            materials.push_back(std::move(m));
        }
        for (Geometry::Mesh& m : d.m_Meshes) {
            if (m.MaterialIndex >= 0) m.MaterialIndex += static_cast<int32_t>(baseMaterial);
            meshes.push_back(std::move(m));
        }
        for (Binding& b : bs) {
            if (b.m_LocalMeshIndex >= meshCount) {
                Warn("mesh component references an out-of-range local mesh of '" + asset + "'");
                b.m_Component->m_MeshIndex = kInvalidMesh;
                continue;
            }
            b.m_Component->m_MeshIndex = baseMesh + b.m_LocalMeshIndex;
            b.m_Component->m_Primitive = MeshComponent::PrimitiveType::None;
        }
    }
    if (!m_Renderer) return;
    m_Renderer->UploadMesh(meshes, materials, textures);
}

bool ImportModel(Renderer& renderer, ECS::Registry& registry, const std::string& rawPath,
                 std::vector<ECS::Entity>* spawned) {  // ApplicationLayer.cpp:815-1031, one path
    const std::string path = NormalizePath(rawPath);
    Loader::ModelData d = Loader::ModelLoader::Load(path);
    if (d.m_Meshes.empty() && d.m_MeshInstances.empty()) return false;
    const size_t initialMeshes = renderer.GetModelCount();
    const std::string stem = std::filesystem::path(path).stem().string();
    const std::string tagRoot = stem.empty() ? std::string("Imported Mesh") : stem;
    const size_t total = !d.m_MeshInstances.empty() ? d.m_MeshInstances.size() : d.m_Meshes.size();
    size_t counter = 0;
    bool any = false;
    auto spawn = [&](size_t local, const glm::mat4& model, const std::string& node) {
        if (local >= d.m_Meshes.size()) {
            Warn("mesh instance references an invalid mesh index");
            return;
        }
        const ECS::Entity e = registry.CreateEntity();
        Transform t{};
        if (!Loader::DecomposeMatrixToTransform(model, t)) Warn("failed to decompose an instance transform");
        registry.AddComponent<Transform>(e, t);
        MeshComponent& m = registry.AddComponent<MeshComponent>(e);
        m.m_MeshIndex = initialMeshes + local;
        m.m_Visible = true;
        m.m_SourceAssetPath = path;
        m.m_SourceMeshIndex = local;
        std::string tag = tagRoot;
        if (!node.empty()) tag += " - " + node;
        if (total > 1) tag += " (" + std::to_string(counter + 1) + ")";
        registry.AddComponent<TagComponent>(e, TagComponent{tag});
        if (spawned) spawned->push_back(e);
        ++counter;
        any = true;
    };
    if (!d.m_MeshInstances.empty()) {
        for (const Loader::MeshInstance& inst : d.m_MeshInstances) spawn(inst.m_MeshIndex, inst.m_ModelMatrix, inst.m_NodeName);
    } else {
        for (size_t i = 0; i < d.m_Meshes.size(); ++i) spawn(i, glm::mat4(1.0f), {});
    }
    if (!any) return false;
    renderer.AppendMeshes(std::move(d.m_Meshes), std::move(d.m_Materials), std::move(d.m_Textures));
    return true;
}

}  // namespace Trident
