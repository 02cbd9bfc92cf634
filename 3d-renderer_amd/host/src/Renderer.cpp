// Renderer.cpp — Trident::Renderer's draw path over the HIP rasterizer C-ABI.
//
// Mirrors the reference's CPU side of the hot path: primitive meshes (Renderer.cpp:72-246),
// ComposeTransform (:417-427), UploadMesh/AppendMeshes/UploadMeshFromCache (:1784-2116), texture
// slots (:3404-3804), GatherMeshDraws (:2910-2994), UpdateUniformBuffer (:5822-6051), the per-draw
// push-constant loop (:5110-5151), per-viewport camera routing (:4545-4574), readback (:1299-1389)
// and frame timing (:6286-6343). Vulkan command recording is replaced by tri_set_frame /
// tri_set_draws / tri_render on one tri_ctx per viewport.
#include "trident/Renderer.h"
#include "trident/ModelLoader.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>

namespace Trident {

namespace {

constexpr const char* kDefaultTextureKey = "renderer://default-white";
constexpr size_t kInvalidMeshIndex = std::numeric_limits<size_t>::max();

void LogError(const char* what, const char* detail) { std::fprintf(stderr, "[Trident] %s: %s\n", what, detail); }

Geometry::Mesh BuildPrimitiveQuadMesh() {
    Geometry::Mesh mesh;
    Vertex v[4]{};
    v[0].Position = {-0.5f, -0.5f, 0.0f};
    v[1].Position = {0.5f, -0.5f, 0.0f};
    v[2].Position = {0.5f, 0.5f, 0.0f};
    v[3].Position = {-0.5f, 0.5f, 0.0f};
    for (Vertex& it : v) {
        it.Normal = {0.0f, 0.0f, 1.0f};
        it.Tangent = {1.0f, 0.0f, 0.0f};
        it.Bitangent = {0.0f, 1.0f, 0.0f};
        it.Color = {1.0f, 1.0f, 1.0f};
    }
    v[0].TexCoord = {0.0f, 0.0f};
    v[1].TexCoord = {1.0f, 0.0f};
    v[2].TexCoord = {1.0f, 1.0f};
    v[3].TexCoord = {0.0f, 1.0f};
    mesh.Vertices.assign(v, v + 4);
    mesh.Indices = {0, 1, 2, 0, 2, 3};  // counter clockwise with the projection Y flip
    return mesh;
}

// BuildSpriteGeometry (Renderer.cpp:2853-2890): a unit quad facing -Z with indices {0, 2, 1, 0, 3, 2}
// (the opposite winding of the quad primitive: a sprite seen from +Z is back-facing and culled, as in
// the reference, whose Default pipeline culls BACK for sprites too).
Geometry::Mesh BuildSpriteQuadMesh() {
    Geometry::Mesh mesh;
    Vertex v[4]{};
    v[0].Position = {-0.5f, -0.5f, 0.0f};
    v[1].Position = {0.5f, -0.5f, 0.0f};
    v[2].Position = {0.5f, 0.5f, 0.0f};
    v[3].Position = {-0.5f, 0.5f, 0.0f};
    for (Vertex& it : v) {
        it.Normal = {0.0f, 0.0f, -1.0f};
        it.Tangent = {1.0f, 0.0f, 0.0f};
        it.Bitangent = {0.0f, 1.0f, 0.0f};
        it.Color = {1.0f, 1.0f, 1.0f};
    }
    v[0].TexCoord = {0.0f, 0.0f};
    v[1].TexCoord = {1.0f, 0.0f};
    v[2].TexCoord = {1.0f, 1.0f};
    v[3].TexCoord = {0.0f, 1.0f};
    mesh.Vertices.assign(v, v + 4);
    mesh.Indices = {0, 2, 1, 0, 3, 2};
    return mesh;
}

Geometry::Mesh BuildPrimitiveCubeMesh() {
    struct Face {
        glm::vec3 n, t, b;
        glm::vec3 p[4];
    };
    const Face faces[6] = {
        {{0, 0, 1}, {1, 0, 0}, {0, 1, 0}, {{-0.5f, -0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f}}},
        {{0, 0, -1}, {-1, 0, 0}, {0, 1, 0}, {{0.5f, -0.5f, -0.5f}, {-0.5f, -0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}}},
        {{1, 0, 0}, {0, 0, -1}, {0, 1, 0}, {{0.5f, -0.5f, 0.5f}, {0.5f, -0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}, {0.5f, 0.5f, 0.5f}}},
        {{-1, 0, 0}, {0, 0, 1}, {0, 1, 0}, {{-0.5f, -0.5f, -0.5f}, {-0.5f, -0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f}, {-0.5f, 0.5f, -0.5f}}},
        {{0, 1, 0}, {1, 0, 0}, {0, 0, -1}, {{-0.5f, 0.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {0.5f, 0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f}}},
        {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}, {{-0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, 0.5f}, {-0.5f, -0.5f, 0.5f}}},
    };
    const glm::vec2 uv[4] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
    Geometry::Mesh mesh;
    uint32_t off = 0;
    for (const Face& f : faces) {
        for (int k = 0; k < 4; ++k) {
            Vertex v{};
            v.Position = f.p[k];
            v.Normal = f.n;
            v.Tangent = f.t;
            v.Bitangent = f.b;
            v.Color = {1.0f, 1.0f, 1.0f};
            v.TexCoord = uv[k];
            mesh.Vertices.push_back(v);
        }
        for (uint32_t i : {0u, 2u, 1u, 0u, 3u, 2u}) mesh.Indices.push_back(off + i);  // CW from outside
        off += 4;
    }
    return mesh;
}

Geometry::Mesh BuildPrimitiveSphereMesh() {
    const uint32_t rings = 16, segments = 24;
    const float radius = 0.5f;
    Geometry::Mesh mesh;
    for (uint32_t r = 0; r <= rings; ++r) {
        const float V = (float)r / (float)rings;
        const float phi = V * glm::pi<float>();
        for (uint32_t s = 0; s <= segments; ++s) {
            const float U = (float)s / (float)segments;
            const float theta = U * glm::two_pi<float>();
            const float sp = std::sin(phi), cp = std::cos(phi), st = std::sin(theta), ct = std::cos(theta);
            const glm::vec3 p{radius * sp * ct, radius * cp, radius * sp * st};
            const glm::vec3 n = glm::normalize(p);
            glm::vec3 t{-st, 0.0f, ct};
            if (glm::length(t) < 0.0001f) t = {1.0f, 0.0f, 0.0f};
            t = glm::normalize(t);
            glm::vec3 b = glm::normalize(glm::cross(n, t));
            if (glm::length(b) < 0.0001f) b = {0.0f, 1.0f, 0.0f};
            Vertex v{};
            v.Position = p;
            v.Normal = n;
            v.Tangent = t;
            v.Bitangent = b;
            v.Color = {1.0f, 1.0f, 1.0f};
            v.TexCoord = {U, 1.0f - V};
            mesh.Vertices.push_back(v);
        }
    }
    const uint32_t row = segments + 1;
    for (uint32_t r = 0; r < rings; ++r)
        for (uint32_t s = 0; s < segments; ++s) {
            const uint32_t i0 = r * row + s, i1 = (r + 1) * row + s, i2 = (r + 1) * row + s + 1, i3 = r * row + s + 1;
            for (uint32_t i : {i0, i2, i1, i0, i3, i2}) mesh.Indices.push_back(i);
        }
    return mesh;
}

glm::mat4 ComposeTransform(const Transform& t) {  // T * Rx * Ry * Rz * S, degrees
    glm::mat4 m{1.0f};
    m = glm::translate(m, t.Position);
    m = glm::rotate(m, glm::radians(t.Rotation.x), glm::vec3{1.0f, 0.0f, 0.0f});
    m = glm::rotate(m, glm::radians(t.Rotation.y), glm::vec3{0.0f, 1.0f, 0.0f});
    m = glm::rotate(m, glm::radians(t.Rotation.z), glm::vec3{0.0f, 0.0f, 1.0f});
    return glm::scale(m, t.Scale);
}

std::string NormalizeTexturePath(const std::string& path) {
    std::string s = path;
    std::replace(s.begin(), s.end(), '\\', '/');
    return s;
}

void CopyMat(const glm::mat4& m, float* out) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = m[c][r];
}

// A viewport's render target: one context, or a group of row bands on several devices (SetDeviceCount).
// Every per-context call of the draw path goes to the context or is broadcast to the group's bands.
struct Target {
    tri_ctx* c;
    tri_group* g;
    int Materials(const tri_material_record* r, uint32_t n) const {
        return g ? tri_group_upload_materials(g, r, n) : tri_upload_materials(c, r, n);
    }
    int Skybox(const uint8_t* f, uint32_t n) const { return g ? tri_group_upload_skybox(g, f, n) : tri_upload_skybox(c, f, n); }
    int AiFrame(const uint8_t* p, uint32_t w, uint32_t h) const {
        return g ? tri_group_upload_ai_frame(g, p, w, h) : tri_upload_ai_frame(c, p, w, h);
    }
    int Texture(uint32_t slot, const uint8_t* p, uint32_t w, uint32_t h) const {
        return g ? tri_group_upload_texture(g, slot, p, w, h) : tri_upload_texture(c, slot, p, w, h);
    }
    int Shadow(const tri_shadow_config* s) const { return g ? tri_group_set_shadow(g, s) : tri_set_shadow(c, s); }
    int Bones(const float* m, uint32_t n) const {
        return g ? tri_group_upload_bone_palette(g, m, n) : tri_upload_bone_palette(c, m, n);
    }
    int Frame(const tri_global_ubo* u, const float* clear) const {
        return g ? tri_group_set_frame(g, u, clear) : tri_set_frame(c, u, clear);
    }
    int Draws(const tri_draw* d, uint32_t n) const { return g ? tri_group_set_draws(g, d, n) : tri_set_draws(c, d, n); }
    int Render() const { return g ? tri_group_render(g) : tri_render(c); }
    int Sync() const { return g ? tri_group_synchronize(g) : tri_synchronize(c); }
    int Output(tri_image* o) const { return g ? tri_group_get_output(g, o) : tri_get_output(c, o); }
    int Blit(uint32_t w, uint32_t h) const { return g ? tri_group_blit_linear(g, nullptr, w, h) : tri_blit_linear(c, nullptr, w, h); }
    int ReadPresent(uint8_t* p) const { return g ? tri_group_read_present(g, p) : tri_read_present(c, p); }
    int Readback(uint8_t* bgra, uint32_t* depth) const {
        return g ? tri_group_readback(g, bgra, depth) : tri_readback(c, bgra, depth);
    }
};

}  // namespace

Renderer::Renderer() = default;
Renderer::~Renderer() { Shutdown(); }

void Renderer::Init() {
    if (m_Initialised) return;
    m_TextureSlots.clear();
    m_TextureSlotLookup.clear();
    TextureSlot white;  // CreateDefaultTexture (Renderer.cpp:3404-3436)
    white.m_SourcePath = kDefaultTextureKey;
    white.m_Data.Width = white.m_Data.Height = 1;
    white.m_Data.Pixels = {0xFF, 0xFF, 0xFF, 0xFF};
    m_TextureSlots.push_back(white);
    m_TextureSlotLookup.emplace(kDefaultTextureKey, 0u);
    m_PerformanceHistory.assign(s_PerformanceHistorySize, FrameTimingSample{});
    CreateSkyboxCubemap();  // CreateDefaultSkybox (Renderer.cpp:3806-3816)
    m_Initialised = true;
    m_Shutdown = false;
}

void Renderer::DestroyViewportTargets() {
    m_Pending.clear();  // (its targets go; tri_destroy / tri_group_destroy wait for their streams)
    auto drop = [](ViewportContext& vc) {
        tri_destroy(vc.m_Ctx);
        tri_group_destroy(vc.m_Group);
        vc.m_Ctx = nullptr;
        vc.m_Group = nullptr;
        vc.m_HasImage = false;
        vc.m_Width = vc.m_Height = 0;
    };
    for (auto& it : m_Viewports) drop(it.second);
    for (auto& it : m_RingTargets)
        for (ViewportContext& vc : it.second) drop(vc);
    m_RingTargets.clear();
    m_LatestTarget.clear();
    tri_destroy(m_LegacyTarget.m_Ctx);
    tri_group_destroy(m_LegacyTarget.m_Group);
    m_LegacyTarget = ViewportContext{};
    m_PresentSource = nullptr;
    m_PresentGroup = nullptr;
    m_PresentLegacy = false;
    // after every context that bound them
    tri_geometry_destroy(m_SharedGeometry);
    m_SharedGeometry = nullptr;
    m_SharedGeometryGeneration = 0;
    for (tri_geometry* g : m_DeviceGeometry) tri_geometry_destroy(g);
    m_DeviceGeometry.clear();
    m_DeviceGeometryGeneration.clear();
}

void Renderer::Shutdown() {
    DestroyViewportTargets();
    m_Viewports.clear();
    if (m_Initialised) m_Shutdown = true;
    m_Initialised = false;
}

void Renderer::SetFramesInFlight(uint32_t n) {
    n = std::min<uint32_t>(std::max<uint32_t>(n, 1u), 4u);
    if (n == m_FramesInFlight) return;
    FinishFrame();
    DestroyViewportTargets();  // rebuilt by the next DrawFrame's PrepareViewport
    m_FramesInFlight = n;
}

// Target `index` of a viewport (0: its m_Viewports entry; 1 .. n-1: the ring's), carrying the viewport's info.
Renderer::ViewportContext& Renderer::TargetOf(uint32_t viewportId, ViewportContext& primary, uint32_t index) {
    if (index == 0) return primary;
    std::vector<ViewportContext>& ring = m_RingTargets[viewportId];
    if (ring.size() < m_FramesInFlight - 1) ring.resize(m_FramesInFlight - 1);  // (sized once per SetFramesInFlight)
    ViewportContext& t = ring[index - 1];
    t.m_Info = primary.m_Info;
    return t;
}

const Renderer::ViewportContext* Renderer::LatestTarget(uint32_t viewportId) const {
    auto it = m_Viewports.find(viewportId);
    if (it == m_Viewports.end()) return nullptr;
    auto li = m_LatestTarget.find(viewportId);
    if (li == m_LatestTarget.end() || li->second == 0) return &it->second;
    auto ri = m_RingTargets.find(viewportId);
    if (ri == m_RingTargets.end() || ri->second.size() < li->second) return &it->second;
    return &ri->second[li->second - 1];
}

bool Renderer::SetDeviceCount(uint32_t count, const std::vector<int32_t>& devices) {
    std::vector<int32_t> devs;
    if (count > 1) {
        if (!devices.empty() && devices.size() != count) {
            LogError("SetDeviceCount", "device list length differs from the count");
            return false;
        }
        for (uint32_t i = 0; i < count; ++i) {
            const int32_t d = devices.empty() ? (int32_t)i : devices[i];
            if (d < 0) {
                LogError("SetDeviceCount", "negative device ordinal");
                return false;
            }
            devs.push_back(d);
        }
    }
    if (devs == m_Devices) return true;
    DestroyViewportTargets();  // rebuilt by the next DrawFrame's PrepareViewport
    m_Devices = devs;
    return true;
}

// Multi-device viewports: one copy of the concatenated buffers per distinct device and generation,
// bound by every viewport's group (tri_group_bind_geometry picks each band's device copy).
bool Renderer::UploadSharedGeometry(std::vector<tri_geometry*>& out) {
    std::vector<int32_t> udev;
    for (int32_t d : m_Devices)
        if (std::find(udev.begin(), udev.end(), d) == udev.end()) udev.push_back(d);
    if (m_DeviceGeometry.size() != udev.size()) {
        for (tri_geometry* g : m_DeviceGeometry) tri_geometry_destroy(g);
        m_DeviceGeometry.assign(udev.size(), nullptr);
        m_DeviceGeometryGeneration.assign(udev.size(), 0);
    }
    const std::vector<tri_mesh_range> ranges = GetMeshRanges();
    for (size_t u = 0; u < udev.size(); ++u) {
        if (!m_DeviceGeometry[u] && tri_geometry_create(udev[u], &m_DeviceGeometry[u]) != TRI_OK) {
            LogError("UploadMeshFromCache", tri_last_error());
            m_DeviceGeometry[u] = nullptr;
            return false;
        }
        if (m_DeviceGeometryGeneration[u] != m_GeometryGeneration) {
            if (tri_geometry_upload(m_DeviceGeometry[u], m_VertexBuffer.data(), m_VertexBuffer.size(), m_IndexBuffer.data(),
                                    m_IndexBuffer.size(), ranges.data(), (uint32_t)ranges.size()) != TRI_OK) {
                LogError("UploadMeshFromCache", tri_last_error());
                return false;
            }
            m_DeviceGeometryGeneration[u] = m_GeometryGeneration;
            ++m_GeometryUploads;
        }
    }
    out = m_DeviceGeometry;
    return true;
}

// Renderer.cpp:3818-3927: the discovered cubemap (KTX, Default/ directory, loose px/nx/... PNG faces),
// else the solid 0x808080 fallback.
void Renderer::CreateSkyboxCubemap() {
    std::string source;
    Loader::CubemapTextureData data = Loader::DiscoverDefaultSkybox(m_AssetsDirectory, source);
    if (!data.IsValid()) {
        data = Loader::CubemapTextureData::CreateSolidColor(0x808080u);
        source = "solid 0x808080";
    }
    m_SkyboxCubemap = std::move(data);
    m_SkyboxSource = source;
    ++m_SkyboxGeneration;
}

void Renderer::SetAssetsDirectory(const std::string& directory) {
    m_AssetsDirectory = directory;
    if (m_Initialised) CreateSkyboxCubemap();
}

bool Renderer::SetSkyboxCubemap(const Loader::CubemapTextureData& cubemap) {
    if (!cubemap.IsValid()) {
        LogError("SetSkyboxCubemap", "cubemap needs 6 square RGBA8 faces");
        return false;
    }
    m_SkyboxCubemap = cubemap;
    m_SkyboxSource = "SetSkyboxCubemap";
    ++m_SkyboxGeneration;
    return true;
}

// ---- geometry ---------------------------------------------------------------------------------
void Renderer::UploadMesh(const std::vector<Geometry::Mesh>& meshes, const std::vector<Geometry::Material>& materials,
                          const std::vector<std::string>& textures) {
    m_GeometryCache = meshes;
    m_Materials = materials;
    for (size_t& p : m_PrimitiveMeshIndices) p = kInvalidMeshIndex;
    ResolveMaterialTextureSlots(textures, 0, m_Materials.size());
    UploadMeshFromCache();
}

void Renderer::AppendMeshes(std::vector<Geometry::Mesh> meshes, std::vector<Geometry::Material> materials,
                            std::vector<std::string> textures) {
    if (meshes.empty()) return;
    const size_t oldMaterials = m_Materials.size();
    for (Geometry::Mesh& m : meshes) {
        if (m.MaterialIndex >= 0) m.MaterialIndex += static_cast<int32_t>(oldMaterials);
        m_GeometryCache.emplace_back(std::move(m));
    }
    const size_t offset = m_Materials.size();
    for (Geometry::Material& m : materials) m_Materials.emplace_back(std::move(m));
    ResolveMaterialTextureSlots(textures, offset, materials.size());
    UploadMeshFromCache();
}

size_t Renderer::GetOrCreatePrimitiveMeshIndex(MeshComponent::PrimitiveType type) {
    if (type == MeshComponent::PrimitiveType::None) return kInvalidMeshIndex;
    const size_t slot = static_cast<size_t>(type) - 1;
    if (slot >= 3) return kInvalidMeshIndex;
    const size_t existing = m_PrimitiveMeshIndices[slot];
    if (existing != kInvalidMeshIndex && existing < m_GeometryCache.size()) return existing;
    const size_t index = CreatePrimitiveMeshInCache(type);
    if (index == kInvalidMeshIndex) return index;
    if (!m_IsUploadingMeshes) UploadMeshFromCache();
    return index;
}

size_t Renderer::CreatePrimitiveMeshInCache(MeshComponent::PrimitiveType type) {
    const size_t slot = static_cast<size_t>(type) - 1;
    if (type == MeshComponent::PrimitiveType::None || slot >= 3) return kInvalidMeshIndex;
    const size_t existing = m_PrimitiveMeshIndices[slot];
    if (existing != kInvalidMeshIndex && existing < m_GeometryCache.size()) return existing;
    Geometry::Mesh mesh = type == MeshComponent::PrimitiveType::Cube     ? BuildPrimitiveCubeMesh()
                          : type == MeshComponent::PrimitiveType::Sphere ? BuildPrimitiveSphereMesh()
                                                                         : BuildPrimitiveQuadMesh();
    Geometry::Material material{};  // primitives: metallic 0, roughness 1 (Renderer.cpp:1900-1906)
    material.BaseColorFactor = {1.0f, 1.0f, 1.0f, 1.0f};
    material.MetallicFactor = 0.0f;
    material.RoughnessFactor = 1.0f;
    material.BaseColorTextureSlot = 0;
    mesh.MaterialIndex = static_cast<int32_t>(m_Materials.size());
    m_Materials.push_back(material);
    m_GeometryCache.push_back(std::move(mesh));
    m_PrimitiveMeshIndices[slot] = m_GeometryCache.size() - 1;
    ++m_MaterialGeneration;
    return m_GeometryCache.size() - 1;
}

void Renderer::EnsurePrimitiveMeshesInCache() {
    if (!m_Registry) return;
    for (ECS::Entity e : m_Registry->GetEntities()) {
        if (!m_Registry->HasComponent<MeshComponent>(e)) continue;
        MeshComponent& c = m_Registry->GetComponent<MeshComponent>(e);
        if (c.m_Primitive == MeshComponent::PrimitiveType::None) continue;
        if (c.m_MeshIndex != kInvalidMeshIndex && c.m_MeshIndex < m_GeometryCache.size()) continue;
        const size_t index = CreatePrimitiveMeshInCache(c.m_Primitive);
        if (index != kInvalidMeshIndex) c.m_MeshIndex = index;
    }
}

void Renderer::UploadMeshFromCache() {  // Renderer.cpp:1965-2116
    m_IsUploadingMeshes = true;
    EnsurePrimitiveMeshesInCache();
    m_VertexBuffer.clear();
    m_IndexBuffer.clear();
    m_MeshDrawInfo.clear();
    m_MeshBoundsMin.clear();
    m_MeshBoundsMax.clear();
    uint32_t firstIndex = 0;
    int32_t baseVertex = 0;
    for (const Geometry::Mesh& mesh : m_GeometryCache) {
        const size_t v0 = m_VertexBuffer.size();
        m_VertexBuffer.resize(v0 + mesh.Vertices.size());
        std::memcpy(m_VertexBuffer.data() + v0, mesh.Vertices.data(), mesh.Vertices.size() * sizeof(Vertex));
        m_IndexBuffer.insert(m_IndexBuffer.end(), mesh.Indices.begin(), mesh.Indices.end());  // mesh-local
        MeshDrawInfo info;
        info.m_FirstIndex = firstIndex;
        info.m_IndexCount = static_cast<uint32_t>(mesh.Indices.size());
        info.m_BaseVertex = baseVertex;
        info.m_MaterialIndex = mesh.MaterialIndex;
        m_MeshDrawInfo.push_back(info);
        glm::vec3 lo{INFINITY}, hi{-INFINITY};  // box of the referenced vertices (shadow frustum fit)
        for (uint32_t idx : mesh.Indices) {
            if (idx >= mesh.Vertices.size()) continue;
            const glm::vec3& p = mesh.Vertices[idx].Position;
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], p[a]);
                hi[a] = std::max(hi[a], p[a]);
            }
        }
        m_MeshBoundsMin.push_back(lo);
        m_MeshBoundsMax.push_back(hi);
        firstIndex += info.m_IndexCount;
        baseVertex += static_cast<int32_t>(mesh.Vertices.size());
    }
    if (m_HasSpriteGeometry) {  // after every cached mesh, outside m_MeshDrawInfo (no MeshComponent reaches it)
        const Geometry::Mesh quad = BuildSpriteQuadMesh();
        const size_t v0 = m_VertexBuffer.size();
        m_VertexBuffer.resize(v0 + quad.Vertices.size());
        std::memcpy(m_VertexBuffer.data() + v0, quad.Vertices.data(), quad.Vertices.size() * sizeof(Vertex));
        m_IndexBuffer.insert(m_IndexBuffer.end(), quad.Indices.begin(), quad.Indices.end());
        m_SpriteDrawInfo.m_FirstIndex = firstIndex;
        m_SpriteDrawInfo.m_IndexCount = static_cast<uint32_t>(quad.Indices.size());
        m_SpriteDrawInfo.m_BaseVertex = baseVertex;
        m_SpriteDrawInfo.m_MaterialIndex = -1;
    }
    m_MeshDrawCommands.clear();
    if (m_Registry) {
        for (ECS::Entity e : m_Registry->GetEntities()) {
            if (!m_Registry->HasComponent<MeshComponent>(e)) continue;
            MeshComponent& c = m_Registry->GetComponent<MeshComponent>(e);
            if (c.m_MeshIndex >= m_MeshDrawInfo.size()) continue;
            const MeshDrawInfo& d = m_MeshDrawInfo[c.m_MeshIndex];
            c.m_FirstIndex = d.m_FirstIndex;
            c.m_IndexCount = d.m_IndexCount;
            c.m_BaseVertex = d.m_BaseVertex;
            c.m_MaterialIndex = d.m_MaterialIndex;
        }
    }
    m_ModelCount = m_GeometryCache.size();
    m_TriangleCount = firstIndex / 3;  // the cached meshes' triangles (the sprite quad is not a model)
    ++m_GeometryGeneration;
    ++m_MaterialGeneration;
    m_IsUploadingMeshes = false;
}

// ---- textures ---------------------------------------------------------------------------------
void Renderer::UploadTexture(const std::string& texturePath, const Loader::TextureData& texture) {
    const std::string key = NormalizeTexturePath(texturePath);
    if (texture.Width <= 0 || texture.Height <= 0 ||
        texture.Pixels.size() < (size_t)texture.Width * texture.Height * 4) {
        LogError("UploadTexture", "texture has no RGBA8 pixel data; using the default slot");
        m_TextureSlotLookup[key] = 0u;
        return;
    }
    auto it = m_TextureSlotLookup.find(key);
    uint32_t slot;
    if (it != m_TextureSlotLookup.end() && it->second != 0) {
        slot = it->second;
    } else {
        if (m_TextureSlots.size() >= TRI_MAX_TEXTURE_SLOTS) {
            LogError("UploadTexture", "all 256 texture slots are in use; using the default slot");
            m_TextureSlotLookup[key] = 0u;
            return;
        }
        slot = static_cast<uint32_t>(m_TextureSlots.size());
        m_TextureSlots.emplace_back();
        m_TextureSlotLookup[key] = slot;
    }
    m_TextureSlots[slot].m_SourcePath = key;
    m_TextureSlots[slot].m_Data = texture;
    ++m_TextureGeneration;
}

int32_t Renderer::ResolveTextureSlot(const std::string& texturePath) {
    const std::string key = NormalizeTexturePath(texturePath);
    if (key.empty()) return 0;
    auto it = m_TextureSlotLookup.find(key);
    if (it != m_TextureSlotLookup.end()) return static_cast<int32_t>(it->second);
    // Load on first use (ResolveTextureSlot -> TextureLoader::Load, Renderer.cpp:3700-3745). Formats
    // stb would decode but that are not restated here (PNG, JPEG) fail like a failed load in the
    // reference: the default slot (:3740-3745).
    const Loader::TextureData data = Loader::TextureLoader::Load(key);
    if (data.Width > 0) {
        UploadTexture(key, data);
        it = m_TextureSlotLookup.find(key);
        if (it != m_TextureSlotLookup.end()) return static_cast<int32_t>(it->second);
    }
    LogError("ResolveTextureSlot", (key + " could not be loaded; using the default slot").c_str());
    m_TextureSlotLookup.emplace(key, 0u);
    return 0;
}

void Renderer::ResolveMaterialTextureSlots(const std::vector<std::string>& textures, size_t offset, size_t count) {
    if (m_Materials.empty()) return;
    const size_t safeOffset = std::min(offset, m_Materials.size());
    const size_t n = std::min(count, m_Materials.size() - safeOffset);
    for (size_t i = 0; i < n; ++i) {
        Geometry::Material& m = m_Materials[safeOffset + i];
        m.BaseColorTextureSlot = 0;
        if (m.BaseColorTextureIndex < 0 || (size_t)m.BaseColorTextureIndex >= textures.size()) continue;
        const std::string key = NormalizeTexturePath(textures[m.BaseColorTextureIndex]);
        if (key.empty()) continue;
        m.BaseColorTextureSlot = ResolveTextureSlot(key);
    }
    ++m_MaterialGeneration;
}

// ---- frame preparation --------------------------------------------------------------------------
void Renderer::GatherMeshDraws() {  // Renderer.cpp:2910-2994
    m_MeshDrawCommands.clear();
    if (!m_Registry) return;
    for (ECS::Entity e : m_Registry->GetEntities()) {
        if (!m_Registry->HasComponent<MeshComponent>(e)) continue;
        MeshComponent& c = m_Registry->GetComponent<MeshComponent>(e);
        if (!c.m_Visible) continue;
        if (c.m_Primitive != MeshComponent::PrimitiveType::None && c.m_MeshIndex == kInvalidMeshIndex) {
            c.m_MeshIndex = GetOrCreatePrimitiveMeshIndex(c.m_Primitive);
            if (c.m_MeshIndex == kInvalidMeshIndex) continue;
        }
        if (c.m_MeshIndex >= m_MeshDrawInfo.size()) continue;
        if (m_MeshDrawInfo[c.m_MeshIndex].m_IndexCount == 0) continue;
        MeshDrawCommand cmd;
        if (m_Registry->HasComponent<Transform>(e)) cmd.m_ModelMatrix = ComposeTransform(m_Registry->GetComponent<Transform>(e));
        if (m_Registry->HasComponent<TextureComponent>(e)) {
            TextureComponent& t = m_Registry->GetComponent<TextureComponent>(e);
            if (t.m_IsDirty || t.m_TextureSlot < 0) {
                t.m_TextureSlot = ResolveTextureSlot(t.m_TexturePath);
                t.m_IsDirty = false;
            }
            cmd.m_TextureComponent = &t;
        }
        if (m_Registry->HasComponent<AnimationComponent>(e))
            cmd.m_AnimationComponent = &m_Registry->GetComponent<AnimationComponent>(e);
        cmd.m_Component = &c;
        cmd.m_Entity = e;
        m_MeshDrawCommands.push_back(cmd);
    }
}

void Renderer::GatherSpriteDraws() {  // Renderer.cpp:2996-3042
    m_SpriteDrawList.clear();
    if (!m_Registry) return;
    for (ECS::Entity e : m_Registry->GetEntities()) {
        if (!m_Registry->HasComponent<Transform>(e) || !m_Registry->HasComponent<SpriteComponent>(e)) continue;
        SpriteComponent& sprite = m_Registry->GetComponent<SpriteComponent>(e);
        if (!sprite.m_Visible) continue;
        TextureComponent* tex = nullptr;
        if (m_Registry->HasComponent<TextureComponent>(e)) {
            tex = &m_Registry->GetComponent<TextureComponent>(e);
            if (tex->m_IsDirty || tex->m_TextureSlot < 0) {
                tex->m_TextureSlot = ResolveTextureSlot(tex->m_TexturePath);
                tex->m_IsDirty = false;
            }
        }
        SpriteDrawCommand cmd;
        cmd.m_ModelMatrix = ComposeTransform(m_Registry->GetComponent<Transform>(e));
        cmd.m_Component = &sprite;
        cmd.m_TextureComponent = tex;
        cmd.m_Entity = e;
        m_SpriteDrawList.push_back(cmd);
    }
}

void Renderer::GatherDraws() {
    GatherMeshDraws();
    GatherSpriteDraws();
    if (!m_SpriteDrawList.empty() && !m_HasSpriteGeometry) {
        // first sprite: the quad joins the device geometry (the reference built its own buffer at Init);
        // the upload clears the mesh commands, which are gathered again (no texture slot changes)
        m_HasSpriteGeometry = true;
        UploadMeshFromCache();
        GatherMeshDraws();
    }
}

// Renderer.cpp:3168-3245: each animated draw gets a slice [offset, offset + count) of one palette
// (count clamped to s_MaxBonesPerSkeleton); draws without a palette keep offset 0 / count 0.
void Renderer::PrepareBonePaletteBuffer() {
    m_BonePalette.clear();
    uint32_t total = 0;
    for (MeshDrawCommand& cmd : m_MeshDrawCommands) {
        cmd.m_BoneOffset = 0;
        cmd.m_BoneCount = 0;
        if (!cmd.m_AnimationComponent || cmd.m_AnimationComponent->m_BoneMatrices.empty()) continue;
        const auto& src = cmd.m_AnimationComponent->m_BoneMatrices;
        const uint32_t n = (uint32_t)std::min<size_t>(src.size(), s_MaxBonesPerSkeleton);
        cmd.m_BoneOffset = total;
        cmd.m_BoneCount = n;
        total += n;
        for (uint32_t b = 0; b < n; ++b) {
            float m[16];
            CopyMat(src[b], m);
            m_BonePalette.insert(m_BonePalette.end(), m, m + 16);
        }
    }
}

void Renderer::BuildDrawList(std::vector<tri_draw>& out) const {  // Renderer.cpp:5110-5151
    out.clear();
    for (const MeshDrawCommand& cmd : m_MeshDrawCommands) {
        if (!cmd.m_Component || cmd.m_Component->m_MeshIndex >= m_MeshDrawInfo.size()) continue;
        const MeshDrawInfo& info = m_MeshDrawInfo[cmd.m_Component->m_MeshIndex];
        if (info.m_IndexCount == 0) continue;
        tri_draw d;
        std::memset(&d, 0, sizeof d);
        d.mesh_index = static_cast<uint32_t>(cmd.m_Component->m_MeshIndex);
        tri_push_constant& pc = d.pc;  // RenderablePushConstant defaults (RenderData.h:16-29)
        CopyMat(cmd.m_ModelMatrix, pc.model);
        pc.tint[0] = pc.tint[1] = pc.tint[2] = pc.tint[3] = 1.0f;
        pc.texture_scale[0] = pc.texture_scale[1] = 1.0f;
        pc.tiling_factor = 1.0f;
        int32_t slot = 0;
        if (cmd.m_TextureComponent && cmd.m_TextureComponent->m_TextureSlot >= 0)
            slot = cmd.m_TextureComponent->m_TextureSlot;
        else if (info.m_MaterialIndex >= 0 && (size_t)info.m_MaterialIndex < m_Materials.size())
            slot = m_Materials[info.m_MaterialIndex].BaseColorTextureSlot;
        pc.texture_slot = slot;
        pc.material_index = info.m_MaterialIndex;
        pc.bone_offset = static_cast<int32_t>(cmd.m_BoneOffset);  // :5145-5146
        pc.bone_count = static_cast<int32_t>(cmd.m_BoneCount);
        out.push_back(d);
    }
    if (!m_HasSpriteGeometry) return;
    for (const SpriteDrawCommand& cmd : m_SpriteDrawList) {  // DrawSprites, Renderer.cpp:3044-3089
        if (!cmd.m_Component) continue;
        const SpriteComponent& sp = *cmd.m_Component;
        tri_draw d;
        std::memset(&d, 0, sizeof d);
        d.mesh_index = static_cast<uint32_t>(m_MeshDrawInfo.size());  // the sprite quad's range
        tri_push_constant& pc = d.pc;
        CopyMat(cmd.m_ModelMatrix, pc.model);
        pc.tint[0] = sp.m_TintColor.x; pc.tint[1] = sp.m_TintColor.y;
        pc.tint[2] = sp.m_TintColor.z; pc.tint[3] = sp.m_TintColor.w;
        pc.texture_scale[0] = sp.m_UVScale.x; pc.texture_scale[1] = sp.m_UVScale.y;
        pc.texture_offset[0] = sp.m_UVOffset.x; pc.texture_offset[1] = sp.m_UVOffset.y;
        pc.tiling_factor = sp.m_TilingFactor;
        pc.use_material_override = sp.m_UseMaterialOverride ? 1 : 0;
        pc.sort_bias = sp.m_SortOffset;
        pc.texture_slot = (cmd.m_TextureComponent && cmd.m_TextureComponent->m_TextureSlot >= 0)
                              ? cmd.m_TextureComponent->m_TextureSlot : 0;
        pc.material_index = -1;  // RenderablePushConstant default (RenderData.h:25)
        out.push_back(d);
    }
}

void Renderer::UpdateUniformBuffer(const Camera* camera, tri_global_ubo& g) const {  // Renderer.cpp:5822-5925
    std::memset(&g, 0, sizeof g);
    if (camera) {
        CopyMat(camera->GetViewMatrix(), g.view);
        CopyMat(camera->GetProjectionMatrix(), g.projection);
        const glm::vec3 p = camera->GetPosition();
        g.camera_position[0] = p.x; g.camera_position[1] = p.y; g.camera_position[2] = p.z;
    } else {
        CopyMat(glm::mat4(1.0f), g.view);
        CopyMat(glm::mat4(1.0f), g.projection);
    }
    g.camera_position[3] = 1.0f;
    g.ambient_color_intensity[0] = m_AmbientColor.x;
    g.ambient_color_intensity[1] = m_AmbientColor.y;
    g.ambient_color_intensity[2] = m_AmbientColor.z;
    g.ambient_color_intensity[3] = m_AmbientIntensity;
    glm::vec3 dir = glm::normalize(glm::vec3{-0.5f, -1.0f, -0.3f});  // s_DefaultDirectional* (Renderer.h:464-466)
    glm::vec3 color{1.0f, 0.98f, 0.92f};
    float intensity = 5.0f;
    uint32_t ndir = 0, npt = 0;
    if (m_Registry) {
        for (ECS::Entity e : m_Registry->GetEntities()) {
            if (!m_Registry->HasComponent<LightComponent>(e)) continue;
            const LightComponent& L = m_Registry->GetComponent<LightComponent>(e);
            if (!L.m_Enabled) continue;
            if (L.m_Type == LightComponent::Type::Directional) {
                if (ndir == 0) {
                    if (glm::dot(L.m_Direction, L.m_Direction) > 0.0001f) dir = glm::normalize(L.m_Direction);
                    color = L.m_Color;
                    intensity = std::max(L.m_Intensity, 0.0f);
                }
                ++ndir;
                continue;
            }
            if (L.m_Type == LightComponent::Type::Point) {
                if (npt >= TRI_MAX_POINT_LIGHTS) continue;
                glm::vec3 pos{0.0f};
                if (m_Registry->HasComponent<Transform>(e)) pos = m_Registry->GetComponent<Transform>(e).Position;
                tri_point_light& pl = g.point_lights[npt++];
                pl.position_range[0] = pos.x; pl.position_range[1] = pos.y; pl.position_range[2] = pos.z;
                pl.position_range[3] = std::max(L.m_Range, 0.0f);
                pl.color_intensity[0] = L.m_Color.x; pl.color_intensity[1] = L.m_Color.y;
                pl.color_intensity[2] = L.m_Color.z; pl.color_intensity[3] = std::max(L.m_Intensity, 0.0f);
            }
        }
    }
    const bool fallback = (ndir == 0 && npt == 0);
    g.directional_light_direction[0] = dir.x; g.directional_light_direction[1] = dir.y;
    g.directional_light_direction[2] = dir.z; g.directional_light_direction[3] = 0.0f;
    g.directional_light_color[0] = color.x; g.directional_light_color[1] = color.y;
    g.directional_light_color[2] = color.z; g.directional_light_color[3] = intensity;
    g.light_counts[0] = (ndir > 0 || fallback) ? 1u : 0u;
    g.light_counts[1] = npt;
    // AiBlendConfig (Renderer.cpp:5916-5925): (strength, 1 / width, 1 / height, 1) while an AI frame is held, else 0
    if (m_AiWidth && m_AiHeight) {
        g.ai_blend_config[0] = m_AiBlendStrength;
        g.ai_blend_config[1] = 1.0f / (float)std::max<uint32_t>(m_AiWidth, 1);
        g.ai_blend_config[2] = 1.0f / (float)std::max<uint32_t>(m_AiHeight, 1);
        g.ai_blend_config[3] = 1.0f;
    } else {
        std::memset(g.ai_blend_config, 0, sizeof g.ai_blend_config);
    }
}

bool Renderer::SubmitAiInterpolation(const float* pixels, uint32_t width, uint32_t height, uint32_t channels) {
    ++m_AiGeneration;
    if (!pixels || width == 0 || height == 0 || channels == 0) {  // no frame: the texture is not ready, no blend
        m_AiFrame.clear();
        m_AiWidth = m_AiHeight = 0;
        return true;
    }
    // UploadAiInterpolationToGpu's packing (Renderer.cpp:1572-1590)
    const size_t n = (size_t)width * height;
    m_AiFrame.resize(n * 4);
    for (size_t p = 0; p < n; ++p)
        for (uint32_t ch = 0; ch < 4; ++ch) {
            float v = 0.0f;
            if (ch < channels) v = pixels[p * channels + ch];
            else if (ch == 3) v = 1.0f;  // opaque when the network omits alpha
            v = std::min(std::max(v, 0.0f), 1.0f);
            m_AiFrame[p * 4 + ch] = (uint8_t)std::round(v * 255.0f);
        }
    m_AiWidth = width;
    m_AiHeight = height;
    return true;
}

bool Renderer::BuildShadowConfig(tri_shadow_config& out) {
    std::memset(&out, 0, sizeof out);
    if (!m_Registry || m_ShadowMapSize == 0) return false;
    const LightComponent* sun = nullptr;  // the directional light UpdateUniformBuffer uses (first enabled)
    for (ECS::Entity e : m_Registry->GetEntities()) {
        if (!m_Registry->HasComponent<LightComponent>(e)) continue;
        const LightComponent& L = m_Registry->GetComponent<LightComponent>(e);
        if (L.m_Enabled && L.m_Type == LightComponent::Type::Directional) {
            sun = &L;
            break;
        }
    }
    if (!sun || !sun->m_ShadowCaster) return false;
    glm::vec3 lo{INFINITY}, hi{-INFINITY};  // world box of the drawn meshes
    for (const MeshDrawCommand& cmd : m_MeshDrawCommands) {
        if (!cmd.m_Component || cmd.m_Component->m_MeshIndex >= m_MeshBoundsMin.size()) continue;
        const glm::vec3 a = m_MeshBoundsMin[cmd.m_Component->m_MeshIndex], b = m_MeshBoundsMax[cmd.m_Component->m_MeshIndex];
        if (a.x > b.x) continue;
        for (int k = 0; k < 8; ++k) {
            const glm::vec4 c{(k & 1) ? b.x : a.x, (k & 2) ? b.y : a.y, (k & 4) ? b.z : a.z, 1.0f};
            const glm::vec4 w = cmd.m_ModelMatrix * c;
            for (int ax = 0; ax < 3; ++ax) {
                lo[ax] = std::min(lo[ax], w[ax]);
                hi[ax] = std::max(hi[ax], w[ax]);
            }
        }
    }
    for (const SpriteDrawCommand& cmd : m_SpriteDrawList) {  // sprites cast too: their quad's corners
        if (!m_HasSpriteGeometry) break;
        for (int k = 0; k < 4; ++k) {
            const glm::vec4 c{(k & 1) ? 0.5f : -0.5f, (k & 2) ? 0.5f : -0.5f, 0.0f, 1.0f};
            const glm::vec4 w = cmd.m_ModelMatrix * c;
            for (int ax = 0; ax < 3; ++ax) {
                lo[ax] = std::min(lo[ax], w[ax]);
                hi[ax] = std::max(hi[ax], w[ax]);
            }
        }
    }
    if (lo.x > hi.x) return false;
    glm::vec3 dir{-0.5f, -1.0f, -0.3f};
    if (glm::dot(sun->m_Direction, sun->m_Direction) > 0.0001f) dir = sun->m_Direction;
    const float d[3] = {dir.x, dir.y, dir.z}, mn[3] = {lo.x, lo.y, lo.z}, mx[3] = {hi.x, hi.y, hi.z};
    if (tri_shadow_fit_ortho(d, mn, mx, out.light_view_proj) != TRI_OK) return false;
    out.size = m_ShadowMapSize;
    out.depth_bias = 0.001f;
    out.slope_bias = 2.0f;
    return true;
}

const Camera* Renderer::GetActiveCamera(const ViewportContext& context) const {  // Renderer.cpp:4545-4574
    const uint32_t id = context.m_Info.ViewportID;
    if (id == 1u) return m_EditorCamera;
    if (id == 2u) return (m_RuntimeCameraReady && m_RuntimeCamera) ? m_RuntimeCamera : m_EditorCamera;
    if (m_EditorCamera) return m_EditorCamera;
    return (m_RuntimeCameraReady && m_RuntimeCamera) ? m_RuntimeCamera : nullptr;
}

const Camera* Renderer::GetActiveCamera() const {
    if (m_EditorCamera) return m_EditorCamera;
    return (m_RuntimeCameraReady && m_RuntimeCamera) ? m_RuntimeCamera : nullptr;
}

void Renderer::SetViewport(uint32_t viewportId, const ViewportInfo& info) {
    ViewportContext& ctx = m_Viewports[viewportId];
    ctx.m_Info = info;
    ctx.m_Info.ViewportID = viewportId;
    m_LastViewport = ctx.m_Info;
    m_ActiveViewportId = viewportId;  // Renderer.cpp:2753-2754
}

ViewportInfo Renderer::GetViewport() const { return m_LastViewport; }

glm::mat4 Renderer::GetViewportViewMatrix(uint32_t id) const {
    auto it = m_Viewports.find(id);
    const Camera* cam = it != m_Viewports.end() ? GetActiveCamera(it->second) : GetActiveCamera();
    return cam ? cam->GetViewMatrix() : glm::mat4(1.0f);
}

glm::mat4 Renderer::GetViewportProjectionMatrix(uint32_t id) const {
    auto it = m_Viewports.find(id);
    const Camera* cam = it != m_Viewports.end() ? GetActiveCamera(it->second) : GetActiveCamera();
    return cam ? cam->GetProjectionMatrix() : glm::mat4(1.0f);
}

std::vector<tri_mesh_range> Renderer::GetMeshRanges() const {
    std::vector<tri_mesh_range> ranges(m_MeshDrawInfo.size());
    for (size_t i = 0; i < ranges.size(); ++i)
        ranges[i] = {m_MeshDrawInfo[i].m_FirstIndex, m_MeshDrawInfo[i].m_IndexCount, m_MeshDrawInfo[i].m_BaseVertex,
                     m_MeshDrawInfo[i].m_MaterialIndex};
    if (m_HasSpriteGeometry)
        ranges.push_back({m_SpriteDrawInfo.m_FirstIndex, m_SpriteDrawInfo.m_IndexCount, m_SpriteDrawInfo.m_BaseVertex,
                          m_SpriteDrawInfo.m_MaterialIndex});
    return ranges;
}

bool Renderer::PrepareViewport(ViewportContext& vc) {
    const uint32_t w = (uint32_t)std::max(vc.m_Info.Size.x, 0.0f), h = (uint32_t)std::max(vc.m_Info.Size.y, 0.0f);
    if (w == 0 || h == 0) return false;
    const bool multi = m_Devices.size() > 1;
    if ((vc.m_Ctx || vc.m_Group) && (vc.m_Width != w || vc.m_Height != h)) {  // CreateOrResizeOffscreenResources
        tri_destroy(vc.m_Ctx);
        tri_group_destroy(vc.m_Group);
        vc.m_Ctx = nullptr;
        vc.m_Group = nullptr;
        vc.m_HasImage = false;
    }
    if (!vc.m_Ctx && !vc.m_Group) {
        int rc;
        if (multi) {  // row bands on m_Devices, assembled on the first band's device
            if (h < m_Devices.size()) return false;
            tri_group_config gc{w, h, (uint32_t)m_Devices.size(), 0u, m_Devices.data(), m_RasterFlags, 0u};
            rc = tri_group_create(&gc, &vc.m_Group);
        } else {
            tri_config cfg{w, h, 0, 0, -1, m_RasterFlags};
            rc = tri_create(&cfg, &vc.m_Ctx);
        }
        if (rc != TRI_OK) {
            LogError("viewport target", tri_last_error());
            vc.m_Ctx = nullptr;
            vc.m_Group = nullptr;
            return false;
        }
        vc.m_Width = w;
        vc.m_Height = h;
        vc.m_GeometryGeneration = vc.m_TextureGeneration = vc.m_MaterialGeneration = vc.m_SkyboxGeneration = 0;
        vc.m_AiGeneration = 0;
        vc.m_Shadow = tri_shadow_config{};  // a fresh context starts without the pre-pass and bones
        vc.m_BonePalette.clear();
    }
    const Target t{vc.m_Ctx, vc.m_Group};
    if (vc.m_GeometryGeneration != m_GeometryGeneration && multi) {
        std::vector<tri_geometry*> geos;
        if (!UploadSharedGeometry(geos)) return false;
        if (tri_group_bind_geometry(vc.m_Group, (uint32_t)geos.size(), geos.data()) != TRI_OK) {
            LogError("UploadMeshFromCache", tri_last_error());
            return false;
        }
        vc.m_GeometryGeneration = m_GeometryGeneration;
    }
    if (vc.m_GeometryGeneration != m_GeometryGeneration) {
        // one device copy of the concatenated buffers per generation, bound by every viewport
        if (!m_SharedGeometry && tri_geometry_create(-1, &m_SharedGeometry) != TRI_OK) {
            LogError("UploadMeshFromCache", tri_last_error());
            return false;
        }
        if (m_SharedGeometryGeneration != m_GeometryGeneration) {
            const std::vector<tri_mesh_range> ranges = GetMeshRanges();
            if (tri_geometry_upload(m_SharedGeometry, m_VertexBuffer.data(), m_VertexBuffer.size(), m_IndexBuffer.data(),
                                    m_IndexBuffer.size(), ranges.data(), (uint32_t)ranges.size()) != TRI_OK) {
                LogError("UploadMeshFromCache", tri_last_error());
                return false;
            }
            m_SharedGeometryGeneration = m_GeometryGeneration;
            ++m_GeometryUploads;
        }
        if (tri_bind_geometry(vc.m_Ctx, m_SharedGeometry) != TRI_OK) {
            LogError("UploadMeshFromCache", tri_last_error());
            return false;
        }
        vc.m_GeometryGeneration = m_GeometryGeneration;
    }
    if (vc.m_MaterialGeneration != m_MaterialGeneration) {  // BuildMaterialPayload (Renderer.cpp:5927-5951)
        std::vector<tri_material_record> recs;
        for (const Geometry::Material& m : m_Materials)
            recs.push_back({{m.BaseColorFactor.x, m.BaseColorFactor.y, m.BaseColorFactor.z, m.BaseColorFactor.w},
                            {m.MetallicFactor, m.RoughnessFactor, 1.0f, 0.0f}});
        if (t.Materials(recs.data(), (uint32_t)recs.size()) != TRI_OK) {
            LogError("material buffer", tri_last_error());
            return false;
        }
        vc.m_MaterialGeneration = m_MaterialGeneration;
    }
    if (vc.m_SkyboxGeneration != m_SkyboxGeneration) {
        const bool ok = m_SkyboxCubemap.IsValid();
        if (t.Skybox(ok ? m_SkyboxCubemap.m_PixelData.data() : nullptr, ok ? m_SkyboxCubemap.m_Width : 0) != TRI_OK) {
            LogError("skybox cubemap", tri_last_error());
            return false;
        }
        vc.m_SkyboxGeneration = m_SkyboxGeneration;
    }
    if (vc.m_AiGeneration != m_AiGeneration) {  // the AI frame texture (UploadAiInterpolationToGpu)
        if (t.AiFrame(m_AiWidth ? m_AiFrame.data() : nullptr, m_AiWidth, m_AiHeight) != TRI_OK) {
            LogError("AI frame texture", tri_last_error());
            return false;
        }
        vc.m_AiGeneration = m_AiGeneration;
    }
    if (vc.m_TextureGeneration != m_TextureGeneration) {
        for (size_t s = 0; s < m_TextureSlots.size(); ++s) {
            const Loader::TextureData& tex = m_TextureSlots[s].m_Data;
            if (t.Texture((uint32_t)s, tex.Pixels.data(), (uint32_t)tex.Width, (uint32_t)tex.Height) != TRI_OK) {
                LogError("texture slot", tri_last_error());
                return false;
            }
        }
        vc.m_TextureGeneration = m_TextureGeneration;
    }
    return true;
}

bool Renderer::BuildFrameInputs(uint32_t viewportId, tri_global_ubo& ubo, std::vector<tri_draw>& draws) {
    auto it = m_Viewports.find(viewportId);
    // viewport id 0 without a registered viewport 0: the legacy present pass when no viewport renders
    if (it == m_Viewports.end() && (viewportId != 0 || !m_Viewports.empty())) return false;
    GatherDraws();
    PrepareBonePaletteBuffer();
    UpdateUniformBuffer(it != m_Viewports.end() ? GetActiveCamera(it->second) : GetActiveCamera(), ubo);
    BuildDrawList(draws);
    return true;
}

bool Renderer::SubmitTarget(ViewportContext& vc, const tri_global_ubo& ubo, const std::vector<tri_draw>& draws,
                            const tri_shadow_config& shadow, bool shadowOn) {
    const Target t{vc.m_Ctx, vc.m_Group};
    if (std::memcmp(&vc.m_Shadow, &shadow, sizeof shadow) != 0) {  // pre-pass on / off / refitted
        if (t.Shadow(shadowOn ? &shadow : nullptr) != TRI_OK) {
            LogError("shadow map", tri_last_error());
            return false;
        }
        vc.m_Shadow = shadow;
    }
    if (vc.m_BonePalette != m_BonePalette) {  // the bone SSBO (binding 4) of this frame
        if (t.Bones(m_BonePalette.data(), (uint32_t)(m_BonePalette.size() / 16)) != TRI_OK) {
            LogError("bone palette", tri_last_error());
            return false;
        }
        vc.m_BonePalette = m_BonePalette;
    }
    const float clear[4] = {m_ClearColor.x, m_ClearColor.y, m_ClearColor.z, m_ClearColor.w};
    if (t.Frame(&ubo, clear) != TRI_OK || t.Draws(draws.data(), (uint32_t)draws.size()) != TRI_OK ||
        t.Render() != TRI_OK) {
        LogError("DrawFrame", tri_last_error());
        return false;
    }
    vc.m_HasImage = t.Output(&vc.m_Image) == TRI_OK;
    return true;
}

void Renderer::DrawFrame() {  // Renderer.cpp:733-837
    const auto t0 = std::chrono::steady_clock::now();
    if (!m_Initialised || m_Shutdown) return;
    // the fence (Renderer.cpp:752-772): the reference waits for the previous frame; with n frames in flight, for
    // frame k - n + 1, whose targets this frame is about to reuse
    const uint32_t inflight = m_Devices.size() > 1 ? 1u : m_FramesInFlight;
    while (m_Pending.size() >= inflight) FinishOldestFrame();
    const uint32_t tix = (uint32_t)(m_FrameCount++ % inflight);
    GatherDraws();
    PrepareBonePaletteBuffer();
    std::vector<tri_draw> draws;
    BuildDrawList(draws);
    tri_shadow_config shadow;
    const bool shadowOn = BuildShadowConfig(shadow);
    std::vector<ViewportContext*> submitted;
    tri_global_ubo lastUbo{};
    // RecordCommandBuffer's per-viewport render passes: the other viewports first, the primary one last
    // (Renderer.cpp:5208-5221), so the uniform block left bound is the primary viewport's
    ViewportContext* activeTarget = nullptr;
    auto pass = [&](uint32_t id, ViewportContext& primary) {
        ViewportContext& vc = TargetOf(id, primary, tix);  // this frame's target of the viewport
        if (!PrepareViewport(vc)) return;
        tri_global_ubo ubo;
        UpdateUniformBuffer(GetActiveCamera(vc), ubo);
        if (!SubmitTarget(vc, ubo, draws, shadow, shadowOn)) return;
        lastUbo = ubo;
        submitted.push_back(&vc);
        m_LatestTarget[id] = tix;
        if (id == m_ActiveViewportId) activeTarget = &vc;
    };
    for (auto& it : m_Viewports)
        if (it.first != m_ActiveViewportId) pass(it.first, it.second);
    auto active = m_Viewports.find(m_ActiveViewportId);
    if (active != m_Viewports.end()) pass(active->first, active->second);
    const bool primaryActive = activeTarget != nullptr;
    // Legacy direct-to-swapchain path (Renderer.cpp:5233, :5498-5590): without a rendered primary viewport
    // the skybox, the meshes and the sprites go straight into the present image at the swapchain extent,
    // cleared to the clear colour, with the uniform block last recorded: the null-camera update
    // (GetActiveCamera()) when no viewport rendered (:5223-5226), else the last viewport pass's.
    ViewportContext* legacy = nullptr;
    if (!primaryActive && m_PresentWidth && m_PresentHeight) {
        m_LegacyTarget.m_Info.Size = glm::vec2((float)m_PresentWidth, (float)m_PresentHeight);
        m_LegacyTarget.m_Info.ViewportID = 0;
        if (PrepareViewport(m_LegacyTarget)) {
            tri_global_ubo ubo = lastUbo;
            if (submitted.empty()) UpdateUniformBuffer(GetActiveCamera(), ubo);
            if (SubmitTarget(m_LegacyTarget, ubo, draws, shadow, shadowOn)) {
                legacy = &m_LegacyTarget;
                submitted.push_back(legacy);
            }
        }
    }
    // Primary viewport -> swapchain image, VK_FILTER_LINEAR (Renderer.cpp:5346-5361), stream-ordered behind its pass.
    PendingFrame pf;
    pf.m_Targets = submitted;
    pf.m_Legacy = legacy;
    if (primaryActive && m_PresentWidth && m_PresentHeight) {
        const Target t{activeTarget->m_Ctx, activeTarget->m_Group};
        if (t.Blit(m_PresentWidth, m_PresentHeight) == TRI_OK) {
            pf.m_Blit = activeTarget;
            pf.m_BlitWidth = m_PresentWidth;
            pf.m_BlitHeight = m_PresentHeight;
        } else {
            LogError("present blit", tri_last_error());
        }
    }
    m_Pending.push_back(std::move(pf));
    // no wait here: the next DrawFrame (or a reader) fences this frame, as the reference fences the previous
    // frame's timeline value at the start of DrawFrame (Renderer.cpp:752-772)
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    RecordFrameTiming(ms);
}

void Renderer::FinishFrame() {  // every frame in flight
    while (!m_Pending.empty()) FinishOldestFrame();
}

void Renderer::FinishOldestFrame() {  // the frame fence (Renderer.cpp:744-772)
    if (m_Pending.empty()) return;
    PendingFrame p = std::move(m_Pending.front());
    m_Pending.pop_front();
    // this frame's present replaces the previous one (none if it failed)
    m_PresentSource = nullptr;
    m_PresentGroup = nullptr;
    m_PresentLegacy = false;
    m_PresentedWidth = m_PresentedHeight = 0;
    // A frame that outgrew the bin/clip queues has grown them inside tri_synchronize and is re-rendered (and its
    // present blit redone), so a presented frame is always complete.
    for (ViewportContext* vc : p.m_Targets) {
        const Target t{vc->m_Ctx, vc->m_Group};
        int rc = t.Sync();
        bool rerendered = false;
        for (int retry = 0; rc == TRI_E_OVERFLOW && retry < 3; ++retry) {
            rc = t.Render();
            if (rc == TRI_OK) rc = t.Sync();
            rerendered = true;
        }
        if (rc != TRI_OK) LogError("frame fence", tri_last_error());
        if (rc == TRI_OK) vc->m_HasImage = t.Output(&vc->m_Image) == TRI_OK;  // a re-render moves a group's buffer
        if (vc == p.m_Legacy && rc == TRI_OK) {
            m_PresentSource = vc->m_Ctx;
            m_PresentGroup = vc->m_Group;
            m_PresentLegacy = true;
            m_PresentedWidth = (uint32_t)vc->m_Info.Size.x;  // the target PrepareViewport sized
            m_PresentedHeight = (uint32_t)vc->m_Info.Size.y;
        }
        if (vc == p.m_Blit && rc != TRI_OK) p.m_Blit = nullptr;
        if (vc == p.m_Blit && rerendered) {  // (the first wait covered the blit behind the pass: same stream)
            if (t.Blit(p.m_BlitWidth, p.m_BlitHeight) != TRI_OK || t.Sync() != TRI_OK) {
                LogError("present blit", tri_last_error());
                p.m_Blit = nullptr;
            }
        }
    }
    if (p.m_Blit) {
        m_PresentSource = p.m_Blit->m_Ctx;
        m_PresentGroup = p.m_Blit->m_Group;
        m_PresentedWidth = p.m_BlitWidth;  // the blit's destination extent
        m_PresentedHeight = p.m_BlitHeight;
    }
}

void Renderer::RecordFrameTiming(double ms) {  // Renderer.cpp:6286-6343
    if (m_PerformanceHistory.empty()) return;
    FrameTimingSample s;
    s.FrameMilliseconds = ms;
    s.FramesPerSecond = ms > 0.0 ? 1000.0 / ms : 0.0;
    s.CaptureTime = std::chrono::system_clock::now();
    m_PerformanceHistory[m_PerformanceHistoryNextIndex] = s;
    m_PerformanceHistoryNextIndex = (m_PerformanceHistoryNextIndex + 1) % m_PerformanceHistory.size();
    m_PerformanceSampleCount = std::min(m_PerformanceSampleCount + 1, m_PerformanceHistory.size());
    FrameTimingStats st;
    st.MinimumMilliseconds = std::numeric_limits<double>::max();
    st.MinimumFPS = std::numeric_limits<double>::max();
    double sumMs = 0.0, sumFps = 0.0;
    for (size_t i = 0; i < m_PerformanceSampleCount; ++i) {
        const FrameTimingSample& x = m_PerformanceHistory[i];
        st.MinimumMilliseconds = std::min(st.MinimumMilliseconds, x.FrameMilliseconds);
        st.MaximumMilliseconds = std::max(st.MaximumMilliseconds, x.FrameMilliseconds);
        st.MinimumFPS = std::min(st.MinimumFPS, x.FramesPerSecond);
        st.MaximumFPS = std::max(st.MaximumFPS, x.FramesPerSecond);
        sumMs += x.FrameMilliseconds;
        sumFps += x.FramesPerSecond;
    }
    st.AverageMilliseconds = sumMs / (double)m_PerformanceSampleCount;
    st.AverageFPS = sumFps / (double)m_PerformanceSampleCount;
    m_PerformanceStats = st;
}

void* Renderer::GetViewportTexture(uint32_t viewportId) const {
    const_cast<Renderer*>(this)->FinishFrame();  // the handle's contents are a completed frame
    const ViewportContext* vc = LatestTarget(viewportId);  // the latest frame's target (frames in flight)
    if (!vc || (!vc->m_Ctx && !vc->m_Group) || !vc->m_HasImage) return nullptr;
    return const_cast<tri_image*>(&vc->m_Image);
}

bool Renderer::ReadViewportPixels(uint32_t viewportId, std::vector<uint8_t>& rgba, std::vector<float>* depth) {
    FinishFrame();
    const ViewportContext* latest = LatestTarget(viewportId);  // the latest frame's target (frames in flight)
    if (!latest || (!latest->m_Ctx && !latest->m_Group)) return false;
    const ViewportContext& vc = *latest;
    std::vector<uint8_t> bgra((size_t)vc.m_Width * vc.m_Height * 4);
    std::vector<uint32_t> dbits;
    if (depth) dbits.resize((size_t)vc.m_Width * vc.m_Height);
    if (Target{vc.m_Ctx, vc.m_Group}.Readback(bgra.data(), depth ? dbits.data() : nullptr) != TRI_OK) {
        LogError("readback", tri_last_error());
        return false;
    }
    rgba.resize(bgra.size());
    for (size_t i = 0; i < bgra.size(); i += 4) {  // QuerySwapchainFormatInfo: BGRA -> RGBA
        rgba[i + 0] = bgra[i + 2];
        rgba[i + 1] = bgra[i + 1];
        rgba[i + 2] = bgra[i + 0];
        rgba[i + 3] = bgra[i + 3];
    }
    if (depth) {
        depth->resize(dbits.size());
        std::memcpy(depth->data(), dbits.data(), dbits.size() * 4);
    }
    return true;
}

bool Renderer::ReadPresentPixels(std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height) {
    FinishFrame();
    if (!m_PresentSource && !m_PresentGroup) return false;
    // sized from the extent the present was produced at, not the current SetPresentExtent (a resize between
    // DrawFrame and this read would otherwise under-size the buffer the readback fills)
    std::vector<uint8_t> bgra((size_t)m_PresentedWidth * m_PresentedHeight * 4);
    const Target t{m_PresentSource, m_PresentGroup};
    if ((m_PresentLegacy ? t.Readback(bgra.data(), nullptr) : t.ReadPresent(bgra.data())) != TRI_OK) {
        LogError("present readback", tri_last_error());
        return false;
    }
    rgba.resize(bgra.size());
    for (size_t i = 0; i < bgra.size(); i += 4) {
        rgba[i + 0] = bgra[i + 2];
        rgba[i + 1] = bgra[i + 1];
        rgba[i + 2] = bgra[i + 0];
        rgba[i + 3] = bgra[i + 3];
    }
    width = m_PresentedWidth;
    height = m_PresentedHeight;
    return true;
}

}  // namespace Trident
