// trident_app.cpp — flat C driver over Trident::Renderer (see host/include/trident_app.h).
// Entity set-up follows Forge's ApplicationLayer: a primitive spawned with Transform +
// MeshComponent (ApplicationLayer.cpp:677-718), lights as LightComponent entities.
#include "trident_app.h"

#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "trident/Renderer.h"
#include "trident/SceneFile.h"
#include "trident/ModelLoader.h"

#include <algorithm>
#include <array>

using namespace Trident;

struct trident_app {
    Renderer renderer;
    ECS::Registry registry;
    EditorCamera editor;
    RuntimeCamera runtime;
};

namespace {

glm::vec3 V3(const float* p, glm::vec3 dflt) { return p ? glm::vec3{p[0], p[1], p[2]} : dflt; }

template <typename F>
int Guard(trident_app* app, F&& f) {
    if (!app) return TRI_E_INVALID;
    try {
        return f();
    } catch (const std::exception&) {
        return TRI_E_INVALID;
    }
}

}  // namespace

extern "C" {

int trident_app_create(uint32_t raster_flags, trident_app** out) {
    if (!out) return TRI_E_INVALID;
    *out = nullptr;
    try {
        auto* app = new trident_app();
        app->renderer.Init();
        app->renderer.SetRasterFlags(raster_flags);
        app->renderer.SetActiveRegistry(&app->registry);
        app->renderer.SetEditorCamera(&app->editor);
        app->renderer.SetRuntimeCamera(&app->runtime);
        *out = app;
        return TRI_OK;
    } catch (const std::exception&) {
        return TRI_E_OOM;
    }
}

void trident_app_destroy(trident_app* app) {
    if (!app) return;
    app->renderer.Shutdown();
    delete app;
}

int trident_app_append_mesh(trident_app* app, const tri_vertex* vertices, uint32_t vertex_count,
                            const uint32_t* indices, uint32_t index_count, const float base_color[4], float metallic,
                            float roughness, const char* texture_path, uint32_t* mesh_index) {
    return Guard(app, [&] {
        if ((!vertices && vertex_count) || (!indices && index_count) || index_count % 3) return TRI_E_INVALID;
        Geometry::Mesh mesh;
        mesh.Vertices.resize(vertex_count);
        if (vertex_count) std::memcpy(static_cast<void*>(mesh.Vertices.data()), vertices, (size_t)vertex_count * sizeof(Vertex));
        mesh.Indices.assign(indices, indices + index_count);
        mesh.MaterialIndex = 0;  // local to this append; AppendMeshes offsets it
        Geometry::Material mat;
        if (base_color) mat.BaseColorFactor = {base_color[0], base_color[1], base_color[2], base_color[3]};
        mat.MetallicFactor = metallic;
        mat.RoughnessFactor = roughness;
        std::vector<std::string> textures;
        if (texture_path && *texture_path) {
            textures.emplace_back(texture_path);
            mat.BaseColorTextureIndex = 0;
        }
        const size_t before = app->renderer.GetModelCount();
        app->renderer.AppendMeshes({mesh}, {mat}, textures);
        if (mesh_index) *mesh_index = static_cast<uint32_t>(before);
        return TRI_OK;
    });
}

int trident_app_upload_texture(trident_app* app, const char* path, const uint8_t* rgba, uint32_t width,
                               uint32_t height) {
    return Guard(app, [&] {
        if (!path || !rgba || !width || !height) return TRI_E_INVALID;
        Loader::TextureData t;
        t.Width = (int)width;
        t.Height = (int)height;
        t.Pixels.assign(rgba, rgba + (size_t)width * height * 4);
        app->renderer.UploadTexture(path, t);
        return TRI_OK;
    });
}

int trident_app_add_mesh_entity(trident_app* app, int primitive, uint32_t mesh_index, const float position[3],
                                const float rotation_deg[3], const float scale[3], uint32_t* entity) {
    return Guard(app, [&] {
        if (primitive < 0 || primitive > 3) return TRI_E_INVALID;
        const ECS::Entity e = app->registry.CreateEntity();
        Transform& t = app->registry.AddComponent<Transform>(e);
        t.Position = V3(position, glm::vec3{0.0f});
        t.Rotation = V3(rotation_deg, glm::vec3{0.0f});
        t.Scale = V3(scale, glm::vec3{1.0f});
        MeshComponent& m = app->registry.AddComponent<MeshComponent>(e);
        m.m_Primitive = static_cast<MeshComponent::PrimitiveType>(primitive);
        if (primitive == 0) m.m_MeshIndex = mesh_index;
        if (entity) *entity = e;
        return TRI_OK;
    });
}

int trident_app_add_sprite_entity(trident_app* app, const float position[3], const float rotation_deg[3],
                                  const float scale[3], const float tint[4], const float uv_scale[2],
                                  const float uv_offset[2], float tiling, uint32_t* entity) {
    return Guard(app, [&] {
        const ECS::Entity e = app->registry.CreateEntity();
        Transform& t = app->registry.AddComponent<Transform>(e);
        t.Position = V3(position, glm::vec3{0.0f});
        t.Rotation = V3(rotation_deg, glm::vec3{0.0f});
        t.Scale = V3(scale, glm::vec3{1.0f});
        SpriteComponent& sp = app->registry.AddComponent<SpriteComponent>(e);
        if (tint) sp.m_TintColor = {tint[0], tint[1], tint[2], tint[3]};
        if (uv_scale) sp.m_UVScale = {uv_scale[0], uv_scale[1]};
        if (uv_offset) sp.m_UVOffset = {uv_offset[0], uv_offset[1]};
        sp.m_TilingFactor = tiling;
        if (entity) *entity = e;
        return TRI_OK;
    });
}

int trident_app_set_sprite_visible(trident_app* app, uint32_t entity, int visible) {
    return Guard(app, [&] {
        if (!app->registry.HasComponent<SpriteComponent>(entity)) return TRI_E_INVALID;
        app->registry.GetComponent<SpriteComponent>(entity).m_Visible = visible != 0;
        return TRI_OK;
    });
}

int trident_app_entity_sprite(trident_app* app, uint32_t entity, float out[10]) {
    return Guard(app, [&] {
        if (!app->registry.HasComponent<SpriteComponent>(entity)) return TRI_E_INVALID;
        const SpriteComponent& sp = app->registry.GetComponent<SpriteComponent>(entity);
        const float v[10] = {sp.m_TintColor.x, sp.m_TintColor.y, sp.m_TintColor.z, sp.m_TintColor.w, sp.m_UVScale.x,
                             sp.m_UVScale.y, sp.m_UVOffset.x, sp.m_UVOffset.y, sp.m_TilingFactor,
                             sp.m_Visible ? 1.0f : 0.0f};
        std::memcpy(out, v, sizeof v);
        return TRI_OK;
    });
}

int trident_app_set_entity_texture(trident_app* app, uint32_t entity, const char* texture_path) {
    return Guard(app, [&] {
        TextureComponent& t = app->registry.AddComponent<TextureComponent>(entity);
        t.m_TexturePath = texture_path ? texture_path : "";
        t.m_TextureSlot = -1;
        t.m_IsDirty = true;
        return TRI_OK;
    });
}

int trident_app_set_entity_transform(trident_app* app, uint32_t entity, const float position[3],
                                     const float rotation_deg[3], const float scale[3]) {
    return Guard(app, [&] {
        if (!app->registry.HasComponent<Transform>(entity)) return TRI_E_INVALID;
        Transform& t = app->registry.GetComponent<Transform>(entity);
        t.Position = V3(position, t.Position);
        t.Rotation = V3(rotation_deg, t.Rotation);
        t.Scale = V3(scale, t.Scale);
        return TRI_OK;
    });
}

int trident_app_set_entity_visible(trident_app* app, uint32_t entity, int visible) {
    return Guard(app, [&] {
        if (!app->registry.HasComponent<MeshComponent>(entity)) return TRI_E_INVALID;
        app->registry.GetComponent<MeshComponent>(entity).m_Visible = visible != 0;
        return TRI_OK;
    });
}

namespace {
void CopySource(const std::string& src, char* out, uint32_t cap) {
    if (!out || cap == 0) return;
    const size_t n = std::min<size_t>(src.size(), cap - 1);
    std::memcpy(out, src.data(), n);
    out[n] = 0;
}
}  // namespace

int trident_app_set_light_shadow_caster(trident_app* app, uint32_t entity, int caster) {
    return Guard(app, [&] {
        if (!app->registry.HasComponent<LightComponent>(entity)) return TRI_E_INVALID;
        app->registry.GetComponent<LightComponent>(entity).m_ShadowCaster = caster != 0;
        return TRI_OK;
    });
}

int trident_app_set_shadow_map_size(trident_app* app, uint32_t size) {
    return Guard(app, [&] {
        if (size > TRI_MAX_DIM) return TRI_E_INVALID;
        app->renderer.SetShadowMapSize(size);
        return TRI_OK;
    });
}

int trident_app_set_device_count(trident_app* app, uint32_t count, const int32_t* devices) {
    return Guard(app, [&] {
        std::vector<int32_t> devs;
        if (devices && count > 1) devs.assign(devices, devices + count);
        return app->renderer.SetDeviceCount(count, devs) ? TRI_OK : TRI_E_INVALID;
    });
}

int trident_app_shadow_config(trident_app* app, tri_shadow_config* out, int* enabled) {
    return Guard(app, [&] {
        if (!out || !enabled) return TRI_E_INVALID;
        tri_global_ubo ubo;
        std::vector<tri_draw> draws;  // GatherMeshDraws for the current registry state
        app->renderer.BuildFrameInputs(app->renderer.GetActiveViewportId(), ubo, draws);
        *enabled = app->renderer.BuildShadowConfig(*out) ? 1 : 0;
        return TRI_OK;
    });
}

int trident_app_viewport_texture(trident_app* app, uint32_t viewport_id, tri_image* out) {
    return Guard(app, [&] {
        if (!out) return TRI_E_INVALID;
        const void* h = app->renderer.GetViewportTexture(viewport_id);
        if (!h) return TRI_E_STATE;
        *out = *static_cast<const tri_image*>(h);
        return TRI_OK;
    });
}

int trident_app_geometry_uploads(trident_app* app, uint64_t* count) {
    return Guard(app, [&] {
        if (!count) return TRI_E_INVALID;
        *count = app->renderer.GetGeometryUploadCount();
        return TRI_OK;
    });
}

int trident_app_set_assets_dir(trident_app* app, const char* directory, char* source, uint32_t source_cap) {
    return Guard(app, [&] {
        if (!directory) return TRI_E_INVALID;
        app->renderer.SetAssetsDirectory(directory);
        CopySource(app->renderer.GetSkyboxSource(), source, source_cap);
        return TRI_OK;
    });
}

int trident_load_image(const char* path, int flip, uint8_t* rgba, uint64_t capacity, uint32_t* width, uint32_t* height) {
    if (!path || !width || !height) return TRI_E_INVALID;
    try {
        Loader::TextureData t;
        if (flip) {
            t = Loader::TextureLoader::Load(path);
        } else {
            std::array<std::string, 6> one;
            one.fill(path);
            const Loader::CubemapTextureData c = Loader::SkyboxTextureLoader::LoadFromFaces(one);
            if (c.m_Width) {
                t.Width = (int)c.m_Width;
                t.Height = (int)c.m_Height;
                t.Pixels.assign(c.m_PixelData.begin(), c.m_PixelData.begin() + (size_t)c.m_Width * c.m_Height * 4);
            }
        }
        if (t.Width <= 0) return TRI_E_INVALID;
        *width = (uint32_t)t.Width;
        *height = (uint32_t)t.Height;
        if (!rgba) return TRI_OK;
        if (capacity < t.Pixels.size()) return TRI_E_OVERFLOW;
        std::memcpy(rgba, t.Pixels.data(), t.Pixels.size());
        return TRI_OK;
    } catch (...) {
        return TRI_E_INVALID;
    }
}

int trident_load_default_skybox(const char* assets_dir, uint8_t* faces, uint64_t capacity, uint32_t* size, char* source,
                                uint32_t source_cap) {
    if (!assets_dir || !size) return TRI_E_INVALID;
    try {
        std::string src;
        const Loader::CubemapTextureData c = Loader::DiscoverDefaultSkybox(assets_dir, src);
        CopySource(src, source, source_cap);
        *size = c.IsValid() ? c.m_Width : 0;
        if (!faces || !c.IsValid()) return TRI_OK;
        if (capacity < c.m_PixelData.size()) return TRI_E_OVERFLOW;
        std::memcpy(faces, c.m_PixelData.data(), c.m_PixelData.size());
        return TRI_OK;
    } catch (...) {
        return TRI_E_INVALID;
    }
}

int trident_app_set_entity_bones(trident_app* app, uint32_t entity, const float* matrices, uint32_t count) {
    return Guard(app, [&] {
        if (count && !matrices) return TRI_E_INVALID;
        AnimationComponent& a = app->registry.HasComponent<AnimationComponent>(entity)
                                    ? app->registry.GetComponent<AnimationComponent>(entity)
                                    : app->registry.AddComponent<AnimationComponent>(entity);
        a.m_BoneMatrices.resize(count);
        for (uint32_t b = 0; b < count; ++b)
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) a.m_BoneMatrices[b][c][r] = matrices[16 * b + 4 * c + r];
        return TRI_OK;
    });
}

int trident_app_add_light(trident_app* app, int type, const float position[3], const float direction[3],
                          const float color[3], float intensity, float range, int enabled, uint32_t* entity) {
    return Guard(app, [&] {
        if (type != TRIDENT_LIGHT_DIRECTIONAL && type != TRIDENT_LIGHT_POINT) return TRI_E_INVALID;
        const ECS::Entity e = app->registry.CreateEntity();
        Transform& t = app->registry.AddComponent<Transform>(e);
        t.Position = V3(position, glm::vec3{0.0f});
        LightComponent& l = app->registry.AddComponent<LightComponent>(e);
        l.m_Type = static_cast<LightComponent::Type>(type);
        l.m_Direction = V3(direction, l.m_Direction);
        l.m_Color = V3(color, l.m_Color);
        l.m_Intensity = intensity;
        l.m_Range = range;
        l.m_Enabled = enabled != 0;
        if (entity) *entity = e;
        return TRI_OK;
    });
}

int trident_app_set_camera(trident_app* app, int which, const float position[3], const float rotation_deg[3],
                           float fov_deg, float near_clip, float far_clip, int ready) {
    return Guard(app, [&] {
        if (which != 0 && which != 1) return TRI_E_INVALID;
        Camera& cam = which == 0 ? static_cast<Camera&>(app->editor) : static_cast<Camera&>(app->runtime);
        cam.SetPosition(V3(position, cam.GetPosition()));
        cam.SetRotation(V3(rotation_deg, cam.GetRotation()));
        cam.SetFieldOfView(fov_deg);
        cam.SetClipPlanes(near_clip, far_clip);
        if (which == 1) app->renderer.SetRuntimeCameraReady(ready != 0);
        return TRI_OK;
    });
}

int trident_app_set_viewport(trident_app* app, uint32_t viewport_id, uint32_t width, uint32_t height) {
    return Guard(app, [&] {
        if (width > TRI_MAX_DIM || height > TRI_MAX_DIM) return TRI_E_INVALID;
        ViewportInfo info;
        info.Size = {(float)width, (float)height};
        app->renderer.SetViewport(viewport_id, info);
        // The viewport panel resizes the camera that renders into it (ApplicationLayer.cpp:253-290).
        if (width && height) {
            const glm::vec2 s{(float)width, (float)height};
            if (viewport_id == 2u) app->runtime.SetViewportSize(s);
            else app->editor.SetViewportSize(s);
        }
        return TRI_OK;
    });
}

int trident_app_set_clear_color(trident_app* app, const float rgba[4]) {
    return Guard(app, [&] {
        if (!rgba) return TRI_E_INVALID;
        app->renderer.SetClearColor({rgba[0], rgba[1], rgba[2], rgba[3]});
        return TRI_OK;
    });
}

int trident_app_set_skybox(trident_app* app, const uint8_t* faces, uint32_t size) {
    return Guard(app, [&] {
        if (!faces || !size) return TRI_E_INVALID;
        Loader::CubemapTextureData d;
        d.m_Width = d.m_Height = size;
        d.m_PixelData.assign(faces, faces + 6ull * size * size * 4);
        return app->renderer.SetSkyboxCubemap(d) ? TRI_OK : TRI_E_INVALID;
    });
}

int trident_app_import_model(trident_app* app, const char* path, uint32_t* entities, uint32_t capacity,
                             uint32_t* count) {
    return Guard(app, [&] {
        if (!path) return TRI_E_INVALID;
        std::vector<ECS::Entity> spawned;
        const bool ok = ImportModel(app->renderer, app->registry, path, &spawned);
        if (count) *count = (uint32_t)spawned.size();
        for (size_t i = 0; entities && i < spawned.size() && i < capacity; ++i) entities[i] = spawned[i];
        return ok ? TRI_OK : TRI_E_INVALID;
    });
}

int trident_app_save_scene(trident_app* app, const char* path, const char* scene_name) {
    return Guard(app, [&] {
        if (!path) return TRI_E_INVALID;
        Scene scene(app->registry, &app->renderer, scene_name ? scene_name : "Untitled");
        scene.Save(path);
        return TRI_OK;
    });
}

int trident_app_load_scene(trident_app* app, const char* path, uint32_t* entity_count) {
    return Guard(app, [&] {
        if (!path) return TRI_E_INVALID;
        Scene scene(app->registry, &app->renderer);
        if (!scene.Load(path)) return TRI_E_INVALID;
        if (entity_count) *entity_count = (uint32_t)scene.GetLoadedEntityCount();
        return TRI_OK;
    });
}

int trident_app_use_scene_camera(trident_app* app) {
    return Guard(app, [&] {
        ECS::Entity chosen = 0;
        bool found = false;
        for (ECS::Entity e : app->registry.GetEntities()) {
            if (!app->registry.HasComponent<CameraComponent>(e)) continue;
            if (!found || app->registry.GetComponent<CameraComponent>(e).m_Primary) {
                const bool primary = app->registry.GetComponent<CameraComponent>(e).m_Primary;
                if (!found || primary) chosen = e;
                found = true;
                if (primary) break;
            }
        }
        if (!found) return TRI_E_INVALID;
        const CameraComponent& c = app->registry.GetComponent<CameraComponent>(chosen);
        RuntimeCamera& cam = app->runtime;
        if (app->registry.HasComponent<Transform>(chosen)) {
            const Transform& t = app->registry.GetComponent<Transform>(chosen);
            cam.SetPosition(t.Position);
            cam.SetRotation(t.Rotation);
        }
        cam.SetProjectionType(c.m_ProjectionType);
        cam.SetFieldOfView(c.m_FieldOfView);
        cam.SetOrthographicSize(c.m_OrthographicSize);
        cam.SetClipPlanes(c.m_NearClip, c.m_FarClip);
        app->renderer.SetRuntimeCameraReady(true);
        return TRI_OK;
    });
}

int trident_app_entity_transform(trident_app* app, uint32_t entity, float out[9]) {
    return Guard(app, [&] {
        if (!out || !app->registry.HasComponent<Transform>(entity)) return TRI_E_INVALID;
        const Transform& t = app->registry.GetComponent<Transform>(entity);
        const float v[9] = {t.Position.x, t.Position.y, t.Position.z, t.Rotation.x, t.Rotation.y,
                            t.Rotation.z, t.Scale.x, t.Scale.y, t.Scale.z};
        std::memcpy(out, v, sizeof v);
        return TRI_OK;
    });
}

int trident_app_entity_mesh(trident_app* app, uint32_t entity, uint64_t out[3]) {
    return Guard(app, [&] {
        if (!out || !app->registry.HasComponent<MeshComponent>(entity)) return TRI_E_INVALID;
        const MeshComponent& m = app->registry.GetComponent<MeshComponent>(entity);
        out[0] = (uint64_t)m.m_MeshIndex;
        out[1] = (uint64_t)m.m_Primitive;
        out[2] = (uint64_t)m.m_SourceMeshIndex;
        return TRI_OK;
    });
}

int trident_app_entity_count(trident_app* app, uint32_t* count) {
    return Guard(app, [&] {
        if (!count) return TRI_E_INVALID;
        *count = (uint32_t)app->registry.GetEntities().size();
        return TRI_OK;
    });
}

int trident_app_set_present_extent(trident_app* app, uint32_t width, uint32_t height) {
    return Guard(app, [&] {
        if (width > TRI_MAX_DIM || height > TRI_MAX_DIM) return TRI_E_INVALID;
        app->renderer.SetPresentExtent(width, height);
        return TRI_OK;
    });
}

int trident_app_set_ai_blend_strength(trident_app* app, float strength) {
    return Guard(app, [&] {
        app->renderer.SetAiBlendStrength(strength);
        return TRI_OK;
    });
}

int trident_app_submit_ai_frame(trident_app* app, const float* pixels, uint32_t width, uint32_t height, uint32_t channels) {
    return Guard(app, [&] {
        if (width > TRI_MAX_DIM || height > TRI_MAX_DIM || channels > 4) return TRI_E_INVALID;
        return app->renderer.SubmitAiInterpolation(pixels, width, height, channels) ? TRI_OK : TRI_E_INVALID;
    });
}

int trident_app_read_present(trident_app* app, uint8_t* rgba, uint32_t width, uint32_t height) {
    return Guard(app, [&] {
        if (!rgba) return TRI_E_INVALID;
        std::vector<uint8_t> px;
        uint32_t w = 0, h = 0;
        if (!app->renderer.ReadPresentPixels(px, w, h)) return TRI_E_STATE;
        if (w != width || h != height) return TRI_E_INVALID;
        std::memcpy(rgba, px.data(), px.size());
        return TRI_OK;
    });
}

int trident_app_draw_frame(trident_app* app) {
    return Guard(app, [&] {
        app->renderer.DrawFrame();
        return TRI_OK;
    });
}

int trident_app_set_frames_in_flight(trident_app* app, uint32_t n) {
    return Guard(app, [&] {
        if (n == 0 || n > 4) return TRI_E_INVALID;
        app->renderer.SetFramesInFlight(n);
        return TRI_OK;
    });
}

int trident_app_finish_frame(trident_app* app) {
    return Guard(app, [&] {
        app->renderer.FinishFrame();
        return TRI_OK;
    });
}

int trident_app_read_pixels(trident_app* app, uint32_t viewport_id, uint8_t* rgba, float* depth) {
    return Guard(app, [&] {
        if (!rgba) return TRI_E_INVALID;
        std::vector<uint8_t> px;
        std::vector<float> d;
        if (!app->renderer.ReadViewportPixels(viewport_id, px, depth ? &d : nullptr)) return TRI_E_STATE;
        std::memcpy(rgba, px.data(), px.size());
        if (depth) std::memcpy(depth, d.data(), d.size() * sizeof(float));
        return TRI_OK;
    });
}

int trident_app_frame_inputs(trident_app* app, uint32_t viewport_id, tri_global_ubo* ubo, tri_draw* draws,
                             uint32_t capacity, uint32_t* draw_count) {
    return Guard(app, [&] {
        if (!ubo || !draw_count) return TRI_E_INVALID;
        std::vector<tri_draw> list;
        if (!app->renderer.BuildFrameInputs(viewport_id, *ubo, list)) return TRI_E_STATE;
        *draw_count = (uint32_t)list.size();
        if (list.size() > capacity || (!draws && !list.empty())) return list.size() > capacity ? TRI_E_OVERFLOW : TRI_E_INVALID;
        if (!list.empty()) std::memcpy(draws, list.data(), list.size() * sizeof(tri_draw));
        return TRI_OK;
    });
}

int trident_app_geometry(trident_app* app, const tri_vertex** vertices, size_t* vertex_count,
                         const uint32_t** indices, size_t* index_count, tri_mesh_range* ranges, uint32_t capacity,
                         uint32_t* range_count) {
    return Guard(app, [&] {
        if (!vertices || !vertex_count || !indices || !index_count || !range_count) return TRI_E_INVALID;
        *vertices = app->renderer.GetVertexBuffer().data();
        *vertex_count = app->renderer.GetVertexBuffer().size();
        *indices = app->renderer.GetIndexBuffer().data();
        *index_count = app->renderer.GetIndexBuffer().size();
        const std::vector<tri_mesh_range> r = app->renderer.GetMeshRanges();
        *range_count = (uint32_t)r.size();
        if (r.size() > capacity) return TRI_E_OVERFLOW;
        if (!r.empty() && ranges) std::memcpy(ranges, r.data(), r.size() * sizeof(tri_mesh_range));
        return TRI_OK;
    });
}

int trident_app_materials(trident_app* app, tri_material_record* out, uint32_t capacity, uint32_t* count) {
    return Guard(app, [&] {
        if (!count) return TRI_E_INVALID;
        const auto& mats = app->renderer.GetMaterials();
        *count = (uint32_t)mats.size();
        if (mats.size() > capacity) return TRI_E_OVERFLOW;
        for (size_t i = 0; i < mats.size() && out; ++i)
            out[i] = {{mats[i].BaseColorFactor.x, mats[i].BaseColorFactor.y, mats[i].BaseColorFactor.z,
                       mats[i].BaseColorFactor.w},
                      {mats[i].MetallicFactor, mats[i].RoughnessFactor, 1.0f, 0.0f}};
        return TRI_OK;
    });
}

int trident_app_frame_timing(trident_app* app, double out[7]) {
    return Guard(app, [&] {
        if (!out) return TRI_E_INVALID;
        const FrameTimingStats& s = app->renderer.GetFrameTimingStats();
        out[0] = s.MinimumMilliseconds;
        out[1] = s.MaximumMilliseconds;
        out[2] = s.AverageMilliseconds;
        out[3] = s.MinimumFPS;
        out[4] = s.MaximumFPS;
        out[5] = s.AverageFPS;
        out[6] = (double)app->renderer.GetFrameTimingHistoryCount();
        return TRI_OK;
    });
}

}  // extern "C"
