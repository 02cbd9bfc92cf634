/* trident_app.h — a flat C driver over the C++ Trident::Renderer shim (host/include/trident/ headers).
 *
 * It plays the part of Trident-Forge's ApplicationLayer (Trident-Forge/src/Layer/ApplicationLayer.cpp)
 * for tests and tools that are not C++: it owns one ECS::Registry, an EditorCamera and a
 * RuntimeCamera, and forwards to RenderCommand. Everything below the shim is the drop-in C-ABI in
 * include/tri_raster.h. All functions return TRI_OK or a negative TRI_E_* code.
 */
#ifndef TRIDENT_APP_H
#define TRIDENT_APP_H

#include <stddef.h>
#include <stdint.h>

#include "../../../include/tri_raster.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct trident_app trident_app;

/* primitive: 0 none, 1 cube, 2 sphere, 3 quad (MeshComponent::PrimitiveType) */
enum { TRIDENT_PRIMITIVE_NONE = 0, TRIDENT_PRIMITIVE_CUBE = 1, TRIDENT_PRIMITIVE_SPHERE = 2, TRIDENT_PRIMITIVE_QUAD = 3 };
enum { TRIDENT_LIGHT_DIRECTIONAL = 0, TRIDENT_LIGHT_POINT = 1 };

int trident_app_create(uint32_t raster_flags, trident_app** out);
void trident_app_destroy(trident_app* app);

/* Renderer::AppendMeshes with one mesh + one material; returns the mesh index in *mesh_index. */
int trident_app_append_mesh(trident_app* app, const tri_vertex* vertices, uint32_t vertex_count,
                            const uint32_t* indices, uint32_t index_count, const float base_color[4],
                            float metallic, float roughness, const char* texture_path, uint32_t* mesh_index);
int trident_app_upload_texture(trident_app* app, const char* path, const uint8_t* rgba, uint32_t width,
                               uint32_t height);

/* Entity with Transform + MeshComponent (primitive, or mesh_index when primitive == 0). */
int trident_app_add_mesh_entity(trident_app* app, int primitive, uint32_t mesh_index, const float position[3],
                                const float rotation_deg[3], const float scale[3], uint32_t* entity);
int trident_app_set_entity_texture(trident_app* app, uint32_t entity, const char* texture_path);
/* Entity with Transform + SpriteComponent (tint, UV scale / offset, tiling; NULL = the component's
 * defaults); drawn after the meshes (GatherSpriteDraws / DrawSprites, Renderer.cpp:2996-3089). A texture
 * goes on with trident_app_set_entity_texture. */
int trident_app_add_sprite_entity(trident_app* app, const float position[3], const float rotation_deg[3],
                                  const float scale[3], const float tint[4], const float uv_scale[2],
                                  const float uv_offset[2], float tiling, uint32_t* entity);
int trident_app_set_sprite_visible(trident_app* app, uint32_t entity, int visible);
/* SpriteComponent of an entity: tint[4], uv_scale[2], uv_offset[2], tiling, visible. */
int trident_app_entity_sprite(trident_app* app, uint32_t entity, float out[10]);
int trident_app_set_entity_transform(trident_app* app, uint32_t entity, const float position[3],
                                     const float rotation_deg[3], const float scale[3]);
int trident_app_set_entity_visible(trident_app* app, uint32_t entity, int visible);
/* AnimationComponent::m_BoneMatrices of an entity (count column-major mat4s; 0 clears the palette):
 * the draw skins with them (PrepareBonePaletteBuffer, Renderer.cpp:3168-3245). */
int trident_app_set_entity_bones(trident_app* app, uint32_t entity, const float* matrices, uint32_t count);
int trident_app_add_light(trident_app* app, int type, const float position[3], const float direction[3],
                          const float color[3], float intensity, float range, int enabled, uint32_t* entity);

/* LightComponent::m_ShadowCaster of a light entity (LightComponent.h:33): a shadow-casting first
 * directional light turns on the shadow-map pre-pass (Renderer::SetShadowMapSize, default 2048). */
int trident_app_set_light_shadow_caster(trident_app* app, uint32_t entity, int caster);
int trident_app_set_shadow_map_size(trident_app* app, uint32_t size);
/* Renderer::SetDeviceCount: with count > 1 every viewport renders as `count` row bands on `devices`
 * (NULL = 0 .. count-1; ordinals may repeat) assembled on the first band's device (tri_group). */
int trident_app_set_device_count(trident_app* app, uint32_t count, const int32_t* devices);
/* The pre-pass configuration DrawFrame would use now (*enabled = 0 when there is none). */
int trident_app_shadow_config(trident_app* app, tri_shadow_config* out, int* enabled);

/* which: 0 editor, 1 runtime. Runtime camera readiness follows `ready`. */
int trident_app_set_camera(trident_app* app, int which, const float position[3], const float rotation_deg[3],
                           float fov_deg, float near_clip, float far_clip, int ready);
int trident_app_set_viewport(trident_app* app, uint32_t viewport_id, uint32_t width, uint32_t height);
int trident_app_set_clear_color(trident_app* app, const float rgba[4]);
/* Renderer::SetSkyboxCubemap: faces [6][size][size] RGBA8 sRGB (+X,-X,+Y,-Y,+Z,-Z). */
int trident_app_set_skybox(trident_app* app, const uint8_t* faces, uint32_t size);

/* Renderer::SetAssetsDirectory: the directory whose Skyboxes/ CreateSkyboxCubemap searches
 * (Renderer.cpp:3830-3927); re-runs the discovery. *source (nullable, source_cap bytes) names the result. */
int trident_app_set_assets_dir(trident_app* app, const char* directory, char* source, uint32_t source_cap);

/* The loaders on their own (no app): TextureLoader::Load (flip = 1: stb's flip-on-load for 2D textures)
 * or one cube face (flip = 0). rgba = NULL queries the size; else capacity must hold width*height*4. */
int trident_load_image(const char* path, int flip, uint8_t* rgba, uint64_t capacity, uint32_t* width,
                       uint32_t* height);
/* DiscoverDefaultSkybox(assets_dir): faces [6][size][size] RGBA8 (+X,-X,+Y,-Y,+Z,-Z); faces = NULL
 * queries *size; *size = 0 when nothing valid was found. */
int trident_load_default_skybox(const char* assets_dir, uint8_t* faces, uint64_t capacity, uint32_t* size,
                                char* source, uint32_t source_cap);

/* Model import as Forge's drop handler (ModelLoader: .obj/.mtl, .gltf, .glb): entities per mesh
 * instance. Up to `capacity` spawned entity ids go to `entities`; *count gets how many were spawned. */
int trident_app_import_model(trident_app* app, const char* path, uint32_t* entities, uint32_t capacity,
                             uint32_t* count);
/* `.trident` scene files (Scene::Save / Scene::Load, ECS/Scene.cpp:80-151). Load replaces every
 * entity and rebuilds imported geometry from the SourceAsset paths; *entity_count may be null. */
int trident_app_save_scene(trident_app* app, const char* path, const char* scene_name);
int trident_app_load_scene(trident_app* app, const char* path, uint32_t* entity_count);
/* The runtime camera follows the scene's primary CameraComponent entity (the first camera entity
 * when none is primary): Transform position / rotation, projection, field of view, clip planes. */
int trident_app_use_scene_camera(trident_app* app);
/* Component inspection for tests: Transform (9 floats) and MeshComponent {mesh_index, primitive,
 * source mesh index} of an entity; TRI_E_INVALID when absent. */
int trident_app_entity_transform(trident_app* app, uint32_t entity, float out[9]);
int trident_app_entity_mesh(trident_app* app, uint32_t entity, uint64_t out[3]);
int trident_app_entity_count(trident_app* app, uint32_t* count);

/* Renderer::SetPresentExtent: DrawFrame then blits the active (last SetViewport) viewport onto a
 * width x height present image (VK_FILTER_LINEAR); 0 x 0 disables. */
int trident_app_set_present_extent(trident_app* app, uint32_t width, uint32_t height);
/* Renderer::SetAiBlendStrength / SubmitAiInterpolation (Default.frag's AI frame blend): width * height * channels
 * floats in [0, 1] (NULL or a zero extent drops the frame). */
int trident_app_set_ai_blend_strength(trident_app* app, float strength);
int trident_app_submit_ai_frame(trident_app* app, const float* pixels, uint32_t width, uint32_t height, uint32_t channels);
int trident_app_read_present(trident_app* app, uint8_t* rgba, uint32_t width, uint32_t height);

int trident_app_draw_frame(trident_app* app);
/* Renderer::FinishFrame: wait for the frame the last draw_frame submitted (the next draw_frame does it first). */
int trident_app_finish_frame(trident_app* app);
/* Renderer::SetFramesInFlight (1..4; 1 = the reference's pacing). */
int trident_app_set_frames_in_flight(trident_app* app, uint32_t n);
/* Renderer::GetViewportTexture: copies the viewport's image handle (TRI_E_STATE before its first frame). */
int trident_app_viewport_texture(trident_app* app, uint32_t viewport_id, tri_image* out);
/* Renderer::GetGeometryUploadCount. */
int trident_app_geometry_uploads(trident_app* app, uint64_t* count);
int trident_app_read_pixels(trident_app* app, uint32_t viewport_id, uint8_t* rgba, float* depth /* nullable */);

/* Frame inputs DrawFrame would submit for a viewport (host-only). */
int trident_app_frame_inputs(trident_app* app, uint32_t viewport_id, tri_global_ubo* ubo, tri_draw* draws,
                             uint32_t capacity, uint32_t* draw_count);
/* The concatenated geometry (pointers stay valid until the next mesh change). */
int trident_app_geometry(trident_app* app, const tri_vertex** vertices, size_t* vertex_count,
                         const uint32_t** indices, size_t* index_count, tri_mesh_range* ranges, uint32_t capacity,
                         uint32_t* range_count);
int trident_app_materials(trident_app* app, tri_material_record* out, uint32_t capacity, uint32_t* count);
/* Renderer::GetFrameTimingStats: min/max/avg ms, min/max/avg fps, sample count. */
int trident_app_frame_timing(trident_app* app, double out[7]);

#ifdef __cplusplus
}
#endif

#endif /* TRIDENT_APP_H */
