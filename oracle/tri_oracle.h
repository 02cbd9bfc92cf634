/*
 * tri_oracle.h — TEST INFRASTRUCTURE. CPU parity oracle for the HIP rasterizer.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.
 * It takes its inputs through the same C-ABI structs as the product (include/tri_raster.h).
 *
 * PARITY STATUS: the reference ships no golden images, no render tests and cannot be built or run
 * here (Windows/MSVC + Vulkan SDK + un-vendored glm; no Vulkan loader/lavapipe/glslang in the
 * image) — see SURVEY.md §4 and §8(c). The oracle is pinned by known-answer tests derived from the
 * reference's shader/glm/pipeline-state definitions (tests/test_oracle_kat.py) and by committed
 * fixtures it generated (tests/golden/); per-pixel parity with the Vulkan driver itself is
 * "parity unpinned".
 */
#ifndef TRI_ORACLE_H
#define TRI_ORACLE_H

#include "../include/tri_raster.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_texture {
    uint32_t slot;
    uint32_t width;
    uint32_t height;
    uint32_t reserved;
    const uint8_t* rgba8_srgb;
} oracle_texture;

typedef struct oracle_scene {
    const tri_vertex* vertices;
    uint64_t vertex_count;
    const uint32_t* indices;
    uint64_t index_count;
    const tri_mesh_range* meshes;
    uint32_t mesh_count;
    uint32_t material_count;
    const tri_material_record* materials;
    const oracle_texture* textures;
    uint32_t texture_count;
    uint32_t bone_count;
    const float* bones;
    const tri_draw* draws;
    uint32_t draw_count;
    uint32_t reserved;
    const tri_global_ubo* ubo;
    float clear_rgba[4];
    /* Skybox cubemap (Renderer.cpp:3818-4110): 6 faces +X,-X,+Y,-Y,+Z,-Z of sky_size^2 RGBA8 sRGB
     * texels, rows top to bottom. NULL / 0 = no skybox pass (background = clear colour). */
    const uint8_t* sky_faces;
    uint32_t sky_size;
    uint32_t sky_reserved;
    /* Shadow-map pre-pass (tri_shadow_config semantics); NULL or size 0 = off.
     * out_shadow_map (nullable) receives the size*size map (float32 depth bits). */
    const tri_shadow_config* shadow;
    uint32_t* out_shadow_map;
    /* AI frame blend (Default.frag:182-191, tri_upload_ai_frame): ai_width x ai_height R8G8B8A8_UNORM texels,
     * rows top to bottom; blends when the UBO's AiBlendConfig asks for it. NULL = no texture. */
    const uint8_t* ai_frame;
    uint32_t ai_width, ai_height;
} oracle_scene;

typedef struct oracle_stats {
    uint64_t triangles_in;
    uint64_t triangles_setup;
    uint64_t triangles_clipped;
    uint64_t fragments_tested;
} oracle_stats;

/* Full-frame render of rows [band_y0, band_y1) (0/0 = all) of a width x height framebuffer.
 * out_bgra: (rows*width) uint32 texels, bytes B,G,R,A. out_depth: float32 bits. threads<=0: 1. */
int oracle_render(const oracle_scene* scene, uint32_t width, uint32_t height, uint32_t band_y0,
                  uint32_t band_y1, int threads, uint32_t* out_bgra, uint32_t* out_depth,
                  oracle_stats* stats);

/* ---- host-side restatements of the reference's CPU code on the path --------------------- */
/* Primitive meshes (Renderer.cpp:72-246). kind: 1 cube, 2 sphere, 3 quad (MeshComponent.h
 * PrimitiveType). Pass NULL buffers to query counts. */
int oracle_build_primitive(int kind, tri_vertex* vertices, uint32_t* vertex_count,
                           uint32_t* indices, uint32_t* index_count);
/* BuildPrimitiveSphereMesh generalised to (rings, segments, radius) — the SURVEY §8(d) C2 scene. */
int oracle_build_uv_sphere(uint32_t rings, uint32_t segments, float radius, tri_vertex* vertices,
                           uint32_t* vertex_count, uint32_t* indices, uint32_t* index_count);
/* ComposeTransform (Renderer.cpp:417-427): T * Rx * Ry * Rz * S, degrees. */
void oracle_compose_transform(const float position[3], const float rotation_deg[3],
                              const float scale[3], float out_model[16]);
/* EditorCamera (EditorCamera.cpp:126-160). projection_type 0 perspective, 1 orthographic. */
void oracle_editor_camera(const float position[3], const float rotation_deg[3], float fov_deg,
                          float viewport_w, float viewport_h, float near_clip, float far_clip,
                          float ortho_size, int projection_type, float out_view[16],
                          float out_proj[16], float out_forward[3]);
/* RuntimeCamera (RuntimeCamera.cpp:166-203). */
void oracle_runtime_camera(const float position[3], const float rotation_deg[3], float fov_deg,
                           float viewport_w, float viewport_h, float near_clip, float far_clip,
                           float ortho_size, int projection_type, float out_view[16],
                           float out_proj[16]);

/* LightComponent (LightComponent.h:19-36) + the light's Transform position. */
typedef struct oracle_light {
    uint32_t type; /* 0 directional, 1 point */
    uint32_t enabled;
    float color[3];
    float intensity;
    float direction[3];
    float range;
    float position[3];
    uint32_t has_transform;
} oracle_light;

/* UpdateUniformBuffer (Renderer.cpp:5822-5925): camera + lights -> GlobalUniformBuffer. */
void oracle_pack_global_ubo(const float view[16], const float proj[16], const float camera_pos[3],
                            int has_camera, const float ambient_color[3], float ambient_intensity,
                            const oracle_light* lights, uint32_t light_count, tri_global_ubo* out);

/* tri_shadow_fit_ortho restated (lookAtRH + orthoRH_ZO over the box corners, 1% margin). */
void oracle_shadow_fit_ortho(const float light_dir[3], const float aabb_min[3], const float aabb_max[3],
                             float out_light_view_proj[16]);

/* The presentation blit (Renderer.cpp:5346-5361, vkCmdBlitImage with VK_FILTER_LINEAR, Vulkan spec
 * "Image Blits": destination texel centres scaled into the source, bilinear over clamp-to-edge taps of
 * UNORM values, UNORM8 round-to-nearest). src: w*h BGRA8 texels, dst: dw*dh. */
void oracle_blit_linear(const uint32_t* src, uint32_t w, uint32_t h, uint32_t* dst, uint32_t dw, uint32_t dh);

#ifdef __cplusplus
}
#endif

#endif
