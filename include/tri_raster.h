/*
 * tri_raster.h — C-ABI drop-in boundary for the MI355X (gfx950) HIP software rasterizer that
 * replaces Trident's Vulkan graphics-pipeline stage (the work recorded by
 * Renderer::RecordCommandBuffer, Trident/src/Renderer/Renderer.cpp:4890-5636, and executed by the
 * driver with Default.vert / Default.frag).
 *
 * Plain C: no torch, no HIP types in the signatures. Device memory, streams and events are owned by
 * the context; callers pass host pointers (copied) except in tri_bind_output / tri_set_stream, which
 * take opaque device pointers / a hipStream_t as void*.
 *
 * Every entry point returns an int status (TRI_OK == 0, negative on error) and records a message
 * readable through tri_last_error() — mirroring the reference's "bool + TR_CORE_* log, no exceptions
 * on the frame path" convention (Renderer.cpp:779-824). One host thread per context; not thread-safe
 * (Application.cpp:82-134 is a single render thread).
 *
 * Which reference interface each entry point replaces is noted next to it. The C++
 * Trident::Renderer-compatible shim (3d-renderer_amd/host/) calls these; INTEGRATION.md shows the
 * binding a Trident maintainer would add.
 */
#ifndef TRI_RASTER_H
#define TRI_RASTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRI_RASTER_ABI_VERSION 2 /* 2: tri_geometry, tri_image, shadow pre-pass, tri_group fences */

/* ---- status codes ---------------------------------------------------------------------- */
#define TRI_OK 0
#define TRI_E_INVALID (-1)     /* bad argument (null, out of range, size mismatch)              */
#define TRI_E_HIP (-2)         /* HIP runtime error (no device, launch failure, ...)            */
#define TRI_E_OOM (-3)         /* device allocation failed                                      */
#define TRI_E_OVERFLOW (-4)    /* a frame overflowed an internal bin/clip buffer; buffers were   *
                                * grown, re-render the frame                                    */
#define TRI_E_UNSUPPORTED (-5) /* combination outside the path (AI blend + shadow pre-pass)     */
#define TRI_E_STATE (-6)       /* call order violated (e.g. render before geometry upload)      */
#define TRI_E_TIMEOUT (-7)     /* a multi-GPU exchange missed its deadline (communicators aborted) */

/* ---- limits mirrored from the reference ----------------------------------------------- */
#define TRI_MAX_POINT_LIGHTS 8   /* kMaxPointLights, UniformBuffer.h:7                           */
#define TRI_MAX_TEXTURE_SLOTS 256 /* Pipeline.h:18 (sampler2D BaseColorSamplers[256])            */
#define TRI_MAX_BONE_INFLUENCES 4 /* Vertex::MaxBoneInfluences, Vertex.h:11                      */
#define TRI_MAX_DIM 8192          /* framebuffer width/height limit (guard-band fixed point)    */

/* ---- GPU ABI structs: byte-identical to the reference's --------------------------------- */

/* Vertex (Trident/src/Renderer/Vertex.h:9-78): glm without SIMD alignment => 100-byte stride.
 * Offsets: Position 0, Normal 12, Tangent 24, Bitangent 36, Color 48, TexCoord 60,
 * BoneIndices 68, BoneWeights 84. */
typedef struct tri_vertex {
    float position[3];
    float normal[3];
    float tangent[3];
    float bitangent[3];
    float color[3];
    float texcoord[2];
    int32_t bone_indices[4];
    float bone_weights[4];
} tri_vertex;

/* MeshDrawInfo (Renderer.h:293-299): one per uploaded mesh; indices are mesh-local and
 * base_vertex is added at draw time (Renderer.cpp:2032-2038, :2062-2077). */
typedef struct tri_mesh_range {
    uint32_t first_index;
    uint32_t index_count;
    int32_t base_vertex;
    int32_t material_index;
} tri_mesh_range;

/* RenderablePushConstant (Trident/src/Renderer/RenderData.h:14-30), 128 bytes. */
typedef struct tri_push_constant {
    float model[16]; /* column-major glm::mat4 */
    float tint[4];
    float texture_scale[2];
    float texture_offset[2];
    float tiling_factor;
    int32_t texture_slot;
    int32_t use_material_override;
    float sort_bias;
    int32_t material_index;
    int32_t padding0;
    int32_t bone_offset;
    int32_t bone_count;
} tri_push_constant;

/* One vkCmdDrawIndexed(IndexCount, 1, FirstIndex, BaseVertex, 0) + its push constant
 * (Renderer.cpp:5110-5151). mesh_index selects a tri_mesh_range. */
typedef struct tri_draw {
    uint32_t mesh_index;
    uint32_t reserved[3];
    tri_push_constant pc;
} tri_draw;

/* PointLightUniform (UniformBuffer.h:10-14). */
typedef struct tri_point_light {
    float position_range[4];  /* xyz = world position, w = radius */
    float color_intensity[4]; /* rgb = colour, w = intensity      */
} tri_point_light;

/* GlobalUniformBuffer (UniformBuffer.h:17-28), 480 bytes std140, as written by
 * Renderer::UpdateUniformBuffer (Renderer.cpp:5822-6051). */
typedef struct tri_global_ubo {
    float view[16];
    float projection[16];
    float camera_position[4];
    float ambient_color_intensity[4];
    float directional_light_direction[4];
    float directional_light_color[4];
    uint32_t light_counts[4];
    float ai_blend_config[4];
    tri_point_light point_lights[TRI_MAX_POINT_LIGHTS];
} tri_global_ubo;

/* MaterialUniformBuffer (UniformBuffer.h:31-35). Only record 0 is read by Default.frag:58-62. */
typedef struct tri_material_record {
    float base_color_factor[4];
    float material_factors[4]; /* x metallic, y roughness, z ambient strength, w reserved */
} tri_material_record;

/* Context configuration. The viewport is always the full width x height framebuffer
 * (Renderer.cpp:5062-5069: x=y=0, minDepth 0, maxDepth 1). band_y0/band_y1 select the row band
 * this context rasterizes (multi-GPU screen partition); 0/0 means all rows. */
typedef struct tri_config {
    uint32_t width;
    uint32_t height;
    uint32_t band_y0;
    uint32_t band_y1;
    int32_t device; /* HIP device ordinal; -1 = current device */
    uint32_t flags; /* TRI_FLAG_* */
} tri_config;

#define TRI_FLAG_NO_DEPTH_OUTPUT 0x1u /* skip the depth write (reference storeOp DONT_CARE) */
#define TRI_FLAG_EXACT_SHADING 0x2u   /* Default.frag with IEEE div/sqrt/powf in the oracle's order *
                                       * (default: hardware rcp/rsq/exp/log; both within 1 LSB)     */
#define TRI_FLAG_CLUSTER_CULL 0x4u    /* cull 512-triangle clusters by their projected boxes on whole *
                                       * frames too (row-band contexts always do); output unchanged  */

/* Per-stage accumulated device time (HIP events on the context stream) and last-frame counters. */
typedef struct tri_timing {
    uint64_t frames;        /* frames timed since the last reset                  */
    double ms_vertex;       /* vs_transform (+ per-vertex divide / viewport / snap) */
    double ms_setup;        /* tri_setup_bin (setup + cull + per-bin queues)       */
    double ms_shadow;       /* shadow-map depth raster (0 without the pre-pass; its set-up/binning  *
                             * shares the set-up pass and is in ms_setup, as is clipping)             */
    double ms_raster;       /* tile_raster_shade (coverage + early-Z + PBR + store) */
    double ms_frame;        /* first kernel start to last kernel end              */
    double reserved;
} tri_timing;

typedef struct tri_frame_stats {
    uint64_t triangles_in;      /* primitives submitted                            */
    uint64_t triangles_setup;   /* primitives surviving clip/cull/snap             */
    uint64_t triangles_clipped; /* primitives that went through geometric clipping */
    uint64_t bin_entries;       /* (triangle, bin) pairs                           */
    uint64_t vertices_shaded;   /* vertex-shader invocations                       */
    uint32_t bins_x, bins_y, bin_size;
    uint32_t path;              /* TRI_PATH_* bits: the fragment path the last frame took (diagnostics) */
} tri_frame_stats;

/* tri_frame_stats.path bits */
#define TRI_PATH_ONE_DRAW   0x1u  /* one draw over a 1x1 texture slot: the single-draw solid instantiation */
#define TRI_PATH_VARY_OBJ   0x2u  /* object-space varyings (no per-frame varying writes)                   */
#define TRI_PATH_OBJ_XFORM  0x4u  /* ... carried through a non-identity model / normal matrix per pixel     */
#define TRI_PATH_OBJ_UCOL   0x8u  /* ... one vertex colour for the whole geometry                           */
#define TRI_PATH_SHADOW    0x10u  /* the shadow-map pre-pass ran                                            */
#define TRI_PATH_OBJ48     0x20u  /* object-space varyings outside the single-draw solid instantiation      */
#define TRI_PATH_IDX_ROUTE 0x40u  /* several draws: vertex slots from the index buffer, no per-primitive record */

/* Shadow-map pre-pass (BASELINE.json config 5). The reference reserves the switch
 * (LightComponent::m_ShadowCaster, Trident/src/ECS/Components/LightComponent.h:33) but renders no shadow
 * map, so this pass is defined here and restated by the oracle:
 *   - every frame, before the main pass, the draws' triangles are rasterised depth-only into a
 *     size x size D32 map by the orthographic light transform `light_view_proj` (column-major, affine:
 *     its last row must be exactly 0,0,0,1): texel (i, j) covers light NDC x in [2i/size - 1, 2(i+1)/size - 1),
 *     y likewise; the main pass's raster rules (8-bit snap, top-left fill, plane depth), no culling,
 *     depth clamp instead of near/far clipping, a slope-scaled depth bias (Vulkan depthBiasSlopeFactor
 *     semantics: + slope_bias * the triangle's largest depth change per texel, before the clamp),
 *     LEQUAL (the map keeps the minimum depth, clear 1.0);
 *     triangles reaching beyond the guard band (|x|, |y| > 2*16000/size - 1 in light NDC) cast nothing;
 *   - in Default.frag the directional light's radiance is scaled by the fraction of a 2x2 bilinear
 *     depth compare (zref - depth_bias <= map) that passes, zref being the fragment's light-space depth;
 *     fragments outside the map are lit. Point lights and ambient are unchanged. */
typedef struct tri_shadow_config {
    uint32_t size;              /* map edge in texels (e.g. 2048); 0 disables the pre-pass         */
    uint32_t flags;             /* reserved, 0                                                      */
    float depth_bias;           /* light-NDC depth subtracted before the compare (e.g. 0.002)       */
    float slope_bias;           /* depthBiasSlopeFactor of the depth pass: each caster's depth is   *
                                 * raised by slope_bias * max(|dz/dx|, |dz/dy|) per texel (e.g. 2) */
    float light_view_proj[16];  /* column-major light ortho * light view                            */
} tri_shadow_config;

typedef struct tri_ctx tri_ctx;

/* ---- lifetime ---------------------------------------------------------------------------- */
/* Renderer::Init (Renderer.h:115, Renderer.cpp:587-648): allocates the colour/depth targets and
 * the default 1x1 white texture in slot 0 (Renderer.cpp:3404-3436). */
int tri_create(const tri_config* config, tri_ctx** out_ctx);
/* Renderer::Shutdown (Renderer.h:116). Null is accepted. */
int tri_destroy(tri_ctx* ctx);
/* Use an external hipStream_t (passed as void*) for every launch/copy; NULL = the context's own. */
int tri_set_stream(tri_ctx* ctx, void* hip_stream);
const char* tri_last_error(void);
int tri_abi_version(void);

/* ---- data upload (copies) ---------------------------------------------------------------- */
/* Renderer::UploadMesh / AppendMeshes -> UploadMeshFromCache (Renderer.h:120-121,
 * Renderer.cpp:1965-2116): one concatenated vertex buffer, one uint32 mesh-local index buffer and
 * one MeshDrawInfo per mesh. Replaces the whole geometry set. */
int tri_upload_geometry(tri_ctx* ctx, const tri_vertex* vertices, uint64_t vertex_count,
                        const uint32_t* indices, uint64_t index_count,
                        const tri_mesh_range* meshes, uint32_t mesh_count);
/* Shared geometry (the reference binds ONE vertex and index buffer for every viewport,
 * Renderer.cpp:1965-2116, :5095-5108): a tri_geometry holds the uploaded meshes on one device and any
 * number of contexts on that device reference it through tri_bind_geometry (NULL returns a context to
 * its own geometry, which tri_upload_geometry fills). Uploading to a shared geometry waits for the
 * device to go idle; contexts pick the new meshes up at their next tri_render. */
typedef struct tri_geometry tri_geometry;
int tri_geometry_create(int32_t device /* -1 = current */, tri_geometry** out_geometry);
int tri_geometry_upload(tri_geometry* geometry, const tri_vertex* vertices, uint64_t vertex_count,
                        const uint32_t* indices, uint64_t index_count, const tri_mesh_range* meshes,
                        uint32_t mesh_count);
int tri_geometry_destroy(tri_geometry* geometry); /* after every context using it is unbound/destroyed */
int tri_bind_geometry(tri_ctx* ctx, tri_geometry* geometry);

/* Material buffer payload (BuildMaterialPayload, Renderer.cpp:5927-5951). count 0 => the default
 * record {1,1,1,1},{1,1,1,0} (Renderer.cpp:5941-5943). */
int tri_upload_materials(tri_ctx* ctx, const tri_material_record* records, uint32_t count);
/* Texture slot upload (PopulateTextureSlot, Renderer.cpp:3469-3620): R8G8B8A8_SRGB texels,
 * row-major, rows already flipped by the loader (TextureLoader.cpp:290-304). slot < 256. */
int tri_upload_texture(tri_ctx* ctx, uint32_t slot, const uint8_t* rgba8_srgb, uint32_t width,
                       uint32_t height);
/* Bone palette SSBO (binding 4, PrepareBonePaletteBuffer Renderer.cpp:3168-3245):
 * column-major mat4s. */
int tri_upload_bone_palette(tri_ctx* ctx, const float* matrices, uint32_t matrix_count);
/* Skybox cubemap (CreateSkyboxCubemap, Renderer.cpp:3818-4110; LoadFromFaces TextureLoader.cpp:
 * 334-830): 6 faces in Vulkan layer order +X,-X,+Y,-Y,+Z,-Z, each size x size RGBA8 sRGB texels, rows
 * top to bottom, one mip. The skybox pass (Skybox.cpp:13-79, Skybox.vert/.frag, cull FRONT, depth
 * LEQUAL without writes) then gives every uncovered pixel its sky colour instead of the clear colour.
 * faces = NULL or size = 0 removes the skybox. */
int tri_upload_skybox(tri_ctx* ctx, const uint8_t* faces_rgba8_srgb, uint32_t size);

/* Default.frag's AI frame-generation blend (Default.frag:182-191). The texture is what UploadAiInterpolationToGpu
 * (Renderer.cpp:1560-1700) fills and EnsureAiTextureResources (:1390-1500) creates: width x height R8G8B8A8_UNORM
 * texels (no sRGB decode), rows top to bottom, sampled LINEAR with CLAMP_TO_EDGE at level 0. A frame whose UBO has
 * AiBlendConfig.w > 0 and w' = clamp(AiBlendConfig.x, 0, 1) > 0 (UpdateUniformBuffer packs (strength, 1 / width,
 * 1 / height, 1) while the texture is ready, Renderer.cpp:5916-5925) replaces every mesh fragment's output c by
 * mix(c, texture(ai, gl_FragCoord.xy * AiBlendConfig.yz), w') before the UNORM store; the skybox pass does not
 * blend. rgba8 = NULL or a zero extent removes the texture (DestroyAiResources). Rendering a blending frame
 * without a texture is TRI_E_STATE; with the shadow pre-pass (not part of the reference) TRI_E_UNSUPPORTED. */
int tri_upload_ai_frame(tri_ctx* ctx, const uint8_t* rgba8_unorm, uint32_t width, uint32_t height);

/* Shadow-map pre-pass for the directional light (see tri_shadow_config). NULL or size 0 disables it
 * (the default: C1-C3 frames are exactly the reference's). size <= TRI_MAX_DIM. */
int tri_set_shadow(tri_ctx* ctx, const tri_shadow_config* config);
/* Host-only helper (no device): the orthographic light transform the shim fits for a shadow-casting
 * directional light travelling along `light_dir` (the UBO's DirectionalLightDirection) over the world
 * box [aabb_min, aabb_max]: glm::lookAtRH from 2 * radius behind the box centre, then glm::orthoRH_ZO
 * over the box corners in light view space (1% margin), so every corner lands inside the map. */
int tri_shadow_fit_ortho(const float light_dir[3], const float aabb_min[3], const float aabb_max[3],
                         float out_light_view_proj[16]);
/* Synchronous copy of the last rendered shadow map: size*size float32 depth bits, row j = light NDC y
 * increasing. TRI_E_STATE when no shadow pass is configured. */
int tri_read_shadow_map(tri_ctx* ctx, uint32_t* depth_bits);

/* ---- per frame --------------------------------------------------------------------------- */
/* UpdateUniformBuffer's vkCmdUpdateBuffer (Renderer.cpp:5958) + the colour clear value
 * (Renderer.cpp:5037-5050, SetClearColor Renderer.h:187). */
int tri_set_frame(tri_ctx* ctx, const tri_global_ubo* ubo, const float clear_rgba[4]);
/* The per-draw loop of RecordCommandBuffer (Renderer.cpp:5110-5151): draws in submission order. */
int tri_set_draws(tri_ctx* ctx, const tri_draw* draws, uint32_t draw_count);
/* Render into caller-owned device buffers (e.g. torch tensors for an RCCL all-gather):
 * colour = band_rows * width uint32 BGRA8 texels, depth = band_rows * width float32. NULL resets
 * to the context's own buffers. */
int tri_bind_output(tri_ctx* ctx, void* device_bgra8, void* device_depth);
/* Enqueue one frame on the context stream (asynchronous: vkQueueSubmit, Renderer.cpp:5679). */
int tri_render(tri_ctx* ctx);
/* Wait for the stream; reports TRI_E_OVERFLOW if a queued frame overflowed an internal buffer. */
int tri_synchronize(tri_ctx* ctx);
/* Frame readback (Renderer.cpp:5297-5338, :1299-1389): synchronous copy of the band, tightly packed
 * BGRA8 (width*4 bytes per row) and float32 depth bits. Either pointer may be NULL. */
int tri_readback(tri_ctx* ctx, uint8_t* bgra8, uint32_t* depth_bits);

/* The context's colour target as an opaque image handle: what Renderer::GetViewportTexture returns
 * instead of a VkDescriptorSet (Renderer.h:235; Forge shows it with ImGui::Image, GameViewportPanel.cpp:66,
 * SceneViewportPanel.cpp:139). Rows top to bottom, B8G8R8A8_UNORM; valid until the context is destroyed,
 * its output is rebound or its size changes; contents are those of the last completed tri_render. */
#define TRI_FORMAT_B8G8R8A8_UNORM 44u /* the VkFormat value of the reference's offscreen target */
typedef struct tri_image {
    void* device_ptr;     /* device memory on `device`                   */
    uint32_t width;
    uint32_t height;      /* rows of the context (its band)              */
    uint32_t pitch_bytes; /* bytes from one row to the next              */
    uint32_t format;      /* TRI_FORMAT_B8G8R8A8_UNORM                   */
    int32_t device;       /* HIP device ordinal                          */
    uint32_t reserved;
} tri_image;
int tri_get_output(tri_ctx* ctx, tri_image* out);

/* Presentation blit (Renderer.cpp:5346-5361: vkCmdBlitImage of the primary viewport's offscreen
 * target onto the swapchain image, VK_FILTER_LINEAR). Scales this context's B8G8R8A8 target to
 * width x height: each destination texel centre maps to the source by the extent ratio, the source
 * is filtered bilinearly on UNORM values with clamp-to-edge taps, and the result is rounded to UNORM8.
 * `dst` is a device pointer to width*height*4 bytes, or NULL for a context-owned present image that
 * tri_read_present copies out. Stream-ordered after the context's last tri_render. Whole frames only
 * (a row-band context returns TRI_E_STATE). */
int tri_blit_linear(tri_ctx* ctx, void* dst, uint32_t width, uint32_t height);
/* Synchronous copy of the context-owned present image of the last tri_blit_linear(ctx, NULL, w, h):
 * w*h*4 bytes of BGRA8. */
int tri_read_present(tri_ctx* ctx, uint8_t* bgra8);

/* ---- lossless 3-byte band transfer (multi-GPU assembly) ----------------------------
 * Replaces nothing in the reference (it has no multi-GPU path); it serves tri_group's and the bench's
 * gather onto the display GPU, whose inbound xGMI bytes bound the N = 8 frame rate.
 * tri_frame_alpha: the alpha byte EVERY pixel of the next tri_render of ctx will have, proven from the
 * context's state (material record 0, each draw's tint and texture slot, the clear colour, the skybox),
 * or -1 when it cannot be proven uniform. A band of such a frame can travel as 3 bytes per pixel. */
int tri_frame_alpha(tri_ctx* ctx, int32_t* alpha);
/* B8G8R8A8 (4 B/pixel, device pointer, 4-B aligned) <-> B, G, R bytes (3 B/pixel, device pointer),
 * stream-ordered on hip_stream (NULL = the null stream). pack: every alpha byte that differs from `alpha`
 * sets *flag (a device uint32, may be NULL) to nonzero — the transfer would not be lossless; unpack writes
 * `alpha` into every pixel. */
int tri_pack_bgr24(const void* bgra8, void* bgr8, uint64_t pixels, uint32_t alpha, uint32_t* flag, void* hip_stream);
int tri_unpack_bgr24(const void* bgr8, void* bgra8, uint64_t pixels, uint32_t alpha, void* hip_stream);
/* The delta bit-plane band format (lossless): the band as a 1-D pixel stream in slots of
 * TRI_DBP_SLOT_PIXELS pixels, each slot_bytes long (a multiple of 16, at least TRI_DBP_MIN_SLOT; TRI_DBP_MAX_SLOT
 * never overflows). Per 64-pixel block and channel, the bit width of the zigzag-mapped pixel-to-pixel differences and
 * that many 64-bit bit planes; alpha is dropped and restored as `alpha` (proven uniform, tri_frame_alpha).
 * tri_dbp_pack: flags[0] |= 1 when a pixel's alpha differs, |= 2 when a slot needed more than slot_bytes (that slot is
 * not decodable: grow slot_bytes and send again); flags[1] = max(flags[1], the largest slot's bytes) — the size the
 * next frames need. Both stream-ordered on hip_stream; stream buffers 16-B aligned, pixel buffers 4-B aligned.
 * tri_dbp_bytes: the stream's size for `pixels` pixels. */
#define TRI_DBP_SLOT_PIXELS 4096u
#define TRI_DBP_MIN_SLOT 176u
#define TRI_DBP_MAX_SLOT 12448u
int tri_dbp_pack(const void* bgra8, uint64_t pixels, uint32_t alpha, void* stream_out, uint32_t slot_bytes,
                 uint32_t* flags, void* hip_stream);
int tri_dbp_unpack(const void* stream_in, uint64_t pixels, uint32_t alpha, uint32_t slot_bytes, void* bgra8,
                   void* hip_stream);
uint64_t tri_dbp_bytes(uint64_t pixels, uint32_t slot_bytes);
/* tri_dbp_unpack of `count` (<= TRI_DBP_MAX_BANDS) streams with one slot size in one launch (the display device's
 * remote bands: a workgroup per slot of any of them); same alignment rules, bands of 0 pixels are skipped. */
#define TRI_DBP_MAX_BANDS 16u
int tri_dbp_unpack_bands(const void* const* streams_in, void* const* bgra8, const uint64_t* pixels, uint32_t count,
                         uint32_t alpha, uint32_t slot_bytes, void* hip_stream);

/* ---- one rank's band exchange (process per GPU) --------------------------------------------- */
/* A process-per-GPU caller (bench.py at N > 1) renders one row band per rank and assembles the frame on the
 * display rank. tri_xfer drives that exchange natively over RCCL communicators of its own: one call per frame
 * renders the band on the context's stream, then on the same stream packs and sends it (a sender) or receives and
 * decodes every remote band into the frame (the display rank) — no per-operation host bookkeeping in the
 * caller (torch.distributed's point-to-point calls cost ≈ 20 µs of host time each). Bootstrap, once per
 * communicator: rank 0 calls tri_xfer_unique_id and the caller broadcasts the TRI_XFER_ID_BYTES bytes (e.g. over
 * torch.distributed); every rank then calls tri_xfer_comm_create (collective). Communicators serve any number of
 * exchanges used one at a time. */
#define TRI_XFER_ID_BYTES 128u
typedef struct tri_xfer_comm tri_xfer_comm;
typedef struct tri_xfer tri_xfer;
typedef struct tri_xfer_config {
    uint32_t width;           /* pixels per row                                                          */
    const uint32_t* band_y;   /* world + 1 row boundaries: rank r renders rows [band_y[r], band_y[r + 1]);
                                 every band has rows except the display's, which may be empty: the
                                 display then renders nothing and only assembles (ctx NULL every frame) */
    uint32_t display;         /* the rank that assembles the frame                                       */
    uint32_t format;          /* TRI_GROUP_FMT_*: the bands' transfer format                             */
    uint32_t slot_bytes;      /* TRI_GROUP_FMT_DBP: the slot size every rank agreed                      */
    uint32_t alpha;           /* packed formats: the proven alpha (tri_frame_alpha)                      */
    uint32_t nbuf;            /* buffer slots (tri_xfer_bind_slot)                                       */
} tri_xfer_config;
int tri_xfer_unique_id(uint8_t* id_out);
int tri_xfer_comm_create(const uint8_t* id, uint32_t world, uint32_t rank, int32_t device, tri_xfer_comm** out);
int tri_xfer_comm_destroy(tri_xfer_comm* comm);
/* comms: one communicator per slot in flight (slot s uses comms[s % comm_count]; each created with the same world,
 * rank and device), so that each one's operations stay on one stream (the slot's context stream). With fewer
 * communicators than slots (e.g. a second ncclCommInitRank failed), a communicator shared by several slots has its
 * operations fenced across their streams by an event (correct, ≈ 2 µs of host time per frame more). */
int tri_xfer_create(tri_xfer_comm* const* comms, uint32_t comm_count, const tri_xfer_config* config, tri_xfer** out);
int tri_xfer_destroy(tri_xfer* xfer);
/* Slot `slot`'s pixel buffer (device, 4-B aligned, caller-owned): this rank's band (a sender) or the whole
 * width × height frame (the display rank, which renders its own band in place at its row offset). */
int tri_xfer_bind_slot(tri_xfer* xfer, uint32_t slot, void* bgra8);
/* One frame into slot `slot`: if ctx is not NULL, bind it to the slot (and `depth`, may be NULL), apply the frame
 * state when given (ubo / draws not NULL: tri_set_frame / tri_set_draws) and tri_render; then, if `exchange`, the
 * band's transfer, on the same stream (the context's; ctx NULL: the slot's last stream, or a stream of the slot's
 * own if it never rendered, so an assemble-only display's slots overlap as render streams do). A slot reused on its
 * stream is ordered behind its previous transfer by stream order; a slot that changes stream is fenced. Every rank
 * must make the same sequence of exchanging calls per slot (the transfers match in order per communicator). */
int tri_xfer_frame(tri_xfer* xfer, uint32_t slot, tri_ctx* ctx, void* depth, const tri_global_ubo* ubo,
                   const float clear_rgba[4], const tri_draw* draws, uint32_t draw_count, uint32_t exchange);
/* Wait for every slot's stream, at most the exchange's timeout (tri_xfer_set_timeout, default 60000 ms; 0 = none):
 * TRI_E_TIMEOUT when it expires, TRI_E_HIP when a communicator reports an asynchronous error — both abort the
 * exchange's communicators (ncclCommAbort; later exchanging frames on them fail with TRI_E_STATE), so the caller can
 * exit instead of hanging the job. Then TRI_E_STATE if a packed band's alpha differed, TRI_E_OVERFLOW if a band
 * outgrew the agreed dbp slot (both lossy). On the display rank these report the senders' bands too: the status
 * travels with each packed band and the decode ORs it in. */
int tri_xfer_synchronize(tri_xfer* xfer);
/* The bounded wait alone (TRI_E_TIMEOUT / TRI_E_HIP as above), without reading the status flags. */
int tri_xfer_wait(tri_xfer* xfer);
int tri_xfer_set_timeout(tri_xfer* xfer, uint32_t timeout_ms);
/* The number of communicators the exchange runs on (comm_count at tri_xfer_create). */
int tri_xfer_comm_count(tri_xfer* xfer, uint32_t* count);
/* Bytes this rank sends and receives per frame; max_slot_bytes (may be NULL; synchronising): the largest dbp slot
 * this rank's packs needed. */
int tri_xfer_info(tri_xfer* xfer, uint64_t* sent_bytes, uint64_t* received_bytes, uint32_t* max_slot_bytes);
/* Loopback transport (tests only; replaces nothing in the reference): `world` tri_xfer exchanges of one process on
 * one device stand in for `world` ranks (RCCL refuses two ranks on one GPU). tri_xfer_comm_create_loopback is
 * tri_xfer_comm_create's counterpart: the k-th communicator each rank creates on a hub forms channel k. Sends become
 * a device copy into the display's receive buffer, ordered by events as ncclSend / ncclRecv order them; every other
 * step of the exchange runs as on N GPUs. Drive the ranks frame by frame, every sender before the display. */
typedef struct tri_xfer_loopback tri_xfer_loopback;
int tri_xfer_loopback_create(uint32_t world, tri_xfer_loopback** out);
int tri_xfer_loopback_destroy(tri_xfer_loopback* hub);
int tri_xfer_comm_create_loopback(tri_xfer_loopback* hub, uint32_t rank, int32_t device, tri_xfer_comm** out);

/* ---- measurement -------------------------------------------------------------------------- */
/* enable = N > 0: HIP events around every stage of every N-th frame (1 = all frames; sampling keeps
 * the event overhead out of throughput runs); 0 = off. Also resets the accumulators. */
int tri_set_timing(tri_ctx* ctx, int enable);
int tri_get_timing(tri_ctx* ctx, tri_timing* out); /* synchronizes                      */
int tri_get_frame_stats(tri_ctx* ctx, tri_frame_stats* out); /* synchronizes           */

/* ---- multi-device frames (SURVEY 8(b) tri_config.device_count; 8(e) screen partition) ---------
 * A tri_group renders one frame on N contexts, context r owning rows [r*H/N, (r+1)*H/N) (sort-first:
 * geometry and uniforms replicated, every context culls clusters to its rows), and assembles the B8G8R8A8
 * frame on the display context's device: bands on that device render straight into the frame, bands
 * on other devices are gathered with RCCL grouped ncclSend / ncclRecv over xGMI (one communicator per
 * distinct device, ncclCommInitAll). One host thread drives the whole group, as Renderer::DrawFrame
 * does (the engine's single render thread, Application.cpp:82-134).
 * The geometry is held once per distinct device (one tri_geometry bound by every band context there).
 * The assembled frame is double-buffered: frame k lands in buffer k % 2, and frame k + 2 overwrites it
 * only after the consumer's fence on frame k (tri_group_present), when one was set — the reference keeps
 * one framebuffer per swapchain image and waits on that image's fence (Renderer.cpp:744-772). */
typedef struct tri_group tri_group;
typedef struct tri_group_config {
    uint32_t width;
    uint32_t height;
    uint32_t device_count;  /* N >= 1 bands                                                       */
    uint32_t display;       /* index of the band whose device holds the assembled frame            */
    const int32_t* devices; /* N HIP ordinals, NULL = 0..N-1; an ordinal may repeat (bands sharing  *
                             * a device are assembled without copies)                               */
    uint32_t flags;         /* TRI_FLAG_* for every band context                                    */
    uint32_t group_flags;   /* TRI_GROUP_* (0 = defaults)                                           */
} tri_group_config;
/* Bands travel to the display device as 4-byte pixels even when tri_frame_alpha proves a uniform alpha
 * (default: the delta bit-plane format then, TRI_GROUP_FMT_DBP below — lossless, restored on arrival). */
#define TRI_GROUP_NO_PACK 0x1u
/* Bands on the display device render into band buffers and travel like remote bands (a device-local copy
 * instead of RCCL): the remote path's buffers, fences and codec on a single GPU (tests, diagnostics). */
#define TRI_GROUP_STAGE_BANDS 0x2u
/* With a proven uniform alpha, bands travel as their B, G, R bytes (3 per pixel) instead of the delta bit-plane
 * format. */
#define TRI_GROUP_PACK_BGR24 0x4u
/* Band transfer formats (tri_group_transfer_format). */
#define TRI_GROUP_FMT_BGRA32 0u /* 4 bytes per pixel                                                  */
#define TRI_GROUP_FMT_BGR24 1u  /* 3 bytes per pixel, the proven alpha restored on arrival           */
/* the delta bit-plane format (tri_dbp_pack): fixed slots of slot_bytes per 4096 pixels, sized at every
 * tri_group_synchronize from the largest slot the frames since the previous one needed (+ 1/16); the first frame
 * uses TRI_DBP_MAX_SLOT, which always fits. A frame with a slot that outgrew its size is reported by
 * tri_group_synchronize as TRI_E_OVERFLOW (its slot is then refitted: render the frame again). */
#define TRI_GROUP_FMT_DBP 2u

int tri_group_create(const tri_group_config* config, tri_group** out_group);
int tri_group_destroy(tri_group* group);
/* The band context of index `band` (uploads, cameras, shadows, timing, readback of its own band). */
int tri_group_context(tri_group* group, uint32_t band, tri_ctx** out_ctx);
/* Broadcasts of the per-context uploads / frame inputs to every band (same semantics as the tri_* calls). */
int tri_group_upload_geometry(tri_group* group, const tri_vertex* vertices, uint64_t vertex_count,
                              const uint32_t* indices, uint64_t index_count, const tri_mesh_range* meshes,
                              uint32_t mesh_count);
int tri_group_upload_materials(tri_group* group, const tri_material_record* records, uint32_t count);
int tri_group_upload_texture(tri_group* group, uint32_t slot, const uint8_t* rgba8_srgb, uint32_t width,
                             uint32_t height);
int tri_group_upload_bone_palette(tri_group* group, const float* matrices, uint32_t matrix_count);
int tri_group_upload_skybox(tri_group* group, const uint8_t* faces_rgba8_srgb, uint32_t size);
int tri_group_upload_ai_frame(tri_group* group, const uint8_t* rgba8_unorm, uint32_t width, uint32_t height);
int tri_group_set_shadow(tri_group* group, const tri_shadow_config* config);
int tri_group_set_frame(tri_group* group, const tri_global_ubo* ubo, const float clear_rgba[4]);
int tri_group_set_draws(tri_group* group, const tri_draw* draws, uint32_t draw_count);
/* Enqueue every band, then the assembly onto the display device (asynchronous). */
int tri_group_render(tri_group* group);
/* Wait for every band and the assembly; TRI_E_OVERFLOW as tri_synchronize (re-render the frame). */
int tri_group_synchronize(tri_group* group);
/* The assembled frame (width*height BGRA8, from the display device) and, optionally, the depth of
 * every band (width*height float32 bits). Synchronous. */
int tri_group_readback(tri_group* group, uint8_t* bgra8, uint32_t* depth_bits);
/* The assembled frame in device memory: its pointer on the display device and that device's ordinal
 * (the buffer of the most recent tri_group_render; complete once its assembly has run). */
int tri_group_frame(tri_group* group, void** device_bgra8, int32_t* device);
/* The same buffer as a tri_image (GetViewportTexture's handle for a multi-device viewport). */
int tri_group_get_output(tri_group* group, tri_image* out);
/* Consumer fence ("frame k presented"): the caller is done reading the most recent frame once the work
 * already enqueued on hip_stream (a stream on the display device) has run; NULL = once the frame's own
 * assembly (and any tri_group_blit_linear of it) has run on the group's assembly stream, i.e. the caller
 * reads nothing further on other streams. Frame k + 2, which reuses that buffer, waits for this point on
 * the device before any band or receive writes it. Without a fence the next-but-one frame overwrites the
 * buffer unconditionally (a caller that reads with tri_group_readback, which synchronises, needs none);
 * a tri_group_blit_linear of frame k is always waited for (it reads the buffer on the assembly stream). */
int tri_group_present(tri_group* group, void* hip_stream);
/* Binds caller-owned geometry objects: for every band, the one of `geometries` on the band's device
 * (TRI_E_INVALID if a band's device has none). count 0 returns the bands to the group's own per-device
 * copies, which tri_group_upload_geometry fills. The objects must outlive the binding. */
int tri_group_bind_geometry(tri_group* group, uint32_t count, tri_geometry* const* geometries);
/* tri_blit_linear / tri_read_present over the assembled frame (the presentation blit of a multi-device
 * viewport, on the display device, stream-ordered after the frame's assembly; frame k + 2's bands and
 * receives wait for the blit of frame k). A blit into a caller-supplied dst does not touch the group's
 * own present target: tri_group_read_present then fails with TRI_E_STATE until a blit with dst = NULL. */
int tri_group_blit_linear(tri_group* group, void* dst, uint32_t width, uint32_t height);
int tri_group_read_present(tri_group* group, uint8_t* bgra8);
/* The most recent frame's band transfer: bytes per pixel on the links (4, 3, or for the delta bit-plane format
 * its stream bytes per pixel rounded up) and the bytes the display device received over RCCL (exact). */
int tri_group_transfer_info(tri_group* group, uint32_t* bytes_per_pixel, uint64_t* inbound_bytes);
/* The most recent frame's transfer format (TRI_GROUP_FMT_*) and, for TRI_GROUP_FMT_DBP, its slot size in bytes
 * per 4096 pixels (0 otherwise); before any frame, the format and slot the next frame would use with packing. */
int tri_group_transfer_format(tri_group* group, uint32_t* format, uint32_t* slot_bytes);

#ifdef __cplusplus
} /* extern "C" */

static_assert(sizeof(tri_vertex) == 100, "Vertex stride must match Trident's 100-byte Vertex");
static_assert(sizeof(tri_push_constant) == 128, "RenderablePushConstant is 128 bytes");
static_assert(sizeof(tri_draw) == 144, "tri_draw layout");
static_assert(sizeof(tri_global_ubo) == 480, "GlobalUniformBuffer is 480 bytes");
static_assert(sizeof(tri_material_record) == 32, "MaterialUniformBuffer is 32 bytes");
static_assert(sizeof(tri_shadow_config) == 80, "tri_shadow_config layout");
static_assert(sizeof(tri_group_config) == 32, "tri_group_config layout");
static_assert(sizeof(tri_image) == 32, "tri_image layout");
#endif

#endif /* TRI_RASTER_H */
