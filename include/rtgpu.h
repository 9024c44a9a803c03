/*
 * rtgpu.h -- C-ABI drop-in boundary for the per-pixel trace/shade hot path of
 * dorukb/Advanced-CPU-Raytracing, re-implemented as hand-written HIP for gfx950.
 *
 * The reference has no plugin/FFI API: its only seam between the CLI driver and
 * the hot path is
 *     Vec3f DorkTracer::Raytracer::RenderPixel(int i, int j, Camera& cam)
 *         (src/raytracer.hpp:19, src/raytracer.cpp:33-36)
 * called once per pixel-sample by renderThreadMain (src/main.cpp:26-130) from the
 * 8-thread row-band block of main() (src/main.cpp:142-196).  This header replaces
 * that block with ONE call per camera (rtg_render), and the scene object graph
 * (src/scene.h:32-89) with a flattened POD description (rtg_scene_desc).
 *
 * Conventions: plain C, no C++ types, no exceptions across the ABI.  Every
 * function returns 0 (RTG_OK) or a negative RTG_ERR_* code; rtg_last_error()
 * returns a thread-local description of the last failure.  Buffers passed in are
 * owned by the caller and never freed by the library.
 */
#ifndef RTGPU_H
#define RTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTG_ABI_VERSION 6

enum rtg_status {
    RTG_OK = 0,
    RTG_ERR_INVALID = -1,     /* bad argument / inconsistent scene description      */
    RTG_ERR_IO = -2,          /* file could not be read / written                    */
    RTG_ERR_PARSE = -3,       /* malformed XML / PLY / image                         */
    RTG_ERR_HIP = -4,         /* HIP runtime error (no device, launch failure, ...)  */
    RTG_ERR_NOMEM = -5,       /* host or device allocation failed                    */
    RTG_ERR_UNSUPPORTED = -6  /* feature outside the implemented hot path            */
};

/* ------------------------------------------------------------------------- */
/* Flattened scene description (all host memory, produced by the XML loader   */
/* below or by any other front end, e.g. an adapter over the reference's own  */
/* DorkTracer::Scene -- see INTEGRATION.md).                                   */
/* ------------------------------------------------------------------------- */

typedef struct { float x, y, z; } rtg_float3;

/* material.hpp:14-20 */
enum rtg_material_type {
    RTG_MAT_MIRROR = 0, RTG_MAT_DIELECTRIC = 1, RTG_MAT_CONDUCTOR = 2,
    RTG_MAT_EMISSIVE = 3, RTG_MAT_DEFAULT = 4
};

/* Material (material.hpp:8-48).  Index in rtg_scene_desc.materials is the
 * reference's matId-1 (raytracer.cpp:73). */
typedef struct {
    int32_t id;
    int32_t type;            /* rtg_material_type */
    int32_t brdf;            /* index into brdfs[] or -1 (Material::brdf == nullptr) */
    int32_t pad0;
    rtg_float3 ambient, diffuse, specular, mirror;
    float phong_exponent;
    float refractive_index;
    float absorption_index;  /* conductorAbsorptionIndex */
    float roughness;
    rtg_float3 absorption;   /* absorptionCoefficient (Beer's law) */
    rtg_float3 radiance;     /* emissive materials only */
} rtg_material;

/* BRDF kinds (parser.cpp:870-982, brdf*.cpp) */
enum rtg_brdf_type {
    RTG_BRDF_PHONG = 0,               /* <OriginalPhong>       brdfPhong.cpp              */
    RTG_BRDF_BLINN_PHONG = 1,         /* <OriginalBlinnPhong>  brdfBlinnPhong.cpp         */
    RTG_BRDF_MODIFIED_PHONG = 2,      /* <ModifiedPhong>       brdfModifiedPhong.cpp      */
    RTG_BRDF_MODIFIED_BLINN_PHONG = 3,/* <ModifiedBlinnPhong>  brdfModifiedBlinnPhong.cpp */
    RTG_BRDF_TORRANCE_SPARROW = 4     /* <TorranceSparrow>     brdfTorranceSparrow.cpp    */
};
typedef struct {
    int32_t id, type;
    float exponent;
    int32_t energy_conserving;   /* BRDF::isEnergyConserving ("normalized" attribute) */
    int32_t kd_fresnel;          /* TorranceSparrow "kdfresnel" */
    int32_t pad0;
} rtg_brdf;

/* Lights (pointLight.h, areaLight.h, directionalLight.h, spotLight.h,
 * sphericalEnvironmentLight.h).  Evaluated in this type order
 * (raytracer.cpp:706-803). */
typedef struct { rtg_float3 position, intensity; } rtg_point_light;
typedef struct {
    rtg_float3 position, normal, radiance;
    rtg_float3 u, v;          /* GetOrthonormalBasis(normal) (areaLight.h:30) */
    float extent, area;
} rtg_area_light;
typedef struct { rtg_float3 dir /* unit */, radiance; } rtg_directional_light;
typedef struct {
    rtg_float3 position, dir /* unit */, intensity;
    float coverage_deg, falloff_deg;
    double cos_half_coverage, cos_half_falloff;   /* spotLight.h:24-25 */
} rtg_spot_light;
typedef struct { int32_t image; int32_t pad0; } rtg_env_light;
/* MeshLight (meshLight.h:9-47), in scene.meshLights order (parser.cpp:1474-1481).
 * object: its index in objects[] (a LightMesh entry); radiance: its own <Radiance> --
 * the emissive material carries the radiance of the LAST LightMesh sharing it
 * (parser.cpp:1484-1487), the light keeps its own (raytracer.cpp:800). */
typedef struct { int32_t object; rtg_float3 radiance; } rtg_mesh_light;

/* Images: texels stored as float, w*h*channels, row-major (LDRImage.h:16-26 keeps
 * the raw 0..255 byte values; HDRImage.h keeps linear floats). */
typedef struct {
    int32_t id, width, height, channels;
    int32_t is_hdr, pad0;
    const float* texels;
} rtg_image;

enum rtg_texture_kind { RTG_TEX_IMAGE = 0, RTG_TEX_PERLIN = 1 };
/* Texture::Textures (texture.h:31-38) plus the replace_background decal */
enum rtg_texture_slot {
    RTG_TEXSLOT_DIFFUSE = 0, RTG_TEXSLOT_SPECULAR = 1, RTG_TEXSLOT_BUMP = 2,
    RTG_TEXSLOT_NORMAL = 3, RTG_TEXSLOT_REPLACE_ALL = 4, RTG_TEXSLOT_NONE = 5
};
typedef struct {
    int32_t id, kind, slot;
    int32_t blend;            /* OperationMode::Blend (decal "blend_kd") */
    int32_t is_background;    /* decal "replace_background" */
    int32_t image;            /* image textures: index into images[] or -1 */
    int32_t nearest;          /* image textures: 1 = nearest, 0 = bilinear */
    float normalizer, bump_factor;
    float noise_scale;        /* perlin */
    int32_t noise_abs;        /* perlin: 1 = "absval", 0 = "linear" */
    int32_t pad0;
} rtg_texture;

/* Objects in the reference's IntersectObjects order (raytracer.cpp:625-643):
 * scene.meshes (Mesh, LightMesh, MeshInstance, Triangle-as-1-face-Mesh;
 * parser.cpp:348-512) followed by scene.spheres (parser.cpp:514-574). */
enum rtg_object_kind { RTG_OBJ_MESH = 0, RTG_OBJ_INSTANCE = 1, RTG_OBJ_SPHERE = 2 };
enum rtg_object_flags {
    RTG_OBJF_SHADOW_SKIP = 1,    /* emissive mesh: skipped by CastShadowRay (raytracer.cpp:590) */
    RTG_OBJF_NORMAL_TWICE = 2,   /* geometry has no UVs: IntersectFace applies the normal
                                    transform once more (mesh.cpp:362-364)               */
    RTG_OBJF_MOTION_BLUR = 4
};
typedef struct {
    int32_t kind;                /* rtg_object_kind */
    int32_t material;            /* 0-based index into materials[] */
    int32_t mesh;                /* geometry index into meshes[] (mesh/instance) */
    int32_t flags;               /* rtg_object_flags */
    int32_t tex_diffuse, tex_specular, tex_normal, tex_bump, tex_replace_all;
    int32_t id;
    /* 4x4 row-major double matrices (matrix.hpp).  For instances inv_transform and
     * inv_transpose are the instance's composed matrices (parser.cpp:429-451) and
     * base_inv_transpose is the base mesh's own (applied first by IntersectFace). */
    double inv_transform[16];
    double inv_transpose[16];
    double base_inv_transpose[16];
    double transform[16];
    float bbox_min[3], bbox_max[3];   /* mesh: local bbox (parser.cpp:1392-1468, with the
                                         FLT_MIN max-corner quirk); instance: world bbox
                                         (parser.cpp:749-805)                            */
    rtg_float3 motion_blur;
    rtg_float3 center;           /* sphere (local space) */
    float radius;
    int32_t pad0;
} rtg_object;

/* Triangle geometry with its BVH in the reference's topology (mesh.cpp:23-156). */
typedef struct {
    int32_t face_offset, face_count;   /* into faces[]   */
    int32_t node_offset, node_count;   /* into nodes[]   */
    int32_t has_uv;
    int32_t id;
    double surface_area;
} rtg_mesh;

/* Faces in the final BVH-permuted order (mesh.cpp:92-102 swaps faces in place). */
typedef struct {
    rtg_float3 v0, v1, v2;      /* object-space vertices (mesh.cpp:203-205) */
    rtg_float3 n;               /* makeUnit(cross(v1-v0, v2-v0)) (parser.cpp:724-733) */
    float uv0[2], uv1[2], uv2[2];
    double area;
} rtg_face;

/* BVH nodes, indices relative to the owning mesh's node_offset; node 0 is the
 * root; children are allocated pairwise (right == left + 1, mesh.cpp:109-122). */
typedef struct {
    float bmin[3], bmax[3];
    int32_t left;               /* -1 for a leaf */
    int32_t first, count;       /* leaf face range (relative to face_offset) */
    int32_t pad0;
} rtg_bvh_node;

/* Camera after Camera::SetupDefault / SetupLookAt (camera.cpp:5-72). */
typedef struct {
    rtg_float3 position, gaze, up, right, q;   /* q = m_q, image-plane corner */
    float left, right_ext, bottom, top, near_dist;
    int32_t width, height, spp;
    float focus_distance, aperture;
    int32_t has_tonemapper;
    float tm_key, tm_burn, tm_saturation, tm_gamma;
    int32_t path_tracing, importance_sampling, next_event, russian_roulette;
    char image_name[256];
} rtg_camera;

typedef struct {
    int32_t background[3];            /* BackgroundColor (integer, parser.cpp:47-53) */
    float shadow_epsilon;             /* Scene::shadow_ray_epsilon */
    int32_t max_recursion_depth;
    int32_t bg_texture;               /* replace_background texture index or -1 */
    rtg_float3 ambient_light;

    const rtg_camera* cameras;        int32_t num_cameras;
    const rtg_material* materials;    int32_t num_materials;
    const rtg_brdf* brdfs;            int32_t num_brdfs;
    const rtg_point_light* point_lights;          int32_t num_point_lights;
    const rtg_area_light* area_lights;            int32_t num_area_lights;
    const rtg_directional_light* dir_lights;      int32_t num_dir_lights;
    const rtg_spot_light* spot_lights;            int32_t num_spot_lights;
    const rtg_env_light* env_lights;              int32_t num_env_lights;
    const rtg_texture* textures;      int32_t num_textures;
    const rtg_image* images;          int32_t num_images;
    const rtg_object* objects;        int32_t num_objects;
    const rtg_mesh* meshes;           int32_t num_meshes;
    const rtg_face* faces;            int64_t num_faces;
    const rtg_bvh_node* nodes;        int64_t num_nodes;
    const rtg_mesh_light* mesh_lights; int32_t num_mesh_lights;
    int32_t pad0;
} rtg_scene_desc;

/* ------------------------------------------------------------------------- */
/* Host ingest: the XML scene format of the reference.                        */
/* ------------------------------------------------------------------------- */
typedef struct rtg_host_scene rtg_host_scene;

/* Replaces DorkTracer::Scene::loadFromXml (parser.cpp:26-577), called from
 * main.cpp:135-137.  Relative asset paths follow the reference: PLY files are
 * opened relative to the current directory (parser.cpp:1404), images as
 * "inputs/<name>" (parser.cpp:107,110). */
int rtg_host_scene_load_xml(const char* xml_path, rtg_host_scene** out);
/* Load flags.  RTG_LOAD_DEVICE_BVH: skip the host BVH build (mesh.cpp:23-156); the
 * description then holds faces in parse order, num_nodes == 0 and every mesh's node range
 * empty, and rtg_scene_create builds the same BVH and face order on the GPU (SURVEY §8f,
 * device scene ingest).  Such a description is for rtg_scene_create only. */
enum rtg_load_flags { RTG_LOAD_DEVICE_BVH = 1 };
int rtg_host_scene_load_xml_ex(const char* xml_path, uint32_t flags, rtg_host_scene** out);
/* The flattened description; valid until rtg_host_scene_free. */
const rtg_scene_desc* rtg_host_scene_desc(const rtg_host_scene* hs);
void rtg_host_scene_free(rtg_host_scene* hs);
/* Convenience accessors (cameras: scene.cameras[i], main.cpp:142-152). */
int rtg_desc_camera_info(const rtg_scene_desc* desc, int camera, int32_t* width,
                         int32_t* height, int32_t* spp, int32_t* has_tonemapper);
int rtg_desc_counts(const rtg_scene_desc* desc, int64_t* num_objects, int64_t* num_faces,
                    int64_t* num_nodes, int64_t* num_lights);
/* Diagnostic (ABI 5, host only, no device): builds the shadow rays' any-hit trees of a
 * description with a BVH as rtg_scene_create does (mode 0 = the reference's BVH collapsed,
 * 1 = binned SAH over its leaves, the default, 2 = large leaves split into faces) and checks
 * them -- every face reached once, box nesting, triangle containment.  out[0..7] = wide
 * nodes, leaf entries, depth, whole-leaf primitives, split faces, split faces kept on their
 * leaf box, violations, built (1) or not (0: leaf encoding exceeded). */
int rtg_desc_anyhit_check(const rtg_scene_desc* desc, int32_t mode, int64_t* out, int32_t n_out);

/* ------------------------------------------------------------------------- */
/* Device scene + render                                                      */
/* ------------------------------------------------------------------------- */
typedef struct rtg_scene rtg_scene;

/* Replaces Raytracer::Raytracer(Scene&) (raytracer.cpp:7-16, which copies the
 * scene): uploads a device-resident replica of `desc` to HIP device `device`.
 * The caller may free `desc` after return.  At most 2^25 faces (RTG_ERR_INVALID
 * beyond: the traversal kernels address records by 32-bit byte offsets). */
int rtg_scene_create(const rtg_scene_desc* desc, int device, rtg_scene** out);
/* The device's traversal data, for inspection and tests: the walk's node records (8 floats
 * per node, pre-order layout of the BVH nodes, the trailing pad node included) and the
 * per-face triangle records (12 floats per face, BVH face order).  Either buffer may be
 * NULL; counts are reported even when the buffers are too small (then nothing is copied). */
int rtg_scene_export_bvh(const rtg_scene* s, float* nodes, int64_t max_nodes, float* tris, int64_t max_faces,
                         int64_t* num_nodes, int64_t* num_faces);
void rtg_scene_destroy(rtg_scene* scene);
int rtg_device_count(int32_t* count);

/* Multi-GPU scene (replaces the reference's 8 row-band threads,
 * main.cpp:38-39,164-185, with the GPUs of one node): one device-resident replica per
 * entry of `devices`, each with its own stream (an entry may repeat: several replicas on
 * one device).  rtg_render on such a scene deals the frame to the replicas -- replica i
 * renders part i of num_devices (rtg_render_opts.part_index) -- and each copies its rows
 * straight into the caller's host buffers: the host framebuffer gather, no collective.
 * rtg_render_device, rtg_scene_timings and rtg_scene_export_bvh use the first replica;
 * rtg_scene_stats sums all replicas. */
int rtg_scene_create_multi(const rtg_scene_desc* desc, const int32_t* devices, int32_t num_devices,
                           rtg_scene** out);
int rtg_scene_num_devices(const rtg_scene* scene, int32_t* num_devices);

enum rtg_render_flags {
    RTG_RENDER_COUNT_STATS = 1,   /* accumulate rtg_stats (slower kernel variant)      */
    RTG_RENDER_ACCUM_ONLY = 2,    /* write the weighted sample sum (r,g,b,w) only; used
                                     when samples are split across devices            */
    RTG_RENDER_FUSED = 4,         /* force the fused per-pixel kernel even where the
                                     wavefront pipeline applies (for cross-checks)     */
    RTG_RENDER_TIMING = 8,        /* record HIP events around every kernel of the
                                     render (last sample pass); see rtg_scene_timings */
    RTG_RENDER_TREE = 16,         /* force the wavefront ray-tree pipeline for scenes with
                                     mirror / conductor / dielectric materials (default:
                                     frames of >= 2^21 pixel-samples; one stream
                                     synchronisation per render once its level sizes are
                                     planned).  ABI 5: for path-tracing cameras, the
                                     wavefront path tracer (opt-in; same image as the
                                     fused kernel bit for bit)                         */
    RTG_RENDER_EXACT_SHADOW = 32, /* shadow rays walk the reference BVH instead of the
                                     any-hit wide BVH (same answers; for cross-checks)  */
    RTG_RENDER_ORDERED = 64,      /* opt-in (ABI 4): camera rays of plain mesh scenes walk
                                     the 4-wide BVH nearest child first with a checked
                                     result (the reference walk where the check fails);
                                     agreement with the reference order is measured, not
                                     proven -- DESIGN.md §5                          */
    RTG_RENDER_SAMPLE_PASSES = 128 /* ABI 6: one sample per pass.  By default the wavefront
                                     and ray-tree pipelines carry several consecutive
                                     samples of the rendered pixels in one pass (about
                                     8 Mi camera rays per pass; env RTG_PASS_RAYS) and
                                     add each pixel's samples in sample order, so the image
                                     is the same bit for bit; this flag restores one
                                     sample per pass (for cross-checks)               */
};

typedef struct {
    int32_t camera;               /* index into cameras[] */
    int32_t sample_begin;         /* first sample index (default 0) */
    int32_t sample_count;         /* number of samples, <0 = camera spp */
    int32_t row_begin, row_end;   /* rows to render, row_end<=0 = all; the reference's
                                     row bands (main.cpp:38-39) are one choice */
    int32_t flags;                /* rtg_render_flags */
    uint64_t seed;                /* counter-based RNG key (stochastic features) */
    /* Image partition (ABI 3).  The rows [row_begin, row_end) are cut into bands of
     * RTG_PART_BAND_ROWS rows (counted from row_begin), dealt round-robin with the order
     * rotated by one slot per round (ABI 5): the k-th band of part p of N is band
     * k * N + ((p - k) mod N) -- so every part samples every position within a round of N
     * bands, and a cost peak a few bands tall (a horizon) is shared out.  A render with part_count > 1 computes and writes only the pixels
     * of part part_index; the union of parts 0..part_count-1 is bit-identical to the
     * whole render (pixels are independent, the RNG is keyed by pixel).  Exception: for
     * a camera with a <Tonemap>, a part's LDR rows hold clamp((int)c), not the tonemapped
     * value -- the tonemapper needs the whole frame (tonemapper.h:28-60); a caller that
     * gathers parts itself runs rtg_tonemap on the gathered float image (multigpu.py
     * finish_frame), while rtg_render on a multi-replica scene does it internally.  This
     * is how the frame is dealt to the GPUs of a node (main.cpp:38-39 deals row bands to
     * threads).  part_count <= 0 means 1. */
    int32_t part_index, part_count;
} rtg_render_opts;

/* ABI 5: 8-row bands (16 in ABI 3-4): 1080 rows over 8 parts give 17 or 16 bands per part
 * (a 0.7 % imbalance) instead of 9 or 8 (6.6 %) */
#define RTG_PART_BAND_ROWS 8

/* The rows of part `part_index` of `part_count` within [row_begin, row_end), as maximal
 * runs of consecutive rows: runs[2k] = first row, runs[2k+1] = one past the last.  Writes
 * up to `cap` runs; *count = number of runs.  Pure host arithmetic (no device needed). */
int rtg_part_runs(int32_t row_begin, int32_t row_end, int32_t part_index, int32_t part_count, int32_t* runs,
                  int32_t cap, int32_t* count);

typedef struct {
    uint64_t camera_rays;         /* primary rays (one per pixel-sample)            */
    uint64_t secondary_rays;      /* reflection / refraction extend rays             */
    uint64_t shadow_rays;         /* CastShadowRay queries                           */
    uint64_t node_visits;         /* BVH node box tests, extend rays                 */
    uint64_t tri_tests;           /* Mesh::IntersectFace calls, extend rays          */
    uint64_t sphere_tests;        /* Sphere::Intersect calls (all rays)              */
    uint64_t object_tests;        /* per-object visits (all rays)                    */
    uint64_t shadow_node_visits;  /* BVH node box tests, shadow rays (early exit)    */
    uint64_t shadow_tri_tests;    /* triangle tests, shadow rays (early exit)        */
    uint64_t shadow_wide_visits;  /* any-hit wide BVH nodes visited (shadow rays; each
                                     tests four child boxes; A/B builds only)          */
    uint64_t shadow_fallbacks;    /* shadow rays the fast any-hit walk left undecided,
                                     answered by the reference walk                    */
    uint64_t extend_wide_visits;  /* RTG_RENDER_ORDERED: wide BVH nodes visited by
                                     camera rays (ABI 4)                               */
    uint64_t extend_fallbacks;    /* RTG_RENDER_ORDERED: camera rays whose check failed,
                                     answered by the reference walk (ABI 4)           */
} rtg_stats;

/* One call per camera, replacing main.cpp:164-185 (threads -> renderThreadMain ->
 * RenderPixel).  Host buffers of width*height*3, layout 3*(x + y*width)
 * (main.cpp:109).  hdr_rgb receives the float colour (what main.cpp:114-116
 * stores for tonemapped cameras); ldr_rgb receives clamp((int)c) (main.cpp:121), or,
 * for a camera with a <Tonemap> rendered over all its rows, the tonemapped image
 * main.cpp:187-192 produces (a row band gets the clamp: tonemap the gathered image
 * with rtg_tonemap).  Either may be NULL. */
int rtg_render(rtg_scene* scene, const rtg_render_opts* opts, float* hdr_rgb, uint8_t* ldr_rgb);

/* Same on device-resident buffers (hipMalloc'd / torch tensors) on `stream`
 * (a hipStream_t, NULL = default stream).  Asynchronous: returns after enqueue.
 * d_accum (width*height*4 floats: sum w*r, sum w*g, sum w*b, sum w) is required
 * with RTG_RENDER_ACCUM_ONLY and ignored otherwise. */
int rtg_render_device(rtg_scene* scene, const rtg_render_opts* opts, float* d_hdr_rgb,
                      uint8_t* d_ldr_rgb, float* d_accum, void* stream);

/* Host framebuffer gather for one process per GPU: enqueue on `stream` the copies of the
 * rows of part opts->part_index (opts as given to rtg_render_device) from full-frame device
 * buffers into the same offsets of full-frame host buffers (either pair may be NULL).  With
 * page-locked host memory (rtg_host_alloc / rtg_host_register, e.g. a shared-memory frame
 * mapped by every rank) the copies are asynchronous DMA. */
int rtg_copy_part_to_host(rtg_scene* scene, const rtg_render_opts* opts, const float* d_hdr_rgb,
                          const uint8_t* d_ldr_rgb, float* hdr_rgb, uint8_t* ldr_rgb, void* stream);

/* Page-locked host memory for frame buffers (hipHostMalloc / hipHostRegister). */
int rtg_host_alloc(size_t bytes, void** out);
int rtg_host_free(void* ptr);
int rtg_host_register(void* ptr, size_t bytes);
int rtg_host_unregister(void* ptr);

/* Normalise an accumulation buffer (sum over devices) into hdr/ldr, host side. */
int rtg_resolve_accum(const float* accum, int32_t width, int32_t height, float* hdr_rgb,
                      uint8_t* ldr_rgb);

/* Stats of the last RTG_RENDER_COUNT_STATS render (waits for the scene's last render,
 * not for the device). */
int rtg_scene_stats(rtg_scene* scene, rtg_stats* out);
int rtg_scene_reset_stats(rtg_scene* scene);

/* Kernel durations (ms, HIP events on the render's stream) of the last render issued
 * with RTG_RENDER_TIMING, for its last sample pass; synchronises on that render.
 * Wavefront pipeline: names "k_primary", "k_shade", "k_shadow", "k_resolve"; fused
 * kernel: "k_render"; ray-tree pipeline: "tree_levels" (all levels' trace / shade /
 * shadow kernels), "tree_resolve".  Writes up to `cap` entries; *count = number of stages. */
int rtg_scene_timings(rtg_scene* scene, float* ms, const char** names, int32_t cap, int32_t* count);
/* ABI 6: samples per pixel the stages rtg_scene_timings reports covered -- the last pass's
 * samples (a pass carries several, RTG_RENDER_SAMPLE_PASSES), or the whole render's for the
 * fused kernel. */
int rtg_scene_timed_samples(const rtg_scene* scene, int32_t* samples);

/* ------------------------------------------------------------------------- */
/* Tonemapping (tonemapper.h, main.cpp:187-192)                               */
/* ------------------------------------------------------------------------- */
/* Tonemapper(opType, keyValue, burnPerct, saturation, gamma) (tonemapper.h:18-25);
 * the parser's defaults are 0.18, 1, 1, 2.2 (parser.cpp:845-863). */
typedef struct { float key, burn_percent, saturation, gamma; } rtg_tonemap_params;

/* Replaces Camera::GetTonemappedImage -> Tonemapper::Tonemap (tonemapper.h:28-60):
 * photographic operator over a whole width*height float RGB image in device memory,
 * writing the 8-bit image main.cpp:195 saves.  Asynchronous on `stream`. */
int rtg_tonemap_device(const float* d_hdr_rgb, int32_t width, int32_t height, const rtg_tonemap_params* params,
                       uint8_t* d_ldr_rgb, int32_t device, void* stream);
/* Same on host buffers (copies through device `device`; synchronous). */
int rtg_tonemap(const float* hdr_rgb, int32_t width, int32_t height, const rtg_tonemap_params* params,
                uint8_t* ldr_rgb, int32_t device);
/* Tonemapper::avgLuminance (tonemapper.h:35-48): exp(sum of log(0.01f + Y) / pixelCount) with
 * the sum taken as the reference takes it, sequentially in pixel order, on host buffers
 * (synchronous).  mode: -1 the library default (3), 3 windowed exact sum with the windows
 * summarised in parallel beforehand (ABI 5), 2 windowed exact sum, 1 plain sequential chain
 * (modes 1-3 give the same bits), 0 parallel fixed-order reduction (last bits differ from
 * the reference's). */
int rtg_tonemap_log_average(const float* hdr_rgb, int32_t width, int32_t height, int32_t mode, double* avg_out,
                            int32_t device);

/* ------------------------------------------------------------------------- */
/* Output (main.cpp:187-195)                                                  */
/* ------------------------------------------------------------------------- */
/* stbi_write_png replacement: 8-bit RGB, zlib-compressed PNG. */
int rtg_write_png(const char* path, int32_t width, int32_t height, const uint8_t* rgb);
/* stbi_write_hdr replacement: Radiance RGBE. */
int rtg_write_hdr(const char* path, int32_t width, int32_t height, const float* rgb);

const char* rtg_last_error(void);
int rtg_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RTGPU_H */
