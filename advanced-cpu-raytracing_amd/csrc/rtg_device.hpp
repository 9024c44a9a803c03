// Device-side data layout for the gfx950 render path.
//
// HBM layout (one replica per GPU, built by rtg_scene_create):
//   nodes[2i]   float4 {min.x, min.y, min.z, max.x}                     32 B record,
//   nodes[2i+1] float4 {max.y, max.z, skip (int), leaf (int)}            one cache line
//     Nodes are the reference's BVH (mesh.cpp:23-156) re-laid in pre-order
//     (left subtree before right) with a miss/skip link, so a stackless walk
//     "hit -> i+1, miss or leaf done -> skip" visits boxes and faces in exactly the
//     order of BVH::IntersectBVH's recursion (bvh.cpp:5-30).
//     leaf < 0: inner node; else (first << 8) | count for first < 2^23, count < 255,
//     or LEAF_EXT with {first, count} in node_ext[i].
//   tris[3f..3f+2] float4 {v0.xyz,0}, {v0-v1,0}, {v0-v2,0}                48 B record
//     (matrixA columns of mesh.cpp:208-210)
//   face_n[f]  float4 {n.xyz, 0}   (read once per hit)
//   face_uv[f] 3 x float2 (meshes with UVs only)
//   face_v12[2f..2f+1] float4 {v1}, {v2} (scenes with normal / bump maps only: the
//     tangent frame of mesh.cpp:390-422 needs v2 - v1 exactly)
// Faces are in the BVH-permuted order, so a leaf is a contiguous, coalescable
// range.  Objects, materials, BRDFs, lights, textures are small tables.
#pragma once

#include <stdint.h>

namespace rtg {

enum { OBJ_MESH = 0, OBJ_INSTANCE = 1, OBJ_SPHERE = 2 };
enum { OBJF_SHADOW_SKIP = 1, OBJF_NORMAL_TWICE = 2, OBJF_MOTION_BLUR = 4, OBJF_HAS_UV = 8,
       OBJF_IDENTITY = 16,     // inverse transform is exactly the identity: traversal skips it
       OBJF_MAPPED = 32 };     // normal or bump map in effect (mesh with UVs, or sphere bump map)

struct DevObject {
    int kind, material, flags, tex_normal;
    int node_begin, node_end;       // global node range of the (base) mesh's BVH
    int tex_diffuse, tex_specular, tex_replace_all, tex_bump;
    float bmin[4], bmax[4];         // mesh: local bbox, instance: world bbox
    float mbv[4];                   // motion blur vector
    float center[4];                // sphere center (xyz) + radius (w)
    double inv[12];                 // rows 0..2 of inverseTransform
    double invT[12];                // rows 0..2 of inverseTransposeTransform
    double baseInvT[12];            // base mesh's inverseTransposeTransform
    int id;                         // Shape::id (XML id; spheres: never a light's id)
    int group_end;                  // first object of an instance group: one past its last member
    int aroot;                      // (base) mesh's root in the any-hit tree (anodes; shadow rays), -1: none
};

// 4-wide BVH node, 128 B (one cache line pair): the four child boxes as SoA float4 rows, then
// the child references -- the any-hit tree of shadow rays (anodes; rtg_ahb.cpp: binned SAH over
// the reference's small leaves and the faces of its large ones); leaf slots (child <= -2) hold a
// range of ahtris entries, leaf = (first << 8) | count, count <= 255.
struct WNode {
    float4 lox, hix, loy, hiy, loz, hiz;
    int4 child;                     // >= 0: wide node; WCHILD_EMPTY; <= -2: leaf
    int4 leaf;                      // leaf slots: see above
};
enum : int { WCHILD_EMPTY = -1 };
// Shadow rays of the wavefront pipeline walk the any-hit tree as wave packets (trace_any_wide;
// undecided rays take the reference walk); the ray-tree pipeline's k_shadow keeps the per-lane
// reference walk (its secondary rays are incoherent: the packet walk measured slower on C5).
// (Rejected shadow walks, removed in round 6: the reference walk as wave packets, an any-hit
// climb from the ray's origin leaf, round 2's collapsed tree on compressed 64-B nodes.)
// Camera rays: RTG_PRIMARY_PACKET -- 2 (default): the reference walk as wave
// packets with scalar-cache records and select face tests (k_primary 0.227 -> 0.205 ms on the
// headline, profiles/r04c_packet_ab.txt); 1: round 2's packet form; 0: per lane.  DESIGN.md §5.
#ifndef RTG_PRIMARY_PACKET
#define RTG_PRIMARY_PACKET 2
#endif

struct DevMaterial {
    int type, brdf, pad0, pad1;
    float ambient[4], diffuse[4], specular[4], mirror[4], absorption[4], radiance[4];
    float phong_exponent, refractive_index, absorption_index, roughness;
};

struct DevBrdf {
    int type, energy_conserving, kd_fresnel, pad0;
    float exponent, pad1, pad2, pad3;
};

struct DevTexture {
    int kind, blend, image, nearest;
    float noise_scale, bump_factor, normalizer, pad0;
    int noise_abs, pad1, pad2, pad3;
};

struct DevImage {
    int width, height, channels, pad0;
    long long offset;               // into the texel pool (floats)
};

struct DevPointLight { float pos[4], intensity[4]; };
struct DevAreaLight { float pos[4], normal[4], radiance[4], u[4], v[4]; float extent, area, pad0, pad1; };
struct DevDirLight { float dir[4], radiance[4]; };
struct DevSpotLight {
    float pos[4], dir[4], intensity[4];
    float coverage_deg, falloff_deg, pad0, pad1;
    double cos_half_coverage, cos_half_falloff;
};

// MeshLight (meshLight.h:9-47): a LightMesh object sampled by SampleDirectLighting
// (raytracer.cpp:780-803).  Its faces (BVH-permuted order, as MeshLight::faces is after
// the in-place BVH build) are copied to light_faces[face_begin, +face_count).
struct DevMeshLight {
    int id, face_begin, face_count, pad0;
    float radiance[4];
    double surface_area, pad1;
    double xf[12];                  // rows 0..2 of Mesh::transform (ApplyTransformToPoint)
};
struct DevLightFace {
    float v0[4], v1[4], v2[4];      // object-space vertices
    double area, pad0;
};

enum : int { LEAF_EXT = 0x7FFFFFFF };

// Scene feature bits (kernel specialisation): spheres, mesh instances, any mesh with a
// non-identity transform or motion blur, BVH leaves of more than kBigLeaf faces.
enum : int { FEAT_SPHERE = 1, FEAT_INSTANCE = 2, FEAT_XFORM = 4, FEAT_BIGLEAF = 8, FEAT_ALL = 15 };
// Shading specialisation of the wavefront k_shade (the other kernels use SK_ALL): the scene
// has textures or normal / bump maps (SK_TEX), BRDFs (SK_BRDF), env / spot / mesh lights
// (SK_XLIGHT).  A variant without a feature compiles its code out; the values are the same.
enum : int { SK_TEX = 1, SK_BRDF = 2, SK_XLIGHT = 4, SK_ALL = 7 };
// A scene with a leaf wider than kBigLeaf faces takes the cooperative walk (FEAT_BIGLEAF);
// inside it, every leaf of more than kCoopLeaf faces is tested by the whole wave (threshold
// 8 / 4 / 2 / 1 / 0: C3 1494 / 1680 / 1781 / 1886 / 1912, C4 1481 / 1537 / 1613 / 1648 / 1555
// Mrays/s).  The selection threshold stays
// higher: the cooperative walk costs ~40% where no leaf needs it, and the headline and C5
// scenes have leaves of up to 4 faces.
#ifndef RTG_COOP_LEAF
#define RTG_COOP_LEAF 1
#endif
constexpr int kCoopLeaf = RTG_COOP_LEAF;
constexpr int kBigLeaf = 8;

// env_direction's table of inner RNG hashes (rtg_common.hpp): three draws per candidate, 4 096
// candidates per environment light, purpose RP_ENV
constexpr int kEnvDraws = 3 * 4096;
constexpr uint32_t kRpEnv = 5;

struct DevScene {
    const float4* __restrict__ nodes;
    const int2* __restrict__ node_ext;
    const float4* __restrict__ tris;
    const float4* __restrict__ face_n;
    const float2* __restrict__ face_uv;
    const float4* __restrict__ face_v12;   // raw v1, v2 per face (scenes with normal / bump maps only)
    const DevObject* __restrict__ objects;
    const float4* __restrict__ group_box;  // per object (group starts only): union of the members' world boxes
    const DevMaterial* __restrict__ materials;
    const DevBrdf* __restrict__ brdfs;
    const DevTexture* __restrict__ textures;
    const DevImage* __restrict__ images;
    const float* __restrict__ texels;
    const DevPointLight* __restrict__ point_lights;
    const DevAreaLight* __restrict__ area_lights;
    const DevDirLight* __restrict__ dir_lights;
    const DevSpotLight* __restrict__ spot_lights;
    const int* __restrict__ env_images;
    const unsigned long long* __restrict__ env_mix;   // per env light kEnvDraws inner RNG hashes (env_direction)
    const DevMeshLight* __restrict__ mesh_lights;
    const DevLightFace* __restrict__ light_faces;
    const int* __restrict__ perm;    // Perlin permutation (512) and gradients (12x3)
    const float* __restrict__ grad;
    int num_objects, num_point, num_area, num_dir, num_spot, num_env, num_mesh;
    int max_depth, bg_texture;
    float eps;
    float ambient[3];
    int background[3];
    int coop;                        // the scene has large leaves (FEAT_BIGLEAF)
    const WNode* __restrict__ anodes;  // any-hit tree (null: shadow rays take the reference walk)
    const float4* __restrict__ ahtris; // its leaf entries: face record, reference leaf node in [0].w
    const int* __restrict__ face_leaf; // per face: its leaf node
    int exact_shadow;                  // RTG_RENDER_EXACT_SHADOW: shadow rays take the reference walk
    int ahb_split;                     // the any-hit tree splits large leaves (AHB_SPLIT)
    int ordered;                       // RTG_RENDER_ORDERED (plain mesh scenes with an any-hit tree)
    // RTG_GUARD builds (fault hunting): table sizes and a violation bit mask (rtg_common.hpp GIDX)
    int* guard;
    int num_faces, num_textures, num_images, num_materials;
};

struct DevCamera {
    float pos[3], gaze[3], up[3], right[3], q[3];
    float left, right_ext, bottom, top;
    float focus_distance, aperture;
    int width, height, spp;
    int path_tracing, next_event, importance_sampling, russian_roulette;   // RendererParams (rendererParams.h)
};

// Image partition (multi-GPU): the rows [row_begin, row_end) are cut into 8-row bands (one
// wave's 8x8 pixel block), dealt round-robin with the order rotated one slot per round: the
// k-th band of part p of N is band k*N + ((p - k) mod N) (rtg_part_runs).  A
// render covers its part's rows only; they are numbered densely ("compact rows", 0 ..
// part_rows-1) for the per-pixel work buffers, and part_row() maps them back to image rows.
struct RenderParams {
    int row_begin, row_end;
    int sample_begin, sample_count;
    int accum_only;
    int tiles_x, tiles_y, num_tiles;    // tiles of 16 x 16 compact pixels (16 compact rows = 2 bands)
    int part_index, part_count, part_rows;
    unsigned long long seed;
    const int* __restrict__ tile_map;   // block -> 16x16 tile of this part (host-built, XCD-aware)
    // Multi-sample passes (wavefront and ray-tree pipelines): one pass carries `slabs`
    // consecutive samples of the part's pixels, so a small part still fills the GPU.  Sample
    // slab j of a pass is blocks [j * slab_tiles, (j + 1) * slab_tiles) of the tile grids
    // (slab_tiles = num_tiles rounded up to the 8 XCDs, so a tile keeps its XCD in every slab;
    // the padding blocks hold no pixels) and work-buffer entries [j * slab_px, (j + 1) * slab_px)
    // (slab_px = 16 * tiles_y * width; the ray trees' level 0: j * width * part_rows).  A pass's
    // colours go to a per-(slab, pixel) buffer and k_accum adds them to the pixel in sample
    // order, so the image is the one-sample passes' bit for bit.  slabs = 1: one sample per pass
    // (no colour buffer; tile grids of num_tiles blocks).
    int slabs, slab_tiles, slab_px;
};

// Wavefront pipeline buffers (rtg_wave.hip), one entry per pixel of the rendered rows
// and one light slot per (pixel, light) in the reference's light order.
struct WaveBufs {
    float* __restrict__ hit_t;
    int* __restrict__ hit_obj;
    int* __restrict__ hit_face;
    float4* __restrict__ base;          // rgb + flags (w): bit0 final, bit1 add a zero child term
    float4* __restrict__ term;          // per light slot: Shade(...) of that light
    unsigned char* __restrict__ occ;    // per light slot: 1 = in shadow
    // shadow-ray queue, one segment of 256 * num_slots entries per k_shade block (no
    // global atomics: a block compacts its rays with wave ballots + one LDS counter)
    float4* __restrict__ q_o;           // origin + initial minT
    float4* __restrict__ q_d;           // dir + acceptance limit
    int* __restrict__ q_slot;           // light slot it decides
    int* __restrict__ q_count;          // per block: entries in its segment
    float4* __restrict__ accum;         // multi-sample: sum w*c, sum w
    float4* __restrict__ col;           // multi-sample passes: colour per (slab, pixel) entry (k_accum)
    // one-slot scenes (at most one light): per queue entry the pixel's base colour + flags
    // and its light term + pixel index, so k_shadow finishes the pixel itself (no k_resolve)
    float4* __restrict__ q_pay;
    int pay3;                           // ... and a third: the environment light's term (one_layout_env)
    int num_slots;                      // lights per pixel
    // large-leaf scenes (FEAT_BIGLEAF), production renders: the camera walk defers each large
    // leaf it reaches to a queue of (ray, leaf, minT at entry) entries, 3 float4 each, tested by
    // k_bigleaf; per pixel the 64-bit (t, object, face) key of the best hit so far
    float4* __restrict__ dq_e;
    int* __restrict__ dq_count;         // [0] camera entries, [1] unsettled pixels, [2] shadow entries
    unsigned long long* __restrict__ hit_key;
    int* __restrict__ shadow_state;     // per shadow queue entry: SS_* bits (deferred any-hit)
    int dq_cap;
};

// One level of the wavefront ray tree (rtg_tree.hip): rays, their hits, the shading node
// each hit becomes and its final value.
struct TreeLevel {
    float4* o;                          // origin, medium
    float4* d;                          // direction, tree level (int bits)
    unsigned long long* key;            // RNG key of the ray-tree node
    float4* miss;                       // miss lookup: env direction, mode (int bits)
    float* t;
    int* obj;
    int* face;
    float4* base;                       // ambient colour, kind | lit flag (int bits)
    float4* coef;                       // mirror reflectance, ratio (conductor / Fresnel reflect)
    float4* ext;                        // refract ratio, material, child 0, child 1 (int bits)
    float4* value;                      // node value (rgb), ray hit something (int bits)
    float4* term;                       // per light slot: Shade term
    unsigned char* occ;                 // per light slot: 1 = in shadow
    int n;                              // rays (host-driven levels) or the capacity the grids cover
    const int* nd;                      // device-driven levels: the level's ray count on the device
};
// Per-block output segments of k_tree_shade: shadow rays (256 x slots per block, the
// k_shadow layout) and child rays (512 per block).
struct TreeSegs {
    float4* q_o;
    float4* q_d;
    int* q_slot;
    int* q_count;
    float4* c_o;
    float4* c_d;
    unsigned long long* c_key;
    float4* c_miss;
    int* c_parent;                      // parent node | slot << 30
    int* c_count;
    int num_slots;
};

// Per-launch ray/traversal counters (RTG_RENDER_COUNT_STATS).
struct DevCounters {
    unsigned long long camera_rays, secondary_rays, shadow_rays, node_visits, tri_tests, sphere_tests,
        object_tests, shadow_node_visits, shadow_tri_tests, shadow_wide_visits, shadow_fallbacks, extend_wide_visits,
        extend_fallbacks, pad0, pad1;
};

}  // namespace rtg
