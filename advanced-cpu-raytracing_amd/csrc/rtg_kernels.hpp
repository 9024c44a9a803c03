#pragma once

#include <hip/hip_runtime.h>

#include "rtg_device.hpp"
#include "rtgpu.h"

namespace rtg {

int max_supported_depth();
// large leaves of the camera walk deferred to k_bigleaf (rtg_wave_shade.hip; RTG_DEFER=0: off)
bool defer_leaves();
// FNV-1a of a camera's device record (view, image size, samples, renderer flags): the ray-tree and
// path plans are kept per frame part of one camera
inline unsigned long long camera_hash(const DevCamera& C) {
    const unsigned char* p = reinterpret_cast<const unsigned char*>(&C);
    unsigned long long h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(DevCamera); ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}
// fused kernel (rtg_mega.hip): any scene
// `ev` (nullable): events recorded around every kernel of the last sample pass
// sk / feat: the scene's shading / traversal features (path-tracing variants, rtg_mega_pt.hip)
hipError_t launch_mega(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* ldr,
                       float* accum, DevCounters* counters, bool stats, int sk, int feat, hipStream_t stream,
                       hipEvent_t* ev);
hipError_t launch_mega_pt(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* ldr,
                          float* accum, DevCounters* counters, int sk, int feat, hipStream_t stream);
hipError_t launch_mega_wh(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* ldr,
                          float* accum, DevCounters* counters, int sk, int feat, hipStream_t stream);
// wavefront pipeline (rtg_wave.hip): scenes without secondary rays / motion blur
hipError_t launch_wave(const DevScene& S, const DevCamera& C, const RenderParams& P, const WaveBufs& W, float* hdr,
                       unsigned char* ldr, DevCounters* counters, bool stats, int feat, int sk, hipStream_t stream,
                       hipEvent_t* ev, int* layout);
// wavefront ray trees (rtg_tree.hip): scenes with mirror / conductor / dielectric materials;
// host-synchronous per tree level (the next level's size); state (buffers) kept in `tree`
struct TreeState;
void tree_destroy(TreeState* tree);
hipError_t launch_tree(TreeState*& tree, const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                       unsigned char* ldr, float4* accum, DevCounters* counters, bool stats, int feat, int sk,
                       hipStream_t stream, hipEvent_t* ev);
// wavefront path tracing (rtg_path.hip): path-tracing cameras without motion blur; path
// queues and frame stacks kept in `path`.  hipErrorNotSupported: a pass needed more than
// its iteration bound (the caller renders with the fused kernel instead)
struct PathState;
void path_destroy(PathState* path);
hipError_t launch_path(PathState*& path, const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                       unsigned char* ldr, float4* accum, DevCounters* counters, bool stats, int feat, int sk,
                       hipStream_t stream, hipEvent_t* ev);
// photographic tonemapper (rtg_tonemap.hip); scratch of tonemap_scratch_bytes()
size_t tonemap_scratch_bytes(long long pixels);
size_t tonemap_avg_offset();   // byte offset of the log-average luminance (double) in the scratch
void launch_log_average(const float* hdr, long long n, int mode, uint32_t idx, void* scratch, hipStream_t st);
hipError_t launch_tonemap(const float* hdr, int width, int height, float key, float burn, float saturation,
                          float gamma, unsigned char* ldr, void* scratch, hipStream_t stream);
// device scene ingest (rtg_bvh.hip): the reference's midpoint BVH of one mesh built on the
// GPU from its faces in parse order (d_faces, device copy of the desc's), written as walk
// records at node index nodeBase and as face arrays at faceOff (BVH order); d_perm
// (nullable) receives the final order (mesh-local indices).  Synchronises `st`.
hipError_t build_mesh_bvh(const rtg_face* d_faces, int n, const float root_mn[3], const float root_mx[3],
                          int faceOff, int nodeBase, float4* d_nodes, int2* d_ext, float4* d_tris, float4* d_fn,
                          float2* d_fuv, float4* d_v12, int* d_perm, int* nodeCount, bool* bigleaf,
                          hipStream_t st);
enum { WAVE_STAGES = 4, MEGA_STAGES = 1, TREE_STAGES = 2, PATH_STAGES = 1, MAX_STAGES = 4 };
// Timed stage layouts (RTG_RENDER_TIMING): which kernels ran between the recorded events.
enum { LAYOUT_WAVE = 0,          // k_primary, k_shade, k_shadow, k_resolve
       LAYOUT_WAVE_ONE = 1,      // k_primary, k_shade, k_shadow (k_shadow_one finishes pixels)
       LAYOUT_WAVE_FUSED = 2,    // k_primary, k_shade_shadow
       LAYOUT_TREE = 3, LAYOUT_MEGA = 4,
       LAYOUT_PATH = 5,            // the last sample pass of the wavefront path tracer
       LAYOUT_WAVE_FRAME = 6 };    // k_frame: the fused layout's whole sample pass in one kernel

}  // namespace rtg
