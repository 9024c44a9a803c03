// Fused ("mega") render kernel: one thread per pixel walks the pixel's whole ray tree
// -- PerformShading (raytracer.cpp:65-134) with the recursion of ComputeMirrorReflection /
// ...Dielectric... / ...Conductor... and, for path-tracing cameras, ComputeGlobalIllumination
// (raytracer.cpp:135-191) unrolled onto an explicit per-thread stack.  Used for path
// tracing, motion blur and small ray-tree frames; other scenes take the wavefront
// pipelines (rtg_wave.hip, rtg_tree.hip).
// the fused kernels keep trav_ray's ray unlaundered (rtg_common.hpp: laundering it costs C2
// 6 %, profiles/r05ag_sphere_launder_ab.txt)
#define RTG_XFORM_LAUNDER 0
#include "rtg_common.hpp"
#include "rtg_kernels.hpp"
#include "rtg_mega_impl.hpp"

namespace rtg {

// ---------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------
template <int MAXD, bool STATS, bool PT>
static hipError_t launch_t(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                           float* accum, DevCounters* cnt, hipStream_t stream) {
    hipLaunchKernelGGL((k_render<MAXD, STATS, PT>), dim3(P.num_tiles), dim3(256), 0, stream, S, C, P, hdr, l, accum,
                       cnt);
    return hipGetLastError();
}

int max_supported_depth() { return 32; }

template <bool STATS>
static hipError_t launch_d(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                           float* accum, DevCounters* cnt, int sk, int feat, hipStream_t stream) {
    const int d = S.max_depth;
    if (C.path_tracing) {
        if (!STATS) {
            // the feature-specialised variants (rtg_mega_pt.hip; RTG_MEGA_GENERAL=1: A/B)
            const hipError_t e = launch_mega_pt(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
            if (e != hipErrorNotSupported) return e;
        }
        // Russian roulette: unbounded GI recursion, cut at 32 ray-tree levels (the frame stack)
        if (d <= 8 && !C.russian_roulette) return launch_t<8, STATS, true>(S, C, P, hdr, l, accum, cnt, stream);
        return launch_t<32, STATS, true>(S, C, P, hdr, l, accum, cnt, stream);
    }
    if (!STATS) {
        const hipError_t e = launch_mega_wh(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
        if (e != hipErrorNotSupported) return e;
    }
    if (d <= 0) return launch_t<0, STATS, false>(S, C, P, hdr, l, accum, cnt, stream);
    if (d <= 8) return launch_t<8, STATS, false>(S, C, P, hdr, l, accum, cnt, stream);
    return launch_t<32, STATS, false>(S, C, P, hdr, l, accum, cnt, stream);
}

static hipError_t launch_any(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                             float* accum, DevCounters* cnt, bool stats, int sk, int feat, hipStream_t stream) {
    return stats ? launch_d<true>(S, C, P, hdr, l, accum, cnt, sk, feat, stream)
                 : launch_d<false>(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
}

hipError_t launch_mega(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                       float* accum, DevCounters* cnt, bool stats, int sk, int feat, hipStream_t stream,
                       hipEvent_t* ev) {
    if (ev) (void)hipEventRecord(ev[0], stream);
    hipError_t e = launch_any(S, C, P, hdr, l, accum, cnt, stats, sk, feat, stream);
    if (ev) (void)hipEventRecord(ev[1], stream);
    return e;
}

}  // namespace rtg
