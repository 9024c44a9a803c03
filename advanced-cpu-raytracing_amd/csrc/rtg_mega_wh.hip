// Ray-tree (Whitted) variants of the fused kernel (rtg_mega_impl.hpp) specialised on the
// scene's shading and traversal features, as rtg_mega_pt.hip's path-tracing ones: C2-like
// scenes (BRDF shading, point / area / directional lights, meshes and spheres) below the
// ray-tree pipeline's frame size.  Same code, same results.
#include <cstdlib>

// the fused kernels keep trav_ray's ray unlaundered (rtg_common.hpp: laundering it costs C2
// 6 %, profiles/r05ag_sphere_launder_ab.txt)
#define RTG_XFORM_LAUNDER 0
#include "rtg_kernels.hpp"
#include "rtg_mega_impl.hpp"

namespace rtg {

template <int MAXD, int SK, int FEAT>
static hipError_t launch_wh(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                            unsigned char* l, float* accum, DevCounters* cnt, hipStream_t stream) {
    hipLaunchKernelGGL((k_render<MAXD, false, false, SK, FEAT>), dim3(P.num_tiles), dim3(256), 0, stream, S, C, P, hdr,
                       l, accum, cnt);
    return hipGetLastError();
}

template <int MAXD, int SK>
static hipError_t launch_wh_feat(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                                 unsigned char* l, float* accum, DevCounters* cnt, int feat, hipStream_t stream) {
    if (feat & FEAT_BIGLEAF) return launch_wh<MAXD, SK, FEAT_SPHERE | FEAT_BIGLEAF>(S, C, P, hdr, l, accum, cnt, stream);
    return launch_wh<MAXD, SK, FEAT_SPHERE>(S, C, P, hdr, l, accum, cnt, stream);
}

template <int MAXD>
static hipError_t launch_wh_sk(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                               unsigned char* l, float* accum, DevCounters* cnt, int sk, int feat, hipStream_t stream) {
    if ((sk & ~SK_BRDF) == 0) return launch_wh_feat<MAXD, SK_BRDF>(S, C, P, hdr, l, accum, cnt, feat, stream);
    return launch_wh_feat<MAXD, SK_BRDF | SK_XLIGHT>(S, C, P, hdr, l, accum, cnt, feat, stream);
}

// hipErrorNotSupported: no specialised variant covers the scene (the caller launches the
// general one)
hipError_t launch_mega_wh(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                          float* accum, DevCounters* cnt, int sk, int feat, hipStream_t stream) {
    if ((sk & SK_TEX) || (feat & (FEAT_INSTANCE | FEAT_XFORM)) || S.max_depth <= 0 || std::getenv("RTG_MEGA_GENERAL"))
        return hipErrorNotSupported;
    if (S.max_depth <= 8) return launch_wh_sk<8>(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
    return launch_wh_sk<32>(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
}

}  // namespace rtg
