// Path-tracing variants of the fused kernel (rtg_mega_impl.hpp) specialised on the scene's
// shading and traversal features, as k_shade and the path tracer's step kernel are: BRDF
// shading with point / area / directional lights (+ env / spot / mesh lights), meshes and
// spheres (small or large leaves).  Scenes with textures, maps, instances or transforms take
// the general instantiation (rtg_mega.hip).  Same code, same results: the feature bits only
// drop code the scene cannot reach.
#include <cstdlib>

// the fused kernels keep trav_ray's ray unlaundered (rtg_common.hpp: laundering it costs C2
// 6 %, profiles/r05ag_sphere_launder_ab.txt)
#define RTG_XFORM_LAUNDER 0
#include "rtg_kernels.hpp"
#include "rtg_mega_impl.hpp"

namespace rtg {

template <int MAXD, int SK, int FEAT>
static hipError_t launch_pt(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                            unsigned char* l, float* accum, DevCounters* cnt, hipStream_t stream) {
    hipLaunchKernelGGL((k_render<MAXD, false, true, SK, FEAT>), dim3(P.num_tiles), dim3(256), 0, stream, S, C, P, hdr,
                       l, accum, cnt);
    return hipGetLastError();
}

template <int MAXD, int SK>
static hipError_t launch_pt_feat(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                                 unsigned char* l, float* accum, DevCounters* cnt, int feat, hipStream_t stream) {
    if (feat & FEAT_BIGLEAF) return launch_pt<MAXD, SK, FEAT_SPHERE | FEAT_BIGLEAF>(S, C, P, hdr, l, accum, cnt, stream);
    return launch_pt<MAXD, SK, FEAT_SPHERE>(S, C, P, hdr, l, accum, cnt, stream);
}

template <int MAXD>
static hipError_t launch_pt_sk(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                               unsigned char* l, float* accum, DevCounters* cnt, int sk, int feat, hipStream_t stream) {
    if ((sk & ~SK_BRDF) == 0) return launch_pt_feat<MAXD, SK_BRDF>(S, C, P, hdr, l, accum, cnt, feat, stream);
    return launch_pt_feat<MAXD, SK_BRDF | SK_XLIGHT>(S, C, P, hdr, l, accum, cnt, feat, stream);
}

// hipErrorNotSupported: no specialised variant covers the scene (the caller launches the
// general one)
hipError_t launch_mega_pt(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                          float* accum, DevCounters* cnt, int sk, int feat, hipStream_t stream) {
    if ((sk & SK_TEX) || (feat & (FEAT_INSTANCE | FEAT_XFORM)) || std::getenv("RTG_MEGA_GENERAL"))
        return hipErrorNotSupported;
    if (S.max_depth <= 8 && !C.russian_roulette) return launch_pt_sk<8>(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
    return launch_pt_sk<32>(S, C, P, hdr, l, accum, cnt, sk, feat, stream);
}

}  // namespace rtg
