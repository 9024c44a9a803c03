// Wavefront pipeline, traversal variants without large leaves (meshes / + spheres / everything) (rtg_wave.hpp).
#include "rtg_wave.hpp"

namespace rtg {

template hipError_t launch_wave_f<0>(const DevScene&, const DevCamera&, const RenderParams&, const WaveBufs&,
                                        float*, unsigned char*, DevCounters*, bool, int, hipStream_t, hipEvent_t*, int*);
template hipError_t launch_wave_f<FEAT_SPHERE>(const DevScene&, const DevCamera&, const RenderParams&, const WaveBufs&,
                                        float*, unsigned char*, DevCounters*, bool, int, hipStream_t, hipEvent_t*, int*);
template hipError_t launch_wave_f<FEAT_ALL & ~FEAT_BIGLEAF>(const DevScene&, const DevCamera&, const RenderParams&, const WaveBufs&,
                                        float*, unsigned char*, DevCounters*, bool, int, hipStream_t, hipEvent_t*, int*);

}  // namespace rtg
