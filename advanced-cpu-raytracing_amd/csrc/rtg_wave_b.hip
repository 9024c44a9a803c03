// Wavefront pipeline, traversal variants with large leaves (cooperative leaf tests) (rtg_wave.hpp).
#include "rtg_wave.hpp"

namespace rtg {

template hipError_t launch_wave_f<FEAT_BIGLEAF>(const DevScene&, const DevCamera&, const RenderParams&, const WaveBufs&,
                                        float*, unsigned char*, DevCounters*, bool, int, hipStream_t, hipEvent_t*, int*);
template hipError_t launch_wave_f<FEAT_SPHERE | FEAT_BIGLEAF>(const DevScene&, const DevCamera&, const RenderParams&, const WaveBufs&,
                                        float*, unsigned char*, DevCounters*, bool, int, hipStream_t, hipEvent_t*, int*);
template hipError_t launch_wave_f<FEAT_ALL>(const DevScene&, const DevCamera&, const RenderParams&, const WaveBufs&,
                                        float*, unsigned char*, DevCounters*, bool, int, hipStream_t, hipEvent_t*, int*);

}  // namespace rtg
