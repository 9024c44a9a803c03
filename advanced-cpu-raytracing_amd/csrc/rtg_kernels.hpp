#pragma once

#include <hip/hip_runtime.h>

#include "rtg_device.hpp"

namespace rtg {

int max_supported_depth();
// fused kernel (rtg_mega.hip): any scene
// `ev` (nullable): events recorded around every kernel of the last sample pass
hipError_t launch_mega(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* ldr,
                       float* accum, DevCounters* counters, bool stats, hipStream_t stream, hipEvent_t* ev);
// wavefront pipeline (rtg_wave.hip): scenes without secondary rays / motion blur
hipError_t launch_wave(const DevScene& S, const DevCamera& C, const RenderParams& P, const WaveBufs& W, float* hdr,
                       unsigned char* ldr, DevCounters* counters, bool stats, int feat, hipStream_t stream,
                       hipEvent_t* ev);
enum { WAVE_STAGES = 4, MEGA_STAGES = 1, MAX_STAGES = 4 };

}  // namespace rtg
