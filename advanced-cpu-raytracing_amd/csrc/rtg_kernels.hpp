#pragma once

#include <hip/hip_runtime.h>

#include "rtg_device.hpp"

namespace rtg {

int max_supported_depth();
// fused kernel (rtg_mega.hip): any scene
hipError_t launch_mega(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* ldr,
                       float* accum, DevCounters* counters, bool stats, hipStream_t stream);
// wavefront pipeline (rtg_wave.hip): scenes without secondary rays / motion blur
hipError_t launch_wave(const DevScene& S, const DevCamera& C, const RenderParams& P, const WaveBufs& W, float* hdr,
                       unsigned char* ldr, DevCounters* counters, bool stats, hipStream_t stream);

}  // namespace rtg
