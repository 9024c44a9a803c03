#pragma once

#include <hip/hip_runtime.h>

#include "rtg_device.hpp"

namespace rtg {

int upload_perlin_tables(const int* perm512, const float* grad36);
int max_supported_depth();
hipError_t launch_render(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* ldr,
                         float* accum, DevCounters* counters, bool stats, hipStream_t stream);

}  // namespace rtg
