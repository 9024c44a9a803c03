// Photographic tonemapper (Tonemapper::Tonemap, tonemapper.h:28-60) on the GPU:
//
//   k_tm_log / k_tm_seqsum   log-average luminance: log(delta + Y) per pixel in double,
//                            then the reference's sequential sum (tonemapper.h:35-48) in
//                            pixel order by one wave -- the same rounding sequence as
//                            the reference, so the average is its average bit for bit
//                            wherever the device log agrees with the host's.  A
//                            dependent chain of W*H double adds: ~3.5 ns per pixel.
//   k_tm_logsum / k_tm_avg   (RTG_TM_SEQSUM=0) the same sum as per-block partials in a
//                            fixed parallel order: ~50x faster, differs from the
//                            reference's sum in the last bits
//   k_tm_hist / k_tm_pick    the burn threshold: the k-th smallest of all 3*W*H channel
//                            values (the reference's std::sort + index), found by an
//                            MSB-first radix select over the order-preserving bit image
//                            of the floats -- four 8-bit passes, each one histogram
//                            (LDS, one global atomic per bin per block) and one
//                            single-thread bucket pick, no host round trip
//   k_tm_map                 TonemapPixel (tonemapper.h:68-92): Reinhard with the
//                            reference's float round trips, saturation, gamma, floor
//
// HBM-bound: 12 B/pixel per pass over the float image, 6 passes + 3 B/pixel written.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtg_kernels.hpp"

namespace rtg {

namespace {

constexpr int kTmThreads = 256;

#ifndef RTG_TM_SEQSUM
#define RTG_TM_SEQSUM 1
#endif

__device__ __forceinline__ uint32_t float_key(float x) {
    const uint32_t b = __float_as_uint(x);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

__global__ __launch_bounds__(kTmThreads) void k_tm_logsum(const float* __restrict__ hdr, long long n,
                                                          double* __restrict__ partial) {
    __shared__ double red[kTmThreads];
    const double delta = 0.01f;
    double s = 0.0;
    for (long long i = blockIdx.x * (long long)kTmThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kTmThreads) {
        const double r = hdr[3 * i], g = hdr[3 * i + 1], b = hdr[3 * i + 2];
        const double lum = 0.2126 * r + 0.7152 * g + 0.0722 * b;
        s += log(delta + lum);
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = kTmThreads / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// log(delta + luminance) of every pixel (tonemapper.h:37-44), in pixel order
__global__ __launch_bounds__(kTmThreads) void k_tm_log(const float* __restrict__ hdr, long long n,
                                                       double* __restrict__ logs) {
    const long long i = blockIdx.x * (long long)kTmThreads + threadIdx.x;
    if (i >= n) return;
    const double delta = 0.01f;
    const double r = hdr[3 * i], g = hdr[3 * i + 1], b = hdr[3 * i + 2];
    const double lum = 0.2126 * r + 0.7152 * g + 0.0722 * b;
    logs[i] = log(delta + lum);
}

// logLuminancesSum += log(...) for i = 0 .. n-1 (tonemapper.h:35-47), one wave.  Each chunk
// of kSeqChunk terms is loaded by the whole wave (coalesced) and staged in LDS; every lane then
// runs the same in-order chain over it (uniform LDS addresses: broadcast reads), while the next
// chunk's loads are already in flight.  avg = exp(sum / pixelCount).
constexpr int kSeqPerLane = 16;
constexpr int kSeqChunk = 64 * kSeqPerLane;
__global__ __launch_bounds__(64) void k_tm_seqsum(const double* __restrict__ logs, long long n,
                                                  double* __restrict__ avg, uint32_t* __restrict__ sel,
                                                  uint32_t k) {
    __shared__ double buf[kSeqChunk];
    const int lane = threadIdx.x;
    double r[kSeqPerLane];
#pragma unroll
    for (int u = 0; u < kSeqPerLane; ++u) {
        const long long idx = (long long)u * 64 + lane;
        r[u] = idx < n ? logs[idx] : 0.0;
    }
    double s = 0.0;
    for (long long b = 0; b < n; b += kSeqChunk) {
#pragma unroll
        for (int u = 0; u < kSeqPerLane; ++u) buf[u * 64 + lane] = r[u];
        __syncthreads();
        if (b + kSeqChunk < n) {
#pragma unroll
            for (int u = 0; u < kSeqPerLane; ++u) {
                const long long idx = b + kSeqChunk + (long long)u * 64 + lane;
                r[u] = idx < n ? logs[idx] : 0.0;
            }
        }
        const int m = (n - b) < kSeqChunk ? (int)(n - b) : kSeqChunk;
        if (m == kSeqChunk) {
            // software-pipelined: the next 16 terms are read from LDS while the chain adds
            // the current 16 (the chain is bound by the dependent double-add latency)
            double a[16], c[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) a[k] = buf[k];
            for (int j = 0; j < kSeqChunk; j += 32) {
#pragma unroll
                for (int k = 0; k < 16; ++k) c[k] = buf[j + 16 + k];
#pragma unroll
                for (int k = 0; k < 16; ++k) s += a[k];
                if (j + 32 < kSeqChunk) {
#pragma unroll
                    for (int k = 0; k < 16; ++k) a[k] = buf[j + 32 + k];
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) s += c[k];
            }
        } else {
            for (int j = 0; j < m; ++j) s += buf[j];
        }
        __syncthreads();
    }
    if (lane == 0) {
        avg[0] = exp(s / (double)n);
        sel[0] = 0;
        sel[1] = k;
    }
}

// sum of the block partials in a fixed order; avg = exp(sum / pixelCount)
__global__ __launch_bounds__(kTmThreads) void k_tm_avg(const double* __restrict__ partial, int nb, long long n,
                                                       double* __restrict__ avg, uint32_t* __restrict__ sel,
                                                       uint32_t k) {
    __shared__ double red[kTmThreads];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += kTmThreads) s += partial[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = kTmThreads / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        avg[0] = exp(red[0] / (double)n);
        sel[0] = 0;   // selected key prefix
        sel[1] = k;   // rank still to find inside the selected bucket
    }
}

// histogram of byte `shift` of every key whose bits above it equal the selected prefix
__global__ __launch_bounds__(kTmThreads) void k_tm_hist(const float* __restrict__ v, long long m, int shift,
                                                        const uint32_t* __restrict__ sel, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t prefix = sel[0];
    const uint32_t hiMask = shift >= 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (long long i = blockIdx.x * (long long)kTmThreads + threadIdx.x; i < m; i += (long long)gridDim.x * kTmThreads) {
        const uint32_t key = float_key(v[i]);
        if ((key & hiMask) == (prefix & hiMask)) atomicAdd(&h[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

__global__ void k_tm_pick(int shift, uint32_t* __restrict__ sel, uint32_t* __restrict__ hist) {
    if (threadIdx.x != 0) return;
    uint32_t k = sel[1], cum = 0;
    int b = 0;
    for (; b < 255; ++b) {
        if (cum + hist[b] > k) break;
        cum += hist[b];
    }
    sel[0] |= (uint32_t)b << shift;
    sel[1] = k - cum;
    for (int i = 0; i < 256; ++i) hist[i] = 0;
}

__device__ __forceinline__ float tm_clip(float n, float lower, float upper) {   // std::max(lower, std::min(n, upper))
    const float a = (upper < n) ? upper : n;
    return (lower < a) ? a : lower;
}

__global__ __launch_bounds__(kTmThreads) void k_tm_map(const float* __restrict__ hdr, long long n, float key,
                                                       float burn, float saturation, float gamma,
                                                       const double* __restrict__ avgp,
                                                       const uint32_t* __restrict__ sel,
                                                       unsigned char* __restrict__ ldr) {
    const long long i = blockIdx.x * (long long)kTmThreads + threadIdx.x;
    if (i >= n) return;
    const double avg = avgp[0];
    const double R = hdr[3 * i], G = hdr[3 * i + 1], B = hdr[3 * i + 2];
    const double y_i = 0.2126 * R + 0.7152 * G + 0.0722 * B;
    // Reinhard (tonemapper.h:94-119), returning float
    const double Lxy = (key * y_i) / avg;
    float y_of;
    if (burn > 0.01) {
        double thr = key_float(sel[0]);
        thr = thr * key / avg;
        const double LwhiteSqr = thr * thr;
        y_of = (float)((Lxy * (1 + (Lxy / LwhiteSqr))) / (1.0f + Lxy));
    } else {
        y_of = (float)(Lxy / (1 + Lxy));
    }
    const double y_o = y_of;
    const double r_o = tm_clip((float)(y_o * pow((R / y_i), (double)saturation)), 0.0f, 1.0f);
    const double g_o = tm_clip((float)(y_o * pow((G / y_i), (double)saturation)), 0.0f, 1.0f);
    const double b_o = tm_clip((float)(y_o * pow((B / y_i), (double)saturation)), 0.0f, 1.0f);
    const double gammaInv = 1.0f / gamma;
    auto q = [](double x) {   // std::floor(std::min(255.0, x)) -> int -> unsigned char
        const double m = (x < 255.0) ? x : 255.0;
        return (unsigned char)(int)floor(m);
    };
    ldr[3 * i] = q(255 * pow(r_o, gammaInv));
    ldr[3 * i + 1] = q(255 * pow(g_o, gammaInv));
    ldr[3 * i + 2] = q(255 * pow(b_o, gammaInv));
}

}  // namespace

size_t tonemap_scratch_bytes(long long pixels) {
    return 1024 * sizeof(double) + 2 * sizeof(double) + 258 * sizeof(uint32_t) + 256 +
           (RTG_TM_SEQSUM ? (size_t)pixels * sizeof(double) : 0);
}

hipError_t launch_tonemap(const float* hdr, int width, int height, float key, float burn, float saturation,
                          float gamma, unsigned char* ldr, void* scratch, hipStream_t st) {
    const long long n = (long long)width * height;
    char* p = (char*)scratch;
    double* partial = (double*)p;
    double* avg = partial + 1024;
    uint32_t* sel = (uint32_t*)(avg + 2);
    uint32_t* hist = sel + 2;
    double* logs = (double*)(p + 1024 * sizeof(double) + 2 * sizeof(double) + 258 * sizeof(uint32_t) + 256);
    hipError_t e = hipMemsetAsync(hist, 0, 256 * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    // burn threshold index exactly as tonemapper.h:104-107 (float * int -> float -> int)
    const float thresholdPerct = (100.0f - burn) / 100;
    const int lastIdx = (int)(3 * n) - 1;
    int idx = (int)(thresholdPerct * lastIdx);
    if (idx > lastIdx) idx = lastIdx;
    if (idx < 0) idx = 0;
    const int nb = (int)((n + kTmThreads - 1) / kTmThreads < 1024 ? (n + kTmThreads - 1) / kTmThreads : 1024);
    if (RTG_TM_SEQSUM) {
        hipLaunchKernelGGL(k_tm_log, dim3((unsigned)((n + kTmThreads - 1) / kTmThreads)), dim3(kTmThreads), 0, st,
                           hdr, n, logs);
        hipLaunchKernelGGL(k_tm_seqsum, dim3(1), dim3(64), 0, st, logs, n, avg, sel, (uint32_t)idx);
    } else {
        hipLaunchKernelGGL(k_tm_logsum, dim3(nb), dim3(kTmThreads), 0, st, hdr, n, partial);
        hipLaunchKernelGGL(k_tm_avg, dim3(1), dim3(kTmThreads), 0, st, partial, nb, n, avg, sel, (uint32_t)idx);
    }
    if (burn > 0.01) {
        const long long m = 3 * n;
        const int hb = (int)((m + kTmThreads - 1) / kTmThreads < 2048 ? (m + kTmThreads - 1) / kTmThreads : 2048);
        for (int shift = 24; shift >= 0; shift -= 8) {
            hipLaunchKernelGGL(k_tm_hist, dim3(hb), dim3(kTmThreads), 0, st, hdr, m, shift, sel, hist);
            hipLaunchKernelGGL(k_tm_pick, dim3(1), dim3(64), 0, st, shift, sel, hist);
        }
    }
    hipLaunchKernelGGL(k_tm_map, dim3((unsigned)((n + kTmThreads - 1) / kTmThreads)), dim3(kTmThreads), 0, st, hdr, n,
                       key, burn, saturation, gamma, avg, sel, ldr);
    return hipGetLastError();
}

}  // namespace rtg
