// Photographic tonemapper (Tonemapper::Tonemap, tonemapper.h:28-60) on the GPU:
//
//   k_tm_log + k_tm_winsum   log-average luminance: log(delta + Y) per pixel in double,
//                            then the reference's sequential sum (tonemapper.h:35-48) in
//                            pixel order -- the same rounding sequence as the reference,
//                            so the average is its average bit for bit wherever the
//                            device log agrees with the host's.  k_tm_winsum advances a
//                            8 192-term window per step by exact integer arithmetic
//                            inside a binade (see there); k_tm_seqsum (RTG_TM_SEQSUM=1)
//                            is the plain dependent chain of W*H double adds.
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
#include <stdlib.h>

#include "rtg_kernels.hpp"

namespace rtg {

namespace {

constexpr int kTmThreads = 256;

// log-sum mode: 3 = windowed exact sum with the windows summarised in parallel beforehand
// (k_tm_wtot / k_tm_wguess / k_tm_wsumm + k_tm_winsum<true>), 2 = windowed exact sum
// (k_tm_winsum<false>), 1 = the plain chain (k_tm_seqsum), 0 = parallel fixed-order reduction
// (not the reference's rounding).  The environment variable RTG_TM_SEQSUM overrides it at run
// time (A/B and diagnostics).
#ifndef RTG_TM_SEQSUM
#define RTG_TM_SEQSUM 3
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

// The same sequential sum, an 8 192-term window per step (one block of eight waves, 16
// consecutive terms per thread) instead of an 8 192-add chain.  While
// the running sum s keeps one binade [2^(e-1), 2^e), every representable value there is a
// multiple of u = 2^(e-53), so RN(s + x) = s + u * round(x / u) exactly -- unless x / u is a
// tie (then the parity of s decides) or s + x leaves the binade.  Each thread takes 16
// consecutive terms: k = rint(x / u) (an exact power-of-two scale), a lane-sequential prefix
// and a block scan of the integer-valued k give the running sum in units of u after every term; the
// first term whose result is not strictly inside the binade (or is a tie, or s = 0) stops
// the window.  s jumps to that term's exact running value, the stopping term is added with
// one rounded double add (the reference's own step), and the next window starts after it.
// A window that stops within its first 64 terms (|s| small or near a power of two) is
// finished with the plain rounded chain.  Such a window costs the scan on top of the chain,
// so an input whose running sum keeps hovering near a binade boundary would run slower than
// the plain chain; after kWinSlowRun consecutive short windows the kernel therefore runs
// kWinChainRun windows as the plain chain (no scan) before it tries the shortcut again.
// The result is the reference's sum bit for bit on any input.
constexpr int kWinPer = 16;
constexpr int kWinWaves = 8;
constexpr int kWinThreads = 64 * kWinWaves;
constexpr int kWin = kWinThreads * kWinPer;
constexpr int kWinSlowRun = 4;
constexpr int kWinChainRun = 16;

// Mode 3: every aligned window of kWin terms summarised in parallel before the sequential
// pass.  The binade the running sum will be in at a window's start is guessed from an
// approximate prefix of the window totals (k_tm_wtot, k_tm_wguess); with that binade's unit u,
// k_tm_wsumm forms each term's k = rint(x / u) and the window's total Q and the least and
// greatest of its running partial sums (the prefixes after each term).  The sequential pass
// (k_tm_winsum<true>) then crosses a whole window in one step when the guess is the binade the
// exact running sum s actually has, no term is a tie or too large, sum |k| < 2^52 (so every
// partial sum above is exact), and s + u * partial stays strictly inside the binade for every
// prefix -- exactly the conditions under which the per-window scan of mode 2 would have
// consumed the window whole, with the same result s + u * Q.  Any other window (the binade
// crossings, the first windows while |s| is small, ties) takes mode 2's scan.
struct WinSumm {
    double q, pmin, pmax;   // total and extreme running partials of k = rint(x / u), units of u
    int e, ok;              // guessed binade exponent (frexp) at the window start; usable
};

// approximate window totals (any order)
__global__ __launch_bounds__(256) void k_tm_wtot(const double* __restrict__ logs, long long n, double* __restrict__ wtot) {
    __shared__ double red[256];
    const long long a = (long long)blockIdx.x * kWin;
    double t = 0.0;
    for (int j = threadIdx.x; j < kWin; j += 256) {
        const long long i = a + j;
        if (i < n) t += logs[i];
    }
    red[threadIdx.x] = t;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) wtot[blockIdx.x] = red[0];
}

// approximate running sum at each window start (exclusive prefix of the totals) -> its binade
__global__ void k_tm_wguess(const double* __restrict__ wtot, int nw, WinSumm* __restrict__ summ) {
    if (threadIdx.x != 0) return;
    double s = 0.0;
    for (int w = 0; w < nw; ++w) {
        int e = 0;
        (void)frexp(s, &e);
        summ[w].e = s != 0.0 ? e : INT_MIN;
        s += wtot[w];
    }
}

// window summaries (one block per window, kWinPer consecutive terms per thread)
__global__ __launch_bounds__(kWinThreads) void k_tm_wsumm(const double* __restrict__ logs, long long n,
                                                          WinSumm* __restrict__ summ) {
    __shared__ double wtot[kWinWaves], wlo[kWinWaves], whi[kWinWaves], wabs[kWinWaves];
    __shared__ int wbad[kWinWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long a = (long long)blockIdx.x * kWin;
    const int e = summ[blockIdx.x].e;
    const bool valid = e != INT_MIN;
    double kk[kWinPer];
    double tot = 0.0, absum = 0.0;
    int bad = 0;
#pragma unroll
    for (int t = 0; t < kWinPer; ++t) {
        const long long idx = a + tid * kWinPer + t;
        kk[t] = 0.0;
        if (idx < n && valid) {
            const double y = ldexp(logs[idx], 53 - e);
            const double r = rint(y);
            const bool ok = fabs(y) < 4503599627370496.0 && fabs(y - r) != 0.5;
            bad |= ok ? 0 : 1;
            kk[t] = ok ? r : 0.0;
        }
        tot += kk[t];
        absum += fabs(kk[t]);
    }
    // running partials inside the thread, relative to its start
    double run = 0.0, lo = INFINITY, hi = -INFINITY;
#pragma unroll
    for (int t = 0; t < kWinPer; ++t) {
        const long long idx = a + tid * kWinPer + t;
        run += kk[t];
        if (idx < n) {
            lo = fmin(lo, run);
            hi = fmax(hi, run);
        }
    }
    // block exclusive scan of the thread totals
    double incl = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    double woff = 0.0;
    for (int w = 0; w < wave; ++w) woff += wtot[w];
    double excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0.0;
    excl += woff;
    lo += excl;
    hi += excl;
    // block min / max / sum of |k| / any bad
    double absw = absum;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, d));
        hi = fmax(hi, __shfl_xor(hi, d));
        absw += __shfl_xor(absw, d);
        bad |= __shfl_xor(bad, d);
    }
    if (lane == 0) {
        wlo[wave] = lo;
        whi[wave] = hi;
        wabs[wave] = absw;
        wbad[wave] = bad;
    }
    __syncthreads();
    if (tid == 0) {
        double L = INFINITY, H = -INFINITY, A = 0.0, Q = 0.0;
        int B = 0;
        for (int w = 0; w < kWinWaves; ++w) {
            L = fmin(L, wlo[w]);
            H = fmax(H, whi[w]);
            A += wabs[w];
            Q += wtot[w];
            B |= wbad[w];
        }
        WinSumm& S = summ[blockIdx.x];
        S.q = Q;
        S.pmin = L;
        S.pmax = H;
        S.ok = valid && !B && A < 4503599627370496.0;   // every partial exact and within +-2^52
    }
}

// The same sequential sum, an 8 192-term window per step (one block of eight waves, 16
// consecutive terms per thread) instead of an 8 192-add chain.  While
// the running sum s keeps one binade [2^(e-1), 2^e), every representable value there is a
// multiple of u = 2^(e-53), so RN(s + x) = s + u * round(x / u) exactly -- unless x / u is a
// tie (then the parity of s decides) or s + x leaves the binade.  Each thread takes 16
// consecutive terms: k = rint(x / u) (an exact power-of-two scale), a lane-sequential prefix
// and a block scan of the integer-valued k give the running sum in units of u after every term; the
// first term whose result is not strictly inside the binade (or is a tie, or s = 0) stops
// the window.  s jumps to that term's exact running value, the stopping term is added with
// one rounded double add (the reference's own step), and the next window starts after it.
// A window that stops within its first 64 terms (|s| small or near a power of two) is
// finished with the plain rounded chain.  Such a window costs the scan on top of the chain,
// so an input whose running sum keeps hovering near a binade boundary would run slower than
// the plain chain; after kWinSlowRun consecutive short windows the kernel therefore runs
// kWinChainRun windows as the plain chain (no scan) before it tries the shortcut again.
// SUMM (mode 3): windows end at the aligned kWin boundaries, and an aligned window whose
// summary (k_tm_wsumm) applies to the exact running sum is crossed in one step.
// The result is the reference's sum bit for bit on any input.
template <bool SUMM>
__global__ __launch_bounds__(kWinThreads) void k_tm_winsum(const double* __restrict__ logs, long long n,
                                                           const WinSumm* __restrict__ summ,
                                                           double* __restrict__ avg, uint32_t* __restrict__ sel,
                                                           uint32_t k) {
    __shared__ double buf[kWin];
    __shared__ double wtot[kWinWaves];
    __shared__ int wmin[kWinWaves];
    __shared__ double pshare;
    __shared__ WinSumm sc[kWinThreads];      // SUMM: summaries of windows [cbase, cbase + kWinThreads)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const double lo = 4503599627370497.0, hi = 9007199254740990.0;   // 2^52 + 1, 2^53 - 2
    auto load = [&](double* v, long long at) {
#pragma unroll
        for (int t = 0; t < kWinPer; ++t) {
            const long long idx = at + tid * kWinPer + t;
            v[t] = idx < n ? logs[idx] : 0.0;
        }
    };
    double cur[kWinPer], nxt[kWinPer];
    load(cur, 0);
    double s = 0.0;   // the running sum: the same value in every thread
    long long a = 0;
    long long cbase = -1;
    int slow = 0;     // consecutive short windows; >= kWinSlowRun: chain mode
    while (a < n) {
        if (SUMM && a % kWin == 0 && slow < kWinSlowRun) {
            const long long w = a / kWin;
            if (cbase < 0 || w >= cbase + kWinThreads) {
                __syncthreads();
                cbase = w;
                const long long nw = (n + kWin - 1) / kWin;
                if (cbase + tid < nw) sc[tid] = summ[cbase + tid];
                __syncthreads();
            }
            const WinSumm S = sc[w - cbase];
            int e = 0;
            const double fr = frexp(s, &e);
            if (S.ok && s != 0.0 && e == S.e) {
                const double M = ldexp(fr, 53);
                const bool inside = s > 0.0 ? (M + S.pmin >= lo && M + S.pmax <= hi)
                                            : (M + S.pmax <= -lo && M + S.pmin >= -hi);
                if (inside) {   // the whole window: the scan would have consumed it
                    s = ldexp(M + S.q, e - 53);
                    a += kWin;
                    continue;
                }
            }
            load(cur, a);
        }
        // this window: [a, lim); SUMM: up to the next aligned boundary
        const long long lim = SUMM ? ((a / kWin + 1) * kWin < n ? (a / kWin + 1) * kWin : n) : n;
        const long long rem = lim - a;
        const int wl = rem < kWin ? (int)rem : kWin;   // the window's terms
#pragma unroll
        for (int t = 0; t < kWinPer; ++t) buf[tid * kWinPer + t] = cur[t];
        if (!SUMM) load(nxt, a + kWin);   // speculative: the next window if this one is consumed whole
        if (slow >= kWinSlowRun) {         // chain mode: the reference's rounded adds, no scan
            __syncthreads();
#pragma unroll 8
            for (int j = 0; j < wl; ++j) s = s + buf[j];
            a += wl;
            if (SUMM) { if (a < n) load(cur, a); }
            else {
#pragma unroll
                for (int t = 0; t < kWinPer; ++t) cur[t] = nxt[t];
            }
            if (++slow >= kWinSlowRun + kWinChainRun) slow = 0;
            __syncthreads();
            continue;
        }
        int e = 0;
        const double fr = frexp(s, &e);
        // integers in units of u, held in doubles: every running value of a valid prefix lies in
        // [2^52, 2^53) and every partial sum of its k is a difference of two such values, so all
        // of it is exact; sums that run past the first failing term may round, but nothing past
        // that term is used
        const double M = s != 0.0 ? ldexp(fr, 53) : 0.0;
        const bool neg = s < 0.0;
        double kk[kWinPer];
        double tot = 0.0;
        int bad = kWinPer;   // first term of this thread that cannot take the shortcut
#pragma unroll
        for (int t = 0; t < kWinPer; ++t) {
            const double y = ldexp(cur[t], 53 - e);
            const double r = rint(y);
            const bool tie = fabs(y - r) == 0.5;
            const bool ok = s != 0.0 && fabs(y) < 4503599627370496.0 && !tie && (long long)(tid * kWinPer + t) < rem;
            kk[t] = ok ? r : 0.0;
            if (!ok && bad == kWinPer) bad = t;
            tot += kk[t];
        }
        // block scan of the thread totals: wave scans, then the wave totals in wave order
        double incl = tot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
        if (lane == 63) wtot[wave] = incl;
        __syncthreads();
        double woff = 0.0, all = 0.0;
#pragma unroll
        for (int w = 0; w < kWinWaves; ++w) {
            if (w < wave) woff += wtot[w];
            all += wtot[w];
        }
        double excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 0.0;
        excl += woff;
        double P = M + excl;   // running sum (units of u) before this thread's terms
#pragma unroll
        for (int t = 0; t < kWinPer; ++t) {
            P += kk[t];
            const double mag = neg ? -P : P;
            if (t < bad && (mag < lo || mag > hi)) bad = t;
        }
        int f = bad < kWinPer ? tid * kWinPer + bad : kWin;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
            const int o = __shfl_xor(f, d);
            f = o < f ? o : f;
        }
        if (lane == 0) wmin[wave] = f;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kWinWaves; ++w) f = wmin[w] < f ? wmin[w] : f;
        // exact running value before term f, from the thread that holds term f
        if (f < kWin && tid == f / kWinPer) {
            double pf = M + excl;
            const int tf = f % kWinPer;
#pragma unroll
            for (int t = 0; t < kWinPer; ++t)
                if (t < tf) pf += kk[t];
            pshare = pf;
        }
        __syncthreads();
        const double pf = f >= kWin ? M + all : pshare;
        if (f > 0) s = ldexp(pf, e - 53);
        if (f >= wl) {   // every term of the window took the shortcut
            slow = 0;
            a += wl;
            if (SUMM) { if (a < n && a % kWin != 0) load(cur, a); }
            else {
#pragma unroll
                for (int t = 0; t < kWinPer; ++t) cur[t] = nxt[t];
            }
            __syncthreads();
            continue;
        }
        s = s + buf[f];                    // the stopping term: the reference's rounded add
        if (f < 64) {                      // slow region: finish the window as a chain
            ++slow;
#pragma unroll 8
            for (int j = f + 1; j < wl; ++j) s = s + buf[j];
            a += wl;
            if (SUMM) { if (a < n && (a % kWin != 0 || slow >= kWinSlowRun)) load(cur, a); }
            else {
#pragma unroll
                for (int t = 0; t < kWinPer; ++t) cur[t] = nxt[t];
            }
        } else {
            slow = 0;
            a += f + 1;
            load(cur, a);
        }
        __syncthreads();
    }
    if (tid == 0) {
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
    const size_t nw = (size_t)((pixels + kWin - 1) / kWin);
    return 1024 * sizeof(double) + 2 * sizeof(double) + 258 * sizeof(uint32_t) + 256 +
           (size_t)pixels * sizeof(double) + nw * (sizeof(double) + sizeof(WinSumm)) + 16;
}

// avg = exp(sum of log(delta + Y) / pixelCount) into the scratch's avg slot (tonemap_avg_offset);
// mode < 0: the build / RTG_TM_SEQSUM default
void launch_log_average(const float* hdr, long long n, int mode, uint32_t idx, void* scratch, hipStream_t st) {
    char* p = (char*)scratch;
    double* partial = (double*)p;
    double* avg = partial + 1024;
    uint32_t* sel = (uint32_t*)(avg + 2);
    double* logs = (double*)(p + 1024 * sizeof(double) + 2 * sizeof(double) + 258 * sizeof(uint32_t) + 256);
    static const int dflt = [] {
        const char* v = std::getenv("RTG_TM_SEQSUM");
        return v && *v ? std::atoi(v) : RTG_TM_SEQSUM;
    }();
    if (mode < 0) mode = dflt;
    if (mode > 0) {
        hipLaunchKernelGGL(k_tm_log, dim3((unsigned)((n + kTmThreads - 1) / kTmThreads)), dim3(kTmThreads), 0, st,
                           hdr, n, logs);
        if (mode == 1) {
            hipLaunchKernelGGL(k_tm_seqsum, dim3(1), dim3(64), 0, st, logs, n, avg, sel, idx);
        } else if (mode == 2) {
            hipLaunchKernelGGL(k_tm_winsum<false>, dim3(1), dim3(kWinThreads), 0, st, logs, n, nullptr, avg, sel, idx);
        } else {
            const int nw = (int)((n + kWin - 1) / kWin);
            double* wtot = logs + n;
            WinSumm* summ = reinterpret_cast<WinSumm*>(wtot + nw);
            hipLaunchKernelGGL(k_tm_wtot, dim3(nw), dim3(256), 0, st, logs, n, wtot);
            hipLaunchKernelGGL(k_tm_wguess, dim3(1), dim3(64), 0, st, wtot, nw, summ);
            hipLaunchKernelGGL(k_tm_wsumm, dim3(nw), dim3(kWinThreads), 0, st, logs, n, summ);
            hipLaunchKernelGGL(k_tm_winsum<true>, dim3(1), dim3(kWinThreads), 0, st, logs, n, summ, avg, sel, idx);
        }
    } else {
        const int nb = (int)((n + kTmThreads - 1) / kTmThreads < 1024 ? (n + kTmThreads - 1) / kTmThreads : 1024);
        hipLaunchKernelGGL(k_tm_logsum, dim3(nb), dim3(kTmThreads), 0, st, hdr, n, partial);
        hipLaunchKernelGGL(k_tm_avg, dim3(1), dim3(kTmThreads), 0, st, partial, nb, n, avg, sel, idx);
    }
}

size_t tonemap_avg_offset() { return 1024 * sizeof(double); }

hipError_t launch_tonemap(const float* hdr, int width, int height, float key, float burn, float saturation,
                          float gamma, unsigned char* ldr, void* scratch, hipStream_t st) {
    const long long n = (long long)width * height;
    char* p = (char*)scratch;
    double* partial = (double*)p;
    double* avg = partial + 1024;
    uint32_t* sel = (uint32_t*)(avg + 2);
    uint32_t* hist = sel + 2;
    hipError_t e = hipMemsetAsync(hist, 0, 256 * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    // burn threshold index exactly as tonemapper.h:104-107 (float * int -> float -> int)
    const float thresholdPerct = (100.0f - burn) / 100;
    const int lastIdx = (int)(3 * n) - 1;
    int idx = (int)(thresholdPerct * lastIdx);
    if (idx > lastIdx) idx = lastIdx;
    if (idx < 0) idx = 0;
    launch_log_average(hdr, n, -1, (uint32_t)idx, scratch, st);
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
