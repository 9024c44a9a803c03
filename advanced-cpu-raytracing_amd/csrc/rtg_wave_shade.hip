// Wavefront shading kernels (k_shade variants, k_resolve) and the pipeline dispatcher.
#include <cstring>

#include "rtg_wave.hpp"

namespace rtg {

__global__ __launch_bounds__(256) void k_resolve(const DevCamera C, const RenderParams P, const int sample0,
                                                 const WaveBufs W, const PassOut O) {
    // entries of the pass's slabs (work_index): slab, compact row, column
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int slab = i / P.slab_px, r = i - slab * P.slab_px, crow = r / C.width;
    if (slab >= P.slabs || crow >= P.part_rows) return;
    const int pixel = part_row(P, crow) * C.width + (r - crow * C.width);
    const float4 b = W.base[i];
    const int flags = __float_as_int(b.w);
    f3 color = mk(b.x, b.y, b.z);
    if (!(flags & BASE_FINAL)) {
        f3 sum = mk(0, 0, 0);
        const int s0 = i * W.num_slots;
        for (int l = 0; l < W.num_slots; ++l)
            if (!W.occ[s0 + l]) {
                const float4 t = W.term[s0 + l];
                sum = add(sum, mk(t.x, t.y, t.z));
            }
        color = add(color, sum);
        if (flags & BASE_ADD_ZERO) color = add(color, mk(0, 0, 0));   // depth-0 mirror/dielectric/conductor
    }
    finish_pixel(C, P, sample0 + slab, O, pixel, slab, color);
}

// A multi-sample pass's colours (O.col, one per slab and pixel) into the pixels' accumulation,
// in sample order (accum_samples): the image of one-sample passes, bit for bit.
__global__ __launch_bounds__(256) void k_accum(const DevCamera C, const RenderParams P, const int sample0,
                                               const PassOut O) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int crow = i / C.width;
    if (crow >= P.part_rows) return;
    const int pixel = part_row(P, crow) * C.width + (i - crow * C.width);
    accum_samples(C, P, sample0, P.slabs, O.first, O.last, pixel, O.col + i, (size_t)P.slab_px, O.accum, O.hdr,
                  O.ldr);
}


// RTG_DEFER_DIAG=1: k_hitfix counts pending / checked-out pixels of production renders into
// extend_wide_visits / extend_fallbacks (tools/diag_defer.py); otherwise an uncounted render
// leaves the counters untouched, as every other pipeline does
bool defer_diag() {
    const char* v = std::getenv("RTG_DEFER_DIAG");
    return v && std::strcmp(v, "0") != 0;
}

// Large leaves of the camera walk deferred to k_bigleaf (production renders of large-leaf scenes;
// RTG_DEFER=0: the cooperative walk, A/B)
bool defer_leaves() {
    const char* v = std::getenv("RTG_DEFER");
    return !v || std::strcmp(v, "0") != 0;
}

// RTG_DEFER_ANY: shadow rays of large-leaf scenes -- 0 the cooperative reference walk (A/B,
// exactness cross-check), unset or 1 the deferring any-hit walk.  Round 5, with the lean
// any-hit walk, the deferring walk won on every large-leaf config against round 4's per-pass
// choice on the device (C3 5 527 -> 5 872, C3-ton 5 517 -> 5 602, C4 3 165 -> 3 164 Mrays/s;
// profiles/r05q_deferany_ab.txt), which was then removed
bool defer_any_leaves() {
    const char* v = std::getenv("RTG_DEFER_ANY");
    return !v || std::strcmp(v, "0") != 0;
}

// The fused layout's two kernels as one (k_shade<..., FRAME>, default since round 5;
// RTG_FRAME_KERNEL=0: k_primary + k_shade_shadow)
bool frame_kernel() {
    const char* e = std::getenv("RTG_FRAME_KERNEL");
    return !e || std::strcmp(e, "0") != 0;
}


template <bool STATS>
static hipError_t wave_shade_t(int sk, bool one, const DevScene& S, const DevCamera& C, const RenderParams& P,
                               int s, const WaveBufs& W, const PassOut& O, DevCounters* cnt, hipStream_t st) {
    if (!one) {
        hipLaunchKernelGGL((k_shade<STATS, SK_ALL, SH_GENERAL>), dim3(P.slab_tiles * P.slabs), dim3(256), 0, st, S, C,
                           P, s, W, O, cnt);
        return hipGetLastError();
    }
#define RTG_SK(K)                                                                                                  \
    case K:                                                                                                        \
        hipLaunchKernelGGL((k_shade<STATS, K, SH_ONE>), dim3(P.slab_tiles * P.slabs), dim3(256), 0, st, S, C, P, s, W, \
                           O, cnt);                                                                                 \
        break
    switch (sk & SK_ALL) {
        RTG_SK(0); RTG_SK(1); RTG_SK(2); RTG_SK(3); RTG_SK(4); RTG_SK(5); RTG_SK(6);
        default: RTG_SK(SK_ALL);
    }
#undef RTG_SK
    return hipGetLastError();
}

hipError_t wave_shade(bool stats, int sk, bool one, const DevScene& S, const DevCamera& C, const RenderParams& P,
                      int sample, const WaveBufs& W, const PassOut& O, DevCounters* cnt, hipStream_t st) {
    return stats ? wave_shade_t<true>(sk, one, S, C, P, sample, W, O, cnt, st)
                 : wave_shade_t<false>(sk, one, S, C, P, sample, W, O, cnt, st);
}

void wave_resolve(const DevCamera& C, const RenderParams& P, int sample, const WaveBufs& W, const PassOut& O,
                  hipStream_t st) {
    const long long n = P.slabs > 1 ? (long long)P.slabs * P.slab_px : (long long)P.part_rows * C.width;
    hipLaunchKernelGGL(k_resolve, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, C, P, sample, W, O);
}

void wave_accum(const DevCamera& C, const RenderParams& P, int sample, const WaveBufs& W, const PassOut& O,
                hipStream_t st) {
    const int npix = P.part_rows * C.width;
    hipLaunchKernelGGL(k_accum, dim3((npix + 255) / 256), dim3(256), 0, st, C, P, sample, O);
}

hipError_t launch_wave(const DevScene& S, const DevCamera& C, const RenderParams& P, const WaveBufs& W, float* hdr,
                       unsigned char* l, DevCounters* cnt, bool stats, int feat, int sk, hipStream_t stream,
                       hipEvent_t* ev, int* layout) {
    // traversal variants: meshes only (identity transforms) / + spheres / everything,
    // each with the sequential or the cooperative (large-leaf) BVH walk
    const bool big = (feat & FEAT_BIGLEAF) != 0;
    const int base = feat & ~FEAT_BIGLEAF;
#define RTG_WAVE(F) return launch_wave_f<F>(S, C, P, W, hdr, l, cnt, stats, sk, stream, ev, layout)
    if (base == 0) {
        if (big) RTG_WAVE(FEAT_BIGLEAF);
        RTG_WAVE(0);
    }
    if (base == FEAT_SPHERE) {
        if (big) RTG_WAVE(FEAT_SPHERE | FEAT_BIGLEAF);
        RTG_WAVE(FEAT_SPHERE);
    }
    if (big) RTG_WAVE(FEAT_ALL);
    RTG_WAVE(FEAT_ALL & ~FEAT_BIGLEAF);
#undef RTG_WAVE
}

}  // namespace rtg
