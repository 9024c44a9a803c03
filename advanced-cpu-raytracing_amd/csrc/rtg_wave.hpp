// Wavefront render pipeline (kernels; launched from rtg_wave_*.hip) for scenes whose rays do not branch (no reflection /
// refraction children, no motion blur): every camera ray is one closest-hit query, and
// every hit spawns one shadow query per light.  Per sample pass:
//
//   k_primary  one thread per pixel: GenerateRay + IntersectObjects -> hit (t,obj,face)
//              lean kernel: the traversal loop alone sets its register budget
//   k_shade    one thread per pixel: PerformShading up to the light loop -- ambient,
//              and for every light (reference order: point, area, env, dir, spot) the
//              Shade() term and, where the reference casts one, a shadow ray.  Shadow
//              rays are compacted into a dense queue with a wave ballot + mbcnt prefix
//              sum and one atomic per wave.
//   k_shadow   one thread per queued shadow ray: CastShadowRay as early-exit any-hit
//   k_resolve  one thread per pixel: SampleDirectLighting's sum over unshadowed lights
//              in light order, the PerformShading sum, LDR clamp / spp accumulation
//
// The float operations and their order are those of the fused kernel / the reference
// (only unshadowed terms are summed, left to right), so both paths produce the same bits.
#pragma once
#include <cstdlib>

#include "rtg_common.hpp"
#include "rtg_kernels.hpp"

namespace rtg {

enum { BASE_FINAL = 1, BASE_ADD_ZERO = 2 };

// k_shade's environment-light directions searched by the whole wave (env_direction_wave);
// 0: each lane's own loop (A/B)
#ifndef RTG_ENV_WAVE
#define RTG_ENV_WAVE 1
#endif

// ORD: RTG_RENDER_ORDERED (plain mesh scenes): the checked closest-hit walk on the any-hit tree
// as wave packets (trace_closest_pk), the reference walk where its check fails
#ifndef RTG_ORD_WAVES
#define RTG_ORD_WAVES RTG_WIDE_WAVES_PLAIN
#endif
template <bool STATS, int FEAT, bool ORD = false, bool DEFER = false>
__global__ __launch_bounds__(256, ORD ? RTG_ORD_WAVES : RTG_TRACE_WAVES(FEAT)) void k_primary(
    const DevScene S, const DevCamera C, const RenderParams P, const int sample0, const WaveBufs W,
    DevCounters* counters) {
    int px, py, crow, slab;
    tile_pixel(P, px, py, crow, slab);
    const int sample = sample0 + slab;
    Cnt<STATS> cn;
    if (px < C.width && py < P.row_end) {
        const int pixel = px + py * C.width;
        const int i = work_index(P, C.width, slab, crow, px);
        const uint64_t key = root_key(P.seed, pixel, sample);
        float mbTime;
        Ray ray = camera_ray(C, px, py, key, mbTime);
        cn.cam();
        Hit h;
        if constexpr (ORD) {
            if (!trace_closest_pk<STATS, FEAT>(S, ray, h, cn)) {
                cn.efallback();
                trace<false, STATS, FEAT>(S, ray, mbTime, INFINITY, INFINITY, h, cn);
            }
        } else if constexpr (DEFER) {
            // large leaves deferred to k_bigleaf; k_hitfix settles the pixel (rtg_common.hpp DeferCtx)
            DeferCtx dc{W.dq_e, W.dq_count, W.dq_cap, i, false};
            trace<false, STATS, FEAT, true, true>(S, ray, mbTime, INFINITY, INFINITY, h, cn, &dc);
            if (dc.deferred) {
                W.hit_key[i] = h.obj >= 0 ? obj_key(h.t, h.obj, h.face) : ~0ull;
                W.hit_obj[i] = -2;                         // pending
                flush_counters<STATS>(cn, counters);
                return;
            }
        } else {
            trace<false, STATS, FEAT, RTG_PRIMARY_PACKET != 0 && !(FEAT & FEAT_BIGLEAF)>(S, ray, mbTime, INFINITY,
                                                                                       INFINITY, h, cn);
        }
        W.hit_t[i] = h.t;
        W.hit_obj[i] = h.obj;
        W.hit_face[i] = h.face;
    }
    flush_counters<STATS>(cn, counters);
}

// The deferred large leaves: one wave per queue entry (grid-stride), its lanes testing the leaf's
// faces against the entry's local ray at the minT the walk had at the leaf (IntersectFace's
// acceptance t < minT: the faces the reference's sequential loop could keep), the (t, object,
// face) minimum folded into the pixel's key with one 64-bit atomic min.
template <int FEAT>
__global__ __launch_bounds__(256) void k_bigleaf(const DevScene S, const WaveBufs W) {
    const int n = min(*W.dq_count, W.dq_cap);
    const int lane = threadIdx.x & 63;
    for (int e = (int)((blockIdx.x * 256u + threadIdx.x) >> 6); e < n; e += gridDim.x * 4) {
        const float4 a = W.dq_e[3 * (size_t)e], b = W.dq_e[3 * (size_t)e + 1], q = W.dq_e[3 * (size_t)e + 2];
        Ray lr;
        lr.o = mk(a.x, a.y, a.z);
        lr.d = mk(b.x, b.y, b.z);
        const float minT = a.w;
        const int ray = __float_as_int(b.w), first = __float_as_int(q.x), cnt = __float_as_int(q.y);
        const int k = __float_as_int(q.z);
        uint64_t best = ~0ull;
        for (int f = first + lane; f < first + cnt; f += 64) {
            float t;
            if (tri_test_fast(S, f, lr, minT, t)) {
                const uint64_t key = obj_key(t, k, f);
                best = key < best ? key : best;
            }
        }
        best = wave_min_key(best, __ballot(1));
        if (lane == 0 && best != ~0ull) atomicMin(&W.hit_key[ray], (unsigned long long)best);
    }
}

// A pending pixel's hit from its key, checked: the winner's reference leaf box (and an
// instance's world box) must pass the exact slab test at next_up(t) -- else the reference walk
// decides (rtg_common.hpp DeferCtx).
// (diagnostics, RTG_DEFER_DIAG=1 only -- counters is null otherwise: extend_wide_visits counts
// the pending pixels and extend_fallbacks those the check sent to the reference walk)
template <int FEAT>
__global__ __launch_bounds__(256) void k_hitfix(const DevScene S, const DevCamera C, const RenderParams P,
                                                const int sample0, const WaveBufs W, DevCounters* counters) {
    int px, py, crow, slab;
    tile_pixel(P, px, py, crow, slab);
    const int sample = sample0 + slab;
    const int i = work_index(P, C.width, slab, crow, px);
    const bool pending = px < C.width && py < P.row_end && W.hit_obj[i] == -2;
    const uint64_t pm = __ballot(pending);
    if (counters && pm && (threadIdx.x & 63) == __ffsll((long long)pm) - 1)
        atomicAdd(&counters->extend_wide_visits, (unsigned long long)__popcll(pm));
    if (!pending) return;
    const uint64_t key = W.hit_key[i];
    const int pixel = px + py * C.width;
    float mbTime;
    Ray ray = camera_ray(C, px, py, root_key(P.seed, pixel, sample), mbTime);
    Hit h;
    h.t = INFINITY;
    h.obj = -1;
    h.face = -1;
    bool sure = true;
    if (key != ~0ull) {
        h.t = __uint_as_float((uint32_t)(key >> 32));
        h.obj = (int)((key >> 20) & 0xFFFu);
        const int f = (int)(key & 0xFFFFFu);
        const DevObject& ob = S.objects[h.obj];
        if (ob.kind == OBJ_SPHERE) {
            h.face = -1;
        } else {
            h.face = f;
            const float up = next_up(h.t);
            if (ob.kind == OBJ_INSTANCE)
                sure &= box_hit(ob.bmin[0], ob.bmin[1], ob.bmin[2], ob.bmax[0], ob.bmax[1], ob.bmax[2], ray, up);
            const Ray lr = (FEAT & FEAT_XFORM) ? trav_ray(ob, ray, mbTime) : ray;
            const int leaf = S.face_leaf[f];
            const float4 a = S.nodes[2 * leaf], b = S.nodes[2 * leaf + 1];
            sure &= box_hit(a.x, a.y, a.z, a.w, b.x, b.y, lr, up);
        }
    }
    // a winner that fails the check: the pixel goes to k_refwalk (the reference walk, one ray per
    // wave); its slot in the (now consumed) entry memory, the count in dq_count[1]
    const uint64_t fm = __ballot(!sure);
    if (fm) {
        const int lane = threadIdx.x & 63, lead = __ffsll((long long)fm) - 1;
        int base = 0;
        if (lane == lead) {
            base = atomicAdd(W.dq_count + 1, __popcll(fm));
            if (counters) atomicAdd(&counters->extend_fallbacks, (unsigned long long)__popcll(fm));
        }
        base = __shfl(base, lead);
        if (!sure) {
            reinterpret_cast<int*>(W.dq_e)[base + __popcll(fm & ((1ull << lane) - 1ull))] = i;
            return;
        }
    }
    W.hit_t[i] = h.t;
    W.hit_obj[i] = h.obj;
    W.hit_face[i] = h.face;
}

// IntersectObjects for one ray per wave (the pixels k_hitfix could not settle): every lane holds
// the same ray and takes the same decisions, and a leaf's faces are dealt over the lanes, 64 at a
// time -- the minimum (t, face) with t below minT of each chunk is exactly what the reference's
// sequential loop keeps from it (acceptance t < minT, minT shrinking), so the walk is the
// reference walk with its leaf loops run 64 wide.
template <int FEAT>
DEV bool trace_wave(const DevScene& S, Ray& r, float mbTime, Hit& h) {
    const int lane = threadIdx.x & 63;
    h.t = INFINITY;
    h.obj = -1;
    h.face = -1;
    const RayRcp rq = ray_rcp(r);
    for (int k = 0; k < S.num_objects; ++k) {
        const DevObject& ob = S.objects[k];
        if ((FEAT & FEAT_INSTANCE) && ob.group_end > k) {
            const float4 ga = S.group_box[2 * k], gb = S.group_box[2 * k + 1];
            if (!box_hit_fast(ga.x, ga.y, ga.z, gb.x, gb.y, gb.z, r, rq, h.t)) {
                k = ob.group_end - 1;
                continue;
            }
        }
        if ((FEAT & FEAT_SPHERE) && ob.kind == OBJ_SPHERE) {
            const Ray lr = trav_ray(ob, r, mbTime);
            float t;
            if (sphere_t(ob, lr, h.t, t)) { h.t = t; h.obj = k; h.face = -1; h.o = r.o; }
            continue;
        }
        if ((FEAT & FEAT_INSTANCE) && ob.kind == OBJ_INSTANCE) {
            Ray wr = r;
            if (ob.flags & OBJF_MOTION_BLUR) wr.o = add(wr.o, muls(ld3(ob.mbv), mbTime));
            if (!box_hit_fast(ob.bmin[0], ob.bmin[1], ob.bmin[2], ob.bmax[0], ob.bmax[1], ob.bmax[2], wr, rq, h.t)) {
                r.o = wr.o;
                continue;
            }
        }
        const Ray lr = (FEAT & FEAT_XFORM) ? trav_ray(ob, r, mbTime) : r;
        const RayRcp q = ray_rcp(lr);
        float minT = h.t;
        int face = -1;
        for (int i = ob.node_begin; i < ob.node_end;) {
            const float4 a = S.nodes[2 * i], b = S.nodes[2 * i + 1];
            const int skip = __float_as_int(b.z), leaf = __float_as_int(b.w);
            if (!box_hit_fast(a.x, a.y, a.z, a.w, b.x, b.y, lr, q, minT)) {
                i = skip;
                continue;
            }
            if (leaf < 0) {
                ++i;
                continue;
            }
            int first = leaf >> 8, cnt = leaf & 255;
            if (leaf == LEAF_EXT) {
                const int2 e = S.node_ext[i];
                first = e.x;
                cnt = e.y;
            }
            for (int c0 = first; c0 < first + cnt; c0 += 64) {
                const int f = c0 + lane;
                float t;
                const bool ok = f < first + cnt && tri_test_fast(S, f, lr, minT, t);
                const uint64_t best = wave_min_key(ok ? hit_key(t, f) : ~0ull, __ballot(1));
                if (best != ~0ull) {
                    minT = __uint_as_float((uint32_t)(best >> 32));
                    face = (int)(uint32_t)best;
                }
            }
            i = skip;
        }
        if (face >= 0) { h.t = minT; h.obj = k; h.face = face; h.o = r.o; }
    }
    return h.obj >= 0;
}

template <int FEAT>
__global__ __launch_bounds__(256) void k_refwalk(const DevScene S, const DevCamera C, const RenderParams P,
                                                 const int sample0, const WaveBufs W) {
    const int n = W.dq_count[1];
    for (int e = (int)((blockIdx.x * 256u + threadIdx.x) >> 6); e < n; e += gridDim.x * 4) {
        const int i = reinterpret_cast<const int*>(W.dq_e)[e];
        const int slab = i / P.slab_px;
        const int pixel = work_pixel(P, C.width, slab, i);
        const int py = pixel / C.width, px = pixel - py * C.width;
        float mbTime;
        Ray ray = camera_ray(C, px, py, root_key(P.seed, pixel, sample0 + slab), mbTime);
        Hit h;
        trace_wave<FEAT>(S, ray, mbTime, h);
        if ((threadIdx.x & 63) == 0) {
            W.hit_t[i] = h.t;
            W.hit_obj[i] = h.obj;
            W.hit_face[i] = h.face;
        }
    }
}

// wave-aggregated append to the block's queue segment: ballot + mbcnt rank, one LDS
// atomic per wave; returns this lane's index in the segment (or -1)
DEV int queue_append(bool want, int* lds_count) {
    const unsigned long long mask = __ballot(want);
    if (!mask) return -1;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(lds_count, __popcll(mask));
    base = __shfl(base, leader);
    const int rank = __popcll(mask & ((1ull << lane) - 1ull));
    return want ? base + rank : -1;
}

// Output of a sample pass: final image (spp 1) or the multi-sample accumulator; a pass of
// several sample slabs (RenderParams::slabs > 1) writes each colour to `col` (work-buffer
// index) and k_accum adds them to the accumulator in sample order.
struct PassOut {
    float* hdr;
    unsigned char* ldr;
    float4* accum;
    int first, last;
    float4* col;
};

// renderThreadMain's per-pixel end of a sample pass (main.cpp:80-121): the colour itself at
// 1 spp, else the Gaussian-weighted accumulation, divided out after the last sample.  A
// multi-sample pass stores the colour in the pixel's entry of its sample slab (work_index,
// derived from the pixel here: the callers keep only the pixel live across their walks).
DEV void finish_pixel(const DevCamera& C, const RenderParams& P, int sample, const PassOut& O, int pixel, int slab,
                      f3 color) {
    if (O.col) {
        const int py = pixel / C.width, px = pixel - py * C.width;
        const int r = py - P.row_begin;
        const int crow = ((r >> 3) / P.part_count) * 8 + (r & 7);   // part_row's inverse
        O.col[work_index(P, C.width, slab, crow, px)] = make_float4(color.x, color.y, color.z, 0.f);
        return;
    }
    if (C.spp <= 1 && !P.accum_only) {
        const size_t idx = 3 * (size_t)pixel;
        if (O.hdr) { O.hdr[idx] = color.x; O.hdr[idx + 1] = color.y; O.hdr[idx + 2] = color.z; }
        if (O.ldr) { O.ldr[idx] = ldr(color.x); O.ldr[idx + 1] = ldr(color.y); O.ldr[idx + 2] = ldr(color.z); }
        return;
    }
    int pk = pixel;                  // (recomputed, not merged with the caller's key: see area_light)
    asm volatile("" : "+v"(pk));
    const float gw = sample_weight(C.spp, sample, root_key(P.seed, pk, sample));
    float4 a = O.first ? make_float4(0.f, 0.f, 0.f, 0.f) : O.accum[pixel];
    a.x += color.x * gw;
    a.y += color.y * gw;
    a.z += color.z * gw;
    a.w += gw;
    O.accum[pixel] = a;
    if (O.last && !P.accum_only) {
        const f3 c = mk(a.x / a.w, a.y / a.w, a.z / a.w);
        const size_t idx = 3 * (size_t)pixel;
        if (O.hdr) { O.hdr[idx] = c.x; O.hdr[idx + 1] = c.y; O.hdr[idx + 2] = c.z; }
        if (O.ldr) { O.ldr[idx] = ldr(c.x); O.ldr[idx + 1] = ldr(c.y); O.ldr[idx + 2] = ldr(c.z); }
    }
}

// PerformShading's sum for a pixel with at most one light (k_resolve's loop, one slot):
// ambient + (0 + term if the light is unoccluded) [+ the zero child term].
DEV f3 resolve_one(f3 base, int flags, bool has_term, f3 term, bool occluded) {
    if (flags & BASE_FINAL) return base;
    f3 sum = mk(0, 0, 0);
    if (has_term && !occluded) sum = add(sum, term);
    f3 color = add(base, sum);
    if (flags & BASE_ADD_ZERO) color = add(color, mk(0, 0, 0));   // depth-0 mirror/dielectric/conductor
    return color;
}

// The same with a second, unshadowed term after it (one shadow-casting point / area light
// followed by an environment light, which casts no shadow ray, raytracer.cpp:741-755): k_resolve's
// loop over the two slots -- (0 + term if unoccluded) + env term.
DEV f3 resolve_two(f3 base, int flags, bool has_term, f3 term, bool occluded, bool has_term2, f3 term2) {
    if (flags & BASE_FINAL) return base;
    f3 sum = mk(0, 0, 0);
    if (has_term && !occluded) sum = add(sum, term);
    if (has_term2) sum = add(sum, term2);
    f3 color = add(base, sum);
    if (flags & BASE_ADD_ZERO) color = add(color, mk(0, 0, 0));   // depth-0 mirror/dielectric/conductor
    return color;
}

// PerformShading's sum with the unoccluded light terms already summed in light order.
DEV f3 resolve_sum(f3 base, int flags, f3 sum) {
    if (flags & BASE_FINAL) return base;
    f3 color = add(base, sum);
    if (flags & BASE_ADD_ZERO) color = add(color, mk(0, 0, 0));   // depth-0 mirror/dielectric/conductor
    return color;
}

// SK: shading variant (rtg_common.hpp SK_*).  MODE:
//   SH_GENERAL  every light slot's term and occlusion flag to the per-pixel buffers, shadow
//               rays to the block's queue segment (k_shadow, k_resolve follow);
//   SH_ONE      at most one light with a shadow ray, and at most one environment light after
//               it (W.pay3; C4's point + environment light): the pixel is finished here when
//               it casts no shadow ray, else its base colour and light term(s) travel with
//               the shadow ray in the queue (q_pay) and k_shadow_one finishes it;
//   SH_FUSED    at most one light, plain shading (SK 0): the lane casts its own shadow ray
//               (any-hit walk of FEAT, FAST) and finishes its pixel -- no queue.  Almost
//               every pixel of a scene that fills the frame casts one, and the ones that do
//               not leave whole waves idle only along silhouettes.
//   SH_FUSED_N  the same for plain scenes with several point / area / directional lights:
//               each light's Shade term and its shadow ray in turn, the unoccluded terms
//               summed in light order as k_resolve sums them (a separate instantiation: the
//               loop costs the one-light kernel 15 %)
enum { SH_GENERAL = 0, SH_ONE = 1, SH_FUSED = 2, SH_FUSED_N = 3 };
// FRAME (SH_FUSED / SH_FUSED_N only; RTG_FRAME_KERNEL): the lane also traces its camera ray
// (k_primary's walk) instead of reading the hit buffers -- the whole sample pass in one launch
template <bool STATS, int SK, int MODE, int FEAT = 0, bool FAST = false, bool FRAME = false>
__global__ __launch_bounds__(256, MODE >= SH_FUSED ? (FAST ? RTG_WIDE_WAVES(FEAT) : RTG_TRACE_WAVES(FEAT))
                                                   : RTG_SHADE_WAVES) void k_shade(const DevScene S, const DevCamera C,
                                                                                   const RenderParams P,
                                                                                   const int sample0, const WaveBufs W,
                                                                                   const PassOut O,
                                                                                   DevCounters* counters) {
    constexpr bool ONE = MODE != SH_GENERAL;
    __shared__ int seg_count;
    if (threadIdx.x == 0) seg_count = 0;
    __syncthreads();
    int px, py, crow, slab;
    tile_pixel(P, px, py, crow, slab);
    const int sample = sample0 + slab;
    const size_t seg = (size_t)blockIdx.x * 256 * (ONE ? 1 : W.num_slots);   // (ONE: one shadow ray per pixel)
    Cnt<STATS> cn;
    const bool valid = px < C.width && py < P.row_end;
    const int pixel = valid ? px + py * C.width : 0;
    const int i = valid ? work_index(P, C.width, slab, crow, px) : 0;
    const uint64_t key = root_key(P.seed, pixel, sample);
    static_assert(!FRAME || MODE >= SH_FUSED, "the frame kernel is the fused layout's");
    Hit fh;                          // FRAME: the camera ray's hit
    fh.obj = -1;
    if constexpr (FRAME) {
        if (valid) {
            float mbt;
            Ray cr = camera_ray(C, px, py, key, mbt);
            cn.cam();
            trace<false, STATS, FEAT, RTG_PRIMARY_PACKET != 0 && !(FEAT & FEAT_BIGLEAF)>(S, cr, mbt, INFINITY, INFINITY,
                                                                                           fh, cn);
        }
    }
    const int obj = FRAME ? fh.obj : (valid ? W.hit_obj[i] : -1);
    // the camera walk's deferral counters back to zero for the next pass (k_bigleaf / k_refwalk,
    // their last readers, ran before this kernel; no memset launch per pass)
    if (!FRAME && W.dq_e && blockIdx.x == 0 && threadIdx.x == 0) {
        W.dq_count[0] = 0;
        W.dq_count[1] = 0;
    }
    // lanes that need the light loop
    bool lit = false;
    ShadeCtx c;
    f3 w_o = mk(0, 0, 0);
    f3 base = mk(0, 0, 0);           // ONE: the pixel's base colour, flags, light term
    int bflags = 0;
    f3 term1 = mk(0, 0, 0);
    bool has_term = false, pushed = false;
    f3 term2 = mk(0, 0, 0);          // SH_ONE: the environment light's term after the shadowed one
    bool has_term2 = false;
    float4 ro = make_float4(0.f, 0.f, 0.f, 0.f), rd = ro;      // SH_FUSED: the shadow ray
    auto put_base = [&](f3 col, int flags) {
        if (ONE) { base = col; bflags = flags; }
        else W.base[i] = make_float4(col.x, col.y, col.z, __int_as_float(flags));
    };
    if (valid) {
        float mbTime;
        Ray ray = camera_ray(C, px, py, key, mbTime);
        if (obj < 0) {
            put_base(miss_color<SK>(S, C, px, py, ray.d), BASE_FINAL);
        } else {
            const DevObject& ob = S.objects[obj];
            Hit h;
            h.t = FRAME ? fh.t : W.hit_t[i];
            h.obj = obj;
            h.face = FRAME ? fh.face : W.hit_face[i];
            h.o = ray.o;
            c.ob = &ob;
            c.mat = &S.materials[ob.material];
            c.s = surface<STATS, (SK & SK_TEX) != 0>(S, ray, mbTime, h, cn);
            w_o = makeUnit(sub(ld3(C.pos), c.s.p));
            const DevMaterial& mat = *c.mat;
            if (mat.type == 3) {                                    // Emissive (raytracer.cpp:81-84)
                put_base(muls(muls(ld3(mat.radiance), 2.0f), (float)RT_PI), BASE_FINAL);
            } else if ((SK & SK_TEX) && ob.tex_replace_all >= 0) {  // replace_all (:87-89)
                put_base(tex_rgb(S, S.textures[ob.tex_replace_all], c.s.u, c.s.v), BASE_FINAL);
            } else {
                // primary rays travel in vacuum (medium 1.0): ambient + direct always apply
                f3 color = add(mk(0, 0, 0), mulv(mk(S.ambient[0], S.ambient[1], S.ambient[2]), ld3(mat.ambient)));
                const int flags = (mat.type == 0 || mat.type == 1 || mat.type == 2) ? BASE_ADD_ZERO : 0;
                put_base(color, flags);
                lit = true;
            }
        }
    }
    // ---- lights, in SampleDirectLighting's order (raytracer.cpp:706-803)
    int slot = i * W.num_slots;
    // the hit point and normal by reference: a lane that is not lit never reads them (every use
    // is behind `lit` / push's `want`), and selected copies kept a second set of six VGPRs live
    // next to the surface record through the light loops (36 B of scratch per lane at seven waves)
    const f3 &p = c.s.p, &n = c.s.n;
    if constexpr (MODE == SH_FUSED_N) {
        // SK 0: point, area and directional lights only, in that order; one shadow-walk call site
        f3 sum = mk(0, 0, 0);
        const int np = S.num_point, na = S.num_area, nsl = np + na + S.num_dir;
        for (int sl = 0; sl < nsl && lit; ++sl) {
            f3 term, tgt;
            bool directional = false;
            if (sl < np) {
                const f3 lp = ld3(S.point_lights[sl].pos);
                f3 w_i = makeUnit(sub(lp, p));
                float dist = len(sub(lp, p));
                term = shade<false, SK>(S, c, w_i, w_o, divs(ld3(S.point_lights[sl].intensity), dist * dist));
                tgt = lp;
            } else if (sl < np + na) {
                const int l = sl - np;
                const DevAreaLight& L = S.area_lights[l];
                float offU = rnd(key, RP_AREA, 2 * l) - 0.5f;
                float offV = rnd(key, RP_AREA, 2 * l + 1) - 0.5f;
                const f3 sp = add(add(ld3(L.pos), muls(ld3(L.u), L.extent * offU)), muls(ld3(L.v), L.extent * offV));
                f3 w_i = sub(sp, p);
                float dist = len(w_i);
                float dSqr = dist * dist;
                w_i = divs(w_i, dist);
                float lc = dot(ld3(L.normal), neg(w_i));
                if (lc < 0) lc = dot(ld3(L.normal), w_i);
                term = shade<false, SK>(S, c, w_i, w_o, muls(ld3(L.radiance), L.area * lc / dSqr));
                tgt = sp;
            } else {
                const f3 ldir = ld3(S.dir_lights[sl - np - na].dir);
                term = shade<false, SK>(S, c, neg(ldir), w_o, ld3(S.dir_lights[sl - np - na].radiance));
                tgt = ldir;
                directional = true;
            }
            // IsInShadow / IsInShadowDirectional (raytracer.cpp:555-584)
            cn.shd();
            const f3 o = add(p, muls(n, S.eps));
            float4 qo, qd;
            if (directional) {
                const f3 d = neg(tgt);
                qo = make_float4(o.x, o.y, o.z, INFINITY);
                qd = make_float4(d.x, d.y, d.z, INFINITY);
            } else {
                const f3 dir = sub(tgt, p);
                const float lightT = len(dir);
                const f3 d = divs(dir, lightT);
                qo = make_float4(o.x, o.y, o.z, lightT + 0.01f);
                qd = make_float4(d.x, d.y, d.z, lightT);
            }
            if (!shadow_occluded<STATS, FEAT, FAST>(S, W, 0, qo, qd, cn)) sum = add(sum, term);
        }
        if (valid) finish_pixel(C, P, sample, O, pixel, slab, resolve_sum(base, bflags, sum));
    } else {
    auto push = [&](bool want, f3 target_dir_or_pos, bool directional) {
        // IsInShadow / IsInShadowDirectional shadow-ray set-up (raytracer.cpp:555-584)
        float4 qo, qd;
        if (want) {
            cn.shd();
            const f3 o = add(p, muls(n, S.eps));
            if (directional) {
                const f3 d = neg(target_dir_or_pos);
                qo = make_float4(o.x, o.y, o.z, INFINITY);
                qd = make_float4(d.x, d.y, d.z, INFINITY);
            } else {
                const f3 dir = sub(target_dir_or_pos, p);
                const float lightT = len(dir);
                const f3 d = divs(dir, lightT);
                qo = make_float4(o.x, o.y, o.z, lightT + 0.01f);
                qd = make_float4(d.x, d.y, d.z, lightT);
            }
        }
        if constexpr (ONE) {
            // (SH_ONE: queued after the light loops, with every term of the pixel)
            if (want) { ro = qo; rd = qd; pushed = true; }
            return;
        }
        const int qi = queue_append(want, &seg_count);
        if (want) {
            const size_t q = seg + qi;
            W.q_o[q] = qo;
            W.q_d[q] = qd;
            W.q_slot[q] = slot;
            W.occ[slot] = 0;
        }
    };
    auto put = [&](f3 t) {
        if constexpr (MODE == SH_ONE) {
            if (has_term) { term2 = t; has_term2 = true; }   // the environment light after the shadowed one
            else { term1 = t; has_term = true; }
        } else if constexpr (ONE) {
            term1 = t;
            has_term = true;
        } else {
            W.term[slot] = make_float4(t.x, t.y, t.z, 0.f);
        }
    };
    auto point_light = [&](int l) {
        const f3 lp = ld3(S.point_lights[l].pos);
        if (lit) {
            f3 w_i = makeUnit(sub(lp, p));
            float dist = len(sub(lp, p));
            put(shade<false, SK>(S, c, w_i, w_o, divs(ld3(S.point_lights[l].intensity), dist * dist)));
        }
        push(lit, lp, false);
    };
    auto area_light = [&](int l) {
        f3 sp = mk(0, 0, 0);
        if (lit) {
            const DevAreaLight& L = S.area_lights[l];
            // the pixel's RNG key again (a few integer ops) rather than two VGPRs kept through the
            // point lights' shading; the laundered pixel index stops the compiler from merging it
            // with the first computation
            int pk = pixel;
            asm volatile("" : "+v"(pk));
            const uint64_t akey = root_key(P.seed, pk, sample);
            float offU = rnd(akey, RP_AREA, 2 * l) - 0.5f;
            float offV = rnd(akey, RP_AREA, 2 * l + 1) - 0.5f;
            sp = add(add(ld3(L.pos), muls(ld3(L.u), L.extent * offU)), muls(ld3(L.v), L.extent * offV));
            f3 w_i = sub(sp, p);
            float dist = len(w_i);
            float dSqr = dist * dist;
            w_i = divs(w_i, dist);
            float lc = dot(ld3(L.normal), neg(w_i));
            if (lc < 0) lc = dot(ld3(L.normal), w_i);
            put(shade<false, SK>(S, c, w_i, w_o, muls(ld3(L.radiance), L.area * lc / dSqr)));
        }
        push(lit, sp, false);
    };
    auto dir_light = [&](int l) {
        const f3 ldir = ld3(S.dir_lights[l].dir);
        if (lit) put(shade<false, SK>(S, c, neg(ldir), w_o, ld3(S.dir_lights[l].radiance)));
        push(lit, ldir, true);
    };
    for (int l = 0; l < S.num_point; ++l, ++slot) point_light(l);
    for (int l = 0; l < S.num_area; ++l, ++slot) area_light(l);
    if constexpr ((SK & SK_XLIGHT) != 0) {
        for (int l = 0; l < S.num_env; ++l, ++slot) {
            // (the wave searches its lanes' directions together; every lane takes part)
#if RTG_ENV_WAVE
            const f3 sd = env_direction_wave(S, lit ? n : mk(0, 0, 1), key, l, lit);
#else
            const f3 sd = lit ? env_direction(S, n, key, l) : mk(0, 0, 0);
#endif
            if (lit) {                                               // no shadow ray (:741-755)
                put(shade<false, SK>(S, c, n, w_o, env_sample(S, l, sd)));
                if (!ONE) W.occ[slot] = 0;
            }
        }
    }
    for (int l = 0; l < S.num_dir; ++l, ++slot) dir_light(l);
    if constexpr ((SK & SK_XLIGHT) != 0) {
        for (int l = 0; l < S.num_spot; ++l, ++slot) {
            const DevSpotLight& L = S.spot_lights[l];
            const f3 lp = ld3(L.pos);
            if (lit) {
                f3 w_i = makeUnit(sub(lp, p));
                float distToPoint = len(sub(p, lp));                 // spotLight.h:33-57
                f3 toPoint = divs(sub(p, lp), distToPoint);
                double alpha = angleBetween(ld3(L.dir), toPoint);
                f3 E;
                if (alpha <= 0 || alpha > (L.coverage_deg / 2.0f)) {
                    E = mk(0, 0, 0);
                } else {
                    float distSqr = distToPoint * distToPoint;
                    E = divs(ld3(L.intensity), distSqr);
                    if (alpha > (L.falloff_deg / 2.0f)) {
                        double cosAlpha = cos(alpha * (RT_PI / 180.0f));
                        double sv = pow((cosAlpha - L.cos_half_coverage) / (L.cos_half_falloff - L.cos_half_coverage),
                                        (double)4.0f);
                        E = muls(E, (float)sv);
                    }
                }
                put(shade<false, SK>(S, c, w_i, w_o, E));
            }
            push(lit, lp, false);
        }
        for (int l = 0; l < S.num_mesh; ++l, ++slot) {              // mesh lights (:780-803)
            f3 sp = mk(0, 0, 0);
            if (lit) {
                f3 E;
                mesh_light_sample(S, l, key, sp, E);
                f3 w_i = sub(sp, p);
                float dist = len(w_i);
                w_i = divs(w_i, dist);
                put(shade<false, SK>(S, c, w_i, w_o, E));
            }
            push(lit, sp, false);
        }
    }
    if constexpr (MODE == SH_FUSED) {
        if (pushed) {
            const bool occluded = shadow_occluded<STATS, FEAT, FAST>(S, W, 0, ro, rd, cn);
            finish_pixel(C, P, sample, O, pixel, slab, resolve_one(base, bflags, true, term1, occluded));
        } else if (valid) {
            finish_pixel(C, P, sample, O, pixel, slab, resolve_one(base, bflags, has_term, term1, false));
        }
    }
    if constexpr (MODE == SH_ONE) {
        // the shadow ray with the pixel's base colour and terms, or the pixel finished here
        const int qi = queue_append(pushed, &seg_count);
        if (pushed) {
            const size_t q = seg + qi;
            W.q_o[q] = ro;
            W.q_d[q] = rd;
            const size_t pq = (W.pay3 ? 3 : 2) * q;
            W.q_pay[pq] = make_float4(base.x, base.y, base.z, __int_as_float(bflags));
            W.q_pay[pq + 1] = make_float4(term1.x, term1.y, term1.z, __int_as_float(pixel));
            if (W.pay3) W.q_pay[pq + 2] = make_float4(term2.x, term2.y, term2.z, __int_as_float(has_term2 ? 1 : 0));
        } else if (valid) {
            finish_pixel(C, P, sample, O, pixel, slab, resolve_two(base, bflags, has_term, term1, false, has_term2, term2));
        }
    }
    }
    __syncthreads();
    if (threadIdx.x == 0) W.q_count[blockIdx.x] = seg_count;
    flush_counters<STATS>(cn, counters);
}

// The end of a queued pixel of the one-shadow-light layout: its PerformShading sum from the
// payload k_shade queued with the shadow ray (base colour, the shadowed light's term, W.pay3:
// the environment light's term after it) and the shadow ray's answer.
DEV void finish_one(const DevCamera& C, const RenderParams& P, int sample, const PassOut& O, const WaveBufs& W,
                    size_t q, int slab, bool occluded) {
    const size_t pq = (W.pay3 ? 3 : 2) * q;
    const float4 b = W.q_pay[pq], t = W.q_pay[pq + 1];
    f3 color;
    if (W.pay3) {
        const float4 t2 = W.q_pay[pq + 2];
        color = resolve_two(mk(b.x, b.y, b.z), __float_as_int(b.w), true, mk(t.x, t.y, t.z), occluded,
                            __float_as_int(t2.w) != 0, mk(t2.x, t2.y, t2.z));
    } else {
        color = resolve_one(mk(b.x, b.y, b.z), __float_as_int(b.w), true, mk(t.x, t.y, t.z), occluded);
    }
    finish_pixel(C, P, sample, O, __float_as_int(t.w), slab, color);
}

// One-shadow-light scenes: CastShadowRay for a queued pixel, then its PerformShading sum and the
// end of the sample pass (what k_resolve does for the general case).
template <bool STATS, int FEAT, bool FAST, bool DEFER = false>
__global__ __launch_bounds__(256, FAST ? RTG_WIDE_WAVES(FEAT) : RTG_TRACE_WAVES(FEAT)) void k_shadow_one(
    const DevScene S, const DevCamera C, const RenderParams P, const int sample0, const WaveBufs W, const PassOut O,
    DevCounters* counters) {
    const int slab = (int)(blockIdx.x / (unsigned)P.slab_tiles);    // the k_shade block's sample slab
    const int k = threadIdx.x;
    const size_t q = (size_t)blockIdx.x * 256 + k;
    Cnt<STATS> cn;
    if (k < W.q_count[blockIdx.x]) {
        bool occluded;
        if constexpr (DEFER) {
            // large leaves queued (k_bigleaf_any): a pending ray is finished by k_shadow_fin_one
            const int st = shadow_state_defer<STATS, FEAT>(S, W, q, W.q_o[q], W.q_d[q], cn);
            W.shadow_state[q] = st;
            occluded = st == SS_OCC;
            if (st == SS_PENDING) {
                flush_counters<STATS>(cn, counters);
                return;
            }
        } else {
            occluded = shadow_occluded<STATS, FEAT, FAST>(S, W, q, W.q_o[q], W.q_d[q], cn);
        }
        finish_one(C, P, sample0 + slab, O, W, q, slab, occluded);
    }
    flush_counters<STATS>(cn, counters);
}

// Pending shadow rays after k_bigleaf_any: occluded by a queued leaf, undecided (the reference
// walk decides), else unoccluded -- then the pixel is finished as k_shadow_one would have.
template <int FEAT>
__global__ __launch_bounds__(256) void k_shadow_fin_one(const DevScene S, const DevCamera C, const RenderParams P,
                                                        const int sample0, const WaveBufs W, const PassOut O) {
    const int slab = (int)(blockIdx.x / (unsigned)P.slab_tiles);
    const int k = threadIdx.x;
    const size_t q = (size_t)blockIdx.x * 256 + k;
    if (blockIdx.x == 0 && k == 0) W.dq_count[2] = 0;   // (k_bigleaf_any, its last reader, is done)
    if (k >= W.q_count[blockIdx.x]) return;
    const int st = W.shadow_state[q];
    if (!(st & SS_PENDING)) return;
    bool occluded = (st & SS_OCC) != 0;
    if (!occluded && (st & SS_UNDECIDED)) {
        const float4 o = W.q_o[q], d = W.q_d[q];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        Cnt<false> cn;
        Hit h;
        occluded = trace<true, false, FEAT>(S, r, 0.f, o.w, d.w, h, cn);
    }
    finish_one(C, P, sample0 + slab, O, W, q, slab, occluded);
}

// The same for the general layout: the answer goes to the light slot's occlusion byte.
template <int FEAT>
__global__ __launch_bounds__(256) void k_shadow_fin(const DevScene S, const WaveBufs W) {
    const int k = blockIdx.y * 256 + threadIdx.x;
    const size_t q = ((size_t)blockIdx.x * W.num_slots) * 256 + k;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) W.dq_count[2] = 0;   // (as k_shadow_fin_one)
    if (k >= W.q_count[blockIdx.x]) return;
    const int st = W.shadow_state[q];
    if (!(st & SS_PENDING)) return;
    bool occluded = (st & SS_OCC) != 0;
    if (!occluded && (st & SS_UNDECIDED)) {
        const float4 o = W.q_o[q], d = W.q_d[q];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        Cnt<false> cn;
        Hit h;
        occluded = trace<true, false, FEAT>(S, r, 0.f, o.w, d.w, h, cn);
    }
    if (occluded) W.occ[W.q_slot[q]] = 1;
}



// Shading / resolve launches (rtg_wave_shade.hip): k_shade<STATS, sk, SH_ONE or SH_GENERAL>
// for the scene's shading variant, and k_resolve.
hipError_t wave_shade(bool stats, int sk, bool one, const DevScene& S, const DevCamera& C, const RenderParams& P,
                      int sample, const WaveBufs& W, const PassOut& O, DevCounters* cnt, hipStream_t st);
void wave_resolve(const DevCamera& C, const RenderParams& P, int sample, const WaveBufs& W, const PassOut& O,
                  hipStream_t st);
// the end of a multi-sample pass: every pixel's slab colours into its accumulation (k_accum)
void wave_accum(const DevCamera& C, const RenderParams& P, int sample, const WaveBufs& W, const PassOut& O,
                hipStream_t st);
bool frame_kernel();
bool defer_leaves();
bool defer_any_leaves();
bool defer_diag();

// One traversal variant's pass sequence (instantiated in rtg_wave_a.hip / rtg_wave_b.hip).
template <bool STATS, int FEAT>
hipError_t launch_wave_t(const DevScene& S, const DevCamera& C, const RenderParams& P, const WaveBufs& W, float* hdr,
                         unsigned char* l, DevCounters* cnt, int sk, hipStream_t st, hipEvent_t* ev, int* layout) {
    const int nshadow = S.num_point + S.num_area + S.num_dir + S.num_spot + S.num_mesh;
    // at most one light with a shadow ray (and at most one environment light after it):
    // k_shade / k_shadow_one finish the pixels (no k_resolve); shading variants for this case
    // only (every other scene takes the general k_shade)
    const bool one = W.q_pay != nullptr && (W.num_slots <= 1 || W.pay3);
    const int scene_sk = sk;
    if (!one) sk = SK_ALL;
    // the any-hit packet walk unless RTG_RENDER_EXACT_SHADOW asks for the reference walk
    // (large-leaf scenes: the split any-hit tree cuts their pole fans into small leaves; with
    // RTG_AHB=ref / exact they keep the cooperative reference walk)
    // large-leaf scenes (production renders): the any-hit walk with their large leaves queued
    // (k_bigleaf_any; RTG_DEFER_ANY=0: the cooperative reference walk)
    const bool defer_any = !STATS && (FEAT & FEAT_BIGLEAF) && W.dq_e && W.shadow_state &&
                           S.anodes && !S.ahb_split && !S.exact_shadow && defer_any_leaves();
    const bool fast = S.anodes != nullptr && (!(FEAT & FEAT_BIGLEAF) || S.ahb_split || defer_any) && !S.exact_shadow;
    // shading fused with the shadow ray: plain shading, the fast any-hit walk
    const bool fused = scene_sk == 0 && fast && !(FEAT & FEAT_BIGLEAF) && nshadow > 0;
    *layout = fused ? (frame_kernel() && !(FEAT == 0 && S.ordered) ? LAYOUT_WAVE_FRAME : LAYOUT_WAVE_FUSED)
                    : (one ? LAYOUT_WAVE_ONE : LAYOUT_WAVE);
    const int s_end = P.sample_begin + P.sample_count;
    // passes of P.slabs consecutive samples (the last one what is left)
    for (int s = P.sample_begin; s < s_end; s += P.slabs) {
        RenderParams Pp = P;
        Pp.slabs = s_end - s < P.slabs ? s_end - s : P.slabs;
        const int nb = Pp.slab_tiles * Pp.slabs;       // blocks of the tile grids
        const int first = s == P.sample_begin, last = s + Pp.slabs == s_end;
        // several slabs: colours per (slab, pixel), k_accum adds them in sample order
        const PassOut O{hdr, l, W.accum, first, last, Pp.slabs > 1 ? W.col : nullptr};
        hipEvent_t* e5 = last ? ev : nullptr;
        hipError_t e;
        if (e5) (void)hipEventRecord(e5[0], st);
        bool ordered = false;
        if constexpr (FEAT == 0) {
            if (S.ordered) {
                hipLaunchKernelGGL((k_primary<STATS, 0, true>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W, cnt);
                ordered = true;
            }
        }
        // the fused layout's sample pass as one launch (k_frame; RTG_FRAME_KERNEL=0: k_primary +
        // k_shade_shadow, A/B): round 5, with both walks lean, 0.311 -> 0.288 ms per headline frame
        // and a part of 1/8 of it 0.0428 -> 0.0403 ms (profiles/r05k_frame_kernel_ab.txt)
        const bool frame = fused && frame_kernel() && !ordered;
        // large-leaf scenes: the camera walk defers large leaves (k_bigleaf, k_hitfix; production
        // renders only -- counting renders keep the cooperative walk and the reference's counts)
        bool deferred = false;
        if constexpr (!STATS && (FEAT & FEAT_BIGLEAF) != 0) {
            if (!ordered && !frame && W.dq_e && S.face_leaf && S.num_objects < 4096 && S.num_faces < (1 << 20)) {
                hipLaunchKernelGGL((k_primary<STATS, FEAT, false, true>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W, cnt);
                hipLaunchKernelGGL((k_bigleaf<FEAT>), dim3(2048), dim3(256), 0, st, S, W);
                hipLaunchKernelGGL((k_hitfix<FEAT>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W,
                                   defer_diag() ? cnt : nullptr);
                // (one unsettled pixel's reference walk per wave, grid-stride: C4 has ~2 000 per
                // sample; 256 or 2 048 blocks per sample measured the same, profiles/r05g_c4_refwalk_ab.txt;
                // round 6: both settled inside k_shade instead -- C3 +0.4 %, C4 -2.4 % (k_shade's
                // registers), profiles/r06j_shade_settle_ab.txt)
                hipLaunchKernelGGL((k_refwalk<FEAT>), dim3(256 * Pp.slabs), dim3(256), 0, st, S, C, Pp, s, W);
                deferred = true;
            }
        }
        if (!ordered && !frame && !deferred)
            hipLaunchKernelGGL((k_primary<STATS, FEAT>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W, cnt);
        if (e5 && !frame) (void)hipEventRecord(e5[1], st);
        if (frame) {
            if constexpr (!(FEAT & FEAT_BIGLEAF)) {
                if (one)
                    hipLaunchKernelGGL((k_shade<STATS, 0, SH_FUSED, FEAT, true, true>), dim3(nb), dim3(256), 0, st, S, C,
                                       Pp, s, W, O, cnt);
                else
                    hipLaunchKernelGGL((k_shade<STATS, 0, SH_FUSED_N, FEAT, true, true>), dim3(nb), dim3(256), 0, st, S,
                                       C, Pp, s, W, O, cnt);
            }
            if (e5) (void)hipEventRecord(e5[1], st);             // LAYOUT_WAVE_FRAME: one stage
        } else if (fused) {
            if constexpr (!(FEAT & FEAT_BIGLEAF)) {
                if (one)
                    hipLaunchKernelGGL((k_shade<STATS, 0, SH_FUSED, FEAT, true>), dim3(nb), dim3(256), 0, st, S, C, Pp,
                                       s, W, O, cnt);
                else
                    hipLaunchKernelGGL((k_shade<STATS, 0, SH_FUSED_N, FEAT, true>), dim3(nb), dim3(256), 0, st, S, C,
                                       Pp, s, W, O, cnt);
            }
            if (e5) (void)hipEventRecord(e5[2], st);
        } else if (one) {
            e = wave_shade(STATS, sk, true, S, C, Pp, s, W, O, cnt, st);
            if (e != hipSuccess) return e;
            if (e5) (void)hipEventRecord(e5[2], st);
            if (nshadow > 0) {
                if (defer_any) {
                    if constexpr (!STATS && (FEAT & FEAT_BIGLEAF)) {
                        hipLaunchKernelGGL((k_shadow_one<STATS, FEAT, true, true>), dim3(nb), dim3(256), 0, st, S, C, Pp,
                                           s, W, O, cnt);
                        hipLaunchKernelGGL((k_bigleaf_any<FEAT>), dim3(2048), dim3(256), 0, st, S, W);
                        hipLaunchKernelGGL((k_shadow_fin_one<FEAT>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W, O);
                    }
                } else if (fast)
                    hipLaunchKernelGGL((k_shadow_one<STATS, FEAT, true>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W, O,
                                       cnt);
                else
                    hipLaunchKernelGGL((k_shadow_one<STATS, FEAT, false>), dim3(nb), dim3(256), 0, st, S, C, Pp, s, W,
                                       O, cnt);
            }
            if (e5) (void)hipEventRecord(e5[3], st);
        } else {
            e = wave_shade(STATS, SK_ALL, false, S, C, Pp, s, W, O, cnt, st);
            if (e != hipSuccess) return e;
            if (e5) (void)hipEventRecord(e5[2], st);
            if (nshadow > 0) {
                const dim3 g(nb, nshadow);
                if (defer_any) {
                    if constexpr (!STATS && (FEAT & FEAT_BIGLEAF)) {
                        hipLaunchKernelGGL((k_shadow<STATS, FEAT, true, true>), g, dim3(256), 0, st, S, W, cnt);
                        hipLaunchKernelGGL((k_bigleaf_any<FEAT>), dim3(2048), dim3(256), 0, st, S, W);
                        hipLaunchKernelGGL((k_shadow_fin<FEAT>), g, dim3(256), 0, st, S, W);
                    }
                } else if (fast) {
                    hipLaunchKernelGGL((k_shadow<STATS, FEAT, true>), g, dim3(256), 0, st, S, W, cnt);
                } else {
                    hipLaunchKernelGGL((k_shadow<STATS, FEAT, false>), g, dim3(256), 0, st, S, W, cnt);
                }
            }
            if (e5) (void)hipEventRecord(e5[3], st);
            wave_resolve(C, Pp, s, W, O, st);
            if (e5) (void)hipEventRecord(e5[4], st);
        }
        if (O.col) wave_accum(C, Pp, s, W, O, st);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int FEAT>
hipError_t launch_wave_f(const DevScene& S, const DevCamera& C, const RenderParams& P, const WaveBufs& W, float* hdr,
                         unsigned char* l, DevCounters* cnt, bool stats, int sk, hipStream_t st, hipEvent_t* ev,
                         int* layout) {
    return stats ? launch_wave_t<true, FEAT>(S, C, P, W, hdr, l, cnt, sk, st, ev, layout)
                 : launch_wave_t<false, FEAT>(S, C, P, W, hdr, l, cnt, sk, st, ev, layout);
}
// traversal variants, split over two translation units (compile time)
#define RTG_WAVE_DECL(F)                                                                                          \
    extern template hipError_t launch_wave_f<F>(const DevScene&, const DevCamera&, const RenderParams&,             \
                                                const WaveBufs&, float*, unsigned char*, DevCounters*, bool, int, \
                                                hipStream_t, hipEvent_t*, int*);
RTG_WAVE_DECL(0)
RTG_WAVE_DECL(FEAT_SPHERE)
RTG_WAVE_DECL(FEAT_BIGLEAF)
RTG_WAVE_DECL(FEAT_SPHERE | FEAT_BIGLEAF)
RTG_WAVE_DECL(FEAT_ALL)
RTG_WAVE_DECL(FEAT_ALL & ~FEAT_BIGLEAF)
#undef RTG_WAVE_DECL

}  // namespace rtg
