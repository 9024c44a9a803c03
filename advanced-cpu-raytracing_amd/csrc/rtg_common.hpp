// Device code shared by the render kernels (rtg_mega.hip, rtg_wave.hip): camera rays,
// threaded BVH traversal, Cramer's-rule triangle and analytic sphere tests, textures,
// the five BRDFs, Shade, direct lighting and shadow rays.
//
// Numerics: this file is compiled with -ffp-contract=off and IEEE div/sqrt, and every
// expression keeps the reference's association and float/double choices, so the
// only differences from the CPU path are the last-ulp results of transcendental
// library calls (powf, acosf, expf, atan2f, double pow/cos).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtg_device.hpp"

// Minimum waves per SIMD the kernels are compiled for (__launch_bounds__'s second argument:
// the register budget is 512 / waves).  The fused kernel at its natural 256 VGPR + AGPRs runs
// one wave per SIMD; two (a few hundred spilled registers) measured 5% faster on C2 and
// 40-60% faster on path tracing, four slower.  The traversal kernels of plain scenes (meshes
// with small leaves, spheres: 57-84 VGPRs) run at eight (+8% on C5); the large-leaf, instance
// and transform variants (88-129 VGPRs) keep their natural allocation -- eight costs C3 20-30%
// -- except the instance ones, at five (+8% on C4).
#ifndef RTG_MEGA_WAVES
#define RTG_MEGA_WAVES 2
#endif
// A fused-kernel build for four waves per SIMD faulted once in round 1 (an out-of-range scratch
// address in k_render<0>): guarded and plain rebuilds of this code did not
// reproduce it and no index of the kernel is out of range, but the cause is not identified, so
// builds above two waves stay experimental and must say so (make EXTRA="-DRTG_MEGA_WAVES=4
// -DRTG_MEGA_WAVES_EXPERIMENTAL=1").
#if RTG_MEGA_WAVES > 2 && !defined(RTG_MEGA_WAVES_EXPERIMENTAL)
#error "RTG_MEGA_WAVES > 2 is experimental (round-1 scratch fault, DESIGN.md §7): add -DRTG_MEGA_WAVES_EXPERIMENTAL=1"
#endif
#ifndef RTG_LEAN_WAVES
#define RTG_LEAN_WAVES 8
#endif
// k_shade (212 VGPRs natural) at three waves: -17% kernel time on the headline; the tree
// pipeline's k_tree_shade at three costs C5 5%
#ifndef RTG_SHADE_WAVES
#define RTG_SHADE_WAVES 3
#endif
#ifndef RTG_TREE_SHADE_WAVES
#define RTG_TREE_SHADE_WAVES 1
#endif
#ifndef RTG_BIGLEAF_LEAN
#define RTG_BIGLEAF_LEAN 0
#endif
// instance scenes' walks (camera and any-hit) at six waves: C4 2 944 -> 3 150 Mrays/s, C3-ton
// 5 450 -> 5 600 (profiles/r05n_pairs_inst6_deferany_ab.txt)
#ifndef RTG_INST_WAVES
#define RTG_INST_WAVES 6
#endif
#define RTG_TRACE_WAVES(FEAT) \
    (((FEAT) & ~(FEAT_SPHERE | (RTG_BIGLEAF_LEAN ? FEAT_BIGLEAF : 0))) \
         ? (((FEAT) & FEAT_INSTANCE) ? RTG_INST_WAVES : 1) : RTG_LEAN_WAVES)

namespace rtg {

#define DEV __device__ __forceinline__

// RTG_GUARD=1 (fault-hunting builds only): every table index taken from a hit record or an
// object, and the fused kernel's frame-stack index, is range-checked; a bad one sets bit
// `code` of S.guard[0] (printed by rtg_scene_destroy) and is clamped so the run goes on.
#ifndef RTG_GUARD
#define RTG_GUARD 0
#endif
#if RTG_GUARD
#define GIDX(S, i, n, code) \
    ([&]() -> int { const int i_ = (i); if (i_ < 0 || i_ >= (n)) { atomicOr((S).guard, 1 << (code)); return 0; } return i_; }())
#else
#define GIDX(S, i, n, code) (i)
#endif

// ---------------------------------------------------------------------------
// helperMath.cpp
// ---------------------------------------------------------------------------
struct f3 { float x, y, z; };
DEV f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
DEV f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
DEV f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
DEV f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
DEV f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
DEV f3 neg(f3 a) { return mk(a.x * -1.0f, a.y * -1.0f, a.z * -1.0f); }
DEV float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DEV float len(f3 a) { return sqrtf((a.x * a.x) + (a.y * a.y) + (a.z * a.z)); }
DEV f3 makeUnit(f3 a) { float l = len(a); return mk(a.x / l, a.y / l, a.z / l); }
DEV float fmax0(float v) { return (0.0f < v) ? v : 0.0f; }          // std::max(0.0f, v)

DEV void onb(f3 r, f3& u, f3& v) {                                     // helperMath.cpp:59-85
    float ax = fabsf(r.x), ay = fabsf(r.y), az = fabsf(r.z);
    f3 rp = r;
    if (ax < ay) { if (ax < az) rp.x = 1.0f; else rp.z = 1.0f; }
    else { if (ay < az) rp.y = 1.0f; else rp.z = 1.0f; }
    u = makeUnit(cross(rp, r));
    v = makeUnit(cross(r, u));
}

#define RT_PI 3.14159265358979323846
DEV double angleBetween(f3 a, f3 b) {                                  // helperMath.cpp:154-157
    float d = dot(a, b);
    float c = (-1.0f < d) ? d : -1.0f;      // std::max(-1.0f, d)
    c = (c < 1.0f) ? c : 1.0f;              // std::min(1.0f, c)
    return (double)acosf(c) * (double)(180.0f / RT_PI);
}
DEV double cosDeg(double a) { return cos(a * (RT_PI / 180.0f)); }      // helperMath.cpp:158-161

// matrix.hpp:56-81 (double accumulation, w column included)
DEV f3 xform(const double* m, f3 v, float w) {
    return mk((float)(m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3] * w),
              (float)(m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7] * w),
              (float)(m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11] * w));
}

// counter-based RNG (replaces the shared mt19937 streams; keyed by pixel, sample and
// ray-tree node so results do not depend on thread / GPU count)
DEV uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
DEV float rnd(uint64_t key, uint32_t purpose, uint32_t idx) {
    uint64_t h = mix64(key ^ mix64(((uint64_t)purpose << 32) | idx));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}
DEV uint64_t child_key(uint64_t key, int slot) { return mix64(key + 0x632BE59BD9B4E019ULL * (uint64_t)(slot + 1)); }
DEV uint64_t root_key(uint64_t seed, int pixel, int sample) {
    return mix64(mix64(seed ^ 0xD1B54A32D192ED03ULL) ^ ((uint64_t)(uint32_t)pixel * 0x9E3779B97F4A7C15ULL) ^
                 ((uint64_t)(uint32_t)sample << 1));
}
// double draw (std::uniform_real_distribution<> of MeshLight::getSample, meshLight.h:31-36)
DEV double rndd(uint64_t key, uint32_t purpose, uint32_t idx) {
    uint64_t h = mix64(key ^ mix64(((uint64_t)purpose << 32) | idx));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
enum { RP_MOTION = 1, RP_DOF = 2, RP_JITTER = 3, RP_AREA = 4, RP_ENV = 5, RP_ROUGH_REFL = 6, RP_ROUGH_REFR = 7,
       RP_GI = 8, RP_MESHLIGHT = 9 };

// ---------------------------------------------------------------------------
// Counters
// ---------------------------------------------------------------------------
template <bool STATS> struct Cnt {
    template <bool ANY> DEV void node() {}
    template <bool ANY> DEV void tri() {}
    template <bool ANY> DEV void tri_n(uint32_t) {}
    DEV void sph() {} DEV void obj() {}
    DEV void cam() {} DEV void sec() {} DEV void shd() {}
    DEV void wnode() {}
    DEV void fallback() {}
    DEV void ewnode() {}
    DEV void efallback() {}
};
template <> struct Cnt<true> {
    uint32_t nodes = 0, tris = 0, sphs = 0, objs = 0, cams = 0, secs = 0, shds = 0, snodes = 0, stris = 0, wnodes = 0,
             fallbacks = 0, ewnodes = 0, efallbacks = 0;
    DEV void wnode() { ++wnodes; }
    DEV void ewnode() { ++ewnodes; }
    DEV void efallback() { ++efallbacks; }
    DEV void fallback() { ++fallbacks; }
    template <bool ANY> DEV void node() { if (ANY) ++snodes; else ++nodes; }
    template <bool ANY> DEV void tri() { if (ANY) ++stris; else ++tris; }
    template <bool ANY> DEV void tri_n(uint32_t n) { if (ANY) stris += n; else tris += n; }
    DEV void sph() { ++sphs; } DEV void obj() { ++objs; }
    DEV void cam() { ++cams; } DEV void sec() { ++secs; } DEV void shd() { ++shds; }
};

// ---------------------------------------------------------------------------
// Geometry
// ---------------------------------------------------------------------------
struct Ray {
    f3 o, d;
};

// BoundingBox::doesIntersectWith (shape.hpp:78-100): true divisions, x-slab by
// comparison, y/z by fmin/fmax (NaN-ignoring), accept iff tmax>0 && tmax>=tmin && tmin<minT.
DEV bool box_hit(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, const Ray& r, float minT) {
    float tx1 = (mnx - r.o.x) / r.d.x;
    float tx2 = (mxx - r.o.x) / r.d.x;
    float tmin = tx1, tmax = tx2;
    if (tx1 > tx2) { tmin = tx2; tmax = tx1; }
    float ty1 = (mny - r.o.y) / r.d.y;
    float ty2 = (mxy - r.o.y) / r.d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (mnz - r.o.z) / r.d.z;
    float tz2 = (mxz - r.o.z) / r.d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    return tmax > 0 && tmax >= tmin && tmin < minT;
}

// The same predicate at a fraction of the cost.  Each slab distance (m - o) / d is
// computed as (m - o) * rcp(d): with v_rcp_f32 (<= 1 ulp) and two roundings the result is
// within 2^-22 |t| of the correctly rounded quotient, and min/max keep that bound.  Each
// of the three decisions is taken from the fast values only when they are farther than
// 4x that bound from the decision boundary; otherwise the exact division test above
// decides.  Hence the accepted set of boxes -- and every counter -- is identical.
// `fast` is false when a direction component is 0, subnormal or huge (rcp inexact /
// special values): those rays always take the exact test.
struct RayRcp {
    float ix, iy, iz;
    bool fast;
};
DEV RayRcp ray_rcp(const Ray& r) {
    RayRcp q;
    q.ix = __builtin_amdgcn_rcpf(r.d.x);
    q.iy = __builtin_amdgcn_rcpf(r.d.y);
    q.iz = __builtin_amdgcn_rcpf(r.d.z);
    const float lo = 0x1p-60f, hi = 0x1p60f;
    const float ax = fabsf(r.d.x), ay = fabsf(r.d.y), az = fabsf(r.d.z);
    q.fast = ax >= lo && ax <= hi && ay >= lo && ay <= hi && az >= lo && az <= hi;
    return q;
}
// UNI: the exact fallback as a wave-uniform branch (wave packets: every lane tests the same box)
// `on` (UNI only): lanes whose result is used -- the others do not vote for the fallback
template <bool UNI = false>
DEV bool box_hit_fast(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, const Ray& r,
                      const RayRcp& q, float minT, bool on = true) {
    // branch-free: every condition is evaluated (bitwise &, no short circuit), so the
    // common path is straight-line code with one rarely taken branch to the exact test
    const float tx1 = (mnx - r.o.x) * q.ix, tx2 = (mxx - r.o.x) * q.ix;
    const float ty1 = (mny - r.o.y) * q.iy, ty2 = (mxy - r.o.y) * q.iy;
    const float tz1 = (mnz - r.o.z) * q.iz, tz2 = (mxz - r.o.z) * q.iz;
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    const float atmin = fabsf(tmin), atmax = fabsf(tmax);
    const float slack = fmaf(0x1p-20f, atmin + atmax, 1e-30f);   // (fma: one rounding, tighter)
    // all three decisions clear of their boundaries.  NaN fails every comparison and an
    // infinite tmin or tmax makes the slack infinite, so both take the exact test; with both
    // finite, minT = inf passes the last test (tmax >= tmin decided, tmin < inf exact)
    // (round 4: dropping the separate range and minT = inf terms took the headline k_primary
    // 0.2052 -> 0.1915 ms, profiles/r04y_slab_lean_ab.txt)
    const bool sure = (int)q.fast & (atmax >= 1e-30f) & (fabsf(tmax - tmin) > slack) &
                      (fabsf(tmin - minT) > fmaf(0x1p-20f, atmin, 1e-30f));
    bool hit = (tmax > 0) & (tmax >= tmin) & (tmin < minT);
    if constexpr (UNI) {
        if (__builtin_expect(__ballot(on & !sure) != 0, 0)) {
            if (on & !sure) hit = box_hit(mnx, mny, mnz, mxx, mxy, mxz, r, minT);
        }
        return hit;
    }
    if (__builtin_expect(!sure, 0)) return box_hit(mnx, mny, mnz, mxx, mxy, mxz, r, minT);
    return hit;
}

// NaN-propagating minimum of three (IEEE 754-2019 minimum; v_minimum3_f32 on gfx950):
// vmin3(a, b, c) > 0 is exactly (a > 0) & (b > 0) & (c > 0), NaN included
DEV float vmin3(float a, float b, float c) {
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}

// box_hit_fast<true> for the camera packet walk with the lane's participation folded in, each
// predicate one comparison.  act = rel > 0 (rel = i + 1 - resume: the lane's own walk reaches
// this node).  When sure, the three decisions are clear of their boundaries, so each is the
// sign of one exactly-signed quantity -- tmax, tmax - tmin (nonzero: |.| > slack) and minT - tmin
// (a rounded difference has the sign of the exact one) -- and the conjunction is min(...) > 0;
// `sure` is min(|tmax - tmin| - slack, |tmin - minT| - slack', |tmax| - 1e-30) > 0 (each a rounded
// difference: exact sign; the last a hair stricter than >=), slack0 = inf when the ray's
// reciprocals are not exact enough (q.fast).  A NaN term leaves the lane unsure; a sure lane has
// no NaN among tmax, d1, d2.  Unsure lanes inside their walk take the exact test (uniform branch).
// Returns a value whose sign is the answer (> 0: the lane takes part and the box passes), so a
// caller's ballot of `> 0` is one comparison; actf > 0: the lane takes part.
// INT: actf is an integer (rel), so `act & !sure` is one comparison, !(max(su, 0.5 - actf) > 0).
// box_pass_t takes the six slab distances (m - o) * rcp; the box for the exact fallback.
template <bool INT = false>
DEV float box_pass_t(float tx1, float tx2, float ty1, float ty2, float tz1, float tz2, float mnx, float mny, float mnz,
                     float mxx, float mxy, float mxz, const Ray& r, float minT, float actf, float slack0) {
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    const float atmin = fabsf(tmin), atmax = fabsf(tmax);
    const float d1 = tmax - tmin, d2 = minT - tmin;
    // (NaN-propagating minimum, v_minimum3_f32: any NaN term -- an infinite box face, inf - inf
    // -- leaves the lane unsure)
    const float su = vmin3(fabsf(d1) - fmaf(0x1p-20f, atmin + atmax, slack0), fabsf(d2) - fmaf(0x1p-20f, atmin, slack0),
                           atmax - 1e-30f);
    float pv = __builtin_elementwise_minimum(fminf(fminf(tmax, d1), d2), actf);   // (a NaN actf: not taking part)
    const bool unsure = INT ? !(fmaxf(su, 0.5f - actf) > 0.0f) : (actf > 0.0f) & !(su > 0.0f);
    if (__builtin_expect(__ballot(unsure) != 0, 0)) {
        if (unsure) pv = box_hit(mnx, mny, mnz, mxx, mxy, mxz, r, minT) ? 1.0f : -1.0f;
    }
    return pv;
}
template <bool INT = false>
DEV float box_pass_v(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, const Ray& r, const RayRcp& q,
                     float minT, float actf, float slack0) {
    const float tx1 = (mnx - r.o.x) * q.ix, tx2 = (mxx - r.o.x) * q.ix;
    const float ty1 = (mny - r.o.y) * q.iy, ty2 = (mxy - r.o.y) * q.iy;
    const float tz1 = (mnz - r.o.z) * q.iz, tz2 = (mxz - r.o.z) * q.iz;
    return box_pass_t<INT>(tx1, tx2, ty1, ty2, tz1, tz2, mnx, mny, mnz, mxx, mxy, mxz, r, minT, actf, slack0);
}
DEV bool box_pass_pk(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, const Ray& r, const RayRcp& q,
                     float minT, int rel, float slack0) {
    // rel = i + 1 - resume > 0: the lane's walk reaches the node (as a float: sign exact)
    // (compared after the merge: the caller's ballot of it is then that comparison's mask)
    return box_pass_v<true>(mnx, mny, mnz, mxx, mxy, mxz, r, q, minT, (float)rel, slack0) > 0.0f;
}

// determinant (helperMath.cpp:132-138)
DEV float det3(float m00, float m01, float m02, float m10, float m11, float m12, float m20, float m21, float m22) {
    float first = m00 * (m11 * m22 - m12 * m21);
    float second = m10 * (m02 * m21 - m01 * m22);
    float third = m20 * (m01 * m12 - m11 * m02);
    return first + second + third;
}

// Mesh::IntersectFace (mesh.cpp:201-240): Cramer's rule, early outs in the same order.
// Returns t (or a value failing 0<t<minT) and beta/gamma.
DEV bool tri_test(const DevScene& S, int f, const Ray& r, float minT, float& tout, float* bg = nullptr) {
    const float4 A = S.tris[3 * f], E1 = S.tris[3 * f + 1], E2 = S.tris[3 * f + 2];
    const float dx = r.d.x, dy = r.d.y, dz = r.d.z;
    float detA = det3(E1.x, E2.x, dx, E1.y, E2.y, dy, E1.z, E2.z, dz);
    if (detA == 0) return false;
    const float sx = A.x - r.o.x, sy = A.y - r.o.y, sz = A.z - r.o.z;
    float beta = det3(sx, E2.x, dx, sy, E2.y, dy, sz, E2.z, dz) / detA;
    if (beta < 0) return false;
    float gama = det3(E1.x, sx, dx, E1.y, sy, dy, E1.z, sz, dz) / detA;
    if (gama < 0 || gama + beta > 1) return false;
    float t = det3(E1.x, E2.x, sx, E1.y, E2.y, sy, E1.z, E2.z, sz) / detA;
    if (bg) { bg[0] = beta; bg[1] = gama; }
    tout = t;
    return t > 0.0f && t < minT;
}

// Mesh::IntersectFace on a face record (any-hit tree entries: a copy of S.tris[3f..3f+2]).
DEV bool tri_test_rec(const float4* R, const Ray& r, float minT, float& tout) {
    const float4 A = R[0], E1 = R[1], E2 = R[2];
    const float dx = r.d.x, dy = r.d.y, dz = r.d.z;
    float detA = det3(E1.x, E2.x, dx, E1.y, E2.y, dy, E1.z, E2.z, dz);
    if (detA == 0) return false;
    const float sx = A.x - r.o.x, sy = A.y - r.o.y, sz = A.z - r.o.z;
    float beta = det3(sx, E2.x, dx, sy, E2.y, dy, sz, E2.z, dz) / detA;
    if (beta < 0) return false;
    float gama = det3(E1.x, sx, dx, E1.y, sy, dy, E1.z, sz, dz) / detA;
    if (gama < 0 || gama + beta > 1) return false;
    float t = det3(E1.x, E2.x, sx, E1.y, E2.y, sy, E1.z, E2.z, sz) / detA;
    tout = t;
    return t > 0.0f && t < minT;
}

// tri_test for traversal: beta and gamma from one reciprocal of detA, with the decisions
// beta<0, gamma<0 (exact signs unless a quotient underflows) and beta+gamma>1 (taken
// only when clear of 1 by 4x the error bound) identical to the division form; t itself
// is the correctly rounded quotient.  Falls back to tri_test when unsure.
DEV bool tri_test_fast(const DevScene& S, int f, const Ray& r, float minT, float& tout) {
    const float4 A = S.tris[3 * f], E1 = S.tris[3 * f + 1], E2 = S.tris[3 * f + 2];
    const float dx = r.d.x, dy = r.d.y, dz = r.d.z;
    const float detA = det3(E1.x, E2.x, dx, E1.y, E2.y, dy, E1.z, E2.z, dz);
    if (detA == 0) return false;
    const float ad = fabsf(detA);
    if (ad >= 0x1p-100f && ad <= 0x1p100f) {
        const float rd = __builtin_amdgcn_rcpf(detA);
        const float sx = A.x - r.o.x, sy = A.y - r.o.y, sz = A.z - r.o.z;
        const float nb = det3(sx, E2.x, dx, sy, E2.y, dy, sz, E2.z, dz);
        const float beta = nb * rd;
        const bool bsure = nb == 0.0f || fabsf(beta) > 1e-30f;
        if (bsure) {
            if (beta < 0) return false;
            const float ng = det3(E1.x, sx, dx, E1.y, sy, dy, E1.z, sz, dz);
            const float gama = ng * rd;
            const bool gsure = ng == 0.0f || fabsf(gama) > 1e-30f;
            if (gsure) {
                if (gama < 0) return false;
                const float sum = gama + beta;
                if (fabsf(sum - 1.0f) > fmaf(0x1p-19f, sum, 0x1p-22f)) {
                    if (sum > 1) return false;
                    float t = det3(E1.x, E2.x, sx, E1.y, E2.y, sy, E1.z, E2.z, sz) / detA;
                    tout = t;
                    return t > 0.0f && t < minT;
                }
            }
        }
    }
    return tri_test(S, f, r, minT, tout);
}
// The same on a face record (any-hit tree entries).
DEV bool tri_test_fast_rec(const float4* R, const Ray& r, float minT, float& tout) {
    const float4 A = R[0], E1 = R[1], E2 = R[2];
    const float dx = r.d.x, dy = r.d.y, dz = r.d.z;
    const float detA = det3(E1.x, E2.x, dx, E1.y, E2.y, dy, E1.z, E2.z, dz);
    if (detA == 0) return false;
    const float ad = fabsf(detA);
    if (ad >= 0x1p-100f && ad <= 0x1p100f) {
        const float rd = __builtin_amdgcn_rcpf(detA);
        const float sx = A.x - r.o.x, sy = A.y - r.o.y, sz = A.z - r.o.z;
        const float nb = det3(sx, E2.x, dx, sy, E2.y, dy, sz, E2.z, dz);
        const float beta = nb * rd;
        const bool bsure = nb == 0.0f || fabsf(beta) > 1e-30f;
        if (bsure) {
            if (beta < 0) return false;
            const float ng = det3(E1.x, sx, dx, E1.y, sy, dy, E1.z, sz, dz);
            const float gama = ng * rd;
            const bool gsure = ng == 0.0f || fabsf(gama) > 1e-30f;
            if (gsure) {
                if (gama < 0) return false;
                const float sum = gama + beta;
                if (fabsf(sum - 1.0f) > fmaf(0x1p-19f, sum, 0x1p-22f)) {
                    if (sum > 1) return false;
                    float t = det3(E1.x, E2.x, sx, E1.y, E2.y, sy, E1.z, E2.z, sz) / detA;
                    tout = t;
                    return t > 0.0f && t < minT;
                }
            }
        }
    }
    return tri_test_rec(R, r, minT, tout);
}

// tri_test_fast_rec with selects (wave packets, where every lane tests the same face, and the
// per-lane walk under RTG_SEQ_SEL): the same decisions -- the early outs become lane masks,
// and the two costly parts (the t division, the exact fallback) wave-uniform branches taken
// when some lane needs them.
// `on`: lanes whose result is used (the others neither take the division nor the fallback)
DEV bool tri_test_sel(const float4* R, const Ray& r, float limit, float& tout, bool on = true) {
    const float4 A = R[0], E1 = R[1], E2 = R[2];
    const float dx = r.d.x, dy = r.d.y, dz = r.d.z;
    const float detA = det3(E1.x, E2.x, dx, E1.y, E2.y, dy, E1.z, E2.z, dz);
    const float ad = fabsf(detA);
    const float rd = __builtin_amdgcn_rcpf(detA);
    const float sx = A.x - r.o.x, sy = A.y - r.o.y, sz = A.z - r.o.z;
    const float nb = det3(sx, E2.x, dx, sy, E2.y, dy, sz, E2.z, dz);
    const float ng = det3(E1.x, sx, dx, E1.y, sy, dy, E1.z, sz, dz);
    const float beta = nb * rd, gama = ng * rd, sum = gama + beta;
    const bool zero = detA == 0;
    const bool range = (ad >= 0x1p-100f) & (ad <= 0x1p100f);
    const bool bsure = (nb == 0.0f) | (fabsf(beta) > 1e-30f);
    const bool gsure = (ng == 0.0f) | (fabsf(gama) > 1e-30f);
    const bool ssure = fabsf(sum - 1.0f) > fmaf(0x1p-19f, sum, 0x1p-22f);
    // tri_test_fast_rec's decision tree: false / t test / exact fallback
    const bool b_out = range & bsure & (beta < 0);
    const bool g_out = range & bsure & !(beta < 0) & gsure & (gama < 0);
    const bool s_ok = range & bsure & !(beta < 0) & gsure & !(gama < 0) & ssure;
    const bool no = zero | b_out | g_out | (s_ok & (sum > 1)) | !on;
    const bool tt = on & !zero & s_ok & !(sum > 1);
    bool hit = false;
    if (__ballot(tt)) {
        const float t = det3(E1.x, E2.x, sx, E1.y, E2.y, sy, E1.z, E2.z, sz) / detA;
        tout = t;
        hit = tt & (t > 0.0f) & (t < limit);
    }
    const bool unsure = !no & !tt;
    if (__builtin_expect(__ballot(unsure) != 0, 0)) {
        if (unsure) hit = tri_test_rec(R, r, limit, tout);
    }
    return hit;
}

// tri_test_sel with every decision a single comparison of a value (the packet walks' face
// tests; lanes with onf > 0 take part).  Returns a value > 0 exactly when IntersectFace
// accepts the face with 0 < t < limit (t in tout).  Sure candidates: |detA| in range (strict),
// beta and gama above 1e-30 and 1 - sum above the bound of tri_test_fast_rec (each a rounded
// difference, so its sign is the comparison's); sure rejections: detA == 0, or in range and
// beta or gama below -1e-30 or sum - 1 above the bound (any one decides, in whatever order the
// reference tests them: each makes IntersectFace return false).  Everything else -- also the
// exact zeros nb == 0 / ng == 0 that tri_test_fast_rec takes as sure -- takes the exact test
// (uniform branch).  AND is the NaN-propagating minimum, OR the NaN-dropping max.
DEV float tri_test_pk(const float4* R, const Ray& r, float limit, float& tout, float onf) {
    const float4 A = R[0], E1 = R[1], E2 = R[2];
    const float dx = r.d.x, dy = r.d.y, dz = r.d.z;
    const float detA = det3(E1.x, E2.x, dx, E1.y, E2.y, dy, E1.z, E2.z, dz);
    const float ad = fabsf(detA);
    const float rd = __builtin_amdgcn_rcpf(detA);
    const float sx = A.x - r.o.x, sy = A.y - r.o.y, sz = A.z - r.o.z;
    const float nb = det3(sx, E2.x, dx, sy, E2.y, dy, sz, E2.z, dz);
    const float ng = det3(E1.x, sx, dx, E1.y, sy, dy, E1.z, sz, dz);
    const float beta = nb * rd, gama = ng * rd, sum = gama + beta;
    const float sslack = fmaf(0x1p-19f, sum, 0x1p-22f);
    const float rng = __builtin_elementwise_minimum(ad - 0x1p-100f, 0x1p100f - ad);
    const float ttv = __builtin_elementwise_minimum(vmin3(beta - 1e-30f, gama - 1e-30f, (1.0f - sum) - sslack),
                                                    __builtin_elementwise_minimum(rng, onf));
    const float rjv = __builtin_elementwise_minimum(fmaxf(fmaxf(-1e-30f - beta, -1e-30f - gama), (sum - 1.0f) - sslack),
                                                    rng);
    float hv = -1.0f;
    if (__ballot(ttv > 0.0f)) {
        const float t = det3(E1.x, E2.x, sx, E1.y, E2.y, sy, E1.z, E2.z, sz) / detA;
        tout = t;
        hv = vmin3(ttv, t, limit - t);               // 0 < t < limit (rounded difference: exact sign)
    }
    const bool unsure = (onf > 0.0f) & !(ttv > 0.0f) & !(rjv > 0.0f) & (detA != 0.0f);
    if (__builtin_expect(__ballot(unsure) != 0, 0)) {
        if (unsure) hv = tri_test_rec(R, r, limit, tout) ? 1.0f : -1.0f;
    }
    return hv;
}

// Wave-uniform records through the scalar cache (the compiler keeps vector loads here: the
// kernels store to global memory, so it cannot prove the records unclobbered).  Read-only
// scene data, written by copies before the launch.
typedef int rtg_s16 __attribute__((ext_vector_type(16)));
typedef int rtg_s8 __attribute__((ext_vector_type(8)));
typedef int rtg_s4 __attribute__((ext_vector_type(4)));
DEV const void* uniform_ptr(const void* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const void*)(((uint64_t)hi << 32) | lo);
}
DEV void sload_wnode(const WNode* p, rtg_s16& a, rtg_s16& b) {   // 128 B
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(uniform_ptr(p)) : "memory");
}
DEV void sload_rec(const float4* p, rtg_s8& a, rtg_s4& b) {      // 48 B: a face record
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x20\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(uniform_ptr(p)) : "memory");
}
DEV void sload_node(const float4* p, rtg_s8& a) {                // 32 B: a reference BVH node
    asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(a) : "s"(uniform_ptr(p)) : "memory");
}
DEV float4 f4(int x, int y, int z, int w) {
    return make_float4(__int_as_float(x), __int_as_float(y), __int_as_float(z), __int_as_float(w));
}
// 64-bit lexicographic (t, face) key of a candidate hit; t > 0, so the float bits order
// like the values.  Non-candidates: ~0.
DEV uint64_t hit_key(float t, int f) { return ((uint64_t)__float_as_uint(t) << 32) | (uint32_t)f; }

// Minimum of `key` over the lanes set in `em` (the wave's active lanes).  A butterfly
// needs every lane; with a partial exec mask (image-edge tiles, rays that skip an
// instance, the fused kernel's ray trees) the active lanes' keys are read one by one.
DEV uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
DEV uint64_t wave_min_key(uint64_t key, uint64_t em) {
    if (em == ~0ull) {
        const int lane = threadIdx.x & 63;
        for (int m = 1; m < 64; m <<= 1) {
            const uint64_t other = shfl64(key, lane ^ m);
            if (other < key) key = other;
        }
        return key;
    }
    uint64_t acc = ~0ull;
    while (em) {
        const int l = __ffsll((long long)em) - 1;
        em &= em - 1;
        const uint64_t v = shfl64(key, l);
        if (v < acc) acc = v;
    }
    return acc;
}

// Sequential form: each lane tests its leaves' faces in order inside the walk (scenes
// whose leaves are all small: the lean kernels).
// (Loading node i + 1 -- where a passing inner node descends -- before node i is tested measured
// slower too: C5 1 712 -> 1 205 Mrays/s at eight waves (spills), 1 435 at seven (1 630 without
// the prefetch), C2 12 700 -> 12 100; the walks' memory traffic, not the chain's latency alone,
// bounds them (profiles/r05r_seq_prefetch_ab.txt).)
// (A "while-while" form -- an inner loop over boxes until the lane stands on a passing leaf,
// the faces after it, Aila & Laine HPG 2009 -- measured slower: k_primary 0.238 -> 0.309 ms,
// C5 1471 -> 954 Mrays/s; profiles/r03l_*.  The lanes that reach a leaf early idle in the box
// loop, and every lane pays the loop's exit bookkeeping per node.)
// the per-lane walk's face test with selects (tri_test_sel) and the slab test's exact fallback
// as a wave-uniform branch (1: k_primary 0.238 -> 0.228 ms, C5 1488 -> 1584 Mrays/s,
// profiles/r03seq_ab.txt) or with per-lane early outs and a divergent fallback (0).  Kernels
// with the cooperative large-leaf walk keep 0 (C3-ton's k_shadow 0.711 -> 0.774 ms with 1)
#ifndef RTG_SEQ_SEL
#define RTG_SEQ_SEL 1
#endif
template <bool ANY, bool STATS, bool SEL = RTG_SEQ_SEL != 0>
DEV bool walk_bvh_seq(const DevScene& S, int i, const int end, const Ray& r, float& minT, int& hitFace, float limit,
                      Cnt<STATS>& c) {
    bool hit = false;
    const RayRcp q = ray_rcp(r);
    while (i < end) {
        const float4 a = S.nodes[2 * i];
        const float4 b = S.nodes[2 * i + 1];
        c.template node<ANY>();
        const int skip = __float_as_int(b.z);
        if (box_hit_fast<SEL>(a.x, a.y, a.z, a.w, b.x, b.y, r, q, minT)) {
            const int leaf = __float_as_int(b.w);
            if (leaf >= 0) {
                int first = leaf >> 8, cnt = leaf & 255;
                if (leaf == LEAF_EXT) {
                    const int2 e = S.node_ext[i];
                    first = e.x;
                    cnt = e.y;
                }
                for (int f = first; f < first + cnt; ++f) {
                    c.template tri<ANY>();
                    float t;
                    if (SEL ? tri_test_sel(S.tris + 3 * f, r, minT, t) : tri_test_fast(S, f, r, minT, t)) {
                        minT = t;
                        hitFace = f;
                        hit = true;
                        if (ANY && t < limit) return true;
                    }
                }
                i = skip;
            } else {
                i = i + 1;
            }
        } else {
            i = skip;
        }
    }
    return hit;
}

// Conservative slab test: accepts every box the exact test (box_hit) accepts at minT.  The
// fast slab distances (m - o) * rcp(d) are within 2^-22 |t| of the exact quotients (RayRcp,
// q.fast), so exact tmax > 0, tmax >= tmin, tmin < minT imply the tests below on the fast
// values (minTc = minT (1 + 2^-21); the 1e-30 terms cover subnormal products).  (An fma form
// m * rcp - o * rcp saves six instructions but its error scales with |o * rcp|, which loosens
// the test badly for rays with a small direction component: measured 2x slower.)

struct SlabRay {
    f3 o;
    float ix, iy, iz;
};
DEV SlabRay slab_ray(const Ray& r, const RayRcp& q) {
    SlabRay s;
    s.o = r.o;
    s.ix = q.ix; s.iy = q.iy; s.iz = q.iz;
    return s;
}
DEV bool slab_cons(float lx, float ly, float lz, float hx, float hy, float hz, const SlabRay& s, float minTc,
                   float& tnear) {
    const float tx1 = (lx - s.o.x) * s.ix, tx2 = (hx - s.o.x) * s.ix;
    const float ty1 = (ly - s.o.y) * s.iy, ty2 = (hy - s.o.y) * s.iy;
    const float tz1 = (lz - s.o.z) * s.iz, tz2 = (hz - s.o.z) * s.iz;
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    tnear = tmin;
    return (tmax > -1e-30f) & (tmax >= fmaf(tmin, 1.0f - 0x1p-21f, -1e-30f)) & (tmin < minTc);
}

// One step's large leaves, tested by the whole wave at once.  Every lane that reached a
// large leaf in this step (`coop`) posts an event -- its ray, minT and leaf -- to the wave's
// table in LDS; the (event, face) pairs of all events are dealt over the wave's lanes, and
// each candidate hit lowers its event's (t, face) key with an LDS 64-bit atomic min.  The
// result per event is the minimum over the leaf's faces with t < minT -- what the lane's
// own sequential loop would keep -- with no per-event reduction chain, and the faces'
// loads independent of each other.  Returns the calling lane's key (~0: none).
// Block size 256 (four waves, one table each), the size of every traversal kernel.
struct CoopEvent {
    float ox, oy, oz, dx, dy, dz, minT;
    int first, cnt, start;
    unsigned long long best;
};
DEV void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
DEV uint64_t coop_leaf_tests(const DevScene& S, uint64_t coop, const Ray& r, float minT, int first, int cnt) {
    __shared__ CoopEvent table[4][64];
    CoopEvent* E = table[threadIdx.x >> 6];
    const uint64_t em = __ballot(1);
    const int lane = threadIdx.x & 63;
    const int nact = __popcll(em);
    const int rank = __popcll(em & ((1ull << lane) - 1ull));
    const int ne = __popcll(coop);
    const int slot = cnt > 0 ? __popcll(coop & ((1ull << lane) - 1ull)) : -1;
    if (slot >= 0) {
        CoopEvent& e = E[slot];
        e.ox = r.o.x; e.oy = r.o.y; e.oz = r.o.z;
        e.dx = r.d.x; e.dy = r.d.y; e.dz = r.d.z;
        e.minT = minT;
        e.first = first;
        e.cnt = cnt;
        e.best = ~0ull;
    }
    wave_lds_sync();
    int total = 0, start = 0;
    for (int k = 0; k < ne; ++k) {
        if (k == slot) start = total;
        total += E[k].cnt;
    }
    if (slot >= 0) E[slot].start = start;
    wave_lds_sync();
    for (int w = rank; w < total; w += nact) {
        int lo = 0, hi = ne - 1;                        // last event with start <= w
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (E[mid].start <= w) lo = mid;
            else hi = mid - 1;
        }
        const CoopEvent& e = E[lo];
        Ray lr;
        lr.o = mk(e.ox, e.oy, e.oz);
        lr.d = mk(e.dx, e.dy, e.dz);
        const int f = e.first + (w - e.start);
        float t;
        if (tri_test_fast(S, f, lr, e.minT, t)) atomicMin(&E[lo].best, (unsigned long long)hit_key(t, f));
    }
    wave_lds_sync();
    const uint64_t mine = slot >= 0 ? (uint64_t)E[slot].best : ~0ull;
    wave_lds_sync();                                    // the table is rewritten next step
    return mine;
}

// BVH::IntersectBVH (bvh.cpp:5-30) as a stackless pre-order walk (rtg_device.hpp).
// ANY: stop at the first accepted face with t < limit (CastShadowRay semantics).
//
// Leaves of up to kCoopLeaf faces are tested by their lane in order.  Larger leaves
// (the reference's midpoint split keeps faces with equal centroid coordinates
// together, e.g. fans around a mesh pole, in leaves of hundreds of faces) are tested
// cooperatively: the walk loop runs while any lane of the wave is active, and every
// lane that reached such a leaf in this step has it tested by all active lanes of the
// wave in parallel, followed by a (t, face) minimum reduction.  That is exactly the
// sequential result: IntersectFace's acceptance is t < minT with minT shrinking over
// the leaf, so the survivor is the smallest t -- the first face among equal t -- of the
// faces with t < minT at leaf entry; for ANY, "some face with t < min(minT, limit)".
template <bool ANY, bool STATS, bool COOP>
DEV bool walk_bvh(const DevScene& S, int i, const int end, const Ray& r, float& minT, int& hitFace, float limit,
                  Cnt<STATS>& c) {
    if constexpr (!COOP) return walk_bvh_seq<ANY, STATS>(S, i, end, r, minT, hitFace, limit, c);
    // general kernels (the fused one) on scenes without large leaves: the plain walk, without
    // the wave-uniform loop and its per-step ballots (a uniform branch)
    if (!S.coop) return walk_bvh_seq<ANY, STATS, false>(S, i, end, r, minT, hitFace, limit, c);
    bool hit = false;
    const RayRcp q = ray_rcp(r);
    bool active = i < end;
    while (__ballot(active)) {
        int coopFirst = 0, coopCnt = 0;
        if (active) {
            const float4 a = S.nodes[2 * i];
            const float4 b = S.nodes[2 * i + 1];
            c.template node<ANY>();
            const int skip = __float_as_int(b.z);
            if (box_hit_fast(a.x, a.y, a.z, a.w, b.x, b.y, r, q, minT)) {
                const int leaf = __float_as_int(b.w);
                if (leaf >= 0) {
                    int first = leaf >> 8, cnt = leaf & 255;
                    if (leaf == LEAF_EXT) {
                        const int2 e = S.node_ext[i];
                        first = e.x;
                        cnt = e.y;
                    }
                    if (cnt > kCoopLeaf) {
                        coopFirst = first;
                        coopCnt = cnt;
                    } else {
                        for (int f = first; f < first + cnt; ++f) {
                            c.template tri<ANY>();
                            float t;
                            if (tri_test_fast(S, f, r, minT, t)) {
                                minT = t;
                                hitFace = f;
                                hit = true;
                                if (ANY && t < limit) {
                                    active = false;
                                    break;
                                }
                            }
                        }
                    }
                    i = skip;
                } else {
                    i = i + 1;
                }
            } else {
                i = skip;
            }
            if (i >= end) active = false;
        }
        const uint64_t coop = __ballot(coopCnt > 0);
        if (coop) {
            const uint64_t best = coop_leaf_tests(S, coop, r, minT, coopFirst, coopCnt);
            if (coopCnt > 0) {
                // counted as the whole leaf: the wave tests every face of it, also for any-hit
                // rays, where the sequential walk stops at the first accepted face (so C3/C4
                // shadow tri_tests depend on RTG_COOP_LEAF; images do not)
                c.template tri_n<ANY>((uint32_t)coopCnt);
                if (best != ~0ull) {
                    minT = __uint_as_float((uint32_t)(best >> 32));
                    hitFace = (int)(uint32_t)best;
                    hit = true;
                    if (ANY && minT < limit) active = false;
                }
            }
        }
    }
    return hit;
}

// Packet form of walk_bvh_seq for coherent rays (a wave's 8x8 pixel tile of camera rays,
// or the tile's shadow rays towards one light): the wave walks ONE pre-order node sequence,
// the union of its lanes' walks, with a wave-uniform node index -- node and triangle records
// are scalar loads (one per wave, through the scalar cache, no per-lane addresses for the
// texture path) -- and every lane keeps its own walk exactly: a lane whose box test fails at
// node n sets resume = skip(n) and sits out until the wave reaches resume, i.e. it ignores
// n's subtree [n, skip(n)) precisely as its own stackless walk would.  Each lane therefore
// tests the same boxes and faces, in the same order, with the same minT, as walk_bvh_seq --
// same hits, same ties, same counters -- and the wave only adds masked-off idle lanes.
// The wave advances to i + 1 when some active lane enters node i's subtree, else to skip(i);
// if no lane is active at i (ANY lanes that finished), it jumps to the lanes' minimum resume.
DEV int wave_min_int(int v) {
    for (int m = 1; m < 64; m <<= 1) {
        const int o = __shfl_xor(v, m);
        v = o < v ? o : v;
    }
    return v;
}

// SC (RTG_PRIMARY_PACKET 2): the round-3 machinery of the any-hit packet walk -- the 32-B node
// and 48-B face records through the scalar cache (inline s_load: one load per wave), the face
// test with selects (tri_test_sel: early outs as lane masks, the t division and the exact
// fallback as wave-uniform branches) and the slab test's exact fallback as a wave-uniform
// branch; lanes outside their own walk take no part in either fallback.  SC = false: round 2's
// form (vector loads of the uniform address, per-lane face tests).
// Deferred large leaves (FEAT_BIGLEAF scenes, camera walk of production renders; k_bigleaf /
// k_hitfix in rtg_wave.hpp).  A lane that reaches a leaf of more than kDeferLeaf faces appends
// (its local ray, minT at entry, the leaf, its object, its pixel) to a queue and walks on
// without lowering minT.  Exact: the walk then visits a superset of the reference's boxes (its
// minT never drops below the reference's: only the deferred leaves' acceptances are missing
// from it, and every face the reference accepts elsewhere it accepts too), so the minimum in
// (t, object, face) order over its accepted faces and the deferred leaves' faces with t below
// their entry minT is at or below the reference's answer h; a candidate below h was never
// reached by the reference, i.e. it was culled at a minT above its t, so its own leaf box
// enters after t (hit before its box: rounding only).  Hence a winner whose leaf box passes at
// next_up(t) IS h; k_hitfix checks exactly that and runs the reference walk otherwise.
constexpr int kDeferLeaf = 16;
// A leaf is deferred only for the lanes of a wave that reach it when they are few; when many
// reach it together the wave tests it in the walk, every lane busy (RTG_DEFER_LANES: A/B)
// packet walks address their scalar records by 32-bit byte offsets: two scalar ops fewer per
// record than a 64-bit index; scenes are limited to 2^25 faces (rtg_scene_create), which keeps
// every node, wide node and face-record array below 4 GiB (k_primary 0.1881 -> 0.1828 ms,
// profiles/r04aa_addr_on_ab.txt)
template <int BYTES, typename T>
DEV const T* rec_at(const T* base, int i) {
    return (const T*)((const char*)base + (uint32_t)i * (uint32_t)BYTES);
}
#ifndef RTG_DEFER_LANES
#define RTG_DEFER_LANES 16
#endif
// (Round 5 also started node i + 1's record -- where a passing inner node descends -- while node
// i was tested, waiting for it at the end of the step: k_frame 0.2878 -> 0.2912 ms, C3-ton +1 %,
// C4 -0.7 %; profiles/r05ac_pk_prefetch_ab.txt.  The scalar loads' latency is already covered by
// the other waves.)
// (The camera packet walk's slab distances as three packed pairs of the node record: six fewer
// VALU per node step in the listing, but k_frame 0.289 -> 0.300 ms on the GPU,
// profiles/r05n_pairs_inst6_deferany_ab.txt -- removed.)
// (A/B parts of the lean packet walks: the any-hit walk, the closest-hit walk's face test)
struct DeferCtx {
    float4* e;
    int* count;
    int cap;
    int ray;                          // the pixel's work-buffer index
    bool deferred;                    // this lane appended an entry
};
// (t, object, face) as one 64-bit key: t > 0 orders like its bits; objects < 2^12, faces < 2^20
// (defer_ok); a sphere's face field is all ones
DEV uint64_t obj_key(float t, int k, int f) {
    return ((uint64_t)__float_as_uint(t) << 32) | ((uint64_t)(uint32_t)k << 20) | (uint64_t)((uint32_t)f & 0xFFFFFu);
}

template <bool ANY, bool STATS, bool SC = false, bool DEFER = false>
DEV bool walk_bvh_packet(const DevScene& S, int begin, int end, const Ray& r, float& minT, int& hitFace,
                         float limit, Cnt<STATS>& c, DeferCtx* dc = nullptr, int k = 0) {
    // the node range is the object's (wave-uniform): SGPRs, so the loop index and its bound stay
    // scalar; "a face was accepted" is read off hitFace at the end instead of a lane mask kept
    // through every iteration
    begin = __builtin_amdgcn_readfirstlane(begin);
    end = __builtin_amdgcn_readfirstlane(end);
    const int face0 = hitFace;
    bool hit = false;
    const RayRcp q = ray_rcp(r);
    const float slack0 = q.fast ? 1e-30f : INFINITY;   // box_pass_pk: a ray off the fast path is never sure
    const int kDone = 0x7FFFFFFF;
    int resume = begin;                              // per lane: first node it takes part in again
    int i = begin;                                   // wave-uniform
    while (i < end) {
        bool act = resume <= i;
        if (ANY && !__ballot(act)) {                 // only after ANY lanes finished
            const int all = __ballot(1) == ~0ull ? wave_min_int(resume) : [&] {
                int m = kDone;
                uint64_t em = __ballot(1);
                while (em) {
                    const int l = __ffsll((long long)em) - 1;
                    em &= em - 1;
                    const int v = __shfl(resume, l);
                    m = v < m ? v : m;
                }
                return m;
            }();
            i = __builtin_amdgcn_readfirstlane(all);
            continue;
        }
        i = __builtin_amdgcn_readfirstlane(i);
        const int ip1 = i + 1;                       // (shared by rel and the next-node select)
        float4 a, b;
        int ndr[8];
        if constexpr (SC) {
            rtg_s8 nd;
            sload_node(rec_at<32>(S.nodes, i), nd);
            a = f4(nd[0], nd[1], nd[2], nd[3]);
            b = f4(nd[4], nd[5], nd[6], nd[7]);
#pragma unroll
            for (int u = 0; u < 8; ++u) ndr[u] = nd[u];
        } else {
            a = S.nodes[2 * i];
            b = S.nodes[2 * i + 1];
        }
        const int skip = __float_as_int(b.z);
        const int leaf = __float_as_int(b.w);
        bool pass;
        if constexpr (SC) {
            if (act) c.template node<ANY>();
            pass = box_pass_pk(a.x, a.y, a.z, a.w, b.x, b.y, r, q, minT, ip1 - resume, slack0);
            // a lane inside its walk that fails the box resumes at the box's skip; lanes outside it
            // already wait for a node past this box's subtree (resume >= skip), as do lanes that pass
            resume = max(resume, pass ? 0 : skip);
        } else {
            pass = false;
            if (act) {
                c.template node<ANY>();
                pass = box_hit_fast(a.x, a.y, a.z, a.w, b.x, b.y, r, q, minT);
                if (!pass) resume = skip;
            }
        }
        // the next node and the leaf to test in five scalar instructions (the compiler kept the
        // two wave-uniform conditions as 64-bit masks with selects and branches between them):
        // lf = the leaf word when some lane passed, else 0 (no faces); next = lf < 0 (a passed
        // inner box) ? its first child : its skip
        const int cur = i;
        int lf;
        {
            const uint64_t pm = __builtin_amdgcn_ballot_w64(pass);
            int nx;
            asm("s_cmp_lg_u64 %[pm], 0\n\t"
                "s_cselect_b32 %[lf], %[leaf], 0\n\t"
                "s_cmp_lt_i32 %[lf], 0\n\t"
                "s_cselect_b32 %[nx], %[ip1], %[skip]"
                : [lf] "=&s"(lf), [nx] "=&s"(nx)
                : [pm] "s"(pm), [leaf] "s"(leaf), [ip1] "s"(ip1), [skip] "s"(skip)
                : "scc");
            i = nx;
        }
        if (lf > 0) {
            {
                int first = leaf >> 8, cnt = leaf & 255;
                if (leaf == LEAF_EXT) {
                    const int2 e = S.node_ext[cur];
                    first = __builtin_amdgcn_readfirstlane(e.x);
                    cnt = __builtin_amdgcn_readfirstlane(e.y);
                }
                if constexpr (DEFER) {
                    const uint64_t m = __ballot(pass);
                    if (cnt > kDeferLeaf && __popcll(m) <= RTG_DEFER_LANES) {
                        // one atomic per wave for the lanes that reached the leaf
                        const int lane = threadIdx.x & 63, lead = __ffsll((long long)m) - 1;
                        int base = 0;
                        if (lane == lead) base = atomicAdd(dc->count, __popcll(m));
                        base = __shfl(base, lead);
                        const int slot = base + __popcll(m & ((1ull << lane) - 1ull));
                        if (pass && slot < dc->cap) {
                            float4* q = dc->e + 3 * (size_t)slot;
                            q[0] = make_float4(r.o.x, r.o.y, r.o.z, minT);
                            q[1] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(dc->ray));
                            q[2] = make_float4(__int_as_float(first), __int_as_float(cnt), __int_as_float(k), 0.f);
                            dc->deferred = true;
                            pass = false;                // queued: no test here, minT unchanged
                        }
                        // (a lane whose entry did not fit tests the leaf below)
                    }
                }
                for (int f = first; f < first + cnt; ++f) {
                    if constexpr (SC) {
                        rtg_s8 ra;
                        rtg_s4 rb;
                        sload_rec(rec_at<48>(S.tris, f), ra, rb);
                        const float4 R[3] = {f4(ra[0], ra[1], ra[2], ra[3]), f4(ra[4], ra[5], ra[6], ra[7]),
                                             f4(rb[0], rb[1], rb[2], rb[3])};
                        if (pass) c.template tri<ANY>();
                        float t;
                        const bool ok = tri_test_pk(R, r, minT, t, pass ? 1.0f : -1.0f) > 0.0f;
                        minT = ok ? t : minT;
                        hitFace = ok ? f : hitFace;
                        if (ANY) {
                            const bool fin = ok & (t < limit);
                            pass &= !fin;
                            resume = fin ? kDone : resume;
                        }
                    } else if (pass) {
                        c.template tri<ANY>();
                        float t;
                        if (tri_test_fast(S, f, r, minT, t)) {
                            minT = t;
                            hitFace = f;
                            hit = true;
                            if (ANY && t < limit) {
                                pass = false;
                                resume = kDone;
                            }
                        }
                    }
                }
            }
        }
    }
    if constexpr (SC) return hit | (hitFace != face0);
    return hit;
}

#ifndef RTG_XFORM_LAUNDER
#define RTG_XFORM_LAUNDER 1
#endif
// Sphere::Intersect (sphere.cpp:13-78): root selection and acceptance; lo/ld local ray.
DEV bool sphere_t(const DevObject& ob, const Ray& lr, float minT, float& tout) {
    const f3 center = mk(ob.center[0], ob.center[1], ob.center[2]);
    const float radius = ob.center[3];
    f3 oc = sub(lr.o, center);
    float c = dot(oc, oc) - (radius * radius);
    float b = 2 * dot(lr.d, oc);
    float a = dot(lr.d, lr.d);
    float delta = b * b - (4 * a * c);
    if (delta < 0.0f) return false;
    delta = sqrtf(delta);
    a = (float)(2.0 * a);
    float t1 = (-b + delta) / a;
    float t2 = (-b - delta) / a;
    float t = t1 < t2 ? t1 : t2;
    if (t1 < t2) { t = (t1 > 0.0f) ? t1 : t2; }
    else if (t2 < t1) { t = (t2 > 0.0f) ? t2 : t1; }
    tout = t;
    return t < minT && t > 0.0f;
}

DEV Ray local_ray(const DevObject& ob, const Ray& r, float mbTime) {
    Ray lr;
    lr.o = xform(ob.inv, r.o, 1.0f);
    lr.d = xform(ob.inv, r.d, 0.0f);
    if (ob.flags & OBJF_MOTION_BLUR) lr.o = add(lr.o, muls(ld3(ob.mbv), mbTime));
    return lr;
}
// Traversal-only variant: an exact identity transform changes at most the sign of a zero
// component (1*x + 0*y + ...), which no box / triangle / sphere decision or t value
// depends on, so it is skipped.  Shading (surface()) always applies the full transform.
DEV Ray trav_ray(const DevObject& ob, const Ray& r0, float mbTime) {
    // the ray laundered, so the compiler does not hoist the transform's double conversions of
    // it out of the caller's object loop (twelve VGPRs live through every mesh walk, spilled at
    // eight waves): C5's k_tree_trace / k_shadow 28 B of scratch -> 0, C5 1 715 -> 1 787 Mrays/s
    // (profiles/r05ag_sphere_launder_ab.txt); the fused kernels (rtg_mega*.hip) set
    // RTG_XFORM_LAUNDER 0 -- C2 loses 6 % with it
    Ray r = r0;
#if RTG_XFORM_LAUNDER
    asm volatile("" : "+v"(r.o.x), "+v"(r.o.y), "+v"(r.o.z), "+v"(r.d.x), "+v"(r.d.y), "+v"(r.d.z));
#endif
    if (!(ob.flags & OBJF_IDENTITY)) return local_ray(ob, r, mbTime);
    Ray lr = r;
    if (ob.flags & OBJF_MOTION_BLUR) lr.o = add(lr.o, muls(ld3(ob.mbv), mbTime));
    return lr;
}

struct Hit {
    float t;
    int obj, face;     // face < 0: sphere
    f3 o;              // world ray origin when the hit was accepted (normal/uv are computed then)
};

// IntersectObjects (raytracer.cpp:625-643) / CastShadowRay (raytracer.cpp:585-623).
// Closest hit: shared minT across objects, earlier object wins ties (strict <).
// Any hit (ANY): skip emissive meshes, true as soon as a hit with t < limit exists.
// The ray is updated in place like the reference's: an instance with motion blur whose
// bbox test fails leaves its offset on the ray origin (instancedMesh.cpp:18-60).
// FEAT (scene features the caller guarantees absent when the bit is clear) lets the
// traversal kernels drop whole code paths -- and their registers -- for plain scenes.
template <bool ANY, bool STATS, int FEAT = FEAT_ALL, bool PK = false, bool DEFER = false>
DEV bool trace(const DevScene& S, Ray& r, float mbTime, float minT, float limit, Hit& h, Cnt<STATS>& c,
               DeferCtx* dc = nullptr) {
    h.t = minT;
    h.obj = -1;
    h.face = -1;
    // instance world-bbox tests: the division-free slab test (same decisions, box_hit_fast);
    // the motion-blur quirk moves r.o between objects, never r.d
    const RayRcp rq = (FEAT & FEAT_INSTANCE) ? ray_rcp(r) : RayRcp{};
    int gskip = 0;                   // packet walks: this lane skips objects below gskip
    for (int k = 0; k < S.num_objects; ++k) {
        const DevObject& ob = S.objects[k];
        // Instance groups (runs of consecutive instances without motion blur): every member's
        // world box lies inside the group's, and the slab test is monotone in the box and in
        // minT, so a group box that fails at the current minT fails for every member tested
        // after it -- the members can be skipped with the same result.
        // Packet walks keep the object index wave-uniform (walk_bvh_packet needs one node
        // range per wave): a lane whose group box fails sits the group out, and the wave
        // jumps over it when every lane does.
        if ((FEAT & FEAT_INSTANCE) && ob.group_end > k) {
            const float4 ga = S.group_box[2 * k], gb = S.group_box[2 * k + 1];
            if constexpr (PK) {
                if (k >= gskip && !box_hit_fast(ga.x, ga.y, ga.z, gb.x, gb.y, gb.z, r, rq, h.t)) gskip = ob.group_end;
                if (!__ballot(k >= gskip)) {
                    k = ob.group_end - 1;
                    continue;
                }
            } else if (!box_hit_fast(ga.x, ga.y, ga.z, gb.x, gb.y, gb.z, r, rq, h.t)) {
                k = ob.group_end - 1;
                continue;
            }
        }
        if (PK && k < gskip) continue;
        c.obj();
        if ((FEAT & FEAT_SPHERE) && ob.kind == OBJ_SPHERE) {
            c.sph();
            Ray lr = trav_ray(ob, r, mbTime);
            float t;
            if (sphere_t(ob, lr, h.t, t)) {
                h.t = t; h.obj = k; h.face = -1; h.o = r.o;
                if (ANY && t < limit) return true;
            }
            continue;
        }
        if (ANY && (ob.flags & OBJF_SHADOW_SKIP)) continue;
        if ((FEAT & FEAT_INSTANCE) && ob.kind == OBJ_INSTANCE) {
            // InstancedMesh::Intersect (instancedMesh.cpp:16-66): world bbox first
            Ray wr = r;
            if (ob.flags & OBJF_MOTION_BLUR) wr.o = add(wr.o, muls(ld3(ob.mbv), mbTime));
            if (!box_hit_fast(ob.bmin[0], ob.bmin[1], ob.bmin[2], ob.bmax[0], ob.bmax[1], ob.bmax[2], wr, rq, h.t)) {
                r.o = wr.o;
                continue;
            }
        }
        // Mesh::Intersect (mesh.cpp:158-188); the mesh bbox test equals the root-node test
        Ray lr = (FEAT & FEAT_XFORM) ? trav_ray(ob, r, mbTime) : r;
        int face = -1;
        float t = h.t;
        bool found;
        if constexpr (PK)
            found = walk_bvh_packet<ANY, STATS, RTG_PRIMARY_PACKET == 2, DEFER>(S, ob.node_begin, ob.node_end, lr, t,
                                                                                  face, limit, c, dc, k);
        else found = walk_bvh<ANY, STATS, (FEAT & FEAT_BIGLEAF) != 0>(S, ob.node_begin, ob.node_end, lr, t, face, limit, c);
        if (found) {
            h.t = t; h.obj = k; h.face = face; h.o = r.o;
            if (ANY && t < limit) return true;
        }
    }
    return !ANY && h.obj >= 0;
}

// ---------------------------------------------------------------------------
// Shadow rays on the any-hit wide BVH (WNode, rtg_device.hpp)
// ---------------------------------------------------------------------------
// CastShadowRay (raytracer.cpp:585-623) answers one boolean: with minT0 = the initial minT
// (lightT + 0.01, or inf) and limit = lightT, the reference walks the objects in order,
// each with its BVH in its own order, minT shrinking to every accepted hit, and answers
// true once a hit with t < limit is found.  Until then minT_cur lies in [limit, minT0].
// For a face f of reference leaf L (box B_L), with tri_ok(f) = "IntersectFace accepts f
// with 0 < t < limit" (its early outs do not depend on minT):
//   * sufficient: tri_ok(f) and slab(B_L, limit) [and, for an instance, its world box at
//     limit].  Every ancestor box of L contains B_L (unions of face boxes, exact min/max),
//     and the slab test is monotone in the box and in minT, so every box on L's path
//     passes at any minT_cur >= limit, and f is accepted with t < limit <= minT_cur;
//   * necessary: some f with tri_ok(f) and slab(B_L, minT0) (same monotonicity).
// The wide walk visits every leaf whose box passes at minT0 (each wide child box contains
// the leaf boxes below it; the child test is conservative), in any order, and answers 1 at
// the first face meeting the sufficient condition.  A face meeting only the necessary one
// (its leaf box entry within rounding of lightT -- a light lying on a surface) or a full
// traversal stack make the answer "undecided" (-1): the caller then runs the reference
// walk for that ray.  0: no face meets the necessary condition -- not in shadow.
// k_shadow<FAST> / the fused shade kernel (the wide walk + the in-place reference fallback)
// compiled for this many waves per SIMD.  (Round 3's per-lane walk, removed: five waves, 96
// VGPRs, 0.228 ms on the headline.)  Packet walk: 81 VGPRs and no LDS stack at five, six 0.211 ms, seven
// 0.215, eight 0.216 (profiles/r03pk4_*); instance scenes keep RTG_INST_WAVES.  Round 4, after
// the leaner slab test and mask copies: five 0.193, six 0.1804, seven 0.1742, eight 0.270 ms
// (spills), large-leaf configurations unchanged (profiles/r04ad_wide_waves_ab.txt, r04ae_wide_waves_configs_ab.txt)
#ifndef RTG_WIDE_WAVES_PLAIN
#define RTG_WIDE_WAVES_PLAIN 7
#endif
// instance scenes' any-hit walks (their own knob): the deferring shadow walk spills 124 B per
// lane at six waves, 76 at five and none at four (118 VGPRs), and six is the fastest -- C4
// 3 163 / 3 093 / 2 963 Mrays/s (profiles/r05w_c4_any_waves_ab.txt): occupancy over spill traffic
#ifndef RTG_INST_ANY_WAVES
#define RTG_INST_ANY_WAVES 6
#endif
#define RTG_WIDE_WAVES(FEAT) (((FEAT) & FEAT_INSTANCE) ? RTG_INST_ANY_WAVES : RTG_WIDE_WAVES_PLAIN)


// DEFER (large-leaf scenes, the packet walk): a leaf slot of more than RTG_DEFER_ANY_LEAF entries
// that at most RTG_DEFER_ANY_LANES lanes reach is queued for those lanes (k_bigleaf_any) instead
// of tested; the decisions are the same per face wherever they are taken, so the answer is
// unchanged.  (Per lane, walk_wide_any, measured slower: C3 4 735, C3-ton 2 844, C4 2 150
// Mrays/s against 4 400 / 5 333 / 2 494 for the packet, profiles/r04p_any_walk_ab.txt.)
#ifndef RTG_DEFER_ANY_LANES
#define RTG_DEFER_ANY_LANES 16
#endif
#ifndef RTG_DEFER_ANY_LEAF
#define RTG_DEFER_ANY_LEAF 16
#endif
struct AnyDefer {
    float4* e;
    int* count;
    int cap;
    int q;                            // the shadow ray's queue entry
    bool deferred;
};
// One mesh's any-hit tree (rtg_ahb.cpp; local ray lr) walked as a wave packet.  inst_conf: the
// instance's world box passes at limit (true for plain meshes).  Returns 1 / 0 / -1 as above.
// The wave visits one node sequence, the
// union of its live lanes' walks, so node, face and reference-leaf records are wave-uniform
// (scalar loads through the scalar cache, nothing through the vector memory path) and the
// stack is wave-uniform too (64 LDS words per wave, written by one live lane).  A lane tests a child, a face or a
// leaf box wherever the wave goes, also below boxes it failed itself: every decision is the
// exact one above (sufficient -> 1, necessary only -> undecided), so extra tests change no
// answer, and every leaf a lane's own walk reaches is still visited.  A lane leaves the packet
// at its first sufficient face; the wave stops when no live lane is left or the stack is empty.
// The nearest inner child of the first live lane goes next, the others onto the stack.
#define RTG_PK_STACK 64
// the packet walk's face tests with selects and wave-uniform branches (1: k_shade_shadow 0.211 ->
// 0.190 ms, profiles/r03sel_ab.txt) or per-lane early outs (0)
#ifndef RTG_PK_MAX_STEPS
#define RTG_PK_MAX_STEPS 4096
#endif
// slab_cons as a value (> 0: the conservative test passes and the lane walks, livef > 0): tmax >
// -1e-30 is tmax + 1e-30 > 0 and tmin < minTc is minTc - tmin > 0 (exact: rounded sums and
// differences keep their signs); tmax >= tmin (1 - 2^-21) - 1e-30 is loosened by another 1e-30
// so that it becomes a strict comparison too -- the test only has to keep every box the exact
// test keeps (walk_wide_any_pk: extra boxes change no answer).
DEV float slab_cons_v(float lx, float ly, float lz, float hx, float hy, float hz, const SlabRay& s, float minTc,
                      float& tnear, float livef) {
    const float tx1 = (lx - s.o.x) * s.ix, tx2 = (hx - s.o.x) * s.ix;
    const float ty1 = (ly - s.o.y) * s.iy, ty2 = (hy - s.o.y) * s.iy;
    const float tz1 = (lz - s.o.z) * s.iz, tz2 = (hz - s.o.z) * s.iz;
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    tnear = tmin;
    return __builtin_elementwise_minimum(
        vmin3(tmax + 1e-30f, (tmax - fmaf(tmin, 1.0f - 0x1p-21f, -1e-30f)) + 1e-30f, minTc - tmin), livef);
}

template <bool STATS, bool DEFER = false>
DEV int walk_wide_any_pk(const DevScene& S, int node, const Ray& lr, float minT0, float limit, bool inst_conf,
                         Cnt<STATS>& c, AnyDefer* ad = nullptr) {
    // The lane state as values, every wave-level test one comparison (the mask version kept
    // live / occluded / undecided and the four child masks as SGPR pairs merged at every block
    // and spilled to VGPR lanes): livef > 0 walking, occ / und flags, a child's hk > 0 taking it.
    const RayRcp q = ray_rcp(lr);
    const float minTc = minT0 * (1.0f + 0x1p-21f);
    const SlabRay sr = slab_ray(lr, q);
    const float slack0 = q.fast ? 1e-30f : INFINITY;
    const float icf = inst_conf ? 1.0f : -1.0f;
    float livef = q.fast ? 1.0f : -1.0f;
    int occ = 0;
    int und = q.fast ? 0 : 1;                        // zero / tiny direction component: reference walk
    __shared__ int pk_stack[4][RTG_PK_STACK];        // the wave's stack (256-thread blocks)
    int* const stk = pk_stack[(threadIdx.x >> 6) & 3];
    int sp = 0;                                      // wave-uniform
    node = __builtin_amdgcn_readfirstlane(node);
    int steps = 0;                                   // bound: a walk visits each node once
    while (__ballot(livef > 0.0f)) {
        if (++steps > RTG_PK_MAX_STEPS) {
            und |= livef > 0.0f;
            break;
        }
        node = __builtin_amdgcn_readfirstlane(node);
        rtg_s16 na, nb;
        sload_wnode(rec_at<128>(S.anodes, node), na, nb);
        if (livef > 0.0f) c.wnode();
        float tn[4], hv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            hv[k] = slab_cons_v(__int_as_float(na[k]), __int_as_float(na[8 + k]), __int_as_float(nb[k]),
                                __int_as_float(na[4 + k]), __int_as_float(na[12 + k]), __int_as_float(nb[4 + k]), sr,
                                minTc, tn[k], livef);
        const int lead = __ffsll((long long)__ballot(livef > 0.0f)) - 1;
        int next = -1;
        float nextT = INFINITY;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int cr = nb[8 + k], lfw = nb[12 + k];
            float hk = hv[k];
            if (cr == WCHILD_EMPTY || !__ballot(hk > 0.0f)) continue;
            if (cr >= 0) {
                const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tn[k]), lead));
                int spill = cr;
                if (t < nextT) {
                    spill = next;
                    next = cr;
                    nextT = t;
                }
                if (spill >= 0) {
                    if (sp < RTG_PK_STACK) {             // written by the first live lane
                        if ((int)(threadIdx.x & 63) == lead) stk[sp] = spill;
                        ++sp;
                    } else {
                        und |= livef > 0.0f;
                    }
                }
                continue;
            }
            const int first = lfw >> 8, cnt = lfw & 255;
            if constexpr (DEFER) {
                const uint64_t m = __ballot(hk > 0.0f);
                if (cnt > RTG_DEFER_ANY_LEAF && __popcll(m) <= RTG_DEFER_ANY_LANES) {
                    const int lane = threadIdx.x & 63, ld = __ffsll((long long)m) - 1;
                    int base = 0;
                    if (lane == ld) base = atomicAdd(ad->count, __popcll(m));
                    base = __shfl(base, ld);
                    const int slot = base + __popcll(m & ((1ull << lane) - 1ull));
                    if (hk > 0.0f && slot < ad->cap) {
                        float4* qe = ad->e + 3 * (size_t)slot;
                        qe[0] = make_float4(lr.o.x, lr.o.y, lr.o.z, minT0);
                        qe[1] = make_float4(lr.d.x, lr.d.y, lr.d.z, limit);
                        qe[2] = make_float4(__int_as_float(first), __int_as_float(cnt), __int_as_float(ad->q),
                                            __int_as_float((int)inst_conf));
                        ad->deferred = true;
                        hk = -1.0f;
                    }
                }
            }
            for (int e = first; e < first + cnt; ++e) {
                rtg_s8 ra;
                rtg_s4 rb;
                sload_rec(rec_at<48>(S.ahtris, e), ra, rb);
                if (hk > 0.0f) c.template tri<true>();
                const float4 R[3] = {f4(ra[0], ra[1], ra[2], ra[3]), f4(ra[4], ra[5], ra[6], ra[7]), f4(rb[0], rb[1], rb[2], rb[3])};
                float t;
                const float okv = tri_test_pk(R, lr, limit, t, hk);
                if (!__ballot(okv > 0.0f)) continue;
                // the exact decisions on the face's reference leaf box: reachable at minT0
                // (necessary), and at limit (sufficient, for an instance whose world box passes)
                rtg_s8 rn;
                sload_node(rec_at<32>(S.nodes, ra[3]), rn);
                const float rv = box_pass_v(__int_as_float(rn[0]), __int_as_float(rn[1]), __int_as_float(rn[2]),
                                            __int_as_float(rn[3]), __int_as_float(rn[4]), __int_as_float(rn[5]), lr, q,
                                            minT0, okv, slack0);
                const float sv = box_pass_v(__int_as_float(rn[0]), __int_as_float(rn[1]), __int_as_float(rn[2]),
                                            __int_as_float(rn[3]), __int_as_float(rn[4]), __int_as_float(rn[5]), lr, q,
                                            limit, __builtin_elementwise_minimum(rv, icf), slack0);
                const bool suff = sv > 0.0f;
                occ = suff ? 1 : occ;
                livef = suff ? -1.0f : livef;
                hk = suff ? -1.0f : hk;
                und |= (rv > 0.0f) & !suff;
            }
        }
        if (!__ballot(livef > 0.0f)) break;
        if (next >= 0) {
            node = next;
            continue;
        }
        if (sp == 0) break;
        node = stk[--sp];
    }
    return occ ? 1 : (und ? -1 : 0);
}

// CastShadowRay on the wide BVH: objects in any order (the answer is a boolean), spheres
// exactly (a sphere hit with t < limit is accepted at any minT_cur >= limit, one with
// t >= limit never decides).  Returns 1 / 0 / -1 (undecided: run trace<true>).
template <bool STATS, int FEAT, bool DEFER = false>
DEV int trace_any_wide(const DevScene& S, const Ray& r, float minT0, float limit, Cnt<STATS>& c,
                       AnyDefer* ad = nullptr) {
    const RayRcp rq = (FEAT & FEAT_INSTANCE) ? ray_rcp(r) : RayRcp{};
    if ((FEAT & FEAT_INSTANCE) && !rq.fast) return -1;
    bool undecided = false;
    int gskip = 0;                   // packet walks: this lane skips objects below gskip
    for (int k = 0; k < S.num_objects; ++k) {
        const DevObject& ob = S.objects[k];
        if ((FEAT & FEAT_INSTANCE) && ob.group_end > k) {
            const float4 ga = S.group_box[2 * k], gb = S.group_box[2 * k + 1];
            // the packet walk needs one object (one root) per wave: a lane whose group box
            // fails sits the group out, and the wave jumps over it when every lane does
            if (k >= gskip && !box_hit_fast(ga.x, ga.y, ga.z, gb.x, gb.y, gb.z, r, rq, minT0))
                gskip = ob.group_end;
            if (!__ballot(k >= gskip)) {
                k = ob.group_end - 1;
                continue;
            }
        }
        if (k < gskip) continue;
        c.obj();
        if ((FEAT & FEAT_SPHERE) && ob.kind == OBJ_SPHERE) {
            c.sph();
            Ray lr = trav_ray(ob, r, 0.f);
            float t;
            if (sphere_t(ob, lr, limit, t)) return 1;
            continue;
        }
        if (ob.flags & OBJF_SHADOW_SKIP) continue;
        bool conf = true;
        if ((FEAT & FEAT_INSTANCE) && ob.kind == OBJ_INSTANCE) {
            if (!box_hit_fast(ob.bmin[0], ob.bmin[1], ob.bmin[2], ob.bmax[0], ob.bmax[1], ob.bmax[2], r, rq, minT0))
                continue;
            conf = box_hit_fast(ob.bmin[0], ob.bmin[1], ob.bmin[2], ob.bmax[0], ob.bmax[1], ob.bmax[2], r, rq, limit);
        }
        const Ray lr = (FEAT & FEAT_XFORM) ? trav_ray(ob, r, 0.f) : r;
        if (ob.aroot < 0) return -1;                 // no any-hit tree for this mesh: reference walk
        const int res = walk_wide_any_pk<STATS, DEFER>(S, ob.aroot, lr, minT0, limit, conf, c, ad);
        if (res > 0) return 1;
        undecided |= res < 0;
    }
    return undecided ? -1 : 0;
}

// ---------------------------------------------------------------------------
// Opt-in ordered closest hit (RTG_RENDER_ORDERED; meshes with identity transforms only)
// ---------------------------------------------------------------------------
// IntersectObjects' answer is the last face it accepts.  Let C be the faces IntersectFace
// accepts at minT = inf whose reference leaf box passes the slab test at inf, and f* the
// minimum of C in the (t, object, face) order.  Every accepted face is in C, faces before f*
// in the walk have larger t (a smaller or equal t would precede f* in that order), so when
// the reference reaches f* its minT exceeds t* and f* is accepted, and nothing after it can
// be.  It reaches f* for certain if f*'s leaf box passes at t* (tmin <= t*: every ancestor
// box contains it, the slab test is monotone in box and minT).  This walk visits the 4-wide
// BVH nearest child first and culls a child only when its conservative entry distance is
// beyond the best t so far, so it finds f* unless a face of C hides in a culled box with
// t below the box's entry -- rounding on a box boundary or an ill-conditioned triangle, which
// no cheap test excludes.  The result is therefore checked, not proven: the winner's leaf box
// must pass exactly at t* and no box may have been culled within 2^-16 (relative) of t*;
// otherwise (or on a stack overflow) the caller runs the reference walk.  No hit at all is
// exact (nothing is culled before a face is found).  Off by default; tests report its
// agreement with the reference order (tests/test_gpu_ordered.py).
// Smallest float above a positive x (inf stays inf): "minT = next_up(t)" accepts t' <= t.
DEV float next_up(float x) { return x == INFINITY ? x : __uint_as_float(__float_as_uint(x) + 1u); }

// ---------------------------------------------------------------------------
// Closest hit on the any-hit tree as wave packets (RTG_RENDER_ORDERED, mode 2: the default
// ordered walk)
// ---------------------------------------------------------------------------
// Order candidates by (t, object, face): the face index is the BVH-order one, so within a mesh
// it is the reference walk's order.  Let C be the faces IntersectFace accepts at minT = inf
// whose reference leaf box B_L passes the slab test at inf (the faces the reference can reach
// at all), and V the visible ones: B_L passes at next_up(t_f), i.e. B_L's entry is at most t_f
// (spheres count as visible).  IntersectObjects returns min(V) -- unless a face of C \ V (a
// hidden face: hit before its own leaf box's entry, by rounding alone) lies below min(V):
//   * when the reference reaches the ancestors of v = min(V) its minT exceeds t_v or is already
//     at most t_v; every ancestor box contains B_L(v), and the slab test is monotone in box and
//     minT, so the reference ends at or below v;
//   * a face f of C below the reference's answer h was not accepted although t_f < minT, so an
//     ancestor failed at some minT > t_f, hence B_L(f) fails at a minT above t_f: f is hidden.
// This walk finds min(V) on any tree whose boxes contain the reference leaf boxes (the any-hit
// tree's: unions of the B_L, exact float min / max): a child is culled only when its
// conservative slab test fails at the lane's best t, which a box holding a face of V below that
// best cannot do.  Hidden faces met in the walk are kept as a lower candidate; if one lies below
// the result, the lane takes the reference walk.  A hidden face in a culled box cannot be ruled
// out by a cheap test (its Cramer-rule t may sit below the box entry by rounding, without bound
// for rays grazing the face), so the result is checked like round 3's ordered walk: a lane whose
// culled boxes came within 2^-16 (relative) of its t takes the reference walk too.
//
// As a packet: the wave walks one node sequence (scalar-cache node / face / leaf records), the
// union of its lanes' walks; leaf children are tested before the inner ones (they can only lower
// t), the first lane with a passing inner child picks the nearest next, the others go onto the
// wave's LDS stack with the least entry distance of the lanes that passed them, and a popped entry
// no lane can still use is dropped (recorded as a cull at that distance).  Returns false for a lane
// whose result is not certain (caller: reference walk).
DEV bool hit_less(float t, int k, int f, float bt, int bk, int bf) {
    return (t < bt) | ((t == bt) & ((k < bk) | ((k == bk) & (f < bf))));
}
DEV bool slab_cons2(float lx, float ly, float lz, float hx, float hy, float hz, const SlabRay& s, float minTc,
                    float& tnear, bool& hinf) {
    const float tx1 = (lx - s.o.x) * s.ix, tx2 = (hx - s.o.x) * s.ix;
    const float ty1 = (ly - s.o.y) * s.iy, ty2 = (hy - s.o.y) * s.iy;
    const float tz1 = (lz - s.o.z) * s.iz, tz2 = (hz - s.o.z) * s.iz;
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    tnear = tmin;
    hinf = (tmax > -1e-30f) & (tmax >= fmaf(tmin, 1.0f - 0x1p-21f, -1e-30f));
    return hinf & (tmin < minTc);
}
// wave minimum of a non-negative float (the lanes that do not take part hold +inf)
DEV float wave_min_pos(float v) {
    uint32_t u = __float_as_uint(v);
    for (int m = 1; m < 64; m <<= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)u, m);
        u = o < u ? o : u;
    }
    return __uint_as_float(u);
}
DEV float cull_limit(float t) { return t * (1.0f + 0x1p-20f); }   // inf stays inf

struct ClosestState {
    float bestT, hidT, cullMin;
    int bestK, bestF, hidK, hidF;
};

template <bool STATS>
DEV bool walk_closest_pk(const DevScene& S, int node, const int k, const Ray& lr, const RayRcp& q, const SlabRay& sr,
                         ClosestState& B, Cnt<STATS>& c) {
    __shared__ int ck_node[4][RTG_PK_STACK];
    __shared__ float ck_tn[4][RTG_PK_STACK];
    int* const stk = ck_node[(threadIdx.x >> 6) & 3];
    float* const stn = ck_tn[(threadIdx.x >> 6) & 3];
    // the stack is written by the first active lane (edge tiles run with partial waves)
    const bool writer = (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
    int sp = 0;                                      // wave-uniform
    int steps = 0;
    node = __builtin_amdgcn_readfirstlane(node);
    while (true) {
        if (++steps > RTG_PK_MAX_STEPS) return false;
        node = __builtin_amdgcn_readfirstlane(node);
        rtg_s16 na, nb;
        sload_wnode(rec_at<128>(S.anodes, node), na, nb);
        const float4 lox = f4(na[0], na[1], na[2], na[3]), hix = f4(na[4], na[5], na[6], na[7]);
        const float4 loy = f4(na[8], na[9], na[10], na[11]), hiy = f4(na[12], na[13], na[14], na[15]);
        const float4 loz = f4(nb[0], nb[1], nb[2], nb[3]), hiz = f4(nb[4], nb[5], nb[6], nb[7]);
        const int cidx[4] = {nb[8], nb[9], nb[10], nb[11]};
        const int lidx[4] = {nb[12], nb[13], nb[14], nb[15]};
        c.ewnode();
        const float minTc = cull_limit(B.bestT);
        float tn[4];
        bool h[4], hi[4];
        h[0] = slab_cons2(lox.x, loy.x, loz.x, hix.x, hiy.x, hiz.x, sr, minTc, tn[0], hi[0]);
        h[1] = slab_cons2(lox.y, loy.y, loz.y, hix.y, hiy.y, hiz.y, sr, minTc, tn[1], hi[1]);
        h[2] = slab_cons2(lox.z, loy.z, loz.z, hix.z, hiy.z, hiz.z, sr, minTc, tn[2], hi[2]);
        h[3] = slab_cons2(lox.w, loy.w, loz.w, hix.w, hiy.w, hiz.w, sr, minTc, tn[3], hi[3]);
        // leaf children first: their faces can only lower t
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (cidx[j] == WCHILD_EMPTY || cidx[j] >= 0) continue;
            if (hi[j] & !h[j]) B.cullMin = fminf(B.cullMin, tn[j]);
            if (!__ballot(h[j])) continue;
            const int first = lidx[j] >> 8, cnt = lidx[j] & 255;
            for (int e = first; e < first + cnt; ++e) {
                rtg_s8 ra;
                rtg_s4 rb;
                sload_rec(rec_at<48>(S.ahtris, e), ra, rb);
                const float4 R[3] = {f4(ra[0], ra[1], ra[2], ra[3]), f4(ra[4], ra[5], ra[6], ra[7]),
                                     f4(rb[0], rb[1], rb[2], rb[3])};
                const int f = ra[7];
                if (h[j]) c.template tri<false>();
                float t;
                const bool ok = h[j] & tri_test_sel(R, lr, INFINITY, t, h[j]);
                const bool better = ok && hit_less(t, k, f, B.bestT, B.bestK, B.bestF);
                if (!__ballot(better)) continue;
                rtg_s8 rn;
                sload_node(rec_at<32>(S.nodes, ra[3]), rn);
                const float bx0 = __int_as_float(rn[0]), by0 = __int_as_float(rn[1]), bz0 = __int_as_float(rn[2]);
                const float bx1 = __int_as_float(rn[3]), by1 = __int_as_float(rn[4]), bz1 = __int_as_float(rn[5]);
                // visible: the reference leaf box passes at next_up(t) (its entry is at most t)
                const bool vis = better & box_hit_fast<true>(bx0, by0, bz0, bx1, by1, bz1, lr, q, next_up(t), better);
                const bool hcand = better & !vis;
                // a hidden face counts only if the reference can reach it at all (B_L passes at inf)
                const bool hid = hcand & box_hit_fast<true>(bx0, by0, bz0, bx1, by1, bz1, lr, q, INFINITY, hcand);
                if (vis) { B.bestT = t; B.bestK = k; B.bestF = f; }
                if (hid && hit_less(t, k, f, B.hidT, B.hidK, B.hidF)) { B.hidT = t; B.hidK = k; B.hidF = f; }
            }
        }
        // inner children against the (possibly lowered) best t: the nearest passing child of the
        // first lane that has one goes next, the others onto the stack
        const float minTc2 = cull_limit(B.bestT);
        bool h2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool inner = cidx[j] >= 0;
            h2[j] = inner & h[j] & (tn[j] < minTc2);
            if (inner & hi[j] & !h2[j]) B.cullMin = fminf(B.cullMin, tn[j]);
        }
        const uint64_t any = __ballot(h2[0] | h2[1] | h2[2] | h2[3]);
        int next = -1;
        if (any) {
            const int lead = __ffsll((long long)any) - 1;
            float nextT = INFINITY, nextTw = INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!__ballot(h2[j])) continue;
                const float tl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h2[j] ? tn[j] : INFINITY), lead));
                const float tw = wave_min_pos(h2[j] ? fmaxf(tn[j], 0.0f) : INFINITY);
                int spill = cidx[j];
                float spillT = tw;
                if (next < 0 || tl < nextT) {
                    spill = next;
                    spillT = nextTw;
                    next = cidx[j];
                    nextT = tl;
                    nextTw = tw;
                }
                if (spill >= 0) {
                    if (sp >= RTG_PK_STACK) return false;   // stack full: every lane takes the reference walk
                    if (writer) { stk[sp] = spill; stn[sp] = spillT; }
                    ++sp;
                }
            }
        }
        if (next >= 0) {
            node = next;
            continue;
        }
        // pop the next entry some lane can still use; the others are culls at their distance
        bool found = false;
        while (sp > 0) {
            --sp;
            const int n = stk[sp];
            const float tw = stn[sp];
            if (__ballot(tw < cull_limit(B.bestT))) {
                node = n;
                found = true;
                break;
            }
            B.cullMin = fminf(B.cullMin, tw);
        }
        if (!found) break;
    }
    return true;
}

// IntersectObjects on the any-hit trees (meshes with identity transforms and spheres only:
// FEAT 0 / FEAT_SPHERE).  true: h holds the reference's answer; false: take the reference walk.
template <bool STATS, int FEAT>
DEV bool trace_closest_pk(const DevScene& S, const Ray& r, Hit& h, Cnt<STATS>& c) {
    static_assert((FEAT & ~FEAT_SPHERE) == 0, "meshes with identity transforms and spheres only");
    const RayRcp q = ray_rcp(r);
    const SlabRay sr = slab_ray(r, q);
    ClosestState B;
    B.bestT = B.hidT = B.cullMin = INFINITY;
    B.bestK = B.bestF = B.hidK = B.hidF = 0x7FFFFFFF;
    bool sure = q.fast;                              // zero / tiny direction component: reference walk
    for (int k = 0; k < S.num_objects; ++k) {
        const DevObject& ob = S.objects[k];
        c.obj();
        if ((FEAT & FEAT_SPHERE) && ob.kind == OBJ_SPHERE) {
            c.sph();
            float t;
            // a later object wins only with a strictly smaller t (sphere_t: 0 < t < minT)
            if (sphere_t(ob, r, B.bestT, t)) { B.bestT = t; B.bestK = k; B.bestF = -1; }
            continue;
        }
        if (ob.aroot < 0) return false;
        sure &= walk_closest_pk<STATS>(S, ob.aroot, k, r, q, sr, B, c);
    }
    sure &= !hit_less(B.hidT, B.hidK, B.hidF, B.bestT, B.bestK, B.bestF);
    sure &= !(B.bestT < INFINITY && B.cullMin <= B.bestT * (1.0f + 0x1p-16f));
    h.t = B.bestT;
    h.obj = B.bestT < INFINITY ? B.bestK : -1;
    h.face = B.bestT < INFINITY ? B.bestF : -1;
    h.o = r.o;
    return sure;
}

// ---------------------------------------------------------------------------
// Hit reconstruction: normal / uv of the winning primitive
// ---------------------------------------------------------------------------
DEV float tiledUV(float x) {                                           // mesh.cpp:382-389
    if (x > 1.0001f) {
        x = x - floorf(x);
        if (x < 0.0001) x = 1.0f;
    }
    return x;
}

struct Surf {
    f3 p, n;
    float u, v;
};

DEV f3 mesh_mapped_normal(const DevScene& S, const DevObject& ob, int face, f3 lp, float u, float v);
DEV f3 sphere_bumped_normal(const DevScene& S, const DevObject& ob, f3 p, float phi, float theta, float u, float v);

// MAPS = false: the scene has no normal / bump maps (OBJF_MAPPED never set; k_shade variants)
template <bool STATS, bool MAPS = true>
DEV Surf surface(const DevScene& S, const Ray& r, float mbTime, const Hit& h, Cnt<STATS>& c) {
    const DevObject& ob = S.objects[GIDX(S, h.obj, S.num_objects, 0)];
    Surf s;
    s.p = add(r.o, muls(r.d, h.t));                                    // raytracer.cpp:69
    s.u = s.v = 0.f;
    Ray hr;
    hr.o = h.o;
    hr.d = r.d;
    Ray lr = local_ray(ob, hr, mbTime);
    if (h.face < 0) {                                                  // sphere.cpp:71-175
        const f3 center = mk(ob.center[0], ob.center[1], ob.center[2]);
        f3 lp = add(lr.o, muls(lr.d, h.t));
        f3 p = sub(lp, center);
        float phi = atan2f(p.z, p.x);
        float theta = acosf(p.y / ob.center[3]);
        s.u = (float)((-phi + RT_PI) / (2.0f * RT_PI));
        s.v = (float)(theta / RT_PI);
        f3 n = (MAPS && (ob.flags & OBJF_MAPPED)) ? sphere_bumped_normal(S, ob, p, phi, theta, s.u, s.v)
                                        : makeUnit(sub(lp, center));
        s.n = makeUnit(xform(ob.invT, n, 0.0f));
        return s;
    }
    f3 n = ld3(&S.face_n[GIDX(S, h.face, S.num_faces, 3)].x);
    if (ob.flags & OBJF_NORMAL_TWICE) n = makeUnit(xform(ob.baseInvT, n, 0.0f));   // mesh.cpp:363
    if (ob.flags & OBJF_HAS_UV) {                                                     // mesh.cpp:245-262
        float bg[2], t;
        tri_test(S, h.face, lr, INFINITY, t, bg);
        const float2 a = S.face_uv[3 * h.face], b = S.face_uv[3 * h.face + 1], cc = S.face_uv[3 * h.face + 2];
        float u = a.x + bg[0] * (b.x - a.x) + bg[1] * (cc.x - a.x);
        float v = a.y + bg[0] * (b.y - a.y) + bg[1] * (cc.y - a.y);
        s.u = tiledUV(u);
        s.v = tiledUV(v);
        if (MAPS && (ob.flags & OBJF_MAPPED)) {
            // IntersectFace's local hit point (mesh.cpp:242), then the base mesh's transform
            const f3 lp = add(lr.o, muls(lr.d, h.t));
            n = makeUnit(xform(ob.baseInvT, mesh_mapped_normal(S, ob, h.face, lp, s.u, s.v), 0.0f));
        }
    }
    s.n = makeUnit(xform(ob.invT, n, 0.0f));                                          // mesh.cpp:179 / instancedMesh.cpp:57
    return s;
}

// ---------------------------------------------------------------------------
// Textures (imageTexture.h, perlinTexture.h) and environment light
// ---------------------------------------------------------------------------
DEV f3 texel(const DevScene& S, const DevImage& im, int i, int j) {     // LDRImage.h:16-26
    const long long idx = (long long)im.channels * ((long long)i + (long long)j * im.width);
    const long long n = (long long)im.width * im.height * im.channels;
    const float* t = S.texels + im.offset;
    // linear indexing as in the reference (an x+1 read at the last column takes the next
    // row's first texel); reads outside the image, undefined in the reference, give 0
    return mk((idx >= 0 && idx < n) ? t[idx] : 0.f, (idx + 1 >= 0 && idx + 1 < n) ? t[idx + 1] : 0.f,
              (idx + 2 >= 0 && idx + 2 < n) ? t[idx + 2] : 0.f);
}

DEV f3 image_rgb(const DevScene& S, const DevTexture& tx, float u, float v) {   // imageTexture.h:60-73,111-133
    const DevImage im = S.images[GIDX(S, tx.image, S.num_images, 1)];
    if (tx.nearest) {
        int i = (int)(u * im.width);
        int j = (int)(v * im.height);
        i = (im.width - 1 < i) ? im.width - 1 : i;
        j = (im.height - 1 < j) ? im.height - 1 : j;
        return texel(S, im, i, j);
    }
    float fi = u * im.width, fj = v * im.height;
    float hiw = (float)(im.width - 1), hih = (float)(im.height - 1);
    fi = (hiw < fi) ? hiw : fi; fi = (fi < 0.0f) ? 0.0f : fi;          // std::max(lower, std::min(n, upper))
    fj = (hih < fj) ? hih : fj; fj = (fj < 0.0f) ? 0.0f : fj;
    float p = floorf(fi), q = floorf(fj);
    float dx = fi - p, dy = fj - q;
    float w1 = (1 - dx) * (1 - dy), w2 = dx * (1 - dy), w3 = (1 - dx) * dy, w4 = dx * dy;
    int ip = (int)p, iq = (int)q;
    return add(add(add(muls(texel(S, im, ip, iq), w1), muls(texel(S, im, ip + 1, iq), w2)),
                   muls(texel(S, im, ip, iq + 1), w3)), muls(texel(S, im, ip + 1, iq + 1), w4));
}


DEV double perlin_f(float x) {                                          // perlinTexture.h:153-160
    x = fabsf(x);
    if (x > 1) return 0;
    float xSqr = x * x;
    float xCube = xSqr * x;
    return (-6 * xCube * xSqr) + 15 * xCube * x - 10 * xCube + 1;
}
DEV float gdot(const float* grad, int g, float x, float y, float z) {
    return grad[3 * g] * x + grad[3 * g + 1] * y + grad[3 * g + 2] * z;
}
DEV float perlin(const DevScene& S, const DevTexture& tx, float x, float y, float z) {   // perlinTexture.h:57-123
    x *= tx.noise_scale; y *= tx.noise_scale; z *= tx.noise_scale;
    int X = (int)floorf(x), Y = (int)floorf(y), Z = (int)floorf(z);
    float dx = x - X, dy = y - Y, dz = z - Z;
    X = X & 255; Y = Y & 255; Z = Z & 255;
    const int* p = S.perm;
    const float* gr = S.grad;
    int ind0 = p[X + p[Y + p[Z]]] % 12;
    int ind1 = p[X + p[Y + p[Z + 1]]] % 12;
    int ind2 = p[X + p[Y + 1 + p[Z]]] % 12;
    int ind3 = p[X + p[Y + 1 + p[Z + 1]]] % 12;
    int ind4 = p[X + 1 + p[Y + p[Z]]] % 12;
    int ind5 = p[X + 1 + p[Y + p[Z + 1]]] % 12;
    int ind6 = p[X + 1 + p[Y + 1 + p[Z]]] % 12;
    int ind7 = p[X + 1 + p[Y + 1 + p[Z + 1]]] % 12;
    double c0 = gdot(gr, ind0, dx, dy, dz), c1 = gdot(gr, ind4, dx - 1, dy, dz), c2 = gdot(gr, ind2, dx, dy - 1, dz),
           c3 = gdot(gr, ind6, dx - 1, dy - 1, dz), c4 = gdot(gr, ind1, dx, dy, dz - 1), c5 = gdot(gr, ind5, dx - 1, dy, dz - 1),
           c6 = gdot(gr, ind3, dx, dy - 1, dz - 1), c7 = gdot(gr, ind7, dx - 1, dy - 1, dz - 1);
    double fdx = perlin_f(dx), fdy = perlin_f(dy), fdz = perlin_f(dz);
    double fdx1 = perlin_f(dx - 1), fdy1 = perlin_f(dy - 1), fdz1 = perlin_f(dz - 1);
    double w0 = fdx * fdy * fdz, w1 = fdx1 * fdy * fdz, w2 = fdx * fdy1 * fdz, w3 = fdx1 * fdy1 * fdz;
    double w4 = fdx * fdy * fdz1, w5 = fdx1 * fdy * fdz1, w6 = fdx * fdy1 * fdz1, w7 = fdx1 * fdy1 * fdz1;
    double total = w0 * c0 + w1 * c1 + w2 * c2 + w3 * c3 + w4 * c4 + w5 * c5 + w6 * c6 + w7 * c7;
    if (!tx.noise_abs) return (float)((total + 1) / 2.0f);
    return (float)fabs(total);
}

DEV f3 tex_rgb(const DevScene& S, const DevTexture& tx, float u, float v) {
    if (tx.kind == 1) return mk(180.f, 30.f, 180.f);                    // PerlinTexture::GetRGBSample
    return image_rgb(S, tx, u, v);
}

// ---------------------------------------------------------------------------
// Normal / bump mapping (mesh.cpp:263-358, sphere.cpp:116-193)
// ---------------------------------------------------------------------------
// GetTangentAndBitangentForTriangle (mesh.cpp:390-422)
DEV void tri_tangents(f3 vert0, f3 vert1, f3 vert2, float2 v0_uv, float2 v1_uv, float2 v2_uv, f3& tan, f3& bitan) {
    f3 e1 = makeUnit(sub(vert1, vert0));
    f3 e2 = makeUnit(sub(vert2, vert1));
    float v0u = tiledUV(v0_uv.x), v0v = tiledUV(v0_uv.y);
    float v1u = tiledUV(v1_uv.x), v1v = tiledUV(v1_uv.y);
    float v2u = tiledUV(v2_uv.x), v2v = tiledUV(v2_uv.y);
    float u1 = v1u - v0u, v1 = v1v - v0v;
    float u2 = v2u - v1u, v2 = v2v - v1v;
    float det = 1.0f / (u1 * v2 - v1 * u2);
    tan = mk(det * (v2 * e1.x - v1 * e2.x), det * (v2 * e1.y - v1 * e2.y), det * (v2 * e1.z - v1 * e2.z));
    const float nd = -det;
    bitan = mk(nd * u2 * e1.x + det * u1 * e2.x, nd * u2 * e1.y + det * u1 * e2.y, nd * u2 * e1.z + det * u1 * e2.z);
    tan = makeUnit(tan);
    bitan = makeUnit(bitan);
}
// GetTransformedNormal (helperMath.cpp:86-109): 3x3 double Matrix product, row by row
DEV f3 tbn_normal(f3 tan, f3 bitan, f3 normal, f3 sn) {
    double r0 = 0.0f, r1 = 0.0f, r2 = 0.0f;
    r0 += (double)tan.x * (double)sn.x; r0 += (double)bitan.x * (double)sn.y; r0 += (double)normal.x * (double)sn.z;
    r1 += (double)tan.y * (double)sn.x; r1 += (double)bitan.y * (double)sn.y; r1 += (double)normal.y * (double)sn.z;
    r2 += (double)tan.z * (double)sn.x; r2 += (double)bitan.z * (double)sn.y; r2 += (double)normal.z * (double)sn.z;
    return makeUnit(mk((float)r0, (float)r1, (float)r2));
}
// perlin bump: N minus the surface part of the height gradient (mesh.cpp:290-309, sphere.cpp:123-138)
DEV f3 perlin_bump(const DevScene& S, const DevTexture& bm, f3 N, f3 p, float bf, bool scaled) {
    const float eps = 0.001;
    float h0 = perlin(S, bm, p.x, p.y, p.z);
    float hxyz = scaled ? h0 * bf : h0;
    float gx = perlin(S, bm, p.x + eps, p.y, p.z), gy = perlin(S, bm, p.x, p.y + eps, p.z),
          gz = perlin(S, bm, p.x, p.y, p.z + eps);
    if (scaled) { gx = gx * bf; gy = gy * bf; gz = gz * bf; }
    f3 gradient = mk((gx - hxyz) / eps, (gy - hxyz) / eps, (gz - hxyz) / eps);
    f3 gParallel = muls(N, dot(gradient, N));
    f3 surfaceGradient = sub(gradient, gParallel);
    return makeUnit(sub(N, surfaceGradient));
}
// Normal of a mapped mesh face in the base mesh's object space, before its transform.
DEV f3 mesh_mapped_normal(const DevScene& S, const DevObject& ob, int face, f3 lp, float u, float v) {
    const f3 N = ld3(&S.face_n[face].x);
    const float4 a = S.tris[3 * face], b = S.face_v12[2 * face], c = S.face_v12[2 * face + 1];
    f3 tan, bitan;
    tri_tangents(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(c.x, c.y, c.z), S.face_uv[3 * face],
                 S.face_uv[3 * face + 1], S.face_uv[3 * face + 2], tan, bitan);
    if (ob.tex_normal >= 0) {                                            // mesh.cpp:263-272
        f3 sn = tex_rgb(S, S.textures[ob.tex_normal], u, v);
        sn = sub(divs(sn, 127.5f), mk(1, 1, 1));
        sn = makeUnit(sn);
        return tbn_normal(tan, bitan, N, sn);
    }
    const DevTexture& bm = S.textures[ob.tex_bump];
    if (bm.kind == 1) return perlin_bump(S, bm, N, lp, bm.bump_factor, true);
    // image bump map, forward differences (mesh.cpp:310-352)
    const DevImage im = S.images[bm.image];
    const float width = (float)im.width, height = (float)im.height;
    int i = (int)(u * (width - 1));
    int j = (int)(v * (height - 1));
    int nextI = i + 1, nextJ = j + 1;
    if ((float)i == width - 1) nextI = i;
    if ((float)j == height - 1) nextJ = j;
    f3 t0 = texel(S, im, i, j), tu = texel(S, im, nextI, j), tv = texel(S, im, i, nextJ);
    float h_uv = (t0.x + t0.y + t0.z) / 3.0f;                            // MakeGreyscale (mesh.cpp:195-197)
    float hDeltaU = (tu.x + tu.y + tu.z) / 3.0f;
    float hDeltaV = (tv.x + tv.y + tv.z) / 3.0f;
    const float bumpFactor = bm.bump_factor;
    f3 q_u = add(tan, muls(N, (hDeltaU - h_uv) * bumpFactor));
    f3 q_v = add(bitan, muls(N, (hDeltaV - h_uv) * bumpFactor));
    f3 nn = cross(q_v, q_u);
    f3 n = makeUnit(nn);
    if (nn.x * N.x <= 0 && nn.y * N.y <= 0 && nn.z * N.z <= 0) n = muls(n, -1.0f);
    else if (fabsf(nn.y - N.y) > 0.9f || fabsf(nn.x - N.x) > 0.9f || fabsf(nn.z - N.z) > 0.9f) n = muls(n, -1.0f);
    return n;
}
// Bumped sphere normal in local space (sphere.cpp:116-170, tangents sphere.cpp:181-193).
DEV f3 sphere_bumped_normal(const DevScene& S, const DevObject& ob, f3 p, float phi, float theta, float u, float v) {
    const float radius = ob.center[3];
    f3 tan = mk((float)(2 * RT_PI * (double)p.z), 0.0f, (float)(-2 * RT_PI * (double)p.x));
    f3 bitan = mk((float)(RT_PI * (double)p.y * (double)cosf(phi)),
                  (float)((double)(-radius) * RT_PI * (double)sinf(theta)),
                  (float)(RT_PI * (double)p.y * (double)sinf(phi)));
    tan = makeUnit(tan);
    bitan = makeUnit(bitan);
    const f3 N = makeUnit(cross(bitan, tan));
    const DevTexture& bm = S.textures[ob.tex_bump];
    if (bm.kind == 1) return perlin_bump(S, bm, N, p, 1.0f, false);
    const DevImage im = S.images[bm.image];
    int i = (int)(u * (float)im.width);
    int j = (int)(v * (float)im.height);
    const float normalizer = bm.normalizer, bumpFactor = bm.bump_factor;
    f3 c1 = divs(texel(S, im, i + 1, j), normalizer), c0 = divs(texel(S, im, i, j), normalizer),
       c2 = divs(texel(S, im, i, j + 1), normalizer);
    float h1 = (c1.x + c1.y + c1.z) * bumpFactor;                        // MakeGreyscale (sphere.cpp:9-11)
    float h_uv = (c0.x + c0.y + c0.z) * bumpFactor;
    float h2 = (c2.x + c2.y + c2.z) * bumpFactor;
    f3 q_u = add(tan, muls(N, h1 - h_uv));
    f3 q_v = add(bitan, muls(N, h2 - h_uv));
    return makeUnit(cross(q_v, q_u));
}

// SphericalEnvironmentLight::GetSample (sphericalEnvironmentLight.h:22-34)
DEV f3 env_sample(const DevScene& S, int e, f3 dir) {
    const DevImage im = S.images[S.env_images[e]];
    float u = (float)((1 + (atan2f(dir.x, -dir.z) / RT_PI)) / 2.0f);
    float v = (float)(acosf(dir.y) / RT_PI);
    int i = (int)(im.width * u);
    int j = (int)(im.height * v);
    return muls(muls(texel(S, im, i, j), (float)2), (float)RT_PI);
}

// GetDirection (sphericalEnvironmentLight.h:36-61): rejection sampling, returns the
// un-normalised candidate.  The reference spins forever on a NaN normal; bounded here.
// The draws are rnd(key, RP_ENV, e * 16384 + 3k + c); the inner hash of (purpose, index) does
// not depend on the key, so it comes from a table (S.env_mix, kEnvDraws per light, built by
// rtg_scene_create with the same mix64): one 64-bit hash per draw instead of two, the same bits.
// A wave runs until its last lane accepts (~17 candidates for 64 lanes at acceptance pi/12),
// and the table index is the loop counter, so the loads are scalar.
static_assert(RP_ENV == kRpEnv, "env_mix table purpose");
DEV float rnd_mixed(uint64_t key, uint64_t inner) {
    const uint64_t h = mix64(key ^ inner);
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}
DEV f3 env_direction(const DevScene& S, f3 surfaceNormal, uint64_t key, int e) {
    f3 n = makeUnit(surfaceNormal);
    f3 cand = mk(0, 0, 0);
    const unsigned long long* T = S.env_mix + (size_t)e * kEnvDraws;
    for (uint32_t k = 0; k < 4096; ++k) {
        cand.x = 2.0f * rnd_mixed(key, T[3 * k]) - 1.0f;
        cand.y = 2.0f * rnd_mixed(key, T[3 * k + 1]) - 1.0f;
        cand.z = 2.0f * rnd_mixed(key, T[3 * k + 2]) - 1.0f;
        float length = len(cand);
        if (length <= 1.0f && dot(n, cand) > 0.0f) break;
    }
    return cand;
}

// The same search for a whole wave (every lane calls it; `want`: the lane needs a direction).
// A lane's loop runs until its first accepted candidate (3.8 on average at acceptance pi/12),
// but the wave's until its last lane's (~17 for 64 lanes); here the lanes still searching get
// the others' help: with na of them, each gets g = 64 / na lanes testing its candidates
// k .. k+g-1 at once, and takes the smallest accepted index -- the candidate its own loop
// returns (the first accepted of 0..4095, else the 4095th), computed by the same operations.
DEV f3 env_candidate(const unsigned long long* T, uint64_t key, int k) {
    return mk(2.0f * rnd_mixed(key, T[3 * k]) - 1.0f, 2.0f * rnd_mixed(key, T[3 * k + 1]) - 1.0f,
              2.0f * rnd_mixed(key, T[3 * k + 2]) - 1.0f);
}
// position of the r-th (from 0) set bit of m (r < popcount(m))
DEV int nth_set_bit(uint64_t m, int r) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t lo = m & ((1ull << w) - 1ull);
        const int c = __popcll(lo);
        const bool up = r >= c;
        r = up ? r - c : r;
        m = up ? m >> w : lo;
        pos = up ? pos + w : pos;
    }
    return pos;
}
DEV f3 env_direction_wave(const DevScene& S, f3 surfaceNormal, uint64_t key, int e, bool want) {
    const f3 n = makeUnit(surfaceNormal);
    const unsigned long long* T = S.env_mix + (size_t)e * kEnvDraws;
    const int lane = threadIdx.x & 63;
    int k = 0;
    bool done = !want;
    f3 cand = mk(0, 0, 0);
    for (;;) {
        const uint64_t act = __ballot(!done);
        if (!act) break;
        const int na = __popcll(act);
        const int g = 64 / na;
        if (g == 1) {                  // more than 32 searching: each tests its own next candidate
            if (!done) {
                const f3 c = env_candidate(T, key, k);
                if ((len(c) <= 1.0f && dot(n, c) > 0.0f) || ++k >= 4096) {
                    cand = c;
                    done = true;
                }
            }
            continue;
        }
        const int r = lane / g;                            // the searcher this lane helps
        const bool helper = r < na;
        const int owner = helper ? nth_set_bit(act, r) : lane;
        const uint64_t okey = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(key >> 32), owner) << 32) |
                              (uint32_t)__shfl((int)(uint32_t)key, owner);
        const f3 on = mk(__shfl(n.x, owner), __shfl(n.y, owner), __shfl(n.z, owner));
        const int kk = __shfl(k, owner) + (lane - r * g);
        f3 c = mk(0, 0, 0);
        bool acc = false;
        if (helper && kk < 4096) {
            c = env_candidate(T, okey, kk);
            acc = len(c) <= 1.0f && dot(on, c) > 0.0f;
        }
        const uint64_t am = __ballot(acc);
        const int rank = __popcll(act & ((1ull << lane) - 1ull));
        const uint64_t mine = done ? 0ull : (am >> (rank * g)) & (g >= 64 ? ~0ull : (1ull << g) - 1ull);
        const int src = mine ? rank * g + __ffsll((long long)mine) - 1 : lane;
        const f3 w = mk(__shfl(c.x, src), __shfl(c.y, src), __shfl(c.z, src));
        if (!done) {
            if (mine) {
                cand = w;
                done = true;
            } else if ((k += g) >= 4096) {
                cand = env_candidate(T, key, 4095);
                done = true;
            }
        }
    }
    return cand;
}

// ---------------------------------------------------------------------------
// BRDFs (brdf*.cpp) and Shade (raytracer.cpp:192-206, 478-554)
// ---------------------------------------------------------------------------
DEV f3 brdf_apply(const DevBrdf& B, float refrIdx, f3 kd, f3 ks, f3 w_i, f3 w_o, f3 normal) {
    const float th = (float)angleBetween(w_i, normal);
    const double ex = (double)B.exponent;
    switch (B.type) {
        case 0: {                                                       // brdfPhong.cpp:11-20
            if (th >= 90.0f || th < 0) return mk(0, 0, 0);
            f3 r = makeUnit(sub(muls(muls(normal, 2.0f), dot(normal, w_i)), w_i));
            double angleR = angleBetween(r, w_o);
            return add(kd, muls(ks, (float)(pow(cosDeg(angleR), ex) / cosDeg(th))));
        }
        case 1: {                                                       // brdfBlinnPhong.cpp:11-20
            if (th >= 90.0f) return mk(0, 0, 0);
            f3 half = divs(add(w_i, w_o), len(add(w_i, w_o)));
            double a = angleBetween(half, normal);
            return add(kd, muls(ks, (float)(pow(cosDeg(a), ex) / cosDeg(th))));
        }
        case 2: {                                                       // brdfModifiedPhong.cpp:14-33
            if (th >= 90.0f || th < 0) return mk(0, 0, 0);
            f3 r = makeUnit(sub(muls(muls(normal, 2.0f), dot(normal, w_i)), w_i));
            double angleR = angleBetween(r, w_o);
            if (B.energy_conserving) {
                f3 kdTerm = muls(kd, (float)(1.0f / RT_PI));
                double ksCons = (B.exponent + 2) / (2 * RT_PI);
                double cosTerm = pow(cosDeg(angleR), ex);
                return add(kdTerm, muls(ks, (float)(ksCons * cosTerm)));
            }
            return add(kd, muls(ks, (float)pow(cosDeg(angleR), ex)));
        }
        case 3: {                                                       // brdfModifiedBlinnPhong.cpp:11-29
            if (th >= 90.0f) return mk(0, 0, 0);
            f3 half = divs(add(w_i, w_o), len(add(w_i, w_o)));
            double a = angleBetween(half, normal);
            if (B.energy_conserving) {
                f3 kdTerm = muls(kd, (float)(1.0f / RT_PI));
                double ksCons = (B.exponent + 8) / (8 * RT_PI);
                double cosTerm = pow(cosDeg(a), ex);
                return add(kdTerm, muls(ks, (float)(ksCons * cosTerm)));
            }
            return add(kd, muls(ks, (float)pow(cosDeg(a), ex)));
        }
        default: {                                                      // brdfTorranceSparrow.cpp:15-59
            if (th >= 90.0f) return mk(0, 0, 0);
            f3 half = divs(add(w_i, w_o), len(add(w_i, w_o)));
            double cosAlpha = dot(half, normal);
            double d = (ex + 2) * pow(cosAlpha, ex) / (2 * RT_PI);
            double cosbeta = dot(half, w_o), n = refrIdx;
            double r0 = pow(n - 1, 2.0) / pow(n + 1, 2.0);
            double f = r0 + (1.0 - r0) * pow((1.0 - cosbeta), 5.0);
            double ndoth = dot(normal, half), ndotwo = dot(normal, w_o), ndotwi = dot(normal, w_i), wodoth = dot(w_o, half);
            double ga = 2.0f * ndoth * ndotwo / wodoth, gb = 2.0 * ndoth * ndotwi / wodoth;
            double gm = (gb < ga) ? gb : ga;
            double g = (gm < 1.0) ? gm : 1.0;
            double kdCoeff = (1.0f / RT_PI);
            if (B.kd_fresnel) kdCoeff *= (1 - f);
            f3 kdTerm = muls(kd, (float)kdCoeff);
            double costheta = dot(normal, w_i), cosphi = dot(normal, w_o);
            f3 ksTerm = muls(ks, (float)((d * f * g) / (4 * costheta * cosphi)));
            return add(kdTerm, ksTerm);
        }
    }
}

struct ShadeCtx {
    const DevObject* ob;
    const DevMaterial* mat;
    Surf s;
};

template <bool TEX = true>
DEV f3 kd_coeff(const DevScene& S, const ShadeCtx& c) {                // raytracer.cpp:478-508
    f3 refl = ld3(c.mat->diffuse);
    if (TEX && c.ob->tex_diffuse >= 0) {
        const DevTexture tx = S.textures[GIDX(S, c.ob->tex_diffuse, S.num_textures, 2)];
        f3 t;
        if (tx.kind == 1) { float p = perlin(S, tx, c.s.p.x, c.s.p.y, c.s.p.z); t = mk(p, p, p); }
        else t = divs(image_rgb(S, tx, c.s.u, c.s.v), 255.0f);
        refl = tx.blend ? divs(add(t, ld3(c.mat->diffuse)), 2.0f) : t;
    }
    return refl;
}
template <bool TEX = true>
DEV f3 ks_coeff(const DevScene& S, const ShadeCtx& c) {                // raytracer.cpp:509-539 (reads diffuseTex)
    f3 refl = ld3(c.mat->specular);
    if (TEX && c.ob->tex_specular >= 0 && c.ob->tex_diffuse >= 0) {
        const DevTexture tx = S.textures[GIDX(S, c.ob->tex_diffuse, S.num_textures, 2)];
        f3 t;
        if (tx.kind == 1) { float p = perlin(S, tx, c.s.p.x, c.s.p.y, c.s.p.z); t = mk(p, p, p); }
        else t = divs(image_rgb(S, tx, c.s.u, c.s.v), 255.0f);
        refl = tx.blend ? divs(add(t, ld3(c.mat->diffuse)), 2.0f) : t;
    }
    return refl;
}

// Shade (raytracer.cpp:192-206).  TP: also ray.throughput *= brdf (:202), which Russian
// roulette reads (path tracing only).
template <bool TP = false, int SK = SK_ALL>
DEV f3 shade(const DevScene& S, const ShadeCtx& c, f3 w_i, f3 w_o, f3 Li, f3* tp = nullptr) {
    constexpr bool TEX = (SK & SK_TEX) != 0;
    if ((SK & SK_BRDF) && c.mat->brdf >= 0) {
        float costheta_i = fmax0(dot(w_i, c.s.n));
        f3 kd = kd_coeff<TEX>(S, c), ks = ks_coeff<TEX>(S, c);
        f3 res = brdf_apply(S.brdfs[c.mat->brdf], c.mat->refractive_index, kd, ks, w_i, w_o, c.s.n);
        if (TP) *tp = mulv(*tp, res);
        return muls(mulv(res, Li), costheta_i);
    }
    f3 kd = kd_coeff<TEX>(S, c);                                        // GetDiffuse
    float costheta = fmax0(dot(w_i, c.s.n));
    f3 diff = muls(mulv(kd, Li), costheta);
    f3 ks = ks_coeff<TEX>(S, c);                                        // GetSpecular
    f3 half = divs(add(w_i, w_o), len(add(w_i, w_o)));
    float cosAlpha = fmax0(dot(c.s.n, half));
    f3 spec = muls(mulv(ks, Li), powf(cosAlpha, c.mat->phong_exponent));
    return add(diff, spec);
}

// IsInShadow (raytracer.cpp:567-584); IsInShadowDirectional (:555-566)
template <bool STATS>
DEV bool in_shadow(const DevScene& S, f3 p, f3 n, f3 lightPos, float mbTime, Cnt<STATS>& c) {
    f3 dir = sub(lightPos, p);
    float lightT = len(dir);
    Ray sr;
    sr.d = divs(dir, lightT);
    sr.o = add(p, muls(n, S.eps));
    Hit h;
    c.shd();
    return trace<true, STATS>(S, sr, mbTime, lightT + 0.01f, lightT, h, c);
}
template <bool STATS>
DEV bool in_shadow_dir(const DevScene& S, f3 p, f3 n, f3 lightDir, float mbTime, Cnt<STATS>& c) {
    Ray sr;
    sr.d = neg(lightDir);
    sr.o = add(p, muls(n, S.eps));
    Hit h;
    c.shd();
    return trace<true, STATS>(S, sr, mbTime, INFINITY, INFINITY, h, c);
}

// One light of SampleDirectLighting (raytracer.cpp:701-805), slots in the reference's
// type order point, area, env, dir, spot: the incident direction, the irradiance and,
// where the reference casts one, the shadow ray (IsInShadow :567-584 /
// IsInShadowDirectional :555-566).
// MeshLight::getSample (meshLight.h:27-47) and the irradiance of SampleDirectLighting's
// mesh-light branch (raytracer.cpp:780-803: radiance * weight * 2 * M_PI, no distance
// term).  The reference draws the face from uniform_int_distribution(0, faceCount) --
// inclusive, so 1 draw in faceCount+1 indexes past the face vector (undefined); here the
// face is uniform over the faceCount faces.
DEV void mesh_light_sample(const DevScene& S, int l, uint64_t key, f3& pos, f3& E) {
    const DevMeshLight& L = S.mesh_lights[l];
    int k = (int)(rndd(key, RP_MESHLIGHT, 3 * l) * L.face_count);
    k = k < L.face_count ? k : L.face_count - 1;
    const DevLightFace& F = S.light_faces[L.face_begin + k];
    const double selectionWeight = F.area / L.surface_area;
    const double rand1 = rndd(key, RP_MESHLIGHT, 3 * l + 1);
    const double rand2 = rndd(key, RP_MESHLIGHT, 3 * l + 2);
    const f3 a = ld3(F.v0), b = ld3(F.v1), c = ld3(F.v2);
    f3 q = add(muls(b, (float)(1 - rand2)), muls(c, (float)rand2));
    pos = add(muls(a, (float)(1 - sqrt(rand1))), muls(q, (float)sqrt(rand1)));
    pos = xform(L.xf, pos, 1.0f);                                      // ApplyTransformToPoint(transform)
    E = muls(muls(muls(ld3(L.radiance), (float)selectionWeight), 2.0f), (float)RT_PI);
}

struct LightSample {
    f3 w_i, E;
    bool shadow;
    bool skip;         // mesh light hit by this node's GI ray (raytracer.cpp:784): no term
    Ray sr;
    float minT, limit;
};
// SK without SK_XLIGHT: the scene has no env / spot / mesh lights (their code is left out).
template <int SK = SK_ALL>
DEV LightSample light_sample(const DevScene& S, int slot, f3 p, f3 n, uint64_t key, int skipId = -1) {
    LightSample ls;
    ls.shadow = true;
    ls.skip = false;
    ls.sr.o = add(p, muls(n, S.eps));
    f3 lpos = mk(0, 0, 0);
    bool positional = true;
    int i = slot;
    constexpr bool XL = (SK & SK_XLIGHT) != 0;
    if (i < S.num_point) {
        const f3 lp = ld3(S.point_lights[i].pos);
        lpos = lp;
        ls.w_i = makeUnit(sub(lp, p));
        float dist = len(sub(lp, p));
        ls.E = divs(ld3(S.point_lights[i].intensity), dist * dist);
    } else if ((i -= S.num_point) < S.num_area) {
        const DevAreaLight& L = S.area_lights[i];
        float offU = rnd(key, RP_AREA, 2 * i) - 0.5f;                     // areaLight.h:34-41
        float offV = rnd(key, RP_AREA, 2 * i + 1) - 0.5f;
        f3 sp = add(add(ld3(L.pos), muls(ld3(L.u), L.extent * offU)), muls(ld3(L.v), L.extent * offV));
        lpos = sp;
        f3 w_i = sub(sp, p);
        float dist = len(w_i);
        float dSqr = dist * dist;
        w_i = divs(w_i, dist);
        float lc = dot(ld3(L.normal), neg(w_i));
        if (lc < 0) lc = dot(ld3(L.normal), w_i);
        ls.w_i = w_i;
        ls.E = muls(ld3(L.radiance), L.area * lc / dSqr);
    } else if (XL && (i -= S.num_area) < S.num_env) {                     // no shadow ray (:741-755)
        f3 sd = env_direction(S, n, key, i);
        ls.E = env_sample(S, i, sd);
        ls.w_i = n;
        ls.shadow = false;
    } else if (!XL || (i -= S.num_env) < S.num_dir) {
        if (!XL) i -= S.num_area;
        const f3 ldir = ld3(S.dir_lights[i].dir);
        ls.w_i = neg(ldir);
        ls.E = ld3(S.dir_lights[i].radiance);
        ls.sr.d = neg(ldir);
        ls.minT = INFINITY;
        ls.limit = INFINITY;
        positional = false;
    } else if ((i -= S.num_dir) >= S.num_spot) {
        i -= S.num_spot;                                                // mesh lights (:780-803)
        ls.skip = S.mesh_lights[i].id == skipId;
        f3 sp, E;
        mesh_light_sample(S, i, key, sp, E);
        lpos = sp;
        f3 w_i = sub(sp, p);
        float dist = len(w_i);
        ls.w_i = divs(w_i, dist);
        ls.E = E;
    } else {
        const DevSpotLight& L = S.spot_lights[i];
        const f3 lp = ld3(L.pos);
        lpos = lp;
        ls.w_i = makeUnit(sub(lp, p));
        // SpotLight::GetIrradiance (spotLight.h:33-57)
        float distToPoint = len(sub(p, lp));
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
                double sv = pow((cosAlpha - L.cos_half_coverage) / (L.cos_half_falloff - L.cos_half_coverage), (double)4.0f);
                E = muls(E, (float)sv);
            }
        }
        ls.E = E;
    }
    if (ls.shadow && positional) {
        f3 dir = sub(lpos, p);
        float lightT = len(dir);
        ls.sr.d = divs(dir, lightT);
        ls.minT = lightT + 0.01f;
        ls.limit = lightT;
    }
    return ls;
}

// SampleDirectLighting (raytracer.cpp:701-805): the unshadowed lights' Shade terms summed in
// slot order.  One trace and one Shade call site for all light types (the BRDF code and the
// traversal are inlined once).
// TP / skipId: path tracing -- throughput update per Shade, and the mesh light the node's
// GI ray hit is not sampled (raytracer.cpp:92,784).
// SK / FEAT: shading and traversal features the scene may use (the path tracer's variants).
template <bool STATS, bool TP = false, int SK = SK_ALL, int FEAT = FEAT_ALL>
DEV f3 direct(const DevScene& S, const ShadeCtx& c, f3 w_o, float mbTime, uint64_t key, Cnt<STATS>& cn,
              int skipId = -1, f3* tp = nullptr) {
    f3 color = mk(0, 0, 0);
    const f3 p = c.s.p, n = c.s.n;
    const int nslots = S.num_point + S.num_area + S.num_env + S.num_dir + S.num_spot + S.num_mesh;
    for (int l = 0; l < nslots; ++l) {
        LightSample ls = light_sample<SK>(S, l, p, n, key, skipId);
        if (ls.skip) continue;
        if (ls.shadow) {
            Hit h;
            cn.shd();
            if (trace<true, STATS, FEAT>(S, ls.sr, mbTime, ls.minT, ls.limit, h, cn)) continue;
        }
        color = add(color, shade<TP, SK>(S, c, ls.w_i, w_o, ls.E, tp));
    }
    return color;
}

// Raytracer::Reflect (raytracer.cpp:424-440)
DEV f3 reflect(f3 normal, f3 w_o, float roughness, uint64_t key, uint32_t purpose) {
    f3 r = makeUnit(sub(muls(muls(normal, 2.0f), dot(normal, w_o)), w_o));
    if (roughness > 0.001) {
        f3 u, v;
        onb(r, u, v);
        float psi1 = rnd(key, purpose, 0) - 0.5f;
        float psi2 = rnd(key, purpose, 1) - 0.5f;
        return makeUnit(add(r, muls(add(muls(u, psi1), muls(v, psi2)), roughness)));
    }
    return r;
}

DEV f3 beer(float x, const float* c, f3 L0) {                          // raytracer.cpp:416-423
    return mk(L0.x * expf(-c[0] * x), L0.y * expf(-c[1] * x), L0.z * expf(-c[2] * x));
}


// GenerateRay (raytracer.cpp:661-699) + Camera::GetImagePlanePosition (camera.cpp:74-80)
DEV Ray camera_ray(const DevCamera& C, int px, int py, uint64_t key, float& mbTime) {
    const f3 q = ld3(C.q), right = ld3(C.right), up = ld3(C.up), cpos = ld3(C.pos);
    float su = (float)((px + 0.5) * (double)(C.right_ext - C.left) / C.width);
    float sv = (float)((py + 0.5) * (double)(C.top - C.bottom) / C.height);
    f3 ipp = add(add(q, muls(right, su)), muls(up, -sv));
    Ray ray;
    ray.o = cpos;
    if (C.aperture > 0.0001) {
        f3 aps = ray.o;
        float first01 = 2.0f * rnd(key, RP_DOF, 0) - 1.0f;
        aps = add(aps, muls(up, first01 * C.aperture * 0.5f));
        float second01 = 2.0f * rnd(key, RP_DOF, 1) - 1.0f;
        aps = add(aps, muls(right, second01 * C.aperture * 0.5f));
        f3 dir = makeUnit(sub(ray.o, ipp));
        float tFd = C.focus_distance / dot(dir, ld3(C.gaze));
        f3 bent = add(ray.o, muls(dir, tFd));
        ray.d = makeUnit(sub(bent, aps));
        ray.o = aps;
    } else {
        ray.d = makeUnit(sub(ipp, ray.o));
    }
    mbTime = rnd(key, RP_MOTION, 0);
    return ray;
}

// PerPixel miss branch (raytracer.cpp:49-62)
template <int SK = SK_ALL>
DEV f3 miss_color(const DevScene& S, const DevCamera& C, int px, int py, f3 dir) {
    if ((SK & SK_TEX) && S.bg_texture >= 0) {
        float u = px / (float)C.width, v = py / (float)C.height;
        return tex_rgb(S, S.textures[S.bg_texture], u, v);
    }
    if ((SK & SK_XLIGHT) && S.num_env > 0) return env_sample(S, 0, dir);
    return mk((float)S.background[0], (float)S.background[1], (float)S.background[2]);
}

// Gaussian2D (gaussian.h:3-21) with sigma = 1/6 pixel
DEV float gauss_weight(float x, float y) {
    const float sigma = 1.0f / 6.0f;
    const float sigmaSqr = sigma * sigma;
    const float c1 = (float)(1.0f / (2.0f * RT_PI * sigmaSqr));
    float exponent = (float)(-0.5 * ((x * x + y * y) / sigmaSqr));
    return c1 * expf(exponent);
}

// renderThreadMain's stratified jitter (main.cpp:66-76) feeds only the Gaussian weight;
// samples beyond nRows*nCols keep (0,0) (the reused `samples` vector, main.cpp:47).
DEV float sample_weight(int spp, int s, uint64_t key) {
    const int nRows = (int)sqrt((double)spp);
    const int nCols = nRows;
    float sx = 0.f, sy = 0.f;
    if (s < nRows * nCols) {
        const int row = s / nCols, col = s % nCols;
        float psi1 = rnd(key, RP_JITTER, 0), psi2 = rnd(key, RP_JITTER, 1);
        sx = (col + psi1) / nCols;
        sy = (row + psi2) / nRows;
    }
    return gauss_weight(sx - 0.5f, sy - 0.5f);
}

// x86 cvttss2si + clamp (helperMath.cpp:140-152): out-of-range and NaN give INT_MIN -> 0
DEV unsigned char ldr(float c) {
    int i = (c > -2147483904.0f && c < 2147483648.0f) ? (int)c : (int)0x80000000;
    return (unsigned char)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

// The end of a multi-sample pass for one pixel (RenderParams::slabs): its colours of samples
// sample0, sample0 + 1, ... (col[j * stride]) added to the accumulator one after the other with
// the Gaussian sample weights -- the operations, in the order, of one-sample passes
// (renderThreadMain's spp loop, main.cpp:80-121) -- and after the frame's last sample the pixel
// itself.  first: the pass starts the render's accumulation.
DEV void accum_samples(const DevCamera& C, const RenderParams& P, int sample0, int nslab, bool first, bool last,
                       int pixel, const float4* __restrict__ col, size_t stride, float4* __restrict__ accum,
                       float* __restrict__ hdr, unsigned char* __restrict__ ldrOut) {
    float4 a = first ? make_float4(0.f, 0.f, 0.f, 0.f) : accum[pixel];
    for (int j = 0; j < nslab; ++j) {
        const float4 c = col[j * stride];
        const int s = sample0 + j;
        const float gw = sample_weight(C.spp, s, root_key(P.seed, pixel, s));
        a.x += c.x * gw;
        a.y += c.y * gw;
        a.z += c.z * gw;
        a.w += gw;
    }
    accum[pixel] = a;
    if (last && !P.accum_only) {
        const size_t idx = 3 * (size_t)pixel;
        const float r = a.x / a.w, g = a.y / a.w, b = a.z / a.w;
        if (hdr) { hdr[idx] = r; hdr[idx + 1] = g; hdr[idx + 2] = b; }
        if (ldrOut) { ldrOut[idx] = ldr(r); ldrOut[idx + 1] = ldr(g); ldrOut[idx + 2] = ldr(b); }
    }
}

// 16x16-pixel tile per 256-thread block, 8x8 per wave; tiles dealt so that consecutive
// tiles share an XCD (blocks b and b+8 share one under round-robin dispatch).
// Image row of compact row `crow` of this render's part (RenderParams): compact rows are
// the part's 8-row bands in order.
// Band kb of part p of N is band kb * N + ((p - kb) mod N) of the row range (rtgpu.h
// RTG_PART_BAND_ROWS: round-robin, rotated by one slot per round).
DEV int part_row(const RenderParams& P, int crow) {
    const int kb = crow >> 3;
    int slot = (P.part_index - kb) % P.part_count;
    if (slot < 0) slot += P.part_count;
    return P.row_begin + ((kb * P.part_count + slot) << 3) + (crow & 7);
}
// Image pixel of compact pixel index i (= crow * width + x).
DEV int part_pixel(const RenderParams& P, int width, int i) {
    const int crow = i / width;
    return part_row(P, crow) * width + (i - crow * width);
}

// The ray trees' level-0 order (rtg_tree.hip): compact index i -> image pixel in 8x8 tiles
// (8-row bands of the part, each band's 8-column chunks in order; a band of fewer rows or a
// last chunk of fewer columns keeps its pixels in row-major order), so a wave's 64 camera rays
// -- and, through the per-block ordered child appends, their reflected and refracted rays --
// come from one 8x8 block of the image instead of a 64-pixel strip of a row.  A bijection of
// [0, width * part_rows) onto the part's pixels.  RTG_TREE_TILES=0: row-major (part_pixel).
DEV int tree_pixel(const RenderParams& P, int width, int i) {
    const int band = i / (8 * width), j = i - band * 8 * width;
    const int rb = min(8, P.part_rows - 8 * band);        // rows of this band
    const int fc = width >> 3, full = fc * 8 * rb;         // pixels in whole 8-column chunks
    int x, y;
    if (j < full) {
        const int c = j / (8 * rb), k = j - c * 8 * rb;
        x = 8 * c + (k & 7);
        y = k >> 3;
    } else {
        const int rw = width & 7, k = j - full;
        x = 8 * fc + k % rw;
        y = k / rw;
    }
    return part_row(P, 8 * band + y) * width + x;
}

// tile_pixel also returns the compact row and the block's sample slab (multi-sample passes,
// RenderParams::slabs): the pixel's work-buffer entry is slab * slab_px + crow * width + px
// (work_index).  A padding block of a slab (its index past num_tiles) holds no pixel: px is
// past every image width.
DEV void tile_pixel(const RenderParams& P, int& px, int& py, int& crow, int& slab) {
    slab = (int)(blockIdx.x / (unsigned)P.slab_tiles);
    const int b = (int)blockIdx.x - slab * P.slab_tiles;
    if (b >= P.num_tiles) {
        px = 1 << 24;
        crow = 0;
        py = P.row_end;
        return;
    }
    const int tile = P.tile_map[b];
    const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    px = tx * 16 + (w & 1) * 8 + (l & 7);
    crow = ty * 16 + (w >> 1) * 8 + (l >> 3);
    py = part_row(P, crow);
}
DEV void tile_pixel(const RenderParams& P, int& px, int& py) {
    int crow, slab;
    tile_pixel(P, px, py, crow, slab);
}
DEV int work_index(const RenderParams& P, int width, int slab, int crow, int px) {
    return slab * P.slab_px + crow * width + px;
}
// The image pixel of work-buffer entry i of sample slab `slab` (inverse of work_index).
DEV int work_pixel(const RenderParams& P, int width, int slab, int i) {
    const int r = i - slab * P.slab_px, crow = r / width;
    return part_row(P, crow) * width + (r - crow * width);
}

template <bool STATS>
DEV void flush_counters(Cnt<STATS>& cn, DevCounters* counters) {
    if constexpr (STATS) {
        unsigned long long v[13] = {cn.cams, cn.secs, cn.shds, cn.nodes, cn.tris, cn.sphs, cn.objs, cn.snodes, cn.stris,
                                    cn.wnodes, cn.fallbacks, cn.ewnodes, cn.efallbacks};
        for (int k = 0; k < 13; ++k) {
            unsigned long long x = v[k];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            if ((threadIdx.x & 63) == 0 && x) atomicAdd(&((unsigned long long*)counters)[k], x);
        }
    }
}

// Shadow queue in per-block segments (rtg_wave.hip k_shade, rtg_tree.hip k_tree_shade):
// one thread per queued shadow ray, CastShadowRay (raytracer.cpp:585-623).
// FAST (the wavefront pipeline): the RTG_SHADOW_MODE walk, its undecided rays by the
// reference walk in place (moving them to a second kernel to shed the reference walk's
// registers measured slower: the extra launch and the wide walk's own ~100 VGPRs); otherwise
// (the ray-tree pipeline, or RTG_RENDER_EXACT_SHADOW) the reference walk per lane,
// early-exit any-hit.
// grid (shade blocks, slots): block (b, c) takes entries [256c, 256c+256) of segment b
// CastShadowRay's answer for queue entry q (origin + initial minT o, direction + limit d).
// DEFER (large-leaf scenes, fast walk): the any-hit walk may queue large leaves; a ray with no
// answer of its own but queued leaves is pending (k_bigleaf_any, k_shadow_fin decide it)
enum : int { SS_PENDING = 1, SS_OCC = 2, SS_UNDECIDED = 4 };
template <bool STATS, int FEAT>
DEV int shadow_state_defer(const DevScene& S, const WaveBufs& W, size_t q, float4 o, float4 d, Cnt<STATS>& cn) {
    Ray r;
    r.o = mk(o.x, o.y, o.z);
    r.d = mk(d.x, d.y, d.z);
    AnyDefer ad{W.dq_e, W.dq_count + 2, W.dq_cap, (int)q, false};
    int res = trace_any_wide<STATS, FEAT, true>(S, r, o.w, d.w, cn, &ad);
    if (res < 0) {                                   // undecided: the reference walk (queued leaves moot)
        cn.fallback();
        Hit h;
        res = trace<true, STATS, FEAT>(S, r, 0.f, o.w, d.w, h, cn) ? 1 : 0;
    } else if (res == 0 && ad.deferred) {
        return SS_PENDING;
    }
    return res > 0 ? SS_OCC : 0;
}
template <bool STATS, int FEAT, bool FAST>
DEV bool shadow_occluded(const DevScene& S, const WaveBufs& W, size_t q, float4 o, float4 d, Cnt<STATS>& cn) {
    Ray r;
    r.o = mk(o.x, o.y, o.z);
    r.d = mk(d.x, d.y, d.z);
    int res = -1;
    if constexpr (FAST) {
        res = trace_any_wide<STATS, FEAT>(S, r, o.w, d.w, cn);
        if (res < 0) {                               // undecided: the reference walk
            cn.fallback();
            Hit h;
            res = trace<true, STATS, FEAT>(S, r, 0.f, o.w, d.w, h, cn) ? 1 : 0;
        }
    } else {
        Hit h;
        res = trace<true, STATS, FEAT>(S, r, 0.f, o.w, d.w, h, cn) ? 1 : 0;
    }
    return res > 0;
}

template <bool STATS, int FEAT, bool FAST, bool DEFER = false>
__global__ __launch_bounds__(256, FAST ? RTG_WIDE_WAVES(FEAT) : RTG_TRACE_WAVES(FEAT)) void k_shadow(
    const DevScene S, const WaveBufs W, DevCounters* counters) {
    const int k = blockIdx.y * 256 + threadIdx.x;
    const size_t q = ((size_t)blockIdx.x * W.num_slots) * 256 + k;
    Cnt<STATS> cn;
    if (k < W.q_count[blockIdx.x]) {
        if constexpr (DEFER) {
            const int st = shadow_state_defer<STATS, FEAT>(S, W, q, W.q_o[q], W.q_d[q], cn);
            W.shadow_state[q] = st;
            if (st == SS_OCC) W.occ[W.q_slot[q]] = 1;
        } else if (shadow_occluded<STATS, FEAT, FAST>(S, W, q, W.q_o[q], W.q_d[q], cn)) {
            W.occ[W.q_slot[q]] = 1;
        }
    }
    flush_counters<STATS>(cn, counters);
}

// The shadow rays' queued large leaves: one wave per entry, each lane taking entries (face
// records of the any-hit tree) 64 apart and the exact decisions of walk_wide_any on each --
// a sufficient face (the leaf box passes at limit) occludes, a face reaching only at minT0
// leaves the ray undecided -- OR-ed into the ray's state.
template <int FEAT>
__global__ __launch_bounds__(256) void k_bigleaf_any(const DevScene S, const WaveBufs W) {
    const int n = min(W.dq_count[2], W.dq_cap);
    const int lane = threadIdx.x & 63;
    for (int e = (int)((blockIdx.x * 256u + threadIdx.x) >> 6); e < n; e += gridDim.x * 4) {
        const float4 a = W.dq_e[3 * (size_t)e], b = W.dq_e[3 * (size_t)e + 1], c4 = W.dq_e[3 * (size_t)e + 2];
        Ray lr;
        lr.o = mk(a.x, a.y, a.z);
        lr.d = mk(b.x, b.y, b.z);
        const float minT0 = a.w, limit = b.w;
        const int first = __float_as_int(c4.x), cnt = __float_as_int(c4.y), q = __float_as_int(c4.z);
        const bool conf = __float_as_int(c4.w) != 0;
        const RayRcp rq = ray_rcp(lr);
        int bits = 0;
        for (int x = first + lane; x < first + cnt; x += 64) {
            const float4* R = S.ahtris + 3 * (size_t)x;
            float t;
            if (!tri_test_fast_rec(R, lr, limit, t)) continue;
            const int ref = __float_as_int(R[0].w);
            const float4 na = S.nodes[2 * ref], nb = S.nodes[2 * ref + 1];
            if (!box_hit_fast(na.x, na.y, na.z, na.w, nb.x, nb.y, lr, rq, minT0)) continue;
            bits |= (conf && box_hit_fast(na.x, na.y, na.z, na.w, nb.x, nb.y, lr, rq, limit)) ? SS_OCC : SS_UNDECIDED;
        }
        const uint64_t occ = __ballot(bits & SS_OCC), und = __ballot(bits & SS_UNDECIDED);
        if (lane == 0 && (occ | und)) atomicOr(W.shadow_state + q, (occ ? SS_OCC : 0) | (und ? SS_UNDECIDED : 0));
    }
}

// A pending shadow ray's answer: occluded by a queued leaf, undecided (the reference walk), or
// not occluded; the general layout records it in occ, the one-light layout finishes the pixel.
DEV bool pending_occluded(int st) { return (st & SS_OCC) != 0; }

}  // namespace rtg
