// Wavefront ray trees: the mirror / conductor / dielectric recursion of PerformShading
// (raytracer.cpp:65-134, 208-472) as levels of compacted ray queues, for scenes whose
// materials spawn secondary rays (the fused kernel keeps one thread per pixel walking
// the whole tree with a per-thread stack; that costs 256 VGPRs and scratch).
//
// Per sample pass, level L = 0, 1, ... holds every ray of depth L of every pixel's tree:
//
//   k_tree_gen      level 0: the camera rays (GenerateRay, raytracer.cpp:661-699)
//   k_tree_trace    closest hit of every ray of the level (lean traversal kernel)
//   k_tree_shade    one node per hit: surface, ambient, per-light Shade terms and their
//                   shadow rays (queued per block), the node's kind and its child rays
//                   (queued per block, two slots per node); misses get their value here
//   k_shadow        the level's shadow rays (the pipeline's any-hit kernel)
//   k_tree_scan     prefix over the per-block child counts -> next level size
//   k_tree_compact  child rays into the next level's dense arrays, child links
//   ...
//   k_tree_resolve  levels deepest first: colour = base + unoccluded terms in light order,
//                   then the reference's combine with the children's values (mirror,
//                   conductor, total internal reflection, Fresnel reflect + refract with
//                   Beer's law); level 0 writes the pixel (or its spp accumulation)
//
// Every value is computed by the same expressions in the same order as the recursion
// (rtg_mega.hip / the reference), so the result is bit-identical to the fused kernel.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rtg_common.hpp"
#include "rtg_kernels.hpp"

namespace rtg {

// the level's ray count: the device's (device-driven levels, written by the previous level's
// k_tree_scan) or the host's
DEV int level_n(const TreeLevel& L) { return L.nd ? *L.nd : L.n; }

enum : int { TK_FINAL = 0, TK_LEAF = 1, TK_ADDZERO = 2, TK_MIRROR = 3, TK_CONDUCTOR = 4, TK_TIR = 5, TK_DIEL = 6 };
enum : int { TK_LIT = 16 };
enum : int { TM_ZERO = 0, TM_ENV = 1 };

// Level 0 of a pass of P.slabs samples: ray i is sample sample0 + i / npix of the part's pixel
// tree_pixel(i mod npix) (npix = width * part_rows), so each slab is one sample's camera rays in
// the 8x8-tile order.
DEV int level0_pixel(const RenderParams& P, int width, int i, int& slab) {
    const int npix = width * P.part_rows;
    slab = i / npix;
    return tree_pixel(P, width, i - slab * npix);
}

__global__ __launch_bounds__(256) void k_tree_gen(const DevCamera C, const RenderParams P, const int sample0,
                                                  const TreeLevel L0) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= L0.n) return;
    int slab;
    const int pixel = level0_pixel(P, C.width, i, slab);
    const int px = pixel % C.width, py = pixel / C.width;
    const uint64_t key = root_key(P.seed, pixel, sample0 + slab);
    float mbTime;
    Ray r = camera_ray(C, px, py, key, mbTime);
    L0.o[i] = make_float4(r.o.x, r.o.y, r.o.z, 1.0f);
    L0.d[i] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(0));
    L0.key[i] = key;
}

// Closest hit of every ray of the level: the per-lane reference walk (the levels below the
// camera's are incoherent -- round 5 measured packets on level 0 or on every level, the checked
// closest-hit walk of the any-hit tree and a persistent refilling walk, all slower:
// profiles/r05g_c5_tree_walks_ab.txt, r05y_c5_closest_ab.txt, r05z_c5_persistent_ab.txt; round 6,
// 64-B node records with quantised child boxes: C5 1 780 -> 1 575 Mrays/s, r06h_c5_qnodes_ab.txt)
template <bool STATS, int FEAT>
__global__ __launch_bounds__(256, RTG_TRACE_WAVES(FEAT)) void k_tree_trace(const DevScene S, const TreeLevel L,
                                                                           const int level, DevCounters* counters) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    Cnt<STATS> cn;
    if (i < level_n(L)) {
        const float4 o = L.o[i], d = L.d[i];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        if (level == 0) cn.cam();
        else cn.sec();
        Hit h;
        trace<false, STATS, FEAT>(S, r, 0.f, INFINITY, INFINITY, h, cn);
        L.t[i] = h.t;
        L.obj[i] = h.obj;
        L.face[i] = h.face;
    }
    flush_counters<STATS>(cn, counters);
}

// wave-aggregated append into a block segment (ballot + mbcnt rank + one LDS atomic)
DEV int seg_append(bool want, int* lds_count) {
    const unsigned long long mask = __ballot(want);
    if (!mask) return -1;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(lds_count, __popcll(mask));
    base = __shfl(base, leader);
    return want ? base + __popcll(mask & ((1ull << lane) - 1ull)) : -1;
}

// SK: shading features the scene may use (rtg_common.hpp SK_*): the general variant and one
// without BRDFs and env / spot / mesh lights (C5: textures, point lights).
#ifndef RTG_TREE_SHADE_WAVES_LEAN
#define RTG_TREE_SHADE_WAVES_LEAN 2
#endif
template <bool STATS, int SK = SK_ALL>
__global__ __launch_bounds__(256, SK == SK_ALL ? RTG_TREE_SHADE_WAVES : RTG_TREE_SHADE_WAVES_LEAN) void k_tree_shade(const DevScene S, const DevCamera C, const TreeLevel L,
                                                    const int level, const RenderParams P, const TreeSegs G,
                                                    DevCounters* counters) {
    __shared__ int nShadow, nChild;
    if (threadIdx.x == 0) { nShadow = 0; nChild = 0; }
    __syncthreads();
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < level_n(L);
    Cnt<STATS> cn;
    ShadeCtx c;
    bool lit = false;
    f3 w_o = mk(0, 0, 0);
    uint64_t key = 0;
    // children to spawn: count (0..2), rays
    int nch = 0;
    Ray ch0, ch1;
    float med0 = 1.0f, med1 = 1.0f;
    f3 miss0 = mk(0, 0, 0), miss1 = mk(0, 0, 0);
    int mm0 = TM_ZERO, mm1 = TM_ZERO;
    int depth = 0;
    if (valid) {
        const float4 o = L.o[i], d = L.d[i];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        const float medium = o.w;
        depth = S.max_depth - __float_as_int(d.w);
        key = L.key[i];
        const int obj = L.obj[i];
        if (obj < 0) {
            f3 v;
            if (level == 0) {
                int slab;
                const int pixel = level0_pixel(P, C.width, i, slab);
                v = miss_color<SK>(S, C, pixel % C.width, pixel / C.width, r.d);
            } else {
                const float4 m = L.miss[i];
                v = __float_as_int(m.w) == TM_ENV
                        ? (((SK & SK_XLIGHT) && S.num_env > 0) ? env_sample(S, 0, mk(m.x, m.y, m.z)) : mk(0, 0, 0))
                        : mk(0, 0, 0);
            }
            L.base[i] = make_float4(0, 0, 0, __int_as_float(TK_FINAL));
            L.value[i] = make_float4(v.x, v.y, v.z, __int_as_float(0));
        } else {
            const DevObject& ob = S.objects[obj];
            Hit h;
            h.t = L.t[i];
            h.obj = obj;
            h.face = L.face[i];
            h.o = r.o;
            c.ob = &ob;
            c.mat = &S.materials[ob.material];
            c.s = surface<STATS, (SK & SK_TEX) != 0>(S, r, 0.f, h, cn);
            const f3 eye = level == 0 ? ld3(C.pos) : r.o;
            w_o = makeUnit(sub(eye, c.s.p));
            const DevMaterial& mat = *c.mat;
            const bool inside = medium > 1.00001f;
            if (mat.type == 3) {                                        // Emissive (raytracer.cpp:81-84)
                const f3 e = muls(muls(ld3(mat.radiance), 2.0f), (float)RT_PI);
                L.base[i] = make_float4(0, 0, 0, __int_as_float(TK_FINAL));
                L.value[i] = make_float4(e.x, e.y, e.z, __int_as_float(1));
            } else if ((SK & SK_TEX) && ob.tex_replace_all >= 0) {      // replace_all (:87-89)
                const f3 e = tex_rgb(S, S.textures[ob.tex_replace_all], c.s.u, c.s.v);
                L.base[i] = make_float4(0, 0, 0, __int_as_float(TK_FINAL));
                L.value[i] = make_float4(e.x, e.y, e.z, __int_as_float(1));
            } else {
                f3 color = mk(0, 0, 0);
                if (!inside) {
                    color = add(color, mulv(mk(S.ambient[0], S.ambient[1], S.ambient[2]), ld3(mat.ambient)));
                    lit = true;
                }
                const f3 n = c.s.n, hp = c.s.p;
                int kind = TK_LEAF;
                float4 coef = make_float4(0, 0, 0, 0);
                float rT = 0.f;
                if (mat.type == 0) {                                    // Mirror (raytracer.cpp:442-472)
                    if (depth <= 0) {
                        kind = TK_ADDZERO;
                    } else {
                        kind = TK_MIRROR;
                        coef = make_float4(mat.mirror[0], mat.mirror[1], mat.mirror[2], 0.f);
                        ch0.d = reflect(n, w_o, mat.roughness, key, RP_ROUGH_REFL);
                        ch0.o = add(hp, muls(n, S.eps));
                        med0 = 1.0f;
                        miss0 = ch0.d;
                        mm0 = TM_ENV;
                        nch = 1;
                    }
                } else if (mat.type == 2) {                             // Conductor (raytracer.cpp:208-254)
                    if (depth <= 0) {
                        kind = TK_ADDZERO;
                    } else {
                        f3 dd = neg(w_o);
                        float cosTheta = -dot(dd, n);
                        float n2 = mat.refractive_index, k2 = mat.absorption_index;
                        float n2k2 = n2 * n2 + k2 * k2;
                        float n2cosTheta2 = 2 * n2 * cosTheta;
                        float cosThetaSqr = cosTheta * cosTheta;
                        float rs = (n2k2 - n2cosTheta2 + cosThetaSqr) / (n2k2 + n2cosTheta2 + cosThetaSqr);
                        float rp = (n2k2 * cosThetaSqr - n2cosTheta2 + 1) / (n2k2 * cosThetaSqr + n2cosTheta2 + 1);
                        float reflectRatio = (float)(0.5 * (rs + rp));
                        if (!(reflectRatio > 0.0001)) {
                            kind = TK_ADDZERO;
                        } else {
                            kind = TK_CONDUCTOR;
                            coef = make_float4(mat.mirror[0], mat.mirror[1], mat.mirror[2], reflectRatio);
                            ch0.d = reflect(n, w_o, mat.roughness, key, RP_ROUGH_REFL);
                            ch0.o = add(hp, muls(n, S.eps));
                            med0 = 1.0f;
                            mm0 = TM_ZERO;
                            nch = 1;
                        }
                    }
                } else if (mat.type == 1) {                             // Dielectric (raytracer.cpp:261-415)
                    if (depth <= 0) {
                        kind = TK_ADDZERO;
                    } else {
                        float n1 = medium, n2 = mat.refractive_index;
                        f3 dd = neg(w_o);
                        f3 modN = n;
                        float cosTheta = -dot(dd, modN);
                        bool isEntering = cosTheta > 0.f;
                        float objN = n2;
                        if (!isEntering) {
                            n1 = n2; n2 = 1.0f; objN = 1.0f;
                            cosTheta = fabsf(cosTheta);
                            modN = neg(modN);
                        }
                        float rr = n1 / n2;
                        float sinThetaSqr = 1 - (cosTheta * cosTheta);
                        float criticalTerm = rr * rr * sinThetaSqr;
                        if (criticalTerm > 1) {
                            kind = TK_TIR;
                            ch0.d = reflect(modN, w_o, mat.roughness, key, RP_ROUGH_REFL);
                            ch0.o = add(hp, muls(modN, S.eps));
                            med0 = medium;
                            mm0 = TM_ZERO;
                            nch = 1;
                        } else {
                            float cosPhi = sqrtf(1 - criticalTerm);
                            float n2cosTheta = n2 * cosTheta;
                            float n1cosPhi = n1 * cosPhi;
                            float rpar = (n2cosTheta - n1cosPhi) / (n2cosTheta + n1cosPhi);
                            float rperp = (n1 * cosTheta - n2 * cosPhi) / (n1 * cosTheta + n2 * cosPhi);
                            float rReflect = (rpar * rpar + rperp * rperp) / 2;
                            kind = TK_DIEL;
                            coef = make_float4(0, 0, 0, rReflect);
                            rT = 1 - rReflect;
                            ch0.d = reflect(modN, w_o, mat.roughness, key, RP_ROUGH_REFL);
                            ch0.o = add(hp, muls(modN, S.eps));
                            med0 = isEntering ? objN : 1.0f;
                            miss0 = ch0.d;
                            mm0 = TM_ENV;
                            // refracted ray (raytracer.cpp:362-392)
                            f3 wr = sub(muls(add(dd, muls(modN, cosTheta)), rr), muls(modN, cosPhi));
                            if (mat.roughness > 0.001) {
                                f3 u, v;
                                onb(wr, u, v);
                                float psi1 = rnd(key, RP_ROUGH_REFR, 0) - 0.5f;
                                float psi2 = rnd(key, RP_ROUGH_REFR, 1) - 0.5f;
                                wr = makeUnit(add(wr, muls(add(muls(u, psi1), muls(v, psi2)), mat.roughness)));
                            } else {
                                wr = makeUnit(wr);
                            }
                            ch1.o = add(hp, muls(neg(modN), S.eps));
                            ch1.d = wr;
                            med1 = isEntering ? objN : 1.0f;
                            miss1 = ch0.d;                  // refracted miss: reflected dir (:408)
                            mm1 = TM_ENV;
                            nch = 2;
                        }
                    }
                }
                L.base[i] = make_float4(color.x, color.y, color.z, __int_as_float(kind | (lit ? TK_LIT : 0)));
                L.coef[i] = coef;
                L.ext[i] = make_float4(rT, __int_as_float(ob.material), __int_as_float(-1), __int_as_float(-1));
            }
        }
    }
    // ---- light slots of lit nodes: Shade terms + shadow rays (SampleDirectLighting order)
    const int ns = G.num_slots;
    for (int l = 0; l < ns; ++l) {
        LightSample ls;
        if (lit) {
            ls = light_sample<SK>(S, l, c.s.p, c.s.n, key);
            const f3 t = shade<false, SK>(S, c, ls.w_i, w_o, ls.E);
            L.term[(size_t)i * ns + l] = make_float4(t.x, t.y, t.z, 0.f);
            L.occ[(size_t)i * ns + l] = 0;
        }
        const bool want = lit && ls.shadow;
        const int qi = seg_append(want, &nShadow);
        if (want) {
            cn.shd();
            const size_t q = (size_t)blockIdx.x * 256 * ns + qi;
            G.q_o[q] = make_float4(ls.sr.o.x, ls.sr.o.y, ls.sr.o.z, ls.minT);
            G.q_d[q] = make_float4(ls.sr.d.x, ls.sr.d.y, ls.sr.d.z, ls.limit);
            G.q_slot[q] = i * ns + l;
        }
    }
    // ---- child rays (slot 0, slot 1)
    for (int s = 0; s < 2; ++s) {
        const bool want = nch > s;
        const int ci = seg_append(want, &nChild);
        if (want) {
            const size_t q = (size_t)blockIdx.x * 512 + ci;
            const Ray& r = s == 0 ? ch0 : ch1;
            const f3 m = s == 0 ? miss0 : miss1;
            G.c_o[q] = make_float4(r.o.x, r.o.y, r.o.z, s == 0 ? med0 : med1);
            G.c_d[q] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(S.max_depth - depth + 1));
            G.c_key[q] = child_key(key, s);
            G.c_miss[q] = make_float4(m.x, m.y, m.z, __int_as_float(s == 0 ? mm0 : mm1));
            G.c_parent[q] = i | (s << 30);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        G.q_count[blockIdx.x] = nShadow;
        G.c_count[blockIdx.x] = nChild;
    }
    flush_counters<STATS>(cn, counters);
}

// exclusive prefix over the per-block child counts (one block); total -> offs[nb] and, for
// device-driven levels, min(total, cap) -> *next_n (the next level's count) with *overflow
// set when the planned capacity (0 past the planned levels) is exceeded
__global__ __launch_bounds__(1024) void k_tree_scan(const int* __restrict__ cnt, int nb, int* __restrict__ offs,
                                                    int* __restrict__ next_n, int cap, int* __restrict__ overflow) {
    __shared__ int part[1024];
    const int t = threadIdx.x;
    const int per = (nb + 1023) / 1024;
    const int b0 = t * per, b1 = min(nb, b0 + per);
    int s = 0;
    for (int b = b0; b < b1; ++b) s += cnt[b];
    part[t] = s;
    __syncthreads();
    for (int w = 1; w < 1024; w <<= 1) {
        const int v = t >= w ? part[t - w] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;
    for (int b = b0; b < b1; ++b) {
        offs[b] = run;
        run += cnt[b];
    }
    if (t == 1023) {
        offs[nb] = part[1023];
        if (next_n) {
            *next_n = part[1023] < cap ? part[1023] : cap;
            if (part[1023] > cap) *overflow = 1;
        }
    }
}

// Child rays into the next level's dense arrays in append order (round 5 measured grouping a
// block's children by direction octant: no change, profiles/r05g_c5_tree_walks_ab.txt), and
// the parents' child links.
__global__ __launch_bounds__(256) void k_tree_compact(const TreeSegs G, const int* __restrict__ offs,
                                                      const TreeLevel cur, const TreeLevel nxt, const int cap) {
    const int b = blockIdx.x;
    const int n = G.c_count[b], base = offs[b];
    for (int k = threadIdx.x; k < n; k += 256) {
        const int dst = base + k;
        if (dst >= cap) break;                       // over the planned capacity (k_tree_scan flagged it)
        const size_t q = (size_t)b * 512 + k;
        nxt.o[dst] = G.c_o[q];
        nxt.d[dst] = G.c_d[q];
        nxt.key[dst] = G.c_key[q];
        nxt.miss[dst] = G.c_miss[q];
        const int p = G.c_parent[q];
        const int parent = p & 0x3FFFFFFF, slot = p >> 30;
        int* ext = reinterpret_cast<int*>(&cur.ext[parent]);
        ext[2 + slot] = dst;
    }
}

__global__ __launch_bounds__(256) void k_tree_resolve(const DevScene S, const DevCamera C, const RenderParams P,
                                                      const int sample, const int first, const int last,
                                                      const TreeLevel L, const TreeLevel Lc, const int level,
                                                      const int num_slots,
                                                      float* __restrict__ hdr, unsigned char* __restrict__ ldrOut,
                                                      float4* __restrict__ accum) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= level_n(L)) return;
    const float4 b = L.base[i];
    const int kb = __float_as_int(b.w);
    const int kind = kb & 15;
    f3 value;
    if (kind == TK_FINAL) {
        const float4 v = L.value[i];
        value = mk(v.x, v.y, v.z);
    } else {
        f3 color = mk(b.x, b.y, b.z);
        if (kb & TK_LIT) {
            f3 sum = mk(0, 0, 0);
            const size_t s0 = (size_t)i * num_slots;
            for (int l = 0; l < num_slots; ++l)
                if (!L.occ[s0 + l]) {
                    const float4 t = L.term[s0 + l];
                    sum = add(sum, mk(t.x, t.y, t.z));
                }
            color = add(color, sum);
        }
        if (kind == TK_LEAF) {
            value = color;
        } else if (kind == TK_ADDZERO) {
            value = add(color, mk(0, 0, 0));
        } else {
            const float4 cf = L.coef[i];
            const float4 ex = L.ext[i];
            const f3 coef = mk(cf.x, cf.y, cf.z);
            const DevMaterial& pm = S.materials[__float_as_int(ex.y)];
            auto child = [&](int slot, f3& v, bool& vHit, float& vT, float& vMed) {
                const int ci = __float_as_int(slot == 0 ? ex.z : ex.w);
                if (ci < 0) {
                    // a child dropped by a device-driven level over its planned capacity: the
                    // overflow flag is set and the render is redone host-driven
                    v = mk(0, 0, 0);
                    vHit = false;
                    vT = 0.f;
                    vMed = 1.f;
                    return;
                }
                const float4 cv = Lc.value[ci];
                v = mk(cv.x, cv.y, cv.z);
                vHit = __float_as_int(cv.w) != 0;
                vT = Lc.t[ci];
                vMed = Lc.o[ci].w;
            };
            f3 v0;
            bool h0;
            float t0, m0;
            child(0, v0, h0, t0, m0);
            f3 term;
            if (kind == TK_MIRROR) {
                term = mulv(coef, v0);
            } else if (kind == TK_CONDUCTOR) {
                term = muls(h0 ? mulv(coef, v0) : mk(0, 0, 0), cf.w);
            } else if (kind == TK_TIR) {
                term = h0 ? ((m0 > 1.0001) ? beer(t0, pm.absorption, v0) : v0) : mk(0, 0, 0);
            } else {
                const f3 refl = (h0 && m0 > 1.00001f) ? beer(t0, pm.absorption, v0) : v0;
                f3 v1;
                bool h1;
                float t1, m1;
                child(1, v1, h1, t1, m1);
                const f3 refr = (h1 && m1 > 1.001f) ? beer(t1, pm.absorption, v1) : v1;
                term = add(muls(refl, cf.w), muls(refr, ex.x));
            }
            value = add(color, term);
        }
    }
    if (level > 0 || P.slabs > 1) {     // (a multi-sample pass: k_tree_accum adds level 0's values)
        L.value[i] = make_float4(value.x, value.y, value.z, __int_as_float(L.obj[i] >= 0 ? 1 : 0));
        return;
    }
    // level 0: the pixel (RenderPixel's colour), spp accumulation as k_resolve
    const int pixel = tree_pixel(P, C.width, i);
    if (C.spp <= 1 && !P.accum_only) {
        const size_t idx = 3 * (size_t)pixel;
        if (hdr) { hdr[idx] = value.x; hdr[idx + 1] = value.y; hdr[idx + 2] = value.z; }
        if (ldrOut) { ldrOut[idx] = ldr(value.x); ldrOut[idx + 1] = ldr(value.y); ldrOut[idx + 2] = ldr(value.z); }
        return;
    }
    const float gw = sample_weight(C.spp, sample, root_key(P.seed, pixel, sample));
    float4 a = first ? make_float4(0.f, 0.f, 0.f, 0.f) : accum[pixel];
    // (accum_samples, rtg_common.hpp: the same operations over a multi-sample pass's slabs)
    a.x += value.x * gw;
    a.y += value.y * gw;
    a.z += value.z * gw;
    a.w += gw;
    accum[pixel] = a;
    if (last && !P.accum_only) {
        const f3 cc = mk(a.x / a.w, a.y / a.w, a.z / a.w);
        const size_t idx = 3 * (size_t)pixel;
        if (hdr) { hdr[idx] = cc.x; hdr[idx + 1] = cc.y; hdr[idx + 2] = cc.z; }
        if (ldrOut) { ldrOut[idx] = ldr(cc.x); ldrOut[idx + 1] = ldr(cc.y); ldrOut[idx + 2] = ldr(cc.z); }
    }
}

// The end of a multi-sample pass: every pixel's level-0 values of the pass's slabs added to its
// accumulation in sample order (accum_samples) -- the one-sample passes' operations bit for bit.
__global__ __launch_bounds__(256) void k_tree_accum(const DevCamera C, const RenderParams P, const int sample0,
                                                    const int first, const int last, const TreeLevel L0,
                                                    float* __restrict__ hdr, unsigned char* __restrict__ ldrOut,
                                                    float4* __restrict__ accum) {
    const int npix = C.width * P.part_rows;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= npix) return;
    accum_samples(C, P, sample0, P.slabs, first != 0, last != 0, tree_pixel(P, C.width, i), L0.value + i,
                  (size_t)npix, accum, hdr, ldrOut);
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
namespace {

template <typename T>
hipError_t grow(T*& p, size_t& cap, size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = n + n / 4 + 1024;
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
}

}  // namespace

struct TreeState {
    struct Level {
        TreeLevel L{};
        size_t cap = 0, cap_slots = 0;
        // separate capacities per array (grown together)
        size_t co = 0, cd = 0, ck = 0, cm = 0, ct = 0, cob = 0, cf = 0, cb = 0, cc = 0, ce = 0, cv = 0, cte = 0, coc = 0;
    };
    std::vector<Level> levels;
    TreeSegs G{};
    size_t c_qo = 0, c_qd = 0, c_qs = 0, c_qc = 0, c_o = 0, c_d = 0, c_k = 0, c_m = 0, c_p = 0, c_cc = 0, c_off = 0;
    int* offs = nullptr;
    int* h_total = nullptr;     // pinned host words: [0] a level's size, [1..4] the streams' overflow flags
    // device-driven levels: per level the ray count (written by the previous level's scan) and
    // the overflow flag; the plan = capacities per level learned from a host-driven pass of
    // the same frame part (plan_key)
    int* d_counts = nullptr;    // kMaxLevels + 1 ints, [kMaxLevels] = overflow
    std::vector<size_t> plan;
    std::vector<long long> plan_key;
    int sk = SK_ALL;            // the scene's shading features (k_tree_shade variant)
    // multi-stream planned passes (tree_streams): the other streams' level buffers and the
    // streams; fork / join events and two "resolve done" events (sample order of the resolves)
    std::vector<TreeState*> twins;
    std::vector<hipStream_t> xst;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_res[2] = {nullptr, nullptr};
    ~TreeState() {
        for (TreeState* t : twins) delete t;
        for (hipStream_t x : xst) (void)hipStreamDestroy(x);
        for (hipEvent_t e : {ev_fork, ev_join, ev_res[0], ev_res[1]})
            if (e) (void)hipEventDestroy(e);
        auto f = [](void* p) { if (p) (void)hipFree(p); };
        for (auto& lv : levels) {
            TreeLevel& L = lv.L;
            f(L.o); f(L.d); f(L.key); f(L.miss); f(L.t); f(L.obj); f(L.face); f(L.base); f(L.coef); f(L.ext);
            f(L.value); f(L.term); f(L.occ);
        }
        f(G.q_o); f(G.q_d); f(G.q_slot); f(G.q_count); f(G.c_o); f(G.c_d); f(G.c_key); f(G.c_miss); f(G.c_parent);
        f(G.c_count); f(offs); f(d_counts);
        if (h_total) (void)hipHostFree(h_total);
    }
};
constexpr int kMaxLevels = 64;

static hipError_t ensure_level(TreeState::Level& lv, size_t n, int ns) {
    TreeLevel& L = lv.L;
    hipError_t e;
#define G_(ptr, c, cnt) if ((e = grow(ptr, lv.c, cnt)) != hipSuccess) return e
    G_(L.o, co, n); G_(L.d, cd, n); G_(L.key, ck, n); G_(L.miss, cm, n); G_(L.t, ct, n); G_(L.obj, cob, n);
    G_(L.face, cf, n); G_(L.base, cb, n); G_(L.coef, cc, n); G_(L.ext, ce, n); G_(L.value, cv, n);
    G_(L.term, cte, n * (size_t)(ns > 0 ? ns : 1)); G_(L.occ, coc, n * (size_t)(ns > 0 ? ns : 1));
#undef G_
    L.n = (int)n;
    L.nd = nullptr;
    return hipSuccess;
}

static hipError_t ensure_segs(TreeState& T, size_t blocks, int ns) {
    TreeSegs& G = T.G;
    hipError_t e;
    const size_t nq = blocks * 256 * (size_t)(ns > 0 ? ns : 1), nc = blocks * 512;
#define G_(ptr, c, cnt) if ((e = grow(ptr, T.c, cnt)) != hipSuccess) return e
    G_(G.q_o, c_qo, nq); G_(G.q_d, c_qd, nq); G_(G.q_slot, c_qs, nq); G_(G.q_count, c_qc, blocks);
    G_(G.c_o, c_o, nc); G_(G.c_d, c_d, nc); G_(G.c_key, c_k, nc); G_(G.c_miss, c_m, nc); G_(G.c_parent, c_p, nc);
    G_(G.c_count, c_cc, blocks); G_(T.offs, c_off, blocks + 1);
#undef G_
    G.num_slots = ns;
    return hipSuccess;
}

void tree_destroy(TreeState* t) { delete t; }

// One level's trace / shade / shadow / scan launches (rays: L's count, on the host or device).
// (Round 5 measured an XCD-aware block order for the levels' grids -- no change,
// profiles/r05s_tree_xcd_ab.txt -- and the levels' shadow rays on the any-hit tree as packets
// or per lane -- slower, r05g_c5_tree_walks_ab.txt: they keep the per-lane reference walk.)
template <bool STATS, int FEAT>
static void level_launches(TreeState& T, const DevScene& S, const DevCamera& C, const RenderParams& P, int s,
                           int level, TreeLevel& L, int blocks, int ns, int* next_n, int cap_next, DevCounters* cnt,
                           hipStream_t st) {
    if (level == 0) hipLaunchKernelGGL(k_tree_gen, dim3(blocks), dim3(256), 0, st, C, P, s, L);
    hipLaunchKernelGGL((k_tree_trace<STATS, FEAT>), dim3(blocks), dim3(256), 0, st, S, L, level, cnt);
    if ((T.sk & ~SK_TEX) == 0)
        hipLaunchKernelGGL((k_tree_shade<STATS, SK_TEX>), dim3(blocks), dim3(256), 0, st, S, C, L, level, P, T.G, cnt);
    else
        hipLaunchKernelGGL((k_tree_shade<STATS, SK_ALL>), dim3(blocks), dim3(256), 0, st, S, C, L, level, P, T.G, cnt);
    if (ns > 0) {
        WaveBufs W{};
        W.q_o = T.G.q_o; W.q_d = T.G.q_d; W.q_slot = T.G.q_slot; W.q_count = T.G.q_count;
        W.occ = L.occ;
        W.num_slots = ns;
        W.hit_obj = L.obj;              // the hits the shadow rays leave (their origin leaf)
        W.hit_face = L.face;
        hipLaunchKernelGGL((k_shadow<STATS, FEAT, false>), dim3(blocks, ns), dim3(256), 0, st, S, W, cnt);
    }
    hipLaunchKernelGGL(k_tree_scan, dim3(1), dim3(1024), 0, st, T.G.c_count, blocks, T.offs, next_n, cap_next,
                       T.d_counts ? T.d_counts + kMaxLevels : nullptr);
}

// Host-driven sample pass: after each level the next level's size comes back to the host
// (one stream synchronisation per level), the arrays grow to it.  `sizes` receives the
// level sizes (the plan of device-driven passes).
template <bool STATS, int FEAT>
static hipError_t tree_pass_sync(TreeState& T, const DevScene& S, const DevCamera& C, const RenderParams& P, int s,
                                 bool first, bool last, float* hdr, unsigned char* l, float4* accum, DevCounters* cnt,
                                 hipStream_t st, hipEvent_t* ev, std::vector<size_t>& sizes) {
    const int ns = S.num_point + S.num_area + S.num_env + S.num_dir + S.num_spot + S.num_mesh;
    const int npix = P.part_rows * C.width;
    hipError_t e;
    size_t n = (size_t)npix * P.slabs;
    int level = 0;
    sizes.assign(1, n);
    if (ev) (void)hipEventRecord(ev[0], st);
    for (;; ++level) {
        if ((int)T.levels.size() <= level) T.levels.emplace_back();
        if ((e = ensure_level(T.levels[level], n, ns)) != hipSuccess) return e;
        TreeLevel& L = T.levels[level].L;
        const int blocks = (int)((n + 255) / 256);
        if ((e = ensure_segs(T, (size_t)blocks, ns)) != hipSuccess) return e;
        level_launches<STATS, FEAT>(T, S, C, P, s, level, L, blocks, ns, nullptr, 0, cnt, st);
        if ((e = hipMemcpyAsync(T.h_total, T.offs + blocks, sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        const size_t nn = (size_t)*T.h_total;
        if (nn == 0) break;
        if (level + 1 >= kMaxLevels) return hipErrorInvalidValue;
        sizes.push_back(nn);
        if ((int)T.levels.size() <= level + 1) T.levels.emplace_back();
        if ((e = ensure_level(T.levels[level + 1], nn, ns)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_tree_compact, dim3(blocks), dim3(256), 0, st, T.G, T.offs, T.levels[level].L,
                           T.levels[level + 1].L, (int)nn);
        n = nn;
    }
    if (ev) (void)hipEventRecord(ev[1], st);
    for (int lv = level; lv >= 0; --lv) {
        const TreeLevel& L = T.levels[lv].L;
        const TreeLevel& Lc = lv < level ? T.levels[lv + 1].L : L;
        const int blocks = (int)((L.n + 255) / 256);
        hipLaunchKernelGGL(k_tree_resolve, dim3(blocks), dim3(256), 0, st, S, C, P, s, (int)first, (int)last, L,
                           Lc, lv, ns, hdr, l, accum);
    }
    if (P.slabs > 1)
        hipLaunchKernelGGL(k_tree_accum, dim3((npix + 255) / 256), dim3(256), 0, st, C, P, s, (int)first, (int)last,
                           T.levels[0].L, hdr, l, accum);
    if (ev) (void)hipEventRecord(ev[2], st);
    return hipGetLastError();
}

// Device-driven sample pass: no host synchronisation.  The levels follow the plan (capacity
// per level); each level's grids cover its capacity and its kernels read the level's ray count
// on the device (written by the previous level's scan), blocks past it exit at once.  A level
// that outgrows its capacity, or children past the planned depth, set the overflow flag; the
// caller checks it once per render and redoes the render host-driven.
// wait_res / rec_res (two-stream passes): the resolve phase waits for the previous pass's
// resolves (the other stream) and marks its own end -- the accumulation stays in sample order.
template <bool STATS, int FEAT>
static hipError_t tree_pass_async(TreeState& T, const DevScene& S, const DevCamera& C, const RenderParams& P, int s,
                                  bool first, bool last, float* hdr, unsigned char* l, float4* accum,
                                  DevCounters* cnt, hipStream_t st, hipEvent_t* ev, hipEvent_t wait_res = nullptr,
                                  hipEvent_t rec_res = nullptr) {
    const int ns = S.num_point + S.num_area + S.num_env + S.num_dir + S.num_spot + S.num_mesh;
    const int D = (int)T.plan.size();
    if (ev) (void)hipEventRecord(ev[0], st);
    for (int level = 0; level < D; ++level) {
        TreeLevel& L = T.levels[level].L;
        L.n = (int)T.plan[level];
        L.nd = level == 0 ? nullptr : T.d_counts + level;
        const int blocks = (int)((T.plan[level] + 255) / 256);
        const bool more = level + 1 < D;
        level_launches<STATS, FEAT>(T, S, C, P, s, level, L, blocks, ns, T.d_counts + level + 1,
                                    more ? (int)T.plan[level + 1] : 0, cnt, st);
        if (more) {
            TreeLevel& Ln = T.levels[level + 1].L;
            Ln.n = (int)T.plan[level + 1];
            Ln.nd = T.d_counts + level + 1;
            hipLaunchKernelGGL(k_tree_compact, dim3(blocks), dim3(256), 0, st, T.G, T.offs, L, Ln,
                               (int)T.plan[level + 1]);
        }
    }
    if (ev) (void)hipEventRecord(ev[1], st);
    if (wait_res) (void)hipStreamWaitEvent(st, wait_res, 0);
    for (int lv = D - 1; lv >= 0; --lv) {
        const TreeLevel& L = T.levels[lv].L;
        const TreeLevel& Lc = lv + 1 < D ? T.levels[lv + 1].L : L;
        const int blocks = (int)((T.plan[lv] + 255) / 256);
        hipLaunchKernelGGL(k_tree_resolve, dim3(blocks), dim3(256), 0, st, S, C, P, s, (int)first, (int)last, L,
                           Lc, lv, ns, hdr, l, accum);
    }
    if (P.slabs > 1) {
        const int npix = P.part_rows * C.width;
        hipLaunchKernelGGL(k_tree_accum, dim3((npix + 255) / 256), dim3(256), 0, st, C, P, s, (int)first, (int)last,
                           T.levels[0].L, hdr, l, accum);
    }
    if (rec_res) (void)hipEventRecord(rec_res, st);
    if (ev) (void)hipEventRecord(ev[2], st);
    return hipGetLastError();
}

// Planned passes on several streams (RTG_TREE_STREAMS, default 3, at most 4; 1: one stream):
// pass k runs on stream k mod N (stream 0 the render's), each with its own level buffers, so one
// pass's level boundaries -- the tails of its trace / shade / shadow grids, the one-block scan,
// the small deep levels -- are filled by the others' work (C5: 1 789 -> 2 235 Mrays/s with two,
// 2 270 with three, 2 232 with four; profiles/r06l_c5_two_streams_ab.txt, r06m_c5_streams_ab.txt).  The resolves wait for the previous pass's resolves, so
// the accumulation keeps its sample order (the same bits as one stream); a pass with timing
// events (the render's last) and host-driven passes run on the render's stream after a join.
static int tree_streams() {
    const char* e = std::getenv("RTG_TREE_STREAMS");
    const int n = e ? std::atoi(e) : 3;
    return n < 1 ? 1 : n > 4 ? 4 : n;
}

// RTG_TREE_SYNC=1: every pass host-driven (one synchronisation per level; A/B)
static bool tree_sync_only() { return std::getenv("RTG_TREE_SYNC") != nullptr; }

template <bool STATS, int FEAT>
static hipError_t tree_run(TreeState& T, const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                           unsigned char* l, float4* accum, DevCounters* cnt, hipStream_t st, hipEvent_t* ev) {
    hipError_t e;
    if (!T.h_total) {
        if ((e = hipHostMalloc(&T.h_total, 8 * sizeof(int))) != hipSuccess) return e;
        if ((e = hipMalloc(&T.d_counts, (kMaxLevels + 1) * sizeof(int))) != hipSuccess) return e;
    }
    const int ns = S.num_point + S.num_area + S.num_env + S.num_dir + S.num_spot + S.num_mesh;
    // the plan belongs to one frame part of one camera (its view and samples decide the level
    // sizes): two cameras of a scene at the same size keep apart
    const std::vector<long long> key = {P.row_begin, P.row_end, P.part_index, P.part_count, C.width, C.height,
                                        (long long)(size_t)S.objects, S.max_depth, (long long)camera_hash(C), P.slabs};
    const int NS = STATS ? 1 : tree_streams();
    auto prepare_one = [&](TreeState& U) -> hipError_t {
        // capacities and block segments of the plan; the overflow flag cleared
        hipError_t r;
        for (size_t lv = 0; lv < U.plan.size(); ++lv) {
            if (U.levels.size() <= lv) U.levels.emplace_back();
            if ((r = ensure_level(U.levels[lv], U.plan[lv], ns)) != hipSuccess) return r;
        }
        if ((r = ensure_segs(U, (*std::max_element(U.plan.begin(), U.plan.end()) + 255) / 256, ns)) != hipSuccess)
            return r;
        return hipMemsetAsync(U.d_counts + kMaxLevels, 0, sizeof(int), st);
    };
    auto prepare = [&]() -> hipError_t {
        hipError_t r;
        if ((r = prepare_one(T)) != hipSuccess || NS == 1) return r;
        if (!T.ev_fork)
            for (hipEvent_t* pe : {&T.ev_fork, &T.ev_join, &T.ev_res[0], &T.ev_res[1]})
                if ((r = hipEventCreateWithFlags(pe, hipEventDisableTiming)) != hipSuccess) return r;
        while ((int)T.twins.size() < NS - 1) {
            hipStream_t x;
            if ((r = hipStreamCreateWithFlags(&x, hipStreamNonBlocking)) != hipSuccess) return r;
            T.xst.push_back(x);
            T.twins.push_back(new TreeState());
        }
        for (int k = 0; k < NS - 1; ++k) {
            TreeState& U = *T.twins[k];
            if (!U.d_counts && (r = hipMalloc(&U.d_counts, (kMaxLevels + 1) * sizeof(int))) != hipSuccess) return r;
            U.sk = T.sk;
            U.plan = T.plan;
            U.plan_key = T.plan_key;
            if ((r = prepare_one(U)) != hipSuccess) return r;
        }
        return hipSuccess;
    };
    auto make_plan = [&](const std::vector<size_t>& seen) {
        // the level sizes seen, with a margin for sampled (stochastic) trees
        // (RTG_TREE_PLAN_TIGHT=1, tests: one ray short of the sizes seen, so every planned
        // render overflows and is redone host-driven)
        const bool tight = std::getenv("RTG_TREE_PLAN_TIGHT") != nullptr;
        T.plan.clear();
        for (size_t k = 0; k < seen.size(); ++k)
            T.plan.push_back(k == 0 ? seen[k] : tight ? (seen[k] > 1 ? seen[k] - 1 : seen[k]) : seen[k] + seen[k] / 4 + 1024);
        T.plan_key = key;
    };
    for (int attempt = 0; attempt < 2; ++attempt) {
        // attempt 0: planned passes when this frame part has a plan, else the first pass
        // host-driven and the rest planned from it; attempt 1 (a level outgrew the plan):
        // every pass host-driven, re-planning
        // (counted renders stay host-driven: a planned render that overflows would be redone and
        // its discarded pass counted twice)
        const bool adapt = attempt == 0 && !tree_sync_only() && !STATS;
        bool planned = adapt && T.plan_key == key && !T.plan.empty();
        bool any_async = false;
        if (planned && (e = prepare()) != hipSuccess) return e;
        std::vector<size_t> seen;
        int n_async = 0;                 // planned passes issued (their parity picks the stream)
        bool forked = false, used2 = false;
        auto join = [&]() {              // the render's stream waits for the others
            if (!forked) return;
            for (int k = 0; k < NS - 1; ++k) {
                (void)hipEventRecord(T.ev_join, T.xst[k]);
                (void)hipStreamWaitEvent(st, T.ev_join, 0);
            }
            forked = false;
        };
        // passes of P.slabs consecutive samples; a shorter last pass (what is left) runs
        // host-driven: its level sizes are not the plan's
        const int s_end = P.sample_begin + P.sample_count;
        for (int s = P.sample_begin; s < s_end; s += P.slabs) {
            RenderParams Pp = P;
            Pp.slabs = s_end - s < P.slabs ? s_end - s : P.slabs;
            const bool first = s == P.sample_begin, last = s + Pp.slabs == s_end;
            hipEvent_t* pev = last ? ev : nullptr;
            if (planned && Pp.slabs == P.slabs) {
                if (NS > 1 && !forked && !pev) {  // (before this pass: the next ones may overlap it)
                    (void)hipEventRecord(T.ev_fork, st);
                    for (int k = 0; k < NS - 1; ++k) (void)hipStreamWaitEvent(T.xst[k], T.ev_fork, 0);
                    forked = used2 = true;
                }
                const int sx = pev ? 0 : n_async % NS;     // stream (and level buffers) of this pass
                if (pev) join();         // the timed pass alone on the render's stream
                hipEvent_t wait = NS > 1 && n_async > 0 ? T.ev_res[(n_async - 1) & 1] : nullptr;
                hipEvent_t rec = NS > 1 ? T.ev_res[n_async & 1] : nullptr;
                e = tree_pass_async<STATS, FEAT>(sx ? *T.twins[sx - 1] : T, S, C, Pp, s, first, last, hdr, l, accum,
                                                 cnt, sx ? T.xst[sx - 1] : st, pev, wait, rec);
                any_async = true;
                ++n_async;
            } else if (planned) {
                join();
                // (the render's last pass: the planned passes before it are untouched -- buffers
                // only grow -- and the next render re-prepares the plan)
                std::vector<size_t> sizes;
                e = tree_pass_sync<STATS, FEAT>(T, S, C, Pp, s, first, last, hdr, l, accum, cnt, st, pev, sizes);
            } else {
                std::vector<size_t> sizes;
                e = tree_pass_sync<STATS, FEAT>(T, S, C, Pp, s, first, last, hdr, l, accum, cnt, st, pev, sizes);
                if (sizes.size() > seen.size()) seen.resize(sizes.size(), 0);
                for (size_t k = 0; k < sizes.size(); ++k) seen[k] = std::max(seen[k], sizes[k]);
                if (e == hipSuccess && adapt) {
                    make_plan(seen);
                    planned = true;
                    e = prepare();
                }
            }
            if (e != hipSuccess) return e;
        }
        join();
        if (!any_async) {
            if (!seen.empty()) make_plan(seen);
            return hipSuccess;
        }
        // one synchronisation per render: did a level outgrow the plan (on any stream's buffers)?
        const int nf = used2 ? NS : 1;
        for (int k = 0; k < nf; ++k)
            if ((e = hipMemcpyAsync(T.h_total + 1 + k, (k ? T.twins[k - 1]->d_counts : T.d_counts) + kMaxLevels,
                                    sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess)
                return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        bool overflow = false;
        for (int k = 0; k < nf; ++k) overflow |= T.h_total[1 + k] != 0;
        if (!overflow) return hipSuccess;
        T.plan.clear();
    }
    return hipSuccess;
}

hipError_t launch_tree(TreeState*& T, const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                       unsigned char* l, float4* accum, DevCounters* cnt, bool stats, int feat, int sk,
                       hipStream_t st, hipEvent_t* ev) {
    if (!T) T = new TreeState();
    T->sk = sk;
    const bool big = (feat & FEAT_BIGLEAF) != 0;
    const int base = feat & ~FEAT_BIGLEAF;
#define RTG_TREE(F)                                                                     \
    return stats ? tree_run<true, F>(*T, S, C, P, hdr, l, accum, cnt, st, ev)           \
                 : tree_run<false, F>(*T, S, C, P, hdr, l, accum, cnt, st, ev)
    if (base == 0) {
        if (big) RTG_TREE(FEAT_BIGLEAF);
        RTG_TREE(0);
    }
    if (base == FEAT_SPHERE) {
        if (big) RTG_TREE(FEAT_SPHERE | FEAT_BIGLEAF);
        RTG_TREE(FEAT_SPHERE);
    }
    if (big) RTG_TREE(FEAT_ALL);
    RTG_TREE(FEAT_ALL & ~FEAT_BIGLEAF);
#undef RTG_TREE
}

}  // namespace rtg
