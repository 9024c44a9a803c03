// Fused ("mega") render kernel: one thread per pixel walks the pixel's whole ray tree
// -- PerformShading (raytracer.cpp:65-134) with the recursion of ComputeMirrorReflection /
// ...Dielectric... / ...Conductor... and, for path-tracing cameras, ComputeGlobalIllumination
// (raytracer.cpp:135-191) unrolled onto an explicit per-thread stack.  Used for path
// tracing, motion blur and small ray-tree frames; other scenes take the wavefront
// pipelines (rtg_wave.hip, rtg_tree.hip).
#include <type_traits>

#include "rtg_common.hpp"
#include "rtg_kernels.hpp"

namespace rtg {

// ---------------------------------------------------------------------------
// Ray tree: PerformShading (raytracer.cpp:65-134) with the recursion of
// ComputeMirrorReflection / ...Dielectric... / ...Conductor... unrolled onto an
// explicit per-thread stack.  Children are evaluated depth-first in the
// reference's order and combined with the reference's expressions, so the
// summation association is identical.
// ---------------------------------------------------------------------------
enum { FK_MIRROR = 0, FK_CONDUCTOR = 1, FK_TIR = 2, FK_DIEL = 3, FK_GI = 4 };

struct Frame {
    f3 color;          // GI + ambient + direct of this node
    f3 coef;           // mirror reflectance
    f3 refl;           // dielectric: finished reflected term
    f3 reflDir;        // dielectric: reflected direction (env lookups)
    f3 rOrigin, rDir;  // dielectric: refracted ray (unnormalised dir)
    int kind, stage;
    float ratio, rT;   // conductor ratio / dielectric rReflect, rRefract
    float rMedium, roughness;
    float selfT, selfMedium;
    int matIdx, depth;
    uint64_t key;
};
// Path-tracing frames carry more state; the Whitted kernels keep the small frame (their
// per-thread stacks live in scratch: 8 frames of ~120 B vs ~200 B).
struct FramePT : Frame {
    f3 tp;             // the node's ray.throughput (children inherit it)
    // FK_GI: the shading point, waiting for its global-illumination child
    Surf s;
    f3 w_o, giDir;
    float mbTime;
    int obj, skip;     // skip: id of the light mesh the GI ray hit (raytracer.cpp:173-175)
};
template <bool PT> using FrameT = typename std::conditional<PT, FramePT, Frame>::type;

struct Node {          // a ray that hit something, about to be shaded
    Ray r;
    Hit h;
    f3 eye;
    float medium, mbTime;
    int depth;
    uint64_t key;
    f3 tp;
};

struct Child {
    Ray r;
    float medium;
    f3 tp;
    int slot;          // RNG child slot: 0 reflected, 1 refracted, 2 global illumination
};

// PerformShading after the global-illumination term (raytracer.cpp:98-134): ambient +
// direct lighting (unless inside a medium, or path tracing without next-event
// estimation), then the material's children.  Returns true and fills `f` / `ch` if the node
// spawns a child; otherwise `out` is the node's final colour.
template <bool STATS, bool PT>
DEV bool shade_rest(const DevScene& S, const DevCamera& C, const ShadeCtx& c, f3 w_o, float medium, int depth,
                    uint64_t key, float t, float mbTime, f3 tp, f3 color, int skip, f3& out, FrameT<PT>& f, Child& ch,
                    Cnt<STATS>& cn) {
    const DevMaterial& mat = *c.mat;
    const float refractiveIndexOfVacuum = 1.00001;
    const bool inside = medium > refractiveIndexOfVacuum;
    const bool sampleDirect = !PT || C.next_event;
    if (!inside && sampleDirect) {
        color = add(color, mulv(mk(S.ambient[0], S.ambient[1], S.ambient[2]), ld3(mat.ambient)));
        color = add(color, direct<STATS, PT>(S, c, w_o, mbTime, key, cn, skip, &tp));
    }
    const f3 n = c.s.n, hp = c.s.p;
    if (mat.type == 0) {                                                // Mirror (raytracer.cpp:442-472)
        if (depth <= 0) { out = add(color, mk(0, 0, 0)); return false; }
        f.kind = FK_MIRROR;
        f.coef = ld3(mat.mirror);
        ch.r.d = reflect(n, w_o, mat.roughness, key, RP_ROUGH_REFL);
        ch.r.o = add(hp, muls(n, S.eps));
        ch.medium = 1.0f;
    } else if (mat.type == 2) {                                         // Conductor (raytracer.cpp:208-254)
        if (depth <= 0) { out = add(color, mk(0, 0, 0)); return false; }
        f3 d = neg(w_o);
        float cosTheta = -dot(d, n);
        float n2 = mat.refractive_index, k2 = mat.absorption_index;
        float n2k2 = n2 * n2 + k2 * k2;
        float n2cosTheta2 = 2 * n2 * cosTheta;
        float cosThetaSqr = cosTheta * cosTheta;
        float rs = (n2k2 - n2cosTheta2 + cosThetaSqr) / (n2k2 + n2cosTheta2 + cosThetaSqr);
        float rp = (n2k2 * cosThetaSqr - n2cosTheta2 + 1) / (n2k2 * cosThetaSqr + n2cosTheta2 + 1);
        float reflectRatio = (float)(0.5 * (rs + rp));
        if (!(reflectRatio > 0.0001)) { out = add(color, mk(0, 0, 0)); return false; }
        f.kind = FK_CONDUCTOR;
        f.coef = ld3(mat.mirror);
        f.ratio = reflectRatio;
        ch.r.d = reflect(n, w_o, mat.roughness, key, RP_ROUGH_REFL);
        ch.r.o = add(hp, muls(n, S.eps));
        ch.medium = 1.0f;
    } else if (mat.type == 1) {                                         // Dielectric (raytracer.cpp:261-415)
        if (depth <= 0) { out = add(color, mk(0, 0, 0)); return false; }
        float n1 = medium, n2 = mat.refractive_index;
        f3 d = neg(w_o);
        f3 modN = n;
        float cosTheta = -dot(d, modN);
        bool isEntering = cosTheta > 0.f;
        float objN = n2;
        if (!isEntering) {
            n1 = n2; n2 = 1.0f; objN = 1.0f;
            cosTheta = fabsf(cosTheta);
            modN = neg(modN);
        }
        float r = n1 / n2;
        float sinThetaSqr = 1 - (cosTheta * cosTheta);
        float criticalTerm = r * r * sinThetaSqr;
        if (criticalTerm > 1) {
            f.kind = FK_TIR;
            ch.r.d = reflect(modN, w_o, mat.roughness, key, RP_ROUGH_REFL);
            ch.r.o = add(hp, muls(modN, S.eps));
            ch.medium = medium;
        } else {
            float cosPhi = sqrtf(1 - criticalTerm);
            float n2cosTheta = n2 * cosTheta;
            float n1cosPhi = n1 * cosPhi;
            float rpar = (n2cosTheta - n1cosPhi) / (n2cosTheta + n1cosPhi);
            float rperp = (n1 * cosTheta - n2 * cosPhi) / (n1 * cosTheta + n2 * cosPhi);
            float rReflect = (rpar * rpar + rperp * rperp) / 2;
            f.kind = FK_DIEL;
            f.stage = 0;
            f.ratio = rReflect;
            f.rT = 1 - rReflect;
            ch.r.d = reflect(modN, w_o, mat.roughness, key, RP_ROUGH_REFL);
            ch.r.o = add(hp, muls(modN, S.eps));
            ch.medium = isEntering ? objN : 1.0f;
            f.reflDir = ch.r.d;
            f.rDir = sub(muls(add(d, muls(modN, cosTheta)), r), muls(modN, cosPhi));
            f.rOrigin = add(hp, muls(neg(modN), S.eps));
            f.rMedium = isEntering ? objN : 1.0f;
            f.roughness = mat.roughness;
        }
    } else {
        out = color;                                                    // Default material
        return false;
    }
    f.color = color;
    f.matIdx = (int)(c.mat - S.materials);
    f.depth = depth;
    f.key = key;
    f.selfT = t;
    f.selfMedium = medium;
    if constexpr (PT) f.tp = tp;
    ch.tp = tp;
    ch.slot = 0;
    return true;
}

// Shape::id of the object a GI ray hit, when its material is emissive (raytracer.cpp:171-176)
DEV int emissive_hit_id(const DevScene& S, const Hit& h, bool hit) {
    if (!hit) return -1;
    const DevObject& o = S.objects[GIDX(S, h.obj, S.num_objects, 4)];
    return S.materials[GIDX(S, o.material, S.num_materials, 5)].type == 3 ? o.id : -1;
}

// Shades `cur` (PerformShading, raytracer.cpp:65-134).  Returns true and fills `f`/`ch` if
// the node spawns a child ray (path tracing: its GI ray first); otherwise `out` is the
// node's final colour.  `level`: frames on the stack (the node's depth in the ray tree).
template <int MAXD, bool STATS, bool PT>
DEV bool shade_node(const DevScene& S, const DevCamera& C, const Node& cur, int level, f3& out, FrameT<PT>& f, Child& ch,
                    Cnt<STATS>& cn) {
    const DevObject& ob = S.objects[GIDX(S, cur.h.obj, S.num_objects, 6)];
    ShadeCtx c;
    c.ob = &ob;
    c.mat = &S.materials[GIDX(S, ob.material, S.num_materials, 7)];
    c.s = surface<STATS>(S, cur.r, cur.mbTime, cur.h, cn);
    const DevMaterial& mat = *c.mat;
    const f3 w_o = makeUnit(sub(cur.eye, c.s.p));
    if (mat.type == 3) {                                                // Emissive
        out = muls(muls(ld3(mat.radiance), 2.0f), (float)RT_PI);
        return false;
    }
    if (ob.tex_replace_all >= 0) {
        out = tex_rgb(S, S.textures[GIDX(S, ob.tex_replace_all, S.num_textures, 8)], c.s.u, c.s.v);
        return false;
    }
    f3 tp = cur.tp;
    if constexpr (PT) {
        // ComputeGlobalIllumination (raytracer.cpp:135-191) up to its IntersectObjects
        bool gi = true;
        if (C.russian_roulette) {
            float probTest = rnd(cur.key, RP_GI, 0);
            float mx = (tp.x < tp.z) ? tp.z : tp.x;                    // std::max(x, std::max(x, z))
            float maxThroughput = (tp.x < mx) ? mx : tp.x;
            if (probTest > maxThroughput && cur.depth <= 0) gi = false;
            else tp = divs(tp, maxThroughput);
        } else if (cur.depth <= 0) {
            gi = false;
        }
        if (level >= MAXD) gi = false;                                  // frame-stack bound
        if (gi) {
            float rand1 = rnd(cur.key, RP_GI, 1);
            float rand2 = rnd(cur.key, RP_GI, 2);
            float phi = (float)(2 * RT_PI * rand1);
            float theta = C.importance_sampling ? asinf(sqrtf(rand2)) : acosf(rand2);
            f3 u, v;
            onb(c.s.n, u, v);
            f3 dir = add(add(muls(muls(u, sinf(theta)), cosf(phi)), muls(c.s.n, cosf(theta))),
                         muls(muls(v, sinf(theta)), sinf(phi)));
            dir = makeUnit(dir);
            f.kind = FK_GI;
            f.s = c.s;
            f.obj = cur.h.obj;
            f.w_o = w_o;
            f.giDir = dir;
            f.tp = tp;
            f.mbTime = cur.mbTime;
            f.skip = -1;
            f.matIdx = ob.material;
            f.depth = cur.depth;
            f.key = cur.key;
            f.selfT = cur.h.t;
            f.selfMedium = cur.medium;
            ch.r.d = dir;
            ch.r.o = add(c.s.p, muls(c.s.n, 0.0001f));
            ch.medium = cur.medium;
            ch.tp = tp;
            ch.slot = 2;
            return true;
        }
        return shade_rest<STATS, PT>(S, C, c, w_o, cur.medium, cur.depth, cur.key, cur.h.t, cur.mbTime, tp,
                                     add(mk(0, 0, 0), mk(0, 0, 0)), -1, out, f, ch, cn);
    }
    return shade_rest<STATS, PT>(S, C, c, w_o, cur.medium, cur.depth, cur.key, cur.h.t, cur.mbTime, tp, mk(0, 0, 0),
                                 -1, out, f, ch, cn);
}

DEV f3 env_or_zero(const DevScene& S, f3 dir) {
    return S.num_env > 0 ? env_sample(S, 0, dir) : mk(0, 0, 0);
}

// Whole ray tree of one pixel sample; returns RenderPixel's colour
// (raytracer.cpp:38-63).  A single trace call site: the loop holds one pending ray
// (camera ray, a frame's first child, a dielectric frame's refracted child, or a path
// tracing node's GI ray).
template <int MAXD, bool STATS, bool PT>
DEV f3 render_sample(const DevScene& S, const DevCamera& C, int px, int py, uint64_t key, Cnt<STATS>& cn) {
    float mbTime;
    Ray R = camera_ray(C, px, py, key, mbTime);
    const f3 cpos = ld3(C.pos);
    cn.cam();
    // pending ray: medium, remaining depth, RNG key, throughput;
    // pend: 0 camera, 1 first child, 2 refracted, 3 global illumination
    float rMedium = 1.0f;
    int rDepth = S.max_depth;
    uint64_t rKey = key;
    f3 rTp = mk(1.0f, 1.0f, 1.0f);
    int pend = 0;

    FrameT<PT> stack[MAXD > 0 ? MAXD : 1];
    int sp = 0;
    f3 value;
    bool vHit;
    float vT = 0.f, vMedium = 1.f;
    for (;;) {
        Node cur;
        const bool hit = trace<false, STATS>(S, R, mbTime, INFINITY, INFINITY, cur.h, cn);
        if (pend == 0 && !hit) return miss_color(S, C, px, py, R.d);
        if constexpr (PT) {
            if (pend == 3) stack[GIDX(S, sp - 1, MAXD, 9)].skip = emissive_hit_id(S, cur.h, hit);
        }
        if (hit) {
            cur.r = R;
            cur.eye = pend == 0 ? cpos : R.o;
            cur.medium = rMedium;
            cur.mbTime = mbTime;
            cur.depth = rDepth;
            cur.key = rKey;
            cur.tp = rTp;
            // ---- shade; a node with children pushes a frame and continues with its first child
            Child ch;
            const bool spawn = shade_node<MAXD, STATS, PT>(S, C, cur, sp, value,
                                                           stack[MAXD > 0 ? GIDX(S, sp, MAXD, 10) : 0], ch, cn);
            if (MAXD > 0 && spawn) {
                const FrameT<PT>& f = stack[GIDX(S, sp, MAXD, 11)];
                ++sp;
                cn.sec();
                R = ch.r;
                rMedium = ch.medium;
                rDepth = f.depth - 1;
                rKey = child_key(f.key, ch.slot);
                rTp = ch.tp;
                pend = ch.slot == 2 ? 3 : 1;
                continue;
            }
            vHit = true;
            vT = cur.h.t;
            vMedium = cur.medium;
        } else {
            // a child missed (ComputeMirrorReflection :461-470, dielectric :351-356, :408 --
            // the refracted miss looks the environment up in the reflected direction; a GI
            // ray that misses contributes nothing, :169-189)
            const FrameT<PT>& f = stack[MAXD > 0 ? GIDX(S, sp - 1, MAXD, 12) : 0];
            if (f.kind == FK_MIRROR || f.kind == FK_DIEL) value = env_or_zero(S, f.kind == FK_MIRROR ? R.d : f.reflDir);
            else value = mk(0, 0, 0);
            vHit = false;
        }
        // ---- propagate finished values up the stack
        bool descended = false;
        while (MAXD > 0 && sp > 0) {
            FrameT<PT>& f = stack[GIDX(S, sp - 1, MAXD, 13)];
            if constexpr (PT) {
              if (f.kind == FK_GI) {
                // the GI ray's radiance: Shade(...) * 2 * pi (raytracer.cpp:177-188), then the
                // rest of PerformShading with colour = 0 + GI
                ShadeCtx c;
                c.ob = &S.objects[GIDX(S, f.obj, S.num_objects, 14)];
                c.mat = &S.materials[GIDX(S, f.matIdx, S.num_materials, 15)];
                c.s = f.s;
                f3 tp = f.tp;
                f3 gi = mk(0, 0, 0);
                if (vHit) gi = muls(muls(shade<true>(S, c, f.giDir, f.w_o, value, &tp), 2.0f), (float)RT_PI);
                const float selfT = f.selfT, selfMedium = f.selfMedium;
                const int depth = f.depth;
                const uint64_t nkey = f.key;
                Child ch;
                f3 out;
                if (shade_rest<STATS, PT>(S, C, c, f.w_o, selfMedium, depth, nkey, selfT, f.mbTime, tp,
                                          add(mk(0, 0, 0), gi), f.skip, out, f, ch, cn)) {
                    cn.sec();
                    R = ch.r;
                    rMedium = ch.medium;
                    rDepth = depth - 1;
                    rKey = child_key(nkey, 0);
                    rTp = ch.tp;
                    pend = 1;
                    descended = true;
                    break;
                }
                value = out;
                vHit = true;
                vT = selfT;
                vMedium = selfMedium;
                --sp;
                continue;
              }
            }
            const DevMaterial& pm = S.materials[GIDX(S, f.matIdx, S.num_materials, 16)];
            if (f.kind == FK_DIEL && f.stage == 0) {
                f.refl = (vHit && vMedium > 1.00001f) ? beer(vT, pm.absorption, value) : value;
                f.stage = 1;
                // refracted ray (raytracer.cpp:362-392)
                f3 wr = f.rDir;
                if (f.roughness > 0.001) {
                    f3 u, v;
                    onb(wr, u, v);
                    float psi1 = rnd(f.key, RP_ROUGH_REFR, 0) - 0.5f;
                    float psi2 = rnd(f.key, RP_ROUGH_REFR, 1) - 0.5f;
                    wr = makeUnit(add(wr, muls(add(muls(u, psi1), muls(v, psi2)), f.roughness)));
                } else {
                    wr = makeUnit(wr);
                }
                R.o = f.rOrigin;
                R.d = wr;
                rMedium = f.rMedium;
                rDepth = f.depth - 1;
                rKey = child_key(f.key, 1);
                if constexpr (PT) rTp = f.tp;
                pend = 2;
                cn.sec();
                descended = true;
                break;
            }
            f3 term;
            if (f.kind == FK_MIRROR) {
                term = mulv(f.coef, value);
            } else if (f.kind == FK_CONDUCTOR) {
                term = muls(vHit ? mulv(f.coef, value) : mk(0, 0, 0), f.ratio);
            } else if (f.kind == FK_TIR) {
                term = vHit ? ((vMedium > 1.0001) ? beer(vT, pm.absorption, value) : value) : mk(0, 0, 0);
            } else {
                f3 refr = (vHit && vMedium > 1.001f) ? beer(vT, pm.absorption, value) : value;
                term = add(muls(f.refl, f.ratio), muls(refr, f.rT));
            }
            value = add(f.color, term);
            vHit = true;
            vT = f.selfT;
            vMedium = f.selfMedium;
            --sp;
        }
        if (!descended) return value;
    }
}

template <int MAXD, bool STATS, bool PT>
__global__ __launch_bounds__(256, RTG_MEGA_WAVES) void k_render(DevScene S, DevCamera C, RenderParams P, float* __restrict__ hdr,
                                                unsigned char* __restrict__ ldrOut, float* __restrict__ accum,
                                                DevCounters* __restrict__ counters) {
    int px, py;
    tile_pixel(P, px, py);
    Cnt<STATS> cn;
    if (px < C.width && py < P.row_end) {
        const int pixel = px + py * C.width;
        f3 color;
        if (C.spp <= 1 && !P.accum_only) {
            color = render_sample<MAXD, STATS, PT>(S, C, px, py, root_key(P.seed, pixel, 0), cn);
        } else {
            // renderThreadMain multisampling (main.cpp:60-101): stratified jitter only
            // feeds the Gaussian weights; every sample traces the pixel centre.
            f3 acc = mk(0, 0, 0);
            float sumW = 0.0f;
            for (int s = P.sample_begin; s < P.sample_begin + P.sample_count; ++s) {
                const uint64_t key = root_key(P.seed, pixel, s);
                const float gw = sample_weight(C.spp, s, key);
                f3 col = render_sample<MAXD, STATS, PT>(S, C, px, py, key, cn);
                acc.x += col.x * gw;
                acc.y += col.y * gw;
                acc.z += col.z * gw;
                sumW += gw;
            }
            if (P.accum_only) {
                float4* a4 = reinterpret_cast<float4*>(accum);
                a4[pixel] = make_float4(acc.x, acc.y, acc.z, sumW);
                color = mk(0, 0, 0);
            } else {
                color = mk(acc.x / sumW, acc.y / sumW, acc.z / sumW);
            }
        }
        if (!P.accum_only) {
            const size_t idx = 3 * (size_t)pixel;
            if (hdr) { hdr[idx] = color.x; hdr[idx + 1] = color.y; hdr[idx + 2] = color.z; }
            if (ldrOut) { ldrOut[idx] = ldr(color.x); ldrOut[idx + 1] = ldr(color.y); ldrOut[idx + 2] = ldr(color.z); }
        }
    }
    flush_counters<STATS>(cn, counters);
}

// ---------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------
template <int MAXD, bool STATS, bool PT>
static hipError_t launch_t(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                           float* accum, DevCounters* cnt, hipStream_t stream) {
    hipLaunchKernelGGL((k_render<MAXD, STATS, PT>), dim3(P.num_tiles), dim3(256), 0, stream, S, C, P, hdr, l, accum,
                       cnt);
    return hipGetLastError();
}

int max_supported_depth() { return 32; }

template <bool STATS>
static hipError_t launch_d(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                           float* accum, DevCounters* cnt, hipStream_t stream) {
    const int d = S.max_depth;
    if (C.path_tracing) {
        // Russian roulette: unbounded GI recursion, cut at 32 ray-tree levels (the frame stack)
        if (d <= 8 && !C.russian_roulette) return launch_t<8, STATS, true>(S, C, P, hdr, l, accum, cnt, stream);
        return launch_t<32, STATS, true>(S, C, P, hdr, l, accum, cnt, stream);
    }
    if (d <= 0) return launch_t<0, STATS, false>(S, C, P, hdr, l, accum, cnt, stream);
    if (d <= 8) return launch_t<8, STATS, false>(S, C, P, hdr, l, accum, cnt, stream);
    return launch_t<32, STATS, false>(S, C, P, hdr, l, accum, cnt, stream);
}

static hipError_t launch_any(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                             float* accum, DevCounters* cnt, bool stats, hipStream_t stream) {
    return stats ? launch_d<true>(S, C, P, hdr, l, accum, cnt, stream)
                 : launch_d<false>(S, C, P, hdr, l, accum, cnt, stream);
}

hipError_t launch_mega(const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr, unsigned char* l,
                       float* accum, DevCounters* cnt, bool stats, hipStream_t stream, hipEvent_t* ev) {
    if (ev) (void)hipEventRecord(ev[0], stream);
    hipError_t e = launch_any(S, C, P, hdr, l, accum, cnt, stats, stream);
    if (ev) (void)hipEventRecord(ev[1], stream);
    return e;
}

}  // namespace rtg
