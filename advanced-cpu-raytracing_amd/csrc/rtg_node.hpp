// Ray-tree nodes shared by the fused kernel (rtg_mega.hip) and the wavefront path-tracing
// pipeline (rtg_path.hip): the frame kinds of PerformShading's recursion and the node shading
// steps, so both evaluate every node with the same code.
#pragma once

#include <type_traits>

#include "rtg_common.hpp"

namespace rtg {

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
template <bool STATS, bool PT, int SK = SK_ALL, int FEAT = FEAT_ALL>
DEV bool shade_rest(const DevScene& S, const DevCamera& C, const ShadeCtx& c, f3 w_o, float medium, int depth,
                    uint64_t key, float t, float mbTime, f3 tp, f3 color, int skip, f3& out, FrameT<PT>& f, Child& ch,
                    Cnt<STATS>& cn) {
    const DevMaterial& mat = *c.mat;
    const float refractiveIndexOfVacuum = 1.00001;
    const bool inside = medium > refractiveIndexOfVacuum;
    const bool sampleDirect = !PT || C.next_event;
    if (!inside && sampleDirect) {
        color = add(color, mulv(mk(S.ambient[0], S.ambient[1], S.ambient[2]), ld3(mat.ambient)));
        color = add(color, direct<STATS, PT, SK, FEAT>(S, c, w_o, mbTime, key, cn, skip, &tp));
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

// The arguments of a pending shade_rest call: a node past its global-illumination term
// (raytracer.cpp:98-134 with colour = GI so far).
struct RestArgs {
    ShadeCtx c;
    f3 w_o;
    float medium;
    int depth;
    uint64_t key;
    float t, mbTime;
    f3 tp, color;
    int skip;
};
enum { NS_DONE = 0, NS_SPAWN = 1, NS_REST = 2 };

// Shades `cur` (PerformShading, raytracer.cpp:65-134) up to shade_rest.  Returns NS_DONE
// (`out` = the node's final colour: emissive, replace_all), NS_SPAWN (path tracing: the GI ray
// in `f`/`ch`) or NS_REST (`a`: the shade_rest call that finishes the node).  `level`: frames
// on the stack (the node's depth in the ray tree).
// maxd: the frame-stack bound (levels); SK: shading features the scene may use.
template <bool STATS, bool PT, int SK = SK_ALL>
DEV int shade_node_pre(const DevScene& S, const DevCamera& C, const Node& cur, int level, int maxd, f3& out,
                       FrameT<PT>& f, Child& ch, RestArgs& a, Cnt<STATS>& cn) {
    const DevObject& ob = S.objects[GIDX(S, cur.h.obj, S.num_objects, 6)];
    ShadeCtx c;
    c.ob = &ob;
    c.mat = &S.materials[GIDX(S, ob.material, S.num_materials, 7)];
    c.s = surface<STATS, (SK & SK_TEX) != 0>(S, cur.r, cur.mbTime, cur.h, cn);
    const DevMaterial& mat = *c.mat;
    const f3 w_o = makeUnit(sub(cur.eye, c.s.p));
    if (mat.type == 3) {                                                // Emissive
        out = muls(muls(ld3(mat.radiance), 2.0f), (float)RT_PI);
        return NS_DONE;
    }
    if ((SK & SK_TEX) && ob.tex_replace_all >= 0) {
        out = tex_rgb(S, S.textures[GIDX(S, ob.tex_replace_all, S.num_textures, 8)], c.s.u, c.s.v);
        return NS_DONE;
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
        if (level >= maxd) gi = false;                                  // frame-stack bound
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
            return NS_SPAWN;
        }
    }
    a.c = c;
    a.w_o = w_o;
    a.medium = cur.medium;
    a.depth = cur.depth;
    a.key = cur.key;
    a.t = cur.h.t;
    a.mbTime = cur.mbTime;
    a.tp = tp;
    a.color = PT ? add(mk(0, 0, 0), mk(0, 0, 0)) : mk(0, 0, 0);
    a.skip = -1;
    return NS_REST;
}

template <bool STATS, bool PT, int SK = SK_ALL, int FEAT = FEAT_ALL>
DEV bool rest_call(const DevScene& S, const DevCamera& C, const RestArgs& a, f3& out, FrameT<PT>& f, Child& ch,
                   Cnt<STATS>& cn) {
    return shade_rest<STATS, PT, SK, FEAT>(S, C, a.c, a.w_o, a.medium, a.depth, a.key, a.t, a.mbTime, a.tp, a.color, a.skip,
                                 out, f, ch, cn);
}

// shade_node_pre + its shade_rest: returns true and fills `f`/`ch` if the node spawns a child
// ray (path tracing: its GI ray first); otherwise `out` is the node's final colour.
template <int MAXD, bool STATS, bool PT, int SK = SK_ALL, int FEAT = FEAT_ALL>
DEV bool shade_node(const DevScene& S, const DevCamera& C, const Node& cur, int level, f3& out, FrameT<PT>& f, Child& ch,
                    Cnt<STATS>& cn) {
    RestArgs a;
    const int r = shade_node_pre<STATS, PT, SK>(S, C, cur, level, MAXD, out, f, ch, a, cn);
    if (r != NS_REST) return r == NS_SPAWN;
    return rest_call<STATS, PT, SK, FEAT>(S, C, a, out, f, ch, cn);
}

template <int SK = SK_ALL>
DEV f3 env_or_zero(const DevScene& S, f3 dir) {
    return ((SK & SK_XLIGHT) && S.num_env > 0) ? env_sample(S, 0, dir) : mk(0, 0, 0);
}

// The pending ray of a walk: the ray, its medium, remaining depth, RNG key, throughput and
// which child it is (0 camera ray, 1 a frame's first child, 2 a dielectric frame's refracted
// child, 3 a path-tracing node's GI ray).
struct Pending {
    Ray R;
    float medium;
    int depth;
    uint64_t key;
    f3 tp;
    int pend;
};

// A finished node handed to its parent frame: its colour, whether its ray hit something, and
// its hit distance and medium (Beer's law on the parent's side).
struct ChildVal {
    f3 value;
    bool hit;
    float t, medium;
};

// The child `ch` of frame `f` (just filled by shade_node / shade_rest) becomes the pending ray.
template <bool STATS, bool PT>
DEV void spawn_child(const FrameT<PT>& f, const Child& ch, Pending& p, Cnt<STATS>& cn) {
    cn.sec();
    p.R = ch.r;
    p.medium = ch.medium;
    p.depth = f.depth - 1;
    p.key = child_key(f.key, ch.slot);
    p.tp = ch.tp;
    p.pend = ch.slot == 2 ? 3 : 1;
}

// The value of a child ray of frame `f` that missed (ComputeMirrorReflection :461-470,
// dielectric :351-356, :408 -- the refracted miss looks the environment up in the reflected
// direction; a GI ray that misses contributes nothing, :169-189).  `dir`: the child's direction.
template <bool PT, int SK = SK_ALL>
DEV f3 miss_value(const DevScene& S, const FrameT<PT>& f, f3 dir) {
    if (f.kind == FK_MIRROR || f.kind == FK_DIEL) return env_or_zero<SK>(S, f.kind == FK_MIRROR ? dir : f.reflDir);
    return mk(0, 0, 0);
}

// Resumes frame `f` once its pending child finished with `v`, up to shade_rest.  Returns
// NS_SPAWN (a dielectric frame's refracted child is the pending ray `p`; `f` updated in place,
// it stays on the stack), NS_DONE (`v` = the frame's value, the frame is popped) or NS_REST
// (a path-tracing frame whose GI ray finished: `a`, the shade_rest call that goes on with the
// frame -- which writes `f` anew).
template <bool STATS, bool PT, int SK = SK_ALL>
DEV int resume_pre(const DevScene& S, const DevCamera& C, FrameT<PT>& f, ChildVal& v, Pending& p, RestArgs& a,
                   Cnt<STATS>& cn) {
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
            if (v.hit) gi = muls(muls(shade<true, SK>(S, c, f.giDir, f.w_o, v.value, &tp), 2.0f), (float)RT_PI);
            a.c = c;
            a.w_o = f.w_o;
            a.medium = f.selfMedium;
            a.depth = f.depth;
            a.key = f.key;
            a.t = f.selfT;
            a.mbTime = f.mbTime;
            a.tp = tp;
            a.color = add(mk(0, 0, 0), gi);
            a.skip = f.skip;
            return NS_REST;
        }
    }
    const DevMaterial& pm = S.materials[GIDX(S, f.matIdx, S.num_materials, 16)];
    if (f.kind == FK_DIEL && f.stage == 0) {
        f.refl = (v.hit && v.medium > 1.00001f) ? beer(v.t, pm.absorption, v.value) : v.value;
        f.stage = 1;
        // refracted ray (raytracer.cpp:362-392)
        f3 wr = f.rDir;
        if (f.roughness > 0.001) {
            f3 u, w;
            onb(wr, u, w);
            float psi1 = rnd(f.key, RP_ROUGH_REFR, 0) - 0.5f;
            float psi2 = rnd(f.key, RP_ROUGH_REFR, 1) - 0.5f;
            wr = makeUnit(add(wr, muls(add(muls(u, psi1), muls(w, psi2)), f.roughness)));
        } else {
            wr = makeUnit(wr);
        }
        p.R.o = f.rOrigin;
        p.R.d = wr;
        p.medium = f.rMedium;
        p.depth = f.depth - 1;
        p.key = child_key(f.key, 1);
        if constexpr (PT) p.tp = f.tp;
        p.pend = 2;
        cn.sec();
        return NS_SPAWN;
    }
    f3 term;
    if (f.kind == FK_MIRROR) {
        term = mulv(f.coef, v.value);
    } else if (f.kind == FK_CONDUCTOR) {
        term = muls(v.hit ? mulv(f.coef, v.value) : mk(0, 0, 0), f.ratio);
    } else if (f.kind == FK_TIR) {
        term = v.hit ? ((v.medium > 1.0001) ? beer(v.t, pm.absorption, v.value) : v.value) : mk(0, 0, 0);
    } else {
        f3 refr = (v.hit && v.medium > 1.001f) ? beer(v.t, pm.absorption, v.value) : v.value;
        term = add(muls(f.refl, f.ratio), muls(refr, f.rT));
    }
    v.value = add(f.color, term);
    v.hit = true;
    v.t = f.selfT;
    v.medium = f.selfMedium;
    return NS_DONE;
}

// A node finished by shade_rest (`spawned`: its first material child in `f`/`ch`): the child
// becomes the pending ray, or the node's colour `out` the finished value `v`.
template <bool STATS, bool PT>
DEV void rest_done(bool spawned, const RestArgs& a, const FrameT<PT>& f, const Child& ch, f3 out, Pending& p,
                   ChildVal& v, Cnt<STATS>& cn) {
    if (spawned) {
        spawn_child<STATS, PT>(f, ch, p, cn);
        return;
    }
    v.value = out;
    v.hit = true;
    v.t = a.t;
    v.medium = a.medium;
}

// resume_pre + its shade_rest: returns true if the frame spawns its next child (the pending
// ray `p`; `f` stays on the stack), false if it is finished (`v` = its value).
template <bool STATS, bool PT, int SK = SK_ALL, int FEAT = FEAT_ALL>
DEV bool resume_frame(const DevScene& S, const DevCamera& C, FrameT<PT>& f, ChildVal& v, Pending& p, Cnt<STATS>& cn) {
    RestArgs a;
    const int r = resume_pre<STATS, PT, SK>(S, C, f, v, p, a, cn);
    if (r != NS_REST) return r == NS_SPAWN;
    Child ch;
    f3 out;
    const bool spawned = rest_call<STATS, PT, SK, FEAT>(S, C, a, out, f, ch, cn);
    rest_done<STATS, PT>(spawned, a, f, ch, out, p, v, cn);
    return spawned;
}

}  // namespace rtg
