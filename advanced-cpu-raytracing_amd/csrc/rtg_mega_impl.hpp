// The fused kernel's device code (rtg_mega.hip, rtg_mega_pt.hip): one thread per pixel walks
// the pixel's whole ray tree -- PerformShading (raytracer.cpp:65-134) with the recursion of
// ComputeMirrorReflection / ...Dielectric... / ...Conductor... and, for path-tracing cameras,
// ComputeGlobalIllumination (raytracer.cpp:135-191) unrolled onto an explicit per-thread stack.
#pragma once

#include "rtg_common.hpp"
#include "rtg_node.hpp"

namespace rtg {

// ---------------------------------------------------------------------------
// Whole ray tree of one pixel sample; returns RenderPixel's colour
// (raytracer.cpp:38-63).  A single trace call site: the loop holds one pending ray
// (camera ray, a frame's first child, a dielectric frame's refracted child, or a path
// tracing node's GI ray).  The node steps (shade_node, resume_frame) are rtg_node.hpp's,
// shared with the wavefront path-tracing pipeline.
// SK / FEAT: the scene's shading and traversal features (a superset; the path-tracing
// variants of rtg_mega_pt.hip), everything by default.
template <int MAXD, bool STATS, bool PT, int SK = SK_ALL, int FEAT = FEAT_ALL>
DEV f3 render_sample(const DevScene& S, const DevCamera& C, int px, int py, uint64_t key, Cnt<STATS>& cn) {
    float mbTime;
    Pending p;
    p.R = camera_ray(C, px, py, key, mbTime);
    const f3 cpos = ld3(C.pos);
    cn.cam();
    p.medium = 1.0f;
    p.depth = S.max_depth;
    p.key = key;
    p.tp = mk(1.0f, 1.0f, 1.0f);
    p.pend = 0;

    FrameT<PT> stack[MAXD > 0 ? MAXD : 1];
    int sp = 0;
    ChildVal v;
    v.t = 0.f;
    v.medium = 1.f;
    for (;;) {
        Node cur;
        const bool hit = trace<false, STATS, FEAT>(S, p.R, mbTime, INFINITY, INFINITY, cur.h, cn);
        if (p.pend == 0 && !hit) return miss_color<SK>(S, C, px, py, p.R.d);
        if constexpr (PT) {
            if (p.pend == 3) stack[GIDX(S, sp - 1, MAXD, 9)].skip = emissive_hit_id(S, cur.h, hit);
        }
        if (hit) {
            cur.r = p.R;
            cur.eye = p.pend == 0 ? cpos : p.R.o;
            cur.medium = p.medium;
            cur.mbTime = mbTime;
            cur.depth = p.depth;
            cur.key = p.key;
            cur.tp = p.tp;
            // ---- shade; a node with children pushes a frame and continues with its first child
            Child ch;
            const bool spawn = shade_node<MAXD, STATS, PT, SK, FEAT>(S, C, cur, sp, v.value,
                                                           stack[MAXD > 0 ? GIDX(S, sp, MAXD, 10) : 0], ch, cn);
            if (MAXD > 0 && spawn) {
                spawn_child<STATS, PT>(stack[GIDX(S, sp, MAXD, 11)], ch, p, cn);
                ++sp;
                continue;
            }
            v.hit = true;
            v.t = cur.h.t;
            v.medium = cur.medium;
        } else {
            v.value = miss_value<PT, SK>(S, stack[MAXD > 0 ? GIDX(S, sp - 1, MAXD, 12) : 0], p.R.d);
            v.hit = false;
        }
        // ---- propagate finished values up the stack
        bool descended = false;
        while (MAXD > 0 && sp > 0) {
            if (resume_frame<STATS, PT, SK, FEAT>(S, C, stack[GIDX(S, sp - 1, MAXD, 13)], v, p, cn)) {
                descended = true;
                break;
            }
            --sp;
        }
        if (!descended) return v.value;
    }
}

template <int MAXD, bool STATS, bool PT, int SK = SK_ALL, int FEAT = FEAT_ALL>
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
            color = render_sample<MAXD, STATS, PT, SK, FEAT>(S, C, px, py, root_key(P.seed, pixel, 0), cn);
        } else {
            // renderThreadMain multisampling (main.cpp:60-101): stratified jitter only
            // feeds the Gaussian weights; every sample traces the pixel centre.
            f3 acc = mk(0, 0, 0);
            float sumW = 0.0f;
            for (int s = P.sample_begin; s < P.sample_begin + P.sample_count; ++s) {
                const uint64_t key = root_key(P.seed, pixel, s);
                const float gw = sample_weight(C.spp, s, key);
                f3 col = render_sample<MAXD, STATS, PT, SK, FEAT>(S, C, px, py, key, cn);
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

}  // namespace rtg
