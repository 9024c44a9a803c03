// Fused ("mega") render kernel: one thread per pixel walks the pixel's whole ray tree
// -- PerformShading (raytracer.cpp:65-134) with the recursion of ComputeMirrorReflection /
// ...Dielectric... / ...Conductor... and, for path-tracing cameras, ComputeGlobalIllumination
// (raytracer.cpp:135-191) unrolled onto an explicit per-thread stack.  Used for path
// tracing, motion blur and small ray-tree frames; other scenes take the wavefront
// pipelines (rtg_wave.hip, rtg_tree.hip).
#include "rtg_common.hpp"
#include "rtg_kernels.hpp"
#include "rtg_node.hpp"

namespace rtg {

// ---------------------------------------------------------------------------
// Whole ray tree of one pixel sample; returns RenderPixel's colour
// (raytracer.cpp:38-63).  A single trace call site: the loop holds one pending ray
// (camera ray, a frame's first child, a dielectric frame's refracted child, or a path
// tracing node's GI ray).  The node steps (shade_node, resume_frame) are rtg_node.hpp's,
// shared with the wavefront path-tracing pipeline.
template <int MAXD, bool STATS, bool PT>
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
        const bool hit = trace<false, STATS>(S, p.R, mbTime, INFINITY, INFINITY, cur.h, cn);
        if (p.pend == 0 && !hit) return miss_color(S, C, px, py, p.R.d);
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
            const bool spawn = shade_node<MAXD, STATS, PT>(S, C, cur, sp, v.value,
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
            v.value = miss_value<PT>(S, stack[MAXD > 0 ? GIDX(S, sp - 1, MAXD, 12) : 0], p.R.d);
            v.hit = false;
        }
        // ---- propagate finished values up the stack
        bool descended = false;
        while (MAXD > 0 && sp > 0) {
            if (resume_frame<STATS, PT>(S, C, stack[GIDX(S, sp - 1, MAXD, 13)], v, p, cn)) {
                descended = true;
                break;
            }
            --sp;
        }
        if (!descended) return v.value;
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
