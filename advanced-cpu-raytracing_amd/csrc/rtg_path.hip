// Wavefront path tracing: PerformShading with ComputeGlobalIllumination (raytracer.cpp:65-191)
// for path-tracing cameras, as iterations over compacted queues of paths instead of one thread
// walking a pixel's whole ray tree (the fused kernel, rtg_mega.hip, keeps up to 32 frames of
// ~200 B per thread in registers and scratch, at two waves per SIMD).
//
// A path is one pixel sample's walk of its ray tree: a pending ray and a stack of frames (the
// nodes waiting for a child).  The stacks live in HBM, one 208-byte frame per level, chunked in
// float4 planes so a wave's loads of one chunk are contiguous.  Per sample pass:
//
//   k_path_gen    the camera rays (GenerateRay, raytracer.cpp:661-699), every path active
//   per iteration (until no path is active):
//     k_path_trace  closest hit of every active path's pending ray (lean traversal kernel)
//     k_path_step   the rest of the fused kernel's loop body for each active path: shade the
//                   hit node (shade_node: the GI ray, or ambient + direct lighting with its
//                   shadow rays + the material's child), or hand the child's value up the
//                   stack (resume_frame) until a frame spawns its next child; paths with a
//                   new pending ray are appended to the next iteration's queue, finished
//                   ones write their pixel (or the spp accumulation, in sample order)
//
// The node steps are rtg_node.hpp's, the same code the fused kernel runs, with the same RNG
// keys, so the image is bit-identical to the fused kernel's.
//
// (Round 4's split step -- three kernels by node kind at two waves per SIMD each -- was
// bit-identical and slower, pt_cornell 2 588 -> 1 441 Mrays/s, profiles/r04v_ptwave_split.txt:
// every unwinding level that needs shade_rest cost an iteration of four launches where the single
// kernel unwinds in place; removed in round 6.)
//
// Path regeneration (cameras with Russian roulette; RTG_PATH_REGEN=1 / 0
// forces it on / off): a pass covers all of the render's samples.  Path slot i is pixel i of the chunk; when
// its sample finishes, the step kernel accumulates it and starts the slot's next sample (its
// camera ray) in the same iteration, so the queue stays full until the last samples and each
// pixel's samples are still summed in sample order (one slot does them one after another).  A
// per-sample pass instead ends in the tail of its few longest paths (pt_rr: Russian-roulette
// chains), once per sample.  Without Russian roulette there is no such tail, and mixing the
// samples' stages in one queue costs more than it saves: a wave whose lanes sit at different
// depths pays for every lane's unwinding of its stack each iteration (1024^2 x 16 spp: pt_rr
// 1 048 -> 1 405 Mrays/s with regeneration, pt_cornell 2 642 -> 1 725, pt_nee 3 629 -> 1 871;
// profiles/r05p_ptwave_regen.txt).
//
// Iterations are host-driven on a plan's first pass (each iteration's queue size comes back
// to the host); the sizes seen become the plan of later passes, which launch every iteration
// with no host synchronisation (grid-stride kernels read the queue size on the device).  A
// planned pass with paths left after its last iteration sets an overflow flag, checked once
// per render; the render is then redone host-driven.
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rtg_common.hpp"
#include "rtg_kernels.hpp"
#include "rtg_node.hpp"

#ifndef RTG_PATH_STEP_WAVES
#define RTG_PATH_STEP_WAVES 1
#endif

namespace rtg {

constexpr int kFrameChunks = (int)((sizeof(FramePT) + 15) / 16);
constexpr int kPathMaxIter = 4096;           // iterations per pass (the fused kernel beyond)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winvalid-offsetof"
constexpr int kSkipOffset = (int)offsetof(FramePT, skip);
#pragma clang diagnostic pop
static_assert(kSkipOffset % 4 == 0, "FramePT::skip alignment");

struct PathBufs {
    // pending ray by path: origin + medium, direction + remaining depth (int bits), RNG key,
    // throughput + (pend | stack depth << 8 | sample within the pass << 16) (int bits)
    float4* ro;
    float4* rd;
    unsigned long long* key;
    float4* tp;
    float4* frames;     // chunk k of the level-lv frame of path i: frames[(lv * kFrameChunks + k) * cap + i]
    int* act0;          // queues of active paths (even / odd iterations)
    int* act1;
    int* cnt;           // per iteration: active paths; [kPathMaxIter + 1]: overflow flag
    float* ht;          // closest hits by queue position
    int* hobj;
    int* hface;
    int cap;            // paths per pass
};

DEV size_t chunk_at(const PathBufs& B, int lv, int k, int i) {
    return ((size_t)lv * kFrameChunks + k) * (size_t)B.cap + i;
}

DEV void frame_store(const PathBufs& B, int lv, int i, const FramePT& f) {
    float4 t[kFrameChunks];
    __builtin_memcpy(t, &f, sizeof(FramePT));
#pragma unroll
    for (int k = 0; k < kFrameChunks; ++k) B.frames[chunk_at(B, lv, k, i)] = t[k];
}

DEV void frame_load(const PathBufs& B, int lv, int i, FramePT& f) {
    float4 t[kFrameChunks];
#pragma unroll
    for (int k = 0; k < kFrameChunks; ++k) t[k] = B.frames[chunk_at(B, lv, k, i)];
    __builtin_memcpy(&f, t, sizeof(FramePT));
}

// FramePT::skip of the level-lv frame (the GI ray's emissive hit, raytracer.cpp:171-176)
DEV void frame_store_skip(const PathBufs& B, int lv, int i, int skip) {
    float4* c = &B.frames[chunk_at(B, lv, kSkipOffset / 16, i)];
    reinterpret_cast<int*>(c)[(kSkipOffset % 16) / 4] = skip;
}

// the path's sample finished with `value`: its pixel, or the spp accumulation (in sample order)
DEV void path_pixel(const DevCamera& C, const RenderParams& P, int sample, int first, int last, int pixel, f3 value,
                    float* __restrict__ hdr, unsigned char* __restrict__ ldrOut, float4* __restrict__ accum) {
    if (C.spp <= 1 && !P.accum_only) {
        const size_t idx = 3 * (size_t)pixel;
        if (hdr) { hdr[idx] = value.x; hdr[idx + 1] = value.y; hdr[idx + 2] = value.z; }
        if (ldrOut) { ldrOut[idx] = ldr(value.x); ldrOut[idx + 1] = ldr(value.y); ldrOut[idx + 2] = ldr(value.z); }
    } else {
        // renderThreadMain multisampling (main.cpp:60-101), samples summed in order
        const float gw = sample_weight(C.spp, sample, root_key(P.seed, pixel, sample));
        float4 a = first ? make_float4(0.f, 0.f, 0.f, 0.f) : accum[pixel];
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
}

// path i's camera ray (GenerateRay, raytracer.cpp:661-699) for `sample`, the k-th of its pass
template <bool STATS>
DEV void path_camera(const DevCamera& C, const RenderParams& P, const PathBufs& B, int sample, int k, int pixel,
                     int i, int max_depth, Cnt<STATS>& cn) {
    const uint64_t key = root_key(P.seed, pixel, sample);
    float mbTime;
    const Ray r = camera_ray(C, pixel % C.width, pixel / C.width, key, mbTime);
    cn.cam();
    B.ro[i] = make_float4(r.o.x, r.o.y, r.o.z, 1.0f);
    B.rd[i] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(max_depth));
    B.key[i] = key;
    B.tp[i] = make_float4(1.0f, 1.0f, 1.0f, __int_as_float(k << 16));
}

template <bool STATS>
__global__ __launch_bounds__(256) void k_path_gen(const DevCamera C, const RenderParams P, const PathBufs B,
                                                  const int sample, const int base, const int n, const int max_depth,
                                                  DevCounters* counters) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    Cnt<STATS> cn;
    if (i < n) {
        path_camera<STATS>(C, P, B, sample, 0, part_pixel(P, C.width, base + i), i, max_depth, cn);
        B.act0[i] = i;
        if (i == 0) B.cnt[0] = n;
    }
    flush_counters<STATS>(cn, counters);
}

template <bool STATS, int FEAT>
__global__ __launch_bounds__(256, RTG_TRACE_WAVES(FEAT)) void k_path_trace(const DevScene S, const PathBufs B,
                                                                           const int it, DevCounters* counters) {
    const int* act = (it & 1) ? B.act1 : B.act0;
    const int n = B.cnt[it];
    Cnt<STATS> cn;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int path = act[i];
        const float4 o = B.ro[path], d = B.rd[path];
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        Hit h;
        trace<false, STATS, FEAT>(S, r, 0.f, INFINITY, INFINITY, h, cn);
        B.ht[i] = h.t;
        B.hobj[i] = h.obj;
        B.hface[i] = h.face;
    }
    flush_counters<STATS>(cn, counters);
}

// One iteration of render_sample's loop (rtg_mega.hip) after its trace, per active path.
// SK / FEAT: the scene's shading and traversal features (a superset of them); maxd: the frame
// levels (the fused kernel's MAXD).  The pass runs samples [sample, sample + count) of each
// path, the render samples [first, last].
template <bool STATS, int SK, int FEAT>
__global__ __launch_bounds__(256, RTG_PATH_STEP_WAVES) void k_path_step(
    const DevScene S, const DevCamera C, const RenderParams P, const PathBufs B, const int it, const int sample,
    const int first, const int last, const int count, const int base, const int maxd, float* __restrict__ hdr,
    unsigned char* __restrict__ ldrOut, float4* __restrict__ accum, DevCounters* counters) {
    const int* act = (it & 1) ? B.act1 : B.act0;
    int* nact = (it & 1) ? B.act0 : B.act1;
    const int n = B.cnt[it];
    const f3 cpos = ld3(C.pos);
    Cnt<STATS> cn;
    for (int i0 = blockIdx.x * 256; i0 < n; i0 += gridDim.x * 256) {
        const int i = i0 + threadIdx.x;
        bool cont = false;
        int path = 0;
        if (i < n) {
            path = act[i];
            const float4 o = B.ro[path], d = B.rd[path], t4 = B.tp[path];
            Pending p;
            p.R.o = mk(o.x, o.y, o.z);
            p.R.d = mk(d.x, d.y, d.z);
            p.medium = o.w;
            p.depth = __float_as_int(d.w);
            p.key = B.key[path];
            p.tp = mk(t4.x, t4.y, t4.z);
            const int ps = __float_as_int(t4.w);
            p.pend = ps & 255;
            int sp = (ps >> 8) & 255;
            const int k = ps >> 16;
            Node cur;
            cur.h.t = B.ht[i];
            cur.h.obj = B.hobj[i];
            cur.h.face = B.hface[i];
            cur.h.o = p.R.o;
            const bool hit = cur.h.obj >= 0;
            const int pixel = part_pixel(P, C.width, base + path);
            ChildVal v;
            v.t = 0.f;
            v.medium = 1.f;
            bool done = true;
            if (p.pend == 0 && !hit) {
                v.value = miss_color<SK>(S, C, pixel % C.width, pixel / C.width, p.R.d);
            } else {
                if (p.pend == 3) frame_store_skip(B, sp - 1, path, emissive_hit_id(S, cur.h, hit));
                // one shade_rest call site for the hit node and for resumed GI frames: `rest`
                // pending for the frame at level restLevel (sp: the hit node, pushed if it
                // spawns; sp - 1: a resumed frame, popped if it does not)
                FramePT f;
                RestArgs a;
                bool have = false, descended = false, rest = false;
                int restLevel = 0;
                if (hit) {
                    cur.r = p.R;
                    cur.eye = p.pend == 0 ? cpos : p.R.o;
                    cur.medium = p.medium;
                    cur.mbTime = 0.f;
                    cur.depth = p.depth;
                    cur.key = p.key;
                    cur.tp = p.tp;
                    Child ch;
                    const int r = shade_node_pre<STATS, true, SK>(S, C, cur, sp, maxd, v.value, f, ch, a, cn);
                    if (r == NS_SPAWN) {
                        spawn_child<STATS, true>(f, ch, p, cn);
                        frame_store(B, sp, path, f);
                        ++sp;
                        descended = true;
                    } else if (r == NS_REST) {
                        rest = true;
                        restLevel = sp;
                    } else {
                        v.hit = true;
                        v.t = cur.h.t;
                        v.medium = cur.medium;
                    }
                } else {
                    frame_load(B, sp - 1, path, f);
                    have = true;
                    v.value = miss_value<true, SK>(S, f, p.R.d);
                    v.hit = false;
                }
                // ---- finish nodes and hand finished values up the stack
                while (!descended) {
                    if (rest) {
                        rest = false;
                        Child ch;
                        f3 out;
                        const bool spawned = rest_call<STATS, true, SK, FEAT>(S, C, a, out, f, ch, cn);
                        rest_done<STATS, true>(spawned, a, f, ch, out, p, v, cn);
                        sp = restLevel;
                        if (spawned) {
                            frame_store(B, restLevel, path, f);
                            ++sp;
                            descended = true;
                            break;
                        }
                    }
                    if (sp == 0) break;
                    if (!have) frame_load(B, sp - 1, path, f);
                    have = false;
                    const int r = resume_pre<STATS, true, SK>(S, C, f, v, p, a, cn);
                    if (r == NS_SPAWN) {
                        frame_store(B, sp - 1, path, f);
                        descended = true;
                    } else if (r == NS_REST) {
                        rest = true;
                        restLevel = sp - 1;
                    } else {
                        --sp;
                    }
                }
                done = !descended;
            }
            if (done) {
                const int s = sample + k;
                path_pixel(C, P, s, s == first, s == last, pixel, v.value, hdr, ldrOut, accum);
                // regeneration: the slot's next sample
                if (k + 1 < count) {
                    path_camera<STATS>(C, P, B, s + 1, k + 1, pixel, path, S.max_depth, cn);
                    cont = true;
                }
            } else {
                B.ro[path] = make_float4(p.R.o.x, p.R.o.y, p.R.o.z, p.medium);
                B.rd[path] = make_float4(p.R.d.x, p.R.d.y, p.R.d.z, __int_as_float(p.depth));
                B.key[path] = p.key;
                B.tp[path] = make_float4(p.tp.x, p.tp.y, p.tp.z, __int_as_float(p.pend | (sp << 8) | (k << 16)));
                cont = true;
            }
        }
        // wave-aggregated append to the next iteration's queue
        const unsigned long long mask = __ballot(cont);
        if (mask) {
            const int lane = threadIdx.x & 63;
            const int leader = __ffsll((long long)mask) - 1;
            int qb = 0;
            if (lane == leader) qb = atomicAdd(&B.cnt[it + 1], __popcll(mask));
            qb = __shfl(qb, leader);
            if (cont) nact[qb + __popcll(mask & ((1ull << lane) - 1ull))] = path;
        }
    }
    flush_counters<STATS>(cn, counters);
}

// paths left after a planned pass's last iteration: the plan was too short
__global__ void k_path_check(int* cnt, int last_it) {
    if (threadIdx.x == 0 && cnt[last_it] != 0) cnt[kPathMaxIter + 1] = 1;
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct PathState {
    PathBufs B{};
    size_t cap = 0;                 // paths the buffers hold
    int levels = 0;                 // frame levels the buffers hold
    int* h = nullptr;               // pinned host words: [0] a queue size, [1] the overflow flag
    std::vector<int> plan;          // grid paths per iteration of planned passes
    std::vector<long long> plan_key;
    ~PathState() { release(); if (h) (void)hipHostFree(h); }
    void release() {
        auto f = [](void* p) { if (p) (void)hipFree(p); };
        f(B.ro); f(B.rd); f(B.key); f(B.tp); f(B.frames); f(B.act0); f(B.act1); f(B.cnt); f(B.ht); f(B.hobj);
        f(B.hface);
        B = PathBufs{};
        cap = 0;
        levels = 0;
    }
};

void path_destroy(PathState* t) { delete t; }

static hipError_t ensure_paths(PathState& T, size_t n, int levels) {
    if (T.cap >= n && T.levels >= levels) return hipSuccess;
    n = std::max(n, T.cap);
    levels = std::max(levels, T.levels);
    T.release();
    hipError_t e;
    // an allocation that fails leaves the render to the fused kernel (hipErrorNotSupported)
#define A_(ptr, bytes)                                  \
    if ((e = hipMalloc(&ptr, bytes)) != hipSuccess) {   \
        (void)hipGetLastError();                        \
        T.release();                                    \
        return hipErrorNotSupported;                    \
    }
    A_(T.B.ro, n * 16); A_(T.B.rd, n * 16); A_(T.B.key, n * 8); A_(T.B.tp, n * 16);
    A_(T.B.frames, n * (size_t)levels * kFrameChunks * 16);
    A_(T.B.act0, n * 4); A_(T.B.act1, n * 4); A_(T.B.cnt, (kPathMaxIter + 2) * sizeof(int));
    A_(T.B.ht, n * 4); A_(T.B.hobj, n * 4); A_(T.B.hface, n * 4);
#undef A_
    T.B.cap = (int)n;
    T.cap = n;
    T.levels = levels;
    return hipSuccess;
}

static int grid_for(long long paths) { return (int)std::max(1ll, std::min((paths + 255) / 256, 1ll << 16)); }

using GenFn = void (*)(const DevCamera, const RenderParams, const PathBufs, const int, const int, const int, const int,
                       DevCounters*);
using TraceFn = void (*)(const DevScene, const PathBufs, const int, DevCounters*);
using StepFn = void (*)(const DevScene, const DevCamera, const RenderParams, const PathBufs, const int, const int,
                        const int, const int, const int, const int, const int, float*, unsigned char*, float4*,
                        DevCounters*);
struct PathKernels {
    GenFn gen;
    TraceFn trace;
    StepFn step;
};

// Iterations a pass may take: kPathMaxIter, or fewer with RTG_PATH_ITER_CAP (tests: the bound
// reached by short passes)
static int path_iter_cap() {
    const char* v = std::getenv("RTG_PATH_ITER_CAP");
    const int c = v ? std::atoi(v) : kPathMaxIter;
    return c > 0 && c < kPathMaxIter ? c : kPathMaxIter;
}

// One pass over paths [base, base + n) of the frame part: samples [s, s + count) of each path
// (count > 1: regeneration).  plan == nullptr: host-driven (one synchronisation per iteration;
// `seen` receives the queue sizes); otherwise the plan's iterations, no synchronisation.
static hipError_t path_pass(PathState& T, const PathKernels& K, const DevScene& S, const DevCamera& C,
                            const RenderParams& P, int maxd, int s, int count, int base, int n, float* hdr,
                            unsigned char* l, float4* accum, DevCounters* cnt, hipStream_t st, hipEvent_t* ev,
                            const PathState* plan, std::vector<int>& seen) {
    hipError_t e;
    const PathBufs& B = T.B;
    if ((e = hipMemsetAsync(B.cnt, 0, (kPathMaxIter + 1) * sizeof(int), st)) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[0], st);
    hipLaunchKernelGGL(K.gen, dim3((n + 255) / 256), dim3(256), 0, st, C, P, B, s, base, n, S.max_depth, cnt);
    auto iteration = [&](int it, long long paths) {
        const int g = grid_for(paths);
        hipLaunchKernelGGL(K.trace, dim3(g), dim3(256), 0, st, S, B, it, cnt);
        hipLaunchKernelGGL(K.step, dim3(g), dim3(256), 0, st, S, C, P, B, it, s, P.sample_begin,
                           P.sample_begin + P.sample_count - 1, count, base, maxd, hdr, l, accum, cnt);
    };
    if (plan) {
        const int D = (int)plan->plan.size();
        if (D > path_iter_cap()) return hipErrorInvalidValue;   // (path_run caps its plans)
        for (int it = 0; it < D; ++it) iteration(it, plan->plan[it]);
        hipLaunchKernelGGL(k_path_check, dim3(1), dim3(64), 0, st, B.cnt, D);
    } else {
        long long paths = n;
        seen.assign(1, n);
        for (int it = 0;; ++it) {
            if (it >= path_iter_cap()) return hipErrorNotSupported;   // the fused kernel takes the render
            iteration(it, paths);
            if ((e = hipMemcpyAsync(T.h, B.cnt + it + 1, sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess)
                return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            paths = T.h[0];
            if (paths == 0) break;
            seen.push_back((int)paths);
        }
    }
    if (ev) (void)hipEventRecord(ev[1], st);
    return hipGetLastError();
}

// RTG_PATH_SYNC=1: every pass host-driven (A/B)
static bool path_sync_only() { return std::getenv("RTG_PATH_SYNC") != nullptr; }

// samples per pass: all of the render's with regeneration (Russian roulette, or
// RTG_PATH_REGEN=1), at most 64; one otherwise
static int path_pass_samples(const PathKernels& K, const DevCamera& C, const RenderParams& P) {
    const char* v = std::getenv("RTG_PATH_REGEN");
    const bool regen = v ? std::strcmp(v, "0") != 0 : C.russian_roulette != 0;
    if (!regen) return 1;
    return std::max(1, std::min(P.sample_count, 64));
}

static hipError_t path_run(PathState& T, const PathKernels& K, bool stats, const DevScene& S, const DevCamera& C,
                           const RenderParams& P, int maxd, float* hdr, unsigned char* l, float4* accum,
                           DevCounters* cnt, hipStream_t st, hipEvent_t* ev) {
    hipError_t e;
    if (!T.h && (e = hipHostMalloc(&T.h, 4 * sizeof(int))) != hipSuccess) return e;
    const int npix = P.part_rows * C.width;
    // paths per pass: up to 2^20, and at most half the device memory free now (the frame stacks:
    // 208 B x maxd levels per path -- 6.9 GB at 2^20 paths x 32 levels)
    const size_t per_path = (size_t)maxd * kFrameChunks * 16 + 96;
    size_t mem_free = 0, mem_total = 0;
    if (hipMemGetInfo(&mem_free, &mem_total) != hipSuccess) {
        (void)hipGetLastError();
        mem_free = (size_t)1 << 40;
    }
    mem_free += T.cap * (size_t)T.levels * kFrameChunks * 16;        // the buffers held now are reusable
    const long long budget = std::max<long long>(1 << 16, (long long)(mem_free / 2 / per_path));
    const int chunk = (int)std::min<long long>(std::min(npix, 1 << 20), budget);
    const int per_pass = path_pass_samples(K, C, P);
    if ((e = ensure_paths(T, (size_t)chunk, maxd)) != hipSuccess) return e;
    const std::vector<long long> key = {P.row_begin, P.row_end, P.part_index, P.part_count, C.width, C.height,
                                        (long long)(size_t)S.objects, S.max_depth, (long long)chunk, maxd,
                                        (long long)camera_hash(C), (long long)per_pass};
    for (int attempt = 0; attempt < 2; ++attempt) {
        // attempt 0: planned passes when this frame part has a plan (the first pass otherwise
        // host-driven, planning the rest); attempt 1 (a plan was too short): host-driven.
        // Counted renders (stats) run host-driven: a redone render would count twice.
        const bool adapt = attempt == 0 && !path_sync_only() && !stats;
        bool planned = adapt && T.plan_key == key && !T.plan.empty();
        bool any_planned = false;
        if ((e = hipMemsetAsync(T.B.cnt + kPathMaxIter + 1, 0, sizeof(int), st)) != hipSuccess) return e;
        std::vector<int> seen_max;
        for (int base = 0; base < npix; base += chunk) {
            const int n = std::min(chunk, npix - base);
            const int s_end = P.sample_begin + P.sample_count;
            for (int s = P.sample_begin; s < s_end; s += per_pass) {
                const int count = std::min(per_pass, s_end - s);
                hipEvent_t* pev = (s + count == s_end && base + chunk >= npix) ? ev : nullptr;
                std::vector<int> seen;
                e = path_pass(T, K, S, C, P, maxd, s, count, base, n, hdr, l, accum, cnt, st, pev,
                              planned ? &T : nullptr, seen);
                if (e != hipSuccess) return e;
                if (planned) {
                    any_planned = true;
                    continue;
                }
                if (seen.size() > seen_max.size()) seen_max.resize(seen.size(), 0);
                for (size_t k = 0; k < seen.size(); ++k) seen_max[k] = std::max(seen_max[k], seen[k]);
                if (adapt) {
                    // the queue sizes seen with a margin, and a few more iterations (sampled
                    // trees vary between passes; an empty iteration costs two short launches).
                    // RTG_PATH_PLAN_TIGHT=1 (tests): one iteration short of the passes seen, so
                    // every planned pass leaves paths and the render is redone host-driven
                    const bool tight = std::getenv("RTG_PATH_PLAN_TIGHT") != nullptr;
                    T.plan.clear();
                    for (size_t k = 0; k < seen_max.size(); ++k) {
                        T.plan.push_back((int)std::min<long long>(n, seen_max[k] + seen_max[k] / 4 + 1024));
                    }
                    const int extra = tight ? 0 : std::max(4, (int)seen_max.size() / 4);
                    for (int k = 0; k < extra; ++k) {
                        T.plan.push_back(T.plan.back());
                    }
                    if (tight && T.plan.size() > 1) {
                        T.plan.pop_back();
                    }
                    // at most kPathMaxIter iterations: the per-iteration counters (cnt) end
                    // there.  A pass that needs more leaves paths after the last planned
                    // iteration; k_path_check flags it and the render is redone host-driven,
                    // which hands a pass that long to the fused kernel (hipErrorNotSupported)
                    const size_t cap = (size_t)path_iter_cap();
                    if (T.plan.size() > cap) {
                        T.plan.resize(cap);
                    }
                    T.plan_key = key;
                    planned = true;
                }
            }
        }
        if (!any_planned) return hipSuccess;
        // one synchronisation per render: did a planned pass leave paths unfinished?
        if ((e = hipMemcpyAsync(T.h + 1, T.B.cnt + kPathMaxIter + 1, sizeof(int), hipMemcpyDeviceToHost, st)) !=
            hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        if (T.h[1] == 0) return hipSuccess;
        T.plan.clear();
    }
    return hipSuccess;
}

// the fused kernel's frame-stack bound (rtg_mega.hip launch_d)
static int path_max_depth(const DevScene& S, const DevCamera& C) {
    return (S.max_depth <= 8 && !C.russian_roulette) ? 8 : 32;
}

template <bool STATS>
static TraceFn trace_kernel(int feat) {
    const bool big = (feat & FEAT_BIGLEAF) != 0;
    const int base = feat & ~FEAT_BIGLEAF;
    if (base == 0) return big ? k_path_trace<STATS, FEAT_BIGLEAF> : k_path_trace<STATS, 0>;
    if (base == FEAT_SPHERE) return big ? k_path_trace<STATS, FEAT_SPHERE | FEAT_BIGLEAF> : k_path_trace<STATS, FEAT_SPHERE>;
    return big ? k_path_trace<STATS, FEAT_ALL> : k_path_trace<STATS, FEAT_ALL & ~FEAT_BIGLEAF>;
}

// step kernel variants: shading features BRDF / BRDF + env, spot, mesh lights / all; traversal
// features meshes + spheres (small or large leaves) / all.  Counted renders: the general one.
template <int SK>
static StepFn step_kernel_sk(int feat) {
    if (feat & (FEAT_INSTANCE | FEAT_XFORM)) return k_path_step<false, SK, FEAT_ALL>;
    return (feat & FEAT_BIGLEAF) ? k_path_step<false, SK, FEAT_SPHERE | FEAT_BIGLEAF> : k_path_step<false, SK, FEAT_SPHERE>;
}
static StepFn step_kernel(int sk, int feat) {
    if ((sk & ~SK_BRDF) == 0) return step_kernel_sk<SK_BRDF>(feat);
    if ((sk & ~(SK_BRDF | SK_XLIGHT)) == 0) return step_kernel_sk<SK_BRDF | SK_XLIGHT>(feat);
    return step_kernel_sk<SK_ALL>(feat);
}

hipError_t launch_path(PathState*& T, const DevScene& S, const DevCamera& C, const RenderParams& P, float* hdr,
                       unsigned char* l, float4* accum, DevCounters* cnt, bool stats, int feat, int sk,
                       hipStream_t st, hipEvent_t* ev) {
    if (!T) T = new PathState();
    PathKernels K{};
    if (stats) {
        K.gen = k_path_gen<true>;
        K.trace = trace_kernel<true>(feat);
        K.step = k_path_step<true, SK_ALL, FEAT_ALL>;
    } else {
        K.gen = k_path_gen<false>;
        K.trace = trace_kernel<false>(feat);
        K.step = step_kernel(sk, feat);
    }
    return path_run(*T, K, stats, S, C, P, path_max_depth(S, C), hdr, l, accum, cnt, st, ev);
}

}  // namespace rtg
