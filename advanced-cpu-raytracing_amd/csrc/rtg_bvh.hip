// Device scene ingest: face preparation (parser.cpp:579-747, the
// centroid and bounding box the split reads) and the reference's midpoint BVH
// (Mesh::ConstructBVH / RecursiveBVHBuild / RecomputeBoundingBox, mesh.cpp:23-156) built
// on the GPU, level by level, with the same face permutation as the recursive build.
//
// The reference partitions a node's face range in place with a two-pointer swap loop
// (mesh.cpp:91-100): i scans up past faces whose centroid is below the split, every other
// face is swapped to position j and j moves down.  Its result has a closed form, so every
// face's destination is computed in parallel:
//   S = number of "small" faces (centroid < split) -- the left child's size;
//   a = S + [face at S is big]: the loop examined positions [0, a) from the left and
//       [a, n) from the right (positions n-1, n-2, ... -- the R sequence);
//   left slot q < S: the face at q if small, else the k-th small of the R sequence, where
//       k counts the bigs in [0, q];
//   bigs go right in examination order from position n-1 down: the k-th big of [0, a)
//       has rank idx(k-1) + 1 (idx(j) = R index of the j-th small of R, idx(0) = -1);
//       a big at R index m has rank m + 1, i.e. it moves from q to q - 1.
// (Verified against the sequential loop on random inputs; leaves keep the permutation the
// loop leaves behind even when one half is empty, as the reference does.)
//
// Child boxes are RecomputeBoundingBox's sequential min/max: std::min keeps the first of
// equal values, which matters only for the sign of a zero; the parallel reduction keys
// each value with its position so the first-seen zero wins, exactly.
//
// Output: the walk layout of rtg_device.hpp (pre-order, skip links) and the face arrays in
// the final order -- identical bits to the host build (tests/test_gpu_ingest.py).
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <type_traits>
#include <vector>

#include "rtg_common.hpp"
#include "rtg_kernels.hpp"

namespace rtg {

namespace {

struct BvhTmp {
    int* perm; int* perm2;          // face (mesh-local original index) at each position
    int* seg; int* seg2;            // active node of each position (-1: settled in a leaf)
    int* big;                       // 1: centroid >= split
    int* bigscan;                   // inclusive prefix sum of big over the mesh's positions
    int* selL; int* selR;           // select tables: k-th left big -> q, j-th right small -> m
    float* cen;                     // centroid, 3 per face (original order)
    float* fbox;                    // face bbox mn.xyz mx.xyz, 6 per face (original order)
    // nodes (BFS ids)
    float* nbox;                    // 6 per node
    int* first; int* count; int* left;
    int* axis; float* split; int* S; int* a; int* dosplit; int* childoff;
    unsigned long long* keys;       // 6 per node: child-box reduction keys
    int* size; int* pos;
    int* bigleaf;                   // any leaf wider than kBigLeaf
    void* scan_tmp; size_t scan_bytes;
};

DEV unsigned int ord_key(float v) {            // order-preserving, -0 == +0
    unsigned int u = __float_as_uint(v == 0.0f ? 0.0f : v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// face preparation: centroid (parser.cpp:596-599, (a + b + c) / 3) and bbox (:600-620)
__global__ void k_face_prep(const rtg_face* __restrict__ faces, int n, float* __restrict__ cen,
                            float* __restrict__ fbox) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f >= n) return;
    const rtg_face F = faces[f];
    const f3 a = mk(F.v0.x, F.v0.y, F.v0.z), b = mk(F.v1.x, F.v1.y, F.v1.z), c = mk(F.v2.x, F.v2.y, F.v2.z);
    const f3 ce = divs(add(add(a, b), c), 3.0f);
    cen[3 * f] = ce.x; cen[3 * f + 1] = ce.y; cen[3 * f + 2] = ce.z;
    auto mn = [](float x, float y) { return (y < x) ? y : x; };     // std::min
    auto mx = [](float x, float y) { return (x < y) ? y : x; };     // std::max
    float* o = fbox + 6 * (size_t)f;
    o[0] = mn(mn(a.x, b.x), c.x); o[1] = mn(mn(a.y, b.y), c.y); o[2] = mn(mn(a.z, b.z), c.z);
    o[3] = mx(mx(a.x, b.x), c.x); o[4] = mx(mx(a.y, b.y), c.y); o[5] = mx(mx(a.z, b.z), c.z);
}

__global__ void k_init(BvhTmp T, int n) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    T.perm[p] = p;
    T.seg[p] = 0;
}

// split axis and position of every node of the level (mesh.cpp:58-87)
__global__ void k_split(BvhTmp T, int lo, int hi) {
    const int v = lo + blockIdx.x * 256 + threadIdx.x;
    if (v >= hi) return;
    const float* b = T.nbox + 6 * (size_t)v;
    float lenX = b[3] - b[0], lenY = b[4] - b[1], lenZ = b[5] - b[2];
    float sp;
    int ax;
    if (lenX > lenY) {
        if (lenX > lenZ) { sp = b[0] + lenX * 0.5f; ax = 0; }
        else { sp = b[2] + lenZ * 0.5f; ax = 2; }
    } else {
        if (lenY > lenZ) { sp = b[1] + lenY * 0.5f; ax = 1; }
        else { sp = b[2] + lenZ * 0.5f; ax = 2; }
    }
    T.axis[v] = ax;
    T.split[v] = sp;
}

__global__ void k_flag(BvhTmp T, int n) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const int v = T.seg[p];
    int bg = 0;
    if (v >= 0) bg = !(T.cen[3 * T.perm[p] + T.axis[v]] < T.split[v]);
    T.big[p] = bg;
}

DEV int bigs_before(const BvhTmp& T, int p) { return p > 0 ? T.bigscan[p - 1] : 0; }

// S, a, and whether the node splits (mesh.cpp:101-104: one half empty -> leaf)
__global__ void k_count(BvhTmp T, int lo, int hi) {
    const int v = lo + blockIdx.x * 256 + threadIdx.x;
    if (v >= hi) return;
    const int f = T.first[v], c = T.count[v];
    int s = c, aa = c, ds = 0;
    if (c >= 2) {
        const int bigs = T.bigscan[f + c - 1] - bigs_before(T, f);
        s = c - bigs;
        aa = s + ((s < c) ? T.big[f + s] : 0);
        ds = (s > 0 && s < c) ? 1 : 0;
    }
    T.S[v] = s;
    T.a[v] = aa;
    T.dosplit[v] = ds;
}

__global__ void k_select(BvhTmp T, int n) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const int v = T.seg[p];
    if (v < 0 || T.count[v] < 2) return;
    const int f = T.first[v], c = T.count[v], q = p - f, last = f + c - 1;
    const int bg = T.big[p];
    if (q < T.a[v]) {
        if (bg) T.selL[f + (T.bigscan[p] - bigs_before(T, f)) - 1] = q;
    } else if (!bg) {
        const int smalls = (last - p + 1) - (T.bigscan[last] - bigs_before(T, p));
        T.selR[f + smalls - 1] = last - p;
    }
}

__global__ void k_permute(BvhTmp T, int n, int childBase) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const int v = T.seg[p];
    if (v < 0 || T.count[v] < 2) {
        T.perm2[p] = T.perm[p];
        T.seg2[p] = -1;
        return;
    }
    const int f = T.first[v], c = T.count[v], q = p - f, last = f + c - 1;
    const int bg = T.big[p];
    int np;
    if (q < T.a[v]) {
        if (!bg) {
            np = q;
        } else {
            const int k = T.bigscan[p] - bigs_before(T, f);
            const int rank = k >= 2 ? T.selR[f + k - 2] + 1 : 0;
            np = c - 1 - rank;
        }
    } else if (bg) {
        np = q - 1;
    } else {
        const int smalls = (last - p + 1) - (T.bigscan[last] - bigs_before(T, p));
        np = T.selL[f + smalls - 1];
    }
    T.perm2[f + np] = T.perm[p];
    int ns = -1;
    if (T.dosplit[v]) {
        const int lc = childBase + 2 * T.childoff[v];
        ns = np < T.S[v] ? lc : lc + 1;
    }
    T.seg2[f + np] = ns;
}

// children: ids, ranges, reduction keys reset
__global__ void k_children(BvhTmp T, int lo, int hi, int childBase) {
    const int v = lo + blockIdx.x * 256 + threadIdx.x;
    if (v >= hi) return;
    if (!T.dosplit[v]) { T.left[v] = -1; return; }
    const int lc = childBase + 2 * T.childoff[v];
    T.left[v] = lc;
    T.first[lc] = T.first[v];
    T.count[lc] = T.S[v];
    T.first[lc + 1] = T.first[v] + T.S[v];
    T.count[lc + 1] = T.count[v] - T.S[v];
    for (int k = 0; k < 2; ++k)
        for (int j = 0; j < 6; ++j) T.keys[6 * (size_t)(lc - childBase + k) + j] = j < 3 ? ~0ull : 0ull;
}

// RecomputeBoundingBox (mesh.cpp:136-156) as keyed min / max: (value, position) for min
// (first of equal values), (value, ~position) for max (first of equal values)
__global__ void k_child_box(BvhTmp T, int n, int childBase) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    const int v = p < n ? T.seg[p] : -1;
    const int lane = threadIdx.x & 63;
    unsigned long long k6[6];
    if (v >= 0) {
        const float* b = T.fbox + 6 * (size_t)T.perm[p];
        for (int j = 0; j < 3; ++j) k6[j] = ((unsigned long long)ord_key(b[j]) << 32) | (unsigned)p;
        for (int j = 3; j < 6; ++j) k6[j] = ((unsigned long long)ord_key(b[j]) << 32) | (unsigned)(~p);
    } else {
        for (int j = 0; j < 3; ++j) k6[j] = ~0ull;
        for (int j = 3; j < 6; ++j) k6[j] = 0ull;
    }
    const int v0 = __shfl(v, 0);
    const bool uniform = __ballot(v != v0) == 0;
    if (uniform) {
        if (v0 < 0) return;
        for (int off = 32; off > 0; off >>= 1)
            for (int j = 0; j < 6; ++j) {
                const unsigned long long o = ((unsigned long long)(unsigned)__shfl_xor((int)(k6[j] >> 32), off) << 32) |
                                             (unsigned)__shfl_xor((int)(unsigned)k6[j], off);
                if (j < 3) { if (o < k6[j]) k6[j] = o; }
                else if (o > k6[j]) k6[j] = o;
            }
        if (lane == 0)
            for (int j = 0; j < 6; ++j) {
                unsigned long long* dst = &T.keys[6 * (size_t)(v0 - childBase) + j];
                if (j < 3) atomicMin(dst, k6[j]); else atomicMax(dst, k6[j]);
            }
    } else if (v >= 0) {
        for (int j = 0; j < 6; ++j) {
            unsigned long long* dst = &T.keys[6 * (size_t)(v - childBase) + j];
            if (j < 3) atomicMin(dst, k6[j]); else atomicMax(dst, k6[j]);
        }
    }
}

__global__ void k_child_box_final(BvhTmp T, int lo, int hi) {
    const int v = lo + blockIdx.x * 256 + threadIdx.x;
    if (v >= hi) return;
    for (int j = 0; j < 6; ++j) {
        const unsigned long long k = T.keys[6 * (size_t)(v - lo) + j];
        const unsigned lowp = (unsigned)k;
        const int pos = j < 3 ? (int)lowp : (int)(~lowp);
        T.nbox[6 * (size_t)v + j] = T.fbox[6 * (size_t)T.perm[pos] + j];
    }
}

__global__ void k_size(BvhTmp T, int lo, int hi) {
    const int v = lo + blockIdx.x * 256 + threadIdx.x;
    if (v >= hi) return;
    const int l = T.left[v];
    T.size[v] = l < 0 ? 1 : 1 + T.size[l] + T.size[l + 1];
}

__global__ void k_pos(BvhTmp T, int lo, int hi) {
    const int v = lo + blockIdx.x * 256 + threadIdx.x;
    if (v >= hi) return;
    const int l = T.left[v];
    if (l < 0) return;
    T.pos[l] = T.pos[v] + 1;
    T.pos[l + 1] = T.pos[v] + 1 + T.size[l];
}

// the walk's node records (rtg_device.hpp) at base + pre-order position
__global__ void k_write_nodes(BvhTmp T, int nn, int base, int faceOff, float4* __restrict__ nodes,
                              int2* __restrict__ ext) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= nn) return;
    const float* b = T.nbox + 6 * (size_t)v;
    const int at = base + T.pos[v];
    const int skip = at + T.size[v];
    int leaf = -1;
    int2 e = make_int2(-1, 0);
    if (T.left[v] < 0) {
        const int first = faceOff + T.first[v], cnt = T.count[v];
        leaf = (first < (1 << 23) && cnt < 255) ? (first << 8) | cnt : LEAF_EXT;
        e = make_int2(first, cnt);
        if (cnt > kBigLeaf) atomicOr(T.bigleaf, 1);
    }
    nodes[2 * at] = make_float4(b[0], b[1], b[2], b[3]);
    nodes[2 * at + 1] = make_float4(b[4], b[5], __int_as_float(skip), __int_as_float(leaf));
    ext[at] = e;
}

// faces in the final order: walk records (mesh.cpp:203-215 matrixA columns), normal, uv,
// raw v1/v2 (normal / bump maps)
__global__ void k_write_faces(BvhTmp T, const rtg_face* __restrict__ faces, int n, int faceOff,
                              float4* __restrict__ tris, float4* __restrict__ fn, float2* __restrict__ fuv,
                              float4* __restrict__ v12) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const rtg_face F = faces[T.perm[p]];
    const size_t g = (size_t)faceOff + p;
    tris[3 * g] = make_float4(F.v0.x, F.v0.y, F.v0.z, 0.f);
    tris[3 * g + 1] = make_float4(F.v0.x - F.v1.x, F.v0.y - F.v1.y, F.v0.z - F.v1.z, 0.f);
    tris[3 * g + 2] = make_float4(F.v0.x - F.v2.x, F.v0.y - F.v2.y, F.v0.z - F.v2.z, 0.f);
    fn[g] = make_float4(F.n.x, F.n.y, F.n.z, 0.f);
    if (fuv) {
        fuv[3 * g] = make_float2(F.uv0[0], F.uv0[1]);
        fuv[3 * g + 1] = make_float2(F.uv1[0], F.uv1[1]);
        fuv[3 * g + 2] = make_float2(F.uv2[0], F.uv2[1]);
    }
    if (v12) {
        v12[2 * g] = make_float4(F.v1.x, F.v1.y, F.v1.z, 0.f);
        v12[2 * g + 1] = make_float4(F.v2.x, F.v2.y, F.v2.z, 0.f);
    }
}

inline int nblk(long long n) { return (int)((n + 255) / 256); }

}  // namespace

#define BVH_TRY(x)                                \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) { cleanup(); return e_; } \
    } while (0)

hipError_t build_mesh_bvh(const rtg_face* d_faces, int n, const float root_mn[3], const float root_mx[3],
                          int faceOff, int nodeBase, float4* d_nodes, int2* d_ext, float4* d_tris, float4* d_fn,
                          float2* d_fuv, float4* d_v12, int* d_perm, int* nodeCount, bool* bigleaf,
                          hipStream_t st) {
    BvhTmp T;
    std::memset(&T, 0, sizeof(T));
    std::vector<void*> allocs;
    auto cleanup = [&]() { for (void* p : allocs) (void)hipFree(p); };
    auto alloc = [&](auto*& p, size_t count) -> hipError_t {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, count * sizeof(*p) + 16);
        if (e == hipSuccess) { allocs.push_back(q); p = (std::remove_reference_t<decltype(p)>)q; }
        return e;
    };
    const size_t N = (size_t)n, NN = 2 * N;   // at most 2n - 1 nodes
    BVH_TRY(alloc(T.perm, N)); BVH_TRY(alloc(T.perm2, N)); BVH_TRY(alloc(T.seg, N)); BVH_TRY(alloc(T.seg2, N));
    BVH_TRY(alloc(T.big, N)); BVH_TRY(alloc(T.bigscan, N)); BVH_TRY(alloc(T.selL, N)); BVH_TRY(alloc(T.selR, N));
    BVH_TRY(alloc(T.cen, 3 * N)); BVH_TRY(alloc(T.fbox, 6 * N));
    BVH_TRY(alloc(T.nbox, 6 * NN)); BVH_TRY(alloc(T.first, NN)); BVH_TRY(alloc(T.count, NN)); BVH_TRY(alloc(T.left, NN));
    BVH_TRY(alloc(T.axis, NN)); BVH_TRY(alloc(T.split, NN)); BVH_TRY(alloc(T.S, NN)); BVH_TRY(alloc(T.a, NN));
    BVH_TRY(alloc(T.dosplit, NN)); BVH_TRY(alloc(T.childoff, NN)); BVH_TRY(alloc(T.keys, 6 * N + 12));
    BVH_TRY(alloc(T.size, NN)); BVH_TRY(alloc(T.pos, NN)); BVH_TRY(alloc(T.bigleaf, 1));
    size_t sb1 = 0, sb2 = 0;
    BVH_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, sb1, T.big, T.bigscan, n, st));
    BVH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, sb2, T.dosplit, T.childoff, (int)NN, st));
    T.scan_bytes = sb1 > sb2 ? sb1 : sb2;
    BVH_TRY(hipMalloc(&T.scan_tmp, T.scan_bytes + 16));
    allocs.push_back(T.scan_tmp);

    // root: the mesh bbox (parser.cpp:1393-1468, FLT_MIN max-corner quirk included)
    float rb[6] = {root_mn[0], root_mn[1], root_mn[2], root_mx[0], root_mx[1], root_mx[2]};
    int zero = 0, nn0 = n;
    BVH_TRY(hipMemcpyAsync(T.nbox, rb, sizeof(rb), hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(T.first, &zero, sizeof(int), hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(T.count, &nn0, sizeof(int), hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(T.bigleaf, &zero, sizeof(int), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_face_prep, dim3(nblk(n)), dim3(256), 0, st, d_faces, n, T.cen, T.fbox);
    hipLaunchKernelGGL(k_init, dim3(nblk(n)), dim3(256), 0, st, T, n);
    BVH_TRY(hipGetLastError());

    std::vector<std::pair<int, int>> levels;     // BFS id range per level
    int lo = 0, hi = 1;
    int* h_split = nullptr;
    BVH_TRY(hipHostMalloc(&h_split, 2 * sizeof(int)));
    while (lo < hi) {
        levels.emplace_back(lo, hi);
        const int m = hi - lo;
        hipLaunchKernelGGL(k_split, dim3(nblk(m)), dim3(256), 0, st, T, lo, hi);
        hipLaunchKernelGGL(k_flag, dim3(nblk(n)), dim3(256), 0, st, T, n);
        BVH_TRY(hipcub::DeviceScan::InclusiveSum(T.scan_tmp, T.scan_bytes, T.big, T.bigscan, n, st));
        hipLaunchKernelGGL(k_count, dim3(nblk(m)), dim3(256), 0, st, T, lo, hi);
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(T.scan_tmp, T.scan_bytes, T.dosplit + lo, T.childoff + lo, m, st));
        hipLaunchKernelGGL(k_select, dim3(nblk(n)), dim3(256), 0, st, T, n);
        hipLaunchKernelGGL(k_permute, dim3(nblk(n)), dim3(256), 0, st, T, n, hi);
        hipLaunchKernelGGL(k_children, dim3(nblk(m)), dim3(256), 0, st, T, lo, hi, hi);
        BVH_TRY(hipGetLastError());
        BVH_TRY(hipMemcpyAsync(&h_split[0], T.childoff + hi - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        BVH_TRY(hipMemcpyAsync(&h_split[1], T.dosplit + hi - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        BVH_TRY(hipStreamSynchronize(st));
        const int nsplit = h_split[0] + h_split[1];
        std::swap(T.perm, T.perm2);
        std::swap(T.seg, T.seg2);
        if (nsplit > 0) {
            hipLaunchKernelGGL(k_child_box, dim3(nblk(n)), dim3(256), 0, st, T, n, hi);
            hipLaunchKernelGGL(k_child_box_final, dim3(nblk(2 * nsplit)), dim3(256), 0, st, T, hi, hi + 2 * nsplit);
            BVH_TRY(hipGetLastError());
        }
        lo = hi;
        hi = hi + 2 * nsplit;
    }
    (void)hipHostFree(h_split);
    const int total = hi;
    for (int L = (int)levels.size() - 1; L >= 0; --L)
        hipLaunchKernelGGL(k_size, dim3(nblk(levels[L].second - levels[L].first)), dim3(256), 0, st, T,
                           levels[L].first, levels[L].second);
    BVH_TRY(hipMemcpyAsync(T.pos, &zero, sizeof(int), hipMemcpyHostToDevice, st));
    for (size_t L = 0; L < levels.size(); ++L)
        hipLaunchKernelGGL(k_pos, dim3(nblk(levels[L].second - levels[L].first)), dim3(256), 0, st, T,
                           levels[L].first, levels[L].second);
    hipLaunchKernelGGL(k_write_nodes, dim3(nblk(total)), dim3(256), 0, st, T, total, nodeBase, faceOff, d_nodes, d_ext);
    hipLaunchKernelGGL(k_write_faces, dim3(nblk(n)), dim3(256), 0, st, T, d_faces, n, faceOff, d_tris, d_fn, d_fuv,
                       d_v12);
    BVH_TRY(hipGetLastError());
    if (d_perm) BVH_TRY(hipMemcpyAsync(d_perm, T.perm, N * sizeof(int), hipMemcpyDeviceToDevice, st));
    int bl = 0;
    BVH_TRY(hipMemcpyAsync(&bl, T.bigleaf, sizeof(int), hipMemcpyDeviceToHost, st));
    BVH_TRY(hipStreamSynchronize(st));
    *nodeCount = total;
    *bigleaf = bl != 0;
    cleanup();
    return hipSuccess;
}

}  // namespace rtg
