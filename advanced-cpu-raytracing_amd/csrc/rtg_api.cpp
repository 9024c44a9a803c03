// C-ABI implementation (include/rtgpu.h): scene ingest, device upload, render.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include <tuple>
#include <cstdlib>

#include "host_assets.hpp"
#include "host_scene.hpp"
#include "rtg_ahb.hpp"
#include "rtg_device.hpp"
#include "rtg_kernels.hpp"
#include "rtgpu.h"

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return set_err(RTG_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// Ken Perlin's reference permutation ("Improving Noise", SIGGRAPH 2002), duplicated to
// 512 entries, and the 12 cube-edge gradients -- the tables perlinTexture.cpp:5-37 uses.
const int kPerm256[256] = {
    151, 160, 137, 91,  90,  15,  131, 13,  201, 95,  96,  53,  194, 233, 7,   225, 140, 36,  103, 30,  69,  142,
    8,   99,  37,  240, 21,  10,  23,  190, 6,   148, 247, 120, 234, 75,  0,   26,  197, 62,  94,  252, 219, 203,
    117, 35,  11,  32,  57,  177, 33,  88,  237, 149, 56,  87,  174, 20,  125, 136, 171, 168, 68,  175, 74,  165,
    71,  134, 139, 48,  27,  166, 77,  146, 158, 231, 83,  111, 229, 122, 60,  211, 133, 230, 220, 105, 92,  41,
    55,  46,  245, 40,  244, 102, 143, 54,  65,  25,  63,  161, 1,   216, 80,  73,  209, 76,  132, 187, 208, 89,
    18,  169, 200, 196, 135, 130, 116, 188, 159, 86,  164, 100, 109, 198, 173, 186, 3,   64,  52,  217, 226, 250,
    124, 123, 5,   202, 38,  147, 118, 126, 255, 82,  85,  212, 207, 206, 59,  227, 47,  16,  58,  17,  182, 189,
    28,  42,  223, 183, 170, 213, 119, 248, 152, 2,   44,  154, 163, 70,  221, 153, 101, 155, 167, 43,  172, 9,
    129, 22,  39,  253, 19,  98,  108, 110, 79,  113, 224, 232, 178, 185, 112, 104, 218, 246, 97,  228, 251, 34,
    242, 193, 238, 210, 144, 12,  191, 179, 162, 241, 81,  51,  145, 235, 249, 14,  239, 107, 49,  192, 214, 31,
    181, 199, 106, 157, 184, 84,  204, 176, 115, 121, 50,  45,  127, 4,   150, 254, 138, 236, 205, 93,  222, 114,
    67,  29,  24,  72,  243, 141, 128, 195, 78,  66,  215, 61,  156, 180};
const float kGrad[36] = {1, 1, 0, -1, 1, 0, 1, -1, 0, -1, -1, 0, 1, 0, 1, -1, 0, 1,
                         1, 0, -1, -1, 0, -1, 0, 1, 1, 0, -1, 1, 0, 1, -1, 0, -1, -1};

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t count) {
        if (p) { (void)hipFree(p); p = nullptr; }
        n = count;
        return count ? hipMalloc(&p, count * sizeof(T)) : hipSuccess;
    }
    hipError_t upload(const std::vector<T>& v) {
        if (p) { (void)hipFree(p); p = nullptr; }   // hipFree waits for the device
        n = v.size();
        if (n == 0) return hipSuccess;
        hipError_t e = hipMalloc(&p, n * sizeof(T));
        if (e != hipSuccess) return e;
        return hipMemcpy(p, v.data(), n * sizeof(T), hipMemcpyHostToDevice);
    }
};

void f4(float* dst, const rtg_float3& v, float w = 0.f) { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = w; }

}  // namespace

// Wavefront work buffers of one render context (rtg_scene::work).
struct WaveWork {
    size_t pixels = 0, tiles = 0;
    int slots = 0;
    bool col = false;                 // with the multi-sample colour buffer
    int pay = 0;                      // one-layout payload float4s per queue entry
    void* mem = nullptr;
    void* dq = nullptr;               // deferred-leaf queue + per-pixel hit keys (ensure_defer)
    size_t dq_nq = 0;                 // its shadow-state entries
    size_t dq_pixels = 0;             // the pixel count its hit-key array (and so its layout) was sized for
    rtg::WaveBufs W{};
};
constexpr int kWorkCtx = 1;
struct TileMap {
    int tx, ty;
    DevBuf<int> map;
};

struct rtg_scene {
    int device = 0;
    rtg::DevScene ds;
    std::vector<rtg_camera> cameras;
    int max_depth = 0;
    DevBuf<float4> nodes, tris, face_n;
    int node_count = 0;               // nodes in use (device-built BVH: <= nodes.n / 2)
    DevBuf<int2> node_ext;
    DevBuf<int> env_images;
    DevBuf<unsigned long long> env_mix;
    DevBuf<float2> face_uv;
    DevBuf<float4> face_v12;
    DevBuf<rtg::DevMeshLight> mesh_lights;
    DevBuf<rtg::DevLightFace> light_faces;
    DevBuf<rtg::DevObject> objects;
    DevBuf<float4> group_box;
    DevBuf<rtg::DevMaterial> materials;
    DevBuf<rtg::DevBrdf> brdfs;
    DevBuf<rtg::DevTexture> textures;
    DevBuf<rtg::DevImage> images;
    DevBuf<float> texels;
    DevBuf<rtg::DevPointLight> point_lights;
    DevBuf<rtg::DevAreaLight> area_lights;
    DevBuf<rtg::DevDirLight> dir_lights;
    DevBuf<rtg::DevSpotLight> spot_lights;
    DevBuf<rtg::DevCounters> counters;
    DevBuf<rtg::WNode> anodes;
    DevBuf<float4> ahtris;
    DevBuf<int> face_leaf;
    DevBuf<int> guard;                // RTG_GUARD builds: index-violation bits
    DevBuf<int> perm;
    DevBuf<float> grad;
    bool wave_ok = false;             // scene renders on the wavefront pipeline
    bool tree_ok = false;             // scene may render on the wavefront ray-tree pipeline
    rtg::TreeState* tree = nullptr;   // its buffers
    bool path_ok = false;             // path-tracing cameras may render on the wavefront path tracer
    rtg::PathState* path = nullptr;   // its buffers
    int feat = rtg::FEAT_ALL;         // scene feature bits (traversal specialisation)
    int num_slots = 0;                // lights per pixel (wavefront light slots)
    int shade_sk = rtg::SK_ALL;       // shading features (k_shade variant, rtg_common.hpp SK_*)
    // wavefront buffers, grown on demand
    WaveWork work[kWorkCtx];
    // scratch for the host-buffer entry point
    float* d_hdr = nullptr;
    unsigned char* d_ldr = nullptr;
    size_t d_pixels = 0;
    // block -> tile tables, one per (tiles_x, tiles_y) met (never re-uploaded: kernels of
    // several streams may be reading them)
    std::vector<std::unique_ptr<TileMap>> tile_maps;
    // RTG_RENDER_TIMING events (stage k runs between ev[k] and ev[k+1])
    hipEvent_t ev[rtg::MAX_STAGES + 1] = {};
    int timed_layout = -1;            // stage layout of the last timed render (rtg_kernels.hpp LAYOUT_*)
    int timed_samples = 1;            // samples per pixel its timed stages covered (rtg_scene_timed_samples)
    // the scene's own stream (rtg_render) and the event marking the end of its last render
    // on whatever stream it was issued (rtg_scene_stats waits for it, not for the device)
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    // rtg_scene_create_multi: the other replicas (replica i renders part i of 1 + size())
    std::vector<rtg_scene*> replicas;
    ~rtg_scene() {
        for (rtg_scene* r : replicas) delete r;
        (void)hipSetDevice(device);
        if (guard.p) {
            int bits = 0;
            if (hipMemcpy(&bits, guard.p, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess && bits)
                std::fprintf(stderr, "rtgpu guard: index violations, bits 0x%x\n", bits);
        }
        if (tree) rtg::tree_destroy(tree);
        if (path) rtg::path_destroy(path);
        if (done) (void)hipEventDestroy(done);
        if (stream) (void)hipStreamDestroy(stream);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (d_hdr) (void)hipFree(d_hdr);
        if (d_ldr) (void)hipFree(d_ldr);
        for (auto& w : work) {
            if (w.mem) (void)hipFree(w.mem);
            if (w.dq) (void)hipFree(w.dq);
        }
    }
};

extern "C" {

const char* rtg_last_error(void) { return g_err.c_str(); }
int rtg_abi_version(void) { return RTG_ABI_VERSION; }

// Build provenance (not part of the ABI): the SHA-256 prefix of the sources this library was
// compiled from (csrc/*, include/rtgpu.h, the Makefile's recipe), so that smoke() can show the
// prebuilt library that travels to the GPU box is the build of the tree it runs beside.
#ifndef RTG_SRC_HASH
#define RTG_SRC_HASH "unknown"
#endif
extern "C" __attribute__((visibility("default"))) const char rtg_source_hash[] = RTG_SRC_HASH;

int rtg_host_scene_load_xml(const char* xml_path, rtg_host_scene** out) {
    return rtg_host_scene_load_xml_ex(xml_path, 0, out);
}

int rtg_host_scene_load_xml_ex(const char* xml_path, uint32_t flags, rtg_host_scene** out) {
    if (!xml_path || !out) return set_err(RTG_ERR_INVALID, "null argument");
    *out = nullptr;
    if (flags & ~(uint32_t)RTG_LOAD_DEVICE_BVH) return set_err(RTG_ERR_INVALID, "unknown load flags 0x%x", flags);
    std::unique_ptr<rtg_host_scene> hs(new (std::nothrow) rtg_host_scene);
    if (!hs) return set_err(RTG_ERR_NOMEM, "out of memory");
    std::string err;
    hs->s.deferBvh = (flags & RTG_LOAD_DEVICE_BVH) != 0;
    int rc = hs->s.load(xml_path, err);
    if (rc != RTG_OK) return set_err(rc, "%s: %s", xml_path, err.c_str());
    *out = hs.release();
    return RTG_OK;
}

const rtg_scene_desc* rtg_host_scene_desc(const rtg_host_scene* hs) { return hs ? &hs->s.desc : nullptr; }
void rtg_host_scene_free(rtg_host_scene* hs) { delete hs; }

int rtg_desc_camera_info(const rtg_scene_desc* d, int camera, int32_t* width, int32_t* height, int32_t* spp,
                         int32_t* has_tonemapper) {
    if (!d || camera < 0 || camera >= d->num_cameras) return set_err(RTG_ERR_INVALID, "bad camera index %d", camera);
    const rtg_camera& c = d->cameras[camera];
    if (width) *width = c.width;
    if (height) *height = c.height;
    if (spp) *spp = c.spp;
    if (has_tonemapper) *has_tonemapper = c.has_tonemapper;
    return RTG_OK;
}

int rtg_desc_counts(const rtg_scene_desc* d, int64_t* num_objects, int64_t* num_faces, int64_t* num_nodes,
                    int64_t* num_lights) {
    if (!d) return set_err(RTG_ERR_INVALID, "null desc");
    if (num_objects) *num_objects = d->num_objects;
    if (num_faces) *num_faces = d->num_faces;
    if (num_nodes) *num_nodes = d->num_nodes;
    if (num_lights)
        *num_lights = (int64_t)d->num_point_lights + d->num_area_lights + d->num_dir_lights + d->num_spot_lights +
                      d->num_env_lights + d->num_mesh_lights;
    return RTG_OK;
}

int rtg_scene_export_bvh(const rtg_scene* s, float* nodes, int64_t max_nodes, float* tris, int64_t max_faces,
                         int64_t* num_nodes, int64_t* num_faces) {
    if (!s) return set_err(RTG_ERR_INVALID, "null scene");
    const int64_t nn = s->node_count, nf = (int64_t)(s->tris.n / 3);
    if (num_nodes) *num_nodes = nn;
    if (num_faces) *num_faces = nf;
    HIP_TRY(hipSetDevice(s->device));
    if (nodes && max_nodes >= nn) HIP_TRY(hipMemcpy(nodes, s->nodes.p, nn * 2 * sizeof(float4), hipMemcpyDeviceToHost));
    if (tris && max_faces >= nf) HIP_TRY(hipMemcpy(tris, s->tris.p, nf * 3 * sizeof(float4), hipMemcpyDeviceToHost));
    return RTG_OK;
}

int rtg_device_count(int32_t* count) {
    if (!count) return set_err(RTG_ERR_INVALID, "null argument");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = e == hipSuccess ? n : 0;
    return RTG_OK;
}

// Device ingest: every mesh's BVH and face order built on the GPU (rtg_bvh.hip) straight
// into the scene's walk buffers; facePerm receives the final order (mesh lights sample it).
static int build_bvh_on_device(rtg_scene* sc, const rtg_scene_desc* d, bool anyUV, bool anyMapped,
                               std::vector<int>& meshBegin, std::vector<int>& meshEnd, bool& bigleaf,
                               std::vector<int>& facePerm) {
    const int64_t F = d->num_faces;
    const size_t maxNodes = (size_t)2 * F + 1;          // <= 2n - 1 per mesh, + the pad node
    HIP_TRY(sc->nodes.alloc(2 * maxNodes));
    HIP_TRY(sc->node_ext.alloc(maxNodes));
    HIP_TRY(sc->tris.alloc(3 * F));
    HIP_TRY(sc->face_n.alloc(F));
    if (anyUV) HIP_TRY(sc->face_uv.alloc(3 * F));
    if (anyMapped) HIP_TRY(sc->face_v12.alloc(2 * F));
    HIP_TRY(hipMemset(sc->nodes.p, 0, sc->nodes.n * sizeof(float4)));
    rtg_face* dfaces = nullptr;
    int* dperm = nullptr;
    HIP_TRY(hipMalloc(&dfaces, F * sizeof(rtg_face)));
    struct Free { void* p; ~Free() { if (p) (void)hipFree(p); } } freeFaces{dfaces};
    HIP_TRY(hipMemcpy(dfaces, d->faces, F * sizeof(rtg_face), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&dperm, F * sizeof(int)));
    Free freePerm{dperm};
    hipStream_t st = nullptr;
    int nodeBase = 0;
    for (int m = 0; m < d->num_meshes; ++m) {
        const rtg_mesh& M = d->meshes[m];
        if (M.face_count <= 0 || M.face_offset < 0 || M.face_offset + (int64_t)M.face_count > F)
            return set_err(RTG_ERR_INVALID, "mesh %d: bad face range", m);
        // root box: the mesh's bbox (parser.cpp:1393-1468), carried by its Mesh object
        const rtg_object* owner = nullptr;
        for (int i = 0; i < d->num_objects && !owner; ++i)
            if (d->objects[i].kind == RTG_OBJ_MESH && d->objects[i].mesh == m) owner = &d->objects[i];
        if (!owner) return set_err(RTG_ERR_INVALID, "mesh %d: no Mesh object carries its bbox", m);
        int count = 0;
        bool bl = false;
        HIP_TRY(rtg::build_mesh_bvh(dfaces + M.face_offset, M.face_count, owner->bbox_min, owner->bbox_max,
                                    M.face_offset, nodeBase, sc->nodes.p, sc->node_ext.p, sc->tris.p, sc->face_n.p,
                                    anyUV ? sc->face_uv.p : nullptr, anyMapped ? sc->face_v12.p : nullptr,
                                    dperm + M.face_offset, &count, &bl, st));
        meshBegin[m] = nodeBase;
        meshEnd[m] = nodeBase + count;
        nodeBase += count;
        bigleaf |= bl;
    }
    sc->node_count = nodeBase + 1;                      // + the zeroed pad node
    facePerm.resize(F);
    HIP_TRY(hipMemcpy(facePerm.data(), dperm, F * sizeof(int), hipMemcpyDeviceToHost));
    for (int m = 0; m < d->num_meshes; ++m)
        for (int k = 0; k < d->meshes[m].face_count; ++k) facePerm[d->meshes[m].face_offset + k] += d->meshes[m].face_offset;
    return RTG_OK;
}

// The reference's BVH (mesh.cpp:23-156, as the description carries it) re-laid in pre-order
// with skip links (rtg_device.hpp): a stackless walk "hit -> i+1, miss or leaf done -> skip"
// visits boxes and faces in the order of BVH::IntersectBVH's recursion (bvh.cpp:5-30).
static int reference_preorder(const rtg_scene_desc* d, std::vector<float4>& nodes, std::vector<int2>& next,
                              std::vector<int>& meshBegin, std::vector<int>& meshEnd, bool& bigleaf) {
    nodes.reserve(2 * d->num_nodes); next.reserve(d->num_nodes);
    for (int m = 0; m < d->num_meshes; ++m) {
        const rtg_mesh& M = d->meshes[m];
        const rtg_bvh_node* N = d->nodes + M.node_offset;
        const int base = (int)(nodes.size() / 2);
        meshBegin[m] = base;
        // pre-order, recording each node's subtree end for the skip link
        std::vector<int> order;
        order.reserve(M.node_count);
        std::vector<int> stack{0};
        while (!stack.empty()) {
            int k = stack.back();
            stack.pop_back();
            if (k < 0 || k >= M.node_count) return set_err(RTG_ERR_INVALID, "mesh %d: corrupt BVH", m);
            order.push_back(k);
            if (N[k].left >= 0) { stack.push_back(N[k].left + 1); stack.push_back(N[k].left); }
        }
        std::vector<int> pos(M.node_count, -1);
        for (size_t i = 0; i < order.size(); ++i) pos[order[i]] = (int)i;
        std::vector<int> size(M.node_count, 1);
        for (int i = (int)order.size() - 1; i >= 0; --i) {
            int k = order[i];
            if (N[k].left >= 0) size[k] = 1 + size[N[k].left] + size[N[k].left + 1];
        }
        for (int k : order) {
            const rtg_bvh_node& n = N[k];
            int skip = base + pos[k] + size[k];
            const int first = M.face_offset + n.first;
            int leaf = -1;
            if (n.left < 0) leaf = (first < (1 << 23) && n.count < 255) ? (first << 8) | n.count : rtg::LEAF_EXT;
            if (n.left < 0 && n.count > rtg::kBigLeaf) bigleaf = true;
            float4 a, b;
            a.x = n.bmin[0]; a.y = n.bmin[1]; a.z = n.bmin[2]; a.w = n.bmax[0];
            b.x = n.bmax[1]; b.y = n.bmax[2];
            std::memcpy(&b.z, &skip, 4);
            std::memcpy(&b.w, &leaf, 4);
            nodes.push_back(a); nodes.push_back(b);
            next.push_back(make_int2(n.left < 0 ? first : -1, n.left < 0 ? n.count : 0));
        }
        meshEnd[m] = (int)(nodes.size() / 2);
    }

    return RTG_OK;
}

// Any-hit trees of every mesh (rtg_ahb.cpp).  `reach` bounds |A - o| in the mesh's local space
// for every shadow ray: origins are surface points and ends light points (a directional
// light's ray matters only inside the scene), so the world box of every object and light,
// mapped into each object's local space, bounds both.  False (and no trees) when a leaf
// entry range does not fit its encoding: shadow rays then take the reference walk.
static bool anyhit_trees(const rtg_scene_desc* d, const std::vector<float4>& nd, const std::vector<int2>& nx,
                         const std::vector<int>& meshBegin, const std::vector<int>& meshEnd, const float4* htp, int mode,
                         std::vector<rtg::WNode>& anodes, std::vector<float4>& ahtris, std::vector<int>& aroot,
                         rtg::AhbStats& ast) {
    double wlo[3] = {INFINITY, INFINITY, INFINITY}, whi[3] = {-INFINITY, -INFINITY, -INFINITY};
    auto addp = [&](double x, double y, double z) {
        const double p[3] = {x, y, z};
        for (int k = 0; k < 3; ++k) { wlo[k] = std::min(wlo[k], p[k]); whi[k] = std::max(whi[k], p[k]); }
    };
    auto xf = [](const double* m, const double* p, double* o) {
        for (int r = 0; r < 3; ++r) o[r] = m[4 * r] * p[0] + m[4 * r + 1] * p[1] + m[4 * r + 2] * p[2] + m[4 * r + 3];
    };
    for (int i = 0; i < d->num_objects; ++i) {
        const rtg_object& o = d->objects[i];
        double lo[3], hi[3];
        if (o.kind == RTG_OBJ_SPHERE) {
            for (int k = 0; k < 3; ++k) {
                lo[k] = (&o.center.x)[k] - std::fabs((double)o.radius);
                hi[k] = (&o.center.x)[k] + std::fabs((double)o.radius);
            }
        } else {
            for (int k = 0; k < 3; ++k) { lo[k] = o.bbox_min[k]; hi[k] = o.bbox_max[k]; }
        }
        for (int c = 0; c < 8; ++c) {
            const double p[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
            if (o.kind == RTG_OBJ_INSTANCE) { addp(p[0], p[1], p[2]); continue; }   // world box already
            double w[3];
            xf(o.transform, p, w);
            addp(w[0], w[1], w[2]);
        }
    }
    for (int i = 0; i < d->num_point_lights; ++i)
        addp(d->point_lights[i].position.x, d->point_lights[i].position.y, d->point_lights[i].position.z);
    for (int i = 0; i < d->num_spot_lights; ++i)
        addp(d->spot_lights[i].position.x, d->spot_lights[i].position.y, d->spot_lights[i].position.z);
    for (int i = 0; i < d->num_area_lights; ++i) {
        const rtg_area_light& L = d->area_lights[i];
        for (int c = 0; c < 4; ++c) {
            const double su = (c & 1) ? 0.5 : -0.5, sv = (c & 2) ? 0.5 : -0.5;
            addp(L.position.x + (L.u.x * su + L.v.x * sv) * L.extent, L.position.y + (L.u.y * su + L.v.y * sv) * L.extent,
                 L.position.z + (L.u.z * su + L.v.z * sv) * L.extent);
        }
    }
    // reach = the diagonal of the local-space box holding the mesh and every world point (the
    // distance |A - o| between a face and a shadow ray's origin is below it)
    std::vector<double> reach(d->num_meshes, 0.0);
    for (int i = 0; i < d->num_objects; ++i) {
        const rtg_object& o = d->objects[i];
        if (o.kind == RTG_OBJ_SPHERE) continue;
        double lo[3], hi[3];
        for (int k = 0; k < 3; ++k) { lo[k] = o.bbox_min[k]; hi[k] = o.bbox_max[k]; }
        for (int c = 0; c < 8 && std::isfinite(wlo[0]); ++c) {
            const double p[3] = {(c & 1) ? whi[0] : wlo[0], (c & 2) ? whi[1] : wlo[1], (c & 4) ? whi[2] : wlo[2]};
            double l[3];
            xf(o.inv_transform, p, l);
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], l[k]); hi[k] = std::max(hi[k], l[k]); }
        }
        const double diag = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                      (hi[2] - lo[2]) * (hi[2] - lo[2]));
        reach[o.mesh] = std::max(reach[o.mesh], diag);
    }
    aroot.assign(d->num_meshes, -1);
    bool ahbOk = true;
    for (int m = 0; m < d->num_meshes && ahbOk; ++m) {
        if (meshEnd[m] <= meshBegin[m]) continue;
        aroot[m] = rtg::build_ahb(nd, nx, meshBegin[m], meshEnd[m], htp, reach[m], (rtg::AhbMode)mode, anodes,
                                  ahtris, &ast);
        if (aroot[m] == -2) ahbOk = false;      // leaf encoding exceeded: shadow rays take the reference walk
    }
    if (!ahbOk) { anodes.clear(); ahtris.clear(); aroot.assign(d->num_meshes, -1); }
    return ahbOk;
}

int rtg_scene_create(const rtg_scene_desc* d, int device, rtg_scene** out) {
    if (!d || !out) return set_err(RTG_ERR_INVALID, "null argument");
    *out = nullptr;
    // the packet walks address records by 32-bit byte offsets (rtg_common.hpp rec_at)
    if (d->num_faces > ((int64_t)1 << 25))
        return set_err(RTG_ERR_INVALID, "%lld faces: at most 2^25 per scene", (long long)d->num_faces);
    for (int i = 0; i < d->num_mesh_lights; ++i) {
        const int o = d->mesh_lights ? d->mesh_lights[i].object : -1;
        if (o < 0 || o >= d->num_objects || d->objects[o].kind != RTG_OBJ_MESH ||
            d->meshes[d->objects[o].mesh].face_count <= 0)
            return set_err(RTG_ERR_INVALID, "mesh light %d: bad object", i);
    }
    if (d->max_recursion_depth > rtg::max_supported_depth())
        return set_err(RTG_ERR_UNSUPPORTED, "MaxRecursionDepth %d > %d", d->max_recursion_depth, rtg::max_supported_depth());
    for (int i = 0; i < d->num_objects; ++i) {
        const rtg_object& o = d->objects[i];
        if (o.kind == RTG_OBJ_SPHERE && o.tex_normal >= 0)
            return set_err(RTG_ERR_UNSUPPORTED, "sphere %d: normal map (the reference leaves the normal unset, "
                           "sphere.cpp:95-113)", i);
        if ((o.tex_normal >= d->num_textures) || (o.tex_bump >= d->num_textures))
            return set_err(RTG_ERR_INVALID, "object %d: bad normal / bump texture", i);
        if (o.tex_normal >= 0 && d->textures[o.tex_normal].kind == RTG_TEX_IMAGE &&
            (d->textures[o.tex_normal].image < 0 || d->textures[o.tex_normal].image >= d->num_images))
            return set_err(RTG_ERR_INVALID, "object %d: normal map without an image", i);
        if (o.tex_bump >= 0 && d->textures[o.tex_bump].kind == RTG_TEX_IMAGE &&
            (d->textures[o.tex_bump].image < 0 || d->textures[o.tex_bump].image >= d->num_images))
            return set_err(RTG_ERR_INVALID, "object %d: bump map without an image", i);
        if (o.material < 0 || o.material >= d->num_materials) return set_err(RTG_ERR_INVALID, "object %d: bad material", i);
        if (o.kind != RTG_OBJ_SPHERE && (o.mesh < 0 || o.mesh >= d->num_meshes))
            return set_err(RTG_ERR_INVALID, "object %d: bad mesh", i);
    }
    for (int i = 0; i < d->num_images; ++i)
        if (d->images[i].channels < 1 || !d->images[i].texels) return set_err(RTG_ERR_INVALID, "image %d: no texels", i);

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return set_err(RTG_ERR_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return set_err(RTG_ERR_INVALID, "device %d out of range (%d devices)", device, ndev);
    HIP_TRY(hipSetDevice(device));

    std::unique_ptr<rtg_scene> sc(new (std::nothrow) rtg_scene);
    if (!sc) return set_err(RTG_ERR_NOMEM, "out of memory");
    sc->device = device;
    sc->max_depth = d->max_recursion_depth;
    sc->cameras.assign(d->cameras, d->cameras + d->num_cameras);

    // Device ingest (desc without a BVH, RTG_LOAD_DEVICE_BVH): face preparation and the
    // midpoint BVH are built on the GPU (rtg_bvh.hip); otherwise the host-built reference
    // topology is re-laid here.
    const bool gpuBuild = d->num_faces > 0 && d->num_nodes == 0;
    bool anyMapped = false;
    for (int i = 0; i < d->num_objects; ++i) {
        const rtg_object& o = d->objects[i];
        const bool uvmesh = o.kind != RTG_OBJ_SPHERE && d->meshes[o.mesh].has_uv;
        if ((uvmesh && o.tex_normal >= 0) || ((uvmesh || o.kind == RTG_OBJ_SPHERE) && o.tex_bump >= 0)) anyMapped = true;
    }

    // ---- BVH: reference topology -> pre-order with skip links (rtg_device.hpp)
    std::vector<float4> nodes;
    std::vector<int2> next;
    bool bigleaf = false;
    std::vector<int> meshBegin(d->num_meshes), meshEnd(d->num_meshes);
    if (!gpuBuild) {
        const int rc = reference_preorder(d, nodes, next, meshBegin, meshEnd, bigleaf);
        if (rc) return rc;
    }

    nodes.push_back(make_float4(0.f, 0.f, 0.f, 0.f));     // pad node: walk_bvh prefetches i+1
    nodes.push_back(make_float4(0.f, 0.f, 0.f, 0.f));

    // ---- faces (already BVH-permuted)
    bool anyUV = false;
    for (int m = 0; m < d->num_meshes; ++m) anyUV |= d->meshes[m].has_uv != 0;
    const size_t hostFaces = gpuBuild ? 0 : (size_t)d->num_faces;
    std::vector<float4> tris(3 * hostFaces), fn(hostFaces);
    std::vector<float2> fuv(anyUV ? 3 * hostFaces : 0);
    std::vector<int> facePerm;      // device build: final position -> desc face (per mesh offset)
    if (gpuBuild) {
        int rc = build_bvh_on_device(sc.get(), d, anyUV, anyMapped, meshBegin, meshEnd, bigleaf, facePerm);
        if (rc) return rc;
    }
    for (int64_t f = 0; f < (int64_t)hostFaces; ++f) {
        const rtg_face& F = d->faces[f];
        tris[3 * f] = make_float4(F.v0.x, F.v0.y, F.v0.z, 0.f);
        tris[3 * f + 1] = make_float4(F.v0.x - F.v1.x, F.v0.y - F.v1.y, F.v0.z - F.v1.z, 0.f);
        tris[3 * f + 2] = make_float4(F.v0.x - F.v2.x, F.v0.y - F.v2.y, F.v0.z - F.v2.z, 0.f);
        fn[f] = make_float4(F.n.x, F.n.y, F.n.z, 0.f);
        if (anyUV) {
            fuv[3 * f] = make_float2(F.uv0[0], F.uv0[1]);
            fuv[3 * f + 1] = make_float2(F.uv1[0], F.uv1[1]);
            fuv[3 * f + 2] = make_float2(F.uv2[0], F.uv2[1]);
        }
    }

    // ---- objects
    std::vector<rtg::DevObject> objs(d->num_objects);
    int feat = 0;
    for (int i = 0; i < d->num_objects; ++i) {
        const rtg_object& o = d->objects[i];
        rtg::DevObject& D = objs[i];
        std::memset(&D, 0, sizeof(D));
        D.kind = o.kind;
        D.material = o.material;
        D.flags = o.flags;
        if (o.kind != RTG_OBJ_SPHERE) {
            D.node_begin = meshBegin[o.mesh];
            D.node_end = meshEnd[o.mesh];
            if (d->meshes[o.mesh].has_uv) D.flags |= rtg::OBJF_HAS_UV;
        }
        D.tex_diffuse = o.tex_diffuse;
        D.tex_specular = o.tex_specular;
        D.tex_replace_all = o.tex_replace_all;
        // maps only act where the reference reads them: mesh faces with UVs (mesh.cpp:245-358)
        // and sphere bump maps (sphere.cpp:116-170)
        const bool uvmesh = o.kind != RTG_OBJ_SPHERE && d->meshes[o.mesh].has_uv;
        D.tex_normal = uvmesh ? o.tex_normal : -1;
        D.tex_bump = (uvmesh && o.tex_normal < 0) || o.kind == RTG_OBJ_SPHERE ? o.tex_bump : -1;
        if (D.tex_normal >= 0 || D.tex_bump >= 0) D.flags |= rtg::OBJF_MAPPED;
        for (int k = 0; k < 3; ++k) { D.bmin[k] = o.bbox_min[k]; D.bmax[k] = o.bbox_max[k]; }
        f4(D.mbv, o.motion_blur);
        f4(D.center, o.center, o.radius);
        bool ident = true;
        for (int k = 0; k < 12; ++k) {
            D.inv[k] = o.inv_transform[k];
            D.invT[k] = o.inv_transpose[k];
            D.baseInvT[k] = o.base_inv_transpose[k];
            ident &= o.inv_transform[k] == ((k % 5 == 0) ? 1.0 : 0.0);
        }
        if (ident) D.flags |= rtg::OBJF_IDENTITY;
        D.id = o.kind == RTG_OBJ_SPHERE ? INT32_MIN : o.id;   // spheres never carry a light's id
        if (o.kind == RTG_OBJ_SPHERE) feat |= rtg::FEAT_SPHERE;
        else if (o.kind == RTG_OBJ_INSTANCE) feat |= rtg::FEAT_INSTANCE;
        else if (!ident || (o.flags & RTG_OBJF_MOTION_BLUR)) feat |= rtg::FEAT_XFORM;
    }
    // shadow-ray acceleration (rtg_common.hpp): the any-hit wide BVH (trace_any_wide) and
    // face -> reference leaf (its exact leaf-box decisions, the deferred leaves' checks).
    // RTG_NO_FAST_SHADOW=1: shadow rays walk the reference BVH top-down.
    std::vector<rtg::WNode> anodes;
    std::vector<float4> ahtris;
    int ahbMode = rtg::AHB_EXACT;
    std::vector<int> faceLeaf;
    for (int i = 0; i < d->num_objects; ++i) objs[i].aroot = -1;
    if (!std::getenv("RTG_NO_FAST_SHADOW") && d->num_meshes > 0) {
        std::vector<float4> dn;
        std::vector<int2> dx;
        if (gpuBuild) {
            dn.resize(2 * (size_t)sc->node_count);
            HIP_TRY(hipMemcpy(dn.data(), sc->nodes.p, dn.size() * sizeof(float4), hipMemcpyDeviceToHost));
            dx.resize((size_t)sc->node_count);
            HIP_TRY(hipMemcpy(dx.data(), sc->node_ext.p, dx.size() * sizeof(int2), hipMemcpyDeviceToHost));
        }
        const std::vector<float4>& nd = gpuBuild ? dn : nodes;
        const std::vector<int2>& nx = gpuBuild ? dx : next;
        auto leafv = [&](int i) { int l; std::memcpy(&l, &nd[2 * i + 1].w, 4); return l; };
        faceLeaf.assign((size_t)d->num_faces, -1);
        for (int m = 0; m < d->num_meshes; ++m)
            for (int p = meshBegin[m]; p < meshEnd[m]; ++p) {
                const int l = leafv(p);
                if (l < 0) continue;
                int first = l >> 8, cnt = l & 255;
                if (l == rtg::LEAF_EXT) { first = nx[p].x; cnt = nx[p].y; }
                for (int f = first; f < first + cnt; ++f) faceLeaf[f] = p;
            }

        // any-hit tree per mesh (anyhit_trees, rtg_ahb.cpp)
        std::vector<float4> ht;
        const float4* htp = tris.data();
        if (gpuBuild) {
            ht.resize(3 * (size_t)d->num_faces);
            HIP_TRY(hipMemcpy(ht.data(), sc->tris.p, ht.size() * sizeof(float4), hipMemcpyDeviceToHost));
            htp = ht.data();
        }
        const char* am = std::getenv("RTG_AHB");
        ahbMode = !am ? rtg::AHB_EXACT : (std::strcmp(am, "ref") == 0 ? rtg::AHB_REF
                                          : std::strcmp(am, "split") == 0 ? rtg::AHB_SPLIT : rtg::AHB_EXACT);
        rtg::AhbStats ast;
        std::vector<int> aroot;
        anyhit_trees(d, nd, nx, meshBegin, meshEnd, htp, ahbMode, anodes, ahtris, aroot, ast);
        for (int i = 0; i < d->num_objects; ++i)
            objs[i].aroot = d->objects[i].kind != RTG_OBJ_SPHERE ? aroot[d->objects[i].mesh] : -1;
        if (std::getenv("RTG_AHB_VERBOSE"))
            std::fprintf(stderr, "rtgpu any-hit tree (mode %d): %lld nodes, %lld entries, depth %d, %lld leaf prims, "
                                 "%lld face prims (%lld on their leaf box)\n",
                         ahbMode, ast.nodes, ast.entries, ast.max_depth, ast.leaf_prims, ast.face_prims, ast.exact_faces);
    }
    // instance groups: runs of consecutive instances without motion blur, chunked by ~sqrt of
    // the run length, with the exact (min/max) union of the members' world boxes
    std::vector<float4> gbox(2 * (size_t)d->num_objects, make_float4(0.f, 0.f, 0.f, 0.f));
    for (int k = 0; k < d->num_objects;) {
        auto eligible = [&](int i) {
            return objs[i].kind == rtg::OBJ_INSTANCE && !(objs[i].flags & rtg::OBJF_MOTION_BLUR);
        };
        if (!eligible(k)) { ++k; continue; }
        int e = k;
        while (e < d->num_objects && eligible(e)) ++e;
        const int run = e - k;
        const int gsz = std::max(4, (int)std::lround(std::sqrt((double)run)));
        for (int g = k; g < e; g += gsz) {
            const int ge = std::min(e, g + gsz);
            if (ge - g < 2) continue;
            float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = g; i < ge; ++i)
                for (int c = 0; c < 3; ++c) {
                    mn[c] = std::min(mn[c], objs[i].bmin[c]);
                    mx[c] = std::max(mx[c], objs[i].bmax[c]);
                }
            objs[g].group_end = ge;
            gbox[2 * g] = make_float4(mn[0], mn[1], mn[2], 0.f);
            gbox[2 * g + 1] = make_float4(mx[0], mx[1], mx[2], 0.f);
        }
        k = e;
    }
    // wavefront eligibility: no ray-tree children and no motion blur
    bool branching = false, blur = false;
    for (int i = 0; i < d->num_materials; ++i) {
        int t = d->materials[i].type;
        branching |= (t == RTG_MAT_MIRROR || t == RTG_MAT_DIELECTRIC || t == RTG_MAT_CONDUCTOR);
    }
    for (int i = 0; i < d->num_objects; ++i) blur |= (d->objects[i].flags & RTG_OBJF_MOTION_BLUR) != 0;
    sc->feat = feat | (bigleaf ? rtg::FEAT_BIGLEAF : 0);
    // RTG_NO_COOP=1: large leaves tested by their own lane (the sequential walk handles any
    // leaf size; the cooperative one is only faster)
    if (std::getenv("RTG_NO_COOP")) sc->feat &= ~rtg::FEAT_BIGLEAF;
    sc->tree_ok = !blur && d->max_recursion_depth > 0 && branching;
    sc->wave_ok = !blur && (d->max_recursion_depth <= 0 || !branching);
    sc->path_ok = !blur;
    sc->num_slots = d->num_point_lights + d->num_area_lights + d->num_env_lights + d->num_dir_lights +
                    d->num_spot_lights + d->num_mesh_lights;
    // shading features: textures / maps (incl. a background texture), BRDFs, env / spot / mesh
    // lights
    {
        int sk = 0;
        for (int i = 0; i < d->num_objects; ++i)
            if (objs[i].tex_diffuse >= 0 || objs[i].tex_specular >= 0 || objs[i].tex_replace_all >= 0 ||
                (objs[i].flags & rtg::OBJF_MAPPED))
                sk |= rtg::SK_TEX;
        if (d->bg_texture >= 0) sk |= rtg::SK_TEX;
        for (int i = 0; i < d->num_materials; ++i)
            if (d->materials[i].brdf >= 0) sk |= rtg::SK_BRDF;
        if (d->num_env_lights + d->num_spot_lights + d->num_mesh_lights > 0) sk |= rtg::SK_XLIGHT;
        sc->shade_sk = sk;
    }
    // mesh lights (meshLight.h): their faces in MeshLight::faces order (the BVH-permuted one)
    std::vector<rtg::DevMeshLight> mls(d->num_mesh_lights);
    std::vector<rtg::DevLightFace> lfs;
    for (int i = 0; i < d->num_mesh_lights; ++i) {
        const rtg_object& o = d->objects[d->mesh_lights[i].object];
        const rtg_mesh& M = d->meshes[o.mesh];
        rtg::DevMeshLight& L = mls[i];
        std::memset(&L, 0, sizeof(L));
        L.id = o.id;
        L.face_begin = (int)lfs.size();
        L.face_count = M.face_count;
        f4(L.radiance, d->mesh_lights[i].radiance);
        L.surface_area = M.surface_area;
        for (int k = 0; k < 12; ++k) L.xf[k] = o.transform[k];
        for (int f = 0; f < M.face_count; ++f) {
            const rtg_face& F = d->faces[gpuBuild ? facePerm[M.face_offset + f] : M.face_offset + f];
            rtg::DevLightFace lf;
            std::memset(&lf, 0, sizeof(lf));
            f4(lf.v0, F.v0); f4(lf.v1, F.v1); f4(lf.v2, F.v2);
            lf.area = F.area;
            lfs.push_back(lf);
        }
    }
    std::vector<rtg::DevMaterial> mats(d->num_materials);
    for (int i = 0; i < d->num_materials; ++i) {
        const rtg_material& m = d->materials[i];
        rtg::DevMaterial& D = mats[i];
        std::memset(&D, 0, sizeof(D));
        D.type = m.type;
        D.brdf = m.brdf;
        f4(D.ambient, m.ambient); f4(D.diffuse, m.diffuse); f4(D.specular, m.specular); f4(D.mirror, m.mirror);
        f4(D.absorption, m.absorption); f4(D.radiance, m.radiance);
        D.phong_exponent = m.phong_exponent;
        D.refractive_index = m.refractive_index;
        D.absorption_index = m.absorption_index;
        D.roughness = m.roughness;
    }
    std::vector<rtg::DevBrdf> brdfs(d->num_brdfs);
    for (int i = 0; i < d->num_brdfs; ++i) {
        std::memset(&brdfs[i], 0, sizeof(brdfs[i]));
        brdfs[i].type = d->brdfs[i].type;
        brdfs[i].energy_conserving = d->brdfs[i].energy_conserving;
        brdfs[i].kd_fresnel = d->brdfs[i].kd_fresnel;
        brdfs[i].exponent = d->brdfs[i].exponent;
    }
    std::vector<rtg::DevTexture> texs(d->num_textures);
    for (int i = 0; i < d->num_textures; ++i) {
        const rtg_texture& t = d->textures[i];
        std::memset(&texs[i], 0, sizeof(texs[i]));
        texs[i].kind = t.kind;
        texs[i].blend = t.blend;
        texs[i].image = t.image;
        texs[i].nearest = t.nearest;
        texs[i].noise_scale = t.noise_scale;
        texs[i].bump_factor = t.bump_factor;
        texs[i].normalizer = t.normalizer;
        texs[i].noise_abs = t.noise_abs;
    }
    // texel pool; each image padded with one extra row + 4 floats so the reference's
    // edge reads (bilinear p+1, 1-channel RGB reads) stay inside the allocation
    std::vector<rtg::DevImage> imgs(d->num_images);
    std::vector<float> pool;
    for (int i = 0; i < d->num_images; ++i) {
        const rtg_image& im = d->images[i];
        imgs[i].width = im.width; imgs[i].height = im.height; imgs[i].channels = im.channels;
        imgs[i].offset = (long long)pool.size();
        size_t n = (size_t)im.width * im.height * im.channels;
        pool.insert(pool.end(), im.texels, im.texels + n);
        pool.insert(pool.end(), (size_t)im.width * im.channels + 4, 0.f);
    }
    std::vector<rtg::DevPointLight> pls(d->num_point_lights);
    for (int i = 0; i < d->num_point_lights; ++i) {
        f4(pls[i].pos, d->point_lights[i].position);
        f4(pls[i].intensity, d->point_lights[i].intensity);
    }
    std::vector<rtg::DevAreaLight> als(d->num_area_lights);
    for (int i = 0; i < d->num_area_lights; ++i) {
        const rtg_area_light& a = d->area_lights[i];
        std::memset(&als[i], 0, sizeof(als[i]));
        f4(als[i].pos, a.position); f4(als[i].normal, a.normal); f4(als[i].radiance, a.radiance);
        f4(als[i].u, a.u); f4(als[i].v, a.v);
        als[i].extent = a.extent; als[i].area = a.area;
    }
    std::vector<rtg::DevDirLight> dls(d->num_dir_lights);
    for (int i = 0; i < d->num_dir_lights; ++i) {
        f4(dls[i].dir, d->dir_lights[i].dir);
        f4(dls[i].radiance, d->dir_lights[i].radiance);
    }
    std::vector<rtg::DevSpotLight> sls(d->num_spot_lights);
    for (int i = 0; i < d->num_spot_lights; ++i) {
        const rtg_spot_light& s = d->spot_lights[i];
        std::memset(&sls[i], 0, sizeof(sls[i]));
        f4(sls[i].pos, s.position); f4(sls[i].dir, s.dir); f4(sls[i].intensity, s.intensity);
        sls[i].coverage_deg = s.coverage_deg; sls[i].falloff_deg = s.falloff_deg;
        sls[i].cos_half_coverage = s.cos_half_coverage; sls[i].cos_half_falloff = s.cos_half_falloff;
    }
    std::vector<int> envs(d->num_env_lights);
    for (int i = 0; i < d->num_env_lights; ++i) {
        envs[i] = d->env_lights[i].image;
        if (envs[i] < 0 || envs[i] >= d->num_images) return set_err(RTG_ERR_INVALID, "env light %d: bad image", i);
    }

    if (!gpuBuild) {
        sc->node_count = (int)(nodes.size() / 2);
        HIP_TRY(sc->nodes.upload(nodes)); HIP_TRY(sc->node_ext.upload(next)); HIP_TRY(sc->tris.upload(tris));
        HIP_TRY(sc->face_n.upload(fn)); HIP_TRY(sc->face_uv.upload(fuv));
    }
    if (anyMapped && !gpuBuild) {
        std::vector<float4> v12(2 * d->num_faces);
        for (int64_t f = 0; f < d->num_faces; ++f) {
            const rtg_face& F = d->faces[f];
            v12[2 * f] = make_float4(F.v1.x, F.v1.y, F.v1.z, 0.f);
            v12[2 * f + 1] = make_float4(F.v2.x, F.v2.y, F.v2.z, 0.f);
        }
        HIP_TRY(sc->face_v12.upload(v12));
    }
    HIP_TRY(sc->objects.upload(objs)); HIP_TRY(sc->group_box.upload(gbox)); HIP_TRY(sc->materials.upload(mats)); HIP_TRY(sc->brdfs.upload(brdfs));
    HIP_TRY(sc->textures.upload(texs)); HIP_TRY(sc->images.upload(imgs)); HIP_TRY(sc->texels.upload(pool));
    HIP_TRY(sc->point_lights.upload(pls)); HIP_TRY(sc->area_lights.upload(als)); HIP_TRY(sc->dir_lights.upload(dls));
    HIP_TRY(sc->spot_lights.upload(sls)); HIP_TRY(sc->env_images.upload(envs));
    {
        // env_direction's key-independent inner hashes: mix64(RP_ENV << 32 | e * 16384 + j)
        auto mix = [](uint64_t z) {
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
            return z ^ (z >> 31);
        };
        std::vector<unsigned long long> em((size_t)d->num_env_lights * rtg::kEnvDraws);
        for (int e = 0; e < d->num_env_lights; ++e)
            for (int j = 0; j < rtg::kEnvDraws; ++j)
                em[(size_t)e * rtg::kEnvDraws + j] =
                    mix(((uint64_t)rtg::kRpEnv << 32) | (uint32_t)((uint32_t)e * 16384u + (uint32_t)j));
        HIP_TRY(sc->env_mix.upload(em));
    }
    HIP_TRY(sc->mesh_lights.upload(mls)); HIP_TRY(sc->light_faces.upload(lfs));
    HIP_TRY(sc->anodes.upload(anodes));
    HIP_TRY(sc->ahtris.upload(ahtris));
    HIP_TRY(sc->face_leaf.upload(faceLeaf));
    std::vector<rtg::DevCounters> zero(1);
    std::memset(zero.data(), 0, sizeof(rtg::DevCounters));
    HIP_TRY(sc->counters.upload(zero));
    {
        std::vector<int> perm(512);
        for (int i = 0; i < 512; ++i) perm[i] = kPerm256[i & 255];
        HIP_TRY(sc->perm.upload(perm));
        HIP_TRY(sc->grad.upload(std::vector<float>(kGrad, kGrad + 36)));
    }

    rtg::DevScene& S = sc->ds;
    std::memset(&S, 0, sizeof(S));
    S.nodes = sc->nodes.p; S.node_ext = sc->node_ext.p; S.tris = sc->tris.p; S.face_n = sc->face_n.p;
    S.face_uv = sc->face_uv.p;
    S.face_v12 = sc->face_v12.p;
    S.mesh_lights = sc->mesh_lights.p;
    S.light_faces = sc->light_faces.p;
    S.num_mesh = d->num_mesh_lights;
    S.objects = sc->objects.p; S.group_box = sc->group_box.p; S.materials = sc->materials.p; S.brdfs = sc->brdfs.p;
    S.textures = sc->textures.p; S.images = sc->images.p; S.texels = sc->texels.p;
    S.point_lights = sc->point_lights.p; S.area_lights = sc->area_lights.p; S.dir_lights = sc->dir_lights.p;
    S.spot_lights = sc->spot_lights.p; S.env_images = sc->env_images.p; S.env_mix = sc->env_mix.p;
    S.perm = sc->perm.p; S.grad = sc->grad.p;
    S.num_objects = d->num_objects; S.num_point = d->num_point_lights; S.num_area = d->num_area_lights;
    S.num_dir = d->num_dir_lights; S.num_spot = d->num_spot_lights; S.num_env = d->num_env_lights;
    S.max_depth = d->max_recursion_depth;
    S.bg_texture = d->bg_texture;
    S.eps = d->shadow_epsilon;
    S.ambient[0] = d->ambient_light.x; S.ambient[1] = d->ambient_light.y; S.ambient[2] = d->ambient_light.z;
    for (int k = 0; k < 3; ++k) S.background[k] = d->background[k];
    S.coop = (sc->feat & rtg::FEAT_BIGLEAF) ? 1 : 0;
    S.anodes = anodes.empty() ? nullptr : sc->anodes.p;
    S.ahtris = ahtris.empty() ? nullptr : sc->ahtris.p;
    S.ahb_split = ahbMode == rtg::AHB_SPLIT && !anodes.empty();
    S.num_faces = (int)d->num_faces;
    S.num_textures = d->num_textures;
    S.num_images = d->num_images;
    S.num_materials = d->num_materials;
    HIP_TRY(sc->guard.alloc(1));
    HIP_TRY(hipMemset(sc->guard.p, 0, sizeof(int)));
    S.guard = sc->guard.p;
    S.face_leaf = faceLeaf.empty() ? nullptr : sc->face_leaf.p;
    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&sc->done, hipEventDisableTiming));
    HIP_TRY(hipDeviceSynchronize());
    *out = sc.release();
    return RTG_OK;
}

int rtg_scene_create_multi(const rtg_scene_desc* d, const int32_t* devices, int32_t n, rtg_scene** out) {
    if (!d || !out || !devices || n < 1) return set_err(RTG_ERR_INVALID, "bad device list");
    *out = nullptr;
    rtg_scene* first = nullptr;
    int rc = rtg_scene_create(d, devices[0], &first);
    if (rc) return rc;
    std::unique_ptr<rtg_scene> sc(first);
    for (int i = 1; i < n; ++i) {
        rtg_scene* r = nullptr;
        rc = rtg_scene_create(d, devices[i], &r);
        if (rc) return rc;
        sc->replicas.push_back(r);
    }
    *out = sc.release();
    return RTG_OK;
}

int rtg_scene_num_devices(const rtg_scene* s, int32_t* n) {
    if (!s || !n) return set_err(RTG_ERR_INVALID, "null argument");
    *n = 1 + (int32_t)s->replicas.size();
    return RTG_OK;
}

void rtg_scene_destroy(rtg_scene* s) {
    delete s;
}

// Band k of part `part` of `parts` (rtgpu.h RTG_PART_BAND_ROWS; part_row in rtg_common.hpp):
// round-robin, rotated by one slot per round of `parts` bands.  Increasing in k.
static int part_band(int part, int parts, int k) {
    int slot = (part - k) % parts;
    if (slot < 0) slot += parts;
    return k * parts + slot;
}

int rtg_part_runs(int32_t row_begin, int32_t row_end, int32_t part, int32_t parts, int32_t* runs, int32_t cap,
                  int32_t* count) {
    if (!count) return set_err(RTG_ERR_INVALID, "null argument");
    if (parts <= 0) parts = 1;
    if (part < 0 || part >= parts || row_begin < 0 || row_end < row_begin)
        return set_err(RTG_ERR_INVALID, "bad partition (part %d of %d, rows [%d, %d))", part, parts, row_begin, row_end);
    int n = 0, r0 = -1, r1 = -1;
    for (int k = 0, b = part_band(part, parts, 0); row_begin + b * RTG_PART_BAND_ROWS < row_end;
         b = part_band(part, parts, ++k)) {
        const int a = row_begin + b * RTG_PART_BAND_ROWS, e = std::min(a + RTG_PART_BAND_ROWS, (int)row_end);
        if (a == r1) { r1 = e; continue; }
        if (r0 >= 0) { if (runs && n < cap) { runs[2 * n] = r0; runs[2 * n + 1] = r1; } ++n; }
        r0 = a; r1 = e;
    }
    if (r0 >= 0) { if (runs && n < cap) { runs[2 * n] = r0; runs[2 * n + 1] = r1; } ++n; }
    *count = n;
    return RTG_OK;
}

// Block -> tile assignment.  The hardware deals workgroups to the 8 XCDs round-robin
// (block b runs on XCD b % 8), and each XCD has its own L2: each XCD gets whole 64x64-pixel
// super-tiles (4x4 tiles), dealt round-robin over the image, so an XCD's blocks share BVH nodes
// in its L2 while every XCD sees a spread of the image (traversal cost varies strongly with
// image position: one contiguous band per XCD left XCDs idle, 3.1 -> 5.3 Grays/s on the headline
// when this was fixed; super-tiles of 32 / 128 / 256 px and row-major tiles measured no better,
// DESIGN.md §4).
static std::vector<int> build_tile_map(int tx, int ty) {
    const int n = tx * ty;
    std::vector<int> order(n);
    for (int t = 0; t < n; ++t) order[t] = t;
    const int S = 4, stx = (tx + S - 1) / S;
    auto key = [&](int t) {
        const int x = t % tx, y = t / tx;
        const int st = (y / S) * stx + x / S;
        return std::make_tuple(st % 8, st / 8, (y % S) * S + x % S);
    };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key(a) < key(b); });
    // block 8k + x (XCD x) takes the k-th tile of XCD x's contiguous share of `order`
    std::vector<int> map(n);
    int prefix = 0;
    for (int x = 0; x < 8; ++x) {
        const int cnt = (n - x + 7) / 8;
        for (int k = 0; k < cnt; ++k) map[8 * k + x] = order[prefix + k];
        prefix += cnt;
    }
    return map;
}

static int ensure_tile_map(rtg_scene* s, int tx, int ty, const int** out) {
    for (auto& m : s->tile_maps)
        if (m->tx == tx && m->ty == ty) {
            *out = m->map.p;
            return RTG_OK;
        }
    HIP_TRY(hipSetDevice(s->device));
    std::unique_ptr<TileMap> m(new TileMap{tx, ty, {}});
    HIP_TRY(m->map.upload(build_tile_map(tx, ty)));
    *out = m->map.p;
    s->tile_maps.push_back(std::move(m));
    return RTG_OK;
}

static int prepare(rtg_scene* s, const rtg_render_opts* o, rtg::DevCamera& C, rtg::RenderParams& P) {
    if (!s || !o) return set_err(RTG_ERR_INVALID, "null argument");
    if (o->camera < 0 || o->camera >= (int)s->cameras.size()) return set_err(RTG_ERR_INVALID, "bad camera %d", o->camera);
    const rtg_camera& c = s->cameras[o->camera];
    if (c.width <= 0 || c.height <= 0) return set_err(RTG_ERR_INVALID, "camera %d has an empty image", o->camera);
    std::memset(&C, 0, sizeof(C));
    auto cp = [](float* d, const rtg_float3& v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; };
    cp(C.pos, c.position); cp(C.gaze, c.gaze); cp(C.up, c.up); cp(C.right, c.right); cp(C.q, c.q);
    C.left = c.left; C.right_ext = c.right_ext; C.bottom = c.bottom; C.top = c.top;
    C.focus_distance = c.focus_distance; C.aperture = c.aperture;
    C.width = c.width; C.height = c.height; C.spp = c.spp < 1 ? 1 : c.spp;
    C.path_tracing = c.path_tracing; C.next_event = c.next_event;
    C.importance_sampling = c.importance_sampling; C.russian_roulette = c.russian_roulette;
    std::memset(&P, 0, sizeof(P));
    P.row_begin = o->row_begin < 0 ? 0 : o->row_begin;
    P.row_end = (o->row_end <= 0 || o->row_end > c.height) ? c.height : o->row_end;
    if (P.row_begin >= P.row_end) return set_err(RTG_ERR_INVALID, "empty row range");
    P.sample_begin = o->sample_begin < 0 ? 0 : o->sample_begin;
    P.sample_count = o->sample_count < 0 ? C.spp : o->sample_count;
    P.accum_only = (o->flags & RTG_RENDER_ACCUM_ONLY) ? 1 : 0;
    if (!P.accum_only && (P.sample_begin != 0 || P.sample_count != C.spp))
        return set_err(RTG_ERR_INVALID, "a partial sample range requires RTG_RENDER_ACCUM_ONLY");
    P.part_count = o->part_count <= 0 ? 1 : o->part_count;
    P.part_index = o->part_index;
    if (P.part_index < 0 || P.part_index >= P.part_count)
        return set_err(RTG_ERR_INVALID, "part %d of %d", P.part_index, P.part_count);
    // this part's bands of RTG_PART_BAND_ROWS rows (part_row in rtg_common.hpp) and its row
    // count; tiles of 16 compact rows (two bands; a wave's 8 rows are one band)
    static_assert(RTG_PART_BAND_ROWS == 8, "part_row's band shift");
    const int bands = (P.row_end - P.row_begin + RTG_PART_BAND_ROWS - 1) / RTG_PART_BAND_ROWS;
    int own = 0;
    while (part_band(P.part_index, P.part_count, own) < bands) ++own;
    P.part_rows = 0;
    if (own > 0) {
        const int lastBand = part_band(P.part_index, P.part_count, own - 1);
        P.part_rows = (own - 1) * RTG_PART_BAND_ROWS +
                      std::min(RTG_PART_BAND_ROWS, P.row_end - P.row_begin - lastBand * RTG_PART_BAND_ROWS);
    }
    P.tiles_x = (c.width + 15) / 16;
    P.tiles_y = (P.part_rows + 15) / 16;
    P.num_tiles = P.tiles_x * P.tiles_y;
    if (P.num_tiles == 0) return RTG_OK;   // nothing of this part in the row range
    // one sample per pass until launch() chooses more (pass_slabs)
    P.slabs = 1;
    P.slab_tiles = P.num_tiles;
    P.slab_px = 16 * P.tiles_y * c.width;
    P.seed = o->seed;
    const int* map = nullptr;
    int rc = ensure_tile_map(s, P.tiles_x, P.tiles_y, &map);
    if (rc) return rc;
    P.tile_map = map;
    return RTG_OK;
}

// The wavefront pipeline's one-shadow-light layout (rtg_wave.hpp SH_ONE): payload float4s per
// queued shadow ray -- 2 with at most one light, 3 with one point / area light followed by one
// environment light (its term travels with the shadow ray: C4), 0 otherwise (general layout)
static int one_payload(const rtg_scene* s) {
    const rtg::DevScene& S = s->ds;
    if (s->num_slots <= 1) return 2;
    if (s->num_slots == 2 && S.num_env == 1 && S.num_point + S.num_area == 1 && S.num_dir + S.num_spot + S.num_mesh == 0)
        return 3;
    return 0;
}

// Sizes the wavefront buffers for `pixels` pixel entries x `slots` light slots and `tiles`
// shade blocks (queue segments of 256 * slots entries), one allocation; `pay`: one-layout
// payload float4s per queue entry (one_payload); `col`: with the colour buffer of multi-sample
// passes (one float4 per entry).
static int ensure_wave(WaveWork& ww, size_t pixels, int slots, size_t tiles, int pay, bool col = false) {
    if (ww.mem && ww.pixels >= pixels && ww.slots >= slots && ww.tiles >= tiles && ww.pay >= pay && (ww.col || !col))
        return RTG_OK;
    if (ww.dq) { (void)hipFree(ww.dq); ww.dq = nullptr; }
    if (ww.mem) { (void)hipFree(ww.mem); ww.mem = nullptr; }
    pixels = std::max(pixels, ww.pixels);
    tiles = std::max(tiles, ww.tiles);
    col = col || ww.col;
    pay = std::max(pay, ww.pay);
    const size_t ns = pixels * (size_t)std::max(slots, 1);
    const size_t nq = tiles * 256 * (size_t)std::max(slots, 1);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    size_t off[13], total = 0;
    const size_t sz[13] = {pixels * 4, pixels * 4, pixels * 4, pixels * 16, ns * 16, ns, nq * 16, nq * 16, nq * 4,
                           tiles * 4, pixels * 16, (size_t)tiles * 256 * 16 * pay, col ? pixels * 16 : 0};
    for (int k = 0; k < 13; ++k) { off[k] = total; total += al(sz[k]); }
    HIP_TRY(hipMalloc(&ww.mem, total));
    char* b = (char*)ww.mem;
    rtg::WaveBufs& W = ww.W;
    W.hit_t = (float*)(b + off[0]); W.hit_obj = (int*)(b + off[1]); W.hit_face = (int*)(b + off[2]);
    W.base = (float4*)(b + off[3]); W.term = (float4*)(b + off[4]); W.occ = (unsigned char*)(b + off[5]);
    W.q_o = (float4*)(b + off[6]); W.q_d = (float4*)(b + off[7]); W.q_slot = (int*)(b + off[8]);
    W.q_count = (int*)(b + off[9]); W.accum = (float4*)(b + off[10]);
    W.q_pay = pay ? (float4*)(b + off[11]) : nullptr;
    W.pay3 = pay == 3;
    ww.pay = pay;
    W.col = col ? (float4*)(b + off[12]) : nullptr;
    ww.col = col;
    ww.pixels = pixels;
    ww.slots = slots;
    ww.tiles = tiles;
    W.dq_e = nullptr;
    W.dq_count = nullptr;
    W.hit_key = nullptr;
    W.shadow_state = nullptr;
    W.dq_cap = 0;
    ww.dq_nq = 0;
    ww.dq_pixels = 0;
    return RTG_OK;
}

// The deferred-leaf queue of a large-leaf scene's camera walk (WaveBufs dq_*, hit_key): two
// entries per pixel of capacity (an entry that does not fit is tested in the walk).
// Layout [256 B counts | pixels x 8 B keys | cap x 48 B entries | nq x 4 B states]: the entry
// and state offsets depend on the pixel count, so a buffer laid out for fewer pixels is never
// reused (the 1 024-entry floor on cap alone would let keys overrun the entries).
static int ensure_defer(WaveWork& ww, size_t pixels, size_t nq) {
    if (ww.dq && ww.dq_pixels >= pixels && ww.W.dq_cap >= (int)std::max<size_t>(2 * pixels, 1024) && ww.dq_nq >= nq)
        return RTG_OK;
    if (ww.dq) { (void)hipFree(ww.dq); ww.dq = nullptr; }
    nq = std::max(nq, ww.dq_nq);
    pixels = std::max(pixels, ww.dq_pixels);
    const size_t cap = std::max<size_t>(2 * pixels, 1024);
    const size_t bytes = 256 + pixels * 8 + cap * 48 + nq * 4;
    HIP_TRY(hipMalloc(&ww.dq, bytes));
    // the counters start at zero; the kernels after their last readers zero them for the next
    // pass (k_shade: camera entries / unsettled pixels, k_shadow_fin*: shadow entries)
    HIP_TRY(hipMemset(ww.dq, 0, 256));
    char* b = (char*)ww.dq;
    ww.W.dq_count = (int*)b;
    ww.W.hit_key = (unsigned long long*)(b + 256);
    ww.W.dq_e = (float4*)(b + 256 + pixels * 8);
    ww.W.shadow_state = (int*)(b + 256 + pixels * 8 + cap * 48);
    ww.W.dq_cap = (int)cap;
    ww.dq_nq = nq;
    ww.dq_pixels = pixels;
    return RTG_OK;
}

// The render pipeline a frame part takes (launch): path tracer, ray trees, wavefront, fused.
enum { PIPE_PATH, PIPE_TREE, PIPE_WAVE, PIPE_MEGA };
static int pipeline(const rtg_scene* s, const rtg_render_opts* o, const rtg::DevCamera& C, const rtg::RenderParams& P) {
    if (C.path_tracing && s->path_ok && !(o->flags & RTG_RENDER_FUSED) && (o->flags & RTG_RENDER_TREE)) return PIPE_PATH;
    const long long work = (long long)P.part_rows * C.width * P.sample_count;
    const bool fused_only = (o->flags & RTG_RENDER_FUSED) || C.path_tracing;
    if (s->tree_ok && !fused_only && ((o->flags & RTG_RENDER_TREE) || work >= (1ll << 21))) return PIPE_TREE;
    if (s->wave_ok && !fused_only) return PIPE_WAVE;
    return PIPE_MEGA;
}

// Samples per pass of the wavefront and ray-tree pipelines (RenderParams::slabs): as many as
// keep a pass at most ~RTG_PASS_RAYS camera rays (default 16 Mi: a 1920x1080 frame of 8 samples,
// two 3840x2160 samples -- against 8 Mi: C4 3 519 -> 3 563 Mrays/s in flight, 3 203 -> 3 356
// serial, C5 2 265 -> 2 329; profiles/r06u_pass_rays_ab.txt), spread evenly over the passes.  A pass's launches then stay full when
// a GPU renders a small part of the frame, and a frame of few passes pays the tail of its
// slowest waves (C3's pole fans, C5's deepest trees) once per pass, not once per sample.
// RTG_PASS_RAYS=0: one sample per pass (round 5's passes; the image is the same bit for bit).
static int pass_slabs(const rtg::RenderParams& P, int width) {
    const char* v = std::getenv("RTG_PASS_RAYS");
    const long long target = v ? std::atoll(v) : (16ll << 20);
    const long long px = (long long)P.part_rows * width;
    if (target <= 0 || P.sample_count <= 1 || px <= 0) return 1;
    const long long k = std::max(1ll, std::min<long long>(target / px, P.sample_count));
    const long long passes = (P.sample_count + k - 1) / k;
    return (int)((P.sample_count + passes - 1) / passes);
}

// samples of the last pass (the one RTG_RENDER_TIMING times)
static int last_pass_samples(const rtg::RenderParams& P) {
    return P.sample_count - ((P.sample_count - 1) / P.slabs) * P.slabs;
}

static int launch(rtg_scene* s, const rtg_render_opts* o, const rtg::DevCamera& C, const rtg::RenderParams& P0,
                  float* d_hdr, uint8_t* d_ldr, float* d_accum, hipStream_t stream) {
    WaveWork& ww = s->work[0];
    int pipe = pipeline(s, o, C, P0);
    rtg::RenderParams P = P0;
    if ((pipe == PIPE_WAVE || pipe == PIPE_TREE) && !(o->flags & RTG_RENDER_SAMPLE_PASSES)) {
        P.slabs = pass_slabs(P, C.width);
        if (P.slabs > 1) P.slab_tiles = (P.num_tiles + 7) & ~7;   // a tile keeps its XCD in every slab
    }
    const bool stats = (o->flags & RTG_RENDER_COUNT_STATS) != 0;
    // RTG_RENDER_EXACT_SHADOW: shadow rays walk the reference BVH (cross-checks of the wide one)
    rtg::DevScene ds = s->ds;
    if (o->flags & RTG_RENDER_EXACT_SHADOW) ds.exact_shadow = 1;
    // RTG_RENDER_ORDERED: the checked closest-hit walk on the any-hit tree (its leaf boxes must be
    // the reference's: not the split tree).  (Round 3's per-lane walk of the reference tree
    // collapsed to 4 wide was removed in round 6.)
    if ((o->flags & RTG_RENDER_ORDERED) && ds.anodes && !ds.ahb_split && ds.face_leaf) ds.ordered = 1;
    hipEvent_t* ev = nullptr;
    if (o->flags & RTG_RENDER_TIMING) {
        for (auto& e : s->ev)
            if (!e) HIP_TRY(hipEventCreate(&e));
        ev = s->ev;
    }
    // ray trees: the wavefront tree pipeline for large frames (it synchronises once per tree
    // level), the fused kernel otherwise; RTG_RENDER_TREE / RTG_RENDER_FUSED force either.
    // Path tracing: the fused kernel; the wavefront path tracer (rtg_path.hip, same image bit
    // for bit) with RTG_RENDER_TREE -- measured slower than the fused kernel on the path-tracing
    // fixtures, so it is opt-in
    if (pipe == PIPE_PATH) {
        float4* acc = (float4*)d_accum;
        if (!P.accum_only && C.spp > 1) {   // internal accumulator indexed by absolute pixel
            int rc = ensure_wave(ww, (size_t)C.width * C.height, s->num_slots, (size_t)P.num_tiles, 0);
            if (rc) return rc;
            acc = ww.W.accum;
        }
        // a counted render that falls back to the fused kernel must not keep the abandoned
        // pass's counts: snapshot the counters, restore them before the fused kernel runs
        rtg::DevCounters snap{};
        if (stats) {
            HIP_TRY(hipMemcpyAsync(&snap, s->counters.p, sizeof(snap), hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
        }
        const hipError_t pe = rtg::launch_path(s->path, ds, C, P, d_hdr, d_ldr, acc, s->counters.p, stats, s->feat,
                                               s->shade_sk, stream, ev);
        if (pe == hipSuccess) {
            if (ev) { s->timed_layout = rtg::LAYOUT_PATH; s->timed_samples = 1; }
            return RTG_OK;
        }
        if (pe != hipErrorNotSupported) HIP_TRY(pe);
        (void)hipGetLastError();
        if (stats) {
            HIP_TRY(hipMemcpyAsync(s->counters.p, &snap, sizeof(snap), hipMemcpyHostToDevice, stream));
            HIP_TRY(hipStreamSynchronize(stream));
        }
        pipe = PIPE_MEGA;                   // path-tracing cameras: the fused kernel
    }
    if (pipe == PIPE_TREE) {
        float4* acc = (float4*)d_accum;
        if (!P.accum_only && C.spp > 1) {   // internal accumulator indexed by absolute pixel
            int rc = ensure_wave(ww, (size_t)C.width * C.height, s->num_slots, (size_t)P.num_tiles, 0);
            if (rc) return rc;
            acc = ww.W.accum;
        }
        HIP_TRY(rtg::launch_tree(s->tree, ds, C, P, d_hdr, d_ldr, acc, s->counters.p, stats, s->feat, s->shade_sk,
                                 stream, ev));
        if (ev) { s->timed_layout = rtg::LAYOUT_TREE; s->timed_samples = last_pass_samples(P); }
        return RTG_OK;
    }
    if (pipe == PIPE_WAVE) {
        // work-buffer entries and shade blocks of a pass (all its sample slabs)
        const size_t entries = P.slabs > 1 ? (size_t)P.slabs * P.slab_px : (size_t)P.part_rows * C.width;
        const size_t blocks = (size_t)P.slab_tiles * P.slabs;
        int rc = ensure_wave(ww, entries, s->num_slots, blocks, one_payload(s), P.slabs > 1);
        if (rc) return rc;

        rtg::WaveBufs W = ww.W;
        W.num_slots = s->num_slots;
        if (P.accum_only) W.accum = (float4*)d_accum;
        else if (C.spp > 1) {   // internal accumulator indexed by absolute pixel
            size_t need = (size_t)C.width * C.height;
            if (need > ww.pixels) {
                int rc2 = ensure_wave(ww, need, s->num_slots, blocks, one_payload(s), P.slabs > 1);
                if (rc2) return rc2;
                W = ww.W;
                W.num_slots = s->num_slots;
            }
        }
        if ((s->feat & rtg::FEAT_BIGLEAF) && !stats && rtg::defer_leaves()) {
            rc = ensure_defer(ww, entries, blocks * 256 * std::max(s->num_slots, 1));
            if (rc) return rc;
            W.dq_e = ww.W.dq_e;
            W.dq_count = ww.W.dq_count;
            W.hit_key = ww.W.hit_key;
            W.shadow_state = ww.W.shadow_state;
            W.dq_cap = ww.W.dq_cap;
        }
        int layout = rtg::LAYOUT_WAVE;
        HIP_TRY(rtg::launch_wave(ds, C, P, W, d_hdr, d_ldr, s->counters.p, stats, s->feat, s->shade_sk, stream, ev,
                                 &layout));
        if (ev) { s->timed_layout = layout; s->timed_samples = last_pass_samples(P); }
        return RTG_OK;
    }
    HIP_TRY(rtg::launch_mega(ds, C, P, d_hdr, d_ldr, d_accum, s->counters.p, stats, s->shade_sk, s->feat, stream, ev));
    if (ev) { s->timed_layout = rtg::LAYOUT_MEGA; s->timed_samples = P.sample_count; }
    return RTG_OK;
}

int rtg_render_device(rtg_scene* s, const rtg_render_opts* o, float* d_hdr, uint8_t* d_ldr, float* d_accum,
                      void* stream) {
    rtg::DevCamera C;
    rtg::RenderParams P;
    int rc = prepare(s, o, C, P);
    if (rc) return rc;
    if (P.accum_only && !d_accum) return set_err(RTG_ERR_INVALID, "RTG_RENDER_ACCUM_ONLY needs an accumulation buffer");
    if (P.num_tiles == 0) return RTG_OK;
    HIP_TRY(hipSetDevice(s->device));
    rc = launch(s, o, C, P, d_hdr, d_ldr, d_accum, (hipStream_t)stream);
    if (rc) return rc;
    // the completion marker rtg_scene_stats waits for (round 4 measured a render without it: the
    // same part-frame time, profiles/r04f_parts_ab.jsonl)
    HIP_TRY(hipEventRecord(s->done, (hipStream_t)stream));
    return RTG_OK;
}

// D2H of the rows of opts' part: one async copy per run of consecutive rows, straight into
// the same offsets of the host frame (layout 3*(x + y*width), main.cpp:109).
static int copy_part(const rtg_render_opts* o, int width, int height, const float* d_hdr, const uint8_t* d_ldr,
                     float* hdr, uint8_t* ldr, hipStream_t st) {
    const int rb = o->row_begin < 0 ? 0 : o->row_begin;
    const int re = (o->row_end <= 0 || o->row_end > height) ? height : o->row_end;
    int32_t n = 0;
    int rc = rtg_part_runs(rb, re, o->part_index, o->part_count, nullptr, 0, &n);
    if (rc) return rc;
    std::vector<int32_t> runs(2 * (size_t)n);
    rc = rtg_part_runs(rb, re, o->part_index, o->part_count, runs.data(), n, &n);
    if (rc) return rc;
    for (int k = 0; k < n; ++k) {
        const size_t off = (size_t)runs[2 * k] * width * 3, cnt = (size_t)(runs[2 * k + 1] - runs[2 * k]) * width * 3;
        if (hdr && d_hdr) HIP_TRY(hipMemcpyAsync(hdr + off, d_hdr + off, cnt * sizeof(float), hipMemcpyDeviceToHost, st));
        if (ldr && d_ldr) HIP_TRY(hipMemcpyAsync(ldr + off, d_ldr + off, cnt, hipMemcpyDeviceToHost, st));
    }
    return RTG_OK;
}

int rtg_copy_part_to_host(rtg_scene* s, const rtg_render_opts* o, const float* d_hdr, const uint8_t* d_ldr,
                          float* hdr_rgb, uint8_t* ldr_rgb, void* stream) {
    if (!s || !o) return set_err(RTG_ERR_INVALID, "null argument");
    if (o->camera < 0 || o->camera >= (int)s->cameras.size()) return set_err(RTG_ERR_INVALID, "bad camera %d", o->camera);
    const rtg_camera& c = s->cameras[o->camera];
    HIP_TRY(hipSetDevice(s->device));
    return copy_part(o, c.width, c.height, d_hdr, d_ldr, hdr_rgb, ldr_rgb, (hipStream_t)stream);
}

// (Round 4's overlapped host path -- the frame rendered in row chunks on two streams, each
// chunk's rows copied to the host under the next chunks -- measured slower than one launch + one
// copy at every chunk count, profiles/r04d_hostpath.jsonl, and was removed in round 6; page-locked
// frames take the direct writes below.)

// The device's view of a page-locked host buffer (rtg_host_alloc / rtg_host_register), or null.
static void* device_view(void* p) {
    if (!p) return nullptr;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}
// Page-locked caller frames (rtg_host_alloc / rtg_host_register, as the CLIs and the shared
// frame of multigpu.py allocate them): the kernels write the pixels straight into the frame over
// the bus -- no device frame and no copy after the render, the writes overlap the rendering
// (headline 1080p frame: 0.53 -> 0.46 ms per frame, profiles/r04e_hostpath.jsonl).  Pageable
// frames take the render + copy path.  RTG_HOST_DIRECT=0: render + copy always (A/B).
static bool host_direct() {
    const char* v = std::getenv("RTG_HOST_DIRECT");
    return !v || std::strcmp(v, "0") != 0;
}

// Replaces main.cpp:164-185.  With replicas (rtg_scene_create_multi) replica i renders part
// i of n on its own stream and copies its rows into the caller's buffers; the renders of all
// replicas are enqueued before any copy (a copy to pageable memory may block the host), then
// every stream is synchronised -- never the whole device.
int rtg_render(rtg_scene* s, const rtg_render_opts* o, float* hdr_rgb, uint8_t* ldr_rgb) {
    if (!s || !o) return set_err(RTG_ERR_INVALID, "null argument");
    if (o->flags & RTG_RENDER_ACCUM_ONLY) return set_err(RTG_ERR_INVALID, "use rtg_render_device for RTG_RENDER_ACCUM_ONLY");
    std::vector<rtg_scene*> reps(1, s);
    reps.insert(reps.end(), s->replicas.begin(), s->replicas.end());
    const int n = (int)reps.size();
    if (n > 1 && o->part_count > 1)
        return set_err(RTG_ERR_INVALID, "a multi-device scene deals its own partition (part_count must be <= 1)");
    if (o->camera < 0 || o->camera >= (int)s->cameras.size()) return set_err(RTG_ERR_INVALID, "bad camera %d", o->camera);
    const rtg_camera& cam = s->cameras[o->camera];
    std::vector<rtg_render_opts> ro(n, *o);
    bool whole = false;
    if (n == 1 && host_direct() && !cam.has_tonemapper && (hdr_rgb || ldr_rgb)) {
        float* dh = (float*)device_view(hdr_rgb);
        uint8_t* dl = (uint8_t*)device_view(ldr_rgb);
        if ((!hdr_rgb || dh) && (!ldr_rgb || dl)) {
            rtg::DevCamera C;
            rtg::RenderParams P;
            int rc = prepare(s, o, C, P);
            if (rc) return rc;
            if (P.num_tiles == 0) return RTG_OK;
            HIP_TRY(hipSetDevice(s->device));
            rc = launch(s, o, C, P, dh, dl, nullptr, s->stream);
            if (rc) return rc;
            HIP_TRY(hipEventRecord(s->done, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            return RTG_OK;
        }
    }
    for (int i = 0; i < n; ++i) {
        rtg_scene* r = reps[i];
        if (n > 1) { ro[i].part_index = i; ro[i].part_count = n; }
        rtg::DevCamera C;
        rtg::RenderParams P;
        int rc = prepare(r, &ro[i], C, P);
        if (rc) return rc;
        whole = P.row_begin == 0 && P.row_end == C.height && (n > 1 || P.part_count == 1);
        HIP_TRY(hipSetDevice(r->device));
        const size_t pixels = (size_t)C.width * C.height;
        if (r->d_pixels < pixels) {
            HIP_TRY(hipStreamSynchronize(r->stream));
            if (r->d_hdr) { (void)hipFree(r->d_hdr); r->d_hdr = nullptr; }
            if (r->d_ldr) { (void)hipFree(r->d_ldr); r->d_ldr = nullptr; }
            r->d_pixels = 0;
            HIP_TRY(hipMalloc(&r->d_hdr, pixels * 3 * sizeof(float)));
            HIP_TRY(hipMalloc(&r->d_ldr, pixels * 3));
            r->d_pixels = pixels;
        }
        if (P.num_tiles == 0) continue;
        rc = launch(r, &ro[i], C, P, r->d_hdr, r->d_ldr, nullptr, r->stream);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(r->done, r->stream));
    }
    // tonemapped camera over the whole image: the LDR output is the tonemapped image
    // (main.cpp:187-192); it needs every pixel, so with several parts it runs on the
    // gathered float image
    const bool tonemap = cam.has_tonemapper && whole;
    const rtg_tonemap_params tp = {cam.tm_key, cam.tm_burn, cam.tm_saturation, cam.tm_gamma};
    if (tonemap && n == 1) {
        int rc = rtg_tonemap_device(s->d_hdr, cam.width, cam.height, &tp, s->d_ldr, s->device, s->stream);
        if (rc) return rc;
    }
    std::vector<float> tmp;
    float* hdr = hdr_rgb;
    if (tonemap && n > 1 && ldr_rgb && !hdr) {
        tmp.resize((size_t)cam.width * cam.height * 3);
        hdr = tmp.data();
    }
    for (int i = 0; i < n; ++i) {
        HIP_TRY(hipSetDevice(reps[i]->device));
        int rc = copy_part(&ro[i], cam.width, cam.height, reps[i]->d_hdr, reps[i]->d_ldr, hdr,
                           (tonemap && n > 1) ? nullptr : ldr_rgb, reps[i]->stream);
        if (rc) return rc;
    }
    for (int i = 0; i < n; ++i) {
        HIP_TRY(hipSetDevice(reps[i]->device));
        HIP_TRY(hipStreamSynchronize(reps[i]->stream));
    }
    if (tonemap && n > 1 && ldr_rgb) return rtg_tonemap(hdr, cam.width, cam.height, &tp, ldr_rgb, s->device);
    return RTG_OK;
}

int rtg_host_alloc(size_t bytes, void** out) {
    if (!out || !bytes) return set_err(RTG_ERR_INVALID, "bad arguments");
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocPortable));
    return RTG_OK;
}

int rtg_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return RTG_OK;
}

int rtg_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return set_err(RTG_ERR_INVALID, "bad arguments");
    HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterPortable));
    return RTG_OK;
}

int rtg_host_unregister(void* p) {
    if (!p) return set_err(RTG_ERR_INVALID, "null argument");
    HIP_TRY(hipHostUnregister(p));
    return RTG_OK;
}

int rtg_tonemap_device(const float* d_hdr, int32_t w, int32_t h, const rtg_tonemap_params* tp, uint8_t* d_ldr,
                       int32_t device, void* stream) {
    if (!d_hdr || !d_ldr || !tp || w <= 0 || h <= 0) return set_err(RTG_ERR_INVALID, "bad tonemap arguments");
    HIP_TRY(hipSetDevice(device));
    hipStream_t st = (hipStream_t)stream;
    void* scratch = nullptr;
    HIP_TRY(hipMallocAsync(&scratch, rtg::tonemap_scratch_bytes((long long)w * h), st));
    hipError_t e = rtg::launch_tonemap(d_hdr, w, h, tp->key, tp->burn_percent, tp->saturation, tp->gamma, d_ldr, scratch, st);
    hipError_t e2 = hipFreeAsync(scratch, st);
    HIP_TRY(e);
    HIP_TRY(e2);
    return RTG_OK;
}

int rtg_tonemap(const float* hdr, int32_t w, int32_t h, const rtg_tonemap_params* tp, uint8_t* ldr, int32_t device) {
    if (!hdr || !ldr || !tp || w <= 0 || h <= 0) return set_err(RTG_ERR_INVALID, "bad tonemap arguments");
    HIP_TRY(hipSetDevice(device));
    const size_t n = (size_t)w * h * 3;
    float* dh = nullptr;
    uint8_t* dl = nullptr;
    HIP_TRY(hipMalloc(&dh, n * sizeof(float)));
    if (hipMalloc(&dl, n) != hipSuccess) { (void)hipFree(dh); return set_err(RTG_ERR_NOMEM, "device allocation failed"); }
    int rc = RTG_OK;
    if (hipMemcpy(dh, hdr, n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) rc = set_err(RTG_ERR_HIP, "copy failed");
    if (!rc) rc = rtg_tonemap_device(dh, w, h, tp, dl, device, nullptr);
    if (!rc && hipMemcpy(ldr, dl, n, hipMemcpyDeviceToHost) != hipSuccess) rc = set_err(RTG_ERR_HIP, "copy failed");
    (void)hipFree(dh);
    (void)hipFree(dl);
    return rc;
}

int rtg_tonemap_log_average(const float* hdr, int32_t w, int32_t h, int32_t mode, double* avg_out, int32_t device) {
    if (!hdr || !avg_out || w <= 0 || h <= 0 || mode > 3) return set_err(RTG_ERR_INVALID, "bad log-average arguments");
    HIP_TRY(hipSetDevice(device));
    const size_t n = (size_t)w * h;
    float* dh = nullptr;
    void* scratch = nullptr;
    HIP_TRY(hipMalloc(&dh, 3 * n * sizeof(float)));
    if (hipMalloc(&scratch, rtg::tonemap_scratch_bytes((long long)n)) != hipSuccess) {
        (void)hipFree(dh);
        return set_err(RTG_ERR_NOMEM, "device allocation failed");
    }
    int rc = RTG_OK;
    if (hipMemcpy(dh, hdr, 3 * n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) rc = set_err(RTG_ERR_HIP, "copy failed");
    if (!rc) {
        rtg::launch_log_average(dh, (long long)n, mode, 0, scratch, nullptr);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpy(avg_out, (char*)scratch + rtg::tonemap_avg_offset(), sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
            rc = set_err(RTG_ERR_HIP, "log-average failed");
    }
    (void)hipFree(dh);
    (void)hipFree(scratch);
    return rc;
}

int rtg_resolve_accum(const float* accum, int32_t w, int32_t h, float* hdr, uint8_t* ldr) {
    if (!accum || w <= 0 || h <= 0) return set_err(RTG_ERR_INVALID, "bad accumulation buffer");
    for (size_t p = 0; p < (size_t)w * h; ++p) {
        const float* a = accum + 4 * p;
        for (int k = 0; k < 3; ++k) {
            float c = a[k] / a[3];
            if (hdr) hdr[3 * p + k] = c;
            if (ldr) {
                int i = (c > -2147483904.0f && c < 2147483648.0f) ? (int)c : (int)0x80000000;
                ldr[3 * p + k] = (uint8_t)(i < 0 ? 0 : (i > 255 ? 255 : i));
            }
        }
    }
    return RTG_OK;
}

int rtg_scene_stats(rtg_scene* s, rtg_stats* out) {
    if (!s || !out) return set_err(RTG_ERR_INVALID, "null argument");
    std::vector<rtg_scene*> reps(1, s);
    reps.insert(reps.end(), s->replicas.begin(), s->replicas.end());
    std::memset(out, 0, sizeof(*out));
    for (rtg_scene* r : reps) {
        HIP_TRY(hipSetDevice(r->device));
        rtg::DevCounters c;
        HIP_TRY(hipEventSynchronize(r->done));
        HIP_TRY(hipMemcpy(&c, r->counters.p, sizeof(c), hipMemcpyDeviceToHost));
        out->camera_rays += c.camera_rays;
        out->secondary_rays += c.secondary_rays;
        out->shadow_rays += c.shadow_rays;
        out->node_visits += c.node_visits;
        out->tri_tests += c.tri_tests;
        out->sphere_tests += c.sphere_tests;
        out->object_tests += c.object_tests;
        out->shadow_node_visits += c.shadow_node_visits;
        out->shadow_tri_tests += c.shadow_tri_tests;
        out->shadow_wide_visits += c.shadow_wide_visits;
        out->shadow_fallbacks += c.shadow_fallbacks;
        out->extend_wide_visits += c.extend_wide_visits;
        out->extend_fallbacks += c.extend_fallbacks;
    }
    return RTG_OK;
}

int rtg_scene_reset_stats(rtg_scene* s) {
    if (!s) return set_err(RTG_ERR_INVALID, "null argument");
    std::vector<rtg_scene*> reps(1, s);
    reps.insert(reps.end(), s->replicas.begin(), s->replicas.end());
    for (rtg_scene* r : reps) {
        HIP_TRY(hipSetDevice(r->device));
        HIP_TRY(hipEventSynchronize(r->done));
        // on the scene's (non-blocking) stream, complete before return: ordered before the
        // next render whichever stream that one runs on
        HIP_TRY(hipMemsetAsync(r->counters.p, 0, sizeof(rtg::DevCounters), r->stream));
        HIP_TRY(hipStreamSynchronize(r->stream));
    }
    return RTG_OK;
}

int rtg_scene_timings(rtg_scene* s, float* ms, const char** names, int32_t cap, int32_t* count) {
    // stage names per layout (rtg_kernels.hpp LAYOUT_*)
    static const char* kNames[7][rtg::MAX_STAGES] = {{"k_primary", "k_shade", "k_shadow", "k_resolve"},
                                                     {"k_primary", "k_shade", "k_shadow"},
                                                     {"k_primary", "k_shade_shadow"},
                                                     {"tree_levels", "tree_resolve"},
                                                     {"k_render"},
                                                     {"path_iterations"},
                                                     {"k_frame"}};
    static const int kCount[7] = {rtg::WAVE_STAGES, 3, 2, rtg::TREE_STAGES, rtg::MEGA_STAGES, rtg::PATH_STAGES, 1};
    if (!s || !count) return set_err(RTG_ERR_INVALID, "null argument");
    if (s->timed_layout < 0) return set_err(RTG_ERR_INVALID, "no render was issued with RTG_RENDER_TIMING");
    HIP_TRY(hipSetDevice(s->device));
    const int n = kCount[s->timed_layout];
    HIP_TRY(hipEventSynchronize(s->ev[n]));
    const char* const* nm = kNames[s->timed_layout];
    for (int k = 0; k < n && k < cap; ++k) {
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, s->ev[k], s->ev[k + 1]));
        if (ms) ms[k] = t;
        if (names) names[k] = nm[k];
    }
    *count = n;
    return RTG_OK;
}

int rtg_scene_timed_samples(const rtg_scene* s, int32_t* samples) {
    if (!s || !samples) return set_err(RTG_ERR_INVALID, "null argument");
    if (s->timed_layout < 0) return set_err(RTG_ERR_INVALID, "no render was issued with RTG_RENDER_TIMING");
    *samples = s->timed_samples;
    return RTG_OK;
}

int rtg_write_png(const char* path, int32_t w, int32_t h, const uint8_t* rgb) {
    std::string err;
    if (!path || !rgb || w <= 0 || h <= 0) return set_err(RTG_ERR_INVALID, "bad arguments");
    if (!rtg::write_png(path, w, h, rgb, err)) return set_err(RTG_ERR_IO, "%s", err.c_str());
    return RTG_OK;
}

int rtg_write_hdr(const char* path, int32_t w, int32_t h, const float* rgb) {
    std::string err;
    if (!path || !rgb || w <= 0 || h <= 0) return set_err(RTG_ERR_INVALID, "bad arguments");
    if (!rtg::write_hdr(path, w, h, rgb, err)) return set_err(RTG_ERR_IO, "%s", err.c_str());
    return RTG_OK;
}

}  // extern "C"

extern "C" int rtg_desc_anyhit_check(const rtg_scene_desc* d, int32_t mode, int64_t* out, int32_t n_out) {
    if (!d || !out || n_out < 8 || mode < 0 || mode > 2) return set_err(RTG_ERR_INVALID, "bad argument");
    if (d->num_faces > 0 && d->num_nodes == 0) return set_err(RTG_ERR_INVALID, "description without a BVH");
    try {
        std::vector<float4> nodes;
        std::vector<int2> next;
        std::vector<int> meshBegin(d->num_meshes), meshEnd(d->num_meshes);
        bool bigleaf = false;
        int rc = reference_preorder(d, nodes, next, meshBegin, meshEnd, bigleaf);
        if (rc) return rc;
        nodes.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
        nodes.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
        std::vector<float4> tris(3 * (size_t)d->num_faces);
        for (int64_t f = 0; f < d->num_faces; ++f) {
            const rtg_face& F = d->faces[f];
            tris[3 * f] = make_float4(F.v0.x, F.v0.y, F.v0.z, 0.f);
            tris[3 * f + 1] = make_float4(F.v0.x - F.v1.x, F.v0.y - F.v1.y, F.v0.z - F.v1.z, 0.f);
            tris[3 * f + 2] = make_float4(F.v0.x - F.v2.x, F.v0.y - F.v2.y, F.v0.z - F.v2.z, 0.f);
        }
        std::vector<rtg::WNode> anodes;
        std::vector<float4> ahtris;
        std::vector<int> aroot;
        rtg::AhbStats ast;
        const bool ok = anyhit_trees(d, nodes, next, meshBegin, meshEnd, tris.data(), mode, anodes, ahtris, aroot, ast);
        long long bad = 0;
        for (int m = 0; m < d->num_meshes && ok; ++m)
            bad += rtg::ahb_validate(anodes, ahtris, aroot[m], nodes, next, meshBegin[m], meshEnd[m], tris.data());
        const int64_t v[8] = {ast.nodes, ast.entries, ast.max_depth, ast.leaf_prims, ast.face_prims, ast.exact_faces,
                              bad, ok ? 1 : 0};
        for (int k = 0; k < 8; ++k) out[k] = v[k];
    } catch (const std::bad_alloc&) {
        return set_err(RTG_ERR_NOMEM, "out of memory");
    }
    return RTG_OK;
}
