// ORACLE -- test infrastructure only.  CPU restatement of the reference's per-pixel
// trace/shade path, used by tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg as the CHECKER.  Nothing in the product (librtgpu.so, rtgpu CLI)
// links, loads or calls this file.
//
// It restates, over the flattened rtg_scene_desc, the reference's own recursive
// structure:
//   RenderPixel/PerPixel          raytracer.cpp:33-63
//   IntersectObjects              raytracer.cpp:625-643
//   Mesh::Intersect               mesh.cpp:158-188
//   InstancedMesh::Intersect      instancedMesh.cpp:16-66
//   BVH::IntersectBVH (recursive) bvh.cpp:5-30
//   Mesh::IntersectFace           mesh.cpp:201-372
//   Sphere::Intersect             sphere.cpp:13-180
//   BoundingBox::doesIntersect    shape.hpp:78-100
//   PerformShading                raytracer.cpp:65-134
//   Shade / GetDiffuse / ...      raytracer.cpp:192-206, 474-554
//   SampleDirectLighting          raytracer.cpp:701-805 (+ MeshLight::getSample, meshLight.h:27-47)
//   ComputeGlobalIllumination     raytracer.cpp:135-191 (path tracing, Russian roulette)
//   IsInShadow / CastShadowRay    raytracer.cpp:555-623
//   Mirror/Dielectric/Conductor   raytracer.cpp:208-472
//   BRDFs                         brdf{Phong,BlinnPhong,ModifiedPhong,ModifiedBlinnPhong,TorranceSparrow}.cpp
//   Lights                        areaLight.h, spotLight.h, sphericalEnvironmentLight.h
//   Textures                      imageTexture.h:60-133, perlinTexture.h:57-160
//   renderThreadMain sampling     main.cpp:42-125, gaussian.h
// with one deliberate substitution: the reference's shared std::mt19937 streams are
// replaced by the counter-based RNG the GPU path uses (keyed by pixel, sample and
// ray-tree node), so stochastic scenes are comparable bit-for-bit with the GPU and
// statistically with the reference.  Deterministic scenes need no RNG at all and are
// pinned bit-for-bit against the reference itself (oracle/_ref, tests/golden).
//
// Build: g++ -O2 -ffp-contract=off (no FMA contraction, like the reference binary).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "rtgpu.h"

namespace {

// ---------------- helperMath.cpp ----------------
struct Vec3f { float x = 0, y = 0, z = 0; };
Vec3f V(float x, float y, float z) { Vec3f r; r.x = x; r.y = y; r.z = z; return r; }
Vec3f V(const rtg_float3& a) { return V(a.x, a.y, a.z); }
Vec3f operator+(const Vec3f& a, const Vec3f& b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
Vec3f operator-(const Vec3f& a, const Vec3f& b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
Vec3f operator*(const Vec3f& a, const Vec3f& b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
Vec3f operator*(const Vec3f& a, float s) { return V(a.x * s, a.y * s, a.z * s); }
Vec3f operator/(const Vec3f& a, float s) { return V(a.x / s, a.y / s, a.z / s); }
Vec3f operator-(const Vec3f& a) { return V(a.x * -1.0f, a.y * -1.0f, a.z * -1.0f); }
float dot(const Vec3f& a, const Vec3f& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
Vec3f cross(const Vec3f& a, const Vec3f& b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
float len(Vec3f a) { return sqrtf((a.x * a.x) + (a.y * a.y) + (a.z * a.z)); }
Vec3f makeUnit(Vec3f a) { float l = len(a); return V(a.x / l, a.y / l, a.z / l); }
float determinant(float m[3][3]) {
    float firstTerm = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]);
    float secondTerm = m[1][0] * (m[0][2] * m[2][1] - m[0][1] * m[2][2]);
    float thirdTerm = m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2]);
    return firstTerm + secondTerm + thirdTerm;
}
void GetOrthonormalBasis(Vec3f r, Vec3f& u, Vec3f& v) {
    float absX = std::fabs(r.x), absY = std::fabs(r.y), absZ = std::fabs(r.z);
    Vec3f rPrime = r;
    if (absX < absY) { if (absX < absZ) rPrime.x = 1.0f; else rPrime.z = 1.0f; }
    else { if (absY < absZ) rPrime.y = 1.0f; else rPrime.z = 1.0f; }
    u = makeUnit(cross(rPrime, r));
    v = makeUnit(cross(r, u));
}
const double RAD2DEG = (180.0f / M_PI);
const double DEG2RAD = (M_PI / 180.0f);
template <class T> const T& smin(const T& a, const T& b) { return (b < a) ? b : a; }   // std::min
template <class T> const T& smax(const T& a, const T& b) { return (a < b) ? b : a; }   // std::max
double angleBetweenUnitVectors(const Vec3f& v1, const Vec3f& v2) {
    return std::acos(smin(1.0f, smax(-1.0f, dot(v1, v2)))) * RAD2DEG;
}
double cosDeg(double a) { return std::cos(a * DEG2RAD); }

// matrix.hpp ApplyTransform (double, rows 0..2)
Vec3f applyT(const double* t, Vec3f v, float w) {
    Vec3f r;
    r.x = t[0] * v.x + t[1] * v.y + t[2] * v.z + t[3] * w;
    r.y = t[4] * v.x + t[5] * v.y + t[6] * v.z + t[7] * w;
    r.z = t[8] * v.x + t[9] * v.y + t[10] * v.z + t[11] * w;
    return r;
}

// ---------------- counter-based RNG (identical to the GPU path) ----------------
uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
float rnd(uint64_t key, uint32_t purpose, uint32_t idx) {
    uint64_t h = mix64(key ^ mix64(((uint64_t)purpose << 32) | idx));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}
uint64_t child_key(uint64_t key, int slot) { return mix64(key + 0x632BE59BD9B4E019ULL * (uint64_t)(slot + 1)); }
uint64_t root_key(uint64_t seed, int pixel, int sample) {
    return mix64(mix64(seed ^ 0xD1B54A32D192ED03ULL) ^ ((uint64_t)(uint32_t)pixel * 0x9E3779B97F4A7C15ULL) ^
                 ((uint64_t)(uint32_t)sample << 1));
}
double rndd(uint64_t key, uint32_t purpose, uint32_t idx) {
    uint64_t h = mix64(key ^ mix64(((uint64_t)purpose << 32) | idx));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
enum { RP_MOTION = 1, RP_DOF = 2, RP_JITTER = 3, RP_AREA = 4, RP_ENV = 5, RP_ROUGH_REFL = 6, RP_ROUGH_REFR = 7,
       RP_GI = 8, RP_MESHLIGHT = 9 };
// Russian roulette never ends a path that keeps hitting diffuse surfaces (the throughput
// it tests is renormalised to 1 at every bounce, raytracer.cpp:137-146), so the
// reference recursion is unbounded; the GPU keeps at most kMaxLevel nested ray-tree
// nodes (its per-thread frame stack) and so does this restatement.
const int kMaxLevel = 32;

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
const float kGrad[12][3] = {{1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1},
                            {1, 0, -1}, {-1, 0, -1}, {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1}};

struct Counters {
    uint64_t camera = 0, secondary = 0, shadow = 0, nodes = 0, tris = 0, spheres = 0, objects = 0;
    uint64_t snodes = 0, stris = 0;   // traversal work of shadow rays
    bool in_shadow = false;
    void node() { if (in_shadow) snodes++; else nodes++; }
    void tri() { if (in_shadow) stris++; else tris++; }
};

// ---------------- ray.hpp ----------------
struct HitInfo {
    bool hasHit = false;
    int matId = 0;                    // 0-based material index here
    float minT = INFINITY;
    Vec3f normal, hitPoint;
    float u = 0, v = 0;
    int obj = -1;
};
struct Ray {
    Vec3f origin, dir;
    HitInfo hitInfo;
    float refractiveIndexOfCurrentMedium = 1.0f;
    float motionBlurTime = 0.f;
    Vec3f throughput = V(1.0f, 1.0f, 1.0f);
    uint64_t key = 0;
    int level = 0;                    // ray-tree level (camera ray 0)
};

class Tracer {
public:
    Tracer(const rtg_scene_desc& d, const rtg_camera& c, Counters& k) : S(d), cam(c), cnt(k) {
        for (int i = 0; i < 512; ++i) perm[i] = kPerm256[i & 255];
    }

    // Test diagnostics (oracle_render_pixel): an environment lookup whose texel coordinate
    // (width * u or height * v, before the int truncation) lies within env_eps of a texel
    // boundary is "near"; the distinct near coordinates (axis, value) are numbered in order of
    // first use, and the lookups at a coordinate whose bit is set in env_flip take the texel on
    // the other side of the boundary -- what a last-ulp different atan2f / acosf result does on
    // the device (the same direction, e.g. every sample of a pixel whose camera ray misses,
    // gives the same result there).
    float env_eps = 0.0f;
    uint64_t env_flip = 0;
    std::vector<std::pair<int, float>> env_near;

    // Raytracer::PerPixel (raytracer.cpp:38-63)
    Vec3f PerPixel(int coordX, int coordY, uint64_t key) {
        Ray ray = GenerateRay(coordX, coordY, key);
        cnt.camera++;
        IntersectObjects(ray);
        if (ray.hitInfo.hasHit) {
            Vec3f eye = V(cam.position);
            return PerformShading(ray, eye, S.max_recursion_depth);
        } else if (S.bg_texture >= 0) {
            float u = coordX / (float)cam.width;
            float v = coordY / (float)cam.height;
            return TexRGB(S.textures[S.bg_texture], u, v);
        } else if (S.num_env_lights > 0) {
            return EnvSample(0, ray.dir);
        }
        return V((float)S.background[0], (float)S.background[1], (float)S.background[2]);
    }

private:
    const rtg_scene_desc& S;
    const rtg_camera& cam;
    Counters& cnt;
    int perm[512];

    // ---- camera.cpp:74-80 + raytracer.cpp:661-699
    Ray GenerateRay(int i, int j, uint64_t key) {
        Ray ray;
        float su = (i + 0.5) * (cam.right_ext - cam.left) / cam.width;
        float sv = (j + 0.5) * (cam.top - cam.bottom) / cam.height;
        Vec3f imagePlanePos = V(cam.q) + V(cam.right) * su + V(cam.up) * -sv;
        ray.origin = V(cam.position);
        if (cam.aperture > 0.0001) {
            Vec3f aps = ray.origin;
            float first01 = 2.0f * rnd(key, RP_DOF, 0) - 1.0f;
            aps = aps + V(cam.up) * (first01 * cam.aperture * 0.5f);
            float second01 = 2.0f * rnd(key, RP_DOF, 1) - 1.0f;
            aps = aps + V(cam.right) * (second01 * cam.aperture * 0.5f);
            Vec3f dir = makeUnit(ray.origin - imagePlanePos);
            float tFd = cam.focus_distance / dot(dir, V(cam.gaze));
            Vec3f bent = ray.origin + dir * tFd;
            ray.dir = makeUnit(bent - aps);
            ray.origin = aps;
        } else {
            ray.dir = makeUnit(imagePlanePos - ray.origin);
        }
        ray.hitInfo.hasHit = false;
        ray.hitInfo.minT = INFINITY;
        ray.refractiveIndexOfCurrentMedium = 1.0f;
        ray.motionBlurTime = rnd(key, RP_MOTION, 0);
        ray.key = key;
        return ray;
    }

    Ray GenerateSecondaryRay(const Ray& original, Vec3f newDir, Vec3f newOrigin, int slot) {   // raytracer.cpp:645-660
        Ray ray;
        ray.dir = newDir;
        ray.origin = newOrigin;
        ray.hitInfo.hasHit = false;
        ray.hitInfo.minT = INFINITY;
        ray.refractiveIndexOfCurrentMedium = original.refractiveIndexOfCurrentMedium;
        ray.motionBlurTime = original.motionBlurTime;
        ray.throughput = original.throughput;
        ray.key = child_key(original.key, slot);
        ray.level = original.level + 1;
        return ray;
    }

    // ---- shape.hpp:78-100
    static bool BoxHit(const float* mn, const float* mx, const Ray& ray) {
        float tx1 = (mn[0] - ray.origin.x) / ray.dir.x;
        float tx2 = (mx[0] - ray.origin.x) / ray.dir.x;
        float tmin = tx1, tmax = tx2;
        if (tx1 > tx2) { tmin = tx2; tmax = tx1; }
        float ty1 = (mn[1] - ray.origin.y) / ray.dir.y;
        float ty2 = (mx[1] - ray.origin.y) / ray.dir.y;
        tmin = std::fmax(tmin, std::fmin(ty1, ty2));
        tmax = std::fmin(tmax, std::fmax(ty1, ty2));
        float tz1 = (mn[2] - ray.origin.z) / ray.dir.z;
        float tz2 = (mx[2] - ray.origin.z) / ray.dir.z;
        tmin = std::fmax(tmin, std::fmin(tz1, tz2));
        tmax = std::fmin(tmax, std::fmax(tz1, tz2));
        return tmax > 0 && tmax >= tmin && tmin < ray.hitInfo.minT;
    }

    static float TiledUV(float x) {                                       // mesh.cpp:382-389
        if (x > 1.0001f) { x = x - std::floor(x); if (x < 0.0001) x = 1.0f; }
        return x;
    }

    // ---- mesh.cpp:201-372
    bool IntersectFace(Ray& ray, const rtg_mesh& M, int faceIdx, const rtg_object& ob) {
        const rtg_face& face = S.faces[M.face_offset + faceIdx];
        cnt.tri();
        Vec3f v0 = V(face.v0), v1 = V(face.v1), v2 = V(face.v2);
        float matrixA[3][3] = {{v0.x - v1.x, v0.x - v2.x, ray.dir.x},
                               {v0.y - v1.y, v0.y - v2.y, ray.dir.y},
                               {v0.z - v1.z, v0.z - v2.z, ray.dir.z}};
        float detA = determinant(matrixA);
        if (detA == 0) return false;
        float matrixBeta[3][3] = {{v0.x - ray.origin.x, v0.x - v2.x, ray.dir.x},
                                  {v0.y - ray.origin.y, v0.y - v2.y, ray.dir.y},
                                  {v0.z - ray.origin.z, v0.z - v2.z, ray.dir.z}};
        float beta = determinant(matrixBeta) / detA;
        if (beta < 0) return false;
        float matrixGama[3][3] = {{v0.x - v1.x, v0.x - ray.origin.x, ray.dir.x},
                                  {v0.y - v1.y, v0.y - ray.origin.y, ray.dir.y},
                                  {v0.z - v1.z, v0.z - ray.origin.z, ray.dir.z}};
        float gama = determinant(matrixGama) / detA;
        if (gama < 0 || gama + beta > 1) return false;
        float matrixT[3][3] = {{v0.x - v1.x, v0.x - v2.x, v0.x - ray.origin.x},
                               {v0.y - v1.y, v0.y - v2.y, v0.y - ray.origin.y},
                               {v0.z - v1.z, v0.z - v2.z, v0.z - ray.origin.z}};
        float t = determinant(matrixT) / detA;
        if (!(t > 0.0f && t < ray.hitInfo.minT)) return false;
        ray.hitInfo.minT = t;
        ray.hitInfo.hasHit = true;
        ray.hitInfo.normal = V(face.n);
        ray.hitInfo.hitPoint = ray.origin + ray.dir * ray.hitInfo.minT;
        if (M.has_uv) {
            float u = face.uv0[0] + beta * (face.uv1[0] - face.uv0[0]) + gama * (face.uv2[0] - face.uv0[0]);
            float v = face.uv0[1] + beta * (face.uv1[1] - face.uv0[1]) + gama * (face.uv2[1] - face.uv0[1]);
            u = TiledUV(u);
            v = TiledUV(v);
            ray.hitInfo.u = u;
            ray.hitInfo.v = v;
            // normal or bump map of the base mesh (mesh.cpp:263-358), then the base mesh's
            // inverse transpose; Mesh::Intersect / InstancedMesh::Intersect apply the
            // object's once more (mesh.cpp:179, instancedMesh.cpp:57)
            if (ob.tex_normal >= 0) {
                Vec3f sampledNormal = TexRGB(S.textures[ob.tex_normal], u, v);
                sampledNormal = sampledNormal / (127.5f) - V(1, 1, 1);
                sampledNormal = makeUnit(sampledNormal);
                Vec3f tan, bitan;
                TangentBitangentForTriangle(v0, v1, v2, face.uv0, face.uv1, face.uv2, tan, bitan);
                ray.hitInfo.normal = TransformedNormal(tan, bitan, V(face.n), sampledNormal);
                ray.hitInfo.normal = makeUnit(applyT(ob.base_inv_transpose, ray.hitInfo.normal, 0.0f));
            } else if (ob.tex_bump >= 0) {
                const rtg_texture& bm = S.textures[ob.tex_bump];
                Vec3f tan, bitan;
                TangentBitangentForTriangle(v0, v1, v2, face.uv0, face.uv1, face.uv2, tan, bitan);
                Vec3f N = V(face.n);
                if (bm.kind == RTG_TEX_PERLIN) {
                    Vec3f gradient;
                    float eps = 0.001;
                    const Vec3f& p = ray.hitInfo.hitPoint;
                    float bf = bm.bump_factor;
                    float hxyz = Perlin(bm, p.x, p.y, p.z) * bf;
                    gradient.x = (Perlin(bm, p.x + eps, p.y, p.z) * bf - hxyz) / eps;
                    gradient.y = (Perlin(bm, p.x, p.y + eps, p.z) * bf - hxyz) / eps;
                    gradient.z = (Perlin(bm, p.x, p.y, p.z + eps) * bf - hxyz) / eps;
                    Vec3f gParallel = N * dot(gradient, N);
                    Vec3f surfaceGradient = gradient - gParallel;
                    Vec3f newNormal = N - surfaceGradient;
                    ray.hitInfo.normal = makeUnit(newNormal);
                } else {
                    const rtg_image& im = S.images[bm.image];
                    float width = im.width, height = im.height;
                    int i = (int)(u * (width - 1));
                    int j = (int)(v * (height - 1));
                    int nextI = i + 1, nextJ = j + 1;
                    if (i == width - 1) nextI = i;
                    if (j == height - 1) nextJ = j;
                    Vec3f c = Texel(im, i, j);
                    float h_uv = (c.x + c.y + c.z) / 3.0f;                  // MakeGreyscale, mesh.cpp:195-197
                    c = Texel(im, nextI, j);
                    float hDeltaU = (c.x + c.y + c.z) / 3.0f;
                    c = Texel(im, i, nextJ);
                    float hDeltaV = (c.x + c.y + c.z) / 3.0f;
                    float bumpFactor = bm.bump_factor;
                    Vec3f q_u = tan + N * ((hDeltaU - h_uv) * bumpFactor);
                    Vec3f q_v = bitan + N * ((hDeltaV - h_uv) * bumpFactor);
                    Vec3f newNormal = cross(q_v, q_u);
                    ray.hitInfo.normal = makeUnit(newNormal);
                    if (newNormal.x * N.x <= 0 && newNormal.y * N.y <= 0 && newNormal.z * N.z <= 0)
                        ray.hitInfo.normal = ray.hitInfo.normal * -1;
                    else if (std::abs(newNormal.y - N.y) > 0.9f || std::abs(newNormal.x - N.x) > 0.9f ||
                             std::abs(newNormal.z - N.z) > 0.9f)
                        ray.hitInfo.normal = ray.hitInfo.normal * -1;
                }
                ray.hitInfo.normal = makeUnit(applyT(ob.base_inv_transpose, ray.hitInfo.normal, 0.0f));
            }
        } else {
            // base mesh's own inverse transpose (for instances: the base mesh's)
            ray.hitInfo.normal = makeUnit(applyT(ob.base_inv_transpose, ray.hitInfo.normal, 0.0f));
        }
        return true;
    }

    // ---- mesh.cpp:390-422
    static void TangentBitangentForTriangle(Vec3f vert0, Vec3f vert1, Vec3f vert2, const float* v0_uv,
                                            const float* v1_uv, const float* v2_uv, Vec3f& tan, Vec3f& bitan) {
        Vec3f e1 = makeUnit(vert1 - vert0);
        Vec3f e2 = makeUnit(vert2 - vert1);
        float v0u = TiledUV(v0_uv[0]), v0v = TiledUV(v0_uv[1]);
        float v1u = TiledUV(v1_uv[0]), v1v = TiledUV(v1_uv[1]);
        float v2u = TiledUV(v2_uv[0]), v2v = TiledUV(v2_uv[1]);
        float u1 = v1u - v0u, v1 = v1v - v0v;
        float u2 = v2u - v1u, v2 = v2v - v1v;
        float det = 1.0f / (u1 * v2 - v1 * u2);
        tan.x = det * (v2 * e1.x - v1 * e2.x);
        tan.y = det * (v2 * e1.y - v1 * e2.y);
        tan.z = det * (v2 * e1.z - v1 * e2.z);
        bitan.x = -det * u2 * e1.x + det * u1 * e2.x;
        bitan.y = -det * u2 * e1.y + det * u1 * e2.y;
        bitan.z = -det * u2 * e1.z + det * u1 * e2.z;
        tan = makeUnit(tan);
        bitan = makeUnit(bitan);
    }
    // ---- helperMath.cpp:86-109: TBN (double Matrix) x sampled normal
    static Vec3f TransformedNormal(Vec3f tan, Vec3f bitan, Vec3f normal, Vec3f s) {
        const double m[3][3] = {{tan.x, bitan.x, normal.x}, {tan.y, bitan.y, normal.y}, {tan.z, bitan.z, normal.z}};
        const double vec[3] = {s.x, s.y, s.z};
        double r[3];
        for (int i = 0; i < 3; ++i) {
            r[i] = 0.0f;
            for (int k = 0; k < 3; ++k) r[i] += m[i][k] * vec[k];
        }
        return makeUnit(V((float)r[0], (float)r[1], (float)r[2]));
    }
    // ---- sphere.cpp:181-193
    static void TangentBitangentAroundPoint(Vec3f p, float radius, float phi, float theta, Vec3f& tan, Vec3f& bitan) {
        tan.x = 2 * M_PI * p.z;
        tan.y = 0;
        tan.z = -2 * M_PI * p.x;
        bitan.x = M_PI * p.y * std::cos(phi);
        bitan.y = -radius * M_PI * std::sin(theta);
        bitan.z = M_PI * p.y * std::sin(phi);
        tan = makeUnit(tan);
        bitan = makeUnit(bitan);
    }

    // ---- bvh.cpp:5-30
    // count_root=false: the root box was just tested as the mesh bbox (mesh.cpp:172 tests
    // this->bbox, which equals bvh[0].bbox) -- counted once, as the GPU walk does
    bool IntersectBVH(int node, Ray& ray, const rtg_mesh& M, const rtg_object& ob, bool count_root = true) {
        const rtg_bvh_node& n = S.nodes[M.node_offset + node];
        if (count_root) cnt.node();
        if (!BoxHit(n.bmin, n.bmax, ray)) return false;
        bool hasHit = false;
        if (n.left < 0 && n.count > 0) {
            for (int i = n.first; i < n.first + n.count; i++)
                if (IntersectFace(ray, M, i, ob)) hasHit = true;
        } else {
            bool hitLeft = IntersectBVH(n.left, ray, M, ob);
            bool hitRight = IntersectBVH(n.left + 1, ray, M, ob);
            if (hitLeft || hitRight) hasHit = true;
        }
        return hasHit;
    }

    // ---- mesh.cpp:158-188
    bool MeshIntersect(Ray& ray, const rtg_object& ob, int objIdx) {
        cnt.objects++;
        const rtg_mesh& M = S.meshes[ob.mesh];
        Vec3f oc = ray.origin, dc = ray.dir;
        ray.origin = applyT(ob.inv_transform, ray.origin, 1.0f);
        ray.dir = applyT(ob.inv_transform, ray.dir, 0.0f);
        if (ob.flags & RTG_OBJF_MOTION_BLUR) ray.origin = ray.origin + V(ob.motion_blur) * ray.motionBlurTime;
        cnt.node();
        if (BoxHit(ob.bbox_min, ob.bbox_max, ray)) {
            bool hasHit = IntersectBVH(0, ray, M, ob, false);
            ray.origin = oc;
            ray.dir = dc;
            if (hasHit) {
                ray.hitInfo.hitPoint = ray.origin + ray.dir * ray.hitInfo.minT;
                ray.hitInfo.normal = makeUnit(applyT(ob.inv_transpose, ray.hitInfo.normal, 0.0f));
                ray.hitInfo.matId = ob.material;
                ray.hitInfo.obj = objIdx;
            }
            return hasHit;
        }
        ray.origin = oc;
        ray.dir = dc;
        return false;
    }

    // ---- instancedMesh.cpp:16-66
    bool InstanceIntersect(Ray& ray, const rtg_object& ob, int objIdx) {
        cnt.objects++;
        bool hasHit = false;
        Vec3f oc = ray.origin, dc = ray.dir;
        if (ob.flags & RTG_OBJF_MOTION_BLUR) ray.origin = ray.origin + V(ob.motion_blur) * ray.motionBlurTime;
        if (BoxHit(ob.bbox_min, ob.bbox_max, ray)) {
            ray.origin = oc;
            ray.origin = applyT(ob.inv_transform, ray.origin, 1.0f);
            ray.dir = applyT(ob.inv_transform, ray.dir, 0.0f);
            if (ob.flags & RTG_OBJF_MOTION_BLUR) ray.origin = ray.origin + V(ob.motion_blur) * ray.motionBlurTime;
            hasHit = IntersectBVH(0, ray, S.meshes[ob.mesh], ob);
            if (hasHit) {
                ray.hitInfo.hitPoint = oc + dc * ray.hitInfo.minT;
                ray.hitInfo.matId = ob.material;
                ray.hitInfo.obj = objIdx;
                ray.hitInfo.normal = makeUnit(applyT(ob.inv_transpose, ray.hitInfo.normal, 0.0f));
            }
            ray.origin = oc;
            ray.dir = dc;
        }
        // when the bbox test fails the motion-blur offset stays on the ray (reference behaviour)
        return hasHit;
    }

    // ---- sphere.cpp:13-180 (a sphere normal map leaves the normal unset in the reference: rejected)
    bool SphereIntersect(Ray& r, const rtg_object& ob, int objIdx) {
        cnt.spheres++;
        cnt.objects++;
        Vec3f center = V(ob.center);
        float radius = ob.radius;
        Vec3f oc0 = r.origin, dc0 = r.dir;
        r.origin = applyT(ob.inv_transform, r.origin, 1.0f);
        r.dir = applyT(ob.inv_transform, r.dir, 0.0f);
        if (ob.flags & RTG_OBJF_MOTION_BLUR) r.origin = r.origin + V(ob.motion_blur) * r.motionBlurTime;
        Vec3f oc = r.origin - center;
        float t;
        float c = dot(oc, oc) - (radius * radius);
        float b = 2 * dot(r.dir, oc);
        float a = dot(r.dir, r.dir);
        float delta = b * b - (4 * a * c);
        if (delta < 0.0f) { r.origin = oc0; r.dir = dc0; return false; }
        delta = sqrtf(delta);
        a = 2.0 * a;
        float t1 = (-b + delta) / a;
        float t2 = (-b - delta) / a;
        t = t1 < t2 ? t1 : t2;
        if (t1 < t2) { if (t1 > 0.0f) t = t1; else t = t2; }
        else if (t2 < t1) { if (t2 > 0.0f) t = t2; else t = t1; }
        Vec3f localhitPoint = r.origin + r.dir * t;
        r.origin = oc0;
        r.dir = dc0;
        if (t < r.hitInfo.minT && t > 0.0f) {
            r.hitInfo.minT = t;
            r.hitInfo.matId = ob.material;
            r.hitInfo.obj = objIdx;
            r.hitInfo.hasHit = true;
            r.hitInfo.hitPoint = r.origin + r.dir * t;
            Vec3f p = localhitPoint - center;
            float phi = std::atan2(p.z, p.x);
            float theta = std::acos(p.y / radius);
            float u = (-phi + M_PI) / (2.0f * M_PI);
            float v = theta / M_PI;
            r.hitInfo.u = u;
            r.hitInfo.v = v;
            if (ob.tex_bump >= 0) {                                         // sphere.cpp:116-170
                const rtg_texture& bm = S.textures[ob.tex_bump];
                Vec3f tan, bitan;
                TangentBitangentAroundPoint(p, radius, phi, theta, tan, bitan);
                Vec3f N = makeUnit(cross(bitan, tan));
                if (bm.kind == RTG_TEX_PERLIN) {
                    Vec3f gradient;
                    float eps = 0.001;
                    float hxyz = Perlin(bm, p.x, p.y, p.z);
                    gradient.x = (Perlin(bm, p.x + eps, p.y, p.z) - hxyz) / eps;
                    gradient.y = (Perlin(bm, p.x, p.y + eps, p.z) - hxyz) / eps;
                    gradient.z = (Perlin(bm, p.x, p.y, p.z + eps) - hxyz) / eps;
                    Vec3f gParallel = N * dot(gradient, N);
                    Vec3f surfaceGradient = gradient - gParallel;
                    Vec3f newNormal = N - surfaceGradient;
                    r.hitInfo.normal = makeUnit(newNormal);
                } else {
                    const rtg_image& im = S.images[bm.image];
                    float width = im.width, height = im.height;
                    int i = (int)(u * width);
                    int j = (int)(v * height);
                    float normalizer = bm.normalizer;
                    float bumpFactor = bm.bump_factor;
                    Vec3f c = Texel(im, i + 1, j) / normalizer;
                    float h1 = (c.x + c.y + c.z) * bumpFactor;                // MakeGreyscale, sphere.cpp:9-11
                    c = Texel(im, i, j) / normalizer;
                    float h_uv = (c.x + c.y + c.z) * bumpFactor;
                    c = Texel(im, i, j + 1) / normalizer;
                    float h2 = (c.x + c.y + c.z) * bumpFactor;
                    Vec3f q_u = tan + N * (h1 - h_uv);
                    Vec3f q_v = bitan + N * (h2 - h_uv);
                    Vec3f newNormal = cross(q_v, q_u);
                    r.hitInfo.normal = makeUnit(newNormal);
                }
            } else {
                r.hitInfo.normal = makeUnit(localhitPoint - center);
            }
            r.hitInfo.normal = makeUnit(applyT(ob.inv_transpose, r.hitInfo.normal, 0.0f));
            return true;
        }
        return false;
    }

    bool ObjectIntersect(Ray& ray, int k) {
        const rtg_object& ob = S.objects[k];
        if (ob.kind == RTG_OBJ_SPHERE) return SphereIntersect(ray, ob, k);
        if (ob.kind == RTG_OBJ_INSTANCE) return InstanceIntersect(ray, ob, k);
        return MeshIntersect(ray, ob, k);
    }

    void IntersectObjects(Ray& ray) {                                      // raytracer.cpp:625-643
        for (int i = 0; i < S.num_objects; i++) ObjectIntersect(ray, i);
    }

    bool CastShadowRay(Ray& shadowRay, float lightSourceT) {              // raytracer.cpp:585-623
        cnt.shadow++;
        cnt.in_shadow = true;
        bool r = false;
        for (int i = 0; i < S.num_objects; i++) {
            const rtg_object& ob = S.objects[i];
            if (ob.kind != RTG_OBJ_SPHERE && (ob.flags & RTG_OBJF_SHADOW_SKIP)) continue;
            ObjectIntersect(shadowRay, i);
            if (shadowRay.hitInfo.hasHit && shadowRay.hitInfo.minT < lightSourceT) { r = true; break; }
        }
        cnt.in_shadow = false;
        return r;
    }

    bool IsInShadow(Ray& originalRay, Vec3f lightPos) {                   // raytracer.cpp:567-584
        Ray shadowRay;
        shadowRay.dir = lightPos - originalRay.hitInfo.hitPoint;
        float lightSourceT = len(shadowRay.dir);
        shadowRay.dir = shadowRay.dir / lightSourceT;
        shadowRay.origin = originalRay.hitInfo.hitPoint + originalRay.hitInfo.normal * S.shadow_epsilon;
        shadowRay.hitInfo.hasHit = false;
        shadowRay.hitInfo.minT = lightSourceT + 0.01f;
        shadowRay.motionBlurTime = originalRay.motionBlurTime;
        return CastShadowRay(shadowRay, lightSourceT);
    }

    bool IsInShadowDirectional(Ray& originalRay, Vec3f lightDir) {        // raytracer.cpp:555-566
        Ray shadowRay;
        shadowRay.dir = -lightDir;
        shadowRay.origin = originalRay.hitInfo.hitPoint + originalRay.hitInfo.normal * S.shadow_epsilon;
        shadowRay.hitInfo.hasHit = false;
        shadowRay.hitInfo.minT = INFINITY;
        shadowRay.motionBlurTime = originalRay.motionBlurTime;
        return CastShadowRay(shadowRay, INFINITY);
    }

    // ---- textures
    Vec3f Texel(const rtg_image& im, int i, int j) {                       // LDRImage.h:16-26
        long long idx = (long long)im.channels * ((long long)i + (long long)j * im.width);
        long long n = (long long)im.width * im.height * im.channels;
        auto at = [&](long long k) { return (k >= 0 && k < n) ? im.texels[k] : 0.0f; };
        return V(at(idx), at(idx + 1), at(idx + 2));
    }
    Vec3f ImageRGB(const rtg_texture& tx, float u, float v) {               // imageTexture.h:60-73,111-133
        const rtg_image& im = S.images[tx.image];
        if (tx.nearest) {
            int i = (int)(u * im.width), j = (int)(v * im.height);
            i = smin(im.width - 1, i);
            j = smin(im.height - 1, j);
            return Texel(im, i, j);
        }
        float i = smax(0.0f, smin(u * im.width, (float)(im.width - 1)));
        float j = smax(0.0f, smin(v * im.height, (float)(im.height - 1)));
        float p = std::floor(i), q = std::floor(j);
        float dx = i - p, dy = j - q;
        float w1 = (1 - dx) * (1 - dy), w2 = dx * (1 - dy), w3 = (1 - dx) * dy, w4 = dx * dy;
        return Texel(im, p, q) * w1 + Texel(im, p + 1, q) * w2 + Texel(im, p, q + 1) * w3 + Texel(im, p + 1, q + 1) * w4;
    }
    static double PerlinF(float x) {
        x = std::abs(x);
        if (x > 1) return 0;
        float xSqr = x * x;
        float xCube = xSqr * x;
        return (-6 * xCube * xSqr) + 15 * xCube * x - 10 * xCube + 1;
    }
    static float GDot(int g, float x, float y, float z) { return kGrad[g][0] * x + kGrad[g][1] * y + kGrad[g][2] * z; }
    float Perlin(const rtg_texture& tx, float x, float y, float z) {      // perlinTexture.h:57-123
        x *= tx.noise_scale; y *= tx.noise_scale; z *= tx.noise_scale;
        int X = std::floor(x), Y = std::floor(y), Z = std::floor(z);
        float dx = x - X, dy = y - Y, dz = z - Z;
        X = X & 255; Y = Y & 255; Z = Z & 255;
        const int* p = perm;
        int i0 = p[X + p[Y + p[Z]]] % 12, i1 = p[X + p[Y + p[Z + 1]]] % 12;
        int i2 = p[X + p[Y + 1 + p[Z]]] % 12, i3 = p[X + p[Y + 1 + p[Z + 1]]] % 12;
        int i4 = p[X + 1 + p[Y + p[Z]]] % 12, i5 = p[X + 1 + p[Y + p[Z + 1]]] % 12;
        int i6 = p[X + 1 + p[Y + 1 + p[Z]]] % 12, i7 = p[X + 1 + p[Y + 1 + p[Z + 1]]] % 12;
        double c0 = GDot(i0, dx, dy, dz), c1 = GDot(i4, dx - 1, dy, dz), c2 = GDot(i2, dx, dy - 1, dz);
        double c3 = GDot(i6, dx - 1, dy - 1, dz), c4 = GDot(i1, dx, dy, dz - 1), c5 = GDot(i5, dx - 1, dy, dz - 1);
        double c6 = GDot(i3, dx, dy - 1, dz - 1), c7 = GDot(i7, dx - 1, dy - 1, dz - 1);
        double fdx = PerlinF(dx), fdy = PerlinF(dy), fdz = PerlinF(dz);
        double fdx1 = PerlinF(dx - 1), fdy1 = PerlinF(dy - 1), fdz1 = PerlinF(dz - 1);
        double w0 = fdx * fdy * fdz, w1 = fdx1 * fdy * fdz, w2 = fdx * fdy1 * fdz, w3 = fdx1 * fdy1 * fdz;
        double w4 = fdx * fdy * fdz1, w5 = fdx1 * fdy * fdz1, w6 = fdx * fdy1 * fdz1, w7 = fdx1 * fdy1 * fdz1;
        double total = w0 * c0 + w1 * c1 + w2 * c2 + w3 * c3 + w4 * c4 + w5 * c5 + w6 * c6 + w7 * c7;
        if (!tx.noise_abs) return (total + 1) / 2.0f;
        return std::abs(total);
    }
    Vec3f TexRGB(const rtg_texture& tx, float u, float v) {
        if (tx.kind == RTG_TEX_PERLIN) return V(180, 30, 180);
        return ImageRGB(tx, u, v);
    }

    Vec3f EnvSample(int e, Vec3f dir) {                                     // sphericalEnvironmentLight.h:22-34
        const rtg_image& im = S.images[S.env_lights[e].image];
        float u = (1 + (std::atan2(dir.x, -dir.z) / M_PI)) / 2.0f;
        float v = std::acos(dir.y) / M_PI;
        int i = im.width * u;
        int j = im.height * v;
        if (env_eps > 0.0f) {
            auto flip = [&](int axis, float c, int& k) {
                const float fr = c - std::floor(c);
                if (fr < env_eps || fr > 1.0f - env_eps) {
                    size_t id = 0;
                    while (id < env_near.size() && env_near[id] != std::make_pair(axis, c)) ++id;
                    if (id == env_near.size()) env_near.push_back({axis, c});
                    if (id < 64 && ((env_flip >> id) & 1)) k += fr < 0.5f ? -1 : 1;
                }
            };
            flip(0, im.width * u, i);
            flip(1, im.height * v, j);
        }
        return Texel(im, i, j) * 2 * M_PI;
    }
    Vec3f EnvDirection(Vec3f surfaceNormal, uint64_t key, int e) {         // sphericalEnvironmentLight.h:36-61
        Vec3f n = makeUnit(surfaceNormal);
        Vec3f candidate;
        for (uint32_t k = 0; k < 4096; ++k) {
            uint32_t base = (uint32_t)e * 16384u + 3u * k;
            candidate.x = 2.0f * rnd(key, RP_ENV, base) - 1.0f;
            candidate.y = 2.0f * rnd(key, RP_ENV, base + 1) - 1.0f;
            candidate.z = 2.0f * rnd(key, RP_ENV, base + 2) - 1.0f;
            float length = len(candidate);
            if (length <= 1.0f && dot(n, candidate) > 0.0f) break;
        }
        return candidate;
    }

    Vec3f DiffuseCoeff(const Ray& ray, const rtg_object& ob, const rtg_material& mat) {   // raytracer.cpp:478-508
        Vec3f reflectance = V(mat.diffuse);
        if (ob.tex_diffuse >= 0) {
            const rtg_texture& tx = S.textures[ob.tex_diffuse];
            Vec3f textureKd;
            if (tx.kind == RTG_TEX_PERLIN) {
                Vec3f hp = ray.hitInfo.hitPoint;
                float s = Perlin(tx, hp.x, hp.y, hp.z);
                textureKd = V(s, s, s);
            } else {
                textureKd = ImageRGB(tx, ray.hitInfo.u, ray.hitInfo.v) / 255.0f;
            }
            reflectance = tx.blend ? (textureKd + V(mat.diffuse)) / 2.0f : textureKd;
        }
        return reflectance;
    }
    Vec3f SpecularCoeff(const Ray& ray, const rtg_object& ob, const rtg_material& mat) {  // raytracer.cpp:509-539
        Vec3f reflectance = V(mat.specular);
        if (ob.tex_specular >= 0 && ob.tex_diffuse >= 0) {
            const rtg_texture& tx = S.textures[ob.tex_diffuse];
            Vec3f textureKs;
            if (tx.kind == RTG_TEX_PERLIN) {
                Vec3f hp = ray.hitInfo.hitPoint;
                float s = Perlin(tx, hp.x, hp.y, hp.z);
                textureKs = V(s, s, s);
            } else {
                textureKs = ImageRGB(tx, ray.hitInfo.u, ray.hitInfo.v) / 255.0f;
            }
            reflectance = tx.blend ? (textureKs + V(mat.diffuse)) / 2.0f : textureKs;
        }
        return reflectance;
    }

    // ---- brdf*.cpp
    Vec3f BrdfApply(const rtg_brdf& B, const rtg_material& mat, Vec3f kd, Vec3f ks, Vec3f w_i, Vec3f w_o, Vec3f normal) {
        const float exponent = B.exponent;
        switch (B.type) {
            case RTG_BRDF_PHONG: {
                float angleTheta_i = angleBetweenUnitVectors(w_i, normal);
                if (angleTheta_i >= 90.0f || angleTheta_i < 0) return V(0, 0, 0);
                Vec3f r = makeUnit((normal * 2.0f * dot(normal, w_i)) - w_i);
                double angleR = angleBetweenUnitVectors(r, w_o);
                return kd + ks * (std::pow(cosDeg(angleR), exponent) / cosDeg(angleTheta_i));
            }
            case RTG_BRDF_BLINN_PHONG: {
                float angleTheta_i = angleBetweenUnitVectors(w_i, normal);
                if (angleTheta_i >= 90.0f) return V(0, 0, 0);
                Vec3f half = (w_i + w_o) / len(w_i + w_o);
                double a = angleBetweenUnitVectors(half, normal);
                return kd + ks * (std::pow(cosDeg(a), exponent) / cosDeg(angleTheta_i));
            }
            case RTG_BRDF_MODIFIED_PHONG: {
                float angleTheta_i = angleBetweenUnitVectors(w_i, normal);
                if (angleTheta_i >= 90.0f || angleTheta_i < 0) return V(0, 0, 0);
                Vec3f r = makeUnit((normal * 2.0f * dot(normal, w_i)) - w_i);
                double angleR = angleBetweenUnitVectors(r, w_o);
                if (B.energy_conserving) {
                    Vec3f kdTerm = kd * (1.0f / M_PI);
                    double ksCons = (exponent + 2) / (2 * M_PI);
                    double cosTerm = std::pow(cosDeg(angleR), exponent);
                    return kdTerm + ks * (ksCons * cosTerm);
                }
                return kd + ks * std::pow(cosDeg(angleR), exponent);
            }
            case RTG_BRDF_MODIFIED_BLINN_PHONG: {
                float angleTheta_i = angleBetweenUnitVectors(w_i, normal);
                if (angleTheta_i >= 90.0f) return V(0, 0, 0);
                Vec3f half = (w_i + w_o) / len(w_i + w_o);
                double a = angleBetweenUnitVectors(half, normal);
                if (B.energy_conserving) {
                    Vec3f kdTerm = kd * (1.0f / M_PI);
                    double ksCons = (exponent + 8) / (8 * M_PI);
                    double cosTerm = std::pow(cosDeg(a), exponent);
                    return kdTerm + ks * (ksCons * cosTerm);
                }
                return kd + ks * std::pow(cosDeg(a), exponent);
            }
            default: {
                float angleTheta_i = angleBetweenUnitVectors(w_i, normal);
                if (angleTheta_i >= 90.0f) return V(0, 0, 0);
                Vec3f half = (w_i + w_o) / len(w_i + w_o);
                double ex = exponent;
                double cosAlpha = dot(half, normal);
                double d = (ex + 2) * std::pow(cosAlpha, ex) / (2 * M_PI);
                double cosbeta = dot(half, w_o), n = mat.refractive_index;
                double r0 = std::pow(n - 1, 2) / std::pow(n + 1, 2);
                double f = r0 + (1.0 - r0) * std::pow((1.0 - cosbeta), 5.0);
                double ndoth = dot(normal, half), ndotwo = dot(normal, w_o), ndotwi = dot(normal, w_i);
                double wodoth = dot(w_o, half);
                double g = smin(1.0, smin(2.0f * ndoth * ndotwo / wodoth, 2.0 * ndoth * ndotwi / wodoth));
                double kdCoeff = (1.0f / M_PI);
                if (B.kd_fresnel) kdCoeff *= (1 - f);
                Vec3f kdTerm = kd * kdCoeff;
                double costheta = dot(normal, w_i), cosphi = dot(normal, w_o);
                Vec3f ksTerm = ks * ((d * f * g) / (4 * costheta * cosphi));
                return kdTerm + ksTerm;
            }
        }
    }

    // ---- raytracer.cpp:135-191 (GetNormalizedRandom draws -> counter RNG keyed by the node)
    Vec3f ComputeGlobalIllumination(Ray& ray, const rtg_material& orgMat, Vec3f& w_o, int recDepth, int& hitMeshLightId) {
        if (cam.russian_roulette) {
            float probTest = rnd(ray.key, RP_GI, 0);
            float maxThroughput = smax(ray.throughput.x, smax(ray.throughput.x, ray.throughput.z));
            if (probTest > maxThroughput && recDepth <= 0) return V(0, 0, 0);
            ray.throughput = ray.throughput / maxThroughput;
        } else if (recDepth <= 0) {
            return V(0, 0, 0);
        }
        if (ray.level >= kMaxLevel) return V(0, 0, 0);           // frame-stack bound (see kMaxLevel)
        float rand1 = rnd(ray.key, RP_GI, 1);
        float rand2 = rnd(ray.key, RP_GI, 2);
        float phi = 2 * M_PI * rand1;
        float theta = 0.0f;
        if (cam.importance_sampling) theta = std::asin(std::sqrt(rand2));
        else theta = std::acos(rand2);
        Vec3f u, v;
        GetOrthonormalBasis(ray.hitInfo.normal, u, v);
        Vec3f newDir = u * std::sin(theta) * std::cos(phi) + ray.hitInfo.normal * std::cos(theta) +
                       v * std::sin(theta) * std::sin(phi);
        newDir = makeUnit(newDir);
        Vec3f newOrigin = ray.hitInfo.hitPoint + ray.hitInfo.normal * 0.0001;
        Ray globalRay = GenerateSecondaryRay(ray, newDir, newOrigin, 2);
        cnt.secondary++;
        IntersectObjects(globalRay);
        Vec3f globalRaysColor = V(0, 0, 0);
        if (globalRay.hitInfo.hasHit) {
            const rtg_material& mat = S.materials[globalRay.hitInfo.matId];
            if (mat.type == RTG_MAT_EMISSIVE) hitMeshLightId = ShapeId(globalRay.hitInfo.obj);
            Vec3f transferredLight = PerformShading(globalRay, globalRay.origin, recDepth - 1);
            globalRaysColor = Shade(ray, orgMat, globalRay.dir, w_o, transferredLight) * 2.0f * M_PI;
        }
        return globalRaysColor;
    }
    // Shape::id of an object (spheres never get one in the reference: no light matches it)
    int ShapeId(int obj) const { return S.objects[obj].kind == RTG_OBJ_SPHERE ? INT32_MIN : S.objects[obj].id; }

    // ---- meshLight.h:27-47 (face drawn uniformly over the faceCount faces; the reference's
    // uniform_int_distribution(0, faceCount) also draws the out-of-range index faceCount)
    void MeshLightSample(int l, uint64_t key, Vec3f& pos, double& weight) {
        const rtg_mesh_light& L = S.mesh_lights[l];
        const rtg_object& ob = S.objects[L.object];
        const rtg_mesh& M = S.meshes[ob.mesh];
        int k = (int)(rndd(key, RP_MESHLIGHT, 3 * l) * M.face_count);
        if (k >= M.face_count) k = M.face_count - 1;
        const rtg_face& face = S.faces[M.face_offset + k];
        double selectionWeight = face.area / M.surface_area;
        double rand1 = rndd(key, RP_MESHLIGHT, 3 * l + 1);
        double rand2 = rndd(key, RP_MESHLIGHT, 3 * l + 2);
        Vec3f a = V(face.v0), b = V(face.v1), c = V(face.v2);
        Vec3f q = b * (1 - rand2) + c * rand2;
        pos = a * (1 - std::sqrt(rand1)) + q * std::sqrt(rand1);
        pos = applyT(ob.transform, pos, 1.0f);
        weight = selectionWeight;
    }

    Vec3f Shade(Ray& ray, const rtg_material& mat, Vec3f w_i, Vec3f w_o, Vec3f Li) {   // raytracer.cpp:192-206
        const rtg_object& ob = S.objects[ray.hitInfo.obj];
        if (mat.brdf >= 0) {
            float costheta_i = smax(0.0f, dot(w_i, ray.hitInfo.normal));
            Vec3f kd = DiffuseCoeff(ray, ob, mat);
            Vec3f ks = SpecularCoeff(ray, ob, mat);
            Vec3f res = BrdfApply(S.brdfs[mat.brdf], mat, kd, ks, w_i, w_o, ray.hitInfo.normal);
            ray.throughput = ray.throughput * res;
            return res * Li * costheta_i;
        }
        Vec3f kd = DiffuseCoeff(ray, ob, mat);
        float costheta = smax(0.0f, dot(w_i, ray.hitInfo.normal));
        Vec3f diffuse = kd * Li * costheta;
        Vec3f ks = SpecularCoeff(ray, ob, mat);
        Vec3f half = (w_i + w_o) / len(w_i + w_o);
        float cosAlpha = smax(0.0f, dot(ray.hitInfo.normal, half));
        Vec3f specular = ks * Li * std::pow(cosAlpha, mat.phong_exponent);
        return diffuse + specular;
    }

    Vec3f SampleDirectLighting(Ray& ray, const rtg_material& mat, Vec3f& w_o, int lightIDToSkip) {   // raytracer.cpp:701-805
        Vec3f color = V(0, 0, 0);
        for (int i = 0; i < S.num_point_lights; i++) {
            const rtg_point_light& light = S.point_lights[i];
            if (IsInShadow(ray, V(light.position))) continue;
            Vec3f w_i = makeUnit(V(light.position) - ray.hitInfo.hitPoint);
            float distToLight = len(V(light.position) - ray.hitInfo.hitPoint);
            Vec3f E = V(light.intensity) / (distToLight * distToLight);
            color = color + Shade(ray, mat, w_i, w_o, E);
        }
        for (int i = 0; i < S.num_area_lights; i++) {
            const rtg_area_light& L = S.area_lights[i];
            float offsetU = rnd(ray.key, RP_AREA, 2 * i) - 0.5f;
            float offsetV = rnd(ray.key, RP_AREA, 2 * i + 1) - 0.5f;
            Vec3f lightSamplePos = V(L.position) + (V(L.u) * (L.extent * offsetU)) + (V(L.v) * (L.extent * offsetV));
            if (IsInShadow(ray, lightSamplePos)) continue;
            Vec3f w_i = lightSamplePos - ray.hitInfo.hitPoint;
            float distToLight = len(w_i);
            float dSqr = distToLight * distToLight;
            w_i = w_i / distToLight;
            float lCostheta = dot(V(L.normal), -w_i);
            if (lCostheta < 0) lCostheta = dot(V(L.normal), w_i);
            Vec3f E = V(L.radiance) * (L.area * lCostheta / dSqr);
            color = color + Shade(ray, mat, w_i, w_o, E);
        }
        for (int i = 0; i < S.num_env_lights; i++) {
            Vec3f sampleDir = EnvDirection(ray.hitInfo.normal, ray.key, i);
            Vec3f E = EnvSample(i, sampleDir);
            Vec3f w_i = ray.hitInfo.normal;
            color = color + Shade(ray, mat, w_i, w_o, E);
        }
        for (int i = 0; i < S.num_dir_lights; i++) {
            const rtg_directional_light& L = S.dir_lights[i];
            if (IsInShadowDirectional(ray, V(L.dir))) continue;
            Vec3f w_i = -(V(L.dir));
            color = color + Shade(ray, mat, w_i, w_o, V(L.radiance));
        }
        for (int i = 0; i < S.num_spot_lights; i++) {
            const rtg_spot_light& L = S.spot_lights[i];
            if (IsInShadow(ray, V(L.position))) continue;
            Vec3f w_i = makeUnit(V(L.position) - ray.hitInfo.hitPoint);
            // SpotLight::GetIrradiance (spotLight.h:33-57)
            Vec3f point = ray.hitInfo.hitPoint;
            float distToPoint = len(point - V(L.position));
            Vec3f toPoint = (point - V(L.position)) / distToPoint;
            double alpha = angleBetweenUnitVectors(V(L.dir), toPoint);
            Vec3f E;
            if (alpha <= 0 || alpha > (L.coverage_deg / 2.0f)) {
                E = V(0, 0, 0);
            } else {
                float distSqr = distToPoint * distToPoint;
                E = V(L.intensity) / distSqr;
                if (alpha > (L.falloff_deg / 2.0f)) {
                    double cosAlpha = std::cos(alpha * DEG2RAD);
                    double s = std::pow((cosAlpha - L.cos_half_coverage) / (L.cos_half_falloff - L.cos_half_coverage), 4.0f);
                    E = E * (float)s;
                }
            }
            color = color + Shade(ray, mat, w_i, w_o, E);
        }
        for (int i = 0; i < S.num_mesh_lights; i++) {
            const rtg_mesh_light& L = S.mesh_lights[i];
            if (S.objects[L.object].id == lightIDToSkip) continue;
            Vec3f lightSamplePos;
            double weight;
            MeshLightSample(i, ray.key, lightSamplePos, weight);
            if (IsInShadow(ray, lightSamplePos)) continue;
            Vec3f w_i = lightSamplePos - ray.hitInfo.hitPoint;
            float distToLight = len(w_i);
            w_i = w_i / distToLight;
            Vec3f rad = V(L.radiance) * weight * 2 * M_PI;
            color = color + Shade(ray, mat, w_i, w_o, rad);
        }
        return color;
    }

    Vec3f Reflect(Vec3f normal, Vec3f w_o, float roughness, uint64_t key, uint32_t purpose) {   // raytracer.cpp:424-440
        Vec3f r = makeUnit((normal * 2.0f * dot(normal, w_o)) - w_o);
        if (roughness > 0.001) {
            Vec3f u, v;
            GetOrthonormalBasis(r, u, v);
            float psi1 = rnd(key, purpose, 0) - 0.5f;
            float psi2 = rnd(key, purpose, 1) - 0.5f;
            return makeUnit(r + (u * psi1 + v * psi2) * roughness);
        }
        return r;
    }

    static Vec3f BeersLaw(float x, Vec3f c, Vec3f L_0) {                  // raytracer.cpp:416-423
        Vec3f res;
        res.x = L_0.x * std::exp(-c.x * x);
        res.y = L_0.y * std::exp(-c.y * x);
        res.z = L_0.z * std::exp(-c.z * x);
        return res;
    }

    Vec3f EnvOrZero(Vec3f dir) { return S.num_env_lights > 0 ? EnvSample(0, dir) : V(0, 0, 0); }

    Vec3f ComputeMirrorReflection(Ray& originalRay, const rtg_material& mat, Vec3f& w_o, int recursionDepth) {
        if (recursionDepth <= 0) return V(0, 0, 0);
        Vec3f w_r = Reflect(originalRay.hitInfo.normal, w_o, mat.roughness, originalRay.key, RP_ROUGH_REFL);
        Vec3f origin = originalRay.hitInfo.hitPoint + originalRay.hitInfo.normal * S.shadow_epsilon;
        Ray reflectedRay = GenerateSecondaryRay(originalRay, w_r, origin, 0);
        reflectedRay.refractiveIndexOfCurrentMedium = 1.0f;
        cnt.secondary++;
        IntersectObjects(reflectedRay);
        if (reflectedRay.hitInfo.hasHit)
            return V(mat.mirror) * PerformShading(reflectedRay, reflectedRay.origin, recursionDepth - 1);
        if (S.num_env_lights > 0) return V(mat.mirror) * EnvSample(0, reflectedRay.dir);
        return V(0, 0, 0);
    }

    Vec3f ComputeConductorFresnelReflection(Ray& originalRay, const rtg_material& mat, Vec3f& w_o, int recDepth) {
        if (recDepth <= 0) return V(0, 0, 0);
        Vec3f d = -w_o;
        float cosTheta = -dot(d, originalRay.hitInfo.normal);
        float n2 = mat.refractive_index;
        float k2 = mat.absorption_index;
        float n2k2 = n2 * n2 + k2 * k2;
        float n2cosTheta2 = 2 * n2 * cosTheta;
        float cosThetaSqr = cosTheta * cosTheta;
        float rs = (n2k2 - n2cosTheta2 + cosThetaSqr) / (n2k2 + n2cosTheta2 + cosThetaSqr);
        float rp = (n2k2 * cosThetaSqr - n2cosTheta2 + 1) / (n2k2 * cosThetaSqr + n2cosTheta2 + 1);
        float reflectRatio = 0.5 * (rs + rp);
        if (reflectRatio > 0.0001) {
            Vec3f reflectedRaysColor;
            Vec3f w_reflected = Reflect(originalRay.hitInfo.normal, w_o, mat.roughness, originalRay.key, RP_ROUGH_REFL);
            Vec3f origin = originalRay.hitInfo.hitPoint + originalRay.hitInfo.normal * S.shadow_epsilon;
            Ray reflectedRay = GenerateSecondaryRay(originalRay, w_reflected, origin, 0);
            reflectedRay.refractiveIndexOfCurrentMedium = 1.0f;
            cnt.secondary++;
            IntersectObjects(reflectedRay);
            if (reflectedRay.hitInfo.hasHit)
                reflectedRaysColor = V(mat.mirror) * PerformShading(reflectedRay, reflectedRay.origin, recDepth - 1);
            else
                reflectedRaysColor = V(0, 0, 0);
            return reflectedRaysColor * reflectRatio;
        }
        return V(0, 0, 0);
    }

    Vec3f ComputeDielectric(Ray& originalRay, const rtg_material& mat, Vec3f& w_o, float n1, float n2, int recDepth) {
        if (recDepth <= 0) return V(0, 0, 0);
        Vec3f d = -w_o;
        Vec3f modifiedNormal = originalRay.hitInfo.normal;
        float cosTheta = -dot(d, modifiedNormal);
        bool isEntering = cosTheta > 0.f;
        float objN = n2;
        if (!isEntering) {
            n1 = n2;
            n2 = 1.0f;
            objN = 1.0f;
            cosTheta = std::fabs(cosTheta);
            modifiedNormal = -modifiedNormal;
        }
        float r = n1 / n2;
        float sinThetaSqr = 1 - (cosTheta * cosTheta);
        float criticalTerm = r * r * sinThetaSqr;
        if (criticalTerm > 1) {
            Vec3f w_r = Reflect(modifiedNormal, w_o, mat.roughness, originalRay.key, RP_ROUGH_REFL);
            Vec3f newOrigin = originalRay.hitInfo.hitPoint + modifiedNormal * S.shadow_epsilon;
            Ray reflectedRay = GenerateSecondaryRay(originalRay, w_r, newOrigin, 0);
            cnt.secondary++;
            IntersectObjects(reflectedRay);
            Vec3f reflectedRaysColor = V(0, 0, 0);
            if (reflectedRay.hitInfo.hasHit) {
                reflectedRaysColor = PerformShading(reflectedRay, reflectedRay.origin, recDepth - 1);
                if (reflectedRay.refractiveIndexOfCurrentMedium > 1.0001)
                    reflectedRaysColor = BeersLaw(reflectedRay.hitInfo.minT, V(mat.absorption), reflectedRaysColor);
            }
            return reflectedRaysColor;
        }
        float cosPhi = std::sqrt(1 - criticalTerm);
        float n2cosTheta = n2 * cosTheta;
        float n1cosPhi = n1 * cosPhi;
        float rparallel = (n2cosTheta - n1cosPhi) / (n2cosTheta + n1cosPhi);
        float rperp = (n1 * cosTheta - n2 * cosPhi) / (n1 * cosTheta + n2 * cosPhi);
        float rReflect = (rparallel * rparallel + rperp * rperp) / 2;
        float rRefract = 1 - rReflect;

        Vec3f w_reflected = Reflect(modifiedNormal, w_o, mat.roughness, originalRay.key, RP_ROUGH_REFL);
        Vec3f newOrigin = originalRay.hitInfo.hitPoint + modifiedNormal * S.shadow_epsilon;
        Ray reflectedRay = GenerateSecondaryRay(originalRay, w_reflected, newOrigin, 0);
        cnt.secondary++;
        IntersectObjects(reflectedRay);
        reflectedRay.refractiveIndexOfCurrentMedium = isEntering ? objN : 1.0f;
        Vec3f reflectedRaysColor = V(0, 0, 0);
        if (reflectedRay.hitInfo.hasHit) {
            reflectedRaysColor = PerformShading(reflectedRay, reflectedRay.origin, recDepth - 1);
            if (reflectedRay.refractiveIndexOfCurrentMedium > 1.00001f)
                reflectedRaysColor = BeersLaw(reflectedRay.hitInfo.minT, V(mat.absorption), reflectedRaysColor);
        } else {
            reflectedRaysColor = EnvOrZero(reflectedRay.dir);
        }

        Vec3f refractedRaysColor;
        {
            Vec3f w_refracted = (d + modifiedNormal * cosTheta) * r - modifiedNormal * cosPhi;
            if (mat.roughness > 0.001) {
                Vec3f u, v;
                GetOrthonormalBasis(w_refracted, u, v);
                float psi1 = rnd(originalRay.key, RP_ROUGH_REFR, 0) - 0.5f;
                float psi2 = rnd(originalRay.key, RP_ROUGH_REFR, 1) - 0.5f;
                w_refracted = makeUnit(w_refracted + (u * psi1 + v * psi2) * mat.roughness);
            } else {
                w_refracted = makeUnit(w_refracted);
            }
            Vec3f refrOrigin = originalRay.hitInfo.hitPoint + (-modifiedNormal) * S.shadow_epsilon;
            Ray refractedRay = GenerateSecondaryRay(originalRay, w_refracted, refrOrigin, 1);
            refractedRay.refractiveIndexOfCurrentMedium = isEntering ? objN : 1.0f;
            cnt.secondary++;
            IntersectObjects(refractedRay);
            refractedRaysColor = V(0, 0, 0);
            if (refractedRay.hitInfo.hasHit) {
                refractedRaysColor = PerformShading(refractedRay, refractedRay.origin, recDepth - 1);
                if (refractedRay.refractiveIndexOfCurrentMedium > 1.001f)
                    refractedRaysColor = BeersLaw(refractedRay.hitInfo.minT, V(mat.absorption), refractedRaysColor);
            } else {
                refractedRaysColor = EnvOrZero(reflectedRay.dir);
            }
        }
        return reflectedRaysColor * rReflect + refractedRaysColor * rRefract;
    }

    Vec3f PerformShading(Ray& ray, Vec3f eyePos, int recursionDepth) {   // raytracer.cpp:65-134
        ray.hitInfo.hitPoint = ray.origin + ray.dir * ray.hitInfo.minT;
        Vec3f color = V(0, 0, 0);
        const rtg_material& mat = S.materials[ray.hitInfo.matId];
        const rtg_object& ob = S.objects[ray.hitInfo.obj];
        Vec3f w_o = makeUnit(eyePos - ray.hitInfo.hitPoint);
        float refractiveIndexOfVacuum = 1.00001;
        bool travellingInsideAnObject = ray.refractiveIndexOfCurrentMedium > refractiveIndexOfVacuum;
        if (mat.type == RTG_MAT_EMISSIVE) return V(mat.radiance) * 2.0f * M_PI;
        if (ob.tex_replace_all >= 0) return TexRGB(S.textures[ob.tex_replace_all], ray.hitInfo.u, ray.hitInfo.v);
        int hitLightMeshId = -1;
        if (cam.path_tracing) color = color + ComputeGlobalIllumination(ray, mat, w_o, recursionDepth, hitLightMeshId);
        bool sampleDirectLight = !cam.path_tracing || cam.next_event;
        if (!travellingInsideAnObject && sampleDirectLight) {
            color = color + V(S.ambient_light) * V(mat.ambient);
            color = color + SampleDirectLighting(ray, mat, w_o, hitLightMeshId);
        }
        if (mat.type == RTG_MAT_MIRROR) {
            color = color + ComputeMirrorReflection(ray, mat, w_o, recursionDepth);
        } else if (mat.type == RTG_MAT_DIELECTRIC) {
            float n1 = ray.refractiveIndexOfCurrentMedium;
            color = color + ComputeDielectric(ray, mat, w_o, n1, mat.refractive_index, recursionDepth);
        } else if (mat.type == RTG_MAT_CONDUCTOR) {
            color = color + ComputeConductorFresnelReflection(ray, mat, w_o, recursionDepth);
        }
        return color;
    }
};

// Gaussian2D (gaussian.h:3-21), sigma = pixelWidth / 6
float GaussWeight(float x, float y) {
    float sigma = 1.0f / 6.0f;
    float sigmaSqr = sigma * sigma;
    float c1 = 1.0f / (2.0f * M_PI * sigmaSqr);
    float exponent = -0.5 * ((x * x + y * y) / sigmaSqr);
    return c1 * std::exp(exponent);
}

// x86 (int) conversion + clamp (helperMath.cpp:140-152); out-of-range/NaN -> INT_MIN
unsigned char Clamp8(float c) {
    int i = (c > -2147483904.0f && c < 2147483648.0f) ? (int)c : (int)0x80000000;
    return (unsigned char)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

// renderThreadMain's per-pixel sample loop (main.cpp:60-121): the colour at 1 spp, else the
// Gaussian-weighted mean of the samples; with `accum`, (sum w*c, sum w) goes there and false is
// returned.
bool PixelValue(Tracer& tr, int x, int y, int W, int spp, uint64_t seed, int sample_begin, int sample_count,
                float* accum, Vec3f& color) {
    const int pixel = x + y * W;
    const int nRows = std::sqrt(spp), nCols = nRows;
    if (spp <= 1 && !accum) {
        color = tr.PerPixel(x, y, root_key(seed, pixel, 0));
        return true;
    }
    Vec3f acc;
    float sumW = 0.0f;
    for (int s = sample_begin; s < sample_begin + sample_count; ++s) {
        uint64_t key = root_key(seed, pixel, s);
        float sx = 0.f, sy = 0.f;
        if (s < nRows * nCols) {
            int row = s / nCols, col = s % nCols;
            float psi1 = rnd(key, RP_JITTER, 0), psi2 = rnd(key, RP_JITTER, 1);
            sx = (col + psi1) / nCols;
            sy = (row + psi2) / nRows;
        }
        Vec3f c = tr.PerPixel(x, y, key);
        float gw = GaussWeight(sx - 0.5f, sy - 0.5f);
        acc.x += c.x * gw;
        acc.y += c.y * gw;
        acc.z += c.z * gw;
        sumW += gw;
    }
    if (accum) {
        float* a = accum + 4 * (size_t)pixel;
        a[0] = acc.x; a[1] = acc.y; a[2] = acc.z; a[3] = sumW;
        return false;
    }
    color = V(acc.x / sumW, acc.y / sumW, acc.z / sumW);
    return true;
}

}  // namespace

extern "C" {

// Test diagnostics: pixel (x, y) of camera `camera` as oracle_render computes it, with the
// environment-lookup flips of Tracer::env_eps / env_flip (tests/test_gpu_configs.py explains
// each pixel outside the parity bound by the texel flips of last-ulp atan2f / acosf results).
// n_near receives the number of lookups within env_eps of a texel boundary.
int oracle_render_pixel(const rtg_scene_desc* desc, int camera, int x, int y, uint64_t seed, float env_eps,
                        uint64_t env_flip, float* rgb, int32_t* n_near) {
    if (!desc || camera < 0 || camera >= desc->num_cameras || !rgb) return -1;
    const rtg_camera& cam = desc->cameras[camera];
    if (x < 0 || y < 0 || x >= cam.width || y >= cam.height) return -1;
    Counters cnt;
    Tracer tr(*desc, cam, cnt);
    tr.env_eps = env_eps;
    tr.env_flip = env_flip;
    Vec3f c;
    PixelValue(tr, x, y, cam.width, cam.spp < 1 ? 1 : cam.spp, seed, 0, cam.spp < 1 ? 1 : cam.spp, nullptr, c);
    rgb[0] = c.x; rgb[1] = c.y; rgb[2] = c.z;
    if (n_near) *n_near = (int32_t)tr.env_near.size();
    return 0;
}

// Renders camera `camera` rows [row_begin,row_end) (row_end<=0: all) into
// hdr (w*h*3 floats) / ldr (w*h*3 bytes); either may be NULL.  accum (w*h*4), if
// non-NULL, receives the per-pixel (sum w*c, sum w) of samples
// [sample_begin, sample_begin+sample_count) instead (sample_count<0: spp).
// `stats` (9 x uint64: camera, secondary, shadow, nodes, tris, spheres, objects, shadow
// nodes, shadow tris) may be NULL.
int oracle_render(const rtg_scene_desc* desc, int camera, int row_begin, int row_end, int sample_begin,
                  int sample_count, uint64_t seed, int threads, float* hdr, uint8_t* ldr, float* accum,
                  uint64_t* stats) {
    if (!desc || camera < 0 || camera >= desc->num_cameras) return -1;
    if (desc->num_faces > 0 && desc->num_nodes == 0) return -2;   // RTG_LOAD_DEVICE_BVH description: no BVH
    const rtg_camera& cam = desc->cameras[camera];
    const int W = cam.width, H = cam.height;
    const int spp = cam.spp < 1 ? 1 : cam.spp;
    if (row_end <= 0 || row_end > H) row_end = H;
    if (row_begin < 0) row_begin = 0;
    if (sample_begin < 0) sample_begin = 0;
    if (sample_count < 0) sample_count = spp;
    if (threads < 1) threads = 1;
    std::vector<Counters> counts(threads);
    auto work = [&](int t) {
        Tracer tr(*desc, cam, counts[t]);
        for (int y = row_begin + t; y < row_end; y += threads) {
            for (int x = 0; x < W; ++x) {
                const int pixel = x + y * W;
                Vec3f color;
                if (!PixelValue(tr, x, y, W, spp, seed, sample_begin, sample_count, accum, color)) continue;
                const size_t idx = 3 * (size_t)pixel;
                if (hdr) { hdr[idx] = color.x; hdr[idx + 1] = color.y; hdr[idx + 2] = color.z; }
                if (ldr) { ldr[idx] = Clamp8(color.x); ldr[idx + 1] = Clamp8(color.y); ldr[idx + 2] = Clamp8(color.z); }
            }
        }
    };
    if (threads == 1) work(0);
    else {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(work, t);
        for (auto& t : th) t.join();
    }
    if (stats) {
        std::memset(stats, 0, 9 * sizeof(uint64_t));
        for (auto& c : counts) {
            stats[0] += c.camera; stats[1] += c.secondary; stats[2] += c.shadow; stats[3] += c.nodes;
            stats[4] += c.tris; stats[5] += c.spheres; stats[6] += c.objects; stats[7] += c.snodes;
            stats[8] += c.stris;
        }
    }
    return 0;
}

// Tonemapper::Tonemap (tonemapper.h:28-60, photographic operator): the log-average
// luminance as one sequential double sum, the burn threshold from the sorted list of all
// channel values (float), and TonemapPixel's double math with its float round trips
// (Reinhard returns float, clip takes and returns float, gammaInv = 1.0f / gamma).
static float TmClip(float n, float lower, float upper) { return std::max(lower, std::min(n, upper)); }

int oracle_tonemap(const float* hdr, int width, int height, float key, float burn, float saturation, float gamma,
                   uint8_t* ldr) {
    if (!hdr || !ldr || width <= 0 || height <= 0) return 1;
    const float delta = 0.01f;
    const size_t n = (size_t)width * height;
    std::vector<float> sorted(3 * n);
    double logSum = 0.0f;
    for (size_t i = 0; i < n; i++) {
        double r = sorted[3 * i + 0] = hdr[3 * i + 0];
        double g = sorted[3 * i + 1] = hdr[3 * i + 1];
        double b = sorted[3 * i + 2] = hdr[3 * i + 2];
        double lum = 0.2126 * r + 0.7152 * g + 0.0722 * b;
        logSum += std::log(delta + lum);
    }
    long pixelCount = width * height;
    const double avg = std::exp(logSum / (double)pixelCount);
    std::sort(sorted.begin(), sorted.end());
    auto reinhard = [&](double Y) -> float {
        double Lxy = (key * Y) / avg;
        if (burn > 0.01) {
            float thresholdPerct = (100.0f - burn) / 100;
            int lastIdx = (int)sorted.size() - 1;
            int idx = std::min(lastIdx, (int)(thresholdPerct * lastIdx));
            double thr = sorted[idx];
            thr = thr * key / avg;
            double LwhiteSqr = thr * thr;
            return (Lxy * (1 + (Lxy / LwhiteSqr))) / (1.0f + Lxy);
        }
        return Lxy / (1 + Lxy);
    };
    for (size_t i = 0; i < n; i++) {
        double R = hdr[3 * i], G = hdr[3 * i + 1], B = hdr[3 * i + 2];
        double y_i = 0.2126 * R + 0.7152 * G + 0.0722 * B;
        double y_o = reinhard(y_i);
        double r_o = TmClip(y_o * std::pow((R / y_i), saturation), 0.0f, 1.0f);
        double g_o = TmClip(y_o * std::pow((G / y_i), saturation), 0.0f, 1.0f);
        double b_o = TmClip(y_o * std::pow((B / y_i), saturation), 0.0f, 1.0f);
        double gammaInv = 1.0f / gamma;
        int cx = std::floor(std::min(255.0, 255 * std::pow(r_o, gammaInv)));
        int cy = std::floor(std::min(255.0, 255 * std::pow(g_o, gammaInv)));
        int cz = std::floor(std::min(255.0, 255 * std::pow(b_o, gammaInv)));
        ldr[3 * i] = (uint8_t)cx;
        ldr[3 * i + 1] = (uint8_t)cy;
        ldr[3 * i + 2] = (uint8_t)cz;
    }
    return 0;
}

// Test / diagnostics helper: histogram of leaf sizes of the description's BVHs (hist[k] =
// leaves with k faces, k < n; larger leaves land in hist[n-1]); returns the largest leaf.
int oracle_leaf_hist(const rtg_scene_desc* d, int64_t* hist, int n) {
    int mx = 0;
    for (int64_t i = 0; i < d->num_nodes; ++i) {
        const rtg_bvh_node& b = d->nodes[i];
        if (b.left >= 0) continue;
        mx = std::max(mx, (int)b.count);
        if (hist && n > 0) ++hist[std::min(n - 1, (int)b.count)];
    }
    return mx;
}

// Test helper: image i of a parsed description (texels as the loader stored them, for the
// image-decoder parity tests).  info = {width, height, channels, is_hdr}; out may be null.
int oracle_image(const rtg_scene_desc* d, int i, int32_t* info, float* out) {
    if (!d || i < 0 || i >= d->num_images) return -1;
    const rtg_image& im = d->images[i];
    info[0] = im.width; info[1] = im.height; info[2] = im.channels; info[3] = im.is_hdr;
    if (out) std::memcpy(out, im.texels, sizeof(float) * (size_t)im.width * im.height * im.channels);
    return 0;
}

}  // extern "C"
