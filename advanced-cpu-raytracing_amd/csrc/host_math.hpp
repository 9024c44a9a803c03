// Host-side float/double helpers with the exact operation order of the reference's
// helperMath.cpp / matrix.hpp, used while building the flattened scene (face
// normals, centroids, bboxes, camera frames, transforms).  Compiled with
// -ffp-contract=off so no FMA contraction changes a rounding.
#pragma once

#include <cmath>

#include "rtgpu.h"

namespace rtg {

struct V3 {
    float x = 0.f, y = 0.f, z = 0.f;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : (i == 2 ? z : x)); }
};
// helperMath.cpp:5-52
inline V3 operator+(const V3& a, const V3& b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(const V3& a, const V3& b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(const V3& a, const V3& b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator*(const V3& a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
inline V3 operator/(const V3& a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
inline V3 operator-(const V3& a) { return V3(a.x * -1.0f, a.y * -1.0f, a.z * -1.0f); }
inline float dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(const V3& a, const V3& b) {
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float len(const V3& a) { return sqrtf((a.x * a.x) + (a.y * a.y) + (a.z * a.z)); }
inline V3 makeUnit(const V3& a) {
    float l = len(a);
    return V3(a.x / l, a.y / l, a.z / l);
}
// helperMath.cpp:59-85 (abs resolves to the float overload)
inline void orthonormalBasis(V3 r, V3& u, V3& v) {
    float ax = std::fabs(r.x), ay = std::fabs(r.y), az = std::fabs(r.z);
    V3 rp = r;
    if (ax < ay) {
        if (ax < az) rp.x = 1.0f; else rp.z = 1.0f;
    } else {
        if (ay < az) rp.y = 1.0f; else rp.z = 1.0f;
    }
    u = makeUnit(cross(rp, r));
    v = makeUnit(cross(r, u));
}
inline rtg_float3 to_f3(const V3& a) { rtg_float3 r = {a.x, a.y, a.z}; return r; }
inline V3 from_f3(const rtg_float3& a) { return V3(a.x, a.y, a.z); }

// matrix.hpp: 4x4 double matrices, row-major
struct M4 {
    double m[4][4];
    bool valid = true;   // false for the 0x0 Matrix left by an unsupported rotation axis
    static M4 zero() { M4 r; for (auto& row : r.m) for (double& x : row) x = 0.0; return r; }
    static M4 identity() { M4 r = zero(); for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0f; return r; }
    static M4 translation(double tx, double ty, double tz) {
        M4 t = identity(); t.m[0][3] = tx; t.m[1][3] = ty; t.m[2][3] = tz; return t;
    }
    static M4 scale(double sx, double sy, double sz) {
        M4 s = zero(); s.m[0][0] = sx; s.m[1][1] = sy; s.m[2][2] = sz; s.m[3][3] = 1.0f; return s;
    }
    static M4 rotX(double a) {
        M4 r = zero(); r.m[0][0] = r.m[3][3] = 1.0f; r.m[1][1] = r.m[2][2] = std::cos(a);
        r.m[1][2] = -std::sin(a); r.m[2][1] = std::sin(a); return r;
    }
    static M4 rotY(double a) {
        M4 r = zero(); r.m[0][0] = r.m[2][2] = std::cos(a); r.m[1][1] = r.m[3][3] = 1.0f;
        r.m[0][2] = std::sin(a); r.m[2][0] = -std::sin(a); return r;
    }
    static M4 rotZ(double a) {
        M4 r = zero(); r.m[0][0] = r.m[1][1] = std::cos(a); r.m[2][2] = r.m[3][3] = 1.0f;
        r.m[1][0] = std::sin(a); r.m[0][1] = -std::sin(a); return r;
    }
    M4 operator*(const M4& b) const {   // matrix.hpp:91-107 (sum starts at 0.0f)
        M4 r = zero();
        r.valid = valid && b.valid;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                r.m[i][j] = 0.0f;
                for (int k = 0; k < 4; ++k) r.m[i][j] += m[i][k] * b.m[k][j];
            }
        return r;
    }
    M4 transpose() const {
        M4 r = zero(); r.valid = valid;
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) r.m[j][i] = m[i][j];
        return r;
    }
    void to(double* out16) const { for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) out16[i * 4 + j] = m[i][j]; }
};

// matrix.hpp:56-81: double accumulation, result narrowed to float
inline V3 apply(const M4& t, V3 v, float w) {
    V3 r;
    r.x = (float)(t.m[0][0] * v.x + t.m[0][1] * v.y + t.m[0][2] * v.z + t.m[0][3] * w);
    r.y = (float)(t.m[1][0] * v.x + t.m[1][1] * v.y + t.m[1][2] * v.z + t.m[1][3] * w);
    r.z = (float)(t.m[2][0] * v.x + t.m[2][1] * v.y + t.m[2][2] * v.z + t.m[2][3] * w);
    return r;
}
inline V3 applyPoint(const M4& t, V3 p) { return apply(t, p, 1.0f); }
inline V3 applyVector(const M4& t, V3 v) { return apply(t, v, 0.0f); }

}  // namespace rtg
