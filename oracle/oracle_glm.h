// oracle_glm.h — TEST INFRASTRUCTURE (parity oracle). Not part of the product; only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Scalar restatement of the glm subset the reference's hot path uses. glm is an empty, un-vendored
// submodule in the reference (.gitmodules: Trident/vendor/glm -> ThatTanishqTak/glm.git, pinned
// commit unrecoverable offline), so each function below restates glm's published definition
// (glm 0.9.9/1.0 family, GLM_FORCE_* not defined anywhere in the reference — Core/Utilities.h:11),
// keeping glm's operation order so float results match what the reference computes on the CPU.
// Column-major: m[c][r].
#pragma once

#include <cmath>
#include <cstring>

namespace oracle {

struct vec2 { float x, y; };
struct vec3 { float x, y, z; };
struct vec4 { float x, y, z, w; };
struct quat { float w, x, y, z; };
struct mat4 { float m[4][4]; };  // m[column][row]
struct mat3 { float m[3][3]; };

inline mat4 mat4_identity() {
    mat4 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0f;
    return r;
}
inline mat4 mat4_zero() { mat4 r{}; return r; }

inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(vec3 a, vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }

// glm compute_dot: tmp = a*b; return (tmp.x + tmp.y) + tmp.z
inline float dot(vec3 a, vec3 b) {
    const float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return (tx + ty) + tz;
}
inline vec3 cross(vec3 x, vec3 y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
// glm::normalize: v * inversesqrt(dot(v, v)), inversesqrt(x) = 1 / sqrt(x)
inline vec3 normalize(vec3 v) {
    const float s = 1.0f / std::sqrt(dot(v, v));
    return v * s;
}
inline float length(vec3 v) { return std::sqrt(dot(v, v)); }

// glm::radians: degrees * static_cast<T>(0.01745329251994329576923690768489)
inline float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
inline vec3 radians(vec3 d) { return {radians(d.x), radians(d.y), radians(d.z)}; }

// glm operator*(mat4, vec4): (m0*v0 + m1*v1) + (m2*v2 + m3*v3), component-wise.
inline vec4 mul(const mat4& a, vec4 v) {
    vec4 r;
    float* rp = &r.x;
    for (int i = 0; i < 4; ++i) {
        const float add0 = a.m[0][i] * v.x + a.m[1][i] * v.y;
        const float add1 = a.m[2][i] * v.z + a.m[3][i] * v.w;
        rp[i] = add0 + add1;
    }
    return r;
}

// glm operator*(mat4, mat4): Result[j] = ((A0*B[j][0] + A1*B[j][1]) + A2*B[j][2]) + A3*B[j][3]
inline mat4 mul(const mat4& a, const mat4& b) {
    mat4 r;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            float s = a.m[0][i] * b.m[j][0];
            s = s + a.m[1][i] * b.m[j][1];
            s = s + a.m[2][i] * b.m[j][2];
            s = s + a.m[3][i] * b.m[j][3];
            r.m[j][i] = s;
        }
    return r;
}

// glm::translate(m, v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
inline mat4 translate(const mat4& m, vec3 v) {
    mat4 r = m;
    for (int i = 0; i < 4; ++i)
        r.m[3][i] = ((m.m[0][i] * v.x + m.m[1][i] * v.y) + m.m[2][i] * v.z) + m.m[3][i];
    return r;
}

// glm::rotate(m, angle, axis) (matrix_transform.inl)
inline mat4 rotate(const mat4& m, float angle, vec3 v) {
    const float c = std::cos(angle);
    const float s = std::sin(angle);
    const vec3 axis = normalize(v);
    const vec3 temp = axis * (1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = temp.x * axis.y + s * axis.z;
    R[0][2] = temp.x * axis.z - s * axis.y;
    R[1][0] = temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = temp.y * axis.z + s * axis.x;
    R[2][0] = temp.z * axis.x + s * axis.y;
    R[2][1] = temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    mat4 r;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 4; ++i)
            r.m[j][i] = (m.m[0][i] * R[j][0] + m.m[1][i] * R[j][1]) + m.m[2][i] * R[j][2];
    for (int i = 0; i < 4; ++i) r.m[3][i] = m.m[3][i];
    return r;
}

// glm::scale(m, v)
inline mat4 scale(const mat4& m, vec3 v) {
    mat4 r = m;
    for (int i = 0; i < 4; ++i) {
        r.m[0][i] = m.m[0][i] * v.x;
        r.m[1][i] = m.m[1][i] * v.y;
        r.m[2][i] = m.m[2][i] * v.z;
    }
    return r;
}

// glm::quat(vec3 eulerAngle) (type_quat.inl)
inline quat quat_from_euler(vec3 e) {
    const vec3 c{std::cos(e.x * 0.5f), std::cos(e.y * 0.5f), std::cos(e.z * 0.5f)};
    const vec3 s{std::sin(e.x * 0.5f), std::sin(e.y * 0.5f), std::sin(e.z * 0.5f)};
    quat q;
    q.w = c.x * c.y * c.z + s.x * s.y * s.z;
    q.x = s.x * c.y * c.z - c.x * s.y * s.z;
    q.y = c.x * s.y * c.z + s.x * c.y * s.z;
    q.z = c.x * c.y * s.z - s.x * s.y * c.z;
    return q;
}
inline quat conjugate(quat q) { return {q.w, -q.x, -q.y, -q.z}; }
// glm::normalize(quat); quat dot = (w*w + x*x) + (y*y + z*z)
inline quat normalize(quat q) {
    const float len = std::sqrt((q.w * q.w + q.x * q.x) + (q.y * q.y + q.z * q.z));
    if (len <= 0.0f) return {1.0f, 0.0f, 0.0f, 0.0f};
    const float inv = 1.0f / len;
    return {q.w * inv, q.x * inv, q.y * inv, q.z * inv};
}
// glm quat * vec3
inline vec3 rotate(quat q, vec3 v) {
    const vec3 qv{q.x, q.y, q.z};
    const vec3 uv = cross(qv, v);
    const vec3 uuv = cross(qv, uv);
    return v + ((uv * q.w) + uuv) * 2.0f;
}
// glm::mat3_cast / mat4_cast
inline mat4 mat4_cast(quat q) {
    mat4 r = mat4_identity();
    const float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
    const float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
    const float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
    r.m[0][0] = 1.0f - 2.0f * (qyy + qzz);
    r.m[0][1] = 2.0f * (qxy + qwz);
    r.m[0][2] = 2.0f * (qxz - qwy);
    r.m[1][0] = 2.0f * (qxy - qwz);
    r.m[1][1] = 1.0f - 2.0f * (qxx + qzz);
    r.m[1][2] = 2.0f * (qyz + qwx);
    r.m[2][0] = 2.0f * (qxz + qwy);
    r.m[2][1] = 2.0f * (qyz - qwx);
    r.m[2][2] = 1.0f - 2.0f * (qxx + qyy);
    return r;
}

// glm::perspectiveRH_ZO (ext/matrix_clip_space.inl)
inline mat4 perspectiveRH_ZO(float fovy, float aspect, float zNear, float zFar) {
    const float tanHalfFovy = std::tan(fovy / 2.0f);
    mat4 r = mat4_zero();
    r.m[0][0] = 1.0f / (aspect * tanHalfFovy);
    r.m[1][1] = 1.0f / (tanHalfFovy);
    r.m[2][2] = zFar / (zNear - zFar);
    r.m[2][3] = -1.0f;
    r.m[3][2] = -(zFar * zNear) / (zFar - zNear);
    return r;
}
// glm::perspectiveRH_NO == glm::perspective without GLM_FORCE_DEPTH_ZERO_TO_ONE
inline mat4 perspectiveRH_NO(float fovy, float aspect, float zNear, float zFar) {
    const float tanHalfFovy = std::tan(fovy / 2.0f);
    mat4 r = mat4_zero();
    r.m[0][0] = 1.0f / (aspect * tanHalfFovy);
    r.m[1][1] = 1.0f / (tanHalfFovy);
    r.m[2][2] = -(zFar + zNear) / (zFar - zNear);
    r.m[2][3] = -1.0f;
    r.m[3][2] = -(2.0f * zFar * zNear) / (zFar - zNear);
    return r;
}
// glm::orthoRH_ZO
inline mat4 orthoRH_ZO(float l, float rr, float b, float t, float n, float f) {
    mat4 r = mat4_identity();
    r.m[0][0] = 2.0f / (rr - l);
    r.m[1][1] = 2.0f / (t - b);
    r.m[2][2] = -1.0f / (f - n);
    r.m[3][0] = -(rr + l) / (rr - l);
    r.m[3][1] = -(t + b) / (t - b);
    r.m[3][2] = -n / (f - n);
    return r;
}
// glm::ortho == orthoRH_NO
inline mat4 orthoRH_NO(float l, float rr, float b, float t, float n, float f) {
    mat4 r = mat4_identity();
    r.m[0][0] = 2.0f / (rr - l);
    r.m[1][1] = 2.0f / (t - b);
    r.m[2][2] = -2.0f / (f - n);
    r.m[3][0] = -(rr + l) / (rr - l);
    r.m[3][1] = -(t + b) / (t - b);
    r.m[3][2] = -(f + n) / (f - n);
    return r;
}
// glm::lookAtRH
inline mat4 lookAtRH(vec3 eye, vec3 center, vec3 up) {
    const vec3 f = normalize(center - eye);
    const vec3 s = normalize(cross(f, up));
    const vec3 u = cross(s, f);
    mat4 r = mat4_identity();
    r.m[0][0] = s.x; r.m[1][0] = s.y; r.m[2][0] = s.z;
    r.m[0][1] = u.x; r.m[1][1] = u.y; r.m[2][1] = u.z;
    r.m[0][2] = -f.x; r.m[1][2] = -f.y; r.m[2][2] = -f.z;
    r.m[3][0] = -dot(s, eye);
    r.m[3][1] = -dot(u, eye);
    r.m[3][2] = dot(f, eye);
    return r;
}

}  // namespace oracle
