// glm_subset.h — the slice of glm the Trident renderer API and its CPU-side frame preparation use,
// restated (the reference's glm submodule is not vendored in the snapshot). Column-major, float,
// glm's operation order (so matrices match what the reference computes on its CPU):
// mat4 * mat4, mat4 * vec4, translate / rotate / scale, radians, quat(euler), mat4_cast, conjugate,
// perspectiveRH_ZO / perspective(RH_NO), orthoRH_ZO / ortho(RH_NO), lookAt(RH), normalize, cross, dot.
#pragma once

#include <cmath>

namespace glm {

struct vec2 {
    float x = 0, y = 0;
    vec2() = default;
    constexpr vec2(float a, float b) : x(a), y(b) {}
    explicit constexpr vec2(float s) : x(s), y(s) {}
    float& operator[](int i) { return (&x)[i]; }
    const float& operator[](int i) const { return (&x)[i]; }
};

struct vec3 {
    float x = 0, y = 0, z = 0;
    vec3() = default;
    constexpr vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit constexpr vec3(float s) : x(s), y(s), z(s) {}
    float& operator[](int i) { return (&x)[i]; }
    const float& operator[](int i) const { return (&x)[i]; }
};

struct vec4 {
    float x = 0, y = 0, z = 0, w = 0;
    vec4() = default;
    constexpr vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    explicit constexpr vec4(float s) : x(s), y(s), z(s), w(s) {}
    constexpr vec4(const vec3& v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
    float& operator[](int i) { return (&x)[i]; }
    const float& operator[](int i) const { return (&x)[i]; }
};

struct ivec4 {
    int x = 0, y = 0, z = 0, w = 0;
    ivec4() = default;
    explicit constexpr ivec4(int s) : x(s), y(s), z(s), w(s) {}
    constexpr ivec4(int a, int b, int c, int d) : x(a), y(b), z(c), w(d) {}
};

struct uvec4 {
    unsigned x = 0, y = 0, z = 0, w = 0;
};

struct quat {
    float w = 1, x = 0, y = 0, z = 0;  // glm::qua storage order differs; fields are named
    quat() = default;
    constexpr quat(float w_, float x_, float y_, float z_) : w(w_), x(x_), y(y_), z(z_) {}
    explicit quat(const vec3& eulerRadians);
};

struct mat4 {
    vec4 c[4];  // columns
    mat4() = default;
    explicit mat4(float s) {
        c[0] = vec4(s, 0, 0, 0); c[1] = vec4(0, s, 0, 0); c[2] = vec4(0, 0, s, 0); c[3] = vec4(0, 0, 0, s);
    }
    vec4& operator[](int i) { return c[i]; }
    const vec4& operator[](int i) const { return c[i]; }
};

inline vec3 operator+(const vec3& a, const vec3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(const vec3& a, const vec3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator-(const vec3& a) { return {-a.x, -a.y, -a.z}; }
inline vec3 operator*(const vec3& a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, const vec3& a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator*(const vec3& a, const vec3& b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline vec4 operator*(const vec4& a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline vec4 operator+(const vec4& a, const vec4& b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline bool operator==(const vec3& a, const vec3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

inline float dot(const vec3& a, const vec3& b) {  // glm compute_dot: (x + y) + z
    const vec3 t = a * b;
    return (t.x + t.y) + t.z;
}
inline vec3 cross(const vec3& x, const vec3& y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline float inversesqrt(float x) { return 1.0f / std::sqrt(x); }
inline vec3 normalize(const vec3& v) { return v * inversesqrt(dot(v, v)); }
inline float length(const vec3& v) { return std::sqrt(dot(v, v)); }
inline float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
inline vec3 radians(const vec3& d) { return {radians(d.x), radians(d.y), radians(d.z)}; }
template <typename T>
inline T pi() { return static_cast<T>(3.14159265358979323846264338327950288); }
template <typename T>
inline T two_pi() { return static_cast<T>(6.28318530717958647692528676655900576); }
inline float clamp(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

inline vec4 operator*(const mat4& m, const vec4& v) {  // (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
    const vec4 add0 = m[0] * v.x + m[1] * v.y;
    const vec4 add1 = m[2] * v.z + m[3] * v.w;
    return add0 + add1;
}
inline mat4 operator*(const mat4& a, const mat4& b) {  // column j: ((A0*b0 + A1*b1) + A2*b2) + A3*b3
    mat4 r;
    for (int j = 0; j < 4; ++j) r[j] = ((a[0] * b[j].x + a[1] * b[j].y) + a[2] * b[j].z) + a[3] * b[j].w;
    return r;
}

inline mat4 translate(const mat4& m, const vec3& v) {
    mat4 r = m;
    r[3] = ((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3];
    return r;
}
inline mat4 rotate(const mat4& m, float angle, const vec3& v) {
    const float c = std::cos(angle), s = std::sin(angle);
    const vec3 axis = normalize(v);
    const vec3 temp = (1.0f - c) * axis;
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
    for (int j = 0; j < 3; ++j) r[j] = (m[0] * R[j][0] + m[1] * R[j][1]) + m[2] * R[j][2];
    r[3] = m[3];
    return r;
}
inline mat4 scale(const mat4& m, const vec3& v) {
    mat4 r = m;
    r[0] = m[0] * v.x;
    r[1] = m[1] * v.y;
    r[2] = m[2] * v.z;
    return r;
}

inline quat::quat(const vec3& e) {  // glm::qua(vec3 eulerAngle)
    const vec3 c{std::cos(e.x * 0.5f), std::cos(e.y * 0.5f), std::cos(e.z * 0.5f)};
    const vec3 s{std::sin(e.x * 0.5f), std::sin(e.y * 0.5f), std::sin(e.z * 0.5f)};
    w = c.x * c.y * c.z + s.x * s.y * s.z;
    x = s.x * c.y * c.z - c.x * s.y * s.z;
    y = c.x * s.y * c.z + s.x * c.y * s.z;
    z = c.x * c.y * s.z - s.x * s.y * c.z;
}
inline quat conjugate(const quat& q) { return {q.w, -q.x, -q.y, -q.z}; }
inline quat normalize(const quat& q) {
    const float len = std::sqrt((q.w * q.w + q.x * q.x) + (q.y * q.y + q.z * q.z));
    if (len <= 0.0f) return {1.0f, 0.0f, 0.0f, 0.0f};
    const float o = 1.0f / len;
    return {q.w * o, q.x * o, q.y * o, q.z * o};
}
inline vec3 operator*(const quat& q, const vec3& v) {
    const vec3 qv{q.x, q.y, q.z};
    const vec3 uv = cross(qv, v), uuv = cross(qv, uv);
    return v + ((uv * q.w) + uuv) * 2.0f;
}
inline vec3 rotate(const quat& q, const vec3& v) { return q * v; }
inline mat4 mat4_cast(const quat& q) {
    mat4 r(1.0f);
    const float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
    const float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
    const float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
    r[0].x = 1.0f - 2.0f * (qyy + qzz); r[0].y = 2.0f * (qxy + qwz); r[0].z = 2.0f * (qxz - qwy);
    r[1].x = 2.0f * (qxy - qwz); r[1].y = 1.0f - 2.0f * (qxx + qzz); r[1].z = 2.0f * (qyz + qwx);
    r[2].x = 2.0f * (qxz + qwy); r[2].y = 2.0f * (qyz - qwx); r[2].z = 1.0f - 2.0f * (qxx + qyy);
    return r;
}

inline mat4 perspectiveRH_ZO(float fovy, float aspect, float n, float f) {
    const float t = std::tan(fovy / 2.0f);
    mat4 r(0.0f);
    r[0].x = 1.0f / (aspect * t);
    r[1].y = 1.0f / t;
    r[2].z = f / (n - f);
    r[2].w = -1.0f;
    r[3].z = -(f * n) / (f - n);
    return r;
}
inline mat4 perspective(float fovy, float aspect, float n, float f) {  // RH_NO (default clip space)
    const float t = std::tan(fovy / 2.0f);
    mat4 r(0.0f);
    r[0].x = 1.0f / (aspect * t);
    r[1].y = 1.0f / t;
    r[2].z = -(f + n) / (f - n);
    r[2].w = -1.0f;
    r[3].z = -(2.0f * f * n) / (f - n);
    return r;
}
inline mat4 orthoRH_ZO(float l, float rr, float b, float t, float n, float f) {
    mat4 r(1.0f);
    r[0].x = 2.0f / (rr - l);
    r[1].y = 2.0f / (t - b);
    r[2].z = -1.0f / (f - n);
    r[3].x = -(rr + l) / (rr - l);
    r[3].y = -(t + b) / (t - b);
    r[3].z = -n / (f - n);
    return r;
}
inline mat4 ortho(float l, float rr, float b, float t, float n, float f) {  // RH_NO
    mat4 r(1.0f);
    r[0].x = 2.0f / (rr - l);
    r[1].y = 2.0f / (t - b);
    r[2].z = -2.0f / (f - n);
    r[3].x = -(rr + l) / (rr - l);
    r[3].y = -(t + b) / (t - b);
    r[3].z = -(f + n) / (f - n);
    return r;
}
inline mat4 lookAt(const vec3& eye, const vec3& center, const vec3& up) {  // RH
    const vec3 f = normalize(center - eye);
    const vec3 s = normalize(cross(f, up));
    const vec3 u = cross(s, f);
    mat4 r(1.0f);
    r[0].x = s.x; r[1].x = s.y; r[2].x = s.z;
    r[0].y = u.x; r[1].y = u.y; r[2].y = u.z;
    r[0].z = -f.x; r[1].z = -f.y; r[2].z = -f.z;
    r[3].x = -dot(s, eye);
    r[3].y = -dot(u, eye);
    r[3].z = dot(f, eye);
    return r;
}

}  // namespace glm
