// tmpt_math.h -- bit-exact restatement of the reference's per-path arithmetic,
// usable from host C++ and gfx950 device code.
//
// Every function reproduces the rounding sequence of the reference built on
// GLM 0.9.9.5:
//   dot       = (x*x' + y*y') + z*z'        glm/detail/func_geometric.inl:52-53
//   cross     term order                    func_geometric.inl:74-77
//   normalize = v * (1 / sqrt(dot(v, v)))   func_geometric.inl:88, func_exponential.inl:138
//   min/max   ternaries                     func_common.inl:17-29, clamp :504-507
// The translation units that include this header are compiled with
// -ffp-contract=off (no FMA contraction), default correctly rounded f32
// division/sqrt and IEEE denormals: see toymeshpathtracer_amd/csrc/Makefile.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TMPT_HD __host__ __device__ __forceinline__

namespace tmpt {

constexpr float kPI = 3.1415926f;   // maths.h:14
constexpr float kMinT = 0.001f;     // main.cpp:30
constexpr float kMaxT = 1.0e7f;     // main.cpp:31
constexpr int kMaxDepth = 10;       // main.cpp:33
constexpr float kDetEps = 1e-5f;    // maths.cpp:339

struct f3 {
    float x, y, z;
};

TMPT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
TMPT_HD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
TMPT_HD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
TMPT_HD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
TMPT_HD f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
TMPT_HD f3 operator*(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
TMPT_HD f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
TMPT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
TMPT_HD f3 cross(f3 x, f3 y)
{
    return f3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
TMPT_HD f3 normalize(f3 v) { return v * (1.0f / sqrtf(dot(v, v))); }
TMPT_HD float length(f3 v) { return sqrtf(dot(v, v)); }
TMPT_HD float gmin(float x, float y) { return (y < x) ? y : x; }
TMPT_HD float gmax(float x, float y) { return (x < y) ? y : x; }
TMPT_HD f3 vmin(f3 a, f3 b) { return f3{gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)}; }
TMPT_HD f3 vmax(f3 a, f3 b) { return f3{gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)}; }
TMPT_HD float saturate(float v) { return gmin(gmax(v, 0.0f), 1.0f); }  // maths.h:16-19

// ---------------------------------------------------------------- RNG
// XorShift32 / RandomFloat01, maths.cpp:5-18
TMPT_HD uint32_t xorshift32(uint32_t& state)
{
    uint32_t x = state;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 15;
    state = x;
    return x;
}
TMPT_HD float key_to_float01(uint32_t key24) { return (float)(key24 & 0xFFFFFFu) / 16777216.0f; }
TMPT_HD float random_float01(uint32_t& state) { return key_to_float01(xorshift32(state)); }

// RandomInUnitDisk, maths.cpp:20-28; the draws of one argument list are taken
// left to right (x first): SURVEY.md §0.4.
// `draws` counts the RNG draws taken (2 per try; the speculative row engine
// needs each sample's draw count, tmpt_render.hip render_rowspec).
TMPT_HD f3 random_in_unit_disk(uint32_t& state, uint32_t& draws)
{
    f3 p;
    do {
        float rx = random_float01(state);
        float ry = random_float01(state);
        draws += 2u;
        p = 2.0f * mk(rx, ry, 0.0f) - mk(1.0f, 1.0f, 0.0f);
    } while (dot(p, p) >= 1.0f);
    return p;
}
TMPT_HD f3 random_in_unit_disk(uint32_t& state)
{
    uint32_t draws = 0;
    return random_in_unit_disk(state, draws);
}

// Angle of RandomUnitVector for a 24-bit key, maths.cpp:34: (r * 2) * kPI.
TMPT_HD float unit_angle(uint32_t key24) { return key_to_float01(key24) * 2.0f * kPI; }

// cosf / sinf of the host libm (glibc 2.35: sysdeps/ieee754/flt-32/s_sinf.c,
// s_cosf.c, sincosf.h, sincosf_data.c -- the ARM optimized-routines
// algorithm) restated for the angles RandomUnitVector produces (0 <= a < 2pi,
// so only the |a| < 2^-12, |a| < pi/4 and |a| < 120 paths): the float is
// widened to double, reduced by n = round(a * 2/pi) with the 2^24-scaled
// integer trick of the non-TOINT_INTRINSICS build, and the sine or cosine
// polynomial is evaluated in double, then rounded to float once.  The
// result is bit-identical to the host's cosf/sinf for all 2^24 keys (the
// glibc FMA and SSE2 variants alike; tests/test_host.py checks every key on
// the host, tests/test_gpu_parity.py on the device), so the device needs no
// libm table.
TMPT_HD float glibc_sincosf_poly(double x, double x2, bool neg, int n)
{
    if ((n & 1) == 0) {  // sine polynomial
        const double x3 = x * x2;
        const double s1 = __builtin_fma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
        const double x7 = x3 * x2;
        const double s = __builtin_fma(x3, -0x1.555545995a603p-3, x);
        return (float)__builtin_fma(x7, s1, s);
    }
    // cosine polynomial (negated in the table entry of quadrants 2 and 3)
    const double g = neg ? -1.0 : 1.0;
    const double x4 = x2 * x2;
    const double c2 = __builtin_fma(x2, g * 0x1.99343027bf8c3p-16, g * -0x1.6c087e89a359dp-10);
    const double c1 = __builtin_fma(x2, g * -0x1.ffffffd0c621cp-2, g);
    const double x6 = x4 * x2;
    const double c = __builtin_fma(x4, g * 0x1.55553e1068f19p-5, c1);
    return (float)__builtin_fma(x6, c2, c);
}

TMPT_HD uint32_t glibc_abstop12(float f) { return (__builtin_bit_cast(uint32_t, f) >> 20) & 0x7FFu; }

TMPT_HD void glibc_sincosf_unit(float a, float& c, float& s)
{
    // One path for every angle, no branches: for 0 <= a < pi/4 the reduction
    // gives n = 0 and xr = a exactly (fma(-0, pi/2, x) = x), so it evaluates
    // glibc's |a| < pi/4 polynomials; for a < 2^-12 those round to glibc's
    // sin = a, cos = 1 (the terms beyond x and 1 are below half an ulp).
    // Both polynomials are evaluated once and swapped by quadrant parity.
    // All 2^24 keys are checked against the host libm (tests/test_host.py)
    // and on the device (tests/test_gpu_parity.py).
    const double x = a;
    const double r = x * 0x1.45F306DC9C883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double xr = __builtin_fma(-(double)n, 0x1.921FB54442D18p0, x);
    const double xs = ((n & 3) == 1 || (n & 3) == 2) ? -xr : xr;  // sign[n & 3] = {1, -1, -1, 1}
    const double x2 = xr * xr;
    const bool neg = (n & 2) != 0;
    const float ps = glibc_sincosf_poly(xs, x2, neg, 0);  // sine polynomial
    const float pc = glibc_sincosf_poly(xs, x2, neg, 1);  // cosine polynomial
    const bool odd = (n & 1) != 0;
    s = odd ? pc : ps;
    c = odd ? ps : pc;
}

// RandomUnitVector, maths.cpp:30-38 (cosf/sinf of the host libm, above).
TMPT_HD f3 random_unit_vector(uint32_t& state)
{
    float z = random_float01(state) * 2.0f - 1.0f;
    uint32_t key = xorshift32(state) & 0xFFFFFFu;
    float r = sqrtf(1.0f - z * z);
    float cs, sn;
    glibc_sincosf_unit(unit_angle(key), cs, sn);
    return mk(r * cs, r * sn, z);
}

// Per-pixel seed (DESIGN.md "RNG seeding"): main.cpp:204's y*9781+1 applied
// to the linear pixel index; 0 (a fixed point of xorshift) is remapped.
TMPT_HD uint32_t pixel_seed(uint32_t x, uint32_t y, uint32_t w)
{
    uint32_t s = (y * w + x) * 9781u + 1u;
    return s ? s : 0x6D2B79F5u;
}
TMPT_HD uint32_t row_seed(uint32_t y) { return y * 9781u + 1u; }  // main.cpp:204

// Sample seeding (TMPT_SEED_SAMPLE): sample s of a pixel starts
// kSampleStride xorshift steps per sample into the pixel's own stream, so the
// samples of a pixel are independent work.  xorshift32 is linear over
// GF(2)^32, so the jump is the 32x32 bit matrix J_s = M^(s * kSampleStride),
// applied through four byte tables: jt[s*1024 + 256k + b] = J_s (b << 8k).
constexpr uint32_t kSampleStride = 65536u;
TMPT_HD uint32_t sample_seed(const uint32_t* __restrict__ jt, uint32_t s, uint32_t seed)
{
    const uint32_t* t = jt + (size_t)s * 1024u;
    return t[seed & 255u] ^ t[256u + ((seed >> 8) & 255u)] ^ t[512u + ((seed >> 16) & 255u)] ^
           t[768u + (seed >> 24)];
}

// ---------------------------------------------------------------- camera
// Field order of Camera, maths.h:106-111 (= tmpt_camera in include/tmpt.h).
struct Camera {
    f3 origin, lower_left, horizontal, vertical, u, v, w;
    float lens_radius;
};

// Camera::GetRay, maths.h:93-104
TMPT_HD void camera_get_ray(const Camera& c, float s, float t, uint32_t& state, f3& o, f3& d,
                            uint32_t& draws)
{
    f3 rd = c.lens_radius * random_in_unit_disk(state, draws);
    f3 offset = c.u * rd.x + c.v * rd.y;
    o = c.origin + offset;
    d = normalize(c.lower_left + s * c.horizontal + t * c.vertical - c.origin - offset);
}
TMPT_HD void camera_get_ray(const Camera& c, float s, float t, uint32_t& state, f3& o, f3& d)
{
    uint32_t draws = 0;
    camera_get_ray(c, s, t, state, o, d, draws);
}

// One camera sample of TraceImageBody, main.cpp:212-216 (draws left to right);
// `draws` += the RNG draws it took (2 + 2 per disk try).
TMPT_HD void camera_sample(const Camera& c, uint32_t x, uint32_t y, float invW, float invH,
                           uint32_t& state, f3& o, f3& d, uint32_t& draws)
{
    float su = ((float)x + random_float01(state)) * invW;
    float sv = ((float)y + random_float01(state)) * invH;
    draws += 2u;
    camera_get_ray(c, su, sv, state, o, d, draws);
}
TMPT_HD void camera_sample(const Camera& c, uint32_t x, uint32_t y, float invW, float invH,
                           uint32_t& state, f3& o, f3& d)
{
    uint32_t draws = 0;
    camera_sample(c, x, y, invW, invH, state, o, d, draws);
}

// ---------------------------------------------------------------- geometry
// The decision part of RayIntersectTriangleImproved (maths.cpp:339-380) on a
// precomputed (v0, e1 = v1-v0, e2 = v2-v0): identical roundings, so the same
// accept/reject and the same t, u, v bits.
TMPT_HD bool mt_test(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float tMin, float tMax, float& t, float& u,
                     float& v)
{
    f3 pvec = cross(d, e2);
    float det = dot(e1, pvec);
    if (det > -kDetEps && det < kDetEps) return false;
    float invDet = 1.0f / det;
    f3 tvec = o - v0;
    u = dot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return false;
    f3 qvec = cross(tvec, e1);
    v = dot(d, qvec) * invDet;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = dot(e2, qvec) * invDet;
    return t >= tMin && t <= tMax;
}

// The same test without early exits: every quantity is computed and the
// four rejections of maths.cpp:345-371 are combined at the end. Each value is
// the same expression of the same inputs, so an accepted hit has the same
// bits, and a rejected one is rejected (NaNs fail the final t range test as
// they fail the reference's). For wave64 code, where a divergent early exit
// saves nothing unless the whole wave leaves.
TMPT_HD bool mt_test_flat(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float tMin, float tMax, float& t, float& u,
                          float& v)
{
    const f3 pvec = cross(d, e2);
    const float det = dot(e1, pvec);
    const float invDet = 1.0f / det;
    const f3 tvec = o - v0;
    u = dot(tvec, pvec) * invDet;
    const f3 qvec = cross(tvec, e1);
    v = dot(d, qvec) * invDet;
    t = dot(e2, qvec) * invDet;
    const bool small = det > -kDetEps && det < kDetEps;
    const bool out_u = u < 0.0f || u > 1.0f;
    const bool out_v = v < 0.0f || u + v > 1.0f;
    return !small && !out_u && !out_v && t >= tMin && t <= tMax;
}

// Hit record of the accepted triangle, maths.cpp:375-377.
TMPT_HD f3 hit_pos(f3 v0, f3 v1, f3 v2, float u, float v)
{
    return (1.0f - u - v) * v0 + u * v1 + v * v2;
}
TMPT_HD f3 tri_normal(f3 v0, f3 v1, f3 v2) { return normalize(cross(v1 - v0, v2 - v0)); }

// ---------------------------------------------------------------- shading
TMPT_HD f3 light_dir() { return normalize(mk(-0.7f, 1.0f, 0.5f)); }  // main.cpp:36
// albedo * kLightColor, main.cpp:53,37,67 (evaluated left to right)
TMPT_HD f3 light_albedo() { return mk(0.7f, 0.7f, 0.7f) * mk(0.7f, 0.6f, 0.5f); }

// The scalar of main.cpp:66-67 before the shadow test is applied:
// fmax(0, dot(kLightDir, nl)), nl the normal facing against the ray.
TMPT_HD float light_cosine(f3 normal, f3 ray_dir)
{
    f3 nl = dot(normal, ray_dir) < 0 ? normal : -normal;
    float c = dot(light_dir(), nl);
    return c > 0.0f ? c : 0.0f;  // fmax(0, c), NaN -> 0
}

// Sky gradient, main.cpp:106-107
TMPT_HD f3 sky(f3 dir)
{
    float t = 0.5f * (dir.y + 1.0f);
    return ((1.0f - t) * mk(1.0f, 1.0f, 1.0f) + t * mk(0.5f, 0.7f, 1.0f)) * 0.5f;
}

// One step of the backward recurrence, main.cpp:112-116, for a bounce whose
// light is light_albedo()*cosine (0 when shadowed) and attenuation 0.7.
TMPT_HD f3 backward_step(f3 color, float cosine)
{
    f3 le = mk(0.0f, 0.0f, 0.0f) + light_albedo() * cosine;  // outLightE += ..., main.cpp:48,67
    return le + mk(0.7f, 0.7f, 0.7f) * color;
}

// Pixel write, main.cpp:221-233
TMPT_HD uint32_t pack_pixel(f3 col, float spp_recip)
{
    col = col * spp_recip;
    uint32_t r = (uint32_t)(uint8_t)(saturate(sqrtf(col.x)) * 255.0f);
    uint32_t g = (uint32_t)(uint8_t)(saturate(sqrtf(col.y)) * 255.0f);
    uint32_t b = (uint32_t)(uint8_t)(saturate(sqrtf(col.z)) * 255.0f);
    return r | (g << 8) | (b << 16) | (255u << 24);
}

}  // namespace tmpt
