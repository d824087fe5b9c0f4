/*
 * tmpt_oracle.c -- CPU restatement of pr0g/ToyMeshPathTracer's hot path
 * (Trace -> Scatter -> Scene::HitScene), the checker for the HIP product.
 *
 * TEST INFRASTRUCTURE ONLY (see tmpt_oracle.h for who may load it and how it
 * is pinned).  Build: oracle/Makefile, gcc -O2 -ffp-contract=off.
 *
 * All reference citations are /root/reference/source/<file>:<line>.
 * GLM op order: dot = (x*x'+y*y')+z*z'
 * (glm/detail/func_geometric.inl:52-53), cross term order
 * (func_geometric.inl:74-77), normalize = v * (1/sqrt(dot(v,v)))
 * (func_geometric.inl:88, func_exponential.inl:138), min/max/clamp ternaries
 * (func_common.inl:17-29, :504-507).
 */
#include "tmpt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define K_PI 3.1415926f /* maths.h:14 */
static const float kMinT = 0.001f;    /* main.cpp:30 */
static const float kMaxT = 1.0e7f;    /* main.cpp:31 */
#define K_MAX_DEPTH 10                /* main.cpp:33 */

/* ------------------------------------------------------------------------ */
/* vec3 with GLM 0.9.9.5 semantics                                          */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 x, v3 y)
{
    return V(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
static inline v3 vnormalize(v3 v) { return vscale(v, 1.0f / sqrtf(vdot(v, v))); }
static inline float vlength(v3 v) { return sqrtf(vdot(v, v)); }
static inline float gmin(float x, float y) { return (y < x) ? y : x; } /* func_common.inl:17-21 */
static inline float gmax(float x, float y) { return (x < y) ? y : x; } /* func_common.inl:24-29 */
static inline v3 vmin(v3 a, v3 b) { return V(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
static inline v3 vmax(v3 a, v3 b) { return V(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
static inline float saturate(float v) { return gmin(gmax(v, 0.0f), 1.0f); } /* maths.h:16-19 */
static inline v3 vload(const float* p) { return V(p[0], p[1], p[2]); }
static inline void vstore(float* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
static inline float vget(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

/* ------------------------------------------------------------------------ */
/* RNG (maths.cpp:5-38)                                                     */
/* ------------------------------------------------------------------------ */
uint32_t orc_xorshift32(uint32_t* state) /* maths.cpp:5-13 */
{
    uint32_t x = *state;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 15;
    *state = x;
    return x;
}

/* Jump-ahead of the maths.cpp:5-13 xorshift by n steps (state after n calls).
 * One step is linear over GF(2)^32: x' = M x with M = (I+L15)(I+R17)(I+L13).
 * M^n by square-and-multiply on 32-column bit matrices (column j = image of
 * bit j).  Sample seeding (ORC_SEED_SAMPLE): sample s starts at
 * M^(2^16 s) of the pixel seed. */
static uint32_t orc_gf2_apply(const uint32_t* m, uint32_t x)
{
    uint32_t r = 0;
    for (int j = 0; j < 32; ++j)
        if (x >> j & 1u) r ^= m[j];
    return r;
}

static void orc_gf2_mul(const uint32_t* a, const uint32_t* b, uint32_t* out) /* out = a*b */
{
    uint32_t t[32];
    for (int j = 0; j < 32; ++j) t[j] = orc_gf2_apply(a, b[j]);
    memcpy(out, t, sizeof t);
}

uint32_t orc_xorshift32_jump(uint32_t state, uint64_t n)
{
    uint32_t m[32], acc[32];
    for (int j = 0; j < 32; ++j) {
        uint32_t x = 1u << j;
        orc_xorshift32(&x);
        m[j] = x;
        acc[j] = 1u << j;
    }
    while (n) {
        if (n & 1u) orc_gf2_mul(m, acc, acc);
        orc_gf2_mul(m, m, m);
        n >>= 1;
    }
    return orc_gf2_apply(acc, state);
}

static void orc_jump_matrix(uint64_t n, uint32_t* acc) /* columns of M^n */
{
    uint32_t m[32];
    for (int j = 0; j < 32; ++j) {
        uint32_t x = 1u << j;
        orc_xorshift32(&x);
        m[j] = x;
        acc[j] = 1u << j;
    }
    while (n) {
        if (n & 1u) orc_gf2_mul(m, acc, acc);
        orc_gf2_mul(m, m, m);
        n >>= 1;
    }
}

uint32_t orc_sample_seed(uint32_t seed, uint32_t smp)
{
    return orc_xorshift32_jump(seed, (uint64_t)smp * ORC_SAMPLE_STRIDE);
}

float orc_random_float01(uint32_t* state) /* maths.cpp:15-18 */
{
    return (float)(orc_xorshift32(state) & 0xFFFFFFu) / 16777216.0f;
}

/* maths.cpp:20-28; the two draws in one argument list are sequenced
 * left-to-right (x first), the clang order that reproduces the committed
 * result*.png. */
void orc_random_in_unit_disk(uint32_t* state, float out[3])
{
    v3 p;
    do {
        float rx = orc_random_float01(state);
        float ry = orc_random_float01(state);
        p = vsub(vscale(V(rx, ry, 0.0f), 2.0f), V(1.0f, 1.0f, 0.0f));
    } while (vdot(p, p) >= 1.0f);
    vstore(out, p);
}

void orc_unit_angle_sincos(uint32_t key24, float* c, float* s)
{
    float r = (float)(key24 & 0xFFFFFFu) / 16777216.0f;
    float a = r * 2.0f * K_PI; /* maths.cpp:34: (r*2)*kPI */
    *c = cosf(a);
    *s = sinf(a);
}

void orc_unit_sincos_range(uint32_t key0, uint32_t n, float* out)
{
    for (uint32_t i = 0; i < n; ++i) orc_unit_angle_sincos(key0 + i, &out[2 * (size_t)i], &out[2 * (size_t)i + 1]);
}

void orc_random_unit_vector(uint32_t* state, float out[3]) /* maths.cpp:30-38 */
{
    float z = orc_random_float01(state) * 2.0f - 1.0f;
    float a = orc_random_float01(state) * 2.0f * K_PI;
    float r = sqrtf(1.0f - z * z);
    float x = r * cosf(a);
    float y = r * sinf(a);
    out[0] = x; out[1] = y; out[2] = z;
}

/* Per-pixel seed (pixel mode, DESIGN.md "RNG seeding"): main.cpp:204's
 * y*9781+1 generalised to the linear pixel index; 0 is a fixed point of
 * xorshift, so it is remapped. */
uint32_t orc_pixel_seed(int32_t x, int32_t y, int32_t w)
{
    uint32_t p = (uint32_t)y * (uint32_t)w + (uint32_t)x;
    uint32_t s = p * 9781u + 1u;
    return s ? s : 0x6D2B79F5u;
}

/* ------------------------------------------------------------------------ */
/* Camera (maths.cpp:40-59, maths.h:93-104)                                  */
/* ------------------------------------------------------------------------ */
void orc_camera_init(orc_camera* cam, const float lf[3], const float la[3], const float vup_[3],
                     float vfov, float aspect, float aperture, float focusDist)
{
    v3 lookFrom = vload(lf), lookAt = vload(la), vup = vload(vup_);
    cam->lens_radius = aperture * 0.5f;
    float theta = vfov * K_PI / 180.0f;
    float halfHeight = tanf(theta * 0.5f);
    float halfWidth = aspect * halfHeight;
    v3 origin = lookFrom;
    v3 w = vnormalize(vsub(lookFrom, lookAt));
    v3 u = vnormalize(vcross(vup, w));
    v3 v = vcross(w, u);
    v3 llc = vsub(vsub(vsub(origin, vscale(u, halfWidth * focusDist)),
                       vscale(v, halfHeight * focusDist)),
                  vscale(w, focusDist));
    v3 horizontal = vscale(u, 2.0f * halfWidth * focusDist);
    v3 vertical = vscale(v, 2.0f * halfHeight * focusDist);
    vstore(cam->origin, origin);
    vstore(cam->lower_left, llc);
    vstore(cam->horizontal, horizontal);
    vstore(cam->vertical, vertical);
    vstore(cam->u, u);
    vstore(cam->v, v);
    vstore(cam->w, w);
}

/* main.cpp:295-307 */
void orc_camera_for_scene(orc_camera* cam, const float bmin_[3], const float bmax_[3],
                          int32_t w, int32_t h, int32_t is_sponza)
{
    v3 sceneMin = vload(bmin_), sceneMax = vload(bmax_);
    v3 sceneSize = vsub(sceneMax, sceneMin);
    v3 sceneCenter = vscale(vadd(sceneMin, sceneMax), 0.5f);
    v3 lookfrom = vadd(sceneCenter, vmul(sceneSize, V(0.3f, 0.6f, 1.2f)));
    if (is_sponza) lookfrom = V(-5.96f, 4.08f, -1.22f);
    v3 lookat = vadd(sceneCenter, vmul(sceneSize, V(0.0f, -0.1f, 0.0f)));
    const float distToFocus = vlength(vsub(lookfrom, lookat));
    const float aperture = 0.03f;
    float lf[3], la[3], up[3] = {0.0f, 1.0f, 0.0f};
    vstore(lf, lookfrom);
    vstore(la, lookat);
    orc_camera_init(cam, lf, la, up, 60.0f, (float)w / (float)h, aperture, distToFocus);
}

void orc_camera_get_ray(const orc_camera* cam, float s, float t, uint32_t* state,
                        float out_orig[3], float out_dir[3])
{
    float d[3];
    orc_random_in_unit_disk(state, d);
    v3 rd = vscale(vload(d), cam->lens_radius);
    v3 offset = vadd(vscale(vload(cam->u), rd.x), vscale(vload(cam->v), rd.y));
    v3 origin = vload(cam->origin);
    v3 dir = vsub(vsub(vadd(vadd(vload(cam->lower_left), vscale(vload(cam->horizontal), s)),
                            vscale(vload(cam->vertical), t)),
                       origin),
                  offset);
    vstore(out_orig, vadd(origin, offset));
    vstore(out_dir, vnormalize(dir));
}

/* ------------------------------------------------------------------------ */
/* Intersection primitives                                                  */
/* ------------------------------------------------------------------------ */
typedef struct { v3 v0, v1, v2; } tri_t;
typedef struct { v3 pos, normal; float t; } hit_t;

/* RayIntersectTriangleImproved, maths.cpp:339-380 (Epsilon = 1e-5f, :339) */
static inline int ray_tri(v3 ro, v3 rd, const tri_t* tri, float tMin, float tMax, hit_t* out,
                          float* out_u, float* out_v)
{
    const v3 edge1 = vsub(tri->v1, tri->v0);
    const v3 edge2 = vsub(tri->v2, tri->v0);
    v3 pvec = vcross(rd, edge2);
    const float det = vdot(edge1, pvec);
    if (det > -1e-5f && det < 1e-5f) return 0;
    const float invDet = 1.0f / det;
    const v3 tvec = vsub(ro, tri->v0);
    float u = vdot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return 0;
    const v3 qvec = vcross(tvec, edge1);
    float v = vdot(rd, qvec) * invDet;
    if (v < 0.0f || u + v > 1.0f) return 0;
    const float t = vdot(edge2, qvec) * invDet;
    if (t >= tMin && t <= tMax) {
        out->t = t;
        float w = 1.0f - u - v;
        out->pos = vadd(vadd(vscale(tri->v0, w), vscale(tri->v1, u)), vscale(tri->v2, v));
        out->normal = vnormalize(vcross(edge1, edge2));
        if (out_u) { *out_u = u; *out_v = v; }
        return 1;
    }
    return 0;
}

/* RayHitAabb, maths.h:116-134; r_inv.dir is 1/dir (scene.cpp:92-93) */
static inline int ray_hit_aabb(v3 o, v3 invd, v3 bmin, v3 bmax, float tMin, float tMax)
{
    for (int c = 0; c < 3; ++c) {
        float oc = vget(o, c), ic = vget(invd, c);
        float t0 = (vget(bmin, c) - oc) * ic;
        float t1 = (vget(bmax, c) - oc) * ic;
        if (ic < 0.0f) { float tmp = t0; t0 = t1; t1 = tmp; }
        tMin = t0 > tMin ? t0 : tMin;
        tMax = t1 < tMax ? t1 : tMax;
        if (tMax < tMin) return 0;
    }
    return 1;
}

/* ---- tri/box SAT, maths.cpp:163-298 (used only by the octree build) ---- */
#define AXISTEST_X01(a, b, fa, fb)                                 \
    p0 = a * v0.y - b * v0.z;                                      \
    p2 = a * v2.y - b * v2.z;                                      \
    if (p0 < p2) { mn = p0; mx = p2; } else { mn = p2; mx = p0; }  \
    rad = fa * hs.y + fb * hs.z;                                   \
    if (mn > rad || mx < -rad) return 0;
#define AXISTEST_X2(a, b, fa, fb)                                  \
    p0 = a * v0.y - b * v0.z;                                      \
    p1 = a * v1.y - b * v1.z;                                      \
    if (p0 < p1) { mn = p0; mx = p1; } else { mn = p1; mx = p0; }  \
    rad = fa * hs.y + fb * hs.z;                                   \
    if (mn > rad || mx < -rad) return 0;
#define AXISTEST_Y02(a, b, fa, fb)                                 \
    p0 = -a * v0.x + b * v0.z;                                     \
    p2 = -a * v2.x + b * v2.z;                                     \
    if (p0 < p2) { mn = p0; mx = p2; } else { mn = p2; mx = p0; }  \
    rad = fa * hs.x + fb * hs.z;                                   \
    if (mn > rad || mx < -rad) return 0;
#define AXISTEST_Y1(a, b, fa, fb)                                  \
    p0 = -a * v0.x + b * v0.z;                                     \
    p1 = -a * v1.x + b * v1.z;                                     \
    if (p0 < p1) { mn = p0; mx = p1; } else { mn = p1; mx = p0; }  \
    rad = fa * hs.x + fb * hs.z;                                   \
    if (mn > rad || mx < -rad) return 0;
#define AXISTEST_Z12(a, b, fa, fb)                                 \
    p1 = a * v1.x - b * v1.y;                                      \
    p2 = a * v2.x - b * v2.y;                                      \
    if (p2 < p1) { mn = p2; mx = p1; } else { mn = p1; mx = p2; }  \
    rad = fa * hs.x + fb * hs.y;                                   \
    if (mn > rad || mx < -rad) return 0;
#define AXISTEST_Z0(a, b, fa, fb)                                  \
    p0 = a * v0.x - b * v0.y;                                      \
    p1 = a * v1.x - b * v1.y;                                      \
    if (p0 < p1) { mn = p0; mx = p1; } else { mn = p1; mx = p0; }  \
    rad = fa * hs.x + fb * hs.y;                                   \
    if (mn > rad || mx < -rad) return 0;
#define FINDMINMAX(x0, x1, x2, mn, mx) \
    mn = mx = x0;                      \
    if (x1 < mn) mn = x1;              \
    if (x1 > mx) mx = x1;              \
    if (x2 < mn) mn = x2;              \
    if (x2 > mx) mx = x2;

/* PlaneIntersectAabb, maths.cpp:165-197 */
static int plane_box(v3 normal, v3 vert, v3 maxbox)
{
    float vmin_[3], vmax_[3];
    for (int q = 0; q <= 2; q++) {
        float v = vget(vert, q), mb = vget(maxbox, q);
        if (vget(normal, q) > 0.0f) {
            vmin_[q] = -mb - v;
            vmax_[q] = mb - v;
        } else {
            vmin_[q] = mb - v;
            vmax_[q] = -mb - v;
        }
    }
    if (vdot(normal, vload(vmin_)) > 0.0f) return 0;
    if (vdot(normal, vload(vmax_)) >= 0.0f) return 1;
    return 0;
}

/* TriangleIntersectAabb, maths.cpp:199-298 */
static int tri_box(v3 bc, v3 hs, const tri_t* t)
{
    float mn, mx, p0, p1, p2, rad, fex, fey, fez;
    v3 v0 = vsub(t->v0, bc), v1 = vsub(t->v1, bc), v2 = vsub(t->v2, bc);
    v3 e0 = vsub(v1, v0), e1 = vsub(v2, v1), e2 = vsub(v0, v2);

    fex = fabsf(e0.x); fey = fabsf(e0.y); fez = fabsf(e0.z);
    AXISTEST_X01(e0.z, e0.y, fez, fey);
    AXISTEST_Y02(e0.z, e0.x, fez, fex);
    AXISTEST_Z12(e0.y, e0.x, fey, fex);

    fex = fabsf(e1.x); fey = fabsf(e1.y); fez = fabsf(e1.z);
    AXISTEST_X01(e1.z, e1.y, fez, fey);
    AXISTEST_Y02(e1.z, e1.x, fez, fex);
    AXISTEST_Z0(e1.y, e1.x, fey, fex);

    fex = fabsf(e2.x); fey = fabsf(e2.y); fez = fabsf(e2.z);
    AXISTEST_X2(e2.z, e2.y, fez, fey);
    AXISTEST_Y1(e2.z, e2.x, fez, fex);
    AXISTEST_Z12(e2.y, e2.x, fey, fex);

    FINDMINMAX(v0.x, v1.x, v2.x, mn, mx);
    if (mn > hs.x || mx < -hs.x) return 0;
    FINDMINMAX(v0.y, v1.y, v2.y, mn, mx);
    if (mn > hs.y || mx < -hs.y) return 0;
    FINDMINMAX(v0.z, v1.z, v2.z, mn, mx);
    if (mn > hs.z || mx < -hs.z) return 0;

    v3 normal = vcross(e0, e1);
    if (!plane_box(normal, v0, hs)) return 0;
    return 1;
}

/* ------------------------------------------------------------------------ */
/* Scene                                                                    */
/* ------------------------------------------------------------------------ */
typedef struct {
    v3 bmin, bmax;
    int32_t first_child; /* -1 for leaf; children are first_child..+7 */
    int32_t tri_off, tri_cnt;
} oct_node;

typedef struct {
    v3 bmin, bmax;   /* conservatively inflated */
    int32_t left, right; /* internal: children; leaf: left=-1, right unused */
    int32_t tri_off, tri_cnt;
} bvh_node;

struct orc_scene {
    int32_t n;
    tri_t* tris;
    int32_t accel, tie_mode;
    /* octree */
    oct_node* oct;
    int64_t n_oct, cap_oct;
    int32_t* oct_tris;
    int64_t n_oct_tris, cap_oct_tris;
    /* bvh */
    bvh_node* bvh;
    int64_t n_bvh;
    int32_t* bvh_tris;
};

static int64_t oct_alloc_node(orc_scene* s)
{
    if (s->n_oct == s->cap_oct) {
        s->cap_oct = s->cap_oct ? s->cap_oct * 2 : 1024;
        s->oct = (oct_node*)realloc(s->oct, (size_t)s->cap_oct * sizeof(oct_node));
    }
    return s->n_oct++;
}

static void oct_push_tris(orc_scene* s, const int32_t* ids, int32_t cnt, int64_t node)
{
    if (s->n_oct_tris + cnt > s->cap_oct_tris) {
        while (s->n_oct_tris + cnt > s->cap_oct_tris)
            s->cap_oct_tris = s->cap_oct_tris ? s->cap_oct_tris * 2 : 4096;
        s->oct_tris = (int32_t*)realloc(s->oct_tris, (size_t)s->cap_oct_tris * sizeof(int32_t));
    }
    if (cnt > 0) memcpy(s->oct_tris + s->n_oct_tris, ids, (size_t)cnt * sizeof(int32_t)); /* (UBSan: no NULL to memcpy) */
    s->oct[node].tri_off = (int32_t)s->n_oct_tris;
    s->oct[node].tri_cnt = cnt;
    s->n_oct_tris += cnt;
}

/* OctreeNode::Subdivide / InternalDivide, scene.cpp:99-160.  `ids` is the
 * node's triangle list (indices into the scene copy, in reference order). */
static void oct_subdivide(orc_scene* s, int64_t node, int32_t* ids, int32_t cnt, int depth)
{
    if (!(cnt > 10 && depth < 10)) { /* scene.cpp:101 */
        s->oct[node].first_child = -1;
        oct_push_tris(s, ids, cnt, node);
        return;
    }
    int cdepth = depth + 1; /* InternalDivide(depth + 1), scene.cpp:103 */
    v3 pmin = s->oct[node].bmin, pmax = s->oct[node].bmax;
    const v3 half = vscale(vsub(pmax, pmin), 0.5f);
    int64_t first = s->n_oct;
    for (int i = 0; i < 8; ++i) oct_alloc_node(s);
    s->oct[node].first_child = (int32_t)first;
    s->oct[node].tri_off = 0;
    s->oct[node].tri_cnt = 0;
    static const float ox[8] = {0, 1, 0, 1, 0, 1, 0, 1};
    static const float oy[8] = {0, 0, 0, 0, 1, 1, 1, 1};
    static const float oz[8] = {0, 0, 1, 1, 0, 0, 1, 1};
    for (int i = 0; i < 8; ++i) { /* scene.cpp:119-141 */
        v3 cmin;
        if (i == 0) cmin = pmin;
        else if (i == 7) cmin = vadd(pmin, half);
        else cmin = vadd(pmin, V(ox[i] ? half.x : 0.0f, oy[i] ? half.y : 0.0f, oz[i] ? half.z : 0.0f));
        s->oct[first + i].bmin = cmin;
        s->oct[first + i].bmax = vadd(cmin, half);
    }
    int32_t* sub = (int32_t*)malloc((size_t)(cnt > 0 ? cnt : 1) * sizeof(int32_t));
    for (int i = 0; i < 8; ++i) { /* scene.cpp:144-157 */
        int64_t c = first + i;
        v3 cmin = s->oct[c].bmin, cmax = s->oct[c].bmax;
        v3 center = vscale(vadd(cmin, cmax), 0.5f);
        v3 hd = vscale(vsub(cmax, cmin), 0.5f);
        int32_t m = 0;
        for (int32_t k = 0; k < cnt; ++k)
            if (tri_box(center, hd, &s->tris[ids[k]])) sub[m++] = ids[k];
        oct_subdivide(s, c, sub, m, cdepth);
    }
    free(sub);
}

/* HitSceneInternal, scene.cpp:21-52 */
static void oct_hit(const orc_scene* s, int64_t node, v3 ro, v3 rd, v3 inv, float tMin, float tMax,
                    hit_t* outHit, int32_t* hitId, float* hitMinT)
{
    const oct_node* nd = &s->oct[node];
    if (!ray_hit_aabb(ro, inv, nd->bmin, nd->bmax, tMin, tMax)) return;
    if (nd->first_child < 0) {
        for (int32_t k = 0; k < nd->tri_cnt; ++k) {
            int32_t id = s->oct_tris[nd->tri_off + k];
            hit_t hit;
            if (ray_tri(ro, rd, &s->tris[id], tMin, tMax, &hit, NULL, NULL)) {
                int take = hit.t < *hitMinT;
                if (s->tie_mode == ORC_TIE_INDEX && hit.t == *hitMinT && *hitId >= 0 && id < *hitId)
                    take = 1;
                if (take) {
                    *hitMinT = hit.t;
                    *hitId = id;
                    *outHit = hit;
                }
            }
        }
    } else {
        for (int i = 0; i < 8; ++i)
            oct_hit(s, nd->first_child + i, ro, rd, inv, tMin, tMax, outHit, hitId, hitMinT);
    }
}

/* ---- exact-semantics BVH (own structure; DESIGN.md "scene query contract") ----
 * Same answer as a linear scan with strict '<' (lowest index among equal t):
 * boxes are inflated and the slab test is slackened so culling is
 * conservative, and ties are broken on the triangle index. */
#define BVH_PAD_REL 1e-5f
#define BVH_TFAR_SLACK 1.00001f

typedef struct { float c; int32_t id; } cent_t;
static int cmp_cent(const void* a, const void* b)
{
    const cent_t* x = (const cent_t*)a;
    const cent_t* y = (const cent_t*)b;
    if (x->c < y->c) return -1;
    if (x->c > y->c) return 1;
    return (x->id > y->id) - (x->id < y->id);
}

static void tri_bounds(const tri_t* t, v3* lo, v3* hi)
{
    *lo = vmin(vmin(t->v0, t->v1), t->v2);
    *hi = vmax(vmax(t->v0, t->v1), t->v2);
    float px = BVH_PAD_REL * (fmaxf(fabsf(lo->x), fabsf(hi->x)) + (hi->x - lo->x)) + 1e-30f;
    float py = BVH_PAD_REL * (fmaxf(fabsf(lo->y), fabsf(hi->y)) + (hi->y - lo->y)) + 1e-30f;
    float pz = BVH_PAD_REL * (fmaxf(fabsf(lo->z), fabsf(hi->z)) + (hi->z - lo->z)) + 1e-30f;
    *lo = V(lo->x - px, lo->y - py, lo->z - pz);
    *hi = V(hi->x + px, hi->y + py, hi->z + pz);
}

static int32_t bvh_build_rec(orc_scene* s, int32_t* ids, int32_t lo_i, int32_t hi_i, cent_t* scratch)
{
    int32_t node = (int32_t)s->n_bvh++;
    v3 bl = V(INFINITY, INFINITY, INFINITY), bh = V(-INFINITY, -INFINITY, -INFINITY);
    v3 cl = bl, ch = bh;
    for (int32_t k = lo_i; k < hi_i; ++k) {
        v3 l, h;
        tri_bounds(&s->tris[ids[k]], &l, &h);
        bl = vmin(bl, l);
        bh = vmax(bh, h);
        v3 c = vscale(vadd(l, h), 0.5f);
        cl = vmin(cl, c);
        ch = vmax(ch, c);
    }
    s->bvh[node].bmin = bl;
    s->bvh[node].bmax = bh;
    int32_t cnt = hi_i - lo_i;
    if (cnt <= 4) {
        s->bvh[node].left = -1;
        s->bvh[node].right = -1;
        s->bvh[node].tri_off = lo_i;
        s->bvh[node].tri_cnt = cnt;
        return node;
    }
    v3 ext = vsub(ch, cl);
    int axis = (ext.x >= ext.y && ext.x >= ext.z) ? 0 : (ext.y >= ext.z ? 1 : 2);
    for (int32_t k = lo_i; k < hi_i; ++k) {
        v3 l, h;
        tri_bounds(&s->tris[ids[k]], &l, &h);
        scratch[k - lo_i].c = vget(vadd(l, h), axis);
        scratch[k - lo_i].id = ids[k];
    }
    qsort(scratch, (size_t)cnt, sizeof(cent_t), cmp_cent);
    for (int32_t k = lo_i; k < hi_i; ++k) ids[k] = scratch[k - lo_i].id;
    int32_t mid = lo_i + cnt / 2;
    int32_t l = bvh_build_rec(s, ids, lo_i, mid, scratch);
    int32_t r = bvh_build_rec(s, ids, mid, hi_i, scratch);
    s->bvh[node].left = l;
    s->bvh[node].right = r;
    s->bvh[node].tri_off = 0;
    s->bvh[node].tri_cnt = 0;
    return node;
}

static inline float safe_inv(float d)
{
    if (fabsf(d) < 1e-20f) d = copysignf(1e-20f, d);
    return 1.0f / d;
}

static inline int slab_conservative(v3 o, v3 inv, v3 bmin, v3 bmax, float tfar_max)
{
    float tx0 = (bmin.x - o.x) * inv.x, tx1 = (bmax.x - o.x) * inv.x;
    float ty0 = (bmin.y - o.y) * inv.y, ty1 = (bmax.y - o.y) * inv.y;
    float tz0 = (bmin.z - o.z) * inv.z, tz1 = (bmax.z - o.z) * inv.z;
    float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tfar_max));
    return tn <= tf * BVH_TFAR_SLACK;
}

static void bvh_hit(const orc_scene* s, v3 ro, v3 rd, float tMin, float tMax, hit_t* outHit,
                    int32_t* hitId, float* hitMinT)
{
    v3 inv = V(safe_inv(rd.x), safe_inv(rd.y), safe_inv(rd.z));
    int32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const bvh_node* nd = &s->bvh[stack[--sp]];
        if (!slab_conservative(ro, inv, nd->bmin, nd->bmax, *hitMinT)) continue;
        if (nd->left < 0) {
            for (int32_t k = 0; k < nd->tri_cnt; ++k) {
                int32_t id = s->bvh_tris[nd->tri_off + k];
                hit_t hit;
                if (ray_tri(ro, rd, &s->tris[id], tMin, tMax, &hit, NULL, NULL)) {
                    if (hit.t < *hitMinT || (hit.t == *hitMinT && *hitId >= 0 && id < *hitId)) {
                        *hitMinT = hit.t;
                        *hitId = id;
                        *outHit = hit;
                    }
                }
            }
        } else {
            stack[sp++] = nd->right;
            stack[sp++] = nd->left;
        }
    }
}

orc_scene* orc_scene_create(const float* tris, int32_t n, int32_t accel, int32_t tie_mode,
                            const float oct_min[3], const float oct_max[3])
{
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->n = n;
    s->accel = accel;
    s->tie_mode = tie_mode;
    s->tris = (tri_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(tri_t)); /* scene.cpp:54-57 */
    for (int32_t i = 0; i < n; ++i) {
        s->tris[i].v0 = vload(tris + 9 * i);
        s->tris[i].v1 = vload(tris + 9 * i + 3);
        s->tris[i].v2 = vload(tris + 9 * i + 6);
    }
    int32_t* ids = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    for (int32_t i = 0; i < n; ++i) ids[i] = i;
    if (accel == ORC_ACCEL_OCTREE) { /* BuildOctree, scene.cpp:75-83 */
        int64_t root = oct_alloc_node(s);
        s->oct[root].bmin = vload(oct_min);
        s->oct[root].bmax = vload(oct_max);
        oct_subdivide(s, root, ids, n, 0);
    } else if (accel == ORC_ACCEL_BVH && n > 0) {
        s->bvh = (bvh_node*)malloc((size_t)(2 * n + 1) * sizeof(bvh_node));
        cent_t* scratch = (cent_t*)malloc((size_t)n * sizeof(cent_t));
        bvh_build_rec(s, ids, 0, n, scratch);
        free(scratch);
        s->bvh_tris = ids;
        ids = NULL;
    }
    free(ids);
    return s;
}

void orc_scene_destroy(orc_scene* s)
{
    if (!s) return;
    free(s->tris);
    free(s->oct);
    free(s->oct_tris);
    free(s->bvh);
    free(s->bvh_tris);
    free(s);
}

void orc_scene_stats(const orc_scene* s, int64_t out[4])
{
    int64_t leaves = 0;
    for (int64_t i = 0; i < s->n_oct; ++i) leaves += s->oct[i].first_child < 0;
    out[0] = s->accel == ORC_ACCEL_BVH ? s->n_bvh : s->n_oct;
    out[1] = leaves;
    out[2] = s->n_oct_tris;
    out[3] = s->n;
}

/* FNV-1a over the octree in depth-first preorder (each node's box bits, then
 * for a leaf its triangle count and list) -- the same walk the library's
 * tmpt_octree_digest hashes, so the two octrees can be compared node for node. */
static void fnv_word(uint64_t* h, uint32_t w)
{
    for (int b = 0; b < 4; ++b) *h = (*h ^ ((w >> (8 * b)) & 255u)) * 1099511628211ull;
}
static void oct_digest_rec(const orc_scene* s, int64_t node, uint64_t* h)
{
    const oct_node* nd = &s->oct[node];
    const float f[6] = {nd->bmin.x, nd->bmin.y, nd->bmin.z, nd->bmax.x, nd->bmax.y, nd->bmax.z};
    for (int k = 0; k < 6; ++k) {
        uint32_t u;
        memcpy(&u, &f[k], 4);
        fnv_word(h, u);
    }
    fnv_word(h, nd->first_child < 0 ? 1u : 0u);
    if (nd->first_child < 0) {
        fnv_word(h, (uint32_t)nd->tri_cnt);
        for (int32_t k = 0; k < nd->tri_cnt; ++k) fnv_word(h, (uint32_t)s->oct_tris[nd->tri_off + k]);
    } else {
        for (int i = 0; i < 8; ++i) oct_digest_rec(s, nd->first_child + i, h);
    }
}

uint64_t orc_octree_digest(const orc_scene* s)
{
    uint64_t h = 1469598103934665603ull;
    if (s->accel == ORC_ACCEL_OCTREE && s->n_oct > 0) oct_digest_rec(s, 0, &h);
    return h;
}

static void oct_depths(const orc_scene* s, int64_t node, int32_t depth, int32_t* info, int64_t cap)
{
    if (node < cap) info[3 * node + 2] = depth;
    const oct_node* nd = &s->oct[node];
    if (nd->first_child >= 0)
        for (int i = 0; i < 8; ++i) oct_depths(s, nd->first_child + i, depth + 1, info, cap);
}

int64_t orc_octree_nodes(const orc_scene* s, float* boxes, int32_t* info, int64_t cap)
{
    if (s->accel != ORC_ACCEL_OCTREE) return 0;
    const int64_t m = s->n_oct < cap ? s->n_oct : cap;
    for (int64_t i = 0; i < m; ++i) {
        const oct_node* nd = &s->oct[i];
        vstore(boxes + 6 * i, nd->bmin);
        vstore(boxes + 6 * i + 3, nd->bmax);
        info[3 * i] = nd->first_child;
        info[3 * i + 1] = nd->first_child < 0 ? nd->tri_cnt : 0;
    }
    if (s->n_oct > 0 && m > 0) oct_depths(s, 0, 0, info, m);
    return s->n_oct;
}

int32_t orc_octree_leaf(const orc_scene* s, int64_t node, int32_t* ids, int32_t cap)
{
    if (s->accel != ORC_ACCEL_OCTREE || node < 0 || node >= s->n_oct || s->oct[node].first_child >= 0) return 0;
    const oct_node* nd = &s->oct[node];
    for (int32_t k = 0; k < nd->tri_cnt && k < cap; ++k) ids[k] = s->oct_tris[nd->tri_off + k];
    return nd->tri_cnt;
}

void orc_ray_box_batch(const float* rays, int64_t n, const float box[6], float tmin, float tmax, uint8_t* out)
{
    const v3 lo = vload(box), hi = vload(box + 3);
    for (int64_t i = 0; i < n; ++i) {
        const v3 o = vload(rays + 6 * i), d = vload(rays + 6 * i + 3);
        const v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); /* scene.cpp:92-93 */
        out[i] = (uint8_t)ray_hit_aabb(o, inv, lo, hi, tmin, tmax);
    }
}

/* Scene::HitScene, scene.cpp:86-97 (returns the triangle index, not 1) */
static int32_t hit_scene(const orc_scene* s, v3 ro, v3 rd, float tMin, float tMax, hit_t* out)
{
    int32_t hitId = -1;
    float hitMinT = tMax;
    if (s->n == 0) return -1;
    if (s->accel == ORC_ACCEL_OCTREE) {
        v3 inv = V(1.0f / rd.x, 1.0f / rd.y, 1.0f / rd.z);
        oct_hit(s, 0, ro, rd, inv, tMin, tMax, out, &hitId, &hitMinT);
    } else if (s->accel == ORC_ACCEL_BVH) {
        bvh_hit(s, ro, rd, tMin, tMax, out, &hitId, &hitMinT);
    } else {
        for (int32_t i = 0; i < s->n; ++i) {
            hit_t hit;
            if (ray_tri(ro, rd, &s->tris[i], tMin, tMax, &hit, NULL, NULL) && hit.t < hitMinT) {
                hitMinT = hit.t;
                hitId = i;
                *out = hit;
            }
        }
    }
    return hitId;
}

int32_t orc_hit_scene(const orc_scene* s, const float orig[3], const float dir[3], float tmin,
                      float tmax, float hit_out[7])
{
    hit_t h;
    int32_t id = hit_scene(s, vload(orig), vload(dir), tmin, tmax, &h);
    if (id >= 0) {
        vstore(hit_out, h.pos);
        vstore(hit_out + 3, h.normal);
        hit_out[6] = h.t;
    }
    return id;
}

typedef struct {
    const orc_scene* s;
    const float* rays;
    int64_t n;
    float tmin, tmax;
    float* hits;
    int32_t* ids;
    atomic_llong next;
} batch_job;

static void* batch_worker(void* arg)
{
    batch_job* j = (batch_job*)arg;
    for (;;) {
        int64_t b = atomic_fetch_add(&j->next, 1024);
        if (b >= j->n) break;
        int64_t e = b + 1024 < j->n ? b + 1024 : j->n;
        for (int64_t i = b; i < e; ++i) {
            j->ids[i] = orc_hit_scene(j->s, j->rays + 6 * i, j->rays + 6 * i + 3, j->tmin, j->tmax,
                                      j->hits + 7 * i);
        }
    }
    return NULL;
}

void orc_hit_batch(const orc_scene* s, const float* rays, int64_t n, float tmin, float tmax,
                   float* hits, int32_t* ids, int32_t nthreads)
{
    batch_job j;
    j.s = s; j.rays = rays; j.n = n; j.tmin = tmin; j.tmax = tmax; j.hits = hits; j.ids = ids;
    atomic_init(&j.next, 0);
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, batch_worker, &j);
    batch_worker(&j);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
}

/* ------------------------------------------------------------------------ */
/* Tracer                                                                   */
/* ------------------------------------------------------------------------ */
static v3 light_dir(void) /* main.cpp:36 */
{
    return vnormalize(V(-0.7f, 1.0f, 0.5f));
}

/* Scatter, main.cpp:44-73 */
static void scatter(const orc_scene* s, v3 rdir_in, const hit_t* hit, v3* outAtten, v3* outLightE,
                    uint32_t* rng, uint64_t* rays, v3* out_o, v3* out_d)
{
    const v3 kLightDir = light_dir();
    const v3 kLightColor = V(0.7f, 0.6f, 0.5f); /* main.cpp:37 */
    *outLightE = V(0.0f, 0.0f, 0.0f);
    v3 albedo = V(0.7f, 0.7f, 0.7f);
    *outAtten = albedo;
    ++*rays;
    hit_t lightHit;
    int32_t id = hit_scene(s, hit->pos, kLightDir, kMinT, kMaxT, &lightHit);
    if (id == -1) {
        v3 rdir = rdir_in;
        v3 nl = vdot(hit->normal, rdir) < 0 ? hit->normal : vneg(hit->normal);
        float d = vdot(kLightDir, nl);
        float f = fmaxf(0.0f, d); /* fmax(0, x): NaN -> 0 */
        *outLightE = vadd(*outLightE, vscale(vmul(albedo, kLightColor), f));
    }
    float r[3];
    orc_random_unit_vector(rng, r);
    v3 target = vadd(vadd(hit->pos, hit->normal), vload(r));
    *out_o = hit->pos;
    *out_d = vnormalize(vsub(target, hit->pos));
}

/* Trace, main.cpp:82-119 */
static v3 trace(const orc_scene* s, v3 ro, v3 rd, uint32_t* rng, uint64_t* rays)
{
    v3 light[K_MAX_DEPTH], atten[K_MAX_DEPTH];
    int depth = 0;
    v3 color = V(0.0f, 0.0f, 0.0f);
    while (depth < K_MAX_DEPTH) {
        ++*rays;
        hit_t hit;
        int32_t id = hit_scene(s, ro, rd, kMinT, kMaxT, &hit);
        if (id != -1) {
            v3 no, nd;
            scatter(s, rd, &hit, &atten[depth], &light[depth], rng, rays, &no, &nd);
            ro = no;
            rd = nd;
            ++depth;
        } else {
            float t = 0.5f * (rd.y + 1.0f);
            color = vscale(vadd(vscale(V(1.0f, 1.0f, 1.0f), 1.0f - t), vscale(V(0.5f, 0.7f, 1.0f), t)),
                           0.5f);
            break;
        }
    }
    for (int i = depth - 1; i >= 0; --i) color = vadd(light[i], vmul(atten[i], color));
    return color;
}

void orc_trace(const orc_scene* s, const float orig[3], const float dir[3], uint32_t* rng,
               float out_col[3], uint64_t* rays)
{
    vstore(out_col, trace(s, vload(orig), vload(dir), rng, rays));
}

/* TraceImageBody::operator() for one row, main.cpp:192-238.  Seeding:
 * row (main.cpp:204, the stream threads along the row), pixel (one stream per
 * pixel, its samples in sequence) or sample (sample smp of the pixel starts at
 * M^(smp * 2^16) of the pixel seed: jumps[smp] = that matrix's columns). */
/* Pixels x = xa, xa + xs, ... < xb of row y (row seeding: always the whole
 * row, its stream runs through every pixel). */
static uint64_t render_row(const orc_scene* s, const orc_camera* cam, int32_t w, int32_t h,
                           int32_t spp, int32_t seed_mode, int64_t y, int64_t xa, int64_t xb, int64_t xs,
                           uint8_t* image, const uint32_t* jumps)
{
    const float invWidth = 1.0f / (float)w;     /* main.cpp:186 */
    const float invHeight = 1.0f / (float)h;    /* main.cpp:187 */
    const float sppRecip = 1.0f / (float)spp;   /* main.cpp:188 */
    uint64_t rays = 0;
    uint32_t rngState = (uint32_t)y * 9781u + 1u; /* main.cpp:204 */
    if (seed_mode == ORC_SEED_ROW) {
        xa = 0;
        xb = w;
        xs = 1;
    }
    for (int64_t x = xa; x < xb; x += xs) {
        if (seed_mode == ORC_SEED_PIXEL) rngState = orc_pixel_seed((int32_t)x, (int32_t)y, w);
        v3 col = V(0.0f, 0.0f, 0.0f);
        const uint32_t pseed = orc_pixel_seed((int32_t)x, (int32_t)y, w);
        for (int64_t smp = 0; smp < spp; smp++) {
            if (seed_mode == ORC_SEED_SAMPLE) rngState = orc_gf2_apply(jumps + 32 * smp, pseed);
            /* main.cpp:212-216, arguments sequenced left to right */
            float su = ((float)x + orc_random_float01(&rngState)) * invWidth;
            float sv = ((float)y + orc_random_float01(&rngState)) * invHeight;
            float o[3], d[3];
            orc_camera_get_ray(cam, su, sv, &rngState, o, d);
            col = vadd(col, trace(s, vload(o), vload(d), &rngState, &rays));
        }
        col = vscale(col, sppRecip);
        col.x = sqrtf(col.x);
        col.y = sqrtf(col.y);
        col.z = sqrtf(col.z);
        const int64_t lookup = (y * w + x) * 4;
        image[lookup + 0] = (uint8_t)(saturate(col.x) * 255.0f);
        image[lookup + 1] = (uint8_t)(saturate(col.y) * 255.0f);
        image[lookup + 2] = (uint8_t)(saturate(col.z) * 255.0f);
        image[lookup + 3] = 255;
    }
    return rays;
}

/* Work units: rows (grain 1, main.cpp:329-331), or -- pixel and sample
 * seeding, where pixels are independent -- row pieces of kUnitPixels
 * rendered pixels, so a few rows still spread over every thread. */
enum { kUnitPixels = 64 };

typedef struct {
    const orc_scene* s;
    const orc_camera* cam;
    int32_t w, h, spp, seed_mode, y0, y1, step, x0, xstep;
    int64_t pieces; /* units per row */
    uint8_t* rgba;
    const uint32_t* jumps;
    atomic_llong next;
    atomic_ullong rays;
} render_job;

static void* render_worker(void* arg)
{
    render_job* j = (render_job*)arg;
    uint64_t local = 0;
    for (;;) {
        int64_t k = atomic_fetch_add(&j->next, 1);
        int64_t r = k / j->pieces, p = k - r * j->pieces;
        int64_t y = (int64_t)j->y0 + r * j->step;
        if (y >= j->y1) break;
        const int64_t span = (int64_t)kUnitPixels * j->xstep;
        const int64_t xa = j->x0 + p * span;
        int64_t xb = xa + span;
        if (xb > j->w) xb = j->w;
        local += render_row(j->s, j->cam, j->w, j->h, j->spp, j->seed_mode, y, xa, xb, j->xstep, j->rgba,
                            j->jumps);
    }
    atomic_fetch_add(&j->rays, local);
    return NULL;
}

uint64_t orc_render(const orc_scene* s, const orc_camera* cam, int32_t w, int32_t h, int32_t spp,
                    int32_t seed_mode, int32_t y0, int32_t y1, int32_t row_step, int32_t nthreads,
                    uint8_t* rgba)
{
    return orc_render_ex(s, cam, w, h, spp, seed_mode, y0, y1, row_step, 0, 1, nthreads, rgba);
}

uint64_t orc_render_ex(const orc_scene* s, const orc_camera* cam, int32_t w, int32_t h, int32_t spp,
                       int32_t seed_mode, int32_t y0, int32_t y1, int32_t row_step, int32_t x0,
                       int32_t x_step, int32_t nthreads, uint8_t* rgba)
{
    render_job j;
    j.s = s; j.cam = cam; j.w = w; j.h = h; j.spp = spp; j.seed_mode = seed_mode;
    j.y0 = y0; j.y1 = y1 < h ? y1 : h; j.step = row_step > 0 ? row_step : 1; j.rgba = rgba;
    j.x0 = x0 < 0 ? 0 : x0;
    j.xstep = x_step > 0 ? x_step : 1;
    if (seed_mode == ORC_SEED_ROW) {
        j.x0 = 0;
        j.xstep = 1;
        j.pieces = 1;
    } else {
        const int64_t npx = j.x0 < w ? (w - j.x0 + j.xstep - 1) / j.xstep : 0;
        j.pieces = npx > 0 ? (npx + kUnitPixels - 1) / kUnitPixels : 1;
    }
    uint32_t* jumps = NULL;
    if (seed_mode == ORC_SEED_SAMPLE) { /* M^(smp * stride) for every sample index */
        uint32_t stride[32];
        jumps = (uint32_t*)malloc(sizeof(uint32_t) * 32 * (size_t)(spp > 0 ? spp : 1));
        if (!jumps) return 0;
        orc_jump_matrix(ORC_SAMPLE_STRIDE, stride);
        for (int b = 0; b < 32; ++b) jumps[b] = 1u << b;
        for (int32_t k = 1; k < spp; ++k) orc_gf2_mul(stride, jumps + 32 * (k - 1), jumps + 32 * k);
    }
    j.jumps = jumps;
    atomic_init(&j.next, 0);
    atomic_init(&j.rays, 0);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, render_worker, &j);
    render_worker(&j);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    free(jumps);
    return atomic_load(&j.rays);
}

/* ------------------------------------------------------------------------ */
/* OBJ ingest: objparser.cpp:34-355 + LoadScene main.cpp:122-170            */
/* ------------------------------------------------------------------------ */
static int parse_int(const char* s, const char** end) /* objparser.cpp:34-60 */
{
    while (*s == ' ' || *s == '\t') s++;
    int sign = (*s == '-');
    s += (*s == '-' || *s == '+');
    unsigned int result = 0;
    for (;;) {
        if ((unsigned)(*s - '0') < 10) result = result * 10 + (unsigned)(*s - '0');
        else break;
        s++;
    }
    *end = s;
    return sign ? -(int)result : (int)result;
}

static float parse_float(const char* s, const char** end) /* objparser.cpp:62-131 */
{
    static const double digits[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9};
    static const double powers[] = {1e0,  1e+1,  1e+2,  1e+3,  1e+4,  1e+5,  1e+6,  1e+7,
                                    1e+8, 1e+9,  1e+10, 1e+11, 1e+12, 1e+13, 1e+14, 1e+15,
                                    1e+16, 1e+17, 1e+18, 1e+19, 1e+20, 1e+21, 1e+22};
    while (*s == ' ' || *s == '\t') s++;
    double sign = (*s == '-') ? -1 : 1;
    s += (*s == '-' || *s == '+');
    double result = 0;
    int power = 0;
    while ((unsigned)(*s - '0') < 10) {
        result = result * 10 + digits[*s - '0'];
        s++;
    }
    if (*s == '.') {
        s++;
        while ((unsigned)(*s - '0') < 10) {
            result = result * 10 + digits[*s - '0'];
            s++;
            power--;
        }
    }
    if ((*s | ' ') == 'e') {
        s++;
        int expsign = (*s == '-') ? -1 : 1;
        s += (*s == '-' || *s == '+');
        int exppower = 0;
        while ((unsigned)(*s - '0') < 10) {
            exppower = exppower * 10 + (*s - '0');
            s++;
        }
        power += expsign * exppower;
    }
    *end = s;
    if ((unsigned)(-power) < sizeof(powers) / sizeof(powers[0]))
        return (float)(sign * result / powers[-power]);
    else if ((unsigned)power < sizeof(powers) / sizeof(powers[0]))
        return (float)(sign * result * powers[power]);
    else
        return (float)(sign * result * pow(10.0, power));
}

static const char* parse_face(const char* s, int* vi, int* vti, int* vni) /* objparser.cpp:133-155 */
{
    while (*s == ' ' || *s == '\t') s++;
    *vi = parse_int(s, &s);
    if (*s != '/') return s;
    s++;
    if (*s != '/') *vti = parse_int(s, &s);
    if (*s != '/') return s;
    s++;
    *vni = parse_int(s, &s);
    return s;
}

typedef struct {
    float* v; size_t nv, cv;
    int* f; size_t nf, cf;
    size_t nvt, nvn;
} objf;

static int fixup_index(int index, size_t size) /* objparser.cpp:29-32 */
{
    return (index >= 0) ? index - 1 : (int)size + index;
}

static void obj_line(objf* o, const char* line) /* objparser.cpp:185-302 (v, vt, vn, f) */
{
    if (line[0] == 'v' && line[1] == ' ') {
        const char* s = line + 2;
        float x = parse_float(s, &s);
        float y = parse_float(s, &s);
        float z = parse_float(s, &s);
        if (o->nv + 3 > o->cv) {
            o->cv = o->cv ? o->cv * 2 : 96;
            o->v = (float*)realloc(o->v, o->cv * sizeof(float));
        }
        o->v[o->nv++] = x;
        o->v[o->nv++] = y;
        o->v[o->nv++] = z;
    } else if (line[0] == 'v' && line[1] == 't' && line[2] == ' ') {
        o->nvt += 3;
    } else if (line[0] == 'v' && line[1] == 'n' && line[2] == ' ') {
        o->nvn += 3;
    } else if (line[0] == 'f' && line[1] == ' ') {
        const char* s = line + 2;
        size_t v = o->nv / 3, vt = o->nvt / 3, vn = o->nvn / 3;
        int fv = 0;
        int f[3][3] = {{0}};
        while (*s) {
            int vi = 0, vti = 0, vni = 0;
            s = parse_face(s, &vi, &vti, &vni);
            if (vi == 0) break;
            f[fv][0] = fixup_index(vi, v);
            f[fv][1] = fixup_index(vti, vt);
            f[fv][2] = fixup_index(vni, vn);
            if (fv == 2) { /* fan triangulation, objparser.cpp:263-276 */
                if (o->nf + 9 > o->cf) {
                    o->cf = o->cf ? o->cf * 2 : 288;
                    o->f = (int*)realloc(o->f, o->cf * sizeof(int));
                }
                memcpy(&o->f[o->nf], f, 9 * sizeof(int));
                o->nf += 9;
                f[1][0] = f[2][0];
                f[1][1] = f[2][1];
                f[1][2] = f[2][2];
            } else {
                fv++;
            }
        }
    }
}

int orc_load_scene(const char* path, float** out_tris, int32_t* out_n, float out_bmin[3],
                   float out_bmax[3])
{
    FILE* fp = fopen(path, "rb");
    if (!fp) return -1;
    fseek(fp, 0, SEEK_END);
    long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)sz + 1);
    size_t got = fread(buf, 1, (size_t)sz, fp);
    fclose(fp);
    buf[got] = 0;
    objf o;
    memset(&o, 0, sizeof(o));
    /* objparser.cpp:313-351: lines split at '\n', last line without '\n' too */
    char* line = buf;
    char* endp = buf + got;
    while (line < endp) {
        char* eol = (char*)memchr(line, '\n', (size_t)(endp - line));
        if (!eol) {
            obj_line(&o, line);
            break;
        }
        *eol = 0;
        obj_line(&o, line);
        line = eol + 1;
    }
    free(buf);

    /* LoadScene, main.cpp:132-162 */
    v3 bmin = V(+1.0e6f, +1.0e6f, +1.0e6f);
    v3 bmax = V(-1.0e6f, -1.0e6f, -1.0e6f);
    int32_t n = (int32_t)(o.nf / 9);
    float* tris = (float*)malloc((size_t)(n + 2) * 9 * sizeof(float));
    for (int32_t i = 0; i < n; ++i) {
        int idx[3] = {o.f[i * 9 + 0] * 3, o.f[i * 9 + 3] * 3, o.f[i * 9 + 6] * 3};
        for (int k = 0; k < 3; ++k) {
            v3 vv = V(o.v[idx[k] + 0], o.v[idx[k] + 1], o.v[idx[k] + 2]);
            vstore(tris + 9 * i + 3 * k, vv);
        }
        for (int k = 0; k < 3; ++k) {
            v3 vv = vload(tris + 9 * i + 3 * k);
            bmin = vmin(bmin, vv);
            bmax = vmax(bmax, vv);
        }
    }
    v3 size = vsub(bmax, bmin);
    v3 extra = vscale(size, 0.7f);
    float* f0 = tris + 9 * n;
    float* f1 = tris + 9 * (n + 1);
    vstore(f0 + 0, V(bmin.x - extra.x, bmin.y, bmin.z - extra.z));
    vstore(f0 + 3, V(bmin.x - extra.x, bmin.y, bmax.z + extra.z));
    vstore(f0 + 6, V(bmax.x + extra.x, bmin.y, bmin.z - extra.z));
    vstore(f1 + 0, V(bmin.x - extra.x, bmin.y, bmax.z + extra.z));
    vstore(f1 + 3, V(bmax.x + extra.x, bmin.y, bmax.z + extra.z));
    vstore(f1 + 6, V(bmax.x + extra.x, bmin.y, bmin.z - extra.z));
    free(o.v);
    free(o.f);
    *out_tris = tris;
    *out_n = n + 2;
    vstore(out_bmin, bmin);
    vstore(out_bmax, bmax);
    return 0;
}

void orc_free(void* p) { free(p); }
