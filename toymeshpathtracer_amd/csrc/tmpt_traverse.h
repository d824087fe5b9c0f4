// tmpt_traverse.h -- LBVH2 traversal for gfx950: closest hit (Scene::HitScene,
// scene.cpp:128-140) and any hit (the shadow query of Scatter, main.cpp:57-60,
// whose only consumer is the hit/miss bit).
//
// * Scene query contract: result = the reference's closest hit over
//   all triangles with strict '<', i.e. ties go to the lowest triangle index.
//   Box culling is conservative (padded leaf boxes, stretched far distance),
//   so the Moller-Trumbore test alone -- bit-identical to maths.cpp:339-380 --
//   decides every hit.
// * Stack: the first SL entries of each lane live in LDS (layout [depth][lane],
//   so a wave's accesses to one depth hit 64 distinct banks); deeper entries
//   spill to a per-lane global area (never more than kStackTotal in all).
// * Slab test in fma form t = b*inv - o*inv (not bit-exact, only conservative,
//   which is all culling needs), min3/max3 reductions.
#pragma once

#include "tmpt_internal.h"

namespace tmpt {

// 1/d for box culling only (never for a reported value): v_rcp_f32 (1 ulp).
// The slab distances are already off the exact ones by the rounding of o/d
// and of the fma; box padding (kBoxPadRel, ~84 ulp of the coordinates) and
// kTfarSlack absorb both, so culling stays conservative.
__device__ __forceinline__ float safe_inv(float d)
{
    float a = fabsf(d) < 1e-20f ? copysignf(1e-20f, d) : d;
    return __builtin_amdgcn_rcpf(a);
}

struct TravRay {
    f3 o, d;
    float ix, iy, iz;  // 1/d (finite)
    float ox, oy, oz;  // o * inv
    uint32_t offx, offy, offz;  // BVH4F byte offset of the near plane per axis (far = ^16)
};

__device__ __forceinline__ TravRay make_trav_ray(f3 o, f3 d)
{
    TravRay r;
    r.o = o;
    r.d = d;
    r.ix = safe_inv(d.x);
    r.iy = safe_inv(d.y);
    r.iz = safe_inv(d.z);
    r.ox = o.x * r.ix;
    r.oy = o.y * r.iy;
    r.oz = o.z * r.iz;
    // 1/d > 0: the lo plane is entered first; < 0: the hi plane (never 0: safe_inv)
    r.offx = signbit(r.ix) ? 16u : 0u;
    r.offy = signbit(r.iy) ? 48u : 32u;
    r.offz = signbit(r.iz) ? 80u : 64u;
    return r;
}

__device__ __forceinline__ float min3f(float a, float b, float c) { return fminf(fminf(a, b), c); }
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// entry distance of a box, or +inf-like rejection via the returned flag
__device__ __forceinline__ bool slab(const TravRay& r, float lx, float ly, float lz, float hx,
                                     float hy, float hz, float tlo, float tmax, float& tnear)
{
    float t0x = __builtin_fmaf(lx, r.ix, -r.ox), t1x = __builtin_fmaf(hx, r.ix, -r.ox);
    float t0y = __builtin_fmaf(ly, r.iy, -r.oy), t1y = __builtin_fmaf(hy, r.iy, -r.oy);
    float t0z = __builtin_fmaf(lz, r.iz, -r.oz), t1z = __builtin_fmaf(hz, r.iz, -r.oz);
    float tn = max3f(fminf(t0x, t1x), fminf(t0y, t1y), fmaxf(fminf(t0z, t1z), tlo));
    float tf = min3f(fmaxf(t0x, t1x), fmaxf(t0y, t1y), fminf(fmaxf(t0z, t1z), tmax));
    tnear = tn;
    return tn <= tf * kTfarSlack;
}

// Pins a loaded triangle record's used words in registers at this point (no
// instruction emitted), so the compiler cannot sink their loads into the
// branches that consume them.
__device__ __forceinline__ void materialize(float4& a, float4& b, float4& c)
{
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z),
                 "+v"(b.w), "+v"(c.x), "+v"(c.y));
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;

// Per-lane traversal stack: the top SL entries in LDS ([depth][lane], a wave's
// access to one depth hits 64 banks), deeper ones in a per-lane global area.
// The LDS pointer is address-space-3 typed so the compiler emits ds_read /
// ds_write; a generic pointer let it merge the two pop paths into one FLAT
// load, which goes through the vector-memory address unit (TA) like a global
// load -- one extra TA slot per traversal step.
template <int BLOCK, int SL>
struct TravStack {
    lds_u32* lds;    // &s_stack[threadIdx.x]; entry k at lds[k * BLOCK]
    uint32_t* glob;  // kStackTotal - SL entries of this lane
    const lds_u4* top = nullptr;  // LDS copy of BVH4 nodes [0, ntop) (FMT 4), 4 uint4 each
    uint32_t ntop = 0;
    __device__ __forceinline__ TravStack(uint32_t* l, uint32_t* g) : lds((lds_u32*)l), glob(g) {}
    __device__ __forceinline__ void push(int& sp, int v)
    {
        if (SL >= kStackTotal || sp < SL) lds[sp * BLOCK] = (uint32_t)v;
        else glob[sp - SL] = (uint32_t)v;
        ++sp;
    }
    // Up to three pushes (c0 first, c2 last = popped first), branch-free while
    // the LDS part has room for three: the valid ones are compacted into
    // consecutive slots by selects and all three slots are written (slots
    // above the new depth are free, so the extra writes are harmless).
    __device__ __forceinline__ void push3(int& sp, bool v0, int c0, bool v1, int c1, bool v2, int c2)
    {
        if (sp + 3 <= SL) {
            const int s0 = v0 ? c0 : (v1 ? c1 : c2);
            const int s1 = (v0 && v1) ? c1 : c2;
            lds[sp * BLOCK] = (uint32_t)s0;
            lds[(sp + 1) * BLOCK] = (uint32_t)s1;
            lds[(sp + 2) * BLOCK] = (uint32_t)c2;
            sp += (int)v0 + (int)v1 + (int)v2;
        } else {
            if (v0) push(sp, c0);
            if (v1) push(sp, c1);
            if (v2) push(sp, c2);
        }
    }
    __device__ __forceinline__ int pop(int& sp)
    {
        --sp;
        if (SL >= kStackTotal) return (int)lds[sp * BLOCK];
        uint32_t v = lds[min(sp, SL - 1) * BLOCK];
        if (sp >= SL) v = glob[sp - SL];
        return (int)v;
    }
};

struct SceneView {
    const BvhNode* __restrict__ nodes;
    const Bvh4Node* __restrict__ nodes4;
    const char* __restrict__ nodes4f;  // Bvh4FNode array, addressed by byte offset
    const TriPre* __restrict__ tri_pre;
    const TriOrig* __restrict__ tri_orig;
    int32_t n;
    ShadowGrid sg;  // by value: axes, origin, scale, device arrays (R = 0: none)
    int32_t n_nodes4 = 0;
};

struct TravCount {
    uint32_t nodes = 0, tris = 0;
};

// Resumable traversal state of one lane (registers).
struct TravState {
    int node;   // next node (>=0 internal, <0 leaf = ~slot)
    int sp;     // stack depth
    int best;   // original triangle index of the current closest hit, -1 if none
    float bt, bu, bv;
};

__device__ __forceinline__ void trav_init(TravState& ts, float tmax)
{
    ts.node = 0;
    ts.sp = 0;
    ts.best = -1;
    ts.bt = tmax;
    ts.bu = ts.bv = 0.0f;
}

// One traversal step: one internal node (both child boxes) or one leaf
// triangle.  Returns true when the query is finished (stack empty, or the
// first accepted hit of an any-hit query).
template <bool ANY, bool COUNT, int BLOCK, int SL>
__device__ __forceinline__ bool trav_step(const SceneView& sv, const TravRay& r, float tlo,
                                          float tmin, float tmax, TravState& ts,
                                          TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    if (ts.node >= 0) {
        const float4* p = reinterpret_cast<const float4*>(sv.nodes + ts.node);
        float4 a = p[0], b = p[1], c = p[2];
        int4 lk = reinterpret_cast<const int4*>(p)[3];
        if (COUNT) ++cnt.nodes;
        float tn0, tn1;
        bool h0 = slab(r, a.x, a.y, a.z, a.w, b.x, b.y, tlo, ts.bt, tn0);
        bool h1 = slab(r, b.z, b.w, c.x, c.y, c.z, c.w, tlo, ts.bt, tn1);
        if (h0 && h1) {
            int nearc = lk.x, farc = lk.y;
            if (tn1 < tn0) { nearc = lk.y; farc = lk.x; }
            st.push(ts.sp, farc);
            ts.node = nearc;
            return false;
        }
        if (h0 || h1) {
            ts.node = h0 ? lk.x : lk.y;
            return false;
        }
    } else {
        const float4* p = reinterpret_cast<const float4*>(sv.tri_pre + (~ts.node));
        float4 a = p[0], b = p[1], c = p[2];
        if (COUNT) ++cnt.tris;
        float t, u, v;
        if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), tmin, tmax,
                    t, u, v)) {
            int id = __float_as_int(c.y);
            if (t < ts.bt || (t == ts.bt && ts.best >= 0 && id < ts.best)) {
                ts.bt = t;
                ts.bu = u;
                ts.bv = v;
                ts.best = id;
                if (ANY) return true;
            }
        }
    }
    if (ts.sp == 0) return true;
    ts.node = st.pop(ts.sp);
    return false;
}

// 2^e for the signed exponent byte e of a BVH4Q node (bits 0-7 of `b`)
__device__ __forceinline__ float exp_scale(uint32_t b) { return __uint_as_float((uint32_t)((int)(int8_t)(b & 0xFFu) + 127) << 23); }
// x * 2^e for the signed exponent byte e at bit `sh` of w: v_bfe_i32 + v_ldexp_f32,
// exact (a power-of-two scaling, no under/overflow for the 1/d of a unit direction)
__device__ __forceinline__ float exp_mul(float x, uint32_t w, int sh)
{
    return __builtin_amdgcn_ldexpf(x, (int)__builtin_amdgcn_sbfe(w, sh, 8));
}

template <bool ANY, bool COUNT>
__device__ __forceinline__ bool leaf_tris(const SceneView& sv, const TravRay& r, float tmin,
                                          float tmax, TravState& ts, uint32_t code,
                                          TravCount& cnt)
{
    const uint32_t first = code & kLeafFirstMask;
    const uint32_t n = ((code >> kLeafCountShift) & 15u) + 1u;
    for (uint32_t k = 0; k < n; ++k) {
        const float4* p = reinterpret_cast<const float4*>(sv.tri_pre + first + k);
        float4 a = p[0], b = p[1], c = p[2];
        if (COUNT) ++cnt.tris;
        float t, u, v;
        if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), tmin, tmax,
                    t, u, v)) {
            int id = __float_as_int(c.y);
            if (t < ts.bt || (t == ts.bt && ts.best >= 0 && id < ts.best)) {
                ts.bt = t;
                ts.bu = u;
                ts.bv = v;
                ts.best = id;
                if (ANY) return true;
            }
        }
    }
    return false;
}

// One step over the 4-wide quantised BVH: one node (four child boxes decoded
// as origin + q*2^e, slab distances t = q*(2^e/d) + (origin-o)/d, one fma per
// plane) or one leaf (its triangle range).  Closest hit: hit children sorted
// near to far (5-exchange network), nearest taken, others pushed far first.
template <bool ANY, bool COUNT, int BLOCK, int SL, bool SORT = !ANY>
__device__ __forceinline__ bool trav_step4(const SceneView& sv, const TravRay& r, float tlo,
                                           float tmin, float tmax, TravState& ts,
                                           TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    if (ts.node >= 0) {
        const uint4* p = reinterpret_cast<const uint4*>(sv.nodes4 + ts.node);
        uint4 A = p[0], B = p[1], C = p[2];
        int4 L = reinterpret_cast<const int4*>(p)[3];
        if (COUNT) ++cnt.nodes;
        const float ax = exp_scale(A.w) * r.ix, bx = (__uint_as_float(A.x) - r.o.x) * r.ix;
        const float ay = exp_scale(A.w >> 8) * r.iy, by = (__uint_as_float(A.y) - r.o.y) * r.iy;
        const float az = exp_scale(A.w >> 16) * r.iz, bz = (__uint_as_float(A.z) - r.o.z) * r.iz;
        const uint32_t mask = A.w >> 24;
        float key[4];
        int ch[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sh = 8 * k;
            float t0x = __builtin_fmaf((float)((B.x >> sh) & 255u), ax, bx);
            float t1x = __builtin_fmaf((float)((B.y >> sh) & 255u), ax, bx);
            float t0y = __builtin_fmaf((float)((B.z >> sh) & 255u), ay, by);
            float t1y = __builtin_fmaf((float)((B.w >> sh) & 255u), ay, by);
            float t0z = __builtin_fmaf((float)((C.x >> sh) & 255u), az, bz);
            float t1z = __builtin_fmaf((float)((C.y >> sh) & 255u), az, bz);
            float tn = max3f(fminf(t0x, t1x), fminf(t0y, t1y), fmaxf(fminf(t0z, t1z), tlo));
            float tf = min3f(fmaxf(t0x, t1x), fmaxf(t0y, t1y), fminf(fmaxf(t0z, t1z), ts.bt));
            bool hit = ((mask >> k) & 1u) && tn <= tf * kTfarSlack;
            key[k] = hit ? tn : INFINITY;
        }
        int nh = (key[0] != INFINITY) + (key[1] != INFINITY) + (key[2] != INFINITY) +
                 (key[3] != INFINITY);
        if (nh > 0) {
            if (SORT) {
#define TMPT_CSWAP(i, j)                                            \
    if (key[j] < key[i]) {                                          \
        float tk = key[i]; key[i] = key[j]; key[j] = tk;             \
        int tc = ch[i]; ch[i] = ch[j]; ch[j] = tc;                   \
    }
                TMPT_CSWAP(0, 1) TMPT_CSWAP(2, 3) TMPT_CSWAP(0, 2) TMPT_CSWAP(1, 3) TMPT_CSWAP(1, 2)
#undef TMPT_CSWAP
                // hits now occupy 0..nh-1, nearest first
                if (nh > 3) st.push(ts.sp, ch[3]);
                if (nh > 2) st.push(ts.sp, ch[2]);
                if (nh > 1) st.push(ts.sp, ch[1]);
                ts.node = ch[0];
            } else {
                int next = 0;
                bool have = false;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (key[k] != INFINITY) {
                        if (!have) {
                            next = ch[k];
                            have = true;
                        } else {
                            st.push(ts.sp, ch[k]);
                        }
                    }
                }
                ts.node = next;
            }
            return false;
        }
    } else {
        if (leaf_tris<ANY, COUNT>(sv, r, tmin, tmax, ts, (uint32_t)ts.node, cnt)) return true;
    }
    if (ts.sp == 0) return true;
    ts.node = st.pop(ts.sp);
    return false;
}

// Same step with the query kind chosen per lane at run time (the persistent
// path engine mixes closest-hit and shadow queries in one wave): children are
// always visited near to far; a shadow query stops at its first accepted hit.
template <bool COUNT, int BLOCK, int SL>
__device__ __forceinline__ bool trav_step4_mixed(const SceneView& sv, const TravRay& r, bool any,
                                                 TravState& ts, TravStack<BLOCK, SL>& st,
                                                 TravCount& cnt)
{
    if (ts.node >= 0) {
        const uint4* p = reinterpret_cast<const uint4*>(sv.nodes4 + ts.node);
        uint4 A = p[0], B = p[1], C = p[2];
        int4 L = reinterpret_cast<const int4*>(p)[3];
        if (COUNT) ++cnt.nodes;
        const float ax = exp_scale(A.w) * r.ix, bx = (__uint_as_float(A.x) - r.o.x) * r.ix;
        const float ay = exp_scale(A.w >> 8) * r.iy, by = (__uint_as_float(A.y) - r.o.y) * r.iy;
        const float az = exp_scale(A.w >> 16) * r.iz, bz = (__uint_as_float(A.z) - r.o.z) * r.iz;
        const uint32_t mask = A.w >> 24;
        float key[4];
        int ch[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sh = 8 * k;
            float t0x = __builtin_fmaf((float)((B.x >> sh) & 255u), ax, bx);
            float t1x = __builtin_fmaf((float)((B.y >> sh) & 255u), ax, bx);
            float t0y = __builtin_fmaf((float)((B.z >> sh) & 255u), ay, by);
            float t1y = __builtin_fmaf((float)((B.w >> sh) & 255u), ay, by);
            float t0z = __builtin_fmaf((float)((C.x >> sh) & 255u), az, bz);
            float t1z = __builtin_fmaf((float)((C.y >> sh) & 255u), az, bz);
            float tn = max3f(fminf(t0x, t1x), fminf(t0y, t1y), fmaxf(fminf(t0z, t1z), 0.0f));
            float tf = min3f(fmaxf(t0x, t1x), fmaxf(t0y, t1y), fminf(fmaxf(t0z, t1z), ts.bt));
            bool hit = ((mask >> k) & 1u) && tn <= tf * kTfarSlack;
            key[k] = hit ? tn : INFINITY;
        }
        int nh = (key[0] != INFINITY) + (key[1] != INFINITY) + (key[2] != INFINITY) +
                 (key[3] != INFINITY);
        if (nh > 0) {
#define TMPT_CSWAP(i, j)                                            \
    if (key[j] < key[i]) {                                          \
        float tk = key[i]; key[i] = key[j]; key[j] = tk;             \
        int tc = ch[i]; ch[i] = ch[j]; ch[j] = tc;                   \
    }
            TMPT_CSWAP(0, 1) TMPT_CSWAP(2, 3) TMPT_CSWAP(0, 2) TMPT_CSWAP(1, 3) TMPT_CSWAP(1, 2)
#undef TMPT_CSWAP
            if (nh > 3) st.push(ts.sp, ch[3]);
            if (nh > 2) st.push(ts.sp, ch[2]);
            if (nh > 1) st.push(ts.sp, ch[1]);
            ts.node = ch[0];
            return false;
        }
    } else {
        const uint32_t code = (uint32_t)ts.node;
        const uint32_t first = code & kLeafFirstMask;
        const uint32_t n = ((code >> kLeafCountShift) & 15u) + 1u;
        for (uint32_t k = 0; k < n; ++k) {
            const float4* p = reinterpret_cast<const float4*>(sv.tri_pre + first + k);
            float4 a = p[0], b = p[1], c = p[2];
            if (COUNT) ++cnt.tris;
            float t, u, v;
            if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), kMinT, kMaxT,
                        t, u, v)) {
                int id = __float_as_int(c.y);
                if (t < ts.bt || (t == ts.bt && ts.best >= 0 && id < ts.best)) {
                    ts.bt = t;
                    ts.bu = u;
                    ts.bv = v;
                    ts.best = id;
                    if (any) return true;
                }
            }
        }
    }
    if (ts.sp == 0) return true;
    ts.node = st.pop(ts.sp);
    return false;
}

typedef float v2f __attribute__((ext_vector_type(2)));

// One step over BVH4F (f32 child boxes): near/far planes chosen by the ray's
// octant (byte offsets), slab distances by packed fma over child pairs, so a
// node costs 12 v_pk_fma + 4 compares per child instead of per-child unpacking
// and min/max.  The same children, links, order and leaf handling as
// trav_step4_mixed; boxes are the unquantised padded boxes (tighter).
template <bool COUNT, int BLOCK, int SL>
__device__ __forceinline__ bool trav_step4f_mixed(const SceneView& sv, const TravRay& r, bool any,
                                                  TravState& ts, TravStack<BLOCK, SL>& st,
                                                  TravCount& cnt)
{
    if (ts.node >= 0) {
        const uint32_t nb = (uint32_t)ts.node << 7;
        const char* base = sv.nodes4f;
        const float4 nx = *reinterpret_cast<const float4*>(base + (nb | r.offx));
        const float4 fx = *reinterpret_cast<const float4*>(base + (nb | (r.offx ^ 16u)));
        const float4 ny = *reinterpret_cast<const float4*>(base + (nb | r.offy));
        const float4 fy = *reinterpret_cast<const float4*>(base + (nb | (r.offy ^ 16u)));
        const float4 nz = *reinterpret_cast<const float4*>(base + (nb | r.offz));
        const float4 fz = *reinterpret_cast<const float4*>(base + (nb | (r.offz ^ 16u)));
        const int4 L = *reinterpret_cast<const int4*>(base + (nb | 96u));
        if (COUNT) ++cnt.nodes;
        const v2f ix = {r.ix, r.ix}, iy = {r.iy, r.iy}, iz = {r.iz, r.iz};
        const v2f ox = {-r.ox, -r.ox}, oy = {-r.oy, -r.oy}, oz = {-r.oz, -r.oz};
#define TMPT_PL(V, I, O, lo2, hi2)                                                   \
        const v2f lo2 = __builtin_elementwise_fma((v2f){V.x, V.y}, I, O);               \
        const v2f hi2 = __builtin_elementwise_fma((v2f){V.z, V.w}, I, O);
        TMPT_PL(nx, ix, ox, nx01, nx23)
        TMPT_PL(fx, ix, ox, fx01, fx23)
        TMPT_PL(ny, iy, oy, ny01, ny23)
        TMPT_PL(fy, iy, oy, fy01, fy23)
        TMPT_PL(nz, iz, oz, nz01, nz23)
        TMPT_PL(fz, iz, oz, fz01, fz23)
#undef TMPT_PL
        const float tnear[4] = {nx01.x, nx01.y, nx23.x, nx23.y};
        const float tnear_y[4] = {ny01.x, ny01.y, ny23.x, ny23.y};
        const float tnear_z[4] = {nz01.x, nz01.y, nz23.x, nz23.y};
        const float tfar[4] = {fx01.x, fx01.y, fx23.x, fx23.y};
        const float tfar_y[4] = {fy01.x, fy01.y, fy23.x, fy23.y};
        const float tfar_z[4] = {fz01.x, fz01.y, fz23.x, fz23.y};
        float key[4];
        int ch[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float tn = fmaxf(fmaxf(tnear[k], tnear_y[k]), fmaxf(tnear_z[k], 0.0f));
            float tf = fminf(fminf(tfar[k], tfar_y[k]), fminf(tfar_z[k], ts.bt));
            key[k] = tn <= tf * kTfarSlack ? tn : INFINITY;
        }
        int nh = (key[0] != INFINITY) + (key[1] != INFINITY) + (key[2] != INFINITY) +
                 (key[3] != INFINITY);
        if (nh > 0) {
#define TMPT_CSWAP(i, j)                                            \
    if (key[j] < key[i]) {                                          \
        float tk = key[i]; key[i] = key[j]; key[j] = tk;             \
        int tc = ch[i]; ch[i] = ch[j]; ch[j] = tc;                   \
    }
            TMPT_CSWAP(0, 1) TMPT_CSWAP(2, 3) TMPT_CSWAP(0, 2) TMPT_CSWAP(1, 3) TMPT_CSWAP(1, 2)
#undef TMPT_CSWAP
            if (nh > 3) st.push(ts.sp, ch[3]);
            if (nh > 2) st.push(ts.sp, ch[2]);
            if (nh > 1) st.push(ts.sp, ch[1]);
            ts.node = ch[0];
            return false;
        }
    } else {
        const uint32_t code = (uint32_t)ts.node;
        const uint32_t first = code & kLeafFirstMask;
        const uint32_t n = ((code >> kLeafCountShift) & 15u) + 1u;
        for (uint32_t k = 0; k < n; ++k) {
            const float4* p = reinterpret_cast<const float4*>(sv.tri_pre + first + k);
            float4 a = p[0], b = p[1], c = p[2];
            if (COUNT) ++cnt.tris;
            float t, u, v;
            if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), kMinT, kMaxT,
                        t, u, v)) {
                int id = __float_as_int(c.y);
                if (t < ts.bt || (t == ts.bt && ts.best >= 0 && id < ts.best)) {
                    ts.bt = t;
                    ts.bu = u;
                    ts.bv = v;
                    ts.best = id;
                    if (any) return true;
                }
            }
        }
    }
    if (ts.sp == 0) return true;
    ts.node = st.pop(ts.sp);
    return false;
}

// One step over BVH4Q (64-B quantised nodes) with the BVH4F step's decoding:
// near/far byte planes picked per axis by the ray's octant (one v_cndmask per
// plane dword), t = q * (2^e/d) + fma(origin, 1/d, -o/d) by packed fma over
// child pairs, no per-child min/max and no mask test (empty slots carry an
// inverted box and link to the null leaf).  4 loads per node (the TA cost of a
// divergent gather scales with bytes per lane) at ~BVH4F's VALU count.
template <bool COUNT, int BLOCK, int SL, int SORTK = 0, bool TOPC = false, int KIND = 0>
__device__ __forceinline__ bool trav_step4q2_mixed(const SceneView& sv, const TravRay& r, bool any,
                                                   TravState& ts, TravStack<BLOCK, SL>& st,
                                                   TravCount& cnt)
{
    // KIND 1 / 2: the caller guarantees the lane is at a node / at a leaf (a
    // voted round), so the other kind's code is not emitted at all
    if (KIND == 1 || (KIND == 0 && ts.node >= 0)) {
        // 32-bit byte offset off an SGPR base: one VALU for the address
        uint4 A, B, C;
        int4 L;
        if (!TOPC || (uint32_t)ts.node >= st.ntop) {
            const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(sv.nodes4) +
                                                            ((uint32_t)ts.node << 6));
            A = p[0], B = p[1], C = p[2];
            L = reinterpret_cast<const int4*>(p)[3];
        } else {  // top levels: the block's LDS copy
            const lds_u4* q = st.top + ((uint32_t)ts.node << 2);
            const u32x4 a4 = q[0], b4 = q[1], c4 = q[2], l4 = q[3];
            A = make_uint4(a4.x, a4.y, a4.z, a4.w);
            B = make_uint4(b4.x, b4.y, b4.z, b4.w);
            C = make_uint4(c4.x, c4.y, c4.z, c4.w);
            L = make_int4((int)l4.x, (int)l4.y, (int)l4.z, (int)l4.w);
        }
        if (COUNT) ++cnt.nodes;
        const float sx = exp_mul(r.ix, A.w, 0), sy = exp_mul(r.iy, A.w, 8), sz = exp_mul(r.iz, A.w, 16);
        const float bx = __builtin_fmaf(__uint_as_float(A.x), r.ix, -r.ox);
        const float by = __builtin_fmaf(__uint_as_float(A.y), r.iy, -r.oy);
        const float bz = __builtin_fmaf(__uint_as_float(A.z), r.iz, -r.oz);
        const bool ngx = r.offx != 0u, ngy = r.offy != 32u, ngz = r.offz != 64u;
        const uint32_t qnx = ngx ? B.y : B.x, qfx = ngx ? B.x : B.y;
        const uint32_t qny = ngy ? B.w : B.z, qfy = ngy ? B.z : B.w;
        const uint32_t qnz = ngz ? C.y : C.x, qfz = ngz ? C.x : C.y;
        const v2f s2x = {sx, sx}, s2y = {sy, sy}, s2z = {sz, sz};
        const v2f b2x = {bx, bx}, b2y = {by, by}, b2z = {bz, bz};
#define TMPT_QB(Q, k) (float)(((Q) >> (8 * (k))) & 255u)
#define TMPT_QP(Q, S, Bv, lo2, hi2)                                                              \
        const v2f lo2 = __builtin_elementwise_fma((v2f){TMPT_QB(Q, 0), TMPT_QB(Q, 1)}, S, Bv);     \
        const v2f hi2 = __builtin_elementwise_fma((v2f){TMPT_QB(Q, 2), TMPT_QB(Q, 3)}, S, Bv);
        TMPT_QP(qnx, s2x, b2x, nx01, nx23)
        TMPT_QP(qfx, s2x, b2x, fx01, fx23)
        TMPT_QP(qny, s2y, b2y, ny01, ny23)
        TMPT_QP(qfy, s2y, b2y, fy01, fy23)
        TMPT_QP(qnz, s2z, b2z, nz01, nz23)
        TMPT_QP(qfz, s2z, b2z, fz01, fz23)
#undef TMPT_QP
#undef TMPT_QB
        const float tnx[4] = {nx01.x, nx01.y, nx23.x, nx23.y};
        const float tny[4] = {ny01.x, ny01.y, ny23.x, ny23.y};
        const float tnz[4] = {nz01.x, nz01.y, nz23.x, nz23.y};
        const float tfx[4] = {fx01.x, fx01.y, fx23.x, fx23.y};
        const float tfy[4] = {fy01.x, fy01.y, fy23.x, fy23.y};
        const float tfz[4] = {fz01.x, fz01.y, fz23.x, fz23.y};
        float key[4];
        int ch[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float tn = fmaxf(fmaxf(tnx[k], tny[k]), fmaxf(tnz[k], 0.0f));
            float tf = fminf(fminf(tfx[k], tfy[k]), fminf(tfz[k], ts.bt));
            key[k] = tn <= tf * kTfarSlack ? tn : INFINITY;
        }
        if (SORTK == 0) {  // all hit children near to far (misses sort last as +inf)
#define TMPT_CSWAP(i, j)                                            \
    if (key[j] < key[i]) {                                          \
        float tk = key[i]; key[i] = key[j]; key[j] = tk;             \
        int tc = ch[i]; ch[i] = ch[j]; ch[j] = tc;                   \
    }
            TMPT_CSWAP(0, 1) TMPT_CSWAP(2, 3) TMPT_CSWAP(0, 2) TMPT_CSWAP(1, 3) TMPT_CSWAP(1, 2)
#undef TMPT_CSWAP
            if (key[0] != INFINITY) {
                if (key[3] != INFINITY) st.push(ts.sp, ch[3]);
                if (key[2] != INFINITY) st.push(ts.sp, ch[2]);
                if (key[1] != INFINITY) st.push(ts.sp, ch[1]);
                ts.node = ch[0];
                return false;
            }
        } else {  // nearest child next; the others pushed pairwise-ordered only
            const bool s01 = key[1] < key[0], s23 = key[3] < key[2];
            const float ka = s01 ? key[1] : key[0], kao = s01 ? key[0] : key[1];
            const int ca = s01 ? ch[1] : ch[0], cao = s01 ? ch[0] : ch[1];
            const float kb = s23 ? key[3] : key[2], kbo = s23 ? key[2] : key[3];
            const int cb = s23 ? ch[3] : ch[2], cbo = s23 ? ch[2] : ch[3];
            const bool sab = kb < ka;
            const float kn = sab ? kb : ka, kno = sab ? ka : kb;
            const int cn = sab ? cb : ca, cno = sab ? ca : cb;
            if (kn != INFINITY) {
                st.push3(ts.sp, kbo != INFINITY, cbo, kao != INFINITY, cao, kno != INFINITY, cno);
                ts.node = cn;
                return false;
            }
        }
    }
    if (KIND == 2 || (KIND == 0 && ts.node < 0)) {
        const uint32_t code = (uint32_t)ts.node;
        const uint32_t first = code & kLeafFirstMask;
        const uint32_t n = ((code >> kLeafCountShift) & 15u) + 1u;
        const char* base = reinterpret_cast<const char*>(sv.tri_pre);
        // Accepts (t, u, v, id) by the closest-hit order; true = any-hit query done.
        auto tri = [&](const float4& a, const float4& b, const float4& c) -> bool {
            if (COUNT) ++cnt.tris;
            float t, u, v;
            if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), kMinT, kMaxT,
                        t, u, v)) {
                int id = __float_as_int(c.y);
                if (t < ts.bt || (t == ts.bt && ts.best >= 0 && id < ts.best)) {
                    ts.bt = t;
                    ts.bu = u;
                    ts.bv = v;
                    ts.best = id;
                    if (any) return true;
                }
            }
            return false;
        };
        // Both triangles of a (typical) 2-triangle leaf are loaded at once, all
        // 40 B each, before any test: left alone the compiler sinks the vertex
        // load behind the determinant test and the second triangle's loads
        // behind the first's, three dependent memory latencies per leaf step.
        const float4* p0 = reinterpret_cast<const float4*>(base + first * (uint32_t)sizeof(TriPre));
        const float4* p1 = reinterpret_cast<const float4*>(base + (first + (n > 1u ? 1u : 0u)) *
                                                                       (uint32_t)sizeof(TriPre));
        float4 a0 = p0[0], b0 = p0[1], c0 = p0[2];
        float4 a1 = p1[0], b1 = p1[1], c1 = p1[2];
        materialize(a0, b0, c0);
        materialize(a1, b1, c1);
        if (KIND == 2) {
            // voted leaf round: both tests without early exits (the two
            // dependency chains interleave), then the closest-hit order
            // (triangle 0 first; an any-hit query stops at the first accept)
            float t0, u0, w0, t1, u1, w1;
            if (COUNT) cnt.tris += n > 1u ? 2u : 1u;
            const bool ok0 = mt_test_flat(r.o, r.d, mk(a0.x, a0.y, a0.z), mk(a0.w, b0.x, b0.y),
                                          mk(b0.z, b0.w, c0.x), kMinT, kMaxT, t0, u0, w0);
            const bool ok1 = mt_test_flat(r.o, r.d, mk(a1.x, a1.y, a1.z), mk(a1.w, b1.x, b1.y),
                                          mk(b1.z, b1.w, c1.x), kMinT, kMaxT, t1, u1, w1) &&
                             n > 1u;
            const int id0 = __float_as_int(c0.y), id1 = __float_as_int(c1.y);
            const bool acc0 = ok0 && (t0 < ts.bt || (t0 == ts.bt && ts.best >= 0 && id0 < ts.best));
            ts.bt = acc0 ? t0 : ts.bt;
            ts.bu = acc0 ? u0 : ts.bu;
            ts.bv = acc0 ? w0 : ts.bv;
            ts.best = acc0 ? id0 : ts.best;
            const bool acc1 = ok1 && !(any && acc0) &&
                              (t1 < ts.bt || (t1 == ts.bt && ts.best >= 0 && id1 < ts.best));
            ts.bt = acc1 ? t1 : ts.bt;
            ts.bu = acc1 ? u1 : ts.bu;
            ts.bv = acc1 ? w1 : ts.bv;
            ts.best = acc1 ? id1 : ts.best;
            if (any && (acc0 || acc1)) return true;
        } else {  // a lone lane (row chains) gains more from the early exits
            if (tri(a0, b0, c0)) return true;
            if (n > 1u && tri(a1, b1, c1)) return true;
        }
        for (uint32_t k = 2; k < n; ++k) {
            const float4* p = reinterpret_cast<const float4*>(base + (first + k) * (uint32_t)sizeof(TriPre));
            if (tri(p[0], p[1], p[2])) return true;
        }
        if (KIND == 2 && ts.sp <= SL) {  // branch-free pop from the LDS part
            const uint32_t top = st.lds[(uint32_t)max(ts.sp - 1, 0) * BLOCK];
            const bool done = ts.sp == 0;
            ts.node = (int)top;
            ts.sp -= done ? 0 : 1;
            return done;
        }
    }
    if (ts.sp == 0) return true;
    ts.node = st.pop(ts.sp);
    return false;
}

// node format of the persistent engine: 0 = BVH4Q (mask + min/max decode),
// 1 = BVH4F (f32 boxes), 2 = BVH4Q with octant decode
template <int FMT, bool COUNT, int BLOCK, int SL>
__device__ __forceinline__ bool trav_step_fmt(const SceneView& sv, const TravRay& r, bool any,
                                              TravState& ts, TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    if (FMT == 1) return trav_step4f_mixed<COUNT>(sv, r, any, ts, st, cnt);
    if (FMT == 2) return trav_step4q2_mixed<COUNT, BLOCK, SL, 0>(sv, r, any, ts, st, cnt);
    if (FMT == 3) return trav_step4q2_mixed<COUNT, BLOCK, SL, 1>(sv, r, any, ts, st, cnt);
    if (FMT == 4) return trav_step4q2_mixed<COUNT, BLOCK, SL, 1, true>(sv, r, any, ts, st, cnt);
    return trav_step4_mixed<COUNT>(sv, r, any, ts, st, cnt);
}

template <bool WIDE, bool ANY, bool COUNT, int BLOCK, int SL, bool SORT = !ANY>
__device__ __forceinline__ bool trav_step_w(const SceneView& sv, const TravRay& r, float tlo,
                                            float tmin, float tmax, TravState& ts,
                                            TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    if (WIDE) return trav_step4<ANY, COUNT, BLOCK, SL, SORT>(sv, r, tlo, tmin, tmax, ts, st, cnt);
    return trav_step<ANY, COUNT>(sv, r, tlo, tmin, tmax, ts, st, cnt);
}

// A ray with a NaN in its origin or direction can never be accepted by
// Moller-Trumbore (det, u, v and t all become NaN and every comparison of
// maths.cpp:345-371 is false), so the reference's HitScene returns -1 for it.
// It arises when normalize(target - pos) meets a zero vector (main.cpp:72:
// the random unit vector exactly cancels the normal).  Traversing it would
// visit every node (NaN slab distances never cull), so it is answered as a
// miss up front; it still counts as a ray.
__device__ __forceinline__ bool ray_has_nan(f3 o, f3 d)
{
    return __builtin_isnan(o.x) | __builtin_isnan(o.y) | __builtin_isnan(o.z) | __builtin_isnan(d.x) |
           __builtin_isnan(d.y) | __builtin_isnan(d.z);
}

// Shadow query through the light-space grid (tmpt_shadow.hip): is some
// triangle hit by (p, light_dir()) with t in [kMinT, kMaxT]?  One cell, a
// binary search past the triangles that end below p along L, then the
// bit-exact Moller-Trumbore test in order until one accepts.  Returns the
// original triangle index of that hit or -1 (t, u, v of the hit).
__device__ __forceinline__ int shadow_grid_hit(const SceneView& sv, f3 p, f3 ldir, float& t, float& u,
                                               float& v)
{
    const ShadowGrid& g = sv.sg;
    const float pu = p.x * g.U[0] + p.y * g.U[1] + p.z * g.U[2];
    const float pv = p.x * g.V[0] + p.y * g.V[1] + p.z * g.V[2];
    const float fu = (pu - g.u0) * g.inv_cu, fv = (pv - g.v0) * g.inv_cv;
    // outside the padded projection of every triangle (or NaN): nothing to hit
    if (!(fu >= 0.0f && fu < (float)g.R && fv >= 0.0f && fv < (float)g.R)) return -1;
    const uint32_t c = (uint32_t)(int)fv * (uint32_t)g.R + (uint32_t)(int)fu;
    uint32_t lo = g.start[c];
    const uint32_t end = g.start[c + 1];
    // a hit at t >= kMinT reaches dot(p, L) + kMinT up L; the margin covers
    // float rounding of dot(p, L) and of Moller-Trumbore's t
    const float dl = p.x * ldir.x + p.y * ldir.y + p.z * ldir.z;
    const float thr = dl + kMinT - 1e-4f * (1.0f + fabsf(dl));
    uint32_t hi = end;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (g.tmax[m] < thr) lo = m + 1;
        else hi = m;
    }
    for (uint32_t k = lo; k < end; ++k) {
        const float4* q = reinterpret_cast<const float4*>(sv.tri_pre + g.slot[k]);
        const float4 a = q[0], b = q[1], cc = q[2];
        if (mt_test(p, ldir, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, cc.x), kMinT, kMaxT, t, u, v))
            return __float_as_int(cc.y);
    }
    return -1;
}

// The shadow-grid cell of a shadow ray's origin as a tri_pre range
// {first, count} (count 0: no triangle can be hit).
__device__ __forceinline__ uint2 shadow_grid_cell(const SceneView& sv, f3 p)
{
    const ShadowGrid& g = sv.sg;
    const float pu = p.x * g.U[0] + p.y * g.U[1] + p.z * g.U[2];
    const float pv = p.x * g.V[0] + p.y * g.V[1] + p.z * g.V[2];
    const float fu = (pu - g.u0) * g.inv_cu, fv = (pv - g.v0) * g.inv_cv;
    if (!(fu >= 0.0f && fu < (float)g.R && fv >= 0.0f && fv < (float)g.R)) return make_uint2(0u, 0u);
    return g.cell[(uint32_t)(int)fv * (uint32_t)g.R + (uint32_t)(int)fu];
}

// Whole query in one call.  Returns the original triangle index or -1.
template <bool WIDE, bool ANY, bool COUNT, int BLOCK, int SL>
__device__ __forceinline__ int traverse(const SceneView& sv, const TravRay& r, float tmin,
                                        float tmax, float& bt, float& bu, float& bv,
                                        TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    TravState ts;
    trav_init(ts, tmax);
    if (sv.n > 0 && !ray_has_nan(r.o, r.d)) {
        const float tlo = fminf(tmin, 0.0f);
        while (!trav_step_w<WIDE, ANY, COUNT>(sv, r, tlo, tmin, tmax, ts, st, cnt)) {
        }
    }
    bt = ts.bt;
    bu = ts.bu;
    bv = ts.bv;
    return ts.best;
}

// pos and normal of an accepted hit (maths.cpp:375-377)
__device__ __forceinline__ void hit_record(const SceneView& sv, int id, float u, float v, f3& pos,
                                           f3& nrm)
{
    const float4* p = reinterpret_cast<const float4*>(sv.tri_orig + id);
    float4 a = p[0], b = p[1], c = p[2];
    f3 v0 = mk(a.x, a.y, a.z), v1 = mk(a.w, b.x, b.y), v2 = mk(b.z, b.w, c.x);
    pos = hit_pos(v0, v1, v2, u, v);
    nrm = mk(c.y, c.z, c.w);
}

}  // namespace tmpt
