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

__device__ __forceinline__ float safe_inv(float d)
{
    float a = fabsf(d) < 1e-20f ? copysignf(1e-20f, d) : d;
    return 1.0f / a;
}

struct TravRay {
    f3 o, d;
    float ix, iy, iz;  // 1/d (finite)
    float ox, oy, oz;  // o * inv
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

template <int BLOCK, int SL>
struct TravStack {
    uint32_t* lds;   // &s_stack[threadIdx.x]; entry k at lds[k * BLOCK]
    uint32_t* glob;  // kStackTotal - SL entries of this lane
    __device__ __forceinline__ void push(int& sp, int v)
    {
        if (SL >= kStackTotal || sp < SL) lds[sp * BLOCK] = (uint32_t)v;
        else glob[sp - SL] = (uint32_t)v;
        ++sp;
    }
    __device__ __forceinline__ int pop(int& sp)
    {
        --sp;
        if (SL >= kStackTotal || sp < SL) return (int)lds[sp * BLOCK];
        return (int)glob[sp - SL];
    }
};

struct SceneView {
    const BvhNode* __restrict__ nodes;
    const TriPre* __restrict__ tri_pre;
    const TriOrig* __restrict__ tri_orig;
    const float2* __restrict__ sincos;
    int32_t n;
};

struct TravCount {
    uint32_t nodes = 0, tris = 0;
};

// Closest hit.  Returns the original triangle index or -1; t/u/v of the hit.
template <bool ANY, bool COUNT, int BLOCK, int SL>
__device__ __forceinline__ int traverse(const SceneView& sv, const TravRay& r, float tmin,
                                        float tmax, float& bt, float& bu, float& bv,
                                        TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    int best = -1;
    bt = tmax;
    if (sv.n <= 0) return -1;
    const float tlo = fminf(tmin, 0.0f);
    int sp = 0;
    int node = 0;
    for (;;) {
        if (node >= 0) {
            const float4* p = reinterpret_cast<const float4*>(sv.nodes + node);
            float4 a = p[0], b = p[1], c = p[2];
            int4 lk = reinterpret_cast<const int4*>(p)[3];
            if (COUNT) ++cnt.nodes;
            float tn0, tn1;
            bool h0 = slab(r, a.x, a.y, a.z, a.w, b.x, b.y, tlo, bt, tn0);
            bool h1 = slab(r, b.z, b.w, c.x, c.y, c.z, c.w, tlo, bt, tn1);
            if (h0 && h1) {
                int nearc = lk.x, farc = lk.y;
                if (tn1 < tn0) { nearc = lk.y; farc = lk.x; }
                st.push(sp, farc);
                node = nearc;
            } else if (h0) {
                node = lk.x;
            } else if (h1) {
                node = lk.y;
            } else {
                if (sp == 0) break;
                node = st.pop(sp);
            }
        } else {
            const float4* p = reinterpret_cast<const float4*>(sv.tri_pre + (~node));
            float4 a = p[0], b = p[1], c = p[2];
            if (COUNT) ++cnt.tris;
            float t, u, v;
            if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), tmin, tmax,
                        t, u, v)) {
                int id = __float_as_int(c.y);
                if (t < bt || (t == bt && best >= 0 && id < best)) {
                    bt = t;
                    bu = u;
                    bv = v;
                    best = id;
                    if (ANY) return best;
                }
            }
            if (sp == 0) break;
            node = st.pop(sp);
        }
    }
    return best;
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
