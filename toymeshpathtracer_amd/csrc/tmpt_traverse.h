// tmpt_traverse.h -- BVH4Q traversal for gfx950: closest hit (Scene::HitScene,
// scene.cpp:86-97) and any hit (the shadow query of Scatter, main.cpp:57-60,
// whose only consumer is the hit/miss bit).  Every engine (persistent path
// kernel, wavefront, megakernel, batched HitScene) steps the same function,
// trav_step4q2_mixed.
//
// * Scene query contract: the BVH finds the closest hit over all
//   triangles.  Box culling is conservative (padded leaf boxes, stretched far
//   distance), so the Moller-Trumbore test alone -- bit-identical to
//   maths.cpp:339-380 -- decides every hit.  When two or more triangles share
//   the closest t, the lowest index is kept and the query is flagged
//   (bit 0 of TravState::best): the reference keeps the first of them in its
//   octree's visit order (scene.cpp:29-48), so with the scene's octree built
//   (tmpt_scene_build_octree) a flagged query is answered again over that
//   octree, exactly as HitSceneInternal walks it (octree_closest below).
// * Stack: the first SL entries of each lane live in LDS (layout [depth][lane],
//   so a wave's accesses to one depth hit 64 distinct banks); deeper entries
//   spill to a per-lane global area (never more than kStackTotal in all).
// * Slab test in fma form t = q*(2^e/d) + (origin*inv - o*inv) (not bit-exact,
//   only conservative, which is all culling needs).
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
    uint32_t offx, offy, offz;  // octant: near plane per axis (16 / 48 / 80 = the hi plane)
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

// x * 2^e for the signed exponent byte e at bit `sh` of w: v_bfe_i32 + v_ldexp_f32,
// exact (a power-of-two scaling, no under/overflow for the 1/d of a unit direction)
__device__ __forceinline__ float exp_mul(float x, uint32_t w, int sh)
{
    return __builtin_amdgcn_ldexpf(x, (int)__builtin_amdgcn_sbfe(w, sh, 8));
}

// Pins a loaded triangle record's used words in registers at this point (no
// instruction emitted), so the compiler cannot sink their loads into the
// branches that consume them.
__device__ __forceinline__ void materialize(float4& a, float4& b, float4& c)
{
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z),
                 "+v"(b.w), "+v"(c.x), "+v"(c.y));
}

typedef float v2f __attribute__((ext_vector_type(2)));
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
    const lds_u4* top = nullptr;  // LDS copy of BVH4 nodes [0, ntop) (TOPC steps), 4 uint4 each
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
    const Bvh4Node* __restrict__ nodes4;
    const TriPre* __restrict__ tri_pre;
    const TriOrig* __restrict__ tri_orig;
    int32_t n;
    int32_t n_nodes4 = 0;
    // the reference's octree (null: none built, or option tie_rule = index):
    // one pointer to its device-side view, read only by the rare flagged
    // queries (the kernels keep one SGPR pair live for it, not four)
    const OctView* __restrict__ oct = nullptr;
    // the crack test's first stage (octree_flag), by value so every finished
    // query reads it from kernel-argument registers, not through `oct`:
    // {reach, drift.xyz} of OctGrid
    float4 crack = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    // build option layout=soa (tmpt_internal.h SoaScene): the same nodes and
    // triangle records as planes, read by the SOA instantiations
    SoaScene soa;
#ifdef TMPT_CHECK
    uint32_t* chk = nullptr;  // Scene::chk (tmpt_internal.h kChk*)
#endif
};

// TMPT_CHK(chk, ok, code, what): in the checked build, true (and `code`
// recorded) when `ok` fails, so the caller can end the query before the bad
// access; in the product build a constant false that evaluates nothing.
#ifdef TMPT_CHECK
__device__ __noinline__ void chk_fail(uint32_t* chk, uint32_t code, int what)
{
    if (chk == nullptr) return;
    __hip_atomic_fetch_or(&chk[0], code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&chk[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&chk[2], (uint32_t)what, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define TMPT_CHK(chk, ok, code, what) (__builtin_expect(!(ok), 0) && (chk_fail((chk), (code), (int)(what)), true))
#define TMPT_CHK_PARAMS , uint32_t *chk, int64_t n_refs, int32_t n_tri
#define TMPT_CHK_ARGS(sv) , (sv).chk, (sv).oct->n_refs, (sv).n
#else
#define TMPT_CHK(chk, ok, code, what) false
#define TMPT_CHK_PARAMS
#define TMPT_CHK_ARGS(sv)
#endif

struct TravCount {
    uint32_t nodes = 0, tris = 0;
};

// Resumable traversal state of one lane (registers).
struct TravState {
    int node;   // next node (>=0 internal, <0 leaf = ~slot)
    int sp;     // stack depth
    int best;   // during traversal: 2 x the triangle index of the current closest hit
                // (TriPre stores it doubled), | 1 when another triangle was accepted at
                // the same t; -1 if none.  settle_closest turns it into the index.
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

// One step over BVH4Q (64-B quantised nodes): one node or one leaf.
// Node: near/far byte planes picked per axis by the ray's octant (one
// v_cndmask per plane dword), t = q * (2^e/d) + fma(origin, 1/d, -o/d) by
// packed fma over child pairs, no per-child min/max and no mask test (empty
// slots carry an inverted box and link to the null leaf); the nearest hit
// child is next, the others are pushed pairwise-ordered.  Leaf: its triangles'
// Moller-Trumbore tests (bit-exact, maths.cpp:339-380) with t in [tmin, tmax];
// ties on t keep the lowest triangle index and set bit 0 (the caller settles
// them, settle_closest).  `any` (run time): stop at the
// first accepted triangle (the shadow query).  Returns true when the query is
// finished; ts.node is undefined after that (the next query re-inits it).
// tlo: lower clamp of a box's entry distance, min(tmin, 0) (boxes behind the
// origin hold no t >= 0 hit); the path engines pass the reference's constant
// range kMinT..kMaxT (main.cpp:30-31), the batched HitScene any per-ray range.
// KIND 1 / 2: the caller guarantees the lane is at a node / at a leaf (a voted
// round), so the other kind's code is not emitted.  TOPC: node indices below
// st.ntop are read from the block's LDS copy of the top levels.
// NEG: the query's range may reach behind the origin (the batched HitScene's
// per-ray ranges): the far-distance slack is applied by magnitude, so it
// widens a box's interval for negative distances too (kTfarSlack alone would
// shrink it there); the path engines' range kMinT..kMaxT never needs it.
template <bool COUNT, int BLOCK, int SL, bool TOPC = false, int KIND = 0, bool SOA = false, bool NEG = false,
          bool FLAG = false>
__device__ __forceinline__ bool trav_step4q2_mixed(const SceneView& sv, const TravRay& r, bool any,
                                                   TravState& ts, TravStack<BLOCK, SL>& st,
                                                   TravCount& cnt, float tlo = 0.0f, float tmin = kMinT,
                                                   float tmax = kMaxT)
{
    // KIND 1 / 2: the caller guarantees the lane is at a node / at a leaf (a
    // voted round), so the other kind's code is not emitted at all
    if (KIND == 1 || (KIND == 0 && ts.node >= 0)) {
        if (TMPT_CHK(sv.chk, (uint32_t)ts.node < (uint32_t)sv.n_nodes4, kChkNode, ts.node)) return true;
        // 32-bit byte offset off an SGPR base: one VALU for the address
        uint4 A, B, C;
        int4 L;
        if (SOA && (!TOPC || (uint32_t)ts.node >= st.ntop)) {  // four planes: 16 + 16 + 8 + 16 B
            const uint32_t k = (uint32_t)ts.node;
            A = sv.soa.na[k], B = sv.soa.nb[k], L = sv.soa.nd[k];
            const uint2 c2 = sv.soa.nc[k];
            C = make_uint4(c2.x, c2.y, 0u, 0u);
        } else if (!TOPC || (uint32_t)ts.node >= st.ntop) {
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
            float tn = fmaxf(fmaxf(tnx[k], tny[k]), fmaxf(tnz[k], tlo));
            float tf = fminf(fminf(tfx[k], tfy[k]), fminf(tfz[k], ts.bt));
            const float tf_slack = NEG ? tf + fabsf(tf) * (kTfarSlack - 1.0f) : tf * kTfarSlack;
            key[k] = tn <= tf_slack ? tn : INFINITY;
        }
        {  // nearest child next; the others pushed pairwise-ordered only
            const bool s01 = key[1] < key[0], s23 = key[3] < key[2];
            const float ka = s01 ? key[1] : key[0], kao = s01 ? key[0] : key[1];
            const int ca = s01 ? ch[1] : ch[0], cao = s01 ? ch[0] : ch[1];
            const float kb = s23 ? key[3] : key[2], kbo = s23 ? key[2] : key[3];
            const int cb = s23 ? ch[3] : ch[2], cbo = s23 ? ch[2] : ch[3];
            const bool sab = kb < ka;
            const float kn = sab ? kb : ka, kno = sab ? ka : kb;
            const int cn = sab ? cb : ca, cno = sab ? ca : cb;
            if (kn != INFINITY) {
                if (TMPT_CHK(sv.chk, ts.sp + 3 <= kStackTotal, kChkStack, ts.sp)) return true;
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
        // records [0, n] (record n: the null leaf's)
        if (TMPT_CHK(sv.chk, first + n <= (uint32_t)sv.n + 1u, kChkLeaf, code)) return true;
        const char* base = reinterpret_cast<const char*>(sv.tri_pre);
        // Accepts (t, u, v, id) by the closest-hit order; true = any-hit query done.
        auto tri = [&](const float4& a, const float4& b, const float4& c) -> bool {
            if (COUNT) ++cnt.tris;
            float t, u, v;
            if (mt_test(r.o, r.d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c.x), tmin, tmax,
                        t, u, v)) {
                // id = 2 x index: comparing it with best (2 x index | tie bit)
                // orders the indices; the tie bit never decides
                const int id = __float_as_int(c.y);
                // (no triangle is accepted at t == tmax, the initial bt: the
                // flag it sets on best = -1 leaves -1)
                const bool tie = t == ts.bt;
                if (t < ts.bt || (!FLAG && tie && id < ts.best)) {
                    ts.bt = t;
                    ts.bu = u;
                    ts.bv = v;
                    ts.best = id | (int)tie;
                    if (any) return true;
                } else {
                    ts.best |= (int)tie;
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
        float4 a0, b0, c0, a1, b1, c1;
        if (SOA) {  // three planes: 16 + 16 + 8 B per triangle
            const uint32_t f1 = first + (n > 1u ? 1u : 0u);
            a0 = sv.soa.ta[first], b0 = sv.soa.tb[first];
            a1 = sv.soa.ta[f1], b1 = sv.soa.tb[f1];
            const float2 q0 = sv.soa.tc[first], q1 = sv.soa.tc[f1];
            c0 = make_float4(q0.x, q0.y, 0.0f, 0.0f);
            c1 = make_float4(q1.x, q1.y, 0.0f, 0.0f);
        } else {
            a0 = p0[0], b0 = p0[1], c0 = p0[2];
            a1 = p1[0], b1 = p1[1], c1 = p1[2];
        }
        materialize(a0, b0, c0);
        materialize(a1, b1, c1);
        if (KIND == 2) {
            // voted leaf round: both tests without early exits (the two
            // dependency chains interleave), then the closest-hit order
            // (triangle 0 first; an any-hit query stops at the first accept)
            float t0, u0, w0, t1, u1, w1;
            if (COUNT) cnt.tris += n > 1u ? 2u : 1u;
            const bool ok0 = mt_test_flat(r.o, r.d, mk(a0.x, a0.y, a0.z), mk(a0.w, b0.x, b0.y),
                                          mk(b0.z, b0.w, c0.x), tmin, tmax, t0, u0, w0);
            const bool ok1 = mt_test_flat(r.o, r.d, mk(a1.x, a1.y, a1.z), mk(a1.w, b1.x, b1.y),
                                          mk(b1.z, b1.w, c1.x), tmin, tmax, t1, u1, w1) &&
                             n > 1u;
            const int id0 = __float_as_int(c0.y), id1 = __float_as_int(c1.y);
            // FLAG: the first triangle met keeps a tie (the flag sends the query
            // to be answered again); otherwise the lower index takes it
            const bool tie0 = ok0 && t0 == ts.bt;
            const bool acc0 = ok0 && (t0 < ts.bt || (!FLAG && tie0 && id0 < ts.best));
            ts.bt = acc0 ? t0 : ts.bt;
            ts.bu = acc0 ? u0 : ts.bu;
            ts.bv = acc0 ? w0 : ts.bv;
            ts.best = (acc0 ? id0 : ts.best) | (int)tie0;
            const bool tie1 = ok1 && !(any && acc0) && t1 == ts.bt;
            const bool acc1 = ok1 && !(any && acc0) && (t1 < ts.bt || (!FLAG && tie1 && id1 < ts.best));
            ts.bt = acc1 ? t1 : ts.bt;
            ts.bu = acc1 ? u1 : ts.bu;
            ts.bv = acc1 ? w1 : ts.bv;
            ts.best = (acc1 ? id1 : ts.best) | (int)tie1;
            if (any && (acc0 || acc1)) return true;
        } else {  // a lone lane (row chains) gains more from the early exits
            if (tri(a0, b0, c0)) return true;
            if (n > 1u && tri(a1, b1, c1)) return true;
        }
        for (uint32_t k = 2; k < n; ++k) {
            if (SOA) {
                const float2 q = sv.soa.tc[first + k];
                if (tri(sv.soa.ta[first + k], sv.soa.tb[first + k], make_float4(q.x, q.y, 0.0f, 0.0f))) return true;
            } else {
                const float4* p = reinterpret_cast<const float4*>(base + (first + k) * (uint32_t)sizeof(TriPre));
                if (tri(p[0], p[1], p[2])) return true;
            }
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

// ---------------------------------------------------------------- reference octree
// RayHitAabb (maths.h:116-134) in the reference's own arithmetic: the slab
// distances from the inverted direction (scene.cpp:92-93), swapped when it is
// negative, the range narrowed by its ternaries, rejected once empty.  Exact,
// not conservative: it decides which leaves the reference visits.
__device__ __forceinline__ bool ref_slab(f3 o, f3 inv, float4 lo, float4 hi, float tmin, float tmax)
{
    const float oc[3] = {o.x, o.y, o.z}, ic[3] = {inv.x, inv.y, inv.z};
    const float lc[3] = {lo.x, lo.y, lo.z}, hc[3] = {hi.x, hi.y, hi.z};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float t0 = (lc[c] - oc[c]) * ic[c], t1 = (hc[c] - oc[c]) * ic[c];
        if (ic[c] < 0.0f) {
            const float sw = t0;
            t0 = t1;
            t1 = sw;
        }
        tmin = t0 > tmin ? t0 : tmin;
        tmax = t1 < tmax ? t1 : tmax;
        if (tmax < tmin) return false;
    }
    return true;
}

__device__ __forceinline__ f3 ref_inverse(f3 d) { return mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }

// HitScene's first step, the root box test (scene.cpp:25 on the root): a ray
// that misses the root misses the scene, whatever the triangles say.  Only a
// ray from outside the root box can fail it while hitting a triangle (one
// that grazes the root's faces at the floor's corners, main.cpp:153-162 puts
// them on the root's boundary).
__device__ __forceinline__ bool root_slab(const OctNode* __restrict__ nodes, f3 o, f3 d, float tmin, float tmax)
{
    return ref_slab(o, ref_inverse(d), nodes[0].lo, nodes[0].hi, tmin, tmax);
}

__device__ __forceinline__ bool octree_root_hit(const SceneView& sv, f3 o, f3 d, float tmin, float tmax)
{
    return root_slab(sv.oct->nodes, o, d, tmin, tmax);
}

// HitSceneInternal (scene.cpp:21-52) over the preorder octree: a node whose
// box fails the slab test is skipped with its subtree (its skip link); a
// leaf tests its triangles in list order with the query's range (tMax is
// never shrunk, scene.cpp:32) and keeps a hit only if t < the best so far
// (scene.cpp:34), so among equal t the first met in child order 0..7 wins.
// Returns the triangle index or -1; (t, u, v) of the hit, e1/e2 formed as
// maths.cpp:341-342 forms them.  `target`: the closest t over all triangles
// (the BVH's answer): no triangle has a smaller one, so the first met at
// exactly `target` is the reference's answer and the walk stops there.
// The walk itself takes plain pointers and returns by value.
struct OctHit {
    int best;
    float t, u, v;
};

__device__ __forceinline__ OctHit octree_walk(const OctNode* __restrict__ nodes, const int32_t* __restrict__ refs,
                                               int n_oct, const TriOrig* __restrict__ tris, f3 o, f3 d,
                                               float tmin, float tmax, float target TMPT_CHK_PARAMS)
{
    const f3 inv = ref_inverse(d);
    OctHit h{-1, tmax, 0.0f, 0.0f};
#ifdef TMPT_EXP_WALKSTAT  // cost experiment: nodes and triangles a walk visits
    uint32_t wn = 0, wt = 0;
#endif
    for (int i = 0; i < n_oct;) {
#ifdef TMPT_EXP_WALKSTAT
        ++wn;
#endif
        const float4 lo = nodes[i].lo, hi = nodes[i].hi;
        if (!ref_slab(o, inv, lo, hi, tmin, tmax)) {
            const int skip = __float_as_int(lo.w);
            if (TMPT_CHK(chk, skip > i && skip <= n_oct, kChkOctSkip, skip)) break;
            i = skip;
            continue;
        }
        const int ref = __float_as_int(hi.w);
        if (ref >= 0) {
            if (TMPT_CHK(chk, (int64_t)ref < n_refs && (int64_t)ref + refs[ref] < n_refs, kChkOctRef, ref)) break;
            const int cnt = refs[ref];
            for (int k = 1; k <= cnt; ++k) {
                const int id = refs[ref + k];
                if (TMPT_CHK(chk, (uint32_t)id < (uint32_t)n_tri, kChkTri, id)) continue;
                const float4* p = reinterpret_cast<const float4*>(tris + id);
                const float4 a = p[0], b = p[1], c = p[2];
                const f3 v0 = mk(a.x, a.y, a.z), v1 = mk(a.w, b.x, b.y), v2 = mk(b.z, b.w, c.x);
                float t, u, v;
#ifdef TMPT_EXP_WALKSTAT
                ++wt;
#endif
                if (mt_test(o, d, v0, v1 - v0, v2 - v0, tmin, tmax, t, u, v) && t < h.t) {
                    h = OctHit{id, t, u, v};
                    if (t == target) {  // first at the minimum: nothing can replace it
                        i = n_oct;
                        break;
                    }
                }
            }
        }
        ++i;  // a leaf's skip link is the next node; an inner node descends to child 0
    }
#ifdef TMPT_EXP_WALKSTAT
    extern __device__ unsigned long long g_walkstat[4];
    atomicAdd(&g_walkstat[0], (unsigned long long)wn);
    atomicAdd(&g_walkstat[1], (unsigned long long)wt);
    atomicMax(&g_walkstat[2], (unsigned long long)wn);
    atomicAdd(&g_walkstat[3], 1ull);
#endif
    return h;
}

__device__ __forceinline__ int octree_closest(const SceneView& sv, f3 o, f3 d, float tmin, float tmax, float target,
                                              float& bt, float& bu, float& bv)
{
    const OctHit h =
        octree_walk(sv.oct->nodes, sv.oct->refs, sv.oct->n, sv.tri_orig, o, d, tmin, tmax, target TMPT_CHK_ARGS(sv));
    bt = h.t;
    bu = h.u;
    bv = h.v;
    return h.best;
}

// Whether a hit at t on the ray (o, d) may lie in one of the octree's cracks
// (tmpt_internal.h OctGrid): for some axis k the hit point is within band[k]
// of a plane of the octree's finest grid and the ray drifted less than
// 2 band[k] along k over min(t, reach) -- it ran along that plane, where a
// gap between two subtrees' boxes can hide the leaves that hold the triangle
// from the reference's walk.  The plane distance is evaluated as the host's
// flat-triangle test evaluates it (tmpt_octree.cpp plane_dist).
// The second stage: for the axes whose drift the first stage flagged, whether
// the hit point lies within band of a plane of that axis.
TMPT_HD bool octree_crack_planes(const OctGrid& g, f3 o, f3 d, float t, bool ax, bool ay, bool az)
{
    const float oc[3] = {o.x, o.y, o.z}, dc[3] = {d.x, d.y, d.z};
    const bool on[3] = {ax, ay, az};
    bool f = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float rel = fmaf(t, dc[k], oc[k]) - g.r0[k];
        const float j = rintf(rel * g.inv_cell[k]);
        f |= on[k] && fabsf(fmaf(-j, g.cell[k], rel)) <= g.band[k];
    }
    return f;
}

// Both stages (the host check hook's form of the device test).
TMPT_HD bool octree_crack(const OctGrid& g, f3 o, f3 d, float t)
{
    const float span = fminf(t, g.reach);
    const bool ax = fabsf(d.x) * span <= g.drift[0], ay = fabsf(d.y) * span <= g.drift[1],
               az = fabsf(d.z) * span <= g.drift[2];
    return (ax | ay | az) && octree_crack_planes(g, o, d, t, ax, ay, az);
}

// Whether a finished query is one the octree answers: bit 0 of TravState::best
// (a tie on t, or a triangle lying flat on an octree plane -- its record's
// index is odd) or a hit that may lie in a crack.  The any-hit query's bit 0
// can only come from a flat triangle (it stops at its first accept).
__device__ __forceinline__ bool octree_flag(const SceneView& sv, const TravRay& r, const TravState& ts)
{
    if (sv.oct == nullptr || ts.best < 0) return false;
    if ((ts.best & 1) != 0) return true;
    // first stage from the by-value copy (no memory round trip); the plane
    // distances, rarely needed, through the view
    const float span = fminf(ts.bt, sv.crack.x);
    const bool ax = fabsf(r.d.x) * span <= sv.crack.y, ay = fabsf(r.d.y) * span <= sv.crack.z,
               az = fabsf(r.d.z) * span <= sv.crack.w;
#ifdef TMPT_EXP_CRACKSTAT  // cost experiment: how often each stage runs and fires
    {
        extern __device__ unsigned long long g_crackstat[4];
        const bool s2 = (ax | ay | az) && octree_crack_planes(sv.oct->grid, r.o, r.d, ts.bt, ax, ay, az);
        atomicAdd(&g_crackstat[0], 1ull);
        if (ax | ay | az) atomicAdd(&g_crackstat[1], 1ull);
        if (s2) atomicAdd(&g_crackstat[2], 1ull);
        if (ts.bt < sv.crack.x) atomicAdd(&g_crackstat[3], 1ull);
        return s2;
    }
#endif
    return (ax | ay | az) && octree_crack_planes(sv.oct->grid, r.o, r.d, ts.bt, ax, ay, az);
}

// counts a query octree_flag sent to the octree: ties[0] (bit 0) or ties[6] (crack)
__device__ __forceinline__ void octree_count(const OctView* ov, int best)
{
    atomicAdd(&ov->ties[(best & 1) ? 0 : 6], 1ull);
}

// A finished closest-hit query: the triangle index from TravState::best; a
// flagged query is answered again over the octree (the reference's pick among
// tied triangles, its whole answer for that ray); without an octree the
// lowest index stands.  (The walk stops at the first triangle at the BVH's
// closest t, which is the reference's answer when it reaches it: nothing lies
// nearer.)
template <int BLOCK, int SL, bool TOPC, bool SOA, bool NEG>
__device__ __forceinline__ void settle_closest(const SceneView& sv, const TravRay& r, float tlo, float tmin,
                                               float tmax, TravState& ts, TravStack<BLOCK, SL>& st)
{
    (void)tlo;
    (void)st;
    if (octree_flag(sv, r, ts)) {
        octree_count(sv.oct, ts.best);
        ts.best = octree_closest(sv, r.o, r.d, tmin, tmax, ts.bt, ts.bt, ts.bu, ts.bv);
    } else {
        ts.best >>= 1;  // -1 stays -1
    }
}

// A finished any-hit query (the shadow ray's hit / miss bit): a hit the
// reference's octree might not see (a flat triangle, a crack) is answered by
// its walk; otherwise the first accepted triangle stands.
__device__ __forceinline__ void settle_any(const SceneView& sv, const TravRay& r, float tmin, float tmax,
                                           TravState& ts)
{
    if (octree_flag(sv, r, ts)) {
        octree_count(sv.oct, ts.best);
        float t, u, v;
        ts.best = octree_closest(sv, r.o, r.d, tmin, tmax, -INFINITY, t, u, v);
    } else {
        ts.best >>= 1;  // the doubled index of the first accepted triangle (-1 stays -1)
    }
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

// Whole query in one call, t in [tmin, tmax] (Scene::HitScene, scene.cpp:86-97).
// Returns the original triangle index or -1; (bt, bu, bv) of the hit.  TOPC:
// the caller's block holds the top BVH levels in LDS (st.top).
// CHECK_ANY = false: the caller knows no shadow answer needs the octree
// (PathCtl::oct_shadow is 0 wherever it runs), so the any-hit query skips
// settle_any and its walk.
template <bool ANY, bool COUNT, int BLOCK, int SL, bool TOPC = false, bool SOA = false, bool NEG = false,
          bool CHECK_ANY = true>
__device__ __forceinline__ int traverse(const SceneView& sv, const TravRay& r, float tmin,
                                        float tmax, float& bt, float& bu, float& bv,
                                        TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    TravState ts;
    trav_init(ts, tmax);
    if (sv.n > 0 && !ray_has_nan(r.o, r.d)) {
        const float tlo = fminf(tmin, 0.0f);
        while (!trav_step4q2_mixed<COUNT, BLOCK, SL, TOPC, 0, SOA, NEG>(sv, r, ANY, ts, st, cnt, tlo, tmin, tmax)) {
        }
        if (!ANY) settle_closest<BLOCK, SL, TOPC, SOA, NEG>(sv, r, tlo, tmin, tmax, ts, st);
        else if (CHECK_ANY) settle_any(sv, r, tmin, tmax, ts);
        else ts.best >>= 1;
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
    if (TMPT_CHK(sv.chk, (uint32_t)id < (uint32_t)max(sv.n, 1), kChkTri, id)) id = 0;
    const float4* p = reinterpret_cast<const float4*>(sv.tri_orig + id);
    float4 a = p[0], b = p[1], c = p[2];
    f3 v0 = mk(a.x, a.y, a.z), v1 = mk(a.w, b.x, b.y), v2 = mk(b.z, b.w, c.x);
    pos = hit_pos(v0, v1, v2, u, v);
    nrm = mk(c.y, c.z, c.w);
}

}  // namespace tmpt
