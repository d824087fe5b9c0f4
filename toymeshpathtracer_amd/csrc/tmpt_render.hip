// tmpt_render.hip -- the path tracer of main.cpp:44-119 / 172-246 on gfx950.
//
// Engines (DESIGN.md "Kernels"):
//  * wavefront (pixel mode): per-pixel path state in HBM (SoA), one slot per
//    pixel of the tile; every iteration runs
//        extend  closest-hit traversal of the active queue     (persistent waves)
//        shade   hit -> shadow ray + next bounce; miss/max depth -> backward
//                recurrence, accumulate, next camera sample or pixel write
//        shadow  any-hit traversal of the shadow queue          (persistent waves)
//    queues are compacted with wave64 ballot + mbcnt prefix and ONE atomic per
//    wave.  Samples of a pixel stay sequential (its RNG stream threads through
//    them, main.cpp:204-218), so parallelism is over pixels.
//  * megakernel: one lane per pixel (pixel mode) or per row (row mode: the
//    unmodified reference RNG chain, H-way parallel -- a correctness mode).
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <vector>

#include "tmpt.h"
#include "tmpt_internal.h"
#include "tmpt_traverse.h"

namespace tmpt {

struct RenderArgs {
    Camera cam;
    int32_t W, H, spp, seed_mode, band_rows, shard, nshards, tile_rows;
    float invW, invH, spp_recip;
    int64_t slots;  // tile_rows * W
    // progressive spp: samples [smp_begin, smp_end) this call; prog = per-pixel
    // {colour sum, rng} carried between calls (null: one full pass)
    int32_t smp_begin, smp_end;
    float out_recip;  // 1/spp for the final pass, 1/smp_end for a preview
    float4* prog;
    // sample seeding (TMPT_SEED_SAMPLE): jump tables of sample_seed (null in the
    // other modes); a lane's run of samples ends where smp & bmask == 0 (its
    // block of the persistent engine; 2047 = never inside 1..1024)
    const uint32_t* jt;
    uint32_t bmask;
    // row seeding in the megakernel: rows per wave (lanes 0..row_lanes-1 each
    // run one row's chain; the rest of the wave idles)
    int32_t row_lanes;
    // camera rays take the reference's root box test first (SceneView::oct
    // set and the lens may lie outside the root box: render() decides)
    int32_t root_check;
};

__device__ __forceinline__ int tile_row_to_y(const RenderArgs& a, int lr)
{
    int lb = lr / a.band_rows, r = lr - lb * a.band_rows;
    return (lb * a.nshards + a.shard) * a.band_rows + r;
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// wave64 ballot straight from the predicate (HIP's __ballot widens the bool to
// an int and compares it again: two extra VALU per call in the hot loops)
__device__ __forceinline__ uint64_t wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wany(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// s_memtime (shader clock), for the PROF build of k_path only
__device__ __forceinline__ uint64_t stamp()
{
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// wave64 sum of a 32-bit value (all lanes must call)
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    return v;
}

// Compacted append: every lane of the wave calls; lanes with pred get
// consecutive slots, one atomic per wave (ballot + mbcnt prefix).
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred)
{
    uint64_t m = wballot(pred);
    if (m == 0) return 0;
    int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    return base + below;
}

template <int BLOCK, bool COUNT>
__device__ __forceinline__ void flush_counts(unsigned long long* counters, uint32_t rays,
                                             const TravCount& cnt)
{
    uint32_t r = wave_sum(rays);
    uint32_t nv = COUNT ? wave_sum(cnt.nodes) : 0u;
    uint32_t nt = COUNT ? wave_sum(cnt.tris) : 0u;
    if (lane_id() == 0) {
        atomicAdd(&counters[0], (unsigned long long)r);
        if (COUNT) {
            atomicAdd(&counters[1], (unsigned long long)nv);
            atomicAdd(&counters[2], (unsigned long long)nt);
        }
    }
}

// ============================================================ megakernel
// Whole query; TOPC: the top BVH4 levels from the block's LDS copy (the
// latency-bound row chains).
template <bool ANY, bool COUNT, bool TOPC, int BLOCK, int SL, bool CHECK_ANY = true>
__device__ __forceinline__ int mega_query(const SceneView& sv, f3 o, f3 d, float& t, float& u, float& v,
                                          TravStack<BLOCK, SL>& st, TravCount& cnt)
{
    return traverse<ANY, COUNT, BLOCK, SL, TOPC, false, false, CHECK_ANY>(sv, make_trav_ray(o, d), kMinT, kMaxT, t, u,
                                                                          v, st, cnt);
}

// rays: closest-hit queries, srays: shadow queries (the same counter where the
// caller does not split them)
// CHECK_ANY: the shadow answers are checked against the octree (settle_any);
// the deferred-tie redo passes false (tie_defer is off wherever a shadow
// answer can need the octree, PathCtl::oct_shadow)
template <bool COUNT, int BLOCK, int SL, bool TOPC = false, bool CHECK_ANY = true>
__device__ __forceinline__ f3 trace_path(const SceneView& sv, f3 o, f3 d, uint32_t& rng,
                                         uint32_t& rays, uint32_t& srays, TravStack<BLOCK, SL>& st, float* lbuf,
                                         TravCount& cnt, bool root_check, int depth0 = 0)
{
    int depth = depth0;  // > 0: a path resumed at its depth0-th closest-hit query, lbuf[0, depth0) set
    f3 color = mk(0.0f, 0.0f, 0.0f);
    while (depth < kMaxDepth) {  // Trace, main.cpp:89-110
        ++rays;
        float t, u, v;
        int id = -1;
        if (depth == 0 && root_check && !octree_root_hit(sv, o, d, kMinT, kMaxT)) {
            atomicAdd(&sv.oct->ties[1], 1ull);  // the camera ray misses the reference's root box
        } else {
            id = mega_query<false, COUNT, TOPC>(sv, o, d, t, u, v, st, cnt);
        }
        if (id >= 0) {
            f3 pos, nrm;
            hit_record(sv, id, u, v, pos, nrm);
            ++srays;  // shadow ray, main.cpp:57-59 (always counted)
            float lc = light_cosine(nrm, d);
            if (lc > 0.0f) {  // a zero light term does not depend on the answer
                float ts, us, vs;
                int sid = mega_query<true, COUNT, TOPC, BLOCK, SL, CHECK_ANY>(sv, pos, light_dir(), ts, us, vs, st, cnt);
                if (sid >= 0) lc = 0.0f;
            }
            lbuf[depth * BLOCK] = lc;
            f3 rnd = random_unit_vector(rng);  // main.cpp:71-72
            f3 target = pos + nrm + rnd;
            d = normalize(target - pos);
            o = pos;
            ++depth;
        } else {
            color = sky(d);
            break;
        }
    }
    for (int i = depth - 1; i >= 0; --i) color = backward_step(color, lbuf[i * BLOCK]);
    return color;
}

template <bool COUNT, int BLOCK, int SL, bool TOPC = false>
__device__ __forceinline__ uint32_t render_pixel(const SceneView& sv, const RenderArgs& a, int x,
                                                 int y, uint32_t& rng, uint32_t& rays,
                                                 TravStack<BLOCK, SL>& st, float* lbuf,
                                                 TravCount& cnt)
{
    f3 col = mk(0.0f, 0.0f, 0.0f);
    const uint32_t pseed = rng;
    for (int s = 0; s < a.spp; ++s) {  // main.cpp:209-219
        f3 o, d;
        if (a.jt) rng = sample_seed(a.jt, (uint32_t)s, pseed);  // sample seeding
        camera_sample(a.cam, (uint32_t)x, (uint32_t)y, a.invW, a.invH, rng, o, d);
        col = col + trace_path<COUNT, BLOCK, SL, TOPC>(sv, o, d, rng, rays, rays, st, lbuf, cnt, a.root_check != 0);
    }
    return pack_pixel(col, a.spp_recip);
}

#ifdef TMPT_EXP_WALKSTAT
__device__ unsigned long long g_walkstat[4];
#endif
#ifdef TMPT_EXP_CRACKSTAT
__device__ unsigned long long g_crackstat[4];
#endif
#ifdef TMPT_EXP_WAVETIME  // timeline experiment: per wave, s_memrealtime at start / main loop end / exit
constexpr int kWaveTimeMax = 16384;
__device__ unsigned long long g_wavetime[3 * kWaveTimeMax];
__device__ unsigned long long g_rowtime[kWaveTimeMax];  // streaming row engine: when each row's chain ended
__device__ unsigned long long g_claimtime[kWaveTimeMax];  // streaming row engine: each worker wave's last claim
#endif

// ============================================================ octree walk, one wave
__device__ __forceinline__ float rlane(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ int rlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// octree_walk (tmpt_traverse.h) for ONE query, run by the whole wave (every
// lane active, every argument wave-uniform): the lanes test the slab of 64
// consecutive preorder nodes at once and the DFS then steps through that
// window on scalar masks (a failed node jumps to its skip link, a passed one
// to the next node), so a window costs one memory round trip instead of one
// per node; a visited leaf's triangles are tested one per lane, and the leaf
// keeps what the serial scan would: the first triangle at the leaf's least t
// when that t beats the best so far (strict <, scene.cpp:34).  The walk
// stops at the first triangle at `target` (nothing is nearer).  The
// reference visits ~100 nodes per tied query on the bench frame (up to ~950:
// tools/ diag TMPT_EXP_WALKSTAT, profiles/r04_ties/walkstat_n1.log).
__device__ __forceinline__ OctHit octree_walk_wave(const OctNode* __restrict__ nodes, const int32_t* __restrict__ refs,
                                                   int n_oct, const TriOrig* __restrict__ tris, f3 o, f3 d,
                                                   float tmin, float tmax, float target TMPT_CHK_PARAMS)
{
    const f3 inv = ref_inverse(d);
    const int lane = lane_id();
    OctHit h{-1, tmax, 0.0f, 0.0f};
    int i = 0;
    while (i < n_oct) {
        const int j = i + lane;
        bool pass = false;
        int skip = 0, ref = -1;
        if (j < n_oct) {
            const float4 lo = nodes[j].lo, hi = nodes[j].hi;
            pass = ref_slab(o, inv, lo, hi, tmin, tmax);
            skip = __float_as_int(lo.w);
            ref = __float_as_int(hi.w);
        }
        const uint64_t P = wballot(pass), L = wballot(pass && ref >= 0);
        int cur = i;
        const int end = min(i + 64, n_oct);
        while (cur < end) {
            const int k = cur - i;
            if (((P >> k) & 1ull) == 0) {
                const int sk = rlane(skip, k);
                if (TMPT_CHK(chk, sk > cur && sk <= n_oct, kChkOctSkip, sk)) return h;
                cur = sk;
                continue;
            }
            if ((L >> k) & 1ull) {
                const int r = rlane(ref, k);
                if (TMPT_CHK(chk, (int64_t)r < n_refs && (int64_t)r + refs[r] < n_refs, kChkOctRef, r)) return h;
                const int cnt = refs[r];
                for (int b = 0; b < cnt; b += 64) {
                    float t = INFINITY, u = 0.0f, v = 0.0f;
                    int id = -1;
                    bool ok = false;
                    if (b + lane < cnt) {
                        id = refs[r + 1 + b + lane];
                        if (TMPT_CHK(chk, (uint32_t)id < (uint32_t)n_tri, kChkTri, id)) id = 0;
                        const float4* p = reinterpret_cast<const float4*>(tris + id);
                        const float4 a = p[0], bb = p[1], c = p[2];
                        const f3 v0 = mk(a.x, a.y, a.z), v1 = mk(a.w, bb.x, bb.y), v2 = mk(bb.z, bb.w, c.x);
                        ok = mt_test(o, d, v0, v1 - v0, v2 - v0, tmin, tmax, t, u, v);
                    }
                    float m = ok ? t : INFINITY;
                    for (int off = 32; off > 0; off >>= 1) m = fminf(m, __shfl_xor(m, off));
                    const float mt = rlane(m, 0);
                    if (mt < h.t) {
                        const int f = (int)__builtin_ctzll(wballot(ok && t == mt));
                        h = OctHit{rlane(id, f), mt, rlane(u, f), rlane(v, f)};
                        if (mt == target) return h;
                    }
                }
            }
            ++cur;  // a leaf's skip link is the next node; an inner node descends to child 0
        }
        i = cur;
    }
    return h;
}

// ============================================================ deferred ties
// A sample the deferring sample kernel (k_path DEFER) dropped on a flagged
// closest hit is traced again from that query on by one lane, ties settled
// (trace_path's queries end in settle_closest).  The drop records where the
// path stopped -- the query's ray, the RNG state, its depth and the light
// terms of the bounces before it (redo_state_put) -- so the re-trace resumes
// there instead of restarting the sample; its colour goes
// to the colour buffer, where k_resolve_px sums it in sample order.  The list
// entry is (pixel, sample | depth << 16).
constexpr uint32_t kRedoEmpty = 0xFFFFFFFFu;  // a list entry not yet written
constexpr uint32_t kRedoDone = 0xFFFFFFFEu;   // an entry already traced
constexpr int kRedoTaken = 27, kRedoWaves = 28, kRedoTraced = 29;  // counters[]: tickets, waves past the main loop, traced
constexpr int kRedoState4 = 5;  // float4 per slot: o.xyz rng, d.xyz -, light[0..9], -, -
static_assert(2 * 4 + kMaxDepth <= 4 * kRedoState4, "redo state slot too small");

// the state words go out write-through (agent scope: another XCD's lane reads
// them), before the entry that publishes them (release fence in the caller)
__device__ __forceinline__ void redo_state_put(float4* ps, f3 o, f3 d, uint32_t rng, const float* light, uint32_t depth,
                                               uint32_t ls)
{
    float* w = reinterpret_cast<float*>(ps);
    const float h[8] = {o.x, o.y, o.z, __uint_as_float(rng), d.x, d.y, d.z, 0.0f};
#pragma unroll
    for (int i = 0; i < 7; ++i) __hip_atomic_store(&w[i], h[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = 0; i < depth; ++i)
        __hip_atomic_store(&w[8 + i], light[i * ls], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int BLOCK, int SL>
__device__ __forceinline__ void redo_sample(const SceneView& sv, const RenderArgs& a, uint32_t pix, uint32_t smp_depth,
                                            const float4* __restrict__ ps, float4* __restrict__ sbuf, uint32_t sb_ss,
                                            uint32_t sb_sp, uint32_t& rays_e, uint32_t& rays_s,
                                            TravStack<BLOCK, SL>& st, float* lbuf)
{
    const uint32_t smp = smp_depth & 0xFFFFu, depth = smp_depth >> 16;
    const float* w = reinterpret_cast<const float*>(ps);
    float h[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) h[i] = __hip_atomic_load(&w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = 0; i < depth; ++i)
        lbuf[i * BLOCK] = __hip_atomic_load(&w[8 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t rng = __float_as_uint(h[3]);
    TravCount cnt;
    const f3 c = trace_path<false, BLOCK, SL, true, false>(sv, mk(h[0], h[1], h[2]), mk(h[4], h[5], h[6]), rng, rays_e,
                                                           rays_s, st, lbuf, cnt, false, (int)depth);
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store((f32x4){c.x, c.y, c.z, 0.0f},
                                reinterpret_cast<f32x4*>(sbuf + ((size_t)smp * sb_ss + (size_t)pix * sb_sp)));
}

__device__ __forceinline__ uint2 redo_load(const uint2* p)
{
    const unsigned long long w =
        __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint2((uint32_t)w, (uint32_t)(w >> 32));
}

__device__ __forceinline__ void redo_put(uint2* p, uint32_t pix, uint32_t smp_depth)
{
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), ((unsigned long long)smp_depth << 32) | pix,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void redo_mark(uint2* p)
{
    __hip_atomic_store(reinterpret_cast<unsigned int*>(p), kRedoDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The entries the deferring launch left untraced (its waves gave up waiting,
// see k_path's redo phase): one lane per entry, grid-stride.
template <int BLOCK, int SL>
__global__ void __launch_bounds__(BLOCK) k_redo(SceneView sv, RenderArgs a, uint2* __restrict__ list, uint32_t cap,
                                                const float4* __restrict__ state, float4* __restrict__ sbuf,
                                                uint32_t sb_ss, uint32_t sb_sp,
                                                uint32_t* __restrict__ ovf, unsigned long long* __restrict__ counters)
{
    __shared__ uint32_t s_stack[SL * BLOCK];
    __shared__ float s_light[kMaxDepth * BLOCK];
    __shared__ uint4 s_top[kTopNodes * 4];
    const int64_t gtid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    TravStack<BLOCK, SL> st{&s_stack[threadIdx.x], ovf + gtid * (kStackTotal - SL)};
    const uint32_t ntop = (uint32_t)min(kTopNodes, sv.n_nodes4);
    const uint4* g = reinterpret_cast<const uint4*>(sv.nodes4);
    for (uint32_t i = threadIdx.x; i < ntop * 4; i += BLOCK) s_top[i] = g[i];
    __syncthreads();
    st.top = (const lds_u4*)s_top;
    st.ntop = ntop;
    const uint32_t n = (uint32_t)min(counters[kRedoCounter], (unsigned long long)cap);
    uint32_t rays_e = 0, rays_s = 0;
    for (uint32_t i = (uint32_t)gtid; i < n; i += gridDim.x * BLOCK) {
        const uint2 e = list[i];
        if (e.x >= kRedoDone) continue;
        redo_sample<BLOCK, SL>(sv, a, e.x, e.y, state + (size_t)i * kRedoState4, sbuf, sb_ss, sb_sp, rays_e, rays_s,
                               st, &s_light[threadIdx.x]);
    }
    const uint32_t re = wave_sum(rays_e), rs = wave_sum(rays_s);
    if (lane_id() == 0 && re + rs) {
        atomicAdd(&counters[0], (unsigned long long)(re + rs));
        atomicAdd(&counters[3], (unsigned long long)re);
        atomicAdd(&counters[kRedoRaysCounter], (unsigned long long)(re + rs));
    }
}

// the deferred-tie list and its per-slot state (freed together)
static void free_redo(Scene& s)
{
    if (s.redo) (void)hipFree(s.redo);
    if (s.redo_state) (void)hipFree(s.redo_state);
    s.redo = nullptr;
    s.redo_state = nullptr;
    s.redo_cap = 0;
}
static bool alloc_redo(Scene& s, int64_t cap)
{
    free_redo(s);
    if (hipMalloc(&s.redo, sizeof(uint2) * (size_t)cap) != hipSuccess ||
        hipMalloc(&s.redo_state, sizeof(float4) * kRedoState4 * (size_t)cap) != hipSuccess) {
        (void)hipGetLastError();
        free_redo(s);
        return false;
    }
    s.redo_cap = (uint32_t)cap;
    return true;
}

template <bool ROW, bool COUNT, int BLOCK, int SL>
__global__ void __launch_bounds__(BLOCK) k_mega(SceneView sv, RenderArgs a,
                                                uint32_t* __restrict__ out,
                                                uint32_t* __restrict__ ovf,
                                                unsigned long long* __restrict__ counters)
{
    __shared__ uint32_t s_stack[SL * BLOCK];
    __shared__ float s_light[kMaxDepth * BLOCK];
    const int64_t gtid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    TravStack<BLOCK, SL> st{&s_stack[threadIdx.x], ovf + gtid * (kStackTotal - SL)};
    float* lbuf = &s_light[threadIdx.x];
    // ROW (one latency-bound chain per wave): the persistent engine's node step,
    // with the top BVH4 levels copied to LDS
    constexpr bool TOPC = ROW;
    if (TOPC) {
        __shared__ uint4 s_top[TOPC ? kTopNodes * 4 : 1];
        const uint32_t ntop = (uint32_t)min(kTopNodes, sv.n_nodes4);
        const uint4* g = reinterpret_cast<const uint4*>(sv.nodes4);
        for (uint32_t i = threadIdx.x; i < ntop * 4; i += BLOCK) s_top[i] = g[i];
        __syncthreads();
        st.top = (const lds_u4*)s_top;
        st.ntop = ntop;
    }
    uint32_t rays = 0;
    TravCount cnt;
    const int64_t items = ROW ? (int64_t)a.tile_rows : a.slots;
    // ROW: lane l < row_lanes of wave v takes rows v*row_lanes + l, strided
    // over the grid's waves (one chain per lane, spread over the SIMDs)
    const int64_t first = ROW ? (lane_id() < a.row_lanes ? (gtid >> 6) * a.row_lanes + lane_id() : items) : gtid;
    const int64_t stride = ROW ? (int64_t)gridDim.x * (BLOCK / 64) * a.row_lanes : (int64_t)gridDim.x * BLOCK;
    for (int64_t w = first; w < items; w += stride) {
        if (ROW) {
            int lr = (int)w;
            int y = tile_row_to_y(a, lr);
            uint32_t rng = row_seed((uint32_t)y);  // main.cpp:204, unmodified
            for (int x = 0; x < a.W; ++x)
                out[(int64_t)lr * a.W + x] = render_pixel<COUNT, BLOCK, SL, TOPC>(sv, a, x, y, rng, rays, st, lbuf, cnt);
        } else {
            int lr = (int)(w / a.W), x = (int)(w - (int64_t)lr * a.W);
            int y = tile_row_to_y(a, lr);
            uint32_t rng = pixel_seed((uint32_t)x, (uint32_t)y, (uint32_t)a.W);
            out[w] = render_pixel<COUNT, BLOCK, SL, TOPC>(sv, a, x, y, rng, rays, st, lbuf, cnt);
        }
    }
    flush_counts<BLOCK, COUNT>(counters, rays, cnt);
}

// ============================================================ batched HitScene
// Scene::HitScene (scene.cpp:86-97) over a batch: rays n x {o.xyz, d.xyz}
// with one [tmin, tmax] for all (RANGED = 0), or n x {o.xyz, d.xyz, tmin, tmax}
// (RANGED = 1, the per-call range of scene.h:36-37).  hits n x {pos, normal, t}
// where ids >= 0.
// NEG: the range can start behind the origin (every per-ray range, and a
// single range with tmin < 0): the traversal's far-distance slack by magnitude.
template <bool ANY, bool RANGED, int BLOCK, int SL, bool SOA = false, bool NEG = RANGED>
__global__ void __launch_bounds__(BLOCK) k_intersect(SceneView sv, const float* __restrict__ rays,
                                                     int64_t n, float tmin, float tmax,
                                                     float* __restrict__ hits,
                                                     int32_t* __restrict__ ids,
                                                     uint32_t* __restrict__ ovf)
{
    __shared__ uint32_t s_stack[SL * BLOCK];
    const int64_t gtid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    TravStack<BLOCK, SL> st{&s_stack[threadIdx.x], ovf + gtid * (kStackTotal - SL)};
    TravCount cnt;
    constexpr int kStride = RANGED ? 8 : 6;
    for (int64_t i = gtid; i < n; i += (int64_t)gridDim.x * BLOCK) {
        const float* r = rays + kStride * i;
        f3 o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
        const float t0 = RANGED ? r[6] : tmin, t1 = RANGED ? r[7] : tmax;
        float t, u, v;
        int id = -1;
        // with the reference's octree: its root box test first (scene.cpp:25)
        if (sv.oct && !octree_root_hit(sv, o, d, t0, t1)) {
            atomicAdd(&sv.oct->ties[1], 1ull);
        } else {
            // a range that may start behind the origin: sign-aware slack (NEG)
            id = traverse<ANY, false, BLOCK, SL, false, SOA, NEG>(sv, make_trav_ray(o, d), t0, t1, t, u, v, st, cnt);
        }
        ids[i] = id;
        if (id >= 0) {
            f3 pos, nrm;
            hit_record(sv, id, u, v, pos, nrm);
            float* h = hits + 7 * i;
            h[0] = pos.x; h[1] = pos.y; h[2] = pos.z;
            h[3] = nrm.x; h[4] = nrm.y; h[5] = nrm.z;
            h[6] = t;
        }
    }
}

// ============================================================ wavefront
// Queues are segmented: the P path slots are cut into kSeg contiguous ranges
// of seg_cap slots (seg_cap a multiple of the 256-slot shade block); segment j
// of a queue holds only entries of slots in range j, at [j*seg_cap, +count_j).
// Every counter and fetch head sits on its own 64-B line, so the producers'
// wave appends and the consumers' chunk reservations spread over kSeg words
// instead of serialising on one (MI355X_MICROARCH.md: one word saturates at
// ~88 atomics/us).
constexpr int kSeg = 64;  // == wave width: one lane probes one segment
static_assert(kSeg == 64, "segment probing maps segments to the 64 lanes of a wave");
constexpr int kCtr = 16;  // words between counters (64 B)
constexpr uint32_t kChunk = 64;  // queue entries a wave reserves per atomic
constexpr uint32_t kSkip = 0x80000000u;  // queue-entry flag: path stopped at kMaxDepth
constexpr uint32_t kDone = 0xFFFFFFFFu;  // depth value of a finished pixel

struct WfState {
    uint32_t* rng;
    uint32_t* smp;
    uint32_t* depth;
    float* col;    // [3][P]
    float* light;  // [kMaxDepth][P]
    float* ray;    // [6][P]  o.xyz d.xyz
    float* hit;    // [3][P]  t u v
    int32_t* hid;  // [P]
    float* sho;    // [3][P] shadow origin
    // Extend queues (per parity): kSeg * nbins sub-queues of seg_cap entries,
    // sub-queue seg * nbins + bin holding the rays of segment seg whose
    // direction falls in octant bin (the low log2(nbins) bits of the sign
    // mask; nbins = 1: no binning), so a wave's 64-entry reservation holds
    // rays from nearby pixels in one octant (sort-by-bounce: every iteration's
    // queue is one bounce).  Counters and fetch heads per sub-queue.
    uint32_t* q[2];
    uint32_t* qs;    // shadow queue: kSeg segments (shadow rays share one direction)
    uint32_t* cnt[2];  // extend sub-queue counts per parity, kSeg * nbins counters (stride kCtr)
    uint32_t* cnt_s;   // shadow queue counts
    uint32_t* head_e;  // fetch heads
    uint32_t* head_s;
    uint32_t* total;   // [0]: entries of the queue the next iteration consumes
    uint32_t* iter_log;  // optional (TMPT_ITER_LOG): per-iteration queue sizes
    unsigned long long* tot;  // [0] extend rays [1] shadow rays [2,3] extend node/tri visits [4,5] shadow
    int64_t P;
    uint32_t seg_cap;
    uint32_t nbins;  // 1, 2, 4 or 8
    int walk_check;  // relaxed head check before a walking wave's atomic (low load, binned queues)
    int root_check;  // RenderArgs::root_check: camera rays (depth 0) take the root box test
};

// octant bin of a direction: bit 0 = x < 0, bit 1 = y < 0, bit 2 = z < 0, low bits only
__device__ __forceinline__ uint32_t dir_bin(f3 d, uint32_t nbins)
{
    const uint32_t o = (uint32_t)signbit(d.x) | ((uint32_t)signbit(d.y) << 1) | ((uint32_t)signbit(d.z) << 2);
    return o & (nbins - 1u);
}

template <int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_wf_generate(RenderArgs a, WfState s)
{
    int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p < kSeg) {  // initial queue: every slot, in slot order, in bin 0 of its segment
        int64_t lo = p * s.seg_cap;
        int64_t c = s.P - lo;
        s.cnt[0][p * s.nbins * kCtr] = (uint32_t)(c < 0 ? 0 : (c > s.seg_cap ? s.seg_cap : c));
    }
    if (p >= s.P) return;
    int lr = (int)(p / a.W), x = (int)(p - (int64_t)lr * a.W);
    int y = tile_row_to_y(a, lr);
    uint32_t rng = pixel_seed((uint32_t)x, (uint32_t)y, (uint32_t)a.W);
    f3 o, d;
    camera_sample(a.cam, (uint32_t)x, (uint32_t)y, a.invW, a.invH, rng, o, d);
    const int64_t P = s.P;
    s.rng[p] = rng;
    s.smp[p] = 0;
    s.depth[p] = 0;
    s.col[p] = 0.0f; s.col[P + p] = 0.0f; s.col[2 * P + p] = 0.0f;
    s.ray[p] = o.x; s.ray[P + p] = o.y; s.ray[2 * P + p] = o.z;
    s.ray[3 * P + p] = d.x; s.ray[4 * P + p] = d.y; s.ray[5 * P + p] = d.z;
    const int64_t seg = p / s.seg_cap;  // sub-queue (seg, 0) starts at seg * nbins * seg_cap
    s.q[0][seg * s.nbins * s.seg_cap + (p - seg * s.seg_cap)] = (uint32_t)p;
}

// Persistent traversal with lane refill ("dynamic fetch", Aila & Laine 2009,
// re-derived for wave64 and segmented queues): every lane keeps a resumable
// traversal state in registers.  A wave holds a reservation of up to kChunk
// queue entries (uniform, in SGPRs); whenever >= REFILL lanes are idle they
// take the next entries of the reservation (ballot + mbcnt ranks).  An empty
// reservation is renewed by ONE atomic on the head of the wave's current
// segment; exhausted segments are skipped, starting from the wave's own, so
// waves work on nearby pixels and the heads see few atomics.  Lanes run
// STEPS traversal steps between refill checks, each step of the kind (node or
// leaf) more lanes are waiting for.
template <bool ANY, bool COUNT, int BLOCK, int SL, bool TOPC, int MINW, int STEPS = 4, int REFILL = 8>
__global__ void __launch_bounds__(BLOCK, MINW) k_wf_trace(SceneView sv, WfState s, int parity,
                                                          uint32_t* __restrict__ ovf)
{
    __shared__ uint32_t s_stack[SL * BLOCK];
    const int64_t gtid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    TravStack<BLOCK, SL> st{&s_stack[threadIdx.x], ovf + gtid * (kStackTotal - SL)};
    if (TOPC) {  // the top BVH4 levels in LDS (as k_path)
        __shared__ uint4 s_top[TOPC ? kTopNodes * 4 : 1];
        const uint32_t ntop = (uint32_t)min(kTopNodes, sv.n_nodes4);
        const uint4* g = reinterpret_cast<const uint4*>(sv.nodes4);
        for (uint32_t i = threadIdx.x; i < ntop * 4; i += BLOCK) s_top[i] = g[i];
        __syncthreads();
        st.top = (const lds_u4*)s_top;
        st.ntop = ntop;
    }
    TravCount cnt;
    uint32_t traced = 0;
    const uint32_t* q = ANY ? s.qs : s.q[parity];
    const uint32_t* counts = ANY ? s.cnt_s : s.cnt[parity];
    uint32_t* heads = ANY ? s.head_s : s.head_e;
    const int64_t P = s.P;
    const f3 ldir = light_dir();
    const uint64_t lt = (1ull << lane_id()) - 1ull;
    const uint32_t wave_gid = (uint32_t)(gtid >> 6);
    const uint32_t nq = ANY ? (uint32_t)kSeg : (uint32_t)kSeg * s.nbins;  // sub-queues
    uint32_t seg = wave_gid % nq;  // current sub-queue; starts spread over the frame
    bool drained = false;
    uint32_t walked = 0;
    uint32_t res = 0, res_end = 0;          // reservation [res, res_end) of queue positions
    bool active = false;
    uint32_t p = 0;
    uint32_t steps = 0, max_steps = 0;  // COUNT builds: longest query of this lane
    TravRay r;
    TravState ts;
    for (;;) {
        uint64_t idle = wballot(!active);
        uint32_t nidle = (uint32_t)__popcll(idle);
        if (nidle >= (uint32_t)REFILL && (res < res_end || !drained)) {
            while (res >= res_end && !drained) {  // renew the reservation (wave-uniform)
                const uint32_t c = counts[seg * kCtr];
                uint32_t b = c;
                // at low load (walk_check) a wave walking past its own
                // sub-queue takes a relaxed look at the head first, so an
                // exhausted sub-queue costs no atomic (every wave walks all of
                // them at the end of an iteration: 1/8 shard 310 -> 193 ms);
                // at full load that extra round trip per renewal costs more
                // than it saves (N = 1: 550 -> 773 ms), so the atomic alone
                if (c != 0 && (walked == 0 || !s.walk_check ||
                               __hip_atomic_load(&heads[seg * kCtr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < c)) {
                    if (lane_id() == 0) b = atomicAdd(&heads[seg * kCtr], kChunk);
                    b = (uint32_t)__shfl((int)b, 0);
                }
                if (b < c) {
                    res = seg * s.seg_cap + b;
                    res_end = seg * s.seg_cap + min(b + kChunk, c);
                    walked = 0;
                } else {  // sequential walk: try the next sub-queue, give up after all of them
                    seg = seg + 1 == nq ? 0u : seg + 1;
                    if (++walked == nq) drained = true;
                }
            }
            uint32_t take = min(nidle, res_end - res);
            uint32_t k = (uint32_t)__popcll(idle & lt);
            if (!active && k < take) {
                uint32_t e = q[res + k];
                if (!(e & kSkip)) {  // flagged entries: stopped at kMaxDepth, nothing to trace
                    p = e;
                    f3 o, d;
                    if (ANY) {
                        o = mk(s.sho[p], s.sho[P + p], s.sho[2 * P + p]);
                        d = ldir;
                    } else {
                        o = mk(s.ray[p], s.ray[P + p], s.ray[2 * P + p]);
                        d = mk(s.ray[3 * P + p], s.ray[4 * P + p], s.ray[5 * P + p]);
                    }
                    r = make_trav_ray(o, d);
                    trav_init(ts, kMaxT);
                    ++traced;
                    steps = 0;
                    const bool root_miss = !ANY && s.root_check && s.depth[p] == 0 &&
                                           !octree_root_hit(sv, o, d, kMinT, kMaxT);
                    if (root_miss) atomicAdd(&sv.oct->ties[1], 1ull);
                    if (sv.n > 0 && !ray_has_nan(o, d) && !root_miss) {
                        active = true;
                    } else if (!ANY) {  // provably no hit (NaN ray, empty scene, root box): a counted miss
                        s.hid[p] = -1;
                    }
                }
            }
            res += take;
        }
        if (!wany(active)) {
            if (res >= res_end && drained) break;
            continue;
        }
        if (active) {
            bool done = false;
            for (int k = 0; k < STEPS; ++k) {
                // one step kind per round: inner nodes or leaves, whichever more
                // lanes are waiting for, so each load issues with more lanes
                const uint64_t at_leaf = wballot(!done && ts.node < 0);
                const uint64_t at_node = wballot(!done && ts.node >= 0);
                if (at_leaf == 0 && at_node == 0) break;
                const bool leaf_round = __popcll(at_leaf) > __popcll(at_node);
                // the kind is wave-uniform: a scalar branch to the step that has
                // only that kind's code (as in k_path's voted rounds)
                if (leaf_round) {
                    if (!done && ts.node < 0) {
                        done = trav_step4q2_mixed<COUNT, BLOCK, SL, TOPC, 2>(sv, r, ANY, ts, st, cnt);
                        if (COUNT) ++steps;
                    }
                } else if (!done && ts.node >= 0) {
                    done = trav_step4q2_mixed<COUNT, BLOCK, SL, TOPC, 1>(sv, r, ANY, ts, st, cnt);
                    if (COUNT) ++steps;
                }
            }
            if (done) {
                active = false;
                if (COUNT) max_steps = max(max_steps, steps);
                if (ANY) {
                    if (octree_flag(sv, r, ts)) settle_any(sv, r, kMinT, kMaxT, ts);  // a flat triangle, a crack
                    if (ts.best >= 0) s.light[(int64_t)(s.depth[p] - 1) * P + p] = 0.0f;
                } else {
                    settle_closest<BLOCK, SL, TOPC, false, false>(sv, r, 0.0f, kMinT, kMaxT, ts, st);
                    s.hid[p] = ts.best;
                    s.hit[P + p] = ts.bu;
                    s.hit[2 * P + p] = ts.bv;
                }
            }
        }
    }
    uint32_t rr = wave_sum(traced);
    uint32_t nv = COUNT ? wave_sum(cnt.nodes) : 0u;
    uint32_t nt = COUNT ? wave_sum(cnt.tris) : 0u;
    if (lane_id() == 0) {
        atomicAdd(&s.tot[ANY ? 1 : 0], (unsigned long long)rr);
        if (COUNT) {
            atomicAdd(&s.tot[ANY ? 4 : 2], (unsigned long long)nv);
            atomicAdd(&s.tot[ANY ? 5 : 3], (unsigned long long)nt);
        }
    }
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) max_steps = max(max_steps, (uint32_t)__shfl_xor((int)max_steps, off));
        if (lane_id() == 0) atomicMax(&s.tot[ANY ? 7 : 6], (unsigned long long)max_steps);
    }
}

// shade: one lane per path slot, in slot order, so every state access is
// coalesced.  Every unfinished path was extended this iteration (or stopped at
// kMaxDepth), so each needs exactly one shading step.  Appends (wave-compacted)
// to the block's segment of the other parity's extend queue and of the shadow
// queue; writes finished pixels.
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_wf_shade(SceneView sv, RenderArgs a, WfState s,
                                                    int parity, uint32_t* __restrict__ out)
{
    const int64_t P = s.P;
    const int64_t p64 = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t p = (uint32_t)p64;
    const uint32_t seg = (uint32_t)(((int64_t)blockIdx.x * BLOCK) / s.seg_cap);
    uint32_t depth = p64 < P ? s.depth[p] : kDone;
    bool cont = false, shadow = false;
    uint32_t bin = 0;  // octant bin of the next extend ray
    if (depth != kDone) {
        uint32_t rng = s.rng[p];
        f3 d = mk(s.ray[3 * P + p], s.ray[4 * P + p], s.ray[5 * P + p]);
        int id = depth < (uint32_t)kMaxDepth ? s.hid[p] : -1;
        bool finish = true;
        f3 color = mk(0.0f, 0.0f, 0.0f);
        if (depth < (uint32_t)kMaxDepth) {
            if (id >= 0) {  // Scatter, main.cpp:44-73
                f3 pos, nrm;
                hit_record(sv, id, s.hit[P + p], s.hit[2 * P + p], pos, nrm);
                s.light[(int64_t)depth * P + p] = light_cosine(nrm, d);  // zeroed by shadow if occluded
                s.sho[p] = pos.x; s.sho[P + p] = pos.y; s.sho[2 * P + p] = pos.z;
                f3 rnd = random_unit_vector(rng);
                f3 target = pos + nrm + rnd;
                d = normalize(target - pos);
                s.ray[p] = pos.x; s.ray[P + p] = pos.y; s.ray[2 * P + p] = pos.z;
                s.ray[3 * P + p] = d.x; s.ray[4 * P + p] = d.y; s.ray[5 * P + p] = d.z;
                ++depth;
                shadow = true;
                cont = true;  // depth == kMaxDepth: finished next iteration, after its shadow
                finish = false;
            } else {
                color = sky(d);  // main.cpp:106-107
            }
        }
        if (finish) {
            for (int k = (int)depth - 1; k >= 0; --k)
                color = backward_step(color, s.light[(int64_t)k * P + p]);
            f3 col = mk(s.col[p], s.col[P + p], s.col[2 * P + p]) + color;
            uint32_t smp = s.smp[p] + 1;
            s.smp[p] = smp;
            depth = 0;
            if (smp < (uint32_t)a.spp) {
                s.col[p] = col.x; s.col[P + p] = col.y; s.col[2 * P + p] = col.z;
                int lr = (int)(p / (uint32_t)a.W), x = (int)(p - (uint32_t)lr * (uint32_t)a.W);
                int y = tile_row_to_y(a, lr);
                f3 o;
                if (a.jt) rng = sample_seed(a.jt, smp, pixel_seed((uint32_t)x, (uint32_t)y, (uint32_t)a.W));
                camera_sample(a.cam, (uint32_t)x, (uint32_t)y, a.invW, a.invH, rng, o, d);
                s.ray[p] = o.x; s.ray[P + p] = o.y; s.ray[2 * P + p] = o.z;
                s.ray[3 * P + p] = d.x; s.ray[4 * P + p] = d.y; s.ray[5 * P + p] = d.z;
                cont = true;
            } else {
                out[p] = pack_pixel(col, a.spp_recip);
                depth = kDone;
            }
        }
        s.depth[p] = depth;
        s.rng[p] = rng;
        if (cont && depth != (uint32_t)kMaxDepth) bin = dir_bin(d, s.nbins);
    }
    // the next extend ray into its (segment, octant) sub-queue: one ballot
    // and at most one atomic per wave and bin
    for (uint32_t b = 0; b < s.nbins; ++b) {
        const bool mine = cont && bin == b;
        const uint32_t sq = seg * s.nbins + b;
        const uint32_t qi = wave_append(&s.cnt[parity ^ 1][sq * kCtr], mine);
        if (mine) s.q[parity ^ 1][sq * s.seg_cap + qi] = depth == (uint32_t)kMaxDepth ? (p | kSkip) : p;
    }
    uint32_t si = wave_append(&s.cnt_s[seg * kCtr], shadow);
    if (shadow) s.qs[seg * s.seg_cap + si] = p;
}

// after the extend of `parity` was consumed: zero its counts and the heads;
// publish the size of the next queue for the host's termination check
__global__ void __launch_bounds__(kSeg) k_wf_advance(WfState s, int parity, int it)
{
    int j = threadIdx.x;
    uint32_t next = 0, cur = 0;
    for (uint32_t k = (uint32_t)j; k < (uint32_t)kSeg * s.nbins; k += kSeg) {  // extend sub-queues
        next += s.cnt[parity ^ 1][k * kCtr];
        cur += s.cnt[parity][k * kCtr];
        s.cnt[parity][k * kCtr] = 0;
        s.head_e[k * kCtr] = 0;
    }
    if (s.iter_log) {  // debug: rays of this iteration's extend (consumed queue) and shadow
        uint32_t e = wave_sum(cur);
        uint32_t sh = wave_sum(s.cnt_s[j * kCtr]);
        if (j == 0) {
            s.iter_log[2 * it] = e;
            s.iter_log[2 * it + 1] = sh;
        }
    }
    s.cnt_s[j * kCtr] = 0;
    s.head_s[j * kCtr] = 0;
    next = wave_sum(next);
    if (j == 0) s.total[0] = next;
}

// ============================================================ persistent path engine
// One persistent kernel per frame.  Every lane owns one pixel at a time and
// runs its whole sample sequence (the RNG stream threads through the samples,
// main.cpp:204-218); the extend / shadow / shade stages of the wavefront
// engine become per-lane states scheduled inside the wave:
//   * traversal rounds: lanes with a query in flight (closest hit or shadow,
//     mixed) take STEPS steps; each step runs only the kind (inner node or
//     leaf) that more lanes are waiting for;
//   * shading rounds: once >= SHADE_MIN lanes have a finished query (or none is
//     traversing), those lanes shade (Scatter / sky / backward recurrence /
//     next camera sample / pixel write) and idle lanes take new pixels, a
//     64-pixel reservation per atomic on segmented heads.
// No per-bounce grid-wide synchronisation and no path state in HBM: light
// scalars and the pending bounce ray live in LDS.
// Pixel supply: the tile's pixel ranks are cut into chunks of kChunk;
// segment s owns chunks s, s+kSeg, s+2kSeg, ... and its head counts the
// chunks taken, so all segments together hand out ranks in increasing order
// (the waves walk segments from their own one, one atomic per chunk).  Rank r
// is pixel order[r] (a cost-descending order from a pilot pass) or r itself.
// Streaming row engine (SAMP 4, render_rowstream): the speculative row chains
// of render_rowspec without iterations.  One persistent launch: chaser waves
// (the first blocks, one lane per row) walk each row's chain as soon as the
// unit it needs is done and plan pixel windows ahead of it; worker waves take
// units from the rows' windows and trace them shadow-free.  A unit (row,
// pixel p, offset j) starts at M^(2j) row_seed, like render_rowspec's.
//   slots[row][kRssT + 1]: pixel windows, word = (p+1) << 48 | q << 24 | hi
//     (offsets [q, hi) of pixel p not handed out yet; slot p % kRssT; the last
//     slot is the chain's demand window for the current pixel); workers take
//     offsets by CAS, the chaser plans and extends by CAS
//   res[row][p % kRssT][j % R]: a finished unit, word = ((p+1) << 24 | j) << 28
//     | draws | rays << 14 | closest-hit rays << 19, written by atomicMax, so a
//     late unit of a pixel kRssT back never overwrites a live one
//   chainpos[row] = x << 32 | c: the chain's pixel and next sample's offset
//   list[(row * W + x) * spp + k] = offset of sample k of pixel x on the chain
//   ctl: [0] rows done, [1] abort, [2] chain progress ticks, [3] error, [4] P,
//        [5..11] statistics, [12] block arrival tickets (the first nchase are chasers)
#ifndef TMPT_RSS_T
#define TMPT_RSS_T 8
#endif
constexpr int kRssT = TMPT_RSS_T;
#ifndef TMPT_PATH_STEPS
#define TMPT_PATH_STEPS 16
#endif
#ifndef TMPT_PIX_STEPS
#define TMPT_PIX_STEPS 24
#endif
#ifndef TMPT_ROW_STEPS
#define TMPT_ROW_STEPS 16
#endif
#ifndef TMPT_ROW_SHADE_MIN
#define TMPT_ROW_SHADE_MIN 24
#endif
#ifndef TMPT_SHADE_MIN
#define TMPT_SHADE_MIN 16
#endif
#ifndef TMPT_SPARSE
#define TMPT_SPARSE 2
#endif  // live pixel windows per row at most kRssT - 1 (plus the demand slot)
static_assert(kRssT >= 4 && kRssT <= 31, "the worker's pick key holds the slot in 5 bits");
constexpr uint32_t kRssM24 = 0xFFFFFFu;
struct RsStream {
    unsigned long long* __restrict__ slots;
    unsigned long long* __restrict__ res;
    unsigned long long* __restrict__ chainpos;
    uint32_t* __restrict__ list;
    uint32_t* __restrict__ rowrays;    // [row][2]: chain rays, closest-hit
    uint32_t* __restrict__ lo;         // [row][kRssT]: chaser-private window starts
    uint32_t* __restrict__ ctl;
    const uint32_t* __restrict__ anchors;  // [row][na]: M^(2^15 a) row_seed
    const uint32_t* __restrict__ t1;       // M^(2c), c < 128 (byte tables)
    const uint32_t* __restrict__ t2;       // M^(256 b), b < 128
    uint32_t na, R, rmask;
    uint32_t jlimit;        // na * 2^14: offsets with an anchor
    int nrows, nchase, nw;  // rows, chaser blocks, live pixel windows per row
    float spread;
    // live windows and spread follow the live rows (the load law of the
    // launch-time rule, applied as rows finish): room = room_lanes / live rows;
    // dyn bit 0: windows, bit 1: spread (an option fixes either)
    float room_lanes;
    uint32_t dyn;
    uint32_t watchdog;      // 100-MHz ticks without chain progress before the workers abort
    int test_abort;         // option rowstream_test_abort: chasers leave at once (the abort path's test)
};

// M^(2j) row_seed of row `row` (j < na * 2^14)
__device__ __forceinline__ uint32_t rss_state(const RsStream& S, int row, uint32_t j)
{
    uint32_t s = S.anchors[(size_t)row * S.na + (j >> 14)];
    s = sample_seed(S.t2, (j >> 7) & 127u, s);
    return sample_seed(S.t1, j & 127u, s);
}

struct PathCtl {
    uint32_t* heads;  // kSeg chunk counters, stride kCtr
    uint32_t nchunks;
    // SIMD-balanced first chunks (ordered pass, cost-descending chunks): the
    // wave of rank r on the d-th SIMD to register takes chunk r*nsimd + d (r
    // even) or r*nsimd + nsimd-1-d (r odd), so every SIMD's resident waves sum
    // to about the same work.  Every chunk has a claim word: the first chunk
    // and the segment supply both claim, so a chunk the placement left
    // unassigned (uneven waves per SIMD) is still taken, and none twice.
    // simd_reg = 2 words per hardware SIMD key (waves seen, dense index + 1)
    // plus a dense counter at kSimdKeys*2.  null = off.
    uint32_t* simd_reg;
    uint32_t* claim;  // nchunks words, zeroed per launch
    uint32_t nsimd, wps;
    int64_t P;
    const uint32_t* __restrict__ order;  // rank -> pixel, or null
    uint32_t* __restrict__ cost_out;     // per-pixel traversal steps of this call, or null
    // dynamic issue priority (longest remaining first): each shading round the
    // wave estimates its lanes' remaining traversal steps (steps so far per
    // finished sample x samples left) and sets s_setprio 3/2/1/0 at the
    // thresholds dprio[0] > dprio[1] > dprio[2] (steps); dprio[0] = 0: off.
    // With dprio_cost (the pilot pass's per-pixel steps), the thresholds are
    // fractions of the heaviest pixel's (order[0]) projected remaining steps.
    float dprio[3];
    const uint32_t* __restrict__ dprio_cost;
    uint32_t lane_cap;  // pixels a wave holds at once (64: all lanes)
    uint32_t chunk;     // ranks per chunk (kChunk, or lane_cap when capped)
    // Sample seeding: the supply hands out units = (pixel, block of blk
    // samples), nblk blocks per pixel, unit u = pixel * nblk + block (P counts
    // units).  With nblk > 1 each sample's colour goes to sbuf[s * slots + pixel]
    // and k_resolve sums them in sample order (main.cpp:218's col += Trace).
    uint32_t nblk, blk;
    uint32_t blk0;  // progressive pass: the block of its first sample (units = the pass's blocks)
    // the frame's tail (option sample_tail): units >= ua are single samples,
    // unit ua + v = sample v % blk of block ua + v / blk, so the last units
    // handed out are one sample long, not one block
    uint32_t ua;
    float4* __restrict__ sbuf;
    uint32_t sb_ss, sb_sp;  // sbuf index = sample * sb_ss + pixel * sb_sp ([pixel][sample]: 1, spp)
    uint32_t pair;          // sample pairs (2k, 2k+1) of a unit written back to back (one 32-B sector)
    // Speculative row seeding (SAMP 2, render_rowspec): unit u traces ONE
    // sample of tile pixel upix[u] from RNG state ustate[u] and writes its
    // colour with w = draws | rays << 27 to rs_out[u], and its final RNG state
    // to rs_end[u]
    const uint32_t* __restrict__ upix;
    const uint32_t* __restrict__ ustate;
    float4* __restrict__ rs_out;
    uint32_t* __restrict__ rs_end;
    const uint32_t* __restrict__ p_dev;  // the unit count (replaces P, nchunks at launch)
    // no-shadow speculation (option rowspec_noshadow): the speculative pass skips
    // shadow traversals (they never change a sample's draws); the chain's
    // samples are traced again in full at the end of the frame, unit u as
    // sample uslot[u] of its pixel, colour into sbuf (resolved in order)
    int rs_noshadow;
    const uint32_t* __restrict__ uslot;
    RsStream rss;  // SAMP 4
    // Deferred ties (SAMP 1, k_path DEFER): the main loop carries no octree
    // walk; a sample whose closest-hit query ends on a flagged tie is dropped
    // and (pixel, sample) appended to redo (counters[kRedoCounter] counts them,
    // redo_cap entries are kept, kRedoEmpty until written).  Waves past the
    // main loop trace the listed samples again, ties settled (redo_sample);
    // k_redo takes any they leave.
    uint2* __restrict__ redo;
    float4* __restrict__ redo_state;  // kRedoState4 float4 per slot: where the dropped path stopped
    uint32_t redo_cap;
    uint32_t redo_inline;  // 0 (test hook, option redo_inline): no redo phase, k_redo takes every entry
    uint32_t redo_lanes;   // lanes per wave that take redo tickets (1..64)
    // With the octree: shadow answers can need it too (a flat triangle in the
    // scene, or the light direction can run along a crack; render_persistent
    // decides) -- the finished shadow queries are checked as closest hits are
    // (octree_flag), so HELP and DEFER are off then.
    uint32_t oct_shadow;
};

constexpr uint32_t kSimdKeys = 8u * 8u * 2u * 16u * 4u;  // XCC x SE x SH x CU x SIMD (HW_ID fields)

// Rank of this wave among the waves resident on its SIMD -- its hardware wave
// slot, which the dispatcher fills oldest first, so rank 0 is the wave the
// SIMD's arbiter favours (oldest first) -- and the SIMD's dense registration
// index (PathCtl::simd_reg).  Lane 0 registers; the first wave of a SIMD to
// arrive draws the dense index and publishes it, later ones wait for it (it
// is already running: it won the claim before them).
__device__ __forceinline__ uint2 simd_rank(uint32_t* reg)
{
    uint32_t r = 0, d = 0;
    if (lane_id() == 0) {
        const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;  // XCC_ID
        const uint32_t key = ((((xcc * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u +
                               ((hw >> 8) & 15u)) * 4u) + ((hw >> 4) & 3u);
        r = hw & 15u;  // wave slot
        if (atomicAdd(&reg[2 * key], 1u) == 0) {
            d = atomicAdd(&reg[2 * kSimdKeys], 1u);
            __hip_atomic_store(&reg[2 * key + 1], d + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            uint32_t v;
            while ((v = __hip_atomic_load(&reg[2 * key + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
                __builtin_amdgcn_s_sleep(2);
            d = v - 1u;
        }
    }
    return make_uint2((uint32_t)__shfl((int)r, 0), (uint32_t)__shfl((int)d, 0));
}

__device__ __forceinline__ unsigned long long rss_ld(const unsigned long long* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t rss_ld32(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long rss_win(uint32_t p, uint32_t q, uint32_t hi)
{
    return ((unsigned long long)(p + 1u) << 48) | ((unsigned long long)q << 24) | hi;
}

// The chaser of render_rowstream: lane = row.  Walks the row's chain through
// the finished units (k_rs_chase's walk, main.cpp:209-219), records each chain
// sample's offset, plans pixel windows ahead (k_rs_plan's placement: pixel x + i
// expected i - 1 pixels after the current pixel's expected end, +- spread *
// sqrt(i) pixels) and, when the chain needs an offset no window covers, opens
// it (the demand window for a start before the current window, an extension
// past its end).  Exits when its rows are done or the launch aborts.
template <int BLOCK>
__device__ void rss_chaser(const RenderArgs& a, const RsStream& S, int wave)
{
    const int row = wave * 64 + lane_id();
    const bool mine = row < S.nrows;
    const uint32_t W = (uint32_t)a.W, spp = (uint32_t)a.spp, T = (uint32_t)kRssT;
    uint32_t c = 0, x = 0, k = 0, pdraws = 0, rays = 0, erays = 0, planned = 0;
    uint32_t n_wait = 0, n_ext = 0, n_pre = 0, n_sweep = 0;  // statistics (ctl[8..11])
    uint32_t stuck = 0;  // sweeps the chain has waited at the same (x, c)
    float mean = 17.0f;  // draws per sample before any is seen (k_rs_init)
    float spread = S.spread;
    uint32_t nw = (uint32_t)S.nw;
    bool done = !mine, err = false;
    unsigned long long* slot = S.slots + (size_t)(mine ? row : 0) * (T + 1u);
    uint32_t* lo = S.lo + (size_t)(mine ? row : 0) * T;
    const unsigned long long* res = S.res + (size_t)(mine ? row : 0) * T * S.R;
    const uint32_t cap_span = S.R - 64u;  // live offsets ahead of the chain: under one ring
    // plan pixel q (> x) from the chain's position
    auto plan = [&](uint32_t q) {
        const float E = (float)spp * mean * 0.5f, rest = (float)(spp - k) * mean * 0.5f;
        const float i = (float)(q - x);
        const float P = (float)c + rest + (i - 1.0f) * E;
        const float lo_f = fmaxf((float)c, P - spread * sqrtf(i) * E);
        const float hi_f = P + E + spread * sqrtf(i + 1.0f) * E + 2.0f;
        const uint32_t l = (uint32_t)lo_f, h = min((uint32_t)hi_f, c + cap_span);
        lo[q % T] = l;
        __hip_atomic_exchange(&slot[q % T], rss_win(q, min(l, h), h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (mine) {  // the first pixel from offset 0, then the lookahead windows
        const float E = (float)spp * mean * 0.5f;
        const uint32_t h = min((uint32_t)(E + S.spread * E) + 2u, cap_span);
        lo[0] = 0;
        __hip_atomic_exchange(&slot[0], rss_win(0, 0, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        planned = 0;
        while (planned + 1u < min(W, (uint32_t)S.nw)) plan(++planned);
    }
    for (;;) {
        bool moved = false;
        if (!done) {
            for (int it = 0; it < 64; ++it) {
                const unsigned long long w = rss_ld(res + (size_t)(x % T) * S.R + (c & S.rmask));
                if ((w >> 28) != (((unsigned long long)(x + 1u) << 24) | c)) {
                    // not finished, or no window holds (x, c): looked at once
                    // the chain has waited two sweeps (usually the unit is in flight)
                    if (++stuck < 3u) break;
                    stuck = 0;
                    const unsigned long long sw = rss_ld(&slot[x % T]);
                    const uint32_t q = (uint32_t)(sw >> 24) & kRssM24, hi = (uint32_t)sw & kRssM24;
                    const uint32_t l = lo[x % T];
                    const uint32_t rest = (uint32_t)((float)(spp - k) * mean * 0.65f) + 16u;
                    ++n_wait;
                    if (c < l) {  // the pixel starts before its window: demand [c, l)
                        ++n_pre;
                        __hip_atomic_exchange(&slot[T], rss_win(x, c, min(l, c + cap_span)), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                        lo[x % T] = c;
                    } else if (c >= hi) {  // past the window's end: a new window from c
                        // (everything below hi was handed out; the workers' adds
                        // past hi handed out nothing, so q restarts at c)
                        ++n_ext;
                        __hip_atomic_exchange(&slot[x % T], rss_win(x, c, c + min(rest, cap_span)),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    (void)q;
                    break;
                }
                stuck = 0;
                const uint32_t draws = (uint32_t)w & 0x3FFFu;
                rays += (uint32_t)(w >> 14) & 31u;
                erays += (uint32_t)(w >> 19) & 15u;
                pdraws += draws;
                S.list[((size_t)row * W + x) * spp + k] = c;  // sample k of pixel x: offset c
                c += draws >> 1;
                moved = true;
                if (c + cap_span >= S.jlimit) {  // offsets past the anchors (or 24-bit words): abort, fall back
                    err = true;
                    done = true;
                    break;
                }
                if (++k == spp) {  // pixel done (main.cpp:221-233 packs it in the final pass)
                    mean = (float)pdraws / (float)k;
                    k = 0;
                    pdraws = 0;
                    if (++x == W) {
                        done = true;
                        break;
                    }
                    if (S.dyn) {  // the rows still chasing set the room per row
                        const uint32_t live = (uint32_t)S.nrows - min((uint32_t)S.nrows, rss_ld32(&S.ctl[0]));
                        const float room = S.room_lanes / (float)max(live, 1u);
                        if (S.dyn & 1u)
                            nw = (uint32_t)min((int)kRssT - 1, max(2, (int)rintf(2.6f + 1.5f * __logf(fmaxf(room, 1e-3f)))));
                        if (S.dyn & 2u) spread = fminf(0.25f, fmaxf(0.0f, 0.055f * room - 0.015f));
                    }
                    while (planned + 1u < W && planned < x + nw - 1u) plan(++planned);
                }
            }
            if (moved) __hip_atomic_store(&S.chainpos[row], ((unsigned long long)x << 32) | c, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
            if (done) {
#ifdef TMPT_EXP_WAVETIME
                if (row < kWaveTimeMax) g_rowtime[row] = __builtin_amdgcn_s_memrealtime();
#endif
                S.rowrays[2 * row] = rays;
                S.rowrays[2 * row + 1] = erays;
                if (err) {
                    atomicExch(&S.ctl[3], 1u);
                    atomicExch(&S.ctl[1], 1u);
                }
                __threadfence();
                atomicAdd(&S.ctl[0], 1u);
            }
        }
        const uint64_t mv = wballot(moved);
        if (lane_id() == 0 && mv) atomicAdd(&S.ctl[2], 1u);
        ++n_sweep;
        if (!wany(!done)) break;
        if (rss_ld32(&S.ctl[1]) != 0u) break;  // aborted
        if (!mv) __builtin_amdgcn_s_sleep(8);
    }
    if (mine) {
        atomicAdd(&S.ctl[8], n_wait);
        atomicAdd(&S.ctl[9], n_ext);
        atomicAdd(&S.ctl[10], n_pre);
    }
    if (lane_id() == 0) atomicAdd(&S.ctl[11], n_sweep);
}


template <bool COUNT, int BLOCK, int SL, int STEPS, int SHADE_MIN, int OCC = 1, int TAIL = 0, int PROF = 0,
          int HELP = 0, int SAMP = 0, bool SOA = false, int TIES = 0>
__global__ void __launch_bounds__(BLOCK, OCC) k_path(SceneView sv, RenderArgs a, PathCtl pc,
                                                uint32_t* __restrict__ out,
                                                uint32_t* __restrict__ ovf,
                                                unsigned long long* __restrict__ counters)
{
    // TIES: how closest hits tied on t are answered.  0: the leaf keeps the
    // lowest index beside the tie flag and a flagged query is re-answered over
    // the octree when there is one (else the lowest index stands); 2: the
    // octree is there (the caller guarantees it), so the leaf keeps the first
    // triangle met and only flags the tie, and the octree answers; 1 (DEFER,
    // sample seeding): as 2, but a flagged sample is dropped and traced again
    // in the redo phase -- the main loop carries no octree walk.
    constexpr bool DEFER = TIES == 1, FLAG = TIES != 0;
    __shared__ uint32_t s_stack[SL * BLOCK];
    // SAMP 3, 4 (shadow-free speculation): no light terms, no pending next ray
    __shared__ float s_light[SAMP >= 3 ? 1 : kMaxDepth * BLOCK];
    // OCC 5 (5 waves per SIMD, <= 32 KB of LDS per block): only the scattered
    // ray's direction is kept while its bounce's shadow query runs -- its
    // origin is the shadow ray's (r.o)
    constexpr bool NEXT3 = OCC >= 5;
    __shared__ float s_next[SAMP >= 3 ? 1 : (NEXT3 ? 3 : 6) * BLOCK];
    if (SAMP == 4) {
        // The chaser role goes by arrival, not by blockIdx: the first nchase
        // blocks to START take it, so every chaser is resident by construction
        // and the workers' spin on chain progress cannot wait on a block that
        // the dispatcher holds back behind them.
        __shared__ uint32_t s_ticket;
        if (threadIdx.x == 0) s_ticket = atomicAdd(&pc.rss.ctl[12], 1u);
        __syncthreads();
        const uint32_t ticket = s_ticket;
        if ((int)ticket < pc.rss.nchase) {
            if (!pc.rss.test_abort) rss_chaser<BLOCK>(a, pc.rss, (int)(ticket * (BLOCK / 64) + threadIdx.x / 64));
            return;
        }
    }
    const int64_t gtid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    TravStack<BLOCK, SL> st{&s_stack[threadIdx.x], ovf + gtid * (kStackTotal - SL)};
    constexpr uint32_t LS = BLOCK;  // stride between a lane's LDS entries
    float* light = &s_light[threadIdx.x];
    float* nxt = &s_next[threadIdx.x];
    // HELP: lane ids of this round's offloading lanes, by rank (per wave)
    __shared__ uint8_t s_pair[HELP ? BLOCK : 1];
    {  // the top BVH4 levels (nodes are numbered level by level) in LDS
        // HELP: 4 nodes fewer, so s_pair keeps the block at 4 per CU
        constexpr int kTop = OCC >= 5 ? kTopNodes5 : (HELP ? kTopNodes - 4 : kTopNodes);
        __shared__ uint4 s_top[kTop * 4];
        const uint32_t ntop = (uint32_t)min(kTop, sv.n_nodes4);
        const uint4* g = reinterpret_cast<const uint4*>(sv.nodes4);
        for (uint32_t i = threadIdx.x; i < ntop * 4; i += BLOCK) s_top[i] = g[i];
        __syncthreads();
        st.top = (const lds_u4*)s_top;
        st.ntop = ntop;
    }
    // SAMP: the sample kernel has none of pixel mode's pilot order, balanced
    // first chunks, priorities or progressive state; compiling them out frees
    // the scalar registers they held
    constexpr bool kFull = !SAMP;
    float dp0 = kFull ? pc.dprio[0] : 0.0f, dp1 = kFull ? pc.dprio[1] : 0.0f, dp2 = kFull ? pc.dprio[2] : 0.0f;
    if (kFull && pc.dprio_cost && pc.order && a.smp_begin > 0) {  // relative thresholds (wave-uniform)
        const float sc = (float)pc.dprio_cost[pc.order[0]] * (float)(a.smp_end - a.smp_begin) / (float)a.smp_begin;
        dp0 *= sc;
        dp1 *= sc;
        dp2 *= sc;
    }
    TravCount cnt, cnt_s;  // COUNT: closest-hit and shadow queries apart
    uint32_t rays_e = 0, rays_s = 0;
    const f3 ldir = light_dir();
    const uint64_t lt = (1ull << lane_id()) - 1ull;
    uint32_t seg = (uint32_t)(gtid >> 6) % kSeg, walked = 0;
    uint32_t res = 0, res_end = 0;
    if (SAMP == 2 || SAMP == 3) {  // the speculative row engine plans its units on the device
        pc.P = *pc.p_dev;
        pc.nchunks = (uint32_t)((pc.P + pc.chunk - 1) / pc.chunk);
    }
    bool exhausted = SAMP == 4 ? false : pc.P == 0;
    // SAMP 4: the row the wave takes units from (it moves on when that row has
    // none), the row and pixel of its reservation, the watchdog's last seen
    // chain progress and when it changed
    uint32_t crow = SAMP == 4 ? (uint32_t)((gtid >> 6) % (int64_t)max(1, pc.rss.nrows)) : 0u;
    uint32_t srow = 0, spx = 0, wd_tick = 0, n_claim = 0, n_miss = 0, n_cas = 0;  // (ctl[5..7])
    uint32_t crow_rng = (uint32_t)(gtid >> 6) * 2654435761u + 1u;
    uint64_t wd_time = 0;
    if (kFull && pc.simd_reg && !exhausted) {  // SIMD-balanced first chunk
        const uint2 rd = simd_rank(pc.simd_reg);
        if (rd.x < pc.wps && rd.y < pc.nsimd) {
            const uint32_t c = rd.x * pc.nsimd + ((rd.x & 1u) ? pc.nsimd - 1u - rd.y : rd.y);
            uint32_t got = 0;
            if (c < pc.nchunks && lane_id() == 0) got = atomicExch(&pc.claim[c], 1u) == 0u;
            if (__shfl((int)got, 0)) {
                res = c * pc.chunk;
                res_end = (uint32_t)min<int64_t>((int64_t)res + pc.chunk, pc.P);
            } else if (c < pc.nchunks && lane_id() == 0) {
                atomicAdd(&counters[21], 1ull);  // balance diagnostics: lost the claim
            }
        } else if (lane_id() == 0) {
            atomicAdd(&counters[20 + (rd.x >= pc.wps ? 2 : 3)], 1ull);  // slot beyond wps / no dense index
        }
        // a wave left without a first chunk waits ~20 us before the segment
        // supply, so it does not take a chunk another wave is about to claim
        if (res >= res_end)
            for (int k = 0; k < 6; ++k) __builtin_amdgcn_s_sleep(127);
    }
#ifdef TMPT_EXP_WAVETIME
    const int wt_id = (int)(gtid >> 6);
    if (lane_id() == 0 && wt_id < kWaveTimeMax) g_wavetime[3 * wt_id] = __builtin_amdgcn_s_memrealtime();
#endif
    bool has_pix = false, in_query = false, qany = false;
    // HELP (shadow offload to idle lanes): once the pixel supply is exhausted, a
    // lane without a pixel becomes a helper that traces another lane's shadow
    // query (Scatter's HitScene toward the light only gates that bounce's light
    // term, main.cpp:57-67: it feeds neither the RNG stream nor the path), so
    // the owner's chain goes on with the scattered ray at once.  The owner's
    // light slot holds -cosine while the answer is pending (the cosine is > 0
    // whenever a shadow query is traced); the helper writes 0 (occluded) or
    // the cosine.  A path whose slots are still pending waits (`waiting`)
    // before its backward recurrence.
    bool helper = false, waiting = false;
    uint32_t hown = 0;  // helper: owner lane << 4 | light slot
    uint32_t pix = 0, rng = 0, smp = 0, depth = 0;
    // SAMP: the four jump-table words of the next sample's seed, loaded one
    // camera phase ahead (pf_smp = the sample they belong to), so a new sample
    // does not wait for their memory round trip
    uint32_t pf0 = 0, pf1 = 0, pf2 = 0, pf3 = 0, pf_smp = 0xFFFFFFFFu, pf_pix = 0;
    // SAMP 2: the unit held, the ray counts at its start, the camera's RNG draws
    uint32_t cur_unit = 0, re0 = 0, rs0 = 0, ndraw = 0;
    bool single = false;  // SAMP 1: the unit is one sample of the frame's tail (PathCtl::ua)
    uint32_t psteps = 0;  // traversal steps of this pixel in this call (pc.cost_out)
    // COUNT: wave-uniform round statistics (node/leaf rounds and their stepping
    // lanes, shading rounds, lanes wanting shading, lanes traversing meanwhile)
    uint64_t rs_nr = 0, rs_nl = 0, rs_lr = 0, rs_ll = 0, rs_sr = 0, rs_sl = 0, rs_st = 0;
    // PROF: wave-uniform s_memtime cycles in shading rounds, node rounds, leaf rounds
    uint64_t pt_shade = 0, pt_node = 0, pt_leaf = 0, pt_t = PROF ? stamp() : 0;
    // PROF >= 2: the shading round split (pixel fetch, hit/finish shading, camera, query set-up)
    uint64_t ps_fetch = 0, ps_shade = 0, ps_cam = 0, ps_start = 0;
    f3 col = mk(0.0f, 0.0f, 0.0f);
    TravRay r;
    TravState ts;
    trav_init(ts, kMaxT);

    for (;;) {
        const bool wants = has_pix ? !in_query : (HELP && helper ? !in_query : !exhausted);
        const uint64_t need = wballot(wants);
        const uint64_t trav = wballot(in_query);
        // Sparse waves (TAIL = D > 0): a wave shades once SHADE_MIN lanes wait, or
        // -- when fewer than D*SHADE_MIN lanes still hold a pixel -- once 1/D of
        // them wait, so the last pixels of a wave (the frame's critical path at
        // low load) do not idle until every other lane's query has finished.
        int shade_min = SHADE_MIN;
        if (TAIL > 0) {
            const int act = __popcll(wballot(has_pix));
            shade_min = max(1, min(SHADE_MIN, act / TAIL));
        }
        if (need != 0 && (__popcll(need) >= shade_min || trav == 0)) {
            if (COUNT || PROF >= 3) {
                ++rs_sr;
                rs_sl += (uint64_t)__popcll(need);
                rs_st += (uint64_t)__popcll(trav);
            }
            // Each lane decides at most one next query this round; camera
            // sampling and the query set-up are emitted once, after the
            // branches, so the wave runs each at most once per round.
            bool cam = false, start = false, sany = false;
            f3 so = mk(0.0f, 0.0f, 0.0f), sd = so;
            // ---- new pixels for idle lanes (wave-uniform reservation)
            const uint64_t nopix = wballot(!has_pix && !(HELP && helper) && !exhausted);
            if (SAMP == 4 && nopix != 0 && res >= res_end && !exhausted) {
                // offsets of one pixel window, as many as the wave has idle
                // lanes (a held reservation would delay units the chain may be
                // waiting for): the row's demand window first, then its live
                // windows in pixel order.  Lane i < T reads slot i, lane T the
                // demand slot; the pick takes its offsets with one fetch-add,
                // and the word it returns says which window they belong to
                // (the chaser may have re-planned the slot meanwhile), so no
                // offset handed out is ever lost; adds past a window's end
                // hand out nothing.
                const RsStream& S = pc.rss;
                const uint32_t T = (uint32_t)kRssT;
                // a wave with lanes still tracing looks at 1 row per round, an idle one at 4
                const int natt = wany(has_pix) ? 1 : 4;
                for (int att = 0; att < natt && res >= res_end; ++att) {
                    const uint32_t x = (uint32_t)(rss_ld(&S.chainpos[crow]) >> 32);
                    bool moved_on = true;
                    if (x < (uint32_t)a.W) {
                        unsigned long long* sl = S.slots + (size_t)crow * (T + 1u);
                        const uint32_t ln = (uint32_t)lane_id();
                        unsigned long long w = 0;
                        if (ln <= T) w = rss_ld(&sl[ln]);
                        const uint32_t p1 = (uint32_t)(w >> 48), q = (uint32_t)(w >> 24) & kRssM24;
                        const uint32_t hi = (uint32_t)w & kRssM24;
                        const bool valid = ln <= T && p1 > x && p1 <= (uint32_t)a.W && q < hi;
                        // priority: demand, then the lowest pixel; key unique per lane
                        uint32_t key = valid ? (((ln == T ? 0u : p1 - x) << 5) | ln) : 0xFFFFFFFFu;
                        // (over all 64 lanes: the pick must be wave-uniform)
                        for (int off = 1; off < 64; off <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, off));
                        if (key != 0xFFFFFFFFu) {
                            moved_on = false;
                            const int pick = (int)(key & 31u);
                            uint32_t got = 0, gq = 0, gp = 0;
                            if (ln == (uint32_t)pick) {
                                const uint32_t n = min((uint32_t)__popcll(nopix), hi - q);
                                const unsigned long long old = atomicAdd(&sl[ln], (unsigned long long)n << 24);
                                const uint32_t op = (uint32_t)(old >> 48), oq = (uint32_t)(old >> 24) & kRssM24;
                                const uint32_t ohi = (uint32_t)old & kRssM24;
                                if (op != 0u && oq < ohi) {
                                    got = min(n, ohi - oq);
                                    gq = oq;
                                    gp = op - 1u;
                                }
                            }
                            got = (uint32_t)__shfl((int)got, pick);
                            if (!got) ++n_cas;
                            if (got) {
                                ++n_claim;
#ifdef TMPT_EXP_WAVETIME  // the row workers: when each wave last found speculation work
                                if (lane_id() == 0 && wt_id < kWaveTimeMax)
                                    g_claimtime[wt_id] = __builtin_amdgcn_s_memrealtime();
#endif
                                res = (uint32_t)__shfl((int)gq, pick);
                                res_end = res + got;
                                srow = crow;
                                spx = (uint32_t)__shfl((int)gp, pick);
                            }
                        }
                    }
                    if (moved_on) {  // no work there: a pseudo-random next row spreads the waves
                        ++n_miss;
                        crow_rng ^= crow_rng << 13;
                        crow_rng ^= crow_rng >> 17;
                        crow_rng ^= crow_rng << 5;
                        crow = crow_rng % (uint32_t)S.nrows;
                        // (taking the laggier of two random rows instead measured within
                        // noise: profiles/r05_experiments/row_pick2.log)
                    }
                }
                if (res >= res_end && (rss_ld32(&S.ctl[0]) >= (uint32_t)S.nrows || rss_ld32(&S.ctl[1]) != 0u))
                    exhausted = true;  // every row's chain is done (or the launch aborted)
            }
            if (nopix != 0) {
                while (SAMP != 4 && res >= res_end && !exhausted) {
                    // chunks of segment seg: seg, seg + kSeg, ...
                    const uint32_t c = seg < pc.nchunks ? (pc.nchunks - 1u - seg) / (uint32_t)kSeg + 1u : 0u;
                    uint32_t b = c;
                    if (c != 0) {
                        if (lane_id() == 0) b = atomicAdd(&pc.heads[seg * kCtr], 1u);
                        b = (uint32_t)__shfl((int)b, 0);
                    }
                    if (b < c && kFull && pc.claim) {  // taken as some wave's balanced first chunk?
                        uint32_t got = 0;
                        if (lane_id() == 0) got = atomicExch(&pc.claim[seg + b * (uint32_t)kSeg], 1u) == 0u;
                        if (!__shfl((int)got, 0)) continue;
                    }
                    if (b < c) {
                        res = (seg + b * (uint32_t)kSeg) * pc.chunk;
                        res_end = (uint32_t)min<int64_t>((int64_t)res + pc.chunk, pc.P);
                    } else {
                        seg = (seg + 1) & 63u;
                        if (++walked == kSeg) exhausted = true;
                    }
                }
                uint32_t take = min((uint32_t)__popcll(nopix), res_end - res);
                if (pc.lane_cap < 64u)  // low load: pixels spread over all resident waves
                    take = min(take, pc.lane_cap - min(pc.lane_cap, (uint32_t)__popcll(wballot(has_pix))));
                const uint32_t k = (uint32_t)__popcll(nopix & lt);
                if (!has_pix && ((nopix >> lane_id()) & 1ull) && k < take) {
                    uint32_t smp0 = (uint32_t)a.smp_begin;
                    if (SAMP == 4) {  // streaming row engine: offset res + k of pixel spx of row srow
                        cur_unit = res + k;
                        pix = srow * (uint32_t)a.W + spx;
                        re0 = rays_e;
                        rs0 = rays_s;
                    } else if (SAMP >= 2) {  // speculative row seeding: one sample from a given state
                        cur_unit = res + k;
                        // no unit arrays: the chain list's unit u is sample u % spp of tile pixel u / spp
                        pix = pc.upix ? pc.upix[cur_unit] : cur_unit / (uint32_t)a.spp;
                        if (pc.uslot) smp0 = pc.uslot[cur_unit];
                        else if (!pc.upix) smp0 = cur_unit - pix * (uint32_t)a.spp;
                        re0 = rays_e;
                        rs0 = rays_s;
                    } else if (SAMP && pc.nblk > 1) {  // sample seeding: (pixel, block) units
                        const uint32_t unit = res + k;
                        uint32_t q = unit, sub = 0u;  // block, sample within it (tail units)
                        single = unit >= pc.ua;
                        if (single) {
                            const uint32_t v = unit - pc.ua, qv = v / pc.blk;
                            q = pc.ua + qv;
                            sub = v - qv * pc.blk;
                        }
                        pix = q / pc.nblk;
                        smp0 = (q - pix * pc.nblk + pc.blk0) * pc.blk + sub;  // blk0: a progressive pass's first block
                    } else {
                        pix = (kFull && pc.order) ? pc.order[res + k] : res + k;
                    }
                    psteps = 0;
                    has_pix = true;
                    const int lr = (int)(pix / (uint32_t)a.W);
                    const int x = (int)(pix - (uint32_t)lr * (uint32_t)a.W);
                    if (SAMP == 4) {
                        rng = rss_state(pc.rss, (int)srow, cur_unit);
                    } else if (SAMP >= 2) {
                        rng = pc.ustate[cur_unit];
                    } else if (!kFull || a.smp_begin == 0) {
                        rng = pixel_seed((uint32_t)x, (uint32_t)tile_row_to_y(a, lr), (uint32_t)a.W);
                        col = mk(0.0f, 0.0f, 0.0f);
                    } else {  // progressive: continue the previous pass's stream and sum
                        const float4 pv = a.prog[pix];
                        col = mk(pv.x, pv.y, pv.z);
                        rng = __float_as_uint(pv.w);
                    }
                    smp = smp0;
                    depth = 0;
                    cam = true;
                }
                res += take;
            }
            if (HELP && helper && !in_query) {  // deliver a finished offloaded shadow query
                float* ol = &s_light[(threadIdx.x & ~63u) + (hown >> 4) + (hown & 15u) * BLOCK];
                const float v = *ol;
                *ol = ts.best >= 0 ? 0.0f : -v;
                helper = false;
            }
            if (HELP) __atomic_signal_fence(__ATOMIC_SEQ_CST);
            uint64_t ps_t = 0;
            if (PROF >= 2) {
                ps_t = stamp();
                ps_fetch += ps_t - pt_t;
            }
            // Finished closest hits flagged as ties (not DEFER): each answered
            // over the octree by the whole wave (octree_walk_wave), one after
            // another -- here, where every lane is active.  A HELP lane
            // waiting on shadow answers holds no fresh query.
            // (the row engines, SAMP >= 2, answer in the closest-hit branch
            // with the serial walk: the wave walk's registers spill there --
            // row seeding 927 -> 888 MRays/s)
            // Also the crack queries (octree_flag), and -- where the host says a
            // shadow answer can need it (PathCtl::oct_shadow: a flat triangle in
            // the scene, or a light direction that can run along a crack) --
            // finished shadow queries whose hit the reference may not see: the
            // walk's closest answer gives their hit / miss bit.
            bool settled = false;
            if (!DEFER && SAMP < 2) {
                const bool fin = has_pix && !in_query && !cam && !(HELP && waiting) && (!qany || pc.oct_shadow);
                uint64_t T = wballot(fin && octree_flag(sv, r, ts));
                if (T != 0) {
                    const OctView* ov = sv.oct;
                    do {
                        const int l = (int)__builtin_ctzll(T);
                        T &= T - 1;
                        const f3 qo = mk(rlane(r.o.x, l), rlane(r.o.y, l), rlane(r.o.z, l));
                        const f3 qd = mk(rlane(r.d.x, l), rlane(r.d.y, l), rlane(r.d.z, l));
                        const OctHit h = octree_walk_wave(ov->nodes, ov->refs, ov->n, sv.tri_orig, qo, qd, kMinT, kMaxT,
                                                          rlane(qany ? -INFINITY : ts.bt, l) TMPT_CHK_ARGS(sv));
                        if (lane_id() == l) {
                            octree_count(ov, ts.best);
                            ts.best = h.best;
                            ts.bt = h.t;
                            ts.bu = h.u;
                            ts.bv = h.v;
                            settled = true;
                        }
                    } while (T != 0);
                }
            }
            // ---- finished queries: shade
            bool finish = false, want_off = false;
            f3 color = mk(0.0f, 0.0f, 0.0f);
            if (has_pix && !in_query && !cam) {
                if (HELP && waiting) {  // path ended, shadow answers were pending
                    finish = true;
                    if (depth < (uint32_t)kMaxDepth) color = sky(r.d);
                } else if (!qany) {  // closest hit (Trace, main.cpp:91-109)
                    // the triangle index (2 x index | tie flag in the leaves'
                    // records); a tie was answered over the octree at the top of
                    // the round, or (DEFER) drops the sample here
                    bool drop = false;
                    if (DEFER) {
                        // the deferring kernel: a tied sample is dropped here
                        // (its rays so far uncounted: depth + 1 closest-hit
                        // queries and one shadow query per earlier hit) and
                        // traced again whole by redo_sample.  It finishes at
                        // once with colour x = -1 (no path colour is negative),
                        // which the colour-buffer stores below skip.
                        drop = octree_flag(sv, r, ts);
                        if (wany(drop)) {
                            if (drop) {
                                const unsigned long long slot = atomicAdd(&counters[kRedoCounter], 1ull);
                                // write-through (sc1): a plain store would sit in this
                                // XCD's L2, unseen by a waiting lane on another XCD
                                // until evicted, and its write-back at the kernel's end
                                // could land after that lane's done-mark and undo it
                                // (k_redo then traced the sample again: rays counted
                                // twice -- MI355X_MICROARCH.md, per-XCD L2s)
                                if (slot < (unsigned long long)pc.redo_cap) {
                                    redo_state_put(pc.redo_state + (size_t)slot * kRedoState4, r.o, r.d, rng, light,
                                                   depth, LS);
                                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // state before entry
                                    redo_put(pc.redo + slot, pix, smp | (depth << 16));
                                }
                                // the re-trace counts this query again and the rest of the
                                // path; the bounces before it stay counted here
                                rays_e -= 1u;
                                depth = 0;
                                ts.best = -1;
                            }
                        }
                        ts.best >>= 1;  // -1 stays -1
                    } else if (SAMP >= 2) {
                        const bool tie = octree_flag(sv, r, ts);
                        if (wany(tie)) {
                            if (tie) settle_closest<BLOCK, SL, true, SOA, false>(sv, r, 0.0f, kMinT, kMaxT, ts, st);
                        }
                        if (!tie) ts.best >>= 1;
                    } else if (!settled) {
                        ts.best >>= 1;  // the index (a tie was answered above)
                    }
                    if (ts.best >= 0) {  // Scatter, main.cpp:44-73
                        // the hit record's loads go out first; RandomUnitVector
                        // (RNG + sincos, independent of them) runs while they are
                        // in flight -- the same draws, the same values
                        const float4* hp = reinterpret_cast<const float4*>(sv.tri_orig + ts.best);
                        float4 ha = hp[0], hb = hp[1], hc = hp[2];
                        f3 rnd = random_unit_vector(rng);
                        materialize(ha, hb, hc);
                        const f3 nrm = mk(hc.y, hc.z, hc.w);
                        const f3 pos = hit_pos(mk(ha.x, ha.y, ha.z), mk(ha.w, hb.x, hb.y), mk(hb.z, hb.w, hc.x),
                                               ts.bu, ts.bv);
                        const float lc = light_cosine(nrm, r.d);
                        if (SAMP < 3) light[depth * LS] = lc;  // zeroed if occluded
                        f3 target = pos + nrm + rnd;
                        f3 nd = normalize(target - pos);
                        ++depth;
                        if (SAMP < 3 && lc > 0.0f && !(SAMP == 2 && pc.rs_noshadow)) {
                            if (NEXT3) {
                                nxt[0] = nd.x; nxt[LS] = nd.y; nxt[2 * LS] = nd.z;
                            } else {
                                nxt[0] = pos.x; nxt[LS] = pos.y; nxt[2 * LS] = pos.z;
                                nxt[3 * LS] = nd.x; nxt[4 * LS] = nd.y; nxt[5 * LS] = nd.z;
                            }
                            start = true;  // shadow query toward the light
                            sany = true;
                            so = pos;
                            sd = ldir;
                            want_off = HELP != 0;
                        } else {  // nothing to trace (no light term)
                            // The reference still calls HitScene for the shadow ray
                            // (main.cpp:57, counted), but a surface turned away from
                            // the light adds max(0, cos) = 0 whatever it answers
                            // (main.cpp:59-67): count the query, skip the traversal.
                            ++rays_s;
                            if (depth < (uint32_t)kMaxDepth) {
                                start = true;  // the scattered ray of this bounce
                                so = pos;
                                sd = nd;
                            } else {
                                finish = true;  // kMaxDepth hits, colour stays 0 (main.cpp:88-89)
                            }
                        }
                    } else {
                        color = sky(r.d);  // main.cpp:106-107
                        if (DEFER && drop) color.x = -1.0f;
                        finish = true;
                    }
                } else if (SAMP < 3) {  // shadow query of bounce depth-1
                    if (SAMP == 2 && pc.oct_shadow && octree_flag(sv, r, ts))
                        settle_any(sv, r, kMinT, kMaxT, ts);  // the row engines' serial walk (pixel, sample: above)
                    if (ts.best >= 0) light[(depth - 1) * LS] = 0.0f;
                    if (depth < (uint32_t)kMaxDepth) {
                        start = true;  // the scattered ray of that bounce
                        if (NEXT3) {  // the shadow ray started at the hit point
                            so = r.o;
                            sd = mk(nxt[0], nxt[LS], nxt[2 * LS]);
                        } else {
                            so = mk(nxt[0], nxt[LS], nxt[2 * LS]);
                            sd = mk(nxt[3 * LS], nxt[4 * LS], nxt[5 * LS]);
                        }
                    } else {
                        finish = true;  // kMaxDepth hits, colour stays 0 (main.cpp:88-89)
                    }
                }
            }
            if (HELP) {  // pair lanes starting a shadow query with idle lanes
                const uint64_t S = wballot(want_off);
                // lanes left without a pixel after this round's fetch (supply
                // exhausted, or the wave's pixel cap reached) are free to help
                const uint64_t I = S ? wballot(!has_pix && !helper && !in_query) : 0ull;
                if (I != 0) {
                    const uint32_t n = min(__popcll(S), __popcll(I));
                    const uint32_t ks = (uint32_t)__popcll(S & lt), ki = (uint32_t)__popcll(I & lt);
                    const uint32_t wb = threadIdx.x & ~63u;
                    if (want_off && ks < n) s_pair[wb + ks] = (uint8_t)lane_id();
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    const bool idle = ((I >> lane_id()) & 1ull) != 0 && ki < n;
                    const int src = idle ? (int)s_pair[wb + ki] : (int)lane_id();
                    const float hx = __shfl(so.x, src), hy = __shfl(so.y, src), hz = __shfl(so.z, src);
                    const uint32_t hs = (uint32_t)__shfl((int)depth, src) - 1u;
                    if (want_off && ks < n) {  // offloaded: go on with the scattered ray
                        light[(depth - 1) * LS] = -light[(depth - 1) * LS];
                        sany = false;
                        if (depth < (uint32_t)kMaxDepth) {
                            sd = NEXT3 ? mk(nxt[0], nxt[LS], nxt[2 * LS]) : mk(nxt[3 * LS], nxt[4 * LS], nxt[5 * LS]);
                        } else {
                            start = false;
                            finish = true;  // kMaxDepth hits, colour stays 0 (main.cpp:88-89)
                        }
                    }
                    if (idle) {
                        helper = true;
                        hown = ((uint32_t)src << 4) | hs;
                        start = true;
                        sany = true;
                        so = mk(hx, hy, hz);
                        sd = ldir;
                    }
                }
            }
            if (finish) {
                bool pend = false;
                if (HELP)
                    for (int kk = 0; kk < (int)depth; ++kk) pend |= light[kk * LS] < 0.0f;
                waiting = pend;
                if (!pend) {
                    if (SAMP < 3)
                        for (int kk = (int)depth - 1; kk >= 0; --kk)
                            color = backward_step(color, light[kk * LS]);
                    if (SAMP == 2 && pc.sbuf) {  // a chain sample traced in full: k_resolve sums in order
                        typedef float f32x4 __attribute__((ext_vector_type(4)));
                        __builtin_nontemporal_store((f32x4){color.x, color.y, color.z, 0.0f},
                                                    reinterpret_cast<f32x4*>(pc.sbuf + ((size_t)smp * pc.sb_ss +
                                                                                        (size_t)pix * pc.sb_sp)));
                    } else if (SAMP == 4) {  // streaming row engine: the unit's word for the chaser
                        const uint32_t draws = ndraw + 2u * depth;
                        const uint32_t ne = rays_e - re0, nr = ne + rays_s - rs0;  // <= 10, <= 20
                        const uint32_t row = pix / (uint32_t)a.W, p = pix - row * (uint32_t)a.W;
                        if (draws > 0x3FFFu) atomicExch(&pc.rss.ctl[3], 2u);  // cannot happen: 8k disk tries
                        const unsigned long long word =
                            ((((unsigned long long)(p + 1u) << 24) | cur_unit) << 28) |
                            (unsigned long long)(min(draws, 0x3FFFu) | (nr << 14) | (ne << 19));
                        atomicMax(pc.rss.res + ((size_t)row * kRssT + p % kRssT) * pc.rss.R + (cur_unit & pc.rss.rmask),
                                  word);
                    } else if (SAMP >= 2) {  // speculative row seeding: render_rowspec's chase consumes it
                        // draws: the camera's, and RandomUnitVector's 2 at each of the
                        // `depth` hits (main.cpp:71, drawn at the 10th hit too)
                        const uint32_t draws = ndraw + 2u * depth;
                        const uint32_t ne = rays_e - re0, nr = ne + rays_s - rs0;  // <= 10, <= 20
                        // SAMP 3 (the shadow-free pass): no colour, the chain is traced again
                        pc.rs_out[cur_unit] =
                            make_float4(SAMP == 3 ? 0.0f : color.x, SAMP == 3 ? 0.0f : color.y, SAMP == 3 ? 0.0f : color.z,
                                        __uint_as_float(draws | (nr << 23) | (ne << 28)));
                        pc.rs_end[cur_unit] = rng;
                    } else if (SAMP && pc.sbuf) {  // sample seeding, blocks: k_resolve_px sums in sample order
                        typedef float f32x4 __attribute__((ext_vector_type(4)));
                        f32x4* dst = reinterpret_cast<f32x4*>(pc.sbuf + ((size_t)smp * pc.sb_ss + (size_t)pix * pc.sb_sp));
                        // paired stores (pc.pair): an even sample with a successor in
                        // the unit is held in `col` (unused with a colour buffer) and
                        // written with it, back to back into one 32-B sector
                        const bool odd = (smp & 1u) != 0u;
                        if (pc.pair && !odd && !single && smp + 1u < (uint32_t)a.smp_end && ((smp + 1u) & a.bmask) != 0u) {
                            col = color;
                        } else {
                            // DEFER: a dropped sample's slot (x = -1) is redo_sample's
                            if (pc.pair && odd && !single && (!DEFER || !(col.x < 0.0f)))
                                __builtin_nontemporal_store((f32x4){col.x, col.y, col.z, 0.0f}, dst - 1);
                            if (!DEFER || !(color.x < 0.0f))
                                __builtin_nontemporal_store((f32x4){color.x, color.y, color.z, 0.0f}, dst);
                        }
                    } else
                        col = col + color;
                    ++smp;
                    depth = 0;
                    if (smp < (uint32_t)a.smp_end && (!SAMP || ((smp & a.bmask) != 0u && !single))) {
                        cam = true;
                    } else {
                        if (kFull && a.prog) a.prog[pix] = make_float4(col.x, col.y, col.z, __uint_as_float(rng));
                        if (kFull && pc.cost_out) pc.cost_out[pix] = psteps;
                        if (SAMP < 2 && (!SAMP || !pc.sbuf)) out[pix] = pack_pixel(col, a.out_recip);
                        has_pix = false;
                    }
                }
            }
            if (PROF >= 2) {
                const uint64_t t = stamp();
                ps_shade += t - ps_t;
                ps_t = t;
            }
            if (cam) {  // next camera sample of this lane's pixel (main.cpp:212-216)
                const int lr = (int)(pix / (uint32_t)a.W);
                const int x = (int)(pix - (uint32_t)lr * (uint32_t)a.W);
                const uint32_t y = (uint32_t)tile_row_to_y(a, lr);
                if (SAMP == 1) {
                    const uint32_t ps = pixel_seed((uint32_t)x, y, (uint32_t)a.W);
                    rng = (pf_smp == smp && pf_pix == pix) ? (pf0 ^ pf1 ^ pf2 ^ pf3) : sample_seed(a.jt, smp, ps);
                    // the block's next sample: its table words now, XORed at its start
                    const uint32_t* t = a.jt + (size_t)(smp + 1u) * 1024u;
                    const bool more = smp + 1u < (uint32_t)a.smp_end && ((smp + 1u) & a.bmask) != 0u && !single;
                    const uint32_t* tt = more ? t : a.jt;
                    pf0 = tt[ps & 255u];
                    pf1 = tt[256u + ((ps >> 8) & 255u)];
                    pf2 = tt[512u + ((ps >> 16) & 255u)];
                    pf3 = tt[768u + (ps >> 24)];
                    pf_smp = more ? smp + 1u : 0xFFFFFFFFu;
                    pf_pix = pix;
                }
                if (SAMP >= 2) {
                    ndraw = 0;
                    camera_sample(a.cam, (uint32_t)x, y, a.invW, a.invH, rng, so, sd, ndraw);
                } else {
                    camera_sample(a.cam, (uint32_t)x, y, a.invW, a.invH, rng, so, sd);
                }
                start = true;
            }
            if (PROF >= 2) {
                const uint64_t t = stamp();
                ps_cam += t - ps_t;
                ps_t = t;
            }
            if (start) {
                r = make_trav_ray(so, sd);
                trav_init(ts, kMaxT);
                qany = sany;
                if (sany) ++rays_s; else ++rays_e;
                in_query = sv.n > 0 && !ray_has_nan(so, sd);  // NaN ray / no triangles: a counted miss
                if (!DEFER && a.root_check && cam && in_query && !octree_root_hit(sv, so, sd, kMinT, kMaxT)) {
                    in_query = false;  // a camera ray outside the reference's root box: a counted miss
                    atomicAdd(&sv.oct->ties[1], 1ull);
                }
            }
            if (PROF >= 2) ps_start += stamp() - ps_t;
        }
        if (dp0 > 0.0f) {  // longest remaining traversal work first (wave-uniform)
            float rem = 0.0f;
            if (has_pix)
                rem = smp > (uint32_t)a.smp_begin
                          ? (float)psteps * (float)((uint32_t)a.smp_end - smp) *
                                __builtin_amdgcn_rcpf((float)(smp - (uint32_t)a.smp_begin))
                          : 3.0e38f;
            for (int o = 32; o > 0; o >>= 1) rem = fmaxf(rem, __shfl_xor(rem, o));
            if (rem >= dp0) __builtin_amdgcn_s_setprio(3);
            else if (rem >= dp1) __builtin_amdgcn_s_setprio(2);
            else if (rem >= dp2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (PROF) {
            const uint64_t t = stamp();
            pt_shade += t - pt_t;
            pt_t = t;
        }
        if (!wany(in_query)) {
            if (exhausted && !wany(has_pix)) break;
            if (SAMP == 4 && !wany(has_pix)) {  // nothing to take yet: wait for the chasers
                // watchdog: no chain progress anywhere for ~1 s means the
                // chasers cannot run; abort (the host re-renders the frame
                // with render_rowspec) rather than spin forever
                const uint32_t tick = rss_ld32(&pc.rss.ctl[2]);
                const uint64_t now = __builtin_amdgcn_s_memrealtime();  // 100 MHz
                if (tick != wd_tick || wd_time == 0) {
                    wd_tick = tick;
                    wd_time = now;
                } else if (now - wd_time > (uint64_t)pc.rss.watchdog) {
                    if (lane_id() == 0) atomicExch(&pc.rss.ctl[1], 1u);
                    exhausted = true;
                }
                __builtin_amdgcn_s_sleep(32);
            }
            continue;
        }
        for (int k = 0; k < STEPS; ++k) {  // traversal rounds
            // two compares straight to lane masks (a ballot of a combined bool
            // made the compiler materialise it in a VGPR and compare again)
            const uint64_t q = wballot(in_query);
            const uint64_t at_leaf = q & wballot(ts.node < 0);
            const uint64_t at_node = q & ~at_leaf;
            if (q == 0) break;
            // 32-bit counts, so the vote stays a scalar compare (the 64-bit
            // popcount compare was widened onto the VALU)
            const uint32_t n_leaf = (uint32_t)__builtin_popcount((uint32_t)at_leaf) +
                                    (uint32_t)__builtin_popcount((uint32_t)(at_leaf >> 32));
            const uint32_t n_node = (uint32_t)__builtin_popcount((uint32_t)at_node) +
                                    (uint32_t)__builtin_popcount((uint32_t)(at_node >> 32));
            const bool leaf_round = n_leaf > n_node;
            if (COUNT || PROF >= 3) {
                if (!leaf_round) { ++rs_nr; rs_nl += (uint64_t)__popcll(at_node); }
                if (leaf_round) { ++rs_lr; rs_ll += (uint64_t)__popcll(at_leaf); }
            }
            if (!COUNT) {
                // voted round: the kind is wave-uniform, so only its code runs
                // (a scalar branch instead of exec-mask splits around both)
                const bool stepping = in_query && ((ts.node < 0) == leaf_round);
                bool done = false;
                if (leaf_round) {
                    if (stepping) done = trav_step4q2_mixed<false, BLOCK, SL, true, 2, SOA, false, FLAG>(sv, r, qany, ts, st, cnt);
                } else {
                    if (stepping) done = trav_step4q2_mixed<false, BLOCK, SL, true, 1, SOA, false, FLAG>(sv, r, qany, ts, st, cnt);
                }
                if (done) in_query = false;
                if (stepping && ((kFull && pc.cost_out) || dp0 > 0.0f)) ++psteps;
            } else if (in_query && (ts.node < 0) == leaf_round) {
                TravCount c1;
                if (trav_step4q2_mixed<COUNT, BLOCK, SL, true, 0, SOA, false, FLAG>(sv, r, qany, ts, st, c1)) in_query = false;
                TravCount& dst = qany ? cnt_s : cnt;
                dst.nodes += c1.nodes;
                dst.tris += c1.tris;
                if ((kFull && pc.cost_out) || dp0 > 0.0f) ++psteps;
            }
            if (PROF) {
                const uint64_t t = stamp();
                (leaf_round ? pt_leaf : pt_node) += t - pt_t;
                pt_t = t;
            }
        }
    }
#ifdef TMPT_EXP_WAVETIME
    if (lane_id() == 0 && wt_id < kWaveTimeMax) g_wavetime[3 * wt_id + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (DEFER && pc.redo_inline) {
        // Redo phase: the wave's main loop is over; it traces the samples the
        // main loops dropped on ties (one per lane, by ticket), while the other
        // waves finish theirs, so the re-traces fill the frame's tail.  The
        // list is final by a completion count: a lane waits on an entry while
        // some wave of the grid is still in its main loop (kRedoWaves < waves)
        // and leaves once every wave is past it and no ticket below the list
        // length is left.  The grid is the co-resident block count
        // (occupancy_grid), so every wave reaches its redo phase and no entry
        // is left to k_redo (stats redo_late = 0, asserted by the GPU suite).
        // kRedoGuard is only a deadlock guard for a dispatcher that holds
        // blocks back behind resident ones (the GPU shared with another
        // process): after 20 ms in which neither the list nor the count of
        // waves past their main loop changed, the wave leaves its tickets to
        // k_redo.  A wave waits through the frame's tail only, and the count
        // changes every time a wave leaves its main loop (the main loops end
        // within ~2 ms of each other), so a working launch never sees 20 ms
        // without a change; round 5's 250 ms cost each frame of 4 processes
        // sharing one GPU (the gloo rehearsal) a quarter second once the
        // deferral ran at their shard size.  (Counting started waves instead
        // of the grid cost 2 % in register allocation, measured.)
        constexpr uint64_t kRedoGuard = 2000000;  // s_memrealtime ticks (100 MHz): 20 ms
        const unsigned long long waves = (unsigned long long)gridDim.x * (BLOCK / 64);
        // pc.redo_lanes lanes of the wave take tickets: a re-trace is one
        // lane's whole path, so fewer per wave spread them over more waves
        // (the wave waits for its slowest lane).  Bench frame, k_path ms with
        // 64 / 16 / 4 / 1 lanes: 1/8 shard 27.3 / 26.4 / 26.1 / 25.8, N=1
        // 184.8 / 184.9 / 184.5 (profiles/r04_ties/redo_lanes_*.log): 4
        uint32_t t = 0;
        if (lane_id() == 0) {
            atomicAdd(&counters[kRedoWaves], 1ull);
            t = (uint32_t)atomicAdd(&counters[kRedoTaken], (unsigned long long)pc.redo_lanes);
        }
        t = lane_id() < pc.redo_lanes ? (uint32_t)__shfl((int)t, 0) + lane_id() : 0xFFFFFFFFu;
        unsigned long long seen = ~0ull;
        uint64_t since = 0;
        for (;;) {
            const unsigned long long listed =
                __hip_atomic_load(&counters[kRedoCounter], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t lim = (uint32_t)min(listed, (unsigned long long)pc.redo_cap);
            uint2 e = make_uint2(kRedoEmpty, 0u);
            if (t < lim) e = redo_load(pc.redo + t);
            const bool have = e.x < kRedoDone;
            if (wany(have)) {
                if (have) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the entry before its state
                    redo_sample<BLOCK, SL>(sv, a, e.x, e.y, pc.redo_state + (size_t)t * kRedoState4, pc.sbuf, pc.sb_ss,
                                           pc.sb_sp, rays_e, rays_s, st, light);
                    redo_mark(pc.redo + t);
                    atomicAdd(&counters[kRedoTraced], 1ull);
                    t = (uint32_t)atomicAdd(&counters[kRedoTaken], 1ull);
                }
                since = 0;
                continue;
            }
            const unsigned long long past =
                __hip_atomic_load(&counters[kRedoWaves], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (past >= waves && !wany(t < lim)) break;
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            const unsigned long long sig = (past << 40) ^ listed;
            if (sig != seen || since == 0) {
                seen = sig;
                since = now;
            } else if (now - since > kRedoGuard) {
                break;
            }
            __builtin_amdgcn_s_sleep(16);
        }
    }
#ifdef TMPT_EXP_WAVETIME
    if (lane_id() == 0 && wt_id < kWaveTimeMax) g_wavetime[3 * wt_id + 2] = __builtin_amdgcn_s_memrealtime();
#endif
    if (SAMP == 4 && lane_id() == 0) {
        atomicAdd(&pc.rss.ctl[5], n_claim);
        atomicAdd(&pc.rss.ctl[6], n_miss);
        atomicAdd(&pc.rss.ctl[7], n_cas);
    }
    uint32_t re = wave_sum(rays_e), rs = wave_sum(rays_s);
    uint32_t nv = COUNT ? wave_sum(cnt.nodes) : 0u;
    uint32_t nt = COUNT ? wave_sum(cnt.tris) : 0u;
    uint32_t nvs = COUNT ? wave_sum(cnt_s.nodes) : 0u;
    uint32_t nts = COUNT ? wave_sum(cnt_s.tris) : 0u;
    if (lane_id() == 0) {
        atomicAdd(&counters[0], (unsigned long long)(re + rs));
        atomicAdd(&counters[3], (unsigned long long)re);
        if (COUNT) {
            atomicAdd(&counters[1], (unsigned long long)nv);
            atomicAdd(&counters[2], (unsigned long long)nt);
            atomicAdd(&counters[4], (unsigned long long)nvs);
            atomicAdd(&counters[5], (unsigned long long)nts);
        }
        if (COUNT || PROF >= 3) {
            atomicAdd(&counters[6], (unsigned long long)rs_nr);
            atomicAdd(&counters[7], (unsigned long long)rs_nl);
            atomicAdd(&counters[8], (unsigned long long)rs_lr);
            atomicAdd(&counters[9], (unsigned long long)rs_ll);
            atomicAdd(&counters[10], (unsigned long long)rs_sr);
            atomicAdd(&counters[11], (unsigned long long)rs_sl);
            atomicAdd(&counters[12], (unsigned long long)rs_st);
        }
        if (PROF) {
            atomicAdd(&counters[13], (unsigned long long)pt_shade);
            atomicAdd(&counters[14], (unsigned long long)pt_node);
            atomicAdd(&counters[15], (unsigned long long)pt_leaf);
        }
        if (PROF >= 2) {
            atomicAdd(&counters[16], (unsigned long long)ps_fetch);
            atomicAdd(&counters[17], (unsigned long long)ps_shade);
            atomicAdd(&counters[18], (unsigned long long)ps_cam);
            atomicAdd(&counters[19], (unsigned long long)ps_start);
        }
    }
}

// TMPT_PAIR=<h>: every 64-rank chunk takes h ranks from the expensive end of the
// order and 64-h from the cheap end, so a wave's cheap pixels finish early and
// its lanes then help (HELP) with the expensive ones' shadow queries.
__global__ void __launch_bounds__(256) k_pair_order(const uint32_t* __restrict__ order, int64_t P, int32_t h,
                                                     uint32_t* __restrict__ paired)
{
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= P) return;
    const int64_t full = P / 64, c = r / 64, i = r - c * 64;
    const int64_t m = c < full ? 64 : P - full * 64;  // ranks in this chunk
    const int64_t hc = c < full ? h : (m * h + 63) / 64;  // expensive ranks in this chunk
    const int64_t src = i < hc ? c * h + i : P - 1 - (c * (64 - h) + (i - hc));
    paired[r] = order[src];
}

// Pilot ordering: 3x3 box sum of each pixel's pilot-pass traversal steps,
// as a 16-bit key that sorts ascending = most expensive first.
__global__ void __launch_bounds__(256) k_order_keys(const uint32_t* __restrict__ cost, int32_t W,
                                                     int32_t rows, uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ vals)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)W * rows) return;
    const int y = (int)(i / W), x = (int)(i - (int64_t)y * W);
    uint32_t sum = 0;
    for (int dy = -1; dy <= 1; ++dy) {
        const int yy = y + dy;
        if (yy < 0 || yy >= rows) continue;
        for (int dx = -1; dx <= 1; ++dx) {
            const int xx = x + dx;
            if (xx >= 0 && xx < W) sum += cost[(int64_t)yy * W + xx];
        }
    }
    keys[i] = 65535u - min(sum, 65535u);
    vals[i] = (uint32_t)i;
}

// Sample seeding with several blocks per pixel: the pixel's colour is the sum
// of its samples' colours in sample order (main.cpp:209-219, col += Trace),
// then main.cpp:221-233.  The buffer is [pixel][sample]: one wave per 64
// pixels stages 16 samples of each in LDS with coalesced 256-B reads (16
// lanes per pixel run), then every lane sums its own pixel's samples in order.
// A progressive pass (prog != null) sums its samples [s_begin, s_end) onto the
// sum the previous pass left in prog (none when s_begin = 0), keeps the new sum
// there, and writes the preview with out_recip = 1/s_end (the full render's
// 1/spp on the last pass).
__global__ void __launch_bounds__(64) k_resolve_px(const float4* __restrict__ sbuf, int64_t P, int32_t spp,
                                                    float spp_recip, uint32_t* __restrict__ out,
                                                    int32_t s_begin = 0, int32_t s_end = -1,
                                                    float4* __restrict__ prog = nullptr)
{
    constexpr int kC = 16;                  // samples per staged chunk
    __shared__ float4 tile[64][kC + 1];     // +1: a lane's row starts on another bank
    const int64_t p0 = (int64_t)blockIdx.x * 64;
    const int t = threadIdx.x;
    const int np = (int)min<int64_t>(64, P - p0);
    if (s_end < 0) s_end = spp;
    f3 col = mk(0.0f, 0.0f, 0.0f);
    if (prog && s_begin > 0 && t < np) {
        const float4 c = prog[p0 + t];
        col = mk(c.x, c.y, c.z);
    }
    for (int32_t s0 = s_begin; s0 < s_end; s0 += kC) {
        const int nc = min(kC, s_end - s0);
        for (int e = t; e < 64 * kC; e += 64) {
            const int i = e / kC, j = e - i * kC;
            if (i < np && j < nc) tile[i][j] = sbuf[(size_t)(p0 + i) * (size_t)spp + (size_t)(s0 + j)];
        }
        __syncthreads();
        if (t < np)
            for (int j = 0; j < nc; ++j) col = col + mk(tile[t][j].x, tile[t][j].y, tile[t][j].z);
        __syncthreads();
    }
    if (t < np) {
        if (prog) prog[p0 + t] = make_float4(col.x, col.y, col.z, 0.0f);
        out[p0 + t] = pack_pixel(col, spp_recip);
    }
}

// ============================================================ speculative row seeding
// Row seeding (main.cpp:204) threads ONE xorshift stream through a row's
// pixels and samples, and a sample's draws depend on its path, so a row is a
// sequential chain (the megakernel runs one lane per row).  But a sample is
// a pure function of (pixel, start state), and every draw site takes two
// draws (maths.cpp:25, 32-33, main.cpp:214-215), so the next sample starts
// an even number of draws after this one's start.  render_rowspec traces,
// for each row, one sample at EVERY even offset 2j of a window past the
// row's current state (units of k_path<SAMP 2>), then a chase walks the
// chain through the window: take the sample at offset 0, add its colour in
// sample order, jump to offset + its draws, ...  Each window costs ~draws/2
// traces per chain sample (speculation), but all of them run in parallel.
#ifndef TMPT_RS_OCC
#define TMPT_RS_OCC 5
#endif
constexpr int kRsOcc3 = TMPT_RS_OCC;  // blocks per CU of the shadow-free pass (5 waves per SIMD)
constexpr int kRsMaxWin = 32;  // windows per row and iteration: this pixel + up to 31 lookaheads

struct RowSpec {
    int row0, nrows;  // this group's tile rows [row0, row0 + nrows)
    // per row of the group: chain state, current pixel and samples done in it,
    // its draws so far and the previous pixel's mean draws per sample (window
    // sizing), chain rays (all, closest-hit), unit offsets (nrows + 1)
    uint32_t *rng, *x, *k, *pdraws, *prev_mean, *rays, *erays, *offs;
    // window i (pixel x + i) of row r: offsets [ws[i*nrows + r], + win[i*nrows + r]);
    // window 0 starts at 0; win = 0: none
    uint32_t *win, *ws;
    uint32_t* short_win;  // iterations whose window ended before the pixel did (diagnostic)
    float4* col;
    uint32_t* total;  // units of this iteration
    unsigned long long* planned;  // units over all iterations (diagnostic)
    uint32_t wmax;
    float spread;   // windows from expected positions +- spread * sqrt(i) pixels
    int nwin;       // windows per row (1 = no lookahead)
    // no-shadow speculation: the chase lists the chain's samples (tile pixel,
    // start state, sample index) for the full re-trace; scratch holds a row's
    // (unit, sample index) pairs of one iteration (scap per row)
    uint32_t *lpix, *lstate, *lslot, *lcount;
    uint2* scratch;
    uint32_t scap;
    // Chains: a row is a chain of cw = W pixels x cspp = spp samples from the
    // row seed.  Pixel chains (pixel seeding, render_pixel_chains): chain r is
    // tile pixel cpix[r] alone (cw = 1), its samples smp0 .. smp0 + cspp - 1,
    // from the RNG state the pilot pass left in cinit[pixel].w.
    const uint32_t* cpix;
    const float4* cinit;
    int cw, cspp, smp0;
};

// Decode of a unit's rs_out.w: draws | rays << 23 | extend rays << 28.
constexpr uint32_t kRsDrawBits = 23;

__global__ void __launch_bounds__(256) k_rs_init(RenderArgs a, RowSpec rs)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rs.nrows) return;
    rs.rng[r] = rs.cpix ? __float_as_uint(rs.cinit[rs.cpix[r]].w)           // pixel chain: after its pilot
                        : row_seed((uint32_t)tile_row_to_y(a, rs.row0 + r));  // main.cpp:204, unmodified
    rs.x[r] = rs.k[r] = rs.pdraws[r] = rs.rays[r] = rs.erays[r] = rs.short_win[r] = 0u;
    rs.prev_mean[r] = __float_as_uint(17.0f);  // draws per sample before any is seen
    rs.col[r] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// Windows per row.  E = a pixel's expected units (spp x mean draws per
// sample / 2: even offsets only), the mean the larger of this pixel's so far
// and the previous pixel's.  Pixel x + i is expected to start c_i = e0 +
// (i - 1) E units ahead (e0 = this pixel's expected rest) and end c_i + E,
// each give or take spread * sqrt(i) * E; window i spans its start's and its
// end's ranges (window 0 starts at 0).  Exclusive scan into offs; total units.
// One block.
__global__ void __launch_bounds__(1024) k_rs_plan(RenderArgs a, RowSpec rs)
{
    __shared__ uint32_t part[1024];
    const int rows = rs.nrows;
    const int per = (rows + 1023) / 1024;
    const int r0 = min(rows, (int)threadIdx.x * per), r1 = min(rows, r0 + per);
    uint32_t sum = 0;
    for (int r = r0; r < r1; ++r) {
        const uint32_t x = rs.x[r];
        uint32_t t = 0;  // end of the previous window
        float mean = 0.0f, e0 = 0.0f, E = 0.0f;
        if (x < (uint32_t)rs.cw) {
            const uint32_t k = rs.k[r];
            mean = __uint_as_float(rs.prev_mean[r]);
            if (k > 0) mean = fmaxf(mean, (float)rs.pdraws[r] / (float)k);
            e0 = (float)((uint32_t)rs.cspp - k) * mean * 0.5f;  // expected units to this pixel's end
            E = (float)rs.cspp * mean * 0.5f;                   // ... of one whole pixel
        }
        for (int i = 0; i < rs.nwin; ++i) {
            uint32_t w = 0, s = 0;
            if (x + (uint32_t)i < (uint32_t)rs.cw) {
                const float ci = i == 0 ? 0.0f : e0 + (float)(i - 1) * E;
                const float ui = i == 0 ? 0.0f : rs.spread * sqrtf((float)i) * E;
                const float ce = e0 + (float)i * E, ue = rs.spread * sqrtf((float)(i + 1)) * E;
                s = i == 0 ? 0u : min(t, (uint32_t)fmaxf(0.0f, ci - ui));
                w = min(rs.wmax, (uint32_t)(ce + ue) + 2u - min(s, (uint32_t)(ce + ue)));
                t = s + w;
            }
            rs.win[i * rows + r] = w;
            rs.ws[i * rows + r] = s;
            sum += w;
        }
    }
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan of the thread sums
        const uint32_t v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t o = part[threadIdx.x] - sum;
    for (int r = r0; r < r1; ++r) {
        rs.offs[r] = o;
        for (int i = 0; i < rs.nwin; ++i) o += rs.win[i * rows + r];
    }
    if (threadIdx.x == 1023) {
        rs.offs[rows] = part[1023];
        *rs.total = part[1023];
        atomicAdd(rs.planned, (unsigned long long)part[1023]);
    }
}

// Unit u -> (row, window i, offset index j): pixel x + i and start state
// M^(2j) rng[row].  Launched over the largest possible count; the plan's
// total bounds it.
__global__ void __launch_bounds__(256) k_rs_fill(RenderArgs a, RowSpec rs, const uint32_t* __restrict__ jt2,
                                                 uint32_t* __restrict__ upix, uint32_t* __restrict__ ustate)
{
    const uint32_t u = blockIdx.x * 256 + threadIdx.x;
    if (u >= *rs.total) return;
    int lo = 0, hi = rs.nrows - 1;  // last row with offs <= u
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rs.offs[mid] <= u) lo = mid;
        else hi = mid - 1;
    }
    uint32_t l = u - rs.offs[lo];
    int i = 0;
    for (; i + 1 < rs.nwin && l >= rs.win[i * rs.nrows + lo]; ++i) l -= rs.win[i * rs.nrows + lo];
    const uint32_t j = rs.ws[i * rs.nrows + lo] + l;
    upix[u] = rs.cpix ? rs.cpix[lo] : (uint32_t)(rs.row0 + lo) * (uint32_t)a.W + rs.x[lo] + (uint32_t)i;
    ustate[u] = sample_seed(jt2, j, rs.rng[lo]);
}

// The chase, one thread per row: the chain's samples in order through the
// windows (main.cpp:209-219), each pixel packed after its spp-th (:221-233);
// on into window i + 1 when the next pixel's first sample falls in it.
__global__ void __launch_bounds__(64) k_rs_chase(RenderArgs a, RowSpec rs, const float4* __restrict__ rs_out,
                                                 const uint32_t* __restrict__ rs_end, uint32_t* __restrict__ out,
                                                 const uint32_t* __restrict__ upix, const uint32_t* __restrict__ ustate)
{
    const int r = blockIdx.x * 64 + threadIdx.x;
    const int rows = rs.nrows;
    const bool listing = rs.lpix != nullptr;  // no-shadow speculation: list the chain, no colours
    uint32_t n = r < rows ? rs.win[r] : 0u, nl = 0;
    if (n > 0) {
        uint32_t k = rs.k[r], x = rs.x[r], pdraws = rs.pdraws[r], rays = rs.rays[r], erays = rs.erays[r];
        const float4 c0 = rs.col[r];
        f3 col = mk(c0.x, c0.y, c0.z);
        // window i: offsets [lo, lo + n) at wb
        uint32_t j = 0, last = 0xFFFFFFFFu, lo = 0, wb = rs.offs[r];
        int i = 0;
        while (j >= lo && j - lo < n) {
            const uint32_t idx = wb + (j - lo);
            const float4 t = rs_out[idx];
            const uint32_t w = __float_as_uint(t.w);
            const uint32_t draws = w & ((1u << kRsDrawBits) - 1u);
            rays += (w >> kRsDrawBits) & 31u;
            erays += w >> 28;
            pdraws += draws;
            if (listing) rs.scratch[(size_t)r * rs.scap + nl++] = make_uint2(idx, (uint32_t)rs.smp0 + k);
            else col = col + mk(t.x, t.y, t.z);  // col += Trace(...), main.cpp:218
            last = idx;
            j += draws >> 1;
            if (++k == (uint32_t)rs.cspp) {  // the rest of this window belongs to this pixel: dropped
                if (!listing) out[(size_t)(rs.row0 + r) * a.W + x] = pack_pixel(col, a.spp_recip);
                rs.prev_mean[r] = __float_as_uint((float)pdraws / (float)k);
                ++x;
                k = 0;
                pdraws = 0;
                col = mk(0.0f, 0.0f, 0.0f);
                if (++i >= rs.nwin) break;
                wb += n;
                n = rs.win[i * rows + r];
                lo = rs.ws[i * rows + r];
                if (n == 0) break;
            }
        }
        if (last != 0xFFFFFFFFu) rs.rng[r] = rs_end[last];  // the next sample's start state
        if (k != 0) ++rs.short_win[r];
        rs.k[r] = k;
        rs.x[r] = x;
        rs.pdraws[r] = pdraws;
        rs.rays[r] = rays;
        rs.erays[r] = erays;
        rs.col[r] = make_float4(col.x, col.y, col.z, 0.0f);
    }
    if (!listing) return;
    // the row's chain samples into the frame's list: one atomic per wave
    uint32_t incl = nl;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, off);
        if ((threadIdx.x & 63) >= (unsigned)off) incl += v;
    }
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 63) base = atomicAdd(rs.lcount, incl);
    base = (uint32_t)__shfl((int)base, 63) + incl - nl;
    for (uint32_t t = 0; t < nl; ++t) {
        const uint2 e = rs.scratch[(size_t)r * rs.scap + t];
        rs.lpix[base + t] = upix[e.x];
        rs.lstate[base + t] = ustate[e.x];
        rs.lslot[base + t] = e.y;
    }
}

// The same chase for the listing (shadow-free) pass, one wave per row: the
// row's unit words are staged in LDS with coalesced loads first, so the
// chain's walk -- one dependent read per chain sample -- runs on LDS latency
// instead of a global round trip each (the one-thread-per-row kernel spent
// ~3.6 us per chain sample there).  The chain's (unit, sample) pairs collect
// in LDS and the wave copies them into the frame's list.  Rows with more
// units than kChaseUnits walk from global memory; the host only picks this
// kernel when a row's chain samples per iteration fit kChaseList.
constexpr uint32_t kChaseUnits = 8192, kChaseList = 2048;
__global__ void __launch_bounds__(64) k_rs_chase_lds(RenderArgs a, RowSpec rs, const float4* __restrict__ rs_out,
                                                     const uint32_t* __restrict__ rs_end,
                                                     const uint32_t* __restrict__ upix,
                                                     const uint32_t* __restrict__ ustate)
{
    __shared__ uint32_t s_w[kChaseUnits];
    __shared__ uint2 s_l[kChaseList];
    __shared__ uint32_t s_n, s_base;
    const int r = blockIdx.x;
    const int rows = rs.nrows;
    const uint32_t lane = threadIdx.x;
    if (rs.win[r] == 0) return;  // row finished (block-uniform)
    const uint32_t u0 = rs.offs[r], nu = rs.offs[r + 1] - u0;
    const bool staged = nu <= kChaseUnits;
    if (staged)
        for (uint32_t i = lane; i < nu; i += 64) s_w[i] = __float_as_uint(rs_out[u0 + i].w);
    __syncthreads();
    if (lane == 0) {
        uint32_t k = rs.k[r], x = rs.x[r], pdraws = rs.pdraws[r], rays = rs.rays[r], erays = rs.erays[r];
        uint32_t n = rs.win[r], nl = 0;
        uint32_t j = 0, last = 0xFFFFFFFFu, lo = 0, wb = u0;
        int i = 0;
        while (j >= lo && j - lo < n) {
            const uint32_t idx = wb + (j - lo);
            const uint32_t w = staged ? s_w[idx - u0] : __float_as_uint(rs_out[idx].w);
            const uint32_t draws = w & ((1u << kRsDrawBits) - 1u);
            rays += (w >> kRsDrawBits) & 31u;
            erays += w >> 28;
            pdraws += draws;
            s_l[nl++] = make_uint2(idx, (uint32_t)rs.smp0 + k);
            last = idx;
            j += draws >> 1;
            if (++k == (uint32_t)rs.cspp) {  // the rest of this window belongs to this pixel: dropped
                rs.prev_mean[r] = __float_as_uint((float)pdraws / (float)k);
                ++x;
                k = 0;
                pdraws = 0;
                if (++i >= rs.nwin) break;
                wb += n;
                n = rs.win[i * rows + r];
                lo = rs.ws[i * rows + r];
                if (n == 0) break;
            }
        }
        if (last != 0xFFFFFFFFu) rs.rng[r] = rs_end[last];  // the next sample's start state
        if (k != 0) ++rs.short_win[r];
        rs.k[r] = k;
        rs.x[r] = x;
        rs.pdraws[r] = pdraws;
        rs.rays[r] = rays;
        rs.erays[r] = erays;
        s_n = nl;
        s_base = nl ? atomicAdd(rs.lcount, nl) : 0u;
    }
    __syncthreads();
    const uint32_t nl = s_n, base = s_base;
    for (uint32_t t = lane; t < nl; t += 64) {
        const uint2 e = s_l[t];
        rs.lpix[base + t] = upix[e.x];
        rs.lstate[base + t] = ustate[e.x];
        rs.lslot[base + t] = e.y;
    }
}

// render_rowstream: each row's anchor states M^(2^15 a) row_seed, a < na, from
// the byte tables of M^(2^15 a0) (j1) and M^(2^20 a1) (j2), a = 32 a1 + a0;
// thread 0 also publishes the final pass's unit count.
__global__ void __launch_bounds__(256) k_rss_anchors(RenderArgs a, RsStream S, const uint32_t* __restrict__ j1,
                                                     const uint32_t* __restrict__ j2)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i == 0) S.ctl[4] = (uint32_t)((size_t)a.slots * (size_t)a.spp);
    if (i >= (size_t)S.nrows * S.na) return;
    const int row = (int)(i / S.na);
    const uint32_t an = (uint32_t)(i - (size_t)row * S.na);
    const uint32_t seed = row_seed((uint32_t)tile_row_to_y(a, row));  // main.cpp:204, unmodified
    const_cast<uint32_t*>(S.anchors)[i] = sample_seed(j2, an >> 5, sample_seed(j1, an & 31u, seed));
}

// The chain list's offsets -> start states, in place (unit u: row u / spp / W).
__global__ void __launch_bounds__(256) k_rss_states(RenderArgs a, RsStream S)
{
    const size_t u = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= (size_t)a.slots * (size_t)a.spp) return;
    const int row = (int)(u / ((size_t)a.spp * (size_t)a.W));
    S.list[u] = rss_state(S, row, S.list[u]);
}

// The chain rays of render_rowstream's rows: counters[0] all, [3] closest-hit.
__global__ void __launch_bounds__(256) k_rss_count(RsStream S, unsigned long long* counters)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    unsigned long long sv = r < S.nrows ? S.rowrays[2 * r] : 0u, se = r < S.nrows ? S.rowrays[2 * r + 1] : 0u;
    for (int off = 32; off > 0; off >>= 1) {
        sv += __shfl_xor(sv, off);
        se += __shfl_xor(se, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counters[0], sv);
        atomicAdd(&counters[3], se);
    }
}

// The chain's rays (the reference's count): counters[0] all, [3] closest-hit.
__global__ void __launch_bounds__(256) k_rs_count(RowSpec rs, unsigned long long* counters)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    const uint32_t v = r < rs.nrows ? rs.rays[r] : 0u, e = r < rs.nrows ? rs.erays[r] : 0u;
    unsigned long long sv = v, se = e;
    for (int off = 32; off > 0; off >>= 1) {
        sv += __shfl_xor(sv, off);
        se += __shfl_xor(se, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counters[0], sv);
        atomicAdd(&counters[3], se);
    }
}

// ============================================================ host side
namespace {

constexpr int kBlk = 256;
constexpr int kSL = 16;  // LDS stack entries per lane
// the 5-wave path kernels (OCC 5): 30 KB of LDS per block -- a 12-entry LDS
// stack, the scattered ray's direction only, kTopNodes5 top nodes
constexpr int kPathSL5 = 12;

int occupancy_grid(const void* fn, int block, size_t dyn_lds, int device)
{
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, dyn_lds) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        cus < 1)
        cus = 256;
    return per_cu * cus;
}

int ensure_ws(Scene& s, size_t bytes)
{
    if (s.ws_bytes >= bytes) return 0;
    if (s.ws) (void)hipFree(s.ws);
    s.ws = nullptr;
    s.ws_bytes = 0;
    TMPT_HIP(hipMalloc(&s.ws, bytes));
    s.ws_bytes = bytes;
    return 0;
}

SceneView view(const Scene& s)
{
    SceneView v{s.nodes4, s.tri_pre, s.tri_orig, s.n, s.n_nodes4};
    v.soa = s.soa;
#ifdef TMPT_CHECK
    v.chk = s.chk;
    // TMPT_CHECK_SELFTEST=1 (the report's own test, tests/test_gpu_check.py):
    // the view claims a single BVH node, so every query that descends past
    // the root fails the node test
    if (const char* e = getenv("TMPT_CHECK_SELFTEST"))
        if (atoi(e) == 1) v.n_nodes4 = std::min(v.n_nodes4, 1);
#endif
    if (s.oct && s.opt.tie_rule == 0) {  // the reference's visit order for ties
        v.oct = s.oct_view;
        const OctGrid& g = s.oct_grid;
        v.crack = make_float4(g.reach, g.drift[0], g.drift[1], g.drift[2]);
    }
    return v;
}

// Columns of M^n, M the xorshift32 step as a GF(2) 32x32 matrix (maths.cpp:5-13):
// column j = image of bit j.
void gf2_mul(const uint32_t* x, const uint32_t* y, uint32_t* out)  // out = x * y
{
    uint32_t t[32];
    for (int j = 0; j < 32; ++j) {
        uint32_t r = 0;
        for (int i = 0; i < 32; ++i)
            if ((y[j] >> i) & 1u) r ^= x[i];
        t[j] = r;
    }
    memcpy(out, t, sizeof t);
}

void xorshift_power(uint64_t n, uint32_t* acc)
{
    uint32_t m[32];
    for (int j = 0; j < 32; ++j) {
        uint32_t v = 1u << j;
        m[j] = xorshift32(v);
        acc[j] = 1u << j;
    }
    for (; n; n >>= 1) {
        if (n & 1u) gf2_mul(m, acc, acc);
        gf2_mul(m, m, m);
    }
}

}  // namespace

// sample_seed's byte tables for jumps J_i = M^(i * stride), i in [0, count)
void jump_tables(uint64_t stride_steps, int32_t count, std::vector<uint32_t>& tab)
{
    uint32_t stride[32], J[32];
    xorshift_power(stride_steps, stride);
    for (int j = 0; j < 32; ++j) J[j] = 1u << j;
    tab.assign((size_t)count * 1024u, 0u);
    for (int32_t i = 0; i < count; ++i) {
        uint32_t* t = tab.data() + (size_t)i * 1024u;
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 1; b < 256; ++b)  // table[b] = table[b without its lowest bit] ^ column
                t[256 * k + b] = t[256 * k + (b & (b - 1u))] ^ J[8 * k + __builtin_ctz(b)];
        gf2_mul(stride, J, J);
    }
}

// sample_seed's byte tables for samples [0, spp): J_s = M^(s * kSampleStride)
void sample_jump_tables(int32_t spp, std::vector<uint32_t>& tab) { jump_tables(kSampleStride, spp, tab); }

namespace {

RenderArgs make_args(const tmpt_camera* c, const tmpt_render_desc* d)
{
    RenderArgs a;
    a.cam.origin = mk(c->origin[0], c->origin[1], c->origin[2]);
    a.cam.lower_left = mk(c->lower_left[0], c->lower_left[1], c->lower_left[2]);
    a.cam.horizontal = mk(c->horizontal[0], c->horizontal[1], c->horizontal[2]);
    a.cam.vertical = mk(c->vertical[0], c->vertical[1], c->vertical[2]);
    a.cam.u = mk(c->u[0], c->u[1], c->u[2]);
    a.cam.v = mk(c->v[0], c->v[1], c->v[2]);
    a.cam.w = mk(c->w[0], c->w[1], c->w[2]);
    a.cam.lens_radius = c->lens_radius;
    a.W = d->width;
    a.H = d->height;
    a.spp = d->spp;
    a.seed_mode = d->seed_mode;
    a.band_rows = d->band_rows > 0 ? d->band_rows : d->height;
    a.shard = d->num_shards > 1 ? d->shard : 0;
    a.nshards = d->num_shards > 1 ? d->num_shards : 1;
    a.tile_rows = tmpt_tile_rows(d);
    a.invW = 1.0f / (float)d->width;             // main.cpp:186
    a.invH = 1.0f / (float)d->height;            // main.cpp:187
    a.spp_recip = 1.0f / (float)d->spp;          // main.cpp:188
    a.slots = (int64_t)a.tile_rows * a.W;
    a.smp_begin = d->spp_begin;
    a.smp_end = d->spp_count > 0 ? d->spp_begin + d->spp_count : d->spp;
    a.out_recip = a.smp_end == d->spp ? a.spp_recip : 1.0f / (float)a.smp_end;
    a.prog = nullptr;
    a.jt = nullptr;
    a.bmask = 2047u;
    a.row_lanes = 1;  // one row per wave: measured fastest
    a.root_check = 0;
    return a;
}


template <bool ROW, bool COUNT>
int launch_mega(Scene& s, const RenderArgs& a, uint32_t* out, unsigned long long* counters)
{
    auto fn = k_mega<ROW, COUNT, kBlk, kSL>;
    int grid = occupancy_grid((const void*)fn, kBlk, 0, s.device);
    // ROW: one wave per row_lanes rows (up to the resident grid)
    int64_t items = ROW ? ((int64_t)a.tile_rows + a.row_lanes - 1) / a.row_lanes * 64 : a.slots;
    grid = (int)std::min<int64_t>(grid, (items + kBlk - 1) / kBlk);
    grid = std::max(grid, 1);
    size_t ovf_bytes = (size_t)grid * kBlk * (kStackTotal - kSL) * sizeof(uint32_t);
    if (ensure_ws(s, ovf_bytes)) return -1;
    fn<<<grid, kBlk, 0, s.stream>>>(view(s), a, out, (uint32_t*)s.ws, counters);
    TMPT_HIP(hipGetLastError());
    return 0;
}

}  // namespace

int render_megakernel(Scene& s, const RenderArgs& a, uint32_t* d_out, bool count,
                      unsigned long long* d_counters)
{
    const bool row = a.seed_mode == TMPT_SEED_ROW;
    if (row) return count ? launch_mega<true, true>(s, a, d_out, d_counters) : launch_mega<true, false>(s, a, d_out, d_counters);
    return count ? launch_mega<false, true>(s, a, d_out, d_counters) : launch_mega<false, false>(s, a, d_out, d_counters);
}
// Wavefront driver.  The host enqueues iterations without reading the queue
// sizes (the kernels read them from device memory) and checks for completion
// every kCheck iterations.
int render_wavefront(Scene& s, const RenderArgs& a, uint32_t* d_out, bool count)
{
    const int64_t P = a.slots;
    if (P >= (int64_t)kSkip) {
        set_error("wavefront: tile too large");
        return -22;
    }
    // top BVH levels from LDS in both passes, no occupancy floor: measured best
    // against no LDS copy and 5-8 waves per SIMD (profiles/r03_wavefront_ab/)
    constexpr bool kTopE = true, kTopS = true;
    constexpr int kWE = 1, kWS = 1;
    auto trace_e = count ? k_wf_trace<false, true, kBlk, kSL, kTopE, kWE> : k_wf_trace<false, false, kBlk, kSL, kTopE, kWE>;
    auto trace_s = count ? k_wf_trace<true, true, kBlk, kSL, kTopS, kWS> : k_wf_trace<true, false, kBlk, kSL, kTopS, kWS>;
    const int sl = kSL;
    int grid_t = occupancy_grid((const void*)trace_e, kBlk, 0, s.device);
    const int grid_sh = (int)((P + kBlk - 1) / kBlk);
    const size_t seg_cap = (size_t)(((P + kSeg - 1) / kSeg + kBlk - 1) / kBlk) * kBlk;
    const uint32_t nbins = (uint32_t)s.opt.wf_bins;  // extend sub-queues per segment (octant bins)
    const size_t qcap = seg_cap * kSeg * nbins, qcap_s = seg_cap * kSeg;
    const size_t Pz = (size_t)P;
    size_t ovf_words = (size_t)grid_t * kBlk * (kStackTotal - sl);
    // layout of the workspace
    size_t words = 0;
    auto take = [&](size_t w) { size_t o = words; words += (w + 63) & ~size_t(63); return o; };
    const size_t ctr_words = (size_t)kSeg * kCtr, ectr_words = ctr_words * nbins;
    size_t o_rng = take(Pz), o_smp = take(Pz), o_depth = take(Pz), o_col = take(3 * Pz),
           o_light = take(kMaxDepth * Pz), o_ray = take(6 * Pz), o_hit = take(3 * Pz),
           o_hid = take(Pz), o_sho = take(3 * Pz), o_q0 = take(qcap), o_q1 = take(qcap),
           o_qs = take(qcap_s), o_ctl = take(3 * ectr_words + 2 * ctr_words + 64), o_tot = take(16),
           o_ovf = take(ovf_words);
#ifdef TMPT_DIAG
    const bool log_iters = getenv("TMPT_ITER_LOG") != nullptr;  // diagnostic build: queue sizes per iteration
#else
    const bool log_iters = false;
#endif
    const int64_t max_log = (int64_t)a.spp * (kMaxDepth + 2) + 64 + 16;
    size_t o_log = log_iters ? take(2 * (size_t)max_log) : 0;
    if (ensure_ws(s, words * 4)) return -1;
    uint32_t* w = (uint32_t*)s.ws;
    WfState st;
    st.rng = w + o_rng;
    st.smp = w + o_smp;
    st.depth = w + o_depth;
    st.col = (float*)(w + o_col);
    st.light = (float*)(w + o_light);
    st.ray = (float*)(w + o_ray);
    st.hit = (float*)(w + o_hit);
    st.hid = (int32_t*)(w + o_hid);
    st.sho = (float*)(w + o_sho);
    st.q[0] = w + o_q0;
    st.q[1] = w + o_q1;
    st.qs = w + o_qs;
    st.cnt[0] = w + o_ctl;
    st.cnt[1] = st.cnt[0] + ectr_words;
    st.head_e = st.cnt[1] + ectr_words;
    st.cnt_s = st.head_e + ectr_words;
    st.head_s = st.cnt_s + ctr_words;
    st.total = st.head_s + ctr_words;
    st.tot = (unsigned long long*)(w + o_tot);
    st.iter_log = log_iters ? w + o_log : nullptr;
    st.P = P;
    st.seg_cap = (uint32_t)seg_cap;
    st.nbins = nbins;
    // low load: under two queue entries per resident traversal lane; binned
    // queues always (most of their sub-queues are empty)
    st.walk_check = nbins > 1 || P < 2 * (int64_t)grid_t * kBlk;
    st.root_check = a.root_check;
    uint32_t* ovf = w + o_ovf;
    hipStream_t str = s.stream;

    TMPT_HIP(hipMemsetAsync(w + o_ctl, 0, (3 * ectr_words + 2 * ctr_words + 64) * 4, str));
    TMPT_HIP(hipMemsetAsync(st.tot, 0, 8 * sizeof(unsigned long long), str));
    if (st.iter_log) TMPT_HIP(hipMemsetAsync(st.iter_log, 0, 8 * (size_t)max_log, str));
    k_wf_generate<kBlk><<<(int)((std::max<int64_t>(P, kSeg) + kBlk - 1) / kBlk), kBlk, 0, str>>>(a, st);

    // per-launch timing of the traversal kernels
    std::vector<hipEvent_t> ev;
    auto new_ev = [&]() {
        hipEvent_t e;
        (void)hipEventCreate(&e);
        ev.push_back(e);
        return e;
    };
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ext_ev, sh_ev;
    uint32_t* h_cnt = nullptr;
    TMPT_HIP(hipHostMalloc((void**)&h_cnt, 16, hipHostMallocDefault));
    const int kCheck = 8;
    int parity = 0;
    int64_t it = 0;
    int rc = 0;
    for (;;) {
        for (int k = 0; k < kCheck; ++k, ++it) {
            hipEvent_t e0 = new_ev(), e1 = new_ev(), e2 = new_ev(), e3 = new_ev();
            (void)hipEventRecord(e0, str);
            trace_e<<<grid_t, kBlk, 0, str>>>(view(s), st, parity, ovf);
            (void)hipEventRecord(e1, str);
            k_wf_shade<kBlk><<<grid_sh, kBlk, 0, str>>>(view(s), a, st, parity, d_out);
            (void)hipEventRecord(e2, str);
            trace_s<<<grid_t, kBlk, 0, str>>>(view(s), st, parity, ovf);
            (void)hipEventRecord(e3, str);
            k_wf_advance<<<1, kSeg, 0, str>>>(st, parity, (int)std::min<int64_t>(it, max_log - 1));
            ext_ev.push_back({e0, e1});
            sh_ev.push_back({e2, e3});
            parity ^= 1;
        }
        if (hipGetLastError() != hipSuccess) { rc = -1; break; }
        if (hipMemcpyAsync(h_cnt, st.total, 4, hipMemcpyDeviceToHost, str) != hipSuccess ||
            hipStreamSynchronize(str) != hipSuccess) { rc = -1; break; }
        if (h_cnt[0] == 0) break;
        if (it > (int64_t)a.spp * (kMaxDepth + 2) + 64) {  // each pixel needs <= spp*(kMaxDepth+1) iterations
            set_error("wavefront: iteration bound exceeded");
            rc = -3;
            break;
        }
    }
    unsigned long long tot[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rc == 0) {
        TMPT_HIP(hipMemcpyAsync(tot, st.tot, sizeof(tot), hipMemcpyDeviceToHost, str));
        TMPT_HIP(hipStreamSynchronize(str));
        if (log_iters) {
            std::vector<uint32_t> lg(2 * (size_t)std::min<int64_t>(it, max_log));
            TMPT_HIP(hipMemcpy(lg.data(), st.iter_log, lg.size() * 4, hipMemcpyDeviceToHost));
            for (size_t k = 0; k < lg.size() / 2; ++k)
                fprintf(stderr, "tmpt-iter %zu extend %u shadow %u\n", k, lg[2 * k], lg[2 * k + 1]);
            if (count) fprintf(stderr, "tmpt-max-steps extend %llu shadow %llu\n", tot[6], tot[7]);
        }
    }
    double ems = 0, sms = 0;
    for (auto& pr : ext_ev) { float ms = 0; (void)hipEventElapsedTime(&ms, pr.first, pr.second); ems += ms; }
    for (auto& pr : sh_ev) { float ms = 0; (void)hipEventElapsedTime(&ms, pr.first, pr.second); sms += ms; }
    for (auto e : ev) (void)hipEventDestroy(e);
    (void)hipHostFree(h_cnt);
    if (rc) {
        if (rc == -1) set_error("wavefront: HIP error");
        return rc;
    }
    s.extend_ms = ems;
    s.shadow_ms = sms;
    s.extend_rays = tot[0];
    s.shadow_rays = tot[1];
    s.node_visits = tot[2];
    s.tri_tests = tot[3];
    s.shadow_node_visits = tot[4];
    s.shadow_tri_tests = tot[5];
    s.extend_launches = it;
    s.shadow_launches = it;
    s.iterations = it;
    return 0;
}

// The heaviest pixels of a pixel-seeded frame as speculative chains
// (render_rowspec's engine with a chain = one pixel): pixel cpix[r], its
// samples smp0 .. smp0 + cspp - 1, from the state the pilot pass left in
// cinit[pixel] (colour sum of samples 0 .. smp0-1, RNG state in .w).
struct PixelChains {
    const uint32_t* cpix;
    const float4* cinit;
    int n, smp0, cspp;
};
int render_rowspec(Scene& s, const RenderArgs& a, uint32_t* d_out, unsigned long long* d_counters,
                   const PixelChains* ch = nullptr);

// The chains' pixels: the pilot's colour sum, then samples smp0 .. spp-1 from
// the colour buffer, in sample order (main.cpp:218), packed (main.cpp:221-233).
__global__ void __launch_bounds__(256) k_resolve_chains(PixelChains ch, const float4* __restrict__ sbuf, int32_t spp,
                                                        float spp_recip, uint32_t* __restrict__ out)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= ch.n) return;
    const uint32_t p = ch.cpix[r];
    const float4 c0 = ch.cinit[p];
    f3 col = mk(c0.x, c0.y, c0.z);
    for (int32_t k = ch.smp0; k < spp; ++k) {
        const float4 c = sbuf[(size_t)p * (size_t)spp + (size_t)k];
        col = col + mk(c.x, c.y, c.z);
    }
    out[p] = pack_pixel(col, spp_recip);
}

// PathCtl::oct_shadow: whether a shadow query's answer can need the octree --
// a triangle lying flat on one of its planes, or a light direction that can
// drift along a crack (octree_crack's test at the smallest t a hit can have,
// kMinT): the constant light of main.cpp:36 never can in these scenes, but
// the test is the device's own.
static uint32_t oct_shadow_check(const Scene& s)
{
    if (!s.oct_view || s.opt.tie_rule != 0) return 0u;
    if (s.oct_flat > 0) return 1u;
    const f3 ld = light_dir();
    const float l[3] = {fabsf(ld.x), fabsf(ld.y), fabsf(ld.z)};
    for (int k = 0; k < 3; ++k)
        if (l[k] * fminf(kMinT, s.oct_grid.reach) <= s.oct_grid.drift[k]) return 1u;
    return 0u;
}

// Persistent path engine: one launch per frame (shard).
int render_persistent(Scene& s, const RenderArgs& a, uint32_t* d_out, bool count,
                      unsigned long long* d_counters)
{
    const Options& o = s.opt;
    // HIP events around each k_path launch (pilot: 0-1, final: 2-3) on the
    // stream it runs on: the dominant kernel's own time for the roofline
    if (!s.path_ev[0])
        for (auto& e : s.path_ev) TMPT_HIP(hipEventCreate(&e));
    // traversal rounds between shading checks / lanes waiting that trigger a
    // shading round (A/B on the bench frame at 1 and 8 shards);
    // sparse-wave shading threshold divisor (k_path TAIL): 2 -- bench frame,
    // pixel seeding 235.2 -> 231.9 ms at N=1, 1/8 shard unchanged (41.0 ms);
    // sample seeding 220.4 -> 218.2 ms at N=1, 29.4 -> 29.0 ms at 1/8
    // (TMPT_PATH_STEPS / TMPT_SHADE_MIN / TMPT_SPARSE: A/B builds, tools/ab_build.sh)
    constexpr int kPathSL = 16, kPathSteps = TMPT_PATH_STEPS, kShadeMin = TMPT_SHADE_MIN, kSparse = TMPT_SPARSE;
    // pixel seeding's kernels: 24 rounds between shading checks -- re-swept at
    // 5 waves per SIMD (whole renders, steps 16 / 24 / 32: 1/8 shard 36.4 /
    // 35.2 / 36.1 ms, 1/4 63.7 / 63.2 / 65.1, N=1 198.0 / 196.0 / 208.9; the
    // sample kernels 172.3 / 172.8 / 182.9 keep 16; 20 and 28 both lose to 24,
    // +1.4 % at 1/8; profiles/r06_experiments/cadence_5waves*.log,
    // cadence_pixel_20_24_28.log)
    constexpr int kPixSteps = TMPT_PIX_STEPS;
    using PathFn = decltype(&k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse>);
    // pixel seeding, and sample seeding (its own instantiation: the pixel-mode
    // kernel keeps its register allocation)
    // layout=soa: the sample kernel reads the SoA planes (the A/B of DESIGN.md
    // section 3; the other engines keep the AoS records)
    const bool soa = s.soa.na != nullptr;
    PathFn fn = a.jt ? (count ? (soa ? k_path<true, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1, true>
                                     : k_path<true, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1>)
                              : (soa ? k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1, true>
                                     : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1>))
                     : (count ? k_path<true, kBlk, kPathSL, kPixSteps, kShadeMin, 4, kSparse>
                              : k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 4, kSparse>);
    const PathFn fn_default = fn;
    int prof = 0;
#ifdef TMPT_DIAG
    // diagnostic build only: TMPT_PROF=1 s_memtime split of wave time (shading /
    // node / leaf rounds); 2: + shading-round split; 3: + per-round cycle counts
    // (more registers: compare its times only among PROF=3 runs)
    if (const char* pe = getenv("TMPT_PROF")) prof = count ? 0 : atoi(pe);
    if (prof && !a.jt)
        fn = prof >= 3 ? k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 1, kSparse, 3>
           : prof == 2 ? k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 1, kSparse, 2>
                       : k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 1, kSparse, 1>;
    if (prof && a.jt)
        fn = prof >= 2 ? k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 1, kSparse, 2, 0, 1>
                       : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 1, kSparse, 1, 0, 1>;
#endif
    // Sample seeding's path kernels run 5 waves per SIMD (OCC 5: the 30-KB LDS
    // layout, 96 VGPRs; option path_waves): the lanes below are theirs
    const bool waves5 = a.jt && !count && !prof && !soa && o.path_waves != 4;
    // Pixel seeding's instantiations too, but only with several pixels per
    // lane: at low load a pixel's sample chain is the frame's critical path
    // and a fifth wave on the SIMD slows every chain (whole renders, 4 / 5
    // waves: N=1 207.2 / 197.6 ms, 1/2 116.9 / 113.9, 1/4 63.6 / 65.7, 1/8
    // 36.2 / 39.1; profiles/r06_experiments/occ5/ab_pixel_waves.log), so from
    // 3 pixels per 4-wave lane (option path_waves 5 forces it, 4 keeps 4)
    // (every OCC 5 instantiation has the same LDS and VGPR footprint, so one
    // of them gives the 5-wave grid)
    const int grid4 = occupancy_grid((const void*)fn, kBlk, 0, s.device);
    const int grid5 = occupancy_grid(
        (const void*)k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 1, false, 1>, kBlk, 0,
        s.device);
    const bool waves5p = !a.jt && !count && !prof &&
                         (o.path_waves == 5 || (o.path_waves == 0 && a.slots >= 3 * (int64_t)grid4 * kBlk));
    const int grid = waves5 || waves5p ? grid5 : grid4;
    // Sample seeding: the work units are (pixel, block of blk samples).  The
    // block is the largest power of two up to 8 that still leaves >=
    // kUnitsPerLane units per resident lane.  Bench frame (1-row bands,
    // k_path ms): N=1 blk 2/4/8 = 220.7/217.8/217.3; 1/2 shard blk 1/2/4/8 =
    // 113.3/110.9/110.2/111.7; 1/4 blk 1/2/4 = 57.1/56.2/56.6; 1/8 blk 1/2/4/8
    // = 29.4/29.4/30.2/32.7 -- best at ~63 units per lane while the frame
    // ended on a lane's last block (rounds 2-4: 60 picked 8, 4, 2, 1 at N = 1,
    // 2, 4, 8).  With the single-sample tail units below the end no longer
    // depends on the block, and fewer, longer blocks win (round 5, k_path ms,
    // profiles/r05_experiments/blk_tail_*.log): 1/8 blk 1 / 2 / 4 / 8 with a
    // 4-block tail 25.55 / 24.93 / 24.54 / 24.73, 1/4 blk 2 / 4 / 8 49.24 /
    // 48.22 / 48.31, N=1 blk 8 / 16 / 32 186.27 / 186.25 / 188.92, 1/2 blk
    // 8 / 16 94.47 / 95.09 -- so 15 units per lane and at most 8 samples: 8,
    // 8, 8, 4 at N = 1, 2, 4, 8.  Option sample_block fixes it.
    uint32_t blk = 1u, nblk = 1u, blk0 = 0u;
    // Progressive passes in sample seeding (samples [s0, s1) of every pixel):
    // the units are the blocks of the pass -- a block size that divides s0, so
    // the blocks keep their alignment -- and every sample's colour goes to the
    // colour buffer; k_resolve_px adds the pass's samples, in order, to the sum
    // the previous pass left (main.cpp:218 summed across the passes).
    const bool pass = a.jt && (a.smp_begin > 0 || a.smp_end < a.spp);
    const int64_t s0 = a.smp_begin, s1 = a.smp_end;
    if (a.jt) {
        // (15 units per 4-wave lane; with 5 waves per SIMD a quarter more lanes
        // share the work, and 12 per lane picks the same blocks as 15 did:
        // 8, 8, 8, 4 at N = 1, 2, 4, 8 -- round 6, profiles/r06_experiments/occ5/)
        const int64_t kUnitsPerLane = waves5 ? 12 : 15;
        const int64_t lanes0 = (int64_t)grid * kBlk;
        blk = 1u;
        while ((int64_t)blk * 2 <= 8 && blk * 2u <= (uint32_t)(s1 - s0) &&
               a.slots * ((s1 - s0 + blk * 2 - 1) / (blk * 2)) >= kUnitsPerLane * lanes0)
            blk *= 2u;
        if (o.sample_block > 0) blk = (uint32_t)o.sample_block;
        while (a.slots * ((s1 - s0 + blk - 1) / blk) >= (1ll << 31)) blk *= 2u;  // 32-bit unit ids
        while (s0 % blk) blk /= 2u;  // a pass's first sample starts a block
        // the alignment can undo the 32-bit guard above (e.g. 4K x 1024 spp
        // from spp_begin 2: blocks of 2, ~4.2 G units): the unit ids, res and
        // nchunks are uint32, so such a pass is refused, not wrapped
        if (a.slots * ((s1 - s0 + blk - 1) / blk) >= (1ll << 31)) {
            set_error("tmpt_render: this progressive pass (samples " + std::to_string(s0) + ".." +
                      std::to_string(s1) + " of " + std::to_string(a.slots) +
                      " pixels) needs more than 2^31 sample units at the block size its first sample allows (" +
                      std::to_string(blk) + "): start passes at a multiple of a larger power of two, or render "
                      "the frame in one call");
            return -22;
        }
        blk0 = (uint32_t)(s0 / blk);
        nblk = (uint32_t)((s1 + blk - 1) / blk - blk0);
        // Several blocks per pixel need the per-sample colour buffer (16 B per
        // sample of the tile: 2.1 GB at 1080p x 64).  If it does not fit in 3/4
        // of the free device memory (or the sbuf_max option), the pixel is one
        // unit: same image, only the tail of a small shard is longer.  A
        // progressive pass needs the buffer whatever its block count.
        if (nblk > 1 || pass) {
            const size_t need = sizeof(float4) * (size_t)a.spp * (size_t)a.slots;
            size_t fr = 0, tot = 0;
            size_t budget = hipMemGetInfo(&fr, &tot) == hipSuccess ? fr / 4 * 3 : 0;
            budget += s.sbuf_bytes;  // the buffer already held is free for this call
            if (o.sbuf_max > 0.0) budget = std::min(budget, (size_t)o.sbuf_max);
            if (need > budget) {
                if (pass) {
                    set_error("tmpt_render: progressive passes in sample seeding need the per-sample colour buffer (" +
                              std::to_string(need >> 20) + " MiB), which does not fit: render the frame in one call");
                    return -12;
                }
                while (blk < (uint32_t)a.spp) blk *= 2u;
                nblk = 1u;
            }
        }
    }
    int64_t P = a.slots * (int64_t)nblk;  // units the supply hands out
    // Sample seeding's tail (option sample_tail): the last sample_tail blocks
    // per resident lane are handed out as single samples, so a lane's last
    // unit is one sample, not a block of blk, and the waves leave their main
    // loops closer together: bench frame, N=1, blocks of 8, the main loops
    // ended over 8.6 ms without it and over 1.7 ms with 8 blocks per lane
    // (profiles/r05_wavetime/; the deferred re-traces are then the last
    // ~2 ms).  k_path, tail 0 / 8 blocks per lane: N=1 188.0 / 186.0 ms, 1/2
    // 96.1 / 94.7 ms (16: slower again, the single units' own seed jumps;
    // profiles/r05_experiments/sample_tail*.log).  With the longer blocks
    // above: a quarter of a lane's samples, at most 64 (N=1 and 1/2: 8 blocks
    // of 8; 1/4: 4 of 8; 1/8: 4 of 4).
    uint32_t ua = 0xFFFFFFFFu;
    // (only when every block is full: a partial last block would map tail
    // units to samples past the pass's end)
    // Auto (-1): a quarter of a lane's samples, at most 64, in blocks.
    int64_t tail_blocks = o.sample_tail;
    if (tail_blocks < 0) {
        const int64_t spl = a.slots * (s1 - s0) / std::max<int64_t>(1, (int64_t)grid * kBlk);  // samples per lane
        const int64_t b = std::max<uint32_t>(1u, blk);
        tail_blocks = std::max<int64_t>(1, (std::min<int64_t>(64, spl / 4) + b - 1) / b);
    }
    if (a.jt && nblk > 1 && blk >= 2u && tail_blocks > 0 && (s1 - s0) % blk == 0) {
        int64_t nb = std::min<int64_t>(P, tail_blocks * grid * kBlk);
        while (nb > 0 && (P - nb) + nb * (int64_t)blk >= (1ll << 31)) nb /= 2;
        if (nb > 0) {
            ua = (uint32_t)(P - nb);
            P = (P - nb) + nb * (int64_t)blk;
        }
    }
    // Pilot ordering (SURVEY §8e "pull tiles dynamically", at pixel grain): when
    // a shard has several pixels per resident lane, the frame ends with the
    // chains of the pixels started last.  A first pass runs `pilot` samples of
    // every pixel and records its traversal steps; the remaining samples run
    // with pixels handed out most expensive first (3x3-smoothed pilot cost).
    // The passes continue each pixel's RNG stream and colour sum exactly as
    // progressive spp does, so the image is the single-pass image bit for bit.
    // 4 pilot samples; 2 at low load (at most ~2.5 pixels per resident lane,
    // where the pilot pass is a tail of its own: 1/8 shard 42.2 -> 41.3 ms,
    // 1/4 74.6 -> 73.5 ms).  Option pilot (0 = off).
    int pilot = 2 * P <= 5 * (int64_t)grid * kBlk ? 2 : 4;
    if (o.pilot >= 0) pilot = o.pilot;
    const bool ordered = pilot > 0 && !count && !a.jt && a.smp_begin == 0 && a.smp_end == a.spp &&
                         a.spp >= 2 * pilot && P < (1ll << 31);
    // Shadow offload at low load (k_path HELP): with at most ~2.5 pixels per
    // resident lane the frame is bound by the most expensive pixels' chains, and
    // 27-28 % of their traversal work is shadow queries, which feed neither the
    // RNG stream nor the path (main.cpp:57-67).  Lanes without a pixel then trace
    // other lanes' shadow queries, and (ordered passes) each 64-rank chunk pairs
    // `pair` expensive ranks with 64-pair cheap ones, whose lanes free up early.
    // Bench frame: 1/4 shard 86.4 -> 77.2 ms (pair 56), 1/8 shard 45.7 -> 43.9 ms
    // (pair 52).  Re-measured in round 5 as whole renders (help on / off,
    // profiles/r05_experiments/*_help.log): 1080p N=1 214.4 / 210.6 ms, 1/2
    // 116.6 / 120.6, 1/4 63.9 / 75.5, 1/8 36.4 / 38.8; 4K x 256 1/2 1599.6 /
    // 1531.5, 1/4 838.6 / 814.5, 1/8 450.3 / 467.9 -- it wins up to ~4 pixels
    // per resident lane and loses from ~8 (the extra shading code), so it is
    // on at <= 4.5.  Options help and pair override the choice.
    const int64_t lanes = (int64_t)grid * kBlk;
    int help = ordered && fn == fn_default && 2 * P <= 9 * lanes ? 1 : 0;
    if (o.help >= 0) help = o.help != 0 && !count && !prof && !a.jt;
    const uint32_t oct_shadow = oct_shadow_check(s);
    if (oct_shadow) help = 0;  // the helpers' shadow answers are not checked
    int pair = help && ordered ? (2 * P <= 3 * lanes ? 52 : 56) : 0;
    if (o.pair >= 0) pair = o.pair;
    if (help)
        fn = waves5p ? k_path<false, kBlk, kPathSL5, kPixSteps, kShadeMin, 5, kSparse, 0, 1>
                     : k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 4, kSparse, 0, 1>;
    else if (waves5p)
        fn = k_path<false, kBlk, kPathSL5, kPixSteps, kShadeMin, 5, kSparse>;
    // pixel seeding with the octree there: the leaves only flag ties (TIES 2)
    if (!a.jt && !count && !prof && s.oct_view && o.tie_rule == 0)
        fn = help ? (waves5p ? k_path<false, kBlk, kPathSL5, kPixSteps, kShadeMin, 5, kSparse, 0, 1, 0, false, 2>
                             : k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 4, kSparse, 0, 1, 0, false, 2>)
                  : (waves5p ? k_path<false, kBlk, kPathSL5, kPixSteps, kShadeMin, 5, kSparse, 0, 0, 0, false, 2>
                             : k_path<false, kBlk, kPathSL, kPixSteps, kShadeMin, 4, kSparse, 0, 0, 0, false, 2>);
    // stack spill areas for either kind of kernel's lanes (4 waves, 16 LDS
    // entries; 5 waves, 12)
    const size_t ovf_words = std::max((size_t)grid4 * (kStackTotal - kPathSL),
                                      (size_t)std::max(grid4, grid5) * (kStackTotal - kPathSL5)) * kBlk;
    const size_t head_words = (size_t)kSeg * kCtr;
    const size_t hist_words = ordered ? radix_sort_hist_words((int32_t)P) : 0;
    const size_t reg_words = ordered ? 2 * (size_t)kSimdKeys + 64 + (size_t)P : 0;  // + claim words
    const size_t extra_words = ordered ? (size_t)P * (4 + 5) + hist_words + reg_words : 0;
    if (ensure_ws(s, (ovf_words + head_words + extra_words) * 4)) return -1;
    uint32_t* heads = (uint32_t*)s.ws + ovf_words;
    TMPT_HIP(hipMemsetAsync(heads, 0, head_words * 4, s.stream));
    PathCtl pc;
    memset(&pc, 0, sizeof(pc));
    pc.heads = heads;
    pc.oct_shadow = oct_shadow;
    pc.P = P;
    pc.nblk = nblk;
    pc.blk = blk;
    pc.blk0 = blk0;
    pc.ua = ua;
    RenderArgs as = a;  // sample seeding: a lane's run of samples is its block
    if (a.jt) {
        as.bmask = nblk > 1 ? blk - 1u : 2047u;
        if (nblk > 1 || pass) {
            const size_t need = sizeof(float4) * (size_t)a.spp * (size_t)a.slots;
            if (s.sbuf_bytes < need) {
                if (s.sbuf) (void)hipFree(s.sbuf);
                s.sbuf = nullptr;
                s.sbuf_bytes = 0;
                TMPT_HIP(hipMalloc(&s.sbuf, need));
                s.sbuf_bytes = need;
            }
            pc.sbuf = s.sbuf;
        }
    }
    // sbuf is [pixel][sample] with nontemporal stores (a 16-B store into a
    // [sample][pixel] line pulled the whole line into L2 -- 27 GB of extra
    // fetches per 1080p frame); k_resolve_px reads it through LDS
    pc.sb_ss = 1u;
    pc.sb_sp = (uint32_t)a.spp;
    // A unit of >= 2 samples holds each even sample's colour until the next one
    // and writes both into the same 32-B sector (spp even: sectors align), so
    // the two 16-B halves can leave L2 as one write instead of two (option sbuf_pair)
    pc.pair = pc.sbuf && blk >= 2u && a.spp % 2 == 0 && o.sbuf_pair ? 1u : 0u;
    // Small shards (at most a quarter as many pixels as resident lanes): a wave
    // holds at most 32 pixels at once, so the pixels spread over more SIMD
    // slots and each wave's chain -- the frame's critical path at that load --
    // has fewer lanes to interleave (bench frame, 1/32 shard: 44.1 -> 40.9 ms;
    // at 1/16 (half the lanes) it measured 44.4 -> 45.5 ms, so not there; 16
    // lanes per wave was slower still).  Option wave_cap fixes the cap.
    {
        const int64_t waves = std::max<int64_t>(1, (int64_t)grid * (kBlk / 64));
        int64_t c = P <= waves * 16 ? 32 : 64;
        if (o.wave_cap > 0) c = o.wave_cap;
        pc.lane_cap = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(64, c));
    }
    pc.chunk = std::min<uint32_t>(kChunk, pc.lane_cap);
    pc.nchunks = (uint32_t)((P + pc.chunk - 1) / pc.chunk);
    auto final_launch = [&](const RenderArgs& af) -> int {
        TMPT_HIP(hipEventRecord(s.path_ev[2], s.stream));
        fn<<<grid, kBlk, 0, s.stream>>>(view(s), af, pc, d_out, (uint32_t*)s.ws, d_counters);
        TMPT_HIP(hipGetLastError());
        TMPT_HIP(hipEventRecord(s.path_ev[3], s.stream));
        return 0;
    };
    if (!ordered) {
        // Deferred ties (PathCtl::redo, k_path DEFER): with per-sample colours
        // (sbuf) a tied sample can be traced again on its own, so the main loop
        // runs without the octree walk and root-box test (and takes the first
        // triangle met on a tie, flagged) and the launch's waves trace the
        // dropped samples in their tail (k_redo the rest).  Only when no camera
        // ray needs the root-box test (root_check = 0).  Auto: at >= 192 samples
        // per resident lane (4 waves per SIMD), where the tail hides the
        // re-traces -- bench frame, k_path ms, base (no octree) / ties settled
        // inline / deferred: N=1 184.8 / 190.2 / 185.3, 1/2 93.1 / 96.3 / 94.9,
        // 1/4 47.7 / 49.4 / 49.8, 1/8 24.6 / 25.5 / 27.1;
        // with 5 waves per SIMD the deferring kernel wins down to the 1/8
        // shard (51 samples per lane; inline / deferred with its block rule:
        // 1/4 47.3 / 45.9, 1/8 24.3 / 24.2 ms), so from 48 per lane
        // (profiles/r06_experiments/occ5/ab_low_rules.log)
        const bool defer = a.jt && !count && !prof && !soa && pc.sbuf && a.root_check == 0 && o.tie_defer != 0 &&
                           !oct_shadow &&
                           (o.tie_defer > 0 || a.slots * (int64_t)a.spp >= (waves5 ? 48 : 192) * lanes);
        bool redo = defer && s.oct_view && o.tie_rule == 0;
        if (redo && o.redo_cap > 0 && s.redo_cap != (uint32_t)o.redo_cap) free_redo(s);  // the test hook's size
        if (redo && s.redo_cap == 0) {
            int64_t cap = std::min<int64_t>(1ll << 31, std::max<int64_t>(1 << 16, a.slots * (int64_t)a.spp / 128));
            if (o.redo_cap > 0) cap = o.redo_cap;
            (void)alloc_redo(s, cap);
        }
        const bool redo_nomem = redo && s.redo_cap == 0;
        if (redo_nomem) redo = false;
        // (the deferring kernel keeps the first triangle met on a tie and flags
        // it: only the redo pass gives those samples their answer)
        // (with the octree but no deferral: the leaf only flags ties, TIES 2)
        // five waves per SIMD (waves5, option path_waves; the 30-KB LDS layout
        // of OCC 5, 96 VGPRs): bench frame, k_path ms, 4 / 5 waves, same box:
        // N=1 185.6 / 171.0, 1/2 94.3 / 87.7
        PathFn fn_main = fn;
        if (redo)
            fn_main = waves5 ? k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 1, false, 1>
                             : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1, false, 1>;
        else if (fn == fn_default && a.jt && !count && !soa && s.oct_view && o.tie_rule == 0)
            fn_main = waves5 ? k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 1, false, 2>
                             : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1, false, 2>;
        else if (waves5 && fn == fn_default)
            fn_main = k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 1>;
        // the launch's grid is the launched kernel's co-resident block count
        // (the deferred re-traces' completion count relies on it)
        int grid_main = occupancy_grid((const void*)fn_main, kBlk, 0, s.device);
        if ((size_t)grid_main * kBlk * (kStackTotal - kPathSL5) > ovf_words) {
            set_error("tmpt_render: internal: stack spill area sized for fewer lanes");
            return -1;
        }
        s.tie_path = !(s.oct_view && o.tie_rule == 0) ? 0 : redo ? 2 : redo_nomem ? 3 : 1;
        s.path_launches = 1;
        for (int attempt = 0;; ++attempt) {
            pc.redo = redo ? s.redo : nullptr;
            pc.redo_state = redo ? s.redo_state : nullptr;
            pc.redo_cap = redo ? s.redo_cap : 0u;
            pc.redo_inline = o.redo_inline ? 1u : 0u;
            pc.redo_lanes = (uint32_t)std::max(1, std::min(64, o.redo_lanes));
            if (redo) TMPT_HIP(hipMemsetAsync(s.redo, 0xFF, sizeof(uint2) * (size_t)s.redo_cap, s.stream));
            TMPT_HIP(hipEventRecord(s.path_ev[2], s.stream));
            fn_main<<<grid_main, kBlk, 0, s.stream>>>(view(s), as, pc, d_out, (uint32_t*)s.ws, d_counters);
            TMPT_HIP(hipGetLastError());
            TMPT_HIP(hipEventRecord(s.path_ev[3], s.stream));
            if (!redo) break;
            // the list's count and the entries the launch traced itself
            TMPT_HIP(hipMemcpyAsync(s.counters_host + kRedoCounter, d_counters + kRedoCounter,
                                    4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s.stream));
            TMPT_HIP(hipStreamSynchronize(s.stream));
            const unsigned long long n = s.counters_host[kRedoCounter];
            const unsigned long long traced = s.counters_host[kRedoTraced];
            s.redo_samples = (int64_t)n;
            if (n > s.redo_cap && attempt == 0) {
                // the list overflowed: grow it to the count (the same frame lists
                // the same samples) or, failing that, render with the exact kernel
                if (!(n < (1ull << 31) && alloc_redo(s, (int64_t)n))) {
                    redo = false;
                    fn_main = waves5
                                  ? k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 1, false, 2>
                                  : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 1, false, 2>;
                    grid_main = occupancy_grid((const void*)fn_main, kBlk, 0, s.device);
                    s.redo_samples = 0;
                    s.tie_path = 3;
                }
                TMPT_HIP(hipMemsetAsync(d_counters, 0, kRenderCounters * sizeof(unsigned long long), s.stream));
                TMPT_HIP(hipMemsetAsync(heads, 0, head_words * 4, s.stream));
                continue;
            }
            s.redo_late = (int64_t)(std::min<unsigned long long>(n, s.redo_cap) - std::min(traced, n));
            if (traced < std::min<unsigned long long>(n, s.redo_cap)) {  // entries the launch left
                TMPT_HIP(hipEventRecord(s.path_ev[0], s.stream));
                k_redo<kBlk, kPathSL><<<grid, kBlk, 0, s.stream>>>(view(s), as, s.redo, s.redo_cap, s.redo_state,
                                                                  pc.sbuf, pc.sb_ss, pc.sb_sp, (uint32_t*)s.ws,
                                                                  d_counters);
                TMPT_HIP(hipGetLastError());
                TMPT_HIP(hipEventRecord(s.path_ev[1], s.stream));
                s.redo_launches = 1;  // timed apart from k_path (tmpt_stats.redo_ms)
            }
            break;
        }
        if (pc.sbuf) {
            k_resolve_px<<<(unsigned)((a.slots + 63) / 64), 64, 0, s.stream>>>(
                pc.sbuf, a.slots, a.spp, a.out_recip, d_out, a.smp_begin, a.smp_end, pass ? a.prog : nullptr);
            TMPT_HIP(hipGetLastError());
        }
        return 0;
    }
    s.tie_path = s.oct_view && o.tie_rule == 0 ? 1 : 0;  // pixel seeding answers in the main loop
    uint32_t* base = heads + head_words;
    float4* state = reinterpret_cast<float4*>(base);  // P x {colour sum, rng}
    uint32_t* cost = base + 4 * (size_t)P;
    uint32_t* keys = cost + P;
    uint32_t* vals = keys + P;
    uint32_t* tkeys = vals + P;
    uint32_t* tvals = tkeys + P;
    uint32_t* hist = tvals + P;
    uint32_t* simd_reg = hist + hist_words;
    RenderArgs a1 = a;  // pass 1: samples [0, pilot), per-pixel steps
    a1.smp_end = pilot;
    a1.out_recip = 1.0f / (float)pilot;
    a1.prog = state;
    pc.cost_out = cost;
    TMPT_HIP(hipEventRecord(s.path_ev[0], s.stream));
    fn<<<grid, kBlk, 0, s.stream>>>(view(s), a1, pc, d_out, (uint32_t*)s.ws, d_counters);
    TMPT_HIP(hipGetLastError());
    TMPT_HIP(hipEventRecord(s.path_ev[1], s.stream));
    k_order_keys<<<(unsigned)((P + 255) / 256), 256, 0, s.stream>>>(cost, a.W, a.tile_rows, keys, vals);
    const int which = radix_sort_pairs(keys, vals, tkeys, tvals, (int32_t)P, 16, hist, s.stream);
    TMPT_HIP(hipMemsetAsync(heads, 0, head_words * 4, s.stream));
    RenderArgs a2 = a;  // pass 2: samples [pilot, spp), most expensive pixels first
    a2.smp_begin = pilot;
    a2.prog = state;
    pc.cost_out = nullptr;
    pc.order = which ? tvals : vals;
    // Pixel chains (low load): at about one pixel per resident lane the frame
    // ends on the sample chains of its heaviest pixels.
    // The `chains` heaviest per 1024 (the head of the cost order) leave pass 2
    // and run as speculative chains instead -- render_rowspec's engine with one
    // pixel per chain: every even RNG offset of a window past the pilot's state
    // traced shadow-free, the chain walked through it, its samples traced again
    // in full -- so their samples run side by side, not in sequence.  Same
    // image: each sample is a pure function of (pixel, start state), summed in
    // sample order after the pilot's sum (k_resolve_chains).  Option pixel_chains.
    int64_t nch = 0;
    {
        int per1024 = 0;  // measured: no gain at the 1/8 shard, so off by default
        if (o.pixel_chains >= 0) per1024 = o.pixel_chains;
        nch = std::min<int64_t>(P, (P * per1024 + 1023) / 1024);
    }
    if (nch > 0) {
        const PixelChains ch{pc.order, state, (int)nch, pilot, a.spp - pilot};
        const int rc = render_rowspec(s, a, d_out, d_counters, &ch);
        if (rc < 0) return rc;
        if (rc == 0) {  // pass 2 takes the rest of the order
            pc.order += nch;
            pc.P = P - nch;
            pc.nchunks = (uint32_t)((pc.P + pc.chunk - 1) / pc.chunk);
        }
        s.chain_pixels = rc == 0 ? nch : 0;
    }
    if (pair > 0 && pair < 64 && pc.chunk == 64u) {
        uint32_t* paired = which ? vals : tvals;
        k_pair_order<<<(unsigned)((pc.P + 255) / 256), 256, 0, s.stream>>>(pc.order, pc.P, pair, paired);
        pc.order = paired;
    }
    // SIMD-balanced first chunks (PathCtl::simd_reg): with the chunks in
    // descending cost, the resident waves of every SIMD take one chunk from
    // each quarter, alternating ends, instead of the launch order's heaviest or
    // lightest of every quarter.  Option balance.
    if (o.balance) {
        int dev_cus = 0;
        if (hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, s.device) != hipSuccess ||
            dev_cus < 1)
            dev_cus = 256;
        const uint32_t per_cu = (uint32_t)std::max(1, grid / dev_cus);  // blocks per CU
        pc.simd_reg = simd_reg;
        pc.nsimd = (uint32_t)dev_cus * 4u;
        pc.wps = per_cu * (uint32_t)(kBlk / 64) / 4u;
        pc.claim = simd_reg + 2 * (size_t)kSimdKeys + 64;
        TMPT_HIP(hipMemsetAsync(simd_reg, 0, reg_words * 4, s.stream));
    }
    // Dynamic priority (PathCtl::dprio) in cost-ordered passes of up to ~12
    // pixels per resident lane: the heaviest waves start at the top level and
    // step down as their projected remaining work falls below 32 / 21 / 10.5 %
    // of the heaviest pixel's, so the issue slots go to the waves with the
    // most work left instead of to the oldest.  Bench frame, 1/8 shard 44.9 ->
    // 42.4 ms, 1/4 78.9 -> 75.3 ms (with the balanced first chunks; rounds
    // 1-2).  It was on only with the helpers until round 5, which measured it
    // without them (whole renders, on / off, profiles/r05_experiments/dprio_*):
    // 1080p N=1 207.1 / 209.8 ms (7.9 pixels per lane: the pass ends over
    // ~24 ms as the last pixels' 64-sample chains run out,
    // profiles/r05_wavetime/), 4K x 256 1/4 807.5 / 820.9 (7.9 per lane), but
    // 1/2 1550.4 / 1528.5 and N=1 3023.4 / 2969.0 (15.8 and 31.6 per lane: the
    // tail is short against the pass and the priority's own cost shows).
    // Option dprio.
    if (ordered && o.dprio && P <= 12 * lanes) {
        pc.dprio[0] = 0.32f;
        pc.dprio[1] = 0.21f;
        pc.dprio[2] = 0.105f;
        pc.dprio_cost = cost;
    }
    if (final_launch(a2)) return -1;
    s.path_launches = 2;
    return 0;
}

// Streaming row engine (RsStream above): one k_path<SAMP 4> launch whose first
// blocks chase the rows' chains while the rest trace the windows' units, then
// the chain's samples in full (k_path<SAMP 2> over the chain list) and the
// in-order sums (k_resolve_px).  Returns 1 when it does not apply (limits,
// memory) and 2 when the launch aborted (its watchdog: no chain progress for
// ~1 s); the caller runs render_rowspec instead.
int render_rowstream(Scene& s, const RenderArgs& a, uint32_t* d_out, unsigned long long* d_counters)
{
    const Options& o = s.opt;
    // a shading round once 24 lanes wait (16 before round 6): whole row renders,
    // 16 / 24 / 28 / 32, N=1 1835.9 / 1811.4 / 1811.9 / 1833.8 ms, 1/2 1034.8 /
    // 1023.5 / 1023.6, 1/8 432.1 / 430.4 / 427.6 / 428.3; 24 or 32 rounds per
    // check instead of 16: -0.8 / +1.2 % at N=1 (profiles/r06_experiments/row_cadence*.log)
    constexpr int kPathSL = 16, kPathSteps = TMPT_ROW_STEPS, kShadeMin = TMPT_ROW_SHADE_MIN, kSparse = 2;
    // with the reference's octree answering (tie_rule visit) the leaves only
    // flag a tie and keep the first triangle met (TIES 2): the flagged query's
    // answer comes from the octree either way, so the lowest-index bookkeeping
    // is not needed (option row_flag_leaves 0 keeps it, for A/B)
    const bool flag = s.oct_view && o.tie_rule == 0 && o.row_flag_leaves;
    using RsFn = decltype(&k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 2>);
    // the chain's full re-trace at 5 waves per SIMD (option path_waves, as the
    // sample kernels: the 30-KB LDS layout of OCC 5)
    const bool w5 = o.path_waves != 4;
    const RsFn fn2 = flag ? (w5 ? k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 2, false, 2>
                                : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 2, false, 2>)
                          : (w5 ? k_path<false, kBlk, kPathSL5, kPathSteps, kShadeMin, 5, kSparse, 0, 0, 2>
                                : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 2>);
    RsFn fn4 = flag ? k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, kRsOcc3, kSparse, 0, 0, 4, false, 2>
                    : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, kRsOcc3, kSparse, 0, 0, 4>;
    // the workers at 4 waves per SIMD (no spills) for light loads (option row_occ)
    const RsFn fn4_occ4 = flag ? k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 4, false, 2>
                               : k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 4>;
    const int rows = a.tile_rows;
    const uint32_t W = (uint32_t)a.W, spp = (uint32_t)a.spp, T = (uint32_t)kRssT;
    const size_t lcap = (size_t)a.slots * spp;  // chain samples of the tile
    // a pixel's offsets per window ~ spp x 8.5 (draws / 2); the ring holds the
    // live windows with room to spare (pow2 >= 16 x spp x 8)
    uint32_t R = 1024;
    while (R < 128u * spp) R <<= 1;
    // offsets live in 24-bit fields: ~8.5 per sample on average, 14 allowed,
    // plus 2^20 of room for the workers' fetch-adds past a window's end
    if (rows < 1 || W > 4094u || (uint64_t)W * spp * 14u + R + (1u << 20) >= (1ull << 24) || lcap >= (1ull << 31))
        return 1;
    int grid = occupancy_grid((const void*)fn4, kBlk, 0, s.device);
    const int grid2 = occupancy_grid((const void*)fn2, kBlk, 0, s.device);
    const int nchase = (rows + kBlk - 1) / kBlk;  // blocks of 4 waves x 64 rows
    if (grid <= 2 * nchase) return 1;
    {
        // 5 waves per SIMD (96 VGPRs, 10 spilled dwords) win at full load, 4
        // (no spills) once the GPU has room per row: bench frame, row seeding,
        // 4 / 5 / 6 waves, N=1 1944.7 / 1854.6 / 1889.9 ms, 1/8 436.0 / 450.5 /
        // 477.1 ms; 4 / 5 waves at 1/2 1048.8 / 1043.6, 1/4 639.7 / 658.9, 1/8
        // 434.4 / 450.4 ms (room 1.1, 2.2, 4.4; profiles/r05_experiments/
        // row_worker_occupancy*.log): 4 waves from room 1.6
        const double room5 = (double)(grid - nchase) * kBlk / ((double)rows * (double)spp * 8.5);
        const bool occ4 = o.row_occ == 4 || (o.row_occ == 0 && room5 >= 1.6);
        const int g4 = occ4 ? occupancy_grid((const void*)fn4_occ4, kBlk, 0, s.device) : 0;
        if (occ4 && g4 > 2 * nchase) {
            fn4 = fn4_occ4;
            grid = g4;
        }
    }
    // live windows per row: 2.6 + 1.5 ln(room), room = resident lanes per
    // pixel window of all rows, within 2..kRssT-1.  Bench frame, 64 spp
    // (profiles/r03_rowspec/stream_windows_*, with the spread rule below):
    // best 2 windows at N = 1 (1.82 s), 3 at 1/2 (1.05 s), 4 at 1/4 (0.65 s),
    // 4-5 at 1/8 (0.44 s); this rule picks 2, 3, 4, 5
    const int64_t lanes = (int64_t)(grid - nchase) * kBlk;
    const double E_est = (double)spp * 8.5;
    const double room = (double)lanes / ((double)rows * E_est);  // resident lanes per pixel window of all rows
    // Round 5: the chasers re-apply both rules as rows finish (RsStream::dyn,
    // room per live row): the rows end over ~500 ms of the 1.7 s launch
    // (profiles/r05_wavetime/row_*.log) and the ones left get more windows;
    // N=1 1909 -> 1875 ms, 1/2 1085 -> 1054, 1/8 462.5 -> 459.6 (option
    // rowstream_dynamic; profiles/r05_experiments/row_dynamic_windows.log).
    // More slots per row (TMPT_RSS_T=16) changed nothing (row_rss16.log).
    int nw = (int)std::lround(2.6 + 1.5 * std::log(std::max(room, 1e-3)));
    nw = std::max(2, std::min(kRssT - 1, nw));
    if (o.rowspec_windows > 0) nw = std::min(kRssT - 1, o.rowspec_windows);
    const uint32_t na = (uint32_t)(((uint64_t)W * spp * 14u + R) >> 14) + 1u;
    const size_t ovf_words = std::max((size_t)grid * (kStackTotal - kPathSL), (size_t)grid2 * (kStackTotal - kPathSL5)) * kBlk;
    const size_t head_words = (size_t)kSeg * kCtr;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b_res = al((size_t)rows * T * R * 8), b_slots = al((size_t)rows * (T + 1) * 8),
                 b_pos = al((size_t)rows * 8), b_rays = al((size_t)rows * 2 * 4), b_lo = al((size_t)rows * T * 4),
                 b_ctl = al(64), b_ctr = al(24 * 8), b_anch = al((size_t)rows * na * 4),
                 b_ovf = al((ovf_words + head_words) * 4);
    const size_t zero_bytes = b_res + b_slots + b_pos + b_rays + b_lo + b_ctl + b_ctr;
    const size_t need = zero_bytes + b_anch + b_ovf;
    const size_t lneed = lcap * sizeof(uint32_t), sneed = lcap * sizeof(float4);
    {
        size_t fr = 0, tot = 0;
        const size_t budget = (hipMemGetInfo(&fr, &tot) == hipSuccess ? fr / 4 * 3 : 0) + s.rss_bytes +
                              s.rs_list_bytes + s.sbuf_bytes;
        if (need + lneed + sneed > budget) return 1;
    }
    auto grow = [](void*& p, size_t& have, size_t want) -> int {
        if (have >= want) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        have = 0;
        if (hipMalloc(&p, want) != hipSuccess) return -1;
        have = want;
        return 0;
    };
    // HBM short after the budget check (another allocation raced it): the
    // iterated engine may still fit, so fall back rather than fail the frame
    // (grow() has freed the old buffer; the failed hipMalloc's error is cleared)
    if (grow(s.rss_buf, s.rss_bytes, need) || grow(s.rs_list, s.rs_list_bytes, lneed)) {
        (void)hipGetLastError();
        return 1;
    }
    {
        void* sb = s.sbuf;
        const int g = grow(sb, s.sbuf_bytes, sneed);
        s.sbuf = static_cast<float4*>(sb);
        if (g) {
            (void)hipGetLastError();
            return 1;
        }
    }
    if (!s.rss_tab) {  // M^(2c) and M^(256b) for c, b < 128; M^(2^15 a0), M^(2^20 a1) for a0, a1 < 32
        std::vector<uint32_t> tab, t;
        jump_tables(2, 128, t);
        tab.insert(tab.end(), t.begin(), t.end());
        jump_tables(256, 128, t);
        tab.insert(tab.end(), t.begin(), t.end());
        jump_tables(1ull << 15, 32, t);
        tab.insert(tab.end(), t.begin(), t.end());
        jump_tables(1ull << 20, 32, t);
        tab.insert(tab.end(), t.begin(), t.end());
        uint32_t* nt = nullptr;
        TMPT_HIP(hipMalloc(&nt, tab.size() * sizeof(uint32_t)));
        if (hipMemcpy(nt, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(nt);
            set_error("render_rowstream: jump table upload failed");
            return -1;
        }
        s.rss_tab = nt;
    }
    if (!s.rss_host) TMPT_HIP(hipHostMalloc((void**)&s.rss_host, 16 * sizeof(uint32_t), hipHostMallocDefault));
    char* p = static_cast<char*>(s.rss_buf);
    RsStream S;
    memset(&S, 0, sizeof(S));
    S.res = reinterpret_cast<unsigned long long*>(p);
    p += b_res;
    S.slots = reinterpret_cast<unsigned long long*>(p);
    p += b_slots;
    S.chainpos = reinterpret_cast<unsigned long long*>(p);
    p += b_pos;
    S.rowrays = reinterpret_cast<uint32_t*>(p);
    p += b_rays;
    S.lo = reinterpret_cast<uint32_t*>(p);
    p += b_lo;
    S.ctl = reinterpret_cast<uint32_t*>(p);
    p += b_ctl;
    unsigned long long* spec_ctr = reinterpret_cast<unsigned long long*>(p);  // traced (not chain) rays
    p += b_ctr;
    S.anchors = reinterpret_cast<uint32_t*>(p);
    p += b_anch;
    uint32_t* ovf = reinterpret_cast<uint32_t*>(p);
    uint32_t* heads = ovf + ovf_words;
    S.list = static_cast<uint32_t*>(s.rs_list);
    S.t1 = s.rss_tab;
    S.t2 = s.rss_tab + 128 * 1024;
    S.na = na;
    S.jlimit = na << 14;
    S.R = R;
    S.rmask = R - 1u;
    S.nrows = rows;
    S.nchase = nchase;
    S.nw = nw;
    S.watchdog = o.rowstream_test_abort ? 200000u : 100000000u;  // ~1 s (2 ms when testing the abort)
    S.test_abort = o.rowstream_test_abort;
    // window spread in pixels: 0.055 x room - 0.015, within 0..0.25.  Bench
    // frame, 64 spp (profiles/r03_rowspec/stream_spread_*): best at 0 - 0.02
    // for N = 1 (1.82 s; 2.03 s at the earlier 0.10), 0.06 - 0.08 at 1/2, 0.12 -
    // 0.15 at 1/4, 0.18 - 0.22 at 1/8 (0.44 s); at full load the chaser's demand
    // and extension windows are cheaper than a wide spread
    S.spread = o.rowspec_spread >= 0.0f ? o.rowspec_spread
                                        : (float)std::min(0.25, std::max(0.0, 0.055 * room - 0.015));
    S.room_lanes = (float)((double)lanes / E_est);
    S.dyn = o.rowstream_dynamic ? ((o.rowspec_windows > 0 ? 0u : 1u) | (o.rowspec_spread >= 0.0f ? 0u : 2u)) : 0u;
    TMPT_HIP(hipMemsetAsync(s.rss_buf, 0, zero_bytes, s.stream));
    {
        const size_t n = (size_t)rows * na;
        k_rss_anchors<<<(unsigned)((n + 255) / 256), 256, 0, s.stream>>>(a, S, s.rss_tab + 256 * 1024,
                                                                        s.rss_tab + 288 * 1024);
        TMPT_HIP(hipGetLastError());
    }
    RenderArgs as = a;
    as.jt = nullptr;
    as.bmask = 0u;  // every unit is one sample
    as.smp_begin = 0;
    as.smp_end = a.spp;
    PathCtl pc;
    memset(&pc, 0, sizeof(pc));
    pc.heads = heads;
    pc.nblk = pc.blk = 1u;
    pc.lane_cap = 64u;
    pc.chunk = kChunk;
    pc.rs_noshadow = 1;
    pc.oct_shadow = oct_shadow_check(s);
    pc.rss = S;
    fn4<<<grid, kBlk, 0, s.stream>>>(view(s), as, pc, d_out, ovf, spec_ctr);
    TMPT_HIP(hipGetLastError());
    TMPT_HIP(hipMemcpyAsync(s.rss_host, S.ctl, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
    TMPT_HIP(hipStreamSynchronize(s.stream));
#ifdef TMPT_EXP_WAVETIME
    {
        std::vector<unsigned long long> w(3 * kWaveTimeMax, 0ull), r(kWaveTimeMax, 0ull), cl(kWaveTimeMax, 0ull);
        if (hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_wavetime), w.size() * 8) == hipSuccess &&
            hipMemcpyFromSymbol(r.data(), HIP_SYMBOL(g_rowtime), r.size() * 8) == hipSuccess &&
            hipMemcpyFromSymbol(cl.data(), HIP_SYMBOL(g_claimtime), cl.size() * 8) == hipSuccess) {
            unsigned long long t0 = ~0ull, tend = 0;
            for (int i = 0; i < kWaveTimeMax; ++i)
                if (w[3 * i] && w[3 * i + 2]) {
                    t0 = std::min(t0, w[3 * i]);
                    tend = std::max(tend, w[3 * i + 2]);
                }
            std::vector<double> rt;
            for (int i = 0; i < std::min(rows, kWaveTimeMax); ++i)
                if (r[i]) rt.push_back((r[i] - t0) * 0.01);
            std::sort(rt.begin(), rt.end());
            auto q = [&](double f) { return rt.empty() ? 0.0 : rt[std::min(rt.size() - 1, (size_t)(f * (rt.size() - 1)))]; };
            fprintf(stderr, "rowstream rows %zu done at us p0/p10/p50/p90/p99/p100 %.0f/%.0f/%.0f/%.0f/%.0f/%.0f; "
                            "last worker exit %.0f\n",
                    rt.size(), q(0), q(0.1), q(0.5), q(0.9), q(0.99), q(1), (tend - t0) * 0.01);
            std::vector<double> lc;  // each worker wave's last claim of speculation work
            for (int i = 0; i < kWaveTimeMax; ++i)
                if (w[3 * i] && w[3 * i + 2] && cl[i]) lc.push_back((cl[i] - t0) * 0.01);
            std::sort(lc.begin(), lc.end());
            auto ql = [&](double f) { return lc.empty() ? 0.0 : lc[std::min(lc.size() - 1, (size_t)(f * (lc.size() - 1)))]; };
            fprintf(stderr, "rowstream workers %zu: last claim at us p0/p10/p25/p50/p75/p90/p100 "
                            "%.0f/%.0f/%.0f/%.0f/%.0f/%.0f/%.0f\n",
                    lc.size(), ql(0), ql(0.1), ql(0.25), ql(0.5), ql(0.75), ql(0.9), ql(1));
            std::fill(w.begin(), w.end(), 0ull);
            std::fill(r.begin(), r.end(), 0ull);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wavetime), w.data(), w.size() * 8);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rowtime), r.data(), r.size() * 8);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_claimtime), r.data(), r.size() * 8);
        }
    }
#endif
    if (s.rss_host[1] != 0u || s.rss_host[3] != 0u || s.rss_host[0] != (uint32_t)rows) {
#ifdef TMPT_DIAG
        fprintf(stderr, "rowstream: aborted (rows done %u of %d, abort %u, error %u); iterated engine instead\n",
                s.rss_host[0], rows, s.rss_host[1], s.rss_host[3]);
#endif
        return 2;  // launched and aborted: the caller falls back and records it (tmpt_stats.stream_fallbacks)
    }
    // the chain's samples in full (shadows included), then the in-order sums
    k_rss_states<<<(unsigned)((lcap + 255) / 256), 256, 0, s.stream>>>(a, S);
    PathCtl pc2 = pc;
    pc2.upix = nullptr;  // unit u = sample u % spp of tile pixel u / spp
    pc2.uslot = nullptr;
    pc2.ustate = S.list;
    pc2.p_dev = S.ctl + 4;
    pc2.rs_noshadow = 0;
    pc2.sbuf = s.sbuf;
    pc2.sb_ss = 1u;
    pc2.sb_sp = spp;
    TMPT_HIP(hipMemsetAsync(heads, 0, head_words * 4, s.stream));
    fn2<<<grid2, kBlk, 0, s.stream>>>(view(s), as, pc2, d_out, ovf, spec_ctr + 16);
    k_resolve_px<<<(unsigned)((a.slots + 63) / 64), 64, 0, s.stream>>>(s.sbuf, a.slots, a.spp, a.spp_recip, d_out);
    k_rss_count<<<(unsigned)((rows + 255) / 256), 256, 0, s.stream>>>(S, d_counters);
    TMPT_HIP(hipGetLastError());
    s.path_launches = 1;
#ifdef TMPT_DIAG
    if (getenv("TMPT_ROWSPEC_LOG")) {
        unsigned long long c[2] = {0, 0}, t = 0;
        TMPT_HIP(hipMemcpyAsync(c, d_counters, sizeof(c), hipMemcpyDeviceToHost, s.stream));
        TMPT_HIP(hipMemcpyAsync(&t, spec_ctr, sizeof(t), hipMemcpyDeviceToHost, s.stream));
        TMPT_HIP(hipStreamSynchronize(s.stream));
        fprintf(stderr,
                "rowstream: %d rows, %d worker blocks + %d chaser blocks, ring %u, %d windows, traced rays %llu for "
                "%llu chain rays (x%.2f), chain ticks %u\n"
                "rowstream: claims %u, row misses %u, lost CAS %u; chaser waits %u, extensions %u, prefixes %u, "
                "sweeps %u\n",
                rows, grid - nchase, nchase, R, nw, t, c[0], c[0] ? (double)t / (double)c[0] : 0.0, s.rss_host[2],
                s.rss_host[5], s.rss_host[6], s.rss_host[7], s.rss_host[8], s.rss_host[9], s.rss_host[10],
                s.rss_host[11]);
    }
#endif
    return 0;
}

// Speculative row seeding (k_rs_* above): iterations of plan -> fill ->
// k_path<SAMP 2> -> chase until every row of the tile has its W pixels.  Each
// iteration moves every unfinished row through (usually) one pixel.  The rows
// are split into G groups, each iterating on its own stream, so one group's
// k_path tail overlaps another's work; the unit counts stay on the device and
// the host only checks for completion every kCheck iterations.
int render_rowspec(Scene& s, const RenderArgs& a, uint32_t* d_out, unsigned long long* d_counters,
                   const PixelChains* ch)
{
    const Options& o = s.opt;
    // rows: a.tile_rows chains of W pixels x spp samples; pixel chains (ch):
    // ch->n chains of one pixel x ch->cspp samples
    const int cspp = ch ? ch->cspp : a.spp;
    constexpr int kPathSL = 16, kPathSteps = 16, kShadeMin = 16, kSparse = 2, kCheck = 64;
    auto fn = k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, 4, kSparse, 0, 0, 2>;
    // the shadow-free pass: its own instantiation (no shadow, light or colour
    // code, no light / next-ray LDS): 96 VGPRs, 5 waves per SIMD (6 waves: 80
    // VGPRs and 21 spilled dwords, neutral)
    auto fn3 = k_path<false, kBlk, kPathSL, kPathSteps, kShadeMin, kRsOcc3, kSparse, 0, 0, 3>;
    const int grid = occupancy_grid((const void*)fn, kBlk, 0, s.device);
    const int grid3 = occupancy_grid((const void*)fn3, kBlk, 0, s.device);
    const int rows = ch ? ch->n : a.tile_rows;
    // window cap: one iteration covers a pixel's samples at up to 2 * wmax / spp
    // = 48 draws per sample (the stand-in sponza averages ~17, its deepest rows
    // ~25; a cap of 24 draws left those rows one short window per pixel, and
    // the slowest row sets the iteration count)
    uint32_t wmax = (uint32_t)std::min<int64_t>(8192, std::max<int64_t>(64, (int64_t)cspp * 24));
    if (o.rowspec_wmax > 0) wmax = (uint32_t)o.rowspec_wmax;
    // row groups, each on its own stream (one group: 3 % slower)
    const int G = std::max(1, std::min(std::min(o.rowspec_groups, kRowSpecMaxGroups), rows));
    // every group's k_path gets the whole resident grid (splitting the GPU
    // between the groups, or reserving fewer than 64 units per wave, did not help)
    const int pgrid = grid, pgrid3 = grid3;
    const uint32_t chunk = kChunk;
    // lookahead windows (pixels x+1, x+2, ...; each around its expected
    // start and end): one iteration covers up to nwin pixels of a row.  The
    // extra speculation is cheap while the GPU has room: nwin ~ 5 units per
    // resident lane over the rows' expected pixel windows (~17 draws per
    // sample), 2..kRsMaxWin -- 2 on the whole bench frame, 8 from 1/4 of it.
    // The far windows' spread grows with a pixel's units E = spp x ~8.5, so
    // the windows of one iteration are also capped at ~4400 units per row
    // (8 windows at 64 spp).  Measured (profiles/r02_rowspec/rs16): 640x360x4
    // suzanne 88 -> 51 ms with 8 -> 32 windows; the 1/8 shard of the bench
    // frame 708 ms with 8 windows, 746 with 18.
    const int64_t lanes = (int64_t)pgrid * kBlk;
    const double E_est = (double)cspp * 8.5;
    int nwin = (int)std::lround(std::min((double)lanes * 5.0 / ((double)rows * E_est), 4400.0 / E_est));
    nwin = std::max(2, std::min(kRsMaxWin, nwin));
    if (o.rowspec_windows > 0) nwin = std::min(kRsMaxWin, o.rowspec_windows);
    if (ch) nwin = 1;  // a pixel chain has one pixel: no lookahead windows
    const uint32_t jmax = (uint32_t)nwin * wmax;  // window i ends by (i + 1) * wmax
    // Speculate without shadow traversals and re-trace the chain in full at the
    // end (the frame's chain list and colour buffer must fit; else the colours
    // come from the speculative pass).  Bench frame 3.03 -> 2.49 s, 1/8 shard
    // 0.71 -> 0.61 s (profiles/r02_rowspec/rs19).  Option rowspec_noshadow.
    bool noshadow = o.rowspec_noshadow != 0 || ch;
    // chain samples of the tile (pixel chains: theirs); the colour buffer is
    // the tile's [pixel][sample] in either case
    const size_t lcap = ch ? (size_t)ch->n * (size_t)cspp : (size_t)a.slots * (size_t)a.spp;
    const uint32_t scap = (uint32_t)nwin * (uint32_t)cspp;  // a row's chain samples per iteration
    if (noshadow) {
        const size_t lneed = lcap * 3 * sizeof(uint32_t) + (size_t)rows * scap * sizeof(uint2) + 256;
        const size_t sneed = (size_t)a.slots * (size_t)a.spp * sizeof(float4);
        size_t fr = 0, tot = 0;
        const size_t budget = (hipMemGetInfo(&fr, &tot) == hipSuccess ? fr / 4 * 3 : 0) + s.rs_list_bytes + s.sbuf_bytes;
        if (lcap >= (1ull << 32) || lneed + sneed > budget) {
            if (ch) return 1;  // pixel chains need the re-trace: the caller renders them in pass 2
            noshadow = false;  // does not fit: the colours come from the speculative pass
        } else {
            if (s.rs_list_bytes < lneed) {
                if (s.rs_list) (void)hipFree(s.rs_list);
                s.rs_list = nullptr;
                s.rs_list_bytes = 0;
                TMPT_HIP(hipMalloc(&s.rs_list, lneed));
                s.rs_list_bytes = lneed;
            }
            if (s.sbuf_bytes < sneed) {
                if (s.sbuf) (void)hipFree(s.sbuf);
                s.sbuf = nullptr;
                s.sbuf_bytes = 0;
                TMPT_HIP(hipMalloc(&s.sbuf, sneed));
                s.sbuf_bytes = sneed;
            }
        }
    }
    uint32_t* lpix = nullptr;
    uint32_t* lstate = nullptr;
    uint32_t* lslot = nullptr;
    uint32_t* lcount = nullptr;
    uint2* scratch = nullptr;
    if (noshadow) {
        lcount = static_cast<uint32_t*>(s.rs_list);
        scratch = reinterpret_cast<uint2*>(static_cast<char*>(s.rs_list) + 256);
        lpix = reinterpret_cast<uint32_t*>(scratch + (size_t)rows * scap);
        lstate = lpix + lcap;
        lslot = lstate + lcap;
    }
    if (s.jt2_n < (int32_t)jmax) {  // J_j = M^(2j): the state 2j draws on
        std::vector<uint32_t> tab;
        jump_tables(2, (int32_t)jmax, tab);
        uint32_t* nt = nullptr;
        TMPT_HIP(hipMalloc(&nt, tab.size() * sizeof(uint32_t)));
        if (hipMemcpy(nt, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(nt);
            set_error("tmpt_render: jump table upload failed");
            return -1;
        }
        if (s.jt2) (void)hipFree(s.jt2);
        s.jt2 = nt;
        s.jt2_n = (int32_t)jmax;
    }
    const size_t ovf_words = (size_t)std::max(pgrid, pgrid3) * kBlk * (kStackTotal - kPathSL);
    const size_t head_words = (size_t)kSeg * kCtr;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    auto group_rows = [&](int g) { return rows / G + (g < rows % G ? 1 : 0); };
    auto group_bytes = [&](int g) {
        const size_t R = (size_t)group_rows(g), U = R * jmax;
        return al(U * (sizeof(float4) + 3 * sizeof(uint32_t)) + R * sizeof(float4) +
                  ((9 + 2 * (size_t)kRsMaxWin) * R + 2) * sizeof(uint32_t) +
                  (ovf_words + head_words) * sizeof(uint32_t));
    };
    size_t need = al(24 * sizeof(unsigned long long));
    for (int g = 0; g < G; ++g) need += group_bytes(g);
    if (s.rs_bytes < need) {
        if (s.rs_buf) (void)hipFree(s.rs_buf);
        s.rs_buf = nullptr;
        s.rs_bytes = 0;
        TMPT_HIP(hipMalloc(&s.rs_buf, need));
        s.rs_bytes = need;
    }
    if (!s.rs_host) TMPT_HIP(hipHostMalloc((void**)&s.rs_host, kRowSpecMaxGroups * sizeof(uint32_t)));
    for (int g = 0; g < G; ++g)
        if (!s.rs_stream[g]) {
            TMPT_HIP(hipStreamCreateWithFlags(&s.rs_stream[g], hipStreamNonBlocking));
            TMPT_HIP(hipEventCreateWithFlags(&s.rs_event[g], hipEventDisableTiming));
        }
    if (!s.rs_event[kRowSpecMaxGroups]) TMPT_HIP(hipEventCreateWithFlags(&s.rs_event[kRowSpecMaxGroups], hipEventDisableTiming));
    char* p = static_cast<char*>(s.rs_buf);
    unsigned long long* spec_ctr = reinterpret_cast<unsigned long long*>(p);  // every traced unit's rays
    p += al(24 * sizeof(unsigned long long));
    struct Group {
        RowSpec rs;
        PathCtl pc;
        float4* rs_out;
        uint32_t *upix, *ustate, *rs_end, *heads, *ovf;
        size_t U;
        hipStream_t st;
    };
    std::vector<Group> gs(G);
    RenderArgs as = a;
    as.jt = nullptr;
    as.bmask = 0u;  // every unit is one sample
    as.smp_begin = 0;
    as.smp_end = a.spp;
    int row0 = 0;
    for (int g = 0; g < G; ++g) {
        Group& q = gs[g];
        char* gp = p;
        p += group_bytes(g);
        const size_t R = (size_t)group_rows(g);
        q.U = R * jmax;
        q.st = s.rs_stream[g];
        q.rs.row0 = row0;
        q.rs.nrows = (int)R;
        q.rs.wmax = wmax;
        q.rs.nwin = nwin;
        // window placement: expected positions +- spread * sqrt(i) pixels;
        // bench frame, 64 spp (profiles/r02_rowspec/rs15): spread 0.08 / 0.1 /
        // 0.12 / 0.15 = 3.06 / 3.03 / 3.04 / 3.10 s whole, 0.85 / 0.74 / 0.69 /
        // 0.67 s at 1/8 -- wider at low load, where speculation is cheap
        // (with shadow-free speculation: 1/8 shard spread 0.154 / 0.2 = 640 / 576 ms,
        // whole frame 0.106 / 0.14 / 0.2 = 2.51 / 2.52 / 2.62 s, rs20)
        q.rs.spread = o.rowspec_spread >= 0.0f ? o.rowspec_spread : 0.07f + 0.016f * (float)nwin;
        row0 += (int)R;
        q.rs_out = reinterpret_cast<float4*>(gp);
        gp += q.U * sizeof(float4);
        q.rs.col = reinterpret_cast<float4*>(gp);
        gp += R * sizeof(float4);
        uint32_t* w = reinterpret_cast<uint32_t*>(gp);
        q.upix = w;
        q.ustate = q.upix + q.U;
        q.rs_end = q.ustate + q.U;
        w = q.rs_end + q.U;
        uint32_t** fields[] = {&q.rs.rng, &q.rs.x, &q.rs.k, &q.rs.pdraws, &q.rs.prev_mean,
                               &q.rs.rays, &q.rs.erays, &q.rs.short_win};
        for (uint32_t** f : fields) {
            *f = w;
            w += R;
        }
        q.rs.win = w;  // kRsMaxWin x R each
        w += kRsMaxWin * R;
        q.rs.ws = w;
        w += kRsMaxWin * R;
        q.rs.offs = w;  // rows + 1
        w += R + 1;
        q.rs.total = w;
        w += 1;
        q.ovf = w;
        q.heads = w + ovf_words;
        memset(&q.pc, 0, sizeof(q.pc));
        q.pc.heads = q.heads;
        q.pc.nblk = q.pc.blk = 1u;
        q.pc.lane_cap = 64u;
        q.pc.chunk = chunk;
        q.pc.upix = q.upix;
        q.pc.ustate = q.ustate;
        q.pc.rs_out = q.rs_out;
        q.pc.rs_end = q.rs_end;
        q.pc.p_dev = q.rs.total;
        q.pc.rs_noshadow = noshadow ? 1 : 0;
        q.pc.oct_shadow = oct_shadow_check(s);
        q.rs.lpix = lpix;
        q.rs.lstate = lstate;
        q.rs.lslot = lslot;
        q.rs.lcount = lcount;
        q.rs.scratch = scratch ? scratch + (size_t)q.rs.row0 * scap : nullptr;
        q.rs.scap = scap;
        q.rs.planned = spec_ctr + 8;
        q.rs.cpix = ch ? ch->cpix + q.rs.row0 : nullptr;
        q.rs.cinit = ch ? ch->cinit : nullptr;
        q.rs.cw = ch ? 1 : a.W;
        q.rs.cspp = cspp;
        q.rs.smp0 = ch ? ch->smp0 : 0;
    }
    // the groups start after the work already on the scene's stream (the
    // caller's wait), and that stream resumes after all of them
    TMPT_HIP(hipMemsetAsync(spec_ctr, 0, 24 * sizeof(unsigned long long), s.stream));
    if (noshadow) TMPT_HIP(hipMemsetAsync(lcount, 0, 4, s.stream));
    TMPT_HIP(hipEventRecord(s.rs_event[kRowSpecMaxGroups], s.stream));
    for (Group& q : gs) {
        TMPT_HIP(hipStreamWaitEvent(q.st, s.rs_event[kRowSpecMaxGroups], 0));
        k_rs_init<<<(unsigned)((q.rs.nrows + 255) / 256), 256, 0, q.st>>>(a, q.rs);
    }
    TMPT_HIP(hipGetLastError());
    // the listing pass's chase walks in LDS (one wave per row) when a row's
    // chain samples of one iteration fit its list; option rowspec_chase 0 = the
    // one-thread-per-row kernel
    const bool chase_lds = noshadow && o.rowspec_chase != 0 && (uint64_t)nwin * (uint64_t)cspp <= kChaseList;
    int it = 0;
    // every iteration moves each unfinished row by >= 1 sample, so W * spp bounds them
    const int64_t max_it = (int64_t)(ch ? 1 : a.W) * cspp + kCheck;
    bool done = false;
    // pixel chains finish in a few iterations: the host looks after each one
    // (an empty iteration still launches the persistent grid, ~0.3 ms)
    const int check = ch ? 1 : kCheck;
    while (!done && it < max_it) {
        for (int c = 0; c < check; ++c, ++it)
            for (Group& q : gs) {
                k_rs_plan<<<1, 1024, 0, q.st>>>(a, q.rs);
                k_rs_fill<<<(unsigned)((q.U + 255) / 256), 256, 0, q.st>>>(a, q.rs, s.jt2, q.upix, q.ustate);
                TMPT_HIP(hipMemsetAsync(q.heads, 0, head_words * 4, q.st));
                if (noshadow) fn3<<<pgrid3, kBlk, 0, q.st>>>(view(s), as, q.pc, d_out, q.ovf, spec_ctr);
                else fn<<<pgrid, kBlk, 0, q.st>>>(view(s), as, q.pc, d_out, q.ovf, spec_ctr);
                if (chase_lds)
                    k_rs_chase_lds<<<(unsigned)q.rs.nrows, 64, 0, q.st>>>(a, q.rs, q.rs_out, q.rs_end, q.upix,
                                                                         q.ustate);
                else
                    k_rs_chase<<<(unsigned)((q.rs.nrows + 63) / 64), 64, 0, q.st>>>(a, q.rs, q.rs_out, q.rs_end,
                                                                                    d_out, q.upix, q.ustate);
            }
        TMPT_HIP(hipGetLastError());
        // the last plan of each group: 0 units = the group was already done
        for (int g = 0; g < G; ++g)
            TMPT_HIP(hipMemcpyAsync(&s.rs_host[g], gs[g].rs.total, 4, hipMemcpyDeviceToHost, gs[g].st));
        done = true;
        for (int g = 0; g < G; ++g) {
            TMPT_HIP(hipStreamSynchronize(gs[g].st));
            done = done && s.rs_host[g] == 0;
        }
    }
    if (!done) {  // cannot happen: every iteration moves each unfinished row on
        set_error("render_rowspec: rows unfinished after " + std::to_string(it) + " iterations");
        for (Group& q : gs) (void)hipStreamSynchronize(q.st);
        return -1;
    }
    for (int g = 0; g < G; ++g) {
        k_rs_count<<<(unsigned)((gs[g].rs.nrows + 255) / 256), 256, 0, gs[g].st>>>(gs[g].rs, d_counters);
        TMPT_HIP(hipEventRecord(s.rs_event[g], gs[g].st));
        TMPT_HIP(hipStreamWaitEvent(s.stream, s.rs_event[g], 0));
    }
    TMPT_HIP(hipGetLastError());
    if (noshadow) {  // the chain's samples in full (shadows included), then the in-order sums
        PathCtl pc2 = gs[0].pc;
        pc2.upix = lpix;
        pc2.ustate = lstate;
        pc2.uslot = lslot;
        pc2.p_dev = lcount;
        pc2.rs_noshadow = 0;
        pc2.sbuf = s.sbuf;
        pc2.sb_ss = 1u;
        pc2.sb_sp = (uint32_t)a.spp;
        TMPT_HIP(hipMemsetAsync(gs[0].heads, 0, head_words * 4, s.stream));
        fn<<<pgrid, kBlk, 0, s.stream>>>(view(s), as, pc2, d_out, gs[0].ovf, spec_ctr + 16);
        if (ch)
            k_resolve_chains<<<(unsigned)((ch->n + 255) / 256), 256, 0, s.stream>>>(*ch, s.sbuf, a.spp, a.spp_recip,
                                                                                   d_out);
        else
            k_resolve_px<<<(unsigned)((a.slots + 63) / 64), 64, 0, s.stream>>>(s.sbuf, a.slots, a.spp, a.spp_recip,
                                                                                d_out);
        TMPT_HIP(hipGetLastError());
    }
    s.path_launches = it;
#ifdef TMPT_DIAG
    if (getenv("TMPT_ROWSPEC_LOG")) {
        unsigned long long c[2] = {0, 0};
        TMPT_HIP(hipMemcpyAsync(c, d_counters, sizeof(c), hipMemcpyDeviceToHost, s.stream));
        unsigned long long t = 0;
        TMPT_HIP(hipMemcpyAsync(&t, spec_ctr, sizeof(t), hipMemcpyDeviceToHost, s.stream));
        std::vector<uint32_t> sw(rows), pm(rows);
        for (Group& q : gs) {
            TMPT_HIP(hipMemcpyAsync(sw.data() + q.rs.row0, q.rs.short_win, q.rs.nrows * 4, hipMemcpyDeviceToHost, s.stream));
            TMPT_HIP(hipMemcpyAsync(pm.data() + q.rs.row0, q.rs.prev_mean, q.rs.nrows * 4, hipMemcpyDeviceToHost, s.stream));
        }
        TMPT_HIP(hipStreamSynchronize(s.stream));
        double pmsum = 0.0;
        for (uint32_t v : pm) {
            float f;
            memcpy(&f, &v, 4);
            pmsum += f;
        }
        unsigned long long planned = 0;
        TMPT_HIP(hipMemcpy(&planned, spec_ctr + 8, sizeof(planned), hipMemcpyDeviceToHost));
        fprintf(stderr, "rowspec: last pixel's draws per sample, mean over rows %.2f; units planned %llu (%.1f rays each)\n",
                rows ? pmsum / rows : 0.0, planned, planned ? (double)t / (double)planned : 0.0);
        uint64_t swsum = 0;
        uint32_t swmax = 0;
        for (uint32_t v : sw) {
            swsum += v;
            swmax = std::max(swmax, v);
        }
        fprintf(stderr,
                "rowspec: %d iterations enqueued, %d groups of %d blocks, window cap %u, %d windows, traced rays "
                "%llu for %llu chain rays (x%.2f); short windows per row: mean %.1f max %u\n",
                it, G, pgrid, wmax, nwin, t, c[0], c[0] ? (double)t / (double)c[0] : 0.0,
                rows ? (double)swsum / rows : 0.0, swmax);
    }
#endif
    return 0;
}

// rays: n x 6 floats (one [tmin, tmax] for all) or, ranged, n x 8 (per ray)
// the render counters (device), their pinned host copy and the render's two
// timing events: created once per scene, so a render call costs no allocation
// (it matters for the small shards of a multi-GPU frame); the octree's
// counters live in the same array (Scene::ties)
int ensure_counters(Scene& s)
{
    if (s.counters) return 0;
    TMPT_HIP(hipMalloc(&s.counters, kRenderCounters * sizeof(unsigned long long)));
    TMPT_HIP(hipMemset(s.counters, 0, kRenderCounters * sizeof(unsigned long long)));
    TMPT_HIP(hipHostMalloc((void**)&s.counters_host, kRenderCounters * sizeof(unsigned long long),
                           hipHostMallocDefault));
    for (auto& e : s.render_ev) TMPT_HIP(hipEventCreate(&e));
    s.ties = s.counters + kTieCounter;
#ifdef TMPT_CHECK
    TMPT_HIP(hipMalloc(&s.chk, 4 * sizeof(uint32_t)));
    TMPT_HIP(hipMemset(s.chk, 0, 4 * sizeof(uint32_t)));
#endif
    return 0;
}

// The checked build's report (tmpt_internal.h kChk*): after a call's kernels
// are done, kCheckError with the codes, the count and the last offending
// value when any index test failed (the word triple is cleared for the next
// call); 0 otherwise, and always 0 in the product build.
int check_report(Scene& s, const char* what)
{
#ifdef TMPT_CHECK
    if (!s.chk) return 0;
    uint32_t h[3] = {0, 0, 0};
    TMPT_HIP(hipDeviceSynchronize());
    TMPT_HIP(hipMemcpy(h, s.chk, sizeof(h), hipMemcpyDeviceToHost));
    if (h[0] == 0) return 0;
    TMPT_HIP(hipMemset(s.chk, 0, 4 * sizeof(uint32_t)));
    char msg[256];
    snprintf(msg, sizeof(msg),
             "%s: device index check failed: codes 0x%x (1 node, 2 leaf, 4 stack, 8 octree skip, 16 octree refs, "
             "32 triangle id), %u times, last value %d",
             what, h[0], h[1], (int)h[2]);
    fprintf(stderr, "tmpt: %s\n", msg);
    set_error(msg);
    return kCheckError;
#else
    (void)s;
    (void)what;
    return 0;
#endif
}

int intersect_batch(Scene& s, const float* d_rays, int64_t n, float tmin, float tmax, bool any, bool ranged,
                    float* d_hits, int32_t* d_ids)
{
    if (ensure_counters(s)) return -1;
    TMPT_HIP(hipMemsetAsync(s.ties, 0, 2 * sizeof(unsigned long long), s.stream));
    TMPT_HIP(hipMemsetAsync(s.counters + kCrackCounter, 0, sizeof(unsigned long long), s.stream));
    const bool soa = s.soa.na != nullptr;
    // one range starting behind the origin takes the NEG slack too
    const bool neg1 = !ranged && tmin < 0.0f;
    auto fn = soa ? (ranged ? (any ? k_intersect<true, true, kBlk, kSL, true> : k_intersect<false, true, kBlk, kSL, true>)
                    : neg1  ? (any ? k_intersect<true, false, kBlk, kSL, true, true>
                                   : k_intersect<false, false, kBlk, kSL, true, true>)
                            : (any ? k_intersect<true, false, kBlk, kSL, true> : k_intersect<false, false, kBlk, kSL, true>))
                  : (ranged ? (any ? k_intersect<true, true, kBlk, kSL> : k_intersect<false, true, kBlk, kSL>)
                    : neg1  ? (any ? k_intersect<true, false, kBlk, kSL, false, true>
                                   : k_intersect<false, false, kBlk, kSL, false, true>)
                            : (any ? k_intersect<true, false, kBlk, kSL> : k_intersect<false, false, kBlk, kSL>));
    int grid = occupancy_grid((const void*)fn, kBlk, 0, s.device);
    grid = (int)std::max<int64_t>(1, std::min<int64_t>(grid, (n + kBlk - 1) / kBlk));
    size_t ovf_bytes = (size_t)grid * kBlk * (kStackTotal - kSL) * sizeof(uint32_t);
    if (ensure_ws(s, ovf_bytes)) return -1;
    fn<<<grid, kBlk, 0, s.stream>>>(view(s), d_rays, n, tmin, tmax, d_hits, d_ids, (uint32_t*)s.ws);
    TMPT_HIP(hipGetLastError());
    TMPT_HIP(hipMemcpyAsync(s.counters_host + kTieCounter, s.ties, 2 * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost, s.stream));
    TMPT_HIP(hipMemcpyAsync(s.counters_host + kCrackCounter, s.counters + kCrackCounter, sizeof(unsigned long long),
                            hipMemcpyDeviceToHost, s.stream));
    return 0;
}

int render(Scene& s, const tmpt_camera* cam, const tmpt_render_desc* d, uint32_t* d_out,
           uint64_t* ray_count)
{
    RenderArgs a = make_args(cam, d);
    bool count = (d->flags & TMPT_FLAG_COUNT_VISITS) != 0;
    // progressive spp: keep per-pixel state for the shard between calls
    const bool progressive = a.smp_begin > 0 || a.smp_end < a.spp;
    if (progressive) {
        const int32_t key[6] = {d->width, d->height, d->spp, a.band_rows, a.shard, a.nshards};
        // the carried colour sums and RNG states belong to one camera: a pass
        // with another camera (or seeding) must not blend into them
        uint64_t cam_key = 1469598103934665603ull;
        const unsigned char* cb = reinterpret_cast<const unsigned char*>(cam);
        for (size_t i = 0; i < sizeof(tmpt_camera); ++i) cam_key = (cam_key ^ cb[i]) * 1099511628211ull;
        cam_key = (cam_key ^ (uint32_t)d->seed_mode) * 1099511628211ull;
        if (a.smp_begin > 0 &&
            (memcmp(key, s.prog_key, sizeof(key)) != 0 || s.prog_key[6] != a.smp_begin || s.prog_cam != cam_key)) {
            set_error("tmpt_render: spp_begin does not continue the previous pass of this shard "
                      "(same camera, size, spp and shard)");
            return -22;
        }
        s.prog_cam = cam_key;
        if (s.prog_slots < (size_t)a.slots) {
            if (s.prog) (void)hipFree(s.prog);
            s.prog = nullptr;
            s.prog_slots = 0;
            TMPT_HIP(hipMalloc(&s.prog, sizeof(float4) * (size_t)a.slots));
            s.prog_slots = (size_t)a.slots;
        }
        a.prog = s.prog;
        memcpy(s.prog_key, key, sizeof(key));
        s.prog_key[6] = -1;  // valid again only once this pass completes
    }
    if (a.seed_mode == TMPT_SEED_SAMPLE) {  // jump tables of sample_seed, grown to spp
        if (s.jt_spp < a.spp) {
            std::vector<uint32_t> tab;
            sample_jump_tables(a.spp, tab);
            uint32_t* nt = nullptr;
            TMPT_HIP(hipMalloc(&nt, tab.size() * sizeof(uint32_t)));
            if (hipMemcpy(nt, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipFree(nt);
                set_error("tmpt_render: jump table upload failed");
                return -1;
            }
            if (s.jt) (void)hipFree(s.jt);
            s.jt = nt;
            s.jt_spp = a.spp;
        }
        a.jt = s.jt;
    }
    if (d->flags & TMPT_FLAG_WAIT_STREAM) {  // order after the caller's stream (tmpt.h)
        if (!s.wait_ev) TMPT_HIP(hipEventCreateWithFlags(&s.wait_ev, hipEventDisableTiming));
        hipError_t e = hipEventRecord(s.wait_ev, reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(d->wait_stream)));
        if (e == hipSuccess) e = hipStreamWaitEvent(s.stream, s.wait_ev, 0);
        if (e != hipSuccess) {
            set_error(std::string("tmpt_render: wait_stream: ") + hipGetErrorString(e));
            return -1;
        }
    }
    if (ensure_counters(s)) return -1;
    // camera rays take the reference's root box test unless the whole lens
    // (origin +- lens_radius along u and v) lies inside the root box by more
    // than tMin and a rounding margin: a ray from inside always passes it
    if (s.oct && s.opt.tie_rule == 0) {
        const float o[3] = {a.cam.origin.x, a.cam.origin.y, a.cam.origin.z};
        const float uu[3] = {a.cam.u.x, a.cam.u.y, a.cam.u.z}, vv[3] = {a.cam.v.x, a.cam.v.y, a.cam.v.z};
        bool inside = true;
        for (int c = 0; c < 3; ++c) {
            const double r = (double)a.cam.lens_radius * (std::fabs((double)uu[c]) + std::fabs((double)vv[c]));
            const double m = 2.0 * kMinT + 1e-4 * ((double)s.oct_hi[c] - (double)s.oct_lo[c]);
            inside = inside && (double)o[c] - r > (double)s.oct_lo[c] + m && (double)o[c] + r < (double)s.oct_hi[c] - m;
        }
        a.root_check = inside ? 0 : 1;
    }
    unsigned long long* d_counters = s.counters;
    TMPT_HIP(hipMemsetAsync(d_counters, 0, kRenderCounters * sizeof(unsigned long long), s.stream));
    hipEvent_t e0 = s.render_ev[0], e1 = s.render_ev[1];
    TMPT_HIP(hipEventRecord(e0, s.stream));
    int rc = 0;
    const bool wave = d->engine == TMPT_ENGINE_WAVEFRONT && a.seed_mode != TMPT_SEED_ROW;
    const bool persistent = d->engine == TMPT_ENGINE_PERSISTENT && a.seed_mode != TMPT_SEED_ROW;
    // row seeding on the persistent engine: the speculative row chains
    // (render_rowspec); instrumented renders and option rowspec=0 run the
    // megakernel's one lane per row
    const bool rowspec = d->engine == TMPT_ENGINE_PERSISTENT && a.seed_mode == TMPT_SEED_ROW && !count &&
                         !progressive && s.opt.rowspec != 0;
    if (progressive && !persistent) {
        set_error("tmpt_render: progressive spp needs the persistent engine");
        return -22;
    }
    s.extend_ms = s.shadow_ms = 0;
    s.extend_rays = s.shadow_rays = s.node_visits = s.tri_tests = 0;
    s.shadow_node_visits = s.shadow_tri_tests = 0;
    s.extend_launches = s.shadow_launches = s.iterations = 0;
    s.row_engine = 0;
    s.stream_fallbacks = 0;
    s.chain_pixels = 0;
    s.redo_samples = 0;
    s.redo_late = 0;
    s.redo_launches = 0;
    s.redo_ms = 0.0;
    s.redo_rays = 0;
    s.tie_path = 0;
    if (a.slots > 0) {
        if (wave) rc = render_wavefront(s, a, d_out, count);
        else if (persistent) rc = render_persistent(s, a, d_out, count, d_counters);
        else if (rowspec) {
            // the streaming engine, or the iterated one where it does not apply
            rc = s.opt.rowspec_stream != 0 && s.opt.rowspec_noshadow != 0 ? render_rowstream(s, a, d_out, d_counters)
                                                                          : 1;
            s.row_engine = rc == 0 ? 3 : 2;
            if (rc == 2) {  // the streaming launch aborted: its counters are partial, start over
                s.stream_fallbacks = 1;
                TMPT_HIP(hipMemsetAsync(d_counters, 0, kRenderCounters * sizeof(unsigned long long), s.stream));
            }
            if (rc == 1 || rc == 2) rc = render_rowspec(s, a, d_out, d_counters);
        } else {
            rc = render_megakernel(s, a, d_out, count, d_counters);
            if (a.seed_mode == TMPT_SEED_ROW) s.row_engine = 1;
        }
    }
    (void)hipEventRecord(e1, s.stream);
    hipError_t se = rc == 0 ? hipMemcpyAsync(s.counters_host, d_counters, kRenderCounters * sizeof(unsigned long long),
                                             hipMemcpyDeviceToHost, s.stream)
                            : hipSuccess;
    const hipError_t se2 = hipStreamSynchronize(s.stream);
    if (se == hipSuccess) se = se2;
    unsigned long long c[kRenderCounters] = {};
    if (rc == 0 && se == hipSuccess) memcpy(c, s.counters_host, sizeof(c));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rc) return rc;
    if (se != hipSuccess) {
        set_error(std::string("render: ") + hipGetErrorString(se));
        return -1;
    }
    s.render_ms = ms;
    s.tie_queries = c[kTieCounter];
    s.root_misses = c[kTieCounter + 1];
    s.crack_queries = c[kCrackCounter];
#ifdef TMPT_EXP_WAVETIME
    {
        std::vector<unsigned long long> w(3 * kWaveTimeMax, 0ull);
        if (hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_wavetime), w.size() * 8) == hipSuccess) {
            std::vector<double> st, ml, ex;
            unsigned long long t0 = ~0ull;
            for (int i = 0; i < kWaveTimeMax; ++i)
                if (w[3 * i] && w[3 * i + 2]) t0 = std::min(t0, w[3 * i]);
            for (int i = 0; i < kWaveTimeMax; ++i)
                if (w[3 * i] && w[3 * i + 2]) {
                    st.push_back((w[3 * i] - t0) * 0.01);  // 100 MHz ticks -> us
                    ml.push_back((w[3 * i + 1] - t0) * 0.01);
                    ex.push_back((w[3 * i + 2] - t0) * 0.01);
                }
            auto pct = [](std::vector<double> v, double q) {
                if (v.empty()) return 0.0;
                std::sort(v.begin(), v.end());
                return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1)))];
            };
            fprintf(stderr, "waves %zu; start us p0/p50/p100 %.0f/%.0f/%.0f; main loop end p0/p10/p50/p90/p100 "
                            "%.0f/%.0f/%.0f/%.0f/%.0f; exit p0/p50/p99/p100 %.0f/%.0f/%.0f/%.0f\n",
                    st.size(), pct(st, 0), pct(st, 0.5), pct(st, 1), pct(ml, 0), pct(ml, 0.1), pct(ml, 0.5),
                    pct(ml, 0.9), pct(ml, 1), pct(ex, 0), pct(ex, 0.5), pct(ex, 0.99), pct(ex, 1));
            std::fill(w.begin(), w.end(), 0ull);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wavetime), w.data(), w.size() * 8);
        }
    }
#endif
#ifdef TMPT_EXP_CRACKSTAT
    {
        unsigned long long w[4] = {0, 0, 0, 0};
        if (hipMemcpyFromSymbol(w, HIP_SYMBOL(g_crackstat), sizeof(w)) == hipSuccess && w[0]) {
            fprintf(stderr, "crack test: %llu finished hits, first stage true %llu (%.3f %%), both stages %llu, "
                            "t < reach %llu (%.3f %%)\n",
                    w[0], w[1], 100.0 * w[1] / w[0], w[2], w[3], 100.0 * w[3] / w[0]);
            const unsigned long long z[4] = {0, 0, 0, 0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_crackstat), z, sizeof(z));
        }
    }
#endif
#ifdef TMPT_EXP_WALKSTAT
    {
        unsigned long long w[4] = {0, 0, 0, 0};
        if (hipMemcpyFromSymbol(w, HIP_SYMBOL(g_walkstat), sizeof(w)) == hipSuccess && w[3]) {
            fprintf(stderr, "octree walks %llu: nodes %.1f, triangles %.1f per walk, max nodes %llu\n", w[3],
                    (double)w[0] / w[3], (double)w[1] / w[3], w[2]);
            const unsigned long long z[4] = {0, 0, 0, 0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_walkstat), z, sizeof(z));
        }
    }
#endif
    if (progressive) s.prog_key[6] = a.smp_end < a.spp ? a.smp_end : -1;
    if (persistent) {  // one kernel for both query kinds
        // k_path launches only (the render's other kernels: order keys, sort,
        // resolve, memsets excluded)
        float k1 = 0.0f, k0 = 0.0f;
        (void)hipEventElapsedTime(&k1, s.path_ev[2], s.path_ev[3]);
        if (s.path_launches == 2) (void)hipEventElapsedTime(&k0, s.path_ev[0], s.path_ev[1]);
        s.extend_ms = (double)k0 + (double)k1;
        if (s.redo_launches) {  // the k_redo launch after the main one: its own figure
            float kr = 0.0f;
            (void)hipEventElapsedTime(&kr, s.path_ev[0], s.path_ev[1]);
            s.redo_ms = kr;
            s.redo_rays = c[kRedoRaysCounter];
        }
        s.extend_rays = c[3];
        s.shadow_rays = c[0] - c[3];
        s.node_visits = c[1];
        s.tri_tests = c[2];
        s.shadow_node_visits = c[4];
        s.shadow_tri_tests = c[5];
        s.extend_launches = s.path_launches;  // same k_path instantiation per launch
        s.iterations = 1;
#ifdef TMPT_DIAG
        if (c[13] + c[14] + c[15]) {
            const double tot = (double)(c[13] + c[14] + c[15]);
            fprintf(stderr, "k_path wave time: shading %.1f%%, node rounds %.1f%%, leaf rounds %.1f%% "
                            "(%.3g wave-cycles)\n",
                    100.0 * c[13] / tot, 100.0 * c[14] / tot, 100.0 * c[15] / tot, tot);
            if (c[6] && c[8] && c[10])
                fprintf(stderr, "  cycles per round: node %.0f (%.1f lanes), leaf %.0f (%.1f lanes), shading %.0f "
                                "(%.1f lanes shading, %.1f traversing); rounds node %llu leaf %llu shading %llu\n",
                        (double)c[14] / c[6], (double)c[7] / c[6], (double)c[15] / c[8], (double)c[9] / c[8],
                        (double)c[13] / c[10], (double)c[11] / c[10], (double)c[12] / c[10], c[6], c[8], c[10]);
            if (c[16] + c[17] + c[18] + c[19])
                fprintf(stderr, "  shading split: ballots+pixel fetch %.1f%%, shade/finish %.1f%%, camera %.1f%%, "
                                "query set-up %.1f%% (of all wave time)\n",
                        100.0 * c[16] / tot, 100.0 * c[17] / tot, 100.0 * c[18] / tot, 100.0 * c[19] / tot);
        }
        if (count && getenv("TMPT_ROUND_LOG"))  // wave-round efficiency
            fprintf(stderr,
                    "k_path rounds: node %llu (%.1f lanes), leaf %llu (%.1f lanes), shade %llu "
                    "(%.1f wanting, %.1f traversing)\n",
                    c[6], c[6] ? (double)c[7] / c[6] : 0.0, c[8], c[8] ? (double)c[9] / c[8] : 0.0,
                    c[10], c[10] ? (double)c[11] / c[10] : 0.0, c[10] ? (double)c[12] / c[10] : 0.0);
#endif
    } else if (rowspec) {
        s.extend_ms = ms;
        s.extend_rays = c[3];
        s.shadow_rays = c[0] - c[3];
        s.extend_launches = s.path_launches;
        s.iterations = s.path_launches;
    } else if (!wave) {
        s.extend_ms = ms;
        s.extend_rays = c[0];
        s.node_visits = c[1];
        s.tri_tests = c[2];
        s.extend_launches = 1;
    }
    if (ray_count) *ray_count = wave ? (s.extend_rays + s.shadow_rays) : c[0];
    return 0;
}

}  // namespace tmpt
