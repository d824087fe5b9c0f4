// tmpt_bvh.hip -- on-device LBVH build for gfx950, replacing the reference's
// octree build (Scene::BuildOctree / OctreeNode::Subdivide, scene.cpp:75-83, 99-160).
//
// Pipeline (all on the scene's stream; DESIGN.md "LBVH build"):
//   1. k_tri_prep     per triangle: TriOrig record (v0,v1,v2,normal), padded leaf
//                     box, centroid; centroid bounds by block reduction + one
//                     ordered-int atomic per block and axis
//   2. k_morton       30-bit Morton code of the normalised centroid
//   3. radix sort     4 x 8-bit LSD passes; per pass: tile histograms, one scan,
//                     stable scatter ranked with wave64 ballots (no LDS atomics)
//   4. k_karras       Karras 2012 hierarchy over (code, index) keys
//   5. k_depth        node depth by walking parent links (<= 62 steps)
//   6. k_refit_level  boxes bottom-up, one launch per level: the kernel boundary
//                     is the only inter-workgroup synchronisation, so no
//                     cross-XCD release/acquire is needed
//   or, the default, PLOC (Meister & Bittner 2018) over the same sorted keys:
//      k_ploc_nn / k_ploc_merge / k_ploc_compact per iteration, then
//      top-down leaf numbering (k_ploc_offsets / relabel / vals)
//   7. k_tri_pre      leaf-ordered TriPre records
//   8. k_bvh4_level   top-down collapse to the 4-wide quantised BVH, one launch
//                     per level (greedy largest-area opening, or the SAH-optimal
//                     forests of k_sah_level)
// The build is outside the timed region of the reference (main.cpp:312 vs
// :319) and of bench.py; it is timed separately (Scene::build_ms).
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <string>
#include <chrono>
#include <cmath>
#include <mutex>
#include <thread>
#include <vector>

#include "tmpt_internal.h"

namespace tmpt {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t f2ord(float f)
{
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u)
{
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

struct Soa6 {  // leaf or node boxes, structure of arrays for coalesced sweeps
    float *lx, *ly, *lz, *hx, *hy, *hz;
};

__global__ void __launch_bounds__(kBlock) k_tri_prep(const float* __restrict__ tris9, int32_t n,
                                                     TriOrig* __restrict__ orig, Soa6 box,
                                                     float* __restrict__ cent,
                                                     uint32_t* __restrict__ cbounds /*6*/)
{
    __shared__ uint32_t red[6][kBlock / 64];
    int i = blockIdx.x * kBlock + threadIdx.x;
    float c[3] = {INFINITY, INFINITY, INFINITY};
    float cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (i < n) {
        const float* t = tris9 + 9 * (int64_t)i;
        f3 v0 = mk(t[0], t[1], t[2]), v1 = mk(t[3], t[4], t[5]), v2 = mk(t[6], t[7], t[8]);
        f3 nrm = tri_normal(v0, v1, v2);
        orig[i].a = f4(v0.x, v0.y, v0.z, v1.x);
        orig[i].b = f4(v1.y, v1.z, v2.x, v2.y);
        orig[i].c = f4(v2.z, nrm.x, nrm.y, nrm.z);
        f3 lo = vmin(vmin(v0, v1), v2), hi = vmax(vmax(v0, v1), v2);
        float px = kBoxPadRel * (fmaxf(fabsf(lo.x), fabsf(hi.x)) + (hi.x - lo.x)) + 1e-30f;
        float py = kBoxPadRel * (fmaxf(fabsf(lo.y), fabsf(hi.y)) + (hi.y - lo.y)) + 1e-30f;
        float pz = kBoxPadRel * (fmaxf(fabsf(lo.z), fabsf(hi.z)) + (hi.z - lo.z)) + 1e-30f;
        box.lx[i] = lo.x - px; box.ly[i] = lo.y - py; box.lz[i] = lo.z - pz;
        box.hx[i] = hi.x + px; box.hy[i] = hi.y + py; box.hz[i] = hi.z + pz;
        float cx = 0.5f * (lo.x + hi.x), cy = 0.5f * (lo.y + hi.y), cz = 0.5f * (lo.z + hi.z);
        cent[i] = cx; cent[n + i] = cy; cent[2 * n + i] = cz;
        c[0] = cmax[0] = cx; c[1] = cmax[1] = cy; c[2] = cmax[2] = cz;
    }
    // wave64 reductions, then one atomic per block and component
    uint32_t v[6] = {f2ord(c[0]), f2ord(c[1]), f2ord(c[2]),
                     f2ord(cmax[0]), f2ord(cmax[1]), f2ord(cmax[2])};
    for (int off = 32; off > 0; off >>= 1) {
        for (int k = 0; k < 3; ++k) v[k] = min(v[k], (uint32_t)__shfl_xor((int)v[k], off));
        for (int k = 3; k < 6; ++k) v[k] = max(v[k], (uint32_t)__shfl_xor((int)v[k], off));
    }
    int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
        for (int k = 0; k < 6; ++k) red[k][wave] = v[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        int k = threadIdx.x;
        uint32_t r = red[k][0];
        for (int w = 1; w < kBlock / 64; ++w) r = k < 3 ? min(r, red[k][w]) : max(r, red[k][w]);
        if (k < 3) atomicMin(&cbounds[k], r);
        else atomicMax(&cbounds[k], r);
    }
}

__device__ __forceinline__ uint32_t expand10(uint32_t v)
{
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void __launch_bounds__(kBlock) k_morton(const float* __restrict__ cent, int32_t n,
                                                   const uint32_t* __restrict__ cbounds,
                                                   uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float q[3];
    for (int k = 0; k < 3; ++k) {
        float lo = ord2f(cbounds[k]), hi = ord2f(cbounds[3 + k]);
        float ext = hi - lo;
        float x = ext > 0.0f ? (cent[k * n + i] - lo) / ext : 0.5f;
        q[k] = fminf(fmaxf(x * 1024.0f, 0.0f), 1023.0f);
    }
    keys[i] = (expand10((uint32_t)q[0]) << 2) | (expand10((uint32_t)q[1]) << 1) |
              expand10((uint32_t)q[2]);
    vals[i] = (uint32_t)i;
}

// ---------------------------------------------------------------- radix sort
constexpr int kSortItems = 4;
constexpr int kSortTile = kBlock * kSortItems;

__global__ void __launch_bounds__(kBlock) k_sort_hist(const uint32_t* __restrict__ keys, int32_t n,
                                                      int shift, int nblocks,
                                                      uint32_t* __restrict__ hist)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    int base = blockIdx.x * kSortTile;
    for (int r = 0; r < kSortItems; ++r) {
        int i = base + r * kBlock + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];  // digit-major
}

// exclusive scan of m entries by one block of 1024 threads
__global__ void __launch_bounds__(1024) k_scan_1block(uint32_t* __restrict__ a, int m)
{
    __shared__ uint32_t part[1024];
    int per = (m + 1023) / 1024;
    int b = threadIdx.x * per, e = min(b + per, m);
    uint32_t s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;  // exclusive
    for (int i = b; i < e; ++i) {
        uint32_t x = a[i];
        a[i] = run;
        run += x;
    }
}

// Stable scatter: keys of a tile are ranked in (round, thread) order; within a
// wave, lanes with the same digit are found by 8 ballots (one per digit bit).
__global__ void __launch_bounds__(kBlock) k_sort_scatter(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout,
                                                         uint32_t* __restrict__ vout, int32_t n,
                                                         int shift, int nblocks,
                                                         const uint32_t* __restrict__ offs)
{
    __shared__ uint32_t run[256];
    __shared__ uint32_t wcnt[kBlock / 64][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    run[threadIdx.x] = offs[threadIdx.x * nblocks + blockIdx.x];
    const uint64_t lt = (1ull << lane) - 1ull;
    int base = blockIdx.x * kSortTile;
    for (int r = 0; r < kSortItems; ++r) {
        for (int w = 0; w < kBlock / 64; ++w) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        int i = base + r * kBlock + threadIdx.x;
        bool valid = i < n;
        uint32_t key = valid ? kin[i] : 0u, val = valid ? vin[i] : 0u;
        uint32_t dg = (key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
        for (int bit = 0; bit < 8; ++bit) {
            uint64_t bal = __ballot((dg >> bit) & 1u);
            peers &= ((dg >> bit) & 1u) ? bal : ~bal;
        }
        uint32_t wrank = (uint32_t)__popcll(peers & lt);
        if (valid && wrank == 0) wcnt[wave][dg] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[dg] + wrank;
            for (int w = 0; w < wave; ++w) pos += wcnt[w][dg];
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
        uint32_t add = 0;
        for (int w = 0; w < kBlock / 64; ++w) add += wcnt[w][threadIdx.x];
        run[threadIdx.x] += add;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- hierarchy
__device__ __forceinline__ int delta(const uint32_t* __restrict__ keys, int32_t n, int i, int j)
{
    if (j < 0 || j > n - 1) return -1;
    uint32_t a = keys[i], b = keys[j];
    if (a == b) return 32 + __clz((int)((uint32_t)i ^ (uint32_t)j));
    return __clz((int)(a ^ b));
}

// Karras, "Maximizing Parallelism in the Construction of BVHs, Octrees and k-d
// Trees" (HPG 2012), Fig. 4.  Children: >=0 internal, <0 leaf (~slot).
__global__ void __launch_bounds__(kBlock) k_karras(const uint32_t* __restrict__ keys, int32_t n,
                                                   int2* __restrict__ child,
                                                   int2* __restrict__ range,
                                                   int32_t* __restrict__ parent_int,
                                                   int32_t* __restrict__ parent_leaf)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n - 1) return;
    int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    int j = i + l * d;
    int dnode = delta(keys, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    int gamma = i + s * d + min(d, 0);
    int lo = min(i, j), hi = max(i, j);
    int c0 = (lo == gamma) ? ~gamma : gamma;
    int c1 = (hi == gamma + 1) ? ~(gamma + 1) : gamma + 1;
    child[i] = make_int2(c0, c1);
    range[i] = make_int2(lo, hi);  // the node covers sorted leaf slots lo..hi
    if (c0 < 0) parent_leaf[~c0] = i; else parent_int[c0] = i;
    if (c1 < 0) parent_leaf[~c1] = i; else parent_int[c1] = i;
    if (i == 0) parent_int[0] = -1;
}

__global__ void __launch_bounds__(kBlock) k_depth(const int32_t* __restrict__ parent_int,
                                                  int32_t m, int32_t* __restrict__ depth,
                                                  int32_t* __restrict__ max_depth)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    int dd = 0;
    for (int p = i; p > 0 && dd < 4096; p = parent_int[p]) ++dd;
    depth[i] = dd;
    atomicMax(max_depth, dd);
}

__device__ __forceinline__ void child_box(int c, const Soa6& leaf, const uint32_t* __restrict__ vals,
                                          const Soa6& ib, float b[6])
{
    if (c < 0) {
        int o = (int)vals[~c];
        b[0] = leaf.lx[o]; b[1] = leaf.ly[o]; b[2] = leaf.lz[o];
        b[3] = leaf.hx[o]; b[4] = leaf.hy[o]; b[5] = leaf.hz[o];
    } else {
        b[0] = ib.lx[c]; b[1] = ib.ly[c]; b[2] = ib.lz[c];
        b[3] = ib.hx[c]; b[4] = ib.hy[c]; b[5] = ib.hz[c];
    }
}

__global__ void __launch_bounds__(kBlock) k_refit_level(const int2* __restrict__ child,
                                                        const int32_t* __restrict__ depth,
                                                        int32_t m, int level, Soa6 leaf,
                                                        const uint32_t* __restrict__ vals, Soa6 ib)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= m || depth[i] != level) return;
    int2 c = child[i];
    float a[6], b[6];
    child_box(c.x, leaf, vals, ib, a);
    child_box(c.y, leaf, vals, ib, b);
    ib.lx[i] = fminf(a[0], b[0]); ib.ly[i] = fminf(a[1], b[1]); ib.lz[i] = fminf(a[2], b[2]);
    ib.hx[i] = fmaxf(a[3], b[3]); ib.hy[i] = fmaxf(a[4], b[4]); ib.hz[i] = fmaxf(a[5], b[5]);
}

// ---------------------------------------------------------------- PLOC
// Parallel Locally-Ordered Clustering (Meister & Bittner, TVCG 2018) over the
// Morton order: every cluster finds its nearest neighbour (smallest union
// surface area) within +-r positions; mutual pairs merge into a new node; the
// survivors are compacted in order.  Produces SAH-grade trees from the same
// sorted keys as the LBVH.  Nodes are numbered in creation order (children
// before parents), the root is the last one.
__device__ __forceinline__ float half_area(float lx, float ly, float lz, float hx, float hy, float hz)
{
    float dx = hx - lx, dy = hy - ly, dz = hz - lz;
    return dx * dy + dy * dz + dz * dx;
}

__global__ void __launch_bounds__(kBlock) k_ploc_init(int32_t n, Soa6 leaf, const uint32_t* __restrict__ vals,
                                                      int32_t* __restrict__ cid, Soa6 cb)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    int o = (int)vals[i];
    cid[i] = ~i;
    cb.lx[i] = leaf.lx[o]; cb.ly[i] = leaf.ly[o]; cb.lz[i] = leaf.lz[o];
    cb.hx[i] = leaf.hx[o]; cb.hy[i] = leaf.hy[o]; cb.hz[i] = leaf.hz[o];
}

__global__ void __launch_bounds__(kBlock) k_ploc_nn(int32_t N, int r, Soa6 cb, int32_t* __restrict__ nn)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    const float lx = cb.lx[i], ly = cb.ly[i], lz = cb.lz[i], hx = cb.hx[i], hy = cb.hy[i], hz = cb.hz[i];
    float best = INFINITY;
    int bj = -1;
    const int j0 = max(0, i - r), j1 = min(N - 1, i + r);
    for (int j = j0; j <= j1; ++j) {
        if (j == i) continue;
        float d = half_area(fminf(lx, cb.lx[j]), fminf(ly, cb.ly[j]), fminf(lz, cb.lz[j]),
                            fmaxf(hx, cb.hx[j]), fmaxf(hy, cb.hy[j]), fmaxf(hz, cb.hz[j]));
        if (d < best) {  // ascending j: ties keep the lower index
            best = d;
            bj = j;
        }
    }
    nn[i] = bj;
}

__global__ void __launch_bounds__(kBlock) k_ploc_merge(int32_t N, const int32_t* __restrict__ nn,
                                                       int32_t* __restrict__ cid, Soa6 cb,
                                                       uint32_t* __restrict__ valid, int2* __restrict__ child,
                                                       Soa6 ib, int32_t* __restrict__ size,
                                                       int32_t* __restrict__ iter, int it,
                                                       uint32_t* __restrict__ counter)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    int j = nn[i];
    bool mutual = j >= 0 && nn[j] == i;
    if (mutual && i < j) {
        int k = (int)atomicAdd(counter, 1u);
        int c0 = cid[i], c1 = cid[j];
        child[k] = make_int2(c0, c1);
        float lx = fminf(cb.lx[i], cb.lx[j]), ly = fminf(cb.ly[i], cb.ly[j]), lz = fminf(cb.lz[i], cb.lz[j]);
        float hx = fmaxf(cb.hx[i], cb.hx[j]), hy = fmaxf(cb.hy[i], cb.hy[j]), hz = fmaxf(cb.hz[i], cb.hz[j]);
        ib.lx[k] = lx; ib.ly[k] = ly; ib.lz[k] = lz; ib.hx[k] = hx; ib.hy[k] = hy; ib.hz[k] = hz;
        size[k] = (c0 < 0 ? 1 : size[c0]) + (c1 < 0 ? 1 : size[c1]);
        iter[k] = it;
        cid[i] = k;
        cb.lx[i] = lx; cb.ly[i] = ly; cb.lz[i] = lz; cb.hx[i] = hx; cb.hy[i] = hy; cb.hz[i] = hz;
        valid[i] = 1;
    } else {
        valid[i] = (mutual && i > j) ? 0u : 1u;
    }
}

__global__ void __launch_bounds__(kBlock) k_ploc_compact(int32_t N, const uint32_t* __restrict__ valid,
                                                         const uint32_t* __restrict__ pos,
                                                         const int32_t* __restrict__ cid, Soa6 cb,
                                                         int32_t* __restrict__ cid2, Soa6 cb2)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= N || !valid[i]) return;
    uint32_t d = pos[i];
    cid2[d] = cid[i];
    cb2.lx[d] = cb.lx[i]; cb2.ly[d] = cb.ly[i]; cb2.lz[d] = cb.lz[i];
    cb2.hx[d] = cb.hx[i]; cb2.hy[d] = cb.hy[i]; cb2.hz[d] = cb.hz[i];
}

// Leaf renumbering so every subtree covers a contiguous slot range (needed by
// multi-triangle leaves): top-down offsets, one launch per PLOC iteration in
// reverse (a node's parent was created in a later iteration).
__global__ void __launch_bounds__(kBlock) k_ploc_offsets(int32_t m, int it, const int32_t* __restrict__ iter,
                                                         const int2* __restrict__ child,
                                                         const int32_t* __restrict__ size,
                                                         int32_t* __restrict__ off,
                                                         uint32_t* __restrict__ new_slot)
{
    int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= m || iter[k] != it) return;
    int o = off[k];
    int2 c = child[k];
    int s0 = c.x < 0 ? 1 : size[c.x];
    if (c.x >= 0) off[c.x] = o; else new_slot[~c.x] = (uint32_t)o;
    if (c.y >= 0) off[c.y] = o + s0; else new_slot[~c.y] = (uint32_t)(o + s0);
}

__global__ void __launch_bounds__(kBlock) k_ploc_relabel(int32_t m, int2* __restrict__ child,
                                                         const int32_t* __restrict__ off,
                                                         const int32_t* __restrict__ size,
                                                         int2* __restrict__ range,
                                                         const uint32_t* __restrict__ new_slot)
{
    int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    int2 c = child[k];
    if (c.x < 0) c.x = ~(int)new_slot[~c.x];
    if (c.y < 0) c.y = ~(int)new_slot[~c.y];
    child[k] = c;
    range[k] = make_int2(off[k], off[k] + size[k] - 1);
}

__global__ void __launch_bounds__(kBlock) k_ploc_vals(int32_t n, const uint32_t* __restrict__ new_slot,
                                                      const uint32_t* __restrict__ vals,
                                                      uint32_t* __restrict__ vals2)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) vals2[new_slot[i]] = vals[i];
}

// ---------------------------------------------------------------- BVH4Q collapse
__device__ __forceinline__ float box_area(const float b[6])
{
    float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;
}

__device__ __forceinline__ void node_or_leaf_box(int c, const Soa6& leaf,
                                                 const uint32_t* __restrict__ vals, const Soa6& ib,
                                                 float b[6])
{
    child_box(c, leaf, vals, ib, b);
}

// ---------------------------------------------------------------- SAH collapse (DP)
// Optimal BVH2 -> BVH4 collapse under the surface-area cost model (the dynamic
// programme of Ylitie, Karras & Laine 2017, "Efficient incoherent ray
// traversal on GPUs through compressed wide BVHs", for 4 children and
// multi-triangle leaves).  For every BVH2 node n, F(n, j) = the least cost of
// representing n's subtree as a forest of at most j roots (j = 1..4):
//   F(n,1) = min( A(n)(c_leaf + c_tri count(n))     [leaf, count <= leaf_max],
//                 A(n) c_node + min_k F(l,k) + F(r,4-k) )   [wide node]
//   F(n,j) = min( F(n,j-1), min_k F(l,k) + F(r,j-k) )
// computed bottom-up one BVH2 level per launch (levels from a BFS), then the
// top-down collapse expands each wide node's forest from the stored choices.
struct SahCost {
    float c_node, c_leaf, c_tri;
};

__global__ void __launch_bounds__(kBlock) k_bfs_level(const int2* __restrict__ child,
                                                      const int32_t* __restrict__ cur, int nc,
                                                      int32_t* __restrict__ next,
                                                      uint32_t* __restrict__ counter)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nc) return;
    const int2 c = child[cur[i]];
    if (c.x >= 0) next[atomicAdd(counter, 1u)] = c.x;
    if (c.y >= 0) next[atomicAdd(counter, 1u)] = c.y;
}

__global__ void __launch_bounds__(kBlock) k_sah_level(const int2* __restrict__ child,
                                                      const int2* __restrict__ range, Soa6 leaf,
                                                      const uint32_t* __restrict__ vals, Soa6 ib,
                                                      const int32_t* __restrict__ nodes, int nn,
                                                      float4* __restrict__ F, uint32_t* __restrict__ dec,
                                                      int leaf_max, SahCost cost)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nn) return;
    const int n = nodes[i];
    const int2 c = child[n];
    float fl[5], fr[5];
    auto child_f = [&](int ch, float f[5]) {
        if (ch < 0) {  // one triangle: a leaf whatever the root budget
            float b[6];
            child_box(ch, leaf, vals, ib, b);
            const float v = box_area(b) * (cost.c_leaf + cost.c_tri);
            f[1] = f[2] = f[3] = f[4] = v;
        } else {
            const float4 q = F[ch];
            f[1] = q.x; f[2] = q.y; f[3] = q.z; f[4] = q.w;
        }
    };
    child_f(c.x, fl);
    child_f(c.y, fr);
    float b[6];
    child_box(n, leaf, vals, ib, b);
    const float an = box_area(b);
    const int cnt = range[n].y - range[n].x + 1;
    uint32_t d = 0;
    // wide node: its children are the best forest of <= 4 roots of l and r
    float best4 = INFINITY;
    int k4 = 1;
    for (int k = 1; k <= 3; ++k) {
        const float v = fl[k] + fr[4 - k];
        if (v < best4) { best4 = v; k4 = k; }
    }
    const float ci = an * cost.c_node + best4;
    const float cl = cnt <= leaf_max ? an * (cost.c_leaf + cost.c_tri * (float)cnt) : INFINITY;
    float f[5];
    if (cl <= ci) { f[1] = cl; d |= 1u; } else { f[1] = ci; }
    d |= (uint32_t)k4 << 1;
    for (int j = 2; j <= 4; ++j) {
        float bs = f[j - 1];
        int bk = 0;  // 0: keep the forest of j-1 roots
        for (int k = 1; k < j; ++k) {
            const float v = fl[k] + fr[j - k];
            if (v < bs) { bs = v; bk = k; }
        }
        f[j] = bs;
        d |= (uint32_t)bk << (3 + 2 * (j - 2));
    }
    F[n] = make_float4(f[1], f[2], f[3], f[4]);
    dec[n] = d;
}

// the roots of node n's forest of <= j roots (j >= 2 uses the split choices;
// j = 1 is n itself)
__device__ __forceinline__ int sah_expand(const int2* __restrict__ child,
                                          const uint32_t* __restrict__ dec, int n, int j, int out[4])
{
    int stn[8], stj[8], sp = 0, no = 0;
    stn[sp] = n; stj[sp] = j; ++sp;
    while (sp > 0) {
        --sp;
        int cn = stn[sp], cj = stj[sp];
        for (;;) {
            if (cn < 0 || cj == 1) { out[no++] = cn; break; }
            const int k = (int)((dec[cn] >> (3 + 2 * (cj - 2))) & 3u);
            if (k == 0) { --cj; continue; }
            const int2 c = child[cn];
            stn[sp] = c.y; stj[sp] = cj - k; ++sp;
            cn = c.x;
            cj = k;
        }
    }
    return no;
}

// One level of the top-down BVH2 -> BVH4Q collapse.  Each frontier entry
// (BVH2 node, BVH4 slot) takes up to 4 children by repeatedly opening the
// largest-area internal child; a BVH2 subtree of <= leaf_max triangles becomes
// one leaf over its contiguous range of sorted slots (LBVH subtrees are
// contiguous).  Child boxes are quantised outward to 8 bits in the node frame.
__global__ void __launch_bounds__(kBlock) k_bvh4_level(const int2* __restrict__ child,
                                                       const int2* __restrict__ range, Soa6 leaf,
                                                       const uint32_t* __restrict__ vals, Soa6 ib,
                                                       const int2* __restrict__ frontier, int nf,
                                                       int2* __restrict__ next,
                                                       uint32_t* __restrict__ counters,
                                                       Bvh4Node* __restrict__ out, int leaf_max,
                                                       int n_tris, const uint32_t* __restrict__ dec)
{
    int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nf) return;
    const int src = frontier[i].x, dst = frontier[i].y;
    int cand[4];
    int nc;
    auto count_of = [&](int c) { return c < 0 ? 1 : range[c].y - range[c].x + 1; };
    // with the SAH choices (dec): a subtree is a leaf where the DP chose one
    auto is_leaf = [&](int c) { return dec ? (c < 0 || (dec[c] & 1u)) : count_of(c) <= leaf_max; };
    if (src < 0 || (dec ? (dec[src] & 1u) != 0 : count_of(src) <= leaf_max)) {  // one leaf
        cand[0] = src;
        nc = 1;
    } else if (dec) {
        const int2 c = child[src];
        const int k4 = (int)((dec[src] >> 1) & 3u);
        nc = sah_expand(child, dec, c.x, k4, cand);
        nc += sah_expand(child, dec, c.y, 4 - k4, cand + nc);
    } else {
        cand[0] = child[src].x;
        cand[1] = child[src].y;
        nc = 2;
        while (nc < 4) {
            int best = -1;
            float best_a = -1.0f;
            for (int k = 0; k < nc; ++k) {
                int c = cand[k];
                if (c >= 0 && count_of(c) > leaf_max) {
                    float b[6];
                    node_or_leaf_box(c, leaf, vals, ib, b);
                    float a = box_area(b);
                    if (a > best_a) { best_a = a; best = k; }
                }
            }
            if (best < 0) break;
            int c = cand[best];
            cand[best] = child[c].x;
            cand[nc++] = child[c].y;
        }
    }
    float bx[4][6];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < nc; ++k) {
        node_or_leaf_box(cand[k], leaf, vals, ib, bx[k]);
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], bx[k][a]);
            hi[a] = fmaxf(hi[a], bx[k][3 + a]);
        }
    }
    uint32_t ebits = 0, mask = 0;
    uint32_t qlo[3] = {0, 0, 0}, qhi[3] = {0, 0, 0};
    double scale[3];
    for (int a = 0; a < 3; ++a) {
        double ext = (double)hi[a] - (double)lo[a];
        int e = (int)ceil(log2(fmax(ext, 1e-30) / 255.0));
        e = max(-126, min(127, e));
        scale[a] = ldexp(1.0, e);
        ebits |= ((uint32_t)e & 0xFFu) << (8 * a);  // signed byte: scale = 2^e (ldexp in the traversal)
    }
    // empty slots: inverted quantised box (lo 255 > hi 0) and a link to the null
    // leaf, so a step that does not consult the mask still finds nothing there
    const int null_leaf = (int)(0x80000000u | (uint32_t)n_tris);
    int4 links = make_int4(null_leaf, null_leaf, null_leaf, null_leaf);
    int* lk = &links.x;
    for (int k = nc; k < 4; ++k)
        for (int a = 0; a < 3; ++a) qlo[a] |= 255u << (8 * k);
    for (int k = 0; k < nc; ++k) {
        for (int a = 0; a < 3; ++a) {
            double l = floor(((double)bx[k][a] - (double)lo[a]) / scale[a]);
            double h = ceil(((double)bx[k][3 + a] - (double)lo[a]) / scale[a]);
            uint32_t ql = (uint32_t)fmin(fmax(l, 0.0), 255.0);
            uint32_t qh = (uint32_t)fmin(fmax(h, 0.0), 255.0);
            qlo[a] |= ql << (8 * k);
            qhi[a] |= qh << (8 * k);
        }
        mask |= 1u << k;
        int c = cand[k];
        if (c < 0) {  // BVH2 leaf: one triangle at sorted slot ~c
            lk[k] = (int)(0x80000000u | (uint32_t)(~c));
        } else if (is_leaf(c)) {
            lk[k] = (int)(0x80000000u | ((uint32_t)(count_of(c) - 1) << kLeafCountShift) |
                          (uint32_t)range[c].x);
        } else {
            uint32_t slot = atomicAdd(&counters[0], 1u);
            uint32_t qi = atomicAdd(&counters[1], 1u);
            next[qi] = make_int2(c, (int)slot);
            lk[k] = (int)slot;
        }
    }
    out[dst].a = f4(lo[0], lo[1], lo[2], __uint_as_float(ebits | (mask << 24)));
    out[dst].b = make_uint4(qlo[0], qhi[0], qlo[1], qhi[1]);
    out[dst].c = make_uint4(qlo[2], qhi[2], 0u, 0u);
    out[dst].d = links;
}

__global__ void __launch_bounds__(kBlock) k_tri_pre(const float* __restrict__ tris9, int32_t n,
                                                    const uint32_t* __restrict__ vals,
                                                    TriPre* __restrict__ pre)
{
    int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    int o = (int)vals[k];
    const float* t = tris9 + 9 * (int64_t)o;
    f3 v0 = mk(t[0], t[1], t[2]), v1 = mk(t[3], t[4], t[5]), v2 = mk(t[6], t[7], t[8]);
    f3 e1 = v1 - v0, e2 = v2 - v0;  // maths.cpp:341-342, same roundings
    pre[k].a = f4(v0.x, v0.y, v0.z, e1.x);
    pre[k].b = f4(e1.y, e1.z, e2.x, e2.y);
    pre[k].c = f4(e2.z, __int_as_float(2 * o), 0.0f, 0.0f);  // doubled: TravState::best's tie bit is bit 0
}

inline int blocks_for(int64_t n, int b) { return (int)((n + b - 1) / b); }

// layout=soa: the AoS records split into planes (tmpt_internal.h SoaScene)
__global__ void __launch_bounds__(kBlock) k_soa_planes(const Bvh4Node* __restrict__ nodes, int32_t n4,
                                                       const TriPre* __restrict__ pre, int32_t n1, uint4* na,
                                                       uint4* nb, uint2* nc, int4* nd, float4* ta, float4* tb,
                                                       float2* tc)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k < n4) {
        const Bvh4Node v = nodes[k];
        na[k] = make_uint4(__float_as_uint(v.a.x), __float_as_uint(v.a.y), __float_as_uint(v.a.z),
                           __float_as_uint(v.a.w));
        nb[k] = v.b;
        nc[k] = make_uint2(v.c.x, v.c.y);
        nd[k] = v.d;
    }
    if (k < n1) {
        const TriPre t = pre[k];
        ta[k] = t.a;
        tb[k] = t.b;
        tc[k] = make_float2(t.c.x, t.c.y);
    }
}

// The octree's flat triangles (tmpt_internal.h OctGrid): bit 0 of the doubled
// index in the leaf-ordered records (and the SoA plane) set where flat[index],
// cleared elsewhere, so an accepted flat triangle flags its query.
__global__ void __launch_bounds__(kBlock) k_mark_flat(TriPre* __restrict__ pre, float2* __restrict__ tc, int32_t n,
                                                      const uint8_t* __restrict__ flat)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const int w = __float_as_int(pre[k].c.y);
    const int v = (w & ~1) | (flat ? (int)flat[w >> 1] : 0);
    pre[k].c.y = __int_as_float(v);
    if (tc) tc[k].y = __int_as_float(v);
}

}  // namespace

int mark_flat_triangles(Scene& s, const std::vector<uint8_t>& flat)
{
    if (s.n <= 0) return 0;
    uint8_t* d = nullptr;
    const bool any = std::find(flat.begin(), flat.end(), (uint8_t)1) != flat.end();
    if (any) {
        TMPT_HIP(hipMalloc(&d, (size_t)s.n));
        if (hipMemcpy(d, flat.data(), (size_t)s.n, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            set_error("mark_flat_triangles: upload failed");
            return -1;
        }
    }
    k_mark_flat<<<blocks_for(s.n, kBlock), kBlock, 0, s.stream>>>(s.tri_pre, const_cast<float2*>(s.soa.tc), s.n, d);
    const hipError_t e = hipGetLastError();
    const hipError_t e2 = hipStreamSynchronize(s.stream);
    if (d) (void)hipFree(d);
    TMPT_HIP(e);
    TMPT_HIP(e2);
    return 0;
}

int build_soa(Scene& s)
{
    const size_t n4 = (size_t)std::max(s.n_nodes4, 1), n1 = (size_t)s.n + 1;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_nb = al(16 * n4), o_nc = o_nb + al(16 * n4), o_nd = o_nc + al(8 * n4), o_ta = o_nd + al(16 * n4),
                 o_tb = o_ta + al(16 * n1), o_tc = o_tb + al(16 * n1), total = o_tc + al(8 * n1);
    if (s.soa_buf) (void)hipFree(s.soa_buf);
    s.soa_buf = nullptr;
    s.soa = SoaScene();
    TMPT_HIP(hipMalloc(&s.soa_buf, total));
    char* b = static_cast<char*>(s.soa_buf);
    uint4* na = reinterpret_cast<uint4*>(b);
    uint4* nb = reinterpret_cast<uint4*>(b + o_nb);
    uint2* nc = reinterpret_cast<uint2*>(b + o_nc);
    int4* nd = reinterpret_cast<int4*>(b + o_nd);
    float4* ta = reinterpret_cast<float4*>(b + o_ta);
    float4* tb = reinterpret_cast<float4*>(b + o_tb);
    float2* tc = reinterpret_cast<float2*>(b + o_tc);
    k_soa_planes<<<blocks_for((int64_t)std::max(n4, n1), kBlock), kBlock, 0, s.stream>>>(
        s.nodes4, s.n_nodes4, s.tri_pre, (int32_t)n1, na, nb, nc, nd, ta, tb, tc);
    TMPT_HIP(hipGetLastError());
    TMPT_HIP(hipStreamSynchronize(s.stream));
    s.soa = SoaScene{na, nb, nc, nd, ta, tb, tc};
    return 0;
}

// LSD radix sort of (key, value) pairs by the low `bits` bits of the key
// (stable; 8 bits per pass, ping-pong).  hist: 256 * ceil(n / kSortTile)
// words.  Returns the buffer pair holding the result (0: keys/vals, 1: tmp).
int radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* tkeys, uint32_t* tvals, int32_t n,
                     int bits, uint32_t* hist, hipStream_t st)
{
    const int nb = std::max(1, blocks_for(n, kSortTile));
    uint32_t *ki = keys, *vi = vals, *ko = tkeys, *vo = tvals;
    int which = 0;
    for (int shift = 0; shift < bits; shift += 8) {
        k_sort_hist<<<nb, kBlock, 0, st>>>(ki, n, shift, nb, hist);
        k_scan_1block<<<1, 1024, 0, st>>>(hist, 256 * nb);
        k_sort_scatter<<<nb, kBlock, 0, st>>>(ki, vi, ko, vo, n, shift, nb, hist);
        std::swap(ki, ko);
        std::swap(vi, vo);
        which ^= 1;
    }
    return which;
}

size_t radix_sort_hist_words(int32_t n) { return 256 * (size_t)std::max(1, blocks_for(n, kSortTile)); }

int build_lbvh(Scene& s, const float* d_tris9)
{
    const int32_t n = s.n;
    hipStream_t st = s.stream;
    auto t0 = std::chrono::steady_clock::now();
    const int32_t m = n >= 2 ? n - 1 : 1;  // internal nodes
    s.n_nodes = m;
    TMPT_HIP(hipMalloc(&s.nodes4, sizeof(Bvh4Node) * (size_t)m));
    // one extra slot: the null triangle (all zero: det = 0, never accepted) that
    // empty BVH4 child slots link to
    TMPT_HIP(hipMalloc(&s.tri_pre, sizeof(TriPre) * ((size_t)n + 1)));
    TMPT_HIP(hipMemsetAsync(s.tri_pre + n, 0, sizeof(TriPre), st));
    TMPT_HIP(hipMalloc(&s.tri_orig, sizeof(TriOrig) * (size_t)std::max(n, 1)));
    if (n == 0) {
        TMPT_HIP(hipMemsetAsync(s.nodes4, 0, sizeof(Bvh4Node), st));
        s.max_depth = 0;
        return 0;
    }
    // scratch
    const int nb_sort = blocks_for(n, kSortTile);
    size_t nn = (size_t)n;
    std::vector<void*> tmp;
    auto alloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        tmp.push_back(p);
        return p;
    };
    auto free_all = [&]() {
        for (void* p : tmp) (void)hipFree(p);
        tmp.clear();
    };
    float* leafbuf = (float*)alloc(6 * nn * sizeof(float));
    float* ibbuf = (float*)alloc(6 * (size_t)m * sizeof(float));
    float* cent = (float*)alloc(3 * nn * sizeof(float));
    uint32_t* cb = (uint32_t*)alloc(6 * sizeof(uint32_t));
    uint32_t* k0 = (uint32_t*)alloc(nn * 4);
    uint32_t* v0 = (uint32_t*)alloc(nn * 4);
    uint32_t* k1 = (uint32_t*)alloc(nn * 4);
    uint32_t* v1 = (uint32_t*)alloc(nn * 4);
    uint32_t* hist = (uint32_t*)alloc((size_t)256 * nb_sort * 4);
    int2* child = (int2*)alloc((size_t)m * sizeof(int2));
    int2* range = (int2*)alloc((size_t)m * sizeof(int2));
    int2* fr0 = (int2*)alloc((size_t)m * sizeof(int2));
    int2* fr1 = (int2*)alloc((size_t)m * sizeof(int2));
    uint32_t* c4 = (uint32_t*)alloc(2 * sizeof(uint32_t));
    int32_t* pint = (int32_t*)alloc((size_t)m * 4);
    int32_t* pleaf = (int32_t*)alloc(nn * 4);
    int32_t* depth = (int32_t*)alloc((size_t)m * 4);
    int32_t* maxd = (int32_t*)alloc(4);
    if (!leafbuf || !ibbuf || !cent || !cb || !k0 || !v0 || !k1 || !v1 || !hist || !child ||
        !range || !fr0 || !fr1 || !c4 || !pint || !pleaf || !depth || !maxd) {
        free_all();
        set_error("build_lbvh: out of device memory");
        return -1;
    }
    Soa6 leaf{leafbuf, leafbuf + nn, leafbuf + 2 * nn, leafbuf + 3 * nn, leafbuf + 4 * nn,
              leafbuf + 5 * nn};
    size_t mm = (size_t)m;
    Soa6 ib{ibbuf, ibbuf + mm, ibbuf + 2 * mm, ibbuf + 3 * mm, ibbuf + 4 * mm, ibbuf + 5 * mm};
    uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    int rc = 0;
    do {
        if (hipMemcpyAsync(cb, init, sizeof(init), hipMemcpyHostToDevice, st) != hipSuccess) { rc = -1; break; }
        if (hipMemsetAsync(maxd, 0, 4, st) != hipSuccess) { rc = -1; break; }
        k_tri_prep<<<blocks_for(n, kBlock), kBlock, 0, st>>>(d_tris9, n, s.tri_orig, leaf, cent, cb);
        k_morton<<<blocks_for(n, kBlock), kBlock, 0, st>>>(cent, n, cb, k0, v0);
        uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
        for (int pass = 0; pass < 4; ++pass) {
            k_sort_hist<<<nb_sort, kBlock, 0, st>>>(ki, n, 8 * pass, nb_sort, hist);
            k_scan_1block<<<1, 1024, 0, st>>>(hist, 256 * nb_sort);
            k_sort_scatter<<<nb_sort, kBlock, 0, st>>>(ki, vi, ko, vo, n, 8 * pass, nb_sort, hist);
            std::swap(ki, ko);
            std::swap(vi, vo);
        }
        // sorted (ki, vi)
        const bool ploc = s.opt.builder == 0 && n > 1;
        if (n == 1) {
            s.max_depth = 0;
        } else {
            k_karras<<<blocks_for(m, kBlock), kBlock, 0, st>>>(ki, n, child, range, pint, pleaf);
        k_depth<<<blocks_for(m, kBlock), kBlock, 0, st>>>(pint, m, depth, maxd);
        int32_t hmax = 0;
        if (hipMemcpyAsync(&hmax, maxd, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) { rc = -1; break; }
        s.max_depth = hmax;
        if (hmax + 2 > kStackTotal) {
            set_error("build_lbvh: tree depth " + std::to_string(hmax) + " exceeds the traversal stack");
            rc = -2;
            break;
        }
            for (int L = hmax; L >= 0; --L)
                k_refit_level<<<blocks_for(m, kBlock), kBlock, 0, st>>>(child, depth, m, L, leaf, vi, ib);
        }
        // binary tree the BVH4Q is collapsed from: the LBVH, or a PLOC tree
        const int2* tchild = child;
        const int2* trange = range;
        Soa6 tib = ib;
        const uint32_t* tvals = vi;
        int troot = n == 1 ? ~0 : 0;
        if (ploc) {
            const int r = s.opt.ploc_radius;  // search radius; node visits vs r measured in DESIGN.md
            int32_t* cidA = (int32_t*)alloc(nn * 4);
            int32_t* cidB = (int32_t*)alloc(nn * 4);
            float* cbAb = (float*)alloc(6 * nn * 4);
            float* cbBb = (float*)alloc(6 * nn * 4);
            int32_t* nnb = (int32_t*)alloc(nn * 4);
            uint32_t* valid = (uint32_t*)alloc(nn * 4);
            uint32_t* pos = (uint32_t*)alloc(nn * 4);
            int2* pchild = (int2*)alloc(mm * sizeof(int2));
            int2* prange = (int2*)alloc(mm * sizeof(int2));
            float* pibb = (float*)alloc(6 * mm * 4);
            int32_t* psize = (int32_t*)alloc(mm * 4);
            int32_t* piter = (int32_t*)alloc(mm * 4);
            int32_t* poff = (int32_t*)alloc(mm * 4);
            uint32_t* new_slot = (uint32_t*)alloc(nn * 4);
            uint32_t* pvals = (uint32_t*)alloc(nn * 4);
            uint32_t* pcounter = (uint32_t*)alloc(4);
            if (!cidA || !cidB || !cbAb || !cbBb || !nnb || !valid || !pos || !pchild || !prange || !pibb ||
                !psize || !piter || !poff || !new_slot || !pvals || !pcounter) {
                set_error("build: out of device memory (PLOC)");
                rc = -1;
                break;
            }
            auto soa = [](float* b, size_t k) { return Soa6{b, b + k, b + 2 * k, b + 3 * k, b + 4 * k, b + 5 * k}; };
            Soa6 cbA = soa(cbAb, nn), cbB = soa(cbBb, nn), pib = soa(pibb, mm);
            if (hipMemsetAsync(pcounter, 0, 4, st) != hipSuccess || hipMemsetAsync(poff, 0, mm * 4, st) != hipSuccess) {
                rc = -1;
                break;
            }
            k_ploc_init<<<blocks_for(n, kBlock), kBlock, 0, st>>>(n, leaf, vi, cidA, cbA);
            int N = n, it = 0;
            while (N > 1) {
                k_ploc_nn<<<blocks_for(N, kBlock), kBlock, 0, st>>>(N, r, cbA, nnb);
                k_ploc_merge<<<blocks_for(N, kBlock), kBlock, 0, st>>>(N, nnb, cidA, cbA, valid, pchild, pib,
                                                                       psize, piter, it, pcounter);
                uint32_t tail[2];
                if (hipMemcpyAsync(pos, valid, (size_t)N * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) { rc = -1; break; }
                k_scan_1block<<<1, 1024, 0, st>>>(pos, N);
                if (hipMemcpyAsync(&tail[0], pos + N - 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipMemcpyAsync(&tail[1], valid + N - 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess) { rc = -1; break; }
                k_ploc_compact<<<blocks_for(N, kBlock), kBlock, 0, st>>>(N, valid, pos, cidA, cbA, cidB, cbB);
                std::swap(cidA, cidB);
                std::swap(cbA, cbB);
                int next = (int)(tail[0] + tail[1]);
                if (next >= N) { set_error("build: PLOC made no progress"); rc = -2; break; }
                N = next;
                ++it;
            }
            if (rc) break;
            for (int k = it - 1; k >= 0; --k)
                k_ploc_offsets<<<blocks_for(m, kBlock), kBlock, 0, st>>>(m, k, piter, pchild, psize, poff, new_slot);
            k_ploc_relabel<<<blocks_for(m, kBlock), kBlock, 0, st>>>(m, pchild, poff, psize, prange, new_slot);
            k_ploc_vals<<<blocks_for(n, kBlock), kBlock, 0, st>>>(n, new_slot, vi, pvals);
            tchild = pchild;
            trange = prange;
            tib = pib;
            tvals = pvals;
            troot = m - 1;  // the last merge creates the root
            s.ploc_iters = it;
        }
        k_tri_pre<<<blocks_for(n, kBlock), kBlock, 0, st>>>(d_tris9, n, tvals, s.tri_pre);
        // binary tree -> BVH4Q, top-down, one launch per level
        const int leaf_max = s.opt.leaf_max;
        s.leaf_max = leaf_max;
        // collapse=1: SAH-optimal collapse (fewer, fuller nodes: 13.2k vs 16.7k
        // on the sponza stand-in, but measured ~2% slower there); default greedy
        // largest-area opening
        const bool sah = s.opt.collapse == 1 && n >= 2;
        uint32_t* dec = nullptr;
        if (sah) {
            const SahCost cost{1.0f, s.opt.sah_c_leaf, s.opt.sah_c_tri};
            int32_t* ord = (int32_t*)alloc((size_t)m * 4);
            float4* Fc = (float4*)alloc((size_t)m * sizeof(float4));
            dec = (uint32_t*)alloc((size_t)m * 4);
            if (!ord || !Fc || !dec) { set_error("build: out of device memory"); rc = -1; break; }
            std::vector<int> off = {0, 1};
            uint32_t zero = 0, cnt = 0;
            if (hipMemcpyAsync(ord, &troot, 4, hipMemcpyHostToDevice, st) != hipSuccess) { rc = -1; break; }
            while (off.back() > off[off.size() - 2]) {  // BFS: one level of internal nodes per launch
                const int b0 = off[off.size() - 2], b1 = off.back();
                if (hipMemcpyAsync(c4, &zero, 4, hipMemcpyHostToDevice, st) != hipSuccess) { rc = -1; break; }
                k_bfs_level<<<blocks_for(b1 - b0, kBlock), kBlock, 0, st>>>(tchild, ord + b0, b1 - b0, ord + b1, c4);
                if (hipMemcpyAsync(&cnt, c4, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess) { rc = -1; break; }
                off.push_back(b1 + (int)cnt);
            }
            if (rc) break;
            for (int L = (int)off.size() - 3; L >= 0; --L)  // deepest level first
                k_sah_level<<<blocks_for(off[L + 1] - off[L], kBlock), kBlock, 0, st>>>(
                    tchild, trange, leaf, tvals, tib, ord + off[L], off[L + 1] - off[L], Fc, dec, leaf_max, cost);
        }
        int2 root = make_int2(troot, 0);
        uint32_t hc[2] = {1u, 0u};
        if (hipMemcpyAsync(fr0, &root, sizeof(root), hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(c4, hc, sizeof(hc), hipMemcpyHostToDevice, st) != hipSuccess) { rc = -1; break; }
        int nf = 1, levels = 0;
        int2 *fa = fr0, *fb = fr1;
        while (nf > 0) {
            k_bvh4_level<<<blocks_for(nf, kBlock), kBlock, 0, st>>>(tchild, trange, leaf, tvals, tib, fa, nf,
                                                                    fb, c4, s.nodes4, leaf_max, n, dec);
            ++levels;
            if (hipMemcpyAsync(hc, c4, sizeof(hc), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) { rc = -1; break; }
            nf = (int)hc[1];
            hc[1] = 0;
            if (hipMemcpyAsync(c4 + 1, &hc[1], 4, hipMemcpyHostToDevice, st) != hipSuccess) { rc = -1; break; }
            std::swap(fa, fb);
        }
        if (rc) break;
        s.n_nodes4 = (int32_t)hc[0];
        s.depth4 = levels;
        if (3 * levels + 1 > kStackTotal) {
            set_error("build_lbvh: BVH4 depth " + std::to_string(levels) + " exceeds the traversal stack");
            rc = -2;
            break;
        }
    } while (0);
    hipError_t e = hipGetLastError();
    hipError_t e2 = hipStreamSynchronize(st);
    free_all();
    if (rc == -1 || e != hipSuccess || e2 != hipSuccess) {
        set_error(std::string("build_lbvh: ") + hipGetErrorString(e != hipSuccess ? e : e2));
        return -1;
    }
    if (rc) return rc;
    if (s.opt.layout == 1 && build_soa(s)) return -1;
    s.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

}  // namespace tmpt
