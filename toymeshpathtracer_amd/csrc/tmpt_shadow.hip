// tmpt_shadow.hip -- light-space grid for the shadow query (the HitScene call
// of Scatter, main.cpp:57-60).
//
// The light is directional (kLightDir, main.cpp:36): every shadow ray of a
// frame is parallel to L, so a shadow ray is a point in the plane orthogonal
// to L plus a half-line along L.  The grid covers that plane with R x R cells;
// each cell lists, sorted by how far up L they reach (t_max = max_v dot(v, L)),
// the triangles whose projection overlaps the cell (triangle-vs-rectangle
// separating-axis test in double precision, rectangles padded so float
// rounding of the ray's projection and Moller-Trumbore's acceptance just
// outside an edge stay inside the padding).  A shadow query maps its origin to
// one cell, skips (binary search) the triangles that end below the origin, and
// runs the bit-exact Moller-Trumbore test (maths.cpp:339-380) on the rest until
// one accepts.  The query only needs whether SOME triangle is hit in
// [kMinT, kMaxT] (main.cpp:59-60), and every triangle that could be hit is in
// the list, so the answer is the linear scan's -- the grid only replaces the
// BVH as the culling structure, as the BVH replaced the octree.
//
// Build (untimed, like the BVH): per triangle its bbox rows -> one work item
// per (triangle, row) -> overlapping cells counted, scanned, written as
// (cell, t_max, slot) -> two stable radix sorts (t_max, then cell) -> cell
// starts.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "tmpt_internal.h"

namespace tmpt {

void set_error(const std::string& msg);

namespace {

constexpr int kB = 256;
inline int nblk(int64_t n) { return (int)std::max<int64_t>(1, (n + kB - 1) / kB); }

struct Frame {  // light-space projection, double precision for the build
    double U[3], V[3], L[3];
    double u0, v0, cu, cv, eps;
    int R;
};

__device__ __forceinline__ double dotd(const double a[3], double x, double y, double z)
{
    return a[0] * x + a[1] * y + a[2] * z;
}

__device__ __forceinline__ void tri_vertices(const TriPre* __restrict__ pre, const TriOrig* __restrict__ orig,
                                             int slot, double v[3][3])
{
    const int id = __float_as_int(pre[slot].c.y);
    const TriOrig t = orig[id];
    v[0][0] = t.a.x; v[0][1] = t.a.y; v[0][2] = t.a.z;
    v[1][0] = t.a.w; v[1][1] = t.b.x; v[1][2] = t.b.y;
    v[2][0] = t.b.z; v[2][1] = t.b.w; v[2][2] = t.c.x;
}

struct TriRows {
    int iu0, iu1, iv0, iv1;
};

__device__ __forceinline__ TriRows tri_cells(const Frame& f, const double p[3][2])
{
    double lu = fmin(p[0][0], fmin(p[1][0], p[2][0])) - f.eps, hu = fmax(p[0][0], fmax(p[1][0], p[2][0])) + f.eps;
    double lv = fmin(p[0][1], fmin(p[1][1], p[2][1])) - f.eps, hv = fmax(p[0][1], fmax(p[1][1], p[2][1])) + f.eps;
    TriRows r;
    r.iu0 = (int)fmax(0.0, floor((lu - f.u0) / f.cu));
    r.iu1 = (int)fmin((double)(f.R - 1), floor((hu - f.u0) / f.cu));
    r.iv0 = (int)fmax(0.0, floor((lv - f.v0) / f.cv));
    r.iv1 = (int)fmin((double)(f.R - 1), floor((hv - f.v0) / f.cv));
    return r;
}

__device__ __forceinline__ void project(const Frame& f, const double v[3][3], double p[3][2])
{
    for (int k = 0; k < 3; ++k) {
        p[k][0] = dotd(f.U, v[k][0], v[k][1], v[k][2]);
        p[k][1] = dotd(f.V, v[k][0], v[k][1], v[k][2]);
    }
}

// Does the padded cell (iu, iv) overlap the projected triangle?  Separating
// axes: the cell's own axes are the bbox range already; the triangle's three
// edge normals remain.  Degenerate projections (a triangle seen edge-on) keep
// the bbox test only, which is conservative.
__device__ __forceinline__ bool cell_overlaps(const Frame& f, const double p[3][2], int iu, int iv)
{
    const double x0 = f.u0 + iu * f.cu - f.eps, x1 = f.u0 + (iu + 1) * f.cu + f.eps;
    const double y0 = f.v0 + iv * f.cv - f.eps, y1 = f.v0 + (iv + 1) * f.cv + f.eps;
    const double area = (p[1][0] - p[0][0]) * (p[2][1] - p[0][1]) - (p[1][1] - p[0][1]) * (p[2][0] - p[0][0]);
    if (area == 0.0) return true;
    const double s = area > 0.0 ? 1.0 : -1.0;
    for (int e = 0; e < 3; ++e) {
        const double* a = p[e];
        const double* b = p[(e + 1) % 3];
        const double ex = b[0] - a[0], ey = b[1] - a[1];
        // inside side: s * cross(edge, P - a) >= 0; is any corner inside (within tolerance)?
        const double c00 = s * (ex * (y0 - a[1]) - ey * (x0 - a[0]));
        const double c10 = s * (ex * (y0 - a[1]) - ey * (x1 - a[0]));
        const double c01 = s * (ex * (y1 - a[1]) - ey * (x0 - a[0]));
        const double c11 = s * (ex * (y1 - a[1]) - ey * (x1 - a[0]));
        if (fmax(fmax(c00, c10), fmax(c01, c11)) < 0.0) return false;
    }
    return true;
}

__global__ void __launch_bounds__(kB) k_sg_rows(const TriPre* __restrict__ pre, const TriOrig* __restrict__ orig,
                                                int32_t n, Frame f, uint32_t* __restrict__ rows,
                                                float* __restrict__ tmax)
{
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    double v[3][3], p[3][2];
    tri_vertices(pre, orig, k, v);
    project(f, v, p);
    const TriRows r = tri_cells(f, p);
    rows[k] = r.iu1 >= r.iu0 && r.iv1 >= r.iv0 ? (uint32_t)(r.iv1 - r.iv0 + 1) : 0u;
    double t = fmax(dotd(f.L, v[0][0], v[0][1], v[0][2]),
                    fmax(dotd(f.L, v[1][0], v[1][1], v[1][2]), dotd(f.L, v[2][0], v[2][1], v[2][2])));
    t += 1e-6 * (fabs(t) + 1.0);  // rounded up: the stored reach never undershoots
    tmax[k] = (float)t;
}

__global__ void __launch_bounds__(kB) k_sg_items(const TriPre* __restrict__ pre, const TriOrig* __restrict__ orig,
                                                 int32_t n, Frame f, const uint32_t* __restrict__ row_off,
                                                 int2* __restrict__ items)
{
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    double v[3][3], p[3][2];
    tri_vertices(pre, orig, k, v);
    project(f, v, p);
    const TriRows r = tri_cells(f, p);
    if (r.iu1 < r.iu0 || r.iv1 < r.iv0) return;
    uint32_t o = row_off[k];
    for (int iv = r.iv0; iv <= r.iv1; ++iv) items[o++] = make_int2(k, iv);
}

// one (triangle, row) item: count (WRITE = 0) or emit (WRITE = 1) its cells
template <int WRITE>
__global__ void __launch_bounds__(kB) k_sg_cells(const TriPre* __restrict__ pre, const TriOrig* __restrict__ orig,
                                                 const int2* __restrict__ items, int64_t nitems, Frame f,
                                                 uint32_t* __restrict__ count_or_off,
                                                 const float* __restrict__ tmax, uint32_t* __restrict__ ecell,
                                                 uint32_t* __restrict__ ekey, uint32_t* __restrict__ eslot)
{
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= nitems) return;
    const int k = items[i].x, iv = items[i].y;
    double v[3][3], p[3][2];
    tri_vertices(pre, orig, k, v);
    project(f, v, p);
    const TriRows r = tri_cells(f, p);
    uint32_t c = 0, o = WRITE ? count_or_off[i] : 0u;
    // sortable key of t_max: flip so that unsigned order = float order
    const uint32_t tb = __float_as_uint(tmax[k]);
    const uint32_t key = (tb & 0x80000000u) ? ~tb : (tb | 0x80000000u);
    for (int iu = r.iu0; iu <= r.iu1; ++iu) {
        if (!cell_overlaps(f, p, iu, iv)) continue;
        if (WRITE) {
            ecell[o + c] = (uint32_t)(iv * f.R + iu);
            ekey[o + c] = key;
            eslot[o + c] = (uint32_t)k;
        }
        ++c;
    }
    if (!WRITE) count_or_off[i] = c;
}

__global__ void __launch_bounds__(kB) k_sg_gather(const uint32_t* __restrict__ perm, int64_t ne,
                                                  const uint32_t* __restrict__ src, uint32_t* __restrict__ dst)
{
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < ne) dst[i] = src[perm[i]];
}

__global__ void __launch_bounds__(kB) k_sg_cellrec(const uint32_t* __restrict__ start, uint32_t ncells,
                                                   uint32_t base, uint2* __restrict__ cell)
{
    const int64_t c = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (c >= ncells) return;
    cell[c] = make_uint2(base + start[c], start[c + 1] - start[c]);
}

__global__ void __launch_bounds__(kB) k_sg_copy_tris(const TriPre* __restrict__ src, const uint32_t* __restrict__ slot,
                                                     int64_t ne, TriPre* __restrict__ dst)
{
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < ne) dst[i] = src[slot[i]];
}

__global__ void __launch_bounds__(kB) k_sg_final(const uint32_t* __restrict__ perm, int64_t ne,
                                                 const uint32_t* __restrict__ eslot, const float* __restrict__ tmax,
                                                 uint32_t* __restrict__ out_slot, float* __restrict__ out_tmax)
{
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= ne) return;
    const uint32_t s = eslot[perm[i]];
    out_slot[i] = s;
    out_tmax[i] = tmax[s];
}

// start[c] = first entry of cell c (entries sorted by cell); start[R*R] = ne
__global__ void __launch_bounds__(kB) k_sg_starts(const uint32_t* __restrict__ cell_sorted, int64_t ne,
                                                  uint32_t ncells, uint32_t* __restrict__ start)
{
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i > ne) return;
    const uint32_t c = i < ne ? cell_sorted[i] : ncells;
    const uint32_t p = i > 0 ? cell_sorted[i - 1] + 1u : 0u;
    for (uint32_t cc = p; cc <= c && cc <= ncells; ++cc) start[cc] = (uint32_t)i;
}

// exclusive scan on the host for modest arrays (per-triangle rows, per-item counts)
int scan_on_host(uint32_t* d, int64_t n, uint64_t* total, hipStream_t st)
{
    std::vector<uint32_t> h((size_t)n);
    if (n && hipMemcpyAsync(h.data(), d, (size_t)n * 4, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
    if (hipStreamSynchronize(st) != hipSuccess) return -1;
    uint64_t run = 0;
    for (auto& x : h) {
        uint64_t v = x;
        if (run > 0xFFFFFFFFull) return -2;
        x = (uint32_t)run;
        run += v;
    }
    if (run > 0xFFFFFFFFull) return -2;
    *total = run;
    if (n && hipMemcpyAsync(d, h.data(), (size_t)n * 4, hipMemcpyHostToDevice, st) != hipSuccess) return -1;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

}  // namespace

void free_shadow_grid(Scene& s)
{
    if (s.sgrid.start) (void)hipFree(s.sgrid.start);
    if (s.sgrid.tmax) (void)hipFree(s.sgrid.tmax);
    if (s.sgrid.slot) (void)hipFree(s.sgrid.slot);
    if (s.sgrid.cell) (void)hipFree(s.sgrid.cell);
    s.sgrid = ShadowGrid{};
}

// Build the grid for the scene's (device) triangles; host_tris = the same
// n x 9 floats on the host (for the projected bounds).  R = cells per side
// (TMPT_SHADOW_GRID, 0 = no grid).
int build_shadow_grid(Scene& s, const float* host_tris)
{
    free_shadow_grid(s);
    // Off by default: measured slower than the BVH any-hit query on the bench
    // frame (393 vs 263 ms: 3.8 triangle tests per shadow ray against 6 node
    // + 1.6 triangle steps, from a 127 MB copy array instead of the L2-resident
    // tri_pre, behind one more dependent load in the shading round).
    // TMPT_SHADOW_GRID=<cells per side> builds it (A/B, tests).
    int R = 0;
    if (const char* e = getenv("TMPT_SHADOW_GRID")) R = std::max(0, std::min(4096, atoi(e)));
    const int32_t n = s.n;
    if (R == 0 || n == 0) return 0;
    hipStream_t st = s.stream;
    // frame: L = the float light direction the shadow rays use, U, V orthonormal
    const f3 lf = light_dir();
    Frame f;
    f.L[0] = lf.x; f.L[1] = lf.y; f.L[2] = lf.z;
    {
        const double a[3] = {0.0, 0.0, 1.0};
        double u[3] = {f.L[1] * a[2] - f.L[2] * a[1], f.L[2] * a[0] - f.L[0] * a[2], f.L[0] * a[1] - f.L[1] * a[0]};
        double un = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
        for (int k = 0; k < 3; ++k) f.U[k] = u[k] / un;
        f.V[0] = f.L[1] * f.U[2] - f.L[2] * f.U[1];
        f.V[1] = f.L[2] * f.U[0] - f.L[0] * f.U[2];
        f.V[2] = f.L[0] * f.U[1] - f.L[1] * f.U[0];
    }
    double lu = INFINITY, hu = -INFINITY, lv = INFINITY, hv = -INFINITY, amax = 0.0;
    for (int64_t i = 0; i < (int64_t)n * 3; ++i) {
        const float* p = host_tris + 3 * i;
        const double u = f.U[0] * p[0] + f.U[1] * p[1] + f.U[2] * p[2];
        const double v = f.V[0] * p[0] + f.V[1] * p[1] + f.V[2] * p[2];
        lu = std::min(lu, u); hu = std::max(hu, u);
        lv = std::min(lv, v); hv = std::max(hv, v);
        amax = std::max({amax, std::fabs((double)p[0]), std::fabs((double)p[1]), std::fabs((double)p[2])});
    }
    if (!(hu >= lu) || !(hv >= lv) || !std::isfinite(hu - lu) || !std::isfinite(hv - lv)) return 0;  // no grid
    // padding: float rounding of a ray's projection (a few ulp of |p|) and MT's
    // acceptance just outside an edge, both far below 1e-5 relative
    const double ext = std::max(hu - lu, hv - lv);
    f.eps = 1e-5 * (amax + ext) + 1e-12;
    f.R = R;
    f.u0 = lu - 2 * f.eps;
    f.v0 = lv - 2 * f.eps;
    f.cu = std::max((hu - lu + 4 * f.eps) / R, 1e-30);
    f.cv = std::max((hv - lv + 4 * f.eps) / R, 1e-30);

    std::vector<void*> tmp;
    auto alloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 4)) != hipSuccess) return nullptr;
        tmp.push_back(p);
        return p;
    };
    auto free_tmp = [&]() {
        for (void* p : tmp) (void)hipFree(p);
        tmp.clear();
    };
    int rc = 0;
    do {
        uint32_t* rows = (uint32_t*)alloc((size_t)n * 4);
        float* tmaxv = (float*)alloc((size_t)n * 4);
        if (!rows || !tmaxv) { rc = -1; break; }
        k_sg_rows<<<nblk(n), kB, 0, st>>>(s.tri_pre, s.tri_orig, n, f, rows, tmaxv);
        uint64_t nitems = 0;
        if ((rc = scan_on_host(rows, n, &nitems, st))) break;
        int2* items = (int2*)alloc(nitems * sizeof(int2));
        uint32_t* ioff = (uint32_t*)alloc(nitems * 4);
        if (!items || !ioff) { rc = -1; break; }
        k_sg_items<<<nblk(n), kB, 0, st>>>(s.tri_pre, s.tri_orig, n, f, rows, items);
        k_sg_cells<0><<<nblk((int64_t)nitems), kB, 0, st>>>(s.tri_pre, s.tri_orig, items, (int64_t)nitems, f,
                                                            ioff, tmaxv, nullptr, nullptr, nullptr);
        uint64_t ne = 0;
        if ((rc = scan_on_host(ioff, (int64_t)nitems, &ne, st))) break;
        if (ne >= (1ull << 31)) { rc = -2; break; }
        uint32_t* ecell = (uint32_t*)alloc(ne * 4);
        uint32_t* ekey = (uint32_t*)alloc(ne * 4);
        uint32_t* eslot = (uint32_t*)alloc(ne * 4);
        uint32_t* idx = (uint32_t*)alloc(ne * 4);
        uint32_t* k2 = (uint32_t*)alloc(ne * 4);
        uint32_t* i2 = (uint32_t*)alloc(ne * 4);
        uint32_t* hist = (uint32_t*)alloc(radix_sort_hist_words((int32_t)ne) * 4);
        if (!ecell || !ekey || !eslot || !idx || !k2 || !i2 || !hist) { rc = -1; break; }
        k_sg_cells<1><<<nblk((int64_t)nitems), kB, 0, st>>>(s.tri_pre, s.tri_orig, items, (int64_t)nitems, f,
                                                            ioff, tmaxv, ecell, ekey, eslot);
        // entry order: by t_max, then (stable) by cell
        std::vector<uint32_t> iota(ne);
        for (uint64_t i = 0; i < ne; ++i) iota[i] = (uint32_t)i;
        if (hipMemcpyAsync(idx, iota.data(), ne * 4, hipMemcpyHostToDevice, st) != hipSuccess) { rc = -1; break; }
        int w = radix_sort_pairs(ekey, idx, k2, i2, (int32_t)ne, 32, hist, st);
        uint32_t* perm = w ? i2 : idx;
        uint32_t* spare = w ? idx : i2;
        uint32_t* ckey = w ? ekey : k2;  // free key buffer for the cell keys
        uint32_t* ckey2 = w ? k2 : ekey;
        k_sg_gather<<<nblk((int64_t)ne), kB, 0, st>>>(perm, (int64_t)ne, ecell, ckey);
        int bits = 1;
        while ((1u << bits) < (uint32_t)R * (uint32_t)R) ++bits;
        bits = (bits + 7) / 8 * 8;
        int w2 = radix_sort_pairs(ckey, perm, ckey2, spare, (int32_t)ne, bits, hist, st);
        uint32_t* fperm = w2 ? spare : perm;
        uint32_t* fcell = w2 ? ckey2 : ckey;
        const uint32_t ncells = (uint32_t)R * (uint32_t)R;
        ShadowGrid g{};
        if (hipMalloc(&g.start, ((size_t)ncells + 1) * 4) != hipSuccess ||
            hipMalloc(&g.tmax, std::max<size_t>(ne, 1) * 4) != hipSuccess ||
            hipMalloc(&g.slot, std::max<size_t>(ne, 1) * 4) != hipSuccess) {
            if (g.start) (void)hipFree(g.start);
            if (g.tmax) (void)hipFree(g.tmax);
            if (g.slot) (void)hipFree(g.slot);
            rc = -1;
            break;
        }
        k_sg_final<<<nblk((int64_t)ne), kB, 0, st>>>(fperm, (int64_t)ne, eslot, tmaxv, g.slot, g.tmax);
        k_sg_starts<<<nblk((int64_t)ne + 1), kB, 0, st>>>(fcell, (int64_t)ne, ncells, g.start);
        if (hipStreamSynchronize(st) != hipSuccess) {
            (void)hipFree(g.start);
            (void)hipFree(g.tmax);
            (void)hipFree(g.slot);
            rc = -1;
            break;
        }
        for (int k = 0; k < 3; ++k) {
            g.U[k] = (float)f.U[k];
            g.V[k] = (float)f.V[k];
        }
        g.u0 = (float)f.u0;
        g.v0 = (float)f.v0;
        g.inv_cu = (float)(1.0 / f.cu);
        g.inv_cv = (float)(1.0 / f.cv);
        g.R = R;
        g.n_entries = (int64_t)ne;
        // the leaf-step form: tri_pre grows by one TriPre copy per entry
        const uint64_t base = (uint64_t)n + 1;  // scene slots + the null triangle
        if (base + ne >= (1ull << kLeafCountShift)) {
            (void)hipFree(g.start);
            (void)hipFree(g.tmax);
            (void)hipFree(g.slot);
            rc = -2;
            break;
        }
        TriPre* pre2 = nullptr;
        if (hipMalloc(&g.cell, (size_t)ncells * sizeof(uint2)) != hipSuccess ||
            hipMalloc(&pre2, (size_t)(base + ne) * sizeof(TriPre)) != hipSuccess) {
            if (g.cell) (void)hipFree(g.cell);
            (void)hipFree(g.start);
            (void)hipFree(g.tmax);
            (void)hipFree(g.slot);
            rc = -1;
            break;
        }
        (void)hipMemcpyAsync(pre2, s.tri_pre, (size_t)base * sizeof(TriPre), hipMemcpyDeviceToDevice, st);
        k_sg_copy_tris<<<nblk((int64_t)ne), kB, 0, st>>>(s.tri_pre, g.slot, (int64_t)ne, pre2 + base);
        k_sg_cellrec<<<nblk((int64_t)ncells), kB, 0, st>>>(g.start, ncells, (uint32_t)base, g.cell);
        if (hipStreamSynchronize(st) != hipSuccess) { rc = -1; break; }
        (void)hipFree(s.tri_pre);
        s.tri_pre = pre2;
        g.base = (int32_t)base;
        s.sgrid = g;
        if (getenv("TMPT_GRID_LOG")) {  // diagnostic: list lengths
            std::vector<uint32_t> hs((size_t)ncells + 1);
            if (hipMemcpy(hs.data(), g.start, hs.size() * 4, hipMemcpyDeviceToHost) == hipSuccess) {
                uint32_t mx = 0;
                uint64_t nonempty = 0;
                for (uint32_t c = 0; c < ncells; ++c) {
                    uint32_t l = hs[c + 1] - hs[c];
                    mx = std::max(mx, l);
                    nonempty += l > 0;
                }
                fprintf(stderr, "shadow grid %dx%d: %llu entries (%llu items), %llu non-empty cells, mean %.2f max %u\n", R, R,
                        (unsigned long long)ne, (unsigned long long)nitems, (unsigned long long)nonempty,
                        nonempty ? (double)ne / nonempty : 0.0, mx);
                fprintf(stderr, "  frame u0 %.6g v0 %.6g cu %.6g cv %.6g eps %.3g\n", f.u0, f.v0, f.cu, f.cv, f.eps);
            }
        }
    } while (0);
    free_tmp();
    if (rc) {
        set_error(rc == -2 ? "shadow grid: too many entries" : "shadow grid: HIP error");
        return rc;
    }
    return 0;
}

}  // namespace tmpt
