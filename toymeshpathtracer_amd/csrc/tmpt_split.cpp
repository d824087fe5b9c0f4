// tmpt_split.cpp -- early split clipping of the scene's large triangles
// (Ernst & Greiner 2007, "Early Split Clipping for Bounding Volume
// Hierarchies"), host side of the BVH build (build option `split`).
//
// A triangle whose box is large against the scene (a wall, a floor slab: on
// the sponza stand-in 1 % of the triangles hold 69 % of the area) gives the
// BVH a leaf box that most rays crossing the room overlap.  Such a triangle
// enters the build as several references instead: its box is halved along its
// longest axis, recursively, and each piece is the box of the triangle
// clipped to that half (Sutherland-Hodgman, in double), rounded outward to
// float.  The pieces' boxes cover the whole triangle, so culling stays
// conservative; every reference points at the same triangle, so the
// Moller-Trumbore test -- and with it every answer -- is unchanged
// (tmpt_traverse.h ignores a tie of a triangle with itself).  Output: per
// reference its triangle (~index: the whole triangle, whose padded box the
// device computes as without splitting) and, for a piece, its box.  Scene set-up,
// outside the timed region like the reference's BuildOctree (main.cpp:312).
#include <math.h>

#include <algorithm>
#include <vector>

#include "tmpt_internal.h"

namespace tmpt {

namespace {

struct P3 {
    double v[3];
};

// keeps the part of polygon `in` on the side x_k <= c (keep_lo) or >= c
void clip(const std::vector<P3>& in, int k, double c, bool keep_lo, std::vector<P3>& out)
{
    out.clear();
    const size_t n = in.size();
    for (size_t i = 0; i < n; ++i) {
        const P3& a = in[i];
        const P3& b = in[(i + 1) % n];
        const double da = keep_lo ? c - a.v[k] : a.v[k] - c, db = keep_lo ? c - b.v[k] : b.v[k] - c;
        if (da >= 0.0) out.push_back(a);
        if ((da >= 0.0) != (db >= 0.0)) {
            const double t = da / (da - db);
            P3 p;
            for (int q = 0; q < 3; ++q) p.v[q] = a.v[q] + t * (b.v[q] - a.v[q]);
            p.v[k] = c;
            out.push_back(p);
        }
    }
}

void bounds(const std::vector<P3>& poly, double lo[3], double hi[3])
{
    for (int q = 0; q < 3; ++q) {
        lo[q] = INFINITY;
        hi[q] = -INFINITY;
    }
    for (const P3& p : poly)
        for (int q = 0; q < 3; ++q) {
            lo[q] = std::min(lo[q], p.v[q]);
            hi[q] = std::max(hi[q], p.v[q]);
        }
}

// float rounded outward
float down(double x)
{
    float f = (float)x;
    return (double)f > x ? nextafterf(f, -INFINITY) : f;
}
float up(double x)
{
    float f = (float)x;
    return (double)f < x ? nextafterf(f, INFINITY) : f;
}

struct Splitter {
    double lim;  // a piece stops splitting once its box's largest extent is at most this
    std::vector<float>* boxes;
    std::vector<int32_t>* ref_tri;

    void emit(const std::vector<P3>& poly, int32_t tri)
    {
        double lo[3], hi[3];
        bounds(poly, lo, hi);
        for (int q = 0; q < 3; ++q) boxes->push_back(down(lo[q]));
        for (int q = 0; q < 3; ++q) boxes->push_back(up(hi[q]));
        ref_tri->push_back(tri);
    }

    void piece(std::vector<P3> poly, int32_t tri, int depth)
    {
        double lo[3], hi[3];
        bounds(poly, lo, hi);
        int k = 0;
        for (int q = 1; q < 3; ++q)
            if (hi[q] - lo[q] > hi[k] - lo[k]) k = q;
        if (hi[k] - lo[k] <= lim || depth >= 10 || poly.size() < 3) {
            emit(poly, tri);
            return;
        }
        const double c = 0.5 * (lo[k] + hi[k]);
        std::vector<P3> l, h;
        clip(poly, k, c, true, l);
        clip(poly, k, c, false, h);
        // a half that is only the cut itself (every vertex on the plane: the
        // triangle merely touches it there) is covered by the other half
        auto real = [&](const std::vector<P3>& q) {
            if (q.size() < 3) return false;
            for (const P3& p : q)
                if (p.v[k] != c) return true;
            return false;
        };
        const bool rl = real(l), rh = real(h);
        if (rl) piece(std::move(l), tri, depth + 1);
        if (rh) piece(std::move(h), tri, depth + 1);
        if (!rl && !rh) emit(poly, tri);  // degenerate: keep the whole piece
    }
};

}  // namespace

int32_t split_references(const float* tris9, int32_t n, float frac, std::vector<float>& boxes,
                         std::vector<int32_t>& ref_tri)
{
    boxes.clear();
    ref_tri.clear();
    float slo[3] = {INFINITY, INFINITY, INFINITY}, shi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = 0; i < (size_t)n * 3; ++i)
        for (int q = 0; q < 3; ++q) {
            slo[q] = std::min(slo[q], tris9[3 * i + q]);
            shi[q] = std::max(shi[q], tris9[3 * i + q]);
        }
    double ext = 0.0;
    for (int q = 0; q < 3; ++q) ext = std::max(ext, (double)shi[q] - (double)slo[q]);
    Splitter sp{frac * ext, &boxes, &ref_tri};
    boxes.reserve((size_t)n * 6);
    ref_tri.reserve((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        const float* t = tris9 + 9 * (size_t)i;
        std::vector<P3> poly(3);
        for (int v = 0; v < 3; ++v)
            for (int q = 0; q < 3; ++q) poly[(size_t)v].v[q] = t[3 * v + q];
        double lo[3], hi[3];
        bounds(poly, lo, hi);
        double e = 0.0;
        for (int q = 0; q < 3; ++q) e = std::max(e, hi[q] - lo[q]);
        if (!(e <= sp.lim) && std::isfinite(e)) {
            sp.piece(std::move(poly), i, 0);
        } else {  // the whole triangle: ~index, its box is the one the device computes (k_tri_prep)
            for (int q = 0; q < 6; ++q) boxes.push_back(0.0f);
            ref_tri.push_back(~i);
        }
    }
    return (int32_t)ref_tri.size();
}

}  // namespace tmpt
