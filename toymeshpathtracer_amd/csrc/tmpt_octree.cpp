// tmpt_octree.cpp -- the reference's octree, built on the host.
//
// The device answers HitScene from its BVH4Q, whose answer is the closest
// hit over all triangles.  The reference walks an 8-way octree instead
// (scene.cpp:21-52) and keeps the FIRST triangle of the smallest t in its
// depth-first visit order, and its root box test can drop a ray that only
// grazes the root.  The traversal flags the queries where that can matter --
// a tie on t; a closest hit near one of the octree's finest-level planes on a
// ray that runs almost within that plane, where the 1-2 ulp cracks between
// sibling boxes (min + half + half) can hide the hit (octree_grid); a hit on
// a triangle flat in such a plane, which may be in no leaf at all
// (octree_flat_triangles) -- and those, and only those, are answered again
// over this octree on the device (tmpt_traverse.h octree_closest, octree_flag).  So the octree has to be the
// reference's node for node: the same boxes (bmin/bmax halved in float,
// scene.cpp:109-141), the same triangle lists (the separating-axis overlap
// test of maths.cpp:165-298 in its own rounding order), the same limits
// (more than 10 triangles and depth below 10, scene.cpp:101).
//
// Layout (tmpt_internal.h OctNode): depth-first preorder, each node's skip
// link pointing past its subtree, so the device walks it without a stack.
// The 8 subtrees of the root are built on their own threads and spliced.
// Like the reference's BuildOctree (main.cpp:312, outside the timed region
// :319-333), this is scene set-up, not part of a render.
#include <string.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "tmpt_internal.h"

namespace tmpt {

namespace {

inline float comp(f3 v, int q) { return q == 0 ? v.x : (q == 1 ? v.y : v.z); }

// PlaneIntersectAabb (maths.cpp:165-197): does the plane through `vert` with
// normal `n` meet the box [-half, half]?  The nearest and farthest box corners
// along n, offset by -vert, tested with glm::dot's (x*x' + y*y') + z*z'.
bool plane_meets_box(f3 n, f3 vert, f3 half)
{
    float near_c[3], far_c[3];
    for (int q = 0; q < 3; ++q) {
        const float h = comp(half, q), v = comp(vert, q);
        const bool pos = comp(n, q) > 0.0f;
        near_c[q] = pos ? -h - v : h - v;
        far_c[q] = pos ? h - v : -h - v;
    }
    if (dot(n, mk(near_c[0], near_c[1], near_c[2])) > 0.0f) return false;
    return dot(n, mk(far_c[0], far_c[1], far_c[2])) >= 0.0f;
}

// One cross-product axis of the separating-axis test (the AXISTEST_* macros,
// maths.cpp:112-156): the two distinct vertex projections pa, pb (ordered as
// the macro orders its pair) against the box's projected radius.
inline bool axis_separates(float pa, float pb, float rad)
{
    const float lo = pa < pb ? pa : pb, hi = pa < pb ? pb : pa;
    return lo > rad || hi < -rad;
}

// The triangle's extent on one box axis (FINDMINMAX, maths.cpp:158-163) against
// the half size.
inline bool extent_separates(float a, float b, float c, float h)
{
    float lo = a, hi = a;
    if (b < lo) lo = b;
    if (b > hi) hi = b;
    if (c < lo) lo = c;
    if (c > hi) hi = c;
    return lo > h || hi < -h;
}

// TriangleIntersectAabb (maths.cpp:199-298): Akenine-Moller's triangle / box
// overlap with the box centred at `c`, half size `h`.  The nine edge axes in
// the reference's order (its early exits do not change the answer, only the
// rounding of each projection does, so each one is formed as the macro does:
// products, then one difference), then the box axes, then the plane.
bool tri_overlaps_box(f3 c, f3 h, const f3* tri)
{
    const f3 v0 = tri[0] - c, v1 = tri[1] - c, v2 = tri[2] - c;
    const f3 e[3] = {v1 - v0, v2 - v1, v0 - v2};
    // vertex pairs per edge: x and y axes use (v0, v2) for edges 0 and 1 and
    // (v0, v1) for edge 2; the z axis (v1, v2), (v0, v1), (v1, v2), each pair
    // in the order its macro compares them
    const f3* xy_pair[3][2] = {{&v0, &v2}, {&v0, &v2}, {&v0, &v1}};
    const f3* z_pair[3][2] = {{&v2, &v1}, {&v0, &v1}, {&v2, &v1}};  // Z12 orders (p2, p1)
    for (int k = 0; k < 3; ++k) {
        const f3 E = e[k];
        const float ax = fabsf(E.x), ay = fabsf(E.y), az = fabsf(E.z);
        const f3 &p = *xy_pair[k][0], &q = *xy_pair[k][1];
        // x: a = E.z, b = E.y -> a*v.y - b*v.z, rad = |E.z| h.y + |E.y| h.z
        if (axis_separates(E.z * p.y - E.y * p.z, E.z * q.y - E.y * q.z, az * h.y + ay * h.z)) return false;
        // y: -a*v.x + b*v.z with a = E.z, b = E.x, rad = |E.z| h.x + |E.x| h.z
        if (axis_separates(-E.z * p.x + E.x * p.z, -E.z * q.x + E.x * q.z, az * h.x + ax * h.z)) return false;
        // z: a*v.x - b*v.y with a = E.y, b = E.x, rad = |E.y| h.x + |E.x| h.y
        const f3 &r = *z_pair[k][0], &s = *z_pair[k][1];
        if (axis_separates(E.y * r.x - E.x * r.y, E.y * s.x - E.x * s.y, ay * h.x + ax * h.y)) return false;
    }
    if (extent_separates(v0.x, v1.x, v2.x, h.x)) return false;
    if (extent_separates(v0.y, v1.y, v2.y, h.y)) return false;
    if (extent_separates(v0.z, v1.z, v2.z, h.z)) return false;
    return plane_meets_box(cross(e[0], e[1]), v0, h);
}

inline float int_bits(int32_t v)
{
    float f;
    memcpy(&f, &v, 4);
    return f;
}
inline int32_t bits_int(float f)
{
    int32_t v;
    memcpy(&v, &f, 4);
    return v;
}

struct Builder {
    const f3* tris;  // 3 vertices per triangle
    OctreeHost out;

    // child k of [lo, hi] (scene.cpp:119-141): bit 0 of k offsets x, bit 1 z,
    // bit 2 y by the parent's half size; child 0 keeps the parent's min
    // without an addition (a -0 coordinate stays -0)
    static void child_box(f3 lo, f3 half, int k, f3& clo, f3& chi)
    {
        clo = k == 0 ? lo : lo + mk((k & 1) ? half.x : 0.0f, (k & 4) ? half.y : 0.0f, (k & 2) ? half.z : 0.0f);
        chi = clo + half;
    }

    // the triangles of `ids` that overlap child box [clo, chi], in order
    // (scene.cpp:144-154: centre and half size from the child's own box)
    void filter(f3 clo, f3 chi, const std::vector<int32_t>& ids, std::vector<int32_t>& sub) const
    {
        const f3 c = (clo + chi) * 0.5f, h = (chi - clo) * 0.5f;
        sub.clear();
        for (int32_t id : ids)
            if (tri_overlaps_box(c, h, tris + 3 * (size_t)id)) sub.push_back(id);
    }

    void node(f3 lo, f3 hi, const std::vector<int32_t>& ids, int depth)
    {
        const size_t me = out.nodes.size();
        out.nodes.push_back(OctNode{make_float4(lo.x, lo.y, lo.z, 0.0f), make_float4(hi.x, hi.y, hi.z, 0.0f)});
        out.depth = std::max(out.depth, depth);
        if (ids.size() > 10 && depth < 10) {  // scene.cpp:101
            out.nodes[me].hi.w = int_bits(-1);
            const f3 half = (hi - lo) * 0.5f;  // dimensions() * 0.5f, scene.cpp:109
            std::vector<int32_t> sub;
            sub.reserve(ids.size());
            for (int k = 0; k < 8; ++k) {
                f3 clo, chi;
                child_box(lo, half, k, clo, chi);
                filter(clo, chi, ids, sub);
                node(clo, chi, sub, depth + 1);
            }
        } else {
            out.nodes[me].hi.w = int_bits((int32_t)out.refs.size());
            out.refs.push_back((int32_t)ids.size());
            out.refs.insert(out.refs.end(), ids.begin(), ids.end());
            ++out.leaves;
        }
        out.nodes[me].lo.w = int_bits((int32_t)out.nodes.size());
    }
};

}  // namespace

void build_octree(const float* tris9, int32_t n, const float bmin[3], const float bmax[3], OctreeHost& out)
{
    std::vector<f3> v((size_t)n * 3);
    for (size_t i = 0; i < v.size(); ++i) v[i] = mk(tris9[3 * i], tris9[3 * i + 1], tris9[3 * i + 2]);
    const f3 lo = mk(bmin[0], bmin[1], bmin[2]), hi = mk(bmax[0], bmax[1], bmax[2]);
    std::vector<int32_t> all((size_t)n);
    for (int32_t i = 0; i < n; ++i) all[(size_t)i] = i;  // BuildOctree: the scene's triangle order
    out = OctreeHost();
    if (!(all.size() > 10)) {  // a leaf root
        Builder b{v.data(), {}};
        b.node(lo, hi, all, 0);
        out = std::move(b.out);
        return;
    }
    // the root's 8 subtrees on their own threads, spliced in child order
    const f3 half = (hi - lo) * 0.5f;
    Builder part[8];
    std::vector<std::thread> th;
    for (int k = 0; k < 8; ++k) {
        part[k].tris = v.data();
        th.emplace_back([&, k]() {
            f3 clo, chi;
            Builder::child_box(lo, half, k, clo, chi);
            std::vector<int32_t> sub;
            part[k].filter(clo, chi, all, sub);
            part[k].node(clo, chi, sub, 1);
        });
    }
    for (auto& t : th) t.join();
    size_t nn = 1, nr = 0;
    for (auto& p : part) {
        nn += p.out.nodes.size();
        nr += p.out.refs.size();
    }
    out.nodes.reserve(nn);
    out.refs.reserve(nr);
    out.nodes.push_back(OctNode{make_float4(lo.x, lo.y, lo.z, int_bits((int32_t)nn)),
                                make_float4(hi.x, hi.y, hi.z, int_bits(-1))});
    for (auto& p : part) {
        const int32_t on = (int32_t)out.nodes.size(), orf = (int32_t)out.refs.size();
        for (OctNode nd : p.out.nodes) {
            nd.lo.w = int_bits(bits_int(nd.lo.w) + on);
            const int32_t r = bits_int(nd.hi.w);
            if (r >= 0) nd.hi.w = int_bits(r + orf);
            out.nodes.push_back(nd);
        }
        out.refs.insert(out.refs.end(), p.out.refs.begin(), p.out.refs.end());
        out.leaves += p.out.leaves;
        out.depth = std::max(out.depth, p.out.depth);
    }
}

// The crack grid (tmpt_internal.h OctGrid): every node box face lies on a plane
// r0 + j * cell of the finest level to within the largest offset found here
// (the rounding of min + half + half down the tree); the band adds margin for
// the device's float evaluation of the plane and of the hit point.
void octree_grid(const OctreeHost& t, const float bmin[3], const float bmax[3], OctGrid& g)
{
    const double scale = std::ldexp(1.0, t.depth);
    float cmin = INFINITY;
    for (int k = 0; k < 3; ++k) {
        const double r0 = bmin[k], size = (double)bmax[k] - (double)bmin[k];
        const double cell = size > 0.0 ? size / scale : 1.0;
        double w = 0.0;
        for (const OctNode& nd : t.nodes) {
            const double v[2] = {comp(mk(nd.lo.x, nd.lo.y, nd.lo.z), k), comp(mk(nd.hi.x, nd.hi.y, nd.hi.z), k)};
            for (double x : v) w = std::max(w, std::fabs(x - (r0 + std::nearbyint((x - r0) / cell) * cell)));
        }
        const float ulp = std::nextafter(std::max(std::fabs(bmin[k]), std::fabs(bmax[k])), INFINITY) -
                          std::max(std::fabs(bmin[k]), std::fabs(bmax[k]));
        g.r0[k] = bmin[k];
        g.cell[k] = (float)cell;
        g.inv_cell[k] = (float)(1.0 / cell);
        g.band[k] = (float)(4.0 * w + 8.0 * (double)ulp);
        g.drift[k] = 2.0f * g.band[k];
        cmin = std::min(cmin, (float)cell);
    }
    g.reach = 0.5f * cmin;
}

// Distance of x to the nearest plane of axis k, as the device evaluates it
// (tmpt_traverse.h octree_crack), and that plane's number.
static float plane_dist(const OctGrid& g, int k, float x, float& j)
{
    const float rel = x - g.r0[k];
    j = rintf(rel * g.inv_cell[k]);
    return fabsf(fmaf(-j, g.cell[k], rel));
}

// Triangles the reference's octree may not hold where a ray hits them (DESIGN.md
// section 2, "the derived bound"): (F1) all three vertices within 2 band of one
// plane -- the triangle can lie in a crack, in no leaf at all; (F2) a triangle
// nearly parallel to a plane family that comes within band of one of its
// planes: its plane leaves the 2-band slab around that plane only beyond
// `reach` of a point inside it (sin(angle) * reach <= 2 band), so near such a
// point it may meet neither leaf either side of the crack robustly.
int32_t octree_flat_triangles(const float* tris9, int32_t n, const OctGrid& g, std::vector<uint8_t>& flat)
{
    flat.assign((size_t)n, 0);
    int32_t count = 0;
    for (int32_t i = 0; i < n; ++i) {
        const float* v = tris9 + 9 * (size_t)i;
        for (int k = 0; k < 3 && !flat[(size_t)i]; ++k) {  // F1
            float j0, j1, j2;
            const float d0 = plane_dist(g, k, v[k], j0), d1 = plane_dist(g, k, v[3 + k], j1),
                        d2 = plane_dist(g, k, v[6 + k], j2);
            const float lim = 2.0f * g.band[k];
            if (j0 == j1 && j1 == j2 && d0 <= lim && d1 <= lim && d2 <= lim) flat[(size_t)i] = 1;
        }
        if (!flat[(size_t)i]) {  // F2
            const double e1[3] = {(double)v[3] - v[0], (double)v[4] - v[1], (double)v[5] - v[2]};
            const double e2[3] = {(double)v[6] - v[0], (double)v[7] - v[1], (double)v[8] - v[2]};
            const double nr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                                  e1[0] * e2[1] - e1[1] * e2[0]};
            const double len = std::sqrt(nr[0] * nr[0] + nr[1] * nr[1] + nr[2] * nr[2]);
            for (int k = 0; k < 3 && len > 0.0 && !flat[(size_t)i]; ++k) {
                const double nk = std::fabs(nr[k]) / len, sin_a = std::sqrt(std::max(0.0, 1.0 - nk * nk));
                if (sin_a * (double)g.reach > 2.0 * (double)g.band[k]) continue;
                const double lo = std::min({(double)v[k], (double)v[3 + k], (double)v[6 + k]}) - g.band[k];
                const double hi = std::max({(double)v[k], (double)v[3 + k], (double)v[6 + k]}) + g.band[k];
                // a plane r0 + j cell inside [lo, hi]
                if (std::floor((hi - g.r0[k]) / g.cell[k]) >= std::ceil((lo - g.r0[k]) / g.cell[k])) flat[(size_t)i] = 1;
            }
        }
        count += flat[(size_t)i];
    }
    return count;
}

uint64_t octree_digest(const OctreeHost& t)
{
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint32_t w) {
        for (int b = 0; b < 4; ++b) h = (h ^ ((w >> (8 * b)) & 255u)) * 1099511628211ull;
    };
    auto fbits = [](float f) {
        uint32_t u;
        memcpy(&u, &f, 4);
        return u;
    };
    for (const OctNode& nd : t.nodes) {
        mix(fbits(nd.lo.x)), mix(fbits(nd.lo.y)), mix(fbits(nd.lo.z));
        mix(fbits(nd.hi.x)), mix(fbits(nd.hi.y)), mix(fbits(nd.hi.z));
        const int32_t r = bits_int(nd.hi.w);
        mix(r < 0 ? 0u : 1u);
        if (r >= 0)
            for (int32_t k = 0; k <= t.refs[(size_t)r]; ++k) mix((uint32_t)t.refs[(size_t)r + (size_t)k]);
    }
    return h;
}

}  // namespace tmpt
