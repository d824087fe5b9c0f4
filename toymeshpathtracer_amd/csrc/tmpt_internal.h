// tmpt_internal.h -- device data layout and the scene object behind the C ABI.
//
// HBM layout of one scene (DESIGN.md "Data layout in HBM"):
//   nodes4   Bvh4Node[<= n-1]     64 B  4-wide BVH, quantised child boxes,
//                                        numbered level by level (the top
//                                        kTopNodes are copied to LDS)
//   tri_pre  TriPre[n + 1]        48 B  leaf order: v0, e1 = v1-v0, e2 = v2-v0,
//                                        original index (the Moller-Trumbore operands)
//   tri_orig TriOrig[n]           48 B  original order: v0, v1, v2 and the geometric
//                                        normal, read once per accepted hit
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "tmpt_math.h"

namespace tmpt {

// 4-wide node with quantised child boxes (DESIGN.md "BVH4Q"): 64 B, one
// half cache line, 4 x dwordx4 loads for FOUR child boxes.
//   a: origin.xyz (node box min, f32), w = exponents ex,ey,ez (bytes 0-2,
//      signed: scale = 2^e) | child-valid mask (byte 3)
//   b: qlo.x[4], qhi.x[4], qlo.y[4], qhi.y[4]   (uint8 per child, child k in byte k)
//   c: qlo.z[4], qhi.z[4], 0, 0
//   d: child links: >=0 node index; <0 leaf = 0x80000000 | (count-1)<<27 | first slot
// A child box decodes as origin + q*scale (q*scale exact), quantised outward
// from the padded boxes, so culling stays conservative.
struct alignas(16) Bvh4Node {
    float4 a;
    uint4 b;
    uint4 c;
    int4 d;
};
static_assert(sizeof(Bvh4Node) == 64, "BVH4Q node is one half cache line");

constexpr int kLeafCountShift = 27;
constexpr uint32_t kLeafFirstMask = (1u << kLeafCountShift) - 1u;
constexpr int kLeafMaxTris = 16;
constexpr int kTopNodes = 120;  // BVH4 nodes held in LDS per path block (7.5 KB)
// The same in the 5-wave path kernels (OCC 5): 5 KB, so a block's LDS is 30 KB
// (12-entry stack 12 KB, light terms 10 KB, pending ray 3 KB, top nodes 5 KB).
// Five such blocks fit a CU; with 104 nodes (31.5 KB) they did not (the
// occupancy API still said 5, and the launch's tail waited for blocks that
// were never resident), 72-96 nodes measured alike.
constexpr int kTopNodes5 = 80;

struct alignas(16) TriPre {
    float4 a;  // v0.xyz, e1.x
    float4 b;  // e1.yz, e2.xy
    float4 c;  // e2.z, 2 x original index (int bits; bit 0 is the traversal's tie flag), 0, 0
};
struct alignas(16) TriOrig {
    float4 a;  // v0.xyz, v1.x
    float4 b;  // v1.yz, v2.xy
    float4 c;  // v2.z, normal.xyz
};

// The reference's own octree (Scene::BuildOctree, scene.cpp:75-83, 99-160),
// kept for the answers the BVH cannot give by itself: which of several
// triangles that tie on t the reference returns (its first strict '<' in
// depth-first child order 0..7, scene.cpp:29-48) and the rays its root box
// test drops.  Nodes in depth-first preorder, 32 B each:
//   lo = box min.xyz, w = skip (int bits): the node after this subtree
//   hi = box max.xyz, w = ref  (int bits): -1 for an inner node; a leaf's
//        triangles are refs[ref + 1 .. ref + refs[ref]] in the reference's order
// Built on the host (the reference's build is untimed too, main.cpp:312 vs
// :319) by tmpt_octree.cpp; read by the device only for flagged queries.
struct alignas(16) OctNode {
    float4 lo;
    float4 hi;
};
static_assert(sizeof(OctNode) == 32, "octree node: two dwordx4 loads");

// The octree's cracks ("cracks"): a child box is its
// parent's min plus half the parent's size, its max that plus half again, so
// the boxes of two neighbouring subtrees need not share a face bit for bit --
// one subtree can end an ulp or two before the next begins.  A ray that runs
// inside such a gap, nearly parallel to it, passes no leaf there, and the
// reference misses a triangle the exact closest hit finds; a triangle lying
// flat inside a gap is in no leaf at all.  The planes of the octree are the
// grid r0 + j * cell (cell = root size / 2^depth) to within `band`, so the
// queries that can land in a gap are known from the hit alone:
//   crack  hit point within band[k] of a plane of axis k, and the ray moved
//          less than 2 band[k] along k over min(t, reach) -- it ran along
//          the gap -- for some axis k;
//   flat   the hit triangle lies within 2 band[k] of one plane (its TriPre
//          index is odd: marked when the octree is built).
// Both are answered over the octree, as ties are.
struct OctGrid {
    // first 16 B: what every finished query reads (one scalar dwordx4 load)
    float reach;        // half the smallest cell: t beyond which a ray's drift along k is judged
    float drift[3];     // 2 x band: the drift along k that counts as running along a plane
    float r0[3];        // root box min
    float inv_cell[3];  // 2^depth / root size
    float cell[3];      // root size / 2^depth
    float band[3];      // 4 x the largest plane offset of any node box + 8 ulp of the root's coordinates
};

// What the kernels see of it (one device-side struct, so a kernel keeps one
// pointer live): nodes, leaf lists, node count, the counters of the queries
// it answered ([0] ties, [1] root-box misses, [6] crack / flat-triangle
// queries; Scene::ties), the crack grid.
struct OctView {
    const OctNode* nodes;
    const int32_t* refs;
    int32_t n;
    int32_t flat;  // triangles marked flat (0: the any-hit answers need no check)
    unsigned long long* ties;
    OctGrid grid;
    int64_t n_refs;  // entries of refs (the checked build's bound)
};

// Device bounds checks, the checked build only (make CHECK=1: -DTMPT_CHECK,
// ../_lib_check; tools/check_build.sh).  The traversal, both octree walks and
// the hit-record loads test each index before they use it -- BVH node, leaf
// range, stack depth, octree skip link and reference list, triangle id --
// and a failed test ends that query and ORs its code into Scene::chk
// ({codes, count, last offending value}); the API call then fails with
// kCheckError and names the codes (tmpt_last_error).  The product build
// compiles none of it.
constexpr uint32_t kChkNode = 1u, kChkLeaf = 2u, kChkStack = 4u, kChkOctSkip = 8u, kChkOctRef = 16u,
                   kChkTri = 32u;
constexpr int kCheckError = -30;

struct OctreeHost {
    std::vector<OctNode> nodes;
    std::vector<int32_t> refs;
    int32_t leaves = 0, depth = 0;
};

// Subdivide / InternalDivide of scene.cpp:99-160 from the root box [bmin, bmax]
// (main.cpp:312: the scene bounds +- 0.7 x their size)
void build_octree(const float* tris9, int32_t n, const float bmin[3], const float bmax[3], OctreeHost& out);
// FNV-1a over the preorder walk (node boxes' bits, leaf triangle lists): the
// structure check the CPU tests compare with the oracle's octree
uint64_t octree_digest(const OctreeHost& t);
// The crack grid of an octree (tmpt_octree.cpp) and the triangles that lie
// flat on one of its planes (flat[i] = 1).
void octree_grid(const OctreeHost& t, const float bmin[3], const float bmax[3], OctGrid& g);
int32_t octree_flat_triangles(const float* tris9, int32_t n, const OctGrid& g, std::vector<uint8_t>& flat);

// Build option layout=soa (the north star's "SoA" A/B):
// the BVH4Q nodes and the leaf-ordered triangle records as planes, each plane
// one load of a step -- node planes a (origin, exponents), b (x / y byte
// planes), c (z byte planes, 8 B: no padding), d (child links); triangle
// planes a (v0, e1.x), b (e1.yz, e2.xy), c (e2.z, index: 8 B).  56 B per node
// and 40 B per triangle instead of 64 and 48, in 4 and 3 separate lines.
struct SoaScene {
    const uint4* __restrict__ na = nullptr;
    const uint4* __restrict__ nb = nullptr;
    const uint2* __restrict__ nc = nullptr;
    const int4* __restrict__ nd = nullptr;
    const float4* __restrict__ ta = nullptr;
    const float4* __restrict__ tb = nullptr;
    const float2* __restrict__ tc = nullptr;
};

// Box culling is conservative (DESIGN.md "Scene query contract"): leaf boxes are
// inflated by kBoxPadRel * (|coord| + extent) and the far slab distance is
// stretched by kTfarSlack, so every triangle the reference would accept is
// reached and Moller-Trumbore alone decides.
constexpr float kBoxPadRel = 1e-5f;
constexpr float kTfarSlack = 1.00001f;

// Stack: SL entries per lane live in LDS, the rest spill to a global per-lane
// area.  BVH4Q: <= 3 entries per level.  The build rejects trees that could
// exceed kStackTotal (DESIGN.md "Traversal").
constexpr int kStackTotal = 128;

constexpr int kRowSpecMaxGroups = 8;  // speculative row engine: row groups (streams)
constexpr int kRenderCounters = 32;   // ray / visit / round counters of one render
constexpr int kTieCounter = 24;       // [24] tied queries re-answered over the octree, [25] root-box misses,
                                      // [30] crack / flat-triangle queries re-answered over it (ties[6])
constexpr int kCrackCounter = 30;
constexpr int kRedoRaysCounter = 31;  // rays of the k_redo launch (part of [0])
constexpr int kRedoCounter = 26;      // samples the deferred-tie sample kernel left to the redo pass

// Per-scene options: the library's control plane in place of environment
// variables (include/tmpt.h documents each key).  Build options are fixed when
// the scene is created; render options apply to the renders after they are set.
struct Options {
    // build (tmpt_scene_create_ex)
    int builder = 0;      // 0 = PLOC (Meister & Bittner 2018), 1 = LBVH (Karras 2012)
    int layout = 0;       // 0 = AoS records (64-B nodes, 48-B triangles), 1 = also SoA planes (SoaScene)
    int leaf_max = 2;     // triangles per BVH4 leaf, 1..kLeafMaxTris
    int collapse = 0;     // BVH2 -> BVH4: 0 = greedy largest-area opening, 1 = SAH-optimal
    int ploc_radius = 32; // PLOC nearest-neighbour search radius
    float sah_c_leaf = 0.7f, sah_c_tri = 0.5f;  // SAH collapse costs (inner node = 1)
    // render (tmpt_scene_set_option)
    int sample_block = 0;     // sample seeding: samples per work unit, a power of two (0 = auto)
    int rowstream_dynamic = 1;  // row seeding, streaming: windows and spread follow the live rows
    int row_flag_leaves = 1;    // row seeding, streaming, octree answering: flag-only leaves (TIES 2)
    int row_occ = 0;            // row seeding, streaming: worker waves per SIMD (0 = by load, 4, 5)
    int sample_tail = -1;     // sample seeding: blocks per resident lane run as single samples at the end (-1 auto)
    double sbuf_max = 0.0;    // sample seeding: cap on the per-sample colour buffer, bytes (0 = 3/4 of free HBM)
    int sbuf_pair = 1;        // sample seeding: a unit's sample pairs written back to back into one 32-B sector
    int pilot = -1;           // pixel seeding: pilot-pass samples of the cost ordering (-1 auto, 0 off)
    int help = -1;            // pixel seeding: shadow offload to idle lanes (-1 auto, 0 off, 1 on)
    int pair = -1;            // pixel seeding: expensive ranks per 64-rank chunk with offload (-1 auto)
    int balance = 1;          // pixel seeding: SIMD-balanced first chunks
    int dprio = 1;            // pixel seeding: longest-remaining-first wave priority with offload
    int wave_cap = 0;         // pixel seeding: pixels a wave holds at once (0 auto, else 1..64)
    int pixel_chains = -1;    // pixel seeding, ordered: heaviest pixels per 1024 run as speculative chains (-1 auto)
    int rowspec = 1;          // row seeding: speculative row engine (0 = one lane per row chain)
    int rowspec_wmax = 0;     // row seeding: units per window (0 = auto: 24 x spp)
    int rowspec_windows = 0;  // row seeding: windows per row and iteration (0 = auto)
    float rowspec_spread = -1.0f;  // row seeding: window spread in pixels (-1 = auto)
    int rowspec_groups = 2;   // row seeding: row groups on their own streams
    int rowspec_noshadow = 1; // row seeding: shadow-free speculation + one full re-trace of the chain
    int rowspec_chase = 1;    // row seeding, shadow-free: the chase walks LDS-staged units, one wave per row
    int rowspec_stream = 1;   // row seeding: the streaming row engine (one launch; 0 = iterations)
    int rowstream_test_abort = 0;  // test hook: the streaming engine's chasers leave at once, so its
                                   // watchdog aborts the launch and the iterated engine renders the frame
    int wf_bins = 1;          // wavefront engine: extend sub-queues per segment by direction octant (1, 2, 4, 8)
    int tie_rule = 0;         // closest hits tied on t: 0 = the reference's octree visit order (needs
                              // tmpt_scene_build_octree), 1 = the lowest triangle index
    int tie_defer = -1;       // sample seeding, octree rule: tied samples left to a redo pass, so the
                              // main kernel carries no octree walk (-1 auto, 0 off, 1 on)
    int redo_cap = 0;         // test hook: the redo list's capacity in entries (0 = auto; a small one
                              // overflows, and the frame is rendered again with the list grown)
    int redo_lanes = 4;       // tie_defer: lanes per wave that take re-traces in the launch's tail
    int path_waves = 0;       // path-kernel waves per SIMD (0 = auto: 5 in sample seeding, in pixel seeding
                              // from 3 pixels per 4-wave lane; 4 or 5)
    int redo_inline = 1;      // test hook: 0 = the deferring kernel's waves leave every dropped sample
                              // to the k_redo launch (its fallback) instead of tracing them in their tail
};
int options_parse(Options& o, const char* text, bool allow_build);
int options_set(Options& o, const char* key, double value, bool allow_build);
int options_get(const Options& o, const char* key, double* value);

struct Scene {
    int device = 0;
    int32_t n = 0;          // triangles incl. the floor
    int32_t n_nodes = 0;    // internal nodes of the binary tree the BVH4 is collapsed from
    int32_t max_depth = 0;  // of the LBVH (Karras builder)
    Bvh4Node* nodes4 = nullptr;
    int32_t n_nodes4 = 0, depth4 = 0, leaf_max = 0, ploc_iters = 0;
    TriPre* tri_pre = nullptr;
    TriOrig* tri_orig = nullptr;
    void* soa_buf = nullptr;  // layout=soa: the planes of SoaScene, one allocation
    SoaScene soa;
    std::vector<float> tris_host;  // the triangles as given (Scene::Scene keeps its copy too)
    // the reference's octree (tmpt_scene_build_octree), and the counter of
    // closest-hit queries answered through it in the current call
    OctNode* oct = nullptr;
    int32_t* oct_refs = nullptr;
    OctView* oct_view = nullptr;  // device copy of {oct, oct_refs, n_oct, ties}
    int32_t n_oct = 0, oct_leaves = 0, oct_depth = 0;
    int32_t oct_flat = 0;  // triangles flat on one of the octree's planes (OctView::flat)
    OctGrid oct_grid{};    // its crack grid (OctView::grid)
    int64_t n_oct_refs = 0;
    double oct_build_ms = 0.0;
    float oct_lo[3] = {0, 0, 0}, oct_hi[3] = {0, 0, 0};
    unsigned long long* ties = nullptr;  // [0] re-answered ties, [1] root-box misses
    uint64_t tie_queries = 0, root_misses = 0, crack_queries = 0;
    // row seeding: the engine of the last render (0 none, 1 one lane per row,
    // 2 iterated speculative, 3 streaming) and whether the streaming engine's
    // launch aborted and was re-rendered by the iterated one
    int32_t row_engine = 0, stream_fallbacks = 0;
    int64_t chain_pixels = 0;  // pixel seeding: pixels of the last render run as speculative chains
    Options opt;  // build and render options (tmpt_scene_create_ex / tmpt_scene_set_option)
    hipEvent_t wait_ev = nullptr;  // TMPT_FLAG_WAIT_STREAM: reused across renders
    unsigned long long* counters = nullptr;       // a render's ray / visit counters (device)
    unsigned long long* counters_host = nullptr;  // their pinned host copy
    uint32_t* chk = nullptr;  // the checked build's device word triple (kChk* codes), else unused
    hipEvent_t render_ev[2] = {nullptr, nullptr}; // first / last kernel of a render
    hipStream_t stream = nullptr;
    double build_ms = 0.0;
    // render workspace (grown on demand, reused across calls)
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // progressive spp: per-pixel {colour sum xyz, rng} of the last pass, and the
    // shard it belongs to (width, height, spp, band_rows, shard, num_shards, next sample)
    float4* prog = nullptr;
    size_t prog_slots = 0;
    int32_t prog_key[7] = {0, 0, 0, 0, 0, 0, -1};
    uint64_t prog_cam = 0;  // FNV-1a of the camera (and seed mode) of that pass
    // sample seeding: sample_seed's jump tables for samples [0, jt_spp), and the
    // per-sample colour buffer of block-split pixels (tmpt_render.hip k_resolve)
    uint32_t* jt = nullptr;
    int32_t jt_spp = 0;
    float4* sbuf = nullptr;
    size_t sbuf_bytes = 0;
    // deferred ties (PathCtl::redo): the redo list, its capacity in entries,
    // and the samples the last render left to the redo pass
    uint2* redo = nullptr;
    uint32_t redo_cap = 0;
    float4* redo_state = nullptr;  // per redo slot: where its path stopped (tmpt_render.hip kRedoState4)
    int64_t redo_samples = 0;
    int64_t redo_late = 0;   // of them, left by the launch's tail to the k_redo launch
    int32_t redo_launches = 0;  // k_redo launches of the last render
    int32_t tie_path = 0;       // tmpt_stats.tie_path of the last render
    double redo_ms = 0.0;       // and their time (not in extend_ms)
    uint64_t redo_rays = 0;     // and their rays (in the render's count)
    // speculative row seeding (tmpt_render.hip render_rowspec): jump tables
    // M^(2j) for j in [0, jt2_n), and its row/unit buffers
    uint32_t* jt2 = nullptr;
    int32_t jt2_n = 0;
    void* rs_buf = nullptr;
    size_t rs_bytes = 0;
    hipStream_t rs_stream[kRowSpecMaxGroups] = {};      // one per row group
    hipEvent_t rs_event[kRowSpecMaxGroups + 1] = {};    // group ends; [max]: the start
    uint32_t* rs_host = nullptr;                        // pinned: each group's last unit count
    void* rs_list = nullptr;                            // no-shadow speculation: the chain list
    size_t rs_list_bytes = 0;
    // streaming row engine (render_rowstream): rings, windows, anchors; its
    // jump tables (M^(2c), M^(256b), M^(2^15 a0), M^(2^20 a1)); pinned control words
    void* rss_buf = nullptr;
    size_t rss_bytes = 0;
    uint32_t* rss_tab = nullptr;
    uint32_t* rss_host = nullptr;
    int path_launches = 1;  // k_path launches of the last persistent render (pilot ordering: 2)
    hipEvent_t path_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // around the pilot / final k_path
    // statistics of the last render
    double render_ms = 0.0;
    double extend_ms = 0.0;
    double shadow_ms = 0.0;
    uint64_t extend_rays = 0, shadow_rays = 0;
    int64_t extend_launches = 0, shadow_launches = 0, iterations = 0;
    uint64_t node_visits = 0, tri_tests = 0;  // only with TMPT_FLAG_COUNT_VISITS
    uint64_t shadow_node_visits = 0, shadow_tri_tests = 0;
};

// error plumbing: last error is thread-local, ints cross the ABI, never exceptions
void set_error(const std::string& msg);
const char* last_error();

#define TMPT_HIP(call)                                                                  \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            ::tmpt::set_error(std::string(#call) + ": " + hipGetErrorString(e_));       \
            return -1;                                                                  \
        }                                                                               \
    } while (0)

// tmpt_bvh.hip
int build_lbvh(Scene& s, const float* d_tris9);
int build_soa(Scene& s);  // layout=soa planes from the built AoS records
// the octree's flat triangles marked in the leaf-ordered records (bit 0 of the
// doubled index), the others cleared; flat has s.n entries (empty: clear all)
int mark_flat_triangles(Scene& s, const std::vector<uint8_t>& flat);
// tmpt_render.hip: the scene's counters, pinned copy and render events (once)
int ensure_counters(Scene& s);
int check_report(Scene& s, const char* what);
// tmpt_render.hip: sample_seed's byte tables for samples [0, spp) (1024 words each)
void sample_jump_tables(int32_t spp, std::vector<uint32_t>& tab);
// device radix sort of (key, value) pairs (tmpt_bvh.hip); returns 0 if the
// result is in (keys, vals), 1 if in (tkeys, tvals)
int radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* tkeys, uint32_t* tvals, int32_t n,
                     int bits, uint32_t* hist, hipStream_t st);
size_t radix_sort_hist_words(int32_t n);

TMPT_HD float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }

}  // namespace tmpt
