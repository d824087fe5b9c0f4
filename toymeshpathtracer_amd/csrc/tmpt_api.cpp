// tmpt_api.cpp -- the C ABI of include/tmpt.h.  Status ints cross the
// boundary; no exception escapes (every entry point catches).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "tmpt.h"
#include "tmpt_internal.h"
#include "tmpt_traverse.h"

namespace tmpt {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

int load_obj(const char* path, std::vector<float>& tris, f3& bmin, f3& bmax);
void camera_init(tmpt_camera* cam, f3 lookFrom, f3 lookAt, f3 vup, float vfov, float aspect,
                 float aperture, float focusDist);
void camera_for_scene(tmpt_camera* cam, f3 sceneMin, f3 sceneMax, int w, int h, bool sponza);
int write_png(const char* path, const uint8_t* rgba, int w, int h);
int render(Scene& s, const tmpt_camera* cam, const tmpt_render_desc* d, uint32_t* d_out,
           uint64_t* ray_count);
int intersect_batch(Scene& s, const float* d_rays, int64_t n, float tmin, float tmax, bool any, bool ranged,
                    float* d_hits, int32_t* d_ids);

// RandomUnitVector's (cos a, sin a) over a key range, as the renderers compute it
__global__ void k_unit_sincos(uint32_t key0, uint32_t n, float2* out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float c, s;
    glibc_sincosf_unit(unit_angle((key0 + i) & 0xFFFFFFu), c, s);
    out[i] = make_float2(c, s);
}

// ---------------------------------------------------------------- multi-device gather
// Frame assembly on the root device: the gathered tiles are [rank][max_rows][W]
// (equal-size padded blocks, as ncclGather delivers them); frame row y belongs
// to rank y % nd as its tile row y / nd (1-row bands dealt round-robin).
__global__ void k_assemble_rows(const uint32_t* __restrict__ gathered, int32_t nd, int32_t max_rows, int32_t W,
                                int32_t H, uint32_t* __restrict__ frame)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)W * H) return;
    const int32_t y = (int32_t)(i / W), x = (int32_t)(i - (int64_t)y * W);
    frame[i] = gathered[((int64_t)(y % nd) * max_rows + y / nd) * W + x];
}

// RCCL, resolved at run time (dlopen of librccl.so.1: in a process where torch
// already loaded its RCCL the same library is reused, so there is one RCCL and
// one HIP runtime; the library itself loads without RCCL).
struct Rccl {
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl& rccl()
{
    static Rccl r = []() {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
        x.comm_init_all = (decltype(x.comm_init_all))dlsym(h, "ncclCommInitAll");
        x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
        x.gather = (decltype(x.gather))dlsym(h, "ncclGather");
        x.reduce = (decltype(x.reduce))dlsym(h, "ncclReduce");
        x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
        x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        x.ok = x.comm_init_all && x.comm_destroy && x.gather && x.reduce && x.group_start && x.group_end &&
               x.error_string;
        return x;
    }();
    return r;
}

// ---------------------------------------------------------------- options
// The keys of include/tmpt.h "Scene options", in one table: name, build-time
// or not, range, and the member they set.
namespace {
struct OptionDef {
    const char* name;
    bool build;
    double lo, hi;
    int Options::*i;
    float Options::*f;
    double Options::*d;
};
const OptionDef kOptions[] = {
    {"builder", true, 0, 1, &Options::builder, nullptr, nullptr},
    {"layout", true, 0, 1, &Options::layout, nullptr, nullptr},
    {"leaf_max", true, 1, kLeafMaxTris, &Options::leaf_max, nullptr, nullptr},
    {"collapse", true, 0, 1, &Options::collapse, nullptr, nullptr},
    {"ploc_radius", true, 1, 256, &Options::ploc_radius, nullptr, nullptr},
    {"sah_c_leaf", true, 0, 1e6, nullptr, &Options::sah_c_leaf, nullptr},
    {"sah_c_tri", true, 0, 1e6, nullptr, &Options::sah_c_tri, nullptr},
    {"sample_block", false, 0, 1024, &Options::sample_block, nullptr, nullptr},
    {"sample_tail", false, -1, 64, &Options::sample_tail, nullptr, nullptr},
    {"sbuf_max", false, 0, 1e18, nullptr, nullptr, &Options::sbuf_max},
    {"sbuf_pair", false, 0, 1, &Options::sbuf_pair, nullptr, nullptr},
    {"pilot", false, -1, 512, &Options::pilot, nullptr, nullptr},
    {"help", false, -1, 1, &Options::help, nullptr, nullptr},
    {"pair", false, -1, 63, &Options::pair, nullptr, nullptr},
    {"balance", false, 0, 1, &Options::balance, nullptr, nullptr},
    {"dprio", false, 0, 1, &Options::dprio, nullptr, nullptr},
    {"wave_cap", false, 0, 64, &Options::wave_cap, nullptr, nullptr},
    {"pixel_chains", false, -1, 1024, &Options::pixel_chains, nullptr, nullptr},
    {"tie_defer", false, -1, 1, &Options::tie_defer, nullptr, nullptr},
    {"redo_cap", false, 0, 1 << 30, &Options::redo_cap, nullptr, nullptr},
    {"redo_inline", false, 0, 1, &Options::redo_inline, nullptr, nullptr},
    {"redo_lanes", false, 1, 64, &Options::redo_lanes, nullptr, nullptr},
    {"path_waves", false, 0, 5, &Options::path_waves, nullptr, nullptr},
    {"rowspec", false, 0, 1, &Options::rowspec, nullptr, nullptr},
    {"rowspec_wmax", false, 0, 16384, &Options::rowspec_wmax, nullptr, nullptr},
    {"rowspec_windows", false, 0, 32, &Options::rowspec_windows, nullptr, nullptr},
    {"rowspec_spread", false, -1, 100, nullptr, &Options::rowspec_spread, nullptr},
    {"rowspec_groups", false, 1, kRowSpecMaxGroups, &Options::rowspec_groups, nullptr, nullptr},
    {"rowspec_noshadow", false, 0, 1, &Options::rowspec_noshadow, nullptr, nullptr},
    {"rowspec_chase", false, 0, 1, &Options::rowspec_chase, nullptr, nullptr},
    {"rowspec_stream", false, 0, 1, &Options::rowspec_stream, nullptr, nullptr},
    {"rowstream_dynamic", false, 0, 1, &Options::rowstream_dynamic, nullptr, nullptr},
    {"row_flag_leaves", false, 0, 1, &Options::row_flag_leaves, nullptr, nullptr},
    {"row_occ", false, 0, 5, &Options::row_occ, nullptr, nullptr},
    {"wf_bins", false, 1, 8, &Options::wf_bins, nullptr, nullptr},
    {"rowstream_test_abort", false, 0, 1, &Options::rowstream_test_abort, nullptr, nullptr},
    {"tie_rule", false, 0, 1, &Options::tie_rule, nullptr, nullptr},
};

const OptionDef* find_option(const char* key)
{
    for (const OptionDef& d : kOptions)
        if (strcmp(d.name, key) == 0) return &d;
    return nullptr;
}
}  // namespace

int options_set(Options& o, const char* key, double v, bool allow_build)
{
    const OptionDef* d = key ? find_option(key) : nullptr;
    if (!d) {
        set_error(std::string("unknown option '") + (key ? key : "(null)") + "'");
        return -22;
    }
    if (d->build && !allow_build) {
        set_error(std::string("option '") + key + "' is a build option: give it to tmpt_scene_create_ex");
        return -22;
    }
    if (!(v >= d->lo && v <= d->hi)) {
        set_error(std::string("option '") + key + "' out of range [" + std::to_string(d->lo) + ", " +
                  std::to_string(d->hi) + "]");
        return -22;
    }
    if (d->i) {
        if (v != (double)(long long)v) {
            set_error(std::string("option '") + key + "' takes an integer");
            return -22;
        }
        if ((strcmp(key, "row_occ") == 0 || strcmp(key, "path_waves") == 0) && v != 0 && v != 4 && v != 5) {
            set_error(std::string("option '") + key + "' takes 0 (auto), 4 or 5");  // waves per SIMD
            return -22;
        }
        if ((strcmp(key, "sample_block") == 0 || strcmp(key, "wf_bins") == 0) && v > 0 &&
            ((long long)v & ((long long)v - 1)) != 0) {
            set_error(std::string("option '") + key + "' must be a power of two");
            return -22;
        }
        o.*(d->i) = (int)v;
    } else if (d->f) {
        o.*(d->f) = (float)v;
    } else {
        o.*(d->d) = v;
    }
    return 0;
}

int options_get(const Options& o, const char* key, double* v)
{
    const OptionDef* d = key ? find_option(key) : nullptr;
    if (!d) {
        set_error(std::string("unknown option '") + (key ? key : "(null)") + "'");
        return -22;
    }
    *v = d->i ? (double)(o.*(d->i)) : d->f ? (double)(o.*(d->f)) : o.*(d->d);
    return 0;
}

// "key=value,key=value" (spaces allowed); builder=ploc|lbvh and
// collapse=greedy|sah also take their names
int options_parse(Options& o, const char* text, bool allow_build)
{
    if (!text) return 0;
    std::string t(text);
    size_t pos = 0;
    while (pos <= t.size()) {
        size_t end = t.find(',', pos);
        if (end == std::string::npos) end = t.size();
        std::string item = t.substr(pos, end - pos);
        pos = end + 1;
        item.erase(0, item.find_first_not_of(" \t"));
        item.erase(item.find_last_not_of(" \t") + 1);
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos) {
            set_error("option '" + item + "' has no value (key=value)");
            return -22;
        }
        std::string key = item.substr(0, eq), val = item.substr(eq + 1);
        key.erase(key.find_last_not_of(" \t") + 1);
        val.erase(0, val.find_first_not_of(" \t"));
        if (key == "builder" && (val == "ploc" || val == "lbvh")) val = val == "lbvh" ? "1" : "0";
        if (key == "collapse" && (val == "greedy" || val == "sah")) val = val == "sah" ? "1" : "0";
        if (key == "tie_rule" && (val == "visit" || val == "index")) val = val == "index" ? "1" : "0";
        if (key == "layout" && (val == "aos" || val == "soa")) val = val == "soa" ? "1" : "0";
        char* endp = nullptr;
        const double v = strtod(val.c_str(), &endp);
        if (val.empty() || !endp || *endp != '\0') {
            set_error("option '" + key + "': bad value '" + val + "'");
            return -22;
        }
        if (int rc = options_set(o, key.c_str(), v, allow_build)) return rc;
    }
    return 0;
}

}  // namespace tmpt

struct tmpt_scene {
    tmpt::Scene s;
};

using namespace tmpt;

#define TMPT_GUARD_BEGIN try {
#define TMPT_GUARD_END                                  \
    }                                                   \
    catch (const std::bad_alloc&) {                     \
        set_error("out of host memory");                \
        return -1;                                      \
    }                                                   \
    catch (...) {                                       \
        set_error("unexpected C++ exception");          \
        return -1;                                      \
    }

namespace {
int bad(const char* msg)
{
    set_error(msg);
    return -22;
}
}  // namespace

extern "C" {

int tmpt_abi_version(void) { return TMPT_ABI_VERSION; }
const char* tmpt_last_error(void) { return last_error(); }
void tmpt_free(void* p) { free(p); }

int tmpt_unit_sincos(int32_t device, uint32_t key0, uint32_t n, float* out)
{
    TMPT_GUARD_BEGIN
    if (!out && n) return bad("tmpt_unit_sincos: null argument");
    if (n == 0) return 0;
    if (device < 0) {
        for (uint32_t i = 0; i < n; ++i)
            glibc_sincosf_unit(unit_angle((key0 + i) & 0xFFFFFFu), out[2 * (size_t)i], out[2 * (size_t)i + 1]);
        return 0;
    }
    int ndev = 0;
    TMPT_HIP(hipGetDeviceCount(&ndev));
    if (device >= ndev) return bad("tmpt_unit_sincos: no such device");
    TMPT_HIP(hipSetDevice(device));
    float2* d = nullptr;
    TMPT_HIP(hipMalloc(&d, sizeof(float2) * (size_t)n));
    k_unit_sincos<<<(n + 255u) / 256u, 256>>>(key0, n, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, d, sizeof(float2) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) {
        set_error(std::string("tmpt_unit_sincos: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
    TMPT_GUARD_END
}

int tmpt_load_obj(const char* path, float** out_tris, int32_t* out_n, float out_bmin[3],
                  float out_bmax[3])
{
    TMPT_GUARD_BEGIN
    if (!path || !out_tris || !out_n) return bad("tmpt_load_obj: null argument");
    std::vector<float> tris;
    f3 bmin, bmax;
    int rc = load_obj(path, tris, bmin, bmax);
    if (rc) return rc;
    float* p = (float*)malloc(tris.size() * sizeof(float));
    if (!p) return bad("tmpt_load_obj: out of memory");
    memcpy(p, tris.data(), tris.size() * sizeof(float));
    *out_tris = p;
    *out_n = (int32_t)(tris.size() / 9);
    if (out_bmin) { out_bmin[0] = bmin.x; out_bmin[1] = bmin.y; out_bmin[2] = bmin.z; }
    if (out_bmax) { out_bmax[0] = bmax.x; out_bmax[1] = bmax.y; out_bmax[2] = bmax.z; }
    return 0;
    TMPT_GUARD_END
}

int tmpt_camera_init(tmpt_camera* cam, const float lf[3], const float la[3], const float up[3],
                     float vfov, float aspect, float aperture, float focus_dist)
{
    if (!cam || !lf || !la || !up) return bad("tmpt_camera_init: null argument");
    camera_init(cam, mk(lf[0], lf[1], lf[2]), mk(la[0], la[1], la[2]), mk(up[0], up[1], up[2]),
                vfov, aspect, aperture, focus_dist);
    return 0;
}

int tmpt_camera_for_scene(tmpt_camera* cam, const float bmin[3], const float bmax[3],
                          int32_t width, int32_t height, int32_t is_sponza)
{
    if (!cam || !bmin || !bmax) return bad("tmpt_camera_for_scene: null argument");
    if (width < 1 || height < 1) return bad("tmpt_camera_for_scene: bad size");
    camera_for_scene(cam, mk(bmin[0], bmin[1], bmin[2]), mk(bmax[0], bmax[1], bmax[2]), width,
                     height, is_sponza != 0);
    return 0;
}

int tmpt_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int tmpt_scene_create(const float* tris, int32_t n, int32_t device, tmpt_scene** out)
{
    return tmpt_scene_create_ex(tris, n, device, nullptr, out);
}

int tmpt_scene_create_ex(const float* tris, int32_t n, int32_t device, const char* options, tmpt_scene** out)
{
    TMPT_GUARD_BEGIN
    if (!out || n < 0 || (n > 0 && !tris)) return bad("tmpt_scene_create: bad arguments");
    *out = nullptr;
    (void)hipGetLastError();  // a failed call before this one must not fail the build's checks
    Options opt;
    if (int rc = options_parse(opt, options, true)) {
        set_error(std::string("tmpt_scene_create: ") + last_error());
        return rc;
    }
    int ndev = 0;
    TMPT_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return bad("tmpt_scene_create: no such device");
    TMPT_HIP(hipSetDevice(device));
    tmpt_scene* h = new tmpt_scene();
    Scene& s = h->s;
    s.opt = opt;
    s.device = device;
    s.n = n;
    auto fail = [&](int rc) {
        tmpt_scene_destroy(h);
        return rc;
    };
    if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess)
        return fail((set_error("hipStreamCreate failed"), -1));
    float* d_tris = nullptr;
    if (n > 0) {
        if (hipMalloc(&d_tris, sizeof(float) * 9 * (size_t)n) != hipSuccess)
            return fail((set_error("tmpt_scene_create: out of device memory"), -1));
        if (hipMemcpy(d_tris, tris, sizeof(float) * 9 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d_tris);
            return fail((set_error("tmpt_scene_create: upload failed"), -1));
        }
    }
    // Scene::Scene's copy (scene.cpp:54-57): the octree's input, and the split references'
    s.tris_host.assign(tris, tris + 9 * (size_t)n);
    int rc = build_lbvh(s, d_tris);
    if (d_tris) (void)hipFree(d_tris);
    if (rc) return fail(rc);
    *out = h;
    return 0;
    TMPT_GUARD_END
}

int tmpt_scene_destroy(tmpt_scene* h)
{
    if (!h) return 0;
    Scene& s = h->s;
    (void)hipSetDevice(s.device);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    for (auto& st : s.rs_stream)  // the speculative row engine's group streams
        if (st) (void)hipStreamSynchronize(st);
    if (s.nodes4) (void)hipFree(s.nodes4);
    if (s.oct) (void)hipFree(s.oct);
    if (s.oct_refs) (void)hipFree(s.oct_refs);
    if (s.oct_view) (void)hipFree(s.oct_view);
    if (s.soa_buf) (void)hipFree(s.soa_buf);
    if (s.prog) (void)hipFree(s.prog);
    if (s.jt) (void)hipFree(s.jt);
    if (s.sbuf) (void)hipFree(s.sbuf);
    if (s.redo) (void)hipFree(s.redo);
    if (s.redo_state) (void)hipFree(s.redo_state);
    if (s.jt2) (void)hipFree(s.jt2);
    if (s.rs_buf) (void)hipFree(s.rs_buf);
    for (auto& st : s.rs_stream)
        if (st) (void)hipStreamDestroy(st);
    for (auto& ev : s.rs_event)
        if (ev) (void)hipEventDestroy(ev);
    if (s.rs_host) (void)hipHostFree(s.rs_host);
    if (s.rs_list) (void)hipFree(s.rs_list);
    if (s.rss_buf) (void)hipFree(s.rss_buf);
    if (s.rss_tab) (void)hipFree(s.rss_tab);
    if (s.rss_host) (void)hipHostFree(s.rss_host);
    if (s.wait_ev) (void)hipEventDestroy(s.wait_ev);
    if (s.counters) (void)hipFree(s.counters);
    if (s.chk) (void)hipFree(s.chk);
    if (s.counters_host) (void)hipHostFree(s.counters_host);
    for (auto e : s.render_ev)
        if (e) (void)hipEventDestroy(e);
    if (s.tri_pre) (void)hipFree(s.tri_pre);
    if (s.tri_orig) (void)hipFree(s.tri_orig);
    if (s.ws) (void)hipFree(s.ws);
    for (auto e : s.path_ev)
        if (e) (void)hipEventDestroy(e);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    delete h;
    return 0;
}

int tmpt_scene_build_octree(tmpt_scene* h, const float bmin[3], const float bmax[3])
{
    TMPT_GUARD_BEGIN
    if (!h || !bmin || !bmax) return bad("tmpt_scene_build_octree: null argument");
    Scene& s = h->s;
    if ((int64_t)s.tris_host.size() != 9 * (int64_t)s.n) return bad("tmpt_scene_build_octree: no triangle copy");
    TMPT_HIP(hipSetDevice(s.device));
    const auto t0 = std::chrono::steady_clock::now();
    OctreeHost t;
    build_octree(s.tris_host.data(), s.n, bmin, bmax, t);
    if (t.refs.size() >= (size_t)INT32_MAX || t.nodes.size() >= (size_t)INT32_MAX)
        return bad("tmpt_scene_build_octree: octree too large");
    OctNode* d_nodes = nullptr;
    int32_t* d_refs = nullptr;
    const size_t nb = t.nodes.size() * sizeof(OctNode), rb = std::max<size_t>(1, t.refs.size()) * sizeof(int32_t);
    if (hipMalloc(&d_nodes, nb) != hipSuccess || hipMalloc(&d_refs, rb) != hipSuccess ||
        hipMemcpy(d_nodes, t.nodes.data(), nb, hipMemcpyHostToDevice) != hipSuccess ||
        (t.refs.size() && hipMemcpy(d_refs, t.refs.data(), t.refs.size() * sizeof(int32_t), hipMemcpyHostToDevice) !=
                              hipSuccess)) {
        if (d_nodes) (void)hipFree(d_nodes);
        if (d_refs) (void)hipFree(d_refs);
        return (set_error("tmpt_scene_build_octree: out of device memory"), -1);
    }
    if (ensure_counters(s)) {
        (void)hipFree(d_nodes);
        (void)hipFree(d_refs);
        return -1;
    }
    if (s.stream) (void)hipStreamSynchronize(s.stream);  // a render in flight may still read the old one
    if (!s.oct_view && hipMalloc(&s.oct_view, sizeof(OctView)) != hipSuccess) {
        (void)hipFree(d_nodes);
        (void)hipFree(d_refs);
        return (set_error("tmpt_scene_build_octree: out of device memory"), -1);
    }
    // the crack grid and the flat triangles (tmpt_internal.h OctGrid), marked
    // in the BVH's triangle records so that a hit on one flags its query
    OctGrid grid;
    octree_grid(t, bmin, bmax, grid);
    std::vector<uint8_t> flat;
    const int32_t n_flat = octree_flat_triangles(s.tris_host.data(), s.n, grid, flat);
    if (mark_flat_triangles(s, flat)) {
        (void)hipFree(d_nodes);
        (void)hipFree(d_refs);
        return -1;
    }
    const OctView ov{d_nodes, d_refs, (int32_t)t.nodes.size(), n_flat, s.ties, grid, (int64_t)t.refs.size()};
    if (hipMemcpy(s.oct_view, &ov, sizeof(ov), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d_nodes);
        (void)hipFree(d_refs);
        // the previous octree (if any) stays in use: give the records back its
        // own flat marks (none without one), so marks and octree agree
        std::vector<uint8_t> old_flat((size_t)s.n, 0);
        if (s.oct) (void)octree_flat_triangles(s.tris_host.data(), s.n, s.oct_grid, old_flat);
        (void)mark_flat_triangles(s, old_flat);
        return (set_error("tmpt_scene_build_octree: upload failed"), -1);
    }
    if (s.oct) (void)hipFree(s.oct);
    if (s.oct_refs) (void)hipFree(s.oct_refs);
    s.oct = d_nodes;
    s.oct_refs = d_refs;
    s.n_oct = (int32_t)t.nodes.size();
    s.n_oct_refs = (int64_t)t.refs.size();
    s.oct_leaves = t.leaves;
    s.oct_depth = t.depth;
    s.oct_flat = n_flat;
    s.oct_grid = grid;
    for (int c = 0; c < 3; ++c) {
        s.oct_lo[c] = bmin[c];
        s.oct_hi[c] = bmax[c];
    }
    s.oct_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
    TMPT_GUARD_END
}

int tmpt_octree_bounds(const float bmin[3], const float bmax[3], float box[6])
{
    if (!bmin || !bmax || !box) return bad("tmpt_octree_bounds: null argument");
    const f3 lo = mk(bmin[0], bmin[1], bmin[2]), hi = mk(bmax[0], bmax[1], bmax[2]);
    const f3 extra = (hi - lo) * 0.7f;  // main.cpp:296-297
    const f3 a = lo - extra, b = hi + extra;  // main.cpp:312
    box[0] = a.x, box[1] = a.y, box[2] = a.z, box[3] = b.x, box[4] = b.y, box[5] = b.z;
    return 0;
}

int tmpt_octree_digest(const float* tris, int32_t n, const float bmin[3], const float bmax[3], uint64_t out[5])
{
    TMPT_GUARD_BEGIN
    if (n < 0 || (n > 0 && !tris) || !bmin || !bmax || !out) return bad("tmpt_octree_digest: bad arguments");
    OctreeHost t;
    build_octree(tris, n, bmin, bmax, t);
    out[0] = t.nodes.size();
    out[1] = (uint64_t)t.leaves;
    out[2] = t.refs.size() - (uint64_t)t.leaves;  // triangle references (the count words excluded)
    out[3] = (uint64_t)t.depth;
    out[4] = octree_digest(t);
    return 0;
    TMPT_GUARD_END
}

int tmpt_octree_flags(const float* tris, int32_t n, const float bmin[3], const float bmax[3], const float* rays,
                      const float* t, const int32_t* ids, int64_t n_rays, uint8_t* flags, float grid[13])
{
    TMPT_GUARD_BEGIN
    if (n < 0 || (n > 0 && !tris) || !bmin || !bmax || n_rays < 0 || (n_rays > 0 && (!rays || !t || !ids || !flags)))
        return bad("tmpt_octree_flags: bad arguments");
    OctreeHost oh;
    build_octree(tris, n, bmin, bmax, oh);
    OctGrid g;
    octree_grid(oh, bmin, bmax, g);
    std::vector<uint8_t> flat;
    octree_flat_triangles(tris, n, g, flat);
    for (int64_t i = 0; i < n_rays; ++i) {
        const float* r = rays + 6 * i;
        const int32_t id = ids[i];
        uint8_t f = 0;
        if (id >= 0 && id < n)
            f = (uint8_t)(flat[(size_t)id] | (octree_crack(g, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), t[i]) ? 2 : 0));
        flags[i] = f;
    }
    if (grid) {
        for (int k = 0; k < 3; ++k) {
            grid[k] = g.r0[k];
            grid[3 + k] = g.inv_cell[k];
            grid[6 + k] = g.cell[k];
            grid[9 + k] = g.band[k];
        }
        grid[12] = g.reach;
    }
    return 0;
    TMPT_GUARD_END
}

int tmpt_scene_set_option(tmpt_scene* h, const char* key, double value)
{
    TMPT_GUARD_BEGIN
    if (!h) return bad("tmpt_scene_set_option: null scene");
    return options_set(h->s.opt, key, value, false);
    TMPT_GUARD_END
}

int tmpt_scene_get_option(const tmpt_scene* h, const char* key, double* value)
{
    TMPT_GUARD_BEGIN
    if (!h || !value) return bad("tmpt_scene_get_option: null argument");
    return options_get(h->s.opt, key, value);
    TMPT_GUARD_END
}

namespace {
// the batched HitScene: stride 6 (one range) or 8 (per-ray tmin, tmax)
int scene_hit(const tmpt_scene* hc, const float* rays, int64_t n, float tmin, float tmax, bool ranged,
              int32_t any_hit, float* hits, int32_t* ids)
{
    if (!hc || n < 0 || (n > 0 && (!rays || !hits || !ids))) return bad("tmpt_scene_hit: bad arguments");
    if (n == 0) return 0;
    const size_t rs = ranged ? 32 : 24;
    Scene& s = const_cast<tmpt_scene*>(hc)->s;
    TMPT_HIP(hipSetDevice(s.device));
    float *d_rays = nullptr, *d_hits = nullptr;
    int32_t* d_ids = nullptr;
    auto cleanup = [&]() {
        if (d_rays) (void)hipFree(d_rays);
        if (d_hits) (void)hipFree(d_hits);
        if (d_ids) (void)hipFree(d_ids);
    };
    if (hipMalloc(&d_rays, rs * (size_t)n) != hipSuccess || hipMalloc(&d_hits, 28 * (size_t)n) != hipSuccess ||
        hipMalloc(&d_ids, 4 * (size_t)n) != hipSuccess) {
        cleanup();
        return bad("tmpt_scene_hit: out of device memory");
    }
    int rc = 0;
    if (hipMemcpy(d_rays, rays, rs * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_hits, hits, 28 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess)
        rc = (set_error("tmpt_scene_hit: upload failed"), -1);
    if (!rc) rc = intersect_batch(s, d_rays, n, tmin, tmax, any_hit != 0, ranged, d_hits, d_ids);
    if (!rc && (hipStreamSynchronize(s.stream) != hipSuccess ||
                hipMemcpy(hits, d_hits, 28 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(ids, d_ids, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = (set_error("tmpt_scene_hit: kernel or readback failed"), -1);
    if (!rc) {
        s.tie_queries = s.counters_host[kTieCounter];
        s.root_misses = s.counters_host[kTieCounter + 1];
        s.crack_queries = s.counters_host[kCrackCounter];
    }
    if (!rc) rc = check_report(s, "tmpt_scene_hit");
    cleanup();
    return rc;
}
}  // namespace

int tmpt_scene_hit(const tmpt_scene* hc, const float* rays, int64_t n, float tmin, float tmax,
                   int32_t any_hit, float* hits, int32_t* ids)
{
    TMPT_GUARD_BEGIN
    return scene_hit(hc, rays, n, tmin, tmax, false, any_hit, hits, ids);
    TMPT_GUARD_END
}

int tmpt_scene_hit_ranged(const tmpt_scene* hc, const float* rays8, int64_t n, int32_t any_hit, float* hits,
                          int32_t* ids)
{
    TMPT_GUARD_BEGIN
    return scene_hit(hc, rays8, n, 0.0f, 0.0f, true, any_hit, hits, ids);
    TMPT_GUARD_END
}

int32_t tmpt_tile_rows(const tmpt_render_desc* d)
{
    if (!d || d->height < 1) return 0;
    int band = d->band_rows > 0 ? d->band_rows : d->height;
    int ns = d->num_shards > 1 ? d->num_shards : 1;
    int sh = ns > 1 ? d->shard : 0;
    int nbands = (d->height + band - 1) / band;
    int rows = 0;
    for (int b = sh; b < nbands; b += ns) rows += std::min(band, d->height - b * band);
    return rows;
}

int32_t tmpt_tile_row_to_y(const tmpt_render_desc* d, int32_t r)
{
    int band = d->band_rows > 0 ? d->band_rows : d->height;
    int ns = d->num_shards > 1 ? d->num_shards : 1;
    int sh = ns > 1 ? d->shard : 0;
    int lb = r / band;
    return (lb * ns + sh) * band + (r - lb * band);
}

int tmpt_render(tmpt_scene* h, const tmpt_camera* cam, const tmpt_render_desc* d,
                uint8_t* rgba_out, uint64_t* ray_count)
{
    TMPT_GUARD_BEGIN
    if (!h || !cam || !d || !rgba_out) return bad("tmpt_render: null argument");
    // main.cpp:258-280 argument ranges
    if (d->width < 1 || d->width > 10000) return bad("tmpt_render: invalid width");
    if (d->height < 1 || d->height > 10000) return bad("tmpt_render: invalid height");
    if (d->spp < 1 || d->spp > 1024) return bad("tmpt_render: invalid samplesPerPixel");
    if (d->seed_mode != TMPT_SEED_ROW && d->seed_mode != TMPT_SEED_PIXEL && d->seed_mode != TMPT_SEED_SAMPLE)
        return bad("tmpt_render: invalid seed_mode");
    if (d->engine != TMPT_ENGINE_WAVEFRONT && d->engine != TMPT_ENGINE_MEGAKERNEL &&
        d->engine != TMPT_ENGINE_PERSISTENT)
        return bad("tmpt_render: invalid engine");
    if (d->num_shards > 1 && (d->shard < 0 || d->shard >= d->num_shards))
        return bad("tmpt_render: invalid shard");
    if (d->spp_begin < 0 || d->spp_begin >= d->spp || d->spp_count < 0 ||
        d->spp_count > d->spp - d->spp_begin)
        return bad("tmpt_render: invalid spp_begin / spp_count");
    const bool progressive = d->spp_begin > 0 || (d->spp_count > 0 && d->spp_count < d->spp);
    if (progressive && (d->engine != TMPT_ENGINE_PERSISTENT || d->seed_mode == TMPT_SEED_ROW))
        return bad("tmpt_render: progressive spp needs the persistent engine and pixel or sample seeding");
    (void)hipGetLastError();  // clear a stale error of an earlier failed call (launch checks read it)
    Scene& s = h->s;
    TMPT_HIP(hipSetDevice(s.device));
    const int32_t rows = tmpt_tile_rows(d);
    const size_t bytes = (size_t)rows * (size_t)d->width * 4;
    const bool dev_out = (d->flags & TMPT_FLAG_OUT_DEVICE) != 0;
    uint32_t* d_out = nullptr;
    if (dev_out) d_out = (uint32_t*)rgba_out;
    else if (bytes && hipMalloc(&d_out, bytes) != hipSuccess) return bad("tmpt_render: out of device memory");
    int rc = render(s, cam, d, d_out, ray_count);
    if (!rc) rc = check_report(s, "tmpt_render");
    if (!rc && !dev_out && bytes) {
        if (hipMemcpy(rgba_out, d_out, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            rc = (set_error("tmpt_render: readback failed"), -1);
    }
    if (!dev_out && d_out) (void)hipFree(d_out);
    return rc;
    TMPT_GUARD_END
}

int tmpt_render_multi(const float* tris, int32_t n, const float* octree_box, const tmpt_camera* cam,
                      const tmpt_render_desc* desc, const int32_t* devices, int32_t ndevices, uint8_t* rgba_full,
                      uint64_t* ray_count, double* seconds)
{
    TMPT_GUARD_BEGIN
    if (!cam || !desc || !devices || ndevices < 1 || !rgba_full || (n > 0 && !tris))
        return bad("tmpt_render_multi: bad arguments");
    if (desc->width < 1 || desc->width > 10000 || desc->height < 1 || desc->height > 10000)
        return bad("tmpt_render_multi: invalid width / height");
    const int nd = ndevices;
    const int W = desc->width, H = desc->height;
    bool unique = true;
    for (int g = 0; g < nd; ++g)
        for (int k = 0; k < g; ++k) unique = unique && devices[g] != devices[k];
    const bool use_rccl = unique && rccl().ok;
    if ((desc->flags & TMPT_FLAG_REQUIRE_RCCL) && !use_rccl)
        return bad(unique ? "tmpt_render_multi: RCCL (librccl.so.1) not available"
                          : "tmpt_render_multi: RCCL needs distinct devices (a device is listed twice)");
    std::vector<tmpt_scene*> scenes((size_t)nd, nullptr);
    std::vector<int> rcs((size_t)nd, 0);
    std::vector<std::string> errs((size_t)nd);
    // per rank: its padded tile and ray count on its device; on rank 0 also the
    // gathered tiles, the frame and the summed count
    const int max_rows = (H + nd - 1) / nd;
    const size_t tile_bytes = (size_t)max_rows * (size_t)W * 4;
    std::vector<uint8_t*> d_tile((size_t)nd, nullptr);
    std::vector<uint64_t*> d_rays((size_t)nd, nullptr);
    std::vector<hipStream_t> streams((size_t)nd, nullptr);
    uint8_t* d_gather = nullptr;
    uint32_t* d_frame = nullptr;
    uint64_t* d_total = nullptr;
    std::vector<ncclComm_t> comms;
    auto cleanup = [&]() {  // touches only devices whose resources exist (a bad ordinal is never set)
        for (int g = 0; g < nd; ++g)
            if (streams[(size_t)g]) {
                (void)hipSetDevice(devices[g]);
                (void)hipStreamSynchronize(streams[(size_t)g]);
            }
        for (ncclComm_t c : comms)
            if (c) (void)rccl().comm_destroy(c);
        for (int g = 0; g < nd; ++g) {
            if (!streams[(size_t)g] && !d_tile[(size_t)g] && !d_rays[(size_t)g]) continue;
            (void)hipSetDevice(devices[g]);
            if (d_tile[(size_t)g]) (void)hipFree(d_tile[(size_t)g]);
            if (d_rays[(size_t)g]) (void)hipFree(d_rays[(size_t)g]);
            if (streams[(size_t)g]) (void)hipStreamDestroy(streams[(size_t)g]);
        }
        if (d_gather || d_frame || d_total) {
            (void)hipSetDevice(devices[0]);
            if (d_gather) (void)hipFree(d_gather);
            if (d_frame) (void)hipFree(d_frame);
            if (d_total) (void)hipFree(d_total);
        }
        for (auto* sc : scenes) tmpt_scene_destroy(sc);
        (void)hipGetLastError();  // leave no sticky error behind for this thread's next call
    };
    auto fail = [&](const std::string& msg, int rc) {
        cleanup();
        set_error("tmpt_render_multi: " + msg);
        return rc;
    };
    {  // scene per device, concurrently (error text is thread-local: keep each thread's)
        std::vector<std::thread> th;
        for (int g = 0; g < nd; ++g)
            th.emplace_back([&, g]() {
                rcs[(size_t)g] = tmpt_scene_create(tris, n, devices[g], &scenes[(size_t)g]);
                if (!rcs[(size_t)g] && octree_box)  // main.cpp:312
                    rcs[(size_t)g] = tmpt_scene_build_octree(scenes[(size_t)g], octree_box, octree_box + 3);
                if (rcs[(size_t)g]) errs[(size_t)g] = tmpt_last_error();
            });
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < nd; ++g)
        if (rcs[(size_t)g]) return fail(errs[(size_t)g], rcs[(size_t)g]);
    for (int g = 0; g < nd; ++g) {
        if (hipSetDevice(devices[g]) != hipSuccess || hipStreamCreateWithFlags(&streams[(size_t)g], hipStreamNonBlocking) ||
            hipMalloc(&d_tile[(size_t)g], tile_bytes) != hipSuccess ||
            hipMalloc(&d_rays[(size_t)g], sizeof(uint64_t)) != hipSuccess ||
            hipMemsetAsync(d_tile[(size_t)g], 0, tile_bytes, streams[(size_t)g]) != hipSuccess)
            return fail("out of device memory", -1);
    }
    if (hipSetDevice(devices[0]) != hipSuccess || hipMalloc(&d_gather, tile_bytes * (size_t)nd) != hipSuccess ||
        hipMalloc(&d_frame, (size_t)W * H * 4) != hipSuccess || hipMalloc(&d_total, sizeof(uint64_t)) != hipSuccess)
        return fail("out of device memory (root)", -1);
    if (use_rccl) {  // single-process form of SURVEY.md §8e: one communicator per device
        comms.assign((size_t)nd, nullptr);
        const ncclResult_t r = rccl().comm_init_all(comms.data(), nd, devices);
        if (r != ncclSuccess) {
            comms.clear();
            return fail(std::string("ncclCommInitAll: ") + rccl().error_string(r), -1);
        }
    }
    for (int g = 0; g < nd; ++g) (void)hipStreamSynchronize(streams[(size_t)g]);
    std::vector<tmpt_render_desc> ds((size_t)nd, *desc);
    std::vector<uint64_t> rays((size_t)nd, 0);
    const auto t0 = std::chrono::steady_clock::now();
    {  // every device renders its rows into its device tile, one host thread each
        std::vector<std::thread> th;
        for (int g = 0; g < nd; ++g)
            th.emplace_back([&, g]() {
                tmpt_render_desc& d = ds[(size_t)g];
                d.band_rows = 1;  // rows dealt round-robin: statistically equal shards
                d.shard = g;
                d.num_shards = nd;
                d.flags = TMPT_FLAG_OUT_DEVICE;
                rcs[(size_t)g] = tmpt_render(scenes[(size_t)g], cam, &d, d_tile[(size_t)g], &rays[(size_t)g]);
                if (rcs[(size_t)g]) errs[(size_t)g] = tmpt_last_error();
                else if (hipSetDevice(devices[g]) != hipSuccess ||
                         hipMemcpyAsync(d_rays[(size_t)g], &rays[(size_t)g], sizeof(uint64_t), hipMemcpyHostToDevice,
                                        streams[(size_t)g]) != hipSuccess ||
                         hipStreamSynchronize(streams[(size_t)g]) != hipSuccess)
                    rcs[(size_t)g] = -1, errs[(size_t)g] = "ray count upload failed";
            });
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < nd; ++g)
        if (rcs[(size_t)g]) return fail(errs[(size_t)g], rcs[(size_t)g]);
    uint64_t total = 0;
    if (use_rccl) {
        // ONE gather of the equal-size padded tiles to device 0 over xGMI and a
        // uint64 sum of the ray counts, grouped (one thread drives every device)
        ncclResult_t r = rccl().group_start();
        for (int g = 0; g < nd && r == ncclSuccess; ++g) {
            r = rccl().gather(d_tile[(size_t)g], g == 0 ? d_gather : nullptr, tile_bytes, ncclUint8, 0,
                              comms[(size_t)g], streams[(size_t)g]);
            if (r == ncclSuccess)
                r = rccl().reduce(d_rays[(size_t)g], g == 0 ? d_total : nullptr, 1, ncclUint64, ncclSum, 0,
                                  comms[(size_t)g], streams[(size_t)g]);
        }
        const ncclResult_t re = rccl().group_end();
        if (r == ncclSuccess) r = re;
        if (r != ncclSuccess) return fail(std::string("RCCL gather: ") + rccl().error_string(r), -1);
        for (int g = 0; g < nd; ++g)
            if (hipSetDevice(devices[g]) != hipSuccess || hipStreamSynchronize(streams[(size_t)g]) != hipSuccess)
                return fail("gather failed", -1);
        (void)hipSetDevice(devices[0]);
        if (hipMemcpy(&total, d_total, sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
            return fail("ray count readback failed", -1);
    } else {
        // a device listed more than once (RCCL ranks need distinct devices):
        // the same gather as device-to-device copies into the root's buffer
        (void)hipSetDevice(devices[0]);
        for (int g = 0; g < nd; ++g) {
            if (hipMemcpyPeerAsync(d_gather + (size_t)g * tile_bytes, devices[0], d_tile[(size_t)g], devices[g],
                                   tile_bytes, streams[0]) != hipSuccess)
                return fail("device-to-device gather failed", -1);
            total += rays[(size_t)g];
        }
    }
    (void)hipSetDevice(devices[0]);
    k_assemble_rows<<<(unsigned)(((int64_t)W * H + 255) / 256), 256, 0, streams[0]>>>(
        reinterpret_cast<const uint32_t*>(d_gather), nd, max_rows, W, H, d_frame);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(streams[0]) != hipSuccess)
        return fail("frame assembly failed", -1);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (hipMemcpy(rgba_full, d_frame, (size_t)W * H * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("frame readback failed", -1);
    cleanup();
    if (ray_count) *ray_count = total;
    if (seconds) *seconds = dt;
    return 0;
    TMPT_GUARD_END
}

int tmpt_get_stats(const tmpt_scene* h, tmpt_stats* o)
{
    if (!h || !o) return bad("tmpt_get_stats: null argument");
    const Scene& s = h->s;
    memset(o, 0, sizeof(*o));
    o->render_ms = s.render_ms;
    o->extend_ms = s.extend_ms;
    o->shadow_ms = s.shadow_ms;
    o->extend_rays = s.extend_rays;
    o->shadow_rays = s.shadow_rays;
    o->extend_launches = s.extend_launches;
    o->shadow_launches = s.shadow_launches;
    o->iterations = s.iterations;
    o->node_visits = s.node_visits;
    o->tri_tests = s.tri_tests;
    o->shadow_node_visits = s.shadow_node_visits;
    o->shadow_tri_tests = s.shadow_tri_tests;
    o->build_ms = s.build_ms;
    o->bvh_nodes = s.n_nodes;
    o->bvh_depth = s.max_depth;
    o->n_tris = s.n;
    o->device = s.device;
    o->bvh4_nodes = s.n_nodes4;
    o->bvh4_depth = s.depth4;
    o->leaf_max = s.leaf_max;
    o->builder_iters = s.ploc_iters;
    o->octree_nodes = s.n_oct;
    o->octree_leaves = s.oct_leaves;
    o->octree_refs = s.n_oct ? s.n_oct_refs - s.oct_leaves : 0;
    o->octree_build_ms = s.oct_build_ms;
    o->tie_queries = s.tie_queries;
    o->root_misses = s.root_misses;
    o->row_engine = s.row_engine;
    o->stream_fallbacks = s.stream_fallbacks;
    o->octree_depth = s.oct_depth;
    o->tie_rule = s.oct && s.opt.tie_rule == 0 ? 0 : 1;
    o->chain_pixels = s.chain_pixels;
    o->redo_samples = s.redo_samples;
    o->redo_late = s.redo_late;
    o->crack_queries = s.crack_queries;
    o->octree_flat = s.oct ? s.oct_flat : 0;
    o->redo_launches = s.redo_launches;
    o->redo_ms = s.redo_ms;
    o->redo_rays = s.redo_rays;
    o->tie_path = s.tie_path;
    o->reserved_stats = 0;
    return 0;
}

int tmpt_write_png(const char* path, const uint8_t* rgba, int32_t w, int32_t h)
{
    TMPT_GUARD_BEGIN
    if (!path || !rgba || w < 1 || h < 1) return bad("tmpt_write_png: bad arguments");
    return write_png(path, rgba, w, h);
    TMPT_GUARD_END
}

}  // extern "C"
