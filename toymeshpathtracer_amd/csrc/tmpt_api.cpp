// tmpt_api.cpp -- the C ABI of include/tmpt.h.  Status ints cross the
// boundary; no exception escapes (every entry point catches).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "tmpt.h"
#include "tmpt_internal.h"

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
int intersect_batch(Scene& s, const float* d_rays, int64_t n, float tmin, float tmax, bool any,
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
    TMPT_GUARD_BEGIN
    if (!out || n < 0 || (n > 0 && !tris)) return bad("tmpt_scene_create: bad arguments");
    *out = nullptr;
    int ndev = 0;
    TMPT_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return bad("tmpt_scene_create: no such device");
    TMPT_HIP(hipSetDevice(device));
    tmpt_scene* h = new tmpt_scene();
    Scene& s = h->s;
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
    int rc = build_lbvh(s, d_tris);
    if (d_tris) (void)hipFree(d_tris);
    if (rc) return fail(rc);
    {
        auto t0 = std::chrono::steady_clock::now();
        rc = build_shadow_grid(s, tris);
        if (rc) return fail(rc);
        s.build_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
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
    if (s.nodes) (void)hipFree(s.nodes);
    if (s.nodes4) (void)hipFree(s.nodes4);
    if (s.nodes4f) (void)hipFree(s.nodes4f);
    if (s.prog) (void)hipFree(s.prog);
    if (s.jt) (void)hipFree(s.jt);
    if (s.sbuf) (void)hipFree(s.sbuf);
    if (s.jt2) (void)hipFree(s.jt2);
    if (s.rs_buf) (void)hipFree(s.rs_buf);
    for (auto& st : s.rs_stream)
        if (st) (void)hipStreamDestroy(st);
    for (auto& ev : s.rs_event)
        if (ev) (void)hipEventDestroy(ev);
    if (s.rs_host) (void)hipHostFree(s.rs_host);
    if (s.rs_list) (void)hipFree(s.rs_list);
    free_shadow_grid(s);
    if (s.tri_pre) (void)hipFree(s.tri_pre);
    if (s.tri_orig) (void)hipFree(s.tri_orig);
    if (s.ws) (void)hipFree(s.ws);
    for (auto e : s.path_ev)
        if (e) (void)hipEventDestroy(e);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    delete h;
    return 0;
}

int tmpt_scene_hit(const tmpt_scene* hc, const float* rays, int64_t n, float tmin, float tmax,
                   int32_t any_hit, float* hits, int32_t* ids)
{
    TMPT_GUARD_BEGIN
    if (!hc || n < 0 || (n > 0 && (!rays || !hits || !ids))) return bad("tmpt_scene_hit: bad arguments");
    if (n == 0) return 0;
    Scene& s = const_cast<tmpt_scene*>(hc)->s;
    TMPT_HIP(hipSetDevice(s.device));
    float *d_rays = nullptr, *d_hits = nullptr;
    int32_t* d_ids = nullptr;
    auto cleanup = [&]() {
        if (d_rays) (void)hipFree(d_rays);
        if (d_hits) (void)hipFree(d_hits);
        if (d_ids) (void)hipFree(d_ids);
    };
    if (hipMalloc(&d_rays, 24 * (size_t)n) != hipSuccess || hipMalloc(&d_hits, 28 * (size_t)n) != hipSuccess ||
        hipMalloc(&d_ids, 4 * (size_t)n) != hipSuccess) {
        cleanup();
        return bad("tmpt_scene_hit: out of device memory");
    }
    int rc = 0;
    if (hipMemcpy(d_rays, rays, 24 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_hits, hits, 28 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess)
        rc = (set_error("tmpt_scene_hit: upload failed"), -1);
    if (!rc) rc = intersect_batch(s, d_rays, n, tmin, tmax, any_hit != 0, d_hits, d_ids);
    if (!rc && (hipStreamSynchronize(s.stream) != hipSuccess ||
                hipMemcpy(hits, d_hits, 28 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(ids, d_ids, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = (set_error("tmpt_scene_hit: kernel or readback failed"), -1);
    cleanup();
    return rc;
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
    if (progressive && (d->engine != TMPT_ENGINE_PERSISTENT || d->seed_mode != TMPT_SEED_PIXEL))
        return bad("tmpt_render: progressive spp needs the persistent engine and pixel seeding");
    Scene& s = h->s;
    TMPT_HIP(hipSetDevice(s.device));
    const int32_t rows = tmpt_tile_rows(d);
    const size_t bytes = (size_t)rows * (size_t)d->width * 4;
    const bool dev_out = (d->flags & TMPT_FLAG_OUT_DEVICE) != 0;
    uint32_t* d_out = nullptr;
    if (dev_out) d_out = (uint32_t*)rgba_out;
    else if (bytes && hipMalloc(&d_out, bytes) != hipSuccess) return bad("tmpt_render: out of device memory");
    int rc = render(s, cam, d, d_out, ray_count);
    if (!rc && !dev_out && bytes) {
        if (hipMemcpy(rgba_out, d_out, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            rc = (set_error("tmpt_render: readback failed"), -1);
    }
    if (!dev_out && d_out) (void)hipFree(d_out);
    return rc;
    TMPT_GUARD_END
}

int tmpt_render_multi(const float* tris, int32_t n, const tmpt_camera* cam, const tmpt_render_desc* desc,
                      const int32_t* devices, int32_t ndevices, uint8_t* rgba_full, uint64_t* ray_count,
                      double* seconds)
{
    TMPT_GUARD_BEGIN
    if (!cam || !desc || !devices || ndevices < 1 || !rgba_full || (n > 0 && !tris))
        return bad("tmpt_render_multi: bad arguments");
    const int nd = ndevices;
    std::vector<tmpt_scene*> scenes((size_t)nd, nullptr);
    std::vector<int> rcs((size_t)nd, 0);
    std::vector<std::string> errs((size_t)nd);
    auto destroy_all = [&]() {
        for (auto* sc : scenes) tmpt_scene_destroy(sc);
    };
    {  // scene per device, concurrently (error text is thread-local: keep each thread's)
        std::vector<std::thread> th;
        for (int g = 0; g < nd; ++g)
            th.emplace_back([&, g]() {
                rcs[(size_t)g] = tmpt_scene_create(tris, n, devices[g], &scenes[(size_t)g]);
                if (rcs[(size_t)g]) errs[(size_t)g] = tmpt_last_error();
            });
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < nd; ++g)
        if (rcs[(size_t)g]) {
            destroy_all();
            return (set_error("tmpt_render_multi: " + errs[(size_t)g]), rcs[(size_t)g]);
        }
    std::vector<tmpt_render_desc> ds((size_t)nd, *desc);
    std::vector<std::vector<uint8_t>> tiles((size_t)nd);
    std::vector<uint64_t> rays((size_t)nd, 0);
    for (int g = 0; g < nd; ++g) {
        tmpt_render_desc& d = ds[(size_t)g];
        d.band_rows = nd > 1 ? 1 : desc->band_rows;  // rows dealt round-robin: balanced shards
        d.shard = g;
        d.num_shards = nd;
        d.flags = 0;
        tiles[(size_t)g].resize((size_t)std::max(0, tmpt_tile_rows(&d)) * (size_t)std::max(0, d.width) * 4);
    }
    const auto t0 = std::chrono::steady_clock::now();
    {
        std::vector<std::thread> th;
        for (int g = 0; g < nd; ++g)
            th.emplace_back([&, g]() {
                rcs[(size_t)g] = tmpt_render(scenes[(size_t)g], cam, &ds[(size_t)g], tiles[(size_t)g].data(),
                                             &rays[(size_t)g]);
                if (rcs[(size_t)g]) errs[(size_t)g] = tmpt_last_error();
            });
        for (auto& t : th) t.join();
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t total = 0;
    for (int g = 0; g < nd; ++g) {
        if (rcs[(size_t)g]) {
            destroy_all();
            return (set_error("tmpt_render_multi: " + errs[(size_t)g]), rcs[(size_t)g]);
        }
        total += rays[(size_t)g];
        const tmpt_render_desc& d = ds[(size_t)g];
        const int rows = tmpt_tile_rows(&d);
        for (int r = 0; r < rows; ++r) {
            const int y = tmpt_tile_row_to_y(&d, r);
            memcpy(rgba_full + (size_t)y * d.width * 4, tiles[(size_t)g].data() + (size_t)r * d.width * 4,
                   (size_t)d.width * 4);
        }
    }
    destroy_all();
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
