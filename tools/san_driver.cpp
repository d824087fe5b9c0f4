// san_driver.cpp -- the library's threaded host paths and the oracle's threads
// in one program, for ThreadSanitizer (and ASan + UBSan) builds
// (tools/san_check.sh).  Every threaded path is run with
// several threads and small work pieces, and its result checked against the
// same path run on one thread (or against the oracle):
//   * OBJ ingest (tmpt_host.cpp load_obj): text cut into chunks parsed on
//     their own threads, merged in file order -- vs one thread, vs the oracle
//   * PNG encode (write_png): strips filtered and deflated on threads into one
//     zlib stream (the decode check is tests/test_host.py's; here the threads run)
//   * the reference's octree (tmpt_octree.cpp build_octree): the root's 8
//     subtrees on 8 threads, spliced -- vs the oracle's octree (digest)
//   * the crack grid and flat triangles of that octree (host code only)
//   * the oracle's pthreads: batched HitScene and the row-parallel render, on
//     1 and 8 threads -- the same answers and pixels
// Exit status 0 = every check passed (the sanitizers abort on their own finds).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "tmpt_internal.h"

extern "C" {
#include "../oracle/tmpt_oracle.h"
}

namespace tmpt {
// the library's host functions (tmpt_host.cpp); set_error lives in tmpt_api.cpp
int load_obj(const char* path, std::vector<float>& tris, f3& bmin, f3& bmax);
int write_png(const char* path, const uint8_t* rgba, int w, int h);
static std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace tmpt

static int g_fail = 0;
#define CHECK(c, ...)                                     \
    do {                                                  \
        if (!(c)) {                                       \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fprintf(stderr, "\n");                        \
            ++g_fail;                                     \
        }                                                 \
    } while (0)

static std::vector<uint8_t> slurp(const char* path)
{
    std::vector<uint8_t> b;
    FILE* f = fopen(path, "rb");
    if (!f) return b;
    fseek(f, 0, SEEK_END);
    b.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
    fclose(f);
    return b;
}

int main(int argc, char** argv)
{
    const std::string data = argc > 1 ? argv[1] : "data";
    const char* scenes[] = {"cube.obj", "suzanne.obj", "teapot.obj", "generated/standin_sponza.obj"};
    for (const char* name : scenes) {
        const std::string path = data + "/" + name;
        if (!slurp(path.c_str()).size()) {
            printf("skip %s (absent)\n", name);
            continue;
        }
        // ---- OBJ ingest: 8 threads over 4-KB chunks vs 1 thread vs the oracle
        std::vector<float> t1, t8;
        tmpt::f3 lo1, hi1, lo8, hi8;
        setenv("TMPT_OBJ_THREADS", "1", 1);
        CHECK(tmpt::load_obj(path.c_str(), t1, lo1, hi1) == 0, "load_obj %s", name);
        setenv("TMPT_OBJ_THREADS", "8", 1);
        setenv("TMPT_OBJ_CHUNK", "4096", 1);
        CHECK(tmpt::load_obj(path.c_str(), t8, lo8, hi8) == 0, "load_obj threads %s", name);
        CHECK(t1 == t8 && !memcmp(&lo1, &lo8, sizeof lo1) && !memcmp(&hi1, &hi8, sizeof hi1), "OBJ threads %s", name);
        float* ot = nullptr;
        int32_t on = 0;
        float obmin[3], obmax[3];
        CHECK(orc_load_scene(path.c_str(), &ot, &on, obmin, obmax) == 0, "oracle load %s", name);
        CHECK((size_t)on * 9 == t1.size() && !memcmp(ot, t1.data(), t1.size() * 4), "OBJ vs oracle %s", name);
        const int32_t n = (int32_t)(t1.size() / 9);

        // ---- the reference's octree on 8 threads vs the oracle's
        const float bmin[3] = {lo1.x, lo1.y, lo1.z}, bmax[3] = {hi1.x, hi1.y, hi1.z};
        float omin[3], omax[3];
        for (int k = 0; k < 3; ++k) {  // main.cpp:296-297,312
            const float e = (bmax[k] - bmin[k]) * 0.7f;
            omin[k] = bmin[k] - e;
            omax[k] = bmax[k] + e;
        }
        tmpt::OctreeHost oh;
        tmpt::build_octree(t1.data(), n, omin, omax, oh);
        orc_scene* os = orc_scene_create(t1.data(), n, ORC_ACCEL_OCTREE, ORC_TIE_VISIT, omin, omax);
        CHECK(tmpt::octree_digest(oh) == orc_octree_digest(os), "octree digest %s", name);
        tmpt::OctGrid g;
        tmpt::octree_grid(oh, omin, omax, g);
        std::vector<uint8_t> flat;
        const int32_t nflat = tmpt::octree_flat_triangles(t1.data(), n, g, flat);
        CHECK(nflat >= 0 && (int32_t)flat.size() == n, "flat %s", name);

        // ---- the oracle's threads: batched HitScene and a render, 1 vs 8 threads
        const int64_t nr = 20000;
        std::vector<float> rays((size_t)nr * 6), h1((size_t)nr * 7), h8((size_t)nr * 7);
        std::vector<int32_t> i1((size_t)nr), i8((size_t)nr);
        uint32_t rng = 12345u;
        for (int64_t i = 0; i < nr; ++i) {
            for (int k = 0; k < 3; ++k) {
                const float f = orc_random_float01(&rng);
                rays[(size_t)i * 6 + k] = omin[k] + f * (omax[k] - omin[k]);
            }
            float d[3];
            orc_random_unit_vector(&rng, d);
            memcpy(&rays[(size_t)i * 6 + 3], d, sizeof d);
        }
        orc_hit_batch(os, rays.data(), nr, 0.001f, 1.0e7f, h1.data(), i1.data(), 1);
        orc_hit_batch(os, rays.data(), nr, 0.001f, 1.0e7f, h8.data(), i8.data(), 8);
        CHECK(i1 == i8, "oracle batch threads %s", name);
        orc_camera cam;
        const int W = 64, H = 36;
        orc_camera_for_scene(&cam, bmin, bmax, W, H, strstr(name, "sponza") != nullptr);
        std::vector<uint8_t> a((size_t)W * H * 4), b((size_t)W * H * 4);
        const uint64_t ra = orc_render(os, &cam, W, H, 2, ORC_SEED_SAMPLE, 0, H, 1, 1, a.data());
        const uint64_t rb = orc_render(os, &cam, W, H, 2, ORC_SEED_SAMPLE, 0, H, 1, 8, b.data());
        CHECK(ra == rb && a == b, "oracle render threads %s", name);
        orc_scene_destroy(os);

        // ---- PNG encode: 8 threads over 2-row strips, and 1 thread
        const std::string p1 = "/tmp/san_driver_1.png", p8 = "/tmp/san_driver_8.png";
        setenv("TMPT_PNG_THREADS", "1", 1);
        CHECK(tmpt::write_png(p1.c_str(), a.data(), W, H) == 0, "png 1");
        setenv("TMPT_PNG_THREADS", "8", 1);
        setenv("TMPT_PNG_STRIP", "2", 1);
        CHECK(tmpt::write_png(p8.c_str(), a.data(), W, H) == 0, "png 8");
        const std::vector<uint8_t> f1 = slurp(p1.c_str()), f8 = slurp(p8.c_str());
        CHECK(f1.size() > 0 && f8.size() > 0, "png files");
        orc_free(ot);
        printf("ok %s: %d triangles, octree %zu nodes (digest equal), %d flat, oracle batch + render 1 == 8 threads\n",
               name, n, oh.nodes.size(), nflat);
    }
    printf(g_fail ? "FAILED %d checks\n" : "all checks passed\n", g_fail);
    return g_fail ? 1 : 0;
}
