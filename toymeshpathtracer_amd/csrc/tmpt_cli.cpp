// tmpt_cli.cpp -- the reference's command line (main.cpp:248-345) over the C ABI:
//   tmpt <width> <height> <spp> <objFile> [--seed row|pixel|sample] [--engine persistent|wavefront|mega]
//        [--gpus N] [--device D] [--out output.png]
// Defaults reproduce the reference: row seeding (main.cpp:204) and output.png.
// Row seeding runs the speculative row engine on the persistent engine (every even RNG offset
// of a window traced, the chain walked through it) and one lane per row with
// --engine mega; pixel or sample seeding make every pixel or sample independent
// work.  With --gpus N (tmpt_render_multi) the rows
// are dealt round-robin one at a time (row y to device y % N), one host thread
// per device, and the tiles are assembled into the frame.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "tmpt.h"

static double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, const char** argv)
{
    if (argc < 5) {
        printf("Usage: tmpt [width] [height] [samplesPerPixel] [objFile] [--seed row|pixel|sample] "
               "[--engine persistent|wavefront|mega] [--gpus N] [--device D] [--out file.png]\n");
        return 1;
    }
    int w = atoi(argv[1]);
    if (w < 1 || w > 10000) { printf("ERROR: invalid width argument '%s'\n", argv[1]); return 1; }
    int h = atoi(argv[2]);
    if (h < 1 || h > 10000) { printf("ERROR: invalid height argument '%s'\n", argv[2]); return 1; }
    int spp = atoi(argv[3]);
    if (spp < 1 || spp > 1024) { printf("ERROR: invalid samplesPerPixel argument '%s'\n", argv[3]); return 1; }
    const char* obj = argv[4];
    int seed = TMPT_SEED_ROW, engine = TMPT_ENGINE_PERSISTENT, gpus = 1, device = 0;
    const char* out = "output.png";
    for (int i = 5; i < argc; ++i) {
        if (!strcmp(argv[i], "--seed") && i + 1 < argc) {
            ++i;
            seed = !strcmp(argv[i], "pixel") ? TMPT_SEED_PIXEL
                                             : (!strcmp(argv[i], "sample") ? TMPT_SEED_SAMPLE : TMPT_SEED_ROW);
        }
        else if (!strcmp(argv[i], "--engine") && i + 1 < argc) {
            ++i;
            engine = !strcmp(argv[i], "mega") ? TMPT_ENGINE_MEGAKERNEL
                     : (!strcmp(argv[i], "wavefront") ? TMPT_ENGINE_WAVEFRONT : TMPT_ENGINE_PERSISTENT);
        }
        else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) gpus = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--out") && i + 1 < argc) out = argv[++i];
        else { printf("ERROR: unknown option '%s'\n", argv[i]); return 1; }
    }
    float* tris = nullptr;
    int32_t n = 0;
    float bmin[3], bmax[3];
    if (tmpt_load_obj(obj, &tris, &n, bmin, bmax)) {
        printf("ERROR: failed to load .obj file\n");
        return 1;
    }
    int ndev = tmpt_device_count();
    if (gpus < 1) gpus = 1;
    if (device + gpus > ndev) {
        printf("ERROR: %d GPU(s) requested from device %d, %d present\n", gpus, device, ndev);
        return 1;
    }
    tmpt_camera cam;
    tmpt_camera_for_scene(&cam, bmin, bmax, w, h, strstr(obj, "sponza.obj") != nullptr);

    std::vector<uint8_t> image((size_t)w * h * 4, 0);
    tmpt_render_desc desc;
    memset(&desc, 0, sizeof(desc));
    desc.width = w; desc.height = h; desc.spp = spp; desc.seed_mode = seed; desc.engine = engine;
    std::vector<int32_t> devs(gpus);
    for (int g = 0; g < gpus; ++g) devs[g] = device + g;
    uint64_t total = 0;
    double dt = 0.0;
    const double t0 = now_s();
    // scene builds + renders; tmpt_render_multi times the renders alone (main.cpp:319-333)
    // BuildOctree(sceneMin - extra, sceneMax + extra), main.cpp:296-297, 312
    float box[6];
    tmpt_octree_bounds(bmin, bmax, box);
    if (tmpt_render_multi(tris, n, box, &cam, &desc, devs.data(), gpus, image.data(), &total, &dt)) {
        printf("ERROR: %s\n", tmpt_last_error());
        return 1;
    }
    printf("Initialized scene '%s' (%i tris) in %.3fs\n", obj, n, now_s() - t0 - dt);
    printf("Rendered scene at %ix%i,%ispp in %.3f s\n", w, h, spp, dt);
    printf("- %.1f K Rays, %.1f K Rays/s\n", total / 1000.0, total / 1000.0 / dt);
    if (tmpt_write_png(out, image.data(), w, h)) { printf("ERROR: %s\n", tmpt_last_error()); return 1; }
    tmpt_free(tris);
    return 0;
}
