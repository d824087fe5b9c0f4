/*
 * oracle_cli.c -- command-line driver for the CPU oracle (test infrastructure).
 * Mirrors main.cpp:248-345: <width> <height> <spp> <objfile>, plus options
 *   --seed row|pixel|sample  --accel octree|bvh|linear  --tie visit|index
 *   --threads N  --out file.rgba (raw RGBA, row 0 = bottom, as in memory)
 */
#include "tmpt_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv)
{
    if (argc < 5) {
        printf("Usage: oracle_cli [width] [height] [samplesPerPixel] [objFile] [options]\n");
        return 1;
    }
    int w = atoi(argv[1]), h = atoi(argv[2]), spp = atoi(argv[3]);
    const char* obj = argv[4];
    int seed = ORC_SEED_ROW, accel = ORC_ACCEL_OCTREE, tie = ORC_TIE_VISIT;
    int threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    const char* out = NULL;
    for (int i = 5; i < argc; ++i) {
        if (!strcmp(argv[i], "--seed") && i + 1 < argc) {
            ++i;
            seed = !strcmp(argv[i], "pixel") ? ORC_SEED_PIXEL : (!strcmp(argv[i], "sample") ? ORC_SEED_SAMPLE : ORC_SEED_ROW);
        }
        else if (!strcmp(argv[i], "--accel") && i + 1 < argc) {
            ++i;
            accel = !strcmp(argv[i], "bvh") ? ORC_ACCEL_BVH
                    : (!strcmp(argv[i], "linear") ? ORC_ACCEL_LINEAR : ORC_ACCEL_OCTREE);
        } else if (!strcmp(argv[i], "--tie") && i + 1 < argc) tie = !strcmp(argv[++i], "index");
        else if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--out") && i + 1 < argc) out = argv[++i];
    }
    if (w < 1 || w > 10000 || h < 1 || h > 10000 || spp < 1 || spp > 1024) {
        printf("ERROR: invalid arguments\n");
        return 1;
    }
    float* tris;
    int32_t n;
    float bmin[3], bmax[3];
    if (orc_load_scene(obj, &tris, &n, bmin, bmax)) {
        printf("ERROR: failed to load .obj file\n");
        return 1;
    }
    float extra[3], omin[3], omax[3];
    for (int k = 0; k < 3; ++k) {
        extra[k] = (bmax[k] - bmin[k]) * 0.7f;
        omin[k] = bmin[k] - extra[k];
        omax[k] = bmax[k] + extra[k];
    }
    double t0 = now_s();
    orc_scene* s = orc_scene_create(tris, n, accel, tie, omin, omax);
    double tb = now_s() - t0;
    orc_camera cam;
    orc_camera_for_scene(&cam, bmin, bmax, w, h, strstr(obj, "sponza.obj") != NULL);
    uint8_t* img = (uint8_t*)calloc((size_t)w * h * 4, 1);
    t0 = now_s();
    uint64_t rays = orc_render(s, &cam, w, h, spp, seed, 0, h, 1, threads, img);
    double dt = now_s() - t0;
    printf("Initialized scene '%s' (%i tris), accel build %.3fs\n", obj, n, tb);
    printf("Rendered scene at %ix%i,%ispp in %.3f s\n", w, h, spp, dt);
    printf("- %.1f K Rays, %.1f K Rays/s\n", rays / 1000.0, rays / 1000.0 / dt);
    if (out) {
        FILE* f = fopen(out, "wb");
        fwrite(img, 1, (size_t)w * h * 4, f);
        fclose(f);
    }
    free(img);
    orc_scene_destroy(s);
    orc_free(tris);
    return 0;
}
