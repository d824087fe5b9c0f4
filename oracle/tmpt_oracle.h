/*
 * tmpt_oracle.h -- CPU restatement of pr0g/ToyMeshPathTracer's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (toymeshpathtracer_amd/, libtmpt.so) never links or calls it.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - the reference cannot be built here (it needs Intel TBB, which the image
 *     lacks; a shim would be a stand-in header, which this project does not
 *     write), so the restatement is pinned against
 *       (a) the reference's own golden renders result{1..4}*.png
 *           (statistical: macOS libm produced them), and
 *       (b) the raw-RGBA SHA-256 prefixes + ray counts of the reference binary
 *           that SURVEY.md §8c records for 640x360x4 row mode.
 *   - every function cites the reference file:line it restates.
 *
 * Float semantics: compiled with -ffp-contract=off, no fast-math, so every
 * operation rounds exactly where GLM 0.9.9.5 rounds.
 */
#ifndef TMPT_ORACLE_H
#define TMPT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Camera, field-for-field maths.h:106-111. */
typedef struct {
    float origin[3], lower_left[3], horizontal[3], vertical[3], u[3], v[3], w[3];
    float lens_radius;
} orc_camera;

typedef struct orc_scene orc_scene;

/* scene query accelerators */
enum { ORC_ACCEL_OCTREE = 0, ORC_ACCEL_BVH = 1, ORC_ACCEL_LINEAR = 2 };
/* tie handling among equal-t hits:
 *   ORC_TIE_VISIT: first found in visit order wins (strict '<', scene.cpp:34)
 *   ORC_TIE_INDEX: lowest triangle index wins (= linear scan with strict '<') */
enum { ORC_TIE_VISIT = 0, ORC_TIE_INDEX = 1 };
/* RNG seeding: ROW = main.cpp:204 unmodified; PIXEL = per-pixel seed */
enum { ORC_SEED_ROW = 0, ORC_SEED_PIXEL = 1, ORC_SEED_SAMPLE = 2 };
/* sample seeding: sample s of a pixel starts ORC_SAMPLE_STRIDE xorshift steps per
 * sample into the pixel's stream (state = M^(s * stride) * pixel seed) */
#define ORC_SAMPLE_STRIDE 65536u

/* ---- RNG / sampling KATs (maths.cpp:5-38) ---- */
uint32_t orc_xorshift32(uint32_t* state);
uint32_t orc_xorshift32_jump(uint32_t state, uint64_t n);
/* start state of sample `smp` of the pixel whose pixel-mode seed is `seed` */
uint32_t orc_sample_seed(uint32_t seed, uint32_t smp);
float    orc_random_float01(uint32_t* state);
void     orc_random_in_unit_disk(uint32_t* state, float out[3]);
void     orc_random_unit_vector(uint32_t* state, float out[3]);
uint32_t orc_pixel_seed(int32_t x, int32_t y, int32_t w);

/* ---- Camera (maths.cpp:40-59, maths.h:93-104, main.cpp:295-307) ---- */
void orc_camera_init(orc_camera* cam, const float look_from[3], const float look_at[3],
                     const float vup[3], float vfov, float aspect, float aperture,
                     float focus_dist);
void orc_camera_for_scene(orc_camera* cam, const float bmin[3], const float bmax[3],
                          int32_t w, int32_t h, int32_t is_sponza);
void orc_camera_get_ray(const orc_camera* cam, float s, float t, uint32_t* state,
                        float out_orig[3], float out_dir[3]);

/* ---- OBJ ingest (objparser.cpp:13-355, main.cpp:122-170) ----
 * Returns 0 on success. *out_tris = malloc'd (n+2)*9 floats incl. the 2 floor
 * triangles; bounds are the OBJ-only bounds (main.cpp:132-151). */
int  orc_load_scene(const char* path, float** out_tris, int32_t* out_n,
                    float out_bmin[3], float out_bmax[3]);
void orc_free(void* p);

/* ---- Scene query (scene.h:17-43, scene.cpp) ---- */
orc_scene* orc_scene_create(const float* tris, int32_t n, int32_t accel, int32_t tie_mode,
                            const float oct_min[3], const float oct_max[3]);
void       orc_scene_destroy(orc_scene* s);
/* HitScene (scene.cpp:86-97) with the triangle index reported (-1 on miss).
 * hit_out = {pos.xyz, normal.xyz, t}; written only on a hit. */
int32_t    orc_hit_scene(const orc_scene* s, const float orig[3], const float dir[3],
                         float tmin, float tmax, float hit_out[7]);
/* batched: rays = n x {ox,oy,oz,dx,dy,dz}; hits n x 7; ids n */
void       orc_hit_batch(const orc_scene* s, const float* rays, int64_t n, float tmin,
                         float tmax, float* hits, int32_t* ids, int32_t nthreads);
/* statistics of the octree (node count, leaf count, triangle references) */
void       orc_scene_stats(const orc_scene* s, int64_t out[4]);
/* FNV-1a of the octree's preorder walk (box bits, leaf lists): see the C file */
uint64_t   orc_octree_digest(const orc_scene* s);
/* The octree's nodes in storage order (the root first, each node's 8 children
 * contiguous): boxes n x {min.xyz, max.xyz}, info n x {first child or -1,
 * leaf triangle count, depth}.  Writes min(n, cap) nodes; returns n.  Test
 * generators aim rays at these boxes' faces, edges and corners. */
int64_t    orc_octree_nodes(const orc_scene* s, float* boxes, int32_t* info, int64_t cap);
/* A leaf's triangle list in the reference's order (ids[0..min(count, cap))); returns its count */
int32_t    orc_octree_leaf(const orc_scene* s, int64_t node, int32_t* ids, int32_t cap);
/* The reference's slab test (maths.h:116-134 over 1/dir, scene.cpp:92-93) of
 * each ray against one box: out[i] = 1 if RayHitAabb passes. */
void       orc_ray_box_batch(const float* rays, int64_t n, const float box[6], float tmin, float tmax,
                             uint8_t* out);

/* ---- Tracer (main.cpp:44-119, 172-246) ----
 * Renders rows y = y0, y0+row_step, ... < y1 into rgba (full-frame layout,
 * W*H*4, row 0 = bottom, rows not rendered are left untouched).
 * Returns the ray count (every HitScene call, main.cpp:57,91), as uint64. */
uint64_t orc_render(const orc_scene* s, const orc_camera* cam, int32_t w, int32_t h,
                    int32_t spp, int32_t seed_mode, int32_t y0, int32_t y1,
                    int32_t row_step, int32_t nthreads, uint8_t* rgba);
/* The same over the pixels x = x0, x0 + x_step, ... of each of those rows
 * (pixel and sample seeding; row seeding renders whole rows: its stream runs
 * through every pixel of the row).  Returns 0 rays if out of memory. */
uint64_t orc_render_ex(const orc_scene* s, const orc_camera* cam, int32_t w, int32_t h,
                       int32_t spp, int32_t seed_mode, int32_t y0, int32_t y1,
                       int32_t row_step, int32_t x0, int32_t x_step, int32_t nthreads, uint8_t* rgba);

/* One path (Trace, main.cpp:82-119) from a given ray; rng advanced in place.
 * Returns the colour; *rays incremented by the HitScene calls made. */
void orc_trace(const orc_scene* s, const float orig[3], const float dir[3],
               uint32_t* rng, float out_col[3], uint64_t* rays);

/* (cos a, sin a) for the 24-bit RNG key k, with a = ((k/2^24)*2)*kPI exactly as
 * RandomUnitVector computes it (maths.cpp:33-36). */
void orc_unit_angle_sincos(uint32_t key24, float* c, float* s);
/* the same for keys [key0, key0 + n): out = n x {cos, sin} */
void orc_unit_sincos_range(uint32_t key0, uint32_t n, float* out);

#ifdef __cplusplus
}
#endif
#endif
