/*
 * tmpt.h -- C ABI of libtmpt.so, the MI355X-native (gfx950) hot path of
 * pr0g/ToyMeshPathTracer: Trace() -> Scatter() -> Scene::HitScene().
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes
 * (0 = ok, < 0 = error; message in tmpt_last_error(); -30 only from the
 * checked build, make CHECK=1: a device index test failed during the call),
 * no C++ exceptions and no
 * torch types cross this boundary.  Every entry point names the reference
 * interface it replaces (/root/reference/source/<file>:<line>); INTEGRATION.md
 * shows the reference-side binding.
 *
 * Threading: one scene per device.  Calls on different scenes may run from
 * different host threads at once; one scene handle is not re-entrant for
 * concurrent render calls.  Host buffers are caller-owned; device memory is
 * library-owned unless a flag says the caller passes a device pointer.
 */
#ifndef TMPT_H
#define TMPT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMPT_ABI_VERSION 9  /* 2: progressive spp (spp_begin / spp_count); 3: tmpt_render_multi;
                              4: tmpt_unit_sincos; 5: wait_stream (TMPT_FLAG_WAIT_STREAM),
                              progressive continuation keyed on the camera,
                              TMPT_SEED_SAMPLE; 6: scene options (tmpt_scene_create_ex,
                              tmpt_scene_set_option / get_option) replace the
                              library's environment variables, tmpt_scene_hit_ranged
                              (per-ray tmin / tmax), tmpt_render_multi gathers over RCCL;
                              7: tmpt_scene_build_octree (the reference's octree: its answer
                              for closest hits tied on t and for rays its root box drops),
                              option tie_rule, tmpt_octree_digest, tmpt_stats octree / tie /
                              row-engine fields, tmpt_render_multi takes the octree box,
                              options tie_defer / redo_cap, tmpt_stats.redo_samples;
                              8: the octree answers crack queries and flat triangles too
                              (tmpt_stats.crack_queries, octree_flat), tmpt_stats.redo_launches /
                              redo_ms (k_redo apart from the k_path launches);
                              9: tmpt_stats.tie_path (how the last render answered the
                              octree's queries, and whether the deferred form fell back) */

typedef struct tmpt_scene tmpt_scene; /* opaque, device-resident */

/* Camera, field for field maths.h:106-111 */
typedef struct {
    float origin[3], lower_left[3], horizontal[3], vertical[3], u[3], v[3], w[3];
    float lens_radius;
} tmpt_camera;

/* RNG seeding of the xorshift32 stream (maths.cpp:5-13):
 *   ROW    the reference: seed y*9781+1 per row, threaded along the row
 *          (main.cpp:204) -- one lane per row
 *   PIXEL  seed (y*W+x)*9781+1 per pixel (0 remapped), its samples in sequence
 *   SAMPLE the pixel's seed as in PIXEL, sample s starting 2^16 * s steps into
 *          that stream (a GF(2) jump), so the samples of a pixel are
 *          independent work; the sum stays in sample order */
enum { TMPT_SEED_ROW = 0, TMPT_SEED_PIXEL = 1, TMPT_SEED_SAMPLE = 2 };

/* render engines */
enum {
    TMPT_ENGINE_WAVEFRONT = 0,  /* generate/extend/shade/shadow kernels over compacted queues */
    TMPT_ENGINE_MEGAKERNEL = 1, /* one lane per pixel (pixel mode) or per row (row mode) */
    TMPT_ENGINE_PERSISTENT = 2  /* pixel mode: one persistent kernel per frame, lanes own pixels and
                                   schedule extend / shadow / shade per wave (row mode: the speculative
                                   row engine -- every even RNG offset of a window traced, the chain
                                   walked through it; instrumented row renders: megakernel) */
};

/* render flags */
enum {
    TMPT_FLAG_OUT_DEVICE = 1,    /* rgba_out is a device pointer on the scene's device */
    TMPT_FLAG_COUNT_VISITS = 2,  /* instrumented traversal: node visits / triangle tests */
    TMPT_FLAG_WAIT_STREAM = 4,   /* the render starts after the work enqueued on desc->wait_stream */
    TMPT_FLAG_REQUIRE_RCCL = 8   /* tmpt_render_multi: fail unless the gather runs over RCCL */
};

/* One render call = one shard of one frame (TraceImageBody over its rows,
 * main.cpp:180-246).  Rows are grouped in bands of band_rows rows; this call
 * renders the bands b with b % num_shards == shard, in increasing b, into a
 * compact tile of full-width rows (RGBA8, row 0 = the lowest rendered row,
 * as in the reference's in-memory image, main.cpp:229).  band_rows = 0 means
 * one band of the whole height. */
typedef struct {
    int32_t width, height, spp;
    int32_t seed_mode;  /* TMPT_SEED_ROW (main.cpp:204), TMPT_SEED_PIXEL or TMPT_SEED_SAMPLE */
    int32_t band_rows;
    int32_t shard, num_shards;
    int32_t engine;
    int32_t flags;
    /* Progressive spp (persistent engine, pixel or sample seeding): this call runs samples
     * [spp_begin, spp_begin + spp_count) of every pixel (spp_count 0 = to spp).
     * A call with spp_begin > 0 continues the per-pixel state (RNG, colour sum)
     * the previous call on this scene left for the same shard, so the passes
     * together equal one full render bit for bit; each pass writes a preview
     * (colour sum / samples so far, main.cpp:221-233 at that count) and the
     * pass that reaches spp writes the final image.  The continuation must use
     * the same camera, size, spp and shard as the pass before it (checked). */
    int32_t spp_begin, spp_count;
    int32_t reserved0;
    /* Stream ordering (TMPT_FLAG_WAIT_STREAM): a hipStream_t of the caller on
     * the scene's device (0 = its null stream).  The render's kernels run on
     * the scene's own non-blocking stream; with the flag they start only
     * after everything enqueued on wait_stream before the call -- e.g. a
     * collective still reading the device buffer a previous render wrote, or
     * the caller's fill of it.  The call returns once the render is complete
     * on the device, so work the caller enqueues afterwards sees the result. */
    uint64_t wait_stream;
    int32_t reserved[2];
} tmpt_render_desc;

/* Statistics of the last render on a scene (HIP-event timed on the scene's
 * stream, i.e. the stream the kernels are launched on). */
typedef struct {
    double render_ms;             /* first kernel to last kernel of the call */
    double extend_ms, shadow_ms;  /* summed closest-hit / any-hit kernel time (persistent engine:
                                     extend_ms = its k_path launches, both query kinds) */
    uint64_t extend_rays, shadow_rays;
    int64_t extend_launches, shadow_launches, iterations;
    uint64_t node_visits, tri_tests; /* extend (closest-hit) kernel, with TMPT_FLAG_COUNT_VISITS */
    uint64_t shadow_node_visits, shadow_tri_tests; /* shadow (any-hit) kernel, same flag */
    double build_ms;                 /* LBVH build of the scene */
    int32_t bvh_nodes, bvh_depth, n_tris, device;
    int32_t bvh4_nodes, bvh4_depth, leaf_max, builder_iters; /* 4-wide tree; PLOC passes (0 = LBVH) */
    /* the reference's octree (tmpt_scene_build_octree; 0 when none) */
    int32_t octree_nodes, octree_leaves;
    int64_t octree_refs;             /* triangle references in its leaves */
    double octree_build_ms;          /* host build */
    /* the last render or HitScene call: closest-hit queries whose t two or more
     * triangles share, answered again in the octree's visit order; and queries
     * the reference's root box test rejected (answered as misses) */
    uint64_t tie_queries, root_misses;
    int32_t row_engine;       /* last render in row seeding: 0 none, 1 one lane per row (megakernel),
                                 2 iterated speculative engine, 3 streaming speculative engine */
    int32_t stream_fallbacks; /* 1: the streaming engine's launch aborted (no chain progress) and the
                                 frame was rendered again by the iterated engine */
    int32_t octree_depth;
    int32_t tie_rule;         /* in effect: 0 octree visit order, 1 lowest index (no octree / option) */
    int64_t chain_pixels;     /* pixel seeding: pixels the last render ran as speculative chains */
    int64_t redo_samples;     /* sample seeding, tie_defer: samples the last render traced again */
    int64_t redo_late;        /* of them, left to the second launch (the main launch's tail did not take them) */
    /* (ABI 8) closest-hit queries answered over the octree because they may run in one of its
     * cracks (a hit near an octree plane on a ray nearly parallel to it) or hit a triangle
     * lying flat on a plane (octree_flat of them in the scene); see tmpt_scene_build_octree */
    uint64_t crack_queries;
    int32_t octree_flat;
    int32_t redo_launches;    /* sample seeding, tie_defer: k_redo launches of the last render (0 or 1) */
    double redo_ms;           /* their time; extend_ms holds the main k_path launches only */
    uint64_t redo_rays;       /* their queries (part of the render's ray count) */
    /* (ABI 9) how the last render answered the queries the octree decides: 0 none (no octree,
     * tie_rule = index, or not a k_path render), 1 in the main loop (the wave's octree walk or
     * the serial walk), 2 deferred (tie_defer: dropped samples traced again in the launch's
     * tail), 3 deferral chosen but its list could not be allocated: answered in the main loop */
    int32_t tie_path;
    int32_t reserved_stats;
} tmpt_stats;

/* ---- host side: scene ingest and camera (not kernels) ------------------- */

/* LoadScene (main.cpp:122-170) over objParseFile (objparser.cpp:304-355):
 * positions of every face, fan-triangulated, plus the 2 floor triangles.
 * *out_tris = n*9 floats (caller frees with tmpt_free); bounds are of the OBJ
 * triangles only (main.cpp:132-151).  Returns 0, or <0 if the file can't be read. */
int tmpt_load_obj(const char* path, float** out_tris, int32_t* out_n, float out_bmin[3],
                  float out_bmax[3]);
void tmpt_free(void* p);

/* Camera::Camera (maths.cpp:40-59) */
int tmpt_camera_init(tmpt_camera* cam, const float look_from[3], const float look_at[3],
                     const float vup[3], float vfov, float aspect, float aperture,
                     float focus_dist);
/* camera placement of main.cpp:295-307 (is_sponza: strstr(path,"sponza.obj")) */
int tmpt_camera_for_scene(tmpt_camera* cam, const float bmin[3], const float bmax[3],
                          int32_t width, int32_t height, int32_t is_sponza);

/* ---- device side --------------------------------------------------------- */

int tmpt_device_count(void);

/* Scene::Scene (scene.h:19, scene.cpp:54-57) + Scene::BuildOctree
 * (scene.h:26, scene.cpp:75-83): copies n triangles (n*9 floats, v0 v1 v2)
 * to `device` and builds the BVH there.  The caller keeps ownership of tris.
 * tmpt_scene_create = tmpt_scene_create_ex with no options. */
int tmpt_scene_create(const float* tris, int32_t n, int32_t device, tmpt_scene** out);

/* Scene options: the library's whole control plane (no environment variables;
 * the reference has no counterpart -- its constants are compiled in).  Every
 * option has a default that reproduces the measured-best configuration; all of
 * them change speed, never the image or the HitScene answers (tie_rule aside).
 * `options` = "key=value,key=value" (NULL or "" = defaults); an unknown key or
 * a value out of range is an error (-22).
 * Build options (only at creation):
 *   builder      ploc (0, default) | lbvh (1): PLOC (Meister & Bittner 2018) or
 *                Karras 2012 LBVH over the same 30-bit Morton order
 *   layout       aos (0, default) | soa (1): the sample-seeding path kernel and the
 *                batched HitScene also get the nodes and triangle records as
 *                planes (56 B / 40 B per node / triangle in 4 / 3 separate
 *                lines) -- the measured A/B of DESIGN.md section 3
 *   leaf_max     triangles per BVH4 leaf, 1..16 (default 2)
 *   collapse     greedy (0, default) | sah (1): BVH2 -> BVH4 collapse
 *   ploc_radius  PLOC search radius, 1..256 (default 32)
 *   sah_c_leaf, sah_c_tri  SAH collapse costs (defaults 0.7, 0.5; inner node 1)
 * Render options (tmpt_scene_set_option; apply to later renders on the scene):
 *   sample_block     sample seeding: samples per work unit, power of two (0 = auto)
 *   sample_tail      sample seeding: the frame's last sample_tail x (resident lanes) blocks run
 *                    as single-sample units, so the frame ends on one sample, not one block
 *                    (-1 = auto: a quarter of a lane's samples, at most 64; 0 = off)
 *   sbuf_max         sample seeding: cap in bytes on the per-sample colour
 *                    buffer (0 = 3/4 of free HBM); over the cap a pixel is one unit
 *   sbuf_pair        sample seeding: a unit's samples 2k and 2k+1 written back to back into
 *                    one 32-B sector of the colour buffer (1) or each on its own (0)
 *   pilot            pixel seeding: pilot samples of the cost-ordered supply (-1 = auto, 0 = off)
 *   help, pair       pixel seeding: shadow offload to idle lanes (-1 = auto, 0, 1)
 *                    and expensive ranks per 64-rank chunk (-1 = auto, 0..63)
 *   balance, dprio   pixel seeding: SIMD-balanced first chunks (1), longest-
 *                    remaining-first wave priority in cost-ordered passes (1)
 *   wave_cap         pixel seeding: pixels a wave holds at once (0 = auto, 1..64)
 *   pixel_chains     pixel seeding, cost-ordered: the heaviest pixels per 1024 that run as
 *                    speculative chains (every even RNG offset past the pilot traced,
 *                    the chain walked through them) instead of in pass 2 (-1 = auto, 0 = off)
 *   rowspec          row seeding on the persistent engine: 1 = speculative row
 *                    engine, 0 = one lane per row chain
 *   rowspec_wmax, rowspec_windows, rowspec_spread, rowspec_groups,
 *   rowspec_noshadow, rowspec_chase, rowspec_stream, rowstream_dynamic
 *                    speculative row engine: units per window (0 = auto),
 *                    windows per row and iteration (0 = auto, 1..32), window
 *                    spread in pixels (-1 = auto), row groups/streams (1..8),
 *                    shadow-free speculation + one full re-trace (1), the
 *                    chase over LDS-staged units, one wave per row (1), the
 *                    streaming engine: one launch, chains walked on the device
 *                    as units finish (1, the default; 0 = host-driven iterations,
 *                    also the fallback when the streaming engine does not apply),
 *                    its windows and spread following the rows still chasing
 *                    (1; 0 = fixed at the launch's load)
 *   row_flag_leaves  row seeding, streaming, with the octree answering ties: the
 *                    leaves only flag a tie (1; 0 = lowest-index bookkeeping, A/B)
 *   row_occ          row seeding, streaming: worker waves per SIMD (0 = by load:
 *                    5 at full load, 4 with room; or 4, 5)
 *   rowstream_test_abort  test hook (0): 1 makes the streaming engine's chaser
 *                    blocks leave at once, so its watchdog (~2 ms then, ~1 s
 *                    normally) aborts the launch and the iterated engine renders
 *                    the frame -- the abort-and-fallback path, reported in
 *                    tmpt_stats.stream_fallbacks
 *   wf_bins          wavefront engine: each segment's extend queue split by the
 *                    rays' direction octant into 1, 2, 4 or 8 sub-queues (1)
 *   tie_rule         visit (0, default) | index (1): closest hits tied on t take the
 *                    reference's octree visit order (needs tmpt_scene_build_octree)
 *                    or the lowest triangle index -- the one option that can change
 *                    an answer, by design: index is the exact-semantics contract
 *   tie_defer        sample seeding with the colour buffer: a sample whose closest hit
 *                    is a tie is dropped by the main loop (built without the octree
 *                    walk) and traced again, ties settled, by the launch's waves once
 *                    their main loop is done (-1 = auto, 0 = off: ties settled in the
 *                    main loop, 1 = on); the image and ray counts are the same either way
 *   redo_lanes       tie_defer: lanes per wave that take the re-traces (1..64, default 4)
 *   path_waves       waves per SIMD of the persistent path kernels (0 = auto, 4 or 5; 5: a 12-entry LDS
 *                    stack and 80 LDS top nodes, 30 KB of LDS per block and 96 VGPRs per lane).  Auto:
 *                    5 in sample seeding and the row engine's re-trace, 5 in pixel seeding from 3 pixels
 *                    per 4-wave lane
 *   redo_cap         test hook (0 = auto): the capacity of tie_defer's sample list; a
 *                    frame that overflows it is rendered again with the list grown
 *   redo_inline      test hook (1): 0 leaves every dropped sample to the second launch
 *                    that otherwise takes only those the main launch's tail did not */
int tmpt_scene_create_ex(const float* tris, int32_t n, int32_t device, const char* options, tmpt_scene** out);
int tmpt_scene_set_option(tmpt_scene* scene, const char* key, double value);
int tmpt_scene_get_option(const tmpt_scene* scene, const char* key, double* value);
/* Scene::BuildOctree (scene.h:26, scene.cpp:75-83; called by main.cpp:312
 * with the OBJ bounds +- 0.7 x their size): builds the reference's octree
 * (scene.cpp:99-160, host) over the scene's triangles and keeps it on the
 * device.  The BVH answers every query; the octree answers the kinds of
 * query where the reference's answer can differ from the BVH's closest hit: a
 * closest hit whose t two or more triangles share (the reference keeps the
 * first in its depth-first visit order, scene.cpp:29-48), a ray its root
 * box test rejects (scene.cpp:25), and a hit the reference's octree can miss
 * through a crack between neighbouring subtrees (their boxes' faces differ by
 * the rounding of min + half + half): a hit point near an octree plane on a
 * ray nearly parallel to that plane, or a triangle lying flat on one (stats
 * crack_queries, octree_flat).  Without it (or with option tie_rule = index)
 * ties go to the lowest triangle index and no ray is rejected.
 * Must not run while a render or HitScene call on the scene is in flight on
 * another host thread: it synchronises the scene's stream and frees the old
 * octree (a caller's wait_stream is not waited on). */
int tmpt_scene_build_octree(tmpt_scene* scene, const float bmin[3], const float bmax[3]);
/* The root box main.cpp:312 gives BuildOctree: sceneMin - extra, sceneMax + extra
 * with extra = (sceneMax - sceneMin) * 0.7 (main.cpp:296-297); bmin / bmax
 * are tmpt_load_obj's OBJ bounds.  box = {min.xyz, max.xyz}. */
int tmpt_octree_bounds(const float bmin[3], const float bmax[3], float box[6]);
/* Check hook (host only, no device): the octree tmpt_scene_build_octree would
 * build: out = {nodes, leaves, triangle references, depth, FNV-1a digest of
 * the preorder walk (box bits, leaf lists)}.  Tests compare it with the
 * oracle's octree. */
int tmpt_octree_digest(const float* tris, int32_t n, const float bmin[3], const float bmax[3], uint64_t out[5]);
/* Check hook (host only, no device): which of n_rays answered queries the
 * octree re-answers besides ties -- rays n_rays x {o.xyz, d.xyz}, t and ids the
 * closest (or first) hit of each (ids < 0: a miss, never flagged):
 * flags[i] = 1 the hit triangle lies flat on an octree plane, | 2 the hit may
 * lie in a crack (the device's own octree_crack test).  grid (may be NULL) =
 * {r0.xyz, 1/cell.xyz, cell.xyz, band.xyz, reach} of that octree. */
int tmpt_octree_flags(const float* tris, int32_t n, const float bmin[3], const float bmax[3], const float* rays,
                      const float* t, const int32_t* ids, int64_t n_rays, uint8_t* flags, float grid[13]);
/* Scene::~Scene (scene.h:20) */
int tmpt_scene_destroy(tmpt_scene* scene);

/* Scene::HitScene (scene.h:36-37, scene.cpp:86-97), batched:
 * rays = n x {orig.xyz, dir.xyz} (dir normalised), hits = n x {pos.xyz,
 * normal.xyz, t} written where ids[i] >= 0; ids[i] = index of the closest
 * triangle or -1 (the reference returns 1 instead of the index).  any_hit != 0
 * stops at the first accepted triangle (the shadow query's semantics: only
 * ids[i] >= 0 is meaningful).  Host pointers. */
int tmpt_scene_hit(const tmpt_scene* scene, const float* rays, int64_t n, float tmin, float tmax,
                   int32_t any_hit, float* hits, int32_t* ids);
/* The same with the range per ray, as each HitScene call takes it
 * (scene.h:36-37: HitScene(ray, tMin, tMax, hit)): rays8 = n x {orig.xyz,
 * dir.xyz, tmin, tmax}.  t is accepted in [tmin, tmax]. */
int tmpt_scene_hit_ranged(const tmpt_scene* scene, const float* rays8, int64_t n, int32_t any_hit,
                          float* hits, int32_t* ids);

/* tbb::parallel_for(rows, TraceImageBody) (main.cpp:329-331, 180-246):
 * renders desc's shard into rgba_out (tmpt_tile_rows(desc) * width * 4 bytes).
 * *ray_count = every HitScene call (main.cpp:57,91), counted in uint64. */
int tmpt_render(tmpt_scene* scene, const tmpt_camera* cam, const tmpt_render_desc* desc,
                uint8_t* rgba_out, uint64_t* ray_count);
/* main.cpp:312-331 over several devices in ONE process (SURVEY.md §8e's
 * single-process form): a scene per entry of devices[] (created here, freed on
 * return), the frame's rows dealt round-robin to them (1-row bands), one host
 * thread per device rendering into a device tile, then ONE RCCL gather
 * (ncclCommInitAll over devices[], ncclGather of the equal-size tiles to
 * devices[0] over xGMI, ncclReduce of the uint64 ray counts) and the rows
 * de-interleaved on devices[0] into rgba_full (width*height*4, row 0 =
 * bottom, as tmpt_render).  RCCL ranks need distinct devices: with a device
 * listed twice the gather is device-to-device copies instead (or an error
 * with TMPT_FLAG_REQUIRE_RCCL in desc->flags).  desc's band_rows, shard and
 * num_shards are taken over; *seconds = wall time from the renders' start to
 * the assembled frame on devices[0] (scene builds excluded, main.cpp:319-333);
 * *ray_count = all devices' rays.  The one-process-per-GPU form is bench.py
 * (torch.distributed + RCCL).  octree_box: each device's scene also builds the
 * reference's octree over it (tmpt_scene_build_octree), as main.cpp:312 does. */
int tmpt_render_multi(const float* tris, int32_t n, const float* octree_box /* bmin[3], bmax[3] or NULL */,
                      const tmpt_camera* cam, const tmpt_render_desc* desc, const int32_t* devices,
                      int32_t ndevices, uint8_t* rgba_full, uint64_t* ray_count, double* seconds);

/* rows in the tile of desc's shard; global row of tile row r */
int32_t tmpt_tile_rows(const tmpt_render_desc* desc);
int32_t tmpt_tile_row_to_y(const tmpt_render_desc* desc, int32_t r);

int tmpt_get_stats(const tmpt_scene* scene, tmpt_stats* out);

/* PNG writer (stbi_write_png with flip-on-write, main.cpp:341-342):
 * rgba rows bottom-up as rendered. */
int tmpt_write_png(const char* path, const uint8_t* rgba, int32_t width, int32_t height);

/* RandomUnitVector's (cos a, sin a) (maths.cpp:33-36: a = ((k / 2^24) * 2) * kPI,
 * then libm cosf/sinf) for the RNG keys [key0, key0 + n): out = n x {cos, sin}
 * (host memory).  device >= 0: computed by the device code the renderers run;
 * device < 0: the same restatement on the host.  A check hook -- the
 * reference has no counterpart; tests compare it with the host libm. */
int tmpt_unit_sincos(int32_t device, uint32_t key0, uint32_t n, float* out);

const char* tmpt_last_error(void);
int tmpt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TMPT_H */
