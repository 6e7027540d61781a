/*
 * mcpt_hip.h — C ABI of the MI355X path-tracing hot path (libmcpt_hip.so).
 *
 * The reference drives its per-sample loop through C++ module interfaces
 * (MonteCarloPathTracing/ is abbreviated MCPT/ below):
 *   RayGeneration::init/generateRay        MCPT/raygeneration.h:15-17, raygeneration.cpp:29-67
 *   SceneBuild::buildScene/init            MCPT/scenebuild.h:31-33,   scenebuild.cpp:50-101,149-169
 *   SceneBase::intersect/shade             MCPT/scenebuild.h:15-16,   scenebuild.cpp:103-145
 *   ColorOut::init/outputColorCL           MCPT/colorout.h:6-8,       colorout.cpp:31-73
 *   OpenCL::init/update (the frame loop)   MCPT/OpenCLApp.h:4-5,      OpenCLApp.cpp:36-82
 *   ThirdPartyWrapper::loadObject/outputPicture  MCPT/thirdpartywrapper.h:13-16
 *   Auxiliary::parseCamera                 MCPT/auxiliary.h:27,       auxiliary.cpp:20-71
 *   BVH::HLBVH<CPU>                        MCPT/BVH/hlbvh.h:10-26,    hlbvh.cpp:92-200
 * Every entry point below names the interface it replaces.
 *
 * Conventions
 *  - Plain C: POD structs, pointers + sizes, int status (0 = MCPT_OK, < 0 =
 *    error), no exceptions cross the boundary; mcpt_last_error() explains the
 *    last failure of the calling thread.
 *  - Record structs are byte-identical to MCPT/objdef.h:21-99 (Camera 80 B,
 *    Ray 48 B, Hit 48 B, Triangle 64 B, Material 48 B, BVHNode 64 B), so a
 *    reference host can hand its own vectors over unchanged.
 *  - "_dev" pointers are device (HBM) pointers, "stream" is a hipStream_t
 *    passed as void* (NULL = default stream).  Host pointers are never
 *    retained after a call returns.
 *  - A context is bound to one GPU and is not thread-safe: one host thread or
 *    process per GPU (multi-GPU = one process per GPU).
 */
#ifndef MCPT_HIP_H
#define MCPT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status */
#define MCPT_OK 0
#define MCPT_ERR_ARG (-1)      /* bad argument / size mismatch              */
#define MCPT_ERR_HIP (-2)      /* HIP runtime failure                        */
#define MCPT_ERR_IO (-3)       /* file could not be read / written           */
#define MCPT_ERR_PARSE (-4)    /* malformed OBJ / MTL / JSON                 */
#define MCPT_ERR_LIMIT (-5)    /* BVH deeper than the reference's stack[64]  */
#define MCPT_ERR_NOGPU (-6)    /* no HIP device / device index out of range  */

/* ------------------------------------------------------ records (objdef.h) */
typedef struct mcpt_camera {        /* objdef.h:21-27, 80 B */
  float center[4], direction[4], up[4], horizontal[4];
  float arg;                        /* vertical fov in radians              */
  float tmin;
  uint32_t camera_type;             /* 0 perspective, 1 orthographic        */
  float pad;
} mcpt_camera;

typedef struct mcpt_ray {           /* objdef.h:29-39, 48 B */
  float origin[4];                  /* .w bits: int term_depth              */
  float direction[4];               /* .w bits: int pixel id                */
  float ratio[4];                   /* unused by the reference              */
} mcpt_ray;

typedef struct mcpt_hit {           /* objdef.h:41-48, 48 B */
  float normal[4];
  float point[4];
  float t;                          /* FLT_MAX = miss                       */
  uint32_t triangle_id;
  uint32_t material_id;
  uint32_t pad;
} mcpt_hit;

typedef struct mcpt_triangle {      /* objdef.h:50-56, 64 B */
  float v[3][4];
  float normal[4];                  /* .w bits: int material id             */
} mcpt_triangle;

enum {                              /* objdef.h:58-67 */
  MCPT_DIFFUSE = 1,
  MCPT_GLOSSY = 2,
  MCPT_TRANSPARENT = 3,
  MCPT_LIGHT = 4
};

typedef struct mcpt_material {      /* objdef.h:69-79, 48 B */
  int32_t type;
  float Ni, Ns, pad;
  float kd[4];
  float ka_ks[4];                   /* ka for LIGHT, ks for GLOSSY          */
} mcpt_material;

typedef struct mcpt_bvh_node {      /* objdef.h:91-99, 64 B */
  float bbmin[4], bbmax[4], pad[4];
  int32_t parent, left, right, pad2;/* leaf: left == right == triangle id   */
} mcpt_bvh_node;

/* ray.origin.w / term_depth bitfield (shade.cl:100-206) */
#define MCPT_TERMINATED 0xFF000000u
#define MCPT_INSIDE     0x00FF0000u
#define MCPT_DEPTH_MASK 0x0000FFFFu

/* -------------------------------------------------------- opaque handles */
typedef struct mcpt_ctx mcpt_ctx;
typedef struct mcpt_scene mcpt_scene;

/* Render modes for the fused path.
 *  MCPT_MODE_EXACT   — reference arithmetic, traversal order and tie rule;
 *                      closest-hit pruning only where it cannot change the
 *                      accepted hit.  The default.
 *  MCPT_MODE_NOPRUNE — exhaustive left-first traversal exactly as
 *                      objdef.h:240-275 (slow; parity cross-check).          */
#define MCPT_MODE_EXACT   0
#define MCPT_MODE_NOPRUNE 1

typedef struct mcpt_render_params {
  int32_t width, height;            /* config width/height (= camera.resolution) */
  int32_t max_depth;                /* config "maxdepth"  (-D MAX_DEPTH)   */
  int32_t max_attempt;              /* config "attempt"   (-D MAX_ATTEMPT) */
  int32_t frame_begin;              /* first frame index of this call (attemptCount) */
  int32_t frames;                   /* frames to render in this call       */
  int32_t stripe_rows;              /* multi-GPU tile: rows per stripe      */
  int32_t stripe_index;             /* this GPU's stripe residue            */
  int32_t stripe_count;             /* number of GPUs (1 = whole image)     */
  int32_t mode;                     /* MCPT_MODE_*                          */
  int32_t frames_per_launch;        /* frames per block (a lane runs one pixel
                                       for one block, then hands it on);
                                       <= 0: auto (mcpt_tuning.block_entries);
                                       images over 67 M pixels (no hand-off
                                       area) run one block of at most
                                       max_block_frames frames per launch */
  int32_t schedule;                 /* MCPT_SCHED_*: how k_render batches leaf
                                       tests (results identical; speed only) */
} mcpt_render_params;

/* Leaf-test schedules of the fused kernel (bit-identical results):
 *  MCPT_SCHED_SINGLE — one triangle per lane per leaf phase (the value of a
 *                      zero-initialised mcpt_render_params)
 *  MCPT_SCHED_PAIRED — a lane whose next stack entry is also a leaf tests
 *                      both in one phase (measured faster on C2-C5: +2-9 %;
 *                      the Python host's default);
 *  Renderer.tune_schedule() picks one by timing both. */
#define MCPT_SCHED_SINGLE 0
#define MCPT_SCHED_PAIRED 1

typedef struct mcpt_stats {
  uint64_t segments;                /* rays alive at intersect entry, all frames */
  uint64_t node_visits;             /* nodes whose children were tested (EXACT: 4-wide) */
  uint64_t tri_tests;               /* triangle tests                        */
  uint64_t bad_material;            /* hits on an unknown material type      */
  double   kernel_ms;               /* device time of the last render call   */
  int32_t  launches;                /* kernel launches of the last render call */
  int32_t  frames_per_block;        /* block size the last render call used   */
  uint64_t wave_node_phases;        /* wave-level node steps (SIMT efficiency = */
  uint64_t wave_leaf_phases;        /*  node_visits / (64 * wave_node_phases)) */
  uint64_t wave_shade_phases;
  uint64_t order_fallbacks;         /* EXACT: segments re-searched in the     */
                                    /*  reference's left-first order         */
  uint64_t wave_iterations;         /* k_render loop iterations, all waves    */
  uint64_t lane_waiting;            /* lane-iterations spent waiting for the
                                       previous frame block of its pixel     */
  uint64_t lane_idle;               /* lane-iterations with no pixel (queue
                                       claim pending, or the launch's tail)  */
  int32_t  stack_window;            /* 1: the last call ran the LDS-window stack */
  int32_t  workgroups;              /* 64-lane waves per launch (the resident grid;
                                       a k_render workgroup holds 4 of them)      */
  uint64_t debug_violations;        /* MCPT_DEBUG builds: stack-bound, node- and
                                       triangle-index violations k_render caught
                                       (always 0 in release builds)           */
  uint64_t phase_ticks[4];          /* MCPT_PHASE_TIMING builds: shader-clock ticks
                                       all waves spent in fetch, T, L, S (0 in
                                       release builds)                        */
  uint64_t leaf_rejects;            /* stats on, quantized tree: leaves the search
                                       reached whose exact box the ray misses */
  int32_t  quantized;               /* 1: the last call searched the 64-B
                                       quantized tree (EXACT mode)            */
  int32_t  primary_cache;           /* 0: the last call traced every frame's
                                       primary ray; 1: it read the cached
                                       primary hits; 2: it computed them too  */
  double   primary_ms;              /* primary_cache 2: device time of the
                                       primary-hit pass (part of kernel_ms)   */
  int32_t  top_levels;              /* the search tree's top levels the last
                                       call kept in LDS (mcpt_tuning.top_levels) */
} mcpt_stats;

/* Launch-plan knobs of the fused kernel (speed only: every setting gives the
 * same bits).  A zero-initialised struct means "defaults"; each field <= 0
 * keeps its default.  Replaces the environment knobs of earlier builds:
 * nothing is read from the environment on the render path. */
typedef struct mcpt_tuning {
  int32_t leaf_threshold;   /* lanes with a pending leaf before the L phase runs,
                               for a wave of 64 live lanes (default 4 single /
                               16 paired schedule; scaled to the live lanes)   */
  int32_t shade_threshold;  /* lanes waiting before the S phase runs, for 64
                               live lanes (32; scaled the same way)            */
  int32_t queue_chunk;      /* queue entries a wave claims per atomic (4)        */
  int32_t block_entries;    /* auto frames-per-block: smallest block count (at
                               least 2) that gives every resident lane this many
                               queue entries (8)                                 */
  int32_t max_block_frames; /* frames-per-block upper bound of auto plans and of
                               images over 67 M pixels (32)                      */
  int32_t stack_window;     /* 0 auto (default), 1 the 32-entry LDS window with
                               a global spill, 2 the whole stack in LDS          */
  int32_t lds_pad;          /* extra LDS bytes per workgroup (occupancy
                               experiments; 0)                                    */
  int32_t queues;           /* work queues (1..8; 8: one per XCD)              */
  int32_t fetch_threshold;  /* lanes of a wave needing a new queue entry before
                               the wave claims and starts them together (1)    */
  int32_t quantized;        /* EXACT search tree: 0 auto (the 64-B quantized
                               nodes when the 128-B tree exceeds 32 MiB, the
                               GPU's aggregate L2), 1 quantized whenever the
                               scene has them, 2 the 128-B nodes                 */
  int32_t primary_cache;    /* every frame re-shoots the same primary ray, so its
                               hit is computed once per (scene, camera, image,
                               stripes, mode) and kept in the context: 0 auto
                               (a call of >= 2 frames, or a one-frame call of
                               the previous call's view, computes it; every
                               call with a matching one reads it), 1 always,
                               2 never                                          */
  int32_t last_block_frames; /* auto frames-per-block, one-launch calls of two
                               or more blocks: the last block of every pixel
                               is this many frames and the others share the
                               rest evenly (a short last block shortens the
                               launch's tail); 0 auto (ceil(frames / 8) from
                               6 pixels per resident lane, ceil(frames / 4)
                               from 2.5 on a whole image (stripe_count 1),
                               else equal blocks), -1 equal blocks            */
  int32_t tile_order;       /* order of the 8x8 pixel tiles in the work queues:
                               0 auto (the primary-hit pass measures each
                               pixel's primary-ray traversal; tiles whose
                               costliest pixel is dearest start first, so the
                               longest per-pixel chains do not start last), 1
                               the image order, 2 by the tile's summed cost    */
  int32_t pixel_spread;     /* how the queues' pixel slots map to a wave's
                               lanes: 0 auto (spread up to 2.5 pixels per
                               resident lane: strong-scaled shares, where each
                               pixel's own chain sets the time; tile-major
                               above), 1 tile-major (a wave's 64
                               consecutive slots are one 8x8 tile), 2 spread
                               (they are one pixel of each of 64 tiles, so one
                               tile's dear pixels run in different waves)      */
  int32_t top_levels;       /* EXACT: the search tree's top levels kept in LDS,
                               where a segment descends through them as it
                               begins instead of one T-phase gather per level:
                               0 auto (2; 4 on trees over 4 MiB), 1-4 levels,
                               -1 none                                           */
} mcpt_tuning;

/* ------------------------------------------------------- version / errors */
/* The ABI revision this header describes.  It changes whenever a struct
 * passed across the boundary changes size or layout, or an entry point its
 * arguments (3: mcpt_tuning's tile_order / pixel_spread,
 * mcpt_set_pixel_segments' capacity; 4: the rejected T-phase-helper and
 * merged-gather knobs and counters removed from mcpt_tuning / mcpt_stats,
 * `top_levels` added to both).
 * A binding checks mcpt_abi_version() == MCPT_ABI_VERSION once at load and
 * refuses a library built from another header.                           */
#define MCPT_ABI_VERSION 4
int32_t mcpt_abi_version(void);
const char *mcpt_version(void);
const char *mcpt_last_error(void);

/* ----------------------------------------------------------- host side
 * Everything here is plain C++ on the host; no GPU needed.               */

/* Auxiliary::parseCamera (auxiliary.cpp:20-71): JSON camera -> Camera.   */
int mcpt_parse_camera(const double position[3], const double lookat[3],
                      const double up[3], double fov_deg, mcpt_camera *out);

/* MTL record -> Material, thirdpartywrapper.cpp:65-97 precedence:
 * ior != 1 -> TRANSPARENT; any Ka > 0 -> LIGHT; Ns != 1 -> GLOSSY; else DIFFUSE. */
int mcpt_classify_material(float ior, const float ambient[3], const float diffuse[3],
                           const float specular[3], float shininess, mcpt_material *out);

/* ThirdPartyWrapper::loadObject (thirdpartywrapper.cpp:25-99) on an
 * OBJ + its MTL library: two-call pattern — call with NULL outputs to get
 * the counts, then again with arrays of that size.  Triangles come out
 * with v[] filled and normal zeroed (SceneCL packs them, below);
 * mat_index[i] is the per-face material index (-1 if none).            */
int mcpt_load_obj(const char *directory, const char *objname,
                  mcpt_triangle *tris, int32_t *mat_index, int64_t *n_tris,
                  mcpt_material *mats, int32_t *n_mats);

/* SceneCL ctor packing (scenebuild.cpp:58-62): normal = normalize(cross(
 * v1-v0, v2-v0)), normal.w <- material index bits.  In place.           */
int mcpt_pack_triangles(mcpt_triangle *tris, const int32_t *mat_index, int64_t n);

/* HLBVH<CPU>::build (hlbvh.cpp:92-200): Morton LBVH, 2n-1 nodes, root 0,
 * leaves at [n-1, 2n-2].  nodes must hold 2n-1 records.                 */
int mcpt_build_hlbvh(const mcpt_triangle *tris, int64_t n, mcpt_bvh_node *nodes);

/* Max DFS stack depth the reference traversal needs on this tree.      */
int mcpt_bvh_stack_depth(const mcpt_bvh_node *nodes, int64_t n_nodes, int32_t *depth);

/* BVH::TEST::SAH (bvhtest.cpp:97-108), the "testbvh" SAH line: the float
 * result (Cinn * area of nodes [0, size/2) + Ctri * area of the rest, summed
 * in double, over the root's area) widened to double.                     */
int mcpt_bvh_sah(const mcpt_bvh_node *nodes, int64_t n_nodes, double *sah);

/* ThirdPartyWrapper::outputPicture (thirdpartywrapper.cpp:14-23):
 * stbi_write_hdr with vertical flip, 4 components in, RGB out.           */
int mcpt_write_hdr(const char *path, int32_t width, int32_t height,
                   const float *rgba, int32_t flip_vertically);
/* Same encoder into memory: returns the byte count (call with NULL first);
 * MCPT_ERR_ARG if `cap` is too small for it.                              */
int64_t mcpt_encode_hdr(int32_t width, int32_t height, const float *rgba,
                        int32_t flip_vertically, uint8_t *out, int64_t cap);

/* ---------------------------------------------------------- device side */

/* OpenCLBasic::init (oclbasic.cpp:75-122) equivalent: bind to a GPU.     */
int mcpt_ctx_create(int32_t device, mcpt_ctx **out);
int mcpt_ctx_destroy(mcpt_ctx *ctx);
int mcpt_device_count(int32_t *count);

/* SceneBuild::buildScene (scenebuild.cpp:50-101,149-156): upload the packed
 * triangles + reference BVH + materials; converted to the device layout
 * (child-box nodes, Cramer-ready triangles — DESIGN.md §2) once here.   */
int mcpt_scene_upload(mcpt_ctx *ctx, const mcpt_triangle *tris, int64_t n_tris,
                      const mcpt_bvh_node *nodes, int64_t n_nodes,
                      const mcpt_material *mats, int32_t n_mats, mcpt_scene **out);
int mcpt_scene_destroy(mcpt_scene *scene);
/* The same with the scene already in HBM (tris_dev packed as
 * mcpt_pack_triangles leaves them, nodes_dev in the HLBVH layout, e.g. from
 * mcpt_build_hlbvh_device + mcpt_treelet_gpu_device): every device structure,
 * the EXACT path's SAH search tree included, built on the GPU, the same
 * bytes as mcpt_scene_upload's.  Synchronises `stream`.                  */
int mcpt_scene_upload_device(mcpt_ctx *ctx, const mcpt_triangle *tris_dev, int64_t n_tris,
                             const mcpt_bvh_node *nodes_dev, int64_t n_nodes, const mcpt_material *mats,
                             int32_t n_mats, void *stream, mcpt_scene **out);
/* A scene's device arrays copied to the host (introspection).  which: 0 the
 * search tree (128-B nodes), 1 its quantized nodes, 2 the reference tree
 * 4-wide, 3 the binary child-box nodes, 4 triangles, 5 quantized-path
 * triangles, 6 int32[4] {stack_depth, stack_depth4, quantized, n_internal}.
 * *bytes = the size (host NULL: size only).                               */
int mcpt_scene_read(const mcpt_scene *scene, int32_t which, void *host, int64_t cap, int64_t *bytes);

/* Fused per-pixel path loop: for every pixel of this GPU's stripes and
 * frames [frame_begin, frame_begin+frames): generateRay -> maxdepth x
 * (intersect, shade) -> history accumulate, exactly the per-pixel effect of
 * OpenCL::update (OpenCLApp.cpp:57-82) + ColorOut (colorout.cpp:40-73).
 * seeds/hist/count are W*H device arrays (u32, float4, i32) that persist
 * across calls; pixels outside this GPU's stripes are left untouched.
 * Stream-ordered and asynchronous: the call enqueues its work on `stream`
 * and returns (mcpt_get_stats waits for it).  One stream per context at a
 * time: the context's queue heads and hand-off area are reused by every
 * call.                                                                  */
int mcpt_render_frames(mcpt_ctx *ctx, const mcpt_scene *scene, const mcpt_camera *cam,
                       const mcpt_render_params *params, uint32_t *seeds_dev,
                       float *hist_dev, int32_t *count_dev, void *stream);

/* Launch-plan knobs (speed only), kept in the context; NULL resets them.  */
int mcpt_set_tuning(mcpt_ctx *ctx, const mcpt_tuning *tuning);
int mcpt_get_tuning(mcpt_ctx *ctx, mcpt_tuning *out);
/* Forget the primary-hit cache (mcpt_tuning.primary_cache): the next render
 * call traces or recomputes its primary hits itself (bench.py's timed call). */
int mcpt_drop_caches(mcpt_ctx *ctx);

/* Per-image state in HBM for C/C++ hosts that do not manage device memory
 * themselves: the reference's randBuffer (scenebuild.cpp:113-120),
 * frameBuffer and sampleCount (colorout.cpp), W*H each.  create copies the
 * host seeds in and zeroes mean and count; buffers() returns the device
 * pointers mcpt_render_frames takes; download copies any of them back to
 * host arrays (NULL skips one) after the context's work on `stream` is done
 * (ColorOut's dump read, colorout.cpp:55-68).                            */
typedef struct mcpt_state mcpt_state;
int mcpt_state_create(mcpt_ctx *ctx, int32_t width, int32_t height, const uint32_t *seeds_host, mcpt_state **out);
int mcpt_state_buffers(mcpt_state *st, uint32_t **seeds_dev, float **hist_dev, int32_t **count_dev);
int mcpt_download(mcpt_ctx *ctx, const mcpt_state *st, float *hist_rgba, int32_t *count, uint32_t *seeds,
                  void *stream);
/* Checkpoint / resume: mcpt_upload writes host arrays (NULL skips one) into
 * the state, ordered on `stream` before later renders; a state saved with
 * mcpt_download and uploaded into a fresh one continues the render exactly
 * (the per-pixel seed chain, mean and count are the whole of it). */
int mcpt_upload(mcpt_ctx *ctx, mcpt_state *st, const float *hist_rgba, const int32_t *count, const uint32_t *seeds,
                void *stream);
int mcpt_state_destroy(mcpt_state *st);

/* Wavefront kernels on the reference's AoS records, one per reference
 * kernel, for drop-in use and kernel-level parity:                       */
/* rayGenerator.cl generateRay (W x H NDRange)                            */
int mcpt_generate_rays(mcpt_ctx *ctx, const mcpt_camera *cam, int32_t width, int32_t height,
                       mcpt_ray *rays_dev, void *stream);
/* intersect.cl intersectRays (tmin = EPSILON 1e-3, oclbasic.h:193)        */
int mcpt_intersect(mcpt_ctx *ctx, const mcpt_scene *scene, const mcpt_ray *rays_dev,
                   int64_t n, mcpt_hit *hits_dev, float tmin, int32_t mode, void *stream);
/* shade.cl shade (-D MAX_DEPTH)                                           */
int mcpt_shade(mcpt_ctx *ctx, const mcpt_scene *scene, mcpt_ray *rays_dev,
               const mcpt_hit *hits_dev, float *color_dev, uint32_t *seeds_dev, int64_t n,
               int32_t max_depth, void *stream);
/* history.cl func (-D MAX_ATTEMPT): running mean of non-zero samples      */
int mcpt_accumulate(mcpt_ctx *ctx, float *color_dev, float *hist_dev, int32_t *count_dev,
                    int64_t n, int32_t max_attempt, void *stream);
/* testkernel.cl func, ColorOut's display pass (colorout.cpp:58-70): per
 * pixel (pow(r, 1/2.2f), pow(g, 1/2.2f), pow(b, 1/2.2f), 0) into a float4
 * buffer (the reference writes it to its RGBA32F GL texture).  The reference
 * shows the current frame's colours before MAX_ATTEMPT and frameBuffer (the
 * running mean, mcpt_state's hist) after.  n = pixels; may run in place.    */
int mcpt_gamma_preview(mcpt_ctx *ctx, const float *color_dev, float *out_dev, int64_t n, void *stream);

/* Counters of the last render call (segments etc. need stats enabled);
 * waits for that call's work to finish.                                   */
int mcpt_set_stats(mcpt_ctx *ctx, int32_t enabled);
int mcpt_get_stats(mcpt_ctx *ctx, mcpt_stats *out);

/* Diagnostics: with stats on, every render call adds each pixel's segments
 * (the chain of work its frames are, one sequential seed chain per pixel)
 * into counts_dev[y * width + x] and the k_render loop iterations its lane
 * spent on it into iters_dev (width*height u32 each on the device, zeroed by
 * the caller; either may be NULL); NULL, NULL stops it.  n_pixels is the
 * buffers' capacity in pixels: a call whose image has more pixels collects
 * nothing (never writes past them).                                        */
int mcpt_set_pixel_segments(mcpt_ctx *ctx, uint32_t *counts_dev, uint32_t *iters_dev, int64_t n_pixels);
/* The primary-hit pass's per-pixel traversal cost of the cached view (loop
 * iterations of k_render's PRIM form, or node steps + triangle tests of
 * k_primary), width*height u32 to the host; *n = 0 when no cache is held.
 * Pixels outside the cached call's own row stripes read 0.                */
int mcpt_get_primary_cost(mcpt_ctx *ctx, uint32_t *out, int64_t cap, int64_t *n);

/* Diagnostics (MCPT_PHASE_TIMING builds, libmcpt_hip_timing.so): the
 * timeline of every 64-lane wave of the last render call's last k_render
 * launch, 8 words each: start, the first moment one of its lanes found every
 * work queue dry, end, the latest start of a queue entry (s_memrealtime
 * ticks, 100 MHz, chip-wide clock), loop iterations, entries started,
 * lane-iterations spent waiting for a pixel's previous block, XCD.  Waits
 * for the call.  Release builds log nothing: *n_workgroups = 0.  out may be
 * NULL to ask for the count.                                               */
int mcpt_get_wave_log(mcpt_ctx *ctx, uint64_t *out, int64_t cap_workgroups, int64_t *n_workgroups);

/* Diagnostics (MCPT_PHASE_TIMING builds): for a render call of one launch
 * with at most 16 M (pixel, block) entries, the low 32 bits of the 100 MHz
 * s_memrealtime clock at each entry's claim, start (its pixel's previous
 * block published) and end, 3 words per entry at (pixel * blocks + block) * 3
 * (0: never claimed).  *n_entries = pixels * blocks (0 otherwise, and on
 * release builds).  Waits for the call.                                    */
int mcpt_get_entry_log(mcpt_ctx *ctx, uint32_t *out, int64_t cap_entries, int64_t *n_entries, int32_t *blocks);

/* HLBVH::build (MCPT/BVH/hlbvh.cpp:92-200) on the GPU: triangles and the
 * 2n-1 output nodes are DEVICE pointers; the tree is bit-identical to
 * mcpt_build_hlbvh's (finite vertices).  Synchronises `stream`.           */
int mcpt_build_hlbvh_device(const mcpt_triangle *tris_dev, int64_t n, mcpt_bvh_node *nodes_dev, void *stream);

/* TreeletBVH<CPU> (MCPT/BVH/treeletBVH.cpp:343-372, the reference's
 * "bvhtype": "treelet", scenebuild.cpp:70-73) on the GPU, in place on a
 * DEVICE array of 2n-1 nodes as mcpt_build_hlbvh[_device] lays them out:
 * Karras-Aila treelets of up to 7 leaves rebuilt bottom-up with the
 * reference's heap order, subset DP and refit, bit-identical to the
 * reference's sequential pass.  MCPT_ERR_ARG when the reference's own SAH
 * recursion would not terminate on the tree (treeletBVH.cpp:327 quirk).
 * Synchronises `stream`.                                                  */
int mcpt_treelet_device(mcpt_bvh_node *nodes_dev, int64_t n_nodes, void *stream);

/* TreeletBVH<GPU> (MCPT/BVH/treeletBVH.cpp:413-438 + kernels/treeletBVH.cl:230-531):
 * the GPU treelet kernel the reference runs on a fresh HLBVH for EVERY
 * bvhtype before rendering (SceneCL's ctor falls through into its GPUBVH
 * block, scenebuild.cpp:66-95), so the tree its intersect kernel reads.  In
 * place on a DEVICE array of 2n-1 nodes in the HLBVH layout (internal nodes
 * [0, n-2], leaves [n-1, 2n-2]).  The kernel's warp-synchronous behaviour is
 * restated deterministically: its pickNode argmax, lockstep
 * reductions and tie stores (highest lane lands), its refit SAH without
 * /rootArea (treeletBVH.cl:524-525), FP as ROCm's OpenCL compiler builds it
 * for gfx950.  Parity unpinned (treeletBVH.cl:80-81 does not compile).
 * Synchronises `stream`.                                                  */
int mcpt_treelet_gpu_device(mcpt_bvh_node *nodes_dev, int64_t n_nodes, void *stream);
/* Same on a HOST array, the way the reference host uses it on its own node
 * vector (upload, restructure, read back; scenebuild.cpp:89-94,
 * bvhtest.cpp:503-511), on the calling thread's current device.           */
int mcpt_treelet_gpu(mcpt_bvh_node *nodes, int64_t n_nodes);

/* BVH quality metrics of "testbvh" (bvhtest.cpp:448-530), on the GPU.
 * EPO_GPU (bvhtest.cpp:288-321 + kernels/EPO.cl:133-197): per-triangle EPO
 * area and triangle area into the caller's DEVICE arrays (n_tris floats
 * each), bit-identical to the reference kernel; *epo (optional) = their
 * double sums in index order, divided, as the float EPO_GPU returns.
 * *clip_overflows (optional) counts triangles whose clipped polygon exceeds
 * the reference kernel's 8-entry arrays (undefined behaviour there).       */
int mcpt_bvh_epo_device(const mcpt_bvh_node *nodes_dev, const mcpt_triangle *tris_dev, int64_t n_tris,
                        float *epo_dev, float *area_dev, double *epo, uint64_t *clip_overflows, void *stream);
/* LCV (bvhtest.cpp:324-444): leaves hit per pixel-centre camera ray into
 * counts_dev (width*height u32, index i*height + j as the reference pushes
 * its rays), *lcv (optional) = their standard deviation (float result).    */
int mcpt_bvh_lcv_device(const mcpt_bvh_node *nodes_dev, int64_t n_nodes, const mcpt_camera *cam,
                        int32_t width, int32_t height, uint32_t *counts_dev, double *lcv, void *stream);

/* Streaming-read bandwidth of this GPU's HBM (GB/s, best of 5 reads of
 * `bytes` after a warm-up): the measured roofline denominator SURVEY.md
 * §8(d) asks for next to the 8 TB/s spec.                                 */
int mcpt_measure_read_bw(mcpt_ctx *ctx, int64_t bytes, double *gbps);

/* Counter calibration for the roofline: gathers every
 * record of a fresh table_bytes table (a power of two, evicted from the
 * Infinity Cache first) once, in scrambled order, as whole record_bytes
 * records (64: k_render's triangles, 128: its nodes) with one 16-B load per
 * lane and slot.  The known byte count is table_bytes; rocprofv3's
 * FETCH_SIZE for kernel k_gather_probe against it gives the counter's scale
 * for this access shape.  *ms = the kernel's device time.                  */
int mcpt_gather_probe(mcpt_ctx *ctx, int32_t record_bytes, int64_t table_bytes, double *ms);

/* Device self-check of the inline sin/cos used by randomDirection
 * (shade.cl:40-59) against the ocml library calls the reference kernel
 * makes: mismatching bit patterns over the 32768 angles 2*pi*r/32768 and
 * over every float in [0, 8). Both counts are 0 on a correct build.       */
int mcpt_selfcheck_trig(mcpt_ctx *ctx, int64_t *angle_mismatches, int64_t *range_mismatches);
/* The Phong lobe's pow restatement (cl_pow_lobe, mcpt_refmath.h) against
 * ocml's pow_f32 over every float of its domain (0, 1 + 2^-10], for each of
 * the n exponents ys (the scenes' Ns); *mismatches = differing results.      */
int mcpt_selfcheck_pow(mcpt_ctx *ctx, const float *ys, int32_t n, int64_t *mismatches);

#ifdef __cplusplus
}
#endif
#endif /* MCPT_HIP_H */
