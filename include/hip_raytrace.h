/*
 * hip_raytrace.h -- C ABI of libhip_raytrace.so, the MI355X (gfx950) drop-in for the compute side
 * of hindlet/EPQ_Raytracer: the path-trace dispatch (assets/raytracing.glsl) and the progressive
 * frame accumulator (assets/image_combiner.glsl).
 *
 * What each entry point replaces (reference paths relative to the reference repo root):
 *   hrt_create       RayTracePipeline::new      src/raytrace_pipeline.rs:51-97   (pipeline + R8G8B8A8 image :67-73)
 *                    DiffusePipeline::new       src/diffuse.rs:35-66             (accumulated image :50-56)
 *   hrt_set_scene    create_ray_subbuffer / create_sphere_subbuffer / create_mesh_subbuffer uploads
 *                                               src/raytrace_pipeline.rs:75-77, :302, :337, :349, :359, :371-372
 *   hrt_trace        RayTracePipeline::compute  src/raytrace_pipeline.rs:162-187 (pc->init == 0)
 *                    RayTracePipeline::init     src/raytrace_pipeline.rs:190-213 (pc->init != 0)
 *                    -> dispatch + push constants  src/raytrace_pipeline.rs:216-266
 *   hrt_accumulate   DiffusePipeline::next_frame src/diffuse.rs:73-101 (-> dispatch :103-136)
 *   hrt_read_image   RayTracePipeline::image / DiffusePipeline::image  src/raytrace_pipeline.rs:156, src/diffuse.rs:69
 *                    (on a row-tile partition with a communicator: the RCCL framebuffer gather, hrt_comm_*)
 *   hrt_synchronize  then_signal_fence_and_flush().unwrap() + fence wait  src/raytrace_pipeline.rs:179-183
 *   hrt_last_error   the .unwrap() panics (every Vulkan call in src/raytrace_pipeline.rs / src/diffuse.rs)
 *
 * Records are byte-identical to the GLSL std430 structs (assets/raytracing.glsl:51-111) and the
 * 124-byte push-constant block (assets/raytracing.glsl:135-153, src/raytrace_pipeline.rs:125-139),
 * so a Rust caller can pass its raytrace_shader::* slices verbatim.
 *
 * Conventions: every function returns hrt_status (0 = OK).  No exceptions cross the ABI.  Host
 * arrays are borrowed for the duration of the call only.  A context is NOT thread-safe: use it from
 * one host thread.  All work on a context is ordered on the context's own HIP stream
 * (== the reference's GpuFuture chaining); hrt_trace / hrt_accumulate return without waiting.
 * Internally a trace runs on one of three trace lanes (own stream + trace image) so that frame k+1's
 * trace overlaps frame k's tail; the combiner, reads and every other call stay in call order on the
 * context's stream, so results equal the serial loop's byte for byte (HRT_OPT_OVERLAP).
 */
#ifndef HIP_RAYTRACE_H
#define HIP_RAYTRACE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 6 (r06): hrt_release_caches; HRT_DEBUG_OPT_STACK_LIMIT.
 * 5 (r05): HRT_DIAG_WQ_STEPS_* / WQ_MEMBERS (HRT_NUM_DIAG 29), HRT_DEBUG_OPT_TIMELINE + hrt_debug_timeline.
 * 4 (r04): hrt_debug_wq_protocol; hrt_stats.last_frames; HRT_DIAG_SKY_* / PRIMARY_LANES / LOOP_ITERS /
 * LIVE_LANES (HRT_NUM_DIAG 24).
 * 3 (r03): hrt_debug_band_flatten.
 * 2 (r03): HRT_ERR_COMM, HRT_IMG_LOCAL, HRT_OPT_COMM_TIMEOUT_MS, collective error agreement;
 * hrt_debug_bvh_wq_nodes' width parameter; HRT_NUM_DIAG / HRT_NUM_SCENE_INFO grown (r02). */
#define HRT_ABI_VERSION 6u

typedef enum hrt_status {
  HRT_OK = 0,
  HRT_ERR_INVALID_ARGUMENT = 1, /* bad pointer / size / count / push-constant field */
  HRT_ERR_NO_DEVICE = 2,        /* no HIP device, or the requested ordinal does not exist */
  HRT_ERR_OUT_OF_MEMORY = 3,
  HRT_ERR_NO_SCENE = 4,         /* hrt_trace before hrt_set_scene */
  HRT_ERR_HIP = 5,              /* a HIP runtime call failed; hrt_last_error has the text */
  HRT_ERR_IO = 6,               /* file not found / unparsable (host helpers) */
  HRT_ERR_COMM = 7              /* a collective (hrt_comm_init, hrt_read_image on a joined context) failed
                                   on ANOTHER rank, timed out or was aborted; every rank of the call
                                   returns an error and none is left blocked (hrt_comm.cpp) */
} hrt_status;

/* ---- std430 records (assets/raytracing.glsl:51-111) ---------------------------------------- */

/* RayTracingMaterial, raytracing.glsl:51-55.  settings = (specular probability, metallic, fuzz,
 * invisible flag == 1.0).  Built by src/materials.rs:13-94. */
typedef struct hrt_material {
  float colour[4];
  float emission[4]; /* rgb, strength */
  float settings[4];
} hrt_material;

/* Ray, raytracing.glsl:66-68: camera-space sample centre around (1,0,0) (w unused). */
typedef struct hrt_ray {
  float sample_centre[4];
} hrt_ray;

/* Sphere, raytracing.glsl:71-75 */
typedef struct hrt_sphere {
  float centre[3];
  float radius;
  hrt_material material;
} hrt_sphere;

/* Triangle, raytracing.glsl:79-84 (w components unused) */
typedef struct hrt_triangle {
  float a[4];
  float edge_one[4]; /* b - a */
  float edge_two[4]; /* c - a */
  float normal[4];   /* edge_one x edge_two, NOT normalised */
} hrt_triangle;

/* Mesh, raytracing.glsl:87-93: triangles[first_index .. first_index+len) */
typedef struct hrt_mesh {
  float min_point[3];
  uint32_t first_index;
  float max_point[3];
  uint32_t len;
  hrt_material material;
} hrt_mesh;

/* PushConstants, raytracing.glsl:135-153 (std430, 124 bytes) */
typedef struct hrt_push_constants {
  float cam_pos[4];
  float cam_alignment_mat[16]; /* column-major mat4; mat3(M) is used */
  int32_t num_rays;
  int32_t num_spheres;
  int32_t num_meshes;
  int32_t num_samples;
  float jitter_size;
  int32_t max_bounces;
  uint32_t use_environment_light; /* GLSL bool */
  uint32_t rng_offset;
  uint32_t init; /* GLSL bool: 1 -> clear the trace image to (0,0,0,1) */
  uint32_t width;
  uint32_t height;
} hrt_push_constants;

/* ---- context ------------------------------------------------------------------------------ */

typedef enum hrt_mode {
  HRT_MODE_RGBA8 = 0,  /* reference-faithful: trace + accumulator images are R8G8B8A8_UNORM */
  HRT_MODE_RGBA32F = 1 /* fp32 images, same arithmetic without the per-frame 8-bit requantization */
} hrt_mode;

typedef enum hrt_image_id {
  HRT_IMG_TRACE = 0,
  HRT_IMG_ACCUM = 1,
  /* flag, OR-ed with one of the above: this context's LOCAL rows even when it is joined to a
   * communicator -- not a collective (checkpoints of a partition, per-rank inspection) */
  HRT_IMG_LOCAL = 0x100
} hrt_image_id;
typedef enum hrt_format { HRT_FMT_RGBA8 = 0, HRT_FMT_RGBA32F = 1 } hrt_format;

typedef struct hrt_create_info {
  uint32_t width;      /* full image size (image_size[0]) */
  uint32_t height;     /* image_size[1] */
  int32_t device;      /* HIP device ordinal; -1 = the calling thread's current device */
  uint32_t mode;       /* hrt_mode */
  /* Image-space partition (multi-GPU row tiles).  Rows are grouped into tiles of
   * row_tile rows; this context renders tiles t with t % part_count == part_index and stores them
   * compacted (local row r <-> global row ((r / row_tile) * part_count + part_index) * row_tile
   * + r % row_tile).  part_count == 0 or 1 means the whole image. */
  uint32_t row_tile;
  uint32_t part_index;
  uint32_t part_count;
} hrt_create_info;

typedef struct hrt_layout {
  uint32_t width, height;   /* full image */
  uint32_t local_rows;      /* rows stored by this context (padded: equal on every part) */
  uint32_t row_tile, part_index, part_count;
  uint32_t mode;
} hrt_layout;

typedef struct hrt_stats {
  uint64_t segments;      /* world_hit calls (raytracing.glsl:317) over all traces since reset */
  uint64_t tri_tests;     /* ray-triangle tests (Sum over AABB-passing meshes of len) since reset */
  uint64_t traces;        /* non-init trace dispatches since reset */
  uint64_t accumulates;   /* combiner dispatches since reset */
  float last_trace_ms;    /* device time of the last trace dispatch (HIP events) */
  float total_trace_ms;   /* device time of all trace dispatches since reset */
  uint64_t wave_steps;    /* sum over work items of the item's longest per-lane segment count: lane
                             efficiency = segments / (64 * wave_steps).  A frame run of a multi-frame
                             launch (hrt_compute_n) is one item: each lane's segments summed over the
                             run's pixel-frames it took (any pixel of the tile), so the figure is
                             comparable between launches of the same shape only */
  uint32_t last_kernel;   /* hrt_kernel the last trace ran (HRT_KERNEL_AUTO resolved) */
  uint32_t last_block;    /* its workgroup size (threads) */
  uint32_t last_frames;   /* frames the last trace launch held (hrt_compute_n packs up to
                             HRT_OPT_FRAMES_PER_LAUNCH into one launch; 1 for hrt_trace) (ABI 4) */
  uint32_t reserved;
} hrt_stats;

/* The layouts every binding relies on (the Rust declarations in INTEGRATION.md are checked against
 * these by tests/test_rust_binding.py): std430 record sizes, the push block, and the host structs. */
#ifdef __cplusplus
#define HRT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define HRT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif
HRT_STATIC_ASSERT(sizeof(hrt_material) == 48, "std430 RayTracingMaterial");
HRT_STATIC_ASSERT(sizeof(hrt_ray) == 16, "std430 Ray");
HRT_STATIC_ASSERT(sizeof(hrt_sphere) == 64, "std430 Sphere");
HRT_STATIC_ASSERT(sizeof(hrt_triangle) == 64, "std430 Triangle");
HRT_STATIC_ASSERT(sizeof(hrt_mesh) == 80, "std430 Mesh");
HRT_STATIC_ASSERT(offsetof(hrt_mesh, len) == 28 && offsetof(hrt_mesh, material) == 32, "std430 Mesh layout");
HRT_STATIC_ASSERT(sizeof(hrt_push_constants) == 124, "push constant block (src/raytrace_pipeline.rs:125-139)");
HRT_STATIC_ASSERT(offsetof(hrt_push_constants, num_rays) == 80 && offsetof(hrt_push_constants, jitter_size) == 96 &&
                      offsetof(hrt_push_constants, height) == 120,
                  "push constant layout");
HRT_STATIC_ASSERT(sizeof(hrt_create_info) == 28 && offsetof(hrt_create_info, part_count) == 24, "hrt_create_info");
HRT_STATIC_ASSERT(sizeof(hrt_layout) == 28 && offsetof(hrt_layout, mode) == 24, "hrt_layout");
HRT_STATIC_ASSERT(sizeof(hrt_stats) == 64 && offsetof(hrt_stats, last_trace_ms) == 32 &&
                      offsetof(hrt_stats, wave_steps) == 40 && offsetof(hrt_stats, last_kernel) == 48 &&
                      offsetof(hrt_stats, last_frames) == 56,
                  "hrt_stats: 64 bytes since ABI 4");

typedef struct hrt_context hrt_context;

/* Trace kernel variants (HRT_OPT_KERNEL_VARIANT).  All produce byte-identical frames and counters;
 * they differ only in how much of the reference's brute-force work they prove unnecessary. */
typedef enum hrt_kernel {
  HRT_KERNEL_AUTO = 0,        /* BUNDLE below 256 mesh triangles; then, with a useful hierarchy
                                 (HRT_SCENE_BVH_SAH_MILLI <= 100), BUNDLE_WQ while it fits LDS; else
                                 BUNDLE_CULL_LDS while the triangle buffer fits LDS (else BUNDLE_CULL)
                                 below 4096 triangles (any count for a poor hierarchy); BUNDLE_BVH above */
  HRT_KERNEL_LITERAL = 1,     /* raytracing.glsl's loop shape, the full test on every triangle */
  HRT_KERNEL_BRUTE = 2,       /* fused sample/bounce loop, two-stage exact pre-test, triangles via SGPRs */
  HRT_KERNEL_BRUTE_LDS = 3,   /* BRUTE with the scene resident in LDS (falls back to BRUTE above 160 KiB) */
  HRT_KERNEL_BUNDLE = 4,      /* primary rays: lane-parallel bundle cull; bounces: deferred, BRUTE test */
  HRT_KERNEL_BUNDLE_CULL = 5, /* BUNDLE + lane-parallel origin-box / direction-cone cull of bounce rays */
  HRT_KERNEL_BUNDLE_BVH = 6,  /* BUNDLE + per-lane BVH traversal of bounce rays (hierarchy built by
                                 hrt_set_scene; falls back to BUNDLE_CULL above 64 meshes or 2^18
                                 mesh triangles) */
  HRT_KERNEL_BUNDLE_CULL_LDS = 7, /* BUNDLE_CULL with the triangle buffer resident in LDS (512/1024-thread
                                    workgroups; falls back to BUNDLE_CULL above ~3,300 triangles) */
  HRT_KERNEL_BUNDLE_BVH_LDS = 8,  /* BUNDLE_BVH with the hierarchy and triangles in LDS (1024-thread
                                    workgroups; falls back to BUNDLE_BVH when they exceed 160 KiB) */
  HRT_KERNEL_BUNDLE_WQ = 9        /* bounce segments through the hierarchy as (ray, node) / (ray, triangle)
                                    pairs on per-wave LDS stacks, 64 pairs per step (1024-thread
                                    persistent workgroups, nodes in LDS; falls back to BUNDLE_BVH_LDS when
                                    they do not fit or leaves exceed 4 triangles) */
} hrt_kernel;

/* Option keys for hrt_set_option. */
typedef enum hrt_option {
  /* trace kernel variant (hrt_kernel), default HRT_KERNEL_AUTO */
  HRT_OPT_KERNEL_VARIANT = 1,
  /* 1 = count segments / triangle tests on the device (default); 0 = off; 2 = also the bundle
   * kernels' cull diagnostics (hrt_get_diagnostics) */
  HRT_OPT_COUNTERS = 2,
  /* bundle kernel: a wave runs its bounce (non-primary) segments once this many lanes wait for one,
   * or when no lane has a primary segment left (1..64; default 0 = auto: 28 for BUNDLE_WQ (36 with per-node radii), else 48;
   * results do not depend on it) */
  HRT_OPT_SECONDARY_BATCH = 3,
  /* BUNDLE_BVH / BUNDLE_WQ: triangles per leaf of the hierarchy the next hrt_set_scene builds (1..16;
   * default 0 = auto: 2 up to 8192 mesh triangles, else 4) */
  HRT_OPT_BVH_LEAF_SIZE = 4,
  /* persistent kernels: a heavy tile (HRT_OPT_SPLIT_FACTOR) of the previous trace runs as this many
   * work items of 8/k rows each, scheduled first: at most this many (1 = off, 2, 4, 8; default 0 =
   * auto: BUNDLE_WQ 8, the others 1), 2 / 4 / 8 as the tile's cost passes 1 / 2 / 4 x the heavy
   * threshold.  The frame's time is set by its slowest tiles' sample chains; results do not depend on it. */
  HRT_OPT_SPLIT = 5,
  /* heavy tile: its cost in the previous trace exceeds this multiple of a resident wave's fair share
   * (sum of tile costs / resident waves), to an eighth octave (0: every tile is heavy; default -1 =
   * auto: BUNDLE_WQ 1.25 in a launch of several frames (hrt_compute_n), else 2 (3 when a resident
   * wave gets at most 6 tiles); the others 3 when there are more than 4 tiles per resident wave, else 1) */
  HRT_OPT_SPLIT_FACTOR = 6,
  /* persistent kernels: heavy tiles (as above) run at raised wave issue priority (1 default, 0 off;
   * libhip_raytrace_debug.so only: 2 = a planned trace runs ONLY the heavy tiles, the frame is
   * incomplete -- a diagnostics mode the production library rejects) */
  HRT_OPT_PRIORITY = 7,
  /* libhip_raytrace_debug.so only (latency experiments): persistent kernels launch workgroups for at
   * most this many CUs (0 = all).  The production library rejects the key. */
  HRT_OPT_GRID_CUS = 8,
  /* BUNDLE_CULL_LDS with HRT_OPT_SPLIT = 1: heavy tiles run cooperatively, every wave of a workgroup
   * on the same tile with the bounce cull's chunks dealt out over the waves (1 default, 0 off) */
  HRT_OPT_COOP = 9,
  /* BUNDLE_WQ: per-wave node-pair stack capacity (0 = what fits the LDS, default; else at most that,
   * rounded down to a multiple of 64, >= 128).  A step that could overflow it walks its pairs'
   * subtrees stacklessly instead; results do not depend on it (tests force the fallback with 128). */
  HRT_OPT_WQ_NODE_CAP = 10,
  /* persistent kernels: the first trace of a context (no previous tile costs) is preceded by a
   * 1-sample probe trace into a scratch image whose per-tile costs plan it (1 default, 0 off).
   * Frames, counters and the trace timing are unaffected. */
  HRT_OPT_PROBE = 11,
  /* hrt_compute_n: frames traced by one persistent launch (default 64, 1 = one launch per frame;
   * also capped at 1 GiB of frame images).  Results do not depend on it. */
  HRT_OPT_FRAMES_PER_LAUNCH = 12,
  /* hrt_trace: consecutive traces rotate over this many trace lanes (own stream + trace image) so that
   * the next frame's trace starts while the current one finishes (default 3; 0 or 1 = one lane, each
   * trace after the previous frame's combiner).  Results do not depend on it.  Diagnostics
   * (HRT_OPT_COUNTERS = 2) use one lane. */
  HRT_OPT_OVERLAP = 13,
  /* hrt_trace: a trace issued while another lane's trace still runs launches its persistent grid over
   * 1/value of the CUs (default 2; 1 = always every CU), so consecutive frames share the chip; a trace
   * issued to an idle GPU always gets every CU.  Results do not depend on it. */
  HRT_OPT_BUSY_SPLIT = 14,
  /* BUNDLE_WQ: children tested per node visit in the hierarchy the next hrt_set_scene builds (2 = the
   * binary tree, 3 or 4 = groups of up to that many collapsed from it; default 4).  Results do not
   * depend on it. */
  HRT_OPT_BVH_WIDTH = 15,
  /* BUNDLE_WQ: the radius R in a node's box margin a + b R (DESIGN.md "BVH cull": R bounds the ray
   * origin's distance to every vertex below the node).  1 = the origin's distance to the farthest
   * scene-box corner (once per ray); 2 = to the farthest corner of the node's own box (per node: more
   * arithmetic, tighter boxes where margins are wide); default 0 = auto: 2 when
   * HRT_SCENE_BVH_MARGIN_MILLI > 100 (cave), else 1.  Results do not depend on it. */
  HRT_OPT_WQ_NODE_RADIUS = 16,
  /* hrt_comm_init / collective hrt_read_image: milliseconds a rank waits for its peers in the status
   * agreement or the gather before it aborts the communicator (ncclCommAbort) and returns
   * HRT_ERR_COMM (default 120000; 0 = wait forever).  Per context. */
  HRT_OPT_COMM_TIMEOUT_MS = 17,
  /* hrt_trace + hrt_accumulate (the realtime loop): 1 = the combine of a traced frame is deferred --
   * the trace writes a slot of a ring of up to 16 frame images (allocated by the first trace, at most
   * 512 MiB) and the recorded frames are folded into the accumulator in frame order at the next
   * hrt_read_image / hrt_synchronize / hrt_stream / hrt_compute_n or when the ring is full, so no
   * combiner kernel waits between two traces; 0 (default) = one combiner dispatch per hrt_accumulate.
   * The bytes are the same either way.  Measured on island 1080p (r03b): 2.81-2.86 ms per frame
   * deferred against 2.53 immediate -- without the combiners pacing them, the three lanes' persistent
   * traces all run at once and contend for the CUs -- so it is off by default. */
  HRT_OPT_DEFER_COMBINE = 18,
  /* libhip_raytrace_debug.so only (tests): the value-th device allocation of the next hrt_set_scene
   * fails with HRT_ERR_OUT_OF_MEMORY (0 = off) */
  HRT_DEBUG_OPT_FAIL_ALLOC = 1001,
  /* libhip_raytrace_debug.so only (tests): BUNDLE_WQ's per-wave triangle-pair stack holds at most this
   * many pairs (0 = what fits; else >= 128, rounded down to a multiple of 64): bursts of kept leaves
   * beyond it are tested in place, the path the tests force with 128.  Results do not depend on it. */
  HRT_DEBUG_OPT_WQ_TRI_CAP = 1002,
  /* libhip_raytrace_debug.so only (tests): 1 = the persistent kernels' waves always take their work
   * items 4 at a time, so a multi-frame launch runs frame runs (an item's consecutive frames in one
   * pass, hrt_kernels.hip trace_fused_split) at any image size -- the full frames take them only while
   * many items remain.  Results do not depend on it. */
  HRT_DEBUG_OPT_GRAB_RUNS = 1003,
  /* builds with -DHRT_TIMELINE=1 only (tuning, tools/timeline.py): record, for each work item the persistent
   * kernels execute, its start / end time (s_memrealtime, 100 MHz), item word, frame, run length and
   * resident wave -- up to value records per launch (hrt_debug_timeline).  Other builds reject the key. */
  HRT_DEBUG_OPT_TIMELINE = 1004,
  /* libhip_raytrace_debug.so only (tests): an hrt_compute_n frame-image allocation of more than value
   * bytes fails as if the device were out of memory (0 = off), so the fallback from a whole launch's
   * images to the call's own frames runs.  Results do not depend on it. */
  HRT_DEBUG_OPT_STACK_LIMIT = 1005
} hrt_option;

/* Cull diagnostics of the bundle kernels (HRT_OPT_COUNTERS = 2), summed since the last reset. */
typedef enum hrt_diag {
  HRT_DIAG_PRIMARY_ITERS = 0,      /* wave iterations that ran the primary bundle path */
  HRT_DIAG_PRIMARY_CONSIDERED = 1, /* camera-facing triangles bounded (per wave) */
  HRT_DIAG_PRIMARY_SURVIVORS = 2,  /* ... of which survived the bundle cull */
  HRT_DIAG_BOUNCE_ITERS = 3,       /* wave iterations that ran a bounce batch */
  HRT_DIAG_BOUNCE_CONSIDERED = 4,  /* triangles bounded by the bounce pre-cull (per wave) */
  HRT_DIAG_BOUNCE_SURVIVORS = 5,   /* ... of which survived */
  HRT_DIAG_BOUNCE_LANES = 6,       /* lanes in bounce batches */
  HRT_DIAG_BVH_VISITS = 7,         /* BUNDLE_BVH: node visits summed over bounce lanes */
  HRT_DIAG_BVH_PRIM_TESTS = 8,     /* BUNDLE_BVH: leaf triangles reached, summed over bounce lanes */
  HRT_DIAG_BVH_BAND_TESTS = 9,     /* BUNDLE_BVH: grazing-band triangles tested, summed over bounce lanes */
  HRT_DIAG_PRIMARY_CYCLES = 10,    /* shader clocks per wave in the primary cull + tests, summed */
  HRT_DIAG_BOUNCE_CYCLES = 11,     /* ... in the bounce-batch path */
  HRT_DIAG_SHADE_CYCLES = 12,      /* ... in shading (scatter, RNG, colour) */
  HRT_DIAG_BOUNCE_STAGE2 = 13,     /* BUNDLE_CULL: bounce survivors with some lane's num_t > 0 */
  HRT_DIAG_BOUNCE_FRONT = 14,      /* ... and some such lane front-facing (dn < 0) */
  HRT_DIAG_BVH_TRIPS = 15,         /* BUNDLE_BVH: traversal loop iterations per bounce batch (wave), summed */
  HRT_DIAG_BVH_LEAF_TRIPS = 16,    /* ... of which some lane tested a leaf */
  HRT_DIAG_BAND_SCAN_MAX = 17,     /* BUNDLE_WQ: grazing-band entries of the longest list per bounce batch, summed */
  HRT_DIAG_BAND_SCAN_LEN = 18,     /* ... of every bounce lane's list, summed */
  HRT_DIAG_SKY_ITEMS = 19,         /* work items (waves) whose primary list is empty: every segment a miss */
  HRT_DIAG_SKY_CYCLES = 20,        /* ... their shader clocks per wave, summed */
  HRT_DIAG_PRIMARY_LANES = 21,     /* fused loop: primary lanes of the iterations that ran the primary path */
  HRT_DIAG_LOOP_ITERS = 22,        /* fused-loop iterations (waves) */
  HRT_DIAG_LIVE_LANES = 23,        /* ... and their lanes not yet done, summed */
  HRT_DIAG_WQ_STEPS_16 = 24,       /* BUNDLE_WQ: pair steps with 1-16 node pairs (waves) */
  HRT_DIAG_WQ_STEPS_32 = 25,       /* ... 17-32 */
  HRT_DIAG_WQ_STEPS_48 = 26,       /* ... 33-48 */
  HRT_DIAG_WQ_STEPS_64 = 27,       /* ... 49-64 */
  HRT_DIAG_WQ_MEMBERS = 28,        /* ... valid members of the popped node groups, summed (vs 4 slots each) */
  HRT_NUM_DIAG = 29
} hrt_diag;

/* What hrt_set_scene built for BUNDLE_BVH (hrt_get_scene_info). */
typedef enum hrt_scene_info {
  HRT_SCENE_BVH_NODES = 0,      /* hierarchy nodes */
  HRT_SCENE_BVH_PRIMS = 1,      /* (mesh, triangle) entries in its leaves */
  HRT_SCENE_BVH_IRREGULAR = 2,  /* entries outside the cull analysis (non-finite, normal != e1 x e2, ...):
                                   tested against every bounce ray */
  HRT_SCENE_BVH_NEVER = 3,      /* entries with a zero normal, which the reference never accepts */
  HRT_SCENE_BVH_BUILT = 4,      /* 1 if built (0: > 64 meshes or > 2^18 entries -> BUNDLE_BVH runs BUNDLE_CULL) */
  HRT_SCENE_BVH_BAND_ENTRIES = 5, /* grazing-band list entries over all direction cells */
  HRT_SCENE_BVH_SAH_MILLI = 6,  /* 1000 x the expected leaf triangle tests of a uniform random ray per
                                   entry (surface-area estimate): < ~30 for a useful hierarchy; large
                                   overlapping triangles (a soup) give ~500, and auto then culls instead */
  HRT_SCENE_BVH_MARGIN_MILLI = 7, /* 1000 x the mean over nodes of the box margin at R = the scene box's
                                     diagonal / the box's largest extent (island 26, cave 197) */
  HRT_NUM_SCENE_INFO = 8
} hrt_scene_info;

uint32_t hrt_abi_version(void);
/* Identity of the device code (hash of the kernel sources and build flags): measurement records
 * (profiles/pmc_traffic.json) carry it, so counters of an older kernel are never applied to this one. */
const char* hrt_build_id(void);
/* 1 for libhip_raytrace_debug.so (accepts the debug-only options above), 0 for the production library. */
uint32_t hrt_debug_build(void);
/* libhip_raytrace_debug.so: every device buffer of the context is surrounded by 4 KiB guard bands of a
 * fixed pattern; this synchronizes and counts the buffers and those whose bands were overwritten (a
 * kernel wrote outside its buffer).  The production library returns HRT_ERR_INVALID_ARGUMENT. */
hrt_status hrt_debug_check_guards(hrt_context* ctx, uint32_t* buffers, uint32_t* corrupted);

hrt_status hrt_create(const hrt_create_info* info, hrt_context** out_ctx);
void hrt_destroy(hrt_context* ctx);

/* Upload the scene.  rays: n_rays == width*height records indexed by global pixel id x + y*W
 * (or NULL / 0 to keep the rays of an earlier hrt_generate_rays / hrt_set_scene).
 * spheres/tris/meshes may be NULL when their count is 0 (the reference's "null object" records are
 * not needed).  Every mesh range must lie inside [0, n_tri).  Copies before returning. */
hrt_status hrt_set_scene(hrt_context* ctx, const hrt_ray* rays, uint32_t n_rays, const hrt_sphere* spheres,
                         uint32_t n_spheres, const hrt_triangle* tris, uint32_t n_tris, const hrt_mesh* meshes,
                         uint32_t n_meshes);

/* One dispatch of raytracing.glsl (or its init clear when pc->init != 0).  pc->width/height must
 * equal the context's; pc->num_spheres/num_meshes must not exceed the uploaded counts. */
hrt_status hrt_trace(hrt_context* ctx, const hrt_push_constants* pc);

/* One dispatch of image_combiner.glsl with next_image = this context's trace image. */
hrt_status hrt_accumulate(hrt_context* ctx, uint32_t frame);

/* The frame loop of compute_n_then_render (src/raytracing_app.rs:198-227, without the present):
 * for k = pc->rng_offset .. pc->rng_offset + n - 1, one trace of pc with rng_offset = k followed by
 * hrt_accumulate(ctx, k) -- byte for byte the result of that loop of hrt_trace / hrt_accumulate
 * calls, the trace image holding the last frame afterwards.  The persistent kernels trace up to
 * HRT_OPT_FRAMES_PER_LAUNCH frames in one launch (each frame its own image), so that the long
 * per-pixel sample chains of one frame run beside the other frames' work instead of ending each
 * frame alone; the combiner then folds the frames in order.  pc->init must be 0. */
hrt_status hrt_compute_n(hrt_context* ctx, const hrt_push_constants* pc, uint32_t n);

/* Copy an image (row-major, x 4 channels) into dst, host or device memory.  Blocking.
 *  - Without a communicator, or with image_id | HRT_IMG_LOCAL: this context's local rows
 *    (local_rows x width); bytes >= that in fmt.
 *  - With one (hrt_comm_init / hrt_comm_init_all): the FULL frame (height x width), gathered from every
 *    part with one ncclGather to rank 0 and un-interleaved on rank 0's device.  hrt_comm_init: a
 *    collective -- every rank calls it; dst / bytes are used on rank 0 only (may be NULL elsewhere).
 *    Every rank first agrees on the call's status: if any rank's arguments or local image are bad,
 *    every rank returns an error (HRT_ERR_COMM on the others) and none enters the gather; a peer that
 *    does not arrive within HRT_OPT_COMM_TIMEOUT_MS aborts the communicator (later calls: HRT_ERR_COMM).
 *    hrt_comm_init_all: any context of the group may call it alone; the frame lands in dst. */
hrt_status hrt_read_image(hrt_context* ctx, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes);

/* Checkpoint / resume (new): overwrite this context's local rows of the accumulated
 * image with bytes an earlier hrt_read_image(HRT_IMG_ACCUM, fmt) returned, in the context's own format
 * (HRT_FMT_RGBA8 for HRT_MODE_RGBA8, HRT_FMT_RGBA32F for HRT_MODE_RGBA32F; bytes = local_rows * width
 * * 4 or 16).  Continuing with frame numbers from the saved count reproduces an uninterrupted render
 * byte for byte.  src may be host or device memory. */
hrt_status hrt_load_accumulator(hrt_context* ctx, uint32_t fmt, const void* src, size_t bytes);

/* ---- multi-GPU framebuffer gather (RCCL is loaded on first use) ------------------- */
#define HRT_COMM_ID_BYTES 128 /* == sizeof(ncclUniqueId) */
typedef enum hrt_comm_transport {
  HRT_COMM_NONE = 0,        /* no communicator */
  HRT_COMM_RCCL = 1,        /* hrt_comm_init: one process / thread per GPU, ncclCommInitRank */
  HRT_COMM_RCCL_GROUP = 2,  /* hrt_comm_init_all on distinct devices: ncclCommInitAll, grouped ncclGather */
  HRT_COMM_DEVICE_COPY = 3  /* hrt_comm_init_all with contexts sharing a device: device-to-device copies */
} hrt_comm_transport;
/* A fresh RCCL unique id (ncclGetUniqueId) for hrt_comm_init; rank 0 creates it and shares the bytes. */
hrt_status hrt_comm_unique_id(uint8_t id[HRT_COMM_ID_BYTES]);
/* Joins ctx -- part `rank` of a `world`-way row-tile partition (hrt_create_info), or the whole image
 * when world == 1 -- to the communicator named by id.  Collective: blocks until all ranks joined.
 * The root's buffers are allocated before the communicator is created, and the ranks agree on the
 * outcome: a rank whose partition does not match or whose allocation failed makes every rank return
 * an error with no communicator (a NULL id, rank >= world or a missing RCCL cannot join at all). */
hrt_status hrt_comm_init(hrt_context* ctx, const uint8_t id[HRT_COMM_ID_BYTES], uint32_t rank, uint32_t world);
/* One process driving every part: ctxs[i] must be part i of n (same size, mode, row tile). */
hrt_status hrt_comm_init_all(hrt_context* const* ctxs, uint32_t n);
/* rank / world / hrt_comm_transport of ctx's communicator (0 / 1 / HRT_COMM_NONE without one). */
hrt_status hrt_comm_info(const hrt_context* ctx, uint32_t* rank, uint32_t* world, uint32_t* transport);

hrt_status hrt_get_layout(const hrt_context* ctx, hrt_layout* out);
hrt_status hrt_synchronize(hrt_context* ctx);
hrt_status hrt_get_stats(hrt_context* ctx, hrt_stats* out); /* synchronizes */
hrt_status hrt_reset_stats(hrt_context* ctx);
hrt_status hrt_get_diagnostics(hrt_context* ctx, uint64_t* out, uint32_t count); /* synchronizes */
/* Diagnostics (HRT_OPT_COUNTERS = 2): per 8x8 tile of the last trace, row-major over ceil(W/8) x
 * ceil(local_rows/8) tiles, 4 values: shader clocks (slowest work item), bounce iterations, bounce
 * survivor tests, bounce-phase clocks (the frame's critical path is its slowest tile).  count =
 * values (at most 4 x tiles). */
hrt_status hrt_get_tile_profile(hrt_context* ctx, uint64_t* out, uint32_t count);
/* Extension (no reference counterpart): out[i] = hrt_scene_info i for i < count, from the last
 * hrt_set_scene. */
hrt_status hrt_get_scene_info(hrt_context* ctx, uint32_t* out, uint32_t count);

/* On-device ray centres: fills the context's ray buffer with exactly the records
 * hrt_host_create_rays would produce (create_ray_subbuffer, src/raytrace_pipeline.rs:289-338) for
 * the context's width x height, without the host array or its upload.  A later hrt_set_scene may then
 * pass rays == NULL, n_rays == 0 to keep them.  default_jitter (may be NULL) receives :337's value. */
hrt_status hrt_generate_rays(hrt_context* ctx, float camera_focal_length, float viewport_height, const float up[3],
                             float* default_jitter);
/* Copies n (<= width*height) ray records of the context to host memory (verification). */
hrt_status hrt_read_rays(hrt_context* ctx, hrt_ray* out, uint32_t n);

/* Present interop (replaces the reference's image -> texture hand-off,
 * src/raytracing_app.rs:196-227): import memory the presenting API exported as an opaque POSIX fd
 * (Vulkan: VK_KHR_external_memory_fd, vkGetMemoryFdKHR on the staging buffer's memory, size = its
 * allocation size) and map [offset, offset + bytes) into *dev_ptr.  On success the fd belongs to
 * the import.  hrt_read_image(ctx, HRT_IMG_ACCUM, fmt, *dev_ptr, bytes) then writes each frame
 * there device to device.  Imports are released by hrt_release_external_memory or hrt_destroy. */
hrt_status hrt_import_external_memory(hrt_context* ctx, int fd, uint64_t size, uint64_t offset, uint64_t bytes,
                                      void** dev_ptr);
hrt_status hrt_release_external_memory(hrt_context* ctx, void* dev_ptr);
/* Test support for the above: device memory exported as an fd (HIP VMM) and the exporter's own
 * mapping of it (*ptr, *size rounded to the allocation granularity); hrt_debug_unmap_memory frees it. */
hrt_status hrt_debug_export_memory(int device, uint64_t bytes, int* fd, void** ptr, uint64_t* size);
hrt_status hrt_debug_unmap_memory(void* ptr, uint64_t size);
/* Test support: the kernels' shared-reciprocal normalize / division and sqrt paths (hrt_math.h) vs
 * the compiler's IEEE sequences, bit for bit, on n hashed inputs of device `device`.
 * out = {normalize mismatches, division mismatches, sqrt mismatches, fast-path cases}. */
hrt_status hrt_debug_math_check(int device, uint32_t n, uint32_t seed, uint64_t out[4]);
/* Test support: the kernels' RNG-domain shortcuts (sqrt of u01 draws and of -2 log(u01), sin/cos of the
 * RNG's angles without the range guard) against the general routines over all 2^32 states.
 * out = {sqrt mismatches, sincos mismatches, Lambertian-shortcut premise or folded-scaling violations
 * (hrt_kernels.hip adjust_dir, hrt_math.h u01_mul), values where the bare hardware square root differs from
 * the correctly rounded one on u01 draws, and on -2 log(u01)}. */
hrt_status hrt_debug_math_check_rng(int device, uint64_t out[5]);
/* Test support: the trace kernel's flattening of a wave's grazing-band lists (64 lanes, lane l's list
 * of n[l] entries starting at entry b0[l]) into 64-slot rounds.  owner_entry[(r * 64 + l) * 2 + {0, 1}] =
 * the owner lane and entry index of slot r * 64 + l (entry 0 past the end), r < rounds <= 4096;
 * *total = the slots in all (the sum of n). */
hrt_status hrt_debug_band_flatten(int device, const uint32_t n[64], const uint32_t b0[64], uint32_t rounds,
                                  uint32_t* owner_entry, uint32_t* total);
/* Test support: the pair traversal's cross-lane LDS handoffs (BUNDLE_WQ's stacks and closest-hit slots) on
 * a scripted run of one wave of 64 lanes over `rounds` <= 1024 rounds.  Slot l starts at seed[l].  Round r:
 * the top min(take[r], depth) stack entries are popped (popped[r * 64 + l] = the entry lane l < take
 * read, else 0xFFFFFFFF); lane l with tgt[r * 64 + l] < 64 reads that slot (seen[r * 64 + l]) and lowers it
 * to val[r * 64 + l] (u64 minimum); then lane l pushes cnt[r * 64 + l] <= 4 entries (r << 16 | l << 8 | k),
 * k-major over the lanes in lane order (while the stack holds at most 8192 - 256).  slots[l] = the final
 * slots, *depth = the final stack depth. */
hrt_status hrt_debug_wq_protocol(int device, uint32_t rounds, const uint32_t* cnt, const uint32_t* take,
                                 const uint32_t* tgt, const uint64_t* val, const uint64_t seed[64], uint32_t* popped,
                                 uint64_t* seen, uint64_t slots[64], uint32_t* depth);
/* Test support: the context's grazing-band structure as the device holds it (hrt_set_scene): the 32 B
 * per-cell records of BUNDLE_WQ (8 words: list start, length, first 12 entries as half-words; rec_words >=
 * 8 x cells), the offsets (off_words >= cells + 1) and the entry words (16-bit entries two to a word unless
 * wide; list_cap >= the words).  A NULL or too small buffer is skipped.  info = {cells, entries, wide,
 * records present}. */
hrt_status hrt_debug_band_records(hrt_context* ctx, uint32_t* rec, uint64_t rec_words, uint32_t* off, uint64_t off_words,
                                  uint32_t* list_words, uint64_t list_cap, uint32_t info[4]);
/* Tuning support: trace lane 0's per-8x8-tile costs as the last persistent launch on it recorded them
 * (shader clocks / 16 summed over the launch's frames; the next launch's plan input), count <= tiles. */
hrt_status hrt_debug_tile_costs(hrt_context* ctx, uint32_t* out, uint32_t count);
/* HRT_TIMELINE builds: the last trace launch's item records (4 words each: start, tile list built, end,
 * item | frame << 32 | run << 40 | sky << 47 | wave << 48), at most cap of them copied; *count = the records the launch wrote (<= the
 * HRT_DEBUG_OPT_TIMELINE capacity).  Other builds: HRT_ERR_INVALID_ARGUMENT. */
hrt_status hrt_debug_timeline(hrt_context* ctx, uint64_t* out, uint32_t cap, uint32_t* count);
hrt_status hrt_set_option(hrt_context* ctx, uint32_t key, int64_t value);

/* The context's HIP stream (hipStream_t), for callers that interoperate: work enqueued on it after
 * hrt_accumulate / hrt_compute_n follows them (a trace is joined by the combiner that reads it). */
void* hrt_stream(hrt_context* ctx);

/* Drops the library's process-wide host caches: the grazing-band lists of the last two scenes that
 * hrt_set_scene built (shared by every context of one scene so that a rank group or a test suite builds
 * them once; ~100 MB of host memory each for island, ~130 MB for cave).  Contexts keep working; the next
 * hrt_set_scene of such a scene rebuilds its lists (~0.5 s).  *freed_bytes (may be NULL) receives the
 * bytes released.  Thread-safe. */
hrt_status hrt_release_caches(uint64_t* freed_bytes);

/* Text of the last error on ctx (or of the last hrt_create failure when ctx is NULL). */
const char* hrt_last_error(const hrt_context* ctx);

#ifdef __cplusplus
}
#endif

#endif /* HIP_RAYTRACE_H */
