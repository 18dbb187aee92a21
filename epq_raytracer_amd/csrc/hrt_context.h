// hrt_context.h -- the context behind the C ABI (internal; shared by hrt_api.cpp and hrt_comm.cpp).
//
// A context owns everything the reference's RayTracePipeline + DiffusePipeline own on the Vulkan
// side (src/raytrace_pipeline.rs:31-46, src/diffuse.rs:22-30): the scene buffers, the trace image,
// the accumulated image and the queue -- plus counters, timing events and, for a row-tile partition,
// the RCCL communicator of the framebuffer gather.
//
// Streams.  `stream` (the context's stream, hrt_stream) carries every operation except the trace
// kernels of hrt_trace, which rotate over up to three trace lanes, each with its own stream, trace
// image, planner buffers and camera lists.  Frame k+1's trace does not depend on frame k's (only the
// combiner folds them, in order), so the next frame's trace starts on the CUs the current one's last
// work items leave idle (the reference's realtime loop, src/main.rs:41-57, dispatches one trace +
// combine per frame).  With three lanes frame k+2's trace waits only for frame k-1's combiner, which
// has long run, so a combiner that cannot get a CU while a persistent trace holds them all never
// stalls the next trace.  Ordering is by events only:
//   * a lane's trace waits for `lane.free` -- recorded on `stream` after the last operation that read
//     the lane's buffers (the combiner of the frame it traced before, a read_image, compute_n);
//   * an operation on `stream` that reads a lane's trace image waits for `lane.done`.
// Results are the serial loop's bytes by construction: the combiner runs in call order on one stream.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "hip_raytrace.h"

namespace hrt {

constexpr int kNumCounters = 3 + HRT_NUM_DIAG;  // segments, triangle tests, wave steps, diagnostics
constexpr int kLanes = 3;  // trace lanes (HRT_OPT_OVERLAP uses 1..kLanes of them)

struct EventPair {
  hipEvent_t start = nullptr, stop = nullptr;
  uint32_t frames = 1;  // frames the timed launch traced
};

// Device buffers of one uploaded scene (hrt_set_scene builds a complete new set, then swaps it in).
struct SceneBufs {
  float4* rays = nullptr;
  hrt_sphere* spheres = nullptr;
  hrt_triangle* tris = nullptr;
  float4* tri_nhat = nullptr;      // normalize(tri.normal) per triangle
  hrt_mesh* meshes = nullptr;
  float4* bvh_nodes = nullptr;     // BUNDLE_BVH hierarchy (hrt_bvh.h)
  float4* bvh_wq_nodes = nullptr;  // its 48 B node image for BUNDLE_WQ (nullptr above 65535 nodes)
  float4* bvh_prims = nullptr;
  float4* bvh_irregular = nullptr;
  uint32_t* bvh_band_off = nullptr;
  uint32_t* bvh_entries = nullptr;
  uint32_t* bvh_keybase = nullptr;
  void* bvh_band = nullptr;          // grazing-band entries: prim indices, 2 B (4 B when bvh_band_wide)
  float4* bvh_band_nhat = nullptr;   // per prim: n^ (the entries' pre-check)
  uint32_t bvh_band_wide = 0;
  uint32_t bvh_band_bits = 0;        // bit width of the longest band list
  // per trace lane: compacted camera-facing records of the frame (camera_lists)
  uint32_t* cam_meta[kLanes] = {};  // cam_start[n_meshes], cam_count[n_meshes]
  float4* cam_tris[kLanes] = {};    // 64 B each
  float4* cam_cull[kLanes] = {};    // 80 B each
  uint32_t n_spheres = 0, n_tris = 0, n_meshes = 0, cam_capacity = 0;
  uint32_t bvh_info[HRT_NUM_SCENE_INFO] = {};  // hrt_get_scene_info
  float bvh_abs_coef = 0.0f, bvh_rel_t = 0.0f, bvh_band_tau = 0.0f, bvh_band_a1 = 0.0f;
  uint32_t bvh_built_leaf = 4, bvh_dir_res = 64;
  uint32_t bvh_wq_n = 0, bvh_wq_width = 2;  // BUNDLE_WQ image: nodes, largest group
};
void free_scene(hrt_context* ctx, SceneBufs& s, bool keep_rays);

// One trace lane (see the header comment).
struct Lane {
  hipStream_t stream = nullptr;
  uint32_t* trace8 = nullptr;  // local_rows x W rgba8 (RGBA8 mode)
  float4* trace32 = nullptr;   // or float4 (RGBA32F mode)
  uint32_t* sched = nullptr;      // persistent kernels' scheduler words (hrt_kernels.h)
  uint32_t* tile_cost = nullptr;  // per 8x8 tile
  uint32_t* item_buf = nullptr;   // planned work items (tiles x 64)
  uint32_t* tl_cache = nullptr;   // the persistent kernels' whole-tile lists (tiles x hrt::kTlRecWords, tile_lists)
  bool plan_valid = false;        // tile_cost describes this lane's last trace (same scene)
  // the lane's camera lists (camera_lists) hold the records of this camera position (same scene):
  // a trace from the same position skips rebuilding them
  bool cam_ready = false;
  uint32_t cam_key[4] = {};       // cam_pos bits, num_meshes
  bool tl_ready = false;          // tl_cache holds the tile lists of tl_key's camera (tile_lists ran)
  uint32_t tl_key[14] = {};       // cam_pos, mat3 of cam_alignment_mat, jitter_size bits, num_meshes
  hipEvent_t done = nullptr;      // recorded on `stream` after each trace / clear of the lane
  hipEvent_t free = nullptr;      // recorded on the context stream after the lane's last reader
  bool done_set = false, free_set = false;
  void* image() const { return trace8 ? (void*)trace8 : (void*)trace32; }
};

// Multi-GPU framebuffer gather (hrt_comm.cpp).
struct Comm;
void comm_release(hrt_context* ctx);

// Pinned host staging for uploads: two chunks, filled by the CPU while the DMA engine drains the other.
struct Staging {
  void* buf[2] = {};
  hipEvent_t ev[2] = {};
  bool used[2] = {};
  size_t chunk = 0;
};

}  // namespace hrt

struct hrt_context {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t width = 0, height = 0, mode = HRT_MODE_RGBA8;
  uint32_t row_tile = 0, part_index = 0, part_count = 1, local_rows = 0;

  hrt::SceneBufs scene;
  uint32_t n_rays = 0;
  bool scene_set = false;

  hrt::Lane lane[hrt::kLanes];
  int cur_lane = 0;           // lane of the most recent trace (its image is "the trace image")
  bool lane_used = false;     // a trace / init has run since creation
  uint32_t busy_split = 2;    // HRT_OPT_BUSY_SPLIT: grid share of a trace launched while another runs
  uint32_t overlap = hrt::kLanes;  // HRT_OPT_OVERLAP: trace lanes in rotation (1: every trace on lane 0)

  uint32_t* accum8 = nullptr;
  float4* accum32 = nullptr;
  void* scratch = nullptr;  // format conversion for hrt_read_image
  unsigned long long* counters = nullptr;
  unsigned long long* tile_cycles = nullptr;  // diagnostics: shader clocks per 8x8 tile of the last trace
  uint32_t split_k = 0, split_prio = 1;  // split 0: auto (per kernel, launch_trace)
  int32_t split_factor = -1;  // auto
  uint32_t grid_cus = 0;  // HRT_OPT_GRID_CUS (debug build; 0: every CU)
  uint32_t coop = 1;      // HRT_OPT_COOP
  uint32_t wq_node_cap = 0;  // HRT_OPT_WQ_NODE_CAP (0 = auto)
  uint32_t probe = 1;        // HRT_OPT_PROBE
  uint32_t frames_per_launch = 64;  // HRT_OPT_FRAMES_PER_LAUNCH (hrt_compute_n)
  void* frame_stack = nullptr;      // hrt_compute_n: frame_stack_frames trace images
  uint32_t frame_stack_frames = 0;
  uint32_t frame_stack_failed = 0;  // a whole-launch stack of this many frames did not fit: not retried
  uint32_t num_cus = 0;
  uint32_t bvh_leaf = 0;  // HRT_OPT_BVH_LEAF_SIZE for the next hrt_set_scene (0 = auto, hrt_bvh.h)
  uint32_t wq_node_radius = 0;  // HRT_OPT_WQ_NODE_RADIUS (0 = auto)
  uint32_t bvh_width = 4;  // HRT_OPT_BVH_WIDTH (hrt_bvh.h kWqDefaultWidth) for the next hrt_set_scene
  int64_t debug_fail_alloc = 0;   // debug build: fail the n-th device allocation of the next hrt_set_scene
  uint32_t debug_grab_runs = 0;   // debug build: HRT_DEBUG_OPT_GRAB_RUNS
  int64_t debug_stack_limit = 0;  // debug build: HRT_DEBUG_OPT_STACK_LIMIT (frame-stack bytes that fit)
  uint32_t debug_wq_tri_cap = 0;  // debug build: HRT_DEBUG_OPT_WQ_TRI_CAP (triangle-pair stack capacity)
  unsigned long long* timeline = nullptr;  // HRT_TIMELINE builds: HRT_DEBUG_OPT_TIMELINE records (4 u64 each)
  uint32_t* timeline_count = nullptr;
  uint32_t timeline_cap = 0;

  int variant = 0;
  bool counters_on = true;
  bool diag_on = false;
  uint32_t sec_batch = 0;  // HRT_OPT_SECONDARY_BATCH (0 = auto per kernel, launch_trace)
  int last_kernel = 0, last_block = 0;  // what the last hrt_trace launched (hrt_stats)
  uint32_t last_frames = 0;             // ... and the frames that launch held

  struct Import {
    hipExternalMemory_t mem;
    void* ptr;
  };
  std::vector<Import> imports;           // hrt_import_external_memory (released by hrt_destroy)
  std::vector<hrt::EventPair> event_pool;  // reusable
  std::vector<hrt::EventPair> pending;     // recorded, not yet harvested (a ring of kMaxPending)
  uint64_t traces = 0, accumulates = 0;
  float last_ms = 0.0f, total_ms = 0.0f;

  struct Guard {
    void* ptr;
    size_t bytes;
  };
  std::vector<Guard> guards;  // debug build: guarded device allocations (hrt_debug_check_guards)
  hrt::Staging staging;
  // Deferred combiner (HRT_OPT_DEFER_COMBINE).  The accumulator is observable only through
  // hrt_read_image / hrt_stream / hrt_synchronize, so hrt_accumulate after an hrt_trace only records
  // (ring slot, frame): the trace wrote a slot of a ring of frame images instead of its lane's image,
  // and the recorded frames are folded in frame order (accumulate_frames_*, the hrt_compute_n combiner)
  // at the next observation or when the ring is full -- the per-frame combine's bytes, without a
  // combiner kernel queued between every two traces.
  void* ring = nullptr;        // ring_n frame images (context format), allocated by the first trace
  uint32_t ring_n = 0, ring_next = 0;
  int cur_slot = -1;           // ring slot of the most recent trace (-1: its lane's own image)
  struct Pend {
    uint32_t slot, frame;
  };
  std::vector<Pend> pend;      // recorded, not yet folded (consecutive slots and frames)
  hipEvent_t fold_done = nullptr;  // recorded on `stream` after the last fold (a slot's next trace waits)
  bool fold_set = false;
  uint32_t defer = 0;          // HRT_OPT_DEFER_COMBINE (off: measured slower, hip_raytrace.h)
  hrt::Comm* comm = nullptr;  // hrt_comm_init / hrt_comm_init_all
  uint32_t comm_timeout_ms = 120000;  // HRT_OPT_COMM_TIMEOUT_MS (0: wait forever)

  std::string err;

  size_t npix() const { return (size_t)local_rows * width; }
  size_t px_bytes() const { return mode == HRT_MODE_RGBA8 ? 4 : 16; }
  size_t num_tiles() const { return (size_t)((width + 7) / 8) * ((local_rows + 7) / 8); }
};

namespace hrt {

hrt_status fail(hrt_context* ctx, hrt_status st, const std::string& msg);
hrt_status hip_fail(hrt_context* ctx, hipError_t e, const char* what);
hrt_status bind(hrt_context* ctx);               // make the context's device current
hipError_t dev_alloc(hrt_context* ctx, void** p, size_t bytes);  // guarded in the debug build
void dev_free(hrt_context* ctx, void* p);
hrt_status join_lanes(hrt_context* ctx);         // the context stream waits for every lane's trace
hrt_status wait_lane(hrt_context* ctx, int l);   // ... for lane l's trace
hrt_status release_lane(hrt_context* ctx, int l);  // lane l's buffers are free after the stream's work so far
// Reads image_id of this context's local rows in its own pixel format, ordered on ctx->stream (the
// accumulator after every deferred combine has been folded).
const void* local_image(hrt_context* ctx, uint32_t image_id);
// Folds the deferred combines (hrt_context::pend) into the accumulator on ctx->stream.
hrt_status flush_combines(hrt_context* ctx);
// dst <- npix pixels at src (context format) converted to fmt via scratch, ordered on ctx->stream; blocking.
hrt_status copy_frame_out(hrt_context* ctx, const void* src, size_t npix, uint32_t fmt, void* dst, void* scratch);
// hrt_read_image on a context with a communicator (hrt_comm.cpp); arg = the caller's own argument
// check, agreed on by every rank of a process communicator before any of them gathers.
hrt_status comm_read_image(hrt_context* ctx, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes,
                           hrt_status arg);

}  // namespace hrt

#define HRT_HIP(ctx, call)                                        \
  do {                                                            \
    hipError_t e_ = (call);                                       \
    if (e_ != hipSuccess) return ::hrt::hip_fail((ctx), e_, #call); \
  } while (0)
