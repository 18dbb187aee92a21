// hrt_api.cpp -- the C ABI of libhip_raytrace.so (include/hip_raytrace.h).
//
// A context owns everything the reference's RayTracePipeline + DiffusePipeline own on the Vulkan
// side (src/raytrace_pipeline.rs:31-46, src/diffuse.rs:22-30): the scene buffers, the trace image,
// the accumulated image, the queue (here: one HIP stream) -- plus the device counters and timing
// events that the reference does not have.  Memory is allocated once per context; hrt_trace and
// hrt_accumulate only enqueue kernels (no allocation, no host sync), so a caller may capture them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "hip_raytrace.h"
#include "hrt_bvh.h"
#include "hrt_host.h"
#include "hrt_kernels.h"

static_assert(sizeof(hrt_material) == 48, "std430 RayTracingMaterial");
static_assert(sizeof(hrt_ray) == 16, "std430 Ray");
static_assert(sizeof(hrt_sphere) == 64, "std430 Sphere");
static_assert(sizeof(hrt_triangle) == 64, "std430 Triangle");
static_assert(sizeof(hrt_mesh) == 80, "std430 Mesh");
static_assert(sizeof(hrt_push_constants) == 124, "push constant block (src/raytrace_pipeline.rs:125-139)");
static_assert(offsetof(hrt_push_constants, num_rays) == 80, "push layout");
static_assert(offsetof(hrt_push_constants, height) == 120, "push layout");

namespace {

thread_local std::string g_create_error;
constexpr int kNumCounters = 3 + HRT_NUM_DIAG;  // segments, triangle tests, wave steps, diagnostics

struct EventPair {
  hipEvent_t start = nullptr, stop = nullptr;
  uint32_t frames = 1;  // frames the timed launch traced
};

}  // namespace

struct hrt_context {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t width = 0, height = 0, mode = HRT_MODE_RGBA8;
  uint32_t row_tile = 0, part_index = 0, part_count = 1, local_rows = 0;

  float4* rays = nullptr;
  hrt_sphere* spheres = nullptr;
  hrt_triangle* tris = nullptr;
  hrt_mesh* meshes = nullptr;
  uint32_t n_rays = 0, n_spheres = 0, n_tris = 0, n_meshes = 0;
  bool scene_set = false;

  uint32_t* trace8 = nullptr;
  uint32_t* accum8 = nullptr;
  float4* trace32 = nullptr;
  float4* accum32 = nullptr;
  void* scratch = nullptr;  // format conversion for hrt_read_image
  unsigned long long* counters = nullptr;
  unsigned long long* tile_cycles = nullptr;  // diagnostics: shader clocks per 8x8 tile of the last trace
  uint32_t* sched = nullptr;      // persistent kernels' scheduler words (hrt_kernels.h)
  uint32_t* tile_cost = nullptr;  // per 8x8 tile
  uint32_t* item_buf = nullptr;   // planned work items (tiles x 64: a heavy tile runs as up to 64 items)
  bool plan_valid = false;        // tile_cost describes the last trace (same size, persistent kernel)
  uint32_t split_k = 0, split_prio = 1;  // split 0: auto (per kernel, launch_trace)
  int32_t split_factor = -1;  // auto
  uint32_t grid_cus = 0;  // HRT_OPT_GRID_CUS (0: every CU)
  uint32_t coop = 1;      // HRT_OPT_COOP
  uint32_t wq_node_cap = 0;  // HRT_OPT_WQ_NODE_CAP (0 = auto)
  uint32_t probe = 1;        // HRT_OPT_PROBE
  uint32_t frames_per_launch = 64;  // HRT_OPT_FRAMES_PER_LAUNCH (hrt_compute_n)
  void* frame_stack = nullptr;      // hrt_compute_n: frame_stack_frames trace images
  uint32_t frame_stack_frames = 0;
  uint32_t num_cus = 0;
  uint32_t* cam_meta = nullptr;   // bundle variants: cam_start[n_meshes], cam_count[n_meshes]
  uint32_t cam_capacity = 0;      // sum of mesh lengths
  float4* cam_tris = nullptr;     // compacted camera-facing records (64 B each)
  float4* cam_cull = nullptr;     // bundle-cull records (80 B each)
  float4* bvh_nodes = nullptr;    // BUNDLE_BVH hierarchy (hrt_bvh.h), built by hrt_set_scene
  float4* bvh_wq_nodes = nullptr; // its 48 B node image for BUNDLE_WQ (nullptr above 65535 nodes)
  float4* bvh_prims = nullptr;
  float4* bvh_irregular = nullptr;
  uint32_t* bvh_band_off = nullptr;
  uint32_t* bvh_entries = nullptr;
  uint32_t* bvh_keybase = nullptr;
  uint2* bvh_band = nullptr;       // grazing-band entries, 8 B (hrt_bvh.h kBand*)
  uint32_t bvh_info[HRT_NUM_SCENE_INFO] = {};  // hrt_get_scene_info
  float bvh_abs_coef = 0.0f, bvh_rel_t = 0.0f;
  uint32_t bvh_leaf = 4;
  uint32_t bvh_built_leaf = 4;   // leaf size of the hierarchy the last hrt_set_scene built
  uint32_t bvh_dir_res = 64;     // direction cells per face edge of its band lists

  int variant = 0;
  bool counters_on = true;
  bool diag_on = false;
  uint32_t sec_batch = 0;  // HRT_OPT_SECONDARY_BATCH (0 = auto per kernel, launch_trace)
  int last_kernel = 0, last_block = 0;  // what the last hrt_trace launched (hrt_stats)

  struct Import {
    hipExternalMemory_t mem;
    void* ptr;
  };
  std::vector<Import> imports;           // hrt_import_external_memory (released by hrt_destroy)
  std::vector<EventPair> event_pool;     // reusable
  std::vector<EventPair> pending;        // recorded, not yet harvested
  uint64_t traces = 0, accumulates = 0;
  float last_ms = 0.0f, total_ms = 0.0f;

  std::string err;

  size_t npix() const { return (size_t)local_rows * width; }
  size_t num_tiles() const { return (size_t)((width + 7) / 8) * ((local_rows + 7) / 8); }
};

namespace {

hrt_status fail(hrt_context* ctx, hrt_status st, const std::string& msg) {
  if (ctx)
    ctx->err = msg;
  else
    g_create_error = msg;
  return st;
}

hrt_status hip_fail(hrt_context* ctx, hipError_t e, const char* what) {
  std::string msg = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
  return fail(ctx, e == hipErrorOutOfMemory ? HRT_ERR_OUT_OF_MEMORY : HRT_ERR_HIP, msg);
}

#define HRT_HIP(ctx, call)                                      \
  do {                                                          \
    hipError_t e_ = (call);                                     \
    if (e_ != hipSuccess) return hip_fail((ctx), e_, #call);    \
  } while (0)

// Make the context's device current for the calling thread (contexts may live on any device).
hrt_status bind(hrt_context* ctx) {
  HRT_HIP(ctx, hipSetDevice(ctx->device));
  return HRT_OK;
}

template <typename T>
void free_dev(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

hrt_status harvest_events(hrt_context* ctx) {
  for (auto& ev : ctx->pending) {
    HRT_HIP(ctx, hipEventSynchronize(ev.stop));
    float ms = 0.0f;
    HRT_HIP(ctx, hipEventElapsedTime(&ms, ev.start, ev.stop));
    ctx->last_ms = ms / (float)ev.frames;  // per frame
    ctx->total_ms += ms;
    ctx->event_pool.push_back(ev);
  }
  ctx->pending.clear();
  return HRT_OK;
}

}  // namespace

extern "C" uint32_t hrt_abi_version(void) { return HRT_ABI_VERSION; }

extern "C" hrt_status hrt_create(const hrt_create_info* info, hrt_context** out_ctx) {
  g_create_error.clear();
  if (!info || !out_ctx) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_create: null argument");
  *out_ctx = nullptr;
  if (info->mode != HRT_MODE_RGBA8 && info->mode != HRT_MODE_RGBA32F)
    return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_create: unknown mode");
  if (info->width == 0 || info->height == 0)
    return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_create: zero image size");
  if ((uint64_t)info->width * info->height > (1ull << 31))
    return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_create: image larger than 2^31 pixels");
  const uint32_t parts = info->part_count == 0 ? 1 : info->part_count;
  if (parts > 1 && (info->row_tile == 0 || info->part_index >= parts))
    return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_create: bad row-tile partition");

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(nullptr, HRT_ERR_NO_DEVICE, "hrt_create: no HIP device visible");
  int dev = info->device;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  if (dev >= ndev) return fail(nullptr, HRT_ERR_NO_DEVICE, "hrt_create: device ordinal out of range");

  auto* ctx = new hrt_context();
  ctx->device = dev;
  ctx->width = info->width;
  ctx->height = info->height;
  ctx->mode = info->mode;
  ctx->part_count = parts;
  if (parts > 1) {
    ctx->row_tile = info->row_tile;
    ctx->part_index = info->part_index;
    const uint32_t tiles = (info->height + info->row_tile - 1) / info->row_tile;
    const uint32_t tiles_per_part = (tiles + parts - 1) / parts;
    ctx->local_rows = tiles_per_part * info->row_tile;
  } else {
    ctx->row_tile = info->height;
    ctx->part_index = 0;
    ctx->local_rows = info->height;
  }

  auto bail = [&](hrt_status st) {
    std::string msg = ctx->err;
    hrt_destroy(ctx);
    return fail(nullptr, st, msg);
  };
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return bail(st);
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "hipStreamCreate"));
  const size_t np = ctx->npix();
  if (ctx->mode == HRT_MODE_RGBA8) {
    if ((e = hipMalloc((void**)&ctx->trace8, np * 4)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(trace)"));
    if ((e = hipMalloc((void**)&ctx->accum8, np * 4)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(accum)"));
  } else {
    if ((e = hipMalloc((void**)&ctx->trace32, np * 16)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(trace)"));
    if ((e = hipMalloc((void**)&ctx->accum32, np * 16)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(accum)"));
  }
  if ((e = hipMalloc(&ctx->scratch, np * 16)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(scratch)"));
  if ((e = hipMalloc((void**)&ctx->counters, kNumCounters * sizeof(unsigned long long))) != hipSuccess)
    return bail(hip_fail(ctx, e, "hipMalloc(counters)"));
  {
    const size_t tiles = ctx->num_tiles();
    if ((e = hipMalloc((void**)&ctx->sched, 256 * 4)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(sched)"));
    if ((e = hipMalloc((void**)&ctx->tile_cost, (tiles ? tiles : 1) * 4)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipMalloc(tile costs)"));
    if ((e = hipMalloc((void**)&ctx->item_buf, (tiles ? tiles : 1) * 64 * 4)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipMalloc(items)"));
  }
  {
    int cus = 0;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipDeviceGetAttribute(CUs)"));
    ctx->num_cus = cus > 0 ? (uint32_t)cus : 1u;
  }
  if ((e = hipMemsetAsync(ctx->counters, 0, kNumCounters * sizeof(unsigned long long), ctx->stream)) != hipSuccess)
    return bail(hip_fail(ctx, e, "hipMemset(counters)"));
  // Fresh images read as the cleared state (0,0,0,1) until the first dispatch writes them.
  if ((e = hrt::launch_clear(ctx->trace8, ctx->trace32, np, ctx->stream)) != hipSuccess)
    return bail(hip_fail(ctx, e, "clear"));
  if ((e = hrt::launch_clear(ctx->accum8, ctx->accum32, np, ctx->stream)) != hipSuccess)
    return bail(hip_fail(ctx, e, "clear"));
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return bail(hip_fail(ctx, e, "hipStreamSynchronize"));
  *out_ctx = ctx;
  return HRT_OK;
}

extern "C" void hrt_destroy(hrt_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  free_dev(ctx->rays);
  free_dev(ctx->spheres);
  free_dev(ctx->tris);
  free_dev(ctx->meshes);
  free_dev(ctx->trace8);
  free_dev(ctx->accum8);
  free_dev(ctx->trace32);
  free_dev(ctx->accum32);
  free_dev(ctx->scratch);
  free_dev(ctx->counters);
  free_dev(ctx->tile_cycles);
  free_dev(ctx->cam_meta);
  free_dev(ctx->cam_tris);
  free_dev(ctx->cam_cull);
  free_dev(ctx->bvh_nodes);
  free_dev(ctx->bvh_wq_nodes);
  free_dev(ctx->bvh_prims);
  free_dev(ctx->bvh_irregular);
  free_dev(ctx->bvh_band_off);
  free_dev(ctx->bvh_band);
  free_dev(ctx->bvh_entries);
  free_dev(ctx->bvh_keybase);
  free_dev(ctx->sched);
  free_dev(ctx->tile_cost);
  free_dev(ctx->item_buf);
  free_dev(ctx->frame_stack);
  for (auto& im : ctx->imports) (void)hipDestroyExternalMemory(im.mem);
  for (auto& ev : ctx->event_pool) {
    (void)hipEventDestroy(ev.start);
    (void)hipEventDestroy(ev.stop);
  }
  for (auto& ev : ctx->pending) {
    (void)hipEventDestroy(ev.start);
    (void)hipEventDestroy(ev.stop);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

namespace {

template <typename T>
hrt_status upload(hrt_context* ctx, T*& dst, const T* src, uint32_t n, const char* what) {
  free_dev(dst);
  const size_t bytes = (size_t)(n ? n : 1) * sizeof(T);  // keep a valid pointer for empty lists
  HRT_HIP(ctx, hipMalloc((void**)&dst, bytes));
  if (n) HRT_HIP(ctx, hipMemcpyAsync(dst, src, (size_t)n * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  (void)what;
  return HRT_OK;
}

}  // namespace

extern "C" hrt_status hrt_set_scene(hrt_context* ctx, const hrt_ray* rays, uint32_t n_rays, const hrt_sphere* spheres,
                                    uint32_t n_spheres, const hrt_triangle* tris, uint32_t n_tris,
                                    const hrt_mesh* meshes, uint32_t n_meshes) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  const bool keep_rays = !rays && n_rays == 0 && ctx->rays && ctx->n_rays == (uint64_t)ctx->width * ctx->height;
  if (!keep_rays && ((uint64_t)n_rays != (uint64_t)ctx->width * ctx->height || !rays))
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT,
                "hrt_set_scene: need width*height rays (or NULL after hrt_generate_rays)");
  if ((n_spheres && !spheres) || (n_tris && !tris) || (n_meshes && !meshes))
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_set_scene: null record array with nonzero count");
  for (uint32_t m = 0; m < n_meshes; ++m) {
    if ((uint64_t)meshes[m].first_index + meshes[m].len > n_tris)
      return fail(ctx, HRT_ERR_INVALID_ARGUMENT,
                  "hrt_set_scene: mesh " + std::to_string(m) + " triangle range exceeds the triangle buffer");
  }
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  static_assert(sizeof(float4) == sizeof(hrt_ray), "ray record");
  if (!keep_rays &&
      (st = upload(ctx, ctx->rays, reinterpret_cast<const float4*>(rays), n_rays, "rays")) != HRT_OK)
    return st;
  if ((st = upload(ctx, ctx->spheres, spheres, n_spheres, "spheres")) != HRT_OK) return st;
  if ((st = upload(ctx, ctx->tris, tris, n_tris, "triangles")) != HRT_OK) return st;
  if ((st = upload(ctx, ctx->meshes, meshes, n_meshes, "meshes")) != HRT_OK) return st;
  uint64_t cap = 0;
  for (uint32_t m = 0; m < n_meshes; ++m) cap += meshes[m].len;
  if (cap > 0xFFFFFFFFull) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_set_scene: too many mesh triangles");
  // bundle-variant buffers: per-frame compacted camera-facing records (filled by camera_lists)
  free_dev(ctx->cam_meta);
  free_dev(ctx->cam_tris);
  free_dev(ctx->cam_cull);
  HRT_HIP(ctx, hipMalloc((void**)&ctx->cam_meta, (size_t)(n_meshes ? 2 * n_meshes : 2) * 4));
  HRT_HIP(ctx, hipMalloc((void**)&ctx->cam_tris, (size_t)(cap ? cap : 1) * 64));
  HRT_HIP(ctx, hipMalloc((void**)&ctx->cam_cull, (size_t)(cap ? cap : 1) * 80));
  ctx->cam_capacity = (uint32_t)cap;
  // bounce-segment hierarchy (BUNDLE_BVH)
  hrt::BvhHost bvh;
  const bool built = hrt::build_bvh(tris, n_tris, meshes, n_meshes, ctx->bvh_leaf, bvh);
  free_dev(ctx->bvh_nodes);
  free_dev(ctx->bvh_wq_nodes);
  free_dev(ctx->bvh_prims);
  free_dev(ctx->bvh_irregular);
  free_dev(ctx->bvh_band_off);
  free_dev(ctx->bvh_band);
  free_dev(ctx->bvh_entries);
  free_dev(ctx->bvh_keybase);
  if (built) {
    auto up = [&](auto*& dst, const auto& v) -> hrt_status {
      const size_t bytes = v.size() * sizeof(v[0]);
      HRT_HIP(ctx, hipMalloc((void**)&dst, bytes ? bytes : 16));
      if (bytes) HRT_HIP(ctx, hipMemcpyAsync(dst, v.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
      return HRT_OK;
    };
    if ((st = up(ctx->bvh_nodes, bvh.nodes)) != HRT_OK) return st;
    if (bvh.wq_ok && (st = up(ctx->bvh_wq_nodes, bvh.wq_nodes)) != HRT_OK) return st;
    if ((st = up(ctx->bvh_prims, bvh.prims)) != HRT_OK) return st;
    if ((st = up(ctx->bvh_irregular, bvh.irregular)) != HRT_OK) return st;
    if ((st = up(ctx->bvh_band_off, bvh.band_off)) != HRT_OK) return st;
    if ((st = up(ctx->bvh_band, bvh.band_list)) != HRT_OK) return st;  // 8 B entries
    if ((st = up(ctx->bvh_entries, bvh.entries)) != HRT_OK) return st;
    if ((st = up(ctx->bvh_keybase, bvh.key_base)) != HRT_OK) return st;
  }
  ctx->bvh_info[0] = bvh.n_nodes;
  ctx->bvh_info[1] = bvh.n_prims;
  ctx->bvh_info[2] = bvh.n_irregular;
  ctx->bvh_info[3] = bvh.n_never;
  ctx->bvh_info[4] = built ? 1u : 0u;
  ctx->bvh_abs_coef = bvh.abs_coef;
  ctx->bvh_dir_res = bvh.dir_res;
  ctx->bvh_built_leaf = std::max(1u, std::min(ctx->bvh_leaf, hrt::kBvhMaxLeafCount));  // leaves hold at most this
  ctx->bvh_rel_t = bvh.rel_t;
  ctx->bvh_info[5] = (uint32_t)(bvh.band_list.size() / 2);
  ctx->bvh_info[6] = (uint32_t)std::min(1e9, bvh.sah_tri_frac * 1000.0 + 0.5);
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));  // host arrays are only borrowed
  if (!keep_rays) ctx->n_rays = n_rays;
  ctx->plan_valid = false;  // tile costs describe the old scene
  ctx->n_spheres = n_spheres;
  ctx->n_tris = n_tris;
  ctx->n_meshes = n_meshes;
  ctx->scene_set = true;
  return HRT_OK;
}

namespace {

// Validates a dispatch's push block against the context (hrt_trace / hrt_compute_n).
hrt_status check_dispatch(hrt_context* ctx, const hrt_push_constants* pc, const char* who) {
  if (!ctx->scene_set) return fail(ctx, HRT_ERR_NO_SCENE, std::string(who) + ": hrt_set_scene has not been called");
  if (pc->width != ctx->width || pc->height != ctx->height)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, std::string(who) + ": push constant width/height differ from the context");
  if (pc->num_spheres < 0 || (uint32_t)pc->num_spheres > ctx->n_spheres || pc->num_meshes < 0 ||
      (uint32_t)pc->num_meshes > ctx->n_meshes)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, std::string(who) + ": num_spheres/num_meshes exceed the uploaded scene");
  return HRT_OK;
}

// The kernel argument block of a dispatch of pc into the context's trace image.
hrt::TraceParams make_params(hrt_context* ctx, const hrt_push_constants* pc) {
  hrt::TraceParams p{};
  p.rays = ctx->rays;
  p.spheres = ctx->spheres;
  p.tris = ctx->tris;
  p.meshes = ctx->meshes;
  p.img8 = ctx->trace8;
  p.img32 = ctx->trace32;
  p.counters = ctx->counters_on ? ctx->counters : nullptr;
  p.diag = ctx->diag_on ? ctx->counters + 3 : nullptr;
  p.tile_cycles = ctx->diag_on ? ctx->tile_cycles : nullptr;
  p.pc = *pc;
  p.local_rows = ctx->local_rows;
  p.row_tile = ctx->row_tile;
  p.part_index = ctx->part_index;
  p.part_count = ctx->part_count;
  p.n_tris = ctx->n_tris;
  p.cam_start = ctx->cam_meta;
  p.cam_count = ctx->cam_meta + ctx->n_meshes;
  p.cam_list_capacity = ctx->cam_capacity;
  p.cam_tris = ctx->cam_tris;
  p.cam_cull = ctx->cam_cull;
  p.sec_batch = ctx->sec_batch;
  p.sched = ctx->sched;
  p.tile_cost = ctx->tile_cost;
  p.item_buf = ctx->item_buf;
  p.split_k = ctx->split_k;
  p.split_factor = ctx->split_factor;
  p.split_prio = ctx->split_prio;
  p.coop = ctx->coop;
  p.wq_ncap = ctx->wq_node_cap;  // request; launch_trace sizes the stacks
  p.plan_valid = ctx->plan_valid ? 1u : 0u;
  p.num_cus = ctx->grid_cus ? std::min(ctx->grid_cus, ctx->num_cus) : ctx->num_cus;
  p.bvh_nodes = ctx->bvh_info[4] ? ctx->bvh_nodes : nullptr;
  p.bvh_wq_nodes = ctx->bvh_info[4] ? ctx->bvh_wq_nodes : nullptr;
  p.bvh_prims = ctx->bvh_prims;
  p.bvh_irregular = ctx->bvh_irregular;
  p.bvh_band_off = ctx->bvh_band_off;
  p.bvh_dir_res = ctx->bvh_dir_res;
  p.bvh_sah_milli = ctx->bvh_info[6];
  p.bvh_band = ctx->bvh_band;
  p.bvh_entries = ctx->bvh_entries;
  p.bvh_keybase = ctx->bvh_keybase;
  p.bvh_n_prims = ctx->bvh_info[1];
  p.bvh_n_meshes = ctx->n_meshes;
  p.bvh_n_nodes = ctx->bvh_info[0];
  p.bvh_abs_coef = ctx->bvh_abs_coef;
  p.bvh_rel_t = ctx->bvh_rel_t;
  p.bvh_n_irregular = ctx->bvh_info[2];
  p.bvh_max_leaf = ctx->bvh_built_leaf;
  p.n_frames = 1;
  p.frame_stride = ctx->npix();
  return p;
}

bool persistent_kernel(int k) {
  return k == HRT_KERNEL_BUNDLE_WQ || k == HRT_KERNEL_BUNDLE_CULL_LDS || k == HRT_KERNEL_BUNDLE_BVH_LDS;
}

// One trace launch of p.n_frames frames (timed by a HIP event pair counted as that many traces).
hrt_status launch_frames(hrt_context* ctx, hrt::TraceParams& p) {
  if (ctx->diag_on && !ctx->tile_cycles) {
    HRT_HIP(ctx, hipMalloc((void**)&ctx->tile_cycles, ctx->num_tiles() * 4 * sizeof(unsigned long long)));
    p.tile_cycles = ctx->tile_cycles;
  }
  if (ctx->diag_on)
    HRT_HIP(ctx, hipMemsetAsync(ctx->tile_cycles, 0, ctx->num_tiles() * 4 * sizeof(unsigned long long), ctx->stream));
  const int variant = ctx->variant;
  EventPair ev;
  if (!ctx->event_pool.empty()) {
    ev = ctx->event_pool.back();
    ctx->event_pool.pop_back();
  } else {
    HRT_HIP(ctx, hipEventCreate(&ev.start));
    HRT_HIP(ctx, hipEventCreate(&ev.stop));
  }
  ev.frames = p.n_frames > 1 ? p.n_frames : 1u;
  // First trace of a persistent kernel (no tile costs yet): a 1-sample probe trace into the scratch
  // image measures the tiles' relative costs so that this trace already follows a plan (HRT_OPT_PROBE).
  const int resolved = hrt::resolve_variant(p, variant);
  if (ctx->probe && !ctx->plan_valid && ctx->num_tiles() >= 1024 && persistent_kernel(resolved)) {
    hrt::TraceParams q = p;
    q.pc.num_samples = 1;
    q.n_frames = 1;
    q.img8 = ctx->trace8 ? reinterpret_cast<uint32_t*>(ctx->scratch) : nullptr;
    q.img32 = ctx->trace32 ? reinterpret_cast<float4*>(ctx->scratch) : nullptr;
    q.counters = nullptr;
    q.diag = nullptr;
    q.tile_cycles = nullptr;
    q.probe = 1u;
    int ran = 0, blk = 0;
    if (hipError_t pe = hrt::launch_trace(q, variant, ctx->stream, &ran, &blk); pe != hipSuccess) {
      ctx->event_pool.push_back(ev);
      return hip_fail(ctx, pe, "probe trace launch");
    }
    p.plan_valid = 1u;
  }
  HRT_HIP(ctx, hipEventRecord(ev.start, ctx->stream));
  hipError_t e = hrt::launch_trace(p, variant, ctx->stream, &ctx->last_kernel, &ctx->last_block);
  // the persistent kernels recorded this trace's tile costs: the next one can follow a plan
  ctx->plan_valid = e == hipSuccess && persistent_kernel(ctx->last_kernel);
  if (e != hipSuccess) {
    ctx->event_pool.push_back(ev);
    return hip_fail(ctx, e, "trace kernel launch");
  }
  HRT_HIP(ctx, hipEventRecord(ev.stop, ctx->stream));
  ctx->pending.push_back(ev);
  ctx->traces += ev.frames;
  if (ctx->pending.size() > 256) return harvest_events(ctx);  // bound the pending list
  return HRT_OK;
}

}  // namespace

extern "C" hrt_status hrt_trace(hrt_context* ctx, const hrt_push_constants* pc) {
  if (!ctx || !pc) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  if (pc->init) {  // RayTracePipeline::init, src/raytrace_pipeline.rs:190-213
    HRT_HIP(ctx, hrt::launch_clear(ctx->trace8, ctx->trace32, ctx->npix(), ctx->stream));
    return HRT_OK;
  }
  if ((st = check_dispatch(ctx, pc, "hrt_trace")) != HRT_OK) return st;
  hrt::TraceParams p = make_params(ctx, pc);
  return launch_frames(ctx, p);
}

extern "C" hrt_status hrt_compute_n(hrt_context* ctx, const hrt_push_constants* pc, uint32_t n) {
  if (!ctx || !pc) return HRT_ERR_INVALID_ARGUMENT;
  if (pc->init) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_compute_n: init dispatches go through hrt_trace");
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  if ((st = check_dispatch(ctx, pc, "hrt_compute_n")) != HRT_OK) return st;
  hrt::TraceParams p = make_params(ctx, pc);
  const size_t np = ctx->npix(), px_bytes = ctx->trace8 ? 4 : 16;
  // Frames per launch: up to HRT_OPT_FRAMES_PER_LAUNCH, and at most 1 GiB of frame images.
  const uint32_t cap = (uint32_t)std::max<size_t>(
      1, std::min<size_t>(ctx->frames_per_launch, ((size_t)1 << 30) / std::max<size_t>(np * px_bytes, 1)));
  const bool batch = persistent_kernel(hrt::resolve_variant(p, ctx->variant)) && cap > 1 && n > 1;
  if (batch && ctx->frame_stack_frames < std::min(cap, n)) {
    free_dev(ctx->frame_stack);
    ctx->frame_stack_frames = 0;
    HRT_HIP(ctx, hipMalloc(&ctx->frame_stack, (size_t)std::min(cap, n) * np * px_bytes));
    ctx->frame_stack_frames = std::min(cap, n);
  }
  for (uint32_t done = 0; done < n;) {
    // near-equal launches: ceil(remaining / cap) of them
    const uint32_t left = n - done, launches = batch ? (left + cap - 1) / cap : left;
    const uint32_t nf = (left + launches - 1) / launches;
    hrt::TraceParams q = p;
    q.pc.rng_offset = pc->rng_offset + done;  // u32, wrapping like the per-frame loop's pushes
    q.n_frames = nf;
    q.plan_valid = ctx->plan_valid ? 1u : 0u;
    if (nf > 1) {
      q.img8 = ctx->trace8 ? reinterpret_cast<uint32_t*>(ctx->frame_stack) : nullptr;
      q.img32 = ctx->trace32 ? reinterpret_cast<float4*>(ctx->frame_stack) : nullptr;
    }
    if ((st = launch_frames(ctx, q)) != HRT_OK) return st;
    for (uint32_t f = 0; f < nf; ++f) {  // DiffusePipeline::next_frame(frame) in frame order
      const uint32_t* t8 = nf > 1 && q.img8 ? q.img8 + f * np : ctx->trace8;
      const float4* t32 = nf > 1 && q.img32 ? q.img32 + f * np : ctx->trace32;
      HRT_HIP(ctx, hrt::launch_accumulate(ctx->accum8, t8, ctx->accum32, t32, np, q.pc.rng_offset + f, ctx->stream));
      ctx->accumulates++;
    }
    if (nf > 1)  // the trace image holds the last frame, as after the per-frame loop
      HRT_HIP(ctx, hipMemcpyAsync(ctx->trace8 ? (void*)ctx->trace8 : (void*)ctx->trace32,
                                  static_cast<const char*>(ctx->frame_stack) + (size_t)(nf - 1) * np * px_bytes,
                                  np * px_bytes, hipMemcpyDeviceToDevice, ctx->stream));
    done += nf;
  }
  return HRT_OK;
}

extern "C" hrt_status hrt_accumulate(hrt_context* ctx, uint32_t frame) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  HRT_HIP(ctx, hrt::launch_accumulate(ctx->accum8, ctx->trace8, ctx->accum32, ctx->trace32, ctx->npix(), frame,
                                      ctx->stream));
  ctx->accumulates++;
  return HRT_OK;
}

extern "C" hrt_status hrt_read_image(hrt_context* ctx, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes) {
  if (!ctx || !dst) return HRT_ERR_INVALID_ARGUMENT;
  if (image_id != HRT_IMG_TRACE && image_id != HRT_IMG_ACCUM)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: unknown image id");
  if (fmt != HRT_FMT_RGBA8 && fmt != HRT_FMT_RGBA32F)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: unknown format");
  const size_t np = ctx->npix();
  const size_t need = np * (fmt == HRT_FMT_RGBA8 ? 4 : 16);
  if (bytes < need) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: destination too small");
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  const bool accum = image_id == HRT_IMG_ACCUM;
  const void* src = nullptr;
  if (ctx->mode == HRT_MODE_RGBA8) {
    const uint32_t* s8 = accum ? ctx->accum8 : ctx->trace8;
    if (fmt == HRT_FMT_RGBA8) {
      src = s8;
    } else {
      HRT_HIP(ctx, hrt::launch_convert(s8, (float4*)ctx->scratch, nullptr, nullptr, np, ctx->stream));
      src = ctx->scratch;
    }
  } else {
    const float4* s32 = accum ? ctx->accum32 : ctx->trace32;
    if (fmt == HRT_FMT_RGBA32F) {
      src = s32;
    } else {
      HRT_HIP(ctx, hrt::launch_convert(nullptr, nullptr, s32, (uint32_t*)ctx->scratch, np, ctx->stream));
      src = ctx->scratch;
    }
  }
  HRT_HIP(ctx, hipMemcpyAsync(dst, src, need, hipMemcpyDefault, ctx->stream));
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HRT_OK;
}

extern "C" hrt_status hrt_get_layout(const hrt_context* ctx, hrt_layout* out) {
  if (!ctx || !out) return HRT_ERR_INVALID_ARGUMENT;
  out->width = ctx->width;
  out->height = ctx->height;
  out->local_rows = ctx->local_rows;
  out->row_tile = ctx->row_tile;
  out->part_index = ctx->part_index;
  out->part_count = ctx->part_count;
  out->mode = ctx->mode;
  return HRT_OK;
}

extern "C" hrt_status hrt_synchronize(hrt_context* ctx) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HRT_OK;
}

extern "C" hrt_status hrt_get_stats(hrt_context* ctx, hrt_stats* out) {
  if (!ctx || !out) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if ((st = harvest_events(ctx)) != HRT_OK) return st;
  unsigned long long c[kNumCounters] = {};
  HRT_HIP(ctx, hipMemcpy(c, ctx->counters, sizeof c, hipMemcpyDeviceToHost));
  out->segments = c[0];
  out->tri_tests = c[1];
  out->traces = ctx->traces;
  out->accumulates = ctx->accumulates;
  out->wave_steps = c[2];
  out->last_kernel = (uint32_t)ctx->last_kernel;
  out->last_block = (uint32_t)ctx->last_block;
  out->last_trace_ms = ctx->last_ms;
  out->total_trace_ms = ctx->total_ms;
  return HRT_OK;
}

extern "C" hrt_status hrt_get_diagnostics(hrt_context* ctx, uint64_t* out, uint32_t count) {
  if (!ctx || !out || count > HRT_NUM_DIAG) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  unsigned long long c[kNumCounters] = {};
  HRT_HIP(ctx, hipMemcpy(c, ctx->counters, sizeof c, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < count; ++i) out[i] = c[3 + i];
  return HRT_OK;
}

extern "C" hrt_status hrt_generate_rays(hrt_context* ctx, float camera_focal_length, float viewport_height,
                                        const float up[3], float* default_jitter) {
  if (!ctx || !up) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  float first[3], px[3], py[3];
  const uint32_t n = hrt_host_ray_grid(ctx->width, ctx->height, camera_focal_length, viewport_height, up, first, px,
                                       py, default_jitter);
  const size_t want = (size_t)ctx->width * ctx->height;
  if (!ctx->rays || ctx->n_rays != want) {
    free_dev(ctx->rays);
    HRT_HIP(ctx, hipMalloc((void**)&ctx->rays, (want ? want : 1) * sizeof(float4)));
  }
  if (n) HRT_HIP(ctx, hrt::launch_make_rays(ctx->rays, ctx->width, ctx->height, first, px, py, ctx->stream));
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->n_rays = (uint32_t)want;
  return HRT_OK;
}

extern "C" hrt_status hrt_import_external_memory(hrt_context* ctx, int fd, uint64_t size, uint64_t offset,
                                                 uint64_t bytes, void** dev_ptr) {
  if (!ctx || fd < 0 || !dev_ptr || bytes == 0 || offset + bytes > size)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_import_external_memory: bad fd / size / range");
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  hipExternalMemoryHandleDesc desc{};
  desc.type = hipExternalMemoryHandleTypeOpaqueFd;
  desc.handle.fd = fd;
  desc.size = size;
  hipExternalMemory_t mem = nullptr;
  HRT_HIP(ctx, hipImportExternalMemory(&mem, &desc));
  hipExternalMemoryBufferDesc bd{};
  bd.offset = offset;
  bd.size = bytes;
  void* ptr = nullptr;
  if (hipError_t e = hipExternalMemoryGetMappedBuffer(&ptr, mem, &bd); e != hipSuccess) {
    (void)hipDestroyExternalMemory(mem);
    return hip_fail(ctx, e, "hipExternalMemoryGetMappedBuffer");
  }
  ctx->imports.push_back({mem, ptr});
  *dev_ptr = ptr;
  return HRT_OK;
}

extern "C" hrt_status hrt_release_external_memory(hrt_context* ctx, void* dev_ptr) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  for (size_t i = 0; i < ctx->imports.size(); ++i) {
    if (ctx->imports[i].ptr == dev_ptr) {
      hrt_status st = hrt_synchronize(ctx);  // no pending write into it
      if (st != HRT_OK) return st;
      HRT_HIP(ctx, hipDestroyExternalMemory(ctx->imports[i].mem));
      ctx->imports.erase(ctx->imports.begin() + (long)i);
      return HRT_OK;
    }
  }
  return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_release_external_memory: not an imported pointer");
}

// Test support: device memory exported as a POSIX fd (HIP virtual memory management), i.e. what the
// presenting API hands to hrt_import_external_memory; *ptr is the exporter's own mapping of it.
extern "C" hrt_status hrt_debug_export_memory(int device, uint64_t bytes, int* fd, void** ptr, uint64_t* size) {
  if (!fd || !ptr || !size || bytes == 0) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "bad arguments");
  hipError_t e = hipSetDevice(device);
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  prop.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
  size_t gran = 0;
  if (e == hipSuccess) e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
  const size_t sz = gran ? (bytes + gran - 1) / gran * gran : bytes;
  hipMemGenericAllocationHandle_t h{};
  if (e == hipSuccess) e = hipMemCreate(&h, sz, &prop, 0);
  if (e == hipSuccess) e = hipMemExportToShareableHandle(fd, h, hipMemHandleTypePosixFileDescriptor, 0);
  void* va = nullptr;
  if (e == hipSuccess) e = hipMemAddressReserve(&va, sz, 0, nullptr, 0);
  if (e == hipSuccess) e = hipMemMap(va, sz, 0, h, 0);
  if (e == hipSuccess) {
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(va, sz, &acc, 1);
  }
  if (e == hipSuccess) e = hipMemRelease(h);  // the mapping keeps the allocation alive
  if (e != hipSuccess) {
    g_create_error = std::string("export: ") + hipGetErrorString(e);
    return HRT_ERR_HIP;
  }
  *ptr = va;
  *size = sz;
  return HRT_OK;
}

extern "C" hrt_status hrt_debug_unmap_memory(void* ptr, uint64_t size) {
  if (hipMemUnmap(ptr, size) != hipSuccess || hipMemAddressFree(ptr, size) != hipSuccess) return HRT_ERR_HIP;
  return HRT_OK;
}

extern "C" hrt_status hrt_read_rays(hrt_context* ctx, hrt_ray* out, uint32_t n) {
  if (!ctx || (!out && n) || (uint64_t)n > ctx->n_rays || !ctx->rays)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_rays: no rays or n too large");
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if (n) HRT_HIP(ctx, hipMemcpy(out, ctx->rays, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost));
  return HRT_OK;
}

extern "C" hrt_status hrt_get_tile_profile(hrt_context* ctx, uint64_t* out, uint32_t count) {
  if (!ctx || !out || count > 4 * ctx->num_tiles() || !ctx->tile_cycles)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_get_tile_profile: needs HRT_OPT_COUNTERS = 2 and a trace");
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  HRT_HIP(ctx, hipMemcpy(out, ctx->tile_cycles, (size_t)count * 8, hipMemcpyDeviceToHost));
  return HRT_OK;
}

extern "C" hrt_status hrt_get_scene_info(hrt_context* ctx, uint32_t* out, uint32_t count) {
  if (!ctx || !out || count > HRT_NUM_SCENE_INFO) return HRT_ERR_INVALID_ARGUMENT;
  for (uint32_t i = 0; i < count; ++i) out[i] = ctx->bvh_info[i];
  return HRT_OK;
}

extern "C" hrt_status hrt_reset_stats(hrt_context* ctx) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if ((st = harvest_events(ctx)) != HRT_OK) return st;
  HRT_HIP(ctx, hipMemsetAsync(ctx->counters, 0, kNumCounters * sizeof(unsigned long long), ctx->stream));
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->traces = ctx->accumulates = 0;
  ctx->last_ms = ctx->total_ms = 0.0f;
  return HRT_OK;
}

extern "C" hrt_status hrt_set_option(hrt_context* ctx, uint32_t key, int64_t value) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  switch (key) {
    case HRT_OPT_KERNEL_VARIANT:
      if (value < HRT_KERNEL_AUTO || value > HRT_KERNEL_BUNDLE_WQ)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "kernel variant must be an hrt_kernel value (0..9)");
      ctx->variant = (int)value;
      return HRT_OK;
    case HRT_OPT_COUNTERS:
      if (value < 0 || value > 2) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "counters option must be 0, 1 or 2");
      ctx->counters_on = value != 0;
      ctx->diag_on = value == 2;
      return HRT_OK;
    case HRT_OPT_SECONDARY_BATCH:
      if (value < 0 || value > 64)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "secondary batch must be 0 (auto) or in [1, 64]");
      ctx->sec_batch = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_SPLIT:
      if (value < 0 || value > 64 || (value & (value - 1)) != 0)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "split must be 0 (auto) or a power of two up to 64");
      ctx->split_k = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_SPLIT_FACTOR:
      if (value < -1 || value > 1000000)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "split factor must be -1 (auto) or 0..1000000");
      ctx->split_factor = (int32_t)value;
      return HRT_OK;
    case HRT_OPT_PRIORITY:
      if (value < 0 || value > 2) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "priority must be 0, 1 or 2");
      ctx->split_prio = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_PROBE:
      if (value != 0 && value != 1) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "probe must be 0 or 1");
      ctx->probe = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_FRAMES_PER_LAUNCH:
      if (value < 1 || value > 1024)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "frames per launch must be in [1, 1024]");
      ctx->frames_per_launch = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_WQ_NODE_CAP:
      if (value != 0 && (value < 128 || value > (1 << 20)))
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "wq node cap must be 0 (auto) or in [128, 2^20]");
      ctx->wq_node_cap = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_COOP:
      if (value != 0 && value != 1) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "coop must be 0 or 1");
      ctx->coop = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_GRID_CUS:
      if (value < 0) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "grid CUs must be >= 0");
      ctx->grid_cus = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_BVH_LEAF_SIZE:
      if (value < 1 || value > hrt::kBvhMaxLeafCount)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "BVH leaf size must be in [1, 16]");
      ctx->bvh_leaf = (uint32_t)value;
      return HRT_OK;
    default:
      return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "unknown option key");
  }
}

extern "C" void* hrt_stream(hrt_context* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

extern "C" const char* hrt_last_error(const hrt_context* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}
