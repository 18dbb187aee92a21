// hrt_api.cpp -- the C ABI of libhip_raytrace.so (include/hip_raytrace.h).
//
// The context (hrt_context.h) owns everything the reference's RayTracePipeline + DiffusePipeline own
// on the Vulkan side (src/raytrace_pipeline.rs:31-46, src/diffuse.rs:22-30).  Memory is allocated by
// hrt_create, hrt_set_scene and hrt_set_option; hrt_trace and hrt_accumulate only enqueue work (no
// allocation) and block only when kMaxPending timed traces are still outstanding.  hrt_compute_n
// allocates its frame images on first use.
//
// Built twice: libhip_raytrace.so (production) and, with -DHRT_DEBUG_OPTIONS, libhip_raytrace_debug.so,
// which also accepts the diagnostics-only options (HRT_OPT_PRIORITY = 2, HRT_OPT_GRID_CUS,
// HRT_DEBUG_OPT_FAIL_ALLOC, HRT_DEBUG_OPT_WQ_TRI_CAP) that leave frames incomplete, inject failures or
// force rare paths.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "hip_raytrace.h"
#include "hrt_bvh.h"
#include "hrt_context.h"
#include "hrt_host.h"
#include "hrt_kernels.h"

// (the record, push-block, hrt_create_info / hrt_layout / hrt_stats sizes and offsets are
// static_asserted by include/hip_raytrace.h itself, for every translation unit that includes it)
static_assert(sizeof(hrt_stats) == 64, "hrt_stats: ABI 4");

namespace {

thread_local std::string g_create_error;
constexpr size_t kMaxPending = 256;              // timed traces held before the oldest is harvested
constexpr size_t kStagingChunk = (size_t)8 << 20;  // pinned upload chunk (two of them)

template <typename T>
void free_dev(hrt_context* ctx, T*& p) {
  hrt::dev_free(ctx, (void*)p);
  p = nullptr;
}

// Folds the oldest timed trace into the stats (blocks until it has finished).
hrt_status harvest_one(hrt_context* ctx) {
  hrt::EventPair ev = ctx->pending.front();
  ctx->pending.erase(ctx->pending.begin());
  ctx->event_pool.push_back(ev);
  HRT_HIP(ctx, hipEventSynchronize(ev.stop));
  float ms = 0.0f;
  HRT_HIP(ctx, hipEventElapsedTime(&ms, ev.start, ev.stop));
  ctx->last_ms = ms / (float)ev.frames;  // per frame
  ctx->total_ms += ms;
  return HRT_OK;
}

hrt_status harvest_events(hrt_context* ctx) {
  while (!ctx->pending.empty()) {
    hrt_status st = harvest_one(ctx);
    if (st != HRT_OK) return st;
  }
  return HRT_OK;
}

// Every stream of the context drained.
hrt_status sync_all(hrt_context* ctx) {
  for (auto& l : ctx->lane)
    if (l.stream) HRT_HIP(ctx, hipStreamSynchronize(l.stream));
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HRT_OK;
}

}  // namespace

namespace hrt {

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

hrt_status bind(hrt_context* ctx) {
  HRT_HIP(ctx, hipSetDevice(ctx->device));
  return HRT_OK;
}

hrt_status wait_lane(hrt_context* ctx, int l) {
  if (ctx->lane[l].done_set) HRT_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->lane[l].done, 0));
  return HRT_OK;
}

hrt_status join_lanes(hrt_context* ctx) {
  for (int l = 0; l < kLanes; ++l) {
    hrt_status st = wait_lane(ctx, l);
    if (st != HRT_OK) return st;
  }
  return HRT_OK;
}

hrt_status release_lane(hrt_context* ctx, int l) {
  HRT_HIP(ctx, hipEventRecord(ctx->lane[l].free, ctx->stream));
  ctx->lane[l].free_set = true;
  return HRT_OK;
}

// Device allocations.  The debug build surrounds every allocation with kGuardBytes of a fixed
// pattern on each side (hrt_debug_check_guards verifies them: a kernel writing past a buffer's end
// or before its start shows up there).
#ifdef HRT_DEBUG_OPTIONS
constexpr size_t kGuardBytes = 4096;
constexpr int kGuardByte = 0xA5;
#endif

hipError_t dev_alloc(hrt_context* ctx, void** p, size_t bytes) {
#ifdef HRT_DEBUG_OPTIONS
  char* base = nullptr;
  hipError_t e = hipMalloc((void**)&base, bytes + 2 * kGuardBytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return e;
  }
  if ((e = hipMemset(base, kGuardByte, kGuardBytes)) != hipSuccess ||
      (e = hipMemset(base + kGuardBytes + bytes, kGuardByte, kGuardBytes)) != hipSuccess) {
    (void)hipFree(base);
    *p = nullptr;
    return e;
  }
  *p = base + kGuardBytes;
  ctx->guards.push_back({*p, bytes});
  return hipSuccess;
#else
  (void)ctx;
  return hipMalloc(p, bytes);
#endif
}

void dev_free(hrt_context* ctx, void* p) {
  if (!p) return;
#ifdef HRT_DEBUG_OPTIONS
  for (size_t i = 0; i < ctx->guards.size(); ++i)
    if (ctx->guards[i].ptr == p) {
      ctx->guards.erase(ctx->guards.begin() + (long)i);
      (void)hipFree(static_cast<char*>(p) - kGuardBytes);
      return;
    }
#else
  (void)ctx;
#endif
  (void)hipFree(p);
}

// The trace image: the most recent trace's ring slot, or its lane's own image.
void* trace_image(hrt_context* ctx) {
  if (ctx->cur_slot >= 0) return static_cast<char*>(ctx->ring) + (size_t)ctx->cur_slot * ctx->npix() * ctx->px_bytes();
  return ctx->lane[ctx->cur_lane].image();
}

const void* local_image(hrt_context* ctx, uint32_t image_id) {
  if (image_id == HRT_IMG_ACCUM) {
    if (flush_combines(ctx) != HRT_OK) return nullptr;
    return ctx->accum8 ? (const void*)ctx->accum8 : (const void*)ctx->accum32;
  }
  if (wait_lane(ctx, ctx->cur_lane) != HRT_OK) return nullptr;
  return trace_image(ctx);
}

hrt_status flush_combines(hrt_context* ctx) {
  if (ctx->pend.empty()) return HRT_OK;
  // the folds read slots that traces on every lane wrote: after each lane's latest trace
  hrt_status st = join_lanes(ctx);
  if (st != HRT_OK) return st;
  const size_t np = ctx->npix(), fb = np * ctx->px_bytes();
  for (size_t i = 0; i < ctx->pend.size();) {
    size_t j = i;  // a run of consecutive slots (no wrap) and frames: one pass over the stack
    while (j + 1 < ctx->pend.size() && ctx->pend[j + 1].slot == ctx->pend[j].slot + 1 &&
           ctx->pend[j + 1].frame == ctx->pend[j].frame + 1)
      ++j;
    char* base = static_cast<char*>(ctx->ring) + (size_t)ctx->pend[i].slot * fb;
    HRT_HIP(ctx, launch_accumulate_frames(ctx->accum8, ctx->accum8 ? reinterpret_cast<const uint32_t*>(base) : nullptr,
                                          ctx->accum32, ctx->accum32 ? reinterpret_cast<const float4*>(base) : nullptr,
                                          np, (uint32_t)(j - i + 1), ctx->pend[i].frame, ctx->stream));
    i = j + 1;
  }
  ctx->pend.clear();
  HRT_HIP(ctx, hipEventRecord(ctx->fold_done, ctx->stream));
  ctx->fold_set = true;
  return HRT_OK;
}

void free_scene(hrt_context* ctx, SceneBufs& s, bool keep_rays) {
  if (!keep_rays) free_dev(ctx, s.rays);
  free_dev(ctx, s.spheres);
  free_dev(ctx, s.tris);
  free_dev(ctx, s.tri_nhat);
  free_dev(ctx, s.meshes);
  free_dev(ctx, s.bvh_nodes);
  free_dev(ctx, s.bvh_wq_nodes);
  free_dev(ctx, s.bvh_prims);
  free_dev(ctx, s.bvh_irregular);
  free_dev(ctx, s.bvh_band_off);
  free_dev(ctx, s.bvh_band);
  free_dev(ctx, s.bvh_band_nhat);
  free_dev(ctx, s.bvh_band_rec);
  free_dev(ctx, s.bvh_entries);
  free_dev(ctx, s.bvh_keybase);
  for (int l = 0; l < kLanes; ++l) {
    free_dev(ctx, s.cam_meta[l]);
    free_dev(ctx, s.cam_tris[l]);
    free_dev(ctx, s.cam_cull[l]);
  }
}

}  // namespace hrt

using hrt::fail;
using hrt::hip_fail;
using hrt::bind;

extern "C" uint32_t hrt_abi_version(void) { return HRT_ABI_VERSION; }

extern "C" hrt_status hrt_debug_check_guards(hrt_context* ctx, uint32_t* buffers, uint32_t* corrupted) {
  if (!ctx || !buffers || !corrupted) return HRT_ERR_INVALID_ARGUMENT;
  *buffers = *corrupted = 0;
#ifdef HRT_DEBUG_OPTIONS
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  std::vector<unsigned char> g(hrt::kGuardBytes);
  for (const auto& r : ctx->guards) {
    bool bad = false;
    for (int side = 0; side < 2 && !bad; ++side) {
      const char* at = side == 0 ? static_cast<const char*>(r.ptr) - hrt::kGuardBytes : static_cast<const char*>(r.ptr) + r.bytes;
      HRT_HIP(ctx, hipMemcpy(g.data(), at, g.size(), hipMemcpyDeviceToHost));
      for (unsigned char b : g) bad |= b != hrt::kGuardByte;
    }
    ++*buffers;
    *corrupted += bad ? 1u : 0u;
  }
  return HRT_OK;
#else
  return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_check_guards: only libhip_raytrace_debug.so guards buffers");
#endif
}

// Tuning support: lane 0's per-tile costs as the last persistent launch on it recorded them (the next
// launch's plan input; shader clocks / 16 per 8x8 tile, summed over the launch's frames).
extern "C" hrt_status hrt_debug_tile_costs(hrt_context* ctx, uint32_t* out, uint32_t count) {
  if (!ctx || !out) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if (!ctx->lane[0].tile_cost) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_tile_costs: no trace yet");
  const uint32_t n = std::min(count, (uint32_t)ctx->num_tiles());
  HRT_HIP(ctx, hipMemcpy(out, ctx->lane[0].tile_cost, (size_t)n * 4, hipMemcpyDeviceToHost));
  return HRT_OK;
}

// Test support: the context's grazing-band structure as the device holds it -- the per-cell records
// (band_records), the offsets and the entry words -- so a test can hold the device-built records to the
// lists they summarise.  info = {cells, entries, wide (32-bit entries), records present}.
extern "C" hrt_status hrt_debug_band_records(hrt_context* ctx, uint32_t* rec, uint64_t rec_words, uint32_t* off,
                                             uint64_t off_words, uint32_t* list_words, uint64_t list_cap,
                                             uint32_t info[4]) {
  if (!ctx || !info) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  const hrt::SceneBufs& s = ctx->scene;
  const uint64_t cells = s.bvh_band_off ? 6ull * s.bvh_dir_res * s.bvh_dir_res : 0ull;
  const uint64_t entries = s.bvh_info[HRT_SCENE_BVH_BAND_ENTRIES];
  const uint64_t words = s.bvh_band_wide ? entries : (entries + 1) / 2;
  info[0] = (uint32_t)cells;
  info[1] = (uint32_t)entries;
  info[2] = s.bvh_band_wide;
  info[3] = s.bvh_band_rec ? 1u : 0u;
  if (rec && s.bvh_band_rec && rec_words >= cells * 8)
    HRT_HIP(ctx, hipMemcpy(rec, s.bvh_band_rec, cells * 32, hipMemcpyDeviceToHost));
  if (off && s.bvh_band_off && off_words >= cells + 1)
    HRT_HIP(ctx, hipMemcpy(off, s.bvh_band_off, (cells + 1) * 4, hipMemcpyDeviceToHost));
  if (list_words && s.bvh_band && list_cap >= words && words)
    HRT_HIP(ctx, hipMemcpy(list_words, s.bvh_band, words * 4, hipMemcpyDeviceToHost));
  return HRT_OK;
}

#ifndef HRT_BUILD_ID
#define HRT_BUILD_ID "unknown"
#endif
extern "C" const char* hrt_build_id(void) { return HRT_BUILD_ID; }

extern "C" uint32_t hrt_debug_build(void) {
#ifdef HRT_DEBUG_OPTIONS
  return 1u;
#else
  return 0u;
#endif
}

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
  if ((e = hrt::ensure_kernel_attributes(ctx->device)) != hipSuccess)
    return bail(hip_fail(ctx, e, "hipFuncSetAttribute(dynamic LDS)"));
  const size_t np = ctx->npix(), tiles = std::max<size_t>(ctx->num_tiles(), 1);
  for (auto& l : ctx->lane) {
    if ((e = hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipStreamCreate(lane)"));
    if ((e = hipEventCreateWithFlags(&l.done, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&l.free, hipEventDisableTiming)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipEventCreate(lane)"));
    if (ctx->mode == HRT_MODE_RGBA8)
      e = hrt::dev_alloc(ctx, (void**)&l.trace8, np * 4);
    else
      e = hrt::dev_alloc(ctx, (void**)&l.trace32, np * 16);
    if (e != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(trace)"));
    if ((e = hrt::dev_alloc(ctx, (void**)&l.sched, hrt::kSchedWords * 4)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(sched)"));
    if ((e = hrt::dev_alloc(ctx, (void**)&l.tile_cost, tiles * 4)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipMalloc(tile costs)"));
    if ((e = hrt::dev_alloc(ctx, (void**)&l.item_buf, tiles * 64 * 4)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipMalloc(items)"));
    if ((e = hrt::dev_alloc(ctx, (void**)&l.tl_cache, tiles * hrt::kTlRecWords * 4)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipMalloc(tile lists)"));
  }
  if (ctx->mode == HRT_MODE_RGBA8)
    e = hrt::dev_alloc(ctx, (void**)&ctx->accum8, np * 4);
  else
    e = hrt::dev_alloc(ctx, (void**)&ctx->accum32, np * 16);
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(accum)"));
  if ((e = hrt::dev_alloc(ctx, (void**)&ctx->scratch, np * 16)) != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(scratch)"));
  if ((e = hipEventCreateWithFlags(&ctx->fold_done, hipEventDisableTiming)) != hipSuccess)
    return bail(hip_fail(ctx, e, "hipEventCreate(fold)"));
  if ((e = hrt::dev_alloc(ctx, (void**)&ctx->counters, hrt::kNumCounters * sizeof(unsigned long long))) != hipSuccess)
    return bail(hip_fail(ctx, e, "hipMalloc(counters)"));
  {
    int cus = 0;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device)) != hipSuccess)
      return bail(hip_fail(ctx, e, "hipDeviceGetAttribute(CUs)"));
    ctx->num_cus = cus > 0 ? (uint32_t)cus : 1u;
  }
  if ((e = hipMemsetAsync(ctx->counters, 0, hrt::kNumCounters * sizeof(unsigned long long), ctx->stream)) != hipSuccess)
    return bail(hip_fail(ctx, e, "hipMemset(counters)"));
  // Fresh images read as the cleared state (0,0,0,1) until the first dispatch writes them.
  for (auto& l : ctx->lane)
    if ((e = hrt::launch_clear(l.trace8, l.trace32, np, ctx->stream)) != hipSuccess) return bail(hip_fail(ctx, e, "clear"));
  if ((e = hrt::launch_clear(ctx->accum8, ctx->accum32, np, ctx->stream)) != hipSuccess)
    return bail(hip_fail(ctx, e, "clear"));
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return bail(hip_fail(ctx, e, "hipStreamSynchronize"));
  *out_ctx = ctx;
  return HRT_OK;
}

extern "C" void hrt_destroy(hrt_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (auto& l : ctx->lane)
    if (l.stream) (void)hipStreamSynchronize(l.stream);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  hrt::comm_release(ctx);
  (void)hipSetDevice(ctx->device);
  hrt::free_scene(ctx, ctx->scene, false);
  for (auto& l : ctx->lane) {
    free_dev(ctx, l.trace8);
    free_dev(ctx, l.trace32);
    free_dev(ctx, l.sched);
    free_dev(ctx, l.tile_cost);
    free_dev(ctx, l.item_buf);
    free_dev(ctx, l.tl_cache);
    if (l.done) (void)hipEventDestroy(l.done);
    if (l.free) (void)hipEventDestroy(l.free);
    if (l.stream) (void)hipStreamDestroy(l.stream);
  }
  free_dev(ctx, ctx->accum8);
  free_dev(ctx, ctx->accum32);
  free_dev(ctx, ctx->scratch);
  free_dev(ctx, ctx->counters);
  free_dev(ctx, ctx->tile_cycles);
  free_dev(ctx, ctx->timeline);
  free_dev(ctx, ctx->timeline_count);
  free_dev(ctx, ctx->frame_stack);
  free_dev(ctx, ctx->ring);
  if (ctx->fold_done) (void)hipEventDestroy(ctx->fold_done);
  for (int i = 0; i < 2; ++i) {
    if (ctx->staging.buf[i]) (void)hipHostFree(ctx->staging.buf[i]);
    if (ctx->staging.ev[i]) (void)hipEventDestroy(ctx->staging.ev[i]);
  }
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

// hrt_set_scene's device allocations (the debug build can fail the n-th one: HRT_DEBUG_OPT_FAIL_ALLOC).
struct SceneAlloc {
  hrt_context* ctx;
  int64_t count = 0;
  hipError_t operator()(void** p, size_t bytes) {
    ++count;
    if (ctx->debug_fail_alloc > 0 && count == ctx->debug_fail_alloc) return hipErrorOutOfMemory;
    return hrt::dev_alloc(ctx, p, bytes ? bytes : 16);
  }
};

// Host -> device copy through the context's pinned staging chunks: the CPU fills one chunk while the
// DMA engine drains the other (the reference's upload points, src/raytrace_pipeline.rs:302,337,349,
// 359,371-372, stage through host-visible buffers the same way).
hrt_status stage_upload(hrt_context* ctx, void* dst, const void* src, size_t bytes) {
  auto& s = ctx->staging;
  if (!s.chunk) {  // both chunks and events into locals; published only when all four exist
    void* buf[2] = {};
    hipEvent_t ev[2] = {};
    hipError_t e = hipSuccess;
    for (int i = 0; i < 2 && e == hipSuccess; ++i)
      if ((e = hipHostMalloc(&buf[i], kStagingChunk, hipHostMallocDefault)) == hipSuccess)
        e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
      for (int i = 0; i < 2; ++i) {
        if (buf[i]) (void)hipHostFree(buf[i]);
        if (ev[i]) (void)hipEventDestroy(ev[i]);
      }
      return hip_fail(ctx, e, "hrt_set_scene: pinned staging");
    }
    for (int i = 0; i < 2; ++i) {
      s.buf[i] = buf[i];
      s.ev[i] = ev[i];
      s.used[i] = false;
    }
    s.chunk = kStagingChunk;
  }
  for (size_t off = 0, k = 0; off < bytes; off += s.chunk, ++k) {
    const int i = (int)(k & 1);
    const size_t n = std::min(s.chunk, bytes - off);
    if (s.used[i]) HRT_HIP(ctx, hipEventSynchronize(s.ev[i]));  // the DMA has left this chunk
    std::memcpy(s.buf[i], static_cast<const char*>(src) + off, n);
    HRT_HIP(ctx, hipMemcpyAsync(static_cast<char*>(dst) + off, s.buf[i], n, hipMemcpyHostToDevice, ctx->stream));
    HRT_HIP(ctx, hipEventRecord(s.ev[i], ctx->stream));
    s.used[i] = true;
  }
  return HRT_OK;
}

// Allocate dst (>= 16 B, so empty lists keep a valid pointer) and upload bytes of src into it.
hrt_status alloc_upload(hrt_context* ctx, SceneAlloc& alloc, void** dst, const void* src, size_t bytes,
                        const char* what) {
  if (hipError_t e = alloc(dst, bytes); e != hipSuccess) {
    *dst = nullptr;
    return hip_fail(ctx, e, (std::string("hrt_set_scene: hipMalloc(") + what + ")").c_str());
  }
  return bytes ? stage_upload(ctx, *dst, src, bytes) : HRT_OK;
}

// The band lists' 16-bit image, padded to whole dwords (hrt_kernels.hip band_entry reads dwords).
std::vector<uint16_t> band16(const std::vector<uint32_t>& list) {
  std::vector<uint16_t> v(list.begin(), list.end());
  v.resize((v.size() + 1) & ~(size_t)1, 0);
  return v;
}

// Fills s with a complete device copy of the scene (everything but the kept rays).
hrt_status build_scene(hrt_context* ctx, hrt::SceneBufs& s, const hrt_ray* rays, uint32_t n_rays, bool keep_rays,
                       const hrt_sphere* spheres, uint32_t n_spheres, const hrt_triangle* tris, uint32_t n_tris,
                       const hrt_mesh* meshes, uint32_t n_meshes) {
  SceneAlloc alloc{ctx};
  hrt_status st;
  if (keep_rays)
    s.rays = ctx->scene.rays;
  else if ((st = alloc_upload(ctx, alloc, (void**)&s.rays, rays, (size_t)n_rays * sizeof(float4), "rays")) != HRT_OK)
    return st;
  if ((st = alloc_upload(ctx, alloc, (void**)&s.spheres, spheres, (size_t)n_spheres * 64, "spheres")) != HRT_OK ||
      (st = alloc_upload(ctx, alloc, (void**)&s.tris, tris, (size_t)n_tris * 64, "triangles")) != HRT_OK ||
      (st = alloc_upload(ctx, alloc, (void**)&s.meshes, meshes, (size_t)n_meshes * 80, "meshes")) != HRT_OK)
    return st;
  {  // the hit normal of each triangle, once (resolve_hit reads it instead of normalizing per hit)
    hipError_t e = alloc((void**)&s.tri_nhat, (size_t)(n_tris ? n_tris : 1) * sizeof(float4));
    if (e == hipSuccess) e = hrt::launch_tri_normals(s.tris, s.tri_nhat, n_tris, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "hrt_set_scene: triangle normals");
  }
  uint64_t cap = 0;
  for (uint32_t m = 0; m < n_meshes; ++m) cap += meshes[m].len;
  if (cap > 0xFFFFFFFFull) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_set_scene: too many mesh triangles");
  // bundle-variant buffers, one set per trace lane: per-frame compacted camera-facing records
  for (int l = 0; l < hrt::kLanes; ++l) {
    hipError_t e;
    if ((e = alloc((void**)&s.cam_meta[l], (size_t)(n_meshes ? 2 * n_meshes : 2) * 4)) != hipSuccess ||
        (e = alloc((void**)&s.cam_tris[l], (size_t)(cap ? cap : 1) * 64)) != hipSuccess ||
        (e = alloc((void**)&s.cam_cull[l], (size_t)(cap ? cap : 1) * 80)) != hipSuccess)
      return hip_fail(ctx, e, "hrt_set_scene: hipMalloc(camera lists)");
  }
  s.cam_capacity = (uint32_t)cap;
  // bounce-segment hierarchy (BUNDLE_BVH / BUNDLE_WQ)
  hrt::BvhHost bvh;
  // auto leaf size: 2, 3, then 4 for scenes BUNDLE_WQ takes -- the smallest whose grouped image leaves
  // the LDS stacks kAutoLeafWqStack entries (island: 2; cave: 3, whose leaves of 2 need 104 KB of
  // nodes); 4 above 8192 entries
  uint32_t leaf = ctx->bvh_leaf ? ctx->bvh_leaf : hrt::auto_leaf_size(cap);
  // (the hierarchy alone while the leaf size is chosen, then the band lists once)
  bool built = hrt::build_bvh(tris, n_tris, meshes, n_meshes, leaf, bvh, ctx->bvh_width, hrt::kBandTau, false);
  while (built && ctx->bvh_leaf == 0 && leaf < 4 &&
         !(bvh.wq_ok && hrt::wq_stack_cap(bvh.wq_n_nodes, bvh.wq_width, leaf) >= hrt::kAutoLeafWqStack)) {
    ++leaf;
    built = hrt::build_bvh(tris, n_tris, meshes, n_meshes, leaf, bvh, ctx->bvh_width, hrt::kBandTau, false);
  }
  if (built) hrt::build_bands(bvh);
  const double margin_frac = bvh.margin_frac;
  if (built) {
    auto up = [&](auto*& dst, const auto& v, const char* what) -> hrt_status {
      return alloc_upload(ctx, alloc, (void**)&dst, v.data(), v.size() * sizeof(v[0]), what);
    };
    if ((st = up(s.bvh_nodes, bvh.nodes, "bvh nodes")) != HRT_OK) return st;
    if (bvh.wq_ok && (st = up(s.bvh_wq_nodes, bvh.wq_nodes, "bvh wq nodes")) != HRT_OK) return st;
    if ((st = up(s.bvh_prims, bvh.prims, "bvh prims")) != HRT_OK ||
        (st = up(s.bvh_irregular, bvh.irregular, "bvh irregular")) != HRT_OK ||
        (st = up(s.bvh_band_off, bvh.band_off, "band offsets")) != HRT_OK ||
        (st = bvh.band_wide() ? up(s.bvh_band, bvh.band_list, "band lists")
                              : up(s.bvh_band, band16(bvh.band_list), "band lists")) != HRT_OK ||
        (st = up(s.bvh_band_nhat, bvh.band_nhat, "band normals")) != HRT_OK ||
        (st = up(s.bvh_entries, bvh.entries, "bvh entries")) != HRT_OK ||
        (st = up(s.bvh_keybase, bvh.key_base, "bvh key bases")) != HRT_OK)
      return st;
    // BUNDLE_WQ's per-cell band records (hrt_kernels.hip band_cell), built on the device from the lists
    // just uploaded: one 32 B record per direction cell (6 x 1,024^2 cells: 201 MB), 16-bit lists only.
    // They only save memory traffic: where they do not fit, the lookups read the offsets and lists (the
    // same bytes, tests/test_gpu_boundary.py::test_failed_set_scene_keeps_the_previous_scene).
    const size_t cells = bvh.band_off.empty() ? 0 : bvh.band_off.size() - 1;
    if (!bvh.band_wide() && cells) {
      hipError_t e = alloc((void**)&s.bvh_band_rec, cells * 32);
      if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();  // (not a sticky error)
        s.bvh_band_rec = nullptr;
      } else if (e == hipSuccess) {
        e = hrt::launch_band_records(s.bvh_band_off, static_cast<const uint32_t*>(s.bvh_band), s.bvh_band_rec,
                                     (uint32_t)cells, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "hrt_set_scene: band records");
      } else {
        return hip_fail(ctx, e, "hrt_set_scene: hipMalloc(band records)");
      }
    }
  }
  s.bvh_info[HRT_SCENE_BVH_NODES] = bvh.n_nodes;
  s.bvh_info[HRT_SCENE_BVH_PRIMS] = bvh.n_prims;
  s.bvh_info[HRT_SCENE_BVH_IRREGULAR] = bvh.n_irregular;
  s.bvh_info[HRT_SCENE_BVH_NEVER] = bvh.n_never;
  s.bvh_info[HRT_SCENE_BVH_BUILT] = built ? 1u : 0u;
  s.bvh_info[HRT_SCENE_BVH_BAND_ENTRIES] = (uint32_t)bvh.band_list.size();
  s.bvh_band_wide = bvh.band_wide() ? 1u : 0u;
  {
    uint32_t longest = 0;
    for (size_t c = 0; c + 1 < bvh.band_off.size(); ++c) longest = std::max(longest, bvh.band_off[c + 1] - bvh.band_off[c]);
    s.bvh_band_bits = 0;
    while (s.bvh_band_bits < 32 && (longest >> s.bvh_band_bits)) ++s.bvh_band_bits;
  }
  s.bvh_info[HRT_SCENE_BVH_SAH_MILLI] = (uint32_t)std::min(1e9, bvh.sah_tri_frac * 1000.0 + 0.5);
  s.bvh_info[HRT_SCENE_BVH_MARGIN_MILLI] = (uint32_t)std::min(1e9, margin_frac * 1000.0 + 0.5);
  s.bvh_abs_coef = bvh.abs_coef;
  s.bvh_band_tau = built ? bvh.band_tau : hrt::kBandTau;
  s.bvh_band_a1 = built ? bvh.band_a1 : 0.0f;
  s.bvh_rel_t = bvh.rel_t;
  s.bvh_dir_res = bvh.dir_res;
  s.bvh_built_leaf = std::max(1u, std::min(leaf, hrt::kBvhMaxLeafCount));  // leaves hold at most this
  s.bvh_wq_n = bvh.wq_ok ? bvh.wq_n_nodes : 0u;
  s.bvh_wq_width = bvh.wq_width;
  s.n_spheres = n_spheres;
  s.n_tris = n_tris;
  s.n_meshes = n_meshes;
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));  // host arrays are only borrowed
  return HRT_OK;
}

}  // namespace

extern "C" hrt_status hrt_set_scene(hrt_context* ctx, const hrt_ray* rays, uint32_t n_rays, const hrt_sphere* spheres,
                                    uint32_t n_spheres, const hrt_triangle* tris, uint32_t n_tris,
                                    const hrt_mesh* meshes, uint32_t n_meshes) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  const bool keep_rays =
      !rays && n_rays == 0 && ctx->scene.rays && ctx->n_rays == (uint64_t)ctx->width * ctx->height;
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
  if ((st = sync_all(ctx)) != HRT_OK) return st;  // no trace in flight reads the buffers replaced below
  // The new scene is built completely beside the old one and swapped in only on success, so a failed
  // call (allocation, upload) leaves the previous scene -- buffers and counts -- intact.
  hrt::SceneBufs s;
  st = build_scene(ctx, s, rays, n_rays, keep_rays, spheres, n_spheres, tris, n_tris, meshes, n_meshes);
  if (st != HRT_OK) {
    (void)hipStreamSynchronize(ctx->stream);
    hrt::free_scene(ctx, s, keep_rays);
    ctx->debug_fail_alloc = 0;
    return st;
  }
  hrt::free_scene(ctx, ctx->scene, keep_rays);
  ctx->scene = s;
  ctx->debug_fail_alloc = 0;
  if (!keep_rays) ctx->n_rays = n_rays;
  for (auto& l : ctx->lane) l.plan_valid = l.cam_ready = l.tl_ready = false;  // costs, camera and tile lists of the old scene
  ctx->scene_set = true;
  return HRT_OK;
}

namespace {

// Validates a dispatch's push block against the context (hrt_trace / hrt_compute_n).
hrt_status check_dispatch(hrt_context* ctx, const hrt_push_constants* pc, const char* who) {
  if (!ctx->scene_set) return fail(ctx, HRT_ERR_NO_SCENE, std::string(who) + ": hrt_set_scene has not been called");
  if (pc->width != ctx->width || pc->height != ctx->height)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, std::string(who) + ": push constant width/height differ from the context");
  if (pc->num_spheres < 0 || (uint32_t)pc->num_spheres > ctx->scene.n_spheres || pc->num_meshes < 0 ||
      (uint32_t)pc->num_meshes > ctx->scene.n_meshes)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, std::string(who) + ": num_spheres/num_meshes exceed the uploaded scene");
  return HRT_OK;
}

// The kernel argument block of a dispatch of pc into trace lane l's image.
hrt::TraceParams make_params(hrt_context* ctx, const hrt_push_constants* pc, int l) {
  const hrt::SceneBufs& s = ctx->scene;
  const hrt::Lane& lane = ctx->lane[l];
  hrt::TraceParams p{};
  p.rays = s.rays;
  p.spheres = s.spheres;
  p.tris = s.tris;
  p.tri_nhat = s.tri_nhat;
  p.meshes = s.meshes;
  p.img8 = lane.trace8;
  p.img32 = lane.trace32;
  p.counters = ctx->counters_on ? ctx->counters : nullptr;
  p.diag = ctx->diag_on ? ctx->counters + 3 : nullptr;
  p.tile_cycles = ctx->diag_on ? ctx->tile_cycles : nullptr;
  p.pc = *pc;
  p.local_rows = ctx->local_rows;
  p.row_tile = ctx->row_tile;
  p.part_index = ctx->part_index;
  p.part_count = ctx->part_count;
  p.n_tris = s.n_tris;
  p.cam_start = s.cam_meta[l];
  p.cam_count = s.cam_meta[l] + s.n_meshes;
  p.cam_list_capacity = s.cam_capacity;
  p.cam_tris = s.cam_tris[l];
  p.cam_cull = s.cam_cull[l];
  p.sec_batch = ctx->sec_batch;
  p.sched = lane.sched;
  p.tile_cost = lane.tile_cost;
  p.item_buf = lane.item_buf;
  p.tl_cache = lane.tl_cache;
  p.split_k = ctx->split_k;
  p.split_factor = ctx->split_factor;
  p.split_prio = ctx->split_prio;
  p.coop = ctx->coop;
  p.wq_ncap = ctx->wq_node_cap;  // request; launch_trace sizes the stacks
  p.wq_tcap = ctx->debug_wq_tri_cap;  // (debug) request
  p.grab_always = ctx->debug_grab_runs;  // (debug) frame runs at any size
  p.timeline = ctx->timeline;
  p.timeline_count = ctx->timeline_count;
  p.timeline_cap = ctx->timeline_cap;
  p.plan_valid = lane.plan_valid ? 1u : 0u;
  p.num_cus = ctx->grid_cus ? std::min(ctx->grid_cus, ctx->num_cus) : ctx->num_cus;
  const bool built = s.bvh_info[HRT_SCENE_BVH_BUILT] != 0;
  p.bvh_nodes = built ? s.bvh_nodes : nullptr;
  p.bvh_wq_nodes = built ? s.bvh_wq_nodes : nullptr;
  p.bvh_wq_n_nodes = s.bvh_wq_n;
  p.bvh_wq_width = s.bvh_wq_width;
  p.bvh_prims = s.bvh_prims;
  p.bvh_irregular = s.bvh_irregular;
  p.bvh_band_off = s.bvh_band_off;
  p.bvh_dir_res = s.bvh_dir_res;
  p.bvh_sah_milli = s.bvh_info[HRT_SCENE_BVH_SAH_MILLI];
  p.bvh_band = s.bvh_band;
  p.bvh_band_nhat = s.bvh_band_nhat;
  p.bvh_band_rec = s.bvh_band_rec;
  p.bvh_band_wide = s.bvh_band_wide;
  p.bvh_band_bits = s.bvh_band_bits;
  p.bvh_entries = s.bvh_entries;
  p.bvh_keybase = s.bvh_keybase;
  p.bvh_n_prims = s.bvh_info[HRT_SCENE_BVH_PRIMS];
  p.bvh_n_meshes = s.n_meshes;
  p.bvh_n_nodes = s.bvh_info[HRT_SCENE_BVH_NODES];
  p.bvh_abs_coef = s.bvh_abs_coef;
  p.bvh_rel_t = s.bvh_rel_t;
  p.bvh_band_tau = s.bvh_band_tau;
  p.bvh_band_a1 = s.bvh_band_a1;
  p.bvh_node_r = ctx->wq_node_radius == 2 ||
                 (ctx->wq_node_radius == 0 && s.bvh_info[HRT_SCENE_BVH_MARGIN_MILLI] > hrt::kNodeRadiusMarginMilli);
  p.bvh_n_irregular = s.bvh_info[HRT_SCENE_BVH_IRREGULAR];
  p.bvh_max_leaf = s.bvh_built_leaf;
  p.n_frames = 1;
  p.frame_stride = ctx->npix();
  return p;
}

bool persistent_kernel(int k) {
  return k == HRT_KERNEL_BUNDLE_WQ || k == HRT_KERNEL_BUNDLE_CULL_LDS || k == HRT_KERNEL_BUNDLE_BVH_LDS;
}
// The kernels whose launch (re)builds the lane's camera lists (launch_trace runs camera_lists before
// them); LITERAL, BRUTE and BRUTE_LDS neither build nor read the lists.
bool builds_camera_lists(int k) {
  return persistent_kernel(k) || k == HRT_KERNEL_BUNDLE || k == HRT_KERNEL_BUNDLE_CULL || k == HRT_KERNEL_BUNDLE_BVH;
}

// One trace launch of p.n_frames frames on `stream` with lane l's planner buffers (timed by a HIP
// event pair counted as that many traces).
hrt_status launch_frames(hrt_context* ctx, hrt::TraceParams& p, hipStream_t stream, int l) {
  if (ctx->diag_on)
    HRT_HIP(ctx, hipMemsetAsync(ctx->tile_cycles, 0, ctx->num_tiles() * 4 * sizeof(unsigned long long), stream));
  if (ctx->timeline) HRT_HIP(ctx, hipMemsetAsync(ctx->timeline_count, 0, sizeof(uint32_t), stream));  // this launch's
  const int variant = ctx->variant;
  if (ctx->pending.size() >= kMaxPending) {
    hrt_status st = harvest_one(ctx);
    if (st != HRT_OK) return st;
  }
  hrt::EventPair ev;
  if (!ctx->event_pool.empty()) {
    ev = ctx->event_pool.back();
    ctx->event_pool.pop_back();
  } else {
    HRT_HIP(ctx, hipEventCreate(&ev.start));
    HRT_HIP(ctx, hipEventCreate(&ev.stop));
  }
  ev.frames = p.n_frames > 1 ? p.n_frames : 1u;
  hrt::Lane& lane = ctx->lane[l];
  // First trace of a persistent kernel on this lane (no tile costs yet): a 1-sample probe trace into the
  // lane's own image (fully overwritten by the trace that follows on the same stream) measures the
  // tiles' relative costs so that this trace already follows a plan (HRT_OPT_PROBE).
  const int resolved = hrt::resolve_variant(p, variant);
  // camera lists: rebuilt only when the lane's were built for another position (or scene)
  uint32_t key[4];
  std::memcpy(key, p.pc.cam_pos, 12);
  key[3] = p.pc.num_meshes;
  p.cam_lists_ready = lane.cam_ready && std::memcmp(key, lane.cam_key, sizeof key) == 0 ? 1u : 0u;
  lane.cam_ready = false;  // until a launch has rebuilt them
  // the persistent kernels' tile lists (tile_lists): a function of the camera (position, the mat3 the
  // kernels read, jitter), the meshes and the ray centres -- rebuilt when the camera differs from the one
  // they were built for, after hrt_set_scene or hrt_generate_rays, and after a launch of another kernel
  uint32_t tkey[14];
  std::memcpy(tkey, p.pc.cam_pos, 12);
  for (int i = 0, j = 0; i < 11; ++i)
    if (i % 4 != 3) std::memcpy(&tkey[3 + j++], &p.pc.cam_alignment_mat[i], 4);
  std::memcpy(&tkey[12], &p.pc.jitter_size, 4);
  tkey[13] = p.pc.num_meshes;
  p.tl_lists_ready = lane.tl_ready && std::memcmp(tkey, lane.tl_key, sizeof tkey) == 0 ? 1u : 0u;
  lane.tl_ready = false;
  if (ctx->probe && !lane.plan_valid && ctx->num_tiles() >= 1024 && persistent_kernel(resolved)) {
    hrt::TraceParams q = p;
    q.pc.num_samples = 1;
    q.n_frames = 1;
    q.img8 = lane.trace8;
    q.img32 = lane.trace32;
    q.counters = nullptr;
    q.diag = nullptr;
    q.tile_cycles = nullptr;
    q.probe = 1u;
    int ran = 0, blk = 0;
    if (hipError_t pe = hrt::launch_trace(q, variant, stream, &ran, &blk); pe != hipSuccess) {
      ctx->event_pool.push_back(ev);
      return hip_fail(ctx, pe, "probe trace launch");
    }
    p.plan_valid = 1u;
    if (builds_camera_lists(ran)) p.cam_lists_ready = 1u;  // the probe built them
    if (persistent_kernel(ran)) p.tl_lists_ready = 1u;     // (and the tile lists)
  }
  HRT_HIP(ctx, hipEventRecord(ev.start, stream));
  hipError_t e = hrt::launch_trace(p, variant, stream, &ctx->last_kernel, &ctx->last_block);
  if (e == hipSuccess) ctx->last_frames = ev.frames;
  // the persistent kernels recorded this trace's tile costs: the lane's next trace can follow a plan
  lane.plan_valid = e == hipSuccess && persistent_kernel(ctx->last_kernel);
  // (only a kernel that built the lists leaves them valid: a LITERAL / BRUTE trace from this position
  // followed by a bundle kernel must rebuild them)
  if (e == hipSuccess && builds_camera_lists(ctx->last_kernel)) {
    lane.cam_ready = true;
    std::memcpy(lane.cam_key, key, sizeof key);
  }
  if (e == hipSuccess && persistent_kernel(ctx->last_kernel)) {
    lane.tl_ready = true;
    std::memcpy(lane.tl_key, tkey, sizeof tkey);
  }
  if (e != hipSuccess) {
    ctx->event_pool.push_back(ev);
    return hip_fail(ctx, e, "trace kernel launch");
  }
  HRT_HIP(ctx, hipEventRecord(ev.stop, stream));
  ctx->pending.push_back(ev);
  ctx->traces += ev.frames;
  return HRT_OK;
}

// The deferred combiner's ring of frame images: up to 16 frames within 512 MiB; none (immediate
// combines) when fewer than 4 frames fit.  Allocated once, by the first trace that needs it.
constexpr size_t kRingBytes = (size_t)512 << 20;
hrt_status ensure_ring(hrt_context* ctx) {
  if (ctx->ring || ctx->ring_n == 0xFFFFFFFFu) return HRT_OK;
  const size_t fb = ctx->npix() * ctx->px_bytes();
  const size_t n = std::min<size_t>(16, kRingBytes / std::max<size_t>(fb, 1));
  if (n < 4) {
    ctx->ring_n = 0xFFFFFFFFu;  // (never: frames this large combine immediately)
    return HRT_OK;
  }
  HRT_HIP(ctx, hrt::dev_alloc(ctx, &ctx->ring, n * fb));
  ctx->ring_n = (uint32_t)n;
  ctx->ring_next = 0;
  return HRT_OK;
}

// The lane the next trace runs on (rotating over HRT_OPT_OVERLAP lanes, after the lane's last reader).
hrt_status begin_lane(hrt_context* ctx, int* out) {
  // (diagnostics and the timeline record into one buffer per context: one lane, so no two launches
  // interleave their records or reset each other's count -- ADVICE r05)
  const int n = ctx->diag_on || ctx->timeline ? 1 : (int)std::max(1u, ctx->overlap);
  const int l = ctx->lane_used ? (ctx->cur_lane + 1) % n : 0;
  hrt::Lane& lane = ctx->lane[l];
  if (lane.free_set) HRT_HIP(ctx, hipStreamWaitEvent(lane.stream, lane.free, 0));
  *out = l;
  return HRT_OK;
}

hrt_status end_lane(hrt_context* ctx, int l) {
  HRT_HIP(ctx, hipEventRecord(ctx->lane[l].done, ctx->lane[l].stream));
  ctx->lane[l].done_set = true;
  ctx->cur_lane = l;
  ctx->lane_used = true;
  return HRT_OK;
}

}  // namespace

extern "C" hrt_status hrt_trace(hrt_context* ctx, const hrt_push_constants* pc) {
  if (!ctx || !pc) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  if (!pc->init && (st = check_dispatch(ctx, pc, "hrt_trace")) != HRT_OK) return st;
  // The frame's image: the next ring slot when combines are deferred (the ring is allocated by the
  // first such trace; a slot still waiting for its fold forces the fold first), else the lane's own.
  int slot = -1;
  if (!pc->init && ctx->defer) {
    if ((st = ensure_ring(ctx)) != HRT_OK) return st;
    if (ctx->ring) {
      slot = (int)ctx->ring_next;
      // (the flush clears ctx->pend: decide first, flush outside the loop)
      const bool busy = std::any_of(ctx->pend.begin(), ctx->pend.end(),
                                    [&](const auto& pd) { return pd.slot == (uint32_t)slot; });
      if (busy && (st = hrt::flush_combines(ctx)) != HRT_OK) return st;
    }
  }
  int l = 0;
  if ((st = begin_lane(ctx, &l)) != HRT_OK) return st;
  hrt::Lane& lane = ctx->lane[l];
  if (pc->init) {  // RayTracePipeline::init, src/raytrace_pipeline.rs:190-213
    HRT_HIP(ctx, hrt::launch_clear(lane.trace8, lane.trace32, ctx->npix(), lane.stream));
  } else {
    hrt::TraceParams p = make_params(ctx, pc, l);
    if (slot >= 0) {  // after the fold that last read the slot
      if (ctx->fold_set) HRT_HIP(ctx, hipStreamWaitEvent(lane.stream, ctx->fold_done, 0));
      char* img = static_cast<char*>(ctx->ring) + (size_t)slot * ctx->npix() * ctx->px_bytes();
      p.img8 = lane.trace8 ? reinterpret_cast<uint32_t*>(img) : nullptr;
      p.img32 = lane.trace32 ? reinterpret_cast<float4*>(img) : nullptr;
    }
    // Throughput mode: when another lane's trace is still running, this one shares the chip with it
    // (a persistent grid over 1 / HRT_OPT_BUSY_SPLIT of the CUs), so two frames' long sample chains run
    // side by side instead of the next frame waiting for every CU; an idle GPU gets the whole grid.
    if (ctx->busy_split > 1) {
      bool busy = false;
      for (int o = 0; o < hrt::kLanes; ++o)
        if (o != l && ctx->lane[o].done_set && hipEventQuery(ctx->lane[o].done) == hipErrorNotReady) busy = true;
      if (busy) p.num_cus = std::max(1u, p.num_cus / ctx->busy_split);
    }
    if ((st = launch_frames(ctx, p, lane.stream, l)) != HRT_OK) return st;
  }
  ctx->cur_slot = slot;
  if (slot >= 0) ctx->ring_next = (uint32_t)(slot + 1) % ctx->ring_n;
  return end_lane(ctx, l);
}

// The frame stack's allocation (the debug build can make it fail above HRT_DEBUG_OPT_STACK_LIMIT bytes).
static hipError_t stack_alloc(hrt_context* ctx, void** p, size_t bytes) {
#ifdef HRT_DEBUG_OPTIONS
  if (ctx->debug_stack_limit > 0 && bytes > (size_t)ctx->debug_stack_limit) return hipErrorOutOfMemory;
#endif
  return hrt::dev_alloc(ctx, p, bytes);
}

extern "C" hrt_status hrt_compute_n(hrt_context* ctx, const hrt_push_constants* pc, uint32_t n) {
  if (!ctx || !pc) return HRT_ERR_INVALID_ARGUMENT;
  if (pc->init) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_compute_n: init dispatches go through hrt_trace");
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  if ((st = check_dispatch(ctx, pc, "hrt_compute_n")) != HRT_OK) return st;
  if (n == 0) return HRT_OK;
  // The whole loop runs on the context stream with lane 0's buffers, after every lane's last trace
  // and every deferred combine (frames fold in call order).
  if ((st = hrt::flush_combines(ctx)) != HRT_OK) return st;
  if ((st = hrt::join_lanes(ctx)) != HRT_OK) return st;
  hrt::TraceParams p = make_params(ctx, pc, 0);
  hrt::Lane& lane = ctx->lane[0];
  const size_t np = ctx->npix(), px_bytes = ctx->px_bytes();
  // Frames per launch: up to HRT_OPT_FRAMES_PER_LAUNCH, and at most 1 GiB of frame images.
  const uint32_t cap = (uint32_t)std::max<size_t>(
      1, std::min<size_t>(ctx->frames_per_launch, ((size_t)1 << 30) / std::max<size_t>(np * px_bytes, 1)));
  bool batch = persistent_kernel(hrt::resolve_variant(p, ctx->variant)) && cap > 1 && n > 1;
  // The stack is sized for a whole launch of cap frames at once (a stack grown from a short first call --
  // bench.py's 5 warm-up frames -- was re-allocated by the next longer call, a device synchronisation and
  // ~0.3 ms of hipFree / hipMalloc inside that call).  Where that does not fit (several contexts on one
  // device, little free memory) the call's own min(cap, n) frames are allocated instead; where even those
  // do not fit, the call runs with the stack it has (more, shorter launches) or one launch per frame.
  // Never an error: the frames are the same bytes whatever the launches hold.
  if (batch && ctx->frame_stack_frames < cap) {
    const uint32_t need = std::min(cap, n);
    void* fresh = nullptr;
    uint32_t fresh_frames = 0;
    auto try_alloc = [&](uint32_t frames) {
      if (stack_alloc(ctx, &fresh, (size_t)frames * np * px_bytes) == hipSuccess) {
        fresh_frames = frames;
        return true;
      }
      (void)hipGetLastError();  // (a failed allocation is not a sticky error)
      fresh = nullptr;
      return false;
    };
    if (ctx->frame_stack_failed != cap && !try_alloc(cap)) ctx->frame_stack_failed = cap;
    if (!fresh && ctx->frame_stack_frames < need) (void)try_alloc(need);
    if (fresh) {
      HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
      free_dev(ctx, ctx->frame_stack);
      ctx->frame_stack = fresh;
      ctx->frame_stack_frames = fresh_frames;
    }
  }
  const uint32_t lcap = batch ? std::min(cap, ctx->frame_stack_frames) : 1;  // frames per launch this call
  batch = batch && lcap > 1;
  for (uint32_t done = 0; done < n;) {
    // near-equal launches: ceil(remaining / lcap) of them
    const uint32_t left = n - done, launches = batch ? (left + lcap - 1) / lcap : left;
    const uint32_t nf = (left + launches - 1) / launches;
    hrt::TraceParams q = p;
    q.pc.rng_offset = pc->rng_offset + done;  // u32, wrapping like the per-frame loop's pushes
    q.n_frames = nf;
    q.plan_valid = lane.plan_valid ? 1u : 0u;
    if (nf > 1) {
      q.img8 = lane.trace8 ? reinterpret_cast<uint32_t*>(ctx->frame_stack) : nullptr;
      q.img32 = lane.trace32 ? reinterpret_cast<float4*>(ctx->frame_stack) : nullptr;
    }
    if ((st = launch_frames(ctx, q, ctx->stream, 0)) != HRT_OK) return st;
    // DiffusePipeline::next_frame(frame) for each frame, in frame order: one pass over the stack
    if (nf > 1)
      HRT_HIP(ctx, hrt::launch_accumulate_frames(ctx->accum8, q.img8, ctx->accum32, q.img32, np, nf, q.pc.rng_offset,
                                                 ctx->stream));
    else
      HRT_HIP(ctx, hrt::launch_accumulate(ctx->accum8, lane.trace8, ctx->accum32, lane.trace32, np, q.pc.rng_offset,
                                          ctx->stream));
    ctx->accumulates += nf;
    if (nf > 1)  // the trace image holds the last frame, as after the per-frame loop
      HRT_HIP(ctx, hipMemcpyAsync(lane.image(), static_cast<const char*>(ctx->frame_stack) + (size_t)(nf - 1) * np * px_bytes,
                                  np * px_bytes, hipMemcpyDeviceToDevice, ctx->stream));
    done += nf;
  }
  ctx->cur_lane = 0;
  ctx->cur_slot = -1;  // the trace image is lane 0's
  ctx->lane_used = true;
  return hrt::release_lane(ctx, 0);  // lane 0's next trace follows this loop
}

extern "C" hrt_status hrt_accumulate(hrt_context* ctx, uint32_t frame) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  const int l = ctx->cur_lane;  // next_image = the most recent trace
  if (ctx->cur_slot >= 0 && ctx->defer) {
    // deferred: the next frame of a run of consecutive slots and frames, else the run is folded first
    const uint32_t s = (uint32_t)ctx->cur_slot;
    if (!ctx->pend.empty()) {
      const hrt_context::Pend& b = ctx->pend.back();
      if (!(s == b.slot + 1 && frame == b.frame + 1) && (st = hrt::flush_combines(ctx)) != HRT_OK) return st;
    }
    ctx->pend.push_back({s, frame});
    ctx->accumulates++;
    return HRT_OK;
  }
  if ((st = hrt::flush_combines(ctx)) != HRT_OK) return st;  // frames fold in call order
  if ((st = hrt::wait_lane(ctx, l)) != HRT_OK) return st;
  void* img = hrt::trace_image(ctx);
  HRT_HIP(ctx, hrt::launch_accumulate(ctx->accum8, ctx->accum8 ? static_cast<uint32_t*>(img) : nullptr, ctx->accum32,
                                      ctx->accum32 ? static_cast<float4*>(img) : nullptr, ctx->npix(), frame,
                                      ctx->stream));
  ctx->accumulates++;
  return hrt::release_lane(ctx, l);
}

namespace {

// dst <- src (npix pixels of the context's format) in format fmt, ordered on ctx->stream; blocking.
hrt_status copy_out(hrt_context* ctx, const void* src, size_t npix, uint32_t fmt, void* dst, void* scratch) {
  const size_t need = npix * (fmt == HRT_FMT_RGBA8 ? 4 : 16);
  const bool native = (ctx->mode == HRT_MODE_RGBA8) == (fmt == HRT_FMT_RGBA8);
  if (!native) {
    if (ctx->mode == HRT_MODE_RGBA8)
      HRT_HIP(ctx, hrt::launch_convert((const uint32_t*)src, (float4*)scratch, nullptr, nullptr, npix, ctx->stream));
    else
      HRT_HIP(ctx, hrt::launch_convert(nullptr, nullptr, (const float4*)src, (uint32_t*)scratch, npix, ctx->stream));
    src = scratch;
  }
  HRT_HIP(ctx, hipMemcpyAsync(dst, src, need, hipMemcpyDefault, ctx->stream));
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HRT_OK;
}

}  // namespace

extern "C" hrt_status hrt_read_image(hrt_context* ctx, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  const bool local = (image_id & HRT_IMG_LOCAL) != 0;
  image_id &= ~(uint32_t)HRT_IMG_LOCAL;
  hrt_status arg = HRT_OK;
  if (image_id != HRT_IMG_TRACE && image_id != HRT_IMG_ACCUM)
    arg = fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: unknown image id");
  else if (fmt != HRT_FMT_RGBA8 && fmt != HRT_FMT_RGBA32F)
    arg = fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: unknown format");
  // the framebuffer gather: a collective, so a bad argument is agreed on by every rank, not returned here
  if (ctx->comm && !local) return hrt::comm_read_image(ctx, image_id, fmt, dst, bytes, arg);
  if (arg != HRT_OK) return arg;
  if (!dst) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: null destination");
  const size_t np = ctx->npix();
  if (bytes < np * (fmt == HRT_FMT_RGBA8 ? 4 : 16))
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: destination too small");
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  const void* src = hrt::local_image(ctx, image_id);
  if (!src) return fail(ctx, HRT_ERR_HIP, "hrt_read_image: lane wait failed");
  if ((st = copy_out(ctx, src, np, fmt, dst, ctx->scratch)) != HRT_OK) return st;
  return image_id == HRT_IMG_TRACE ? hrt::release_lane(ctx, ctx->cur_lane) : HRT_OK;
}

// Checkpoint / resume: the accumulator is the whole state of a progressive render
// besides the frame counter (frame k traces with rng_offset = k), so restoring the bytes
// hrt_read_image(HRT_IMG_ACCUM) returned -- in the context's own format, no conversion -- and
// continuing with the saved frame number renders exactly what an uninterrupted run would.
extern "C" hrt_status hrt_load_accumulator(hrt_context* ctx, uint32_t fmt, const void* src, size_t bytes) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  const uint32_t native = ctx->accum8 ? HRT_FMT_RGBA8 : HRT_FMT_RGBA32F;
  if (fmt != native)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_load_accumulator: format must be the context's own (no conversion)");
  if (!src) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_load_accumulator: null source");
  const size_t need = ctx->npix() * (fmt == HRT_FMT_RGBA8 ? 4 : 16);
  if (bytes != need) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_load_accumulator: size differs from the local image");
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  if ((st = hrt::flush_combines(ctx)) != HRT_OK) return st;  // (overwritten below, but in call order)
  if ((st = sync_all(ctx)) != HRT_OK) return st;  // no accumulate in flight
  void* dst = ctx->accum8 ? (void*)ctx->accum8 : (void*)ctx->accum32;
  // on the context stream (non-blocking w.r.t. the null stream): the next hrt_accumulate follows it
  HRT_HIP(ctx, hipMemcpyAsync(dst, src, need, hipMemcpyDefault, ctx->stream));  // host or device source
  HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HRT_OK;
}

namespace hrt {
hrt_status copy_frame_out(hrt_context* ctx, const void* src, size_t npix, uint32_t fmt, void* dst, void* scratch) {
  return copy_out(ctx, src, npix, fmt, dst, scratch);
}
}  // namespace hrt

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
  if ((st = hrt::flush_combines(ctx)) != HRT_OK) return st;  // every accumulate has run after a sync
  return sync_all(ctx);
}

extern "C" hrt_status hrt_get_stats(hrt_context* ctx, hrt_stats* out) {
  if (!ctx || !out) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if ((st = harvest_events(ctx)) != HRT_OK) return st;
  unsigned long long c[hrt::kNumCounters] = {};
  HRT_HIP(ctx, hipMemcpy(c, ctx->counters, sizeof c, hipMemcpyDeviceToHost));
  out->segments = c[0];
  out->tri_tests = c[1];
  out->traces = ctx->traces;
  out->accumulates = ctx->accumulates;
  out->wave_steps = c[2];
  out->last_kernel = (uint32_t)ctx->last_kernel;
  out->last_block = (uint32_t)ctx->last_block;
  out->last_frames = ctx->last_frames;
  out->reserved = 0;
  out->last_trace_ms = ctx->last_ms;
  out->total_trace_ms = ctx->total_ms;
  return HRT_OK;
}

extern "C" hrt_status hrt_get_diagnostics(hrt_context* ctx, uint64_t* out, uint32_t count) {
  if (!ctx || !out || count > HRT_NUM_DIAG) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  unsigned long long c[hrt::kNumCounters] = {};
  HRT_HIP(ctx, hipMemcpy(c, ctx->counters, sizeof c, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < count; ++i) out[i] = c[3 + i];
  return HRT_OK;
}

extern "C" hrt_status hrt_generate_rays(hrt_context* ctx, float camera_focal_length, float viewport_height,
                                        const float up[3], float* default_jitter) {
  if (!ctx || !up) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = bind(ctx);
  if (st != HRT_OK) return st;
  if ((st = sync_all(ctx)) != HRT_OK) return st;  // no trace in flight reads the rays
  float first[3], px[3], py[3];
  const uint32_t n = hrt_host_ray_grid(ctx->width, ctx->height, camera_focal_length, viewport_height, up, first, px,
                                       py, default_jitter);
  const size_t want = (size_t)ctx->width * ctx->height;
  if (!ctx->scene.rays || ctx->n_rays != want) {
    free_dev(ctx, ctx->scene.rays);
    ctx->n_rays = 0;
    HRT_HIP(ctx, hrt::dev_alloc(ctx, (void**)&ctx->scene.rays, (want ? want : 1) * sizeof(float4)));
  }
  for (auto& l : ctx->lane) l.tl_ready = false;  // the tile lists were built from the old ray centres
  if (n) HRT_HIP(ctx, hrt::launch_make_rays(ctx->scene.rays, ctx->width, ctx->height, first, px, py, ctx->stream));
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

// Test support: hrt_math.h's shared-reciprocal normalize / division and sqrt paths against the
// compiler's IEEE sequences on n hashed inputs; out = {normalize, div3, sqrt mismatches, fast cases}.
extern "C" hrt_status hrt_debug_math_check(int device, uint32_t n, uint32_t seed, uint64_t out[4]) {
  if (!out) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_math_check: null out");
  unsigned long long* d = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc((void**)&d, 4 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(d, 0, 4 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hrt::launch_math_check(n, seed, d, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, d, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hrt_debug_math_check");
  return HRT_OK;
}

// Test support: the RNG-domain shortcuts (sqrt_rng, spec_sincos_angle) against the general routines
// over all 2^32 u01 states; out = {sqrt mismatches, sincos mismatches}.
extern "C" hrt_status hrt_debug_math_check_rng(int device, uint64_t out[5]) {
  if (!out) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_math_check_rng: null out");
  unsigned long long* d = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc((void**)&d, 5 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(d, 0, 5 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hrt::launch_math_check_rng(d, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, d, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hrt_debug_math_check_rng");
  return HRT_OK;
}

// Test support: the pair traversal's cross-lane LDS handoffs (hrt_kernels.hip lds_put / lds_get /
// wq_slot_*, wave_handoff) on a scripted run of one wave; the host model is tests/test_gpu_boundary.py's.
extern "C" hrt_status hrt_debug_wq_protocol(int device, uint32_t rounds, const uint32_t* cnt, const uint32_t* take,
                                            const uint32_t* tgt, const uint64_t* val, const uint64_t seed[64],
                                            uint32_t* popped, uint64_t* seen, uint64_t slots[64], uint32_t* depth) {
  if (!cnt || !take || !tgt || !val || !seed || !popped || !seen || !slots || !depth || rounds == 0 || rounds > 1024)
    return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_wq_protocol: bad arguments");
  for (uint32_t i = 0; i < rounds * 64u; ++i)
    if (cnt[i] > 4u) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_wq_protocol: cnt > 4");
  const size_t nr = (size_t)rounds * 64;
  // device layout: u64 [val nr][seed 64][seen nr][slots 64], then u32 [cnt nr][take rounds][tgt nr][popped nr][depth]
  const size_t b64 = (2 * nr + 128) * 8, b32 = (3 * nr + rounds + 1) * 4;
  char* d = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc((void**)&d, b64 + b32);
  unsigned long long* dval = reinterpret_cast<unsigned long long*>(d);
  unsigned long long* dseed = dval + nr;
  unsigned long long* dseen = dseed + 64;
  unsigned long long* dslots = dseen + nr;
  uint32_t* dcnt = reinterpret_cast<uint32_t*>(d + b64);
  uint32_t* dtake = dcnt + nr;
  uint32_t* dtgt = dtake + rounds;
  uint32_t* dpop = dtgt + nr;
  uint32_t* ddepth = dpop + nr;
  if (e == hipSuccess) e = hipMemset(d, 0, b64 + b32);
  if (e == hipSuccess) e = hipMemcpy(dval, val, nr * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dseed, seed, 64 * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dcnt, cnt, nr * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dtake, take, rounds * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dtgt, tgt, nr * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hrt::launch_wq_protocol_check(rounds, dcnt, dtake, dtgt, dval, dseed, dpop, dseen, dslots, ddepth, nullptr);
  if (e == hipSuccess) e = hipMemcpy(popped, dpop, nr * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(seen, dseen, nr * 8, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(slots, dslots, 64 * 8, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(depth, ddepth, 4, hipMemcpyDeviceToHost);
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hrt_debug_wq_protocol");
  return HRT_OK;
}

// Test support: the band lists' wave flattening (hrt_kernels.hip BandFlat) on 64 given lists;
// owner_entry[(r * 64 + l) * 2 + {0, 1}] = owner lane and entry of slot r * 64 + l, r < rounds.
extern "C" hrt_status hrt_debug_band_flatten(int device, const uint32_t n[64], const uint32_t b0[64], uint32_t rounds,
                                             uint32_t* owner_entry, uint32_t* total) {
  if (!n || !b0 || !owner_entry || !total || rounds == 0 || rounds > 4096)
    return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_band_flatten: bad arguments");
  uint32_t* d = nullptr;
  const size_t words = 128 + (size_t)rounds * 128 + 1;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc((void**)&d, words * 4);
  if (e == hipSuccess) e = hipMemcpy(d, n, 64 * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 64, b0, 64 * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hrt::launch_band_flatten_check(d, d + 64, rounds, d + 128, nullptr);
  if (e == hipSuccess) e = hipMemcpy(owner_entry, d + 128, (size_t)rounds * 128 * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(total, d + 128 + (size_t)rounds * 128, 4, hipMemcpyDeviceToHost);
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hrt_debug_band_flatten");
  return HRT_OK;
}

extern "C" hrt_status hrt_debug_unmap_memory(void* ptr, uint64_t size) {
  if (hipMemUnmap(ptr, size) != hipSuccess || hipMemAddressFree(ptr, size) != hipSuccess) return HRT_ERR_HIP;
  return HRT_OK;
}

extern "C" hrt_status hrt_read_rays(hrt_context* ctx, hrt_ray* out, uint32_t n) {
  if (!ctx || (!out && n) || (uint64_t)n > ctx->n_rays || !ctx->scene.rays)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_rays: no rays or n too large");
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if (n) HRT_HIP(ctx, hipMemcpy(out, ctx->scene.rays, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost));
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
  for (uint32_t i = 0; i < count; ++i) out[i] = ctx->scene.bvh_info[i];
  return HRT_OK;
}

extern "C" hrt_status hrt_reset_stats(hrt_context* ctx) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  hrt_status st = hrt_synchronize(ctx);
  if (st != HRT_OK) return st;
  if ((st = harvest_events(ctx)) != HRT_OK) return st;
  HRT_HIP(ctx, hipMemsetAsync(ctx->counters, 0, hrt::kNumCounters * sizeof(unsigned long long), ctx->stream));
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
      if (value == 2 && !ctx->tile_cycles) {  // allocated here, so that hrt_trace never allocates
        hrt_status st = hrt_synchronize(ctx);
        if (st != HRT_OK) return st;
        HRT_HIP(ctx, hrt::dev_alloc(ctx, (void**)&ctx->tile_cycles,
                               std::max<size_t>(ctx->num_tiles(), 1) * 4 * sizeof(unsigned long long)));
      }
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
#ifdef HRT_DEBUG_OPTIONS
      if (value < 0 || value > 2) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "priority must be 0, 1 or 2");
#else
      if (value < 0 || value > 1)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT,
                    "priority must be 0 or 1 (2, heavy tiles only, is in libhip_raytrace_debug.so)");
#endif
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
    case HRT_OPT_OVERLAP:
      if (value < 0 || value > hrt::kLanes)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "overlap must be 0..3 trace lanes (0 and 1: one lane)");
      ctx->overlap = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_BUSY_SPLIT:
      if (value < 1 || value > 8) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "busy split must be in [1, 8]");
      ctx->busy_split = (uint32_t)value;
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
    case HRT_OPT_BVH_WIDTH:
      if (value < 2 || value > (int64_t)hrt::kWqMaxWidth)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "BVH width must be in [2, 4]");
      ctx->bvh_width = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_WQ_NODE_RADIUS:
      if (value < 0 || value > 2) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "wq node radius must be 0 (auto), 1 or 2");
      ctx->wq_node_radius = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_DEFER_COMBINE: {
      if (value < 0 || value > 1) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "defer combine must be 0 or 1");
      hrt_status st = bind(ctx);
      if (st == HRT_OK) st = hrt::flush_combines(ctx);
      if (st != HRT_OK) return st;
      ctx->defer = (uint32_t)value;
      return HRT_OK;
    }
    case HRT_OPT_COMM_TIMEOUT_MS:
      if (value < 0 || value > 0xFFFFFFFFll)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "comm timeout must be in [0, 2^32) ms (0 = wait forever)");
      ctx->comm_timeout_ms = (uint32_t)value;
      return HRT_OK;
    case HRT_OPT_BVH_LEAF_SIZE:
      if (value < 0 || value > hrt::kBvhMaxLeafCount)
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "BVH leaf size must be 0 (auto) or in [1, 16]");
      ctx->bvh_leaf = (uint32_t)value;
      return HRT_OK;
#ifdef HRT_DEBUG_OPTIONS
    case HRT_OPT_GRID_CUS:
      if (value < 0) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "grid CUs must be >= 0");
      ctx->grid_cus = (uint32_t)value;
      return HRT_OK;
    case HRT_DEBUG_OPT_FAIL_ALLOC:
      if (value < 0) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "fail-alloc index must be >= 0");
      ctx->debug_fail_alloc = value;
      return HRT_OK;
    case HRT_DEBUG_OPT_WQ_TRI_CAP:
      if (value != 0 && (value < 128 || value > (1 << 20)))
        return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "wq tri cap must be 0 (auto) or in [128, 2^20]");
      ctx->debug_wq_tri_cap = (uint32_t)value;
      return HRT_OK;
    case HRT_DEBUG_OPT_GRAB_RUNS:
      if (value < 0 || value > 1) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "grab runs must be 0 or 1");
      ctx->debug_grab_runs = (uint32_t)value;
      return HRT_OK;
    case HRT_DEBUG_OPT_STACK_LIMIT:
      if (value < 0) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "stack limit must be >= 0");
      ctx->debug_stack_limit = value;
      ctx->frame_stack_failed = 0;
      return HRT_OK;
#else
    case HRT_OPT_GRID_CUS:
    case HRT_DEBUG_OPT_FAIL_ALLOC:
    case HRT_DEBUG_OPT_WQ_TRI_CAP:
    case HRT_DEBUG_OPT_GRAB_RUNS:
    case HRT_DEBUG_OPT_STACK_LIMIT:
      return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "debug option: only libhip_raytrace_debug.so accepts it");
#endif
    case HRT_DEBUG_OPT_TIMELINE:
#if HRT_TIMELINE
      if (value <= 0 || value > (1 << 24)) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "timeline capacity in [1, 2^24]");
      if (ctx->timeline) {
        HRT_HIP(ctx, hipDeviceSynchronize());  // (every lane's stream: a launch may still be recording)
        free_dev(ctx, ctx->timeline);
        free_dev(ctx, ctx->timeline_count);
      }
      HRT_HIP(ctx, hrt::dev_alloc(ctx, (void**)&ctx->timeline, (size_t)value * 4 * sizeof(unsigned long long)));
      HRT_HIP(ctx, hrt::dev_alloc(ctx, (void**)&ctx->timeline_count, sizeof(uint32_t)));
      HRT_HIP(ctx, hipMemset(ctx->timeline_count, 0, sizeof(uint32_t)));
      ctx->timeline_cap = (uint32_t)value;
      return HRT_OK;
#else
      return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "timeline option: only builds with -DHRT_TIMELINE=1 accept it");
#endif
    default:
      return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "unknown option key");
  }
}

// Test / tuning support (HRT_TIMELINE builds): the last trace launch's per-item records.
extern "C" hrt_status hrt_debug_timeline(hrt_context* ctx, uint64_t* out, uint32_t cap, uint32_t* count) {
  if (!ctx || !out || !count) return HRT_ERR_INVALID_ARGUMENT;
  if (!ctx->timeline) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_debug_timeline: HRT_DEBUG_OPT_TIMELINE not set");
  if (bind(ctx) != HRT_OK) return HRT_ERR_HIP;
  HRT_HIP(ctx, hipDeviceSynchronize());
  uint32_t n = 0;
  HRT_HIP(ctx, hipMemcpy(&n, ctx->timeline_count, sizeof n, hipMemcpyDeviceToHost));
  n = std::min(n, ctx->timeline_cap);
  *count = n;
  HRT_HIP(ctx, hipMemcpy(out, ctx->timeline, (size_t)std::min(n, cap) * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return HRT_OK;
}

// Work the caller enqueues on the stream follows every accumulate so far: the deferred ones are folded.
extern "C" void* hrt_stream(hrt_context* ctx) {
  if (!ctx || bind(ctx) != HRT_OK || hrt::flush_combines(ctx) != HRT_OK) return ctx ? (void*)ctx->stream : nullptr;
  return (void*)ctx->stream;
}

extern "C" hrt_status hrt_release_caches(uint64_t* freed_bytes) {
  const uint64_t bytes = hrt::release_band_cache();
  if (freed_bytes) *freed_bytes = bytes;
  return HRT_OK;
}

extern "C" const char* hrt_last_error(const hrt_context* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}
