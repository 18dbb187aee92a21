// hrt_comm.cpp -- the multi-GPU framebuffer gather behind hrt_read_image.
//
// A row-tile partition renders with no exchange at all (a pixel depends only on scene, camera,
// rng_offset and its global id, assets/raytracing.glsl:376-385); the one collective is the gather of
// the framebuffer for the present (the reference's image(), src/raytrace_pipeline.rs:156 and
// src/diffuse.rs:69, handed to RenderPassOverFrame::render).  Every part stores the same number of
// local rows, so it is ONE ncclGather (RCCL extension, rccl.h:745) of equal-size blocks to rank 0,
// followed by the row un-interleave on rank 0's device (assemble_rows) and the copy to the caller.
//
// Two ways to form the group:
//   * hrt_comm_init       -- one process (or host thread) per GPU, ncclCommInitRank with an id from
//                            hrt_comm_unique_id (the torch.distributed.run layout of bench.py);
//   * hrt_comm_init_all   -- one process driving every context (the reference's single Rust process):
//                            ncclCommInitAll over the contexts' devices and grouped ncclGather calls;
//                            contexts that share a device (oversubscription, tests on one GPU) use
//                            device-to-device copies instead, through the same assembly.
// RCCL is loaded with dlopen on the first hrt_comm_* call, so single-GPU users never load it.
//
// Errors on the process path (hrt_comm_init, read_process) follow hrt_comm_protocol.h: every rank
// agrees on the call's status (a 4-byte ncclAllReduce) before any data moves, so an error on one rank
// is an error on every rank instead of peers blocked forever in the collective; waits are bounded by
// HRT_OPT_COMM_TIMEOUT_MS and a timeout or RCCL async error aborts the communicator (ncclCommAbort).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "hip_raytrace.h"
#include "hrt_comm_protocol.h"
#include "hrt_context.h"
#include "hrt_kernels.h"

namespace {

struct Rccl {
  bool loaded = false;
  std::string error;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRankConfig) comm_init_rank_config = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) r.error = std::string("librccl.so.1 lacks ") + name;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank_config, "ncclCommInitRankConfig");
    sym(r.comm_init_all, "ncclCommInitAll");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.comm_abort, "ncclCommAbort");
    sym(r.async_error, "ncclCommGetAsyncError");
    sym(r.gather, "ncclGather");
    sym(r.all_reduce, "ncclAllReduce");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.error_string, "ncclGetErrorString");
    r.loaded = r.error.empty();
  });
  return &r;
}

std::string nccl_msg(const char* what, ncclResult_t res) {
  const Rccl* r = rccl();
  return std::string(what) + ": " + (r->error_string ? r->error_string(res) : "RCCL error") + " (" +
         std::to_string((int)res) + ")";
}

}  // namespace

namespace hrt {

struct Group {
  std::vector<hrt_context*> members;  // members[i] renders part i; members[0] is the root
  bool broken = false;                // a member was destroyed
};

struct Comm {
  uint32_t rank = 0, world = 1, transport = HRT_COMM_NONE;
  ncclComm_t nccl = nullptr;     // nullptr for in-process device copies (or after an abort)
  bool broken = false;           // aborted after a failure / timeout: every later collective fails
  std::shared_ptr<Group> group;  // hrt_comm_init_all
  hipEvent_t ev = nullptr;       // in-process copies: this member's image is ready / has been read
  int* dev_status = nullptr;     // hrt_comm_init: the status agreement's all-reduce word (device)
  int* host_status = nullptr;    // ... and its pinned host copy
  // root (rank 0) only
  void* gather_buf = nullptr;  // world x local image (rank-major)
  void* frame_buf = nullptr;   // the assembled full frame, context pixel format
  void* conv_buf = nullptr;    // the full frame in the other format (hrt_read_image fmt conversion)
};

namespace {

// Frees a communicator that is not (or no longer) attached to ctx.
void free_comm(hrt_context* ctx, Comm* c) {
  if (!c) return;
  (void)hipSetDevice(ctx->device);
  if (c->nccl && rccl()->comm_destroy) (void)rccl()->comm_destroy(c->nccl);
  dev_free(ctx, c->gather_buf);
  dev_free(ctx, c->frame_buf);
  dev_free(ctx, c->conv_buf);
  dev_free(ctx, c->dev_status);
  if (c->host_status) (void)hipHostFree(c->host_status);
  if (c->ev) (void)hipEventDestroy(c->ev);
  delete c;
}

}  // namespace

void comm_release(hrt_context* ctx) {
  Comm* c = ctx->comm;
  if (!c) return;
  if (c->group) {
    c->group->broken = true;
    for (auto& m : c->group->members)
      if (m == ctx) m = nullptr;
  }
  free_comm(ctx, c);
  ctx->comm = nullptr;
}

namespace {

hrt_status alloc_root(hrt_context* ctx, Comm* c) {
  const size_t local = ctx->npix() * ctx->px_bytes(), full = (size_t)ctx->width * ctx->height;
  HRT_HIP(ctx, dev_alloc(ctx, &c->gather_buf, std::max<size_t>((size_t)c->world * local, 16)));
  HRT_HIP(ctx, dev_alloc(ctx, &c->frame_buf, full * ctx->px_bytes()));
  HRT_HIP(ctx, dev_alloc(ctx, &c->conv_buf, full * (ctx->mode == HRT_MODE_RGBA8 ? 16 : 4)));
  return HRT_OK;
}

// The context's partition must be part `rank` of `world` (or the whole image for a world of 1).
bool partition_matches(const hrt_context* ctx, uint32_t rank, uint32_t world) {
  return world == 1 ? ctx->part_count == 1 : ctx->part_count == world && ctx->part_index == rank;
}

// Root: un-interleave the gathered blocks into frame_buf and copy it out in fmt (blocking).
hrt_status assemble_and_copy(hrt_context* root, Comm* c, uint32_t fmt, void* dst) {
  const uint32_t row_words = (uint32_t)(root->width * root->px_bytes() / 4);
  const uint32_t row_tile = c->world == 1 ? root->height : root->row_tile;
  HRT_HIP(root, launch_assemble_rows(static_cast<const uint32_t*>(c->gather_buf), static_cast<uint32_t*>(c->frame_buf),
                                     row_words, root->height, root->local_rows, row_tile, c->world, root->stream));
  return copy_frame_out(root, c->frame_buf, (size_t)root->width * root->height, fmt, dst, c->conv_buf);
}

hrt_status check_dst(hrt_context* ctx, uint32_t fmt, void* dst, size_t bytes) {
  const size_t need = (size_t)ctx->width * ctx->height * (fmt == HRT_FMT_RGBA8 ? 4 : 16);
  if (!dst || bytes < need)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: the gathered frame needs width x height pixels");
  return HRT_OK;
}

hrt_status alloc_status(hrt_context* ctx, Comm* c) {
  HRT_HIP(ctx, dev_alloc(ctx, (void**)&c->dev_status, 64));
  HRT_HIP(ctx, hipHostMalloc((void**)&c->host_status, 64, hipHostMallocDefault));
  return HRT_OK;
}

// The RCCL transport of hrt_comm_protocol.h on the context's stream.  Every wait polls the stream and
// the communicator's async error, up to the context's HRT_OPT_COMM_TIMEOUT_MS.
struct RcclTransport {
  hrt_context* ctx;
  Comm* c;
  const void* src = nullptr;  // the gather's send block (this rank's local image)
  size_t count = 0;

  std::chrono::steady_clock::time_point deadline() const {
    return std::chrono::steady_clock::now() + std::chrono::milliseconds(ctx->comm_timeout_ms);
  }
  // The communicator is non-blocking: an RCCL call may return ncclInProgress while it is still being
  // set up / enqueued.  Polls its async state until settled (or the deadline); true on ncclSuccess.
  bool settle(ncclResult_t r) {
    const auto end = deadline();
    for (uint32_t spin = 0; r == ncclInProgress; ++spin) {
      if (rccl()->async_error(c->nccl, &r) != ncclSuccess) return false;
      if (r != ncclInProgress) break;
      if (ctx->comm_timeout_ms && std::chrono::steady_clock::now() > end) return false;
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    return r == ncclSuccess;
  }
  // The work enqueued on the context's stream has finished, with no RCCL async error, by the deadline.
  bool wait() {
    const auto end = deadline();
    for (uint32_t spin = 0;; ++spin) {
      const hipError_t q = hipStreamQuery(ctx->stream);
      if (q == hipSuccess) return true;
      if (q != hipErrorNotReady) {
        hip_fail(ctx, q, "hrt_comm: stream");
        return false;
      }
      ncclResult_t ae = ncclSuccess;
      if (rccl()->async_error(c->nccl, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress)) return false;
      if (ctx->comm_timeout_ms && std::chrono::steady_clock::now() > end) return false;
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  bool agree(int mine, int* max_over_ranks) {
    if (!c->nccl || !c->dev_status || !c->host_status) return false;
    *c->host_status = mine;
    if (hipMemcpyAsync(c->dev_status, c->host_status, sizeof(int), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
      return false;
    if (!settle(rccl()->all_reduce(c->dev_status, c->dev_status, 1, ncclInt32, ncclMax, c->nccl, ctx->stream)))
      return false;
    if (hipMemcpyAsync(c->host_status, c->dev_status, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
      return false;
    if (!wait()) return false;
    *max_over_ranks = *c->host_status;
    return true;
  }
  bool collective() {
    return settle(rccl()->gather(src, c->rank == 0 ? c->gather_buf : nullptr, count, ncclUint8, 0, c->nccl,
                                 ctx->stream)) &&
           wait();
  }
  void abort() {
    if (c->nccl && rccl()->comm_abort) (void)rccl()->comm_abort(c->nccl);
    c->nccl = nullptr;
  }
};

hrt_status outcome(hrt_context* ctx, const proto::Outcome& o) {
  return o.msg.empty() ? o.status : fail(ctx, o.status, o.msg);
}

// One process per GPU: this rank's block goes to rank 0, which assembles and copies the frame.  Every
// rank computes its local status and enters the agreement; only if all are OK does any rank gather.
hrt_status read_process(hrt_context* ctx, Comm* c, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes,
                        hrt_status local) {
  if (c->broken)
    return fail(ctx, HRT_ERR_COMM, "hrt_read_image: the communicator was aborted after an earlier failure");
  if (local == HRT_OK && c->rank == 0) local = check_dst(ctx, fmt, dst, bytes);
  const hrt_status bound = bind(ctx);
  if (local == HRT_OK) local = bound;
  RcclTransport t{ctx, c};
  if (local == HRT_OK && !(t.src = local_image(ctx, image_id)))
    local = fail(ctx, HRT_ERR_HIP, "hrt_read_image: lane wait failed");
  t.count = ctx->npix() * ctx->px_bytes();
  const proto::Outcome o = proto::run(t, local, c->rank, "hrt_read_image");
  if (o.aborted) c->broken = true;
  if (o.status != HRT_OK) return outcome(ctx, o);
  hrt_status st;
  if (c->rank == 0 && (st = assemble_and_copy(ctx, c, fmt, dst)) != HRT_OK) return st;
  return image_id == HRT_IMG_TRACE ? release_lane(ctx, ctx->cur_lane) : HRT_OK;
}

// One process, every context: grouped RCCL gathers (distinct devices) or device copies, then the
// root's assembly.  Any member may call it; the frame lands in dst.
hrt_status read_group(hrt_context* ctx, Comm* c, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes,
                      hrt_status arg) {
  if (arg != HRT_OK) return arg;  // one caller drives every member: nobody waits in a collective
  Group& g = *c->group;
  if (g.broken) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_read_image: a context of the group was destroyed");
  hrt_context* root = g.members[0];
  Comm* rc = root->comm;
  hrt_status st = check_dst(ctx, fmt, dst, bytes);
  if (st != HRT_OK) return st;
  const size_t count = root->npix() * root->px_bytes();
  std::vector<const void*> src(g.members.size());
  for (size_t i = 0; i < g.members.size(); ++i) {
    hrt_context* m = g.members[i];
    if ((st = bind(m)) != HRT_OK) return st;
    if (!(src[i] = local_image(m, image_id))) return fail(ctx, HRT_ERR_HIP, "hrt_read_image: lane wait failed");
  }
  if (c->transport == HRT_COMM_RCCL_GROUP) {
    ncclResult_t r = rccl()->group_start();
    for (size_t i = 0; r == ncclSuccess && i < g.members.size(); ++i) {
      hrt_context* m = g.members[i];
      (void)hipSetDevice(m->device);
      r = rccl()->gather(src[i], i == 0 ? rc->gather_buf : nullptr, count, ncclUint8, 0, m->comm->nccl, m->stream);
    }
    const ncclResult_t r2 = rccl()->group_end();
    if (r != ncclSuccess || r2 != ncclSuccess) return fail(ctx, HRT_ERR_HIP, nccl_msg("ncclGather", r ? r : r2));
  } else {  // contexts sharing a device: copies into the root's gather buffer, ordered by events
    if ((st = bind(root)) != HRT_OK) return st;
    for (size_t i = 0; i < g.members.size(); ++i) {
      hrt_context* m = g.members[i];
      if (i) {
        HRT_HIP(m, hipEventRecord(m->comm->ev, m->stream));
        HRT_HIP(root, hipStreamWaitEvent(root->stream, m->comm->ev, 0));
      }
      HRT_HIP(root, hipMemcpyAsync(static_cast<char*>(rc->gather_buf) + i * count, src[i], count, hipMemcpyDefault,
                                   root->stream));
    }
    // the members' next writes of these images follow the copies
    HRT_HIP(root, hipEventRecord(rc->ev, root->stream));
    for (size_t i = 1; i < g.members.size(); ++i)
      HRT_HIP(g.members[i], hipStreamWaitEvent(g.members[i]->stream, rc->ev, 0));
  }
  if ((st = bind(root)) != HRT_OK) return st;
  if ((st = assemble_and_copy(root, rc, fmt, dst)) != HRT_OK) {
    if (root != ctx) ctx->err = root->err;
    return st;
  }
  for (auto* m : g.members) {
    if ((st = bind(m)) != HRT_OK) return st;
    HRT_HIP(m, hipStreamSynchronize(m->stream));
    if (image_id == HRT_IMG_TRACE && (st = release_lane(m, m->cur_lane)) != HRT_OK) return st;
  }
  return bind(ctx);
}

}  // namespace

hrt_status comm_read_image(hrt_context* ctx, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes,
                           hrt_status arg) {
  Comm* c = ctx->comm;
  return c->group ? read_group(ctx, c, image_id, fmt, dst, bytes, arg)
                  : read_process(ctx, c, image_id, fmt, dst, bytes, arg);
}

}  // namespace hrt

using hrt::fail;

extern "C" hrt_status hrt_comm_unique_id(uint8_t id[HRT_COMM_ID_BYTES]) {
  if (!id) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_unique_id: null id");
  const Rccl* r = rccl();
  if (!r->loaded) return fail(nullptr, HRT_ERR_NO_DEVICE, r->error);
  static_assert(sizeof(ncclUniqueId) == HRT_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId uid;
  ncclResult_t res = r->get_unique_id(&uid);
  if (res != ncclSuccess) return fail(nullptr, HRT_ERR_HIP, nccl_msg("ncclGetUniqueId", res));
  std::memcpy(id, &uid, sizeof uid);
  return HRT_OK;
}

extern "C" hrt_status hrt_comm_init(hrt_context* ctx, const uint8_t id[HRT_COMM_ID_BYTES], uint32_t rank,
                                    uint32_t world) {
  // Arguments without which this rank cannot join the communicator at all.
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  if (!id || world == 0 || rank >= world || world > hrt::proto::kMaxWorld)
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_init: bad id / rank / world");
  const Rccl* r = rccl();
  if (!r->loaded) return fail(ctx, HRT_ERR_NO_DEVICE, r->error);
  hrt_status st = hrt::bind(ctx);
  if (st != HRT_OK) return st;
  // Everything else is agreed on after the communicator exists: a rank with a bad partition or a failed
  // allocation still joins, so that its peers are not left blocked in ncclCommInitRank, and then every
  // rank returns the error with no communicator.
  auto* c = new hrt::Comm();
  c->rank = rank;
  c->world = world;
  c->transport = HRT_COMM_RCCL;
  hrt_status local = HRT_OK;
  if (ctx->comm)
    local = fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_init: the context already has a communicator");
  else if (!hrt::partition_matches(ctx, rank, world))
    local = fail(ctx, HRT_ERR_INVALID_ARGUMENT,
                 "hrt_comm_init: the context's partition must be part `rank` of `world` (hrt_create_info)");
  if (hrt::alloc_status(ctx, c) != HRT_OK && local == HRT_OK) local = HRT_ERR_OUT_OF_MEMORY;
  // the root's gather buffers BEFORE the communicator (a failure is then agreed on, not a missing rank)
  if (local == HRT_OK && rank == 0) local = hrt::alloc_root(ctx, c);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  // non-blocking, so that a peer that never joins costs a timeout (then an abort), not a hang
  ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
  config.blocking = 0;
  ncclResult_t res = r->comm_init_rank_config(&c->nccl, (int)world, uid, (int)rank, &config);
  hrt::RcclTransport t{ctx, c};
  if ((res != ncclSuccess && res != ncclInProgress) || !c->nccl || !t.settle(res)) {
    t.abort();
    hrt::free_comm(ctx, c);
    // a rank that failed its own checks keeps its message; otherwise the init itself failed
    return local != HRT_OK ? local
                           : fail(ctx, HRT_ERR_COMM, "hrt_comm_init: ncclCommInitRankConfig failed or timed out (" +
                                                         nccl_msg("status", res) + "); the communicator was aborted");
  }
  const hrt::proto::Outcome o = hrt::proto::agree(t, local, rank, "hrt_comm_init");
  if (o.status != HRT_OK) {
    hrt::free_comm(ctx, c);  // (an aborted communicator is already gone)
    return hrt::outcome(ctx, o);
  }
  ctx->comm = c;
  return HRT_OK;
}

extern "C" hrt_status hrt_comm_init_all(hrt_context* const* ctxs, uint32_t n) {
  if (!ctxs || n == 0) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_init_all: no contexts");
  std::set<int> devs;
  for (uint32_t i = 0; i < n; ++i) {
    const hrt_context* m = ctxs[i];
    if (!m || m->comm) return fail(nullptr, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_init_all: null context or one with a communicator");
    if (!hrt::partition_matches(m, i, n) || m->width != ctxs[0]->width || m->height != ctxs[0]->height ||
        m->mode != ctxs[0]->mode || m->row_tile != ctxs[0]->row_tile || m->local_rows != ctxs[0]->local_rows)
      return fail(nullptr, HRT_ERR_INVALID_ARGUMENT,
                  "hrt_comm_init_all: ctxs[i] must be part i of n of the same image, mode and row tile");
    devs.insert(m->device);
  }
  const bool use_rccl = devs.size() == n;
  std::vector<ncclComm_t> comms(n, nullptr);
  if (use_rccl) {
    const Rccl* r = rccl();
    if (!r->loaded) return fail(nullptr, HRT_ERR_NO_DEVICE, r->error);
    std::vector<int> dl(n);
    for (uint32_t i = 0; i < n; ++i) dl[i] = ctxs[i]->device;
    ncclResult_t res = r->comm_init_all(comms.data(), (int)n, dl.data());
    if (res != ncclSuccess) return fail(nullptr, HRT_ERR_HIP, nccl_msg("ncclCommInitAll", res));
  }
  auto group = std::make_shared<hrt::Group>();
  group->members.assign(ctxs, ctxs + n);
  hrt_status st = HRT_OK;
  for (uint32_t i = 0; i < n; ++i) {
    hrt_context* m = ctxs[i];
    auto* c = new hrt::Comm();
    c->rank = i;
    c->world = n;
    c->transport = use_rccl ? HRT_COMM_RCCL_GROUP : HRT_COMM_DEVICE_COPY;
    c->nccl = comms[i];
    c->group = group;
    m->comm = c;
    if (st == HRT_OK && (st = hrt::bind(m)) == HRT_OK) {
      if (hipError_t e = hipEventCreateWithFlags(&c->ev, hipEventDisableTiming); e != hipSuccess)
        st = hrt::hip_fail(m, e, "hipEventCreate(comm)");
      else if (i == 0)
        st = hrt::alloc_root(m, c);
    }
    if (st != HRT_OK) fail(nullptr, st, m->err);
  }
  if (st != HRT_OK) {
    for (uint32_t i = 0; i < n; ++i) hrt::comm_release(ctxs[i]);
    return st;
  }
  return HRT_OK;
}

extern "C" hrt_status hrt_comm_info(const hrt_context* ctx, uint32_t* rank, uint32_t* world, uint32_t* transport) {
  if (!ctx) return HRT_ERR_INVALID_ARGUMENT;
  const hrt::Comm* c = ctx->comm;
  if (rank) *rank = c ? c->rank : 0;
  if (world) *world = c ? c->world : 1;
  if (transport) *transport = c ? c->transport : HRT_COMM_NONE;
  return HRT_OK;
}
