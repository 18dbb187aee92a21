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
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "hip_raytrace.h"
#include "hrt_context.h"
#include "hrt_kernels.h"

namespace {

struct Rccl {
  bool loaded = false;
  std::string error;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGather) gather = nullptr;
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
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_init_all, "ncclCommInitAll");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.gather, "ncclGather");
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
  ncclComm_t nccl = nullptr;     // nullptr for in-process device copies
  std::shared_ptr<Group> group;  // hrt_comm_init_all
  hipEvent_t ev = nullptr;       // in-process copies: this member's image is ready / has been read
  // root (rank 0) only
  void* gather_buf = nullptr;  // world x local image (rank-major)
  void* frame_buf = nullptr;   // the assembled full frame, context pixel format
  void* conv_buf = nullptr;    // the full frame in the other format (hrt_read_image fmt conversion)
};

void comm_release(hrt_context* ctx) {
  Comm* c = ctx->comm;
  if (!c) return;
  (void)hipSetDevice(ctx->device);
  if (c->nccl && rccl()->comm_destroy) (void)rccl()->comm_destroy(c->nccl);
  dev_free(ctx, c->gather_buf);
  dev_free(ctx, c->frame_buf);
  dev_free(ctx, c->conv_buf);
  if (c->ev) (void)hipEventDestroy(c->ev);
  if (c->group) {
    c->group->broken = true;
    for (auto& m : c->group->members)
      if (m == ctx) m = nullptr;
  }
  delete c;
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

// One process per GPU: this rank's block goes to rank 0, which assembles and copies the frame.
hrt_status read_process(hrt_context* ctx, Comm* c, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes) {
  hrt_status st;
  if (c->rank == 0 && (st = check_dst(ctx, fmt, dst, bytes)) != HRT_OK) return st;
  if ((st = bind(ctx)) != HRT_OK) return st;
  const void* src = local_image(ctx, image_id);
  if (!src) return fail(ctx, HRT_ERR_HIP, "hrt_read_image: lane wait failed");
  const size_t count = ctx->npix() * ctx->px_bytes();
  ncclResult_t r = rccl()->gather(src, c->rank == 0 ? c->gather_buf : nullptr, count, ncclUint8, 0, c->nccl, ctx->stream);
  if (r != ncclSuccess) return fail(ctx, HRT_ERR_HIP, nccl_msg("ncclGather", r));
  if (c->rank == 0) {
    if ((st = assemble_and_copy(ctx, c, fmt, dst)) != HRT_OK) return st;
  } else {
    HRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return image_id == HRT_IMG_TRACE ? release_lane(ctx, ctx->cur_lane) : HRT_OK;
}

// One process, every context: grouped RCCL gathers (distinct devices) or device copies, then the
// root's assembly.  Any member may call it; the frame lands in dst.
hrt_status read_group(hrt_context* ctx, Comm* c, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes) {
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

hrt_status comm_read_image(hrt_context* ctx, uint32_t image_id, uint32_t fmt, void* dst, size_t bytes) {
  Comm* c = ctx->comm;
  return c->group ? read_group(ctx, c, image_id, fmt, dst, bytes) : read_process(ctx, c, image_id, fmt, dst, bytes);
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
  if (!ctx || !id || world == 0 || rank >= world) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_init: bad rank/world");
  if (ctx->comm) return fail(ctx, HRT_ERR_INVALID_ARGUMENT, "hrt_comm_init: the context already has a communicator");
  if (!hrt::partition_matches(ctx, rank, world))
    return fail(ctx, HRT_ERR_INVALID_ARGUMENT,
                "hrt_comm_init: the context's partition must be part `rank` of `world` (hrt_create_info)");
  const Rccl* r = rccl();
  if (!r->loaded) return fail(ctx, HRT_ERR_NO_DEVICE, r->error);
  hrt_status st = hrt::bind(ctx);
  if (st != HRT_OK) return st;
  auto* c = new hrt::Comm();
  c->rank = rank;
  c->world = world;
  c->transport = HRT_COMM_RCCL;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  ncclResult_t res = r->comm_init_rank(&c->nccl, (int)world, uid, (int)rank);
  if (res != ncclSuccess) {
    delete c;
    return fail(ctx, HRT_ERR_HIP, nccl_msg("ncclCommInitRank", res));
  }
  ctx->comm = c;
  if (rank == 0 && (st = hrt::alloc_root(ctx, c)) != HRT_OK) {
    std::string msg = ctx->err;
    hrt::comm_release(ctx);
    return fail(ctx, st, msg);
  }
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
