// hrt_comm_protocol.h -- the error protocol of the one-process-per-GPU framebuffer gather
// (hrt_comm.cpp), independent of the transport so that it is unit-tested on the CPU
// (tests/cpp/comm_protocol_test.cpp: threads as ranks) as well as driven by RCCL on the GPU.
//
// The hazard: hrt_comm_init and hrt_read_image are collective.  A
// rank that returns an error BEFORE entering the collective (a bad destination on rank 0, a failed
// allocation, a lane wait that failed) leaves every peer blocked in it forever.  The protocol:
//
//   1. every rank enters an AGREEMENT step whatever its local status -- an all-reduce (max) of
//      encode(local status, rank), 4 bytes;
//   2. if any rank failed, every rank returns an error (the failing rank its own status, the others
//      HRT_ERR_COMM naming the failing rank) and NO rank enters the data collective;
//   3. otherwise the data collective runs;
//   4. a transport failure or a wait past the deadline (a peer that never arrived, an RCCL async
//      error) aborts the communicator (ncclCommAbort) -- the caller marks it broken, every later
//      collective call fails at once -- and returns HRT_ERR_COMM.
//
// Transport (duck-typed): bool agree(int mine, int* max_over_ranks); bool collective(); void abort();
// each returns false on failure or timeout (the transport owns the deadline).
#pragma once

#include <cstdint>
#include <string>

#include "hip_raytrace.h"

namespace hrt {
namespace proto {

constexpr int kRankBits = 12;  // world <= 4096
constexpr uint32_t kMaxWorld = 1u << kRankBits;

// 0 for HRT_OK; else status and rank in one int whose max over the ranks is the largest failing
// status (of the highest failing rank).
inline int encode(hrt_status st, uint32_t rank) { return st == HRT_OK ? 0 : ((int)st << kRankBits) | (int)rank; }
inline hrt_status decoded_status(int v) { return (hrt_status)(v >> kRankBits); }
inline uint32_t decoded_rank(int v) { return (uint32_t)v & (kMaxWorld - 1); }

struct Outcome {
  hrt_status status = HRT_OK;
  bool aborted = false;      // the communicator was aborted: the caller marks it broken
  bool ran_collective = false;
  std::string msg;           // for hrt_last_error (empty when status is this rank's own local error)
};

// Steps 1-2: every rank calls this with its local status; the result is the same decision on every
// rank (all proceed, or all return an error).
template <class Transport>
Outcome agree(Transport& t, hrt_status local, uint32_t rank, const char* what) {
  Outcome o;
  int agreed = 0;
  if (!t.agree(encode(local, rank), &agreed)) {
    t.abort();
    o.status = HRT_ERR_COMM;
    o.aborted = true;
    o.msg = std::string(what) + ": the status agreement between the ranks failed or timed out "
            "(a rank never arrived); the communicator was aborted";
    return o;
  }
  if (agreed != 0) {
    if (local != HRT_OK) {
      o.status = local;  // the caller's own error message stands
    } else {
      o.status = HRT_ERR_COMM;
      o.msg = std::string(what) + ": rank " + std::to_string(decoded_rank(agreed)) + " failed with status " +
              std::to_string((int)decoded_status(agreed)) + "; no rank entered the collective";
    }
  }
  return o;
}

// Steps 1-4 for a call whose data collective is t.collective().
template <class Transport>
Outcome run(Transport& t, hrt_status local, uint32_t rank, const char* what) {
  Outcome o = agree(t, local, rank, what);
  if (o.status != HRT_OK) return o;
  o.ran_collective = true;
  if (!t.collective()) {
    t.abort();
    o.status = HRT_ERR_COMM;
    o.aborted = true;
    o.msg = std::string(what) + ": the collective failed or timed out; the communicator was aborted";
  }
  return o;
}

}  // namespace proto
}  // namespace hrt
