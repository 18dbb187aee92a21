// CPU test of the collective error protocol (epq_raytracer_amd/csrc/hrt_comm_protocol.h) that
// hrt_comm_init and hrt_read_image run over RCCL: ranks are threads, the transport is a shared-memory
// all-reduce / gather with the same deadline semantics as the RCCL transport (a rank that never
// arrives makes the others time out and abort).  Prints one JSON line per scenario:
//   {"scenario": ..., "status": [per rank], "gathered": [per rank], "aborted": [per rank], "ms": wall}
// tests/test_comm_protocol.py runs it and checks that no scenario hangs and that an error on any rank
// (rank 0's bad destination included) is an error on every rank with no gather.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hrt_comm_protocol.h"

namespace {

using clock_t_ = std::chrono::steady_clock;

// A rendezvous of `world` ranks per round; a round completes when every rank has arrived.
struct Fabric {
  int world;
  int timeout_ms;
  std::mutex m;
  std::condition_variable cv;
  std::vector<long> round_arrivals;  // per round id: arrivals so far
  std::vector<int> round_max;
  bool aborted = false;

  Fabric(int w, int t) : world(w), timeout_ms(t), round_arrivals(16, 0), round_max(16, 0) {}

  // Returns false on timeout or when another rank aborted.
  bool meet(int round, int value, int* max_out) {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    round_arrivals[round]++;
    round_max[round] = std::max(round_max[round], value);
    cv.notify_all();
    const bool ok = cv.wait_for(lk, std::chrono::milliseconds(timeout_ms),
                                [&] { return aborted || round_arrivals[round] == world; });
    if (!ok || round_arrivals[round] != world) return false;
    if (max_out) *max_out = round_max[round];
    return true;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

struct ThreadTransport {
  Fabric* f;
  int next_round = 0;
  bool gathered = false;
  bool did_abort = false;
  bool agree(int mine, int* max_over_ranks) { return f->meet(next_round++, mine, max_over_ranks); }
  bool collective() {
    gathered = f->meet(next_round++, 0, nullptr);
    return gathered;
  }
  void abort() {
    did_abort = true;
    f->abort();
  }
};

struct Scenario {
  std::string name;
  int world;
  std::function<hrt_status(int)> local;  // per-rank local status (the call's own checks)
  int absent = -1;                       // a rank that never calls (crashed before the collective)
  bool init_only = false;                // hrt_comm_init: agreement only, no data collective
};

void run(const Scenario& sc) {
  Fabric fabric(sc.world, 300);
  std::vector<int> status(sc.world, -1), gathered(sc.world, 0), aborted(sc.world, 0);
  std::vector<std::thread> th;
  const auto t0 = clock_t_::now();
  for (int r = 0; r < sc.world; ++r) {
    if (r == sc.absent) continue;
    th.emplace_back([&, r] {
      ThreadTransport t{&fabric};
      const hrt_status local = sc.local(r);
      const hrt::proto::Outcome o = sc.init_only ? hrt::proto::agree(t, local, (uint32_t)r, "hrt_comm_init")
                                                 : hrt::proto::run(t, local, (uint32_t)r, "hrt_read_image");
      status[r] = (int)o.status;
      gathered[r] = t.gathered ? 1 : 0;
      aborted[r] = o.aborted ? 1 : 0;
    });
  }
  for (auto& x : th) x.join();
  const double ms = std::chrono::duration<double, std::milli>(clock_t_::now() - t0).count();
  auto arr = [](const std::vector<int>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]);
    return s + "]";
  };
  std::printf("{\"scenario\": \"%s\", \"world\": %d, \"absent\": %d, \"status\": %s, \"gathered\": %s, "
              "\"aborted\": %s, \"ms\": %.1f}\n",
              sc.name.c_str(), sc.world, sc.absent, arr(status).c_str(), arr(gathered).c_str(), arr(aborted).c_str(),
              ms);
  std::fflush(stdout);
}

}  // namespace

int main() {
  const auto ok = [](int) { return HRT_OK; };
  std::vector<Scenario> all = {
      {"all_ok", 8, ok},
      {"rank0_bad_destination", 8, [](int r) { return r == 0 ? HRT_ERR_INVALID_ARGUMENT : HRT_OK; }},
      {"rank5_lane_wait_failed", 8, [](int r) { return r == 5 ? HRT_ERR_HIP : HRT_OK; }},
      {"two_ranks_fail", 4, [](int r) { return r == 1 ? HRT_ERR_OUT_OF_MEMORY : r == 3 ? HRT_ERR_INVALID_ARGUMENT : HRT_OK; }},
      {"rank3_absent", 4, ok, 3},
      {"rank0_absent", 2, ok, 0},
      {"single_rank_ok", 1, ok},
      {"single_rank_bad", 1, [](int) { return HRT_ERR_INVALID_ARGUMENT; }},
      {"init_partition_mismatch_rank2", 4, [](int r) { return r == 2 ? HRT_ERR_INVALID_ARGUMENT : HRT_OK; }, -1, true},
      {"init_root_alloc_failed", 8, [](int r) { return r == 0 ? HRT_ERR_OUT_OF_MEMORY : HRT_OK; }, -1, true},
      {"init_all_ok", 8, ok, -1, true},
  };
  for (const auto& sc : all) run(sc);
  return 0;
}
