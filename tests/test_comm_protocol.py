"""The collective error protocol of the multi-GPU gather (epq_raytracer_amd/csrc/hrt_comm_protocol.h),
CPU only: tests/cpp/comm_protocol_test runs hrt_comm_init's and hrt_read_image's protocol with threads
as ranks over a shared-memory transport with the RCCL transport's deadline semantics (VERDICT r02
weak #5 / ADVICE r02: rank 0 used to return on a bad destination before entering ncclGather, leaving
every peer blocked).  The reference has no multi-GPU path; what it gathers is image()
(src/raytrace_pipeline.rs:156, src/diffuse.rs:69)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "comm_protocol_test")
OK, INVALID, OOM, HIP, COMM = 0, 1, 3, 5, 7


@pytest.fixture(scope="module")
def scenarios():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "comm_protocol_test"], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return {d["scenario"]: d for d in map(json.loads, r.stdout.splitlines())}


def test_all_ranks_ok_gather(scenarios):
    s = scenarios["all_ok"]
    assert s["status"] == [OK] * 8 and s["gathered"] == [1] * 8 and not any(s["aborted"])


def test_rank0_argument_error_is_an_error_on_every_rank(scenarios):
    s = scenarios["rank0_bad_destination"]
    assert s["status"] == [INVALID] + [COMM] * 7   # rank 0 keeps its own status, peers get HRT_ERR_COMM
    assert s["gathered"] == [0] * 8                  # nobody entered the gather
    assert not any(s["aborted"]) and s["ms"] < 250   # decided by the agreement, not by a timeout


@pytest.mark.parametrize("name,failing", [("rank5_lane_wait_failed", {5: HIP}),
                                          ("two_ranks_fail", {1: OOM, 3: INVALID})])
def test_peer_errors_propagate(scenarios, name, failing):
    s = scenarios[name]
    assert s["status"] == [failing.get(r, COMM) for r in range(s["world"])]
    assert not any(s["gathered"]) and not any(s["aborted"])


@pytest.mark.parametrize("name", ["rank3_absent", "rank0_absent"])
def test_a_rank_that_never_arrives_times_out_and_aborts(scenarios, name):
    s = scenarios[name]
    present = [r for r in range(s["world"]) if r != s["absent"]]
    assert all(s["status"][r] == COMM and s["aborted"][r] == 1 for r in present)
    assert not any(s["gathered"])
    assert s["ms"] < 5000  # bounded by the transport's deadline (300 ms here)


def test_single_rank(scenarios):
    assert scenarios["single_rank_ok"]["status"] == [OK] and scenarios["single_rank_ok"]["gathered"] == [1]
    assert scenarios["single_rank_bad"]["status"] == [INVALID] and scenarios["single_rank_bad"]["gathered"] == [0]


def test_init_agreement(scenarios):
    """hrt_comm_init: a partition mismatch or the root's failed allocation (now made BEFORE
    ncclCommInitRank) fails the init on every rank; nobody keeps a half-formed communicator."""
    assert scenarios["init_partition_mismatch_rank2"]["status"] == [COMM, COMM, INVALID, COMM]
    assert scenarios["init_root_alloc_failed"]["status"] == [OOM] + [COMM] * 7
    assert scenarios["init_all_ok"]["status"] == [OK] * 8
