"""bench.py's launch logic, CPU only (VERDICT r02 missing #1: `bench.py --gpus N` without torchrun used
to print a single-rank line).  resolve_launch decides between spawning the ranks and running as one;
spawn_ranks starts fresh rank processes with the torch.distributed.run environment and propagates the
first failure.  The ranks here are small Python stand-ins, not the benchmark (which needs a GPU)."""
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_resolve_launch():
    assert bench.resolve_launch(1, {}) == ("rank", 1)
    assert bench.resolve_launch(8, {}) == ("spawn", 8)          # no launcher: bench.py starts 8 ranks
    assert bench.resolve_launch(4, {"WORLD_SIZE": "4"}) == ("rank", 4)
    assert bench.resolve_launch(1, {"WORLD_SIZE": "1"}) == ("rank", 1)
    with pytest.raises(SystemExit, match="WORLD_SIZE=8"):
        bench.resolve_launch(2, {"WORLD_SIZE": "8"})            # contradicts the launcher: an error
    with pytest.raises(SystemExit, match="WORLD_SIZE=1"):
        bench.resolve_launch(8, {"WORLD_SIZE": "1"})            # never a silent single-rank line
    with pytest.raises(SystemExit):
        bench.resolve_launch(0, {})


def test_spawned_ranks_get_the_distributed_environment(tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    code = ("import os, sys; e = os.environ; "
            "open(os.path.join(sys.argv[1], e['RANK']), 'w').write(' '.join(e[k] for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', 'BENCH_SPAWNED')))")
    assert bench.spawn_ranks(3, [str(out)], cmd=[sys.executable, "-c", code]) == 0
    got = {p.name: p.read_text().split() for p in out.iterdir()}
    assert sorted(got) == ["0", "1", "2"]
    ports = {v[4] for v in got.values()}
    assert len(ports) == 1 and int(ports.pop()) > 0              # one rendezvous for all ranks
    for r, v in got.items():
        assert v[:4] == [r, r, "3", "127.0.0.1"] and v[5] == "1"


def test_a_failing_rank_ends_the_job_with_its_status(tmp_path):
    """Rank 1 fails at once; rank 0 would run for a minute: spawn_ranks returns rank 1's status
    promptly and leaves no rank running."""
    pidfile = tmp_path / "pid0"
    code = ("import os, sys, time; r = os.environ['RANK']; "
            "open(sys.argv[1], 'w').write(str(os.getpid())) if r == '0' else None; "
            "time.sleep(60) if r == '0' else sys.exit(3)")
    t = time.time()
    assert bench.spawn_ranks(2, [str(pidfile)], cmd=[sys.executable, "-c", code]) == 3
    assert time.time() - t < 30
    for _ in range(50):
        if pidfile.exists():
            break
        time.sleep(0.1)
    pid = int(pidfile.read_text())
    with pytest.raises(ProcessLookupError):
        os.kill(pid, 0)  # terminated (and reaped) by spawn_ranks


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """Run as a rank under a launcher with the RCCL gather and no GPU: a clear error, not a line."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "needs 2 GPUs" in r.stderr
    assert "metric" not in r.stdout


def test_assemble_ranks_says_whether_rccl_saw_every_rank():
    """The N > 1 line's "ranks" object: the communicator's world as each rank's
    library reports it (hrt_comm_info), the rank ids, and each rank's kernel and gather times."""
    def rec(r, cw=8, cr=None, g=1.5):
        return {"rank": r, "rccl_rank": r if cr is None else cr, "rccl_world": cw, "transport": 1,
                "kernel_ms": 0.3 + 0.01 * r, "gather_ms": None if g is None else g + r, "segments": 1000 + r}
    ok = bench.assemble_ranks([rec(r) for r in reversed(range(8))], 8)
    assert ok["rccl_ok"] and ok["rccl_world"] == {"min": 8, "max": 8} and ok["rccl_ranks"] == list(range(8))
    assert ok["kernel_ms"][0] == 0.3 and ok["kernel_ms_max"] == 0.37 and ok["gather_ms_max"] == 8.5
    assert ok["segments"] == [1000 + r for r in range(8)] and ok["transport"] == [1]
    split = bench.assemble_ranks([rec(r, cw=1, cr=0) if r == 3 else rec(r) for r in range(8)], 8)
    assert not split["rccl_ok"] and split["rccl_world"] == {"min": 1, "max": 8}
    assert not bench.assemble_ranks([rec(r) for r in range(7)], 8)["rccl_ok"]  # a rank never reported
    assert bench.assemble_ranks([rec(r, cw=2, g=None) for r in range(2)], 2)["gather_ms_max"] is None


def test_rank_records_reach_rank_0_over_gloo(tmp_path):
    """Two stand-in ranks (gloo on the CPU, the real rank_record / all_gather_object / assemble_ranks with a
    stand-in context whose comm_info is the library's answer) produce rank 0's "ranks" object."""
    out = tmp_path / "ranks.json"
    code = (
        "import json, os, sys; sys.path.insert(0, sys.argv[2]); import bench, torch.distributed as dist\n"
        "dist.init_process_group('gloo'); r, w = dist.get_rank(), dist.get_world_size()\n"
        "class Ctx:\n"
        "    def comm_info(self): return (r, w, 1)\n"
        "recs = [None] * w\n"
        "dist.all_gather_object(recs, bench.rank_record(Ctx(), r, w, True, 0.5 + r, 2.0 * (r + 1), 10 + r))\n"
        "if r == 0: open(sys.argv[1], 'w').write(json.dumps(bench.assemble_ranks(recs, w)))\n"
        "dist.barrier(); dist.destroy_process_group()\n")
    assert bench.spawn_ranks(2, [str(out), ROOT], cmd=[sys.executable, "-c", code]) == 0
    import json
    got = json.loads(out.read_text())
    assert got["rccl_ok"] and got["rccl_world"] == {"min": 2, "max": 2} and got["rccl_ranks"] == [0, 1]
    assert got["kernel_ms"] == [0.5, 1.5] and got["gather_ms"] == [2.0, 4.0] and got["gather_ms_max"] == 4.0


def test_gloo_rehearsal_has_no_rccl_claims():
    recs = [{"rank": r, "rccl_rank": None, "rccl_world": None, "transport": 0, "kernel_ms": 1.0, "gather_ms": 4.0,
             "segments": 10} for r in range(2)]
    got = bench.assemble_ranks(recs, 2)
    assert got["rccl_ok"] is None and got["rccl_world"] is None and got["rccl_ranks"] is None
    assert got["gather_ms_max"] == 4.0 and got["reported"] == 2
