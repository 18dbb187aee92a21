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
