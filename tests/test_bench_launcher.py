"""bench.py --gpus N launches its own ranks when no launcher set WORLD_SIZE (CPU; a BFTSIM_TESTING stub
stands in for the GPU work of each rank): one process per rank with torch.distributed.run's environment,
rank 0's JSON line relayed, a failing rank fails the run, and the parent never imports torch / touches HIP."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, *argv, fail_rank=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(BFTSIM_TESTING="1", BFTSIM_BENCH_STUB_DIR=str(tmp_path))
    if fail_rank is not None:
        env["BFTSIM_BENCH_STUB_FAIL"] = str(fail_rank)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus_n_spawns_n_ranks_with_launcher_environment(tmp_path):
    r = _bench(tmp_path, "--gpus", "4", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1                                   # only rank 0's line on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["steps"] == 3 and out["warmup"] == 1
    parent = json.load(open(tmp_path / "parent.json"))
    assert parent["gpu_modules"] == []                       # the parent never imported torch / bftsim
    ranks = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    ports = {x["MASTER_PORT"] for x in ranks}
    assert len(ports) == 1 and ports.pop().isdigit()
    for r, x in enumerate(ranks):
        assert (x["RANK"], x["LOCAL_RANK"], x["WORLD_SIZE"], x["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "4", "4")
        assert x["MASTER_ADDR"] == "127.0.0.1"
        assert x["pid"] in parent["pids"] and x["ppid"] != x["pid"]   # fresh children, not an exec


def test_a_failing_rank_fails_the_run(tmp_path):
    r = _bench(tmp_path, "--gpus", "2", "--steps", "1", "--warmup", "0", fail_rank=1)
    assert r.returncode == 3


def test_gpus_1_runs_in_process(tmp_path):
    r = _bench(tmp_path, "--gpus", "1", "--steps", "2", "--warmup", "0")
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["n_gpus"] == 1
    assert not (tmp_path / "parent.json").exists()
    x = json.load(open(tmp_path / "rank0.json"))
    assert x["WORLD_SIZE"] is None                            # no launcher, no spawned environment


def test_external_launcher_environment_is_used(tmp_path):
    """under torch.distributed.run (WORLD_SIZE set) bench.py is one rank and spawns nothing"""
    env = dict(os.environ, BFTSIM_TESTING="1", BFTSIM_BENCH_STUB_DIR=str(tmp_path), WORLD_SIZE="2", RANK="1",
               LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == ""      # rank 1 prints nothing
    assert not (tmp_path / "parent.json").exists()
    assert json.load(open(tmp_path / "rank1.json"))["WORLD_SIZE"] == "2"
