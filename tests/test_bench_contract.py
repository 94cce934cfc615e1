"""bench.py driver contract on CPU: one JSON line from rank 0 with whole-job tokens/s, run as 2 DP ranks under
torch.distributed.run (gloo), the way the driver launches it for N > 1 (the GPU path differs only in the device)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(extra, n=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "4",
           "--warmup", "2", "--model", "tiny-llama", "--prefix-tokens", "200", "--threads", "4", "--min-out", "4",
           "--max-out", "8", "--user-tokens", "8", "--ttft-samples", "4", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1" if n > 2 else "2")
    p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=500)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_dp2_json_line():
    d = _run([])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 2 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 8
    assert d["scaling"] == "weak" and d["higher_is_better"] is True


@pytest.mark.timeout(600)
def test_bench_tp2_json_line():
    """--tp 2: one replica of two ranks (leader schedules, follower mirrors) — the 70B TP configuration's path."""
    d = _run(["--tp", "2"])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp1-tp2" and d["config"]["global_batch"] == 4


def _check_ranks(d, n, tp):
    """The self-verifying part of a multi-rank line: one record per rank, every rank counted once, the replicas'
    token counts add up to the whole-job value's tokens, and the process groups are the ones asked for."""
    assert d["ranks"] == n and len(d["per_rank"]) == n
    assert sorted(r["rank"] for r in d["per_rank"]) == list(range(n))
    replicas = [r for r in d["per_rank"] if r["role"] == "replica"]
    assert len(replicas) == n // tp and all(r["tok_s"] > 0 and r["ms_per_step"] > 0 for r in replicas)
    assert all(r["out_tokens"] == 0 for r in d["per_rank"] if r["role"] == "tp_follower")
    assert abs(sum(r["out_tokens"] for r in replicas) / (d["ms_per_step"] * d["steps"] / 1e3) - d["value"]) \
        <= 0.02 * d["value"] + 1
    assert d["dist"]["initialized"] and d["dist"]["world_size"] == n and d["dist"]["backend"] == "gloo"
    if tp > 1:
        assert d["dist"]["tp_group_size"] == tp
    else:
        assert "tp_group_size" not in d["dist"]
    # pre-flight fields a first 8-GPU run explains itself with: peer matrix, collective registration, RCCL version
    pre = d["preflight"]
    assert pre["world"] == n and pre["tp"] == tp and "rccl_version" in pre
    assert isinstance(pre["peer_access"], list) and pre["visible_devices"] == len(pre["peer_access"])
    assert pre["world_backend"] == "gloo"
    if tp > 1:
        assert pre["tp_group_size"] == tp and pre["custom_collectives"]["tp"].startswith("off")


@pytest.mark.timeout(900)
def test_bench_dp4_per_rank_records():
    """DP = 4 (the driver's N = 4 launch shape): four replica records, gloo world of 4."""
    d = _run([], n=4)
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp4"
    _check_ranks(d, 4, 1)


@pytest.mark.timeout(900)
def test_bench_tp2x2_per_rank_records():
    """TP = 2 x 2 replicas over 4 ranks: two replica leaders, two followers, TP groups of 2."""
    d = _run(["--tp", "2"], n=4)
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp2-tp2" and d["config"]["global_batch"] == 8
    _check_ranks(d, 4, 2)


@pytest.mark.timeout(600)
def test_bench_spawns_ranks_without_launcher():
    """``python bench.py --gpus 2`` with no torchrun: the parent starts the 2 ranks itself (no exec), relays rank 0's
    single JSON line, and the window contains new turns (staggered steady state) so TTFT is always sampled."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--model", "tiny-llama", "--prefix-tokens", "200", "--threads", "4", "--min-out", "4", "--max-out", "8",
           "--user-tokens", "8", "--ttft-samples", "4"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=500)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["ttft_samples"] >= 4 and d["ttft_p50_ms"] is not None


def test_bench_rejects_rank_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny-llama"],
                       cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def test_stationary_reply_budget():
    """Setup puts each slot at a random point of a length-biased reply: the remaining-token distribution has the
    stationary mean (E[n^2]/(2 E[n]) for uniform lengths in [lo, hi])."""
    import random
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    args = bench.parse(["--min-out", "128", "--max-out", "384"])
    th = bench.ThreadSim(0, [], random.Random(0), args, 128256)
    rem = []
    for _ in range(20000):
        n, done = th.reply_budget(stationary=True)
        assert 0 <= done < n
        rem.append(n - done)
    lo, hi = 128, 384
    ns = range(lo, hi + 1)
    expect = sum(n * n for n in ns) / sum(ns) / 2
    assert abs(sum(rem) / len(rem) - expect) < 0.03 * expect
