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


def _run(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
           "--warmup", "2", "--model", "tiny-llama", "--prefix-tokens", "200", "--threads", "4", "--min-out", "4",
           "--max-out", "8", "--reply-tokens", "16", "--user-tokens", "8", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="2")
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
