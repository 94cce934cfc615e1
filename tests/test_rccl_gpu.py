"""RCCL on the MI355X: the hot-path collectives of parallel/comm.py over a real "nccl" (= RCCL) process group.

One GPU box can hold only a one-rank RCCL group (RCCL refuses two ranks on one device), so this checks what a single
rank can: the RCCL library initialises on gfx950 with ``device_id`` binding (as parallel/state.py does), and the
paths every TP/EP rank takes at scale run through it — the prefill-size all-reduce (> the custom all-reduce's
buffer, bf16 and fp32 split-K slab inputs), the vocab-parallel logit all-gather, the leader broadcast of
tp_broadcast_from_leader and the capacity-padded all_to_all_single of the EP fallback — with results equal to the
one-rank identities. Runs in a child process so the test process keeps no process group."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import torch, torch.distributed as dist
    from kafka_llm_service_amd.parallel import comm
    from kafka_llm_service_amd import ops
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    g = dist.group.WORLD
    assert dist.get_backend(g) == "nccl", dist.get_backend(g)
    torch.manual_seed(0)
    # prefill-size all-reduce: 512 x 8192 bf16 = 8 MiB (beyond any custom-AR buffer) through dist.all_reduce
    x = torch.randn(512, 8192, device=dev, dtype=torch.bfloat16)
    ref = x.clone()
    y = comm.all_reduce(x, g)
    torch.cuda.synchronize()
    assert torch.equal(y, ref), "bf16 all_reduce"
    # fp32 split-K slabs [S, T, n]: reduced to bf16 by the slab kernel, then RCCL
    s = torch.randn(4, 64, 4096, device=dev)
    y = comm.all_reduce(s, g)
    torch.cuda.synchronize()
    assert (y.float() - s.sum(0)).abs().max().item() < 0.05, "slab all_reduce"
    # vocab-parallel logits all-gather
    lg = torch.randn(64, 16032, device=dev)
    out = comm.all_gather_lastdim(lg, 1, g)
    assert torch.equal(out, lg), "all_gather_lastdim"
    # leader broadcast
    b = torch.arange(1000, device=dev, dtype=torch.int64)
    dist.broadcast(b, src=0, group=g)
    assert torch.equal(b, torch.arange(1000, device=dev)), "broadcast"
    # EP all_to_all_single fallback (capacity-padded rows)
    inp = torch.randn(256, 4096, device=dev, dtype=torch.bfloat16)
    o = torch.empty_like(inp)
    comm.all_to_all_single(o, inp, g)
    torch.cuda.synchronize()
    assert torch.equal(o, inp), "all_to_all_single"
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL OK", torch.cuda.get_device_name(0))
""")


def test_rccl_one_rank_collectives():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + os.getpid() % 1000), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "RCCL OK" in p.stdout
