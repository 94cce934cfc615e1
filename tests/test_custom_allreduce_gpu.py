"""Custom one-shot all-reduce (csrc/allreduce.hip) == RCCL all-reduce, on >= 2 GPUs of one node (skipped on a
single-GPU box: the one-shot kernel needs its peers on other devices)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _main(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(rank)})
    import torch.distributed as dist

    from kafka_llm_service_amd.parallel.custom_allreduce import CustomAllReduce

    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    cpu = dist.new_group(list(range(world)), backend="gloo")
    car = CustomAllReduce(cpu, rank, world, max_bytes=4 << 20)
    ok = True
    for n in (8, 4096 * 8, 64 * 8192, 1 << 20):
        for it in range(3):
            g = torch.Generator(device="cuda").manual_seed(1000 * n + 10 * it + rank)
            x = torch.randn(n, device="cuda", generator=g).to(torch.bfloat16)
            ref = x.float().clone()
            dist.all_reduce(ref)
            car.all_reduce(x)
            torch.cuda.synchronize()
            ok &= bool(((x.float() - ref).abs().max() <= 0.05 * ref.abs().max() + 1e-2).item())
    car.check()
    car.close()
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_custom_allreduce_matches_rccl():
    world = 2 if torch.cuda.device_count() < 4 else 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_main, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(res.values()) and len(res) == world
