"""Probe: can two RCCL ranks share one GPU on this image? (one all_reduce of 1 MiB; prints the result or the error)."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
    x = torch.full((1 << 18,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank}: sum {x[0].item()} (expect 3.0)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        main()
        sys.exit(0)
    import subprocess

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29731", WORLD_SIZE="2")
    ps = [subprocess.Popen([sys.executable, __file__], env=dict(env, RANK=str(r))) for r in range(2)]
    rc = 0
    for p in ps:
        try:
            rc = rc or p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            rc = 124
    for p in ps:
        if p.poll() is None:
            p.kill()
    print("probe rc", rc)
