#!/usr/bin/env python3
"""Per-step plan broadcast of a TP group (engine/tp_worker.py): gloo (two tensor broadcasts over TCP loopback) vs the
native shared-memory ring (runtime/csrc/plan_channel.cpp), at 2..8 ranks on the CPU (VERDICT r02 Weak #7).

Plan shapes are the ones the leader actually ships (model_runner.pack_plan): a Llama-3-70B TP=8 decode step of 64
threads on ~20k-token contexts — i64 = 4 x 64 + late rows, i32 = block tables [64, need] + q_limit + decode /
cascade items, sampling params — with the block tables compacted to the columns that hold pages ("compact", what is
shipped now) and at the full graph-bucket width ("wide", 2048 columns). Per (ranks, channel, shape): median and p99
of the time from the leader's send to the LAST follower holding the plan, over 300 steps (a gloo barrier-free
one-way measurement: each follower stamps its receive on a shared clock, CLOCK_MONOTONIC). One JSON line each."""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import time

import numpy as np
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _plan(cols: int, B: int = 64):
    i64 = np.arange(4 * B + 8, dtype=np.int64)
    i32 = np.arange(B * cols + B + 2 * 32 * 8 + 64 * 8, dtype=np.int32)
    samp = np.zeros(B * 4 * 6, dtype=np.uint8)
    payload = np.concatenate([i64.view(np.uint8), i32.view(np.uint8), samp])
    hdr = np.zeros(32, dtype=np.int64)
    hdr[0] = 1
    hdr[1 + 15 + 5] = payload.size
    return hdr, payload


def _main(rank, world, port, kind, cols, steps, q):
    import faulthandler

    faulthandler.dump_traceback_later(float(os.environ.get("PLAN_BENCH_HANG_S", "240")), exit=True)
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(rank), "KAFKA_PLAN_CHANNEL": kind})
    torch.set_num_threads(1)
    import torch.distributed as dist

    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.parallel import state as pstate

    pstate.init(tp=world, backend="gloo", device="cpu")
    tr = tp_worker.transport()
    hdr, payload = _plan(cols)
    stamps = []
    for i in range(steps + 20):
        dist.barrier(group=pstate.get().cpu_group)
        if rank == 0:
            t = time.monotonic_ns()
            hdr[2] = t  # the leader's send time rides in the header
            tr.send(hdr, payload)
        else:
            h, p = tr.recv()
            t_rx = time.monotonic_ns()
            assert p.size == payload.size
            if i >= 20:
                stamps.append(t_rx - int(h[2]))
            tr.done()
    if rank == 0:
        tr.release()
    else:
        assert tr.recv() is None
    q.put((rank, stamps, tr.kind))
    tp_worker.close_transport()
    pstate.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    lines = []
    for world in [int(x) for x in args.ranks.split(",")]:
        for kind in ("gloo", "shm"):
            for shape, cols in (("compact", 1270), ("wide", 2048)):
                ctx = mp.get_context("spawn")
                q = ctx.Queue()
                port = _port()
                ps = [ctx.Process(target=_main, args=(r, world, port, kind, cols, args.steps, q))
                      for r in range(world)]
                for p in ps:
                    p.start()
                res = [q.get(timeout=300) for _ in ps]
                for p in ps:
                    p.join(timeout=60)
                per_step = np.max(np.array([s for r, s, _ in res if r != 0]), axis=0) / 1e3  # last follower, us
                used = {k for _, _, k in res}
                d = {"ranks": world, "channel": kind, "used": sorted(used)[0], "plan": shape,
                     "plan_kb": round(_plan(cols)[1].nbytes / 1024, 1), "p50_us": round(float(np.median(per_step)), 1),
                     "p99_us": round(float(np.percentile(per_step, 99)), 1),
                     "mean_us": round(float(statistics.fmean(per_step)), 1)}
                print(json.dumps(d), flush=True)
                lines.append(d)
    if args.out:
        with open(args.out, "w") as f:
            f.write("\n".join(json.dumps(x) for x in lines) + "\n")


if __name__ == "__main__":
    main()
