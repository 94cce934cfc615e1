"""Custom one-shot all-reduce for decode-sized tensor-parallel messages.

Llama-3-70B at TP=8 does 160 all-reduces of [B, 8192] bf16 (1 MiB at B = 64) per decode step. A ring all-reduce
(RCCL) is bound by one xGMI link per direction and pays 2(N-1) hop latencies; the MI355X mesh gives every GPU 7
point-to-point links, so the one-shot algorithm — every rank reads all 7 peers' copies concurrently and reduces
locally — moves the message in one hop at ~7 links' bandwidth (csrc/allreduce.hip).

Setup: each rank allocates one fine-grained uncached buffer (flags + 2 x max_bytes data halves), the IPC handles are
exchanged over the gloo control group, every rank maps every peer's buffer. Calls are stream-ordered and
hipGraph-capturable (buffers are registered up front; the epoch is a kernel argument). Messages above ``max_bytes``
(prefill chunks) go to RCCL. Enabled with ``KAFKA_CUSTOM_AR=1`` (``parallel/state.init``) — 2, 4 or 8 ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from kafka_llm_service_amd.ops._ext import ext


class CustomAllReduce:
    def __init__(self, cpu_group, rank: int, world: int, max_bytes: int = 8 << 20, nblocks: int = 64):
        if world not in (2, 4, 8):
            raise ValueError("custom all-reduce supports 2, 4 or 8 ranks")
        self.rank, self.world = rank, world
        self.max_bytes = max_bytes
        self.nblocks = nblocks
        self.epoch = 0
        e = ext()
        self.own = e.car_alloc(2 * max_bytes)
        handles = [None] * world
        dist.all_gather_object(handles, e.car_ipc_handle(self.own), group=cpu_group)
        self.bases = []
        self._opened = []
        for r, h in enumerate(handles):
            if r == rank:
                self.bases.append(self.own)
            else:
                p = e.car_open(h)
                self._opened.append(p)
                self.bases.append(p)
        dist.barrier(group=cpu_group)

    def should_use(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        self.epoch += 1
        ext().car_all_reduce(x, self.bases, self.rank, self.epoch, self.max_bytes, self.nblocks)
        return x

    def check(self) -> None:
        """Raise if any wait timed out (a peer never arrived). Synchronises; for tests and health checks."""
        if ext().car_error(self.own):
            raise RuntimeError("custom all-reduce: a peer did not arrive within 2 s")

    def close(self) -> None:
        e = ext()
        for p in self._opened:
            e.car_close(p)
        self._opened = []
        if self.own:
            e.car_free(self.own)
            self.own = 0
