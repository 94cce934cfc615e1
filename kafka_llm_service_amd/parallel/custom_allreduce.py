"""Custom one-shot all-reduce for decode-sized tensor-parallel messages.

Llama-3-70B at TP=8 does 160 all-reduces of [B, 8192] bf16 (1 MiB at B = 64) per decode step. A ring all-reduce
(RCCL) is bound by one xGMI link per direction and pays 2(N-1) hop latencies; the MI355X mesh gives every GPU 7
point-to-point links, so the one-shot algorithm — every rank reads all 7 peers' copies concurrently and reduces
locally — moves the message in one hop at ~7 links' bandwidth (csrc/allreduce.hip).

Setup: each rank allocates one fine-grained uncached buffer (flags + per-block epoch counters + 2 x max_bytes data
halves), the IPC handles are exchanged over the gloo control group, every rank maps every peer's buffer. Calls are
stream-ordered and hipGraph-capturable: the buffers are registered up front and the call counters live in device
memory (each block advances its own), so a replayed graph runs fresh epochs. Every call uses the same ``nblocks``.

``all_reduce_add_rmsnorm`` fuses the layer seam of a TP decoder: residual += allreduce(x); out = rmsnorm(residual)
(x may be the fp32 split-K slabs of the decode GEMM). Messages above ``max_bytes`` (prefill chunks) go to RCCL.
On by default for TP 2/4/8 on GPUs (``parallel/state.init``; ``KAFKA_CUSTOM_AR=0`` = RCCL for every message); the same
protocol runs between processes that share one GPU (tests/test_custom_allreduce_gpu.py on a 1-GPU box).

Failure handling:
  * setup is collective: every rank takes part in the same exchanges whether its own allocation / IPC mapping
    worked or not, and the group enables the custom path only if it worked on EVERY rank (one rank on RCCL while
    its peers run the custom kernel would hang or mix collectives);
  * a peer that stops arriving makes the kernel set its error word after 2 s (and skip waits from then on); the
    engine copies that word back with every step's sampled ids (``error_async``) and raises on collect, so the
    replica fails (503 + respawn) instead of returning tokens computed from stale peer data.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from kafka_llm_service_amd.ops._ext import ext


def _is_slab(x: torch.Tensor) -> bool:
    return x.dtype == torch.float32 and x.dim() == 3


class CustomAllReduceUnavailable(RuntimeError):
    """Raised on EVERY rank of the group when the custom path could not be set up on at least one of them."""


class CustomAllReduce:
    def __init__(self, cpu_group, rank: int, world: int, max_bytes: int = 8 << 20, nblocks: int = 64):
        if world not in (2, 4, 8):
            raise ValueError("custom all-reduce supports 2, 4 or 8 ranks")
        self.rank, self.world = rank, world
        self.max_bytes = max_bytes
        self.nblocks = nblocks
        e = ext()
        self.own, self._opened, self.bases = 0, [], []
        handle = None
        try:
            self.own = e.car_alloc(2 * max_bytes)
            handle = e.car_ipc_handle(self.own)
        except Exception:  # noqa: BLE001 - reported collectively below
            handle = None
        handles = [None] * world
        dist.all_gather_object(handles, handle, group=cpu_group)  # every rank, failed or not
        ok = all(h is not None for h in handles)
        if ok:
            try:
                for r, h in enumerate(handles):
                    if r == rank:
                        self.bases.append(self.own)
                    else:
                        p = e.car_open(h)
                        self._opened.append(p)
                        self.bases.append(p)
            except Exception:  # noqa: BLE001
                ok = False
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=cpu_group)  # the group's decision, the same everywhere
        if int(flag.item()) == 0:
            self.close()
            raise CustomAllReduceUnavailable(f"custom all-reduce setup failed on some rank (this rank ok={ok})")
        from kafka_llm_service_amd.utils import faults

        self._fi_skip, self._fi_calls = faults.get().car_skip_call, 0

    def _fits(self, x: torch.Tensor) -> bool:
        n = x.shape[1] * x.shape[2] if _is_slab(x) else x.numel()
        return x.is_cuda and x.is_contiguous() and n % 8 == 0 and n * 2 <= self.max_bytes

    def should_use(self, x: torch.Tensor) -> bool:
        return (x.dtype == torch.bfloat16 or _is_slab(x)) and self._fits(x)

    def _skip(self) -> bool:
        """Fault injection (KAFKA_FI_CAR_SKIP_CALL): this rank does not take part in its n-th call."""
        n = self._fi_skip
        if not n:
            return False
        self._fi_calls += 1
        return self._fi_calls == n

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum over the group of x (bf16, in place unless ``out``) or of a split-K slab (into a new bf16 tensor)."""
        if _is_slab(x) and out is None:
            out = torch.empty(x.shape[1], x.shape[2], dtype=torch.bfloat16, device=x.device)
        if not self._skip():
            ext().car_all_reduce(x, out, self.bases, self.rank, self.max_bytes, self.nblocks)
        return x if out is None else out

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                               out: torch.Tensor, pre: torch.Tensor | None = None) -> torch.Tensor:
        """residual += allreduce(x); out = rmsnorm(residual) * w — one launch. ``pre``: the row's first columns,
        already all-reduced (bf16 [T, dpre]); x then holds only the remaining columns (overlapped TP seam)."""
        if not self._skip():
            ext().car_all_reduce_add_rmsnorm(x, residual, w, float(eps), out, self.bases, self.rank, self.max_bytes,
                                             self.nblocks, pre)
        return out

    def fits_bytes(self, nbytes: int) -> bool:
        return nbytes % 16 == 0 and nbytes <= self.max_bytes

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        """recv[p] = peer p's send[self.rank] for send/recv [world, ...] (contiguous, equal parts): the expert
        dispatch / return of the MoE layers over the same IPC buffers and epochs (csrc/allreduce.hip a2a_pull_kernel;
        no host sync, graph-capturable)."""
        bpd = send.numel() * send.element_size() // self.world
        if not self._skip():
            ext().car_a2a(send, recv, int(bpd), False, self.bases, self.rank, self.max_bytes, self.nblocks)
        return recv

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        """recv[p] = peer p's send (recv = world parts of send's size)."""
        if not self._skip():
            ext().car_a2a(send, recv, int(send.numel() * send.element_size()), True, self.bases, self.rank,
                          self.max_bytes, self.nblocks)
        return recv

    def check(self) -> None:
        """Raise if any wait timed out (a peer never arrived). Synchronises; for tests and health checks."""
        if ext().car_error(self.own):
            raise RuntimeError("custom all-reduce: a peer did not arrive within 2 s")

    def timing(self) -> tuple:
        """(call durations in us of the last <= 128 calls, oldest first, this rank's call count): block 0's entry /
        exit stamps of the 100 MHz constant clock (csrc/allreduce.hip AR_TIME_OFF). Synchronises with a private
        stream only: for /metrics, never the step path."""
        import numpy as np

        ring, epoch = ext().car_timing(self.own)
        r = ring.numpy().view(np.uint64)
        n = min(int(epoch), r.shape[0])
        slots = [(int(epoch) - k) & (r.shape[0] - 1) for k in range(n - 1, -1, -1)]
        st, en = r[slots, 0].astype(np.int64), r[slots, 1].astype(np.int64)
        ok = (en >= st) & (st > 0)
        return (en[ok] - st[ok]) / 100.0, int(epoch)

    def error_async(self, out: torch.Tensor, idx: int) -> None:
        """Stream-ordered copy of the error word into ``out[idx]`` (pinned int32): read it once the stream passed."""
        ext().car_error_async(self.own, out, int(idx))

    def close(self) -> None:
        if not self.own and not self._opened:
            return
        e = ext()
        for p in self._opened:
            e.car_close(p)
        self._opened = []
        if self.own:
            e.car_free(self.own)
            self.own = 0
