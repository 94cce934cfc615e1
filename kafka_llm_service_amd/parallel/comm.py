"""Collectives used on the hot path.

``all_reduce`` picks, per call, between
  * the custom one-shot xGMI all-reduce (``parallel/custom_allreduce.py``; every GPU reads its 7 peers' buffers over
    its 7 point-to-point links at once and reduces locally — one hop instead of a ring's 2(N-1)) for decode-sized
    messages, when it has been registered for the group, and
  * RCCL (``torch.distributed.all_reduce`` on the "nccl" backend) for everything else (prefill chunks).

SURVEY.md §2.7 / §5.8 give the message sizes: [B, d] bf16 = B x 16 KiB for 70B at TP=8.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_CUSTOM = {}  # group -> CustomAllReduce


def register_custom(group, impl) -> None:
    _CUSTOM[group] = impl


def get_custom(group):
    return _CUSTOM.get(group)


def _host_all_reduce(x: torch.Tensor, group) -> torch.Tensor:
    """A device tensor over a gloo group (tests that put several ranks on one GPU, where RCCL refuses to run): the
    sum goes through host memory."""
    h = x.cpu()
    dist.all_reduce(h, group=group)
    x.copy_(h)
    return x


def _is_gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def all_reduce(x: torch.Tensor, group) -> torch.Tensor:
    """Sum of ``x`` over ``group``: bf16 in place, or — for fp32 split-K slabs [S, T, n] — into a new bf16 [T, n]."""
    impl = _CUSTOM.get(group)
    if impl is not None and impl.should_use(x):
        return impl.all_reduce(x)
    from kafka_llm_service_amd import ops

    x = ops.slab_reduce(x)
    if x.is_cuda and _is_gloo(group):
        return _host_all_reduce(x, group)
    dist.all_reduce(x, group=group)
    return x


def all_reduce_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor,
                           group) -> torch.Tensor:
    """The TP layer seam: residual += allreduce(x); out = rmsnorm(residual) * w. One custom-all-reduce launch when
    the message fits its buffer (the reduce, the residual add and the next RMSNorm fused), else RCCL + the fused
    add+RMSNorm kernel."""
    impl = _CUSTOM.get(group)
    if impl is not None and impl.should_use(x) and residual.is_contiguous():
        return impl.all_reduce_add_rmsnorm(x, residual, w, eps, out)
    from kafka_llm_service_amd import ops

    return ops.fused_add_rmsnorm(all_reduce(x, group), residual, w, eps, out=out)


def pipelined_linear_all_reduce(x: torch.Tensor, w: torch.Tensor, group, chunks: int) -> torch.Tensor:
    """sum over ``group`` of x @ w^T for a prefill-sized row-parallel seam, with the GEMM and the library all-reduce
    pipelined over ``chunks`` row blocks: block i's all-reduce is issued asynchronously (RCCL runs it on its own HIP
    stream, ordered after the block's GEMM) while block i+1's GEMM runs on the compute stream; the compute stream
    waits for every block only at the end. The weight is re-read per block (a prefill GEMM is compute-bound) and the
    per-element sums are the library all-reduce's, so the result equals the unchunked seam's."""
    T = x.shape[0]
    y = torch.empty(T, w.shape[0], dtype=x.dtype, device=x.device)
    bounds = [T * i // chunks for i in range(chunks + 1)]
    works = []
    host = x.is_cuda and _is_gloo(group)  # several ranks on one GPU (tests): through host memory, serially
    for a, b in zip(bounds[:-1], bounds[1:]):
        if b <= a:
            continue
        torch.matmul(x[a:b], w.t(), out=y[a:b])
        if host:
            _host_all_reduce(y[a:b], group)
        else:
            works.append(dist.all_reduce(y[a:b], group=group, async_op=True))
    for wk in works:
        wk.wait()
    return y


def all_gather_lastdim(x: torch.Tensor, world: int, group) -> torch.Tensor:
    x = x.contiguous()
    if x.is_cuda and _is_gloo(group):
        parts = [torch.empty_like(x, device="cpu") for _ in range(world)]
        dist.all_gather(parts, x.cpu(), group=group)
        return torch.cat(parts, dim=-1).to(x.device)
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x, group=group)
    return torch.cat(parts, dim=-1)


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, group, out_splits: list[int] | None = None,
                      in_splits: list[int] | None = None) -> torch.Tensor:
    """dist.all_to_all_single; device tensors over a gloo group (several ranks on one GPU) go through host memory."""
    if inp.is_cuda and _is_gloo(group):
        h = torch.empty_like(out, device="cpu")
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)
        return out
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, world: int, group) -> torch.Tensor:
    """out [world * n, ...] = concat over ranks of inp [n, ...] (host-staged over gloo)."""
    if inp.is_cuda and _is_gloo(group):
        parts = [torch.empty_like(inp, device="cpu") for _ in range(world)]
        dist.all_gather(parts, inp.contiguous().cpu(), group=group)
        out.copy_(torch.cat(parts, 0))
        return out
    dist.all_gather_into_tensor(out, inp.contiguous(), group=group)
    return out
