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


def all_reduce(x: torch.Tensor, group) -> torch.Tensor:
    impl = _CUSTOM.get(group)
    if impl is not None and impl.should_use(x):
        return impl.all_reduce(x)
    dist.all_reduce(x, group=group)
    return x


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits: list[int], in_splits: list[int],
                      group) -> torch.Tensor:
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out
