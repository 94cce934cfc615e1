"""CPU placement for one-process-per-GPU runs (bench ranks, DP replicas, TP ranks on one host).

Eight engine processes each run a Python host loop (~4 ms of CPU per 8 ms decode step) plus torch's intra-op
OpenMP pool. Left alone, eight pools sized to the whole machine spin on the same cores as the host loops. Local
process r of n gets its own contiguous 1/n of the allowed CPUs (contiguous ranges keep GPU r's process on the
socket of its CPU half on the usual 2-socket, 8-GPU nodes) and an OpenMP pool no larger than that. Call before the
process touches the GPU or creates threads.
"""
from __future__ import annotations

import os


def pin_local_process(r: int, n: int) -> list[int] | None:
    """Restrict this process to slice r of n of its allowed CPUs; returns the CPUs, or None if not pinned."""
    if n <= 1:
        return None
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    k = len(cpus) // n
    if k < 2:
        return None
    mine = cpus[(r % n) * k:(r % n + 1) * k]
    os.sched_setaffinity(0, mine)
    cur = os.environ.get("OMP_NUM_THREADS", "")
    os.environ["OMP_NUM_THREADS"] = str(min(k, int(cur) if cur.isdigit() and int(cur) > 0 else 16))
    return mine
