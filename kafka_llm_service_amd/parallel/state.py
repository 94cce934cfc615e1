"""Process-group state: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl" on ROCm) / gloo on CPU.

Layout of a node of ``world`` ranks:
  * ``tp`` consecutive ranks form one tensor-parallel group (Megatron column/row split, 2 all-reduces per layer),
  * the remaining factor ``dp = world // tp`` are independent engine replicas (DP) — each replica owns its own KV
    cache and its own threads (thread-affinity routing: ``route`` / ``DPClient`` in ``engine/client.py``);
    replicas never communicate on the hot path.
  * ``ep`` (Mixtral) re-uses the TP group: experts are partitioned over its ranks; activations are already
    replicated after the attention all-reduce, so each rank gathers its experts' tokens locally and one all-reduce
    combines the partial outputs (``models/moe.py``; README "Expert parallelism").
  * every collective has a timeout (``KAFKA_COLLECTIVE_TIMEOUT_S``, default 300 s): a hung peer fails the replica's
    process instead of blocking it forever; the DP client then marks it down (HTTP 503 / error frames) and respawns.

The reference service has no collectives at all; this module is new.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from datetime import timedelta

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world: int = 1
    rank: int = 0
    local_rank: int = 0
    tp: int = 1
    tp_rank: int = 0
    dp: int = 1
    dp_rank: int = 0
    tp_group: object = None  # torch ProcessGroup over the tp ranks (None when tp == 1)
    cpu_group: object = None  # gloo group over the tp ranks for host-side broadcasts (scheduler decisions)
    backend: str = "none"
    # DP attention (init_dp_attention): ranks of one EP group run their own sequences, experts sharded over them
    ep: int = 1
    ep_rank: int = 0
    ep_group: object = None
    ep_cpu_group: object = None  # gloo: the per-step agreement on the all-to-all capacity
    # custom IPC collective per group: "registered", "off (...)" or "fallback: <reason>" (preflight())
    custom_status: dict = field(default_factory=dict)

    @property
    def is_tp_leader(self) -> bool:
        return self.tp_rank == 0


_STATE = ParallelState()


def get() -> ParallelState:
    return _STATE


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def init(tp: int = 1, backend: str | None = None, device: str | None = None) -> ParallelState:
    """Initialise torch.distributed from the torchrun env (no-op for a single process) and build the TP/DP groups."""
    global _STATE
    world, rank, local_rank = env_world()
    if world % tp != 0:
        raise ValueError(f"world size {world} not divisible by tp={tp}")
    st = ParallelState(world=world, rank=rank, local_rank=local_rank, tp=tp, tp_rank=rank % tp, dp=world // tp,
                       dp_rank=rank // tp)
    if world > 1:
        backend = backend or os.environ.get("KAFKA_TP_BACKEND") or None  # tests: "gloo" for ranks sharing one GPU
        if backend is None:
            backend = "nccl" if (device or "").startswith("cuda") or (device is None and torch.cuda.is_available()) \
                else "gloo"
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if backend == "nccl":
                torch.cuda.set_device(local_rank)
                kw["device_id"] = torch.device("cuda", local_rank)
            dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=_timeout(), **kw)
        st.backend = backend
        if tp > 1:
            for g in range(world // tp):
                ranks = list(range(g * tp, (g + 1) * tp))
                pg = dist.new_group(ranks, backend=backend, timeout=_timeout())
                cpg = dist.new_group(ranks, backend="gloo", timeout=_timeout()) if backend != "gloo" else pg
                if rank in ranks:
                    st.tp_group, st.cpu_group = pg, cpg
            on_gpu = (device or "").startswith("cuda") or (device is None and torch.cuda.is_available())
            if not on_gpu:
                st.custom_status["tp"] = "off (not a GPU group)"
            elif tp not in (2, 4, 8):
                st.custom_status["tp"] = f"off (tp={tp} unsupported)"
            elif os.environ.get("KAFKA_CUSTOM_AR", "1") != "1":
                st.custom_status["tp"] = "off (KAFKA_CUSTOM_AR=0)"
            else:
                _register_custom_ar(st, tp)
    _STATE = st
    return st


def init_dp_attention(ep: int, backend: str | None = None, device: str | None = None) -> ParallelState:
    """Data-parallel attention + expert parallelism (Mixtral): tp = 1, every ``ep`` consecutive ranks form an EP
    group — each runs its own sequences with whole attention weights and its own KV cache, and the group shares the
    experts through the device-side all-to-all of models/moe.py (the custom IPC transport registered on the group
    when it can be set up, RCCL / gloo otherwise)."""
    global _STATE
    st = init(tp=1, backend=backend, device=device)
    if ep <= 1:
        return st
    if st.world % ep:
        raise ValueError(f"world size {st.world} not divisible by ep={ep}")
    backend = st.backend
    st.ep, st.ep_rank = ep, st.rank % ep
    for g in range(st.world // ep):
        ranks = list(range(g * ep, (g + 1) * ep))
        pg = dist.new_group(ranks, backend=backend, timeout=_timeout())
        cpg = dist.new_group(ranks, backend="gloo", timeout=_timeout()) if backend != "gloo" else pg
        if st.rank in ranks:
            st.ep_group, st.ep_cpu_group = pg, cpg
    on_gpu = (device or "").startswith("cuda") or (device is None and torch.cuda.is_available())
    st.custom_status["ep"] = "off (not a GPU group)" if not on_gpu else f"off (ep={ep} unsupported)"
    if on_gpu and ep in (2, 4, 8) and os.environ.get("KAFKA_CUSTOM_AR", "1") == "1":
        import logging

        from . import comm
        from .custom_allreduce import CustomAllReduce, CustomAllReduceUnavailable

        try:
            comm.register_custom(st.ep_group, CustomAllReduce(st.ep_cpu_group, st.ep_rank, ep))
            st.custom_status["ep"] = "registered"
        except CustomAllReduceUnavailable as e:
            st.custom_status["ep"] = f"fallback: {e}"
            logging.getLogger("kafka.parallel").exception("IPC all-to-all unavailable; using the library collective")
    _STATE = st
    return st


def _register_custom_ar(st: ParallelState, tp: int) -> None:
    """The one-shot xGMI all-reduce for decode-sized messages (parallel/custom_allreduce.py); RCCL stays the path for
    everything else, and for all of it when the IPC mapping cannot be set up on some rank — a decision the group
    takes together (CustomAllReduce's setup is collective), so no rank runs RCCL while its peers run the custom
    kernel (logged, not fatal)."""
    import logging

    from . import comm
    from .custom_allreduce import CustomAllReduce, CustomAllReduceUnavailable

    try:
        comm.register_custom(st.tp_group, CustomAllReduce(st.cpu_group, st.tp_rank, tp))
        st.custom_status["tp"] = "registered"
    except CustomAllReduceUnavailable as e:
        st.custom_status["tp"] = f"fallback: {e}"
        logging.getLogger("kafka.parallel").exception("custom all-reduce unavailable; using RCCL for every message")
        if os.environ.get("KAFKA_REQUIRE_CUSTOM_AR", "0") == "1":
            raise


def preflight() -> dict:
    """What a first multi-GPU run needs to explain itself (bench.py puts it in its JSON line): the peer-access matrix
    of the visible devices (xGMI P2P, which the custom all-reduce's IPC buffers need), each group's custom-collective
    status (registered / off / fallback with the reason), the RCCL version and the group sizes."""
    st = _STATE
    out: dict = {"custom_collectives": dict(st.custom_status), "tp": st.tp, "ep": st.ep, "world": st.world}
    try:
        v = torch.cuda.nccl.version() if torch.cuda.is_available() else None
        out["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else v
    except Exception as e:  # noqa: BLE001 — informational
        out["rccl_version"] = f"unavailable: {type(e).__name__}"
    if torch.cuda.is_available():
        n = torch.cuda.device_count()
        out["visible_devices"] = n
        out["peer_access"] = [[1 if i == j else int(torch.cuda.can_device_access_peer(i, j)) for j in range(n)]
                              for i in range(n)]
    else:
        out["visible_devices"] = 0
        out["peer_access"] = []
    if dist.is_initialized():
        out["world_backend"] = dist.get_backend()
        for name in ("tp", "ep"):
            g = getattr(st, f"{name}_group", None)
            if g is not None:
                out[f"{name}_backend"] = dist.get_backend(g)
                out[f"{name}_group_size"] = dist.get_world_size(g)
    return out


def custom_ar():
    """The TP group's CustomAllReduce, or None (RCCL only / TP = 1)."""
    if _STATE.tp == 1:
        return None
    from . import comm

    return comm.get_custom(_STATE.tp_group)


def _timeout() -> timedelta:
    return timedelta(seconds=float(os.environ.get("KAFKA_COLLECTIVE_TIMEOUT_S", "300")))


def set_state(st: ParallelState) -> None:
    global _STATE
    _STATE = st


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    """Sum over the TP group (bf16; fp32 split-K slabs come back as a bf16 sum)."""
    st = _STATE
    if st.tp == 1:
        return x
    from . import comm

    return comm.all_reduce(x, st.tp_group)


def tp_all_reduce_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                              out: torch.Tensor) -> torch.Tensor:
    from . import comm

    return comm.all_reduce_add_rmsnorm(x, residual, w, eps, out, _STATE.tp_group)


def tp_linear_all_reduce(x: torch.Tensor, w: torch.Tensor, chunks: int) -> torch.Tensor:
    """allreduce(x @ w^T) over the TP group, GEMM blocks pipelined against the library all-reduce
    (comm.pipelined_linear_all_reduce)."""
    from . import comm

    return comm.pipelined_linear_all_reduce(x, w, _STATE.tp_group, chunks)


def tp_all_gather_lastdim(x: torch.Tensor) -> torch.Tensor:
    st = _STATE
    if st.tp == 1:
        return x
    from . import comm

    return comm.all_gather_lastdim(x, st.tp, st.tp_group)


def tp_broadcast_from_leader(x: torch.Tensor) -> torch.Tensor:
    """In place: every rank of the TP group gets the leader's ``x`` (device tensors over RCCL; over a gloo group —
    several ranks on one GPU in tests — through host memory)."""
    st = _STATE
    if st.tp == 1:
        return x
    src = st.rank - st.tp_rank
    if x.is_cuda and dist.get_backend(st.tp_group) == "gloo":
        h = x.cpu()
        dist.broadcast(h, src=src, group=st.tp_group)
        x.copy_(h)
        return x
    dist.broadcast(x, src=src, group=st.tp_group)
    return x


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
