"""Tensor-parallel engine groups: one process per GPU, a leader that schedules and followers that mirror its steps.

Design (SURVEY.md §2.4 "TP", §2.7 "broadcast scheduler decisions rank0 -> TP ranks"):
  * every rank of a TP group builds the same engine on its own GPU with its own weight shard (Megatron column/row
    split, ``models/weights.py``) and an identical KV page pool (the pool size is agreed by a MIN all-reduce, so page
    ids mean the same thing everywhere);
  * only the leader (tp_rank 0) runs the scheduler, the radix prefix cache and sampling. Each step it plans the batch
    on the host (``ModelRunner.build_host``: packed int64/int32 buffers + a few scalars, a few KB) and broadcasts that
    plan over the gloo group. Followers upload the same plan and run the same forward; the two all-reduces per layer
    (after O and down) and the vocab-parallel logit all-gather go over RCCL/xGMI on the device group;
  * a ``None`` plan tells followers to exit.
The host broadcast is the ONLY control traffic, so followers can never disagree with the leader about batch
composition, page ids or work items — correct by construction, and the data-plane collectives stay on the GPU.

``DPClient(engine_cfg, n_replicas, tp=k)`` (engine/client.py) spawns ``n_replicas`` such groups (dp x tp processes,
GPU ``dp_idx * tp + tp_rank``); each group gets its own rendezvous port, so replicas stay independent.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

from kafka_llm_service_amd.engine.model_runner import _PLAN_SCALARS, PLAN_HDR, pack_plan, unpack_plan
from kafka_llm_service_amd.parallel import state as pstate

log = logging.getLogger("kafka.tp")


def leader_src() -> int:
    """Global rank of this process's TP-group leader."""
    st = pstate.get()
    return st.rank - st.tp_rank


def attach_leader(engine) -> None:
    """Make ``engine`` (tp_rank 0) broadcast every launched step to its followers: a fixed int64 header and one
    uint8 payload (model_runner.pack_plan), two gloo tensor broadcasts — no pickling on the step path."""
    st = pstate.get()
    if st.tp == 1:
        return
    src, grp = leader_src(), st.cpu_group

    def bcast(host, sp):
        hdr, payload = pack_plan(host, sp)
        dist.broadcast(torch.from_numpy(hdr), src=src, group=grp)
        dist.broadcast(torch.from_numpy(payload), src=src, group=grp)

    engine.runner.broadcast = bcast


def release_followers() -> None:
    st = pstate.get()
    if st.tp > 1 and st.is_tp_leader:
        dist.broadcast(torch.zeros(PLAN_HDR, dtype=torch.int64), src=leader_src(), group=st.cpu_group)


@torch.inference_mode()
def follower_loop(engine) -> int:
    """Mirror the leader's steps until it sends the exit header. Returns the number of steps run. The follower only
    enqueues: its GPU runs each step when the collectives of that step meet the leader's (two steps can be in
    flight, as on the leader)."""
    st = pstate.get()
    src, grp = leader_src(), st.cpu_group
    runner = engine.runner
    n = 0
    hdr = torch.zeros(PLAN_HDR, dtype=torch.int64)
    while True:
        dist.broadcast(hdr, src=src, group=grp)
        if int(hdr[0]) == 0:
            return n
        payload = torch.empty(int(hdr[1 + len(_PLAN_SCALARS) + 5]), dtype=torch.uint8)
        dist.broadcast(payload, src=src, group=grp)
        host, sp = unpack_plan(hdr.numpy(), payload.numpy())
        runner.follower_launch(host, sp)
        n += 1


def build_tp_engine(cfg_dict: dict, tp: int):
    """Inside a process whose RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* env describe one TP group: init the groups and
    build this rank's engine shard."""
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine

    cfg = EngineConfig(**cfg_dict)
    dev = cfg.device
    if dev is None and torch.cuda.is_available():
        dev = f"cuda:{int(os.environ.get('LOCAL_RANK', '0')) % torch.cuda.device_count()}"
    st = pstate.init(tp=tp, device=dev or "cpu")
    cfg.device = dev or "cpu"
    cfg.tp, cfg.tp_rank = tp, st.tp_rank
    eng = LLMEngine(cfg)
    if st.is_tp_leader:
        attach_leader(eng)
    return eng, st


def tp_worker_main(dp_idx: int, tp_rank: int, tp: int, port: int, cfg_dict: dict, conn) -> None:
    """Process entry of one rank of one TP replica (spawned by DPClient). The leader serves the request pipe; the
    followers mirror steps."""
    from kafka_llm_service_amd.engine.client import serve_pipe

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(tp),
                       "RANK": str(tp_rank), "LOCAL_RANK": str(dp_idx * tp + tp_rank)})
    try:
        eng, st = build_tp_engine(cfg_dict, tp)
    except BaseException as e:  # noqa: BLE001 - reported to the parent
        conn.send(("fatal", repr(e)))
        return
    conn.send(("ready", {"device": str(eng.device), "kv_pages": eng.num_blocks, "tp_rank": st.tp_rank}))
    try:
        if st.is_tp_leader:
            serve_pipe(eng, conn)
            release_followers()
        else:
            follower_loop(eng)
    finally:
        pstate.destroy()
