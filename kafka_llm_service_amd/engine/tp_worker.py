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

Plan transport (``KAFKA_PLAN_CHANNEL``): ``shm`` (default) is the native shared-memory ring of
``runtime/csrc/plan_channel.cpp`` — the leader memcpys each plan into a slot and bumps a sequence word, followers
spin/yield on it and read the slot in place (zero copy), acking once the plan is uploaded; ``gloo`` is two tensor
broadcasts over the TCP control group. A plan larger than a slot is announced through the ring and sent over gloo.
``benchmarks/plan_bcast_bench.py`` measures both at 2..8 ranks (profiles/r03/plan_bcast_*).

``DPClient(engine_cfg, n_replicas, tp=k)`` (engine/client.py) spawns ``n_replicas`` such groups (dp x tp processes,
GPU ``dp_idx * tp + tp_rank``); each group gets its own rendezvous port, so replicas stay independent.
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch
import torch.distributed as dist

from kafka_llm_service_amd.engine.model_runner import PLAN_HDR, PLAN_PAYLOAD_IDX, pack_plan, unpack_plan
from kafka_llm_service_amd.parallel import state as pstate

log = logging.getLogger("kafka.tp")


def leader_src() -> int:
    """Global rank of this process's TP-group leader."""
    st = pstate.get()
    return st.rank - st.tp_rank


_HDR_BYTES = PLAN_PAYLOAD_IDX             # header slot holding the payload size
_GLOO_MARK = 2                           # hdr[0]: the payload of this plan follows over gloo (larger than a slot)


class PlanTransport:
    """Leader -> followers plan transport of one TP group (see the module docstring). ``send`` on the leader,
    ``recv`` + ``done`` on followers; ``close`` on both."""

    def __init__(self, kind: str | None = None, slot_bytes: int | None = None, nslots: int = 3):
        st = pstate.get()
        self.src, self.grp, self.leader = leader_src(), st.cpu_group, st.is_tp_leader
        self.timeout = float(os.environ.get("KAFKA_COLLECTIVE_TIMEOUT_S", "300"))
        kind = kind or os.environ.get("KAFKA_PLAN_CHANNEL", "shm")
        slot_bytes = slot_bytes or int(os.environ.get("KAFKA_PLAN_SLOT_BYTES", str(4 << 20)))
        self.ch = None
        if kind == "shm":
            self.ch = self._open_shm(st, slot_bytes, nslots)
        self.kind = "shm" if self.ch is not None else "gloo"

    def _open_shm(self, st, slot_bytes: int, nslots: int):
        """Collective: the leader creates the segment (if /dev/shm has room), every rank learns the name and
        attaches; any failure anywhere -> the whole group uses gloo."""
        import uuid

        from kafka_llm_service_amd.runtime import native

        name, ch = None, None
        if self.leader:
            try:
                free = os.statvfs("/dev/shm").f_bavail * os.statvfs("/dev/shm").f_frsize
                if free > 4 * nslots * slot_bytes:
                    name = f"/kafka_plan_{os.getpid()}_{uuid.uuid4().hex[:8]}"
                    ch = native().PlanChannel(name, nslots, slot_bytes, st.tp - 1)
            except Exception:  # noqa: BLE001 - fall back to gloo
                log.exception("shared-memory plan channel unavailable")
                name, ch = None, None
        box = [name]
        dist.broadcast_object_list(box, src=self.src, group=self.grp)
        name = box[0]
        ok = name is not None
        if ok and not self.leader:
            try:
                ch = native().PlanChannel(name, st.tp_rank - 1)
            except Exception:  # noqa: BLE001
                log.exception("could not attach the plan channel %s", name)
                ok, ch = False, None
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.grp)
        if int(flag.item()) == 0:
            if ch is not None:
                ch.close()
            return None
        if self.leader:
            # every follower has attached: drop the name now (the mappings stay valid), so a group killed with
            # SIGKILL by the stall monitor / respawn leaves nothing in /dev/shm
            ch.unlink()
        return ch

    # --- leader ---------------------------------------------------------------------------------------------------
    def send(self, hdr: np.ndarray, payload: np.ndarray) -> None:
        if self.ch is not None:
            if 16 + hdr.nbytes + payload.nbytes <= self.ch.slot_bytes:
                self.ch.publish(hdr, payload, self.timeout)
                return
            mark = hdr.copy()
            mark[0] = _GLOO_MARK
            self.ch.publish(mark, np.zeros(0, dtype=np.uint8), self.timeout)
        else:
            dist.broadcast(torch.from_numpy(hdr), src=self.src, group=self.grp)
            if int(hdr[0]) == 0:  # exit: no payload
                return
        dist.broadcast(torch.from_numpy(payload), src=self.src, group=self.grp)

    def release(self) -> None:
        self.send(np.zeros(PLAN_HDR, dtype=np.int64), np.zeros(0, dtype=np.uint8))

    # --- followers ------------------------------------------------------------------------------------------------
    def recv(self) -> tuple[np.ndarray, np.ndarray] | None:
        """The next plan (header, payload), or None at exit. Views into the ring stay valid until ``done()``."""
        if self.ch is not None:
            # no time limit while the leader process lives: an idle replica is not a dead one (the channel
            # raises at once when the leader's pid is gone; in-step waits stay bounded by self.timeout)
            hdr, payload = self.ch.recv(-1.0)
            if int(hdr[0]) == 0:
                self.ch.ack()
                return None
            if int(hdr[0]) != _GLOO_MARK:
                return hdr, payload
            hdr = hdr.copy()
            self.ch.ack()
        else:
            t = torch.zeros(PLAN_HDR, dtype=torch.int64)
            dist.broadcast(t, src=self.src, group=self.grp)
            hdr = t.numpy()
            if int(hdr[0]) == 0:
                return None
        p = torch.empty(int(hdr[_HDR_BYTES]), dtype=torch.uint8)
        dist.broadcast(p, src=self.src, group=self.grp)
        hdr = hdr.copy()
        hdr[0] = 1
        self._gloo_plan = True
        return hdr, p.numpy()

    def done(self) -> None:
        """The plan from the last ``recv`` has been consumed (uploaded): release its ring slot."""
        if getattr(self, "_gloo_plan", False):
            self._gloo_plan = False
            return
        if self.ch is not None:
            self.ch.ack()

    def close(self) -> None:
        if self.ch is not None:
            self.ch.close()
            self.ch = None


_TRANSPORT: PlanTransport | None = None


def transport() -> PlanTransport:
    """The process's plan transport (created collectively on first use; closed at exit so the leader's
    shared-memory segment never outlives the group)."""
    global _TRANSPORT
    if _TRANSPORT is None:
        import atexit

        _TRANSPORT = PlanTransport()
        atexit.register(close_transport)
    return _TRANSPORT


def attach_leader(engine) -> None:
    """Make ``engine`` (tp_rank 0) broadcast every launched step to its followers: a fixed int64 header and one
    uint8 payload (model_runner.pack_plan) through the group's PlanTransport — no pickling on the step path."""
    st = pstate.get()
    if st.tp == 1:
        return
    tr = transport()

    def bcast(host, sp):
        hdr, payload = pack_plan(host, sp)
        tr.send(hdr, payload)

    engine.runner.broadcast = bcast


def release_followers() -> None:
    st = pstate.get()
    if st.tp > 1 and st.is_tp_leader:
        transport().release()


@torch.inference_mode()
def follower_loop(engine) -> int:
    """Mirror the leader's steps until it sends the exit header. Returns the number of steps run. The follower only
    enqueues: its GPU runs each step when the collectives of that step meet the leader's (two steps can be in
    flight, as on the leader)."""
    runner = engine.runner
    tr = transport()
    n = 0
    while True:
        msg = tr.recv()
        if msg is None:
            return n
        host, sp = unpack_plan(*msg)
        runner.follower_launch(host, sp)
        tr.done()
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
    if tp > 1:
        transport()  # collective: every rank of the group sets up the plan transport together
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
        close_transport()
        pstate.destroy()


def close_transport() -> None:
    global _TRANSPORT
    if _TRANSPORT is not None:
        _TRANSPORT.close()
        _TRANSPORT = None
