"""Data-parallel attention + expert parallelism for Mixtral (BASELINE config 5's "expert all-to-all" layout).

Each rank of an EP group is a full serving engine for its own sequences — whole attention / norm / vocabulary
weights, its own KV cache, scheduler and request stream — and holds 1/ep of every layer's experts. A MoE layer sends
each of the rank's (token, expert) pairs to the rank that owns the expert and brings the results back
(models/moe.py ``_a2a`` with ``dp``: device-side dispatch / routing / combine kernels, the IPC all-to-all of
parallel/custom_allreduce.py or the library all-to-all). Versus the default tensor-parallel attention with an
all-reduce combine, every rank moves only its own tokens' rows and attention work and KV are split, not replicated.

Lockstep: every layer's all-to-all needs every rank, so the group runs one forward per step on every rank
(``LLMEngine.step_lockstep``): the ranks agree on (max tokens, any unfinished, stop flag) once per step — the
largest step sets the all-to-all capacity — and a rank without tokens runs an expert-only step that serves the
other ranks' rows. The agreement goes through a shared-memory board (``runtime/csrc/group_board.cpp``: a few cache
lines, microseconds; gloo all-reduce only if the board cannot be set up), and the engine plans ahead as in
``LLMEngine.step``: step n+1 is planned, agreed and launched while step n still runs (one forward per call keeps the
collectives in line; the host never waits on the GPU between steps). An idle group does not poll collectives: each
rank sleeps on its request pipe and the board's wake counter, and the rank that receives a request wakes the others.

Entry points: ``build_dpa_engine`` (inside a process of a torch.distributed world whose ranks form the EP groups),
``generate_lockstep`` (offline / bench), ``serve_pipe_lockstep`` (a replica of the API server's engine client).
"""
from __future__ import annotations

import logging
import time

import torch
import torch.distributed as dist

from kafka_llm_service_amd.engine.sequence import SamplingParams

log = logging.getLogger("kafka.dp_attention")


def build_dpa_engine(cfg_dict: dict, ep: int):
    """(engine, parallel state) of this rank: DP attention over groups of ``ep`` consecutive ranks."""
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.parallel import state as pstate

    st = pstate.init_dp_attention(ep, device=cfg_dict.get("device"))
    cfg = EngineConfig(**dict(cfg_dict, tp=1, tp_rank=0, dp_attention=True))
    return LLMEngine(cfg), st


_BOARDS: dict = {}


def make_board(st):
    """The EP group's shared-memory agreement board (collective over the group's gloo group: the group's first rank
    creates the segment, every rank attaches, the name is unlinked once all have); None -> gloo agreement."""
    key = (st.rank, st.ep)
    if key in _BOARDS:
        return _BOARDS[key]
    import os
    import uuid

    from kafka_llm_service_amd.runtime import native

    grp = st.ep_cpu_group
    src = st.rank - st.ep_rank
    name, board = None, None
    if st.ep_rank == 0 and os.environ.get("KAFKA_DPA_BOARD", "1") == "1":
        try:
            name = f"/kafka_board_{os.getpid()}_{uuid.uuid4().hex[:8]}"
            board = native().GroupBoard(name, st.ep, 0, True)
        except Exception:  # noqa: BLE001 - gloo fallback
            log.exception("shared-memory agreement board unavailable")
            name, board = None, None
    box = [name]
    dist.broadcast_object_list(box, src=src, group=grp)
    ok = box[0] is not None
    if ok and st.ep_rank != 0:
        try:
            board = native().GroupBoard(box[0], st.ep, st.ep_rank, False)
        except Exception:  # noqa: BLE001
            log.exception("could not attach the agreement board %s", box[0])
            ok, board = False, None
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=grp)
    if int(flag.item()) == 0:
        if board is not None:
            board.close()
        board = None
    elif st.ep_rank == 0:
        board.unlink()  # every rank has attached: nothing outlives a killed group in /dev/shm
    _BOARDS[key] = board
    return board


class Agree:
    """(tokens, unfinished, flag[, ...]) -> group maxima: the shared-memory board's exchange, or one gloo all-reduce
    of the EP group. ``board`` is exposed for the idle wait (wake counter)."""

    def __init__(self, st, timeout_s: float | None = None):
        import os

        self.grp = st.ep_cpu_group
        self.board = make_board(st)
        self.timeout = float(os.environ.get("KAFKA_COLLECTIVE_TIMEOUT_S", "300")) if timeout_s is None else timeout_s

    def __call__(self, vals: tuple[int, ...]) -> tuple[int, ...]:
        if self.board is not None:
            import numpy as np

            return tuple(int(v) for v in self.board.exchange(np.asarray(vals, dtype=np.int64), self.timeout))
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.grp)
        return tuple(int(v) for v in t)


def make_agree(st) -> Agree:
    return Agree(st)


def generate_lockstep(eng, st, prompts: list[list[int]], params: SamplingParams) -> list[list[int]]:
    """Generate this rank's prompts (possibly none) in lockstep with the rest of its EP group: returns when every
    rank of the group has finished."""
    agree = make_agree(st)
    rids = [f"dpa{st.rank}-{i}" for i in range(len(prompts))]
    for rid, p in zip(rids, prompts):
        eng.add_request(rid, p, params)
    out: dict[str, list[int]] = {rid: [] for rid in rids}
    while True:
        outs, busy, _, _ = eng.step_lockstep(agree)
        for o in outs:
            out[o.request_id].extend(o.new_token_ids)
        if not busy:
            return [out[r] for r in rids]


def _idle_wait(conn, board, wake_seen: int, idle_since: float, hb_left: float) -> str | None:
    """An idle group. With the board: sleep until a message arrives on this rank's pipe ("msg") or a peer bumps the
    wake counter past ``wake_seen`` — the group's agreed reading before it went idle — ("wake": that peer is entering
    a group step, join it), or the heartbeat is due (None: do NOT step, the peers are asleep). No collective is
    polled. Without a board: one pipe poll backing off from 2 to 50 ms, then "msg" (every wake-up is one gloo
    agreement of the group, which the ranks reach on their own backoffs)."""
    idle = time.monotonic() - idle_since
    if board is None:
        conn.poll(min(0.05, 0.002 * (1 + int(idle * 10))))
        return "msg"
    t_end = time.monotonic() + hb_left
    while True:
        if board.wake_count() > wake_seen:
            return "wake"
        if conn.poll(0.0005 if idle < 1.0 else 0.002):
            return "msg"
        if time.monotonic() >= t_end:
            return None
        idle = time.monotonic() - idle_since


def serve_pipe_lockstep(eng, st, conn) -> None:
    """The request loop of one DP-attention rank behind the API server's engine client: like engine/client.py
    serve_pipe (same message protocol), but the rank steps whenever ANY rank of its group has work. While the whole
    group is idle the ranks sleep on their pipes (``_idle_wait``, ADVICE r03: no collective polling of an idle
    group). Protocol (shared-memory board): an idle rank enters a group step only if it has work of its own or a
    stop (then it first bumps the board's wake counter) or a peer woke it; a message that brings no work (health,
    pin, abort) is answered without stepping. Every bump is made by a rank that is about to step, so a woken rank
    always finds its peer in the agreement; the wake reading is part of each agreement, so a bump is never missed
    or double-counted across idle periods."""
    from kafka_llm_service_amd.engine.client import HEARTBEAT_S

    agree = make_agree(st)
    board = agree.board
    pinned: list[int] | None = None
    last_hb = 0.0
    busy = 0  # the group's busy flag, as last agreed
    wake_seen = 0
    idle_since = time.monotonic()
    while True:
        now = time.monotonic()
        if now - last_hb >= HEARTBEAT_S:
            conn.send(("hb", eng.stats["steps"]))
            last_hb = now
        woke = False
        if not busy:
            r = _idle_wait(conn, board, wake_seen, idle_since, max(0.0, HEARTBEAT_S - (now - last_hb)))
            if r is None:
                continue  # heartbeat only
            woke = r == "wake"
        stop = False
        while conn.poll(0):
            msg = conn.recv()
            kind = msg[0]
            if kind == "add":
                _, rid, prompt, pdict, *_ = msg
                try:
                    if isinstance(prompt, tuple):
                        if pinned is None or len(pinned) < prompt[1]:
                            raise ValueError("prompt references a shared prefix this replica was not sent")
                        prompt = pinned[:prompt[1]] + prompt[2]
                    eng.add_request(rid, prompt, SamplingParams(**pdict))
                except Exception as e:  # noqa: BLE001 - reported to the client as an error frame
                    conn.send(("error", rid, str(e)))
            elif kind == "abort":
                eng.abort(msg[1])
            elif kind == "pin":
                pinned = list(msg[1])
                eng.pin_prefix(pinned)
            elif kind == "health":
                kv = eng.kv_stats()
                conn.send(("health", {"running": eng.num_running, "waiting": eng.num_waiting,
                                      "kv_free_pages": kv["free"] + kv["evictable"],
                                      "kv_total_pages": kv["num_blocks"], "prefix_hit_tokens": kv["hit_tokens"],
                                      "output_tokens": eng.stats["output_tokens"], "steps": eng.stats["steps"],
                                      "perf": eng.perf_stats()}))
            elif kind == "stop":
                stop = True
                break
        mine = eng.has_unfinished()
        if board is not None and not busy:
            if not (mine or stop or woke):
                continue  # nothing for the group (health / pin / abort): the peers stay asleep
            if mine or stop:
                board.wake()  # peers asleep in _idle_wait join this group step
        # every rank takes part in every agreement, busy or not; a stop seen by any rank stops the whole group
        # after the same step (nobody is left waiting in a collective for a peer that has exited)
        wake_read = board.wake_count() if board is not None else 0
        outs, busy, stopping, ext = eng.step_lockstep(agree, flag=int(stop), extra=(wake_read,))
        wake_seen = ext[0]
        if not busy:
            idle_since = time.monotonic() if idle_since is None else idle_since
        else:
            idle_since = None
        if outs:
            conn.send(("out", [(o.request_id, o.new_token_ids, o.finished, o.finish_reason, o.num_prompt_tokens,
                                o.num_output_tokens, o.num_cached_tokens) for o in outs], time.perf_counter()))
        if stopping:
            conn.send(("stopped",))
            return


def dpa_worker_main(rank: int, ep: int, port: int, cfg_dict: dict, conn) -> None:
    """Process entry of one DP-attention rank (engine/client.py DPClient with ``dp_attention``)."""
    import os

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(ep),
                       "RANK": str(rank), "LOCAL_RANK": str(rank)})
    from kafka_llm_service_amd.parallel import state as pstate

    try:
        dev = cfg_dict.get("device")
        if dev is None and torch.cuda.is_available():
            dev = f"cuda:{rank % torch.cuda.device_count()}"
        eng, st = build_dpa_engine(dict(cfg_dict, device=dev), ep)
    except BaseException as e:  # noqa: BLE001
        conn.send(("fatal", repr(e)))
        return
    conn.send(("ready", {"device": str(eng.device), "kv_pages": eng.num_blocks, "ep_rank": st.ep_rank}))
    try:
        serve_pipe_lockstep(eng, st, conn)
    finally:
        pstate.destroy()
