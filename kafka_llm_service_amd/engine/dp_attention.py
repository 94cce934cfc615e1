"""Data-parallel attention + expert parallelism for Mixtral (BASELINE config 5's "expert all-to-all" layout).

Each rank of an EP group is a full serving engine for its own sequences — whole attention / norm / vocabulary
weights, its own KV cache, scheduler and request stream — and holds 1/ep of every layer's experts. A MoE layer sends
each of the rank's (token, expert) pairs to the rank that owns the expert and brings the results back
(models/moe.py ``_a2a`` with ``dp``: device-side dispatch / routing / combine kernels, the IPC all-to-all of
parallel/custom_allreduce.py or the library all-to-all). Versus the default tensor-parallel attention with an
all-reduce combine, every rank moves only its own tokens' rows and attention work and KV are split, not replicated.

Lockstep: every layer's all-to-all needs every rank, so the group runs one forward per step on every rank
(``LLMEngine.step_lockstep``): the ranks agree on (max tokens, any unfinished) with one host all-reduce per step —
the largest step sets the all-to-all capacity — and a rank without tokens runs an expert-only step that serves the
other ranks' rows. Scheduling is synchronous in this mode (one forward per ``step`` call keeps the collectives in
line), and decode steps are not graph-captured.

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


def make_agree(st):
    """(tokens, unfinished, flag) -> group maxima, over the EP group's gloo group (one 24-byte all-reduce per
    step)."""
    grp = st.ep_cpu_group

    def agree(vals: tuple[int, ...]) -> tuple[int, ...]:
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=grp)
        return tuple(int(v) for v in t)
    return agree


def generate_lockstep(eng, st, prompts: list[list[int]], params: SamplingParams) -> list[list[int]]:
    """Generate this rank's prompts (possibly none) in lockstep with the rest of its EP group: returns when every
    rank of the group has finished."""
    agree = make_agree(st)
    rids = [f"dpa{st.rank}-{i}" for i in range(len(prompts))]
    for rid, p in zip(rids, prompts):
        eng.add_request(rid, p, params)
    out: dict[str, list[int]] = {rid: [] for rid in rids}
    while True:
        outs, busy, _ = eng.step_lockstep(agree)
        for o in outs:
            out[o.request_id].extend(o.new_token_ids)
        if not busy:
            return [out[r] for r in rids]


def serve_pipe_lockstep(eng, st, conn) -> None:
    """The request loop of one DP-attention rank behind the API server's engine client: like engine/client.py
    serve_pipe (same message protocol), but the rank steps whenever ANY rank of its group has work, and idles in
    short polls so a new request on a peer starts its group step within ~2 ms."""
    from kafka_llm_service_amd.engine.client import HEARTBEAT_S

    agree = make_agree(st)
    pinned: list[int] | None = None
    last_hb = 0.0
    busy = 0
    while True:
        now = time.monotonic()
        if now - last_hb >= HEARTBEAT_S:
            conn.send(("hb", eng.stats["steps"]))
            last_hb = now
        stop = False
        while conn.poll(0 if busy else 0.002):
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
                                      "output_tokens": eng.stats["output_tokens"], "steps": eng.stats["steps"]}))
            elif kind == "stop":
                stop = True
                break
            busy = int(eng.has_unfinished())
        # every rank takes part in every agreement, busy or not; a stop seen by any rank stops the whole group
        # after the same step (nobody is left waiting in a collective for a peer that has exited)
        outs, busy, stopping = eng.step_lockstep(agree, flag=int(stop))
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
