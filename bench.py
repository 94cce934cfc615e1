#!/usr/bin/env python3
"""Headline benchmark: output tok/s + p50 TTFT, Llama-3-8B, 64 concurrent multi-turn threads per MI355X.

BASELINE.json metric: "output tok/s + p50 TTFT, Llama-3-8B, 64 concurrent threads, 1/2/4/8 MI355X"
(configs 2-3: Llama-3 8B bf16 TP=1, 64 concurrent threads with 4-turn history, per-thread prefix-KV reuse).

Launch: ``python bench.py --gpus N`` runs N ranks. Under ``torch.distributed.run`` (the driver's N > 1 launch) every
process is one rank; without a launcher and N > 1 this process becomes a parent that never touches the GPU and
starts N child ranks itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env), relays rank 0's JSON line and
exits with the worst child exit code. ``--gpus`` must equal the number of ranks (checked).

Workload (synthetic data, random-init Llama-3-8B weights — no checkpoints/datasets are reachable offline):
  * every thread's prompt = the shared Kafka system prefix (default 18,000 tokens: the reference's ~70k-char system
    prompt + ~6.6k chars of tool schemas) + its own history + a new user message (32-96 tokens);
  * a thread slot runs conversations of 2H+1 turns (H = --history-turns = 4), so the history in front of a new
    turn holds 0..2H earlier turns — 4 on average, ~1.3k tokens — and each reply streams
    max_tokens in [128, 384] (ignore_eos, T = 0.7). When a conversation ends the slot starts a new one (a new
    thread: only the shared prefix is cached);
  * STEADY STATE FROM THE FIRST STEP: at setup every slot is put at a random point of its life — a random turn of
    its conversation and, inside the in-flight reply, a random number of already-generated tokens (reply length
    drawn length-biased, position uniform: the stationary distribution of this renewal process). Completions and
    new-turn admissions (prefix-cache hits on the shared prefix and on the thread's own history, then a short
    prefill) therefore happen at the steady rate in every window; a 20-step window measures the same thing a
    300-step one does;
  * ``--mixed-prefix F``: a fraction F of the slots use a different system prompt (threads created with their own
    system message, quirk Q4 of SURVEY.md §2.9) — the multi-group cascade case;
  * ``--tool-frac F``: a fraction F of the slots decode under ``tool_choice="required"`` for their whole reply —
    back-to-back grammar-constrained tool calls over the server's tool schemas (ToolCallLoop), so every one of their
    tokens goes through the sampler's device-side grammar masks / forced tokens (engine/logits_proc.py) — and
    ``--penalty-frac F`` slots carry presence / frequency penalties (device-side counts). Off in the headline;
    the A/B that shows those threads no longer stall the batch (VERDICT r03 "Next round" #3);
  * DP: one engine replica per GPU (one process per GPU), 64 threads per replica (weak scaling).

A "step" is one engine iteration (one continuous-batching forward over the mixed decode/prefill batch, sampling
included). W untimed warmup steps, then exactly K timed steps between barrier + synchronize; value = total output
tokens of all ranks / max rank time.

TTFT (first token of a new turn, engine-level: request arrival -> sampled token on the host; the first content
frame of /root/reference/server.py:338-356) is sampled from every new turn that ARRIVES at or after the start of
the timed window; completions are ~threads/mean(reply) per step (~0.25 at 64 threads), so after the K timed steps
the engine keeps stepping under the same load (untimed, not counted in ``value``) until ``--ttft-samples`` turns
have their first token (``ttft_extra_steps`` reports how many steps that took).

vs_baseline: the reference publishes no number for this metric; the ratio is to the derived
MI355X bound for exactly this workload (~17k tok/s on one GPU with cascade attention, BASELINE.md §3 /
SURVEY.md §6.4), per GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import socket
import subprocess
import sys
import time

METRIC = "output tok/s + p50 TTFT, Llama-3-8B, 64 concurrent threads, 1/2/4/8 MI355X"  # BASELINE.json
BOUND_TOKS_PER_GPU = 17000.0  # derived 1-GPU bound with cascade attention on the ~18k prefix


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="number of ranks (one per GPU)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel size per replica (e.g. 8 for llama3-70b)")
    ap.add_argument("--dp-attention", action="store_true",
                    help="MoE models: all ranks form one data-parallel-attention EP group (engine/dp_attention.py)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--threads", type=int, default=64, help="concurrent threads per replica")
    ap.add_argument("--prefix-tokens", type=int, default=18000, help="shared system prefix (0 = short prompt)")
    ap.add_argument("--mixed-prefix", type=float, default=0.0,
                    help="fraction of threads on a second system prompt (multi-group cascade)")
    ap.add_argument("--tool-frac", type=float, default=0.0,
                    help="fraction of threads decoding back-to-back grammar-constrained tool calls")
    ap.add_argument("--penalty-frac", type=float, default=0.0,
                    help="fraction of threads with presence / frequency penalties")
    ap.add_argument("--history-turns", type=int, default=4, help="mean earlier turns in front of a new turn")
    ap.add_argument("--user-tokens", type=int, default=64, help="mean user-message tokens")
    ap.add_argument("--min-out", type=int, default=128)
    ap.add_argument("--max-out", type=int, default=384)
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--ttft-samples", type=int, default=64, help="new turns whose TTFT is sampled")
    ap.add_argument("--ttft-max-steps", type=int, default=4000)
    ap.add_argument("--no-cascade", action="store_true")
    ap.add_argument("--graphs", action="store_true", default=None,
                    help="hipGraph decode steps (default: on for --tp > 1, off at TP = 1)")
    ap.add_argument("--no-graphs", dest="graphs", action="store_false")
    ap.add_argument("--kv-run-pages", type=int, default=1,
                    help="KV pages handed out per growth step in consecutive runs (EngineConfig.kv_run_pages)")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"],
                    help="paged KV cache precision (fp8 = e4m3 + per-token scales; an opt-in A/B, not the headline)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------------------------
# parent: N child ranks without a launcher (never initialises the GPU itself)
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        out = None if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=out))
    rc = 0
    try:
        for p in procs:
            c = p.wait()
            rc = rc or c
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


# ---------------------------------------------------------------------------------------------------------------
def bench_tools() -> list[dict]:
    """The server's tool schemas (weather, counter, planner, shell, notebook; server/state.py)."""
    from kafka_llm_service_amd.server_tools import NotebookTools, PlannerTools, ShellTools, count_tool, get_weather_tool

    tools = [get_weather_tool, count_tool] + PlannerTools(None).tools + ShellTools(None).tools + \
        NotebookTools(None).tools
    return [t.definition for t in tools]


class ToolCallLoop:
    """allowed_tokens_fn of a ``--tool-frac`` thread: one ``tool_choice="required"`` tool call after another for the
    whole reply (the same grammar the agent loop decodes tool calls with, engine/constrained.py), so the thread is
    constrained at every token and keeps its reply length (no stop token)."""

    def __init__(self, tok, tools):
        from kafka_llm_service_amd.engine.constrained import ToolCallConstraint

        self._mk = lambda: ToolCallConstraint(tok, tools, "required")
        self.c = self._mk()
        self.base = 0  # output index where the current call starts

    def _cur(self, out):
        if self.c.done:
            self.base += self.c._n
            self.c = self._mk()
        return out[self.base:]

    def __call__(self, out):
        spec = self.c(self._cur(out))
        if spec is None and self.c.done:  # the call just ended: the next token opens the next call
            spec = self.c(self._cur(out))
        return spec

    def plan_state(self, out):
        return self.c.plan_state(self._cur(out))

    def rollback_at(self, out, slot):
        if slot < self.base:
            return False
        return self.c.rollback_at(out[self.base:], slot - self.base)


class ThreadSim:
    """One thread slot: the conversation's history token ids, its system prefix and the turn in flight."""

    def __init__(self, tid: int, prefix: list[int], rng: random.Random, args, vocab: int):
        self.tid = tid
        self.rng = rng
        self.args = args
        self.vocab = vocab
        self.prefix = prefix
        self.turns_total = 2 * args.history_turns + 1
        self.conv = 0
        self._new_conversation(rng.randrange(self.turns_total))
        self.resumed: list[int] = []
        self.pending_user: list[int] = []

    def _rand(self, n):
        return [self.rng.randrange(1000, min(self.vocab, 120000)) for _ in range(n)]

    def _user_len(self) -> int:
        u = self.args.user_tokens
        return self.rng.randint(max(1, u // 2), max(1, u + u // 2))

    def _reply_len(self) -> int:
        return self.rng.randint(self.args.min_out, self.args.max_out)

    def _new_conversation(self, turn: int) -> None:
        self.conv += 1
        self.turn = turn
        self.history = []
        for _ in range(turn):
            self.history += self._rand(self._user_len()) + self._rand(self._reply_len())

    def reply_budget(self, stationary: bool) -> tuple[int, int]:
        """(reply length, tokens of it already generated). ``stationary``: a turn observed at a random instant —
        length-biased length, uniform position (the renewal process's stationary state)."""
        lo, hi = self.args.min_out, self.args.max_out
        if not stationary:
            return self._reply_len(), 0
        while True:
            n = self.rng.randint(lo, hi)
            if self.rng.random() * hi < n:
                return n, self.rng.randrange(n)

    def next_prompt(self, done: int = 0) -> list[int]:
        self.pending_user = self._rand(self._user_len())
        self.resumed = self._rand(done)
        return self.prefix + self.history + self.pending_user + self.resumed

    def complete(self, out_ids: list[int]) -> None:
        self.history += self.pending_user + self.resumed + out_ids
        self.turn += 1
        if self.turn >= self.turns_total:
            self._new_conversation(0)


def stratified_budgets(threads, args, rng: random.Random) -> list[tuple[int, int]]:
    """(reply length, tokens already generated) per slot at setup, drawn from the renewal process's stationary law
    (ThreadSim.reply_budget) with the slots' REMAINING lengths stratified: slot i gets the (i + U)/n quantile of
    the stationary residual-life distribution (strata shuffled over the slots). Every slot's marginal is the
    stationary one, so the expected load of any window is unchanged, but the new-turn arrivals of the first ~E[n]
    steps land close to their expected count instead of Poisson-scattered around it: a 20-step window (about five
    arrivals at 64 threads) otherwise swings by +-6 % ms/step with the seed (profiles/r03/bench_stationarity.txt)."""
    lo, hi, n = args.min_out, args.max_out, len(threads)
    if n == 0:
        return []
    # residual r (tokens left, 1..hi): P(r) ∝ P(reply >= r) for a reply length uniform on [lo, hi]
    w = [(hi - max(r, lo) + 1) for r in range(1, hi + 1)]
    tot = float(sum(w))
    cdf, acc = [], 0.0
    for x in w:
        acc += x / tot
        cdf.append(acc)
    strata = list(range(n))
    rng.shuffle(strata)
    out = []
    for th, k in zip(threads, strata):
        u = (k + rng.random()) / n
        r = next((i + 1 for i, c in enumerate(cdf) if c >= u), hi)
        length = rng.randint(max(lo, r), hi)  # reply length given the residual: uniform on [max(lo, r), hi]
        out.append((length, length - r))
    return out


def main(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    from kafka_llm_service_amd.utils.affinity import pin_local_process

    pin_local_process(int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks")
    if world % args.tp:
        raise SystemExit(f"bench.py: {world} ranks not divisible by --tp {args.tp}")
    from kafka_llm_service_amd.parallel import state as pstate

    dev = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
    tp = args.tp
    dpa = args.dp_attention and world > 1
    if dpa:
        if tp != 1:
            raise SystemExit("bench.py: --dp-attention runs with --tp 1 (attention is data-parallel)")
        st = pstate.init_dp_attention(world, device=dev)
    else:
        st = pstate.init(tp=tp, device=dev) if world > 1 else pstate.get()
        if tp > 1 and dev.startswith("cuda") and st.custom_status.get("tp") != "registered" and \
                not os.environ.get("KAFKA_ALLOW_AR_FALLBACK"):
            # the TP configuration is measured on the custom xGMI all-reduce; a silent RCCL fallback would report a
            # different system (KAFKA_ALLOW_AR_FALLBACK=1 runs it anyway)
            raise SystemExit(f"bench.py: TP={tp} custom all-reduce not registered ({st.custom_status.get('tp')})")
    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams

    cfg = EngineConfig(model=args.model, device=dev, seed=args.seed, max_num_seqs=max(256, 2 * args.threads),
                       use_cascade=not args.no_cascade, use_graphs=args.graphs, kv_dtype=args.kv_dtype,
                       max_model_len=131072 if args.prefix_tokens > 6000 else 8192, tp=tp, tp_rank=st.tp_rank, dp_attention=dpa,
                       kv_run_pages=args.kv_run_pages)
    eng = LLMEngine(cfg)
    leaders = None
    if tp > 1:
        import torch.distributed as dist

        # TP followers mirror their leader's steps; the timing barriers run among the leaders only
        leaders = dist.new_group(list(range(0, world, tp)), backend="gloo")
        if not st.is_tp_leader:
            tp_worker.follower_loop(eng)
            return _report(args, world, rank, dev, eng, {"out_tokens": 0, "ttft": [], "extra": 0}, 0.0, 0.0)
        tp_worker.attach_leader(eng)
    if dpa:  # every rank steps in lockstep with its EP group (one forward per step on every rank)
        from kafka_llm_service_amd.engine import dp_attention

        agree = dp_attention.make_agree(st)

        def gen(ps, sp):
            return dp_attention.generate_lockstep(eng, st, ps, sp)

        def step():
            return eng.step_lockstep(agree)[0]
    else:
        gen, step = eng.generate, eng.step
    V = eng.model_cfg.vocab_size
    rng = random.Random(args.seed * 7919 + rank)
    prefix = [rng.randrange(1000, min(V, 120000)) for _ in range(args.prefix_tokens)]
    prefix_b = [rng.randrange(1000, min(V, 120000)) for _ in range(args.prefix_tokens)]
    n_b = int(round(args.mixed_prefix * args.threads))
    threads = [ThreadSim(i, prefix_b if i < n_b else prefix,
                         random.Random(args.seed * 1000 + rank * 100003 + i), args, V)
               for i in range(args.threads)]

    # ---- setup (untimed): every slot at a random point of its life (see the module docstring); the shared
    # prefix(es), each thread's history and its in-flight reply's already-generated tokens go into the prefix cache
    t_setup = time.perf_counter()
    budgets = stratified_budgets(threads, args, random.Random(args.seed * 31 + rank))
    prompts = [th.next_prompt(done) for th, (_, done) in zip(threads, budgets)]
    warm = SamplingParams(temperature=0, max_tokens=1, ignore_eos=True)
    for p in {tuple(t.prefix) for t in threads if t.prefix}:
        gen([list(p) + [5]], warm)
    gen(prompts, warm)
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    eng.runner.rows_hist = [0] * len(eng.runner.rows_hist)  # the histogram covers the warm-up + timed steps only

    req_thread = {}
    n_tool = int(round(args.tool_frac * args.threads))
    n_pen = int(round(args.penalty_frac * args.threads))
    tools = bench_tools() if n_tool else None
    if n_tool:
        from kafka_llm_service_amd.engine.tokenizer import tokenizer_for_model

        tok = tokenizer_for_model(eng.model_cfg)

    def submit(th: ThreadSim, prompt: list[int] | None = None, n_left: int | None = None, resumed=False):
        rid = f"t{th.tid}-c{th.conv}-turn{th.turn}"
        if prompt is None:
            n_left, _ = th.reply_budget(stationary=False)
            prompt = th.next_prompt(0)
        kw = {}
        if th.tid < n_tool:
            kw["allowed_tokens_fn"] = ToolCallLoop(tok, tools)
        elif th.tid < n_tool + n_pen:
            kw.update(presence_penalty=0.3, frequency_penalty=0.2)
        sp = SamplingParams(temperature=args.temperature, max_tokens=n_left, ignore_eos=True,
                            seed=th.tid * 1000003 + th.conv * 1009 + th.turn, **kw)
        seq = eng.add_request(rid, prompt, sp)
        req_thread[rid] = (th, seq, resumed)

    for th, p, (n, done) in zip(threads, prompts, budgets):
        submit(th, p, n - done, resumed=True)

    timing = {"out_tokens": 0, "ttft": [], "extra": 0}
    window = [float("inf")]

    steplog = [] if os.environ.get("KAFKA_BENCH_STEPLOG") else None  # per-step trace for the stationarity check

    def run_step(record: bool):
        ts = time.perf_counter()
        outs = step()
        if steplog is not None:
            st = getattr(eng.runner, "last_stats", None) or {}  # the step launched by this call (outs lag one step)
            steplog.append((ts, len(outs), sum(1 for o in outs if o.num_output_tokens == 1), st.get("T"),
                            st.get("s_total")))
        for o in outs:
            th, seq, resumed = req_thread[o.request_id]
            if record:
                timing["out_tokens"] += len(o.new_token_ids)
            if o.num_output_tokens == 1 and not resumed and seq.arrival >= window[0]:
                timing["ttft"].append(seq.first_token_time - seq.arrival)
            if o.finished:
                del req_thread[o.request_id]
                th.complete(seq.output_ids)
                submit(th)

    for _ in range(args.warmup):
        run_step(False)
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    _barrier(leaders)
    host0 = dict(eng.host_s)
    prof = None
    if os.environ.get("KAFKA_CPROFILE"):  # host-side profile of the timed steps only (scripts/gpu_cpu_prof.sh)
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    eng.runner.step_events = [] if dev.startswith("cuda") else None
    t0 = time.perf_counter()
    window[0] = t0
    for _ in range(args.steps):
        run_step(True)
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    ev = eng.runner.step_events
    eng.runner.step_events = None
    if ev:
        # GPU time inside the timed steps' spans (plan upload .. token download, kernel gaps included) vs the GPU
        # time between consecutive spans (idle unless the host had already queued the next step)
        per_step = [a.elapsed_time(b) for a, b in ev]
        timing["gpu_per_step"] = per_step  # (KAFKA_BENCH_STEPLOG: the per-step trace carries them)
        inside = sum(per_step)
        between = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(len(ev) - 1)]
        timing["gpu_ms"] = {"in_step": round(inside / len(ev), 3),
                            "between_steps": round(sum(max(0.0, x) for x in between) / max(1, len(between)), 3)}
    timing["host_ms"] = {k: round((eng.host_s[k] - host0[k]) * 1e3 / max(1, args.steps), 3) for k in host0}
    if prof is not None:
        import pstats

        prof.disable()
        with open(os.environ["KAFKA_CPROFILE"], "w") as f:
            ps = pstats.Stats(prof, stream=f)
            ps.sort_stats("tottime").print_stats(50)
            ps.sort_stats("cumtime").print_stats(60)
    _barrier(leaders)
    # ---- TTFT: keep the same load running (untimed) until enough new turns have produced their first token
    def want_more() -> bool:
        more = len(timing["ttft"]) < args.ttft_samples and timing["extra"] < args.ttft_max_steps
        if dpa:  # the group keeps stepping while any rank still needs samples
            more = bool(agree((int(more),))[0])
        return more
    while want_more():
        run_step(False)
        timing["extra"] += 1
    _barrier(leaders)
    if steplog is not None:
        with open(os.environ["KAFKA_BENCH_STEPLOG"], "w") as f:
            for i, (ts, n, first, rows, ctx) in enumerate(steplog):
                nxt = steplog[i + 1][0] if i + 1 < len(steplog) else ts
                rec = {"i": i, "timed": args.warmup <= i < args.warmup + args.steps,
                       "ms": round((nxt - ts) * 1e3, 3), "outs": n, "first_tokens": first, "rows": rows,
                       "s_total": ctx}
                g = timing.get("gpu_per_step") or []
                if rec["timed"] and i - args.warmup < len(g):
                    rec["gpu_ms"] = round(g[i - args.warmup], 3)
                f.write(json.dumps(rec) + "\n")
    if tp > 1:
        tp_worker.release_followers()
    return _report(args, world, rank, dev, eng, timing, t1 - t0, setup_s)


def _barrier(group) -> None:
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier(group=group)


def _rank_record(args, rank, dev, timing, elapsed, eng) -> dict:
    """This rank's line of the bench record: its device (index, PCI location, uuid), role and own rate."""
    import torch

    rec = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": dev,
           "role": "tp_follower" if args.tp > 1 and rank % args.tp else "replica",
           "out_tokens": int(timing["out_tokens"]),
           "tok_s": round(timing["out_tokens"] / elapsed, 1) if elapsed > 0 else 0.0,
           "ms_per_step": round(elapsed / args.steps * 1e3, 3) if elapsed > 0 else None,
           "steps": int(eng.stats.get("steps", 0)), "pci": dev}
    if dev.startswith("cuda"):
        idx = torch.device(dev).index or 0
        p = torch.cuda.get_device_properties(idx)
        rec.update(device_index=idx, pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
                   uuid=str(getattr(p, "uuid", "")), visible_devices=os.environ.get("HIP_VISIBLE_DEVICES",
                                                                                    os.environ.get("CUDA_VISIBLE_DEVICES")))
    return rec


def _report(args, world, rank, dev, eng, timing, elapsed, setup_s):
    import torch

    from kafka_llm_service_amd.parallel import state as pstate

    ttfts = sorted(timing["ttft"])
    extra = timing["extra"]
    me = _rank_record(args, rank, dev, timing, elapsed, eng)
    ranks = [me]
    dist_info = {"initialized": False}
    pre = pstate.preflight()
    if world > 1:
        import torch.distributed as dist

        # gloo over the host: the result exchange needs no device collective
        g = dist.new_group(list(range(world)), backend="gloo")
        ranks = [None] * world
        dist.all_gather_object(ranks, me, group=g)
        st = pstate.get()
        dist_info = {"initialized": True, "backend": dist.get_backend(), "world_size": dist.get_world_size()}
        if st.tp_group is not None:
            dist_info.update(tp_backend=dist.get_backend(st.tp_group), tp_group_size=dist.get_world_size(st.tp_group))
        if getattr(st, "ep_group", None) is not None:
            dist_info.update(ep_backend=dist.get_backend(st.ep_group), ep_group_size=dist.get_world_size(st.ep_group))
        if dev.startswith("cuda"):
            seen = {}
            for r in ranks:
                key = r["pci"]
                if key in seen:
                    raise SystemExit(f"bench.py: ranks {seen[key]} and {r['rank']} resolved to the same GPU {key} "
                                     "(check LOCAL_RANK / HIP_VISIBLE_DEVICES)")
                seen[key] = r["rank"]
        stats = torch.tensor([timing["out_tokens"], elapsed, extra], dtype=torch.float64)
        toks = stats[:1].clone()
        dist.all_reduce(toks, group=g)
        tmax = stats[1:].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX, group=g)
        total_tokens, elapsed, extra = float(toks.item()), float(tmax[0].item()), int(tmax[1].item())
        allt = [None] * world
        dist.all_gather_object(allt, ttfts, group=g)
        ttfts = sorted(t for part in allt for t in part)
    else:
        total_tokens = float(timing["out_tokens"])
    value = total_tokens / elapsed if elapsed > 0 else 0.0
    p50 = ttfts[len(ttfts) // 2] * 1e3 if ttfts else None
    p99 = ttfts[min(len(ttfts) - 1, int(len(ttfts) * 0.99))] * 1e3 if ttfts else None
    kv = eng.kv_stats()
    dp = world // args.tp
    headline = (args.model, args.threads, args.prefix_tokens, args.tp, args.tool_frac, args.penalty_frac) == \
        ("llama3-8b", 64, 18000, 1, 0.0, 0.0)
    res = {
        "metric": METRIC if headline else
        f"output tok/s + p50 TTFT, {args.model}, {args.threads} concurrent threads per replica",
        "value": round(value, 1), "unit": "tok/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(value / (BOUND_TOKS_PER_GPU * world), 3) if headline else None,
        "dtype": "bf16",
        "data": "synthetic (random-init weights, random token ids)",
        "config": {"model": args.model, "global_batch": args.threads * dp,
                   "seq_len": args.prefix_tokens + args.history_turns * (args.user_tokens + (args.min_out +
                                                                                         args.max_out) // 2)
                   + args.user_tokens,
                   "parallelism": (f"dpattn{world}-ep{world}" if args.dp_attention and world > 1 else
                                   f"dp{dp}" + (f"-tp{args.tp}" if args.tp > 1 else "")),
                   "threads_per_gpu": args.threads * dp // world,
                   "shared_prefix_tokens": args.prefix_tokens, "history_turns": args.history_turns,
                   "mixed_prefix": args.mixed_prefix, "max_out": [args.min_out, args.max_out],
                   "temperature": args.temperature, "cascade": not args.no_cascade, "graphs": eng.cfg.use_graphs,
                   "kv_dtype": args.kv_dtype, "tool_frac": args.tool_frac, "penalty_frac": args.penalty_frac},
        "ttft_p50_ms": round(p50, 2) if p50 else None, "ttft_p99_ms": round(p99, 2) if p99 else None,
        "ttft_samples": len(ttfts), "ttft_extra_steps": extra,
        "vs_baseline_basis": "derived 1-GPU bound 17k tok/s/GPU (BASELINE.md §3); reference publishes none",
        "setup_s": round(setup_s, 2),
        "prefix_hit_rate": round(kv["hit_tokens"] / max(1, kv["query_tokens"]), 4),
        "preemptions": eng.sched.num_preemptions,
        "planned_ahead_frac": round(eng.stats.get("planned_ahead", 0) / max(1, eng.stats.get("steps", 1)), 4),
        "planned_late_frac": round(eng.stats.get("planned_late", 0) / max(1, eng.stats.get("steps", 1)), 4),
        "step_rows_hist": dict(zip(("<=64", "65-96", "97-128", "129-256", ">256"), eng.runner.rows_hist)),
        "grammar_rollbacks": eng.stats.get("grammar_rollbacks", 0),
        "graph_stats": dict(eng.runner.graphs.stats) if eng.runner.graphs is not None else None,
        "host_ms_per_step": timing.get("host_ms"),  # rank 0's engine host time per timed step, by activity
        "gpu_ms_per_step": timing.get("gpu_ms"),  # rank 0: GPU time inside step spans / idle between them
        # self-verification of multi-GPU runs: one record per rank (which GPU it ran on, its own rate and step time;
        # TP followers report 0 tokens: their leader streams the replica's tokens) and the process groups' backends /
        # sizes as torch.distributed reports them (backend "nccl" is RCCL on ROCm)
        "ranks": world,
        "per_rank": ranks,
        "dist": dist_info,
        # pre-flight of the multi-GPU paths (parallel/state.py preflight): peer-access matrix of the visible devices,
        # custom collective registration per group (or the fallback reason), RCCL version, group sizes
        "preflight": pre,
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    pstate.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
