#!/usr/bin/env python3
"""Headline benchmark: output tok/s + p50 TTFT, Llama-3-8B, 64 concurrent multi-turn threads per MI355X.

BASELINE.json metric: "output tok/s + p50 TTFT, Llama-3-8B, 64 concurrent threads, 1/2/4/8 MI355X"
(configs 2-3: Llama-3 8B bf16 TP=1, 64 concurrent threads with 4-turn history, per-thread prefix-KV reuse).

Workload (synthetic data, random-init Llama-3-8B weights — no checkpoints/datasets are reachable offline):
  * every thread's prompt = the shared Kafka system prefix (default 18,000 tokens: the reference's ~70k-char system
    prompt + ~6.6k chars of tool schemas) + its own 4-turn history (~1.3k tokens: 4 x (64 user +
    256 assistant)) + a new 64-token user message;
  * each thread loops forever: submit the next turn, stream max_tokens in [128, 384] (ignore_eos, T=0.7), append the
    reply to its history, submit the next turn immediately — so the engine sees continuous batching with prefix hits
    on the shared prefix AND on each thread's own history, the way /v1/threads/{id}/chat/completions traffic does;
  * DP: one engine replica per GPU (one process per GPU under torchrun), 64 threads per replica (weak scaling).

A "step" is one engine iteration (one continuous-batching forward over the mixed decode/prefill batch, sampling
included). W untimed warmup steps, then exactly K timed steps between barrier + synchronize; value = total output
tokens of all ranks / max rank time. vs_baseline divides by the reference's own 64-thread streaming ceiling
(22.3k chunks/s with an instant stub LLM).
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import torch

METRIC = "output tok/s + p50 TTFT, Llama-3-8B, 64 concurrent threads, 1/2/4/8 MI355X"  # BASELINE.json
BASELINE_TOKS = 22300.0  # stub chunks/s, 64 threads, stream (reference plumbing ceiling)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel size per replica (e.g. 8 for llama3-70b)")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--threads", type=int, default=64, help="concurrent threads per GPU")
    ap.add_argument("--prefix-tokens", type=int, default=18000, help="shared system prefix (0 = short prompt)")
    ap.add_argument("--history-turns", type=int, default=4)
    ap.add_argument("--user-tokens", type=int, default=64)
    ap.add_argument("--reply-tokens", type=int, default=256)
    ap.add_argument("--min-out", type=int, default=128)
    ap.add_argument("--max-out", type=int, default=384)
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--no-cascade", action="store_true")
    ap.add_argument("--graphs", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


class ThreadSim:
    """One chat thread: history token ids + the turn currently in flight."""

    def __init__(self, tid: int, prefix: list[int], rng: random.Random, args, vocab: int):
        self.tid = tid
        self.rng = rng
        self.args = args
        self.vocab = vocab
        self.history: list[int] = []
        for _ in range(args.history_turns):
            self.history += self._rand(args.user_tokens) + self._rand(args.reply_tokens)
        self.prefix = prefix
        self.turn = 0
        self.inflight = None

    def _rand(self, n):
        return [self.rng.randrange(1000, min(self.vocab, 120000)) for _ in range(n)]

    def next_prompt(self) -> list[int]:
        self.pending_user = self._rand(self.args.user_tokens)
        return self.prefix + self.history + self.pending_user

    def complete(self, out_ids: list[int]) -> None:
        self.history += self.pending_user + out_ids
        self.turn += 1


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from kafka_llm_service_amd.parallel import state as pstate

    dev = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
    tp = args.tp
    st = pstate.init(tp=tp, device=dev) if world > 1 else pstate.get()
    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams

    cfg = EngineConfig(model=args.model, device=dev, seed=args.seed, max_num_seqs=max(256, 2 * args.threads),
                       max_num_batched_tokens=8192, use_cascade=not args.no_cascade, use_graphs=args.graphs,
                       max_model_len=131072 if args.prefix_tokens > 6000 else 8192, tp=tp, tp_rank=st.tp_rank)
    eng = LLMEngine(cfg)
    leaders = None
    if tp > 1:
        import torch.distributed as dist

        # TP followers mirror their leader's steps; the timing barriers run among the leaders only
        leaders = dist.new_group(list(range(0, world, tp)), backend="gloo")
        if not st.is_tp_leader:
            tp_worker.follower_loop(eng)
            return _report(args, world, rank, dev, eng, {"out_tokens": 0, "ttft": []}, 0.0, 0.0)
        tp_worker.attach_leader(eng)
    V = eng.model_cfg.vocab_size
    rng = random.Random(args.seed * 7919 + rank)
    prefix = [rng.randrange(1000, min(V, 120000)) for _ in range(args.prefix_tokens)]
    threads = [ThreadSim(i, prefix, random.Random(args.seed * 1000 + rank * 100003 + i), args, V)
               for i in range(args.threads)]

    # ---- setup (untimed): populate the prefix cache with the shared prefix and each thread's history
    t_setup = time.perf_counter()
    if prefix:
        eng.generate([prefix + [5]], SamplingParams(temperature=0, max_tokens=1, ignore_eos=True))
    eng.generate([t.prefix + t.history for t in threads], SamplingParams(temperature=0, max_tokens=1,
                                                                            ignore_eos=True))
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    req_thread = {}
    counter = [0]

    def submit(th: ThreadSim):
        rid = f"t{th.tid}-turn{th.turn}"
        n_out = th.rng.randint(args.min_out, args.max_out)
        sp = SamplingParams(temperature=args.temperature, max_tokens=n_out, ignore_eos=True,
                            seed=th.tid * 1000 + th.turn)
        seq = eng.add_request(rid, th.next_prompt(), sp)
        req_thread[rid] = (th, seq)
        counter[0] += 1

    for th in threads:
        submit(th)

    timing = {"out_tokens": 0, "ttft": []}
    window = [None]

    def run_step(record: bool):
        outs = eng.step()
        now = time.perf_counter()
        for o in outs:
            th, seq = req_thread[o.request_id]
            if record:
                timing["out_tokens"] += len(o.new_token_ids)
                if o.num_output_tokens == 1 and seq.arrival >= window[0]:
                    timing["ttft"].append(seq.first_token_time - seq.arrival)
            if o.finished:
                del req_thread[o.request_id]
                th.complete(seq.output_ids)
                submit(th)
        return now

    for _ in range(args.warmup):
        run_step(False)
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    _barrier(leaders)
    prof = None
    if os.environ.get("KAFKA_CPROFILE"):  # host-side profile of the timed steps only (scripts/gpu_cpu_prof.sh)
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    window[0] = t0
    for _ in range(args.steps):
        run_step(True)
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    if prof is not None:
        import pstats

        prof.disable()
        with open(os.environ["KAFKA_CPROFILE"], "w") as f:
            st = pstats.Stats(prof, stream=f)
            st.sort_stats("tottime").print_stats(50)
            st.sort_stats("cumtime").print_stats(60)
    _barrier(leaders)
    if tp > 1:
        tp_worker.release_followers()
    return _report(args, world, rank, dev, eng, timing, t1 - t0, setup_s)


def _barrier(group) -> None:
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier(group=group)


def _report(args, world, rank, dev, eng, timing, elapsed, setup_s):
    from kafka_llm_service_amd.parallel import state as pstate

    local_stats = torch.tensor([timing["out_tokens"], elapsed], dtype=torch.float64)
    ttfts = sorted(timing["ttft"])
    if world > 1:
        import torch.distributed as dist

        dev_t = local_stats.to(dev)
        toks = dev_t[:1].clone()
        dist.all_reduce(toks)
        tmax = dev_t[1:].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        total_tokens, elapsed = float(toks.item()), float(tmax.item())
        # gather TTFT samples for the global p50
        n = torch.tensor([len(ttfts)], device=dev)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n)
        m = int(max(s.item() for s in sizes)) or 1
        buf = torch.full((m,), float("nan"), dtype=torch.float64, device=dev)
        if ttfts:
            buf[:len(ttfts)] = torch.tensor(ttfts, dtype=torch.float64, device=dev)
        bufs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf)
        allt = torch.cat(bufs).cpu()
        ttfts = sorted(allt[~torch.isnan(allt)].tolist())
    else:
        total_tokens = float(timing["out_tokens"])
    value = total_tokens / elapsed
    p50 = ttfts[len(ttfts) // 2] * 1e3 if ttfts else None
    p99 = ttfts[min(len(ttfts) - 1, int(len(ttfts) * 0.99))] * 1e3 if ttfts else None
    kv = eng.kv_stats()
    res = {
        "metric": METRIC if (args.model, args.threads) == ("llama3-8b", 64) else
        f"output tok/s + p50 TTFT, {args.model}, {args.threads} concurrent threads per replica",
        "value": round(value, 1), "unit": "tok/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(value / BASELINE_TOKS, 3), "dtype": "bf16",
        "data": "synthetic (random-init weights, random token ids)",
        "config": {"model": args.model, "global_batch": args.threads * (world // args.tp), "seq_len": args.prefix_tokens
                   + args.history_turns * (args.user_tokens + args.reply_tokens) + args.user_tokens,
                   "parallelism": f"dp{world // args.tp}" + (f"-tp{args.tp}" if args.tp > 1 else ""), "threads_per_gpu": args.threads,
                   "shared_prefix_tokens": args.prefix_tokens, "history_turns": args.history_turns,
                   "max_out": [args.min_out, args.max_out], "temperature": args.temperature,
                   "cascade": not args.no_cascade, "graphs": args.graphs},
        "ttft_p50_ms": round(p50, 2) if p50 else None, "ttft_p99_ms": round(p99, 2) if p99 else None,
        "ttft_samples": len(ttfts), "setup_s": round(setup_s, 2),
        "prefix_hit_rate": round(kv["hit_tokens"] / max(1, kv["query_tokens"]), 4),
        "preemptions": eng.sched.num_preemptions,
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    pstate.destroy()


if __name__ == "__main__":
    sys.exit(main())
