"""Continuous-batching scheduler (iteration level) with chunked prefill, prefix-cache admission and preemption.

Every engine step the scheduler builds one mixed batch under a token budget:
  1. every RUNNING sequence that has exactly its last sampled token left to compute contributes one DECODE token
     (decode has priority, so a long cold prefill never stalls the streams of other threads);
  2. RUNNING sequences that are part-way through their prompt continue their prefill chunk;
  3. WAITING sequences are admitted FCFS: the KV manager matches their prompt against the prefix tree (shared system
     prompt + the thread's own history), allocates pages for the uncached tail, and the tail is
     prefilled in chunks of at most the remaining budget.
When the KV pool cannot grow a running sequence, the most recently admitted sequence is preempted by recompute: its
private pages are freed, its committed pages stay in the prefix tree, so its re-admission is mostly a cache hit.

The reference service has no scheduler — concurrency is one asyncio loop forwarding requests to a remote API
(/root/reference/server.py:384-523); this component replaces that.
"""
from __future__ import annotations

import math
from collections import deque
from dataclasses import dataclass, field

from kafka_llm_service_amd.engine.sequence import PENDING, Sequence, SeqStatus


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_prefill_chunk: int = 8192
    max_model_len: int = 131072
    max_blocks_per_seq: int = 8192
    # TPOT guard: while at least `tpot_guard_decodes` streams are decoding, a step takes at most this many prefill
    # tokens (0 = no guard) — a cold 18k-token admission is spread over many steps instead of stalling every stream
    # for one ~100 ms step; a new turn of a cached thread (tens of tokens) still fits in the next step
    prefill_tokens_while_decoding: int = 512
    tpot_guard_decodes: int = 16
    # Row fit: while the guard holds, prefill is also capped so the whole step stays within `step_rows_fit` rows
    # (0 = off) as long as that leaves at least `step_rows_fit_min` prefill tokens. Steps of <= 128 rows run the
    # weight-streaming decode GEMM (ops.STREAM_MAX_M); a 64-stream step that admits 100 new-turn tokens would
    # otherwise take hipBLASLt at M = 164 (~172 vs ~128 us of GEMM per Llama-3-8B layer, profiles/wstream_sweep_r01.log,
    # profiles/r02/gemm_sweep_M129_320.log). A new turn longer than the room is chunked over two steps.
    step_rows_fit: int = 0
    step_rows_fit_min: int = 32
    # Burst splitting: new prefills admitted into one step may cost at most this many token-equivalents, a token at
    # context position c counting 1 + c / attn_equiv_keys (its GEMM work plus its attention over c keys: at
    # Llama-3-8B shapes ~30k keys of attention cost as much as the token's projections). The first admission of a
    # step is never held back (a single cold prefill keeps its full chunk), so this only splits a BURST of new
    # turns — e.g. 64 threads x 40 new tokens against a 37k-token shared prefix, ~5.6k token-equivalents — over
    # a few steps, first arrivals first, instead of one ~100 ms step that every one of them waits for (0 = off).
    # Optional: with a deep queue at least ceil(sqrt(burst_sqrt_k x waiting)) admissions go into a step regardless
    # of the budget (the group size minimizing the mean completion of n equal jobs over steps of floor + group x
    # job). Measured on MI355X it only trades later turns for the synchronized first one (profiles/r03/
    # serve_burst_ab.jsonl: turn-0 p50 ~240 vs ~255 ms, turns 1-3 ~100-180 vs ~50-70 ms), so it is off (0).
    # Budget 384 (was 512): served burst (64 threads x 4 turns) p50 41-43 vs 47-53 ms, p99 196 vs 215-243 ms; 256
    # doubles the first turn's p50; the headline moves -0.1..-0.3 % (profiles/r05/serve/burst_budget_*.log,
    # profiles/r05/bench_ab_prefill_budget_384.jsonl); 768-2048 were worse in round 4 (profiles/r04/serve/)
    prefill_cost_budget: int = 384
    attn_equiv_keys: int = 30000
    burst_sqrt_k: float = 0.0


@dataclass
class ScheduledBatch:
    decode: list[Sequence] = field(default_factory=list)
    # (seq, start, end): compute tokens [start, end) of seq; samples iff end == seq.total_len
    prefill: list[tuple[Sequence, int, int]] = field(default_factory=list)
    preempted: list[Sequence] = field(default_factory=list)
    cut: list[Sequence] = field(default_factory=list)  # finished by the scheduler (outgrew the KV pool)

    @property
    def num_tokens(self) -> int:
        return len(self.decode) + sum(e - s for _, s, e in self.prefill)

    @property
    def empty(self) -> bool:
        return not self.decode and not self.prefill


class NeedSync(Exception):
    """A speculative plan would have to preempt: plan again once the in-flight step has landed."""


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, kv):
        self.cfg = cfg
        self.kv = kv
        self.page = kv.page
        self.waiting: deque[Sequence] = deque()
        self.running: list[Sequence] = []
        self.num_preemptions = 0

    def add(self, seq: Sequence) -> None:
        if seq.total_len >= self.cfg.max_model_len:
            raise ValueError(f"prompt of {seq.total_len} tokens exceeds max_model_len={self.cfg.max_model_len}")
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def _preempt_one(self, batch: ScheduledBatch, protect: Sequence) -> bool:
        for victim in reversed(self.running):
            if victim is protect:
                continue
            self._evict(victim)
            batch.preempted.append(victim)
            if victim in batch.decode:
                batch.decode.remove(victim)
            return True
        return False

    def _evict(self, seq: Sequence) -> None:
        self.kv.free_sequence(seq.seq_id)
        self.running.remove(seq)
        seq.status = SeqStatus.WAITING
        seq.num_computed = 0
        seq.preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(seq)

    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        if seq in self.running:
            self.running.remove(seq)
        else:
            try:
                self.waiting.remove(seq)
            except ValueError:
                pass
        if self.kv.has_seq(seq.seq_id):
            self.kv.free_sequence(seq.seq_id)

    @staticmethod
    def _grammar_plannable(seq: Sequence) -> bool:
        """May a grammar-constrained row be planned ahead of its in-flight token? Constraints that can speculate
        past a pending token (``ToolCallConstraint.plan_state``: free strings, digits, the first token of "auto")
        say so; any other allowed_tokens_fn waits while its last token is PENDING."""
        fn = seq.params.allowed_tokens_fn
        ps = getattr(fn, "plan_state", None)
        if ps is None:
            return seq.output_ids[-1:] != [PENDING]
        return ps(seq.output_ids) == "ok"

    def _cost(self, start: int, end: int) -> float:
        """Token-equivalents of prefilling positions [start, end) (SchedulerConfig.prefill_cost_budget)."""
        n = end - start
        return n * (1.0 + (start + end) * 0.5 / max(1, self.cfg.attn_equiv_keys))

    def schedule(self, speculative: bool = False) -> ScheduledBatch:
        """Build the next batch. ``speculative``: planned while the previous step is still on the GPU (its sampled
        tokens are PENDING placeholders): sequences whose pending token is their last by length, and grammar-constrained
        sequences whose next mask depends on a pending token, are left out, and a plan that would need a preemption is
        abandoned (``NeedSync``) — the engine then plans after the step lands."""
        cfg = self.cfg
        batch = ScheduledBatch()
        budget = cfg.max_num_batched_tokens
        # 1. decodes (and their page growth, preempting from the tail if the pool is dry)
        for seq in list(self.running):
            if seq.status != SeqStatus.RUNNING or seq.remaining != 1:
                continue
            if speculative and (len(seq.output_ids) >= seq.params.max_tokens or seq.total_len >= cfg.max_model_len):
                continue
            if speculative and seq.params.allowed_tokens_fn is not None and not self._grammar_plannable(seq):
                # its grammar state (the mask of the next token) needs the token still being sampled (a choice:
                # tool name / enum / boolean), or a landed token broke the grammar's guess: this row alone sits
                # out the plan-ahead step and rejoins once the token has landed — the other rows keep the pipeline
                continue
            while not self.kv.ensure_capacity(seq.seq_id, seq.total_len):
                if speculative:
                    raise NeedSync()
                if not self._preempt_one(batch, seq):
                    # alone and still out of pages: the sequence has outgrown the whole KV pool -> end it by length
                    self.finish(seq, "length")
                    batch.cut.append(seq)
                    break
            if seq.status != SeqStatus.RUNNING:
                continue
            batch.decode.append(seq)
            budget -= 1
        if cfg.prefill_tokens_while_decoding and len(batch.decode) >= cfg.tpot_guard_decodes:
            budget = min(budget, cfg.prefill_tokens_while_decoding)
            room = cfg.step_rows_fit - len(batch.decode)
            if cfg.step_rows_fit and room >= cfg.step_rows_fit_min:
                budget = min(budget, room)
        # 2. running prefills
        for seq in list(self.running):
            if budget <= 0:
                break
            # remaining == 1 sequences were scheduled as decodes in phase 1
            if seq.status != SeqStatus.RUNNING or seq.remaining <= 1:
                continue
            n = min(seq.remaining, budget, cfg.max_prefill_chunk)
            end = seq.num_computed + n
            if not self.kv.ensure_capacity(seq.seq_id, end):
                continue
            batch.prefill.append((seq, seq.num_computed, end))
            budget -= n
        # 3. admissions
        cost = sum(self._cost(a, b) for _, a, b in batch.prefill)
        admitted = 0
        group = math.ceil(math.sqrt(cfg.burst_sqrt_k * len(self.waiting))) if cfg.burst_sqrt_k else 1
        while self.waiting and budget > 0 and len(self.running) < cfg.max_num_seqs:
            seq = self.waiting[0]
            toks = seq.all_ids()
            cached = self.kv.add_sequence(seq.seq_id, toks)
            n = min(seq.total_len - cached, budget, cfg.max_prefill_chunk)
            end = cached + n
            c = self._cost(cached, end)
            if cfg.prefill_cost_budget and admitted >= group and cost + c > cfg.prefill_cost_budget:
                self.kv.free_sequence(seq.seq_id)  # next step (its prefix match is redone then)
                break
            if not self.kv.ensure_capacity(seq.seq_id, end):
                self.kv.free_sequence(seq.seq_id)
                break
            cost += c
            admitted += 1
            self.waiting.popleft()
            seq.num_cached = cached if seq.preemptions == 0 else seq.num_cached
            seq.num_computed = cached
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
            if end - cached == 1 and end == seq.total_len:
                batch.decode.append(seq)
            else:
                batch.prefill.append((seq, cached, end))
            budget -= n
        return batch
