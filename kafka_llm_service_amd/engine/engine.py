"""LLMEngine: KV cache allocation + scheduler + model runner + output processing (one replica, one TP group).

Synchronous core API (used by bench.py, tests and the async driver):
    eng = LLMEngine(EngineConfig(model="llama3-8b"))
    eng.add_request("r1", prompt_ids, SamplingParams(max_tokens=64))
    while eng.has_unfinished(): outs = eng.step()       # -> list[StepOutput]

The async driver (``engine/async_engine.py``) runs ``step()`` on a dedicated thread so the API event loop never
blocks on the GPU (SURVEY.md §2.4 "Engine step loop must not run on the API event loop").
"""
from __future__ import annotations

import logging
import os
import time
from collections import deque
from dataclasses import dataclass, field, replace

import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.model_runner import ModelRunner
from kafka_llm_service_amd.engine.scheduler import NeedSync, Scheduler, SchedulerConfig
from kafka_llm_service_amd.engine.sequence import PENDING, SamplingParams, Sequence, StepOutput
from kafka_llm_service_amd.models.config import ModelConfig, get_config
from kafka_llm_service_amd.models.weights import build_model
from kafka_llm_service_amd.runtime import KVManager
from kafka_llm_service_amd.obs import trace
from kafka_llm_service_amd.utils import faults

log = logging.getLogger("kafka.engine")


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    weights: str | None = None          # safetensors dir/file; None = seeded random init
    seed: int = 0
    device: str | None = None           # default cuda:<local rank> when a GPU is present, else cpu
    tp: int = 1
    tp_rank: int = 0
    kv_fraction: float = 0.80           # of free device memory after weights
    num_kv_blocks: int | None = None    # explicit pool size (pages of 16 tokens)
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_prefill_chunk: int = 8192
    prefill_tokens_while_decoding: int = 512  # TPOT guard (engine/scheduler.py); 0 = off
    step_rows_fit: int | None = None    # row fit (engine/scheduler.py); None = env KAFKA_STEP_ROWS_FIT, default 0
    max_model_len: int = 131072
    enable_prefix_cache: bool = True
    # pages a decoding sequence takes at a time as ONE run of consecutive block ids (the spare ones reserved for it):
    # a thread's history then lies in long runs of the pool (runtime/csrc/kv_manager.cpp)
    kv_run_pages: int = 1
    use_cascade: bool = True
    cascade_min_prefix: int = 512
    target_wgs: int = 256               # tile-kernel workgroups per pass (8-wave WGs, one per CU)
    prefill_kv_chunk: int = 1024        # a new turn on > 2x this many cached keys splits its key range so all
                                        # tiles make ~target_wgs workgroups (chunks >= min(256, this))
    # hipGraph decode steps (engine/graphs.py): None = on for TP > 1 on GPUs (every rank launches ~800 kernels per
    # step there), off at TP = 1 (the host already runs a step ahead: measured no faster, profiles/r02/graphs_ab_*)
    use_graphs: bool | None = None
    # paged KV cache: "bf16", or "fp8" = e4m3 with one power-of-two scale per (token, kv head) for K and for V
    # (half the bytes per page: twice the pages, half the decode attention traffic; ops/csrc/rope_kv.hip)
    kv_dtype: str = "bf16"
    # decode GEMMs: "stream" = weight-streaming MFMA kernel on wave-tiled weight copies (csrc/wstream_gemm.hip),
    # "blas" = hipBLASLt only; "auto" = stream on GPU (env KAFKA_DECODE_GEMM overrides)
    decode_gemm: str = "auto"           # auto | stream | stream_only (tiled weights only) | blas
    async_scheduling: bool = True       # plan step n+1 on the host while step n runs on the GPU
    # Mixtral data-parallel attention (engine/dp_attention.py): this rank serves its own sequences with whole
    # attention weights; experts are sharded over parallel.state's EP group and every step runs in lockstep with
    # the group (step_lockstep; planned ahead like step())
    dp_attention: bool = False
    eos_token_ids: list[int] = field(default_factory=list)

    def resolve_device(self) -> torch.device:
        if self.device:
            return torch.device(self.device)
        if torch.cuda.is_available():
            import os

            return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
        return torch.device("cpu")


@dataclass
class _Plan:
    batch: object
    host: object
    sampled: list
    seqs: list
    n_added: int


@dataclass
class _InFlight:
    sampled: list           # sequences with a row in the step's sampler output
    slots: list             # index of each one's PENDING placeholder in its output_ids
    launched: object        # ModelRunner.Launched
    t0: float


def _agree_min(n: int) -> int:
    import torch.distributed as dist

    from kafka_llm_service_amd.parallel import state as pstate

    st = pstate.get()
    if st.tp == 1 or not dist.is_initialized():
        return n
    t = torch.tensor([n], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.cpu_group)
    return int(t.item())


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model_cfg: ModelConfig | None = None, model=None):
        self.cfg = cfg
        self.model_cfg = model_cfg or get_config(cfg.model)
        self.device = cfg.resolve_device()
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        mc = self.model_cfg
        t0 = time.perf_counter()
        dpa = None
        if cfg.dp_attention:
            from kafka_llm_service_amd.parallel import state as pstate

            st = pstate.get()
            dpa = (st.ep, st.ep_rank)
        self.model = model or build_model(mc, self.device, tp=cfg.tp, tp_rank=cfg.tp_rank, seed=cfg.seed,
                                          weights=cfg.weights, max_positions=min(cfg.max_model_len,
                                                                                 mc.max_position_embeddings),
                                          dp_attention=dpa)
        mode = os.environ.get("KAFKA_DECODE_GEMM", cfg.decode_gemm)
        if mode == "auto":
            mode = "stream" if self.device.type == "cuda" else "blas"
        if mode == "stream" and not self.model.stream:
            need = self.model.stream_weight_bytes()
            free = torch.cuda.mem_get_info(self.device)[0] if self.device.type == "cuda" else need * 4
            if need <= 0.5 * free:
                self.model.enable_stream_weights()  # before the KV pool is sized from the free memory
            else:  # e.g. Llama-3-70B on one GPU: a second copy of 140 GB would starve the KV pool
                log.warning("wave-tiled weight copy (%.1f GB) does not fit next to the KV pool (%.1f GB free): "
                            "keeping tiled weights only (prefill untiles per projection)", need / 1e9, free / 1e9)
                self.model.enable_stream_weights(tiled_only=True)
        elif mode == "stream_only" and not self.model.stream:
            self.model.enable_stream_weights(tiled_only=True)
        if self.model.tiled_only and cfg.max_num_seqs > self.model.stream_max_m:
            # decode batches beyond the streaming kernel's rows would untile every projection every step
            log.info("tiled-only weights: max_num_seqs %d -> %d", cfg.max_num_seqs, self.model.stream_max_m)
            cfg.max_num_seqs = self.model.stream_max_m
        self.load_s = time.perf_counter() - t0
        self.eos = set(cfg.eos_token_ids or mc.eos_token_ids)
        hkv, D, L = self.model.hkv, self.model.D, mc.num_layers
        page_bytes = L * ops.kv_page_bytes(hkv, D, cfg.kv_dtype)
        self.fi = faults.get()
        if self.fi.kv_blocks:
            nb = self.fi.kv_blocks
        elif cfg.num_kv_blocks:
            nb = cfg.num_kv_blocks
        elif self.device.type == "cuda":
            free, _ = torch.cuda.mem_get_info(self.device)
            nb = int(free * cfg.kv_fraction) // page_bytes
        else:
            nb = 4096
        if cfg.tp > 1:
            nb = _agree_min(nb)  # every rank of the TP group indexes the same page ids
        self.num_blocks = nb
        # zeroed once: attention tiles read whole 16-key pages and 32-key blocks, and a masked key still multiplies
        # its V row by p = 0 — finite leftovers of other sequences are harmless, NaN bit patterns in never-written
        # memory are not (0 * NaN = NaN; tests/test_engine_gpu.py poisons the allocator to keep this honest)
        kshape, vshape, kv_dt = ops.kv_cache_shapes(nb, hkv, D, cfg.kv_dtype)
        self.k_cache = torch.zeros(L, *kshape, dtype=kv_dt, device=self.device)
        self.v_cache = torch.zeros(L, *vshape, dtype=kv_dt, device=self.device)
        self.kvm = KVManager(nb, 16, cfg.enable_prefix_cache, cfg.kv_run_pages)
        max_blocks = (cfg.max_model_len + 15) // 16
        self.sched = Scheduler(SchedulerConfig(max_num_seqs=cfg.max_num_seqs,
                                               max_num_batched_tokens=cfg.max_num_batched_tokens,
                                               max_prefill_chunk=cfg.max_prefill_chunk,
                                               prefill_tokens_while_decoding=cfg.prefill_tokens_while_decoding,
                                               step_rows_fit=self._step_rows_fit(),
                                               prefill_cost_budget=int(os.environ.get("KAFKA_PREFILL_COST_BUDGET",
                                                                                      "384")),
                                               burst_sqrt_k=float(os.environ.get("KAFKA_BURST_SQRT_K", "0")),
                                               max_model_len=cfg.max_model_len, max_blocks_per_seq=max_blocks),
                               self.kvm)
        kc = [self.k_cache[i] for i in range(L)]
        vc = [self.v_cache[i] for i in range(L)]
        self.runner = ModelRunner(self.model, kc, vc, self.kvm, cfg.max_num_seqs, max_blocks,
                                  cascade_min_prefix=cfg.cascade_min_prefix, use_cascade=cfg.use_cascade,
                                  target_wgs=cfg.target_wgs, prefill_kv_chunk=cfg.prefill_kv_chunk)
        if cfg.use_graphs is None:  # env KAFKA_GRAPHS=0/1 overrides the default (on for TP > 1 on GPUs)
            env = os.environ.get("KAFKA_GRAPHS")
            cfg.use_graphs = (env == "1") if env in ("0", "1") else (cfg.tp > 1 and self.device.type == "cuda")
            cfg.use_graphs = cfg.use_graphs and self.device.type == "cuda"
        if cfg.use_graphs:
            from kafka_llm_service_amd.engine.graphs import DecodeGraphs

            self.runner.graphs = DecodeGraphs(self.runner)
        self.requests: dict[str, Sequence] = {}
        self.stats = {"steps": 0, "prompt_tokens": 0, "cached_tokens": 0, "output_tokens": 0, "step_time": 0.0,
                      "replans": 0, "planned_ahead": 0, "planned_late": 0}
        # host seconds per activity (plan: schedule + build_host, launch: enqueue a step, wait: blocked on a step's
        # tokens, finish: bookkeeping of landed tokens) — the bench reports them per step
        self.host_s = {"plan": 0.0, "launch": 0.0, "wait": 0.0, "finish": 0.0}
        self._inflight: _InFlight | None = None  # the step on the GPU that has not been collected yet
        self.step_ms: deque = deque(maxlen=512)  # intervals between consecutive step completions (busy periods)
        self._t_done = 0.0
        self._coll_mark = (0, 0)  # (collective calls, steps) at the last perf_stats() read
        self._n_added = 0
        self.stop_checker_factory = None  # set by the frontend: (request params) -> incremental stop-string checker
        log.info("engine ready: %s tp=%d kv pages=%d (%s, %.1f GB) load %.1fs", mc.name, cfg.tp, nb, cfg.kv_dtype,
                 nb * page_bytes / 1e9, self.load_s)

    # ------------------------------------------------------------------------------------------------------------

    def _step_rows_fit(self) -> int:
        """Row fit of the scheduler (engine/scheduler.py): explicit config, else env KAFKA_STEP_ROWS_FIT, else on
        (ops.STREAM_MAX_M) only for tiled-only weights — there a step beyond the streaming kernel's rows untiles
        every projection for hipBLASLt, which costs far more than splitting a new turn over two steps (Llama-3-70B
        on one GPU: profiles/r02/bench_70b_tp1_*), while with both weight copies the fit measured slower
        (profiles/r02/step_rows_fit_rejected.jsonl)."""
        if self.cfg.step_rows_fit is not None:
            return self.cfg.step_rows_fit
        env = os.environ.get("KAFKA_STEP_ROWS_FIT")
        if env is not None:
            return int(env)
        # 128 rather than the kernel's 256: with two row tiles the streaming GEMM is slower per row, and splitting a
        # long new turn costs less (Llama-3-70B TP = 1: 1,516 vs 1,422 tok/s, TTFT 140 vs 119 ms,
        # profiles/r02/bench_70b_tp1_rowfit256_ab.jsonl)
        return ops.STREAM_MAX_M if self.model.tiled_only else 0

    def add_request(self, request_id: str, prompt_ids: list[int], params: SamplingParams | None = None,
                    meta: dict | None = None) -> Sequence:
        if request_id in self.requests:
            raise ValueError(f"duplicate request id {request_id}")
        params = params or SamplingParams()
        if len(prompt_ids) + 1 > self.cfg.max_model_len:
            raise ValueError(f"This model's maximum context length is {self.cfg.max_model_len} tokens. However, "
                             f"your messages resulted in {len(prompt_ids)} tokens.")
        pool_tokens = self.num_blocks * 16
        if len(prompt_ids) + 1 > pool_tokens:
            # a sequence that can never fit the KV pool would stall the scheduler; refuse it like an over-long prompt
            raise ValueError(f"This model's maximum context length is {pool_tokens} tokens on this replica (KV "
                             f"pool). However, your messages resulted in {len(prompt_ids)} tokens.")
        V = self.model_cfg.vocab_size
        if prompt_ids and (min(prompt_ids) < 0 or max(prompt_ids) >= V):
            # an out-of-range id would read past the embedding table on the GPU (a device fault, not an exception)
            raise ValueError(f"prompt token ids must lie in [0, {V}); got [{min(prompt_ids)}, {max(prompt_ids)}]")
        if params.tool_grammar is not None and params.allowed_tokens_fn is None:
            from kafka_llm_service_amd.engine.constrained import ToolCallConstraint
            from kafka_llm_service_amd.engine.tokenizer import tokenizer_for_model

            g = params.tool_grammar
            c = ToolCallConstraint(tokenizer_for_model(self.model_cfg), g.get("tools") or [], g.get("tool_choice"))
            params = replace(params, allowed_tokens_fn=c, stop_token_ids=list(params.stop_token_ids) + [c.end])
        seq = Sequence(request_id, prompt_ids, params, meta)
        if self.stop_checker_factory is not None and params.stop:
            seq.stop_checker = self.stop_checker_factory(params)
        self.requests[request_id] = seq
        self.sched.add(seq)
        self._n_added += 1
        return seq

    def abort(self, request_id: str) -> None:
        seq = self.requests.pop(request_id, None)
        if seq is not None and not seq.finished:
            while seq.output_ids and seq.output_ids[-1] == PENDING:  # tokens of in-flight steps are void now
                seq.output_ids.pop()
            self.sched.finish(seq, "abort")

    def has_unfinished(self) -> bool:
        return self.sched.has_work()

    @property
    def num_running(self) -> int:
        return len(self.sched.running)

    @property
    def num_waiting(self) -> int:
        return len(self.sched.waiting)

    # ------------------------------------------------------------------------------------------------------------
    def step(self) -> list[StepOutput]:
        """Run one engine iteration and return the tokens it produced.

        With ``async_scheduling`` the GPU always has the NEXT step queued behind the one being waited on: step n+1 is
        planned on the host (scheduling, page allocation, block tables, attention work items) and LAUNCHED while step
        n still runs, then step n is collected. Decode rows of n+1 whose input token is being sampled by n carry a
        PENDING placeholder; the runner copies those ids device-side from n's sampler output, so the host never waits
        for a token before enqueueing the next forward. Rows planned for sequences that then finish at n (EOS, stop
        string, abort) compute one void token that is discarded; sequences that will finish by length are left out of
        speculative plans up front. Penalties and grammar masks run inside the sampler kernel (engine/logits_proc.py):
        a grammar-constrained row whose next mask depends on a token still in flight sits out ONE plan-ahead step
        (the others keep the pipeline); a token the grammar forces is known at launch and written at once. A plan
        that would have to preempt is redone synchronously. TP leaders plan ahead too: their followers sample the
        same ids on their own GPUs."""
        if self.fi.active:
            self.fi.on_step()
        cut: list[StepOutput] = []
        if self._inflight is None:
            t_p = time.perf_counter()
            with trace.span("schedule"):
                batch = self.sched.schedule()
                cut = self._cut_outputs(batch)
                if batch.empty:
                    return cut
                host, sampled = self.runner.build_host(batch)
            self.host_s["plan"] += time.perf_counter() - t_p
            self._inflight = self._launch(batch, host, sampled, None)
        cur = self._inflight
        self._inflight = None
        plan = None
        if self.cfg.async_scheduling:
            t_p = time.perf_counter()
            with trace.span("plan_ahead"):
                plan = self._speculate()
            self.host_s["plan"] += time.perf_counter() - t_p
        if plan is not None and not self._needs_landed(plan.sampled):
            self.stats["planned_ahead"] += 1
            self._inflight = self._launch(plan.batch, plan.host, plan.sampled, cur)
            plan = None
        outs = cut + self._finish_step(cur)
        if plan is not None:
            if plan.n_added != self._n_added or any(s.finished for s in plan.seqs):
                self.stats["replans"] += 1  # dropped: the next call plans again with the landed tokens
            else:  # planned while n ran, launched after it landed: the GPU idles for the launch
                self.stats["planned_late"] += 1
                self._inflight = self._launch(plan.batch, plan.host, plan.sampled, None)
        return outs

    def step_lockstep(self, agree, flag: int = 0, extra: tuple = ()) -> tuple[list[StepOutput], int, int, tuple]:
        """One DP-attention group step: EXACTLY one forward on every rank of the group (an expert-only idle step on
        a rank without tokens), so the per-layer all-to-alls line up. ``agree((tokens, unfinished, flag, *extra))``
        returns the group maxima; the largest step sets the all-to-all capacity. Returns (outputs, group max
        unfinished — 0: every rank is idle, group max flag — e.g. a stop request seen by any rank, group maxima of
        ``extra``).

        With ``async_scheduling`` (default) it pipelines like ``step``: the NEXT step is planned (speculatively, its
        decode inputs PENDING), agreed and launched while the previous one is still on the GPU, then the previous
        one is collected — the host never waits for the GPU between group steps, and the agreement itself is a
        shared-memory exchange (engine/dp_attention.py)."""
        cut: list[StepOutput] = []
        batch = host = sampled = None
        if self._inflight is None or not self.cfg.async_scheduling:
            batch = self.sched.schedule()
            cut = self._cut_outputs(batch)
            if not batch.empty:
                host, sampled = self.runner.build_host(batch)
        else:
            with trace.span("plan_ahead"):
                plan = self._speculate()
            if plan is not None:
                batch, host, sampled = plan.batch, plan.host, plan.sampled
        T = host.T if host is not None else 0
        got = agree((T, int(self.has_unfinished()), int(flag)) + tuple(extra))
        t_max, busy, fl, ext = got[0], got[1], got[2], tuple(got[3:])
        cur, self._inflight = self._inflight, None
        if t_max > 0:
            # the all-to-all capacity: the group's largest step, bucketed to a power of two so captured decode graphs
            # (keyed by it) are reused across steps; every rank derives the same value from the agreed maximum
            self.model.ep_t_cap = 1 << max(3, (t_max - 1).bit_length())
            self.stats["group_steps"] = self.stats.get("group_steps", 0) + 1
            if host is None:
                with trace.span("dp_idle_step"):
                    self.model.dp_idle_step()
            else:
                if cur is not None:
                    self.stats["planned_ahead"] += 1
                self._inflight = self._launch(batch, host, sampled, cur)
        outs = cut + (self._finish_step(cur) if cur is not None else [])
        if not self.cfg.async_scheduling and self._inflight is not None:
            nxt, self._inflight = self._inflight, None
            outs += self._finish_step(nxt)
        return outs, busy, fl, ext

    @staticmethod
    def _needs_landed(sampled: list[Sequence]) -> bool:
        """True if a row's grammar state would read a token that is still PENDING and cannot be speculated past (the
        speculative scheduler leaves such rows out by the same predicate, so this only guards the invariant;
        penalties are device-side and never need landed tokens)."""
        for s in sampled:
            if s.params.allowed_tokens_fn is not None and not Scheduler._grammar_plannable(s):
                return True
        return False

    def _launch(self, batch, host, sampled: list[Sequence], prev: "_InFlight | None") -> "_InFlight":
        t0 = time.perf_counter()
        with trace.span("launch", B=host.B, T=host.T):
            launched = self.runner.launch(host, sampled, prev.launched if prev is not None else None)
        self.host_s["launch"] += time.perf_counter() - t0
        # advance computed counts + register completed pages in the prefix tree (the step's KV writes are ordered
        # before any later reader on the stream); the sampled tokens are pending until the step lands
        for s in batch.decode:
            s.num_computed = s.total_len
        for s, a, b in batch.prefill:
            s.num_computed = b
        for s in batch.decode:
            self.kvm.commit(s.seq_id, s.num_computed)
        for s, a, b in batch.prefill:
            self.kvm.commit(s.seq_id, s.num_computed)
        slots = []
        known = launched.known or {}
        for i, s in enumerate(sampled):
            slots.append(len(s.output_ids))
            s.output_ids.append(known.get(i, PENDING))  # a grammar-forced token is known now; others land later
        return _InFlight(sampled, slots, launched, t0)

    def _finish_step(self, cur: "_InFlight") -> list[StepOutput]:
        t_w = time.perf_counter()
        with trace.span("collect"):
            toks = self.runner.collect(cur.launched)
        now = time.perf_counter()
        self.host_s["wait"] += now - t_w
        if now - self._t_done < 1.0:  # back-to-back steps: the interval is this GPU's step time
            self.step_ms.append((now - self._t_done) * 1e3)
        self._t_done = now
        self.stats["step_time"] += now - cur.t0
        self.stats["steps"] += 1
        outs: list[StepOutput] = []
        for s, idx, t in zip(cur.sampled, cur.slots, toks):
            if s.finished:  # ended (stop / abort) while this step was in flight: its row was void
                continue
            rb = getattr(s.params.allowed_tokens_fn, "rollback_at", None)
            if rb is not None and rb(s.output_ids, idx):
                # drawn under a grammar mask that was planned on a wrong guess about the previous (then pending)
                # token: discard it and recompute the last position (its KV write was correct: the input token was
                # the real one, gathered on the device)
                del s.output_ids[idx:]
                s.num_computed = s.total_len - 1
                if s.params.presence_penalty or s.params.frequency_penalty:
                    self.runner.lp.uncount(s, t)  # the sampler counted it on the device
                self.stats["grammar_rollbacks"] = self.stats.get("grammar_rollbacks", 0) + 1
                continue
            s.output_ids[idx] = t
            self.kvm.append_token(s.seq_id, t)
            if s.first_token_time is None:
                s.first_token_time = now
                self.stats["prompt_tokens"] += len(s.prompt_ids)
                self.stats["cached_tokens"] += s.num_cached
            s.last_token_time = now
            self.stats["output_tokens"] += 1
            n_out = idx + 1
            reason = self._check_stop(s, t, n_out)
            if reason:
                del s.output_ids[n_out:]  # rows already planned past the end
                self.sched.finish(s, reason)
                self.requests.pop(s.request_id, None)
                trace.request_span(s, now)
            outs.append(StepOutput(s.request_id, [t], reason is not None, reason, len(s.prompt_ids), n_out,
                                   s.num_cached))
        self.host_s["finish"] += time.perf_counter() - now
        return outs

    def _cut_outputs(self, batch) -> list[StepOutput]:
        outs = []
        for s in batch.cut:
            self.requests.pop(s.request_id, None)
            outs.append(StepOutput(s.request_id, [], True, "length", len(s.prompt_ids), len(s.output_ids),
                                   s.num_cached))
        return outs

    def _speculate(self) -> _Plan | None:
        try:
            batch = self.sched.schedule(speculative=True)
        except NeedSync:
            return None
        if batch.empty:
            return None
        host, sampled = self.runner.build_host(batch)
        seqs = list(batch.decode) + [s for s, _, _ in batch.prefill]
        return _Plan(batch, host, sampled, seqs, self._n_added)

    def _check_stop(self, s: Sequence, t: int, n_out: int) -> str | None:
        p = s.params
        if not p.ignore_eos and t in self.eos:
            return "stop"
        if t in p.stop_token_ids:
            return "stop"
        if s.stop_checker is not None and s.stop_checker(t):
            return "stop"
        if n_out >= p.max_tokens:
            return "length"
        if len(s.prompt_ids) + n_out >= self.cfg.max_model_len:
            return "length"
        return None

    # ------------------------------------------------------------------------------------------------------------
    def generate(self, prompts: list[list[int]], params: SamplingParams | list[SamplingParams]) -> list[list[int]]:
        """Blocking helper: run prompts to completion, return output token ids (tests, smoke, offline use)."""
        ps = params if isinstance(params, list) else [params] * len(prompts)
        ids = [f"gen-{time.perf_counter_ns()}-{i}" for i in range(len(prompts))]
        seqs = [self.add_request(i, p, sp) for i, p, sp in zip(ids, prompts, ps)]
        while any(not s.finished for s in seqs):
            self.step()
        return [s.output_ids for s in seqs]

    def pin_prefix(self, token_ids: list[int]) -> int:
        """Hold the cached pages of ``token_ids`` (e.g. the shared Kafka system prompt + tool schemas) so LRU eviction
        under KV pressure never drops them (SURVEY.md §2.8 "pinned hot prefix"). Returns the number of pinned tokens
        (whole pages that are already in the prefix cache); ``unpin_prefix`` releases them."""
        self.unpin_prefix()
        sid = -(1 << 40)  # outside the id range of real sequences
        n = self.kvm.add_sequence(sid, list(token_ids) + [0])  # + sentinel: a full last page can match too
        self._pinned = sid
        return n

    def unpin_prefix(self) -> None:
        sid = getattr(self, "_pinned", None)
        if sid is not None and self.kvm.has_seq(sid):
            self.kvm.free_sequence(sid)
        self._pinned = None

    def perf_stats(self) -> dict:
        """Per-GPU step time (quantiles over the last <= 512 busy steps) and, with an IPC collective (TP custom
        all-reduce / DP-attention all-to-all), its time per call and per step (the kernels' own
        clock stamps: graph replays included)."""
        d: dict = {"device": str(self.device), "steps": self.stats["steps"]}
        if self.step_ms:
            xs = sorted(self.step_ms)
            q = lambda f: xs[min(len(xs) - 1, int(f * len(xs)))]  # noqa: E731
            d.update(step_ms_mean=round(sum(xs) / len(xs), 3), step_ms_p50=round(q(0.5), 3),
                     step_ms_p99=round(q(0.99), 3))
        car = self.runner._custom_ar() if self.device.type == "cuda" else None
        if car is not None:
            try:
                us, calls = car.timing()
            except Exception:  # noqa: BLE001 - diagnostics only
                us, calls = None, 0
            if us is not None and len(us):
                c0, s0 = self._coll_mark
                steps = self.stats["steps"]
                per_step = (calls - c0) / (steps - s0) if steps > s0 else 0.0
                self._coll_mark = (calls, steps)
                d.update(collective_calls=calls, collective_us_per_call=round(float(us.mean()), 2),
                         collective_calls_per_step=round(per_step, 2),
                         collective_ms_per_step=round(float(us.mean()) * per_step / 1e3, 3))
        return d

    def kv_stats(self) -> dict:
        d = dict(self.kvm.stats())
        d["num_blocks"] = self.num_blocks
        return d
