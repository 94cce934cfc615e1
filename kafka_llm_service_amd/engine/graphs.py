"""hipGraph decode runner (SURVEY.md §2.8 "hipGraph decode runner: capture decode steps per batch-size bucket with
static buffers", §7.4 #7 "hipGraph + dynamic paged metadata").

A decode-only step (B running threads, one token each) launches ~11 kernels per layer — 364 for Llama-3-8B — from
Python. Captured once per LAYOUT as a hipGraph, the whole step (embedding, 32 layers of GEMMs / norms / RoPE+KV
write / cascade + split-K paged attention / merge, final norm, lm_head, sampler) becomes one ``replay``: the CPU
cost drops from ~2 ms to ~20 us, which is what lets the host keep up with short decode steps (small batches, TP
shards) and leaves the CPU free for the API loop.

Layout key: (B, decode work items (padded to a power of two), partial slots, prefix work items, cascade on/off, packed-buffer sizes,
greedy, logits processing on/off). Everything that changes from step to step — token ids, positions, KV slots, block
tables, sequence lengths, cascade work items, sampling parameters, seeds and the rows' logits-processing entries
(grammar mask rows / forced tokens / penalty slots, engine/logits_proc.py: the mask and count tables sit at fixed
addresses) — lives in STATIC device buffers that are refreshed (one async H2D each) before the replay;
intermediates (activations, attention partials, logits) come from a graph memory pool shared by all captured
layouts. Steps with prefill rows run eagerly. Under tensor parallelism every rank captures the same layouts from the same broadcast plans: the graph
ends with this rank's vocab shard of the logits (the layer seams' custom xGMI all-reduces are inside it — their call
counters live in device memory), and the logit all-gather + sampler run eagerly after the replay.

``backend="fake"`` re-runs the captured closure instead of a device graph: on CPU it checks the property a graph
relies on — a replay reads ONLY the static buffers (tests/test_graphs.py).
"""
from __future__ import annotations

import copy
import logging
from collections import OrderedDict

import numpy as np
import torch

from kafka_llm_service_amd import ops

log = logging.getLogger("kafka.graphs")


class _FakeGraph:
    """Graph stand-in: 'capture' runs the closure once, 'replay' runs it again."""

    def __init__(self, fn):
        self.fn = fn
        fn()

    def replay(self) -> None:
        self.fn()


class _Entry:
    __slots__ = ("graph", "s64", "s32", "f32", "topk", "seeds", "out", "layout", "local", "proc", "static", "offs")


class DecodeGraphs:
    def __init__(self, runner, max_graphs: int = 8, backend: str | None = None):
        self.runner = runner
        self.max_graphs = max_graphs
        self.backend = backend or ("cuda" if runner.device.type == "cuda" else "fake")
        self.graphs: OrderedDict[tuple, _Entry] = OrderedDict()
        self.pool = torch.cuda.graph_pool_handle() if self.backend == "cuda" else None
        self.disabled = False
        self.stats = {"captures": 0, "replays": 0}

    def key(self, h, sp) -> tuple:
        # DP attention: the step's all-to-all capacity (agreed by the group, bucketed) is baked into the captured
        # MoE layers, so it is part of the layout
        cap = self.runner.model.ep_t_cap if getattr(self.runner.model, "dp_attention", False) else 0
        return (h.B, h.n_dec_items, h.s_total, h.n_prefix_items, bool(h.cascade_prefix), h.i64.size, h.i32.size,
                h.n_late, h.late_off, sp.greedy, sp.proc is not None, cap)

    def eligible(self, h, sp) -> bool:
        return not self.disabled and h.B > 0 and h.T == h.B and h.n_items == 0

    # ------------------------------------------------------------------------------------------------------------
    def run(self, h, sp) -> torch.Tensor | None:
        k = self.key(h, sp)
        e = self.graphs.get(k)
        if e is None:
            e, local = self._capture(k, h, sp)
            if e is None:  # capture failed on some rank: the warm run already computed this step
                if self.runner.model.tp == 1:
                    return local
                return self._finish_tp(local, h, sp)
        else:
            self.graphs.move_to_end(k)
            self._load(e, h, sp)
            e.graph.replay()
            self.stats["replays"] += 1
            local = e.local
        if self.runner.model.tp == 1:
            return e.out  # sampled inside the graph
        return self._finish_tp(local, h, sp)

    def _finish_tp(self, local: torch.Tensor, h, sp) -> torch.Tensor:
        """After a TP replay: all-gather the vocab shards, sample (every rank, same seeds), leave the ids in tok_buf."""
        from kafka_llm_service_amd.parallel import state as pstate

        r = self.runner
        logits = pstate.tp_all_gather_lastdim(local)[:, :r.vocab]
        toks = r.sample_device(logits, sp)
        r.tok_buf[:toks.shape[0]].copy_(toks)
        return toks

    def _agree(self, ok: bool) -> bool:
        """The TP group's verdict on a capture: True only if it worked on every rank (gloo MIN on the control
        group; one small collective per captured layout, never on a replay)."""
        if self.runner.model.tp == 1:
            return ok
        import torch.distributed as dist

        from kafka_llm_service_amd.parallel import state as pstate

        st = pstate.get()
        if st.cpu_group is None or not dist.is_initialized():
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.cpu_group)
        return bool(int(t.item()))

    def _load(self, e: _Entry, h, sp) -> None:
        # every static input of the graph refreshed by ONE host->device copy into its packed buffer (an upload plus
        # a device copy per input cost ~10 copy kernels and their launch gaps per step)
        sampled = not sp.greedy
        arrays = [np.asarray(h.i64, dtype=np.int64), np.asarray(h.i32, dtype=np.int32),
                  np.concatenate([sp.temp, sp.topp]).astype(np.float32, copy=False) if sampled else None,
                  np.asarray(sp.topk, dtype=np.int32) if sampled else None,
                  np.asarray(sp.seeds, dtype=np.int64) if sampled else None,
                  np.asarray(sp.proc, dtype=np.int32) if sp.proc is not None else None]
        self.runner.stager.upload_into(arrays, e.offs, e.static)

    def _capture(self, k: tuple, h, sp) -> tuple[_Entry, torch.Tensor | None]:
        r = self.runner
        dev = r.device
        n = h.n_rows
        e = _Entry()
        # static inputs: one packed device buffer (256-B aligned views), refreshed by one copy per replay
        parts = [(h.i64.size, torch.int64), (h.i32.size, torch.int32), (2 * n, torch.float32), (n, torch.int32),
                 (n, torch.int64), (n * 8 if sp.proc is not None else 0, torch.int32)]
        e.offs, off = [], 0
        for cnt, dt in parts:
            e.offs.append(off)
            off = (off + cnt * torch.tensor([], dtype=dt).element_size() + 255) & ~255
        e.static = torch.empty(max(off, 256), dtype=torch.uint8, device=dev)
        views = [e.static[o:o + cnt * torch.tensor([], dtype=dt).element_size()].view(dt)
                 for o, (cnt, dt) in zip(e.offs, parts)]
        e.s64, e.s32, e.f32, e.topk, e.seeds = views[:5]
        e.out = torch.empty(n, dtype=torch.int64, device=dev)
        e.proc = views[5].view(n, 8) if sp.proc is not None else None
        kw = dict(r.proc_tables(sp), proc=e.proc) if sp.proc is not None else {}
        e.layout = copy.copy(h)
        e.layout.i64 = e.layout.i32 = None
        e.layout.patch = []
        greedy = sp.greedy
        tp = r.model.tp > 1

        def step():
            inp = r.views(e.s64, e.s32, e.layout)
            if tp:  # the graph ends at this rank's logit shard (see the module docstring)
                e.local = r.model.forward(inp, r.k_caches, r.v_caches, gather=False)
                return
            logits = r.model.forward(inp, r.k_caches, r.v_caches)
            if greedy:
                toks = ops.sample(logits, torch.zeros(n, device=dev), **kw)
            else:
                toks = ops.sample(logits, e.f32[:n], e.f32[n:], e.topk, e.seeds, **kw)
            e.out.copy_(toks)
            r.tok_buf[:n].copy_(toks)  # input ids of the next step's late rows (ModelRunner.views)

        self._load(e, h, sp)
        e.local = None
        if self.backend == "fake":
            e.graph = _FakeGraph(step)
            warm = e.local
        else:
            # warm up on a side stream (library workspaces, lazy inits): this run computes THIS step (tokens and
            # its KV writes, and under TP its collectives — a failure here is a failed step, raised as such); the
            # capture pass that follows records the kernels without executing them
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                step()
            torch.cuda.current_stream().wait_stream(side)
            warm = e.local  # this step's logit shard (TP); the capture pass below only records
            ok = True
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.pool):
                    step()
                e.graph = g
            except Exception:  # noqa: BLE001 - never let capture problems take the engine down
                log.exception("hipGraph capture failed")
                ok = False
            if not self._agree(ok):
                # Every rank of the TP group switches to eager decode on the same step (a rank alone would make
                # collective calls its peers never match). The step itself is NOT run again — the warm run already
                # computed it (its tokens, KV writes and, under TP, its collectives): return that result.
                log.warning("hipGraph decode disabled for this engine (capture failed on some rank)")
                self.disabled = True
                return None, (e.out if r.model.tp == 1 else warm)
        self.graphs[k] = e
        self.stats["captures"] += 1
        while len(self.graphs) > self.max_graphs:
            self.graphs.popitem(last=False)
        return e, warm
