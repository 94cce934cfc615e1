"""Custom one-shot all-reduce (csrc/allreduce.hip) and a TP=2 engine on a 1-GPU box.

RCCL refuses two ranks on one device, but the custom all-reduce's protocol (IPC-mapped uncached buffers, per-block
device epochs, flags, parity halves, system-coherent loads) is the same between two processes that share a GPU as
between two GPUs: the ranks here run on ``cuda:(rank % device_count)`` with a gloo control group, and every result
is checked against a gloo/CPU reference of the same sum. The engine test runs a TP=2 group on one GPU — custom
all-reduce on every layer seam (fused with the residual add and the next RMSNorm), gloo for the logit all-gather —
against the TP=1 model."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port, local):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(local)})


def _gloo_sum(t, group):
    import torch.distributed as dist

    h = t.float().cpu()
    dist.all_reduce(h, group=group)
    return h


def _ar_main(rank, world, port, q):
    dev = rank % torch.cuda.device_count()
    _env(rank, world, port, dev)
    import torch.distributed as dist

    from kafka_llm_service_amd import ops
    from kafka_llm_service_amd.parallel.custom_allreduce import CustomAllReduce

    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group(list(range(world)), backend="gloo")
    car = CustomAllReduce(grp, rank, world, max_bytes=4 << 20)
    errs = {}
    # 1. bf16 in place, several sizes, three calls each (epochs advance on the device)
    for n in (8, 4096 * 8, 64 * 8192, 1 << 20):
        for it in range(3):
            g = torch.Generator(device="cuda").manual_seed(1000 * n + 10 * it + rank)
            x = torch.randn(n, device="cuda", generator=g).to(torch.bfloat16)
            ref = _gloo_sum(x, grp)
            car.all_reduce(x)
            torch.cuda.synchronize()
            errs[f"bf16 n={n} it={it}"] = ((x.float().cpu() - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
    # 2. fp32 split-K slab input [S, T, d] -> bf16 [T, d]
    g = torch.Generator(device="cuda").manual_seed(77 + rank)
    slab = torch.randn(4, 64, 4096, device="cuda", generator=g)
    ref = _gloo_sum(slab.sum(0).to(torch.bfloat16), grp)
    y = car.all_reduce(slab)
    torch.cuda.synchronize()
    errs["slab"] = ((y.float().cpu() - ref).abs().max() / ref.abs().max()).item()
    # 3. fused seam: residual += allreduce(x); out = rmsnorm(residual) * w
    for T, d in ((64, 4096), (5, 8192), (130, 1024)):
        g = torch.Generator(device="cuda").manual_seed(5 * T + d)
        resid = torch.randn(T, d, device="cuda", generator=g).to(torch.bfloat16)  # same on both ranks
        w = torch.randn(d, device="cuda", generator=g).to(torch.bfloat16)
        x = (torch.randn(T, d, device="cuda", generator=g) + rank).to(torch.bfloat16)
        r_ref = resid.clone()
        o_ref = ops.fused_add_rmsnorm(_gloo_sum(x, grp).to(torch.bfloat16).cuda(), r_ref, w, 1e-5)
        out = torch.empty_like(resid)
        car.all_reduce_add_rmsnorm(x, resid, w, 1e-5, out)
        torch.cuda.synchronize()
        errs[f"fused T={T} d={d} resid"] = ((resid.float() - r_ref.float()).abs().max() / r_ref.abs().max()).item()
        errs[f"fused T={T} d={d} out"] = ((out.float() - o_ref.float()).abs().max() / o_ref.abs().max()).item()
    # 4. hipGraph: two all-reduces captured once, replayed with fresh inputs (device-side epochs advance)
    xs = torch.zeros(64 * 1024, device="cuda", dtype=torch.bfloat16)
    ys = torch.zeros(64 * 1024, device="cuda", dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up (real calls: both ranks take part)
        car.all_reduce(xs)
        car.all_reduce(ys)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        car.all_reduce(xs)
        car.all_reduce(ys)
    for it in range(3):
        g = torch.Generator(device="cuda").manual_seed(900 + 7 * it + rank)
        a = torch.randn(xs.numel(), device="cuda", generator=g).to(torch.bfloat16)
        b = torch.randn(ys.numel(), device="cuda", generator=g).to(torch.bfloat16)
        ra, rb = _gloo_sum(a, grp), _gloo_sum(b, grp)
        xs.copy_(a)
        ys.copy_(b)
        graph.replay()
        torch.cuda.synchronize()
        errs[f"graph it={it}"] = max(((xs.float().cpu() - ra).abs().max() / ra.abs().max()).item(),
                                     ((ys.float().cpu() - rb).abs().max() / rb.abs().max()).item())
    torch.cuda.synchronize()
    timed_out = False
    try:
        car.check()
    except RuntimeError:
        timed_out = True
    car.close()
    q.put((rank, errs, timed_out))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_custom_allreduce_protocol():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_ar_main, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, errs, timed_out = q.get(timeout=240)
        res[r] = (errs, timed_out)
    for p in ps:
        p.join(timeout=60)
    for r, (errs, timed_out) in res.items():
        assert not timed_out, f"rank {r}: a peer wait timed out"
        bad = {k: v for k, v in errs.items() if v > 0.02}
        assert not bad, f"rank {r}: {bad}"


CFG = dict(model="small-llama", num_kv_blocks=1024, max_model_len=4096)


def _prompts(vocab):
    g = torch.Generator().manual_seed(21)
    pre = torch.randint(0, vocab, (300,), generator=g).tolist()
    return [pre + torch.randint(0, vocab, (n,), generator=g).tolist() for n in (3, 60, 150)]


def _capture_logits(eng, prompts, sp):
    seen = []
    orig = eng.runner.sample_device

    def sample_device(logits, p):
        seen.append(logits.float().cpu())
        return orig(logits, p)

    eng.runner.sample_device = sample_device
    outs = eng.generate(prompts, sp)
    eng.runner.sample_device = orig
    return outs, seen


def _tp_main(rank, world, port, q, graphs, model):
    dev = rank % torch.cuda.device_count()
    _env(rank, world, port, dev)
    os.environ["KAFKA_TP_BACKEND"] = "gloo"
    if model.endswith("+a2a"):  # experts dispatched / combined by all-to-all instead of the all-reduce combine
        os.environ["KAFKA_MOE_A2A"] = "1"
    if model.endswith("+overlap"):  # O / down projections in column halves pipelined against their all-reduces
        os.environ["KAFKA_TP_OVERLAP"] = "1"
        model = model.replace("+overlap", "")
    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.engine.sequence import SamplingParams
    from kafka_llm_service_amd.parallel import comm
    from kafka_llm_service_amd.parallel import state as pstate

    eng, st = tp_worker.build_tp_engine(dict(CFG, model=model.replace("+a2a", ""), device=f"cuda:{dev}",
                                             use_graphs=graphs), tp=world)
    a2a_calls = [0]
    if model.endswith("+a2a"):
        # the whole MoE block — router, device routing, EP dispatch, IPC all-to-all, expert GEMMs, return, combine,
        # all-gather — must never synchronise with the host: torch raises on any sync
        from kafka_llm_service_amd.models.moe import MoEBlock

        orig_call = MoEBlock.__call__

        def checked(self, x, lw):
            if torch.cuda.is_current_stream_capturing():
                return orig_call(self, x, lw)
            torch.cuda.set_sync_debug_mode("error")
            try:
                return orig_call(self, x, lw)
            finally:
                torch.cuda.set_sync_debug_mode("default")
                a2a_calls[0] += 1
        MoEBlock.__call__ = checked
    if os.environ.get("KAFKA_TP_OVERLAP") == "1":
        from kafka_llm_service_amd.models.llama import TransformerLM

        orig_seam = TransformerLM._overlapped_seam

        def counted(self, *a, **kw):
            a2a_calls[0] += 1  # the overlapped seam ran (eager, or recorded into a graph)
            return orig_seam(self, *a, **kw)
        TransformerLM._overlapped_seam = counted
    try:
        assert os.environ.get("KAFKA_CUSTOM_AR", "1") == "0" or comm.get_custom(st.tp_group) is not None, \
            "custom all-reduce not registered"
        if st.is_tp_leader:
            sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
            outs, seen = _capture_logits(eng, _prompts(eng.model_cfg.vocab_size), sp)
            tp_worker.release_followers()
            g = eng.runner.graphs
            q.put(("leader", outs, [s.numpy() for s in seen], g.stats if g is not None else None,
                   eng.stats["planned_ahead"], a2a_calls[0], eng.perf_stats()))
        else:
            n = tp_worker.follower_loop(eng)
            q.put(("follower", n, a2a_calls[0]))
        if comm.get_custom(st.tp_group) is not None:
            comm.get_custom(st.tp_group).check()
    finally:
        pstate.destroy()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,graphs", [("small-llama", False), ("small-llama", True), ("tiny-mixtral", False),
                                          ("tiny-mixtral+a2a", False), ("tiny-mixtral+a2a", True),
                                          ("small-llama+overlap", False), ("small-llama+overlap", True)],
                         ids=["eager", "graphs", "mixtral-ep", "mixtral-ep-a2a", "mixtral-ep-a2a-graphs",
                              "overlap", "overlap-graphs"])
def test_tp2_engine_on_one_gpu_matches_tp1(cuda, model, graphs):
    """TP=2 (Mixtral: experts sharded over the 2 ranks, EP) on one GPU == the TP=1 model: same first-step logits up
    to reduction order, every greedy token the dense oracle's argmax."""
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_tp_main, args=(r, 2, port, q, graphs, model)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        m = q.get(timeout=240)
        res[m[0]] = m[1:]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs, seen, gstats, ahead, a2a_lead, perf = res["leader"]
    assert res["follower"][0] >= 6 and ahead > 0
    if os.environ.get("KAFKA_CUSTOM_AR", "1") == "1":  # collective time from the kernels' clock stamps
        assert perf.get("collective_us_per_call", 0) > 0 and perf.get("collective_calls_per_step", 0) > 0, perf
    if graphs:
        assert gstats["replays"] >= 1
    if model.endswith(("+a2a", "+overlap")):  # eager MoE calls under sync-debug "error" / overlapped seams ran
        assert a2a_lead > 0 and res["follower"][1] > 0
    ref = LLMEngine(EngineConfig(**dict(CFG, model=model.replace("+a2a", "").replace("+overlap", ""),
                                        device="cuda:0")))
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    want_outs, want = _capture_logits(ref, _prompts(ref.model_cfg.vocab_size), sp)
    # first step (prefill of all prompts, identical batches): the TP=2 logits equal TP=1 up to bf16 reduction order
    got0, want0 = torch.from_numpy(seen[0]), want[0]
    assert got0.shape == want0.shape
    assert (got0 - want0).abs().max().item() < 0.05 * want0.abs().max().item() + 0.05
    from kafka_llm_service_amd.models.oracle import dense_logits

    for p, o in zip(_prompts(ref.model_cfg.vocab_size), outs):  # every TP=2 token is the TP=1 model's argmax
        lg = dense_logits(ref.model, p + o)
        for i, tok in enumerate(o):
            row = lg[len(p) - 1 + i]
            assert (row.max() - row[tok]).item() < 0.15


def _tp_skip_main(rank, world, port, q):
    dev = rank % torch.cuda.device_count()
    _env(rank, world, port, dev)
    os.environ["KAFKA_TP_BACKEND"] = "gloo"
    if rank == 1:  # the follower stops taking part in one layer-seam all-reduce (a peer that never arrives)
        os.environ["KAFKA_FI_CAR_SKIP_CALL"] = "20"
    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.engine.model_runner import CollectiveError
    from kafka_llm_service_amd.engine.sequence import SamplingParams
    from kafka_llm_service_amd.parallel import state as pstate
    from kafka_llm_service_amd.utils import faults

    faults.reset()
    eng, st = tp_worker.build_tp_engine(dict(CFG, device=f"cuda:{dev}", use_graphs=False), tp=world)
    try:
        if st.is_tp_leader:
            sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
            try:
                eng.generate(_prompts(eng.model_cfg.vocab_size), sp)
                q.put(("leader", "finished without an error"))
            except CollectiveError as e:
                q.put(("leader", f"raised: {e}"))
            tp_worker.release_followers()
        else:
            tp_worker.follower_loop(eng)
            q.put(("follower", "done"))
    finally:
        pstate.destroy()


@pytest.mark.timeout(300)
def test_tp2_custom_allreduce_lost_peer_fails_the_step(cuda):
    """A TP peer that skips a custom all-reduce call makes the leader's wait time out (2 s): the error word rides
    back with the step's sampled ids and the engine raises CollectiveError (replica failure -> 503 + respawn) instead
    of streaming tokens computed from stale peer data (VERDICT r02 Missing #5)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_tp_skip_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        m = q.get(timeout=240)
        res[m[0]] = m[1]
    for p in ps:
        p.join(timeout=60)
    assert res["leader"].startswith("raised"), res["leader"]


def _dpa_gpu_main(rank, world, port, q, layout, graphs=False):
    dev = rank % torch.cuda.device_count()
    _env(rank, world, port, dev)
    os.environ["KAFKA_TP_BACKEND"] = "gloo"
    from kafka_llm_service_amd.engine import dp_attention
    from kafka_llm_service_amd.engine.sequence import SamplingParams
    from kafka_llm_service_amd.models.moe import MoEBlock
    from kafka_llm_service_amd.parallel import comm
    from kafka_llm_service_amd.parallel import state as pstate

    calls = [0]
    for name in ("__call__", "serve_idle"):  # no host sync anywhere in a MoE layer, busy or idle
        orig = getattr(MoEBlock, name)

        def checked(self, *a, _orig=orig, **kw):
            torch.cuda.set_sync_debug_mode("error")
            try:
                return _orig(self, *a, **kw)
            finally:
                torch.cuda.set_sync_debug_mode("default")
                calls[0] += 1
        setattr(MoEBlock, name, checked)
    eng, st = dp_attention.build_dpa_engine(dict(CFG, model="tiny-mixtral", device=f"cuda:{dev}", use_graphs=graphs),
                                            ep=world)
    try:
        assert comm.get_custom(st.ep_group) is not None, "IPC all-to-all not registered on the EP group"
        mine = [p for i, p in enumerate(_prompts(eng.model_cfg.vocab_size))
                if (i % world if layout == "spread" else 0) == rank]
        sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
        outs = dp_attention.generate_lockstep(eng, st, mine, sp)
        comm.get_custom(st.ep_group).check()
        g = eng.runner.graphs
        q.put((rank, outs, eng.stats["group_steps"], calls[0], g.stats["replays"] if g is not None else 0,
               eng.stats["planned_ahead"]))
    finally:
        pstate.destroy()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("layout,graphs", [("spread", False), ("one_idle", False), ("spread", True)],
                         ids=["spread", "one_idle", "spread_graphs"])
def test_dp_attention_mixtral_on_one_gpu(cuda, layout, graphs):
    """Mixtral with data-parallel attention, EP = 2 over two processes on one GPU: each rank decodes its own
    sequences (or none), every MoE layer exchanges rows through the device-side dispatch + IPC all-to-all without
    a host sync, and every greedy token is the EP = 1 model's argmax up to bf16 rounding."""
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.models.oracle import dense_logits

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_dpa_gpu_main, args=(r, 2, port, q, layout, graphs)) for r in range(2)]
    for p in ps:
        p.start()
    res = {m[0]: m[1:] for m in (q.get(timeout=240) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] and res[0][2] > 0 and res[1][2] > 0
    assert res[0][4] > 0  # the group planned ahead (pipelined lockstep)
    if graphs:
        assert res[0][3] > 0 and res[1][3] > 0  # decode steps replayed from captured graphs on both ranks
    ref = LLMEngine(EngineConfig(**dict(CFG, model="tiny-mixtral", device="cuda:0")))
    prompts = _prompts(ref.model_cfg.vocab_size)
    for r in (0, 1):
        mine = [p for i, p in enumerate(prompts) if (i % 2 if layout == "spread" else 0) == r]
        assert len(res[r][0]) == len(mine)
        for p, o in zip(mine, res[r][0]):
            lg = dense_logits(ref.model, p + o)
            for i, tok in enumerate(o):
                row = lg[len(p) - 1 + i]
                assert (row.max() - row[tok]).item() < 0.15


def _dpa_skip_main(rank, world, port, q):
    dev = rank % torch.cuda.device_count()
    _env(rank, world, port, dev)
    os.environ["KAFKA_TP_BACKEND"] = "gloo"
    if rank == 1:  # this rank stops taking part in one expert all-to-all (a peer that never arrives)
        os.environ["KAFKA_FI_CAR_SKIP_CALL"] = "12"
    from kafka_llm_service_amd.engine import dp_attention
    from kafka_llm_service_amd.engine.model_runner import CollectiveError
    from kafka_llm_service_amd.engine.sequence import SamplingParams
    from kafka_llm_service_amd.parallel import comm
    from kafka_llm_service_amd.parallel import state as pstate
    from kafka_llm_service_amd.utils import faults

    faults.reset()
    eng, st = dp_attention.build_dpa_engine(dict(CFG, model="tiny-mixtral", device=f"cuda:{dev}"), ep=world)
    try:
        assert comm.get_custom(st.ep_group) is not None
        mine = [p for i, p in enumerate(_prompts(eng.model_cfg.vocab_size)) if i % world == rank]
        sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
        try:
            dp_attention.generate_lockstep(eng, st, mine, sp)
            q.put((rank, "finished without an error"))
        except CollectiveError as e:
            q.put((rank, f"raised: {e}"))
        except Exception as e:  # noqa: BLE001 - e.g. the group's gloo agreement after the other rank failed
            q.put((rank, f"other: {type(e).__name__}"))
    finally:
        os._exit(0)  # no collective teardown with a peer that may have failed


@pytest.mark.timeout(300)
def test_dp_attention_lost_peer_fails_the_step(cuda):
    """with data-parallel attention (tp = 1) the EP group's IPC all-to-all error word must ride back
    with the step's ids like the TP all-reduce's does — a peer that skips one expert all-to-all makes the other
    rank raise CollectiveError instead of streaming tokens built from stale expert rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_dpa_skip_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        while 0 not in res:
            m = q.get(timeout=240)
            res[m[0]] = m[1]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert res[0].startswith("raised"), res
