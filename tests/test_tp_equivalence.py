"""Tensor parallelism on CPU (gloo, world_size 2, 127.0.0.1): a TP=2 engine group — leader schedules and broadcasts
step plans, follower mirrors them, per-layer all-reduces + vocab-parallel logit all-gather over the group — computes
the same function as TP=1 (SURVEY.md §4.4 "Distributed: TP=2/4/8 logits == TP=1")."""
import asyncio
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.models.oracle import dense_logits

CFG = dict(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048)
GREEDY = SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True)


def _prompts(long: bool = False):
    g = torch.Generator().manual_seed(11)
    pre = torch.randint(0, 5000, (700 if long else 48,), generator=g).tolist()
    return [pre + torch.randint(0, 5000, (n,), generator=g).tolist() for n in (3, 21, 40)]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _group_main(rank: int, world: int, port: int, q, extra: dict) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(rank)})
    extra = dict(extra)
    os.environ.update(extra.pop("_env", {}))
    proc = extra.pop("_proc", False)
    long = extra.pop("_long", False)
    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.parallel import state as pstate

    eng, st = tp_worker.build_tp_engine(dict(CFG, **extra), tp=world)
    try:
        if st.is_tp_leader:
            outs = eng.generate(_prompts(long), _proc_params() if proc else GREEDY)
            tp_worker.release_followers()
            g = eng.runner.graphs
            q.put(("outs", outs, eng.num_blocks, eng.stats["planned_ahead"], g.stats if g is not None else None))
        else:
            n = tp_worker.follower_loop(eng)
            g = eng.runner.graphs
            q.put(("follower_steps", n, g.stats if g is not None else None))
    finally:
        pstate.destroy()


TOOLS = [{"type": "function", "function": {"name": "get_weather", "parameters": {
    "type": "object", "required": ["location"], "properties": {"location": {"type": "string"}}}}}]


def _proc_params():
    """Per-prompt params with device-side logits processing: a grammar-constrained tool call, penalties, plain."""
    return [SamplingParams(temperature=0.0, max_tokens=60, ignore_eos=True,
                           tool_grammar={"tools": TOOLS, "tool_choice": "required"}),
            SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True, frequency_penalty=0.5,
                           presence_penalty=0.5),
            GREEDY]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("extra", [{}, {"use_graphs": True}, {"_env": {"KAFKA_PLAN_CHANNEL": "gloo"}},
                                   {"_env": {"KAFKA_PLAN_SLOT_BYTES": "1024"}}, {"_long": True}],
                         ids=["eager", "graphs", "gloo_channel", "oversized_plans", "pipelined_prefill_seams"])
def test_tp2_generate_matches_tp1(extra):
    """Leader plans step n+1 while n runs (late decode inputs filled device-side on EVERY rank from its own sampler
    output); with ``use_graphs`` every rank captures and replays the decode layouts (fake graph backend on CPU:
    replays read only the static buffers) and samples after the logit all-gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_group_main, args=(r, 2, port, q, extra)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((m[0], m[1:]) for m in (q.get(timeout=240) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs, nb, ahead, gstats = res["outs"]
    assert res["follower_steps"][0] >= GREEDY.max_tokens and nb == 256
    assert ahead > 0  # TP leaders plan ahead
    if extra.get("use_graphs"):
        assert gstats["replays"] >= 1 and res["follower_steps"][1]["replays"] == gstats["replays"]
    ref = LLMEngine(EngineConfig(**CFG))
    prompts = _prompts(extra.get("_long", False))  # _long: a 2 x 700-token prefill step -> GEMM || all-reduce blocks
    # TP=2 reduces in a different order (bf16): tokens must be the TP=1 model's argmax up to a small logit margin
    for p, o in zip(prompts, outs):
        lg = dense_logits(ref.model, p + o)
        for i, tok in enumerate(o):
            row = lg[len(p) - 1 + i]
            assert (row.max() - row[tok]).item() < 0.05


def _capture_logits(eng, prompt):
    """Run one prefill step through the engine and return the logits the sampler saw."""
    seen = []
    orig = eng.runner.sample_device

    def sample_device(logits, sp):
        seen.append(logits.float().clone())
        return orig(logits, sp)

    eng.runner.sample_device = sample_device
    eng.generate([prompt], SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
    eng.runner.sample_device = orig
    return torch.cat(seen)


def _logits_main(rank: int, world: int, port: int, q, model: str) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(rank)})
    if model.endswith("+a2a"):  # expert all-to-all dispatch/combine instead of the all-reduce combine
        os.environ["KAFKA_MOE_A2A"] = "1"
        model = model[:-4]
    from kafka_llm_service_amd.engine import tp_worker
    from kafka_llm_service_amd.parallel import state as pstate

    eng, st = tp_worker.build_tp_engine(dict(CFG, model=model), tp=world)
    try:
        if st.is_tp_leader:
            lg = _capture_logits(eng, _prompts()[1])
            tp_worker.release_followers()
            q.put(lg.float().numpy())  # numpy pickles by value: no fd hand-off that dies with this process
        else:
            tp_worker.follower_loop(eng)
    finally:
        pstate.destroy()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral", "tiny-mixtral+a2a"])
def test_tp2_logits_close_to_tp1(model):
    """Dense: Megatron TP=2. Mixtral: attention TP=2 + expert parallel EP=2 over the same group, with the
    all-reduce combine or the all-to-all dispatch/combine (+a2a)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_logits_main, args=(r, 2, port, q, model)) for r in range(2)]
    for p in procs:
        p.start()
    got = torch.from_numpy(q.get(timeout=240))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _capture_logits(LLMEngine(EngineConfig(**dict(CFG, model=model.replace("+a2a", "")))), _prompts()[1])
    assert got.shape == want.shape
    assert torch.allclose(got, want, atol=3e-2, rtol=0), (got - want).abs().max()


@pytest.mark.timeout(300)
def test_dp_client_with_tp_groups():
    """The server's engine client: 1 replica x TP=2 processes, requests through the leader's pipe."""
    from kafka_llm_service_amd.engine.client import DPClient

    cli = DPClient(EngineConfig(**CFG), 1, tp=2)

    async def run():
        outs = []
        for i, p in enumerate(_prompts()[:2]):
            toks = []
            async for o in cli.generate(f"r{i}", p, GREEDY, routing_key="t"):
                toks += o.new_token_ids
            outs.append(toks)
        h = cli.health()
        await cli.close()
        return outs, h

    outs, h = asyncio.run(run())
    assert [len(o) for o in outs] == [5, 5] and h["replicas"] == 1


def test_plan_wire_format_roundtrip():
    import numpy as np

    from kafka_llm_service_amd.engine.model_runner import HostStep, SampleParams, pack_plan, unpack_plan

    h = HostStep(B=3, T=40, nbt=4, bt_w=32, n_rows=4, s_total=5, n_dec_items=6, n_prefix_items=2, cascade_prefix=512,
                 n_items=1, prefill_splits=0, n_late=2, late_off=123)
    h.i64 = np.arange(125, dtype=np.int64)
    h.i32 = np.arange(4 * 32 + 77, dtype=np.int32)
    from kafka_llm_service_amd.engine.logits_proc import ProcUpdates

    sp = SampleParams(np.array([0.7, 0, 1, 2], np.float32), np.ones(4, np.float32), np.array([0, 5, 0, 1], np.int32),
                      np.array([1, 2, 3, 1 << 40], np.int64), None, False)
    hdr, payload = pack_plan(h, sp)
    h2, sp2 = unpack_plan(hdr, payload)
    for f in ("B", "T", "nbt", "bt_w", "n_rows", "s_total", "n_dec_items", "n_prefix_items", "cascade_prefix",
              "n_items", "prefill_splits", "n_late", "late_off"):
        assert getattr(h2, f) == getattr(h, f), f
    assert (h2.i64 == h.i64).all() and (h2.i32 == h.i32).all()
    for f in ("temp", "topp", "topk", "seeds"):
        assert (getattr(sp2, f) == getattr(sp, f)).all()
    assert sp2.greedy is False and sp2.proc is None and sp2.upd is None
    # with logits-processing rows and table updates (grammar mask rows + penalty slots to clear): every rank
    # rebuilds the same device tables from the plan
    proc = np.arange(32, dtype=np.int32).reshape(4, 8)
    upd = ProcUpdates(np.array([3, 9], np.int32), np.arange(2 * 5, dtype=np.int32).reshape(2, 5) - 4,
                      np.array([7], np.int32))
    sp.proc, sp.upd = proc, upd
    h3, sp3 = unpack_plan(*pack_plan(h, sp))
    assert (h3.i32 == h.i32).all() and (sp3.seeds == sp.seeds).all()
    assert (sp3.proc == proc).all() and (sp3.upd.mask_rows == upd.mask_rows).all()
    assert (sp3.upd.mask_words == upd.mask_words).all() and (sp3.upd.zero_slots == upd.zero_slots).all()


def test_ep_ops_roundtrip_equals_direct_moe_on_cpu():
    """dispatch -> (simulated) all-to-all -> device routing -> per-expert function -> return -> weighted combine
    == sum_j w_j f_{e_j}(x) computed directly, for every rank's owned tokens (CPU references of csrc/moe.hip ep_*)."""
    import torch

    from kafka_llm_service_amd import ops

    torch.manual_seed(0)
    T, d, E, k, ep = 23, 64, 8, 2, 4
    El = E // ep
    x = torch.randn(T, d).to(torch.bfloat16)
    r = ops.moe_route(torch.randn(T, E).to(torch.bfloat16), k)
    Tl, C, MR = ops.ep_layout(T, ep, k, El, d)
    scale = torch.arange(1, E + 1, dtype=torch.float32)  # expert e multiplies its row by e + 1
    imgs, slots = [], []
    for q in range(ep):
        lo, hi = min(T, q * Tl), min(T, (q + 1) * Tl)
        img, slot = ops.ep_dispatch(x, r.topk_e, lo, hi - lo, El, ep, C, MR)
        imgs.append(img)
        slots.append(slot)
    backs = []
    for p in range(ep):
        recv = torch.stack([imgs[s][p] for s in range(ep)])
        rr = ops.ep_recv_route(recv, C, El)
        y = torch.zeros(ep * (C + MR), d)
        rows = recv.view(-1, d)
        for e in range(El):
            a, b = int(rr.expert_off[e]), int(rr.expert_off[e + 1])
            idx = rr.perm_tok[a:b].long()
            y[idx] = rows[idx].float() * scale[p * El + e]
        backs.append(y.to(torch.bfloat16).view(ep, C + MR, d))
    for q in range(ep):
        lo, hi = min(T, q * Tl), min(T, (q + 1) * Tl)
        back = torch.stack([backs[p][q] for p in range(ep)])  # the return all-to-all
        out = torch.zeros(Tl, d, dtype=torch.bfloat16)
        ops.ep_combine(back, slots[q], r.topk_w, lo, hi - lo, out)
        want = sum(r.topk_w[lo:hi, j:j + 1] * x[lo:hi].float() * scale[r.topk_e[lo:hi, j].long()][:, None]
                   for j in range(k))
        torch.testing.assert_close(out[:hi - lo].float(), want, atol=0.1, rtol=2e-2)


def _dpa_owner(layout: str, i: int) -> int:
    return i % 2 if layout == "spread" else 0


def _dpa_main(rank: int, world: int, port: int, q, layout, board: str = "1", graphs: bool = False) -> None:
    """One rank of a DP-attention group: its own prompts (possibly none), experts sharded over the group."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(rank), "KAFKA_DPA_BOARD": board})
    from kafka_llm_service_amd.engine import dp_attention
    from kafka_llm_service_amd.parallel import state as pstate

    eng, st = dp_attention.build_dpa_engine(dict(CFG, model="tiny-mixtral", use_graphs=graphs), ep=world)
    try:
        assert eng.model.dp_attention and eng.model.ep == world and eng.model.tp == 1
        assert eng.model.layers[0].w13.shape[0] == eng.model_cfg.num_experts // world
        mine = [p for i, p in enumerate(_prompts()) if _dpa_owner(layout, i) == rank]
        outs = dp_attention.generate_lockstep(eng, st, mine, GREEDY)
        g = eng.runner.graphs
        q.put((rank, outs, eng.stats["group_steps"], eng.stats["planned_ahead"],
               dp_attention.make_board(st) is not None, g.stats["replays"] if g is not None else 0))
    finally:
        pstate.destroy()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("layout,board,graphs", [("spread", "1", False), ("one_idle", "1", False),
                                                 ("spread", "0", False), ("spread", "1", True)],
                         ids=["spread", "one_idle", "spread_gloo_agree", "spread_graphs"])
def test_dp_attention_mixtral_matches_single_rank(layout, board, graphs):
    """Mixtral with data-parallel attention over 2 ranks (each rank its own sequences, whole attention weights,
    half the experts, device-side all-to-all dispatch/combine in lockstep): every greedy token is the EP=1 model's
    argmax up to a small logit margin — also when one rank has no sequences at all and only serves its experts.
    The group plans ahead (step n+1 agreed and launched before step n is collected) and agrees through the
    shared-memory board (or gloo when the board is off)."""
    from kafka_llm_service_amd.models.oracle import dense_logits

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dpa_main, args=(r, 2, port, q, layout, board, graphs)) for r in range(2)]
    for p in procs:
        p.start()
    res = {m[0]: m[1:] for m in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1]  # lockstep: the same number of group steps on both ranks
    assert res[0][2] > 0  # planned ahead
    assert res[0][3] == res[1][3] == (board == "1")
    if graphs:  # decode steps replayed from captured layouts (fake graph backend on CPU: static buffers only)
        assert res[0][4] > 0 and res[1][4] > 0
    ref = LLMEngine(EngineConfig(**dict(CFG, model="tiny-mixtral")))
    prompts = _prompts()
    for r in (0, 1):
        mine = [p for i, p in enumerate(prompts) if _dpa_owner(layout, i) == r]
        assert len(res[r][0]) == len(mine)
        for p, o in zip(mine, res[r][0]):
            assert len(o) == GREEDY.max_tokens
            lg = dense_logits(ref.model, p + o)
            for i, tok in enumerate(o):
                row = lg[len(p) - 1 + i]
                assert (row.max() - row[tok]).item() < 0.05


@pytest.mark.timeout(300)
@pytest.mark.parametrize("extra", [{"_proc": True}, {"_proc": True, "use_graphs": True},
                                   {"_proc": True, "_env": {"KAFKA_PLAN_SLOT_BYTES": "1024"}}],
                         ids=["eager", "graphs", "oversized_plans"])
def test_tp2_logits_processing_matches_tp1(extra):
    """Grammar masks / forced tokens / penalties under TP: the leader ships the proc rows and the table updates
    (new mask rows of 16 KB: with 1 KB ring slots every such plan takes the oversized-plan gloo fallback) and every
    rank samples identically — the group's tokens equal a TP = 1 engine's with the same parameters."""
    from kafka_llm_service_amd.engine.chat_template import parse_tool_calls
    from kafka_llm_service_amd.engine.tokenizer import get_tokenizer

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_group_main, args=(r, 2, port, q, extra)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((m[0], m[1:]) for m in (q.get(timeout=240) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs = res["outs"][0]
    tok = get_tokenizer("llama3")
    assert parse_tool_calls(tok.decode(outs[0])) and outs[0][-1] == tok.special_id("<|eom_id|>")
    ref = LLMEngine(EngineConfig(**CFG)).generate(_prompts(), _proc_params())
    assert ref[0] == outs[0]  # the grammar leaves few near-ties; forced tokens are exact
    assert len(outs[1]) == len(ref[1]) == 5
