"""Engine integration on CPU (reference ops): paged + prefix-cached + continuously-batched greedy decoding must agree
with the dense cache-free oracle; cold vs warm prefix, cascade, chunked prefill and preemption must not change
the result (SURVEY.md §4.4 "Engine integration")."""
import pytest
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.models.oracle import dense_logits

GREEDY = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)


@pytest.fixture(scope="module")
def base_engine():
    return LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048))


def _engine(model=None, **kw):
    cfg = dict(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg), model=model)


def _prompts(seed=1, shared=70, tails=(5, 17, 40)):
    g = torch.Generator().manual_seed(seed)
    prefix = torch.randint(0, 5000, (shared,), generator=g).tolist()
    return [prefix + torch.randint(0, 5000, (n,), generator=g).tolist() for n in tails]


def _check_against_oracle(model, prompts, outs, tol=0.05):
    for p, o in zip(prompts, outs):
        lg = dense_logits(model, p + o)
        for i, tok in enumerate(o):
            row = lg[len(p) - 1 + i]
            assert (row.max() - row[tok]).item() < tol, f"token {i}: not the oracle's argmax"


def test_greedy_matches_oracle(base_engine):
    prompts = _prompts()
    outs = base_engine.generate(prompts, GREEDY)
    _check_against_oracle(base_engine.model, prompts, outs)


def test_prefix_hit_equals_cold(base_engine):
    prompts = _prompts(seed=2, shared=100)
    cold = _engine(model=base_engine.model, enable_prefix_cache=False).generate(prompts, GREEDY)
    warm_eng = _engine(model=base_engine.model)
    warm_eng.generate([prompts[0][:90] + [1, 2, 3]], GREEDY)  # seeds the tree with the shared prefix
    warm = warm_eng.generate(prompts, GREEDY)
    assert warm_eng.kv_stats()["hit_tokens"] >= 3 * 80
    assert warm == cold


def test_cascade_equals_plain(base_engine):
    prompts = _prompts(seed=3, shared=96, tails=(3, 9, 30, 31))
    e1 = _engine(model=base_engine.model, use_cascade=False)
    e2 = _engine(model=base_engine.model, use_cascade=True, cascade_min_prefix=16)
    e2.generate([prompts[0][:96] + [7]], GREEDY)
    plain = e1.generate(prompts, GREEDY)
    casc = e2.generate(prompts, GREEDY)
    assert max(st["cascade_prefix"] for st in e2.runner.recent_stats) >= 80
    assert casc == plain


def test_chunked_prefill_and_small_budget(base_engine):
    prompts = _prompts(seed=4, shared=50, tails=(60, 3))
    ref = _engine(model=base_engine.model).generate(prompts, GREEDY)
    chunked = _engine(model=base_engine.model, max_num_batched_tokens=24, max_prefill_chunk=16).generate(prompts,
                                                                                                       GREEDY)
    assert chunked == ref


def test_preemption_recompute(base_engine):
    prompts = _prompts(seed=5, shared=20, tails=(30, 30, 30, 30))
    params = SamplingParams(temperature=0.0, max_tokens=20, ignore_eos=True)
    ref = _engine(model=base_engine.model).generate(prompts, params)
    small = _engine(model=base_engine.model, num_kv_blocks=12)
    out = small.generate(prompts, params)
    assert small.sched.num_preemptions > 0
    assert out == ref


def test_sampling_params_validation():
    with pytest.raises(ValueError):
        SamplingParams(temperature=-1)
    with pytest.raises(ValueError):
        SamplingParams(top_p=0)
    assert SamplingParams(temperature=0).greedy


def test_stop_tokens_and_abort(base_engine):
    eng = _engine(model=base_engine.model)
    p = _prompts(seed=6)[0]
    first = eng.generate([p], GREEDY)[0]
    s = eng.add_request("x", p, SamplingParams(temperature=0, max_tokens=10, stop_token_ids=[first[2]]))
    while not s.finished:
        eng.step()
    k = first.index(first[2])
    assert s.finish_reason == "stop" and s.output_ids == first[:k + 1]
    s2 = eng.add_request("y", p, SamplingParams(temperature=0, max_tokens=10))
    eng.step()
    eng.abort("y")
    assert s2.finish_reason == "abort" and not eng.has_unfinished()
    assert eng.kvm.check_invariants()


def test_context_length_error(base_engine):
    eng = _engine(model=base_engine.model, max_model_len=64)
    with pytest.raises(ValueError, match="maximum context length"):
        eng.add_request("z", list(range(100)), GREEDY)


def test_sampling_temperature_reproducible(base_engine):
    eng = _engine(model=base_engine.model)
    p = _prompts(seed=7)[:2]
    sp = SamplingParams(temperature=0.8, top_p=0.9, top_k=50, max_tokens=5, seed=123, ignore_eos=True)
    a = eng.generate(p, sp)
    b = _engine(model=base_engine.model).generate(p, sp)
    assert a == b


def test_split_kv_prefill_equals_plain(base_engine):
    """A new turn on a long cached context: key-range-split prefill tiles + merge == one pass."""
    prompts = _prompts(seed=8, shared=300, tails=(9,))
    ref_eng = _engine(model=base_engine.model)
    ref_eng.generate([prompts[0][:290] + [3]], GREEDY)
    ref = ref_eng.generate(prompts, GREEDY)
    e = _engine(model=base_engine.model, prefill_kv_chunk=32)
    e.generate([prompts[0][:290] + [3]], GREEDY)
    s = e.add_request("q", prompts[0], GREEDY)
    e.step()
    assert max(st["prefill_splits"] for st in e.runner.recent_stats) >= 9
    while not s.finished:
        e.step()
    assert s.output_ids == ref[0]


def test_mixtral_greedy_matches_oracle():
    """MoE engine path (router -> grouped GEMMs -> weighted combine, ops references on CPU) vs the dense oracle."""
    eng = LLMEngine(EngineConfig(model="tiny-mixtral", device="cpu", num_kv_blocks=256, max_model_len=2048))
    prompts = _prompts(seed=5, shared=40, tails=(4, 19))
    outs = eng.generate(prompts, GREEDY)
    _check_against_oracle(eng.model, prompts, outs)


def test_async_scheduling_equals_sync(base_engine):
    """Planning step n+1 while step n is in flight (PENDING tokens patched at launch, plans dropped when requests
    arrive or sequences finish) must not change any output; requests join mid-run and finish at different times."""
    import random

    prompts = _prompts(seed=9, shared=60, tails=(2, 30, 7, 55, 11))
    lens = [3, 9, 5, 12, 7]

    def run(async_on):
        eng = _engine(model=base_engine.model, async_scheduling=async_on)
        rng = random.Random(0)
        pending = list(range(len(prompts)))
        seqs = {}
        while pending or any(not s.finished for s in seqs.values()):
            if pending and rng.random() < 0.4:
                i = pending.pop(0)
                sp = SamplingParams(temperature=0.0, max_tokens=lens[i], ignore_eos=True)
                seqs[i] = eng.add_request(f"r{i}", prompts[i], sp)
            eng.step()
        return [seqs[i].output_ids for i in range(len(prompts))], eng.stats

    sync_out, _ = run(False)
    async_out, st = run(True)
    assert async_out == sync_out
    assert st["planned_ahead"] > 0


def test_overlapped_launch_stops_and_aborts(base_engine):
    """Step n+1 is launched before step n lands (its decode inputs copied device-side from n's sampler output). A
    sequence that stops on a token at n, or is aborted while both steps are in flight, gets no extra token; the
    void row is discarded and every page is freed."""
    prompts = _prompts(seed=13, shared=40, tails=(3, 17, 9))
    ref = _engine(model=base_engine.model, async_scheduling=False)
    free_run = ref.generate(prompts, SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True))
    stop_tok = free_run[1][4]
    sp = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True, stop_token_ids=[stop_tok])
    want = ref.generate(prompts, sp)
    eng = _engine(model=base_engine.model)
    got = eng.generate(prompts, sp)
    assert got == want and len(got[1]) <= 5 and got[1][-1] == stop_tok
    seqs = [eng.add_request(f"a{i}", p, SamplingParams(temperature=0.0, max_tokens=30, ignore_eos=True))
            for i, p in enumerate(prompts)]
    for _ in range(4):
        eng.step()
    eng.abort("a1")
    n_at_abort = len(seqs[1].output_ids)
    while eng.has_unfinished():
        eng.step()
    eng.step()  # drain the last in-flight step
    assert len(seqs[1].output_ids) == n_at_abort and seqs[1].finish_reason == "abort"
    assert [s.output_ids for s in (seqs[0], seqs[2])] == [free_run[0] + s.output_ids[12:] for s in (seqs[0],)] + \
        [free_run[2] + seqs[2].output_ids[12:]]
    assert all(t >= 0 for s in seqs for t in s.output_ids)
    eng.kvm.check_invariants()
    assert eng.kv_stats()["sequences"] == 0


def test_pinned_prefix_survives_eviction(base_engine):
    eng = _engine(model=base_engine.model, num_kv_blocks=64)
    prefix = list(range(3000, 3000 + 160))  # 10 full pages
    eng.generate([prefix + [1, 2]], SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
    assert eng.pin_prefix(prefix) == 160
    eng.kvm.evict_all()
    # a request far larger than the free pool forces eviction pressure; the pinned pages must stay cached
    eng.generate([list(range(9000, 9000 + 700))], SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
    s = eng.add_request("after", prefix + [7], SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True))
    eng.step()
    assert s.num_cached == 160
    eng.unpin_prefix()
    eng.kvm.check_invariants()


def test_kv_pool_limits_are_handled(base_engine):
    eng = _engine(model=base_engine.model, num_kv_blocks=8)  # 128 tokens of KV
    with pytest.raises(ValueError, match="maximum context length"):
        eng.add_request("big", list(range(1000, 1200)), GREEDY)
    # a sequence that outgrows the pool while decoding ends by length instead of stalling the engine
    s = eng.add_request("grow", list(range(1000, 1100)),
                        SamplingParams(temperature=0.0, max_tokens=100, ignore_eos=True))
    outs = []
    for _ in range(200):
        outs += eng.step()
        if s.finished:
            break
    assert s.finished and s.finish_reason == "length" and 0 < len(s.output_ids) < 100
    assert outs[-1].finished and outs[-1].request_id == "grow"
    eng.kvm.check_invariants()


def test_stream_decode_gemm_matches_oracle():
    """Decode steps through the weight-streaming GEMM path (wave-tiled weights, split-K slabs consumed by the RoPE /
    SwiGLU / add+RMSNorm ops; CPU runs the same split decisions on the fp32 references) agree with the oracle."""
    from kafka_llm_service_amd import ops

    eng = _engine(decode_gemm="stream")
    m = eng.model
    assert m.stream and m.layers[0].qkv_t is not None and m.lm_head_t is not None
    assert torch.equal(ops.untile_weight(m.layers[0].down_t), m.layers[0].down)
    assert m.layers[0].glu and torch.equal(ops.untile_weight(m.layers[0].gate_up_t, glu=True), m.layers[0].gate_up)
    # tiny-llama decode shapes take split-K plans, so the slab consumers are exercised
    assert ops.stream_plan(3, m.layers[0].o.shape[0], m.layers[0].o.shape[1])[2] > 1
    prompts = _prompts(seed=9)
    outs = eng.generate(prompts, GREEDY)
    _check_against_oracle(m, prompts, outs)


def test_fused_decode_layer_matches_unfused(monkeypatch):
    """The fused decode layer (deferred RMSNorm in the GEMMs, RoPE + KV write in the QKV finisher, residual add in the
    o / down finishers; models/llama.py _forward_fused) takes every decode step of the stream mode, and generation
    agrees with the unfused layer and with the dense oracle."""
    from kafka_llm_service_amd import ops
    from kafka_llm_service_amd.models import llama

    calls = {"qkv": 0, "res": 0, "glu": 0}
    for name, key in (("linear_qkv_rope", "qkv"), ("linear_res", "res"), ("linear_glu_rs", "glu")):
        orig = getattr(ops, name)

        def wrap(*a, _o=orig, _k=key, **kw):
            calls[_k] += 1
            return _o(*a, **kw)
        monkeypatch.setattr(ops, name, wrap)
    monkeypatch.setattr(llama, "FUSED", True)
    eng = _engine(decode_gemm="stream")
    prompts = _prompts(seed=10)
    fused = eng.generate(prompts, GREEDY)
    L = eng.model_cfg.num_layers
    assert calls["qkv"] >= L and calls["res"] >= 2 * L - 1 and calls["glu"] >= L
    _check_against_oracle(eng.model, prompts, fused)
    monkeypatch.setattr(llama, "FUSED", False)
    n = calls["qkv"]
    plain = _engine(decode_gemm="stream", model=eng.model).generate(prompts, GREEDY)
    assert calls["qkv"] == n  # the unfused path never enters the fused ops
    assert plain == fused


def test_fused_ops_cpu_reference():
    """ops.linear_res / linear_qkv_rope / linear_glu_rs (CPU reference of the FIN epilogues) against the unfused op
    chain: residual add + RMSNorm, then the projection of the normalised rows (RMSNorm deferred through ``ss``)."""
    from kafka_llm_service_amd import ops
    from kafka_llm_service_amd.ops import reference as ref

    torch.manual_seed(3)
    M, d, F, Hq, Hkv = 5, 512, 256, 2, 1
    eps = 1e-5
    resid = torch.randn(M, d).to(torch.bfloat16)
    a = torch.randn(M, F).to(torch.bfloat16)
    w_down = (torch.randn(d, F) * F ** -0.5).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(d)).to(torch.bfloat16)
    r0 = resid.clone()
    xn = torch.empty(M, d, dtype=torch.bfloat16)
    ss = torch.empty(d // 128, M)
    ops.linear_res(a, ops.tile_weight(w_down), resid, nw, xn, ss)
    s_ref = (r0.float() + a.float() @ w_down.float().t()).to(torch.bfloat16)
    assert (resid.float() - s_ref.float()).abs().max() < 2e-2
    assert torch.allclose(ss.sum(0), s_ref.float().pow(2).sum(1), rtol=1e-3)
    normed = ref.rmsnorm(s_ref, nw, eps).float()
    r = ops.fin_row_scale(ss, M, d, eps)
    assert (xn.float() * r[:, None] - normed).abs().max() < 0.05
    # QKV + RoPE of the deferred-normalised rows == rope_kv_write of the normalised rows' projection
    w_qkv = (torch.randn((Hq + 2 * Hkv) * 128, d) * d ** -0.5).to(torch.bfloat16)
    cs = ref.rope_cos_sin(256, 128, 500000.0)
    pos = torch.tensor([3, 9, 0, 100, 255])
    slots = torch.tensor([0, 17, -1, 5, 40])
    q1, q2 = torch.empty(M, Hq, 128, dtype=torch.bfloat16), torch.empty(M, Hq, 128, dtype=torch.bfloat16)
    k1, v1 = torch.zeros(4, Hkv, 16, 128, dtype=torch.bfloat16), torch.zeros(4, Hkv, 128, 16, dtype=torch.bfloat16)
    k2, v2 = k1.clone(), v1.clone()
    ops.linear_qkv_rope(xn, ops.tile_weight(w_qkv), ss, eps, pos, cs, q1, k1, v1, slots, Hq, Hkv)
    ref.rope_kv_write((normed @ w_qkv.float().t()), pos, cs, q2, k2, v2, slots, Hq, Hkv)
    for x1, x2 in ((q1, q2), (k1, k2), (v1, v2)):
        assert (x1.float() - x2.float()).abs().max() < 0.05
    # gate_up with the row scale == SwiGLU of the normalised rows' projection
    w_gu = (torch.randn(2 * F, d) * d ** -0.5).to(torch.bfloat16)
    y = ops.linear_glu_rs(xn, ops.tile_weight(w_gu, glu=True), ss, eps)
    y_ref = ref.silu_mul(normed @ w_gu.float().t())
    assert (y.float() - y_ref.float()).abs().max() < 0.05


def test_stream_plan_rules(monkeypatch):
    """The decode GEMM plan (ops.stream_plan, mirrored from csrc kafka_wstream_plan): row tiles by step size (1 / 2 /
    3 / 4 x 32 rows), 128-deep chunks for four tiles, split-K grown toward the grid target."""
    from kafka_llm_service_amd import ops

    assert [ops.stream_plan(M, 28672, 4096)[0] for M in (1, 32, 33, 64, 65, 96, 97, 128, 129, 192, 193, 256)] == \
        [1, 1, 2, 2, 3, 3, 4, 4, 6, 6, 4, 4]  # 129..192: one 192-row tile; beyond: row tiles of 128
    assert ops.stream_plan(169, 28672, 4096)[1:] == (128, 1) and ops.stream_plan(169, 6144, 4096)[2] == 4
    assert ops.stream_plan(128, 4096, 4096)[1] == 128 and ops.stream_plan(64, 4096, 4096)[1] == 256
    assert ops.stream_plan(64, 28672, 4096)[2] == 1 and ops.stream_plan(64, 6144, 4096)[2] == 4
    assert ops.stream_plan(114, 28672, 4096)[2] == 1  # gate_up unsplit at 97..128 rows (fused SwiGLU)
    assert ops.stream_plan(300, 4096, 4096) is None and ops.stream_plan(64, 4100, 4096) is None


def test_tiled_only_weights_match_stream():
    """Tiled-only mode (the row-major dense weights dropped after tiling, prefill untiles per projection — what a
    model whose second weight copy does not fit gets) generates exactly what the two-copy stream mode does."""
    ref_eng = _engine(decode_gemm="stream")
    eng = _engine(decode_gemm="stream_only")
    m = eng.model
    assert m.tiled_only and m.layers[0].qkv is None and m.layers[0].gate_up is None and m.layers[0].qkv_t is not None
    # tiled-only steps keep to the streaming kernel's rows (scheduler row fit), the two-copy mode does not
    assert eng.sched.cfg.step_rows_fit == ops.STREAM_MAX_M and ref_eng.sched.cfg.step_rows_fit == 0
    prompts = _prompts(seed=9)
    a = ref_eng.generate(prompts, GREEDY)
    b = eng.generate(prompts, GREEDY)
    assert a == b and all(len(x) for x in a)


def test_out_of_vocab_prompt_rejected(base_engine):
    """Token ids outside the vocabulary are refused at admission (on the GPU they would read past the embedding)."""
    V = base_engine.model_cfg.vocab_size
    with pytest.raises(ValueError, match="token ids"):
        base_engine.add_request("oov", [1, 2, V], GREEDY)
    with pytest.raises(ValueError, match="token ids"):
        base_engine.add_request("neg", [-1, 2], GREEDY)
    assert "oov" not in base_engine.requests


def test_multi_group_cascade_equals_plain(base_engine, monkeypatch):
    """Three system prompts (Kafka prompt, a thread created with its own system message — quirk Q4 — and a second
    custom prompt) plus a stateless row with no shared prefix: every group gets its own cascade pass and the
    result equals plain per-row attention (fp32 prefix partials: token-exact; the bf16 default is checked to
    logit tolerance by test_bf16_cascade_partials_close_to_fp32)."""
    groups = [_prompts(seed=10 + i, shared=96, tails=(3, 9, 30)) for i in range(3)]
    loner = _prompts(seed=20, shared=0, tails=(50,))
    prompts = [p for g in groups for p in g] + loner
    e1 = _engine(model=base_engine.model, use_cascade=False)
    e2 = _engine(model=base_engine.model, use_cascade=True, cascade_min_prefix=16)
    e2.runner.cascade_bf16 = False
    for g in groups:
        e2.generate([g[0][:96] + [7]], GREEDY)
    plain = e1.generate(prompts, GREEDY)
    casc = e2.generate(prompts, GREEDY)
    assert max(st["cascade_groups"] for st in e2.runner.recent_stats) == 3
    assert casc == plain


def test_prefix_groups_and_decode_items():
    import numpy as np

    from kafka_llm_service_amd.engine.model_runner import MAX_PARTIALS, decode_items, prefix_groups

    # rows 0,2,4 share pages [10, 11, 12, 13]; rows 1,3 share [10, 20, 21, 22] (same first page, then diverge);
    # row 5 is alone
    bt = np.array([[10, 11, 12, 13, 50], [10, 20, 21, 22, 51], [10, 11, 12, 13, 52], [10, 20, 21, 22, 53],
                   [10, 11, 12, 13, 54], [90, 91, 92, 93, 94]], dtype=np.int32)
    nfull = np.array([4, 4, 5, 4, 4, 4])
    order, groups = prefix_groups(bt, nfull, min_blocks=3)
    assert sorted(order) == list(range(6))
    assert groups == [(3, 4), (2, 4)] and order[:3] == [0, 2, 4] and order[3:5] == [1, 3] and order[5] == 5
    # below min_blocks nothing groups
    assert prefix_groups(bt, nfull, min_blocks=5)[1] == []
    # decode items: pieces cover [kv_start, len) exactly, 32-aligned inside, at most MAX_PARTIALS - npre per row
    lens = np.array([5000, 40, 700, 19000])
    ks = np.array([64, 0, 512, 0])
    npre = np.array([3, 0, 3, 0])
    it = decode_items(lens, ks, npre, hkv=8, target=64)
    for b in range(4):
        rows = it[it[:, 0] == b]
        assert rows[0, 1] == ks[b] and rows[-1, 2] == lens[b]
        assert (rows[1:, 1] == rows[:-1, 2]).all() and (rows[1:, 1] % 32 == 0).all()
        assert (rows[:, 3] == np.arange(len(rows))).all() and (rows[:, 4] == len(rows)).all()
        assert (rows[:, 5] == npre[b]).all() and len(rows) + npre[b] <= MAX_PARTIALS
    assert (it[:, 0] == 3).sum() > (it[:, 0] == 1).sum() == 1  # the long row is split, the short one is not
    # fixed-count items (graph replay): exactly max(B, target // hkv) items, the same coverage rules, null pads
    from kafka_llm_service_amd.engine.model_runner import decode_items_fixed

    rng = np.random.default_rng(3)
    for B, target in ((4, 64), (4, 1344), (64, 1344), (3, 8)):
        lens = rng.integers(300, 30000, B)
        ks = np.minimum(lens - 1, rng.integers(0, 20000, B) // 16 * 16)
        npre = rng.integers(0, 33, B)
        it = decode_items_fixed(lens, ks, npre, hkv=8, target=target)
        assert it.shape[0] == max(B, target // 8)
        real = it[it[:, 3] >= 0]
        for b in range(B):
            rows = real[real[:, 0] == b]
            rows = rows[np.argsort(rows[:, 3])]
            assert rows[0, 1] == ks[b] and rows[-1, 2] == lens[b]
            assert (rows[1:, 1] == rows[:-1, 2]).all() and (rows[1:, 1] % 32 == 0).all() and (rows[:, 2] > rows[:, 1]).all()
            assert (rows[:, 3] == np.arange(len(rows))).all() and (rows[:, 4] == len(rows)).all()
            assert len(rows) + npre[b] <= MAX_PARTIALS


def test_tiled_only_mixtral_and_export(tmp_path):
    """Tiled-only mode on an MoE model: experts stay row-major (no second expert copy), the lm_head keeps only its
    tiled copy, generation equals the two-copy stream mode, and safetensors export untiles what was dropped."""
    from kafka_llm_service_amd.models.weights import build_model, save_safetensors

    base = dict(model="tiny-mixtral", device="cpu", num_kv_blocks=256, max_model_len=2048)
    ref_eng = LLMEngine(EngineConfig(**base, decode_gemm="stream"))
    eng = LLMEngine(EngineConfig(**base, decode_gemm="stream_only"))
    m = eng.model
    assert m.tiled_only and m.lm_head is None and m.lm_head_t is not None
    assert m.layers[0].w13 is not None and m.layers[0].w13_t is None  # experts: one (row-major) copy
    assert eng.cfg.max_num_seqs <= ops.STREAM_KERNEL_MAX_M  # decode batches the streaming kernel takes
    assert m.weight_bytes() >= ref_eng.model.weight_bytes() // 2
    prompts = _prompts(seed=12)
    assert eng.generate(prompts, GREEDY) == ref_eng.generate(prompts, GREEDY)
    save_safetensors(m, tmp_path / "model.safetensors")
    back = build_model(m.cfg, "cpu", weights=str(tmp_path))
    assert torch.equal(back.lm_head, ref_eng.model.lm_head)
    assert torch.equal(back.layers[1].qkv, ref_eng.model.layers[1].qkv)


def test_plan_prefill_items_balances_causal_tiles():
    """A causal 2k-token chunk (32 tiles of 64 tokens, extents 64..2048): tiles longer than the balanced share are
    split into equal key pieces (contiguous merge ranges), short tiles stay whole, items come longest-first, and
    every tile's keys [0, extent) are covered exactly once."""
    from kafka_llm_service_amd.engine.model_runner import plan_prefill_items

    tiles = [(64 * i, 64, 0, 64 * (i + 1), 2048) for i in range(32)]
    items, splits, ranges = plan_prefill_items(tiles, hkv=8, target_wgs=256, min_chunk=256)
    assert splits == 2 and len(ranges) == 1 and ranges[0][1] == 2048
    assert all((it[4] - it[3]) >= (nx[4] - nx[3]) for it, nx in zip(items, items[1:]))
    for q0, cnt, _, ext, _ in tiles:
        mine = sorted((it[3], it[4]) for it in items if it[0] == q0)
        whole = [it for it in items if it[0] == q0 and it[5] < 0]
        if whole:
            assert len(mine) == 1 and mine[0] == (0, 2048)  # kernel clamps to the causal limit itself
            assert not any(lo <= q0 < hi for lo, hi in ranges)
        else:
            assert mine[0][0] == 0 and mine[-1][1] >= ext and all(a[1] == b[0] for a, b in zip(mine, mine[1:]))
            assert any(lo <= q0 < hi for lo, hi in ranges)
    # a short prompt is never split; a many-tile launch only splits past the LDS page bound
    assert plan_prefill_items([(0, 64, 0, 64, 300), (64, 64, 0, 128, 300)], 8, 256, 256)[1] == 0
    many = [(64 * i, 64, 0, 64 * (i + 1), 8192) for i in range(128)]
    assert plan_prefill_items(many, 8, 256, 256)[1] == 0
    # a new turn: 2 tiles against a 20k context -> ~target_wgs workgroups in total
    turn = [(0, 64, 0, 20000, 20064), (64, 40, 0, 20104, 20104)]
    items, splits, ranges = plan_prefill_items(turn, 8, 256, 256)
    assert 200 <= len(items) * 8 <= 256 and ranges == [(0, 104)]
    # several new turns in one step (tiles of mixed lengths, all long): still ONE round of <= 256 workgroups
    burst = [(64 * i, 64, i // 2, 19000 + 300 * i, 19100 + 300 * i) for i in range(5)]
    items, splits, ranges = plan_prefill_items(burst, 8, 256, 256)
    assert 200 <= len(items) * 8 <= 256, len(items) * 8


def test_padded_mixed_steps_match_unpadded(base_engine, monkeypatch):
    """Steps beyond the streaming GEMM's rows (up to 256) padded with inert rows (pad_step_rows) produce the same
    greedy tokens (checked with the streaming bound at 128, so a 150-row step is padded)."""
    from kafka_llm_service_amd.engine.model_runner import pad_step_rows

    monkeypatch.setattr(ops, "STREAM_MAX_M", 128)
    assert [pad_step_rows(t) for t in (64, 128, 129, 160, 168, 170, 185, 192, 250, 256, 300)] == \
        [64, 128, 168, 168, 168, 184, 200, 200, 250, 256, 300]
    prompts = _prompts(seed=21, shared=100, tails=(50,))  # first step: one 150-token prefill -> padded to 168 rows
    ref = _engine(model=base_engine.model).generate(prompts, GREEDY)
    e = _engine(model=base_engine.model)
    e.runner.pad_rows = True
    seen = []
    orig = e.runner.build_host

    def build_host(batch):
        h, ss = orig(batch)
        seen.append(h.T)
        return h, ss
    e.runner.build_host = build_host
    assert e.generate(prompts, GREEDY) == ref
    assert 168 in seen


def test_skinny_projections_match_blas(monkeypatch):
    """KAFKA_SKINNY: the qkv / o / down projections of 129..256-row steps on the skinny GEMM path (its split-K slabs
    consumed by rope / add+RMSNorm like the decode GEMM's) give the same greedy tokens as the dense path."""
    from kafka_llm_service_amd.models import llama

    prompts = _prompts(seed=23, shared=100, tails=(50,))  # first step: one 150-row prefill
    monkeypatch.setattr(ops, "STREAM_MAX_M", 128)  # (150 rows would otherwise stream: 192-row tile)
    e0 = _engine(decode_gemm="stream")
    monkeypatch.setattr(llama, "SKINNY", frozenset())
    ref = e0.generate(prompts, GREEDY)
    monkeypatch.setattr(llama, "SKINNY", frozenset({"qkv", "o", "down"}))
    calls = []
    orig = ops.linear_skinny

    def spy(x, wt, *a, **k):
        calls.append(x.shape[0])
        return orig(x, wt, *a, **k)
    monkeypatch.setattr(ops, "linear_skinny", spy)
    e1 = _engine(decode_gemm="stream", model=e0.model)
    assert e1.generate(prompts, GREEDY) == ref
    assert calls and all(129 <= m <= 256 for m in calls) and len(calls) % 3 == 0


def test_bf16_cascade_partials_close_to_fp32(base_engine, monkeypatch):
    """The tile-v3 cascade hands its prefix partials to the decode kernel as bf16 by default (half the bytes):
    decode-step logits stay within bf16 rounding of the fp32-partial path."""
    prompts = _prompts(seed=31, shared=96, tails=(3, 9, 30))
    logits = {}
    for mode in ("0", "1"):
        e = _engine(model=base_engine.model, use_cascade=True, cascade_min_prefix=16)
        e.runner.cascade_bf16 = mode == "1"
        e.generate([prompts[0][:96] + [7]], GREEDY)
        seen = []
        orig = e.runner.sample_device

        def spy(lg, sp, seen=seen, orig=orig):
            seen.append(lg.float().clone())
            return orig(lg, sp)
        e.runner.sample_device = spy
        e.generate(prompts, GREEDY)
        logits[mode] = seen
        assert e.runner.cascade_bf16 == (mode == "1")
    a, b = logits["0"][1], logits["1"][1]  # first decode step (the cascade pass ran)
    assert a.shape == b.shape
    assert (a - b).abs().max().item() < 0.05 * a.abs().max().item() + 0.05


@pytest.mark.parametrize("join_suffix", [False, True])
def test_new_turn_rows_join_the_prefix_pass(base_engine, join_suffix):
    """New-turn prefill chunks that start behind a cascade group's cached prefix take part in the group's prefix
    pass (model_runner._prefix_joins: one read of the shared pages per step for decode AND prefill rows, fp32
    partials merged with the chunk's own tiles over the keys behind the prefix): the tokens equal plain per-row
    attention, and the joined path actually ran (steps with joined tiles). With ``join_suffix`` the chunk's own
    keys are items of the same cascade launch too: steps with joined tiles then launch no prefill tile kernel."""
    prompts = _prompts(seed=41, shared=160, tails=(5, 23, 40))
    late = _prompts(seed=42, shared=0, tails=(37, 90))  # new turns arriving while the group decodes
    late = [prompts[0][:160] + t for t in late]
    sp = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    outs = []
    for cascade in (False, True):
        e = _engine(model=base_engine.model, use_cascade=cascade, cascade_min_prefix=16, prefill_kv_chunk=64)
        e.runner.cascade_bf16 = False  # fp32 prefix partials: token-exact against the plain path
        e.runner.join_suffix = join_suffix
        e.generate([prompts[0][:160] + [7]], GREEDY)  # the shared prefix is cached
        seqs = [e.add_request(f"r{i}", p, sp) for i, p in enumerate(prompts)]
        for _ in range(3):
            e.step()
        seqs += [e.add_request(f"l{i}", p, sp) for i, p in enumerate(late)]
        while any(not s.finished for s in seqs):
            e.step()
        outs.append([list(s.output_ids) for s in seqs])
        if cascade:
            joined = [st.get("prefix_joined_tiles", 0) for st in e.runner.recent_stats]
            assert max(joined) >= 2, joined
            items = [st["prefill_items"] for st in e.runner.recent_stats if st.get("prefix_joined_tiles")]
            assert (max(items) == 0) if join_suffix else (min(items) > 0), items
    assert outs[0] == outs[1]


def test_retile_joins_contiguous_spans():
    """The prefix pass re-tiles joined prefill tokens: contiguous spans are joined, then cut into full tiles."""
    from kafka_llm_service_amd.engine.model_runner import retile

    assert retile([(i * 30, 30) for i in range(8)], 64) == [(0, 64), (64, 64), (128, 64), (192, 48)]
    assert retile([(0, 64), (64, 36), (200, 10)], 64) == [(0, 64), (64, 36), (200, 10)]
    assert retile([(0, 37), (37, 90)], 64) == [(0, 64), (64, 63)]
    assert retile([], 64) == []


def test_plan_prefill_items_with_prefix_offset():
    """A tile behind a cascade prefix (lo > 0) attends only [lo, extent) and writes partials from slot s0 on."""
    from kafka_llm_service_amd.engine.model_runner import plan_prefill_items

    tiles = [(0, 64, 3, 20000, 20100, 18000, 28), (64, 36, 3, 20100, 20100, 18000, 28), (100, 50, 4, 900, 950)]
    items, splits, ranges = plan_prefill_items(tiles, 8, 256, 256)
    mine = [it for it in items if it[0] in (0, 64)]
    assert mine and all(it[3] >= 18000 and it[5] >= 28 for it in mine)
    assert min(it[3] for it in mine if it[0] == 0) == 18000 and max(it[4] for it in mine if it[0] == 0) >= 20000
    assert splits == max(it[5] for it in items) + 1
    assert any(lo <= 0 and hi >= 100 for lo, hi in ranges)


def test_engine_logits_bounded_by_fp32_forward_cpu(base_engine):
    """The composed-numerics bound of tests/test_numerics_gpu.py on the CPU reference ops (tiny-llama): prefill,
    decode, prefix-cached and cascade rows within K_STD of the fp32 forward and within RATIO of the bf16 forward's
    own error."""
    from tests.test_numerics_gpu import _check, composed_errors

    eng = _engine(model=base_engine.model, cascade_min_prefix=16)
    g = torch.Generator().manual_seed(12)
    _check(composed_errors(eng, [torch.randint(0, 5000, (n,), generator=g).tolist() for n in (9, 33)]), "cpu cold")
    prefix = torch.randint(0, 5000, (96,), generator=g).tolist()
    warm = [prefix + torch.randint(0, 5000, (n,), generator=g).tolist() for n in (3, 20)]
    _check(composed_errors(eng, warm, warm_prefix=prefix), "cpu cascade")
