"""Composed numerics of the engine against an fp32 forward (VERDICT r05 "Next" #8): every logits row the paged engine
samples from — prefill, decode, cascade-prefix and prefix-cached rows — is compared with the dense oracle run in fp32
(models/oracle.py ``fp32=True``). Bound per row: max|engine - fp32| <= K_STD * std(fp32 row), and no more than
RATIO x the error of the plain bf16 PyTorch forward of the same weights (so the hand-written kernels add at most a
bf16-sized error on top of bf16 rounding itself). Argmax checks alone (test_engine_gpu.py) bound nothing when
random-init logits are flat."""
import pytest
import torch

from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.models.oracle import dense_logits

K_STD = 0.25   # max |error| per row, in units of the fp32 row's standard deviation
RATIO = 3.0    # ... and at most this times the bf16 PyTorch forward's own max |error| on the row (+ 0.02 std)


def composed_errors(eng, prompts, warm_prefix=None, max_tokens=6):
    """Run ``prompts`` (all admitted in the first step, same length budget) and return per sampled row:
    (kind, max|engine - fp32| / std, max|bf16 oracle - fp32| / std)."""
    if warm_prefix is not None:
        eng.generate([warm_prefix + [1]], SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True))
    seen = []
    orig = eng.runner.sample_device

    def keep(lg, sp):
        seen.append(lg.float().cpu())
        return orig(lg, sp)

    eng.runner.sample_device = keep
    budget = eng.sched.cfg.prefill_cost_budget
    eng.sched.cfg.prefill_cost_budget = 0  # every prompt admitted in the first step: row j of each step = prompt j
    try:
        outs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=max_tokens, ignore_eos=True))
    finally:
        eng.runner.sample_device = orig
        eng.sched.cfg.prefill_cost_budget = budget
    steps = [t for t in seen if t.shape[0] == len(prompts)]
    assert len(steps) == max_tokens, [t.shape for t in seen]
    rows = []
    for j, (p, o) in enumerate(zip(prompts, outs)):
        f32 = dense_logits(eng.model, p + o, fp32=True).cpu()
        b16 = dense_logits(eng.model, p + o).cpu()
        for i in range(max_tokens):
            r = f32[len(p) - 1 + i]
            sd = r.std().item()
            kind = "prefill" if i == 0 else "decode"
            rows.append((kind, (steps[i][j] - r).abs().max().item() / sd, (b16[len(p) - 1 + i] - r).abs().max().item() / sd))
    return rows


def _check(rows, label):
    worst = max(e for _, e, _ in rows)
    print(f"{label}: engine max|d|/std p50 %.4f max %.4f | bf16 oracle p50 %.4f max %.4f (n=%d)" % (
        sorted(e for _, e, _ in rows)[len(rows) // 2], worst, sorted(b for _, _, b in rows)[len(rows) // 2],
        max(b for _, _, b in rows), len(rows)))
    for kind, e, b in rows:
        assert e <= K_STD, f"{label} {kind} row: engine error {e:.4f} std > {K_STD}"
        assert e <= RATIO * b + 0.02, f"{label} {kind} row: engine error {e:.4f} std vs bf16 forward {b:.4f}"


@pytest.mark.gpu
def test_engine_logits_bounded_by_fp32_forward(cuda):
    """small-llama on the HIP kernels: cold prefill + decode rows, then prefix-cached prompts whose decode runs the
    cascade (shared prefix pass + suffix decode with the fused merge)."""
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", num_kv_blocks=2048, max_model_len=4096,
                                 cascade_min_prefix=64))
    g = torch.Generator().manual_seed(11)
    cold = [torch.randint(0, 50000, (n,), generator=g).tolist() for n in (37, 150, 300)]
    _check(composed_errors(eng, cold), "cold")
    prefix = torch.randint(0, 50000, (400,), generator=g).tolist()
    warm = [prefix + torch.randint(0, 50000, (n,), generator=g).tolist() for n in (3, 40, 90, 7)]
    rows = composed_errors(eng, warm, warm_prefix=prefix)
    assert max(st["cascade_prefix"] for st in eng.runner.recent_stats) > 0, "the cascade did not run"
    _check(rows, "prefix-cached + cascade")
