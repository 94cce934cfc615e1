"""Debug: run an engine on NaN-poisoned device memory (every torch.empty returns NaN garbage) and report the first
step whose logits are not finite — finds reads of uninitialised buffers."""
import os, sys, traceback
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams

model = os.environ.get("DBG_MODEL", "tiny-mixtral")
asyn = os.environ.get("DBG_ASYNC", "1") == "1"
try:
    junk = [torch.full((1 << 28,), float("nan"), device="cuda:0") for _ in range(8)]
    del junk
    e = LLMEngine(EngineConfig(model=model, device="cuda:0", num_kv_blocks=1024, max_model_len=4096,
                               async_scheduling=asyn))
    orig = e.runner.sample_device
    step = [0]

    def chk(logits, sp):
        step[0] += 1
        bad = (~torch.isfinite(logits.float())).sum().item()
        if bad:
            print(f"step {step[0]}: {bad} non-finite logits of {logits.numel()} shape {tuple(logits.shape)}",
                  flush=True)
            os._exit(3)
        return orig(logits, sp)

    e.runner.sample_device = chk
    g = torch.Generator().manual_seed(3)
    V = e.model_cfg.vocab_size
    prefix = torch.randint(0, V, (64,), generator=g).tolist()
    prompts = [prefix + torch.randint(0, V, (n,), generator=g).tolist() for n in (5, 40, 130)]
    outs = e.generate(prompts, SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
    torch.cuda.synchronize()
    print("OK", model, "async", asyn, "steps", step[0], flush=True)
except Exception:
    traceback.print_exc()
    sys.stdout.flush(); sys.stderr.flush()
os._exit(0)
