"""Debug: two fp8 engines in one process (eager, then graphs) — ticket buffers and first-step logits."""
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.models.oracle import dense_logits


def state(tag):
    dev = torch.device("cuda", 0)
    t = ops._TICKETS.get(dev)
    w = ops._SAMPLE_WS.get(dev)
    print(tag, "decode tickets nonzero:", None if t is None else int((t != 0).sum()),
          "sampler tickets nonzero:", None if w is None else int((w[:65536] != 0).sum()), flush=True)


def run(graphs):
    eng = LLMEngine(EngineConfig(model="small-llama", device="cuda:0", num_kv_blocks=1024, max_model_len=4096,
                                 kv_dtype="fp8", use_graphs=graphs))
    g = torch.Generator().manual_seed(11)
    pre = torch.randint(0, 5000, (600,), generator=g).tolist()
    prompts = [pre + torch.randint(0, 5000, (n,), generator=g).tolist() for n in (3, 60, 150, 7)]
    outs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
    torch.cuda.synchronize()
    gaps = []
    for p, o in zip(prompts, outs):
        lg = dense_logits(eng.model, p + o)
        gaps.append([round((lg[len(p) - 1 + i].max() - lg[len(p) - 1 + i][t]).item(), 2) for i, t in enumerate(o)])
    print("graphs" if graphs else "eager", "max gap per prompt", [max(x) for x in gaps], flush=True)
    return eng


state("start")
e1 = run(False)
state("after eager")
del e1
torch.cuda.synchronize()
e2 = run(True)
state("after graphs")
