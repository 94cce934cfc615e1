"""Debug: TP=2 on one GPU (gloo + optional custom all-reduce) vs TP=1 — first-step logits difference."""
import os
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.test_custom_allreduce_gpu import CFG, _capture_logits, _port, _prompts, _tp_main  # noqa: E402


def main():
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams

    ref = LLMEngine(EngineConfig(**dict(CFG, device="cuda:0")))
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    want_outs, want = _capture_logits(ref, _prompts(ref.model_cfg.vocab_size), sp)
    for custom in sys.argv[1:] or ["0", "1"]:
        os.environ["KAFKA_CUSTOM_AR"] = custom
        os.environ["KAFKA_DECODE_GEMM"] = os.environ.get("DBG_GEMM", "auto")
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_tp_main, args=(r, 2, port, q, False)) for r in range(2)]
        for p in ps:
            p.start()
        res = {}
        for _ in ps:
            m = q.get(timeout=240)
            res[m[0]] = m[1:]
        for p in ps:
            p.join(timeout=60)
        outs, seen, _, _ = res["leader"]
        d = [(torch.from_numpy(a) - b).abs().max().item() for a, b in zip(seen, want)]
        print(f"custom={custom} step logit max diffs {['%.3f' % x for x in d]} outs {outs} want {want_outs}",
              flush=True)


if __name__ == "__main__":
    main()
