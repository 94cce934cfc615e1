"""hipGraph decode runner (engine/graphs.py) with the CPU 'fake' backend: a captured step must read only its static
buffers, so replays with new tokens / positions / slots / block tables / seeds give exactly the eager results."""
from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams


def _run(use_graphs, model=None):
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048,
                                 use_graphs=use_graphs, cascade_min_prefix=32), model=model)
    eng.runner.fixed_decode_items = True  # the graphed runner's decode plan (decode_items_fixed) for both runs
    shared = list(range(500, 548))
    prompts = [shared + list(range(900 + 10 * i, 905 + 13 * i)) for i in range(5)]
    params = [SamplingParams(temperature=0.0, max_tokens=9, ignore_eos=True)] * 2 + \
        [SamplingParams(temperature=0.9, top_p=0.9, max_tokens=11, ignore_eos=True, seed=i) for i in range(3)]
    return eng.generate(prompts[:2], params[:2]) + eng.generate(prompts[2:], params[2:]), eng


def test_graph_replays_match_eager():
    eager, e0 = _run(False)
    graphed, e1 = _run(True, model=e0.model)
    assert graphed == eager
    st = e1.runner.graphs.stats
    assert st["captures"] >= 2 and st["replays"] > st["captures"] and not e1.runner.graphs.disabled
