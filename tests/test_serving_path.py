"""The API <-> engine-process serving path (CPU): prompts sent by reference to the pinned shared prefix, the
incremental detokenizer's one-decode fast path, and the timing-only fake engine used for API load tests."""
import multiprocessing as mp
import random
import threading

from kafka_llm_service_amd.engine.client import serve_pipe
from kafka_llm_service_amd.engine.fake import FakeEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.engine.tokenizer import IncrementalDetokenizer, get_tokenizer


class _Recorder(FakeEngine):
    def __init__(self):
        super().__init__(step_ms=0.5)
        self.prompts = {}

    def add_request(self, request_id, prompt_ids, params=None, meta=None):
        self.prompts[request_id] = list(prompt_ids)
        super().add_request(request_id, prompt_ids, params, meta)


def test_prompt_by_reference_to_the_pinned_prefix():
    """("ref", n, suffix) is rebuilt as pinned[:n] + suffix; a reference before any pin is an error frame."""
    a, b = mp.Pipe()
    eng = _Recorder()
    t = threading.Thread(target=serve_pipe, args=(eng, b), daemon=True)
    t.start()
    sp = SamplingParams(max_tokens=2).__dict__
    sp = {k: v for k, v in sp.items() if k != "allowed_tokens_fn"}
    a.send(("add", "r0", ("ref", 3, [9, 9]), sp, 0.0))  # nothing pinned yet
    pin = list(range(100, 140))
    a.send(("pin", pin))
    a.send(("add", "r1", ("ref", 40, [7, 8]), sp, 0.0))
    a.send(("add", "r2", ("ref", 10, [5]), sp, 0.0))
    a.send(("add", "r3", [1, 2, 3], sp))  # plain list, no send timestamp (older senders)
    errors, done = [], set()
    while len(done) < 3:
        msg = a.recv()
        if msg[0] == "error":
            errors.append(msg[1])
        elif msg[0] == "out":
            done |= {o[0] for o in msg[1] if o[2]}
    a.send(("stop",))
    t.join(timeout=10)
    assert errors == ["r0"]
    assert eng.prompts["r1"] == pin + [7, 8]
    assert eng.prompts["r2"] == pin[:10] + [5]
    assert eng.prompts["r3"] == [1, 2, 3]


def test_incremental_detokenizer_fast_path_matches_window_diff():
    """The one-decode-per-token path streams exactly the text of the two-window diff it replaces, including
    multi-byte characters split over tokens and random (pseudo-word / special) ids."""
    tok = get_tokenizer()

    class Window:
        def __init__(self):
            self.ids, self.p, self.r = [], 0, 0

        def add(self, new):
            self.ids.extend(new)
            pre, full = tok.decode(self.ids[self.p:self.r]), tok.decode(self.ids[self.p:])
            if len(full) <= len(pre) or full.endswith("�"):
                return ""
            d = full[len(pre):]
            self.p, self.r = self.r, len(self.ids)
            return d

    rng = random.Random(3)
    base = tok.encode("Hello wörld — ünïcödé 漢字 emoji 😀 test\n" * 3)
    for _ in range(400):
        ids = [rng.choice(base + [rng.randrange(0, 128256) for _ in range(2)]) for _ in range(rng.randint(1, 40))]
        fast, ref = IncrementalDetokenizer(tok), Window()
        assert "".join(fast.add([i]) for i in ids) == "".join(ref.add([i]) for i in ids)


def test_fake_engine_paces_steps_and_finishes_by_length():
    import time

    eng = FakeEngine(step_ms=2.0, prefill_us_per_token=0.0)
    eng.add_request("a", [1] * 10, SamplingParams(max_tokens=3))
    eng.add_request("b", [1] * 10, SamplingParams(max_tokens=1))
    t0 = time.perf_counter()
    outs = []
    while eng.has_unfinished():
        outs += eng.step()
    assert time.perf_counter() - t0 >= 3 * 2e-3 * 0.9
    assert [o.request_id for o in outs if o.finished] == ["b", "a"]
    assert sum(o.request_id == "a" for o in outs) == 3
