"""Failure handling under injected faults (utils/faults.py): engine step failures fail only the
in-flight streams, a crashed or stalled DP replica is detected, its streams error out, its threads are re-routed and
the replica is respawned, a KV-starved pool preempts instead of failing, a down sandbox yields error tool results."""
import asyncio
import os
import time

import pytest

from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.utils import faults

CFG = dict(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048)


@pytest.fixture(autouse=True)
def _clean_faults():
    faults.reset({})
    yield
    faults.reset({})


def _collect(agen):
    async def go():
        out = []
        async for o in agen:
            out += o.new_token_ids
        return out
    return asyncio.run(go())


def test_route_skips_dead_replicas():
    from kafka_llm_service_amd.engine.client import route

    home = route("thread-7", 4, [0] * 4)
    alive = [True] * 4
    alive[home] = False
    alt = route("thread-7", 4, [0] * 4, alive)
    assert alt != home and alive[alt]
    assert route("thread-7", 4, [0] * 4, [False] * 4) == -1
    assert route(None, 3, [5, 1, 2], [True, False, True]) == 2


def test_step_failure_fails_inflight_then_recovers():
    from kafka_llm_service_amd.engine.async_engine import AsyncEngine

    ae = AsyncEngine(lambda: LLMEngine(EngineConfig(**CFG)))
    ae.start()
    try:
        faults.reset({"KAFKA_FI_STEP_ERROR_EVERY": "2"})
        ae.engine.fi = faults.get()
        sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
        with pytest.raises(faults.InjectedFault):
            _collect(ae.generate("a", list(range(100, 140)), sp))
        faults.reset({})
        ae.engine.fi = faults.get()
        out = _collect(ae.generate("b", list(range(100, 140)), sp))
        assert len(out) == 8
        assert ae.engine.num_running == 0 and ae.engine.num_waiting == 0
    finally:
        ae.shutdown()


def test_kv_pressure_preempts_instead_of_failing():
    faults.reset({"KAFKA_FI_KV_BLOCKS": "24"})
    eng = LLMEngine(EngineConfig(**CFG))
    assert eng.num_blocks == 24
    prompts = [list(range(1000 + 50 * i, 1000 + 50 * i + 60)) for i in range(4)]
    outs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True))
    assert all(len(o) == 40 for o in outs) and eng.sched.num_preemptions > 0
    faults.reset({})
    ref = LLMEngine(EngineConfig(**CFG), model=eng.model)
    assert ref.generate(prompts, SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True)) == outs


@pytest.mark.timeout(300)
def test_replica_crash_reroute_and_respawn(monkeypatch):
    from kafka_llm_service_amd.engine.client import DPClient

    monkeypatch.setenv("KAFKA_FI_WORKER_EXIT_AFTER", "3")
    cli = DPClient(EngineConfig(**CFG), 2)
    monkeypatch.delenv("KAFKA_FI_WORKER_EXIT_AFTER")  # respawned replicas are healthy
    sp_long = SamplingParams(temperature=0.0, max_tokens=20, ignore_eos=True)
    sp_short = SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True)
    prompt = list(range(200, 230))
    try:
        async def run():
            from kafka_llm_service_amd.engine.client import route

            home = route("t1", 2, [0, 0])
            with pytest.raises(RuntimeError, match="died"):
                async for _ in cli.generate("r1", prompt, sp_long, routing_key="t1"):
                    pass
            # while the home replica restarts, the thread is served by the other one
            toks = []
            async for o in cli.generate("r2", prompt, sp_short, routing_key="t1"):
                toks += o.new_token_ids
            assert len(toks) == 2
            for _ in range(240):
                if cli._alive[home] and cli.restarts[home] >= 1:
                    break
                await asyncio.sleep(0.5)
            assert cli._alive[home] and cli.restarts[home] >= 1
            toks = []
            async for o in cli.generate("r3", prompt, sp_short, routing_key="t1"):
                toks += o.new_token_ids
            assert len(toks) == 2
        asyncio.run(run())
    finally:
        asyncio.run(cli.close())


@pytest.mark.timeout(300)
def test_stalled_replica_is_killed_and_respawned(monkeypatch):
    from kafka_llm_service_amd.engine.client import DPClient

    monkeypatch.setenv("KAFKA_FI_SLOW_STEP_MS", "8000")
    cli = DPClient(EngineConfig(**CFG), 1, stall_timeout=3.0)
    monkeypatch.delenv("KAFKA_FI_SLOW_STEP_MS")
    try:
        async def run():
            t0 = time.monotonic()
            with pytest.raises(RuntimeError, match="died"):
                async for _ in cli.generate("s1", list(range(300, 320)),
                                            SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)):
                    pass
            assert time.monotonic() - t0 < 8.0  # killed by the stall detector, not by finishing the slow step
            for _ in range(240):
                if cli._alive[0] and cli.restarts[0] >= 1:
                    break
                await asyncio.sleep(0.5)
            toks = []
            async for o in cli.generate("s2", list(range(300, 320)),
                                        SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True)):
                toks += o.new_token_ids
            assert len(toks) == 2
        asyncio.run(run())
    finally:
        asyncio.run(cli.close())


def test_sandbox_down_gives_error_tool_result():
    from kafka_llm_service_amd.sandbox.base import SandboxError
    from kafka_llm_service_amd.sandbox.local import LocalSandbox

    faults.reset({"KAFKA_FI_SANDBOX_DOWN": "1"})
    sb = LocalSandbox("http://127.0.0.1:9")

    async def go():
        assert await sb.get_health_status() is None
        with pytest.raises(SandboxError, match="injected"):
            async for _ in sb.run_tool("shell_exec", {"command": "ls"}):
                pass
        await sb.close()
    asyncio.run(go())
    assert os.environ.get("KAFKA_FI_SANDBOX_DOWN") is None


def test_route_affinity_and_load_spill():
    from kafka_llm_service_amd.engine.client import route

    keys = [f"thread-{i}" for i in range(400)]
    homes = [route(k, 4, [0] * 4) for k in keys]
    assert homes == [route(k, 4, [0] * 4) for k in keys]            # stable
    assert all(homes.count(r) > 60 for r in range(4))                # spread over replicas
    k = keys[0]
    h = homes[0]
    loads = [0] * 4
    loads[h] = 100
    assert route(k, 4, loads, spill_min=48, spill_factor=2.0) != h   # hot spot spills to the least loaded
    loads = [30, 30, 30, 30]
    assert route(k, 4, loads, spill_min=48) == h                     # balanced: stay home


@pytest.mark.timeout(300)
def test_dp_warm_prefix_reaches_every_replica():
    from kafka_llm_service_amd.engine.client import DPClient, route

    cli = DPClient(EngineConfig(**CFG), 2)
    prefix = list(range(4000, 4000 + 96))
    try:
        async def run():
            await cli.warm_prefix(prefix)
            keys = {}
            for i in range(64):  # one thread key homed on each replica
                keys.setdefault(route(f"k{i}", 2, [0, 0]), f"k{i}")
            assert len(keys) == 2
            for r, k in keys.items():
                cached = 0
                async for o in cli.generate(f"after-{r}", prefix + [7, 8],
                                            SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True),
                                            routing_key=k):
                    cached = o.num_cached_tokens
                assert cached == 96, (r, cached)
        asyncio.run(run())
    finally:
        asyncio.run(cli.close())


@pytest.mark.timeout(300)
def test_dp_attention_group_serves_threads_over_http():
    """KAFKA_DP_ATTENTION: the two engine replicas of the API server are one DP-attention EP group (tiny Mixtral,
    CPU, gloo): threads routed to either rank stream their replies while both ranks step in lockstep."""
    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    cfg = ServerConfig(backend="engine", model="tiny-mixtral", sandbox="none", dp=2, dp_attention=True,
                       max_model_len=4096, default_max_tokens=6, prompt_sections=["intro"], warm_prefix=False,
                       ignore_eos=True, engine_kwargs={"device": "cpu", "num_kv_blocks": 512})
    st = ServerState(cfg, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        assert st.engine_client.dpa and st.engine_client.n_replicas == 2
        for i in range(4):
            tid = c.post("/v1/threads").json()["thread_id"]
            r = c.post(f"/v1/threads/{tid}/chat/completions",
                       json={"model": "m", "messages": [{"role": "user", "content": f"hi {i}"}], "stream": False,
                             "max_tokens": 6})
            assert r.status_code == 200 and r.json()["usage"]["completion_tokens"] == 6
            # health / metrics requests reach ONE rank of the idle group at a time: answered without a group
            # step (a lone rank entering the agreement would wait for peers that sleep on their pipes)
            for _ in range(3):
                assert c.get("/metrics").status_code == 200
                time.sleep(0.05)
