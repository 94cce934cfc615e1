"""Native KV block manager + prefix cache (runtime/csrc/kv_manager.cpp): unit + property tests (CPU)."""
import random

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from kafka_llm_service_amd.runtime import KVManager


def test_prefix_match_and_commit():
    kv = KVManager(64, 16, True)
    toks = list(range(100))
    assert kv.add_sequence(1, toks) == 0
    assert kv.ensure_capacity(1, 100)
    assert len(kv.block_table(1)) == 7
    kv.commit(1, 100)
    assert kv.num_cached_pages() == 6  # only full pages
    kv.free_sequence(1)
    assert kv.num_evictable() == 6  # the whole unreferenced chain
    # a new prompt sharing 70 tokens re-uses 4 full pages
    assert kv.add_sequence(2, toks[:70] + [999] * 10) == 64
    # a prompt identical to a cached prefix always leaves >= 1 token to compute
    assert kv.add_sequence(3, toks[:96]) == 80
    assert kv.check_invariants()


def test_dedup_on_commit():
    kv = KVManager(32, 16, True)
    toks = list(range(40))
    kv.add_sequence(1, toks)
    kv.add_sequence(2, toks)
    kv.ensure_capacity(1, 40)
    kv.ensure_capacity(2, 40)
    kv.commit(1, 40)
    kv.commit(2, 40)  # identical pages: seq 2 adopts seq 1's blocks
    assert kv.block_table(1)[:2] == kv.block_table(2)[:2]
    assert kv.common_prefix_blocks([1, 2]) == 2
    assert kv.check_invariants()
    kv.free_sequence(1)
    kv.free_sequence(2)
    assert kv.check_invariants()
    assert kv.num_free() + kv.num_evictable() + (kv.num_cached_pages() - kv.num_evictable()) == 32


def test_eviction_lru():
    kv = KVManager(8, 16, True)
    for sid, base in ((1, 0), (2, 1000)):
        t = list(range(base, base + 64))
        kv.add_sequence(sid, t)
        assert kv.ensure_capacity(sid, 64)
        kv.commit(sid, 64)
        kv.free_sequence(sid)
    assert kv.num_free() == 0 and kv.available() == 8
    # need 5 fresh blocks: evicts leaves LRU-first, seq 1's chain (older) first
    kv.add_sequence(3, list(range(5000, 5080)))
    assert kv.ensure_capacity(3, 80)
    assert kv.stats()["evictions"] == 5
    assert kv.check_invariants()
    assert kv.add_sequence(4, list(range(1000, 1064)) + [1]) == 48  # seq 2's chain survived (3 of 4 pages)


def test_capacity_failure_is_atomic():
    kv = KVManager(4, 16, False)
    kv.add_sequence(1, list(range(10)))
    assert not kv.ensure_capacity(1, 16 * 5)
    assert kv.num_free() == 4
    assert kv.ensure_capacity(1, 64)
    assert kv.num_free() == 0


def test_fill_helpers():
    kv = KVManager(16, 16, True)
    kv.add_sequence(7, list(range(40)))
    kv.ensure_capacity(7, 40)
    bt = np.zeros((2, 8), dtype=np.int32)
    kv.fill_block_tables([7], bt)
    assert list(bt[0, :3]) == kv.block_table(7)
    slots = np.zeros(5, dtype=np.int64)
    kv.fill_slots(7, 14, 19, slots, 0)
    b = kv.block_table(7)
    assert list(slots) == [b[0] * 16 + 14, b[0] * 16 + 15, b[1] * 16, b[1] * 16 + 1, b[1] * 16 + 2]
    with pytest.raises(RuntimeError):
        kv.fill_slots(7, 40, 60, np.zeros(20, dtype=np.int64), 0)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 3), st.integers(0, 5), st.integers(1, 90)), min_size=1, max_size=60),
       st.booleans())
def test_random_ops_keep_invariants(ops, prefix_cache):
    """Random admit / grow / commit / free traffic never double-owns or leaks a block."""
    kv = KVManager(24, 16, prefix_cache)
    live = {}
    rng = random.Random(0)
    base = [rng.randrange(50) for _ in range(200)]
    sid = 0
    for op, a, n in ops:
        if op == 0 and len(live) < 6:
            sid += 1
            toks = base[:n] if a % 2 == 0 else [rng.randrange(50) for _ in range(n)]
            kv.add_sequence(sid, toks)
            live[sid] = len(toks)
        elif op == 1 and live:
            s = sorted(live)[a % len(live)]
            if kv.ensure_capacity(s, live[s] + a):
                kv.append_tokens(s, np.arange(a, dtype=np.int32))
                live[s] += a
        elif op == 2 and live:
            s = sorted(live)[a % len(live)]
            if kv.ensure_capacity(s, live[s]):
                kv.commit(s, live[s])
        elif op == 3 and live:
            s = sorted(live)[a % len(live)]
            kv.free_sequence(s)
            del live[s]
        assert kv.check_invariants()
    for s in list(live):
        kv.free_sequence(s)
    assert kv.check_invariants()
    assert kv.available() == 24


def test_plan_channel_ring_order_backpressure_and_timeout():
    """Native shared-memory plan ring (runtime/csrc/plan_channel.cpp): followers see every plan in order (zero-copy
    views), the leader blocks (bounded) when a follower falls nslots - 1 plans behind, and a dead peer is a
    RuntimeError after the timeout instead of a hang."""
    import os
    import threading

    import numpy as np
    import pytest

    from kafka_llm_service_amd.runtime import native

    rt = native()
    name = f"/kafka_plan_test_{os.getpid()}"
    lead = rt.PlanChannel(name, 3, 4096, 2)
    fol = [rt.PlanChannel(name, i) for i in range(2)]
    got = {0: [], 1: []}

    def follower(i):
        for _ in range(10):
            h, p = fol[i].recv(10.0)
            got[i].append((int(h[1]), bytes(p[:4]), p.size))
            fol[i].ack()

    ts = [threading.Thread(target=follower, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for k in range(10):
        hdr = np.zeros(32, dtype=np.int64)
        hdr[1] = k
        lead.publish(hdr, np.full(100 + k, k, dtype=np.uint8), 10.0)
    for t in ts:
        t.join(10)
    for i in range(2):
        assert got[i] == [(k, bytes([k] * 4), 100 + k) for k in range(10)]
    # back-pressure: with no consumer the leader can run nslots ahead, then times out
    for _ in range(3):
        lead.publish(np.zeros(32, dtype=np.int64), np.zeros(8, dtype=np.uint8), 1.0)
    with pytest.raises(RuntimeError, match="timeout"):
        lead.publish(np.zeros(32, dtype=np.int64), np.zeros(8, dtype=np.uint8), 0.05)
    with pytest.raises(Exception):
        lead.publish(np.zeros(32, dtype=np.int64), np.zeros(8192, dtype=np.uint8), 1.0)  # larger than a slot
    # a follower whose leader stopped publishing times out
    for f in fol:
        for _ in range(3):
            f.recv(1.0)
            f.ack()
    with pytest.raises(RuntimeError, match="timeout"):
        fol[0].recv(0.05)
    for f in fol:
        f.close()
    lead.close()
    assert not os.path.exists(f"/dev/shm{name}")


def test_plan_channel_idle_follower_waits_until_leader_exits():
    """a follower waiting for the next plan must not time out while its leader is merely idle, and must
    fail at once when the leader PROCESS is gone; the leader unlinks the name once the followers have attached
    (a group killed with SIGKILL leaves nothing in /dev/shm)."""
    import os
    import subprocess
    import sys
    import threading
    import time

    import pytest

    from kafka_llm_service_amd.runtime import native

    rt = native()
    name = f"/kafka_plan_idle_{os.getpid()}"
    code = ("import sys, time; sys.path.insert(0, %r); from kafka_llm_service_amd.runtime import native; "
            "ch = native().PlanChannel(%r, 3, 4096, 1); print('up', flush=True); sys.stdin.readline(); "
            "ch.unlink(); print('unlinked', flush=True); time.sleep(600)") % (os.getcwd(), name)
    lead = subprocess.Popen([sys.executable, "-c", code], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert lead.stdout.readline().strip() == "up"
        fol = rt.PlanChannel(name, 0)
        lead.stdin.write("go\n")
        lead.stdin.flush()
        assert lead.stdout.readline().strip() == "unlinked"
        assert not os.path.exists(f"/dev/shm{name}")  # attached mappings outlive the name
        err = []

        def wait():
            try:
                fol.recv(-1.0)
            except RuntimeError as e:
                err.append((time.monotonic(), str(e)))

        t = threading.Thread(target=wait, daemon=True)
        t.start()
        time.sleep(1.5)  # idle leader: the follower keeps waiting (a bounded wait would have raised by now)
        assert t.is_alive() and not err
        t_kill = time.monotonic()
        lead.kill()
        lead.wait()
        t.join(5)
        assert err and "gone" in err[0][1] and err[0][0] - t_kill < 2.0
        fol.close()
    finally:
        if lead.poll() is None:
            lead.kill()
    with pytest.raises(RuntimeError):
        rt.PlanChannel(name, 0)  # nothing left to attach to


def test_page_runs_contiguous_and_invariants():
    """run = 16: a sequence's decode growth comes in runs of consecutive block ids (the spare pages reserved for it),
    a prefill chunk is one run, reserves are reclaimed when the pool runs short, and every page stays in exactly
    one place (free set, a table, a reserve or the tree) under random admit / grow / commit / free traffic."""
    import random

    import numpy as np

    kv = KVManager(600, 16, True, 16)
    assert kv.run == 16
    kv.add_sequence(1, np.arange(1, 200, dtype=np.int32))
    assert kv.ensure_capacity(1, 199)
    bt = kv.block_table(1)
    assert bt == list(range(bt[0], bt[0] + len(bt)))  # one run for the prefill
    for n in range(200, 200 + 16 * 20):  # decode growth: consecutive within each run of 16
        assert kv.ensure_capacity(1, n)
    bt = kv.block_table(1)
    jumps = sum(1 for a, b in zip(bt, bt[1:]) if b != a + 1)
    assert jumps <= 21 and kv.num_reserved() <= 15 and kv.check_invariants()
    rng = random.Random(7)
    live = {1: 200 + 16 * 20}
    for step in range(400):
        op = rng.random()
        if op < 0.2 and len(live) < 12:
            sid = 100 + step
            toks = np.array([rng.randrange(1, 50) for _ in range(rng.randrange(2, 120))], dtype=np.int32)
            kv.add_sequence(sid, toks)
            if kv.ensure_capacity(sid, len(toks)):
                live[sid] = len(toks)
            else:
                kv.free_sequence(sid)
        elif op < 0.75 and live:
            sid = rng.choice(list(live))
            if kv.ensure_capacity(sid, live[sid] + 1):
                kv.append_token(sid, rng.randrange(1, 50))
                live[sid] += 1
                kv.commit(sid, live[sid] - 1)
        elif live:
            sid = rng.choice(list(live))
            kv.free_sequence(sid)
            del live[sid]
        assert kv.check_invariants(), step
    assert kv.available() >= kv.num_free()


def test_reserves_reclaimed_before_cached_pages_are_evicted():
    """A sequence's speculative page reserve (run > 1) goes back to the pool before any cached prefix page is evicted
    (the cache exists for the agent workloads' shared prefixes; a reserve is only a guess)."""
    kv = KVManager(48, 16, True, 16)
    pre = list(range(1, 65))
    kv.add_sequence(1, pre)
    assert kv.ensure_capacity(1, 64)
    kv.commit(1, 64)
    kv.free_sequence(1)
    assert kv.num_evictable() == 4
    kv.add_sequence(2, [7])
    assert kv.ensure_capacity(2, 1) and kv.ensure_capacity(2, 17)  # decode growth: a run, most of it reserved
    assert kv.num_reserved() > 0
    kv.add_sequence(3, list(range(1000, 1000 + 16 * 30)))
    assert kv.ensure_capacity(3, 16 * 30)  # needs more than the free set: reserves first
    assert kv.stats()["evictions"] == 0 and kv.num_reserved() == 0
    assert kv.add_sequence(4, pre + [5]) == 64  # the cached prefix survived
    assert kv.check_invariants()
