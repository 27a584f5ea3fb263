"""Pin the CPU oracle against the reference's own golden vectors and property
tests (vecfc/forkless_cause_test.go).  CPU only."""

import pytest

from oracle import pos, tdag
from oracle import vecfc_oracle as vo
from device_model import DeviceModel


def build_index(scheme):
    nodes, _, names, ordered = tdag.ascii_scheme_for_each(scheme)
    validators = pos.Validators.equal(nodes, 1)
    store = {}
    ix = vo.Index()
    ix.reset(validators, store.get)
    for e in ordered:
        store[e.id] = e
        ix.add(e)
        ix.flush()
    return ix, names, ordered


@pytest.mark.parametrize("case", ["classic_step3", "classic_step4", "classic_step5", "random_80"])
def test_forkless_caused_golden(golden, case):
    """TestForklessCausedClassic (:82-123) and TestForklessCausedRandom (:195-483)."""
    c = next(x for x in golden["fc_cases"] if x["name"] == case)
    ix, names, _ = build_index(c["scheme"])
    assert set(names) == set(c["fc"])
    for who, e1 in names.items():
        for whom, e2 in names.items():
            expect = whom in c["fc"][who]
            assert ix.forkless_cause(e1.id, e2.id) == expect, (who, whom)


def test_ascii_parser_structure(golden):
    """The parser restatement yields the documented shapes: 4 validators and
    80 events (20 per validator, seq 1..20) for the random golden DAG; 15
    validators for the benchmark DAG."""
    c = next(x for x in golden["fc_cases"] if x["name"] == "random_80")
    nodes, events, names, ordered = tdag.ascii_scheme_for_each(c["scheme"])
    assert len(nodes) == 4 and len(ordered) == 80
    for v in nodes:
        assert [e.seq for e in events[v]] == list(range(1, 21))
    b = next(x for x in golden["fc_cases"] if x["name"] == "bench_15")
    nodes, _, _, ordered = tdag.ascii_scheme_for_each(b["scheme"])
    assert len(nodes) == 15 and len(ordered) == 29


def naive_forks_detected(ix, head):
    """testForksDetected (forkless_cause_test.go:491-518)."""
    visited = set()
    detected = {}

    def walk(eid):
        if eid in visited:
            return False
        visited.add(eid)
        e = ix.get_event(eid)
        k = (e.seq, e.creator)
        detected[k] = detected.get(k, 0) + 1
        return True

    walk(head.id)
    ix.dfs_subgraph(head, walk)
    return {k[1] for k, n in detected.items() if n > 1}


def test_random_forks_sanity():
    """TestRandomForksSanity (:520-576): skewed weights, 3 cheaters; merged HB
    of every node's last event flags exactly the cheaters with Seq 0."""
    n = 8
    rng = tdag.SplitMix64(42)
    node_ids = [rng.next() & 0xFFFFFFFF for _ in range(n)]
    w = {v: 1 for v in node_ids}
    w[node_ids[0]] = 2
    w[node_ids[3]] = 2
    w[node_ids[4]] = 3
    validators = pos.Validators(w)
    nodes, evs = tdag.rand_fork_dag(n, 120, 4, cheaters=3, forks_count=30, seed=5, node_ids=node_ids)
    store = {e.id: e for e in evs}
    ix = vo.Index()
    ix.reset(validators, store.get)
    last = {}
    for e in evs:
        ix.add(e)
        last[e.creator] = e
    ix.flush()
    ix.drop_not_flushed()
    for node in nodes:
        mhb = ix.get_merged_highest_before(last[node].id)
        for k, cheater in enumerate(nodes):
            bs = mhb.get(validators.idxs[cheater])
            if k < 3:
                assert bs == vo.FORK_DETECTED
            else:
                assert bs != vo.FORK_DETECTED and bs[0] != 0


RANDOM_FORKS = [  # TestRandomForks parameter table (:579-650)
    dict(nodes=1, parents=1, cheaters=1, events=10, forks=3, reorder=30),
    dict(nodes=2, parents=1, cheaters=1, events=10, forks=3, reorder=20),
    dict(nodes=2, parents=2, cheaters=2, events=10, forks=20, reorder=5),
    dict(nodes=10, parents=4, cheaters=1, events=10, forks=3, reorder=5),
    dict(nodes=10, parents=4, cheaters=10, events=10, forks=3, reorder=3),
    dict(nodes=20, parents=4, cheaters=10, events=5, forks=2, reorder=3),
    dict(nodes=40, parents=4, cheaters=10, events=3, forks=1, reorder=2),
    dict(nodes=5, parents=4, cheaters=2, events=30, forks=30, reorder=2),
]


@pytest.mark.parametrize("i", range(len(RANDOM_FORKS)))
def test_random_forks(i):
    """TestRandomForks (:578-747): fork flags == naive duplicate-(creator,seq)
    DFS; DropNotFlushed erases unflushed vectors; FC invariant under random
    topological reorderings."""
    t = RANDOM_FORKS[i]
    rng = tdag.SplitMix64(1000 + i)
    node_ids = [rng.next() & 0xFFFFFFFF for _ in range(t["nodes"])]
    nodes, evs = tdag.rand_fork_dag(t["nodes"], t["events"], t["parents"], cheaters=t["cheaters"],
                                    forks_count=t["forks"], seed=i, node_ids=node_ids)
    validators = pos.Validators.equal(nodes, 1)
    store = {e.id: e for e in evs}
    ix = vo.Index()
    ix.reset(validators, store.get)
    for e in evs:
        ix.add(e)
    for e in evs:
        hb = ix.get_highest_before(e.id)
        expected = naive_forks_detected(ix, e)
        for v in nodes:
            bs = hb.get(validators.idxs[v])
            assert (bs == vo.FORK_DETECTED) == (v in expected)
            if v in expected:
                assert bs[0] == 0
    fc = {(a.id, b.id): ix.forkless_cause(a.id, b.id) for a in evs for b in evs}
    ix.drop_not_flushed()
    for e in evs:
        assert ix.get_highest_before(e.id) is None
        assert ix.get_lowest_after(e.id) is None
    order = evs
    for _ in range(t["reorder"]):
        order = tdag.by_parents(tdag.shuffle(order, rng))
        for e in order:
            ix.add(e)
        for a in order:
            for b in order:
                assert ix.forkless_cause(a.id, b.id) == fc[(a.id, b.id)]
        ix.drop_not_flushed()


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("shape", [(10, 4, 10, 10, 3), (5, 4, 2, 30, 30), (8, 4, 3, 40, 30), (40, 4, 10, 3, 1)])
def test_device_model_matches_oracle(seed, shape):
    """The algorithm the HIP kernels implement (max-join RAW plane, per-creator
    overlap marks, LowestAfter by range fill; tests/device_model.py) yields the
    oracle's exact HB/LA byte rows and FC on fork-heavy DAGs."""
    n, p, ch, ev, fk = shape
    rng = tdag.SplitMix64(seed * 100 + 7)
    ids = [rng.next() & 0xFFFFFFFF for _ in range(n)]
    nodes, evs = tdag.rand_fork_dag(n, ev, p, cheaters=ch, forks_count=fk, seed=seed * 1000 + n, node_ids=ids)
    validators = pos.Validators.equal(nodes, 1)
    store = {e.id: e for e in evs}
    ix = vo.Index()
    ix.reset(validators, store.get)
    dm = DeviceModel(validators)
    for e in evs:
        ix.add(e)
        dm.add(e)
    for e in evs:
        assert ix.get_highest_before(e.id).to_bytes() == dm.hb_bytes(e.id)
        assert ix.get_lowest_after(e.id).to_bytes() == dm.la_bytes(e.id)
    for a in evs[::3]:
        for b in evs:
            assert ix.forkless_cause(a.id, b.id) == dm.forkless_cause(a.id, b.id)
