"""Batcher -> HIP index: events arriving in random order (children before
parents) are buffered by the level-synchronous batcher and indexed one popped
batch at a time (lx_add_batch per pop).  Rows, branch IDs, merged HB and
ForklessCause equal the oracle fed the same release order, bit for bit."""

import numpy as np
import pytest

from oracle import corc, pos, tdag

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(16, 30, 5, 0, 0, 1), (24, 30, 6, 5, 6, 2), (100, 10, 10, 10, 3, 3)])
def test_batched_ingest_matches_oracle(shape):
    import lachesis_hip as lx
    n, epn, p, ch, fk, seed = shape
    nodes, events = tdag.rand_fork_dag(n, epn, p, ch, fk, seed=seed)
    rng = np.random.default_rng(seed)
    w = {v: int(x) for v, x in zip(nodes, rng.integers(1, 50, n))}
    validators = pos.Validators(w)
    ix = lx.VecfcIndex()
    ix.reset(validators)
    b = lx.batcher.LevelBatcher()
    order = rng.permutation(len(events))
    i, pops = 0, 0
    while i < len(order):
        k = int(rng.integers(1, 4 * n))
        b.push([events[j] for j in order[i:i + k]], validators)
        i += k
        if b.drain_into(ix):
            pops += 1
    assert b.peek()[3] == 0 and len(ix.ids) == len(events) and pops > 1
    by_id = {e.id: e for e in events}
    released = [by_id[x] for x in ix.ids]
    o = corc.OracleIndex(validators.weights)
    assert o.add_batch(*tdag.to_dense(released, validators)) == -1
    for d in range(len(released)):
        assert ix.ix.highest_before(d) == o.hb(d), d
        assert ix.ix.lowest_after(d) == o.la(d), d
        assert ix.ix.branch(d) == o.branch(d), d
        assert ix.ix.merged_highest_before(d) == o.merged_hb(d), d
    lam = np.array([e.lamport for e in released], dtype=np.uint32)
    qa, qb = lx.tools.fc_queries(lam, 50_000, window=32, seed=seed)
    np.testing.assert_array_equal(ix.ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))


def test_drain_isolates_a_rejected_event():
    """One event violating the eventcheck invariants (seq != self-parent seq + 1)
    arrives among valid ones: drain_all rejects exactly it (the reference's
    Process returns an error for that event only), indexes every event that
    does not descend from it, and leaves its descendants pending; the indexed
    part equals the oracle fed the same release order."""
    import lachesis_hip as lx
    nodes, events = tdag.rand_fork_dag(12, 20, 4, 0, 0, seed=4)
    validators = pos.Validators.equal(nodes)
    k = 60
    e = events[k]
    events = list(events)
    events[k] = tdag.Event(e.id, e.creator, e.seq + 7, e.lamport, e.parents, e.name)
    desc, frontier = set(), {e.id}
    for x in events[k + 1:]:
        if any(p in frontier for p in x.parents):
            desc.add(x.id)
            frontier.add(x.id)
    ix = lx.VecfcIndex()
    ix.reset(validators)
    b = lx.batcher.LevelBatcher()
    rng = np.random.default_rng(4)
    order = rng.permutation(len(events))
    rejected = []
    for i in range(0, len(order), 37):
        b.push([events[j] for j in order[i:i + 37]], validators)
        b.drain_all(ix, validators, lambda ev, err: rejected.append((ev.id, err.code)))
    assert rejected == [(e.id, -3)]
    assert set(ix.ids) == {x.id for x in events} - {e.id} - desc
    assert b.peek()[3] == len(desc) > 0
    by_id = {x.id: x for x in events}
    released = [by_id[x] for x in ix.ids]
    o = corc.OracleIndex(validators.weights)
    assert o.add_batch(*tdag.to_dense(released, validators)) == -1
    for d in range(len(released)):
        assert ix.ix.highest_before(d) == o.hb(d), d
        assert ix.ix.lowest_after(d) == o.la(d), d
    N = len(released)
    a = np.repeat(np.arange(N, dtype=np.uint32), N)
    c = np.tile(np.arange(N, dtype=np.uint32), N)
    np.testing.assert_array_equal(ix.ix.forkless_cause_batch(a, c), o.forkless_cause_batch(a, c))
