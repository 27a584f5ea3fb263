"""The level-synchronous batcher (include/lachesis_batcher.h) on the host: no
GPU needed.  Events arrive shuffled (children before parents) in random
chunks; every pop must be a parents-first batch grouped in antichain levels,
release every event exactly once as soon as its ancestors are known, and keep
EventsBuffer's duplicate semantics (gossip/dagordering/event_buffer.go:53-110).
Indexing in the released order gives the same ForklessCause relation as the
creation order (vecfc/forkless_cause_test.go:719-744, reorder invariance)."""

import numpy as np
import pytest

from oracle import corc, pos, tdag


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def drain(lx, events, validators, seed, chunk_max=40, capacity=0):
    rng = np.random.default_rng(seed)
    order = list(rng.permutation(len(events)))
    b = lx.batcher.LevelBatcher(capacity)
    released, batches = [], []
    i = 0
    while i < len(order):
        n = int(rng.integers(1, chunk_max))
        st = b.push([events[k] for k in order[i:i + n]], validators)
        assert (st == 0).all()
        i += n
        evs, cr, sq, off, par, lev, first = b.pop()
        assert first == len(released)
        batches.append((evs, off, par, lev, first))
        released.extend(evs)
    assert b.peek()[3] == 0          # nothing left waiting
    return b, released, batches


@pytest.mark.parametrize("shape", [(8, 20, 3, 0, 0, 1), (12, 25, 4, 3, 5, 2), (30, 10, 6, 6, 4, 3)])
def test_batches_are_parents_first_levels(lx, shape):
    n, epn, p, ch, fk, seed = shape
    nodes, events = tdag.rand_fork_dag(n, epn, p, ch, fk, seed=seed)
    validators = pos.Validators.equal(nodes, 1)
    b, released, batches = drain(lx, events, validators, seed)
    assert sorted(e.id for e in released) == sorted(e.id for e in events)
    dense = {e.id: i for i, e in enumerate(released)}
    for evs, off, par, lev, first in batches:
        level = {}
        for li in range(len(lev) - 1):
            for k in range(int(lev[li]), int(lev[li + 1])):
                e = evs[k]
                got = [int(x) for x in par[int(off[k]):int(off[k + 1])]]
                assert got == [dense[q] for q in e.parents]          # dense parents, self-parent first
                assert all(x < first + k for x in got)               # parents first
                inb = [level[q] for q in e.parents if q in level]
                assert li + 1 == 1 + max(inb, default=0)             # level = 1 + max in-batch parent level
                level[e.id] = li + 1
        for k, e in enumerate(evs):
            assert dense[e.id] == first + k


def test_release_order_keeps_forkless_cause(lx):
    nodes, events = tdag.rand_fork_dag(10, 30, 4, 3, 6, seed=7)
    w = {v: 10 + i for i, v in enumerate(nodes)}
    validators = pos.Validators(w)
    _, released, _ = drain(lx, events, validators, 7)
    a = corc.OracleIndex(validators.weights)
    assert a.add_batch(*tdag.to_dense(events, validators)) == -1
    b = corc.OracleIndex(validators.weights)
    assert b.add_batch(*tdag.to_dense(released, validators)) == -1
    pa = {e.id: i for i, e in enumerate(events)}
    pb = {e.id: i for i, e in enumerate(released)}
    ids = [e.id for e in events]
    for x in ids[::3]:
        for y in ids[::2]:
            assert a.forkless_cause(pa[x], pa[y]) == b.forkless_cause(pb[x], pb[y])


def test_duplicates_unpop_and_reset(lx):
    nodes, events = tdag.rand_fork_dag(4, 6, 3, seed=5)
    validators = pos.Validators.equal(nodes, 1)
    b = lx.batcher.LevelBatcher()
    st = b.push(events[5:], validators)
    assert (st == 0).all()
    assert b.push(events[5:6], validators)[0] == lx.batcher.PUSH_DUPLICATE
    b.push(events[:5], validators)
    ne, _, nl, nw = b.peek()
    assert ne == len(events) and nw == 0 and nl >= 1
    evs, *_ = b.pop()
    assert b.push(events[:1], validators)[0] == lx.batcher.PUSH_CONNECTED
    b.unpop(evs)                        # the index rejected the batch: forget it
    assert b.peek()[0] == 0
    b.push(evs, validators)
    evs2, *_rest = b.pop()
    assert [e.id for e in evs2] == [e.id for e in evs]   # same order, same dense indices
    b.reset()
    assert b.peek() == (0, 0, 0, 0)
    b.push(events, validators)
    assert b.peek()[0] == len(events)


def test_reserve_changes_nothing(lx):
    """lx_batcher_reserve is a capacity hint: the same pops with and without it
    (and the id table rebuilt mid-epoch keeps the released ids)."""
    nodes, events = tdag.rand_fork_dag(16, 30, 4, 3, 4, seed=7)
    validators = pos.Validators.equal(nodes, 1)
    _, rel0, bat0 = drain(lx, events, validators, seed=5)
    _, rel1, bat1 = drain(lx, events, validators, seed=5, capacity=100_000)
    assert [e.id for e in rel0] == [e.id for e in rel1]
    for x, y in zip(bat0, bat1):
        assert [e.id for e in x[0]] == [e.id for e in y[0]] and list(x[2]) == list(y[2]) and list(x[3]) == list(y[3])
