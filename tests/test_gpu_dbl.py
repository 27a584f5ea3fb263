"""k_dbl (lx_dbl.hip): HighestBefore by frontier doubling for fork-free
batches with few branches (BASELINE configs[0]: 5 validators x 1000 events,
a 5,000-level chain).  Rows, branches and ForklessCause must equal the C
oracle and the column walker (option dbl=0) bit for bit, for one batch and
for several batches on top of each other (older parents folded from their
final rows), parents beyond the inline twelve, and a single chain."""

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu

SHAPES = {
    "c1": (5, 1000, 5),        # configs[0]
    "chain": (1, 3000, 1),     # one validator: every event its own level
    "v3": (3, 900, 3),
    "v8p16": (8, 300, 16),     # parents beyond the inline twelve
    "v16": (16, 200, 10),
}


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def oracle_for(d, w):
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    return o


def index_of(lx, d, w, cuts, dbl):
    ix = lx.Index(options={"small_max": 0, "dbl": 1 if dbl else 0})
    ix.reset(w)
    for lo, hi in zip(cuts, cuts[1:]):
        ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
    return ix


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("split", [1, 3])
def test_doubling_equals_oracle_and_walker(lx, shape, split):
    V, epv, P = SHAPES[shape]
    d = lx.tools.gen_dag(V, epv, P, seed=11 + V)
    N = len(d)
    w = [1 + (i % 3) for i in range(V)]
    cuts = [N * k // split for k in range(split + 1)]
    o = oracle_for(d, w)
    ix = index_of(lx, d, w, cuts, True)
    wk = index_of(lx, d, w, cuts, False)
    for i in list(range(0, N, 7)) + [N - 1]:
        assert ix.highest_before(i) == o.hb(i), ("hb", i)
        assert ix.lowest_after(i) == o.la(i), ("la", i)
        assert ix.highest_before(i) == wk.highest_before(i)
        assert ix.lowest_after(i) == wk.lowest_after(i)
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=64, seed=V)
    want = o.forkless_cause_batch(qa, qb)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), want)
    np.testing.assert_array_equal(wk.forkless_cause_batch(qa, qb), want)
    ix.close()
    wk.close()


def test_doubling_then_rollback_and_forks(lx):
    """A fork-free epoch indexed by k_dbl, a DropNotFlushed of its second batch,
    then batches with fork branches (the walker takes over once B > V): every
    row still equals the oracle."""
    d = lx.tools.gen_dag(6, 400, 4, cheaters=2, forks=3, seed=5)
    w = [3, 2, 2, 1, 1, 1]
    N = len(d)
    # the first fork branch opens at the first event whose branch is >= V
    o = oracle_for(d, w)
    first_fork = next(i for i in range(N) if o.branch(i) >= 6)
    a = first_fork // 2
    ix = lx.Index(options={"small_max": 0})
    ix.reset(w)
    ix.add_batch(d.creator[:a], d.seq[:a], d.poff[:a + 1], d.par)
    ix.flush()
    ix.add_batch(d.creator[a:first_fork], d.seq[a:first_fork], d.poff[a:first_fork + 1], d.par)
    ix.drop_not_flushed()
    assert ix.num_events() == a
    ix.add_batch(d.creator[a:first_fork], d.seq[a:first_fork], d.poff[a:first_fork + 1], d.par)
    ix.add_batch(d.creator[first_fork:], d.seq[first_fork:], d.poff[first_fork:], d.par)
    for i in range(0, N, 3):
        assert ix.highest_before(i) == o.hb(i), ("hb", i)
        assert ix.lowest_after(i) == o.la(i), ("la", i)
    ix.close()
