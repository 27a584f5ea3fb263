"""lx_forkless_cause: the per-pair ForklessCause of the unchanged caller
(vecfc/forkless_cause.go:28-38), answered from the index's result cache
(lachesis-base_amd/csrc/lx_fccache.cpp), bit-exact against the C oracle under
the access patterns of abft -- the newest event against a frame's roots
(abft/event_processing.go:149-161), a root against the previous frame's roots
(abft/election/election.go:101-123), old roots replayed after a decided frame
(abft/event_processing.go:102-146) -- with Build-style rollbacks
(abft/indexed_lachesis.go:53-63), evictions and slot reuse."""

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def _oracle(d, w, n):
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator[:n], d.seq[:n], d.poff[:n + 1], d.par) == -1
    return o


@pytest.mark.parametrize("slots", [0, 64, 256, 4096])
@pytest.mark.parametrize("cheaters", [0, 3])
def test_caller_pattern_matches_oracle(lx, slots, cheaters):
    """Events added one at a time; after each Add the newest event asks about
    a window of older "roots" in order, then an older event replays its
    questions (the election / processKnownRoots pattern).  Every answer equals
    the oracle's; a small working set forces evictions, slot reuse past the
    127 column generations, and tile fills."""
    V = 12
    d = lx.tools.gen_dag(V, 40, 4, cheaters=cheaters, forks=4, seed=5 + cheaters)
    w = list(range(30, 30 - V, -1))
    N = len(d)
    o = _oracle(d, w, N)
    ix = lx.Index(options={"fc_cache": slots})
    ix.reset(w)
    rng = np.random.default_rng(slots + cheaters)
    asked = 0
    for e in range(N):
        ix.add_batch(d.creator[e:e + 1], d.seq[e:e + 1], d.poff[e:e + 2], d.par)
        ix.flush()
        if e < 8:
            continue
        lo = max(0, e - 3 * V)
        for b in range(lo, e, 2):                      # newest event vs a frame's roots, in order
            assert ix.forkless_cause(e, b) == bool(o.forkless_cause(e, b)), (e, b)
            asked += 1
        if e % 7 == 0:                                 # an older root replays its questions
            a = int(rng.integers(max(0, e - 4 * V), e))
            for b in range(max(0, a - 2 * V), a, 3):
                assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b)), (a, b)
                asked += 1
    st = ix.fc_cache_stats()
    if slots:
        assert st["calls"] == asked and st["hits"] > asked // 2
        assert st["row_fills"] > 0 and st["tile_fills"] > 0
    ix.close()


def test_rollback_evicts_dropped_events(lx):
    """Add, ask, DropNotFlushed of several unflushed events, re-Add: the
    dropped events leave the working set, the re-added ones (same dense
    indices) are answered afresh."""
    V = 8
    d = lx.tools.gen_dag(V, 30, 3, cheaters=2, forks=3, seed=3)
    w = [3, 3, 2, 2, 2, 1, 1, 1]
    N = len(d)
    o = corc.OracleIndex(w)
    ix = lx.Index(options={"fc_cache": 128})
    ix.reset(w)
    for e in range(N):
        ix.add_batch(d.creator[e:e + 1], d.seq[e:e + 1], d.poff[e:e + 2], d.par)
        o.add(int(d.creator[e]), int(d.seq[e]), d.par[d.poff[e]:d.poff[e + 1]])
        for b in range(max(0, e - 12), e + 1):
            assert ix.forkless_cause(e, b) == bool(o.forkless_cause(e, b))
        if e % 4 == 3:
            ix.drop_not_flushed()                       # rolls back e - 2 .. e
            o.drop_not_flushed()
            # re-add the same events: the same dense indices, recomputed answers
            lo = int(o.num_events())
            for x in range(lo, e + 1):
                ix.add_batch(d.creator[x:x + 1], d.seq[x:x + 1], d.poff[x:x + 2], d.par)
                o.add(int(d.creator[x]), int(d.seq[x]), d.par[d.poff[x]:d.poff[x + 1]])
                for b in range(max(0, x - 12), x + 1):
                    assert ix.forkless_cause(x, b) == bool(o.forkless_cause(x, b))
        if e % 2 == 1:
            ix.flush()
            o.flush()
    ix.close()


def test_reused_index_after_drop_gets_fresh_answers(lx):
    """A dropped event's dense index taken by a different event (another
    validator's): answers for that index are recomputed, not served from the
    dropped event's row or column."""
    d = lx.tools.gen_dag(6, 30, 3, seed=4)
    w = [1] * 6
    N = len(d)
    ix = lx.Index(options={"fc_cache": 64})
    ix.reset(w)
    cut = N - 20
    ix.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par)
    ix.flush()
    o = _oracle(d, w, cut)
    # event `cut` of the DAG, asked about, then dropped
    x = cut
    ix.add_batch(d.creator[x:x + 1], d.seq[x:x + 1], d.poff[x:x + 2], d.par)
    first = [ix.forkless_cause(x, b) for b in range(cut - 30, cut + 1)] + \
            [ix.forkless_cause(a, x) for a in range(cut - 30, cut + 1)]
    ix.drop_not_flushed()
    # a different event lands on index `cut`: the next event of another creator
    y = next(i for i in range(cut + 1, N) if d.creator[i] != d.creator[x]
             and all(p < cut for p in d.par[d.poff[i]:d.poff[i + 1]]))
    par = d.par[d.poff[y]:d.poff[y + 1]]
    ix.add(int(d.creator[y]), int(d.seq[y]), par)
    o.add(int(d.creator[y]), int(d.seq[y]), par)
    for b in range(cut - 30, cut + 1):
        assert ix.forkless_cause(cut, b) == bool(o.forkless_cause(cut, b))
        assert ix.forkless_cause(b, cut) == bool(o.forkless_cause(b, cut))
    assert len(first) == 62
    ix.close()


def test_unknown_events_and_reset(lx):
    d = lx.tools.gen_dag(5, 10, 3, seed=2)
    ix = lx.Index()
    ix.reset([1] * 5)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    N = len(d)
    with pytest.raises(lx.LxError) as ei:
        ix.forkless_cause(N, 0)
    assert ei.value.code == -1
    assert ix.forkless_cause(N - 1, 0) in (True, False)
    ix.reset([1] * 5)                                    # a new epoch: nothing cached survives
    with pytest.raises(lx.LxError):
        ix.forkless_cause(0, 0)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    o = _oracle(d, [1] * 5, N)
    for a in range(N - 10, N):
        for b in range(N):
            assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b))
    ix.close()


def _grid_dag(V, rounds):
    """Round-robin DAG: e(v, s) has parents [e(v, s-1)] + e(u, s-1) of every
    other u.  Returns (events as (creator, seq, parents), index of e(v, s))."""
    evs, at = [], {}
    for s in range(1, rounds + 1):
        for v in range(V):
            par = [] if s == 1 else [at[v, s - 1]] + [at[u, s - 1] for u in range(V) if u != v]
            at[v, s] = len(evs)
            evs.append((v, s, par))
    return evs, at


def test_drop_then_other_creators_fork_same_branch_count(lx):
    """fork of creator 1 (branch V), a tile fill that builds
    the cheater columns for it, DropNotFlushed, then a fork of creator 3 gets
    the same branch number V.  The next tile fill must count branch V for
    creator 3, not creator 1.  Hand-built so the answer depends on it:
    g = e(0, R+1) observes only creator 3's fork branch (not its original
    e(3, R)) and e(2, R); FC(g, e(3, R-1)) holds with creators 0, 2 and 3
    (1 + 1 + 2 >= quorum 4) and fails if branch V is credited to creator 1."""
    V, R = 4, 4
    w = [1, 1, 1, 2]
    evs, at = _grid_dag(V, R)
    o = corc.OracleIndex(w)
    ix = lx.Index(options={"fc_cache": 512})
    ix.reset(w)

    def add(c, s, par):
        ix.add(c, s, par)
        o.add(c, s, par)
        return int(o.num_events()) - 1

    for c, s, par in evs:
        add(c, s, par)
    ix.flush()
    o.flush()
    n0 = len(evs)
    # rows of the base events filled before the fork exists
    for a in range(n0 - V, n0):
        for b in range(n0):
            assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b))
    # creator 1 forks at seq R: branch V
    f1 = add(1, R, [at[1, R - 1]])
    assert o.num_branches() == V + 1
    assert ix.forkless_cause(f1, at[0, 1]) == bool(o.forkless_cause(f1, at[0, 1]))   # row fill of f1
    old = n0 - V
    assert ix.forkless_cause(old, f1) == bool(o.forkless_cause(old, f1))             # older row: tile fill
    tiles0 = ix.fc_cache_stats()["tile_fills"]
    assert tiles0 >= 1
    ix.drop_not_flushed()
    o.drop_not_flushed()
    # creator 3 forks at seq R: the same branch number V, another creator
    f3 = add(3, R, [at[3, R - 1]])
    assert o.num_branches() == V + 1 and o.branch(f3) == V
    g = add(0, R + 1, [at[0, R], f3, at[2, R]])
    b = at[3, R - 1]
    assert bool(o.forkless_cause(g, b))                                              # the case the test is about
    assert ix.forkless_cause(g, b)                                                   # row fill of g (new a)
    assert ix.forkless_cause(old, g) == bool(o.forkless_cause(old, g))               # older row again: tile fill
    assert ix.fc_cache_stats()["tile_fills"] > tiles0
    N = int(o.num_events())
    for a in range(N):                                                               # all answers from the tile
        for b2 in range(N):
            assert ix.forkless_cause(a, b2) == bool(o.forkless_cause(a, b2)), (a, b2)
    ix.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_drop_readd_different_fork_suffix(lx, seed):
    """after each DropNotFlushed a DIFFERENT suffix is added,
    whose forks belong to other creators, with older-row questions
    interleaved so the cache refills by tiles; every answer equals the oracle."""
    V = 8
    w = [5, 4, 3, 3, 2, 2, 1, 1]
    base = lx.tools.gen_dag(V, 12, 3, seed=40 + seed)
    nb = len(base)
    o = corc.OracleIndex(w)
    ix = lx.Index(options={"fc_cache": 256})
    ix.reset(w)
    ix.add_batch(base.creator, base.seq, base.poff, base.par)
    o.add_batch(base.creator, base.seq, base.poff, base.par)
    ix.flush()
    o.flush()
    rng = np.random.default_rng(seed)
    last = {}                                 # creator -> last event of the base
    for e in range(nb):
        last[int(base.creator[e])] = e
    seqs = {v: int(base.seq[last[v]]) for v in range(V)}
    for trial in range(4):
        forkers = rng.choice(V, size=2, replace=False)
        n_before = int(o.num_events())
        tip = dict(last)
        tipseq = dict(seqs)
        added = []
        for step in range(3 * V):
            v = int(rng.integers(V))
            par = [tip[v]] + [tip[u] for u in rng.choice(V, size=3, replace=False) if u != v]
            s = tipseq[v] + 1
            if v in forkers and step < V and rng.random() < 0.7:
                # fork: another event on the same self-parent
                par = [last[v]] + par[1:]
                s = seqs[v] + 1
            ix.add(v, s, par)
            o.add(v, s, par)
            x = int(o.num_events()) - 1
            added.append(x)
            tip[v], tipseq[v] = x, s
            for b in range(max(0, x - 10), x + 1):
                assert ix.forkless_cause(x, b) == bool(o.forkless_cause(x, b)), (trial, x, b)
            if step % 4 == 3:                   # older rows against the new events: tile fills
                a = int(rng.integers(max(0, n_before - 20), x))
                for b in added[-4:]:
                    assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b)), (trial, a, b)
        N = int(o.num_events())
        for a in range(max(0, N - 40), N):
            for b in range(max(0, N - 60), N):
                assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b)), (trial, a, b)
        ix.drop_not_flushed()
        o.drop_not_flushed()
        assert int(o.num_events()) == n_before
    assert ix.fc_cache_stats()["tile_fills"] > 0
    ix.close()


@pytest.mark.parametrize("fork", [False, True])
def test_back_to_back_row_fills_different_asking_events(lx, fork):
    """Misses of different asking events right after one another, nothing
    pending (the k_fc row-fill path, not the fused Add + row launch): the host
    returns as soon as its own answer lands while the rest of the row is still
    being written, and moves on to the next asking event.  Every row must hold
    its own asking event's answers -- then read back as hits and compared with
    the oracle (vecfc/forkless_cause.go:28-38: a cached answer is the answer)."""
    V = 100
    d = lx.tools.gen_dag(V, 100, 10, cheaters=4 if fork else 0, forks=3 if fork else 0, seed=17)
    w = [(1 << 12) // (i + 1) + 1 for i in range(V)]
    N = len(d)
    o = _oracle(d, w, N)
    ix = lx.Index(options={"fc_cache": 4096})
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.flush()
    ix.sync()
    rng = np.random.default_rng(5)
    # a working set of ~3000 b's (each first question brings its next 64 events)
    bs = list(range(N - 3000, N, 64))
    for b in bs:
        assert ix.forkless_cause(N - 1, b) == bool(o.forkless_cause(N - 1, b))
    # back-to-back misses, each a new asking event (not in the working set: a
    # row fill of its own, no tile fill) with one question
    asks = [int(x) for x in rng.choice(np.arange(N // 4, N - 3100), 300, replace=False)]
    for a in asks:
        b = int(rng.integers(N - 3000, N))
        assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b)), (a, b)
    # the rows those fills wrote: every answer, hits or refills
    for a in asks[::5]:
        for b in range(N - 3000, N, 37):
            assert ix.forkless_cause(a, b) == bool(o.forkless_cause(a, b)), (a, b)
    st = ix.fc_cache_stats()
    assert st["row_fills"] >= len(asks) and st["hits"] > 0, st
    ix.close()
