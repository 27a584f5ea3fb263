"""The small-batch (latency) path of Add and the per-call query paths.

abft calls Add once per event (abft/indexed_lachesis.go:53-82) and
ForklessCause once per (event, root) pair (abft/event_processing.go:149-161);
the level batcher hands over one antichain at a time.  lx_add_batch routes
host-pointer batches of up to 2048 events (that fit one workgroup's LDS)
through host branch assignment + one k_small launch per pending run
(lx_small.hip); these tests check that path bit-exactly
against the C oracle and against the device-assigned walker path (k_index),
including mixed sequences of both, rollbacks, errors and deep batches.
"""

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def oracle_for(d, w, hi=None):
    hi = len(d) if hi is None else hi
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator[:hi], d.seq[:hi], d.poff[:hi + 1], d.par) == -1
    return o


def rows_equal(ix, o, events, merged=True):
    for i in events:
        i = int(i)
        assert ix.highest_before(i) == o.hb(i), ("hb", i)
        assert ix.lowest_after(i) == o.la(i), ("la", i)
        assert ix.branch(i) == o.branch(i), ("branch", i)
        if merged:
            assert ix.merged_highest_before(i) == o.merged_hb(i), ("merged", i)


def levels_of(d, lo=0, hi=None):
    """Topological level of every event (1 + highest parent level)."""
    hi = len(d) if hi is None else hi
    lvl = np.zeros(hi, dtype=np.int64)
    for i in range(lo, hi):
        ps = d.par[d.poff[i]:d.poff[i + 1]]
        lvl[i] = 1 + (int(lvl[ps].max()) if len(ps) else -1)
    return lvl


def add_dev(ix, d, lo, hi, dev):
    """Events [lo, hi) through lx_add_batch_dev (always the device-assigned path)."""
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)
    off = (d.poff[lo:hi + 1] - d.poff[lo]).astype(np.uint32)
    c, s, o, p = t(d.creator[lo:hi]), t(d.seq[lo:hi]), t(off), t(d.par[d.poff[lo]:d.poff[hi]] if hi > lo else [0])
    ix.add_batch_dev(hi - lo, c.data_ptr(), s.data_ptr(), o.data_ptr(), p.data_ptr())
    ix.sync()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_chunks_vs_oracle_and_walker(lx, seed, monkeypatch):
    """Fork-heavy DAG in random chunk sizes (1..400) through the small path:
    rows, branch IDs, merged HB and FC equal the oracle and the walker path."""
    d = lx.tools.gen_dag(24, 60, 6, cheaters=5, forks=8, seed=40 + seed)
    w = list(range(48, 24, -1))
    N = len(d)
    o = oracle_for(d, w)
    rng = np.random.default_rng(seed)
    ix = lx.Index()
    ix.reset(w)
    lo, br = 0, []
    while lo < N:
        hi = min(N, lo + int(rng.integers(1, 400)))
        br.extend(int(x) for x in ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par,
                                               want_branches=True))
        lo = hi
    assert br == [o.branch(i) for i in range(N)]
    rows_equal(ix, o, range(N))
    wk = lx.Index(options={"small_max": 0})
    wk.reset(w)
    wk.add_batch(d.creator, d.seq, d.poff, d.par)
    qa, qb = lx.tools.fc_queries(d.lamport, 100_000, window=32, seed=seed)
    want = o.forkless_cause_batch(qa, qb)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), want)
    np.testing.assert_array_equal(wk.forkless_cause_batch(qa, qb), want)
    for i in range(0, N, 7):
        assert ix.highest_before(i) == wk.highest_before(i)
        assert ix.lowest_after(i) == wk.lowest_after(i)
    ix.close()
    wk.close()


def test_mixed_small_and_device_batches(lx):
    """Small host batches and device-assigned batches interleaved on one handle,
    with flushes and rollbacks in between (the host mirror is refreshed after
    device-assigned batches, the LowestAfter tail state stays consistent)."""
    import torch
    dev = torch.device("cuda", 0)
    d = lx.tools.gen_dag(16, 80, 5, cheaters=4, forks=6, seed=77)
    w = [5, 5, 4, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 1, 1, 1]
    N = len(d)
    ix = lx.Index()
    ix.reset(w)
    cuts = [0, 50, 300, 301, 480, 700, 701, 900, 1100, N]
    for k, (lo, hi) in enumerate(zip(cuts, cuts[1:])):
        if k % 2:
            add_dev(ix, d, lo, hi, dev)
        else:
            ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
        if k == 3:
            ix.flush()
        if k in (4, 6):
            # roll back to the flush at k == 3 and re-add the dropped part the other way
            ix.drop_not_flushed()
            assert ix.num_events() == cuts[4]
            for lo2, hi2 in zip(cuts[4:k + 1], cuts[5:k + 2]):
                if k == 4:
                    ix.add_batch(d.creator[lo2:hi2], d.seq[lo2:hi2], d.poff[lo2:hi2 + 1], d.par)
                else:
                    add_dev(ix, d, lo2, hi2, dev)
        o = oracle_for(d, w, hi)
        rows_equal(ix, o, range(0, hi, 3), merged=False)
    o = oracle_for(d, w)
    rows_equal(ix, o, range(N))
    a = np.repeat(np.arange(N, dtype=np.uint32), 64)
    b = np.random.default_rng(1).integers(0, N, len(a)).astype(np.uint32)
    np.testing.assert_array_equal(ix.forkless_cause_batch(a, b), o.forkless_cause_batch(a, b))
    ix.close()


def test_deep_chain_one_batch(lx):
    """2000 levels in one small batch: a single validator's chain plus a second
    validator that references it (every event its own level)."""
    d = lx.tools.gen_dag(2, 1000, 2, seed=5)
    w = [2, 1]
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    assert levels_of(d).max() > 1000
    rows_equal(ix, o, range(len(d)))
    ix.close()


@pytest.mark.parametrize("chunk", [1, 37, 400, 2048])
def test_many_parents_lds_budget(lx, chunk):
    """Events with 40 parents: pending runs launch early when the next batch
    would not fit one k_small workgroup's LDS, and a 2048-event batch (80k
    parents) takes the device-assigned path; results equal the oracle either way."""
    d = lx.tools.gen_dag(64, 40, 40, cheaters=3, forks=4, seed=23)
    w = [1 + (i % 7) for i in range(64)]
    N = len(d)
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    for lo in range(0, N, chunk):
        hi = min(N, lo + chunk)
        ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
    rows_equal(ix, o, range(0, N, 5))
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=16, seed=3)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


def test_level_fed_config3_prefix(lx):
    """BASELINE configs[2] shape (V=1000, Zipf stakes, P=10) fed antichain by
    antichain, the way the level batcher hands it over: 12k events vs the oracle."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 12, 10, seed=9)
    N = len(d)
    o = oracle_for(d, w)
    lvl = levels_of(d)
    ix = lx.Index()
    ix.reset(w)
    # events of one level are contiguous in Add order only if the generator makes
    # them so; feed each maximal run of equal level as a batch (an antichain)
    starts = [0] + [i for i in range(1, N) if lvl[i] != lvl[i - 1]] + [N]
    for lo, hi in zip(starts, starts[1:]):
        ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
    rng = np.random.default_rng(2)
    rows_equal(ix, o, rng.choice(N, 150, replace=False), merged=False)
    qa, qb = lx.tools.fc_queries(d.lamport, 100_000, seed=6)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


@pytest.mark.parametrize("case", ["creator", "seq0", "selfparent", "order", "offsets"])
def test_small_path_errors(lx, case):
    """Errors of the small path: code, offending batch position, state unchanged
    (the checks of k_validate_claim; vecengine/index.go:159-161, eventcheck).
    The events before the offending one were assigned (new fork branches
    among them) and are rolled back: the re-added batch must index as if the
    failed one never happened."""
    d = lx.tools.gen_dag(4, 10, 3, cheaters=1, forks=2, seed=3)
    w = [1, 1, 1, 1]
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator[:20], d.seq[:20], d.poff[:21], d.par)
    cr, sq, par, poff = d.creator.copy(), d.seq.copy(), d.par.copy(), d.poff.copy()
    bad = 24
    if case == "creator":
        cr[bad] = 9
        code = -1
    elif case == "seq0":
        sq[bad] = 0
        code = -3
    elif case == "selfparent":
        sq[bad] += 1
        code = -3
    elif case == "order":
        par[d.poff[bad]] = bad + 3
        code = -2
    else:
        poff[bad + 1] = poff[bad] - 1
        code = -1
    with pytest.raises(lx.LxError) as ei:
        ix.add_batch(cr[20:], sq[20:], poff[20:], par)
    assert ei.value.code == code and ei.value.index == bad - 20
    assert ix.num_events() == 20
    ix.add_batch(d.creator[20:], d.seq[20:], d.poff[20:], d.par)
    rows_equal(ix, oracle_for(d, w), range(len(d)))
    ix.close()


def test_per_call_forkless_cause(lx):
    """The pinned per-call FC path (n <= 65536): n = 1, n = 667 (2/3 V, the
    calcFrameIdx pattern) and unknown events (crit -> LX_ERR_ARG) that leave no
    stale error behind."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 6, 10, seed=4)
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    N = len(d)
    rng = np.random.default_rng(0)
    for n in (1, 2, 667, 4096, 70_000):
        a = rng.integers(N // 2, N, n).astype(np.uint32)
        b = rng.integers(0, N, n).astype(np.uint32)
        np.testing.assert_array_equal(ix.forkless_cause_batch(a, b), o.forkless_cause_batch(a, b))
    assert ix.forkless_cause(N - 1, 0) == bool(o.forkless_cause_batch(np.array([N - 1], np.uint32),
                                                                      np.array([0], np.uint32))[0])
    with pytest.raises(lx.LxError):
        ix.forkless_cause(N + 5, 0)
    ix.sync()   # the failed pinned call leaves nothing for lx_sync to report
    a = np.array([N - 1, 3], dtype=np.uint32)
    np.testing.assert_array_equal(ix.forkless_cause_batch(a, a[::-1].copy()), o.forkless_cause_batch(a, a[::-1].copy()))
    ix.close()


@pytest.mark.parametrize("shape", [(12, 40, 5, 4, 8, 21), (100, 12, 10, 10, 10, 11), (30, 30, 6, 0, 0, 5)])
def test_batched_getters(lx, shape):
    """lx_get_{highest_before,lowest_after,merged_highest_before}_batch
    (device-encoded rows, vecfc/store_vectors.go:26-51, vecengine/index.go:235-250)
    equal the oracle's byte rows for every event, in shuffled order with repeats;
    a short buffer and an unknown event are errors."""
    import ctypes
    n, ev, p, ch, fk, seed = shape
    d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
    w = sorted((int(x) for x in np.random.default_rng(seed).integers(1, 9, n)), reverse=True)
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    N = len(d)
    evs = np.random.default_rng(seed).permutation(np.concatenate([np.arange(N), np.arange(0, N, 5)])).astype(np.uint32)
    for got, want in ((ix.highest_before_batch(evs), o.hb), (ix.lowest_after_batch(evs), o.la),
                      (ix.merged_highest_before_batch(evs), o.merged_hb)):
        for e, g in zip(evs, got):
            assert g == want(int(e)), int(e)
    from lachesis_hip.capi import u32p, u64p, u8p
    e2 = np.array([0, N - 1], dtype=np.uint32)
    off = np.zeros(3, dtype=np.uint64)
    buf = np.zeros(8, dtype=np.uint8)
    rc = ix.L.lx_get_highest_before_batch(ix.h, 2, e2.ctypes.data_as(u32p), off.ctypes.data_as(u64p),
                                          buf.ctypes.data_as(u8p), len(buf))
    assert rc == -1 and off[2] == len(o.hb(0)) + len(o.hb(N - 1))
    with pytest.raises(lx.LxError):
        ix.merged_highest_before_batch([0, N])
    ix.close()


def test_vecfc_api_surface(lx):
    """vecfc.NewIndex(crit, LiteConfig()), NewIndexWithEngine over the same
    engine, GetEngineCallbacks, BranchesInfo and DfsSubgraph through the
    facade (vecfc/index.go:52-130, vecengine/branches_info.go:15-53,
    vecengine/traversal.go:10-37) agree with the Python reference restatement."""
    from oracle import pos, tdag
    from oracle import vecfc_oracle as vo
    nodes, evs = tdag.rand_fork_dag(8, 15, 4, cheaters=2, forks_count=4, seed=6)
    validators = pos.Validators.equal(nodes)
    store = {e.id: e for e in evs}
    crits = []
    g = lx.new_index(crits.append, lx.lite_config())
    g.reset(validators, store.get)
    o = vo.Index()
    o.reset(validators, store.get)
    for e in evs:
        g.add(e)
        o.add(e)
    g2 = lx.new_index_with_engine(crits.append, lx.lite_config(), g)
    cb = g2.get_engine_callbacks()
    for e in evs[::5]:
        assert cb["GetHighestBefore"](e.id).to_bytes() == o.get_highest_before(e.id).to_bytes()
        assert cb["GetLowestAfter"](e.id).to_bytes() == o.get_lowest_after(e.id).to_bytes()
    assert cb["NewHighestBefore"](5).to_bytes() == bytes(40) and cb["NewLowestAfter"](5).to_bytes() == bytes(20)
    cb["SetHighestBefore"](evs[0].id, None)
    assert len(crits) == 1
    last, creators, by = g2.branches_info()
    bi = o.branches_info()
    assert (last, creators, by) == (list(bi.last_seq), list(bi.creator_idxs), [list(x) for x in bi.by_creators])
    g2.init_branches_info()
    head = evs[-1]
    seen_g, seen_o = [], []
    g2.dfs_subgraph(head, lambda x: (seen_g.append(x), True)[1] if seen_g.count(x) == 0 else False)
    o.dfs_subgraph(head, lambda x: (seen_o.append(x), True)[1] if seen_o.count(x) == 0 else False)
    assert seen_g == seen_o and len(seen_g) > 10


def test_vecfc_engine_shared_state(lx):
    """Two vecfc.Index facades over one engine (NewIndexWithEngine) share the
    epoch state: a flush, a drop and a reset through one are what the other
    sees -- its Adds resolve parents and its queries resolve events through the
    same map (the reference shares its Engine, vecfc/index.go:80-89)."""
    from oracle import pos, tdag
    from oracle import vecfc_oracle as vo
    nodes, evs = tdag.rand_fork_dag(6, 12, 3, cheaters=1, forks_count=3, seed=8)
    validators = pos.Validators.equal(nodes)
    store = {e.id: e for e in evs}
    g = lx.new_index(None, lx.lite_config())
    g.reset(validators, store.get)
    g2 = lx.new_index_with_engine(None, lx.lite_config(), g)
    o = vo.Index()
    o.reset(validators, store.get)
    half = len(evs) // 2
    for e in evs[:half]:
        g.add(e)
        o.add(e)
    g.flush()
    o.flush()
    for e in evs[half:half + 5]:          # unflushed, dropped through the other facade
        g2.add(e)
    g2.drop_not_flushed()
    assert g.get_highest_before(evs[half].id) is None
    for e in evs[half:]:                  # re-added through the first, queried through the second
        g.add(e)
        o.add(e)
    for a in evs[::3]:
        assert g2.get_highest_before(a.id).to_bytes() == o.get_highest_before(a.id).to_bytes()
        for b in evs[::4]:
            assert g2.forkless_cause(a.id, b.id) == o.forkless_cause(a.id, b.id)
    g2.reset(validators, store.get)       # a reset through the second empties the first
    assert g.get_highest_before(evs[0].id) is None
    for e in evs[:4]:
        g.add(e)
    assert g2.get_lowest_after(evs[0].id) is not None


def test_pending_run_flush_drop_readd(lx):
    """Small batches coalesce into a pending run that reaches the device only
    when it grows to 2048 events or something reads the index: flushes in
    between, DropNotFlushed of events still pending (host-only rollback,
    including fork branches they opened), of events partly launched (a query
    launched the run), and re-adds at the same dense indices -- rows, branch
    IDs and FC equal the oracle's at every step."""
    d = lx.tools.gen_dag(12, 80, 4, cheaters=3, forks=6, seed=17)
    w = [3, 3, 3, 2, 2, 2, 2, 1, 1, 1, 1, 1]
    N = len(d)
    o = corc.OracleIndex(w)
    ix = lx.Index()
    ix.reset(w)
    rng = np.random.default_rng(3)
    e = 0
    while e < N:
        k = min(N - e, int(rng.integers(1, 40)))
        br = ix.add_batch(d.creator[e:e + k], d.seq[e:e + k], d.poff[e:e + k + 1], d.par, want_branches=True)
        for i in range(e, e + k):
            assert o.add(int(d.creator[i]), int(d.seq[i]), d.par[d.poff[i]:d.poff[i + 1]]) == 0
        assert [int(x) for x in br] == [o.branch(i) for i in range(e, e + k)]
        r = rng.random()
        if r < 0.25:                                  # drop what is not flushed (pending or launched)
            if rng.random() < 0.5:
                ix.highest_before(e)                  # a read launches the pending run first
            ix.drop_not_flushed()
            o.drop_not_flushed()
            e = int(o.num_events())
            assert ix.num_events() == e and ix.num_branches() == o.num_branches()
            continue
        if r < 0.7:
            ix.flush()
            o.flush()
        e += k
        if rng.random() < 0.2:
            j = int(rng.integers(0, e))
            assert ix.highest_before(j) == o.hb(j) and ix.lowest_after(j) == o.la(j)
    ix.flush()
    rows_equal(ix, o, range(N))
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=24, seed=5)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


@pytest.mark.parametrize("V,epv,P,batch", [(5, 1000, 5, 1), (5, 600, 3, 7), (16, 300, 6, 1), (3, 900, 2, 33)])
def test_deep_runs_by_frontier_doubling(lx, V, epv, P, batch):
    """BASELINE configs[0]'s regime, Add by Add (vecengine/index.go:71-75): a
    few validators, every event its own DAG level, so each 2048-event pending
    run is ~2048 levels deep and is indexed by k_small_dbl (frontier doubling
    in one workgroup) instead of level by level.  Every row, branch and merged
    row equals the oracle's, and FC of all recent pairs; the same stream with
    option dbl=0 (k_small, level by level) gives identical answers."""
    d = lx.tools.gen_dag(V, epv, P, seed=V + epv)
    N = len(d)
    w = [1 + (i * 3) % 7 for i in range(V)]
    o = oracle_for(d, w)
    outs = []
    for dbl in (1, 0):
        ix = lx.Index(options={"dbl": dbl})
        ix.reset(w)
        for lo in range(0, N, batch):
            hi = min(N, lo + batch)
            ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1] - d.poff[lo], d.par[d.poff[lo]:])
            ix.flush()
        ev = np.arange(0, N, 1 if N <= 3000 else 3)
        if dbl:
            rows_equal(ix, o, ev)
        qa = np.repeat(np.arange(N - 300, N, dtype=np.uint32), 300)
        qb = np.tile(np.arange(N - 600, N - 300, dtype=np.uint32), 300)
        got = ix.forkless_cause_batch(qa, qb)
        np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))
        outs.append((got, ix.rows_np(0, np.arange(N, dtype=np.uint32))[1], ix.rows_np(1, np.arange(N, dtype=np.uint32))[1]))
        ix.close()
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)
