"""Write-back of Flush to the reference's kvdb tables and restart from them
(SURVEY 8f row 2), through the C ABI (lx_writeback_prepare / _fetch).

Checked against the oracle's flushable tables (oracle/vecfc_oracle.py restates
vecengine/vecfc with their v|S, v|s, v|b, v|B tables): at every Flush the keys
the oracle writes and their bytes equal the GPU write-back; BranchesInfo
equals oracle/rlp.py's encoding of the oracle's BranchesInfo (spec-pinned RLP,
see oracle/rlp.py).  Restart mirrors abft/restart_test.go:156-188 at the index
level: a fresh handle restored from a copy of the persisted tables continues
bit-exactly.  At full size (BASELINE configs[3]) the rows written back for
table "s" are exactly the rows whose LowestAfter bytes changed.
"""

import numpy as np
import pytest

from oracle import corc, pos, rlp, tdag
from oracle import vecfc_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def be32(x):
    return int(x).to_bytes(4, "big")


def oracle_puts(o):
    """The Puts the oracle's next Flush commits (vecengine/index.go:78-85)."""
    bi = o.bi
    return {"S": dict(o.tbl_hb.dirty), "s": dict(o.tbl_la.dirty),
            "b": {k: be32(v) for k, v in o.tbl_branch.dirty.items()},
            "B": rlp.encode_branches_info(bi.last_seq, bi.creator_idxs, bi.by_creators)}


def by_id(g, wb):
    return {t: {g.ids[k]: v for k, v in wb[t].items()} for t in ("S", "s", "b")}


SHAPES = [
    # nodes, events/node, parents, cheaters, forks, seed
    (6, 30, 3, 2, 6, 1), (10, 25, 4, 3, 5, 2), (16, 20, 5, 0, 0, 3), (24, 15, 6, 5, 4, 4), (70, 4, 8, 8, 2, 5),
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s[-1]) for s in SHAPES])
def test_writeback_equals_oracle_puts(lx, shape):
    n, epn, p, ch, fk, seed = shape
    nodes, evs = tdag.rand_fork_dag(n, epn, p, cheaters=ch, forks_count=fk, seed=seed)
    rng = np.random.default_rng(seed)
    validators = pos.Validators({v: int(x) for v, x in zip(nodes, rng.integers(1, 9, n))})
    store = {e.id: e for e in evs}
    o = vo.Index()
    o.reset(validators, store.get)
    g = lx.VecfcIndex()
    g.reset(validators)
    i = i_flushed = flushes = drops = 0
    while i < len(evs):
        part = evs[i:i + int(rng.integers(1, 12))]
        for e in part:
            o.add(e)
        g.add_events(part)
        act = rng.random()
        if act < 0.2:
            # rolls back to the last flush (vecengine/index.go:88-96): redo from there
            o.drop_not_flushed()
            g.drop_not_flushed()
            drops += 1
            i = i_flushed
            continue
        i += len(part)
        if act < 0.6 or i >= len(evs):
            i_flushed = i
            want = oracle_puts(o)
            wb = g.ix.writeback()
            got = by_id(g, wb)
            assert got["S"] == want["S"]
            assert got["s"] == want["s"]
            assert got["b"] == want["b"]
            assert wb["B"] == want["B"]
            o.flush()
            g.flush()
            flushes += 1
    assert flushes > 3 and drops > 0


def test_writeback_state_errors(lx):
    d = lx.tools.gen_dag(4, 10, 3, seed=3)
    ix = lx.Index()
    ix.reset([1, 1, 1, 1])
    ix.add_batch(d.creator[:8], d.seq[:8], d.poff[:9], d.par)
    wb = ix.writeback()
    assert sorted(wb["S"]) == list(range(8)) and set(wb["s"]) >= set(range(8))
    ix.flush()
    wb = ix.writeback()                      # nothing added since: only table B
    assert not wb["S"] and not wb["s"] and not wb["b"] and wb["B"]
    import ctypes
    ix.add_batch(d.creator[8:12], d.seq[8:12], d.poff[8:13], d.par)
    with pytest.raises(lx.LxError):          # fetch without a current prepare
        ix._chk(ix.L.lx_writeback_fetch(ix.h, None, None, None, None, None, None, None))
    wb2 = lx.capi.LxWriteback()
    ix._chk(ix.L.lx_writeback_prepare(ix.h, ctypes.byref(wb2)))
    ix.add_batch(d.creator[12:14], d.seq[12:14], d.poff[12:15], d.par)
    with pytest.raises(lx.LxError):          # invalidated by the Add
        ix._chk(ix.L.lx_writeback_fetch(ix.h, None, None, None, None, None, None, None))


def test_restart_from_persisted_tables(lx):
    """GENERATOR/RESTORED of abft/restart_test.go at the index level: flush
    after every event into a DB; at random points rebuild the index from a copy
    of the DB; the persisted tables equal the oracle's and the restored index
    answers like the oracle."""
    nodes, evs = tdag.rand_fork_dag(10, 30, 4, cheaters=3, forks_count=6, seed=7)
    validators = pos.Validators({v: 1 + (k % 3) for k, v in enumerate(nodes)})
    store = {e.id: e for e in evs}
    o = vo.Index()
    o.reset(validators, store.get)
    db = {}
    g = lx.VecfcIndex()
    g.reset(validators)
    rng = np.random.default_rng(3)
    restarts = 0
    for e in evs:
        o.add(e)
        o.flush()
        g.add(e)
        g.flush(db)
        if rng.random() < 0.08:
            copy = {t: dict(v) for t, v in db.items()}
            g.ix.close()
            g = lx.VecfcIndex()
            g.restore(validators, copy, store.get)
            db = copy
            restarts += 1
    assert restarts >= 3
    assert db["S"] == o.tbl_hb.flushed
    assert db["s"] == o.tbl_la.flushed
    assert db["b"] == {k: be32(v) for k, v in o.tbl_branch.flushed.items()}
    bi = o.tbl_binfo.flushed[b"c"]
    assert db["B"][b"c"] == rlp.encode_branches_info(bi.last_seq, bi.creator_idxs, bi.by_creators)
    for a in evs[::3]:
        assert g.get_highest_before(a.id).to_bytes() == o.get_highest_before(a.id).to_bytes()
        assert g.get_lowest_after(a.id).to_bytes() == o.get_lowest_after(a.id).to_bytes()
        for b in evs[::7]:
            assert g.forkless_cause(a.id, b.id) == o.forkless_cause(a.id, b.id)


def test_restore_detects_inconsistent_db(lx):
    nodes, evs = tdag.rand_fork_dag(5, 10, 3, seed=9)
    validators = pos.Validators.equal(nodes)
    store = {e.id: e for e in evs}
    db = {}
    g = lx.VecfcIndex()
    g.reset(validators)
    g.add_events(evs)
    g.flush(db)
    bad = {t: dict(v) for t, v in db.items()}
    k = evs[3].id
    bad["s"][k] = bad["s"][k][:-4] + bytes([bad["s"][k][-4] ^ 1]) + bad["s"][k][-3:]
    h = lx.VecfcIndex()
    with pytest.raises(RuntimeError, match="inconsistent DB"):
        h.restore(validators, bad, store.get)
    h2 = lx.VecfcIndex()
    h2.restore(validators, db, store.get)
    assert h2.get_lowest_after(k).to_bytes() == db["s"][k]


def test_writeback_full_size_config4(lx):
    """BASELINE configs[3] at full size (V=100, 10 double-signers, 100k events),
    flushing every 10k events: table-s rows written back = rows whose
    LowestAfter bytes changed since the previous flush (new rows included),
    with the bytes of a handle that never flushed; tables S/b/B equal that
    handle's; a sample of rows equals the C oracle."""
    d = lx.tools.gen_dag(100, 1000, 10, cheaters=10, forks=10, seed=2)
    w = [1] * 100
    N = len(d)
    A = lx.Index(event_capacity=N)
    B = lx.Index(event_capacity=N)
    A.reset(w)
    B.reset(w)
    prev = {}
    step = 10_000
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        for ix in (A, B):
            ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
        wa = A.writeback()
        wb = B.writeback()                   # never flushed: every row of the epoch
        assert sorted(wa["S"]) == list(range(lo, hi))
        assert all(wa["S"][k] == wb["S"][k] and wa["b"][k] == wb["b"][k] for k in wa["S"])
        changed = {k for k, v in wb["s"].items() if prev.get(k) != v}
        assert set(wa["s"]) == changed
        assert all(wa["s"][k] == wb["s"][k] for k in wa["s"])
        assert wa["B"] == wb["B"]
        prev = wb["s"]
        A.flush()
    assert A.num_branches() > 100
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    for i in range(0, N, 997):
        assert prev[i] == o.la(i) and wb["S"][i] == o.hb(i), i
