"""Restart from the persisted tables without replay (lx_load_rows /
lx_load_finish).

abft/restart_test.go:156-188 builds a fresh index over a copy of the epoch DB
and continues.  Here the DB is the one the reference's own index would have
written: the Python oracle (oracle/vecfc_oracle.py restates vecengine/vecfc
with their flushable tables v|S, v|s, v|b, v|B) is run, its flushed tables are
handed to a fresh GPU index, and both continue adding events -- rows, branch
IDs, merged HB and ForklessCause must stay identical.  Tables that cannot come
from one epoch must be refused ("inconsistent DB", the reference's crit).
"""

import numpy as np
import pytest

from oracle import pos, rlp, tdag
from oracle import vecfc_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def be32(x):
    return int(x).to_bytes(4, "big")


def oracle_db(o):
    """The flushed tables of the oracle's epoch DB (what a restart reads)."""
    bi = o.tbl_binfo.flushed.get(b"c")
    db = {"S": dict(o.tbl_hb.flushed), "s": dict(o.tbl_la.flushed),
          "b": {k: be32(v) for k, v in o.tbl_branch.flushed.items()}, "B": {}}
    if bi is not None:
        db["B"][b"c"] = rlp.encode_branches_info(bi.last_seq, bi.creator_idxs, bi.by_creators)
    return db


def same(g, o, evs, fc_pairs=True):
    for e in evs:
        assert g.get_highest_before(e.id).to_bytes() == o.get_highest_before(e.id).to_bytes(), e
        assert g.get_lowest_after(e.id).to_bytes() == o.get_lowest_after(e.id).to_bytes(), e
        assert g.get_merged_highest_before(e.id).to_bytes() == o.get_merged_highest_before(e.id).to_bytes(), e
        assert g.get_event_branch_id(e.id) == o.get_event_branch_id(e.id), e
    if fc_pairs:
        for a in evs[::2]:
            for b in evs[::3]:
                assert g.forkless_cause(a.id, b.id) == o.forkless_cause(a.id, b.id), (a, b)


SHAPES = [
    # nodes, events/node, parents, cheaters, forks, seed
    (6, 30, 3, 2, 6, 1), (10, 25, 4, 3, 5, 2), (16, 20, 5, 0, 0, 3), (24, 15, 6, 5, 4, 4),
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s[-1]) for s in SHAPES])
@pytest.mark.parametrize("dropped", [False, True])
def test_load_oracle_tables_mid_epoch(lx, shape, dropped):
    """Load the oracle's flushed tables mid-epoch (optionally after unflushed
    events were dropped, vecengine/index.go:88-96), continue adding on both
    sides with flushes and drops; everything stays identical."""
    n, epn, p, ch, fk, seed = shape
    nodes, evs = tdag.rand_fork_dag(n, epn, p, cheaters=ch, forks_count=fk, seed=seed)
    rng = np.random.default_rng(seed)
    validators = pos.Validators({v: int(x) for v, x in zip(nodes, rng.integers(1, 9, n))})
    store = {e.id: e for e in evs}
    o = vo.Index()
    o.reset(validators, store.get)
    cut = len(evs) // 2
    for k, e in enumerate(evs[:cut]):
        o.add(e)
        if k % 7 == 0 or k == cut - 1:
            o.flush()
    if dropped:
        for e in evs[cut:cut + 9]:
            o.add(e)
        o.drop_not_flushed()
    g = lx.VecfcIndex()
    g.restore(validators, oracle_db(o), store.get)
    assert g.ix.num_events() == cut
    same(g, o, evs[:cut])
    i = cut
    while i < len(evs):
        part = evs[i:i + int(rng.integers(1, 10))]
        for e in part:
            o.add(e)
        g.add_events(part)
        if rng.random() < 0.2:
            o.drop_not_flushed()
            g.drop_not_flushed()
            continue
        o.flush()
        g.flush()
        i += len(part)
    same(g, o, evs)


def test_restart_loop_from_gpu_writeback(lx):
    """GENERATOR / RESTORED at the index level (restart_test.go:69-238): the GPU
    index writes its tables back at every flush; at random points a fresh
    handle is built from a copy of them and continues."""
    nodes, evs = tdag.rand_fork_dag(12, 30, 5, cheaters=4, forks_count=8, seed=11)
    validators = pos.Validators({v: 1 + (k % 4) for k, v in enumerate(nodes)})
    store = {e.id: e for e in evs}
    o = vo.Index()
    o.reset(validators, store.get)
    db = {}
    g = lx.VecfcIndex()
    g.reset(validators)
    rng = np.random.default_rng(5)
    restarts = 0
    for e in evs:
        o.add(e)
        o.flush()
        g.add(e)
        g.flush(db)
        if rng.random() < 0.1:
            copy = {t: dict(v) for t, v in db.items()}
            g.ix.close()
            g = lx.VecfcIndex()
            g.restore(validators, copy, store.get)
            db = copy
            restarts += 1
    assert restarts >= 3
    assert db["S"] == o.tbl_hb.flushed and db["s"] == o.tbl_la.flushed
    same(g, o, evs[::2])


def _base_db(lx, seed=9, cheaters=3):
    nodes, evs = tdag.rand_fork_dag(8, 20, 4, cheaters=cheaters, forks_count=6, seed=seed)
    validators = pos.Validators.equal(nodes)
    store = {e.id: e for e in evs}
    o = vo.Index()
    o.reset(validators, store.get)
    for e in evs:
        o.add(e)
    o.flush()
    return evs, validators, store, o, oracle_db(o)


def _flip(b, k, x=1):
    return b[:k] + bytes([b[k] ^ x]) + b[k + 1:]


CORRUPTIONS = ["la_entry", "hb_seq", "hb_minseq", "branch_id", "hb_length", "bi_last_seq", "bi_creator", "marker",
               "missing_parent", "marker_honest", "marker_nofork"]
MARKER = bytes(4) + (0x7FFFFFFF).to_bytes(4, "little")


@pytest.mark.parametrize("kind", CORRUPTIONS)
def test_load_refuses_inconsistent_tables(lx, kind):
    """Each kind of table damage is refused with crit("inconsistent DB"); the
    undamaged tables load (and a handle refused once loads fine after reset)."""
    evs, validators, store, o, db = _base_db(lx, cheaters=0 if kind == "marker_nofork" else 3)
    bad = {t: dict(v) for t, v in db.items()}
    e = evs[len(evs) // 2]
    if kind == "la_entry":
        bad["s"][e.id] = _flip(bad["s"][e.id], 0)
    elif kind == "hb_seq":
        # an entry e raised above its self-parent's: (j, v) is first observed from
        # e's branch by e, so lowering it contradicts LowestAfter((j, v))
        e = next(x for x in evs[len(evs) // 2:] if x.seq > 1)
        row, prow = bytearray(bad["S"][e.id]), db["S"][e.parents[0]]
        seq_at = lambda r, k: int.from_bytes(r[8 * k:8 * k + 4], "little") if 8 * k < len(r) else 0
        j = next(k for k in range(len(row) // 8) if k != o.get_event_branch_id(e.id)
                 and seq_at(row, k) > max(1, seq_at(prow, k)))
        row[8 * j:8 * j + 4] = (seq_at(row, j) - 1).to_bytes(4, "little")
        bad["S"][e.id] = bytes(row)
    elif kind == "hb_minseq":
        row = bytearray(bad["S"][e.id])
        j = next(k for k in range(len(row) // 8) if row[8 * k] and row[8 * k + 4] != 0xFF)
        row[8 * j + 4] ^= 2
        bad["S"][e.id] = bytes(row)
    elif kind == "branch_id":
        bad["b"][e.id] = be32((int.from_bytes(bad["b"][e.id], "big") + 1) % len(validators.weights))
    elif kind == "hb_length":
        bad["S"][e.id] = bad["S"][e.id] + bytes(8)
    elif kind in ("bi_last_seq", "bi_creator"):
        bi = o.tbl_binfo.flushed[b"c"]
        last, cr = list(bi.last_seq), list(bi.creator_idxs)
        if kind == "bi_last_seq":
            last[0] += 1
        else:
            cr[-1] = (cr[-1] + 1) % len(validators.weights)
        bad["B"][b"c"] = rlp.encode_branches_info(last, cr, bi.by_creators)
    elif kind == "marker":
        # a fork marker {0, MaxInt32} the vectors do not imply -> replaced by a plain entry
        k, j = next((x, j) for x in evs for j in range(len(db["S"][x.id]) // 8)
                    if db["S"][x.id][8 * j:8 * j + 8] == bytes(4) + (0x7FFFFFFF).to_bytes(4, "little"))
        row = bytearray(bad["S"][k.id])
        row[8 * j:8 * j + 8] = bytes(8)
        bad["S"][k.id] = bytes(row)
    elif kind in ("marker_honest", "marker_nofork"):
        # a fork marker in the column of a creator with one branch (in a fork-free
        # epoch: anywhere) -- the reference marks cheaters' branches only
        # (vecengine/index.go:173-209); loading it would feed 0x80000000 to the walker
        by = o.tbl_binfo.flushed[b"c"].by_creators
        honest = [bs[0] for bs in by if len(bs) == 1]
        row = bytearray(bad["S"][e.id])
        j = next(k for k in honest if k != o.get_event_branch_id(e.id) and 8 * k < len(row) and row[8 * k])
        row[8 * j:8 * j + 8] = MARKER
        bad["S"][e.id] = bytes(row)
    else:
        del bad["b"][evs[3].id]
    h = lx.VecfcIndex()
    with pytest.raises(RuntimeError, match="inconsistent DB"):
        h.restore(validators, bad, store.get)
    h.restore(validators, db, store.get)
    same(h, o, evs[::3], fc_pairs=False)


def test_load_full_size_config4(lx):
    """BASELINE configs[3] at full size (V=100, 10 double-signers x 10 forks,
    100k events): write back every 25k events, restore a fresh handle from the
    tables (raw seqs behind ~every cheater column rebuilt, markers re-derived
    and checked, every LowestAfter entry verified), then both handles continue
    with the same events -- all rows and 200k ForklessCause answers equal."""
    d = lx.tools.gen_dag(100, 1000, 10, cheaters=10, forks=10, seed=2)
    w = [1] * 100
    N = len(d)
    cut = 60_000
    A = lx.Index(event_capacity=N)
    A.reset(w)
    tabs = {"S": {}, "s": {}, "b": {}}
    for lo in range(0, cut, 25_000):
        hi = min(cut, lo + 25_000)
        A.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
        wb = A.writeback()
        for t in ("S", "s", "b"):
            tabs[t].update(wb[t])
        bi = wb["B"]
        A.flush()
    R = lx.Index(event_capacity=N)
    R.reset(w)
    off = d.poff[:cut + 1]
    R.load_rows(d.creator[:cut], d.seq[:cut], off, d.par, b"".join(tabs["b"][k] for k in range(cut)),
                [tabs["S"][k] for k in range(cut)], [tabs["s"][k] for k in range(cut)])
    R.load_finish(bi)
    assert R.num_branches() == A.num_branches() > 100
    for ix in (A, R):
        ix.add_batch(d.creator[cut:], d.seq[cut:], d.poff[cut:], d.par)
    ev = np.arange(0, N, 7, dtype=np.uint32)
    assert R.highest_before_batch(ev) == A.highest_before_batch(ev)
    assert R.lowest_after_batch(ev) == A.lowest_after_batch(ev)
    assert R.merged_highest_before_batch(ev) == A.merged_highest_before_batch(ev)
    qa, qb = lx.tools.fc_queries(d.lamport, 200_000, seed=8)
    np.testing.assert_array_equal(R.forkless_cause_batch(qa, qb), A.forkless_cause_batch(qa, qb))
    A.close()
    R.close()


def test_entry_points_refused_while_loading(lx):
    """Between lx_load_rows and lx_load_finish the branch table is not rebuilt:
    ForklessCause, the getters, Flush, DropNotFlushed and the write-back return
    LX_ERR_STATE; after lx_load_finish they answer as the writing handle."""
    d = lx.tools.gen_dag(10, 30, 4, cheaters=2, forks=3, seed=13)
    w = [1] * 10
    A = lx.Index()
    A.reset(w)
    A.add_batch(d.creator, d.seq, d.poff, d.par)
    wb = A.writeback()
    A.flush()
    N = len(d)
    R = lx.Index()
    R.reset(w)
    R.load_rows(d.creator, d.seq, d.poff, d.par, b"".join(wb["b"][k] for k in range(N)),
                [wb["S"][k] for k in range(N)], [wb["s"][k] for k in range(N)])
    for call in (lambda: R.forkless_cause(N - 1, 0), lambda: R.highest_before(0), lambda: R.lowest_after(0),
                 lambda: R.merged_highest_before(0), lambda: R.branch(0), R.flush, R.drop_not_flushed,
                 R.writeback, R.branches_info):
        with pytest.raises(lx.LxError) as ei:
            call()
        assert ei.value.code == -4
    R.load_finish(wb["B"])
    for i in range(0, N, 5):
        assert R.highest_before(i) == A.highest_before(i) and R.lowest_after(i) == A.lowest_after(i)
    qa, qb = lx.tools.fc_queries(d.lamport, 5000, seed=2)
    np.testing.assert_array_equal(R.forkless_cause_batch(qa, qb), A.forkless_cause_batch(qa, qb))
    A.close()
    R.close()
