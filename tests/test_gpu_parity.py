"""Parity of the HIP path with the oracle (run on an MI355X: pytest -m gpu).

Every test calls the product through the C ABI (lachesis_hip over
liblachesis_hip.so) and compares with the CPU oracle on the same seeded input:
bit-exact HB / LA bytes, branch IDs, merged HB and ForklessCause booleans.
"""

import numpy as np
import pytest

from oracle import corc, pos, tdag
from oracle import vecfc_oracle as vo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


@pytest.fixture
def opts(monkeypatch):
    """Set lx_set_option values for every Index this test creates."""
    from lachesis_hip import capi

    def set_(**kw):
        for k, v in kw.items():
            monkeypatch.setitem(capi.DEFAULT_OPTIONS, k, v)
    return set_


@pytest.fixture(params=["small", "big"], autouse=True)
def add_path(request, opts):
    """Every test runs twice: host-pointer batches of <= 3072 events take the
    small-batch path (host branch assignment + k_small, lx_small.hip) by
    default; option small_max=0 sends every batch through the device-assigned
    walker path (k_index)."""
    if request.param == "big":
        opts(small_max=0)
    elif request.node.get_closest_marker("big_only"):
        pytest.skip("every batch of this test is larger than the small path takes")
    return request.param


def oracle_for(dag, weights, flush_each=False):
    o = corc.OracleIndex(weights)
    r = o.add_batch(dag.creator, dag.seq, dag.poff, dag.par, flush_each=flush_each)
    assert r == -1
    return o


def compare_rows(ix, o, events, check_merged=True):
    for i in events:
        i = int(i)
        assert ix.highest_before(i) == o.hb(i), ("hb", i)
        assert ix.lowest_after(i) == o.la(i), ("la", i)
        assert ix.branch(i) == o.branch(i), ("branch", i)
        if check_merged:
            assert ix.merged_highest_before(i) == o.merged_hb(i), ("merged", i)


# ---------------------------------------------------------------- golden tables
@pytest.mark.parametrize("case", ["classic_step3", "classic_step4", "classic_step5", "random_80"])
@pytest.mark.parametrize("batched", [False, True])
def test_golden_forkless_cause(lx, golden, case, batched):
    """TestForklessCausedClassic / TestForklessCausedRandom through the HIP path."""
    c = next(x for x in golden["fc_cases"] if x["name"] == case)
    nodes, _, names, ordered = tdag.ascii_scheme_for_each(c["scheme"])
    validators = pos.Validators.equal(nodes, 1)
    ix = lx.VecfcIndex()
    ix.reset(validators)
    if batched:
        ix.add_events(ordered)
    else:
        for e in ordered:
            ix.add(e)
            ix.flush()
    for who, e1 in names.items():
        for whom, e2 in names.items():
            assert ix.forkless_cause(e1.id, e2.id) == (whom in c["fc"][who]), (who, whom)


def test_golden_bench15_rows(lx, golden):
    c = next(x for x in golden["fc_cases"] if x["name"] == "bench_15")
    nodes, _, names, ordered = tdag.ascii_scheme_for_each(c["scheme"])
    validators = pos.Validators.equal(nodes, 1)
    store = {e.id: e for e in ordered}
    py = vo.Index()
    py.reset(validators, store.get)
    ix = lx.VecfcIndex()
    ix.reset(validators)
    for e in ordered:
        py.add(e)
        ix.add(e)
    for e in ordered:
        assert ix.get_highest_before(e.id).to_bytes() == py.get_highest_before(e.id).to_bytes()
        assert ix.get_lowest_after(e.id).to_bytes() == py.get_lowest_after(e.id).to_bytes()
        for f in ordered:
            assert ix.forkless_cause(e.id, f.id) == py.forkless_cause(e.id, f.id)


# ---------------------------------------------------------------- random fork DAGs
FORK_SHAPES = [
    # nodes, events/node, parents, cheaters, forks, seed
    (1, 10, 1, 1, 3, 0), (2, 10, 1, 1, 3, 1), (2, 10, 2, 2, 20, 2), (10, 10, 4, 1, 3, 3),
    (10, 10, 4, 10, 3, 4), (20, 5, 4, 10, 2, 5), (40, 3, 4, 10, 1, 6), (5, 30, 4, 2, 30, 7),
    (8, 60, 4, 3, 30, 8), (30, 40, 6, 5, 8, 9), (64, 20, 8, 6, 6, 10), (100, 12, 10, 10, 10, 11),
]


@pytest.mark.parametrize("shape", FORK_SHAPES)
def test_fork_dag_rows_and_fc(lx, shape):
    n, ev, p, ch, fk, seed = shape
    d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
    rng = np.random.default_rng(seed)
    weights = sorted((int(x) for x in rng.integers(1, 9, n)), reverse=True)
    o = oracle_for(d, weights)
    ix = lx.Index()
    ix.reset(weights)
    br = ix.add_batch(d.creator, d.seq, d.poff, d.par, want_branches=True)
    assert ix.num_branches() == o.num_branches()
    assert [int(x) for x in br] == [o.branch(i) for i in range(len(d))]
    compare_rows(ix, o, range(len(d)))
    N = len(d)
    a = np.repeat(np.arange(N, dtype=np.uint32), N)
    b = np.tile(np.arange(N, dtype=np.uint32), N)
    if len(a) > 400_000:
        sel = rng.choice(len(a), 400_000, replace=False)
        a, b = a[sel], b[sel]
    np.testing.assert_array_equal(ix.forkless_cause_batch(a, b), o.forkless_cause_batch(a, b))
    ls, cr = ix.branches_info()
    assert len(ls) == o.num_branches()


@pytest.mark.parametrize("cheaters", [20, 40, 70])
@pytest.mark.parametrize("fk", ["1", "0"])
def test_fork_fc_paths(lx, cheaters, fk, opts):
    """The fork-path ForklessCause kernels: every plane column streamed with a
    32-bit (<= 32 cheaters) or 64-bit cheater mask (k_fc_fk), and the cheater
    fix-up loop (k_fc<.., true>: > 64 cheaters, or LX_FC_FK=0), all equal to
    the oracle; Zipf stakes so the per-creator dedupe weighs differently."""
    opts(fc_fk=int(fk))
    n = 100
    d = lx.tools.gen_dag(n, 14, 10, cheaters=cheaters, forks=4, seed=cheaters)
    weights = [(1 << 20) // (i + 1) for i in range(n)]
    o = oracle_for(d, weights)
    ix = lx.Index()
    ix.reset(weights)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    assert ix.num_branches() == o.num_branches() > n
    N = len(d)
    rng = np.random.default_rng(cheaters)
    a = rng.integers(0, N, 300_000, dtype=np.uint32)
    b = np.minimum(a, rng.integers(0, N, 300_000, dtype=np.uint32))
    b = np.where(rng.random(300_000) < 0.5, np.maximum(a.astype(np.int64) - rng.integers(0, 400, 300_000), 0), b).astype(np.uint32)
    np.testing.assert_array_equal(ix.forkless_cause_batch(a, b), o.forkless_cause_batch(a, b))


@pytest.mark.parametrize("chunk", [1, 7, 64, 1000])
def test_batching_is_bit_exact(lx, chunk):
    """lx_add_batch over any split equals per-event Add (fork-heavy DAG)."""
    d = lx.tools.gen_dag(12, 40, 5, cheaters=4, forks=8, seed=21)
    w = [1] * 12
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    N = len(d)
    for lo in range(0, N, chunk):
        hi = min(N, lo + chunk)
        ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
    compare_rows(ix, o, range(N))


def test_drop_not_flushed_rollback(lx):
    """Rollback to the last flush undoes new rows, LA entries set in old rows,
    fork branches and branch claims; re-adding reproduces the oracle."""
    d = lx.tools.gen_dag(10, 30, 4, cheaters=3, forks=6, seed=5)
    w = list(range(10, 0, -1))
    N = len(d)
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    cut = N // 3
    ix.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par)
    ix.flush()
    B_flushed = ix.num_branches()
    o2 = corc.OracleIndex(w)
    o2.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par)
    for attempt in range(3):
        hi = cut + (N - cut) * (attempt + 1) // 3
        ix.add_batch(d.creator[cut:hi], d.seq[cut:hi], d.poff[cut:hi + 1], d.par)
        ix.drop_not_flushed()
        assert ix.num_events() == cut
        assert ix.num_branches() == B_flushed
        compare_rows(ix, o2, range(cut))
    ix.add_batch(d.creator[cut:], d.seq[cut:], d.poff[cut:], d.par)
    compare_rows(ix, o, range(N))


def test_build_then_drop_per_event(lx):
    """IndexedLachesis.Build pattern (abft/indexed_lachesis.go:53-63): every
    event is first added and dropped (Build), then added and flushed (Process)."""
    d = lx.tools.gen_dag(6, 25, 3, cheaters=2, forks=5, seed=13)
    w = [3, 3, 2, 2, 1, 1]
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    for i in range(len(d)):
        s = slice(i, i + 1)
        ix.add_batch(d.creator[s], d.seq[s], d.poff[i:i + 2], d.par)
        ix.drop_not_flushed()
        ix.add_batch(d.creator[s], d.seq[s], d.poff[i:i + 2], d.par)
        ix.flush()
    compare_rows(ix, o, range(len(d)))


def test_reorder_invariance(lx):
    """TestRandomForks (:719-744): FC over all pairs is invariant under random
    parents-first reorderings (branch IDs may differ)."""
    n = 8
    nodes, evs = tdag.rand_fork_dag(n, 12, 4, cheaters=3, forks_count=5, seed=17)
    validators = pos.Validators.equal(nodes)
    ref = lx.VecfcIndex()
    ref.reset(validators)
    ref.add_events(evs)
    fc = {(a.id, b.id): ref.forkless_cause(a.id, b.id) for a in evs for b in evs}
    rng = tdag.SplitMix64(99)
    order = evs
    for _ in range(3):
        order = tdag.by_parents(tdag.shuffle(order, rng))
        ix = lx.VecfcIndex()
        ix.reset(validators)
        ix.add_events(order)
        for a in order:
            for b in order:
                assert ix.forkless_cause(a.id, b.id) == fc[(a.id, b.id)]
        ix.drop_not_flushed()
        for e in order:
            assert ix.get_highest_before(e.id) is None


def test_random_forks_sanity_merged(lx):
    """TestRandomForksSanity (:520-576) through the HIP path."""
    n = 8
    rng = tdag.SplitMix64(42)
    node_ids = [rng.next() & 0xFFFFFFFF for _ in range(n)]
    w = {v: 1 for v in node_ids}
    w[node_ids[0]] = 2
    w[node_ids[3]] = 2
    w[node_ids[4]] = 3
    validators = pos.Validators(w)
    nodes, evs = tdag.rand_fork_dag(n, 300, 4, cheaters=3, forks_count=30, seed=5, node_ids=node_ids)
    ix = lx.VecfcIndex()
    ix.reset(validators)
    ix.add_events(evs)
    ix.flush()
    ix.drop_not_flushed()
    last = {}
    for e in evs:
        last[e.creator] = e
    for node in nodes:
        mhb = ix.get_merged_highest_before(last[node].id)
        for k, cheater in enumerate(nodes):
            bs = mhb.get(validators.idxs[cheater])
            assert bs.is_fork_detected() == (k < 3)
            if k < 3:
                assert bs.seq == 0
            else:
                assert bs.seq != 0


def test_errors_leave_state_unchanged(lx):
    d = lx.tools.gen_dag(4, 10, 3, seed=3)
    w = [1, 1, 1, 1]
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator[:20], d.seq[:20], d.poff[:21], d.par)
    bad_par = d.par.copy()
    # a parent index >= its own index: out of order (vecengine/index.go:159-161)
    lo, hi = d.poff[25], d.poff[26]
    bad_par[lo] = 30
    with pytest.raises(lx.LxError) as ei:
        ix.add_batch(d.creator[20:], d.seq[20:], d.poff[20:], bad_par)
    assert ei.value.code == -2 and ei.value.index == 5
    assert ix.num_events() == 20
    with pytest.raises(lx.LxError):
        ix.forkless_cause(0, 25)
    ix.add_batch(d.creator[20:], d.seq[20:], d.poff[20:], d.par)
    o = oracle_for(d, w)
    compare_rows(ix, o, range(len(d)))


# ---------------------------------------------------------------- configs
def test_config1_full(lx):
    """BASELINE configs[0]: 5 validators x 1000 events, P=5, no forks."""
    d = lx.tools.gen_dag(5, 1000, 5, seed=1)
    w = [1] * 5
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    compare_rows(ix, o, range(0, len(d), 7))
    qa, qb = lx.tools.fc_queries(d.lamport, 200_000, seed=4)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))


def test_config4_scaled(lx):
    """BASELINE configs[3] shape (V=100, 10 cheaters x F=10) at 60 events per
    validator (6k events): bit-exact rows, branches and FC vs the oracle."""
    d = lx.tools.gen_dag(100, 60, 10, cheaters=10, forks=10, seed=2)
    w = [1] * 100
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    N = len(d)
    for lo in range(0, N, 1500):
        ix.add_batch(d.creator[lo:lo + 1500], d.seq[lo:lo + 1500], d.poff[lo:min(N, lo + 1500) + 1], d.par)
    assert ix.num_branches() == o.num_branches() > 100
    compare_rows(ix, o, range(0, N, 3))
    qa, qb = lx.tools.fc_queries(d.lamport, 300_000, seed=5)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))


def test_config4_full(lx):
    """BASELINE configs[3] at full size: V=100, first 10 validators double-sign
    (F=10 forks each), 1000 events per validator (100k events, ~157 branches):
    bit-exact branch IDs, every 5th HB/LA/merged row and 300k FC vs the oracle;
    indexed as one batch and as per-level-sized batches."""
    d = lx.tools.gen_dag(100, 1000, 10, cheaters=10, forks=10, seed=2)
    w = [1] * 100
    o = oracle_for(d, w)
    N = len(d)
    qa, qb = lx.tools.fc_queries(d.lamport, 300_000, seed=5)
    want = o.forkless_cause_batch(qa, qb)
    for chunk in (N, 64):
        ix = lx.Index(event_capacity=N)
        ix.reset(w)
        br = []
        for lo in range(0, N, chunk):
            hi = min(N, lo + chunk)
            br.extend(int(x) for x in ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par,
                                                   want_branches=True))
        assert ix.num_branches() == o.num_branches() > 100
        assert br == [o.branch(i) for i in range(N)]
        compare_rows(ix, o, range(0, N, 5 if chunk == N else 97))
        np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), want)
        ix.close()


def test_config3_shape_skewed(lx):
    """BASELINE configs[2] shape: V=1000, Zipf weights floor(2^20/(i+1)), P=10,
    at 8 events per validator (8k events) vs the oracle."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 8, 10, seed=3)
    o = oracle_for(d, w)
    ix = lx.Index()
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    compare_rows(ix, o, range(0, len(d), 97))
    qa, qb = lx.tools.fc_queries(d.lamport, 100_000, seed=6)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))


def _rows_in_chunks(ix, o, mode, events, chunk):
    """GPU and oracle rows of `events` (mode 0 HighestBefore, 1 LowestAfter),
    chunk by chunk: yields (offsets, bytes) pairs of both."""
    for lo in range(0, len(events), chunk):
        ev = events[lo:lo + chunk]
        yield ix.rows_np(mode, ev), o.rows(mode, ev)


@pytest.mark.big_only
def test_full_size_config3_prefix_vs_oracle(lx):
    """BASELINE configs[2] at full size (V=1000, Zipf stakes, 10M events, one
    batch -- the bench workload) against the C oracle on the first 500k
    events, EVERY row: HighestBefore rows of prefix events are final, so they
    must be byte-identical; LowestAfter: every entry the oracle has set is
    final and must be identical, and an entry the oracle has not set must be 0
    or come from an event after the prefix (a seq beyond the prefix's last seq
    of that branch); ForklessCause of 1M pairs between prefix events must be
    identical (an entry set after the prefix never counts for a prefix a)."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 10_000, 10, seed=1)
    N = len(d)
    ix = lx.Index(event_capacity=N)
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    P = 500_000
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator[:P], d.seq[:P], d.poff[:P + 1], d.par) == -1
    last = np.zeros(V, dtype=np.uint32)                    # last seq of each branch inside the prefix
    np.maximum.at(last, d.creator[:P], d.seq[:P])
    ev = np.arange(P, dtype=np.uint32)
    for (go, gb), (oo, ob) in _rows_in_chunks(ix, o, 0, ev, 50_000):
        np.testing.assert_array_equal(go, oo)
        assert np.array_equal(gb, ob)
    for (go, gb), (oo, ob) in _rows_in_chunks(ix, o, 1, ev, 50_000):
        np.testing.assert_array_equal(go, oo)              # no forks: every LA row is 4 V bytes on both sides
        g = gb.view(np.uint32).reshape(-1, V)
        want = ob.view(np.uint32).reshape(-1, V)
        set_ = want != 0
        assert np.array_equal(g[set_], want[set_])
        later = g[~set_]
        assert np.all((later == 0) | (later > np.broadcast_to(last, g.shape)[~set_]))
    qa, qb = lx.tools.fc_queries(d.lamport[:P], 1_000_000, seed=5)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch_mt(qa, qb, 16))
    ix.close()


@pytest.mark.big_only
@pytest.mark.parametrize("walk_opts", [None, {"seg_xmap": 1}])
def test_config3_shape_1m_default_segments_vs_oracle(lx, walk_opts):
    """The headline walk as shipped, pinned end to end: BASELINE configs[2]'s
    shape (V=1000, Zipf stakes, P=10) at 1,000 events per validator (1M
    events), indexed as one batch with DEFAULT options.  seg_auto then walks
    it as three side-by-side Add-order segments of 12-column slices (the 10M
    headline's exact configuration: k_index_segs<12 columns, 7 drains>), so the
    later segments -- their boundary parents, their partial-event fix-up
    (k_seg_partial) and their edge LowestAfter pass (k_seg_la_edge) -- lie
    inside the oracle's coverage.  EVERY HighestBefore and LowestAfter row of
    the epoch byte-identical, branch IDs, and 1M ForklessCause pairs of which
    most span the segment boundary (vecengine/index.go:144-233,
    vecengine/traversal.go:13-37, vecfc/forkless_cause.go:40-82).  walk_opts:
    the slice -> workgroup mapping of option seg_xmap (whole 8-slice groups
    per XCD)."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 1000, 10, seed=11)
    N = len(d)
    ix = lx.Index(event_capacity=N, options=walk_opts)
    ix.reset(w)
    br = ix.add_batch(d.creator, d.seq, d.poff, d.par, want_branches=True)
    st = ix.segment_stats()
    assert st["segments"] == 3, st                        # the side-by-side form of the headline
    cut, cut2 = st["first_event"][1], st["first_event"][2]
    assert 0 < cut < cut2 < N and cut % 64 == 0 and cut2 % 64 == 0, st
    assert st["partial"][1] > 0 and st["partial"][2] > 0, st
    assert np.array_equal(np.asarray(br, dtype=np.uint32), d.creator)   # fork-free: branch = creator
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ev = np.arange(N, dtype=np.uint32)
    for mode in (0, 1):
        for (go, gb), (oo, ob) in _rows_in_chunks(ix, o, mode, ev, 50_000):
            np.testing.assert_array_equal(go, oo)
            assert np.array_equal(gb, ob), mode
    # 1M pairs: half with a among the first 20k events of segment 1 or 2 and b
    # up to 25k events before it (most of them in the segment before), half of
    # the bench's shape (a uniform, b within 64 Lamport of a)
    rng = np.random.default_rng(12)
    qa1 = (np.where(rng.integers(0, 2, 500_000) == 0, cut, cut2) + rng.integers(0, 20_000, 500_000)).astype(np.int64)
    qb1 = qa1 - rng.integers(1, 25_000, 500_000)
    qa2, qb2 = lx.tools.fc_queries(d.lamport, 500_000, window=64, seed=13)
    qa = np.concatenate([qa1, qa2]).astype(np.uint32)
    qb = np.concatenate([qb1, qb2]).astype(np.uint32)
    assert int((((qa >= cut) & (qb < cut)) | ((qa >= cut2) & (qb < cut2))).sum()) > 250_000
    got = ix.forkless_cause_batch(qa, qb)
    want = o.forkless_cause_batch_mt(qa, qb, 16)
    np.testing.assert_array_equal(got, want)
    assert 0.05 < want.mean() < 0.95                     # both answers occur
    ix.close()


def _planes_equal_on_device(ixs, n, cols, chunk_rows=1 << 18):
    """Both planes of two handles compared on the GPU, chunk by chunk: the
    rows are copied device to device into torch buffers (hipMemcpy) and
    compared there, so 2 x 87 GB never crosses PCIe."""
    import ctypes
    import torch
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    planes = [ix.device_planes() for ix in ixs]
    strides = {p[2] for p in planes}
    assert len(strides) == 1
    stride = strides.pop()
    bufs = [torch.empty((chunk_rows, stride), dtype=torch.int32, device="cuda") for _ in ixs]
    for k in (0, 1):                                       # 0: hb, 1: la
        for lo in range(0, n, chunk_rows):
            m = min(chunk_rows, n - lo)
            for buf, p in zip(bufs, planes):
                src = p[k] + lo * stride * 4
                assert hip.hipMemcpy(buf.data_ptr(), src, m * stride * 4, 3) == 0
            torch.cuda.synchronize()
            if not torch.equal(bufs[0][:m, :cols], bufs[1][:m, :cols]):
                bad = (bufs[0][:m, :cols] != bufs[1][:m, :cols]).nonzero()[:5].tolist()
                raise AssertionError(f"plane {k} rows {lo}..{lo + m}: first mismatches {bad}")


@pytest.mark.big_only
def test_full_size_config3_segments_equal_single_walk(lx):
    """BASELINE configs[2] at full size (10M events, the bench workload): the
    default handle (three side-by-side segments of 12-column slices) and a
    seg_auto=0 handle (ONE 4-column walk of the batch) hold byte-identical
    HighestBefore and LowestAfter planes, every row -- the segments of the
    shipped walk after the first included.  The single walk is the one pinned
    to the oracle at full size on its 500k prefix (above) and in every
    smaller configs[2]-shaped test."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 10_000, 10, seed=1)
    N = len(d)
    ixs = []
    for auto in (1, 0):
        ix = lx.Index(event_capacity=N, options={"seg_auto": auto})
        ix.reset(w)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ix.sync()
        st = ix.segment_stats()
        assert st["segments"] == (3 if auto else 0), st
        ixs.append(ix)
    _planes_equal_on_device(ixs, N, V)
    qa, qb = lx.tools.fc_queries(d.lamport, 1 << 22, seed=21)
    np.testing.assert_array_equal(ixs[0].forkless_cause_batch(qa, qb), ixs[1].forkless_cause_batch(qa, qb))
    for ix in ixs:
        ix.close()


@pytest.mark.big_only
def test_full_size_config2_vs_oracle(lx):
    """BASELINE configs[1] at full size (V=100, 1M events) against the C
    oracle over the whole epoch: every HighestBefore row, every LowestAfter row
    (byte-identical, lengths included) and 1M ForklessCause answers."""
    V = 100
    d = lx.tools.gen_dag(V, 10_000, 10, seed=1)
    N = len(d)
    ix = lx.Index(event_capacity=N)
    ix.reset([1] * V)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    o = corc.OracleIndex([1] * V)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ev = np.arange(N, dtype=np.uint32)
    for mode in (0, 1):
        for (go, gb), (oo, ob) in _rows_in_chunks(ix, o, mode, ev, 250_000):
            np.testing.assert_array_equal(go, oo)
            assert np.array_equal(gb, ob), mode
    qa, qb = lx.tools.fc_queries(d.lamport, 1_000_000, window=64, seed=9)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch_mt(qa, qb, 16))
    ix.close()


@pytest.mark.big_only
def test_full_size_properties_config2(lx):
    """BASELINE configs[1] at full size (V=100, 1M events): size-independent
    properties.  (i) HB of an event on branch j at seq s equals s on column j;
    (ii) LA/HB duality: LA(x)[j]=s  <=>  HB((j,s))[br(x)] >= seq(x) and
    HB((j,s-1))[br(x)] < seq(x); (iii) HB monotone along each branch."""
    V = 100
    d = lx.tools.gen_dag(V, 10_000, 10, seed=1)
    ix = lx.Index(event_capacity=len(d))
    ix.reset([1] * V)
    N = len(d)
    step = 250_000
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1], d.par)
    rng = np.random.default_rng(0)
    # index of event (creator c, seq s) in creation order: (s-1)*V + c
    ev = lambda c, s: (s - 1) * V + c
    for x in rng.integers(0, N - 5 * V, 200):
        x = int(x)
        hb = np.frombuffer(ix.highest_before(x), dtype=np.uint32).reshape(-1, 2)
        cx, sx = int(d.creator[x]), int(d.seq[x])
        assert hb[cx, 0] == sx
        la = np.frombuffer(ix.lowest_after(x), dtype=np.uint32)
        for j in rng.integers(0, V, 5):
            j = int(j)
            s = int(la[j])
            if s == 0:
                continue
            hbj = np.frombuffer(ix.highest_before(ev(j, s)), dtype=np.uint32).reshape(-1, 2)
            assert hbj[cx, 0] >= sx
            if s > 1:
                hbp = np.frombuffer(ix.highest_before(ev(j, s - 1)), dtype=np.uint32).reshape(-1, 2)
                assert hbp[cx, 0] < sx
            nxt = ev(cx, sx + 1)
            if nxt < N:
                hbn = np.frombuffer(ix.highest_before(nxt), dtype=np.uint32).reshape(-1, 2)
                assert np.all(hbn[:, 0] >= hb[:, 0])
    # FC sample against a direct evaluation from the getters
    qa, qb = lx.tools.fc_queries(d.lamport, 2000, seed=9)
    got = ix.forkless_cause_batch(qa, qb)
    for a, b, g in zip(qa[:300], qb[:300], got[:300]):
        hb = np.frombuffer(ix.highest_before(int(a)), dtype=np.uint32).reshape(-1, 2)[:, 0]
        la = np.frombuffer(ix.lowest_after(int(b)), dtype=np.uint32)
        cnt = int(np.sum((la != 0) & (la <= hb[:len(la)])))
        assert bool(g) == (cnt >= ix.quorum())


# ---------------------------------------------------------------- walker variants
# The shipped walker (block layout: 16-event blocks per wave, a quad of lanes
# per event, 4 drain waves) on 1-, 2- and 4-column slices, the last with the
# 16-bit packed slot unit (default while every seq fits) and with two units.
WALKER_VARIANTS = [{"cpw": 0}, {"cpw": 1}, {"cpw": 2}, {"cpw": 4}, {"cpw": 4, "pack16": 0}]


@pytest.mark.big_only
@pytest.mark.parametrize("env", WALKER_VARIANTS, ids=lambda e: "-".join("%s%s" % (k, v) for k, v in e.items()))
def test_walker_variants(lx, env, opts):
    """Every shipped walker configuration (slice widths, slot layouts) is
    bit-exact; the DAG is long enough (6000 events, cheaters) that ring slots
    are reused and parents older than the ring take the L2 path."""
    opts(**env)
    d = lx.tools.gen_dag(24, 250, 6, 4, 6, 21)
    weights = list(range(40, 16, -1))
    o = oracle_for(d, weights)
    ix = lx.Index()
    ix.reset(weights)
    br = ix.add_batch(d.creator, d.seq, d.poff, d.par, want_branches=True)
    assert [int(x) for x in br] == [o.branch(i) for i in range(len(d))]
    rng = np.random.default_rng(5)
    compare_rows(ix, o, rng.choice(len(d), 1500, replace=False))
    qa, qb = lx.tools.fc_queries(d.lamport, 200_000, window=32, seed=4)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


@pytest.mark.big_only
@pytest.mark.parametrize("cpw", ["4", "4u", "1", "2"])
def test_walker_many_parents(lx, cpw, opts):
    """Events with more parents than a record holds inline (16 > 12) take the
    overflow path of the walker, on each slice width (4u: two slot units per
    event instead of the packed 16-bit one)."""
    if cpw.endswith("u"):
        cpw = cpw[:-1]
        opts(pack16=0)
    opts(cpw=int(cpw))
    d = lx.tools.gen_dag(30, 120, 16, 3, 4, 77)
    assert int(np.max(np.diff(d.poff))) > 12
    weights = list(range(70, 40, -1))
    o = oracle_for(d, weights)
    ix = lx.Index()
    ix.reset(weights)
    br = ix.add_batch(d.creator, d.seq, d.poff, d.par, want_branches=True)
    assert [int(x) for x in br] == [o.branch(i) for i in range(len(d))]
    compare_rows(ix, o, range(len(d)))
    qa, qb = lx.tools.fc_queries(d.lamport, 100_000, window=32, seed=8)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


@pytest.mark.big_only
def test_walker_seqs_beyond_16_bits(lx, opts):
    """4-column slices with seqs above 0xFFFF: the walker must not use the
    packed 16-bit slot units (rows and FC still equal the oracle)."""
    opts(cpw=4)
    weights = [3, 2]
    big = lx.tools.gen_dag(2, 66000, 2, 0, 0, 6)
    assert int(big.seq.max()) > 0xFFFF
    o = oracle_for(big, weights)
    ix = lx.Index()
    ix.reset(weights)
    ix.add_batch(big.creator, big.seq, big.poff, big.par)
    rng = np.random.default_rng(9)
    compare_rows(ix, o, np.concatenate([rng.choice(len(big), 2000, replace=False), np.arange(len(big) - 300, len(big))]))
    qa, qb = lx.tools.fc_queries(big.lamport, 100_000, window=32, seed=3)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


def far_parent_dag(lx, n_nodes, n, seed):
    """A valid DAG whose non-self parents are uniform over ALL earlier events:
    many parents lie thousands of events back, beyond the walker's LDS ring, so
    their slots are reused while their children wait (the L2 fallback paths)."""
    rng = np.random.default_rng(seed)
    creator = np.zeros(n, dtype=np.uint32)
    seq = np.zeros(n, dtype=np.uint32)
    lam = np.zeros(n, dtype=np.uint32)
    poff = [0]
    par = []
    last = [-1] * n_nodes
    for i in range(n):
        c = int(rng.integers(n_nodes))
        ps = [last[c]] if last[c] >= 0 else []
        if i:
            for x in rng.integers(0, i, size=int(rng.integers(0, 5))):
                if int(x) not in ps and creator[int(x)] != c:
                    ps.append(int(x))
        creator[i] = c
        seq[i] = (seq[last[c]] + 1) if last[c] >= 0 else 1
        lam[i] = 1 + max([int(lam[p]) for p in ps], default=0)
        last[c] = i
        par.extend(ps)
        poff.append(len(par))
    return lx.tools.Dag(creator, seq, lam, np.array(poff, dtype=np.uint64), np.array(par or [0], dtype=np.uint32),
                        n_nodes)


@pytest.mark.big_only
@pytest.mark.parametrize("cpw", [4, 1, 2])
def test_walker_far_parents(lx, cpw, opts):
    """Parents far older than the ring (slot reuse while an event waits) in
    one batch and across batches, for each slice width, bit-exact."""
    opts(cpw=cpw)
    d = far_parent_dag(lx, 16, 12000, 91)
    weights = list(range(50, 34, -1))
    o = oracle_for(d, weights)
    for chunks in (1, 3):
        ix = lx.Index()
        ix.reset(weights)
        cuts = np.linspace(0, len(d), chunks + 1).astype(int)
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            p0, p1 = int(d.poff[lo]), int(d.poff[hi])
            ix.add_batch(d.creator[lo:hi], d.seq[lo:hi], d.poff[lo:hi + 1] - p0, d.par[p0:p1])
        rng = np.random.default_rng(chunks)
        compare_rows(ix, o, rng.choice(len(d), 1500, replace=False))
        qa, qb = lx.tools.fc_queries(d.lamport, 100_000, window=64, seed=4)
        np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
        ix.close()


def test_reset_reuses_planes(lx):
    """lx_reset on a used handle (same layout) clears exactly what the next epoch
    may read: epoch 1 dirties fork-branch columns, epoch 2 (different V, new
    forks, more events) must still equal a fresh oracle bit for bit."""
    ix = lx.Index()
    for (n, ev, p, ch, fk, seed) in [(20, 120, 5, 5, 8, 31), (24, 150, 6, 6, 6, 32), (20, 40, 4, 3, 4, 33)]:
        d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
        w = list(range(60, 60 - n, -1))
        o = oracle_for(d, w)
        ix.reset(w)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        assert ix.num_branches() == o.num_branches() > n
        compare_rows(ix, o, range(len(d)))
        qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=32, seed=seed)
        np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix.close()


@pytest.mark.parametrize("shards", [1, 2])
def test_reset_shrinking_validator_set(lx, shards):
    """Epochs without forks followed by one with fewer validators: the previous
    epoch's original columns beyond the new V become fork columns and must read
    as empty (reset zeroes the columns rows may have written)."""
    ixs = [lx.Index(shard_rank=r, shard_count=shards) for r in range(shards)]
    for (n, ev, p, ch, fk, seed) in [(40, 60, 6, 0, 0, 41), (24, 80, 5, 0, 0, 42), (16, 90, 5, 4, 6, 43)]:
        d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
        w = list(range(70, 70 - n, -1))
        o = oracle_for(d, w)
        for ix in ixs:
            ix.reset(w)
            ix.add_batch(d.creator, d.seq, d.poff, d.par)
        qa, qb = lx.tools.fc_queries(d.lamport, 40_000, window=32, seed=seed)
        if shards == 1:
            compare_rows(ixs[0], o, range(len(d)))
            got = ixs[0].forkless_cause_batch(qa, qb)
        else:
            from test_gpu_shards import exchange, fc
            exchange(ixs)
            got = fc(lx, ixs, qa, qb)
        np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))
    for ix in ixs:
        ix.close()


@pytest.mark.parametrize("i", range(8))
def test_random_forks_gpu(lx, i):
    """TestRandomForks (vecfc/forkless_cause_test.go:578-747) through the HIP
    index: every event's HighestBefore fork flags equal the naive
    duplicate-(creator, seq) DFS over its subgraph (testForksDetected,
    :491-518, walked with the facade's DfsSubgraph); DropNotFlushed erases the
    unflushed vectors; ForklessCause is invariant under random topological
    reorderings (:719-744)."""
    from test_oracle_golden import RANDOM_FORKS, naive_forks_detected
    t = RANDOM_FORKS[i]
    rng = tdag.SplitMix64(1000 + i)
    node_ids = [rng.next() & 0xFFFFFFFF for _ in range(t["nodes"])]
    nodes, evs = tdag.rand_fork_dag(t["nodes"], t["events"], t["parents"], cheaters=t["cheaters"],
                                    forks_count=t["forks"], seed=i, node_ids=node_ids)
    validators = pos.Validators.equal(nodes, 1)
    store = {e.id: e for e in evs}
    ix = lx.VecfcIndex()
    ix.reset(validators, store.get)
    for e in evs:
        ix.add(e)
    for e in evs:
        hb = ix.get_highest_before(e.id)
        expected = naive_forks_detected(ix, e)
        for v in nodes:
            bs = hb.get(validators.idxs[v])
            assert bs.is_fork_detected() == (v in expected), (e.id, v)
            if v in expected:
                assert bs.seq == 0
    ids = [e.id for e in evs]

    def fc_all():
        qa = np.array([ix.pos[a] for a in ids for _ in ids], dtype=np.uint32)
        qb = np.array([ix.pos[b] for _ in ids for b in ids], dtype=np.uint32)
        return ix.ix.forkless_cause_batch(qa, qb)

    fc = fc_all()
    assert fc[:5].tolist() == [ix.forkless_cause(ids[0], b) for b in ids[:5]]
    ix.drop_not_flushed()
    for e in evs:
        assert ix.get_highest_before(e.id) is None
        assert ix.get_lowest_after(e.id) is None
    order = evs
    for _ in range(min(t["reorder"], 5)):
        order = tdag.by_parents(tdag.shuffle(order, rng))
        ix.add_events(order)
        np.testing.assert_array_equal(fc_all(), fc)
        ix.drop_not_flushed()


def _all_pairs_fc(ix, o, n):
    a = np.repeat(np.arange(n, dtype=np.uint32), n)
    b = np.tile(np.arange(n, dtype=np.uint32), n)
    np.testing.assert_array_equal(ix.forkless_cause_batch(a, b), o.forkless_cause_batch(a, b))


def test_la_tail_stale_rows(lx):
    """The LowestAfter plane is not zeroed at reset: after each batch the
    entries no branch has observed yet are zeroed (tail pass).  Epoch 1 dirties
    every row; epoch 2 has idle validators (branches without events), arrives
    in batches, is flushed, dropped and re-added with a longer stream that
    reaches rows epoch 2 had not used yet -- rows, all-pairs FC equal the oracle
    after every step."""
    ix = lx.Index()
    d1 = lx.tools.gen_dag(20, 60, 5, 0, 0, 51)
    w1 = [3] * 20
    ix.reset(w1)
    ix.add_batch(d1.creator, d1.seq, d1.poff, d1.par)
    _all_pairs_fc(ix, oracle_for(d1, w1), len(d1))

    d2 = lx.tools.gen_dag(16, 40, 4, 3, 4, 52)      # creators 0..15 of 20: 16..19 idle
    w2 = [5, 5, 4, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1]
    N = len(d2)
    ix.reset(w2)
    cuts = [0, 37, 150, 151, 300]
    for lo, hi in zip(cuts, cuts[1:]):
        ix.add_batch(d2.creator[lo:hi], d2.seq[lo:hi], d2.poff[lo:hi + 1], d2.par)
        o = corc.OracleIndex(w2)
        assert o.add_batch(d2.creator[:hi], d2.seq[:hi], d2.poff[:hi + 1], d2.par) == -1
        compare_rows(ix, o, range(hi), check_merged=False)
        _all_pairs_fc(ix, o, hi)
    ix.flush()
    ix.add_batch(d2.creator[300:420], d2.seq[300:420], d2.poff[300:421], d2.par)
    ix.drop_not_flushed()
    ix.add_batch(d2.creator[300:], d2.seq[300:], d2.poff[300:], d2.par)   # longer than the dropped part
    o = oracle_for(d2, w2)
    compare_rows(ix, o, range(N))
    _all_pairs_fc(ix, o, N)
    ix.close()


def test_la_memset_mode_matches(lx, opts):
    """Option la_memset=1 (zero the whole LowestAfter plane at reset, no tail
    pass) gives the same rows and FC as the default tail mode."""
    opts(la_memset=1)
    ix = lx.Index()
    for (n, ev, p, ch, fk, seed) in [(20, 50, 5, 3, 4, 61), (12, 40, 4, 2, 3, 62)]:
        d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
        w = list(range(40, 40 - n, -1))
        ix.reset(w)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        o = oracle_for(d, w)
        compare_rows(ix, o, range(len(d)))
        _all_pairs_fc(ix, o, len(d))
    ix.close()
