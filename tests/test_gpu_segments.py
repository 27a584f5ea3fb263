"""The segmented walk (option "segments", lx_segment.hip, DESIGN.md section
6b): a batch walked as G Add-order segments, each with its boundary parents as
own entries only, then fixed up from the frontier rows and the gathered rows
of the segments' first levels, LowestAfter filled from the final rows.  The
results must be the reference's: HB / LA bytes, branch IDs, merged HB and
ForklessCause against the C oracle, and whole planes against the ordinary
walk at larger sizes."""

import ctypes

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def make_index(lx, monkeypatch, G, cap=0, **more):
    from lachesis_hip import capi
    opts = dict(capi.DEFAULT_OPTIONS)
    opts.update(small_max=0, segments=G, **more)
    monkeypatch.setattr(capi, "DEFAULT_OPTIONS", opts)
    return lx.Index(event_capacity=cap) if cap else lx.Index()


def rows_equal_oracle(ix, o, events):
    for mode in (0, 1):
        (go, gb), (oo, ob) = ix.rows_np(mode, events), o.rows(mode, events)
        assert np.array_equal(go, oo) and np.array_equal(gb, ob), ("rows", mode)


def fc_sample(ix, o, n, k, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n, k).astype(np.uint32)
    b = np.clip(a.astype(np.int64) - rng.integers(0, 400, k), 0, n - 1).astype(np.uint32)
    np.testing.assert_array_equal(ix.forkless_cause_batch(a, b), o.forkless_cause_batch(a, b))


SHAPES = [
    # V, events/validator, parents, cheaters, forks, seed
    (50, 40, 6, 0, 0, 1),
    (100, 30, 10, 0, 0, 2),
    (64, 40, 8, 6, 6, 3),        # fork branches created inside later segments
    (30, 60, 16, 3, 10, 4),      # parents beyond the inline twelve
    (200, 12, 3, 0, 0, 5),       # segments shorter than one level: chains of gathered fix-ups
]


@pytest.mark.parametrize("G", [2, 3, 8, 32])
@pytest.mark.parametrize("shape", SHAPES)
def test_segmented_batch_vs_oracle(lx, monkeypatch, shape, G):
    V, epv, P, ch, fk, seed = shape
    d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
    if len(d) < 64 * G:
        pytest.skip("batch shorter than 64 events per segment")
    w = [1 + (i * 7) % 5 for i in range(V)]
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ix = make_index(lx, monkeypatch, G)
    ix.reset(w)
    br = ix.add_batch(d.creator, d.seq, d.poff, d.par, want_branches=True)
    st = ix.segment_stats()
    assert st["segments"] == G and st["first_event"][-1] == len(d)
    assert [int(x) for x in br] == [o.branch(i) for i in range(len(d))]
    ev = np.arange(len(d), dtype=np.uint32)
    rows_equal_oracle(ix, o, ev)
    for i in range(0, len(d), max(1, len(d) // 300)):
        assert ix.merged_highest_before(i) == o.merged_hb(i), i
    fc_sample(ix, o, len(d), 200_000, seed)


@pytest.mark.parametrize("G", [2, 5])
def test_segmented_second_batch(lx, monkeypatch, G):
    """Rows before the batch (final, with fork marks) are the frontier of
    segment 0; a later segmented batch, a flush and a rollback of it."""
    V = 40
    d = lx.tools.gen_dag(V, 80, 6, 4, 8, seed=9)
    w = [3 + i % 4 for i in range(V)]
    N = len(d)
    cut, cut2 = N // 3, 2 * N // 3
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ix = make_index(lx, monkeypatch, G)
    ix.reset(w)
    ix.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par)
    ix.flush()
    ix.add_batch(d.creator[cut:cut2], d.seq[cut:cut2], d.poff[cut:cut2 + 1] - d.poff[cut], d.par[d.poff[cut]:])
    assert ix.segment_stats()["first_event"][0] == cut
    ix.flush()
    # a batch that is dropped again, then the rest
    ix.add_batch(d.creator[cut2:], d.seq[cut2:], d.poff[cut2:] - d.poff[cut2], d.par[d.poff[cut2]:])
    ix.drop_not_flushed()
    ix.add_batch(d.creator[cut2:], d.seq[cut2:], d.poff[cut2:] - d.poff[cut2], d.par[d.poff[cut2]:])
    rows_equal_oracle(ix, o, np.arange(N, dtype=np.uint32))
    fc_sample(ix, o, N, 100_000, 4)


def _plane(ptr, rows, stride, cols):
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.empty((rows, stride), dtype=np.uint32)
    assert hip.hipMemcpy(out.ctypes.data, ptr, out.nbytes, 2) == 0
    return out[:, :cols]


@pytest.mark.parametrize("G", [4, 8])
def test_segmented_config3_shape_planes(lx, monkeypatch, G):
    """V = 1000 with Zipf stakes (BASELINE configs[2]'s shape), 150k events:
    both planes byte-identical to the ordinary walk's (g = 0 with seg_auto = 0:
    ONE walk of the batch, not the side-by-side segments seg_auto would pick at
    this size), which the parity tests pin to the oracle; a prefix of rows
    against the oracle directly."""
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 150, 10, seed=1)
    N = len(d)
    planes = []
    for g in (0, G):
        ix = make_index(lx, monkeypatch, g, cap=N, seg_auto=0 if g == 0 else 1)
        ix.reset(w)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ix.sync()
        if g == 0:
            assert ix.segment_stats()["segments"] == 0      # really the single walk
        hb, la, stride, _ = ix.device_planes()
        planes.append((_plane(hb, N, stride, V), _plane(la, N, stride, V)))
        if g:
            st = ix.segment_stats()
            assert sum(st["partial"]) < N // 4, st["partial"]
            o = corc.OracleIndex(w)
            P = 20_000
            assert o.add_batch(d.creator[:P], d.seq[:P], d.poff[:P + 1], d.par) == -1
            ev = np.arange(0, P, 7, dtype=np.uint32)
            (go, gb), (oo, ob) = ix.rows_np(0, ev), o.rows(0, ev)
            assert np.array_equal(gb, ob)
            fc_sample(ix, o, P, 100_000, 5)
        ix.close()
    np.testing.assert_array_equal(planes[0][0], planes[1][0])
    np.testing.assert_array_equal(planes[0][1], planes[1][1])


@pytest.mark.parametrize("shape", [(60, 2500, 8, 3, 4), (100, 1400, 10, 0, 0)])
def test_auto_segments_side_by_side(lx, monkeypatch, shape):
    """A walk of few columns leaves CUs idle: the batch is split on its own
    (seg_auto, the default) into Add-order segments walked by one launch side
    by side.  Both planes byte-identical to the single walk (seg_auto = 0),
    HighestBefore rows of a prefix and ForklessCause against the oracle."""
    V, epv, P, ch, fk = shape
    d = lx.tools.gen_dag(V, epv, P, ch, fk, seed=17)
    N = len(d)
    w = [1 + (i * 7) % 11 for i in range(V)]
    planes = []
    for auto in (0, 1):
        ix = lx.Index(event_capacity=N, options={"seg_auto": auto})
        ix.reset(w)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ix.sync()
        B = ix.num_branches()
        hb, la, stride, _ = ix.device_planes()
        planes.append((_plane(hb, N, stride, B), _plane(la, N, stride, B)))
        if auto:
            st = ix.segment_stats()
            assert st["segments"] >= 2, st
            o = corc.OracleIndex(w)
            Pn = 20_000
            assert o.add_batch(d.creator[:Pn], d.seq[:Pn], d.poff[:Pn + 1], d.par) == -1
            ev = np.arange(0, Pn, 9, dtype=np.uint32)
            # HighestBefore of a prefix (its LowestAfter rows fill from later events)
            assert np.array_equal(ix.rows_np(0, ev)[1], o.rows(0, ev)[1])
            fc_sample(ix, o, Pn, 50_000, 3)
        ix.close()
    np.testing.assert_array_equal(planes[0][0], planes[1][0])
    np.testing.assert_array_equal(planes[0][1], planes[1][1])
