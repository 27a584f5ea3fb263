"""The walker on 8- and 12-column slices (packed 16-bit slot units in two 16-B
units: fork-free epochs whose seqs fit 16 bits), alone and as side-by-side segments:
rows and ForklessCause against the C oracle, planes byte-identical to the
4-column walk."""

import ctypes

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def _plane(ptr, rows, stride, cols):
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.empty((rows, stride), dtype=np.uint32)
    assert hip.hipMemcpy(out.ctypes.data, ptr, out.nbytes, 2) == 0
    return out[:, :cols]


def planes_of(lx, d, w, opts):
    ix = lx.Index(event_capacity=len(d), options=dict(small_max=0, dbl=0, **opts))
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    hb, la, stride, _ = ix.device_planes()
    B = ix.num_branches()
    out = (_plane(hb, len(d), stride, B), _plane(la, len(d), stride, B))
    return ix, out


@pytest.mark.parametrize("cpw", [8, 12])
@pytest.mark.parametrize("shape", [(24, 250, 6), (13, 400, 5), (30, 120, 16), (200, 60, 10)])
def test_cpw8_walk_vs_oracle_and_cpw4(lx, shape, cpw):
    """One walk on 8-column slices (ring slots reused, parents beyond the
    inline twelve, a partly filled last slice, many slices)."""
    V, epv, P = shape
    d = lx.tools.gen_dag(V, epv, P, seed=31 + V)
    w = [1 + (i * 5) % 9 for i in range(V)]
    N = len(d)
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ix8, p8 = planes_of(lx, d, w, {"cpw": cpw, "seg_auto": 0})
    ix4, p4 = planes_of(lx, d, w, {"cpw": 4, "seg_auto": 0})
    np.testing.assert_array_equal(p8[0], p4[0])
    np.testing.assert_array_equal(p8[1], p4[1])
    ev = np.arange(0, N, 5, dtype=np.uint32)
    for mode in (0, 1):
        assert np.array_equal(ix8.rows_np(mode, ev)[1], o.rows(mode, ev)[1]), mode
    qa, qb = lx.tools.fc_queries(d.lamport, 100_000, window=32, seed=V)
    np.testing.assert_array_equal(ix8.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    ix8.close()
    ix4.close()


@pytest.mark.parametrize("cpw,G", [(8, 4), (12, 3), (12, 4)])
@pytest.mark.parametrize("shape", [(64, 2100, 10), (100, 1400, 8), (1000, 60, 10)])
def test_cpw8_side_by_side_segments(lx, shape, cpw, G):
    """Segments side by side on 8- / 12-column slices (one k_index_segs
    launch; V = 1000 at 12 columns: 84 slices, three walks on 256 CUs)
    byte-identical to one walk."""
    V, epv, P = shape
    d = lx.tools.gen_dag(V, epv, P, seed=5)
    w = [1] * V
    ix8, p8 = planes_of(lx, d, w, {"cpw": cpw, "segments": G})
    st = ix8.segment_stats()
    assert st["segments"] == G, st
    ix1, p1 = planes_of(lx, d, w, {"seg_auto": 0})
    np.testing.assert_array_equal(p8[0], p1[0])
    np.testing.assert_array_equal(p8[1], p1[1])
    ix8.close()
    ix1.close()


@pytest.mark.parametrize("cpw", [8, 12])
def test_cpw8_falls_back_with_forks(lx, cpw):
    """cpw = 8 / 12 on a fork epoch walks 4-column slices (8-column slots need
    packed fork-free values): rows still equal the oracle."""
    d = lx.tools.gen_dag(20, 150, 6, 3, 4, seed=9)
    w = [2] * 20
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ix, _ = planes_of(lx, d, w, {"cpw": cpw})
    ev = np.arange(0, len(d), 3, dtype=np.uint32)
    for mode in (0, 1):
        assert np.array_equal(ix.rows_np(mode, ev)[1], o.rows(mode, ev)[1]), mode
    ix.close()


@pytest.mark.parametrize("shape", [(600, 300, 8), (250, 700, 10)])
def test_auto_12_column_segments_equal_single_walk(lx, shape):
    """Default options on fork-free epochs whose width seg_pick walks as
    side-by-side 12-column segments (V = 600: 50 slices, 5 walks; V = 250:
    21 slices, many walks): planes byte-identical to one 4-column walk, and
    a prefix of rows equal to the oracle."""
    V, epv, P = shape
    d = lx.tools.gen_dag(V, epv, P, seed=V)
    w = [1 + (i * 7) % 11 for i in range(V)]
    ixa, pa = planes_of(lx, d, w, {})
    st = ixa.segment_stats()
    assert st["segments"] >= 2 and st["one_launch"], st
    ix1, p1 = planes_of(lx, d, w, {"seg_auto": 0, "cpw": 4})
    np.testing.assert_array_equal(pa[0], p1[0])
    np.testing.assert_array_equal(pa[1], p1[1])
    o = corc.OracleIndex(w)
    n = 20_000
    assert o.add_batch(d.creator[:n], d.seq[:n], d.poff[:n + 1], d.par) == -1
    ev = np.arange(0, n, 7, dtype=np.uint32)
    assert np.array_equal(ixa.rows_np(0, ev)[1], o.rows(0, ev)[1])
    ixa.close()
    ix1.close()


def _far_dag(lx, n_nodes, n, seed):
    """Valid fork-free DAG whose non-self parents are uniform over all earlier
    events: with n >> 65535, many parents lie more than 16 bits of distance
    back, so their compact records are 'wide' (lx_internal.h CRec)."""
    rng = np.random.default_rng(seed)
    creator = rng.integers(0, n_nodes, size=n).astype(np.uint32)
    seq = np.zeros(n, dtype=np.uint32)
    lam = np.zeros(n, dtype=np.uint32)
    last = [-1] * n_nodes
    poff = [0]
    par = []
    for i in range(n):
        c = int(creator[i])
        ps = [last[c]] if last[c] >= 0 else []
        if i:
            for x in rng.integers(0, i, size=int(rng.integers(0, 4))):
                x = int(x)
                if x not in ps and int(creator[x]) != c:
                    ps.append(x)
        seq[i] = seq[last[c]] + 1 if last[c] >= 0 else 1
        lam[i] = 1 + max((int(lam[p]) for p in ps), default=0)
        last[c] = i
        par.extend(ps)
        poff.append(len(par))
    return lx.tools.Dag(creator, seq, lam, np.array(poff, dtype=np.uint64), np.array(par, dtype=np.uint32), n_nodes)


@pytest.mark.parametrize("cpw", [8, 12])
def test_compact_records_far_parents(lx, cpw):
    """The 8- / 12-column walks stream 32-B compact records (parents as 16-bit
    distances back); events with a parent 65535+ events back fall back to the
    full record.  Planes equal the walk over the 64-B records (option crec=0)
    and the 4-column walk, rows equal the C oracle, one walk and three
    segments side by side (option crec=1; the default streams the 64-B
    records)."""
    V = 16
    d = _far_dag(lx, V, 90_000, 5)
    dist = np.repeat(np.arange(len(d), dtype=np.int64), np.diff(d.poff.astype(np.int64))) - d.par.astype(np.int64)
    assert (dist >= 0xFFFF).sum() > 1000   # many wide records
    w = list(range(40, 40 - V, -1))
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ixc, pc = planes_of(lx, d, w, {"cpw": cpw, "seg_auto": 0, "crec": 1})
    ixf, pf = planes_of(lx, d, w, {"cpw": cpw, "seg_auto": 0, "crec": 0})
    ix4, p4 = planes_of(lx, d, w, {"cpw": 4, "seg_auto": 0})
    for k in (0, 1):
        np.testing.assert_array_equal(pc[k], pf[k])
        np.testing.assert_array_equal(pc[k], p4[k])
    ev = np.arange(0, len(d), 7, dtype=np.uint32)
    for mode in (0, 1):
        assert np.array_equal(ixc.rows_np(mode, ev)[1], o.rows(mode, ev)[1]), mode
    ixs, ps = planes_of(lx, d, w, {"cpw": cpw, "segments": 3, "crec": 1})
    for k in (0, 1):
        np.testing.assert_array_equal(ps[k], p4[k])
    for ix in (ixc, ixf, ix4, ixs):
        ix.close()
