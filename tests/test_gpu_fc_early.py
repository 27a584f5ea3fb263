"""k_fc's early exit (option fc_early): on fork-free
epochs whose 256 heaviest validators can reach the quorum alone, a query reads
the rest of its rows only when their count leaves the quorum open.  The
answers must equal the whole-row kernel's and the oracle's
(vecfc/forkless_cause.go:63-82), including queries on unknown events; epochs
where it cannot decide early (equal stakes) must not use it."""

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


# fc_early_lanes: 32 lanes per query (rounds of 128 / 256 / 512 columns, the
# default) or 16 (k_fc_early<., 16>: its own width-16 shuffles, rounds of 64 /
# 128 / 256 columns)
@pytest.mark.parametrize("lanes", [32, 16])
@pytest.mark.parametrize("V,epv,zipf", [(300, 60, True), (1000, 30, True), (600, 40, True), (300, 60, False),
                                         (1000, 30, False)])
def test_early_exit_equals_whole_rows_and_oracle(lx, V, epv, zipf, lanes):
    d = lx.tools.gen_dag(V, epv, 10, seed=V + epv)
    w = [(1 << 20) // (i + 1) for i in range(V)] if zipf else [3] * V
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ix = lx.Index(event_capacity=len(d))
    ix.set_option("fc_early_lanes", lanes)
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    qa, qb = lx.tools.fc_queries(d.lamport, 200_000, window=64, seed=3)
    # far pairs too (mostly true) and pairs in both orders
    rng = np.random.default_rng(V)
    qa2 = rng.integers(0, len(d), 50_000).astype(np.uint32)
    qb2 = rng.integers(0, len(d), 50_000).astype(np.uint32)
    qa, qb = np.concatenate([qa, qa2, qb2]), np.concatenate([qb, qb2, qa2])
    want = o.forkless_cause_batch(qa, qb)
    ix.fc_early_counters()
    got = ix.forkless_cause_batch(qa, qb)
    nq, nsecond, nfull = ix.fc_early_counters()
    np.testing.assert_array_equal(got, want)
    if V <= 512:
        assert nq == 0              # rows of <= 128 uint4 run 32 lanes per query: no early path
    elif zipf:
        assert nq == len(qa) and nfull <= nsecond < nq, (nq, nsecond, nfull)
        assert nsecond > 0, nsecond                      # some queries needed more than 256 columns
    else:
        assert nq == 0              # equal stakes, 256 of 1000 columns < 2/3: whole rows
    ix.set_option("fc_early", 0)
    np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), want)
    assert ix.fc_early_counters()[0] == 0
    assert 0.05 < want.mean() < 0.95
    ix.close()


@pytest.mark.parametrize("lanes", [32, 16])
def test_early_exit_unknown_events(lx, lanes):
    """Queries on events past the index answer 0xFF through the early path too
    (V = 600: rows of 150 uint4; a launch of 2^14 queries, the smallest that
    takes the early path; the device's counter shows every query went through
    it).  A small launch keeps whole rows."""
    V = 600
    d = lx.tools.gen_dag(V, 20, 10, seed=4)
    w = [(1 << 20) // (i + 1) for i in range(V)]
    ix = lx.Index(event_capacity=len(d))
    ix.set_option("fc_early_lanes", lanes)
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    import torch
    dev = torch.device("cuda", 0)
    n = 1 << 14
    qa, qb = lx.tools.fc_queries(d.lamport, n, window=64, seed=5)
    qa[:3] = [0, len(d) + 5, 7]
    qb[:3] = [len(d) + 9, 1, 3]
    ta = torch.from_numpy(qa.view(np.int32)).to(dev)
    tb = torch.from_numpy(qb.view(np.int32)).to(dev)
    out = torch.zeros(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ix.fc_early_counters()
    ix.forkless_cause_batch_dev(n, ta.data_ptr(), tb.data_ptr(), out.data_ptr())
    with pytest.raises(Exception):
        ix.sync()                                        # the unknown-event flag is reported
    got = out.cpu().numpy()
    assert got[0] == 0xFF and got[1] == 0xFF and got[2] in (0, 1)
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    np.testing.assert_array_equal(got[3:], o.forkless_cause_batch(qa[3:], qb[3:]))
    assert ix.fc_early_counters()[0] == n
    # a launch below 2^14 queries reads whole rows
    ix.forkless_cause_batch(qa[3:1000], qb[3:1000])
    assert ix.fc_early_counters()[0] == 0
    ix.close()
