"""Pin the QuorumIndexer restatement (oracle/emitter_oracle.py) to the
reference's golden parent choices (emitter/ancestor/quorum_indexer_test.go:
22-76, TestCasualityStrategy) and to its median / metric definitions.  CPU only."""

import json
import os

import pytest

from emitter_harness import oracle_backend, run_named_parents
from oracle import emitter_oracle as eo

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def emitter_golden():
    with open(os.path.join(HERE, "golden", "emitter_golden.json"), encoding="utf-8") as f:
        return json.load(f)


def test_golden_fixture_shape(emitter_golden):
    g = emitter_golden
    assert g["weights"] == [5, 6, 7, 8, 9] and g["cap"] == 2
    assert sorted(g["expected"]) == ["0", "1", "2", "3", "4"]
    assert all(len(v) == 5 for v in g["expected"].values())


@pytest.mark.parametrize("batched", [False, True])
def test_casuality_strategy_oracle(emitter_golden, batched):
    """Every stage / node pick of TestCasualityStrategy, and every pick is
    independent of Go's map order (unique positive maximum)."""
    bad = run_named_parents(emitter_golden, oracle_backend(emitter_golden["cap"]), batched=batched)
    assert bad == []


def test_wrong_cap_breaks_golden(emitter_golden):
    """The golden choices depend on the metric: an uncapped metric picks
    differently somewhere, so the test above really checks the metric."""
    bad = run_named_parents(emitter_golden, oracle_backend(1000))
    assert bad


def test_wmedian_and_seq_of():
    # utils/wmedian/median.go:11-21: first value whose running weight reaches stop
    vals = [(9, 1), (7, 2), (7, 3), (1, 4)]
    assert eo.wmedian_of(vals, 1)[0] == 9
    assert eo.wmedian_of(vals, 4)[0] == 7
    assert eo.wmedian_of(vals, 7)[0] == 1
    with pytest.raises(RuntimeError):
        eo.wmedian_of(vals, 11)
    # seqOf (:70-75): fork-detected -> MaxUint32/2 - 1
    assert eo.seq_of((0, 0x7FFFFFFF)) == 0x7FFFFFFE
    assert eo.seq_of((5, 3)) == 5


def test_capped_metric_cases():
    fn = eo.capped_metric([3, 5], 2)
    assert fn(4, 0, 4, 0) == 0            # update <= median
    assert fn(1, 6, 5, 0) == 0            # update <= current
    assert fn(1, 0, 2, 1) == 5            # diff 1 * w
    assert fn(1, 0, 9, 1) == 10           # capped at 2 * w
    assert fn(1, 2, 9, 0) == 6 - 3        # median < current: cap(8) - cap(1)


@pytest.mark.parametrize("forks", [0, 3])
def test_numpy_quorum_indexer_matches_restatement(forks):
    """The bench's CPU baseline (DenseQuorumIndexerNp) against the scalar
    restatement's median / metric functions on the same merged rows."""
    import numpy as np
    from lachesis_hip import tools
    from oracle import corc
    V = 12
    d = tools.gen_dag(V, 30, 4, cheaters=2 if forks else 0, forks=forks, seed=5)
    w = [1 + (i % 4) * 3 for i in range(V)]
    ix = corc.OracleIndex(w)
    assert ix.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    ix.flush()
    qi = eo.DenseQuorumIndexerNp(w, ix, cap=2)
    quorum = sum(w) * 2 // 3 + 1
    fn = eo.capped_metric(w, 2)
    matrix = [[0] * V for _ in range(V)]
    sp = [0] * V

    def seqs(e):
        r = np.frombuffer(ix.merged_hb(e), dtype=np.uint32).reshape(-1, 2)
        return [eo.seq_of((int(r[i, 0]), int(r[i, 1]))) for i in range(V)]

    checked = 0
    for e in range(len(d)):
        c = int(d.creator[e])
        qi.process_event(e, c, c == 0)
        s = seqs(e)
        for i in range(V):
            matrix[i][c] = s[i]
            if c == 0:
                sp[i] = s[i]
        if e % 37 == 36:
            med = [eo.wmedian_of(sorted(((matrix[i][k], w[k]) for k in range(V)), key=lambda p: -p[0]), quorum)[0]
                   for i in range(V)]
            cand = list(range(max(0, e - 20), e + 1))
            want = [sum(fn(med[i], sp[i], seqs(x)[i], i) for i in range(V)) & 0xFFFFFFFFFFFFFFFF for x in cand]
            assert list(qi.metric_of(cand)) == want
            assert list(qi.median) == med
            checked += len(cand)
    assert checked > 100
