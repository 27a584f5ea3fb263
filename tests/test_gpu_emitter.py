"""Parity of the HIP QuorumIndexer (include/lachesis_emitter.h) with the
restatement of emitter/ancestor.QuorumIndexer (oracle/emitter_oracle.py).

* the golden parent choices of TestCasualityStrategy
  (quorum_indexer_test.go:22-76) through the GPU matrix / medians / metrics;
* seeded fork DAGs (cheaters, skewed stakes): matrix, self-parent seqs,
  weighted medians and GetMetricOf of every event after every batch of
  ProcessEvent calls, bit-exact, for two caps;
* error paths.
"""

import json
import os

import numpy as np
import pytest

from emitter_harness import run_named_parents
from oracle import corc, pos, tdag
from oracle import emitter_oracle as eo
from oracle import vecfc_oracle as vo

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


@pytest.fixture(scope="module")
def emitter_golden():
    with open(os.path.join(HERE, "golden", "emitter_golden.json"), encoding="utf-8") as f:
        return json.load(f)


def gpu_backend(lx, cap):
    def make(validators, ordered):
        ix = lx.VecfcIndex()
        ix.reset(validators)
        ix.add_events(ordered)
        qis = [lx.emitter.QuorumIndexer(ix, cap) for _ in validators.ids]
        choose = lambda ex, opts, st: (lx.emitter.choose_parents(ex, opts, st), True)  # noqa: E731
        return ix, qis, choose
    return make


@pytest.mark.parametrize("batched", [False, True])
def test_casuality_strategy_gpu(lx, emitter_golden, batched):
    bad = run_named_parents(emitter_golden, gpu_backend(lx, emitter_golden["cap"]), batched=batched)
    assert bad == []


class _DenseMerged:
    """dagi for the oracle QuorumIndexer: merged HB bytes from the C oracle."""

    def __init__(self, o, pos_of):
        self.o, self.pos_of = o, pos_of

    def get_merged_highest_before(self, eid):
        return vo.HighestBeforeSeq(raw=self.o.merged_hb(self.pos_of[eid]))


def _skewed(n):
    return [max(1, (1 << 12) // (i + 1)) for i in range(n)]


@pytest.mark.parametrize("shape", [
    # V, events/node, parents, cheaters, forks, seed, weights
    (7, 25, 3, 0, 0, 1, "equal"),
    (12, 30, 4, 3, 5, 2, "skewed"),
    (40, 12, 6, 8, 4, 3, "skewed"),
    (100, 8, 10, 10, 3, 4, "equal"),
    (1000, 3, 10, 0, 0, 5, "zipf"),          # BASELINE configs[4] scale: V = 1000, Zipf stakes
])
def test_quorum_indexer_matches_oracle(lx, shape):
    V, epn, P, cheaters, forks, seed, wk = shape
    nodes, events = tdag.rand_fork_dag(V, epn, P, cheaters, forks, seed=seed)
    w = [1] * V if wk == "equal" else _skewed(V) if wk == "skewed" else [(1 << 20) // (i + 1) for i in range(V)]
    validators = pos.Validators(dict(zip(nodes, w)))
    o = corc.OracleIndex(validators.weights)
    cr, sq, off, par = tdag.to_dense(events, validators)
    assert o.add_batch(cr, sq, off, par) == -1
    pos_of = {e.id: i for i, e in enumerate(events)}

    ix = lx.VecfcIndex()
    ix.reset(validators)
    ix.add_events(events)
    rng = np.random.default_rng(seed)
    me = int(rng.integers(V))                     # the emitting validator (idx)
    caps = (2, 7)
    oq = {c: eo.QuorumIndexer(validators, _DenseMerged(o, pos_of), eo.capped_metric(validators.weights, c))
          for c in caps}
    gq = {c: lx.emitter.QuorumIndexer(ix, c) for c in caps}
    ids = [e.id for e in events]
    i = 0
    rounds = 0
    while i < len(events):
        n = int(rng.integers(1, 3 * V))
        chunk = events[i:i + n]
        flags = [1 if validators.idxs[e.creator] == me else 0 for e in chunk]
        for c in caps:
            for e, f in zip(chunk, flags):
                oq[c].process_event(e, bool(f))
            gq[c].process_events(chunk, flags)
        i += n
        rounds += 1
        if rounds % 3 and i < len(events):
            continue
        for c in caps:
            assert np.array_equal(gq[c].get_global_matrix(), np.array(oq[c].get_global_matrix())), (c, i)
            assert list(gq[c].get_self_parent_seqs()) == oq[c].get_self_parent_seqs(), (c, i)
            assert list(gq[c].get_global_median_seqs()) == oq[c].get_global_median_seqs(), (c, i)
            got = gq[c].get_metrics_of(ids)
            exp = [oq[c].get_metric_of(x) for x in ids]
            assert list(map(int, got)) == exp, (c, i)


def test_quorum_indexer_errors_and_reset(lx):
    nodes, events = tdag.rand_fork_dag(5, 6, 3, seed=9)
    validators = pos.Validators.equal(nodes, 1)
    ix = lx.VecfcIndex()
    ix.reset(validators)
    ix.add_events(events)
    q = lx.emitter.QuorumIndexer(ix, 2)
    # unknown dense event -> LX_ERR_ARG, state unchanged
    bad = np.array([len(events) + 5], dtype=np.uint32)
    rc = q.L.lx_qi_process_events(q.h, 1, bad.ctypes.data_as(lx.capi.u32p), None)
    assert rc < 0 and "unknown event" in q.L.lx_qi_last_error(q.h).decode()
    assert not q.get_global_matrix().any()
    q.process_events(events, [0] * len(events))
    assert q.get_global_matrix().any()
    # new epoch: matrix zeroed, medians of an all-zero matrix are 0
    ix.reset(validators)
    q.reset()
    assert not q.get_global_matrix().any()
    assert not q.get_global_median_seqs().any()
