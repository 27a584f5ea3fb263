"""The unchanged caller's call sequence on the HIP index (lachesis_hip.dropin:
IndexedLachesis.Process restated in C++, per-event Add, per-pair
ForklessCause through lx_forkless_cause, Flush, DropNotFlushed,
GetMergedHighestBefore) -- abft/indexed_lachesis.go:69-82,
abft/event_processing.go:102-189, abft/election/election.go:101-123.

configs[4] (C5) at full size: frames, roots per frame and blocks equal
tests/golden/abft_c5.npz, and the call sequence (hash of every Add /
ForklessCause / Flush / DropNotFlushed in order) equals the C abft
restatement's (tests/golden/dropin_c5.json, make_dropin_golden.py); fork DAGs
against the restatement with working sets small enough to evict and to take
the whole-matrix fills."""

import json
import os

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_dropin_c5_matches_golden():
    from lachesis_hip import dropin, tools
    z = np.load(os.path.join(HERE, "golden", "abft_c5.npz"))
    with open(os.path.join(HERE, "golden", "dropin_c5.json")) as f:
        g = json.load(f)
    V, epv, P, _, _, seed = (int(x) for x in z["config"])
    d = tools.gen_dag(V, epv, P, 0, 0, seed=seed)
    w = z["weights"]
    r = dropin.replay(d, w, z["frames"], kind="hip")
    np.testing.assert_array_equal(r["frames"], z["frames"])
    np.testing.assert_array_equal(r["roots_per_frame"][:len(z["roots_per_frame"])], z["roots_per_frame"])
    np.testing.assert_array_equal(r["block_frame"], z["block_frame"])
    np.testing.assert_array_equal(r["block_atropos"], z["block_atropos"])
    np.testing.assert_array_equal(r["block_nconf"], np.diff(z["confirmed_off"]))
    assert not r["block_ncheat"].any()
    assert str(r["trace_hash"]) == g["hash"]
    assert (r["fc_calls"], r["adds"], r["flushes"], r["drops"]) == (g["fc_calls"], g["adds"], g["flushes"], g["drops"])
    st = r["fc_cache"]
    assert st["calls"] == g["fc_calls"] and st["hits"] > 0.99 * st["calls"]


@pytest.mark.parametrize("slots", [-1, 64, 192])
@pytest.mark.parametrize("shape", [(20, 40, 5, 3, 4), (24, 50, 6, 0, 0)])
def test_dropin_fork_dags_match_restatement(shape, slots):
    from lachesis_hip import dropin, tools
    V, epv, P, ch, fk = shape
    d = tools.gen_dag(V, epv, P, cheaters=ch, forks=fk, seed=3)
    w = [1 + (i % 3) for i in range(V)] if ch else [(1 << 20) // (i + 1) for i in range(V)]
    rc, c, frames = corc.AbftOracle(w).process_batch(d.creator, d.seq, d.poff, d.par)
    assert rc == 0 and c == len(d)
    o = corc.AbftOracle(w)
    rc, c, _ = o.process_batch(d.creator, d.seq, d.poff, d.par, frames)
    assert rc == 0
    tr = o.trace()
    r = dropin.replay(d, w, frames, kind="hip", fc_cache=slots)
    assert r["trace_hash"] == tr["hash"] and r["fc_calls"] == tr["fc_calls"]
    np.testing.assert_array_equal(r["frames"], frames)
    assert list(r["block_atropos"]) == [b[2] for b in o.blocks]
    assert list(r["block_ncheat"]) == [len(b[3]) for b in o.blocks]
    assert list(r["block_nconf"]) == [len(b[4]) for b in o.blocks]
    if slots == 64:
        assert r["fc_cache"]["tile_fills"] > 0 or r["fc_cache"]["row_fills"] > 0
