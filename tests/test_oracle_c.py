"""The C restatement (oracle/csrc/oracle.c) is byte-identical to the Python
restatement (pinned to the reference golden tables).  CPU only."""

import numpy as np
import pytest

from oracle import corc, pos, tdag
from oracle import vecfc_oracle as vo


def _pair(events, validators, flush_every=0):
    store = {e.id: e for e in events}
    py = vo.Index()
    py.reset(validators, store.get)
    c = corc.OracleIndex(validators.weights)
    creator, seq, off, par = tdag.to_dense(events, validators)
    for i, e in enumerate(events):
        py.add(e)
        assert c.add(int(creator[i]), int(seq[i]), par[off[i]:off[i + 1]]) == 0
        if flush_every and i % flush_every == 0:
            py.flush()
            c.flush()
    return py, c


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("shape", [(1, 1, 1, 10, 3), (2, 2, 2, 10, 20), (10, 4, 10, 10, 3),
                                   (5, 4, 2, 30, 30), (8, 4, 3, 40, 30), (40, 4, 10, 3, 1), (12, 5, 0, 20, 0)])
def test_c_oracle_matches_python(seed, shape):
    n, p, ch, ev, fk = shape
    rng = tdag.SplitMix64(seed + 11)
    ids = [rng.next() & 0xFFFFFFFF for _ in range(n)]
    nodes, evs = tdag.rand_fork_dag(n, ev, p, cheaters=ch, forks_count=fk, seed=seed * 7 + n, node_ids=ids)
    w = {v: 1 + (k % 3) for k, v in enumerate(nodes)}
    validators = pos.Validators(w)
    py, c = _pair(evs, validators, flush_every=7)
    assert c.num_branches() == len(py.bi.creator_idxs)
    for i, e in enumerate(evs):
        assert c.hb(i) == py.get_highest_before(e.id).to_bytes()
        assert c.la(i) == py.get_lowest_after(e.id).to_bytes()
        assert c.branch(i) == py.get_event_branch_id(e.id)
        assert c.merged_hb(i) == py.get_merged_highest_before(e.id).to_bytes()
    a = np.array([i for i in range(len(evs)) for _ in range(len(evs))], dtype=np.uint32)
    b = np.array([j for _ in range(len(evs)) for j in range(len(evs))], dtype=np.uint32)
    got = c.forkless_cause_batch(a, b)
    exp = [py.forkless_cause(evs[i].id, evs[j].id) for i, j in zip(a, b)]
    assert list(got) == [int(x) for x in exp]


def test_c_oracle_drop_not_flushed():
    nodes, evs = tdag.rand_fork_dag(6, 20, 3, cheaters=2, forks_count=5, seed=3)
    validators = pos.Validators.equal(nodes)
    store = {e.id: e for e in evs}
    py = vo.Index()
    py.reset(validators, store.get)
    c = corc.OracleIndex(validators.weights)
    creator, seq, off, par = tdag.to_dense(evs, validators)
    half = len(evs) // 2
    for i in range(half):
        py.add(evs[i])
        c.add(int(creator[i]), int(seq[i]), par[off[i]:off[i + 1]])
    py.flush()
    c.flush()
    for i in range(half, len(evs)):
        py.add(evs[i])
        c.add(int(creator[i]), int(seq[i]), par[off[i]:off[i + 1]])
    py.drop_not_flushed()
    c.drop_not_flushed()
    assert c.num_events() == half
    for i in range(half):
        assert c.la(i) == py.get_lowest_after(evs[i].id).to_bytes()
        assert c.hb(i) == py.get_highest_before(evs[i].id).to_bytes()
    # re-add after rollback
    for i in range(half, len(evs)):
        py.add(evs[i])
        assert c.add(int(creator[i]), int(seq[i]), par[off[i]:off[i + 1]]) == 0
    for i in range(len(evs)):
        assert c.la(i) == py.get_lowest_after(evs[i].id).to_bytes()
        assert c.hb(i) == py.get_highest_before(evs[i].id).to_bytes()


def test_c_oracle_golden(golden):
    for case in golden["fc_cases"]:
        if case["fc"] is None:
            continue
        nodes, _, names, ordered = tdag.ascii_scheme_for_each(case["scheme"])
        validators = pos.Validators.equal(nodes)
        c = corc.OracleIndex(validators.weights)
        creator, seq, off, par = tdag.to_dense(ordered, validators)
        assert c.add_batch(creator, seq, off, par, flush_each=True) == -1
        posn = {e.id: i for i, e in enumerate(ordered)}
        for who, e1 in names.items():
            for whom, e2 in names.items():
                assert c.forkless_cause(posn[e1.id], posn[e2.id]) == (whom in case["fc"][who])


# ---------------------------------------------------------------------------- abft
from oracle import abft_oracle as ao  # noqa: E402
from abft_harness import FakeLachesis, node_ids  # noqa: E402
from oracle.tdag import SplitMix64  # noqa: E402


@pytest.mark.parametrize("shape", [([1, 1, 1, 1], 1, 40, 3, 1), ([1, 2, 3, 4, 5], 0, 40, 4, 2),
                                   ([1, 2, 1, 2, 1, 2, 1, 2, 1, 2], 3, 30, 5, 3),
                                   ([5 + (i % 7) for i in range(30)], 4, 12, 6, 4)])
@pytest.mark.parametrize("seal", [None, 3])
def test_abft_c_matches_python(shape, seal):
    """abft_oracle.c == abft_oracle.py: frames, roots, blocks (Atropos,
    cheaters, ApplyEvent order), epoch seal point."""
    weights, cheaters, epn, pc, seed = shape
    nodes = node_ids(len(weights), seed=seed)
    _, evs = tdag.rand_fork_dag(len(nodes), epn, pc, cheaters=cheaters, forks_count=10, node_ids=nodes,
                                rng=SplitMix64(seed))
    t = FakeLachesis(dict(zip(nodes, weights)))
    if seal:
        t.apply_block = lambda b: t.store.get_validators() if t.store.last_decided_frame + 1 == seal else None
    frames, done = [], 0
    for e in evs:
        t.build(e)
        assert t.process(e) is None
        frames.append(e.frame)
        done += 1
        if t.store.get_epoch() != 1:
            break
    v = t.store.get_validators() if not seal else pos.Validators(dict(zip(nodes, weights)))
    creator, seq, off, flat = tdag.to_dense(evs, v)
    c = corc.AbftOracle(v.weights, seal=(lambda ep, f: list(v.weights) if f == seal else None) if seal else None)
    rc, consumed, out = c.process_batch(creator, seq, off, flat)
    assert rc == 0 and consumed == done
    assert list(out[:done]) == frames
    pos_of = {e.id: i for i, e in enumerate(evs)}
    want = [(ep, f, pos_of[a], tuple(v.idxs[x] for x in ch), tuple(pos_of[x] for x in conf))
            for ep, f, a, ch, conf in t.block_list]
    assert c.blocks == want
    if not seal:
        for f in range(1, max(frames) + 1):
            assert [pos_of[x.id] for x in t.store.roots.get(f, [])] == list(c.frame_roots(f))


def test_c_oracle_fc_multithreaded_equals_single():
    """The OpenMP FC batch (bench cpu_baseline, all host cores) answers exactly
    what the single-threaded restatement answers, forks included."""
    from lachesis_hip import tools
    d = tools.gen_dag(12, 40, 4, 3, 5, 7)
    o = corc.OracleIndex([5, 4, 4, 3, 3, 2, 2, 2, 1, 1, 1, 1])
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = tools.fc_queries(d.lamport, 40_000, window=20, seed=9)
    np.testing.assert_array_equal(o.forkless_cause_batch_mt(qa, qb, 4), o.forkless_cause_batch(qa, qb))
