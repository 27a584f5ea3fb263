"""GPU parity of the batched abft caller (include/lachesis_abft.h) against the
abft restatement (oracle/abft_oracle.py, itself pinned to the reference's
abft tests by tests/test_abft_oracle.py).

Bit-exact: every event's frame, root slots per frame, every block (decided
frame, Atropos, cheaters, confirmed events in ApplyEvent order), epoch seals,
and the event at which each sealing frame was decided.
"""

import pytest

from oracle import abft_oracle as ao
from oracle import tdag
from oracle.tdag import SplitMix64
from abft_harness import FakeLachesis, compare_results, mutate_validators, node_ids, topo_shuffle
from test_abft_oracle import decode_root_name

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["classic_roots", "random_roots"])
@pytest.mark.parametrize("batched", [False, True])
def test_special_named_roots_gpu(golden, case, batched):
    """TestLachesisClassicRoots / TestLachesisRandomRoots on the GPU path."""
    c = next(x for x in golden["roots_cases"] if x["name"] == case)
    nodes, _, names, ordered = tdag.ascii_scheme_for_each(c["scheme"])
    t = FakeLachesis({v: 1 for v in nodes}, backend="gpu")
    if batched:
        consumed, err = t.process_batch(ordered, claimed=False)
        assert err is None and consumed == len(ordered)
    else:
        for e in ordered:
            t.build(e)
            assert t.process(e) is None
    for name, e in names.items():
        want_frame, want_root = decode_root_name(name)
        sp = ao.self_parent(e)
        sp_frame = names_by_id(names)[sp].frame if sp is not None else 0
        assert e.frame == want_frame, name
        assert (e.frame != sp_frame) == want_root, name


def names_by_id(names):
    return {e.id: e for e in names.values()}


def gen_events(weights, cheaters, events_per_node, parent_count, seed, forks=10):
    nodes = node_ids(len(weights), seed=seed)
    _, evs = tdag.rand_fork_dag(len(nodes), events_per_node, parent_count, cheaters=cheaters,
                                forks_count=forks, node_ids=nodes, rng=SplitMix64(seed))
    return nodes, evs


def run(backend, nodes, weights, evs, mode, chunk=None, seal_every=None, mutate=False, options=None, claim=None):
    """Processes evs (frames computed by Build semantics, or claimed: claim =
    {event id: frame}, Process's checkAndSaveEvent) and returns the observable
    results."""
    t = FakeLachesis(dict(zip(nodes, weights)), backend=backend, options=options)
    sealed_at = []
    if seal_every:
        def apply_block(block):
            if t.store.last_decided_frame + 1 == seal_every:
                v = t.store.get_validators()
                return mutate_validators(v) if mutate else v
            return None
        t.apply_block = apply_block
    frames = {}
    i = 0
    epoch0 = t.store.get_epoch()
    while i < len(evs):
        if mode == "event":
            part = evs[i:i + 1]
        else:
            part = evs[i:i + (chunk or len(evs))]
        for e in part:
            e.frame = claim[e.id] if claim else 0
        consumed, err = t.process_batch(part, claimed=bool(claim))
        assert err is None, err
        for e in part[:consumed]:
            frames[e.id] = e.frame
        i += consumed
        if t.store.get_epoch() != epoch0:
            sealed_at.append(part[consumed - 1].id)
            break
    return dict(frames=frames, blocks=list(t.block_list), sealed_at=sealed_at,
                last=(t.store.get_epoch(), t.store.last_decided_frame))


SHAPES = [
    # (weights, cheaters, events/node, parents, seed)
    ([1, 1, 1, 1], 0, 40, 3, 1),
    ([1, 2, 3, 4], 0, 40, 4, 2),
    ([11, 11, 11, 67], 0, 40, 4, 3),
    ([1] * 10, 0, 30, 5, 4),
    ([1, 1, 1, 1], 1, 40, 3, 5),
    ([1, 2, 1, 2, 1, 2, 1, 2, 1, 2], 3, 30, 5, 6),
    ([0xFFFFFFFF // 8, 0xFFFFFFFF // 8, 0xFFFFFFFF // 4], 0, 40, 3, 7),
    ([5 + (i % 7) for i in range(40)], 4, 15, 8, 8),
]


@pytest.mark.parametrize("fc16", [1, 0])
@pytest.mark.parametrize("shape", SHAPES, ids=[str(i) for i in range(len(SHAPES))])
def test_abft_matches_oracle(shape, fc16):
    """fc16: fork-free epochs take the packed root-FC kernel (k_root_fc16,
    16-bit seqs; shape 6's weights >= 2^16 take its high-half dot products)
    or the 32-bit one."""
    weights, cheaters, epn, pc, seed = shape
    nodes, evs = gen_events(weights, cheaters, epn, pc, seed)
    ref = run("oracle", nodes, weights, evs, "event")
    assert len(ref["blocks"]) >= 3
    for mode, chunk in (("event", None), ("batch", None), ("batch", 7), ("batch", 64)):
        got = run("gpu", nodes, weights, evs, mode, chunk, options={"fc16": fc16})
        assert got["frames"] == ref["frames"], (mode, chunk)
        assert got["blocks"] == ref["blocks"], (mode, chunk)
        assert got["last"] == ref["last"], (mode, chunk)
    # claimed frames (Process): all frame steps of a batch enqueued at once
    # (claimed_batch) or step by step; elections decided ahead (elect_ahead
    # rounds each, one wait) or round by round (0)
    for cb, chunk, ea in ((1, None, 3), (1, 7, 3), (0, None, 0), (1, None, 2), (1, 64, 0)):
        got = run("gpu", nodes, weights, evs, "batch", chunk,
                  options={"fc16": fc16, "claimed_batch": cb, "elect_ahead": ea}, claim=ref["frames"])
        assert got["frames"] == ref["frames"], ("claimed", cb, chunk, ea)
        assert got["blocks"] == ref["blocks"], ("claimed", cb, chunk, ea)
        assert got["last"] == ref["last"], ("claimed", cb, chunk, ea)


@pytest.mark.parametrize("elect_ahead", [3, 0])
@pytest.mark.parametrize("mutate", [False, True])
def test_abft_seal_matches_oracle(mutate, elect_ahead):
    """Epoch sealed by EndBlock: same sealing event, same blocks, validators
    mutated or not (frame_decide.go:11-58)."""
    weights = [1, 2, 1, 2, 1, 2, 1, 2, 1, 2]
    nodes, evs = gen_events(weights, 0, 60, 5, 11)
    ref = run("oracle", nodes, weights, evs, "event", seal_every=3, mutate=mutate)
    assert ref["sealed_at"]
    # claimed: the events up to the sealing one (the later ones' frames belong
    # to the next epoch; a batch checks every claim before its elections)
    upto = [e for e in evs if e.id in ref["frames"]]
    for chunk, claim in ((None, None), (50, None), (None, ref["frames"]), (50, ref["frames"])):
        got = run("gpu", nodes, weights, upto if claim else evs, "batch", chunk, seal_every=3, mutate=mutate,
                  claim=claim, options={"elect_ahead": elect_ahead})
        assert got["sealed_at"] == ref["sealed_at"]
        assert got["blocks"] == ref["blocks"]
        assert got["last"] == ref["last"]
        assert got["frames"] == ref["frames"]


def test_abft_three_instances_reordered_gpu():
    """testLachesisRandomAndReset's consensus check on the GPU path: three
    instances, different topological orders (one batched), equal blocks over
    several sealed epochs."""
    weights = [1, 2, 1, 2, 1, 2, 1, 2, 1, 2]
    nodes = node_ids(len(weights), seed=77)
    wmap = dict(zip(nodes, weights))
    lchs = [FakeLachesis(wmap, backend="gpu") for _ in range(3)]
    max_blocks = 5
    for lch in lchs:
        def apply_block(block, lch=lch):
            if lch.store.last_decided_frame + 1 == max_blocks:
                return lch.store.get_validators()
            return None
        lch.apply_block = apply_block
    rng = SplitMix64(1234)
    ordered = {}
    for epoch in (1, 2, 3):
        out = []

        def build(e):
            if lchs[0].store.get_epoch() != epoch:
                return False
            lchs[0].build(e)
            assert lchs[0].process(e) is None
            out.append(e)
            return True
        tdag.rand_fork_dag(len(nodes), 100, 5, cheaters=3, forks_count=10, node_ids=nodes, rng=rng, build=build,
                           eid_base=epoch * 10**6)
        ordered[epoch] = out
        assert lchs[0].store.get_epoch() == epoch + 1
    for epoch in (1, 2, 3):
        for k, lch in enumerate(lchs[1:]):
            evs = topo_shuffle(ordered[epoch], rng)
            if k == 0:
                for e in evs:
                    assert lch.process(e) is None
                    if lch.store.get_epoch() != epoch:
                        break
            else:
                consumed, err = lch.process_batch(evs)
                assert err is None
            assert lch.store.get_epoch() == epoch + 1
    compare_results(lchs)


@pytest.mark.parametrize("delta", [1, -1, 1000])
@pytest.mark.parametrize("claimed_batch", [1, 0])
def test_abft_wrong_frame_gpu(delta, claimed_batch):
    """checkAndSaveEvent: a wrong claimed frame is rejected (ErrWrongFrame),
    the events before it are processed, the event is dropped from the index.
    delta 1000: a claim above every root frame (the batched path cuts there);
    delta -1: an under-claim, which calcFrameIdx's loop bound accepts
    (event_processing.go:180-186) -- the oracle, Process per event on the same
    claims, says where the first error falls."""
    weights = [1, 1, 1, 1]
    nodes, evs = gen_events(weights, 0, 30, 3, 21)
    ref = run("oracle", nodes, weights, evs, "event")
    t = FakeLachesis(dict(zip(nodes, weights)), backend="gpu", options={"claimed_batch": claimed_batch})
    good = [ref["frames"][e.id] for e in evs]
    bad = next(i for i, e in enumerate(evs) if i > 40 and ao.self_parent(e) is not None)
    for e, f in zip(evs, good):
        e.frame = f
    evs[bad].frame = good[bad] + delta
    o = FakeLachesis(dict(zip(nodes, weights)))
    o_consumed = len(evs)
    for i, e in enumerate(evs):
        if o.process(e) is not None:
            o_consumed = i
            break
    consumed, err = t.process_batch(evs)
    assert consumed == o_consumed and (err is None) == (o_consumed == len(evs))
    assert [e.frame for e in evs[:consumed]] == [o.frame_of(e.id) for e in evs[:consumed]]
    assert t.block_list == o.block_list
    if delta == -1:
        return
    assert consumed == bad
    evs[bad].frame = good[bad]
    consumed2, err = t.process_batch(evs[bad:])
    assert err is None and consumed2 == len(evs) - bad
    assert t.block_list == ref["blocks"]


def test_abft_build_gpu():
    """Build sets the frame of a self-emitted event without adding it."""
    weights = [1, 1, 1, 1, 1]
    nodes, evs = gen_events(weights, 0, 20, 4, 31)
    o = FakeLachesis(dict(zip(nodes, weights)))
    g = FakeLachesis(dict(zip(nodes, weights)), backend="gpu")
    for e in evs:
        o.build(e)
        f = e.frame
        e.frame = 0
        g.build(e)
        assert e.frame == f
        assert o.process(e) is None
        assert g.process(e) is None
    assert g.block_list == o.block_list


def load_golden(name):
    import os
    import numpy as np
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "abft_%s.npz" % name))


def blocks_of(g):
    out = []
    for k in range(len(g["block_frame"])):
        ch = g["cheaters"][g["cheaters_off"][k]:g["cheaters_off"][k + 1]]
        cf = g["confirmed"][g["confirmed_off"][k]:g["confirmed_off"][k + 1]]
        out.append((1, int(g["block_frame"][k]), int(g["block_atropos"][k]), tuple(map(int, ch)),
                    tuple(map(int, cf))))
    return out


@pytest.mark.parametrize("name,chunks,fc16,claimed,blog", [("c4", 1, 1, 0, 0), ("c4", 7, 1, 0, 0), ("c5", 1, 1, 0, 0),
                                                           ("c5", 3, 1, 0, 0), ("c5", 1, 0, 0, 0), ("c4", 1, 1, 1, 0),
                                                           ("c4", 7, 1, 1, 0), ("c5", 1, 1, 1, 0), ("c5", 3, 0, 1, 0),
                                                           ("c4", 7, 1, 1, 1), ("c5", 1, 1, 1, 1)])
def test_abft_full_size_vs_oracle(name, chunks, fc16, claimed, blog):
    """BASELINE configs 4 (100 validators, 10 % double-signers, 100k events)
    and 5 (1000 validators, Zipf stakes, 50k events) at full size: frames of
    every event, roots per frame and every block (Atropos, cheaters, ApplyEvent
    order) equal the C abft restatement's (tests/golden/make_abft_golden.py),
    whole epoch in one batch or in chunks."""
    import numpy as np
    from lachesis_hip import abft, tools
    g = load_golden(name)
    V, epn, P, ch, fk, seed = map(int, g["config"])
    d = tools.gen_dag(V, epn, P, cheaters=ch, forks=fk, seed=seed)
    # blog: no callbacks, the library's block log (option block_log 2)
    lch = abft.DenseLachesis(g["weights"], event_capacity=len(d), block_log=bool(blog))
    lch.set_option("fc16", fc16)   # c5 (Zipf stakes, no forks): packed root-FC kernel unless 0
    frames = np.zeros(len(d), dtype=np.uint32)
    bounds = np.linspace(0, len(d), chunks + 1).astype(np.int64)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        c, s, off, par = d.slice(lo, hi)
        # claimed: the golden frames as Process's claims (bench.py's abft leg)
        rc, consumed, out = lch.process_batch(c, s, off, par, g["frames"][lo:hi] if claimed else None)
        assert rc == 0 and consumed == hi - lo
        frames[lo:hi] = out

    assert np.array_equal(frames, g["frames"])
    assert [len(lch.frame_roots(f)) for f in range(len(g["roots_per_frame"]))] == list(g["roots_per_frame"])
    assert lch.blocks == blocks_of(g)


@pytest.mark.parametrize("name", ["c4", "c5"])
def test_abft_block_log_sweep_equals_dfs(name):
    """block_log 1 without ApplyEvent confirms a batch's blocks by one sweep
    over the parent lists (lx_abft.cpp confirm_sweep) instead of one DFS per
    block: the same GetEventConfirmedOn for every event and the same blocks
    as the callbacks' DFS path, claimed batches whole and in chunks."""
    import numpy as np
    from lachesis_hip import abft, tools
    g = load_golden(name)
    V, epn, P, ch, fk, seed = map(int, g["config"])
    d = tools.gen_dag(V, epn, P, cheaters=ch, forks=fk, seed=seed)
    want = blocks_of(g)
    for chunks in (1, 5):
        runs = {}
        for mode in ("dfs", "sweep"):
            lch = abft.DenseLachesis(g["weights"], event_capacity=len(d), apply_events=False,
                                     block_log=(mode == "sweep"))
            bounds = np.linspace(0, len(d), chunks + 1).astype(np.int64)
            for lo, hi in zip(bounds[:-1], bounds[1:]):
                c, s_, off, par = d.slice(lo, hi)
                rc, consumed, out = lch.process_batch(c, s_, off, par, g["frames"][lo:hi])
                assert rc == 0 and consumed == hi - lo
            runs[mode] = (lch.confirmed_on(len(d)), [b[:4] for b in lch.blocks])
            lch.close()
        assert np.array_equal(runs["dfs"][0], runs["sweep"][0]), chunks
        assert runs["dfs"][1] == runs["sweep"][1] == [b[:4] for b in want], chunks
        assert (runs["sweep"][0] > 0).sum() == sum(len(b[4]) for b in want)
