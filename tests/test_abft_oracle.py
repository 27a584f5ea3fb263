"""Pin the abft restatement (oracle/abft_oracle.py) to the reference's own abft
tests.  CPU only.

* TestLachesisClassicRoots / TestLachesisRandomRoots
  (abft/event_processing_root_test.go:15-301): frame and root-ness of every
  event, encoded in the event names.
* TestProcessRoot (abft/election/election_test.go:35-294): decided frame,
  Atropos and decisive roots of 5 elections under a fake observe relation, for
  random topological orders.
* testLachesisRandomAndReset (abft/event_processing_test.go:60-168): three
  instances fed different topological orders (and epoch resets) produce the
  same blocks, epochs sealed every maxEpochBlocks frames, validators mutated.
* testConfirmBlocks (abft/frame_decide_test.go:57-124): re-running
  onFrameDecided on unconfirmed events reproduces the blocks.
"""

import json
import os

import pytest

from oracle import abft_oracle as ao
from oracle import pos, tdag
from oracle import vecfc_oracle as vo
from oracle.tdag import SplitMix64
from abft_harness import FakeLachesis, compare_results, gen_epoch, mutate_validators, node_ids, topo_shuffle

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def abft_golden():
    with open(os.path.join(HERE, "golden", "abft_golden.json"), encoding="utf-8") as f:
        return json.load(f)


def decode_root_name(name):
    """event_processing_root_test.go:251-262."""
    frame = int(name.split(".")[0][1:2])
    return frame, name == name.upper()


@pytest.mark.parametrize("case", ["classic_roots", "random_roots"])
@pytest.mark.parametrize("index", ["python", "c"])
def test_special_named_roots(golden, case, index):
    c = next(x for x in golden["roots_cases"] if x["name"] == case)
    nodes, _, _, _ = tdag.ascii_scheme_for_each(c["scheme"])
    t = FakeLachesis({v: 1 for v in nodes}, vo.Index() if index == "python" else ao.DenseOracleIndex())

    def process(e, name):
        e.epoch = t.store.get_epoch()
        t.build(e)
        assert t.process(e) is None

    _, _, names, _ = tdag.ascii_scheme_for_each(c["scheme"], process)
    for name, e in names.items():
        want_frame, want_root = decode_root_name(name)
        sp = ao.self_parent(e)
        sp_frame = t.frame_of(sp) if sp is not None else 0
        assert (e.frame != sp_frame) == want_root, name
        assert e.frame == want_frame, name


def election_case(c, order_seed):
    """testProcessRoot (election_test.go:172-285)."""
    roots = {}
    frame_roots = {}
    edges = set()
    ordered = []

    def process(e, name):
        frame = int(name.split("_")[1])
        slot = ao.RootAndSlot(e.id, frame, e.creator)
        roots[e.id] = slot
        frame_roots.setdefault(frame, []).append(slot)
        no_prev = name.startswith("+")
        sp = ao.self_parent(e)
        for p in e.parents:
            if p == sp and no_prev:
                continue
            edges.add((e.id, p))
        ordered.append(e)

    nodes, _, _, _ = tdag.ascii_scheme_for_each(c["scheme"], process)
    # validator IDs follow the first event name of each column; node names
    # are "node" + upper(first letter) (ascii_scheme.go:197-208)
    first = {}
    for e in ordered:
        first.setdefault(e.creator, e.name.lstrip("+"))
    weights = {v: c["weights"]["node" + first[v][0].upper()] for v in nodes}
    validators = pos.Validators(weights)
    el = ao.Election(validators, 0, lambda a, b: (a, b) in edges, lambda f: frame_roots.get(f, []))
    order = topo_shuffle(ordered, SplitMix64(order_seed)) if order_seed else ordered
    exp = c["expected"]
    already = False
    for e in order:
        got = el.process_root(roots[e.id])
        decisive = exp is not None and e.name in exp["decisive"]
        if decisive or already:
            assert got is not None, e.name
            assert got == (exp["frame"], exp["atropos"])
            already = True
        else:
            assert got is None, e.name
    return already


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5])
def test_election_golden(abft_golden, seed):
    n_decided = 0
    for c in abft_golden["election_cases"]:
        n_decided += election_case(c, seed)
    assert n_decided == 4


WEIGHT_SETS = [
    ("1", [1], 0),
    ("big1", [0xFFFFFFFF // 2], 0),
    ("big3", [0xFFFFFFFF // 8, 0xFFFFFFFF // 8, 0xFFFFFFFF // 4], 0),
    ("4", [1, 2, 3, 4], 0),
    ("3_1", [1, 1, 1, 1], 1),
    ("67_33_4", [11, 11, 11, 67], 3),
    ("2_8_10", [1, 2, 1, 2, 1, 2, 1, 2, 1, 2], 3),
]


def lachesis_random(weights, cheaters, mutate, reset, events_per_node=200, epochs=5, seed=0):
    """testLachesisRandomAndReset (event_processing_test.go:60-158)."""
    nodes = node_ids(len(weights), seed=len(weights) * 31 + cheaters + seed)
    wmap = dict(zip(nodes, weights))
    lchs = [FakeLachesis(wmap) for _ in range(3)]
    max_epoch_blocks = events_per_node // 20
    for lch in lchs:
        def apply_block(block, lch=lch):
            if lch.store.last_decided_frame + 1 == max_epoch_blocks:
                v = lch.store.get_validators()
                return mutate_validators(v) if mutate else v
            return None
        lch.apply_block = apply_block
    rng = SplitMix64(len(nodes) + cheaters + 1000 * seed)
    parent_count = min(5, len(nodes))
    ordered, states = {}, {}
    for epoch in range(1, epochs + 1):
        ordered[epoch] = gen_epoch(lchs[0], nodes, weights, cheaters, events_per_node, parent_count,
                                   rng, epoch, eid_base=epoch * 10**6)
        states[lchs[0].store.get_epoch()] = lchs[0].store.get_validators()
        assert lchs[0].store.get_epoch() == epoch + 1, "epoch wasn't sealed"
    for epoch in range(1, epochs + 1):
        for lch in lchs[1:]:
            if reset and epoch != epochs - 1 and rng.below(2) == 0:
                lch.lch.reset(epoch + 1, states[epoch + 1])
                continue
            for e in topo_shuffle(ordered[epoch], rng):
                assert lch.process(e) is None
                if lch.store.get_epoch() != epoch:
                    break
            assert lch.store.get_epoch() == epoch + 1, "epoch wasn't sealed"
    compare_results(lchs)
    return lchs


@pytest.mark.parametrize("name,weights,cheaters", WEIGHT_SETS)
def test_lachesis_random(name, weights, cheaters):
    for mutate, reset in ((False, False), (False, True), (True, False)):
        lchs = lachesis_random(weights, cheaters if not mutate else 0, mutate, reset)
        assert sum(lchs[0].epoch_blocks.values()) >= 3


@pytest.mark.parametrize("name,weights,cheaters", WEIGHT_SETS)
def test_confirm_blocks(name, weights, cheaters):
    """testConfirmBlocks (frame_decide_test.go:57-124)."""
    nodes = node_ids(len(weights), seed=len(weights) + cheaters)
    t = FakeLachesis(dict(zip(nodes, weights)))
    frames, blocks = [], []

    def apply_block(block):
        frames.append(t.store.last_decided_frame + 1)
        blocks.append(block)
        return None
    t.apply_block = apply_block

    def build(e):
        e.epoch = 1
        t.build(e)
        assert t.process(e) is None
        return True
    tdag.rand_fork_dag(len(nodes), 60, min(5, len(nodes)), cheaters=cheaters, forks_count=10,
                       node_ids=nodes, rng=SplitMix64(len(nodes) + cheaters), build=build)
    t.store.confirmed.clear()
    for frame, block in list(zip(frames, blocks)):
        t.lch._on_frame_decided(frame, block.atropos)
        got = t.blocks[t.last_block]
        assert len(got[1]) <= cheaters
        assert got[0] == block.atropos and list(got[1]) == block.cheaters
    assert len(blocks) >= 60 // 5
