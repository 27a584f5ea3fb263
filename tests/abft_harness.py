"""Test harness shared by the abft oracle tests and the GPU abft parity tests.

Mirrors ``abft/common_test.go`` (FakeLachesis / FakeLachesis: blocks keyed by
(epoch, frame), an ``apply_block`` hook that may seal the epoch) and the event
drivers of ``abft/event_processing_test.go`` / ``frame_decide_test.go``.
"""

from oracle import abft_oracle as ao
from oracle import pos, tdag
from oracle.tdag import SplitMix64


class FakeLachesis:
    """TestLachesis of abft/common_test.go:30-115 over the oracle (``index`` = a vecfc.Index
    restatement)."""

    def __init__(self, weights_by_id, index=None, backend="oracle", options=None):
        self.events = {}
        if backend == "gpu":
            # the product: lachesis_hip.abft over the HIP library
            from lachesis_hip import abft
            self.lch = abft.IndexedLachesis(pos.Validators(weights_by_id), epoch=ao.FIRST_EPOCH)
            for k, v in (options or {}).items():
                self.lch.set_option(k, v)
            self.store = self.lch.store
        else:
            self.store = ao.Store()
            self.store.apply_genesis(ao.FIRST_EPOCH, pos.Validators(weights_by_id))
            self.index = index if index is not None else ao.DenseOracleIndex()
            self.lch = ao.IndexedLachesis(self.store, self.events.get, self.index)
        self.blocks = {}
        self.block_list = []          # (epoch, frame, atropos, cheaters, confirmed)
        self.epoch_blocks = {}
        self.last_block = (0, 0)
        self.apply_block = None
        self.lch.bootstrap(self._begin_block)

    def _begin_block(self, block):
        confirmed = []

        def end_block():
            key = (self.store.get_epoch(), self.store.last_decided_frame + 1)
            self.blocks[key] = (block.atropos, tuple(block.cheaters), self.store.get_validators().ids,
                                tuple(self.store.get_validators().weights))
            self.block_list.append((key[0], key[1], block.atropos, tuple(block.cheaters), tuple(confirmed)))
            if self.last_block[0] != key[0] and key[1] != 1:
                raise AssertionError("first frame must be 1")
            self.epoch_blocks[key[0]] = self.epoch_blocks.get(key[0], 0) + 1
            self.last_block = key
            if self.apply_block is not None:
                return self.apply_block(block)
            return None
        return (lambda e: confirmed.append(e.id)), end_block

    def build(self, e):
        self.lch.build(e)

    def process(self, e):
        self.events[e.id] = e
        return self.lch.process(e)

    def process_batch(self, events, claimed=True):
        """GPU: one lx_abft_process_batch call; oracle: Process per event.
        Returns (consumed, err); consumed < len(events) without error = the
        epoch was sealed."""
        for e in events:
            self.events[e.id] = e
        if hasattr(self.lch, "process_batch"):
            return self.lch.process_batch(events, claimed)
        epoch = self.store.get_epoch()
        for i, e in enumerate(events):
            if not claimed:
                self.lch.build(e)
            err = self.lch.process(e)
            if err is not None:
                return i, err
            if self.store.get_epoch() != epoch:
                return i + 1, None
        return len(events), None

    def frame_of(self, eid):
        return self.events[eid].frame


def mutate_validators(validators):
    """common_test.go:117-126 with a splitmix64 stream seeded by the total
    weight instead of Go's math/rand."""
    r = SplitMix64(validators.total_weight)
    w = {}
    for vid, wt in zip(validators.ids, validators.weights):
        w[vid] = wt * (500 + r.below(500)) // 1000 + 1
    return pos.Validators(w)


def topo_shuffle(events, rng):
    """reorder() of event_processing_test.go:160-168: a random topological
    order (random permutation, then parents first)."""
    arr = tdag.shuffle(events, rng)
    ids = {e.id for e in arr}
    placed = set()
    pending = {}
    out = []

    def place(e):
        stack = [e]
        while stack:
            x = stack[-1]
            missing = [p for p in x.parents if p in ids and p not in placed]
            if missing:
                stack.extend(pending[p] for p in missing)
                continue
            stack.pop()
            if x.id not in placed:
                placed.add(x.id)
                out.append(x)

    for e in arr:
        pending[e.id] = e
    for e in arr:
        if e.id not in placed:
            place(e)
    return out


def gen_epoch(lch0, nodes, weights, cheaters, events_per_node, parent_count, rng, epoch, eid_base):
    """One epoch of testLachesisRandomAndReset (event_processing_test.go:103-128):
    events are Built and Processed on instance 0 as they are generated; once
    the epoch is sealed, Build refuses the rest."""
    ordered = []

    def build(e):
        if lch0.store.get_epoch() != epoch:
            return False
        e.epoch = epoch
        lch0.build(e)
        err = lch0.process(e)
        assert err is None, err
        ordered.append(e)
        return True

    tdag.rand_fork_dag(len(nodes), events_per_node, parent_count, cheaters=cheaters, forks_count=10,
                       node_ids=nodes, rng=rng, build=build, eid_base=eid_base)
    return ordered


def compare_results(lchs):
    """compareResults (event_processing_test.go:170-204)."""
    for i in range(len(lchs) - 1):
        for j in range(i + 1, len(lchs)):
            a, b = lchs[i], lchs[j]
            assert a.store.last_decided_frame == b.store.last_decided_frame
            assert a.store.get_epoch() == b.store.get_epoch()
            assert a.store.get_validators().ids == b.store.get_validators().ids
            assert a.store.get_validators().weights == b.store.get_validators().weights
            for ep in range(1, a.store.get_epoch() + 1):
                both = min(a.epoch_blocks.get(ep, 0), b.epoch_blocks.get(ep, 0))
                for f in range(1, both):
                    assert a.blocks[(ep, f)] == b.blocks[(ep, f)], (ep, f)


def node_ids(n, seed=99):
    r = SplitMix64(seed)
    out = []
    while len(out) < n:
        v = r.next() & 0xFFFFFFFF
        if v and v not in out:
            out.append(v)
    return out
