"""testSpecialNamedParents (emitter/ancestor/quorum_indexer_test.go:78-199)
restated over a pluggable index / QuorumIndexer backend, so the same driver
checks the oracle (CPU) and the HIP QuorumIndexer (GPU) against the golden
parent choices of TestCasualityStrategy."""

from oracle import emitter_oracle as eo
from oracle import pos, tdag


def node_names(nodes, events):
    """ascii_scheme.go:200-208: "node" + upper(first letter of the first event)."""
    out = {}
    for v in nodes:
        name = events[v][0].name
        out[v] = "node" + (name[4:5] if name.startswith("node") else name[0:1]).upper()
    return out


def run_named_parents(golden, make_backend, batched=False):
    """``make_backend(validators, ordered) -> (index, [qi per validator idx],
    choose_parents)`` where ``choose_parents`` returns (parents,
    order_independent) -- a pick that depends on Go's map order is reported; the index is fully built from ``ordered`` first, as the
    reference test does (:133-137).  Returns a list of mismatches
    (stage, node, expected, got, order_independent)."""
    nodes, events, names, ordered = tdag.ascii_scheme_for_each(golden["scheme"])
    validators = pos.Validators(dict(zip(nodes, golden["weights"])))
    nname = node_names(nodes, events)
    _, qis, choose = make_backend(validators, ordered)

    stages = []
    for e in ordered:
        st = int(e.name.split(".")[1])
        while len(stages) <= st:
            stages.append([])
        stages[st].append(e)

    heads = []            # insertion-ordered set
    tips = {}
    bad = []
    for st, ee in enumerate(stages):
        for e in ee:
            for p in e.parents:
                if p in heads:
                    heads.remove(p)
            heads.append(e.id)
            tips[e.creator] = e.id
            if not batched:
                for i, vid in enumerate(validators.ids):
                    qis[i].process_event(e, e.creator == vid)
        if batched and ee:
            for i, vid in enumerate(validators.ids):
                qis[i].process_events(ee, [1 if e.creator == vid else 0 for e in ee])
        for vid in nodes:
            sp = tips.get(vid)
            qi = qis[validators.idxs[vid]]
            strategies = [qi.search_strategy(), qi.search_strategy()]
            existing = [sp] if sp is not None else []
            parents, det = choose(existing, list(heads), strategies)
            if sp is not None and parents[0] != sp:
                bad.append((st, nname[vid], "self-parent first", parents, det))
            got = eo.parents_to_string(parents)
            exp = golden["expected"][str(st)][nname[vid]]
            if got != exp or not det:
                bad.append((st, nname[vid], exp, got, det))
    return bad


def oracle_backend(cap):
    """The CPU restatement: vecfc_oracle.Index + emitter_oracle.QuorumIndexer."""
    from oracle import vecfc_oracle as vo

    def make(validators, ordered):
        store = {}
        ix = vo.Index()
        ix.reset(validators, store.get)
        for e in ordered:
            store[e.id] = e
            ix.add(e)
        fn = eo.capped_metric(validators.weights, cap)
        qis = [_OracleQI(eo.QuorumIndexer(validators, ix, fn)) for _ in validators.ids]
        return ix, qis, eo.choose_parents
    return make


class _OracleQI:
    def __init__(self, qi):
        self.qi = qi

    def process_event(self, e, self_event):
        self.qi.process_event(e, self_event)

    def process_events(self, events, flags):
        for e, f in zip(events, flags):
            self.qi.process_event(e, bool(f))

    def search_strategy(self):
        return self.qi.search_strategy()
