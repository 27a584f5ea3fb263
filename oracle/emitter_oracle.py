"""CPU restatement of the emitter's QuorumIndexer (TEST INFRASTRUCTURE ONLY,
see oracle/__init__.py).

Follows, statement by statement:

* ``QuorumIndexer``   -- emitter/ancestor/quorum_indexer.go:20-158
  (ProcessEvent :86-98, recacheState :100-121, GetMetricOf :123-136, the
  getters :138-158, seqOf :70-75);
* ``wmedian_of``      -- utils/wmedian/median.go:11-21;
* ``MetricStrategy``  -- emitter/ancestor/weighted.go:7-27 (+ the transparent
  MetricFnCache of metric_cache.go);
* ``choose_parents``  -- emitter/ancestor/search.go:14-34;
* ``capped_metric``   -- the DiffMetricFn of quorum_indexer_test.go:117-131.

The DAG index is any object with ``get_merged_highest_before(id)`` returning a
vector with ``get(i) -> (seq, min_seq)`` (``vecfc_oracle.Index``).

Nondeterminism of the reference: ``ChooseParents`` iterates Go maps
(``hash.EventsSet.Slice``), so the option order is random; ``Choose`` keeps the
first strictly greater metric, and the last option when every metric is 0.
``MetricStrategy.choose`` here also reports whether the pick is independent of
the option order (a unique positive maximum, or a single option), which is what
makes the reference's own golden expectations deterministic.
"""

from .vecfc_oracle import FORK_DETECTED

FORK_SEQ = 0xFFFFFFFF // 2 - 1          # seqOf: math.MaxUint32/2 - 1


def seq_of(bs):
    """quorum_indexer.go:70-75."""
    if tuple(bs) == FORK_DETECTED:
        return FORK_SEQ
    return bs[0]


def wmedian_of(values, stop):
    """utils/wmedian/median.go:11-21: values are (seq, weight) already sorted."""
    cur = 0
    for v in values:
        cur += v[1]
        if cur >= stop:
            return v
    raise RuntimeError("invalid median")


def capped_metric(weights, cap):
    """The diffMetricFn of quorum_indexer_test.go:117-131 (capFn with ``cap``)."""
    def cap_fn(diff, w):
        return cap * w if diff > cap else diff * w

    def fn(median, current, update, v):
        if update <= median or update <= current:
            return 0
        if median < current:
            return cap_fn(update - median, weights[v]) - cap_fn(current - median, weights[v])
        return cap_fn(update - median, weights[v])
    return fn


class QuorumIndexer:
    """quorum_indexer.go:20-43; ``validators`` = oracle.pos.Validators."""

    def __init__(self, validators, dagi, diff_metric_fn):
        n = len(validators)
        self.v = validators
        self.dagi = dagi
        self.fn = diff_metric_fn
        self.matrix = [[0] * n for _ in range(n)]      # row = validator, column = creator
        self.self_parent_seqs = [0] * n
        self.median_seqs = [0] * n
        self.dirty = True

    def process_event(self, e, self_event):
        """:86-98."""
        vc = self.dagi.get_merged_highest_before(e.id)
        c = self.v.idxs[e.creator]
        for i in range(len(self.v)):
            s = seq_of(vc.get(i))
            self.matrix[i][c] = s
            if self_event:
                self.self_parent_seqs[i] = s
        self.dirty = True

    def recache_state(self):
        """:100-121 (the stable sort here and Go's sort.Slice give the same
        median: the crossing point of the weight sum never depends on the order
        inside a group of equal seqs)."""
        for i in range(len(self.v)):
            pairs = sorted(((self.matrix[i][k], self.v.weights[k]) for k in range(len(self.v))),
                           key=lambda p: -p[0])
            self.median_seqs[i] = wmedian_of(pairs, self.v.quorum())[0]
        self.dirty = False

    def get_metric_of(self, eid):
        """:123-136 (Metric is uint64)."""
        if self.dirty:
            self.recache_state()
        vc = self.dagi.get_merged_highest_before(eid)
        m = 0
        for i in range(len(self.v)):
            m += self.fn(self.median_seqs[i], self.self_parent_seqs[i], seq_of(vc.get(i)), i)
        return m & 0xFFFFFFFFFFFFFFFF

    def search_strategy(self):
        if self.dirty:
            self.recache_state()
        return MetricStrategy(self.get_metric_of)

    def get_global_median_seqs(self):
        if self.dirty:
            self.recache_state()
        return list(self.median_seqs)

    def get_global_matrix(self):
        return [list(r) for r in self.matrix]

    def get_self_parent_seqs(self):
        return list(self.self_parent_seqs)


class MetricStrategy:
    """weighted.go:7-27."""

    def __init__(self, metric_fn):
        self.metric_fn = metric_fn

    def choose(self, existing, options):
        """Returns (index, order_independent)."""
        ms = [self.metric_fn(o) for o in options]
        max_i, max_w = 0, 0
        for i, w in enumerate(ms):
            if max_w == 0 or w > max_w:
                max_i, max_w = i, w
        unique = len(options) == 1 or (max_w > 0 and ms.count(max_w) == 1)
        return max_i, unique


def choose_parents(existing, options, strategies):
    """search.go:14-34.  Options are taken in sorted order (the reference's
    are in map order); returns (parents, order_independent)."""
    opts = set(options) - set(existing)
    parents = list(existing)
    det = True
    for st in strategies:
        if not opts:
            break
        cur = sorted(opts, key=str)
        best, unique = st.choose(parents, cur)
        det = det and unique
        parents.append(cur[best])
        opts.discard(cur[best])
    return parents, det


def parents_to_string(pp, name_of=str):
    """quorum_indexer_test.go:201-214: self-parent first, the rest sorted."""
    names = [name_of(p) for p in pp]
    if len(names) >= 3:
        names = names[:1] + sorted(names[1:])
    return "[" + ", ".join(names) + "]"


class DenseQuorumIndexerNp:
    """The same QuorumIndexer over a dense-index C oracle (``corc.OracleIndex``)
    with numpy arrays and the capped metric built in -- the CPU timing baseline
    of bench.py (a vectorised port: ProcessEvent writes one matrix column,
    recacheState sorts every row at once, GetMetricOf evaluates the capped
    difference over all validators).  ``weights`` in idx order; events are
    dense indices.  Checked against ``QuorumIndexer`` by
    tests/test_emitter_oracle.py."""

    def __init__(self, weights, index, cap=2):
        import numpy as np
        self.np = np
        self.w = np.asarray(weights, dtype=np.int64)
        self.V = len(weights)
        self.ix = index
        self.cap = cap
        self.quorum = int(self.w.sum()) * 2 // 3 + 1
        self.matrix = np.zeros((self.V, self.V), dtype=np.int64)   # [validator, creator]
        self.sp = np.zeros(self.V, dtype=np.int64)
        self.median = np.zeros(self.V, dtype=np.int64)
        self.dirty = True

    def _seqs(self, ev):
        """seqOf of the merged HighestBefore row (quorum_indexer.go:70-75)."""
        np = self.np
        r = np.frombuffer(self.ix.merged_hb(ev), dtype=np.uint32).reshape(-1, 2)[:self.V].astype(np.int64)
        s = np.zeros(self.V, dtype=np.int64)
        s[:len(r)] = r[:, 0]
        fork = (r[:, 0] == 0) & (r[:, 1] == 0x7FFFFFFF)
        s[:len(r)][fork] = FORK_SEQ
        return s

    def process_event(self, ev, creator, self_event):
        s = self._seqs(ev)
        self.matrix[:, creator] = s
        if self_event:
            self.sp[:] = s
        self.dirty = True

    def recache(self):
        np = self.np
        order = np.argsort(-self.matrix, axis=1, kind="stable")
        ws = np.cumsum(self.w[order], axis=1)
        k = np.argmax(ws >= self.quorum, axis=1)
        self.median = np.take_along_axis(self.matrix, order, axis=1)[np.arange(self.V), k]
        self.dirty = False

    def metric_of(self, evs):
        np = self.np
        if self.dirty:
            self.recache()
        out = np.zeros(len(evs), dtype=np.uint64)
        cap = self.cap
        for i, ev in enumerate(evs):
            u = self._seqs(ev)
            m, cur = self.median, self.sp
            d_um = np.minimum(u - m, cap) * self.w
            d_cm = np.minimum(cur - m, cap) * self.w
            val = np.where(m < cur, d_um - d_cm, d_um)
            val = np.where((u <= m) | (u <= cur), 0, val)
            out[i] = np.uint64(int(val.sum()) & 0xFFFFFFFFFFFFFFFF)
        return out
