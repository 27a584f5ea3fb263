"""emitter/ancestor.QuorumIndexer over include/lachesis_emitter.h.

Shaped like the reference (emitter/ancestor/quorum_indexer.go:20-158,
weighted.go, search.go) so the parity tests read like
quorum_indexer_test.go.  The matrix, the self-parent seqs and the weighted
medians live on the GPU next to the index's HighestBefore plane
(lachesis-base_amd/csrc/lx_emitter.{cpp,hip}); this module only keeps the
event-ID -> dense-index map of the :class:`VecfcIndex` it is built on.

The reference's DiffMetricFn is a Go closure; the library evaluates the
capped-difference metric of quorum_indexer_test.go:117-131 on the device with
the cap as a parameter (``cap``).  ``choose_parents`` is the host-side
ChooseParents (search.go:14-34); a MetricStrategy asks the metrics of all
options in one batched call.
"""

import ctypes

import numpy as np

from .capi import LxError, _p, u8p, u32p, u64p, vp


class QuorumIndexer:
    """NewQuorumIndexer(validators, dagi, capped metric) (quorum_indexer.go:33-43).

    ``dagi`` is a :class:`lachesis_hip.VecfcIndex` (its epoch's validators are
    the QuorumIndexer's).  Call :meth:`reset` after the index's epoch reset."""

    def __init__(self, dagi, cap=2):
        self.dagi = dagi
        self.L = dagi.ix.L
        self.cap = int(cap)
        h = vp()
        rc = self.L.lx_qi_create(dagi.ix.h, ctypes.byref(h))
        if rc != 0:
            raise LxError(rc, dagi.ix.L.lx_last_error(dagi.ix.h).decode())
        self.h = h
        self.V = len(dagi.validators.weights)

    def close(self):
        if getattr(self, "h", None):
            self.L.lx_qi_destroy(self.h)
            self.h = None

    __del__ = close

    def _chk(self, rc):
        if rc != 0:
            raise LxError(rc, self.L.lx_qi_last_error(self.h).decode())

    def reset(self):
        self._chk(self.L.lx_qi_reset(self.h))
        self.V = len(self.dagi.validators.weights)

    def _dense(self, ids):
        out = np.empty(len(ids), dtype=np.uint32)
        for k, eid in enumerate(ids):
            i = self.dagi._idx(eid)
            if i is None:
                raise LxError(-2, "event %r not indexed" % (eid,))
            out[k] = i
        return out

    # ProcessEvent (:86-98), batched: events in order, self flags per event
    def process_events(self, events, self_event):
        ev = self._dense([e.id for e in events])
        fl = np.ascontiguousarray(self_event, dtype=np.uint8)
        if len(ev):
            self._chk(self.L.lx_qi_process_events(self.h, len(ev), _p(ev, u32p), _p(fl, u8p)))

    def process_event(self, e, self_event):
        self.process_events([e], [1 if self_event else 0])

    # GetMetricOf (:123-136), batched
    def get_metrics_of(self, ids):
        ev = self._dense(ids)
        out = np.zeros(len(ev), dtype=np.uint64)
        if len(ev):
            self._chk(self.L.lx_qi_metric_of(self.h, len(ev), _p(ev, u32p), self.cap, _p(out, u64p)))
        return out

    def get_metric_of(self, eid):
        return int(self.get_metrics_of([eid])[0])

    def search_strategy(self):
        return MetricStrategy(self.get_metrics_of)

    def get_global_median_seqs(self):
        out = np.zeros(self.V, dtype=np.uint32)
        self._chk(self.L.lx_qi_median_seqs(self.h, _p(out, u32p)))
        return out

    def get_global_matrix(self):
        """V x V, row = validator, column = creator (Matrix.Row, :55-57)."""
        out = np.zeros(self.V * self.V, dtype=np.uint32)
        self._chk(self.L.lx_qi_matrix(self.h, _p(out, u32p)))
        return out.reshape(self.V, self.V)

    def get_self_parent_seqs(self):
        out = np.zeros(self.V, dtype=np.uint32)
        self._chk(self.L.lx_qi_self_parent_seqs(self.h, _p(out, u32p)))
        return out


class MetricStrategy:
    """weighted.go:7-27: the option with the maximum metric (first strictly
    greater wins; the last one if every metric is 0)."""

    def __init__(self, metrics_fn):
        self.metrics_fn = metrics_fn

    def choose(self, existing, options):
        ms = self.metrics_fn(list(options))
        max_i, max_w = 0, 0
        for i, w in enumerate(ms):
            w = int(w)
            if max_w == 0 or w > max_w:
                max_i, max_w = i, w
        return max_i


def choose_parents(existing, options, strategies):
    """search.go:14-34 (options in the caller's order)."""
    opts = [o for o in dict.fromkeys(options) if o not in set(existing)]
    parents = list(existing)
    for st in strategies:
        if not opts:
            break
        best = st.choose(parents, opts)
        parents.append(opts[best])
        del opts[best]
    return parents

