"""Synthetic workload tooling (build/libdag_tools.so): tdag-structured DAGs and
ForklessCause query sets.  Bit-identical to oracle/tdag.py:rand_fork_dag."""

import ctypes
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS_PATH = os.path.join(_PKG, "build", "libdag_tools.so")
_t = None

u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


def _lib():
    global _t
    if _t is None:
        if not os.path.exists(TOOLS_PATH):
            raise ImportError("tools library not built: %s" % TOOLS_PATH)
        L = ctypes.CDLL(TOOLS_PATH)
        L.dag_gen.restype = ctypes.c_int64
        L.dag_gen.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_uint64, u32p, u32p, u32p, u64p, u32p, ctypes.c_uint64]
        L.fc_queries.restype = None
        L.fc_queries.argtypes = [ctypes.c_uint64, u32p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, u32p, u32p]
        _t = L
    return _t


class Dag:
    """Dense DAG in Add order: creator column, seq, lamport, CSR parents."""

    def __init__(self, creator, seq, lamport, poff, par, n_nodes):
        self.creator, self.seq, self.lamport, self.poff, self.par = creator, seq, lamport, poff, par
        self.n_nodes = n_nodes

    def __len__(self):
        return len(self.creator)

    def slice(self, lo, hi):
        """Events [lo, hi) as a batch (parents keep global indices)."""
        off = self.poff[lo:hi + 1]
        return (self.creator[lo:hi], self.seq[lo:hi], off, self.par)


def gen_dag(n_nodes, events_per_node, parent_count, cheaters=0, forks=0, seed=1):
    L = _lib()
    n = n_nodes * events_per_node
    creator = np.zeros(n, dtype=np.uint32)
    seq = np.zeros(n, dtype=np.uint32)
    lam = np.zeros(n, dtype=np.uint32)
    poff = np.zeros(n + 1, dtype=np.uint64)
    cap = n * max(parent_count, 1)
    par = np.zeros(max(cap, 1), dtype=np.uint32)
    np_ = L.dag_gen(n_nodes, events_per_node, parent_count, cheaters, forks, seed,
                    creator.ctypes.data_as(u32p), seq.ctypes.data_as(u32p), lam.ctypes.data_as(u32p),
                    poff.ctypes.data_as(u64p), par.ctypes.data_as(u32p), cap)
    if np_ < 0:
        raise RuntimeError("parent buffer too small")
    return Dag(creator, seq, lam, poff, par[:max(np_, 1)], n_nodes)


def level_order(dag):
    """The same DAG in level order: events sorted by Lamport time (= 1 + the
    longest parent chain, which is the DAG level for tdag-structured DAGs),
    ties kept in Add order -- the order a level-synchronous batcher
    (lx_batcher_pop) releases a whole epoch in.  Parents are renumbered; each
    event keeps its parent list order (self-parent first)."""
    n = len(dag)
    perm = np.argsort(dag.lamport, kind="stable")
    inv = np.empty(n, dtype=np.uint32)
    inv[perm] = np.arange(n, dtype=np.uint32)
    counts = np.diff(dag.poff).astype(np.int64)
    new_counts = counts[perm]
    poff = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(new_counts, out=poff[1:])
    total = int(poff[-1])
    idx = np.repeat(dag.poff[:-1][perm].astype(np.int64) - poff[:-1].astype(np.int64), new_counts) + \
        np.arange(total, dtype=np.int64)
    par = inv[dag.par[idx]] if total else dag.par[:1].copy()
    return Dag(dag.creator[perm].copy(), dag.seq[perm].copy(), dag.lamport[perm].copy(), poff, par, dag.n_nodes)


def fc_queries(lamport, nq, window=64, seed=7):
    L = _lib()
    lamport = np.ascontiguousarray(lamport, dtype=np.uint32)
    qa = np.zeros(nq, dtype=np.uint32)
    qb = np.zeros(nq, dtype=np.uint32)
    L.fc_queries(len(lamport), lamport.ctypes.data_as(u32p), nq, window, seed,
                 qa.ctypes.data_as(u32p), qb.ctypes.data_as(u32p))
    return qa, qb
