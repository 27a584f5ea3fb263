"""Drop-in replay: the unchanged caller's per-event / per-pair calls on an index.

ctypes binding of tools/lx_dropin.cpp (liblx_bench.so): IndexedLachesis.Process
restated in C++ (abft/indexed_lachesis.go:69-82, abft/event_processing.go,
abft/election), making exactly the reference's index calls -- Add per event,
ForklessCause per (event, root) pair, Flush, DropNotFlushed,
GetMergedHighestBefore per decided frame -- on

* ``kind="hip"``: the HIP library through its C ABI (lx_forkless_cause and its
  result cache -- the path a cgo shim binds);
* ``kind="cpu"``: a CPU index handed in as C function pointers (bench.py's
  cpu_baseline leg and the tests pass the C restatement this way) behind the
  reference's ForklessCause LRU;
* ``kind="recorded"``: the answers a previous run recorded (the caller's own
  time, without an index).
"""

import ctypes
import os

import numpy as np

from .capi import LxFcStats, load_library

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p
KINDS = {"hip": 0, "cpu": 1, "recorded": 2}


class DropinCfg(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("device", ctypes.c_int), ("fc_cache", ctypes.c_int64),
                ("lru_pairs", ctypes.c_uint32), ("cpu", vp), ("cpu_add", vp), ("cpu_flush", vp), ("cpu_drop", vp),
                ("cpu_fc", vp), ("cpu_merged_hb", vp), ("rec_fc", u8p), ("rec_fc_cap", ctypes.c_uint64),
                ("rec_mhb", u8p), ("rec_mhb_cap", ctypes.c_uint64), ("max_events", ctypes.c_uint64)]


class DropinOut(ctypes.Structure):
    _fields_ = [("frames", u32p), ("roots_per_frame", u32p), ("frames_cap", ctypes.c_uint32),
                ("block_frame", u32p), ("block_atropos", u32p), ("block_ncheat", u32p), ("block_nconf", u32p),
                ("blocks_cap", ctypes.c_uint32), ("checkpoint_s", ctypes.POINTER(ctypes.c_double)),
                ("events", ctypes.c_uint64), ("blocks", ctypes.c_uint64), ("fc_calls", ctypes.c_uint64),
                ("adds", ctypes.c_uint64), ("flushes", ctypes.c_uint64), ("drops", ctypes.c_uint64),
                ("merged_hb_calls", ctypes.c_uint64), ("trace_hash", ctypes.c_uint64),
                ("seconds", ctypes.c_double), ("add_seconds", ctypes.c_double), ("max_frame", ctypes.c_uint32),
                ("fc", LxFcStats), ("lru_hits", ctypes.c_uint64)]


_lib = None


def _bench_lib():
    global _lib
    if _lib is None:
        load_library()   # the HIP library first (one HIP runtime per process, see capi.load_library)
        L = ctypes.CDLL(os.path.join(_PKG, "build", "liblx_bench.so"))
        L.lx_dropin_replay.restype = ctypes.c_int
        L.lx_dropin_replay.argtypes = [ctypes.POINTER(DropinCfg), ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p,
                                       u64p, u32p, u32p, ctypes.POINTER(DropinOut), ctypes.c_char_p, ctypes.c_uint32]
        _lib = L
    return _lib


class Recording:
    """Buffers a run writes its ForklessCause answers and merged rows into
    (kind "hip" / "cpu"), and a "recorded" run reads them back."""

    def __init__(self, fc_cap, V, mhb_cap=4096):
        self.fc = np.zeros(max(fc_cap, 1), dtype=np.uint8)
        self.mhb = np.zeros(max(mhb_cap, 1) * 8 * V, dtype=np.uint8)
        self.mhb_cap = mhb_cap


def replay(dag, weights, claimed, kind="hip", device=0, fc_cache=-1, cpu=None, lru_pairs=20000, record=None,
           max_events=0):
    """Process the DAG's events (claimed frames) through the caller restatement
    on one backend.  ``cpu``: dict of C function pointers (ints) "h", "add",
    "flush", "drop", "fc", "merged_hb" (oracle/csrc/oracle.c signatures).
    Returns a dict of results and timings."""
    L = _bench_lib()
    N = len(dag)
    w = np.ascontiguousarray(weights, dtype=np.uint32)
    cr = np.ascontiguousarray(dag.creator, dtype=np.uint32)
    sq = np.ascontiguousarray(dag.seq, dtype=np.uint32)
    po = np.ascontiguousarray(dag.poff, dtype=np.uint64)
    pa = np.ascontiguousarray(dag.par if len(dag.par) else [0], dtype=np.uint32)
    cl = np.ascontiguousarray(claimed, dtype=np.uint32)
    cfg = DropinCfg()
    cfg.kind = KINDS[kind]
    cfg.device = device
    cfg.fc_cache = fc_cache
    cfg.lru_pairs = lru_pairs if kind == "cpu" else 0
    cfg.max_events = max_events
    if kind == "cpu":
        cfg.cpu, cfg.cpu_add, cfg.cpu_flush, cfg.cpu_drop = cpu["h"], cpu["add"], cpu["flush"], cpu["drop"]
        cfg.cpu_fc, cfg.cpu_merged_hb = cpu["fc"], cpu["merged_hb"]
    if record is not None:
        cfg.rec_fc = record.fc.ctypes.data_as(u8p)
        cfg.rec_fc_cap = len(record.fc)
        cfg.rec_mhb = record.mhb.ctypes.data_as(u8p)
        cfg.rec_mhb_cap = record.mhb_cap
    frames = np.zeros(N, dtype=np.uint32)
    rpf = np.zeros(4096, dtype=np.uint32)
    bcap = 4096
    bf, ba, bc, bn = (np.zeros(bcap, dtype=np.uint32) for _ in range(4))
    ck = np.zeros(N // 1000 + 1, dtype=np.float64)
    out = DropinOut()
    out.frames = frames.ctypes.data_as(u32p)
    out.roots_per_frame = rpf.ctypes.data_as(u32p)
    out.frames_cap = len(rpf)
    out.block_frame, out.block_atropos = bf.ctypes.data_as(u32p), ba.ctypes.data_as(u32p)
    out.block_ncheat, out.block_nconf = bc.ctypes.data_as(u32p), bn.ctypes.data_as(u32p)
    out.blocks_cap = bcap
    out.checkpoint_s = ck.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    err = ctypes.create_string_buffer(512)
    rc = L.lx_dropin_replay(ctypes.byref(cfg), len(w), w.ctypes.data_as(u32p), N, cr.ctypes.data_as(u32p),
                            sq.ctypes.data_as(u32p), po.ctypes.data_as(u64p), pa.ctypes.data_as(u32p),
                            cl.ctypes.data_as(u32p), ctypes.byref(out), err, 512)
    if rc != 0:
        raise RuntimeError("lx_dropin_replay (%s): %d %s" % (kind, rc, err.value.decode()))
    nb = min(out.blocks, bcap)
    M = out.events
    return {"events": M, "frames": frames[:M], "roots_per_frame": rpf[:out.max_frame + 2],
            "block_frame": bf[:nb], "block_atropos": ba[:nb], "block_ncheat": bc[:nb], "block_nconf": bn[:nb],
            "checkpoint_s": ck[:M // 1000], "fc_calls": out.fc_calls, "adds": out.adds, "flushes": out.flushes,
            "drops": out.drops, "merged_hb_calls": out.merged_hb_calls, "trace_hash": out.trace_hash,
            "seconds": out.seconds, "add_seconds": out.add_seconds, "lru_hits": out.lru_hits,
            "fc_cache": {k: getattr(out.fc, k) for k, _ in LxFcStats._fields_}}
