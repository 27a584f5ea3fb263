"""ctypes binding of include/lachesis_hip.h (dense event indices)."""

import ctypes
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# LX_LIB: another build of the same library (diagnostics: make wprof)
LIB_PATH = os.environ.get("LX_LIB") or os.path.join(_PKG, "build", "liblachesis_hip.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p

# (name, restype, argtypes) for every entry point of include/lachesis_hip.h
SIGNATURES = [
    ("lx_create", ctypes.c_int, [vp, ctypes.POINTER(vp)]),
    ("lx_destroy", None, [vp]),
    ("lx_last_error", ctypes.c_char_p, [vp]),
    ("lx_set_option", ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int64]),
    ("lx_reset", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_add_batch", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u32p, u64p, u32p, u32p, u32p]),
    ("lx_add_batch_dev", ctypes.c_int, [vp, ctypes.c_uint32, vp, vp, vp, vp, u32p]),
    ("lx_flush", ctypes.c_int, [vp]),
    ("lx_drop_not_flushed", ctypes.c_int, [vp]),
    ("lx_writeback_prepare", ctypes.c_int, [vp, vp]),
    ("lx_writeback_fetch", ctypes.c_int, [vp, u64p, u8p, u32p, u64p, u8p, u8p, u8p]),
    ("lx_load_rows", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u32p, u64p, u32p, u8p, u64p, u8p, u64p, u8p]),
    ("lx_load_finish", ctypes.c_int, [vp, u8p, ctypes.c_uint32]),
    ("lx_num_events", ctypes.c_uint64, [vp]),
    ("lx_num_branches", ctypes.c_uint32, [vp]),
    ("lx_at_least_one_fork", ctypes.c_int, [vp]),
    ("lx_forkless_cause_batch", ctypes.c_int, [vp, ctypes.c_uint64, u32p, u32p, u8p]),
    ("lx_forkless_cause", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, u8p]),
    ("lx_fc_cache_stats", ctypes.c_int, [vp, vp]),
    ("lx_forkless_cause_batch_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, vp]),
    ("lx_fc_early_counters", ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_uint64)]),
    ("lx_forkless_cause_partial_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, vp]),
    ("lx_fc_combine_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp]),
    ("lx_fc_shard_early", ctypes.c_int, [vp, u32p]),
    ("lx_fc_shard_decide_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp]),
    ("lx_fc_shard_undecided_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, vp, vp, vp, vp, vp, u64p]),
    ("lx_fc_shard_answer_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, ctypes.c_uint64, vp, vp, vp, vp]),
    ("lx_quorum", ctypes.c_uint32, [vp]),
    ("lx_get_highest_before", ctypes.c_int, [vp, ctypes.c_uint32, u8p, ctypes.c_uint32, u32p]),
    ("lx_get_lowest_after", ctypes.c_int, [vp, ctypes.c_uint32, u8p, ctypes.c_uint32, u32p]),
    ("lx_get_merged_highest_before", ctypes.c_int, [vp, ctypes.c_uint32, u8p, ctypes.c_uint32, u32p]),
    ("lx_get_highest_before_batch", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u64p, u8p, ctypes.c_uint64]),
    ("lx_get_lowest_after_batch", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u64p, u8p, ctypes.c_uint64]),
    ("lx_get_merged_highest_before_batch", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u64p, u8p, ctypes.c_uint64]),
    ("lx_get_event_branch_id", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_get_server_stats", ctypes.c_int, [vp, u64p]),
    ("lx_live_handles", ctypes.c_int, []),
    ("lx_fc_early_rounds", ctypes.c_int, [vp, u64p]),
    ("lx_device_bytes", ctypes.c_int, [vp, u64p]),
    ("lx_get_rows_dev", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, ctypes.c_uint64, vp]),
    ("lx_row_bytes_max", ctypes.c_int, [vp, u64p]),
    ("lx_rowseg_rows_unroute", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint64, vp, vp, vp]),
    ("lx_rowseg_get_rows", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint64, vp, vp, ctypes.c_uint64, vp]),
    ("lx_get_branches_info", ctypes.c_int, [vp, u32p, u32p, ctypes.c_uint32, u32p]),
    ("lx_shard_of", ctypes.c_int, [vp, u32p, u32p]),
    ("lx_shard_range", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u32p]),
    ("lx_shard_block", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, u64p]),
    ("lx_shard_wire", ctypes.c_int, [vp, u32p]),
    ("lx_la_pack_dev", ctypes.c_int, [vp, ctypes.c_uint32, vp, vp]),
    ("lx_la_unpack_dev", ctypes.c_int, [vp, ctypes.c_uint32, vp, vp]),
    ("lx_la_own_dev", ctypes.c_int, [vp, vp]),
    ("lx_shard_dirty", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_shard_dirty_set", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_shard_dirty_commit", ctypes.c_int, [vp]),
    ("lx_shard_block_wire", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_la_pack_wire_dev", ctypes.c_int, [vp, ctypes.c_uint32, vp, ctypes.c_uint32]),
    ("lx_la_unpack_wire_dev", ctypes.c_int, [vp, ctypes.c_uint32, vp, ctypes.c_uint32]),
    ("lx_last_stats", ctypes.c_int, [vp, vp]),
    ("lx_last_walk_clock", ctypes.c_int, [vp, vp]),
    ("lx_last_segment_stats", ctypes.c_int, [vp, vp]),
    ("lx_rowseg_range", ctypes.c_int, [vp, u32p, u32p]),
    ("lx_rowseg_bounds", ctypes.c_int, [vp, u32p]),
    ("lx_rowseg_row_words", ctypes.c_int, [vp, u32p]),
    ("lx_rowseg_request_cap", ctypes.c_int, [vp, u32p]),
    ("lx_rowseg_requests", ctypes.c_int, [vp, vp, ctypes.c_uint32, u32p]),
    ("lx_rowseg_serve", ctypes.c_int, [vp, ctypes.c_uint32, vp, vp, vp]),
    ("lx_rowseg_receive", ctypes.c_int, [vp, ctypes.c_uint32, vp, vp, vp, u32p]),
    ("lx_rowseg_la", ctypes.c_int, [vp, u64p]),
    ("lx_rowseg_la_fetch", ctypes.c_int, [vp, vp]),
    ("lx_rowseg_la_apply", ctypes.c_int, [vp, ctypes.c_uint64, vp]),
    ("lx_rowseg_finish", ctypes.c_int, [vp]),
    ("lx_rowseg_fc_route", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, vp, vp, u64p]),
    ("lx_rowseg_fc_need", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, ctypes.c_uint64, u64p]),
    ("lx_rowseg_la_serve", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp]),
    ("lx_rowseg_la_store", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp]),
    ("lx_rowseg_fc_unroute", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp]),
    ("lx_rowseg_forkless_cause", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp, u64p]),
    ("lx_device_planes", ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), u32p, ctypes.POINTER(vp)]),
    ("lx_sync", ctypes.c_int, [vp]),
    ("lx_shard_comm_unique_id", ctypes.c_int, [u8p]),
    ("lx_shard_comm_create", ctypes.c_int, [vp, u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(vp)]),
    ("lx_shard_comm_destroy", None, [vp]),
    ("lx_shard_comm_last_error", ctypes.c_char_p, [vp]),
    ("lx_shard_exchange", ctypes.c_int, [vp]),
    ("lx_rowseg_of", ctypes.c_int, [vp, u32p, u32p]),
    ("lx_rowseg_comm_create", ctypes.c_int, [vp, u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(vp)]),
    ("lx_rowseg_exchange", ctypes.c_int, [vp, u64p]),
    ("lx_shard_exchange_layout", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, u64p, u32p, u64p]),
    ("lx_forkless_cause_sharded_dev", ctypes.c_int, [vp, ctypes.c_uint64, vp, vp, vp]),
    ("lx_shard_fc_undecided", ctypes.c_int, [vp, u64p]),
    ("lx_shard_get_rows", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint64, vp, vp, ctypes.c_uint64, vp]),
    # include/lachesis_abft.h
    ("lx_abft_create", ctypes.c_int, [vp, ctypes.POINTER(vp)]),
    ("lx_abft_destroy", None, [vp]),
    ("lx_abft_last_error", ctypes.c_char_p, [vp]),
    ("lx_abft_set_option", ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int64]),
    ("lx_abft_bootstrap", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, vp]),
    ("lx_abft_reset", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, u32p]),
    ("lx_abft_process_batch", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u32p, u64p, u32p, u32p, u32p, u32p]),
    ("lx_abft_build", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p]),
    ("lx_abft_epoch", ctypes.c_uint32, [vp]),
    ("lx_abft_last_decided_frame", ctypes.c_uint32, [vp]),
    ("lx_abft_frame_roots", ctypes.c_int, [vp, ctypes.c_uint32, u32p, ctypes.c_uint32, u32p]),
    ("lx_abft_event_frame", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_abft_event_confirmed_on", ctypes.c_int, [vp, ctypes.c_uint32, u32p]),
    ("lx_abft_last_stats", ctypes.c_int, [vp, vp]),
    ("lx_abft_block_log", ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp]),
    # include/lachesis_emitter.h
    ("lx_qi_create", ctypes.c_int, [vp, ctypes.POINTER(vp)]),
    ("lx_qi_destroy", None, [vp]),
    ("lx_qi_last_error", ctypes.c_char_p, [vp]),
    ("lx_qi_reset", ctypes.c_int, [vp]),
    ("lx_qi_process_events", ctypes.c_int, [vp, ctypes.c_uint32, u32p, u8p]),
    ("lx_qi_median_seqs", ctypes.c_int, [vp, u32p]),
    ("lx_qi_matrix", ctypes.c_int, [vp, u32p]),
    ("lx_qi_self_parent_seqs", ctypes.c_int, [vp, u32p]),
    ("lx_qi_metric_of", ctypes.c_int, [vp, ctypes.c_uint32, u32p, ctypes.c_uint32, u64p]),
    # include/lachesis_batcher.h
    ("lx_batcher_create", ctypes.c_int, [ctypes.POINTER(vp)]),
    ("lx_batcher_destroy", None, [vp]),
    ("lx_batcher_last_error", ctypes.c_char_p, [vp]),
    ("lx_batcher_reset", ctypes.c_int, [vp]),
    ("lx_batcher_reserve", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("lx_batcher_push", ctypes.c_int, [vp, ctypes.c_uint32, u64p, u32p, u32p, u64p, u64p, u8p]),
    ("lx_batcher_peek", ctypes.c_int, [vp, u32p, u64p, u32p, u32p]),
    ("lx_batcher_pop", ctypes.c_int, [vp, u64p, u32p, u32p, u64p, u32p, u32p, u64p]),
    ("lx_batcher_unpop", ctypes.c_int, [vp]),
    ("lx_batcher_dense", ctypes.c_int, [vp, ctypes.c_uint64, u32p]),
]


class LxConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("event_capacity", ctypes.c_uint64),
                ("branch_reserve", ctypes.c_uint32), ("shard_rank", ctypes.c_uint32),
                ("shard_count", ctypes.c_uint32)]


class LxStats(ctypes.Structure):
    _fields_ = [("ms_assign", ctypes.c_float), ("ms_index", ctypes.c_float),
                ("ms_marks", ctypes.c_float), ("index_launches", ctypes.c_uint32)]


class LxFcStats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("hits", ctypes.c_uint64), ("row_fills", ctypes.c_uint64),
                ("tile_fills", ctypes.c_uint64), ("pairs", ctypes.c_uint64), ("slots", ctypes.c_uint32),
                ("slots_used", ctypes.c_uint32), ("miss_ns", ctypes.c_uint64), ("wait_ns", ctypes.c_uint64),
                ("launch_ns", ctypes.c_uint64), ("quiesce_ns", ctypes.c_uint64), ("fused", ctypes.c_uint64)]


class LxSegStats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint32), ("first_event", ctypes.c_uint32 * 65), ("partial", ctypes.c_uint32 * 64),
                ("walk_ms", ctypes.c_float * 64), ("partial_ms", ctypes.c_float), ("la_ms", ctypes.c_float),
                ("one_launch", ctypes.c_uint32)]


class LxWriteback(ctypes.Structure):
    _fields_ = [("first_event", ctypes.c_uint64), ("n_events", ctypes.c_uint64), ("n_la_rows", ctypes.c_uint64),
                ("hb_bytes", ctypes.c_uint64), ("la_bytes", ctypes.c_uint64), ("bi_bytes", ctypes.c_uint32)]


class LxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("lachesis_hip error %d: %s" % (code, msg))
        self.code = code


def load_library(path=LIB_PATH):
    """Load the HIP library; raises if it is missing (no fallback path)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch-ROCm bundles its own
        # libamdhip64.so.7 (same soname as /opt/rocm's).  Loading torch first
        # makes this library bind to torch's copy; loading ours first would
        # make torch bind to /opt/rocm's, and torch then finds no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(path):
            raise ImportError("HIP library not built: %s (run __graft_entry__.build())" % path)
        L = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


# lx_set_option values applied to every new Index (tests select implementation
# paths this way, e.g. {"small_max": 0}; every option gives identical results)
DEFAULT_OPTIONS = {}


class Index:
    """Dense-index handle over lx_* (one GPU, one epoch at a time)."""

    def __init__(self, device=0, event_capacity=0, branch_reserve=0, shard_rank=0, shard_count=1, options=None):
        self.L = load_library()
        cfg = LxConfig(device, event_capacity, branch_reserve, shard_rank, shard_count)
        h = vp()
        rc = self.L.lx_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise LxError(rc, "lx_create failed (device %d)" % device)
        self.h = h
        for k, v in dict(DEFAULT_OPTIONS, **(options or {})).items():
            self.set_option(k, v)

    def set_option(self, name, value):
        """lx_set_option (path selection; results never change)."""
        self._chk(self.L.lx_set_option(self.h, name.encode(), int(value)))

    def close(self):
        if getattr(self, "h", None):
            self.L.lx_destroy(self.h)
            self.h = None

    __del__ = close

    def _chk(self, rc):
        if rc != 0:
            raise LxError(rc, self.L.lx_last_error(self.h).decode())
        return rc

    # lifecycle ---------------------------------------------------------------
    def reset(self, weights_by_idx):
        w = _u32(weights_by_idx)
        self._chk(self.L.lx_reset(self.h, len(w), _p(w, u32p)))

    def add_batch(self, creator_idx, seq, parent_off, parent_idx, want_branches=False):
        creator_idx = _u32(creator_idx)
        seq = _u32(seq)
        off = np.ascontiguousarray(parent_off, dtype=np.uint64)
        par = _u32(parent_idx) if len(parent_idx) else np.zeros(1, dtype=np.uint32)
        n = len(creator_idx)
        out = np.zeros(n, dtype=np.uint32) if want_branches else None
        err = ctypes.c_uint32(0xFFFFFFFF)
        rc = self.L.lx_add_batch(self.h, n, _p(creator_idx, u32p), _p(seq, u32p), _p(off, u64p),
                                 _p(par, u32p), _p(out, u32p) if out is not None else None,
                                 ctypes.byref(err))
        if rc != 0:
            e = LxError(rc, self.L.lx_last_error(self.h).decode())
            e.index = err.value
            raise e
        return out

    def add_batch_dev(self, n, creator_ptr, seq_ptr, poff_ptr, par_ptr):
        err = ctypes.c_uint32(0xFFFFFFFF)
        rc = self.L.lx_add_batch_dev(self.h, n, creator_ptr, seq_ptr, poff_ptr, par_ptr, ctypes.byref(err))
        self._chk(rc)

    def add(self, creator_idx, seq, parents):
        return int(self.add_batch([creator_idx], [seq], [0, len(parents)], list(parents), True)[0])

    def flush(self):
        self._chk(self.L.lx_flush(self.h))

    def drop_not_flushed(self):
        self._chk(self.L.lx_drop_not_flushed(self.h))

    def writeback(self):
        """The Puts of the next Flush (lx_writeback_prepare + fetch), keyed by
        dense event index: {"S": {ev: HB bytes}, "s": {ev: LA bytes},
        "b": {ev: 4-B big-endian branch ID}, "B": RLP(BranchesInfo)}."""
        wb = LxWriteback()
        self._chk(self.L.lx_writeback_prepare(self.h, ctypes.byref(wb)))
        n, m = wb.n_events, wb.n_la_rows
        hb_off = np.zeros(n + 1, dtype=np.uint64)
        hb = np.zeros(max(wb.hb_bytes, 1), dtype=np.uint8)
        la_ev = np.zeros(max(m, 1), dtype=np.uint32)
        la_off = np.zeros(m + 1, dtype=np.uint64)
        la = np.zeros(max(wb.la_bytes, 1), dtype=np.uint8)
        br = np.zeros(max(4 * n, 1), dtype=np.uint8)
        bi = np.zeros(max(wb.bi_bytes, 1), dtype=np.uint8)
        self._chk(self.L.lx_writeback_fetch(self.h, _p(hb_off, u64p), _p(hb, u8p), _p(la_ev, u32p), _p(la_off, u64p),
                                            _p(la, u8p), _p(br, u8p), _p(bi, u8p)))
        hb_b, la_b, br_b = hb.tobytes(), la.tobytes(), br.tobytes()
        f = wb.first_event
        return {"S": {f + i: hb_b[hb_off[i]:hb_off[i + 1]] for i in range(n)},
                "s": {int(la_ev[k]): la_b[la_off[k]:la_off[k + 1]] for k in range(m)},
                "b": {f + i: br_b[4 * i:4 * i + 4] for i in range(n)},
                "B": bi.tobytes()[:wb.bi_bytes]}

    def load_rows(self, creator_idx, seq, parent_off, parent_idx, branch_be, hb_rows, la_rows):
        """lx_load_rows: events in a parents-first order with their persisted
        table bytes (branch_be: 4 bytes per event; hb_rows / la_rows: lists of
        bytes)."""
        creator_idx = _u32(creator_idx)
        seq = _u32(seq)
        off = np.ascontiguousarray(parent_off, dtype=np.uint64)
        par = _u32(parent_idx) if len(parent_idx) else np.zeros(1, dtype=np.uint32)
        br = np.frombuffer(bytes(branch_be) or b"\0", dtype=np.uint8).copy()
        hb_off = np.zeros(len(hb_rows) + 1, dtype=np.uint64)
        hb_off[1:] = np.cumsum([len(r) for r in hb_rows])
        la_off = np.zeros(len(la_rows) + 1, dtype=np.uint64)
        la_off[1:] = np.cumsum([len(r) for r in la_rows])
        hb = np.frombuffer(b"".join(hb_rows) or b"\0", dtype=np.uint8).copy()
        la = np.frombuffer(b"".join(la_rows) or b"\0", dtype=np.uint8).copy()
        self._chk(self.L.lx_load_rows(self.h, len(creator_idx), _p(creator_idx, u32p), _p(seq, u32p), _p(off, u64p),
                                      _p(par, u32p), _p(br, u8p), _p(hb_off, u64p), _p(hb, u8p), _p(la_off, u64p),
                                      _p(la, u8p)))

    def load_finish(self, bi_rlp):
        b = np.frombuffer(bytes(bi_rlp) or b"\0", dtype=np.uint8).copy()
        self._chk(self.L.lx_load_finish(self.h, _p(b, u8p), len(bi_rlp)))

    def num_events(self):
        return self.L.lx_num_events(self.h)

    def num_branches(self):
        return self.L.lx_num_branches(self.h)

    def at_least_one_fork(self):
        return bool(self.L.lx_at_least_one_fork(self.h))

    def quorum(self):
        return self.L.lx_quorum(self.h)

    # queries -----------------------------------------------------------------
    def forkless_cause_batch(self, a, b):
        a = _u32(a)
        b = _u32(b)
        out = np.zeros(len(a), dtype=np.uint8)
        if len(a):
            self._chk(self.L.lx_forkless_cause_batch(self.h, len(a), _p(a, u32p), _p(b, u32p), _p(out, u8p)))
        return out

    def forkless_cause(self, a, b):
        """lx_forkless_cause: one pair, as the reference's callers ask it (the
        index's result cache answers repeated questions)."""
        out = ctypes.c_uint8()
        self._chk(self.L.lx_forkless_cause(self.h, int(a), int(b), ctypes.byref(out)))
        return bool(out.value)

    def fc_cache_stats(self):
        st = LxFcStats()
        self._chk(self.L.lx_fc_cache_stats(self.h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in LxFcStats._fields_}

    def get_server_stats(self):
        """Single-row getters: rows the resident row server served, its
        launches, and calls that launched their own kernel instead."""
        out = np.zeros(3, dtype=np.uint64)
        self._chk(self.L.lx_get_server_stats(self.h, _p(out, u64p)))
        return {"served": int(out[0]), "launches": int(out[1]), "fallbacks": int(out[2])}

    def device_bytes(self):
        """Device memory this handle holds (lx_device_bytes), bytes."""
        out = np.zeros(4, dtype=np.uint64)
        self._chk(self.L.lx_device_bytes(self.h, _p(out, u64p)))
        return {"planes": int(out[0]), "receive": int(out[1]), "per_event": int(out[2]), "other": int(out[3]),
                "total": int(out.sum())}

    def live_handles(self):
        """Index handles alive in this process (the row server's auto mode)."""
        return int(self.L.lx_live_handles())

    def forkless_cause_batch_dev(self, n, a_ptr, b_ptr, out_ptr, stream=None):
        self._chk(self.L.lx_forkless_cause_batch_dev(self.h, n, a_ptr, b_ptr, out_ptr, stream))

    def fc_early_rounds(self):
        """(queries on the early path, of them reading columns 128-255, 256-511,
        the rest) since the last call (lx_fc_early_rounds)."""
        out = np.zeros(4, dtype=np.uint64)
        self._chk(self.L.lx_fc_early_rounds(self.h, _p(out, u64p)))
        return tuple(int(x) for x in out)

    def fc_early_counters(self):
        """(queries the kernel decided on its early path, of them past the first
        round, past the second: whole rows) since the last call."""
        q, f2, fw = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._chk(self.L.lx_fc_early_counters(self.h, ctypes.byref(q), ctypes.byref(f2), ctypes.byref(fw)))
        return q.value, f2.value, fw.value

    def forkless_cause_partial_dev(self, n, a_ptr, b_ptr, partial_ptr, stream=None):
        self._chk(self.L.lx_forkless_cause_partial_dev(self.h, n, a_ptr, b_ptr, partial_ptr, stream))

    def fc_combine_dev(self, n, sum_ptr, out_ptr, stream=None):
        self._chk(self.L.lx_fc_combine_dev(self.h, n, sum_ptr, out_ptr, stream))

    # ---- column-shard early exit (include/lachesis_hip.h lx_fc_shard_*)
    def fc_shard_early(self):
        """(applies, rest): whether shard 0 can decide queries alone on this
        epoch, and the stake of the other shards."""
        rest = ctypes.c_uint32()
        ok = self.L.lx_fc_shard_early(self.h, ctypes.byref(rest))
        return bool(ok), rest.value

    def fc_shard_decide_dev(self, n, partial_ptr, mask_ptr, stream=None):
        self._chk(self.L.lx_fc_shard_decide_dev(self.h, n, partial_ptr, mask_ptr, stream))

    def fc_shard_undecided_dev(self, n, mask_ptr, a_ptr, b_ptr, partial_ptr, idx_ptr, a_out, b_out, p_out):
        """The undecided queries compacted in query order; returns their count."""
        m = ctypes.c_uint64()
        self._chk(self.L.lx_fc_shard_undecided_dev(self.h, n, mask_ptr, a_ptr, b_ptr, partial_ptr, idx_ptr, a_out, b_out,
                                                   p_out, ctypes.byref(m)))
        return m.value

    def fc_shard_answer_dev(self, n, mask_ptr, m, idx_ptr, sum_ptr, out_ptr, stream=None):
        self._chk(self.L.lx_fc_shard_answer_dev(self.h, n, mask_ptr, m, idx_ptr, sum_ptr, out_ptr, stream))

    def sync(self):
        self._chk(self.L.lx_sync(self.h))

    def _bytes(self, f, ev):
        n = ctypes.c_uint32()
        self._chk(f(self.h, ev, None, 0, ctypes.byref(n)))
        buf = (ctypes.c_uint8 * max(n.value, 1))()
        self._chk(f(self.h, ev, buf, n.value, ctypes.byref(n)))
        return bytes(buf[:n.value])

    def highest_before(self, ev):
        return self._bytes(self.L.lx_get_highest_before, ev)

    def lowest_after(self, ev):
        return self._bytes(self.L.lx_get_lowest_after, ev)

    def merged_highest_before(self, ev):
        return self._bytes(self.L.lx_get_merged_highest_before, ev)

    def _rows(self, f, evs):
        evs = _u32(evs)
        n = len(evs)
        off = np.zeros(n + 1, dtype=np.uint64)
        buf = np.zeros(max(8 * n * self.num_branches(), 1), dtype=np.uint8)   # >= every row (B >= V)
        self._chk(f(self.h, n, _p(evs, u32p), _p(off, u64p), _p(buf, u8p), len(buf)))
        b = buf.tobytes()
        return [b[off[i]:off[i + 1]] for i in range(n)]

    def rows_np(self, mode, evs):
        """Rows of many events in one call, as numpy arrays (offsets[n + 1],
        bytes): mode 0 HighestBefore, 1 LowestAfter, 2 merged HighestBefore."""
        f = (self.L.lx_get_highest_before_batch, self.L.lx_get_lowest_after_batch,
             self.L.lx_get_merged_highest_before_batch)[mode]
        evs = _u32(evs)
        n = len(evs)
        off = np.zeros(n + 1, dtype=np.uint64)
        self._chk(f(self.h, n, _p(evs, u32p), _p(off, u64p), None, 0))
        buf = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
        self._chk(f(self.h, n, _p(evs, u32p), _p(off, u64p), _p(buf, u8p), len(buf)))
        return off, buf[:int(off[-1])]

    def highest_before_batch(self, evs):
        """lx_get_highest_before_batch: list of byte rows."""
        return self._rows(self.L.lx_get_highest_before_batch, evs)

    def lowest_after_batch(self, evs):
        return self._rows(self.L.lx_get_lowest_after_batch, evs)

    def merged_highest_before_batch(self, evs):
        return self._rows(self.L.lx_get_merged_highest_before_batch, evs)

    def branch(self, ev):
        out = ctypes.c_uint32()
        self._chk(self.L.lx_get_event_branch_id(self.h, ev, ctypes.byref(out)))
        return out.value

    def branches_info(self):
        n = ctypes.c_uint32()
        self._chk(self.L.lx_get_branches_info(self.h, None, None, 0, ctypes.byref(n)))
        ls = np.zeros(n.value, dtype=np.uint32)
        cr = np.zeros(n.value, dtype=np.uint32)
        self._chk(self.L.lx_get_branches_info(self.h, _p(ls, u32p), _p(cr, u32p), n.value, ctypes.byref(n)))
        return ls, cr

    # column shards -------------------------------------------------------------
    def shard_range(self, shard):
        lo, hi = ctypes.c_uint32(), ctypes.c_uint32()
        self._chk(self.L.lx_shard_range(self.h, shard, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def shard_block(self, src, dst):
        n = ctypes.c_uint64()
        self._chk(self.L.lx_shard_block(self.h, src, dst, ctypes.byref(n)))
        return n.value

    def shard_of(self):
        r, c = ctypes.c_uint32(), ctypes.c_uint32()
        self._chk(self.L.lx_shard_of(self.h, ctypes.byref(r), ctypes.byref(c)))
        return r.value, c.value

    def shard_wire_bytes(self):
        """Bytes per LowestAfter entry in pack/unpack buffers (2 while every seq < 2^16, else 4)."""
        b = ctypes.c_uint32()
        self._chk(self.L.lx_shard_wire(self.h, ctypes.byref(b)))
        return b.value

    def shard_block_wire(self, dst):
        """Narrowest bytes per entry for this shard's outgoing block to ``dst`` (1, 2 or 4)."""
        b = ctypes.c_uint32()
        self._chk(self.L.lx_shard_block_wire(self.h, dst, ctypes.byref(b)))
        return b.value

    def la_pack_wire_dev(self, dst, out_ptr, width):
        self._chk(self.L.lx_la_pack_wire_dev(self.h, dst, out_ptr, width))

    def la_unpack_wire_dev(self, src, in_ptr, width):
        self._chk(self.L.lx_la_unpack_wire_dev(self.h, src, in_ptr, width))

    def la_pack_dev(self, dst, out_ptr):
        self._chk(self.L.lx_la_pack_dev(self.h, dst, out_ptr, None))

    def la_unpack_dev(self, src, in_ptr):
        self._chk(self.L.lx_la_unpack_dev(self.h, src, in_ptr, None))

    def la_own_dev(self):
        self._chk(self.L.lx_la_own_dev(self.h, None))

    # incremental LowestAfter exchange (lachesis_hip.shard.ShardedIndex.exchange)
    def shard_dirty(self):
        """Per branch the first seq of this shard's rows changed since the last
        committed exchange (LX_NONE: other shards' branches, unchanged ones)."""
        nb = self.num_branches()
        d = np.zeros(max(nb, 1), dtype=np.uint32)
        self._chk(self.L.lx_shard_dirty(self.h, nb, _p(d, u32p)))
        return d[:nb]

    def shard_dirty_set(self, dmin):
        d = np.ascontiguousarray(dmin, dtype=np.uint32)
        self._chk(self.L.lx_shard_dirty_set(self.h, len(d), _p(d, u32p)))

    def shard_dirty_commit(self):
        self._chk(self.L.lx_shard_dirty_commit(self.h))

    def last_stats(self):
        st = LxStats()
        self._chk(self.L.lx_last_stats(self.h, ctypes.byref(st)))
        return {"ms_assign": st.ms_assign, "ms_index": st.ms_index, "ms_marks": st.ms_marks}

    def walk_clock(self):
        """Shader clock of the last walk (lx_last_walk_clock): median / min / max
        MHz over its workgroups, the median workgroup's walk in ms, and per XCD
        the median clock and the slowest workgroup's walk."""
        out = (ctypes.c_float * 20)()
        self._chk(self.L.lx_last_walk_clock(self.h, out))
        return {"mhz_median": out[0], "mhz_min": out[1], "mhz_max": out[2], "walk_ms": out[3],
                "xcd_mhz": [round(out[4 + x], 1) for x in range(8)],
                "xcd_walk_ms_max": [round(out[12 + x], 2) for x in range(8)]}

    # ---- row-segment rank (options seg_count / seg_rank; lachesis_hip.rowseg drives the exchange)
    def rowseg_range(self):
        lo, hi = ctypes.c_uint32(), ctypes.c_uint32()
        self._chk(self.L.lx_rowseg_range(self.h, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def rowseg_of(self):
        """(seg_rank, seg_count) of the handle; (0, 1) for a whole index."""
        r, g = ctypes.c_uint32(), ctypes.c_uint32()
        self._chk(self.L.lx_rowseg_of(self.h, ctypes.byref(r), ctypes.byref(g)))
        return r.value, g.value

    def rowseg_bounds(self, G):
        b = np.zeros(G + 1, dtype=np.uint32)
        self._chk(self.L.lx_rowseg_bounds(self.h, _p(b, u32p)))
        return [int(x) for x in b]

    def row_bytes_max(self):
        """The longest row a getter can return (8 x max(branches, validators))."""
        b = ctypes.c_uint64()
        self._chk(self.L.lx_row_bytes_max(self.h, ctypes.byref(b)))
        return b.value

    def get_rows_dev(self, mode, n, ev_ptr, out_ptr, slot_bytes, len_ptr):
        """lx_get_rows_dev: rows of n device event ids into a device buffer
        (row i at out + i * slot_bytes, lengths as uint32; 0xFFFFFFFF: not held)."""
        self._chk(self.L.lx_get_rows_dev(self.h, mode, n, ev_ptr, out_ptr, slot_bytes, len_ptr))

    def rowseg_row_words(self):
        w = ctypes.c_uint32()
        self._chk(self.L.lx_rowseg_row_words(self.h, ctypes.byref(w)))
        return w.value

    def rowseg_request_cap(self):
        c = ctypes.c_uint32()
        self._chk(self.L.lx_rowseg_request_cap(self.h, ctypes.byref(c)))
        return c.value

    def rowseg_requests(self, ids_ptr, cap, G):
        c = np.zeros(G, dtype=np.uint32)
        self._chk(self.L.lx_rowseg_requests(self.h, ids_ptr, cap, _p(c, u32p)))
        return [int(x) for x in c]

    def rowseg_serve(self, n, ids_ptr, rows_ptr, ready_ptr):
        self._chk(self.L.lx_rowseg_serve(self.h, n, ids_ptr, rows_ptr, ready_ptr))

    def rowseg_receive(self, n, ids_ptr, rows_ptr, ready_ptr):
        left = ctypes.c_uint32()
        self._chk(self.L.lx_rowseg_receive(self.h, n, ids_ptr, rows_ptr, ready_ptr, ctypes.byref(left)))
        return left.value

    def rowseg_la(self, G):
        c = np.zeros(G, dtype=np.uint64)
        self._chk(self.L.lx_rowseg_la(self.h, _p(c, u64p)))
        return [int(x) for x in c]

    def rowseg_la_fetch(self, ptr):
        self._chk(self.L.lx_rowseg_la_fetch(self.h, ptr))

    def rowseg_la_apply(self, n, ptr):
        self._chk(self.L.lx_rowseg_la_apply(self.h, n, ptr))

    def rowseg_finish(self):
        self._chk(self.L.lx_rowseg_finish(self.h))

    # ForklessCause of any pair across row-segment ranks (lachesis_hip.rowseg.RowSegments.forkless_cause_dev)
    def rowseg_fc_route(self, n, qa_ptr, qb_ptr, ra_ptr, rb_ptr, perm_ptr, G):
        c = np.zeros(G, dtype=np.uint64)
        self._chk(self.L.lx_rowseg_fc_route(self.h, n, qa_ptr, qb_ptr, ra_ptr, rb_ptr, perm_ptr, _p(c, u64p)))
        return [int(x) for x in c]

    def rowseg_fc_need(self, m, ra_ptr, rb_ptr, ids_ptr, cap, G):
        c = np.zeros(G, dtype=np.uint64)
        self._chk(self.L.lx_rowseg_fc_need(self.h, m, ra_ptr, rb_ptr, ids_ptr, cap, _p(c, u64p)))
        return [int(x) for x in c]

    def rowseg_la_serve(self, n, ids_ptr, rows_ptr):
        self._chk(self.L.lx_rowseg_la_serve(self.h, n, ids_ptr, rows_ptr))

    def rowseg_la_store(self, n, ids_ptr, rows_ptr):
        self._chk(self.L.lx_rowseg_la_store(self.h, n, ids_ptr, rows_ptr))

    def rowseg_fc_unroute(self, n, perm_ptr, ans_ptr, out_ptr):
        self._chk(self.L.lx_rowseg_fc_unroute(self.h, n, perm_ptr, ans_ptr, out_ptr))

    def segment_stats(self):
        """Timings of the last segmented batch (option "segments")."""
        st = LxSegStats()
        self._chk(self.L.lx_last_segment_stats(self.h, ctypes.byref(st)))
        G = st.segments
        return {"segments": G, "first_event": list(st.first_event[:G + 1]), "partial": list(st.partial[:G]),
                "walk_ms": list(st.walk_ms[:G]), "partial_ms": st.partial_ms, "la_ms": st.la_ms,
                "one_launch": bool(st.one_launch)}

    def device_planes(self):
        hb, la, st = vp(), vp(), vp()
        stride = ctypes.c_uint32()
        self._chk(self.L.lx_device_planes(self.h, ctypes.byref(hb), ctypes.byref(la), ctypes.byref(stride),
                                          ctypes.byref(st)))
        return hb.value, la.value, stride.value, st.value


def shard_comm_unique_id():
    """RCCL communicator id (128 bytes) for ShardComm; create on one rank, share with all."""
    L = load_library()
    buf = (ctypes.c_uint8 * 128)()
    rc = L.lx_shard_comm_unique_id(buf)
    if rc != 0:
        raise LxError(rc, "ncclGetUniqueId failed (RCCL not loadable?)")
    return bytes(buf)


class ShardComm:
    """lx_shard_comm: the column-shard collectives issued by the library itself
    over RCCL on the index handle's stream (the path a Go caller binds;
    lachesis_hip.shard.ShardedIndex does the same through torch.distributed)."""

    def __init__(self, index, unique_id, nranks, rank):
        self.L = index.L
        self.ix = index
        self.c = vp()
        idb = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        rc = self.L.lx_shard_comm_create(index.h, idb, nranks, rank, ctypes.byref(self.c))
        if rc != 0:
            raise LxError(rc, "lx_shard_comm_create: " + self.L.lx_shard_comm_last_error(None).decode())

    def _chk(self, rc):
        if rc != 0:
            raise LxError(rc, self.L.lx_shard_comm_last_error(self.c).decode())

    def exchange(self):
        self._chk(self.L.lx_shard_exchange(self.c))

    def forkless_cause_dev(self, n, a_ptr, b_ptr, out_ptr):
        self._chk(self.L.lx_forkless_cause_sharded_dev(self.c, n, a_ptr, b_ptr, out_ptr))

    def fc_undecided(self):
        """Queries the last forkless_cause_dev sent to every shard (lx_shard_fc_undecided)."""
        u = ctypes.c_uint64()
        self._chk(self.L.lx_shard_fc_undecided(self.c, ctypes.byref(u)))
        return u.value

    def get_rows_dev(self, mode, n, ev_ptr, out_ptr, slot_bytes, len_ptr):
        """Whole vector getter rows on column shards (lx_shard_get_rows, collective)."""
        self._chk(self.L.lx_shard_get_rows(self.c, mode, n, ev_ptr, out_ptr, slot_bytes, len_ptr))

    def close(self):
        if self.c:
            self.L.lx_shard_comm_destroy(self.c)
            self.c = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RowsegComm(ShardComm):
    """lx_rowseg_comm_create / lx_rowseg_exchange: the row-segment exchanges
    issued by the library over RCCL (the Go path; lachesis_hip.rowseg runs the
    same protocol through torch.distributed).  The index has seg_count =
    nranks, seg_rank = rank."""

    def __init__(self, index, unique_id, nranks, rank):
        self.L = index.L
        self.ix = index
        self.c = vp()
        idb = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        rc = self.L.lx_rowseg_comm_create(index.h, idb, nranks, rank, ctypes.byref(self.c))
        if rc != 0:
            raise LxError(rc, "lx_rowseg_comm_create: " + self.L.lx_shard_comm_last_error(None).decode())

    def exchange(self):
        st = np.zeros(4, dtype=np.uint64)
        self._chk(self.L.lx_rowseg_exchange(self.c, _p(st, u64p)))
        return {"row_rounds": int(st[0]), "rows_received": int(st[1]), "la_sent": int(st[2]),
                "la_received": int(st[3])}

    def forkless_cause_dev(self, n, a_ptr, b_ptr, out_ptr):
        """ForklessCause of any pairs of the epoch (lx_rowseg_forkless_cause):
        queries to owner(a), remote LowestAfter rows to it, answers back."""
        st = np.zeros(4, dtype=np.uint64)
        self._chk(self.L.lx_rowseg_forkless_cause(self.c, n, a_ptr, b_ptr, out_ptr, _p(st, u64p)))
        return {"routed_away": int(st[0]), "answered": int(st[1]), "rows_received": int(st[2]),
                "rows_sent": int(st[3])}

    def get_rows_dev(self, mode, n, ev_ptr, out_ptr, slot_bytes, len_ptr):
        """The vector getter rows of n device ids of any rank
        (lx_rowseg_get_rows, collective): row i at out + i * slot_bytes."""
        self._chk(self.L.lx_rowseg_get_rows(self.c, mode, n, ev_ptr, out_ptr, slot_bytes, len_ptr))
