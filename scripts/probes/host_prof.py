"""Where the host time of level-fed Add goes (the direct mode of
lx_bench_feed_levels on C3 levels): the build_hprof library (make hprof)
counts TSC cycles per section of lx_add_batch's small path and of
flush_pending.  Prints one JSON object: ns per event of each section."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]

import numpy as np  # noqa: E402
from lachesis_hip import tools  # noqa: E402

NAMES = ["validate", "pre_loop", "main_loop", "post_loop", "flush_image", "flush_hip", "add_batch_total", "-", "-", "-", "-", "-", "f_stage_slot", "f_memcpy_ev", "f_sort_meta", "f_pl_old_rest"]


def main():
    bdir = os.path.join(ROOT, "lachesis-base_amd", sys.argv[1] if len(sys.argv) > 1 else "build_hprof")
    V, epv = 1000, int(os.environ.get("EPV", "1300"))
    w = np.array([(1 << 20) // (i + 1) for i in range(V)], dtype=np.uint32)
    d = tools.gen_dag(V, epv, 10, 0, 0, seed=1)
    B = ctypes.CDLL(os.path.join(bdir, "liblx_bench.so"))
    L = ctypes.CDLL(os.path.join(bdir, "liblachesis_hip.so"))
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    f = B.lx_bench_feed_levels
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p, u64p, u32p, ctypes.c_uint64,
                  ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_uint32]
    prof = getattr(L, "lx_host_prof", None)
    res = []
    for rep in range(3):
        hp = (ctypes.c_uint64 * 16)()
        if prof:
            prof(hp, 1)
        out = (ctypes.c_double * 8)()
        err = ctypes.create_string_buffer(512)
        rc = f(0, V, w.ctypes.data_as(u32p), len(d), d.creator.ctypes.data_as(u32p), d.seq.ctypes.data_as(u32p),
               d.poff.ctypes.data_as(u64p), d.par.ctypes.data_as(u32p), 200_000, 1_000_000, 0, out, err, 512)
        assert rc == 0, err.value
        r = {"events_per_sec": out[0], "events": out[1], "add_s": out[3]}
        if prof:
            prof(hp, 1)
            # the counters include the history batch and the warm-up levels; the
            # TSC rate from the timed add_s is not needed: report cycles per event
            ev = max(1, hp[10])
            r["cycles_per_event"] = {n: hp[k] / ev for k, n in enumerate(NAMES) if n != "-"}
            r["small_events"] = int(hp[10])
            r["small_calls"] = int(hp[11])
            r["flushes"] = int(hp[9])
        res.append(r)
    print(json.dumps({"lib": bdir, "runs": res}))


if __name__ == "__main__":
    main()
