"""Level-fed Add throughput on C3 (tools/lx_latency.cpp lx_bench_feed_levels):
levels added one lx_add_batch + lx_flush each (direct) or through lx_batcher,
with the host time split.  For rocprofv3:
    rocprofv3 --kernel-trace --stats -d DIR -- python3 scripts/feed_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]

import numpy as np  # noqa: E402
import lachesis_hip as lx  # noqa: E402


def main():
    V, epv = 1000, int(os.environ.get("EPV", "1300"))
    w = np.array([(1 << 20) // (i + 1) for i in range(V)], dtype=np.uint32)
    d = lx.tools.gen_dag(V, epv, 10, 0, 0, seed=1)
    lx.load_library()
    L = ctypes.CDLL(os.path.join(ROOT, "lachesis-base_amd", "build", "liblx_bench.so"))
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    f = L.lx_bench_feed_levels
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p, u64p, u32p, ctypes.c_uint64,
                  ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_uint32]
    res = {}
    for mode, name in ((0, "direct"), (1, "batcher")):
        out = (ctypes.c_double * 8)()
        err = ctypes.create_string_buffer(512)
        rc = f(0, V, w.ctypes.data_as(u32p), len(d), d.creator.ctypes.data_as(u32p), d.seq.ctypes.data_as(u32p),
               d.poff.ctypes.data_as(u64p), d.par.ctypes.data_as(u32p), 200_000, 1_000_000, mode, out, err, 512)
        assert rc == 0, err.value
        res[name] = {"events_per_sec": out[0], "events": out[1], "levels": out[2], "add_s": out[3],
                     "batcher_s": out[4], "final_sync_s": out[5]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
