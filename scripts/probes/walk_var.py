"""(Ran once against an experimental build with the option `walk_var`; the
option and its kernel variants were removed after this measurement --
profiles/r04/walker/)

C3 walk with the shipped default options (two side-by-side segments of
8-column slices) under each compute / drain wave split of the 16-wave
8-column walker (option walk_var: 0 = 8 / 7 shipped, 1 = 10 / 5, 2 = 11 / 4,
3 = 9 / 6), alternated twice; planes of each variant compared with the
shipped one on the device."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V, epv = int(os.environ.get("WT_V", "1000")), int(os.environ.get("WT_EPV", "10000"))
d = lx.tools.gen_dag(V, epv, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(V)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipMemcpy.restype = ctypes.c_int
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def step(ix):
    ix.reset(w)
    ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
    ix.sync()
    return max(ix.segment_stats()["walk_ms"])


def planes_equal(a, b, cols, chunk_rows=1 << 18):
    pa, pb = a.device_planes(), b.device_planes()
    stride = pa[2]
    ba = torch.empty((chunk_rows, stride), dtype=torch.int32, device=dev)
    bb = torch.empty_like(ba)
    for k in (0, 1):
        for lo in range(0, N, chunk_rows):
            m = min(chunk_rows, N - lo)
            assert hip.hipMemcpy(ba.data_ptr(), pa[k] + lo * stride * 4, m * stride * 4, 3) == 0
            assert hip.hipMemcpy(bb.data_ptr(), pb[k] + lo * stride * 4, m * stride * 4, 3) == 0
            torch.cuda.synchronize()
            if not torch.equal(ba[:m, :cols], bb[:m, :cols]):
                return False
    return True


base = lx.Index(event_capacity=N)
other = lx.Index(event_capacity=N)
step(base)
VARS = [int(x) for x in os.environ.get("WV", "0 3 4 5").split()]
res = {v: [] for v in VARS}
for rnd in range(2):
    for v in VARS:
        other.set_option(os.environ.get("WOPT", "walk_var"), v)
        step(other)
        res[v] += [step(other), step(other)]
        print(json.dumps({"round": rnd, "walk_var": v, "walk_ms": res[v][-2:]}), flush=True)
        if rnd == 0:
            print(json.dumps({"walk_var": v, "planes_equal_shipped": planes_equal(base, other, base.num_branches())}),
                  flush=True)
print(json.dumps({"walk_ms_median": {str(v): float(np.median(x)) for v, x in res.items()}}))
