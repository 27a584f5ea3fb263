"""(Needs the 16-column walker of commit 85cab53, measured slower and removed
from the library: profiles/r05/cpw16/)

C3 walk on 16-column slices (three 16-B slot units, 63 slices at V = 1000,
four Add-order segments side by side on 256 CUs) against the shipped
12-column form (three segments), same box, alternating A B A B; the planes
of the two forms compared on the device (both must equal the 4-column walk
that the parity tests pin to the oracle)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V, epv = 1000, 10000
d = lx.tools.gen_dag(V, epv, 10, seed=1)
w = [(1 << 20) // (i + 1) for i in range(V)]
variants = [("cpw12_auto", {}), ("cpw16_seg4", {"cpw": 16, "segments": 4})]
for extra in sys.argv[1:]:
    variants.append((extra, json.loads(extra)))
res = {k: [] for k, _ in variants}
ixs = {k: lx.Index(options=dict(o), event_capacity=len(d)) for k, o in variants}
for rep in range(4):
    for k, _ in variants:
        ix = ixs[k]
        ix.reset(w)
        ix.sync()
        t0 = time.perf_counter()
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ix.sync()
        st = ix.last_stats()
        sg = ix.segment_stats()
        res[k].append({"step_ms": (time.perf_counter() - t0) * 1e3, "index_ms": st["ms_index"],
                       "walk_ms": sg["walk_ms"][:sg["segments"]], "segments": sg["segments"],
                       "partial": int(sum(sg["partial"])), "partial_ms": sg["partial_ms"], "la_ms": sg["la_ms"]})
        print(json.dumps({k: res[k][-1]}), flush=True)
# planes equal (chunked compare on the device)
names = [k for k, _ in variants]
ref = ixs[names[0]]
hb0, la0, stride, _ = ref.device_planes()
N = len(d)
same = {}
for k in names[1:]:
    hb1, la1, s1, _ = ixs[k].device_planes()
    assert s1 == stride
    ok = True
    for p0, p1 in ((hb0, hb1), (la0, la1)):
        for lo in range(0, N, 500_000):
            n = min(500_000, N - lo) * stride
            a = torch.empty(n, dtype=torch.int32, device="cuda")
            b = torch.empty(n, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            lx.capi.load_library()
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so.7")
            hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            assert hip.hipMemcpy(a.data_ptr(), p0 + 4 * lo * stride, 4 * n, 3) == 0
            assert hip.hipMemcpy(b.data_ptr(), p1 + 4 * lo * stride, 4 * n, 3) == 0
            ok = ok and bool(torch.equal(a, b))
    same[k] = ok
summary = {k: {"index_ms_median": float(np.median([r["index_ms"] for r in res[k][1:]])),
               "step_ms_median": float(np.median([r["step_ms"] for r in res[k][1:]]))} for k in names}
print(json.dumps({"summary": summary, "planes_equal_to_" + names[0]: same}), flush=True)
