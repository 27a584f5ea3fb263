"""(Ran once against an experimental build with the option `walk_lean`; the
option and its kernel variants were removed after this measurement --
profiles/r04/walker/)

C3 walk: the shipped default (two side-by-side segments of 8-column slices,
one walk per CU) against the LDS-lean 8-column walker (option walk_lean: two
walks per CU) at G = 2, 3, 4 side-by-side segments (options segments / cpw);
the lean G = 4 planes are compared with the default's on the device."""
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


def run(opts, reps=4):
    ix = lx.Index(event_capacity=N, options=opts)
    ks, walks = [], []
    for r in range(reps):
        ix.reset(w)
        ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
        ix.sync()
        ks.append(ix.last_stats()["ms_index"])
        st = ix.segment_stats()
        walks.append(max(st["walk_ms"]) if st["segments"] else None)
    st = ix.segment_stats()
    return ix, {"opts": opts, "ms_index_median": float(np.median(ks[1:])), "walk_ms": walks[1:],
                "segments": st["segments"], "one_launch": st["one_launch"], "partial": st["partial"],
                "partial_ms": st["partial_ms"], "la_ms": st["la_ms"]}


def planes_equal(a, b, cols, chunk_rows=1 << 18):
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    pa, pb = a.device_planes(), b.device_planes()
    stride = pa[2]
    assert pb[2] == stride
    ba = torch.empty((chunk_rows, stride), dtype=torch.int32, device=dev)
    bb = torch.empty_like(ba)
    for k in (0, 1):
        for lo in range(0, N, chunk_rows):
            m = min(chunk_rows, N - lo)
            assert hip.hipMemcpy(ba.data_ptr(), pa[k] + lo * stride * 4, m * stride * 4, 3) == 0
            assert hip.hipMemcpy(bb.data_ptr(), pb[k] + lo * stride * 4, m * stride * 4, 3) == 0
            torch.cuda.synchronize()
            if not torch.equal(ba[:m, :cols], bb[:m, :cols]):
                return {"plane": k, "rows": lo}
    return None


base, r0 = run(None)
print(json.dumps({"default": r0}), flush=True)
res = {"default": r0}
for G in (2, 3, 4):
    ix, r = run({"segments": G, "cpw": 8, "walk_lean": 1})
    res["lean_g%d" % G] = r
    print(json.dumps({"lean_g%d" % G: r}), flush=True)
    if G == 4:
        bad = planes_equal(base, ix, base.num_branches())
        res["lean_g4_planes_equal_default"] = bad is None
        print(json.dumps({"lean_g4_planes_equal_default": bad is None, "first_bad": bad}), flush=True)
    ix.close()
base.close()
print(json.dumps(res))
