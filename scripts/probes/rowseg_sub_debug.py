"""Debug: row-segment ranks with sub-segments on a fork DAG (native driver over
the in-process transport): mismatching LowestAfter entries against a whole index."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import lachesis_hip as lx  # noqa: E402

lx.load_library()
L = ctypes.CDLL(os.path.join(ROOT, "lachesis-base_amd", "build", "librowseg_fake.so"))
L.lx_fake_rowseg_exchange.restype = ctypes.c_int
L.lx_fake_rowseg_exchange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_uint32]
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipMemcpy.restype = ctypes.c_int
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def planes(ix, N):
    ix.sync()
    hb, la, stride, _ = ix.device_planes()
    out = []
    for p in (hb, la):
        a = np.empty((N, stride), dtype=np.uint32)
        assert hip.hipMemcpy(a.ctypes.data, p, a.nbytes, 2) == 0
        out.append(a)
    return out


V, epv, P, ch, fk, seed = 28, 60, 6, 5, 6, 3
d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
N = len(d)
rng = np.random.default_rng(seed)
weights = [int(x) for x in rng.integers(1, 40, V)]
ref = lx.Index(device=0, options={"small_max": 0})
ref.reset(weights)
br = ref.add_batch(d.creator, d.seq, d.poff, d.par, want_branches=True)
B = ref.num_branches()
rhb, rla = planes(ref, N)
print("N", N, "B", B, "V", V)
rowof = {}
for x in range(N):
    rowof[(int(br[x]), int(d.seq[x]))] = x
seg2 = lx.Index(device=0, options={"small_max": 0, "segments": 4})
seg2.reset(weights)
seg2.add_batch(d.creator, d.seq, d.poff, d.par)
shb, sla = planes(seg2, N)
print("single-GPU segments=4:", seg2.segment_stats().get("first_event"), "hb bad", int((shb[:, :B] != rhb[:, :B]).sum()),
      "la bad", int((sla[:, :B] != rla[:, :B]).sum()))
seg2.close()
for world, sub in ((2, 1), (2, 2), (2, 2), (2, 3), (3, 2)):
    ranks = []
    for r in range(world):
        ix = lx.Index(device=0, options={"seg_count": world, "seg_rank": r, "small_max": 0, "seg_sub": sub})
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ranks.append(ix)
    hs = (ctypes.c_void_p * world)(*[ix.h for ix in ranks])
    stats = (ctypes.c_uint64 * (4 * world))()
    err = ctypes.create_string_buffer(512)
    rc = L.lx_fake_rowseg_exchange(hs, world, stats, err, 512)
    print("world", world, "sub", sub, "rc", rc, err.value.decode(), list(stats))
    for r, ix in enumerate(ranks):
        lo, hi = ix.rowseg_range()
        st = ix.segment_stats()
        hb, la = planes(ix, N)
        bad_hb = np.argwhere(hb[lo:hi, :B] != rhb[lo:hi, :B])
        bad = np.argwhere(la[lo:hi, :B] != rla[lo:hi, :B])
        print(" rank", r, "rows", lo, hi, "segs", st.get("segments"), "first", st.get("first_event"),
              "partial", st.get("partial"), "one_launch", st.get("one_launch"),
              "hb bad", len(bad_hb), "la bad", len(bad))
        if len(bad):
            rows = sorted(set(int(lo + i) for i, _ in bad))
            print("   bad rows", len(rows), rows[:40], "...", rows[-10:])
            print("   bad cols", sorted(set(int(c) for _, c in bad)))
        for (i, c) in bad[:40]:
            x = lo + i
            g, w = int(la[x, c]), int(rla[x, c])
            print("   row", x, "br", int(br[x]), "seq", int(d.seq[x]), "col", c, "got", g, "(row", rowof.get((int(c), g)),
                  ") want", w, "(row", rowof.get((int(c), w)), ")")
    for ix in ranks:
        ix.close()
