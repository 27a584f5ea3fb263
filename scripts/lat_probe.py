"""Per-call probe for rocprofv3 --hip-trace: single-event Adds (Process and
Build patterns), per-call ForklessCause and getters on a V=1000 epoch.
Usage: rocprofv3 --hip-trace --kernel-trace --stats -d DIR -- python3 scripts/lat_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]

import numpy as np  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V = 1000
w = [(1 << 20) // (i + 1) for i in range(V)]
d = lx.tools.gen_dag(V, 30, 10, seed=1)
N = len(d)
H = 20_000
ix = lx.Index(event_capacity=N)
ix.reset(w)
ix.add_batch(d.creator[:H], d.seq[:H], d.poff[:H + 1], d.par)
ix.flush()
ix.sync()
reps = int(os.environ.get("REPS", "1000"))
t0 = time.perf_counter()
for i in range(H, H + reps):
    ix.add_batch(d.creator[i:i + 1], d.seq[i:i + 1], d.poff[i:i + 2], d.par)
    ix.flush()
ix.sync()
t1 = time.perf_counter()
i = H + reps
for _ in range(reps):
    ix.add_batch(d.creator[i:i + 1], d.seq[i:i + 1], d.poff[i:i + 2], d.par)
    ix.drop_not_flushed()
ix.sync()
t2 = time.perf_counter()
a = np.array([i - 1], dtype=np.uint32)
b = np.array([5], dtype=np.uint32)
for _ in range(reps):
    ix.forkless_cause_batch(a, b)
t3 = time.perf_counter()
for _ in range(reps):
    ix.merged_highest_before(i - 1)
t4 = time.perf_counter()
print("python-side us/call: add+flush %.1f  add+drop %.1f  fc1 %.1f  merged %.1f" % (
    (t1 - t0) / reps * 1e6, (t2 - t1) / reps * 1e6, (t3 - t2) / reps * 1e6, (t4 - t3) / reps * 1e6))
