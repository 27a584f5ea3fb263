"""The reference caller's call sequence on the index for configs[4] (C5),
computed by the C abft restatement (oracle/csrc/abft_oracle.c, TEST
INFRASTRUCTURE) in Process mode with the events' claimed frames
(tests/golden/abft_c5.npz) and the reference's ForklessCause LRU
(DefaultConfig, 20000 pairs, vecfc/index.go:52-61):

    python tests/golden/make_dropin_golden.py

Writes tests/golden/dropin_c5.json: the trace hash of abft_oracle.c's abo_trace
(Add / ForklessCause / Flush / DropNotFlushed records, in order), the call
counts, and the oracle's wall time.  tests/test_gpu_dropin.py replays the same
epoch through the HIP library with lachesis_hip.dropin and compares."""

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]


def main():
    from lachesis_hip import tools
    from oracle import corc
    z = np.load(os.path.join(HERE, "abft_c5.npz"))
    V, epv, P = 1000, 50, 10
    d = tools.gen_dag(V, epv, P, 0, 0, seed=1)
    w = [int(x) for x in z["weights"]]
    o = corc.AbftOracle(w)
    o.set_fc_cache(20000)
    t0 = time.time()
    rc, c, frames = o.process_batch(d.creator, d.seq, d.poff, d.par, z["frames"])
    dt = time.time() - t0
    assert rc == 0 and c == len(d) and np.array_equal(frames, z["frames"])
    tr = o.trace()
    out = dict(tr, events=len(d), lru_pairs=20000, oracle_seconds=dt,
               blocks=len(o.blocks), hash=str(tr["hash"]))
    with open(os.path.join(HERE, "dropin_c5.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
