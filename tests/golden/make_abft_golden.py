"""Expected abft results for the BASELINE configs at full size, computed by the
C abft restatement (oracle/csrc/abft_oracle.c, checked against the Python
restatement by tests/test_oracle_c.py, which tests/test_abft_oracle.py pins to
the reference's abft tests).

    python tests/golden/make_abft_golden.py [c4|c5]...

Writes ``tests/golden/abft_<cfg>.npz`` (plain arrays, no pickles):
frames (per event, Add order), roots_per_frame, and the blocks: frame,
atropos, cheaters (CSR), confirmed events (ApplyEvent order, CSR).  The DAGs
come from the splitmix64 tdag generator (lachesis_hip.tools.gen_dag, identical
to oracle/tdag.py), so the GPU tests regenerate them instead of storing them.
"""

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]

# name: (V, events per validator, parents, cheaters, forks, weights, seed)
CONFIGS = {
    "c4": (100, 1000, 10, 10, 10, "equal", 1),
    "c5": (1000, 50, 10, 0, 0, "zipf", 1),
}


def weights_for(V, kind):
    if kind == "zipf":
        return [(1 << 20) // (i + 1) for i in range(V)]
    return [1] * V


def main(names):
    from lachesis_hip import tools
    from oracle import corc
    for name in names:
        V, epn, P, ch, fk, wk, seed = CONFIGS[name]
        d = tools.gen_dag(V, epn, P, cheaters=ch, forks=fk, seed=seed)
        w = weights_for(V, wk)
        c = corc.AbftOracle(w)
        t0 = time.time()
        rc, consumed, frames = c.process_batch(d.creator, d.seq, d.poff, d.par)
        dt = time.time() - t0
        assert rc == 0 and consumed == len(d), (rc, consumed)
        roots = [len(c.frame_roots(f)) for f in range(int(frames.max()) + 2)]
        b = c.blocks
        ch_off = np.cumsum([0] + [len(x[3]) for x in b]).astype(np.uint64)
        cf_off = np.cumsum([0] + [len(x[4]) for x in b]).astype(np.uint64)
        np.savez_compressed(
            os.path.join(HERE, "abft_%s.npz" % name),
            config=np.array([V, epn, P, ch, fk, seed], dtype=np.uint64),
            weights=np.array(w, dtype=np.uint32),
            frames=frames.astype(np.uint32),
            roots_per_frame=np.array(roots, dtype=np.uint32),
            block_frame=np.array([x[1] for x in b], dtype=np.uint32),
            block_atropos=np.array([x[2] for x in b], dtype=np.uint32),
            cheaters_off=ch_off,
            cheaters=np.array([v for x in b for v in x[3]], dtype=np.uint32),
            confirmed_off=cf_off,
            confirmed=np.array([v for x in b for v in x[4]], dtype=np.uint32),
            oracle_seconds=np.array([dt]))
        print("%s: %d events, %d blocks, max frame %d, oracle %.1fs (%.0f events/s)"
              % (name, len(d), len(b), frames.max(), dt, len(d) / dt))


if __name__ == "__main__":
    main(sys.argv[1:] or list(CONFIGS))
