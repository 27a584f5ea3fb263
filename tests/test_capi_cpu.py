"""C-ABI library checks that need no GPU: it loads, exports every symbol the
public header declares, and the synthetic-DAG tools match the oracle's
generator bit for bit."""

import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import tdag


def header_symbols():
    src = ""
    for name in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if name.endswith(".h"):
            src += open(os.path.join(ROOT, "include", name)).read()
    # entry points (not the callback members of lx_abft_callbacks: "(*name)(")
    return sorted(set(re.findall(r"\b(lx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from lachesis_hip import capi
    L = capi.load_library()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    bound = {n for n, _, _ in capi.SIGNATURES}
    assert bound == set(syms), "ctypes table out of sync with the header"


def test_library_is_gfx950_code_object():
    from lachesis_hip import capi
    data = open(capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_cpu_fallback_without_gpu():
    """On a machine without a GPU the product fails loudly (no CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from lachesis_hip import Index, LxError
    with pytest.raises(LxError):
        Index(device=0)


@pytest.mark.parametrize("shape", [(4, 20, 3, 0, 0, 1), (6, 15, 4, 2, 5, 9), (10, 10, 4, 10, 3, 3), (1, 12, 1, 1, 3, 5)])
def test_tools_generator_matches_oracle(shape):
    from lachesis_hip import tools
    n, ev, p, ch, fk, seed = shape
    d = tools.gen_dag(n, ev, p, ch, fk, seed)
    _, evs = tdag.rand_fork_dag(n, ev, p, cheaters=ch, forks_count=fk, seed=seed)
    assert len(d) == len(evs)
    for i, e in enumerate(evs):
        assert d.creator[i] == (e.creator - 1)
        assert d.seq[i] == e.seq
        assert d.lamport[i] == e.lamport
        assert list(d.par[d.poff[i]:d.poff[i + 1]]) == e.parents


def test_fc_query_window():
    from lachesis_hip import tools
    d = tools.gen_dag(8, 50, 4, seed=2)
    qa, qb = tools.fc_queries(d.lamport, 5000, window=16, seed=3)
    la, lb = d.lamport[qa].astype(np.int64), d.lamport[qb].astype(np.int64)
    assert np.all(lb <= la) and np.all(lb >= la - 16)


def test_vecfc_config_api():
    """vecfc.DefaultConfig / LiteConfig (vecfc/index.go:52-66) with cachescale
    rounding (utils/cachescale/ratio.go:18-25): LiteConfig's HighestBefore
    cache is 1639 bytes."""
    import lachesis_hip as lx
    c = lx.default_config()
    assert (c.caches.forkless_cause_pairs, c.caches.highest_before_seq_size, c.caches.lowest_after_seq_size) == \
        (20000, 160 * 1024, 160 * 1024)
    c = lx.lite_config()
    assert (c.caches.forkless_cause_pairs, c.caches.highest_before_seq_size) == (200, 1639)
    assert lx.Ratio(3, 2).U64(10) == 7
