"""The column-shard LowestAfter exchange driver on CPU (the RCCL
path's send/recv schedule had never run with more than one rank).

lx_shard_exchange (csrc/lx_shard_rccl.cpp) is lx::shard_exchange_run
(csrc/lx_shard_exchange.h) over RCCL; tests/csrc/shard_fake.cpp runs the same
driver with G threads over an in-process transport and a model of each rank's
index, and checks every exchanged entry, 4-byte aligned block offsets on both
sides, and the byte-wire fallback / retry schedule.  The layout function is
also checked against the library's exported lx_shard_exchange_layout and the
Python ShardedIndex's shard_layout."""

import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "lachesis-base_amd", "build")
u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)


@pytest.fixture(scope="module")
def fake():
    L = ctypes.CDLL(os.path.join(BUILD, "libshard_fake.so"))
    L.lx_fake_shard_exchange.restype = ctypes.c_int
    L.lx_fake_shard_exchange.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                                 u64p, ctypes.c_char_p, ctypes.c_uint32]
    L.lx_fake_shard_layout.restype = None
    L.lx_fake_shard_layout.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u64p, u32p, u64p]
    return L


@pytest.mark.parametrize("G,V,N", [(2, 16, 200), (3, 13, 150), (5, 40, 300), (7, 30, 240), (8, 64, 400),
                                   (8, 12, 100)])
@pytest.mark.parametrize("skew", [0, 1])
def test_exchange_driver_fake_transport(fake, G, V, N, skew):
    """G ranks exchange 12 times over a drifting epoch (uneven creator ranges,
    ranks without columns at G=8/V=12, odd entry counts); every rank ends with
    exactly its columns of every row."""
    stats = np.zeros(3, dtype=np.uint64)
    err = ctypes.create_string_buffer(512)
    rc = fake.lx_fake_shard_exchange(G, V, N, 1000 * G + V, 12, skew, stats.ctypes.data_as(u64p), err, 512)
    assert rc == 0, err.value.decode()
    assert stats[1] > 0 and stats[2] > 0          # the byte wire was used, entries moved
    if skew:
        assert stats[0] > 0                       # and a block fell back to the wide width


def test_layout_matches_library_and_python(fake):
    """One layout for all three implementations: 4-byte aligned block starts."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "lachesis-base_amd"))
    from lachesis_hip.shard import shard_layout
    lib = ctypes.CDLL(os.path.join(BUILD, "liblachesis_hip.so"))
    lib.lx_shard_exchange_layout.restype = ctypes.c_int
    lib.lx_shard_exchange_layout.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u64p, u32p, u64p]
    rng = np.random.default_rng(1)
    for _ in range(200):
        G = int(rng.integers(1, 9))
        r = int(rng.integers(0, G))
        ent = rng.integers(0, 50, G).astype(np.uint64)
        wid = rng.choice([1, 2, 4], G).astype(np.uint32)
        a = np.zeros(G + 1, dtype=np.uint64)
        b = np.zeros(G + 1, dtype=np.uint64)
        fake.lx_fake_shard_layout(G, r, ent.ctypes.data_as(u64p), wid.ctypes.data_as(u32p), a.ctypes.data_as(u64p))
        assert lib.lx_shard_exchange_layout(G, r, ent.ctypes.data_as(u64p), wid.ctypes.data_as(u32p),
                                            b.ctypes.data_as(u64p)) == 0
        c = shard_layout(G, r, [int(x) for x in ent], [int(x) for x in wid])
        assert list(a) == list(b) == c
        assert all(x % 4 == 0 for x in c)
        for q in range(G):
            assert c[q + 1] - c[q] >= (0 if q == r else int(ent[q]) * int(wid[q]))
