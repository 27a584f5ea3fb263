"""The resident row server behind the single-row getters (k_get_server,
csrc/lx_persist.hip): GetHighestBefore / GetLowestAfter
/ GetMergedHighestBefore (vecfc/store_vectors.go:26-51,
vecengine/index.go:235-250) answered by a one-wave kernel that stays resident
between calls must give the oracle's bytes -- also for LowestAfter rows that
change under it as events are added (rows written by kernels on another
queue), across its idle exit and relaunch, across buffer growth (new
arguments), and with the option off.  The mechanics tests force the server on
(get_server = 2): other tests' handles may be alive in this process, and the
default (1) uses the server only while one handle exists.  The device refuses
an event outside the handle's rows by itself (an error, never a fault)."""

import time

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


def _oracle(d, w):
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    return o


@pytest.mark.parametrize("shape", [(12, 40, 5, 4, 8, 21), (100, 12, 10, 10, 10, 11), (1000, 3, 8, 0, 0, 5)])
def test_server_rows_equal_oracle(lx, shape):
    n, ev, p, ch, fk, seed = shape
    d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
    w = sorted((int(x) for x in np.random.default_rng(seed).integers(1, 9, n)), reverse=True)
    o = _oracle(d, w)
    ix = lx.Index(options={"get_server": 2})
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    N = len(d)
    evs = np.random.default_rng(seed).permutation(N)[:400]
    for e in evs:
        e = int(e)
        assert ix.highest_before(e) == o.hb(e), e
        assert ix.lowest_after(e) == o.la(e), e
        assert ix.merged_highest_before(e) == o.merged_hb(e), e
    st = ix.get_server_stats()
    assert st["served"] >= 3 * len(evs) - 3, st       # the server answered (not the launch path)
    assert st["launches"] >= 1, st
    ix.close()


def test_server_sees_rows_added_meanwhile(lx):
    """Events added one at a time between single-row calls: the server (its own
    queue) must read the LowestAfter rows the Add kernels just changed."""
    d = lx.tools.gen_dag(24, 30, 6, 0, 0, 3)
    w = [1 + (i % 5) for i in range(24)]
    N = len(d)
    ix = lx.Index(options={"get_server": 2})
    ix.reset(w)
    half = N // 2
    ix.add_batch(d.creator[:half], d.seq[:half], d.poff[:half + 1], d.par)
    rng = np.random.default_rng(1)
    for e in range(half, N):
        p0, p1 = int(d.poff[e]), int(d.poff[e + 1])
        ix.add(int(d.creator[e]), int(d.seq[e]), [int(x) for x in d.par[p0:p1]])
        ix.sync()
        probe = [int(x) for x in rng.integers(0, e + 1, 3)] + [int(x) for x in d.par[p0:p1]]
        for b in probe:
            assert ix.lowest_after(b) == ix.lowest_after_batch([b])[0], (e, b)
            assert ix.highest_before(b) == ix.highest_before_batch([b])[0], (e, b)
    o = _oracle(d, w)
    for e in range(N):
        assert ix.lowest_after(e) == o.la(e), e
        assert ix.merged_highest_before(e) == o.merged_hb(e), e
    assert ix.get_server_stats()["served"] > 0
    ix.close()


def test_server_idle_exit_relaunch_and_growth(lx):
    d = lx.tools.gen_dag(40, 50, 6, 3, 4, 9)
    w = [1 + (i % 7) for i in range(40)]
    N = len(d)
    o = _oracle(d, w)
    ix = lx.Index(event_capacity=64, options={"get_server": 2})     # the planes grow (new pointers) while the server lives
    ix.reset(w)
    cut = N // 3
    ix.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par)
    ix.sync()
    ix.highest_before(0)
    launches0 = ix.get_server_stats()["launches"]
    time.sleep(0.01)                     # > its 250 us idle limit: it has left
    assert ix.highest_before(1) is not None
    assert ix.get_server_stats()["launches"] > launches0
    ix.add_batch(d.creator[cut:], d.seq[cut:], d.poff[cut:] - d.poff[cut], d.par[d.poff[cut]:])
    ix.sync()
    for e in range(0, N, 7):
        assert ix.highest_before(e) == o.hb(e), e
        assert ix.lowest_after(e) == o.la(e), e
        assert ix.merged_highest_before(e) == o.merged_hb(e), e
    # option off: every call launches, same bytes
    ix.set_option("get_server", 0)
    f0 = ix.get_server_stats()["fallbacks"]
    for e in range(1, N, 11):
        assert ix.lowest_after(e) == o.la(e), e
    assert ix.get_server_stats()["fallbacks"] > f0
    ix.close()


def test_server_leaves_for_device_sync(lx):
    """A device-wide synchronization right after a getter waits for the server's
    idle exit only (250 us), never for its 0.5 s deadline."""
    import torch
    d = lx.tools.gen_dag(16, 20, 4, 0, 0, 2)
    ix = lx.Index()
    ix.reset([1] * 16)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    worst = 0.0
    for e in range(0, len(d), 13):
        ix.highest_before(e)
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        worst = max(worst, time.perf_counter() - t0)
    assert worst < 0.05, worst
    ix.close()


def test_server_idle_boundary_race(lx):
    """Requests spaced around the server's 250 us idle limit: some arrive as
    it decides to leave; each is still answered (a relaunch or the launch
    path), with the oracle's bytes."""
    d = lx.tools.gen_dag(30, 20, 5, 0, 0, 4)
    w = [1 + (i % 3) for i in range(30)]
    o = _oracle(d, w)
    ix = lx.Index(options={"get_server": 2})
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    N = len(d)
    for i in range(300):
        e = (i * 37) % N
        assert ix.highest_before(e) == o.hb(e), e
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.00018 + 0.00002 * (i % 7):   # 180-300 us
            pass
    st = ix.get_server_stats()
    assert st["served"] + st["fallbacks"] >= 300 and st["launches"] >= 2, st
    ix.close()


def test_server_refuses_unknown_event_on_device(lx):
    """An event past the handle's rows that reaches the device (the host's own
    check turned off, option getter_host_check = 0) is refused by the row
    server and by the row kernel -- an error, no row read -- and the server
    keeps answering valid requests afterwards (vecfc/store_vectors.go:40-65:
    getters of an unknown event return nil; the reference's caller never asks)."""
    d = lx.tools.gen_dag(20, 15, 5, 2, 3, 6)
    w = [1 + (i % 4) for i in range(20)]
    o = _oracle(d, w)
    ix = lx.Index(options={"get_server": 2, "getter_host_check": 0})
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    ix.sync()
    assert ix.highest_before(3) == o.hb(3)
    s0 = ix.get_server_stats()
    for bad in (0xFFFFFFF0, 0x7FFFFFFF, 1 << 28):
        for f in (ix.highest_before, ix.lowest_after, ix.merged_highest_before):
            with pytest.raises(lx.capi.LxError):
                f(bad)
    s1 = ix.get_server_stats()
    assert s1["served"] > s0["served"], (s0, s1)          # the server answered them (with the error)
    for e in range(0, len(d), 17):
        assert ix.highest_before(e) == o.hb(e), e
        assert ix.lowest_after(e) == o.la(e), e
    assert ix.get_server_stats()["served"] > s1["served"]
    ix.set_option("get_server", 0)                        # the launch path has the same bound
    with pytest.raises(lx.capi.LxError):
        ix.lowest_after(0xFFFFFFF0)
    with pytest.raises(lx.capi.LxError):
        ix.highest_before_batch([1, 0xFFFFFFF0, 2])
    assert ix.lowest_after(5) == o.la(5)
    ix.close()


def test_server_auto_mode_with_several_handles(lx):
    """Option get_server = 1 (default): the server runs only while the handle
    is the process's only one."""
    import gc
    gc.collect()
    d = lx.tools.gen_dag(16, 20, 4, 0, 0, 2)
    w = [1] * 16
    a = lx.Index()
    a.reset(w)
    a.add_batch(d.creator, d.seq, d.poff, d.par)
    a.sync()
    b = lx.Index()
    assert a.live_handles() >= 2
    s0 = a.get_server_stats()
    for e in range(0, len(d), 9):
        a.highest_before(e)
    s1 = a.get_server_stats()
    assert s1["served"] == s0["served"] and s1["fallbacks"] > s0["fallbacks"], (s0, s1)
    b.close()
    if a.live_handles() == 1:             # (another test's handle may still be alive)
        for e in range(0, len(d), 9):
            a.highest_before(e)
        assert a.get_server_stats()["served"] > s1["served"]
    a.close()


def test_more_streams_than_hw_queues(lx):
    """Six handles (six streams, more than the box's GPU_MAX_HW_QUEUES = 4)
    interleaving one-event Adds and single-row getters: no call waits for a
    resident server on a shared queue (the default mode leaves the server
    off while several handles exist), and every row equals the oracle's."""
    K = 6
    d = lx.tools.gen_dag(30, 40, 6, 0, 0, 8)
    w = [1 + (i % 5) for i in range(30)]
    o = _oracle(d, w)
    N = len(d)
    half = N // 2
    ixs = []
    for _ in range(K):
        ix = lx.Index()
        ix.reset(w)
        ix.add_batch(d.creator[:half], d.seq[:half], d.poff[:half + 1], d.par)
        ix.sync()
        ixs.append(ix)
    t = []
    for e in range(half, min(N, half + 200)):
        p0, p1 = int(d.poff[e]), int(d.poff[e + 1])
        for ix in ixs:
            t0 = time.perf_counter()
            ix.add(int(d.creator[e]), int(d.seq[e]), [int(x) for x in d.par[p0:p1]])
            ix.sync()
            row = ix.highest_before(e)
            t.append(time.perf_counter() - t0)
            assert row == o.hb(e), e
    for ix in ixs:
        assert ix.get_server_stats()["served"] == 0
        ix.close()
    t = np.sort(np.array(t))
    # a wait behind a resident server would cost its 250 us idle exit
    assert t[len(t) // 2] < 250e-6, t[len(t) // 2]
