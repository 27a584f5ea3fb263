"""Row segments across GPUs.

One process per GPU; rank r holds an :class:`~lachesis_hip.Index` with
options ``seg_count=world, seg_rank=r`` and adds the epoch as one batch.
Every rank assigns every event's branch (replicated metadata), but walks and
owns only the rows of its Add-order segment (``rowseg_range``): the walk of
an epoch of D DAG levels takes ~D/G levels per rank.  :meth:`RowSegments.exchange`
then connects the segments:

* rows -- a segment's first levels ("partial" events, whose rows miss the
  last event of some branch before the segment) take the max of the final
  rows they reference, which live on earlier ranks; the LowestAfter pass also
  needs the row before each branch's first own event.  Each round: the ids
  go to their owners (``all_to_all_single``), the owners answer with the rows
  and a ready flag (a partial row of an owner still waiting is not final),
  the rows come back; rounds repeat until no rank waits (one round when a
  segment is longer than the DAG's observation depth);
* LowestAfter -- a rank's range fill reaches rows of earlier segments: those
  entries travel as (row, column, seq) triples to their owners.

A rank's planes hold its own rows only (about 1/G of the epoch, plus receive
areas for the rows it gets from the others), so a G-GPU index holds an epoch
G times the height one GPU can.

Afterwards :meth:`RowSegments.forkless_cause_dev` answers ForklessCause of ANY
pair of the epoch (vecfc/forkless_cause.go:40-82): each rank's queries go to
owner(a), which holds HB(a); the LowestAfter rows of the b outside its
segment come from their owners; the answers go back in the caller's order
(DESIGN.md section 6c), and :meth:`RowSegments.get_rows_dev` /
:meth:`RowSegments.get_rows` answer the vector getters (GetHighestBefore,
GetLowestAfter, GetMergedHighestBefore; vecfc/store_vectors.go:26-51,
vecengine/index.go:235-250) for events of every rank the same way: ids to
their owners, encoded rows back.  The reference has no multi-process index
(vecfc/index.go is single-node): this is the MI355X scale-out of the same
computation, bit-exact to the single index (tests/test_gpu_rowseg.py).
"""

import torch
import torch.distributed as dist


class RowSegments:
    def __init__(self, index, group=None, device=None):
        """``index``: this rank's handle (options seg_count = world, seg_rank = rank)."""
        self.ix = index
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        # gloo moves host tensors only: stage device buffers through the host
        # (a rehearsal mode for several ranks sharing one GPU; RCCL is the product)
        self.stage = dist.get_backend(group) == "gloo" and self.device.type == "cuda"
        self.last = {}
        self.last_fc = {}
        self._bufs = {}   # device buffers of forkless_cause_dev, grown on demand

    def _a2a(self, recv, send, recv_n, send_n):
        if self.stage:
            r = recv.cpu()
            dist.all_to_all_single(r, send.cpu(), output_split_sizes=recv_n, input_split_sizes=send_n, group=self.group)
            recv.copy_(r)
        else:
            dist.all_to_all_single(recv, send, output_split_sizes=recv_n, input_split_sizes=send_n, group=self.group)
            # the library reads `recv` on its own stream
            torch.cuda.current_stream(self.device).synchronize()

    def _counts(self, send_n):
        s = torch.tensor(send_n, dtype=torch.int64, device="cpu" if self.stage else self.device)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return [int(x) for x in r.cpu()]

    def _sum(self, x):
        t = torch.tensor([x], dtype=torch.int64, device="cpu" if self.stage else self.device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return int(t.item())

    def exchange(self):
        """Both exchanges and lx_rowseg_finish, after this rank's add_batch."""
        ix, G, dev = self.ix, self.world, self.device
        W = ix.rowseg_row_words()
        cap = max(1, ix.rowseg_request_cap())
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        rounds = 0
        rows_moved = 0
        while True:
            counts = ix.rowseg_requests(ids.data_ptr(), cap, G)
            if self._sum(sum(counts)) == 0:
                break
            rounds += 1
            total = sum(counts)
            recv_n = self._counts(counts)
            asked = torch.empty(max(1, sum(recv_n)), dtype=torch.int32, device=dev)
            self._a2a(asked[:sum(recv_n)], ids[:total], recv_n, counts)
            m = sum(recv_n)
            out_rows = torch.empty(max(1, m) * W, dtype=torch.int32, device=dev)
            out_ready = torch.empty(max(1, m), dtype=torch.int32, device=dev)
            ix.rowseg_serve(m, asked.data_ptr(), out_rows.data_ptr(), out_ready.data_ptr())
            got_rows = torch.empty(max(1, total) * W, dtype=torch.int32, device=dev)
            got_ready = torch.empty(max(1, total), dtype=torch.int32, device=dev)
            self._a2a(got_rows[:total * W], out_rows[:m * W], [c * W for c in counts], [c * W for c in recv_n])
            self._a2a(got_ready[:total], out_ready[:m], counts, recv_n)
            ix.rowseg_receive(total, ids.data_ptr(), got_rows.data_ptr(), got_ready.data_ptr())
            rows_moved += total
            if rounds > G + 1:
                raise RuntimeError("row-segment row exchange did not converge")
        la_counts = ix.rowseg_la(G)
        n_send = sum(la_counts)
        send = torch.empty(max(1, 3 * n_send), dtype=torch.int32, device=dev)
        ix.rowseg_la_fetch(send.data_ptr())
        recv_n = self._counts(la_counts)
        n_recv = sum(recv_n)
        recv = torch.empty(max(1, 3 * n_recv), dtype=torch.int32, device=dev)
        self._a2a(recv[:3 * n_recv], send[:3 * n_send], [3 * c for c in recv_n], [3 * c for c in la_counts])
        ix.rowseg_la_apply(n_recv, recv.data_ptr())
        ix.rowseg_finish()
        self.last = {"row_rounds": rounds, "rows_received": rows_moved, "la_entries_sent": n_send,
                     "la_entries_received": n_recv}
        return self.last

    def _buf(self, name, n, dtype=torch.int32):
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = torch.empty(max(1, n), dtype=dtype, device=self.device)
            self._bufs[name] = b
        return b

    def forkless_cause_dev(self, n, qa, qb, out, timing=False):
        """ForklessCause of this rank's n queries (device tensors qa, qb of
        int32 event ids, out uint8), collectively with every rank.  With
        ``timing`` the k_fc launch over the routed pairs is bracketed by HIP
        events on the library's stream (last_fc["kernel_ms"]), and the rest of
        the call is split by host clocks into the library's device steps
        (route, need, serve, store, unroute: each completed on return --
        last_fc["device_ms"], per step in "device_steps_ms") and the
        collectives between them (last_fc["collective_ms"])."""
        import time
        ix, G = self.ix, self.world
        dev_ms = {}
        coll = [0.0]

        def dstep(name, f, *a):
            t = time.perf_counter()
            r = f(*a)
            dev_ms[name] = dev_ms.get(name, 0.0) + (time.perf_counter() - t) * 1e3
            return r

        def cstep(f, *a):
            t = time.perf_counter()
            r = f(*a)
            coll[0] += (time.perf_counter() - t) * 1e3
            return r

        ra, rb = self._buf("ra", n), self._buf("rb", n)
        perm = self._buf("perm", n)
        send_n = dstep("route", ix.rowseg_fc_route, n, qa.data_ptr(), qb.data_ptr(), ra.data_ptr(), rb.data_ptr(),
                       perm.data_ptr(), G)
        recv_n = cstep(self._counts, send_n)
        m = sum(recv_n)
        xa, xb = self._buf("xa", m), self._buf("xb", m)
        cstep(self._a2a, xa[:m], ra[:n], recv_n, send_n)
        cstep(self._a2a, xb[:m], rb[:n], recv_n, send_n)
        ids = self._buf("ids", m)
        need_n = dstep("need", ix.rowseg_fc_need, m, xa.data_ptr(), xb.data_ptr(), ids.data_ptr(), max(1, m), G)
        ask_n = cstep(self._counts, need_n)
        nn, na = sum(need_n), sum(ask_n)
        W = ix.rowseg_row_words()
        asked = self._buf("asked", na)
        cstep(self._a2a, asked[:na], ids[:nn], ask_n, need_n)
        rows = self._buf("rows", na * W)
        dstep("serve", ix.rowseg_la_serve, na, asked.data_ptr(), rows.data_ptr())
        got = self._buf("got", nn * W)
        cstep(self._a2a, got[:nn * W], rows[:na * W], [c * W for c in need_n], [c * W for c in ask_n])
        dstep("store", ix.rowseg_la_store, nn, ids.data_ptr(), got.data_ptr())
        ans = self._buf("ans", m, torch.uint8)
        ev = None
        if timing:
            st = torch.cuda.ExternalStream(ix.device_planes()[3], device=self.device)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(st)
        t = time.perf_counter()
        ix.forkless_cause_batch_dev(m, xa.data_ptr(), xb.data_ptr(), ans.data_ptr())
        if ev is not None:
            ev[1].record(st)
        ix.sync()
        fc_wall = (time.perf_counter() - t) * 1e3
        back = self._buf("back", n, torch.uint8)
        cstep(self._a2a, back[:n], ans[:m], send_n, recv_n)
        dstep("unroute", ix.rowseg_fc_unroute, n, perm.data_ptr(), back.data_ptr(), out.data_ptr())
        self.last_fc = {"routed_away": n - send_n[self.rank], "answered": m, "rows_received": nn, "rows_sent": na,
                        "device_ms": sum(dev_ms.values()), "device_steps_ms": dev_ms, "collective_ms": coll[0],
                        "fc_wall_ms": fc_wall}
        if ev is not None:
            self.last_fc["kernel_ms"] = ev[0].elapsed_time(ev[1])
        return self.last_fc

    def get_rows_dev(self, mode, n, ev):
        """The vector getter rows of this rank's n events (device int32 tensor
        ``ev``, events of any rank), collectively with every rank: mode 0
        HighestBefore, 1 LowestAfter, 2 merged HighestBefore (reference byte
        layouts).  Returns (rows uint8 [n, slot] on the device, lengths int64
        [n]); a length of 0xFFFFFFFF marks an event outside the epoch."""
        ix, G = self.ix, self.world
        slot = (ix.row_bytes_max() + 15) // 16 * 16
        ra, rb = self._buf("g_ra", n), self._buf("g_rb", n)
        perm = self._buf("g_perm", n)
        # owner(ev) routing (the ForklessCause route with b = a), permutation kept
        send_n = ix.rowseg_fc_route(n, ev.data_ptr(), ev.data_ptr(), ra.data_ptr(), rb.data_ptr(), perm.data_ptr(), G)
        recv_n = self._counts(send_n)
        m = sum(recv_n)
        asked = self._buf("g_asked", m)
        self._a2a(asked[:m], ra[:n], recv_n, send_n)
        words = slot // 4
        rows = self._buf("g_rows", m * words)
        lens = self._buf("g_lens", m)
        ix.get_rows_dev(mode, m, asked.data_ptr(), rows.data_ptr(), slot, lens.data_ptr())
        back = self._buf("g_back", n * words)
        blen = self._buf("g_blen", n)
        self._a2a(back[:n * words], rows[:m * words], [c * words for c in send_n], [c * words for c in recv_n])
        self._a2a(blen[:n], lens[:m], send_n, recv_n)
        p = perm[:n].long()
        out = torch.empty((n, words), dtype=torch.int32, device=self.device)
        out[p] = back[:n * words].view(n, words)
        olen = torch.empty(n, dtype=torch.int64, device=self.device)
        olen[p] = blen[:n].long() & 0xFFFFFFFF
        self.last_get = {"routed_away": n - send_n[self.rank], "answered": m}
        return out.view(torch.uint8).view(n, slot), olen

    def get_rows(self, mode, events):
        """get_rows_dev from host event ids: a list of byte rows (None for an
        event outside the epoch)."""
        import numpy as np
        ev = torch.from_numpy(np.ascontiguousarray(events, dtype=np.uint32).view(np.int32)).to(self.device)
        rows, lens = self.get_rows_dev(mode, len(events), ev)
        rows, lens = rows.cpu().numpy(), lens.cpu().numpy()
        return [None if int(k) == 0xFFFFFFFF else bytes(rows[i, :int(k)]) for i, k in enumerate(lens)]
