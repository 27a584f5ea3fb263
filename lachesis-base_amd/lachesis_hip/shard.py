"""Column-sharded index across GPUs.

One process per GPU; rank r holds an :class:`~lachesis_hip.Index` created
with ``shard_rank=r, shard_count=world`` and indexes the same event stream
as every other rank, but only the branches whose creator lies in its creator
range (``lx_shard_range``).  HighestBefore needs no communication (a column
depends only on the same column of the parents).  Two steps do:

* :meth:`ShardedIndex.exchange` -- before ForklessCause, every rank needs the
  LowestAfter entries of *its* columns for events on the other ranks'
  branches.  Block (src -> dst) = rows on src's branches x dst's columns
  (``lx_shard_block``); one ``all_to_all_single`` moves all of them.
* :meth:`ShardedIndex.forkless_cause_dev` -- each rank sums the stake of its
  own creators that ``b`` is forkless-caused by (``lx_forkless_cause_partial_dev``;
  bit 31 carries "a observes branch(b) as forked" from the owning rank); one
  ``all_reduce`` adds the partials and ``lx_fc_combine_dev`` applies quorum.

The reference has no multi-process index (vecfc/index.go is single-node);
this is the MI355X-side scale-out of the same computation, bit-exact to the
unsharded index (tests/test_gpu_shards.py).

The protocol is written against a small provider interface (the methods of
:class:`~lachesis_hip.Index` used below) so the collective plumbing can be
exercised with gloo on CPU (tests/test_shard_protocol.py).
"""

import torch
import torch.distributed as dist

try:
    from .capi import LxError
except ImportError:          # the protocol tests load this module without the library
    LxError = RuntimeError
LX_ERR_WIRE = -7             # include/lachesis_hip.h
WIRE_RETRY = 8               # csrc/lx_shard_exchange.h kWireRetry


def shard_layout(G, self_rank, entries, widths):
    """Offsets of the blocks in one rank's exchange buffer (G + 1 entries):
    block q holds entries[q] x widths[q] bytes starting at a multiple of 4
    (the own block is empty) -- lx_shard_exchange_layout."""
    off, o = [], 0
    for q in range(G):
        off.append(o)
        if q != self_rank:
            o += (entries[q] * widths[q] + 3) & ~3
    off.append(o)
    return off


class ShardedIndex:
    def __init__(self, index, group=None, device=None):
        """``index``: this rank's handle (shard_rank = rank, shard_count = world)."""
        self.ix = index
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        # gloo moves host tensors only: stage device buffers through the host
        # (a rehearsal mode for several ranks sharing one GPU; RCCL is the product)
        self.stage = dist.get_backend(group) == "gloo" and self.device.type == "cuda"
        self._bufs = {}
        self._last_w = []        # width each destination got last time (byte-wire fallbacks)
        self._count = 0
        self.last_bytes = 0      # bytes this rank sent in the last exchange

    def all_to_all(self, recv, send, recv_n, send_n):
        if self.stage:
            r = recv.cpu()
            dist.all_to_all_single(r, send.cpu(), output_split_sizes=recv_n, input_split_sizes=send_n, group=self.group)
            recv.copy_(r)
        else:
            dist.all_to_all_single(recv, send, output_split_sizes=recv_n, input_split_sizes=send_n, group=self.group)

    def all_reduce_sum(self, t):
        if self.stage:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    # ------------------------------------------------------------------ LA
    def exchange(self):
        """All-to-all of LowestAfter blocks; returns the entry counts sent.

        The protocol of lx_shard_exchange (csrc/lx_shard_exchange.h): blocks
        travel as bytes, each at 1 byte per entry when every entry is within
        127 of its row's seq (the pack checks as it goes and reports
        LX_ERR_WIRE otherwise), else at the epoch width (2 while every seq <
        2^16, else 4); a destination that needed the wide width starts there
        next time (the byte wire is retried every WIRE_RETRY exchanges); a
        G-int all-to-all tells the receivers the widths; every block starts at
        a multiple of 4 bytes on both sides (shard_layout)."""
        r, G = self.rank, self.world
        if G == 1 and hasattr(self.ix, "shard_of") and self.ix.shard_of()[1] == 1:
            # one rank, a whole handle: every row is local, nothing moves -- the
            # collectives still run (zero-length blocks), so a one-rank group
            # exercises the same device-tensor paths as G ranks
            self._min([0])
            w = self._widths([0])
            buf = self._buf("send", 4)
            self.all_to_all(self._buf("recv", 4)[:0], buf[:0], [0], [0])
            self.last_wire = ([0], w)
            self.last_bytes = 0
            return [0]
        incr = hasattr(self.ix, "shard_dirty")
        if incr:
            # only the rows written since the last exchange (lx_shard_dirty): each
            # rank knows the first changed row of its own branches, the
            # element-wise min over the ranks gives everyone every branch's
            self.ix.shard_dirty_set(self._min(self.ix.shard_dirty()))
        send_n = [self.ix.shard_block(r, t) if t != r else 0 for t in range(G)]
        recv_n = [self.ix.shard_block(s, r) if s != r else 0 for s in range(G)]
        per_block = hasattr(self.ix, "la_pack_wire_dev")
        wb = self.ix.shard_wire_bytes() if hasattr(self.ix, "shard_wire_bytes") else 4
        if len(self._last_w) != G:
            self._last_w = [0] * G
        retry = self._count % WIRE_RETRY == 0
        send_w = [0] * G
        for t in range(G):
            if t != r and send_n[t]:
                send_w[t] = 1 if per_block and (self._last_w[t] <= 1 or retry) else wb
        send = self._buf("send", shard_layout(G, r, send_n, [wb] * G)[-1])   # room for the widest case
        q0 = 0
        while q0 < G:
            so = shard_layout(G, r, send_n, send_w)
            q = q0
            while q < G:
                if q != r and send_n[q]:
                    if per_block:
                        try:
                            self.ix.la_pack_wire_dev(q, send.data_ptr() + so[q], send_w[q])
                        except LxError as e:
                            if e.code != LX_ERR_WIRE or send_w[q] != 1:
                                raise
                            send_w[q] = wb          # later blocks shift: resume packing here
                            break
                    else:
                        self.ix.la_pack_dev(q, send.data_ptr() + so[q])
                q += 1
            q0 = q
        for t in range(G):
            if t != r and send_n[t]:
                self._last_w[t] = send_w[t]
        self._count += 1
        recv_w = self._widths(send_w) if per_block else [wb if s != r else 0 for s in range(G)]
        for s in range(G):
            if s != r and recv_n[s] and recv_w[s] not in (1, 2, 4):
                raise RuntimeError("rank %d announced wire width %d" % (s, recv_w[s]))
        ro = shard_layout(G, r, recv_n, recv_w)
        send_b = [so[t + 1] - so[t] for t in range(G)]
        recv_b = [ro[s + 1] - ro[s] for s in range(G)]
        recv = self._buf("recv", ro[-1])
        self.ix.sync()   # packs run on the library stream; the collective on torch's
        if G > 1:
            self.all_to_all(recv[:ro[-1]], send[:so[-1]], recv_b, send_b)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        for s in range(G):
            if s != r and recv_n[s]:
                if per_block:
                    self.ix.la_unpack_wire_dev(s, recv.data_ptr() + ro[s], recv_w[s])
                else:
                    self.ix.la_unpack_dev(s, recv.data_ptr() + ro[s])
        self.ix.la_own_dev()     # own rows x own columns, no communication
        self.ix.sync()
        if incr:
            self.ix.shard_dirty_commit()
        self.last_wire = (send_w, recv_w)
        self.last_bytes = so[-1]
        return send_n

    def _min(self, v):
        """Element-wise minimum over the ranks of a uint32 numpy vector."""
        import numpy as np
        if len(v) == 0:
            return v
        dev = self.device if (self.device.type == "cuda" and not self.stage) else torch.device("cpu")
        t = torch.from_numpy(np.asarray(v, dtype=np.int64)).to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return t.cpu().numpy().astype(np.uint32)

    def _widths(self, send_w):
        """Tell every rank the width of the block this rank sends it; returns recv widths."""
        G = self.world
        dev = self.device if (self.device.type == "cuda" and not self.stage) else torch.device("cpu")
        sw = torch.tensor(send_w, dtype=torch.int32, device=dev)
        rw = torch.empty(G, dtype=torch.int32, device=dev)
        dist.all_to_all_single(rw, sw, group=self.group)
        return [int(x) for x in rw.tolist()]

    def _buf(self, name, nbytes):
        """Byte staging buffer for the exchange, kept between calls (grown on demand)."""
        cur = self._bufs.get(name)
        if cur is None or cur.numel() < max(nbytes, 1):
            self._bufs[name] = None
            cur = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
            self._bufs[name] = cur
        return cur

    def all_reduce_max(self, t):
        if self.stage:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MAX, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)

    def broadcast0(self, t):
        """Rank 0's tensor to every rank (in place)."""
        if self.stage:
            h = t.cpu()
            dist.broadcast(h, 0, group=self.group)
            t.copy_(h)
        else:
            dist.broadcast(t, 0, group=self.group)

    # ------------------------------------------------------------------ FC
    EARLY_MIN = 1 << 14   # csrc/lx_shard_rccl.cpp kShardEarlyMin: smaller calls keep one pass

    def _kernel_timer(self, timing):
        """HIP events on the library's stream around the partial-sum launches
        (kernel_ms in last_fc), or None."""
        if not timing or self.device.type != "cuda" or not hasattr(self.ix, "device_planes"):
            return None
        if getattr(self, "_lib_stream", None) is None:
            self._lib_stream = torch.cuda.ExternalStream(self.ix.device_planes()[3], device=self.device)
        return [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]

    def forkless_cause_dev(self, a, b, out=None, early=None, timing=False):
        """ForklessCause for device int32 index tensors ``a``, ``b`` -> uint8 tensor.

        Calls of >= EARLY_MIN queries on epochs where shard 0 can decide alone
        (lx_fc_shard_early: fork-free, shard 0's heaviest creators) take the
        early exit: shard 0 sums its creators' stake for every
        query and decides those whose sum reaches the quorum or cannot reach it
        with the other shards' stake added; its decisions are broadcast and
        only the undecided queries get the other shards' partials and the
        all-reduce.  ``early``: None (auto), False (always one pass).
        ``timing``: last_fc["kernel_ms"] = this rank's partial-sum launch(es)."""
        n = a.numel()
        if out is None:
            out = torch.empty(n, dtype=torch.uint8, device=self.device)
        ok = False
        if early is not False and n >= self.EARLY_MIN and self.world > 1 and hasattr(self.ix, "fc_shard_early"):
            ok = self.ix.fc_shard_early()[0]
        tm = self._kernel_timer(timing)
        if not ok:
            part = self._buf("fc_part", 4 * n).view(torch.int32)[:n]
            if tm:
                tm[0].record(self._lib_stream)
            self.ix.forkless_cause_partial_dev(n, a.data_ptr(), b.data_ptr(), part.data_ptr())
            if tm:
                tm[1].record(self._lib_stream)
            self.ix.sync()
            # partials are uint32 (stake sum < 2^31 plus at most one bit-31 mark, from
            # the rank owning branch(b)); the true total fits 32 bits, so the int32
            # wrap-around sum of the all-reduce is exact
            self.all_reduce_sum(part)   # (one rank: the identity, through the same collective)
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            self.ix.fc_combine_dev(n, part.data_ptr(), out.data_ptr())
            self.ix.sync()
            self.last_fc = {"n": n, "undecided": n, "early": False, "partial_queries": n}
            if tm:
                self.last_fc["kernel_ms"] = tm[0].elapsed_time(tm[1])
            return out
        W = (n + 63) // 64
        mask = self._buf("fc_mask", 16 * W).view(torch.int64)[:2 * W]
        q = self._buf("fc_q", 16 * n).view(torch.int32)
        idx, a2, b2, p2 = q[:n], q[n:2 * n], q[2 * n:3 * n], q[3 * n:4 * n]
        s0 = self.rank == 0
        part = None
        if s0:
            part = self._buf("fc_part", 4 * n).view(torch.int32)[:n]
            if tm:
                tm[0].record(self._lib_stream)
            self.ix.forkless_cause_partial_dev(n, a.data_ptr(), b.data_ptr(), part.data_ptr())
            if tm:
                tm[1].record(self._lib_stream)
            self.ix.fc_shard_decide_dev(n, part.data_ptr(), mask.data_ptr())
        self.ix.sync()
        self.broadcast0(mask)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        m = self.ix.fc_shard_undecided_dev(n, mask.data_ptr(), a.data_ptr(), b.data_ptr(),
                                           part.data_ptr() if s0 else None, idx.data_ptr(), a2.data_ptr(),
                                           b2.data_ptr(), p2.data_ptr() if s0 else None)
        if m:
            if not s0:
                if tm:
                    tm[0].record(self._lib_stream)
                self.ix.forkless_cause_partial_dev(m, a2.data_ptr(), b2.data_ptr(), p2.data_ptr())
                if tm:
                    tm[1].record(self._lib_stream)
                self.ix.sync()
            self.all_reduce_sum(p2[:m])
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
        self.ix.fc_shard_answer_dev(n, mask.data_ptr(), m, idx.data_ptr(), p2.data_ptr(), out.data_ptr())
        self.ix.sync()
        self.last_fc = {"n": n, "undecided": m, "early": True, "partial_queries": n if s0 else m}
        if tm:
            self.last_fc["kernel_ms"] = tm[0].elapsed_time(tm[1]) if (s0 or m) else 0.0
        return out

    # ------------------------------------------------------------------ getters
    def get_rows_dev(self, mode, n, ev):
        """Whole vector getter rows (mode 0 HighestBefore, 1 LowestAfter, 2
        merged HighestBefore; reference byte layouts) of n device int32 event
        ids, collectively with every rank (the same ids): each rank encodes its
        own branches (lx_get_rows_dev on a shard: zeros elsewhere), a sum over
        the ranks joins them (every word has one writer) and a max gives the
        length.  LowestAfter needs the exchange since the last Add.  Returns
        (rows uint8 [n, slot] on the device, lengths int64 [n]; 0xFFFFFFFF: not
        an event of the epoch)."""
        slot = (self.ix.row_bytes_max() + 15) // 16 * 16
        words = slot // 4
        rows = self._buf("g_rows", 4 * n * words).view(torch.int32)[:n * words]
        lens = self._buf("g_lens", 4 * n).view(torch.int32)[:n]
        self.ix.get_rows_dev(mode, n, ev.data_ptr(), rows.data_ptr(), slot, lens.data_ptr())
        self.all_reduce_sum(rows)
        ln = lens.long() & 0xFFFFFFFF           # (int32 max would order 0xFFFFFFFF below every length)
        self.all_reduce_max(ln)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        return rows.view(torch.uint8).view(n, slot).clone(), ln

    def get_rows(self, mode, events):
        """get_rows_dev from host event ids: a list of byte rows (None for an
        event outside the epoch)."""
        import numpy as np
        ev = torch.from_numpy(np.ascontiguousarray(events, dtype=np.uint32).view(np.int32)).to(self.device)
        rows, lens = self.get_rows_dev(mode, len(events), ev)
        rows, lens = rows.cpu().numpy(), lens.cpu().numpy()
        return [None if int(k) == 0xFFFFFFFF else bytes(rows[i, :int(k)]) for i, k in enumerate(lens)]


class ShardedDagIndexer:
    """abft.DagIndexer (vecfc.Index's surface as abft/indexed_lachesis.go:17-99
    and abft/lachesis.go:56-57 use it) over a column-sharded index: every rank
    runs the same caller on the same events, and each call here is collective.

    add / flush / drop_not_flushed go to this rank's shard handle (each indexes
    every event, its own creators' columns); forkless_cause runs the LowestAfter
    exchange when an Add changed the LowestAfter rows since the last one, then
    the partial sums and their all-reduce; get_merged_highest_before joins the
    shards' rows (creators are shard-local, so every shard encodes its own
    creators' merged entries).  Event ids map to dense indices in Add order,
    as the cgo shim keeps them."""

    def __init__(self, sharded):
        self.sx = sharded
        self.ix = sharded.ix
        self.validators = None

    def reset(self, validators, get_event=None):
        self.validators = validators
        self.ix.reset(list(validators.weights))
        self.pos, self.ids, self.n_flushed = {}, [], 0
        self._stale = False

    def add(self, e):
        ps = []
        for p in e.parents:    # self-parent first, as dag.Event keeps them
            if p not in self.pos:
                raise ValueError("processed out of order, parent not found")   # vecengine/index.go:159-161
            ps.append(self.pos[p])
        self.ix.add(self.validators.idxs[e.creator], e.seq, ps)
        self.pos[e.id] = len(self.ids)
        self.ids.append(e.id)
        self._stale = True

    def flush(self):
        self.ix.flush()
        self.n_flushed = len(self.ids)

    def drop_not_flushed(self):
        if len(self.ids) == self.n_flushed:
            return
        self.ix.drop_not_flushed()
        for eid in self.ids[self.n_flushed:]:
            del self.pos[eid]
        del self.ids[self.n_flushed:]
        self._stale = True

    def _fresh(self):
        if self._stale:
            self.sx.exchange()
            self._stale = False

    def forkless_cause(self, a, b):
        self._fresh()
        d = self.sx.device
        qa = torch.tensor([self.pos[a]], dtype=torch.int32, device=d)
        qb = torch.tensor([self.pos[b]], dtype=torch.int32, device=d)
        return bool(self.sx.forkless_cause_dev(qa, qb, early=False).cpu()[0])

    def get_merged_highest_before(self, eid):
        from .vecfc import HighestBeforeSeq
        return HighestBeforeSeq(self.sx.get_rows(2, [self.pos[eid]])[0])

    def get_highest_before(self, eid):
        from .vecfc import HighestBeforeSeq
        return HighestBeforeSeq(self.sx.get_rows(0, [self.pos[eid]])[0])

    def get_lowest_after(self, eid):
        from .vecfc import LowestAfterSeq
        self._fresh()
        return LowestAfterSeq(self.sx.get_rows(1, [self.pos[eid]])[0])
