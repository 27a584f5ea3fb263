// lx_shard_exchange.h -- the LowestAfter all-to-all of the column shards
//  as a host-side driver over two interfaces, so that the
// same code runs over RCCL in the library (lx_shard_rccl.cpp) and over an
// in-process fake transport in the CPU tests (tests/csrc/shard_fake.cpp).
//
//   Ops (one rank's index): block(src, dst, &entries), wire(&bytes),
//       pack(dst, buf, width) -> 0 | LX_ERR_WIRE (width 1 and an entry does not
//       fit) | error, unpack(src, buf, width), own(), send_buf(bytes),
//       recv_buf(bytes); the incremental exchange: branches(&B) (0: whole
//       blocks always), dirty(B, dmin), dirty_set(B, dmin), commit()
//   Net (the collectives): widths(send_w[G], recv_w[G]) -- every rank tells
//       every peer the width of the block it sends it; blocks(send, so, sb,
//       recv, ro, rb) -- grouped point-to-point moves of the blocks;
//       min_u32(v, n) -- element-wise minimum over the ranks, in place
//
// Incremental: each rank reports, for its own branches, the first row whose
// LowestAfter entries can have changed since the last exchange
// (lx_shard_dirty); the element-wise min over the ranks gives every rank the
// same dirty row lists (lx_shard_dirty_set), so blocks hold only the rows
// written since then -- bytes scale with the events added, not the epoch.
//
// Wire widths: a block goes at 1 byte per entry when it fits, else at the
// epoch width (2 while every seq < 2^16, else 4).  A sender that had to fall
// back for a destination starts there at the wide width next time (a failed
// byte pack costs a pack and a check), re-trying the byte wire every
// kWireRetry exchanges.  Every block starts at a multiple of 4 bytes on both
// sides (shard_layout), so unpack kernels read aligned 2- and 4-byte words.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/lachesis_hip.h"

namespace lx {

constexpr uint32_t kWireRetry = 8;

// Block offsets of one rank's send (or receive) buffer: block q holds
// entries[q] x width[q] bytes at off[q], off[q] a multiple of 4; off[G] is the
// buffer size.  The own block (q == self) is empty.
inline uint64_t shard_layout(uint32_t G, uint32_t self, const uint64_t *entries, const uint32_t *width,
                             uint64_t *off) {
    uint64_t o = 0;
    for (uint32_t q = 0; q < G; q++) {
        off[q] = o;
        if (q != self) o += (entries[q] * width[q] + 3) & ~3ull;
    }
    off[G] = o;
    return o;
}

struct ExchangeState {
    std::vector<uint32_t> last_w;   // width each destination got last time (0: never sent)
    uint64_t count = 0;             // exchanges so far
};

template <class Ops, class Net>
int shard_exchange_run(Ops &ops, Net &net, uint32_t r, uint32_t G, ExchangeState &st) {
    if (G <= 1) return 0;
    if (st.last_w.size() != G) st.last_w.assign(G, 0);
    uint32_t wb = 4;
    int rc;
    if ((rc = ops.wire(&wb))) return rc;
    std::vector<uint64_t> sn(G, 0), rn(G, 0), so(G + 1), ro(G + 1), sb(G, 0), rb(G, 0);
    std::vector<uint32_t> sw(G, 0), rw(G, 0), wide(G, wb);
    uint32_t nb = 0;
    if ((rc = ops.branches(&nb))) return rc;
    if (nb) {
        std::vector<uint32_t> dm(nb);
        if ((rc = ops.dirty(nb, dm.data())) || (rc = net.min_u32(dm.data(), nb)) || (rc = ops.dirty_set(nb, dm.data())))
            return rc;
    }
    for (uint32_t q = 0; q < G; q++) {
        if (q == r) continue;
        if ((rc = ops.block(r, q, &sn[q])) || (rc = ops.block(q, r, &rn[q]))) return rc;
    }
    // room for every block at the wide width
    uint8_t *send = ops.send_buf(shard_layout(G, r, sn.data(), wide.data(), so.data()));
    if (!send) return LX_ERR_NOMEM;
    const bool retry = st.count % kWireRetry == 0;
    for (uint32_t q = 0; q < G; q++) {
        if (q == r || !sn[q]) continue;
        sw[q] = (st.last_w[q] > 1 && !retry) ? wb : 1u;
    }
    // pack at the chosen widths; a misfit on the byte wire falls back, the
    // layout is recomputed and packing resumes at that block (earlier blocks
    // keep their offsets)
    for (uint32_t q0 = 0; q0 < G;) {
        shard_layout(G, r, sn.data(), sw.data(), so.data());
        uint32_t q = q0;
        for (; q < G; q++) {
            if (q == r || !sn[q]) continue;
            rc = ops.pack(q, send + so[q], sw[q]);
            if (rc == LX_ERR_WIRE && sw[q] == 1) {
                sw[q] = wb;
                break;
            }
            if (rc) return rc;
        }
        q0 = q;
    }
    for (uint32_t q = 0; q < G; q++) {
        sb[q] = q == r ? 0 : sn[q] * sw[q];
        if (q != r && sn[q]) st.last_w[q] = sw[q];
    }
    if ((rc = net.widths(sw.data(), rw.data()))) return rc;
    for (uint32_t q = 0; q < G; q++) {
        if (q == r || !rn[q]) {
            rw[q] = 0;
            continue;
        }
        if (rw[q] != 1 && rw[q] != 2 && rw[q] != 4) return LX_ERR_STATE;
        rb[q] = rn[q] * rw[q];
    }
    uint8_t *recv = ops.recv_buf(shard_layout(G, r, rn.data(), rw.data(), ro.data()));
    if (!recv) return LX_ERR_NOMEM;
    if ((rc = net.blocks(send, so.data(), sb.data(), recv, ro.data(), rb.data()))) return rc;
    for (uint32_t q = 0; q < G; q++)
        if (rb[q] && (rc = ops.unpack(q, recv + ro[q], rw[q]))) return rc;
    if ((rc = ops.own())) return rc;
    if (nb && (rc = ops.commit())) return rc;
    st.count++;
    return 0;
}

}  // namespace lx
