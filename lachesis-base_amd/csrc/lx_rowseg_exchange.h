// lx_rowseg_exchange.h -- the two exchanges that join row segments (DESIGN.md
// section 6b) as a host-side driver over two interfaces, so that the same code
// runs over RCCL in the library (lx_rowseg_exchange in lx_shard_rccl.cpp) and
// over an in-process transport in the GPU tests (tests/csrc/rowseg_fake.cpp).
// It is the protocol lachesis_hip/rowseg.py runs over torch.distributed:
//
//   rows, in rounds until no rank waits: the ids of the rows this rank needs
//     go to their owners (grouped by owner, lx_rowseg_requests), the owners
//     answer with the rows and a ready flag each (lx_rowseg_serve), the rows
//     come back (lx_rowseg_receive);
//   LowestAfter: (row, column, seq) triples to the owners of the rows
//     (lx_rowseg_la / lx_rowseg_la_fetch / lx_rowseg_la_apply);
//   then lx_rowseg_finish.
//
//   Ops (this rank's index handle and device buffers): row_words(), request_cap(),
//     requests(ids, cap, counts[G]), serve(n, ids, rows, ready), receive(n, ids,
//     rows, ready), la(counts[G]), la_fetch(buf), la_apply(n, buf), finish(),
//     buf(slot, bytes) -> device buffer `slot` of at least `bytes`
//   Net (the collectives): sum(x) -> sum over ranks; counts(send[G], recv[G])
//     -- every rank tells every peer how many items it sends it; move(send,
//     send_bytes[G], recv, recv_bytes[G]) -- blocks grouped by rank in rank
//     order on both sides (the own block included), like all_to_all_single
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/lachesis_hip.h"

namespace lx {

struct RowsegExchangeStats {
    uint32_t rounds = 0;
    uint64_t rows_received = 0, la_sent = 0, la_received = 0;
};

enum RowsegBuf : int {
    kRsIds = 0, kRsAsked, kRsOutRows, kRsOutReady, kRsGotRows, kRsGotReady, kRsLaSend, kRsLaRecv,
    // ForklessCause across ranks (rowseg_fc_run)
    kRqA, kRqB, kRqPerm, kRqRecvA, kRqRecvB, kRqIds, kRqAsked, kRqRows, kRqGotRows, kRqAns, kRqAnsBack,
    // the vector getters across ranks (rowseg_get_run)
    kRgA, kRgB, kRgPerm, kRgAsked, kRgRows, kRgLens, kRgBack, kRgBackLens,
    kRsBufs
};

template <class Ops, class Net>
int rowseg_exchange_run(Ops &ops, Net &net, uint32_t G, RowsegExchangeStats &st) {
    st = RowsegExchangeStats{};
    int rc;
    uint32_t W = 0, cap = 0;
    if ((rc = ops.row_words(&W)) || (rc = ops.request_cap(&cap))) return rc;
    uint32_t *ids = static_cast<uint32_t *>(ops.buf(kRsIds, 4ull * (cap ? cap : 1)));
    if (!ids) return LX_ERR_NOMEM;
    std::vector<uint32_t> cnt(G);
    std::vector<uint64_t> send_n(G), recv_n(G), sb(G), rb(G);
    for (;;) {
        if ((rc = ops.requests(ids, cap, cnt.data()))) return rc;
        uint64_t total = 0;
        for (uint32_t q = 0; q < G; q++) total += send_n[q] = cnt[q];
        uint64_t all = 0;
        if ((rc = net.sum(total, &all))) return rc;
        if (!all) break;
        if (++st.rounds > G + 1) return LX_ERR_STATE;   // a segment shorter than the DAG's observation depth G times over
        if ((rc = net.counts(send_n.data(), recv_n.data()))) return rc;
        uint64_t m = 0;
        for (uint32_t q = 0; q < G; q++) m += recv_n[q];
        uint32_t *asked = static_cast<uint32_t *>(ops.buf(kRsAsked, 4 * (m + 1)));
        uint32_t *out_rows = static_cast<uint32_t *>(ops.buf(kRsOutRows, 4 * (m * W + 1)));
        uint32_t *out_ready = static_cast<uint32_t *>(ops.buf(kRsOutReady, 4 * (m + 1)));
        uint32_t *got_rows = static_cast<uint32_t *>(ops.buf(kRsGotRows, 4 * (total * W + 1)));
        uint32_t *got_ready = static_cast<uint32_t *>(ops.buf(kRsGotReady, 4 * (total + 1)));
        if (!asked || !out_rows || !out_ready || !got_rows || !got_ready) return LX_ERR_NOMEM;
        // ids to their owners
        for (uint32_t q = 0; q < G; q++) sb[q] = 4 * send_n[q], rb[q] = 4 * recv_n[q];
        if ((rc = net.move(ids, sb.data(), asked, rb.data()))) return rc;
        if ((rc = ops.serve((uint32_t)m, asked, out_rows, out_ready))) return rc;
        // rows and ready flags back, in the order they were asked
        for (uint32_t q = 0; q < G; q++) sb[q] = 4ull * W * recv_n[q], rb[q] = 4ull * W * send_n[q];
        if ((rc = net.move(out_rows, sb.data(), got_rows, rb.data()))) return rc;
        for (uint32_t q = 0; q < G; q++) sb[q] = 4 * recv_n[q], rb[q] = 4 * send_n[q];
        if ((rc = net.move(out_ready, sb.data(), got_ready, rb.data()))) return rc;
        if ((rc = ops.receive((uint32_t)total, ids, got_rows, got_ready))) return rc;
        st.rows_received += total;
    }
    if ((rc = ops.la(send_n.data()))) return rc;
    uint64_t ns = 0;
    for (uint32_t q = 0; q < G; q++) ns += send_n[q];
    uint32_t *tr = static_cast<uint32_t *>(ops.buf(kRsLaSend, 12 * (ns + 1)));
    if (!tr) return LX_ERR_NOMEM;
    if ((rc = ops.la_fetch(tr))) return rc;
    if ((rc = net.counts(send_n.data(), recv_n.data()))) return rc;
    uint64_t nr = 0;
    for (uint32_t q = 0; q < G; q++) nr += recv_n[q];
    uint32_t *rtr = static_cast<uint32_t *>(ops.buf(kRsLaRecv, 12 * (nr + 1)));
    if (!rtr) return LX_ERR_NOMEM;
    for (uint32_t q = 0; q < G; q++) sb[q] = 12 * send_n[q], rb[q] = 12 * recv_n[q];
    if ((rc = net.move(tr, sb.data(), rtr, rb.data()))) return rc;
    if ((rc = ops.la_apply(nr, rtr))) return rc;
    st.la_sent = ns;
    st.la_received = nr;
    return ops.finish();
}

struct RowsegFcStats {
    uint64_t routed_away = 0, answered = 0, rows_received = 0, rows_sent = 0;
};

// ForklessCause of any pair of the epoch (lx_rowseg_fc_* in lachesis_hip.h,
// DESIGN.md section 6c): queries to owner(a), LA rows of remote b to owner(a),
// answers back.  More Ops: fc_route(n, qa, qb, ra, rb, perm, counts[G]),
// fc_need(m, ra, rb, ids, cap, counts[G]), la_serve(n, ids, rows),
// la_store(n, ids, rows), fc_pairs(m, ra, rb, ans) (completed on return),
// fc_unroute(n, perm, ans, out), rank().
template <class Ops, class Net>
int rowseg_fc_run(Ops &ops, Net &net, uint32_t G, uint64_t n, const uint32_t *qa, const uint32_t *qb, uint8_t *out,
                  RowsegFcStats &st) {
    st = RowsegFcStats{};
    int rc;
    uint32_t W = 0;
    if ((rc = ops.row_words(&W))) return rc;
    const uint32_t me = ops.rank();
    std::vector<uint64_t> send_n(G), recv_n(G), sb(G), rb(G);
    uint32_t *ra = static_cast<uint32_t *>(ops.buf(kRqA, 4 * (n + 1)));
    uint32_t *rbq = static_cast<uint32_t *>(ops.buf(kRqB, 4 * (n + 1)));
    uint32_t *perm = static_cast<uint32_t *>(ops.buf(kRqPerm, 4 * (n + 1)));
    if (!ra || !rbq || !perm) return LX_ERR_NOMEM;
    if ((rc = ops.fc_route(n, qa, qb, ra, rbq, perm, send_n.data()))) return rc;
    for (uint32_t q = 0; q < G; q++)
        if (q != me) st.routed_away += send_n[q];
    if ((rc = net.counts(send_n.data(), recv_n.data()))) return rc;
    uint64_t m = 0;
    for (uint32_t q = 0; q < G; q++) m += recv_n[q];
    uint32_t *xa = static_cast<uint32_t *>(ops.buf(kRqRecvA, 4 * (m + 1)));
    uint32_t *xb = static_cast<uint32_t *>(ops.buf(kRqRecvB, 4 * (m + 1)));
    uint8_t *ans = static_cast<uint8_t *>(ops.buf(kRqAns, m + 1));
    uint8_t *back = static_cast<uint8_t *>(ops.buf(kRqAnsBack, n + 1));
    if (!xa || !xb || !ans || !back) return LX_ERR_NOMEM;
    for (uint32_t q = 0; q < G; q++) sb[q] = 4 * send_n[q], rb[q] = 4 * recv_n[q];
    if ((rc = net.move(ra, sb.data(), xa, rb.data())) || (rc = net.move(rbq, sb.data(), xb, rb.data()))) return rc;
    // LA rows of the remote b
    std::vector<uint64_t> need_n(G), ask_n(G);
    uint32_t *ids = static_cast<uint32_t *>(ops.buf(kRqIds, 4 * (m + 1)));
    if (!ids) return LX_ERR_NOMEM;
    if ((rc = ops.fc_need(m, xa, xb, ids, m, need_n.data()))) return rc;
    if ((rc = net.counts(need_n.data(), ask_n.data()))) return rc;
    uint64_t nn = 0, na = 0;
    for (uint32_t q = 0; q < G; q++) nn += need_n[q], na += ask_n[q];
    uint32_t *asked = static_cast<uint32_t *>(ops.buf(kRqAsked, 4 * (na + 1)));
    uint32_t *rows = static_cast<uint32_t *>(ops.buf(kRqRows, 4 * (na * W + 1)));
    uint32_t *got = static_cast<uint32_t *>(ops.buf(kRqGotRows, 4 * (nn * W + 1)));
    if (!asked || !rows || !got) return LX_ERR_NOMEM;
    for (uint32_t q = 0; q < G; q++) sb[q] = 4 * need_n[q], rb[q] = 4 * ask_n[q];
    if ((rc = net.move(ids, sb.data(), asked, rb.data()))) return rc;
    if ((rc = ops.la_serve(na, asked, rows))) return rc;
    for (uint32_t q = 0; q < G; q++) sb[q] = 4ull * W * ask_n[q], rb[q] = 4ull * W * need_n[q];
    if ((rc = net.move(rows, sb.data(), got, rb.data()))) return rc;
    if ((rc = ops.la_store(nn, ids, got))) return rc;
    st.rows_received = nn;
    st.rows_sent = na;
    // the pairs, then the answers back in the order they came
    if ((rc = ops.fc_pairs(m, xa, xb, ans))) return rc;
    st.answered = m;
    for (uint32_t q = 0; q < G; q++) sb[q] = recv_n[q], rb[q] = send_n[q];
    if ((rc = net.move(ans, sb.data(), back, rb.data()))) return rc;
    return ops.fc_unroute(n, perm, back, out);
}

// The vector getters of events on any rank (lx_rowseg_get_rows): ids to their
// owners (the ForklessCause route with b = a), rows encoded there
// (lx_get_rows_dev), rows and lengths back, put in the caller's order.  More
// Ops: get_rows(mode, m, ids, rows, slot, lens) (completed on return),
// rows_unroute(n, perm, rows, slot, lens, out, out_lens).
template <class Ops, class Net>
int rowseg_get_run(Ops &ops, Net &net, uint32_t G, uint32_t mode, uint64_t n, const uint32_t *ev, uint8_t *out,
                   uint64_t slot, uint32_t *out_len) {
    int rc;
    std::vector<uint64_t> send_n(G), recv_n(G), sb(G), rb(G);
    uint32_t *ra = static_cast<uint32_t *>(ops.buf(kRgA, 4 * (n + 1)));
    uint32_t *rbq = static_cast<uint32_t *>(ops.buf(kRgB, 4 * (n + 1)));
    uint32_t *perm = static_cast<uint32_t *>(ops.buf(kRgPerm, 4 * (n + 1)));
    if (!ra || !rbq || !perm) return LX_ERR_NOMEM;
    if ((rc = ops.fc_route(n, ev, ev, ra, rbq, perm, send_n.data()))) return rc;
    if ((rc = net.counts(send_n.data(), recv_n.data()))) return rc;
    uint64_t m = 0;
    for (uint32_t q = 0; q < G; q++) m += recv_n[q];
    uint32_t *asked = static_cast<uint32_t *>(ops.buf(kRgAsked, 4 * (m + 1)));
    uint8_t *rows = static_cast<uint8_t *>(ops.buf(kRgRows, slot * (m + 1)));
    uint32_t *lens = static_cast<uint32_t *>(ops.buf(kRgLens, 4 * (m + 1)));
    uint8_t *back = static_cast<uint8_t *>(ops.buf(kRgBack, slot * (n + 1)));
    uint32_t *blen = static_cast<uint32_t *>(ops.buf(kRgBackLens, 4 * (n + 1)));
    if (!asked || !rows || !lens || !back || !blen) return LX_ERR_NOMEM;
    for (uint32_t q = 0; q < G; q++) sb[q] = 4 * send_n[q], rb[q] = 4 * recv_n[q];
    if ((rc = net.move(ra, sb.data(), asked, rb.data()))) return rc;
    if ((rc = ops.get_rows(mode, m, asked, rows, slot, lens))) return rc;
    for (uint32_t q = 0; q < G; q++) sb[q] = slot * recv_n[q], rb[q] = slot * send_n[q];
    if ((rc = net.move(rows, sb.data(), back, rb.data()))) return rc;
    for (uint32_t q = 0; q < G; q++) sb[q] = 4 * recv_n[q], rb[q] = 4 * send_n[q];
    if ((rc = net.move(lens, sb.data(), blen, rb.data()))) return rc;
    return ops.rows_unroute(n, perm, back, slot, blen, out, out_len);
}

}  // namespace lx
