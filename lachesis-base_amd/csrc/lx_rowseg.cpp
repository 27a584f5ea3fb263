// lx_rowseg.cpp -- row segments: the segmented walk (lx_segment.hip) spread
// over ranks, one GPU each.
//
// Every rank takes the same epoch as one batch (branch assignment and the
// J_k tables are replicated metadata work) but walks, fixes up and owns only
// the rows of its segment [lo, hi).  Two exchanges connect the ranks, both
// driven by the caller's collectives (lachesis_hip/rowseg.py over
// torch.distributed / RCCL):
//   rows   -- a partial event's fix-up reads final rows of earlier segments
//             (and the LowestAfter pass needs the row before each branch's
//             first own event): lx_rowseg_requests groups the ids by owner,
//             owners answer with lx_rowseg_serve, lx_rowseg_receive stores
//             them; a row that is not final yet (a partial event whose owner
//             still waits) is answered "not ready" and asked again next
//             round -- at most G - 1 rounds, one when segments are longer
//             than the DAG's observation depth.
//   LowestAfter -- an own event's range fill reaches rows of earlier
//             segments: those entries leave as (row, column, seq) triples
//             per owner (lx_rowseg_la) and are written there
//             (lx_rowseg_la_apply).
// lx_rowseg_finish sets the own rows' fork marks; then ForklessCause answers
// queries between own events.
//
// Memory: a rank's planes hold its own rows only -- [lo, hi), about 1/G of
// the epoch (rs_planes) -- plus two receive areas sized by what arrives: the
// HighestBefore rows its partial events and its LowestAfter pass read from
// other ranks (rs_rhb, one row per distinct requested row), and the
// LowestAfter rows of one ForklessCause batch's remote b (rs_rla).  The
// reference's tables S / s (vecfc/store_vectors.go:26-65) have no epoch-height
// limit; neither has the G-GPU index: its height per GPU falls as 1/G.
#include "lx_index.h"

using namespace lxi;

namespace {



SegArgs rs_seg_args(lx_index *h) {
    SegArgs a{};
    a.hb = h->hb;
    a.la = h->la;
    a.stride = h->pstride;
    a.B = h->B;
    a.bs = 0;
    const uint32_t GS = h->rs_count * h->rs_sub;   // segments: rs_sub per rank
    a.n = h->rs_seg_lo[GS];
    a.G = GS;
    for (uint32_t k = 0; k <= GS; k++) a.seg_lo[k] = h->rs_seg_lo[k];
    a.ev_branch = h->ev_branch;
    a.ev_seq = h->ev_seq;
    a.branch_first = h->branch_first;
    a.branch_len = h->branch_len;
    a.brow = h->brow;
    a.s_cap = h->s_cap;
    a.jt = h->seg_jt;
    a.cnt = h->seg_cnt;
    a.pcount = h->seg_cnt + h->B;
    a.pflag = h->seg_mf;
    a.plist = h->seg_plist;
    a.elist = h->seg_elist;
    a.ecount = a.pcount + GS;
    a.own_seg = h->rs_rank * h->rs_sub;
    a.own_lo = h->rs_lo;
    a.per_rank = h->rs_sub;
    a.rhb = h->rs_rhb;
    a.hslot = h->rs_hslot;
    return a;
}

RsArgs rs_args(lx_index *h) {
    RsArgs r{};
    r.hb = h->hb;
    r.la = h->la;
    r.stride = h->pstride;
    r.B = h->B;
    r.lo = h->rs_lo;
    r.hi = h->rs_hi;
    r.pflag = h->seg_mf + h->rs_lo;
    r.partials_done = h->rs_state >= 2 ? 1u : 0u;
    r.need = h->rs_need;
    r.req = h->rs_req;
    r.req_count = h->rs_ctr;
    r.remaining = h->rs_ctr + 1;
    r.rhb = h->rs_rhb;
    r.hslot = h->rs_hslot;
    return r;
}

// the rank's own rows of an n-event epoch (the bounds rs_begin cuts: Add-order
// thirds on multiples of 64); hb / la become virtual bases, so every kernel
// addresses an own row e at plane + e * pstride as in whole planes
void own_bounds(const lx_index *h, uint32_t n, uint32_t *lo, uint32_t *hi) {
    const uint32_t G = h->rs_count, k = h->rs_rank;
    *lo = (uint32_t)((uint64_t)n * k / G / 64 * 64);
    *hi = k + 1 == G ? n : (uint32_t)((uint64_t)n * (k + 1) / G / 64 * 64);
}

RsqArgs rsq_args(const lx_index *h) {
    RsqArgs a{};
    a.G = h->rs_count;
    a.self = h->rs_rank;
    a.n_all = (uint32_t)h->n_events;
    a.lo = h->rs_lo;
    a.hi = h->rs_hi;
    a.B = h->B;
    for (uint32_t q = 0; q <= h->rs_count; q++) a.seg_lo[q] = h->rs_seg_lo[q * h->rs_sub];   // rank bounds
    return a;
}

int rsq_tmp(lx_index *h, uint64_t n) {
    size_t need = 0;
    HIPCHK(h, lx::rsq_tmp_bytes(n ? n : 1, h->rs_count, &need));
    if (need <= h->rsq_tmp_bytes && h->rsq_tmp) return 0;
    if (h->rsq_tmp) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(h->rsq_tmp);
        h->rsq_tmp = nullptr;
        h->rsq_tmp_bytes = 0;
    }
    HIPCHK(h, hipMalloc(&h->rsq_tmp, need ? need : 1));
    h->rsq_tmp_bytes = need;
    return 0;
}

int rs_check(lx_index *h, int state) {
    if (!h) return LX_ERR_ARG;
    if (!h->rowseg()) return h->fail(LX_ERR_STATE, "not a row-segment rank (options seg_count / seg_rank)");
    if (state >= 0 && h->rs_state != state)
        return h->fail(LX_ERR_STATE, "row-segment step out of order (state %d, expected %d)", h->rs_state, state);
    return h->hip(set_dev(h->device), "set device");
}

// the own partial events' rows from the rows they reference (every other
// rank's one final and present by now), own sub-segment by own sub-segment:
// a later one may reference rows of an earlier one, final after its fix-up
int rs_fix_partials(lx_index *h) {
    if (h->rs_npartial) {
        SegArgs a = rs_seg_args(h);
        HIPCHK(h, hipEventRecord(h->seg_ev[2], h->stream));
        for (uint32_t t = 0; t < h->rs_sub; t++)
            HIPCHK(h, lx::launch_seg_partial(a, a.own_seg + t, h->rs_npart[t], h->stream));
        HIPCHK(h, hipEventRecord(h->seg_ev[3], h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        HIPCHK(h, hipEventElapsedTime(&h->seg_stats.partial_ms, h->seg_ev[2], h->seg_ev[3]));
    }
    h->rs_state = 2;
    return 0;
}

}  // namespace

int rs_planes(lx_index *h, uint32_t n) {
    uint32_t lo, hi;
    own_bounds(h, n, &lo, &hi);
    const uint64_t rows = hi - lo;
    if (!h->rs_hb_mem || rows > h->rs_mem_rows || h->rs_mem_pstride != h->pstride) {
        rs_planes_free(h);
        HIPCHK(h, dalloc(&h->rs_hb_mem, rows * h->pstride));
        HIPCHK(h, dalloc(&h->rs_la_mem, rows * h->pstride));
        // a new HB allocation is zeroed here (its pad columns past the
        // epoch's branches are never written by the walk); the LA rows are
        // not: rs_begin zeroes the own rows at every batch before the walk
        // fills them.  Receive-area rows are read only where rs_lslot /
        // rs_hslot stamp them for the current batch.
        HIPCHK(h, hipMemsetAsync(h->rs_hb_mem, 0, rows * h->pstride * 4, h->stream));
        h->rs_mem_rows = rows;
        h->rs_mem_pstride = h->pstride;
    }
    h->hb = h->rs_hb_mem - (uint64_t)lo * h->pstride;
    h->la = h->rs_la_mem - (uint64_t)lo * h->pstride;
    return 0;
}

void rs_planes_free(lx_index *h) {
    if (!h->rs_hb_mem && !h->rs_la_mem) return;
    (void)hipStreamSynchronize(h->stream);
    if (h->rs_hb_mem) (void)hipFree(h->rs_hb_mem);
    if (h->rs_la_mem) (void)hipFree(h->rs_la_mem);
    h->rs_hb_mem = h->rs_la_mem = nullptr;
    h->hb = h->la = nullptr;
    h->rs_mem_rows = 0;
    h->rs_mem_pstride = 0;
}

void rs_free(lx_index *h) {
    void *p[] = {h->rs_need, h->rs_req, h->rs_ctr, h->rs_ids, h->rs_out, h->rs_send,
                 h->rs_stamp, h->rsq_scratch, h->rsq_list, h->rsq_ctr, h->rsq_tmp,
                 h->rs_hslot, h->rs_rhb, h->rs_lslot, h->rs_rla};
    for (void *q : p)
        if (q) (void)hipFree(q);
    h->rs_hslot = h->rs_rhb = h->rs_lslot = h->rs_rla = nullptr;
    h->rs_hslot_cap = h->rs_rhb_cap = h->rs_lslot_cap = h->rs_rla_cap = 0;
    h->rs_need = h->rs_req = h->rs_ctr = h->rs_ids = h->rs_out = h->rs_send = nullptr;
    h->rs_need_cap = h->rs_req_cap = h->rs_ids_cap = h->rs_out_cap = h->rs_send_cap = h->rs_ctr_cap = 0;
    h->rs_stamp = h->rsq_scratch = h->rsq_list = h->rsq_ctr = nullptr;
    h->rsq_tmp = nullptr;
    h->rs_stamp_cap = h->rsq_scratch_cap = h->rsq_list_cap = h->rsq_ctr_cap = 0;
    h->rsq_tmp_bytes = 0;
    h->rs_gen = 0;
    h->rs_state = 0;
}

// lx_add_batch on a row-segment rank (the epoch's only batch, assigned): walk
// the own segment, list the rows its partial events and its LowestAfter pass
// need from the other ranks
int rs_begin(lx_index *h, IndexArgs ia, const uint32_t *poff, hipStream_t s) {
    const uint32_t G = h->rs_count, k = h->rs_rank, n = ia.n;
    // sub-segments per rank: the segment count auto_segments would pick for a
    // rank's share of the epoch (the same on every rank: it depends only on
    // the epoch and the device), or option seg_sub; each >= 64 events
    uint32_t S = h->rs_sub_opt, cpw = ia.cpw_hint;
    if (!S) {
        uint32_t c = 0;
        S = seg_pick(h, (uint64_t)n / G, &c);
        if (S >= 2) cpw = c;
        else S = 1;
    }
    S = std::max<uint32_t>(1, std::min<uint32_t>({S, kMaxSegments / G, kSegLaunchMax}));
    while (S > 1 && (uint64_t)n / G < 128ull * S) S--;
    h->rs_sub = S;
    for (uint32_t q = 0; q < G; q++) {
        const uint64_t r0 = (uint64_t)n * q / G / 64 * 64, r1 = q + 1 == G ? n : (uint64_t)n * (q + 1) / G / 64 * 64;
        for (uint32_t t = 0; t < S; t++) h->rs_seg_lo[q * S + t] = (uint32_t)(r0 + (r1 - r0) * t / S / 64 * 64);
    }
    h->rs_seg_lo[G * S] = n;
    h->rs_lo = h->rs_seg_lo[k * S];
    h->rs_hi = h->rs_seg_lo[(k + 1) * S];
    {
        uint32_t lo, hi;
        own_bounds(h, n, &lo, &hi);
        if (lo != h->rs_lo || hi != h->rs_hi) return h->fail(LX_ERR_STATE, "row-segment bounds disagree with the planes");
    }
    int rc;
    if ((rc = grow_scratch(h, &h->seg_jt, &h->seg_jt_cap, (uint64_t)(G * S + 1) * h->B)) ||
        (rc = grow_scratch(h, &h->seg_cnt, &h->seg_cnt_cap, (uint64_t)h->B + 2 * kMaxSegments)) ||
        (rc = grow_scratch(h, &h->seg_mf, &h->seg_mf_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->seg_plist, &h->seg_plist_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->seg_elist, &h->seg_elist_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->rs_need, &h->rs_need_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->rs_hslot, &h->rs_hslot_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->rs_lslot, &h->rs_lslot_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->rs_ctr, &h->rs_ctr_cap, (uint64_t)2 + 2 * kMaxSegments)))
        return rc;
    while (h->seg_ev.size() < 6) {
        hipEvent_t e;
        HIPCHK(h, hipEventCreate(&e));
        h->seg_ev.push_back(e);
    }
    h->rs_state = 0;
    // no LowestAfter row of another segment has been received in this epoch
    if ((rc = grow_scratch(h, &h->rs_stamp, &h->rs_stamp_cap, (uint64_t)n))) return rc;
    HIPCHK(h, hipMemsetAsync(h->rs_stamp, 0, (uint64_t)n * 4, s));
    h->rs_gen = 0;
    SegArgs a = rs_seg_args(h);
    HIPCHK(h, lx::launch_seg_tables(a, s));
    // the own rows' LowestAfter is written by the own pass and the others' triples only
    HIPCHK(h, hipMemsetAsync(h->la + (uint64_t)h->rs_lo * h->pstride, 0,
                             (uint64_t)(h->rs_hi - h->rs_lo) * h->pstride * 4, s));
    ia.seg = 1;
    ia.ev_branch = h->ev_branch;
    ia.ev_seq = h->ev_seq;
    const IndexArgs ib = ia;   // the batch's walk arguments (records from event 0)
    const uint32_t k0 = a.own_seg;
    // the own sub-segments: one k_index_segs launch side by side when they fit
    // the CUs (as a single-GPU batch), else one walk each
    if (S > 1) ia.cpw_hint = cpw >= 8 && (!ia.pack16 || ia.mask) ? 4 : cpw;
    const bool conc = S > 1 && S * seg_walk_grid(h, ia.cpw_hint) <= h->n_cus;
    HIPCHK(h, hipEventRecord(h->seg_ev[0], s));
    for (uint32_t t = 0; t < S; t++) {
        if (conc && t) break;
        IndexArgs sk = ia;
        const uint32_t b0 = h->rs_seg_lo[k0 + t];
        sk.batch_start = conc ? h->rs_lo : b0;
        sk.n = conc ? h->rs_hi - h->rs_lo : h->rs_seg_lo[k0 + t + 1] - b0;
        sk.rec = ib.rec + sk.batch_start;
        sk.crec = ib.crec ? ib.crec + sk.batch_start : nullptr;
        sk.poff_in = poff + sk.batch_start;
        sk.seg_j = a.jt + (uint64_t)(k0 + t) * a.B;
        sk.seg_flag = a.pflag + sk.batch_start;
        sk.seg_list = a.plist + sk.batch_start;
        sk.seg_count = a.pcount + k0 + t;
        if (conc) {
            sk.seg_g = S;
            sk.seg_B = a.B;
            for (uint32_t u = 0; u <= S; u++) sk.seg_lo[u] = h->rs_seg_lo[k0 + u];
        }
        HIPCHK(h, lx::launch_index(sk, s));
    }
    HIPCHK(h, hipEventRecord(h->seg_ev[1], s));
    HIPCHK(h, hipMemcpyAsync(h->rs_npart, a.pcount + k0, 4ull * S, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    h->rs_npartial = 0;
    for (uint32_t t = 0; t < S; t++) h->rs_npartial += h->rs_npart[t];
    // the rows to ask for: at most every referenced branch of every partial
    // event plus one per branch, and never more than the events before lo
    const uint64_t want = std::min<uint64_t>((uint64_t)h->rs_npartial * h->B + h->B, (uint64_t)h->rs_lo + 1);
    if ((rc = grow_scratch(h, &h->rs_req, &h->rs_req_cap, want)) ||
        (rc = grow_scratch(h, &h->rs_ids, &h->rs_ids_cap, want)))
        return rc;
    HIPCHK(h, hipMemsetAsync(h->rs_need, 0, (uint64_t)n * 4, s));
    HIPCHK(h, hipMemsetAsync(h->rs_ctr, 0, (2 + 2 * kMaxSegments) * 4, s));
    RsArgs r = rs_args(h);
    HIPCHK(h, lx::launch_rs_refs(a, r, h->rs_npart, s));
    HIPCHK(h, hipMemcpyAsync(h->rs_ctr + 1, h->rs_ctr, 4, hipMemcpyDeviceToDevice, s));
    uint32_t nreq = 0;
    HIPCHK(h, hipMemcpyAsync(&nreq, h->rs_ctr, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    h->rs_nreq = nreq;
    // the receive area: one row per distinct requested row (rs_hslot set by k_rs_refs)
    if ((rc = grow_scratch(h, &h->rs_rhb, &h->rs_rhb_cap, (uint64_t)std::max<uint32_t>(nreq, 1) * h->pstride)))
        return rc;
    lx_seg_stats &st = h->seg_stats;
    st = lx_seg_stats{};
    st.segments = G;
    for (uint32_t q = 0; q <= G; q++) st.first_event[q] = h->rs_seg_lo[q * S];
    st.partial[k] = h->rs_npartial;
    st.one_launch = conc ? 1u : 0u;
    HIPCHK(h, hipEventElapsedTime(&st.walk_ms[k], h->seg_ev[0], h->seg_ev[1]));
    h->rs_state = 1;
    if (!nreq) return rs_fix_partials(h);
    return 0;
}

extern "C" {

int lx_rowseg_bounds(const lx_index *h, uint32_t *lo) {
    if (!h || !lo) return LX_ERR_ARG;
    if (!h->rowseg() || !h->rs_state) return LX_ERR_STATE;
    for (uint32_t q = 0; q <= h->rs_count; q++) lo[q] = h->rs_seg_lo[q * h->rs_sub];
    return 0;
}

int lx_rowseg_row_words(const lx_index *h, uint32_t *words) {
    if (!h || !words) return LX_ERR_ARG;
    *words = h->B;
    return 0;
}

int lx_rowseg_requests(lx_index *h, uint32_t *ids, uint32_t cap, uint32_t *counts) {
    int rc;
    if ((rc = rs_check(h, -1))) return rc;
    if (!counts) return LX_ERR_ARG;
    if (h->rs_state < 1 || h->rs_state > 2) return h->fail(LX_ERR_STATE, "row-segment requests outside the row exchange");
    for (uint32_t q = 0; q < h->rs_count; q++) counts[q] = 0;
    if (h->rs_state == 2 || !h->rs_nreq) return 0;
    if (ids && cap < h->rs_nreq) return h->fail(LX_ERR_ARG, "request buffer of %u ids < %u", cap, h->rs_nreq);
    SegArgs a = rs_seg_args(h);
    RsArgs r = rs_args(h);
    HIPCHK(h, lx::launch_rs_bucket(a, r, h->rs_nreq, ids ? ids : h->rs_ids, h->rs_ctr + 2, h->stream));
    HIPCHK(h, hipMemcpyAsync(counts, h->rs_ctr + 2, h->rs_count * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_request_cap(const lx_index *h, uint32_t *cap) {
    if (!h || !cap) return LX_ERR_ARG;
    *cap = h->rowseg() ? h->rs_nreq : 0u;
    return 0;
}

int lx_rowseg_serve(lx_index *h, uint32_t n, const uint32_t *ids, uint32_t *rows, uint32_t *ready) {
    int rc;
    if ((rc = rs_check(h, -1))) return rc;
    if (h->rs_state < 1 || h->rs_state > 2) return h->fail(LX_ERR_STATE, "row-segment serve outside the row exchange");
    RsArgs r = rs_args(h);
    HIPCHK(h, lx::launch_rs_gather(r, ids, n, rows, ready, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_receive(lx_index *h, uint32_t n, const uint32_t *ids, const uint32_t *rows, const uint32_t *ready,
                      uint32_t *remaining) {
    int rc;
    if ((rc = rs_check(h, -1))) return rc;
    if (h->rs_state < 1 || h->rs_state > 2) return h->fail(LX_ERR_STATE, "row-segment receive outside the row exchange");
    uint32_t left = 0;
    if (h->rs_state == 1) {
        RsArgs r = rs_args(h);
        HIPCHK(h, lx::launch_rs_scatter(r, ids, n, rows, ready, h->stream));
        HIPCHK(h, hipMemcpyAsync(&left, h->rs_ctr + 1, 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (!left && (rc = rs_fix_partials(h))) return rc;
    }
    if (remaining) *remaining = left;
    return 0;
}

int lx_rowseg_la(lx_index *h, uint64_t *counts) {
    int rc;
    if ((rc = rs_check(h, 2))) return rc;
    if (!counts) return LX_ERR_ARG;
    const uint32_t G = h->rs_count;
    if (!h->rs_out_per) h->rs_out_per = 1u << 18;
    std::vector<uint32_t> c(G);
    // the own events whose LowestAfter range reaches rows before the segment
    // (per own sub-segment: rows up to its J, in earlier own sub-segments or
    // other ranks' segments)
    SegArgs a = rs_seg_args(h);
    const uint32_t S = h->rs_sub, k0 = a.own_seg;
    uint32_t ne[kMaxSegments] = {};
    HIPCHK(h, hipEventRecord(h->seg_ev[4], h->stream));
    for (uint32_t t = 0; t < S; t++) HIPCHK(h, lx::launch_seg_edges(a, k0 + t, h->rs_npart[t], h->stream));
    HIPCHK(h, hipMemcpyAsync(ne, a.ecount + k0, 4ull * S, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (int attempt = 0; attempt < 2; attempt++) {
        if ((rc = grow_scratch(h, &h->rs_out, &h->rs_out_cap, 3ull * G * h->rs_out_per))) return rc;
        a.out = h->rs_out;
        a.out_count = h->rs_ctr + 2 + kMaxSegments;
        a.out_cap = h->rs_out_per;
        HIPCHK(h, hipMemsetAsync(a.out_count, 0, G * 4, h->stream));
        for (uint32_t t = 0; t < S; t++) HIPCHK(h, lx::launch_seg_la_edge(a, k0 + t, ne[t], h->stream));
        HIPCHK(h, hipEventRecord(h->seg_ev[5], h->stream));
        HIPCHK(h, hipMemcpyAsync(c.data(), a.out_count, G * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        const uint32_t mx = *std::max_element(c.begin(), c.end());
        if (mx <= h->rs_out_per) break;
        // too many entries for a destination: larger buckets, the same pass
        // again (it writes only these buckets)
        h->rs_out_per = (uint64_t)mx + mx / 4;
        if (attempt) return h->fail(LX_ERR_STATE, "row-segment LowestAfter buckets overflowed twice");
    }
    HIPCHK(h, hipEventElapsedTime(&h->seg_stats.la_ms, h->seg_ev[4], h->seg_ev[5]));
    uint64_t tot = 0;
    for (uint32_t q = 0; q < G; q++) tot += c[q];
    if ((rc = grow_scratch(h, &h->rs_send, &h->rs_send_cap, 3 * tot + 3))) return rc;
    uint64_t o = 0;
    for (uint32_t q = 0; q < G; q++) {
        counts[q] = c[q];
        if (c[q])
            HIPCHK(h, hipMemcpyAsync(h->rs_send + 3 * o, h->rs_out + 3ull * q * h->rs_out_per, 12ull * c[q],
                                     hipMemcpyDeviceToDevice, h->stream));
        o += c[q];
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->rs_nsend = o;
    h->rs_state = 3;
    return 0;
}

int lx_rowseg_la_fetch(lx_index *h, uint32_t *triples) {
    int rc;
    if ((rc = rs_check(h, 3))) return rc;
    if (h->rs_nsend)
        HIPCHK(h, hipMemcpyAsync(triples, h->rs_send, 12ull * h->rs_nsend, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_la_apply(lx_index *h, uint64_t n, const uint32_t *triples) {
    int rc;
    if ((rc = rs_check(h, 3))) return rc;
    RsArgs r = rs_args(h);
    HIPCHK(h, lx::launch_rs_la_apply(r, triples, n, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_finish(lx_index *h) {
    int rc;
    if ((rc = rs_check(h, 3))) return rc;
    if (h->B > h->V && h->n_cheat) {
        MarkArgs m{};
        m.hb = h->hb;
        m.stride = h->pstride;
        m.cmap = nullptr;
        m.batch_start = h->rs_lo;
        m.n = h->rs_hi - h->rs_lo;
        m.V = h->V;
        m.ev_branch = h->ev_branch;
        m.ev_bbefore = h->ev_bbefore;
        m.branch_first = h->branch_first;
        m.n_cheat = h->n_cheat;
        m.cheat_off = h->cheat_off;
        m.cheat_br = h->cheat_br;
        HIPCHK(h, lx::launch_marks(m, h->stream));
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->rs_state = 4;
    return 0;
}

// ---- ForklessCause of any pair of the epoch (lx_rowseg_fc.hip)

int lx_rowseg_fc_route(lx_index *h, uint64_t n, const uint32_t *qa, const uint32_t *qb, uint32_t *ra, uint32_t *rb,
                       uint32_t *perm, uint64_t *counts) {
    int rc;
    if ((rc = rs_check(h, 4))) return rc;
    if (!counts || (n && (!qa || !qb || !ra || !rb || !perm))) return LX_ERR_ARG;
    if (n >= 0x7FFFFFFFull) return h->fail(LX_ERR_ARG, "too many queries in one batch");
    const uint32_t G = h->rs_count;
    if ((rc = grow_scratch(h, &h->rsq_scratch, &h->rsq_scratch_cap, 3 * n + 3)) ||
        (rc = grow_scratch(h, &h->rsq_ctr, &h->rsq_ctr_cap, (uint64_t)2 * kMaxSegments + 2)) || (rc = rsq_tmp(h, n)))
        return rc;
    const RsqArgs a = rsq_args(h);
    HIPCHK(h, lx::launch_rsq_route(a, qa, qb, n, h->rsq_scratch, h->rsq_tmp, h->rsq_tmp_bytes, ra, rb, perm, h->rsq_ctr,
                                   h->stream));
    uint32_t c[kMaxSegments];
    HIPCHK(h, hipMemcpyAsync(c, h->rsq_ctr, 4ull * G, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (uint32_t q = 0; q < G; q++) counts[q] = c[q];
    return 0;
}

int lx_rowseg_fc_need(lx_index *h, uint64_t m, const uint32_t *ra, const uint32_t *rb, uint32_t *ids, uint64_t cap,
                      uint64_t *counts) {
    int rc;
    if ((rc = rs_check(h, 4))) return rc;
    if (!counts || (m && (!ra || !rb))) return LX_ERR_ARG;
    const uint32_t G = h->rs_count;
    if (h->rs_gen >= 0x7FFFFFF0u) {   // stamps about to wrap: forget every received row
        HIPCHK(h, hipMemsetAsync(h->rs_stamp, 0, h->n_events * 4, h->stream));
        h->rs_gen = 0;
    }
    h->rs_gen++;
    const uint64_t lim = std::min<uint64_t>(m, h->n_events);
    if ((rc = grow_scratch(h, &h->rsq_list, &h->rsq_list_cap, lim + 1)) ||
        (rc = grow_scratch(h, &h->rsq_ctr, &h->rsq_ctr_cap, (uint64_t)2 * kMaxSegments + 2)))
        return rc;
    const RsqArgs a = rsq_args(h);
    uint32_t *cnt = h->rsq_ctr + kMaxSegments;
    HIPCHK(h, hipMemsetAsync(cnt, 0, 4, h->stream));
    HIPCHK(h, lx::launch_rsq_need(a, ra, rb, m, h->rs_stamp, 2 * h->rs_gen, h->rsq_list, cnt, h->stream));
    uint32_t nl = 0;
    HIPCHK(h, hipMemcpyAsync(&nl, cnt, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->rsq_nlist = nl;
    if (nl && (!ids || cap < nl)) return h->fail(LX_ERR_ARG, "id buffer of %llu < %u rows", (unsigned long long)cap, nl);
    if ((rc = rsq_tmp(h, nl))) return rc;
    HIPCHK(h, lx::launch_rsq_group(a, h->rsq_list, nl, h->rsq_tmp, h->rsq_tmp_bytes, ids, h->rsq_ctr, h->stream));
    uint32_t c[kMaxSegments];
    HIPCHK(h, hipMemcpyAsync(c, h->rsq_ctr, 4ull * G, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (uint32_t q = 0; q < G; q++) counts[q] = c[q];
    return 0;
}

int lx_rowseg_la_serve(lx_index *h, uint64_t n, const uint32_t *ids, uint32_t *rows) {
    int rc;
    if ((rc = rs_check(h, 4))) return rc;
    if (n && (!ids || !rows)) return LX_ERR_ARG;
    if (n > 0xFFFFFFFFull) return LX_ERR_ARG;
    HIPCHK(h, lx::launch_rsq_la_gather(rsq_args(h), h->la, h->pstride, ids, (uint32_t)n, rows, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_la_store(lx_index *h, uint64_t n, const uint32_t *ids, const uint32_t *rows) {
    int rc;
    if ((rc = rs_check(h, 4))) return rc;
    if (n && (!ids || !rows)) return LX_ERR_ARG;
    if (n > 0xFFFFFFFFull) return LX_ERR_ARG;
    // the batch's receive area: row i = ids[i] (one store per batch, after lx_rowseg_fc_need)
    if ((rc = grow_scratch(h, &h->rs_rla, &h->rs_rla_cap, std::max<uint64_t>(n, 1) * h->pstride))) return rc;
    HIPCHK(h, lx::launch_rsq_la_store(rsq_args(h), h->rs_rla, h->pstride, ids, (uint32_t)n, rows, h->rs_stamp,
                                      h->rs_lslot, 2 * h->rs_gen + 1, h->stream));
    return 0;
}

int lx_rowseg_fc_unroute(lx_index *h, uint64_t n, const uint32_t *perm, const uint8_t *ans, uint8_t *out) {
    int rc;
    if ((rc = rs_check(h, 4))) return rc;
    if (n && (!perm || !ans || !out)) return LX_ERR_ARG;
    HIPCHK(h, lx::launch_rsq_unroute(perm, ans, n, out, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_rows_unroute(lx_index *h, uint64_t n, const uint32_t *perm, const uint8_t *rows, uint64_t slot_bytes,
                           const uint32_t *len, uint8_t *out, uint32_t *out_len) {
    int rc;
    if ((rc = rs_check(h, 4))) return rc;
    if (n && (!perm || !rows || !len || !out || !out_len)) return LX_ERR_ARG;
    if (slot_bytes % 16 || n > 0x7FFFFFFFull) return h->fail(LX_ERR_ARG, "row slot must be a multiple of 16 bytes");
    HIPCHK(h, lx::launch_rows_unroute(perm, rows, slot_bytes, len, n, out, out_len, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_rowseg_of(const lx_index *h, uint32_t *rank, uint32_t *count) {
    if (!h || !rank || !count) return LX_ERR_ARG;
    *rank = h->rowseg() ? h->rs_rank : 0u;
    *count = h->rowseg() ? h->rs_count : 1u;
    return 0;
}

int lx_rowseg_range(const lx_index *h, uint32_t *lo, uint32_t *hi) {
    if (!h || !lo || !hi) return LX_ERR_ARG;
    if (!h->rowseg() || !h->rs_state) return LX_ERR_STATE;
    *lo = h->rs_lo;
    *hi = h->rs_hi;
    return 0;
}

}  // extern "C"
