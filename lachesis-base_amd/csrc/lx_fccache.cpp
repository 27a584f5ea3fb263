// lx_fccache.cpp -- lx_forkless_cause: ForklessCause for one (a, b) pair, the
// way the unchanged caller asks it.
//
// The reference's callers ask one pair per call: forklessCausedByQuorumOn
// loops over GetFrameRoots(f) (abft/event_processing.go:149-161), the
// election's observedRoots over the previous frame's roots
// (abft/election/election.go:101-123), processKnownRoots replays them after
// every decided frame (abft/event_processing.go:102-146).  vecfc keeps an LRU
// of answers (vecfc/forkless_cause.go:28-38, vecfc/index.go:91-95); here the
// index keeps a result matrix over a working set of events and fills it a
// row at a time on the GPU:
//
//  * working set: up to W events, each in a slot; every event that asks (a)
//    or is asked about (b) joins it, and a newly asked b brings the next
//    kWindow events of its Add order with it (the roots of a frame are asked
//    in insertion order, most of them for the first time by the same event);
//  * M[W][W] bytes in pinned, device-mapped host memory: M[sa][sb] =
//    g7[sb] << 1 | FC(ev[sa], ev[sb]), valid while the column's generation
//    g7[sb] (1..126, bumped when the slot gets a new event) matches -- a slot's
//    reuse invalidates its column without touching W rows;
//  * a miss on a row that was just created (a new asking event) or on the last
//    asking event's row evaluates a against every slot in one k_fc launch
//    (FcArgs.qa_bcast) whose answers land in M directly; a miss on an older
//    row -- processKnownRoots replaying the roots of several frames -- fills
//    the whole matrix with one k_root_fc tile launch (every row and column
//    staged through LDS once per 64 x 64 tile) and k_fc_tile_out.
//
// Exactness: FC(a, b) is immutable once a is indexed (SURVEY Appendix A.5:
// a later LowestAfter entry of b on branch j is the seq of an event a does
// not observe), which is why the reference never invalidates its LRU except
// at Reset; here DropNotFlushed also evicts the dropped events, because dense
// indices are reused afterwards (hashes are not).
#include "lx_index.h"

#include <algorithm>
#include <chrono>
#include <cstring>

using namespace lxi;

namespace {

constexpr uint32_t kWindow = 64;   // events after a newly asked b that join the working set with it

int fcc_quiesce(lx_index *h, FcCache *c);

}  // namespace

struct FcCache {
    uint32_t W = 0, used = 0;
    // slot events and generations: written by the host (pinned), read by the
    // fill kernels from a device mirror -- a fill never reads host memory over
    // the bus; the slots changed since the mirror was written are `dirty`
    // (k_add1_row takes up to kAdd1Delta of them in its arguments, else the
    // mirror is copied before the fill)
    uint32_t *evk = nullptr;                        // event per slot (free: a valid fallback, 0)
    uint8_t *g7 = nullptr;                          // column generation per slot, 1..126
    uint32_t *evk_d = nullptr;                      // device mirrors
    uint8_t *g7_d = nullptr;
    std::vector<uint32_t> dirty;
    std::vector<uint8_t> dmark;
    bool dirty_all = true;
    uint8_t *M = nullptr, *M_dev = nullptr;         // [W][W], pinned and device-mapped: answers land here
    // the last fill: it writes row inflight_sa of M (a tile fill: every row)
    // while the host goes on as soon as its own answer landed; a row is reused
    // (cleared for a new occupant) only after that fill has finished.  A fill
    // of a row cleared for it (a new asking event) is finished once every
    // entry carries the generation it was launched with; any other fill (a
    // refill of a row whose entries already match, a tile fill) by an event
    // recorded after it
    hipEvent_t filled = nullptr;
    bool inflight = false;
    bool inflight_fresh = false;                    // the row was cleared for this fill: generations tell
    bool inflight_tile = false;
    uint32_t inflight_sa = 0, inflight_n = 0;
    std::vector<uint8_t> g7_launch;                 // the column generations the in-flight row fill writes
    lx_index *h = nullptr;
    // k_add1_row's per-slot {count, sum} words (one per 128-B line), zero between launches
    uint32_t *d_rsum = nullptr;
    std::vector<uint32_t> ev;                       // slot -> event (LX_NONE: free)
    std::vector<uint8_t> ref;                       // clock reference bits
    std::vector<uint32_t> free_slots;
    uint32_t hand = 0;
    // event -> slot, indexed by the dense event index (LX_NONE: not in the set)
    std::vector<uint32_t> slot_of;
    uint32_t last_a = LX_NONE, last_sa = LX_NONE;
    // tile fills: partial sums and the cheaters' branch columns (k_root_fc)
    uint32_t *d_psum = nullptr;
    uint64_t psum_cap = 0;
    uint32_t *d_k = nullptr;                         // kcol | kflag | kw, k_cap entries each
    // k_B: the branch count the columns were built for; 0 = stale.  A drop can
    // remove one creator's fork branch and a later Add give the same branch
    // number to another creator's fork, so every DropNotFlushed clears it
    uint32_t n_k = 0, k_B = 0, k_cap = 0;
    lx_fc_stats st{};

    uint32_t find(uint32_t e) const { return e < slot_of.size() ? slot_of[e] : LX_NONE; }
    void map_put(uint32_t e, uint32_t s) {
        if (e >= slot_of.size()) slot_of.resize(std::max<size_t>(2 * slot_of.size(), (size_t)e + 1024), LX_NONE);
        slot_of[e] = s;
    }
    void map_erase(uint32_t e) {
        if (e < slot_of.size()) slot_of[e] = LX_NONE;
    }
    void mark(uint32_t s) {
        if (!dmark[s]) {
            dmark[s] = 1;
            dirty.push_back(s);
        }
    }
    void free_slot(uint32_t s) {
        map_erase(ev[s]);
        ev[s] = LX_NONE;
        evk[s] = 0;
        mark(s);
        free_slots.push_back(s);
        if (last_sa == s) last_a = last_sa = LX_NONE;
    }
    // a slot for event e (clock replacement; never p0 or p1)
    uint32_t insert(uint32_t e, uint32_t p0, uint32_t p1) {
        uint32_t s;
        if (!free_slots.empty()) {
            s = free_slots.back();
            free_slots.pop_back();
        } else if (used < W) {
            s = used++;
        } else {
            for (;;) {
                const uint32_t x = hand;
                hand = (hand + 1) % W;
                if (x == p0 || x == p1) continue;
                if (ref[x]) { ref[x] = 0; continue; }
                s = x;
                break;
            }
            free_slot(s);
            free_slots.pop_back();
        }
        ev[s] = e;
        evk[s] = e;
        mark(s);
        map_put(e, s);
        // 1..126: a row fill writes 0xFF for a query it cannot answer, and
        // 0xFF >> 1 = 127 must never equal a valid generation
        g7[s] = (uint8_t)(g7[s] % 126u + 1u);
        // row s is cleared for its new occupant (and, when the generation
        // wraps, column s in every row): the fill in flight must not be
        // writing them any more
        if (inflight && (inflight_tile || s == inflight_sa || g7[s] == 1)) (void)fcc_quiesce(h, this);
        if (g7[s] == 1)   // the generation wrapped: entries of an old occupant could match again
            for (uint32_t r = 0; r < W; r++) M[(uint64_t)r * W + s] = 0;
        memset(M + (uint64_t)s * W, 0, W);
        ref[s] = 1;
        return s;
    }
    void clear() {
        std::fill(slot_of.begin(), slot_of.end(), LX_NONE);
        std::fill(ev.begin(), ev.end(), LX_NONE);
        for (uint32_t s = 0; s < W; s++) evk[s] = 0;
        dirty_all = true;
        std::fill(ref.begin(), ref.end(), 0);
        free_slots.clear();
        used = 0;
        hand = 0;
        last_a = last_sa = LX_NONE;
        k_B = 0;
    }
};

namespace {

void fcc_free(FcCache *c) {
    if (!c) return;
    for (void *p : {(void *)c->evk, (void *)c->g7, (void *)c->M})
        if (p) (void)hipHostFree(p);
    if (c->evk_d) (void)hipFree(c->evk_d);
    if (c->g7_d) (void)hipFree(c->g7_d);
    if (c->filled) (void)hipEventDestroy(c->filled);
    if (c->d_rsum) (void)hipFree(c->d_rsum);
    if (c->d_psum) (void)hipFree(c->d_psum);
    if (c->d_k) (void)hipFree(c->d_k);
    delete c;
}

int fcc_make(lx_index *h) {
    if (h->fcc) return 0;
    const uint32_t W = h->fcc_slots;
    FcCache *c = new FcCache();
    c->W = W;
    c->h = h;
    void *d = nullptr;
    auto pin = [&](void **host, void **dev, uint64_t bytes) -> hipError_t {
        hipError_t e = hipHostMalloc(host, bytes, hipHostMallocMapped);
        if (e != hipSuccess) return e;
        return hipHostGetDevicePointer(dev, *host, 0);
    };
    hipError_t e = hipHostMalloc((void **)&c->evk, 4ull * W, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->g7, W, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void **)&c->evk_d, 4ull * W);
    if (e == hipSuccess) e = hipMalloc((void **)&c->g7_d, W);
    if (e == hipSuccess) { e = pin((void **)&c->M, &d, (uint64_t)W * W); c->M_dev = static_cast<uint8_t *>(d); }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->filled, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc((void **)&c->d_rsum, 8ull * kAdd1PsumStride * W);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_rsum, 0, 8ull * kAdd1PsumStride * W, h->stream);
    if (e != hipSuccess) {
        fcc_free(c);
        return h->hip(e, "ForklessCause cache (pinned memory)");
    }
    memset(c->g7, 0, W);
    memset(c->M, 0, (uint64_t)W * W);
    c->dmark.assign(W, 0);
    c->g7_launch.assign(W, 0);
    c->ev.assign(W, LX_NONE);
    c->ref.assign(W, 0);
    c->clear();
    c->st.slots = W;
    h->fcc = c;
    return 0;
}

// the cheaters' branch columns for k_root_fc, grouped by creator, original first
int fcc_cheaters(lx_index *h, FcCache *c) {
    if (c->k_B == h->B) return 0;
    std::vector<uint32_t> col, flag, kw;
    for (uint32_t v = 0; v < h->V; v++) {
        const auto &l = h->by_creator[v];
        if (l.size() < 2) continue;
        for (size_t i = 0; i < l.size(); i++) {
            col.push_back(l[i]);
            flag.push_back((i == 0 ? 1u : 0u) | (i + 1 == l.size() ? 2u : 0u));
            kw.push_back(i + 1 == l.size() ? h->weights[v] : 0u);
        }
    }
    c->n_k = (uint32_t)col.size();
    if (c->n_k > c->k_cap) {
        if (c->d_k) {
            HIPCHK(h, hipStreamSynchronize(h->stream));
            (void)hipFree(c->d_k);
        }
        c->d_k = nullptr;
        c->k_cap = 0;
        HIPCHK(h, hipMalloc((void **)&c->d_k, 12ull * c->n_k));
        c->k_cap = c->n_k;
    }
    if (c->n_k) {
        std::vector<uint32_t> all(col);
        all.insert(all.end(), flag.begin(), flag.end());
        all.insert(all.end(), kw.begin(), kw.end());
        // sized for this B: the copy runs before any tile launch on the stream
        HIPCHK(h, hipMemcpyAsync(c->d_k, all.data(), 4ull * all.size(), hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    c->k_B = h->B;
    return 0;
}

// the device mirror of the slots brought up to date (stream-ordered before the
// fill that follows; the host waits for that fill's answer, so the copy has
// read the pinned arrays before the host changes them again)
int fcc_sync_mirror(lx_index *h, FcCache *c) {
    if (!c->dirty_all && c->dirty.empty()) return 0;
    HIPCHK(h, hipMemcpyAsync(c->evk_d, c->evk, 4ull * c->W, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(c->g7_d, c->g7, c->W, hipMemcpyHostToDevice, h->stream));
    for (uint32_t s : c->dirty) c->dmark[s] = 0;
    c->dirty.clear();
    c->dirty_all = false;
    return 0;
}

// a against every slot in use: one k_fc launch, answers into M's row sa.  The
// asking event travels in the kernel arguments: the host may move on to the
// next miss (and its next a) while this fill still runs
int fcc_row(lx_index *h, FcCache *c, uint32_t a, uint32_t sa) {
    FcArgs f;
    int rc = lx_fc_args(h, c->used, c->evk_d, c->evk_d, c->M_dev + (uint64_t)sa * c->W, nullptr, &f);
    if (rc) return rc;
    f.qa_bcast = 1;
    f.qa_imm = a;
    f.out_tag = c->g7_d;
    f.status = h->status + 2;   // the pinned-path sink: every slot holds a known event
    HIPCHK(h, lx::launch_fc(f, h->ncols, h->B > h->V, h->stream));
    c->st.row_fills++;
    c->st.pairs += c->used;
    return 0;
}

// every slot against every slot: k_root_fc tiles + k_fc_tile_out into M
int fcc_tile(lx_index *h, FcCache *c) {
    int rc;
    if ((rc = fcc_cheaters(h, c))) return rc;
    const uint32_t n = c->used, words = (n + 31) / 32, rp = words * 32;
    const uint32_t ncols = (h->V + 31) / 32 * 32;
    const uint32_t splits = lx::root_fc_splits(n, n, ncols);
    const uint32_t col_split = ((ncols + splits - 1) / splits + 31) / 32 * 32;
    const uint32_t n_split = (ncols + col_split - 1) / col_split;
    const uint64_t need = (uint64_t)n_split * n * rp;
    if (need > c->psum_cap) {
        if (c->d_psum) {
            HIPCHK(h, hipStreamSynchronize(h->stream));
            (void)hipFree(c->d_psum);
        }
        c->d_psum = nullptr;
        c->psum_cap = 0;
        HIPCHK(h, dalloc(&c->d_psum, need));
        c->psum_cap = need;
    }
    RootFcArgs r{};
    r.hb = h->hb;
    r.la = h->la;
    r.stride = h->pstride;
    r.cand = c->evk_d;
    r.n_cand = n;
    r.roots = c->evk_d;
    r.n_roots = n;
    r.roots_fallback = c->evk[0];
    r.ncols = ncols;
    r.wpad = h->wpad;
    r.quorum = h->quorum;
    r.n_k = c->n_k;
    r.kcol = c->d_k;
    r.kflag = c->d_k + c->n_k;
    r.kw = c->d_k + 2ull * c->n_k;
    r.ev_branch = h->ev_branch;
    r.psum = c->d_psum;
    r.words = words;
    r.col_split = col_split;
    r.n_split = n_split;
    HIPCHK(h, lx::launch_root_fc(r, h->B > h->V, h->pack16 && h->max_seq <= 0xFFFFu, h->stream));
    HIPCHK(h, lx::launch_fc_tile_out(c->d_psum, n_split, n, rp, n, h->quorum, c->g7_d, c->M_dev, c->W, h->stream));
    c->st.tile_fills++;
    c->st.pairs += (uint64_t)n * n;
    return 0;
}

// the last fill has finished writing M (by the time the caller asks again it
// normally has): a fill of a freshly cleared row once every entry of its row
// carries the generation it was launched with (the entries were 0 before it);
// a refill of a row whose entries already matched, or a tile fill, by its event
int fcc_quiesce(lx_index *h, FcCache *c) {
    if (!c->inflight) return 0;
    const auto tq = std::chrono::steady_clock::now();
    if (!c->inflight_tile && c->inflight_fresh) {
        const volatile uint8_t *row = c->M + (uint64_t)c->inflight_sa * c->W;
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t s = 0;
        for (uint32_t k = 0; s < c->inflight_n; k++) {
            if ((row[s] >> 1) == c->g7_launch[s]) {
                s++;
                continue;
            }
            if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                HIPCHK(h, hipStreamSynchronize(h->stream));
                break;
            }
        }
    } else {
        HIPCHK(h, hipEventSynchronize(c->filled));
    }
    c->inflight = false;
    c->inflight_fresh = c->inflight_tile = false;
    c->st.quiesce_ns +=
        (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tq).count();
    return 0;
}

// wait for M[sa][sb] to carry the column's generation (the answer of the fill
// just enqueued): a spin on pinned memory returns ~5 us sooner than a stream
// synchronization (scripts/probes/sync_latency.hip); on timeout the stream is
// synchronized, which also reports a failed launch
int fcc_wait_answer(lx_index *h, FcCache *c, uint32_t sa, uint32_t sb) {
    const volatile uint8_t *m = c->M + (uint64_t)sa * c->W + sb;
    const uint8_t want = c->g7[sb];
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0;; k++) {
        if ((*m >> 1) == want) return 0;
        if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) break;
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    c->inflight = false;
    return 0;
}

inline bool fcc_hit(FcCache *c, uint32_t a, uint32_t b, uint8_t *out) {
    const uint32_t sa = a == c->last_a ? c->last_sa : c->find(a);
    if (sa == LX_NONE) return false;
    const uint32_t sb = c->find(b);
    if (sb == LX_NONE) return false;
    const uint8_t m = c->M[(uint64_t)sa * c->W + sb];
    if ((m >> 1) != c->g7[sb]) return false;
    c->ref[sa] = c->ref[sb] = 1;
    c->last_a = a;
    c->last_sa = sa;
    *out = m & 1u;
    return true;
}

int fcc_query(lx_index *h, uint32_t a, uint32_t b, uint8_t *out) {
    FcCache *c = h->fcc;
    c->st.calls++;
    int rc;
    const auto t_miss = std::chrono::steady_clock::now();
    if (c->inflight) {
        // the last fill may still be writing this entry (the caller returned as
        // soon as its own answer landed): when that fill answers it -- its row
        // (or the tile), a column whose generation has not changed since the
        // launch -- wait for the entry alone, then it is a hit.  (A tag that
        // matches is always a right answer: the row belongs to the same asking
        // event since its clear, and FC(a, b) never changes; only reusing a
        // row needs the whole fill finished, insert() waits for that.)
        const uint32_t sa = c->find(a), sb = c->find(b);
        if (sa != LX_NONE && sb != LX_NONE && (c->inflight_tile || sa == c->inflight_sa) && sa < c->inflight_n &&
            sb < c->inflight_n && c->g7_launch[sb] == c->g7[sb]) {
            if ((rc = fcc_wait_answer(h, c, sa, sb))) return rc;
            if (fcc_hit(c, a, b, out)) {
                c->st.hits++;
                return 0;
            }
        }
    }
    HIPCHK(h, set_dev(h->device));
    // (the pending run is launched with or before the fill below: the fills read
    // rows of the events it adds; the slot bookkeeping here is host-only)
    uint32_t sa = c->find(a);
    const bool a_new = sa == LX_NONE;
    if (a_new) sa = c->insert(a, LX_NONE, LX_NONE);
    uint32_t sb = c->find(b);
    if (sb == LX_NONE) {
        sb = c->insert(b, sa, LX_NONE);
        for (uint64_t e = (uint64_t)b + 1; e < (uint64_t)b + kWindow && e < h->n_events; e++)
            if (c->find((uint32_t)e) == LX_NONE) c->insert((uint32_t)e, sa, sb);
    }
    // a new asking event that is the pending run's only event (Add, then the
    // caller's first ForklessCause): one launch adds it and fills its row; the
    // slots changed since the mirror was written travel in its arguments
    const auto t_launch = std::chrono::steady_clock::now();
    rc = 1;
    if (a_new && !c->dirty_all && c->dirty.size() <= kAdd1Delta) {
        Add1Delta d{};
        d.n = (uint32_t)c->dirty.size();
        for (uint32_t i = 0; i < d.n; i++) {
            const uint32_t x = c->dirty[i];
            d.slot[i] = x;
            d.ev[i] = c->evk[x];
            d.tag[i] = c->g7[x];
        }
        rc = flush_add1_row(h, a, c->evk_d, c->used, c->g7_d, c->M_dev + (uint64_t)sa * c->W, c->d_rsum, &d);
        if (rc == 0) {   // the kernel stores them into the mirror
            for (uint32_t x : c->dirty) c->dmark[x] = 0;
            c->dirty.clear();
        }
    }
    const bool fused = rc == 0;
    if (fused) c->st.fused++;
    bool tile = false;
    if (rc == 1) {
        if ((rc = flush_pending(h)) || (rc = fcc_sync_mirror(h, c))) return rc;
        if (a_new || a == c->last_a) {
            rc = fcc_row(h, c, a, sa);
        } else {
            rc = fcc_tile(h, c);
            tile = true;
        }
    } else if (!rc) {
        c->st.row_fills++;
        c->st.pairs += c->used;
    }
    if (rc) return rc;
    c->inflight = true;
    c->inflight_fresh = !tile && a_new;   // k_add1_row runs only for a new asking event
    c->inflight_tile = tile;
    c->inflight_sa = sa;
    c->inflight_n = c->used;
    memcpy(c->g7_launch.data(), c->g7, c->used);
    if (!c->inflight_fresh) HIPCHK(h, hipEventRecord(c->filled, h->stream));
    const auto t_wait = std::chrono::steady_clock::now();
    c->st.launch_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_wait - t_launch).count();
    if ((rc = fcc_wait_answer(h, c, sa, sb))) return rc;
    const auto t_end = std::chrono::steady_clock::now();
    c->st.miss_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_end - t_miss).count();
    c->st.wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_end - t_wait).count();
    const uint8_t m = c->M[(uint64_t)sa * c->W + sb];
    if ((m >> 1) != c->g7[sb]) return h->fail(LX_ERR_STATE, "ForklessCause cache: fill left (%u, %u) unanswered", a, b);
    c->ref[sa] = c->ref[sb] = 1;
    c->last_a = a;
    c->last_sa = sa;
    *out = m & 1u;
    return 0;
}

}  // namespace

void fcc_destroy(lx_index *h) {
    if (h->fcc) (void)hipStreamSynchronize(h->stream);   // no fill in flight afterwards
    fcc_free(h->fcc);
    h->fcc = nullptr;
}

void fcc_clear(lx_index *h) {
    if (!h->fcc) return;
    (void)fcc_quiesce(h, h->fcc);
    h->fcc->clear();
}

void fcc_forget_from(lx_index *h, uint64_t n) {
    FcCache *c = h->fcc;
    if (!c) return;
    (void)fcc_quiesce(h, c);
    for (uint32_t s = 0; s < c->used; s++)
        if (c->ev[s] != LX_NONE && c->ev[s] >= n) c->free_slot(s);
    c->k_B = 0;   // the branch -> creator map may change under the same B
}

extern "C" {

int lx_forkless_cause(lx_index *h, uint32_t a, uint32_t b, uint8_t *out) {
    if (!h || !out) return LX_ERR_ARG;
    // hit path first: the cache exists only for whole, non-segmented handles, and
    // holds only events < n_events (dropped ones are forgotten), so an unknown
    // event misses here and is reported below
    if (FcCache *c = h->fcc; c && !h->loading && fcc_hit(c, a, b, out)) {
        c->st.calls++;
        c->st.hits++;
        return 0;
    }
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "ForklessCause before lx_reset");
    if (h->loading) return h->fail(LX_ERR_STATE, "index is loading (lx_load_finish first)");
    if (a >= h->n_events || b >= h->n_events)
        return h->fail(LX_ERR_ARG, "ForklessCause on an unknown event");   // forkless_cause.go:43-61 (crit)
    if (h->sharded() || h->rowseg() || !h->fcc_slots) return lx_forkless_cause_batch(h, 1, &a, &b, out);
    if (!h->fcc) {
        // W^2 bytes of pinned host memory (64 MiB at the default 8192 slots):
        // when the host cannot pin them, the handle answers without the cache
        int rc = fcc_make(h);
        if (rc == LX_ERR_NOMEM) {
            h->fcc_slots = 0;
            return lx_forkless_cause_batch(h, 1, &a, &b, out);
        }
        if (rc) return rc;
        if (fcc_hit(h->fcc, a, b, out)) return h->fail(LX_ERR_STATE, "ForklessCause cache: hit in an empty cache");
    }
    return fcc_query(h, a, b, out);
}

int lx_fc_cache_stats(const lx_index *h, lx_fc_stats *out) {
    if (!h || !out) return LX_ERR_ARG;
    if (h->fcc) {
        *out = h->fcc->st;
        out->slots_used = h->fcc->used - (uint32_t)h->fcc->free_slots.size();
    } else {
        *out = lx_fc_stats{};
        out->slots = h->fcc_slots;
    }
    return 0;
}

}  // extern "C"
