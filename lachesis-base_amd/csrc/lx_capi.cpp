// lx_capi.cpp -- host engine behind the C ABI (include/lachesis_hip.h).
//
// Mirrors the lifecycle of vecfc.Index / vecengine.Engine (Reset, Add, Flush,
// DropNotFlushed, ForklessCause, getters) on top of the device planes of
// lx_internal.h.  Host state is O(branches); all per-event work is on the GPU.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "lx_index.h"

using namespace lxi;

// Host-time counters of the small Add path (make hprof: build_hprof/, read by
// lx_host_prof; absent from the default build)
#ifdef LX_HOST_PROF
#include <x86intrin.h>
static uint64_t g_hprof[16];
#define HP_T(v) const uint64_t v = __rdtsc()
#define HP_ADD(k, t0) (g_hprof[k] += __rdtsc() - (t0))
#define HP_CNT(k, x) (g_hprof[k] += (x))
extern "C" void lx_host_prof(uint64_t out[16], int reset) {
    memcpy(out, g_hprof, sizeof g_hprof);
    if (reset) memset(g_hprof, 0, sizeof g_hprof);
}
#else
#define HP_T(v)
#define HP_ADD(k, t0)
#define HP_CNT(k, x)
#endif

// Between lx_load_rows and lx_load_finish the branch table, B, the cheater
// tables and the branch lengths are not rebuilt yet: every entry point that
// reads or changes the epoch refuses (the load is finished or reset first).
#define NOT_LOADING(h)                                                                            \
    do {                                                                                          \
        if ((h)->loading) return (h)->fail(LX_ERR_STATE, "index is loading (lx_load_finish first)"); \
    } while (0)
// entry points that read whole rows of any event: not on a row-segment rank
#define WHOLE_INDEX(h)                                                                            \
    do {                                                                                          \
        if ((h)->rowseg()) return (h)->fail(LX_ERR_STATE, "needs a whole index (a row-segment rank holds its own rows)"); \
    } while (0)

// index handles alive in this process (the row server's option get_server = 1)
static std::atomic<int> g_live_handles{0};

namespace {

void free_wb(lx_index *h) {
    void *p[] = {h->wb_flag, h->wb_pos, h->wb_la_rows, h->wb_hb_rows, h->wb_buf, h->wb_len, h->wb_la_off,
                 h->wb_hb_off, h->wb_tmp};
    for (void *x : p)
        if (x) (void)hipFree(x);
    h->wb_flag = h->wb_pos = h->wb_la_rows = h->wb_hb_rows = h->wb_buf = nullptr;
    h->wb_len = h->wb_la_off = h->wb_hb_off = nullptr;
    h->wb_tmp = nullptr;
    h->wb_cap = h->wb_buf_cap = 0;
    h->wb_tmp_bytes = 0;
    h->wb_ready = false;
}

void free_all(lx_index *h) {
    free_wb(h);
    rs_planes_free(h);   // a row-segment rank's hb / la are virtual bases into its own allocations
    void *ptrs[] = {h->hb, h->la, h->ev_creator, h->ev_seq, h->ev_branch, h->ev_bbefore, h->ev_sp,
                    h->first_child, h->first_root, h->branch_first, h->branch_creator, h->branch_len, h->brow,
                    h->wpad, h->col_list, h->cheat_off, h->cheat_br, h->cheat_creator, h->b_creator, h->b_seq,
                    h->b_poff, h->b_par, h->b_isfork, h->b_rank, h->b_tmpbr, h->b_jmp, h->b_rec, h->scan_tmp,
                    h->q_a, h->q_b, h->q_out, h->b_crec};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    void *tptrs[] = {h->tail_zw, h->tail_lo, h->tail_cmin, h->wire_flag};
    for (void *p : tptrs)
        if (p) (void)hipFree(p);
    h->tail_zw = h->tail_lo = h->tail_cmin = h->wire_flag = nullptr;
    h->tail_cap = 0;
    void *lptrs[] = {h->cheat_brl, h->cheat_crl, h->cmap, h->lap, h->wloc, h->cheat_of, h->fk_w, h->fk_c, h->fk_wch};
    for (void *p : lptrs)
        if (p) (void)hipFree(p);
    h->cheat_brl = h->cheat_crl = h->cmap = h->lap = h->wloc = nullptr;
    void *gptrs[] = {h->seg_jt, h->seg_cnt, h->seg_mf, h->seg_plist, h->seg_elist};
    for (void *p : gptrs)
        if (p) (void)hipFree(p);
    h->seg_jt = h->seg_cnt = h->seg_mf = h->seg_plist = h->seg_elist = nullptr;
    h->seg_jt_cap = h->seg_cnt_cap = h->seg_mf_cap = h->seg_plist_cap = h->seg_elist_cap = 0;
    rs_free(h);
    h->fk_w = h->fk_c = h->fk_wch = nullptr;
    h->fk_cap = 0;
    h->fk_hi4 = 0;
    h->cheat_of = nullptr;
    h->cheat_of_cap = 0;
    h->cmap_cap = 0;
    for (uint32_t *p : h->sc_rows)
        if (p) (void)hipFree(p);
    void *sptrs[] = {h->sc_flag, h->sc_pos, h->sc_cols, h->sc_tmp};
    for (void *p : sptrs)
        if (p) (void)hipFree(p);
    h->sc_rows.clear();
    h->sc_nrows.clear();
    h->sc_flag = h->sc_pos = h->sc_cols = nullptr;
    h->sc_tmp = nullptr;
    h->sc_cap = 0;
    h->sc_tmp_bytes = 0;
    h->sc_events = ~0ull;
    h->sc_cols_B = 0;
    for (void *p : {(void *)h->sx_len, (void *)h->sx_dmin, (void *)h->sx_rows, (void *)h->sx_meta})
        if (p) (void)hipFree(p);
    h->sx_len = h->sx_dmin = h->sx_rows = h->sx_meta = nullptr;
    h->sx_cap = 0;
    h->sx_rows_cap = h->sx_meta_cap = 0;
    h->sx_full = true;
    h->sx_active = false;
    h->hb = h->la = nullptr;
    h->ev_creator = h->ev_seq = h->ev_branch = h->ev_bbefore = h->ev_sp = h->first_child = nullptr;
    h->first_root = h->branch_first = h->branch_creator = h->branch_len = h->brow = h->wpad = h->col_list = nullptr;
    h->cheat_off = h->cheat_br = h->cheat_creator = nullptr;
    h->b_creator = h->b_seq = h->b_poff = h->b_par = h->b_isfork = h->b_rank = h->b_tmpbr = h->b_jmp = nullptr;
    h->b_rec = nullptr;
    h->b_crec = nullptr;
    h->scan_tmp = nullptr;
    h->q_a = h->q_b = nullptr;
    h->q_out = nullptr;
    h->n_cap = h->stride = h->pstride = h->s_cap = 0;
    h->batch_cap = h->par_cap = h->q_cap = h->cheat_cap = 0;
    h->scan_bytes = 0;
}

// a shard's produced LowestAfter rows lap[(col * s_cap + s) * stride + j] in a
// new shape (local columns, seq capacity, branch capacity), contents kept
int relayout_lap(lx_index *h, uint32_t ncol, uint32_t nscap, uint32_t nstride) {
    uint32_t *n = nullptr;
    const uint64_t words = (uint64_t)ncol * nscap * nstride;
    HIPCHK(h, dalloc(&n, words));
    HIPCHK(h, hipMemsetAsync(n, 0, words * 4, h->stream));
    if (h->lap) {
        const uint32_t oc = std::min(h->pstride, ncol), os = std::min(h->s_cap, nscap);
        for (uint32_t k = 0; k < oc && os; k++)
            HIPCHK(h, lx::launch_copy_rows(n + (uint64_t)k * nscap * nstride, nstride,
                                           h->lap + (uint64_t)k * h->s_cap * h->stride, h->stride, os,
                                           std::min(h->stride, nstride), h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(h->lap);
    }
    h->lap = n;
    return 0;
}

// per-event arrays + planes for n_cap events (copies the first `keep` events)
int grow_events(lx_index *h, uint64_t need) {
    if (need <= h->n_cap) return 0;
    uint64_t cap = std::max<uint64_t>({need, h->n_cap + h->n_cap / 2, 4096});
    uint64_t keep = h->hwm;
    uint32_t **arrs[] = {&h->ev_creator, &h->ev_seq, &h->ev_branch, &h->ev_bbefore, &h->ev_sp, &h->first_child};
    for (uint32_t **a : arrs) {
        uint32_t *n = nullptr;
        HIPCHK(h, dalloc(&n, cap));
        if (*a && keep) HIPCHK(h, hipMemcpyAsync(n, *a, keep * 4, hipMemcpyDeviceToDevice, h->stream));
        if (*a) { HIPCHK(h, hipStreamSynchronize(h->stream)); (void)hipFree(*a); }
        *a = n;
    }
    HIPCHK(h, lx::launch_fill_u32(h->first_child + keep, cap - keep, LX_NONE, h->stream));
    // (a row-segment rank allocates the planes of its own rows when it takes
    // its batch: rs_planes)
    uint32_t **planes[] = {&h->hb, &h->la};
    for (uint32_t **p : planes) {
        if (h->rowseg()) break;
        uint32_t *n = nullptr;
        HIPCHK(h, dalloc(&n, cap * h->pstride));
        HIPCHK(h, hipMemsetAsync(n, 0, cap * h->pstride * 4, h->stream));
        if (*p && keep) HIPCHK(h, hipMemcpyAsync(n, *p, keep * h->pstride * 4, hipMemcpyDeviceToDevice, h->stream));
        if (*p) { HIPCHK(h, hipStreamSynchronize(h->stream)); (void)hipFree(*p); }
        *p = n;
    }
    h->n_cap = cap;
    return 0;
}

// LowestAfter tail state sized to the branch capacity; a new table starts at
// zw = 0 (the next pass re-zeroes every unobserved tail: always correct)
int ensure_tail(lx_index *h) {
    if (h->tail_cap >= h->stride && h->tail_zw) return 0;
    void *tptrs[] = {h->tail_zw, h->tail_lo, h->tail_cmin};
    if (h->tail_zw) HIPCHK(h, hipStreamSynchronize(h->stream));
    for (void *p : tptrs)
        if (p) (void)hipFree(p);
    h->tail_zw = h->tail_lo = h->tail_cmin = nullptr;
    const uint64_t t = h->stride;
    HIPCHK(h, dalloc(&h->tail_zw, t * t));
    HIPCHK(h, dalloc(&h->tail_lo, t * t));
    HIPCHK(h, dalloc(&h->tail_cmin, t));
    HIPCHK(h, hipMemsetAsync(h->tail_zw, 0, t * t * 4, h->stream));
    h->tail_cap = h->stride;
    return 0;
}

int la_tail(lx_index *h, hipStream_t s) {
    int rc;
    if ((rc = ensure_tail(h))) return rc;
    TailArgs t{};
    t.la = h->la;
    t.hb = h->hb;
    t.stride = h->pstride;
    t.brow = h->brow;
    t.s_cap = h->s_cap;
    t.branch_first = h->branch_first;
    t.branch_len = h->branch_len;
    t.B = h->B;
    t.zw = h->tail_zw;
    t.lo = h->tail_lo;
    t.cmin = h->tail_cmin;
    t.tcap = h->tail_cap;
    HIPCHK(h, lx::launch_la_tail(t, s));
    h->tail_dirty = true;
    return 0;
}

// branch capacity (= plane stride) and per-branch arrays
int grow_branches(lx_index *h, uint32_t need) {
    if (need <= h->stride) return 0;
    uint32_t ns = round_up(std::max<uint32_t>(need, h->stride + h->stride / 4), 64);
    uint32_t os = h->stride;
    uint64_t keep = h->hwm;
    if (h->sharded()) {
        // planes hold local columns; the produced LowestAfter rows are B wide
        int rc;
        if (h->lap && (rc = relayout_lap(h, h->pstride, h->s_cap, ns))) return rc;
        uint32_t *nc = nullptr;
        HIPCHK(h, dalloc(&nc, ns));
        HIPCHK(h, lx::launch_fill_u32(nc, ns, LX_NONE, h->stream));
        if (h->cmap) HIPCHK(h, hipMemcpyAsync(nc, h->cmap, (uint64_t)std::min(os, h->cmap_cap) * 4, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (h->cmap) (void)hipFree(h->cmap);
        h->cmap = nc;
        h->cmap_cap = ns;
    } else if (h->hb && !h->rowseg()) {   // (row-segment planes: rs_planes, at the batch)
        uint32_t **planes[] = {&h->hb, &h->la};
        for (uint32_t **p : planes) {
            uint32_t *n = nullptr;
            HIPCHK(h, dalloc(&n, h->n_cap * ns));
            HIPCHK(h, hipMemsetAsync(n, 0, h->n_cap * ns * 4, h->stream));
            HIPCHK(h, lx::launch_copy_rows(n, ns, *p, os, keep, os, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
            (void)hipFree(*p);
            *p = n;
        }
    }
    uint32_t **arrs[] = {&h->branch_first, &h->branch_creator, &h->branch_len, &h->wpad, &h->col_list};
    for (uint32_t **a : arrs) {
        uint32_t *n = nullptr;
        HIPCHK(h, dalloc(&n, ns));
        HIPCHK(h, hipMemsetAsync(n, 0, (uint64_t)ns * 4, h->stream));
        if (*a) HIPCHK(h, hipMemcpyAsync(n, *a, (uint64_t)os * 4, hipMemcpyDeviceToDevice, h->stream));
        if (*a) { HIPCHK(h, hipStreamSynchronize(h->stream)); (void)hipFree(*a); }
        *a = n;
    }
    uint32_t *nb = nullptr;
    HIPCHK(h, dalloc(&nb, (uint64_t)ns * h->s_cap));
    if (h->brow) {
        HIPCHK(h, hipMemcpyAsync(nb, h->brow, (uint64_t)os * h->s_cap * 4, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(h->brow);
    }
    h->brow = nb;
    h->stride = ns;
    if (!h->sharded()) h->pstride = ns;
    return 0;
}

int grow_scap(lx_index *h, uint32_t need) {
    if (need <= h->s_cap) return 0;
    uint32_t ns = std::max<uint32_t>({need, h->s_cap + h->s_cap / 2, 256});
    uint32_t *nb = nullptr;
    HIPCHK(h, dalloc(&nb, (uint64_t)h->stride * ns));
    if (h->brow && h->s_cap) {
        HIPCHK(h, lx::launch_copy_rows(nb, ns, h->brow, h->s_cap, h->stride, h->s_cap, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(h->brow);
    }
    h->brow = nb;
    if (h->sharded()) {
        int rc;
        if ((rc = relayout_lap(h, h->pstride, ns, h->stride))) return rc;
    }
    h->s_cap = ns;
    return 0;
}

// a shard's plane columns (own originals + own fork branches) beyond pstride
int grow_local(lx_index *h, uint32_t need) {
    if (need <= h->pstride) return 0;
    uint32_t np = round_up(std::max<uint32_t>(need, h->pstride + h->pstride / 4), 16);
    int rc;
    if ((rc = relayout_lap(h, np, h->s_cap, h->stride))) return rc;
    uint32_t **planes[] = {&h->hb, &h->la};
    for (uint32_t **p : planes) {
        uint32_t *n = nullptr;
        HIPCHK(h, dalloc(&n, h->n_cap * np));
        HIPCHK(h, hipMemsetAsync(n, 0, h->n_cap * np * 4, h->stream));
        if (*p) HIPCHK(h, lx::launch_copy_rows(n, np, *p, h->pstride, h->hwm, h->pstride, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (*p) (void)hipFree(*p);
        *p = n;
    }
    uint32_t *nw = nullptr;
    HIPCHK(h, dalloc(&nw, np));
    HIPCHK(h, hipMemsetAsync(nw, 0, np * 4ull, h->stream));
    if (h->wloc) HIPCHK(h, hipMemcpyAsync(nw, h->wloc, h->pstride * 4ull, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->wloc) (void)hipFree(h->wloc);
    h->wloc = nw;
    h->pstride = np;
    return 0;
}

int ensure_batch(lx_index *h, uint64_t n, uint64_t npar) {
    if (n > h->batch_cap) {
        uint64_t cap = std::max<uint64_t>(n, 1024);
        uint32_t **arrs[] = {&h->b_creator, &h->b_seq, &h->b_isfork, &h->b_rank, &h->b_tmpbr, &h->b_jmp};
        for (uint32_t **a : arrs) {
            if (*a) (void)hipFree(*a);
            HIPCHK(h, dalloc(a, cap));
        }
        if (h->b_poff) (void)hipFree(h->b_poff);
        HIPCHK(h, dalloc(&h->b_poff, cap + 1));
        if (h->b_rec) (void)hipFree(h->b_rec);
        HIPCHK(h, dalloc(&h->b_rec, (cap + 63) / 64 * 64));   // whole 64-record rounds (round-blocked SoA)
        if (h->b_crec) (void)hipFree(h->b_crec);
        HIPCHK(h, dalloc(&h->b_crec, (cap + 63) / 64 * 64));
        size_t sb = 0;
        HIPCHK(h, lx::scan_tmp_bytes((uint32_t)cap, &sb));
        if (h->scan_tmp) (void)hipFree(h->scan_tmp);
        HIPCHK(h, hipMalloc(&h->scan_tmp, sb ? sb : 1));
        h->scan_bytes = sb;
        h->batch_cap = cap;
    }
    if (npar > h->par_cap) {
        uint64_t cap = std::max<uint64_t>(npar, 4096);
        if (h->b_par) (void)hipFree(h->b_par);
        HIPCHK(h, dalloc(&h->b_par, cap));
        h->par_cap = cap;
    }
    return 0;
}

// column list of this shard + cheater CSR (restricted to owned creators)
int rebuild_columns(lx_index *h) {
    std::vector<uint32_t> cols;
    for (uint32_t b = 0; b < h->B; b++) {
        uint32_t c = h->h_branch_creator[b];
        if (c >= h->own_lo && c < h->own_hi) cols.push_back(b);
    }
    h->ncols = (uint32_t)cols.size();
    if (!cols.empty())
        HIPCHK(h, hipMemcpyAsync(h->col_list, cols.data(), cols.size() * 4, hipMemcpyHostToDevice, h->stream));
    std::vector<uint32_t> off{0}, br, cr;
    for (uint32_t c = h->own_lo; c < h->own_hi; c++) {
        const auto &l = h->by_creator[c];
        if (l.size() < 2) continue;
        cr.push_back(c);
        br.insert(br.end(), l.begin(), l.end());
        off.push_back((uint32_t)br.size());
    }
    h->n_cheat = (uint32_t)cr.size();
    const std::vector<uint32_t> cr_glob = cr;   // cr becomes plane columns below (shards)
    if (h->V > h->cheat_of_cap) {
        if (h->cheat_of) (void)hipFree(h->cheat_of);
        h->cheat_of = nullptr;
        h->cheat_of_cap = 0;
        HIPCHK(h, dalloc(&h->cheat_of, h->V));
        h->cheat_of_cap = h->V;
    }
    std::vector<int32_t> co(h->V, -1);   // alive until the sync below
    for (uint32_t k = 0; k < cr.size(); k++) co[cr[k]] = (int32_t)k;
    HIPCHK(h, hipMemcpyAsync(h->cheat_of, co.data(), h->V * 4ull, hipMemcpyHostToDevice, h->stream));
    uint64_t need = std::max<uint64_t>({off.size(), br.size(), 1});
    if (need > h->cheat_cap) {
        uint64_t cap = std::max<uint64_t>(need * 2, 256);
        uint32_t **arrs[] = {&h->cheat_off, &h->cheat_br, &h->cheat_creator, &h->cheat_brl, &h->cheat_crl};
        for (uint32_t **a : arrs) {
            if (*a) (void)hipFree(*a);
            HIPCHK(h, dalloc(a, cap));
        }
        h->cheat_cap = cap;
    }
    if (h->n_cheat) {
        HIPCHK(h, hipMemcpyAsync(h->cheat_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->cheat_br, br.data(), br.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->cheat_creator, cr.data(), cr.size() * 4, hipMemcpyHostToDevice, h->stream));
        if (h->sharded()) {
            for (auto &x : br) x = h->h_cmap[x];
            for (auto &x : cr) x = h->h_cmap[x];
        }
        HIPCHK(h, hipMemcpyAsync(h->cheat_brl, br.data(), br.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->cheat_crl, cr.data(), cr.size() * 4, hipMemcpyHostToDevice, h->stream));
    }
    // fork-path FC tables (k_fc_fk streams every plane column; <= 64 cheaters
    // per handle, beyond that the cheater fix-up loop of k_fc<.., true>)
    std::vector<uint32_t> fw, fc, wch;   // alive until the sync below
    h->fk_hi4 = 0;
    if (h->fc_fk && h->n_cheat && h->n_cheat <= kFcFkMaxCheaters) {
        const uint32_t npc = h->sharded() ? h->nloc : h->B;
        const uint64_t cap = round_up(npc, 4);
        if (cap > h->fk_cap) {
            uint32_t **arrs[] = {&h->fk_w, &h->fk_c};
            for (uint32_t **a : arrs) {
                if (*a) (void)hipFree(*a);
                *a = nullptr;
            }
            h->fk_cap = 0;
            for (uint32_t **a : arrs) HIPCHK(h, dalloc(a, cap + cap / 2));
            h->fk_cap = cap + cap / 2;
        }
        if (!h->fk_wch) HIPCHK(h, dalloc(&h->fk_wch, kFcFkMaxCheaters));
        fw.assign(cap, 0);
        fc.assign(cap, LX_NONE);
        for (uint32_t b : cols) {
            const uint32_t c = h->h_branch_creator[b];
            const uint32_t pc = h->sharded() ? h->h_cmap[b] : b;
            if (pc >= cap) return h->fail(LX_ERR_STATE, "fork FC table: plane column %u past %u", pc, npc);
            if (co[c] >= 0) fc[pc] = (uint32_t)co[c];
            else fw[pc] = b < h->V ? h->weights[c] : 0u;
        }
        wch.assign(kFcFkMaxCheaters, 0);
        for (uint32_t k = 0; k < h->n_cheat; k++) wch[k] = h->weights[cr_glob[k]];
        HIPCHK(h, hipMemcpyAsync(h->fk_w, fw.data(), cap * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->fk_c, fc.data(), cap * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->fk_wch, wch.data(), wch.size() * 4, hipMemcpyHostToDevice, h->stream));
        h->fk_hi4 = (uint32_t)(cap / 4);
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

BatchArgs batch_args(lx_index *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint32_t *poff,
                     const uint32_t *par) {
    BatchArgs a{};
    a.n = n;
    a.batch_start = (uint32_t)h->n_events;
    a.V = h->V;
    a.B0 = h->B;
    a.creator = creator;
    a.seq = seq;
    a.poff = poff;
    a.par = par;
    a.ev_creator = h->ev_creator;
    a.ev_seq = h->ev_seq;
    a.ev_branch = h->ev_branch;
    a.ev_bbefore = h->ev_bbefore;
    a.ev_sp = h->ev_sp;
    a.first_child = h->first_child;
    a.first_root = h->first_root;
    a.branch_first = h->branch_first;
    a.branch_creator = h->branch_creator;
    a.branch_len = h->branch_len;
    a.brow = h->brow;
    a.s_cap = h->s_cap;
    a.isfork = h->b_isfork;
    a.rank = h->b_rank;
    a.tmp_br = h->b_tmpbr;
    a.jmp = h->b_jmp;
    a.rec = h->b_rec;
    a.status = h->status;
    return a;
}

// The batch walked as h->segments Add-order segments, the partial events'
// rows gathered, LowestAfter filled from the final rows (lx_segment.hip,
// DESIGN.md section 6b).  `ia` is the batch's ordinary walk; timings into
// seg_stats.
// Workgroups of one walk of the batch's columns (launch_index's slice choice,
// rounded to the 8 XCDs)
// -- the CUs a walk holds: 12-column slices count only the real slices (the
// launch's rounding workgroups leave at once and free their CUs for the next
// walk's: V = 1000, 84 slices, three walks side by side)
uint32_t walk_grid(const lx_index *h, uint32_t cpw_hint) {
    const uint32_t nc = h->ncols, cpw = cpw_hint ? cpw_hint : (nc <= 256 ? 1 : nc <= 512 ? 2 : 4);
    const uint32_t slices = (nc + cpw - 1) / cpw;
    return cpw == 12 ? slices : (slices + 7) / 8 * 8;
}

// Segments walked at once on idle compute units: a walk of few columns leaves
// most CUs idle (C2: 100 columns, 104 workgroups on 256 CUs), and its time is
// the batch's DAG depth x pass latency, so G concurrent Add-order segments
// walk ~1/G of the levels each.  Wider slices free more CUs for more
// segments at a longer pass (relative pass costs of 1-, 2- and 4-column
// slices as measured on C2: 1, 1.15, 1.28): the slice width with the
// smallest pass / G wins.  0 when the batch stays one walk; *cpw = the width.
uint32_t auto_segments(const lx_index *h, uint64_t n, uint32_t *cpw) {
    if (!h->seg_auto || h->sharded() || h->rowseg() || h->segments > 1 || !h->ncols) return 0;
    return seg_pick(h, n, cpw);
}

}  // namespace

// the segment count and slice width auto_segments would pick for n events
// (row-segment ranks split their own segment by it too, lx_rowseg.cpp)
uint32_t seg_pick(const lx_index *h, uint64_t n, uint32_t *cpw) {
    static const float kPass[13] = {0, 1.0f, 1.15f, 0, 1.28f, 0, 0, 0, kPass8, 0, 0, 0, kPass12};
    // 8- and 12-column slices: packed 16-bit slots only (every seq <= 0xFFFF, no forks)
    const bool w8 = h->pack16 && h->max_seq <= 0xFFFFu && h->B <= h->V;
    uint32_t best_g = 0;
    float best = 1.0f;   // one walk at the default width
    for (uint32_t c : {1u, 2u, 4u, 8u, 12u}) {
        if ((h->cpw_hint && c != h->cpw_hint) || (c >= 8 && !w8)) continue;
        uint32_t G = std::min<uint32_t>(h->n_cus / walk_grid(h, c), kSegLaunchMax);
        while (G >= 2 && n < (uint64_t)G * kAutoSegEvents) G--;
        if (G >= 2 && kPass[c] / G < best) {
            best = kPass[c] / G;
            best_g = G;
            *cpw = c;
        }
    }
    return best_g;
}

uint32_t seg_walk_grid(const lx_index *h, uint32_t cpw) { return walk_grid(h, cpw); }

namespace {

int seg_walk(lx_index *h, IndexArgs ia, const uint32_t *poff, hipStream_t s, uint32_t G, uint32_t cpw) {
    const uint32_t n = ia.n, bs = ia.batch_start;
    SegArgs a{};
    a.hb = h->hb;
    a.la = h->la;
    a.stride = h->pstride;
    a.B = h->B;
    a.bs = bs;
    a.n = n;
    a.G = G;
    for (uint32_t k = 0; k < G; k++) a.seg_lo[k] = bs + (uint32_t)((uint64_t)n * k / G / 64 * 64);
    a.seg_lo[G] = bs + n;
    a.ev_branch = h->ev_branch;
    a.ev_seq = h->ev_seq;
    a.branch_first = h->branch_first;
    a.branch_len = h->branch_len;
    a.brow = h->brow;
    a.s_cap = h->s_cap;
    a.own_seg = LX_NONE;
    a.per_rank = 1;
    int rc;
    if ((rc = grow_scratch(h, &h->seg_jt, &h->seg_jt_cap, (uint64_t)(G + 1) * h->B)) ||
        (rc = grow_scratch(h, &h->seg_cnt, &h->seg_cnt_cap, (uint64_t)h->B + 2 * kMaxSegments)) ||
        (rc = grow_scratch(h, &h->seg_mf, &h->seg_mf_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->seg_plist, &h->seg_plist_cap, (uint64_t)n)) ||
        (rc = grow_scratch(h, &h->seg_elist, &h->seg_elist_cap, (uint64_t)n)))
        return rc;
    a.jt = h->seg_jt;
    a.cnt = h->seg_cnt;
    a.pcount = h->seg_cnt + h->B;
    a.pflag = h->seg_mf;
    a.plist = h->seg_plist;
    a.elist = h->seg_elist;
    a.ecount = a.pcount + G;
    while (h->seg_ev.size() < 2 * G + 3) {
        hipEvent_t e;
        HIPCHK(h, hipEventCreate(&e));
        h->seg_ev.push_back(e);
    }
    hipEvent_t *ev = h->seg_ev.data();
    HIPCHK(h, lx::launch_seg_tables(a, s));
    // one launch for all G when they fit the CUs side by side (one workgroup
    // per CU each: k_index_segs); otherwise one walk after the other
    ia.cpw_hint = cpw >= 8 && (!ia.pack16 || ia.mask) ? 4 : cpw;
    cpw = ia.cpw_hint;
    const bool conc = G <= kSegLaunchMax && G * walk_grid(h, cpw) <= h->n_cus;
    ia.seg = 1;
    ia.ev_branch = h->ev_branch;
    ia.ev_seq = h->ev_seq;
    if (conc) {
        IndexArgs sk = ia;
        sk.seg_g = G;
        sk.seg_B = a.B;
        for (uint32_t k = 0; k <= G; k++) sk.seg_lo[k] = a.seg_lo[k];
        sk.seg_j = a.jt;
        sk.seg_flag = a.pflag;
        sk.seg_list = a.plist;
        sk.seg_count = a.pcount;
        HIPCHK(h, hipEventRecord(ev[0], s));
        HIPCHK(h, lx::launch_index(sk, s));
        for (uint32_t k = 0; k < G; k++) HIPCHK(h, hipEventRecord(ev[2 * k + 1], s));
    }
    for (uint32_t k = 0; k < G && !conc; k++) {
        IndexArgs sk = ia;
        sk.batch_start = a.seg_lo[k];
        sk.n = a.seg_lo[k + 1] - a.seg_lo[k];
        sk.rec = ia.rec + (a.seg_lo[k] - bs);
        sk.crec = ia.crec ? ia.crec + (a.seg_lo[k] - bs) : nullptr;
        sk.poff_in = poff + (a.seg_lo[k] - bs);
        sk.seg_j = a.jt + (uint64_t)k * a.B;
        sk.seg_flag = a.pflag + (a.seg_lo[k] - bs);
        sk.seg_list = a.plist + (a.seg_lo[k] - bs);
        sk.seg_count = a.pcount + k;
        HIPCHK(h, hipEventRecord(ev[2 * k], s));
        HIPCHK(h, lx::launch_index(sk, s));
        HIPCHK(h, hipEventRecord(ev[2 * k + 1], s));
    }
    uint32_t pc[kMaxSegments], ec[kMaxSegments];
    HIPCHK(h, hipMemcpyAsync(pc, a.pcount, G * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    for (uint32_t k = 0; k < G; k++) HIPCHK(h, lx::launch_seg_partial(a, k, pc[k], s));
    HIPCHK(h, hipEventRecord(ev[2 * G], s));
    for (uint32_t k = 0; k < G; k++) HIPCHK(h, lx::launch_seg_edges(a, k, pc[k], s));
    HIPCHK(h, hipMemcpyAsync(ec, a.ecount, G * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    for (uint32_t k = 0; k < G; k++) HIPCHK(h, lx::launch_seg_la_edge(a, k, ec[k], s));
    HIPCHK(h, hipEventRecord(ev[2 * G + 1], s));
    HIPCHK(h, hipStreamSynchronize(s));
    lx_seg_stats &st = h->seg_stats;
    st = lx_seg_stats{};
    st.segments = G;
    st.one_launch = conc ? 1u : 0u;
    for (uint32_t k = 0; k < G; k++) {
        st.first_event[k] = a.seg_lo[k];
        st.partial[k] = pc[k];
        HIPCHK(h, hipEventElapsedTime(&st.walk_ms[k], ev[conc ? 0 : 2 * k], ev[2 * k + 1]));
    }
    st.first_event[G] = a.seg_lo[G];
    HIPCHK(h, hipEventElapsedTime(&st.partial_ms, ev[2 * G - 1], ev[2 * G]));
    HIPCHK(h, hipEventElapsedTime(&st.la_ms, ev[2 * G], ev[2 * G + 1]));
    return 0;
}

int add_batch_dev(lx_index *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint32_t *poff,
                  const uint32_t *par, uint32_t *err_index) {
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "lx_add_batch before lx_reset");
    if (h->loading) return h->fail(LX_ERR_STATE, "lx_add_batch during a load (lx_load_finish first)");
    if (n == 0) return 0;
    if (h->rowseg()) {
        if (h->n_events || h->rs_state) return h->fail(LX_ERR_STATE, "a row-segment rank takes one batch per epoch");
        if (h->rs_rank >= h->rs_count) return h->fail(LX_ERR_ARG, "seg_rank %u >= seg_count %u", h->rs_rank, h->rs_count);
        if (n < 64ull * h->rs_count) return h->fail(LX_ERR_ARG, "row segments need >= 64 events per rank");
    }
    h->wb_ready = false;
    if (h->n_events + n >= 0xFFFFFFF0ull) return h->fail(LX_ERR_ARG, "too many events in one epoch");
    h->hm_ok = false;           // the device assigns this batch: the host mirror is refreshed on demand
    h->stats_lazy = false;
    int rc;
    if ((rc = grow_events(h, h->n_events + n))) return rc;
    if ((rc = ensure_batch(h, n, 0))) return rc;
    hipStream_t s = h->stream;

    HIPCHK(h, hipEventRecord(h->ev[0], s));
    HIPCHK(h, hipMemsetAsync(h->status, 0, kStatusWords * 4, s));
    HIPCHK(h, hipMemsetAsync(h->status + 8, 0xFF, 8, s));
    BatchArgs a = batch_args(h, n, creator, seq, poff, par);
    HIPCHK(h, lx::launch_batch_prepare(a, h->scan_tmp, h->scan_bytes, s));
    uint32_t st[16];
    uint32_t nforks = 0;
    HIPCHK(h, hipMemcpyAsync(st, h->status, sizeof st, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(&nforks, h->b_rank + (n - 1), 4, hipMemcpyDeviceToHost, s));
    uint32_t npar32 = 0;
    HIPCHK(h, hipMemcpyAsync(&npar32, poff + n, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    uint64_t e64;
    memcpy(&e64, st + 8, 8);
    if (e64 != ~0ull) {
        HIPCHK(h, lx::launch_undo_claims(a, s));
        HIPCHK(h, hipStreamSynchronize(s));
        uint32_t pos = (uint32_t)(e64 >> 8), code = (uint32_t)(e64 & 0xFF);
        if (err_index) *err_index = pos;
        if (code == 2) return h->fail(LX_ERR_ORDER, "event %u: processed out of order, parent not found", pos);
        if (code == 1) return h->fail(LX_ERR_ARG, "event %u: creator idx out of range", pos);
        return h->fail(LX_ERR_EVENT, "event %u: violates seq/self-parent invariants (eventcheck)", pos);
    }
    uint32_t bmax = st[2];
    h->last_npar = npar32;
    uint32_t B_new = h->B + nforks;
    if ((rc = grow_branches(h, B_new))) return rc;
    h->max_seq = std::max(h->max_seq, bmax);
    if ((rc = grow_scap(h, h->max_seq))) return rc;
    a = batch_args(h, n, creator, seq, poff, par);   // pointers may have moved
    a.nofork = (nforks == 0 && B_new == h->V) ? 1u : 0u;
    // compact records for the 8- / 12-column walks: fork-free epoch, every
    // branch and seq within 16 bits (the packed-slot condition)
    h->b_crec_ok = a.nofork && h->B == h->V && h->pack16 && h->max_seq <= 0xFFFFu && B_new <= 0xFFFFu && h->crec_opt;
    a.crec = h->b_crec_ok ? h->b_crec : nullptr;
    // pointer jumping along in-batch self-parent chains: a chain has at most
    // min(n, max seq) events, ceil(log2) + 1 rounds resolve it (k_finalize flags
    // an unresolved event, checked below); none without forks
    uint32_t rounds = 1;
    while (rounds < 32 && (1ull << (rounds - 1)) < std::min<uint64_t>(n, bmax)) rounds++;
    HIPCHK(h, lx::launch_batch_finish(a, a.nofork ? 0u : rounds + 1, s));
    if (nforks) {
        std::vector<uint32_t> cr(nforks), fs(nforks);
        HIPCHK(h, hipMemcpyAsync(cr.data(), h->branch_creator + h->B, nforks * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(fs.data(), h->branch_first + h->B, nforks * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        for (uint32_t i = 0; i < nforks; i++) {
            h->h_branch_creator.push_back(cr[i]);
            h->h_branch_first.push_back(fs[i]);
            h->by_creator[cr[i]].push_back(h->B + i);
            if (h->sharded())
                h->h_cmap.push_back(cr[i] >= h->own_lo && cr[i] < h->own_hi ? h->nloc++ : LX_NONE);
        }
        if (h->sharded()) {
            if ((rc = grow_local(h, h->nloc))) return rc;
            HIPCHK(h, hipMemcpyAsync(h->cmap + h->B, h->h_cmap.data() + h->B, nforks * 4ull, hipMemcpyHostToDevice, s));
        }
    }
    h->B = B_new;
    h->pcols_used = std::max(h->pcols_used, h->sharded() ? h->nloc : h->B);
    if (nforks || h->ncols == 0)
        if ((rc = rebuild_columns(h))) return rc;

    IndexArgs ia{};
    ia.hb = h->hb;
    ia.la = h->la;
    ia.stride = h->pstride;
    ia.cmap = h->sharded() ? h->cmap : nullptr;
    ia.lap = h->sharded() ? h->lap : nullptr;
    ia.lap_stride = h->stride;
    ia.batch_start = (uint32_t)h->n_events;
    ia.n = n;
    ia.rec = h->b_rec;
    ia.crec = h->b_crec_ok ? h->b_crec : nullptr;
    ia.par_in = par;
    ia.poff_in = poff;
    ia.col_list = h->col_list;
    ia.ncols = h->ncols;
    ia.branch_first = h->branch_first;
    ia.brow = h->brow;
    ia.s_cap = h->s_cap;
    ia.mask = (h->B > h->V) ? 1u : 0u;
    ia.cpw_hint = h->cpw_hint;
    ia.pack16 = h->pack16 && h->max_seq <= 0xFFFFu;
    ia.seg_xmap = h->seg_xmap_opt ? 1u : 0u;
    if (ia.cpw_hint >= 8 && (!ia.pack16 || ia.mask)) ia.cpw_hint = 4;   // 8- / 12-column slots: packed, fork-free
    const size_t prof_n = (size_t)kProfBlocks * kProfWaves * kProfSlots;
    if (!h->d_clk) {
        HIPCHK(h, hipMalloc(&h->d_clk, (1 + 3ull * kClkBlocks) * 8));
        HIPCHK(h, hipMemsetAsync(h->d_clk, 0, (1 + 3ull * kClkBlocks) * 8, s));
    }
    ia.clk = h->d_clk;
    if (h->prof) {
        HIPCHK(h, hipMalloc(&ia.prof, prof_n * 8));
        HIPCHK(h, hipMemsetAsync(ia.prof, 0, prof_n * 8, s));
    }
    HIPCHK(h, hipEventRecord(h->ev[1], s));
    if (h->rowseg()) {
        if ((rc = rs_planes(h, n))) return rc;   // own rows only (+ the virtual bases)
        ia.hb = h->hb;
        ia.la = h->la;
        if ((rc = rs_begin(h, ia, poff, s))) return rc;
    } else if (h->segments > 1 && !h->sharded() && n >= 64ull * h->segments) {
        if ((rc = seg_walk(h, ia, poff, s, h->segments, h->cpw_hint))) return rc;
    } else if (h->dbl && !ia.mask && !h->sharded() && h->B <= kDblMaxB && n >= 16ull * h->B && n <= 0xFFFFu &&
               dbl_lds_bytes(n, h->B) <= kDblLds) {
        // few branches, no forks: HB by frontier doubling in one workgroup
        // (the walker's time is levels x pass, and such epochs are deep chains)
        DblArgs da{};
        da.hb = h->hb;
        da.la = h->la;
        da.stride = h->pstride;
        da.bs = (uint32_t)h->n_events;
        da.n = n;
        da.B = h->B;
        da.rec = h->b_rec;
        da.par = par;
        da.poff = poff;
        da.ev_branch = h->ev_branch;
        da.ev_seq = h->ev_seq;
        da.branch_first = h->branch_first;
        da.brow = h->brow;
        da.s_cap = h->s_cap;
        HIPCHK(h, lx::launch_dbl(da, s));
    } else if (uint32_t cpw = 0, G = auto_segments(h, n, &cpw); G) {
        if ((rc = seg_walk(h, ia, poff, s, G, cpw))) return rc;
    } else {
        HIPCHK(h, lx::launch_index(ia, s));
    }
    HIPCHK(h, hipEventRecord(h->ev[2], s));
    if (h->prof) {
        std::vector<unsigned long long> pv(prof_n);
        HIPCHK(h, hipMemcpyAsync(pv.data(), ia.prof, prof_n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        HIPCHK(h, hipFree(ia.prof));
        // summary over workgroups: compute waves (lane sums), loader, drains
        double sum[kProfWaves * kProfSlots] = {0};
        uint32_t nb = 0;
        for (uint32_t b = 0; b < (uint32_t)kProfBlocks; b++) {
            const unsigned long long *pb = pv.data() + (size_t)b * kProfWaves * kProfSlots;
            if (!pb[9]) continue;
            nb++;
            for (int i = 0; i < kProfWaves * kProfSlots; i++) sum[i] += (double)pb[i];
        }
        fprintf(stderr, "[lx_prof] n=%u blocks=%u (means per block)\n", n, nb);
        {
            // the slowest workgroups: wall (max over its waves) and the compute waves' no-record passes
            std::vector<std::pair<double, uint32_t>> wb;
            for (uint32_t b = 0; b < (uint32_t)kProfBlocks; b++) {
                const unsigned long long *pb = pv.data() + (size_t)b * kProfWaves * kProfSlots;
                double wmax = 0;
                for (int w = 0; w < kProfWaves; w++) wmax = std::max(wmax, (double)pb[w * kProfSlots + 9]);
                if (wmax > 0) wb.push_back({wmax, b});
            }
            std::sort(wb.rbegin(), wb.rend());
            for (size_t i = 0; i < wb.size() && i < 6; i++) {
                const unsigned long long *pb = pv.data() + (size_t)wb[i].second * kProfWaves * kProfSlots;
                double norec = 0;
                for (int w = 0; w < kProfWaves; w++)
                    if (pb[w * kProfSlots + 10] == 0) norec += (double)pb[w * kProfSlots + 7];
                fprintf(stderr, "[lx_prof] slow block %u (xcd %u): wall_us=%.0f compute norec=%.0f\n", wb[i].second,
                        wb[i].second % 8, wb[i].first / 100.0, norec);
            }
            if (!wb.empty())
                fprintf(stderr, "[lx_prof] median block wall_us=%.0f\n", wb[wb.size() / 2].first / 100.0);
        }
        for (int w = 0; w < kProfWaves; w++) {
            const double *q = sum + w * kProfSlots;
            if (!q[9]) continue;
            const double role = q[10] / (nb ? nb : 1);
            if (role > 1.5) {
                fprintf(stderr, "[lx_prof] wave %d drain: wall_us=%.0f rounds=%.0f spin=%.0f busy_us=%.0f fills=%.0f brc_miss=%.0f\n",
                        w, q[9] / nb / 100.0, q[3] / nb, q[0] / nb, q[6] / nb / 100.0, q[4] / nb, q[5] / nb);
            } else if (role > 0.5) {
                fprintf(stderr, "[lx_prof] wave %d loader: wall_us=%.0f rounds=%.0f iter=%.0f slot_wait=%.0f sleeps=%.0f\n", w,
                        q[9] / nb / 100.0, q[3] / nb, q[0] / nb, q[1] / nb, q[2] / nb);
            } else {
                fprintf(stderr, "[lx_prof] wave %d: wall_us=%.0f wave_passes=%.0f lane: pass=%.0f spin=%.0f chunk=%.0f done=%.0f slow=%.0f fill=%.0f wm=%.0f norec=%.0f  ns/pass=%.1f\n",
                        w, q[9] / nb / 100.0, q[8] / nb, q[0] / nb, q[1] / nb, q[2] / nb, q[3] / nb, q[4] / nb, q[5] / nb, q[6] / nb,
                        q[7] / nb, q[9] * 10.0 / (q[8] > 0 ? q[8] : 1));
                if (q[14] == 0 && q[15] > 0)
                    fprintf(stderr, "[lx_prof] wave %d blocks ahead of the fetched one: landed records %.1f, issued %.1f; behind it: drained %.1f\n",
                            w, q[11] / q[15], q[12] / q[15], q[13] / q[15]);
                if (q[14] > 0)
                    fprintf(stderr, "[lx_prof] wave %d cycles/pass: fetch=%.0f (record rt %.0f) fold=%.0f (ring rt %.0f) ovf=%.0f complete=%.0f total=%.0f\n", w,
                            q[10] / q[8], q[5] / q[8], q[11] / q[8], q[15] / q[8], q[12] / q[8], q[13] / q[8], q[14] / q[8]);
            }
        }
    }
    if (h->B > h->V && h->n_cheat && !h->rowseg()) {   // a row-segment rank marks its rows at lx_rowseg_finish
        MarkArgs m{};
        m.hb = h->hb;
        m.stride = h->pstride;
        m.cmap = h->sharded() ? h->cmap : nullptr;
        m.batch_start = (uint32_t)h->n_events;
        m.n = n;
        m.V = h->V;
        m.ev_branch = h->ev_branch;
        m.ev_bbefore = h->ev_bbefore;
        m.branch_first = h->branch_first;
        m.n_cheat = h->n_cheat;
        m.cheat_off = h->cheat_off;
        m.cheat_br = h->cheat_br;
        HIPCHK(h, lx::launch_marks(m, s));
    }
    if (!h->sharded() && !h->rowseg() && h->la_tail) {
        if ((rc = la_tail(h, s))) return rc;
    }
    HIPCHK(h, hipEventRecord(h->ev[3], s));
    h->n_events += n;
    h->hwm = std::max(h->hwm, h->n_events);
    HIPCHK(h, hipStreamSynchronize(s));
    uint32_t unresolved = 0;
    HIPCHK(h, hipMemcpy(&unresolved, h->status + 4, 4, hipMemcpyDeviceToHost));
    if (unresolved) return h->fail(LX_ERR_STATE, "branch assignment left %u events unresolved", unresolved);
    float t0 = 0, t1 = 0, t2 = 0;
    HIPCHK(h, hipEventElapsedTime(&t0, h->ev[0], h->ev[1]));
    HIPCHK(h, hipEventElapsedTime(&t1, h->ev[1], h->ev[2]));
    HIPCHK(h, hipEventElapsedTime(&t2, h->ev[2], h->ev[3]));
    h->stats.ms_assign = t0;
    h->stats.ms_index = t1;
    h->stats.ms_marks = t2;
    h->stats.index_launches = 1;
    return 0;
}

}  // namespace

int lx_fc_args(lx_index *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out, uint32_t *partial,
               FcArgs *fa) {
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "ForklessCause before lx_reset");
    NOT_LOADING(h);
    if (h->rowseg() && h->rs_state != 4)
        return h->fail(LX_ERR_STATE, "row-segment rank: ForklessCause before lx_rowseg_finish");
    FcArgs f{};
    f.hb = h->hb;
    f.la = h->la;
    f.stride = h->pstride;
    f.n_events = h->rowseg() ? h->rs_hi : (uint32_t)h->n_events;
    f.ev_lo = h->rowseg() ? h->rs_lo : 0u;
    f.b_stamp = h->rowseg() ? h->rs_stamp : nullptr;
    f.n_all = (uint32_t)h->n_events;
    f.la_recv = h->rowseg() ? h->rs_rla : nullptr;
    f.b_slot = h->rowseg() ? h->rs_lslot : nullptr;
    f.b_arrived = 2 * h->rs_gen + 1;
    f.n = n;
    f.qa = a;
    f.qb = b;
    f.out = out;
    f.partial = partial;
    if (h->sharded()) {
        f.wpad = h->wloc;     // local columns: own originals first
        f.vlo4 = 0;
        f.vhi4 = (h->own_hi - h->own_lo + 3) / 4;
        f.cmap = h->cmap;
    } else {
        f.wpad = h->wpad;
        f.vlo4 = h->own_lo / 4;
        f.vhi4 = (h->own_hi + 3) / 4;
        f.cmap = nullptr;
    }
    f.cheat_brl = h->cheat_brl;
    f.cheat_crl = h->cheat_crl;
    f.fk_w = h->fk_w;
    f.fk_c = h->fk_c;
    f.fk_wch = h->fk_wch;
    f.fk_hi4 = h->fk_hi4;
    f.quorum = h->quorum;
    f.ev_branch = h->ev_branch;
    f.ev_creator = h->ev_creator;
    f.n_cheat = h->n_cheat;
    f.cheat_off = h->cheat_off;
    f.cheat_br = h->cheat_br;
    f.cheat_creator = h->cheat_creator;
    f.own_lo = h->own_lo;
    f.own_hi = h->own_hi;
    f.branch_creator = h->branch_creator;
    f.status = h->status;
    // early exit (k_fc_early: fork-free whole rows of more than 512 columns --
    // launch_fc's 64-lane width, the gate matches what runs): rounds of the
    // first 128, 256, 512 columns and the rest, when the heaviest 512 columns
    // can reach the quorum alone (else no round before the last can decide)
    // Small launches (the FC cache's row fills, calcFrameIdx-sized batches) keep
    // whole rows: all of a row's loads in one round is the shortest latency,
    // and the caller waits for the launch (drop-in C5: 4 rounds cost ~1.4 us
    // per miss)
    if (!partial && !h->sharded() && h->B == h->V && h->fc_early && f.vhi4 - f.vlo4 > 128 && n >= kFcEarlyMinQueries) {
        const uint32_t L = h->fc_early_lanes;   // rounds of 4L, 8L, 16L columns
        uint64_t w128 = 0, w256 = 0, w512 = 0, wt = 0;
        for (uint32_t c = f.vlo4 * 4; c < h->V && c < f.vhi4 * 4; c++) {
            const uint32_t k = c - f.vlo4 * 4;
            wt += h->weights[c];
            if (k < 4 * L) w128 += h->weights[c];
            if (k < 8 * L) w256 += h->weights[c];
            if (k < 16 * L) w512 += h->weights[c];
        }
        if (w512 >= h->quorum && wt - w128 <= 0xFFFFFFFFull) {
            if (!h->d_fc_full) {
                // zeroed and synchronized before any launch can count into it,
                // whatever stream runs that launch
                unsigned long long *p = nullptr;
                HIPCHK(h, hipMalloc((void **)&p, 32));
                hipError_t e = hipMemsetAsync(p, 0, 32, h->stream);
                if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
                if (e != hipSuccess) {
                    (void)hipFree(p);
                    return h->hip(e, "ForklessCause early-exit counters");
                }
                h->d_fc_full = p;
            }
            f.early = 1;
            f.early_rest = (uint32_t)(wt - w128);
            f.early_rest2 = (uint32_t)(wt - w256);
            f.early_rest3 = (uint32_t)(wt - w512);
            f.early_lanes = L;
            f.early_full = h->d_fc_full;
        }
    }
    h->fc_unchecked = true;   // a query it cannot answer flags status[1]; lx_sync reports it
    *fa = f;
    return 0;
}

namespace {

void shard_bounds(const lx_index *h, uint32_t r, uint32_t *lo, uint32_t *hi) {
    auto bound = [&](uint32_t q) {
        return q >= h->shard_count ? h->V : (uint32_t)((uint64_t)h->V * q / h->shard_count) & ~3u;
    };
    *lo = bound(r);
    *hi = bound(r + 1);
}

std::vector<uint32_t> shard_cols(const lx_index *h, uint32_t q) {
    uint32_t lo, hi;
    shard_bounds(h, q, &lo, &hi);
    std::vector<uint32_t> cols;
    for (uint32_t b = 0; b < h->B; b++)
        if (h->h_branch_creator[b] >= lo && h->h_branch_creator[b] < hi) cols.push_back(b);
    return cols;
}

int upload_cols(lx_index *h);
int ensure_shard_cols(lx_index *h);

// rows (events) whose branch belongs to each shard, at the current event count
// (and every shard's column list)
int ensure_shard_rows(lx_index *h) {
    if (h->sc_events == h->n_events && h->sc_B == h->B) return 0;
    const uint32_t n = (uint32_t)h->n_events;
    const uint32_t G = h->shard_count;
    if (n > h->sc_cap || h->sc_rows.size() != G) {
        for (uint32_t *p : h->sc_rows)
            if (p) (void)hipFree(p);
        h->sc_rows.assign(G, nullptr);
        uint64_t cap = std::max<uint64_t>(n, 4096);
        for (uint32_t q = 0; q < G; q++) HIPCHK(h, dalloc(&h->sc_rows[q], cap));
        if (h->sc_flag) (void)hipFree(h->sc_flag);
        if (h->sc_pos) (void)hipFree(h->sc_pos);
        HIPCHK(h, dalloc(&h->sc_flag, cap));
        HIPCHK(h, dalloc(&h->sc_pos, cap));
        size_t sb = 0;
        HIPCHK(h, lx::scan_tmp_bytes((uint32_t)cap, &sb));
        if (h->sc_tmp) (void)hipFree(h->sc_tmp);
        HIPCHK(h, hipMalloc(&h->sc_tmp, sb ? sb : 1));
        h->sc_tmp_bytes = sb;
        h->sc_cap = cap;
    }
    h->sc_nrows.assign(G, 0);
    for (uint32_t q = 0; q < G; q++) {
        uint32_t lo, hi;
        shard_bounds(h, q, &lo, &hi);
        HIPCHK(h, lx::launch_shard_rows(h->ev_branch, h->branch_creator, n, lo, hi, h->sc_flag, h->sc_pos, h->sc_tmp,
                                        h->sc_tmp_bytes, h->sc_rows[q], h->stream));
        if (n) HIPCHK(h, hipMemcpyAsync(&h->sc_nrows[q], h->sc_pos + (n - 1), 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (int rc = upload_cols(h)) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->sc_events = h->n_events;
    h->sc_B = h->B;
    return 0;
}

// the column lists alone (the incremental exchange lists its rows itself)
int ensure_shard_cols(lx_index *h) {
    if (h->sc_cols && h->sc_cols_B == h->B) return 0;
    if (int rc = upload_cols(h)) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

// every shard's column list on the device (rebuilt with the shard rows, when
// the event count or the branch set changed)
int upload_cols(lx_index *h) {
    std::vector<uint32_t> all;
    h->sc_col_off.assign(1, 0);
    for (uint32_t q = 0; q < h->shard_count; q++) {
        std::vector<uint32_t> c = shard_cols(h, q);
        all.insert(all.end(), c.begin(), c.end());
        h->sc_col_off.push_back((uint32_t)all.size());
    }
    if (h->sc_cols) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(h->sc_cols);
    }
    HIPCHK(h, dalloc(&h->sc_cols, all.size()));
    if (!all.empty())
        HIPCHK(h, hipMemcpyAsync(h->sc_cols, all.data(), all.size() * 4, hipMemcpyHostToDevice, h->stream));
    h->sc_cols_B = h->B;
    return 0;
}

int read_u32(lx_index *h, const uint32_t *dev, uint32_t *out) {
    HIPCHK(h, hipMemcpy(out, dev, 4, hipMemcpyDeviceToHost));
    return 0;
}

// the LowestAfter fills of the events added since the last flush (rollback and write-back)
UnfillArgs unfill_args(lx_index *h) {
    UnfillArgs u{};
    u.hb = h->hb;
    u.la = h->la;
    u.stride = h->pstride;
    u.cmap = h->sharded() ? h->cmap : nullptr;
    u.lap = h->sharded() ? h->lap : nullptr;
    u.lap_stride = h->stride;
    u.lo = (uint32_t)h->n_flushed;
    u.hi = (uint32_t)h->n_events;
    u.B = h->B;
    u.ev_seq = h->ev_seq;
    u.ev_branch = h->ev_branch;
    u.ev_bbefore = h->ev_bbefore;
    u.ev_sp = h->ev_sp;
    u.ev_creator = h->ev_creator;
    u.first_child = h->first_child;
    u.first_root = h->first_root;
    u.branch_len = h->branch_len;
    u.branch_first = h->branch_first;
    u.brow = h->brow;
    u.s_cap = h->s_cap;
    u.B_keep = h->B_flushed;
    return u;
}

// ---- write-back helpers
int ensure_wb(lx_index *h, uint64_t n) {
    if (n <= h->wb_cap && h->wb_flag) return 0;
    void *keep_buf = h->wb_buf;
    uint64_t keep_cap = h->wb_buf_cap;
    h->wb_buf = nullptr;
    free_wb(h);
    h->wb_buf = (uint32_t *)keep_buf;
    h->wb_buf_cap = keep_cap;
    const uint64_t cap = std::max<uint64_t>(n, 4096);
    HIPCHK(h, dalloc(&h->wb_flag, cap));
    HIPCHK(h, dalloc(&h->wb_pos, cap));
    HIPCHK(h, dalloc(&h->wb_la_rows, cap));
    HIPCHK(h, dalloc(&h->wb_hb_rows, cap));
    HIPCHK(h, dalloc(&h->wb_len, cap + 1));
    HIPCHK(h, dalloc(&h->wb_la_off, cap + 1));
    HIPCHK(h, dalloc(&h->wb_hb_off, cap + 1));
    size_t tb = 0;
    HIPCHK(h, lx::persist_tmp_bytes((uint32_t)cap, &tb));
    HIPCHK(h, hipMalloc(&h->wb_tmp, tb ? tb : 1));
    h->wb_tmp_bytes = tb;
    h->wb_cap = cap;
    return 0;
}

RowsArgs rows_args(lx_index *h, uint32_t hb, const uint32_t *rows, uint32_t n) {
    RowsArgs a{};
    a.plane = hb ? h->hb : h->la;
    a.stride = h->stride;
    a.rows = rows;
    a.n = n;
    a.B = h->B;
    a.ev_bbefore = h->ev_bbefore;
    a.ev_branch = h->ev_branch;
    a.branch_first = h->branch_first;
    a.hb = hb;
    return a;
}

// encoded rows -> host, in chunks of at most kWbChunk bytes of device staging
constexpr uint64_t kWbChunk = 256ull << 20;

int rows_to_host(lx_index *h, uint32_t hb, const uint32_t *rows, const uint64_t *off_dev, uint32_t n,
                 uint64_t *off_host, uint8_t *bytes) {
    std::vector<uint64_t> off(n + 1);
    HIPCHK(h, hipMemcpyAsync(off.data(), off_dev, (n + 1) * 8ull, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (off_host) memcpy(off_host, off.data(), (n + 1) * 8ull);
    if (!bytes || !n || !off[n]) return 0;
    uint64_t row_max = 0;
    for (uint32_t i = 0; i < n; i++) row_max = std::max(row_max, off[i + 1] - off[i]);
    const uint64_t want = std::max(std::min(off[n], kWbChunk), row_max);
    if (want > h->wb_buf_cap) {
        if (h->wb_buf) (void)hipFree(h->wb_buf);
        h->wb_buf = nullptr;
        h->wb_buf_cap = 0;
        HIPCHK(h, dalloc(&h->wb_buf, (want + 3) / 4));
        h->wb_buf_cap = want;
    }
    for (uint32_t i0 = 0; i0 < n;) {
        uint32_t i1 = i0 + 1;
        while (i1 < n && off[i1 + 1] - off[i0] <= h->wb_buf_cap) i1++;
        RowsArgs a = rows_args(h, hb, rows + i0, i1 - i0);
        HIPCHK(h, lx::launch_encode_rows(a, off_dev + i0, off[i0], h->wb_buf, h->stream));
        HIPCHK(h, hipMemcpyAsync(bytes + off[i0], h->wb_buf, off[i1] - off[i0], hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        i0 = i1;
    }
    return 0;
}

// go-ethereum rlp (v1.9.22) of BranchesInfo{[]idx.Event, []idx.Validator,
// [][]idx.Validator} (vecengine/branches_info.go:9-13): structs and slices are
// lists, uints are minimal big-endian strings (0 = 0x80, < 0x80 = the byte)
void rlp_uint(std::string &o, uint32_t x) {
    if (x == 0) { o.push_back((char)0x80); return; }
    if (x < 0x80) { o.push_back((char)x); return; }
    const int nb = (x >> 24) ? 4 : (x >> 16) ? 3 : (x >> 8) ? 2 : 1;
    o.push_back((char)(0x80 + nb));
    for (int i = nb - 1; i >= 0; i--) o.push_back((char)(x >> (8 * i)));
}

void rlp_list(std::string &o, const std::string &payload) {
    const uint64_t n = payload.size();
    if (n <= 55) {
        o.push_back((char)(0xC0 + n));
    } else {
        int nb = 0;
        for (uint64_t t = n; t; t >>= 8) nb++;
        o.push_back((char)(0xF7 + nb));
        for (int i = nb - 1; i >= 0; i--) o.push_back((char)(n >> (8 * i)));
    }
    o += payload;
}

int branches_info_rlp(lx_index *h, std::string *out) {
    std::vector<uint32_t> len(h->B);
    HIPCHK(h, hipMemcpyAsync(len.data(), h->branch_len, h->B * 4ull, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    std::string last, cr, by, body;
    for (uint32_t b = 0; b < h->B; b++) {
        rlp_uint(last, len[b] ? h->h_branch_first[b] + len[b] - 1 : 0);   // BranchIDLastSeq
        rlp_uint(cr, h->h_branch_creator[b]);                              // BranchIDCreatorIdxs
    }
    for (const auto &l : h->by_creator) {                                  // BranchIDByCreators
        std::string x;
        for (uint32_t b : l) rlp_uint(x, b);
        rlp_list(by, x);
    }
    rlp_list(body, last);
    rlp_list(body, cr);
    rlp_list(body, by);
    out->clear();
    rlp_list(*out, body);
    return 0;
}

// ---- per-call queries: pinned, device-mapped host buffer (host and device pointer)
constexpr uint64_t kFcPinnedMax = 1u << 16;

int ensure_qp(lx_index *h, uint64_t bytes, uint8_t **host, uint8_t **dev) {
    if (bytes > h->qp_cap || !h->qp) {
        if (h->qp) {
            HIPCHK(h, hipStreamSynchronize(h->stream));
            (void)hipHostFree(h->qp);
        }
        h->qp = h->qp_dev = nullptr;
        h->qp_cap = 0;
        const uint64_t cap = std::max<uint64_t>(bytes, 1u << 16);
        HIPCHK(h, hipHostMalloc((void **)&h->qp, cap, hipHostMallocMapped));
        void *d = nullptr;
        HIPCHK(h, hipHostGetDevicePointer(&d, h->qp, 0));   // once per buffer, not per call
        h->qp_dev = static_cast<uint8_t *>(d);
        h->qp_cap = cap;
    }
    *host = h->qp;
    *dev = h->qp_dev;
    return 0;
}

// ---- small-batch (latency) path (lx_small.hip)

// Refresh the host mirror after batches the device assigned (big path): the
// immutable per-event fields of the events not mirrored yet, branch lengths whole.
int hm_sync(lx_index *h) {
    if (h->hm_ok) return 0;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint64_t n = h->n_events, lo = std::min(h->hm_n, n);
    rawvec<uint32_t> *v[] = {&h->hm_creator, &h->hm_seq, &h->hm_branch, &h->hm_bbefore};
    const uint32_t *d[] = {h->ev_creator, h->ev_seq, h->ev_branch, h->ev_bbefore};
    for (int k = 0; k < 4; k++) {
        v[k]->resize(n);
        if (n > lo) HIPCHK(h, hipMemcpy(v[k]->data() + lo, d[k] + lo, (n - lo) * 4, hipMemcpyDeviceToHost));
    }
    h->hm_blen.resize(h->B);
    HIPCHK(h, hipMemcpy(h->hm_blen.data(), h->branch_len, h->B * 4ull, hipMemcpyDeviceToHost));
    h->hm_n = n;
    h->hm_ok = true;
    return 0;
}

// pinned staging image of `words` uint32 (the slot's previous copy has finished
// reading it) and a device image at least as large.  A slot that must grow
// grows every slot to the same size at once: the slots are used in turn, and
// growing them one by one put a pinned allocation (~0.1-0.3 ms) into each of
// the next kSlots calls -- the latency leg's add1024 tail
int stage_slot(lx_index *h, uint64_t words, uint32_t **out, int *slot) {
    const int k = (int)h->st_next;
    h->st_next = (h->st_next + 1) % lx_index::kSlots;
    if (h->st_used[k]) HIPCHK(h, hipEventSynchronize(h->st_copied[k]));
    if (words > h->st_pin_cap[k] || words > h->st_dev_cap[k]) {
        const uint64_t cap = std::max<uint64_t>(words + words / 2, 16384);
        HIPCHK(h, hipStreamSynchronize(h->stream));   // every copy and kernel that read a slot
        for (int j = 0; j < lx_index::kSlots; j++) {
            if (cap > h->st_pin_cap[j]) {
                if (h->st_pin[j]) (void)hipHostFree(h->st_pin[j]);
                h->st_pin[j] = nullptr;
                h->st_pin_cap[j] = 0;
                HIPCHK(h, hipHostMalloc((void **)&h->st_pin[j], cap * 4, hipHostMallocDefault));
                h->st_pin_cap[j] = cap;
            }
            if (cap > h->st_dev_cap[j]) {
                if (h->st_dev[j]) (void)hipFree(h->st_dev[j]);
                h->st_dev[j] = nullptr;
                h->st_dev_cap[j] = 0;
                HIPCHK(h, dalloc(&h->st_dev[j], cap));
                h->st_dev_cap[j] = cap;
            }
        }
    }
    *out = h->st_pin[k];
    *slot = k;
    return 0;
}

}  // namespace

// Launch the pending run of small-path events [pend_bs, pend_bs + pend_n): the
// staged image (records, parents, the run's topological levels, new branches,
// touched branch lengths), one k_small, then the fork marks.  Every entry point
// that reads the device state or enqueues after it calls this first.
int flush_pending(lx_index *h) {
    if (!h->pend_n) return 0;
    HP_T(f0);
    const uint32_t n = h->pend_n;
    const uint64_t bs = h->pend_bs;
    const uint32_t B0 = h->pend_B0, B = h->B;
    const uint32_t L = h->pend_maxlvl + 1, nf = B - B0;
    // branches the run touched (each once)
    h->sm_touched.clear();
    if (h->touch_mark.size() < B) h->touch_mark.resize(B, 0);
    const uint32_t tm = ++h->touch_stamp;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t br = h->pend_ev[i].q0.x;
        if (h->touch_mark[br] != tm) { h->touch_mark[br] = tm; h->sm_touched.push_back(br); }
    }
    const uint32_t n_blen = (uint32_t)h->sm_touched.size();
    // in-run parents (run positions) and "old" entries -- parents older than the
    // run, and the older previous branch event of a branch's first event in it
    // -- were split as the events were added (add_batch_small)
    const uint32_t n_pl = (uint32_t)h->pend_pl.size(), n_old = (uint32_t)h->pend_old.size(), nh = h->pend_nh;
    if (small_lds_bytes(n, nh, L, n_pl) > kSmallLds)   // add_batch_small keeps runs within it
        return h->fail(LX_ERR_STATE, "pending run exceeds the k_small LDS budget");
    // regions 16-B aligned: the kernel copies meta and the in-run list to LDS as uint4
    const uint64_t w_ev = 12ull * n, w_meta = (2ull * n + 3) & ~3ull, w_pl = ((n_pl + 7ull) & ~7ull) / 2;
    const uint64_t words = w_ev + w_meta + w_pl + 2ull * n_old + (L + 1) + 2ull * nf + 2ull * n_blen;
    uint32_t *img;
    int slot = -1, rc;
    const bool inl = words <= kSmallInline;   // small enough for the kernel arguments
    HP_T(g0);
    if (inl) img = h->sm_inl.img;
    else if ((rc = stage_slot(h, words, &img, &slot))) return rc;
    HP_ADD(12, g0);
    HP_T(g1);
    memcpy(img, h->pend_ev.data(), w_ev * 4);
    HP_ADD(13, g1);
    HP_T(g2);
    // meta in level order (counting sort; Add order inside a level), level offsets
    uint2 *meta = reinterpret_cast<uint2 *>(img + w_ev);
    uint32_t *ipl = img + w_ev + w_meta;
    uint2 *iold = reinterpret_cast<uint2 *>(ipl + w_pl);
    uint32_t *loff = reinterpret_cast<uint32_t *>(iold + n_old);
    h->sm_cnt.assign(L + 1, 0);
    for (uint32_t i = 0; i < n; i++) h->sm_cnt[h->pend_lvl[i] + 1]++;
    for (uint32_t l = 0; l < L; l++) h->sm_cnt[l + 1] += h->sm_cnt[l];
    for (uint32_t l = 0; l <= L; l++) loff[l] = h->sm_cnt[l];
    for (uint32_t i = 0; i < n; i++) meta[h->sm_cnt[h->pend_lvl[i]]++] = h->pend_meta[i];
    HP_ADD(14, g2);
    HP_T(g3);
    if (n_pl) memcpy(ipl, h->pend_pl.data(), n_pl * 2ull);
    if (n_old) memcpy(iold, h->pend_old.data(), n_old * 8ull);
    uint32_t *nfirst = loff + L + 1, *ncreator = nfirst + nf, *blen = ncreator + nf;
    for (uint32_t x = 0; x < nf; x++) {
        nfirst[x] = h->h_branch_first[B0 + x];
        ncreator[x] = h->h_branch_creator[B0 + x];
    }
    for (uint32_t x = 0; x < n_blen; x++) {
        blen[2 * x] = h->sm_touched[x];
        blen[2 * x + 1] = h->hm_blen[h->sm_touched[x]];
    }
    HP_ADD(15, g3);
    HP_ADD(4, f0);
    HP_T(f1);
    hipStream_t s = h->stream;
    if (!inl) {
        // device image `slot` is free once the kernel that read it finished
        // the copy is a kernel on this stream (a copy-engine transfer waited
        // for the previous run's kernel and then handed over to the compute
        // queue, tens of us between every two runs of a level-fed stream)
        HIPCHK(h, lx::launch_stage(h->st_dev[slot], img, words, s));
        HIPCHK(h, hipEventRecord(h->st_copied[slot], s));
    }
    SmallArgs &a = h->sm_inl.a;
    a = SmallArgs{};
    a.hb = h->hb;
    a.la = h->la;
    a.stride = h->pstride;
    a.bs = (uint32_t)bs;
    a.n = n;
    a.B0 = B0;
    a.B = B;
    a.img = inl ? nullptr : h->st_dev[slot];
    a.o_meta = (uint32_t)w_ev;
    a.o_pl = (uint32_t)(w_ev + w_meta);
    a.o_old = (uint32_t)(w_ev + w_meta + w_pl);
    a.o_loff = (uint32_t)(loff - img);
    a.n_pl = n_pl;
    a.n_old = n_old;
    a.n_h0 = nh;
    a.n_levels = L;
    a.o_nfirst = (uint32_t)(nfirst - img);
    a.o_ncreator = (uint32_t)(ncreator - img);
    a.o_blen = (uint32_t)(blen - img);
    a.n_blen = n_blen;
    a.ev_creator = h->ev_creator;
    a.ev_seq = h->ev_seq;
    a.ev_branch = h->ev_branch;
    a.ev_bbefore = h->ev_bbefore;
    a.ev_sp = h->ev_sp;
    a.first_child = h->first_child;
    a.first_root = h->first_root;
    a.branch_first = h->branch_first;
    a.branch_creator = h->branch_creator;
    a.branch_len = h->branch_len;
    a.brow = h->brow;
    a.s_cap = h->s_cap;
    a.mask = B > h->V ? 1u : 0u;
    if (h->small_timing) HIPCHK(h, hipEventRecord(h->ev[1], s));
    // a deep run of few fork-free branches (per-event Adds of configs[0]: every
    // event its own level) by frontier doubling instead of level by level
    const bool dbl = h->dbl && !inl && !a.mask && B <= kDblMaxB && L >= kSmallDblLevels &&
                     small_dbl_lds_bytes(n, B, nh) <= kDblLds;
    HIPCHK(h, inl ? lx::launch_small_inline(h->sm_inl, s) : dbl ? lx::launch_small_dbl(a, s) : lx::launch_small(a, s));
    if (!inl) h->st_used[slot] = true;
    if (h->small_timing) HIPCHK(h, hipEventRecord(h->ev[2], s));
    if (B > h->V && h->n_cheat) {
        MarkArgs m{};
        m.hb = h->hb;
        m.stride = h->pstride;
        m.batch_start = (uint32_t)bs;
        m.n = n;
        m.V = h->V;
        m.ev_branch = h->ev_branch;
        m.ev_bbefore = h->ev_bbefore;
        m.branch_first = h->branch_first;
        m.n_cheat = h->n_cheat;
        m.cheat_off = h->cheat_off;
        m.cheat_br = h->cheat_br;
        HIPCHK(h, lx::launch_marks(m, s));
    }
    h->pend_n = 0;
    h->stats = lx_stats{};
    h->stats.index_launches = 1;
    h->stats_lazy = h->small_timing;
    HP_ADD(5, f1);
    HP_CNT(9, 1);
    return 0;
}

// The pending run is one fork-free event a: add it and fill the FC cache row
// of a against the n_slots events of evk in one k_add1_row launch (the
// unchanged caller's Add-then-ForklessCause miss; lx_fccache.cpp).  Returns 1
// (nothing enqueued) when the run is not of that shape; the caller then
// flushes and fills separately.
int flush_add1_row(lx_index *h, uint32_t a, uint32_t *evk_dev, uint32_t n_slots, uint8_t *tag_dev, uint8_t *out_dev,
                   uint32_t *psum_dev, const Add1Delta *delta) {
    if (h->pend_n != 1 || h->pend_bs != a || h->B != h->V || h->pend_B0 != h->B || h->n_cheat || h->small_timing ||
        h->sharded() || h->rowseg() || !n_slots)
        return 1;
    const SmallEv &e = h->pend_ev[0];
    // parents: all older than the run (one event), in its "old" entries
    Add1RowArgs r{};
    uint32_t np = 0;
    for (const uint2 &o : h->pend_old)
        if (!(o.x & 0x80000000u)) {
            if (np == kAdd1MaxPar) return 1;
            r.par[np++] = o.y;
        }
    if (np != e.q0.w) return 1;
    r.hb = h->hb;
    r.la = h->la;
    r.stride = h->pstride;
    r.a = a;
    r.e = e;
    r.blen = h->hm_blen[e.q0.x];
    r.B = h->B;
    r.w_br = h->weights[e.q0.x];
    r.ev_creator = h->ev_creator;
    r.ev_seq = h->ev_seq;
    r.ev_branch = h->ev_branch;
    r.ev_bbefore = h->ev_bbefore;
    r.ev_sp = h->ev_sp;
    r.first_child = h->first_child;
    r.first_root = h->first_root;
    r.branch_len = h->branch_len;
    r.brow = h->brow;
    r.branch_first = h->branch_first;
    r.s_cap = h->s_cap;
    r.evk = evk_dev;
    r.n_slots = n_slots;
    r.tag = tag_dev;
    r.out = out_dev;
    r.wpad = h->wpad;
    r.quorum = h->quorum;
    r.psum = psum_dev;
    if (delta) {
        r.nd = delta->n;
        for (uint32_t i = 0; i < delta->n; i++) {
            r.d_slot[i] = delta->slot[i];
            r.d_ev[i] = delta->ev[i];
            r.d_tag[i] = delta->tag[i];
        }
    }
    HIPCHK(h, lx::launch_add1_row(r, h->stream));
    h->pend_n = 0;
    h->stats = lx_stats{};
    h->stats.index_launches = 1;
    h->stats_lazy = false;
    return 0;
}

namespace {

// flush_pending for a launch on stream s: a foreign stream is not ordered after
// the handle's, so it waits for the run to finish
int flush_before(lx_index *h, hipStream_t s) {
    if (!h->pend_n) return 0;
    int rc = flush_pending(h);
    if (rc) return rc;
    if (s != h->stream) HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

// A run of n events with npar parents fits one k_small workgroup's LDS (the h0
// slots are at most one per branch existing before the run, and levels <= n).
inline bool small_fits(const lx_index *h, uint64_t n, uint64_t npar) {
    return n <= kSmallMaxN && npar <= 0xFFFF &&
           small_lds_bytes(n, std::min<uint64_t>(n, h->B), n, npar + 3 * n) <= kSmallLds;
}

// Add for a batch of at most small_max events, host pointers, unsharded handle.
// Validation and branch assignment run on the host in Add order -- the
// reference's own sequential fillGlobalBranchID (vecengine/index.go:105-141:
// a root continues the creator's branch iff its lastSeq is 0, a self-parented
// event continues its self-parent's branch iff lastSeq + 1 == seq, otherwise a
// new branch) over the mirrored metadata -- with the checks and error codes of
// k_validate_claim.  The batch joins the pending run of small-path events
// (pend_*); the run is launched as one k_small (level by level inside the
// kernel) when it reaches kPendLaunch events, or before anything reads or
// orders after the device state (flush_pending).  Nothing waits: errors are
// known before anything is enqueued, and a DropNotFlushed of events that are
// still pending costs no device work at all.
int add_batch_small(lx_index *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff,
                    const uint32_t *par, uint32_t *out_branch, uint32_t *err_index) {
    int rc;
    if (!h->hm_ok) {
        HIPCHK(h, set_dev(h->device));
        if ((rc = hm_sync(h))) return rc;
    }
    HP_T(a0);
    const uint64_t bs = h->n_events;
    // events [0, m) have monotone parent offsets (the error at m, if any, is
    // reported after those before it, in Add order)
    uint32_t m = 0;
    while (m < n && poff[m + 1] >= poff[m]) m++;
    const uint64_t npar_b = poff[m] - poff[0];
    HP_ADD(0, a0);
    // the run launches before it would outgrow one k_small (LDS, small_fits)
    if (h->pend_n && !small_fits(h, h->pend_n + n, h->pend_npar + npar_b) &&
        ((rc = h->hip(set_dev(h->device), "set device")) || (rc = flush_pending(h))))
        return rc;
    HP_T(a1);
    if (!h->pend_n) {
        h->pend_bs = bs;
        h->pend_B0 = h->B;
        h->pend_maxlvl = 0;
        h->pend_ev.clear();
        h->pend_lvl.clear();
        h->pend_meta.clear();
        h->pend_pl.clear();
        h->pend_old.clear();
        h->pend_npar = 0;
        h->pend_nh = 0;
    }
    const uint64_t pbs = h->pend_bs;
    const uint32_t B0 = h->B, pn0 = h->pend_n, nh0 = h->pend_nh, maxlvl0 = h->pend_maxlvl;
    const size_t pl0 = h->pend_pl.size(), old0 = h->pend_old.size();
    uint32_t B = B0, bmax = 0;
    if (h->hm_creator.capacity() < bs + n) {
        // the mirror grows with the epoch: reserve for the device capacity at once
        const uint64_t c = std::max<uint64_t>(2 * (bs + n), h->n_cap);
        for (auto *v : {&h->hm_creator, &h->hm_seq, &h->hm_branch, &h->hm_bbefore}) v->reserve(c);
    }
    h->hm_creator.resize(bs + n);
    h->hm_seq.resize(bs + n);
    h->hm_branch.resize(bs + n);
    h->hm_bbefore.resize(bs + n);
    h->pend_ev.resize(pn0 + n);
    h->pend_lvl.resize(pn0 + n);
    h->pend_meta.resize(pn0 + n);
    h->sm_undo.resize(n);
    // the split lists sized for the worst case once, written through raw
    // pointers, trimmed after the loop (the per-parent push_backs of round 3's
    // first version cost a capacity check each)
    h->pend_pl.resize(pl0 + npar_b + 3ull * n);
    h->pend_old.resize(old0 + npar_b + n);
    uint16_t *const plb = h->pend_pl.data();
    uint2 *const ob = h->pend_old.data();
    uint32_t *const lvlb = h->pend_lvl.data();
    uint2 *const metab = h->pend_meta.data();
    SmallEv *const evb = h->pend_ev.data();
    uint32_t *const mc = h->hm_creator.data(), *const ms = h->hm_seq.data(), *const mb = h->hm_branch.data(),
                   *const mbb = h->hm_bbefore.data();
    uint2 *const undo = h->sm_undo.data();   // {branch, length before} per event, for a rollback
    uint32_t *blen = h->hm_blen.data(), *bfirst = h->h_branch_first.data();
    const uint32_t V = h->V;
    size_t npl = pl0, nold = old0;
    uint32_t maxlvl = maxlvl0, nh = nh0;
    int code = 0;
    bool nonmono = false;
    uint32_t bad = 0;
    HP_ADD(1, a1);
    HP_T(a2);
    // validation (the checks and error codes of k_validate_claim), branch
    // assignment and the parent split in one pass; an error rolls the batch
    // back below (nothing of it was enqueued)
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t g = bs + i;
        const uint32_t c = creator[i], s = seq[i];
        if (i == m) { nonmono = true; bad = i; break; }
        const uint64_t p0 = poff[i], p1 = poff[i + 1];
        if (c >= V) { code = LX_ERR_ARG; bad = i; break; }
        if (s == 0 || s >= 0x7FFFFFFEu) { code = LX_ERR_EVENT; bad = i; break; }
        // level inside the run; parents split into in-run positions (chunks of
        // 4, padded with the event's own position) and older events (k_small)
        const uint32_t pi = pn0 + i;
        const uint32_t e_pl = (uint32_t)npl, e_old = (uint32_t)nold;
        uint32_t lvl = 0;
        for (uint64_t x = p0; x < p1; x++) {
            const uint32_t gp = par[x];
            if (gp >= g) { code = LX_ERR_ORDER; break; }
            if (gp >= pbs) {
                lvl = std::max(lvl, lvlb[gp - pbs] + 1);
                plb[npl++] = (uint16_t)(gp - pbs);
            } else {
                ob[nold++] = make_uint2(pi, gp);
            }
        }
        if (code) { bad = i; break; }
        const uint32_t sp = s > 1 ? (p1 > p0 ? par[p0] : LX_NONE) : LX_NONE;
        uint32_t br = 0;
        bool cont = false;
        if (s > 1) {
            // eventcheck: a self-parent of the same creator with seq - 1 (in the
            // mirror already, this batch's earlier events included)
            if (sp == LX_NONE || mc[sp] != c || ms[sp] + 1 != s) { code = LX_ERR_EVENT; bad = i; break; }
            const uint32_t bsp = mb[sp];
            const uint32_t len = blen[bsp];
            const uint32_t last = len ? bfirst[bsp] + len - 1 : 0;
            if (last + 1 == s) { br = bsp; cont = true; }
        } else if (blen[c] == 0) {
            br = c;
            cont = true;
        }
        const uint32_t bb = B;
        if (!cont) {
            br = B++;
            h->h_branch_first.push_back(s);
            h->h_branch_creator.push_back(c);
            h->by_creator[c].push_back(br);
            h->hm_blen.push_back(0);
            blen = h->hm_blen.data();
            bfirst = h->h_branch_first.data();
        }
        undo[i] = make_uint2(br, blen[br]);
        blen[br] = s - bfirst[br] + 1;
        mc[g] = c;
        ms[g] = s;
        mb[g] = br;
        mbb[g] = bb;
        while (npl & 3) plb[npl++] = (uint16_t)pi;
        metab[pi] = make_uint2(pi | ((uint32_t)npl - e_pl) / 4 << 16, e_pl / 4);
        const uint32_t prev = (cont && s > 1) ? sp : LX_NONE;
        uint32_t hslot = LX_NONE;
        if (prev != LX_NONE && prev < pbs) {
            hslot = nh++;
            ob[nold++] = make_uint2(0x80000000u | hslot, prev);
        }
        lvlb[pi] = lvl;
        maxlvl = std::max(maxlvl, lvl);
        bmax = std::max(bmax, s);
        SmallEv &e = evb[pi];
        e.q0 = make_uint4(br, s, prev, (uint32_t)(p1 - p0));
        e.q1 = make_uint4(e_old, bfirst[br], sp, bb);
        e.q2 = make_uint4(c, cont ? kSmallCont : 0u, LX_NONE, hslot);
        if (cont && sp != LX_NONE && sp >= pbs) evb[sp - pbs].q2.z = (uint32_t)g;
        if (out_branch) out_branch[i] = br;
    }
    HP_ADD(2, a2);
    HP_T(a3);
    // the batch rolled back: the host mirror as before it, the run without it
    auto rollback = [&](uint32_t done) {
        for (uint32_t i = done; i-- > 0;)
            if (undo[i].x < B0) h->hm_blen[undo[i].x] = undo[i].y;
        h->hm_blen.resize(B0);
        h->h_branch_first.resize(B0);
        h->h_branch_creator.resize(B0);
        for (auto &l : h->by_creator)
            while (!l.empty() && l.back() >= B0) l.pop_back();
        for (auto *v : {&h->hm_creator, &h->hm_seq, &h->hm_branch, &h->hm_bbefore}) v->resize(bs);
        h->pend_ev.resize(pn0);
        h->pend_lvl.resize(pn0);
        h->pend_meta.resize(pn0);
        h->pend_pl.resize(pl0);
        h->pend_old.resize(old0);
        h->pend_nh = nh0;
        h->pend_maxlvl = maxlvl0;
        for (uint32_t i = 0; i < pn0; i++)
            if (h->pend_ev[i].q2.z != LX_NONE && h->pend_ev[i].q2.z >= bs) h->pend_ev[i].q2.z = LX_NONE;
    };
    if (code || nonmono) {
        rollback(bad);
        if (err_index) *err_index = bad;
        if (nonmono) return h->fail(LX_ERR_ARG, "parent offsets not monotone");
        if (code == LX_ERR_ORDER) return h->fail(code, "event %u: processed out of order, parent not found", bad);
        if (code == LX_ERR_ARG) return h->fail(code, "event %u: creator idx out of range", bad);
        return h->fail(code, "event %u: violates seq/self-parent invariants (eventcheck)", bad);
    }
    h->pend_pl.resize(npl);
    h->pend_old.resize(nold);
    h->pend_nh = nh;
    h->pend_maxlvl = maxlvl;
    // capacity (rare re-layouts sync the stream; the pending run is not on the
    // device yet); on failure the host mirror and the run are rolled back
    h->max_seq = std::max(h->max_seq, bmax);
    const bool grows = bs + n > h->n_cap || B > h->stride || h->max_seq > h->s_cap;
    if (grows || B != B0 || h->ncols == 0 || h->pend_n + n >= kPendLaunch)
        if ((rc = h->hip(set_dev(h->device), "set device"))) return rc;
    if ((rc = grow_events(h, bs + n)) || (rc = grow_branches(h, B)) || (rc = grow_scap(h, h->max_seq))) {
        rollback(n);
        return rc;
    }
    h->wb_ready = false;
    h->B = B;
    h->pcols_used = std::max(h->pcols_used, B);
    if (B != B0 || h->ncols == 0)
        if ((rc = rebuild_columns(h))) return rc;
    h->n_events += n;
    h->hwm = std::max(h->hwm, h->n_events);
    h->hm_n = h->n_events;
    h->last_npar = poff[n] - poff[0];
    h->pend_npar += poff[n] - poff[0];
    h->pend_n = pn0 + n;
    HP_ADD(3, a3);
    if (h->pend_n >= kPendLaunch) return flush_pending(h);
    return 0;
}

}  // namespace

// =============================================================================== C ABI
extern "C" {

int lx_create(const lx_config *cfg, lx_index **out) {
    if (!out) return LX_ERR_ARG;
    lx_index *h = new lx_index();
    if (cfg) {
        h->device = cfg->device;
        h->cap_hint = cfg->event_capacity;
        h->reserve = cfg->branch_reserve;
        h->shard_rank = cfg->shard_rank;
        h->shard_count = cfg->shard_count ? cfg->shard_count : 1;
    }
    if (h->shard_rank >= h->shard_count) { delete h; return LX_ERR_ARG; }
    if (hipSetDevice(h->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&h->status, kStatusWords * 4) != hipSuccess ||
        hipMemset(h->status, 0, kStatusWords * 4) != hipSuccess) {
        delete h;
        return LX_ERR_HIP;
    }
#ifdef LX_WALKER_PROF
    if (const char *d = getenv("LX_PROF")) h->prof = (d[0] == '1');   // counters build only (make WPROF=1)
#endif
    for (auto &e : h->ev)
        if (hipEventCreate(&e) != hipSuccess) {
            delete h;
            return LX_ERR_HIP;
        }
    for (auto &e : h->st_copied)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            delete h;
            return LX_ERR_HIP;
        }
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) == hipSuccess && cus > 0)
            h->n_cus = (uint32_t)cus;
    }
    g_live_handles.fetch_add(1, std::memory_order_relaxed);
    *out = h;
    return 0;
}

void lx_destroy(lx_index *h) {
    if (!h) return;
    g_live_handles.fetch_sub(1, std::memory_order_relaxed);
    (void)hipSetDevice(h->device);
    srv_stop(h);
    if (h->srv_stream) (void)hipStreamDestroy(h->srv_stream);
    if (h->srv_host) (void)hipHostFree(h->srv_host);
    (void)hipStreamSynchronize(h->stream);
    fcc_destroy(h);
    free_all(h);
    if (h->status) (void)hipFree(h->status);
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : h->st_copied)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : h->seg_ev) (void)hipEventDestroy(e);
    for (auto *p : h->st_pin)
        if (p) (void)hipHostFree(p);
    for (auto *p : h->st_dev)
        if (p) (void)hipFree(p);
    if (h->qp) (void)hipHostFree(h->qp);
    if (h->ld_buf) (void)hipFree(h->ld_buf);
    if (h->d_fc_full) (void)hipFree(h->d_fc_full);
    if (h->d_clk) (void)hipFree(h->d_clk);
    for (void *q : {(void *)h->fcs_flag, (void *)h->fcs_pos, h->fcs_tmp})
        if (q) (void)hipFree(q);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char *lx_last_error(const lx_index *h) { return h ? h->err.c_str() : "null handle"; }

int lx_last_walk_clock(lx_index *h, float out[20]) {
    if (!h || !out) return LX_ERR_ARG;
    for (int i = 0; i < 20; i++) out[i] = 0.0f;
    if (!h->d_clk) return 0;
    HIPCHK(h, set_dev(h->device));
    std::vector<unsigned long long> v(1 + 3ull * kClkBlocks);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(v.data(), h->d_clk, v.size() * 8, hipMemcpyDeviceToHost));
    std::vector<float> mhz, ms, xm[8], xt[8];
    const uint64_t g = std::min<uint64_t>(v[0], kClkBlocks);
    for (uint64_t b = 0; b < g; b++) {
        const unsigned long long cyc = v[1 + 3 * b], tick = v[2 + 3 * b], xcc = v[3 + 3 * b];
        if (!tick || !cyc) continue;   // a workgroup without a walk (rounding, or none of the columns)
        const float f = (float)((double)cyc / (double)tick * 100.0), t = (float)((double)tick / 1e5);
        mhz.push_back(f);
        ms.push_back(t);
        if (xcc < 8) {
            xm[xcc].push_back(f);
            xt[xcc].push_back(t);
        }
    }
    if (mhz.empty()) return 0;
    auto med = [](std::vector<float> &x) {
        std::sort(x.begin(), x.end());
        return x.empty() ? 0.0f : x[x.size() / 2];
    };
    out[0] = med(mhz);
    out[1] = mhz.front();
    out[2] = mhz.back();
    out[3] = med(ms);
    for (int x = 0; x < 8; x++) {
        out[4 + x] = med(xm[x]);
        std::sort(xt[x].begin(), xt[x].end());
        out[12 + x] = xt[x].empty() ? 0.0f : xt[x].back();
    }
    return 0;
}

int lx_fc_early_rounds(lx_index *h, uint64_t out[4]) {
    if (!h || !out) return LX_ERR_ARG;
    HIPCHK(h, set_dev(h->device));
    uint64_t c[4] = {0, 0, 0, 0};
    if (h->d_fc_full) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        HIPCHK(h, hipMemcpy(c, h->d_fc_full, 32, hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemsetAsync(h->d_fc_full, 0, 32, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    out[0] = c[2];   // queries the kernel decided on the early path (device count)
    out[1] = c[0];   // of them read columns 128-255
    out[2] = c[1];   // ... 256-511
    out[3] = c[3];   // ... the rest of both rows
    return 0;
}

int lx_fc_early_counters(lx_index *h, uint64_t *queries, uint64_t *second_round, uint64_t *whole_rows) {
    if (!queries || !second_round || !whole_rows) return LX_ERR_ARG;
    uint64_t r[4];
    const int rc = lx_fc_early_rounds(h, r);
    if (rc) return rc;
    *queries = r[0];
    *second_round = r[1];
    *whole_rows = r[3];
    return 0;
}

int lx_set_option(lx_index *h, const char *name, int64_t value) {
    if (!h || !name) return LX_ERR_ARG;
    const std::string k(name);
    if (k == "small_max") {
        if (value < 0) return h->fail(LX_ERR_ARG, "small_max < 0");
        h->small_max = (uint32_t)std::min<int64_t>(value, kSmallMaxN);
    } else if (k == "fc_fk") {
        h->fc_fk = value != 0;
    } else if (k == "fc_early") {
        h->fc_early = value != 0;
    } else if (k == "fc_early_lanes") {
        if (value != 16 && value != 32) return h->fail(LX_ERR_ARG, "fc_early_lanes must be 16 or 32");
        h->fc_early_lanes = (uint32_t)value;
    } else if (k == "cpw") {
        if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 12)
            return h->fail(LX_ERR_ARG, "cpw must be 0, 1, 2, 4, 8 or 12 (8, 12: fork-free epochs with seqs <= 0xFFFF)");
        h->cpw_hint = (uint32_t)value;
    } else if (k == "pack16") {
        h->pack16 = value != 0;
    } else if (k == "crec") {
        h->crec_opt = value != 0;
    } else if (k == "seg_xmap") {
        h->seg_xmap_opt = value != 0;
    } else if (k == "realloc_records") {
        // diagnostics (walk slow-mode probe): move the batch's record buffers
        // to a fresh allocation now (the new one taken before the old is freed)
        if (value) {
            HIPCHK(h, set_dev(h->device));
            HIPCHK(h, hipStreamSynchronize(h->stream));
            const uint64_t n = (h->batch_cap + 63) / 64 * 64;
            auto move = [&](auto **b) -> int {
                if (!*b) return 0;
                std::remove_reference_t<decltype(*b)> nb = nullptr;
                HIPCHK(h, dalloc(&nb, n));
                (void)hipFree(*b);
                *b = nb;
                return 0;
            };
            if (int rc = move(&h->b_rec)) return rc;
            if (int rc = move(&h->b_crec)) return rc;
        }
    } else if (k == "dbl") {
        h->dbl = value != 0;
    } else if (k == "seg_auto") {
        h->seg_auto = value != 0;
    } else if (k == "la_memset") {
        if (h->have_epoch) return h->fail(LX_ERR_STATE, "la_memset must be set before lx_reset");
        h->la_tail = value == 0;
    } else if (k == "shard_wire") {
        if (value != 0 && value != 2 && value != 4) return h->fail(LX_ERR_ARG, "shard_wire must be 0, 2 or 4");
        h->wire_force = (uint32_t)value;
    } else if (k == "timing") {
        h->small_timing = value != 0;
    } else if (k == "seg_count" || k == "seg_rank") {
        if (h->have_epoch) return h->fail(LX_ERR_STATE, "%s must be set before lx_reset", name);
        if (h->sharded()) return h->fail(LX_ERR_STATE, "row segments on a column shard");
        if (value < 0 || value > (int64_t)kMaxSegments) return h->fail(LX_ERR_ARG, "%s must be 0..%u", name, kMaxSegments);
        (k == "seg_count" ? h->rs_count : h->rs_rank) = (uint32_t)value;
    } else if (k == "segments") {
        if (value < 0 || value > (int64_t)kMaxSegments) return h->fail(LX_ERR_ARG, "segments must be 0..%u", kMaxSegments);
        if (value > 1 && h->sharded()) return h->fail(LX_ERR_STATE, "segments on a column shard");
        h->segments = (uint32_t)value;
    } else if (k == "seg_sub") {
        // row-segment ranks: sub-segments each rank walks side by side (0: auto);
        // every rank of a job must use the same value
        if (value < 0 || value > (int64_t)kSegLaunchMax) return h->fail(LX_ERR_ARG, "seg_sub must be 0..%u", kSegLaunchMax);
        h->rs_sub_opt = (uint32_t)value;
    } else if (k == "get_server") {
        // single-row getters through the resident row server (default 1)
        if (value < 0 || value > 2) return h->fail(LX_ERR_ARG, "get_server must be 0, 1 (auto) or 2");
        h->srv_opt = (int)value;
        if (!h->srv_opt) srv_stop(h);
    } else if (k == "getter_host_check") {
        // 0 (tests only): getters skip the host's event check, so an unknown
        // event reaches the row kernel's / row server's own bound
        h->get_host_check = value != 0;
    } else if (k == "fc_cache") {
        if (value < 0 || value > 16384) return h->fail(LX_ERR_ARG, "fc_cache must be 0..16384");
        fcc_destroy(h);
        h->fcc_slots = value ? round_up((uint32_t)value, 64) : 0;
        h->fcc_slots_set = true;
    } else {
        return h->fail(LX_ERR_ARG, "unknown option %s", name);
    }
    return 0;
}

int lx_reset(lx_index *h, uint32_t nv, const uint32_t *w) {
    if (!h || (nv && !w)) return LX_ERR_ARG;
    if (nv == 0) return h->fail(LX_ERR_ARG, "empty validator set");
    uint64_t tot = 0;
    for (uint32_t i = 0; i < nv; i++) {
        if (w[i] == 0) return h->fail(LX_ERR_ARG, "zero weight at idx %u (builder drops such validators)", i);
        tot += w[i];
    }
    if (tot > 0x7FFFFFFFull) return h->fail(LX_ERR_ARG, "validators weight overflow");   // validators.go:101-110
    HIPCHK(h, set_dev(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->pend_n = 0;     // a pending run of the old epoch is simply forgotten
    h->wb_ready = false;
    h->V = nv;
    h->weights.assign(w, w + nv);
    h->quorum = (uint32_t)(tot * 2 / 3 + 1);
    shard_bounds(h, h->shard_rank, &h->own_lo, &h->own_hi);
    h->sc_events = ~0ull;
    h->sx_full = true;      // a new epoch: the next LowestAfter exchange is whole
    h->sx_active = false;
    uint32_t reserve = h->reserve ? h->reserve : std::max<uint32_t>(64, nv / 16);
    uint32_t want_stride = round_up(nv + reserve, 64);
    // a shard stores its own columns: originals + a share of the fork reserve
    const uint32_t norig = h->own_hi - h->own_lo;
    const uint32_t want_p = h->sharded() ? round_up(norig + std::max<uint32_t>(16, reserve / h->shard_count), 16)
                                         : want_stride;
    // (re)allocate when the layout changes; otherwise zero what the last epoch used
    if (want_stride > h->stride || (h->stride && want_stride * 2 < h->stride) || want_p > h->pstride ||
        (h->pstride && want_p * 2 < h->pstride)) {
        free_all(h);
        h->stride = 0;
        int rc;
        h->s_cap = 0;
        h->pstride = h->sharded() ? want_p : 0;
        if ((rc = grow_branches(h, want_stride))) return rc;
        if (h->sharded()) HIPCHK(h, dalloc(&h->wloc, h->pstride));
        uint32_t s0 = 1024;
        if (h->cap_hint) s0 = (uint32_t)std::min<uint64_t>(h->cap_hint / nv + 64, 0x7FFFFFFF);
        if ((rc = grow_scap(h, s0))) return rc;
        h->hwm = 0;
        if ((rc = grow_events(h, h->cap_hint ? h->cap_hint : 4096))) return rc;
    } else if (h->hwm && h->rowseg()) {
        // a row-segment rank: its own rows are rewritten (HB by the walk and the
        // fix-up, LA zeroed at the batch, rs_begin); only the metadata resets
        HIPCHK(h, lx::launch_fill_u32(h->first_child, h->hwm, LX_NONE, h->stream));
        h->hwm = 0;
    } else if (h->hwm) {
        // HB: the walker rewrites the original columns of every new event's row
        // (the original branches always exist); only the fork-branch columns can
        // keep stale values for rows written before such a branch existed
        // (only columns some row may have written: a previous epoch's originals
        // or fork branches beyond this epoch's originals)
        const uint32_t no = h->sharded() ? norig : nv;
        const uint32_t used = std::min(h->pcols_used, h->pstride);
        if (used > no)
            HIPCHK(h, hipMemset2DAsync(h->hb + no, (size_t)h->pstride * 4, 0, (size_t)(used - no) * 4, h->hwm, h->stream));
        // a shard's query plane is rewritten whole by the exchange (full blocks,
        // zeros included) before any ForklessCause: only its fill target needs zeroing
        if (h->lap) {
            HIPCHK(h, hipMemsetAsync(h->lap, 0, (uint64_t)h->pstride * h->s_cap * h->stride * 4, h->stream));
        } else if (h->la_tail) {
            // every entry (x, j < B) of a row is rewritten after its batch (fill or
            // tail, la_tail): only fork-branch columns of old rows need zeroing
            if (used > no)
                HIPCHK(h, hipMemset2DAsync(h->la + no, (size_t)h->pstride * 4, 0, (size_t)(used - no) * 4, h->hwm, h->stream));
            if (h->tail_zw && h->tail_dirty)
                HIPCHK(h, hipMemsetAsync(h->tail_zw, 0, (uint64_t)h->tail_cap * h->tail_cap * 4, h->stream));
            h->tail_dirty = false;
        } else {
            HIPCHK(h, hipMemsetAsync(h->la, 0, h->hwm * h->pstride * 4, h->stream));
        }
        HIPCHK(h, lx::launch_fill_u32(h->first_child, h->hwm, LX_NONE, h->stream));
        h->hwm = 0;
    }
    if (h->sharded()) {
        h->h_cmap.assign(nv, LX_NONE);
        for (uint32_t c = h->own_lo; c < h->own_hi; c++) h->h_cmap[c] = c - h->own_lo;
        h->nloc = norig;
        std::vector<uint32_t> wl(h->pstride, 0);
        for (uint32_t c = h->own_lo; c < h->own_hi; c++) wl[c - h->own_lo] = w[c];
        HIPCHK(h, hipMemcpyAsync(h->wloc, wl.data(), (uint64_t)h->pstride * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, lx::launch_fill_u32(h->cmap, h->cmap_cap, LX_NONE, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->cmap, h->h_cmap.data(), nv * 4ull, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (h->first_root) (void)hipFree(h->first_root);
    HIPCHK(h, dalloc(&h->first_root, nv));
    HIPCHK(h, lx::launch_fill_u32(h->first_root, nv, LX_NONE, h->stream));
    std::vector<uint32_t> ones(nv, 1), idx(nv), wp(h->stride, 0);
    for (uint32_t i = 0; i < nv; i++) idx[i] = i;
    for (uint32_t i = h->own_lo; i < h->own_hi; i++) wp[i] = w[i];
    HIPCHK(h, hipMemsetAsync(h->branch_len, 0, (uint64_t)h->stride * 4, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->branch_first, ones.data(), nv * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->branch_creator, idx.data(), nv * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->wpad, wp.data(), (uint64_t)h->stride * 4, hipMemcpyHostToDevice, h->stream));
    h->n_events = h->n_flushed = 0;
    h->rs_state = 0;
    h->pcols_used = h->sharded() ? norig : nv;
    h->B = h->B_flushed = nv;
    h->max_seq = 0;
    h->h_branch_creator = idx;
    h->h_branch_first = ones;
    h->by_creator.assign(nv, {});
    for (uint32_t i = 0; i < nv; i++) h->by_creator[i].push_back(i);
    h->hm_ok = true;
    h->hm_n = 0;
    for (auto *v : {&h->hm_creator, &h->hm_seq, &h->hm_branch, &h->hm_bbefore}) v->clear();
    h->hm_blen.assign(nv, 0);
    h->stats_lazy = false;
    h->loading = false;
    h->have_epoch = true;
    if (!h->fcc_slots_set) {
        // two frames of roots (C5, V = 1000: 2048 slots miss as often as 4032 and
        // fill rows half as long; profiles/r03/dropin)
        const uint32_t w = std::min<uint32_t>(8192, std::max<uint32_t>(512, round_up(2 * nv, 64)));
        if (w != h->fcc_slots) fcc_destroy(h);
        h->fcc_slots = w;
    }
    fcc_clear(h);
    h->ncols = 0;
    return rebuild_columns(h);
}

int lx_add_batch(lx_index *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff,
                 const uint32_t *par, uint32_t *out_branch, uint32_t *err_index) {
    if (!h) return LX_ERR_ARG;
    HP_T(e0);
    if (n == 0) return 0;
    if (!creator || !seq || !poff) return h->fail(LX_ERR_ARG, "null input");
    uint64_t base = poff[0], npar = poff[n] - poff[0];
    if (poff[n] < poff[0] || npar >= 0xFFFFFFFFull) return h->fail(LX_ERR_ARG, "bad parent offsets");
    if (h->loading) return h->fail(LX_ERR_STATE, "lx_add_batch during a load (lx_load_finish first)");
    // the small path makes no HIP call unless it launches or grows (it sets the device then)
    if (h->have_epoch && !h->sharded() && !h->rowseg() && n <= std::min(h->small_max, kSmallMaxN) &&
        small_fits(h, n, npar)) {
        const int rs = add_batch_small(h, n, creator, seq, poff, par, out_branch, err_index);
        HP_ADD(6, e0);
        HP_CNT(10, n);
        HP_CNT(11, 1);
        return rs;
    }
    HIPCHK(h, set_dev(h->device));
    int rc;
    if ((rc = flush_pending(h))) return rc;
    // the batch goes to the device as one pinned image {creator, seq, parent
    // offsets, parents} (16-B aligned parts) copied by k_stage into a device
    // image the walk reads in place: pageable hipMemcpyAsync of the four arrays
    // cost ~0.5 ms per 50k-event batch
    const uint64_t a4 = (n + 3ull) / 4 * 4, o4 = (n + 4ull) / 4 * 4;
    const uint64_t words = 2 * a4 + o4 + npar;
    uint32_t *img = nullptr;
    int slot = 0;
    if ((rc = stage_slot(h, words, &img, &slot))) return rc;
    memcpy(img, creator, n * 4ull);
    memcpy(img + a4, seq, n * 4ull);
    uint32_t *off = img + 2 * a4;
    for (uint32_t i = 0; i <= n; i++) {
        if (i && poff[i] < poff[i - 1]) return h->fail(LX_ERR_ARG, "parent offsets not monotone");
        off[i] = (uint32_t)(poff[i] - base);
    }
    if (npar) memcpy(img + 2 * a4 + o4, par + base, npar * 4);
    uint32_t *dimg = h->st_dev[slot];
    HIPCHK(h, lx::launch_stage(dimg, img, words, h->stream));
    HIPCHK(h, hipEventRecord(h->st_copied[slot], h->stream));
    h->st_used[slot] = true;
    uint64_t start = h->n_events;
    if ((rc = add_batch_dev(h, n, dimg, dimg + a4, dimg + 2 * a4, dimg + 2 * a4 + o4, err_index))) return rc;
    if (out_branch) HIPCHK(h, hipMemcpy(out_branch, h->ev_branch + start, n * 4ull, hipMemcpyDeviceToHost));
    return 0;
}

int lx_add_batch_dev(lx_index *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint32_t *poff,
                     const uint32_t *par, uint32_t *err_index) {
    if (!h) return LX_ERR_ARG;
    HIPCHK(h, set_dev(h->device));
    {
        const int rc = flush_pending(h);
        if (rc) return rc;
    }
    return add_batch_dev(h, n, creator, seq, poff, par, err_index);
}

int lx_flush(lx_index *h) {
    if (!h) return LX_ERR_ARG;
    NOT_LOADING(h);
    h->wb_ready = false;
    h->n_flushed = h->n_events;
    h->B_flushed = h->B;
    return 0;
}

int lx_drop_not_flushed(lx_index *h) {
    if (!h) return LX_ERR_ARG;
    NOT_LOADING(h);
    WHOLE_INDEX(h);
    if (!h->have_epoch) return 0;
    HIPCHK(h, set_dev(h->device));
    h->wb_ready = false;
    if (h->n_events == h->n_flushed && h->B == h->B_flushed) return 0;
    if (h->pend_n && h->n_flushed >= h->pend_bs) {
        // every dropped event is still in the pending run: it never reached the
        // device, so the rollback is host-only (Build = Add + DropNotFlushed
        // costs no launch)
        const uint32_t keep = (uint32_t)(h->n_flushed - h->pend_bs);
        h->pend_old.resize(h->pend_ev[keep].q1.x);
        h->pend_pl.resize(4ull * h->pend_meta[keep].y);
        h->pend_ev.resize(keep);
        h->pend_lvl.resize(keep);
        h->pend_meta.resize(keep);
        h->pend_maxlvl = 0;
        h->pend_nh = 0;
        h->pend_npar = 0;
        for (uint32_t i = 0; i < keep; i++) {
            SmallEv &e = h->pend_ev[i];
            if (e.q2.z != LX_NONE && e.q2.z >= h->n_flushed) e.q2.z = LX_NONE;
            if (e.q2.w != LX_NONE) h->pend_nh = e.q2.w + 1;
            h->pend_npar += e.q0.w;
            h->pend_maxlvl = std::max(h->pend_maxlvl, h->pend_lvl[i]);
        }
        h->pend_n = keep;
    } else {
        int rc;
        if ((rc = flush_pending(h))) return rc;
        HIPCHK(h, lx::launch_unfill(unfill_args(h), h->stream));
        HIPCHK(h, lx::launch_zero_rows(h->hb, h->la, h->pstride, (uint32_t)h->n_flushed, (uint32_t)h->n_events, h->stream));
        // re-added events may land on rows this epoch has not used yet (stale from an
        // earlier epoch) with seqs the tail table already counts as done: start over
        if (h->tail_zw && h->tail_dirty) {
            HIPCHK(h, hipMemsetAsync(h->tail_zw, 0, (uint64_t)h->tail_cap * h->tail_cap * 4, h->stream));
            h->tail_dirty = false;
        }
    }
    // host mirror: the same rollback of the branch lengths (k_unclaim) and rows
    if (h->hm_ok) {
        for (uint64_t e = h->n_flushed; e < h->n_events; e++) {
            const uint32_t br = h->hm_branch[e];
            if (br < h->B_flushed) h->hm_blen[br] = std::min(h->hm_blen[br], h->hm_seq[e] - h->h_branch_first[br]);
        }
        h->hm_blen.resize(h->B_flushed);
        for (auto *v : {&h->hm_creator, &h->hm_seq, &h->hm_branch, &h->hm_bbefore}) v->resize(h->n_flushed);
    }
    h->hm_n = std::min(h->hm_n, h->n_flushed);
    h->n_events = h->n_flushed;
    fcc_forget_from(h, h->n_flushed);
    h->sx_full = true;      // receivers may hold entries of the dropped events
    h->sx_active = false;
    if (h->B != h->B_flushed) {
        h->B = h->B_flushed;
        h->h_branch_creator.resize(h->B);
        h->h_branch_first.resize(h->B);
        for (auto &l : h->by_creator)
            while (!l.empty() && l.back() >= h->B) l.pop_back();
        if (h->sharded()) {
            // dropped fork columns: their plane columns were zeroed with the rows
            // that used them (rows > n_flushed); older rows never saw them
            for (uint32_t b = h->B; b < h->h_cmap.size(); b++)
                if (h->h_cmap[b] != LX_NONE) h->nloc--;
            h->h_cmap.resize(h->B);
            HIPCHK(h, lx::launch_fill_u32(h->cmap + h->B, h->cmap_cap - h->B, LX_NONE, h->stream));
        }
        return rebuild_columns(h);
    }
    return 0;
}

int lx_writeback_prepare(lx_index *h, lx_writeback *out) {
    if (!h || !out) return LX_ERR_ARG;
    WHOLE_INDEX(h);
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "write-back before lx_reset");
    NOT_LOADING(h);
    {
        const int rc = flush_pending(h);
        if (rc) return rc;
    }
    if (h->shard_count > 1) return h->fail(LX_ERR_STATE, "write-back needs an unsharded handle (shards hold partial rows)");
    HIPCHK(h, set_dev(h->device));
    h->wb_ready = false;
    const uint32_t N = (uint32_t)h->n_events, lo = (uint32_t)h->n_flushed;
    int rc;
    if ((rc = ensure_wb(h, N))) return rc;
    hipStream_t s = h->stream;
    uint32_t n_la = 0;
    if (N > lo) {
        HIPCHK(h, hipMemsetAsync(h->wb_flag, 0, N * 4ull, s));
        HIPCHK(h, lx::launch_dirty_la(unfill_args(h), h->wb_flag, s));
        HIPCHK(h, lx::launch_compact(h->wb_flag, h->wb_pos, N, h->wb_tmp, h->wb_tmp_bytes, h->wb_la_rows, s));
        HIPCHK(h, hipMemcpyAsync(&n_la, h->wb_pos + (N - 1), 4, hipMemcpyDeviceToHost, s));
        HIPCHK(h, lx::launch_iota(h->wb_hb_rows, lo, N - lo, s));
        HIPCHK(h, hipStreamSynchronize(s));
    }
    // byte offsets of both row sets (wb_len is scratch, reused in stream order)
    HIPCHK(h, lx::launch_row_offsets(rows_args(h, 0, h->wb_la_rows, n_la), h->wb_len, h->wb_la_off, h->wb_tmp,
                                     h->wb_tmp_bytes, s));
    HIPCHK(h, lx::launch_row_offsets(rows_args(h, 1, h->wb_hb_rows, N - lo), h->wb_len, h->wb_hb_off, h->wb_tmp,
                                     h->wb_tmp_bytes, s));
    uint64_t tot[2] = {0, 0};
    HIPCHK(h, hipMemcpyAsync(&tot[0], h->wb_la_off + n_la, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(&tot[1], h->wb_hb_off + (N - lo), 8, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    if ((rc = branches_info_rlp(h, &h->wb_bi))) return rc;
    lx_writeback w{};
    w.first_event = lo;
    w.n_events = N - lo;
    w.n_la_rows = n_la;
    w.hb_bytes = tot[1];
    w.la_bytes = tot[0];
    w.bi_bytes = (uint32_t)h->wb_bi.size();
    h->wb = w;
    h->wb_ready = true;
    *out = w;
    return 0;
}

int lx_writeback_fetch(lx_index *h, uint64_t *hb_off, uint8_t *hb_bytes, uint32_t *la_ev, uint64_t *la_off,
                       uint8_t *la_bytes, uint8_t *branch_be, uint8_t *bi_rlp) {
    if (!h) return LX_ERR_ARG;
    if (!h->wb_ready) return h->fail(LX_ERR_STATE, "lx_writeback_fetch without a current lx_writeback_prepare");
    HIPCHK(h, set_dev(h->device));
    const lx_writeback &w = h->wb;
    const uint32_t n = (uint32_t)w.n_events, m = (uint32_t)w.n_la_rows;
    int rc;
    if ((hb_off || hb_bytes) && (rc = rows_to_host(h, 1, h->wb_hb_rows, h->wb_hb_off, n, hb_off, hb_bytes))) return rc;
    if (la_ev && m) {
        HIPCHK(h, hipMemcpyAsync(la_ev, h->wb_la_rows, m * 4ull, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if ((la_off || la_bytes) && (rc = rows_to_host(h, 0, h->wb_la_rows, h->wb_la_off, m, la_off, la_bytes))) return rc;
    if (branch_be && n) {
        std::vector<uint32_t> br(n);
        HIPCHK(h, hipMemcpyAsync(br.data(), h->ev_branch + w.first_event, n * 4ull, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        for (uint32_t i = 0; i < n; i++)
            for (int k = 0; k < 4; k++) branch_be[4 * i + k] = (uint8_t)(br[i] >> (24 - 8 * k));
    }
    if (bi_rlp) memcpy(bi_rlp, h->wb_bi.data(), h->wb_bi.size());
    return 0;
}

uint64_t lx_num_events(const lx_index *h) { return h ? h->n_events : 0; }
uint32_t lx_num_branches(const lx_index *h) { return h ? h->B : 0; }
int lx_at_least_one_fork(const lx_index *h) { return h && h->B > h->V; }
uint32_t lx_quorum(const lx_index *h) { return h ? h->quorum : 0; }

int lx_forkless_cause_batch_dev(lx_index *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out,
                                void *stream) {
    if (!h) return LX_ERR_ARG;
    if (!n) return 0;
    FcArgs f;
    int rc = lx_fc_args(h, n, a, b, out, nullptr, &f);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if ((rc = flush_before(h, s))) return rc;
    HIPCHK(h, lx::launch_fc(f, h->ncols, h->B > h->V, s));
    return 0;
}

int lx_forkless_cause_partial_dev(lx_index *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint32_t *partial,
                                  void *stream) {
    if (!h) return LX_ERR_ARG;
    if (!n) return 0;
    FcArgs f;
    int rc = lx_fc_args(h, n, a, b, nullptr, partial, &f);
    if (rc) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if ((rc = flush_before(h, s))) return rc;
    HIPCHK(h, lx::launch_fc(f, h->ncols, h->B > h->V, s));
    return 0;
}

// ---- column-shard early exit
int lx_fc_shard_early(const lx_index *h, uint32_t *rest) {
    if (!h) return 0;
    if (rest) *rest = 0;
    // fork-free (no shard's partial carries a mark or exceeds its stake) and
    // shard 0 able to decide something alone
    if (!h->sharded() || !h->have_epoch || h->B != h->V || h->weights.size() != h->V) return 0;
    uint32_t lo, hi;
    shard_bounds(h, 0, &lo, &hi);
    uint64_t w0 = 0, wt = 0;
    for (uint32_t c = 0; c < h->V; c++) {
        wt += h->weights[c];
        if (c >= lo && c < hi) w0 += h->weights[c];
    }
    if (wt - w0 > 0xFFFFFFFFull) return 0;
    if (rest) *rest = (uint32_t)(wt - w0);
    return (w0 >= h->quorum || wt - w0 < h->quorum) ? 1 : 0;
}

int lx_fc_shard_decide_dev(lx_index *h, uint64_t n, const uint32_t *partial, uint64_t *mask, void *stream) {
    if (!h || (n && (!partial || !mask))) return LX_ERR_ARG;
    uint32_t rest = 0;
    if (!lx_fc_shard_early(h, &rest)) return h->fail(LX_ERR_STATE, "the column-shard early exit does not apply (lx_fc_shard_early)");
    if (h->shard_rank != 0) return h->fail(LX_ERR_STATE, "only shard 0 decides early (its creators are the heaviest)");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const uint64_t W = (n + 63) / 64;
    HIPCHK(h, lx::launch_fcs_decide(partial, n, h->quorum, rest, reinterpret_cast<unsigned long long *>(mask),
                                    reinterpret_cast<unsigned long long *>(mask) + W, s));
    return 0;
}

int lx_fc_shard_undecided_dev(lx_index *h, uint64_t n, const uint64_t *mask, const uint32_t *a, const uint32_t *b,
                              const uint32_t *partial, uint32_t *idx, uint32_t *a_out, uint32_t *b_out, uint32_t *p_out,
                              uint64_t *m) {
    if (!h || !m || (n && (!mask || !a || !b || !idx || !a_out || !b_out || (partial && !p_out)))) return LX_ERR_ARG;
    if (!h->sharded()) return h->fail(LX_ERR_STATE, "the column-shard early exit needs a column-sharded handle");
    if (n > 0x7FFFFFFFull) return h->fail(LX_ERR_ARG, "too many queries in one call");
    *m = 0;
    if (!n) return 0;
    HIPCHK(h, set_dev(h->device));
    if (n > h->fcs_cap) {
        (void)hipStreamSynchronize(h->stream);
        for (void *q : {(void *)h->fcs_flag, (void *)h->fcs_pos, h->fcs_tmp})
            if (q) (void)hipFree(q);
        h->fcs_flag = h->fcs_pos = nullptr;
        h->fcs_tmp = nullptr;
        h->fcs_cap = 0;
        HIPCHK(h, lxi::dalloc(&h->fcs_flag, n));
        HIPCHK(h, lxi::dalloc(&h->fcs_pos, n));
        HIPCHK(h, lx::fcs_scan_bytes(n, &h->fcs_tmp_bytes));
        HIPCHK(h, hipMalloc(&h->fcs_tmp, std::max<size_t>(h->fcs_tmp_bytes, 16)));
        h->fcs_cap = n;
    }
    HIPCHK(h, lx::launch_fcs_undecided(reinterpret_cast<const unsigned long long *>(mask), n, a, b, partial, h->fcs_flag,
                                       h->fcs_pos, h->fcs_tmp, h->fcs_tmp_bytes, idx, a_out, b_out, p_out, h->stream));
    uint32_t cnt = 0;
    HIPCHK(h, hipMemcpyAsync(&cnt, h->fcs_pos + (n - 1), 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    *m = cnt;
    return 0;
}

int lx_fc_shard_answer_dev(lx_index *h, uint64_t n, const uint64_t *mask, uint64_t m, const uint32_t *idx,
                           const uint32_t *sum, uint8_t *out, void *stream) {
    if (!h || (n && (!mask || !out)) || (m && (!idx || !sum)) || m > n) return LX_ERR_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const uint64_t W = (n + 63) / 64;
    const auto *dec = reinterpret_cast<const unsigned long long *>(mask);
    HIPCHK(h, lx::launch_fcs_answer(dec, dec + W, n, m, idx, sum, h->quorum, out, s));
    return 0;
}

int lx_fc_combine_dev(lx_index *h, uint64_t n, const uint32_t *sum, uint8_t *out, void *stream) {
    if (!h) return LX_ERR_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    HIPCHK(h, lx::launch_fc_combine(sum, out, n, h->quorum, s));
    return 0;
}

int lx_forkless_cause_batch(lx_index *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out) {
    if (!h) return LX_ERR_ARG;
    if (!n) return 0;
    HIPCHK(h, set_dev(h->device));
    {
        const int rc = flush_pending(h);
        if (rc) return rc;
    }
    if (n <= kFcPinnedMax) {
        // per-call sizes (calcFrameIdx asks ~2/3 V pairs, the election |roots|):
        // the kernel reads the pairs from and writes the answers into pinned host
        // memory -- one launch and one stream sync, no copies
        int rc;
        uint8_t *hp, *dp;
        if ((rc = ensure_qp(h, n * 9 + 16, &hp, &dp))) return rc;
        memcpy(hp, a, n * 4);
        memcpy(hp + 4 * n, b, n * 4);
        FcArgs f;
        if ((rc = lx_fc_args(h, n, reinterpret_cast<uint32_t *>(dp), reinterpret_cast<uint32_t *>(dp + 4 * n), dp + 8 * n,
                          nullptr, &f)))
            return rc;
        f.status = h->status + 2;   // k_fc flags status[1] = word 3, the sink; unknown events answer 0xFF
        // completion by the answers themselves: each byte is written once
        // (0, 1 or 0xFF) over a 0xFE the host put there, so the host spins
        // until none is left instead of synchronizing the stream (~5 us)
        volatile uint8_t *ans = hp + 8 * n;
        memset(hp + 8 * n, 0xFE, n);
        HIPCHK(h, lx::launch_fc(f, h->ncols, h->B > h->V, h->stream));
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t i = 0, k = 0; i < n; k++) {
            while (i < n && ans[i] != 0xFE) i++;
            if (i < n && (k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                HIPCHK(h, hipStreamSynchronize(h->stream));
                while (i < n && ans[i] != 0xFE) i++;
                if (i < n) return h->fail(LX_ERR_STATE, "ForklessCause: the kernel left answers unwritten");
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        memcpy(out, hp + 8 * n, n);
        for (uint64_t i = 0; i < n; i++)
            if (out[i] > 1) return h->fail(LX_ERR_ARG, "ForklessCause on an unknown event");   // forkless_cause.go:43-61
        return 0;
    }
    if (n > h->q_cap) {
        uint64_t cap = std::max<uint64_t>(n, 4096);
        if (h->q_a) (void)hipFree(h->q_a);
        if (h->q_b) (void)hipFree(h->q_b);
        if (h->q_out) (void)hipFree(h->q_out);
        HIPCHK(h, dalloc(&h->q_a, cap));
        HIPCHK(h, dalloc(&h->q_b, cap));
        HIPCHK(h, dalloc(&h->q_out, cap));
        h->q_cap = cap;
    }
    HIPCHK(h, hipMemsetAsync(h->status + 1, 0, 4, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->q_a, a, n * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->q_b, b, n * 4, hipMemcpyHostToDevice, h->stream));
    int rc = lx_forkless_cause_batch_dev(h, n, h->q_a, h->q_b, h->q_out, nullptr);
    if (rc) return rc;
    uint32_t bad = 0;
    HIPCHK(h, hipMemcpyAsync(out, h->q_out, n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipMemcpyAsync(&bad, h->status + 1, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (bad) return h->fail(LX_ERR_ARG, "ForklessCause on an unknown event");   // forkless_cause.go:43-61 (crit)
    return 0;
}

int lx_get_event_branch_id(lx_index *h, uint32_t ev, uint32_t *out) {
    if (!h || !out) return LX_ERR_ARG;
    NOT_LOADING(h);
    if (ev >= h->n_events) return h->fail(LX_ERR_ARG, "failed to read event's branch ID (unknown event %u)", ev);
    if (h->hm_ok) {
        *out = h->hm_branch[ev];
        return 0;
    }
    HIPCHK(h, set_dev(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return read_u32(h, h->ev_branch + ev, out);
}

}  // extern "C"

namespace {

// Rows of n events in the reference byte layout (mode 0 HighestBefore, 1
// LowestAfter, 2 merged HighestBefore), encoded on the device by k_get_rows
// straight into the pinned buffer: one launch and one stream sync per call
// (rows of more than kGetChunk bytes go in several).  *rows: row i at
// rows + i * slot; len[i] its byte length.
constexpr uint64_t kGetChunk = 64ull << 20;

// single-row tags: 30 bits (the server's request word), never 0 or kGetSrvStop
uint32_t next_get_tag(lx_index *h) {
    h->get_tag = h->get_tag + 1 >= kGetSrvStop ? 1u : h->get_tag + 1;
    return h->get_tag;
}

// the server's arguments for a single-row GetArgs (memcmp-comparable)
GetSrvArgs srv_args_of(const lx_index *h, const GetArgs &a) {
    GetSrvArgs s;
    memset(&s, 0, sizeof s);
    s.g = a;
    s.g.plane = nullptr;
    s.g.ev = nullptr;
    s.g.ev0 = 0;
    s.g.mode = 0;
    s.g.tag = 0;
    // a server outlives Adds: its bound is the handle's capacity (rows past
    // n_events are zero or stale there; the host check, option
    // getter_host_check, refuses such events before any request is posted),
    // so that an Add between two getters does not relaunch it
    if (!h->rowseg()) s.g.row_hi = (uint32_t)std::min<uint64_t>(h->n_cap, 0xFFFFFFFFull);
    s.hb = h->hb;
    s.la = h->la;
    s.req = h->srv_dev;
    s.exited = reinterpret_cast<uint32_t *>(h->srv_dev + 1);
    return s;
}

// (re)launch the server with the arguments of `a`; it ignores request tags up
// to seen0
int srv_launch(lx_index *h, const GetArgs &a, uint32_t seen0) {
    GetSrvArgs s = srv_args_of(h, a);
    h->srv_args = s;
    s.gen = ++h->srv_gen;
    s.seen0 = seen0;
    s.idle_ticks = 250 * h->srv_ticks_us;          // leave after 250 us without a request
    s.budget_ticks = 500000 * h->srv_ticks_us;     // and after 0.5 s in all
    HIPCHK(h, lx::launch_get_server(s, h->srv_stream));
    h->srv_live = true;
    h->srv_launches++;
    return 0;
}

}  // namespace

// stop a live server (the stop tag, then its stream): it reads nothing but
// the request word between requests
void srv_stop(lx_index *h) {
    if (!h || !h->srv_live) return;
    reinterpret_cast<volatile uint64_t *>(h->srv_host)[0] = kGetSrvStop;
    (void)hipStreamSynchronize(h->srv_stream);
    h->srv_live = false;
}

namespace {

// post one row request to the server when the handle's stream is idle (every
// row the request reads is final); *posted = false: the caller launches
int srv_post(lx_index *h, const GetArgs &a, bool *posted) {
    *posted = false;
    if (!h->srv_opt || a.n != 1 || a.ev) return 0;
    if (h->srv_opt == 1 && g_live_handles.load(std::memory_order_relaxed) > 1) {
        // another handle's streams may share the server's hardware queue
        if (h->srv_live) srv_stop(h);
        return 0;
    }
    // the rows it reads must be final: wait for the stream (usually the tail
    // of a launch whose results the host already has -- a pinned-path
    // ForklessCause, a getter that launched -- so that the next call finds it
    // idle instead of launching again)
    if (hipStreamQuery(h->stream) != hipSuccess && hipStreamSynchronize(h->stream) != hipSuccess) return 0;
    if (!h->srv_host) {
        // what the server needs; without any of it the getters launch as before
        int lo = 0, hi = 0, khz = 0;
        void *p = nullptr, *d = nullptr;
        bool ok = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) == hipSuccess && khz >= 1000 &&
                  hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess;
        if (ok && !h->srv_stream) ok = hipStreamCreateWithPriority(&h->srv_stream, hipStreamNonBlocking, hi) == hipSuccess;
        if (ok) ok = hipHostMalloc(&p, 64, hipHostMallocMapped) == hipSuccess;
        if (ok) ok = hipHostGetDevicePointer(&d, p, 0) == hipSuccess;
        if (!ok) {
            if (p) (void)hipHostFree(p);
            (void)hipGetLastError();
            h->srv_opt = 0;
            return 0;
        }
        memset(p, 0, 64);
        h->srv_ticks_us = (uint64_t)khz / 1000;
        h->srv_host = static_cast<uint64_t *>(p);
        h->srv_dev = static_cast<uint64_t *>(d);
    }
    volatile uint64_t *req = h->srv_host;
    const GetSrvArgs want = srv_args_of(h, a);
    if (h->srv_live && (uint32_t)reinterpret_cast<volatile uint64_t *>(h->srv_host)[1] == h->srv_gen) {
        (void)hipStreamSynchronize(h->srv_stream);   // it left (idle or deadline): its launch has ended
        h->srv_live = false;
    }
    if (h->srv_live && memcmp(&want, &h->srv_args, sizeof want) != 0) srv_stop(h);
    int rc;
    if (!h->srv_live && (rc = srv_launch(h, a, (uint32_t)(req[0] & kGetSrvStop)))) return rc;
    req[0] = (uint64_t)a.ev0 << 32 | (uint64_t)(a.mode & 3u) << 30 | a.tag;
    *posted = true;
    return 0;
}

int get_rows(lx_index *h, uint32_t mode, uint32_t n, const uint32_t *ev, uint8_t **rows, uint64_t *slot,
             const uint32_t **len) {
    const uint64_t sl = ((uint64_t)8 * std::max(h->B, h->V) + 15) / 16 * 16;
    const uint64_t head = ((uint64_t)8 * n + 4 + 15) / 16 * 16;   // events + lengths + completion tag
    uint8_t *hp, *dp;
    int rc;
    if ((rc = ensure_qp(h, head + n * sl, &hp, &dp))) return rc;
    if (n > 1) memcpy(hp, ev, n * 4ull);
    GetArgs a{};
    a.plane = mode == 1 ? h->la : h->hb;
    a.stride = h->stride;
    // one row: the event travels in the arguments (no read of host memory)
    a.ev = n > 1 ? reinterpret_cast<const uint32_t *>(dp) : nullptr;
    a.ev0 = ev[0];
    a.n = n;
    a.B = h->B;
    a.V = h->V;
    a.mode = mode;
    a.forks = h->B > h->V ? 1u : 0u;
    a.ev_bbefore = h->ev_bbefore;
    a.ev_branch = h->ev_branch;
    a.branch_first = h->branch_first;
    a.cheat_of = h->cheat_of;
    a.cheat_off = h->cheat_off;
    a.cheat_br = h->cheat_br;
    a.len = reinterpret_cast<uint32_t *>(dp + 4ull * n);
    a.out = dp + head;
    a.slot = sl;
    // the device's own bound: the events indexed so far on a launch (the
    // resident server's bound is the capacity instead, srv_args_of)
    a.row_lo = h->rowseg() ? h->rs_lo : 0u;
    a.row_hi = h->rowseg() ? h->rs_hi : (uint32_t)h->n_events;
    if (n == 1) {
        // one row (the reference's per-call getters): the resident server
        // answers it when the handle's stream is idle (no launch); otherwise a
        // launch on the stream.  Either publishes a tag after the row and the
        // host spins on it (a stream synchronization costs ~5 us more,
        // scripts/probes/sync_latency.hip); a launch that never lands is caught
        // by the timeout's synchronization
        a.tag = next_get_tag(h);
        a.done = reinterpret_cast<uint32_t *>(dp + 8ull * n);
        const volatile uint32_t *done = reinterpret_cast<const volatile uint32_t *>(hp + 8ull * n);
        bool posted = false;
        if ((rc = srv_post(h, a, &posted))) return rc;
        if (!posted) {
            h->srv_fallbacks++;
            HIPCHK(h, lx::launch_get_rows(a, h->stream));
        }
        const auto t0 = std::chrono::steady_clock::now();
        bool relaunched = false;
        for (uint32_t k = 0; *done != a.tag; k++) {
            if ((k & 63) != 63) continue;
            if (posted && !relaunched && (uint32_t)reinterpret_cast<volatile uint64_t *>(h->srv_host)[1] == h->srv_gen &&
                *done != a.tag) {
                // the server left (idle or its deadline) before it saw the request
                h->srv_live = false;
                if ((rc = srv_launch(h, a, a.tag == 1 ? kGetSrvStop - 1 : a.tag - 1))) return rc;
                relaunched = true;
            }
            if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                if (posted && *done != a.tag) {
                    // the server did not answer: stop it and take the launch path
                    srv_stop(h);
                    if (*done != a.tag) {
                        posted = false;
                        h->srv_fallbacks++;
                        HIPCHK(h, lx::launch_get_rows(a, h->stream));
                    }
                }
                HIPCHK(h, hipStreamSynchronize(h->stream));
                if (*done != a.tag) return h->fail(LX_ERR_STATE, "getter: the row kernel did not complete");
            }
        }
        if (posted) h->srv_served++;
        std::atomic_thread_fence(std::memory_order_acquire);
    } else {
        HIPCHK(h, lx::launch_get_rows(a, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    *rows = hp + head;
    *slot = sl;
    *len = reinterpret_cast<const uint32_t *>(hp + 4ull * n);
    for (uint32_t i = 0; i < n; i++)
        if ((*len)[i] == kGetBadLen) return h->fail(LX_ERR_ARG, "unknown event %u (refused by the row kernel)", ev[i]);
    return 0;
}

int get_check(lx_index *h, uint32_t n, const uint32_t *ev) {
    if (h->sharded())
        return h->fail(LX_ERR_STATE, "a column shard holds its own columns: lx_shard_get_rows (or lx_get_rows_dev + a sum over the shards)");
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "getter before lx_reset");
    NOT_LOADING(h);
    if (h->rowseg()) {
        // a row-segment rank answers for its own rows (final after lx_rowseg_finish);
        // the others' are routed to their owners (lachesis_hip/rowseg.py, lx_rowseg_get_rows)
        if (h->rs_state != 4) return h->fail(LX_ERR_STATE, "row-segment rank: getters before lx_rowseg_finish");
        if (h->get_host_check)
            for (uint32_t i = 0; i < n; i++)
                if (ev[i] < h->rs_lo || ev[i] >= h->rs_hi)
                    return h->fail(ev[i] < h->n_events ? LX_ERR_STATE : LX_ERR_ARG,
                                   "event %u is not a row of this row-segment rank [%u, %u)", ev[i], h->rs_lo, h->rs_hi);
    }
    {
        const int rc = flush_pending(h);
        if (rc) return rc;
    }
    if (h->get_host_check)
        for (uint32_t i = 0; i < n; i++)
            if (ev[i] >= h->n_events) return h->fail(LX_ERR_ARG, "unknown event %u", ev[i]);
    HIPCHK(h, set_dev(h->device));
    return 0;
}

int get_one(lx_index *h, uint32_t mode, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len) {
    if (!h) return LX_ERR_ARG;
    int rc;
    if ((rc = get_check(h, 1, &ev))) return rc;
    uint8_t *rows;
    uint64_t slot;
    const uint32_t *ln;
    if ((rc = get_rows(h, mode, 1, &ev, &rows, &slot, &ln))) return rc;
    if (len) *len = ln[0];
    if (out && cap) memcpy(out, rows, std::min(cap, ln[0]));   // little-endian host
    return 0;
}

int get_batch(lx_index *h, uint32_t mode, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out, uint64_t cap) {
    if (!h || (n && (!ev || !off))) return LX_ERR_ARG;
    int rc;
    if ((rc = get_check(h, n, ev))) return rc;
    off[0] = 0;
    const uint64_t sl = ((uint64_t)8 * std::max(h->B, h->V) + 15) / 16 * 16;
    const uint32_t chunk = (uint32_t)std::max<uint64_t>(1, kGetChunk / sl);
    for (uint32_t i0 = 0; i0 < n; i0 += chunk) {
        const uint32_t m = std::min(chunk, n - i0);
        uint8_t *rows;
        uint64_t slot;
        const uint32_t *ln;
        if ((rc = get_rows(h, mode, m, ev + i0, &rows, &slot, &ln))) return rc;
        for (uint32_t i = 0; i < m; i++) {
            off[i0 + i + 1] = off[i0 + i] + ln[i];
            if (out && off[i0 + i + 1] <= cap) memcpy(out + off[i0 + i], rows + i * slot, ln[i]);
        }
    }
    if (out && off[n] > cap)
        return h->fail(LX_ERR_ARG, "getter buffer too small: %llu bytes needed", (unsigned long long)off[n]);
    return 0;
}

}  // namespace

extern "C" {

int lx_live_handles(void) { return g_live_handles.load(std::memory_order_relaxed); }

int lx_get_server_stats(const lx_index *h, uint64_t out[3]) {
    if (!h || !out) return LX_ERR_ARG;
    out[0] = h->srv_served;
    out[1] = h->srv_launches;
    out[2] = h->srv_fallbacks;
    return 0;
}

int lx_get_highest_before(lx_index *h, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len) {
    return get_one(h, 0, ev, out, cap, len);
}

int lx_get_lowest_after(lx_index *h, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len) {
    return get_one(h, 1, ev, out, cap, len);
}

int lx_get_merged_highest_before(lx_index *h, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len) {
    return get_one(h, 2, ev, out, cap, len);
}

int lx_get_highest_before_batch(lx_index *h, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out,
                                uint64_t cap) {
    return get_batch(h, 0, n, ev, off, out, cap);
}

int lx_get_lowest_after_batch(lx_index *h, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out, uint64_t cap) {
    return get_batch(h, 1, n, ev, off, out, cap);
}

int lx_get_merged_highest_before_batch(lx_index *h, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out,
                                       uint64_t cap) {
    return get_batch(h, 2, n, ev, off, out, cap);
}

int lx_row_bytes_max(const lx_index *h, uint64_t *bytes) {
    if (!h || !bytes) return LX_ERR_ARG;
    *bytes = 8ull * std::max(h->B, h->V);
    return 0;
}

int lx_get_rows_dev(lx_index *h, uint32_t mode, uint32_t n, const uint32_t *ev_dev, uint8_t *out_dev,
                    uint64_t slot_bytes, uint32_t *len_dev) {
    if (!h || mode > 2 || (n && (!ev_dev || !out_dev || !len_dev))) return LX_ERR_ARG;
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "getter before lx_reset");
    NOT_LOADING(h);
    if (h->rowseg() && h->rs_state != 4) return h->fail(LX_ERR_STATE, "row-segment rank: getters before lx_rowseg_finish");
    if (slot_bytes < 8ull * std::max(h->B, h->V) || slot_bytes % 8)
        return h->fail(LX_ERR_ARG, "row slot of %llu bytes < %llu", (unsigned long long)slot_bytes,
                       8ull * std::max(h->B, h->V));
    int rc;
    if ((rc = flush_pending(h))) return rc;
    HIPCHK(h, set_dev(h->device));
    if (!n) return 0;
    GetArgs a{};
    a.plane = mode == 1 ? h->la : h->hb;
    a.stride = h->pstride;
    a.ev = ev_dev;
    a.n = n;
    a.B = h->B;
    a.V = h->V;
    a.mode = mode;
    a.forks = h->B > h->V ? 1u : 0u;
    a.ev_bbefore = h->ev_bbefore;
    a.ev_branch = h->ev_branch;
    a.branch_first = h->branch_first;
    a.cheat_of = h->cheat_of;
    a.cheat_off = h->cheat_off;
    a.cheat_br = h->cheat_br;
    a.len = len_dev;
    a.out = out_dev;
    a.slot = slot_bytes;
    a.row_lo = h->rowseg() ? h->rs_lo : 0u;
    a.row_hi = h->rowseg() ? h->rs_hi : (uint32_t)h->n_events;
    if (h->sharded()) {
        // this shard's branches only, the rest of every slot zero: the shards'
        // slots sum word by word to the whole row (lx_shard_get_rows)
        a.cmap = h->cmap;
        HIPCHK(h, hipMemsetAsync(out_dev, 0, (uint64_t)n * slot_bytes, h->stream));
    }
    HIPCHK(h, lx::launch_get_rows(a, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_get_branches_info(lx_index *h, uint32_t *last_seq, uint32_t *creator_idx, uint32_t cap, uint32_t *n_branches) {
    if (!h) return LX_ERR_ARG;
    NOT_LOADING(h);
    if (n_branches) *n_branches = h->B;
    if (!cap) return 0;
    HIPCHK(h, set_dev(h->device));
    int rc;
    if ((rc = hm_sync(h))) return rc;
    const std::vector<uint32_t> &len = h->hm_blen;
    for (uint32_t b = 0; b < h->B && b < cap; b++) {
        if (last_seq) last_seq[b] = len[b] ? h->h_branch_first[b] + len[b] - 1 : 0;
        if (creator_idx) creator_idx[b] = h->h_branch_creator[b];
    }
    return 0;
}

int lx_shard_of(const lx_index *h, uint32_t *rank, uint32_t *count) {
    if (!h) return LX_ERR_ARG;
    if (rank) *rank = h->shard_rank;
    if (count) *count = h->shard_count;
    return 0;
}

int lx_shard_range(const lx_index *h, uint32_t shard, uint32_t *lo, uint32_t *hi) {
    if (!h || shard >= h->shard_count) return LX_ERR_ARG;
    shard_bounds(h, shard, lo, hi);
    return 0;
}

// Wire width of a LowestAfter block entry: LA entries are seqs or 0, so while
// every seq of the epoch is < 2^16 they travel as uint16 (half the all-to-all
// bytes).  max_seq follows the event stream, which every shard indexes whole,
// so all shards agree on the width.  Option shard_wire=4 forces uint32.
static uint32_t shard_wire_bytes(const lx_index *h) {
    return (h->wire_force != 4 && h->max_seq <= 0xFFFFu) ? 2u : 4u;
}

int lx_shard_wire(lx_index *h, uint32_t *bytes_per_entry) {
    if (!h || !bytes_per_entry) return LX_ERR_ARG;
    *bytes_per_entry = shard_wire_bytes(h);
    return 0;
}

int lx_shard_block(lx_index *h, uint32_t src, uint32_t dst, uint64_t *elems) {
    if (!h || !elems || src >= h->shard_count || dst >= h->shard_count) return LX_ERR_ARG;
    HIPCHK(h, set_dev(h->device));
    int rc;
    if ((rc = h->sx_active ? ensure_shard_cols(h) : ensure_shard_rows(h))) return rc;
    const uint64_t nrows = h->sx_active ? h->sx_roff[src + 1] - h->sx_roff[src] : h->sc_nrows[src];
    *elems = nrows * (h->sc_col_off[dst + 1] - h->sc_col_off[dst]);
    return 0;
}

// rows of shard `rows_of` x columns of shard `cols_of`, moved by `mode`
// (0 pack, 1 unpack, 2 own block, 3 byte-wire check into buf[0]); wire 0 = the
// epoch's width (shard_wire_bytes)
static int la_xfer(lx_index *h, uint32_t rows_of, uint32_t cols_of, uint32_t *buf, int mode, uint32_t wire = 0) {
    if (!h->sharded()) return h->fail(LX_ERR_STATE, "LowestAfter exchange needs a column-sharded handle");
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "exchange before lx_reset");
    HIPCHK(h, set_dev(h->device));
    int rc;
    if ((rc = h->sx_active ? ensure_shard_cols(h) : ensure_shard_rows(h))) return rc;
    const uint32_t c0 = h->sc_col_off[cols_of], c1 = h->sc_col_off[cols_of + 1];
    XferArgs x{};
    x.lap = h->lap;
    x.lap_stride = h->stride;
    x.s_cap = h->s_cap;
    x.la = h->la;
    x.pstride = h->pstride;
    x.cmap = h->cmap;
    x.ev_branch = h->ev_branch;
    x.ev_seq = h->ev_seq;
    x.branch_first = h->branch_first;
    // the dirty rows of an incremental exchange (lx_shard_dirty_set), else every row
    x.rows = h->sx_active ? h->sx_rows + h->sx_roff[rows_of] : h->sc_rows[rows_of];
    x.nrows = h->sx_active ? (uint32_t)(h->sx_roff[rows_of + 1] - h->sx_roff[rows_of]) : h->sc_nrows[rows_of];
    x.cols = h->sc_cols + c0;
    x.ncols = c1 - c0;
    x.buf = buf;
    x.mode = mode;
    x.wire = wire ? wire : shard_wire_bytes(h);
    const bool check = mode == 3 || (mode == 0 && x.wire == 1);
    if (check) {
        if (!h->wire_flag) HIPCHK(h, dalloc(&h->wire_flag, 1));
        HIPCHK(h, hipMemsetAsync(h->wire_flag, 0, 4, h->stream));
        x.flag = h->wire_flag;
        if (mode == 3) x.buf = h->wire_flag;
    }
    HIPCHK(h, lx::launch_la_xfer(x, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (check) {
        uint32_t bad = 0;
        HIPCHK(h, hipMemcpy(&bad, h->wire_flag, 4, hipMemcpyDeviceToHost));
        if (mode == 3) return bad ? 1 : 0;
        if (bad) return h->fail(LX_ERR_WIRE, "LowestAfter block to shard %u does not fit the 1-byte wire", cols_of);
    }
    return 0;
}

int lx_la_pack_dev(lx_index *h, uint32_t dst, uint32_t *out, void *stream) {
    if (!h || dst >= h->shard_count || dst == h->shard_rank || !out) return LX_ERR_ARG;
    (void)stream;
    return la_xfer(h, h->shard_rank, dst, out, 0);
}

int lx_la_unpack_dev(lx_index *h, uint32_t src, const uint32_t *in, void *stream) {
    if (!h || src >= h->shard_count || src == h->shard_rank || !in) return LX_ERR_ARG;
    (void)stream;
    return la_xfer(h, src, h->shard_rank, const_cast<uint32_t *>(in), 1);
}

int lx_shard_block_wire(lx_index *h, uint32_t dst, uint32_t *bytes_per_entry) {
    if (!h || !bytes_per_entry || dst >= h->shard_count || dst == h->shard_rank) return LX_ERR_ARG;
    *bytes_per_entry = shard_wire_bytes(h);
    if (h->wire_force) return 0;               // option shard_wire pins the epoch width
    const int r = la_xfer(h, h->shard_rank, dst, nullptr, 3);
    if (r < 0) return r;
    if (r == 0) *bytes_per_entry = 1;
    return 0;
}

int lx_la_pack_wire_dev(lx_index *h, uint32_t dst, void *out, uint32_t bytes_per_entry) {
    if (!h || dst >= h->shard_count || dst == h->shard_rank || !out) return LX_ERR_ARG;
    if (bytes_per_entry != 1 && bytes_per_entry != 2 && bytes_per_entry != 4) return LX_ERR_ARG;
    if (bytes_per_entry == 1 && h->wire_force)
        return h->fail(LX_ERR_WIRE, "option shard_wire pins the wire to %u bytes", shard_wire_bytes(h));
    return la_xfer(h, h->shard_rank, dst, static_cast<uint32_t *>(out), 0, bytes_per_entry);
}

int lx_la_unpack_wire_dev(lx_index *h, uint32_t src, const void *in, uint32_t bytes_per_entry) {
    if (!h || src >= h->shard_count || src == h->shard_rank || !in) return LX_ERR_ARG;
    if (bytes_per_entry != 1 && bytes_per_entry != 2 && bytes_per_entry != 4) return LX_ERR_ARG;
    return la_xfer(h, src, h->shard_rank, static_cast<uint32_t *>(const_cast<void *>(in)), 1, bytes_per_entry);
}

int lx_la_own_dev(lx_index *h, void *stream) {
    if (!h) return LX_ERR_ARG;
    (void)stream;
    return la_xfer(h, h->shard_rank, h->shard_rank, nullptr, 2);
}

// ---- incremental LowestAfter exchange ("streaming")
//
// An entry LA[(c, s)][j] is written when an event e of branch j first reaches
// (c, s): s in (RAW(prev(e))[c], RAW(e)[c]].  RAW grows
// along a branch, so every entry written since the last exchange lies at
// s > RAW(p_j)[c], p_j = branch j's last event at that exchange (none: from
// the branch's first seq).  dmin[c] = min over the branches with new events
// of RAW(p_j)[c] + 1 is therefore the first row of branch c that can have
// changed; rows below it are unchanged on every receiver.  Only the owner of
// column c holds RAW(.)[c]: each rank reports its own columns, the ranks
// combine them by an element-wise min, and every rank lists the same dirty
// rows for every shard (branch order, then seq).  A DropNotFlushed, reset or
// load makes the next exchange a full one.

int lx_shard_dirty(lx_index *h, uint32_t nb, uint32_t *dmin) {
    if (!h || !dmin) return LX_ERR_ARG;
    if (!h->sharded()) return h->fail(LX_ERR_STATE, "the incremental exchange needs a column-sharded handle");
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "exchange before lx_reset");
    if (nb < h->B) return h->fail(LX_ERR_ARG, "dmin holds %u branches < %u", nb, h->B);
    HIPCHK(h, set_dev(h->device));
    int rc;
    if ((rc = flush_pending(h)) || (rc = ensure_shard_cols(h))) return rc;
    for (uint32_t b = 0; b < nb; b++) dmin[b] = LX_NONE;
    const uint32_t c0 = h->sc_col_off[h->shard_rank], c1 = h->sc_col_off[h->shard_rank + 1];
    if (h->sx_cap < h->stride || !h->sx_len) {
        for (void *p : {(void *)h->sx_len, (void *)h->sx_dmin})
            if (p) (void)hipFree(p);
        h->sx_len = h->sx_dmin = nullptr;
        h->sx_cap = 0;
        HIPCHK(h, dalloc(&h->sx_len, h->stride));
        HIPCHK(h, dalloc(&h->sx_dmin, h->stride));
        HIPCHK(h, hipMemsetAsync(h->sx_len, 0, (uint64_t)h->stride * 4, h->stream));
        h->sx_cap = h->stride;
        h->sx_full = true;
    }
    if (h->sx_full) {
        // whole blocks: every row of every own branch
        const std::vector<uint32_t> own = shard_cols(h, h->shard_rank);
        for (uint32_t c : own) dmin[c] = h->h_branch_first[c];
        return 0;
    }
    if (!h->B || c1 == c0) return 0;
    HIPCHK(h, lx::launch_fill_u32(h->sx_dmin, h->B, LX_NONE, h->stream));
    HIPCHK(h, lx::launch_shard_dmin(h->hb, h->pstride, h->cmap, h->branch_len, h->brow, h->s_cap, h->branch_first,
                                    h->sx_len, h->B, h->sc_cols + c0, c1 - c0, h->sx_dmin, h->stream));
    HIPCHK(h, hipMemcpyAsync(dmin, h->sx_dmin, 4ull * h->B, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int lx_shard_dirty_set(lx_index *h, uint32_t nb, const uint32_t *dmin) {
    if (!h || !dmin) return LX_ERR_ARG;
    if (!h->sharded()) return h->fail(LX_ERR_STATE, "the incremental exchange needs a column-sharded handle");
    if (nb < h->B) return h->fail(LX_ERR_ARG, "dmin holds %u branches < %u", nb, h->B);
    HIPCHK(h, set_dev(h->device));
    int rc;
    if ((rc = ensure_shard_cols(h))) return rc;
    const uint32_t B = h->B, G = h->shard_count;
    std::vector<uint32_t> len(B);
    if (B) HIPCHK(h, hipMemcpyAsync(len.data(), h->branch_len, 4ull * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    // per shard, its branches in order: {branch, first dirty index, row offset}
    std::vector<uint32_t> meta;
    std::vector<uint64_t> moff;
    h->sx_roff.assign(G + 1, 0);
    uint64_t total = 0;
    for (uint32_t q = 0; q < G; q++) {
        h->sx_roff[q] = total;
        for (uint32_t c : shard_cols(h, q)) {
            const uint32_t first = h->h_branch_first[c];
            uint32_t start = len[c];
            if (dmin[c] != LX_NONE) start = dmin[c] <= first ? 0u : std::min(dmin[c] - first, len[c]);
            if (start == len[c]) continue;
            meta.push_back(c);
            meta.push_back(start);
            meta.push_back((uint32_t)total);
            meta.push_back(len[c] - start);
            total += len[c] - start;
        }
    }
    h->sx_roff[G] = total;
    if (total > 0xFFFFFFFFull) return h->fail(LX_ERR_ARG, "too many dirty rows");
    if ((rc = grow_scratch(h, &h->sx_rows, &h->sx_rows_cap, total + 1)) ||
        (rc = grow_scratch(h, &h->sx_meta, &h->sx_meta_cap, (uint64_t)meta.size() + 4)))
        return rc;
    if (!meta.empty()) {
        HIPCHK(h, hipMemcpyAsync(h->sx_meta, meta.data(), meta.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, lx::launch_shard_dirty_rows(h->brow, h->s_cap, h->sx_meta, (uint32_t)(meta.size() / 4), h->sx_rows,
                                              h->stream));
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));   // `meta` is a host temporary
    h->sx_active = true;
    return 0;
}

int lx_shard_dirty_commit(lx_index *h) {
    if (!h) return LX_ERR_ARG;
    if (!h->sharded()) return h->fail(LX_ERR_STATE, "the incremental exchange needs a column-sharded handle");
    HIPCHK(h, set_dev(h->device));
    if (h->sx_len && h->B) {
        HIPCHK(h, hipMemcpyAsync(h->sx_len, h->branch_len, 4ull * h->B, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->sx_full = false;
    }
    h->sx_active = false;
    return 0;
}

int lx_last_stats(const lx_index *h, lx_stats *out) {
    if (!h || !out) return LX_ERR_ARG;
    *out = h->stats;
    if (h->stats_lazy) {
        // small path: the launch is timed by ev[1..2]; wait for it only when asked
        float t = 0;
        if (hipEventSynchronize(h->ev[2]) == hipSuccess && hipEventElapsedTime(&t, h->ev[1], h->ev[2]) == hipSuccess)
            out->ms_index = t;
    }
    return 0;
}

int lx_device_planes(lx_index *h, void **hb, void **la, uint32_t *stride, void **stream) {
    if (!h) return LX_ERR_ARG;
    HIPCHK(h, set_dev(h->device));
    {
        const int rc = flush_pending(h);   // the caller reads the planes in stream order after this
        if (rc) return rc;
    }
    if (hb) *hb = h->hb;
    if (la) *la = h->la;
    if (stride) *stride = h->pstride;
    if (stream) *stream = h->stream;
    return 0;
}

int lx_device_bytes(const lx_index *h, uint64_t out[4]) {
    if (!h || !out) return LX_ERR_ARG;
    const uint64_t ps = h->pstride;
    uint64_t planes = h->rs_hb_mem ? 2 * h->rs_mem_rows * ps * 4 : (h->hb ? 2 * h->n_cap * ps * 4 : 0);
    if (h->lap) planes += (uint64_t)h->pstride * h->s_cap * h->stride * 4;
    const uint64_t recv = 4 * (h->rs_rhb_cap + h->rs_rla_cap);
    uint64_t per_ev = 6 * 4 * h->n_cap;   // creator, seq, branch, bbefore, sp, first_child
    for (uint64_t c : {h->seg_mf_cap, h->seg_plist_cap, h->seg_elist_cap, h->rs_need_cap, h->rs_hslot_cap,
                       h->rs_lslot_cap, h->rs_stamp_cap, h->wb_cap})
        per_ev += 4 * c;
    uint64_t other = 4 * ((uint64_t)h->stride * h->s_cap + 5ull * h->stride + h->tail_cap * (uint64_t)h->tail_cap * 2);
    other += 4 * (8 * h->batch_cap + h->par_cap + 2 * h->q_cap) + h->q_cap + 16 * h->batch_cap;
    other += 4 * (h->rs_req_cap + h->rs_ids_cap + h->rs_out_cap + h->rs_send_cap + h->rsq_scratch_cap + h->rsq_list_cap) +
             h->rsq_tmp_bytes + h->scan_bytes;
    out[0] = planes;
    out[1] = recv;
    out[2] = per_ev;
    out[3] = other;
    return 0;
}

int lx_last_segment_stats(const lx_index *h, lx_seg_stats *out) {
    if (!h || !out) return LX_ERR_ARG;
    *out = h->seg_stats;
    return 0;
}

int lx_sync(lx_index *h) {
    if (!h) return LX_ERR_ARG;
    HIPCHK(h, set_dev(h->device));
    {
        const int rc = flush_pending(h);
        if (rc) return rc;
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    // the unknown-event flag of asynchronous ForklessCause batches: read only
    // when one ran since the last check (a blocking 4-byte copy costs ~10 us,
    // the whole of an Add-and-sync otherwise)
    if (!h->fc_unchecked) return 0;
    h->fc_unchecked = false;
    uint32_t bad = 0;
    HIPCHK(h, hipMemcpy(&bad, h->status + 1, 4, hipMemcpyDeviceToHost));
    if (bad) {
        HIPCHK(h, hipMemset(h->status + 1, 0, 4));
        return h->fail(LX_ERR_ARG, "ForklessCause on an unknown event");
    }
    return 0;
}

// ---- restart from the persisted tables (abft/restart_test.go:156-188)

// go-ethereum rlp (v1.9.22) reader for BranchesInfo: a list of three lists
// (uint, uint, list of uint lists), uints minimal big-endian
struct RlpIn {
    const uint8_t *p, *end;
    bool ok = true;
    // header of the next item: list?, payload bounds
    bool item(bool *list, const uint8_t **b, const uint8_t **e) {
        if (p >= end) return ok = false;
        const uint8_t x = *p;
        uint64_t len = 0, hl = 1;
        if (x < 0x80) { *list = false; *b = p; *e = p + 1; p++; return true; }
        if (x <= 0xB7) { *list = false; len = x - 0x80; }
        else if (x <= 0xBF) { *list = false; hl += x - 0xB7; }
        else if (x <= 0xF7) { *list = true; len = x - 0xC0; }
        else { *list = true; hl += x - 0xF7; }
        if (hl > 1) {
            if ((uint64_t)(end - p) < hl || hl > 9) return ok = false;
            for (uint64_t k = 1; k < hl; k++) len = (len << 8) | p[k];
        }
        if ((uint64_t)(end - p) < hl + len) return ok = false;
        *b = p + hl;
        *e = p + hl + len;
        p = *e;
        return true;
    }
    bool uint_list(const uint8_t *b, const uint8_t *e, std::vector<uint32_t> &out) {
        RlpIn r{b, e};
        while (r.p < r.end) {
            bool l;
            const uint8_t *x, *y;
            if (!r.item(&l, &x, &y) || l || y - x > 4) return ok = false;
            uint32_t v = 0;
            for (const uint8_t *q = x; q < y; q++) v = (v << 8) | *q;
            out.push_back(v);
        }
        return true;
    }
};

static bool decode_branches_info(const uint8_t *d, uint32_t n, std::vector<uint32_t> &last, std::vector<uint32_t> &cr,
                                 std::vector<std::vector<uint32_t>> &by) {
    RlpIn r{d, d + n};
    bool l;
    const uint8_t *b, *e;
    if (!r.item(&l, &b, &e) || !l || r.p != r.end) return false;
    RlpIn body{b, e};
    const uint8_t *x, *y;
    if (!body.item(&l, &x, &y) || !l || !body.uint_list(x, y, last)) return false;
    if (!body.item(&l, &x, &y) || !l || !body.uint_list(x, y, cr)) return false;
    if (!body.item(&l, &x, &y) || !l) return false;
    RlpIn lists{x, y};
    while (lists.p < lists.end) {
        const uint8_t *u, *v;
        if (!lists.item(&l, &u, &v) || !l) return false;
        by.emplace_back();
        if (!lists.uint_list(u, v, by.back())) return false;
    }
    return body.p == body.end && body.ok && lists.ok;
}

static int load_fail(lx_index *h, const char *fmt, uint64_t a = 0, uint64_t b = 0) {
    char buf[256];
    snprintf(buf, sizeof buf, fmt, (unsigned long long)a, (unsigned long long)b);
    h->loading = false;
    h->have_epoch = false;   // the handle needs lx_reset
    return h->fail(LX_ERR_STATE, "inconsistent DB: %s", buf);
}

int lx_load_rows(lx_index *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff,
                 const uint32_t *par, const uint8_t *branch_be, const uint64_t *hb_off, const uint8_t *hb_bytes,
                 const uint64_t *la_off, const uint8_t *la_bytes) {
    if (!h) return LX_ERR_ARG;
    WHOLE_INDEX(h);
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "lx_load_rows before lx_reset");
    if (h->sharded()) return h->fail(LX_ERR_STATE, "lx_load_rows needs an unsharded handle");
    if (!n) return 0;
    if (!creator || !seq || !poff || !branch_be || !hb_off || !hb_bytes || !la_off || !la_bytes)
        return h->fail(LX_ERR_ARG, "null input");
    if (!h->loading) {
        if (h->n_events) return h->fail(LX_ERR_STATE, "lx_load_rows needs a freshly reset handle");
        h->loading = true;
        h->ld_first.assign(h->V, 1);
        h->ld_last.assign(h->V, 0);
        h->ld_count.assign(h->V, 0);
        h->ld_tail.assign(h->V, LX_NONE);
        h->ld_creator.resize(h->V);
        for (uint32_t c = 0; c < h->V; c++) h->ld_creator[c] = c;
        h->ld_par.clear();
        h->ld_poff.assign(1, 0);
        h->ld_B = h->V;
    }
    HIPCHK(h, set_dev(h->device));
    const uint64_t bs = h->n_events;
    uint32_t max_hent = 0, max_lent = 0, bmax = h->max_seq;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t g = bs + i;
        const uint32_t c = creator[i], s = seq[i];
        const uint64_t p0 = poff[i], p1 = poff[i + 1];
        const uint32_t br = ((uint32_t)branch_be[4 * i] << 24) | ((uint32_t)branch_be[4 * i + 1] << 16) |
                            ((uint32_t)branch_be[4 * i + 2] << 8) | branch_be[4 * i + 3];
        if (c >= h->V || s == 0 || s >= 0x7FFFFFFEu || p1 < p0) return load_fail(h, "event %llu: bad creator/seq", g);
        for (uint64_t x = p0; x < p1; x++)
            if (par[x] >= g) return load_fail(h, "event %llu: parent %llu not loaded before it", g, par[x]);
        const uint32_t sp = s > 1 ? (p1 > p0 ? par[p0] : LX_NONE) : LX_NONE;
        if (s > 1 && (sp == LX_NONE || h->hm_creator[sp] != c || h->hm_seq[sp] + 1 != s))
            return load_fail(h, "event %llu: self-parent", g);
        if (br < h->V && br != c) return load_fail(h, "event %llu: branch %llu of another creator", g, br);
        if (br >= (1u << 24)) return load_fail(h, "event %llu: branch ID %llu", g, br);
        if (br >= h->ld_first.size()) {
            h->ld_first.resize(br + 1, 0);
            h->ld_last.resize(br + 1, 0);
            h->ld_count.resize(br + 1, 0);
            h->ld_tail.resize(br + 1, LX_NONE);
            h->ld_creator.resize(br + 1, LX_NONE);
        }
        const bool opens = h->ld_count[br] == 0;
        if (opens) {
            if (br < h->V && s != 1) return load_fail(h, "event %llu: first of branch %llu", g, br);
            h->ld_first[br] = s;
            h->ld_creator[br] = c;
        } else if (h->ld_creator[br] != c || s != h->ld_last[br] + 1 || sp != h->ld_tail[br]) {
            return load_fail(h, "event %llu: does not continue branch %llu", g, br);
        }
        h->ld_last[br] = s;
        h->ld_tail[br] = (uint32_t)g;
        h->ld_count[br]++;
        h->ld_B = std::max(h->ld_B, br + 1);
        // branches before its Add, from the HighestBefore byte length: 8 x (B
        // before + 1) when it opened a fork branch, else 8 x B before
        // (vecengine/index.go:147, vecfc/vector.go:82-89)
        const uint64_t hl = hb_off[i + 1] - hb_off[i], ll = la_off[i + 1] - la_off[i];
        if (hb_off[i + 1] < hb_off[i] || la_off[i + 1] < la_off[i] || hl % 8 || ll % 4 || hl / 8 > 0xFFFFFF || ll / 4 > 0xFFFFFF)
            return load_fail(h, "event %llu: vector byte lengths", g);
        const uint32_t hent = (uint32_t)(hl / 8), lent = (uint32_t)(ll / 4);
        const bool fork_open = opens && br >= h->V;
        const uint32_t bb = fork_open ? br : hent;
        if ((fork_open ? hent != br + 1 : (hent < h->V || br >= hent)) || lent < bb + (fork_open ? 1u : 0u))
            return load_fail(h, "event %llu: vector lengths disagree with branch %llu", g, br);
        max_hent = std::max(max_hent, hent);
        max_lent = std::max(max_lent, lent);
        bmax = std::max(bmax, s);
        h->hm_creator.push_back(c);
        h->hm_seq.push_back(s);
        h->hm_branch.push_back(br);
        h->hm_bbefore.push_back(bb);
        h->ld_par.insert(h->ld_par.end(), par + p0, par + p1);
        h->ld_poff.push_back(h->ld_par.size());
    }
    h->max_seq = bmax;
    int rc;
    if ((rc = grow_events(h, bs + n)) || (rc = grow_branches(h, std::max({h->ld_B, max_hent, max_lent}))) ||
        (rc = grow_scap(h, bmax)))
        return rc;
    hipStream_t st = h->stream;
    // metadata of the chunk (the mirror vectors stay alive until the sync below)
    std::vector<uint32_t> sp(n);
    for (uint32_t i = 0; i < n; i++)
        sp[i] = seq[i] > 1 ? par[poff[i]] : LX_NONE;
    HIPCHK(h, hipMemcpyAsync(h->ev_creator + bs, h->hm_creator.data() + bs, n * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ev_seq + bs, h->hm_seq.data() + bs, n * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ev_branch + bs, h->hm_branch.data() + bs, n * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ev_bbefore + bs, h->hm_bbefore.data() + bs, n * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ev_sp + bs, sp.data(), n * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->branch_first, h->ld_first.data(), h->ld_B * 4ull, hipMemcpyHostToDevice, st));
    // the chunk's table bytes and offsets
    const uint64_t hb_n = hb_off[n] - hb_off[0], la_n = la_off[n] - la_off[0];
    const uint64_t o_hoff = (hb_n + la_n + 15) / 16 * 16, o_loff = o_hoff + 8ull * (n + 1);
    const uint64_t need = o_loff + 8ull * (n + 1);
    if (need > h->ld_buf_cap) {
        if (h->ld_buf) {
            HIPCHK(h, hipStreamSynchronize(st));
            (void)hipFree(h->ld_buf);
        }
        h->ld_buf = nullptr;
        h->ld_buf_cap = 0;
        HIPCHK(h, hipMalloc((void **)&h->ld_buf, need));
        h->ld_buf_cap = need;
    }
    HIPCHK(h, hipMemcpyAsync(h->ld_buf, hb_bytes + hb_off[0], hb_n, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ld_buf + hb_n, la_bytes + la_off[0], la_n, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ld_buf + o_hoff, hb_off, 8ull * (n + 1), hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->ld_buf + o_loff, la_off, 8ull * (n + 1), hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemsetAsync(h->status + 5, 0, 4, st));
    LoadArgs a{};
    a.hb = h->hb;
    a.la = h->la;
    a.stride = h->stride;
    a.bs = (uint32_t)bs;
    a.n = n;
    a.B = h->ld_B;
    a.hb_off = reinterpret_cast<const uint64_t *>(h->ld_buf + o_hoff);
    a.la_off = reinterpret_cast<const uint64_t *>(h->ld_buf + o_loff);
    a.hb_base = hb_off[0];
    a.la_base = la_off[0] - hb_n;   // la bytes follow the hb bytes in the staging buffer
    a.hb_bytes = h->ld_buf;
    a.la_bytes = h->ld_buf;
    a.ev_branch = h->ev_branch;
    a.ev_seq = h->ev_seq;
    a.branch_first = h->branch_first;
    a.brow = h->brow;
    a.s_cap = h->s_cap;
    a.bad = h->status + 5;
    HIPCHK(h, lx::launch_load_rows(a, st));
    uint32_t bad = 0;
    HIPCHK(h, hipMemcpyAsync(&bad, h->status + 5, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (bad) return load_fail(h, "HighestBefore entries (MinSeq, own seq or branch) in events %llu..%llu", bs, bs + n - 1);
    h->n_events = bs + n;
    h->hwm = std::max(h->hwm, h->n_events);
    h->hm_n = h->n_events;
    return 0;
}

int lx_load_finish(lx_index *h, const uint8_t *bi_rlp, uint32_t bi_len) {
    if (!h) return LX_ERR_ARG;
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "lx_load_finish before lx_reset");
    if (!h->loading && h->n_events) return h->fail(LX_ERR_STATE, "lx_load_finish without lx_load_rows");
    if (!bi_rlp) return h->fail(LX_ERR_ARG, "null BranchesInfo");
    HIPCHK(h, set_dev(h->device));
    if (!h->loading) {   // an empty epoch: the initial BranchesInfo
        h->ld_first.assign(h->V, 1);
        h->ld_last.assign(h->V, 0);
        h->ld_count.assign(h->V, 0);
        h->ld_creator.resize(h->V);
        for (uint32_t c = 0; c < h->V; c++) h->ld_creator[c] = c;
        h->ld_poff.assign(1, 0);
        h->ld_B = h->V;
        h->loading = true;
    }
    std::vector<uint32_t> last, cr;
    std::vector<std::vector<uint32_t>> by;
    if (!decode_branches_info(bi_rlp, bi_len, last, cr, by)) return load_fail(h, "RLP(BranchesInfo) malformed");
    const uint32_t V = h->V, B = (uint32_t)last.size();
    if (cr.size() != B || by.size() != V || B < V || B < h->ld_B) return load_fail(h, "BranchesInfo sizes (B %llu)", B);
    h->ld_first.resize(B, 0);
    h->ld_last.resize(B, 0);
    h->ld_count.resize(B, 0);
    h->ld_creator.resize(B, LX_NONE);
    std::vector<std::vector<uint32_t>> want(V);
    for (uint32_t b = 0; b < B; b++) {
        if (cr[b] >= V || (b < V && cr[b] != b)) return load_fail(h, "branch %llu creator", b);
        if (b >= V && !h->ld_count[b]) return load_fail(h, "fork branch %llu has no event", b);
        if (h->ld_count[b] && h->ld_creator[b] != cr[b]) return load_fail(h, "branch %llu creator", b);
        if (last[b] != h->ld_last[b]) return load_fail(h, "branch %llu last seq %llu", b, last[b]);   // branches_info.go:11
        want[cr[b]].push_back(b);
    }
    for (uint32_t c = 0; c < V; c++)
        if (by[c] != want[c]) return load_fail(h, "branches of creator %llu", c);
    const uint64_t N = h->n_events;
    int rc;
    if ((rc = grow_branches(h, B))) return rc;
    h->B = h->B_flushed = B;
    h->h_branch_creator = cr;
    h->h_branch_first.assign(B, 1);
    std::vector<uint32_t> blen(B, 0);
    for (uint32_t b = 0; b < B; b++) {
        if (h->ld_count[b]) h->h_branch_first[b] = h->ld_first[b];
        blen[b] = h->ld_count[b];
    }
    h->by_creator = by;
    h->hm_blen = blen;
    h->hm_ok = true;
    h->hm_n = N;
    // claims: the continuing self-child of each event, each creator's first root
    std::vector<uint32_t> fchild(N, LX_NONE), froot(V, LX_NONE);
    for (uint64_t e = 0; e < N; e++) {
        const uint32_t s = h->hm_seq[e], br = h->hm_branch[e];
        if (s > 1) {
            const uint32_t sp = h->ld_par[h->ld_poff[e]];
            if (h->hm_branch[sp] == br) fchild[sp] = (uint32_t)e;
        } else if (br < V) {
            froot[br] = (uint32_t)e;
        }
    }
    hipStream_t st = h->stream;
    HIPCHK(h, hipMemcpyAsync(h->branch_first, h->h_branch_first.data(), B * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->branch_creator, cr.data(), B * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->branch_len, blen.data(), B * 4ull, hipMemcpyHostToDevice, st));
    if (N) HIPCHK(h, hipMemcpyAsync(h->first_child, fchild.data(), N * 4ull, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(h->first_root, froot.data(), V * 4ull, hipMemcpyHostToDevice, st));
    h->pcols_used = std::max(h->pcols_used, B);
    if ((rc = rebuild_columns(h))) return rc;   // syncs the stream
    if (N) {
        // fork markers only in cheaters' columns (k_load_raw / k_load_check
        // below verify those); a marker anywhere else is corrupt
        std::vector<uint32_t> cheat_col(B, 0);
        for (uint32_t b = 0; b < B; b++) cheat_col[b] = by[cr[b]].size() > 1 ? 1u : 0u;
        uint32_t *d_cc = nullptr;
        HIPCHK(h, hipMalloc((void **)&d_cc, 4ull * B));
        HIPCHK(h, hipMemcpyAsync(d_cc, cheat_col.data(), 4ull * B, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemsetAsync(h->status + 5, 0, 4, st));
        HIPCHK(h, lx::launch_load_marks_ok(h->hb, h->stride, (uint32_t)N, B, d_cc, h->status + 5, st));
        uint32_t bad = 0;
        HIPCHK(h, hipMemcpyAsync(&bad, h->status + 5, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        (void)hipFree(d_cc);
        if (bad) return load_fail(h, "fork marker in a column of a creator with one branch");
    }
    if (B > V && h->n_cheat && N) {
        // raw seqs behind the fork markers (cheaters' columns), then the markers
        // re-derived from them must be exactly the loaded ones
        std::vector<uint32_t> cols;
        for (uint32_t c = 0; c < V; c++)
            if (by[c].size() > 1) cols.insert(cols.end(), by[c].begin(), by[c].end());
        const uint32_t ncc = (uint32_t)cols.size();
        std::vector<uint32_t> lvl(N), perm(N);
        uint32_t L = 0;
        for (uint64_t e = 0; e < N; e++) {
            uint32_t l = 0;
            for (uint64_t k = h->ld_poff[e]; k < h->ld_poff[e + 1]; k++) l = std::max(l, lvl[h->ld_par[k]] + 1);
            lvl[e] = l;
            L = std::max(L, l + 1);
        }
        std::vector<uint32_t> off(L + 1, 0);
        for (uint64_t e = 0; e < N; e++) off[lvl[e] + 1]++;
        for (uint32_t l = 0; l < L; l++) off[l + 1] += off[l];
        std::vector<uint32_t> cur(off.begin(), off.end() - 1);
        for (uint64_t e = 0; e < N; e++) perm[cur[lvl[e]]++] = (uint32_t)e;
        const uint64_t npar = h->ld_par.size();
        uint8_t *scratch = nullptr;
        const uint64_t o_perm = 4ull * ncc, o_off = o_perm + 4ull * N, o_poff = (o_off + 4ull * (L + 1) + 7) / 8 * 8,
                       o_par = o_poff + 8ull * (N + 1), o_lm = o_par + 4ull * std::max<uint64_t>(npar, 1);
        HIPCHK(h, hipMalloc((void **)&scratch, o_lm + N * ncc));
        HIPCHK(h, hipMemcpyAsync(scratch, cols.data(), 4ull * ncc, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(scratch + o_perm, perm.data(), 4ull * N, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(scratch + o_off, off.data(), 4ull * (L + 1), hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(scratch + o_poff, h->ld_poff.data(), 8ull * (N + 1), hipMemcpyHostToDevice, st));
        if (npar) HIPCHK(h, hipMemcpyAsync(scratch + o_par, h->ld_par.data(), 4ull * npar, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemsetAsync(h->status + 5, 0, 4, st));
        LoadRawArgs r{};
        r.hb = h->hb;
        r.stride = h->stride;
        r.cols = reinterpret_cast<const uint32_t *>(scratch);
        r.ncc = ncc;
        r.perm = reinterpret_cast<const uint32_t *>(scratch + o_perm);
        r.lvl_off = reinterpret_cast<const uint32_t *>(scratch + o_off);
        r.n_levels = L;
        r.poff = reinterpret_cast<const uint64_t *>(scratch + o_poff);
        r.par = reinterpret_cast<const uint32_t *>(scratch + o_par);
        r.ev_branch = h->ev_branch;
        r.ev_seq = h->ev_seq;
        r.lm = scratch + o_lm;
        r.bad = h->status + 5;
        HIPCHK(h, lx::launch_load_raw(r, st));
        MarkArgs m{};
        m.hb = h->hb;
        m.stride = h->pstride;
        m.batch_start = 0;
        m.n = (uint32_t)N;
        m.V = V;
        m.ev_branch = h->ev_branch;
        m.ev_bbefore = h->ev_bbefore;
        m.branch_first = h->branch_first;
        m.n_cheat = h->n_cheat;
        m.cheat_off = h->cheat_off;
        m.cheat_br = h->cheat_br;
        HIPCHK(h, lx::launch_marks(m, st));
        HIPCHK(h, lx::launch_load_check(r, (uint32_t)N, st));
        uint32_t bad = 0;
        HIPCHK(h, hipMemcpyAsync(&bad, h->status + 5, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        (void)hipFree(scratch);
        if (bad) return load_fail(h, "fork markers / raw HighestBefore do not follow from the vectors (flags %llu)", bad);
    }
    if (N) {
        LoadVerifyArgs v{};
        v.hb = h->hb;
        v.la = h->la;
        v.stride = h->stride;
        v.n = (uint32_t)N;
        v.B = B;
        v.ev_branch = h->ev_branch;
        v.ev_seq = h->ev_seq;
        v.branch_first = h->branch_first;
        v.branch_len = h->branch_len;
        v.brow = h->brow;
        v.s_cap = h->s_cap;
        v.bad = h->status + 5;
        HIPCHK(h, hipMemsetAsync(h->status + 5, 0, 4, st));
        HIPCHK(h, lx::launch_load_verify_la(v, st));
        uint32_t bad = 0;
        HIPCHK(h, hipMemcpyAsync(&bad, h->status + 5, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        if (bad) return load_fail(h, "LowestAfter rows do not follow from the HighestBefore rows (flags %llu)", bad);
    }
    h->n_flushed = N;
    h->loading = false;
    h->ld_par.clear();
    h->ld_par.shrink_to_fit();
    h->ld_poff.clear();
    h->ld_poff.shrink_to_fit();
    return 0;
}

}  // extern "C"

// view for the abft engine (lx_abft.cpp); see lx_internal.h
int lx_index_view(lx_index *h, IndexView *o) {
    if (!h || !o) return LX_ERR_ARG;
    WHOLE_INDEX(h);
    if (!h->have_epoch) return h->fail(LX_ERR_STATE, "index has no epoch (lx_reset first)");
    {
        const int rc = flush_pending(h);   // abft and the emitter enqueue after the index's work
        if (rc) return rc;
    }
    o->stream = h->stream;
    o->device = h->device;
    o->hb = h->hb;
    o->la = h->la;
    o->stride = h->pstride;
    o->n_events = h->n_events;
    o->V = h->V;
    o->B = h->B;
    o->quorum = h->quorum;
    o->max_seq = h->max_seq;
    o->wpad = h->wpad;
    o->ev_branch = h->ev_branch;
    o->ev_creator = h->ev_creator;
    o->weights = &h->weights;
    o->by_creator = &h->by_creator;
    o->shard_count = h->shard_count;
    return 0;
}
