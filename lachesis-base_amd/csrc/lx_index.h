// lx_index.h -- the index handle behind the C ABI (include/lachesis_hip.h),
// shared by the host engine (lx_capi.cpp) and the ForklessCause result cache
// (lx_fccache.cpp).  Internal: not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/lachesis_hip.h"
#include "lx_internal.h"

struct FcCache;   // lx_fccache.cpp

namespace lxi {

constexpr uint32_t kStatusWords = 64;   // [1] fc bad flag, [2] max seq, [3] pinned-FC sink, [4] unresolved
                                        // branch, [5] load check flags, [8..9] batch error u64, [16..47] jump flags

template <typename T>
hipError_t dalloc(T **p, uint64_t n) {
    *p = nullptr;
    if (!n) n = 1;
    return hipMalloc((void **)p, n * sizeof(T));
}

inline uint32_t round_up(uint32_t x, uint32_t m) { return (x + m - 1) / m * m; }

// std::vector whose resize leaves new elements default-initialised (no zero
// fill): the small Add path sizes its lists for the worst case per batch and
// writes every element it keeps
template <class T>
struct NoInitAlloc : std::allocator<T> {
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    template <class U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using rawvec = std::vector<T, NoInitAlloc<T>>;

// device scratch grown to `need` elements (contents not kept)
template <typename H, typename T>
int grow_scratch(H *h, T **p, uint64_t *cap, uint64_t need) {
    if (*cap >= need && *p) return 0;
    if (*p) {
        if (int rc = h->hip(hipStreamSynchronize(h->stream), "grow_scratch sync")) return rc;
        (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
    }
    if (int rc = h->hip(dalloc(p, need), "grow_scratch")) return rc;
    *cap = need;
    return 0;
}

// hipSetDevice costs microseconds per call; every entry point makes sure the
// handle's device is current, so switch only when it is not
inline hipError_t set_dev(int device) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == device) return hipSuccess;
    return hipSetDevice(device);
}

}  // namespace lxi

struct lx_index {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t shard_rank = 0, shard_count = 1;
    std::string err;

    // epoch
    uint32_t V = 0;
    std::vector<uint32_t> weights;
    uint32_t quorum = 0;
    uint32_t own_lo = 0, own_hi = 0;
    uint64_t n_events = 0, n_flushed = 0, hwm = 0;
    uint32_t B = 0, B_flushed = 0;
    uint32_t max_seq = 0;
    // LowestAfter tail zeroing (unsharded; TailArgs): per-(j, c) done-up-to seqs
    bool la_tail = true;                   // option la_memset=1: zero the whole LA plane at reset instead
    uint32_t *tail_zw = nullptr, *tail_lo = nullptr, *tail_cmin = nullptr;
    uint32_t tail_cap = 0;
    bool tail_dirty = false;               // zw holds progress (a tail pass ran since it was zeroed)
    uint32_t wire_force = 0;               // option shard_wire=4: LowestAfter blocks always uint32
    uint32_t *wire_flag = nullptr;         // device flag of the byte-wire fit check (4 B)
    uint32_t pcols_used = 0;       // plane columns rows may hold non-zero values in (since the last zeroing)
    bool have_epoch = false;

    // host mirror of BranchesInfo (creator / first seq per branch; by creator)
    std::vector<uint32_t> h_branch_creator, h_branch_first;
    std::vector<std::vector<uint32_t>> by_creator;

    // capacities
    uint64_t n_cap = 0;
    uint32_t stride = 0;   // == branch capacity
    uint32_t pstride = 0;  // row stride of hb / la (= stride; a shard's local column capacity)
    uint32_t s_cap = 0;
    uint64_t cap_hint = 0;
    uint32_t reserve = 0;

    // device state
    uint32_t *hb = nullptr, *la = nullptr;
    uint32_t *ev_creator = nullptr, *ev_seq = nullptr, *ev_branch = nullptr, *ev_bbefore = nullptr,
             *ev_sp = nullptr, *first_child = nullptr;
    uint32_t *first_root = nullptr, *branch_first = nullptr, *branch_creator = nullptr, *branch_len = nullptr,
             *brow = nullptr, *wpad = nullptr, *col_list = nullptr;
    uint32_t *cheat_off = nullptr, *cheat_br = nullptr, *cheat_creator = nullptr;
    uint32_t *cheat_brl = nullptr, *cheat_crl = nullptr;   // the same as plane columns (shards)
    int32_t *cheat_of = nullptr;           // creator -> index into the cheater CSR (-1: one branch)
    uint32_t cheat_of_cap = 0;
    uint32_t n_cheat = 0, ncols = 0;
    // fork-path ForklessCause tables per plane column (k_fc_fk; valid when
    // fk_hi4 != 0): weight of a non-cheater's original, cheater index of a
    // cheater's branches, the cheaters' weights
    uint32_t *fk_w = nullptr, *fk_c = nullptr, *fk_wch = nullptr;
    uint64_t fk_cap = 0;
    uint32_t fk_hi4 = 0;
    bool dbl = true;                       // option dbl=0: the column walker for small fork-free batches too
    bool fc_fk = true;                     // option fc_fk=0: the fix-up loop kernel instead
    // column shard (shard_count > 1): own columns only (lx_internal.h)
    std::vector<uint32_t> h_cmap;          // global branch -> plane column / LX_NONE
    uint32_t nloc = 0;                     // plane columns in use
    uint32_t *cmap = nullptr, *lap = nullptr, *wloc = nullptr;
    uint32_t cmap_cap = 0;
    bool sharded() const { return shard_count > 1; }
    uint64_t cheat_cap = 0;
    uint32_t *status = nullptr;

    // batch scratch
    uint64_t batch_cap = 0, par_cap = 0;
    uint32_t *b_creator = nullptr, *b_seq = nullptr, *b_poff = nullptr, *b_par = nullptr;
    uint32_t *b_isfork = nullptr, *b_rank = nullptr, *b_tmpbr = nullptr, *b_jmp = nullptr;
    EventRec *b_rec = nullptr;
    CRec *b_crec = nullptr;                // compact records (lx_internal.h) of the last batch
    bool b_crec_ok = false;                // ... written (fork-free, 16-bit branches and seqs)
    void *scan_tmp = nullptr;
    size_t scan_bytes = 0;

    // query scratch
    uint64_t q_cap = 0;
    uint32_t *q_a = nullptr, *q_b = nullptr;
    uint8_t *q_out = nullptr;

    // column-shard exchange cache (rows per shard at sc_events)
    uint64_t sc_events = ~0ull;
    uint32_t sc_B = 0;
    std::vector<uint32_t *> sc_rows;
    std::vector<uint32_t> sc_nrows;
    uint32_t *sc_flag = nullptr, *sc_pos = nullptr, *sc_cols = nullptr;
    std::vector<uint32_t> sc_col_off;    // shard q's columns: sc_cols[sc_col_off[q] .. sc_col_off[q+1])
    uint64_t sc_cap = 0;
    void *sc_tmp = nullptr;
    size_t sc_tmp_bytes = 0;
    uint32_t sc_cols_B = 0;               // branch count sc_cols was built for
    // incremental LowestAfter exchange (lx_shard_dirty*): per branch the events it
    // had at the last committed exchange; the dirty row lists of every shard
    uint32_t *sx_len = nullptr, *sx_dmin = nullptr;
    uint32_t sx_cap = 0;
    bool sx_full = true;                  // the next exchange sends whole blocks (reset, drop, load)
    bool sx_active = false;               // pack / unpack / lx_shard_block use the dirty lists
    uint32_t *sx_rows = nullptr, *sx_meta = nullptr;
    uint64_t sx_rows_cap = 0, sx_meta_cap = 0;
    std::vector<uint64_t> sx_roff;        // shard q's dirty rows: sx_rows[sx_roff[q] .. sx_roff[q + 1])

    // write-back (lx_writeback_*): dirty-row flags, row lists, byte offsets
    uint64_t wb_cap = 0, wb_buf_cap = 0;
    uint32_t *wb_flag = nullptr, *wb_pos = nullptr, *wb_la_rows = nullptr, *wb_hb_rows = nullptr, *wb_buf = nullptr;
    uint64_t *wb_len = nullptr, *wb_la_off = nullptr, *wb_hb_off = nullptr;
    void *wb_tmp = nullptr;
    size_t wb_tmp_bytes = 0;
    bool wb_ready = false;
    lx_writeback wb{};
    std::string wb_bi;

    // small-batch (latency) path, lx_small.hip: the host assigns branches in Add
    // order from a mirror of the per-event metadata and stages the batch in
    // pinned memory; one H2D copy + one launch, no sync
    uint32_t small_max = kSmallMaxN;       // option small_max: largest batch on this path (0: never)
    bool hm_ok = false;                    // the mirror equals the device metadata
    uint64_t hm_n = 0;                     // events whose (immutable) metadata the mirror holds
    lxi::rawvec<uint32_t> hm_creator, hm_seq, hm_branch, hm_bbefore;
    std::vector<uint32_t> hm_blen;         // per branch: events on it (= device branch_len)
    std::vector<uint32_t> sm_level, sm_cnt, sm_touched;   // scratch
    lxi::rawvec<uint2> sm_undo;            // add_batch_small: {branch, length before} per event
    // the pending run: small-path events assigned on the host but not launched
    // yet, [pend_bs, pend_bs + pend_n), branches from pend_B0 (flush_pending)
    uint32_t pend_n = 0, pend_B0 = 0, pend_maxlvl = 0;
    uint64_t pend_bs = 0;
    lxi::rawvec<SmallEv> pend_ev;          // records (q1.x = offset into pend_old, q2.w = h0 slot)
    lxi::rawvec<uint32_t> pend_lvl;        // topological level inside the run
    lxi::rawvec<uint2> pend_meta;          // per event {position | chunks << 16, chunk offset into pend_pl}
    lxi::rawvec<uint16_t> pend_pl;         // in-run parents (run positions), chunks of 4 (k_small)
    lxi::rawvec<uint2> pend_old;           // {target, global event}: parents older than the run, older prevs
    uint64_t pend_npar = 0;                // parents of the run (LDS budget, small_fits)
    uint32_t pend_nh = 0;                  // h0 slots of the run
    std::vector<uint32_t> touch_mark;      // per branch: stamp of the last run that touched it
    uint32_t touch_stamp = 0;
    // staging images in flight: slot k = a pinned image and its device copy,
    // copied by a kernel on the handle's stream (k_stage)
    static constexpr int kSlots = 4;
    uint32_t *st_pin[kSlots] = {};
    uint64_t st_pin_cap[kSlots] = {};
    hipEvent_t st_copied[kSlots] = {};     // the copy of slot k finished (its pinned image is free)
    bool st_used[kSlots] = {};
    uint32_t st_next = 0;
    uint32_t *st_dev[kSlots] = {};
    uint64_t st_dev_cap[kSlots] = {};
    SmallInlineArgs sm_inl{};              // arguments of the last launch; images of <= kSmallInline words inline
    // restart from the persisted tables (lx_load_rows / lx_load_finish)
    bool loading = false;
    std::vector<uint32_t> ld_first, ld_last, ld_count, ld_creator, ld_tail;   // per branch, as loaded
    std::vector<uint32_t> ld_par;          // parents of every loaded event (dense)
    std::vector<uint64_t> ld_poff;
    uint32_t ld_B = 0;                     // branches seen so far (max ID + 1)
    uint8_t *ld_buf = nullptr;             // device staging of a chunk's bytes and offsets
    uint64_t ld_buf_cap = 0;

    // pinned, device-mapped query buffers (per-call ForklessCause, getters)
    uint8_t *qp = nullptr, *qp_dev = nullptr;
    uint64_t qp_cap = 0;
    uint32_t get_tag = 0;                  // completion tag of the last single-row getter
    bool fc_unchecked = false;             // a ForklessCause launch may have flagged status[1] since lx_sync looked
    // the resident single-row server (k_get_server, option get_server)
    // 0 off; 1 auto: only while this handle is the process's only one (the
    // server holds a hardware queue while resident, and GPU_MAX_HW_QUEUES = 4
    // lets more streams share queues: work queued behind the resident kernel
    // would wait up to its 250-us idle exit); 2 on whatever the handle count
    int srv_opt = 1;
    hipStream_t srv_stream = nullptr;      // its own (high-priority) stream
    uint64_t *srv_host = nullptr, *srv_dev = nullptr;   // pinned: [0] request word, [1] exited gen
    bool srv_live = false;                 // launched and not known to have left
    uint32_t srv_gen = 0;
    GetSrvArgs srv_args{};                 // the live server's arguments (ticks, seen0, gen aside)
    uint64_t srv_ticks_us = 0;             // wall clock ticks per microsecond
    uint64_t srv_served = 0, srv_launches = 0, srv_fallbacks = 0;
    uint32_t *q_sink = nullptr;            // status word the pinned FC path lets the kernel flag into
    bool get_host_check = true;            // option getter_host_check=0 (tests): device bound only

    // timing (HIP events on `stream`)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    lx_stats stats{};
    bool stats_lazy = false;               // small path: ms_index from ev[1..2] on demand
    bool small_timing = false;             // option timing=1: time small-path launches (two event records)
    uint32_t cpw_hint = 0;                 // option cpw: walker columns per workgroup (0 = auto)
    bool pack16 = true;                    // option pack16=0: two slot units per event even for small seqs
    bool seg_xmap_opt = false;             // option seg_xmap=1: 12-column walks keep each HB line's slices on one XCD
    bool crec_opt = false;                 // option crec=1: the 8- / 12-column walks stream the 32-B compact records
    bool prof = false;                     // LX_PROF=1 in make WPROF=1 builds: per-wave walker counters
    uint64_t last_npar = 0;                // parents in the current batch
    FcCache *fcc = nullptr;                // per-pair ForklessCause result cache (lx_fccache.cpp)
    uint32_t fcc_slots = 4096;             // option fc_cache: its working set (0 = no cache)
    bool fcc_slots_set = false;            // set by the option (else sized at lx_reset from V)
    // segmented walk (option segments, lx_segment.hip): scratch and timings of the last batch
    uint32_t segments = 0;
    bool fc_early = true;                  // option fc_early=0: k_fc always reads whole rows
    uint32_t fc_early_lanes = 32;          // option fc_early_lanes: k_fc_early's lanes per query (16 or 32)
    unsigned long long *d_clk = nullptr;       // walk clock records (IndexArgs::clk)
    // column-shard early exit (lx_fc_shard_undecided_dev): flags, scan, scan scratch
    uint32_t *fcs_flag = nullptr, *fcs_pos = nullptr;
    void *fcs_tmp = nullptr;
    uint64_t fcs_cap = 0;
    size_t fcs_tmp_bytes = 0;
    unsigned long long *d_fc_full = nullptr;   // early exit counters (device): past round 1, past round 2, all
    bool seg_auto = true;                  // option seg_auto=0: never split a batch on its own
    uint32_t n_cus = 256;                  // compute units of the device (auto segments)
    uint32_t *seg_jt = nullptr, *seg_cnt = nullptr, *seg_mf = nullptr, *seg_plist = nullptr, *seg_elist = nullptr;
    uint64_t seg_jt_cap = 0, seg_cnt_cap = 0, seg_mf_cap = 0, seg_plist_cap = 0, seg_elist_cap = 0;   // seg_mf: flags
    std::vector<hipEvent_t> seg_ev;
    lx_seg_stats seg_stats{};
    // row-segment rank (options seg_rank / seg_count, lx_rowseg.cpp): one batch
    // per epoch, this rank walks and owns the rows of segment rs_rank
    uint32_t rs_rank = 0, rs_count = 0;
    int rs_state = 0;                      // 0 idle, 1 rows needed, 2 rows final, 3 LowestAfter sent, 4 ready
    uint32_t rs_lo = 0, rs_hi = 0, rs_npartial = 0, rs_nreq = 0;
    // the rank's own segment walked as rs_sub side-by-side sub-segments (option
    // seg_sub, 0: auto); rs_seg_lo then holds rs_count x rs_sub segments
    uint32_t rs_sub = 1, rs_sub_opt = 0;
    uint32_t rs_npart[kMaxSegments] = {};   // partial events per own sub-segment
    uint32_t rs_seg_lo[kMaxSegments + 1] = {};
    uint32_t *rs_need = nullptr, *rs_req = nullptr, *rs_ctr = nullptr, *rs_ids = nullptr, *rs_out = nullptr,
             *rs_send = nullptr;
    uint64_t rs_need_cap = 0, rs_req_cap = 0, rs_ids_cap = 0, rs_out_cap = 0, rs_send_cap = 0, rs_ctr_cap = 0;
    uint64_t rs_out_per = 0;               // triples per destination in rs_out
    uint64_t rs_nsend = 0;                 // triples packed in rs_send (lx_rowseg_la)
    // ForklessCause across ranks (lx_rowseg_fc_*): per event the stamp of its LA
    // row (2 gen: asked in batch gen, 2 gen + 1: received), the batch counter,
    // route / sort scratch
    uint32_t *rs_stamp = nullptr;
    uint64_t rs_stamp_cap = 0;
    uint32_t rs_gen = 0;
    uint32_t *rsq_scratch = nullptr, *rsq_list = nullptr, *rsq_ctr = nullptr;
    uint64_t rsq_scratch_cap = 0, rsq_list_cap = 0, rsq_ctr_cap = 0;
    void *rsq_tmp = nullptr;
    size_t rsq_tmp_bytes = 0;
    uint32_t rsq_nlist = 0;                // distinct remote rows of the last lx_rowseg_fc_need
    // the planes of a row-segment rank hold its own rows only (rs_planes):
    // hb / la are virtual bases (own row e at hb + e * pstride, inside the
    // allocations rs_hb_mem / rs_la_mem of rs_mem_rows rows); rows of other
    // ranks it receives go to receive areas: HighestBefore rows for the
    // partial fix-up (rs_rhb, row rs_hslot[x]), LowestAfter rows for one
    // ForklessCause batch (rs_rla, row rs_lslot[x])
    uint32_t *rs_hb_mem = nullptr, *rs_la_mem = nullptr;
    uint64_t rs_mem_rows = 0;
    uint32_t rs_mem_pstride = 0;
    uint32_t *rs_hslot = nullptr, *rs_rhb = nullptr, *rs_lslot = nullptr, *rs_rla = nullptr;
    uint64_t rs_hslot_cap = 0, rs_rhb_cap = 0, rs_lslot_cap = 0, rs_rla_cap = 0;   // (receive areas: rows x pstride)
    bool rowseg() const { return rs_count >= 1; }   // seg_count = 1: one rank, the whole epoch

    int fail(int code, const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    int hip(hipError_t e, const char *what) {
        if (e == hipSuccess) return 0;
        return fail(e == hipErrorOutOfMemory ? LX_ERR_NOMEM : LX_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    }
};

#define HIPCHK(h, expr)                                  \
    do {                                                 \
        int _rc = (h)->hip((expr), #expr);               \
        if (_rc) return _rc;                             \
    } while (0)


// internal entry points shared by lx_capi.cpp and lx_fccache.cpp
int lx_fc_args(lx_index *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out, uint32_t *partial,
               FcArgs *fa);
int flush_pending(lx_index *h);                 // launch the pending small-path run (lx_capi.cpp)
// slots of the FC cache changed since its device mirror was written
struct Add1Delta {
    uint32_t n;
    uint32_t slot[kAdd1Delta], ev[kAdd1Delta];
    uint8_t tag[kAdd1Delta];
};
int flush_add1_row(lx_index *h, uint32_t a, uint32_t *evk_dev, uint32_t n_slots, uint8_t *tag_dev, uint8_t *out_dev,
                   uint32_t *psum_dev, const Add1Delta *delta);   // 1: not applicable
int rs_begin(lx_index *h, IndexArgs ia, const uint32_t *poff, hipStream_t s);   // lx_rowseg.cpp
int rs_planes(lx_index *h, uint32_t n);          // lx_rowseg.cpp: own rows of an n-event epoch
void rs_planes_free(lx_index *h);
uint32_t seg_pick(const lx_index *h, uint64_t n, uint32_t *cpw);    // lx_capi.cpp (auto_segments)
uint32_t seg_walk_grid(const lx_index *h, uint32_t cpw);
void rs_free(lx_index *h);
void srv_stop(lx_index *h);   // lx_capi.cpp: the resident row server leaves
void fcc_destroy(lx_index *h);
void fcc_clear(lx_index *h);                    // Reset: a new epoch
void fcc_forget_from(lx_index *h, uint64_t n);  // DropNotFlushed: events >= n are gone
