// lx_abft.cpp -- batched abft caller (include/lachesis_abft.h).
//
// Same results as abft.IndexedLachesis.Process called once per event
// (abft/indexed_lachesis.go:65-82), reorganised so that the ForklessCause
// questions of the consensus loop become a few large GPU launches:
//
// Frames (calcFrameIdx, abft/event_processing.go:163-189).  frame(e) is the
// first f >= selfParentFrame(e) at which e is NOT forkless-caused by a quorum
// of roots(f) (capped by the claimed frame, or selfParentFrame+100 in Build);
// roots(f) = events with selfParentFrame < f <= frame.  ForklessCause(e, r)
// can only hold for ancestors r of e, so the answer for e depends only on its
// ancestors and the batch can be solved frame by frame: at step f every
// event still undecided has frame >= f, roots(f) is complete, and every event
// whose loop has reached f asks q_f(e) = quorum(roots(f)) -- all of them in
// one k_root_fc tile launch.  Self-children of those events are evaluated
// speculatively in the same launch (their self-parent usually stops at f).
// An event that passes q_f becomes a root of f+1; its bit row of that launch
// is exactly the observed-roots set the election needs for that root slot.
// A batch in which every event claims its frame needs no steps at all: every
// question is known up front (compute_frames_claimed), one launch answers all.
//
// Election (abft/election/election_math.go:13-114).  Votes of a root slot
// depend only on the slots it observes, so votes are computed per frame
// (round) for all slots at once, for every subject (k_vote_round).  The
// reference skips subjects already decided when a root is processed; that
// only skips work whose result is never read.  The decision for subject v is
// the vote of the first deciding root in processing order =
// atomicMin over (event << 32 | vote); the frame is decided at
// t = max(previous decision, max_{v <= Atropos subject} first decision(v))
// (chooseAtropos, sort_roots.go:10-25), final once no uncomputed slot is older
// than t.  Frames are replayed after each decision as processKnownRoots does.
// Elections of different frames do not read each other, so all of them run
// side by side first (run_elections_ahead), round by round only what remains.
//
// Blocks (abft/lachesis.go:40-86): cheaters from the Atropos' HighestBefore
// fork markers, confirmation DFS in the reference's stack order on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/lachesis_abft.h"
#include "lx_internal.h"

namespace {

constexpr uint32_t NONE = LX_NONE;
constexpr uint32_t kSpecDepth = 4;      // self-children evaluated ahead per launch (LX_SPEC overrides)
constexpr uint32_t kBuildCap = 100;     // calcFrameIdx: selfParentFrame + 100 in Build
constexpr uint32_t kVoteWindow = 64;    // subjects voted on first (chooseAtropos walks idx order)
constexpr uint32_t kElectAhead = 2;     // rounds per election in run_elections_ahead (3: 72 vote launches, slower)

// Device buffers recycled within one abft handle.  Every device operation of
// the handle is enqueued on the index's stream, so a buffer handed back here
// can be reused by later work on that stream without a host sync (frame
// arrays and vote tables come and go with every decided frame: allocating
// them with hipMalloc / hipFree cost ~6 ms per 50k-event epoch).
struct BufPool {
    std::multimap<uint64_t, void *> free;
    void put(void *p, uint64_t bytes) {
        if (p) free.emplace(bytes, p);
    }
    void *take(uint64_t bytes, uint64_t *got) {
        auto it = free.lower_bound(bytes);
        if (it == free.end() || it->first > 4 * bytes + 65536) return nullptr;
        void *p = it->second;
        *got = it->first;
        free.erase(it);
        return p;
    }
    void drain() {
        for (auto &kv : free) (void)hipFree(kv.second);
        free.clear();
    }
};

template <typename T>
struct DVec {
    T *p = nullptr;
    uint64_t cap = 0;
    BufPool *pool = nullptr;
    void release() {
        if (p) {
            if (pool) pool->put(p, cap * sizeof(T));
            else (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
};

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// LX_ABFT_TIMING=1: host wall time between the marks of the batched frame and
// election passes, one line per pass on stderr (diagnostics only)
struct PassTimer {
    const char *name;
    bool on;
    double t0, last;
    std::string out;
    explicit PassTimer(const char *n) : name(n), on(getenv("LX_ABFT_TIMING") != nullptr) {
        if (on) t0 = last = now_ms();
    }
    void mark(const char *what) {
        if (!on) return;
        const double t = now_ms();
        char b[64];
        snprintf(b, sizeof b, " %s=%.3f", what, t - last);
        out += b;
        last = t;
    }
    ~PassTimer() {
        if (on) fprintf(stderr, "abft_timing %s total=%.3f%s\n", name, now_ms() - t0, out.c_str());
    }
};

struct Frame {
    std::vector<uint32_t> ev, creator, dup, bm_len;
    std::vector<uint64_t> bm_off;
    std::vector<uint32_t> last_of;   // creator -> last slot index (for dup)
    uint32_t synced = 0;
    uint32_t voted = 0;              // slots with votes for the current election
    DVec<uint32_t> d_ev, d_creator, d_dup, d_bm_len, votes;
    DVec<uint64_t> d_bm_off;
    void release() {
        d_ev.release();
        d_creator.release();
        d_dup.release();
        d_bm_len.release();
        d_bm_off.release();
        votes.release();
    }
};

// The host-to-device uploads of one step (frame metadata, candidates,
// cheater columns) go out together: data and descriptors are gathered on the
// host, copied into a pinned, device-mapped staging slot, and one k_scatter
// launch moves them (a hipMemcpyAsync from pageable memory per array cost
// ~10 us each, ~250 per epoch at C5).
struct Uploader {
    static constexpr int kSlots = 4;
    uint8_t *pin[kSlots] = {};
    uint64_t cap[kSlots] = {};
    hipEvent_t done[kSlots] = {};
    bool used[kSlots] = {};
    int next = 0;
    std::vector<uint8_t> data;
    std::vector<ScatterDesc> desc;
    uint64_t launches = 0;
    void add(void *dst, const void *src, uint64_t bytes) {
        if (!bytes) return;
        const uint64_t off = data.size();
        data.resize(off + (bytes + 15) / 16 * 16);
        memcpy(data.data() + off, src, bytes);
        desc.push_back(ScatterDesc{dst, off, bytes});
    }
    bool pending() const { return !desc.empty(); }
    // a pending upload writes into [p, p + bytes)
    bool targets(const void *p, uint64_t bytes) const {
        const uint8_t *lo = static_cast<const uint8_t *>(p), *hi = lo + bytes;
        for (const ScatterDesc &d : desc) {
            const uint8_t *x = static_cast<const uint8_t *>(d.dst);
            if (x >= lo && x < hi) return true;
        }
        return false;
    }
    void release() {
        for (int k = 0; k < kSlots; k++) {
            if (pin[k]) (void)hipHostFree(pin[k]);
            if (done[k]) (void)hipEventDestroy(done[k]);
            pin[k] = nullptr;
            done[k] = nullptr;
        }
    }
};

}  // namespace

// blocks decided by the last lx_abft_process_batch (option block_log)
struct BlockLog {
    std::vector<uint32_t> frame, atropos, cheaters, cheat_off{0}, confirmed, conf_off{0};
    void clear() {
        frame.clear();
        atropos.clear();
        cheaters.clear();
        confirmed.clear();
        cheat_off.assign(1, 0);
        conf_off.assign(1, 0);
    }
};

struct lx_abft {
    lx_index *ix = nullptr;
    std::string err;
    lx_abft_callbacks cb{};
    bool booted = false;

    uint32_t epoch = 0, V = 0, quorum = 0;
    std::vector<uint32_t> weights;
    uint32_t last_decided = 0;
    uint64_t t_prev = 0;                // event whose processing decided the last frame

    // per event of the epoch (dense index)
    std::vector<uint32_t> ev_frame, ev_sp, ev_confirmed;
    std::vector<uint64_t> par_off{0};
    std::vector<uint32_t> par;

    BufPool pool;                       // recycled device buffers (all DVecs below)
    Uploader up;                        // batched host-to-device uploads of a step
    uint8_t *q_pin = nullptr;           // k_root_quorum answers, pinned and device-mapped
    uint64_t q_pin_cap = 0;
    uint32_t *rb_pin = nullptr;         // k_readback target (decisions + error word, atropos HB row)
    uint64_t rb_cap = 0;
    std::vector<hipEvent_t> fc_ev;      // pairs around k_root_fc launches (stats.ms_root_fc_gpu)
    uint32_t fc_ev_used = 0;
    std::vector<Frame> frames;          // [0] unused
    DVec<uint32_t> arena;               // bit rows (observed roots) of k_root_fc launches
    uint64_t arena_used = 0;

    // scratch
    DVec<uint32_t> d_cand, d_psum;
    DVec<uint8_t> d_q;
    DVec<unsigned long long> d_dec;
    DVec<uint32_t> d_err;
    DVec<uint32_t> d_kcol, d_kflag, d_kw;
    DVec<uint32_t> ea_votes, ea_err;      // elections decided ahead: vote tables, error words
    DVec<unsigned long long> ea_dec;      // ... decision words per election x subject
    DVec<VoteArgs> ea_args;               // ... launch args, grouped by round
    DVec<RootFcArgs> d_fcargs;            // merged frame steps of a claimed batch: per-step args
    DVec<QuorumArgs> d_qargs;
    uint32_t n_k = 0;
    uint32_t k_B = NONE;                // branch count the cheater columns were built for
    std::vector<uint32_t> h_row;
    bool dec_dirty = true;
    uint32_t vw = 0;                    // subject window [0, vw) of the current election
    uint32_t spec_depth = kSpecDepth;
    bool fc16 = true;                   // option fc16=0: k_root_fc (32-bit) even for 16-bit seqs
    bool claimed_batch = true;          // option claimed_batch=0: claimed batches take the Build path's steps
    uint32_t elect_ahead = kElectAhead;  // option elect_ahead: rounds per election decided ahead (0 = off)
    uint32_t block_log = 0;             // option block_log: without callbacks, log blocks (2: with confirmed events)
    BlockLog blog;
    std::vector<uint32_t> sweep_atropos, sweep_frame, sweep_label;   // confirmations queued for confirm_sweep

    lx_abft_stats stats{};

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
    int ixfail(int rc) {
        err = lx_last_error(ix);
        return rc;
    }
};

#define AHIP(a, expr)                               \
    do {                                            \
        int _rc = (a)->hip((expr), #expr);          \
        if (_rc) return _rc;                        \
    } while (0)
#define ARC(expr)                                   \
    do {                                            \
        int _rc = (expr);                           \
        if (_rc) return _rc;                        \
    } while (0)

namespace {

int flush_uploads(lx_abft *a, hipStream_t s);

template <typename T>
int reserve(lx_abft *a, DVec<T> &v, uint64_t n, uint64_t keep, hipStream_t s) {
    if (n <= v.cap) return 0;
    if (v.p && a->up.targets(v.p, v.cap * sizeof(T))) ARC(flush_uploads(a, s));   // the buffer is about to move
    uint64_t cap = std::max<uint64_t>({n, v.cap + v.cap / 2, 256});
    uint64_t got = 0;
    T *p = static_cast<T *>(a->pool.take(cap * sizeof(T), &got));
    if (p) cap = got / sizeof(T);
    else AHIP(a, hipMalloc((void **)&p, cap * sizeof(T)));
    if (v.p && keep) AHIP(a, hipMemcpyAsync(p, v.p, keep * sizeof(T), hipMemcpyDeviceToDevice, s));
    v.pool = &a->pool;
    v.release();          // stream-ordered reuse: no sync
    v.p = p;
    v.cap = cap;
    return 0;
}

template <typename T>
int upload(lx_abft *a, DVec<T> &v, const std::vector<T> &h, uint64_t from, hipStream_t s) {
    ARC(reserve(a, v, h.size(), from, s));
    if (h.size() > from) a->up.add(v.p + from, h.data() + from, (h.size() - from) * sizeof(T));
    return 0;
}

// the step's uploads in one k_scatter launch (stream-ordered before the
// kernels that read them)
int flush_uploads(lx_abft *a, hipStream_t s) {
    Uploader &u = a->up;
    if (!u.pending()) return 0;
    const int k = u.next;
    u.next = (u.next + 1) % Uploader::kSlots;
    if (!u.done[k]) AHIP(a, hipEventCreateWithFlags(&u.done[k], hipEventDisableTiming));
    if (u.used[k]) AHIP(a, hipEventSynchronize(u.done[k]));
    const uint64_t dbytes = u.desc.size() * sizeof(ScatterDesc);
    const uint64_t need = dbytes + u.data.size();
    if (need > u.cap[k]) {
        if (u.pin[k]) (void)hipHostFree(u.pin[k]);
        u.pin[k] = nullptr;
        u.cap[k] = 0;
        const uint64_t cap = std::max<uint64_t>(need * 2, 1u << 16);
        AHIP(a, hipHostMalloc((void **)&u.pin[k], cap, hipHostMallocMapped));
        u.cap[k] = cap;
    }
    uint64_t max_bytes = 0;
    for (auto &d : u.desc) {
        d.src_off += dbytes;
        max_bytes = std::max<uint64_t>(max_bytes, d.bytes);
    }
    memcpy(u.pin[k], u.desc.data(), dbytes);
    memcpy(u.pin[k] + dbytes, u.data.data(), u.data.size());
    void *dp = nullptr;
    AHIP(a, hipHostGetDevicePointer(&dp, u.pin[k], 0));
    const uint8_t *base = static_cast<const uint8_t *>(dp);
    AHIP(a, lx::launch_scatter(reinterpret_cast<const ScatterDesc *>(base), (uint32_t)u.desc.size(), max_bytes, base,
                               s));
    AHIP(a, hipEventRecord(u.done[k], s));
    u.used[k] = true;
    u.launches++;
    u.desc.clear();
    u.data.clear();
    return 0;
}

// words [0, na) of a and [0, nb) of b (device) into a->rb_pin, then wait for
// the stream: the host reads them at the returned pointer
int readback(lx_abft *a, hipStream_t s, const uint32_t *x, uint32_t na, const uint32_t *y, uint32_t nb,
             const uint32_t **out) {
    const uint64_t need = (uint64_t)na + nb;
    if (need > a->rb_cap) {
        if (a->rb_pin) {
            AHIP(a, hipStreamSynchronize(s));
            (void)hipHostFree(a->rb_pin);
        }
        a->rb_pin = nullptr;
        a->rb_cap = 0;
        const uint64_t cap = std::max<uint64_t>(need * 2, 4096);
        AHIP(a, hipHostMalloc((void **)&a->rb_pin, cap * 4, hipHostMallocMapped));
        a->rb_cap = cap;
    }
    void *dp = nullptr;
    AHIP(a, hipHostGetDevicePointer(&dp, a->rb_pin, 0));
    AHIP(a, lx::launch_readback(static_cast<uint32_t *>(dp), x, na, y, nb, s));
    AHIP(a, hipStreamSynchronize(s));
    *out = a->rb_pin;
    return 0;
}

// HB rows of events rows[k] into a->rb_pin (k * V), then wait for the stream
int readback_rows(lx_abft *a, const IndexView &iv, const std::vector<uint32_t> &rows, const uint32_t **out) {
    const uint64_t need = (uint64_t)rows.size() * a->V;
    if (need > a->rb_cap) {
        if (a->rb_pin) {
            AHIP(a, hipStreamSynchronize(iv.stream));
            (void)hipHostFree(a->rb_pin);
        }
        a->rb_pin = nullptr;
        a->rb_cap = 0;
        const uint64_t cap = std::max<uint64_t>(need * 2, 4096);
        AHIP(a, hipHostMalloc((void **)&a->rb_pin, cap * 4, hipHostMallocMapped));
        a->rb_cap = cap;
    }
    void *dp = nullptr;
    AHIP(a, hipHostGetDevicePointer(&dp, a->rb_pin, 0));
    AHIP(a, lx::launch_gather_rows(static_cast<uint32_t *>(dp), iv.hb, iv.stride, a->V, rows.data(),
                                   (uint32_t)rows.size(), iv.stream));
    AHIP(a, hipStreamSynchronize(iv.stream));
    *out = a->rb_pin;
    return 0;
}

Frame &frame_at(lx_abft *a, uint32_t f) {
    if (a->frames.size() <= f) a->frames.resize(f + 1);
    return a->frames[f];
}

void add_slot(lx_abft *a, uint32_t f, uint32_t e, uint32_t creator, uint64_t bm_off, uint32_t bm_len) {
    Frame &fr = frame_at(a, f);
    if (fr.last_of.empty()) fr.last_of.assign(a->V, NONE);
    uint32_t k = (uint32_t)fr.ev.size();
    fr.ev.push_back(e);
    fr.creator.push_back(creator);
    fr.dup.push_back(fr.last_of[creator]);
    fr.last_of[creator] = k;
    fr.bm_off.push_back(bm_off);
    fr.bm_len.push_back(bm_len);
}

int sync_frame(lx_abft *a, Frame &fr, hipStream_t s) {
    uint32_t from = fr.synced;
    if (from == fr.ev.size()) return 0;
    ARC(upload(a, fr.d_ev, fr.ev, from, s));
    ARC(upload(a, fr.d_creator, fr.creator, from, s));
    ARC(upload(a, fr.d_dup, fr.dup, from, s));
    ARC(upload(a, fr.d_bm_len, fr.bm_len, from, s));
    ARC(upload(a, fr.d_bm_off, fr.bm_off, from, s));
    fr.synced = (uint32_t)fr.ev.size();
    return 0;
}

void clear_epoch(lx_abft *a) {
    for (Frame &f : a->frames) f.release();
    a->frames.clear();
    a->ev_frame.clear();
    a->ev_sp.clear();
    a->ev_confirmed.clear();
    a->sweep_atropos.clear();
    a->sweep_frame.clear();
    a->par_off.assign(1, 0);
    a->par.clear();
    a->arena_used = 0;
    a->last_decided = 0;
    a->t_prev = 0;
    a->dec_dirty = true;
    a->k_B = NONE;
}

int start_epoch(lx_abft *a, uint32_t epoch, uint32_t nv, const uint32_t *w) {
    if (!nv || !w) return a->fail(LX_ERR_ARG, "genesis validators shouldn't be empty");
    int rc = lx_reset(a->ix, nv, w);
    if (rc) return a->ixfail(rc);
    IndexView iv;
    if ((rc = lx_index_view(a->ix, &iv))) return a->ixfail(rc);
    if (iv.shard_count > 1) return a->fail(LX_ERR_STATE, "abft needs an unsharded index");
    clear_epoch(a);
    a->epoch = epoch;
    a->V = nv;
    a->weights.assign(w, w + nv);
    a->quorum = iv.quorum;
    return 0;
}

// Cheaters' branch columns, grouped by creator, original first (k_root_fc).
int refresh_cheaters(lx_abft *a, const IndexView &iv) {
    if (a->k_B == iv.B) return 0;
    std::vector<uint32_t> col, flag, kw;
    for (uint32_t c = 0; c < iv.V; c++) {
        const auto &l = (*iv.by_creator)[c];
        if (l.size() < 2) continue;
        for (size_t i = 0; i < l.size(); i++) {
            col.push_back(l[i]);
            flag.push_back((i == 0 ? 1u : 0u) | (i + 1 == l.size() ? 2u : 0u));
            kw.push_back(i + 1 == l.size() ? (*iv.weights)[c] : 0u);
        }
    }
    a->n_k = (uint32_t)col.size();
    if (a->n_k) {
        ARC(upload(a, a->d_kcol, col, 0, iv.stream));
        ARC(upload(a, a->d_kflag, flag, 0, iv.stream));
        ARC(upload(a, a->d_kw, kw, 0, iv.stream));
    }
    a->k_B = iv.B;
    return 0;
}

// VALU lane-ops per (event, root) pair of the root-FC inner loops (ISA count):
// 2.5 per column in k_root_fc, 1.5 in k_root_fc16 (2 in its 32-column chunks
// holding a weight >= 2^16), over the padded columns
uint64_t fc_ops_per_pair(const lx_abft *a, const IndexView &iv, bool forks, bool seq16, uint32_t ncols) {
    if (forks || !seq16) return 5 * (uint64_t)ncols / 2;
    uint64_t hi_cols = 0;
    for (uint32_t c = 0; c < iv.V; c += 32)
        for (uint32_t j = c; j < std::min(c + 32, iv.V); j++)
            if (a->weights[j] >> 16) {
                hi_cols += 32;
                break;
            }
    return (3 * (uint64_t)ncols + hi_cols) / 2;
}

// One frame step enqueued: bits (cands x roots(f)) into the arena at *row0,
// q per candidate into q_dev (device-mapped pinned memory); nothing waits.
// *launched = false when frame f has no roots (no quorum: the caller's q is 0).
int launch_eval(lx_abft *a, const IndexView &iv, uint32_t f, const uint32_t *cand, uint32_t n, uint8_t *q_dev,
                uint64_t *row0, uint32_t *words_out, bool *launched) {
    hipStream_t s = iv.stream;
    Frame &fr = frame_at(a, f);
    ARC(sync_frame(a, fr, s));
    const uint32_t R = (uint32_t)fr.ev.size();
    const uint32_t words = (R + 31) / 32;
    *row0 = a->arena_used;
    *words_out = words;
    *launched = false;
    ARC(reserve(a, a->arena, a->arena_used + (uint64_t)n * words + 1, a->arena_used, s));
    a->arena_used += (uint64_t)n * words;
    if (!words) return 0;
    ARC(reserve(a, a->d_cand, n, 0, s));
    uint32_t *bits = a->arena.p + *row0;
    // queued only when this step launches (flush_uploads below): a frame
    // without roots must not leave a pending descriptor for d_cand that a
    // later step's upload of the same range could race with
    a->up.add(a->d_cand.p, cand, n * 4ull);
    ARC(refresh_cheaters(a, iv));
    // split the columns when the tiles alone cannot fill the chip
    const uint32_t ncols = (iv.V + 31) / 32 * 32;
    const uint32_t splits = lx::root_fc_splits(n, R, ncols);
    const uint32_t col_split = ((ncols + splits - 1) / splits + 31) / 32 * 32;
    const uint32_t n_split = (ncols + col_split - 1) / col_split;
    ARC(reserve(a, a->d_psum, (uint64_t)n_split * n * words * 32, 0, s));
    RootFcArgs r{};
    r.hb = iv.hb;
    r.la = iv.la;
    r.stride = iv.stride;
    r.cand = a->d_cand.p;
    r.n_cand = n;
    r.roots = fr.d_ev.p;
    r.n_roots = R;
    r.roots_fallback = cand[0];
    r.ncols = ncols;
    r.wpad = iv.wpad;
    r.quorum = a->quorum;
    r.n_k = a->n_k;
    r.kcol = a->d_kcol.p;
    r.kflag = a->d_kflag.p;
    r.kw = a->d_kw.p;
    r.ev_branch = iv.ev_branch;
    r.psum = a->d_psum.p;
    r.words = words;
    r.col_split = col_split;
    r.n_split = n_split;
    ARC(flush_uploads(a, s));
    const uint32_t k = a->fc_ev_used;
    while (a->fc_ev.size() < 2ull * (k + 1)) {
        hipEvent_t e;
        AHIP(a, hipEventCreate(&e));
        a->fc_ev.push_back(e);
    }
    const bool forks = iv.B > iv.V, seq16 = a->fc16 && iv.max_seq <= 0xFFFFu;
    AHIP(a, hipEventRecord(a->fc_ev[2 * k], s));
    AHIP(a, lx::launch_root_fc(r, forks, seq16, s));
    AHIP(a, hipEventRecord(a->fc_ev[2 * k + 1], s));
    a->fc_ev_used = k + 1;
    QuorumArgs qa{};
    qa.psum = a->d_psum.p;
    qa.n_split = n_split;
    qa.bits = bits;
    qa.words = words;
    qa.n_roots = R;
    qa.n_cand = n;
    qa.cand = a->d_cand.p;
    qa.root_ev = fr.d_ev.p;
    qa.creator = fr.d_creator.p;
    qa.dup = fr.d_dup.p;
    qa.wcreator = iv.wpad;
    qa.quorum = a->quorum;
    qa.q = q_dev;   // answers land in pinned host memory
    AHIP(a, lx::launch_root_quorum(qa, s));
    a->stats.fc_launches++;
    a->stats.fc_pairs += (uint64_t)n * R;
    a->stats.fc_pair_cols += (uint64_t)n * R * iv.V;
    a->stats.fc_lane_ops += (uint64_t)n * R * fc_ops_per_pair(a, iv, forks, seq16, ncols);
    *launched = true;
    return 0;
}

// after the stream has drained: k_root_fc times of the launches since the last call
int collect_fc_times(lx_abft *a) {
    for (uint32_t k = 0; k < a->fc_ev_used; k++) {
        float ms = 0;
        AHIP(a, hipEventElapsedTime(&ms, a->fc_ev[2 * k], a->fc_ev[2 * k + 1]));
        a->stats.ms_root_fc_gpu += ms;
    }
    a->fc_ev_used = 0;
    return 0;
}

// pinned, device-mapped q answers for n candidates (contents not kept)
int q_buffer(lx_abft *a, uint64_t n, hipStream_t s, uint8_t **q_dev) {
    if (n > a->q_pin_cap) {
        if (a->q_pin) {
            AHIP(a, hipStreamSynchronize(s));
            (void)hipHostFree(a->q_pin);
        }
        a->q_pin = nullptr;
        a->q_pin_cap = 0;
        const uint64_t cap = std::max<uint64_t>(n, 4096);
        AHIP(a, hipHostMalloc((void **)&a->q_pin, cap, hipHostMallocMapped));
        a->q_pin_cap = cap;
    }
    void *q_dev_v = nullptr;
    AHIP(a, hipHostGetDevicePointer(&q_dev_v, a->q_pin, 0));
    *q_dev = static_cast<uint8_t *>(q_dev_v);
    return 0;
}

// One frame step, answered: bits (cands x roots(f)) into the arena, q per candidate.
int eval_frame(lx_abft *a, const IndexView &iv, uint32_t f, const std::vector<uint32_t> &cand, uint64_t *row0,
               uint32_t *words_out, std::vector<uint8_t> &q) {
    const uint32_t n = (uint32_t)cand.size();
    uint8_t *q_dev = nullptr;
    ARC(q_buffer(a, n, iv.stream, &q_dev));
    bool launched;
    ARC(launch_eval(a, iv, f, cand.data(), n, q_dev, row0, words_out, &launched));
    if (!launched) {
        q.assign(n, 0);   // no roots in frame f: no quorum (WeightCounter of nothing)
        return 0;
    }
    AHIP(a, hipStreamSynchronize(iv.stream));
    q.assign(a->q_pin, a->q_pin + n);
    return collect_fc_times(a);
}

// Frames of a batch in which every event claims its frame (Process,
// event_processing.go:163-189 with the claimed frame as the loop bound).
// Taking the claims of in-batch self-parents as given, every question is
// known up front: event i asks q_f(i) for f in [selfParentFrame(i), claim(i)),
// and roots(f) = the roots of f so far plus the batch events claiming f or
// more above a self-parent frame below f (Store.AddRoot adds a root to every
// frame it passes, store_roots.go:23-27), in event order (the order
// per-event Process adds them).  ForklessCause(i, r) is false for every r that is not an ancestor of
// i, so roots later in event order change none of i's answers.  All frame
// steps are enqueued back to back and answered after one wait.  Up to the
// first event whose computed frame differs from its claim, every claim used
// was verified, so the answers are exact there; process() redoes that prefix
// alone (nothing after it is reported).  A claim above every root frame so far
// + 1 cannot verify (frame top+1 has no roots): the batch is cut there.
int compute_frames_claimed(lx_abft *a, uint64_t base, uint32_t n, const uint32_t *creator, const uint32_t *claimed) {
    PassTimer pt("frames");
    IndexView iv;
    int rc = lx_index_view(a->ix, &iv);
    if (rc) return a->ixfail(rc);
    pt.mark("view");
    hipStream_t s = iv.stream;
    uint32_t top = 0;   // highest frame with a root
    for (uint32_t f = 1; f < a->frames.size(); f++)
        if (!a->frames[f].ev.empty()) top = f;
    std::vector<uint32_t> spf(n, 0), rf(n, NONE);
    uint32_t cut = n, fmin = NONE, fmax = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t sp = a->ev_sp[base + i];
        if (sp == NONE) {   // f = 0: roots(0) is empty -> frame 1 (:184-187)
            rf[i] = 1;
            top = std::max(top, 1u);
            continue;
        }
        spf[i] = sp < base ? a->ev_frame[sp] : claimed[sp - base];
        const uint32_t c = claimed[i];
        if (spf[i] == 0 || c > top + 1) {
            cut = i;
            break;
        }
        if (c > spf[i]) {
            rf[i] = c;
            top = std::max(top, c);
            fmin = std::min(fmin, spf[i]);
            fmax = std::max(fmax, c - 1);
        }
    }
    pt.mark("scan");
    // candidates per frame step (event order) and each event's q slots
    const uint32_t nf = fmin == NONE ? 0 : fmax - fmin + 1;
    std::vector<std::vector<uint32_t>> cand(nf);
    std::vector<std::vector<uint32_t>> new_roots(top + 2);
    std::vector<uint64_t> qoff(nf + 1, 0), row0(nf, 0);
    std::vector<uint32_t> words(nf, 0), pos0(n, 0);
    {
        // list sizes first: one allocation per list
        std::vector<uint32_t> nc(nf, 0), nr(top + 2, 0);
        for (uint32_t i = 0; i < cut; i++) {
            if (a->ev_sp[base + i] == NONE) {
                nr[1]++;
                continue;
            }
            if (rf[i] == NONE) continue;
            for (uint32_t f = spf[i]; f < rf[i]; f++) {
                nc[f - fmin]++;
                nr[f + 1]++;
            }
        }
        for (uint32_t k = 0; k < nf; k++) cand[k].reserve(nc[k]);
        for (uint32_t f = 0; f < top + 2; f++) new_roots[f].reserve(nr[f]);
    }
    for (uint32_t i = 0; i < cut; i++) {
        if (a->ev_sp[base + i] == NONE) {
            new_roots[1].push_back(i);
            continue;
        }
        if (rf[i] == NONE) continue;
        // a root of every frame it passes: spf+1 .. claim (Store.AddRoot, store_roots.go:23-27)
        for (uint32_t f = spf[i] + 1; f <= rf[i]; f++) new_roots[f].push_back(i);
        pos0[i] = (uint32_t)cand[spf[i] - fmin].size();   // position in its first step
        for (uint32_t f = spf[i]; f < claimed[i]; f++) cand[f - fmin].push_back((uint32_t)(base + i));
    }
    for (uint32_t k = 0; k < nf; k++) qoff[k + 1] = qoff[k] + cand[k].size();
    uint8_t *q_dev = nullptr;
    ARC(q_buffer(a, std::max<uint64_t>(qoff[nf], 1), s, &q_dev));
    std::vector<uint8_t> launched(nf, 0);
    // a root's position in the step at f (binary search: cand lists are sorted)
    auto pos_in = [&](uint32_t f, uint32_t i) {
        const auto &c = cand[f - fmin];
        return (uint32_t)(std::lower_bound(c.begin(), c.end(), (uint32_t)(base + i)) - c.begin());
    };
    pt.mark("cands");
    // layout: step k (frame fmin + k) asks cand[k] against every root of its
    // frame (the ones so far + this batch's), bit rows at row0[k] in the arena
    const uint64_t arena0 = a->arena_used;
    std::vector<uint32_t> nroots(nf, 0);
    for (uint32_t k = 0; k < nf; k++) {
        const uint32_t f = fmin + k;
        nroots[k] = (uint32_t)(frame_at(a, f).ev.size() + (f < new_roots.size() ? new_roots[f].size() : 0));
        words[k] = (nroots[k] + 31) / 32;
        row0[k] = a->arena_used;
        a->arena_used += (uint64_t)cand[k].size() * words[k];
        launched[k] = !cand[k].empty() && words[k];
    }
    pt.mark("layout");
    // the roots, frame by frame in event order: a root of f observes the step at
    // f - 1 (its position there and the roots of f - 1 before it by merge walks:
    // every list is in event order)
    for (uint32_t f = 1; f < new_roots.size(); f++) {
        if (new_roots[f].empty()) continue;
        Frame &fr = frame_at(a, f);
        const size_t want = fr.ev.size() + new_roots[f].size();
        fr.ev.reserve(want);
        fr.creator.reserve(want);
        fr.dup.reserve(want);
        fr.bm_off.reserve(want);
        fr.bm_len.reserve(want);
        if (f == 1) {
            for (uint32_t i : new_roots[1]) add_slot(a, 1, (uint32_t)(base + i), creator[i], 0, 0);
            continue;
        }
        const uint32_t k = f - 1 - fmin;
        const auto &nr = new_roots[f - 1];
        const auto &cl = cand[k];
        const uint32_t old_roots = (uint32_t)(frame_at(a, f - 1).ev.size() - nr.size());
        size_t pc = 0, pb = 0;
        for (uint32_t i : new_roots[f]) {
            const uint32_t e = (uint32_t)(base + i);
            while (pc < cl.size() && cl[pc] < e) pc++;
            while (pb < nr.size() && nr[pb] < i) pb++;
            add_slot(a, f, e, creator[i], row0[k] + (uint64_t)pc * words[k], old_roots + (uint32_t)pb);
        }
    }
    pt.mark("slots");
    // every step in one k_root_fc and one k_root_quorum launch
    ARC(reserve(a, a->arena, a->arena_used + 1, arena0, s));
    uint64_t ncand = 0, tiles = 0;
    std::vector<uint32_t> act;
    for (uint32_t k = 0; k < nf; k++)
        if (launched[k]) {
            ARC(sync_frame(a, frame_at(a, fmin + k), s));
            act.push_back(k);
            ncand += cand[k].size();
            tiles += (uint64_t)((nroots[k] + 63) / 64) * ((cand[k].size() + 63) / 64);
        }
    if (!act.empty()) {
        const uint32_t ncols = (iv.V + 31) / 32 * 32;
        const uint32_t max_s = ncols / 128 ? ncols / 128 : 1;   // >= 4 LDS chunks of 32 columns per split
        const uint32_t splits = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((1024 + tiles - 1) / tiles, 1), max_s);
        const uint32_t col_split = ((ncols + splits - 1) / splits + 31) / 32 * 32;
        const uint32_t n_split = (ncols + col_split - 1) / col_split;
        uint64_t npsum = 0;
        for (uint32_t k : act) npsum += (uint64_t)n_split * cand[k].size() * words[k] * 32;
        ARC(reserve(a, a->d_cand, ncand, 0, s));
        ARC(reserve(a, a->d_psum, npsum, 0, s));
        ARC(reserve(a, a->d_fcargs, act.size(), 0, s));
        ARC(reserve(a, a->d_qargs, act.size(), 0, s));
        ARC(refresh_cheaters(a, iv));
        std::vector<RootFcArgs> fa(act.size());
        std::vector<QuorumArgs> qa(act.size());
        uint64_t coff = 0, poff = 0, pairs = 0;
        uint32_t blocks = 0, qblocks = 0;
        for (size_t j = 0; j < act.size(); j++) {
            const uint32_t k = act[j], n_k = (uint32_t)cand[k].size();
            Frame &fr = a->frames[fmin + k];
            a->up.add(a->d_cand.p + coff, cand[k].data(), n_k * 4ull);
            RootFcArgs &r = fa[j];
            r.hb = iv.hb;
            r.la = iv.la;
            r.stride = iv.stride;
            r.cand = a->d_cand.p + coff;
            r.n_cand = n_k;
            r.roots = fr.d_ev.p;
            r.n_roots = nroots[k];
            r.roots_fallback = cand[k][0];
            r.ncols = ncols;
            r.wpad = iv.wpad;
            r.quorum = a->quorum;
            r.n_k = a->n_k;
            r.kcol = a->d_kcol.p;
            r.kflag = a->d_kflag.p;
            r.kw = a->d_kw.p;
            r.ev_branch = iv.ev_branch;
            r.psum = a->d_psum.p + poff;
            r.words = words[k];
            r.col_split = col_split;
            r.n_split = n_split;
            r.block0 = blocks;
            blocks += lx::root_fc_blocks(r);
            QuorumArgs &q = qa[j];
            q.psum = r.psum;
            q.n_split = n_split;
            q.bits = a->arena.p + row0[k];
            q.words = words[k];
            q.n_roots = nroots[k];
            q.n_cand = n_k;
            q.cand = r.cand;
            q.root_ev = fr.d_ev.p;
            q.creator = fr.d_creator.p;
            q.dup = fr.d_dup.p;
            q.wcreator = iv.wpad;
            q.quorum = a->quorum;
            q.q = q_dev + qoff[k];
            q.block0 = qblocks;
            qblocks += (n_k + 3) / 4;
            coff += n_k;
            poff += (uint64_t)n_split * n_k * words[k] * 32;
            pairs += (uint64_t)n_k * nroots[k];
        }
        a->stats.fc_pairs += pairs;
        a->stats.fc_pair_cols += pairs * iv.V;
        a->up.add(a->d_fcargs.p, fa.data(), fa.size() * sizeof(RootFcArgs));
        a->up.add(a->d_qargs.p, qa.data(), qa.size() * sizeof(QuorumArgs));
        pt.mark("args");
        ARC(flush_uploads(a, s));
        pt.mark("upload");
        const bool forks = iv.B > iv.V, seq16 = a->fc16 && iv.max_seq <= 0xFFFFu;
        const uint32_t k = a->fc_ev_used;
        while (a->fc_ev.size() < 2ull * (k + 1)) {
            hipEvent_t e;
            AHIP(a, hipEventCreate(&e));
            a->fc_ev.push_back(e);
        }
        AHIP(a, hipEventRecord(a->fc_ev[2 * k], s));
        AHIP(a, lx::launch_root_fc_multi(a->d_fcargs.p, (uint32_t)act.size(), blocks, forks, seq16, s));
        AHIP(a, hipEventRecord(a->fc_ev[2 * k + 1], s));
        a->fc_ev_used = k + 1;
        AHIP(a, lx::launch_root_quorum_multi(a->d_qargs.p, (uint32_t)act.size(), qblocks, s));
        a->stats.fc_launches++;
        a->stats.fc_lane_ops += pairs * fc_ops_per_pair(a, iv, forks, seq16, ncols);
    }
    pt.mark("launch");
    AHIP(a, hipStreamSynchronize(s));
    pt.mark("wait");
    ARC(collect_fc_times(a));
    a->stats.frame_steps += (uint32_t)act.size();
    for (uint32_t i = 0; i < n; i++) {
        if (i >= cut) {
            a->ev_frame[base + i] = NONE;   // never equals a claim: process() stops here
            continue;
        }
        if (a->ev_sp[base + i] == NONE) {
            a->ev_frame[base + i] = 1;
            continue;
        }
        uint32_t f = spf[i];
        for (uint32_t p = pos0[i]; f < claimed[i]; f++) {
            const uint32_t k = f - fmin;
            if (!launched[k] || !a->q_pin[qoff[k] + (f == spf[i] ? p : pos_in(f, i))]) break;
        }
        a->ev_frame[base + i] = f;
    }
    return 0;
}

// Frames of events [base, base+n) (all already added to the index).
// cap[i]: claimed frame (Process) or NONE = Build's selfParentFrame + 100.
int compute_frames(lx_abft *a, uint64_t base, uint32_t n, const uint32_t *creator, const uint32_t *claimed) {
    if (claimed && a->claimed_batch &&
        std::none_of(claimed, claimed + n, [](uint32_t c) { return c == LX_FRAME_BUILD; }))
        return compute_frames_claimed(a, base, n, creator, claimed);
    IndexView iv;
    int rc = lx_index_view(a->ix, &iv);
    if (rc) return a->ixfail(rc);
    std::vector<uint32_t> cur(n, NONE), cap(n, NONE), child_head(n, NONE), child_next(n, NONE);
    std::map<uint32_t, std::vector<uint32_t>> pending;   // frame -> batch positions whose loop is at it
    for (uint32_t i = 0; i < n; i++) {
        uint32_t sp = a->ev_sp[base + i];
        if (sp != NONE && sp >= base) {
            uint32_t p = (uint32_t)(sp - base);
            child_next[i] = child_head[p];
            child_head[p] = i;
        }
    }
    auto cap_of = [&](uint32_t i, uint32_t sp_frame) {
        uint32_t c = claimed ? claimed[i] : LX_FRAME_BUILD;
        return c == LX_FRAME_BUILD ? sp_frame + kBuildCap : c;
    };
    // resolve(i, f): frame(i) = f; self-children start their loop at f.  A
    // child evaluated speculatively in the same launch is handled by the walk
    // below; the others are queued at f by flush().
    std::vector<std::pair<uint32_t, uint32_t>> pushed;
    auto resolve = [&](uint32_t i, uint32_t f) {
        a->ev_frame[base + i] = f;
        for (uint32_t c = child_head[i]; c != NONE; c = child_next[c]) {
            cur[c] = f;
            cap[c] = cap_of(c, f);
            pushed.emplace_back(c, f);
        }
    };
    auto flush = [&]() {
        for (auto &pc : pushed)
            if (a->ev_frame[base + pc.first] == 0 && cur[pc.first] == pc.second) pending[pc.second].push_back(pc.first);
        pushed.clear();
    };
    for (uint32_t i = 0; i < n; i++) {
        uint32_t sp = a->ev_sp[base + i];
        if (sp == NONE) {
            // f = 0: roots(0) is empty, no quorum -> f stays 0 -> frame 1 (:184-187)
            resolve(i, 1);
            add_slot(a, 1, (uint32_t)(base + i), creator[i], 0, 0);
        } else if (sp < base) {
            cur[i] = a->ev_frame[sp];
            cap[i] = cap_of(i, cur[i]);
            pending[cur[i]].push_back(i);
        }
    }
    flush();

    std::vector<uint8_t> spec(n, 0), q;
    std::vector<uint32_t> cand_pos, cand_ev;
    while (!pending.empty()) {
        const uint32_t f = pending.begin()->first;
        std::vector<uint32_t> Q = std::move(pending.begin()->second);
        pending.erase(pending.begin());
        // Events whose loop bound is f stop without asking (:184: the bound is
        // checked before the quorum) -- with claimed frames that is every
        // non-root event -- and their self-children start at f: drain them
        // all before launching.
        std::vector<uint32_t> ask, work = std::move(Q);
        while (!work.empty()) {
            const uint32_t i = work.back();
            work.pop_back();
            if (f < cap[i]) {
                ask.push_back(i);
                continue;
            }
            resolve(i, f);
            for (auto &pc : pushed) work.push_back(pc.first);
            pushed.clear();
        }
        if (ask.empty()) continue;
        std::sort(ask.begin(), ask.end());
        // speculative self-descendants, spec_depth deep
        cand_pos = ask;
        for (uint32_t i : ask) spec[i] = 2;
        {
            std::vector<uint32_t> lvl = ask, nxt;
            for (uint32_t d = 0; d < a->spec_depth && !lvl.empty() && n > 1; d++) {
                nxt.clear();
                for (uint32_t i : lvl)
                    for (uint32_t c = child_head[i]; c != NONE; c = child_next[c])
                        // a claimed frame above f says i passes q_f: its
                        // children cannot be at f, nothing to speculate
                        if (!spec[c] && cur[c] == NONE && (!claimed || claimed[i] == LX_FRAME_BUILD ||
                                                           claimed[i] <= f)) {
                            spec[c] = 1;
                            nxt.push_back(c);
                            cand_pos.push_back(c);
                        }
                lvl.swap(nxt);
            }
        }
        std::sort(cand_pos.begin(), cand_pos.end());
        cand_ev.resize(cand_pos.size());
        for (size_t k = 0; k < cand_pos.size(); k++) cand_ev[k] = (uint32_t)(base + cand_pos[k]);
        uint64_t row0;
        uint32_t words;
        ARC(eval_frame(a, iv, f, cand_ev, &row0, &words, q));
        for (size_t k = 0; k < cand_pos.size(); k++) {
            const uint32_t i = cand_pos[k];
            const bool own = spec[i] == 2;
            spec[i] = 0;
            // a speculative event counts only if its self-parent stopped at f
            // during this walk (then i's loop is at f too)
            if (!own && (cur[i] != f || a->ev_frame[base + i] != 0)) continue;
            if (f >= cap[i]) {
                resolve(i, f);
            } else if (q[k]) {
                cur[i] = f + 1;                      // root of f+1; its bit row observes roots(f)
                add_slot(a, f + 1, cand_ev[k], creator[i], row0 + k * (uint64_t)words, (uint32_t)frame_at(a, f).ev.size());
                pending[f + 1].push_back(i);
            } else {
                resolve(i, f);
            }
        }
        flush();
        a->stats.frame_steps++;
    }
    return 0;
}

// ---------------------------------------------------------------------------- election

// votes of slots [from, to) of frame g for subjects [v_lo, v_hi) (round g - F)
int vote_slots(lx_abft *a, const IndexView &iv, uint32_t F, uint32_t g, uint32_t from, uint32_t to, uint32_t v_lo,
               uint32_t v_hi) {
    hipStream_t s = iv.stream;
    if (from >= to || v_lo >= v_hi) return 0;
    Frame &fg = frame_at(a, g);
    Frame &fp = frame_at(a, g - 1);
    ARC(sync_frame(a, fg, s));
    ARC(sync_frame(a, fp, s));
    ARC(reserve(a, fg.votes, (uint64_t)fg.ev.size() * a->V, (uint64_t)fg.voted * a->V, s));
    VoteArgs v{};
    v.V = a->V;
    v.voter_ev = fg.d_ev.p + from;
    v.bm_off = fg.d_bm_off.p + from;
    v.bm_len = fg.d_bm_len.p + from;
    v.bm = a->arena.p;
    v.prev_creator = fp.d_creator.p;
    v.prev_dup = fp.d_dup.p;
    v.prev_votes = fp.votes.p;
    v.prev_has_dup = std::any_of(fp.dup.begin(), fp.dup.end(), [](uint32_t d) { return d != NONE; }) ? 1u : 0u;
    v.v_lo = v_lo;
    v.v_hi = v_hi;
    v.wcreator = iv.wpad;
    v.quorum = a->quorum;
    v.votes = fg.votes.p + (uint64_t)from * a->V;
    v.dec = a->d_dec.p;
    v.err = a->d_err.p;
    ARC(flush_uploads(a, s));
    AHIP(a, lx::launch_votes(v, to - from, g == F + 1, s));
    a->stats.vote_launches++;
    return 0;
}

// new slots of frame g, current subject window
int vote_frame(lx_abft *a, const IndexView &iv, uint32_t F, uint32_t g) {
    Frame &fg = frame_at(a, g);
    const uint32_t from = fg.voted, to = (uint32_t)fg.ev.size();
    if (from == to) return 0;
    ARC(vote_slots(a, iv, F, g, from, to, 0, a->vw));
    a->frames[g].voted = to;
    return 0;
}

// widen the subject window of election F to [0, nw) for every voted slot
int widen_window(lx_abft *a, const IndexView &iv, uint32_t F, uint32_t nw) {
    for (uint32_t g = F + 1; g < a->frames.size(); g++) {
        const uint32_t voted = a->frames[g].voted;
        if (!voted) break;
        ARC(vote_slots(a, iv, F, g, 0, voted, a->vw, nw));
    }
    a->vw = nw;
    return 0;
}

// chooseAtropos (SortedIDs = idx order) over the decisions of subjects
// [0, vw): 0 pending, 1 decided (*t, *atropos slot), 2 every subject decided "no"
int atropos_state(const unsigned long long *dec, uint32_t vw, uint64_t *t, uint32_t *obs) {
    uint64_t tmax = 0;
    for (uint32_t v = 0; v < vw; v++) {
        if (dec[v] == ~0ull) return 0;
        tmax = std::max<uint64_t>(tmax, dec[v] >> 32);
        if (dec[v] & 0x80000000ull) {
            *t = tmax;
            *obs = (uint32_t)(dec[v] & kVoteNoRoot);
            return 1;
        }
    }
    return 2;
}

// decision of election F: 0 pending, 1 decided (*t, *atropos slot),
// 2 every subject of the window decided "no" (widen it)
int check_decision(lx_abft *a, const IndexView &iv, uint32_t F, uint64_t *t, uint32_t *obs, int *state) {
    const uint32_t *rb = nullptr;
    ARC(readback(a, iv.stream, reinterpret_cast<const uint32_t *>(a->d_dec.p), 2 * a->vw, a->d_err.p, 1, &rb));
    std::vector<unsigned long long> dec(a->vw);
    memcpy(dec.data(), rb, a->vw * 8ull);
    const uint32_t err = rb[2 * a->vw];
    if (err & kVoteErrTwoRoots)
        return a->fail(LX_ERR_BYZANTINE, "forkless caused by 2 fork roots => more than 1/3W are Byzantine (election frame=%u)", F);
    if (err & kVoteErrQuorum)
        return a->fail(LX_ERR_BYZANTINE, "root must be forkless caused by at least 2/3W of prev roots (election frame=%u)", F);
    if (err & kVoteErrMissing)
        return a->fail(LX_ERR_BYZANTINE, "every root must vote for every not decided subject (election frame=%u)", F);
    *state = atropos_state(dec.data(), a->vw, t, obs);
    if (*state != 2 || a->vw < a->V) return 0;
    return a->fail(LX_ERR_BYZANTINE, "all the roots are decided as 'no', which is possible only if more than 1/3W are Byzantine");
}

int reset_election(lx_abft *a, const IndexView &iv) {
    ARC(reserve(a, a->d_dec, a->V, 0, iv.stream));
    ARC(reserve(a, a->d_err, 1, 0, iv.stream));
    AHIP(a, hipMemsetAsync(a->d_dec.p, 0xFF, a->V * 8ull, iv.stream));
    AHIP(a, hipMemsetAsync(a->d_err.p, 0, 4, iv.stream));
    for (uint32_t g = a->last_decided + 1; g < a->frames.size(); g++) a->frames[g].voted = 0;
    a->vw = std::min<uint32_t>(a->V, kVoteWindow);
    a->dec_dirty = false;
    return 0;
}

// The confirmations of the blocks queued by apply_block (block_log 1, no
// ApplyEvent): block F confirms every not yet confirmed ancestor of its
// Atropos (the DFS of lachesis.go:40-55 stops at confirmed events, whose
// ancestors are all confirmed already), so each event takes the first queued
// block whose Atropos it is an ancestor of.  Events are in Add order (parents
// first): one sweep from the highest Atropos down carries the earliest block
// index to the parents -- the same sets as the blocks' DFS, in one pass over
// the parent lists instead of one stack walk per block.
void confirm_sweep(lx_abft *a) {
    const size_t nb = a->sweep_atropos.size();
    if (!nb) return;
    uint32_t hi = 0;
    for (uint32_t e : a->sweep_atropos) hi = std::max(hi, e);
    std::vector<uint32_t> &lab = a->sweep_label;
    lab.assign((size_t)hi + 1, NONE);
    for (size_t k = nb; k-- > 0;) lab[a->sweep_atropos[k]] = (uint32_t)k;   // earliest block wins
    for (uint32_t e = hi + 1; e-- > 0;) {
        const uint32_t k = lab[e];
        if (k == NONE || a->ev_confirmed[e]) continue;
        a->ev_confirmed[e] = a->sweep_frame[k];
        for (uint64_t j = a->par_off[e]; j < a->par_off[e + 1]; j++) {
            const uint32_t p = a->par[j];
            if (!a->ev_confirmed[p] && k < lab[p]) lab[p] = k;
        }
    }
    a->sweep_atropos.clear();
    a->sweep_frame.clear();
}

// cheaters + confirmation DFS + callbacks; returns 1 in *sealed when EndBlock seals
// (row: the Atropos' HB row already read back, or nullptr)
int apply_block(lx_abft *a, const IndexView &iv, uint32_t F, uint32_t atropos, bool *sealed,
                std::vector<uint32_t> *new_w, const uint32_t *row = nullptr) {
    *sealed = false;
    std::vector<uint32_t> cheaters;
    if (!row) ARC(readback(a, iv.stream, iv.hb + (uint64_t)atropos * iv.stride, a->V, nullptr, 0, &row));
    for (uint32_t c = 0; c < a->V; c++)
        if (row[c] & LX_MARK) cheaters.push_back(c);   // GetMergedHighestBefore(atropos)[c].IsForkDetected()
    // BeginBlock == nil: no confirmation, no seal (lachesis.go:69-71) -- unless
    // the handle logs its blocks itself (option block_log: a BeginBlock that
    // records, no EndBlock)
    const uint32_t log = a->cb.begin_block ? 0u : a->block_log;
    if (!a->cb.begin_block && !log) return 0;
    if (a->cb.begin_block) a->cb.begin_block(a->cb.user, F, atropos, cheaters.data(), (uint32_t)cheaters.size());
    if (log) {
        BlockLog &L = a->blog;
        L.frame.push_back(F);
        L.atropos.push_back(atropos);
        L.cheaters.insert(L.cheaters.end(), cheaters.begin(), cheaters.end());
        L.cheat_off.push_back((uint32_t)L.cheaters.size());
    }
    if (log == 1 && !a->cb.apply_event) {
        // nobody sees the order: the confirmations of this batch's blocks are
        // made by one sweep (confirm_sweep) before anything reads them
        a->sweep_atropos.push_back(atropos);
        a->sweep_frame.push_back(F);
        a->blog.conf_off.push_back(0);
        a->stats.blocks++;
        return 0;
    }
    // dfsSubgraph(atropos, filter) (abft/traversal.go:13-37, lachesis.go:40-55)
    std::vector<uint32_t> stack;
    for (uint32_t walk = atropos;;) {
        if (a->ev_confirmed[walk] == 0) {
            a->ev_confirmed[walk] = F;
            if (a->cb.apply_event) a->cb.apply_event(a->cb.user, walk);
            if (log == 2) a->blog.confirmed.push_back(walk);
            // a parent already confirmed would be popped and skipped: not pushed
            for (uint64_t k = a->par_off[walk]; k < a->par_off[walk + 1]; k++)
                if (a->ev_confirmed[a->par[k]] == 0) stack.push_back(a->par[k]);
        }
        if (stack.empty()) break;
        walk = stack.back();
        stack.pop_back();
    }
    if (a->cb.end_block) {
        uint32_t nv = 0;
        const uint32_t *w = nullptr;
        if (a->cb.end_block(a->cb.user, &nv, &w)) {
            if (!nv || !w) return a->fail(LX_ERR_ARG, "end_block sealed the epoch without validators");
            new_w->assign(w, w + nv);
            *sealed = true;
        }
    }
    if (log) a->blog.conf_off.push_back((uint32_t)a->blog.confirmed.size());
    a->stats.blocks++;
    return 0;
}

// Elections decided ahead.  Election F reads only the root slots of frames
// > F (processKnownRoots replays them after every decision), never the
// outcome of election F-1, so the elections of every frame with two frames of
// roots above it are enqueued together: each with its own vote tables over
// the first subject window and its own decision words, for elect_ahead rounds
// (frames F+1 .. F+elect_ahead), read back after one wait.  The host then
// takes them in frame order as the step-by-step loop would: an election
// decided and final within those rounds is applied (the Atropos HB rows of
// all of them come back in a second wait); the first one that is not
// (pending, every subject of the window "no", a vote error, a slot older than
// its decision left unvoted) hands over to the step-by-step loop, which
// redoes it from scratch.  *sealed_at as in run_elections.
int run_elections_ahead(lx_abft *a, const IndexView &iv, uint64_t *sealed_at, std::vector<uint32_t> *new_w) {
    hipStream_t s = iv.stream;
    const uint32_t R = a->elect_ahead, F0 = a->last_decided + 1;
    if (R < 2 || a->frames.size() < F0 + 3) return 0;
    const uint32_t maxf = (uint32_t)a->frames.size() - 1;
    const uint32_t nE = maxf - 1 - F0;    // elections F0 .. maxf - 2
    const uint32_t vw = std::min<uint32_t>(a->V, kVoteWindow);
    PassTimer pt("elect");
    for (uint32_t f = F0; f <= maxf; f++) ARC(sync_frame(a, frame_at(a, f), s));
    pt.mark("sync_frames");
    // vote tables: election e, round g -> slots(g) x vw
    std::vector<uint64_t> voff;
    uint64_t vtot = 0;
    for (uint32_t e = 0; e < nE; e++)
        for (uint32_t g = F0 + e + 1; g <= std::min(F0 + e + R, maxf); g++) {
            voff.push_back(vtot);
            vtot += (uint64_t)a->frames[g].ev.size() * vw;
        }
    ARC(reserve(a, a->ea_votes, std::max<uint64_t>(vtot, 1), 0, s));
    ARC(reserve(a, a->ea_dec, (uint64_t)nE * vw, 0, s));
    ARC(reserve(a, a->ea_err, nE, 0, s));
    ARC(reserve(a, a->ea_args, voff.size(), 0, s));
    // the tables of round r of every election go out in one launch per kernel
    // (args on the device, grouped by round)
    std::vector<std::vector<VoteArgs>> by_round(R);
    size_t vi = 0;
    for (uint32_t e = 0; e < nE; e++) {
        const uint32_t F = F0 + e;
        const uint32_t *prev = nullptr;
        for (uint32_t g = F + 1; g <= std::min(F + R, maxf); g++, vi++) {
            Frame &fg = a->frames[g], &fp = a->frames[g - 1];
            VoteArgs v{};
            v.V = vw;   // row stride of these tables: subjects [0, vw) only
            v.voter_ev = fg.d_ev.p;
            v.bm_off = fg.d_bm_off.p;
            v.bm_len = fg.d_bm_len.p;
            v.bm = a->arena.p;
            v.prev_creator = fp.d_creator.p;
            v.prev_dup = fp.d_dup.p;
            v.prev_votes = prev;
            v.prev_has_dup = std::any_of(fp.dup.begin(), fp.dup.end(), [](uint32_t d) { return d != NONE; }) ? 1u : 0u;
            v.v_lo = 0;
            v.v_hi = vw;
            v.wcreator = iv.wpad;
            v.quorum = a->quorum;
            v.votes = a->ea_votes.p + voff[vi];
            v.dec = a->ea_dec.p + (uint64_t)e * vw;
            v.err = a->ea_err.p + e;
            v.n_voters = (uint32_t)fg.ev.size();
            by_round[g - F - 1].push_back(v);
            prev = v.votes;
        }
    }
    std::vector<uint64_t> aoff(R + 1, 0);
    for (uint32_t r = 0; r < R; r++) {
        aoff[r + 1] = aoff[r] + by_round[r].size();
        a->up.add(a->ea_args.p + aoff[r], by_round[r].data(), by_round[r].size() * sizeof(VoteArgs));
    }
    ARC(flush_uploads(a, s));
    AHIP(a, hipMemsetAsync(a->ea_dec.p, 0xFF, (uint64_t)nE * vw * 8, s));
    AHIP(a, hipMemsetAsync(a->ea_err.p, 0, nE * 4ull, s));
    for (uint32_t r = 0; r < R; r++) {
        uint32_t mx = 0;
        for (const VoteArgs &v : by_round[r]) mx = std::max(mx, v.n_voters);
        AHIP(a, lx::launch_votes_multi(a->ea_args.p + aoff[r], (uint32_t)by_round[r].size(), mx, vw, r == 0, s));
        a->stats.vote_launches++;
    }
    pt.mark("launch");
    const uint32_t *rb = nullptr;
    ARC(readback(a, s, reinterpret_cast<const uint32_t *>(a->ea_dec.p), 2 * nE * vw, a->ea_err.p, nE, &rb));
    pt.mark("wait");
    std::vector<unsigned long long> dec((uint64_t)nE * vw);
    memcpy(dec.data(), rb, dec.size() * 8);
    std::vector<uint32_t> err(rb + 2ull * nE * vw, rb + 2ull * nE * vw + nE);
    // decided prefix of the elections, in frame order
    struct Decided {
        uint32_t F, atropos;
        uint64_t t;
    };
    std::vector<Decided> done;
    std::vector<uint64_t> L(maxf + 2, ~0ull);   // L[h] = oldest slot of frames >= h
    for (uint32_t h = maxf; h >= 1; h--) {
        L[h] = L[h + 1];
        for (uint32_t x : a->frames[h].ev) L[h] = std::min<uint64_t>(L[h], x);
    }
    for (uint32_t e = 0; e < nE; e++) {
        const uint32_t F = F0 + e;
        uint64_t t = 0;
        uint32_t obs = 0;
        if (err[e] || atropos_state(dec.data() + (uint64_t)e * vw, vw, &t, &obs) != 1) break;
        if (t > L[std::min(F + R, maxf) + 1]) break;   // an older slot is not voted yet
        if (obs >= a->frames[F].ev.size()) break;
        done.push_back({F, a->frames[F].ev[obs], t});
    }
    if (done.empty()) return 0;
    std::vector<uint32_t> rows(done.size());
    for (size_t k = 0; k < done.size(); k++) rows[k] = done[k].atropos;
    pt.mark("decide");
    const uint32_t *hb_rows = nullptr;
    ARC(readback_rows(a, iv, rows, &hb_rows));
    pt.mark("rows");
    for (size_t k = 0; k < done.size(); k++) {
        const uint64_t decided_at = std::max<uint64_t>(done[k].t, a->t_prev);
        bool sealed;
        ARC(apply_block(a, iv, done[k].F, done[k].atropos, &sealed, new_w, hb_rows + k * (uint64_t)a->V));
        if (sealed) {
            *sealed_at = decided_at;
            return 0;
        }
        a->t_prev = decided_at;
        a->last_decided = done[k].F;
    }
    pt.mark("apply");
    for (uint32_t g = 1; g <= a->last_decided && g < a->frames.size(); g++) a->frames[g].votes.release();
    a->dec_dirty = true;
    a->stats.elections_ahead += (uint32_t)done.size();
    return 0;
}

// Runs elections over all known root slots; *sealed_at = event that decided a
// sealing frame (NONE if none).
int run_elections(lx_abft *a, uint64_t *sealed_at, std::vector<uint32_t> *new_w) {
    *sealed_at = ~0ull;
    IndexView iv;
    int rc = lx_index_view(a->ix, &iv);
    if (rc) return a->ixfail(rc);
    ARC(run_elections_ahead(a, iv, sealed_at, new_w));
    if (*sealed_at != ~0ull) return 0;
    for (;;) {
        const uint32_t F = a->last_decided + 1;
        if (a->dec_dirty) ARC(reset_election(a, iv));
        const uint32_t maxf = (uint32_t)a->frames.size() - 1;
        if (a->frames.size() <= F + 1) return 0;
        ARC(sync_frame(a, frame_at(a, F), iv.stream));
        int state = 0;
        uint64_t t = 0;
        uint32_t obs = 0;
        bool checked = false;
        for (uint32_t g = F + 1; g <= maxf; g++) {
            const bool fresh = frame_at(a, g).voted < frame_at(a, g).ev.size();
            ARC(vote_frame(a, iv, F, g));
            if (g < F + 2 || (checked && !fresh)) continue;
            ARC(check_decision(a, iv, F, &t, &obs, &state));
            while (state == 2) {   // all subjects so far decided "no": the Atropos is further down
                ARC(widen_window(a, iv, F, std::min<uint32_t>(a->V, a->vw * 2)));
                ARC(check_decision(a, iv, F, &t, &obs, &state));
            }
            checked = true;
            if (state) {
                // final unless a slot not yet voted in this election is older
                uint64_t L = ~0ull;
                for (uint32_t h = g + 1; h <= maxf; h++) {
                    const Frame &fh = a->frames[h];
                    for (size_t k = fh.voted; k < fh.ev.size(); k++) L = std::min<uint64_t>(L, fh.ev[k]);
                }
                if (t <= L) break;
                state = 0;
            }
        }
        if (!state) return 0;
        const Frame &fF = a->frames[F];
        if (obs >= fF.ev.size()) return a->fail(LX_ERR_STATE, "decided Atropos has no root (frame %u)", F);
        const uint32_t atropos = fF.ev[obs];
        const uint64_t decided_at = std::max<uint64_t>(t, a->t_prev);
        bool sealed;
        ARC(apply_block(a, iv, F, atropos, &sealed, new_w));
        if (sealed) {
            *sealed_at = decided_at;
            return 0;
        }
        a->t_prev = decided_at;
        a->last_decided = F;
        for (uint32_t g = 1; g <= F && g < a->frames.size(); g++) a->frames[g].votes.release();
        a->dec_dirty = true;
    }
}

struct Snapshot {
    std::vector<size_t> sizes;
    uint64_t arena_used;
    uint64_t n_events;
};

Snapshot take_snapshot(lx_abft *a) {
    Snapshot s;
    for (const Frame &f : a->frames) s.sizes.push_back(f.ev.size());
    s.arena_used = a->arena_used;
    s.n_events = a->ev_frame.size();
    return s;
}

void restore_snapshot(lx_abft *a, const Snapshot &s) {
    for (size_t f = 0; f < a->frames.size(); f++) {
        Frame &fr = a->frames[f];
        size_t keep = f < s.sizes.size() ? s.sizes[f] : 0;
        while (fr.ev.size() > keep) {
            uint32_t c = fr.creator.back();
            fr.last_of[c] = fr.dup.back();
            fr.ev.pop_back();
            fr.creator.pop_back();
            fr.dup.pop_back();
            fr.bm_off.pop_back();
            fr.bm_len.pop_back();
        }
        fr.synced = std::min<uint32_t>(fr.synced, (uint32_t)keep);
        fr.voted = std::min<uint32_t>(fr.voted, (uint32_t)keep);
    }
    while (a->frames.size() > s.sizes.size() && a->frames.size() > 1 && a->frames.back().ev.empty()) {
        a->frames.back().release();
        a->frames.pop_back();
    }
    a->arena_used = s.arena_used;
    a->ev_frame.resize(s.n_events);
    a->ev_sp.resize(s.n_events);
    a->ev_confirmed.resize(s.n_events);
    a->sweep_atropos.clear();
    a->sweep_frame.clear();
    a->par_off.resize(s.n_events + 1);
    a->par.resize(a->par_off.back());
}

// adds the batch to the index and the host event tables
int add_events(lx_abft *a, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff,
               const uint32_t *par) {
    PassTimer pt("index");
    uint32_t err_index = 0;
    int rc = lx_add_batch(a->ix, n, creator, seq, poff, par, nullptr, &err_index);
    if (rc) return a->ixfail(rc);
    pt.mark("add_batch");
    const uint64_t e0 = a->ev_sp.size();
    a->ev_sp.resize(e0 + n);
    a->ev_frame.resize(e0 + n, 0);
    a->ev_confirmed.resize(e0 + n, 0);
    a->par_off.reserve(a->par_off.size() + n);
    const uint64_t q0 = a->par.size();
    a->par.insert(a->par.end(), par + poff[0], par + poff[n]);
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t p0 = poff[i], p1 = poff[i + 1];
        a->ev_sp[e0 + i] = seq[i] > 1 && p1 > p0 ? par[p0] : NONE;   // inter/dag/event.go:87-92
        a->par_off.push_back(q0 + (p1 - poff[0]));
    }
    pt.mark("tables");
    return 0;
}

int process(lx_abft *a, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff,
            const uint32_t *par, const uint32_t *claimed, uint32_t *out_frame, uint32_t *consumed) {
    *consumed = 0;
    if (!n) return 0;
    const uint64_t base = a->ev_frame.size();
    Snapshot snap = take_snapshot(a);
    double t0 = now_ms();
    ARC(add_events(a, n, creator, seq, poff, par));
    double t1 = now_ms();
    ARC(compute_frames(a, base, n, creator, claimed));
    double t2 = now_ms();
    a->stats.ms_index += (float)(t1 - t0);
    a->stats.ms_frames += (float)(t2 - t1);
    // checkAndSaveEvent: claimed frame must equal the computed one
    uint32_t bad = n;
    if (claimed)
        for (uint32_t i = 0; i < n; i++)
            if (claimed[i] != LX_FRAME_BUILD && claimed[i] != a->ev_frame[base + i]) { bad = i; break; }
    if (bad < n) {
        // the reference processes the events before the bad one; redo them alone
        restore_snapshot(a, snap);
        int rc = lx_drop_not_flushed(a->ix);
        if (rc) return a->ixfail(rc);
        uint32_t c = 0;
        if (bad) ARC(process(a, bad, creator, seq, poff, par, claimed, out_frame, &c));
        *consumed = c;
        if (c == bad) a->err = "claimed frame mismatched with calculated";
        return c == bad ? LX_ERR_FRAME : 0;
    }
    uint64_t sealed_at;
    std::vector<uint32_t> new_w;
    double t3 = now_ms();
    ARC(run_elections(a, &sealed_at, &new_w));
    confirm_sweep(a);
    double t4 = now_ms();
    a->stats.ms_election += (float)(t4 - t3);
    uint32_t done = n;
    if (sealed_at != ~0ull) done = (uint32_t)(sealed_at - base + 1);
    if (out_frame)
        for (uint32_t i = 0; i < done; i++) out_frame[i] = a->ev_frame[base + i];
    *consumed = done;
    if (sealed_at != ~0ull) {
        ARC(start_epoch(a, a->epoch + 1, (uint32_t)new_w.size(), new_w.data()));
    } else {
        int rc = lx_flush(a->ix);
        if (rc) return a->ixfail(rc);
    }
    return 0;
}

}  // namespace

extern "C" {

int lx_abft_create(lx_index *index, lx_abft **out) {
    if (!index || !out) return LX_ERR_ARG;
    lx_abft *a = new lx_abft();
    a->ix = index;
    *out = a;
    return 0;
}

void lx_abft_destroy(lx_abft *a) {
    if (!a) return;
    for (Frame &f : a->frames) f.release();
    a->arena.release();
    a->d_cand.release();
    a->d_psum.release();
    a->d_q.release();
    a->d_dec.release();
    a->d_err.release();
    a->d_kcol.release();
    a->d_kflag.release();
    a->d_kw.release();
    a->ea_votes.release();
    a->ea_err.release();
    a->ea_dec.release();
    a->ea_args.release();
    a->d_fcargs.release();
    a->d_qargs.release();
    (void)hipDeviceSynchronize();   // queued work may still use pooled buffers
    a->up.release();
    if (a->q_pin) (void)hipHostFree(a->q_pin);
    if (a->rb_pin) (void)hipHostFree(a->rb_pin);
    for (hipEvent_t e : a->fc_ev) (void)hipEventDestroy(e);
    a->pool.drain();
    delete a;
}

const char *lx_abft_last_error(const lx_abft *a) { return a ? a->err.c_str() : "null handle"; }

int lx_abft_bootstrap(lx_abft *a, uint32_t epoch, uint32_t nv, const uint32_t *w, const lx_abft_callbacks *cb) {
    if (!a) return LX_ERR_ARG;
    if (a->booted) return a->fail(LX_ERR_STATE, "already bootstrapped");
    a->cb = cb ? *cb : lx_abft_callbacks{};
    ARC(start_epoch(a, epoch, nv, w));
    a->booted = true;
    return 0;
}

int lx_abft_set_option(lx_abft *a, const char *name, int64_t value) {
    if (!a || !name) return LX_ERR_ARG;
    const std::string k(name);
    if (k == "spec_depth") {
        if (value < 0 || value > 16) return a->fail(LX_ERR_ARG, "spec_depth must be 0..16");
        a->spec_depth = (uint32_t)value;
    } else if (k == "fc16") {
        if (value < 0 || value > 1) return a->fail(LX_ERR_ARG, "fc16 must be 0 or 1");
        a->fc16 = value != 0;
    } else if (k == "claimed_batch") {
        if (value < 0 || value > 1) return a->fail(LX_ERR_ARG, "claimed_batch must be 0 or 1");
        a->claimed_batch = value != 0;
    } else if (k == "block_log") {
        if (value < 0 || value > 2) return a->fail(LX_ERR_ARG, "block_log must be 0, 1 or 2");
        a->block_log = (uint32_t)value;
    } else if (k == "elect_ahead") {
        if (value < 0 || value > 8 || value == 1) return a->fail(LX_ERR_ARG, "elect_ahead must be 0 or 2..8");
        a->elect_ahead = (uint32_t)value;
    } else {
        return a->fail(LX_ERR_ARG, "unknown option %s", name);
    }
    return 0;
}

int lx_abft_reset(lx_abft *a, uint32_t epoch, uint32_t nv, const uint32_t *w) {
    if (!a) return LX_ERR_ARG;
    if (!a->booted) return a->fail(LX_ERR_STATE, "not bootstrapped");
    return start_epoch(a, epoch, nv, w);
}

int lx_abft_process_batch(lx_abft *a, uint32_t n, const uint32_t *creator, const uint32_t *seq,
                          const uint64_t *poff, const uint32_t *par, const uint32_t *claimed, uint32_t *out_frame,
                          uint32_t *consumed) {
    if (!a || !consumed) return LX_ERR_ARG;
    if (!a->booted) return a->fail(LX_ERR_STATE, "not bootstrapped");
    a->stats = lx_abft_stats{};
    a->blog.clear();
    return process(a, n, creator, seq, poff, par, claimed, out_frame, consumed);
}

int lx_abft_block_log(const lx_abft *a, uint32_t *n_blocks, const uint32_t **frame, const uint32_t **atropos,
                      const uint32_t **cheat_off, const uint32_t **cheaters, const uint32_t **conf_off,
                      const uint32_t **confirmed) {
    if (!a || !n_blocks) return LX_ERR_ARG;
    const BlockLog &L = a->blog;
    *n_blocks = (uint32_t)L.frame.size();
    if (frame) *frame = L.frame.data();
    if (atropos) *atropos = L.atropos.data();
    if (cheat_off) *cheat_off = L.cheat_off.data();
    if (cheaters) *cheaters = L.cheaters.data();
    if (conf_off) *conf_off = L.conf_off.data();
    if (confirmed) *confirmed = L.confirmed.data();
    return 0;
}

int lx_abft_build(lx_abft *a, uint32_t creator, uint32_t seq, uint32_t np, const uint32_t *parents,
                  uint32_t *out_frame) {
    if (!a || !out_frame) return LX_ERR_ARG;
    if (!a->booted) return a->fail(LX_ERR_STATE, "not bootstrapped");
    const uint64_t base = a->ev_frame.size();
    Snapshot snap = take_snapshot(a);
    uint64_t poff[2] = {0, np};
    int rc = add_events(a, 1, &creator, &seq, poff, parents);
    if (rc == 0) rc = compute_frames(a, base, 1, &creator, nullptr);
    if (rc == 0) *out_frame = a->ev_frame[base];
    restore_snapshot(a, snap);
    int rc2 = lx_drop_not_flushed(a->ix);
    if (rc) return rc;
    if (rc2) return a->ixfail(rc2);
    return 0;
}

uint32_t lx_abft_epoch(const lx_abft *a) { return a ? a->epoch : 0; }
uint32_t lx_abft_last_decided_frame(const lx_abft *a) { return a ? a->last_decided : 0; }

int lx_abft_frame_roots(lx_abft *a, uint32_t f, uint32_t *out, uint32_t cap, uint32_t *n) {
    if (!a || !n) return LX_ERR_ARG;
    *n = 0;
    if (f >= a->frames.size()) return 0;
    const auto &ev = a->frames[f].ev;
    *n = (uint32_t)ev.size();
    if (out) std::copy(ev.begin(), ev.begin() + std::min<size_t>(cap, ev.size()), out);
    return 0;
}

int lx_abft_event_frame(const lx_abft *a, uint32_t ev, uint32_t *frame) {
    if (!a || !frame || ev >= a->ev_frame.size()) return LX_ERR_ARG;
    *frame = a->ev_frame[ev];
    return 0;
}

int lx_abft_event_confirmed_on(const lx_abft *a, uint32_t ev, uint32_t *frame) {
    if (!a || !frame || ev >= a->ev_confirmed.size()) return LX_ERR_ARG;
    *frame = a->ev_confirmed[ev];
    return 0;
}

int lx_abft_last_stats(const lx_abft *a, lx_abft_stats *out) {
    if (!a || !out) return LX_ERR_ARG;
    *out = a->stats;
    return 0;
}

}  // extern "C"
