// lx_emitter.cpp -- emitter QuorumIndexer behind include/lachesis_emitter.h.
//
// emitter/ancestor.QuorumIndexer (emitter/ancestor/quorum_indexer.go:20-158)
// over the index's device planes.  ProcessEvent only ever overwrites whole
// matrix columns (the event creator's) and the whole self-parent row, so a
// batch of events reduces to the last event per creator plus the last self
// event, applied in one launch (k_qi_update).  recacheState runs lazily, as in
// the reference, when a median or a metric is asked after an update.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lachesis_emitter.h"
#include "lx_internal.h"

namespace {
constexpr uint32_t kQiMaxV = 8192;
}

struct lx_qi {
    lx_index *ix = nullptr;
    std::string err;
    uint32_t V = 0, quorum = 0, B = 0;
    bool dirty = true;
    uint32_t *mt = nullptr, *sp = nullptr, *median = nullptr, *weights = nullptr;
    int32_t *cheat_of = nullptr;
    uint32_t *cheat_off = nullptr, *cheat_br = nullptr;
    uint32_t *d_ev = nullptr, *d_tg = nullptr;
    unsigned long long *d_out = nullptr;
    unsigned long long *lastk = nullptr;   // [V + 1] last batch position per creator / self (k_qi_mark)
    uint32_t gen = 0;
    std::vector<uint32_t> stage;           // host image of a large batch: events, then self flags
    hipEvent_t staged = nullptr;           // its copy has read `stage`
    hipEvent_t done = nullptr;             // the last ProcessEvent launch finished (freeing waits for it)
    uint64_t cap = 0;

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

#define QHIP(q, expr)                               \
    do {                                            \
        int _rc = (q)->hip((expr), #expr);          \
        if (_rc) return _rc;                        \
    } while (0)
#define QRC(expr)                                   \
    do {                                            \
        int _rc = (expr);                           \
        if (_rc) return _rc;                        \
    } while (0)

namespace {

void qi_free(lx_qi *q) {
    void *p[] = {q->mt, q->sp, q->median, q->weights, q->cheat_of, q->cheat_off, q->cheat_br, q->d_ev, q->d_tg,
                 q->d_out, q->lastk};
    for (void *x : p)
        if (x) (void)hipFree(x);
    q->mt = q->sp = q->median = q->weights = nullptr;
    q->cheat_of = nullptr;
    q->cheat_off = q->cheat_br = nullptr;
    q->d_ev = q->d_tg = nullptr;
    q->d_out = nullptr;
    q->lastk = nullptr;
    q->cap = 0;
    q->B = 0;
}

int view(lx_qi *q, IndexView *iv) {
    int rc = lx_index_view(q->ix, iv);
    if (rc) {
        q->err = lx_last_error(q->ix);
        return rc;
    }
    if (iv->shard_count > 1) return q->fail(LX_ERR_STATE, "QuorumIndexer needs an unsharded index");
    if (iv->V != q->V) return q->fail(LX_ERR_STATE, "validators changed (new epoch): call lx_qi_reset");
    QHIP(q, hipSetDevice(iv->device));
    return 0;
}

// cheaters' branch lists: GetMergedHighestBefore gathers over BranchIDByCreators
int refresh_cheaters(lx_qi *q, const IndexView &iv) {
    if (q->B == iv.B) return 0;
    std::vector<int32_t> of(q->V, -1);
    std::vector<uint32_t> off{0}, br;
    for (uint32_t c = 0; c < q->V; c++) {
        const auto &l = (*iv.by_creator)[c];
        if (l.size() < 2) continue;
        of[c] = (int32_t)(off.size() - 1);
        br.insert(br.end(), l.begin(), l.end());
        off.push_back((uint32_t)br.size());
    }
    if (q->cheat_off) (void)hipFree(q->cheat_off);
    if (q->cheat_br) (void)hipFree(q->cheat_br);
    q->cheat_off = q->cheat_br = nullptr;
    QHIP(q, hipMalloc((void **)&q->cheat_off, off.size() * 4));
    QHIP(q, hipMalloc((void **)&q->cheat_br, std::max<size_t>(br.size(), 1) * 4));
    QHIP(q, hipMemcpyAsync(q->cheat_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, iv.stream));
    if (!br.empty()) QHIP(q, hipMemcpyAsync(q->cheat_br, br.data(), br.size() * 4, hipMemcpyHostToDevice, iv.stream));
    QHIP(q, hipMemcpyAsync(q->cheat_of, of.data(), q->V * 4ull, hipMemcpyHostToDevice, iv.stream));
    QHIP(q, hipStreamSynchronize(iv.stream));
    q->B = iv.B;
    return 0;
}

QiArgs qi_args(lx_qi *q, const IndexView &iv) {
    QiArgs a{};
    a.hb = iv.hb;
    a.stride = iv.stride;
    a.V = q->V;
    a.forks = iv.B > iv.V ? 1u : 0u;
    a.cheat_of = q->cheat_of;
    a.cheat_off = q->cheat_off;
    a.cheat_br = q->cheat_br;
    a.weights = q->weights;
    a.quorum = q->quorum;
    a.mt = q->mt;
    a.sp = q->sp;
    a.median = q->median;
    a.ev_creator = iv.ev_creator;
    a.lastk = q->lastk;
    return a;
}

int ensure_cap(lx_qi *q, uint64_t n, hipStream_t s) {
    if (n <= q->cap) return 0;
    const uint64_t cap = std::max<uint64_t>(n, 1024);
    QHIP(q, hipStreamSynchronize(s));   // ProcessEvent launches may still read the old buffers
    if (q->d_ev) (void)hipFree(q->d_ev);
    if (q->d_tg) (void)hipFree(q->d_tg);
    if (q->d_out) (void)hipFree(q->d_out);
    q->d_ev = q->d_tg = nullptr;
    q->d_out = nullptr;
    q->cap = 0;
    QHIP(q, hipMalloc((void **)&q->d_ev, cap * 4));
    QHIP(q, hipMalloc((void **)&q->d_tg, cap * 4));
    QHIP(q, hipMalloc((void **)&q->d_out, cap * 8));
    q->cap = cap;
    return 0;
}

int recache(lx_qi *q, const IndexView &iv) {
    if (!q->dirty) return 0;
    QHIP(q, lx::launch_qi_median(qi_args(q, iv), iv.stream));
    q->dirty = false;
    return 0;
}

int check_events(lx_qi *q, const IndexView &iv, uint32_t n, const uint32_t *ev) {
    for (uint32_t i = 0; i < n; i++)
        if (ev[i] >= iv.n_events) return q->fail(LX_ERR_ARG, "unknown event %u", ev[i]);
    return 0;
}

int copy_out(lx_qi *q, const IndexView &iv, void *dst, const void *src, uint64_t bytes) {
    QHIP(q, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, iv.stream));
    QHIP(q, hipStreamSynchronize(iv.stream));
    return 0;
}

}  // namespace

extern "C" {

int lx_qi_create(lx_index *index, lx_qi **out) {
    if (!index || !out) return LX_ERR_ARG;
    lx_qi *q = new lx_qi();
    q->ix = index;
    int rc = lx_qi_reset(q);
    if (rc) {
        lx_qi_destroy(q);
        return rc;
    }
    *out = q;
    return 0;
}

void lx_qi_destroy(lx_qi *q) {
    if (!q) return;
    if (q->done) (void)hipEventSynchronize(q->done);   // ProcessEvent launches in flight
    qi_free(q);
    if (q->staged) (void)hipEventDestroy(q->staged);
    if (q->done) (void)hipEventDestroy(q->done);
    delete q;
}

const char *lx_qi_last_error(const lx_qi *q) { return q ? q->err.c_str() : "null handle"; }

int lx_qi_reset(lx_qi *q) {
    if (!q) return LX_ERR_ARG;
    IndexView iv;
    int rc = lx_index_view(q->ix, &iv);
    if (rc) {
        q->err = lx_last_error(q->ix);
        return rc;
    }
    if (iv.shard_count > 1) return q->fail(LX_ERR_STATE, "QuorumIndexer needs an unsharded index");
    if (iv.V > kQiMaxV) return q->fail(LX_ERR_ARG, "QuorumIndexer supports up to %u validators", kQiMaxV);
    QHIP(q, hipSetDevice(iv.device));
    if (q->done) QHIP(q, hipEventSynchronize(q->done));   // ProcessEvent launches in flight read the old buffers
    qi_free(q);
    q->V = iv.V;
    q->quorum = iv.quorum;
    const uint64_t V = q->V;
    QHIP(q, hipMalloc((void **)&q->mt, V * V * 4));
    QHIP(q, hipMalloc((void **)&q->sp, V * 4));
    QHIP(q, hipMalloc((void **)&q->median, V * 4));
    QHIP(q, hipMalloc((void **)&q->weights, V * 4));
    QHIP(q, hipMalloc((void **)&q->cheat_of, V * 4));
    QHIP(q, hipMalloc((void **)&q->lastk, (V + 1) * 8));
    QHIP(q, hipMemsetAsync(q->lastk, 0, (V + 1) * 8, iv.stream));
    q->gen = 0;
    QHIP(q, hipMemsetAsync(q->mt, 0, V * V * 4, iv.stream));
    QHIP(q, hipMemsetAsync(q->sp, 0, V * 4, iv.stream));
    QHIP(q, hipMemsetAsync(q->median, 0, V * 4, iv.stream));
    QHIP(q, hipMemcpyAsync(q->weights, iv.weights->data(), V * 4, hipMemcpyHostToDevice, iv.stream));
    QHIP(q, hipStreamSynchronize(iv.stream));
    q->dirty = true;
    q->B = 0;
    return refresh_cheaters(q, iv);
}

int lx_qi_process_events(lx_qi *q, uint32_t n, const uint32_t *ev, const uint8_t *self_event) {
    if (!q || (n && !ev)) return LX_ERR_ARG;
    if (!n) return 0;
    IndexView iv;
    QRC(view(q, &iv));
    QRC(check_events(q, iv, n, ev));
    QRC(refresh_cheaters(q, iv));
    // no host round trip: the device reduces the batch to the last event per
    // creator and the last self event (k_qi_mark / k_qi_apply); nothing to wait for
    QiBatch b{};
    b.n = n;
    if (++q->gen == 0) {   // stamps wrapped: start over
        QHIP(q, hipMemsetAsync(q->lastk, 0, (q->V + 1ull) * 8, iv.stream));
        q->gen = 1;
    }
    b.gen = q->gen;
    if (n <= kQiInline) {
        for (uint32_t i = 0; i < n; i++) {
            b.iev[i] = ev[i];
            if (self_event && self_event[i]) b.iself |= 1u << i;
        }
    } else {
        QRC(ensure_cap(q, (uint64_t)2 * n, iv.stream));
        if (!q->staged) QHIP(q, hipEventCreateWithFlags(&q->staged, hipEventDisableTiming));
        else QHIP(q, hipEventSynchronize(q->staged));
        q->stage.resize(2ull * n);
        for (uint32_t i = 0; i < n; i++) {
            q->stage[i] = ev[i];
            q->stage[n + i] = self_event && self_event[i] ? 1u : 0u;
        }
        QHIP(q, hipMemcpyAsync(q->d_ev, q->stage.data(), 8ull * n, hipMemcpyHostToDevice, iv.stream));
        QHIP(q, hipEventRecord(q->staged, iv.stream));
        b.ev = q->d_ev;
        b.self = q->d_ev + n;
    }
    QHIP(q, lx::launch_qi_apply(qi_args(q, iv), b, iv.stream));
    if (!q->done) QHIP(q, hipEventCreateWithFlags(&q->done, hipEventDisableTiming));
    QHIP(q, hipEventRecord(q->done, iv.stream));
    q->dirty = true;
    return 0;
}

int lx_qi_median_seqs(lx_qi *q, uint32_t *out) {
    if (!q || !out) return LX_ERR_ARG;
    IndexView iv;
    QRC(view(q, &iv));
    QRC(recache(q, iv));
    return copy_out(q, iv, out, q->median, q->V * 4ull);
}

int lx_qi_matrix(lx_qi *q, uint32_t *out) {
    if (!q || !out) return LX_ERR_ARG;
    IndexView iv;
    QRC(view(q, &iv));
    const uint64_t V = q->V;
    std::vector<uint32_t> t(V * V);
    QRC(copy_out(q, iv, t.data(), q->mt, V * V * 4));
    for (uint64_t c = 0; c < V; c++)
        for (uint64_t v = 0; v < V; v++) out[v * V + c] = t[c * V + v];
    return 0;
}

int lx_qi_self_parent_seqs(lx_qi *q, uint32_t *out) {
    if (!q || !out) return LX_ERR_ARG;
    IndexView iv;
    QRC(view(q, &iv));
    return copy_out(q, iv, out, q->sp, q->V * 4ull);
}

int lx_qi_metric_of(lx_qi *q, uint32_t n, const uint32_t *ev, uint32_t cap, uint64_t *out) {
    if (!q || (n && (!ev || !out))) return LX_ERR_ARG;
    if (!n) return 0;
    IndexView iv;
    QRC(view(q, &iv));
    QRC(check_events(q, iv, n, ev));
    QRC(refresh_cheaters(q, iv));
    QRC(recache(q, iv));
    QRC(ensure_cap(q, n, iv.stream));
    QHIP(q, hipMemcpyAsync(q->d_ev, ev, n * 4ull, hipMemcpyHostToDevice, iv.stream));
    QHIP(q, lx::launch_qi_metric(qi_args(q, iv), q->d_ev, n, cap, q->d_out, iv.stream));
    return copy_out(q, iv, out, q->d_out, n * 8ull);
}

}  // extern "C"
