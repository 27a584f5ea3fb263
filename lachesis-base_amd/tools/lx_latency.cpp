// lx_latency.cpp -- per-call latency and antichain-fed throughput of the C ABI,
// driven from native code the way the cgo shim drives it (bench tooling, not
// part of the index library).
//
// The reference's callers use the index one event / one pair at a time:
//   IndexedLachesis.Process: Add(e), ..., Flush            (abft/indexed_lachesis.go:69-82)
//   IndexedLachesis.Build:   Add(e), ..., DropNotFlushed   (abft/indexed_lachesis.go:53-63)
//   calcFrameIdx: ForklessCause(e, root) per root          (abft/event_processing.go:149-161)
//   applyAtropos / emitter: GetMergedHighestBefore(id)     (abft/lachesis.go:57)
// lx_bench_latency times those calls (wall clock around each C call; p50 / p99
// / mean in microseconds) on a history-indexed epoch of the given DAG, then the
// throughput of feeding the DAG antichain by antichain: the events re-ordered
// by topological level (a valid Add order) and each level added as one
// lx_add_batch + lx_flush, directly and through the level batcher.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lachesis_batcher.h"
#include "../../include/lachesis_emitter.h"
#include "../../include/lachesis_hip.h"

namespace {

using clk = std::chrono::steady_clock;
inline double us_since(clk::time_point t0) {
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

struct Stat {
    double p50 = 0, p99 = 0, mean = 0, p999 = 0, max = 0;
};
Stat stat_of(std::vector<double> v) {
    Stat s;
    if (v.empty()) return s;
    std::sort(v.begin(), v.end());
    s.p50 = v[v.size() / 2];
    s.p99 = v[std::min(v.size() - 1, (size_t)(v.size() * 0.99))];
    s.p999 = v[std::min(v.size() - 1, (size_t)(v.size() * 0.999))];
    s.max = v.back();
    double t = 0;
    for (double x : v) t += x;
    s.mean = t / v.size();
    return s;
}

// calls of each kind made before its timed ones: the first call of a kind pays
// one-time setup (a getter's pinned buffers, the row server's stream and its
// kernel's code object, a fill's scratch), reported apart as first_us
constexpr uint32_t kWarm = 3;

// the DAG re-ordered by topological level (stable inside a level), parents remapped
struct Leveled {
    std::vector<uint32_t> creator, seq, par;
    std::vector<uint64_t> poff;
    std::vector<uint64_t> lvl_off;   // event offsets of the levels
};

Leveled by_level(uint64_t N, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff, const uint32_t *par) {
    std::vector<uint32_t> lvl(N);
    uint32_t maxl = 0;
    for (uint64_t i = 0; i < N; i++) {
        uint32_t l = 0;
        for (uint64_t k = poff[i]; k < poff[i + 1]; k++) l = std::max(l, lvl[par[k]] + 1);
        lvl[i] = l;
        maxl = std::max(maxl, l);
    }
    std::vector<uint64_t> cnt(maxl + 2, 0);
    for (uint64_t i = 0; i < N; i++) cnt[lvl[i] + 1]++;
    for (uint32_t l = 0; l <= maxl; l++) cnt[l + 1] += cnt[l];
    Leveled o;
    o.lvl_off.assign(cnt.begin(), cnt.end());
    std::vector<uint32_t> pos(N), order(N);
    for (uint64_t i = 0; i < N; i++) {
        pos[i] = (uint32_t)cnt[lvl[i]]++;
        order[pos[i]] = (uint32_t)i;
    }
    o.creator.resize(N);
    o.seq.resize(N);
    o.poff.resize(N + 1);
    o.par.reserve(poff[N]);
    o.poff[0] = 0;
    for (uint64_t j = 0; j < N; j++) {
        const uint32_t i = order[j];
        o.creator[j] = creator[i];
        o.seq[j] = seq[i];
        for (uint64_t k = poff[i]; k < poff[i + 1]; k++) o.par.push_back(pos[par[k]]);
        o.poff[j + 1] = o.par.size();
    }
    return o;
}

}  // namespace

extern "C" {

// out receives 128 doubles: for each of the 11 call kinds p50, p99, mean (us):
//   0 add n=1 (Process: Add + Flush; host call time, the launch is not waited for)
//   1 add n=1 + lx_sync (completion)
//   2 Build: add n=1 + DropNotFlushed + lx_sync
//   3 one antichain (a level, ~V/(1.6 P) events) add + flush + lx_sync
//   4 add n=1024 + lx_sync
//   5 ForklessCause n=1        6 ForklessCause n=667 (~2/3 V: calcFrameIdx)
//   7 GetHighestBefore         8 GetLowestAfter       9 GetMergedHighestBefore
//  10 getter batch of 64 merged HB rows (lx_get_merged_highest_before_batch)
// then [33] antichain-fed events/s (levels added directly), [34] events fed,
// [35] levels fed, [36] batcher-fed events/s (push a level, pop, add, flush),
// [37] mean events per level; [40..42] lx_forkless_cause of a new event's
// first pair (a cache miss: pending Add + row fill), [43..45] its next pairs
// (hits); [48 + 4 k ..] for call kind k: p99.9, max, the first call of the
// kind (before kWarm untimed calls), the timed calls' count; [96..99] add
// n=1024 + sync split: the add call's p50 / p99, the sync's p50 / p99.
int lx_bench_latency(int device, uint32_t V, const uint32_t *weights, uint64_t N, const uint32_t *creator,
                     const uint32_t *seq, const uint64_t *poff, const uint32_t *par, uint64_t history,
                     uint32_t reps, uint64_t feed_events, double *out, char *err, uint32_t err_cap) {
    auto fail = [&](const char *what, lx_index *h) {
        snprintf(err, err_cap, "%s: %s", what, h ? lx_last_error(h) : "");
        if (h) lx_destroy(h);
        return -1;
    };
    Leveled d = by_level(N, creator, seq, poff, par);
    // history = whole levels
    uint64_t L0 = 0;
    while (L0 + 1 < d.lvl_off.size() && d.lvl_off[L0 + 1] <= history) L0++;
    const uint64_t H = d.lvl_off[L0];
    lx_config cfg{};
    cfg.device = device;
    cfg.event_capacity = std::min<uint64_t>(N, H + 2 * feed_events + 2ull * reps + 400000);
    lx_index *h = nullptr;
    if (lx_create(&cfg, &h)) return fail("lx_create", nullptr);
    if (lx_reset(h, V, weights)) return fail("lx_reset", h);
    if (H && lx_add_batch(h, (uint32_t)H, d.creator.data(), d.seq.data(), d.poff.data(), d.par.data(), nullptr, nullptr))
        return fail("history", h);
    lx_flush(h);
    if (lx_sync(h)) return fail("sync", h);
    uint64_t next = H;   // next event (level order) to add
    uint64_t lv = L0;    // its level
    auto add = [&](uint64_t lo, uint64_t hi) {
        return lx_add_batch(h, (uint32_t)(hi - lo), d.creator.data() + lo, d.seq.data() + lo, d.poff.data() + lo,
                            d.par.data(), nullptr, nullptr);
    };
    std::vector<double> t[11];
    double first[11] = {0};
    // record call r of a kind: the first is one-time setup, the next kWarm - 1
    // are dropped, the rest timed
    auto rec = [&](int kind, uint32_t r, double us) {
        if (r == 0) first[kind] = us;
        if (r >= kWarm) t[kind].push_back(us);
    };
    // 0/1: single events, Process pattern (async; then with completion)
    for (int mode = 0; mode < 2; mode++) {
        for (uint32_t r = 0; r < reps + kWarm && next < N; r++, next++) {
            auto t0 = clk::now();
            if (add(next, next + 1)) return fail("add1", h);
            lx_flush(h);
            if (mode == 1 && lx_sync(h)) return fail("sync", h);
            rec(mode, r, us_since(t0));
        }
        if (lx_sync(h)) return fail("sync", h);
    }
    while (lv + 1 < d.lvl_off.size() && d.lvl_off[lv + 1] <= next) lv++;
    // 2: Build pattern on the next event, repeated (each Build is rolled back)
    for (uint32_t r = 0; r < reps + kWarm; r++) {
        auto t0 = clk::now();
        if (add(next, next + 1)) return fail("build", h);
        if (lx_drop_not_flushed(h)) return fail("drop", h);
        if (lx_sync(h)) return fail("sync", h);
        rec(2, r, us_since(t0));
    }
    // 3: antichains: finish the current level, then whole levels
    if (next < d.lvl_off[lv + 1]) {
        if (add(next, d.lvl_off[lv + 1])) return fail("level", h);
        lx_flush(h);
        next = d.lvl_off[++lv];
    }
    const uint32_t lreps = std::max<uint32_t>(reps / 4, 50);
    for (uint32_t r = 0; r < lreps + kWarm && lv + 1 < d.lvl_off.size(); r++, lv++) {
        auto t0 = clk::now();
        if (add(d.lvl_off[lv], d.lvl_off[lv + 1])) return fail("level", h);
        lx_flush(h);
        if (lx_sync(h)) return fail("sync", h);
        rec(3, r, us_since(t0));
        next = d.lvl_off[lv + 1];
    }
    // 4: 1024-event batches (continuing in level order); the add call and the
    // sync timed apart too
    std::vector<double> t4a, t4s;
    for (uint32_t r = 0; r < std::max<uint32_t>(reps / 10, 200) + kWarm && next + 1024 <= N; r++) {
        auto t0 = clk::now();
        if (add(next, next + 1024)) return fail("add1024", h);
        lx_flush(h);
        const double ta = us_since(t0);
        if (lx_sync(h)) return fail("sync", h);
        const double tt = us_since(t0);
        rec(4, r, tt);
        if (r >= kWarm) {
            t4a.push_back(ta);
            t4s.push_back(tt - ta);
        }
        next += 1024;
    }
    {
        Stat a = stat_of(t4a), b = stat_of(t4s);
        out[96] = a.p50; out[97] = a.p99; out[98] = b.p50; out[99] = b.p99;
    }
    while (lv + 1 < d.lvl_off.size() && d.lvl_off[lv + 1] <= next) lv++;
    if (next < d.lvl_off[lv + 1] && lv + 1 < d.lvl_off.size()) {   // realign to a level boundary
        if (add(next, d.lvl_off[lv + 1])) return fail("level", h);
        lx_flush(h);
        next = d.lvl_off[++lv];
    }
    // 5-10: queries over the indexed events (a among the newest, b anywhere older)
    uint64_t rs = 0x9E3779B97F4A7C15ull;
    auto rnd = [&](uint64_t m) {
        rs ^= rs << 13;
        rs ^= rs >> 7;
        rs ^= rs << 17;
        return rs % m;
    };
    std::vector<uint32_t> qa(667), qb(667);
    std::vector<uint8_t> qo(667);
    for (int kind = 5; kind <= 6; kind++) {
        const uint32_t n = kind == 5 ? 1 : 667;
        for (uint32_t r = 0; r < reps + kWarm; r++) {
            for (uint32_t i = 0; i < n; i++) {
                qa[i] = (uint32_t)(next - 1 - rnd(std::min<uint64_t>(next, 5000)));
                qb[i] = (uint32_t)rnd(next);
            }
            auto t0 = clk::now();
            if (lx_forkless_cause_batch(h, n, qa.data(), qb.data(), qo.data())) return fail("fc", h);
            rec(kind, r, us_since(t0));
        }
    }
    std::vector<uint8_t> row(16 * (V + 4096));
    for (int kind = 7; kind <= 9; kind++) {
        for (uint32_t r = 0; r < reps + kWarm; r++) {
            const uint32_t ev = (uint32_t)(next - 1 - rnd(std::min<uint64_t>(next, 5000)));
            uint32_t len = 0;
            auto t0 = clk::now();
            int rc = kind == 7   ? lx_get_highest_before(h, ev, row.data(), (uint32_t)row.size(), &len)
                     : kind == 8 ? lx_get_lowest_after(h, ev, row.data(), (uint32_t)row.size(), &len)
                                 : lx_get_merged_highest_before(h, ev, row.data(), (uint32_t)row.size(), &len);
            if (rc) return fail("getter", h);
            rec(kind, r, us_since(t0));
        }
    }
    {
        std::vector<uint32_t> evs(64);
        std::vector<uint64_t> off(65);
        std::vector<uint8_t> buf(64ull * 8 * V);
        for (uint32_t r = 0; r < reps / 4 + 1 + kWarm; r++) {
            for (auto &e : evs) e = (uint32_t)(next - 1 - rnd(std::min<uint64_t>(next, 5000)));
            auto t0 = clk::now();
            if (lx_get_merged_highest_before_batch(h, 64, evs.data(), off.data(), buf.data(), buf.size()))
                return fail("getter batch", h);
            rec(10, r, us_since(t0));
        }
    }
    // ForklessCause of one pair through lx_forkless_cause (the drop-in path), as
    // calcFrameIdx asks it: each new event against a fixed set of 8 roots (the
    // events just before the loop).  The new event's first question fills its
    // row of the result cache (a miss: the pending Add and one row launch,
    // waited for); its questions about the other roots are hits.
    {
        std::vector<double> tm, th;
        uint8_t o = 0;
        uint32_t roots[8];
        for (int k = 0; k < 8; k++) roots[k] = (uint32_t)(next - 1 - k);
        for (uint32_t r = 0; r < reps && next < N; r++, next++) {
            if (add(next, next + 1)) return fail("add (fc)", h);
            lx_flush(h);
            const uint32_t a = (uint32_t)next;
            auto t0 = clk::now();
            if (lx_forkless_cause(h, a, roots[0], &o)) return fail("fc pair", h);
            if (r) tm.push_back(us_since(t0));   // the first one also brings the roots in
            for (int k = 1; k < 8; k++) {
                auto t1 = clk::now();
                if (lx_forkless_cause(h, a, roots[k], &o)) return fail("fc pair", h);
                if (r) th.push_back(us_since(t1));
            }
        }
        Stat sm = stat_of(tm), sh = stat_of(th);
        out[40] = sm.p50; out[41] = sm.p99; out[42] = sm.mean;
        out[43] = sh.p50; out[44] = sh.p99; out[45] = sh.mean;
        while (lv + 1 < d.lvl_off.size() && d.lvl_off[lv + 1] <= next) lv++;
        if (next < d.lvl_off[lv + 1] && lv + 1 < d.lvl_off.size()) {   // realign to a level boundary
            if (add(next, d.lvl_off[lv + 1])) return fail("level", h);
            lx_flush(h);
            next = d.lvl_off[++lv];
        }
    }
    for (int k = 0; k < 11; k++) {
        Stat s = stat_of(t[k]);
        out[3 * k] = s.p50;
        out[3 * k + 1] = s.p99;
        out[3 * k + 2] = s.mean;
        out[48 + 4 * k] = s.p999;
        out[48 + 4 * k + 1] = s.max;
        out[48 + 4 * k + 2] = first[k];
        out[48 + 4 * k + 3] = (double)t[k].size();
    }
    // antichain-fed throughput: levels as batches, Add + Flush each, one sync at the end
    {
        const uint64_t lv0 = lv, e0 = next;
        auto t0 = clk::now();
        while (lv + 1 < d.lvl_off.size() && d.lvl_off[lv + 1] - e0 <= feed_events) {
            if (add(d.lvl_off[lv], d.lvl_off[lv + 1])) return fail("feed", h);
            lx_flush(h);
            lv++;
        }
        if (lx_sync(h)) return fail("sync", h);
        const double s = us_since(t0) * 1e-6;
        next = d.lvl_off[lv];
        out[33] = (next - e0) / s;
        out[34] = (double)(next - e0);
        out[35] = (double)(lv - lv0);
        out[37] = (double)(next - e0) / std::max<double>(1, lv - lv0);
    }
    // batcher-fed: each level pushed by id, popped (parents-first release) and added
    {
        lx_batcher *b = nullptr;
        if (lx_batcher_create(&b) || lx_batcher_reserve(b, N)) return fail("batcher", h);
        // the batcher's dense indices must continue the epoch: replay the indexed
        // prefix as released events (pushed and popped without adding)
        std::vector<uint64_t> ids, pids, po;
        auto push_range = [&](uint64_t lo, uint64_t hi) {
            ids.resize(hi - lo);
            po.assign(1, 0);
            pids.clear();
            for (uint64_t i = lo; i < hi; i++) {
                ids[i - lo] = i + 1;
                for (uint64_t k = d.poff[i]; k < d.poff[i + 1]; k++) pids.push_back((uint64_t)d.par[k] + 1);
                po.push_back(pids.size());
            }
            return lx_batcher_push(b, (uint32_t)(hi - lo), ids.data(), d.creator.data() + lo, d.seq.data() + lo,
                                   po.data(), pids.data(), nullptr);
        };
        std::vector<uint64_t> oid, opo;
        std::vector<uint32_t> ocr, osq, opar, olv;
        auto pop = [&](uint32_t *n_out) {
            uint32_t ne = 0, nl = 0, nw = 0;
            uint64_t npar = 0;
            if (lx_batcher_peek(b, &ne, &npar, &nl, &nw)) return -1;
            oid.resize(ne + 1);
            ocr.resize(ne + 1);
            osq.resize(ne + 1);
            opo.resize(ne + 1);
            opar.resize(npar + 1);
            olv.resize(nl + 1);
            *n_out = ne;
            return lx_batcher_pop(b, oid.data(), ocr.data(), osq.data(), opo.data(), opar.data(), olv.data(), nullptr);
        };
        uint32_t ne = 0;
        if (push_range(0, next) || pop(&ne) || ne != next) {
            lx_batcher_destroy(b);
            return fail("batcher replay", h);
        }
        const uint64_t lv0 = lv, e0 = next;
        auto t0 = clk::now();
        while (lv + 1 < d.lvl_off.size() && d.lvl_off[lv + 1] - e0 <= feed_events) {
            if (push_range(d.lvl_off[lv], d.lvl_off[lv + 1]) || pop(&ne)) {
                lx_batcher_destroy(b);
                return fail("batcher feed", h);
            }
            if (ne && lx_add_batch(h, ne, ocr.data(), osq.data(), opo.data(), opar.data(), nullptr, nullptr)) {
                lx_batcher_destroy(b);
                return fail("batcher add", h);
            }
            lx_flush(h);
            lv++;
        }
        if (lx_sync(h)) {
            lx_batcher_destroy(b);
            return fail("sync", h);
        }
        const double s = us_since(t0) * 1e-6;
        out[36] = (d.lvl_off[lv] - e0) / s;
        lx_batcher_destroy(b);
    }
    lx_destroy(h);
    (void)lv;
    return 0;
}

}  // extern "C"

extern "C" {

// Events/s of adding the DAG (its own Add order) in batches of `batch` events
// through lx_add_batch + lx_flush (batch 1 = the reference's per-event Add of
// IndexedLachesis.Process), one lx_sync at the end.  out[0] events/s, out[1]
// seconds.
int lx_bench_feed(int device, uint32_t V, const uint32_t *weights, uint64_t N, const uint32_t *creator,
                  const uint32_t *seq, const uint64_t *poff, const uint32_t *par, uint32_t batch, double *out,
                  char *err, uint32_t err_cap) {
    lx_config cfg{};
    cfg.device = device;
    cfg.event_capacity = N;
    lx_index *h = nullptr;
    if (lx_create(&cfg, &h) || lx_reset(h, V, weights)) {
        snprintf(err, err_cap, "create/reset: %s", h ? lx_last_error(h) : "");
        if (h) lx_destroy(h);
        return -1;
    }
    batch = std::max<uint32_t>(batch, 1);
    auto t0 = clk::now();
    for (uint64_t lo = 0; lo < N; lo += batch) {
        const uint64_t hi = std::min<uint64_t>(N, lo + batch);
        if (lx_add_batch(h, (uint32_t)(hi - lo), creator + lo, seq + lo, poff + lo, par, nullptr, nullptr)) {
            snprintf(err, err_cap, "add: %s", lx_last_error(h));
            lx_destroy(h);
            return -1;
        }
        lx_flush(h);
    }
    const double s_host = us_since(t0) * 1e-6;
    if (lx_sync(h)) {
        snprintf(err, err_cap, "sync: %s", lx_last_error(h));
        lx_destroy(h);
        return -1;
    }
    const double s = us_since(t0) * 1e-6;
    out[0] = N / s;
    out[1] = s;
    out[2] = s_host;       // the Add / Flush calls alone
    out[3] = s - s_host;   // the final lx_sync (device work left when the last call returned)
    lx_destroy(h);
    return 0;
}

}  // extern "C"

extern "C" {

// Level-fed throughput alone (for profiling): the DAG re-ordered by level,
// `history` events added in one batch, 100 levels fed untimed, then levels fed one lx_add_batch +
// lx_flush each (mode 0) or pushed / popped through lx_batcher (mode 1) for
// up to feed_events events, one lx_sync at the end.  out[0] events/s, [1]
// events, [2] levels, [3] seconds in lx_add_batch, [4] seconds in the batcher,
// [5] seconds in the final lx_sync.
int lx_bench_feed_levels(int device, uint32_t V, const uint32_t *weights, uint64_t N, const uint32_t *creator,
                         const uint32_t *seq, const uint64_t *poff, const uint32_t *par, uint64_t history,
                         uint64_t feed_events, int mode, double *out, char *err, uint32_t err_cap) {
    Leveled d = by_level(N, creator, seq, poff, par);
    uint64_t L0 = 0;
    while (L0 + 1 < d.lvl_off.size() && d.lvl_off[L0 + 1] <= history) L0++;
    const uint64_t H = d.lvl_off[L0];
    lx_config cfg{};
    cfg.device = device;
    cfg.event_capacity = std::min<uint64_t>(N, H + feed_events + 100000);
    lx_index *h = nullptr;
    auto fail = [&](const char *what) {
        snprintf(err, err_cap, "%s: %s", what, h ? lx_last_error(h) : "");
        if (h) lx_destroy(h);
        return -1;
    };
    if (lx_create(&cfg, &h) || lx_reset(h, V, weights)) return fail("create");
    if (H && lx_add_batch(h, (uint32_t)H, d.creator.data(), d.seq.data(), d.poff.data(), d.par.data(), nullptr, nullptr))
        return fail("history");
    lx_flush(h);
    if (lx_sync(h)) return fail("sync");
    lx_batcher *b = nullptr;
    std::vector<uint64_t> ids, pids, po, oid, opo;
    std::vector<uint32_t> ocr, osq, opar, olv;
    if (mode == 1) {
        if (lx_batcher_create(&b) || lx_batcher_reserve(b, N)) return fail("batcher");
        // the batcher's dense indices continue the epoch: the history as released events
        ids.resize(H);
        po.assign(1, 0);
        for (uint64_t i = 0; i < H; i++) {
            ids[i] = i + 1;
            for (uint64_t k = d.poff[i]; k < d.poff[i + 1]; k++) pids.push_back((uint64_t)d.par[k] + 1);
            po.push_back(pids.size());
        }
        uint32_t ne = 0, nl = 0, nw = 0;
        uint64_t np = 0;
        if (H) {
            if (lx_batcher_push(b, (uint32_t)H, ids.data(), d.creator.data(), d.seq.data(), po.data(), pids.data(), nullptr) ||
                lx_batcher_peek(b, &ne, &np, &nl, &nw))
                return fail("batcher history");
            oid.resize(ne + 1); ocr.resize(ne + 1); osq.resize(ne + 1); opo.resize(ne + 1);
            opar.resize(np + 1); olv.resize(nl + 1);
            if (lx_batcher_pop(b, oid.data(), ocr.data(), osq.data(), opo.data(), opar.data(), olv.data(), nullptr))
                return fail("batcher history pop");
        }
    }
    std::vector<uint64_t> lv_ids, lv_po, lv_pids;
    uint64_t lv = L0;
    uint64_t e0 = H;
    double t_add = 0, t_bat = 0;
    auto t0 = clk::now();
    const uint64_t warm = 100;   // levels fed untimed first (kernel code objects, allocations)
    for (uint64_t round = 0; round < 2; round++) {
    if (round == 1) {
        if (lx_sync(h)) return fail("sync");
        e0 = d.lvl_off[lv];
        t_add = t_bat = 0;
        t0 = clk::now();
    }
    const uint64_t lv_end = round == 0 ? std::min<uint64_t>(lv + warm, d.lvl_off.size() - 1) : d.lvl_off.size() - 1;
    while (lv < lv_end && d.lvl_off[lv + 1] - e0 <= feed_events) {
        const uint64_t lo = d.lvl_off[lv], hi = d.lvl_off[lv + 1];
        if (mode == 0) {
            auto a0 = clk::now();
            if (lx_add_batch(h, (uint32_t)(hi - lo), d.creator.data() + lo, d.seq.data() + lo, d.poff.data() + lo,
                             d.par.data(), nullptr, nullptr))
                return fail("feed");
            lx_flush(h);
            t_add += us_since(a0) * 1e-6;
        } else {
            lv_ids.resize(hi - lo);
            lv_po.assign(1, 0);
            lv_pids.clear();
            for (uint64_t i = lo; i < hi; i++) {
                lv_ids[i - lo] = i + 1;
                for (uint64_t k = d.poff[i]; k < d.poff[i + 1]; k++) lv_pids.push_back((uint64_t)d.par[k] + 1);
                lv_po.push_back(lv_pids.size());
            }
            auto a0 = clk::now();
            uint32_t ne = 0, nl = 0, nw = 0;
            uint64_t np = 0;
            if (lx_batcher_push(b, (uint32_t)(hi - lo), lv_ids.data(), d.creator.data() + lo, d.seq.data() + lo,
                                lv_po.data(), lv_pids.data(), nullptr) ||
                lx_batcher_peek(b, &ne, &np, &nl, &nw))
                return fail("batcher push");
            if (oid.size() < ne + 1) { oid.resize(ne + 1); ocr.resize(ne + 1); osq.resize(ne + 1); opo.resize(ne + 1); }
            if (opar.size() < np + 1) opar.resize(np + 1);
            if (olv.size() < nl + 1) olv.resize(nl + 1);
            if (lx_batcher_pop(b, oid.data(), ocr.data(), osq.data(), opo.data(), opar.data(), olv.data(), nullptr))
                return fail("batcher pop");
            auto a1 = clk::now();
            if (ne && lx_add_batch(h, ne, ocr.data(), osq.data(), opo.data(), opar.data(), nullptr, nullptr))
                return fail("batcher add");
            lx_flush(h);
            auto a2 = clk::now();
            t_bat += std::chrono::duration<double>(a1 - a0).count();
            t_add += std::chrono::duration<double>(a2 - a1).count();
        }
        lv++;
    }
    }
    auto ts = clk::now();
    if (lx_sync(h)) return fail("sync");
    const double s = us_since(t0) * 1e-6;
    out[0] = (d.lvl_off[lv] - e0) / s;
    out[1] = (double)(d.lvl_off[lv] - e0);
    out[2] = (double)(lv - L0);
    out[3] = t_add;
    out[4] = t_bat;
    out[5] = us_since(ts) * 1e-6;
    if (b) lx_batcher_destroy(b);
    lx_destroy(h);
    return 0;
}

}  // extern "C"

extern "C" {

// The emitter's QuorumIndexer (emitter/ancestor/quorum_indexer.go:86-136) on
// the index, per call as the emitter uses it: the first `history` events
// indexed, then for each of `reps` next events Add + ProcessEvent of that one
// event (lx_qi_process_events n = 1; every event reaches the emitter), and
// every `every`-th event GetMetricOf for `cands` candidate parents (the newest
// event of `cands` validators; lx_qi_metric_of, the medians recomputed lazily
// after the updates as recacheState does).  Validator 0 is the emitter (its
// events are self events).  out[0..2] ProcessEvent p50 / p99 / mean us, [3..5]
// metric batch p50 / p99 / mean us, [6] candidates in the last batch, whose
// metrics land in last_metrics[cands] (the bench checks them on the CPU port).
int lx_bench_qi(int device, uint32_t V, const uint32_t *weights, uint64_t N, const uint32_t *creator,
                const uint32_t *seq, const uint64_t *poff, const uint32_t *par, uint64_t history, uint32_t reps,
                uint32_t every, uint32_t cands, double *out, uint64_t *last_metrics, char *err,
                uint32_t err_cap) {
    lx_config cfg{};
    cfg.device = device;
    cfg.event_capacity = N;
    lx_index *h = nullptr;
    lx_qi *q = nullptr;
    auto fail = [&](const char *what) {
        snprintf(err, err_cap, "%s: %s", what, q ? lx_qi_last_error(q) : h ? lx_last_error(h) : "");
        if (q) lx_qi_destroy(q);
        if (h) lx_destroy(h);
        return -1;
    };
    if (lx_create(&cfg, &h) || lx_reset(h, V, weights)) return fail("create");
    if (lx_add_batch(h, (uint32_t)history, creator, seq, poff, par, nullptr, nullptr)) return fail("history");
    lx_flush(h);
    if (lx_qi_create(h, &q)) return fail("qi create");
    {   // the emitter has seen the history (one batched call)
        std::vector<uint32_t> ev(history);
        std::vector<uint8_t> self(history);
        for (uint64_t i = 0; i < history; i++) ev[i] = (uint32_t)i, self[i] = creator[i] == 0;
        if (lx_qi_process_events(q, (uint32_t)history, ev.data(), self.data())) return fail("qi history");
    }
    std::vector<int64_t> last(V, -1);
    for (uint64_t i = 0; i < history; i++) last[creator[i]] = (int64_t)i;
    std::vector<double> tp, tm;
    std::vector<uint32_t> cv;
    std::vector<uint64_t> mo(cands);
    for (uint32_t r = 0; r < reps && history + r < N; r++) {
        const uint64_t e = history + r;
        if (lx_add_batch(h, 1, creator + e, seq + e, poff + e, par, nullptr, nullptr)) return fail("add");
        lx_flush(h);
        last[creator[e]] = (int64_t)e;
        const uint32_t ev = (uint32_t)e;
        const uint8_t self = creator[e] == 0 ? 1 : 0;   // validator 0 is the emitter
        auto t0 = clk::now();
        if (lx_qi_process_events(q, 1, &ev, &self)) return fail("process event");
        tp.push_back(us_since(t0));
        if (every && r % every == every - 1) {
            cv.clear();
            for (uint32_t c = 0; c < V && cv.size() < cands; c++)
                if (last[c] >= 0) cv.push_back((uint32_t)last[c]);
            auto t1 = clk::now();
            if (lx_qi_metric_of(q, (uint32_t)cv.size(), cv.data(), 2, mo.data())) return fail("metric");
            tm.push_back(us_since(t1));
            std::copy(mo.begin(), mo.begin() + cv.size(), last_metrics);
            out[6] = (double)cv.size();
        }
    }
    Stat a = stat_of(tp), b = stat_of(tm);
    if (tm.empty()) out[6] = 0;
    out[0] = a.p50; out[1] = a.p99; out[2] = a.mean;
    out[3] = b.p50; out[4] = b.p99; out[5] = b.mean;
    lx_qi_destroy(q);
    lx_destroy(h);
    return 0;
}

}  // extern "C"
