// rowseg_fake.cpp -- GPU test harness of the row-segment exchange driver
// (lachesis-base_amd/csrc/lx_rowseg_exchange.h, the code lx_rowseg_exchange
// runs over RCCL): G row-segment handles of one GPU, one thread per rank, the
// library's rowseg ABI as the ops and an in-process transport as the
// collectives (device-to-device copies between the ranks' buffers, barriers).
// RCCL refuses two ranks on one device, so this is how the native multi-rank
// schedule runs on the 1-GPU box.  Test infrastructure only
// (tests/test_gpu_rowseg_native.py).
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../lachesis-base_amd/csrc/lx_rowseg_exchange.h"

namespace {

struct World {
    uint32_t G;
    std::mutex m;
    std::condition_variable cv;
    uint32_t arrived = 0, gen = 0;
    std::vector<uint64_t> val;                       // sum: per rank
    std::vector<std::vector<uint64_t>> cnt;          // counts: [src][dst]
    std::vector<const uint8_t *> sendp;
    std::vector<std::vector<uint64_t>> sb;           // move: [src][dst] bytes
    std::string err;
    explicit World(uint32_t g) : G(g), val(g), cnt(g, std::vector<uint64_t>(g)), sendp(g), sb(g, std::vector<uint64_t>(g)) {}
    bool broken = false;   // a rank left the protocol: every barrier returns at once
    bool barrier() {   // false: the protocol is broken, every rank must stop
        std::unique_lock<std::mutex> l(m);
        if (broken) return false;
        const uint32_t my = gen;
        if (++arrived == G) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else if (!cv.wait_for(l, std::chrono::seconds(60), [&] { return gen != my || broken; })) {
            broken = true;
            if (err.empty()) err = "barrier timeout (a rank left the exchange)";
            cv.notify_all();
        }
        return !broken;
    }
    void fail(const std::string &e) {
        std::lock_guard<std::mutex> l(m);
        if (err.empty()) err = e;
    }
};

struct Ops {
    lx_index *h;
    void *bufs[lx::kRsBufs] = {};
    size_t caps[lx::kRsBufs] = {};
    ~Ops() {
        for (void *p : bufs) (void)hipFree(p);
    }
    int row_words(uint32_t *w) { return lx_rowseg_row_words(h, w); }
    int request_cap(uint32_t *c) { return lx_rowseg_request_cap(h, c); }
    int requests(uint32_t *ids, uint32_t cap, uint32_t *counts) { return lx_rowseg_requests(h, ids, cap, counts); }
    int serve(uint32_t n, const uint32_t *ids, uint32_t *rows, uint32_t *ready) { return lx_rowseg_serve(h, n, ids, rows, ready); }
    int receive(uint32_t n, const uint32_t *ids, const uint32_t *rows, const uint32_t *ready) {
        return lx_rowseg_receive(h, n, ids, rows, ready, nullptr);
    }
    int la(uint64_t *counts) { return lx_rowseg_la(h, counts); }
    int la_fetch(uint32_t *buf) { return lx_rowseg_la_fetch(h, buf); }
    int la_apply(uint64_t n, const uint32_t *buf) { return lx_rowseg_la_apply(h, n, buf); }
    int finish() { return lx_rowseg_finish(h); }
    // ForklessCause across ranks (rowseg_fc_run)
    uint32_t r = 0;
    uint32_t rank() const { return r; }
    int fc_route(uint64_t n, const uint32_t *qa, const uint32_t *qb, uint32_t *ra, uint32_t *rb, uint32_t *perm,
                 uint64_t *counts) {
        return lx_rowseg_fc_route(h, n, qa, qb, ra, rb, perm, counts);
    }
    int fc_need(uint64_t m, const uint32_t *ra, const uint32_t *rb, uint32_t *ids, uint64_t cap, uint64_t *counts) {
        return lx_rowseg_fc_need(h, m, ra, rb, ids, cap, counts);
    }
    int la_serve(uint64_t n, const uint32_t *ids, uint32_t *rows) { return lx_rowseg_la_serve(h, n, ids, rows); }
    int la_store(uint64_t n, const uint32_t *ids, const uint32_t *rows) { return lx_rowseg_la_store(h, n, ids, rows); }
    int fc_pairs(uint64_t m, const uint32_t *a, const uint32_t *b, uint8_t *ans) {
        int rc = lx_forkless_cause_batch_dev(h, m, a, b, ans, nullptr);
        return rc ? rc : lx_sync(h);
    }
    int fc_unroute(uint64_t n, const uint32_t *perm, const uint8_t *ans, uint8_t *out) {
        return lx_rowseg_fc_unroute(h, n, perm, ans, out);
    }
    int get_rows(uint32_t mode, uint64_t m, const uint32_t *ids, uint8_t *rows, uint64_t slot, uint32_t *lens) {
        return lx_get_rows_dev(h, mode, (uint32_t)m, ids, rows, slot, lens);
    }
    int rows_unroute(uint64_t n, const uint32_t *perm, const uint8_t *rows, uint64_t slot, const uint32_t *lens,
                     uint8_t *out, uint32_t *out_len) {
        return lx_rowseg_rows_unroute(h, n, perm, rows, slot, lens, out, out_len);
    }
    void *buf(int k, size_t bytes) {
        if (bytes > caps[k]) {
            (void)hipFree(bufs[k]);
            bufs[k] = nullptr;
            caps[k] = 0;
            if (hipMalloc(&bufs[k], bytes) != hipSuccess) return nullptr;
            caps[k] = bytes;
        }
        return bufs[k];
    }
};

struct Net {
    World &w;
    uint32_t r;
    int sum(uint64_t x, uint64_t *all) {
        w.val[r] = x;
        if (!w.barrier()) return LX_ERR_STATE;
        uint64_t s = 0;
        for (uint64_t v : w.val) s += v;
        *all = s;
        return w.barrier() ? 0 : LX_ERR_STATE;
    }
    int counts(const uint64_t *send, uint64_t *recv) {
        for (uint32_t q = 0; q < w.G; q++) w.cnt[r][q] = send[q];
        if (!w.barrier()) return LX_ERR_STATE;
        for (uint32_t p = 0; p < w.G; p++) recv[p] = w.cnt[p][r];
        return w.barrier() ? 0 : LX_ERR_STATE;
    }
    int move(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb) {
        w.sendp[r] = static_cast<const uint8_t *>(send);
        for (uint32_t q = 0; q < w.G; q++) w.sb[r][q] = sb[q];
        if (!w.barrier()) return LX_ERR_STATE;
        int rc = 0;
        uint64_t ro = 0;
        for (uint32_t p = 0; p < w.G && !rc; p++) {
            uint64_t so = 0;
            for (uint32_t q = 0; q < r; q++) so += w.sb[p][q];
            if (w.sb[p][r] != rb[p]) {
                w.fail("block " + std::to_string(p) + " -> " + std::to_string(r) + ": " + std::to_string(w.sb[p][r]) +
                       " bytes sent, " + std::to_string(rb[p]) + " expected");
                rc = LX_ERR_STATE;
            } else if (rb[p] && hipMemcpy(static_cast<uint8_t *>(recv) + ro, w.sendp[p] + so, rb[p],
                                          hipMemcpyDeviceToDevice) != hipSuccess) {
                w.fail("hipMemcpy");
                rc = LX_ERR_HIP;
            }
            ro += rb[p];
        }
        // a device-to-device hipMemcpy may return before the copy is done, and
        // the handles' streams do not wait for the null stream
        if (!rc && hipDeviceSynchronize() != hipSuccess) {
            w.fail("hipDeviceSynchronize");
            rc = LX_ERR_HIP;
        }
        if (!w.barrier()) return LX_ERR_STATE;   // every copy done before a sender reuses its buffer
        return rc;
    }
};

}  // namespace

extern "C" int lx_fake_rowseg_exchange(void **handles, uint32_t G, uint64_t *stats, char *err, uint32_t err_cap) {
    World w(G);
    std::vector<int> rcs(G, 0);
    std::vector<std::thread> th;
    for (uint32_t r = 0; r < G; r++)
        th.emplace_back([&, r] {
            (void)hipSetDevice(0);
            Ops ops{static_cast<lx_index *>(handles[r])};
            Net net{w, r};
            lx::RowsegExchangeStats st;
            rcs[r] = lx::rowseg_exchange_run(ops, net, G, st);
            if (rcs[r]) {
                w.fail("rank " + std::to_string(r) + ": " + lx_last_error(ops.h));
                std::lock_guard<std::mutex> l(w.m);
                w.broken = true;
                w.cv.notify_all();
            }
            stats[4 * r] = st.rounds;
            stats[4 * r + 1] = st.rows_received;
            stats[4 * r + 2] = st.la_sent;
            stats[4 * r + 3] = st.la_received;
        });
    for (auto &t : th) t.join();
    snprintf(err, err_cap, "%s", w.err.c_str());
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

// ForklessCause across ranks: rank r asks its n[r] queries (device arrays),
// stats[4 r ..] = routed away, answered, LA rows received, sent
extern "C" int lx_fake_rowseg_fc(void **handles, uint32_t G, const uint64_t *n, void **qa, void **qb, void **out,
                                 uint64_t *stats, char *err, uint32_t err_cap) {
    World w(G);
    std::vector<int> rcs(G, 0);
    std::vector<std::thread> th;
    for (uint32_t r = 0; r < G; r++)
        th.emplace_back([&, r] {
            (void)hipSetDevice(0);
            Ops ops{static_cast<lx_index *>(handles[r])};
            ops.r = r;
            Net net{w, r};
            lx::RowsegFcStats st;
            rcs[r] = lx::rowseg_fc_run(ops, net, G, n[r], static_cast<const uint32_t *>(qa[r]),
                                       static_cast<const uint32_t *>(qb[r]), static_cast<uint8_t *>(out[r]), st);
            if (rcs[r]) {
                w.fail("rank " + std::to_string(r) + ": " + lx_last_error(ops.h));
                std::lock_guard<std::mutex> l(w.m);
                w.broken = true;
                w.cv.notify_all();
            }
            stats[4 * r] = st.routed_away;
            stats[4 * r + 1] = st.answered;
            stats[4 * r + 2] = st.rows_received;
            stats[4 * r + 3] = st.rows_sent;
        });
    for (auto &t : th) t.join();
    snprintf(err, err_cap, "%s", w.err.c_str());
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

// the vector getters across ranks: rank r asks for the rows of its n[r] device
// ids (mode 0 HighestBefore, 1 LowestAfter, 2 merged HighestBefore)
extern "C" int lx_fake_rowseg_get_rows(void **handles, uint32_t G, uint32_t mode, const uint64_t *n, void **ev,
                                       void **out, uint64_t slot, void **len, char *err, uint32_t err_cap) {
    World w(G);
    std::vector<int> rcs(G, 0);
    std::vector<std::thread> th;
    for (uint32_t r = 0; r < G; r++)
        th.emplace_back([&, r] {
            (void)hipSetDevice(0);
            Ops ops{static_cast<lx_index *>(handles[r])};
            ops.r = r;
            Net net{w, r};
            rcs[r] = lx::rowseg_get_run(ops, net, G, mode, n[r], static_cast<const uint32_t *>(ev[r]),
                                        static_cast<uint8_t *>(out[r]), slot, static_cast<uint32_t *>(len[r]));
            if (rcs[r]) {
                w.fail("rank " + std::to_string(r) + ": " + lx_last_error(ops.h));
                std::lock_guard<std::mutex> l(w.m);
                w.broken = true;
                w.cv.notify_all();
            }
        });
    for (auto &t : th) t.join();
    snprintf(err, err_cap, "%s", w.err.c_str());
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}
