// shard_fake.cpp -- CPU test harness for the column-shard LowestAfter exchange
// driver (lachesis-base_amd/csrc/lx_shard_exchange.h, the code lx_shard_exchange
// runs over RCCL): G ranks as threads, an in-process transport, and a numpy-free
// model of each rank's index (rows of its branches x everyone's columns).
// Checks after every exchange that each rank holds exactly the LowestAfter
// entries of its columns for every row, that every block sits at a 4-byte
// aligned offset on both sides, and that the byte wire / fallback / retry
// schedule is followed.  Test infrastructure only (tests/test_shard_exchange_cpu.py).
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../lachesis-base_amd/csrc/lx_shard_exchange.h"

namespace {

struct Truth {
    uint32_t N = 0, V = 0, G = 0;
    std::vector<uint32_t> owner;            // rank owning row i (its branch's creator range)
    std::vector<uint32_t> seq;              // row i's own seq
    std::vector<uint32_t> la;               // N x V
    std::vector<std::vector<uint32_t>> rows, cols;
    uint32_t width() const {                // lx_shard_wire: 2 while every value < 2^16
        for (uint32_t v : la)
            if (v > 0xFFFF) return 4;
        for (uint32_t s : seq)
            if (s > 0xFFFF) return 4;
        return 2;
    }
};

struct World {
    uint32_t G;
    std::mutex m;
    std::condition_variable cv;
    uint32_t arrived = 0, gen = 0;
    std::vector<std::vector<uint32_t>> W;   // W[src][dst] announced widths
    std::vector<const uint8_t *> sendp;
    std::vector<const uint64_t *> so, sb;
    std::string err;
    explicit World(uint32_t g) : G(g), W(g, std::vector<uint32_t>(g, 0)), sendp(g), so(g), sb(g) {}
    void barrier() {
        std::unique_lock<std::mutex> l(m);
        const uint32_t my = gen;
        if (++arrived == G) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != my; });
        }
    }
    void fail(const std::string &e) {
        std::lock_guard<std::mutex> l(m);
        if (err.empty()) err = e;
    }
};

struct FakeNet {
    World *w;
    uint32_t r;
    int widths(const uint32_t *sw, uint32_t *rw) {
        for (uint32_t q = 0; q < w->G; q++) w->W[r][q] = sw[q];
        w->barrier();
        for (uint32_t q = 0; q < w->G; q++) rw[q] = w->W[q][r];
        w->barrier();
        return 0;
    }
    int min_u32(uint32_t *, uint32_t) { return 0; }
    int blocks(const uint8_t *send, const uint64_t *so, const uint64_t *sb, uint8_t *recv, const uint64_t *ro,
               const uint64_t *rb) {
        w->sendp[r] = send;
        w->so[r] = so;
        w->sb[r] = sb;
        w->barrier();
        int rc = 0;
        for (uint32_t q = 0; q < w->G; q++) {
            if (q == r) continue;
            if (so[q] % 4 || ro[q] % 4) {
                w->fail("block offset not 4-byte aligned");
                rc = LX_ERR_STATE;
            }
            if (w->sb[q][r] != rb[q]) {
                w->fail("block size mismatch " + std::to_string(q) + "->" + std::to_string(r));
                rc = LX_ERR_STATE;
                continue;
            }
            if (rb[q]) memcpy(recv + ro[q], w->sendp[q] + w->so[q][r], rb[q]);
        }
        w->barrier();
        return rc;
    }
};

struct FakeOps {
    const Truth *t;
    World *w;
    uint32_t r;
    std::vector<uint32_t> got;              // N x V: this rank's query plane (own columns filled)
    std::vector<uint8_t> sbuf, rbuf;
    uint32_t fallbacks = 0, byte_packs = 0;
    int block(uint32_t s, uint32_t d, uint64_t *n) {
        *n = (uint64_t)t->rows[s].size() * t->cols[d].size();
        return 0;
    }
    int wire(uint32_t *wb) {
        *wb = t->width();
        return 0;
    }
    int pack(uint32_t d, uint8_t *buf, uint32_t wd) {
        if ((uintptr_t)buf % (wd == 1 ? 1 : wd)) return LX_ERR_STATE;   // the unpack kernel reads aligned words
        uint64_t k = 0;
        for (uint32_t i : t->rows[r])
            for (uint32_t c : t->cols[d]) {
                const uint32_t v = t->la[(uint64_t)i * t->V + c], s = t->seq[i];
                if (wd == 1) {
                    if (v && (int64_t)v - (int64_t)s + 127 >= 255) {
                        fallbacks++;
                        return LX_ERR_WIRE;
                    }
                    buf[k++] = v ? (uint8_t)(v - s + 128) : 0;
                } else if (wd == 2) {
                    reinterpret_cast<uint16_t *>(buf)[k++] = (uint16_t)v;
                } else {
                    reinterpret_cast<uint32_t *>(buf)[k++] = v;
                }
            }
        if (wd == 1) byte_packs++;
        return 0;
    }
    int unpack(uint32_t s, const uint8_t *buf, uint32_t wd) {
        if ((uintptr_t)buf % (wd == 1 ? 1 : wd)) return LX_ERR_STATE;
        uint64_t k = 0;
        for (uint32_t i : t->rows[s])
            for (uint32_t c : t->cols[r]) {
                uint32_t v;
                if (wd == 1) {
                    const uint32_t b = buf[k++];
                    v = b ? b + t->seq[i] - 128 : 0;
                } else if (wd == 2) {
                    v = reinterpret_cast<const uint16_t *>(buf)[k++];
                } else {
                    v = reinterpret_cast<const uint32_t *>(buf)[k++];
                }
                got[(uint64_t)i * t->V + c] = v;
            }
        return 0;
    }
    int own() {
        for (uint32_t i : t->rows[r])
            for (uint32_t c : t->cols[r]) got[(uint64_t)i * t->V + c] = t->la[(uint64_t)i * t->V + c];
        return 0;
    }
    // no incremental exchange in the model: whole blocks every time
    int branches(uint32_t *nb) {
        *nb = 0;
        return 0;
    }
    int dirty(uint32_t, uint32_t *) { return 0; }
    int dirty_set(uint32_t, const uint32_t *) { return 0; }
    int commit() { return 0; }
    // aligned staging (the device buffers are 256-B aligned)
    uint8_t *send_buf(size_t n) {
        sbuf.assign(n + 256, 0);
        return sbuf.data() + (256 - (uintptr_t)sbuf.data() % 256) % 256;
    }
    uint8_t *recv_buf(size_t n) {
        rbuf.assign(n + 256, 0);
        return rbuf.data() + (256 - (uintptr_t)rbuf.data() % 256) % 256;
    }
};

// uneven creator ranges like lx_shard_range (multiples of 4 except the last)
uint32_t bound(uint32_t V, uint32_t G, uint32_t q) { return q >= G ? V : (uint32_t)((uint64_t)V * q / G) & ~3u; }

}  // namespace

extern "C" {

// G ranks, `rounds` exchanges over a drifting random epoch; returns 0 or -1
// with a message.  stats[0] = byte-wire misfits (fallbacks), stats[1] = byte
// packs, stats[2] = entries moved.
int lx_fake_shard_exchange(uint32_t G, uint32_t V, uint32_t N, uint64_t seed, uint32_t rounds, uint32_t skew,
                           uint64_t *stats, char *err, uint32_t cap) {
    std::mt19937_64 rng(seed);
    Truth t;
    t.N = N;
    t.V = V;
    t.G = G;
    t.cols.resize(G);
    t.rows.resize(G);
    for (uint32_t q = 0; q < G; q++)
        for (uint32_t c = bound(V, G, q); c < bound(V, G, q + 1); c++) t.cols[q].push_back(c);
    t.owner.resize(N);
    t.seq.resize(N);
    t.la.assign((uint64_t)N * V, 0);
    for (uint32_t i = 0; i < N; i++) {
        const uint32_t c = (uint32_t)(rng() % V);   // the row's branch creator
        uint32_t q = 0;
        while (!(c >= bound(V, G, q) && c < bound(V, G, q + 1))) q++;
        t.owner[i] = q;
        t.rows[q].push_back(i);
        t.seq[i] = 1 + (uint32_t)(rng() % 5000);
    }
    World w(G);
    std::vector<FakeOps> ops(G);
    std::vector<lx::ExchangeState> st(G);
    uint64_t moved = 0;
    for (uint32_t q = 0; q < G; q++) ops[q] = FakeOps{&t, &w, q, std::vector<uint32_t>((uint64_t)N * V, 0xDEADBEEF)};
    for (uint32_t round = 0; round < rounds; round++) {
        // values near the row's seq (byte wire fits), some far (skew: blocks of
        // the first row owner's blocks fall back in odd rounds), some zero
        for (uint32_t i = 0; i < N; i++)
            for (uint32_t c = 0; c < V; c++) {
                uint32_t v = 0;
                const uint64_t x = rng() % 10;
                if (x < 6) v = t.seq[i] + (uint32_t)(rng() % 100);
                if (skew && t.owner[i] == t.owner[0] && (round % 2) && x == 9) v = t.seq[i] + 1000 + (uint32_t)(rng() % 60000);
                t.la[(uint64_t)i * V + c] = v;
            }
        std::vector<int> rcs(G, 0);
        std::vector<std::thread> th;
        for (uint32_t q = 0; q < G; q++)
            th.emplace_back([&, q] {
                FakeNet net{&w, q};
                rcs[q] = lx::shard_exchange_run(ops[q], net, q, G, st[q]);
            });
        for (auto &x : th) x.join();
        for (uint32_t q = 0; q < G; q++)
            if (rcs[q] || !w.err.empty()) {
                snprintf(err, cap, "round %u rank %u rc %d: %s", round, q, rcs[q], w.err.c_str());
                return -1;
            }
        for (uint32_t q = 0; q < G; q++)
            for (uint32_t i = 0; i < N; i++)
                for (uint32_t c : t.cols[q])
                    if (ops[q].got[(uint64_t)i * V + c] != t.la[(uint64_t)i * V + c]) {
                        snprintf(err, cap, "round %u rank %u row %u col %u: got %u want %u", round, q, i, c,
                                 ops[q].got[(uint64_t)i * V + c], t.la[(uint64_t)i * V + c]);
                        return -1;
                    }
        for (uint32_t q = 0; q < G; q++) moved += (uint64_t)(N - t.rows[q].size()) * t.cols[q].size();
    }
    stats[0] = stats[1] = 0;
    for (auto &o : ops) {
        stats[0] += o.fallbacks;
        stats[1] += o.byte_packs;
    }
    stats[2] = moved;
    return 0;
}

// the layout helper alone (compared with lx_shard_exchange_layout and the Python one)
void lx_fake_shard_layout(uint32_t G, uint32_t self, const uint64_t *entries, const uint32_t *width, uint64_t *off) {
    lx::shard_layout(G, self, entries, width, off);
}

}  // extern "C"
