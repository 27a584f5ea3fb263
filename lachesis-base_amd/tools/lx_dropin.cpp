// lx_dropin.cpp -- the unchanged caller of the index, restated in C++, driving
// an index through the per-event / per-pair calls the reference makes (bench
// tooling, not part of the index library).
//
// abft.IndexedLachesis.Process(e) (abft/indexed_lachesis.go:69-82) calls, per
// event: Add(e); Lachesis.Process(e) -- calcFrameIdx asks ForklessCause(e, r)
// for the roots r of the frame in GetFrameRoots order until quorum
// (abft/event_processing.go:149-189), the election asks ForklessCause(root,
// r) for every root r of the previous frame (abft/election/election.go:
// 101-123, election_math.go:13-114), a decided frame reads
// GetMergedHighestBefore(atropos) (abft/lachesis.go:57-86) and replays the
// known roots (processKnownRoots, abft/event_processing.go:102-146) -- then
// Flush and the deferred DropNotFlushed.  This driver makes exactly those
// calls, in that order, on one of three backends:
//
//   kind 0: the HIP library (lx_add_batch with one event, lx_forkless_cause,
//           lx_flush, lx_drop_not_flushed, lx_get_merged_highest_before) --
//           the drop-in path a cgo shim binds;
//   kind 1: a CPU index given as function pointers, behind the reference's
//           ForklessCause LRU (simplewlru of lru_pairs entries,
//           vecfc/forkless_cause.go:28-38) -- bench.py's cpu_baseline leg
//           hands in the C restatement (oracle/) this way;
//   kind 2: the answers a previous run recorded, replayed without an index --
//           the caller's own time, so that run time minus it is the time the
//           index took.
//
// The caller's own arithmetic (frames, votes, quorum counters, the
// confirmation DFS) follows abft; its vote sums iterate observed roots in the
// outer loop and subjects in the inner one (contiguous vote rows) -- the same
// sums in a different order, with the reference's per-subject loop kept for
// frames where a validator has two observed roots (forks).  Every index call
// is folded into a hash with the definition of oracle/csrc/abft_oracle.c's
// trace, so tests pin the call sequence to the restatement's.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lachesis_hip.h"

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;
using clk = std::chrono::steady_clock;

uint64_t tr_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

}  // namespace

extern "C" {

typedef struct lx_dropin_cfg {
    int kind;                    // 0 HIP library, 1 CPU function pointers, 2 recorded answers
    int device;                  // kind 0
    int64_t fc_cache;            // kind 0: lx_set_option("fc_cache") (< 0: the library's default)
    uint32_t lru_pairs;          // kind 1: the reference's ForklessCause LRU entries (0: none)
    // kind 1: the CPU index (oracle/csrc/oracle.c signatures)
    void *cpu;
    int (*cpu_add)(void *, uint32_t, uint32_t, uint32_t, const uint32_t *);
    void (*cpu_flush)(void *);
    void (*cpu_drop)(void *);
    int (*cpu_fc)(void *, uint32_t, uint32_t);
    int (*cpu_merged_hb)(void *, uint32_t, uint8_t *, uint32_t, uint32_t *);
    // recorded answers: written by kinds 0 / 1 when non-NULL, read by kind 2
    uint8_t *rec_fc;
    uint64_t rec_fc_cap;
    uint8_t *rec_mhb;            // 8 V bytes per GetMergedHighestBefore call
    uint64_t rec_mhb_cap;        // calls
    uint64_t max_events;         // process at most this many events (0: all)
} lx_dropin_cfg;

typedef struct lx_dropin_out {
    uint32_t *frames;            // [N] claimed frame accepted per event
    uint32_t *roots_per_frame;   // [frames_cap]
    uint32_t frames_cap;
    uint32_t *block_frame, *block_atropos, *block_ncheat, *block_nconf;   // [blocks_cap]
    uint32_t blocks_cap;
    double *checkpoint_s;        // [N / 1000 + 1]: wall seconds after every 1000 events
    // filled:
    uint64_t events, blocks, fc_calls, adds, flushes, drops, merged_hb_calls, trace_hash;
    double seconds, add_seconds;
    uint32_t max_frame;
    lx_fc_stats fc;              // kind 0: the library's cache counters
    uint64_t lru_hits;           // kind 1
} lx_dropin_out;

}  // extern "C"

namespace {

// ---- the reference's ForklessCause LRU (kind 1), restating simplewlru over (a, b)
struct Lru {
    uint32_t cap = 0;
    std::unordered_map<uint64_t, uint32_t> pos;
    std::vector<uint64_t> key;
    std::vector<uint8_t> val;
    std::vector<uint32_t> prev, next;
    uint32_t head = NONE, tail = NONE, n = 0;
    void init(uint32_t c) {
        cap = c;
        key.resize(c); val.resize(c); prev.resize(c); next.resize(c);
        pos.reserve(2 * c);
    }
    void unlink(uint32_t i) {
        if (prev[i] != NONE) next[prev[i]] = next[i]; else head = next[i];
        if (next[i] != NONE) prev[next[i]] = prev[i]; else tail = prev[i];
    }
    void front(uint32_t i) {
        prev[i] = NONE; next[i] = head;
        if (head != NONE) prev[head] = i;
        head = i;
        if (tail == NONE) tail = i;
    }
    int get(uint64_t k) {
        auto it = pos.find(k);
        if (it == pos.end()) return -1;
        unlink(it->second);
        front(it->second);
        return val[it->second];
    }
    void put(uint64_t k, uint8_t v) {
        uint32_t i;
        if (n == cap) {
            i = tail;
            unlink(i);
            pos.erase(key[i]);
        } else {
            i = n++;
        }
        key[i] = k; val[i] = v;
        pos[k] = i;
        front(i);
    }
    void clear() { pos.clear(); head = tail = NONE; n = 0; }
};

struct Slot {                    // a root slot's votes (election_math.go:105-112)
    uint32_t stamp = 0;          // election the votes were cast in
    std::vector<uint8_t> voted, yes;
    std::vector<uint32_t> obs;   // observed root (event)
};

struct Frame {
    std::vector<uint32_t> ev, creator;
    std::vector<Slot> slots;
};

struct VoteV {
    uint8_t yes = 0;
    uint32_t observed = NONE;
};

struct Caller {
    const lx_dropin_cfg &cfg;
    lx_dropin_out &out;
    lx_index *ix = nullptr;
    Lru lru;
    uint64_t rec_fc_n = 0, rec_mhb_n = 0;
    std::string err;
    // epoch
    uint32_t V = 0, quorum = 0;
    std::vector<uint32_t> w;
    const uint32_t *creator = nullptr, *seq = nullptr, *par = nullptr;
    const uint64_t *poff = nullptr;
    uint32_t n = 0;                          // events processed
    std::vector<uint32_t> frame, sp, confirmed;
    std::vector<Frame> fr;
    uint32_t last_decided = 0;
    // election
    uint32_t frame_to_decide = 1, stamp = 0;
    std::vector<uint8_t> dec_has;
    std::vector<VoteV> dec;
    std::vector<uint32_t> cnt, map_slot, map_stamp;
    uint32_t cnt_stamp = 0;
    std::vector<uint32_t> obs, yes_s, no_s, all_s, subj;
    std::vector<uint8_t> notdec, row;
    std::vector<uint32_t> stack;

    Caller(const lx_dropin_cfg &c, lx_dropin_out &o) : cfg(c), out(o) {}

    void tr(uint64_t rec) { out.trace_hash = tr_mix(out.trace_hash ^ rec); }

    // ---- index calls
    int idx_add(uint32_t e) {
        tr((1ull << 62) | e);
        out.adds++;
        const uint32_t np = (uint32_t)(poff[e + 1] - poff[e]);
        const auto t0 = clk::now();
        int rc = 0;
        if (cfg.kind == 0) {
            const uint64_t po[2] = {0, np};
            uint32_t c = creator[e], s = seq[e];
            rc = lx_add_batch(ix, 1, &c, &s, po, par + poff[e], nullptr, nullptr);
            if (rc) err = lx_last_error(ix);
        } else if (cfg.kind == 1) {
            rc = cfg.cpu_add(cfg.cpu, creator[e], seq[e], np, par + poff[e]);
            if (rc) err = "cpu index Add failed";
        }
        out.add_seconds += std::chrono::duration<double>(clk::now() - t0).count();
        return rc;
    }
    void idx_flush() {
        tr((2ull << 62) | n);
        out.flushes++;
        if (cfg.kind == 0) lx_flush(ix);
        else if (cfg.kind == 1) cfg.cpu_flush(cfg.cpu);
    }
    // rollback: events were added since the last Flush (else a no-op call)
    void idx_drop(bool rollback) {
        tr((3ull << 62) | n);
        out.drops++;
        if (cfg.kind == 0) lx_drop_not_flushed(ix);
        else if (cfg.kind == 1) {
            cfg.cpu_drop(cfg.cpu);
            if (rollback) lru.clear();   // dense indices are reused after a rollback (hashes are not)
        }
    }
    // 1 / 0, or < 0 on error
    int fc(uint32_t a, uint32_t b) {
        tr(((uint64_t)a << 32) | b);
        out.fc_calls++;
        int r;
        if (cfg.kind == 0) {
            uint8_t o = 0;
            if (lx_forkless_cause(ix, a, b, &o)) { err = lx_last_error(ix); return -1; }
            r = o;
        } else if (cfg.kind == 1) {
            const uint64_t k = ((uint64_t)a << 32) | b;
            r = cfg.lru_pairs ? lru.get(k) : -1;
            if (r >= 0) {
                out.lru_hits++;
            } else {
                r = cfg.cpu_fc(cfg.cpu, a, b) == 1 ? 1 : 0;
                if (cfg.lru_pairs) lru.put(k, (uint8_t)r);
            }
        } else {
            if (rec_fc_n >= cfg.rec_fc_cap) { err = "recorded answers exhausted"; return -1; }
            return cfg.rec_fc[rec_fc_n++];
        }
        if (cfg.rec_fc) {
            if (rec_fc_n >= cfg.rec_fc_cap) { err = "answer record full"; return -1; }
            cfg.rec_fc[rec_fc_n++] = (uint8_t)r;
        }
        return r;
    }
    // merged HighestBefore row of ev (8 V bytes) into row
    int merged_hb(uint32_t ev) {
        out.merged_hb_calls++;
        row.assign(8ull * V, 0);
        uint32_t len = 0;
        if (cfg.kind == 2) {
            if (rec_mhb_n >= cfg.rec_mhb_cap) { err = "recorded rows exhausted"; return -1; }
            memcpy(row.data(), cfg.rec_mhb + rec_mhb_n++ * 8ull * V, 8ull * V);
            return 0;
        }
        int rc = cfg.kind == 0 ? lx_get_merged_highest_before(ix, ev, row.data(), (uint32_t)row.size(), &len)
                               : cfg.cpu_merged_hb(cfg.cpu, ev, row.data(), (uint32_t)row.size(), &len);
        if (rc) { err = cfg.kind == 0 ? lx_last_error(ix) : "cpu merged HB failed"; return -1; }
        if (cfg.rec_mhb) {
            if (rec_mhb_n >= cfg.rec_mhb_cap) { err = "row record full"; return -1; }
            memcpy(cfg.rec_mhb + rec_mhb_n++ * 8ull * V, row.data(), 8ull * V);
        }
        return 0;
    }

    // ---- abft
    Frame &frame_roots(uint32_t f) {
        if (f >= fr.size()) fr.resize(f + 1);
        return fr[f];
    }
    void election_reset(uint32_t ftd) {          // election.go:87-93
        frame_to_decide = ftd;
        stamp++;
        std::fill(dec_has.begin(), dec_has.end(), 0);
        // votes of frames below the new election are never read again
        for (uint32_t f = 0; f + 1 < ftd && f < fr.size(); f++) fr[f].slots.clear();
    }
    int choose_atropos(uint32_t *atropos) {      // sort_roots.go:10-25
        for (uint32_t v = 0; v < V; v++) {
            if (!dec_has[v]) return 0;
            if (dec[v].yes) { *atropos = dec[v].observed; return 1; }
        }
        err = "all the roots are decided as 'no'";
        return -8;
    }
    Slot &slot_of(uint32_t f, uint32_t k) {
        Frame &r = frame_roots(f);
        if (r.slots.size() < r.ev.size()) r.slots.resize(r.ev.size());
        Slot &s = r.slots[k];
        if (s.voted.size() != V) { s.voted.assign(V, 0); s.yes.assign(V, 0); s.obs.assign(V, NONE); }
        return s;
    }
    // ProcessRoot (election_math.go:13-114) for root slot (frame f, index k)
    int process_root(uint32_t f, uint32_t k, uint32_t *atropos) {
        int rc = choose_atropos(atropos);
        if (rc) return rc;
        const uint32_t F = frame_to_decide;
        if (f <= F) return 0;
        const uint32_t round = f - F;
        const uint32_t root = frame_roots(f).ev[k];
        const Frame &prev = frame_roots(f - 1);
        const uint32_t np = (uint32_t)prev.ev.size();
        obs.clear();
        const uint32_t ms = ++cnt_stamp;
        for (uint32_t j = 0; j < np; j++) {          // observedRoots / observedRootsMap
            const int x = fc(root, prev.ev[j]);
            if (x < 0) return -1;
            if (!x) continue;
            if (round == 1) { map_slot[prev.creator[j]] = j; map_stamp[prev.creator[j]] = ms; }
            else obs.push_back(j);
        }
        Slot &mine = slot_of(f, k);
        if (mine.stamp != stamp) {
            std::fill(mine.voted.begin(), mine.voted.end(), 0);
            mine.stamp = stamp;
        }
        if (round == 1) {
            for (uint32_t v = 0; v < V; v++) {
                if (dec_has[v]) continue;
                const bool y = map_stamp[v] == ms;
                mine.voted[v] = 1;
                mine.yes[v] = y;
                mine.obs[v] = y ? prev.ev[map_slot[v]] : NONE;
            }
            return choose_atropos(atropos);
        }
        // round >= 2: weighted yes / no / all sums over the observed roots
        bool dup = false;
        {
            const uint32_t cs = ++cnt_stamp;
            for (uint32_t j : obs) {
                const uint32_t c = prev.creator[j];
                if (cnt[c] == cs) { dup = true; break; }
                cnt[c] = cs;
            }
        }
        for (uint32_t v = 0; v < V; v++) notdec[v] = !dec_has[v];
        if (!dup) {
            std::fill(yes_s.begin(), yes_s.end(), 0u);
            std::fill(no_s.begin(), no_s.end(), 0u);
            std::fill(all_s.begin(), all_s.end(), 0u);
            std::fill(subj.begin(), subj.end(), NONE);
            uint32_t bad = 0;
            for (uint32_t j : obs) {
                Frame &pf = frame_roots(f - 1);
                if (pf.slots.size() <= j || pf.slots[j].stamp != stamp || pf.slots[j].voted.size() != V) {
                    err = "every root must vote for every not decided subject. possibly roots are processed out of order";
                    return -8;
                }
                const Slot &S = pf.slots[j];
                const uint32_t wc = w[prev.creator[j]];
                const uint8_t *vt = S.voted.data(), *yy = S.yes.data();
                const uint32_t *ob = S.obs.data();
                uint32_t *ys = yes_s.data(), *ns = no_s.data(), *as = all_s.data(), *sj = subj.data();
                const uint8_t *nd = notdec.data();
                for (uint32_t v = 0; v < V; v++) {
                    const uint32_t d = nd[v], t = vt[v], y = yy[v] & d;
                    bad |= d & (t ^ 1u);
                    const uint32_t o = ob[v], s = sj[v];
                    bad |= (y & (s != NONE) & (s != o)) << 1;
                    ys[v] += wc & (0u - y);
                    ns[v] += wc & (0u - ((y ^ d) & t));
                    as[v] += wc & (0u - (d & t));
                    sj[v] = y ? o : s;
                }
            }
            if (bad) {
                err = bad & 1 ? "every root must vote for every not decided subject. possibly roots are processed out of order"
                              : "forkless caused by 2 fork roots => more than 1/3W are Byzantine";
                return -8;
            }
            for (uint32_t v = 0; v < V; v++) {
                if (!notdec[v]) continue;
                if (all_s[v] < quorum) {
                    err = "root must be forkless caused by at least 2/3W of prev roots. possibly roots are processed out of order";
                    return -8;
                }
                const bool y = yes_s[v] >= no_s[v];
                mine.voted[v] = 1;
                mine.yes[v] = y;
                mine.obs[v] = y && subj[v] != NONE ? subj[v] : NONE;
                if (yes_s[v] >= quorum || no_s[v] >= quorum) {
                    dec_has[v] = 1;
                    dec[v].yes = y;
                    dec[v].observed = mine.obs[v];
                }
            }
            return choose_atropos(atropos);
        }
        // a validator with two observed roots: the reference's loop order, per-creator counters
        std::vector<uint32_t> cy(V, 0), cn(V, 0), ca(V, 0);
        uint32_t cst = 0;
        for (uint32_t v = 0; v < V; v++) {
            if (!notdec[v]) continue;
            ++cst;
            uint32_t yes = 0, no = 0, all = 0, subject = NONE;
            for (uint32_t j : obs) {
                const Slot *S = frame_roots(f - 1).slots.size() > j ? &frame_roots(f - 1).slots[j] : nullptr;
                const uint32_t c = prev.creator[j];
                if (!S || S->stamp != stamp || S->voted.size() != V || !S->voted[v]) {
                    err = "every root must vote for every not decided subject. possibly roots are processed out of order";
                    return -8;
                }
                if (S->yes[v] && subject != NONE && subject != S->obs[v]) {
                    err = "forkless caused by 2 fork roots => more than 1/3W are Byzantine";
                    return -8;
                }
                if (S->yes[v]) {
                    subject = S->obs[v];
                    if (cy[c] != cst) { cy[c] = cst; yes += w[c]; }
                } else if (cn[c] != cst) {
                    cn[c] = cst;
                    no += w[c];
                }
                if (ca[c] == cst) {
                    err = "forkless caused by 2 fork roots => more than 1/3W are Byzantine";
                    return -8;
                }
                ca[c] = cst;
                all += w[c];
            }
            if (all < quorum) {
                err = "root must be forkless caused by at least 2/3W of prev roots. possibly roots are processed out of order";
                return -8;
            }
            const bool y = yes >= no;
            mine.voted[v] = 1;
            mine.yes[v] = y;
            mine.obs[v] = y && subject != NONE ? subject : NONE;
            if (yes >= quorum || no >= quorum) {
                dec_has[v] = 1;
                dec[v].yes = y;
                dec[v].observed = mine.obs[v];
            }
        }
        return choose_atropos(atropos);
    }
    // forklessCausedByQuorumOn (event_processing.go:148-161)
    int quorum_on(uint32_t e, uint32_t f) {
        if (f >= fr.size()) return 0;
        const uint32_t cs = ++cnt_stamp;
        uint32_t sum = 0;
        const uint32_t nr = (uint32_t)fr[f].ev.size();
        for (uint32_t j = 0; j < nr; j++) {
            const int x = fc(e, fr[f].ev[j]);
            if (x < 0) return -1;
            if (x) {
                const uint32_t c = fr[f].creator[j];
                if (cnt[c] != cs) { cnt[c] = cs; sum += w[c]; }
            }
            if (sum >= quorum) break;
        }
        return sum >= quorum ? 1 : 0;
    }
    // calcFrameIdx with checkOnly (event_processing.go:163-189)
    int calc_frame(uint32_t e, uint32_t claimed, uint32_t *spf, uint32_t *out_f) {
        *spf = sp[e] == NONE ? 0 : frame[sp[e]];
        uint32_t f = *spf;
        while (f < claimed) {
            const int x = quorum_on(e, f);
            if (x < 0) return -1;
            if (!x) break;
            f++;
        }
        *out_f = f == 0 ? 1 : f;
        return 0;
    }
    // applyAtropos + onFrameDecided (lachesis.go:57-86, frame_decide.go:11-35)
    int on_frame_decided(uint32_t f, uint32_t atropos) {
        if (merged_hb(atropos)) return -1;
        uint32_t nch = 0;
        for (uint32_t c = 0; c < V; c++) {
            uint32_t s, m;
            memcpy(&s, row.data() + 8ull * c, 4);
            memcpy(&m, row.data() + 8ull * c + 4, 4);
            if (s == 0 && m == 0x7FFFFFFFu) nch++;
        }
        uint32_t nconf = 0;
        stack.clear();
        for (uint32_t walk = atropos;;) {           // dfsSubgraph (traversal.go:13-37)
            if (!confirmed[walk]) {
                confirmed[walk] = f;
                nconf++;
                for (uint64_t k = poff[walk]; k < poff[walk + 1]; k++) stack.push_back(par[k]);
            }
            if (stack.empty()) break;
            walk = stack.back();
            stack.pop_back();
        }
        const uint64_t b = out.blocks++;
        if (b < out.blocks_cap) {
            out.block_frame[b] = f;
            out.block_atropos[b] = atropos;
            out.block_ncheat[b] = nch;
            out.block_nconf[b] = nconf;
        }
        last_decided = f;
        election_reset(f + 1);
        return 0;
    }
    int bootstrap_election() {                   // event_processing.go:102-146
        for (;;) {
            uint32_t atropos = NONE;
            int rc = 0;
            for (uint32_t f = last_decided + 1;; f++) {
                const uint32_t nr = f < fr.size() ? (uint32_t)fr[f].ev.size() : 0;
                for (uint32_t k = 0; k < nr && !rc; k++) rc = process_root(f, k, &atropos);
                if (rc || nr == 0) break;
            }
            if (rc < 0) return rc;
            if (rc == 0) return 0;
            if (on_frame_decided(frame_to_decide, atropos)) return -1;
        }
    }
    // IndexedLachesis.Process with the event's claimed frame
    int process(uint32_t e, uint32_t claimed) {
        if (idx_add(e)) return -1;
        n = e + 1;
        frame.push_back(0);
        sp.push_back(seq[e] > 1 && poff[e + 1] > poff[e] ? par[poff[e]] : NONE);
        confirmed.push_back(0);
        uint32_t spf, f;
        if (calc_frame(e, claimed, &spf, &f)) return -1;
        if (f != claimed) {
            n = e;
            idx_drop(true);
            err = "ErrWrongFrame";
            return -7;
        }
        frame[e] = f;
        for (uint32_t g = spf + 1; g <= f; g++) {      // store_roots.go:22-27
            Frame &r = frame_roots(g);
            r.ev.push_back(e);
            r.creator.push_back(creator[e]);
        }
        for (uint32_t g = spf + 1; g <= f; g++) {      // handleElection (event_processing.go:64-100)
            const Frame &r = frame_roots(g);
            uint32_t k = NONE;
            for (uint32_t j = (uint32_t)r.ev.size(); j-- > 0;)
                if (r.ev[j] == e) { k = j; break; }
            uint32_t atropos = NONE;
            int rc = process_root(g, k, &atropos);
            if (rc < 0) return rc;
            if (rc == 0) continue;
            if (on_frame_decided(frame_to_decide, atropos)) return -1;
            if ((rc = bootstrap_election()) < 0) return rc;
        }
        idx_flush();
        idx_drop(false);
        return 0;
    }
};

}  // namespace

extern "C" {

// Replays IndexedLachesis.Process over the events (claimed frames given),
// one epoch, on the backend of cfg.  Returns 0, or < 0 with err filled.
int lx_dropin_replay(const lx_dropin_cfg *cfg, uint32_t V, const uint32_t *weights, uint64_t N, const uint32_t *creator,
                     const uint32_t *seq, const uint64_t *poff, const uint32_t *par, const uint32_t *claimed,
                     lx_dropin_out *out, char *errbuf, uint32_t errcap) {
    Caller c(*cfg, *out);
    auto fail = [&](int rc) {
        snprintf(errbuf, errcap, "%s", c.err.c_str());
        if (c.ix) lx_destroy(c.ix);
        return rc ? rc : -1;
    };
    const uint64_t M = cfg->max_events ? std::min<uint64_t>(N, cfg->max_events) : N;
    out->events = out->blocks = out->fc_calls = out->adds = out->flushes = out->drops = out->merged_hb_calls = 0;
    out->trace_hash = 0;
    out->seconds = out->add_seconds = 0;
    out->lru_hits = 0;
    c.V = V;
    c.w.assign(weights, weights + V);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < V; i++) tot += weights[i];
    c.quorum = (uint32_t)(tot * 2 / 3 + 1);
    c.creator = creator; c.seq = seq; c.poff = poff; c.par = par;
    c.dec_has.assign(V, 0);
    c.dec.assign(V, VoteV{});
    c.cnt.assign(V, 0);
    c.map_slot.assign(V, 0);
    c.map_stamp.assign(V, 0);
    c.yes_s.assign(V, 0); c.no_s.assign(V, 0); c.all_s.assign(V, 0); c.subj.assign(V, NONE);
    c.notdec.assign(V, 0);
    c.frame.reserve(M); c.sp.reserve(M); c.confirmed.reserve(M);
    c.election_reset(1);
    if (cfg->kind == 0) {
        lx_config lc{};
        lc.device = cfg->device;
        lc.event_capacity = M;
        if (lx_create(&lc, &c.ix)) { c.err = "lx_create"; return fail(-1); }
        if (cfg->fc_cache >= 0 && lx_set_option(c.ix, "fc_cache", cfg->fc_cache)) { c.err = lx_last_error(c.ix); return fail(-1); }
        if (lx_reset(c.ix, V, weights)) { c.err = lx_last_error(c.ix); return fail(-1); }
        if (lx_sync(c.ix)) { c.err = lx_last_error(c.ix); return fail(-1); }
    } else if (cfg->kind == 1 && cfg->lru_pairs) {
        c.lru.init(cfg->lru_pairs);
    }
    const auto t0 = clk::now();
    for (uint64_t e = 0; e < M; e++) {
        int rc = c.process((uint32_t)e, claimed[e]);
        if (rc) return fail(rc);
        out->frames[e] = c.frame[e];
        if (out->checkpoint_s && (e + 1) % 1000 == 0)
            out->checkpoint_s[e / 1000] = std::chrono::duration<double>(clk::now() - t0).count();
    }
    if (cfg->kind == 0 && lx_sync(c.ix)) { c.err = lx_last_error(c.ix); return fail(-1); }
    out->seconds = std::chrono::duration<double>(clk::now() - t0).count();
    out->events = M;
    out->max_frame = 0;
    for (uint32_t f = 0; f < c.fr.size(); f++) {
        if (f < out->frames_cap) out->roots_per_frame[f] = (uint32_t)c.fr[f].ev.size();
        if (!c.fr[f].ev.empty()) out->max_frame = f;
    }
    if (cfg->kind == 0) {
        lx_fc_cache_stats(c.ix, &out->fc);
        lx_destroy(c.ix);
    }
    return 0;
}

}  // extern "C"
