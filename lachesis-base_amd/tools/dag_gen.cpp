// dag_gen.cpp -- synthetic tdag-structured DAGs + ForklessCause query sets.
//
// Bench/test tooling (not part of the index library).  The DAG generator is
// bit-identical to oracle/tdag.py:rand_fork_dag (structure of
// inter/dag/tdag/test_common.go:37-136 ForEachRandFork, driven by splitmix64).
// Events come out in creation order, which is a valid Add order.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {
struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return (next() >> 11) % n; }
};
}  // namespace

extern "C" {

// Returns the number of parent entries written, or -1 if par_cap is too small.
// creator[] receives the generation column (0..n_nodes-1).
int64_t dag_gen(uint32_t n_nodes, uint32_t events_per_node, uint32_t parent_count, uint32_t cheaters,
                uint32_t forks_count, uint64_t seed, uint32_t *creator, uint32_t *seq, uint32_t *lamport,
                uint64_t *poff, uint32_t *par, uint64_t par_cap) {
    SplitMix64 rng(seed);
    std::vector<std::vector<uint32_t>> evs(n_nodes);
    std::vector<uint32_t> forks_done(n_nodes, 0);
    const uint32_t n_other = std::min<uint32_t>(parent_count ? parent_count - 1 : 0, n_nodes ? n_nodes - 1 : 0);
    std::vector<uint32_t> others(n_other);
    uint64_t np = 0;
    const uint64_t total = (uint64_t)n_nodes * events_per_node;
    poff[0] = 0;
    for (uint64_t i = 0; i < total; i++) {
        const uint32_t me = (uint32_t)(i % n_nodes);
        uint32_t k = 0;
        while (k < n_other) {
            uint32_t u = (uint32_t)rng.below(n_nodes - 1);
            uint32_t cand = u < me ? u : u + 1;
            bool dup = false;
            for (uint32_t j = 0; j < k; j++)
                if (others[j] == cand) { dup = true; break; }
            if (!dup) others[k++] = cand;
        }
        auto &ee = evs[me];
        int64_t parent = -1;
        if (!ee.empty()) {
            parent = ee.back();
            bool flipped = (rng.below(events_per_node) <= forks_count) || (i < (uint64_t)(n_nodes - 1) * events_per_node);
            if (me < cheaters && ee.size() > 1 && forks_done[me] < forks_count && flipped) {
                parent = ee[rng.below(ee.size() - 1)];
                if (rng.below(ee.size()) == 0) parent = -1;
                forks_done[me]++;
            }
        }
        uint32_t s, lam;
        if (parent < 0) {
            s = 1;
            lam = 1;
        } else {
            if (np + 1 > par_cap) return -1;
            s = seq[parent] + 1;
            lam = lamport[parent] + 1;
            par[np++] = (uint32_t)parent;
        }
        for (uint32_t j = 0; j < n_other; j++) {
            const auto &oe = evs[others[j]];
            if (!oe.empty()) {
                if (np + 1 > par_cap) return -1;
                uint32_t p = oe.back();
                par[np++] = p;
                if (lam <= lamport[p]) lam = lamport[p] + 1;
            }
        }
        creator[i] = me;
        seq[i] = s;
        lamport[i] = lam;
        poff[i + 1] = np;
        ee.push_back((uint32_t)i);
    }
    return (int64_t)np;
}

// ForklessCause query set: a uniform over events, b uniform over
// events with lamport(b) in [lamport(a) - window, lamport(a)].
void fc_queries(uint64_t n_events, const uint32_t *lamport, uint64_t nq, uint32_t window, uint64_t seed,
                uint32_t *qa, uint32_t *qb) {
    std::vector<uint32_t> order(n_events);
    for (uint64_t i = 0; i < n_events; i++) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return lamport[x] < lamport[y]; });
    std::vector<uint32_t> lam(n_events);
    for (uint64_t i = 0; i < n_events; i++) lam[i] = lamport[order[i]];
    SplitMix64 rng(seed);
    for (uint64_t q = 0; q < nq; q++) {
        uint32_t a = (uint32_t)rng.below(n_events);
        uint32_t la = lamport[a];
        uint32_t lo_l = la > window ? la - window : 0;
        uint64_t lo = std::lower_bound(lam.begin(), lam.end(), lo_l) - lam.begin();
        uint64_t hi = std::upper_bound(lam.begin(), lam.end(), la) - lam.begin();
        qa[q] = a;
        qb[q] = order[lo + rng.below(hi - lo)];
    }
}
}
