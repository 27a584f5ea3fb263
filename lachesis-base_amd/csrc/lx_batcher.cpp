// lx_batcher.cpp -- level-synchronous DAG batcher (include/lachesis_batcher.h).
//
// Parents-first buffering as gossip/dagordering.EventsBuffer does it
// (event_buffer.go:53-110), releasing in bulk: a pop takes every event whose
// ancestors are all known, level by level (a level = the events whose last
// missing parent was released by the previous level), push order inside a
// level.  Host-only bookkeeping, O(parents) per event.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lachesis_batcher.h"

namespace {

struct Pending {
    uint64_t id = 0;
    uint32_t creator = 0, seq = 0;
    std::vector<uint64_t> parents;
    uint32_t missing = 0;     // parents not released yet
    uint64_t order = 0;       // push order
    bool live = false;
};

}  // namespace

struct lx_batcher {
    std::string err;
    std::unordered_map<uint64_t, uint32_t> dense;       // released id -> dense index
    std::vector<uint64_t> released;                     // dense index -> id
    std::unordered_map<uint64_t, uint32_t> pend_of;     // pending id -> slot
    std::vector<Pending> pend;
    std::vector<uint32_t> free_slots;
    std::unordered_map<uint64_t, std::vector<uint32_t>> waiters;   // missing parent -> pending slots
    std::vector<uint32_t> ready;                        // slots with missing == 0
    uint64_t next_order = 0;
    // release plan of the next pop (valid while `planned`)
    bool planned = false;
    std::vector<uint32_t> plan;                         // slots in release order
    std::vector<uint32_t> plan_levels;                  // level offsets into plan
    uint64_t plan_parents = 0;
    // the last pop, for lx_batcher_unpop
    uint32_t last_first = 0, last_n = 0;

    int fail(int code, const char *fmt, ...) {
        char buf[256];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
};

namespace {

uint32_t alloc_slot(lx_batcher *b) {
    if (!b->free_slots.empty()) {
        uint32_t s = b->free_slots.back();
        b->free_slots.pop_back();
        return s;
    }
    b->pend.emplace_back();
    return (uint32_t)b->pend.size() - 1;
}

void release_slot(lx_batcher *b, uint32_t s) {
    Pending &p = b->pend[s];
    b->pend_of.erase(p.id);
    p.parents.clear();
    p.live = false;
    b->free_slots.push_back(s);
}

bool by_order(const lx_batcher *b, uint32_t x, uint32_t y) { return b->pend[x].order < b->pend[y].order; }

// the levels the next pop releases (children's missing counts simulated)
void make_plan(lx_batcher *b) {
    if (b->planned) return;
    b->plan.clear();
    b->plan_levels.assign(1, 0);
    b->plan_parents = 0;
    std::unordered_map<uint32_t, uint32_t> dec;   // slot -> parents released by this plan
    std::vector<uint32_t> level = b->ready;
    while (!level.empty()) {
        std::sort(level.begin(), level.end(), [b](uint32_t x, uint32_t y) { return by_order(b, x, y); });
        std::vector<uint32_t> next;
        for (uint32_t s : level) {
            b->plan.push_back(s);
            b->plan_parents += b->pend[s].parents.size();
            auto w = b->waiters.find(b->pend[s].id);
            if (w == b->waiters.end()) continue;
            for (uint32_t c : w->second)
                if (++dec[c] == b->pend[c].missing) next.push_back(c);
        }
        b->plan_levels.push_back((uint32_t)b->plan.size());
        level.swap(next);
    }
    b->planned = true;
}

// missing counts, waiters and the ready list recomputed from scratch
void rebuild_waits(lx_batcher *b) {
    b->waiters.clear();
    b->ready.clear();
    for (uint32_t s = 0; s < b->pend.size(); s++) {
        Pending &p = b->pend[s];
        if (!p.live) continue;
        p.missing = 0;
        for (uint64_t q : p.parents)
            if (!b->dense.count(q)) {
                p.missing++;
                b->waiters[q].push_back(s);
            }
        if (!p.missing) b->ready.push_back(s);
    }
    b->planned = false;
}

}  // namespace

extern "C" {

int lx_batcher_create(lx_batcher **out) {
    if (!out) return LX_ERR_ARG;
    *out = new lx_batcher();
    return 0;
}

void lx_batcher_destroy(lx_batcher *b) { delete b; }

const char *lx_batcher_last_error(const lx_batcher *b) { return b ? b->err.c_str() : "null handle"; }

int lx_batcher_reset(lx_batcher *b) {
    if (!b) return LX_ERR_ARG;
    lx_batcher fresh;
    std::swap(*b, fresh);
    return 0;
}

int lx_batcher_push(lx_batcher *b, uint32_t n, const uint64_t *id, const uint32_t *creator_idx, const uint32_t *seq,
                    const uint64_t *parent_off, const uint64_t *parent_id, uint8_t *out_status) {
    if (!b) return LX_ERR_ARG;
    if (!n) return 0;
    if (!id || !creator_idx || !seq || !parent_off) return b->fail(LX_ERR_ARG, "null input");
    for (uint32_t i = 0; i < n; i++)
        if (parent_off[i + 1] < parent_off[i]) return b->fail(LX_ERR_ARG, "parent offsets not monotone at %u", i);
    if (parent_off[n] > parent_off[0] && !parent_id) return b->fail(LX_ERR_ARG, "null parent ids");
    for (uint32_t i = 0; i < n; i++) {
        uint8_t st = LX_PUSH_QUEUED;
        if (b->dense.count(id[i])) st = LX_PUSH_CONNECTED;          // ErrAlreadyConnectedEvent
        else if (b->pend_of.count(id[i])) st = LX_PUSH_DUPLICATE;   // ErrDuplicateEvent
        if (out_status) out_status[i] = st;
        if (st != LX_PUSH_QUEUED) continue;
        const uint32_t s = alloc_slot(b);
        Pending &p = b->pend[s];
        p.id = id[i];
        p.creator = creator_idx[i];
        p.seq = seq[i];
        p.parents.assign(parent_id + parent_off[i], parent_id + parent_off[i + 1]);
        p.order = b->next_order++;
        p.live = true;
        p.missing = 0;
        for (uint64_t q : p.parents)
            if (!b->dense.count(q)) {
                p.missing++;
                b->waiters[q].push_back(s);
            }
        b->pend_of[p.id] = s;
        if (!p.missing) b->ready.push_back(s);
    }
    b->planned = false;
    return 0;
}

int lx_batcher_peek(lx_batcher *b, uint32_t *n_events, uint64_t *n_parents, uint32_t *n_levels, uint32_t *n_waiting) {
    if (!b) return LX_ERR_ARG;
    make_plan(b);
    if (n_events) *n_events = (uint32_t)b->plan.size();
    if (n_parents) *n_parents = b->plan_parents;
    if (n_levels) *n_levels = (uint32_t)b->plan_levels.size() - 1;
    if (n_waiting) *n_waiting = (uint32_t)(b->pend_of.size() - b->plan.size());
    return 0;
}

int lx_batcher_pop(lx_batcher *b, uint64_t *out_id, uint32_t *out_creator, uint32_t *out_seq, uint64_t *out_parent_off,
                   uint32_t *out_parent_idx, uint32_t *out_level_off, uint64_t *first_dense) {
    if (!b) return LX_ERR_ARG;
    make_plan(b);
    const uint32_t n = (uint32_t)b->plan.size();
    if (n && (!out_id || !out_creator || !out_seq || !out_parent_off || (b->plan_parents && !out_parent_idx)))
        return b->fail(LX_ERR_ARG, "null output");
    const uint32_t base = (uint32_t)b->released.size();
    if (first_dense) *first_dense = base;
    if (out_level_off)
        for (size_t l = 0; l < b->plan_levels.size(); l++) out_level_off[l] = b->plan_levels[l];
    uint64_t k = 0;
    if (out_parent_off) out_parent_off[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        Pending &p = b->pend[b->plan[i]];
        b->dense[p.id] = base + i;
        b->released.push_back(p.id);
        out_id[i] = p.id;
        out_creator[i] = p.creator;
        out_seq[i] = p.seq;
        for (uint64_t q : p.parents) out_parent_idx[k++] = b->dense.at(q);   // released before p
        out_parent_off[i + 1] = k;
    }
    // children still waiting lose the parents this pop released
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t pid = b->pend[b->plan[i]].id;
        auto w = b->waiters.find(pid);
        if (w == b->waiters.end()) continue;
        for (uint32_t c : w->second) b->pend[c].missing--;
        b->waiters.erase(w);
    }
    for (uint32_t i = 0; i < n; i++) release_slot(b, b->plan[i]);
    b->ready.clear();   // every ready event was in the plan
    b->last_first = base;
    b->last_n = n;
    b->plan.clear();
    b->planned = false;
    return 0;
}

int lx_batcher_unpop(lx_batcher *b) {
    if (!b) return LX_ERR_ARG;
    if (b->last_first + b->last_n != b->released.size())
        return b->fail(LX_ERR_STATE, "nothing to unpop (or events were released after it)");
    for (uint32_t i = 0; i < b->last_n; i++) {
        b->dense.erase(b->released.back());
        b->released.pop_back();
    }
    b->last_n = 0;
    rebuild_waits(b);
    return 0;
}

int lx_batcher_dense(const lx_batcher *b, uint64_t id, uint32_t *out) {
    if (!b || !out) return LX_ERR_ARG;
    auto it = b->dense.find(id);
    if (it == b->dense.end()) return LX_ERR_ARG;
    *out = it->second;
    return 0;
}

}  // extern "C"
