// lx_batcher.cpp -- level-synchronous DAG batcher (include/lachesis_batcher.h).
//
// Parents-first buffering as gossip/dagordering.EventsBuffer does it
// (event_buffer.go:53-110), releasing in bulk: a pop takes every event whose
// ancestors are all known, level by level (a level = the events whose last
// missing parent was released by the previous level), push order inside a
// level.  Host-only bookkeeping, flat arrays and one open-addressing table:
//
//  * ids: id -> released dense index, or pending slot (kPend bit); released
//    ids stay for the epoch (ErrAlreadyConnectedEvent, parents' dense indices);
//  * a pending event keeps its parents' ids and, per parent, the resolved
//    dense index -- known at push time for released parents; for the others a
//    waiter node {child, parent position} hangs on the parent (on its pending
//    slot, or in `unknown` while its id has not been pushed) and the pop that
//    releases the parent patches the child's entry and its missing count, so a
//    pop copies resolved entries without looking anything up;
//  * levels are planned with per-slot counters stamped per plan.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/lachesis_batcher.h"

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kPend = 0x80000000u;   // ids value: pending slot (else a dense index)

// open-addressing table uint64 -> uint32 with tombstones (erase is rare: unpop);
// one 16-B entry per slot, so a probe touches one cache line
struct IdMap {
    struct Ent {
        uint64_t key;
        uint32_t val;
        uint32_t st;   // 0 empty, 1 full, 2 deleted
    };
    std::vector<Ent> t;
    uint64_t mask = 0, used = 0, live = 0;
    // ids of consecutive events stay in nearby slots (the low bits vary
    // first), arbitrary 64-bit ids are mixed by the high half
    static uint64_t h(uint64_t k) { return k ^ (k >> 29) ^ (k >> 47); }
    void init(uint64_t cap) {
        uint64_t m = 1024;
        while (m < 2 * cap) m <<= 1;
        t.assign(m, Ent{0, 0, 0});
        mask = m - 1;
        used = live = 0;
        gen++;
    }
    uint32_t find(uint64_t k) const {
        for (uint64_t i = h(k) & mask;; i = (i + 1) & mask) {
            const Ent &e = t[i];
            if (e.st == 0) return kNone;
            if (e.key == k && e.st == 1) return e.val;
        }
    }
    uint32_t *ref(uint64_t k) {
        for (uint64_t i = h(k) & mask;; i = (i + 1) & mask) {
            Ent &e = t[i];
            if (e.st == 0) return nullptr;
            if (e.key == k && e.st == 1) return &e.val;
        }
    }
    // the value of k, or (k absent) insert v and return kNone: one probe
    // sequence; *at = the entry's position (valid until the table grows)
    uint32_t find_or_put(uint64_t k, uint32_t v, uint64_t *at) {
        if ((used + 1) * 2 > mask + 1) grow();
        uint64_t i = h(k) & mask, tomb = ~0ull;
        for (;; i = (i + 1) & mask) {
            Ent &e = t[i];
            if (e.st == 0) break;
            if (e.st == 1 && e.key == k) { *at = i; return e.val; }
            if (e.st == 2 && tomb == ~0ull) tomb = i;
        }
        if (tomb != ~0ull) i = tomb;
        else used++;
        t[i] = Ent{k, v, 1};
        live++;
        *at = i;
        return kNone;
    }
    uint64_t gen = 0;   // bumped when the table is rebuilt: remembered positions are stale
    void put(uint64_t k, uint32_t v) {   // k not present
        if ((used + 1) * 2 > mask + 1) grow();
        uint64_t i = h(k) & mask;
        while (t[i].st == 1) i = (i + 1) & mask;
        if (t[i].st == 0) used++;
        t[i] = Ent{k, v, 1};
        live++;
    }
    void erase(uint64_t k) {
        for (uint64_t i = h(k) & mask;; i = (i + 1) & mask) {
            if (t[i].st == 0) return;
            if (t[i].st == 1 && t[i].key == k) { t[i].st = 2; live--; return; }
        }
    }
    void grow() {
        std::vector<Ent> old;
        old.swap(t);
        init(std::max<uint64_t>(2 * (mask + 1), 2 * live));   // init doubles again: 4x the slots
        for (const Ent &e : old)
            if (e.st == 1) put(e.key, e.val);
    }
};

struct Pending {
    uint64_t id = 0, order = 0;
    uint64_t at = 0, at_gen = 0;    // its ids entry (position, table generation)
    uint32_t creator = 0, seq = 0;
    uint32_t par_off = 0, np = 0;   // into par_id / par_res
    uint32_t missing = 0;           // parents not released yet
    uint32_t waiters = kNone;       // head of the chain of children waiting for this event
    uint32_t plan_stamp = 0, plan_cnt = 0;
    bool live = false;
};

struct Waiter {
    uint32_t child, pos, next;      // child slot, index into par_res, next node
};

}  // namespace

struct lx_batcher {
    std::string err;
    IdMap ids;                                  // id -> dense | kPend | slot
    std::vector<uint64_t> released;             // dense index -> id
    std::vector<Pending> pend;
    std::vector<uint32_t> free_slots;
    uint32_t n_pending = 0;
    std::vector<uint64_t> par_id;               // parents of pending events (ids)
    std::vector<uint32_t> par_res;              // ... resolved dense index, or kNone
    std::vector<Waiter> wnodes;
    std::vector<uint32_t> wfree;
    IdMap unknown;                              // id never pushed -> head of its waiter chain
    std::vector<uint32_t> ready;                // slots with missing == 0
    uint64_t next_order = 0;
    // release plan of the next pop (valid while `planned`)
    bool planned = false;
    uint32_t stamp = 0;
    std::vector<uint32_t> plan, plan_levels, next;
    uint64_t plan_parents = 0;
    // the last pop, for lx_batcher_unpop
    uint32_t last_first = 0, last_n = 0;

    lx_batcher() {
        ids.init(1 << 18);
        unknown.init(1 << 10);
    }

    int fail(int code, const char *fmt, ...) {
        char buf[256];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    uint32_t alloc_slot() {
        if (!free_slots.empty()) {
            const uint32_t s = free_slots.back();
            free_slots.pop_back();
            return s;
        }
        pend.emplace_back();
        return (uint32_t)pend.size() - 1;
    }
    uint32_t alloc_node(uint32_t child, uint32_t pos, uint32_t next_) {
        uint32_t n;
        if (!wfree.empty()) {
            n = wfree.back();
            wfree.pop_back();
            wnodes[n] = Waiter{child, pos, next_};
        } else {
            n = (uint32_t)wnodes.size();
            wnodes.push_back(Waiter{child, pos, next_});
        }
        return n;
    }
    // one parent of pending slot s (entry pos): resolved, or a waiter on it
    void link_parent(uint32_t s, uint32_t pos) {
        const uint64_t q = par_id[pos];
        const uint32_t v = ids.find(q);
        if (v != kNone && !(v & kPend)) {
            par_res[pos] = v;
            return;
        }
        par_res[pos] = kNone;
        pend[s].missing++;
        if (v != kNone) {
            Pending &p = pend[v & ~kPend];
            p.waiters = alloc_node(s, pos, p.waiters);
        } else if (uint32_t *head = unknown.ref(q)) {
            *head = alloc_node(s, pos, *head);
        } else {
            unknown.put(q, alloc_node(s, pos, kNone));
        }
    }
};

namespace {

bool by_order(const lx_batcher *b, uint32_t x, uint32_t y) { return b->pend[x].order < b->pend[y].order; }

void sort_level(lx_batcher *b, std::vector<uint32_t> &lv) {
    for (size_t i = 1; i < lv.size(); i++)
        if (b->pend[lv[i - 1]].order > b->pend[lv[i]].order) {
            std::sort(lv.begin(), lv.end(), [b](uint32_t x, uint32_t y) { return by_order(b, x, y); });
            return;
        }
}

// the levels the next pop releases (children's missing counts simulated)
void make_plan(lx_batcher *b) {
    if (b->planned) return;
    b->plan.clear();
    b->plan_levels.assign(1, 0);
    b->plan_parents = 0;
    const uint32_t st = ++b->stamp;
    std::vector<uint32_t> &cur = b->next;
    cur.assign(b->ready.begin(), b->ready.end());
    size_t lv_begin = 0;
    while (!cur.empty()) {
        sort_level(b, cur);
        lv_begin = b->plan.size();
        b->plan.insert(b->plan.end(), cur.begin(), cur.end());
        b->plan_levels.push_back((uint32_t)b->plan.size());
        cur.clear();
        for (size_t i = lv_begin; i < b->plan.size(); i++) {
            const Pending &p = b->pend[b->plan[i]];
            b->plan_parents += p.np;
            for (uint32_t w = p.waiters; w != kNone; w = b->wnodes[w].next) {
                Pending &c = b->pend[b->wnodes[w].child];
                if (c.plan_stamp != st) { c.plan_stamp = st; c.plan_cnt = 0; }
                if (++c.plan_cnt == c.missing) cur.push_back(b->wnodes[w].child);
            }
        }
    }
    b->planned = true;
}

// missing counts, parent resolutions and waiter chains recomputed from scratch
void rebuild_waits(lx_batcher *b) {
    b->wnodes.clear();
    b->wfree.clear();
    b->unknown.init(1 << 10);
    b->ready.clear();
    for (Pending &p : b->pend) p.waiters = kNone;
    for (uint32_t s = 0; s < b->pend.size(); s++) {
        Pending &p = b->pend[s];
        if (!p.live) continue;
        p.missing = 0;
        for (uint32_t k = 0; k < p.np; k++) b->link_parent(s, p.par_off + k);
    }
    std::vector<uint32_t> order;
    for (uint32_t s = 0; s < b->pend.size(); s++)
        if (b->pend[s].live && !b->pend[s].missing) b->ready.push_back(s);
    sort_level(b, b->ready);
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

int lx_batcher_reserve(lx_batcher *b, uint64_t n_events) {
    if (!b) return LX_ERR_ARG;
    if (2 * (n_events + b->ids.live) > b->ids.mask + 1) {
        // rebuild at the larger size (ids are kept)
        std::vector<IdMap::Ent> old;
        old.swap(b->ids.t);
        b->ids.init(n_events + b->ids.live);
        for (const IdMap::Ent &e : old)
            if (e.st == 1) b->ids.put(e.key, e.val);
    }
    b->released.reserve(n_events);
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
    if (b->n_pending == 0) {            // nothing pending: the parent arenas restart
        b->par_id.clear();
        b->par_res.clear();
    }
    // the batch's parents, appended once (entries of duplicates stay unused)
    const uint64_t arena0 = b->par_id.size();
    b->par_id.insert(b->par_id.end(), parent_id + parent_off[0], parent_id + parent_off[n]);
    b->par_res.resize(b->par_id.size());
    for (uint32_t i = 0; i < n; i++) {
        // the slot this event would take (the table holds it only if the id is new)
        const uint32_t s = b->free_slots.empty() ? (uint32_t)b->pend.size() : b->free_slots.back();
        uint64_t at = 0;
        const uint32_t v = b->ids.find_or_put(id[i], kPend | s, &at);
        uint8_t st = LX_PUSH_QUEUED;
        if (v != kNone) st = (v & kPend) ? LX_PUSH_DUPLICATE : LX_PUSH_CONNECTED;   // ErrDuplicateEvent / ErrAlreadyConnectedEvent
        if (out_status) out_status[i] = st;
        if (st != LX_PUSH_QUEUED) continue;
        if (b->alloc_slot() != s) return b->fail(LX_ERR_STATE, "batcher slot bookkeeping");
        Pending &p = b->pend[s];
        p.id = id[i];
        p.at = at;
        p.at_gen = b->ids.gen;
        p.creator = creator_idx[i];
        p.seq = seq[i];
        p.order = b->next_order++;
        p.live = true;
        p.missing = 0;
        p.waiters = kNone;
        p.par_off = (uint32_t)(arena0 + parent_off[i] - parent_off[0]);
        p.np = (uint32_t)(parent_off[i + 1] - parent_off[i]);
        b->n_pending++;
        // children pushed before this event wait on its id: they move to the slot
        if (b->unknown.live) {
            if (uint32_t *head = b->unknown.ref(p.id)) {
                b->pend[s].waiters = *head;
                b->unknown.erase(p.id);
            }
        }
        for (uint32_t k = 0; k < b->pend[s].np; k++) b->link_parent(s, b->pend[s].par_off + k);
        if (!b->pend[s].missing) b->ready.push_back(s);
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
    if (n_waiting) *n_waiting = b->n_pending - (uint32_t)b->plan.size();
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
        const uint32_t s = b->plan[i];
        Pending &p = b->pend[s];
        const uint32_t dense = base + i;
        // its table entry as remembered at push (one probe less per event)
        if (p.at_gen == b->ids.gen && b->ids.t[p.at].key == p.id && b->ids.t[p.at].st == 1) b->ids.t[p.at].val = dense;
        else *b->ids.ref(p.id) = dense;
        b->released.push_back(p.id);
        out_id[i] = p.id;
        out_creator[i] = p.creator;
        out_seq[i] = p.seq;
        // parents were released before p (earlier pops or earlier in this plan):
        // every entry is resolved
        const uint32_t *res = b->par_res.data() + p.par_off;
        for (uint32_t j = 0; j < p.np; j++) out_parent_idx[k++] = res[j];
        out_parent_off[i + 1] = k;
        // children waiting for p: their entry resolves, their count drops
        for (uint32_t w = p.waiters; w != kNone;) {
            const Waiter wn = b->wnodes[w];
            b->par_res[wn.pos] = dense;
            b->pend[wn.child].missing--;
            b->wfree.push_back(w);
            w = wn.next;
        }
        p.waiters = kNone;
        p.live = false;
        b->free_slots.push_back(s);
    }
    b->n_pending -= n;
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
        b->ids.erase(b->released.back());
        b->released.pop_back();
    }
    b->last_n = 0;
    rebuild_waits(b);
    return 0;
}

int lx_batcher_dense(const lx_batcher *b, uint64_t id, uint32_t *out) {
    if (!b || !out) return LX_ERR_ARG;
    const uint32_t v = b->ids.find(id);
    if (v == kNone || (v & kPend)) return LX_ERR_ARG;
    *out = v;
    return 0;
}

}  // extern "C"
