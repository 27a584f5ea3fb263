/*
 * abft_oracle.c -- plain-C restatement of abft (TEST INFRASTRUCTURE ONLY).
 *
 * The same algorithm as oracle/abft_oracle.py, event by event as the
 * reference runs it, over the C vecfc restatement (oracle.c); used by tests/
 * as the checker at sizes the Python restatement cannot reach (config C5:
 * 1000 validators) and by bench.py's cpu_baseline leg.  tests/test_oracle_c.py
 * checks it against the Python restatement (blocks, frames, roots) on
 * fork-heavy DAGs.  Never linked into the product library.
 *
 *   Process / Build           abft/indexed_lachesis.go:53-82
 *   calcFrameIdx              abft/event_processing.go:163-189 (early exit of
 *                             forklessCausedByQuorumOn, :148-161)
 *   checkAndSaveEvent/AddRoot abft/event_processing.go:50-62, store_roots.go:22-27
 *   handleElection & co       abft/event_processing.go:64-146
 *   ProcessRoot               abft/election/election_math.go:13-114
 *   chooseAtropos             abft/election/sort_roots.go:10-25
 *   onFrameDecided/seal       abft/frame_decide.go:11-58
 *   applyAtropos/confirm      abft/lachesis.go:40-86, abft/traversal.go:13-37
 *
 * Roots are kept in insertion order (see the note in abft_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NONE 0xFFFFFFFFu

/* oracle.c */
void *orc_create(uint32_t V, const uint32_t *weights);
void orc_destroy(void *h);
int orc_add(void *h, uint32_t creator, uint32_t seq, uint32_t np, const uint32_t *parents);
void orc_flush(void *h);
void orc_drop_not_flushed(void *h);
int orc_forkless_cause(void *h, uint32_t a, uint32_t b);
int orc_get_merged_hb(void *h, uint32_t id, uint8_t *out, uint32_t cap, uint32_t *len);

enum { ABO_OK = 0, ABO_ERR_ORDER = -2, ABO_ERR_FRAME = -7, ABO_ERR_BYZANTINE = -8, ABO_ERR_ARG = -1 };

typedef struct {
    void *user;
    void (*begin_block)(void *user, uint32_t frame, uint32_t atropos, const uint32_t *cheaters, uint32_t n);
    void (*apply_event)(void *user, uint32_t ev);
    int (*end_block)(void *user, uint32_t *n_validators, const uint32_t **weights);
} abo_callbacks;

typedef struct {
    uint32_t stamp;          /* election the vote belongs to */
    uint8_t decided, yes;
    uint32_t observed;       /* event, NONE = empty hash */
} vote_t;

typedef struct {
    uint32_t *ev, *creator, n, cap;
    vote_t *votes;           /* [slot][V] */
    uint32_t vcap;
} froots_t;

typedef struct {
    void *ix;
    abo_callbacks cb;
    uint32_t epoch, V, quorum, last_decided;
    uint32_t *w;
    /* events of the epoch */
    uint32_t n, cap;
    uint32_t *frame, *sp, *confirmed;
    uint64_t *poff;
    uint32_t *par;
    uint64_t npar, par_cap;
    /* roots by frame */
    froots_t *fr;
    uint32_t nfr;
    /* election */
    uint32_t frame_to_decide, stamp;
    uint8_t *dec_has;
    vote_t *dec;
    uint32_t *cnt_yes, *cnt_no, *cnt_all, cnt_stamp;
    uint32_t *map_slot;      /* round 1 observedRootsMap: creator -> slot+1 (stamped) */
    uint32_t *map_stamp;
    uint32_t *obs;           /* observed slots scratch */
    uint32_t obs_cap;
    uint32_t *stack;
    uint64_t stack_cap;
    int err;                 /* sticky election error */
    /* the caller's call sequence on the index (IndexedLachesis.Process,
     * abft/indexed_lachesis.go:69-82): counts and a running hash, see abo_trace */
    uint64_t tr_hash, tr_fc, tr_add, tr_flush, tr_drop, tr_fc_hits;
    int timing;
    double t_fc;             /* seconds inside ForklessCause (LRU included) */
    /* the reference's ForklessCause LRU (vecfc/forkless_cause.go:28-38, a
     * simplewlru of IndexCacheConfig.ForklessCausePairs entries of weight 1,
     * vecfc/index.go:52-61); 0 entries = none */
    uint32_t lru_cap, lru_n, lru_head, lru_tail, lru_mask;
    uint64_t *lru_key;
    uint8_t *lru_val;
    uint32_t *lru_prev, *lru_next, *lru_slot;   /* lru_slot: hash slot -> node + 1 */
} abo_t;

static void *xr(void *p, size_t n) {
    void *q = realloc(p, n ? n : 1);
    if (!q) abort();
    return q;
}

/* ---- call-sequence trace: h = splitmix64(h ^ record); records
 *   Add(e) (1 << 62 | e), ForklessCause(a, b) (a << 32 | b), Flush (2 << 62 |
 *   events), DropNotFlushed (3 << 62 | events after it) -- the same definition
 *   as tools/lx_dropin.cpp */
static uint64_t tr_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static void tr(abo_t *a, uint64_t rec) { a->tr_hash = tr_mix(a->tr_hash ^ rec); }

/* ---- simplewlru restated for (a, b) -> bool: hash (linear probing,
 * backward-shift deletion) + recency list */
static uint32_t lru_h(uint64_t k, uint32_t mask) { return (uint32_t)(tr_mix(k) & mask); }
static void lru_unlink(abo_t *a, uint32_t i) {
    uint32_t p = a->lru_prev[i], n = a->lru_next[i];
    if (p != NONE) a->lru_next[p] = n; else a->lru_head = n;
    if (n != NONE) a->lru_prev[n] = p; else a->lru_tail = p;
}
static void lru_front(abo_t *a, uint32_t i) {
    a->lru_prev[i] = NONE;
    a->lru_next[i] = a->lru_head;
    if (a->lru_head != NONE) a->lru_prev[a->lru_head] = i;
    a->lru_head = i;
    if (a->lru_tail == NONE) a->lru_tail = i;
}
static uint32_t lru_find(abo_t *a, uint64_t k, uint32_t *slot) {
    uint32_t h = lru_h(k, a->lru_mask);
    for (;; h = (h + 1) & a->lru_mask) {
        uint32_t v = a->lru_slot[h];
        if (!v) { *slot = h; return NONE; }
        if (a->lru_key[v - 1] == k) { *slot = h; return v - 1; }
    }
}
static void lru_erase_slot(abo_t *a, uint32_t h) {
    uint32_t i = (h + 1) & a->lru_mask;
    a->lru_slot[h] = 0;
    while (a->lru_slot[i]) {          /* backward shift */
        uint32_t v = a->lru_slot[i], want = lru_h(a->lru_key[v - 1], a->lru_mask);
        if (((i - want) & a->lru_mask) >= ((i - h) & a->lru_mask)) {
            a->lru_slot[h] = v;
            a->lru_slot[i] = 0;
            h = i;
        }
        i = (i + 1) & a->lru_mask;
    }
}
static void lru_clear(abo_t *a) {
    if (!a->lru_cap) return;
    memset(a->lru_slot, 0, (size_t)(a->lru_mask + 1) * 4u);
    a->lru_n = 0;
    a->lru_head = a->lru_tail = NONE;
}
void abo_set_fc_cache(void *h, uint32_t pairs) {
    abo_t *a = h;
    free(a->lru_key); free(a->lru_val); free(a->lru_prev); free(a->lru_next); free(a->lru_slot);
    a->lru_key = NULL; a->lru_val = NULL; a->lru_prev = a->lru_next = a->lru_slot = NULL;
    a->lru_cap = pairs;
    if (!pairs) return;
    uint32_t m = 1;
    while (m < 2 * pairs) m <<= 1;
    a->lru_mask = m - 1;
    a->lru_key = xr(NULL, (size_t)pairs * 8u);
    a->lru_val = xr(NULL, pairs);
    a->lru_prev = xr(NULL, (size_t)pairs * 4u);
    a->lru_next = xr(NULL, (size_t)pairs * 4u);
    a->lru_slot = xr(NULL, (size_t)m * 4u);
    lru_clear(a);
}

/* ForklessCause as the caller asks it (vecfc/forkless_cause.go:28-38) */
static int fc_call(abo_t *a, uint32_t x, uint32_t y) {
    const uint64_t k = ((uint64_t)x << 32) | y;
    struct timespec t0, t1;
    if (a->timing) clock_gettime(CLOCK_MONOTONIC, &t0);
    tr(a, k);
    a->tr_fc++;
    int r;
    uint32_t slot, i = a->lru_cap ? lru_find(a, k, &slot) : NONE;
    if (i != NONE) {
        lru_unlink(a, i);
        lru_front(a, i);
        r = a->lru_val[i];
        a->tr_fc_hits++;
    } else {
        r = orc_forkless_cause(a->ix, x, y);
        if (a->lru_cap) {
            if (a->lru_n == a->lru_cap) {     /* evict the oldest */
                uint32_t o = a->lru_tail, os;
                lru_find(a, a->lru_key[o], &os);
                lru_erase_slot(a, os);
                lru_unlink(a, o);
                i = o;
                lru_find(a, k, &slot);        /* the slot may have moved */
            } else {
                i = a->lru_n++;
            }
            a->lru_key[i] = k;
            a->lru_val[i] = (uint8_t)(r == 1);
            a->lru_slot[slot] = i + 1;
            lru_front(a, i);
        }
    }
    if (a->timing) {
        clock_gettime(CLOCK_MONOTONIC, &t1);
        a->t_fc += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    }
    return r;
}

static uint32_t quorum_of(const uint32_t *w, uint32_t V) {
    uint64_t t = 0;
    for (uint32_t i = 0; i < V; i++) t += w[i];
    return (uint32_t)(t * 2 / 3 + 1);
}

static void free_epoch(abo_t *a) {
    for (uint32_t f = 0; f < a->nfr; f++) { free(a->fr[f].ev); free(a->fr[f].creator); free(a->fr[f].votes); }
    free(a->fr);
    a->fr = NULL;
    a->nfr = 0;
    a->n = 0;
    a->npar = 0;
    if (a->ix) orc_destroy(a->ix);
    a->ix = NULL;
    lru_clear(a);          /* Reset purges the ForklessCause cache (vecfc/index.go:103) */
}

static void election_reset(abo_t *a, uint32_t frame_to_decide) {   /* election.go:87-93 */
    a->frame_to_decide = frame_to_decide;
    a->stamp++;
    memset(a->dec_has, 0, a->V);
}

static void new_epoch(abo_t *a, uint32_t epoch, uint32_t V, const uint32_t *w) {
    free_epoch(a);
    a->epoch = epoch;
    a->V = V;
    a->w = xr(a->w, V * 4u);
    memcpy(a->w, w, V * 4u);
    a->quorum = quorum_of(w, V);
    a->ix = orc_create(V, w);
    a->dec_has = xr(a->dec_has, V);
    a->dec = xr(a->dec, V * sizeof(vote_t));
    a->cnt_yes = xr(a->cnt_yes, V * 4u);
    a->cnt_no = xr(a->cnt_no, V * 4u);
    a->cnt_all = xr(a->cnt_all, V * 4u);
    memset(a->cnt_yes, 0, V * 4u);
    memset(a->cnt_no, 0, V * 4u);
    memset(a->cnt_all, 0, V * 4u);
    a->cnt_stamp = 0;
    a->map_slot = xr(a->map_slot, V * 4u);
    a->map_stamp = xr(a->map_stamp, V * 4u);
    memset(a->map_stamp, 0, V * 4u);
    a->last_decided = 0;
}

void *abo_create(uint32_t epoch, uint32_t V, const uint32_t *w, const abo_callbacks *cb) {
    abo_t *a = calloc(1, sizeof(abo_t));
    if (cb) a->cb = *cb;
    a->lru_head = a->lru_tail = NONE;
    new_epoch(a, epoch, V, w);
    election_reset(a, 1);
    return a;
}

void abo_destroy(void *h) {
    abo_t *a = h;
    free_epoch(a);
    free(a->w); free(a->frame); free(a->sp); free(a->confirmed); free(a->poff); free(a->par);
    free(a->dec_has); free(a->dec); free(a->cnt_yes); free(a->cnt_no); free(a->cnt_all);
    free(a->map_slot); free(a->map_stamp); free(a->obs); free(a->stack);
    abo_set_fc_cache(a, 0);
    free(a);
}

static froots_t *frame_roots(abo_t *a, uint32_t f) {
    if (f >= a->nfr) {
        uint32_t n = f + 1 > a->nfr * 2 ? f + 1 : a->nfr * 2;
        a->fr = xr(a->fr, n * sizeof(froots_t));
        memset(a->fr + a->nfr, 0, (n - a->nfr) * sizeof(froots_t));
        a->nfr = n;
    }
    return &a->fr[f];
}

static void add_root(abo_t *a, uint32_t sp_frame, uint32_t e, uint32_t frame, uint32_t creator) {
    for (uint32_t f = sp_frame + 1; f <= frame; f++) {    /* store_roots.go:22-27 */
        froots_t *r = frame_roots(a, f);
        if (r->n == r->cap) {
            r->cap = r->cap ? r->cap * 2 : 64;
            r->ev = xr(r->ev, r->cap * 4u);
            r->creator = xr(r->creator, r->cap * 4u);
        }
        r->ev[r->n] = e;
        r->creator[r->n] = creator;
        r->n++;
    }
}

static vote_t *vote_at(abo_t *a, uint32_t f, uint32_t slot) {
    froots_t *r = frame_roots(a, f);
    if (r->vcap < r->cap) {
        r->votes = xr(r->votes, (size_t)r->cap * a->V * sizeof(vote_t));
        memset(r->votes + (size_t)r->vcap * a->V, 0, (size_t)(r->cap - r->vcap) * a->V * sizeof(vote_t));
        r->vcap = r->cap;
    }
    return r->votes + (size_t)slot * a->V;
}

/* chooseAtropos (sort_roots.go:10-25): 1 decided (*atropos), 0 not, <0 error */
static int choose_atropos(abo_t *a, uint32_t *atropos) {
    for (uint32_t v = 0; v < a->V; v++) {
        if (!a->dec_has[v]) return 0;
        if (a->dec[v].yes) { *atropos = a->dec[v].observed; return 1; }
    }
    return ABO_ERR_BYZANTINE;
}

static void obs_push(abo_t *a, uint32_t *n, uint32_t slot) {
    if (*n == a->obs_cap) { a->obs_cap = a->obs_cap ? a->obs_cap * 2 : 256; a->obs = xr(a->obs, a->obs_cap * 4u); }
    a->obs[(*n)++] = slot;
}

/* ProcessRoot (election_math.go:13-114) for root slot (frame f, index k) */
static int process_root(abo_t *a, uint32_t f, uint32_t k, uint32_t *atropos) {
    int rc = choose_atropos(a, atropos);
    if (rc) return rc;
    const uint32_t F = a->frame_to_decide;
    if (f <= F) return 0;
    const uint32_t round = f - F;
    const uint32_t root = frame_roots(a, f)->ev[k];
    froots_t *prev = frame_roots(a, f - 1);
    vote_t *mine = vote_at(a, f, k);
    uint32_t nobs = 0;
    a->cnt_stamp++;                                   /* observedRootsMap stamp */
    for (uint32_t j = 0; j < prev->n; j++) {
        if (fc_call(a, root, prev->ev[j]) != 1) continue;
        if (round == 1) { a->map_slot[prev->creator[j]] = j; a->map_stamp[prev->creator[j]] = a->cnt_stamp; }
        else obs_push(a, &nobs, j);
    }
    const uint32_t mstamp = a->cnt_stamp;
    for (uint32_t v = 0; v < a->V; v++) {             /* notDecidedRoots: IDs() = idx order */
        if (a->dec_has[v]) continue;
        vote_t vote = {a->stamp, 0, 0, NONE};
        if (round == 1) {
            if (a->map_stamp[v] == mstamp) { vote.yes = 1; vote.observed = prev->ev[a->map_slot[v]]; }
        } else {
            const uint32_t cs = ++a->cnt_stamp;
            uint32_t yes = 0, no = 0, all = 0, subject = NONE;
            vote_t *pv = vote_at(a, f - 1, 0);
            for (uint32_t t = 0; t < nobs; t++) {
                const uint32_t j = a->obs[t], c = prev->creator[j];
                const vote_t *o = &pv[(size_t)j * a->V + v];
                if (o->stamp != a->stamp) return ABO_ERR_BYZANTINE;   /* every root must vote ... */
                if (o->yes && subject != NONE && subject != o->observed) return ABO_ERR_BYZANTINE;
                if (o->yes) {
                    subject = o->observed;
                    if (a->cnt_yes[c] != cs) { a->cnt_yes[c] = cs; yes += a->w[c]; }
                } else {
                    if (a->cnt_no[c] != cs) { a->cnt_no[c] = cs; no += a->w[c]; }
                }
                if (a->cnt_all[c] == cs) return ABO_ERR_BYZANTINE;    /* !allVotes.Count */
                a->cnt_all[c] = cs;
                all += a->w[c];
            }
            if (all < a->quorum) return ABO_ERR_BYZANTINE;
            vote.yes = yes >= no;
            if (vote.yes && subject != NONE) vote.observed = subject;
            vote.decided = yes >= a->quorum || no >= a->quorum;
            if (vote.decided) { a->dec_has[v] = 1; a->dec[v] = vote; }
        }
        mine[v] = vote;
    }
    return choose_atropos(a, atropos);
}

static int forkless_caused_by_quorum_on(abo_t *a, uint32_t e, uint32_t f) {   /* :148-161 */
    if (f >= a->nfr) return 0;
    froots_t *r = &a->fr[f];
    const uint32_t cs = ++a->cnt_stamp;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < r->n; j++) {
        if (fc_call(a, e, r->ev[j]) == 1) {
            uint32_t c = r->creator[j];
            if (a->cnt_all[c] != cs) { a->cnt_all[c] = cs; sum += a->w[c]; }
        }
        if (sum >= a->quorum) break;
    }
    return sum >= a->quorum;
}

static uint32_t calc_frame(abo_t *a, uint32_t e, uint32_t claimed, int check_only, uint32_t *sp_frame) {
    *sp_frame = a->sp[e] == NONE ? 0 : a->frame[a->sp[e]];
    uint32_t max = check_only ? claimed : *sp_frame + 100;
    uint32_t f = *sp_frame;
    while (f < max && forkless_caused_by_quorum_on(a, e, f)) f++;
    return f == 0 ? 1 : f;
}

static int add_event(abo_t *a, uint32_t creator, uint32_t seq, uint32_t np, const uint32_t *parents) {
    tr(a, (1ull << 62) | a->n);
    a->tr_add++;
    int rc = orc_add(a->ix, creator, seq, np, parents);
    if (rc) return rc == -1 ? ABO_ERR_ORDER : ABO_ERR_ARG;
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 1024;
        a->frame = xr(a->frame, a->cap * 4u);
        a->sp = xr(a->sp, a->cap * 4u);
        a->confirmed = xr(a->confirmed, a->cap * 4u);
        a->poff = xr(a->poff, (a->cap + 1) * 8u);
    }
    if (a->n == 0) a->poff[0] = 0;
    if (a->npar + np > a->par_cap) { a->par_cap = (a->npar + np) * 2; a->par = xr(a->par, a->par_cap * 4u); }
    memcpy(a->par + a->npar, parents, np * 4u);
    a->npar += np;
    a->frame[a->n] = 0;
    a->sp[a->n] = (seq > 1 && np > 0) ? parents[0] : NONE;
    a->confirmed[a->n] = 0;
    a->n++;
    a->poff[a->n] = a->npar;
    return 0;
}

static void drop_event(abo_t *a) {     /* DropNotFlushed of the last Add */
    orc_drop_not_flushed(a->ix);
    a->n--;
    a->npar = a->poff[a->n];
    lru_clear(a);          /* dense indices are reused after a rollback (hashes are not) */
}

/* the deferred DropNotFlushed of Process / Build, as a call (a no-op after Flush) */
static void tr_drop(abo_t *a) {
    tr(a, (3ull << 62) | a->n);
    a->tr_drop++;
}

/* applyAtropos (lachesis.go:57-86) + onFrameDecided (frame_decide.go:11-35);
 * returns 1 when the epoch was sealed */
static int on_frame_decided(abo_t *a, uint32_t frame, uint32_t atropos) {
    uint32_t len = 0;
    uint8_t *m = xr(NULL, 8u * a->V + 8u * 4096u);
    orc_get_merged_hb(a->ix, atropos, NULL, 0, &len);
    m = xr(m, len + 8);
    orc_get_merged_hb(a->ix, atropos, m, len, &len);
    uint32_t *cheaters = xr(NULL, (a->V + 1) * 4u), nch = 0;
    for (uint32_t c = 0; c < a->V && 8u * c + 8u <= len; c++) {
        uint32_t s, ms;
        memcpy(&s, m + 8u * c, 4);
        memcpy(&ms, m + 8u * c + 4, 4);
        if (s == 0 && ms == 0x7FFFFFFFu) cheaters[nch++] = c;
    }
    free(m);
    int sealed = 0;
    uint32_t nv = 0;
    const uint32_t *nw = NULL;
    if (a->cb.begin_block) {
        a->cb.begin_block(a->cb.user, frame, atropos, cheaters, nch);
        uint64_t sp = 0;                                  /* dfsSubgraph (traversal.go:13-37) */
        for (uint32_t walk = atropos;;) {
            if (a->confirmed[walk] == 0) {
                a->confirmed[walk] = frame;
                if (a->cb.apply_event) a->cb.apply_event(a->cb.user, walk);
                uint64_t np = a->poff[walk + 1] - a->poff[walk];
                if (sp + np > a->stack_cap) { a->stack_cap = (sp + np) * 2; a->stack = xr(a->stack, a->stack_cap * 4u); }
                for (uint64_t k = 0; k < np; k++) a->stack[sp++] = a->par[a->poff[walk] + k];
            }
            if (!sp) break;
            walk = a->stack[--sp];
        }
        if (a->cb.end_block && a->cb.end_block(a->cb.user, &nv, &nw)) sealed = 1;
    }
    free(cheaters);
    if (sealed) {
        uint32_t *w = xr(NULL, nv * 4u);
        memcpy(w, nw, nv * 4u);
        new_epoch(a, a->epoch + 1, nv, w);               /* sealEpoch + resetEpochStore */
        free(w);
        election_reset(a, 1);
        return 1;
    }
    a->last_decided = frame;
    election_reset(a, frame + 1);
    return 0;
}

static int bootstrap_election(abo_t *a) {                /* event_processing.go:102-146 */
    for (;;) {
        uint32_t atropos = NONE;
        int rc = 0;
        for (uint32_t f = a->last_decided + 1;; f++) {
            froots_t *r = f < a->nfr ? &a->fr[f] : NULL;
            uint32_t nr = r ? r->n : 0;
            for (uint32_t k = 0; k < nr && !rc; k++) rc = process_root(a, f, k, &atropos);
            if (rc || nr == 0) break;
        }
        if (rc < 0) return rc;
        if (rc == 0) return 0;
        if (on_frame_decided(a, a->frame_to_decide, atropos)) return 1;
    }
}

/* IndexedLachesis.Process; claimed = NONE: Build first (frame computed as
 * Build does).  Returns 0, 1 = sealed the epoch, or an error. */
int abo_process(void *h, uint32_t creator, uint32_t seq, uint32_t np, const uint32_t *parents, uint32_t claimed,
                uint32_t *out_frame) {
    abo_t *a = h;
    int rc = add_event(a, creator, seq, np, parents);
    if (rc) return rc;
    const uint32_t e = a->n - 1;
    uint32_t sp_frame;
    if (claimed == NONE) claimed = calc_frame(a, e, 0, 0, &sp_frame);   /* Build */
    uint32_t f = calc_frame(a, e, claimed, 1, &sp_frame);
    if (f != claimed) { drop_event(a); tr_drop(a); return ABO_ERR_FRAME; }
    a->frame[e] = f;
    if (out_frame) *out_frame = f;
    if (sp_frame != f) add_root(a, sp_frame, e, f, creator);
    int sealed = 0;
    for (uint32_t g = sp_frame + 1; g <= f; g++) {        /* handleElection :64-100 */
        froots_t *r = frame_roots(a, g);
        uint32_t k = NONE;
        for (uint32_t j = r->n; j-- > 0;) if (r->ev[j] == e) { k = j; break; }
        uint32_t atropos;
        rc = process_root(a, g, k, &atropos);
        if (rc < 0) return rc;
        if (rc == 0) continue;
        if (on_frame_decided(a, a->frame_to_decide, atropos)) { sealed = 1; break; }
        rc = bootstrap_election(a);
        if (rc < 0) return rc;
        if (rc == 1) { sealed = 1; break; }
    }
    if (!sealed) orc_flush(a->ix);
    tr(a, (2ull << 62) | a->n);           /* IndexedLachesis.Process: Flush, then the deferred drop */
    a->tr_flush++;
    tr_drop(a);
    return sealed;
}

int abo_build(void *h, uint32_t creator, uint32_t seq, uint32_t np, const uint32_t *parents, uint32_t *out_frame) {
    abo_t *a = h;
    int rc = add_event(a, creator, seq, np, parents);
    if (rc) return rc;
    uint32_t sp_frame;
    *out_frame = calc_frame(a, a->n - 1, 0, 0, &sp_frame);
    drop_event(a);
    tr_drop(a);
    return 0;
}

/* batch driver with the semantics of lx_abft_process_batch */
int abo_process_batch(void *h, uint32_t n, const uint32_t *creator, const uint32_t *seq, const uint64_t *poff,
                      const uint32_t *par, const uint32_t *claimed, uint32_t *out_frame, uint32_t *consumed) {
    *consumed = 0;
    for (uint32_t i = 0; i < n; i++) {
        int rc = abo_process(h, creator[i], seq[i], (uint32_t)(poff[i + 1] - poff[i]), par + poff[i],
                             claimed ? claimed[i] : NONE, out_frame ? out_frame + i : NULL);
        if (rc < 0) return rc;
        *consumed = i + 1;
        if (rc == 1) return 0;
    }
    return 0;
}

/* out[0] call-sequence hash, [1] ForklessCause calls, [2] of them LRU hits,
 * [3] Adds, [4] Flushes, [5] DropNotFlushed calls */
void abo_trace(void *h, uint64_t out[6]) {
    abo_t *a = h;
    out[0] = a->tr_hash; out[1] = a->tr_fc; out[2] = a->tr_fc_hits;
    out[3] = a->tr_add; out[4] = a->tr_flush; out[5] = a->tr_drop;
}
void abo_set_timing(void *h, int on) { ((abo_t *)h)->timing = on; }
double abo_fc_seconds(void *h) { return ((abo_t *)h)->t_fc; }

uint32_t abo_epoch(void *h) { return ((abo_t *)h)->epoch; }
uint32_t abo_last_decided_frame(void *h) { return ((abo_t *)h)->last_decided; }
uint32_t abo_num_events(void *h) { return ((abo_t *)h)->n; }
uint32_t abo_event_frame(void *h, uint32_t e) { abo_t *a = h; return e < a->n ? a->frame[e] : 0; }
uint32_t abo_frame_roots(void *h, uint32_t f, uint32_t *out, uint32_t cap) {
    abo_t *a = h;
    if (f >= a->nfr) return 0;
    uint32_t n = a->fr[f].n;
    if (out) memcpy(out, a->fr[f].ev, (n < cap ? n : cap) * 4u);
    return n;
}
