/*
 * oracle.c -- plain-C restatement of vecengine + vecfc (TEST INFRASTRUCTURE ONLY).
 *
 * Used by tests/ as the large-size checker for the HIP path and by bench.py's
 * cpu_baseline leg (kind "port").  Never linked into the product library.
 *
 * Follows the same reference code as oracle/vecfc_oracle.py (which is pinned
 * to the reference's golden FC tables); tests/test_oracle_c.py checks this C
 * restatement byte-for-byte against the Python one on fork-heavy DAGs.
 *
 *   fillGlobalBranchID      vecengine/index.go:105-141
 *   fillEventVectors        vecengine/index.go:144-233 (CollectFrom x parents,
 *                           fork loops, DfsSubgraph + LowestAfter.Visit)
 *   DfsSubgraph             vecengine/traversal.go:13-37
 *   CollectFrom/GatherFrom  vecfc/vector_ops.go:49-96
 *   ForklessCause           vecfc/forkless_cause.go:40-82
 *   WeightCounter / quorum  inter/pos/stake.go:31-60, validators.go:187-189
 *   Flush/DropNotFlushed    vecengine/index.go:78-96 (flushable overlay)
 *
 * Vectors are stored in the reference byte encodings (LE u32 rows; HB =
 * Seq||MinSeq pairs, fork marker {0, MaxInt32}).  Storage is a flushable
 * overlay over dense event ids (the Go side keys by hash; ids here are the
 * dense Add-order indices).  Rows are mutated in the dirty overlay instead of
 * being copied on every Get/Put, so this baseline is at least as fast as the
 * reference's own kvdb-backed path.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAX_INT32 0x7FFFFFFFu

typedef struct {
    uint8_t *p;
    uint32_t len;
    uint32_t cap;
} row_t;

typedef struct {
    row_t *flushed;      /* [ncap] */
    row_t *dirty;        /* [ncap] */
    uint8_t *has_dirty;  /* [ncap] */
    uint32_t *dirty_keys;
    uint64_t n_dirty;
} table_t;

typedef struct {
    uint32_t *last_seq, *creator, n, cap;
    uint32_t **by_creator, *by_len, *by_cap;
} binfo_t;

typedef struct {
    uint32_t V;
    uint32_t *weights;
    uint32_t quorum;
    uint64_t ncap;
    uint64_t n_events;          /* events added (incl. unflushed) */
    uint64_t n_flushed;
    /* event metadata (the getEvent callback in the reference) */
    uint32_t *ev_creator, *ev_seq, *ev_poff, *ev_np;
    uint32_t *parents;
    uint64_t parents_len, parents_cap;
    table_t hb, la, br;         /* tables S, s, b */
    binfo_t bi;                 /* live (nil-able in the reference) */
    binfo_t bi_flushed;
    int bi_live;
    int bi_stored;
    uint32_t *stack;
    uint64_t stack_cap;
    uint8_t *counter;           /* WeightCounter.already */
} orc_t;

static void *xrealloc(void *p, size_t n) {
    void *q = realloc(p, n ? n : 1);
    if (!q) abort();
    return q;
}

/* ---------------- rows (vecfc/vector.go) ---------------- */
static void row_reserve(row_t *r, uint32_t len) {
    if (len > r->cap) {
        uint32_t c = r->cap ? r->cap : 32;
        while (c < len) c *= 2;
        r->p = xrealloc(r->p, c);
        r->cap = c;
    }
}
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

static uint32_t la_get(const row_t *r, uint32_t i) { return (4u * i + 4u <= r->len) ? rd32(r->p + 4u * i) : 0; }
static void la_set(row_t *r, uint32_t i, uint32_t seq) {
    if (4u * i + 4u > r->len) { row_reserve(r, 4u * i + 4u); memset(r->p + r->len, 0, 4u * i + 4u - r->len); r->len = 4u * i + 4u; }
    wr32(r->p + 4u * i, seq);
}
static void hb_get(const row_t *r, uint32_t i, uint32_t *s, uint32_t *m) {
    if (8u * i + 8u <= r->len) { *s = rd32(r->p + 8u * i); *m = rd32(r->p + 8u * i + 4u); }
    else { *s = 0; *m = 0; }
}
static void hb_set(row_t *r, uint32_t i, uint32_t s, uint32_t m) {
    if (8u * i + 8u > r->len) { row_reserve(r, 8u * i + 8u); memset(r->p + r->len, 0, 8u * i + 8u - r->len); r->len = 8u * i + 8u; }
    wr32(r->p + 8u * i, s);
    wr32(r->p + 8u * i + 4u, m);
}
static int is_fork(uint32_t s, uint32_t m) { return s == 0 && m == MAX_INT32; }

/* ---------------- flushable overlay ---------------- */
static void tbl_grow(table_t *t, uint64_t oldcap, uint64_t ncap) {
    t->flushed = xrealloc(t->flushed, ncap * sizeof(row_t));
    t->dirty = xrealloc(t->dirty, ncap * sizeof(row_t));
    t->has_dirty = xrealloc(t->has_dirty, ncap);
    t->dirty_keys = xrealloc(t->dirty_keys, ncap * sizeof(uint32_t));
    memset(t->flushed + oldcap, 0, (ncap - oldcap) * sizeof(row_t));
    memset(t->dirty + oldcap, 0, (ncap - oldcap) * sizeof(row_t));
    memset(t->has_dirty + oldcap, 0, ncap - oldcap);
}
static row_t *tbl_get(table_t *t, uint64_t k) {     /* NULL if absent */
    if (t->has_dirty[k]) return &t->dirty[k];
    if (t->flushed[k].len || t->flushed[k].p) return &t->flushed[k];
    return NULL;
}
static row_t *tbl_put_begin(table_t *t, uint64_t k) {  /* copy-on-write into the overlay */
    if (!t->has_dirty[k]) {
        row_t *f = &t->flushed[k];
        row_t *d = &t->dirty[k];
        row_reserve(d, f->len);
        if (f->len) memcpy(d->p, f->p, f->len);
        d->len = f->len;
        t->has_dirty[k] = 1;
        t->dirty_keys[t->n_dirty++] = (uint32_t)k;
    }
    return &t->dirty[k];
}
static void tbl_flush(table_t *t) {
    for (uint64_t i = 0; i < t->n_dirty; i++) {
        uint32_t k = t->dirty_keys[i];
        row_t tmp = t->flushed[k];
        t->flushed[k] = t->dirty[k];
        if (!t->flushed[k].p) t->flushed[k].p = xrealloc(NULL, 1);
        t->dirty[k] = tmp;
        t->dirty[k].len = 0;
        t->has_dirty[k] = 0;
    }
    t->n_dirty = 0;
}
static void tbl_drop(table_t *t) {
    for (uint64_t i = 0; i < t->n_dirty; i++) {
        uint32_t k = t->dirty_keys[i];
        t->dirty[k].len = 0;
        t->has_dirty[k] = 0;
    }
    t->n_dirty = 0;
}
static void tbl_free(table_t *t, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) { free(t->flushed[i].p); free(t->dirty[i].p); }
    free(t->flushed); free(t->dirty); free(t->has_dirty); free(t->dirty_keys);
}

/* ---------------- BranchesInfo (vecengine/branches_info.go) ---------------- */
static void bi_free(binfo_t *b, uint32_t V) {
    if (b->by_creator) for (uint32_t i = 0; i < V; i++) free(b->by_creator[i]);
    free(b->by_creator); free(b->by_len); free(b->by_cap); free(b->last_seq); free(b->creator);
    memset(b, 0, sizeof(*b));
}
static void bi_push(binfo_t *b, uint32_t last_seq, uint32_t creator) {
    if (b->n == b->cap) {
        b->cap = b->cap ? b->cap * 2 : 16;
        b->last_seq = xrealloc(b->last_seq, b->cap * 4u);
        b->creator = xrealloc(b->creator, b->cap * 4u);
    }
    b->last_seq[b->n] = last_seq;
    b->creator[b->n] = creator;
    b->n++;
}
static void bi_by_push(binfo_t *b, uint32_t c, uint32_t br) {
    if (b->by_len[c] == b->by_cap[c]) {
        b->by_cap[c] = b->by_cap[c] ? b->by_cap[c] * 2 : 4;
        b->by_creator[c] = xrealloc(b->by_creator[c], b->by_cap[c] * 4u);
    }
    b->by_creator[c][b->by_len[c]++] = br;
}
static void bi_initial(binfo_t *b, uint32_t V) {   /* newInitialBranchesInfo :27-45 */
    memset(b, 0, sizeof(*b));
    b->by_creator = calloc(V ? V : 1, sizeof(uint32_t *));
    b->by_len = calloc(V ? V : 1, 4);
    b->by_cap = calloc(V ? V : 1, 4);
    for (uint32_t i = 0; i < V; i++) { bi_push(b, 0, i); bi_by_push(b, i, i); }
}
static void bi_copy(binfo_t *dst, const binfo_t *src, uint32_t V) {
    bi_free(dst, V);
    memset(dst, 0, sizeof(*dst));
    dst->by_creator = calloc(V ? V : 1, sizeof(uint32_t *));
    dst->by_len = calloc(V ? V : 1, 4);
    dst->by_cap = calloc(V ? V : 1, 4);
    for (uint32_t i = 0; i < src->n; i++) bi_push(dst, src->last_seq[i], src->creator[i]);
    for (uint32_t c = 0; c < V; c++)
        for (uint32_t k = 0; k < src->by_len[c]; k++) bi_by_push(dst, c, src->by_creator[c][k]);
}

static void init_branches_info(orc_t *o) {          /* InitBranchesInfo :16-25 */
    if (o->bi_live) return;
    if (o->bi_stored) bi_copy(&o->bi, &o->bi_flushed, o->V);
    else { bi_free(&o->bi, o->V); bi_initial(&o->bi, o->V); }
    o->bi_live = 1;
}

/* ---------------- API ---------------- */
void *orc_create(uint32_t V, const uint32_t *weights) {
    orc_t *o = calloc(1, sizeof(orc_t));
    o->V = V;
    o->weights = xrealloc(NULL, (V ? V : 1) * 4u);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < V; i++) { o->weights[i] = weights[i]; tot += weights[i]; }
    o->quorum = (uint32_t)(tot * 2 / 3 + 1);   /* tot <= MaxUint32/2 (validators.go:108) */
    o->counter = calloc(V ? V : 1, 1);
    return o;
}

void orc_destroy(void *h) {
    orc_t *o = h;
    tbl_free(&o->hb, o->ncap); tbl_free(&o->la, o->ncap); tbl_free(&o->br, o->ncap);
    bi_free(&o->bi, o->V); bi_free(&o->bi_flushed, o->V);
    free(o->ev_creator); free(o->ev_seq); free(o->ev_poff); free(o->ev_np); free(o->parents);
    free(o->stack); free(o->weights); free(o->counter); free(o);
}

static void ensure_cap(orc_t *o, uint64_t n) {
    if (n <= o->ncap) return;
    uint64_t c = o->ncap ? o->ncap : 1024;
    while (c < n) c *= 2;
    tbl_grow(&o->hb, o->ncap, c); tbl_grow(&o->la, o->ncap, c); tbl_grow(&o->br, o->ncap, c);
    o->ev_creator = xrealloc(o->ev_creator, c * 4); o->ev_seq = xrealloc(o->ev_seq, c * 4);
    o->ev_poff = xrealloc(o->ev_poff, c * 4); o->ev_np = xrealloc(o->ev_np, c * 4);
    o->ncap = c;
}

static uint32_t get_branch(orc_t *o, uint32_t id) {
    row_t *r = tbl_get(&o->br, id);
    return r ? rd32(r->p) : 0;
}

/* returns 0 ok, -1 parent not found / out of order, -2 bad creator */
int orc_add(void *h, uint32_t creator, uint32_t seq, uint32_t np, const uint32_t *parents) {
    orc_t *o = h;
    if (creator >= o->V) return -2;
    uint64_t id = o->n_events;
    ensure_cap(o, id + 1);
    init_branches_info(o);
    binfo_t *bi = &o->bi;
    uint32_t n_before = bi->n;

    /* fillGlobalBranchID (index.go:105-141) */
    uint32_t me_br = UINT32_MAX;
    int has_sp = (seq > 1 && np > 0);
    if (!has_sp) {
        if (bi->last_seq[creator] == 0) { bi->last_seq[creator] = seq; me_br = creator; }
    } else {
        if (parents[0] >= id || !tbl_get(&o->br, parents[0])) return -1;
        uint32_t spb = get_branch(o, parents[0]);
        if (bi->last_seq[spb] + 1 == seq) { bi->last_seq[spb] = seq; me_br = spb; }
    }
    if (me_br == UINT32_MAX) {
        bi_push(bi, seq, creator);
        me_br = bi->n - 1;
        bi_by_push(bi, creator, me_br);
    }
    for (uint32_t k = 0; k < np; k++)
        if (parents[k] >= id || !tbl_get(&o->hb, parents[k])) return -1;

    /* record event (getEvent callback) */
    o->ev_creator[id] = creator; o->ev_seq[id] = seq; o->ev_np[id] = np;
    if (o->parents_len + np > o->parents_cap) {
        uint64_t c = o->parents_cap ? o->parents_cap : 4096;
        while (c < o->parents_len + np) c *= 2;
        o->parents = xrealloc(o->parents, c * 4); o->parents_cap = c;
    }
    o->ev_poff[id] = (uint32_t)o->parents_len;
    memcpy(o->parents + o->parents_len, parents, np * 4u);
    o->parents_len += np;

    uint32_t nb = bi->n;
    row_t *hb = tbl_put_begin(&o->hb, id);
    hb->len = 0; row_reserve(hb, 8u * n_before); memset(hb->p, 0, 8u * n_before); hb->len = 8u * n_before;
    row_t *la = tbl_put_begin(&o->la, id);
    la->len = 0; row_reserve(la, 4u * n_before); memset(la->p, 0, 4u * n_before); la->len = 4u * n_before;

    la_set(la, me_br, seq);                  /* InitWithEvent */
    hb_set(hb, me_br, seq, seq);
    for (uint32_t k = 0; k < np; k++) {      /* CollectFrom (vector_ops.go:49-79) */
        row_t *pv = tbl_get(&o->hb, parents[k]);
        for (uint32_t b = 0; b < nb; b++) {
            uint32_t hs, hm; hb_get(pv, b, &hs, &hm);
            if (hs == 0 && !is_fork(hs, hm)) continue;
            uint32_t ms, mm; hb_get(hb, b, &ms, &mm);
            if (is_fork(ms, mm)) continue;
            if (is_fork(hs, hm)) { hb_set(hb, b, 0, MAX_INT32); continue; }
            if (ms == 0 || mm > hm) { mm = hm; hb_set(hb, b, ms, mm); }
            if (ms < hs) { ms = hs; hb_set(hb, b, ms, mm); }
        }
    }
    if (nb > o->V) {                          /* fork loops (index.go:173-209) */
        for (uint32_t n = 0; n < o->V; n++) {
            if (bi->by_len[n] <= 1) continue;
            for (uint32_t k = 0; k < bi->by_len[n]; k++) {
                uint32_t s, m; hb_get(hb, bi->by_creator[n][k], &s, &m);
                if (is_fork(s, m)) {
                    for (uint32_t q = 0; q < bi->by_len[n]; q++) hb_set(hb, bi->by_creator[n][q], 0, MAX_INT32);
                    break;
                }
            }
        }
        for (uint32_t n = 0; n < o->V; n++) {
            uint32_t s0, m0; hb_get(hb, n, &s0, &m0);
            if (is_fork(s0, m0)) continue;
            int hit = 0;
            for (uint32_t x = 0; x < bi->by_len[n] && !hit; x++) {
                for (uint32_t y = 0; y < bi->by_len[n] && !hit; y++) {
                    uint32_t a = bi->by_creator[n][x], b = bi->by_creator[n][y];
                    if (a == b) continue;
                    uint32_t as, am, bs, bm;
                    hb_get(hb, a, &as, &am); hb_get(hb, b, &bs, &bm);
                    if ((!is_fork(as, am) && as == 0) || (!is_fork(bs, bm) && bs == 0)) continue;
                    if (am <= bs && bm <= as) hit = 1;
                }
            }
            if (hit) for (uint32_t q = 0; q < bi->by_len[n]; q++) hb_set(hb, bi->by_creator[n][q], 0, MAX_INT32);
        }
    }
    /* DfsSubgraph + onWalk (traversal.go:13-37, index.go:212-225) */
    uint64_t sp = 0;
    if (o->stack_cap < np + 1) { o->stack_cap = np + 1024; o->stack = xrealloc(o->stack, o->stack_cap * 4); }
    for (uint32_t k = 0; k < np; k++) o->stack[sp++] = parents[k];
    while (sp) {
        uint32_t cur = o->stack[--sp];
        row_t *cr = tbl_get(&o->la, cur);
        if (la_get(cr, me_br) != 0) continue;                 /* Visit -> false */
        cr = tbl_put_begin(&o->la, cur);
        la_set(cr, me_br, seq);                               /* SetLowestAfter */
        uint32_t cnp = o->ev_np[cur];
        if (sp + cnp > o->stack_cap) { o->stack_cap = (sp + cnp) * 2; o->stack = xrealloc(o->stack, o->stack_cap * 4); }
        for (uint32_t k = 0; k < cnp; k++) o->stack[sp++] = o->parents[o->ev_poff[cur] + k];
    }
    row_t *br = tbl_put_begin(&o->br, id);
    row_reserve(br, 4); br->len = 4; wr32(br->p, me_br);
    o->n_events = id + 1;
    return 0;
}

void orc_flush(void *h) {                        /* Engine.Flush :78-85 */
    orc_t *o = h;
    if (o->bi_live) { bi_copy(&o->bi_flushed, &o->bi, o->V); o->bi_stored = 1; }
    tbl_flush(&o->hb); tbl_flush(&o->la); tbl_flush(&o->br);
    o->n_flushed = o->n_events;
}

void orc_drop_not_flushed(void *h) {             /* Engine.DropNotFlushed :88-96 */
    orc_t *o = h;
    o->bi_live = 0;
    tbl_drop(&o->hb); tbl_drop(&o->la); tbl_drop(&o->br);
    o->n_events = o->n_flushed;
}

uint64_t orc_num_events(void *h) { return ((orc_t *)h)->n_events; }
uint32_t orc_num_branches(void *h) { orc_t *o = h; init_branches_info(o); return o->bi.n; }

int orc_get_branch(void *h, uint32_t id, uint32_t *out) {
    orc_t *o = h;
    if (id >= o->n_events) return -1;
    *out = get_branch(o, id);
    return 0;
}

static int copy_row(row_t *r, uint8_t *out, uint32_t cap, uint32_t *len) {
    if (!r) return -1;
    *len = r->len;
    if (out && cap) memcpy(out, r->p, r->len < cap ? r->len : cap);
    return 0;
}
int orc_get_hb(void *h, uint32_t id, uint8_t *out, uint32_t cap, uint32_t *len) {
    orc_t *o = h;
    if (id >= o->n_events) return -1;
    return copy_row(tbl_get(&o->hb, id), out, cap, len);
}
int orc_get_la(void *h, uint32_t id, uint8_t *out, uint32_t cap, uint32_t *len) {
    orc_t *o = h;
    if (id >= o->n_events) return -1;
    return copy_row(tbl_get(&o->la, id), out, cap, len);
}

/* rows of n events (mode 0 HighestBefore, 1 LowestAfter) back to back:
 * off[n + 1] byte offsets (always filled); out may be NULL to size; returns
 * -1 on an unknown event or a short buffer */
int orc_get_rows(void *h, int mode, uint64_t n, const uint32_t *ev, uint64_t *off, uint8_t *out, uint64_t cap) {
    orc_t *o = h;
    uint64_t k = 0;
    off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (ev[i] >= o->n_events) return -1;
        const row_t *r = tbl_get(mode ? &o->la : &o->hb, ev[i]);
        const uint32_t len = r ? r->len : 0;
        if (out) {
            if (k + len > cap) return -1;
            if (len) memcpy(out + k, r->p, len);
        }
        k += len;
        off[i + 1] = k;
    }
    return 0;
}

/* GetMergedHighestBefore (index.go:235-250) + GatherFrom (vector_ops.go:81-96) */
int orc_get_merged_hb(void *h, uint32_t id, uint8_t *out, uint32_t cap, uint32_t *len) {
    orc_t *o = h;
    if (id >= o->n_events) return -1;
    init_branches_info(o);
    row_t *r = tbl_get(&o->hb, id);
    if (o->bi.n <= o->V) return copy_row(r, out, cap, len);
    *len = 8u * o->V;
    for (uint32_t c = 0; c < o->V; c++) {
        uint32_t bs = 0, bm = 0;
        for (uint32_t k = 0; k < o->bi.by_len[c]; k++) {
            uint32_t s, m; hb_get(r, o->bi.by_creator[c][k], &s, &m);
            if (is_fork(s, m)) { bs = s; bm = m; break; }
            if (s > bs) { bs = s; bm = m; }
        }
        if (out && 8u * c + 8u <= cap) { wr32(out + 8u * c, bs); wr32(out + 8u * c + 4u, bm); }
    }
    return 0;
}

/* ForklessCause (forkless_cause.go:40-82) with caller-provided WeightCounter
 * scratch (V bytes); returns 0/1, -1 unknown event.  Read-only on the index
 * once BranchesInfo is initialised. */
static int fc_one(orc_t *o, uint32_t a, uint32_t b, uint8_t *counter) {
    if (a >= o->n_events || b >= o->n_events) return -1;
    row_t *ha = tbl_get(&o->hb, a);
    if (o->bi.n > o->V) {
        uint32_t s, m; hb_get(ha, get_branch(o, b), &s, &m);
        if (is_fork(s, m)) return 0;
    }
    row_t *lb = tbl_get(&o->la, b);
    memset(counter, 0, o->V);
    uint32_t sum = 0;
    for (uint32_t br = 0; br < o->bi.n; br++) {
        uint32_t l = la_get(lb, br);
        uint32_t s, m; hb_get(ha, br, &s, &m);
        if (l <= s && l != 0 && !is_fork(s, m)) {
            uint32_t c = o->bi.creator[br];
            if (!counter[c]) { counter[c] = 1; sum += o->weights[c]; }
        }
    }
    return sum >= o->quorum;
}

int orc_forkless_cause(void *h, uint32_t a, uint32_t b) {
    orc_t *o = h;
    init_branches_info(o);
    return fc_one(o, a, b, o->counter);
}

void orc_forkless_cause_batch(void *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out) {
    for (uint64_t i = 0; i < n; i++) out[i] = (uint8_t)orc_forkless_cause(h, a[i], b[i]);
}

/* The same over `threads` OpenMP threads (the multi-core CPU baseline of
 * SURVEY 8d; the reference's own index is single-threaded by contract). */
void orc_forkless_cause_batch_mt(void *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out,
                                 int threads) {
    orc_t *o = h;
    init_branches_info(o);
#pragma omp parallel num_threads(threads)
    {
        uint8_t *counter = malloc(o->V ? o->V : 1);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) out[i] = (uint8_t)fc_one(o, a[i], b[i], counter);
        free(counter);
    }
}

/* bulk add of a CSR batch; returns index of first failing event or -1 */
int64_t orc_add_batch(void *h, uint64_t n, const uint32_t *creator, const uint32_t *seq,
                      const uint64_t *poff, const uint32_t *parents, int flush_each) {
    for (uint64_t i = 0; i < n; i++) {
        if (orc_add(h, creator[i], seq[i], (uint32_t)(poff[i + 1] - poff[i]), parents + poff[i]) != 0)
            return (int64_t)i;
        if (flush_each) orc_flush(h);
    }
    return -1;
}
