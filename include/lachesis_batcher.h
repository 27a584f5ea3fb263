/*
 * lachesis_batcher.h -- host-side level-synchronous DAG batcher in front of
 * lx_add_batch (BASELINE north_star (1)).
 *
 * Role in the reference: events reach IndexedLachesis.Process one by one,
 * parents first, through gossip/dagordering.EventsBuffer
 * (gossip/dagordering/event_buffer.go:53-110: incomplete events wait until
 * every parent is known; duplicates are dropped with ErrDuplicateEvent, events
 * already connected with ErrAlreadyConnectedEvent, eventcheck/errors.go).
 * The batcher does the same buffering for the GPU index, but releases work in
 * bulk: lx_batcher_pop returns every event whose ancestors are all known, as
 * one parents-first batch grouped into topological levels (level = 1 + the
 * highest level of its parents inside the batch, parents released earlier
 * count as level 0; the events of one level are an antichain), in the form
 * lx_add_batch takes (dense parent indices continuing the epoch's Add order).
 * Inside a level, events keep their push order.  Indexing a popped batch with
 * lx_add_batch is bit-exact to calling the reference's Add for its events in
 * that order (include/lachesis_hip.h).
 *
 * Events are named by caller-chosen distinct uint64 ids (the cgo shim uses a
 * handle per hash.Event).  Host-only: no GPU work, one host thread per handle.
 * Return codes: 0 ok, < 0 error (LX_ERR_* of lachesis_hip.h).
 */
#ifndef LACHESIS_BATCHER_H
#define LACHESIS_BATCHER_H

#include "lachesis_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lx_batcher lx_batcher;

#define LX_PUSH_QUEUED 0u       /* waiting for parents or ready for the next pop */
#define LX_PUSH_DUPLICATE 1u    /* already pending (ErrDuplicateEvent) */
#define LX_PUSH_CONNECTED 2u    /* already released in this epoch (ErrAlreadyConnectedEvent) */

int lx_batcher_create(lx_batcher **out);
void lx_batcher_destroy(lx_batcher *b);
const char *lx_batcher_last_error(const lx_batcher *b);

/* New epoch: nothing released, nothing pending (dense indices restart at 0,
 * as after lx_reset). */
int lx_batcher_reset(lx_batcher *b);

/* Capacity hint: room for the ids of n events in this epoch (as
 * lx_config.event_capacity for the index); the id table otherwise grows, and
 * rehashes, as the epoch fills.  No effect on results. */
int lx_batcher_reserve(lx_batcher *b, uint64_t n_events);

/* Push n events: id, creator idx, seq, parents by id (parent_off has n+1
 * entries into parent_id; self-parent first).  out_status (optional, n
 * entries) receives LX_PUSH_*. */
int lx_batcher_push(lx_batcher *b, uint32_t n, const uint64_t *id, const uint32_t *creator_idx, const uint32_t *seq,
                    const uint64_t *parent_off, const uint64_t *parent_id, uint8_t *out_status);

/* Sizes of the next pop: events, parent entries, levels; and events still
 * waiting for a parent after it. */
int lx_batcher_peek(lx_batcher *b, uint32_t *n_events, uint64_t *n_parents, uint32_t *n_levels, uint32_t *n_waiting);

/* Release the batch lx_batcher_peek described.  Outputs (caller-allocated,
 * sizes from peek): out_id[n], out_creator[n], out_seq[n],
 * out_parent_off[n+1] (into out_parent_idx, starting at 0), out_parent_idx
 * (dense indices of this epoch), out_level_off[n_levels+1] (event offsets of
 * the levels).  The released events get dense indices first_dense .. +n-1
 * (*first_dense, optional). */
int lx_batcher_pop(lx_batcher *b, uint64_t *out_id, uint32_t *out_creator, uint32_t *out_seq, uint64_t *out_parent_off,
                   uint32_t *out_parent_idx, uint32_t *out_level_off, uint64_t *first_dense);

/* After a failed lx_add_batch of the last pop (the index rolled it back with
 * the batch's all-or-nothing rule): forget those events, so they can be pushed
 * again; dense indices are reused. */
int lx_batcher_unpop(lx_batcher *b);

/* Dense index of a released event (LX_ERR_ARG if not released). */
int lx_batcher_dense(const lx_batcher *b, uint64_t id, uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif
