/*
 * lachesis_abft.h -- C ABI of the batched abft caller on top of the HIP index.
 *
 * Drop-in for the consensus loop that drives the index in the reference:
 * abft.IndexedLachesis (abft/indexed_lachesis.go:17-107) = abft.Lachesis
 * (abft/lachesis.go) over abft.Orderer (abft/orderer.go, event_processing.go,
 * frame_decide.go, bootstrap.go) and election.Election (abft/election/).
 * Results -- frames, roots, decided frames, Atropos, cheaters, the order in
 * which confirmed events are applied, epoch sealing -- are those of calling the
 * reference's Process(e) once per event in the given order.  What changes is
 * how the ForklessCause questions are asked: frames of a whole batch are
 * computed level by level in frames, every question of a frame in one GPU
 * tile launch (events x roots of the frame), and election votes of a whole
 * round in one launch.
 *
 * Conventions are those of lachesis_hip.h: dense event indices (Add order of
 * the current epoch; they restart at 0 when an epoch is sealed or reset),
 * validator idx order, caller-owned buffers, 0 = ok / < 0 = error.  The abft
 * handle drives the index handle it was created on (Add, Flush,
 * DropNotFlushed, Reset): do not add events to that index directly.
 * One host thread per handle; callbacks must not call back into the handle.
 */
#ifndef LACHESIS_ABFT_H
#define LACHESIS_ABFT_H

#include "lachesis_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LX_ERR_FRAME -7        /* ErrWrongFrame: claimed frame mismatched (abft/event_processing.go:11-13) */
#define LX_ERR_BYZANTINE -8    /* election sanity errors (abft/election/election_math.go:68-90, sort_roots.go:23) */
#define LX_FRAME_BUILD 0xFFFFFFFFu   /* claimed_frame entry: compute as Build does (cap selfParentFrame+100) */

typedef struct lx_abft lx_abft;

/* lachesis.ConsensusCallbacks + BlockCallbacks (lachesis/consensus.go:21-44).
 * begin_block: decided frame, its Atropos, and the cheaters seen by the Atropos
 *   (validator idxs in idx order; abft/lachesis.go:57-73).
 * apply_event: every event newly confirmed by the block, in the reference's
 *   DFS order from the Atropos (abft/lachesis.go:40-55, abft/traversal.go:13-37).
 * end_block: return 0 to continue the epoch, or 1 to seal it; then
 *   *n_validators / *weights (idx order, valid until the next call into the
 *   library) give the next epoch's validators (frame_decide.go:11-35).
 * Any pointer may be NULL. */
typedef struct lx_abft_callbacks {
    void *user;
    void (*begin_block)(void *user, uint32_t frame, uint32_t atropos, const uint32_t *cheaters, uint32_t n_cheaters);
    void (*apply_event)(void *user, uint32_t ev);
    int (*end_block)(void *user, uint32_t *n_validators, const uint32_t **weights);
} lx_abft_callbacks;

/* NewIndexedLachesis (abft/indexed_lachesis.go:42-51) over an index handle
 * (unsharded). */
int lx_abft_create(lx_index *index, lx_abft **out);
void lx_abft_destroy(lx_abft *a);
const char *lx_abft_last_error(const lx_abft *a);
/* Path selection (results never change):
 *   "spec_depth" self-children evaluated speculatively per frame step (0..16,
 *                default 4)
 *   "fc16"       1 (default): fork-free epochs whose seqs fit 16 bits take the
 *                packed root-FC kernel (two columns per dword); 0: the 32-bit
 *                kernel always
 *   "claimed_batch" 1 (default): a batch whose every event claims its frame
 *                enqueues all its frame steps and waits once; 0: step by step
 *                as in Build
 *   "elect_ahead" rounds per election when the elections of every frame are
 *                enqueued together and read back with one wait (2..8, default
 *                2; 0: round by round, one wait per round)
 *   "block_log"  without a begin_block callback: 1 = the handle logs each
 *                decided block (frame, Atropos, cheaters) and runs the
 *                confirmation as a BeginBlock would, never sealing (no
 *                EndBlock); 2 = also the confirmed events in ApplyEvent order;
 *                read with lx_abft_block_log after the batch.  0 (default):
 *                nil BeginBlock semantics */
int lx_abft_set_option(lx_abft *a, const char *name, int64_t value);

/* ApplyGenesis + Bootstrap (abft/apply_genesis.go:17-44, bootstrap.go:30-52):
 * epoch and validators (weights in idx order); resets the index. */
int lx_abft_bootstrap(lx_abft *a, uint32_t epoch, uint32_t n_validators, const uint32_t *weights,
                      const lx_abft_callbacks *cb);

/* Orderer.Reset (bootstrap.go:54-65): switch to a new empty epoch. */
int lx_abft_reset(lx_abft *a, uint32_t epoch, uint32_t n_validators, const uint32_t *weights);

/* IndexedLachesis.Process (indexed_lachesis.go:65-82) for n events in
 * processing order (parents first; parent_off/parent_idx as lx_add_batch,
 * dense indices of this epoch, self-parent first).  claimed_frame[i] is the
 * event's Frame() field (LX_FRAME_BUILD: trust the computation, i.e. Build
 * then Process).  out_frame (optional) receives every consumed event's frame.
 * Callbacks fire for every frame decided inside the batch, in order.
 * *consumed = events processed: n, or less when
 *   - an event's claimed frame is wrong: returns LX_ERR_FRAME and *consumed is
 *     its position (the events before it are processed, as the reference
 *     processes them before returning ErrWrongFrame for it);
 *   - a block sealed the epoch: returns 0, *consumed counts the events up to
 *     the one whose processing decided the sealing frame; the rest belong to
 *     no epoch and must be re-submitted by the caller (as the reference test
 *     drivers do, abft/event_processing_test.go:145-150).
 * Every claim of the batch is checked before its elections run, so events
 * past a sealing frame carry this epoch's frame or LX_FRAME_BUILD. */
int lx_abft_process_batch(lx_abft *a, uint32_t n, const uint32_t *creator_idx, const uint32_t *seq,
                          const uint64_t *parent_off, const uint32_t *parent_idx, const uint32_t *claimed_frame,
                          uint32_t *out_frame, uint32_t *consumed);

/* The blocks the last lx_abft_process_batch decided (option block_log):
 * block k = frame[k], atropos[k], cheaters[cheat_off[k] .. cheat_off[k+1]),
 * confirmed[conf_off[k] .. conf_off[k+1]) (block_log 2; empty ranges with 1).
 * Pointers stay valid until the next call into the handle; any may be NULL. */
int lx_abft_block_log(const lx_abft *a, uint32_t *n_blocks, const uint32_t **frame, const uint32_t **atropos,
                      const uint32_t **cheat_off, const uint32_t **cheaters, const uint32_t **conf_off,
                      const uint32_t **confirmed);

/* IndexedLachesis.Build (indexed_lachesis.go:53-63): frame of a self-emitted
 * event (added, evaluated, then dropped again). */
int lx_abft_build(lx_abft *a, uint32_t creator_idx, uint32_t seq, uint32_t n_parents, const uint32_t *parents,
                  uint32_t *out_frame);

uint32_t lx_abft_epoch(const lx_abft *a);
uint32_t lx_abft_last_decided_frame(const lx_abft *a);
/* GetFrameRoots (abft/store_roots.go:52-93): root events of a frame. */
int lx_abft_frame_roots(lx_abft *a, uint32_t frame, uint32_t *out_ev, uint32_t cap, uint32_t *n);
int lx_abft_event_frame(const lx_abft *a, uint32_t ev, uint32_t *frame);
/* GetEventConfirmedOn (abft/store_event_confirmed.go:20-30): 0 = not confirmed. */
int lx_abft_event_confirmed_on(const lx_abft *a, uint32_t ev, uint32_t *frame);

/* Wall time of the last lx_abft_process_batch by phase (ms) and its GPU work. */
typedef struct lx_abft_stats {
    float ms_index;      /* Add of the batch (lx_add_batch) */
    float ms_frames;     /* frames + roots (root ForklessCause tiles) */
    float ms_election;   /* votes, decisions */
    float ms_blocks;     /* cheaters, confirmation DFS, callbacks */
    uint32_t frame_steps, fc_launches, vote_launches, blocks;
    uint64_t fc_pairs;   /* (event, root) pairs evaluated */
    uint64_t fc_pair_cols;   /* pairs x validator columns compared by k_root_fc */
    float ms_root_fc_gpu;    /* k_root_fc time on the stream (HIP events around each launch) */
    uint64_t fc_lane_ops;    /* VALU lane-ops the root-FC inner loops issue (ISA count per pair and
                                column: 2.5 in k_root_fc; 1.5 in k_root_fc16, 2 in its 32-column
                                chunks holding a weight >= 2^16) over the padded columns */
    uint32_t elections_ahead;   /* elections decided by run_elections_ahead (all their rounds
                                   enqueued at once) rather than round by round */
} lx_abft_stats;
int lx_abft_last_stats(const lx_abft *a, lx_abft_stats *out);

#ifdef __cplusplus
}
#endif
#endif
