/*
 * lachesis_hip.h -- C ABI of the MI355X-native vector-clock / ForklessCause index.
 *
 * Drop-in replacement for the reference's vecfc.Index (embedding
 * vecengine.Engine) behind the abft.DagIndexer / dagidx interfaces of
 * github.com/Fantom-foundation/lachesis-base.  Each entry point names the
 * reference interface it replaces (file:line in the reference tree).
 *
 * Conventions
 *  - Events are identified by dense indices 0..N-1 in Add order (the Go shim
 *    keeps the hash.Event <-> index map).  Parents are
 *    given as dense indices, self-parent first (inter/dag/event.go:87-92).
 *  - Validators are identified by their idx (inter/pos/validators.go:90-113);
 *    the caller passes weights already sorted in idx order.
 *  - All pointers are caller-owned; the library never retains them.
 *    Functions ending in _dev take device pointers (hipMalloc'd on the
 *    handle's device) and enqueue on the handle's stream unless a stream is
 *    given; everything else takes host pointers and is synchronous.
 *  - Return codes: 0 = ok, < 0 = error (lx_last_error() gives the message).
 *  - One host thread per handle (the reference index is not thread-safe:
 *    abft/indexed_lachesis.go:68).
 *  - Byte layouts returned by the getters are the reference's
 *    (vecfc/vector.go:14-102): LowestAfter = LE u32 per branch;
 *    HighestBefore = LE (Seq u32, MinSeq u32) per branch; fork marker
 *    {0, MaxInt32}.
 */
#ifndef LACHESIS_HIP_H
#define LACHESIS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LX_OK 0
#define LX_ERR_ARG -1          /* bad argument / unknown event (crit in the reference) */
#define LX_ERR_ORDER -2        /* parent not found / out of order (vecengine/index.go:159-161) */
#define LX_ERR_EVENT -3        /* event violates eventcheck invariants (seq/self-parent) */
#define LX_ERR_STATE -4        /* inconsistent state (vecengine/index.go:107-126) */
#define LX_ERR_HIP -5          /* HIP runtime / device error */
#define LX_ERR_NOMEM -6        /* device memory exhausted */
#define LX_ERR_WIRE -7         /* a LowestAfter block does not fit the 1-byte wire (pack it wider) */

#define LX_NO_EVENT 0xFFFFFFFFu

typedef struct lx_index lx_index;

typedef struct lx_config {
    int device;                  /* HIP device ordinal */
    uint64_t event_capacity;     /* events per epoch to pre-allocate (0 = grow on demand) */
    uint32_t branch_reserve;     /* extra branch columns reserved for forks (0 = default) */
    uint32_t shard_rank;         /* column shard (multi-GPU): this rank ...          */
    uint32_t shard_count;        /* ... of shard_count (0 or 1 = unsharded)          */
} lx_config;

/* NewIndex (vecfc/index.go:69-78).  The cache sizes of IndexConfig
 * (vecfc/index.go:16-61) only affect speed in the reference and have no
 * counterpart here. */
int lx_create(const lx_config *cfg, lx_index **out);
void lx_destroy(lx_index *h);
const char *lx_last_error(const lx_index *h);

/* Path selection for tests and tuning; no reference counterpart.  Every
 * option picks between implementations that give identical results (the
 * parity tests run each of them), so no setting changes an answer:
 *   "small_max"  largest host-pointer batch on the latency path (lx_small; 0 = never)
 *   "fc_fk"      0: ForklessCause on fork DAGs by the fix-up loop instead of the cheater-mask kernel
 *   "fc_early"   0: batched ForklessCause always reads whole rows (default 1: on fork-free
 *                epochs where the 256 heaviest validators' stake alone can reach the quorum,
 *                a query reads more of its rows only while their count leaves it open;
 *                lx_fc_early_counters)
 *   "cpw"        walker columns per workgroup: 0 (auto), 1, 2, 4, 8 or 12 (8, 12: packed
 *                fork-free epochs, else 4; 12: whole handles, a sharded one walks 8)
 *   "pack16"     0: two slot units per event even when every seq fits 16 bits
 *   "crec"       1: the 8- / 12-column walks stream 32-B compact event records instead of
 *                the 64-B ones (fork-free epochs, 16-bit branches and seqs)
 *   "fc_early_lanes" 32 (default) or 16 lanes per query in the early-exit ForklessCause
 *   "dbl"        0: the column walker also for fork-free batches of <= 16 branches
 *                (default: HighestBefore by frontier doubling in one workgroup, lx_dbl.hip)
 *   "la_memset"  1: zero the whole LowestAfter plane at lx_reset instead of the tail pass (before lx_reset)
 *   "shard_wire" LowestAfter exchange width: 0 (auto), 2 or 4 bytes
 *   "timing"     1: HIP-event timing of latency-path launches (lx_last_stats)
 *   "fc_cache"   working set of lx_forkless_cause in events (0: no cache; default 2 V, 512..8192).
 *                The result matrix is W^2 bytes of PINNED host memory per handle (64 MiB at
 *                8192, 256 MiB at the 16384 maximum), allocated on the first lx_forkless_cause;
 *                if it cannot be pinned the handle answers through lx_forkless_cause_batch
 *   "seg_count", "seg_rank"  G in 1..64 and r < G, before lx_reset: a row-segment rank
 *                (lx_rowseg_*, below; G = 1: one rank holding the whole epoch, every
 *                exchange and route run with nothing to move); 0 = off
 *   "seg_sub"    row-segment rank: its own segment walked as this many side-by-side
 *                sub-segments (0: auto, as "seg_auto" would split the rank's share; the
 *                same value on every rank of a job)
 *   "segments"   G in 2..64: a batch of >= 64 G events is walked as G Add-order segments
 *                and fixed up (the single-GPU form of the row-segment multi-GPU
 *                protocol; results identical); 0/1 off
 *   "seg_auto"   0: never split a batch on its own (default 1: a batch whose walk
 *                leaves CUs idle -- few columns -- is walked as G segments side by
 *                side in one launch, G = CUs / walk workgroups, >= 32k events each)
 *   "get_server" 0: every single-row getter launches its kernel (default 1: the resident
 *                row server answers them while the stream is idle, lx_get_server_stats)
 *   "realloc_records" 1: diagnostics -- move the batch record buffers to a fresh
 *                allocation now (the walk slow-mode probe)
 * The library reads no environment variables except two diagnostics: the
 * walker-counters build (make WPROF=1) reads LX_PROF, and LX_ABFT_TIMING=1
 * prints the abft passes' host timing marks to stderr. */
int lx_set_option(lx_index *h, const char *name, int64_t value);

/* Reset (vecfc/index.go:98-105, vecengine/index.go:56-68): new epoch with
 * `n_validators` validators whose weights are given in idx order. */
int lx_reset(lx_index *h, uint32_t n_validators, const uint32_t *weights_by_idx);

/* Add (vecengine/index.go:71-75) for a batch of events in Add order.
 * parent_off has n+1 entries into parent_idx (dense indices, self-parent
 * first).  Bit-exact to calling the reference Add once per event in the
 * given order.  All-or-nothing: on error nothing is added and *err_index (if
 * non-NULL) receives the batch position of the first offending event.
 * out_branch (optional, n entries) receives each event's global branch ID
 * (GetEventBranchID, vecengine/store_branches_info.go:83-88). */
int lx_add_batch(lx_index *h, uint32_t n, const uint32_t *creator_idx, const uint32_t *seq,
                 const uint64_t *parent_off, const uint32_t *parent_idx,
                 uint32_t *out_branch, uint32_t *err_index);
/* Same, with the batch already resident in device memory (parent_off is
 * uint32 here: batch-local offsets). */
int lx_add_batch_dev(lx_index *h, uint32_t n, const uint32_t *creator_idx_dev, const uint32_t *seq_dev,
                     const uint32_t *parent_off_dev, const uint32_t *parent_idx_dev, uint32_t *err_index);

/* Flush (vecengine/index.go:78-85) and DropNotFlushed (:88-96): rolls the
 * index back to the last flush, including LowestAfter entries of old events
 * and fork branches created since. */
int lx_flush(lx_index *h);
int lx_drop_not_flushed(lx_index *h);

/* Write-back of Flush to the reference's kvdb tables (vecengine/index.go:78-85,
 * vecfc/store_vectors.go:53-65, vecengine/store_branches_info.go:57-81): the
 * Puts the reference's flushable would commit at this Flush, in its byte
 * formats:
 *   table "S" (HighestBefore, vecfc/index.go:39): the events added since the
 *             last flush, first_event .. first_event + n_events - 1;
 *   table "s" (LowestAfter, vecfc/index.go:40): those events plus every older
 *             event whose LowestAfter gained an entry since (the DFS Visits of
 *             vecengine/index.go:212-225), ascending dense index;
 *   table "b" (branch ID, vecengine/index.go:40): the new events, 4 B big-endian
 *             (inter/idx/internal.go:13-15);
 *   table "B" key "c" (vecengine/index.go:41): RLP(BranchesInfo).
 * lx_writeback_prepare finds the rows on the device and returns the sizes;
 * lx_writeback_fetch encodes them on the device and copies them out (any
 * pointer may be NULL to skip that part; offsets have n+1 entries, in bytes).
 * lx_flush then commits.  Adding, dropping, flushing or resetting in between
 * invalidates the prepared set (LX_ERR_STATE).  Unsharded handles only.
 * Restart: lx_load_rows / lx_load_finish below. */
typedef struct lx_writeback {
    uint64_t first_event, n_events;   /* rows of tables S and b */
    uint64_t n_la_rows;               /* rows of table s */
    uint64_t hb_bytes, la_bytes;      /* value bytes of tables S and s */
    uint32_t bi_bytes;                /* RLP(BranchesInfo) */
} lx_writeback;
int lx_writeback_prepare(lx_index *h, lx_writeback *out);
int lx_writeback_fetch(lx_index *h, uint64_t *hb_off, uint8_t *hb_bytes, uint32_t *la_ev, uint64_t *la_off,
                       uint8_t *la_bytes, uint8_t *branch_be, uint8_t *bi_rlp);

/* Restart from the persisted tables without replay (abft/restart_test.go:156-188
 * rebuilds a fresh index over a copy of the epoch DB; vecengine/index.go:56-68
 * Reset + the lazy reads of vecfc/store_vectors.go:26-51 and
 * vecengine/store_branches_info.go:57-88).  After lx_reset(V, weights):
 *   lx_load_rows(...)  any number of times: the epoch's events in a parents-first
 *                      order the caller chooses (dense indices continue: 0, 1, ...);
 *                      per event its creator idx, seq, parents (self-parent
 *                      first), table "b" value (4-B big-endian branch ID) and
 *                      the bytes of tables "S" (HighestBefore) and "s"
 *                      (LowestAfter); hb_off / la_off have n+1 absolute byte
 *                      offsets into hb_bytes / la_bytes;
 *   lx_load_finish(table "B" key "c": RLP(BranchesInfo)).
 * The loaded epoch counts as flushed; Add, ForklessCause and the getters then
 * continue exactly as in the reference after its restart.  Tables that do not
 * form one consistent epoch (branch chains, creators, byte lengths, MinSeq,
 * LastSeq, BranchesInfo, fork markers the vectors do not imply) return
 * LX_ERR_STATE ("inconsistent DB", the reference's crit) and leave the handle
 * needing lx_reset.  Unsharded handles only. */
int lx_load_rows(lx_index *h, uint32_t n, const uint32_t *creator_idx, const uint32_t *seq,
                 const uint64_t *parent_off, const uint32_t *parent_idx, const uint8_t *branch_be,
                 const uint64_t *hb_off, const uint8_t *hb_bytes, const uint64_t *la_off, const uint8_t *la_bytes);
int lx_load_finish(lx_index *h, const uint8_t *bi_rlp, uint32_t bi_len);

uint64_t lx_num_events(const lx_index *h);
uint32_t lx_num_branches(const lx_index *h);           /* len(BranchIDCreatorIdxs) */
int lx_at_least_one_fork(const lx_index *h);           /* branches_info.go:47-49 */

/* ForklessCause (vecfc/forkless_cause.go:28-82) for n (a, b) pairs. */
int lx_forkless_cause_batch(lx_index *h, uint64_t n, const uint32_t *a, const uint32_t *b, uint8_t *out);
/* Device-resident variant; stream may be NULL (handle stream).  Unknown
 * events yield 0xFF in out and LX_ERR_ARG from the next lx_sync(). */
int lx_forkless_cause_batch_dev(lx_index *h, uint64_t n, const uint32_t *a_dev, const uint32_t *b_dev,
                                uint8_t *out_dev, void *stream);
/* ForklessCause for one pair, as the unchanged caller asks it
 * (vecfc/forkless_cause.go:28-38; per pair from forklessCausedByQuorumOn,
 * abft/event_processing.go:149-161, and the election's observedRoots,
 * abft/election/election.go:101-123).  Answered from the index's result
 * cache -- the counterpart of the reference's ForklessCause LRU -- over a
 * working set of the events recently asking and asked about; a miss fills a
 * whole row (the asking event against the working set) or, for an older row,
 * the whole working set in one launch, so a caller looping over a frame's
 * roots waits for the GPU once per asking event.  Exact: FC(a, b) never
 * changes once a is indexed; DropNotFlushed evicts the dropped events.  Option
 * "fc_cache" sets the working set (0: every call evaluates its pair).
 * Unknown events: LX_ERR_ARG. */
int lx_forkless_cause(lx_index *h, uint32_t a, uint32_t b, uint8_t *out);
typedef struct lx_fc_stats {
    uint64_t calls;         /* lx_forkless_cause calls */
    uint64_t hits;          /* answered from the cache without a launch */
    uint64_t row_fills;     /* misses answered by one row launch (asking event x working set) */
    uint64_t tile_fills;    /* misses answered by one working set x working set launch */
    uint64_t pairs;         /* pairs evaluated on the GPU by the fills */
    uint32_t slots;         /* working set capacity (events) */
    uint32_t slots_used;
    uint64_t miss_ns;       /* host time inside misses (launch + wait), ns */
    uint64_t wait_ns;       /* ... of which waiting for the answer to land */
    uint64_t launch_ns;     /* ... of which inside the fill's enqueue calls (flush, copies, launch) */
    uint64_t quiesce_ns;    /* ... of which waiting for an earlier fill to finish writing */
    uint64_t fused;         /* row fills that were also the asking event's Add (k_add1_row) */
} lx_fc_stats;
int lx_fc_cache_stats(const lx_index *h, lx_fc_stats *out);

/* Batched ForklessCause's early exit (option fc_early) since the last call.
 * The path runs on launches of >= 2^14 queries over fork-free epochs whose
 * rows exceed 512 columns and whose 512 heaviest validators can reach the
 * quorum alone (smaller launches keep one round of whole rows: shorter
 * latency); it reads both rows in
 * rounds of columns [0, 128), [128, 256), [256, 512) and the rest, each only
 * when the count so far leaves the quorum open.  lx_fc_early_rounds: out[0]
 * queries decided on the path (device count), out[1..3] of them the ones that
 * read round 2, round 3, the rest.  lx_fc_early_counters: (out[0], out[1],
 * out[3]).  Synchronize the handle's stream; reset the counts.  Diagnostics
 * (bench). */
int lx_fc_early_rounds(lx_index *h, uint64_t out[4]);
int lx_fc_early_counters(lx_index *h, uint64_t *queries, uint64_t *second_round, uint64_t *whole_rows);

/* Column-sharded partial: stake sum over this shard's creators, plus
 * 0x80000000 when this shard owns branch(b) and A observes it as forked.
 * Sum the partials of all shards (uint32) and apply lx_fc_combine. */
int lx_forkless_cause_partial_dev(lx_index *h, uint64_t n, const uint32_t *a_dev, const uint32_t *b_dev,
                                  uint32_t *partial_dev, void *stream);
int lx_fc_combine_dev(lx_index *h, uint64_t n, const uint32_t *sum_dev, uint8_t *out_dev, void *stream);

/* Column-shard early exit: ForklessCause compares a stake sum
 * in pos.Validators idx order with the quorum (vecfc/forkless_cause.go:63-82),
 * and shard 0 holds the heaviest creators.  From its own partial it decides a
 * query when the partial reaches the quorum (true) or cannot reach it with
 * every other shard's stake added (false); only the undecided queries need the
 * other shards' partials and the all-reduce.  Applies on fork-free epochs
 * where shard 0 can decide something (lx_fc_shard_early: 1, *rest = the stake
 * of shards 1..G-1).  Every rank, collectively:
 *   shard 0:   lx_forkless_cause_partial_dev over all n queries, then
 *              lx_fc_shard_decide_dev -> mask (2 ceil(n/64) words: decided bits,
 *              then answer bits); the mask is broadcast from shard 0;
 *   all:       lx_fc_shard_undecided_dev -> the m undecided queries in query
 *              order (idx, a, b; shard 0 also its partials) -- completed on
 *              return, *m on the host;
 *   shards>0:  lx_forkless_cause_partial_dev over the m undecided pairs;
 *   all:       sum the m partials over the shards, lx_fc_shard_answer_dev.
 * The answers equal lx_fc_combine_dev over the full sums
 * (lx_forkless_cause_sharded_dev and lachesis_hip.shard run it). */
int lx_fc_shard_early(const lx_index *h, uint32_t *rest);
int lx_fc_shard_decide_dev(lx_index *h, uint64_t n, const uint32_t *partial_dev, uint64_t *mask_dev, void *stream);
int lx_fc_shard_undecided_dev(lx_index *h, uint64_t n, const uint64_t *mask_dev, const uint32_t *a_dev,
                              const uint32_t *b_dev, const uint32_t *partial_dev, uint32_t *idx_dev, uint32_t *a_out_dev,
                              uint32_t *b_out_dev, uint32_t *partial_out_dev, uint64_t *m);
int lx_fc_shard_answer_dev(lx_index *h, uint64_t n, const uint64_t *mask_dev, uint64_t m, const uint32_t *idx_dev,
                           const uint32_t *sum_dev, uint8_t *out_dev, void *stream);
uint32_t lx_quorum(const lx_index *h);                 /* pos/validators.go:187-189 */

/* Getters.  *len receives the byte length; out may be NULL to query it.
 * GetHighestBefore / GetLowestAfter (vecfc/store_vectors.go:26-51),
 * GetMergedHighestBefore (vecengine/index.go:235-250 with GatherFrom,
 * vecfc/vector_ops.go:81-96).  Rows are encoded on the device. */
int lx_get_highest_before(lx_index *h, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len);
int lx_get_lowest_after(lx_index *h, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len);
int lx_get_merged_highest_before(lx_index *h, uint32_t ev, uint8_t *out, uint32_t cap, uint32_t *len);
/* The single-row getters above are answered by a resident one-wave kernel
 * (the row server) when the handle's stream is idle: no launch per call, the
 * row and a completion tag land in pinned memory.  It leaves after 250 us
 * without a request (and after 0.5 s in all), so a device-wide synchronization
 * right after a getter may wait that long.  While resident it holds one of
 * the process's hardware queues (GPU_MAX_HW_QUEUES, 4 by default): with more
 * streams than queues, work on a stream sharing its queue would wait for its
 * idle exit.  Option get_server: 1 (default) uses it only while the handle is
 * the process's only one (lx_live_handles), 2 always, 0 never (every call
 * launches).  Either way the kernel refuses an event outside the handle's
 * rows by itself (LX_ERR_ARG), whatever the request word names.  out[0] rows
 * it served, out[1] its launches, out[2] single-row calls that launched
 * instead (stream busy, option off, other handles alive). */
int lx_get_server_stats(const lx_index *h, uint64_t out[3]);
int lx_live_handles(void);   /* index handles created and not destroyed in this process */
/* The same for n events in one call (applyAtropos, abft/lachesis.go:57, and the
 * emitter's candidate loops call GetMergedHighestBefore per event): row i is
 * written at out + off[i], off has n+1 entries (byte offsets, always filled);
 * out may be NULL to query the sizes; a buffer smaller than off[n] gives
 * LX_ERR_ARG (off still filled).  Unknown events: LX_ERR_ARG (the reference's
 * getters return nil for them). */
int lx_get_highest_before_batch(lx_index *h, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out,
                                uint64_t cap);
int lx_get_lowest_after_batch(lx_index *h, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out,
                              uint64_t cap);
int lx_get_merged_highest_before_batch(lx_index *h, uint32_t n, const uint32_t *ev, uint64_t *off, uint8_t *out,
                                       uint64_t cap);
int lx_get_event_branch_id(lx_index *h, uint32_t ev, uint32_t *out);
/* The same rows with device ids in and device rows out (mode 0 HighestBefore,
 * 1 LowestAfter, 2 merged HighestBefore): row i at out_dev + i * slot_bytes,
 * its byte length in len_dev[i] (slot_bytes >= lx_row_bytes_max); an event
 * the handle does not hold -- not indexed, or another row-segment rank's --
 * gets length 0xFFFFFFFF and no row.  Completed on return.  The row-segment
 * getters route ids to their owners and call this there
 * (lachesis_hip/rowseg.py, lx_rowseg_get_rows).  On a column shard each slot
 * holds this shard's branches (merged HighestBefore: its creators) and zeros
 * elsewhere, and len_dev the length this shard's entries imply: the word-wise
 * sum of all shards' slots is the whole row and the maximum of their lengths
 * its length (lx_shard_get_rows; LowestAfter after the exchange). */
int lx_get_rows_dev(lx_index *h, uint32_t mode, uint32_t n, const uint32_t *ev_dev, uint8_t *out_dev,
                    uint64_t slot_bytes, uint32_t *len_dev);
int lx_row_bytes_max(const lx_index *h, uint64_t *bytes);   /* 8 x max(branches, validators) */

/* BranchesInfo (vecengine/branches_info.go:9-14): per branch last seq and
 * creator idx (arrays of cap entries; *n_branches receives B). */
int lx_get_branches_info(lx_index *h, uint32_t *last_seq, uint32_t *creator_idx, uint32_t cap,
                         uint32_t *n_branches);

/* Column shards (multi-GPU).  A handle created with
 * shard_count > 1 indexes only the branches whose creator lies in its creator
 * range and stores only those columns (memory per GPU ~ 1/shard_count):
 * HighestBefore for those columns and complete LowestAfter rows for events on
 * those branches.  Before ForklessCause, shards exchange LowestAfter blocks (an
 * all-to-all): shard s sends lx_la_pack_dev(s -> d) = (rows on s's branches) x
 * (columns of d) and d stores it with lx_la_unpack_dev(from s); lx_la_own_dev
 * moves a shard's own block (its rows x its columns).  After an Add or a
 * DropNotFlushed the exchange is repeated before the next ForklessCause.
 * lx_shard_block gives the entry count of a block and lx_shard_wire the bytes
 * per entry in the pack/unpack buffers: 2 while every seq of the epoch is
 * < 2^16 (entries are seqs or 0), else 4; all shards of an epoch agree on it,
 * so a block occupies entries x wire bytes on both sides.  The three
 * transfer calls run on the handle's stream and return when done (their
 * `stream` argument is reserved; NULL).  The vector getters, write-back, abft
 * and the QuorumIndexer need an unsharded handle. */
int lx_shard_of(const lx_index *h, uint32_t *shard_rank, uint32_t *shard_count);
int lx_shard_range(const lx_index *h, uint32_t shard, uint32_t *creator_lo, uint32_t *creator_hi);
int lx_shard_block(lx_index *h, uint32_t src_shard, uint32_t dst_shard, uint64_t *elems);
int lx_shard_wire(lx_index *h, uint32_t *bytes_per_entry);
int lx_la_pack_dev(lx_index *h, uint32_t dst_shard, uint32_t *out_dev, void *stream);
int lx_la_unpack_dev(lx_index *h, uint32_t src_shard, const uint32_t *in_dev, void *stream);
int lx_la_own_dev(lx_index *h, void *stream);
/* Per-block byte wire: lx_shard_block_wire gives the narrowest width of this
 * shard's outgoing block to dst -- 1 byte per entry when every entry is 0 or
 * within 127 of its row event's own seq (stored as LA - seq + 128; typical: a
 * branch observes an event a few seqs later), else lx_shard_wire's width
 * (option shard_wire pins the latter).  The sender tells the receiver the width
 * (e.g. a G-int all-to-all) and both sides move the block with the _wire_
 * variants; the block occupies entries x width bytes.  Packing at width 1
 * checks as it goes: LX_ERR_WIRE means some entry did not fit, and the caller
 * packs the block again at lx_shard_wire's width (so a sender may skip
 * lx_shard_block_wire and try the byte wire first). */
int lx_shard_block_wire(lx_index *h, uint32_t dst_shard, uint32_t *bytes_per_entry);
int lx_la_pack_wire_dev(lx_index *h, uint32_t dst_shard, void *out_dev, uint32_t bytes_per_entry);
int lx_la_unpack_wire_dev(lx_index *h, uint32_t src_shard, const void *in_dev, uint32_t bytes_per_entry);
/* Incremental exchange (the reference's per-event Add -> Flush cadence,
 * abft/indexed_lachesis.go:69-82, vecengine/index.go:78-96): blocks hold only
 * the rows whose LowestAfter entries can have changed since the last committed
 * exchange.  lx_shard_dirty writes, for each of this shard's branches, the
 * first such seq into dmin[branch] (LX_NONE for the other shards' branches and
 * for unchanged ones; nb >= lx_num_branches); the ranks combine their arrays
 * by an element-wise min (e.g. an all_reduce MIN) and pass the result to
 * lx_shard_dirty_set, after which lx_shard_block / pack / unpack / own move the
 * dirty rows only (every rank lists the same rows, branch by branch in seq
 * order); lx_shard_dirty_commit after the unpacks ends it.  After lx_reset, a
 * DropNotFlushed or a branch-capacity growth the next exchange is whole. */
int lx_shard_dirty(lx_index *h, uint32_t nb, uint32_t *dmin);
int lx_shard_dirty_set(lx_index *h, uint32_t nb, const uint32_t *dmin);
int lx_shard_dirty_commit(lx_index *h);

/* Column shards over RCCL without a Python host (the Go caller): one
 * communicator per shard handle, built from a unique id that rank 0 creates
 * and the caller distributes (as ncclGetUniqueId / ncclCommInitRank).
 * lx_shard_exchange = the LowestAfter all-to-all (pack each block on the
 * 1-byte wire when it fits, else at lx_shard_wire's width -- a destination
 * that needed the wide width starts there next time, the byte wire is retried
 * every 8th exchange; the widths, then the blocks at 4-byte aligned offsets
 * (lx_shard_exchange_layout), as grouped ncclSend/ncclRecv on the handle's
 * stream; unpack; own block);
 * lx_forkless_cause_sharded_dev = partial stake sums, an ncclAllReduce (sum,
 * uint32: exact, the true total fits 32 bits) and the quorum test, all
 * stream-ordered on the handle's stream (calls of >= 2^14 queries on epochs
 * where lx_fc_shard_early applies: shard 0's partials first, an ncclBroadcast
 * of its decisions, the other shards' partials and the all-reduce over the
 * undecided queries only).  Every rank must make the same calls
 * in the same order (collectives).  RCCL is loaded on first use (dlopen of
 * librccl.so.1, reusing a copy the process already holds); nranks must equal
 * the handle's shard_count and rank its shard_rank; one GPU per rank (RCCL
 * refuses two ranks on one device).  lx_shard_comm_last_error(NULL) tells why
 * the calling thread's last lx_shard_comm_create failed. */
typedef struct lx_shard_comm lx_shard_comm;
int lx_shard_comm_unique_id(uint8_t id[128]);
int lx_shard_comm_create(lx_index *h, const uint8_t id[128], uint32_t nranks, uint32_t rank, lx_shard_comm **out);
void lx_shard_comm_destroy(lx_shard_comm *c);
const char *lx_shard_comm_last_error(const lx_shard_comm *c);
int lx_shard_exchange(lx_shard_comm *c);
/* Layout of one rank's exchange buffer (send or receive side): block q of
 * entries[q] x width[q] bytes starts at off[q], a multiple of 4 bytes (the own
 * block, q == self, is empty); off[G] = buffer bytes.  Host-only: every
 * implementation of the exchange (lx_shard_exchange, the Python ShardedIndex,
 * a Go shim doing its own collectives) lays blocks out this way. */
int lx_shard_exchange_layout(uint32_t G, uint32_t self, const uint64_t *entries, const uint32_t *width,
                             uint64_t *off);
int lx_forkless_cause_sharded_dev(lx_shard_comm *c, uint64_t n, const uint32_t *a_dev, const uint32_t *b_dev,
                                  uint8_t *out_dev);
/* Queries the last lx_forkless_cause_sharded_dev sent to every shard: the
 * undecided ones of the early exit (lx_fc_shard_early; calls of >= 2^14
 * queries), else all of them. */
int lx_shard_fc_undecided(const lx_shard_comm *c, uint64_t *undecided);
/* The vector getters on column shards (GetHighestBefore / GetLowestAfter /
 * GetMergedHighestBefore, vecfc/store_vectors.go:26-51, vecengine/index.go:235-250):
 * every rank calls collectively with the same events; each encodes its own
 * branches (lx_get_rows_dev), an ncclAllReduce sums the slots and another takes
 * the maximum length, so every rank gets the whole rows.  LowestAfter rows
 * need the LowestAfter exchange since the last Add (lx_shard_exchange).  slot:
 * >= lx_row_bytes_max, a multiple of 16. */
int lx_shard_get_rows(lx_shard_comm *c, uint32_t mode, uint64_t n, const uint32_t *ev_dev, uint8_t *out_dev,
                      uint64_t slot_bytes, uint32_t *len_dev);

/* Timing of the last lx_add_batch* call, measured with HIP events on the
 * handle's stream (milliseconds): branch assignment + record packing,
 * index walker (HB max-join + LA range fill), fork marks. */
typedef struct lx_stats {
    float ms_assign;
    float ms_index;
    float ms_marks;
    uint32_t index_launches;
} lx_stats;
int lx_last_stats(const lx_index *h, lx_stats *out);

/* The shader clock of the last walk (k_index / k_index_segs): compute wave 0
 * of every workgroup stamps s_memtime (shader cycles) and s_memrealtime
 * (100 MHz) around its walk.  out[0] median, out[1] min, out[2] max clock over
 * the workgroups (MHz), out[3] the median workgroup's walk (ms); per XCD x
 * (HW_REG_XCC_ID): out[4 + x] the median clock of its workgroups, out[12 + x]
 * its slowest workgroup's walk (ms).  A walk's cycle count is set by the DAG;
 * its time is cycles / clock.  Synchronizes the handle's
 * stream; zeros before the first walk.  Diagnostics. */
int lx_last_walk_clock(lx_index *h, float out[20]);

/* Timings of the last segmented batch (option "segments"): per segment its
 * first event, walk time and number of "partial" events (rows that needed
 * the gathered fix-up); then the gathered fix-up and the LowestAfter pass. */
typedef struct lx_seg_stats {
    uint32_t segments;
    uint32_t first_event[65];
    uint32_t partial[64];
    float walk_ms[64];
    float partial_ms, la_ms;
    uint32_t one_launch;    /* 1: the segments were walked side by side by one k_index_segs launch */
} lx_seg_stats;
int lx_last_segment_stats(const lx_index *h, lx_seg_stats *out);

/* Row segments: the segmented walk spread over G ranks, one GPU each
 * (DESIGN.md section 6b).  A handle with options seg_count = G, seg_rank = r
 * takes the epoch as ONE lx_add_batch(_dev) of n >= 64 G events; it assigns
 * every event's branch (replicated metadata) but walks and owns only the rows
 * of segment r, [lo, hi) (lx_rowseg_range).  The caller then runs two
 * exchanges with its collectives (lachesis_hip/rowseg.py):
 *   rows, in rounds until no rank has requests left:
 *     lx_rowseg_requests  -> the ids of the rows this rank still needs into a
 *                            device buffer (lx_rowseg_request_cap ids),
 *                            grouped by owner rank, counts[G];
 *     (ids to their owners) lx_rowseg_serve -> rows (lx_rowseg_row_words
 *                            words each) and ready flags (0: not final yet);
 *     (rows back)          lx_rowseg_receive -> *remaining;
 *   LowestAfter: lx_rowseg_la -> counts[G] of (row, column, seq) triples for
 *     each owner rank, lx_rowseg_la_fetch copies them (grouped by owner) to a
 *     device buffer; each owner lx_rowseg_la_apply's what it gets;
 * then lx_rowseg_finish.  After it, ForklessCause answers queries between own
 * events, and any pair of the epoch through the cross-rank protocol below;
 * the vector getters answer own events (another rank's: LX_ERR_STATE; the
 * caller routes them, lachesis_hip/rowseg.py get_rows over lx_get_rows_dev);
 * write-back, DropNotFlushed and the abft / emitter views need a whole index
 * (LX_ERR_STATE).  The planes hold the own rows only (plus receive areas for
 * rows of other ranks): about 1/G of the epoch per GPU.  Every call has
 * completed on the device when it returns. */
int lx_rowseg_range(const lx_index *h, uint32_t *lo, uint32_t *hi);
int lx_rowseg_of(const lx_index *h, uint32_t *rank, uint32_t *count);   /* options seg_rank / seg_count (0 / 1 when off) */

/* Row segments over RCCL for callers without a Python host (the Go shim): the
 * exchanges above (the protocol of lachesis_hip/rowseg.py) issued by the library
 * on the handle's stream -- ids, rows and LowestAfter triples by grouped
 * ncclSend / ncclRecv, the termination test by ncclAllReduce -- then
 * lx_rowseg_finish.  Create the communicator with the handle's seg_rank /
 * seg_count (an lx_shard_comm; every rank calls collectively, after its
 * lx_add_batch_dev of the epoch).  stats (optional): rounds of the row
 * exchange, rows received, LowestAfter triples sent, received. */
int lx_rowseg_comm_create(lx_index *h, const uint8_t id[128], uint32_t nranks, uint32_t rank, lx_shard_comm **out);
int lx_rowseg_exchange(lx_shard_comm *c, uint64_t stats[4]);
int lx_rowseg_bounds(const lx_index *h, uint32_t *lo /* G + 1 */);
int lx_rowseg_row_words(const lx_index *h, uint32_t *words);
int lx_rowseg_request_cap(const lx_index *h, uint32_t *cap);
int lx_rowseg_requests(lx_index *h, uint32_t *ids_dev, uint32_t cap, uint32_t *counts);
int lx_rowseg_serve(lx_index *h, uint32_t n, const uint32_t *ids_dev, uint32_t *rows_dev, uint32_t *ready_dev);
int lx_rowseg_receive(lx_index *h, uint32_t n, const uint32_t *ids_dev, const uint32_t *rows_dev,
                      const uint32_t *ready_dev, uint32_t *remaining);
int lx_rowseg_la(lx_index *h, uint64_t *counts);
int lx_rowseg_la_fetch(lx_index *h, uint32_t *triples_dev);
int lx_rowseg_la_apply(lx_index *h, uint64_t n, const uint32_t *triples_dev);
int lx_rowseg_finish(lx_index *h);

/* ForklessCause(a, b) of ANY pair of a row-segmented epoch
 * (vecfc/forkless_cause.go:40-82): answered on owner(a)
 * -- HB(a) is there -- with LA(b) shipped from owner(b) when b lies in another
 * segment.  Every rank calls collectively, after lx_rowseg_finish, with its own
 * batch of n queries (device arrays):
 *   lx_rowseg_fc_route   -> the queries grouped by owner(a) into ra / rb, the
 *                           permutation perm (n each), counts[G];
 *   (ra, rb to their owners: m received pairs)
 *   lx_rowseg_fc_need    -> the distinct b of the received pairs outside this
 *                           rank's rows, grouped by owner, into ids (capacity >=
 *                           min(m, events)), counts[G];
 *   (ids to their owners) lx_rowseg_la_serve -> their LA rows (lx_rowseg_row_words
 *                           words each); (rows back) lx_rowseg_la_store;
 *   lx_forkless_cause_batch_dev over the m received pairs (b may now be any
 *                           stored row; lx_sync before moving the answers);
 *   (answers back)        lx_rowseg_fc_unroute -> out[i] for the caller's query i.
 * lx_rowseg_forkless_cause runs the same over RCCL (lx_rowseg_comm_create). */
int lx_rowseg_fc_route(lx_index *h, uint64_t n, const uint32_t *qa_dev, const uint32_t *qb_dev, uint32_t *ra_dev,
                       uint32_t *rb_dev, uint32_t *perm_dev, uint64_t *counts);
int lx_rowseg_fc_need(lx_index *h, uint64_t m, const uint32_t *ra_dev, const uint32_t *rb_dev, uint32_t *ids_dev,
                      uint64_t cap, uint64_t *counts);
int lx_rowseg_la_serve(lx_index *h, uint64_t n, const uint32_t *ids_dev, uint32_t *rows_dev);
int lx_rowseg_la_store(lx_index *h, uint64_t n, const uint32_t *ids_dev, const uint32_t *rows_dev);
int lx_rowseg_fc_unroute(lx_index *h, uint64_t n, const uint32_t *perm_dev, const uint8_t *ans_dev, uint8_t *out_dev);
/* stats (optional): queries routed away, pairs answered here, LA rows received, sent */
int lx_rowseg_forkless_cause(lx_shard_comm *c, uint64_t n, const uint32_t *qa_dev, const uint32_t *qb_dev,
                             uint8_t *out_dev, uint64_t stats[4]);
/* The vector getters of events on any rank (GetHighestBefore / GetLowestAfter
 * / GetMergedHighestBefore, vecfc/store_vectors.go:26-51,
 * vecengine/index.go:235-250), collectively: each rank's n device ids are
 * routed to their owners (lx_rowseg_fc_route with b = a), answered there by
 * lx_get_rows_dev, and the rows come back in the caller's order
 * (lx_rowseg_rows_unroute: row i of `rows` to row perm[i] of out, slot_bytes
 * each, lengths with them).  lx_rowseg_get_rows does all of it over RCCL;
 * lachesis_hip/rowseg.py get_rows over torch.distributed.  Mode and
 * lengths as lx_get_rows_dev (0xFFFFFFFF: no such event). */
int lx_rowseg_rows_unroute(lx_index *h, uint64_t n, const uint32_t *perm_dev, const uint8_t *rows_dev,
                           uint64_t slot_bytes, const uint32_t *len_dev, uint8_t *out_dev, uint32_t *out_len_dev);
int lx_rowseg_get_rows(lx_shard_comm *c, uint32_t mode, uint64_t n, const uint32_t *ev_dev, uint8_t *out_dev,
                       uint64_t slot_bytes, uint32_t *len_dev);

/* Device views for benchmarks/tests (valid until the next add/reset).  On a
 * row-segment rank the planes hold its own rows only: row e is at
 * hb + e * stride for e in lx_rowseg_range, nothing else is addressable. */
int lx_device_planes(lx_index *h, void **hb, void **la, uint32_t *stride, void **stream);
/* Device memory the handle holds, in bytes: out[0] the HighestBefore and
 * LowestAfter planes (a column shard: plus its produced LowestAfter rows;
 * a row-segment rank: its own rows), out[1] a row-segment rank's receive
 * areas (rows of other ranks), out[2] per-event metadata and per-event
 * scratch, out[3] everything else it allocated (branch tables, batch and
 * query scratch). */
int lx_device_bytes(const lx_index *h, uint64_t out[4]);
int lx_sync(lx_index *h);

#ifdef __cplusplus
}
#endif
#endif
