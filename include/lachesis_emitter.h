/*
 * lachesis_emitter.h -- C ABI of the emitter's QuorumIndexer on the HIP index.
 *
 * Drop-in for emitter/ancestor.QuorumIndexer (emitter/ancestor/
 * quorum_indexer.go:20-158), the second consumer of GetMergedHighestBefore:
 *   - the V x V matrix of merged-HighestBefore seqs (row = observed validator,
 *     column = creator of the last event processed for it), globalMatrix;
 *   - the self-parent seqs (the emitter's own last event), selfParentSeqs;
 *   - per row the weighted median at the quorum (recacheState, :100-121 with
 *     utils/wmedian/median.go:11-21), recomputed lazily as in the reference;
 *   - GetMetricOf (:123-136) for a batch of candidate parents.
 * The matrix lives on the device next to the index planes its columns are
 * read from.  seqOf (:70-75) maps a fork-detected entry to MaxUint32/2 - 1.
 *
 * The reference's DiffMetricFn is a Go closure; the library evaluates the
 * capped-difference metric of emitter/ancestor/quorum_indexer_test.go:117-131
 * (cap 2 there) with the cap as a parameter.  Other metrics read the matrix,
 * medians and self-parent seqs back and evaluate on the host.
 *
 * Conventions of lachesis_hip.h (dense event indices of the index's epoch,
 * validator idx order, caller-owned buffers, 0 = ok / < 0 = error).  One
 * QuorumIndexer per emitting validator, as in the reference; after lx_reset
 * of the index (new epoch) call lx_qi_reset (NewQuorumIndexer per epoch).
 * Up to 8192 validators (one LDS-resident sort per matrix row).
 */
#ifndef LACHESIS_EMITTER_H
#define LACHESIS_EMITTER_H

#include "lachesis_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lx_qi lx_qi;

/* NewQuorumIndexer (:33-43) for the index's current validators. */
int lx_qi_create(lx_index *index, lx_qi **out);
void lx_qi_destroy(lx_qi *q);
const char *lx_qi_last_error(const lx_qi *q);
/* New epoch: validators from the index, matrix and seqs zeroed. */
int lx_qi_reset(lx_qi *q);

/* ProcessEvent (:86-98) for n events in order; self_event[i] != 0 marks the
 * emitter's own events (NULL = none). */
int lx_qi_process_events(lx_qi *q, uint32_t n, const uint32_t *ev, const uint8_t *self_event);

/* GetGlobalMedianSeqs (:145-150, V entries), GetGlobalMatrix (:152-154,
 * V x V row-major: out[validator * V + creator]), GetSelfParentSeqs (:156-158). */
int lx_qi_median_seqs(lx_qi *q, uint32_t *out);
int lx_qi_matrix(lx_qi *q, uint32_t *out);
int lx_qi_self_parent_seqs(lx_qi *q, uint32_t *out);

/* GetMetricOf (:123-136) for n candidate events with the capped metric. */
int lx_qi_metric_of(lx_qi *q, uint32_t n, const uint32_t *ev, uint32_t cap, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
