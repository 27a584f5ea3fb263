// lx_internal.h -- shared declarations of the HIP index (kernels + host engine).
//
// Device data layout (all uint32, row-major, rows = dense event index):
//   hb[e*stride + b]  : RAW HighestBefore seq of branch b observed by e
//                       (pure max-join, no fork absorption), bit 31 = fork
//                       marker of creator(b) as seen by e (branches < B_after(e))
//   la[e*stride + b]  : LowestAfter seq (0 = none)
//   brow[b*s_cap + s - first(b)] : dense index of the event of branch b at seq s
// Per event: ev_creator, ev_seq, ev_branch, ev_bbefore (B before Add), ev_sp
// (self-parent or NONE), first_child (first self-child that continued the
// branch, claimed by atomicMin).  Per branch: branch_first, branch_creator,
// branch_len.  See DESIGN.md for the derivation and the reference mapping.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LX_NONE 0xFFFFFFFFu
#define LX_MARK 0x80000000u
#define LX_SEQ_MASK 0x7FFFFFFFu
#define LX_MAXP 12   // parents stored inline in an event record

// Event record consumed by the index kernel: 4 x uint4 = 64 B
//   w0 branch, w1 seq, w2 number of parents, w3 previous event of the same
//   branch (global dense index, NONE if the event opens its branch),
//   w4..w15 the first 12 parents sorted oldest first (global index, NONE pad);
//   parents beyond 12 are read from the batch parent array
#define LX_REC_Q 4
struct EventRec {
    uint4 q[LX_REC_Q];
};

struct IndexArgs {
    uint32_t *hb;
    uint32_t *la;
    uint64_t stride;
    uint32_t batch_start;
    uint32_t n;
    const EventRec *rec;
    const uint32_t *par_in;      // batch parent array (overflow parents)
    const uint32_t *poff_in;     // batch parent offsets
    const uint32_t *col_list;
    uint32_t ncols;
    uint32_t n_slices;           // ceil(ncols / CPW)
    uint32_t slices_per_xcd;
    const uint32_t *branch_first;
    const uint32_t *brow;
    uint32_t s_cap;
    uint32_t mask;               // older rows may carry fork marks
    uint32_t diag_nofill;        // diagnostic timing build: skip the LA fill (LX_DIAG_NOFILL=1)
    uint32_t cpw_hint;           // columns per workgroup (0 = auto; LX_CPW)
    uint32_t ncw_hint;           // compute waves per workgroup (0 = auto; LX_NCW)
    uint32_t width_hint;         // expected antichain width of the batch
    uint32_t rr_hint;            // record ring depth (LX_RR; 0 = auto)
    uint32_t diag;               // timing-only diagnostics (LX_DIAG): 2 no deps, 3 no global stores
    unsigned long long *prof;    // optional per-wave counters (LX_PROF=1), kProfSlots per wave
    uint32_t small;              // small-LDS walker variant (LX_SMALL=1)
};
constexpr int kProfSlots = 16;   // see k_index: passes, spin misses, chunk folds, completes, ...

struct BatchArgs {
    uint32_t n;
    uint32_t batch_start;
    uint32_t V;
    uint32_t B0;                 // branches before the batch
    const uint32_t *creator;     // batch-local inputs
    const uint32_t *seq;
    const uint32_t *poff;        // n+1, batch-local offsets into par
    const uint32_t *par;         // global dense indices
    uint32_t *ev_creator;        // persistent per-event arrays (global index)
    uint32_t *ev_seq;
    uint32_t *ev_branch;
    uint32_t *ev_bbefore;
    uint32_t *ev_sp;
    uint32_t *first_child;
    uint32_t *first_root;        // per creator
    uint32_t *branch_first;
    uint32_t *branch_creator;
    uint32_t *branch_len;
    uint32_t *brow;
    uint32_t s_cap;
    uint32_t *isfork;            // batch scratch (rank after scan)
    uint32_t *rank;
    uint32_t *tmp_br;
    uint32_t *jmp;
    EventRec *rec;
    uint32_t *status;            // [0] err index, [1] err code, [2] max seq, [3..] jump flags
};

struct FcArgs {
    const uint32_t *hb;
    const uint32_t *la;
    uint64_t stride;
    uint32_t n_events;
    uint64_t n;
    const uint32_t *qa;
    const uint32_t *qb;
    uint8_t *out;                // bool result (or NULL)
    uint32_t *partial;           // partial sum (or NULL)
    const uint32_t *wpad;        // weight per column (0 outside [vlo, vhi) originals)
    uint32_t vlo4, vhi4;         // column range in uint4 units
    uint32_t quorum;
    const uint32_t *ev_branch;
    // cheaters of this shard: CSR over all their branches (first = original)
    uint32_t n_cheat;
    const uint32_t *cheat_off;
    const uint32_t *cheat_br;
    const uint32_t *cheat_creator;
    uint32_t own_lo, own_hi;     // creator range owned by this shard
    const uint32_t *branch_creator;
    uint32_t *status;            // status[1] |= bad-event flag
};

struct MarkArgs {
    uint32_t *hb;
    uint64_t stride;
    uint32_t batch_start;
    uint32_t n;
    uint32_t V;
    const uint32_t *ev_branch;
    const uint32_t *ev_bbefore;
    const uint32_t *branch_first;
    uint32_t n_cheat;
    const uint32_t *cheat_off;
    const uint32_t *cheat_br;
};

struct UnfillArgs {
    uint32_t *hb;
    uint32_t *la;
    uint64_t stride;
    uint32_t lo, hi;             // dropped events [lo, hi)
    uint32_t B;                  // branches (columns) to scan
    const uint32_t *ev_seq;
    const uint32_t *ev_branch;
    const uint32_t *ev_bbefore;
    const uint32_t *ev_sp;
    const uint32_t *ev_creator;
    uint32_t *first_child;
    uint32_t *first_root;
    uint32_t *branch_len;
    const uint32_t *branch_first;
    const uint32_t *brow;
    uint32_t s_cap;
    uint32_t B_keep;             // branches that survive the rollback
};

// kernel launchers (lx_kernels.hip); all enqueue on `s`
namespace lx {
hipError_t launch_batch_prepare(const BatchArgs &a, void *scan_tmp, size_t scan_tmp_bytes, hipStream_t s);
hipError_t launch_batch_finish(const BatchArgs &a, hipStream_t s);
hipError_t scan_tmp_bytes(uint32_t n, size_t *bytes);
hipError_t launch_undo_claims(const BatchArgs &a, hipStream_t s);
hipError_t launch_index(const IndexArgs &a, hipStream_t s);
hipError_t launch_marks(const MarkArgs &a, hipStream_t s);
hipError_t launch_fc(const FcArgs &a, uint32_t cols, bool forks, hipStream_t s);
hipError_t launch_fc_combine(const uint32_t *sum, uint8_t *out, uint64_t n, uint32_t quorum, hipStream_t s);
hipError_t launch_unfill(const UnfillArgs &a, hipStream_t s);
hipError_t launch_fill_u32(uint32_t *p, uint64_t n, uint32_t v, hipStream_t s);
hipError_t launch_shard_rows(const uint32_t *ev_branch, const uint32_t *branch_creator, uint32_t n, uint32_t lo,
                             uint32_t hi, uint32_t *flag, uint32_t *pos, void *scan_tmp, size_t scan_bytes,
                             uint32_t *rows, hipStream_t s);
hipError_t launch_la_block(uint32_t *la, uint64_t stride, const uint32_t *rows, uint32_t nrows, const uint32_t *cols,
                           uint32_t ncols, uint32_t *buf, int unpack, hipStream_t s);
hipError_t launch_copy_rows(uint32_t *dst, uint64_t dst_stride, const uint32_t *src, uint64_t src_stride,
                            uint64_t rows, uint64_t cols, hipStream_t s);
}  // namespace lx
