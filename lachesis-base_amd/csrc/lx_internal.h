// lx_internal.h -- shared declarations of the HIP index (kernels + host engine).
//
// Device data layout (all uint32, row-major, rows = dense event index):
//   hb[e*stride + b]  : RAW HighestBefore seq of branch b observed by e
//                       (pure max-join, no fork absorption), bit 31 = fork
//                       marker of creator(b) as seen by e (branches < B_after(e))
//   la[e*stride + b]  : LowestAfter seq (0 = none)
//   brow[b*s_cap + s - first(b)] : dense index of the event of branch b at seq s
// Column-sharded handles store only their own columns:
//   cmap[b]           : plane column of global branch b (NONE: another shard's)
//   hb, la            : rows of pstride = local column capacity (own originals
//                       first, then own fork branches in creation order);
//                       `la` holds the exchanged LowestAfter of own columns
//   lap[(cmap[c]*s_cap + s - first(c)) * stride + j] : LowestAfter entry j of
//                       the event (c, s) of an own branch c, as the walker
//                       produces it (all B columns), the source of the exchange
// Unsharded handles: cmap = NULL (identity), pstride = stride, lap = NULL.
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

// Compact event record (2 x uint4 = 32 B, same round-blocked SoA), written
// beside EventRec for fork-free epochs whose seqs and branches fit 16 bits;
// the 8- / 12-column walkers stream it instead (half the record bytes, twice
// the events in the same LDS ring, 31 DMA rounds in flight instead of 15):
//   c0 branch | seq << 16
//   c1 number of parents | (event - previous event of the branch) << 8
//      (0 when the event opens its branch), or kCrecWide: a parent or the
//      previous event too far back (or > 255 parents) -- that event's walker
//      reads its EventRec from global memory instead
//   c2..c7 the first 12 parents as distances back (event - parent, 16 bits
//      each, low half first), sorted oldest first, 0 past the last parent
#define LX_CREC_Q 2
struct CRec {
    uint4 q[LX_CREC_Q];
};
constexpr uint32_t kCrecWide = 0xFFFFFFFFu;

constexpr uint32_t kSegLaunchMax = 32;   // segments of one k_index_segs launch
struct IndexArgs {
    uint32_t *hb;
    uint32_t *la;
    uint64_t stride;
    uint32_t batch_start;
    uint32_t n;
    const EventRec *rec;
    const CRec *crec;            // compact records (CPW 8 / 12 walks), or NULL
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
    uint32_t cpw_hint;           // columns per workgroup (0 = auto; lx_set_option "cpw", tests)
    unsigned long long *prof;    // per-wave counters (make WPROF=1 builds only), kProfSlots per wave
    unsigned long long *clk;     // walk clock (lx_last_walk_clock): [0] grid size, then per workgroup
                                 // < kClkBlocks {shader cycles, 100 MHz ticks, XCD} of compute wave 0
    const uint32_t *cmap;        // sharded: global branch -> plane column (NULL = identity)
    uint32_t *lap;               // sharded: LowestAfter rows of own branches (fill target)
    uint64_t lap_stride;         // = global branch capacity
    uint32_t pack16;             // every seq of the epoch <= 0xFFFF: 16-B packed slots (4-column block walker)
    // segment walk (lx_segment.hip): parents before batch_start contribute only
    // their own (branch, seq) entry, and no LowestAfter is filled
    uint32_t seg;
    const uint32_t *ev_branch;
    const uint32_t *ev_seq;
    const uint32_t *seg_j;       // J_k: last seq of each branch before the segment
    uint32_t *seg_flag;          // per segment event: set when its row misses some J_k (a "partial" event)
    uint32_t *seg_list;          // partial events (global index), appended
    uint32_t *seg_count;
    // > 0: one launch walks seg_g segments side by side (k_index_segs): segment
    // k = [seg_lo[k], seg_lo[k + 1]), its J table at seg_j + k * seg_B, its
    // partial-event flags / list at the batch offset, its count at seg_count + k
    uint32_t seg_g;
    uint32_t seg_B;
    uint32_t seg_lo[kSegLaunchMax + 1];
    // 12-column side-by-side walks: workgroup -> (walk << 8 | slice), 0xFFFF
    // idle, for workgroups < seg_map_n (launch_index fills it when option
    // seg_xmap is on: every 128-B HB line written by workgroups of one XCD);
    // seg_map_n = 0: seg_chunk's mapping
    uint32_t seg_xmap;           // option seg_xmap (lx_set_option)
    uint32_t seg_map_n;
    uint16_t seg_map[256];
};
// k_dbl (lx_dbl.hip): HighestBefore by frontier doubling in one workgroup's
// LDS, for fork-free batches with few branches
struct DblArgs {
    uint32_t *hb;
    uint32_t *la;
    uint64_t stride;
    uint32_t bs;                 // first event of the batch
    uint32_t n;
    uint32_t B;                  // branches (= validators: no forks)
    const EventRec *rec;
    const uint32_t *par;         // batch parent array (global indices), batch-local offsets
    const uint32_t *poff;
    const uint32_t *ev_branch;
    const uint32_t *ev_seq;
    const uint32_t *branch_first;
    const uint32_t *brow;
    uint32_t s_cap;
};
constexpr uint32_t kDblLds = 160 * 1024 - 256;
constexpr uint32_t kDblMaxB = 16;
__host__ __device__ inline uint64_t dbl_lds_bytes(uint64_t n, uint64_t B) {
    return 4 * (n * B + 3 * B + 3) + 2 * ((n + 1) & ~1ull);
}
constexpr int kProfSlots = 16;   // see k_index: passes, spin misses, chunk folds, completes, ...
constexpr int kProfWaves = 16;   // waves per workgroup in the counter layout
constexpr int kProfBlocks = 4096;
constexpr int kClkBlocks = 1024;   // walk clock records (IndexArgs::clk)

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
    CRec *crec;                  // non-NULL: also write the compact records
    uint32_t *status;            // [0] err index, [1] err code, [2] max seq, [3..] jump flags
    uint32_t nofork;             // no fork branch in the epoch nor in the batch: branch = creator
};

struct FcArgs {
    const uint32_t *hb;
    const uint32_t *la;
    uint64_t stride;
    uint32_t n_events;
    uint32_t ev_lo;              // row-segment rank: queries must lie in [ev_lo, n_events)
    // row-segment rank: b may also be another segment's event whose final LA
    // row was received (b_stamp[b] odd; lx_rowseg_fc.hip); NULL elsewhere
    const uint32_t *b_stamp;
    uint32_t n_all;              // events of the epoch (b_stamp's length)
    // row-segment rank: the LA rows received for this batch live in la_recv
    // (row b_slot[b]); b_stamp[b] == b_arrived marks them (lx_rowseg_fc.hip)
    const uint32_t *la_recv;
    const uint32_t *b_slot;
    uint32_t b_arrived;
    uint64_t n;
    const uint32_t *qa;
    const uint32_t *qb;
    uint8_t *out;                // bool result (or NULL)
    const uint8_t *out_tag;      // optional: out[q] = out_tag[q] << 1 | result (FC cache generations)
    uint32_t qa_bcast;           // 1: every query's a is qa_imm (a row of the FC cache; never read from
                                 // memory the host may rewrite while the fill runs)
    uint32_t qa_imm;
    uint32_t *partial;           // partial sum (or NULL)
    const uint32_t *wpad;        // weight per column (0 outside [vlo, vhi) originals)
    uint32_t vlo4, vhi4;         // column range in uint4 units
    uint32_t quorum;
    // early exit (k_fc_early: fork-free rows of > 512 columns; 0 = off): the
    // weight of the columns past the first 4L, 8L and 16L of the range (L = early_lanes).  The
    // first columns are the heaviest validators (pos.Validators idx order), so
    // their count alone often decides the quorum either way
    uint32_t early_rest;
    uint32_t early_rest2;
    uint32_t early_rest3;
    uint32_t early;
    uint32_t early_lanes;        // lanes per query of k_fc_early: 32 (rounds 128 / 256 / 512 columns) or 16 (64 / 128 / 256)
    unsigned long long *early_full;   // [0] += queries past round 1, [1] += past round 2, [2] += queries
                                      // on the early path, [3] += past round 3 (whole rows)
    const uint32_t *ev_branch;
    const uint32_t *ev_creator;  // creator per event (= creator of its branch)
    // cheaters of this shard: CSR over all their branches (first = original)
    uint32_t n_cheat;
    const uint32_t *cheat_off;
    const uint32_t *cheat_br;
    const uint32_t *cheat_creator;
    const uint32_t *cheat_brl;   // cheat_br / cheat_creator as plane columns
    const uint32_t *cheat_crl;
    const uint32_t *cmap;        // sharded: global branch -> plane column (NULL = identity)
    uint32_t own_lo, own_hi;     // creator range owned by this shard
    const uint32_t *branch_creator;
    uint32_t *status;            // status[1] |= bad-event flag
    // fork DAGs with <= kFcFkMaxCheaters cheaters (fk_hi4 != 0): per plane
    // column [0, 4 fk_hi4) the weight of a non-cheater's original branch
    // (fk_w) and the cheater index of a cheater's branches (fk_c, LX_NONE
    // otherwise); the cheaters' weights (fk_wch)
    const uint32_t *fk_w;
    const uint32_t *fk_c;
    const uint32_t *fk_wch;
    uint32_t fk_hi4;
};
constexpr uint32_t kFcFkMaxCheaters = 64;   // one 64-bit mask per query
constexpr uint64_t kFcEarlyMinQueries = 1u << 14;   // launches this large take the early exit (k_fc_early)

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
    const uint32_t *cmap;        // sharded: global branch -> plane column (NULL = identity)
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
    const uint32_t *cmap;        // sharded: global branch -> plane column (NULL = identity)
    uint32_t *lap;               // sharded: produced LowestAfter rows (see top)
    uint64_t lap_stride;
};

// LowestAfter exchange between column shards: mode 0 pack (lap -> buf),
// 1 unpack (buf -> la), 2 own block (lap -> la); buf is [rows][cols]
struct XferArgs {
    const uint32_t *lap;
    uint64_t lap_stride;
    uint32_t s_cap;
    uint32_t *la;
    uint64_t pstride;
    const uint32_t *cmap;
    const uint32_t *ev_branch;
    const uint32_t *ev_seq;
    const uint32_t *branch_first;
    const uint32_t *rows;        // events (global dense indices)
    uint32_t nrows;
    const uint32_t *cols;        // global branch ids
    uint32_t ncols;
    uint32_t *buf;
    int mode;
    uint32_t *flag;              // set to 1 when a byte-wire pack meets an entry that does not fit
    uint32_t wire;               // bytes per buf entry: 4, 2 (every seq < 2^16) or 1 (LA - seq(row) + 128,
                                 // 0 = no entry; only when the whole block fits, see k_la_xfer mode 3)
};

// LowestAfter tail zeroing (unsharded planes; replaces the epoch-start memset of
// the whole LA plane): after a batch, entry (x, j) of a row x = (c, s) that
// branch j has not observed (s > RAW(last event of j)[c]) must read 0; the fill
// wrote every observed entry.  zw[j][c] = seq up to which (c, .) x j is done.
struct TailArgs {
    uint32_t *la;
    const uint32_t *hb;
    uint64_t stride;             // plane stride (branches)
    const uint32_t *brow;        // [branch][seq - first] -> event row
    uint32_t s_cap;
    const uint32_t *branch_first;
    const uint32_t *branch_len;
    uint32_t B;
    uint32_t *zw;                // [j][c], tcap x tcap
    uint32_t *lo;                // [j][c] scratch: first seq to zero
    uint32_t *cmin;              // [c] min over j of lo
    uint32_t tcap;
};

// ---- small-batch (latency) path (lx_small.hip): the host assigns branches in
// Add order (vecengine/index.go:105-141, exactly the reference's lastSeq rule)
// and stages the batch; one launch writes the metadata and computes HB + LA.
// Per event: 3 x uint4
//   q0 = {branch, seq, prev (previous event of the branch, global; NONE when the
//         event opens its branch), number of parents}
//   q1 = {offset of its entries in the run's "old" list (host only), first seq of
//         the branch, self-parent (global or NONE), branches before Add}
//   q2 = {creator, flags (kSmallCont: continues its branch), final first_child
//         of this event (its continuing self-child in the batch, or NONE),
//         h0 slot: index of prev's HB row among the "old" entries when prev is
//         older than the batch (else NONE)}
constexpr uint32_t kSmallCont = 1u;
constexpr uint32_t kSmallCW = 4;     // columns per workgroup (256 threads = 4 columns x 64 event lanes)
constexpr uint32_t kSmallMaxN = 2048;   // events per small batch (positions are 16-bit; LDS below)
constexpr uint32_t kPendLaunch = 2048;  // a pending run of small batches launches at this size
constexpr uint32_t kSmallDblLevels = 128;   // runs this deep (and <= kDblMaxB branches) go to k_small_dbl
constexpr uint32_t kSmallLds = 160 * 1024 - 256;   // dynamic LDS of one k_small workgroup
struct SmallEv {
    uint4 q0, q1, q2;
};
// dynamic LDS of k_small: val[n] + h0v[nh] (uint4), lmeta (uint2, n rounded to
// even), in-run parents (uint16, rounded to 8), level offsets (L + 1), own
// events (uint16)
__host__ __device__ inline uint64_t small_lds_bytes(uint64_t n, uint64_t nh, uint64_t L, uint64_t npl) {
    return 16 * (n + nh) + 8 * ((n + 1) & ~1ull) + 2 * ((npl + 7) & ~7ull) + 4 * (L + 1) + 2 * n;
}
// dynamic LDS of k_small_dbl: the run's rows and the older previous events'
// rows (B words each), per-branch tables, chain positions (uint16)
__host__ __device__ inline uint64_t small_dbl_lds_bytes(uint64_t n, uint64_t B, uint64_t nh) {
    return 4 * ((n + nh) * B + 4 * B + 3) + 2 * ((n + 1) & ~1ull);
}
struct SmallArgs {
    uint32_t *hb, *la;
    uint64_t stride;
    uint32_t bs, n;              // first global index, events
    uint32_t B0, B;              // branches before / after the batch
    // staged image (uint32 words; records first, 16-B aligned): SmallEv[n] in
    // Add order, then at word offsets: meta (level order, uint2 {batch position
    // | chunks of 4 in-run parents << 16, offset into the in-run list in chunks};
    // padded to 16 B), the in-run parents (batch positions, uint16, each event's
    // list padded to a chunk with its own position; padded to 16 B), the "old" entries (uint2
    // {target, global event}: target = batch position for a parent older than
    // the batch, 0x80000000 | h0 slot for an older prev), level offsets
    // (n_levels + 1), first seqs and creators of branches B0 .. B-1, (branch,
    // events on it) pairs of the branches the batch touched
    const uint32_t *img;         // device copy (NULL: the image is in the kernel arguments)
    uint32_t o_meta, o_pl, o_old, o_loff, o_nfirst, o_ncreator, o_blen;
    uint32_t n_pl, n_old, n_h0;
    uint32_t n_levels;
    uint32_t n_blen;
    uint32_t *ev_creator, *ev_seq, *ev_branch, *ev_bbefore, *ev_sp, *first_child, *first_root;
    uint32_t *branch_first, *branch_creator, *branch_len, *brow;
    uint32_t s_cap;
    uint32_t mask;               // rows may carry fork marks (B > V)
};
// One pending event added and its ForklessCause row of the FC cache filled in
// one launch (lx_small.hip k_add1_row; the unchanged caller's miss path: Add(e)
// then ForklessCause(e, root) for the roots of a frame).  Fork-free epochs only.
constexpr uint32_t kAdd1MaxPar = 32;
constexpr uint32_t kAdd1Delta = 8;      // slot changes carried in k_add1_row's arguments
constexpr uint32_t kAdd1Slots = 128;    // slots (threads) per k_add1_row workgroup
constexpr uint32_t kAdd1PsumStride = 1;    // uint64 words between two slots' partial-sum words (16 = one 128-B line each measured slower: 7.09 vs 6.36 us)
struct Add1RowArgs {
    uint32_t *hb, *la;
    uint64_t stride;
    uint32_t a;                  // global index of the event
    SmallEv e;                   // its record (q0 = {branch, seq, prev, #parents}, ...)
    uint32_t blen;               // branch_len of its branch afterwards
    uint32_t B;                  // branches (= validators: no forks)
    uint32_t w_br;               // weight of its branch
    uint32_t par[kAdd1MaxPar];   // parents, global indices
    uint32_t *ev_creator, *ev_seq, *ev_branch, *ev_bbefore, *ev_sp, *first_child, *first_root;
    uint32_t *branch_len, *brow;
    const uint32_t *branch_first;
    uint32_t s_cap;
    // the row: out[s] = tag[s] << 1 | ForklessCause(a, evk[s]) for s < n_slots
    // (evk / tag: the device mirror of the cache's slots)
    uint32_t *evk;
    uint32_t n_slots;
    uint8_t *tag;
    uint8_t *out;
    const uint32_t *wpad;
    uint32_t quorum;
    uint32_t *psum;              // [n_slots] x kAdd1PsumStride x uint64: {column groups, sum}, zero between launches
    // slots the host changed since the mirror was last written: applied by
    // every reader, stored into the mirror by the column-group-0 workgroups
    uint32_t nd;
    uint32_t d_slot[kAdd1Delta], d_ev[kAdd1Delta];
    uint8_t d_tag[kAdd1Delta];
};

// Batches whose image fits travel in the kernel arguments (no staging copy)
constexpr uint32_t kSmallInline = 768;   // words (3 KB; kernel arguments stay < 4 KB)
struct SmallInlineArgs {
    SmallArgs a;
    alignas(16) uint32_t img[kSmallInline];
};

// ---- write-back to the reference's byte formats (lx_persist.hip)
struct RowsArgs {
    const uint32_t *plane;       // hb or la
    uint64_t stride;
    const uint32_t *rows;        // dense event indices
    uint32_t n;
    uint32_t B;                  // branches in use
    const uint32_t *ev_bbefore;
    const uint32_t *ev_branch;
    const uint32_t *branch_first;
    uint32_t hb;                 // 1: HighestBefore (8 B per branch), 0: LowestAfter (4 B)
};

// restart from the persisted tables (k_load_rows, k_load_raw, k_load_check)
struct LoadArgs {
    uint32_t *hb, *la;
    uint64_t stride;
    uint32_t bs, n;              // first dense index of the chunk, events
    uint32_t B;                  // branches known so far (HB entries must lie below)
    const uint64_t *hb_off, *la_off;   // n + 1 byte offsets (absolute)
    uint64_t hb_base, la_base;   // offsets of the first byte of the chunk's buffers
    const uint8_t *hb_bytes, *la_bytes;
    const uint32_t *ev_branch, *ev_seq;
    const uint32_t *branch_first;
    uint32_t *brow;
    uint32_t s_cap;
    uint32_t *bad;               // |= 1: malformed entry
};
struct LoadRawArgs {
    uint32_t *hb;
    uint64_t stride;
    const uint32_t *cols;        // the cheaters' branch columns
    uint32_t ncc;
    const uint32_t *perm, *lvl_off;   // events by topological level
    uint32_t n_levels;
    const uint64_t *poff;        // whole epoch: parents of event e at par[poff[e] .. poff[e+1])
    const uint32_t *par;
    const uint32_t *ev_branch, *ev_seq;
    uint8_t *lm;                 // [e][k]: entry was loaded as a fork marker
    uint32_t *bad;               // |= 2: raw value differs, 4: markers differ
};

struct LoadVerifyArgs {
    const uint32_t *hb, *la;
    uint64_t stride;
    uint32_t n, B;
    const uint32_t *ev_branch, *ev_seq;
    const uint32_t *branch_first, *branch_len, *brow;
    uint32_t s_cap;
    uint32_t *bad;
};

// batched getters (k_get_rows): mode 0 HighestBefore, 1 LowestAfter, 2 merged HighestBefore
struct GetArgs {
    const uint32_t *plane;       // hb (modes 0, 2) or la (mode 1)
    uint64_t stride;
    const uint32_t *ev;          // events (device-visible; NULL: the one event ev0, n = 1)
    uint32_t ev0;
    uint32_t n;
    uint32_t B, V;
    uint32_t mode;
    uint32_t forks;              // B > V
    const uint32_t *ev_bbefore;
    const uint32_t *ev_branch;
    const uint32_t *branch_first;
    const int32_t *cheat_of;     // creator -> cheater index (-1: one branch)
    const uint32_t *cheat_off;   // CSR over all branches of each cheater (original first)
    const uint32_t *cheat_br;
    uint8_t *out;                // row i at out + i * slot
    uint64_t slot;
    uint32_t *len;               // byte length of row i
    // single-row call (n = 1): `tag` into pinned *done after the row and its
    // length, so the host spins on it instead of synchronizing the stream
    uint32_t *done;
    uint32_t tag;
    // rows the kernel may read: events outside [row_lo, row_hi) are answered
    // with length kGetBadLen and no row (the host turns it into LX_ERR_ARG) --
    // the device's own bound, whatever event a request word names
    uint32_t row_lo, row_hi;
    // column shard: branch -> plane column (LX_NONE: another shard's branch,
    // read as 0); NULL: whole rows
    const uint32_t *cmap;
};
constexpr uint32_t kGetBadLen = 0xFFFFFFFFu;

// the resident single-row server (k_get_server): `g` with plane / ev0 / mode /
// tag filled per request from the request word *req
constexpr uint32_t kGetSrvStop = 0x3FFFFFFFu;   // request tag: leave
struct GetSrvArgs {
    GetArgs g;
    const uint32_t *hb, *la;
    const uint64_t *req;         // pinned: {tag : 30, mode : 2, event : 32}
    uint32_t *exited;            // pinned: gen on leaving
    uint32_t gen;
    uint32_t seen0;              // the last tag answered before this launch
    uint64_t idle_ticks, budget_ticks;   // wall clock (hipDeviceAttributeWallClockRate)
};

// ---- emitter QuorumIndexer (lx_emitter.hip, lx_emitter.cpp)
struct QiArgs {
    const uint32_t *hb;
    uint64_t stride;
    uint32_t V;
    uint32_t forks;              // B > V: fork marks and cheaters' branches exist
    const int32_t *cheat_of;     // creator -> cheater index (-1: one branch)
    const uint32_t *cheat_off;   // CSR over all branches of each cheater
    const uint32_t *cheat_br;
    const uint32_t *weights;     // by validator idx
    uint32_t quorum;
    uint32_t *mt;                // matrix, transposed: mt[creator * V + validator]
    uint32_t *sp;                // self-parent seqs
    uint32_t *median;            // global median seqs
    const uint32_t *ev_creator;
    unsigned long long *lastk;   // [V + 1]: per creator (and [V]: self) the last batch position, gen << 32 | i
};

// a ProcessEvent batch: events inline (n <= kQiInline) or in device memory
constexpr uint32_t kQiInline = 16;
struct QiBatch {
    uint32_t n, gen;
    const uint32_t *ev;          // NULL: inline
    const uint32_t *self;        // per event 0/1 (device, with ev)
    uint32_t iev[kQiInline];
    uint32_t iself;              // inline self flags, bit i
};

// ---- batched abft caller (lx_abft_kernels.hip, lx_abft.cpp)
struct RootFcArgs {
    const uint32_t *hb;
    const uint32_t *la;
    uint64_t stride;
    const uint32_t *cand;        // candidate events (rows of bits)
    uint32_t n_cand;
    const uint32_t *roots;       // root events of one frame (NONE = dropped slot)
    uint32_t n_roots;
    uint32_t roots_fallback;     // any valid event, loaded in place of NONE / padding
    uint32_t ncols;              // original columns scanned (V rounded up to 32)
    const uint32_t *wpad;        // weight per column (0 outside the originals)
    uint32_t quorum;
    uint32_t n_k;                // cheaters' branch columns, grouped by cheater, original first
    const uint32_t *kcol;
    const uint32_t *kflag;       // bit0 first of its group, bit1 last
    const uint32_t *kw;          // weight of the group's creator (on its last column)
    const uint32_t *ev_branch;
    uint32_t *psum;              // out: psum[(z * n_cand + c) * words * 32 + r], partial stake of split z
    uint32_t words;
    uint32_t col_split;          // columns per split (multiple of 32)
    uint32_t n_split;            // column splits (grid z)
    uint32_t block0;             // merged launch: this step's first workgroup
};

struct QuorumArgs {
    const uint32_t *psum;        // partial stake sums of k_root_fc
    uint32_t n_split;
    uint32_t *bits;              // out: bits[c * words + r / 32]
    uint32_t words;
    uint32_t n_roots;
    uint32_t n_cand;
    const uint32_t *cand;        // candidate events (their own slot is skipped)
    const uint32_t *root_ev;     // root events of the frame
    const uint32_t *creator;     // creator idx per root (NONE = dropped)
    const uint32_t *dup;         // previous root of the same creator, or NONE
    const uint32_t *wcreator;    // weight by creator idx
    uint32_t quorum;
    uint8_t *q;                  // out
    uint32_t block0;             // merged launch: this step's first workgroup
};

constexpr uint32_t kVoteVoted = 0x80000000u, kVoteYes = 0x40000000u, kVoteDecided = 0x20000000u,
                   kVoteNoRoot = 0x1FFFFFFFu;
constexpr uint32_t kVoteErrMissing = 1, kVoteErrTwoRoots = 2, kVoteErrQuorum = 4;

// one host-to-device segment of an abft step's batched upload (k_scatter)
struct ScatterDesc {
    void *dst;
    uint64_t src_off;            // into the staging slot
    uint64_t bytes;              // a multiple of 4
};

struct VoteArgs {
    uint32_t V;
    const uint32_t *voter_ev;    // per voter slot (NONE = skip)
    const uint64_t *bm_off;      // voter's observed-roots bitmap (words into bm)
    const uint32_t *bm_len;      // bits valid
    const uint32_t *bm;
    const uint32_t *prev_creator;  // roots of the previous frame
    const uint32_t *prev_dup;
    const uint32_t *prev_votes;  // [root][V]
    uint32_t prev_has_dup;       // some validator has two roots in the previous frame
    uint32_t v_lo, v_hi;         // subject window
    const uint32_t *wcreator;
    uint32_t quorum;
    uint32_t *votes;             // out [voter][V]
    unsigned long long *dec;     // per subject: min (event << 32 | yes << 31 | observed root)
    uint32_t *err;
    uint32_t n_voters;           // voter slots (set by the launchers)
};

// Segmented walk of one batch (lx_segment.hip): the
// batch [bs, bs + n) split into G Add-order segments seg_lo[k] .. seg_lo[k+1],
// each walked with its boundary parents as own entries only (IndexArgs::seg),
// then fixed up to the reference's rows.
constexpr uint32_t kMaxSegments = 64;
constexpr uint64_t kAutoSegEvents = 32768;
constexpr float kPass12 = 2.1f;  // 12-column slices (C3: three walks 50.0 ms vs two 8-column walks 61.2 ms -> 1.7 x 3 / 2 x 50.0 / 61.2)
constexpr float kPass8 = 1.7f;   // pass cost of 8- vs 1-column slices (8 compute + 7 drain waves; C3 one walk: 121.7 ms at 8 columns, 91.4 at 4 = 1.28)
struct SegArgs {
    uint32_t *hb;
    uint32_t *la;
    uint64_t stride;
    uint32_t B;                  // branches after the batch
    uint32_t bs, n, G;
    uint32_t seg_lo[kMaxSegments + 1];
    const uint32_t *ev_branch;
    const uint32_t *ev_seq;
    const uint32_t *branch_first;
    const uint32_t *branch_len;
    const uint32_t *brow;
    uint32_t s_cap;
    uint32_t *jt;                // [(G + 1) * B]: row k = J_k, last seq of each branch before segment k
    uint32_t *cnt;               // [B] seq of each branch's first batch event (0: none), then [G] partial counts, [G] edge counts
    uint32_t *pflag;             // [n] partial flags (k_index drains)
    uint32_t *plist;             // partial events of segment k at plist[seg_lo[k] - bs ..]
    uint32_t *pcount;            // [G]
    // LowestAfter of the rows up to J_k (k_seg_la_edge): the events whose
    // range reaches them -- partial events, their successors on their
    // branch, every branch's first event in the segment
    uint32_t *elist;
    uint32_t *ecount;
    uint32_t own_seg;            // row-segment rank: its first segment; LX_NONE: every segment of the batch
    uint32_t own_lo;             // rows below it are another rank's: their entries go to out[owner rank]
    uint32_t *out;               // per destination rank d: out_cap triples (row, column, seq) at out + 3 d out_cap
    uint32_t *out_count;         // [ranks]
    uint64_t out_cap;
    // row-segment rank: segments per rank (its own segment walked as per_rank
    // side-by-side sub-segments); the owner rank of segment k is k / per_rank
    uint32_t per_rank;
    // row-segment rank: the planes hold the own rows [own_lo, hi) only; the
    // rows of other ranks it received live in rhb at row hslot[x] (NULL:
    // whole planes, every row at its own index)
    const uint32_t *rhb;
    const uint32_t *hslot;
};

// Row-segment multi-GPU exchange (lx_rowseg.cpp): rows a rank needs from the
// others, and the moves of rows and LowestAfter entries between ranks
struct RsArgs {
    uint32_t *hb;
    uint32_t *la;
    uint64_t stride;
    uint32_t B;
    uint32_t lo, hi;             // own events
    const uint32_t *pflag;       // own partial flags (index e - lo)
    uint32_t partials_done;
    uint32_t *need;              // [n_events]: 1 = requested and not received
    uint32_t *req;               // requested rows (appended)
    uint32_t *req_count;
    uint32_t *remaining;
    // received rows: row x of another rank at rhb + hslot[x] * stride (hslot =
    // its position in req, set when it is first requested)
    uint32_t *rhb;
    uint32_t *hslot;
};

// ForklessCause across row-segment ranks (lx_rowseg_fc.hip)
struct RsqArgs {
    uint32_t G, self;            // ranks, this rank
    uint32_t n_all;              // events of the epoch
    uint32_t lo, hi;             // own rows
    uint32_t B;                  // words per shipped LA row
    uint32_t seg_lo[kMaxSegments + 1];
};

// kernel launchers (lx_kernels.hip); all enqueue on `s`
namespace lx {
hipError_t launch_seg_tables(const SegArgs &a, hipStream_t s);
hipError_t launch_seg_partial(const SegArgs &a, uint32_t k, uint32_t count, hipStream_t s);
hipError_t launch_seg_edges(const SegArgs &a, uint32_t k, uint32_t n_partial, hipStream_t s);
hipError_t launch_seg_la_edge(const SegArgs &a, uint32_t k, uint32_t count, hipStream_t s);
hipError_t launch_rs_refs(const SegArgs &a, const RsArgs &r, const uint32_t *n_partial /* per own segment */,
                          hipStream_t s);
hipError_t rsq_tmp_bytes(uint64_t n, uint32_t G, size_t *bytes);
hipError_t launch_rsq_route(const RsqArgs &a, const uint32_t *qa, const uint32_t *qb, uint64_t n, uint32_t *scratch,
                            void *tmp, size_t tmp_bytes, uint32_t *ra, uint32_t *rb, uint32_t *perm, uint32_t *counts,
                            hipStream_t s);
hipError_t launch_rsq_need(const RsqArgs &a, const uint32_t *ra, const uint32_t *rb, uint64_t m, uint32_t *stamp,
                           uint32_t want, uint32_t *list, uint32_t *count, hipStream_t s);
hipError_t launch_rsq_group(const RsqArgs &a, const uint32_t *list, uint32_t n, void *tmp, size_t tmp_bytes,
                            uint32_t *ids, uint32_t *counts, hipStream_t s);
hipError_t launch_rsq_la_gather(const RsqArgs &a, const uint32_t *la, uint64_t stride, const uint32_t *ids,
                                uint32_t n, uint32_t *rows, hipStream_t s);
hipError_t launch_rsq_la_store(const RsqArgs &a, uint32_t *la_recv, uint64_t stride, const uint32_t *ids, uint32_t n,
                               const uint32_t *rows, uint32_t *stamp, uint32_t *slot, uint32_t arrived, hipStream_t s);
hipError_t launch_rsq_unroute(const uint32_t *perm, const uint8_t *ans, uint64_t n, uint8_t *out, hipStream_t s);
hipError_t launch_rows_unroute(const uint32_t *perm, const uint8_t *rows, uint64_t slot, const uint32_t *len,
                               uint64_t n, uint8_t *out, uint32_t *out_len, hipStream_t s);
hipError_t launch_rs_bucket(const SegArgs &a, const RsArgs &r, uint32_t n_req, uint32_t *out, uint32_t *counts,
                            hipStream_t s);
hipError_t launch_rs_gather(const RsArgs &r, const uint32_t *ids, uint32_t n, uint32_t *rows, uint32_t *ready,
                            hipStream_t s);
hipError_t launch_rs_scatter(const RsArgs &r, const uint32_t *ids, uint32_t n, const uint32_t *rows,
                             const uint32_t *ready, hipStream_t s);
hipError_t launch_rs_la_apply(const RsArgs &r, const uint32_t *triples, uint64_t n, hipStream_t s);
hipError_t launch_batch_prepare(const BatchArgs &a, void *scan_tmp, size_t scan_tmp_bytes, hipStream_t s);
hipError_t launch_batch_finish(const BatchArgs &a, uint32_t jump_rounds, hipStream_t s);
hipError_t launch_small(const SmallArgs &a, hipStream_t s);
hipError_t launch_small_dbl(const SmallArgs &a, hipStream_t s);   // needs the image on the device
hipError_t launch_small_inline(const SmallInlineArgs &a, hipStream_t s);
hipError_t launch_add1_row(const Add1RowArgs &a, hipStream_t s);
hipError_t scan_tmp_bytes(uint32_t n, size_t *bytes);
hipError_t launch_undo_claims(const BatchArgs &a, hipStream_t s);
hipError_t launch_index(const IndexArgs &a, hipStream_t s);
hipError_t launch_dbl(const DblArgs &a, hipStream_t s);
hipError_t launch_stage(uint32_t *dst, const uint32_t *src, uint64_t words, hipStream_t s);
hipError_t launch_marks(const MarkArgs &a, hipStream_t s);
hipError_t launch_fc(const FcArgs &a, uint32_t cols, bool forks, hipStream_t s);
hipError_t launch_fc_combine(const uint32_t *sum, uint8_t *out, uint64_t n, uint32_t quorum, hipStream_t s);
// column-shard early exit (lx_fc_shard_*): shard 0's decisions as bits per
// query (dec: decided, ans: the answer), the undecided queries compacted in
// query order, the answers from both
hipError_t launch_fcs_decide(const uint32_t *part, uint64_t n, uint32_t quorum, uint32_t rest, unsigned long long *dec,
                             unsigned long long *ans, hipStream_t s);
hipError_t fcs_scan_bytes(uint64_t n, size_t *bytes);
hipError_t launch_fcs_undecided(const unsigned long long *dec, uint64_t n, const uint32_t *a, const uint32_t *b,
                                const uint32_t *p0, uint32_t *flag, uint32_t *pos, void *tmp, size_t tmp_bytes,
                                uint32_t *idx, uint32_t *a2, uint32_t *b2, uint32_t *p2, hipStream_t s);
hipError_t launch_fcs_answer(const unsigned long long *dec, const unsigned long long *ans, uint64_t n, uint64_t m,
                             const uint32_t *idx, const uint32_t *sum, uint32_t quorum, uint8_t *out, hipStream_t s);
hipError_t launch_unfill(const UnfillArgs &a, hipStream_t s);
hipError_t launch_zero_rows(uint32_t *hb, uint32_t *la, uint64_t stride, uint32_t lo, uint32_t hi, hipStream_t s);
hipError_t launch_la_tail(const TailArgs &a, hipStream_t s);
hipError_t launch_fill_u32(uint32_t *p, uint64_t n, uint32_t v, hipStream_t s);
hipError_t launch_shard_dmin(const uint32_t *hb, uint64_t pstride, const uint32_t *cmap, const uint32_t *branch_len,
                             const uint32_t *brow, uint32_t s_cap, const uint32_t *branch_first, const uint32_t *sx_len,
                             uint32_t B, const uint32_t *cols, uint32_t ncols, uint32_t *dmin, hipStream_t s);
hipError_t launch_shard_dirty_rows(const uint32_t *brow, uint32_t s_cap, const uint32_t *meta, uint32_t nmeta,
                                   uint32_t *rows, hipStream_t s);
hipError_t launch_shard_rows(const uint32_t *ev_branch, const uint32_t *branch_creator, uint32_t n, uint32_t lo,
                             uint32_t hi, uint32_t *flag, uint32_t *pos, void *scan_tmp, size_t scan_bytes,
                             uint32_t *rows, hipStream_t s);
hipError_t launch_la_xfer(const XferArgs &a, hipStream_t s);
hipError_t launch_dirty_la(const UnfillArgs &a, uint32_t *flag, hipStream_t s);
hipError_t persist_tmp_bytes(uint32_t n, size_t *bytes);
hipError_t launch_compact(const uint32_t *flag, uint32_t *pos, uint32_t n, void *tmp, size_t tmp_bytes,
                          uint32_t *rows, hipStream_t s);
hipError_t launch_iota(uint32_t *rows, uint32_t lo, uint32_t n, hipStream_t s);
hipError_t launch_row_offsets(const RowsArgs &a, uint64_t *len, uint64_t *off, void *tmp, size_t tmp_bytes,
                              hipStream_t s);
hipError_t launch_encode_rows(const RowsArgs &a, const uint64_t *off, uint64_t base, uint32_t *out, hipStream_t s);
hipError_t launch_get_rows(const GetArgs &a, hipStream_t s);
hipError_t launch_get_server(const GetSrvArgs &a, hipStream_t s);
hipError_t launch_load_rows(const LoadArgs &a, hipStream_t s);
hipError_t launch_load_raw(const LoadRawArgs &a, hipStream_t s);
hipError_t launch_load_check(const LoadRawArgs &a, uint32_t n, hipStream_t s);
hipError_t launch_load_marks_ok(const uint32_t *hb, uint64_t stride, uint32_t n, uint32_t B, const uint32_t *cheat_col,
                                uint32_t *bad, hipStream_t s);
hipError_t launch_load_verify_la(const LoadVerifyArgs &a, hipStream_t s);
hipError_t launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint32_t n, uint32_t *dst, hipStream_t s);
hipError_t launch_qi_apply(const QiArgs &a, const QiBatch &b, hipStream_t s);
hipError_t launch_qi_median(const QiArgs &a, hipStream_t s);
hipError_t launch_qi_metric(const QiArgs &a, const uint32_t *ev, uint32_t n, uint32_t cap, unsigned long long *out,
                            hipStream_t s);
uint32_t root_fc_splits(uint32_t n_cand, uint32_t n_roots, uint32_t ncols);
hipError_t launch_root_fc(const RootFcArgs &a, bool forks, bool seq16, hipStream_t s);
uint32_t root_fc_blocks(const RootFcArgs &a);
hipError_t launch_root_fc_multi(const RootFcArgs *am, uint32_t n_steps, uint32_t blocks, bool forks, bool seq16,
                                hipStream_t s);
hipError_t launch_root_quorum_multi(const QuorumArgs *am, uint32_t n_steps, uint32_t blocks, hipStream_t s);
hipError_t launch_root_quorum(const QuorumArgs &a, hipStream_t s);
hipError_t launch_fc_tile_out(const uint32_t *psum, uint32_t n_split, uint32_t n_cand, uint32_t rp, uint32_t n_roots,
                              uint32_t quorum, const uint8_t *tag, uint8_t *out, uint64_t pitch, hipStream_t s);
hipError_t launch_votes(const VoteArgs &a, uint32_t n_voters, bool round1, hipStream_t s);
hipError_t launch_votes_multi(const VoteArgs *am, uint32_t n, uint32_t max_voters, uint32_t w, bool round1,
                              hipStream_t s);
hipError_t launch_scatter(const ScatterDesc *desc, uint32_t n, uint64_t max_bytes, const uint8_t *base,
                          hipStream_t s);
hipError_t launch_gather_rows(uint32_t *dst, const uint32_t *src, uint64_t stride, uint32_t V, const uint32_t *rows,
                              uint32_t n, hipStream_t s);
hipError_t launch_readback(uint32_t *dst, const uint32_t *a, uint32_t na, const uint32_t *b, uint32_t nb,
                           hipStream_t s);
hipError_t launch_copy_rows(uint32_t *dst, uint64_t dst_stride, const uint32_t *src, uint64_t src_stride,
                            uint64_t rows, uint64_t cols, hipStream_t s);
}  // namespace lx

// Read-only view of an index handle for the abft engine (lx_capi.cpp).
#include <vector>
struct lx_index;
struct IndexView {
    hipStream_t stream;
    int device;
    uint32_t *hb, *la;
    uint64_t stride;
    uint64_t n_events;
    uint32_t V, B, quorum;
    uint32_t max_seq;            // largest seq indexed this epoch
    const uint32_t *wpad;
    const uint32_t *ev_branch;
    const uint32_t *ev_creator;
    const std::vector<uint32_t> *weights;
    const std::vector<std::vector<uint32_t>> *by_creator;
    uint32_t shard_count;
};
int lx_index_view(lx_index *h, IndexView *out);
