// lx_kernels.hip -- CDNA4 (gfx950) kernels of the vector-clock / ForklessCause index.
//
// Integer, HBM/latency-bound work: no MFMA.  Kernels:
//   batch prepare/finish : parallel branch assignment equivalent to the
//                          sequential fillGlobalBranchID (vecengine/index.go:105-141)
//   k_index              : fused HighestBefore max-join + LowestAfter range fill,
//                          one persistent column-slice walker per workgroup
//                          (replaces CollectFrom x parents and DfsSubgraph,
//                          vecengine/index.go:165-225, vecfc/vector_ops.go:49-79)
//   k_marks              : per-creator fork markers (vecengine/index.go:173-209)
//   k_fc                 : batched ForklessCause (vecfc/forkless_cause.go:40-82)
//   k_unfill/k_unclaim   : DropNotFlushed rollback (vecengine/index.go:88-96)
#include <hipcub/hipcub.hpp>

#include <vector>

#include "lx_internal.h"

namespace lx {

// ----------------------------------------------------------------------------
// error codes stored in the batch status word: (batch_pos << 8) | code
enum : uint32_t { E_ARG = 1, E_ORDER = 2, E_EVENT = 3 };

__device__ __forceinline__ uint32_t ld_l2(const uint32_t *p) {
    // agent-scope relaxed load: global_load ... sc1, bypasses the CU's L1 so a
    // value stored by another wave of this workgroup is never read stale.
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Same, but consumes the value on the spot so the compiler's vmcnt wait lands
// inside the (cold) branch issuing it instead of at the merge point, where it
// would also wait for every store in flight (gfx950 counts stores in vmcnt).
__device__ __forceinline__ uint32_t ld_l2_now(const uint32_t *p) {
    uint32_t v = ld_l2(p);
    asm volatile("" ::"v"(v));
    return v;
}

// ---------------------------------------------------------------------------- batch prepare
// Per-event metadata, eventcheck invariants the index relies on
// (parentscheck/parents_check.go:25-63, basiccheck/basic_check.go:24-44) and
// claims of "first self-child" / "first root".  An in-batch self-parent's
// creator and seq come from the batch inputs (the metadata of this launch's
// other threads is not visible yet).  first_child of rows not yet added is
// always NONE (reset, growth and rollback keep it so): claims land on it.
__global__ void k_validate_claim(BatchArgs a, unsigned long long *err) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    // the batch's highest seq: the workgroup's maximum into tmp_br[block]
    // (free until k_assign), reduced by k_seq_max.  Atomics on one address are
    // performed one by one where every XCD sees them: ~11 ns each, 1.8 ms for
    // one per wave of a 10M-event batch.
    __shared__ uint32_t wmax[4];
    uint32_t smax = e < a.n ? a.seq[e] : 0u;
#pragma unroll
    for (int off = 32; off; off >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, off, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x / 64] = smax;
    __syncthreads();
    if (threadIdx.x == 0) a.tmp_br[blockIdx.x] = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (e >= a.n) return;
    uint32_t g = a.batch_start + e;
    uint32_t c = a.creator[e], s = a.seq[e];
    uint32_t p0 = a.poff[e], p1 = a.poff[e + 1];
    uint32_t code = 0;
    if (c >= a.V) {
        code = E_ARG;
    } else if (s == 0 || s >= 0x7FFFFFFEu) {
        code = E_EVENT;
    } else if (p1 < p0) {
        code = E_ARG;
    } else {
        // the first twelve parents loaded without an early exit, so that the
        // loads are in flight together (a loop that leaves at the first bad
        // parent waits for each load in turn: 1.8 ms of a 10M-event batch)
        const uint32_t np = p1 - p0;
        bool bad = false;
        if (np) {
            uint32_t x[LX_MAXP];
#pragma unroll
            for (uint32_t k = 0; k < LX_MAXP; k++) x[k] = a.par[p0 + min(k, np - 1)];   // clamped: no branch per load
#pragma unroll
            for (uint32_t k = 0; k < LX_MAXP; k++) bad |= x[k] >= g;
            for (uint32_t k = p0 + LX_MAXP; k < p1; k++) bad |= a.par[k] >= g;
        }
        if (bad) code = E_ORDER;
        if (!code && s > 1) {
            if (p1 == p0) {
                code = E_EVENT;
            } else {
                const uint32_t sp = a.par[p0];
                const bool in = sp >= a.batch_start;
                const uint32_t cs = in ? a.creator[sp - a.batch_start] : a.ev_creator[sp];
                const uint32_t ss = in ? a.seq[sp - a.batch_start] : a.ev_seq[sp];
                if (cs != c || ss + 1 != s) code = E_EVENT;
            }
        }
    }
    // (stores after the loads: gfx950's vmcnt counts stores, an earlier store
    // would make every load wait for it)
    a.ev_creator[g] = c;
    a.ev_seq[g] = s;
    if (code) {
        atomicMin(err, ((unsigned long long)e << 8) | code);
        return;
    }
    if (s > 1) atomicMin(&a.first_child[a.par[p0]], g);
    else atomicMin(&a.first_root[c], g);
}

// status[2] = max(status[2], max of v[0 .. n)): one workgroup, one atomic
__global__ __launch_bounds__(1024) void k_seq_max(const uint32_t *v, uint32_t n, uint32_t *out) {
    __shared__ uint32_t wmax[16];
    uint32_t m = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 1024) m = max(m, v[i]);
#pragma unroll
    for (int off = 32; off; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x / 64] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; w++) m = max(m, wmax[w]);
        atomicMax(out, m);
    }
}

// A self-parented event continues its self-parent's branch iff it is the first
// self-child of that parent in Add order (then lastSeq[branch]+1 == seq held at
// its Add time); a root continues the creator's original branch iff it is the
// creator's first root.  Every other event opens a new branch.
__global__ void k_isfork(BatchArgs a) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n) return;
    uint32_t g = a.batch_start + e;
    uint32_t s = a.seq[e];
    uint32_t f = (s > 1) ? (a.first_child[a.par[a.poff[e]]] != g) : (a.first_root[a.creator[e]] != g);
    a.isfork[e] = f;
}

__global__ void k_unclaim_batch(BatchArgs a) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n) return;
    uint32_t c = a.creator[e], s = a.seq[e];
    uint32_t p0 = a.poff[e], p1 = a.poff[e + 1];
    if (s > 1 && p1 > p0) {
        uint32_t sp = a.par[p0];
        if (sp < a.batch_start + a.n && a.first_child[sp] != LX_NONE && a.first_child[sp] >= a.batch_start)
            a.first_child[sp] = LX_NONE;
    } else if (c < a.V) {
        if (a.first_root[c] != LX_NONE && a.first_root[c] >= a.batch_start) a.first_root[c] = LX_NONE;
    }
}

hipError_t scan_tmp_bytes(uint32_t n, size_t *bytes) {
    *bytes = 0;
    return hipcub::DeviceScan::InclusiveSum(nullptr, *bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
}

static inline uint32_t nblk(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

hipError_t launch_batch_prepare(const BatchArgs &a, void *scan_tmp, size_t scan_tmp_bytes, hipStream_t s) {
    unsigned long long *err = (unsigned long long *)(a.status + 8);
    hipLaunchKernelGGL(k_validate_claim, dim3(nblk(a.n, 256)), dim3(256), 0, s, a, err);
    hipLaunchKernelGGL(k_seq_max, dim3(1), dim3(1024), 0, s, a.tmp_br, nblk(a.n, 256), a.status + 2);
    hipLaunchKernelGGL(k_isfork, dim3(nblk(a.n, 256)), dim3(256), 0, s, a);
    size_t tb = scan_tmp_bytes;
    hipError_t r = hipcub::DeviceScan::InclusiveSum(scan_tmp, tb, a.isfork, a.rank, (int)a.n, s);
    if (r != hipSuccess) return r;
    return hipGetLastError();
}

hipError_t launch_undo_claims(const BatchArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_unclaim_batch, dim3(nblk(a.n, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- batch finish
__global__ void k_assign(BatchArgs a) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n) return;
    uint32_t g = a.batch_start + e;
    uint32_t f = a.isfork[e], rk = a.rank[e];
    uint32_t s = a.seq[e], c = a.creator[e];
    a.ev_bbefore[g] = a.B0 + rk - f;
    uint32_t sp = (s > 1) ? a.par[a.poff[e]] : LX_NONE;
    a.ev_sp[g] = sp;
    if (a.nofork) {
        // no fork branch anywhere (B = V before and after the batch): every
        // event continues its creator's original branch (fillGlobalBranchID,
        // vecengine/index.go:105-141), no pointer jumping needed
        a.tmp_br[e] = c;
        a.jmp[e] = e;
    } else if (f) {
        uint32_t br = a.B0 + rk - 1;
        a.branch_first[br] = s;
        a.branch_creator[br] = c;
        a.branch_len[br] = 0;
        a.tmp_br[e] = br;
        a.jmp[e] = e;
    } else if (s == 1) {
        a.tmp_br[e] = c;
        a.jmp[e] = e;
    } else if (sp < a.batch_start) {
        a.tmp_br[e] = a.ev_branch[sp];
        a.jmp[e] = e;
    } else {
        a.tmp_br[e] = LX_NONE;
        a.jmp[e] = sp - a.batch_start;
    }
}

// pointer jumping along in-batch self-parent chains; round r runs only if
// round r-1 saw an unresolved event (flag words status[16 + r])
__global__ void k_jump(BatchArgs a, uint32_t r) {
    if (r > 0 && a.status[16 + r - 1] == 0) return;
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n) return;
    if (a.tmp_br[e] != LX_NONE) return;
    uint32_t j = a.jmp[e];
    uint32_t t = a.tmp_br[j];
    if (t != LX_NONE) {
        a.tmp_br[e] = t;
    } else {
        a.jmp[e] = a.jmp[j];
        a.status[16 + r] = 1;
    }
}

__global__ void k_finalize(BatchArgs a) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n) return;
    uint32_t g = a.batch_start + e;
    uint32_t br = a.tmp_br[e];
    uint32_t s = a.seq[e];
    if (br == LX_NONE) {   // too few jump rounds: reported by the host, nothing written
        atomicAdd(&a.status[4], 1u);
        return;
    }
    a.ev_branch[g] = br;
    uint32_t first = a.branch_first[br];
    a.brow[(uint64_t)br * a.s_cap + (s - first)] = g;
    // a branch is a chain through first_child (its first self-child continues
    // it, k_isfork): the batch's last event of the branch has none, and holds
    // its highest seq -- one plain store per branch instead of an atomic per event
    if (a.first_child[g] == LX_NONE) a.branch_len[br] = s - first + 1;
    uint32_t p0 = a.poff[e], p1 = a.poff[e + 1];
    uint32_t np = p1 - p0;
    uint32_t prev = (s > 1 && !a.isfork[e]) ? a.par[p0] : LX_NONE;
    // inline parents sorted oldest first: the walker folds them in chunks of 4,
    // so the newest (last to complete) chunk is the only one left at the end
    uint32_t w[LX_MAXP];
#pragma unroll
    for (int k = 0; k < LX_MAXP; k++) w[k] = (k < (int)np) ? a.par[p0 + k] : 0xFFFFFFFFu;
#pragma unroll
    for (int i = 1; i < LX_MAXP; i++) {
#pragma unroll
        for (int j = i; j > 0; j--) {
            const uint32_t x = w[j - 1], y = w[j];
            w[j - 1] = min(x, y);
            w[j] = max(x, y);
        }
    }
    // round-blocked SoA: record e's q-th 16 B at [e/64][q][e%64], so 64
    // consecutive records form one contiguous 4-KB block (one LDS-DMA round)
    // and a wave reading field q of 64 consecutive records is conflict-free
    uint4 *rq = reinterpret_cast<uint4 *>(a.rec) + (uint64_t)(e / 64) * 64 * LX_REC_Q + (e % 64);
    rq[0] = make_uint4(br, s, np, prev);
#pragma unroll
    for (int k = 0; k < LX_MAXP / 4; k++) {
        uint32_t v[4];
#pragma unroll
        for (int t = 0; t < 4; t++) v[t] = (4 * k + t < (int)np) ? w[4 * k + t] : LX_NONE;
        rq[64 * (1 + k)] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    if (a.crec) {
        // compact record (lx_internal.h): distances back instead of indices
        // (the host enables it only when every branch and seq fits 16 bits)
        uint32_t d[LX_MAXP];
        bool wide = np > 255u || (prev != LX_NONE && g - prev >= 0xFFFFFFu);
#pragma unroll
        for (int k = 0; k < LX_MAXP; k++) {
            d[k] = (k < (int)np) ? g - w[k] : 0u;
            wide |= d[k] >= 0xFFFFu;
        }
        uint4 *cq = reinterpret_cast<uint4 *>(a.crec) + (uint64_t)(e / 64) * 64 * LX_CREC_Q + (e % 64);
        const uint32_t c1 = wide ? kCrecWide : np | ((prev == LX_NONE ? 0u : g - prev) << 8);
        cq[0] = make_uint4(br | (s << 16), c1, d[0] | (d[1] << 16), d[2] | (d[3] << 16));
        cq[64] = make_uint4(d[4] | (d[5] << 16), d[6] | (d[7] << 16), d[8] | (d[9] << 16), d[10] | (d[11] << 16));
    }
}

hipError_t launch_batch_finish(const BatchArgs &a, uint32_t jump_rounds, hipStream_t s) {
    hipLaunchKernelGGL(k_assign, dim3(nblk(a.n, 256)), dim3(256), 0, s, a);
    jump_rounds = std::min<uint32_t>(jump_rounds, 32);
    for (uint32_t r = 0; r < jump_rounds; r++) hipLaunchKernelGGL(k_jump, dim3(nblk(a.n, 256)), dim3(256), 0, s, a, r);
    hipLaunchKernelGGL(k_finalize, dim3(nblk(a.n, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- index walker
//
// One workgroup owns CPW columns (branches) and walks ALL events of the batch
// in Add order.  Columns are independent (max-join and LowestAfter range fill
// of column c touch only column c of HB and rows of branch c in LA), so the
// workgroups never communicate; one launch covers the whole batch.
//
// The batch's DAG depth (not its size) bounds the walk: every level costs at
// least one pass of the compute loop, so the compute waves do only what the
// critical path needs -- fold parents, publish -- and the rest runs beside them.
// Roles (NCW compute waves + 1 loader + kND drain waves):
//  * loader: streams 64-B event records (round-blocked SoA, one 4-KB block per
//    64 events) into an LDS record ring by LDS-DMA (global_load_lds_dwordx4,
//    up to 15 rounds in flight) and publishes each round with a tag after its
//    own vmcnt wait;
//  * compute waves (block layout): a wave's 16 quads own 16 consecutive
//    events; lane j of a quad folds the inline parents j, j+4, j+8 from their
//    LDS ring slots, the quad merges maxima and readiness by DPP and publishes
//    the event's CPW seqs into its slot.  No global access on the hot path;
//  * drain waves (rounds of 64 events, round r on wave r % kND): store the HB
//    row and do the LowestAfter range fill, reading RAW(prev) from the ring.
// Slots carry their event tag next to the seqs in one 8-B (CPW 1) or 16-B
// (CPW 2) unit, or two 16-B units in separate arrays (CPW 4: {tag, s0, s1, s2},
// {tag, s3}; one unit {tag, s0 | s1 << 16, s2 | s3 << 16, 0} when every seq of
// the epoch fits 16 bits); one lane's ds_read/ds_write of such a unit is a
// single LDS access, so a unit whose tag matches is consistent.  A tag above
// the expected one means the slot was reused: that parent's HB row is read
// from L2 once its drain reports it stored (rare: parents older than the ring,
// or from an earlier batch).  Lanes never block inside a pass, so
// dependencies between lanes of one wave cannot deadlock; drains wait only for
// older events and keep publishing their own progress.
constexpr int kND = 4;               // drain waves
#ifdef LX_PROBE_SKEW
// probe build: drain timestamps of every 32nd round per workgroup, and each
// workgroup's (walk << 16 | slice) -- how far the slices of one walk drift apart
constexpr int kProbeSkewSlots = 2048;
__device__ unsigned long long g_probe_skew[1024 * kProbeSkewSlots];
__device__ uint32_t g_probe_map[1024];
extern "C" int lx_probe_skew_read(unsigned long long *stamps, uint32_t *map) {
    if (hipMemcpyFromSymbol(stamps, HIP_SYMBOL(g_probe_skew), sizeof(g_probe_skew), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(map, HIP_SYMBOL(g_probe_map), sizeof(g_probe_map), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
constexpr int kRR = 1024;            // record ring (events)

template <int CPW>
struct Ring {
    // slots: 64 KB of units (CPW 2 uses one 16-B unit per slot: 2048 slots in 32 KB)
    static constexpr int BYTES = CPW == 2 ? 32768 : 65536;
    static constexpr int N = BYTES / (CPW == 1 ? 8 : CPW == 2 ? 16 : 32);
};

struct alignas(16) WalkShared {
    uint32_t copied[8];      // rounds drained (ring and record data consumed) per drain wave (<= 8 drains)
    uint32_t stored[8];      // rounds whose global stores are complete per drain wave
    uint32_t req;            // a compute lane waits for `stored`: drains flush
    uint32_t p_issued, p_done;   // LX_WALKER_PROF: loader progress (rounds issued / landed)
};

template <int ND = kND>
__device__ __forceinline__ bool round_done(const uint32_t *cnt, uint32_t ev) {
    const uint32_t r = ev / 64;
    return __hip_atomic_load(cnt + (r % ND), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > r / ND;
}

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

// LDS read in inline asm: the compiler orders a plain LDS load after every
// LDS-DMA (global_load_lds) still in flight (an s_waitcnt vmcnt(0))
__device__ __forceinline__ uint32_t lds_ld32(uint32_t addr) {
    uint32_t x;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(addr) : "memory");
    return x;
}

// a slot as read: tag(s) and seqs
template <int CPW>
struct Slot {
    uint32_t t0, t1;       // t1 = second unit's tag (CPW 4), else t0
    uint32_t v[CPW];
};

// one slot (the drains' spin loop and the overflow path): a single access per
// unit, so a spinning drain adds no redundant LDS traffic beside the compute waves
// PK (4-column slices, every seq of the epoch <= 0xFFFF): one 16-B unit
// {tag, s0 | s1 << 16, s2 | s3 << 16, 0} per slot instead of two
__device__ __forceinline__ void unpack16(const u4v &x, uint32_t *v) {
    v[0] = x.y & 0xFFFFu; v[1] = x.y >> 16; v[2] = x.z & 0xFFFFu; v[3] = x.z >> 16;
}
template <int CPW, bool PK = false>
__device__ __forceinline__ void ring_read1(uint32_t A, uint32_t B, uint32_t s, Slot<CPW> &o) {
    if constexpr (PK && (CPW == 8 || CPW == 12)) {
        // two units {tag, s0 | s1 << 16, s2 | s3 << 16, s4 | s5 << 16}, {tag, s6 | s7 << 16, 0, 0}
        // (12 columns: {tag, s6 | s7 << 16, s8 | s9 << 16, s10 | s11 << 16})
        u4v x, y;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(x), "=&v"(y)
                     : "v"(A + s * 16u), "v"(B + s * 16u)
                     : "memory");
        o.t0 = x.x;
        o.t1 = y.x;
        const uint32_t w[6] = {x.y, x.z, x.w, y.y, y.z, y.w};
#pragma unroll
        for (int k = 0; k < CPW; k++) o.v[k] = (k & 1) ? w[(k / 2) % 6] >> 16 : w[(k / 2) % 6] & 0xFFFFu;
        return;
    } else if constexpr (PK) {
        static_assert(CPW == 4, "packed slots: 4-, 8- or 12-column slices");
        u4v x;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x) : "v"(A + s * 16u) : "memory");
        o.t0 = o.t1 = x.x;
        uint32_t v[4];
        unpack16(x, v);
#pragma unroll
        for (int k = 0; k < CPW; k++) o.v[k] = v[k % 4];
        return;
    }
    if (CPW == 1) {
        u2v x;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x) : "v"(A + s * 8u) : "memory");
        o.t0 = o.t1 = x.x;
        o.v[0] = x.y;
    } else if (CPW == 2) {
        u4v x;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x) : "v"(A + s * 16u) : "memory");
        o.t0 = o.t1 = x.x;
        o.v[0] = x.y;
        o.v[1 % CPW] = x.z;
    } else {
        u4v x, y;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(x), "=&v"(y)
                     : "v"(A + s * 16u), "v"(B + s * 16u)
                     : "memory");
        o.t0 = x.x;
        o.t1 = y.x;
        o.v[0] = x.y;
        o.v[1 % CPW] = x.z;
        o.v[2 % CPW] = x.w;
        o.v[3 % CPW] = y.y;
    }
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)p;
}

// field q of the record in record-ring slot `slot` (round-blocked SoA, RQ
// 16-B fields per record: EventRec 4, CRec 2)
template <int RQ = LX_REC_Q>
__device__ __forceinline__ uint32_t rec_off(uint32_t slot, uint32_t q) {
    return (slot & ~63u) * RQ + q * 64u + (slot & 63u);
}

// the loader's wait for its oldest record round: all but the RQ DMAs of each
// of the k younger rounds landed (vmcnt is an immediate: one case per k)
template <int RQ>
__device__ __forceinline__ void wait_rounds(uint32_t k) {
#define LX_VMW(c) case c: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RQ * c) : "memory"); break;
    switch (k) {
        LX_VMW(0) LX_VMW(1) LX_VMW(2) LX_VMW(3) LX_VMW(4) LX_VMW(5) LX_VMW(6) LX_VMW(7)
        LX_VMW(8) LX_VMW(9) LX_VMW(10) LX_VMW(11) LX_VMW(12) LX_VMW(13) LX_VMW(14)
        default:
            if constexpr (RQ == 2) {
                switch (k) {
                    LX_VMW(15) LX_VMW(16) LX_VMW(17) LX_VMW(18) LX_VMW(19) LX_VMW(20) LX_VMW(21) LX_VMW(22)
                    LX_VMW(23) LX_VMW(24) LX_VMW(25) LX_VMW(26) LX_VMW(27) LX_VMW(28) LX_VMW(29)
                    default: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
                }
            } else {
                asm volatile("s_waitcnt vmcnt(56)" ::: "memory");
            }
            break;
    }
#undef LX_VMW
}

// Per-wave walker counters (LX_PROF=1) are compiled in only with
// -DLX_WALKER_PROF (make WPROF=1): the increments cost the compute pass
// several VALU instructions.

#ifdef LX_WALKER_PROF
#define LX_WP(x) x
#else
#define LX_WP(x)
#endif

// MASKED: older rows may carry fork marks in bit 31 (B > V); without forks
// the seq values are used unmasked.
constexpr uint32_t kNullTag = 0xFFFFFFFFu;   // null slot: never an event tag (tags are lp + 1 <= n)
// any of a lane's three parents (expected tag = local index + 1, or kNullTag)
// at least `reach` events before event lp
template <int NPL>
__device__ __forceinline__ bool far_parent(const uint32_t px[NPL], uint32_t lp, uint32_t reach) {
    bool f = false;
#pragma unroll
    for (int k = 0; k < NPL; k++) f |= px[k] != kNullTag && lp - (px[k] - 1u) >= reach;
    return f;
}
// DPP quad permutations (lanes 4q..4q+3): swap neighbours, swap pairs
constexpr int kQuadSwap1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kQuadSwap2 = 0x4E;   // quad_perm [2,3,0,1]
__device__ __forceinline__ uint32_t quad_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kQuadSwap1, 0xF, 0xF, false));
    return max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kQuadSwap2, 0xF, 0xF, false));
}
// packed 16-bit maxima (two columns per dword) and their quad reduction
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_pk_max_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ uint32_t quad_pk_max(uint32_t v) {
    v = pk_max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kQuadSwap1, 0xF, 0xF, true));
    return pk_max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kQuadSwap2, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t quad_and(uint32_t v) {
    v &= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kQuadSwap1, 0xF, 0xF, false);
    return v & (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kQuadSwap2, 0xF, 0xF, false);
}

// Block walker fold: the slot units of a lane's three parents (unit A at pa[k];
// unit B, CPW 4 only, in the B array (RN + 1) * 16 bytes further) and the drain
// watermark at W, one LDS round trip.  tg[k] = the units' tags (equal for one
// unit), pv[k] = the parent's CPW seqs.
template <int CPW, int RN, bool PK = false>
__device__ __forceinline__ void blk_fold(const uint32_t pa[3], uint32_t W, uint32_t tg[3][2], uint32_t pv[3][CPW],
                                         uint32_t &cw) {
    if constexpr (PK && CPW == 4) {
        u4v x0, x1, x2;
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %5\n\t"
            "ds_read_b128 %2, %6\n\t"
            "ds_read_b32 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(cw)
            : "v"(pa[0]), "v"(pa[1]), "v"(pa[2]), "v"(W)
            : "memory");
        const u4v x[3] = {x0, x1, x2};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            // packed: pv[k][0] = s0 | s1 << 16, pv[k][1] = s2 | s3 << 16 (the
            // fold takes packed 16-bit maxima)
            tg[k][0] = tg[k][1] = x[k].x;
            pv[k][0] = x[k].y; pv[k][1 % CPW] = x[k].z; pv[k][2 % CPW] = 0u; pv[k][3 % CPW] = 0u;
        }
        return;
    }
    if constexpr (CPW == 4 || CPW == 8 || CPW == 12) {
        // two units per slot; CPW 8 / 12 (packed): pv[k][0..3 / 5] = packed column pairs
        constexpr uint32_t BOFF = (RN + 1) * 16;
        static_assert(BOFF < 65536, "ds offset field");
        u4v xa0, xb0, xa1, xb1, xa2, xb2;
        asm volatile(
            "ds_read_b128 %0, %7\n\t"
            "ds_read_b128 %1, %7 offset:%10\n\t"
            "ds_read_b128 %2, %8\n\t"
            "ds_read_b128 %3, %8 offset:%10\n\t"
            "ds_read_b128 %4, %9\n\t"
            "ds_read_b128 %5, %9 offset:%10\n\t"
            "ds_read_b32 %6, %11\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(xa0), "=&v"(xb0), "=&v"(xa1), "=&v"(xb1), "=&v"(xa2), "=&v"(xb2), "=&v"(cw)
            : "v"(pa[0]), "v"(pa[1]), "v"(pa[2]), "i"(BOFF), "v"(W)
            : "memory");
        const u4v xa[3] = {xa0, xa1, xa2};
        const u4v xb[3] = {xb0, xb1, xb2};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            tg[k][0] = xa[k].x; tg[k][1] = xb[k].x;
            pv[k][0] = xa[k].y; pv[k][1 % CPW] = xa[k].z; pv[k][2 % CPW] = xa[k].w; pv[k][3 % CPW] = xb[k].y;
            if constexpr (CPW == 12) { pv[k][4] = xb[k].z; pv[k][5] = xb[k].w; }
        }
    } else if constexpr (CPW == 2) {
        u4v x0, x1, x2;
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %5\n\t"
            "ds_read_b128 %2, %6\n\t"
            "ds_read_b32 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(cw)
            : "v"(pa[0]), "v"(pa[1]), "v"(pa[2]), "v"(W)
            : "memory");
        const u4v x[3] = {x0, x1, x2};
#pragma unroll
        for (int k = 0; k < 3; k++) { tg[k][0] = tg[k][1] = x[k].x; pv[k][0] = x[k].y; pv[k][1 % CPW] = x[k].z; }
    } else {
        u2v x0, x1, x2;
        asm volatile(
            "ds_read_b64 %0, %4\n\t"
            "ds_read_b64 %1, %5\n\t"
            "ds_read_b64 %2, %6\n\t"
            "ds_read_b32 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(cw)
            : "v"(pa[0]), "v"(pa[1]), "v"(pa[2]), "v"(W)
            : "memory");
        const u2v x[3] = {x0, x1, x2};
#pragma unroll
        for (int k = 0; k < 3; k++) { tg[k][0] = tg[k][1] = x[k].x; pv[k][0] = x[k].y; }
    }
}

// The walker kernel.  MASKED: older rows may carry fork marks in bit 31
// (B > V); PK: 4-column slices with 16-bit packed slot units (every seq of the
// epoch <= 0xFFFF).
// CR: the compact records (CRec) of 8- / 12-column packed walks
template <int CPW, int NCW, bool MASKED, bool PK, int ND_ = kND, bool CR = false>
__device__ __forceinline__ void index_body(const IndexArgs &a, const uint32_t slice) {
    static_assert(!PK || CPW >= 4, "packed slots: 4-, 8- or 12-column slices");
    static_assert(!CR || (PK && CPW >= 8), "compact records: 8- / 12-column packed walks");
    static_assert(CPW == 1 || CPW == 2 || CPW == 4 || ((CPW == 8 || CPW == 12) && PK && !MASKED), "slot layout");
    static_assert(LX_MAXP == 12, "block walker: 12 inline parents, three per lane of a quad");
    constexpr int ND = ND_;
    static_assert(ND >= 1 && ND <= 8, "drain waves");
    constexpr int RR = CR ? 2 * kRR : kRR;   // record ring (events): 64 KB either way
    constexpr int NT = 64 * (NCW + 1 + ND);
    constexpr int RQ = CR ? LX_CREC_Q : LX_REC_Q;
    constexpr int KB = CPW == 12 ? 64 : 1024 / CPW;   // recent (seq -> event) entries per owned branch
    constexpr int RN = Ring<CPW>::N;
    constexpr int RB16 = Ring<CPW>::BYTES / 16;
    static_assert(RR % 64 == 0 && RR / 64 >= 4 && RR >= 2 * 16 * NCW, "record ring");
    // slot units (A array, then B array for CPW 4), each followed by a null
    // slot (tag kNullTag, values 0) that absent parents point at
    __shared__ uint4 ring[RB16 + 2];
    __shared__ uint4 rrec[RR * RQ];              // event records
    __shared__ uint32_t rtag[RR / 64];           // per record round: batch round index + 1
    __shared__ uint2 brc[CPW * KB];              // {seq, event} of recent events of owned branches
    __shared__ uint4 dummy[128];                 // per-lane targets of suppressed writes
    __shared__ WalkShared sh;
    __shared__ uint32_t sjs[CPW];                // segment walk: J_k of the slice's columns (drains)
    __shared__ uint32_t sfirst[CPW];             // 12-column slices: first seq of each column (drains)
    __shared__ uint32_t slof[CPW];               // drains: max(J_k + 1, first seq) -- the range fill's floor

    if (slice >= a.n_slices) return;

    // null slot: unit A right after the A array (uint4 index RN, or RN / 2 for
    // 8-B units), unit B (CPW 4) after the B array
    constexpr int kNullA = CPW == 1 ? RN / 2 : RN;
    for (int i = threadIdx.x; i < RB16 + 2; i += NT)
        ring[i] = make_uint4((i == kNullA || (CPW >= 4 && i == 2 * RN + 1)) ? kNullTag : 0u, 0, 0, 0);
    for (int i = threadIdx.x; i < RR / 64; i += NT) rtag[i] = 0;
    for (int i = threadIdx.x; i < CPW * KB; i += NT) brc[i] = make_uint2(0, LX_NONE);
    if (threadIdx.x < ND) { sh.copied[threadIdx.x] = 0; sh.stored[threadIdx.x] = 0; }
    if (threadIdx.x < CPW) {
        const uint32_t ci = slice * CPW + threadIdx.x;
        sjs[threadIdx.x] = a.seg && ci < a.ncols ? a.seg_j[CPW == 12 ? ci : a.col_list[ci]] : 0u;
        sfirst[threadIdx.x] = CPW == 12 && ci < a.ncols ? a.branch_first[ci] : 1u;
        const uint32_t cf = ci < a.ncols ? a.branch_first[CPW == 12 ? ci : a.col_list[ci]] : 1u;
        slof[threadIdx.x] = max(sjs[threadIdx.x] + 1u, cf);
    }
    if (threadIdx.x == 0) { sh.req = 0; sh.p_issued = 0; sh.p_done = 0; }
    __syncthreads();

    const uint32_t n = a.n;
    const uint32_t bs = a.batch_start;
    const int wave = threadIdx.x / 64;
    const int lane = threadIdx.x % 64;
    const uint64_t stride = a.stride;
    constexpr uint32_t mask = MASKED ? LX_SEQ_MASK : 0xFFFFFFFFu;
    const uint32_t RA = lds_addr(ring);
    const uint32_t RB = RA + (uint32_t)((RN + 1) * 16);   // second units (CPW 4 only)

    // col = global branch (semantics), pc = plane column (addressing; differs
    // from col only in a column-sharded handle, which stores its own columns).
    // 12-column slices (whole handles only, launch_index) use the identity
    // column list: col = pc = c0 + k, computed where used, and the first seqs
    // live in LDS -- as per-column arrays they held ~60 SGPRs, which spilled
    // to VGPR lanes and cost a v_readlane at every use
    constexpr bool ID = CPW == 12;
    const uint32_t c0 = slice * CPW;
    const uint32_t nval = a.ncols - c0 < (uint32_t)CPW ? a.ncols - c0 : (uint32_t)CPW;
    uint32_t col_[ID ? 1 : CPW], first_[ID ? 1 : CPW], pc_[ID ? 1 : CPW];
    bool valid_[ID ? 1 : CPW];
    bool contig = true;
    if constexpr (ID) {
        contig = nval == (uint32_t)CPW && (c0 % 4) == 0;
    } else {
#pragma unroll
        for (int k = 0; k < CPW; k++) {
            const uint32_t ci = c0 + k;
            valid_[k] = ci < a.ncols;
            col_[k] = valid_[k] ? a.col_list[ci] : 0;
            pc_[k] = valid_[k] ? (a.cmap ? a.cmap[col_[k]] : col_[k]) : 0;
            first_[k] = valid_[k] ? a.branch_first[col_[k]] : 1;
            contig &= valid_[k] && pc_[k] == pc_[0] + k;
        }
        contig &= (pc_[0] % CPW) == 0;
    }
    auto col = [&](int k) -> uint32_t { return ID ? c0 + k : col_[k % (ID ? 1 : CPW)]; };
    auto pc = [&](int k) -> uint32_t { return ID ? c0 + k : pc_[k % (ID ? 1 : CPW)]; };
    auto valid = [&](int k) -> bool { return ID ? (uint32_t)k < nval : valid_[k % (ID ? 1 : CPW)]; };
    auto first = [&](int k) -> uint32_t {
        return ID ? (uint32_t)__builtin_amdgcn_readfirstlane(sfirst[k]) : first_[k % (ID ? 1 : CPW)];
    };

    if (wave == NCW) {
        // ------------------------------------------------------------ loader
        const uint32_t nrounds = (n + 63) / 64;
        // rounds in flight: the DMA round trip is long while the CU's memory
        // queue also carries the drains' stores (the block walker starved at 8)
        constexpr uint32_t DMAX = CR ? 31 : 15;   // vmcnt (6 bits): RQ DMAs per younger round <= 60
        constexpr uint32_t D = RR / 64 - 1 < DMAX ? RR / 64 - 1 : DMAX;
        uint32_t issued = 0, done = 0;
#ifdef LX_WALKER_PROF
        uint32_t l_iter = 0, l_slot = 0, l_sleep = 0;
        const unsigned long long lt0 = wall_clock64();
#endif
        const char *recb = CR ? reinterpret_cast<const char *>(a.crec) : reinterpret_cast<const char *>(a.rec);
        constexpr uint32_t RB_ = RQ * 16;   // record bytes
        while (done < nrounds) {
            bool progressed = false;
            LX_WP(l_iter++;)
            // a round's record slots are free once the drain consumed their
            // previous occupants (events ev - RR: same round offset)
            bool free = issued * 64 < (uint32_t)RR;
            if (!free && issued < nrounds && issued - done < D) {
                const uint32_t r = (issued * 64 - RR) / 64;
                free = __builtin_amdgcn_readfirstlane(lds_ld32(lds_addr(&sh.copied[r % ND]))) > r / ND;
            }
            LX_WP(if (issued < nrounds && issued - done < D && !free) l_slot++;)
            if (issued < nrounds && issued - done < D && free) {
                const uint32_t s0 = (issued * 64) % RR;
                char *dst = reinterpret_cast<char *>(rrec) + (uint64_t)s0 * RB_;
                const uint64_t base = (uint64_t)issued * 64 * RB_;
#pragma unroll
                for (int i = 0; i < RQ; i++)
                    __builtin_amdgcn_global_load_lds((const void *)(recb + base + (uint64_t)(i * 64 + lane) * 16),
                                                     (void *)(dst + i * 1024), 16, 0, 0);
                issued++;
                LX_WP(asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(&sh.p_issued)), "v"(issued) : "memory");)
                progressed = true;
            }
            if (!progressed && issued > done) {
                // the oldest round landed once at most RQ DMAs per younger round remain
                wait_rounds<RQ>(issued - done - 1);
                // (the vmcnt wait above landed the round; a release store would wait for all)
                asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(&rtag[done % (RR / 64)])), "v"(done + 1) : "memory");
                done++;
                LX_WP(asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(&sh.p_done)), "v"(done) : "memory");)
            } else if (!progressed) {
                LX_WP(l_sleep++;)
                __builtin_amdgcn_s_sleep(1);
            }
        }
#ifdef LX_WALKER_PROF
        if (a.prof && lane == 0) {
            unsigned long long *pw = a.prof + ((uint64_t)blockIdx.x * kProfWaves + wave) * kProfSlots;
            atomicAdd(pw + 0, (unsigned long long)l_iter);
            atomicAdd(pw + 1, (unsigned long long)l_slot);
            atomicAdd(pw + 2, (unsigned long long)l_sleep);
            atomicAdd(pw + 3, (unsigned long long)nrounds);
            atomicMax(pw + 9, wall_clock64() - lt0);
            atomicAdd(pw + 10, 1ull);   // role: loader
        }
#endif
        return;
    }

    if (wave > NCW) {
        // ------------------------------------------------------------ drain
        const uint32_t d = wave - NCW - 1;
        uint32_t nd = 0;                 // rounds of this wave completed
        const uint32_t *sj = sjs;        // segment walk: J_k of the slice's columns (LDS)
#ifdef LX_WALKER_PROF
        uint32_t d_spin = 0, d_fill = 0, d_miss = 0;
        const unsigned long long dt0 = wall_clock64();
        unsigned long long d_busy = 0;
#endif
        for (uint32_t R = d; R * 64 < n; R += ND, nd++) {
            const uint32_t ev = R * 64 + lane;
            const uint32_t sl = ev % RN;
            Slot<CPW> me;
            me.t0 = me.t1 = 0;
            // packed 8- / 12-column slots: the spin keeps the raw units and
            // unpacks once after it (12 VALU per spin otherwise)
            u4v mx = {0, 0, 0, 0}, my = {0, 0, 0, 0};
            // wait for the round (keep publishing progress: others may wait on it)
            while (true) {
                bool ready = true;
                if (ev < n) {
                    if constexpr (PK && CPW >= 8) {
                        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                                     : "=&v"(mx), "=&v"(my)
                                     : "v"(RA + sl * 16u), "v"(RB + sl * 16u)
                                     : "memory");
                        ready = mx.x == ev + 1 && my.x == ev + 1;
                    } else {
                        ring_read1<CPW, PK>(RA, RB, sl, me);
                        ready = me.t0 == ev + 1 && me.t1 == ev + 1;
                    }
                }
                if (__all(ready)) break;
                LX_WP(d_spin++;)
                if (__hip_atomic_load(&sh.req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0) __hip_atomic_store(&sh.stored[d], nd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if constexpr (PK && CPW >= 8) {
                me.t0 = mx.x; me.t1 = my.x;
                const uint32_t w6[6] = {mx.y, mx.z, mx.w, my.y, my.z, my.w};
#pragma unroll
                for (int k = 0; k < CPW; k++) me.v[k] = (k & 1) ? w6[(k / 2) % 6] >> 16 : w6[(k / 2) % 6] & 0xFFFFu;
            }
#ifdef LX_WALKER_PROF
            const unsigned long long tb0 = wall_clock64();
#endif
            uint32_t h0[CPW];
            uint32_t prev = LX_NONE, br = 0, seq = 0;
            if (ev < n) {
                const uint4 q0 = rrec[rec_off<RQ>(ev % RR, 0)];
                if constexpr (CR) {
                    br = q0.x & 0xFFFFu; seq = q0.x >> 16;
                    if (q0.y != kCrecWide) {
                        prev = (q0.y >> 8) ? bs + ev - (q0.y >> 8) : LX_NONE;
                    } else {   // rare: the full record (its load waits for this wave's stores)
                        prev = ld_l2_now(reinterpret_cast<const uint32_t *>(
                                             reinterpret_cast<const uint4 *>(a.rec) + (uint64_t)(ev / 64) * 64 * LX_REC_Q + ev % 64) + 3);
                    }
                } else {
                    br = q0.x; seq = q0.y; prev = q0.w;
                }
#pragma unroll
                for (int k = 0; k < CPW; k++) h0[k] = 0;
                if (prev != LX_NONE) {
                    const uint32_t pl = prev - bs;
                    bool got = false;
                    if (pl < n) {
                        Slot<CPW> ps;
                        ring_read1<CPW, PK>(RA, RB, pl % RN, ps);
                        if (ps.t0 == pl + 1 && ps.t1 == pl + 1) {
#pragma unroll
                            for (int k = 0; k < CPW; k++) h0[k] = ps.v[k];
                            got = true;
                        } else {
                            // reused slot: prev's row is (being) stored by a drain
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            if ((pl / 64) % ND != d) {
                                // the other drain may in turn wait for this one: keep
                                // publishing our completed rounds (divergent: every active lane)
                                __hip_atomic_store(&sh.stored[d], nd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                                while (!round_done<ND>(sh.stored, pl)) {
                                    __hip_atomic_store(&sh.req, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    __builtin_amdgcn_s_sleep(1);
                                }
                            }
                        }
                    }
                    if (!got && !(a.seg && pl >= n)) {   // (segment walk: a prev before the segment counts below as J_k)
                        const uint32_t *row = a.hb + (uint64_t)prev * stride;
#pragma unroll
                        for (int k = 0; k < CPW; k++) h0[k] = valid(k) ? ld_l2_now(row + pc(k)) : 0u;
                    }
#pragma unroll
                    for (int k = 0; k < CPW; k++) h0[k] &= mask;
                }
            }
            // ring and record data of this round consumed: slots may be reused
            if (lane == 0) __hip_atomic_store(&sh.copied[d], nd + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef LX_PROBE_SKEW
            // probe build: when each 32nd round was drained, per workgroup (lx_probe_skew_read)
            if (lane == 0 && R % 32 == 0 && R / 32 < kProbeSkewSlots && blockIdx.x < 1024)
                g_probe_skew[blockIdx.x * kProbeSkewSlots + R / 32] = wall_clock64();
#endif
            if (ev < n) {
                const uint32_t *r = me.v;
                if (a.seg) {
                    // segment walk: an event whose row misses the last pre-segment
                    // event of some branch is "partial" (lx_segment.hip fixes it up)
                    bool unc = false;
#pragma unroll
                    for (int k = 0; k < CPW; k++) unc |= (ID || valid(k)) && (r[k] & mask) < sj[k];
                    if (unc && atomicOr(a.seg_flag + ev, 1u) == 0u) a.seg_list[atomicAdd(a.seg_count, 1u)] = bs + ev;
                }
                // HB row (raw values incl. fork bits as published)
                uint32_t *hrow = a.hb + (uint64_t)(bs + ev) * stride;
#ifdef LX_PROBE_NOHB
                (void)hrow;    // probe build: HB row stores compiled out (timing / write counters only)
                if (false) {
#else
                if (contig) {
#endif
                    if (CPW == 1) hrow[pc(0)] = r[0];
                    else if (CPW == 2) *reinterpret_cast<uint2 *>(hrow + pc(0)) = make_uint2(r[0], r[1 % CPW]);
                    else if (CPW == 4) *reinterpret_cast<uint4 *>(hrow + pc(0)) = make_uint4(r[0], r[1 % CPW], r[2 % CPW], r[3 % CPW]);
                    else {
#pragma unroll
                        for (int q = 0; q < CPW / 4; q++) {
#if defined(LX_PROBE_HBNT) || defined(LX_PROBE_NT)   // probe: nontemporal HB stores
                            __builtin_nontemporal_store(
                                u4v{r[(4 * q) % CPW], r[(4 * q + 1) % CPW], r[(4 * q + 2) % CPW], r[(4 * q + 3) % CPW]},
                                reinterpret_cast<u4v *>(hrow + pc(0) + 4 * q));
#else
                            *reinterpret_cast<uint4 *>(hrow + pc(0) + 4 * q) =
                                make_uint4(r[(4 * q) % CPW], r[(4 * q + 1) % CPW], r[(4 * q + 2) % CPW], r[(4 * q + 3) % CPW]);
#endif
                        }
                    }
                } else {
#ifndef LX_PROBE_NOHB
#pragma unroll
                    for (int k = 0; k < CPW; k++)
                        if (valid(k)) hrow[pc(k)] = r[k];
#endif
                }
                {
                    // LowestAfter range fill: events (col, s), s in (h0, r], are first
                    // observed from branch `br` by this event.
                    uint32_t lo[CPW], hi[CPW];
#pragma unroll
                    for (int k = 0; k < CPW; k++) {
                        // segment walk: the rows after J_k only; L is RAW there for this
                        // event and its prev (lx_segment.hip), the rows up to J_k are
                        // filled by k_seg_la_edge
                        lo[k] = max(h0[k] + 1u, slof[k]);
                        // (12-column slices: a column past the epoch's holds 0 in
                        // every slot -- its col never equals a branch -- so it
                        // fills nothing without a check)
                        hi[k] = (ID || valid(k)) ? (r[k] & mask) : 0u;
                    }
                    if (!ID && a.lap) {
                        // sharded: rows of own branches addressed by (column, seq)
#pragma unroll
                        for (int k = 0; k < CPW; k++)
                            for (uint32_t s = lo[k]; s <= hi[k]; s++)
                                a.lap[((uint64_t)pc(k) * a.s_cap + (s - first(k))) * a.lap_stride + br] = seq;
                    } else {
                        char *const la_br = reinterpret_cast<char *>(a.la + br);
                        const uint32_t pitch = (uint32_t)stride * 4u;
                        // the first (usually only) seq of every column's range: all
                        // the recent-event lookups in one LDS round trip
                        uint64_t c0[CPW];
#pragma unroll
                        for (int k = 0; k < CPW; k++)
                            c0[k] = __hip_atomic_load(reinterpret_cast<const uint64_t *>(brc + k * KB + lo[k] % KB),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
                        for (int k = 0; k < CPW; k++) {
                            for (uint32_t s = lo[k]; s <= hi[k]; s++) {
                                const uint64_t cc = s == lo[k] ? c0[k]
                                                               : __hip_atomic_load(reinterpret_cast<const uint64_t *>(brc + k * KB + s % KB),
                                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                uint32_t row = (uint32_t)(cc >> 32);
                                LX_WP(d_fill++;)
                                LX_WP(if ((uint32_t)cc != s) d_miss++;)
                                if ((uint32_t)cc != s) row = ld_l2_now(a.brow + (uint64_t)col(k) * a.s_cap + (s - first(k)));
                                // one 32 x 32 + 64 multiply-add per store: column br of
                                // the LA plane as the base, the row pitch in bytes
                                // (< 4 GB, launch_index) as a 32-bit factor
#if defined(LX_PROBE_LANT) || defined(LX_PROBE_NT)   // probe: nontemporal LA stores
                                __builtin_nontemporal_store(seq, reinterpret_cast<uint32_t *>(la_br + (uint64_t)row * pitch));
#elif defined(LX_PROBE_LASC1)   // probe: LA stores at agent scope (sc1)
                                __hip_atomic_store(reinterpret_cast<uint32_t *>(la_br + (uint64_t)row * pitch), seq,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#elif !defined(LX_PROBE_NOLA)   // probe build NOLA: LowestAfter range-fill stores compiled out
                                *reinterpret_cast<uint32_t *>(la_br + (uint64_t)row * pitch) = seq;
#else
                                asm volatile("" ::"v"(row), "v"(seq));
#endif
                            }
                        }
                    }
                }
            }
            if (__hip_atomic_load(&sh.req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) {
                    __hip_atomic_store(&sh.stored[d], nd + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&sh.req, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            LX_WP(d_busy += wall_clock64() - tb0;)
        }
        // every store of this wave complete; a compute lane or the other drain may wait for it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(&sh.stored[d], 0xFFFFFFFFu, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef LX_WALKER_PROF
        if (a.prof) {
            unsigned long long *pw = a.prof + ((uint64_t)blockIdx.x * kProfWaves + wave) * kProfSlots;
            atomicAdd(pw + 4, (unsigned long long)d_fill);
            atomicAdd(pw + 5, (unsigned long long)d_miss);
            if (lane == 0) {
                atomicAdd(pw + 0, (unsigned long long)d_spin);
                atomicAdd(pw + 3, (unsigned long long)nd);
                atomicAdd(pw + 6, d_busy);
                atomicMax(pw + 9, wall_clock64() - dt0);
                atomicAdd(pw + 10, 2ull);   // role: drain
            }
        }
#endif
        return;
    }

    {
        // ------------------------------------------------------------ compute (block)
        // As the quad layout, but a wave's 16 quads own 16 consecutive events
        // (a block) and the wave moves to its next block (+NCW blocks) only
        // when all 16 have published: record fetch and block advance are
        // wave-uniform branches; per pass only the publish of newly ready
        // quads is divergent.
        // (1- and 2-column slices: one slot unit of 8 / 16 B per event, lane 0
        // of the quad publishes it; 4 columns: units A and B from lanes 0, 1)
        constexpr uint32_t kLeanStuck = 64;
        constexpr uint32_t kLeanFar = 512;
        constexpr uint32_t UA = CPW == 1 ? 8u : 16u;   // bytes of unit A
        const uint32_t ANULL = RA + (uint32_t)RN * UA;
        const uint32_t j = lane & 3, quad = lane >> 2;
        const uint32_t mycol = col(j & (CPW - 1));
        const bool myvalid = j < (uint32_t)CPW && valid(j & (CPW - 1));
        // CPW 8: lane j of a quad also owns column j + 4 (recent-event entries)
        uint32_t mycol2 = 0;
        bool myvalid2 = false;
        if constexpr (CPW == 8) {
#pragma unroll
            for (int k = 4; k < CPW; k++)
                if ((uint32_t)k == j + 4) { mycol2 = col(k); myvalid2 = valid(k); }
        }
        uint32_t blk = __builtin_amdgcn_readfirstlane(wave);   // wave-uniform: scalar loop control
        bool loaded = false, done = true;
        uint32_t br = 0, seq = 0, np = 0, xi = 0;
        bool wxi = false;   // some event of the wave's block has parents beyond the inline twelve (wave-uniform)
        uint32_t wstuck = 0;   // passes since the block fetch (wave-uniform)
        // SPLIT (packed 8- / 12-column slots, two 16-B units per event): lane j
        // of a quad reads unit j & 1 of the parents (j >> 1) + 2i, i < 6, so a
        // lane folds the three data words of one unit and the quad reduces over
        // one DPP step (lanes j, j ^ 2) instead of two, with no unit selects at
        // the publish: ~45 VALU per pass instead of ~70, C3 walk 47.1 -> 43.4 ms
        // (same six 16-B LDS reads per lane); otherwise lane j reads both units
        // of parents j + 4i, i < 3
        constexpr bool SPLIT = PK && CPW >= 8;
        constexpr int NPL = SPLIT ? 6 : 3;   // parent slots per lane
        const uint32_t uoff = (SPLIT && (j & 1)) ? (uint32_t)(RN + 1) * 16u : 0u;   // unit B array
        const uint32_t ANUL = ANULL + uoff;  // this lane's null unit
        auto pidx = [&](int i) -> uint32_t { return SPLIT ? (j >> 1) + 2u * i : j + 4u * i; };
        uint32_t px[NPL], pa[NPL];
#pragma unroll
        for (int i = 0; i < NPL; i++) { px[i] = kNullTag; pa[i] = ANUL; }
        uint32_t r[CPW];
#pragma unroll
        for (int k = 0; k < CPW; k++) r[k] = 0;
        // PK: r packed two columns per dword, refreshed wherever r changes
        // (block fetch, extra parents, the L2 path) instead of every pass;
        // SPLIT keeps only the lane's unit (rpk[0..2])
        constexpr int NH = CPW / 2 > 0 ? CPW / 2 : 1;
        uint32_t rpk[NH];
        // FASTR (12-column slices, SPLIT): r is never materialised -- the own
        // seq and the rare row contributions go straight into the lane's
        // packed unit (rpk[0..2]), which saves the block fetch ~60 VALU
        // (12 compares and selects for r, the repack, the recent-entry select)
        constexpr bool FASTR = SPLIT && ID;
        auto addcol = [&](int c, uint32_t v) {
            if constexpr (FASTR) {
                // column c: unit c / 6, word (c % 6) / 2, half c & 1 (v <= 0xFFFF)
                const uint32_t wv = (c & 1) ? v << 16 : v;
                rpk[((c % 6) / 2) % NH] = (uint32_t)(c / 6) == (j & 1) ? pk_max(rpk[((c % 6) / 2) % NH], wv) : rpk[((c % 6) / 2) % NH];
            } else {
                r[c] = max(r[c], v);
            }
        };
        auto repack = [&](bool fresh) {
            if constexpr (FASTR) {
                return;
            } else if constexpr (SPLIT) {
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    const uint32_t pA = r[(2 * d) % CPW] | (r[(2 * d + 1) % CPW] << 16);
                    const uint32_t pB = 6 + 2 * d < CPW ? r[(6 + 2 * d) % CPW] | (r[(7 + 2 * d) % CPW] << 16) : 0u;
                    const uint32_t q = (j & 1) ? pB : pA;
                    rpk[d] = fresh ? q : pk_max(rpk[d], q);
                }
            } else {
#pragma unroll
                for (int h = 0; h < NH; h++) {
                    const uint32_t q = r[(2 * h) % CPW] | (r[(2 * h + 1) % CPW] << 16);
                    rpk[h] = fresh ? q : pk_max(rpk[h], q);
                }
            }
        };
        repack(true);
        // per-event publish constants, set at the block fetch: LDS targets of
        // this lane's slot unit and recent-event entry (dummy when not its
        // role), the drain watermark that frees the event's slot and the value
        // it must exceed (wneed: rounds of that drain, 0 while the slot is fresh)
        const uint32_t dmy = lds_addr(dummy) + lane * 16u;
        uint32_t wa_pub = dmy, wb_pub = dmy + 1024u, wm_addr = lds_addr(&sh.copied[0]), wneed = 0;
        uint32_t cw = 0;   // that watermark, read with the parents every pass
#ifdef LX_WALKER_PROF
        uint32_t c_pass = 0, c_done = 0, c_slow = 0, c_wm = 0, c_norec = 0;
        unsigned long long c_dland = 0, c_diss = 0, c_dcop = 0, c_fetch = 0;   // record / drain lead over the block, in blocks
        const unsigned long long t_start = wall_clock64();
#endif
        while (blk * 16 < n) {
            LX_WP(c_pass++;)
            const uint32_t lp = blk * 16 + quad;
            const bool live = lp < n;
            if (!loaded) {
                const uint32_t slot = lp % RR;
                const uint32_t ra = lds_addr(rrec) + rec_off<RQ>(slot, 0) * 16u;
                uint32_t tg, w[NPL];
                u4v q0;
                if constexpr (CR) {
                    // compact record: c0..c3, c4..c7 (the next field, 1 KB on)
                    u4v q1;
                    asm volatile(
                        "ds_read_b32 %0, %3\n\t"
                        "ds_read_b128 %1, %4\n\t"
                        "ds_read_b128 %2, %4 offset:1024\n\t"
                        "s_waitcnt lgkmcnt(0)"
                        : "=&v"(tg), "=&v"(q0), "=&v"(q1)
                        : "v"(lds_addr(&rtag[slot / 64])), "v"(ra)
                        : "memory");
                    // this lane's parents (j >> 1) + 2i: half j >> 1 of word 2 + i
                    const uint32_t dw[6] = {q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
                    const uint32_t gl = bs + lp;
                    if (q0.y != kCrecWide) {
#pragma unroll
                        for (int i = 0; i < NPL; i++) w[i] = gl - ((dw[i % 6] >> (16 * (j >> 1))) & 0xFFFFu);
                        q0.z = q0.y & 0xFFu;   // np
                    } else if (live) {
                        // rare: parents too far back for 16 bits -- the full record
                        const uint4 *er = reinterpret_cast<const uint4 *>(a.rec) + (uint64_t)(lp / 64) * 64 * LX_REC_Q + lp % 64;
                        q0.z = ld_l2_now(reinterpret_cast<const uint32_t *>(er) + 2);
#pragma unroll
                        for (int i = 0; i < NPL; i++) {
                            const uint32_t pk = (j >> 1) + 2 * i;
                            w[i] = ld_l2_now(reinterpret_cast<const uint32_t *>(er + 64 * (1 + pk / 4)) + pk % 4);
                        }
                    }
                    {
                        const uint32_t c0 = q0.x;
                        q0.x = c0 & 0xFFFFu;   // branch
                        q0.y = c0 >> 16;       // seq
                    }
                } else if constexpr (SPLIT) {
                    // parents (j >> 1) + 2i: words j >> 1 and (j >> 1) + 2 of
                    // parent fields 1-3 (1 KB apart)
                    asm volatile(
                        "ds_read_b32 %0, %8\n\t"
                        "ds_read_b128 %1, %9\n\t"
                        "ds_read_b32 %2, %10 offset:1024\n\t"
                        "ds_read_b32 %3, %10 offset:1032\n\t"
                        "ds_read_b32 %4, %10 offset:2048\n\t"
                        "ds_read_b32 %5, %10 offset:2056\n\t"
                        "ds_read_b32 %6, %10 offset:3072\n\t"
                        "ds_read_b32 %7, %10 offset:3080\n\t"
                        "s_waitcnt lgkmcnt(0)"
                        : "=&v"(tg), "=&v"(q0), "=&v"(w[0]), "=&v"(w[1 % NPL]), "=&v"(w[2 % NPL]), "=&v"(w[3 % NPL]),
                          "=&v"(w[4 % NPL]), "=&v"(w[5 % NPL])
                        : "v"(lds_addr(&rtag[slot / 64])), "v"(ra), "v"(ra + (j >> 1) * 4u)
                        : "memory");
                } else {
                    asm volatile(
                        "ds_read_b32 %0, %5\n\t"
                        "ds_read_b128 %1, %6\n\t"
                        "ds_read_b32 %2, %7 offset:1024\n\t"
                        "ds_read_b32 %3, %7 offset:2048\n\t"
                        "ds_read_b32 %4, %7 offset:3072\n\t"
                        "s_waitcnt lgkmcnt(0)"
                        : "=&v"(tg), "=&v"(q0), "=&v"(w[0]), "=&v"(w[1 % NPL]), "=&v"(w[2 % NPL])
                        : "v"(lds_addr(&rtag[slot / 64])), "v"(ra), "v"(ra + j * 4u)
                        : "memory");
                }
                if (!__all(!live || tg == lp / 64 + 1)) {
                    LX_WP(c_norec++;)
                    continue;   // wave-uniform: the loader is behind
                }
                br = q0.x; seq = q0.y; np = live ? q0.z : 0u;
#pragma unroll
                for (int k = 0; k < NPL; k++) {
                    const uint32_t pl = w[k] - bs;
                    const bool in = pidx(k) < np;
                    px[k] = in ? pl + 1u : kNullTag;
                    pa[k] = in ? RA + uoff + (pl % RN) * UA : ANUL;
                }
                if constexpr (FASTR) {
                    // the own seq in column br - c0 (past the slice: no column)
                    const uint32_t c = br - c0;
                    const uint32_t hv = (c & 1) ? seq << 16 : seq;
#pragma unroll
                    for (int d = 0; d < 3; d++) rpk[d] = c < nval && c / 6 == (j & 1) && (c % 6) / 2 == (uint32_t)d ? hv : 0u;
                } else {
#pragma unroll
                    for (int k = 0; k < CPW; k++) r[k] = (col(k) == br) ? seq : 0u;
                }
                if (pidx(0) < np && w[0] - bs >= n) {
                    // parents from earlier batches (sorted oldest first): final rows
#pragma unroll
                    for (int k = 0; k < NPL; k++) {
                        if (pidx(k) >= np || w[k] - bs < n) continue;
                        LX_WP(c_slow++;)
                        if (a.seg) {
                            // segment walk: a boundary parent is its own entry only
                            const uint32_t pb = a.ev_branch[w[k]], ps = a.ev_seq[w[k]];
#pragma unroll
                            for (int c = 0; c < CPW; c++)
                                if (valid(c) && col(c) == pb) addcol(c, ps);
                        } else {
                            const uint32_t *row = a.hb + (uint64_t)w[k] * stride;
#pragma unroll
                            for (int c = 0; c < CPW; c++)
                                if (valid(c)) addcol(c, ld_l2_now(row + pc(c)) & mask);
                        }
                        px[k] = kNullTag;
                        pa[k] = ANUL;
                    }
                }
                xi = LX_MAXP;
                wxi = __any(np > (uint32_t)LX_MAXP);
                // a parent far enough back that its slot may already hold a newer event
                // is checked against the L2 path from the first pass on
                wstuck = __any(far_parent<NPL>(px, lp, (uint32_t)RN - kLeanFar)) ? kLeanStuck : 0u;
                {
                    const uint32_t rs = (lp % RN) * UA;
                    wa_pub = j == 0 ? RA + rs : (((CPW == 4 && !PK) || CPW >= 8) && j == 1) ? RB + (lp % RN) * 16u : dmy;
                    if constexpr (CPW == 12) {
                        // lane j of a quad owns columns j, j + 4, j + 8 (recent-event
                        // entries): the own column br - c0 when it is one of them
                        const uint32_t c = br - c0;
                        wb_pub = c < nval && (c & 3) == j ? lds_addr(brc) + (c * KB + seq % KB) * 8u : dmy + 1024u;
                    } else {
                        wb_pub = (myvalid && mycol == br) ? lds_addr(brc) + ((j & (CPW - 1)) * KB + seq % KB) * 8u
                                 : (CPW == 8 && myvalid2 && mycol2 == br) ? lds_addr(brc) + (((j + 4) & (CPW - 1)) * KB + seq % KB) * 8u
                                                                           : dmy + 1024u;
                    }
                    // the slot's previous occupant lp - RN is drained once its
                    // drain wave's `copied` count exceeds its round / ND
                    const uint32_t rr = (lp - RN) / 64;
                    wneed = lp >= (uint32_t)RN ? rr / ND + 1 : 0u;
                    wm_addr = lds_addr(&sh.copied[rr % ND]);
                }
                done = !live;
                loaded = true;
                repack(true);
#ifdef LX_WALKER_PROF
                {
                    const uint32_t pd = __hip_atomic_load(&sh.p_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    const uint32_t pi = __hip_atomic_load(&sh.p_issued, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    uint32_t cm = 0xFFFFFFFFu;
                    for (int d = 0; d < ND; d++)
                        cm = min(cm, __hip_atomic_load(&sh.copied[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) * ND + d);
                    c_dland += (long long)pd * 4 - blk;
                    c_diss += (long long)pi * 4 - blk;
                    c_dcop += (long long)blk - (long long)cm * 4;
                    c_fetch++;
                }
#endif
            }
            // fold (published quads read the null slot).  No per-parent select:
            // the quad publishes only in a pass where all twelve of its slot
            // reads carried the expected tags, so that pass's unconditional
            // max over them is the event's value; r holds only what does not
            // come from the ring (own seq, L2 rows of old / overflow parents)
            uint32_t tg[NPL][2], pv[3][CPW];
            u4v xs[SPLIT ? NPL : 1];   // SPLIT: the lane's six units
            uint32_t tx = 0;
            if constexpr (SPLIT) {
                asm volatile(
                    "ds_read_b128 %0, %7\n\t"
                    "ds_read_b128 %1, %8\n\t"
                    "ds_read_b128 %2, %9\n\t"
                    "ds_read_b128 %3, %10\n\t"
                    "ds_read_b128 %4, %11\n\t"
                    "ds_read_b128 %5, %12\n\t"
                    "ds_read_b32 %6, %13\n\t"
                    "s_waitcnt lgkmcnt(0)"
                    : "=&v"(xs[0]), "=&v"(xs[1 % NPL]), "=&v"(xs[2 % NPL]), "=&v"(xs[3 % NPL]), "=&v"(xs[4 % NPL]),
                      "=&v"(xs[5 % NPL]), "=&v"(cw)
                    : "v"(pa[0]), "v"(pa[1 % NPL]), "v"(pa[2 % NPL]), "v"(pa[3 % NPL]), "v"(pa[4 % NPL]),
                      "v"(pa[5 % NPL]), "v"(wm_addr)
                    : "memory");
#pragma unroll
                for (int k = 0; k < NPL; k++) { tg[k][0] = tg[k][1] = xs[k].x; tx |= xs[k].x ^ px[k]; }
            } else {
                blk_fold<CPW, RN, PK>(pa, wm_addr, tg, pv, cw);
                // tag mismatches OR-ed on the VALU: no compare masks and no mask
                // ANDs on the scalar unit, which the CU's waves share (C3 -1.9 %,
                // C2 -5.2 % against v_cmp + s_and)
#pragma unroll
                for (int k = 0; k < 3; k++) tx |= (tg[k][0] ^ px[k]) | ((PK && CPW == 4) || CPW < 4 ? 0u : (tg[k][1] ^ px[k]));
            }
            // the quad's readiness: its four lanes' mismatches OR-ed by DPP
            // (two VALU steps; the ballot / scalar-shift / per-lane bit test it
            // replaced cost 7 VALU and 3 SALU: C3 walk -3.4 %)
            tx |= (uint32_t)__builtin_amdgcn_mov_dpp((int)tx, kQuadSwap1, 0xF, 0xF, true);
            tx |= (uint32_t)__builtin_amdgcn_mov_dpp((int)tx, kQuadSwap2, 0xF, 0xF, true);
            const bool rdy = tx == 0u;   // all twelve slot tags of the quad as expected
            uint32_t m[CPW];
            uint32_t mp[NH];   // PK: the quad's maxima, two columns per dword
#pragma unroll
            for (int h = 0; h < NH; h++) mp[h] = 0u;
            if constexpr (SPLIT) {
                // the lane's unit over its six parents, then lanes j and j ^ 2
                // (same unit, the other parents): mp[0..2] = the event's unit
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    uint32_t v[NPL];
#pragma unroll
                    for (int k = 0; k < NPL; k++) v[k] = d == 0 ? xs[k].y : d == 1 ? xs[k].z : xs[k].w;
                    const uint32_t t = pk_max(pk_max(pk_max(rpk[d], v[0]), pk_max(v[1 % NPL], v[2 % NPL])),
                                              pk_max(pk_max(v[3 % NPL], v[4 % NPL]), v[5 % NPL]));
                    mp[d] = pk_max(t, (uint32_t)__builtin_amdgcn_mov_dpp((int)t, kQuadSwap2, 0xF, 0xF, true));
                }
            } else if constexpr (PK) {
                // two columns per dword: three packed maxima per dword, the quad
                // reduction on packed words
#pragma unroll
                for (int h = 0; h < NH; h++) {
                    const uint32_t rp = rpk[h];
                    mp[h] = quad_pk_max(pk_max(pk_max(rp, pv[0][h % CPW]), pk_max(pv[1][h % CPW], pv[2][h % CPW])));
                }
            } else {
#pragma unroll
                for (int c = 0; c < CPW; c++) {
                    uint32_t t;
                    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(t) : "v"(r[c]), "v"(pv[0][c]), "v"(pv[1][c]));
                    m[c] = quad_max(max(t, pv[2][c]));
                }
            }
            if (wxi && rdy && !done && xi < np) {   // (the scalar test first: most blocks have none)
                // parents beyond the inline twelve (rare): one per pass, the same on every lane of the quad
                const uint32_t pg = ld_l2_now(a.par_in + a.poff_in[lp] + xi);
                const uint32_t lpp = pg - bs;
                bool ok = false, old = lpp >= n;
                if (!old) {
                    Slot<CPW> ps;
                    ring_read1<CPW, PK>(RA, RB, lpp % RN, ps);
                    if (ps.t0 == lpp + 1 && ps.t1 == lpp + 1) {
#pragma unroll
                        for (int c = 0; c < CPW; c++) addcol(c, ps.v[c]);
                        ok = true;
                    } else if (max(ps.t0, ps.t1) > lpp + 1) {
                        if (round_done<ND>(sh.stored, lpp)) old = true;
                        else __hip_atomic_store(&sh.req, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (old && a.seg && lpp >= n) {
                    const uint32_t pb = a.ev_branch[pg], ps = a.ev_seq[pg];
#pragma unroll
                    for (int c = 0; c < CPW; c++)
                        if (valid(c) && col(c) == pb) addcol(c, ps);
                    ok = true;
                } else if (old) {
                    const uint32_t *row = a.hb + (uint64_t)pg * stride;
#pragma unroll
                    for (int c = 0; c < CPW; c++)
                        if (valid(c)) addcol(c, ld_l2_now(row + pc(c)) & mask);
                    ok = true;
                }
                // the same parent on every lane of the quad: m stays the quad's value
                if constexpr (PK) {
                    repack(false);
#pragma unroll
                    for (int h = 0; h < (SPLIT ? 3 : NH); h++) mp[h] = pk_max(mp[h], rpk[h]);
                } else {
#pragma unroll
                    for (int c = 0; c < CPW; c++) m[c] = max(m[c], r[c]);
                }
                if (quad_and(ok ? 1u : 0u)) xi++;
            }
            {
                // publish, branch-free: a ready quad whose slot's previous
                // occupant (lp - RN) is drained (as of this pass's watermark)
                // writes unit A from lane 0 and unit B from lane 1, and its
                // recent-event entry; every other lane writes the same
                // instructions into its own dummy slot
                const bool fin = rdy && !done && xi >= np && cw >= wneed;
                const uint32_t wa = fin ? wa_pub : dmy;
                const uint32_t wb = fin ? wb_pub : dmy + 1024u;
                u2v y;
                y.x = seq; y.y = bs + lp;
                if constexpr (CPW == 1) {
                    u2v x;
                    x.x = lp + 1; x.y = m[0];
                    asm volatile("ds_write_b64 %2, %3\n\tds_write_b64 %0, %1" : : "v"(wa), "v"(x), "v"(wb), "v"(y) : "memory");
                } else if constexpr (PK && CPW >= 8) {
                    u4v x;   // lane 0: {tag, s01, s23, s45}, lane 1: {tag, s67, 0, 0} (12: {tag, s67, s89, s1011})
                    x.x = lp + 1;
                    if constexpr (SPLIT) {
                        x.y = mp[0]; x.z = mp[1 % NH]; x.w = mp[2 % NH];
                    } else {
                        x.y = j == 0 ? mp[0] : mp[3 % NH];
                        x.z = j == 0 ? mp[1 % NH] : CPW == 12 ? mp[4 % NH] : 0u;
                        x.w = j == 0 ? mp[2 % NH] : CPW == 12 ? mp[5 % NH] : 0u;
                    }
                    asm volatile("ds_write_b64 %2, %3\n\tds_write_b128 %0, %1" : : "v"(wa), "v"(x), "v"(wb), "v"(y) : "memory");
                } else if constexpr (PK) {
                    u4v x;   // lane 0: {tag, s0 | s1 << 16, s2 | s3 << 16, 0}
                    x.x = lp + 1; x.y = mp[0]; x.z = mp[1 % NH]; x.w = 0u;
                    asm volatile("ds_write_b64 %2, %3\n\tds_write_b128 %0, %1" : : "v"(wa), "v"(x), "v"(wb), "v"(y) : "memory");
                } else {
                    u4v x;
                    x.x = lp + 1; x.y = j == 0 ? m[0] : m[3 % CPW]; x.z = j == 0 ? m[1 % CPW] : 0u;
                    x.w = (CPW == 4 && j == 0) ? m[2 % CPW] : 0u;
                    asm volatile("ds_write_b64 %2, %3\n\tds_write_b128 %0, %1" : : "v"(wa), "v"(x), "v"(wb), "v"(y) : "memory");
                }
                LX_WP(c_done += fin ? 1u : 0u;)
                LX_WP(c_wm += (rdy && !done && !fin) ? 1u : 0u;)
                done = done || fin;
                // a published quad reads the null slot from now on: one
                // address for all its lanes, a broadcast instead of twelve
                // scattered 16-B reads in the passes its wave still makes
                // (C3 walk -2 %)
#pragma unroll
                for (int k = 0; k < NPL; k++) pa[k] = done ? ANUL : pa[k];
            }
            if (++wstuck >= kLeanStuck && !rdy && !done) {
                // waiting long (the wave's block fetched >= 64 passes ago): a
                // parent's slot may have been reused by a newer event; its HB
                // row from L2 once its drain stored it
#pragma unroll
                for (int k = 0; k < NPL; k++) {
                    const uint32_t x = px[k];
                    if (x == kNullTag || (tg[k][0] == x && tg[k][1] == x) || max(tg[k][0], tg[k][1]) <= x) continue;
                    if (!round_done<ND>(sh.stored, x - 1u)) {
                        LX_WP(c_wm++;)
                        __hip_atomic_store(&sh.req, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        continue;
                    }
                    LX_WP(c_slow++;)
                    const uint32_t *row = a.hb + (uint64_t)(x - 1u + bs) * stride;
#pragma unroll
                    for (int c = 0; c < CPW; c++)
                        if (valid(c)) addcol(c, ld_l2_now(row + pc(c)) & mask);
                    px[k] = kNullTag;
                    pa[k] = ANUL;
                }
                repack(false);
            }
            if (__all(done)) {
                blk += NCW;
                loaded = false;
            }
        }
#ifdef LX_WALKER_PROF
        if (a.prof) {
            unsigned long long *pw = a.prof + ((uint64_t)blockIdx.x * kProfWaves + wave) * kProfSlots;
            const uint32_t cs[8] = {c_pass, 0u, 0u, c_done, c_slow, 0u, c_wm, c_norec};
#pragma unroll
            for (int i = 0; i < 8; i++) atomicAdd(pw + i, (unsigned long long)cs[i]);
            atomicMax(pw + 8, (unsigned long long)c_pass);
            if (lane == 0) {
                atomicMax(pw + 9, wall_clock64() - t_start);
                atomicAdd(pw + 11, c_dland);
                atomicAdd(pw + 12, c_diss);
                atomicAdd(pw + 13, c_dcop);
                atomicAdd(pw + 15, c_fetch);
            }
        }
#endif
        return;
    }
}

// Walk clock (lx_last_walk_clock): compute wave 0 of each workgroup stamps
// s_memtime (shader cycles) and s_memrealtime (100 MHz) around its walk; the
// ratio is the shader clock the walk ran at (the walk's cycle count is fixed
// by the DAG, its time is cycles / clock: DESIGN.md section 14)
struct WalkClock {
    unsigned long long c0 = 0, r0 = 0;
    __device__ __forceinline__ void start() {
        if (threadIdx.x == 0) asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0), "=s"(r0) :: "memory");
    }
    // ran = false: the workgroup had no walk (a zero record)
    __device__ __forceinline__ void stop(unsigned long long *clk, bool ran) {
        if (threadIdx.x != 0 || !clk) return;
        unsigned long long c1, r1;
        uint32_t xcc;
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1), "=s"(r1) :: "memory");
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (blockIdx.x == 0) clk[0] = gridDim.x;
        if (blockIdx.x < (uint32_t)kClkBlocks) {
            clk[1 + 3 * blockIdx.x] = ran ? c1 - c0 : 0ull;
            clk[2 + 3 * blockIdx.x] = ran ? r1 - r0 : 0ull;
            clk[3 + 3 * blockIdx.x] = xcc;
        }
    }
};

template <int CPW, int NCW, bool MASKED, bool PK, int ND = kND, bool CR = false>
__global__ __launch_bounds__(64 * (NCW + 1 + ND)) void k_index(IndexArgs a) {
    WalkClock wc;
    wc.start();
    // XCD-aware: neighbouring slices share an L2
    const uint32_t slice = (blockIdx.x % 8) * a.slices_per_xcd + blockIdx.x / 8;
    index_body<CPW, NCW, MASKED, PK, ND, CR>(a, slice);
    wc.stop(a.clk, slice < a.n_slices);
}

// 12-column slices, seg_g walks side by side: workgroup g runs on XCD g % 8
// (dispatch deals workgroups round-robin over the XCDs), which takes a
// contiguous chunk of each walk's slices in turn -- walk k gives its S % 8
// remainder slices to the XCDs (x - k * rem) mod 8 < rem, so every XCD holds
// at most ceil(seg_g * S / 8) workgroups (V = 1000: 84 slices, three walks,
// 31-32 per XCD of 32 CUs) and the rounding workgroups leave at once
__device__ __forceinline__ bool seg_chunk(uint32_t g, uint32_t G, uint32_t S, uint32_t *k, uint32_t *slice) {
    const uint32_t base = S / 8, rem = S % 8, x = g % 8;
    uint32_t p = g / 8;
    for (uint32_t kk = 0; kk < G; kk++) {
        const uint32_t sh = (kk * rem) % 8;
        const uint32_t sz = base + (((x + 8 - sh) % 8) < rem ? 1u : 0u);
        if (p < sz) {
            uint32_t start = x * base;
            for (uint32_t y = 0; y < x; y++) start += ((y + 8 - sh) % 8) < rem ? 1u : 0u;
            *k = kk;
            *slice = start + p;
            return true;
        }
        p -= sz;
    }
    return false;
}

// seg_g Add-order segments of a batch walked by one launch, side by side on
// idle CUs (a walk of few columns leaves most of them idle): workgroup
// blockIdx.x walks segment blockIdx.x / (gridDim.x / seg_g) with the
// segment's own batch window, J table and partial-event lists (lx_segment.hip)

template <int CPW, int NCW, bool MASKED, bool PK, int ND = kND, bool CR = false>
__global__ __launch_bounds__(64 * (NCW + 1 + ND)) void k_index_segs(IndexArgs a0) {
    WalkClock wc;
    wc.start();
    uint32_t k, slice;
    if constexpr (CPW == 12) {
        bool ok;
        if (a0.seg_map_n) {
            const uint32_t m = blockIdx.x < a0.seg_map_n ? a0.seg_map[blockIdx.x] : 0xFFFFu;
            ok = m != 0xFFFFu;
            k = m >> 8;
            slice = m & 0xFFu;
        } else {
            ok = seg_chunk(blockIdx.x, a0.seg_g, a0.n_slices, &k, &slice);
        }
        if (!ok) {
            wc.stop(a0.clk, false);
            return;
        }
    } else {
        const uint32_t per = gridDim.x / a0.seg_g, w = blockIdx.x % per;
        k = blockIdx.x / per;
        slice = (w % 8) * a0.slices_per_xcd + w / 8;   // XCD-aware: neighbouring slices share an L2
    }
    IndexArgs a = a0;
    const uint32_t lo = a0.seg_lo[k], off = lo - a0.batch_start;
    a.batch_start = lo;
    a.n = a0.seg_lo[k + 1] - lo;
    a.rec = a0.rec + off;
    a.crec = a0.crec ? a0.crec + off : nullptr;
    a.poff_in = a0.poff_in + off;
    a.seg_j = a0.seg_j + (uint64_t)k * a0.seg_B;
    a.seg_flag = a0.seg_flag + off;
    a.seg_list = a0.seg_list + off;
    a.seg_count = a0.seg_count + k;
#ifdef LX_PROBE_SKEW
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_probe_map[blockIdx.x] = k << 16 | slice;
#endif
    index_body<CPW, NCW, MASKED, PK, ND, CR>(a, slice);
    wc.stop(a0.clk, slice < a.n_slices);
}

template <int CPW, int NCW, int ND = kND>
static hipError_t launch_index_t(const IndexArgs &a0, hipStream_t s) {
    IndexArgs a = a0;
    a.n_slices = (a.ncols + CPW - 1) / CPW;
    a.slices_per_xcd = (a.n_slices + 7) / 8;
    const uint32_t grid = a.slices_per_xcd * 8;
    const dim3 blk(64 * (NCW + 1 + ND));
    if constexpr (CPW >= 8) {   // packed fork-free epochs only
        if (!a.pack16 || a.mask) return hipErrorInvalidValue;
        // (12 columns: at most ceil(seg_g * slices / 8) workgroups per XCD, seg_chunk)
        uint32_t sgrid = CPW == 12 ? 8 * (a.seg_g * (a.n_slices / 8) + (a.seg_g * (a.n_slices % 8) + 7) / 8)
                                   : grid * a.seg_g;
        a.seg_map_n = 0;
        if (CPW == 12 && a.seg_g && a.seg_xmap && a.n_slices <= 255) {
            // option seg_xmap: groups of 8 slices (96 columns = three 128-B HB
            // lines) stay on one XCD, so every HB line is assembled in one L2;
            // whole groups go round-robin to the least-loaded XCD, the short
            // last group of each walk after them
            std::vector<std::vector<uint16_t>> xl(8);
            auto put = [&](uint32_t k, uint32_t s0, uint32_t cnt) {
                uint32_t x = 0;
                for (uint32_t y = 1; y < 8; y++)
                    if (xl[y].size() < xl[x].size()) x = y;
                for (uint32_t s = s0; s < s0 + cnt; s++) xl[x].push_back((uint16_t)(k << 8 | s));
            };
            for (uint32_t k = 0; k < a.seg_g; k++)
                for (uint32_t s0 = 0; s0 + 8 <= a.n_slices; s0 += 8) put(k, s0, 8);
            if (a.n_slices % 8)
                for (uint32_t k = 0; k < a.seg_g; k++) put(k, a.n_slices / 8 * 8, a.n_slices % 8);
            size_t mx = 0;
            for (auto &l : xl) mx = std::max(mx, l.size());
            if (8 * mx <= 256 && 8 * mx <= sgrid + 8) {
                a.seg_map_n = (uint32_t)(8 * mx);
                for (uint32_t g = 0; g < a.seg_map_n; g++)
                    a.seg_map[g] = g / 8 < xl[g % 8].size() ? xl[g % 8][g / 8] : (uint16_t)0xFFFFu;
                sgrid = a.seg_map_n;
            }
        }
        // compact records when the batch wrote them (fork-free, 16-bit branches and seqs)
        if (a.crec && a.seg_g) hipLaunchKernelGGL((k_index_segs<CPW, NCW, false, true, ND, true>), dim3(sgrid), blk, 0, s, a);
        else if (a.crec) hipLaunchKernelGGL((k_index<CPW, NCW, false, true, ND, true>), dim3(grid), blk, 0, s, a);
        else if (a.seg_g) hipLaunchKernelGGL((k_index_segs<CPW, NCW, false, true, ND>), dim3(sgrid), blk, 0, s, a);
        else hipLaunchKernelGGL((k_index<CPW, NCW, false, true, ND>), dim3(grid), blk, 0, s, a);
        return hipGetLastError();
    } else {
    if (a.seg_g) {   // segments side by side (walk_grid-sized blocks of workgroups)
        const dim3 g(grid * a.seg_g);
        if constexpr (CPW == 4) {
            if (a.pack16) {
                if (a.mask) hipLaunchKernelGGL((k_index_segs<CPW, NCW, true, true>), g, blk, 0, s, a);
                else hipLaunchKernelGGL((k_index_segs<CPW, NCW, false, true>), g, blk, 0, s, a);
                return hipGetLastError();
            }
        }
        if (a.mask) hipLaunchKernelGGL((k_index_segs<CPW, NCW, true, false>), g, blk, 0, s, a);
        else hipLaunchKernelGGL((k_index_segs<CPW, NCW, false, false>), g, blk, 0, s, a);
        return hipGetLastError();
    }
    if constexpr (CPW == 4) {
        if (a.pack16) {   // every seq of the epoch fits 16 bits: one 16-B slot unit
            if (a.mask) hipLaunchKernelGGL((k_index<CPW, NCW, true, true>), dim3(grid), blk, 0, s, a);
            else hipLaunchKernelGGL((k_index<CPW, NCW, false, true>), dim3(grid), blk, 0, s, a);
            return hipGetLastError();
        }
    }
    if (a.mask) hipLaunchKernelGGL((k_index<CPW, NCW, true, false>), dim3(grid), blk, 0, s, a);
    else hipLaunchKernelGGL((k_index<CPW, NCW, false, false>), dim3(grid), blk, 0, s, a);
    return hipGetLastError();
    }
}

hipError_t launch_index(const IndexArgs &a, hipStream_t s) {
    if (a.n == 0 || a.ncols == 0) return hipSuccess;
    if (a.stride * 4 > 0xFFFFFFFFull) return hipErrorInvalidValue;   // the drains' 32-bit row pitch
    // columns per workgroup: the fewest that still leave at most ~256
    // workgroups (one per CU); the pass gets shorter with fewer columns per
    // slice, and the walk time is levels x pass latency whatever the number of
    // workgroups.  Compute waves: 8 on 1- / 2-column slices (11 slowed C2 by
    // 7 %), 11 on 4-column slices (16 waves with the loader and 4 drains, the
    // workgroup limit: C3 walk -1.8 % against 8).
    const uint32_t cpw = a.cpw_hint ? a.cpw_hint : (a.ncols <= 256 ? 1 : a.ncols <= 512 ? 2 : 4);
    if (cpw <= 1) return launch_index_t<1, 8>(a, s);
    if (cpw <= 2) return launch_index_t<2, 8>(a, s);
    // 8 columns: twice the drains' work per event (HB row, range fills), so
    // 7 drain waves beside 8 compute waves
    if (cpw == 8) return launch_index_t<8, 8, 7>(a, s);
    // 12 columns (V = 1000: 84 slices, three walks side by side on 256 CUs)
    if (cpw == 12) return a.cmap ? launch_index_t<8, 8, 7>(a, s) : launch_index_t<12, 8, 7>(a, s);
    return launch_index_t<4, 11>(a, s);
}

// ---------------------------------------------------------------------------- fork marks
// For creator n with >= 2 branches at Add(e) time: e observes a fork of n iff two
// observed branches of n overlap in seq.  Because HighestBefore only grows
// along the DAG and the branch set only grows over time, this is exactly the
// reference's marker after CollectFrom propagation + both fork loops
// (vecengine/index.go:165-209); see DESIGN.md section 3.
__global__ void k_marks(MarkArgs a) {
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)a.n * a.n_cheat;
    if (t >= total) return;
    uint32_t e = a.batch_start + (uint32_t)(t / a.n_cheat);
    uint32_t i = (uint32_t)(t % a.n_cheat);
    uint32_t bb = a.ev_bbefore[e];
    uint32_t bafter = bb + (a.ev_branch[e] == bb ? 1u : 0u);
    if (bafter <= a.V) return;
    const uint32_t *lst = a.cheat_br + a.cheat_off[i];
    uint32_t m = a.cheat_off[i + 1] - a.cheat_off[i];
    while (m > 0 && lst[m - 1] >= bafter) m--;
    if (m < 2) return;
    uint32_t *row = a.hb + (uint64_t)e * a.stride;
    const uint32_t *cm = a.cmap;
    bool hit = false;
    for (uint32_t x = 0; x < m && !hit; x++) {
        uint32_t bx = lst[x], sx = row[cm ? cm[bx] : bx] & LX_SEQ_MASK;
        if (!sx) continue;
        uint32_t fx = a.branch_first[bx];
        for (uint32_t y = x + 1; y < m; y++) {
            uint32_t by = lst[y], sy = row[cm ? cm[by] : by] & LX_SEQ_MASK;
            if (!sy) continue;
            uint32_t fy = a.branch_first[by];
            if (fx <= sy && fy <= sx) { hit = true; break; }
        }
    }
    if (hit)
        for (uint32_t x = 0; x < m; x++) row[cm ? cm[lst[x]] : lst[x]] |= LX_MARK;
}

hipError_t launch_marks(const MarkArgs &a, hipStream_t s) {
    uint64_t total = (uint64_t)a.n * a.n_cheat;
    if (!total) return hipSuccess;
    hipLaunchKernelGGL(k_marks, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- ForklessCause
// LPQ lanes per query stream HB(a) and LA(b) as 16-B vectors (8 B per branch of
// algorithmic traffic); branch j < V is creator j, so the per-creator dedupe of
// WeightCounter.CountByIdx (inter/pos/stake.go:47-55) is only needed for the
// fork branches of cheaters, handled after the streaming loop.
__device__ __forceinline__ uint32_t fc_term(uint32_t l, uint32_t h, uint32_t w, bool forks) {
    if (forks) h = ((int32_t)h < 0) ? 0u : h;     // marked branch never counts
    return ((l - 1u) < h) ? w : 0u;               // l != 0 && l <= h
}

// a query the handle cannot answer: a outside [ev_lo, n_events); b too,
// unless a row-segment rank received b's final LowestAfter row for this batch
// (b_stamp[b] == b_arrived).  Such queries read the row ev_lo instead (an own
// row: a row-segment rank's planes start there) and answer 0xFF
__device__ __forceinline__ bool fc_bad(const FcArgs &a, uint32_t A, uint32_t Bq) {
    const bool b_out = (Bq >= a.n_events) | (Bq < a.ev_lo);
    bool bad = (A >= a.n_events) | (A < a.ev_lo);
    if (a.b_stamp) bad |= b_out && (Bq >= a.n_all || a.b_stamp[Bq] != a.b_arrived);
    else bad |= b_out;
    return bad;
}

// LowestAfter row of b: the plane's own row, or (RS: a row-segment rank, b
// another rank's event) the row received for this batch.  A compile-time
// switch: the whole-index kernels carry none of it (an extra branch per
// query had cost k_fc<64> two VGPRs and a wave per SIMD: C3 FC 6.7 -> 9.9 ms)
template <bool RS>
__device__ __forceinline__ const uint32_t *fc_la(const FcArgs &a, uint32_t Bq) {
    if constexpr (RS)
        if (Bq < a.ev_lo || Bq >= a.n_events) return a.la_recv + (uint64_t)a.b_slot[Bq] * a.stride;
    return a.la + (uint64_t)Bq * a.stride;
}

template <int LPQ, bool FORKS, bool RS>
__global__ __launch_bounds__(256) void k_fc(FcArgs a) {
    const int lane = threadIdx.x % LPQ;
    const uint64_t qpb = 256 / LPQ;
    const uint32_t nv = a.vhi4 - a.vlo4;
    // a lane always covers the same columns (lane + t*LPQ): its weights stay in
    // registers for every query; the first kR uint4 of each row are loaded
    // unconditionally (clamped index, masked term) so all 2*kR loads are in
    // flight before the first compare
    constexpr int kR = 4;
    const uint4 *wv = reinterpret_cast<const uint4 *>(a.wpad) + a.vlo4;
    uint4 wr[kR];
#pragma unroll
    for (int t = 0; t < kR; t++) {
        const uint32_t i = lane + t * LPQ;
        wr[t] = i < nv ? wv[i] : make_uint4(0, 0, 0, 0);
    }
    for (uint64_t q = blockIdx.x * qpb + threadIdx.x / LPQ; q < a.n; q += (uint64_t)gridDim.x * qpb) {
        uint32_t A = a.qa_bcast ? a.qa_imm : a.qa[q], Bq = a.qb[q];
        const bool bad = fc_bad(a, A, Bq);
        if (bad) { A = a.ev_lo; Bq = a.ev_lo; }
        // FORKS, lane 0: the early-false inputs first (their loads overlap the rows')
        uint32_t e_bb = 0, e_cb = 0;
        if (FORKS && lane == 0) {
            e_bb = a.ev_branch[Bq];
            e_cb = a.ev_creator[Bq];
        }
        const uint4 *ha = reinterpret_cast<const uint4 *>(a.hb + (uint64_t)A * a.stride) + a.vlo4;
        const uint4 *lb = reinterpret_cast<const uint4 *>(fc_la<RS>(a, Bq)) + a.vlo4;
        uint4 h[kR], l[kR];
#pragma unroll
        for (int t = 0; t < kR; t++) {
            const uint32_t i = min((uint32_t)(lane + t * LPQ), nv ? nv - 1u : 0u);
            if (LPQ == 64) {
                // long rows (> 2 KB): stream past the caches (measured: +2-3 % at
                // V = 1000; short rows keep their L2 / MALL reuse)
                const u4v hv = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(ha + i));
                const u4v lv = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(lb + i));
                h[t] = make_uint4(hv.x, hv.y, hv.z, hv.w);
                l[t] = make_uint4(lv.x, lv.y, lv.z, lv.w);
            } else {
                h[t] = ha[i];
                l[t] = lb[i];
            }
        }
        uint32_t sum = 0;
#pragma unroll
        for (int t = 0; t < kR; t++) {   // wr[t] is zero past the row
            sum += fc_term(l[t].x, h[t].x, wr[t].x, FORKS) + fc_term(l[t].y, h[t].y, wr[t].y, FORKS) +
                   fc_term(l[t].z, h[t].z, wr[t].z, FORKS) + fc_term(l[t].w, h[t].w, wr[t].w, FORKS);
        }
        for (uint32_t i = lane + kR * LPQ; i < nv; i += LPQ) {   // rows longer than kR*LPQ uint4
            const uint4 hh = ha[i], ll = lb[i], w = wv[i];
            sum += fc_term(ll.x, hh.x, w.x, FORKS) + fc_term(ll.y, hh.y, w.y, FORKS) +
                   fc_term(ll.z, hh.z, w.z, FORKS) + fc_term(ll.w, hh.w, w.w, FORKS);
        }
        uint32_t early = 0;
        if (FORKS) {
            const uint32_t *hrow = a.hb + (uint64_t)A * a.stride;
            const uint32_t *lrow = fc_la<RS>(a, Bq);
            uint32_t hm = 0;
            if (lane == 0) {
                const uint32_t hc = a.cmap ? a.cmap[e_bb] : e_bb;   // NONE: another shard's branch
                hm = hc != LX_NONE ? hrow[hc] : 0u;
            }
            // plane columns (cheat_crl / cheat_brl): the creator's original
            // branch and its fork branches
            for (uint32_t c = lane; c < a.n_cheat; c += LPQ) {
                const uint32_t o0 = a.cheat_off[c], o1 = a.cheat_off[c + 1];
                const uint32_t n = a.cheat_crl[c];
                const uint32_t cn = fc_term(lrow[n], hrow[n], 1u, true);
                uint32_t hit = 0;
                for (uint32_t o = o0 + 1; o < o1; o++) {
                    const uint32_t j = a.cheat_brl[o];
                    hit |= fc_term(lrow[j], hrow[j], 1u, true);
                }
                if (!cn && hit) sum += a.wpad[n];
            }
            // early false (forkless_cause.go:49-54); creator(branch(b)) = creator(b)
            if (lane == 0 && e_cb >= a.own_lo && e_cb < a.own_hi && (hm & LX_MARK)) early = 1;
        }
#pragma unroll
        for (int off = LPQ / 2; off > 0; off >>= 1) sum += __shfl_xor(sum, off, LPQ);
        if (lane == 0) {
            if (a.partial) {
                a.partial[q] = sum + (early ? LX_MARK : 0u);
            } else {
                const uint8_t r = bad ? 0xFF : (uint8_t)(!early && sum >= a.quorum);
                a.out[q] = a.out_tag && !bad ? (uint8_t)(a.out_tag[q] << 1 | r) : r;
            }
            if (bad) atomicOr(&a.status[1], 1u);
        }
    }
}

// The early exit (option fc_early; fork-free rows of more than 512 columns):
// ForklessCause compares a stake-weighted count with the quorum
// (vecfc/forkless_cause.go:63-82), and branch j < V is validator j in
// pos.Validators order -- heaviest first -- so the count of the first columns
// often decides the answer: >= quorum is true whatever the rest holds, and
// count + the weight of every remaining column < quorum is false.  L lanes
// per query (L = 32: two queries per wave), in rounds of columns [0, 4L)
// (L = 32: 128 columns, 1 KB of HB(a) and LA(b)), [4L, 8L), [8L, 16L) and the
// rest, each read only when the count so far leaves the quorum open; the next
// query's first round is in flight while the current one is decided.  Same
// answers as the whole-row kernel by construction.  Counters: [0] queries
// past round 1, [1] past round 2, [2] every query of the early path, [3] past
// round 3.
template <bool RS, int L>
__global__ __launch_bounds__(256) void k_fc_early(FcArgs a) {
    const int lane = threadIdx.x % L;
    const uint64_t qpb = 256 / L;
    const uint32_t nv = a.vhi4 - a.vlo4;   // > 128 (lx_fc_args)
    const uint4 *wv = reinterpret_cast<const uint4 *>(a.wpad) + a.vlo4;
    // this lane's weights of the first 16 L columns: uint4 lane, L + lane, 2 L + lane, 3 L + lane
    uint4 wr[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t i = lane + t * L;
        wr[t] = i < nv ? wv[i] : make_uint4(0, 0, 0, 0);
    }
    auto terms = [](const u4v &l, const u4v &h, const uint4 &w) {
        return fc_term(l.x, h.x, w.x, false) + fc_term(l.y, h.y, w.y, false) + fc_term(l.z, h.z, w.z, false) +
               fc_term(l.w, h.w, w.w, false);
    };
    auto reduce = [](uint32_t v) {
#pragma unroll
        for (int off = L / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, L);
        return v;
    };
    uint32_t n1 = 0, n2 = 0, n3 = 0, ne = 0;
    const uint64_t step = (uint64_t)gridDim.x * qpb;
    uint64_t q = blockIdx.x * qpb + threadIdx.x / L;
    uint32_t A = 0, Bq = 0;
    bool bad = false;
    u4v hv = {0, 0, 0, 0}, lv = {0, 0, 0, 0};
    auto first = [&](uint64_t qq, uint32_t &A_, uint32_t &B_, bool &bad_, u4v &h_, u4v &l_) {
        A_ = a.qa_bcast ? a.qa_imm : a.qa[qq];
        B_ = a.qb[qq];
        bad_ = fc_bad(a, A_, B_);
        if (bad_) { A_ = a.ev_lo; B_ = a.ev_lo; }
        h_ = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(a.hb + (uint64_t)A_ * a.stride) + a.vlo4 + lane);
        l_ = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(fc_la<RS>(a, B_)) + a.vlo4 + lane);
    };
    if (q < a.n) first(q, A, Bq, bad, hv, lv);
    for (; q < a.n; q += step) {
        uint32_t An = 0, Bn = 0;
        bool badn = false;
        u4v hn = {0, 0, 0, 0}, ln = {0, 0, 0, 0};
        if (q + step < a.n) first(q + step, An, Bn, badn, hn, ln);
        uint32_t sum = reduce(terms(lv, hv, wr[0]));
        if (sum < a.quorum && sum + a.early_rest >= a.quorum) {
            // round 2: columns 4L-8L
            const u4v *ha = reinterpret_cast<const u4v *>(a.hb + (uint64_t)A * a.stride) + a.vlo4;
            const u4v *lb = reinterpret_cast<const u4v *>(fc_la<RS>(a, Bq)) + a.vlo4;
            uint32_t s1 = 0;
            if (lane + L < nv) s1 = terms(__builtin_nontemporal_load(lb + lane + L), __builtin_nontemporal_load(ha + lane + L), wr[1]);
            sum += reduce(s1);
            n1++;
            if (sum < a.quorum && sum + a.early_rest2 >= a.quorum) {
                // round 3: columns 8L-16L, two uint4 per lane in flight
                uint32_t s2 = 0;
                const uint32_t i2 = lane + 2 * L, i3 = lane + 3 * L;
                u4v h2 = {0, 0, 0, 0}, l2 = {0, 0, 0, 0}, h3 = {0, 0, 0, 0}, l3 = {0, 0, 0, 0};
                if (i2 < nv) { h2 = __builtin_nontemporal_load(ha + i2); l2 = __builtin_nontemporal_load(lb + i2); }
                if (i3 < nv) { h3 = __builtin_nontemporal_load(ha + i3); l3 = __builtin_nontemporal_load(lb + i3); }
                s2 = terms(l2, h2, wr[2]) + terms(l3, h3, wr[3]);
                sum += reduce(s2);
                n2++;
                if (sum < a.quorum && sum + a.early_rest3 >= a.quorum) {
                    // the rest of both rows
                    uint32_t s3 = 0;
                    for (uint32_t i = lane + 4 * L; i < nv; i += L) {
                        const u4v hh = __builtin_nontemporal_load(ha + i);
                        const u4v ll = __builtin_nontemporal_load(lb + i);
                        s3 += terms(ll, hh, wv[i]);
                    }
                    sum += reduce(s3);
                    n3++;
                }
            }
        }
        if (lane == 0) {
            const uint8_t r = bad ? 0xFF : (uint8_t)(sum >= a.quorum);
            a.out[q] = a.out_tag && !bad ? (uint8_t)(a.out_tag[q] << 1 | r) : r;
            if (bad) atomicOr(&a.status[1], 1u);
        }
        A = An; Bq = Bn; bad = badn; hv = hn; lv = ln;
        ne++;
    }
    if (a.early_full && lane == 0 && ne) {
        if (n1) atomicAdd(a.early_full, (unsigned long long)n1);
        if (n2) atomicAdd(a.early_full + 1, (unsigned long long)n2);
        atomicAdd(a.early_full + 2, (unsigned long long)ne);
        if (n3) atomicAdd(a.early_full + 3, (unsigned long long)n3);
    }
}

// Fork DAGs (few cheaters): every plane column is streamed -- originals and
// fork branches alike -- instead of re-reading the cheaters' columns with
// dependent scalar loads after the stream.  A non-cheater's original counts
// its weight directly (fk_w); a counting branch of cheater k sets bit k of the
// query's 64-bit mask (fk_c), the mask is OR-reduced over the query's lanes and
// each set bit adds cheater k's weight once: WeightCounter.CountByIdx's
// per-creator dedupe (inter/pos/stake.go:47-55) over all branches of the
// creator, vecfc/forkless_cause.go:63-78.  Marked branches count 0 (fc_term),
// the early false of forkless_cause.go:49-54 as in k_fc.
template <int LPQ, typename M, bool RS>   // M: the cheater mask, uint32_t (<= 32 cheaters) or uint64_t
__global__ __launch_bounds__(256) void k_fc_fk(FcArgs a) {
    constexpr uint32_t MB = 8 * sizeof(M);
    const int lane = threadIdx.x % LPQ;
    const uint64_t qpb = 256 / LPQ;
    const uint32_t nv = a.fk_hi4;
    constexpr int kR = 4;
    constexpr int kW = (int)MB / LPQ > 0 ? (int)MB / LPQ : 1;
    const uint4 *wv = reinterpret_cast<const uint4 *>(a.fk_w);
    const uint4 *cv = reinterpret_cast<const uint4 *>(a.fk_c);
    // per lane, its columns' weights and cheater bits stay in registers
    uint4 wr[kR];
    M cm[kR][4];
    auto cbit = [](uint32_t k) -> M { return k < MB ? ((M)1 << k) : (M)0; };
#pragma unroll
    for (int t = 0; t < kR; t++) {
        const uint32_t i = lane + t * LPQ;
        const bool in = i < nv;
        wr[t] = in ? wv[i] : make_uint4(0, 0, 0, 0);
        const uint4 c = in ? cv[i] : make_uint4(LX_NONE, LX_NONE, LX_NONE, LX_NONE);
        cm[t][0] = cbit(c.x); cm[t][1] = cbit(c.y); cm[t][2] = cbit(c.z); cm[t][3] = cbit(c.w);
    }
    // this lane's share of the cheaters' weights: cheater lane + t * LPQ
    uint32_t wch[kW];
#pragma unroll
    for (int t = 0; t < kW; t++) {
        const uint32_t k = lane + t * LPQ;
        wch[t] = k < a.n_cheat ? a.fk_wch[k] : 0u;
    }
    for (uint64_t q = blockIdx.x * qpb + threadIdx.x / LPQ; q < a.n; q += (uint64_t)gridDim.x * qpb) {
        uint32_t A = a.qa_bcast ? a.qa_imm : a.qa[q], Bq = a.qb[q];
        const bool bad = fc_bad(a, A, Bq);
        if (bad) { A = a.ev_lo; Bq = a.ev_lo; }
        uint32_t e_bb = 0, e_cb = 0;
        if (lane == 0) {
            e_bb = a.ev_branch[Bq];
            e_cb = a.ev_creator[Bq];
        }
        const uint4 *ha = reinterpret_cast<const uint4 *>(a.hb + (uint64_t)A * a.stride);
        const uint4 *lb = reinterpret_cast<const uint4 *>(fc_la<RS>(a, Bq));
        uint4 h[kR], l[kR];
#pragma unroll
        for (int t = 0; t < kR; t++) {
            const uint32_t i = min((uint32_t)(lane + t * LPQ), nv - 1u);
            if (LPQ == 64) {
                const u4v hv = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(ha + i));
                const u4v lv = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(lb + i));
                h[t] = make_uint4(hv.x, hv.y, hv.z, hv.w);
                l[t] = make_uint4(lv.x, lv.y, lv.z, lv.w);
            } else {
                h[t] = ha[i];
                l[t] = lb[i];
            }
        }
        uint32_t sum = 0;
        M m = 0;
#pragma unroll
        for (int t = 0; t < kR; t++) {   // wr[t] / cm[t] are zero past the row
            const uint32_t hh[4] = {h[t].x, h[t].y, h[t].z, h[t].w};
            const uint32_t ll[4] = {l[t].x, l[t].y, l[t].z, l[t].w};
            const uint32_t ww[4] = {wr[t].x, wr[t].y, wr[t].z, wr[t].w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const bool on = fc_term(ll[c], hh[c], 1u, true) != 0;
                sum += on ? ww[c] : 0u;
                m |= on ? cm[t][c] : (M)0;
            }
        }
        for (uint32_t i = lane + kR * LPQ; i < nv; i += LPQ) {   // rows longer than kR*LPQ uint4
            const uint4 hv = ha[i], lv = lb[i], w = wv[i], cc = cv[i];
            const uint32_t hh[4] = {hv.x, hv.y, hv.z, hv.w};
            const uint32_t ll[4] = {lv.x, lv.y, lv.z, lv.w};
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
            const uint32_t ck[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const bool on = fc_term(ll[c], hh[c], 1u, true) != 0;
                sum += on ? ww[c] : 0u;
                m |= on ? cbit(ck[c]) : (M)0;
            }
        }
        uint32_t early = 0;
        if (lane == 0) {
            const uint32_t hc = a.cmap ? a.cmap[e_bb] : e_bb;   // NONE: another shard's branch
            const uint32_t hm = hc != LX_NONE ? a.hb[(uint64_t)A * a.stride + hc] : 0u;
            if (e_cb >= a.own_lo && e_cb < a.own_hi && (hm & LX_MARK)) early = 1;
        }
        // cheaters with a counting branch: OR over the query's lanes, then each
        // lane adds the weights of its share of them
        if constexpr (MB == 64) {
            uint32_t mlo = (uint32_t)m, mhi = (uint32_t)((uint64_t)m >> 32);
#pragma unroll
            for (int off = LPQ / 2; off > 0; off >>= 1) {
                mlo |= __shfl_xor(mlo, off, LPQ);
                mhi |= __shfl_xor(mhi, off, LPQ);
            }
            m = (M)(((uint64_t)mhi << 32) | mlo);
        } else {
#pragma unroll
            for (int off = LPQ / 2; off > 0; off >>= 1) m |= (M)__shfl_xor((uint32_t)m, off, LPQ);
        }
#pragma unroll
        for (int t = 0; t < kW; t++) sum += (lane + t * LPQ < MB && ((m >> (lane + t * LPQ)) & 1u)) ? wch[t] : 0u;
#pragma unroll
        for (int off = LPQ / 2; off > 0; off >>= 1) sum += __shfl_xor(sum, off, LPQ);
        if (lane == 0) {
            if (a.partial) {
                a.partial[q] = sum + (early ? LX_MARK : 0u);
            } else {
                const uint8_t r = bad ? 0xFF : (uint8_t)(!early && sum >= a.quorum);
                a.out[q] = a.out_tag && !bad ? (uint8_t)(a.out_tag[q] << 1 | r) : r;
            }
            if (bad) atomicOr(&a.status[1], 1u);
        }
    }
}

template <int LPQ>
static hipError_t launch_fc_t(const FcArgs &a, bool forks, hipStream_t s) {
    const uint64_t qpb = 256 / LPQ;
    uint64_t blocks = (a.n + qpb - 1) / qpb;
    if (blocks > 256 * 32) blocks = 256 * 32;
    if (blocks == 0) return hipSuccess;
    const dim3 g((uint32_t)blocks), b(256);
    if (a.la_recv) {   // a row-segment rank: LowestAfter rows of other ranks in the receive area
        if (forks && a.fk_hi4 && a.n_cheat <= 32) hipLaunchKernelGGL((k_fc_fk<LPQ, uint32_t, true>), g, b, 0, s, a);
        else if (forks && a.fk_hi4) hipLaunchKernelGGL((k_fc_fk<LPQ, uint64_t, true>), g, b, 0, s, a);
        else if (forks) hipLaunchKernelGGL((k_fc<LPQ, true, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_fc<LPQ, false, true>), g, b, 0, s, a);
        return hipGetLastError();
    }
    if (forks && a.fk_hi4 && a.n_cheat <= 32) hipLaunchKernelGGL((k_fc_fk<LPQ, uint32_t, false>), g, b, 0, s, a);
    else if (forks && a.fk_hi4) hipLaunchKernelGGL((k_fc_fk<LPQ, uint64_t, false>), g, b, 0, s, a);
    else if (forks) hipLaunchKernelGGL((k_fc<LPQ, true, false>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_fc<LPQ, false, false>), g, b, 0, s, a);
    return hipGetLastError();
}

// lanes per query: ~4 uint4 per lane, so every lane has ~8 16-B loads in flight
// (HB and LA) whatever the row length -- short rows (few validators, or a
// column shard) would otherwise leave one load pair per lane and stay latency-bound
template <int L>
static hipError_t launch_fc_early_t(const FcArgs &a, hipStream_t s) {
    const uint64_t eb = std::min<uint64_t>((a.n + 256 / L - 1) / (256 / L), 256 * 32);
    if (!eb) return hipSuccess;
    if (a.la_recv) hipLaunchKernelGGL((k_fc_early<true, L>), dim3((uint32_t)eb), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_fc_early<false, L>), dim3((uint32_t)eb), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fc(const FcArgs &a, uint32_t cols, bool forks, hipStream_t s) {
    if (forks && !a.fk_hi4 && !a.n_cheat) forks = false;   // no cheater among this handle's creators
    if (a.early && !forks) return a.early_lanes == 16 ? launch_fc_early_t<16>(a, s) : launch_fc_early_t<32>(a, s);
    const uint32_t nv = forks && a.fk_hi4 ? a.fk_hi4 : a.vhi4 - a.vlo4;
    // (rows of <= 8 branches: 2 lanes, twice the queries per wave -- C1's
    // 20-B rows 0.078 -> 0.072 ms per 2^22 queries, profiles/r04/fc_small_rows_r04y.jsonl)
    if (nv <= 2) return launch_fc_t<2>(a, forks, s);
    if (nv <= 16) return launch_fc_t<4>(a, forks, s);
    if (nv <= 32) return launch_fc_t<8>(a, forks, s);
    if (nv <= 64) return launch_fc_t<16>(a, forks, s);
    if (nv <= 128) return launch_fc_t<32>(a, forks, s);
    return launch_fc_t<64>(a, forks, s);
}

__global__ void k_fc_combine(const uint32_t *sum, uint8_t *out, uint64_t n, uint32_t quorum) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint8_t)(sum[i] < LX_MARK && sum[i] >= quorum);
}

hipError_t launch_fc_combine(const uint32_t *sum, uint8_t *out, uint64_t n, uint32_t quorum, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_fc_combine, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, sum, out, n, quorum);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- column-shard early exit
//  Shard 0 holds the heaviest creators (pos.Validators idx
// order, vecfc/forkless_cause.go:63-82 sums stake in that order): from its own
// partial p it decides a query when p >= quorum (true whatever the other
// shards add) or p + rest < quorum (false whatever they add), rest = the stake
// of every other shard -- on fork-free epochs, where no shard's partial
// exceeds its creators' stake and none carries a mark bit.  One bit per query
// in 64-query words: dec (decided), ans (the answer of a decided query).
__global__ __launch_bounds__(256) void k_fcs_decide(const uint32_t *part, uint64_t n, uint32_t quorum, uint32_t rest,
                                                    unsigned long long *dec, unsigned long long *ans) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p = i < n ? part[i] : 0u;
    const bool t = i < n && p >= quorum;
    const bool d = t || (i < n && (uint64_t)p + rest < quorum);
    const unsigned long long bd = __ballot(d), bt = __ballot(t);
    if ((threadIdx.x & 63) == 0 && i < n) {
        dec[i / 64] = bd;
        ans[i / 64] = bt;
    }
}

hipError_t launch_fcs_decide(const uint32_t *part, uint64_t n, uint32_t quorum, uint32_t rest, unsigned long long *dec,
                             unsigned long long *ans, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_fcs_decide, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, part, n, quorum, rest, dec, ans);
    return hipGetLastError();
}

__global__ void k_fcs_flags(const unsigned long long *dec, uint64_t n, uint32_t *flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = ((dec[i / 64] >> (i % 64)) & 1ull) ? 0u : 1u;
}

// the undecided queries in query order (every rank compacts the same bits the
// same way: the all-reduce adds matching partials), shard 0's partials with them
__global__ void k_fcs_gather(const uint32_t *flag, const uint32_t *pos, uint64_t n, const uint32_t *a, const uint32_t *b,
                             const uint32_t *p0, uint32_t *idx, uint32_t *a2, uint32_t *b2, uint32_t *p2) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const uint32_t j = pos[i] - 1;
    idx[j] = (uint32_t)i;
    a2[j] = a[i];
    b2[j] = b[i];
    if (p0) p2[j] = p0[i];
}

hipError_t fcs_scan_bytes(uint64_t n, size_t *bytes) {
    return hipcub::DeviceScan::InclusiveSum(nullptr, *bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
}

hipError_t launch_fcs_undecided(const unsigned long long *dec, uint64_t n, const uint32_t *a, const uint32_t *b,
                                const uint32_t *p0, uint32_t *flag, uint32_t *pos, void *tmp, size_t tmp_bytes,
                                uint32_t *idx, uint32_t *a2, uint32_t *b2, uint32_t *p2, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 g((uint32_t)((n + 255) / 256));
    hipLaunchKernelGGL(k_fcs_flags, g, dim3(256), 0, s, dec, n, flag);
    size_t tb = tmp_bytes;
    hipError_t r = hipcub::DeviceScan::InclusiveSum(tmp, tb, flag, pos, (int)n, s);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL(k_fcs_gather, g, dim3(256), 0, s, flag, pos, n, a, b, p0, idx, a2, b2, p2);
    return hipGetLastError();
}

__global__ void k_fcs_answer(const unsigned long long *dec, const unsigned long long *ans, uint64_t n, uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint8_t)((dec[i / 64] & ans[i / 64]) >> (i % 64) & 1ull);
}

__global__ void k_fcs_scatter(const uint32_t *idx, uint64_t m, const uint32_t *sum, uint32_t quorum, uint8_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) out[idx[j]] = (uint8_t)(sum[j] < LX_MARK && sum[j] >= quorum);
}

hipError_t launch_fcs_answer(const unsigned long long *dec, const unsigned long long *ans, uint64_t n, uint64_t m,
                             const uint32_t *idx, const uint32_t *sum, uint32_t quorum, uint8_t *out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fcs_answer, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, dec, ans, n, out);
    if (m) hipLaunchKernelGGL(k_fcs_scatter, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s, idx, m, sum, quorum, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- rollback
// Zero exactly the LowestAfter entries the dropped events filled: the same
// ranges (h0, h1] as k_index, recomputed from the still-intact HB rows.
__device__ void unclaim_one(const UnfillArgs &a, uint32_t e);

__global__ void k_unfill(UnfillArgs a) {
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)(a.hi - a.lo) * a.B;
    if (t >= total) return;
    // claims and branch lengths of the dropped events (no other thread of this
    // launch reads what this writes)
    if (t < a.hi - a.lo) unclaim_one(a, a.lo + (uint32_t)t);
    uint32_t e = a.lo + (uint32_t)(t / a.B);
    uint32_t c = (uint32_t)(t % a.B);
    const uint32_t pcol = a.cmap ? a.cmap[c] : c;
    if (pcol == LX_NONE) return;                      // another shard's column
    uint32_t br = a.ev_branch[e];
    uint32_t sp = a.ev_sp[e];
    bool fork = (br == a.ev_bbefore[e]);
    uint32_t h1 = a.hb[(uint64_t)e * a.stride + pcol] & LX_SEQ_MASK;
    uint32_t h0 = (sp != LX_NONE && !fork) ? (a.hb[(uint64_t)sp * a.stride + pcol] & LX_SEQ_MASK) : 0u;
    uint32_t first = a.branch_first[c];
    for (uint32_t s = max(h0 + 1u, first); s <= h1; s++) {
        if (a.lap) {
            a.lap[((uint64_t)pcol * a.s_cap + (s - first)) * a.lap_stride + br] = 0;
            continue;
        }
        uint32_t row = a.brow[(uint64_t)c * a.s_cap + (s - first)];
        a.la[(uint64_t)row * a.stride + br] = 0;
    }
}

__device__ void unclaim_one(const UnfillArgs &a, uint32_t e) {
    uint32_t sp = a.ev_sp[e];
    uint32_t br = a.ev_branch[e];
    uint32_t s = a.ev_seq[e];
    a.first_child[e] = LX_NONE;
    if (sp != LX_NONE && sp < a.lo) {
        if (a.first_child[sp] != LX_NONE && a.first_child[sp] >= a.lo) a.first_child[sp] = LX_NONE;
    }
    if (sp == LX_NONE) {
        uint32_t c = a.ev_creator[e];
        if (a.first_root[c] != LX_NONE && a.first_root[c] >= a.lo) a.first_root[c] = LX_NONE;
    }
    if (br < a.B_keep) atomicMin(&a.branch_len[br], s - a.branch_first[br]);
}

// the dropped rows [lo, hi) of both planes, zeroed after k_unfill has read them
__global__ void k_zero_rows(uint4 *hb, uint4 *la, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        hb[i] = make_uint4(0, 0, 0, 0);
        la[i] = make_uint4(0, 0, 0, 0);
    }
}

hipError_t launch_unfill(const UnfillArgs &a, hipStream_t s) {
    if (a.hi <= a.lo) return hipSuccess;
    uint64_t total = (uint64_t)(a.hi - a.lo) * a.B;
    hipLaunchKernelGGL(k_unfill, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_zero_rows(uint32_t *hb, uint32_t *la, uint64_t stride, uint32_t lo, uint32_t hi, hipStream_t s) {
    if (hi <= lo) return hipSuccess;
    const uint64_t n16 = (uint64_t)(hi - lo) * stride / 4;   // stride: a multiple of 16 words
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_zero_rows, dim3(grid), dim3(256), 0, s, reinterpret_cast<uint4 *>(hb + (uint64_t)lo * stride),
                       reinterpret_cast<uint4 *>(la + (uint64_t)lo * stride), n16);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- LowestAfter tail
// The range fill writes LA[(c, s)][j] for every s <= RAW(last_j)[c] (the union
// of (RAW(prev)[c], RAW(e)[c]] along branch j's chain), so instead of zeroing
// the whole plane at epoch start only the unobserved tail (RAW(last_j)[c],
// last(c)] of each (c, j) is zeroed after a batch; zw remembers how far, so a
// later batch touches only new rows.  Typical tails are a few rows per (c, j)
// (the last rounds), an idle validator j costs its column once.
__global__ void k_tail_lo(TailArgs a) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.B) return;
    const uint32_t lc = a.branch_len[c];
    const uint32_t last = lc ? a.branch_first[c] + lc - 1 : 0;
    const uint32_t f = lc ? a.branch_first[c] : 1u;
    for (uint32_t j = blockIdx.y; j < a.B; j += gridDim.y) {
        const uint32_t lj = a.branch_len[j];
        uint32_t t = 0;   // RAW(last event of j)[c]; 0 if j has no event yet
        if (lj) {
            const uint32_t e = a.brow[(uint64_t)j * a.s_cap + (lj - 1)];
            t = a.hb[(uint64_t)e * a.stride + c] & LX_SEQ_MASK;
        }
        const uint64_t o = (uint64_t)j * a.tcap + c;
        const uint32_t z = a.zw[o];
        const uint32_t lo = max(max(t, z) + 1u, f);
        a.lo[o] = lo;
        if (lc) a.zw[o] = max(z, last);
        if (lc && lo <= last) atomicMin(&a.cmin[c], lo);
    }
}

constexpr int kTailReg = 8;   // columns per thread cached in registers (B <= 2048)

__global__ __launch_bounds__(256) void k_tail_zero(TailArgs a) {
    const uint32_t c = blockIdx.x;
    const uint32_t lc = a.branch_len[c];
    const uint32_t s0 = a.cmin[c];
    if (!lc || s0 == 0xFFFFFFFFu) return;
    const uint32_t f = a.branch_first[c], last = f + lc - 1;
    uint32_t lr[kTailReg];
#pragma unroll
    for (int k = 0; k < kTailReg; k++) {
        const uint32_t j = threadIdx.x + 256u * k;
        lr[k] = j < a.B ? a.lo[(uint64_t)j * a.tcap + c] : 0xFFFFFFFFu;
    }
    for (uint32_t s = s0; s <= last; s++) {
        const uint64_t row = a.brow[(uint64_t)c * a.s_cap + (s - f)];
        uint32_t *r = a.la + row * a.stride;
#pragma unroll
        for (int k = 0; k < kTailReg; k++) {
            const uint32_t j = threadIdx.x + 256u * k;
            if (s >= lr[k]) r[j] = 0u;
        }
        for (uint32_t j = threadIdx.x + 256u * kTailReg; j < a.B; j += 256u)
            if (s >= a.lo[(uint64_t)j * a.tcap + c]) r[j] = 0u;
    }
}

hipError_t launch_la_tail(const TailArgs &a, hipStream_t s) {
    if (!a.B) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.cmin, 0xFF, (uint64_t)a.B * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_lo, dim3(nblk(a.B, 256), std::min<uint32_t>(a.B, 65535)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_tail_zero, dim3(a.B), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- column shards
// Multi-GPU column sharding: rows whose branch belongs to
// shard q carry complete LowestAfter rows only on q; shard r needs the columns
// of its own branches for every row.  pack/unpack move the (rows of q) x
// (columns of r) blocks for an all-to-all.
__global__ void k_shard_flags(const uint32_t *ev_branch, const uint32_t *branch_creator, uint32_t n,
                              uint32_t lo, uint32_t hi, uint32_t *flag) {
    uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const uint32_t c = branch_creator[ev_branch[e]];
    flag[e] = (c >= lo && c < hi) ? 1u : 0u;
}

__global__ void k_compact(const uint32_t *flag, const uint32_t *pos, uint32_t n, uint32_t *rows) {
    uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    if (flag[e]) rows[pos[e] - 1] = (uint32_t)e;
}

// buf[i][k] is LowestAfter entry cols[k] of event rows[i] (uint32, or uint16 on
// the wire when every seq of the epoch fits: LA entries are seqs or 0):
//   pack   : from the produced rows (lap) of this shard's branches
//   unpack : into the query plane (la), own columns
//   own    : lap -> la for this shard's rows x its own columns
// A block moves tiles of kXR rows x 256 columns: the tile's row offsets are
// resolved once (event -> branch -> lap row, a chain of dependent loads) into
// LDS, then every thread moves its column for all kXR rows with the loads
// independent of each other -- the per-row lookups no longer serialise the copy.
// byte wire: LA entries are 0 or seqs of a branch observing the row's event,
// typically a few seqs above the row's own seq; a block travels as one byte
// per entry when every entry of it fits (mode 3 checks), else 2 or 4 bytes
__device__ __forceinline__ bool fits8(uint32_t v, uint32_t s) {
    return v == 0u || (uint32_t)((int32_t)v - (int32_t)s + 127) < 255u;   // v - s in [-127, 127]
}

template <uint32_t kXR>
__global__ __launch_bounds__(256) void k_la_xfer(XferArgs a) {
    __shared__ uint64_t s_src[kXR], s_dst[kXR];
    __shared__ uint32_t s_seq[kXR];
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    const uint32_t j = k < a.ncols ? a.cols[k] : 0u;
    const uint32_t jl = (a.mode == 1 || a.mode == 2) && k < a.ncols ? a.cmap[j] : 0u;
    bool bad = false;
    for (uint32_t i0 = blockIdx.y * kXR; i0 < a.nrows; i0 += gridDim.y * kXR) {
        const uint32_t nr = min(kXR, a.nrows - i0);
        __syncthreads();
        if (threadIdx.x < nr) {
            const uint32_t i = i0 + threadIdx.x, e = a.rows[i];
            if (a.mode != 1) {
                const uint32_t b = a.ev_branch[e];
                s_src[threadIdx.x] = ((uint64_t)a.cmap[b] * a.s_cap + (a.ev_seq[e] - a.branch_first[b])) * a.lap_stride;
            } else {
                s_src[threadIdx.x] = (uint64_t)i * a.ncols;
            }
            s_dst[threadIdx.x] = a.mode == 0 ? (uint64_t)i * a.ncols : (uint64_t)e * a.pstride;
            s_seq[threadIdx.x] = a.ev_seq[e];
        }
        __syncthreads();
        if (k >= a.ncols) continue;
        uint32_t v[kXR];
        const uint16_t *in16 = reinterpret_cast<const uint16_t *>(a.buf);
        const uint8_t *in8 = reinterpret_cast<const uint8_t *>(a.buf);
#pragma unroll
        for (uint32_t r = 0; r < kXR; r++) {
            if (r >= nr) continue;
            if (a.mode == 1) {
                const uint64_t o = s_src[r] + k;
                if (a.wire == 1) {
                    const uint32_t c = in8[o];
                    v[r] = c ? c + s_seq[r] - 128u : 0u;
                } else {
                    v[r] = a.wire == 2 ? (uint32_t)in16[o] : a.buf[o];
                }
            } else {
                v[r] = a.lap[s_src[r] + j];
            }
        }
        if (a.mode == 3 || (a.mode == 0 && a.wire == 1)) {
#pragma unroll
            for (uint32_t r = 0; r < kXR; r++)
                if (r < nr) bad |= !fits8(v[r], s_seq[r]);
            if (a.mode == 3) continue;
        }
#pragma unroll
        for (uint32_t r = 0; r < kXR; r++) {
            if (r >= nr) continue;
            if (a.mode == 0) {
                const uint64_t o = s_dst[r] + k;
                if (a.wire == 1) reinterpret_cast<uint8_t *>(a.buf)[o] = v[r] ? (uint8_t)(v[r] - s_seq[r] + 128u) : 0u;
                else if (a.wire == 2) reinterpret_cast<uint16_t *>(a.buf)[o] = (uint16_t)v[r];
                else a.buf[o] = v[r];
            } else {
                a.la[s_dst[r] + jl] = v[r];
            }
        }
    }
    // mode 3 checks into buf[0]; a byte-wire pack reports a misfit in flag[0]
    if (__any(bad) && (threadIdx.x % 64) == 0) atomicOr(a.mode == 3 ? a.buf : a.flag, 1u);
}

template <uint32_t kXR>
static hipError_t launch_la_xfer_t(const XferArgs &a, hipStream_t s) {
    const uint32_t gx = (a.ncols + 255) / 256;
    const uint64_t tiles = (a.nrows + kXR - 1) / kXR;
    const uint32_t gy = (uint32_t)std::min<uint64_t>({tiles, std::max<uint64_t>(1, 16384 / gx), 65535});
    hipLaunchKernelGGL(k_la_xfer<kXR>, dim3(gx, gy), dim3(256), 0, s, a);
    return hipGetLastError();
}

// 16-row tiles (measured on a 1/2 shard of C3: 4 rows 7.7 ms, 8: 7.1, 16: 6.9,
// 32: 8.1, 64: 9.0 per 20-GB transfer; one row per iteration: 12.7)
hipError_t launch_la_xfer(const XferArgs &a, hipStream_t s) {
    if (!a.nrows || !a.ncols) return hipSuccess;
    return launch_la_xfer_t<16>(a, s);
}

// incremental exchange (lx_shard_dirty): for each branch j with events since
// the last exchange, its last event then p_j, and every own column c:
// dmin[c] = min(RAW(p_j)[c] + 1) (p_j none: the branch's first seq)
__global__ __launch_bounds__(256) void k_shard_dmin(const uint32_t *hb, uint64_t pstride, const uint32_t *cmap,
                                                    const uint32_t *branch_len, const uint32_t *brow, uint32_t s_cap,
                                                    const uint32_t *branch_first, const uint32_t *sx_len,
                                                    const uint32_t *cols, uint32_t ncols, uint32_t *dmin) {
    const uint32_t j = blockIdx.x;
    const uint32_t x = sx_len[j];
    if (branch_len[j] <= x) return;   // nothing new on branch j (a drop makes the exchange full instead)
    const uint32_t p0 = x ? brow[(uint64_t)j * s_cap + x - 1] : LX_NONE;
    for (uint32_t k = threadIdx.x; k < ncols; k += blockDim.x) {
        const uint32_t c = cols[k];
        const uint32_t raw = p0 != LX_NONE ? (hb[(uint64_t)p0 * pstride + cmap[c]] & ~LX_MARK) : 0u;
        atomicMin(dmin + c, max(raw + 1u, branch_first[c]));
    }
}

// the dirty rows: per listed branch {c, first index, row offset, count}
__global__ __launch_bounds__(256) void k_shard_dirty_rows(const uint32_t *brow, uint32_t s_cap, const uint32_t *meta,
                                                          uint32_t *rows) {
    const uint32_t *m = meta + 4ull * blockIdx.x;
    const uint32_t c = m[0], start = m[1], off = m[2], cnt = m[3];
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) rows[off + i] = brow[(uint64_t)c * s_cap + start + i];
}

hipError_t launch_shard_dmin(const uint32_t *hb, uint64_t pstride, const uint32_t *cmap, const uint32_t *branch_len,
                             const uint32_t *brow, uint32_t s_cap, const uint32_t *branch_first, const uint32_t *sx_len,
                             uint32_t B, const uint32_t *cols, uint32_t ncols, uint32_t *dmin, hipStream_t s) {
    if (!B || !ncols) return hipSuccess;
    hipLaunchKernelGGL(k_shard_dmin, dim3(B), dim3(256), 0, s, hb, pstride, cmap, branch_len, brow, s_cap,
                       branch_first, sx_len, cols, ncols, dmin);
    return hipGetLastError();
}

hipError_t launch_shard_dirty_rows(const uint32_t *brow, uint32_t s_cap, const uint32_t *meta, uint32_t nmeta,
                                   uint32_t *rows, hipStream_t s) {
    if (!nmeta) return hipSuccess;
    hipLaunchKernelGGL(k_shard_dirty_rows, dim3(nmeta), dim3(256), 0, s, brow, s_cap, meta, rows);
    return hipGetLastError();
}

hipError_t launch_shard_rows(const uint32_t *ev_branch, const uint32_t *branch_creator, uint32_t n, uint32_t lo,
                             uint32_t hi, uint32_t *flag, uint32_t *pos, void *scan_tmp, size_t scan_bytes,
                             uint32_t *rows, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_shard_flags, dim3(nblk(n, 256)), dim3(256), 0, s, ev_branch, branch_creator, n, lo, hi, flag);
    size_t tb = scan_bytes;
    hipError_t r = hipcub::DeviceScan::InclusiveSum(scan_tmp, tb, flag, pos, (int)n, s);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL(k_compact, dim3(nblk(n, 256)), dim3(256), 0, s, flag, pos, n, rows);
    return hipGetLastError();
}


hipError_t launch_fill_u32(uint32_t *p, uint64_t n, uint32_t v, hipStream_t s) {
    if (!n) return hipSuccess;
    return hipMemsetD32Async((hipDeviceptr_t)p, (int)v, n, s);
}

hipError_t launch_copy_rows(uint32_t *dst, uint64_t dst_stride, const uint32_t *src, uint64_t src_stride,
                            uint64_t rows, uint64_t cols, hipStream_t s) {
    if (!rows || !cols) return hipSuccess;
    return hipMemcpy2DAsync(dst, dst_stride * 4, src, src_stride * 4, cols * 4, rows, hipMemcpyDeviceToDevice, s);
}

}  // namespace lx
