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
__global__ void k_meta(BatchArgs a, unsigned long long *err) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n) return;
    uint32_t g = a.batch_start + e;
    uint32_t s = a.seq[e];
    a.ev_creator[g] = a.creator[e];
    a.ev_seq[g] = s;
    a.first_child[g] = LX_NONE;
    atomicMax(&a.status[2], s);
}

// eventcheck invariants the index relies on (parentscheck/parents_check.go:25-63,
// basiccheck/basic_check.go:24-44) and claims of "first self-child" / "first root".
__global__ void k_validate_claim(BatchArgs a, unsigned long long *err) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
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
        for (uint32_t k = p0; k < p1; k++)
            if (a.par[k] >= g) { code = E_ORDER; break; }
        if (!code && s > 1) {
            if (p1 == p0) {
                code = E_EVENT;
            } else {
                uint32_t sp = a.par[p0];
                if (a.ev_creator[sp] != c || a.ev_seq[sp] + 1 != s) code = E_EVENT;
            }
        }
    }
    if (code) {
        atomicMin(err, ((unsigned long long)e << 8) | code);
        return;
    }
    if (s > 1) atomicMin(&a.first_child[a.par[p0]], g);
    else atomicMin(&a.first_root[c], g);
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
    hipLaunchKernelGGL(k_meta, dim3(nblk(a.n, 256)), dim3(256), 0, s, a, err);
    hipLaunchKernelGGL(k_validate_claim, dim3(nblk(a.n, 256)), dim3(256), 0, s, a, err);
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
    if (f) {
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
    a.ev_branch[g] = br;
    uint32_t first = a.branch_first[br];
    a.brow[(uint64_t)br * a.s_cap + (s - first)] = g;
    atomicMax(&a.branch_len[br], s - first + 1);
    uint32_t p0 = a.poff[e], p1 = a.poff[e + 1];
    uint32_t np = p1 - p0;
    uint32_t prev = (s > 1 && !a.isfork[e]) ? 1u : 0u;
    uint32_t w[20];
    w[0] = br;
    w[1] = s;
    w[2] = prev | (np << 8);
    w[3] = p0 + LX_MAXP;
#pragma unroll
    for (int k = 0; k < LX_MAXP; k++) w[4 + k] = (k < (int)np) ? a.par[p0 + k] : LX_NONE;
    EventRec r;
#pragma unroll
    for (int k = 0; k < 5; k++) r.q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    a.rec[e] = r;
}

hipError_t launch_batch_finish(const BatchArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_assign, dim3(nblk(a.n, 256)), dim3(256), 0, s, a);
    for (uint32_t r = 0; r < 32; r++) hipLaunchKernelGGL(k_jump, dim3(nblk(a.n, 256)), dim3(256), 0, s, a, r);
    hipLaunchKernelGGL(k_finalize, dim3(nblk(a.n, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- index walker
//
// One workgroup owns CPW columns (branches) and walks ALL events of the batch
// in Add order.  Columns are independent (max-join and LowestAfter range fill
// of column c touch only column c of HB and rows of branch c in LA), so the
// workgroups never communicate.
//
// Roles inside the workgroup (NT = 9 waves):
//  * wave 8, the loader, streams 80-B event records into an LDS record ring by
//    LDS-DMA (global_load_lds_dwordx4), RR slots, up to RR/64 rounds in flight,
//    and publishes each slot with a tag after its own vmcnt wait;
//  * waves 0-7 compute: lane (g, k) handles column k of events g, g+E, ...
//    (E = 512/CPW).  Their hot path touches only LDS and issues fire-and-forget
//    stores, so no vmcnt wait (which on gfx950 also waits for stores) sits on
//    the DAG's critical path.
// In-batch parents are read from an LDS ring of {tag,seq} granules plus the
// event index of the branch-c event holding the max (so the common LowestAfter
// fill needs no dependent global lookup); a slot overwritten by a later event
// means the parent is older than the ring and its value is read from L2 (slow
// path).  Before a lane overwrites a ring slot it waits until at most SAFE of
// its own stores are in flight, which makes the overwritten parent's HB store
// visible to that slow path.  Lanes never block inside an iteration, so
// intra-wave dependencies cannot deadlock.
constexpr int kRR = 512;     // record ring slots (8 rounds of 64)
constexpr int kBRC = 64;     // recent (seq -> event) entries per owned branch

template <int CPW, int RING, bool FILL>
__global__ __launch_bounds__(576) void k_index(IndexArgs a) {
    constexpr int NT = 576;
    constexpr int E = 512 / CPW;
    constexpr int SAFE = RING / E - 2;
    static_assert(RING % E == 0 && RING / E >= 4, "ring slot reuse must stay within one lane group");
    static_assert(SAFE <= 63, "vmcnt field");
    __shared__ uint2 ring_tv[RING * CPW];       // {tag = batch pos + 1, seq}
    __shared__ uint32_t ring_ix[RING * CPW];    // dense index of the branch event holding seq
    __shared__ uint4 rrec[kRR * 5];             // event records
    __shared__ uint32_t rtag[kRR];
    __shared__ uint2 brc[CPW * kBRC];           // {seq, event} of recent events of owned branches

    const uint32_t w = blockIdx.x;
    const uint32_t slice = (w % 8) * a.slices_per_xcd + (w / 8);   // XCD-aware: neighbouring slices share an L2
    if (slice >= a.n_slices) return;

    for (int i = threadIdx.x; i < RING * CPW; i += NT) ring_tv[i] = make_uint2(0, 0);
    for (int i = threadIdx.x; i < kRR; i += NT) rtag[i] = 0;
    for (int i = threadIdx.x; i < CPW * kBRC; i += NT) brc[i] = make_uint2(0, LX_NONE);
    __syncthreads();

    const uint32_t n = a.n;
    const uint32_t bs = a.batch_start;
    const int wave = threadIdx.x / 64;
    const int lane = threadIdx.x % 64;

    if (wave == 8) {
        // ------------------------------------------------------------ loader
        const uint32_t nrounds = (n + 63) / 64;
        constexpr uint32_t D = kRR / 64;
        uint32_t issued = 0, done = 0;
        const char *recb = reinterpret_cast<const char *>(a.rec);
        const uint64_t rec_bytes = (uint64_t)n * sizeof(EventRec);
        while (done < nrounds) {
            bool progressed = false;
            if (issued < nrounds && issued - done < D) {
                // slots of this round are free once their previous occupants
                // (events ev - kRR) are done on every column of this slice
                const uint32_t ev = issued * 64 + lane;
                bool free = true;
                if (ev < n && ev >= (uint32_t)kRR) {
                    const uint32_t q = ev - kRR;
#pragma unroll
                    for (int k = 0; k < CPW; k++) {
                        const uint32_t ci = slice * CPW + k;
                        if (ci < a.ncols && ring_tv[(q % RING) * CPW + k].x < q + 1) free = false;
                    }
                }
                if (__all(free)) {
                    const uint32_t s0 = (issued * 64) % kRR;
                    char *dst = reinterpret_cast<char *>(rrec) + (uint64_t)s0 * sizeof(EventRec);
                    const uint64_t base = (uint64_t)issued * 64 * sizeof(EventRec);
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        uint64_t off = base + (uint64_t)(i * 64 + lane) * 16;
                        if (off + 16 > rec_bytes) off = 0;   // tail of the last round: harmless filler
                        __builtin_amdgcn_global_load_lds((const void *)(recb + off), (void *)(dst + i * 1024), 16, 0, 0);
                    }
                    issued++;
                    progressed = true;
                }
            }
            if (!progressed && issued > done) {
                // wait for the oldest round: at most 5 DMAs per younger round in flight
                switch (issued - done - 1) {
                    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
                    case 1: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
                    case 2: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
                    case 3: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
                    case 4: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
                    case 5: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
                    case 6: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
                    default: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
                }
                const uint32_t ev = done * 64 + lane;
                if (ev < n) __hip_atomic_store(&rtag[ev % kRR], ev + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                done++;
            } else if (!progressed) {
                __builtin_amdgcn_s_sleep(1);
            }
        }
        return;
    }

    // ---------------------------------------------------------------- compute
    const int k = threadIdx.x % CPW;
    const uint32_t g = threadIdx.x / CPW;
    const uint32_t ci = slice * CPW + k;
    if (ci >= a.ncols) return;
    const uint32_t col = a.col_list[ci];
    const uint32_t first = a.branch_first[col];
    const uint32_t *brow_c = a.brow + (uint64_t)col * a.s_cap;
    const uint64_t stride = a.stride;
    const uint32_t mask = a.mask ? LX_SEQ_MASK : 0xFFFFFFFFu;
    uint2 *brc_k = brc + k * kBRC;

    uint32_t lp = g;
    bool have = false;
    uint32_t br = 0, seq = 0, flags = 0, ovf = 0, np = 0, xi = 0;
    uint32_t par[LX_MAXP];
    uint32_t todo = 0, r = 0, ridx = LX_NONE, v0 = 0;

    while (lp < n) {
        if (!have) {
            const uint32_t slot = lp % kRR;
            if (__hip_atomic_load(&rtag[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != lp + 1) continue;
            const uint4 *rq = rrec + slot * 5;
            const uint4 q0 = rq[0];
            br = q0.x; seq = q0.y; flags = q0.z; ovf = q0.w;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint4 q = rq[1 + j];
                par[4 * j] = q.x; par[4 * j + 1] = q.y; par[4 * j + 2] = q.z; par[4 * j + 3] = q.w;
            }
            np = flags >> 8;
            todo = (np >= LX_MAXP) ? 0xFFFFu : ((1u << np) - 1u);
            xi = LX_MAXP;
            const bool own = (col == br);
            r = own ? seq : 0u;
            ridx = own ? (bs + lp) : LX_NONE;
            v0 = 0;
            have = true;
        }
        // fast path: parents in the LDS ring
        uint32_t slow = 0;
#pragma unroll
        for (int j = 0; j < LX_MAXP; j++) {
            if (todo & (1u << j)) {
                const uint32_t p = par[j];
                const uint32_t lpp = p - bs;
                if (p >= bs) {
                    const uint32_t si = (lpp % RING) * CPW + k;
                    const uint2 t = ring_tv[si];
                    if (t.x == lpp + 1) {
                        const uint32_t v = t.y & mask;
                        const uint32_t vi = ring_ix[si];
                        if (v > r || (v == r && ridx == LX_NONE)) { r = v; ridx = vi; }
                        if (j == 0) v0 = v;
                        todo &= ~(1u << j);
                    } else if (t.x > lpp + 1) {
                        slow |= 1u << j;
                    }
                } else {
                    slow |= 1u << j;
                }
            }
        }
        if (slow) {
            // slow path: parents older than the ring (or from an earlier batch)
#pragma unroll
            for (int j = 0; j < LX_MAXP; j++) {
                if (slow & (1u << j)) {
                    const uint32_t v = ld_l2_now(a.hb + (uint64_t)par[j] * stride + col) & mask;
                    if (v > r) { r = v; ridx = LX_NONE; }
                    if (j == 0) v0 = v;
                    todo &= ~(1u << j);
                }
            }
        }
        if (todo == 0 && xi < np) {
            while (xi < np) {   // parents beyond the inline 16 (rare)
                const uint32_t p = a.par_in[ovf + (xi - LX_MAXP)];
                uint32_t v, vi = LX_NONE;
                if (p < bs) {
                    v = ld_l2(a.hb + (uint64_t)p * stride + col);
                } else {
                    const uint32_t lpp = p - bs;
                    const uint32_t si = (lpp % RING) * CPW + k;
                    const uint2 t = ring_tv[si];
                    if (t.x == lpp + 1) { v = t.y; vi = ring_ix[si]; }
                    else if (t.x > lpp + 1) v = ld_l2(a.hb + (uint64_t)p * stride + col);
                    else break;
                }
                v &= mask;
                if (v > r || (v == r && ridx == LX_NONE)) { r = v; ridx = vi; }
                xi++;
            }
        }
        if (todo == 0 && xi >= np) {
            const uint32_t e = bs + lp;
            a.hb[(uint64_t)e * stride + col] = r;
            if (col == br) brc_k[seq % kBRC] = make_uint2(seq, e);
            if (r != 0 && ridx == LX_NONE) {
                const uint2 c = brc_k[r % kBRC];
                ridx = c.y;
                if (c.x != r) ridx = ld_l2_now(brow_c + (r - first));   // slow path (never if-converted: atomic)
            }
            if (FILL) {
                // LowestAfter range fill: events (col, s), s in (h0, r], are first
                // observed from branch `br` by this event.
                const uint32_t h0 = (flags & 1u) ? v0 : 0u;
                const uint32_t lo = max(h0 + 1u, first);
                if (r >= lo) {
                    a.la[(uint64_t)ridx * stride + br] = seq;
                    for (uint32_t s = lo; s < r; s++) {
                        const uint2 c = brc_k[s % kBRC];
                        uint32_t row = c.y;
                        if (c.x != s) row = ld_l2_now(brow_c + (s - first));
                        a.la[(uint64_t)row * stride + br] = seq;
                    }
                }
            }
            // bound this lane's stores in flight so that the HB store of the
            // event whose slot is overwritten RING/E completions later is done
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SAFE) : "memory");
            const uint32_t si = (lp % RING) * CPW + k;
            ring_ix[si] = ridx;
            __hip_atomic_store(reinterpret_cast<unsigned long long *>(&ring_tv[si]),
                               ((unsigned long long)r << 32) | (lp + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            lp += E;
            have = false;
        }
    }
}

template <int CPW, int RING>
static hipError_t launch_index_t(const IndexArgs &a0, hipStream_t s) {
    IndexArgs a = a0;
    a.n_slices = (a.ncols + CPW - 1) / CPW;
    a.slices_per_xcd = (a.n_slices + 7) / 8;
    uint32_t grid = a.slices_per_xcd * 8;
    if (a.diag_nofill) hipLaunchKernelGGL((k_index<CPW, RING, false>), dim3(grid), dim3(576), 0, s, a);
    else hipLaunchKernelGGL((k_index<CPW, RING, true>), dim3(grid), dim3(576), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_index(const IndexArgs &a, hipStream_t s) {
    if (a.n == 0 || a.ncols == 0) return hipSuccess;
    // aim at >= ~256 workgroups (one per CU) while keeping per-row writes wide;
    // the ring (96 KB) must cover the typical parent distance (~V events back)
    if (a.ncols <= 256) return launch_index_t<1, 8192>(a, s);
    if (a.ncols <= 512) return launch_index_t<2, 4096>(a, s);
    if (a.ncols <= 1024) return launch_index_t<4, 2048>(a, s);
    return launch_index_t<8, 1024>(a, s);
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
    bool hit = false;
    for (uint32_t x = 0; x < m && !hit; x++) {
        uint32_t bx = lst[x], sx = row[bx] & LX_SEQ_MASK;
        if (!sx) continue;
        uint32_t fx = a.branch_first[bx];
        for (uint32_t y = x + 1; y < m; y++) {
            uint32_t by = lst[y], sy = row[by] & LX_SEQ_MASK;
            if (!sy) continue;
            uint32_t fy = a.branch_first[by];
            if (fx <= sy && fy <= sx) { hit = true; break; }
        }
    }
    if (hit)
        for (uint32_t x = 0; x < m; x++) row[lst[x]] |= LX_MARK;
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

template <int LPQ, bool FORKS>
__global__ __launch_bounds__(256) void k_fc(FcArgs a) {
    const int lane = threadIdx.x % LPQ;
    const uint64_t qpb = 256 / LPQ;
    const uint64_t nv = a.vhi4 - a.vlo4;
    for (uint64_t q = blockIdx.x * qpb + threadIdx.x / LPQ; q < a.n; q += (uint64_t)gridDim.x * qpb) {
        uint32_t A = a.qa[q], Bq = a.qb[q];
        const bool bad = (A >= a.n_events) | (Bq >= a.n_events);
        if (bad) { A = 0; Bq = 0; }
        const uint4 *ha = reinterpret_cast<const uint4 *>(a.hb + (uint64_t)A * a.stride) + a.vlo4;
        const uint4 *lb = reinterpret_cast<const uint4 *>(a.la + (uint64_t)Bq * a.stride) + a.vlo4;
        const uint4 *wv = reinterpret_cast<const uint4 *>(a.wpad) + a.vlo4;
        uint32_t sum = 0;
#pragma unroll 4
        for (uint64_t i = lane; i < nv; i += LPQ) {
            const uint4 h = ha[i], l = lb[i], w = wv[i];
            sum += fc_term(l.x, h.x, w.x, FORKS) + fc_term(l.y, h.y, w.y, FORKS) +
                   fc_term(l.z, h.z, w.z, FORKS) + fc_term(l.w, h.w, w.w, FORKS);
        }
        uint32_t early = 0;
        if (FORKS) {
            const uint32_t *hrow = a.hb + (uint64_t)A * a.stride;
            const uint32_t *lrow = a.la + (uint64_t)Bq * a.stride;
            for (uint32_t c = lane; c < a.n_cheat; c += LPQ) {
                const uint32_t o0 = a.cheat_off[c], o1 = a.cheat_off[c + 1];
                const uint32_t n = a.cheat_creator[c];
                const uint32_t cn = fc_term(lrow[n], hrow[n], 1u, true);
                uint32_t hit = 0;
                for (uint32_t o = o0 + 1; o < o1; o++) {
                    const uint32_t j = a.cheat_br[o];
                    hit |= fc_term(lrow[j], hrow[j], 1u, true);
                }
                if (!cn && hit) sum += a.wpad[n];
            }
            if (lane == 0) {
                const uint32_t bb = a.ev_branch[Bq];
                const uint32_t cb = a.branch_creator[bb];
                if (cb >= a.own_lo && cb < a.own_hi && (hrow[bb] & LX_MARK)) early = 1;
            }
        }
#pragma unroll
        for (int off = LPQ / 2; off > 0; off >>= 1) sum += __shfl_xor(sum, off, LPQ);
        if (lane == 0) {
            if (a.partial) {
                a.partial[q] = sum + (early ? LX_MARK : 0u);
            } else {
                a.out[q] = bad ? 0xFF : (uint8_t)(!early && sum >= a.quorum);
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
    if (forks) hipLaunchKernelGGL((k_fc<LPQ, true>), dim3((uint32_t)blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_fc<LPQ, false>), dim3((uint32_t)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fc(const FcArgs &a, uint32_t cols, bool forks, hipStream_t s) {
    const uint32_t nv = a.vhi4 - a.vlo4;
    if (nv <= 16) return launch_fc_t<16>(a, forks, s);
    if (nv <= 32) return launch_fc_t<32>(a, forks, s);
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

// ---------------------------------------------------------------------------- rollback
// Zero exactly the LowestAfter entries the dropped events filled: the same
// ranges (h0, h1] as k_index, recomputed from the still-intact HB rows.
__global__ void k_unfill(UnfillArgs a) {
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)(a.hi - a.lo) * a.B;
    if (t >= total) return;
    uint32_t e = a.lo + (uint32_t)(t / a.B);
    uint32_t c = (uint32_t)(t % a.B);
    uint32_t br = a.ev_branch[e];
    uint32_t sp = a.ev_sp[e];
    bool fork = (br == a.ev_bbefore[e]);
    uint32_t h1 = a.hb[(uint64_t)e * a.stride + c] & LX_SEQ_MASK;
    uint32_t h0 = (sp != LX_NONE && !fork) ? (a.hb[(uint64_t)sp * a.stride + c] & LX_SEQ_MASK) : 0u;
    uint32_t first = a.branch_first[c];
    for (uint32_t s = max(h0 + 1u, first); s <= h1; s++) {
        uint32_t row = a.brow[(uint64_t)c * a.s_cap + (s - first)];
        a.la[(uint64_t)row * a.stride + br] = 0;
    }
}

__global__ void k_unclaim(UnfillArgs a) {
    uint32_t e = a.lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.hi) return;
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

hipError_t launch_unfill(const UnfillArgs &a, hipStream_t s) {
    if (a.hi <= a.lo) return hipSuccess;
    uint64_t total = (uint64_t)(a.hi - a.lo) * a.B;
    hipLaunchKernelGGL(k_unfill, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_unclaim, dim3(nblk(a.hi - a.lo, 256)), dim3(256), 0, s, a);
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
