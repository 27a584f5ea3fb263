// lx_dbl.hip -- HighestBefore of a batch by frontier doubling, for fork-free
// epochs with few branches (BASELINE configs[0]: 5 validators, a 5,000-level
// chain).  The column walker (k_index) needs one dependent pass per DAG level
// (~0.35 us each), so a deep, narrow epoch costs
// levels x pass whatever its size.  Here the whole batch's HB rows live in
// one workgroup's LDS and are iterated to the fixpoint of
//
//   HB[e][c] = max(HB[e][c], max_c' HB[J(e, c')][c])       (compose)
//   HB[e]    = max(HB[e], HB[earlier events of e's branch])  (chain prefix max)
//
// where J(e, c') is the in-batch event of branch c' whose seq HB[e][c'] names
// (fork-free: branch c' is one chain, seq -> event is a lookup).  Starting
// from the direct parents (in-batch parents by their (branch, seq), older ones
// by their final rows), every value is the seq of an ancestor, so HB never
// overshoots; at the fixpoint every parent's row is folded in (its branch's
// entry points at it or a later chain member, whose row dominates it by the
// prefix max), so HB equals CollectFrom's max-join (vecfc/vector_ops.go:49-79)
// over the whole ancestry.  A path of d cross-branch hops is covered after
// ~log2(d) rounds.  LowestAfter is then the range fill of k_index / k_small
// (DESIGN.md section 3): events (c, s), s in (HB(prev)[c], HB(e)[c]], are first
// observed from branch(e) by e.
#include <hip/hip_runtime.h>

#include "lx_internal.h"

namespace lx {

namespace {

constexpr uint32_t kDblThreads = 1024;
constexpr uint32_t kDblU = 4;   // events per thread in flight in the row set-up

__device__ __forceinline__ uint32_t wave_max_scan(uint32_t v, uint32_t lane) {
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v = max(v, u);
    }
    return v;
}

// field 0 of event i's record {branch, seq, parents, previous branch event}:
// records are round-blocked SoA, [i / 64][q][i % 64] (k_finalize)
__device__ __forceinline__ uint4 rec_q0(const EventRec *rec, uint32_t i) {
    return reinterpret_cast<const uint4 *>(rec)[(uint64_t)(i / 64) * 64 * LX_REC_Q + (i % 64)];
}

}  // namespace

__global__ __launch_bounds__(kDblThreads) void k_dbl(DblArgs a) {
    extern __shared__ uint32_t sm[];
    const uint32_t n = a.n, B = a.B, bs = a.bs;
    const uint64_t stride = a.stride;
    uint32_t *hbl = sm;              // n * B: the batch's HB rows
    uint32_t *s0 = hbl + n * B;      // B: first seq of the branch in the batch (~0: none)
    uint32_t *cnt = s0 + B;          // B: events of the branch in the batch
    uint32_t *start = cnt + B;       // B + 1: chain offsets into posl
    uint32_t *flag = start + B + 1;  // [0] changed in this round
    uint16_t *posl = reinterpret_cast<uint16_t *>(flag + 2);   // batch positions, chain (seq) order per branch
    const uint32_t t = threadIdx.x, lane = t % 64, wave = t / 64;

    for (uint32_t c = t; c < B; c += kDblThreads) { s0[c] = 0xFFFFFFFFu; cnt[c] = 0; }
    for (uint32_t x = t; x < n * B; x += kDblThreads) hbl[x] = 0;
    if (t == 0) flag[0] = 0;
    __syncthreads();
    for (uint32_t i = t; i < n; i += kDblThreads) {
        const uint4 q0 = rec_q0(a.rec, i);
        atomicMin(&s0[q0.x], q0.y);
        atomicAdd(&cnt[q0.x], 1u);
    }
    __syncthreads();
    if (t == 0) {
        start[0] = 0;
        for (uint32_t c = 0; c < B; c++) start[c + 1] = start[c] + cnt[c];
    }
    __syncthreads();
    // chain order, and the direct parents: in-batch ones by (branch, seq), older
    // ones by their final rows; kDblU events per thread with their loads in flight
    for (uint32_t i0 = t; i0 < n; i0 += kDblThreads * kDblU) {
        uint4 q0[kDblU];
        uint32_t p0[kDblU], p1[kDblU];
#pragma unroll
        for (uint32_t u = 0; u < kDblU; u++) {
            const uint32_t i = min(i0 + u * kDblThreads, n - 1);
            q0[u] = rec_q0(a.rec, i);
            p0[u] = a.poff[i];
            p1[u] = a.poff[i + 1];
        }
#pragma unroll
        for (uint32_t u = 0; u < kDblU; u++) {
            const uint32_t i = i0 + u * kDblThreads;
            if (i >= n) continue;
            const uint32_t at = start[q0[u].x] + (q0[u].y - s0[q0[u].x]);
            if (at < start[q0[u].x + 1]) posl[at] = (uint16_t)i;   // (always: seqs of a branch are consecutive)
            atomicMax(&hbl[i * B + q0[u].x], q0[u].y);
        }
#pragma unroll
        for (uint32_t u = 0; u < kDblU; u++) {
            const uint32_t i = i0 + u * kDblThreads;
            if (i >= n) continue;
            uint32_t *row = hbl + i * B;
            for (uint32_t k = p0[u]; k < p1[u]; k += 4) {
                uint32_t p[4], br[4], sq[4];
#pragma unroll
                for (uint32_t v = 0; v < 4; v++) p[v] = a.par[min(k + v, p1[u] - 1)];
#pragma unroll
                for (uint32_t v = 0; v < 4; v++) {
                    br[v] = p[v] >= bs ? a.ev_branch[p[v]] : 0u;
                    sq[v] = p[v] >= bs ? a.ev_seq[p[v]] : 0u;
                }
#pragma unroll
                for (uint32_t v = 0; v < 4; v++) {
                    if (k + v >= p1[u]) continue;
                    if (p[v] >= bs) {
                        atomicMax(&row[br[v]], sq[v]);
                    } else {
                        const uint32_t *g = a.hb + (uint64_t)p[v] * stride;
                        for (uint32_t c = 0; c < B; c++) atomicMax(&row[c], g[c]);
                    }
                }
            }
        }
    }
    __syncthreads();

    for (;;) {
        // compose: one thread per cell (e, c); only that thread writes the cell
        bool ch = false;
        for (uint32_t x = t; x < n * B; x += kDblThreads) {
            const uint32_t i = x / B, c = x - i * B;
            const uint32_t *row = hbl + i * B;
            uint32_t v = row[c];
            for (uint32_t c2 = 0; c2 < B; c2++) {
                const uint32_t d = row[c2] - s0[c2];
                if (d < cnt[c2]) v = max(v, hbl[(uint32_t)posl[start[c2] + d] * B + c]);
            }
            if (v != hbl[x]) { hbl[x] = v; ch = true; }
        }
        __syncthreads();
        // chain prefix max: one wave per (branch, column), 64 chain members a step
        for (uint32_t pr = wave; pr < B * B; pr += kDblThreads / 64) {
            const uint32_t c2 = pr / B, k = pr - c2 * B, m = cnt[c2], o = start[c2];
            uint32_t carry = 0;
            for (uint32_t off = 0; off < m; off += 64) {
                const uint32_t idx = off + lane;
                const uint32_t cell = idx < m ? (uint32_t)posl[o + idx] * B + k : 0u;
                const uint32_t old = idx < m ? hbl[cell] : 0u;
                const uint32_t v = max(wave_max_scan(old, lane), carry);
                if (idx < m && v != old) { hbl[cell] = v; ch = true; }
                carry = __shfl(v, 63, 64);
            }
        }
        if (ch) flag[0] = 1;
        __syncthreads();
        const bool more = flag[0] != 0;
        __syncthreads();
        if (!more) break;
        if (t == 0) flag[0] = 0;
        __syncthreads();
    }

    // HB rows out, then the LowestAfter range fill (every row final)
    for (uint32_t x = t; x < n * B; x += kDblThreads) {
        const uint32_t i = x / B, c = x - i * B;
        a.hb[(uint64_t)(bs + i) * stride + c] = hbl[x];
    }
    for (uint32_t x = t; x < n * B; x += kDblThreads) {
        const uint32_t i = x / B, c = x - i * B;
        const uint4 q0 = rec_q0(a.rec, i);   // branch, seq, parents, previous branch event
        const uint32_t prev = q0.w;
        const uint32_t h0 = prev == LX_NONE ? 0u : prev >= bs ? hbl[(prev - bs) * B + c] : a.hb[(uint64_t)prev * stride + c];
        const uint32_t first = a.branch_first[c];
        const uint32_t hi = min(hbl[x], first + a.s_cap - 1u);   // (always hbl[x]: a seq of branch c)
        for (uint32_t s = max(h0 + 1u, first); s <= hi; s++)
            a.la[(uint64_t)a.brow[(uint64_t)c * a.s_cap + (s - first)] * stride + q0.x] = q0.y;
    }
}

hipError_t launch_dbl(const DblArgs &a, hipStream_t s) {
    if (!a.n || !a.B) return hipSuccess;
    if (dbl_lds_bytes(a.n, a.B) > kDblLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_dbl, dim3(1), dim3(kDblThreads), dbl_lds_bytes(a.n, a.B), s, a);
    return hipGetLastError();
}

}  // namespace lx
