// lx_emitter.hip -- CDNA4 (gfx950) kernels of the emitter's QuorumIndexer
// (emitter/ancestor/quorum_indexer.go:20-158) on the index's HighestBefore plane.
//
//   k_qi_apply  : ProcessEvent (:86-98) -- the merged-HighestBefore seqs of an
//                 event (GetMergedHighestBefore, vecengine/index.go:235-250,
//                 mapped by seqOf :70-75) into the matrix column of its
//                 creator, or into the self-parent seqs.  The matrix is kept
//                 transposed (mt[creator][validator]) so an update is one
//                 coalesced row store.
//   k_qi_median : recacheState (:100-121) -- per validator row, the V
//                 (seq, weight) pairs sorted by seq descending (bitonic sort
//                 in LDS) and the weighted median at the quorum
//                 (utils/wmedian/median.go:11-21).  Ties in seq never change
//                 the value returned, so the unstable sort.Slice of the
//                 reference and this sort agree.
//   k_qi_metric : GetMetricOf (:123-136) for a batch of candidate events with
//                 the capped difference metric of quorum_indexer_test.go:
//                 117-131; one wave per event, 64-bit wave sum.
// Integer work, small (V x V); latency- not bandwidth-bound.
#include "lx_internal.h"

namespace lx {

constexpr uint32_t kForkSeq = 0x7FFFFFFEu;   // seqOf(fork detected) = math.MaxUint32/2 - 1

// merged HighestBefore seq of validator v in an HB row (GatherFrom,
// vecfc/vector_ops.go:81-96): marks are per creator and every mark covers the
// creator's original branch v, so "first marked branch wins" reduces to the
// mark of column v; otherwise the greatest seq over v's branches
__device__ __forceinline__ uint32_t merged_seq(const QiArgs &a, const uint32_t *row, uint32_t v) {
    const uint32_t h = row[v];
    if (!a.forks) return h;
    if (h & LX_MARK) return kForkSeq;
    const int32_t k = a.cheat_of[v];
    if (k < 0) return h;
    uint32_t m = h;
    for (uint32_t o = a.cheat_off[k]; o < a.cheat_off[k + 1]; o++) m = max(m, row[a.cheat_br[o]] & LX_SEQ_MASK);
    return m;
}

__global__ void k_gather_u32(const uint32_t *src, const uint32_t *idx, uint32_t n, uint32_t *dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

hipError_t launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint32_t n, uint32_t *dst, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather_u32, dim3((n + 255) / 256), dim3(256), 0, s, src, idx, n, dst);
    return hipGetLastError();
}

// ProcessEvent of a batch without a host round trip: only the last event of
// each creator (and the last self event) writes, so every event stamps its
// batch position into its creator's slot (gen << 32 | i, atomicMax: no reset
// between batches), then the events that won write their whole column
// (the matrix is transposed: one coalesced row) and / or the self row
__device__ __forceinline__ uint32_t qb_ev(const QiBatch &b, uint32_t i) { return b.ev ? b.ev[i] : b.iev[i]; }
__device__ __forceinline__ bool qb_self(const QiBatch &b, uint32_t i) {
    return b.ev ? b.self[i] != 0u : ((b.iself >> i) & 1u) != 0u;
}

__global__ void k_qi_mark(QiArgs a, QiBatch b) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const unsigned long long key = (unsigned long long)b.gen << 32 | i;
    atomicMax(a.lastk + a.ev_creator[qb_ev(b, i)], key);
    if (qb_self(b, i)) atomicMax(a.lastk + a.V, key);
}

__global__ __launch_bounds__(256) void k_qi_apply(QiArgs a, QiBatch b) {
    const uint32_t i = blockIdx.x;
    const uint32_t e = qb_ev(b, i);
    const unsigned long long key = (unsigned long long)b.gen << 32 | i;
    const uint32_t c = a.ev_creator[e];
    const bool col = a.lastk[c] == key;
    const bool self = qb_self(b, i) && a.lastk[a.V] == key;
    if (!col && !self) return;
    const uint32_t *row = a.hb + (uint64_t)e * a.stride;
    uint32_t *dc = a.mt + (uint64_t)c * a.V;
    for (uint32_t v = threadIdx.x; v < a.V; v += blockDim.x) {
        const uint32_t m = merged_seq(a, row, v);
        if (col) dc[v] = m;
        if (self) a.sp[v] = m;
    }
}

hipError_t launch_qi_apply(const QiArgs &a, const QiBatch &b, hipStream_t s) {
    if (!b.n) return hipSuccess;
    hipLaunchKernelGGL(k_qi_mark, dim3((b.n + 255) / 256), dim3(256), 0, s, a, b);
    hipLaunchKernelGGL(k_qi_apply, dim3(b.n), dim3(256), 0, s, a, b);
    return hipGetLastError();
}

// one workgroup per validator row v; P (power of two >= V) 64-bit keys
// seq << 32 | weight in dynamic LDS, padding keys 0 sort last
__global__ __launch_bounds__(256) void k_qi_median(QiArgs a, uint32_t P) {
    extern __shared__ unsigned long long key[];
    __shared__ uint32_t sPart[256];
    __shared__ uint32_t sFirst;
    const uint32_t v = blockIdx.x, T = blockDim.x, tid = threadIdx.x;
    for (uint32_t k = tid; k < P; k += T)
        key[k] = k < a.V ? ((unsigned long long)a.mt[(uint64_t)k * a.V + v] << 32) | a.weights[k] : 0ull;
    if (tid == 0) sFirst = 0xFFFFFFFFu;
    __syncthreads();
    // bitonic sort, descending
    for (uint32_t size = 2; size <= P; size <<= 1) {
        for (uint32_t st = size >> 1; st > 0; st >>= 1) {
            for (uint32_t i = tid; i < P / 2; i += T) {
                const uint32_t lo = 2 * i - (i & (st - 1)), hi = lo + st;
                const unsigned long long x = key[lo], y = key[hi];
                const bool desc = (lo & size) == 0;
                if (desc ? x < y : x > y) {
                    key[lo] = y;
                    key[hi] = x;
                }
            }
            __syncthreads();
        }
    }
    // first position where the running weight reaches the quorum (wmedian.Of);
    // total weight < 2^31, so uint32 sums are exact
    const uint32_t C = (P + T - 1) / T, k0 = min(P, tid * C), k1 = min(P, k0 + C);
    uint32_t part = 0;
    for (uint32_t k = k0; k < k1; k++) part += (uint32_t)key[k];
    sPart[tid] = part;
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t t = 0; t < T; t++) {
            const uint32_t x = sPart[t];
            sPart[t] = acc;
            acc += x;
        }
    }
    __syncthreads();
    uint32_t acc = sPart[tid];
    for (uint32_t k = k0; k < k1; k++) {
        acc += (uint32_t)key[k];
        if (acc >= a.quorum) {
            atomicMin(&sFirst, k);
            break;
        }
    }
    __syncthreads();
    if (tid == 0) a.median[v] = sFirst < P ? (uint32_t)(key[sFirst] >> 32) : 0u;
}

hipError_t launch_qi_median(const QiArgs &a, hipStream_t s) {
    uint32_t P = 64;
    while (P < a.V) P <<= 1;
    if ((uint64_t)P * 8 > 65536) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_qi_median, dim3(a.V), dim3(256), (size_t)P * 8, s, a, P);
    return hipGetLastError();
}

// capped difference metric (quorum_indexer_test.go:117-131), 64-bit like Metric
__device__ __forceinline__ unsigned long long cap_fn(uint32_t diff, uint32_t cap, uint32_t w) {
    return (unsigned long long)(diff > cap ? cap : diff) * w;
}

__global__ __launch_bounds__(256) void k_qi_metric(QiArgs a, const uint32_t *ev, uint32_t n, uint32_t cap,
                                                   unsigned long long *out) {
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (i >= n) return;
    const uint32_t *row = a.hb + (uint64_t)ev[i] * a.stride;
    unsigned long long m = 0;
    for (uint32_t v = lane; v < a.V; v += 64) {
        const uint32_t upd = merged_seq(a, row, v), cur = a.sp[v], med = a.median[v], w = a.weights[v];
        if (upd <= med || upd <= cur) continue;
        m += (med < cur) ? cap_fn(upd - med, cap, w) - cap_fn(cur - med, cap, w) : cap_fn(upd - med, cap, w);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t hi = __shfl_xor((uint32_t)(m >> 32), off, 64), lo = __shfl_xor((uint32_t)m, off, 64);
        m += ((unsigned long long)hi << 32) | lo;
    }
    if (lane == 0) out[i] = m;
}

hipError_t launch_qi_metric(const QiArgs &a, const uint32_t *ev, uint32_t n, uint32_t cap, unsigned long long *out,
                            hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_qi_metric, dim3((n + 3) / 4), dim3(256), 0, s, a, ev, n, cap, out);
    return hipGetLastError();
}

}  // namespace lx
