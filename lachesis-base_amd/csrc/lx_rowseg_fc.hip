// lx_rowseg_fc.hip -- ForklessCause of ANY pair of the epoch on row-segment
// ranks.
//
// After the row exchange rank r owns the final HighestBefore and LowestAfter
// rows of its Add-order segment [lo, hi).  ForklessCause(a, b)
// (vecfc/forkless_cause.go:40-82) reads HB(a) and LA(b), so a query is
// answered on owner(a), and when b lies in another segment LA(b) comes from
// owner(b):
//   route  -- the caller's queries sorted by owner(a) (one 1-pass radix sort
//             on the owner, permutation kept), moved by one all-to-all;
//   need   -- on owner(a), the distinct b outside its rows (deduplicated per
//             batch by a stamp per event: atomicMax to 2 gen), grouped by
//             owner(b);
//   serve / store -- their LA rows (B words each) are gathered by owner(b),
//             moved back and written into the receiving rank's receive area
//             (row i of the batch's sorted id list; b_slot[b] = i), stamp
//             2 gen + 1 -- the planes hold the own rows only;
//   then k_fc over the routed pairs: b is valid when own or stamped 2 gen + 1
//             (a final LA row received for this batch);
//   unroute -- the answers back in the caller's order.
// For the bench's query shape (b within 64 Lamport of a) only the pairs near
// a segment boundary cross: a few thousand LA rows per batch.
#include <hipcub/hipcub.hpp>

#include "lx_internal.h"

namespace lx {

namespace {

__device__ __forceinline__ uint32_t owner_of(const RsqArgs &a, uint32_t e) {
    if (e >= a.n_all) return a.self;   // unknown event: answered (and refused) locally
    uint32_t lo = 0, hi = a.G;         // seg_lo[lo] <= e < seg_lo[hi]
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) / 2;
        if (e >= a.seg_lo[m]) lo = m;
        else hi = m;
    }
    return lo;
}

// owner key per query, identity values, per-owner counts (LDS histogram, one
// global atomic per owner and workgroup)
__global__ void __launch_bounds__(256) k_rsq_keys(RsqArgs a, const uint32_t *qa, uint64_t n, uint32_t *keys,
                                                  uint32_t *vals, uint32_t *counts) {
    __shared__ uint32_t hist[kMaxSegments];
    if (threadIdx.x < a.G) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t o = owner_of(a, qa[i]);
        keys[i] = o;
        vals[i] = (uint32_t)i;
        atomicAdd(&hist[o], 1u);
    }
    __syncthreads();
    if (threadIdx.x < a.G && hist[threadIdx.x]) atomicAdd(counts + threadIdx.x, hist[threadIdx.x]);
}

__global__ void k_rsq_gather(const uint32_t *perm, const uint32_t *qa, const uint32_t *qb, uint64_t n, uint32_t *ra,
                             uint32_t *rb) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = perm[i];
    ra[i] = qa[p];
    rb[i] = qb[p];
}

// the distinct b (outside the own rows) of the routed pairs whose a is own
__global__ void k_rsq_need(RsqArgs a, const uint32_t *ra, const uint32_t *rb, uint64_t m, uint32_t *stamp,
                           uint32_t want, uint32_t *list, uint32_t *count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = ra[i], b = rb[i];
    if (x < a.lo || x >= a.hi || b >= a.n_all || (b >= a.lo && b < a.hi)) return;
    if (atomicMax(stamp + b, want) < want) list[atomicAdd(count, 1u)] = b;
}

// per-owner counts of a sorted id list
__global__ void __launch_bounds__(256) k_rsq_count(RsqArgs a, const uint32_t *ids, uint32_t n, uint32_t *counts) {
    __shared__ uint32_t hist[kMaxSegments];
    if (threadIdx.x < a.G) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&hist[owner_of(a, ids[i])], 1u);
    __syncthreads();
    if (threadIdx.x < a.G && hist[threadIdx.x]) atomicAdd(counts + threadIdx.x, hist[threadIdx.x]);
}

// serve: the own final LA rows (B words) of the asked ids; a row that is not
// own is sent as zeros (the asking rank never asks for one)
__global__ void __launch_bounds__(256) k_rsq_la_gather(RsqArgs a, const uint32_t *la, uint64_t stride,
                                                       const uint32_t *ids, uint32_t *rows) {
    const uint32_t x = ids[blockIdx.x];
    const bool own = x >= a.lo && x < a.hi;
    const uint32_t *src = la + (uint64_t)x * stride;
    uint32_t *dst = rows + (uint64_t)blockIdx.x * a.B;
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) dst[c] = own ? src[c] : 0u;
}

// store: received LA row i into row i of the receive area, then its slot and
// the arrival stamp (k_fc, a later launch, checks both)
__global__ void __launch_bounds__(256) k_rsq_la_store(RsqArgs a, uint32_t *la_recv, uint64_t stride,
                                                      const uint32_t *ids, const uint32_t *rows, uint32_t *stamp,
                                                      uint32_t *slot, uint32_t arrived) {
    const uint32_t x = ids[blockIdx.x];
    if (x >= a.n_all || (x >= a.lo && x < a.hi)) return;   // an own row is never received
    uint32_t *dst = la_recv + (uint64_t)blockIdx.x * stride;
    const uint32_t *src = rows + (uint64_t)blockIdx.x * a.B;
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) dst[c] = src[c];
    if (threadIdx.x == 0) {
        slot[x] = blockIdx.x;
        stamp[x] = arrived;
    }
}

__global__ void k_rsq_unroute(const uint32_t *perm, const uint8_t *ans, uint64_t n, uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[perm[i]] = ans[i];
}

// routed getter rows back in the caller's order: row i (slot bytes, a multiple
// of 16) to row perm[i], its length with it; one workgroup per row
__global__ void __launch_bounds__(256) k_rows_unroute(const uint32_t *perm, const uint8_t *rows, uint64_t slot,
                                                      const uint32_t *len, uint8_t *out, uint32_t *out_len) {
    const uint64_t i = blockIdx.x;
    const uint32_t p = perm[i];
    const uint4 *src = reinterpret_cast<const uint4 *>(rows + i * slot);
    uint4 *dst = reinterpret_cast<uint4 *>(out + (uint64_t)p * slot);
    for (uint64_t k = threadIdx.x; k < slot / 16; k += blockDim.x) dst[k] = src[k];
    if (threadIdx.x == 0) out_len[p] = len[i];
}

inline uint32_t nb(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

uint32_t owner_bits(uint32_t G) {
    uint32_t b = 1;
    while ((1u << b) < G) b++;
    return b;
}

}  // namespace

hipError_t rsq_tmp_bytes(uint64_t n, uint32_t G, size_t *bytes) {
    size_t b1 = 0, b2 = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b1, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                      (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, 0,
                                                      (int)owner_bits(G));
    if (e != hipSuccess) return e;
    e = hipcub::DeviceRadixSort::SortKeys(nullptr, b2, (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
    *bytes = b1 > b2 ? b1 : b2;
    return e;
}

hipError_t launch_rsq_route(const RsqArgs &a, const uint32_t *qa, const uint32_t *qb, uint64_t n, uint32_t *scratch,
                            void *tmp, size_t tmp_bytes, uint32_t *ra, uint32_t *rb, uint32_t *perm, uint32_t *counts,
                            hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(counts, 0, 4ull * a.G, s)) != hipSuccess) return e;
    if (!n) return hipSuccess;
    uint32_t *keys = scratch, *keys2 = scratch + n, *vals = scratch + 2 * n;
    hipLaunchKernelGGL(k_rsq_keys, dim3(nb(n, 256)), dim3(256), 0, s, a, qa, n, keys, vals, counts);
    if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys2, vals, perm, (int)n, 0,
                                                (int)owner_bits(a.G), s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_rsq_gather, dim3(nb(n, 256)), dim3(256), 0, s, perm, qa, qb, n, ra, rb);
    return hipGetLastError();
}

hipError_t launch_rsq_need(const RsqArgs &a, const uint32_t *ra, const uint32_t *rb, uint64_t m, uint32_t *stamp,
                           uint32_t want, uint32_t *list, uint32_t *count, hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_rsq_need, dim3(nb(m, 256)), dim3(256), 0, s, a, ra, rb, m, stamp, want, list, count);
    return hipGetLastError();
}

hipError_t launch_rsq_group(const RsqArgs &a, const uint32_t *list, uint32_t n, void *tmp, size_t tmp_bytes,
                            uint32_t *ids, uint32_t *counts, hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(counts, 0, 4ull * a.G, s)) != hipSuccess) return e;
    if (!n) return hipSuccess;
    // sorted by id = grouped by owner (segments are id ranges, in rank order)
    if ((e = hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, list, ids, (int)n, 0, 32, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_rsq_count, dim3(nb(n, 256)), dim3(256), 0, s, a, ids, n, counts);
    return hipGetLastError();
}

hipError_t launch_rsq_la_gather(const RsqArgs &a, const uint32_t *la, uint64_t stride, const uint32_t *ids,
                                uint32_t n, uint32_t *rows, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rsq_la_gather, dim3(n), dim3(256), 0, s, a, la, stride, ids, rows);
    return hipGetLastError();
}

hipError_t launch_rsq_la_store(const RsqArgs &a, uint32_t *la_recv, uint64_t stride, const uint32_t *ids, uint32_t n,
                               const uint32_t *rows, uint32_t *stamp, uint32_t *slot, uint32_t arrived, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rsq_la_store, dim3(n), dim3(256), 0, s, a, la_recv, stride, ids, rows, stamp, slot, arrived);
    return hipGetLastError();
}

hipError_t launch_rows_unroute(const uint32_t *perm, const uint8_t *rows, uint64_t slot, const uint32_t *len,
                               uint64_t n, uint8_t *out, uint32_t *out_len, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rows_unroute, dim3((uint32_t)n), dim3(256), 0, s, perm, rows, slot, len, out, out_len);
    return hipGetLastError();
}

hipError_t launch_rsq_unroute(const uint32_t *perm, const uint8_t *ans, uint64_t n, uint8_t *out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rsq_unroute, dim3(nb(n, 256)), dim3(256), 0, s, perm, ans, n, out);
    return hipGetLastError();
}

}  // namespace lx
