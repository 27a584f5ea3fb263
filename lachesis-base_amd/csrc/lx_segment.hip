// lx_segment.hip -- the segmented walk's fix-up and LowestAfter pass
// (DESIGN.md section 6b).
//
// A batch [bs, bs + n) is split into G consecutive Add-order segments; segment
// k is walked by k_index with every parent before it (a boundary parent)
// contributing only its own (branch, seq) entry and no LowestAfter fill.  The
// walk leaves L(e): the max-join over the ancestors reached inside the
// segment plus the boundary parents themselves.  With J_k[c] = the last seq of
// branch c before segment k (branches are seq-consecutive chains and RAW grows
// along them), the reference's row is
//   RAW(e) = max(L(e), max_c' RAW((c', min(L(e)[c'], J_k[c']))))
// (every out-of-segment ancestor of e lies below the highest branch-c' event e
// reaches out of the segment, for some c').  An event with L(e) >= J_k in
// every column ("full") is exact already: no event before segment k observes
// a branch-c event after J_k[c], so every term of the max is <= J_k <= L(e).
// The walk's drains flag the others ("partial": the first levels of a
// segment); k_seg_partial gathers their referenced rows, segment by segment
// (a reference always lies in an earlier segment, final by then).
//
// LowestAfter: event e (prev p on its branch) fills (RAW(p)[c], RAW(e)[c]].
// The part above J_k[c] (rows of the segment) is (max(L(p)[c], J_k[c]),
// L(e)[c]] exactly -- above J_k a column of L is RAW -- so the walker's
// drains fill it as in an ordinary walk.  The part up to J_k[c] (rows before
// the segment) is empty unless p misses (c, J_k[c]): p partial, or p before
// the segment (e is its branch's first event in it); k_seg_la_edge fills it
// from the final rows for exactly those events and their partial ones.  Then
// the batch's tail zeroing and fork marks run as after an ordinary walk.
#include "lx_internal.h"

namespace lx {

namespace {

__device__ __forceinline__ uint32_t seg_of(const SegArgs &a, uint32_t e) {
    uint32_t lo = 0, hi = a.G;   // seg_lo[lo] <= e < seg_lo[hi]
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) / 2;
        if (e >= a.seg_lo[m]) lo = m;
        else hi = m;
    }
    return lo;
}

// the row-segment rank owning row e
__device__ __forceinline__ uint32_t rank_of(const SegArgs &a, uint32_t e) {
    return seg_of(a, e) / (a.per_rank ? a.per_rank : 1u);
}

__device__ __forceinline__ uint32_t row_of(const SegArgs &a, uint32_t c, uint32_t s) {
    return a.brow[(uint64_t)c * a.s_cap + (s - a.branch_first[c])];
}

// the final HighestBefore row of event x: at its own index in whole planes and
// for a row-segment rank's own rows; another rank's row it received in rhb
__device__ __forceinline__ const uint32_t *seg_hrow(const SegArgs &a, uint32_t x) {
    if (a.rhb && x < a.own_lo) return a.rhb + (uint64_t)a.hslot[x] * a.stride;
    return a.hb + (uint64_t)x * a.stride;
}

// per batch event, without atomics (a branch is a seq-consecutive chain in
// Add order, so each entry has exactly one writer): the last event of its
// branch in its segment writes its seq as that segment's entry, the branch's
// first batch event writes its own seq into cnt
__global__ void k_seg_scan(SegArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t e = a.bs + i;
    const uint32_t b = a.ev_branch[e], s = a.ev_seq[e], first = a.branch_first[b];
    const uint32_t k = seg_of(a, e);
    // the branch's next event: none, or its row (a later segment ends this one's run)
    const bool last_of_branch = s + 1 - first >= a.branch_len[b];
    if (last_of_branch || a.brow[(uint64_t)b * a.s_cap + (s + 1 - first)] >= a.seg_lo[k + 1])
        a.jt[(uint64_t)(k + 1) * a.B + b] = s;
    if (s == first || a.brow[(uint64_t)b * a.s_cap + (s - 1 - first)] < a.bs) a.cnt[b] = s;
}

// J_0 from the branch lengths before the batch, then J_{k+1} = max(J_k, last in k)
__global__ void k_seg_prefix_j(SegArgs a) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.B) return;
    // cnt[c]: the seq of the branch's first batch event (0: none in the batch)
    const uint32_t before = a.cnt[c] ? a.cnt[c] - a.branch_first[c] : a.branch_len[c];
    uint32_t j = before ? a.branch_first[c] + before - 1 : 0u;
    a.jt[c] = j;
    for (uint32_t k = 1; k <= a.G; k++) {
        uint32_t *p = a.jt + (uint64_t)k * a.B + c;
        j = max(j, *p);
        *p = j;
    }
}

// one workgroup per partial event of segment k (every earlier row final):
// the max of the rows it references, one per branch.  The row indices go to
// LDS first (one pass over the branches, in parallel), then every thread
// streams its columns of those rows eight at a time -- the loads of a group
// in flight together instead of one brow -> row -> max chain per branch
__global__ void __launch_bounds__(256) k_seg_partial(SegArgs a, uint32_t k) {
    extern __shared__ const uint32_t *refs[];   // <= B referenced rows (resolved to their storage)
    __shared__ uint32_t n_refs;
    const uint32_t e = a.plist[a.seg_lo[k] - a.bs + blockIdx.x];
    const uint32_t *J = a.jt + (uint64_t)k * a.B;
    uint32_t *row = a.hb + (uint64_t)e * a.stride;
    if (threadIdx.x == 0) n_refs = 0;
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) {
        const uint32_t m = min(row[c], J[c]);
        if (m) refs[atomicAdd(&n_refs, 1u)] = seg_hrow(a, row_of(a, c, m));
    }
    __syncthreads();
    const uint32_t n = n_refs;
    constexpr int W = 4;   // columns per thread per step
    constexpr uint32_t U = 8;   // referenced rows in flight per thread
    for (uint32_t c0 = threadIdx.x * W; c0 < a.stride; c0 += blockDim.x * W) {
        uint32_t acc[W];
#pragma unroll
        for (int i = 0; i < W; i++) acc[i] = row[c0 + i];
        uint32_t i = 0;
        for (; i + U <= n; i += U) {
            uint4 v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++)
                v[u] = *reinterpret_cast<const uint4 *>(refs[i + u] + c0);
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                acc[0] = max(acc[0], v[u].x & LX_SEQ_MASK);
                acc[1] = max(acc[1], v[u].y & LX_SEQ_MASK);
                acc[2] = max(acc[2], v[u].z & LX_SEQ_MASK);
                acc[3] = max(acc[3], v[u].w & LX_SEQ_MASK);
            }
        }
        for (; i < n; i++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(refs[i] + c0);
            acc[0] = max(acc[0], v.x & LX_SEQ_MASK);
            acc[1] = max(acc[1], v.y & LX_SEQ_MASK);
            acc[2] = max(acc[2], v.z & LX_SEQ_MASK);
            acc[3] = max(acc[3], v.w & LX_SEQ_MASK);
        }
        *reinterpret_cast<uint4 *>(row + c0) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
    }
}

// the events of segment k whose LowestAfter range reaches rows before the
// segment: partial events and their successors, every branch's first event
// (bit 1 of pflag dedupes; the list at elist[seg_lo[k] - bs ..])
__device__ __forceinline__ void edge_want(const SegArgs &a, uint32_t k, uint32_t e) {
    if (!(atomicOr(a.pflag + (e - a.bs), 2u) & 2u))
        a.elist[a.seg_lo[k] - a.bs + atomicAdd(a.ecount + k, 1u)] = e;
}

__global__ void k_seg_edges(SegArgs a, uint32_t k, uint32_t n_partial) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t *J0 = a.jt + (uint64_t)k * a.B, *J1 = a.jt + (uint64_t)(k + 1) * a.B;
    if (t < n_partial) {
        const uint32_t e = a.plist[a.seg_lo[k] - a.bs + t];
        edge_want(a, k, e);
        const uint32_t j = a.ev_branch[e], s = a.ev_seq[e];
        if (s < J1[j]) edge_want(a, k, row_of(a, j, s + 1));
    } else if (t - n_partial < a.B) {
        const uint32_t j = t - n_partial;
        if (J1[j] > J0[j]) edge_want(a, k, row_of(a, j, J0[j] ? J0[j] + 1 : a.branch_first[j]));
    }
}

// one workgroup per listed event e = (j, s) of segment k: the entries
// (c, s'), s' in (RAW(p)[c], min(RAW(e)[c], J_k[c])], from the final rows
__global__ void __launch_bounds__(256) k_seg_la_edge(SegArgs a, uint32_t k) {
    const uint32_t e = a.elist[a.seg_lo[k] - a.bs + blockIdx.x];
    const uint32_t j = a.ev_branch[e], sq = a.ev_seq[e];
    const uint32_t *J = a.jt + (uint64_t)k * a.B;
    const uint32_t *re = a.hb + (uint64_t)e * a.stride;
    const uint32_t *rp = sq > a.branch_first[j] ? seg_hrow(a, row_of(a, j, sq - 1)) : nullptr;
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) {
        const uint32_t hi = min(re[c] & LX_SEQ_MASK, J[c]);
        const uint32_t lo = max(rp ? (rp[c] & LX_SEQ_MASK) + 1u : 1u, a.branch_first[c]);
        for (uint32_t s = lo; s <= hi; s++) {
            const uint32_t x = row_of(a, c, s);
            if (x >= a.own_lo) {
                a.la[(uint64_t)x * a.stride + j] = sq;
            } else {
                // another rank's row: to the owner of its segment
                const uint32_t d = rank_of(a, x);
                const uint32_t p = atomicAdd(a.out_count + d, 1u);
                if (p < a.out_cap) {
                    uint32_t *o = a.out + 3ull * (d * a.out_cap + p);
                    o[0] = x;
                    o[1] = j;
                    o[2] = sq;
                }
            }
        }
    }
}

// ------------------------------------------------------------------ row segments (lx_rowseg.cpp)
__device__ __forceinline__ void rs_want(const RsArgs &r, uint32_t x) {
    if (atomicOr(r.need + x, 1u) == 0u) {
        const uint32_t p = atomicAdd(r.req_count, 1u);
        r.req[p] = x;
        r.hslot[x] = p;   // its row in the receive area
    }
}

// the rows the partial events of own segment k reference (one workgroup per
// partial event); rows of the rank's own earlier sub-segments are final after
// their own fix-up and are not asked for
__global__ void __launch_bounds__(256) k_rs_refs(SegArgs a, RsArgs r, uint32_t k) {
    const uint32_t e = a.plist[a.seg_lo[k] - a.bs + blockIdx.x];
    const uint32_t *J = a.jt + (uint64_t)k * a.B;
    const uint32_t *row = a.hb + (uint64_t)e * a.stride;
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) {
        const uint32_t m = min(row[c], J[c]);
        if (m) {
            const uint32_t x = row_of(a, c, m);
            if (x < r.lo) rs_want(r, x);
        }
    }
}

// the previous event of every branch's first own event (k_seg_la's first prev)
__global__ void k_rs_frontier(SegArgs a, RsArgs r) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.B) return;
    const uint32_t per = a.per_rank ? a.per_rank : 1u;
    const uint32_t j0 = a.jt[(uint64_t)a.own_seg * a.B + c], j1 = a.jt[(uint64_t)(a.own_seg + per) * a.B + c];
    if (j1 > j0 && j0) rs_want(r, row_of(a, c, j0));
}

// the still-needed requests grouped by owner segment: out = [d0 ids][d1 ids]...,
// counts[G] (one workgroup)
__global__ void __launch_bounds__(1024) k_rs_bucket(SegArgs a, RsArgs r, uint32_t n_req, uint32_t *out,
                                                    uint32_t *counts) {
    __shared__ uint32_t cnt[kMaxSegments], off[kMaxSegments];
    const uint32_t R = a.G / (a.per_rank ? a.per_rank : 1u);   // ranks
    if (threadIdx.x < R) cnt[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_req; i += blockDim.x) {
        const uint32_t x = r.req[i];
        if (r.need[x]) atomicAdd(&cnt[rank_of(a, x)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t o = 0;
        for (uint32_t d = 0; d < R; d++) {
            off[d] = o;
            o += cnt[d];
        }
    }
    __syncthreads();
    if (threadIdx.x < R) counts[threadIdx.x] = cnt[threadIdx.x];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_req; i += blockDim.x) {
        const uint32_t x = r.req[i];
        if (r.need[x]) out[atomicAdd(&off[rank_of(a, x)], 1u)] = x;
    }
}

// serve: own final rows (B words each) of the requested ids; ready[i] = 0 for
// a row that is not final yet (a partial event before its fix-up) or not own
__global__ void __launch_bounds__(256) k_rs_gather(RsArgs r, const uint32_t *ids, uint32_t *rows, uint32_t *ready) {
    const uint32_t x = ids[blockIdx.x];
    const bool own = x >= r.lo && x < r.hi;
    const bool ok = own && (r.partials_done || !(r.pflag[x - r.lo] & 1u));
    if (threadIdx.x == 0) ready[blockIdx.x] = ok ? 1u : 0u;
    if (!ok) return;
    const uint32_t *src = r.hb + (uint64_t)x * r.stride;
    uint32_t *dst = rows + (uint64_t)blockIdx.x * r.B;
    for (uint32_t c = threadIdx.x; c < r.B; c += blockDim.x) dst[c] = src[c];
}

// receive: ready rows into the plane; each newly received requested row
// counts down `remaining`
__global__ void __launch_bounds__(256) k_rs_scatter(RsArgs r, const uint32_t *ids, const uint32_t *rows,
                                                    const uint32_t *ready) {
    if (!ready[blockIdx.x]) return;
    const uint32_t x = ids[blockIdx.x];
    uint32_t *dst = r.rhb + (uint64_t)r.hslot[x] * r.stride;   // another rank's row: the receive area
    const uint32_t *src = rows + (uint64_t)blockIdx.x * r.B;
    for (uint32_t c = threadIdx.x; c < r.B; c += blockDim.x) dst[c] = src[c];
    if (threadIdx.x == 0 && atomicExch(r.need + x, 0u) == 1u) atomicSub(r.remaining, 1u);
}

__global__ void k_rs_la_apply(RsArgs r, const uint32_t *t, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = t[3 * i], j = t[3 * i + 1];
    if (x >= r.lo && x < r.hi && j < r.B) r.la[(uint64_t)x * r.stride + j] = t[3 * i + 2];
}

inline uint32_t nb(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

}  // namespace

hipError_t launch_seg_tables(const SegArgs &a, hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(a.jt, 0, (uint64_t)(a.G + 1) * a.B * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.cnt, 0, (uint64_t)(a.B + 2 * a.G) * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.pflag, 0, (uint64_t)a.n * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_scan, dim3(nb(a.n, 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_seg_prefix_j, dim3(nb(a.B, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_seg_partial(const SegArgs &a, uint32_t k, uint32_t count, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_seg_partial, dim3(count), dim3(256), (size_t)a.B * sizeof(void *), s, a, k);
    return hipGetLastError();
}

hipError_t launch_rs_refs(const SegArgs &a, const RsArgs &r, const uint32_t *n_partial, hipStream_t s) {
    const uint32_t per = a.per_rank ? a.per_rank : 1u;
    for (uint32_t k = 0; k < per; k++)
        if (n_partial[k]) hipLaunchKernelGGL(k_rs_refs, dim3(n_partial[k]), dim3(256), 0, s, a, r, a.own_seg + k);
    hipLaunchKernelGGL(k_rs_frontier, dim3(nb(a.B, 256)), dim3(256), 0, s, a, r);
    return hipGetLastError();
}

hipError_t launch_rs_bucket(const SegArgs &a, const RsArgs &r, uint32_t n_req, uint32_t *out, uint32_t *counts,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_rs_bucket, dim3(1), dim3(1024), 0, s, a, r, n_req, out, counts);
    return hipGetLastError();
}

hipError_t launch_rs_gather(const RsArgs &r, const uint32_t *ids, uint32_t n, uint32_t *rows, uint32_t *ready,
                            hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rs_gather, dim3(n), dim3(256), 0, s, r, ids, rows, ready);
    return hipGetLastError();
}

hipError_t launch_rs_scatter(const RsArgs &r, const uint32_t *ids, uint32_t n, const uint32_t *rows,
                             const uint32_t *ready, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rs_scatter, dim3(n), dim3(256), 0, s, r, ids, rows, ready);
    return hipGetLastError();
}

hipError_t launch_rs_la_apply(const RsArgs &r, const uint32_t *triples, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rs_la_apply, dim3(nb(n, 256)), dim3(256), 0, s, r, triples, n);
    return hipGetLastError();
}

hipError_t launch_seg_edges(const SegArgs &a, uint32_t k, uint32_t n_partial, hipStream_t s) {
    hipLaunchKernelGGL(k_seg_edges, dim3(nb((uint64_t)n_partial + a.B, 256)), dim3(256), 0, s, a, k, n_partial);
    return hipGetLastError();
}

hipError_t launch_seg_la_edge(const SegArgs &a, uint32_t k, uint32_t count, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_seg_la_edge, dim3(count), dim3(256), 0, s, a, k);
    return hipGetLastError();
}

}  // namespace lx
