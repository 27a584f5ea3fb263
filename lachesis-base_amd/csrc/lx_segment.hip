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
// (a reference always lies in an earlier segment, final by then).  LowestAfter
// is then the walker's range fill computed from the final rows (k_seg_la), and
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

__device__ __forceinline__ uint32_t row_of(const SegArgs &a, uint32_t c, uint32_t s) {
    return a.brow[(uint64_t)c * a.s_cap + (s - a.branch_first[c])];
}

// per batch event: the last seq of its branch in its segment, and the number
// of batch events per branch
__global__ void k_seg_scan(SegArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t e = a.bs + i;
    const uint32_t b = a.ev_branch[e];
    atomicMax(a.jt + (uint64_t)(seg_of(a, e) + 1) * a.B + b, a.ev_seq[e]);
    atomicAdd(a.cnt + b, 1u);
}

// J_0 from the branch lengths before the batch, then J_{k+1} = max(J_k, last
// in k); the chain positions of the batch's events: [min before, max length)
// into cnt[B + G], cnt[B + G + 1]
__global__ void k_seg_prefix_j(SegArgs a) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.B) return;
    const uint32_t before = a.branch_len[c] - a.cnt[c];
    uint32_t j = before ? a.branch_first[c] + before - 1 : 0u;
    a.jt[c] = j;
    for (uint32_t k = 1; k <= a.G; k++) {
        uint32_t *p = a.jt + (uint64_t)k * a.B + c;
        j = max(j, *p);
        *p = j;
    }
    if (a.own_seg == LX_NONE) {
        if (a.cnt[c]) {
            atomicMin(a.cnt + a.B + a.G, before);
            atomicMax(a.cnt + a.B + a.G + 1, a.branch_len[c]);
        }
    } else {
        // chain positions of the own segment's events of branch c
        const uint32_t j0 = a.jt[(uint64_t)a.own_seg * a.B + c], j1 = a.jt[(uint64_t)(a.own_seg + 1) * a.B + c];
        if (j1 > j0) {
            const uint32_t f = a.branch_first[c];
            atomicMin(a.cnt + a.B + a.G, j0 ? j0 - f + 1 : 0u);
            atomicMax(a.cnt + a.B + a.G + 1, j1 - f + 1);
        }
    }
}

// one workgroup per partial event of segment k (every earlier row final):
// the max of the rows it references, one per branch
__global__ void __launch_bounds__(256) k_seg_partial(SegArgs a, uint32_t k) {
    extern __shared__ uint32_t lrow[];
    const uint32_t e = a.plist[a.seg_lo[k] - a.bs + blockIdx.x];
    const uint32_t *J = a.jt + (uint64_t)k * a.B;
    uint32_t *row = a.hb + (uint64_t)e * a.stride;
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) lrow[c] = row[c];
    __syncthreads();
    constexpr int W = 4;   // columns per thread per step
    for (uint32_t c0 = threadIdx.x * W; c0 < a.stride; c0 += blockDim.x * W) {
        uint32_t acc[W];
#pragma unroll
        for (int i = 0; i < W; i++) acc[i] = row[c0 + i];
        for (uint32_t b = 0; b < a.B; b++) {
            const uint32_t m = min(lrow[b], J[b]);
            if (!m) continue;
            const uint4 v = *reinterpret_cast<const uint4 *>(a.hb + (uint64_t)row_of(a, b, m) * a.stride + c0);
            acc[0] = max(acc[0], v.x & LX_SEQ_MASK);
            acc[1] = max(acc[1], v.y & LX_SEQ_MASK);
            acc[2] = max(acc[2], v.z & LX_SEQ_MASK);
            acc[3] = max(acc[3], v.w & LX_SEQ_MASK);
        }
        *reinterpret_cast<uint4 *>(row + c0) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
    }
}

// LowestAfter from the final rows: event y = (j, k) (the k-th event of
// branch j's chain) first observes the events (c, s), s in
// (RAW(prev)[c], RAW(y)[c]], prev = (j, k - 1) (the
// walker's range fill).  A task is 64 consecutive branches x kLK chain
// positions; it stages the rows of (j, k - 1 .. k + kLK - 1) 64 columns at a
// time through LDS, then a wave's lanes are the 64 branches of one column, so
// the stores of one seq s land in one 256-B run of row (c, s).  Tasks are
// dealt to XCDs in contiguous ranges (branch block major): the LowestAfter
// columns of a branch block are written through one XCD's L2, where the runs
// written by tasks at neighbouring chain positions merge into whole lines.
constexpr int kLJ = 64, kLC = 64, kLK = 16;

__global__ void __launch_bounds__(256) k_seg_la(SegArgs a, uint32_t nkc, uint32_t ntask) {
    __shared__ uint32_t buf[2][kLJ][kLC + 1];
    __shared__ uint32_t yrow[kLK + 1][kLJ];
    __shared__ uint32_t yany[kLK + 1];
    const uint32_t per = (ntask + 7) / 8;
    const uint32_t task = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (task >= ntask) return;
    const uint32_t jb = task / nkc, kc = task % nkc;
    const int64_t k0 = (int64_t)a.k_lo + (int64_t)kc * kLK;
    const uint32_t tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
    if (tid <= kLK) yany[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < (kLK + 1) * kLJ; i += 256) {
        const uint32_t kk = i / kLJ, j = jb * kLJ + i % kLJ;
        const int64_t k = k0 - 1 + kk;
        uint32_t r = LX_NONE;
        if (j < a.B && k >= 0 && k < (int64_t)a.branch_len[j]) r = a.brow[(uint64_t)j * a.s_cap + k];
        yrow[kk][i % kLJ] = r;
        if (kk && r != LX_NONE && r >= a.ev_lo && r < a.ev_hi) yany[kk] = 1;
    }
    __syncthreads();
    const uint32_t j = jb * kLJ + lane;
    const uint32_t fj = j < a.B ? a.branch_first[j] : 0u;
    const uint32_t ncc = (a.B + kLC - 1) / kLC;
    for (uint32_t cc = 0; cc < ncc; cc++) {
        const uint32_t c0 = cc * kLC;
        auto load = [&](uint32_t kk, uint32_t (*dst)[kLC + 1]) {
            for (uint32_t i = tid; i < kLJ * kLC / 4; i += 256) {
                const uint32_t r = i / (kLC / 4), q = i % (kLC / 4);
                const uint32_t y = yrow[kk][r];
                uint4 v = make_uint4(0, 0, 0, 0);
                if (y != LX_NONE) v = *reinterpret_cast<const uint4 *>(a.hb + (uint64_t)y * a.stride + c0 + q * 4);
                dst[r][q * 4 + 0] = v.x & LX_SEQ_MASK;
                dst[r][q * 4 + 1] = v.y & LX_SEQ_MASK;
                dst[r][q * 4 + 2] = v.z & LX_SEQ_MASK;
                dst[r][q * 4 + 3] = v.w & LX_SEQ_MASK;
            }
        };
        int pk = -1;        // chain offset whose rows buf[pb] holds (uniform)
        uint32_t pb = 0;
        for (uint32_t kk = 0; kk < (uint32_t)kLK; kk++) {
            if (!yany[kk + 1]) continue;   // no event of this pass at kk + 1 (uniform)
            if (pk != (int)kk) load(kk, buf[pb]);
            uint32_t (*P)[kLC + 1] = buf[pb];
            uint32_t (*R)[kLC + 1] = buf[pb ^ 1];
            load(kk + 1, R);
            __syncthreads();
            const uint32_t y = yrow[kk + 1][lane];
            if (y != LX_NONE && y >= a.ev_lo && y < a.ev_hi) {
                const uint32_t sq = fj + (uint32_t)(k0 + kk);
                // the wave's 16 columns: ranges first, then every first row
                // lookup in flight at once (the lookups were the pass's
                // critical path when issued one column at a time)
                constexpr int T = kLC / 4;
                uint32_t lo[T], hi[T], x[T];
#pragma unroll
                for (int t = 0; t < T; t++) {
                    const uint32_t ci = wave + 4 * t, c = c0 + ci;
                    const bool v = c < a.B;
                    const uint32_t f = v ? a.branch_first[c] : 1u;
                    hi[t] = v ? R[lane][ci] : 0u;
                    lo[t] = max(P[lane][ci] + 1u, f);
                    x[t] = lo[t] <= hi[t] ? a.brow[(uint64_t)c * a.s_cap + (lo[t] - f)] : 0u;
                }
#pragma unroll
                for (int t = 0; t < T; t++) {
                    const uint32_t c = c0 + wave + 4 * t;
                    for (uint32_t s = lo[t]; s <= hi[t]; s++) {
                        const uint32_t xr = s == lo[t] ? x[t] : row_of(a, c, s);
                        if (xr >= a.own_lo) {
                            a.la[(uint64_t)xr * a.stride + j] = sq;
                        } else {
                            // another rank's row: to the owner of its segment
                            const uint32_t d = seg_of(a, xr);
                            const uint32_t p = atomicAdd(a.out_count + d, 1u);
                            if (p < a.out_cap) {
                                uint32_t *o = a.out + 3ull * (d * a.out_cap + p);
                                o[0] = xr;
                                o[1] = j;
                                o[2] = sq;
                            }
                        }
                    }
                }
            }
            __syncthreads();
            pb ^= 1;
            pk = (int)kk + 1;
        }
    }
}

// ------------------------------------------------------------------ row segments (lx_rowseg.cpp)
__device__ __forceinline__ void rs_want(const RsArgs &r, uint32_t x) {
    if (atomicOr(r.need + x, 1u) == 0u) r.req[atomicAdd(r.req_count, 1u)] = x;
}

// the rows the own partial events reference (one workgroup per partial event)
__global__ void __launch_bounds__(256) k_rs_refs(SegArgs a, RsArgs r) {
    const uint32_t e = a.plist[blockIdx.x];
    const uint32_t *J = a.jt + (uint64_t)a.own_seg * a.B;
    const uint32_t *row = a.hb + (uint64_t)e * a.stride;
    for (uint32_t c = threadIdx.x; c < a.B; c += blockDim.x) {
        const uint32_t m = min(row[c], J[c]);
        if (m) rs_want(r, row_of(a, c, m));
    }
}

// the previous event of every branch's first own event (k_seg_la's first prev)
__global__ void k_rs_frontier(SegArgs a, RsArgs r) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.B) return;
    const uint32_t j0 = a.jt[(uint64_t)a.own_seg * a.B + c], j1 = a.jt[(uint64_t)(a.own_seg + 1) * a.B + c];
    if (j1 > j0 && j0) rs_want(r, row_of(a, c, j0));
}

// the still-needed requests grouped by owner segment: out = [d0 ids][d1 ids]...,
// counts[G] (one workgroup)
__global__ void __launch_bounds__(1024) k_rs_bucket(SegArgs a, RsArgs r, uint32_t n_req, uint32_t *out,
                                                    uint32_t *counts) {
    __shared__ uint32_t cnt[kMaxSegments], off[kMaxSegments];
    if (threadIdx.x < a.G) cnt[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_req; i += blockDim.x) {
        const uint32_t x = r.req[i];
        if (r.need[x]) atomicAdd(&cnt[seg_of(a, x)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t o = 0;
        for (uint32_t d = 0; d < a.G; d++) {
            off[d] = o;
            o += cnt[d];
        }
    }
    __syncthreads();
    if (threadIdx.x < a.G) counts[threadIdx.x] = cnt[threadIdx.x];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_req; i += blockDim.x) {
        const uint32_t x = r.req[i];
        if (r.need[x]) out[atomicAdd(&off[seg_of(a, x)], 1u)] = x;
    }
}

// serve: own final rows (B words each) of the requested ids; ready[i] = 0 for
// a row that is not final yet (a partial event before its fix-up) or not own
__global__ void __launch_bounds__(256) k_rs_gather(RsArgs r, const uint32_t *ids, uint32_t *rows, uint32_t *ready) {
    const uint32_t x = ids[blockIdx.x];
    const bool own = x >= r.lo && x < r.hi;
    const bool ok = own && (r.partials_done || !r.pflag[x - r.lo]);
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
    uint32_t *dst = r.hb + (uint64_t)x * r.stride;
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
    if ((e = hipMemsetAsync(a.cnt, 0, (uint64_t)(a.B + a.G) * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.cnt + a.B + a.G, 0xFF, 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.cnt + a.B + a.G + 1, 0, 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.pflag, 0, (uint64_t)a.n * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_scan, dim3(nb(a.n, 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_seg_prefix_j, dim3(nb(a.B, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_seg_partial(const SegArgs &a, uint32_t k, uint32_t count, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_seg_partial, dim3(count), dim3(256), (size_t)a.B * 4, s, a, k);
    return hipGetLastError();
}

hipError_t launch_rs_refs(const SegArgs &a, const RsArgs &r, uint32_t n_partial, hipStream_t s) {
    if (n_partial) hipLaunchKernelGGL(k_rs_refs, dim3(n_partial), dim3(256), 0, s, a, r);
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

hipError_t launch_seg_la(const SegArgs &a, hipStream_t s) {
    if (a.k_hi <= a.k_lo || !a.B) return hipSuccess;
    const uint32_t nkc = nb(a.k_hi - a.k_lo, kLK), njb = nb(a.B, kLJ);
    const uint32_t ntask = nkc * njb;
    hipLaunchKernelGGL(k_seg_la, dim3(8 * nb(ntask, 8)), dim3(256), 0, s, a, nkc, ntask);
    return hipGetLastError();
}

}  // namespace lx
