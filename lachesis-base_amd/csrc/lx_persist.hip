// lx_persist.hip -- write-back of the index to the reference's kvdb byte
// formats (vecfc/vector.go:14-102, vecfc/store_vectors.go:53-65).
//
//   k_dirty_la    : rows of table "s" a Flush must rewrite -- the new rows plus
//                   every older row k_index range-filled for the events added
//                   since the last flush (the reference's DFS Visits,
//                   vecengine/index.go:212-225); the same ranges as the
//                   rollback kernel k_unfill, recomputed from the HB rows
//   k_row_bytes   : byte length of each row; lengths are history-dependent
//                   (DESIGN.md section 2): max(branches before Add, last
//                   non-empty branch + 1) entries of 8 B (HB) or 4 B (LA)
//   k_encode_rows : the rows in the byte layout -- HighestBefore LE {Seq,
//                   MinSeq} with MinSeq = the branch's first seq and the fork
//                   marker {0, MaxInt32} (vector.go:91-97); LowestAfter LE seq
// Streaming, HBM-bound; one wave per row in the row kernels.
#include <hipcub/hipcub.hpp>

#include "lx_internal.h"

namespace lx {

static inline uint32_t nblk_p(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

__global__ void k_flag_new(uint32_t *flag, uint32_t lo, uint32_t hi) {
    const uint32_t e = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (e < hi) flag[e] = 1u;
}

// (event, column) -> the rows whose LowestAfter entry in the event's branch it set
__global__ void k_dirty_la(UnfillArgs a, uint32_t *flag) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = (uint64_t)(a.hi - a.lo) * a.B;
    if (t >= total) return;
    const uint32_t e = a.lo + (uint32_t)(t / a.B);
    const uint32_t c = (uint32_t)(t % a.B);
    const uint32_t sp = a.ev_sp[e];
    const bool opens = a.ev_branch[e] == a.ev_bbefore[e];
    const uint32_t h1 = a.hb[(uint64_t)e * a.stride + c] & LX_SEQ_MASK;
    const uint32_t h0 = (sp != LX_NONE && !opens) ? (a.hb[(uint64_t)sp * a.stride + c] & LX_SEQ_MASK) : 0u;
    const uint32_t first = a.branch_first[c];
    for (uint32_t s = max(h0 + 1u, first); s <= h1; s++) flag[a.brow[(uint64_t)c * a.s_cap + (s - first)]] = 1u;
}

hipError_t launch_dirty_la(const UnfillArgs &a, uint32_t *flag, hipStream_t s) {
    if (a.hi <= a.lo) return hipSuccess;
    hipLaunchKernelGGL(k_flag_new, dim3(nblk_p(a.hi - a.lo, 256)), dim3(256), 0, s, flag, a.lo, a.hi);
    const uint64_t total = (uint64_t)(a.hi - a.lo) * a.B;
    if (total) hipLaunchKernelGGL(k_dirty_la, dim3(nblk_p(total, 256)), dim3(256), 0, s, a, flag);
    return hipGetLastError();
}

hipError_t persist_tmp_bytes(uint32_t n, size_t *bytes) {
    size_t a = 0, b = 0;
    hipError_t r = hipcub::DeviceScan::InclusiveSum(nullptr, a, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
    if (r != hipSuccess) return r;
    r = hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n + 1);
    *bytes = a > b ? a : b;
    return r;
}

__global__ void k_compact_flags(const uint32_t *flag, const uint32_t *pos, uint32_t n, uint32_t *rows) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n && flag[e]) rows[pos[e] - 1] = e;
}

hipError_t launch_compact(const uint32_t *flag, uint32_t *pos, uint32_t n, void *tmp, size_t tmp_bytes,
                          uint32_t *rows, hipStream_t s) {
    if (!n) return hipSuccess;
    size_t tb = tmp_bytes;
    hipError_t r = hipcub::DeviceScan::InclusiveSum(tmp, tb, flag, pos, (int)n, s);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL(k_compact_flags, dim3(nblk_p(n, 256)), dim3(256), 0, s, flag, pos, n, rows);
    return hipGetLastError();
}

__global__ void k_iota(uint32_t *rows, uint32_t lo, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rows[i] = lo + i;
}

hipError_t launch_iota(uint32_t *rows, uint32_t lo, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_iota, dim3(nblk_p(n, 256)), dim3(256), 0, s, rows, lo, n);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_row_bytes(RowsArgs a, uint64_t *len) {
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (i >= a.n) return;
    const uint32_t e = a.rows[i];
    const uint32_t bb = a.ev_bbefore[e];
    // HB: branches existing after Add(e); LA: every branch (later Visits grow the row)
    const uint32_t lim = a.hb ? bb + (a.ev_branch[e] == bb ? 1u : 0u) : a.B;
    const uint32_t *row = a.plane + (uint64_t)e * a.stride;
    int last = -1;
    for (uint32_t c = lane; c < lim; c += 64)
        if (row[c]) last = (int)c;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) last = max(last, __shfl_xor(last, off, 64));
    if (lane == 0) len[i] = (uint64_t)max(bb, (uint32_t)(last + 1)) * (a.hb ? 8u : 4u);
}

hipError_t launch_row_offsets(const RowsArgs &a, uint64_t *len, uint64_t *off, void *tmp, size_t tmp_bytes,
                              hipStream_t s) {
    hipError_t r = hipMemsetAsync(len + a.n, 0, 8, s);
    if (r != hipSuccess) return r;
    if (a.n) hipLaunchKernelGGL(k_row_bytes, dim3(nblk_p(a.n, 4)), dim3(256), 0, s, a, len);
    size_t tb = tmp_bytes;
    return hipcub::DeviceScan::ExclusiveSum(tmp, tb, len, off, (int)(a.n + 1), s);
}

// rows [0, n) of `a` into out + (off[i] - base) / 4 (off in bytes; HB rows are
// whole 8-B entries, so the uint2 stores are aligned)
__global__ __launch_bounds__(256) void k_encode_rows(RowsArgs a, const uint64_t *off, uint64_t base, uint32_t *out) {
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (i >= a.n) return;
    const uint32_t *row = a.plane + (uint64_t)a.rows[i] * a.stride;
    uint32_t *o = out + (off[i] - base) / 4;
    const uint32_t words = (uint32_t)((off[i + 1] - off[i]) / 4);
    if (a.hb) {
        for (uint32_t c = lane; 2 * c < words; c += 64) {
            const uint32_t v = row[c];
            uint2 x = make_uint2(0u, 0u);
            if (v & LX_MARK) x.y = 0x7FFFFFFFu;                   // forkDetectedSeq
            else if (v) x = make_uint2(v, a.branch_first[c]);     // {Seq, MinSeq}
            *reinterpret_cast<uint2 *>(o + 2 * c) = x;
        }
    } else {
        for (uint32_t c = lane; c < words; c += 64) o[c] = row[c];
    }
}

hipError_t launch_encode_rows(const RowsArgs &a, const uint64_t *off, uint64_t base, uint32_t *out, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(k_encode_rows, dim3(nblk_p(a.n, 4)), dim3(256), 0, s, a, off, base, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- getters
// GetHighestBefore / GetLowestAfter (vecfc/store_vectors.go:26-51) and
// GetMergedHighestBefore (vecengine/index.go:235-250 with GatherFrom,
// vecfc/vector_ops.go:81-96) for a batch of events, encoded on the device in the
// reference byte layout: one wave per event, row i written at out + i * slot
// (pinned host memory: one launch, no copies), its byte length in len[i].
// Merged with forks: per creator the first fork-marked branch wins ({0,
// MaxInt32}), else the strictly greatest Seq (first max wins) with its MinSeq
// (the branch's first seq), else {0, 0}; 8 x V bytes.  Without forks the
// reference returns the raw HighestBefore row.
__global__ __launch_bounds__(256) void k_get_rows(GetArgs a) {
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (i >= a.n) return;
    const uint32_t e = a.ev[i];
    const uint32_t *row = a.plane + (uint64_t)e * a.stride;
    uint32_t *o = reinterpret_cast<uint32_t *>(a.out + (uint64_t)i * a.slot);
    if (a.mode == 2 && a.forks) {
        for (uint32_t c = lane; c < a.V; c += 64) {
            uint2 x = make_uint2(0u, 0u);
            const int32_t k = a.cheat_of[c];
            if (k < 0) {
                const uint32_t v = row[c];
                if (v) x = make_uint2(v & LX_SEQ_MASK, a.branch_first[c]);
            } else {
                for (uint32_t j = a.cheat_off[k]; j < a.cheat_off[k + 1]; j++) {
                    const uint32_t b = a.cheat_br[j];
                    const uint32_t v = row[b];
                    if (v & LX_MARK) { x = make_uint2(0u, 0x7FFFFFFFu); break; }
                    if (v > x.x) x = make_uint2(v, a.branch_first[b]);
                }
            }
            *reinterpret_cast<uint2 *>(o + 2 * c) = x;
        }
        if (lane == 0) a.len[i] = 8u * a.V;
        return;
    }
    const bool hb = a.mode != 1;
    const uint32_t bb = a.ev_bbefore[e];
    const uint32_t lim = hb ? bb + (a.ev_branch[e] == bb ? 1u : 0u) : a.B;
    int last = -1;
    for (uint32_t c = lane; c < lim; c += 64)
        if (row[c]) last = (int)c;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) last = max(last, __shfl_xor(last, off, 64));
    const uint32_t ent = max(bb, (uint32_t)(last + 1));
    if (hb) {
        for (uint32_t c = lane; c < ent; c += 64) {
            const uint32_t v = c < lim ? row[c] : 0u;
            uint2 x = make_uint2(0u, 0u);
            if (v & LX_MARK) x.y = 0x7FFFFFFFu;
            else if (v) x = make_uint2(v, a.branch_first[c]);
            *reinterpret_cast<uint2 *>(o + 2 * c) = x;
        }
    } else {
        for (uint32_t c = lane; c < ent; c += 64) o[c] = row[c];
    }
    if (lane == 0) a.len[i] = ent * (hb ? 8u : 4u);
}

hipError_t launch_get_rows(const GetArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(k_get_rows, dim3(nblk_p(a.n, 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace lx
