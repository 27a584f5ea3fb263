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
// the completion tag of a single-row call: every lane's row stores are made
// visible system-wide before lane 0 publishes the tag (pinned host memory)
__device__ __forceinline__ void get_done(const GetArgs &a, uint32_t lane) {
    if (!a.done) return;
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(a.done, a.tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// row i (event e) by one wave
__device__ __forceinline__ void get_row(const GetArgs &a, uint32_t i, uint32_t e, uint32_t lane) {
    if (e < a.row_lo || e >= a.row_hi || a.mode > 2) {
        // not a row of this handle (or no such mode): no read, an error length
        if (lane == 0) a.len[i] = kGetBadLen;
        get_done(a, lane);
        return;
    }
    const uint32_t *row = a.plane + (uint64_t)e * a.stride;
    uint32_t *o = reinterpret_cast<uint32_t *>(a.out + (uint64_t)i * a.slot);
    // entry of branch c: a column shard holds its own branches' columns only
    // (the others read as 0: the caller sums the shards' rows)
    const uint32_t *cmap = a.cmap;
    auto at = [row, cmap](uint32_t c) -> uint32_t {
        if (!cmap) return row[c];
        const uint32_t pc = cmap[c];
        return pc == LX_NONE ? 0u : row[pc];
    };
    if (a.mode == 2 && a.forks) {
        // 8 creators per lane computed before their stores (loads after a store
        // to host memory would wait for it, see below)
        for (uint32_t c0 = 0; c0 < a.V; c0 += 64 * 8) {
            uint2 xs[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; u++) {
                const uint32_t c = c0 + lane + 64 * u;
                uint2 x = make_uint2(0u, 0u);
                if (c < a.V) {
                    const int32_t k = a.cheat_of[c];
                    if (k < 0) {
                        const uint32_t v = at(c);
                        if (v) x = make_uint2(v & LX_SEQ_MASK, a.branch_first[c]);
                    } else {
                        for (uint32_t j = a.cheat_off[k]; j < a.cheat_off[k + 1]; j++) {
                            const uint32_t b = a.cheat_br[j];
                            const uint32_t v = at(b);
                            if (v & LX_MARK) { x = make_uint2(0u, 0x7FFFFFFFu); break; }
                            if (v > x.x) x = make_uint2(v, a.branch_first[b]);
                        }
                    }
                }
                xs[u] = x;
            }
#pragma unroll
            for (uint32_t u = 0; u < 8; u++) {
                const uint32_t c = c0 + lane + 64 * u;
                if (c < a.V) *reinterpret_cast<uint2 *>(o + 2 * c) = xs[u];
            }
        }
        if (lane == 0) a.len[i] = 8u * a.V;
        get_done(a, lane);
        return;
    }
    const bool hb = a.mode != 1;
    const uint32_t bb = a.ev_bbefore[e];
    const uint32_t lim = hb ? bb + (a.ev_branch[e] == bb ? 1u : 0u) : a.B;
    // the first kGetR x 64 columns (B <= 1024: the whole row) are loaded into
    // registers before any store: gfx950 counts stores in vmcnt, so a load
    // issued after a store to host memory would wait for that store's PCIe
    // round trip -- interleaved, a 1000-column row took 16 of them
    constexpr uint32_t kGetR = 16;
    uint32_t v[kGetR], f[kGetR];
    // (the loads do not wait for lim: entries of branches created after the
    // event's Add are 0 in its HighestBefore row, and masked below anyway)
#pragma unroll
    for (uint32_t u = 0; u < kGetR; u++) {
        const uint32_t c = lane + 64 * u;
        v[u] = c < a.B ? at(c) : 0u;
        f[u] = hb && c < a.B ? a.branch_first[c] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kGetR; u++)
        if (lane + 64 * u >= lim) v[u] = 0u;
    int last = -1;
#pragma unroll
    for (uint32_t u = 0; u < kGetR; u++)
        if (v[u]) last = (int)(lane + 64 * u);
    for (uint32_t c = lane + 64 * kGetR; c < lim; c += 64)   // rows wider than 1024 columns
        if (at(c)) last = (int)c;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) last = max(last, __shfl_xor(last, off, 64));
    const uint32_t ent = max(bb, (uint32_t)(last + 1));
    auto enc = [](uint32_t x, uint32_t first) {
        if (x & LX_MARK) return make_uint2(0u, 0x7FFFFFFFu);   // forkDetectedSeq
        return x ? make_uint2(x, first) : make_uint2(0u, 0u);  // {Seq, MinSeq}
    };
#pragma unroll
    for (uint32_t u = 0; u < kGetR; u++) {
        const uint32_t c = lane + 64 * u;
        if (c >= ent) continue;
        if (hb) *reinterpret_cast<uint2 *>(o + 2 * c) = enc(v[u], f[u]);
        else o[c] = v[u];
    }
    for (uint32_t c0 = 64 * kGetR; c0 < ent; c0 += 64 * kGetR) {   // wider rows: chunks, loads first
#pragma unroll
        for (uint32_t u = 0; u < kGetR; u++) {
            const uint32_t c = c0 + lane + 64 * u;
            v[u] = c < lim ? at(c) : 0u;
            f[u] = hb && c < lim ? a.branch_first[c] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kGetR; u++) {
            const uint32_t c = c0 + lane + 64 * u;
            if (c >= ent) continue;
            if (hb) *reinterpret_cast<uint2 *>(o + 2 * c) = enc(v[u], f[u]);
            else o[c] = v[u];
        }
    }
    if (lane == 0) a.len[i] = ent * (hb ? 8u : 4u);
    get_done(a, lane);
}

__global__ __launch_bounds__(256) void k_get_rows(GetArgs a) {
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (i >= a.n) return;
    get_row(a, i, a.ev ? a.ev[i] : a.ev0, lane);
}

// The resident single-row server: one wave polls the request
// word in pinned memory -- {tag : 30, mode : 2, event : 32}, tag kGetSrvStop =
// leave -- and answers each new tag like k_get_rows answers one row (row,
// length, then the tag into *done).  It leaves after idle_ticks without a
// request or budget_ticks in all (wall clock), publishing `gen` into *exited,
// so the host can tell a server that left from one still coming.  It reads
// only the request word until a request arrives, and the host posts one only
// when the handle's stream is idle and the arguments it was launched with
// still hold (lx_capi.cpp get_rows).
__global__ __launch_bounds__(64) void k_get_server(GetSrvArgs s) {
    const uint32_t lane = threadIdx.x;
    uint32_t seen = s.seen0;
    uint64_t last = wall_clock64();
    const uint64_t deadline = last + s.budget_ticks;
    for (;;) {
        uint64_t w;
        uint32_t q;
        bool go = false;
        for (;;) {
            w = __hip_atomic_load(s.req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            q = __builtin_amdgcn_readfirstlane((uint32_t)w & kGetSrvStop);
            if (q != seen) {
                go = q != kGetSrvStop;
                break;
            }
            const uint64_t now = wall_clock64();
            if (now - last > s.idle_ticks || now > deadline) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if (!go) break;
        // rows written by kernels on other queues (and XCDs) since the last request
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        GetArgs a = s.g;
        a.mode = __builtin_amdgcn_readfirstlane((uint32_t)w >> 30);   // 3: refused by get_row
        a.plane = a.mode == 1 ? s.la : s.hb;
        a.tag = q;
        get_row(a, 0, __builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)), lane);
        seen = q;
        last = wall_clock64();
    }
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(s.exited, s.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------- restart
// Restart from the persisted tables (lx_load_rows / lx_load_finish): table-S
// and table-s bytes of a chunk of events decoded into the planes, one wave per
// event.  HighestBefore entries {Seq, MinSeq}: Seq as the plane value, the
// marker {0, MaxInt32} as LX_MARK (its raw seq is rebuilt by k_load_raw);
// every non-empty entry must carry its branch's first seq as MinSeq and the
// event's own entry must be its seq (InitWithEvent) -- else bad[0] is set.
__global__ __launch_bounds__(256) void k_load_rows(LoadArgs a) {
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (i >= a.n) return;
    const uint32_t g = a.bs + i;
    const uint64_t h0 = a.hb_off[i] - a.hb_base, la0 = a.la_off[i] - a.la_base;
    const uint32_t hent = (uint32_t)((a.hb_off[i + 1] - a.hb_off[i]) / 8);
    const uint32_t lent = (uint32_t)((a.la_off[i + 1] - a.la_off[i]) / 4);
    const uint32_t br = a.ev_branch[g], seq = a.ev_seq[g];
    uint32_t *hrow = a.hb + (uint64_t)g * a.stride;
    uint32_t *lrow = a.la + (uint64_t)g * a.stride;
    bool bad = false;
    for (uint32_t c = lane; c < a.stride; c += 64) {
        uint32_t v = 0;
        if (c < hent) {
            uint2 x;
            memcpy(&x, a.hb_bytes + h0 + 8ull * c, 8);   // byte buffer: no alignment assumed
            if (x.x == 0 && x.y == 0x7FFFFFFFu) {
                v = LX_MARK;
            } else if (x.x) {
                v = x.x;
                bad |= c >= a.B || x.y != a.branch_first[c] || x.x > 0x7FFFFFFDu;
            } else {
                bad |= x.y != 0;
            }
        }
        if (c == br) bad |= !(v == seq || v == LX_MARK);
        hrow[c] = v;
        uint32_t l = 0;
        if (c < lent) memcpy(&l, a.la_bytes + la0 + 4ull * c, 4);
        lrow[c] = l;
    }
    if (lane == 0) a.brow[(uint64_t)br * a.s_cap + (seq - a.branch_first[br])] = g;
    if (__any(bad) && lane == 0) atomicOr(a.bad, 1u);
}

hipError_t launch_load_rows(const LoadArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(k_load_rows, dim3(nblk_p(a.n, 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// Raw seqs behind the persisted fork markers: the max-join of HighestBefore
// recomputed for the cheaters' branch columns (kSmallCW columns per workgroup,
// 64 event lanes, level by level over the whole epoch; parents' values are read
// back from the plane after the level barrier).  An entry loaded as a marker
// takes the raw value and is noted in lm[e * ncc + k]; any other entry must
// equal the recomputed value (else bad[0]).  k_marks then re-derives the
// markers and k_load_check compares them with lm.
__global__ __launch_bounds__(256) void k_load_raw(LoadRawArgs a) {
    constexpr uint32_t CW = kSmallCW, NQ = 256 / CW;
    const uint32_t k = threadIdx.x % CW, q = threadIdx.x / CW;
    const uint32_t kc = blockIdx.x * CW + k;
    const bool valid = kc < a.ncc;
    const uint32_t col = valid ? a.cols[kc] : 0u;
    bool bad = false;
    for (uint32_t L = 0; L < a.n_levels; L++) {
        const uint32_t lo = a.lvl_off[L], hi = a.lvl_off[L + 1];
        for (uint32_t j = lo + q; j < hi && valid; j += NQ) {
            const uint32_t e = a.perm[j];
            uint32_t r = a.ev_branch[e] == col ? a.ev_seq[e] : 0u;
            for (uint64_t p = a.poff[e]; p < a.poff[e + 1]; p++)
                r = max(r, a.hb[(uint64_t)a.par[p] * a.stride + col] & LX_SEQ_MASK);
            uint32_t *cell = a.hb + (uint64_t)e * a.stride + col;
            const uint32_t old = *cell;
            if (old & LX_MARK) {
                a.lm[(uint64_t)e * a.ncc + kc] = 1;
                *cell = r;
            } else {
                a.lm[(uint64_t)e * a.ncc + kc] = 0;
                bad |= old != r;
            }
        }
        __syncthreads();
    }
    if (bad) atomicOr(a.bad, 2u);
}

__global__ void k_load_check(LoadRawArgs a, uint32_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * a.ncc) return;
    const uint32_t e = (uint32_t)(t / a.ncc), kc = (uint32_t)(t % a.ncc);
    const bool marked = (a.hb[(uint64_t)e * a.stride + a.cols[kc]] & LX_MARK) != 0;
    if (marked != (a.lm[t] != 0)) atomicOr(a.bad, 4u);
}

// A fork marker is only valid in a column of a creator with more than one
// branch (vecengine/index.go:173-209 marks cheaters' branches only): any
// other marker cell -- a non-cheater's column, or anywhere in an epoch without
// fork branches -- is a corrupt row.  One thread per (row, column); bad |= 16.
__global__ void k_load_marks_ok(const uint32_t *hb, uint64_t stride, uint32_t n, uint32_t B,
                                const uint32_t *cheat_col, uint32_t *bad) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * B) return;
    const uint32_t e = (uint32_t)(t / B), c = (uint32_t)(t % B);
    if ((hb[(uint64_t)e * stride + c] & LX_MARK) && !cheat_col[c]) atomicOr(bad, 16u);
}

hipError_t launch_load_marks_ok(const uint32_t *hb, uint64_t stride, uint32_t n, uint32_t B, const uint32_t *cheat_col,
                                uint32_t *bad, hipStream_t s) {
    const uint64_t t = (uint64_t)n * B;
    if (!t) return hipSuccess;
    hipLaunchKernelGGL(k_load_marks_ok, dim3((uint32_t)((t + 255) / 256)), dim3(256), 0, s, hb, stride, n, B, cheat_col,
                       bad);
    return hipGetLastError();
}

hipError_t launch_load_raw(const LoadRawArgs &a, hipStream_t s) {
    if (!a.ncc) return hipSuccess;
    hipLaunchKernelGGL(k_load_raw, dim3((a.ncc + kSmallCW - 1) / kSmallCW), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_load_check(const LoadRawArgs &a, uint32_t n, hipStream_t s) {
    const uint64_t t = (uint64_t)n * a.ncc;
    if (!t) return hipSuccess;
    hipLaunchKernelGGL(k_load_check, dim3((uint32_t)((t + 255) / 256)), dim3(256), 0, s, a, n);
    return hipGetLastError();
}

// Every loaded LowestAfter entry must be what the range fill (DESIGN.md
// section 3; the DFS of vecengine/index.go:212-225) gives from the loaded
// HighestBefore rows: LA(x)[j] = s != 0 iff event (j, s) observes x and (j, s-1)
// does not (or s is j's first seq); LA(x)[j] = 0 iff the last event of j does
// not observe x.  One thread per (row, branch); bad |= 8.
__global__ void k_load_verify_la(LoadVerifyArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)a.n * a.B) return;
    const uint32_t x = (uint32_t)(t / a.B), j = (uint32_t)(t % a.B);
    const uint32_t s = a.la[(uint64_t)x * a.stride + j];
    const uint32_t bx = a.ev_branch[x], sx = a.ev_seq[x];
    const uint32_t f = a.branch_first[j], len = a.branch_len[j];
    bool bad;
    if (s) {
        bad = s < f || s - f >= len;
        if (!bad) {
            const uint32_t y = a.brow[(uint64_t)j * a.s_cap + (s - f)];
            bad = (a.hb[(uint64_t)y * a.stride + bx] & LX_SEQ_MASK) < sx;
            if (!bad && s > f) {
                const uint32_t y0 = a.brow[(uint64_t)j * a.s_cap + (s - 1 - f)];
                bad = (a.hb[(uint64_t)y0 * a.stride + bx] & LX_SEQ_MASK) >= sx;
            }
        }
    } else {
        bad = len && (a.hb[(uint64_t)a.brow[(uint64_t)j * a.s_cap + (len - 1)] * a.stride + bx] & LX_SEQ_MASK) >= sx;
    }
    if (bad) atomicOr(a.bad, 8u);
}

hipError_t launch_load_verify_la(const LoadVerifyArgs &a, hipStream_t s) {
    const uint64_t t = (uint64_t)a.n * a.B;
    if (!t) return hipSuccess;
    hipLaunchKernelGGL(k_load_verify_la, dim3((uint32_t)((t + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_get_server(const GetSrvArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_get_server, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_get_rows(const GetArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(k_get_rows, dim3(nblk_p(a.n, 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace lx
