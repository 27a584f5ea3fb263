// lx_small.hip -- the small-batch (latency) path of Add: one launch per batch.
//
// The reference's caller adds one event at a time (abft/indexed_lachesis.go:53-82:
// Process and Build each call Add once, Build then drops it again) or, through
// the level batcher, one antichain at a time.  For such batches the big path
// (branch assignment kernels, the persistent column walker, the LowestAfter
// tail pass) costs far more in launches and syncs than the work itself.  Here
// the host has already assigned branches in Add order (lx_capi.cpp,
// add_batch_small: the lastSeq rule of vecengine/index.go:105-141), sorted the
// run into topological levels and split every event's parents into the ones
// inside the run (batch positions) and the older ones (flush_pending); one
// launch does everything else.  Every workgroup owns kSmallCW = 4 columns
// (branches) and, as k_index, works column by column with no inter-workgroup
// communication, in four phases:
//   0. metadata, branch claims and new branches (workgroup 0, read only by
//      later launches); branch-row entries and zeroed LowestAfter rows of the
//      events on own branches; the level schedule and the in-run parent lists
//      copied to LDS;
//   1. the older parents' HB rows (final in the plane; 16 B = the 4 own
//      columns per parent, many loads in flight) max-ed into each event's LDS
//      value, which starts as its own seq in its own column;
//   2. level by level, LDS only: HighestBefore = the max-join with the in-run
//      parents' values (CollectFrom, vecfc/vector_ops.go:49-79), one barrier per
//      level that waits for LDS operations only;
//   3. HB rows out and the LowestAfter range fill of DESIGN.md section 3 (the
//      DFS of vecengine/index.go:212-225), every event at once.
// A 2048-event run of C3 (~40 levels) used to pay three dependent global
// loads per level (record, parent list, parent value) plus the fill's branch
// row; now a level costs a few LDS round trips.
// Fork marks (k_marks) run after it when the epoch has forks.
#include <algorithm>

#include "lx_internal.h"

namespace lx {

// LDS-only barrier: waits for this wave's LDS operations, not for its global
// stores (on gfx950 vmcnt also counts stores; __syncthreads' workgroup-scope
// release would wait for them).  The memory clobber keeps the compiler from
// moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// global -> LDS copy of n16 uint4, four loads in flight per thread
__device__ __forceinline__ void copy_to_lds(uint4 *dst, const uint4 *src, uint32_t n16, uint32_t t) {
    for (uint32_t x0 = t; x0 < n16; x0 += 256 * 4) {
        uint4 v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) v[u] = src[min(x0 + u * 256, n16 - 1)];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++)
            if (x0 + u * 256 < n16) dst[x0 + u * 256] = v[u];
    }
}

template <bool MASKED>
__device__ __forceinline__ void small_body(const SmallArgs &a, const uint32_t *img) {
    constexpr uint32_t CW = kSmallCW, NQ = 256 / CW, U = 8;
    static_assert(CW == 4, "one uint4 of HB per event and workgroup");
    const SmallEv *ev = reinterpret_cast<const SmallEv *>(img);
    const uint2 *meta = reinterpret_cast<const uint2 *>(img + a.o_meta);
    const uint32_t *pl = img + a.o_pl;
    const uint2 *old = reinterpret_cast<const uint2 *>(img + a.o_old);
    const uint32_t *lvl_off = img + a.o_loff;
    const uint32_t *new_first = img + a.o_nfirst, *new_creator = img + a.o_ncreator, *blen = img + a.o_blen;
    const uint32_t n = a.n, nh = a.n_h0, L = a.n_levels;
    // LDS (small_lds_bytes): val[n] (HB seqs of the 4 own columns), h0v[nh]
    // (HB of an older previous branch event), lmeta[n rounded to even], lpl[n_pl
    // rounded to 8], lloff[L + 1], own[n]
    extern __shared__ uint4 smem4[];
    const uint32_t n2 = (n + 1) & ~1u, npl8 = (a.n_pl + 7) & ~7u;
    uint4 *val = smem4;
    uint4 *h0v = val + n;
    uint2 *lmeta = reinterpret_cast<uint2 *>(h0v + nh);
    uint16_t *lpl = reinterpret_cast<uint16_t *>(lmeta + n2);
    uint32_t *lloff = reinterpret_cast<uint32_t *>(lpl + npl8);
    uint16_t *own = reinterpret_cast<uint16_t *>(lloff + L + 1);
    uint32_t *val32 = reinterpret_cast<uint32_t *>(val);
    uint32_t *h0v32 = reinterpret_cast<uint32_t *>(h0v);
    __shared__ uint32_t n_own;

    const uint32_t t = threadIdx.x;
    const uint32_t k = t % CW, q = t / CW;
    const uint32_t c0 = blockIdx.x * CW;
    const uint32_t col = c0 + k;
    const bool valid = col < a.B;
    const uint32_t first = !valid ? 1u : col >= a.B0 ? new_first[col - a.B0] : a.branch_first[col];
    constexpr uint32_t mask = MASKED ? LX_SEQ_MASK : 0xFFFFFFFFu;
    const uint32_t bs = a.bs;
    const uint64_t stride = a.stride;

    // ---- phase 0: metadata (workgroup 0), branch rows and the list of own
    // events, LDS images
    if (t == 0) n_own = 0;
    __syncthreads();
    if (blockIdx.x == 0) {
        for (uint32_t i = t; i < n; i += 256) {
            const SmallEv e = ev[i];
            const uint32_t g = bs + i;
            a.ev_creator[g] = e.q2.x;
            a.ev_seq[g] = e.q0.y;
            a.ev_branch[g] = e.q0.x;
            a.ev_bbefore[g] = e.q1.w;
            a.ev_sp[g] = e.q1.z;
            a.first_child[g] = e.q2.z;
            if (e.q2.y & kSmallCont) {
                if (e.q1.z == LX_NONE) a.first_root[e.q2.x] = g;
                else if (e.q1.z < bs) a.first_child[e.q1.z] = g;
            }
        }
        for (uint32_t b = t; b < a.B - a.B0; b += 256) {
            a.branch_first[a.B0 + b] = new_first[b];
            a.branch_creator[a.B0 + b] = new_creator[b];
        }
        for (uint32_t i = t; i < a.n_blen; i += 256) a.branch_len[blen[2 * i]] = blen[2 * i + 1];
    }
    copy_to_lds(reinterpret_cast<uint4 *>(lmeta), reinterpret_cast<const uint4 *>(meta), n2 / 2, t);
    copy_to_lds(reinterpret_cast<uint4 *>(lpl), reinterpret_cast<const uint4 *>(pl), npl8 / 8, t);
    for (uint32_t j = t; j <= L; j += 256) lloff[j] = lvl_off[j];
    for (uint32_t x = t; x < nh; x += 256) h0v[x] = make_uint4(0, 0, 0, 0);
    for (uint32_t i0 = t; i0 < n; i0 += 256 * 4) {
        // own seq in its own column (the parents are folded in below); branch
        // rows and the list of the events on own branches
        uint4 q0[4];
        uint32_t f[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t i = min(i0 + u * 256, n - 1);
            q0[u] = ev[i].q0;
            f[u] = ev[i].q1.y;
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t i = i0 + u * 256;
            if (i >= n) continue;
            const uint32_t d = q0[u].x - c0, s = q0[u].y;
            val[i] = make_uint4(d == 0 ? s : 0u, d == 1 ? s : 0u, d == 2 ? s : 0u, d == 3 ? s : 0u);
            if (d < CW) {
                a.brow[(uint64_t)q0[u].x * a.s_cap + (s - f[u])] = bs + i;
                own[atomicAdd(&n_own, 1u)] = (uint16_t)i;
            }
        }
    }
    // LDS only: the global stores above are ordered before phase 3 by the
    // barrier that ends phase 1, and phase 1 reads only rows older than the run
    lds_barrier();
    {
        // zero the LowestAfter rows of own events (whole 16-B groups; stride is a
        // multiple of 64); the range fill of phase 3 writes the observed entries,
        // ordered after these stores by the barrier that ends phase 1
        const uint32_t no = n_own, B4 = (a.B + 3) / 4;
        for (uint32_t x = t; x < no * B4; x += 256) {
            uint4 *row = reinterpret_cast<uint4 *>(a.la + (uint64_t)(bs + own[x / B4]) * stride);
            row[x % B4] = make_uint4(0, 0, 0, 0);
        }
    }
    // phase 3's first records, loaded now so that they are in registers when
    // the levels are done (one dependent global round trip less per launch)
    uint32_t br[U], sq[U], pv[U], sl[U];
    auto load_recs = [&](uint32_t x0) {
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t i = min(x0 + u * NQ, n - 1);
            const uint4 q0 = ev[i].q0, q2 = ev[i].q2;
            br[u] = q0.x;
            sq[u] = q0.y;
            pv[u] = q0.z;
            sl[u] = q2.w;
        }
    };
    load_recs(q);
    // ---- phase 1: parents older than the run (HB rows final in the plane) and
    // the older previous branch events, 16 B (the 4 own columns) per entry,
    // folded into LDS; every entry independent, U loads in flight per thread
    for (uint32_t e0 = t; e0 < a.n_old; e0 += 256 * U) {
        // loads without conditions (clamped to the last entry), so that all U
        // are in flight before the first is used
        uint2 o[U];
        uint4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) o[u] = old[min(e0 + u * 256, a.n_old - 1)];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) v[u] = *reinterpret_cast<const uint4 *>(a.hb + (uint64_t)o[u].y * stride + c0);
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            if (e0 + u * 256 >= a.n_old) continue;
            uint32_t *dst = (o[u].x & 0x80000000u) ? h0v32 + 4 * (o[u].x & 0x7FFFFFFFu) : val32 + 4 * o[u].x;
            atomicMax(dst + 0, v[u].x & mask);
            atomicMax(dst + 1, v[u].y & mask);
            atomicMax(dst + 2, v[u].z & mask);
            atomicMax(dst + 3, v[u].w & mask);
        }
    }
    // branch rows and zeroed rows are read / overwritten below only by this
    // workgroup: the barrier's workgroup-scope release/acquire orders them (an
    // agent-scope fence would write back the XCD's whole L2 on this part)
    __syncthreads();

    // ---- phase 2: HighestBefore level by level, LDS only (CollectFrom,
    // vecfc/vector_ops.go:49-79): the max-join of the in-run parents' values
    // into the value phase 1 left (own seq, older parents).  An event's in-run
    // parents come in chunks of 4 (padded with the event itself, whose value
    // does not change a max); up to 16 parents cost two LDS round trips.  The
    // next level's bounds and first meta entry are read ahead.
    {
        const uint2 *lpl2 = reinterpret_cast<const uint2 *>(lpl);
        uint32_t lo = lloff[0], hi = L ? lloff[1] : 0u;
        uint2 m_next = lo + q < hi ? lmeta[lo + q] : make_uint2(0, 0);
        for (uint32_t l = 0; l < L; l++) {
            const uint32_t hn = l + 2 <= L ? lloff[l + 2] : hi;
            uint2 m = m_next;
            m_next = hi + q < hn ? lmeta[hi + q] : make_uint2(0, 0);
            for (uint32_t j = lo + q; j < hi; j += NQ) {
                if (j != lo + q) m = lmeta[j];
                const uint32_t i = m.x & 0xFFFFu, cnt4 = m.x >> 16, off4 = m.y;
                uint32_t r = val32[4 * i + k];
                for (uint32_t c = 0; c < cnt4; c += 4) {
                    uint2 w[4];
#pragma unroll
                    for (uint32_t u = 0; u < 4; u++) w[u] = lpl2[off4 + min(c + u, cnt4 - 1)];
#pragma unroll
                    for (uint32_t u = 0; u < 4; u++)
                        r = max(max(r, max(val32[4 * (w[u].x & 0xFFFFu) + k], val32[4 * (w[u].x >> 16) + k])),
                                max(val32[4 * (w[u].y & 0xFFFFu) + k], val32[4 * (w[u].y >> 16) + k]));
                }
                val32[4 * i + k] = r;
            }
            lds_barrier();
            lo = hi;
            hi = hn;
        }
    }

    // ---- phase 3: HB rows out, LowestAfter range fill (the
    // DFS of vecengine/index.go:212-225): events (col, s), s in (HB(prev)[col],
    // HB(e)[col]], are first observed from branch(e) by e.  Every event is
    // final; U events per thread at a time keep U branch-row loads in flight.
    if (!valid) return;
    for (uint32_t x0 = q; x0 < n; x0 += NQ * U) {
        // records (the first iteration's were loaded before phase 1) and
        // branch rows loaded without conditions (clamped), U in flight
        uint32_t lo[U], hi[U], row[U];
        if (x0 != q) load_recs(x0);
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t i = x0 + u * NQ, ic = min(i, n - 1);
            const uint32_t r = val32[4 * ic + k];
            // HB(prev) from the run (val) or from phase 1 (h0v): one LDS read at a
            // computed address, no branch (a branch would sink the record loads)
            const uint32_t prev = pv[u];
            const uint32_t *hp = prev == LX_NONE ? val32 + 4 * ic : prev >= bs ? val32 + 4 * (prev - bs) : h0v32 + 4 * sl[u];
            const uint32_t h0 = prev == LX_NONE ? 0u : hp[k];
            lo[u] = max(h0 + 1u, first);
            hi[u] = i < n ? r : 0u;
            if (i < n) a.hb[(uint64_t)(bs + i) * stride + col] = r;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++)
            row[u] = a.brow[(uint64_t)col * a.s_cap + min(lo[u] - first, hi[u] >= lo[u] ? hi[u] - first : 0u)];
#pragma unroll
        for (uint32_t u = 0; u < U; u++)
            if (lo[u] <= hi[u]) a.la[(uint64_t)row[u] * stride + br[u]] = sq[u];
#pragma unroll
        for (uint32_t u = 0; u < U; u++)
            for (uint32_t s = lo[u] + 1; s <= hi[u]; s++)
                a.la[(uint64_t)a.brow[(uint64_t)col * a.s_cap + (s - first)] * stride + br[u]] = sq[u];
    }
}

template <bool MASKED>
__global__ __launch_bounds__(256) void k_small(SmallArgs a) {
    small_body<MASKED>(a, a.img);
}

// the image read straight from the kernel arguments (kernarg segment)
template <bool MASKED>
__global__ __launch_bounds__(256) void k_small_inline(SmallInlineArgs a) {
    small_body<MASKED>(a.a, a.img);
}

// ---- k_add1_row: the unchanged caller's FC-cache miss (lx_fccache.cpp) --
// Add of ONE pending event a and ForklessCause(a, b) for every slot b of the
// cache, one launch.  Workgroup (cg, sg) owns columns [64 cg, 64 cg + 64) and
// slots [128 sg, 128 sg + 128) (>= 256 workgroups at V = 1000, W = 2000: one
// per CU streams its slots' LowestAfter rows):
//   * every thread first issues its slot's loads -- the slot's event and tag
//     from the cache's device mirror (plus the host's changes since, carried
//     in the arguments), then LA(b) on the workgroup's columns and b's branch
//     and seq -- so they are in flight together with wave 0's HB(a) loads;
//   * wave 0 computes HB(a) on its 64 columns (max over the parents' rows, all
//     in flight at once; each workgroup recomputes it, no communication); the
//     sg == 0 workgroups store it and do a's LowestAfter range fill (DESIGN.md
//     section 3), workgroup (0, 0) writes the metadata and a's own LA row;
//   * every thread sums, for its slot b, w_c [0 < LA(b)[c] <= HB(a)[c]] over the
//     workgroup's columns except c = branch(a) -- the only LowestAfter column
//     a's Add writes, in other workgroups -- for which it adds w instead when the
//     column holds branch(b) and a reaches b: in a fork-free epoch LA(b)[br(a)]
//     is set and <= seq(a) iff a reaches b (vecfc/forkless_cause.go:63-82);
//   * per slot the partial sums meet in one 64-bit word by atomics: {number of
//     column groups so far, sum}; the thread whose add completes the count
//     compares the sum with the quorum, writes the answer and clears the word
//     (no last-workgroup pass, no fence).
__global__ __launch_bounds__(kAdd1Slots) void k_add1_row(Add1RowArgs a) {
    __shared__ uint32_t hbv[64], wv[64];
    const uint32_t t = threadIdx.x, cg = blockIdx.x, sg = blockIdx.y;
    const uint32_t s = sg * kAdd1Slots + t;
    const bool has = s < a.n_slots;
    uint32_t b = has ? a.evk[s] : 0u;
    uint32_t tg = has ? a.tag[s] : 0u;
    for (uint32_t u = 0; u < a.nd; u++)      // kernel arguments: scalar loads
        if (a.d_slot[u] == s) {
            b = a.d_ev[u];
            tg = a.d_tag[u];
            if (cg == 0) {
                a.evk[s] = b;
                a.tag[s] = (uint8_t)tg;
            }
        }
    const uint32_t c0 = cg * 64;
    const uint32_t br = a.e.q0.x, seq = a.e.q0.y, prev = a.e.q0.z, np = a.e.q0.w;
    const uint64_t stride = a.stride;
    // the slot's row and metadata, in flight under the HB computation
    const bool other = has && b != a.a;
    const uint32_t bq = other ? b : 0u;
    const uint4 *lr = reinterpret_cast<const uint4 *>(a.la + (uint64_t)bq * stride + c0);
    uint4 l[16];
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) l[i] = lr[i];
    const uint32_t bbr0 = a.ev_branch[bq], bseq0 = a.ev_seq[bq];
    const uint32_t c = c0 + t;
    const bool valid = t < 64 && c < a.B;
    uint32_t r = c == br ? seq : 0u, h0 = 0;
    if (t < 64) {
        const uint32_t cc = valid ? c : 0u;
        uint32_t v[kAdd1MaxPar / 2];
#pragma unroll
        for (uint32_t u = 0; u < kAdd1MaxPar / 2; u++)
            v[u] = np ? a.hb[(uint64_t)a.par[min(u, np - 1)] * stride + cc] : 0u;   // a root has no parents
        const uint32_t hp = prev != LX_NONE ? a.hb[(uint64_t)prev * stride + cc] : 0u;
        for (uint32_t p = kAdd1MaxPar / 2; p < np; p++) r = max(r, a.hb[(uint64_t)a.par[p] * stride + cc]);   // rare
#pragma unroll
        for (uint32_t u = 0; u < kAdd1MaxPar / 2; u++) r = max(r, v[u]);
        h0 = hp;
        hbv[t] = valid ? r : 0u;
        wv[t] = valid && c != br ? a.wpad[c] : 0u;
    } else if (sg == 0 && cg == 0) {
        const uint32_t u = t - 64;
        if (u == 0) {
            const uint32_t g = a.a, sp = a.e.q1.z, creator = a.e.q2.x;
            a.ev_creator[g] = creator;
            a.ev_seq[g] = seq;
            a.ev_branch[g] = br;
            a.ev_bbefore[g] = a.e.q1.w;
            a.ev_sp[g] = sp;
            a.first_child[g] = a.e.q2.z;
            if (a.e.q2.y & kSmallCont) {
                if (sp == LX_NONE) a.first_root[creator] = g;
                else a.first_child[sp] = g;
            }
            a.branch_len[br] = a.blen;
            a.brow[(uint64_t)br * a.s_cap + (seq - a.e.q1.y)] = g;
        }
        // a's LowestAfter row: its own branch observes it at its own seq
        uint4 *row = reinterpret_cast<uint4 *>(a.la + (uint64_t)a.a * stride);
        for (uint32_t x = u; x < (a.B + 3) / 4; x += kAdd1Slots - 64)
            row[x] = make_uint4(4 * x == br ? seq : 0u, 4 * x + 1 == br ? seq : 0u, 4 * x + 2 == br ? seq : 0u,
                                4 * x + 3 == br ? seq : 0u);
    }
    __syncthreads();
    if (has) {
        uint32_t part = 0;
        uint32_t bbr = br, bseq = seq;
        if (other) {
            bbr = bbr0;
            bseq = bseq0;
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                part += (l[i].x - 1u) < hbv[4 * i] ? wv[4 * i] : 0u;
                part += (l[i].y - 1u) < hbv[4 * i + 1] ? wv[4 * i + 1] : 0u;
                part += (l[i].z - 1u) < hbv[4 * i + 2] ? wv[4 * i + 2] : 0u;
                part += (l[i].w - 1u) < hbv[4 * i + 3] ? wv[4 * i + 3] : 0u;
            }
        }
        if (bbr - c0 < 64 && hbv[bbr - c0] >= bseq) part += a.w_br;
        // (kAdd1PsumStride 1: one 128-B line per slot measured slower)
        unsigned long long *w = reinterpret_cast<unsigned long long *>(a.psum) + (uint64_t)s * kAdd1PsumStride;
        const unsigned long long old = atomicAdd(w, (1ull << 32) | part);
        if ((uint32_t)(old >> 32) == gridDim.x - 1) {
            a.out[s] = (uint8_t)(tg << 1 | ((uint32_t)old + part >= a.quorum ? 1u : 0u));
            *w = 0;
        }
    }
    // HB(a) out and a's LowestAfter range fill, off the row's critical path
    if (sg == 0 && valid) {
        a.hb[(uint64_t)a.a * stride + c] = r;
        const uint32_t first = a.branch_first[c];
        // (br, seq) is a itself: its own LowestAfter row is written above
        const uint32_t hi = c == br ? seq - 1 : r;
        for (uint32_t x = max(h0 + 1u, first); x <= hi; x++)
            a.la[(uint64_t)a.brow[(uint64_t)c * a.s_cap + (x - first)] * stride + br] = seq;
    }
}

hipError_t launch_add1_row(const Add1RowArgs &a, hipStream_t s) {
    if (!a.n_slots || !a.B || a.e.q0.w > kAdd1MaxPar || a.nd > kAdd1Delta) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_add1_row, dim3((a.B + 63) / 64, (a.n_slots + kAdd1Slots - 1) / kAdd1Slots), dim3(kAdd1Slots),
                       0, s, a);
    return hipGetLastError();
}

// The pending run's staged image, pinned host memory -> its device copy, on
// the kernel's own stream: no copy-engine hand-off between the runs of a
// level-fed stream (flush_pending)
__global__ __launch_bounds__(256) void k_stage(uint4 *dst, const uint4 *src, uint32_t n16) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_stage(uint32_t *dst, const uint32_t *src, uint64_t words, hipStream_t s) {
    const uint32_t n16 = (uint32_t)((words + 3) / 4);
    if (!n16) return hipSuccess;
    hipLaunchKernelGGL(k_stage, dim3(std::min<uint32_t>((n16 + 255) / 256, 64)), dim3(256), 0, s,
                       reinterpret_cast<uint4 *>(dst), reinterpret_cast<const uint4 *>(src), n16);
    return hipGetLastError();
}

// ---- k_small_dbl: a deep, narrow pending run (the reference's per-event Add
// on configs[0]: 5 validators, every event its own DAG level) -- k_small pays
// one LDS barrier per level, so a 2048-event chain is 2048 dependent steps.
// One workgroup holds the run's whole rows (B <= kDblMaxB columns, fork-free)
// in LDS and iterates them to the fixpoint of k_dbl (lx_dbl.hip: compose
// through the in-run event J(e, c') that HB[e][c'] names, chain prefix max
// per branch), ~log2(depth) rounds; the metadata, branch rows, older parents
// and the LowestAfter range fill are those of k_small, on the same staged
// image.  Every value is the seq of an ancestor and the fixpoint folds in
// every parent, so the rows are CollectFrom's max-join (vecfc/vector_ops.go:49-79).
constexpr uint32_t kSdThreads = 1024;

__global__ __launch_bounds__(kSdThreads) void k_small_dbl(SmallArgs a) {
    extern __shared__ uint32_t sm[];
    const uint32_t *img = a.img;
    const SmallEv *ev = reinterpret_cast<const SmallEv *>(img);
    const uint2 *meta = reinterpret_cast<const uint2 *>(img + a.o_meta);
    const uint16_t *pl = reinterpret_cast<const uint16_t *>(img + a.o_pl);
    const uint2 *old = reinterpret_cast<const uint2 *>(img + a.o_old);
    const uint32_t *new_first = img + a.o_nfirst, *new_creator = img + a.o_ncreator, *blen = img + a.o_blen;
    const uint32_t n = a.n, B = a.B, B0 = a.B0, nh = a.n_h0, bs = a.bs;
    const uint64_t stride = a.stride;
    uint32_t *hbl = sm;              // n * B: the run's HB rows
    uint32_t *h0v = hbl + n * B;     // nh * B: rows of older previous branch events
    uint32_t *s0 = h0v + nh * B;     // B: first seq of the branch in the run (~0: none)
    uint32_t *cnt = s0 + B;          // B: events of the branch in the run
    uint32_t *start = cnt + B;       // B + 1: chain offsets into posl
    uint32_t *first = start + B + 1; // B: the branch's first seq (epoch)
    uint32_t *flag = first + B;      // [0] changed in this round
    uint16_t *posl = reinterpret_cast<uint16_t *>(flag + 2);   // run positions, chain (seq) order per branch
    const uint32_t t = threadIdx.x, lane = t % 64, wave = t / 64;

    // ---- metadata, new branches, branch lengths (k_small phase 0)
    for (uint32_t i = t; i < n; i += kSdThreads) {
        const SmallEv e = ev[i];
        const uint32_t g = bs + i;
        a.ev_creator[g] = e.q2.x;
        a.ev_seq[g] = e.q0.y;
        a.ev_branch[g] = e.q0.x;
        a.ev_bbefore[g] = e.q1.w;
        a.ev_sp[g] = e.q1.z;
        a.first_child[g] = e.q2.z;
        if (e.q2.y & kSmallCont) {
            if (e.q1.z == LX_NONE) a.first_root[e.q2.x] = g;
            else if (e.q1.z < bs) a.first_child[e.q1.z] = g;
        }
        a.brow[(uint64_t)e.q0.x * a.s_cap + (e.q0.y - e.q1.y)] = g;
    }
    for (uint32_t b = t; b < B - B0; b += kSdThreads) {
        a.branch_first[B0 + b] = new_first[b];
        a.branch_creator[B0 + b] = new_creator[b];
    }
    for (uint32_t i = t; i < a.n_blen; i += kSdThreads) a.branch_len[blen[2 * i]] = blen[2 * i + 1];
    for (uint32_t c = t; c < B; c += kSdThreads) {
        s0[c] = 0xFFFFFFFFu;
        cnt[c] = 0;
        first[c] = c >= B0 ? new_first[c - B0] : a.branch_first[c];
    }
    for (uint32_t x = t; x < (n + nh) * B; x += kSdThreads) hbl[x] = 0;   // hbl and h0v
    // zeroed LowestAfter rows of the run's events (whole 16-B groups)
    const uint32_t B4 = (B + 3) / 4;
    for (uint32_t x = t; x < n * B4; x += kSdThreads)
        reinterpret_cast<uint4 *>(a.la + (uint64_t)(bs + x / B4) * stride)[x % B4] = make_uint4(0, 0, 0, 0);
    if (t == 0) flag[0] = 0;
    __syncthreads();
    for (uint32_t i = t; i < n; i += kSdThreads) {
        const uint4 q0 = ev[i].q0;
        atomicMin(&s0[q0.x], q0.y);
        atomicAdd(&cnt[q0.x], 1u);
        hbl[i * B + q0.x] = q0.y;   // own seq in its own column
    }
    __syncthreads();
    if (t == 0) {
        start[0] = 0;
        for (uint32_t c = 0; c < B; c++) start[c + 1] = start[c] + cnt[c];
    }
    __syncthreads();
    // chain order; the direct in-run parents by (branch, seq); the older
    // parents and older previous branch events by their final rows
    for (uint32_t i = t; i < n; i += kSdThreads) {
        const uint4 q0 = ev[i].q0;
        posl[start[q0.x] + (q0.y - s0[q0.x])] = (uint16_t)i;   // seqs of a branch in the run are consecutive
    }
    for (uint32_t j = t; j < n; j += kSdThreads) {
        const uint2 m = meta[j];
        const uint32_t i = m.x & 0xFFFFu, cnt4 = m.x >> 16, off4 = m.y;
        for (uint32_t x = 4 * off4; x < 4 * (off4 + cnt4); x++) {
            const uint32_t p = pl[x];
            if (p == i) continue;   // padding
            const uint4 pq = ev[p].q0;
            atomicMax(&hbl[i * B + pq.x], pq.y);
        }
    }
    for (uint32_t x = t; x < a.n_old * B; x += kSdThreads) {
        const uint2 o = old[x / B];
        const uint32_t c = x % B;
        const uint32_t v = a.hb[(uint64_t)o.y * stride + c];
        if (o.x & 0x80000000u) h0v[(o.x & 0x7FFFFFFFu) * B + c] = v;
        else atomicMax(&hbl[o.x * B + c], v);
    }
    __syncthreads();

    // ---- the fixpoint (k_dbl): compose, then chain prefix max, until nothing changes
    for (;;) {
        bool ch = false;
        for (uint32_t x = t; x < n * B; x += kSdThreads) {
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
        for (uint32_t pr = wave; pr < B * B; pr += kSdThreads / 64) {
            const uint32_t c2 = pr / B, k = pr - c2 * B, m = cnt[c2], o = start[c2];
            uint32_t carry = 0;
            for (uint32_t off = 0; off < m; off += 64) {
                const uint32_t idx = off + lane;
                const uint32_t cell = idx < m ? (uint32_t)posl[o + idx] * B + k : 0u;
                const uint32_t old_v = idx < m ? hbl[cell] : 0u;
                uint32_t v = old_v;
#pragma unroll
                for (uint32_t dd = 1; dd < 64; dd <<= 1) {
                    const uint32_t u = __shfl_up(v, dd, 64);
                    if (lane >= dd) v = max(v, u);
                }
                v = max(v, carry);
                if (idx < m && v != old_v) { hbl[cell] = v; ch = true; }
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

    // ---- HB rows out, then the LowestAfter range fill (k_small phase 3)
    for (uint32_t x = t; x < n * B; x += kSdThreads) {
        const uint32_t i = x / B, c = x - i * B;
        a.hb[(uint64_t)(bs + i) * stride + c] = hbl[x];
    }
    for (uint32_t x = t; x < n * B; x += kSdThreads) {
        const uint32_t i = x / B, c = x - i * B;
        const uint4 q0 = ev[i].q0;
        const uint32_t prev = q0.z;
        const uint32_t h0 = prev == LX_NONE ? 0u : prev >= bs ? hbl[(prev - bs) * B + c] : h0v[ev[i].q2.w * B + c];
        const uint32_t f = first[c];
        for (uint32_t sq = max(h0 + 1u, f); sq <= hbl[x]; sq++)
            a.la[(uint64_t)a.brow[(uint64_t)c * a.s_cap + (sq - f)] * stride + q0.x] = q0.y;
    }
}

hipError_t launch_small_dbl(const SmallArgs &a, hipStream_t s) {
    if (!a.n || !a.B) return hipSuccess;
    if (a.mask || a.B > kDblMaxB || !a.img || small_dbl_lds_bytes(a.n, a.B, a.n_h0) > kDblLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_small_dbl, dim3(1), dim3(kSdThreads), small_dbl_lds_bytes(a.n, a.B, a.n_h0), s, a);
    return hipGetLastError();
}

hipError_t launch_small(const SmallArgs &a, hipStream_t s) {
    if (!a.n || !a.B) return hipSuccess;
    const uint32_t grid = (a.B + kSmallCW - 1) / kSmallCW;
    const size_t lds = small_lds_bytes(a.n, a.n_h0, a.n_levels, a.n_pl);
    if (a.mask) hipLaunchKernelGGL(k_small<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(k_small<false>, dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_small_inline(const SmallInlineArgs &a, hipStream_t s) {
    if (!a.a.n || !a.a.B) return hipSuccess;
    const uint32_t grid = (a.a.B + kSmallCW - 1) / kSmallCW;
    const size_t lds = small_lds_bytes(a.a.n, a.a.n_h0, a.a.n_levels, a.a.n_pl);
    if (a.a.mask) hipLaunchKernelGGL(k_small_inline<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(k_small_inline<false>, dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}

}  // namespace lx
