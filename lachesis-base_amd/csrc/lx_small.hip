// lx_small.hip -- the small-batch (latency) path of Add: one launch per batch.
//
// The reference's caller adds one event at a time (abft/indexed_lachesis.go:53-82:
// Process and Build each call Add once, Build then drops it again) or, through
// the level batcher, one antichain at a time.  For such batches the big path
// (branch assignment kernels, the persistent column walker, the LowestAfter
// tail pass) costs far more in launches and syncs than the work itself.  Here
// the host has already assigned branches in Add order (lx_capi.cpp,
// add_batch_small: the lastSeq rule of vecengine/index.go:105-141) and staged
// the batch as SmallEv records; one launch then does everything else:
//   * workgroup 0 writes the per-event metadata, the branch claims and the new
//     branches (read only by later launches);
//   * every workgroup owns kSmallCW columns (branches) and, as k_index, works
//     column by column with no inter-workgroup communication:
//       - for the batch's events on its own branches: the branch-row entry and
//         a zeroed LowestAfter row (the range fill below writes the observed
//         entries; nothing else may be left from an earlier epoch),
//       - level by level (the host sorts the batch into topological levels),
//         64 event lanes x kSmallCW columns: HighestBefore = max-join of the
//         parents' seqs (in-batch parents from LDS, older ones from the plane;
//         CollectFrom, vecfc/vector_ops.go:49-79) and the LowestAfter range fill
//         of DESIGN.md section 3 (the DFS of vecengine/index.go:212-225).
// Fork marks (k_marks) run after it when the epoch has forks.
#include "lx_internal.h"

namespace lx {

template <bool MASKED>
__device__ __forceinline__ void small_body(const SmallArgs &a, const uint32_t *img) {
    constexpr uint32_t CW = kSmallCW, NQ = 256 / CW;
    const SmallEv *ev = reinterpret_cast<const SmallEv *>(img);
    const uint32_t *par = img + a.o_par, *perm = img + a.o_perm, *lvl_off = img + a.o_loff;
    const uint32_t *new_first = img + a.o_nfirst, *new_creator = img + a.o_ncreator, *blen = img + a.o_blen;
    extern __shared__ uint32_t smem[];
    uint32_t *val = smem;                  // [n][CW]: HB seqs of the batch's events in own columns
    uint32_t *own = smem + a.n * CW;       // batch positions of the events on own branches
    __shared__ uint32_t n_own;

    const uint32_t t = threadIdx.x;
    const uint32_t k = t % CW, q = t / CW;
    const uint32_t c0 = blockIdx.x * CW;
    const uint32_t col = c0 + k;
    const bool valid = col < a.B;
    const uint32_t first = !valid ? 1u : col >= a.B0 ? new_first[col - a.B0] : a.branch_first[col];
    constexpr uint32_t mask = MASKED ? LX_SEQ_MASK : 0xFFFFFFFFu;
    const uint32_t bs = a.bs, n = a.n;
    const uint64_t stride = a.stride;

    if (t == 0) n_own = 0;
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
    __syncthreads();
    for (uint32_t i = t; i < n; i += 256) {
        const uint4 q0 = ev[i].q0;
        if (q0.x >= c0 && q0.x < c0 + CW) {
            a.brow[(uint64_t)q0.x * a.s_cap + (q0.y - ev[i].q1.y)] = bs + i;
            own[atomicAdd(&n_own, 1u)] = i;
        }
    }
    __syncthreads();
    {
        // zero the LowestAfter rows of own events (whole 16-B groups; stride is a multiple of 64)
        const uint32_t no = n_own, B4 = (a.B + 3) / 4;
        for (uint32_t x = t; x < no * B4; x += 256) {
            uint4 *row = reinterpret_cast<uint4 *>(a.la + (uint64_t)(bs + own[x / B4]) * stride);
            row[x % B4] = make_uint4(0, 0, 0, 0);
        }
    }
    // branch rows and zeroed rows are read / overwritten below only by this
    // workgroup: the barrier's workgroup-scope release/acquire orders them (an
    // agent-scope fence would write back the XCD's whole L2 on this part)
    __syncthreads();

    for (uint32_t L = 0; L < a.n_levels; L++) {
        const uint32_t lo = lvl_off[L], hi = lvl_off[L + 1];
        for (uint32_t j = lo + q; j < hi && valid; j += NQ) {
            const uint32_t i = perm[j];
            const uint4 q0 = ev[i].q0;
            const uint32_t po = ev[i].q1.x;
            const uint32_t br = q0.x, seq = q0.y, prev = q0.z, np = q0.w;
            uint32_t r = (col == br) ? seq : 0u;
            uint32_t p = 0;
            for (; p + 4 <= np; p += 4) {
                uint32_t x[4], v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) x[u] = par[po + p + u];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    v[u] = x[u] >= bs ? val[(x[u] - bs) * CW + k] : a.hb[(uint64_t)x[u] * stride + col];
#pragma unroll
                for (int u = 0; u < 4; u++) r = max(r, v[u] & mask);
            }
            for (; p < np; p++) {
                const uint32_t x = par[po + p];
                const uint32_t v = x >= bs ? val[(x - bs) * CW + k] : a.hb[(uint64_t)x * stride + col];
                r = max(r, v & mask);
            }
            a.hb[(uint64_t)(bs + i) * stride + col] = r;
            val[i * CW + k] = r;
            // LowestAfter range fill: events (col, s), s in (HB(prev)[col], r], are first
            // observed from branch br by this event
            uint32_t h0 = 0;
            if (prev != LX_NONE)
                h0 = (prev >= bs ? val[(prev - bs) * CW + k] : a.hb[(uint64_t)prev * stride + col]) & mask;
            for (uint32_t s = max(h0 + 1u, first); s <= r; s++) {
                const uint32_t row = a.brow[(uint64_t)col * a.s_cap + (s - first)];
                a.la[(uint64_t)row * stride + br] = seq;
            }
        }
        __syncthreads();
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

hipError_t launch_small(const SmallArgs &a, hipStream_t s) {
    if (!a.n || !a.B) return hipSuccess;
    const uint32_t grid = (a.B + kSmallCW - 1) / kSmallCW;
    const size_t lds = (size_t)a.n * (kSmallCW + 1) * 4;
    if (a.mask) hipLaunchKernelGGL(k_small<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(k_small<false>, dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_small_inline(const SmallInlineArgs &a, hipStream_t s) {
    if (!a.a.n || !a.a.B) return hipSuccess;
    const uint32_t grid = (a.a.B + kSmallCW - 1) / kSmallCW;
    const size_t lds = (size_t)a.a.n * (kSmallCW + 1) * 4;
    if (a.a.mask) hipLaunchKernelGGL(k_small_inline<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(k_small_inline<false>, dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}

}  // namespace lx
