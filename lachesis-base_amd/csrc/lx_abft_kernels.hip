// lx_abft_kernels.hip -- CDNA4 (gfx950) kernels of the batched abft caller.
//
// The abft orderer (lx_abft.cpp) asks two kinds of questions, both batched:
//
//   k_root_fc      : ForklessCause(e, r) for every candidate e x every root r
//                    of one frame (abft/event_processing.go:148-161 asks it
//                    root by root; election.go:110-124 asks it again per root
//                    slot).  One 64x64 (event x root) tile per workgroup; the
//                    HB rows of the 64 events and the LA rows of the 64 roots
//                    are staged through LDS 32 columns at a time, so each row
//                    is read once per tile instead of once per pair (the pair
//                    kernel k_fc streams 8*B bytes per query).  Integer VALU:
//                    per (pair, column) one compare, one select, one add.
//                    Result: one bit per pair (bits[e][r/32]).
//   k_root_quorum  : per candidate, the stake of the distinct creators of the
//                    roots it forkless-causes, >= quorum
//                    (forklessCausedByQuorumOn, WeightCounter.Count).
//   k_vote_*       : election votes of one round for every root slot of a
//                    frame and every subject validator
//                    (abft/election/election_math.go:13-114): weighted yes/no
//                    sums over the observed roots of the previous frame, the
//                    Byzantine sanity checks, and the earliest deciding root
//                    per subject (atomicMin on (event << 32 | vote)).
#include "lx_internal.h"

namespace lx {

// ---------------------------------------------------------------------------- k_root_fc
constexpr int kTile = 64;     // events x roots per workgroup
constexpr int kKc = 32;       // columns per LDS chunk
constexpr int kLdsPitch = kTile + 4;

template <bool FORKS>
__device__ __forceinline__ uint32_t hb_prep(uint32_t h) {
    // a marked branch never counts (vecfc/forkless_cause.go:73-78)
    return FORKS ? (((int32_t)h < 0) ? 0u : h) : h;
}

// Merged launches (MULTI): the frame steps of a claimed batch in one grid.
// Step k owns blocks [am[k].block0, am[k + 1].block0); its args come from the
// device table (uniform per workgroup: scalar loads).
template <typename A>
__device__ __forceinline__ uint32_t step_of(const A *am, uint32_t n_steps, uint32_t b) {
    uint32_t lo = 0, hi = n_steps;   // last k with am[k].block0 <= b
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (am[mid].block0 <= b) lo = mid;
        else hi = mid;
    }
    return lo;
}

// the step's args and this workgroup's tile (roots bx, events by, column split bz)
__device__ __forceinline__ RootFcArgs fc_step(const RootFcArgs *am, uint32_t n_steps, uint32_t *bx, uint32_t *by,
                                              uint32_t *bz) {
    const uint32_t k = step_of(am, n_steps, blockIdx.x);
    const RootFcArgs a = am[k];
    const uint32_t t = blockIdx.x - a.block0;
    const uint32_t tx = (a.n_roots + kTile - 1) / kTile, ty = (a.n_cand + kTile - 1) / kTile;
    *bx = t % tx;
    *by = (t / tx) % ty;
    *bz = t / (tx * ty);
    return a;
}

// fc_term of k_fc in staged form: (la - 1) < hb'  <=>  la != 0 && la <= hb
template <bool FORKS, bool MULTI>
__global__ __launch_bounds__(256) void k_root_fc(RootFcArgs a1, const RootFcArgs *am, uint32_t n_steps) {
    uint32_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    const RootFcArgs a = MULTI ? fc_step(am, n_steps, &bx, &by, &bz) : a1;
    __shared__ uint32_t sH[kKc][kLdsPitch];
    __shared__ uint32_t sL[kKc][kLdsPitch];
    __shared__ uint32_t sW[kKc];

    const uint32_t tid = threadIdx.x;
    const uint32_t tx = tid & 15, ty = tid >> 4;          // roots tx*4.., events ty*4..
    const uint32_t r0 = bx * kTile, e0 = by * kTile;

    // staging role: row = tid / 4, 8 columns = (tid % 4) * 8
    const uint32_t srow = tid >> 2, spart = (tid & 3) * 8;
    const uint32_t se = e0 + srow < a.n_cand ? a.cand[e0 + srow] : a.cand[0];
    uint32_t sr = r0 + srow < a.n_roots ? a.roots[r0 + srow] : LX_NONE;
    if (sr == LX_NONE) sr = a.roots_fallback;
    const uint4 *hrow = reinterpret_cast<const uint4 *>(a.hb + (uint64_t)se * a.stride + spart);
    const uint4 *lrow = reinterpret_cast<const uint4 *>(a.la + (uint64_t)sr * a.stride + spart);

    uint32_t sum[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) sum[i][k] = 0;

    const uint32_t cs = a.col_split, jlo = bz * cs, jhi = jlo + cs < a.ncols ? jlo + cs : a.ncols;
    for (uint32_t j0 = jlo; j0 < jhi; j0 += kKc) {
        const uint4 h0 = hrow[j0 / 4], h1 = hrow[j0 / 4 + 1];
        const uint4 l0 = lrow[j0 / 4], l1 = lrow[j0 / 4 + 1];
        const uint32_t hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        const uint32_t lv[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
#pragma unroll
        for (int q = 0; q < 8; q++) {
            sH[spart + q][srow] = hb_prep<FORKS>(hv[q]);
            sL[spart + q][srow] = lv[q] - 1u;
        }
        if (tid < kKc) sW[tid] = a.wpad[j0 + tid];
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < kKc; j++) {
            const uint4 h = *reinterpret_cast<const uint4 *>(&sH[j][ty * 4]);
            const uint4 l = *reinterpret_cast<const uint4 *>(&sL[j][tx * 4]);
            const uint32_t w = sW[j];
            const uint32_t hh[4] = {h.x, h.y, h.z, h.w};
            const uint32_t ll[4] = {l.x, l.y, l.z, l.w};
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int k = 0; k < 4; k++) sum[i][k] += (ll[k] < hh[i]) ? w : 0u;
        }
        __syncthreads();
    }

    uint32_t ev[4], rt[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t ei = e0 + ty * 4 + i;
        ev[i] = ei < a.n_cand ? a.cand[ei] : a.cand[0];
        const uint32_t ri = r0 + tx * 4 + i;
        rt[i] = ri < a.n_roots ? a.roots[ri] : LX_NONE;
    }

    uint32_t early = 0;   // bit i*4+k: A observes creator(branch(r)) as forked
    if (FORKS && bz == 0) {
        // Cheaters' branches: creator n counts once if any of its branches
        // counts (WeightCounter.CountByIdx, inter/pos/stake.go:47-55); the main
        // loop counted only the original column n.  Columns come grouped by
        // cheater, original first (kflag bit0 = first, bit1 = last).
        uint32_t orig = 0, acc = 0;
        for (uint32_t t = 0; t < a.n_k; t++) {
            const uint32_t j = a.kcol[t], fl = a.kflag[t];
            uint32_t cm = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t r = rt[k] == LX_NONE ? a.roots_fallback : rt[k];
                const uint32_t l = a.la[(uint64_t)r * a.stride + j] - 1u;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t h = hb_prep<true>(a.hb[(uint64_t)ev[i] * a.stride + j]);
                    cm |= (l < h ? 1u : 0u) << (i * 4 + k);
                }
            }
            if (fl & 1u) { orig = cm; acc = cm; } else acc |= cm;
            if (fl & 2u) {
                const uint32_t m = acc & ~orig, w = a.kw[t];
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int k = 0; k < 4; k++) sum[i][k] += ((m >> (i * 4 + k)) & 1u) ? w : 0u;
            }
        }
        // early false (forkless_cause.go:49-54)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (rt[k] == LX_NONE) continue;
            const uint32_t bb = a.ev_branch[rt[k]];
#pragma unroll
            for (int i = 0; i < 4; i++)
                early |= ((a.hb[(uint64_t)ev[i] * a.stride + bb] >> 31) & 1u) << (i * 4 + k);
        }
    }

    // partial stake sums of this column split; split 0 also carries the
    // cheater fix-ups and the early-false flag (bit 31: total weight < 2^31)
    const uint32_t rp = a.words * 32;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t ei = e0 + ty * 4 + i;
        if (ei >= a.n_cand) continue;
        uint4 o;
        o.x = sum[i][0] | (((early >> (i * 4 + 0)) & 1u) << 31);
        o.y = sum[i][1] | (((early >> (i * 4 + 1)) & 1u) << 31);
        o.z = sum[i][2] | (((early >> (i * 4 + 2)) & 1u) << 31);
        o.w = sum[i][3] | (((early >> (i * 4 + 3)) & 1u) << 31);
        const uint32_t ri = r0 + tx * 4;
        if (ri < rp)
            *reinterpret_cast<uint4 *>(a.psum + ((uint64_t)bz * a.n_cand + ei) * rp + ri) = o;
    }
}

// k_root_fc16: the fork-free k_root_fc for epochs whose seqs fit 16 bits
// (every HB and LA entry <= 0xFFFF).  Two columns share a dword in LDS and one
// packed subtract with unsigned saturation, one packed min and one 2-way dot
// product per weight half take a pair over two columns:
//   max(h - l', 0) != 0  <=>  l' < h      (l' = la - 1 in 16 bits: la = 0
//   never counts, as 0xFFFF < h is false for h <= 0xFFFF)
// min(., 1) is the 0/1 term, and dot2(term, {w_j, w_j+1}) adds the weights of
// both columns; weights >= 2^16 take a second dot2 on their high halves
// (uniform per LDS chunk: __syncthreads_or of the chunk's high halves).
// 1.5 VALU ops per (pair, column) with 16-bit weights, 2 otherwise, against 3
// (compare, select, add) in k_root_fc.
constexpr int kKp = kKc / 2;   // packed dwords per LDS chunk

typedef unsigned short lx_u16x2 __attribute__((ext_vector_type(2)));
// min against an opaque {1, 1}: with a literal one clang rewrites the
// saturating-sub + min pair into two compares and two selects per half
__device__ __forceinline__ uint32_t fc16_term(uint32_t h, uint32_t l, uint32_t ones) {
    const lx_u16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(lx_u16x2, h), __builtin_bit_cast(lx_u16x2, l));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, __builtin_bit_cast(lx_u16x2, ones)));
}

__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(lx_u16x2, a), __builtin_bit_cast(lx_u16x2, b), c, false);
}

template <bool MULTI>
__global__ __launch_bounds__(256) void k_root_fc16(RootFcArgs a1, const RootFcArgs *am, uint32_t n_steps) {
    uint32_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    const RootFcArgs a = MULTI ? fc_step(am, n_steps, &bx, &by, &bz) : a1;
    __shared__ uint32_t sH[kKp][kLdsPitch];
    __shared__ uint32_t sL[kKp][kLdsPitch];
    __shared__ uint32_t sWl[kKp], sWh[kKp];

    const uint32_t tid = threadIdx.x;
    const uint32_t tx = tid & 15, ty = tid >> 4;          // roots tx*4.., events ty*4..
    const uint32_t r0 = bx * kTile, e0 = by * kTile;

    // staging role: row = tid / 4, 8 columns = (tid % 4) * 8 -> 4 packed dwords
    const uint32_t srow = tid >> 2, spart = (tid & 3) * 8;
    const uint32_t se = e0 + srow < a.n_cand ? a.cand[e0 + srow] : a.cand[0];
    uint32_t sr = r0 + srow < a.n_roots ? a.roots[r0 + srow] : LX_NONE;
    if (sr == LX_NONE) sr = a.roots_fallback;
    const uint4 *hrow = reinterpret_cast<const uint4 *>(a.hb + (uint64_t)se * a.stride + spart);
    const uint4 *lrow = reinterpret_cast<const uint4 *>(a.la + (uint64_t)sr * a.stride + spart);

    uint32_t ones = 0x00010001u;
    asm("" : "+v"(ones));   // opaque (fc16_term)
    uint32_t lo[4][4], hi[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) lo[i][k] = hi[i][k] = 0;

    const uint32_t cs = a.col_split, jlo = bz * cs, jhi = jlo + cs < a.ncols ? jlo + cs : a.ncols;
    // the next chunk's rows are loaded into registers while this one computes
    uint4 h0 = hrow[jlo / 4], h1 = hrow[jlo / 4 + 1], l0 = lrow[jlo / 4], l1 = lrow[jlo / 4 + 1];
    uint32_t w0 = tid < kKp ? a.wpad[jlo + 2 * tid] : 0u, w1 = tid < kKp ? a.wpad[jlo + 2 * tid + 1] : 0u;
    for (uint32_t j0 = jlo; j0 < jhi; j0 += kKc) {
        {
            const uint32_t hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
            const uint32_t lv[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                sH[spart / 2 + q][srow] = hv[2 * q] | (hv[2 * q + 1] << 16);
                sL[spart / 2 + q][srow] = ((lv[2 * q] - 1u) & 0xFFFFu) | ((lv[2 * q + 1] - 1u) << 16);
            }
        }
        uint32_t wh = 0;
        if (tid < kKp) {
            sWl[tid] = (w0 & 0xFFFFu) | (w1 << 16);
            wh = (w0 >> 16) | (w1 & 0xFFFF0000u);
            sWh[tid] = wh;
        }
        const bool any_hi = __syncthreads_or(wh != 0);
        const uint32_t jn = j0 + kKc;
        if (jn < jhi) {
            h0 = hrow[jn / 4];
            h1 = hrow[jn / 4 + 1];
            l0 = lrow[jn / 4];
            l1 = lrow[jn / 4 + 1];
            if (tid < kKp) {
                w0 = a.wpad[jn + 2 * tid];
                w1 = a.wpad[jn + 2 * tid + 1];
            }
        }
        if (any_hi) {
#pragma unroll 4
            for (int j = 0; j < kKp; j++) {
                const uint4 h = *reinterpret_cast<const uint4 *>(&sH[j][ty * 4]);
                const uint4 l = *reinterpret_cast<const uint4 *>(&sL[j][tx * 4]);
                const uint32_t wl = sWl[j], wv = sWh[j];
                const uint32_t hh[4] = {h.x, h.y, h.z, h.w};
                const uint32_t ll[4] = {l.x, l.y, l.z, l.w};
uint32_t t[4][4];
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int k = 0; k < 4; k++) t[i][k] = fc16_term(hh[i], ll[k], ones);
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        lo[i][k] = udot2(t[i][k], wl, lo[i][k]);
                        hi[i][k] = udot2(t[i][k], wv, hi[i][k]);
                    }
            }
        } else {
#pragma unroll 4
            for (int j = 0; j < kKp; j++) {
                const uint4 h = *reinterpret_cast<const uint4 *>(&sH[j][ty * 4]);
                const uint4 l = *reinterpret_cast<const uint4 *>(&sL[j][tx * 4]);
                const uint32_t wl = sWl[j];
                const uint32_t hh[4] = {h.x, h.y, h.z, h.w};
                const uint32_t ll[4] = {l.x, l.y, l.z, l.w};
uint32_t t[4][4];
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int k = 0; k < 4; k++) t[i][k] = fc16_term(hh[i], ll[k], ones);
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int k = 0; k < 4; k++) lo[i][k] = udot2(t[i][k], wl, lo[i][k]);
            }
        }
        __syncthreads();
    }

    // partial stake sums of this column split (no cheaters, no early-false flag)
    const uint32_t rp = a.words * 32;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t ei = e0 + ty * 4 + i;
        if (ei >= a.n_cand) continue;
        uint4 o;
        o.x = lo[i][0] + (hi[i][0] << 16);
        o.y = lo[i][1] + (hi[i][1] << 16);
        o.z = lo[i][2] + (hi[i][2] << 16);
        o.w = lo[i][3] + (hi[i][3] << 16);
        const uint32_t ri = r0 + tx * 4;
        if (ri < rp)
            *reinterpret_cast<uint4 *>(a.psum + ((uint64_t)bz * a.n_cand + ei) * rp + ri) = o;
    }
}

uint32_t root_fc_splits(uint32_t n_cand, uint32_t n_roots, uint32_t ncols) {
    // enough workgroups to fill 256 CUs x 4, at least 4 LDS chunks per split
    const uint32_t tiles = ((n_roots + kTile - 1) / kTile) * ((n_cand + kTile - 1) / kTile);
    constexpr uint32_t target = 1024u;
    uint32_t s = tiles ? (target + tiles - 1) / tiles : 1;
    const uint32_t max_s = ncols / (4 * kKc) ? ncols / (4 * kKc) : 1;
    return s < 1 ? 1 : (s > max_s ? max_s : s);
}

hipError_t launch_root_fc(const RootFcArgs &a, bool forks, bool seq16, hipStream_t s) {
    if (!a.n_cand || !a.words) return hipSuccess;
    dim3 grid((a.n_roots + kTile - 1) / kTile, (a.n_cand + kTile - 1) / kTile, a.n_split);
    if (!forks && seq16) hipLaunchKernelGGL(k_root_fc16<false>, grid, dim3(256), 0, s, a, nullptr, 0);
    else if (forks) hipLaunchKernelGGL((k_root_fc<true, false>), grid, dim3(256), 0, s, a, nullptr, 0);
    else hipLaunchKernelGGL((k_root_fc<false, false>), grid, dim3(256), 0, s, a, nullptr, 0);
    return hipGetLastError();
}

uint32_t root_fc_blocks(const RootFcArgs &a) {
    if (!a.n_cand || !a.words) return 0;
    return ((a.n_roots + kTile - 1) / kTile) * ((a.n_cand + kTile - 1) / kTile) * a.n_split;
}

hipError_t launch_root_fc_multi(const RootFcArgs *am, uint32_t n_steps, uint32_t blocks, bool forks, bool seq16,
                                hipStream_t s) {
    if (!n_steps || !blocks) return hipSuccess;
    if (!forks && seq16) hipLaunchKernelGGL(k_root_fc16<true>, dim3(blocks), dim3(256), 0, s, RootFcArgs{}, am, n_steps);
    else if (forks) hipLaunchKernelGGL((k_root_fc<true, true>), dim3(blocks), dim3(256), 0, s, RootFcArgs{}, am, n_steps);
    else hipLaunchKernelGGL((k_root_fc<false, true>), dim3(blocks), dim3(256), 0, s, RootFcArgs{}, am, n_steps);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- k_root_quorum
// One wave per candidate: FC bit per root = (sum over the column splits >=
// quorum, no early-false flag), written to the bit row; then the stake of the
// distinct creators of the roots it forkless-causes (dup[r] = previous root of
// the same creator in the frame list), its own root slot excluded.
constexpr uint32_t kRowWords = 512;   // bit row kept in LDS: up to 16384 roots per frame
template <bool MULTI>
__global__ __launch_bounds__(256) void k_root_quorum(QuorumArgs a1, const QuorumArgs *am, uint32_t n_steps) {
    __shared__ uint32_t sRow[4][kRowWords];
    const QuorumArgs a = MULTI ? am[step_of(am, n_steps, blockIdx.x)] : a1;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x - (MULTI ? a.block0 : 0u)) * 4 + wv;
    if (wave >= a.n_cand) return;
    const uint32_t rp = a.words * 32;
    uint32_t *row = a.bits + (uint64_t)wave * a.words;
    for (uint32_t r0 = 0; r0 < rp; r0 += 64) {
        const uint32_t r = r0 + lane;
        uint32_t sum = 0;
        for (uint32_t z = 0; z < a.n_split; z++) sum += a.psum[((uint64_t)z * a.n_cand + wave) * rp + r];
        const bool ok = r < a.n_roots && !(sum >> 31) && sum >= a.quorum;
        const unsigned long long m = __ballot(ok);
        if (lane < 2 && r0 / 32 + lane < a.words) {
            const uint32_t w = (uint32_t)(m >> (32 * lane));
            row[r0 / 32 + lane] = w;
            sRow[wv][r0 / 32 + lane] = w;
        }
    }
    __syncthreads();   // sRow of this wave complete (waves of a block exit together below)
    const uint32_t self = a.cand[wave];
    uint32_t sum = 0;
    for (uint32_t wi = lane; wi < a.words; wi += 64) {
        uint32_t m = sRow[wv][wi];
        while (m) {
            const uint32_t b = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t r = wi * 32 + b;
            // calcFrameIdx runs before AddRoot (event_processing.go:52-60):
            // an event never counts its own root slot of this frame
            if (a.root_ev[r] == self) continue;
            bool first = true;
            for (uint32_t d = a.dup[r]; d != LX_NONE; d = a.dup[d])
                if ((sRow[wv][d >> 5] >> (d & 31)) & 1u) { first = false; break; }
            if (first) sum += a.wcreator[a.creator[r]];
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    if (lane == 0) a.q[wave] = sum >= a.quorum ? 1 : 0;
}

hipError_t launch_root_quorum(const QuorumArgs &a, hipStream_t s) {
    if (!a.n_cand) return hipSuccess;
    hipLaunchKernelGGL(k_root_quorum<false>, dim3((a.n_cand + 3) / 4), dim3(256), 0, s, a, nullptr, 0);
    return hipGetLastError();
}

hipError_t launch_root_quorum_multi(const QuorumArgs *am, uint32_t n_steps, uint32_t blocks, hipStream_t s) {
    if (!n_steps || !blocks) return hipSuccess;
    hipLaunchKernelGGL(k_root_quorum<true>, dim3(blocks), dim3(256), 0, s, QuorumArgs{}, am, n_steps);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- k_fc_tile_out
// ForklessCause answers of a whole k_root_fc launch as bytes (the per-pair
// result cache, lx_fccache.cpp): out[c * pitch + r] = tag[r] << 1 | FC(cand c,
// root r), FC = (sum over the column splits >= quorum, no early-false flag).
__global__ __launch_bounds__(256) void k_fc_tile_out(const uint32_t *psum, uint32_t n_split, uint32_t n_cand,
                                                     uint32_t rp, uint32_t n_roots, uint32_t quorum, const uint8_t *tag,
                                                     uint8_t *out, uint64_t pitch) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
    if (r >= n_roots || c >= n_cand) return;
    uint32_t sum = 0;
    for (uint32_t z = 0; z < n_split; z++) sum += psum[((uint64_t)z * n_cand + c) * rp + r];
    const uint32_t ok = !(sum >> 31) && sum >= quorum;
    out[(uint64_t)c * pitch + r] = (uint8_t)(tag[r] << 1 | ok);
}

hipError_t launch_fc_tile_out(const uint32_t *psum, uint32_t n_split, uint32_t n_cand, uint32_t rp, uint32_t n_roots,
                              uint32_t quorum, const uint8_t *tag, uint8_t *out, uint64_t pitch, hipStream_t s) {
    if (!n_cand || !n_roots) return hipSuccess;
    hipLaunchKernelGGL(k_fc_tile_out, dim3((n_roots + 255) / 256, n_cand), dim3(256), 0, s, psum, n_split, n_cand, rp,
                       n_roots, quorum, tag, out, pitch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- votes
// vote word: bit31 voted, bit30 yes, bit29 decided, bits 0..28 observed root
// (index into the frame-to-decide's root list; kVoteNoRoot = none).
// Votes of different subjects never mix (election_math.go:53-110 reads only
// votes for the same subject), so each launch computes a subject window
// [v_lo, v_hi); the host widens the window only while chooseAtropos needs it.
// MULTI: one launch for many (election, round) tables, args am[blockIdx.y]
// (init) / am[blockIdx.z] (rounds), each with its own n_voters.
template <bool MULTI>
__global__ void k_vote_init(VoteArgs a1, const VoteArgs *am) {
    const VoteArgs &a = MULTI ? am[blockIdx.y] : a1;
    const uint32_t w = a.v_hi - a.v_lo;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (uint64_t)a.n_voters * w)
        a.votes[(i / w) * a.V + a.v_lo + i % w] = kVoteVoted | kVoteNoRoot;
}

// round 1 (election_math.go:40-52): yes iff the voter forkless-causes the
// subject's root of the frame to decide; observedRootsMap keeps the last root
// of a validator in list order -> atomicMax over the list index.
template <bool MULTI>
__global__ void k_vote_round1(VoteArgs a1, const VoteArgs *am) {
    const VoteArgs &a = MULTI ? am[blockIdx.z] : a1;
    const uint32_t s = blockIdx.y;
    if (s >= a.n_voters) return;
    if (a.voter_ev[s] == LX_NONE) return;
    const uint64_t off = a.bm_off[s];
    const uint32_t len = a.bm_len[s];
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < len; r += gridDim.x * blockDim.x) {
        if (!((a.bm[off + (r >> 5)] >> (r & 31)) & 1u)) continue;
        const uint32_t c = a.prev_creator[r];
        if (c < a.v_lo || c >= a.v_hi) continue;
        atomicMax(&a.votes[(uint64_t)s * a.V + c], kVoteVoted | kVoteYes | r);
    }
}

// round >= 2 (election_math.go:53-110): one workgroup per voter slot.  The
// voter's observed roots are compacted into LDS; 4 waves split them, each
// lane sums one subject of the 64-subject chunk over its wave's share (loads
// independent, so many are in flight), then the 4 partial tallies merge.
constexpr int kVoteSlices = 4;
constexpr uint32_t kObsChunk = 2048;   // observed-root bits compacted per pass
template <bool MULTI>
__global__ __launch_bounds__(256) void k_vote_round(VoteArgs a1, const VoteArgs *am) {
    const VoteArgs &a = MULTI ? am[blockIdx.z] : a1;
    if (blockIdx.y >= a.n_voters) return;   // the whole workgroup: before any barrier
    __shared__ uint32_t sObs[kObsChunk];
    __shared__ uint32_t sWc[kObsChunk];   // stake of each observed root's creator
    __shared__ uint32_t sN;
    __shared__ uint32_t sYes[kVoteSlices][64], sNo[kVoteSlices][64], sAll[kVoteSlices][64], sSubj[kVoteSlices][64],
        sErr[kVoteSlices][64];
    const uint32_t s = blockIdx.y;
    const uint32_t lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
    const uint32_t vev = a.voter_ev[s];
    if (vev == LX_NONE) return;
    const uint64_t off = a.bm_off[s];
    const uint32_t len = a.bm_len[s];
    if (a.prev_has_dup && blockIdx.x == 0) {
        // two observed roots of one validator: allVotes.Count == false
        uint32_t err = 0;
        for (uint32_t r = threadIdx.x; r < len; r += blockDim.x) {
            if (!((a.bm[off + (r >> 5)] >> (r & 31)) & 1u)) continue;
            for (uint32_t d = a.prev_dup[r]; d != LX_NONE; d = a.prev_dup[d])
                if ((a.bm[off + (d >> 5)] >> (d & 31)) & 1u) err |= kVoteErrTwoRoots;
        }
        if (err) atomicOr(a.err, err);
    }
    for (uint32_t v0 = a.v_lo + blockIdx.x * 64; v0 < a.v_hi; v0 += gridDim.x * 64) {
        const uint32_t v = v0 + lane;
        uint32_t yes = 0, no = 0, all = 0, subj = kVoteNoRoot, err = 0;
        for (uint32_t c0 = 0; c0 < len; c0 += kObsChunk) {
            // compact this chunk's observed roots (bit order = root list order)
            if (threadIdx.x == 0) sN = 0;
            __syncthreads();
            const uint32_t clen = len - c0 < kObsChunk ? len - c0 : kObsChunk;
            for (uint32_t wi = threadIdx.x; wi * 32 < clen; wi += blockDim.x) {
                uint32_t m = a.bm[off + c0 / 32 + wi];
                if ((wi + 1) * 32 > clen) m &= (1u << (clen & 31)) - 1u;
                uint32_t base = m ? atomicAdd(&sN, (uint32_t)__builtin_popcount(m)) : 0;
                while (m) {
                    sObs[base++] = c0 + wi * 32 + __builtin_ctz(m);
                    m &= m - 1;
                }
            }
            __syncthreads();
            const uint32_t n = sN;
            // creator stakes of the observed roots, all threads at once (the
            // subject loop below then reads one global word per root: the vote)
            for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) sWc[k] = a.wcreator[a.prev_creator[sObs[k]]];
            __syncthreads();
            if (v < a.v_hi) {
#pragma unroll 8
                for (uint32_t k = slice; k < n; k += kVoteSlices) {
                    const uint32_t r = sObs[k];
                    const uint32_t pv = a.prev_votes[(uint64_t)r * a.V + v];
                    const uint32_t wc = sWc[k];
                    if (!(pv & kVoteVoted)) err |= kVoteErrMissing;
                    const bool py = (pv & kVoteYes) != 0;
                    const uint32_t ix = pv & kVoteNoRoot;
                    if (py && subj != kVoteNoRoot && subj != ix) err |= kVoteErrTwoRoots;
                    subj = py ? ix : subj;
                    yes += py ? wc : 0u;
                    no += py ? 0u : wc;
                    all += wc;
                }
            }
            __syncthreads();
        }
        sYes[slice][lane] = yes;
        sNo[slice][lane] = no;
        sAll[slice][lane] = all;
        sSubj[slice][lane] = subj;
        sErr[slice][lane] = err;
        __syncthreads();
        if (slice == 0 && v < a.v_hi) {
            for (int q = 1; q < kVoteSlices; q++) {
                yes += sYes[q][lane];
                no += sNo[q][lane];
                all += sAll[q][lane];
                err |= sErr[q][lane];
                const uint32_t sq = sSubj[q][lane];
                if (sq != kVoteNoRoot) {
                    if (subj != kVoteNoRoot && subj != sq) err |= kVoteErrTwoRoots;
                    subj = sq;
                }
            }
            if (all < a.quorum) err |= kVoteErrQuorum;
            const bool y = yes >= no;
            const bool dec = yes >= a.quorum || no >= a.quorum;
            const uint32_t obs = y ? subj : kVoteNoRoot;
            a.votes[(uint64_t)s * a.V + v] = kVoteVoted | (y ? kVoteYes : 0u) | (dec ? kVoteDecided : 0u) | obs;
            if (dec) atomicMin(&a.dec[v], ((unsigned long long)vev << 32) | (y ? 0x80000000ull : 0ull) | obs);
            if (err) atomicOr(a.err, err);
        }
        __syncthreads();
    }
}

hipError_t launch_votes(const VoteArgs &a0, uint32_t n_voters, bool round1, hipStream_t s) {
    if (!n_voters || a0.v_hi <= a0.v_lo) return hipSuccess;
    VoteArgs a = a0;
    a.n_voters = n_voters;
    const uint32_t w = a.v_hi - a.v_lo;
    const uint64_t n = (uint64_t)n_voters * w;
    hipLaunchKernelGGL(k_vote_init<false>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, a, nullptr);
    if (round1) {
        hipLaunchKernelGGL(k_vote_round1<false>, dim3(2, n_voters), dim3(256), 0, s, a, nullptr);
    } else {
        const uint32_t gx = (w + 63) / 64 < 16 ? (w + 63) / 64 : 16;
        hipLaunchKernelGGL(k_vote_round<false>, dim3(gx, n_voters), dim3(256), 0, s, a, nullptr);
    }
    return hipGetLastError();
}

// n tables of one round kind in one launch each: args am[0, n) on the device
// (n_voters set per table, max_voters = the largest, w = every table's window)
hipError_t launch_votes_multi(const VoteArgs *am, uint32_t n, uint32_t max_voters, uint32_t w, bool round1,
                              hipStream_t s) {
    if (!n || !max_voters || !w) return hipSuccess;
    const uint64_t cells = (uint64_t)max_voters * w;
    hipLaunchKernelGGL(k_vote_init<true>, dim3((uint32_t)((cells + 255) / 256), n), dim3(256), 0, s, VoteArgs{}, am);
    if (round1) {
        hipLaunchKernelGGL(k_vote_round1<true>, dim3(2, max_voters, n), dim3(256), 0, s, VoteArgs{}, am);
    } else {
        const uint32_t gx = (w + 63) / 64 < 16 ? (w + 63) / 64 : 16;
        hipLaunchKernelGGL(k_vote_round<true>, dim3(gx, max_voters, n), dim3(256), 0, s, VoteArgs{}, am);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- k_scatter
// The host-to-device uploads of one abft step in one launch: descriptors and
// data sit in one pinned, device-mapped staging slot (read once over the bus);
// workgroup (i, c) copies words [c*1024, c*1024+1024) of segment i (4-byte
// words; every upload is a uint32 or uint64 array).  Every word is read by its
// own load and the four loads of a thread are issued before any store, so the
// whole launch waits about one bus round trip, not one per 256 words.
constexpr uint32_t kScatterChunk = 1024;

__global__ __launch_bounds__(256) void k_scatter(const ScatterDesc *d, const uint8_t *base) {
    const ScatterDesc x = d[blockIdx.x];
    const uint32_t *src = reinterpret_cast<const uint32_t *>(base + x.src_off);
    uint32_t *dst = reinterpret_cast<uint32_t *>(x.dst);
    const uint64_t nw = x.bytes / 4, w0 = (uint64_t)blockIdx.y * kScatterChunk + threadIdx.x;
    if (w0 >= nw) return;
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = w0 + u * 256 < nw ? src[w0 + u * 256] : 0u;
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (w0 + u * 256 < nw) dst[w0 + u * 256] = v[u];
}

hipError_t launch_scatter(const ScatterDesc *desc, uint32_t n, uint64_t max_bytes, const uint8_t *base,
                          hipStream_t s) {
    if (!n || !max_bytes) return hipSuccess;
    const uint64_t chunks = (max_bytes / 4 + kScatterChunk - 1) / kScatterChunk;
    if (chunks > 65535) return hipErrorInvalidValue;   // 256 MB per upload: far beyond any abft step
    hipLaunchKernelGGL(k_scatter, dim3(n, (uint32_t)chunks), dim3(256), 0, s, desc, base);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- k_readback
// Small device results (decision words, error flags, one HB row) written
// straight into pinned, device-mapped host memory: one launch instead of a
// blit copy per array through a pageable staging buffer.
__global__ __launch_bounds__(256) void k_readback(uint32_t *dst, const uint32_t *a, uint32_t na, const uint32_t *b,
                                                  uint32_t nb) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < na) dst[i] = a[i];
    else if (i < na + nb) dst[i] = b[i - na];
}

hipError_t launch_readback(uint32_t *dst, const uint32_t *a, uint32_t na, const uint32_t *b, uint32_t nb,
                           hipStream_t s) {
    const uint32_t n = na + nb;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_readback, dim3((n + 255) / 256), dim3(256), 0, s, dst, a, na, b, nb);
    return hipGetLastError();
}

// Rows src[row[k]] (V words each) into dst[k * V] -- the Atropos HB rows of
// the elections decided ahead, written into pinned, device-mapped memory.
constexpr uint32_t kGatherRows = 64;
struct RowList {
    uint32_t row[kGatherRows];
};

__global__ __launch_bounds__(256) void k_gather_rows(uint32_t *dst, const uint32_t *src, uint64_t stride, uint32_t V,
                                                     RowList l) {
    const uint32_t k = blockIdx.y;
    for (uint32_t c = blockIdx.x * 256 + threadIdx.x; c < V; c += gridDim.x * 256)
        dst[(uint64_t)k * V + c] = src[(uint64_t)l.row[k] * stride + c];
}

hipError_t launch_gather_rows(uint32_t *dst, const uint32_t *src, uint64_t stride, uint32_t V, const uint32_t *rows,
                              uint32_t n, hipStream_t s) {
    for (uint32_t k0 = 0; k0 < n; k0 += kGatherRows) {
        RowList l{};
        const uint32_t m = n - k0 < kGatherRows ? n - k0 : kGatherRows;
        for (uint32_t k = 0; k < m; k++) l.row[k] = rows[k0 + k];
        const uint32_t gx = (V + 255) / 256 < 4 ? (V + 255) / 256 : 4;
        hipLaunchKernelGGL(k_gather_rows, dim3(gx ? gx : 1, m), dim3(256), 0, s, dst + (uint64_t)k0 * V, src, stride, V,
                           l);
    }
    return hipGetLastError();
}

}  // namespace lx
