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

// fc_term of k_fc in staged form: (la - 1) < hb'  <=>  la != 0 && la <= hb
template <bool FORKS>
__global__ __launch_bounds__(256) void k_root_fc(RootFcArgs a) {
    __shared__ uint32_t sH[kKc][kLdsPitch];
    __shared__ uint32_t sL[kKc][kLdsPitch];
    __shared__ uint32_t sW[kKc];
    __shared__ uint32_t sBits[kTile][2];

    const uint32_t tid = threadIdx.x;
    const uint32_t tx = tid & 15, ty = tid >> 4;          // roots tx*4.., events ty*4..
    const uint32_t r0 = blockIdx.x * kTile, e0 = blockIdx.y * kTile;

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

    for (uint32_t j0 = 0; j0 < a.ncols; j0 += kKc) {
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
    if (FORKS) {
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

    if (tid < kTile * 2) sBits[tid >> 1][tid & 1] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t nib = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool ok = rt[k] != LX_NONE && !((early >> (i * 4 + k)) & 1u) && sum[i][k] >= a.quorum;
            nib |= (ok ? 1u : 0u) << k;
        }
        if (nib) atomicOr(&sBits[ty * 4 + i][tx >> 3], nib << ((tx & 7) * 4));
    }
    __syncthreads();
    if (tid < kTile * 2) {
        const uint32_t ei = e0 + (tid >> 1);
        const uint32_t wi = blockIdx.x * 2 + (tid & 1);
        if (ei < a.n_cand && wi < a.words) a.bits[(uint64_t)ei * a.words + wi] = sBits[tid >> 1][tid & 1];
    }
}

hipError_t launch_root_fc(const RootFcArgs &a, bool forks, hipStream_t s) {
    if (!a.n_cand || !a.words) return hipSuccess;
    dim3 grid((a.n_roots + kTile - 1) / kTile, (a.n_cand + kTile - 1) / kTile);
    if (grid.x == 0) grid.x = 1;   // no roots: rows of zeros still get written
    if (forks) hipLaunchKernelGGL(k_root_fc<true>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_root_fc<false>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- k_root_quorum
// one wave per candidate; roots with a set bit count their creator once
// (dup[r] = previous root of the same creator in the frame list, or NONE)
__global__ __launch_bounds__(256) void k_root_quorum(QuorumArgs a) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
    if (wave >= a.n_cand) return;
    const uint32_t *row = a.bits + (uint64_t)wave * a.words;
    const uint32_t self = a.cand[wave];
    uint32_t sum = 0;
    for (uint32_t wi = lane; wi < a.words; wi += 64) {
        uint32_t m = row[wi];
        while (m) {
            const uint32_t b = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t r = wi * 32 + b;
            // calcFrameIdx runs before AddRoot (event_processing.go:52-60):
            // an event never counts its own root slot of this frame
            if (a.root_ev[r] == self) continue;
            bool first = true;
            for (uint32_t d = a.dup[r]; d != LX_NONE; d = a.dup[d])
                if ((row[d >> 5] >> (d & 31)) & 1u) { first = false; break; }
            if (first) sum += a.wcreator[a.creator[r]];
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    if (lane == 0) a.q[wave] = sum >= a.quorum ? 1 : 0;
}

hipError_t launch_root_quorum(const QuorumArgs &a, hipStream_t s) {
    if (!a.n_cand) return hipSuccess;
    hipLaunchKernelGGL(k_root_quorum, dim3((a.n_cand + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- votes
// vote word: bit31 voted, bit30 yes, bit29 decided, bits 0..28 observed root
// (index into the frame-to-decide's root list; kVoteNoRoot = none).
// Votes of different subjects never mix (election_math.go:53-110 reads only
// votes for the same subject), so each launch computes a subject window
// [v_lo, v_hi); the host widens the window only while chooseAtropos needs it.
__global__ void k_vote_init(VoteArgs a, uint32_t n_voters) {
    const uint32_t w = a.v_hi - a.v_lo;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (uint64_t)n_voters * w)
        a.votes[(i / w) * a.V + a.v_lo + i % w] = kVoteVoted | kVoteNoRoot;
}

// round 1 (election_math.go:40-52): yes iff the voter forkless-causes the
// subject's root of the frame to decide; observedRootsMap keeps the last root
// of a validator in list order -> atomicMax over the list index.
__global__ void k_vote_round1(VoteArgs a) {
    const uint32_t s = blockIdx.y;
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

// round >= 2 (election_math.go:53-110): one lane per (voter slot, subject),
// a wave = 64 subjects of one voter, so the voter's observed-root bitmap and
// the observed root's creator and weight are wave-uniform.
__global__ __launch_bounds__(256) void k_vote_round(VoteArgs a, uint32_t n_voters) {
    const uint32_t s = blockIdx.y * 4 + threadIdx.y;
    const uint32_t v = a.v_lo + blockIdx.x * 64 + threadIdx.x;
    if (s >= n_voters) return;
    const uint32_t vev = a.voter_ev[s];
    if (vev == LX_NONE || v >= a.v_hi) return;
    const uint64_t off = a.bm_off[s];
    const uint32_t len = a.bm_len[s];
    uint32_t yes = 0, no = 0, all = 0, subj = kVoteNoRoot, err = 0;
    for (uint32_t wi = 0; wi * 32 < len; wi++) {
        uint32_t m = a.bm[off + wi];
        if ((wi + 1) * 32 > len) m &= (1u << (len & 31)) - 1u;
        while (m) {
            const uint32_t b = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t r = wi * 32 + b;
            const uint32_t c = a.prev_creator[r];
            if (a.prev_has_dup)
                for (uint32_t d = a.prev_dup[r]; d != LX_NONE; d = a.prev_dup[d])
                    if ((a.bm[off + (d >> 5)] >> (d & 31)) & 1u) err |= kVoteErrTwoRoots;   // allVotes.Count == false
            const uint32_t pv = a.prev_votes[(uint64_t)r * a.V + v];
            const uint32_t wc = a.wcreator[c];
            if (!(pv & kVoteVoted)) err |= kVoteErrMissing;
            if (pv & kVoteYes) {
                const uint32_t ix = pv & kVoteNoRoot;
                if (subj != kVoteNoRoot && subj != ix) err |= kVoteErrTwoRoots;
                subj = ix;
                yes += wc;
            } else {
                no += wc;
            }
            all += wc;
        }
    }
    if (all < a.quorum) err |= kVoteErrQuorum;
    const bool y = yes >= no;
    const bool dec = yes >= a.quorum || no >= a.quorum;
    const uint32_t obs = y ? subj : kVoteNoRoot;
    a.votes[(uint64_t)s * a.V + v] = kVoteVoted | (y ? kVoteYes : 0u) | (dec ? kVoteDecided : 0u) | obs;
    if (dec)
        atomicMin(&a.dec[v], ((unsigned long long)vev << 32) | (y ? 0x80000000ull : 0ull) | obs);
    if (err) atomicOr(a.err, err);
}

hipError_t launch_votes(const VoteArgs &a, uint32_t n_voters, bool round1, hipStream_t s) {
    if (!n_voters || a.v_hi <= a.v_lo) return hipSuccess;
    const uint32_t w = a.v_hi - a.v_lo;
    const uint64_t n = (uint64_t)n_voters * w;
    hipLaunchKernelGGL(k_vote_init, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, a, n_voters);
    if (round1) {
        hipLaunchKernelGGL(k_vote_round1, dim3(2, n_voters), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_vote_round, dim3((w + 63) / 64, (n_voters + 3) / 4), dim3(64, 4), 0, s, a, n_voters);
    }
    return hipGetLastError();
}

}  // namespace lx
