// kern_fast.hip — the N = 64 FAST consensus kernel (bft_fast64.h) and the block-hash pass
// (bft_hash_suffix_kernel / bft_hash_suffix_loop_kernel + bft_hash_chain_kernel) of the benchmark workload.
#include "bft_hip.h"
#include "bft_fast64.h"

namespace bft {

// FAST kernel (N = 64, big-endian seeds): the closed-form phases only (bft_fast64.h); instances
// needing the general path are saved for the resume kernel
#ifndef BFT_FAST_WAVES_PER_SIMD
#define BFT_FAST_WAVES_PER_SIMD 4   // 110 VGPRs, no scratch; since the canonical tick 4, 5 and 6 (80 VGPRs, 76-88 B/lane of spills) measure the same (profiles/r04/ab_occupancy)
#endif
// the lossless build (cfg3): 4 waves (110 VGPRs, no scratch). At 5 (96 VGPRs, 28 B/lane spilled: one reload per
// canonical tick) a third FAST wave fits a SIMD beside one predicted-lane chain wave: +2.3 % on cfg3 in interleaved
// pairs (2.13e9-2.20e9 against 2.08e9-2.13e9, profiles/r06/ab_fast_waves), within the box-to-box spread; kept at 4
#ifndef BFT_FAST_LOSSLESS_WAVES_PER_SIMD
#define BFT_FAST_LOSSLESS_WAVES_PER_SIMD 4
#endif
#ifndef BFT_FAST_SEEDED_WAVES_PER_SIMD
#define BFT_FAST_SEEDED_WAVES_PER_SIMD 4   // the in-kernel wave hash needs registers: 5 spills to scratch (gpurun r03c: 4 waves +6 %)
#endif
template <bool LOSSY, bool SEEDED>
__global__ __launch_bounds__(64, SEEDED ? BFT_FAST_SEEDED_WAVES_PER_SIMD
                                        : LOSSY ? BFT_FAST_WAVES_PER_SIMD : BFT_FAST_LOSSLESS_WAVES_PER_SIMD)
void bft_consensus_fast_kernel(Params p) {
    extern __shared__ uint8_t lds[];
#ifndef BFT_CONSENSUS_PRIO
#define BFT_CONSENSUS_PRIO 2
#endif
    // win issue arbitration against the hash waves of the previous launch (the hash pass stretches into
    // the issue gaps and still finishes within the step); s_setprio takes an immediate
    if (p.fast_prio == 0u) __builtin_amdgcn_s_setprio(BFT_CONSENSUS_PRIO);
    else if (p.fast_prio == 1u) __builtin_amdgcn_s_setprio(0);
    else if (p.fast_prio == 2u) __builtin_amdgcn_s_setprio(1);
    else if (p.fast_prio == 3u) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
    Fast64<WaveHip, LOSSY, SEEDED> sim(p, lds, blockIdx.x);
    sim.run();
}
hipError_t launch_fast(dim3 grid, hipStream_t s, const Params& p) {
    // the lossless build for schedules without drops and proposer crashes (cfg3): masks are constants;
    // SEEDED (little-endian seeds): the proposer follows the block hashes, computed in-kernel
    const bool lossy = !(p.thr16 == 0 && p.crash_on == 0), seeded = p.need_seed != 0;
    const size_t lds = lds_bytes_fast64(seeded) + p.fast_lds_pad;   // the pad: A/B arms of FAST residency only
    if (seeded) {
        if (lossy) hipLaunchKernelGGL((bft_consensus_fast_kernel<true, true>), grid, dim3(64), lds, s, p);
        else hipLaunchKernelGGL((bft_consensus_fast_kernel<false, true>), grid, dim3(64), lds, s, p);
    } else {
        if (lossy) hipLaunchKernelGGL((bft_consensus_fast_kernel<true, false>), grid, dim3(64), lds, s, p);
        else hipLaunchKernelGGL((bft_consensus_fast_kernel<false, false>), grid, dim3(64), lds, s, p);
    }
    return hipGetLastError();
}

// one lane PAIR per instance: the even lane holds the low 32-bit half of every
// Keccak state word, the odd lane the high half. A 64-bit rotation is one v_alignbit_b32 of this
// lane's half and the partner's (exchanged with one DPP quad_perm swap); theta parities, chi and iota
// are half-local. Per lane and round ~125 VALU instead of ~205 for a whole state in one lane, and
// twice the waves for the chip. The chains are sequential in height and a lone wave issues one VALU
// per ~4 cycles, so the pass is bound by its per-chain issue latency: the pair halves it. (A whole
// state per lane has ~27 % fewer vector instructions per header; it was the large-shard choice while
// the consensus kernel took longer than its 2.25 ms latency, and lost 18 % once it did not:
// profiles/r03/ab_hash.)
#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline uint32_t pair_swap(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
}
template <int N>
__device__ inline uint32_t rotl_pair(uint32_t mine, uint32_t other) {
    if constexpr (N == 0) return mine;
    else if constexpr (N == 32) return other;
    else if constexpr (N < 32) return __builtin_amdgcn_alignbit(mine, other, 32 - N);
    else return __builtin_amdgcn_alignbit(other, mine, 64 - N);
}
__constant__ uint32_t KECCAK_RC_PAIR[2][24] = {
    {0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u, 0x80008081u, 0x00008009u,
     0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au, 0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
     0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u},
    {0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0x80000000u,
     0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u}};

// The 24 rounds fully unrolled (default): round constants become per-round constants instead of a per-lane load
// from constant memory waited for in every round, and the rounds schedule into each other: cfg3 +5 %,
// 2,048 per GPU +10 % (profiles/r04/ab_pair_unroll/). BFT_PAIR_UNROLL=1: the round loop (A/B arm).
#ifndef BFT_PAIR_UNROLL
#define BFT_PAIR_UNROLL 24
#endif
__device__ inline void keccak_f1600_pair(uint32_t X[25], uint32_t odd) {
#if BFT_PAIR_UNROLL > 1
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int rnd = 0; rnd < 24; ++rnd) {
        uint32_t c[5], cs[5], r1[5], t[25], b[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) c[x] = xor3_32(xor3_32(X[x], X[x + 5], X[x + 10]), X[x + 15], X[x + 20]);
#pragma unroll
        for (int x = 0; x < 5; ++x) cs[x] = pair_swap(c[x]);
#pragma unroll
        for (int x = 0; x < 5; ++x) r1[x] = rotl_pair<1>(c[(x + 1) % 5], cs[(x + 1) % 5]);
        // theta's D folded into one 3-input XOR per word (X ^ C[x-1] ^ rot(C[x+1])): 25 v_bitop3 instead of 5 + 25 XORs
#pragma unroll
        for (int i = 0; i < 25; ++i) t[i] = xor3_32(X[i], c[(i % 5 + 4) % 5], r1[i % 5]);
        // rho + pi: b[y + 5*((2x+3y)%5)] = rotl(t[x+5y], r[x+5y])
#define BFT_RHO2(i, n, j) b[j] = rotl_pair<n>(t[i], (n) ? pair_swap(t[i]) : 0u);
        BFT_RHO2(0, 0, 0) BFT_RHO2(1, 1, 10) BFT_RHO2(2, 62, 20) BFT_RHO2(3, 28, 5) BFT_RHO2(4, 27, 15)
        BFT_RHO2(5, 36, 16) BFT_RHO2(6, 44, 1) BFT_RHO2(7, 6, 11) BFT_RHO2(8, 55, 21) BFT_RHO2(9, 20, 6)
        BFT_RHO2(10, 3, 7) BFT_RHO2(11, 10, 17) BFT_RHO2(12, 43, 2) BFT_RHO2(13, 25, 12) BFT_RHO2(14, 39, 22)
        BFT_RHO2(15, 41, 23) BFT_RHO2(16, 45, 8) BFT_RHO2(17, 15, 18) BFT_RHO2(18, 21, 3) BFT_RHO2(19, 8, 13)
        BFT_RHO2(20, 18, 14) BFT_RHO2(21, 2, 24) BFT_RHO2(22, 61, 9) BFT_RHO2(23, 56, 19) BFT_RHO2(24, 14, 4)
#undef BFT_RHO2
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x)
                X[5 * y + x] = b[5 * y + x] ^ (~b[5 * y + (x + 1) % 5] & b[5 * y + (x + 2) % 5]);
        if (BFT_PAIR_UNROLL > 1) X[0] ^= odd ? KECCAK_RC_HI[rnd] : KECCAK_RC_LO[rnd];   // unrolled: constants
        else X[0] ^= KECCAK_RC_PAIR[odd][rnd];
    }
}

#endif

// The pass is split in two kernels so that the sequential chains carry only what chains: prev_hash.
// 1. bft_hash_suffix_kernel, one thread per (instance, height): the header bytes after prev_hash
//    (proposer address, the seeded tx_hash's two Philox draws, height, time, ...) into a suffix row
//    (bft_common.h header_suffix_strided). Fully parallel: a short full-chip pass (bftsim.hip decides
//    where it runs; beside long general kernels, bft_hash_suffix_loop_kernel: a thread per instance).
// 2. bft_hash_chain_kernel, a lane pair per instance: per height, encode prev_hash (36..68 bytes), splice
//    the suffix behind it with one v_alignbyte per message dword (splice_word; the suffix row is in LDS,
//    loaded one height ahead), absorb, permute. Both lanes used to run the whole encoder.
__device__ inline void suffix_row(const Params& p, uint32_t il, uint32_t j) {
    const uint32_t n = p.n_instances, x = p.sfx_x0 + j;
    const uint4 row = *(const uint4*)(p.rec + ((uint64_t)il * p.rows + x) * 4);
    const uint32_t prop = row.y & 0xffffu, var = (row.y >> 16) & 1u;
    const uint64_t time = p.genesis_time + (uint64_t)p.block_period * ((uint64_t)row.z + 1ull);
    header_suffix_strided(p.sfx + (uint64_t)j * SFX_DEV_DW * n + il, n, p.addresses + 20u * prop, p.seed,
                          p.first_instance + il, x, prop, var, time);
}
__global__ __launch_bounds__(256) void bft_hash_suffix_kernel(Params p) {
    const uint32_t K = p.sfx_rows;
    const uint32_t n = p.n_instances;
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;  // n * rows < 2^32 (bftsim.hip)
    const uint32_t j = t / n, il = t - j * n;           // consecutive threads: consecutive instances
    if (j >= K) return;
    if (p.sfx_x0 + j > p.committed_height[il]) return;
    suffix_row(p, il, j);
}
// the same rows with a thread per instance over its heights: few waves, run on the hash stream beside
// the consensus kernels (large shards; launch_hash_suffix)
__global__ __launch_bounds__(256) void bft_hash_suffix_loop_kernel(Params p) {
    const uint32_t il = blockIdx.x * 256u + threadIdx.x;
    if (il >= p.n_instances) return;
    const uint32_t ch = p.committed_height[il];
    for (uint32_t j = 0; j < p.sfx_rows && p.sfx_x0 + j <= ch; ++j) suffix_row(p, il, j);
}

// LDS of a chain block (one wave, 32 lane pairs): per pair a splice buffer and the prefix. Compact (an A/B arm,
// -DBFT_CHAIN_COMPACT=1): the splice buffer stops after the suffix body plus one zero dword that every read past
// the body is clamped to (only a 3-block header's last block reads there), and the two lanes of a pair share one
// prefix buffer (they compute the same words): 13.7 KB per block instead of 21.1 KB, 3 chain waves per SIMD
// instead of 2. Measured 2-4 % slower at every shard size (profiles/r04/ab_chain_lds): more resident chain waves
// only take issue slots from the consensus kernels beside them.
#ifndef BFT_CHAIN_COMPACT
#define BFT_CHAIN_COMPACT 0
#endif
constexpr uint32_t CHAIN_SB = BFT_CHAIN_COMPACT ? 80u : SFX_BUF;        // splice buffer dwords per pair
constexpr uint32_t CHAIN_SB_ZERO = SFX_PAD + SFX_BODY_DW;              // a zero dword (compact: reads past it clamp here)
[[maybe_unused]] constexpr uint32_t CHAIN_PB_SLOTS = BFT_CHAIN_COMPACT ? 32u : 64u;      // prefix buffers per block
static_assert(CHAIN_SB > CHAIN_SB_ZERO && CHAIN_SB % 4u == 0u, "splice buffer layout");

#if defined(__HIP_DEVICE_COMPILE__)
// A lane pair's header hash: absorb the header spliced from the prefix (this lane's dwords `pw`, len_p
// bytes) and the suffix in the pair's splice buffer `sb` (len_s bytes), permute; `prev` <- the hash (both
// lanes: 8 words), `dst` <- this lane's four words of it.
__device__ inline void pair_header_hash(const uint32_t* sb, const uint32_t* pw, uint32_t odd, uint32_t len_p,
                                        uint32_t len_s, uint32_t prev[8], uint32_t* dst) {
    const uint32_t c = 72u - len_p, r = c & 3u, nb = splice_blocks(len_p, len_s);
    const uint32_t* sx = sb + (c >> 2) + odd;         // dword w = 2i + odd of each block
    uint32_t X[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) X[i] = 0;
#pragma unroll
    for (uint32_t i = 0; i < 17; ++i) {               // block 0: the prefix lies here
        uint32_t v = align_bytes(sx[2u * i + 1u], sx[2u * i], r);
        if (i < PFX_WORDS) v |= pw[2u * i];
        X[i] ^= v;
    }
    if (odd & (nb == 1u)) X[16] ^= 0x80000000u;
    keccak_f1600_pair(X, odd);
#pragma unroll 1
    for (uint32_t blk = 1; blk < nb; ++blk) {
        // block 1 reads at most dword 77 of the buffer (c >> 2 <= 9); a third block's reads past the suffix
        // body clamp to the zero dword (compact buffer)
        const uint32_t k0 = (c >> 2) + odd + 34u * blk;
#pragma unroll
        for (uint32_t i = 0; i < 17; ++i) {
            uint32_t ka = k0 + 2u * i, kb = ka + 1u;
            if (BFT_CHAIN_COMPACT) { ka = ka < CHAIN_SB_ZERO ? ka : CHAIN_SB_ZERO; kb = kb < CHAIN_SB_ZERO ? kb : CHAIN_SB_ZERO; }
            X[i] ^= align_bytes(sb[kb], sb[ka], r);
        }
        if (odd & (blk + 1u == nb)) X[16] ^= 0x80000000u;
        keccak_f1600_pair(X, odd);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t o = pair_swap(X[i]);
        dst[2 * i + odd] = X[i];
        prev[2 * i] = odd ? o : X[i];
        prev[2 * i + 1] = odd ? X[i] : o;
    }
}
#endif

__constant__ PfxSel PFX_TBL[16] = {pfx_sel(0), pfx_sel(1), pfx_sel(2), pfx_sel(3), pfx_sel(4), pfx_sel(5),
                                   pfx_sel(6), pfx_sel(7), pfx_sel(8), pfx_sel(9), pfx_sel(10), pfx_sel(11),
                                   pfx_sel(12), pfx_sel(13), pfx_sel(14), pfx_sel(15)};

// One block is exactly one wave (launch_hash_chain): each lane pair reads only its own sbuf / pbuf
// slices, and the __syncthreads below sit inside loops whose trip counts differ between the pairs of a
// block (and after early exits) -- safe only because a one-wave barrier orders the wave's own LDS accesses.
constexpr uint32_t CHAIN_PAIR_BLOCK = 64;
__device__ inline void set_prio(uint32_t k) {      // s_setprio takes an immediate
    if (k == 1u) __builtin_amdgcn_s_setprio(1);
    else if (k == 2u) __builtin_amdgcn_s_setprio(2);
    else if (k >= 3u) __builtin_amdgcn_s_setprio(3);
}
// `cs`: the row-table sets of the launches whose chains this kernel runs (a launch's blocks are contiguous)
__global__ __launch_bounds__(CHAIN_PAIR_BLOCK) void bft_hash_chain_kernel(Params p, ChainSets cs) {
    static_assert(CHAIN_PAIR_BLOCK == 64, "bft_hash_chain_kernel's barriers assume one-wave blocks");
#if defined(__HIP_DEVICE_COMPILE__)
    set_prio(p.chain_prio);
    {
        const uint32_t bps = (p.n_instances + 31u) / 32u, k = blockIdx.x / bps;   // k < cs.count (grid)
        p.sfx = const_cast<uint32_t*>(cs.sfx[k]);
        p.committed_height = const_cast<uint32_t*>(cs.ch[k]);
        p.hash = cs.hash[k];
    }
    const uint32_t blk = blockIdx.x % ((p.n_instances + 31u) / 32u);
    __shared__ __attribute__((aligned(16))) uint32_t sbuf[32 * CHAIN_SB];     // splice buffer per pair
    __shared__ __attribute__((aligned(16))) uint64_t pbuf[CHAIN_PB_SLOTS * (PFX_WORDS + 4)];   // prefix (per pair: compact)
    __shared__ PfxSel ptbl[16];                                                 // header_prefix_perm
    if (threadIdx.x < 16) ptbl[threadIdx.x] = PFX_TBL[threadIdx.x];
    __syncthreads();
    const uint32_t odd = threadIdx.x & 1u, pair = threadIdx.x >> 1;
    const uint32_t il = blk * 32u + pair;
    if (il >= p.n_instances) return;                  // both lanes of a pair leave together
    const uint32_t K = p.sfx_rows, x0 = p.sfx_x0;
    // CHAIN_RECORDED: heights x0 .. min(ch, x0 + K - 1); CHAIN_PREDICTED: every height of the chunk, until the
    // first one without a prediction (suffix length 0); CHAIN_REPAIR: from the first recorded block that differs
    // from its prediction (bft_spec_verify_kernel) up to ch
    uint32_t x1 = x0 + K - 1u, xs = x0;
    if (p.chain_mode != CHAIN_PREDICTED) {
        const uint32_t ch = p.committed_height[il];
        x1 = ch < x1 ? ch : x1;
        if (p.chain_mode == CHAIN_REPAIR) {
            const uint32_t b = cs.bad[blockIdx.x / ((p.n_instances + 31u) / 32u)][il];
            xs = b > x0 ? b : x0;
        }
    }
    if (x1 < xs) return;
    uint32_t* sb = sbuf + pair * CHAIN_SB;
    for (uint32_t i = odd; i < SFX_PAD; i += 2u) sb[i] = 0;
    for (uint32_t i = SFX_PAD + SFX_BODY_DW + odd; i < CHAIN_SB; i += 2u) sb[i] = 0;
    // the parent of xs: genesis, or the hash of xs - 1 (the previous chunk's last, or a verified prediction;
    // written before this kernel on the same stream)
    const uint8_t* ph = xs == 1u ? p.genesis_hash : p.hash + ((uint64_t)il * p.rows + xs - 1u) * 32;
    uint32_t prev[8];
    for (int i = 0; i < 8; ++i)
        prev[i] = (uint32_t)ph[4 * i] | ((uint32_t)ph[4 * i + 1] << 8) | ((uint32_t)ph[4 * i + 2] << 16) |
                  ((uint32_t)ph[4 * i + 3] << 24);
    // this lane's half of the suffix body of the next height, and its length
    constexpr uint32_t HALF = SFX_BODY_DW / 2u;
    const uint32_t n = p.n_instances;
    const uint64_t rstride = (uint64_t)SFX_DEV_DW * n;   // suffix rows: [height][dword][instance]
    const uint32_t* srow = p.sfx + il + (uint64_t)odd * HALF * n;
    uint32_t s[HALF], slen;
    {
        const uint64_t ro = (uint64_t)(xs - x0) * rstride;
#pragma unroll
        for (uint32_t i = 0; i < HALF; ++i) s[i] = srow[ro + (uint64_t)i * n];
        slen = p.sfx[il + ro + (uint64_t)SFX_DEV_LEN_DW * n];
    }
    uint64_t* pb = pbuf + (BFT_CHAIN_COMPACT ? pair : threadIdx.x) * (PFX_WORDS + 4);   // both lanes write the same words
    const uint32_t* pw = (const uint32_t*)pb + odd;
    for (uint32_t x = xs; x <= x1; ++x) {
        const uint32_t len_s = slen;
        if (len_s == 0u) break;                       // no prediction for x (CHAIN_PREDICTED only; both lanes)
#pragma unroll
        for (uint32_t i = 0; i < HALF; ++i) sb[SFX_PAD + odd * HALF + i] = s[i];
        if (x < x1) {                                 // prefetch height x + 1
            const uint64_t ro = (uint64_t)(x + 1u - x0) * rstride;
#pragma unroll
            for (uint32_t i = 0; i < HALF; ++i) s[i] = srow[ro + (uint64_t)i * n];
            slen = p.sfx[il + ro + (uint64_t)SFX_DEV_LEN_DW * n];
        }
        const uint32_t len_p = header_prefix_perm(pb, prev, ptbl);
        __syncthreads();                              // the pair's suffix halves and this lane's prefix
        pair_header_hash(sb, pw, odd, len_p, len_s, prev, (uint32_t*)(p.hash + ((uint64_t)il * p.rows + x) * 32));
        __syncthreads();                              // splice buffer read before the next height's write
    }
#endif
}

// Keccak-f[1600] with the whole state in one lane as 32-bit halves (L low, H high): theta's D folded into one
// 3-input XOR per half-word (v_bitop3_b32), rotations as two v_alignbit_b32, chi one v_bitop3_b32 per half-word:
// ~180 VALU per round. The 24 rounds unrolled: rho-pi permutes the 25 words with period 24, so a round loop pays
// ~80 v_mov per round to move them back to their registers (cfg3 with inline suffixes: 1.81e9-1.84e9 with the loop,
// 1.90e9-1.94e9 unrolled; profiles/r06/ab_lane); one call site in the kernel (code size).
#if defined(__HIP_DEVICE_COMPILE__)
#ifndef BFT_LANE_UNROLL
#define BFT_LANE_UNROLL 24
#endif
__device__ inline void keccak_f1600_lane(uint32_t L[25], uint32_t H[25]) {
#pragma unroll BFT_LANE_UNROLL
    for (int rnd = 0; rnd < 24; ++rnd) {
        uint32_t cl[5], ch[5], rl[5], rh[5], bl[25], bh[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            cl[x] = xor3_32(xor3_32(L[x], L[x + 5], L[x + 10]), L[x + 15], L[x + 20]);
            ch[x] = xor3_32(xor3_32(H[x], H[x + 5], H[x + 10]), H[x + 15], H[x + 20]);
        }
#pragma unroll
        for (int x = 0; x < 5; ++x) rotl_halves<1>(cl[(x + 1) % 5], ch[(x + 1) % 5], rl[x], rh[x]);
#define BFT_RHO_L(i, n, j) rotl_halves<n>(xor3_32(L[i], cl[((i) % 5 + 4) % 5], rl[(i) % 5]), \
                                          xor3_32(H[i], ch[((i) % 5 + 4) % 5], rh[(i) % 5]), bl[j], bh[j]);
        BFT_RHO_L(0, 0, 0) BFT_RHO_L(1, 1, 10) BFT_RHO_L(2, 62, 20) BFT_RHO_L(3, 28, 5) BFT_RHO_L(4, 27, 15)
        BFT_RHO_L(5, 36, 16) BFT_RHO_L(6, 44, 1) BFT_RHO_L(7, 6, 11) BFT_RHO_L(8, 55, 21) BFT_RHO_L(9, 20, 6)
        BFT_RHO_L(10, 3, 7) BFT_RHO_L(11, 10, 17) BFT_RHO_L(12, 43, 2) BFT_RHO_L(13, 25, 12) BFT_RHO_L(14, 39, 22)
        BFT_RHO_L(15, 41, 23) BFT_RHO_L(16, 45, 8) BFT_RHO_L(17, 15, 18) BFT_RHO_L(18, 21, 3) BFT_RHO_L(19, 8, 13)
        BFT_RHO_L(20, 18, 14) BFT_RHO_L(21, 2, 24) BFT_RHO_L(22, 61, 9) BFT_RHO_L(23, 56, 19) BFT_RHO_L(24, 14, 4)
#undef BFT_RHO_L
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x) {
                L[5 * y + x] = bl[5 * y + x] ^ (~bl[5 * y + (x + 1) % 5] & bl[5 * y + (x + 2) % 5]);
                H[5 * y + x] = bh[5 * y + x] ^ (~bh[5 * y + (x + 1) % 5] & bh[5 * y + (x + 2) % 5]);
            }
        L[0] ^= KECCAK_RC_LO[rnd];
        H[0] ^= KECCAK_RC_HI[rnd];
    }
}
#endif

// INLINE: the suffix body dwords a lane keeps in its LDS column. The suffix is at most 212 bytes (address 44, root 35,
// tx_hash <= 67, receipt 35, the scalars and extra 31) plus the domain byte: dwords 0 .. 53; the splice reads every
// dword past the column as 0 (as it reads the row's zero tail). 56 instead of SFX_BODY_DW's 60: 14 KB per chain wave,
// so that more consensus waves fit a CU beside two chain waves per SIMD.
constexpr uint32_t SFX_LDS_DW = 56;
static_assert(SFX_LDS_DW * 4u >= 213u && SFX_LDS_DW <= SFX_BODY_DW && SFX_LDS_DW % 2u == 0u, "inline suffix column");
// Large shards (>= 8,192 instances per launch, bftsim.hip chain_lane_min): a LANE per instance. The whole state in
// one lane: ~180 VALU per round instead of 2 x 118 for a lane pair, i.e. ~24 % fewer instructions per header for
// ~1.5x the chain latency, which a large shard's throughput-bound pipeline hides (cfg3 at 16,384: 1.70e9 with lane
// pairs, 1.82e9-1.85e9 with lanes in batches of 12; profiles/r06/ab_lane).
// The splice reads the suffix row straight from global memory (rows are dword-major across instances, so a load
// instruction touches one row per distinct prefix length in the wave) instead of an LDS splice buffer per lane.
#if defined(__HIP_DEVICE_COMPILE__)
// one instance's chain (launch k of the batch, instance il) by one lane
// INLINE: the lane encodes each height's suffix itself from the recorded row (proposer, variant, time tick) into its
// column of `sl` (LDS, dword j at sl[64 j]) instead of reading a suffix row of bft_hash_suffix_kernel (RECORDED and
// REPAIR modes only)
template <bool INLINE>
__device__ inline void lane_chain(const Params& p, const ChainSets& cs, uint32_t k, uint32_t il, const PfxSel* ptbl,
                                  uint32_t* sl) {
    const uint32_t n = p.n_instances;
    const uint32_t K = p.sfx_rows, x0 = p.sfx_x0;
    uint32_t x1 = x0 + K - 1u, xs = x0;
    if (p.chain_mode != CHAIN_PREDICTED) {
        const uint32_t ch = cs.ch[k][il];
        x1 = ch < x1 ? ch : x1;
        if (p.chain_mode == CHAIN_REPAIR) {
            const uint32_t b = cs.bad[k][il];
            xs = b > x0 ? b : x0;
        }
    }
    if (x1 < xs) return;
    uint8_t* const hash = cs.hash[k];
    const uint32_t* ph = (const uint32_t*)(xs == 1u ? p.genesis_hash : hash + ((uint64_t)il * p.rows + xs - 1u) * 32);
    uint32_t prev[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) prev[i] = ph[i];
    // suffix rows: byte offsets from the set's base (uniform, so the loads take saddr + a 32-bit voffset; a set's
    // rows are < 2 GiB, bftsim.hip); dword j of the row of height x at 4 (il + ((x - x0) SFX_DEV_DW + j) n)
    const char* const sbase = (const char*)cs.sfx[k];
    const uint32_t n4 = 4u * n;                      // < 2^24 (launch_hash_chain_batch): 24-bit multiplies
    const uint32_t* const rec = cs.rec[k] + (uint64_t)il * p.rows * 4u;
    const bool predicted = INLINE && p.chain_mode == CHAIN_PREDICTED;
    uint64_t byz = 0;
    if (predicted) {   // the instance's Byzantine set (bft_spec_byz_kernel's), its permutation in the lane's LDS column
        byz = byz_mask64<64>(p.seed, cs.first[k] + il, p.byz_count, (uint8_t*)sl);
        cs.bad[k][il] = 0xffffffffu;                  // no recorded block differs yet (bft_spec_verify_kernel)
    }
    uint32_t* const pred = predicted ? cs.pred[k] + (uint64_t)il * p.heights : nullptr;
    for (uint32_t x = xs; x <= x1; ++x) {
        const uint32_t rowoff = 4u * il + (x - x0) * SFX_DEV_DW * n4;
        uint32_t len_s;
        if constexpr (INLINE) {                      // the suffix of block x (bft_hash_suffix_kernel's)
            uint32_t prop, var, tick;
            if (p.chain_mode == CHAIN_PREDICTED) {
                // the block the canonical tick would commit, and its prediction word (bft_spec_suffix_kernel's)
                const bool ok = spec_block64(p.seed, cs.first[k] + il, x, byz, 0u, prop, var);
                pred[x - 1u] = ok ? SPEC_VALID | prop | (var << 16) : 0u;
                if (!ok) break;                      // no prediction for x: the chain stops (repaired from here)
                tick = x - 1u;
            } else {                                 // the recorded block
                const uint4 row = *(const uint4*)(rec + 4u * x);
                prop = row.y & 0xffffu;
                var = (row.y >> 16) & 1u;
                tick = row.z;
            }
            HdrWriter w(sl, 64u);
            header_suffix_fields(w, p.addresses + 20u * prop, p.seed, cs.first[k] + il, x, prop, var,
                                 p.genesis_time + (uint64_t)p.block_period * ((uint64_t)tick + 1ull));
            len_s = 8u * w.wi + w.fill;
            w.store(w.wi++, w.acc | (0x01ull << (8u * w.fill)));
            while (w.wi < SFX_LDS_DW / 2u) w.store(w.wi++, 0);
        } else {
            len_s = *(const uint32_t*)(sbase + rowoff + SFX_DEV_LEN_DW * n4);
        }
        if (len_s == 0u) break;                      // no prediction for x (CHAIN_PREDICTED only)
        uint32_t pw[2 * PFX_WORDS];
        const uint32_t len_p = header_prefix_regs(prev, ptbl, pw);
        const uint32_t c = 72u - len_p, r = c & 3u, nb = splice_blocks(len_p, len_s);
        const int j0 = (int)(c >> 2) - (int)SFX_PAD;   // body dword of splice dword q0: -17 .. -9
        // splice-buffer dword j0 + i: the body dword, zero outside [0, BODY) (the pad and the tail)
        auto G = [&](uint32_t jj) -> uint32_t {      // body dword jj < SFX_BODY_DW
            if constexpr (INLINE) return sl[64u * jj];
            else return *(const uint32_t*)(sbase + rowoff + __umul24(jj, n4));
        };
        constexpr int BODY = INLINE ? (int)SFX_LDS_DW : (int)SFX_BODY_DW;   // dwords past it read as 0
        auto S = [&](int j) -> uint32_t {
            const uint32_t v = G((uint32_t)(j < 0 ? 0 : j > BODY - 1 ? BODY - 1 : j));
            return ((j >= 0) & (j < BODY)) ? v : 0u;
        };
        // the state starts as the prefix words (the suffix bytes spliced in below are 0 where the prefix is, so
        // XOR = OR), so the prefix registers die before the block loop
        uint32_t L[25], H[25];
#pragma unroll
        for (int i = 0; i < 25; ++i) {
            L[i] = i < (int)PFX_WORDS ? pw[2 * i] : 0u;
            H[i] = i < (int)PFX_WORDS ? pw[2 * i + 1] : 0u;
        }
        for (uint32_t blk = 0; blk < nb; ++blk) {     // one permutation site (code size)
            uint32_t d[35];
            if (blk == 0u) {                         // the prefix lies here; dwords from 17 on are in the body
#pragma unroll
                for (int i = 0; i < 17; ++i) d[i] = S(j0 + i);
                if constexpr (INLINE) {
#pragma unroll
                    for (int i = 17; i < 35; ++i) d[i] = G((uint32_t)(j0 + i));
                } else {
                    uint32_t vo = rowoff + __umul24((uint32_t)(j0 + 17), n4);
#pragma unroll
                    for (int i = 17; i < 35; ++i, vo += n4) d[i] = *(const uint32_t*)(sbase + vo);
                }
#pragma unroll
                for (int i = 0; i < 34; ++i) d[i] = align_bytes(d[i + 1], d[i], r);
            } else {
#pragma unroll
                for (int i = 0; i < 35; ++i) d[i] = S(j0 + 34 * (int)blk + i);
#pragma unroll
                for (int i = 0; i < 34; ++i) d[i] = align_bytes(d[i + 1], d[i], r);
            }
#pragma unroll
            for (int i = 0; i < 17; ++i) { L[i] ^= d[2 * i]; H[i] ^= d[2 * i + 1]; }
            if (blk + 1u == nb) H[16] ^= 0x80000000u;
            keccak_f1600_lane(L, H);
        }
        uint32_t* dst = (uint32_t*)(hash + ((uint64_t)il * p.rows + x) * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) { prev[2 * i] = L[i]; prev[2 * i + 1] = H[i]; }
        *(uint4*)dst = make_uint4(prev[0], prev[1], prev[2], prev[3]);
        *(uint4*)(dst + 4) = make_uint4(prev[4], prev[5], prev[6], prev[7]);
    }
}
#endif
// Persistent: at most p.chain_grid workgroups (one wave each), each taking 64 instances after another. A chain wave
// runs its instances' 100 heights back to back, so a grid of every task at once held every SIMD slot for the whole
// dispatch and the consensus kernels beside it got none (cfg3: a FAST kernel 0.40 -> 4.6 ms under a 12-launch chain
// dispatch, profiles/r06/traces/r06n_timeline_k16.txt); capped, the chain waves leave slots to them.
// register budget: the inline variant at 4 waves per SIMD (128 VGPRs, no scratch; 149 at 3) so that two chain waves
// fit a SIMD beside two FAST waves (111 VGPRs each): 2 x 128 + 2 x 112 <= 512; the global-row variant (predicted
// chains) at 3
#ifndef BFT_LANE_WAVES_PER_SIMD
#define BFT_LANE_WAVES_PER_SIMD 4
#endif

template <bool INLINE>
__global__ __launch_bounds__(64, INLINE ? BFT_LANE_WAVES_PER_SIMD : 3) void bft_hash_chain_lane_kernel(Params p, ChainSets cs) {
#if defined(__HIP_DEVICE_COMPILE__)
    set_prio(p.chain_prio);
    __shared__ PfxSel ptbl[16];
    extern __shared__ uint32_t sfx_lds[];             // INLINE: [SFX_LDS_DW][64] suffix dwords (launch's dynamic LDS)
    if (threadIdx.x < 16) ptbl[threadIdx.x] = PFX_TBL[threadIdx.x];
    __syncthreads();
    const uint32_t bps = (p.n_instances + 63u) / 64u, tasks = cs.count * bps;
    for (uint32_t t = blockIdx.x; t < tasks; t += gridDim.x) {   // every wave reaches the end of the task list
        const uint32_t k = t / bps, il = (t % bps) * 64u + threadIdx.x;
        if (il < p.n_instances)
            lane_chain<INLINE>(p, cs, k, il, ptbl, INLINE ? sfx_lds + threadIdx.x : nullptr);
    }
#endif
}
static hipError_t launch_lane(uint32_t tasks, const ChainSets& cs, hipStream_t s, const Params& p) {
    const uint32_t g = p.chain_grid && p.chain_grid < tasks ? p.chain_grid : tasks;   // persistent waves
    if (p.chain_inline)                               // the inline suffix columns in dynamic LDS
        hipLaunchKernelGGL(bft_hash_chain_lane_kernel<true>, dim3(g), dim3(64), (size_t)SFX_LDS_DW * 64u * 4u, s, p, cs);
    else hipLaunchKernelGGL(bft_hash_chain_lane_kernel<false>, dim3(g), dim3(64), 0, s, p, cs);
    return hipGetLastError();
}

// Predicted chains (big-endian seeds, N = 64). With big-endian seeds the round-0 proposer of an
// N = 64 instance is validator 0 at every height (validator.rs:33-48: the seed is 0 mod 64), so the block the
// canonical tick commits at height x (spec_block64: proposer 0, the variant the SPLIT draw of view (x, 0) lets
// commit, time tick x - 1) depends on no hash. Its suffix row is encoded and the prev_hash chains run before the
// consensus kernel has recorded anything, i.e. from launch time instead of behind the consensus kernel.
// bft_spec_verify_kernel then compares every recorded block with its prediction, rewrites the suffix rows of
// those that differ and notes the first such height; the chains are re-run from there (CHAIN_REPAIR). A
// predicted hash is kept only where its block and all of its ancestors were predicted right, so every hash is
// the recorded block's by construction.
__global__ __launch_bounds__(256) void bft_spec_byz_kernel(Params p, ChainSets cs) {
    set_prio(p.chain_prio);                           // on the predicted chains' critical path
    __shared__ uint8_t perm[256 * 64];                // byz_mask64's permutation, per thread
    const uint32_t n = p.n_instances, bpl = (n + 255u) / 256u, k = blockIdx.x / bpl;
    const uint32_t il = (blockIdx.x % bpl) * 256u + threadIdx.x;
    if (il >= n) return;
    cs.byz[k][il] = byz_mask64(p.seed, cs.first[k] + il, p.byz_count, perm + 64u * threadIdx.x);
    cs.bad[k][il] = 0xffffffffu;
}
__device__ inline uint64_t spec_time(const Params& p, uint32_t tick) {
    return p.genesis_time + (uint64_t)p.block_period * ((uint64_t)tick + 1ull);
}
// thread per (launch, height, instance), consecutive threads = consecutive instances (the row layout)
__global__ __launch_bounds__(256) void bft_spec_suffix_kernel(Params p, ChainSets cs) {
    set_prio(p.chain_prio);                           // on the predicted chains' critical path
    const uint32_t n = p.n_instances, H = p.heights;
    const uint32_t bpl = (uint32_t)(((uint64_t)n * H + 255u) / 256u), k = blockIdx.x / bpl;
    const uint32_t t = (blockIdx.x % bpl) * 256u + threadIdx.x;   // n * H < 2^32 (bftsim.hip)
    const uint32_t j = t / n, il = t - j * n;
    if (j >= H) return;
    const uint32_t x = j + 1u, inst = cs.first[k] + il;
    uint32_t* row = const_cast<uint32_t*>(cs.sfx[k]) + (uint64_t)j * SFX_DEV_DW * n + il;
    uint32_t prop, var;
    if (!spec_block64(p.seed, inst, x, cs.byz[k][il], 0u, prop, var)) {
        row[(uint64_t)SFX_DEV_LEN_DW * n] = 0u;       // no prediction: the predicted chain stops here
        cs.pred[k][(uint64_t)il * H + j] = 0u;
        return;
    }
    cs.pred[k][(uint64_t)il * H + j] = SPEC_VALID | prop | (var << 16);
    header_suffix_strided(row, n, p.addresses + 20u * prop, p.seed, inst, x, prop, var, spec_time(p, x - 1u));
}
// thread per (launch, instance, height), consecutive threads = consecutive heights (coalesced record rows)
__global__ __launch_bounds__(256) void bft_spec_verify_kernel(Params p, ChainSets cs) {
    const uint32_t n = p.n_instances, H = p.heights;
    const uint32_t bpl = (uint32_t)(((uint64_t)n * H + 255u) / 256u), k = blockIdx.x / bpl;
    const uint32_t t = (blockIdx.x % bpl) * 256u + threadIdx.x;
    const uint32_t il = t / H, x = t - il * H + 1u;
    if (il >= n) return;
    if (x > cs.ch[k][il]) return;
    const uint4 row = *(const uint4*)(cs.rec[k] + ((uint64_t)il * p.rows + x) * 4);
    const uint32_t pw = cs.pred[k][(uint64_t)il * H + x - 1u], inst = cs.first[k] + il;
    if (((pw & SPEC_VALID) != 0u) & ((row.y & 0x1ffffu) == (pw & 0x1ffffu)) & (row.z + 1u == x)) return;
    // the recorded block differs: its own suffix row (as bft_hash_suffix_kernel writes it), and the repair
    // starts at the first such height
    const uint32_t rp = row.y & 0xffffu, rv = (row.y >> 16) & 1u;
    header_suffix_strided(const_cast<uint32_t*>(cs.sfx[k]) + (uint64_t)(x - 1u) * SFX_DEV_DW * n + il, n,
                          p.addresses + 20u * rp, p.seed, inst, x, rp, rv, spec_time(p, row.z));
    atomicMin(&cs.bad[k][il], x);
}
hipError_t launch_spec_suffix(uint32_t n, const ChainSets& cs, hipStream_t s, const Params& p) {
    if (cs.count < 1 || cs.count > CHAIN_MAX_SETS || p.n_instances != n) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bft_spec_byz_kernel, dim3(cs.count * ((n + 255u) / 256u)), dim3(256), 0, s, p, cs);
    const uint32_t bpl = (uint32_t)(((uint64_t)n * p.heights + 255u) / 256u);
    hipLaunchKernelGGL(bft_spec_suffix_kernel, dim3(cs.count * bpl), dim3(256), 0, s, p, cs);
    return hipGetLastError();
}
hipError_t launch_spec_verify(uint32_t n, const ChainSets& cs, hipStream_t s, const Params& p) {
    if (cs.count < 1 || cs.count > CHAIN_MAX_SETS || p.n_instances != n) return hipErrorInvalidValue;
    const uint32_t bpl = (uint32_t)(((uint64_t)n * p.heights + 255u) / 256u);
    hipLaunchKernelGGL(bft_spec_verify_kernel, dim3(cs.count * bpl), dim3(256), 0, s, p, cs);
    return hipGetLastError();
}

// Little-endian seeds, N = 64: the canonical blocks predicted ahead of the consensus kernel by a
// lane pair per instance. The proposer of height x follows from the hash of x - 1, so with the wave hash the
// consensus kernel hashed every height itself (~1,900 VALU per height for one instance); here the chain of
// predictions runs as the block-hash chains do (32 instances per wave). Per height: proposer and committing
// variant (spec_block64), the header suffix by the pair's even lane into the splice buffer, prev_hash,
// Keccak; then the hash row and the prediction word. It ends at H or at the first height without a
// prediction (word 0 there). Fast64::hash_pending takes a prediction only while each recorded block equals
// it, and hashes in the wave from the first one that does not.
__global__ __launch_bounds__(CHAIN_PAIR_BLOCK) void bft_seed_chain_kernel(Params p) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ __attribute__((aligned(16))) uint32_t sbuf[32 * CHAIN_SB];     // splice buffer per pair
    __shared__ __attribute__((aligned(16))) uint64_t pbuf[CHAIN_PB_SLOTS * (PFX_WORDS + 4)];   // prefix (per pair: compact)
    __shared__ PfxSel ptbl[16];
    __shared__ uint32_t slen[32];                                               // suffix length per pair
    if (threadIdx.x < 16) ptbl[threadIdx.x] = PFX_TBL[threadIdx.x];
    __syncthreads();
    const uint32_t odd = threadIdx.x & 1u, pair = threadIdx.x >> 1;
    const uint32_t il = blockIdx.x * 32u + pair;
    if (il >= p.n_instances) return;                  // both lanes of a pair leave together
    const uint32_t n = p.n_instances, inst = p.first_instance + il;
    uint32_t* sb = sbuf + pair * CHAIN_SB;
    // the Byzantine validators: each lane draws them, its 64-byte permutation in the pair's splice buffer
    const uint64_t byz = byz_mask64(p.seed, inst, p.byz_count, (uint8_t*)(sb + SFX_PAD) + 64u * odd);
    __syncthreads();
    for (uint32_t i = odd; i < SFX_PAD; i += 2u) sb[i] = 0;
    for (uint32_t i = SFX_PAD + SFX_BODY_DW + odd; i < CHAIN_SB; i += 2u) sb[i] = 0;
    const uint8_t* ph = p.genesis_hash;
    uint32_t prev[8];
    for (int i = 0; i < 8; ++i)
        prev[i] = (uint32_t)ph[4 * i] | ((uint32_t)ph[4 * i + 1] << 8) | ((uint32_t)ph[4 * i + 2] << 16) |
                  ((uint32_t)ph[4 * i + 3] << 24);
    uint64_t* pb = pbuf + (BFT_CHAIN_COMPACT ? pair : threadIdx.x) * (PFX_WORDS + 4);   // both lanes write the same words
    const uint32_t* pw = (const uint32_t*)pb + odd;
    for (uint32_t x = 1; x <= p.heights; ++x) {
        uint32_t j, var;
        if (!spec_block64(p.seed, inst, x, byz, prev[0], j, var)) {
            if (!odd) p.spec[(uint64_t)x * n + il] = 0u;
            break;
        }
        if (!odd) {                                   // header_suffix_fields of (x, j, var) at time tick x - 1
            HdrWriter w(sb + SFX_PAD, 1u);
            header_suffix_fields(w, p.addresses + 20u * j, p.seed, inst, x, j, var,
                                 p.genesis_time + (uint64_t)p.block_period * (uint64_t)x);
            slen[pair] = 8u * w.wi + w.fill;
            w.store(w.wi++, w.acc | (0x01ull << (8u * w.fill)));
            while (w.wi < SFX_BODY_DW / 2u) w.store(w.wi++, 0);
        }
        const uint32_t len_p = header_prefix_perm(pb, prev, ptbl);
        __syncthreads();                              // the suffix and this lane's prefix
        pair_header_hash(sb, pw, odd, len_p, slen[pair], prev, (uint32_t*)(p.hash + ((uint64_t)il * p.rows + x) * 32));
        if (!odd) p.spec[(uint64_t)x * n + il] = spec_word(j, var, seed_from_words(prev[0], prev[1], 64u, true));
        __syncthreads();                              // splice buffer read before the next height's write
    }
#endif
}
hipError_t launch_seed_chain(uint32_t n, hipStream_t s, const Params& p) {
    hipLaunchKernelGGL(bft_seed_chain_kernel, dim3((n + 31u) / 32u), dim3(CHAIN_PAIR_BLOCK), 0, s, p);
    return hipGetLastError();
}

// Small shards: the chain of one instance by one wave (bft_kwave.h kw50_chain). Workgroup b runs on XCD
// b % 8 (round-robin dispatch): consecutive instances, whose suffix dwords share cache lines (rows are
// dword-major across instances), are given to the same XCD.
__global__ __launch_bounds__(64) void bft_hash_chain_wave_kernel(Params p, ChainSets cs) {
    __shared__ __attribute__((aligned(16))) uint32_t sb[SFX_BUF];
    __shared__ __attribute__((aligned(16))) uint32_t pf[KW_PFX_DW];
    set_prio(p.chain_prio);
    const uint32_t lane = threadIdx.x;
    const uint32_t bps = 8u * ((p.n_instances + 7u) / 8u), k = blockIdx.x / bps, b = blockIdx.x % bps;
    p.sfx = const_cast<uint32_t*>(cs.sfx[k]);
    p.committed_height = const_cast<uint32_t*>(cs.ch[k]);
    p.hash = cs.hash[k];
    const uint32_t per = bps >> 3;                        // bps = 8 * ceil(n / 8)
    const uint32_t il = (b & 7u) * per + (b >> 3);
    if (il >= p.n_instances) return;                      // the whole wave
    const uint32_t K = p.sfx_rows, x0 = p.sfx_x0;
    const uint32_t ch = p.committed_height[il];
    const uint32_t x1 = ch < x0 + K - 1u ? ch : x0 + K - 1u;
    if (x1 < x0) return;
    const uint32_t* ph = (const uint32_t*)(x0 == 1u ? p.genesis_hash : p.hash + ((uint64_t)il * p.rows + x0 - 1u) * 32);
    const uint32_t a_prev = lane < 8u ? ph[lane] : 0u;
    WaveHip wv;
    kw50_chain(wv, lane, sb, pf, p.sfx + il, (uint64_t)SFX_DEV_DW * p.n_instances, p.n_instances, a_prev,
               x1 - x0 + 1u, (uint32_t*)(p.hash + ((uint64_t)il * p.rows + x0) * 32));
}

// heights [x0, x0 + rows) of the block-hash pass: the suffix rows, then the chains
hipError_t launch_hash_suffix(uint32_t n, uint32_t x0, uint32_t rows, uint32_t* sfx, bool loop, hipStream_t s,
                              Params p) {
    p.sfx = sfx;
    p.sfx_rows = rows;
    p.sfx_x0 = x0;
    if (loop) hipLaunchKernelGGL(bft_hash_suffix_loop_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(bft_hash_suffix_kernel, dim3((uint32_t)(((uint64_t)n * rows + 255u) / 256u)), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_hash_chain(uint32_t n, uint32_t x0, uint32_t rows, uint32_t* sfx, uint32_t kind, hipStream_t s,
                             Params p) {
    p.sfx = sfx;
    p.sfx_rows = rows;
    p.sfx_x0 = x0;
    ChainSets cs{};
    cs.count = 1; cs.sfx[0] = sfx; cs.ch[0] = p.committed_height; cs.hash[0] = p.hash;
    cs.rec[0] = p.rec; cs.first[0] = p.first_instance;
    if (kind == CHAIN_KERNEL_LANE && 4ull * n >= (1ull << 24)) kind = CHAIN_KERNEL_PAIR;   // its 24-bit offsets
    if (kind == CHAIN_KERNEL_LANE) return launch_lane((n + 63u) / 64u, cs, s, p);
    else if (kind == CHAIN_KERNEL_WAVE)
        hipLaunchKernelGGL(bft_hash_chain_wave_kernel, dim3(8u * ((n + 7u) / 8u)), dim3(64), 0, s, p, cs);
    else hipLaunchKernelGGL(bft_hash_chain_kernel, dim3((n + 31u) / 32u), dim3(CHAIN_PAIR_BLOCK), 0, s, p, cs);
    return hipGetLastError();
}
hipError_t launch_hash_chain_batch(uint32_t n, const ChainSets& cs, uint32_t kind, hipStream_t s, Params p) {
    p.sfx_rows = p.heights;                               // every height in one chunk (bftsim.hip)
    p.sfx_x0 = 1;
    if (cs.count < 1 || cs.count > CHAIN_MAX_SETS) return hipErrorInvalidValue;
    const bool wave = kind == CHAIN_KERNEL_WAVE;
    if (kind == CHAIN_KERNEL_LANE && 4ull * n >= (1ull << 24)) kind = CHAIN_KERNEL_PAIR;   // its 24-bit offsets
    if (kind == CHAIN_KERNEL_LANE) return launch_lane(cs.count * ((n + 63u) / 64u), cs, s, p);
    if (wave) hipLaunchKernelGGL(bft_hash_chain_wave_kernel, dim3(cs.count * 8u * ((n + 7u) / 8u)), dim3(64), 0, s, p, cs);
    else hipLaunchKernelGGL(bft_hash_chain_kernel, dim3(cs.count * ((n + 31u) / 32u)), dim3(CHAIN_PAIR_BLOCK), 0, s, p, cs);
    return hipGetLastError();
}

}  // namespace bft
