// bft_hip.h — gfx950 wave / workgroup collectives of the consensus kernels and the launchers of the
// kernel translation units (kern_*.hip), which libbftsim's host code (bftsim.hip) calls. The kernels
// are split over several translation units so that they compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/bftsim.h"
#include "bft_common.h"
#include "bft_wave.h"

namespace bft {

// ------------------------------------------------------------------------------ wave ops (gfx950)
struct WaveHip {
    __device__ void init(uint8_t*) {}
    __device__ static uint32_t lane() { return __lane_id(); }
    __device__ static uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
    __device__ static uint32_t shfl_xor(uint32_t v, int m) { return (uint32_t)__shfl_xor((int)v, m, 64); }
    __device__ static uint32_t shfl(uint32_t v, uint32_t src) { return (uint32_t)__shfl((int)v, (int)src, 64); }
    // DPP moves inside 16-lane rows: lane i gets lane i + N (row_shl) / i - N (row_shr); lanes whose
    // source is outside the row get 0
    template <int N> __device__ static uint32_t row_shl(uint32_t v) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x100 + N, 0xF, 0xF, true);
    }
    template <int N> __device__ static uint32_t row_shr(uint32_t v) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x110 + N, 0xF, 0xF, true);
    }
    // ds_bpermute_b32: this lane gets v of lane addr / 4 (addr = byte address, per lane)
    __device__ static uint32_t bperm(uint32_t addr, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v); }
    // the value of lane ^ 1 (DPP quad_perm [1,0,3,2])
    __device__ static uint32_t pair_swap(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); }
    // Keccak-f[1600] by lane pairs: the even lane of a pair holds the low 32-bit half of every state word, the odd
    // lane the high half (the layout of kern_fast.hip's chains). A 64-bit rotation is one v_alignbit_b32 of this
    // lane's half and the partner's (DPP quad_perm [1,0,3,2]); theta's parities, chi and iota are half-local. The
    // round loop is kept (the general kernels' code size); its round constant is a uniform scalar load.
    template <uint32_t N> __device__ static uint32_t rotl_pair(uint32_t mine, uint32_t other) {
        if constexpr (N == 0) return mine;
        else if constexpr (N == 32) return other;
        else if constexpr (N < 32) return __builtin_amdgcn_alignbit(mine, other, 32 - N);
        else return __builtin_amdgcn_alignbit(other, mine, 64 - N);
    }
    __device__ static uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {   // v_bitop3_b32 0x96
#if defined(__HIP_DEVICE_COMPILE__)
        return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
        return a ^ b ^ c;
#endif
    }
    __device__ static void keccak_pair(uint32_t X[25], uint32_t odd) {
#pragma unroll 1
        for (int rnd = 0; rnd < 24; ++rnd) {
            uint32_t c[5], r1[5], t[25], b[25];
            // theta with 3-input XORs (v_bitop3_b32): two per column parity, one per word (X ^ C[x-1] ^ rot(C[x+1]))
#pragma unroll
            for (int x = 0; x < 5; ++x) c[x] = xor3(xor3(X[x], X[x + 5], X[x + 10]), X[x + 15], X[x + 20]);
#pragma unroll
            for (int x = 0; x < 5; ++x) r1[x] = rotl_pair<1>(c[(x + 1) % 5], pair_swap(c[(x + 1) % 5]));
#pragma unroll
            for (int i = 0; i < 25; ++i) t[i] = xor3(X[i], c[(i % 5 + 4) % 5], r1[i % 5]);
#define BFT_RHO_P(i, n, j) b[j] = rotl_pair<n>(t[i], (n) ? pair_swap(t[i]) : 0u);
            BFT_RHO_P(0, 0, 0) BFT_RHO_P(1, 1, 10) BFT_RHO_P(2, 62, 20) BFT_RHO_P(3, 28, 5) BFT_RHO_P(4, 27, 15)
            BFT_RHO_P(5, 36, 16) BFT_RHO_P(6, 44, 1) BFT_RHO_P(7, 6, 11) BFT_RHO_P(8, 55, 21) BFT_RHO_P(9, 20, 6)
            BFT_RHO_P(10, 3, 7) BFT_RHO_P(11, 10, 17) BFT_RHO_P(12, 43, 2) BFT_RHO_P(13, 25, 12) BFT_RHO_P(14, 39, 22)
            BFT_RHO_P(15, 41, 23) BFT_RHO_P(16, 45, 8) BFT_RHO_P(17, 15, 18) BFT_RHO_P(18, 21, 3) BFT_RHO_P(19, 8, 13)
            BFT_RHO_P(20, 18, 14) BFT_RHO_P(21, 2, 24) BFT_RHO_P(22, 61, 9) BFT_RHO_P(23, 56, 19) BFT_RHO_P(24, 14, 4)
#undef BFT_RHO_P
#pragma unroll
            for (int y = 0; y < 5; ++y)
#pragma unroll
                for (int x = 0; x < 5; ++x)
                    X[5 * y + x] = b[5 * y + x] ^ (~b[5 * y + (x + 1) % 5] & b[5 * y + (x + 2) % 5]);
            // both halves' round constants as uniform (scalar) loads, then a select: a per-lane address would be
            // a vector load waited for in every round
            const uint32_t rlo = __builtin_amdgcn_readfirstlane(KECCAK_RC_LO[rnd]);
            const uint32_t rhi = __builtin_amdgcn_readfirstlane(KECCAK_RC_HI[rnd]);
            X[0] ^= odd ? rhi : rlo;
        }
    }
    // set bits of m below this lane (v_mbcnt_lo / hi)
    __device__ static uint32_t rank_below(uint64_t m) {
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    __device__ static uint32_t readlane(uint32_t v, uint32_t l) {      // l wave-uniform
        return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)__builtin_amdgcn_readfirstlane((int)l));
    }
    // a wave-uniform value held in a VGPR → SGPR (frees the VGPR for the lane state)
    __device__ static uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
    __device__ static uint64_t clock() { return __builtin_amdgcn_s_memtime(); }
    __device__ static void sync() {
        // Intra-wave LDS hand-off: the LDS executes one wave's DS instructions in program order,
        // so a later ds_read of any lane sees every earlier ds_write of the wave. Only the
        // compiler must not move memory operations across this point (no s_waitcnt needed).
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    }
    __device__ static uint32_t gload(const uint32_t* p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static void gstore(uint32_t* p, uint32_t v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // 16-byte aligned row store (global_store_dwordx4; L1 is write-through, readers use L2 loads)
    __device__ static void gstore4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
        *(uint4*)p = make_uint4(a, b, c, d);
    }
    __device__ static void lds_add(uint32_t* p, uint32_t v) { atomicAdd(p, v); }
    __device__ static void gadd64(uint64_t* p, uint64_t v) { atomicAdd((unsigned long long*)p, (unsigned long long)v); }
};

// ------------------------------------------------------------- workgroup ops (S = 64*NW lanes)
// One instance per workgroup of NW waves. A collective = per-wave partial (ballot / butterfly)
// written to an LDS slot by each wave's lane 0, one s_barrier, every lane combines the NW
// partials. The slots alternate between two parities: a slot is rewritten only after the next
// collective's barrier, which every lane reaches after finishing its reads of this one.
template <int NW>
struct GroupHip {
    uint64_t* slot;       // LDS: [2 parities][4 words]
    uint32_t par;
    __device__ void init(uint8_t* p) { slot = (uint64_t*)p; par = 0; }
    __device__ uint32_t lane() const { return threadIdx.x; }
    __device__ uint64_t* cur() const { return slot + par * 4u; }
    __device__ Bits<NW> ballot(bool p) {
        uint64_t b = __ballot(p);
        uint64_t* s = cur();
        if (__lane_id() == 0) s[threadIdx.x >> 6] = b;
        __syncthreads();
        Bits<NW> r;
#pragma unroll
        for (int k = 0; k < NW; ++k) r.w[k] = s[k];
        par ^= 1u;
        return r;
    }
    __device__ uint32_t bcast(uint32_t v, uint32_t j) {     // value of lane j (j uniform)
        uint64_t* s = cur();
        if (threadIdx.x == j) s[0] = v;
        __syncthreads();
        uint32_t r = (uint32_t)s[0];
        par ^= 1u;
        return r;
    }
    __device__ uint32_t grp_max(uint32_t v) {
        for (int m = 1; m < 64; m <<= 1) { uint32_t o = (uint32_t)__shfl_xor((int)v, m, 64); v = v > o ? v : o; }
        uint64_t* s = cur();
        if (__lane_id() == 0) s[threadIdx.x >> 6] = v;
        __syncthreads();
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) r = (uint32_t)s[k] > r ? (uint32_t)s[k] : r;
        par ^= 1u;
        return r;
    }
    __device__ uint32_t grp_or(uint32_t v) {
        for (int m = 1; m < 64; m <<= 1) v |= (uint32_t)__shfl_xor((int)v, m, 64);
        uint64_t* s = cur();
        if (__lane_id() == 0) s[threadIdx.x >> 6] = v;
        __syncthreads();
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) r |= (uint32_t)s[k];
        par ^= 1u;
        return r;
    }
    __device__ uint64_t grp_sum64(uint32_t v32) {
        uint64_t v = v32;
        for (int m = 1; m < 64; m <<= 1) {
            uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
            v += (uint64_t)lo | ((uint64_t)hi << 32);
        }
        uint64_t* s = cur();
        if (__lane_id() == 0) s[threadIdx.x >> 6] = v;
        __syncthreads();
        uint64_t r = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) r += s[k];
        par ^= 1u;
        return r;
    }
    __device__ void sync() { __syncthreads(); par ^= 1u; }
    // batched collectives (one barrier each): K ballots; K words each written by at most one lane
    // (wr[k]; an unwritten word reads as stale data, which the caller must not use)
    __device__ uint64_t* big() const { return slot + 8 + par * 64u; }
    template <int K> __device__ void ballot_k(const bool (&p)[K], Bits<NW> (&out)[K]) {
        static_assert(K * NW <= 64, "batched ballot area");
        uint64_t* s = big();
        uint64_t b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) b[k] = __ballot(p[k]);
        if (__lane_id() == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) s[k * NW + (threadIdx.x >> 6)] = b[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int w = 0; w < NW; ++w) out[k].w[w] = s[k * NW + w];
        par ^= 1u;
    }
    // the phase summary's K ballots into the stable LDS area summary() ([K][NW], one barrier): read by
    // every lane until the next phase (Sim::kmask), no register copies
    __device__ uint64_t* summary() const { return slot + 8 + 2u * 64u; }
    template <int K> __device__ void ballot_k_store(const bool (&p)[K], uint64_t* dst) {
        uint64_t b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) b[k] = __ballot(p[k]);
        if (__lane_id() == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) dst[k * NW + (threadIdx.x >> 6)] = b[k];
        }
        __syncthreads();
        par ^= 1u;
    }
    template <int K> __device__ void gather_k(const bool (&wr)[K], const uint32_t (&v)[K], uint32_t (&out)[K]) {
        static_assert(K <= 128, "batched gather area");
        uint32_t* s = (uint32_t*)big();
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (wr[k]) s[k] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) out[k] = s[k];
        par ^= 1u;
    }
    __device__ static uint64_t clock() { return __builtin_amdgcn_s_memtime(); }
    __device__ static uint32_t gload(const uint32_t* p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static void gstore(uint32_t* p, uint32_t v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // 16-byte aligned row store (global_store_dwordx4; L1 is write-through, readers use L2 loads)
    __device__ static void gstore4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
        *(uint4*)p = make_uint4(a, b, c, d);
    }
    __device__ static void lds_add(uint32_t* p, uint32_t v) { atomicAdd(p, v); }
    __device__ static void gadd64(uint64_t* p, uint64_t v) { atomicAdd((unsigned long long*)p, (unsigned long long)v); }
};

// launchers (each in its own translation unit)
// general kernel, NEED_SEED x MODE_FULL / MODE_EXT builds (kern_general.hip, compiled four times)
hipError_t launch_general_0_0(uint32_t seg, dim3 grid, size_t lds, hipStream_t s, const Params& p);
hipError_t launch_general_0_1(uint32_t seg, dim3 grid, size_t lds, hipStream_t s, const Params& p);
hipError_t launch_general_1_0(uint32_t seg, dim3 grid, size_t lds, hipStream_t s, const Params& p);
hipError_t launch_general_1_1(uint32_t seg, dim3 grid, size_t lds, hipStream_t s, const Params& p);
inline hipError_t launch_general(bool need_seed, bool ext, uint32_t seg, dim3 grid, size_t lds, hipStream_t s,
                                 const Params& p) {
    if (need_seed) return ext ? launch_general_1_1(seg, grid, lds, s, p) : launch_general_1_0(seg, grid, lds, s, p);
    return ext ? launch_general_0_1(seg, grid, lds, s, p) : launch_general_0_0(seg, grid, lds, s, p);
}
hipError_t launch_fast(dim3 grid, hipStream_t s, const Params& p);               // kern_fast.hip
// block-hash pass of heights [x0, x0 + rows) for n instances (kern_fast.hip): the header suffix rows,
// then the prev_hash chains that splice them
// (loop: a thread per instance over its heights instead of a thread per (instance, height))
hipError_t launch_hash_suffix(uint32_t n, uint32_t x0, uint32_t rows, uint32_t* sfx, bool loop, hipStream_t s,
                              Params p);
// chain kernels: lane pairs (small shards), one wave per instance (kw50, A/B arm), one lane per instance (large)
constexpr uint32_t CHAIN_KERNEL_PAIR = 0, CHAIN_KERNEL_WAVE = 1, CHAIN_KERNEL_LANE = 2;
hipError_t launch_hash_chain(uint32_t n, uint32_t x0, uint32_t rows, uint32_t* sfx, uint32_t kind, hipStream_t s,
                             Params p);
// the chains of up to CHAIN_MAX_SETS launches (row-table sets) of n instances each, heights 1..H, as one kernel
constexpr uint32_t CHAIN_MAX_SETS = 32;
struct ChainSets {
    uint32_t count;
    const uint32_t* sfx[CHAIN_MAX_SETS];
    const uint32_t* ch[CHAIN_MAX_SETS];
    uint8_t* hash[CHAIN_MAX_SETS];
    // predicted chains (big-endian seeds, N = 64): each launch's instance ids, its Byzantine masks,
    // first height whose recorded block differs from the prediction, recorded rows
    uint32_t first[CHAIN_MAX_SETS];
    uint64_t* byz[CHAIN_MAX_SETS];
    uint32_t* bad[CHAIN_MAX_SETS];
    const uint32_t* rec[CHAIN_MAX_SETS];
    uint32_t* pred[CHAIN_MAX_SETS];       // [n][H] SPEC_VALID | proposer | variant << 16 of each height, or 0
};
// chain kernel modes (Params::chain_mode)
constexpr uint32_t CHAIN_RECORDED = 0;    // heights [x0, min(ch, x0 + rows - 1)] from the recorded rows' suffixes
constexpr uint32_t CHAIN_PREDICTED = 1;   // heights 1..H of the predicted blocks, up to the first without one
constexpr uint32_t CHAIN_REPAIR = 2;      // heights [bad, ch]: from the first recorded block that differs
hipError_t launch_hash_chain_batch(uint32_t n, const ChainSets& cs, uint32_t kind, hipStream_t s, Params p);
// predicted chains: per launch of the batch, the Byzantine masks + the predicted suffix rows (one launch, on
// the stream its chains will run on, ahead of its consensus kernel's completion); per batch, the check of the
// recorded blocks against the predictions (rewriting the suffix rows that differ)
hipError_t launch_spec_suffix(uint32_t n, const ChainSets& cs, hipStream_t s, const Params& p);
hipError_t launch_spec_verify(uint32_t n, const ChainSets& cs, hipStream_t s, const Params& p);
// little-endian seeds, N = 64: the predicted canonical blocks into p.spec / p.hash (kern_fast.hip)
hipError_t launch_seed_chain(uint32_t n, hipStream_t s, const Params& p);
hipError_t launch_resume(dim3 grid, size_t lds, hipStream_t s, const Params& p);  // kern_resume.hip

}  // namespace bft
