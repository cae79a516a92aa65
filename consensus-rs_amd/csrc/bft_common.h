// bft_common.h — definitions shared by the HIP kernels and the host code of libbftsim.
//
// Everything here is a restatement of SPEC.md (the seeded schedule, block identity, quorum,
// proposer selection, header encoding) written for gfx950 lanes: 32/64-bit integer ops only.
// Compiled by hipcc for the device and by the host compiler for libbftsim's host helpers and for
// the CPU wave emulator used by the tests.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BFT_FN __host__ __device__ inline
#else
#define BFT_FN inline
#endif

namespace bft {

// ---------------------------------------------------------------------------------------------
// Parameters of one launch (plain data, copied by value into the kernel argument buffer).
// ---------------------------------------------------------------------------------------------
struct Params {
    uint32_t n;               // validators per instance (1..256)
    uint32_t seg;             // lanes per instance segment: power of two >= n (> 64: one workgroup)
    uint32_t heights;         // H
    uint32_t hcap;            // height limit of the record tables (H + margin): x >= hcap freezes
    uint32_t max_ticks;
    uint32_t block_period;
    uint64_t genesis_time;
    uint64_t seed;
    uint32_t thr16;           // drop threshold (0 = no drops)
    uint32_t byz_count;
    uint32_t crash_thr32;     // proposer-crash threshold (0 = none)
    uint32_t crash_on;
    uint32_t phase_cap;
    uint32_t need_seed;       // N not a power of two: proposer seeds need block hashes in-kernel
    uint64_t silent_mask[4];
    uint32_t first_instance;
    uint32_t n_instances;
    uint32_t genesis_seed;
    uint32_t fast;            // 1: closed-form phase fast paths (0: one message at a time)
    const uint8_t* addresses;         // n*20
    const uint8_t* genesis_hash;      // 32
    // outputs
    uint32_t* committed_height;       // [n_inst]
    uint32_t* flags;                  // [n_inst]
    uint32_t* ticks;                  // [n_inst]
    uint64_t* views;                  // [n_inst]
    uint32_t* rec;                    // [n_inst * hcap * 4] {round, prop|var<<16|set<<24, T, seed}
    uint8_t* hash;                    // [n_inst * hcap * 32]
    uint64_t* trace;                  // optional [n_inst][trace_ticks][n] state digests
    uint32_t trace_ticks;
    uint32_t pad1;
    uint64_t* stamps;                 // diagnostic builds only (BFT_STAMPS): [waves][8] cycles per section
    uint64_t* hist;                   // [130] summed rounds-to-commit (65) + commit-latency (65) bins
    uint32_t window_mask;             // 0: rec/hash rows for every height; else ring of window_mask+1 rows
    uint32_t rows;                    // rec/hash rows per instance (hcap, or the ring size)
    uint32_t* rcs;                    // RoundChangeSet tables: per wave / workgroup rcs_words(seg, rcs_k) words
    uint32_t q;                       // floor(2N/3) (two_thirds_majority, validator.rs:149-154)
    uint32_t nmask;                   // N-1 when N is a power of two (x mod N = x & nmask), else 0
    // FAST launches (bft_wave.h): instances that need the general path are saved and resumed
    uint32_t* resume_flags;           // [n_inst] 1 = saved by the FAST kernel
    uint32_t* resume_q;               // [2 + n_inst] (device): hand-over count, queue head, instance list
    uint32_t* resume_hint;            // host-mapped word: the last resume kernel's count (sizes the next grid)
    uint32_t* save;                   // [n_inst * 64][SAVE_WORDS] per-lane state
    uint64_t save_stride;             // unused (kept for the layout)
    uint32_t resume_mode;             // CPU emulator only: run the MODE_RESUME body
    uint32_t seed_le;                 // BFTSIM_SEED_LE: randon_seed reads U128 little-endian (bftsim.h)
    uint32_t backlog_replay;          // BFTSIM_BACKLOG_REPLAY (SPEC.md §10)
    uint32_t pad3;
    uint32_t* backlog;                // replay mode: per wave / workgroup [S slots][5 words][L lanes]
    // real-crypto mode (SPEC.md §11): every consensus message broadcast is logged for the batched
    // sign / recover pass; a forged sender's messages reach no receiver
    uint32_t* mlog;                   // [n_inst][mlog_cap][MLOG_WORDS] (nullptr: mode off)
    uint32_t* mlog_n;                 // [n_inst] messages logged (may exceed mlog_cap: overflow)
    uint32_t mlog_cap;
    uint32_t pad4;
    uint64_t forged[4];               // validators signing with a key that is not theirs
    uint32_t* vsnap;                  // [n_inst][seg][8] each lane's commit set at its last Core commit
    uint32_t* votes;                  // [n_inst][rows][8] the canonical committer's commit set per height
    // block-hash pass (kern_fast.hip): header suffix rows of heights [sfx_x0, sfx_x0 + sfx_rows)
    uint32_t* sfx;                    // [n_inst][sfx_rows][SFX_DWORDS]
    uint32_t sfx_x0, sfx_rows;
    uint32_t chain_prio;              // s_setprio of the block-hash chain waves (0..3)
    uint32_t fast_lds_pad;            // A/B arms only (BFTSIM_TESTING + BFTSIM_FAST_LDS_PAD): extra LDS per FAST wave
    uint32_t rcs_k;                   // RoundChangeSet rounds per validator (bftsim_set_rcs_capacity)
    uint32_t pad5;
    // little-endian seeds, N = 64: the predicted canonical blocks (bft_seed_chain_kernel; nullptr: none)
    uint32_t* spec;                   // [heights + 1][n_inst] spec_word or 0
    // block-hash chains (kern_fast.hip): CHAIN_RECORDED / CHAIN_PREDICTED / CHAIN_REPAIR (bft_hip.h)
    uint32_t chain_mode;
    uint32_t chain_grid;              // lane-chain kernel: at most this many (persistent) waves; 0: one per task
    uint32_t chain_inline;            // lane-chain kernel: each lane encodes its suffixes (no suffix rows)
    uint32_t fast_prio;               // s_setprio of the FAST kernel + 1 (0: its default, 2; BFTSIM_FAST_PRIO)
};
constexpr uint32_t RCS_DEFAULT_K = 16, RCS_MAX_K = 4096;
// one logged broadcast: {tick, phase | code << 8 | sender << 16, height, round, block id lo, hi,
// flags (MLOG_*), 0}; code = MessageType 1..4 (Preprepare .. RoundChange)
constexpr uint32_t MLOG_WORDS = 8;
constexpr uint32_t MLOG_FORGED = 1u, MLOG_WILD = 2u, MLOG_EQUIV = 4u, MLOG_OLD = 8u;

// flags (same bits as the oracle)
constexpr uint32_t FLAG_SAFETY = 1u, FLAG_PHASE_CAP = 2u, FLAG_CORE_PANIC = 4u, FLAG_OUTBOX = 8u,
                   FLAG_TIMEOUT = 16u, FLAG_RCS_OVERFLOW = 32u, FLAG_WINDOW = 64u;
constexpr uint32_t HIST_BINS = 130;     // [0,65) rounds-to-commit, [65,130) commit latency (ticks)
constexpr int NSTAMP = 18;               // diagnostic builds (BFT_STAMPS): sections per wave

// State (src/protocol/mod.rs:25-30)
constexpr uint32_t ST_ACCEPT_REQUEST = 1, ST_PREPREPARED = 2, ST_PREPARED = 3, ST_COMMITTED = 4;

// MessageType (src/protocol/mod.rs:36-41; ordered Preprepare < Prepare < Commit < RoundChange, the
// derive(PartialOrd) the reference tests at :241-250) and the error classes of Core::check_message.
constexpr int MT_PREPREPARE = 1, MT_PREPARE = 2, MT_COMMIT = 3, MT_ROUND_CHANGE = 4;
constexpr int CM_OK = 0, CM_UNKNOWN = 1, CM_FUTURE_BLOCK = 2, CM_OLD = 3, CM_FUTURE_MSG = 4;
// Core::check_message (core.rs:366-399): a message of `code` for height `vh` at a Core of height `h`
// in state `st`. RoundChange compares only the height; the others need the same height, and in
// AcceptRequest only a Preprepare (the smallest MessageType) is accepted. The round is not compared.
BFT_FN int check_message_class(int code, uint32_t vh, uint32_t h, uint32_t st) {
    if (vh == 0) return CM_UNKNOWN;
    if (code == MT_ROUND_CHANGE) { if (vh > h) return CM_FUTURE_BLOCK; if (vh < h) return CM_OLD; return CM_OK; }
    if (vh > h) return CM_FUTURE_BLOCK;
    if (vh < h) return CM_OLD;
    if (st == ST_ACCEPT_REQUEST) return code > MT_PREPREPARE ? CM_FUTURE_MSG : CM_OK;
    return CM_OK;
}

// ---------------------------------------------------------------------------------------------
// Block identity (SPEC.md §4) packed in 64 bits:
//   [0,24) height  [24,33) proposer  [33] variant  [34] valid  [35,64) time tick
// Equality ignores the time tick (a function of height and proposer).
// ---------------------------------------------------------------------------------------------
constexpr uint64_t BLK_NONE = 0;
constexpr uint64_t BLK_VALID = 1ull << 34;
constexpr uint64_t BLK_ID_MASK = (1ull << 35) - 1;      // height|proposer|variant|valid
constexpr uint64_t BLK_HP_MASK = (1ull << 33) - 1;      // height|proposer
BFT_FN uint64_t blk_make(uint32_t h, uint32_t prop, uint32_t var, uint32_t T) {
    return (uint64_t)(h & 0xffffffu) | ((uint64_t)(prop & 0x1ffu) << 24) | ((uint64_t)(var & 1u) << 33) |
           BLK_VALID | ((uint64_t)T << 35);
}
BFT_FN bool blk_valid(uint64_t b) { return (b & BLK_VALID) != 0; }
BFT_FN uint32_t blk_h(uint64_t b) { return (uint32_t)(b & 0xffffffu); }
BFT_FN uint32_t blk_prop(uint64_t b) { return (uint32_t)((b >> 24) & 0x1ffu); }
BFT_FN uint32_t blk_var(uint64_t b) { return (uint32_t)((b >> 33) & 1u); }
BFT_FN uint32_t blk_T(uint64_t b) { return (uint32_t)(b >> 35); }
BFT_FN bool blk_eq(uint64_t a, uint64_t b) {
    return blk_valid(a) && blk_valid(b) && ((a ^ b) & BLK_ID_MASK) == 0;
}
// 32-bit form of the id without the time tick: height (22 bits) | proposer (8) | variant | valid.
// Equal for two valid blocks iff blk_eq (heights < 2^22 by the hcap limit, proposers < 256); 0 for
// BLK_NONE.
BFT_FN uint32_t blk_d32(uint64_t b) {
    if (!blk_valid(b)) return 0;
    return (uint32_t)(b & 0x3fffffu) | (blk_prop(b) << 22) | (blk_var(b) << 30) | 0x80000000u;
}
// digest comparison; a Byzantine vote's wildcard digest matches both variants (SPEC.md §6)
BFT_FN bool digest_match(uint64_t d, bool wild, uint64_t t) {
    if (!blk_valid(d) || !blk_valid(t)) return false;
    if (((d ^ t) & BLK_HP_MASK) != 0) return false;
    return wild || blk_var(d) == blk_var(t);
}

// ---------------------------------------------------------------------------------------------
// Sender bitmaps of NW 64-bit words (MessageManage / RoundChangeSet sets, a5/a7 of SURVEY §8):
// bit s = validator s. NW = 1 for N <= 64 (the code below then reduces to plain uint64_t
// arithmetic); 2 or 4 for N <= 128 / 256. Word selection by a per-lane index is a select chain,
// never a dynamically indexed register array (which would go to scratch).
// ---------------------------------------------------------------------------------------------
template <int NW>
struct Bits {
    uint64_t w[NW];
    BFT_FN static Bits zero() { Bits b; for (int k = 0; k < NW; ++k) b.w[k] = 0; return b; }
    BFT_FN static Bits from(uint64_t x) { Bits b = zero(); b.w[0] = x; return b; }
    BFT_FN static Bits from(const Bits& x) { return x; }
    BFT_FN static Bits low(uint32_t n) {          // bits [0, n), n <= 64*NW
        if (NW == 1) { Bits b; b.w[0] = n >= 64u ? ~0ull : ((1ull << n) - 1ull); return b; }
        Bits b;
        for (int k = 0; k < NW; ++k) {
            uint32_t lo = 64u * (uint32_t)k;
            b.w[k] = n >= lo + 64u ? ~0ull : (n <= lo ? 0ull : ((1ull << (n - lo)) - 1ull));
        }
        return b;
    }
    BFT_FN static Bits bit(uint32_t i) {
        Bits b;
        for (int k = 0; k < NW; ++k) b.w[k] = ((i >> 6) == (uint32_t)k) ? (1ull << (i & 63u)) : 0ull;
        return b;
    }
    BFT_FN uint64_t word(int i) const {          // 0 outside [0, NW)
        uint64_t x = 0;
        for (int k = 0; k < NW; ++k) x = (i == k) ? w[k] : x;
        return x;
    }
    BFT_FN bool get(uint32_t i) const { return (word((int)(i >> 6)) >> (i & 63u)) & 1ull; }
    // value selects, not a conditional store: LLVM turns `if (k == i/64) w[k] |= b` into a store at the
    // dynamic index w[i/64], which forces the whole kernel object into scratch (S = 256: 840 B/lane)
    BFT_FN void set(uint32_t i) {
        const uint64_t b = 1ull << (i & 63u);
        for (int k = 0; k < NW; ++k) w[k] |= ((i >> 6) == (uint32_t)k) ? b : 0ull;
    }
    BFT_FN bool any() const { uint64_t x = 0; for (int k = 0; k < NW; ++k) x |= w[k]; return x != 0; }
    BFT_FN bool none() const { return !any(); }
    BFT_FN uint32_t popc() const {
        uint32_t c = 0;
        for (int k = 0; k < NW; ++k) c += (uint32_t)__builtin_popcountll(w[k]);
        return c;
    }
    BFT_FN uint32_t ctz_nz() const {             // lowest set bit; the set must be non-empty
        if (NW == 1) return (uint32_t)__builtin_ctzll(w[0]);
        return ctz();
    }
    BFT_FN uint32_t ctz() const {                // lowest set bit, 64*NW if none
        uint32_t r = 64u * NW;
        for (int k = NW - 1; k >= 0; --k) r = w[k] ? 64u * (uint32_t)k + (uint32_t)__builtin_ctzll(w[k]) : r;
        return r;
    }
    BFT_FN uint32_t hibit() const {              // highest set bit, 0 if none
        uint32_t r = 0;
        for (int k = 0; k < NW; ++k) r = w[k] ? 64u * (uint32_t)k + 63u - (uint32_t)__builtin_clzll(w[k]) : r;
        return r;
    }
    BFT_FN void clear_lowest() {
        bool done = false;
        for (int k = 0; k < NW; ++k) {
            bool t = !done && w[k] != 0;
            w[k] = t ? (w[k] & (w[k] - 1ull)) : w[k];
            done = done || t;
        }
    }
    BFT_FN Bits shr(uint32_t s) const {          // s in [0, 64*NW]
        if (NW == 1) { Bits b; b.w[0] = s >= 64u ? 0ull : (w[0] >> s); return b; }
        Bits b;
        int q = (int)(s >> 6);
        uint32_t r = s & 63u;
        for (int j = 0; j < NW; ++j) {
            uint64_t lo = word(j + q), hi = word(j + q + 1);
            b.w[j] = r ? ((lo >> r) | (hi << (64u - r))) : lo;
        }
        return b;
    }
    BFT_FN Bits shl(uint32_t s) const {          // s in [0, 64*NW]
        if (NW == 1) { Bits b; b.w[0] = s >= 64u ? 0ull : (w[0] << s); return b; }
        Bits b;
        int q = (int)(s >> 6);
        uint32_t r = s & 63u;
        for (int j = 0; j < NW; ++j) {
            uint64_t lo = word(j - q), lo2 = word(j - q - 1);
            b.w[j] = r ? ((lo << r) | (lo2 >> (64u - r))) : lo;
        }
        return b;
    }
    BFT_FN Bits operator&(const Bits& o) const { Bits b; for (int k = 0; k < NW; ++k) b.w[k] = w[k] & o.w[k]; return b; }
    BFT_FN Bits operator|(const Bits& o) const { Bits b; for (int k = 0; k < NW; ++k) b.w[k] = w[k] | o.w[k]; return b; }
    BFT_FN Bits operator^(const Bits& o) const { Bits b; for (int k = 0; k < NW; ++k) b.w[k] = w[k] ^ o.w[k]; return b; }
    BFT_FN Bits operator~() const { Bits b; for (int k = 0; k < NW; ++k) b.w[k] = ~w[k]; return b; }
    BFT_FN Bits& operator|=(const Bits& o) { for (int k = 0; k < NW; ++k) w[k] |= o.w[k]; return *this; }
    BFT_FN Bits& operator&=(const Bits& o) { for (int k = 0; k < NW; ++k) w[k] &= o.w[k]; return *this; }
    BFT_FN bool operator==(const Bits& o) const { uint64_t x = 0; for (int k = 0; k < NW; ++k) x |= w[k] ^ o.w[k]; return x == 0; }
    BFT_FN bool operator!=(const Bits& o) const { return !(*this == o); }
};

// ---------------------------------------------------------------------------------------------
// Seeded randomness (SPEC.md §3, §5)
// ---------------------------------------------------------------------------------------------
constexpr uint32_t DOM_DROP = 1, DOM_SPLIT = 2, DOM_CRASH = 3, DOM_BYZ = 4, DOM_TX = 5, DOM_TX2 = 6;

BFT_FN uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// A value held in a scalar register that the compiler must treat as unknown at this point (no-op on
// the host). Used on the launch seed before Philox calls inside the kernels' tick / phase loops:
// otherwise LLVM hoists the 20-word key schedule (and partial rounds on constant counters) out of the
// loops and keeps it live in SGPRs across the whole body, which spills.
#if defined(__HIP_DEVICE_COMPILE__)
#define BFT_OPAQUE_SGPR(x) asm volatile("" : "+s"(x))
#define BFT_OPAQUE_VGPR(x) asm volatile("" : "+v"(x))   // forces the value (and what is computed from it) onto the vector lanes
#else
#define BFT_OPAQUE_SGPR(x) do { } while (0)
#define BFT_OPAQUE_VGPR(x) do { } while (0)
#endif

// Philox4x32-10 (Salmon et al. SC'11); 10 rounds of two 32x32→64 multiplies.
BFT_FN void philox(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // each 32x32 product as one 64-bit result: one v_mad_u64_u32 instead of v_mul_hi_u32 +
        // v_mul_lo_u32 (all three are quarter-rate on the vector ALU)
        const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// a ^ b ^ c as one v_bitop3_b32 on gfx950 (the compiler leaves 3-input XORs as two v_xor_b32)
BFT_FN uint32_t pxor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

// The drop draw of deliver_mask: philox(seed, inst, tick, c2, DOM_DROP) with c2 = (phase << 24) |
// (recv << 8) | j, computed with the products of wave-uniform words taken out of the vector work:
// * round 1: c0 = inst is uniform, so its product is; the fields of c2 are disjoint, so
//   c2 · M1 = base1 + j · M1 with base1 = ((phase << 24) | (recv << 8)) · M1 (once per phase): one 64-bit add;
// * round 2: c2 = hi(inst · M0) ^ DOM_DROP ^ k1 is uniform again, so that product is too.
// Rounds 3-10 are Philox's, each round's two 3-input XORs one v_bitop3_b32 apiece. Same words as philox().
BFT_FN void philox_drop(uint64_t seed, uint32_t inst, uint32_t tick, uint64_t base1, uint32_t j, uint32_t out[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    // the key schedule from opaque scalars: one s_add per key and round here, instead of 20 words LLVM would
    // hoist out of the kernel's loops, spill into VGPR lanes and read back with v_readlane (general kernel)
    BFT_OPAQUE_SGPR(k0);
    BFT_OPAQUE_SGPR(k1);
    const uint64_t q0 = (uint64_t)inst * 0xD2511F53u;                  // uniform
    const uint64_t q1 = base1 + (uint64_t)j * 0xCD9E8D57u;             // = c2 * M1
    uint32_t c0 = pxor3((uint32_t)(q1 >> 32), tick, k0), c1 = (uint32_t)q1;
    uint32_t c2 = (uint32_t)(q0 >> 32) ^ DOM_DROP ^ k1, c3 = (uint32_t)q0;   // uniform
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
        const uint32_t n0 = pxor3((uint32_t)(p1 >> 32), c1, k0), n2 = pxor3((uint32_t)(p0 >> 32), c3, k1);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
BFT_FN uint64_t philox_drop_base(uint32_t phase, uint32_t recv) {
    return (uint64_t)((phase << 24) | (recv << 8)) * 0xCD9E8D57u;
}

BFT_FN uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// first sender of the receiver's rotated delivery order (SPEC.md §3); the hash chain is split so
// the kernel computes the per-instance and per-tick parts once
BFT_FN uint32_t offset_inst_part(uint64_t seed, uint32_t inst) { return lowbias32(inst ^ (uint32_t)seed); }
BFT_FN uint32_t offset_tick_part(uint32_t inst_part, uint32_t tick) { return lowbias32(inst_part ^ tick); }
BFT_FN uint32_t offset_from_parts(uint64_t seed, uint32_t n, uint32_t tick_part, uint32_t phase, uint32_t recv) {
    return mulhi32(lowbias32(tick_part ^ ((phase << 16) | recv) ^ (uint32_t)(seed >> 32)), n);
}
BFT_FN uint32_t delivery_offset(uint64_t seed, uint32_t n, uint32_t inst, uint32_t tick, uint32_t phase,
                                uint32_t recv) {
    return offset_from_parts(seed, n, offset_tick_part(offset_inst_part(seed, inst), tick), phase, recv);
}

// N-bit delivery mask of receiver `recv` for (tick, phase); self always delivered. Only the bits of the
// senders in `present` are meaningful: the Philox draw of an 8-sender block with no sender present is
// skipped (its bits stay 0), which leaves every delivered message unchanged (SPEC.md §3 fixes the draw of
// each (receiver, block), not the order of the draws).
// SKIP = false computes every block (the skip is a branch in the loop; for small segments, where one or
// two blocks cover the instance, it only costs registers)
// the drop bits of one 8-sender block from its Philox words: bit i = chunk i (16 bits) >= thr16
BFT_FN uint64_t drop_byte(const uint32_t w[4], uint32_t thr16) {
    uint64_t byte = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t u = (w[i >> 1] >> (16 * (i & 1))) & 0xffffu;
        if (u >= thr16) byte |= 1ull << i;
    }
    return byte;
}
template <int NW>
BFT_FN void place_byte(Bits<NW>& m, uint32_t j, uint64_t byte) {
    for (int k = 0; k < NW; ++k)
        if ((j >> 3) == (uint32_t)k) m.w[k] |= byte << (8u * (j & 7u));
}
template <int NW, bool SKIP = true>
BFT_FN Bits<NW> deliver_mask(uint64_t seed, uint32_t n, uint32_t thr16, uint32_t inst, uint32_t tick,
                             uint32_t phase, uint32_t recv, const Bits<NW>& present) {
    Bits<NW> all = Bits<NW>::low(n);
    if (thr16 == 0) return all;
    Bits<NW> m = Bits<NW>::zero();
    const uint64_t base1 = philox_drop_base(phase, recv);
    // one block at a time: two independent chains interleaved (two blocks per iteration) measured no faster on
    // drop64 and 18 % slower on cfg2, whose segments need one block (profiles/r04/ab_drop_pairs)
    for (uint32_t j = 0; 8 * j < n; ++j) {
        if (SKIP && ((present.word((int)(j >> 3)) >> (8u * (j & 7u))) & 0xffull) == 0) continue;
        uint32_t w[4];
        philox_drop(seed, inst, tick, base1, j, w);   // = philox(seed, inst, tick, (phase << 24) | (recv << 8) | j, DOM_DROP)
        place_byte(m, j, drop_byte(w, thr16));
    }
    m &= all;
    m.set(recv);
    return m;
}

BFT_FN uint32_t split_bit(uint64_t seed, uint32_t inst, uint32_t h, uint32_t r, uint32_t v) {
    uint32_t w[4];
    philox(seed, inst, h, r, DOM_SPLIT | ((v >> 7) << 8), w);
    uint32_t vv = v & 127u;
    uint32_t word = (vv >> 5) == 0 ? w[0] : (vv >> 5) == 1 ? w[1] : (vv >> 5) == 2 ? w[2] : w[3];
    return (word >> (vv & 31u)) & 1u;
}

BFT_FN bool proposer_crashed(uint64_t seed, uint32_t thr32, uint32_t on, uint32_t inst, uint32_t h, uint32_t r) {
    if (!on) return false;
    uint32_t w[4];
    philox(seed, inst, h, r, DOM_CRASH, w);
    return w[0] < thr32;
}

// ---------------------------------------------------------------------------------------------
// Keccak-256 over the MessagePack header (SPEC.md §7).
// ---------------------------------------------------------------------------------------------
BFT_FN uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

BFT_FN void keccak_f1600_u64(uint64_t a[25]);
// the round constants as 32-bit halves: a constant-memory table on the device (a local array indexed
// in the round loop would be copied into scratch memory at every call)
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const uint32_t KECCAK_RC_LO[24] = {
    0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u, 0x80008081u, 0x00008009u,
    0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au, 0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
    0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ static const uint32_t KECCAK_RC_HI[24] = {
    0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0x80000000u,
    0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u};
#else
static const uint32_t KECCAK_RC_LO[24] = {
    0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u, 0x80008081u, 0x00008009u,
    0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au, 0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
    0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
static const uint32_t KECCAK_RC_HI[24] = {
    0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0x80000000u,
    0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u};
#endif
#if defined(__HIP_DEVICE_COMPILE__)
__host__ inline void keccak_f1600(uint64_t a[25]) { keccak_f1600_u64(a); }
// gfx950 form: the state as 32-bit halves; rotations are two v_alignbit_b32 (funnel shifts),
// the theta parities two 3-input XORs (v_bitop3_b32 0x96) per half, chi one v_bitop3_b32 per half.
__device__ inline uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
template <int N>
__device__ inline void rotl_halves(uint32_t lo, uint32_t hi, uint32_t& ol, uint32_t& oh) {
    if constexpr (N == 0) { ol = lo; oh = hi; }
    else if constexpr (N == 32) { ol = hi; oh = lo; }
    else if constexpr (N < 32) { oh = __builtin_amdgcn_alignbit(hi, lo, 32 - N); ol = __builtin_amdgcn_alignbit(lo, hi, 32 - N); }
    else { oh = __builtin_amdgcn_alignbit(lo, hi, 64 - N); ol = __builtin_amdgcn_alignbit(hi, lo, 64 - N); }
}
__device__ inline void keccak_f1600(uint64_t a[25]) {
    uint32_t L[25], H[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) { L[i] = (uint32_t)a[i]; H[i] = (uint32_t)(a[i] >> 32); }
#pragma unroll 1
    for (int rnd = 0; rnd < 24; ++rnd) {
        uint32_t cl[5], ch[5], dl[5], dh[5], bl[25], bh[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            cl[x] = xor3_32(xor3_32(L[x], L[x + 5], L[x + 10]), L[x + 15], L[x + 20]);
            ch[x] = xor3_32(xor3_32(H[x], H[x + 5], H[x + 10]), H[x + 15], H[x + 20]);
        }
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            uint32_t rl, rh;
            rotl_halves<1>(cl[(x + 1) % 5], ch[(x + 1) % 5], rl, rh);
            dl[x] = cl[(x + 4) % 5] ^ rl;
            dh[x] = ch[(x + 4) % 5] ^ rh;
        }
        // theta + rho + pi: b[y + 5*((2x+3y)%5)] = rotl(a[x+5y] ^ d[x], r[x+5y])
#define BFT_RHO(i, n, j) rotl_halves<n>(L[i] ^ dl[(i) % 5], H[i] ^ dh[(i) % 5], bl[j], bh[j]);
        BFT_RHO(0, 0, 0) BFT_RHO(1, 1, 10) BFT_RHO(2, 62, 20) BFT_RHO(3, 28, 5) BFT_RHO(4, 27, 15)
        BFT_RHO(5, 36, 16) BFT_RHO(6, 44, 1) BFT_RHO(7, 6, 11) BFT_RHO(8, 55, 21) BFT_RHO(9, 20, 6)
        BFT_RHO(10, 3, 7) BFT_RHO(11, 10, 17) BFT_RHO(12, 43, 2) BFT_RHO(13, 25, 12) BFT_RHO(14, 39, 22)
        BFT_RHO(15, 41, 23) BFT_RHO(16, 45, 8) BFT_RHO(17, 15, 18) BFT_RHO(18, 21, 3) BFT_RHO(19, 8, 13)
        BFT_RHO(20, 18, 14) BFT_RHO(21, 2, 24) BFT_RHO(22, 61, 9) BFT_RHO(23, 56, 19) BFT_RHO(24, 14, 4)
#undef BFT_RHO
        // chi
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
#pragma unroll
    for (int i = 0; i < 25; ++i) a[i] = (uint64_t)L[i] | ((uint64_t)H[i] << 32);
}
#else
BFT_FN void keccak_f1600(uint64_t a[25]) { keccak_f1600_u64(a); }
#endif
// the plain 64-bit form (host code, the CPU emulator)
BFT_FN void keccak_f1600_u64(uint64_t a[25]) {
    const uint64_t RC[24] = {
        0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
        0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
        0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
        0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
        0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
        0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
#pragma unroll 1
    for (int rnd = 0; rnd < 24; ++rnd) {
        uint64_t c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];
        uint64_t c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];
        uint64_t c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];
        uint64_t c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];
        uint64_t c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];
        uint64_t d0 = c4 ^ rotl64(c1, 1), d1 = c0 ^ rotl64(c2, 1), d2 = c1 ^ rotl64(c3, 1);
        uint64_t d3 = c2 ^ rotl64(c4, 1), d4 = c3 ^ rotl64(c0, 1);
        // theta + rho + pi (b[y + 5*((2x+3y)%5)] = rotl(a[x+5y], r[x+5y]))
        uint64_t b0 = a[0] ^ d0;
        uint64_t b10 = rotl64(a[1] ^ d1, 1);
        uint64_t b20 = rotl64(a[2] ^ d2, 62);
        uint64_t b5 = rotl64(a[3] ^ d3, 28);
        uint64_t b15 = rotl64(a[4] ^ d4, 27);
        uint64_t b16 = rotl64(a[5] ^ d0, 36);
        uint64_t b1 = rotl64(a[6] ^ d1, 44);
        uint64_t b11 = rotl64(a[7] ^ d2, 6);
        uint64_t b21 = rotl64(a[8] ^ d3, 55);
        uint64_t b6 = rotl64(a[9] ^ d4, 20);
        uint64_t b7 = rotl64(a[10] ^ d0, 3);
        uint64_t b17 = rotl64(a[11] ^ d1, 10);
        uint64_t b2 = rotl64(a[12] ^ d2, 43);
        uint64_t b12 = rotl64(a[13] ^ d3, 25);
        uint64_t b22 = rotl64(a[14] ^ d4, 39);
        uint64_t b23 = rotl64(a[15] ^ d0, 41);
        uint64_t b8 = rotl64(a[16] ^ d1, 45);
        uint64_t b18 = rotl64(a[17] ^ d2, 15);
        uint64_t b3 = rotl64(a[18] ^ d3, 21);
        uint64_t b13 = rotl64(a[19] ^ d4, 8);
        uint64_t b14 = rotl64(a[20] ^ d0, 18);
        uint64_t b24 = rotl64(a[21] ^ d1, 2);
        uint64_t b9 = rotl64(a[22] ^ d2, 61);
        uint64_t b19 = rotl64(a[23] ^ d3, 56);
        uint64_t b4 = rotl64(a[24] ^ d4, 14);
        // chi
        a[0] = b0 ^ (~b1 & b2);   a[1] = b1 ^ (~b2 & b3);   a[2] = b2 ^ (~b3 & b4);
        a[3] = b3 ^ (~b4 & b0);   a[4] = b4 ^ (~b0 & b1);
        a[5] = b5 ^ (~b6 & b7);   a[6] = b6 ^ (~b7 & b8);   a[7] = b7 ^ (~b8 & b9);
        a[8] = b8 ^ (~b9 & b5);   a[9] = b9 ^ (~b5 & b6);
        a[10] = b10 ^ (~b11 & b12); a[11] = b11 ^ (~b12 & b13); a[12] = b12 ^ (~b13 & b14);
        a[13] = b13 ^ (~b14 & b10); a[14] = b14 ^ (~b10 & b11);
        a[15] = b15 ^ (~b16 & b17); a[16] = b16 ^ (~b17 & b18); a[17] = b17 ^ (~b18 & b19);
        a[18] = b18 ^ (~b19 & b15); a[19] = b19 ^ (~b15 & b16);
        a[20] = b20 ^ (~b21 & b22); a[21] = b21 ^ (~b22 & b23); a[22] = b22 ^ (~b23 & b24);
        a[23] = b23 ^ (~b24 & b20); a[24] = b24 ^ (~b20 & b21);
        a[0] ^= RC[rnd];
    }
}

BFT_FN uint32_t hexdigit(uint32_t x) { return x < 10 ? 48u + x : 87u + x; }

// tx_hash words of a candidate (SPEC.md §5, domain TX)
BFT_FN void tx_hash_words(uint64_t seed, uint32_t inst, uint32_t h, uint32_t prop, uint32_t var, uint32_t w[8]) {
    philox(seed, inst, h, (prop << 8) | var, DOM_TX, w);
    philox(seed, inst, h, (prop << 8) | var, DOM_TX2, w + 4);
}

constexpr uint32_t LANE_HASH_BUF = 408;    // 3 rate blocks; the header is at most 274 bytes
constexpr uint32_t HDR_WORDS = LANE_HASH_BUF / 8;

// The MessagePack header (SPEC.md §7) is produced as a stream of little-endian 64-bit words, not
// byte by byte: a field contributes one `put` of up to 8 bytes into a 64-bit accumulator, and every
// completed word is stored once (LDS on the device). The byte layout is exactly the one of
// host_header_bytes() (bft_host.h), which the tests compare against the msgpack package.
struct HdrWriter {
    uint64_t* wb;        // HDR_WORDS words, 8-aligned
    uint32_t* sb;        // or: dword k of the stream at sb[k * stride] (the block-hash pass's suffix rows)
    uint32_t stride;
    uint64_t acc;
    uint32_t fill;       // bytes in acc, 0..7
    uint32_t wi;         // next word index
    BFT_FN explicit HdrWriter(uint64_t* w) : wb(w), sb(nullptr), stride(0), acc(0), fill(0), wi(0) {}
    BFT_FN HdrWriter(uint32_t* s, uint32_t st) : wb(nullptr), sb(s), stride(st), acc(0), fill(0), wi(0) {}
    BFT_FN void store(uint32_t i, uint64_t v) {
        if (stride) {
            sb[(uint64_t)(2u * i) * stride] = (uint32_t)v;
            sb[(uint64_t)(2u * i + 1u) * stride] = (uint32_t)(v >> 32);
        } else {
            wb[i] = v;
        }
    }
    BFT_FN void put(uint64_t v, uint32_t n) {            // 1 <= n <= 8, v < 2^(8n)
        const uint32_t sh = 8u * fill;
        const uint64_t lo = acc | (v << sh);
        const uint32_t nf = fill + n;
        if (nf >= 8u) {
            store(wi++, lo);
            acc = sh ? (v >> (64u - sh)) : 0ull;
            fill = nf - 8u;
        } else {
            acc = lo;
            fill = nf;
        }
    }
    // four bytes of a 32-byte hash as MessagePack uints (0xcc prefix for bytes >= 128)
    BFT_FN void put_hash_word(uint32_t w) {
        uint64_t v = 0;
        uint32_t n = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t b = (w >> (8 * i)) & 0xffu;
            const uint32_t big = b >> 7;
            const uint64_t e = big ? (uint64_t)(0xccu | (b << 8)) : (uint64_t)b;
            v |= e << (8u * n);
            n += 1u + big;
        }
        put(v, n);
    }
    // compact MessagePack uint (rmp's write_uint)
    BFT_FN void put_uint(uint64_t v) {
        if (v < 128u) { put(v, 1); return; }
        if (v < 256u) { put(0xccu | (v << 8), 2); return; }
        if (v < 65536u) { put(0xcdu | ((v >> 8) << 8) | ((v & 0xffu) << 16), 3); return; }
        if (v < 4294967296ull) {
            const uint64_t be = ((v >> 24) & 0xffu) | (((v >> 16) & 0xffu) << 8) | (((v >> 8) & 0xffu) << 16) |
                                ((v & 0xffu) << 24);
            put(0xceu | (be << 8), 5);
            return;
        }
        uint64_t be = 0;
        for (int i = 0; i < 8; ++i) be |= ((v >> (8 * i)) & 0xffu) << (8 * (7 - i));
        put(0xcfu, 1);
        put(be, 8);
    }
    // "0x" + 40 lowercase hex digits of a 20-byte address, as a 42-byte str8 (d9 2a ...)
    BFT_FN void put_address(const uint8_t* addr20) {
        put(0x78302ad9ull, 4);
        for (int k = 0; k < 5; ++k) {
#if defined(__HIP_DEVICE_COMPILE__)
            const uint64_t x = ((const uint32_t*)addr20)[k];    // device table: 20*v is 4-aligned
#else
            const uint64_t x = (uint64_t)addr20[4 * k] | ((uint64_t)addr20[4 * k + 1] << 8) |
                               ((uint64_t)addr20[4 * k + 2] << 16) | ((uint64_t)addr20[4 * k + 3] << 24);
#endif
            // bytes b0..b3 into 16-bit slots, then (hi nibble, lo nibble) per slot
            uint64_t s = (x & 0xffull) | ((x & 0xff00ull) << 8) | ((x & 0xff0000ull) << 16) | ((x & 0xff000000ull) << 24);
            uint64_t nb = ((s >> 4) & 0x000f000f000f000full) | ((s & 0x000f000f000f000full) << 8);
            uint64_t alpha = ((nb + 0x0606060606060606ull) >> 4) & 0x0101010101010101ull;
            put(nb + 0x3030303030303030ull + alpha * 39ull, 8);
        }
    }
    // pad10*1 with the Keccak domain byte 0x01; returns the number of 136-byte blocks
    BFT_FN uint32_t finish() {
        const uint32_t k = 8u * wi + fill;
        const uint32_t nb = k / 136u + 1u;
        wb[wi++] = acc | (0x01ull << (8u * fill));
        const uint32_t end = 17u * nb;
        while (wi < end) wb[wi++] = 0;
        wb[end - 1u] ^= 0x80ull << 56;
        return nb;
    }
};

// The fields of the header of block (x, prop, var) with parent hash `prev` (8 LE words) at `time`.
// Field order = Header declaration order (types/block.rs:16-36). Only prev_hash chains from height to
// height: header_prefix is that field (with the array header), header_suffix_fields everything after it.
BFT_FN void header_prefix_fields(HdrWriter& w, const uint32_t prev[8]) {
    w.put(0x2000dc9dull, 4);                           // array(13); prev_hash: array16(32)
#pragma unroll
    for (int i = 0; i < 8; ++i) w.put_hash_word(prev[i]);
}
BFT_FN void header_suffix_fields(HdrWriter& w, const uint8_t* addr20, uint64_t seed, uint32_t inst, uint32_t h,
                                 uint32_t prop, uint32_t var, uint64_t time) {
    w.put_address(addr20);                             // proposer
    w.put(0x2000dcull, 3);                             // root = EMPTY_HASH
    for (int i = 0; i < 4; ++i) w.put(0, 8);
    w.put(0x2000dcull, 3);                             // tx_hash (seeded, SPEC.md §5)
    uint32_t tx[8];
    tx_hash_words(seed, inst, h, prop, var, tx);
#pragma unroll
    for (int i = 0; i < 8; ++i) w.put_hash_word(tx[i]);
    w.put(0x2000dcull, 3);                             // receipt_hash = EMPTY_HASH
    for (int i = 0; i < 4; ++i) w.put(0, 8);
    w.put(0, 2);                                       // bloom, difficulty
    w.put_uint(h);                                     // height
    w.put(0, 2);                                       // gas_limit, gas_used
    w.put_uint(time);
    w.put(0x2065736e696f439bull, 8);                   // extra = "Coinse base" (minner/mod.rs:113)
    w.put(0xc065736162ull, 5);                         //   ... + votes: None
}
BFT_FN void header_fields(HdrWriter& w, const uint32_t prev[8], const uint8_t* addr20, uint64_t seed,
                          uint32_t inst, uint32_t h, uint32_t prop, uint32_t var, uint64_t time) {
    header_prefix_fields(w, prev);
    header_suffix_fields(w, addr20, seed, inst, h, prop, var, time);
}

// ---- the header spliced from its two parts (the block-hash pass of kern_fast.hip) ----
// Suffix row, per (instance, height), written by a pass over every height at once: the suffix bytes
// (at most 212: address 44, root 35, tx_hash ≤ 67, receipt 35, height ≤ 5, time ≤ 9, the rest 21),
// then the Keccak domain byte 0x01, zero-filled; dword SFX_LEN_DW holds the suffix length. Host rows
// (header_suffix) are SFX_DWORDS contiguous dwords; on the device the rows are dword-major across the
// launch's instances (header_suffix_strided), so that the writes and the chains' reads coalesce.
constexpr uint32_t SFX_DWORDS = 64, SFX_BODY_DW = 60, SFX_LEN_DW = 63, SFX_DEV_LEN_DW = 60, SFX_DEV_DW = 61;
// Splice buffer (dwords): SFX_PAD zero dwords, the suffix body, zeros up to the last dword a 3-block
// message reads. The prefix is 36..68 bytes, so a message dword w is read at byte 4w - len_p + 72.
constexpr uint32_t SFX_PAD = 18, SFX_BUF = 112, PFX_WORDS = 9;
BFT_FN uint32_t header_suffix(uint64_t* wb, const uint8_t* addr20, uint64_t seed, uint32_t inst, uint32_t h,
                              uint32_t prop, uint32_t var, uint64_t time) {   // wb: SFX_DWORDS / 2 words
    HdrWriter w(wb);
    header_suffix_fields(w, addr20, seed, inst, h, prop, var, time);
    const uint32_t len = 8u * w.wi + w.fill;
    wb[w.wi++] = w.acc | (0x01ull << (8u * w.fill));
    while (w.wi < SFX_DWORDS / 2u - 1u) wb[w.wi++] = 0;
    wb[SFX_DWORDS / 2u - 1u] = (uint64_t)len << 32;    // dword SFX_LEN_DW
    return len;
}
// the device layout: dword k of the row at sb[k * stride] (stride = the launch's instance count)
BFT_FN uint32_t header_suffix_strided(uint32_t* sb, uint32_t stride, const uint8_t* addr20, uint64_t seed,
                                      uint32_t inst, uint32_t h, uint32_t prop, uint32_t var, uint64_t time) {
    HdrWriter w(sb, stride);
    header_suffix_fields(w, addr20, seed, inst, h, prop, var, time);
    const uint32_t len = 8u * w.wi + w.fill;
    w.store(w.wi++, w.acc | (0x01ull << (8u * w.fill)));
    while (w.wi < SFX_BODY_DW / 2u) w.store(w.wi++, 0);
    sb[(uint64_t)SFX_DEV_LEN_DW * stride] = len;
    return len;
}
BFT_FN uint32_t header_prefix(uint64_t* wb, const uint32_t prev[8]) {     // wb: PFX_WORDS words
    HdrWriter w(wb);
    header_prefix_fields(w, prev);
    const uint32_t len = 8u * w.wi + w.fill;
    wb[w.wi++] = w.acc;
    while (w.wi < PFX_WORDS) wb[w.wi++] = 0;
    return len;
}
// The prefix for the chains, branch-free: each prev_hash word's MessagePack expansion (a byte >= 128
// becomes 0xcc b) is two v_perm_b32 of {0xcccccccc, w} with selectors from a 16-entry table indexed by
// the word's four high bits, and the expansions are appended to the stream with an unconditional store
// per word (the divergent `put` of HdrWriter costs both of its paths). Same bytes as header_prefix.
struct PfxSel { uint32_t lo, hi; };
BFT_FN constexpr PfxSel pfx_sel(uint32_t idx) {               // output byte k: 4 = 0xcc, i = byte i, 12 = 0
    uint32_t out[8] = {12, 12, 12, 12, 12, 12, 12, 12};
    uint32_t pos = 0;
    for (uint32_t i = 0; i < 4; ++i) {
        if ((idx >> i) & 1u) out[pos++] = 4;
        out[pos++] = i;
    }
    return PfxSel{out[0] | out[1] << 8 | out[2] << 16 | out[3] << 24, out[4] | out[5] << 8 | out[6] << 16 | out[7] << 24};
}
BFT_FN uint32_t perm_bytes(uint32_t s0, uint32_t s1, uint32_t sel) {   // v_perm_b32 (selectors 0..7, 12)
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(s0, s1, sel);
#else
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t d = 0;
    for (int k = 0; k < 4; ++k) {
        const uint32_t q = (sel >> (8 * k)) & 0xffu;
        d |= (q < 8 ? (uint32_t)((v >> (8 * q)) & 0xffu) : 0u) << (8 * k);
    }
    return d;
#endif
}
// `tbl`: pfx_sel(0..15) (LDS on the device); wb: PFX_WORDS + 4 words. Returns the prefix length.
BFT_FN uint32_t header_prefix_perm(uint64_t* wb, const uint32_t prev[8], const PfxSel* tbl) {
    uint64_t acc = 0x2000dc9dull;                     // array(13); prev_hash: array16(32)
    uint32_t fill = 4, wi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t w = prev[i];
        const uint32_t idx = ((((w >> 7) & 0x01010101u) * 0x10204080u) >> 28);   // the four high bits
        const PfxSel sel = tbl[idx];
        const uint64_t v = (uint64_t)perm_bytes(0xccccccccu, w, sel.lo) | ((uint64_t)perm_bytes(0xccccccccu, w, sel.hi) << 32);
        const uint32_t n = 4u + (uint32_t)__builtin_popcount(idx);
        const uint32_t sh = 8u * fill, nf = fill + n;
        const uint64_t lo = acc | (v << sh);
        wb[wi] = lo;                                  // rewritten until the word is complete
        const bool full = nf >= 8u;
        acc = full ? (sh ? v >> (64u - sh) : 0ull) : lo;
        wi += full ? 1u : 0u;
        fill = full ? nf - 8u : nf;
    }
    wb[wi] = acc;
#pragma unroll
    for (uint32_t k = 1; k <= 4; ++k) wb[wi + k] = 0;   // wi >= 4: words past the prefix up to PFX_WORDS
    return 8u * wi + fill;
}
BFT_FN uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t r) {      // ({hi, lo} >> 8r)[31:0], r < 4
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(hi, lo, r);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * r));
#endif
}
// rate blocks of a spliced header: ceil((len_p + len_s + 1) / 136)
BFT_FN uint32_t splice_blocks(uint32_t len_p, uint32_t len_s) { return (len_p + len_s + 136u) / 136u; }
// message dword w of the padded header: `sx` = splice buffer + ((72 - len_p) >> 2), r = (72 - len_p) & 3,
// `pw` = the prefix as dwords (zero past len_p); nb rate blocks (the final 0x80 at dword 34 nb - 1)
BFT_FN uint32_t splice_word(const uint32_t* sx, uint32_t r, const uint32_t* pw, uint32_t w, uint32_t nb) {
    uint32_t v = align_bytes(sx[w + 1u], sx[w], r);
    if (w < 2u * PFX_WORDS) v |= pw[w];
    if (w == 34u * nb - 1u) v ^= 0x80000000u;
    return v;
}
// the header into wb, padded for Keccak; returns the number of rate blocks (2 or 3)
BFT_FN uint32_t header_words(uint64_t* wb, const uint32_t prev[8], const uint8_t* addr20, uint64_t seed,
                             uint32_t inst, uint32_t h, uint32_t prop, uint32_t var, uint64_t time) {
    HdrWriter w(wb);
    header_fields(w, prev, addr20, seed, inst, h, prop, var, time);
    return w.finish();
}
// the header bytes alone (the ledger's stored Header, votes None); returns their length
BFT_FN uint32_t header_raw(uint64_t* wb, const uint32_t prev[8], const uint8_t* addr20, uint64_t seed,
                           uint32_t inst, uint32_t h, uint32_t prop, uint32_t var, uint64_t time) {
    HdrWriter w(wb);
    header_fields(w, prev, addr20, seed, inst, h, prop, var, time);
    const uint32_t len = 8u * w.wi + w.fill;
    if (w.fill) wb[w.wi] = w.acc;
    return len;
}

// Keccak-256 of a candidate header (SPEC.md §7) by ONE lane. `buf`: LANE_HASH_BUF bytes, 8-aligned
// (LDS on the device). prev/out: the hash as 8 little-endian words.
BFT_FN void lane_block_hash(uint8_t* buf, const uint32_t prev[8], const uint8_t* addr20, uint64_t seed,
                            uint32_t inst, uint32_t h, uint32_t prop, uint32_t var, uint64_t time,
                            uint32_t out[8]) {
    uint64_t* wb = (uint64_t*)buf;
    const uint32_t nb = header_words(wb, prev, addr20, seed, inst, h, prop, var, time);
    uint64_t a[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) a[i] = 0;
#pragma unroll 1
    for (uint32_t blk = 0; blk < nb; ++blk) {
        const uint64_t* w = wb + 17u * blk;
#pragma unroll
        for (int i = 0; i < 17; ++i) a[i] ^= w[i];
        keccak_f1600(a);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) { out[2 * i] = (uint32_t)a[i]; out[2 * i + 1] = (uint32_t)(a[i] >> 32); }
}

// header_prefix_perm's words in registers (the lane chain kernel: no per-lane LDS buffer, so more chain waves fit
// a CU): word wi is a select over the words it can be at that step. Field i starts at byte 4 + 4i .. 4 + 8i (each
// hash byte is 1 or 2 bytes), so step i writes one of the words (1 + i) / 2 .. i and the last partial word is one
// of 4 .. 8; the words past it stay 0. pw: the PFX_WORDS words as 2 * PFX_WORDS dwords (low first).
BFT_FN uint32_t header_prefix_regs(const uint32_t prev[8], const PfxSel* tbl, uint32_t pw[2 * PFX_WORDS]) {
    uint64_t wv[PFX_WORDS];
#pragma unroll
    for (uint32_t k = 0; k < PFX_WORDS; ++k) wv[k] = 0;
    uint64_t acc = 0x2000dc9dull;                     // array(13); prev_hash: array16(32)
    uint32_t fill = 4, wi = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t w = prev[i];
        const uint32_t idx = ((((w >> 7) & 0x01010101u) * 0x10204080u) >> 28);   // the four high bits
        const PfxSel sel = tbl[idx];
        const uint64_t v = (uint64_t)perm_bytes(0xccccccccu, w, sel.lo) | ((uint64_t)perm_bytes(0xccccccccu, w, sel.hi) << 32);
        const uint32_t n = 4u + (uint32_t)__builtin_popcount(idx);
        const uint32_t sh = 8u * fill, nf = fill + n;
        const uint64_t lo = acc | (v << sh);
#pragma unroll
        for (uint32_t k = (1u + i) / 2u; k <= i; ++k) wv[k] = wi == k ? lo : wv[k];
        const bool full = nf >= 8u;
        acc = full ? (sh ? v >> (64u - sh) : 0ull) : lo;
        wi += full ? 1u : 0u;
        fill = full ? nf - 8u : nf;
    }
#pragma unroll
    for (uint32_t k = 4; k < PFX_WORDS; ++k) wv[k] = wi == k ? acc : wv[k];
#pragma unroll
    for (uint32_t k = 0; k < PFX_WORDS; ++k) { pw[2 * k] = (uint32_t)wv[k]; pw[2 * k + 1] = (uint32_t)(wv[k] >> 32); }
    return 8u * wi + fill;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// The same hash through the two-kernel block-hash pass's splice (host: the CPU emulator's post-pass).
// sfx: the height's suffix row (SFX_DWORDS dwords, header_suffix).
inline void spliced_block_hash(const uint32_t* sfx, const uint32_t prev[8], uint32_t out[8]) {
    for (int i = 0; i < 8; ++i) out[i] = 0;
    uint32_t buf[SFX_BUF] = {};
    for (uint32_t i = 0; i < SFX_BODY_DW; ++i) buf[SFX_PAD + i] = sfx[i];
    uint64_t pfx[PFX_WORDS + 4], ref[PFX_WORDS];
    PfxSel tbl[16];
    for (uint32_t i = 0; i < 16; ++i) tbl[i] = pfx_sel(i);
    const uint32_t lp = header_prefix_perm(pfx, prev, tbl);
    if (header_prefix(ref, prev) != lp) return;      // leaves `out` unset: the checks fail loudly
    for (uint32_t i = 0; i < PFX_WORDS; ++i) if (ref[i] != pfx[i]) return;
    uint32_t pr[2 * PFX_WORDS];                       // the register form of the lane chain kernel
    if (header_prefix_regs(prev, tbl, pr) != lp) return;
    for (uint32_t i = 0; i < PFX_WORDS; ++i) if (pr[2 * i] != (uint32_t)ref[i] || pr[2 * i + 1] != (uint32_t)(ref[i] >> 32)) return;
    uint32_t pw[2 * PFX_WORDS];
    for (uint32_t i = 0; i < PFX_WORDS; ++i) { pw[2 * i] = (uint32_t)pfx[i]; pw[2 * i + 1] = (uint32_t)(pfx[i] >> 32); }
    const uint32_t c = 72u - lp, nb = splice_blocks(lp, sfx[SFX_LEN_DW]);
    const uint32_t* sx = buf + (c >> 2);
    uint64_t a[25] = {};
    for (uint32_t blk = 0; blk < nb; ++blk) {
        for (uint32_t i = 0; i < 17; ++i) {
            const uint32_t w = 34u * blk + 2u * i;
            a[i] ^= (uint64_t)splice_word(sx, c & 3u, pw, w, nb) | ((uint64_t)splice_word(sx, c & 3u, pw, w + 1u, nb) << 32);
        }
        keccak_f1600(a);
    }
    for (int i = 0; i < 4; ++i) { out[2 * i] = (uint32_t)a[i]; out[2 * i + 1] = (uint32_t)(a[i] >> 32); }
}
#endif

// ---- little-endian seeds, N = 64: the canonical schedule's blocks, predicted ----
// The Byzantine validators of an instance of 64 (SPEC.md §5: partial Fisher-Yates; `perm`: 64 bytes of
// scratch), as Fast64::init_byzantine draws them.
// STRIDE: byte i of `perm` at (i / 4) * 4 * STRIDE + i % 4 (STRIDE 64: a lane's column of a [dword][lane] LDS array)
template <uint32_t STRIDE = 1>
BFT_FN uint64_t byz_mask64(uint64_t seed, uint32_t inst, uint32_t f, uint8_t* perm) {
    auto at = [&](uint32_t i) -> uint8_t& { return perm[(i >> 2) * 4u * STRIDE + (i & 3u)]; };
    for (uint32_t i = 0; i < 64u; ++i) at(i) = (uint8_t)i;
    uint64_t mask = 0;
    if (f > 64u) f = 64u;
    for (uint32_t i = 0; i < f; ++i) {
        uint32_t w[4];
        philox(seed, inst, i, 0, DOM_BYZ, w);
        const uint32_t j = i + w[0] % (64u - i);
        const uint8_t t = at(i); at(i) = at(j); at(j) = t;
        mask |= 1ull << at(i);
    }
    return mask;
}
constexpr uint32_t SPEC_VALID = 0x80000000u;
// Block x as the canonical tick would commit it (bft_fast64.h canonical_tick) if every tick since the
// genesis was canonical: proposer j = seed(tip) mod 64 at round 0 (validator.rs:33-48, 74-77; the tip's
// little-endian U128 seed mod 64 is the low 6 bits of its first hash word); an equivocating proposer
// splits the validators by the SPLIT draw of view (x, 0) (SPEC.md §5) and the variant whose honest
// validators with the Byzantine wildcards exceed Q = 42 commits; neither or both: no prediction (round
// changes or a fork follow). The block's time tick is x - 1. The consumer (Fast64::hash_pending) takes a
// prediction only where the recorded block equals it, height after height.
BFT_FN bool spec_block64(uint64_t seed, uint32_t inst, uint32_t x, uint64_t byz, uint32_t tip_w0, uint32_t& j,
                         uint32_t& var) {
    j = tip_w0 & 63u;
    uint64_t v1m = 0;
    if ((byz >> j) & 1ull) {
        uint32_t w[4];
        philox(seed, inst, x, 0, DOM_SPLIT, w);
        v1m = ((uint64_t)w[0] | ((uint64_t)w[1] << 32)) & ~(1ull << j);
    }
    const uint64_t hon = ~byz;
    const bool k0 = __builtin_popcountll(byz | (hon & ~v1m)) > 42, k1 = __builtin_popcountll(byz | (hon & v1m)) > 42;
    var = k1 ? 1u : 0u;
    return k0 != k1;
}
// {valid, proposer, variant, seed of the block's hash mod 64}
BFT_FN uint32_t spec_word(uint32_t j, uint32_t var, uint32_t seed_next) { return SPEC_VALID | j | (var << 8) | (seed_next << 16); }

// randon_seed (validator.rs:39-48): U128::from(hash[0..8] ++ 0^8) mod n. `le` selects how the
// 16-byte buffer is read (bftsim.h BFTSIM_SEED_*): big-endian (BE64(hash[0..8]) * 2^64) mod n, or
// little-endian LE64(hash[0..8]) mod n.
BFT_FN uint32_t seed_from_hash(const uint8_t* h, uint32_t n, bool le = false) {
    if (le) {
        uint64_t v = 0;
        for (int i = 7; i >= 0; --i) v = (v << 8) | h[i];
        return (uint32_t)(v % n);
    }
    uint64_t be = 0;
    for (int i = 0; i < 8; ++i) be = (be << 8) | h[i];
    uint64_t a = be % n;
    uint64_t t = (0xffffffffffffffffull % n + 1ull) % n;   // 2^64 mod n
    return (uint32_t)((a * t) % n);
}
// the same from the first two little-endian hash words (the kernels' register form)
BFT_FN uint32_t seed_from_words(uint32_t w0, uint32_t w1, uint32_t n, bool le) {
    uint8_t hb[8];
    for (int q = 0; q < 4; ++q) { hb[q] = (uint8_t)(w0 >> (8 * q)); hb[4 + q] = (uint8_t)(w1 >> (8 * q)); }
    return seed_from_hash(hb, n, le);
}

}  // namespace bft
