// bft_wave.h — the batched PBFT core: one wavefront simulates 64/S instances (S <= 64), or one
// workgroup of S = 128 / 256 lanes simulates one instance; one lane per validator (lane =
// reference `Core` actor, src/consensus/pbft/core/core.rs:119-140).
//
// The body is written once against a tiny ops interface W (wave intrinsics, or LDS-exchanged
// workgroup collectives for S > 64, on gfx950; a fiber emulator on the CPU for the tests). Rules
// that keep it correct on all of them:
//   * collectives (ballot, shfl_xor, bcast, group reductions, sync) are only called from
//     segment-uniform control flow; the message handlers below are per-lane code and never
//     call them;
//   * a phase's outbox is published to LDS, then W::sync(), then receivers gather senders'
//     records in their own rotated order (SPEC.md §3) and run the reference handlers one message
//     at a time (SPEC.md §2). Everything they send goes to the per-lane `nx` outbox for the next
//     phase;
//   * the instance's canonical chain lives in global memory (rec/hash tables); the first Core
//     commit of a height is recorded by the segment leader after the phase, in lane order, which
//     is the oracle's receiver order.
#pragma once
#include "bft_common.h"

// Invariant checks of the CPU emulator build (tests/emu, -DBFT_EMU_CHECKS): a violated invariant aborts the run.
// They compile to nothing in the kernels.
#if defined(BFT_EMU_CHECKS) && !defined(__HIP_DEVICE_COMPILE__)
#include <cstdio>
#include <cstdlib>
#define BFT_EMU_CHECK(cond, what)                                                         \
    do {                                                                                  \
        if (!(cond)) { fprintf(stderr, "emu: invariant violated: %s\n", what); abort(); } \
    } while (0)
#else
#define BFT_EMU_CHECK(cond, what) do { } while (0)
#endif

namespace bft {

constexpr int REC_WORDS = 22;            // LDS words per published outbox record

// outbox record flags
constexpr uint32_t F_PP = 1u, F_PP_EQ = 2u, F_PR = 4u, F_PR_W = 8u, F_CM = 16u, F_CM_W = 32u,
                   F_OCM = 64u, F_OCM_W = 128u, F_RC = 256u, F_SYNC = 512u, F_BLK = 1024u;

struct Outbox {
    uint32_t f;
    uint32_t pp_h, pp_r; uint64_t pp_b;
    uint32_t pr_h, pr_r; uint64_t pr_d;
    uint32_t cm_h, cm_r; uint64_t cm_d;
    uint32_t ocm_h, ocm_r; uint64_t ocm_d;
    uint32_t rc_h, rc_r;
    uint32_t sync_h;
    uint32_t blk_lo, blk_hi;
};

// Every field of a kind is written when its flag bit is set and read only while it is set, so an
// empty outbox is f == 0 (the stale fields are never read: no per-phase register clearing).
BFT_FN void outbox_clear(Outbox& o) { o.f = 0; }
BFT_FN void outbox_init(Outbox& o) {
    o.f = 0;
    o.pp_h = o.pp_r = 0; o.pp_b = 0;
    o.pr_h = o.pr_r = 0; o.pr_d = 0;
    o.cm_h = o.cm_r = 0; o.cm_d = 0;
    o.ocm_h = o.ocm_r = 0; o.ocm_d = 0;
    o.rc_h = o.rc_r = 0;
    o.sync_h = 0;
    o.blk_lo = o.blk_hi = 0;
}

// LDS layout of one wave (S <= 64, L = 64 lanes) or one workgroup (S > 64, L = S lanes):
//   [0, L*REC_WORDS*4)                published outbox records (one per lane)
//   (aliases the records)             per-lane commit hand-off {x, blk lo, blk hi, round, seed}
//                                     (also the Fisher-Yates scratch at init): written only after
//                                     every receiver has read the phase's records
//   [.., + 12*L*4)                    gossip outbound cache (backend.rs:141-148), SoA [word][lane]:
//                                     per kind (Preprepare, Prepare, Commit, old Commit) the last
//                                     subject sent {height, round, 32-bit block id}
//   [.., + 528)                       per-wave histogram bins (HIST_BINS words)
// The RoundChangeSet tables are lane-private and touched only by round changes: they live in global
// memory (P.rcs, coalesced SoA per wave: K round words [k][lane], then the sender bitmaps as 2*NW
// 32-bit words [k][j][lane]) so the LDS of a wave stays small enough for 4 waves per SIMD.
//   [.., + 512)                       per-segment shared words (8 per segment for S <= 64; 16 words
//                                     + the group-collective slots at +256 for S > 64)
//   need_seed only:
//   [.., + L*32)                      per-lane commit hash
//   [.., + (64/S)*LANE_HASH_BUF)      one header buffer per segment (S <= 64): the header a segment's deferred
//                                     hash absorbs (resolve_deferred_hash_seg, wave_block_hash). The one-lane
//                                     hashes of the rare paths use a private buffer: 64 per-lane buffers
//                                     (26 KB) held the seeded kernels to one wave per SIMD by LDS
// (The N = 64 FAST kernel has its own, smaller layout: bft_fast64.h.)
template <uint32_t S>
struct Layout {
    static constexpr uint32_t L = S > 64 ? S : 64;
    static constexpr int NW = S > 64 ? (int)(S / 64) : 1;
    static constexpr uint32_t CMT_STRIDE = 8;          // words per lane of the commit hand-off
    static constexpr uint32_t REC_OFF = 0;
    static constexpr uint32_t RC_OFF = REC_OFF + L * (uint32_t)REC_WORDS * 4;
    static constexpr uint32_t CMT_OFF = REC_OFF;
    static constexpr uint32_t CACHE_OFF = RC_OFF;
    static constexpr uint32_t HIST_OFF = CACHE_OFF + 12u * L * 4u;
    static constexpr uint32_t RCS_WORDS_PER_ROUND = (1u + 2u * NW) * L;   // global, per wave and round
    static constexpr uint32_t BL_WORDS = S * 5u * L;  // replay mode: backlog slots, global, per wave
    static constexpr uint32_t SEG_OFF = HIST_OFF + 528;
    static_assert(L * CMT_STRIDE <= L * REC_WORDS, "commit hand-off must fit in the record area");
    static_assert(HIST_BINS * 4 <= 528, "histogram area");
    static constexpr uint32_t GRP_OFF = SEG_OFF + 256;
    // group collectives (S > 64): 2 parities x 4 words, then the batched ballots / gathers of summarize,
    // 2 parities x 64 words, then the phase summary's 13 sender masks (bft_hip.h GroupHip::summary)
    static constexpr uint32_t GRP_BYTES = S > 64 ? 64u + 2u * 8u * 64u + 13u * 8u * (uint32_t)NW : 256u;
    static constexpr uint32_t CHASH_OFF = GRP_OFF + GRP_BYTES;
    static constexpr uint32_t SCR_OFF = CHASH_OFF + L * 32;
    static constexpr uint32_t BYTES_POW2 = CHASH_OFF;
    // (S < 64, seeded) per segment the hash of its last canonical block whose hash a deferred hash patched:
    // {height, 8 words}, the next header's prev_hash without global loads (resolve_deferred_hash_seg)
    static constexpr uint32_t TIPC_OFF = SCR_OFF + (64 / S) * LANE_HASH_BUF, TIPC_BYTES = 48;
    static constexpr uint32_t BYTES_SEED = S > 64 ? SCR_OFF : TIPC_OFF + (64 / S) * TIPC_BYTES;
    static constexpr uint32_t bytes(bool need_seed) { return need_seed ? BYTES_SEED : BYTES_POW2; }
};
// RoundChangeSet table words per wave / workgroup for k rounds per validator (a runtime capacity:
// bftsim_set_rcs_capacity; bftsim_run re-runs an overflowing batch at a larger one)
BFT_FN uint64_t rcs_words(uint32_t seg, uint32_t k) {
    return (uint64_t)k * (seg == 256 ? Layout<256>::RCS_WORDS_PER_ROUND : seg == 128 ? Layout<128>::RCS_WORDS_PER_ROUND
                                                                         : Layout<64>::RCS_WORDS_PER_ROUND);
}
BFT_FN uint32_t backlog_words(uint32_t seg) {      // per wave (S <= 64) or workgroup
    return seg == 256 ? Layout<256>::BL_WORDS : seg == 128 ? Layout<128>::BL_WORDS : seg == 64 ? Layout<64>::BL_WORDS
         : seg == 32 ? Layout<32>::BL_WORDS : seg == 16 ? Layout<16>::BL_WORDS : seg == 8 ? Layout<8>::BL_WORDS
         : Layout<4>::BL_WORDS;
}
BFT_FN uint32_t lds_bytes(uint32_t seg, bool need_seed) {
    return seg == 256 ? Layout<256>::bytes(need_seed) : seg == 128 ? Layout<128>::bytes(need_seed)
         : seg == 64 ? Layout<64>::bytes(need_seed) : seg == 32 ? Layout<32>::bytes(need_seed)
         : seg == 16 ? Layout<16>::bytes(need_seed) : seg == 8 ? Layout<8>::bytes(need_seed)
         : Layout<4>::bytes(need_seed);
}

// Kernel modes:
//   MODE_FULL    every path;
//   MODE_EXT     MODE_FULL plus the opt-in modes: backlog replay (SPEC.md §10) and the real-crypto
//                broadcast log / votes (SPEC.md §11);
//   MODE_RESUME  (S == 64) the full kernel over the instances the N = 64 FAST kernel (bft_fast64.h)
//                handed over, from their saved phase: the FAST kernel saves the state below
//                (SAVE_WORDS per lane, P.save) at the start of a phase it has no closed form for and
//                sets P.resume_flags.
constexpr int MODE_FULL = 0, MODE_EXT = 1, MODE_RESUME = 2;
constexpr uint32_t SAVE_WORDS = 80;
constexpr uint32_t SAVE_COLD = 72;   // words 72..78: outbox kinds that always take the general path

template <class W, bool NEED_SEED, uint32_t S, int MODE = MODE_FULL>
struct Sim {
    static constexpr bool RESUME = MODE == MODE_RESUME;
    // the opt-in modes (backlog replay, real-crypto log and votes) exist only in MODE_EXT builds, so
    // the product kernels carry none of their code or registers
    static constexpr bool EXT = MODE == MODE_EXT;
    // the wave-cooperative header hash of closed-form commits (resolve_deferred_hash)
    static constexpr bool WAVE_HASH = NEED_SEED && S == 64 && MODE == MODE_FULL;
    // segments of 4..32 lanes (several instances per wave): a closed-form commit's header is hashed after the
    // delivery by lane pairs of its segment (resolve_deferred_hash_seg), not by every committing lane alone
    static constexpr bool SEG_HASH = NEED_SEED && S < 64 && MODE == MODE_FULL;
    static_assert(MODE != MODE_RESUME || S == 64, "hand-over modes are for one instance per wave");
    using LY = Layout<S>;
    static constexpr int NW = LY::NW;
    static constexpr uint32_t LDS_REC_OFF = LY::REC_OFF, LDS_RC_OFF = LY::RC_OFF, LDS_CMT_OFF = LY::CMT_OFF,
                              LDS_HIST_OFF = LY::HIST_OFF, LDS_CACHE_OFF = LY::CACHE_OFF,
                              LDS_SEG_OFF = LY::SEG_OFF, LDS_CHASH_OFF = LY::CHASH_OFF, LDS_SCR_OFF = LY::SCR_OFF;
    using M = Bits<NW>;
    const Params& P;
    uint8_t* lds;
    W wv;                    // collectives (stateful for the workgroup flavour)
    // identity
    uint32_t lane, seg_base, me, inst_local, inst;
    M seg_mask;              // this segment's bits in a ballot
    bool is_val, running, byz, core_dead;
    // segment-uniform
    bool seg_done, frozen;
    uint32_t canon_h, done_tick, seg_flags;
    uint64_t canon_tip;      // canonical block at canon_h (segment-uniform cache; 0 at genesis)
    uint32_t canon_tip_seed;
    uint32_t canon_tick;     // tick that recorded canon_h (commit-latency histogram)
    uint64_t views_acc;      // instance-rounds of the recorded heights <= H
    // Core + RoundState (round_state.rs:12-22)
    uint32_t h, r, st;
    bool wait;
    uint64_t lock, pp, pend;
    M prep, comm;            // MessageManage sender sets (protocol/mod.rs:176-209)
    uint32_t n_rcs;          // RoundChangeSet entries (the table itself lives in LDS)
    uint32_t proposer;       // 0xffffffff = None
    // chain tip
    uint32_t last, last_seed;
    int32_t last_T;
    // timers / limiter / miner / sync
    int32_t tick, timer_tick, rc_last_tick, wake_tick;
    uint32_t mint_height, miner_queue, sync_pending;
    uint64_t cand;
    // outbox of the next phase
    Outbox nx;
    // Core commit of this phase (for canonical resolution)
    uint32_t commit_x, commit_round, commit_seed;
    uint32_t off_inst, off_tick;     // hoisted parts of delivery_offset (SPEC.md §3)
    uint64_t commit_blk;
    // (S == 64, NEED_SEED, MODE_FULL) a Core commit of the Prepare/Commit closed form whose header hash
    // is computed after the delivery by the whole wave (resolve_deferred_hash)
    bool hash_defer, in_pc;
    // (SEG_HASH) a hash deferred past its phase (resolve_deferred_hash_seg, end_phase_hashes): the canonical tip
    // was recorded with that stale seed and hash (canon_stale, segment-uniform), this lane's tip seed was taken
    // from it by block gossip (seed_stale)
    bool canon_stale, seed_stale;
    uint32_t lane_flags;
    uint32_t* rcs_base;      // this wave's RoundChangeSet table (global)
    uint32_t rcs_k;          // its capacity in rounds (Params::rcs_k)
    uint32_t* bl_base;       // this wave's backlog slots (global, replay mode)
    uint32_t mlog_cnt;       // real-crypto mode: messages logged so far by this instance (segment-uniform)
#ifdef BFT_STAMPS
    uint64_t st_acc[NSTAMP];
    uint64_t st_t;
#define BFT_STAMP(k) do { uint64_t t_ = wv.clock(); st_acc[k] += t_ - st_t; st_t = t_; } while (0)
#else
#define BFT_STAMP(k) do { } while (0)
#endif

    BFT_FN Sim(const Params& p, uint8_t* l, uint32_t wave_global) : P(p), lds(l) {
        wv.init(lds + LY::GRP_OFF);
        lane = wv.lane();
        seg_base = S >= 64 ? 0u : (lane & ~(S - 1));
        me = lane - seg_base;
        inst_local = S >= 64 ? wave_global : wave_global * (64u / S) + (lane / S);
        inst = p.first_instance + inst_local;
        seg_mask = S >= 64 ? M::low(S) : M::from(((1ull << (S & 63u)) - 1ull) << seg_base);
        bool inst_ok = inst_local < p.n_instances;
        is_val = inst_ok && me < p.n;
        running = is_val && !((p.silent_mask[(me >> 6) & 3u] >> (me & 63u)) & 1ull);
        byz = false;
        core_dead = false;
        seg_done = !inst_ok;
        frozen = false;
        canon_h = 0;
        canon_tip = 0;
        canon_tip_seed = p.genesis_seed;
        canon_tick = 0;
        views_acc = 0;
        done_tick = p.max_ticks;
        seg_flags = 0;
        h = 0; r = 0; st = ST_ACCEPT_REQUEST; wait = false;
        lock = pp = pend = BLK_NONE;
        prep = comm = M::zero();
        n_rcs = 0;
        proposer = 0xffffffffu;
        last = 0; last_seed = p.genesis_seed; last_T = -1;
        tick = 0; timer_tick = -1; rc_last_tick = 0; wake_tick = -1;
        mint_height = 0; miner_queue = 0; sync_pending = 0;
        cand = BLK_NONE;
        for (uint32_t k = 0; k < 12; ++k) *cache_p(k) = 0;
        outbox_init(nx);
        commit_x = 0; commit_round = 0; commit_seed = 0; commit_blk = 0;
        hash_defer = false; in_pc = false;
        canon_stale = false; seed_stale = false;
        mlog_cnt = 0;
        lane_flags = 0;
        off_inst = offset_inst_part(p.seed, inst);
        rcs_k = p.rcs_k;
        rcs_base = p.rcs + (uint64_t)wave_global * rcs_k * LY::RCS_WORDS_PER_ROUND;
        bl_base = p.backlog ? p.backlog + (uint64_t)wave_global * LY::BL_WORDS : nullptr;
        off_tick = 0;
    }

    // ---------------------------------------------------------------- global canonical table
    // row of height x: every height (window_mask == 0), or a ring of the last window_mask+1 heights
    BFT_FN uint64_t row_of(uint32_t x) const {
        return (uint64_t)inst_local * P.rows + (P.window_mask ? (x & P.window_mask) : x);
    }
    BFT_FN uint32_t* rec_row(uint32_t x) const { return P.rec + row_of(x) * 4; }
    BFT_FN uint8_t* hash_row(uint32_t x) const { return P.hash + row_of(x) * 32; }
    // a lookup of canonical height x older than the ring holds
    BFT_FN void check_window(uint32_t x) {
        if (P.window_mask && x + P.window_mask < canon_h) lane_flags |= FLAG_WINDOW;
    }
    // ---------------------------------------------------------------- the wave's Keccak (S == 64)
    // Keccak-f[1600] spread over the wave: lane x + 8y (x, y < 5) holds state word A[x][y] = word x + 5y
    // as two 32-bit halves, so each row y sits in one 16-lane DPP row. Theta's column parities and pi
    // are ds_bpermute shuffles; the x-neighbours of D and chi are DPP row shifts (wrap-around by a
    // second shift and a select). Lanes with x or y >= 5 compute garbage that no valid lane reads.
    // Every lane of the wave calls it. Rho amounts per word and, per destination word, the source word
    // of pi (B[y][2x+3y] = rot(A[x][y]), the table of bft_hash_pair_kernel), packed 10 / 12 per u64.
    BFT_FN static uint32_t kw_rot(uint32_t w) {
        const uint64_t R0 = 0ull | 1ull << 6 | 62ull << 12 | 28ull << 18 | 27ull << 24 | 36ull << 30 | 44ull << 36 |
                            6ull << 42 | 55ull << 48 | 20ull << 54;
        const uint64_t R1 = 3ull | 10ull << 6 | 43ull << 12 | 25ull << 18 | 39ull << 24 | 41ull << 30 | 45ull << 36 |
                            15ull << 42 | 21ull << 48 | 8ull << 54;
        const uint64_t R2 = 18ull | 2ull << 6 | 61ull << 12 | 56ull << 18 | 14ull << 24;
        const uint64_t v = w < 10u ? R0 : (w < 20u ? R1 : R2);
        return (uint32_t)(v >> (6u * (w % 10u))) & 63u;
    }
    BFT_FN static uint32_t kw_src(uint32_t w) {      // the word whose rotated value lands in word w
        const uint64_t S0 = 0ull | 6ull << 5 | 12ull << 10 | 18ull << 15 | 24ull << 20 | 3ull << 25 | 9ull << 30 |
                            10ull << 35 | 16ull << 40 | 22ull << 45 | 1ull << 50 | 7ull << 55;
        const uint64_t S1 = 13ull | 19ull << 5 | 20ull << 10 | 4ull << 15 | 5ull << 20 | 11ull << 25 | 17ull << 30 |
                            23ull << 35 | 2ull << 40 | 8ull << 45 | 14ull << 50 | 15ull << 55;
        const uint64_t S2 = 21ull;
        const uint64_t v = w < 12u ? S0 : (w < 24u ? S1 : S2);
        return (uint32_t)(v >> (5u * (w % 12u))) & 31u;
    }
    BFT_FN static void rotl64_halves(uint32_t lo, uint32_t hi, uint32_t n, uint32_t& ol, uint32_t& oh) {
        const uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        const uint64_t r = n ? ((v << n) | (v >> (64u - n))) : v;
        ol = (uint32_t)r; oh = (uint32_t)(r >> 32);
    }
    // A[x-1], A[x+1], A[x+2] of the same row y (x mod 5) by DPP
    BFT_FN uint32_t xm1(uint32_t v, uint32_t x) { const uint32_t a = wv.template row_shr<1>(v), b = wv.template row_shl<4>(v); return x ? a : b; }
    BFT_FN uint32_t xp1(uint32_t v, uint32_t x) { const uint32_t a = wv.template row_shl<1>(v), b = wv.template row_shr<4>(v); return x < 4u ? a : b; }
    BFT_FN uint32_t xp2(uint32_t v, uint32_t x) { const uint32_t a = wv.template row_shl<2>(v), b = wv.template row_shr<3>(v); return x < 3u ? a : b; }
    BFT_FN void keccak_wave(uint32_t& lo, uint32_t& hi) {
        const uint32_t x = lane & 7u, y = lane >> 3;
        const uint32_t w = (x < 5u && y < 5u) ? x + 5u * y : 0u;   // this lane's word
        const uint32_t rot = kw_rot(w);
        const uint32_t sw = kw_src(w), src = (sw % 5u) + 8u * (sw / 5u);
        const uint32_t xc = x < 5u ? x : 0u;
#pragma unroll 1
        for (int rnd = 0; rnd < 24; ++rnd) {
            // theta: column parities C[x] (rows y' != y by shuffle), D[x] = C[x-1] ^ rotl(C[x+1], 1)
            uint32_t cl = lo, ch = hi;
#pragma unroll
            for (uint32_t k = 1; k < 5u; ++k) {
                const uint32_t j = xc + 8u * ((y + k) % 5u);
                cl ^= wv.shfl(lo, j);
                ch ^= wv.shfl(hi, j);
            }
            const uint32_t aml = xm1(cl, xc), amh = xm1(ch, xc);
            const uint32_t apl = xp1(cl, xc), aph = xp1(ch, xc);
            uint32_t rl, rh;
            rotl64_halves(apl, aph, 1u, rl, rh);
            lo ^= aml ^ rl;
            hi ^= amh ^ rh;
            // rho at the source, pi as a shuffle
            uint32_t tl, th;
            rotl64_halves(lo, hi, rot, tl, th);
            const uint32_t bl = wv.shfl(tl, src), bh = wv.shfl(th, src);
            // chi: A[x][y] = B[x][y] ^ (~B[x+1][y] & B[x+2][y])
            const uint32_t b1l = xp1(bl, xc), b1h = xp1(bh, xc);
            const uint32_t b2l = xp2(bl, xc), b2h = xp2(bh, xc);
            lo = bl ^ (~b1l & b2l);
            hi = bh ^ (~b1h & b2h);
            const bool l0 = lane == 0u;                        // iota
            lo ^= l0 ? KECCAK_RC_LO[rnd] : 0u;
            hi ^= l0 ? KECCAK_RC_HI[rnd] : 0u;
        }
    }
    // Keccak-256 of the header of canonical-parent block b at height x by the whole wave; the header is
    // encoded by lane `enc` into its scratch buffer. Returns the 8 hash words in every lane.
    BFT_FN void wave_block_hash(uint32_t enc, uint32_t x, uint64_t b, uint32_t out[8]) {
        uint64_t* wb = (uint64_t*)(lds + LDS_SCR_OFF);                  // S == 64: the one segment buffer
        uint32_t nb = 0;
        if (lane == enc) {
            uint32_t prev[8];
            prev_hash_words(x - 1u, prev);
            const uint64_t time = P.genesis_time + (uint64_t)P.block_period * ((uint64_t)blk_T(b) + 1ull);
            nb = header_words(wb, prev, P.addresses + 20u * blk_prop(b), P.seed, inst, x, blk_prop(b), blk_var(b), time);
        }
        nb = wv.readlane(nb, enc);
        sync();
        uint32_t lo = 0, hi = 0;
        const uint32_t kx = lane & 7u, word = kx + 5u * (lane >> 3);     // keccak_wave's layout
        for (uint32_t blk = 0; blk < nb; ++blk) {
            if (kx < 5u && word < 17u) {
                const uint64_t w = wb[17u * blk + word];
                lo ^= (uint32_t)w;
                hi ^= (uint32_t)(w >> 32);
            }
            keccak_wave(lo, hi);
        }
        sync();
        for (uint32_t i = 0; i < 4u; ++i) {
            out[2 * i] = wv.readlane(lo, i);
            out[2 * i + 1] = wv.readlane(hi, i);
        }
    }
    // the deferred hashes of this phase's closed-form Core commits: one wave hash for the first
    // committer's block, taken by every committer of the same block; any other block by its own lane
    BFT_FN void resolve_deferred_hash() {
        const bool pend = hash_defer;
        const M pb = ballot(pend);
        if (pb.none()) return;
        hash_defer = false;
        const uint32_t lead = pb.ctz_nz();
        const uint32_t x0 = wv.readlane(commit_x, lead);
        const uint64_t b0 = (uint64_t)wv.readlane((uint32_t)commit_blk, lead) |
                            ((uint64_t)wv.readlane((uint32_t)(commit_blk >> 32), lead) << 32);
        uint32_t out[8];
        wave_block_hash(lead, x0, b0, out);
        // the same height and block id (time tick included) is the same header: the parent is the
        // canonical block x0 - 1 for every lane (chain_insert_core inserts x only on top of x - 1)
        const bool same = pend & (commit_x == x0) & (commit_blk == b0);
        if (same) {
            uint32_t* hs = (uint32_t*)(lds + LDS_CHASH_OFF + lane * 32);
            for (int i = 0; i < 8; ++i) hs[i] = out[i];
            const uint32_t sd = seed_from_words(out[0], out[1], nval(), P.seed_le != 0);
            commit_seed = sd;
            last_seed = sd;
        }
        if (pend & !same) {
            uint32_t prev[8], o[8];
            const uint64_t b = commit_blk;
            const uint32_t x = commit_x;
            prev_hash_words(x - 1u, prev);
            const uint64_t time = P.genesis_time + (uint64_t)P.block_period * ((uint64_t)blk_T(b) + 1ull);
            alignas(8) uint8_t pbuf[LANE_HASH_BUF];                  // private (scratch): a rare path
            lane_block_hash(pbuf, prev, P.addresses + 20u * blk_prop(b), P.seed, inst, x, blk_prop(b), blk_var(b),
                            time, o);
            uint32_t* hs = (uint32_t*)(lds + LDS_CHASH_OFF + lane * 32);
            for (int i = 0; i < 8; ++i) hs[i] = o[i];
            const uint32_t sd = seed_from_words(o[0], o[1], nval(), P.seed_le != 0);
            commit_seed = sd;
            last_seed = sd;
        }
        sync();
    }

    // the deferred hashes of this phase's closed-form Core commits, segments of S < 64 lanes: per segment the
    // first committer's block is hashed by lane pairs (every pair of the segment computes it; its header encoded
    // by that committer into its LDS buffer), and taken by every committer of the same block; any other block
    // by its own lane. Same hashes and seeds as chain_insert_core's lane_block_hash.
    BFT_FN void resolve_deferred_hash_seg() {
        const bool pend = hash_defer;
        const M pb = ballot(pend);
        if (pb.none()) return;
        hash_defer = false;
        const uint64_t sb = (pb.w[0] >> seg_base) & ((1ull << (S & 63u)) - 1ull);
        const uint32_t lead = seg_base + (sb ? (uint32_t)__builtin_ctzll(sb) : 0u);
        // the pending commit is commit_blk (its height blk_h: resolve_commits has cleared commit_x by now)
        const uint64_t b0 = (uint64_t)wv.shfl((uint32_t)commit_blk, lead) |
                            ((uint64_t)wv.shfl((uint32_t)(commit_blk >> 32), lead) << 32);
        const uint32_t x0 = blk_h(b0);
        uint8_t* sbuf = lds + LDS_SCR_OFF + (lane / S) * LANE_HASH_BUF;   // this segment's header buffer
        const uint32_t* wb = (const uint32_t*)sbuf;
        uint32_t nb = 0;
        uint32_t* tipc = (uint32_t*)(lds + LY::TIPC_OFF + (lane / S) * LY::TIPC_BYTES);
        if ((sb != 0u) & (lane == lead)) {
            uint32_t prev[8];
            if (tipc[0] == x0 - 1u) {
#pragma unroll
                for (int i = 0; i < 8; ++i) prev[i] = tipc[1 + i];
            } else {
                prev_hash_words(x0 - 1u, prev);
            }
            const uint64_t time = P.genesis_time + (uint64_t)P.block_period * ((uint64_t)blk_T(b0) + 1ull);
            nb = header_words((uint64_t*)sbuf, prev, P.addresses + 20u * blk_prop(b0),
                              P.seed, inst, x0, blk_prop(b0), blk_var(b0), time);
        }
        BFT_STAMP(16);                                            // (diagnostic) the lead's header encoding
        const uint32_t nbm = ballot(nb > 2u).any() ? 3u : 2u;     // rate blocks: 2 or 3 (header_words)
        nb = wv.shfl(nb, lead);
        sync();                                                   // the headers in LDS
        const uint32_t odd = lane & 1u;
        uint32_t X[25], h4[4];
#pragma unroll
        for (int i = 0; i < 25; ++i) X[i] = 0;
        for (uint32_t blk = 0; blk < nbm; ++blk) {
#pragma unroll
            for (uint32_t i = 0; i < 17u; ++i) X[i] ^= wb[34u * blk + 2u * i + odd];
            wv.keccak_pair(X, odd);                              // W: lane pairs (bft_hip.h), one collective (emulator)
            const bool fin = blk + 1u == nb;                      // a 2-block header's hash is taken here
#pragma unroll
            for (int i = 0; i < 4; ++i) h4[i] = (fin | (blk == 0u)) ? X[i] : h4[i];
        }
        BFT_STAMP(17);                                            // (diagnostic) the lane-pair permutations
        uint32_t out[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t o = wv.pair_swap(h4[i]);
            out[2 * i] = odd ? o : h4[i];
            out[2 * i + 1] = odd ? h4[i] : o;
        }
        sync();                                                   // header buffers read before any rewrite
        const bool same = pend & (commit_blk == b0);
        if (same) {
            uint32_t* hs = (uint32_t*)(lds + LDS_CHASH_OFF + lane * 32);
            for (int i = 0; i < 8; ++i) hs[i] = out[i];
            const uint32_t sd = seed_from_words(out[0], out[1], nval(), P.seed_le != 0);
            commit_seed = sd;
            last_seed = sd;
        }
        if (pend & !same) {
            uint32_t prev[8], o[8];
            const uint64_t b = commit_blk;
            const uint32_t x = blk_h(b);
            prev_hash_words(x - 1u, prev);
            const uint64_t time = P.genesis_time + (uint64_t)P.block_period * ((uint64_t)blk_T(b) + 1ull);
            alignas(8) uint8_t pbuf[LANE_HASH_BUF];                  // private (scratch): a rare path
            lane_block_hash(pbuf, prev, P.addresses + 20u * blk_prop(b), P.seed, inst, x, blk_prop(b), blk_var(b),
                            time, o);
            uint32_t* hs = (uint32_t*)(lds + LDS_CHASH_OFF + lane * 32);
            for (int i = 0; i < 8; ++i) hs[i] = o[i];
            const uint32_t sd = seed_from_words(o[0], o[1], nval(), P.seed_le != 0);
            commit_seed = sd;
            last_seed = sd;
        }
        // The canonical tip recorded this tick by resolve_commits before its hash was known (a hash deferred
        // past its phase): its seed word and hash row are written now by the lowest pending lane that holds
        // that block, and its seed becomes the segment's canonical tip seed and the tip seed of every lane
        // that took the tip by block gossip in the meantime (refresh_tip_from_table).
        const bool holds = pend & (commit_blk == canon_tip) & (canon_tick == (uint32_t)tick);
        const uint64_t hb = (ballot(holds).w[0] >> seg_base) & ((1ull << (S & 63u)) - 1ull);
        const uint32_t hl = seg_base + (hb ? (uint32_t)__builtin_ctzll(hb) : 0u);
        const uint32_t csd = wv.shfl(commit_seed, hl);
        if (hb != 0u) {
            if (lane == hl) {
                rec_row(canon_h)[3] = commit_seed;
                const uint32_t* hs = (const uint32_t*)(lds + LDS_CHASH_OFF + lane * 32);
                uint32_t* dst = (uint32_t*)hash_row(canon_h);
                wv.gstore4(dst, hs[0], hs[1], hs[2], hs[3]);
                wv.gstore4(dst + 4, hs[4], hs[5], hs[6], hs[7]);
                tipc[0] = canon_h;                        // the next height's prev_hash
#pragma unroll
                for (int i = 0; i < 8; ++i) tipc[1 + i] = hs[i];
            }
            canon_tip_seed = csd;
            if (seed_stale) last_seed = csd;
        }
        canon_stale = false;
        seed_stale = false;
        sync();
    }
    // (SEG_HASH) at the top of every phase: the closed-form commits of the phases before keep their hashes
    // pending while nothing in the tick can read them, so that the commits of one height spread over several
    // phases of a tick share one segment hash. They are resolved when the tick's phases end (`fin`); when a
    // pending block was minted before this tick, since its successor can be minted within the tick (miner_mine:
    // T = max(tick, last_T + 1)), while a block of this tick cannot (T > tick); and before a phase that carries a
    // Round Change, which can start a round at the committed height and read its tip seed (start_new_round).
    // One call site of resolve_deferred_hash_seg (it is inlined).
    BFT_FN void phase_hashes(bool fin) {
        const bool pend = hash_defer;
        if (ballot(pend).none()) return;
        const bool now = fin | (pend & (blk_T(commit_blk) < (uint32_t)tick)) | ((nx.f & F_RC) != 0u);
        if (ballot(now).any()) { resolve_deferred_hash_seg(); return; }
        const bool holds = pend & (commit_blk == canon_tip) & (canon_tick == (uint32_t)tick);
        canon_stale = ((ballot(holds).w[0] >> seg_base) & ((1ull << (S & 63u)) - 1ull)) != 0u;
    }

    BFT_FN uint32_t canon_seed(uint32_t x) {
        if (x == 0) return P.genesis_seed;
        if constexpr (SEG_HASH) BFT_EMU_CHECK(!(canon_stale & (x == canon_h)), "canon_seed of a stale canonical tip");
        if (x == canon_h) return canon_tip_seed;
        check_window(x);
        return wv.gload(rec_row(x) + 3);
    }
    // canonical block id at x (x >= 1, must be recorded)
    BFT_FN uint64_t canon_blk(uint32_t x) {
        if (x == canon_h && x != 0) return canon_tip;
        check_window(x);
        uint32_t w1 = wv.gload(rec_row(x) + 1);
        uint32_t T = wv.gload(rec_row(x) + 2);
        return blk_make(x, w1 & 0xffffu, (w1 >> 16) & 1u, T);
    }
    BFT_FN void prev_hash_words(uint32_t x, uint32_t w[8]) {         // hash of canonical block x
        if (x == 0) {
            for (int i = 0; i < 8; ++i)
                w[i] = (uint32_t)P.genesis_hash[4 * i] | ((uint32_t)P.genesis_hash[4 * i + 1] << 8) |
                       ((uint32_t)P.genesis_hash[4 * i + 2] << 16) | ((uint32_t)P.genesis_hash[4 * i + 3] << 24);
            return;
        }
        check_window(x);
        const uint32_t* p = (const uint32_t*)hash_row(x);
        for (int i = 0; i < 8; ++i) w[i] = wv.gload(p + i);
    }

    // ---------------------------------------------------------------- outbox (backend.rs:140-160)
    // The outbound cache of ImplBackend::gossip (backend.rs:141-148): a message identical to the last
    // one of its kind is not sent (nor self-delivered). Kept in LDS, {height, round, blk_d32} per kind.
    BFT_FN uint32_t* cache_p(uint32_t w) const { return (uint32_t*)(lds + LDS_CACHE_OFF) + w * LY::L + lane; }
    BFT_FN bool cache_hit(uint32_t kind, uint32_t vh, uint32_t vr, uint64_t d) {
        const uint32_t d32 = blk_d32(d);
        uint32_t* c = cache_p(3u * kind);
        const uint32_t sd = c[2u * LY::L];
        if (sd != 0 && c[0] == vh && c[LY::L] == vr && sd == d32) return true;
        c[0] = vh; c[LY::L] = vr; c[2u * LY::L] = d32;
        return false;
    }
    BFT_FN void out_preprepare(uint32_t vh, uint32_t vr, uint64_t b, bool equiv) {
        if (cache_hit(0, vh, vr, b)) return;
        if (nx.f & F_PP) { lane_flags |= FLAG_OUTBOX; return; }
        nx.f |= F_PP | (equiv ? F_PP_EQ : 0u); nx.pp_h = vh; nx.pp_r = vr; nx.pp_b = b;
    }
    BFT_FN void out_prepare(uint32_t vh, uint32_t vr, uint64_t d, bool wild) {
        if (cache_hit(1, vh, vr, d)) return;
        if (nx.f & F_PR) { lane_flags |= FLAG_OUTBOX; return; }
        nx.f |= F_PR | (wild ? F_PR_W : 0u); nx.pr_h = vh; nx.pr_r = vr; nx.pr_d = d;
    }
    BFT_FN void out_commit(uint32_t vh, uint32_t vr, uint64_t d, bool wild) {
        if (cache_hit(2, vh, vr, d)) return;
        if (nx.f & F_CM) { lane_flags |= FLAG_OUTBOX; return; }
        nx.f |= F_CM | (wild ? F_CM_W : 0u); nx.cm_h = vh; nx.cm_r = vr; nx.cm_d = d;
    }
    BFT_FN void out_old_commit(uint32_t vh, uint32_t vr, uint64_t d, bool wild) {
        if (cache_hit(3, vh, vr, d)) return;
        if (nx.f & F_OCM) { lane_flags |= FLAG_OUTBOX; return; }
        nx.f |= F_OCM | (wild ? F_OCM_W : 0u);
        nx.ocm_h = vh; nx.ocm_r = vr; nx.ocm_d = d;
    }
    BFT_FN void out_round_change(uint32_t vh, uint32_t vr) {
        if (nx.f & F_RC) { lane_flags |= FLAG_OUTBOX; return; }
        nx.f |= F_RC;
        nx.rc_h = vh; nx.rc_r = vr;
    }
    BFT_FN void out_sync(uint32_t height) {
        if (nx.f & F_SYNC) { if (height < nx.sync_h) nx.sync_h = height; return; }
        nx.f |= F_SYNC; nx.sync_h = height;
    }
    BFT_FN void out_blocks(uint32_t lo, uint32_t hi) {
        if (lo > hi) return;
        if (!(nx.f & F_BLK)) { nx.f |= F_BLK; nx.blk_lo = lo; nx.blk_hi = hi; return; }
        if (lo < nx.blk_lo) nx.blk_lo = lo;
        if (hi > nx.blk_hi) nx.blk_hi = hi;
    }

    // ---------------------------------------------------------------- timers, chain, miner
    BFT_FN void new_round_change_timer() { timer_tick = tick + 1; }     // core.rs:643-657
    BFT_FN void stop_timer() { timer_tick = -1; }                         // core.rs:638-641

    // the tip moved to a block recorded by an earlier phase: refresh its time tick and seed
    BFT_FN void refresh_tip_from_table() {
        if (last == canon_h && canon_h != 0) {            // the common case: tip = canonical tip
            last_T = (int32_t)blk_T(canon_tip);
            last_seed = canon_tip_seed;
            if constexpr (SEG_HASH) seed_stale = canon_stale;
            return;
        }
        check_window(last);
        last_T = (int32_t)wv.gload(rec_row(last) + 2);
        last_seed = wv.gload(rec_row(last) + 3);
        if constexpr (SEG_HASH) seed_stale = false;
    }

    // Chain::insert_block for a Core commit (core/chain.rs:45-71 via backend.rs:163-200)
    BFT_FN void chain_insert_core(uint64_t b) {
        uint32_t x = blk_h(b);
        if (x <= last) return;                              // ChainError::Exists
        if (last + 1 < x) { out_sync(last + 1); return; }    // Not found ancestor → SyncBlock
        if (commit_x != 0) lane_flags |= FLAG_OUTBOX;        // (cannot happen: one insert per phase)
        commit_x = x;
        commit_blk = b;
        commit_round = r;
        if (EXT && P.vsnap) {                               // real-crypto mode: the votes of this commit
            uint32_t* vs = P.vsnap + ((uint64_t)inst_local * S + me) * 8u;   // (core.rs:402-413)
            for (uint32_t k = 0; k < 8u; ++k) vs[k] = k < 2u * NW ? (uint32_t)(comm.w[k >> 1] >> (32u * (k & 1u))) : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // read by the recording lane
#endif
        }
        uint32_t sd = 0;
        if ((WAVE_HASH || SEG_HASH) && in_pc) {
            // the closed form delivers the whole phase: nothing reads this commit's hash or seed before
            // resolve_commits, and resolve_deferred_hash runs just before it
            hash_defer = true;
        } else if (NEED_SEED) {
            uint32_t prev[8], out[8];
            prev_hash_words(last, prev);
            uint64_t time = P.genesis_time + (uint64_t)P.block_period * ((uint64_t)blk_T(b) + 1ull);
            {
                // private (scratch): the commits of the one-message-at-a-time path and the opt-in modes; LDS holds
                // one header buffer per segment only (Layout)
                alignas(8) uint8_t pbuf[LANE_HASH_BUF];
                lane_block_hash(pbuf, prev, P.addresses + 20u * blk_prop(b), P.seed, inst, x, blk_prop(b),
                                blk_var(b), time, out);
            }
            uint32_t* hs = (uint32_t*)(lds + LDS_CHASH_OFF + lane * 32);
            for (int i = 0; i < 8; ++i) hs[i] = out[i];
            sd = seed_from_words(out[0], out[1], nval(), P.seed_le != 0);
        }
        commit_seed = sd;
        last = x;
        last_T = (int32_t)blk_T(b);
        last_seed = sd;
        if constexpr (SEG_HASH) seed_stale = false;         // a deferred hash: resolve_deferred_hash_seg sets it
        out_blocks(x, x);                                   // ChainEvent::NewBlock (chain.rs:61)
        if (x > miner_queue) miner_queue = x;               // ChainEvent::NewHeader (chain.rs:62)
    }

    // handle_msg_middle Block branch (core.rs:75-82): insert lo..hi in order, unverified
    BFT_FN void handle_blocks(uint32_t lo, uint32_t hi) {
        if (hi <= last) return;                             // all Exists
        if (lo > last + 1) { out_sync(last + 1); return; }  // every block is a gap
        uint32_t from = last + 1;
        last = hi;
        refresh_tip_from_table();
        out_blocks(from, hi);
        if (hi > miner_queue) miner_queue = hi;
    }

    // handle_msg_middle Sync branch (core.rs:83-110)
    BFT_FN void handle_sync(uint32_t height) {
        if (height > last) return;
        uint32_t hi = last < height + 101u ? last : height + 101u;
        out_blocks(height, hi);
    }

    // Minner::mine + packet_next_block + next_block + Engine::seal (minner/mod.rs:95-143)
    BFT_FN void miner_mine() {
        uint32_t x = last + 1;
        int32_t T = tick > last_T + 1 ? tick : last_T + 1;
        cand = blk_make(x, me, 0, (uint32_t)T);
        mint_height = x;
        wake_tick = T;
        if (T > tick) return;            // seal sleeps until header.time (backend.rs:437-449)
        wake_tick = -1;
        handle_new_header_event();
    }
    // Minner: Handler<ChainEvent::NewHeader> (minner/mod.rs:56-69)
    BFT_FN void miner_step() {
        if (wake_tick >= 0) return;
        uint32_t q = miner_queue;
        miner_queue = 0;
        if (q != 0 && q >= mint_height) miner_mine();
    }

    // ---------------------------------------------------------------- Core
    BFT_FN bool is_proposer(uint32_t who) const { return proposer == who; }
    BFT_FN uint32_t mod_n(uint32_t x) const { return P.nmask ? (x & P.nmask) : x % P.n; }   // proposer index

    // Core::check_message (core.rs:366-399): 0 ok, 1 unknown, 2 future block, 3 old, 4 future msg
    BFT_FN int check_message(int code, uint32_t vh) const { return check_message_class(code, vh, h, st); }
    BFT_FN void note_future_block(uint32_t vh) { if (vh > sync_pending) sync_pending = vh; }
    BFT_FN void lock_hash() { if (blk_valid(pp)) lock = pp; }               // round_state.rs:100-110

    BFT_FN void send_preprepare(uint64_t req) {                               // preprepare.rs:30-43
        if (h == blk_h(req) && is_proposer(me)) {
            if (proposer_crashed(P.seed, P.crash_thr32, P.crash_on, inst, h, r)) return;
            bool equiv = byz && blk_prop(req) == me && blk_var(req) == 0;
            out_preprepare(h, r, req, equiv);
        }
    }
    BFT_FN void send_prepare() {                                              // prepare.rs:28-38
        out_prepare(h, r, pp, byz);
        if (byz) out_commit(h, r, pp, true);
    }
    BFT_FN void send_commit() { out_commit(h, r, pp, byz); }                 // commit.rs:37-60
    BFT_FN void catchup_round() { wait = true; new_round_change_timer(); }   // core.rs:555-565

    BFT_FN void send_round_change(uint32_t round) {                          // round_change.rs:38-63
        if (rc_last_tick == tick) { new_round_change_timer(); return; }
        rc_last_tick = tick;
        if (r < round) catchup_round();
        out_round_change(h, round);
    }
    // RoundChangeSet table (global, lane-private), SoA [k][lane]: coalesced per wave
    BFT_FN uint32_t* rc_round_p(uint32_t k) const { return rcs_base + k * LY::L + lane; }
    BFT_FN uint32_t* rc_word_p(uint32_t k, uint32_t j) const {
        return rcs_base + (rcs_k + k * 2u * NW + j) * LY::L + lane;
    }
    BFT_FN M rc_set_at(uint32_t k) const {
        M m;
        for (int j = 0; j < NW; ++j) m.w[j] = (uint64_t)*rc_word_p(k, 2 * j) | ((uint64_t)*rc_word_p(k, 2 * j + 1) << 32);
        return m;
    }
    BFT_FN void rc_set_store(uint32_t k, const M& m) {
        for (int j = 0; j < NW; ++j) { *rc_word_p(k, 2 * j) = (uint32_t)m.w[j]; *rc_word_p(k, 2 * j + 1) = (uint32_t)(m.w[j] >> 32); }
    }

    BFT_FN uint32_t rcs_max_round() const {                                  // round_change_set.rs:64-74
        uint32_t mx = 0;
        int total = 0;
        for (uint32_t i = 0; i < n_rcs; ++i) {               // ascending rounds (canonical order)
            int len = (int)rc_set_at(i).popc();
            uint32_t rd = *rc_round_p(i);
            if (len >= total && rd > mx) { mx = rd; total = len; }
        }
        return mx;
    }
    // the entry of `round` (round_change_set.rs:28-35 `entry().or_insert`), inserted empty in ascending
    // round order if absent; -1 when the table is full (flagged: outputs after it are not parity-pinned)
    BFT_FN int rcs_slot(uint32_t round) {
        uint32_t pos = 0;
        while (pos < n_rcs && *rc_round_p(pos) < round) ++pos;
        if (pos == n_rcs || *rc_round_p(pos) != round) {
            if (n_rcs == rcs_k) { lane_flags |= FLAG_RCS_OVERFLOW; return -1; }
            for (uint32_t i = n_rcs; i > pos; --i) {
                *rc_round_p(i) = *rc_round_p(i - 1);
                for (uint32_t j = 0; j < 2u * NW; ++j) *rc_word_p(i, j) = *rc_word_p(i - 1, j);
            }
            *rc_round_p(pos) = round;
            rc_set_store(pos, M::zero());
            n_rcs += 1;
        }
        return (int)pos;
    }
    BFT_FN int rcs_add(uint32_t round, uint32_t sender) {                    // round_change_set.rs:28-35
        const int pos = rcs_slot(round);
        if (pos < 0) return 0;
        M set = rc_set_at((uint32_t)pos) | M::bit(sender);
        rc_set_store((uint32_t)pos, set);
        return (int)set.popc();
    }
    BFT_FN void send_next_round_change() {                                   // round_change.rs:26-36
        uint32_t round = rcs_max_round();
        if (round <= r) send_round_change(r + 1);
        else send_round_change(round);
    }

    BFT_FN void start_new_zero_round() {                                     // core.rs:441-470
        // (SEG_HASH) the tip's seed is read below: its hash must not be pending (phase_hashes resolves it first)
        if constexpr (SEG_HASH) BFT_EMU_CHECK(!seed_stale, "start_new_zero_round reads a stale tip seed");
        uint32_t last_height = last;
        h = last_height + 1;
        r = 0;
        n_rcs = 0;
        lock = pp = pend = BLK_NONE;
        prep = comm = M::zero();
        proposer = mod_n(last_seed);
        wait = false;
        st = ST_ACCEPT_REQUEST;
        new_round_change_timer();
    }

    BFT_FN void start_new_round(uint32_t round) {                            // core.rs:474-551
        uint32_t last_height = last;
        if (last_height > h) return;
        if constexpr (SEG_HASH) BFT_EMU_CHECK(!seed_stale, "start_new_round reads a stale tip seed");
        n_rcs = 0;
        if (!blk_valid(lock)) pp = BLK_NONE;
        prep = comm = M::zero();
        r = round;
        proposer = mod_n(last_seed + round);
        wait = false;
        st = ST_ACCEPT_REQUEST;
        if (is_proposer(me)) {
            if (blk_valid(lock)) {
                send_preprepare(pp);
            } else {
                if (!blk_valid(pend)) { core_dead = true; lane_flags |= FLAG_CORE_PANIC; return; }
                send_preprepare(pend);
            }
        }
        new_round_change_timer();
    }

    BFT_FN void handle_new_header_event() {                // core.rs:154-163 + request.rs:19-42
        if (core_dead) return;
        start_new_zero_round();
        uint64_t req = cand;
        if (h != blk_h(req)) return;                       // OldMessage / FutureMessage
        pend = req;
        send_preprepare(req);
    }

    BFT_FN void handle_timer_event() {                     // core.rs:207-225
        if (last >= h) { stop_timer(); wait = false; }
        else send_next_round_change();
    }

    BFT_FN void core_commit() {                            // core.rs:402-422
        st = ST_COMMITTED;
        chain_insert_core(pp);
    }

    BFT_FN void handle_preprepare(uint32_t src, uint32_t vh, uint32_t vr, uint64_t b, bool equiv) {   // preprepare.rs:45-126
        if (equiv && me != src && split_bit(P.seed, inst, vh, vr, me)) b |= 1ull << 33;
        int res = check_message(1, vh);
        if (res != 0) {
            if (res == 3) {
                uint32_t bh = blk_h(b);
                if (bh > last) return;                                        // InvalidProposal
                if (!blk_eq(canon_blk(bh), b)) return;                        // InvalidProposal
                uint32_t old_prop = mod_n(canon_seed(bh - 1) + vr);
                if (old_prop == src) out_old_commit(vh, vr, b, byz);
            } else if (res != 2) {
                return;
            }
        }
        if (!is_proposer(src)) return;                                        // NotFromProposer
        if (blk_h(b) == 0 || blk_h(b) - 1 > last) { send_next_round_change(); return; }  // verify
        if (st == ST_ACCEPT_REQUEST) {
            if (blk_valid(lock)) {
                if (blk_eq(b, lock)) { pp = b; st = ST_PREPARED; send_commit(); }
                else send_next_round_change();
            } else {
                pp = b; st = ST_PREPREPARED; send_prepare();
            }
        }
    }

    BFT_FN void handle_prepare(uint32_t src, uint32_t vh, uint32_t vr, uint64_t d, bool wild) {   // prepare.rs:48-66
        int res = check_message(2, vh);
        if (res != 0) {
            if (res == CM_FUTURE_BLOCK) note_future_block(vh);
            else if (res == CM_FUTURE_MSG) backlog_store(src, MT_PREPARE, vh, vr, d, wild);
            return;
        }
        if (vh != h || vr != r) return;
        prep.set(src);
        if (blk_valid(lock) && digest_match(d, wild, lock)) { lock_hash(); st = ST_PREPARED; send_commit(); }
        if ((prep | comm).popc() > qval()) { lock_hash(); st = ST_PREPARED; send_commit(); }
    }

    BFT_FN void handle_commit(uint32_t src, uint32_t vh, uint32_t vr, uint64_t d, bool wild) {    // commit.rs:63-111
        int res = check_message(3, vh);
        if (res != 0) {
            if (res == CM_FUTURE_BLOCK) note_future_block(vh);
            else if (res == CM_FUTURE_MSG) backlog_store(src, MT_COMMIT, vh, vr, d, wild);
            return;
        }
        if (!digest_match(d, wild, pp) || vh != h || vr != r) return;
        comm.set(src);
        if (comm.popc() > qval() && st < ST_COMMITTED) { lock_hash(); core_commit(); }
    }

    BFT_FN void handle_round_change(uint32_t src, uint32_t vh, uint32_t mr) {   // round_change.rs:65-98
        int res = check_message(4, vh);
        if (res != 0) { if (res == 2) note_future_block(vh); return; }
        if (r > mr && mr > 0) { send_round_change(mr); return; }
        int n = rcs_add(mr, src);
        if ((uint32_t)n >= qval() + 1u && wait && r < mr) {
            send_round_change(mr);
            start_new_round(mr);
        } else if (wait && r < mr) {                     // FutureRoundMessage (round_change.rs:93-96)
            backlog_store(src, MT_ROUND_CHANGE, vh, mr, 0, false);
        }
    }

    // ---------------------------------------------------------------- backlog replay (SPEC.md §10)
    // BackLogActor (back_log.rs:38-65): per sender the first FutureMessage / FutureRoundMessage is kept.
    // The reference never re-delivers it (outside replay mode nothing is stored: dropped). Slot of
    // sender s: words [s][k][lane], k = {valid | code << 1 | wild << 4, height, round, digest lo, hi}.
    BFT_FN uint32_t* bl_p(uint32_t s, uint32_t k) const { return bl_base + (s * 5u + k) * LY::L + lane; }
    BFT_FN void backlog_store(uint32_t src, int code, uint32_t vh, uint32_t vr, uint64_t d, bool wild) {
        if (!EXT || !P.backlog_replay) return;
        if (*bl_p(src, 0) & 1u) return;                  // or_insert_with: the first message stays
        *bl_p(src, 0) = 1u | ((uint32_t)code << 1) | (wild ? 16u : 0u);
        *bl_p(src, 1) = vh; *bl_p(src, 2) = vr;
        *bl_p(src, 3) = (uint32_t)d; *bl_p(src, 4) = (uint32_t)(d >> 32);
    }
    // the stored messages in ascending sender order, each slot emptied and handled as a BackLogEvent
    // (core.rs:197-204); one that is again a Future(Round)Message is stored again
    BFT_FN void replay_backlog() {
        const uint32_t n = nval();
        for (uint32_t s = 0; s < n; ++s) {
            const uint32_t hd = *bl_p(s, 0);
            if (!(hd & 1u)) continue;
            const uint32_t vh = *bl_p(s, 1), vr = *bl_p(s, 2);
            const uint64_t d = (uint64_t)*bl_p(s, 3) | ((uint64_t)*bl_p(s, 4) << 32);
            *bl_p(s, 0) = 0;
            if (core_dead) return;
            const int code = (int)((hd >> 1) & 7u);
            if (code == MT_PREPARE) handle_prepare(s, vh, vr, d, (hd & 16u) != 0);
            else if (code == MT_COMMIT) handle_commit(s, vh, vr, d, (hd & 16u) != 0);
            else handle_round_change(s, vh, vr);
        }
    }

    // ---------------------------------------------------------------- real-crypto mode (SPEC.md §11)
    // At the start of a phase every sender's consensus messages (the outbox kinds that are
    // GossipMessages: Preprepare, Prepare, old-block Commit, Commit, RoundChange) are broadcast, i.e.
    // signed (core.rs:425-429). They are logged in (sender, kind) order for the batched sign / recover
    // pass; a forged sender's signature recovers a non-validator, so handle_message (core.rs:314-322)
    // drops them at every receiver, the sender included: they leave the outbox here.
    static constexpr uint32_t F_CONS = F_PP | F_PP_EQ | F_PR | F_PR_W | F_CM | F_CM_W | F_OCM | F_OCM_W | F_RC;
    BFT_FN void mlog_put(uint32_t idx, uint32_t code, uint32_t h_, uint32_t r_, uint64_t b, uint32_t fl,
                         uint32_t phase) {
        if (idx >= P.mlog_cap) return;                // counted, not stored: overflow (bftsim_crypto_verify)
        uint32_t* e = P.mlog + ((uint64_t)inst_local * P.mlog_cap + idx) * MLOG_WORDS;
        e[0] = (uint32_t)tick; e[1] = phase | (code << 8) | (me << 16); e[2] = h_; e[3] = r_;
        e[4] = (uint32_t)b; e[5] = (uint32_t)(b >> 32); e[6] = fl; e[7] = 0;
    }
    BFT_FN void crypto_log(bool act, uint32_t phase) {
        const uint32_t f = act ? nx.f : 0u;
        const uint32_t nk = ((f & F_PP) ? 1u : 0u) + ((f & F_PR) ? 1u : 0u) + ((f & F_OCM) ? 1u : 0u) +
                            ((f & F_CM) ? 1u : 0u) + ((f & F_RC) ? 1u : 0u);
        // this lane's first slot: the messages of the lower senders of the segment (3 ballots of nk's bits)
        const M below = seg_mask & M::low(lane);
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (uint32_t b = 0; b < 3; ++b) {
            const M bb = ballot(((nk >> b) & 1u) != 0);
            pre += (bb & below).popc() << b;
            tot += (bb & seg_mask).popc() << b;
        }
        uint32_t idx = mlog_cnt + pre;
        const bool forged = is_val && ((P.forged[(me >> 6) & 3u] >> (me & 63u)) & 1ull);
        const uint32_t ff = forged ? MLOG_FORGED : 0u;
        if (f & F_PP) mlog_put(idx++, MT_PREPREPARE, nx.pp_h, nx.pp_r, nx.pp_b, ff | ((f & F_PP_EQ) ? MLOG_EQUIV : 0u), phase);
        if (f & F_PR) mlog_put(idx++, MT_PREPARE, nx.pr_h, nx.pr_r, nx.pr_d, ff | ((f & F_PR_W) ? MLOG_WILD : 0u), phase);
        if (f & F_OCM) mlog_put(idx++, MT_COMMIT, nx.ocm_h, nx.ocm_r, nx.ocm_d, ff | MLOG_OLD | ((f & F_OCM_W) ? MLOG_WILD : 0u), phase);
        if (f & F_CM) mlog_put(idx++, MT_COMMIT, nx.cm_h, nx.cm_r, nx.cm_d, ff | ((f & F_CM_W) ? MLOG_WILD : 0u), phase);
        if (f & F_RC) mlog_put(idx++, MT_ROUND_CHANGE, nx.rc_h, nx.rc_r, 0, ff, phase);
        mlog_cnt += tot;
        if (forged) nx.f &= ~F_CONS;
    }

    // ---------------------------------------------------------------- phase machinery
    BFT_FN uint32_t* rec_lds(uint32_t l) const { return (uint32_t*)(lds + LDS_REC_OFF) + l * REC_WORDS; }

    BFT_FN void publish() {      // nx → LDS (this lane's slot; only the kinds present), clear nx
        uint32_t* o = rec_lds(lane);
        const uint32_t f = nx.f;
        o[0] = f;
        if (f & F_PP) { o[1] = nx.pp_h; o[2] = nx.pp_r; o[3] = (uint32_t)nx.pp_b; o[4] = (uint32_t)(nx.pp_b >> 32); }
        if (f & F_PR) { o[5] = nx.pr_h; o[6] = nx.pr_r; o[7] = (uint32_t)nx.pr_d; o[8] = (uint32_t)(nx.pr_d >> 32); }
        if (f & F_CM) { o[9] = nx.cm_h; o[10] = nx.cm_r; o[11] = (uint32_t)nx.cm_d; o[12] = (uint32_t)(nx.cm_d >> 32); }
        if (f & F_OCM) { o[13] = nx.ocm_h; o[14] = nx.ocm_r; o[15] = (uint32_t)nx.ocm_d; o[16] = (uint32_t)(nx.ocm_d >> 32); }
        if (f & F_RC) { o[17] = nx.rc_h; o[18] = nx.rc_r; }
        if (f & F_SYNC) o[19] = nx.sync_h;
        if (f & F_BLK) { o[20] = nx.blk_lo; o[21] = nx.blk_hi; }
        outbox_clear(nx);
    }

    BFT_FN void deliver_from(uint32_t s) {     // all messages of sender s (SPEC.md §2 order)
        const uint32_t* m = rec_lds(seg_base + s);
        uint32_t f = m[0];
        if (f == 0) return;
        if (s != me && (f & F_BLK)) handle_blocks(m[20], m[21]);
        if (s != me && (f & F_SYNC)) handle_sync(m[19]);
        if (core_dead) return;
        if (f & F_PP) {
            handle_preprepare(s, m[1], m[2], (uint64_t)m[3] | ((uint64_t)m[4] << 32), (f & F_PP_EQ) != 0);
            if (core_dead) return;
        }
        if (f & F_PR) handle_prepare(s, m[5], m[6], (uint64_t)m[7] | ((uint64_t)m[8] << 32), (f & F_PR_W) != 0);
        if (f & F_OCM) handle_commit(s, m[13], m[14], (uint64_t)m[15] | ((uint64_t)m[16] << 32), (f & F_OCM_W) != 0);
        if (f & F_CM) handle_commit(s, m[9], m[10], (uint64_t)m[11] | ((uint64_t)m[12] << 32), (f & F_CM_W) != 0);
        if (f & F_RC) handle_round_change(s, m[17], m[18]);
    }

    BFT_FN bool pending_local() const {
        return running & ((nx.f != 0) | ((wake_tick < 0) & (miner_queue != 0) & (miner_queue >= mint_height)));
    }

    BFT_FN void t_step() {
        if (tick == 0) {
            start_new_zero_round();          // Core::started (core.rs:144-147)
            miner_mine();                    // Minner::started (minner/mod.rs:43-48)
            return;
        }
        if (wake_tick == tick) { wake_tick = -1; handle_new_header_event(); }
        miner_step();
        if (sync_pending) {
            if (last < sync_pending) out_sync(last + 1);
            sync_pending = 0;
        }
        if (!core_dead && timer_tick == tick) { timer_tick = -1; handle_timer_event(); }
        if (EXT && P.backlog_replay) replay_backlog();   // SPEC.md §10
    }

    // segment collectives: ballots as sender bitmaps; reductions (butterfly inside a wave
    // segment, LDS-combined per-wave partials for a workgroup segment)
    BFT_FN M ballot(bool p) { return M::from(wv.ballot(p)); }
    // segment-uniform value: into a scalar register when the segment is the whole wave
    BFT_FN uint32_t uni(uint32_t v) {
        if constexpr (S == 64) return wv.uni(v);
        else return v;
    }
    BFT_FN uint32_t nval() const { return P.n; }
    BFT_FN uint32_t qval() const { return P.q; }    // floor(2N/3)
    BFT_FN void sync() { wv.sync(); }
    BFT_FN uint32_t seg_max(uint32_t v) {
        if constexpr (S > 64) { return wv.grp_max(v); }
        else {
            for (uint32_t m = 1; m < S; m <<= 1) { uint32_t o = wv.shfl_xor(v, m); v = v > o ? v : o; }
            return v;
        }
    }
    BFT_FN uint64_t seg_sum64(uint32_t v32) {
        if constexpr (S > 64) { return wv.grp_sum64(v32); }
        else {
            uint64_t v = v32;
            for (uint32_t m = 1; m < S; m <<= 1) {
                uint32_t lo = wv.shfl_xor((uint32_t)v, m), hi = wv.shfl_xor((uint32_t)(v >> 32), m);
                v += (uint64_t)lo | ((uint64_t)hi << 32);
            }
            return v;
        }
    }
    BFT_FN uint32_t seg_or(uint32_t v) {
        if constexpr (S > 64) { return wv.grp_or(v); }
        else {
            for (uint32_t m = 1; m < S; m <<= 1) v |= wv.shfl_xor(v, m);
            return v;
        }
    }

    // histogram bins (LDS, per wave / workgroup)
    BFT_FN uint32_t* hist_slot(uint32_t b) const { return (uint32_t*)(lds + LDS_HIST_OFF) + b; }
    // record a new canonical height (segment leader; global stores for the outputs). `ctick` is the
    // tick of the previous canonical record; returns the instance-rounds to add (0 beyond H).
    BFT_FN uint32_t record_canon(uint32_t x, uint64_t b, uint32_t round, uint32_t seed, const uint32_t* hs,
                                 uint32_t ctick, uint32_t committer) {
        uint32_t add = 0;
        if (EXT && P.votes) {                               // the committer's commit set → the block's votes
#if defined(__HIP_DEVICE_COMPILE__)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
            const uint32_t* vs = P.vsnap + ((uint64_t)inst_local * S + committer) * 8u;
            uint32_t* vo = P.votes + row_of(x) * 8u;
            for (uint32_t k = 0; k < 8u; ++k) vo[k] = vs[k];
        }
        if (x <= P.heights) {
            uint32_t lat = (uint32_t)tick - ctick;
            wv.lds_add(hist_slot(round < 64u ? round : 64u), 1u);
            wv.lds_add(hist_slot(65u + (lat < 64u ? lat : 64u)), 1u);
            add = round + 1u;
        }
        // one 16-byte store per row (and two per hash row): whole 32-byte sectors, no partial writes
        wv.gstore4(rec_row(x), round, blk_prop(b) | (blk_var(b) << 16) | (1u << 24), blk_T(b), seed);
        if (NEED_SEED) {
            uint32_t* dst = (uint32_t*)hash_row(x);
            wv.gstore4(dst, hs[0], hs[1], hs[2], hs[3]);
            wv.gstore4(dst + 4, hs[4], hs[5], hs[6], hs[7]);
        }
        return add;
    }

    // first Core commits of the phase → canonical table, in lane order (oracle receiver order). Returns the
    // committed height when every committer of the segment committed the same one (segment-uniform), else 0.
    BFT_FN uint32_t resolve_commits() {
        bool c = commit_x != 0;
        M bal = ballot(c);
        if (bal.none()) return 0;
        if constexpr (S == 64) {
            // one instance per wave: the first committer's values by readlane, and when every committer
            // commits that same height (the common case) the canonical update is computed by all lanes
            // alike from uniform values — no LDS hand-off, no syncs; only the record stores are the
            // leader's. Same results as the general hand-off below (which handles mixed heights).
            const uint32_t lead = bal.ctz_nz();
            const uint32_t x0 = wv.readlane(commit_x, lead);
            const bool other_h = c && commit_x != x0;
            if (!seg_done && ballot(other_h).none()) {
                const uint64_t b0 = (uint64_t)wv.readlane((uint32_t)commit_blk, lead) |
                                    ((uint64_t)wv.readlane((uint32_t)(commit_blk >> 32), lead) << 32);
                const uint32_t r0 = wv.readlane(commit_round, lead), s0 = wv.readlane(commit_seed, lead);
                const bool x0_known = x0 <= canon_h;
                const uint64_t ref = x0_known ? canon_blk(x0) : b0;
                const M badm = ballot(c && !blk_eq(commit_blk, ref));
                bool fr = badm.any();
                if (!x0_known && x0 < P.hcap && (!fr || badm.ctz() > lead)) {
                    if (lane == lead)
                        record_canon(x0, b0, r0, s0, (const uint32_t*)(lds + LDS_CHASH_OFF + lead * 32), canon_tick,
                                     lead - seg_base);
                    views_acc += x0 <= P.heights ? (uint64_t)r0 + 1u : 0u;
                    canon_h = x0; canon_tip = b0; canon_tip_seed = s0; canon_tick = (uint32_t)tick;
                }
                if (x0 >= P.hcap) fr = true;
                if (fr) { frozen = true; seg_flags |= FLAG_SAFETY; }
                commit_x = 0;
                return x0;
            }
        }
        uint32_t* cm = (uint32_t*)(lds + LDS_CMT_OFF) + lane * LY::CMT_STRIDE;
        if (c) {
            cm[0] = commit_x; cm[1] = (uint32_t)commit_blk; cm[2] = (uint32_t)(commit_blk >> 32);
            cm[3] = commit_round; cm[4] = commit_seed;
        }
        sync();
        M segbits = bal & seg_mask;
        uint32_t* segw = (uint32_t*)(lds + LDS_SEG_OFF) + (lane / S) * 8;
        const bool mine = segbits.any() && !seg_done;
        const uint32_t lead = segbits.any() ? segbits.ctz_nz() : 0u;
        // fast path: every committer of the segment commits the same height as the first one
        const uint32_t* cl = (const uint32_t*)(lds + LDS_CMT_OFF) + lead * LY::CMT_STRIDE;
        uint32_t x0 = mine ? cl[0] : 0u;
        uint64_t b0 = mine ? ((uint64_t)cl[1] | ((uint64_t)cl[2] << 32)) : 0ull;
        bool other_h = c && mine && commit_x != x0;
        M mixed = ballot(other_h) & seg_mask;
        bool uniform = mixed.none();
        // canonical block of x0 as it was before this phase (heights are recorded contiguously)
        bool x0_known = x0 <= canon_h;
        uint64_t ref = 0;
        if (mine && uniform) ref = x0_known ? canon_blk(x0) : b0;
        bool bad = mine && uniform && c && !blk_eq(commit_blk, ref);
        M badm = ballot(bad) & seg_mask;
        if (mine && uniform && lane == lead) {
            // lanes below the first violating lane were processed before the freeze
            bool fr = badm.any();
            uint32_t ch = canon_h;
            uint64_t tip = canon_tip;
            uint32_t tseed = canon_tip_seed, ctick = canon_tick;
            uint64_t va = views_acc;
            if (!x0_known && x0 < P.hcap && (!fr || badm.ctz() > lead)) {
                va += record_canon(x0, b0, cl[3], cl[4], (const uint32_t*)(lds + LDS_CHASH_OFF + lead * 32), ctick,
                                   lead - seg_base);
                ch = x0; tip = b0; tseed = cl[4]; ctick = (uint32_t)tick;
            }
            if (x0 >= P.hcap) fr = true;
            segw[0] = ch;
            segw[1] = fr ? 1u : 0u;
            segw[2] = (uint32_t)tip;
            segw[3] = (uint32_t)(tip >> 32);
            segw[4] = tseed;
            segw[5] = (uint32_t)va;
            segw[6] = (uint32_t)(va >> 32);
            segw[7] = ctick;
        }
        if (mine && !uniform && lane == lead) {
            // general case: replay the commits of this phase in lane order
            uint32_t ch = canon_h;
            uint64_t tip = canon_tip;
            uint32_t tseed = canon_tip_seed, ctick = canon_tick;
            uint64_t va = views_acc;
            bool fr = false;
            M bits = segbits;
            while (bits.any()) {
                uint32_t j = bits.ctz_nz();
                bits.clear_lowest();
                const uint32_t* cj = (const uint32_t*)(lds + LDS_CMT_OFF) + j * LY::CMT_STRIDE;
                uint32_t x = cj[0];
                uint64_t b = (uint64_t)cj[1] | ((uint64_t)cj[2] << 32);
                if (x >= P.hcap) { fr = true; break; }
                if (x <= ch) {
                    uint64_t cb = (x == ch) ? tip : ((x == canon_h) ? canon_tip : canon_blk(x));
                    if (!blk_eq(cb, b)) { fr = true; break; }
                } else {
                    // x == ch + 1: heights are recorded contiguously
                    va += record_canon(x, b, cj[3], cj[4], (const uint32_t*)(lds + LDS_CHASH_OFF + j * 32), ctick,
                                       j - seg_base);
                    ch = x; tip = b; tseed = cj[4]; ctick = (uint32_t)tick;
                }
            }
            segw[0] = ch;
            segw[1] = fr ? 1u : 0u;
            segw[2] = (uint32_t)tip;
            segw[3] = (uint32_t)(tip >> 32);
            segw[4] = tseed;
            segw[5] = (uint32_t)va;
            segw[6] = (uint32_t)(va >> 32);
            segw[7] = ctick;
        }
        sync();
        if (mine) {
            canon_h = uni(segw[0]);
            canon_tip = (uint64_t)uni(segw[2]) | ((uint64_t)uni(segw[3]) << 32);
            canon_tip_seed = uni(segw[4]);
            views_acc = (uint64_t)uni(segw[5]) | ((uint64_t)uni(segw[6]) << 32);
            canon_tick = uni(segw[7]);
            if (uni(segw[1])) { frozen = true; seg_flags |= FLAG_SAFETY; }
        }
        commit_x = 0;
        sync();
        return (mine && uniform) ? x0 : 0u;
    }

    BFT_FN uint64_t state_digest() const {
        return (uint64_t)(h & 0xffffu) | ((uint64_t)(r & 0xffu) << 16) | ((uint64_t)(st & 7u) << 24) |
               ((uint64_t)(wait ? 1 : 0) << 27) | ((uint64_t)(last & 0xffffu) << 28) |
               ((uint64_t)(blk_valid(lock) ? 1 : 0) << 44) | ((uint64_t)(blk_valid(pp) ? 1 : 0) << 45) |
               ((uint64_t)(blk_valid(pend) ? 1 : 0) << 46) | ((uint64_t)(core_dead ? 1 : 0) << 47) |
               ((uint64_t)(prep.popc() & 0xffu) << 48) |
               ((uint64_t)(comm.popc() & 0xffu) << 56);
    }

    BFT_FN void init_byzantine() {       // partial Fisher-Yates by the segment's lane 0 (SPEC.md §5)
        uint8_t* perm = lds + LDS_CMT_OFF + seg_base;                   // segment scratch (S bytes)
        uint32_t* segw = (uint32_t*)(lds + LDS_SEG_OFF) + (lane / S) * 8;
        const uint32_t mw = NW == 1 ? 2u : 8u;                            // mask words in segw
        if (me == 0 && !seg_done) {
            uint32_t n = nval();
            for (uint32_t i = 0; i < n; ++i) perm[i] = (uint8_t)i;
            M mask = M::zero();
            uint32_t f = P.byz_count < n ? P.byz_count : n;
            for (uint32_t i = 0; i < f; ++i) {
                uint32_t w[4];
                philox(P.seed, inst, i, 0, DOM_BYZ, w);
                uint32_t j = i + w[0] % (n - i);
                uint8_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
                mask.set(perm[i]);
            }
            for (int k = 0; k < NW; ++k) { segw[mw + 2 * k] = (uint32_t)mask.w[k]; segw[mw + 2 * k + 1] = (uint32_t)(mask.w[k] >> 32); }
        }
        sync();
        M mask;
        for (int k = 0; k < NW; ++k) mask.w[k] = (uint64_t)segw[mw + 2 * k] | ((uint64_t)segw[mw + 2 * k + 1] << 32);
        byz = is_val && !seg_done && mask.get(me);
        sync();
    }

    // ---------------------------------------------------------------- phase fast paths
    // Segment-wide summary of one phase's messages. All masks use segment-local sender bits.
    // For S > 64 (one instance per workgroup) the 13 sender masks stay in LDS (GroupHip::summary(),
    // read where a path needs them: kmask) instead of 13 x NW 64-bit registers per lane; the kinds
    // present are the scalar bits `kinds`.
    enum : uint32_t { KM_PP = 0, KM_PR, KM_CM, KM_OCM, KM_RC, KM_SYNC, KM_BLK, KM_PR_W, KM_PR_V0, KM_PR_V1,
                      KM_CM_W, KM_CM_V0, KM_CM_V1, KM_COUNT };
    static constexpr uint32_t KB_PP1 = 1u << 7;   // kinds: bit k = mask k nonempty (k < 7); KB_PP1: one Preprepare
    struct PhaseSummary {
        uint32_t kinds;                                   // S > 64 only
        M k_pp, k_pr, k_cm, k_ocm, k_rc, k_sync, k_blk;   // S <= 64 only
        M pr_v0, pr_v1, pr_w, cm_v0, cm_v1, cm_w;
        uint32_t pr_h, pr_r, cm_h, cm_r, blk_lo, blk_hi;
        uint64_t pr_cls, cm_cls;              // (height, proposer) class of the digests
        bool u_pr, u_cm, u_blk;               // one view / one digest class / one range
        uint32_t pp_src, pp_h, pp_r, pp_eq;   // the first Preprepare sender and its message
        uint64_t pp_b;
        uint32_t rc_h, rc_r;                  // the first RoundChange sender's view
        bool u_rc;                            // every RoundChange of the segment carries that view
    };
    // how a phase is delivered (segment-uniform): the closed forms read the summary only;
    // the general path reads the published LDS records in each receiver's rotated order
    //   PATH_NONE  nothing in flight in the segment (the event step only);
    //   PATH_PP    one Preprepare and nothing else: every receiver handles that one message;
    //   PATH_RC    RoundChanges of one view and nothing else (deliver_round_change).
    enum : uint32_t { PATH_GENERAL = 0, PATH_BLK = 1, PATH_PC = 2, PATH_NONE = 3, PATH_PP = 4, PATH_RC = 5 };
    BFT_FN uint32_t classify(const PhaseSummary& ps) const {
        if (!P.fast) return PATH_GENERAL;
        if constexpr (S <= 64) {                      // the masks are registers: test them directly
            if ((ps.k_ocm | ps.k_sync).any()) return PATH_GENERAL;
            const bool pc = ps.k_pr.any() || ps.k_cm.any(), blk = ps.k_blk.any(), pp = ps.k_pp.any();
            if (ps.k_rc.any()) return (!pp && !pc && !blk && ps.u_rc) ? PATH_RC : PATH_GENERAL;
            if (pp) return (!pc && !blk && ps.k_pp.popc() == 1u) ? PATH_PP : PATH_GENERAL;
            if (!pc) return blk ? (ps.u_blk ? PATH_BLK : PATH_GENERAL) : PATH_NONE;
            if (!blk && ps.u_pr && ps.u_cm) return PATH_PC;
            return PATH_GENERAL;
        }
        const uint32_t K = ps.kinds;
        if (K & ((1u << KM_OCM) | (1u << KM_SYNC))) return PATH_GENERAL;
        const bool pc = (K & ((1u << KM_PR) | (1u << KM_CM))) != 0, blk = (K & (1u << KM_BLK)) != 0,
                   pp = (K & (1u << KM_PP)) != 0;
        if (K & (1u << KM_RC)) return (!pp && !pc && !blk && ps.u_rc) ? PATH_RC : PATH_GENERAL;
        if (pp) return (!pc && !blk && (K & KB_PP1) != 0) ? PATH_PP : PATH_GENERAL;
        if (!pc) return blk ? (ps.u_blk ? PATH_BLK : PATH_GENERAL) : PATH_NONE;
        if (!blk && ps.u_pr && ps.u_cm) return PATH_PC;
        return PATH_GENERAL;
    }

    BFT_FN M seg_bits(const M& bal) const {
        if constexpr (S >= 64) return bal;
        else return M::from((bal.w[0] >> seg_base) & ((1ull << S) - 1ull));
    }

    // value of lane (seg_base + j) — j is uniform within the segment
    BFT_FN uint32_t from_seg_lane(uint32_t v, uint32_t j) {
        if constexpr (S > 64) return wv.bcast(v, j);
        else if constexpr (S == 64) return wv.readlane(v, j);
        else return wv.shfl(v, seg_base + j);
    }

    // sender mask `k` (KM_*) of the phase: a register of the summary (S <= 64) or the LDS copy (S > 64)
    template <uint32_t k>
    BFT_FN M kmask(const PhaseSummary& ps) const {
        if constexpr (S > 64) {
            M r;
            const uint64_t* src = wv.summary() + k * (uint32_t)NW;
#pragma unroll
            for (int w = 0; w < NW; ++w) r.w[w] = src[w];
            return r;
        } else {
            static_assert(k < KM_COUNT, "mask index");
            return k == KM_PP ? ps.k_pp : k == KM_PR ? ps.k_pr : k == KM_CM ? ps.k_cm : k == KM_OCM ? ps.k_ocm
                 : k == KM_RC ? ps.k_rc : k == KM_SYNC ? ps.k_sync : k == KM_BLK ? ps.k_blk
                 : k == KM_PR_W ? ps.pr_w : k == KM_PR_V0 ? ps.pr_v0 : k == KM_PR_V1 ? ps.pr_v1
                 : k == KM_CM_W ? ps.cm_w : k == KM_CM_V0 ? ps.cm_v0 : ps.cm_v1;
        }
    }
    // every sender with a message of any kind in flight
    BFT_FN M kmask_any(const PhaseSummary& ps) const {
        return kmask<KM_PP>(ps) | kmask<KM_PR>(ps) | kmask<KM_CM>(ps) | kmask<KM_OCM>(ps) | kmask<KM_RC>(ps) |
               kmask<KM_SYNC>(ps) | kmask<KM_BLK>(ps);
    }

    // S > 64 (one instance per workgroup): the same summary with three batched collectives (one barrier
    // each) instead of one barrier per ballot and per leader value: the kinds and digest-variant masks,
    // the leaders' message fields, the uniformity checks
    BFT_FN void summarize_group(PhaseSummary& ps) {
        const uint32_t f = nx.f;
        const bool pp = (f & F_PP) != 0, pr = (f & F_PR) != 0, cm = (f & F_CM) != 0, bk = (f & F_BLK) != 0,
                   rc = (f & F_RC) != 0, prw = (f & F_PR_W) != 0, cmw = (f & F_CM_W) != 0;
        const bool pv1 = blk_var(nx.pr_d) == 1, cv1 = blk_var(nx.cm_d) == 1;
        const bool pred[13] = {pp, pr, cm, (f & F_OCM) != 0, rc, (f & F_SYNC) != 0, bk, (bool)(pr & prw),
                               (bool)(pr & !prw & !pv1), (bool)(pr & !prw & pv1), (bool)(cm & cmw),
                               (bool)(cm & !cmw & !cv1), (bool)(cm & !cmw & cv1)};
        static_assert(KM_PP == 0 && KM_BLK == 6 && KM_CM_V1 == 12, "pred order = KM_* order");
        wv.template ballot_k_store<13>(pred, wv.summary());
        // the first sender of each kind publishes its message fields
        const M kpp = kmask<KM_PP>(ps), kpr = kmask<KM_PR>(ps), kcm = kmask<KM_CM>(ps), kbk = kmask<KM_BLK>(ps),
                krc = kmask<KM_RC>(ps);
        ps.kinds = (kpp.any() ? 1u << KM_PP : 0u) | (kpr.any() ? 1u << KM_PR : 0u) | (kcm.any() ? 1u << KM_CM : 0u) |
                   (kmask<KM_OCM>(ps).any() ? 1u << KM_OCM : 0u) | (krc.any() ? 1u << KM_RC : 0u) |
                   (kmask<KM_SYNC>(ps).any() ? 1u << KM_SYNC : 0u) | (kbk.any() ? 1u << KM_BLK : 0u) |
                   (kpp.popc() == 1u ? KB_PP1 : 0u);
        const uint32_t jpp = kpp.any() ? kpp.ctz_nz() : S, jpr = kpr.any() ? kpr.ctz_nz() : S,
                       jcm = kcm.any() ? kcm.ctz_nz() : S, jbk = kbk.any() ? kbk.ctz_nz() : S,
                       jrc = krc.any() ? krc.ctz_nz() : S;
        const uint64_t pcls = nx.pr_d & BLK_HP_MASK, ccls = nx.cm_d & BLK_HP_MASK;
        const bool lpp = me == jpp, lpr = me == jpr, lcm = me == jcm, lbk = me == jbk, lrc = me == jrc;
        const bool wr[17] = {lpp, lpp, lpp, lpp, lpp, lpr, lpr, lpr, lpr, lcm, lcm, lcm, lcm, lbk, lbk, lrc, lrc};
        const uint32_t val[17] = {nx.pp_h, nx.pp_r, (uint32_t)nx.pp_b, (uint32_t)(nx.pp_b >> 32), f & F_PP_EQ,
                                  nx.pr_h, nx.pr_r, (uint32_t)pcls, (uint32_t)(pcls >> 32),
                                  nx.cm_h, nx.cm_r, (uint32_t)ccls, (uint32_t)(ccls >> 32),
                                  nx.blk_lo, nx.blk_hi, nx.rc_h, nx.rc_r};
        uint32_t g[17];
        wv.template gather_k<17>(wr, val, g);
        const bool any_pp = kpp.any(), any_pr = kpr.any(), any_cm = kcm.any(), any_bk = kbk.any(), any_rc = krc.any();
        ps.pp_src = any_pp ? jpp : 0u;
        ps.pp_h = any_pp ? g[0] : 0u; ps.pp_r = any_pp ? g[1] : 0u;
        ps.pp_b = any_pp ? ((uint64_t)g[2] | ((uint64_t)g[3] << 32)) : 0ull; ps.pp_eq = any_pp ? g[4] : 0u;
        ps.pr_h = any_pr ? g[5] : 0u; ps.pr_r = any_pr ? g[6] : 0u;
        ps.pr_cls = any_pr ? ((uint64_t)g[7] | ((uint64_t)g[8] << 32)) : 0ull;
        ps.cm_h = any_cm ? g[9] : 0u; ps.cm_r = any_cm ? g[10] : 0u;
        ps.cm_cls = any_cm ? ((uint64_t)g[11] | ((uint64_t)g[12] << 32)) : 0ull;
        ps.blk_lo = any_bk ? g[13] : 0u; ps.blk_hi = any_bk ? g[14] : 0u;
        ps.rc_h = any_rc ? g[15] : 0u; ps.rc_r = any_rc ? g[16] : 0u;
        // uniformity against the leaders
        const bool mm[4] = {(bool)(pr & ((nx.pr_h != ps.pr_h) | (nx.pr_r != ps.pr_r) | (pcls != ps.pr_cls))),
                            (bool)(cm & ((nx.cm_h != ps.cm_h) | (nx.cm_r != ps.cm_r) | (ccls != ps.cm_cls))),
                            (bool)(bk & ((nx.blk_lo != ps.blk_lo) | (nx.blk_hi != ps.blk_hi))),
                            (bool)(rc & ((nx.rc_h != ps.rc_h) | (nx.rc_r != ps.rc_r)))};
        M mb[4];
        wv.template ballot_k<4>(mm, mb);
        ps.u_pr = mb[0].none(); ps.u_cm = mb[1].none(); ps.u_blk = mb[2].none(); ps.u_rc = mb[3].none();
    }

    BFT_FN void summarize(PhaseSummary& ps) {
        if constexpr (S > 64) { summarize_group(ps); return; }
        const uint32_t f = nx.f;
        ps.k_pp = seg_bits(ballot((f & F_PP) != 0));
        ps.k_pr = seg_bits(ballot((f & F_PR) != 0));
        ps.k_cm = seg_bits(ballot((f & F_CM) != 0));
        ps.k_ocm = seg_bits(ballot((f & F_OCM) != 0));
        ps.k_rc = seg_bits(ballot((f & F_RC) != 0));
        ps.k_sync = seg_bits(ballot((f & F_SYNC) != 0));
        ps.k_blk = seg_bits(ballot((f & F_BLK) != 0));
        const bool pr = (f & F_PR) != 0, cm = (f & F_CM) != 0, bk = (f & F_BLK) != 0;
        const bool prw = (f & F_PR_W) != 0, cmw = (f & F_CM_W) != 0;
        ps.pr_h = ps.pr_r = ps.cm_h = ps.cm_r = ps.blk_lo = ps.blk_hi = 0;
        ps.pr_cls = ps.cm_cls = 0;
        ps.pr_w = ps.pr_v0 = ps.pr_v1 = ps.cm_w = ps.cm_v0 = ps.cm_v1 = M::zero();
        ps.u_pr = ps.u_cm = ps.u_blk = true;
        // leader of each kind (the first sender of the segment) and uniformity against it
        // (the wave-wide ballots equal the segment masks when the segment is the whole wave)
        const bool pp = (f & F_PP) != 0, rc = (f & F_RC) != 0;
        bool any_pr = S == 64 ? ps.k_pr.any() : ballot(pr).any();
        bool any_cm = S == 64 ? ps.k_cm.any() : ballot(cm).any();
        bool any_bk = S == 64 ? ps.k_blk.any() : ballot(bk).any();
        const bool any_pp = S == 64 ? ps.k_pp.any() : ballot(pp).any();
        const bool any_rc = S == 64 ? ps.k_rc.any() : ballot(rc).any();
        bool mm_pr = false, mm_cm = false, mm_blk = false, mm_rc = false;
        ps.pp_src = ps.pp_h = ps.pp_r = ps.pp_eq = 0; ps.pp_b = 0;
        ps.rc_h = ps.rc_r = 0; ps.u_rc = true;
        if (any_pp) {
            const uint32_t j = ps.k_pp.any() ? ps.k_pp.ctz_nz() : 0u;
            ps.pp_src = j;
            ps.pp_h = from_seg_lane(nx.pp_h, j);
            ps.pp_r = from_seg_lane(nx.pp_r, j);
            ps.pp_b = (uint64_t)from_seg_lane((uint32_t)nx.pp_b, j) | ((uint64_t)from_seg_lane((uint32_t)(nx.pp_b >> 32), j) << 32);
            ps.pp_eq = from_seg_lane(f & F_PP_EQ, j);
        }
        if (any_rc) {
            const uint32_t j = ps.k_rc.any() ? ps.k_rc.ctz_nz() : 0u;
            ps.rc_h = from_seg_lane(nx.rc_h, j);
            ps.rc_r = from_seg_lane(nx.rc_r, j);
            mm_rc = rc & ((nx.rc_h != ps.rc_h) | (nx.rc_r != ps.rc_r));
            ps.u_rc = seg_bits(ballot(mm_rc)).none();
        }
        if (any_pr) {
            uint32_t j = ps.k_pr.any() ? ps.k_pr.ctz_nz() : 0u;
            uint64_t cls = nx.pr_d & BLK_HP_MASK;
            ps.pr_h = from_seg_lane(nx.pr_h, j);
            ps.pr_r = from_seg_lane(nx.pr_r, j);
            ps.pr_cls = (uint64_t)from_seg_lane((uint32_t)cls, j) | ((uint64_t)from_seg_lane((uint32_t)(cls >> 32), j) << 32);
            mm_pr = pr & ((nx.pr_h != ps.pr_h) | (nx.pr_r != ps.pr_r) | (cls != ps.pr_cls));
            ps.pr_w = seg_bits(ballot(pr & prw));
            ps.pr_v0 = seg_bits(ballot(pr & !prw & (blk_var(nx.pr_d) == 0)));
            ps.pr_v1 = seg_bits(ballot(pr & !prw & (blk_var(nx.pr_d) == 1)));
        }
        if (any_cm) {
            uint32_t j = ps.k_cm.any() ? ps.k_cm.ctz_nz() : 0u;
            uint64_t cls = nx.cm_d & BLK_HP_MASK;
            ps.cm_h = from_seg_lane(nx.cm_h, j);
            ps.cm_r = from_seg_lane(nx.cm_r, j);
            ps.cm_cls = (uint64_t)from_seg_lane((uint32_t)cls, j) | ((uint64_t)from_seg_lane((uint32_t)(cls >> 32), j) << 32);
            mm_cm = cm & ((nx.cm_h != ps.cm_h) | (nx.cm_r != ps.cm_r) | (cls != ps.cm_cls));
            ps.cm_w = seg_bits(ballot(cm & cmw));
            ps.cm_v0 = seg_bits(ballot(cm & !cmw & (blk_var(nx.cm_d) == 0)));
            ps.cm_v1 = seg_bits(ballot(cm & !cmw & (blk_var(nx.cm_d) == 1)));
        }
        if (any_bk) {
            uint32_t j = ps.k_blk.any() ? ps.k_blk.ctz_nz() : 0u;
            ps.blk_lo = from_seg_lane(nx.blk_lo, j);
            ps.blk_hi = from_seg_lane(nx.blk_hi, j);
            mm_blk = bk & ((nx.blk_lo != ps.blk_lo) | (nx.blk_hi != ps.blk_hi));
        }
        if (any_pr | any_cm | any_bk) {
            ps.u_pr = seg_bits(ballot(mm_pr)).none();
            ps.u_cm = seg_bits(ballot(mm_cm)).none();
            ps.u_blk = seg_bits(ballot(mm_blk)).none();
        }
    }

    // rotate a sender mask into this receiver's delivery order (position 0 = first delivered)
    BFT_FN M rot(const M& m, uint32_t off) const {
        if (off == 0) return m;
        uint32_t n = nval();
        if constexpr (NW == 1) {                     // 0 < off < n <= 64: both shifts in [1, 63]
            uint64_t nm = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
            return M::from(((m.w[0] >> off) | (m.w[0] << (n - off))) & nm);
        } else {
            return (m.shr(off) | m.shl(n - off)) & M::low(n);
        }
    }
    BFT_FN M unrot(const M& m, uint32_t off) const { return off ? rot(m, nval() - off) : m; }   // inverse of rot
    BFT_FN static M low(uint32_t k) { return M::low(k); }
    // smallest position p in [0,n) with popcount(base | a & low(p+1) | b & low(p)) > q, else n
    BFT_FN uint32_t first_over(const M& base, const M& a, const M& b, uint32_t q) const {
        uint32_t n = nval();
        if ((base | a | (b & low(n - 1))).popc() <= q) return n;
        uint32_t lo = 0, hi = n - 1;                 // answer in [lo, hi]
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if ((base | (a & low(mid + 1)) | (b & low(mid))).popc() > q) hi = mid;
            else lo = mid + 1;
        }
        return lo;
    }
    BFT_FN static uint32_t first_at_or_after(const M& m, uint32_t p) {
        M x = m & ~low(p);
        return x.any() ? x.ctz() : 64u * NW;
    }

    // digests of the class `cls` that match `target` (wildcards match both variants)
    BFT_FN static M class_match(uint64_t cls, const M& v0, const M& v1, const M& w, uint64_t target) {
        if (!blk_valid(target) || ((cls ^ target) & BLK_HP_MASK) != 0) return M::zero();
        return w | (blk_var(target) ? v1 : v0);
    }

    // A phase that carries only Prepares and Commits, each kind with one view and one digest
    // class: the sequential handlers of prepare.rs:48-66 and commit.rs:63-82, evaluated in this
    // receiver's delivery order with prefix masks instead of one message at a time.
    BFT_FN void deliver_prepare_commit(const PhaseSummary& ps, const M& mk, uint32_t off) {
        M PRacc = M::zero(), CMacc = M::zero();
        M prd = mk & kmask<KM_PR>(ps), cmd = mk & kmask<KM_CM>(ps);
        if (prd.any()) {
            int res = check_message(2, ps.pr_h);
            if (res != 0) { if (res == 2) note_future_block(ps.pr_h); }
            else if (ps.pr_h == h && ps.pr_r == r) PRacc = prd;
        }
        if (cmd.any()) {
            int res = check_message(3, ps.cm_h);
            if (res != 0) { if (res == 2) note_future_block(ps.cm_h); }
            else if (ps.cm_h == h && ps.cm_r == r) CMacc = cmd & class_match(ps.cm_cls, kmask<KM_CM_V0>(ps), kmask<KM_CM_V1>(ps), kmask<KM_CM_W>(ps), pp);
        }
        if (PRacc.none() && CMacc.none()) return;
        const uint32_t q = qval();
        uint32_t n = nval();
        M PR = rot(PRacc, off), CM = rot(CMacc, off);
        M U0 = rot(prep | comm, off), C0 = rot(comm, off);
        const uint32_t lastPR = PR.hibit();
        const uint32_t lastCM = CM.hibit();
        // prepare triggers (prepare.rs:54-63). B fires at some prepare iff it fires at the last
        // one (|prep ∪ commit| only grows); commits of the last prepare's sender come after it.
        const bool trigB = PR.any() & ((U0 | PR | (CM & low(lastPR))).popc() > q);
        M lm = M::zero();
        if (blk_valid(lock) && PR.any()) lm = rot(PRacc & class_match(ps.pr_cls, kmask<KM_PR_V0>(ps), kmask<KM_PR_V1>(ps), kmask<KM_PR_W>(ps), lock), off);
        const bool trig = trigB | lm.any();
        // commit quorum events (commit.rs:75-80) exist iff the final count is over q
        const bool cexists = CM.any() & ((C0 | CM).popc() > q);
        uint32_t lastT = 0, t1 = 64u * NW;
        if (trig) {
            if (lm.any()) t1 = lm.ctz_nz();
            if (trigB) {
                lastT = lastPR;                                 // every prepare from tB on
            } else {
                // lock-match triggers only: the first one locks pp, later ones match pp
                M mpp = rot(PRacc & class_match(ps.pr_cls, kmask<KM_PR_V0>(ps), kmask<KM_PR_V1>(ps), kmask<KM_PR_W>(ps), pp), off);
                M T = (mpp & ~low(t1)) | M::bit(t1);
                lastT = T.hibit();
            }
        }
        const uint32_t s0 = st;
        bool fires;          // some commit event runs Core::commit
        uint32_t fin;
        if (trig) {
            fin = (cexists & (lastCM >= lastT)) ? ST_COMMITTED : ST_PREPARED;
            if (s0 < ST_COMMITTED) {
                fires = cexists;
            } else {
                // already committed: a re-commit needs a commit event after the first trigger
                if (trigB) {
                    uint32_t pstar = first_over(U0, PR, CM, q);
                    uint32_t tB = first_at_or_after(PR, pstar);
                    if (tB < t1) t1 = tB;
                }
                fires = cexists & (lastCM >= t1);
            }
        } else {
            fires = cexists & (s0 < ST_COMMITTED);
            fin = fires ? ST_COMMITTED : s0;
        }
        (void)n;
        prep |= PRacc;
        comm |= CMacc;
        if (trig) { lock_hash(); send_commit(); }
        if (fires) { lock_hash(); st = ST_COMMITTED; in_pc = true; chain_insert_core(pp); in_pc = false; }
        st = fin;
    }

    // A phase of RoundChanges that all carry one view (h, R) and nothing else: round_change.rs:65-98 for
    // every delivered sender in this receiver's rotated order, with the RoundChangeSet entry of R updated
    // once. The order matters at one point only, the quorum event (count > q while waiting with r < R:
    // send_round_change + start_new_round, which clears the set; the later senders then fill the fresh
    // set of R); it is found as a prefix count, as the prepare quorum of deliver_prepare_commit.
    BFT_FN void deliver_round_change(const PhaseSummary& ps, const M& mk, uint32_t off) {
        if (core_dead) return;                        // deliver_from: a panicked Core handles nothing
        const M D = mk & kmask<KM_RC>(ps);
        if (D.none()) return;
        const uint32_t R = ps.rc_r;
        const int res = check_message(MT_ROUND_CHANGE, ps.rc_h);
        if (res != 0) { if (res == CM_FUTURE_BLOCK) note_future_block(ps.rc_h); return; }
        const uint32_t k = D.popc();
        if (r > R && R > 0) {                         // every message: send_round_change(R) (round_change.rs:74-77)
            if (rc_last_tick == tick) { new_round_change_timer(); return; }   // all suppressed by the limiter
            rc_last_tick = tick;                      // the first one goes out (r > R: no catchup_round)
            out_round_change(h, R);
            if (k >= 2u) new_round_change_timer();   // the later ones are suppressed: timer re-armed
            return;
        }
        const int pos = rcs_slot(R);
        if (pos < 0) return;                          // table full: every rcs_add returns 0 (flagged)
        const M set = rc_set_at((uint32_t)pos);
        const uint32_t n = nval(), q = qval();
        const M Dr = rot(D, off);
        uint32_t pe = 64u * NW;                       // position of the quorum event, if any
        if (wait && r < R) {
            const uint32_t p0 = first_over(rot(set, off), Dr, M::zero(), q);
            if (p0 < n) pe = first_at_or_after(Dr, p0);
        }
        if (pe >= n) { rc_set_store((uint32_t)pos, set | D); return; }
        const M later = unrot(Dr & ~low(pe + 1u), off);   // senders after the event
        send_round_change(R);
        if (last > h) {                               // start_new_round returns at once (core.rs:476-479):
            rc_set_store((uint32_t)pos, set | D);     // every later sender repeats the event, suppressed
            if (later.any()) new_round_change_timer();   // by the limiter
            return;
        }
        rc_set_store((uint32_t)pos, set | (D & ~later));
        start_new_round(R);                           // clears the RoundChangeSet
        if (core_dead || later.none()) return;
        const int p2 = rcs_slot(R);                   // r == R, wait == false: the later ones are only added
        if (p2 >= 0) rc_set_store((uint32_t)p2, later);
    }

    // ---------------------------------------------------------------- the canonical view, composed
    // A lone Preprepare in flight (PATH_PP) of view (vh, vr) from its proposer, no link drops and no Byzantine
    // validators, and every running validator waiting for it: AcceptRequest at (vh, vr), unlocked, its chain
    // tip vh - 1, no seal about to mine in this phase's event step, and no outbound-cache entry for this
    // subject's Prepare or Commit. Then this phase and the next two have one outcome (the same steps the
    // closed forms take one phase at a time): every running validator accepts (preprepare.rs:87-106) and
    // sends its Prepare; all Prepares cross the quorum (prepare.rs:59-63): lock, Prepared, Commit out; all
    // Commits cross it (commit.rs:63-82): Committed, Core::commit → insert_block (chain.rs:45-71). The Prepare
    // and Commit phases' event steps have nothing queued. One instance per wave or workgroup (the segments of a
    // wave share the phase index), not in the opt-in modes (they log or re-deliver every message: MODE_EXT).
    // Segment-uniform; every lane reaches the ballots.
    // the running validators of an active segment (Sim(): a validator below N that is not silent), from the
    // launch parameters: the senders of every Prepare and Commit of a canonical view
    BFT_FN M running_set() const {
        M m = M::low(nval());
        for (int k = 0; k < NW; ++k) m.w[k] &= ~P.silent_mask[k];
        return m;
    }
    BFT_FN bool canonical_pp(const PhaseSummary& ps, uint32_t path, uint32_t p, bool act) {
        // workgroup segments, and the resume kernel after a FAST hand-over; the S = 64 full kernel (N = 33..63,
        // bftsim_set_fast(h, 0)) keeps its registers (the step's code costs it 140 B/lane of scratch)
        if constexpr (!(S > 64 || MODE == MODE_RESUME)) return false;
        else {
            if ((path != PATH_PP) | (ps.pp_eq != 0u) | (P.thr16 != 0u) | (P.byz_count != 0u) | frozen |
                (p + 2u >= P.phase_cap))
                return false;
            const uint32_t vh = ps.pp_h, vr = ps.pp_r, d32 = blk_d32(ps.pp_b);
            const uint32_t* c1 = cache_p(3);                  // Prepare {h, r, d32}
            const uint32_t* c2 = cache_p(6);                  // Commit
            const bool hit1 = (c1[2u * LY::L] == d32) & (c1[0] == vh) & (c1[LY::L] == vr);
            const bool hit2 = (c2[2u * LY::L] == d32) & (c2[0] == vh) & (c2[LY::L] == vr);
            const bool mines = (wake_tick < 0) & (miner_queue != 0u) & (miner_queue >= mint_height);
            const bool ok = !core_dead & (h == vh) & (r == vr) & (st == ST_ACCEPT_REQUEST) & !blk_valid(lock) &
                            (proposer == ps.pp_src) & (last + 1u == vh) & (blk_h(ps.pp_b) == vh) & !mines & !hit1 & !hit2;
            const M bad = ballot(act & !ok);
            return bad.none() && running_set().popc() > qval();
        }
    }
    BFT_FN void apply_canonical_pp(const PhaseSummary& ps) {
        const uint32_t vh = ps.pp_h, vr = ps.pp_r, d32 = blk_d32(ps.pp_b);
        uint32_t* c1 = cache_p(3);
        uint32_t* c2 = cache_p(6);
        c1[0] = vh; c1[LY::L] = vr; c1[2u * LY::L] = d32;     // send_prepare (the PP phase)
        c2[0] = vh; c2[LY::L] = vr; c2[2u * LY::L] = d32;     // send_commit (the Prepare phase)
        pp = ps.pp_b;
        const M voters = running_set();
        prep = voters;                                        // every running validator's Prepare
        comm = voters;                                        // and Commit
        lock_hash();
        st = ST_COMMITTED;                                    // the Commit phase: Core::commit
        in_pc = true;
        chain_insert_core(pp);
        in_pc = false;
    }

    BFT_FN void deliver_phase(const PhaseSummary& ps, uint32_t path, const M& mk, uint32_t off) {
        if (path == PATH_NONE) return;
        if (path == PATH_PP) {                        // one Preprepare: its handler at every receiver
            if (!core_dead && mk.get(ps.pp_src)) handle_preprepare(ps.pp_src, ps.pp_h, ps.pp_r, ps.pp_b, ps.pp_eq != 0);
            BFT_STAMP(12);
            return;
        }
        if (path == PATH_RC) {
            deliver_round_change(ps, mk, off);
            BFT_STAMP(13);
            return;
        }
        if (path == PATH_BLK) {                       // block gossip with one range
            if ((mk & kmask<KM_BLK>(ps) & ~M::bit(me)).any()) handle_blocks(ps.blk_lo, ps.blk_hi);
            BFT_STAMP(8);
            return;
        }
        if (path == PATH_PC) {
            if (!core_dead) deliver_prepare_commit(ps, mk, off);
            BFT_STAMP(9);
            return;
        }
        // general path: every delivered non-empty sender, in rotated order, one at a time
        if (EXT && P.backlog_replay) replay_backlog();   // the stored messages first (SPEC.md §10)
        M any = kmask_any(ps);
        M c = rot(mk & any, off);
        while (c.any()) {
            uint32_t pos = c.ctz_nz();
            c.clear_lowest();
            uint32_t s = pos + off;
            if (s >= nval()) s -= nval();
            deliver_from(s);
        }
        BFT_STAMP(10);
    }

    // ---------------------------------------------------------------- resume (the FAST kernel's hand-over)
    // persistent per-lane and segment state, word by word (lane g's SAVE_WORDS words contiguous):
    // BFT_STATE_32, BFT_STATE_64, prep, comm, the 12 cache words, the bool bits (byz, core_dead,
    // wait, frozen, seg_done), tick, phase; words SAVE_COLD.. hold the old-Commit / RoundChange / Sync
    // outbox fields. Written by bft_fast64.h Fast64::save_state.
#define BFT_STATE_32(X) X(h) X(r) X(st) X(n_rcs) X(proposer) X(last) X(last_seed) X(last_T) X(timer_tick) \
    X(rc_last_tick) X(wake_tick) X(mint_height) X(miner_queue) X(sync_pending) X(lane_flags) X(canon_h)       \
    X(done_tick) X(seg_flags) X(canon_tip_seed) X(canon_tick) X(nx.f) X(nx.pp_h) X(nx.pp_r) X(nx.pr_h)       \
    X(nx.pr_r) X(nx.cm_h) X(nx.cm_r) X(nx.blk_lo) X(nx.blk_hi)
#define BFT_STATE_64(X) X(lock) X(pp) X(pend) X(cand) X(canon_tip) X(views_acc) X(nx.pp_b) X(nx.pr_d)       \
    X(nx.cm_d)
    BFT_FN void load_state(uint32_t& p) {
        const uint32_t* sv = P.save + ((uint64_t)inst_local * LY::L + lane) * SAVE_WORDS;
        uint32_t k = 0;
#define save_p(k) (sv + (k))
#define BFT_LD32(f) f = (decltype(f))*save_p(k++);
#define BFT_LD64(f) { uint64_t lo_ = *save_p(k++); uint64_t hi_ = *save_p(k++); f = lo_ | (hi_ << 32); }
        BFT_STATE_32(BFT_LD32)
        BFT_STATE_64(BFT_LD64)
        for (int j = 0; j < NW; ++j) { BFT_LD64(prep.w[j]) BFT_LD64(comm.w[j]) }
        for (uint32_t c = 0; c < 12; ++c) *cache_p(c) = *save_p(k++);
        const uint32_t b = *save_p(k++);
        byz = (b & 1u) != 0; core_dead = (b & 2u) != 0; wait = (b & 4u) != 0; frozen = (b & 8u) != 0;
        seg_done = (b & 16u) != 0;
        tick = (int32_t)*save_p(k++);
        p = *save_p(k++);
        nx.ocm_h = sv[SAVE_COLD + 0]; nx.ocm_r = sv[SAVE_COLD + 1];
        nx.ocm_d = (uint64_t)sv[SAVE_COLD + 2] | ((uint64_t)sv[SAVE_COLD + 3] << 32);
        nx.rc_h = sv[SAVE_COLD + 4]; nx.rc_r = sv[SAVE_COLD + 5]; nx.sync_h = sv[SAVE_COLD + 6];
#undef BFT_LD32
#undef BFT_LD64
#undef save_p
    }

    // ---------------------------------------------------------------- the run
    BFT_FN void run() {
#ifdef BFT_STAMPS
        for (int k = 0; k < NSTAMP; ++k) st_acc[k] = 0;
        st_t = wv.clock();
#endif
        // resume mode (S == 64): only instances a FAST launch handed over, from their saved phase
        bool resuming = false;
        uint32_t p0 = 0;
        int32_t tick0 = 0;
        if constexpr (RESUME) {
            {
                if (seg_done || P.resume_flags[inst_local] == 0) return;    // wave-uniform
                load_state(p0);
                tick0 = tick;
                resuming = true;
            }
        }
        if (!resuming && P.byz_count > 0) init_byzantine();
        for (uint32_t b = lane; b < HIST_BINS; b += LY::L) *hist_slot(b) = 0;
        if constexpr (SEG_HASH) if (me == 0) *(uint32_t*)(lds + LY::TIPC_OFF + (lane / S) * LY::TIPC_BYTES) = ~0u;
        sync();
        for (tick = tick0; tick < (int32_t)P.max_ticks; ++tick) {
            if (ballot(!seg_done).none()) break;
            bool act = running & !seg_done & !frozen;
            off_tick = offset_tick_part(off_inst, (uint32_t)tick);
            BFT_STAMP(7);
            if (act && !resuming) t_step();
            if (EXT && P.backlog_replay && !resuming) resolve_commits();   // replayed commits of the T-step
            BFT_STAMP(0);
            const uint32_t pstart = resuming ? p0 : 0u;
            resuming = false;
            for (uint32_t p = pstart;; ++p) {
                bool pend_l = act & !frozen & pending_local();
                M bal = ballot(pend_l);
                if constexpr (SEG_HASH) phase_hashes(bal.none() || p >= P.phase_cap);
                if (bal.none()) break;
                bool seg_pending = (bal & seg_mask).any();
                if (EXT && P.mlog) crypto_log(act && !frozen, p);   // real-crypto mode (SPEC.md §11)
                if (p >= P.phase_cap) {
                    // messages still in flight are dropped (SPEC.md §2)
                    M inflight = ballot(act && nx.f != 0);
                    if ((inflight & seg_mask).any() && !seg_done) seg_flags |= FLAG_PHASE_CAP;
                    outbox_clear(nx);
                    break;
                }
                // segment-wide summary of what is in flight (SPEC.md §2 kinds), before publish
                BFT_STAMP(7);
                PhaseSummary ps;
                summarize(ps);
                BFT_STAMP(1);
                const uint32_t path = classify(ps);
#ifdef BFT_PHASE_CENSUS
                BFT_PHASE_CENSUS(ps, path, me);               // test-only (tests/emu): phase kinds census
#endif
#ifdef BFT_STAMPS
                st_acc[6] += 1;                               // phases (a count, not cycles)
                st_acc[11] += path == PATH_GENERAL ? 1 : 0;   // general-path phases
                st_acc[14] += path == PATH_RC ? 1 : 0;        // round-change phases
                st_acc[15] += path == PATH_NONE ? 1 : 0;      // phases with nothing in flight
#endif
                // records go to LDS only if some segment of the wave takes the general path
                const bool pub = ballot(path == PATH_GENERAL).any();
                if (pub) { publish(); sync(); }
                else outbox_clear(nx);
                BFT_STAMP(2);
                const bool canon = canonical_pp(ps, path, p, act);
                if (canon) {                                  // this phase and the next two, applied
                    if (act) { miner_step(); apply_canonical_pp(ps); }
                } else if (act & seg_pending) {
                    miner_step();                             // event step
                    // the draws of the senders in flight only (a Preprepare phase: one block of 8)
                    const M present = path == PATH_PP ? M::bit(ps.pp_src)
                                    : kmask_any(ps);
                    M mk = path == PATH_NONE ? M::zero()
                                             : deliver_mask<NW, (S >= 64)>(P.seed, nval(), P.thr16, inst, (uint32_t)tick, p,
                                                                             me, present);
                    uint32_t off = (path == PATH_GENERAL || path == PATH_PC || path == PATH_RC)
                                       ? offset_from_parts(P.seed, nval(), off_tick, p, me) : 0u;
                    BFT_STAMP(5);
                    deliver_phase(ps, path, mk, off);
                }
                if (canon) p += 2u;                           // the Prepare and Commit phases, applied
                if (pub) sync();                              // records read before the next publish
                BFT_STAMP(3);
                if constexpr (WAVE_HASH) resolve_deferred_hash();
                const uint32_t xc = resolve_commits();
                BFT_STAMP(4);
                if (frozen) act = false;
                // The block-gossip phase after a commit, fused (as bft_fast64.h does): when a Prepare/Commit phase
                // ends with every committer at height xc, the next phase carries their Blocks ranges [.., xc]. If
                // nothing else is in flight and every running validator already holds xc, handle_blocks is
                // ChainError::Exists for all of them (core.rs:75-82), whatever the delivery masks, and that phase
                // reduces to its event step (same phase index, same miner step). One instance per wave or
                // workgroup only (segments of a wave share the phase loop), and not in the opt-in modes (the
                // crypto log records every broadcast, replay mode re-delivers at every phase).
                if constexpr (S >= 64 && MODE != MODE_EXT) {
                    if ((xc != 0u) & ((path == PATH_PC) | canon) & !frozen & (p + 1u < P.phase_cap)) {
                        const M pb = ballot(act & pending_local());
                        const bool nop = !running | seg_done |
                                         ((((nx.f & ~F_BLK) == 0u) & (((nx.f & F_BLK) == 0u) | (nx.blk_hi == xc))) & (last >= xc));
                        if (pb.any() && ballot(!nop).none()) {
                            ++p;
                            outbox_clear(nx);
                            if (act) miner_step();
                        }
                    }
                }
            }
            if (P.trace && is_val && !seg_done && (uint32_t)tick < P.trace_ticks)
                P.trace[((uint64_t)inst_local * P.trace_ticks + (uint32_t)tick) * nval() + me] = state_digest();
            if (!seg_done && (frozen || canon_h >= P.heights)) { seg_done = true; done_tick = (uint32_t)tick + 1; }
        }
#ifdef BFT_STAMPS
        BFT_STAMP(7);
        if (lane == 0 && P.stamps)
            for (int k = 0; k < NSTAMP; ++k) P.stamps[(uint64_t)(S >= 64 ? inst_local : inst_local / (64u / S)) * NSTAMP + k] = st_acc[k];
#endif
        // outputs (segment lane 0); instance-rounds = sum of (round + 1) over heights <= H
        uint32_t lf = seg_or(lane_flags);
        sync();
        if (P.hist) {                                  // this wave's histogram → the launch totals
            for (uint32_t b = lane; b < HIST_BINS; b += LY::L) {
                const uint32_t v = *hist_slot(b);
                if (v != 0) wv.gadd64(P.hist + b, v);
            }
        }
        if (me == 0 && inst_local < P.n_instances) {
            uint32_t flags = lf | seg_flags;
            if (!frozen && canon_h < P.heights) flags |= FLAG_TIMEOUT;
            uint32_t chh = canon_h < P.heights ? canon_h : P.heights;
            uint64_t views = views_acc;
            P.committed_height[inst_local] = chh;
            P.flags[inst_local] = flags;
            P.ticks[inst_local] = done_tick;
            P.views[inst_local] = views;
            if (EXT && P.mlog) P.mlog_n[inst_local] = mlog_cnt;
        }
    }
};

}  // namespace bft
