// bft_fast64.h — the N = 64 consensus kernel body of the benchmark workload (cfg3), one 64-lane
// wavefront per instance, lane = validator (= one reference `Core`, core.rs:119-140).
//
// It runs the same state machine as the general body (bft_wave.h `Sim`), restricted to the phases
// whose delivery has a closed form — a single Preprepare, Prepare/Commit phases with one view and one
// digest class per kind, block gossip with one range, and message-less event phases. Any other phase
// (RoundChange, Sync, old-block Commits, mixed kinds) hands the instance over to the full kernel
// (`Sim<..., MODE_RESUME>`), which continues from that phase: the hand-over area holds the full
// kernel's state layout, so results are bit-identical by construction (tested by the emulator and
// GPU parity suites against the oracle).
//
// Why a separate body: restricted to these phases, most of a validator's state is implied —
// * the round is 0 (only start_new_round, reached from a RoundChange, changes it), so the proposer of
//   every view is validator 0 (seed ≡ 0 for big-endian U128 seeds and N a power of two, SPEC.md §1);
// * every Preprepare / Prepare / Commit a validator sends carries its current view (h, 0), a Prepare
//   or Commit the digest `pp`, a Preprepare its own candidate: an outbox is flags + the candidate's
//   time tick + one block range;
// * `lock` is either None or equal to `pp` (lock_hash copies pp; pp changes only while unlocked or to
//   the locked block itself), `pend` is None or (h, me, 0, T);
// * a Core commit is `pp` at round 0: one flag bit.
// That leaves ~25 live 32-bit values per lane (the general body keeps ~90), so the kernel runs without
// spills at 6 waves per SIMD (80 VGPRs), and the phase logic is short, mostly branch-free selects.
//
// SEEDED = true: the proposer depends on the previous block hash (little-endian U128 seeds,
// bftsim.h BFTSIM_SEED_LE): proposer = seed(hash of the chain tip) mod 64 at round 0 (validator.rs:33-48,
// 74-77), the same for every validator whose tip is the same block. Each canonical height is hashed by
// the whole wave when it is recorded (bft_kwave.h), before any validator can start the next height, and
// its row carries the seed; a validator's proposer is kept per lane.
#pragma once
#include "bft_common.h"
#include "bft_kwave.h"
#include "bft_wave.h"

namespace bft {

// LDS per wave (bytes)
struct F64Layout {
    static constexpr uint32_t CACHE_OFF = 0;                   // outbound cache, SoA [word][lane]: per kind {h, d32}
    static constexpr uint32_t CACHE_WORDS = 8;                 // 4 kinds (PP, PR, CM, old CM) x 2
    static constexpr uint32_t RING_OFF = CACHE_OFF + CACHE_WORDS * 64 * 4;   // 64 canonical rows x 16 B
    static constexpr uint32_t LAT_OFF = RING_OFF + 64 * 16;    // commit-latency histogram (65 words)
    // cold per-lane state (SoA [word][lane]): sync_pending, rc_last_tick, pend's time tick, (unused),
    // the lane's result flags — off the registers of the hot loop
    static constexpr uint32_t LANE_OFF = LAT_OFF + 65 * 4 + 4;
    static constexpr uint32_t W_SYNC = 0, W_RCLT = 1, W_PENDT = 2, W_PPT = 3, W_LFL = 4, LANE_WORDS = 5;
    static constexpr uint32_t BYTES = LANE_OFF + LANE_WORDS * 64 * 4;
    static constexpr uint32_t KW_OFF = BYTES;                  // SEEDED: the header buffer of the wave hash
    static constexpr uint32_t BYTES_SEEDED = KW_OFF + KW_BUF_BYTES;
    static_assert(KW_OFF % 8 == 0, "8-aligned header buffer");
};
constexpr uint32_t lds_bytes_fast64(bool seeded = false) { return seeded ? F64Layout::BYTES_SEEDED : F64Layout::BYTES; }

// LOSSY = false: the schedule has no link drops and no proposer crashes (thr16 == 0, crash_on == 0,
// e.g. cfg3), so every delivery mask is all ones at compile time
template <class W, bool LOSSY = true, bool SEEDED = false>
struct Fast64 {
    static constexpr uint32_t N = 64, Q = 42;   // floor(2N/3) (validator.rs:149-154)
    // lane flag bits
    static constexpr uint32_t L_ST = 7u, L_WAIT = 8u, L_LOCK = 16u, L_BYZ = 32u, L_RUN = 64u, L_DEAD = 128u,
                              L_PENDV = 256u, L_CMT = 512u, L_PROP = 1024u,   // L_PROP: proposer is set (= 0)
                              L_OBX = 2048u,   // FLAG_OUTBOX of this lane (a second message of a kind in one phase)
                              L_SYNCP = 4096u; // W_SYNC (the delayed sync check's height) is nonzero
    enum : uint32_t { P_GENERAL = 0, P_BLK = 1, P_PC = 2, P_PP = 3, P_NONE = 4, P_CANON = 5 };

    const Params& P;
    uint8_t* lds;
    W wv;
    // identity
    uint32_t me;                       // lane = validator index
    uint32_t inst_local, inst, off_inst, off_tick;
    // wave-uniform
    bool seg_done, frozen;
    uint32_t canon_h, canon_tick, done_tick, seg_flags, flushed;
    uint64_t canon_tip, views_acc;
    uint64_t byz_mask;                 // Byzantine validators of this instance (SPEC.md §6)
    uint32_t pp_T_out;                 // time tick of the proposer's outbox Preprepare
    int32_t tick;
    // SEEDED: the canonical tip's hash (lane l < 8 holds word l) and seed; each lane's round-0 proposer
    uint32_t tip_w, canon_seed, prop_l;
    // per lane (Core + RoundState + chain tip + miner + timers + outbox)
    uint32_t fl;                       // L_* bits; state in bits 0..2
    uint32_t h;
    uint64_t pp, prep, comm;            // MessageManage sender sets (protocol/mod.rs:176-209)
    uint32_t cand_T, last;
    int32_t last_T, timer_tick, wake_tick;
    uint32_t mint_height, miner_queue;
    uint32_t nxf, nx_blo, nx_bhi;
#ifdef BFT_STAMPS
    uint64_t st_acc[NSTAMP];
    uint64_t st_t;
#define F64_STAMP(k) do { uint64_t t_ = wv.clock(); st_acc[k] += t_ - st_t; st_t = t_; } while (0)
#define F64_COUNT(k) do { st_acc[k] += 1; } while (0)
#else
#define F64_STAMP(k) do { } while (0)
#define F64_COUNT(k) do { } while (0)
#endif

    BFT_FN Fast64(const Params& p, uint8_t* l, uint32_t wave_global) : P(p), lds(l) {
        wv.init(nullptr);
        me = wv.lane();
        inst_local = wave_global;
        inst = p.first_instance + inst_local;
        const bool inst_ok = inst_local < p.n_instances;
        const bool running = inst_ok && !((p.silent_mask[0] >> me) & 1ull);
        fl = ST_ACCEPT_REQUEST | (running ? L_RUN : 0u);
        seg_done = !inst_ok;
        frozen = false;
        canon_h = 0; canon_tick = 0; done_tick = p.max_ticks; seg_flags = 0; flushed = 0;
        canon_tip = 0; views_acc = 0; byz_mask = 0; pp_T_out = 0;
        tick = 0;
        h = 0; pp = BLK_NONE; prep = comm = 0;
        cand_T = 0; last = 0;
        last_T = -1; timer_tick = -1; wake_tick = -1;
        mint_height = 0; miner_queue = 0;
        for (uint32_t k = 0; k < F64Layout::LANE_WORDS; ++k) *lane_p(k) = 0;
        nxf = 0; nx_blo = nx_bhi = 0;
        for (uint32_t k = 0; k < F64Layout::CACHE_WORDS; ++k) *cache_p(k) = 0;
        off_inst = offset_inst_part(p.seed, inst);
        off_tick = 0;
        canon_seed = p.genesis_seed;
        hashed_h = 0;
        spec_ok = SEEDED && p.spec != nullptr;
        prop_l = 0;
        tip_w = 0;
        if (SEEDED && me < 8u)
            tip_w = (uint32_t)p.genesis_hash[4 * me] | ((uint32_t)p.genesis_hash[4 * me + 1] << 8) |
                    ((uint32_t)p.genesis_hash[4 * me + 2] << 16) | ((uint32_t)p.genesis_hash[4 * me + 3] << 24);
    }

    // ------------------------------------------------------------------ small helpers
    // the launch seed as an opaque scalar (bft_common.h BFT_OPAQUE_SGPR): keeps Philox key schedules
    // from being hoisted out of the loops
    BFT_FN uint64_t seed() const {
        uint32_t lo = (uint32_t)P.seed, hi = (uint32_t)(P.seed >> 32);
        BFT_OPAQUE_SGPR(lo);
        BFT_OPAQUE_SGPR(hi);
        return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    BFT_FN uint32_t* lane_p(uint32_t w) const { return (uint32_t*)(lds + F64Layout::LANE_OFF) + w * 64u + me; }
    BFT_FN uint32_t lane_flags() const { return *lane_p(F64Layout::W_LFL) | (has(L_OBX) ? FLAG_OUTBOX : 0u); }
    BFT_FN uint32_t proposer() const { return has(L_PROP) ? (SEEDED ? prop_l : 0u) : 0xffffffffu; }
    // seed of canonical block x as recorded (SEEDED; row word 3, the genesis seed at 0)
    BFT_FN uint32_t seed_at(uint32_t x) {
        if (x == 0u) return P.genesis_seed;
        if (x == canon_h) return canon_seed;
        return row_word(x, 3);
    }
    BFT_FN uint32_t st() const { return fl & L_ST; }
    BFT_FN void set_st(uint32_t s) { fl = (fl & ~L_ST) | s; }
    BFT_FN bool has(uint32_t b) const { return (fl & b) != 0; }
    BFT_FN uint32_t uni(uint32_t v) const { return wv.uni(v); }
    BFT_FN uint64_t ballot(bool p) { return wv.ballot(p); }
    BFT_FN uint32_t rl(uint32_t v, uint32_t j) { return wv.readlane(v, j); }
    BFT_FN uint64_t rl64(uint64_t v, uint32_t j) {
        return (uint64_t)wv.readlane((uint32_t)v, j) | ((uint64_t)wv.readlane((uint32_t)(v >> 32), j) << 32);
    }
    BFT_FN static uint64_t rotr(uint64_t m, uint32_t off) { return off ? ((m >> off) | (m << (64u - off))) : m; }
    BFT_FN static uint64_t low(uint32_t k) { return k >= 64u ? ~0ull : ((1ull << k) - 1ull); }
    // blk_eq without short-circuit branches
    BFT_FN static bool beq(uint64_t a, uint64_t b) { return ((a & b & BLK_VALID) != 0) & (((a ^ b) & BLK_ID_MASK) == 0); }
    BFT_FN static uint32_t popc(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }
    BFT_FN static uint32_t hibit(uint64_t m) { return m ? 63u - (uint32_t)__builtin_clzll(m) : 0u; }
    BFT_FN static uint32_t ctz64(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }
    BFT_FN static uint32_t ff1(uint64_t m) { return (uint32_t)__builtin_ctzll(m | (1ull << 63)); }  // 63 for 0

    // ------------------------------------------------------------------ outbound cache (backend.rs:141-148)
    // per kind the last subject sent: {height, 32-bit block id}; the round is always 0 here
    BFT_FN uint32_t* cache_p(uint32_t w) const { return (uint32_t*)(lds + F64Layout::CACHE_OFF) + w * 64u + me; }
    BFT_FN bool cache_hit(uint32_t kind, uint32_t vh, uint64_t d) {
        const uint32_t d32 = blk_d32(d);
        uint32_t* c = cache_p(2u * kind);
        const uint32_t sd = c[64];
        if (sd != 0 && c[0] == vh && sd == d32) return true;
        c[0] = vh;
        c[64] = d32;
        return false;
    }
    // the hand-over area (P.save, the full kernel's layout): cold outbox words go there at once
    BFT_FN uint32_t* save_p() const { return P.save + ((uint64_t)inst_local * 64u + me) * SAVE_WORDS; }

    BFT_FN uint64_t cand() const { return blk_make(mint_height, me, 0, cand_T); }

    // Predicated style: a handler takes a per-lane predicate `c` and updates registers with selects, so
    // the hot paths have no divergent regions that write registers (LLVM's structurizer copies every
    // live value at each nested divergent branch). Only memory stores sit under divergent `if`s, and
    // the rare paths (round changes, sync requests, old Preprepares) run behind uniform ballots.
    // Lane predicates are combined with the non-short-circuit `&` / `|`: `&&` / `||` on per-lane values
    // become nested exec-mask branches (three SALU instructions each), and the one scalar unit of a CU
    // is what bounds this kernel (profiles/r02: +100 SALU per phase cost 2.1x what +100 VALU did).

    // a message of `kind` (view (vh, 0), digest d) through the outbound cache into the outbox
    BFT_FN bool send_kind(bool c, uint32_t kind, uint32_t vh, uint64_t d, uint32_t flag, uint32_t wflag) {
        const uint32_t d32 = blk_d32(d);
        uint32_t* cp = cache_p(2u * kind);
        const uint32_t ch = cp[0], cd = cp[64];
        const bool upd = c & !((cd != 0) & (ch == vh) & (cd == d32));   // cache miss: the message goes out
        cp[0] = upd ? vh : ch;                                         // unconditional (no exec-mask branch)
        cp[64] = upd ? d32 : cd;
        const bool dup = upd & ((nxf & flag) != 0);                    // a second one of its kind this phase
        fl |= dup ? L_OBX : 0u;
        const bool put = upd & !dup;
        nxf |= put ? (flag | (has(L_BYZ) ? wflag : 0u)) : 0u;
        return put;
    }
    BFT_FN void out_preprepare_p(bool c) {                       // view (h, 0), own candidate; equivocates iff Byzantine
        const bool put = send_kind(c, 0, h, cand(), F_PP, F_PP_EQ);
        // only the round-0 proposer (validator 0 with big-endian seeds) proposes here: its Preprepare's time
        // tick is kept wave-uniform (SGPR); two proposers in one phase take the general path (run)
        const uint64_t bp = ballot(put);
        if (bp != 0) pp_T_out = uni(rl(cand_T, SEEDED ? ff1(bp) : 0u));
    }
    BFT_FN void out_prepare_p(bool c) { send_kind(c, 1, h, pp, F_PR, F_PR_W); }   // (h, 0, pp)
    BFT_FN void out_commit_p(bool c) { send_kind(c, 2, h, pp, F_CM, F_CM_W); }
    BFT_FN void out_blocks_p(bool c, uint32_t lo, uint32_t hi) {  // lo <= hi
        const bool hb = (nxf & F_BLK) != 0;
        nx_blo = c ? ((hb & (nx_blo < lo)) ? nx_blo : lo) : nx_blo;
        nx_bhi = c ? ((hb & (nx_bhi > hi)) ? nx_bhi : hi) : nx_bhi;
        nxf |= c ? F_BLK : 0u;
    }
    // the cold kinds always hand the instance over: fields straight to the hand-over area
    BFT_FN void out_old_commit(uint32_t vh, uint64_t d) {
        uint32_t* cp = cache_p(6);
        const uint32_t d32 = blk_d32(d);
        if (cp[64] != 0 && cp[0] == vh && cp[64] == d32) return;
        cp[0] = vh; cp[64] = d32;
        if (nxf & F_OCM) { *lane_p(F64Layout::W_LFL) |= FLAG_OUTBOX; return; }
        nxf |= F_OCM | (has(L_BYZ) ? F_OCM_W : 0u);
        uint32_t* s = save_p() + SAVE_COLD;
        s[0] = vh; s[1] = 0; s[2] = (uint32_t)d; s[3] = (uint32_t)(d >> 32);
    }
    BFT_FN void out_round_change(uint32_t vh, uint32_t vr) {
        if (nxf & F_RC) { *lane_p(F64Layout::W_LFL) |= FLAG_OUTBOX; return; }
        nxf |= F_RC;
        uint32_t* s = save_p() + SAVE_COLD;
        s[4] = vh; s[5] = vr;
    }
    BFT_FN void out_sync(uint32_t height) {
        uint32_t* s = save_p() + SAVE_COLD;
        if (nxf & F_SYNC) { if (height < s[6]) s[6] = height; return; }
        nxf |= F_SYNC;
        s[6] = height;
    }

    // ------------------------------------------------------------------ canonical rows
    // rows (flushed, canon_h] live in an LDS ring of 64 and are written to HBM 64 at a time, one
    // 16-byte row per lane (whole lines instead of single-lane stores)
    BFT_FN uint32_t* ring_row(uint32_t x) const { return (uint32_t*)(lds + F64Layout::RING_OFF) + (x & 63u) * 4u; }
    BFT_FN uint32_t* rec_row(uint32_t x) const { return P.rec + ((uint64_t)inst_local * P.rows + x) * 4; }
    BFT_FN uint32_t row_word(uint32_t x, uint32_t k) {
        if (x > flushed) return ring_row(x)[k];
        return wv.gload(rec_row(x) + k);
    }
    BFT_FN uint64_t canon_blk(uint32_t x) {                      // x >= 1, recorded
        if (x == canon_h) return canon_tip;
        const uint32_t w1 = row_word(x, 1), T = row_word(x, 2);
        return blk_make(x, w1 & 0xffffu, (w1 >> 16) & 1u, T);
    }
    BFT_FN void flush_rows() {                                   // uniform; rows (flushed, canon_h]
        wv.sync();
        const uint32_t x = flushed + 1u + me;
        if (x <= canon_h) {
            const uint32_t* r = ring_row(x);
            wv.gstore4(rec_row(x), r[0], r[1], r[2], r[3]);
        }
        wv.sync();
        flushed = canon_h;
    }
    // a new canonical height (uniform): row, histograms, instance-rounds
    BFT_FN void record_canon(uint32_t x, uint64_t b) {
        const uint32_t cnt = x <= P.heights ? 1u : 0u;             // uniform
        const uint32_t lat = (uint32_t)tick - canon_tick;
        views_acc += cnt;
        if (me == 0) {                                           // one lane: latency histogram and the ring row
            // the wave's own LDS histogram, one writer: a plain read-modify-write (an atomic becomes a
            // scalar loop over the active lanes)
            uint32_t* lb = (uint32_t*)(lds + F64Layout::LAT_OFF) + (lat < 64u ? lat : 64u);
            *lb += cnt;
            uint32_t* r = ring_row(x);
            r[0] = 0; r[1] = blk_prop(b) | (blk_var(b) << 16) | (1u << 24); r[2] = blk_T(b); r[3] = 0;   // seed: hash_pending
        }
        wv.sync();
        canon_h = x;
        canon_tip = b;
        canon_tick = (uint32_t)tick;
        if (canon_h - flushed == 64u) flush_rows();
    }

    // ------------------------------------------------------------------ chain, miner, timers
    BFT_FN void chain_insert_core_p(bool c) {                    // Chain::insert_block of pp (chain.rs:45-71)
        const uint32_t x = blk_h(pp);
        const bool nw = c & (x > last);                          // else ChainError::Exists
        const bool gap = nw & (last + 1 < x);                    // Not found ancestor → SyncBlock
        if (ballot(gap) != 0) { if (gap) out_sync(last + 1); }
        const bool ins = nw & !gap;
        fl |= ins ? L_CMT : 0u;
        last_T = ins ? (int32_t)blk_T(pp) : last_T;
        last = ins ? x : last;
        out_blocks_p(ins, x, x);                                 // ChainEvent::NewBlock
        miner_queue = (ins & (x > miner_queue)) ? x : miner_queue; // ChainEvent::NewHeader
    }
    // handle_msg_middle Block branch (core.rs:75-82) for the uniform range [lo, hi]
    BFT_FN void handle_blocks_p(bool c, uint32_t lo, uint32_t hi) {
        const bool nw = c & (hi > last);
        const bool gap = nw & (lo > last + 1);
        if (ballot(gap) != 0) { if (gap) out_sync(last + 1); }
        const bool ins = nw & !gap;
        // time tick of block hi: the canonical tip, or a recorded row (hi is uniform)
        const int32_t T = hi == canon_h ? (int32_t)blk_T(canon_tip) : (int32_t)uni(row_word(hi, 2));
        const uint32_t from = last + 1;
        last = ins ? hi : last;
        last_T = ins ? T : last_T;
        out_blocks_p(ins, from, hi);
        miner_queue = (ins & (hi > miner_queue)) ? hi : miner_queue;
    }
    BFT_FN void start_new_zero_round_p(bool c) {                 // core.rs:441-470
        h = c ? last + 1 : h;
        if (SEEDED) prop_l = c ? (seed_at(last) & 63u) : prop_l;   // (seed(tip) + round 0) mod 64
        fl = c ? ((fl & ~(L_ST | L_WAIT | L_LOCK | L_PENDV)) | ST_ACCEPT_REQUEST) : fl;
        pp = c ? BLK_NONE : pp;
        prep = c ? 0ull : prep;                                  // MessageManage::new
        comm = c ? 0ull : comm;
        fl |= c ? L_PROP : 0u;                                   // proposer = (seed + round 0) mod 64
        timer_tick = c ? tick + 1 : timer_tick;                  // new_round_change_timer
    }
    BFT_FN void send_preprepare_cand_p(bool c) {                 // preprepare.rs:30-43, req = candidate
        const bool s = c & (h == mint_height) & has(L_PROP) & (me == (SEEDED ? prop_l : 0u));
        if (ballot(s) != 0) {                                    // the proposer proposes
            bool cr = false;
            if (LOSSY && P.crash_on) cr = proposer_crashed(seed(), P.crash_thr32, 1u, inst, h, 0);
            out_preprepare_p(s & !cr);
        }
    }
    BFT_FN void handle_new_header_event_p(bool c) {              // core.rs:154-163 + request.rs:19-42
        c = c & !has(L_DEAD);
        start_new_zero_round_p(c);
        const bool pv = c & (h == mint_height);                  // accept the own candidate
        fl |= pv ? L_PENDV : 0u;
        if (pv) *lane_p(F64Layout::W_PENDT) = cand_T;
        send_preprepare_cand_p(pv);
    }
    BFT_FN void miner_mine_p(bool c) {                           // minner/mod.rs:95-143
        const uint32_t x = last + 1;
        const int32_t T = tick > last_T + 1 ? tick : last_T + 1;
        cand_T = c ? (uint32_t)T : cand_T;
        mint_height = c ? x : mint_height;
        const bool now = c & (T <= tick);                        // seal sleeps until header.time otherwise
        wake_tick = c ? (now ? -1 : T) : wake_tick;
        if (ballot(now) != 0) handle_new_header_event_p(now);
    }
    BFT_FN void miner_step_p() {                                 // Minner: Handler<NewHeader> (minner/mod.rs:56-69)
        const bool ev = has(L_RUN) & (wake_tick < 0);
        const uint32_t q = miner_queue;
        miner_queue = ev ? 0u : miner_queue;
        const bool m = ev & (q != 0) & (q >= mint_height);
        if (ballot(m) != 0) miner_mine_p(m);
    }
    BFT_FN void new_round_change_timer() { timer_tick = tick + 1; }
    BFT_FN void send_round_change(uint32_t round) {              // round_change.rs:38-63 (cold)
        if ((int32_t)*lane_p(F64Layout::W_RCLT) == tick) { new_round_change_timer(); return; }
        *lane_p(F64Layout::W_RCLT) = (uint32_t)tick;
        if (0u < round) { fl |= L_WAIT; new_round_change_timer(); }   // catchup_round (core.rs:555-565)
        out_round_change(h, round);
    }
    // send_next_round_change (round_change.rs:26-36): the RoundChangeSet is empty here (it only fills
    // from RoundChange messages, which hand over), so max_round() = 0 and the target is round 1
    BFT_FN void send_next_round_change() { send_round_change(1); }
    BFT_FN void t_step() {                                       // SPEC.md §2 T-step (running validators)
        const bool run = has(L_RUN);
        if (tick == 0) { start_new_zero_round_p(run); miner_mine_p(run); return; }
        const bool w = run & (wake_tick == tick);                // seal wakes up
        wake_tick = w ? -1 : wake_tick;
        if (ballot(w) != 0) handle_new_header_event_p(w);
        if (ballot(miner_event() != 0) != 0) miner_step_p();
        const bool sp = run & has(L_SYNCP);
        if (ballot(sp) != 0) {
            const uint32_t spv = *lane_p(F64Layout::W_SYNC);
            if (sp & (last < spv)) out_sync(last + 1);
            if (sp) *lane_p(F64Layout::W_SYNC) = 0;
            fl &= sp ? ~L_SYNCP : ~0u;
        }
        const bool tm = run & !has(L_DEAD) & (timer_tick == tick);  // TimerEvent (core.rs:207-225)
        if (ballot(tm) != 0) {
            timer_tick = tm ? -1 : timer_tick;
            const bool caught = tm & (last >= h);
            fl &= caught ? ~L_WAIT : ~0u;
            if (tm & !caught) send_next_round_change();
        }
    }
    // an outbox message or a queued chain event (SPEC.md §2). Integer form, no lane-mask logic: a queued
    // event is wake_tick < 0 and miner_queue >= max(mint_height, 1), i.e. bit 31 of m1 - 1 - mq. A
    // validator that is not running never has either (every handler and the T-step are gated by L_RUN).
    // the queued chain event of a running validator whose seal is not sleeping: miner_queue if
    // wake_tick < 0, else 0 (a validator that is not running never queues one)
    BFT_FN uint32_t miner_event() const { return wake_tick < 0 ? miner_queue : 0u; }
    BFT_FN bool pending_local() const {
        const uint32_t mq = wake_tick < 0 ? miner_queue : 0u;
        const uint32_t m1 = mint_height > 1u ? mint_height : 1u;
        return (nxf | ((m1 + ~mq) >> 31)) != 0;
    }

    // ------------------------------------------------------------------ handlers
    // HandlePreprepare::handle (preprepare.rs:45-126) of the phase's single Preprepare (uniform src, view)
    // sm: the SPLIT bits of view (vh, 0) if the proposer equivocates, else 0 (split_mask)
    BFT_FN void handle_preprepare_p(bool c, uint32_t src, uint32_t vh, uint64_t b, uint64_t sm) {
        // SPEC.md §6: variant 1 to SPLIT receivers
        b |= ((me != src) & (((sm >> me) & 1ull) != 0)) ? (1ull << 33) : 0ull;
        // check_message (core.rs:366-399) of a Preprepare of height vh (uniform): Unknown for 0, OK at h,
        // FutureBlock above h (falls through), OldMessage below
        const bool vok = vh != 0;
        bool go = c & vok & (vh >= h);
        const bool old = c & vok & (vh < h);
        if (ballot(old) != 0) {                                  // a Preprepare of a passed height
            if (old) {
                const uint32_t bh = blk_h(b);
                if (bh <= last && blk_eq(canon_blk(bh), b)) {    // else InvalidProposal
                    // old proposer (preprepare.rs:61-64): seed of block bh - 1, round 0
                    if (src == (SEEDED ? (seed_at(bh - 1u) & 63u) : 0u)) out_old_commit(vh, b);
                    go = true;                                   // falls through (preprepare.rs:52-74)
                }
            }
        }
        go = go & has(L_PROP) & (src == (SEEDED ? prop_l : 0u));   // else NotFromProposer
        const uint32_t bh = blk_h(b);
        const bool bad = go & ((bh == 0) | (bh - 1 > last));    // Backend::verify: unknown ancestor
        const bool acc = go & !bad & (st() == ST_ACCEPT_REQUEST);
        const bool lk = acc & has(L_LOCK);
        const bool lk_ok = lk & beq(b, pp);                      // locked: same block → commit
        const bool unl = acc & !has(L_LOCK);                     // unlocked: accept → prepare
        pp = (lk_ok | unl) ? b : pp;
        fl = lk_ok ? ((fl & ~L_ST) | ST_PREPARED) : unl ? ((fl & ~L_ST) | ST_PREPREPARED) : fl;
        out_prepare_p(unl);                                      // send_prepare
        out_commit_p(lk_ok | (unl & has(L_BYZ)));                // send_commit / Byzantine commit (SPEC.md §6)
        const bool rc = bad | (lk & !lk_ok);
        if (ballot(rc) != 0) { if (rc) send_next_round_change(); }
    }
    BFT_FN void lock_hash() { if (blk_valid(pp)) fl |= L_LOCK; }   // round_state.rs:100-110 (lock = pp)

    // SPLIT bits of receivers 0..63 for view (vh, 0) (SPEC.md §5; split_bit for v < 64): one uniform draw
    // Evaluated on the vector lanes (every lane the same draw): as a scalar Philox it is ~100
    // instructions on the CU's one scalar unit, the kernel's bottleneck.
    BFT_FN uint64_t split_mask(uint32_t vh) const {
        uint32_t v = vh;
        BFT_OPAQUE_VGPR(v);
        uint32_t w[4];
        philox(seed(), inst, v, 0, DOM_SPLIT, w);
        return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    }

    // digests of class `cls` matching `target` (wildcards match both variants)
    BFT_FN static uint64_t class_match(uint64_t cls, uint64_t v0, uint64_t v1, uint64_t w, uint64_t target) {
        if (!blk_valid(target) || ((cls ^ target) & BLK_HP_MASK) != 0) return 0;
        return w | (blk_var(target) ? v1 : v0);
    }
    // smallest p with popcount(base | a & low(p+1) | b & low(p)) > Q, else 64
    BFT_FN static uint32_t first_over(uint64_t base, uint64_t a, uint64_t b) {
        if (popc(base | a | (b & low(63))) <= Q) return 64;
        uint32_t lo = 0, hi = 63;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (popc(base | (a & low(mid + 1)) | (b & low(mid))) > Q) hi = mid;
            else lo = mid + 1;
        }
        return lo;
    }

    struct PC {                         // a Prepare/Commit phase (wave-uniform)
        uint64_t kpr, kcm, v1, pr_cls, cm_cls;   // v1: senders whose digest is variant 1
        uint32_t pr_h, cm_h;
    };
    // senders of `k` whose digest matches `target` of class `cls`: Byzantine wildcards match both variants
    BFT_FN uint64_t class_match_k(uint64_t k, uint64_t v1, uint64_t cls, uint64_t target) const {
        if (!blk_valid(target) || ((cls ^ target) & BLK_HP_MASK) != 0) return 0;
        return k & (byz_mask | (blk_var(target) ? v1 : ~v1));
    }
    // prepare.rs:48-66 and commit.rs:63-82 in this receiver's rotated delivery order, as prefix masks
    // (the closed form of bft_wave.h deliver_prepare_commit with round 0 and lock = pp)
    BFT_FN void deliver_pc(bool rcv, const PC& c, uint64_t mk, uint32_t off) {
        const uint64_t prd = rcv ? (mk & c.kpr) : 0ull, cmd = rcv ? (mk & c.kcm) : 0ull;
        const uint32_t s0 = st();
        // check_message (core.rs:366-399) of a Prepare / Commit of the uniform height vh: Unknown for
        // vh = 0, FutureBlock above h, OK at h once the Core is past AcceptRequest
        const bool sok = s0 != ST_ACCEPT_REQUEST;
        const bool prn = c.pr_h != 0, cmn = c.cm_h != 0;
        // FutureBlockMessage → the delayed sync check (core.rs:58-69)
        const bool fpr = (prd != 0) & prn & (c.pr_h > h), fcm = (cmd != 0) & cmn & (c.cm_h > h);
        if (ballot(fpr | fcm) != 0) {
            if (fpr | fcm) {
                uint32_t v = *lane_p(F64Layout::W_SYNC);
                v = (fpr & (c.pr_h > v)) ? c.pr_h : v;
                v = (fcm & (c.cm_h > v)) ? c.cm_h : v;
                *lane_p(F64Layout::W_SYNC) = v;
                fl |= L_SYNCP;                                   // v > h >= 1
            }
        }
        // digests matching the own pp (class_match_k): a Byzantine sender's wildcard matches both variants
        const uint64_t vsel = byz_mask | (blk_var(pp) ? c.v1 : ~c.v1);
        const bool ppv = blk_valid(pp);
        const bool mpr = ppv & (((c.pr_cls ^ pp) & BLK_HP_MASK) == 0);
        const bool mcm = ppv & (((c.cm_cls ^ pp) & BLK_HP_MASK) == 0);
        const uint64_t PRacc = (prn & sok & (c.pr_h == h)) ? prd : 0ull;
        const uint64_t CMacc = (cmn & sok & (c.cm_h == h) & mcm) ? (cmd & vsel) : 0ull;   // cmd ⊆ kcm
        // Order-free evaluation first. The delivery order (rotation by `off`) only matters when the
        // prepare quorum is crossed by commits delivered before the last prepare, or when a trigger and a
        // commit quorum both occur (which comes last decides Prepared vs Committed); lanes in either case
        // take the exact rotated closed form below (a uniform branch, skipped when no lane needs it).
        const uint64_t U = prep | comm;
        const uint64_t mpp0 = mpr ? (PRacc & vsel) : 0ull;        // PRacc ⊆ kpr
        const uint32_t nUP = popc(U | PRacc);
        const bool pra = PRacc != 0, cma = CMacc != 0;
        const bool cexists = cma & (popc(comm | CMacc) > Q);
        const bool tb_amb = pra & cma & (nUP <= Q) & (popc(U | PRacc | CMacc) > Q);
        bool trig = (pra & (nUP > Q)) | (has(L_LOCK) & (mpp0 != 0));
        const bool committed = s0 >= ST_COMMITTED;
        bool fires = !trig & cexists & !committed;
        uint32_t fin = trig ? ST_PREPARED : (fires ? ST_COMMITTED : s0);
        const bool amb = tb_amb | (trig & cexists);
        if (ballot(amb) != 0) {
            if (amb) {
                const uint64_t PR = rotr(PRacc, off), CM = rotr(CMacc, off);
                const uint64_t U0 = rotr(U, off);
                const uint32_t lastPR = hibit(PR), lastCM = hibit(CM);
                const bool trigB = (PR != 0) & (popc(U0 | PR | (CM & low(lastPR))) > Q);
                const uint64_t mpp = rotr(mpp0, off);
                const uint64_t lm = has(L_LOCK) ? mpp : 0ull;       // lock == pp when locked
                trig = trigB | (lm != 0);
                uint32_t t1 = lm ? ctz64(lm) : 64u;
                const uint32_t lastT = trigB ? lastPR : hibit((mpp & ~low(t1)) | (t1 < 64u ? (1ull << t1) : 0ull));
                if (trig & committed & trigB) {                    // a re-commit needs a commit after the first trigger
                    const uint32_t pstar = first_over(U0, PR, CM);
                    const uint64_t ge = PR & ~low(pstar);
                    const uint32_t tB = ge ? ctz64(ge) : 64u;
                    t1 = tB < t1 ? tB : t1;
                }
                fires = trig ? (committed ? (cexists & (lastCM >= t1)) : cexists) : (cexists & !committed);
                fin = trig ? ((cexists & (lastCM >= lastT)) ? ST_COMMITTED : ST_PREPARED) : (fires ? ST_COMMITTED : s0);
            }
        }
        prep |= PRacc;
        comm |= CMacc;
        fl |= ((trig | fires) & ppv) ? L_LOCK : 0u;               // lock_hash
        out_commit_p(trig);                                      // send_commit
        chain_insert_core_p(fires);                              // Core::commit → insert_block
        set_st(fin);
    }

    // ------------------------------------------------------------------ commits of a phase → canonical chain
    // Returns the committed height when every committer of the phase committed the same one (each of
    // them then has the block range [x0, x0] in its outbox, chain_insert_core_p), else 0.
    // SEEDED: the hash and seed of every height recorded since the last call, in height order (one call site,
    // so the wave hash is inlined once), before any validator can start the next height
    uint32_t hashed_h;
    // SEEDED with predicted blocks (P.spec, bft_seed_chain_kernel): while every recorded height equals its
    // prediction, the prediction's hash (already in P.hash) and seed are the block's; from the first height
    // that differs, the wave hashes as before, from the last matching block's hash
    bool spec_ok;
    BFT_FN void hash_pending() {
        while (hashed_h < canon_h) {                             // uniform
            const uint32_t x = hashed_h + 1u;
            const uint64_t b = canon_blk(x);
            uint32_t sd = 0;
            bool take = false;
            if (spec_ok) {
                const uint32_t sw = x <= P.heights ? uni(wv.gload(P.spec + (uint64_t)x * P.n_instances + inst_local)) : 0u;
                const uint32_t sseed = (sw >> 16) & 0xffu;
                take = (sw == spec_word(blk_prop(b), blk_var(b), sseed)) & (blk_T(b) + 1u == x);
                sd = sseed;
                if (!take) {                                     // the wave hashes from here: the parent's hash
                    spec_ok = false;
                    const uint32_t* ph = x == 1u ? (const uint32_t*)P.genesis_hash
                                                 : (const uint32_t*)(P.hash + ((uint64_t)inst_local * P.rows + x - 1u) * 32);
                    tip_w = me < 8u ? ph[me] : 0u;
                }
            }
            if (!take) {
                const uint64_t time = P.genesis_time + (uint64_t)P.block_period * ((uint64_t)blk_T(b) + 1ull);
                const uint32_t hw = kw50_header_hash(wv, me, lds + F64Layout::KW_OFF, tip_w,
                                                     P.addresses + 20u * blk_prop(b), seed(), inst, x, blk_prop(b),
                                                     blk_var(b), time);
                if (me < 8u) ((uint32_t*)(P.hash + ((uint64_t)inst_local * P.rows + x) * 32))[me] = hw;
                tip_w = hw;
                sd = seed_from_words(uni(rl(hw, 0)), uni(rl(hw, 1)), N, P.seed_le != 0);
            }
            if (me == 0) {                                       // the row's seed word, wherever the row is now
                if (x > flushed) ring_row(x)[3] = sd;
                else wv.gstore(rec_row(x) + 3, sd);
            }
            wv.sync();
            if (x == canon_h) canon_seed = sd;
            hashed_h = x;
        }
    }
    BFT_FN uint32_t resolve_commits() {
        const uint32_t xc = resolve_commits_core();
        if (SEEDED) hash_pending();
        return xc;
    }
    BFT_FN uint32_t resolve_commits_core() {
        const bool c = has(L_CMT);
        const uint64_t bal = ballot(c);
        if (bal == 0) return 0;
        fl &= ~L_CMT;
        if (seg_done) return 0;
        const uint32_t lead = ctz64(bal);
        const uint32_t x = blk_h(pp);
        const uint32_t x0 = uni(rl(x, lead));
        if (ballot(c & (x != x0)) == 0) {
            // every committer commits the first one's height (the common case): uniform update
            const uint64_t b0 = rl64(pp, lead);
            const bool known = x0 <= canon_h;
            const uint64_t ref = known ? canon_blk(x0) : b0;
            const uint64_t badm = ballot(c & !beq(pp, ref));
            bool fr = badm != 0;
            if (!known && x0 < P.hcap && (!fr || ctz64(badm) > lead)) record_canon(x0, b0);
            if (x0 >= P.hcap) fr = true;
            if (fr) { frozen = true; seg_flags |= FLAG_SAFETY; }
            return x0;
        }
        // mixed heights: replay the commits in lane order (the oracle's receiver order)
        uint64_t bits = bal;
        bool fr = false;
        while (bits) {
            const uint32_t j = ctz64(bits);
            bits &= bits - 1ull;
            const uint32_t xj = uni(rl(x, j));
            const uint64_t bj = rl64(pp, j);
            if (xj >= P.hcap) { fr = true; break; }
            if (xj <= canon_h) {
                if (!blk_eq(canon_blk(xj), bj)) { fr = true; break; }
            } else {
                record_canon(xj, bj);                            // xj == canon_h + 1
            }
        }
        if (fr) { frozen = true; seg_flags |= FLAG_SAFETY; }
        return 0;
    }

    // ------------------------------------------------------------------ the canonical height, composed
    // Lossless schedule. When the honest round-0 proposer's Preprepare (view (H, 0); validator 0 with
    // big-endian seeds, seed(tip) mod 64 with little-endian ones) is the only message in flight and every validator waits for it in the state
    // start_new_zero_round left (core.rs:441-470: AcceptRequest, unlocked, chain tip H - 1, nothing
    // queued for the miner), the next four phases have one outcome, and this applies it directly:
    //   PP  — everyone accepts (preprepare.rs:87-106): pp = b, Preprepared, send_prepare; the Byzantine
    //         validators also commit at once (SPEC.md §6);
    //   PC1 — 64 Prepares > Q (prepare.rs:59-63): lock_hash, Prepared, send_commit (the Byzantine ones'
    //         Commits are outbound-cache hits, backend.rs:141-148); their ≤ Q early Commits fire nothing;
    //   PC2 — the honest Commits complete 64 > Q (commit.rs:63-82): Committed, Core::commit →
    //         insert_block (chain.rs:45-71), Blocks out, NewHeader queued;
    //   BLK — the fused block-gossip phase of `run` (ChainError::Exists for everyone) → the miner step.
    // The preconditions make each phase's closed form (handle_preprepare_p, deliver_pc,
    // resolve_commits, the fused phase) take exactly this branch; `macro_ok` (set once per instance)
    // adds every validator running and at most Q Byzantine ones (their early Commits never reach the
    // commit quorum in PC1). Bit-identical by construction; checked by the emulator suite and fuzzer.
    bool macro_ok;
    // It runs in place of the PP phase's classification; the PP phase's event step is skipped, being a
    // no-op (nothing queued for the miner), and the phase's resolve_commits and fused block phase then
    // run unchanged, so the single call sites of record_canon / hash_pending stay single.
    // j: the Preprepare's sender, fj its flags, H its height, sm as in handle_preprepare_p
    BFT_FN bool canonical_step(uint32_t j, uint32_t fj, uint32_t H) {
        if ((canon_h + 1u != H) | (H >= P.hcap)) return false;
        // an equivocating proposer's variant 1 goes to the SPLIT receivers (SPEC.md §5, handle_preprepare_p);
        // one draw, every lane the same: held in SGPRs
        uint64_t v1m = 0;
        if (fj & F_PP_EQ) {
            const uint64_t d = split_mask(H);
            v1m = ((uint64_t)uni((uint32_t)d) | ((uint64_t)uni((uint32_t)(d >> 32)) << 32)) & ~(1ull << j);
        }
        // PC2: a validator commits iff the Byzantine wildcards and the honest Commits of its own variant
        // exceed Q; exactly one variant may commit (both: a fork, neither: round changes — the phase loop)
        const uint64_t hon = ~byz_mask;
        const bool k0 = popc(byz_mask | (hon & ~v1m)) > Q, k1 = popc(byz_mask | (hon & v1m)) > Q;
        if (k0 == k1) return false;
        const bool var = ((v1m >> me) & 1ull) != 0;
        const uint64_t b = blk_make(H, j, var ? 1u : 0u, pp_T_out);
        const uint32_t d32 = blk_d32(b);
        uint32_t* c1 = cache_p(2);                                 // Prepare {h, d32}
        uint32_t* c2 = cache_p(4);                                 // Commit {h, d32}
        const bool hit1 = (c1[64] == d32) & (c1[0] == H), hit2 = (c2[64] == d32) & (c2[0] == H);   // d32 != 0
        const bool ok = (h == H) & (st() == ST_ACCEPT_REQUEST) & ((fl & (L_LOCK | L_DEAD | L_PROP)) == L_PROP) &
                        (last + 1u == H) & (miner_event() == 0u) & (nxf == (me == j ? fj : 0u)) &
                        (!SEEDED | (prop_l == j)) & !hit1 & !hit2;
        if (ballot(!ok) != 0) return false;
        const bool fires = var == k1;
        pp = b;
        prep = ~0ull;                                            // every validator's Prepare
        comm = byz_mask | (hon & (var ? v1m : ~v1m));           // early Byzantine (PP) + matching honest (PC1)
        fl = (fl & ~L_ST) | (fires ? (ST_COMMITTED | L_CMT) : ST_PREPARED) | L_LOCK;
        c1[0] = H; c1[64] = d32;
        c2[0] = H; c2[64] = d32;
        last = fires ? H : last;                                 // insert_block, Blocks [H, H] out
        last_T = fires ? (int32_t)pp_T_out : last_T;
        nx_blo = fires ? H : nx_blo;
        nx_bhi = fires ? H : nx_bhi;
        miner_queue = (fires & (H > miner_queue)) ? H : miner_queue;
        nxf = fires ? (uint32_t)F_BLK : 0u;
        return true;
    }

    // ------------------------------------------------------------------ the canonical tick, composed
    // Lossless schedule; proposer j = 0 (big-endian seeds) or seed(tip) mod 64 (little-endian, SEEDED: the
    // new height is hashed by the wave as resolve_commits does). When a tick starts with every validator where the
    // previous canonical height left it -- its seal waking now for height H = canon_h + 1 (wake_tick ==
    // tick, mint_height == H, chain tip H - 1), nothing in flight or queued -- the whole tick has one
    // outcome, and this applies it to every lane's registers at once:
    //   T-step  — the seal wakes (minner/mod.rs:95-143 → core.rs:154-163): start_new_zero_round
    //             (core.rs:441-470) for everyone, the own candidate accepted as the pending request
    //             (request.rs:19-42), validator j sends its Preprepare (preprepare.rs:30-43); no timer fires
    //             (start_new_zero_round re-arms it first) and no miner event is queued;
    //   PP, PC1, PC2 — canonical_step (above);
    //   commit  — resolve_commits records height H (one digest among the committers);
    //   BLK     — pattern A (every lane committed): the fused block phase; pattern B (an equivocating
    //             proposer split the validators, only one variant committed): two block-gossip phases,
    //             the committers' Blocks [H, H] inserted by the others (core.rs:75-82, chain.rs:45-71) and
    //             then theirs, ChainError::Exists for everyone;
    //   miner   — every lane mines H + 1 at max(tick, block time + 1) (minner/mod.rs:95-143) = the block
    //             time + 1 > tick: the seal sleeps until then (wake_tick).
    // Both patterns end in the same per-lane state except the variant each lane holds (pp, comm) and its
    // state (Committed for the committing variant, Prepared for the other). Phases used: 4 (A) or 5 (B) of
    // phase_cap. Preconditions: the ballot below, k0 != k1 (canonical_step), H < hcap, phase_cap >= 5,
    // and the block time of H (the proposer's cand_T) >= tick. Anything else runs the T-step and phase loop.
    // Bit-identical by construction; checked by the emulator suite and the lossless fuzzer
    // (tests/fuzz_parity.py lossless64).
    BFT_FN bool canonical_tick() {
        const uint32_t H = canon_h + 1u;
        if (frozen | (H >= P.hcap) | (P.phase_cap < 5u)) return false;
        const int32_t t = tick;
        // the round-0 proposer of H: validator 0 with big-endian seeds, seed(tip) mod 64 with little-endian
        // ones (start_new_zero_round_p: the seed of block H - 1 = the canonical tip)
        const uint32_t j = SEEDED ? (canon_seed & 63u) : 0u;
        const uint32_t ptout = uni(rl(cand_T, j));                  // the proposer's block time tick
        if ((int32_t)ptout < t) return false;
        uint32_t* pc = cache_p(0);                                  // Preprepare {h, d32}
        uint32_t* c1 = cache_p(2);                                  // Prepare
        uint32_t* c2 = cache_p(4);                                  // Commit
        const uint32_t hd = (H & 0x3fffffu) | (j << 22) | 0x80000000u;   // blk_d32 of (H, proposer j, variant 0)
        // integer form (one compare per lane, no lane-mask arithmetic on the scalar unit): a nonzero word
        // marks a validator that is not where the previous canonical tick left it; heights are < 2^22, so
        // ((a ^ b) - 1) >> 31 is 1 exactly when a == b
        const uint32_t pc_h = pc[0], pc_d = pc[64];
        const uint32_t pp_hit = (((pc_h ^ H) | (pc_d ^ hd) | (me ^ j)) == 0u) ? 1u : 0u;   // out_preprepare's cache
        const uint32_t bad = (fl & (L_DEAD | L_SYNCP)) | ((uint32_t)wake_tick ^ (uint32_t)t) | miner_queue | nxf |
                             (last ^ canon_h) | (mint_height ^ H) | (((c1[0] ^ H) - 1u) >> 31) |
                             (((c2[0] ^ H) - 1u) >> 31) | pp_hit;
        if (ballot(bad != 0u) != 0) return false;
        // canonical_step's split and quorum decision (the proposer's F_PP_EQ = it is Byzantine)
        uint64_t v1m = 0;
        if ((byz_mask >> j) & 1ull) {
            const uint64_t d = split_mask(H);
            v1m = ((uint64_t)uni((uint32_t)d) | ((uint64_t)uni((uint32_t)(d >> 32)) << 32)) & ~(1ull << j);
        }
        const uint64_t hon = ~byz_mask;
        const bool k0 = popc(byz_mask | (hon & ~v1m)) > Q, k1 = popc(byz_mask | (hon & v1m)) > Q;
        if (k0 == k1) return false;
        // T-step: the pending request and the proposer's Preprepare through its outbound cache
        *lane_p(F64Layout::W_PENDT) = cand_T;
        if (me == j) { pc[0] = H; pc[64] = hd; }
        pp_T_out = ptout;
        if (SEEDED) prop_l = j;
        // PP, PC1, PC2 (canonical_step) and the block phases: the per-lane result
        // this lane's bit of the uniform mask from its 32-bit half (a 64-bit per-lane 1 << me would be one
        // more register pair, spilled at 6 waves per SIMD and reloaded on every tick)
        const uint32_t vw = me < 32u ? (uint32_t)v1m : (uint32_t)(v1m >> 32);
        const bool var = ((vw >> (me & 31u)) & 1u) != 0u;
        const bool fires = var == k1;
        const uint32_t d32 = hd | (var ? (1u << 30) : 0u);
        c1[0] = H; c1[64] = d32;
        c2[0] = H; c2[64] = d32;
        h = H;
        pp = blk_make(H, j, var ? 1u : 0u, ptout);
        prep = ~0ull;
        comm = byz_mask | (hon & (var ? v1m : ~v1m));
        fl = (fl & ~(L_ST | L_WAIT | L_LOCK | L_PENDV | L_CMT)) | L_PROP | L_PENDV | L_LOCK |
             (fires ? ST_COMMITTED : ST_PREPARED);
        timer_tick = t + 1;
        last = H;
        last_T = (int32_t)ptout;
        cand_T = ptout + 1u;
        mint_height = H + 1u;
        wake_tick = (int32_t)ptout + 1;
        miner_queue = 0;
        nxf = 0;
        nx_blo = H;
        nx_bhi = H;
        record_canon(H, blk_make(H, j, k1 ? 1u : 0u, ptout));
        if (SEEDED) hash_pending();                                 // resolve_commits: hash (and seed) of H
        return true;
    }

    // ------------------------------------------------------------------ hand-over to the full kernel
    // the full kernel's save layout (bft_wave.h BFT_STATE_32 / BFT_STATE_64, then prep, comm, the 12
    // cache words, the bool bits, tick, phase); every implied field is expanded here
    BFT_FN void save_state(uint32_t p) {
        flush_rows();
        uint32_t* s = save_p();
        const uint64_t lock = has(L_LOCK) ? pp : BLK_NONE;
        const uint64_t pend = has(L_PENDV) ? blk_make(h, me, 0, *lane_p(F64Layout::W_PENDT)) : BLK_NONE;
        const uint64_t cd = mint_height ? cand() : BLK_NONE;
        const uint64_t ppb = blk_make(h, me, 0, pp_T_out);     // read only where F_PP is set (lane 0)
        const uint32_t lseed = SEEDED ? seed_at(last) : 0u;
        const uint32_t cseed = SEEDED ? canon_seed : 0u;
        const uint32_t w32[29] = {h, 0u, st(), 0u, proposer(), last, lseed, (uint32_t)last_T, (uint32_t)timer_tick,
                                  *lane_p(F64Layout::W_RCLT), (uint32_t)wake_tick, mint_height, miner_queue,
                                  *lane_p(F64Layout::W_SYNC), lane_flags(), canon_h, done_tick, seg_flags, cseed, canon_tick, nxf,
                                  h, 0u, h, 0u, h, 0u, nx_blo, nx_bhi};
        uint32_t k = 0;
        for (uint32_t i = 0; i < 29; ++i) s[k++] = w32[i];
        const uint64_t w64[9] = {lock, pp, pend, cd, canon_tip, views_acc, ppb, pp, pp};
        for (uint32_t i = 0; i < 9; ++i) { s[k++] = (uint32_t)w64[i]; s[k++] = (uint32_t)(w64[i] >> 32); }
        s[k++] = (uint32_t)prep; s[k++] = (uint32_t)(prep >> 32);
        s[k++] = (uint32_t)comm; s[k++] = (uint32_t)(comm >> 32);
        for (uint32_t kind = 0; kind < 4; ++kind) {              // {height, round, d32} per kind
            s[k++] = *cache_p(2u * kind);
            s[k++] = 0u;
            s[k++] = *cache_p(2u * kind + 1u);
        }
        s[k++] = (has(L_BYZ) ? 1u : 0u) | (has(L_DEAD) ? 2u : 0u) | (has(L_WAIT) ? 4u : 0u) | (frozen ? 8u : 0u) |
                 (seg_done ? 16u : 0u);
        s[k++] = (uint32_t)tick;
        s[k++] = p;
    }

    BFT_FN void init_byzantine() {       // partial Fisher-Yates by lane 0 (SPEC.md §5), LDS scratch
        uint8_t* perm = lds + F64Layout::RING_OFF;
        uint32_t* mw = (uint32_t*)(lds + F64Layout::RING_OFF + 64);
        if (me == 0 && !seg_done) {
            for (uint32_t i = 0; i < N; ++i) perm[i] = (uint8_t)i;
            uint64_t mask = 0;
            const uint32_t f = P.byz_count < N ? P.byz_count : N;
            for (uint32_t i = 0; i < f; ++i) {
                uint32_t w[4];
                philox(P.seed, inst, i, 0, DOM_BYZ, w);
                const uint32_t j = i + w[0] % (N - i);
                const uint8_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
                mask |= 1ull << perm[i];
            }
            mw[0] = (uint32_t)mask; mw[1] = (uint32_t)(mask >> 32);
        }
        wv.sync();
        const uint64_t mask = seg_done ? 0ull : (uint64_t)uni(mw[0]) | ((uint64_t)uni(mw[1]) << 32);
        byz_mask = mask;
        if ((mask >> me) & 1ull) fl |= L_BYZ;
        wv.sync();
    }

    // ------------------------------------------------------------------ the run
    BFT_FN void run() {
#ifdef BFT_STAMPS
        for (int k = 0; k < NSTAMP; ++k) st_acc[k] = 0;
        st_t = wv.clock();
#endif
        if (P.byz_count > 0) init_byzantine();
        macro_ok = !LOSSY && ballot(has(L_RUN)) == ~0ull && popc(byz_mask) <= Q;
        uint32_t* lat = (uint32_t*)(lds + F64Layout::LAT_OFF);
        for (uint32_t b = me; b < 65u; b += 64u) lat[b] = 0;
        wv.sync();
        bool bailed = false;
        for (tick = 0; tick < (int32_t)P.max_ticks; ++tick) {
            if (seg_done) break;
            // a run of canonical ticks (lossless schedules): T-step and phases in one closed form each,
            // in a loop of its own (few live values: no copies of the whole state at every branch); the first
            // tick that is not canonical falls through to the T-step and phase loop below, unchanged
            if (!LOSSY && macro_ok && tick != 0) {
                bool stop = false;
                while (canonical_tick()) {
                    F64_STAMP(1);
                    if (canon_h >= P.heights) { seg_done = true; done_tick = (uint32_t)tick + 1; stop = true; break; }
                    if (++tick >= (int32_t)P.max_ticks) { stop = true; break; }
                }
                if (stop) break;
            }
            // act: this instance still runs this tick (uniform); per lane, only running validators
            // (not silent) handle events and messages
            bool act = !frozen;
            off_tick = offset_tick_part(off_inst, (uint32_t)tick);
            F64_STAMP(7);
            // the T-step, only when some running validator has a tick event
            // (a validator that is not running has no events: wake_tick, timer_tick -1, nothing queued)
            if (tick == 0 || ballot((wake_tick == tick) | ((wake_tick < 0) & (miner_queue != 0)) |
                                    has(L_SYNCP) | (!has(L_DEAD) & (timer_tick == tick))) != 0) {
                t_step();
            }
            F64_STAMP(0);
            for (uint32_t p = 0;; ++p) {
                if (!act || ballot(pending_local()) == 0) break;
                if (p >= P.phase_cap) {                          // in-flight messages are dropped (SPEC.md §2)
                    if (ballot(has(L_RUN) && nxf != 0) != 0) seg_flags |= FLAG_PHASE_CAP;
                    nxf = 0;
                    break;
                }
                // the Preprepare in flight: its sender j (the round-0 proposer: validator 0 with big-endian
                // seeds; with SEEDED the first sender, two senders take the general path), its flags and
                // height; the SPLIT draw once per phase for an equivocating sender (SPEC.md §5)
                const uint64_t kpp = ballot((nxf & F_PP) != 0);
                const uint32_t j = SEEDED ? ff1(kpp) : 0u;
                const uint32_t fj = uni(rl(nxf, j)), pp_h = uni(rl(h, j));
                const uint32_t pp_eq = kpp ? (fj & F_PP_EQ) : 0u;
                // the round-0 proposer's Preprepare alone in flight, every validator waiting for it: the
                // height's PP and two Prepare/Commit phases at once (canonical_step)
                const bool canon = !LOSSY && macro_ok && (p + 3u < P.phase_cap) && (kpp == (1ull << j)) &&
                                   ((fj & ~(uint32_t)F_PP_EQ) == F_PP) && canonical_step(j, fj, pp_h);
                uint32_t path = P_CANON, blo = 0, bhi = 0;
                uint64_t kpr = 0, kcm = 0, kblk = 0;
                PC c;
                if (!canon) {
                    // what is in flight, by kind (segment = wave). The classification is branch-free: every
                    // kind's first sender is read whether or not the kind is present, so no per-path values
                    // are merged at control-flow joins (those merges cost a copy of every live value).
                    const uint32_t f = nxf;
                    const bool pr = (f & F_PR) != 0, cm = (f & F_CM) != 0;
                    kpr = ballot(pr); kcm = ballot(cm);
                    kblk = ballot((f & F_BLK) != 0);
                    const uint64_t kcold = ballot((f & (F_OCM | F_RC | F_SYNC)) != 0);
                    const uint32_t jp = ff1(kpr), jc = ff1(kcm), jb = ff1(kblk);
                    const uint64_t cls = pp & BLK_HP_MASK;
                    c.kpr = kpr; c.kcm = kcm;
                    const uint32_t hp = uni(rl(h, jp)), hc = uni(rl(h, jc));
                    c.pr_h = kpr ? hp : 0u;
                    c.cm_h = kcm ? hc : 0u;
                    c.pr_cls = rl64(cls, jp);
                    c.cm_cls = rl64(cls, jc);
                    c.v1 = ballot(blk_var(pp) != 0);
                    blo = uni(rl(nx_blo, jb)); bhi = uni(rl(nx_bhi, jb));
                    if (kcold | (SEEDED ? (kpp & (kpp - 1ull)) : 0ull)) path = P_GENERAL;
                    else if (kpp) path = (kpr | kcm | kblk) == 0 ? P_PP : P_GENERAL;
                    else if (kpr | kcm) path = kblk ? P_GENERAL : P_PC;
                    else path = kblk ? P_BLK : P_NONE;
                    // a PC phase needs one view and digest class per kind, a BLK phase one block range
                    // (integer form: a nonzero XOR marks a mismatch, one compare per lane)
                    const uint32_t cls_lo = (uint32_t)cls, cls_hi = (uint32_t)(cls >> 32);
                    const uint32_t bad_pr = (h ^ c.pr_h) | (cls_lo ^ (uint32_t)c.pr_cls) | (cls_hi ^ (uint32_t)(c.pr_cls >> 32));
                    const uint32_t bad_cm = (h ^ c.cm_h) | (cls_lo ^ (uint32_t)c.cm_cls) | (cls_hi ^ (uint32_t)(c.cm_cls >> 32));
                    const uint32_t bad_pc = (pr ? bad_pr : 0u) | (cm ? bad_cm : 0u);
                    const uint32_t bad_blk = (f & F_BLK) ? ((nx_blo ^ blo) | (nx_bhi ^ bhi)) : 0u;
                    const uint32_t bad = path == P_PC ? bad_pc : (path == P_BLK ? bad_blk : 0u);
                    if (ballot(bad != 0) != 0) path = P_GENERAL;
                    if (path == P_GENERAL) {                          // hand the instance to the full kernel
                        save_state(p);
                        if (me == 0) {
                            P.resume_flags[inst_local] = 1u;
#if defined(__HIP_DEVICE_COMPILE__)
                            if (P.resume_q) P.resume_q[2u + atomicAdd(P.resume_q, 1u)] = inst_local;   // the resume queue
#endif
                        }
                        bailed = true;
                        seg_done = true;
                        break;
                    }
                }
                F64_STAMP(1);
                F64_COUNT(8);
                if (canon) {                                       // PP, PC1, PC2 of the canonical height, applied
                    p += 2u;
                    F64_COUNT(8); F64_COUNT(8); F64_COUNT(9); F64_COUNT(10); F64_COUNT(10); F64_COUNT(12);
                } else if (act) {
                    nxf = 0;
                    // event step: Minner's NewHeader handler, for the validators with queued chain events
                    miner_step_p();   // a no-op for lanes without a queued event (miner_step_p guards the mining)
                    F64_STAMP(2);
                    if (path != P_NONE) {
                        const uint64_t mk = LOSSY ? deliver_mask<1>(seed(), N, P.thr16, inst, (uint32_t)tick, p, me,
                                                                    Bits<1>::from(kpp | kpr | kcm | kblk)).w[0]
                                                  : ~0ull;
                        if (path == P_PC) {
                            const uint32_t off = offset_from_parts(seed(), N, off_tick, p, me);
                            deliver_pc(has(L_RUN) & !has(L_DEAD), c, mk, off);
                            F64_STAMP(4);
                            F64_COUNT(10);
                        } else if (path == P_PP) {
                            handle_preprepare_p(has(L_RUN) & (((mk >> j) & 1ull) != 0) & !has(L_DEAD), j, pp_h,
                                                blk_make(pp_h, j, 0, pp_T_out), pp_eq ? split_mask(pp_h) : 0ull);
                            F64_STAMP(3);
                            F64_COUNT(9);
                        } else {                                  // P_BLK
                            handle_blocks_p(has(L_RUN) & ((mk & kblk & ~(1ull << me)) != 0), blo, bhi);
                            F64_STAMP(5);
                            F64_COUNT(11);
                        }
                    }
                }
                const uint32_t xc = resolve_commits();
                F64_STAMP(6);
                if (frozen) act = false;
                // The block gossip phase after a commit, fused. When a Prepare/Commit phase ends with
                // every committer at height xc, the next phase would be a P_BLK phase with the range
                // [xc, xc] (chain_insert_core_p); if nothing else is in flight and every running
                // validator already has xc, handle_blocks_p is ChainError::Exists for all of them
                // (core.rs:75-82) and that phase reduces to its event step. Same phase index, same
                // miner step: bit-identical, without a second classification per height.
                if (((path == P_PC) | (path == P_CANON)) & (xc != 0) & act & (p + 1 < P.phase_cap)) {
                    if (ballot(((nxf & ~F_BLK) != 0) | (has(L_RUN) & (last < xc))) == 0) {
                        ++p;
                        nxf = 0;
                        miner_step_p();
                        F64_COUNT(8);
                        F64_COUNT(11);
                    }
                }
            }
            if (!seg_done && (frozen || canon_h >= P.heights)) { seg_done = true; done_tick = (uint32_t)tick + 1; }
        }
        if (!bailed) flush_rows();
#ifdef BFT_STAMPS
        F64_STAMP(7);
        if (me == 0 && P.stamps)
            for (int k = 0; k < NSTAMP; ++k) P.stamps[(uint64_t)inst_local * NSTAMP + k] = st_acc[k];
#endif
        // this wave's histograms → the launch totals: every height recorded here was a round-0 commit
        wv.sync();
        if (P.hist) {
            for (uint32_t b = me; b < 65u; b += 64u) {
                const uint32_t v = lat[b];
                if (v != 0) wv.gadd64(P.hist + 65u + b, v);
            }
            if (me == 0 && views_acc != 0) wv.gadd64(P.hist, views_acc);
        }
        uint32_t lf = lane_flags();
        for (uint32_t m = 1; m < 64u; m <<= 1) lf |= wv.shfl_xor(lf, (int)m);
        if (me == 0 && inst_local < P.n_instances && !bailed) {
            uint32_t flags = lf | seg_flags;
            if (!frozen && canon_h < P.heights) flags |= FLAG_TIMEOUT;
            P.committed_height[inst_local] = canon_h < P.heights ? canon_h : P.heights;
            P.flags[inst_local] = flags;
            P.ticks[inst_local] = done_tick;
            P.views[inst_local] = views_acc;
        }
    }
};

}  // namespace bft
