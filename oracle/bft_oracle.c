/*
 * bft_oracle.c — CPU ORACLE (test infrastructure only; see bft_oracle.h).
 *
 * Restates the consensus-rs PBFT core under the deterministic schedule of SPEC.md. One `val`
 * object per reference `Core` actor (src/consensus/pbft/core/core.rs:119-140) plus its chain
 * (src/core/chain.rs), miner (src/minner/mod.rs) and timer (core/timer.rs). Messages are handled
 * one at a time in the canonical delivery order, exactly like the reference handlers; every
 * function cites the reference file:line it follows. All paths are relative to /root/reference.
 *
 * Nothing here is optimised: it is the checker the HIP kernels are compared against.
 */
#include "bft_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <assert.h>

/* ------------------------------------------------------------------------------------------ */
/* Keccak-256 (the `hash` of cryptocurrency-kit, SPEC.md §7)                                   */
/* ------------------------------------------------------------------------------------------ */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static uint64_t rol64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

static void keccak_f(uint64_t A[25]) {
    for (int rnd = 0; rnd < 24; ++rnd) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol64(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                B[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(A[x + 5 * y], KROT[x + 5 * y]);
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= KRC[rnd];
    }
}

void orc_keccak256(const uint8_t *data, size_t len, uint8_t out[32]) {
    uint64_t A[25];
    memset(A, 0, sizeof A);
    const size_t rate = 136;
    uint8_t blk[136];
    size_t off = 0;
    for (;;) {
        size_t take = len - off < rate ? len - off : rate;
        memset(blk, 0, rate);
        memcpy(blk, data + off, take);
        int last = take < rate;
        if (last) {
            blk[take] ^= 0x01;
            blk[rate - 1] ^= 0x80;
        }
        for (int i = 0; i < 17; ++i) {
            uint64_t w = 0;
            for (int b = 0; b < 8; ++b) w |= (uint64_t)blk[8 * i + b] << (8 * b);
            A[i] ^= w;
        }
        keccak_f(A);
        off += take;
        if (last) break;
    }
    for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(A[i] >> (8 * b));
}

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11 / Random123) — the seeded schedule (SPEC.md §5)          */
/* ------------------------------------------------------------------------------------------ */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum { DOM_DROP = 1, DOM_SPLIT = 2, DOM_CRASH = 3, DOM_BYZ = 4, DOM_TX = 5, DOM_TX2 = 6 };

static void philox(uint64_t seed, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t out[4]) {
    uint32_t ctr[4] = {a, b, c, d};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    orc_philox4x32_10(ctr, key, out);
}

/* ------------------------------------------------------------------------------------------ */
/* Validator-set arithmetic (src/consensus/validator.rs)                                       */
/* ------------------------------------------------------------------------------------------ */
/* two_thirds_majority: floor(N * 2.0 / 3.0) in f32 (validator.rs:149-154) == (2N)/3. */
uint32_t orc_two_thirds_majority(uint32_t n) { return (2u * n) / 3u; }

/* randon_seed (validator.rs:39-48): U128(hash[0..8] ++ 0^8) mod N, U128 read big-endian,
 * i.e. (BE64(hash[0..8]) * 2^64) mod N. */
uint32_t orc_seed_from_hash(const uint8_t hash[32], uint32_t n) {
    unsigned __int128 v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | hash[i];
    v <<= 64;
    return (uint32_t)(v % n);
}
/* the same with the byte order of U128::from([u8; 16]) as a switch (bftsim.h BFTSIM_SEED_*):
 * little-endian reads seed_buf = hash[0..8] ++ 0^8 as LE64(hash[0..8]) + 0 * 2^64. */
uint32_t orc_seed_from_hash_order(const uint8_t hash[32], uint32_t n, uint32_t order) {
    if (order == 0) return orc_seed_from_hash(hash, n);
    unsigned __int128 v = 0;
    for (int i = 15; i >= 0; --i) v = (v << 8) | (i < 8 ? hash[i] : 0);
    return (uint32_t)(v % n);
}

/* ------------------------------------------------------------------------------------------ */
/* Header encoding + block hash (src/types/block.rs:16-36,76-84; SPEC.md §7)                   */
/* ------------------------------------------------------------------------------------------ */
static size_t mp_uint(uint8_t *o, uint64_t v) {
    if (v < 128) { o[0] = (uint8_t)v; return 1; }
    if (v < 256) { o[0] = 0xcc; o[1] = (uint8_t)v; return 2; }
    if (v < 65536) { o[0] = 0xcd; o[1] = (uint8_t)(v >> 8); o[2] = (uint8_t)v; return 3; }
    if (v < 4294967296ULL) {
        o[0] = 0xce;
        for (int i = 0; i < 4; ++i) o[1 + i] = (uint8_t)(v >> (24 - 8 * i));
        return 5;
    }
    o[0] = 0xcf;
    for (int i = 0; i < 8; ++i) o[1 + i] = (uint8_t)(v >> (56 - 8 * i));
    return 9;
}
static size_t mp_bytes_as_array(uint8_t *o, const uint8_t *b, size_t n) {
    size_t k = 0;
    if (n < 16) o[k++] = (uint8_t)(0x90 | n);
    else { o[k++] = 0xdc; o[k++] = (uint8_t)(n >> 8); o[k++] = (uint8_t)n; }
    for (size_t i = 0; i < n; ++i) k += mp_uint(o + k, b[i]);
    return k;
}
static size_t mp_address(uint8_t *o, const uint8_t a[20]) {
    static const char hx[] = "0123456789abcdef";
    size_t k = 0;
    o[k++] = 0xd9; o[k++] = 42; o[k++] = '0'; o[k++] = 'x';
    for (int i = 0; i < 20; ++i) { o[k++] = (uint8_t)hx[a[i] >> 4]; o[k++] = (uint8_t)hx[a[i] & 15]; }
    return k;
}

size_t orc_encode_header(uint8_t *o, const uint8_t prev_hash[32], const uint8_t proposer[20],
                         const uint8_t tx_hash[32], uint64_t height, uint64_t gas_limit,
                         uint64_t gas_used, uint64_t time, const uint8_t *extra, size_t extra_len) {
    static const uint8_t zero[32] = {0};
    size_t k = 0;
    o[k++] = 0x9d;                                  /* 13 serialized fields */
    k += mp_bytes_as_array(o + k, prev_hash, 32);   /* prev_hash */
    k += mp_address(o + k, proposer);               /* proposer */
    k += mp_bytes_as_array(o + k, zero, 32);        /* root */
    k += mp_bytes_as_array(o + k, tx_hash, 32);     /* tx_hash */
    k += mp_bytes_as_array(o + k, zero, 32);        /* receipt_hash */
    k += mp_uint(o + k, 0);                         /* bloom */
    k += mp_uint(o + k, 0);                         /* difficulty */
    k += mp_uint(o + k, height);
    k += mp_uint(o + k, gas_limit);
    k += mp_uint(o + k, gas_used);
    k += mp_uint(o + k, time);
    if (extra) k += mp_bytes_as_array(o + k, extra, extra_len);
    else o[k++] = 0xc0;
    o[k++] = 0xc0;                                  /* votes: None (block_hash, block.rs:76-80) */
    return k;
}

static const uint8_t GENESIS_EXTRA[] = "Hello Word!";   /* examples/c1.toml:18 */
static const uint8_t CAND_EXTRA[] = "Coinse base";      /* minner/mod.rs:113 */

void orc_genesis_hash(const orc_config *cfg, uint8_t out[32]) {
    static const uint8_t zero[32] = {0};
    uint8_t buf[512];
    /* store_genesis_block (core/genesis.rs:44-55) */
    size_t n = orc_encode_header(buf, zero, cfg->genesis_proposer, zero, 0, cfg->genesis_gas_used + 10,
                                 cfg->genesis_gas_used, cfg->genesis_time, GENESIS_EXTRA, 11);
    orc_keccak256(buf, n, out);
}

void orc_tx_hash(uint64_t seed, uint32_t instance, uint32_t height, uint32_t proposer,
                 uint32_t variant, uint8_t out[32]) {
    uint32_t w[8];
    philox(seed, instance, height, (proposer << 8) | variant, DOM_TX, w);
    philox(seed, instance, height, (proposer << 8) | variant, DOM_TX2, w + 4);
    for (int i = 0; i < 8; ++i)
        for (int b = 0; b < 4; ++b) out[4 * i + b] = (uint8_t)(w[i] >> (8 * b));
}

/* ------------------------------------------------------------------------------------------ */
/* Seeded schedule pieces (SPEC.md §3, §5, §6)                                                 */
/* ------------------------------------------------------------------------------------------ */
typedef struct { uint64_t w[4]; } bits;
static int bits_get(const bits *b, uint32_t i) { return (int)((b->w[i >> 6] >> (i & 63)) & 1); }
static void bits_set(bits *b, uint32_t i) { b->w[i >> 6] |= 1ULL << (i & 63); }
static int bits_count(const bits *b) {
    return __builtin_popcountll(b->w[0]) + __builtin_popcountll(b->w[1]) +
           __builtin_popcountll(b->w[2]) + __builtin_popcountll(b->w[3]);
}
static int bits_union_count(const bits *a, const bits *b) {
    int c = 0;
    for (int i = 0; i < 4; ++i) c += __builtin_popcountll(a->w[i] | b->w[i]);
    return c;
}

void orc_byz_mask(const orc_config *cfg, uint32_t instance, uint64_t out[4]) {
    uint32_t perm[ORC_MAX_N];
    uint32_t n = cfg->n;
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    memset(out, 0, 4 * sizeof(uint64_t));
    uint32_t f = cfg->byz_count < n ? cfg->byz_count : n;
    for (uint32_t i = 0; i < f; ++i) {
        uint32_t w[4];
        philox(cfg->seed, instance, i, 0, DOM_BYZ, w);
        uint32_t j = i + w[0] % (n - i);
        uint32_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
        out[perm[i] >> 6] |= 1ULL << (perm[i] & 63);
    }
}

static uint32_t thr16(uint32_t ppm) { return (uint32_t)(((uint64_t)ppm * 65536u + 500000u) / 1000000u); }
static uint32_t thr32(uint32_t ppm) { return (uint32_t)(((uint64_t)ppm << 32) / 1000000u); }

void orc_deliver_mask(const orc_config *cfg, uint32_t instance, uint32_t tick, uint32_t phase,
                      uint32_t receiver, uint64_t out[4]) {
    uint32_t n = cfg->n;
    memset(out, 0, 4 * sizeof(uint64_t));
    if (cfg->drop_ppm == 0) {
        for (uint32_t s = 0; s < n; ++s) out[s >> 6] |= 1ULL << (s & 63);
        return;
    }
    uint32_t t = thr16(cfg->drop_ppm);
    for (uint32_t j = 0; 8 * j < n; ++j) {
        uint32_t w[4];
        philox(cfg->seed, instance, tick, (phase << 24) | (receiver << 8) | j, DOM_DROP, w);
        for (uint32_t i = 0; i < 8 && 8 * j + i < n; ++i) {
            uint32_t u = (w[i >> 1] >> (16 * (i & 1))) & 0xffffu;
            uint32_t s = 8 * j + i;
            if (u >= t) out[s >> 6] |= 1ULL << (s & 63);
        }
    }
    out[receiver >> 6] |= 1ULL << (receiver & 63);   /* gossip self-delivery (backend.rs:150) */
}

/* lowbias32 (C. Wellons' integer hash) — cheap per-phase randomness (SPEC.md §3) */
static uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
/* first sender in the receiver's delivery order of (tick, phase): arrival order is a seeded
 * rotation of the sender indices, standing in for random link latencies (SPEC.md §3) */
static uint32_t delivery_offset(const orc_config *cfg, uint32_t instance, uint32_t tick,
                                uint32_t phase, uint32_t receiver) {
    uint32_t h = lowbias32(instance ^ (uint32_t)cfg->seed);
    h = lowbias32(h ^ tick);
    h = lowbias32(h ^ ((phase << 16) | receiver) ^ (uint32_t)(cfg->seed >> 32));
    return (uint32_t)(((uint64_t)h * cfg->n) >> 32);
}

static int split_bit(const orc_config *cfg, uint32_t instance, uint32_t h, uint32_t r, uint32_t v) {
    uint32_t w[4];
    philox(cfg->seed, instance, h, r, DOM_SPLIT | ((v >> 7) << 8), w);
    uint32_t vv = v & 127;
    return (int)((w[vv >> 5] >> (vv & 31)) & 1);
}

static int proposer_crashed(const orc_config *cfg, uint32_t instance, uint32_t h, uint32_t r) {
    if (cfg->proposer_crash_ppm == 0) return 0;
    uint32_t w[4];
    philox(cfg->seed, instance, h, r, DOM_CRASH, w);
    return w[0] < thr32(cfg->proposer_crash_ppm);
}

/* ------------------------------------------------------------------------------------------ */
/* Model state                                                                                */
/* ------------------------------------------------------------------------------------------ */
/* Block identity (SPEC.md §4): (height, proposer, variant); valid==0 is Option::None. */
typedef struct { uint32_t h; uint16_t prop; uint8_t var; uint8_t valid; int64_t T; } blk;
/* T = the candidate's time tick (header.time = genesis_time + period*(T+1)); it is a function of
 * (h, prop) because a validator mines one candidate per height, so equality ignores it. */
static const blk NONE_BLK = {0, 0, 0, 0, 0};
static int blk_eq(blk a, blk b) {
    return a.valid && b.valid && a.h == b.h && a.prop == b.prop && a.var == b.var;
}
/* digest comparison; a Byzantine vote's wildcard digest matches both variants (SPEC.md §6) */
static int digest_match(blk d, int wild, blk target) {
    if (!d.valid || !target.valid) return 0;
    if (d.h != target.h || d.prop != target.prop) return 0;
    return wild || d.var == target.var;
}

/* State enum, src/protocol/mod.rs:25-30 */
enum { ST_ACCEPT_REQUEST = 1, ST_PREPREPARED = 2, ST_PREPARED = 3, ST_COMMITTED = 4 };
/* MessageType, src/protocol/mod.rs:36-41 */
enum { MT_PREPREPARE = 1, MT_PREPARE = 2, MT_COMMIT = 3, MT_ROUND_CHANGE = 4 };
/* the ConsensusError classes that decide what happens next (consensus/error.rs:12-39) */
enum { E_OK = 0, E_UNKNOWN, E_FUTURE_BLOCK, E_OLD, E_FUTURE_MSG };

typedef struct {
    uint8_t has_pp, pp_equiv;
    uint32_t pp_h, pp_r;
    blk pp_blk;
    uint8_t has_pr, pr_wild;
    uint32_t pr_h, pr_r;
    blk pr_d;
    uint8_t has_cm, cm_wild;
    uint32_t cm_h, cm_r;
    blk cm_d;
    uint8_t has_ocm, ocm_wild;
    uint32_t ocm_h, ocm_r;
    blk ocm_d;
    uint8_t has_rc;
    uint32_t rc_h, rc_r;
    uint8_t has_sync;
    uint32_t sync_h;
    uint32_t blk_lo, blk_hi; /* blk_lo == 0: none */
} outbox;

typedef struct { uint32_t round; bits set; } rc_entry;

/* a stored FutureMessage / FutureRoundMessage (backlog replay mode, SPEC.md §10) */
typedef struct { uint8_t valid, code, wild; uint32_t vh, vr; blk d; } bl_entry;
#define RCS_MAX 64

typedef struct {
    int running, core_dead, byz;
    /* Core (core.rs:119-140) + RoundState (round_state.rs:12-22) */
    uint32_t h, r;
    int st, wait;
    blk lock, pp, pend;
    bits prep, comm;
    rc_entry rcs[RCS_MAX];
    int n_rcs;
    uint32_t proposer;        /* ImplValidatorSet.proposer (index); UINT32_MAX = None */
    /* chain (ledger) tip */
    uint32_t last;
    /* timers (core.rs:643-657) and limiter (round_change.rs:39-44) */
    int64_t timer_tick, rc_last_tick;
    /* miner (minner/mod.rs) */
    uint32_t mint_height, miner_queue;
    int64_t wake_tick;
    blk cand;
    /* delayed sync check (core.rs:58-69) */
    uint32_t sync_pending;
    /* gossip outbound cache: last subject sent per kind (backend.rs:141-148) */
    uint32_t s_pp_h, s_pp_r; blk s_pp_b; int s_pp_valid;
    uint32_t s_pr_h, s_pr_r; blk s_pr_d; int s_pr_valid;
    uint32_t s_cm_h, s_cm_r; blk s_cm_d; int s_cm_valid;
    uint32_t s_ocm_h, s_ocm_r; blk s_ocm_d; int s_ocm_valid;
    outbox next, cur;
    bl_entry *bl;             /* [n] per-sender backlog slots (backlog replay mode only) */
} val;

typedef struct {
    int set;
    blk b;
    uint32_t round;
    int64_t T;           /* time tick */
    uint8_t hash[32];
    uint32_t seed;
    int64_t commit_tick; /* tick of the phase that recorded it (commit-latency histogram) */
} canon_entry;

typedef struct {
    const orc_config *cfg;
    uint32_t inst, n, q;   /* q = two_thirds_majority() (strict ">" tests) */
    val *v;
    canon_entry *canon;
    uint32_t canon_cap, canon_h;
    int64_t tick;
    uint32_t flags;
    int frozen;
    /* real-crypto mode (SPEC.md §11): the broadcast log of this instance and the forged senders */
    const uint64_t *forged;
    uint32_t *mlog;        /* [mlog_cap][8] */
    uint32_t mlog_cap, mlog_n;
} world;

static canon_entry *canon_at(world *w, uint32_t x) { return &w->canon[x]; }

/* ------------------------------------------------------------------------------------------ */
/* Outbox (Backend::gossip, backend.rs:140-160, and TcpServer::broadcast, server.rs:376-389)    */
/* ------------------------------------------------------------------------------------------ */
static void out_preprepare(world *w, val *v, uint32_t h, uint32_t r, blk b, int equiv) {
    if (v->s_pp_valid && v->s_pp_h == h && v->s_pp_r == r && blk_eq(v->s_pp_b, b)) return;
    v->s_pp_valid = 1; v->s_pp_h = h; v->s_pp_r = r; v->s_pp_b = b;
    if (v->next.has_pp) { w->flags |= ORC_FLAG_OUTBOX; return; }
    v->next.has_pp = 1; v->next.pp_h = h; v->next.pp_r = r; v->next.pp_blk = b; v->next.pp_equiv = (uint8_t)equiv;
}
static void out_prepare(world *w, val *v, uint32_t h, uint32_t r, blk d, int wild) {
    if (v->s_pr_valid && v->s_pr_h == h && v->s_pr_r == r && blk_eq(v->s_pr_d, d)) return;
    v->s_pr_valid = 1; v->s_pr_h = h; v->s_pr_r = r; v->s_pr_d = d;
    if (v->next.has_pr) { w->flags |= ORC_FLAG_OUTBOX; return; }
    v->next.has_pr = 1; v->next.pr_h = h; v->next.pr_r = r; v->next.pr_d = d; v->next.pr_wild = (uint8_t)wild;
}
static void out_commit(world *w, val *v, uint32_t h, uint32_t r, blk d, int wild) {
    if (v->s_cm_valid && v->s_cm_h == h && v->s_cm_r == r && blk_eq(v->s_cm_d, d)) return;
    v->s_cm_valid = 1; v->s_cm_h = h; v->s_cm_r = r; v->s_cm_d = d;
    if (v->next.has_cm) { w->flags |= ORC_FLAG_OUTBOX; return; }
    v->next.has_cm = 1; v->next.cm_h = h; v->next.cm_r = r; v->next.cm_d = d; v->next.cm_wild = (uint8_t)wild;
}
static void out_old_commit(world *w, val *v, uint32_t h, uint32_t r, blk d, int wild) {
    if (v->s_ocm_valid && v->s_ocm_h == h && v->s_ocm_r == r && blk_eq(v->s_ocm_d, d)) return;
    v->s_ocm_valid = 1; v->s_ocm_h = h; v->s_ocm_r = r; v->s_ocm_d = d;
    if (v->next.has_ocm) { w->flags |= ORC_FLAG_OUTBOX; return; }
    v->next.has_ocm = 1; v->next.ocm_h = h; v->next.ocm_r = r; v->next.ocm_d = d; v->next.ocm_wild = (uint8_t)wild;
}
static void out_round_change(world *w, val *v, uint32_t h, uint32_t r) {
    /* create_time = now_millis (round_change.rs:61): never deduplicated */
    if (v->next.has_rc) { w->flags |= ORC_FLAG_OUTBOX; return; }
    v->next.has_rc = 1; v->next.rc_h = h; v->next.rc_r = r;
}
static void out_sync(world *w, val *v, uint32_t height) {
    /* ChainEvent::SyncBlock → BroadcastEvent::Sync (server.rs:201-208, 226-228) */
    (void)w;
    if (v->next.has_sync) {   /* requests of one phase coalesce to the lowest height */
        if (height < v->next.sync_h) v->next.sync_h = height;
        return;
    }
    v->next.has_sync = 1; v->next.sync_h = height;
}
static void out_blocks(val *v, uint32_t lo, uint32_t hi) {
    /* ChainEvent::NewBlock / PostBlock → BroadcastEvent::Blocks (server.rs:186-194, 222-231);
     * one coalesced ascending range per sender and phase (SPEC.md §2) */
    if (lo > hi) return;
    if (v->next.blk_lo == 0) { v->next.blk_lo = lo; v->next.blk_hi = hi; return; }
    if (lo < v->next.blk_lo) v->next.blk_lo = lo;
    if (hi > v->next.blk_hi) v->next.blk_hi = hi;
}

/* ------------------------------------------------------------------------------------------ */
/* Chain + miner                                                                              */
/* ------------------------------------------------------------------------------------------ */
static void canon_record(world *w, uint32_t x, blk b, uint32_t round);

static uint32_t seed_at(world *w, uint32_t x) { return canon_at(w, x)->seed; }

/* new_round_change_timer (core.rs:643-657): one-shot 3 s timer → next tick */
static void new_round_change_timer(world *w, val *v) { v->timer_tick = w->tick + 1; }
/* stop_timer (core.rs:638-641) */
static void stop_timer(val *v) { v->timer_tick = -1; }

/* Chain::insert_block (core/chain.rs:45-71). via_core: called from Backend::commit. */
static int chain_insert(world *w, val *v, blk b, int via_core) {
    if (b.h <= v->last) return 1;                  /* ChainError::Exists (chain.rs:50-52) */
    if (v->last + 1 < b.h) {                       /* Not found ancestor (chain.rs:53-57) */
        out_sync(w, v, v->last + 1);
        return 2;
    }
    canon_entry *c = canon_at(w, b.h);
    if (c->set) {
        if (!blk_eq(c->b, b)) { w->flags |= ORC_FLAG_SAFETY; w->frozen = 1; return 3; }
    } else {
        assert(via_core);   /* gossip only carries blocks that are already in some chain */
        canon_record(w, b.h, b, v->r);
    }
    v->last = b.h;
    out_blocks(v, b.h, b.h);                       /* ChainEvent::NewBlock (chain.rs:61) */
    if (b.h > v->miner_queue) v->miner_queue = b.h;/* ChainEvent::NewHeader (chain.rs:62) */
    return 0;
}

static void handle_new_header_event(world *w, val *v);

/* Minner::mine + packet_next_block + next_block + Engine::seal (minner/mod.rs:95-143,
 * backend.rs:428-454) */
static void miner_mine(world *w, val *v) {
    uint32_t x = v->last + 1;
    int64_t tparent = canon_at(w, v->last)->T;
    int64_t T = w->tick > tparent + 1 ? w->tick : tparent + 1;
    v->cand.h = x; v->cand.prop = (uint16_t)(v - w->v); v->cand.var = 0; v->cand.valid = 1;
    v->cand.T = T;                    /* header.time (block.rs:82-84) */
    v->mint_height = x;
    v->wake_tick = T;
    if (T > w->tick) return;          /* seal sleeps until header.time (backend.rs:437-449) */
    v->wake_tick = -1;
    handle_new_header_event(w, v);    /* zero delay: NewHeaderEvent now */
}

/* Minner: Handler<ChainEvent::NewHeader> (minner/mod.rs:56-69) */
static void miner_step(world *w, val *v) {
    if (v->wake_tick >= 0) return;                 /* blocked in seal's sleep */
    uint32_t q = v->miner_queue;
    v->miner_queue = 0;
    if (q != 0 && q >= v->mint_height) miner_mine(w, v);
}

/* ------------------------------------------------------------------------------------------ */
/* Core (src/consensus/pbft/core/ *.rs)                                                        */
/* ------------------------------------------------------------------------------------------ */
static uint32_t vidx(world *w, val *v) { return (uint32_t)(v - w->v); }
static int is_proposer(val *v, uint32_t who) { return v->proposer == who; }

/* Core::check_message (core.rs:366-399) */
static int check_message(val *v, int code, uint32_t vh) {
    if (vh == 0) return E_UNKNOWN;
    if (code == MT_ROUND_CHANGE) {
        if (vh > v->h) return E_FUTURE_BLOCK;
        if (vh < v->h) return E_OLD;
        return E_OK;
    }
    if (vh > v->h) return E_FUTURE_BLOCK;
    if (vh < v->h) return E_OLD;
    if (v->st == ST_ACCEPT_REQUEST) {
        if (code > MT_PREPREPARE) return E_FUTURE_MSG;
        return E_OK;
    }
    return E_OK;
}

int orc_check_message(int code, uint32_t msg_height, uint32_t core_height, int state) {
    val v;
    memset(&v, 0, sizeof v);
    v.h = core_height;
    v.st = state;
    return check_message(&v, code, msg_height);
}

/* handle_msg_middle: FutureBlockMessage(h) → SyncBlock after 1 s (core.rs:58-69) */
static void note_future_block(val *v, uint32_t vh) { if (vh > v->sync_pending) v->sync_pending = vh; }

/* RoundState::lock_hash (round_state.rs:100-110) */
static void lock_hash(val *v) { if (v->pp.valid) v->lock = v->pp; }

/* HandlePreprepare::send_preprepare (preprepare.rs:30-43) */
static void send_preprepare(world *w, val *v, blk req) {
    uint32_t me = vidx(w, v);
    if (v->h == req.h && is_proposer(v, me)) {
        if (proposer_crashed(w->cfg, w->inst, v->h, v->r)) return;   /* cfg4 proposer crash */
        int equiv = v->byz && req.prop == me && req.var == 0;       /* SPEC.md §6 */
        out_preprepare(w, v, v->h, v->r, req, equiv);
    }
}

/* HandlePrepare::send_prepare (prepare.rs:28-38) */
static void send_prepare(world *w, val *v) {
    out_prepare(w, v, v->h, v->r, v->pp, v->byz);
    if (v->byz) out_commit(w, v, v->h, v->r, v->pp, 1);            /* SPEC.md §6 */
}

/* HandleCommit::send_commit → broadcast_commit (commit.rs:37-43,54-60) */
static void send_commit(world *w, val *v) {
    assert(v->pp.valid);   /* current_state.proposal().unwrap() */
    out_commit(w, v, v->h, v->r, v->pp, v->byz);
}

/* Core::catchup_round (core.rs:555-565) */
static void catchup_round(world *w, val *v) { v->wait = 1; new_round_change_timer(w, v); }

/* HandleRoundChange::send_round_change (round_change.rs:38-63) */
static void send_round_change(world *w, val *v, uint32_t round) {
    if (v->rc_last_tick == w->tick) {   /* 50 ms limiter */
        new_round_change_timer(w, v);
        return;
    }
    v->rc_last_tick = w->tick;
    if (v->r < round) catchup_round(w, v);
    out_round_change(w, v, v->h, round);
}

/* RoundChangeSet::max_round (round_change_set.rs:64-74), ascending-round iteration */
static uint32_t rcs_max_round(val *v) {
    uint32_t max = 0;
    int total = 0;
    for (int i = 0; i < v->n_rcs; ++i) {
        int len = bits_count(&v->rcs[i].set);
        if (len >= total && v->rcs[i].round > max) { max = v->rcs[i].round; total = len; }
    }
    return max;
}
/* RoundChangeSet::add (round_change_set.rs:28-35) */
static int rcs_add(val *v, uint32_t round, uint32_t sender) {
    int i = 0;
    while (i < v->n_rcs && v->rcs[i].round < round) ++i;
    if (i == v->n_rcs || v->rcs[i].round != round) {
        assert(v->n_rcs < RCS_MAX);
        memmove(&v->rcs[i + 1], &v->rcs[i], (size_t)(v->n_rcs - i) * sizeof(rc_entry));
        memset(&v->rcs[i], 0, sizeof(rc_entry));
        v->rcs[i].round = round;
        v->n_rcs++;
    }
    bits_set(&v->rcs[i].set, sender);
    return bits_count(&v->rcs[i].set);
}

/* HandleRoundChange::send_next_round_change (round_change.rs:26-36) */
static void send_next_round_change(world *w, val *v) {
    uint32_t round = rcs_max_round(v);
    if (round <= v->r) send_round_change(w, v, v->r + 1);
    else send_round_change(w, v, round);
}

/* Core::start_new_zero_round (core.rs:441-470) */
static void start_new_zero_round(world *w, val *v) {
    uint32_t last_height = v->last;
    v->h = last_height + 1;
    v->r = 0;
    v->n_rcs = 0;
    /* update_round_state(.., false) (core.rs:597-600) */
    v->lock = NONE_BLK; v->pp = NONE_BLK; v->pend = NONE_BLK;
    memset(&v->prep, 0, sizeof(bits)); memset(&v->comm, 0, sizeof(bits));
    v->proposer = (seed_at(w, last_height) + 0) % w->n;   /* calc_proposer (validator.rs:74-77) */
    v->wait = 0;
    v->st = ST_ACCEPT_REQUEST;
    new_round_change_timer(w, v);
}

/* Core::start_new_round (core.rs:474-551) */
static void start_new_round(world *w, val *v, uint32_t round) {
    assert(round != 0 && round > v->r);
    uint32_t last_height = v->last;
    assert(!(last_height + 1 < v->h));
    if (last_height > v->h) return;                /* catch-up (core.rs:492-496) */
    v->n_rcs = 0;                                  /* RoundChangeSet::new (core.rs:516) */
    /* update_round_state(view, vals, true) (core.rs:577-596) */
    if (!v->lock.valid) v->pp = NONE_BLK;          /* lock, preprepare carried iff locked */
    memset(&v->prep, 0, sizeof(bits)); memset(&v->comm, 0, sizeof(bits));
    v->r = round;
    v->proposer = (seed_at(w, last_height) + round) % w->n;
    v->wait = 0;
    v->st = ST_ACCEPT_REQUEST;
    if (is_proposer(v, vidx(w, v))) {
        if (v->lock.valid) {
            send_preprepare(w, v, v->pp);
        } else {
            if (!v->pend.valid) {                  /* pending_request.as_ref().unwrap() panics */
                v->core_dead = 1;
                w->flags |= ORC_FLAG_CORE_PANIC;
                return;
            }
            send_preprepare(w, v, v->pend);
        }
    }
    new_round_change_timer(w, v);
}

/* Handler<NewHeaderEvent> (core.rs:154-163) + HandlerRequest::handle (request.rs:19-42) */
static void handle_new_header_event(world *w, val *v) {
    if (v->core_dead) return;                      /* mailbox of a dead actor */
    start_new_zero_round(w, v);
    blk req = v->cand;
    if (v->h > req.h) return;                      /* OldMessage */
    if (v->h < req.h) return;                      /* FutureMessage */
    assert(v->st == ST_ACCEPT_REQUEST);
    v->pend = req;                                 /* accept */
    send_preprepare(w, v, req);
}

/* Handler<TimerEvent> (core.rs:207-225) */
static void handle_timer_event(world *w, val *v) {
    if (v->last >= v->h) {
        stop_timer(v);
        v->wait = 0;
    } else {
        send_next_round_change(w, v);
    }
}

/* Core::commit (core.rs:402-422) → Backend::commit (backend.rs:163-200) */
static void core_commit(world *w, val *v) {
    v->st = ST_COMMITTED;
    assert(bits_count(&v->comm) >= (int)w->q + 1);
    chain_insert(w, v, v->pp, 1);
}

/* HandlePreprepare::handle (preprepare.rs:45-126) */
static void handle_preprepare(world *w, val *v, uint32_t src, const outbox *m) {
    uint32_t me = vidx(w, v);
    blk b = m->pp_blk;
    if (m->pp_equiv && me != src && split_bit(w->cfg, w->inst, m->pp_h, m->pp_r, me)) b.var = 1;
    int res = check_message(v, MT_PREPREPARE, m->pp_h);
    if (res != E_OK) {
        if (res == E_OLD) {
            if (b.h > v->last) return;                                  /* InvalidProposal */
            if (!blk_eq(canon_at(w, b.h)->b, b)) return;                /* InvalidProposal */
            uint32_t pre_height = b.h - 1;
            uint32_t old_prop = (seed_at(w, pre_height) + m->pp_r) % w->n;
            if (old_prop == src) out_old_commit(w, v, m->pp_h, m->pp_r, b, v->byz);
            /* falls through (preprepare.rs:52-74) */
        } else if (res == E_FUTURE_BLOCK) {
            /* falls through (preprepare.rs:75-78) */
        } else {
            return;
        }
    }
    if (!is_proposer(v, src)) return;                                   /* NotFromProposer */
    /* Backend::verify → verify_header (backend.rs:203-242, 319-341) */
    if (b.h == 0 || b.h - 1 > v->last) {                                /* UnknownAncestor */
        send_next_round_change(w, v);
        return;
    }
    if (v->st == ST_ACCEPT_REQUEST) {
        if (v->lock.valid) {
            if (blk_eq(b, v->lock)) {
                v->pp = b;                                              /* accetp */
                v->st = ST_PREPARED;
                send_commit(w, v);
            } else {
                send_next_round_change(w, v);
            }
        } else {
            v->pp = b;
            v->st = ST_PREPREPARED;
            send_prepare(w, v);
        }
    }
}

/* BackLogActor::handle (back_log.rs:38-65): the first message per sender is kept (or_insert_with);
 * reached from handle_check_message on FutureMessage / FutureRoundMessage (core.rs:353-358). The
 * reference never re-delivers it (process_back_log only iterates), so outside replay mode it is dropped. */
static void backlog_store(world *w, val *v, uint32_t src, int code, uint32_t vh, uint32_t vr, blk d, int wild) {
    if (!w->cfg->backlog_mode) return;
    bl_entry *e = &v->bl[src];
    if (e->valid) return;
    e->valid = 1; e->code = (uint8_t)code; e->wild = (uint8_t)wild; e->vh = vh; e->vr = vr; e->d = d;
}

/* HandlePrepare::handle (prepare.rs:48-66) */
static void handle_prepare(world *w, val *v, uint32_t src, const outbox *m) {
    int res = check_message(v, MT_PREPARE, m->pr_h);
    if (res != E_OK) {
        if (res == E_FUTURE_BLOCK) note_future_block(v, m->pr_h);
        else if (res == E_FUTURE_MSG) backlog_store(w, v, src, MT_PREPARE, m->pr_h, m->pr_r, m->pr_d, m->pr_wild);
        return;
    }
    if (m->pr_h != v->h || m->pr_r != v->r) return;                     /* InconsistentSubject */
    bits_set(&v->prep, src);                                            /* accept */
    if (v->lock.valid && digest_match(m->pr_d, m->pr_wild, v->lock)) {
        lock_hash(v);
        v->st = ST_PREPARED;
        send_commit(w, v);
    }
    if (bits_union_count(&v->prep, &v->comm) > (int)w->q) {             /* get_prepare_or_commit_size */
        lock_hash(v);
        v->st = ST_PREPARED;
        send_commit(w, v);
    }
}

/* HandleCommit::handle + verify_commit (commit.rs:63-111) */
static void handle_commit_msg(world *w, val *v, uint32_t src, uint32_t vh, uint32_t vr, blk d, int wild) {
    int res = check_message(v, MT_COMMIT, vh);
    if (res != E_OK) {
        if (res == E_FUTURE_BLOCK) note_future_block(v, vh);
        else if (res == E_FUTURE_MSG) backlog_store(w, v, src, MT_COMMIT, vh, vr, d, wild);
        return;
    }
    assert(v->pp.valid);                                                /* subject().unwrap() */
    if (!digest_match(d, wild, v->pp) || vh != v->h || vr != v->r) return;
    bits_set(&v->comm, src);
    if (bits_count(&v->comm) > (int)w->q && v->st < ST_COMMITTED) {
        lock_hash(v);
        core_commit(w, v);
    }
}

/* HandleRoundChange::handle (round_change.rs:65-98) */
static void handle_round_change_v(world *w, val *v, uint32_t src, uint32_t vh, uint32_t mr) {
    int res = check_message(v, MT_ROUND_CHANGE, vh);
    if (res != E_OK) { if (res == E_FUTURE_BLOCK) note_future_block(v, vh); return; }
    if (v->r > mr && mr > 0) {
        send_round_change(w, v, mr);
        return;
    }
    int n = rcs_add(v, mr, src);
    if (n >= (int)w->q + 1 && v->wait && v->r < mr) {
        send_round_change(w, v, mr);
        start_new_round(w, v, mr);
        return;
    }
    if (v->wait && v->r < mr)   /* FutureRoundMessage (round_change.rs:93-96) → backlog */
        backlog_store(w, v, src, MT_ROUND_CHANGE, vh, mr, NONE_BLK, 0);
}
static void handle_round_change(world *w, val *v, uint32_t src, const outbox *m) {
    handle_round_change_v(w, v, src, m->rc_h, m->rc_r);
}

/* Backlog replay (SPEC.md §10): the stored messages in ascending sender order, each slot emptied and
 * the message handled as a BackLogEvent (core.rs:197-204 → handle_check_message); one that is again a
 * FutureMessage / FutureRoundMessage is stored again. */
static void backlog_replay(world *w, val *v) {
    for (uint32_t s = 0; s < w->n; ++s) {
        bl_entry *e = &v->bl[s];
        if (!e->valid) continue;
        bl_entry m = *e;
        e->valid = 0;
        if (v->core_dead) return;
        if (m.code == MT_PREPARE) {
            outbox o;
            memset(&o, 0, sizeof o);
            o.has_pr = 1; o.pr_h = m.vh; o.pr_r = m.vr; o.pr_d = m.d; o.pr_wild = m.wild;
            handle_prepare(w, v, s, &o);
        } else if (m.code == MT_COMMIT) {
            handle_commit_msg(w, v, s, m.vh, m.vr, m.d, m.wild);
        } else {
            handle_round_change_v(w, v, s, m.vh, m.vr);
        }
        if (w->frozen) return;
    }
}

/* handle_msg_middle Block branch (core.rs:75-82) */
static void handle_blocks(world *w, val *v, uint32_t lo, uint32_t hi) {
    for (uint32_t x = lo; x <= hi; ++x) {
        chain_insert(w, v, canon_at(w, x)->b, 0);
        if (w->frozen) return;
    }
}

/* handle_msg_middle Sync branch (core.rs:83-110) */
static void handle_sync(val *v, uint32_t height) {
    if (height > v->last) return;
    uint32_t hi = v->last < height + 101 ? v->last : height + 101;
    out_blocks(v, height, hi);
}

/* ------------------------------------------------------------------------------------------ */
/* Canonical chain bookkeeping (first writer per height) + hashing                             */
/* ------------------------------------------------------------------------------------------ */
static void set_hash(world *w, uint32_t x);

static void canon_record(world *w, uint32_t x, blk b, uint32_t round) {
    canon_entry *c = canon_at(w, x);
    assert(x < w->canon_cap);
    c->set = 1;
    c->b = b;
    c->round = round;
    c->T = b.T;
    c->commit_tick = w->tick;
    set_hash(w, x);    /* the next height's proposer seed needs it at once */
    if (x > w->canon_h) w->canon_h = x;
}

/* ------------------------------------------------------------------------------------------ */
/* Driver                                                                                     */
/* ------------------------------------------------------------------------------------------ */
static int outbox_empty(const outbox *o) {
    return !(o->has_pp || o->has_pr || o->has_cm || o->has_ocm || o->has_rc || o->has_sync || o->blk_lo);
}

static void deliver_phase(world *w, uint32_t phase) {
    uint32_t n = w->n;
    for (uint32_t r = 0; r < n; ++r) {
        val *v = &w->v[r];
        if (!v->running) continue;
        miner_step(w, v);                               /* event step */
        if (w->frozen) return;
        if (w->cfg->backlog_mode) {                     /* backlog replay (SPEC.md §10) */
            backlog_replay(w, v);
            if (w->frozen) return;
        }
        uint64_t mk[4];
        orc_deliver_mask(w->cfg, w->inst, (uint32_t)w->tick, phase, r, mk);
        bits dm;
        memcpy(dm.w, mk, sizeof mk);
        /* sender-major delivery: each sender's messages of this phase together, senders in
         * the receiver's rotated order; per sender Blocks, Sync, Preprepare, Prepare, old Commit, Commit,
         * RoundChange (SPEC.md §2) */
        uint32_t off = delivery_offset(w->cfg, w->inst, (uint32_t)w->tick, phase, r);
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t s = off + k < n ? off + k : off + k - n;
            if (!bits_get(&dm, s)) continue;
            const outbox *m = &w->v[s].cur;
            if (s != r && m->blk_lo) {                  /* p2p Blocks: not self-delivered */
                handle_blocks(w, v, m->blk_lo, m->blk_hi);
                if (w->frozen) return;
            }
            if (s != r && m->has_sync) handle_sync(v, m->sync_h);
            if (v->core_dead) continue;
            if (m->has_pp) { handle_preprepare(w, v, s, m); if (v->core_dead) continue; }
            if (m->has_pr) handle_prepare(w, v, s, m);
            if (m->has_ocm) handle_commit_msg(w, v, s, m->ocm_h, m->ocm_r, m->ocm_d, m->ocm_wild);
            if (w->frozen) return;
            if (m->has_cm) handle_commit_msg(w, v, s, m->cm_h, m->cm_r, m->cm_d, m->cm_wild);
            if (w->frozen) return;
            if (m->has_rc) handle_round_change(w, v, s, m);
        }
    }
}

static int pending_local(world *w) {
    for (uint32_t i = 0; i < w->n; ++i) {
        val *v = &w->v[i];
        if (!v->running) continue;
        if (!outbox_empty(&v->next)) return 1;
        if (v->wake_tick < 0 && v->miner_queue != 0 && v->miner_queue >= v->mint_height) return 1;
    }
    return 0;
}

/* SPEC.md §11: at the start of a phase the consensus messages of every outbox are broadcast (signed,
 * core.rs:425-429) in (sender, kind) order; a forged sender's messages are dropped by every receiver
 * (handle_message, core.rs:314-322), so they leave the outbox */
static uint64_t blk_pack(blk b) {
    if (!b.valid) return 0;
    return (uint64_t)(b.h & 0xffffffu) | ((uint64_t)(b.prop & 0x1ffu) << 24) | ((uint64_t)(b.var & 1u) << 33) |
           (1ull << 34) | ((uint64_t)b.T << 35);
}
static void mlog_put(world *w, uint32_t phase, uint32_t sender, uint32_t code, uint32_t h, uint32_t r, uint64_t b,
                     uint32_t fl) {
    uint32_t idx = w->mlog_n++;
    if (idx >= w->mlog_cap) return;
    uint32_t *e = w->mlog + (size_t)idx * 8;
    e[0] = (uint32_t)w->tick; e[1] = phase | (code << 8) | (sender << 16); e[2] = h; e[3] = r;
    e[4] = (uint32_t)b; e[5] = (uint32_t)(b >> 32); e[6] = fl; e[7] = 0;
}
static void crypto_log(world *w, uint32_t sender, outbox *o, uint32_t phase) {
    int forged = (int)((w->forged[sender >> 6] >> (sender & 63)) & 1);
    uint32_t ff = forged ? 1u : 0u;                        /* MLOG_FORGED, WILD 2, EQUIV 4, OLD 8 */
    if (o->has_pp) mlog_put(w, phase, sender, 1, o->pp_h, o->pp_r, blk_pack(o->pp_blk), ff | (o->pp_equiv ? 4u : 0u));
    if (o->has_pr) mlog_put(w, phase, sender, 2, o->pr_h, o->pr_r, blk_pack(o->pr_d), ff | (o->pr_wild ? 2u : 0u));
    if (o->has_ocm) mlog_put(w, phase, sender, 3, o->ocm_h, o->ocm_r, blk_pack(o->ocm_d), ff | 8u | (o->ocm_wild ? 2u : 0u));
    if (o->has_cm) mlog_put(w, phase, sender, 3, o->cm_h, o->cm_r, blk_pack(o->cm_d), ff | (o->cm_wild ? 2u : 0u));
    if (o->has_rc) mlog_put(w, phase, sender, 4, o->rc_h, o->rc_r, 0, ff);
    if (forged) o->has_pp = o->has_pr = o->has_ocm = o->has_cm = o->has_rc = 0;
}

static void run_tick(world *w) {
    uint32_t n = w->n;
    /* T-step (SPEC.md §2) */
    for (uint32_t i = 0; i < n; ++i) {
        val *v = &w->v[i];
        if (!v->running) continue;
        if (w->tick == 0) {
            start_new_zero_round(w, v);                 /* Core::started (core.rs:144-147) */
            miner_mine(w, v);                           /* Minner::started (minner/mod.rs:43-48) */
            continue;
        }
        if (v->wake_tick == w->tick) {                  /* seal wakes up */
            v->wake_tick = -1;
            handle_new_header_event(w, v);
        }
        miner_step(w, v);
        if (v->sync_pending) {
            if (v->last < v->sync_pending) out_sync(w, v, v->last + 1);
            v->sync_pending = 0;
        }
        if (!v->core_dead && v->timer_tick == w->tick) {
            v->timer_tick = -1;
            handle_timer_event(w, v);
        }
        if (w->cfg->backlog_mode) {                     /* SPEC.md §10 */
            backlog_replay(w, v);
            if (w->frozen) break;
        }
    }
    for (uint32_t p = 0;; ++p) {
        if (w->frozen) return;
        if (!pending_local(w)) break;
        int capped = p >= w->cfg->phase_cap;
        for (uint32_t i = 0; i < n; ++i) {
            val *v = &w->v[i];
            v->cur = v->next;
            memset(&v->next, 0, sizeof(outbox));
            if (w->mlog && v->running) crypto_log(w, i, &v->cur, p);
            if (capped && !outbox_empty(&v->cur)) w->flags |= ORC_FLAG_PHASE_CAP;
        }
        if (capped) break;
        deliver_phase(w, p);
    }
}

static int run_instance(const orc_config *cfg, uint32_t inst, const orc_result *res, uint64_t idx,
                        uint64_t *trace, uint32_t max_rec);

int orc_run(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances,
            const orc_result *res) {
    for (uint64_t i = 0; i < n_instances; ++i)
        run_instance(cfg, (uint32_t)(first_instance + i), res, i, NULL, 0);
    return 0;
}

int orc_trace(const orc_config *cfg, uint64_t instance, uint64_t *out, uint32_t max_rec) {
    return run_instance(cfg, (uint32_t)instance, NULL, 0, out, max_rec);
}

/* ---- the per-instance run ---------------------------------------------------------------- */
typedef struct { world w; } runner;

static void set_hash(world *w, uint32_t x) {
    const orc_config *cfg = w->cfg;
    canon_entry *c = canon_at(w, x);
    uint8_t tx[32], buf[512];
    orc_tx_hash(cfg->seed, w->inst, x, c->b.prop, c->b.var, tx);
    uint64_t time = cfg->genesis_time + (uint64_t)cfg->block_period * (uint64_t)(c->T + 1);
    size_t len = orc_encode_header(buf, canon_at(w, x - 1)->hash, cfg->addresses + 20u * c->b.prop, tx,
                                   x, 0, 0, time, CAND_EXTRA, 11);
    orc_keccak256(buf, len, c->hash);
    c->seed = orc_seed_from_hash_order(c->hash, w->n, cfg->seed_byte_order);
}

/* per-instance summary of a streamed run (orc_run_stream) */
static void stream_summary(const orc_config *cfg, world *w, uint32_t done_tick, orc_stream *st, uint64_t idx,
                           uint64_t hist[ORC_HIST_BINS]);

static int run_instance_ex(const orc_config *cfg, uint32_t inst, const orc_result *res, uint64_t idx,
                           uint64_t *trace, uint32_t max_rec, orc_stream *st, uint64_t *hist);

static int run_instance(const orc_config *cfg, uint32_t inst, const orc_result *res, uint64_t idx,
                        uint64_t *trace, uint32_t max_rec) {
    return run_instance_ex(cfg, inst, res, idx, trace, max_rec, NULL, NULL);
}

/* real-crypto mode context of the instance being run (orc_run_crypto; single-threaded) */
static const uint64_t *g_forged;
static uint32_t *g_mlog, *g_mlog_n;
static uint32_t g_mlog_cap;

int orc_run_crypto(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances, const orc_result *res,
                   const uint64_t forged[4], uint32_t *mlog, uint32_t *mlog_n, uint32_t mlog_cap) {
    g_forged = forged;
    g_mlog_cap = mlog_cap;
    for (uint64_t i = 0; i < n_instances; ++i) {
        g_mlog = mlog + (size_t)i * mlog_cap * 8;
        g_mlog_n = mlog_n + i;
        run_instance(cfg, (uint32_t)(first_instance + i), res, i, NULL, 0);
    }
    g_forged = NULL; g_mlog = NULL; g_mlog_n = NULL;
    return 0;
}

static int run_instance_ex(const orc_config *cfg, uint32_t inst, const orc_result *res, uint64_t idx,
                           uint64_t *trace, uint32_t max_rec, orc_stream *st, uint64_t *hist) {
    runner *R = (runner *)calloc(1, sizeof(runner));
    world *w = &R->w;
    uint32_t n = cfg->n;
    assert(n >= 1 && n <= ORC_MAX_N);
    w->cfg = cfg;
    w->inst = inst;
    w->n = n;
    w->q = orc_two_thirds_majority(n);
    w->v = (val *)calloc(n, sizeof(val));
    if (g_mlog) { w->forged = g_forged; w->mlog = g_mlog; w->mlog_cap = g_mlog_cap; w->mlog_n = 0; }
    bl_entry *bl_all = cfg->backlog_mode ? (bl_entry *)calloc((size_t)n * n, sizeof(bl_entry)) : NULL;
    if (bl_all)
        for (uint32_t i = 0; i < n; ++i) w->v[i].bl = bl_all + (size_t)i * n;
    w->canon_cap = cfg->heights + 64;
    w->canon = (canon_entry *)calloc(w->canon_cap + 1, sizeof(canon_entry));
    /* genesis (core/genesis.rs:24-59) */
    canon_entry *g = canon_at(w, 0);
    g->set = 1; g->b.h = 0; g->b.valid = 1; g->T = -1; g->round = 0; g->commit_tick = 0;
    orc_genesis_hash(cfg, g->hash);
    g->seed = orc_seed_from_hash_order(g->hash, n, cfg->seed_byte_order);
    uint64_t byz[4];
    orc_byz_mask(cfg, inst, byz);
    for (uint32_t i = 0; i < n; ++i) {
        val *v = &w->v[i];
        v->running = !((cfg->silent_mask[i >> 6] >> (i & 63)) & 1);
        v->byz = (int)((byz[i >> 6] >> (i & 63)) & 1);
        v->proposer = UINT32_MAX;
        v->timer_tick = -1;
        v->rc_last_tick = 0;    /* round_change_limiter = Instant::now() at Core::new (core.rs:308) */
        v->wake_tick = -1;
        v->st = ST_ACCEPT_REQUEST;
    }
    uint32_t done_tick = cfg->max_ticks;
    for (w->tick = 0; w->tick < (int64_t)cfg->max_ticks; ++w->tick) {
        run_tick(w);
        if (trace && (uint64_t)w->tick < max_rec) {
            for (uint32_t i = 0; i < n; ++i) {
                val *v = &w->v[i];
                uint64_t s = (uint64_t)(v->h & 0xffff) | ((uint64_t)(v->r & 0xff) << 16) |
                             ((uint64_t)(v->st & 7) << 24) | ((uint64_t)(v->wait & 1) << 27) |
                             ((uint64_t)(v->last & 0xffff) << 28) | ((uint64_t)v->lock.valid << 44) |
                             ((uint64_t)v->pp.valid << 45) | ((uint64_t)v->pend.valid << 46) |
                             ((uint64_t)v->core_dead << 47) | ((uint64_t)(bits_count(&v->prep) & 0xff) << 48) |
                             ((uint64_t)(bits_count(&v->comm) & 0xff) << 56);
                trace[(uint64_t)w->tick * n + i] = s;
            }
        }
        if (w->frozen || w->canon_h >= cfg->heights) { done_tick = (uint32_t)w->tick + 1; break; }
    }
    if (res) {
        uint32_t H = cfg->heights;
        uint32_t ch = w->canon_h < H ? w->canon_h : H;
        uint32_t flags = w->flags;
        if (!w->frozen && w->canon_h < H) flags |= ORC_FLAG_TIMEOUT;
        res->committed_height[idx] = ch;
        res->flags[idx] = flags;
        res->ticks[idx] = done_tick;
        uint64_t views = 0;
        for (uint32_t x = 1; x <= ch; ++x) {
            canon_entry *c = canon_at(w, x);
            views += (uint64_t)c->round + 1;
            res->round[idx * H + (x - 1)] = (uint16_t)c->round;
            res->proposer[idx * H + (x - 1)] = c->b.prop;
            res->variant[idx * H + (x - 1)] = c->b.var;
            res->time_tick[idx * H + (x - 1)] = (uint32_t)c->T;
            memcpy(res->block_hash + (idx * H + (x - 1)) * 32, c->hash, 32);
        }
        for (uint32_t x = ch + 1; x <= H; ++x) {
            res->round[idx * H + (x - 1)] = 0;
            res->proposer[idx * H + (x - 1)] = 0;
            res->variant[idx * H + (x - 1)] = 0;
            res->time_tick[idx * H + (x - 1)] = 0;
            memset(res->block_hash + (idx * H + (x - 1)) * 32, 0, 32);
        }
        res->views[idx] = views;
    }
    if (st) stream_summary(cfg, w, done_tick, st, idx, hist);
    free(bl_all);
    if (w->mlog) *g_mlog_n = w->mlog_n;
    free(w->v);
    free(w->canon);
    free(R);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const orc_config *cfg;
    uint64_t first, n;
    const orc_result *res;
    uint64_t *next;
    pthread_mutex_t *mu;
} job;

static void *worker(void *arg) {
    job *j = (job *)arg;
    for (;;) {
        pthread_mutex_lock(j->mu);
        uint64_t i = *j->next;
        *j->next += 1;
        pthread_mutex_unlock(j->mu);
        if (i >= j->n) break;
        run_instance(j->cfg, (uint32_t)(j->first + i), j->res, i, NULL, 0);
    }
    return NULL;
}

int orc_run_threads(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances,
                    const orc_result *res, int threads, double *seconds) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    uint64_t next = 0;
    job j = {cfg, first_instance, n_instances, res, &next, &mu};
    for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, worker, &j);
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    free(th);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Size-independent check: re-derive every committed header from its record (proposer, variant,
 * time tick) and the previous hash, Keccak it, compare with the reported block hash. Returns the
 * number of instances whose chain does not verify. Multithreaded; test infrastructure only.      */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const orc_config *cfg;
    uint64_t first, n;
    const orc_result *res;
    uint64_t *next, *bad;
    pthread_mutex_t *mu;
} vjob;

static int verify_one(const orc_config *cfg, uint32_t inst, const orc_result *res, uint64_t i) {
    uint32_t H = cfg->heights;
    uint8_t prev[32], buf[512], tx[32], out[32];
    orc_genesis_hash(cfg, prev);
    uint32_t ch = res->committed_height[i];
    if (ch > H) return 1;
    for (uint32_t x = 1; x <= ch; ++x) {
        uint64_t o = i * H + (x - 1);
        uint32_t prop = res->proposer[o];
        if (prop >= cfg->n) return 1;
        orc_tx_hash(cfg->seed, inst, x, prop, res->variant[o], tx);
        uint64_t time = cfg->genesis_time + (uint64_t)cfg->block_period * ((uint64_t)res->time_tick[o] + 1);
        size_t len = orc_encode_header(buf, prev, cfg->addresses + 20u * prop, tx, x, 0, 0, time, CAND_EXTRA, 11);
        orc_keccak256(buf, len, out);
        if (memcmp(out, res->block_hash + o * 32, 32) != 0) return 1;
        memcpy(prev, out, 32);
    }
    return 0;
}

static void *vworker(void *arg) {
    vjob *j = (vjob *)arg;
    for (;;) {
        pthread_mutex_lock(j->mu);
        uint64_t i = *j->next;
        *j->next += 1;
        pthread_mutex_unlock(j->mu);
        if (i >= j->n) break;
        if (verify_one(j->cfg, (uint32_t)(j->first + i), j->res, i)) {
            pthread_mutex_lock(j->mu);
            *j->bad += 1;
            pthread_mutex_unlock(j->mu);
        }
    }
    return NULL;
}

uint64_t orc_verify_chains(const orc_config *cfg, uint64_t first, uint64_t n, const orc_result *res, int threads) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    uint64_t next = 0, bad = 0;
    vjob j = {cfg, first, n, res, &next, &bad, &mu};
    for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, vworker, &j);
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    free(th);
    return bad;
}

/* ------------------------------------------------------------------------------------------ */
/* Streamed runs: per-instance totals, the tip hash (it commits to the whole chain) and the     */
/* rounds-to-commit / commit-latency histograms of SURVEY.md §8d cfg5, without per-height rows. */
/* ------------------------------------------------------------------------------------------ */
static void stream_summary(const orc_config *cfg, world *w, uint32_t done_tick, orc_stream *st, uint64_t idx,
                           uint64_t hist[ORC_HIST_BINS]) {
    uint32_t H = cfg->heights;
    uint32_t ch = w->canon_h < H ? w->canon_h : H;
    uint32_t flags = w->flags;
    if (!w->frozen && w->canon_h < H) flags |= ORC_FLAG_TIMEOUT;
    uint64_t views = 0;
    for (uint32_t x = 1; x <= ch; ++x) {
        canon_entry *c = canon_at(w, x);
        views += (uint64_t)c->round + 1;
        hist[c->round < 64 ? c->round : 64] += 1;
        int64_t lat = c->commit_tick - canon_at(w, x - 1)->commit_tick;
        hist[65 + (lat < 64 ? lat : 64)] += 1;
    }
    st->committed_height[idx] = ch;
    st->flags[idx] = flags;
    st->ticks[idx] = done_tick;
    st->views[idx] = views;
    memcpy(st->tip_hash + idx * 32, canon_at(w, ch)->hash, 32);
}

typedef struct {
    const orc_config *cfg;
    uint64_t first, n;
    orc_stream *st;
    uint64_t *next;
    pthread_mutex_t *mu;
    uint64_t hist[ORC_HIST_BINS];
} sjob;

static void *stream_worker(void *arg) {
    sjob *j = (sjob *)arg;
    for (;;) {
        pthread_mutex_lock(j->mu);
        uint64_t i = *j->next;
        *j->next += 1;
        pthread_mutex_unlock(j->mu);
        if (i >= j->n) break;
        run_instance_ex(j->cfg, (uint32_t)(j->first + i), NULL, i, NULL, 0, j->st, j->hist);
    }
    return NULL;
}

int orc_run_stream(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances, orc_stream *st,
                   int threads) {
    if (threads < 1) threads = 1;
    memset(st->hist, 0, sizeof st->hist);
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    sjob *jobs = (sjob *)calloc((size_t)threads, sizeof(sjob));
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    uint64_t next = 0;
    for (int t = 0; t < threads; ++t) {
        jobs[t].cfg = cfg; jobs[t].first = first_instance; jobs[t].n = n_instances;
        jobs[t].st = st; jobs[t].next = &next; jobs[t].mu = &mu;
        pthread_create(&th[t], NULL, stream_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        for (int b = 0; b < ORC_HIST_BINS; ++b) st->hist[b] += jobs[t].hist[b];
    }
    free(jobs);
    free(th);
    return 0;
}
