/*
 * bft_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the consensus-rs PBFT core (src/consensus/pbft/core) running the
 * deterministic schedule of SPEC.md. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU comparator. The product path
 * (include/bftsim.h, consensus-rs_amd/) never links or calls it.
 *
 * Parity status: handler semantics follow the reference file:line by file:line (see the .c).
 * Keccak-256 is pinned by its published known answers; Philox4x32-10 by Random123's known
 * answers. Header byte encoding, block hashes and proposer seeds are "parity unpinned": the
 * reference's serialization lives in the unvendored cryptocurrency-kit crate (no Cargo.lock),
 * see DESIGN.md §Oracle.
 */
#ifndef BFT_ORACLE_H
#define BFT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_N 256

typedef struct orc_config {
    uint32_t n;                  /* validators */
    uint32_t heights;            /* H: stop once the canonical chain reaches H */
    uint32_t max_ticks;          /* safety cap on ticks */
    uint32_t block_period;       /* seconds (examples/c1.toml:6 → 3) */
    uint64_t genesis_time;       /* unix seconds (examples/c1.toml:15 → 1536517089) */
    uint64_t seed;
    uint32_t drop_ppm;           /* per-link per-phase drop probability (ppm) */
    uint32_t byz_count;          /* Byzantine (equivocating) validators per instance */
    uint32_t proposer_crash_ppm; /* per-view probability that the proposer stays silent */
    uint32_t phase_cap;          /* max message phases per tick */
    uint64_t silent_mask[4];     /* validators that never run */
    const uint8_t *addresses;    /* n * 20 bytes, ascending (sorted validator set) */
    uint8_t genesis_proposer[20];
    uint64_t genesis_gas_used;   /* gas_limit = gas_used + 10 (genesis.rs:51-53) */
    uint32_t seed_byte_order;    /* 0: U128 read big-endian, 1: little-endian (validator.rs:39-48) */
    uint32_t header_encoding;    /* 0: compact MessagePack (SPEC.md §7) */
    uint32_t backlog_mode;       /* 0: reference (never re-delivered), 1: replay (SPEC.md §10) */
    uint32_t reserved;
} orc_config;

typedef struct orc_result {
    uint32_t *committed_height;  /* [n_inst] */
    uint32_t *flags;             /* [n_inst] */
    uint32_t *ticks;             /* [n_inst] */
    uint64_t *views;             /* [n_inst] instance-rounds: sum over heights of (round+1) */
    uint16_t *round;             /* [n_inst * H] */
    uint16_t *proposer;          /* [n_inst * H] */
    uint8_t  *variant;           /* [n_inst * H] */
    uint32_t *time_tick;         /* [n_inst * H] */
    uint8_t  *block_hash;        /* [n_inst * H * 32] */
} orc_result;

/* flags */
#define ORC_FLAG_SAFETY     1u   /* two different blocks committed at one height */
#define ORC_FLAG_PHASE_CAP  2u   /* messages dropped at the phase cap */
#define ORC_FLAG_CORE_PANIC 4u   /* a Core actor panicked (start_new_round with no request) */
#define ORC_FLAG_OUTBOX     8u   /* a second message of one kind in one phase was dropped */
#define ORC_FLAG_TIMEOUT    16u  /* max_ticks reached before H */

/* primitives (exported for known-answer tests) */
void orc_keccak256(const uint8_t *data, size_t len, uint8_t out[32]);
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t orc_two_thirds_majority(uint32_t n);
int orc_check_message(int code, uint32_t msg_height, uint32_t core_height, int state); /* core.rs:366-399 */
uint32_t orc_seed_from_hash(const uint8_t hash[32], uint32_t n);                 /* big-endian U128 */
uint32_t orc_seed_from_hash_order(const uint8_t hash[32], uint32_t n, uint32_t order); /* 1 = LE */
size_t orc_encode_header(uint8_t *out, const uint8_t prev_hash[32], const uint8_t proposer[20],
                         const uint8_t tx_hash[32], uint64_t height, uint64_t gas_limit,
                         uint64_t gas_used, uint64_t time, const uint8_t *extra, size_t extra_len);
void orc_genesis_hash(const orc_config *cfg, uint8_t out[32]);
void orc_tx_hash(uint64_t seed, uint32_t instance, uint32_t height, uint32_t proposer,
                 uint32_t variant, uint8_t out[32]);
void orc_byz_mask(const orc_config *cfg, uint32_t instance, uint64_t out[4]);
void orc_deliver_mask(const orc_config *cfg, uint32_t instance, uint32_t tick, uint32_t phase,
                      uint32_t receiver, uint64_t out[4]);

/* run instances [first, first+n) ; results indexed 0..n-1 ; returns 0 */
int orc_run(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances,
            const orc_result *res);
/* same, on `threads` std threads; returns elapsed seconds via *seconds */
int orc_run_threads(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances,
                    const orc_result *res, int threads, double *seconds);

/* real-crypto mode (SPEC.md §11), single-threaded: as orc_run, and every consensus message broadcast is
 * logged per instance into mlog[i * mlog_cap * 8 ..] (8 words each, the layout of the GPU log) with its
 * count in mlog_n[i]; the messages of `forged` senders are dropped by every receiver */
int orc_run_crypto(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances, const orc_result *res,
                   const uint64_t forged[4], uint32_t *mlog, uint32_t *mlog_n, uint32_t mlog_cap);

/* number of instances whose committed header chain does not re-hash to the reported hashes */
uint64_t orc_verify_chains(const orc_config *cfg, uint64_t first, uint64_t n, const orc_result *res,
                           int threads);

/* streamed run (no per-height rows): per-instance totals, the hash of the block at
 * committed_height (genesis hash if 0), and summed histograms: hist[0..64] rounds-to-commit of each
 * committed height (64 = overflow), hist[65..129] commit latency in ticks (tick of the phase that
 * recorded height x minus that of x-1; genesis = tick 0; 64 = overflow). */
#define ORC_HIST_BINS 130
typedef struct orc_stream {
    uint32_t *committed_height;  /* [n] */
    uint32_t *flags;             /* [n] */
    uint32_t *ticks;             /* [n] */
    uint64_t *views;             /* [n] */
    uint8_t *tip_hash;           /* [n * 32] */
    uint64_t hist[ORC_HIST_BINS];
} orc_stream;
int orc_run_stream(const orc_config *cfg, uint64_t first_instance, uint64_t n_instances, orc_stream *st,
                   int threads);

/* per-tick state digest of one instance (debug/parity localisation):
 * for each tick t < max_rec, out[t*n + v] = packed state of validator v at the end of tick t */
int orc_trace(const orc_config *cfg, uint64_t instance, uint64_t *out, uint32_t max_rec);

#ifdef __cplusplus
}
#endif
#endif
