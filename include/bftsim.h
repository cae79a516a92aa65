/*
 * bftsim.h — C ABI of libbftsim, the MI355X-native batched PBFT simulator.
 *
 * This is the drop-in boundary for the reference's single-instance consensus path: one call runs
 * many independent, seeded consensus-rs clusters on a gfx950 GPU. The reference interfaces it
 * replaces (all paths in 2892931976/consensus-rs):
 *   - `trait Backend` (src/consensus/backend.rs:45-68) + `ImplBackend::{gossip,commit,verify}`
 *     (backend.rs:140-242): the N Cores of one cluster, their gossip and their chain commits
 *     become one instance simulated on the GPU;
 *   - `trait Engine` (src/consensus/consensus.rs:28-38) + `Minner` (src/minner/mod.rs:28-144):
 *     the height driver becomes the per-instance tick loop;
 *   - `trait ValidatorSet` / `ImplValidatorSet` (src/consensus/validator.rs:10-159): exported below
 *     as plain functions (quorum, proposer seed, sorted set);
 *   - the network entry `HandleMsgFn` (src/p2p/server.rs:45) / `handle_msg_middle`
 *     (src/consensus/pbft/core/core.rs:50-116): replaced by the seeded delivery schedule
 *     (SPEC.md §3).
 * Conventions (mirroring the reference's `Result`): every entry returns 0 on success and a
 * negative code on failure; `bftsim_last_error` explains the last failure. No exceptions or
 * panics cross the ABI. A handle is not thread-safe: use one handle per host thread / GPU.
 * Result buffers are caller-owned.
 */
#ifndef BFTSIM_H
#define BFTSIM_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BFTSIM_OK 0
#define BFTSIM_EINVAL -1      /* bad configuration / arguments */
#define BFTSIM_EHIP -2        /* HIP runtime error */
#define BFTSIM_ENOMEM -3
#define BFTSIM_EUNSUPPORTED -4

/* result flags (per instance) */
#define BFTSIM_FLAG_SAFETY 1u        /* two different blocks committed at one height (frozen) */
#define BFTSIM_FLAG_PHASE_CAP 2u     /* messages dropped at the per-tick phase cap */
#define BFTSIM_FLAG_CORE_PANIC 4u    /* a Core panicked (core.rs:540 unwrap on no request) */
#define BFTSIM_FLAG_OUTBOX 8u        /* a second message of one kind in one phase was dropped */
#define BFTSIM_FLAG_TIMEOUT 16u      /* max_ticks reached before `heights` */
#define BFTSIM_FLAG_RCS_OVERFLOW 32u /* more round-change rounds than the set's capacity (bftsim_set_rcs_capacity) */
#define BFTSIM_FLAG_WINDOW 64u       /* windowed run: a lookup older than the row ring (result unpinned) */

/* Conventions the reference leaves to unvendored crates (SPEC.md §1, §7): they are
 * parity-unpinned, so they are explicit switches here rather than silent assumptions.
 *   seed_byte_order: how `U128::from(seed_buf)` reads the 16-byte buffer hash[0..8] ++ 0^8 in
 *     randon_seed (src/consensus/validator.rs:39-48; `bigint = "4.4.1"`, Cargo.toml:16).
 *     BE: seed = (BE64(hash[0..8]) * 2^64) mod N  (seed == 0 for every power-of-two N);
 *     LE: seed = LE64(hash[0..8]) mod N           (every N needs the block hash in-kernel).
 *   header_encoding: the StorageValue serialization of `Header` behind `hash()` (block.rs:76-80);
 *     only the compact rmp-serde form of SPEC.md §7 exists today.
 *   backlog_mode: what BackLogActor does with FutureMessage / FutureRoundMessage
 *     (src/consensus/pbft/core/back_log.rs:38-91). DROP is the reference (stored, never re-delivered);
 *     REPLAY is the opt-in liveness variant of SPEC.md §10 (not a parity target of the reference). */
#define BFTSIM_SEED_BE 0u
#define BFTSIM_SEED_LE 1u
#define BFTSIM_ENC_RMP_COMPACT 0u
#define BFTSIM_BACKLOG_DROP 0u
#define BFTSIM_BACKLOG_REPLAY 1u

typedef struct bftsim_config {
    uint32_t n;                  /* validators per instance: 1..256 */
    uint32_t heights;            /* stop once the canonical chain reaches this height */
    uint32_t max_ticks;          /* cap on ticks (a tick = block_period = RC timeout) */
    uint32_t block_period;       /* seconds (examples/c1.toml:6) */
    uint64_t genesis_time;       /* examples/c1.toml:15 */
    uint64_t seed;               /* Philox key (SPEC.md §5) */
    uint32_t drop_ppm;           /* per-link per-phase drop probability */
    uint32_t byz_count;          /* equivocating validators per instance (SPEC.md §6) */
    uint32_t proposer_crash_ppm; /* per-view probability that the proposer stays silent */
    uint32_t phase_cap;          /* max message phases per tick */
    uint64_t silent_mask[4];     /* validators that never run */
    const uint8_t *addresses;    /* n*20 bytes, ascending = validator index order */
    uint8_t genesis_proposer[20];
    uint64_t genesis_gas_used;
    uint32_t seed_byte_order;    /* BFTSIM_SEED_BE (default) | BFTSIM_SEED_LE */
    uint32_t header_encoding;    /* BFTSIM_ENC_RMP_COMPACT */
    uint32_t backlog_mode;       /* BFTSIM_BACKLOG_DROP (reference) | BFTSIM_BACKLOG_REPLAY */
    uint32_t reserved;           /* must be 0 */
} bftsim_config;

typedef struct bftsim_result {   /* host buffers, caller-owned; H = config.heights */
    uint64_t *committed_height;  /* [n_inst] canonical chain length (<= H) */
    uint32_t *flags;             /* [n_inst] */
    uint32_t *ticks;             /* [n_inst] ticks used */
    uint64_t *views;             /* [n_inst] instance-rounds: sum of (commit round + 1) */
    uint16_t *round;             /* [n_inst*H] round of the first commit of each height */
    uint16_t *proposer;          /* [n_inst*H] proposer index of the committed block */
    uint8_t *variant;            /* [n_inst*H] 1 = the equivocated second block */
    uint32_t *time_tick;         /* [n_inst*H] header.time = genesis + period*(tick+1) */
    uint8_t *block_hash;         /* [n_inst*H*32] Keccak-256 of the header (block.rs:76-80) */
    uint64_t capacity;           /* instances the buffers above hold: at least the instances the call
                                    writes (bftsim_run's n, bftsim_launched_count's n), else the call
                                    fails with BFTSIM_EINVAL and writes nothing */
} bftsim_result;

typedef struct bftsim_stats {    /* summed over the instances of the last launch */
    uint64_t instances;
    uint64_t committed_heights;
    uint64_t views;              /* instance-rounds */
    uint64_t ticks;
    uint64_t flagged[7];         /* instances with each flag bit set */
    uint64_t round_hist[65];     /* rounds-to-commit: heights committed in round 0..63, [64] = 64+ */
    uint64_t latency_hist[65];   /* commit latency: ticks between the records of heights x-1 and x
                                    (genesis = tick 0), [64] = 64+ */
} bftsim_stats;

typedef struct bftsim bftsim_t;

/* lifecycle */
int bftsim_create(const bftsim_config *cfg, int hip_device, bftsim_t **out);
void bftsim_destroy(bftsim_t *h);
const char *bftsim_last_error(bftsim_t *h);

/* synchronous: run instances [first, first+n) and copy results to host buffers */
int bftsim_run(bftsim_t *h, uint64_t first_instance, uint64_t n_instances, bftsim_result *out);

/* device-resident API (benchmarks): allocate once, launch many times, fetch on demand */
int bftsim_prepare(bftsim_t *h, uint64_t n_instances);
int bftsim_launch(bftsim_t *h, uint64_t first_instance, void *hip_stream);   /* async */
int bftsim_sync(bftsim_t *h);
int bftsim_fetch(bftsim_t *h, bftsim_result *out);
/* the instance range of the last launch [first, first + n): the count bftsim_fetch, _fetch_summary,
 * _export_headers, _export_ledger and _crypto_verify write per-instance rows for (n = 0: nothing launched).
 * Every one of those takes the capacity of the caller's buffers (in instances) and refuses a short one
 * with BFTSIM_EINVAL before writing anything (the reference's Result-returning boundary,
 * src/consensus/backend.rs:45-68) */
int bftsim_launched_count(bftsim_t *h, uint64_t *first_instance, uint64_t *n_instances);
int bftsim_stats_get(bftsim_t *h, bftsim_stats *out);   /* device reduction + copy */
/* multi-GPU (one process per GPU): the instances shard over the ranks with no data-path
 * collective; the statistics of every rank are summed by one RCCL all-reduce over xGMI. Rank 0 makes
 * the 128-byte id (ncclGetUniqueId) and the host hands it to every rank (any channel); each rank
 * then joins with its handle. Replaces the per-node Engine of create_bft_engine
 * (src/consensus/consensus.rs:42-60) with one engine per device and a node-wide statistic.
 * BFTSIM_EUNSUPPORTED when librccl.so.1 cannot be opened. */
/* 0 when librccl.so.1 opens with every entry point this library uses, else BFTSIM_EUNSUPPORTED. Every rank
 * calls it and the ranks agree on the answer (any channel) BEFORE any of them calls bftsim_comm_init:
 * ncclCommInitRank blocks until every rank has joined, so a rank that could not even open the library
 * would leave the others waiting there (bftsim/distributed.py capi_comm_init). */
int bftsim_comm_available(void);
int bftsim_comm_unique_id(uint8_t unique_id[128]);
int bftsim_comm_init(bftsim_t *h, int world_size, int rank, const uint8_t unique_id[128]);
/* bftsim_stats of the last launch summed over every rank (collective: every rank calls it) */
int bftsim_stats_allreduce(bftsim_t *h, bftsim_stats *out);
/* per-kernel device time of the last launch, from HIP events on the launch stream (ms) */
int bftsim_last_kernel_ms(bftsim_t *h, float *consensus_ms, float *hash_ms);
/* summed per-kernel device times (ms) of every launch since the previous call, without blocking
 * between launches (waits only for the launches being summed) */
int bftsim_kernel_ms_sum(bftsim_t *h, double *consensus_ms, double *hash_ms, uint32_t *launches);
/* pipelined launches (power-of-two N; with little-endian seeds at N = 64 too, whose launches carry their own
 * seed chain and no hash pass; the batch throughput mode of the benchmark): a ring of `on` row-table sets
 * (on = 1 means 2; 0 disables; at most 32), each with the scratch of one launch, so that up to `on` launches
 * are in flight. A launch's consensus kernel runs on one of two internal launch streams (four with
 * little-endian seeds) after the caller's earlier work on `hip_stream` and after its set's last hash
 * pass; the prev_hash chains of bftsim_set_hash_batch consecutive launches run as one kernel on one of two
 * internal hash streams (a chain is sequential in height: a launch's chains take ~1.5 ms however many
 * there are, so batching multiplies their throughput). Results of a launch are complete once bftsim_sync
 * returns (it also enqueues a partial hash batch); bftsim_fetch/_stats_get/_fetch_summary read the last
 * launch (and sync as they need). The HIP runtime needs a hardware queue per stream in use (the caller's,
 * two launch and two to four hash streams): GPU_MAX_HW_QUEUES >= 5 in the environment before HIP initialises (HIP's
 * default is 4; bench.py sets 8). Takes effect at the next bftsim_prepare (buffers are re-allocated). */
int bftsim_set_pipeline(bftsim_t *h, int on);
/* pipelined launches: the number of consecutive launches whose block-hash chains run as one kernel (1..32,
 * default 4). A launch waiting for its batch is hashed when the batch fills, at bftsim_sync, or when the ring
 * needs its row-table set again. With big-endian seeds at N = 64 and a lossless schedule (no drops, no proposer
 * crashes) the chains of a batch run on the predicted canonical blocks as soon as the batch is flushed, and are
 * checked against the recorded blocks (and re-run from the first one that differs) once the batch's consensus
 * kernels are done. */
int bftsim_set_hash_batch(bftsim_t *h, uint32_t launches);
/* verification switch: 0 runs N = 64 through the full kernel alone instead of the FAST kernel +
 * resume (results are identical; the default 1 is the fast path) */
int bftsim_set_fast(bftsim_t *h, int on);
/* optional per-tick state digests of the next launch (debug; NULL disables) */
int bftsim_set_trace(bftsim_t *h, uint64_t *host_out, uint32_t trace_ticks);
/* windowed runs for long horizons (10,000 heights x 1M instances): keep only a ring
 * of `window` canonical rows per instance (power of two >= 64; 0 = every height, the default).
 * Block hashes are then computed in-kernel; per-height outputs are not kept (bftsim_fetch fails):
 * read bftsim_fetch_summary and the histograms of bftsim_stats_get. A lookup older than the ring
 * (a validator lagging > window heights) sets BFTSIM_FLAG_WINDOW. */
int bftsim_set_window(bftsim_t *h, uint32_t window);
/* RoundChangeSet capacity: distinct round-change rounds each validator keeps between two resets of its
 * set (the reference's HashMap<u64, MessageManage>, round_change_set.rs:11-35, is unbounded).
 * 1..4096, default 16. A validator needing more sets BFTSIM_FLAG_RCS_OVERFLOW on its instance;
 * bftsim_run then re-runs the batch at twice the capacity until no instance overflows (instances are
 * independent and deterministic, so the others are unchanged), as long as the doubled tables fit in 90 %
 * of the free device memory; otherwise it returns BFTSIM_OK with the flagged results. The grown capacity
 * stays in effect for later prepare / launch / run calls, with tables proportional to it (set it back
 * with this call). Takes effect at the next bftsim_prepare. */
int bftsim_set_rcs_capacity(bftsim_t *h, uint32_t rounds);
/* per-instance outputs of the last launch (any pointer may be NULL; capacity = instances each
 * buffer holds); tip_hash[i*32..] = hash of
 * the block at committed_height[i] (the genesis hash at 0), which commits to the whole chain */
int bftsim_fetch_summary(bftsim_t *h, uint64_t capacity, uint64_t *committed_height, uint32_t *flags, uint32_t *ticks,
                         uint64_t *views, uint8_t *tip_hash);

/* real-crypto mode (SPEC.md §11). Every consensus message the simulation
 * broadcasts is logged; bftsim_crypto_verify then does, batched on the GPU (libbftsig):
 *   - sign it with its sender's key (finalize_message, core.rs:425-429), the Commit seal first
 *     (encrypt_commit_bytes, types/votes.rs:94-101);
 *   - recover its signer and check membership (GossipMessage::address, protocol/mod.rs:103-116;
 *     handle_message, core.rs:314-322), and recover every seal (verify_commit, commit.rs:94-100).
 * A `forged` validator signs with a key that is not its own (keccak of its secret): every receiver
 * drops its consensus messages, which the simulation applies when they are sent. The verify pass
 * proves that assumption message by message (`mismatches` must be 0). Each message is recovered once,
 * as every receiver gets the same bytes (the reference recovers it at each receiver).
 * secrets32: host, n x 32 bytes in the sorted validator order; each must derive the address of its
 * index (else BFTSIM_EINVAL). forged: host, n bytes (NULL = none). log_cap: messages per instance
 * (0 = heights * (4n + 8) + 64n). NULL secrets turn the mode off. Takes effect at the next
 * bftsim_prepare. Needs libbftsig.so next to libbftsim.so; window 0; N = 64 runs the full kernel. */
typedef struct bftsim_crypto_report {
    uint64_t messages;             /* consensus messages broadcast (each signed once) */
    uint64_t seals;                /* Commit seals (signed, then recovered) */
    uint64_t forged;               /* messages of forged senders */
    uint64_t recovered_as_sender;  /* messages whose signature recovers their sender */
    uint64_t mismatches;           /* recovered validity != the simulated delivery: 0 */
    uint64_t seal_errors;          /* seals that do not recover */
    uint64_t signatures;           /* ECDSA signs performed: messages + seals */
    uint64_t recoveries;           /* ECDSA recoveries performed: messages + seals */
    uint64_t log_overflows;        /* instances whose log exceeded log_cap (then the call fails) */
} bftsim_crypto_report;
int bftsim_set_crypto(bftsim_t *h, const uint8_t *secrets32, const uint8_t *forged, uint32_t log_cap);
/* after a launch: the sign / recover pass of its messages; capacity = instances inst_checksum and
 * inst_messages hold (checked when either is non-NULL); inst_checksum (host, n x 32, nullable) =
 * per instance the XOR over its messages of keccak256(signature || seal or 65 zero bytes);
 * inst_messages (host, n, nullable) = messages per instance */
int bftsim_crypto_verify(bftsim_t *h, bftsim_crypto_report *out, uint64_t capacity, uint8_t *inst_checksum,
                         uint32_t *inst_messages);

/* the ledger with votes (real-crypto mode, after bftsim_crypto_verify): for every instance and height
 * x <= committed_height, in slot [i*H + x-1] of `slot_bytes` bytes, the Header that Backend::commit
 * inserts (backend.rs:163-174): the block's header (SPEC.md §7) with votes = the signatures of the
 * Commit messages in the committing Core's commit set at its commit (core.rs:402-413), ascending
 * validator order. hdr_len = 0 beyond the committed height. The hash of a header is the run's
 * block_hash of that height (block_hash() ignores votes, types/block.rs:76-80). Together with
 * block_hash per height this is the ledger's headers + block_hashes_by_height (store/schema.rs). */
uint64_t bftsim_ledger_slot_bytes(uint32_t n_validators);
int bftsim_export_ledger(bftsim_t *h, uint64_t capacity, uint8_t *hdr, uint64_t slot_bytes, uint32_t *hdr_len);

/* ValidatorSet / block helpers on the host (validator.rs, types/block.rs) */
uint32_t bftsim_two_thirds_majority(uint32_t n);                    /* validator.rs:149-154 */
uint32_t bftsim_seed_from_hash(const uint8_t hash[32], uint32_t n); /* validator.rs:39-48 (BE) */
uint32_t bftsim_seed_from_hash_order(const uint8_t hash[32], uint32_t n, uint32_t seed_byte_order);
uint32_t bftsim_calc_proposer(const uint8_t prev_hash[32], uint32_t n, uint64_t round); /* :33-37,74-77 (BE) */
void bftsim_keccak256(const uint8_t *data, size_t len, uint8_t out[32]);
void bftsim_genesis_hash(const bftsim_config *cfg, uint8_t out[32]); /* core/genesis.rs:44-55 */
int bftsim_view_cmp(uint64_t h1, uint64_t r1, uint64_t h2, uint64_t r2); /* consensus/types.rs:81-98 */
/* Core::check_message (src/consensus/pbft/core/core.rs:366-399) as the kernels run it: code =
 * MessageType (protocol/mod.rs:36-41: 1 Preprepare, 2 Prepare, 3 Commit, 4 RoundChange), state =
 * State (protocol/mod.rs:25-30: 1 AcceptRequest .. 4 Committed). Returns BFTSIM_CHECK_* (>= 0), or
 * BFTSIM_EINVAL for codes / states outside those enums. */
#define BFTSIM_CHECK_OK 0
#define BFTSIM_CHECK_UNKNOWN 1        /* ConsensusError::UnknownMessageType (height 0) */
#define BFTSIM_CHECK_FUTURE_BLOCK 2   /* FutureBlockMessage(h) */
#define BFTSIM_CHECK_OLD 3            /* OldMessage */
#define BFTSIM_CHECK_FUTURE_MSG 4     /* FutureMessage (backlog) */
int bftsim_check_message(uint32_t code, uint64_t msg_height, uint64_t core_height, uint32_t state);

/* Ledger export (core/ledger.rs:193-245 `add_block`: the `headers` map Hash -> Header of
 * store/schema.rs:66-68; the `block_hashes_by_height` list is bftsim_result.block_hash): after a
 * launch or run, the MessagePack Header bytes (SPEC.md §7, votes None: commit seals are not
 * modelled) of every committed height of the last launch, host buffers:
 * hdr[(i*H + x-1) * BFTSIM_HEADER_SLOT ...] with hdr_len[i*H + x-1] bytes (0 beyond the committed
 * height); Keccak-256 of those bytes is that height's block hash. capacity = instances the buffers
 * hold (hdr: capacity*H slots, hdr_len: capacity*H words). */
#define BFTSIM_HEADER_SLOT 288
int bftsim_export_headers(bftsim_t *h, uint64_t capacity, uint8_t *hdr, uint32_t *hdr_len);

#ifdef __cplusplus
}
#endif
#endif
