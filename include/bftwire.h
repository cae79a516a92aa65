/*
 * bftwire.h — C ABI of libbftwire: the consensus wire codec of the reference on a gfx950 GPU
 * (SURVEY.md §8f rank 1), batched. Replaces, per batch of messages:
 *   - `Subject::into_bytes` + `GossipMessage::into_payload` (src/consensus/types.rs:101-104,
 *     src/protocol/mod.rs:44-53,118-120) and `RawMessage` framing by `MsgPacketCodec::encode`
 *     (src/p2p/protocol.rs:30-70, src/p2p/codec.rs:43-53, header of src/p2p/server.rs:187)
 *     -> bftwire_encode;
 *   - `GossipMessage::sign_digest` (mod.rs:128-137, what `set_sign` signs) and `CryptoHash::hash`
 *     of the message (the outbound dedup key of `ImplBackend::gossip`, backend.rs:141-148)
 *     -> the two Keccak-256 outputs of bftwire_encode;
 *   - `MsgPacketCodec::decode` + `RawMessage::from_bytes` + `GossipMessage::from_bytes` +
 *     `Subject::from` (codec.rs:18-40, core.rs:50-60) -> bftwire_split_frames (host) + bftwire_decode.
 * Scope: the Subject-carrying messages (Prepare, Commit, RoundChange) — the N^2 traffic of a round —
 * and the block-carrying frames: Preprepare (PrePrepare{view, Block}), Block (Blocks) and Sync (Height).
 * The serializer convention is SPEC.md §9 (rmp-serde compact MessagePack; parity-unpinned against
 * the unvendored cryptocurrency-kit serializer, pinned to the MessagePack spec by the msgpack package).
 * Device pointers everywhere except bftwire_split_frames; calls are asynchronous on `stream`.
 */
#ifndef BFTWIRE_H
#define BFTWIRE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bftwire bftwire_t;

typedef struct bftwire_batch {   /* n messages, structure of arrays */
    uint8_t *code;               /* [n] MessageType: 2 Prepare, 3 Commit, 4 RoundChange */
    uint64_t *round, *height;    /* [n] Subject.view */
    uint8_t *digest;             /* [n*32] Subject.digest */
    uint64_t *create_time;       /* [n] GossipMessage.create_time */
    uint8_t *signature;          /* [n*65] Some(signature) for every message, or NULL = None */
    uint8_t *commit_seal;        /* [n*65] Some(seal) for Commit messages, or NULL = None */
    uint64_t *ttl;               /* [n] RawMessage header ttl, or NULL = 10 (p2p/server.rs:187) */
    uint64_t *raw_time;          /* [n] RawMessage header create_time, or NULL = create_time */
} bftwire_batch;

int bftwire_create(int hip_device, bftwire_t **out);
void bftwire_destroy(bftwire_t *h);
const char *bftwire_last_error(const bftwire_t *h);

/* frames of n messages, back to back, into stream[0, cap): frame_off[n+1] (frame i occupies
 * [frame_off[i], frame_off[i+1]), frame_off[n] = total bytes); sign_digest / msg_hash [n*32]
 * nullable; ok[i] = 0 for an invalid code or a frame beyond cap (not written). */
int bftwire_encode(bftwire_t *h, const bftwire_batch *in, uint64_t n, uint8_t *stream, uint64_t cap,
                   uint64_t *frame_off, uint8_t *sign_digest, uint8_t *msg_hash, uint8_t *ok, void *stream_);
/* fields of n frames (frame i = stream[frame_off[i], frame_off[i+1])) into `out` (every array
 * required; signature / commit_seal zero-filled when None); has_sig / has_seal [n]; ok[i] = 0 for
 * a malformed frame. */
int bftwire_decode(bftwire_t *h, const uint8_t *stream, const uint64_t *frame_off, uint64_t n,
                   const bftwire_batch *out, uint8_t *has_sig, uint8_t *has_seal, uint8_t *ok, void *stream_);
/* ---- block-carrying frames (SPEC.md §9b): PrePrepare consensus messages and the P2P Block / Sync
 * messages of core.rs:75-110. Structs are array-of-structures in device memory; Addresses serialize as
 * "0x" + 40 lowercase hex digits (the Header convention of SPEC.md §7), Vec<u8> / Hash / Signature as
 * arrays of integers. */
#define BFTWIRE_MAX_EXTRA 32
#define BFTWIRE_MAX_VOTES 16
#define BFTWIRE_MAX_TX 2
#define BFTWIRE_MAX_PAYLOAD 64
#define BFTWIRE_NONE 0xffffffffu  /* Option::None for a length / count field */

typedef struct bftwire_tx {         /* Transaction, serde order (types/transaction.rs:16-30) */
    uint64_t nonce, price, gas_limit, amount;
    uint32_t payload_len;           /* <= BFTWIRE_MAX_PAYLOAD */
    uint8_t has_recipient, has_sig, pad[2];
    uint8_t recipient[20];
    uint8_t payload[BFTWIRE_MAX_PAYLOAD];
    uint8_t sig[65];
    uint8_t pad2[7];
} bftwire_tx;                       /* 200 bytes */

typedef struct bftwire_block {      /* Block {header, transactions} (types/block.rs:16-36, 146-149) */
    uint64_t bloom, difficulty, height, gas_limit, gas_used, time;
    uint32_t extra_len;             /* BFTWIRE_NONE: extra None; else <= BFTWIRE_MAX_EXTRA */
    uint32_t n_votes;               /* BFTWIRE_NONE: votes None; else <= BFTWIRE_MAX_VOTES */
    uint32_t n_tx;                  /* <= BFTWIRE_MAX_TX */
    uint32_t pad;
    uint8_t prev_hash[32], root[32], tx_hash[32], receipt_hash[32];
    uint8_t proposer[20];
    uint8_t extra[BFTWIRE_MAX_EXTRA];
    uint8_t votes[BFTWIRE_MAX_VOTES][65];
    uint8_t pad2[4];
    bftwire_tx tx[BFTWIRE_MAX_TX];
} bftwire_block;

typedef struct bftwire_preprepare { /* GossipMessage{Preprepare, PrePrepare{view, Proposal(block)}} */
    uint64_t round, height;         /* PrePrepare.view (types.rs:131-134) */
    uint64_t create_time;           /* GossipMessage.create_time */
    uint64_t ttl, raw_time;         /* RawMessage header */
    uint8_t has_sig, pad[7];
    uint8_t signature[65];
    uint8_t pad2[7];
    bftwire_block block;
} bftwire_preprepare;

/* Preprepare frames (preprepare.rs:30-43 -> finalize_message -> gossip); sign_digest / msg_hash
 * nullable as in bftwire_encode. ok[i] = 0: a field over its BFTWIRE_MAX_* or a frame beyond cap. */
int bftwire_encode_preprepare(bftwire_t *h, const bftwire_preprepare *in, uint64_t n, uint8_t *stream, uint64_t cap,
                              uint64_t *frame_off, uint8_t *sign_digest, uint8_t *msg_hash, uint8_t *ok, void *stream_);
int bftwire_decode_preprepare(bftwire_t *h, const uint8_t *stream, const uint64_t *frame_off, uint64_t n,
                              bftwire_preprepare *out, uint8_t *ok, void *stream_);
/* Block frames: RawMessage{Block, payload = Blocks(blocks[block_off[k] .. block_off[k+1]])} (the
 * PostBlock answer to a Sync, core.rs:86-110); ttl / raw_time [n_frames] nullable (10 / 0) */
int bftwire_encode_blocks(bftwire_t *h, const bftwire_block *blocks, const uint64_t *block_off, uint64_t n_frames,
                          const uint64_t *ttl, const uint64_t *raw_time, uint8_t *stream, uint64_t cap,
                          uint64_t *frame_off, uint8_t *ok, void *stream_);
/* frame k's blocks into out[k * max_per_frame ..], their number into count[k] (ok = 0 beyond max) */
int bftwire_decode_blocks(bftwire_t *h, const uint8_t *stream, const uint64_t *frame_off, uint64_t n_frames,
                          uint32_t max_per_frame, bftwire_block *out, uint32_t *count, uint8_t *ok, void *stream_);
/* Sync frames: RawMessage{Sync, payload = Height} (core.rs:80-85) */
int bftwire_encode_sync(bftwire_t *h, const uint64_t *height, uint64_t n, const uint64_t *ttl, const uint64_t *raw_time,
                        uint8_t *stream, uint64_t cap, uint64_t *frame_off, uint8_t *ok, void *stream_);
int bftwire_decode_sync(bftwire_t *h, const uint8_t *stream, const uint64_t *frame_off, uint64_t n, uint64_t *height,
                        uint8_t *ok, void *stream_);

/* HOST: frame boundaries of a received byte stream (MsgPacketCodec::decode's loop, codec.rs:18-40):
 * writes up to max+1 offsets, returns the number of complete frames (offs[k] = end of frame k-1). */
uint64_t bftwire_split_frames(const uint8_t *host_stream, uint64_t len, uint64_t *offs, uint64_t max);

#ifdef __cplusplus
}
#endif
#endif
