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
 * Scope: the Subject-carrying messages (Prepare, Commit, RoundChange) — the N^2 traffic of a round.
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
/* HOST: frame boundaries of a received byte stream (MsgPacketCodec::decode's loop, codec.rs:18-40):
 * writes up to max+1 offsets, returns the number of complete frames (offs[k] = end of frame k-1). */
uint64_t bftwire_split_frames(const uint8_t *host_stream, uint64_t len, uint64_t *offs, uint64_t max);

#ifdef __cplusplus
}
#endif
#endif
