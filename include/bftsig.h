/*
 * bftsig.h — C ABI of libbftsig: batched secp256k1 recoverable ECDSA on a gfx950 GPU, one lane per
 * item ("real-crypto mode"). The reference interfaces each entry replaces
 * (paths in 2892931976/consensus-rs; the arithmetic itself lives in the unvendored
 * `cryptocurrency-kit` crate = parity ethkey over libsecp256k1):
 *   - bftsig_sign            `Hash::sign(secret)` in `GossipMessage::set_sign` (src/protocol/mod.rs:88-92,
 *                            called per broadcast at src/consensus/pbft/core/core.rs:425-429), the
 *                            commit seal `encrypt_commit_bytes` (src/types/votes.rs:94-101) and
 *                            `ImplBackend::sign` (src/consensus/backend.rs:245-252);
 *   - bftsig_recover         `recover_bytes` + `public_to_address` in `GossipMessage::address`
 *                            (src/protocol/mod.rs:103-116), run for every received message;
 *   - bftsig_verify_address  `verify_address` of the commit seals (src/consensus/pbft/core/commit.rs:96-100,
 *                            src/types/votes.rs:68-92);
 *   - bftsig_secret_to_address `KeyPair::from_secret(..).address()` (the `secret` of examples/c*.toml
 *                            versus the genesis validator list).
 * Formats: secrets and digests 32 bytes big-endian; signatures compact r(32) || s(32) || recid(1)
 * (recid 0..3, as ethkey's `Signature`); public keys X(32) || Y(32); addresses 20 bytes.
 * Signing is deterministic (RFC 6979, libsecp256k1's nonce function) and low-s normalised.
 * Every buffer argument is a DEVICE pointer (hipMalloc / torch CUDA tensors); `stream` is a
 * hipStream_t (NULL = the null stream); calls are asynchronous on that stream.
 * Per-item failures (invalid secret, malformed signature, no recovery) set ok[i] = 0 and zero the
 * outputs of that item; the call itself returns 0. Errors of the call: negative codes as in
 * bftsim.h, text via bftsig_last_error. A handle is not thread-safe.
 */
#ifndef BFTSIG_H
#define BFTSIG_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bftsig bftsig_t;

/* uploads the fixed-base table of G (32 windows x 255 affine points, 510 KB) to the device */
int bftsig_create(int hip_device, bftsig_t **out);
void bftsig_destroy(bftsig_t *h);
const char *bftsig_last_error(const bftsig_t *h);

int bftsig_secret_to_address(bftsig_t *h, const uint8_t *secrets32, uint64_t n, uint8_t *pubs64 /* nullable */,
                             uint8_t *addrs20, uint8_t *ok, void *stream);
/* item i signs digests32[i] with secrets32[key_index ? key_index[i] : i] */
int bftsig_sign(bftsig_t *h, const uint8_t *secrets32, const uint32_t *key_index /* nullable */,
                const uint8_t *digests32, uint64_t n, uint8_t *sigs65, uint8_t *ok, void *stream);
int bftsig_recover(bftsig_t *h, const uint8_t *digests32, const uint8_t *sigs65, uint64_t n,
                   uint8_t *pubs64 /* nullable */, uint8_t *addrs20, uint8_t *ok, void *stream);
/* ok[i] = 1 iff the signature recovers to addrs20[i] (verify_address) */
int bftsig_verify_address(bftsig_t *h, const uint8_t *addrs20, const uint8_t *digests32, const uint8_t *sigs65,
                          uint64_t n, uint8_t *ok, void *stream);

#ifdef __cplusplus
}
#endif
#endif
