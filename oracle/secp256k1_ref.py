"""secp256k1_ref.py — CPU restatement of the ECDSA arithmetic behind the reference's message
signatures. TEST INFRASTRUCTURE ONLY: imported by tests/ and by bench.py's cpu_baseline leg as the
checker, never by the product path (consensus-rs_amd/), which fails loudly without its HIP library.

What the reference calls (all through the unvendored `cryptocurrency-kit` crate, whose `ethkey`
module is parity-ethereum's ethkey over the C library libsecp256k1 — no Cargo.lock pins a version):
  * `GossipMessage::set_sign` -> `Hash::sign(secret)` (src/protocol/mod.rs:88-92; core.rs:425-429):
    recoverable ECDSA over the 32-byte Keccak digest of the message bytes;
  * `GossipMessage::address` -> `recover_bytes` + `public_to_address` (src/protocol/mod.rs:103-116):
    public-key recovery, address = Keccak-256(X||Y)[12:32];
  * commit seals: `encrypt_commit_bytes` (src/types/votes.rs:94-101), checked by `verify_address`
    (src/consensus/pbft/core/commit.rs:96-100);
  * validator identity: `KeyPair::from_secret` -> address (examples/c*.toml `secret`, matched
    against the genesis `validator` list).
Published algorithms restated here: SEC 1 v2 §4.1.3 (ECDSA sign), §4.1.6 (public-key recovery);
RFC 6979 §3.2 (deterministic nonce, HMAC-SHA256 DRBG) exactly as libsecp256k1's
`nonce_function_rfc6979` drives it (key32 || msg32 mod n, no extra data, retry counter); the
libsecp256k1 conventions: low-s normalisation (s > n/2 -> n - s, recid ^= 1), recid bit 1 when
R.x >= n, compact signature r(32, BE) || s(32, BE) || recid(1).

Pinned by: the reference's own fixtures (the five `secret`s of examples/c1..c5.toml derive the
genesis `validator` addresses of examples/c1.toml:14, tests/test_sig_pins.py); the curve
constants (G on the curve, n*G = infinity); SHA-256/HMAC from Python's hashlib/hmac; the
ECDSA verification equation as an independent check of every signature.
Pure-Python big integers: small cases only (about 1 ms per scalar multiplication).
"""
from __future__ import annotations

import hashlib
import hmac

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)


def on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - 7) % P == 0


def point_add(a, b):
    """Affine addition (None = infinity)."""
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def point_mul(k: int, pt=G):
    r = None
    q = pt
    while k:
        if k & 1:
            r = point_add(r, q)
        q = point_add(q, q)
        k >>= 1
    return r


def pubkey(secret: bytes) -> bytes:
    d = int.from_bytes(secret, "big")
    if not 0 < d < N:
        raise ValueError("invalid secret")
    x, y = point_mul(d)
    return x.to_bytes(32, "big") + y.to_bytes(32, "big")


def address(pub64: bytes, keccak256) -> bytes:
    """public_to_address: Keccak-256 of the 64-byte public key, last 20 bytes."""
    return keccak256(pub64)[12:]


def rfc6979_nonces(secret: bytes, msg32: bytes):
    """libsecp256k1 nonce_function_rfc6979: HMAC-DRBG(key32 || (msg mod n)), one 32-byte output per
    retry counter (RFC 6979 §3.2 steps b-h)."""
    m = (int.from_bytes(msg32, "big") % N).to_bytes(32, "big")
    V = b"\x01" * 32
    K = b"\x00" * 32
    K = hmac.new(K, V + b"\x00" + secret + m, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    K = hmac.new(K, V + b"\x01" + secret + m, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    retry = False
    while True:
        if retry:
            K = hmac.new(K, V + b"\x00", hashlib.sha256).digest()
            V = hmac.new(K, V, hashlib.sha256).digest()
        V = hmac.new(K, V, hashlib.sha256).digest()
        retry = True
        yield V


def sign(secret: bytes, msg32: bytes) -> bytes:
    """Recoverable compact signature r || s || recid (libsecp256k1 secp256k1_ecdsa_sign_recoverable)."""
    d = int.from_bytes(secret, "big")
    if not 0 < d < N:
        raise ValueError("invalid secret")
    e = int.from_bytes(msg32, "big") % N
    for nonce in rfc6979_nonces(secret, msg32):
        k = int.from_bytes(nonce, "big")
        if not 0 < k < N:
            continue
        rx, ry = point_mul(k)
        r = rx % N
        recid = (ry & 1) | (2 if rx >= N else 0)
        s = pow(k, N - 2, N) * (e + r * d) % N
        if r == 0 or s == 0:
            continue
        if s > N // 2:
            s = N - s
            recid ^= 1
        return r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([recid])


def recover(msg32: bytes, sig65: bytes):
    """Public key (64 bytes) or None (libsecp256k1 secp256k1_ecdsa_recover)."""
    r = int.from_bytes(sig65[:32], "big")
    s = int.from_bytes(sig65[32:64], "big")
    recid = sig65[64]
    if recid > 3 or not 0 < r < N or not 0 < s < N:
        return None
    x = r + N if recid & 2 else r
    if x >= P:
        return None
    y2 = (x * x * x + 7) % P
    y = pow(y2, (P + 1) // 4, P)
    if y * y % P != y2:
        return None
    if (y & 1) != (recid & 1):
        y = P - y
    e = int.from_bytes(msg32, "big") % N
    rinv = pow(r, N - 2, N)
    q = point_add(point_mul(-e * rinv % N), point_mul(s * rinv % N, (x, y)))
    if q is None:
        return None
    return q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")


def verify(pub64: bytes, msg32: bytes, sig65: bytes) -> bool:
    """Plain ECDSA verification (SEC 1 §4.1.4): an independent check of sign()."""
    r = int.from_bytes(sig65[:32], "big")
    s = int.from_bytes(sig65[32:64], "big")
    if not (0 < r < N and 0 < s < N):
        return False
    Q = (int.from_bytes(pub64[:32], "big"), int.from_bytes(pub64[32:], "big"))
    e = int.from_bytes(msg32, "big") % N
    w = pow(s, N - 2, N)
    pt = point_add(point_mul(e * w % N), point_mul(r * w % N, Q))
    return pt is not None and pt[0] % N == r
