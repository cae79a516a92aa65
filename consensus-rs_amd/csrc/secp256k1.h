// secp256k1.h — batched recoverable ECDSA on secp256k1 for gfx950 lanes (one signature per lane),
// the "real-crypto" half of the reference's per-message cost:
//   * sign     — `Hash::sign(secret)` behind GossipMessage::set_sign (src/protocol/mod.rs:88-92,
//                core.rs:425-429) and the commit seal `encrypt_commit_bytes` (src/types/votes.rs:94-101);
//   * recover  — `recover_bytes` + `public_to_address` behind GossipMessage::address
//                (src/protocol/mod.rs:103-116) and `verify_address` (commit.rs:96-100);
//   * address  — `KeyPair::from_secret(..).address()` (validator identity, examples/c*.toml).
// The arithmetic is the published one libsecp256k1 (via parity's ethkey inside the unvendored
// `cryptocurrency-kit`) implements: SEC 1 ECDSA with RFC 6979 nonces, low-s normalisation, compact
// r || s || recid signatures. Restated for the CPU in oracle/secp256k1_ref.py (the checker).
//
// Representation: 256-bit integers as 8 little-endian 32-bit limbs (one VGPR each); field elements
// mod p = 2^256 - 2^32 - 977 kept fully reduced; products by 32x32->64 multiply-adds
// (v_mad_u64_u32) and the special-form reduction 2^256 = 2^32 + 977 (mod p). Points in Jacobian
// coordinates (a = 0 formulas); k*G through a fixed-base table of 32 windows x 255 affine points
// (8-bit windows, 510 KB, L2-resident), k*R through the GLV split and signed 4-bit digits. Written once as host+device code
// (BFT_FN): the same source runs on the GPU and, host-compiled, in the CPU tests.
#pragma once
#include "bft_common.h"

namespace bft {
namespace secp {

// Everything on the arithmetic path is forced inline: an out-of-line call passes its by-reference
// points through scratch memory and spills the callee-saved VGPRs (measured: 2.5 KB scratch per lane).
#define SECP_FN __attribute__((always_inline)) BFT_FN
// host test builds count the multiplications of one operation (the roofline's work model)
#ifdef SECP_COUNT_OPS
extern uint64_t secp_op_count[4];      // fe_mul, fe_sqr, sc_mul, sc_sqr
#define SECP_COUNT(k) (++secp_op_count[k])
#else
#define SECP_COUNT(k) ((void)0)
#endif

struct U256 {
    uint32_t v[8];
};

// ------------------------------------------------------------------------------ constants
SECP_FN U256 c_p() { return U256{{0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}}; }
SECP_FN U256 c_n() { return U256{{0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}}; }
SECP_FN U256 c_nhalf() { return U256{{0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu}}; }
// 2^256 - n (129 bits)
constexpr uint32_t NC0 = 0x2FC9BEBFu, NC1 = 0x402DA173u, NC2 = 0x50B75FC4u, NC3 = 0x45512319u;
SECP_FN U256 c_gx() { return U256{{0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu, 0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu}}; }
SECP_FN U256 c_gy() { return U256{{0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u, 0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u}}; }

// ------------------------------------------------------------------------------ 256-bit helpers
SECP_FN U256 u_zero() { return U256{{0, 0, 0, 0, 0, 0, 0, 0}}; }
SECP_FN U256 u_small(uint32_t x) { return U256{{x, 0, 0, 0, 0, 0, 0, 0}}; }
SECP_FN bool u_is_zero(const U256& a) {
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x |= a.v[i];
    return x == 0;
}
SECP_FN bool u_eq(const U256& a, const U256& b) {
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x |= a.v[i] ^ b.v[i];
    return x == 0;
}
// a >= b
SECP_FN bool u_ge(const U256& a, const U256& b) {
    uint64_t br = 0;
    for (int i = 0; i < 8; ++i) {
        uint64_t d = (uint64_t)a.v[i] - b.v[i] - br;
        br = (d >> 63) & 1u;
    }
    return br == 0;
}
// r = a + b, returns the carry
SECP_FN uint32_t u_add(U256& r, const U256& a, const U256& b) {
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (uint64_t)a.v[i] + b.v[i];
        r.v[i] = (uint32_t)c;
        c >>= 32;
    }
    return (uint32_t)c;
}
// r = a - b, returns the borrow
SECP_FN uint32_t u_sub(U256& r, const U256& a, const U256& b) {
    uint64_t br = 0;
    for (int i = 0; i < 8; ++i) {
        uint64_t d = (uint64_t)a.v[i] - b.v[i] - br;
        r.v[i] = (uint32_t)d;
        br = (d >> 63) & 1u;
    }
    return (uint32_t)br;
}
SECP_FN U256 u_sel(bool c, const U256& a, const U256& b) {
    U256 r;
    for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}
SECP_FN uint32_t u_bit(const U256& a, uint32_t i) { return (a.v[i >> 5] >> (i & 31u)) & 1u; }
SECP_FN uint32_t u_nibble(const U256& a, uint32_t i) { return (a.v[i >> 3] >> (4u * (i & 7u))) & 15u; }
SECP_FN uint32_t u_byte(const U256& a, uint32_t i) { return (a.v[i >> 2] >> (8u * (i & 3u))) & 255u; }

// big-endian 32 bytes <-> limbs
SECP_FN U256 u_from_be(const uint8_t* b) {
    U256 r;
    for (int i = 0; i < 8; ++i) {
        const uint8_t* q = b + 28 - 4 * i;
        r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
    return r;
}
SECP_FN void u_to_be(const U256& a, uint8_t* b) {
    for (int i = 0; i < 8; ++i) {
        uint8_t* q = b + 28 - 4 * i;
        q[0] = (uint8_t)(a.v[i] >> 24); q[1] = (uint8_t)(a.v[i] >> 16); q[2] = (uint8_t)(a.v[i] >> 8); q[3] = (uint8_t)a.v[i];
    }
}

// 512-bit product t[16] = a * b (row-wise 32x32->64 multiply-adds)
SECP_FN void u_mul_wide(uint32_t t[16], const U256& a, const U256& b) {
    for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint64_t x = (uint64_t)a.v[i] * b.v[j] + t[i + j] + c;
            t[i + j] = (uint32_t)x;
            c = x >> 32;
        }
        t[i + 8] = (uint32_t)c;
    }
}
// squaring: cross products once, doubled, plus the diagonal
SECP_FN void u_sqr_wide(uint32_t t[16], const U256& a) {
    for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = i + 1; j < 8; ++j) {
            uint64_t x = (uint64_t)a.v[i] * a.v[j] + t[i + j] + c;
            t[i + j] = (uint32_t)x;
            c = x >> 32;
        }
        t[i + 8] = (uint32_t)c;
    }
    uint32_t top = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {          // double
        uint32_t nt = t[i] >> 31;
        t[i] = (t[i] << 1) | top;
        top = nt;
    }
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {           // + diagonal
        uint64_t sq = (uint64_t)a.v[i] * a.v[i];
        c += (uint64_t)t[2 * i] + (uint32_t)sq;
        t[2 * i] = (uint32_t)c;
        c >>= 32;
        c += (uint64_t)t[2 * i + 1] + (uint32_t)(sq >> 32);
        t[2 * i + 1] = (uint32_t)c;
        c >>= 32;
    }
}

// ------------------------------------------------------------------------------ field mod p
// t[16] mod p, using 2^256 = 0x1000003D1 (mod p)
SECP_FN U256 fe_reduce_wide(const uint32_t t[16]) {
    U256 r;
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {       // lo + hi*977 + (hi << 32)
        c += (uint64_t)t[k] + (uint64_t)t[8 + k] * 977u + (k > 0 ? (uint64_t)t[7 + k] : 0ull);
        r.v[k] = (uint32_t)c;
        c >>= 32;
    }
    uint64_t top = c + t[15];           // < 2^33
    // + top * 0x1000003D1
    uint64_t m = top * 977u;
    c = (uint64_t)r.v[0] + (uint32_t)m;
    r.v[0] = (uint32_t)c; c >>= 32;
    c += (uint64_t)r.v[1] + (m >> 32) + (uint32_t)top;
    r.v[1] = (uint32_t)c; c >>= 32;
    c += (uint64_t)r.v[2] + (top >> 32);
    r.v[2] = (uint32_t)c; c >>= 32;
#pragma unroll
    for (int k = 3; k < 8; ++k) {
        c += r.v[k];
        r.v[k] = (uint32_t)c;
        c >>= 32;
    }
    if (c) {                             // wrapped past 2^256 once more: the value is now tiny
        uint64_t d = (uint64_t)r.v[0] + 0x3D1u;
        r.v[0] = (uint32_t)d; d >>= 32;
        d += (uint64_t)r.v[1] + 1u;
        r.v[1] = (uint32_t)d; d >>= 32;
        // the whole ripple of the carry bit, unrolled (adding a zero carry changes nothing): an early exit on
        // d == 0 made the limbs a dynamically indexed private array, 36 B of scratch per lane in every secp kernel
        uint32_t cy = (uint32_t)d;                   // 0 or 1
#pragma unroll
        for (int k = 2; k < 8; ++k) { r.v[k] += cy; cy = r.v[k] < cy ? 1u : 0u; }
    }
    U256 s;
    uint32_t br = u_sub(s, r, c_p());
    return br ? r : s;
}
SECP_FN U256 fe_mul(const U256& a, const U256& b) {
    SECP_COUNT(0);
    uint32_t t[16];
    u_mul_wide(t, a, b);
    return fe_reduce_wide(t);
}
SECP_FN U256 fe_sqr(const U256& a) {
    SECP_COUNT(1);
    uint32_t t[16];
    u_sqr_wide(t, a);
    return fe_reduce_wide(t);
}
SECP_FN U256 fe_add(const U256& a, const U256& b) {
    U256 r, s;
    uint32_t c = u_add(r, a, b);
    uint32_t br = u_sub(s, r, c_p());
    return (c || !br) ? s : r;
}
SECP_FN U256 fe_sub(const U256& a, const U256& b) {
    U256 r, s;
    uint32_t br = u_sub(r, a, b);
    u_add(s, r, c_p());
    return br ? s : r;
}
SECP_FN U256 fe_neg(const U256& a) { return fe_sub(u_zero(), a); }
SECP_FN U256 fe_sqr_n(U256 a, int n) {
    for (int i = 0; i < n; ++i) a = fe_sqr(a);
    return a;
}
// a^(2^223 - 1) and the shared head of the inverse / square-root addition chains (libsecp256k1's)
SECP_FN void fe_chain_head(const U256& a, U256& x2, U256& x22, U256& x223) {
    x2 = fe_mul(fe_sqr(a), a);
    U256 x3 = fe_mul(fe_sqr(x2), a);
    U256 x6 = fe_mul(fe_sqr_n(x3, 3), x3);
    U256 x9 = fe_mul(fe_sqr_n(x6, 3), x3);
    U256 x11 = fe_mul(fe_sqr_n(x9, 2), x2);
    x22 = fe_mul(fe_sqr_n(x11, 11), x11);
    U256 x44 = fe_mul(fe_sqr_n(x22, 22), x22);
    U256 x88 = fe_mul(fe_sqr_n(x44, 44), x44);
    U256 x176 = fe_mul(fe_sqr_n(x88, 88), x88);
    U256 x220 = fe_mul(fe_sqr_n(x176, 44), x44);
    x223 = fe_mul(fe_sqr_n(x220, 3), x3);
}
// a^(p-2)
SECP_FN U256 fe_inv(const U256& a) {
    U256 x2, x22, x223;
    fe_chain_head(a, x2, x22, x223);
    U256 t = fe_mul(fe_sqr_n(x223, 23), x22);
    t = fe_mul(fe_sqr_n(t, 5), a);
    t = fe_mul(fe_sqr_n(t, 3), x2);
    return fe_mul(fe_sqr_n(t, 2), a);
}
// a^((p+1)/4): a square root when one exists (the caller checks r^2 == a)
SECP_FN U256 fe_sqrt(const U256& a) {
    U256 x2, x22, x223;
    fe_chain_head(a, x2, x22, x223);
    U256 t = fe_mul(fe_sqr_n(x223, 23), x22);
    t = fe_mul(fe_sqr_n(t, 6), x2);
    return fe_sqr_n(t, 2);
}

// ------------------------------------------------------------------------------ scalars mod n
// lo(8) + hi(len) * (2^256 - n) into out (8 + len + 4 limbs)
template <int LEN>
SECP_FN void sc_fold(const uint32_t* lo, const uint32_t* hi, uint32_t* out) {
    constexpr int OL = 8 + LEN + 4;
    const uint32_t nc[5] = {NC0, NC1, NC2, NC3, 1u};
    for (int i = 0; i < OL; ++i) out[i] = i < 8 ? lo[i] : 0u;
#pragma unroll
    for (int i = 0; i < LEN; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            uint64_t x = (uint64_t)hi[i] * nc[j] + out[i + j] + c;
            out[i + j] = (uint32_t)x;
            c = x >> 32;
        }
#pragma unroll
        for (int k = i + 5; k < OL; ++k) {
            c += out[k];
            out[k] = (uint32_t)c;
            c >>= 32;
        }
    }
}
SECP_FN U256 sc_reduce_wide(const uint32_t t[16]) {
    uint32_t a[20], b[17], c[14];
    sc_fold<8>(t, t + 8, a);        // < 2^386: 13 limbs used
    sc_fold<5>(a, a + 8, b);        // < 2^260: 9 limbs used
    sc_fold<1>(b, b + 8, c);        // < 2^256 + 2^133
    U256 r;
    for (int i = 0; i < 8; ++i) r.v[i] = c[i];
    if (c[8]) {                     // one more 2^256 -> 2^256 - n (r is tiny then)
        const uint32_t e[1] = {c[8]};
        uint32_t d[13];
        sc_fold<1>(c, e, d);
        for (int i = 0; i < 8; ++i) r.v[i] = d[i];
    }
    U256 s;
    if (!u_sub(s, r, c_n())) r = s;
    if (!u_sub(s, r, c_n())) r = s;
    return r;
}
SECP_FN U256 sc_mul(const U256& a, const U256& b) {
    SECP_COUNT(2);
    uint32_t t[16];
    u_mul_wide(t, a, b);
    return sc_reduce_wide(t);
}
SECP_FN U256 sc_sqr(const U256& a) {
    SECP_COUNT(3);
    uint32_t t[16];
    u_sqr_wide(t, a);
    return sc_reduce_wide(t);
}
SECP_FN U256 sc_add(const U256& a, const U256& b) {
    U256 r, s;
    uint32_t c = u_add(r, a, b);
    uint32_t br = u_sub(s, r, c_n());
    return (c || !br) ? s : r;
}
SECP_FN U256 sc_neg(const U256& a) {
    if (u_is_zero(a)) return a;
    U256 r;
    u_sub(r, c_n(), a);
    return r;
}
// x mod n for x < 2^256
SECP_FN U256 sc_from_u256(const U256& a) {
    U256 s;
    return u_sub(s, a, c_n()) ? a : s;
}
// a^(n-2) (Fermat): sliding-window chain over the constant exponent (generated offline: 252 squarings,
// 58 multiplications by the odd powers u1..u15, all at compile-time-constant indices, so no scratch)
SECP_FN U256 sc_sqr_n(U256 a, int n) {
    for (int i = 0; i < n; ++i) a = sc_sqr(a);
    return a;
}
SECP_FN U256 sc_inv(const U256& a) {
    const U256 u1 = a;
    const U256 u2 = sc_sqr(a);
    const U256 u3 = sc_mul(u2, u1), u5 = sc_mul(u3, u2), u7 = sc_mul(u5, u2), u9 = sc_mul(u7, u2);
    const U256 u11 = sc_mul(u9, u2), u13 = sc_mul(u11, u2), u15 = sc_mul(u13, u2);
    U256 r = u15;
    for (int i = 0; i < 30; ++i) r = sc_mul(sc_sqr_n(r, 4), u15);   // the run of ones at the top
    r = sc_mul(sc_sqr_n(r, 3), u7);
    r = sc_mul(sc_sqr_n(r, 5), u11);
    r = sc_mul(sc_sqr_n(r, 3), u5);
    r = sc_mul(sc_sqr_n(r, 4), u5);
    r = sc_mul(sc_sqr_n(r, 4), u7);
    r = sc_mul(sc_sqr_n(r, 5), u13);
    r = sc_mul(sc_sqr_n(r, 2), u3);
    r = sc_mul(sc_sqr_n(r, 5), u7);
    r = sc_mul(sc_sqr_n(r, 6), u13);
    r = sc_mul(sc_sqr_n(r, 5), u11);
    r = sc_mul(sc_sqr_n(r, 4), u13);
    r = sc_mul(sc_sqr_n(r, 3), u1);
    r = sc_mul(sc_sqr_n(r, 6), u5);
    r = sc_mul(sc_sqr_n(r, 10), u7);
    r = sc_mul(sc_sqr_n(r, 4), u7);
    r = sc_mul(sc_sqr_n(r, 5), u15);
    r = sc_mul(sc_sqr_n(r, 4), u15);
    r = sc_mul(sc_sqr_n(r, 5), u9);
    r = sc_mul(sc_sqr_n(r, 6), u11);
    r = sc_mul(sc_sqr_n(r, 4), u13);
    r = sc_mul(sc_sqr_n(r, 5), u3);
    r = sc_mul(sc_sqr_n(r, 6), u13);
    r = sc_mul(sc_sqr_n(r, 10), u13);
    r = sc_mul(sc_sqr_n(r, 4), u9);
    r = sc_mul(sc_sqr_n(r, 9), u9);
    r = sc_mul(sc_sqr_n(r, 4), u15);
    r = sc_mul(sc_sqr_n(r, 1), u1);
    return r;
}

// ------------------------------------------------------------------------------ points (a = 0)
struct Jac {
    U256 x, y, z;
    uint32_t inf;
};
struct Aff {
    U256 x, y;
};
SECP_FN Jac jac_inf() { Jac r; r.x = u_small(1); r.y = u_small(1); r.z = u_zero(); r.inf = 1; return r; }
SECP_FN Jac jac_from_aff(const Aff& a) { Jac r; r.x = a.x; r.y = a.y; r.z = u_small(1); r.inf = 0; return r; }

// dbl-2009-l: 2M + 5S
SECP_FN Jac jac_dbl(const Jac& p) {
    if (p.inf) return p;
    U256 A = fe_sqr(p.x);
    U256 B = fe_sqr(p.y);
    U256 C = fe_sqr(B);
    U256 t = fe_sqr(fe_add(p.x, B));
    t = fe_sub(fe_sub(t, A), C);
    U256 D = fe_add(t, t);
    U256 E = fe_add(fe_add(A, A), A);
    U256 F = fe_sqr(E);
    Jac r;
    r.x = fe_sub(F, fe_add(D, D));
    U256 C8 = fe_add(C, C);
    C8 = fe_add(C8, C8);
    C8 = fe_add(C8, C8);
    r.y = fe_sub(fe_mul(E, fe_sub(D, r.x)), C8);
    U256 yz = fe_mul(p.y, p.z);
    r.z = fe_add(yz, yz);
    r.inf = u_is_zero(p.y) ? 1u : 0u;     // (cannot happen on secp256k1: no point of order 2)
    return r;
}
// madd-2007-bl: p + q with q affine (7M + 4S)
SECP_FN Jac jac_add_aff(const Jac& p, const Aff& q) {
    if (p.inf) return jac_from_aff(q);
    U256 Z1Z1 = fe_sqr(p.z);
    U256 U2 = fe_mul(q.x, Z1Z1);
    U256 S2 = fe_mul(q.y, fe_mul(p.z, Z1Z1));
    U256 H = fe_sub(U2, p.x);
    U256 rr = fe_sub(S2, p.y);
    if (u_is_zero(H)) {
        if (u_is_zero(rr)) return jac_dbl(p);
        return jac_inf();
    }
    rr = fe_add(rr, rr);
    U256 HH = fe_sqr(H);
    U256 I = fe_add(HH, HH);
    I = fe_add(I, I);
    U256 J = fe_mul(H, I);
    U256 V = fe_mul(p.x, I);
    Jac r;
    r.x = fe_sub(fe_sub(fe_sqr(rr), J), fe_add(V, V));
    U256 yj = fe_mul(p.y, J);
    r.y = fe_sub(fe_mul(rr, fe_sub(V, r.x)), fe_add(yj, yj));
    r.z = fe_sub(fe_sub(fe_sqr(fe_add(p.z, H)), Z1Z1), HH);
    r.inf = 0;
    return r;
}
// add-2007-bl: general Jacobian addition (11M + 5S)
SECP_FN Jac jac_add(const Jac& p, const Jac& q) {
    if (p.inf) return q;
    if (q.inf) return p;
    U256 Z1Z1 = fe_sqr(p.z), Z2Z2 = fe_sqr(q.z);
    U256 U1 = fe_mul(p.x, Z2Z2), U2 = fe_mul(q.x, Z1Z1);
    U256 S1 = fe_mul(p.y, fe_mul(q.z, Z2Z2)), S2 = fe_mul(q.y, fe_mul(p.z, Z1Z1));
    U256 H = fe_sub(U2, U1);
    U256 rr = fe_sub(S2, S1);
    if (u_is_zero(H)) {
        if (u_is_zero(rr)) return jac_dbl(p);
        return jac_inf();
    }
    rr = fe_add(rr, rr);
    U256 H2 = fe_add(H, H);
    U256 I = fe_sqr(H2);
    U256 J = fe_mul(H, I);
    U256 V = fe_mul(U1, I);
    Jac r;
    r.x = fe_sub(fe_sub(fe_sqr(rr), J), fe_add(V, V));
    U256 sj = fe_mul(S1, J);
    r.y = fe_sub(fe_mul(rr, fe_sub(V, r.x)), fe_add(sj, sj));
    U256 zz = fe_sub(fe_sub(fe_sqr(fe_add(p.z, q.z)), Z1Z1), Z2Z2);
    r.z = fe_mul(zz, H);
    r.inf = 0;
    return r;
}
SECP_FN bool jac_to_aff(const Jac& p, Aff& a) {
    if (p.inf) return false;
    U256 zi = fe_inv(p.z);
    U256 zi2 = fe_sqr(zi);
    a.x = fe_mul(p.x, zi2);
    a.y = fe_mul(p.y, fe_mul(zi2, zi));
    return true;
}

// fixed-base table: tbl[w*255 + (j-1)] = j * 2^(8w) * G (affine), w < 32, 1 <= j <= 255
constexpr uint32_t GTAB_WINDOWS = 32, GTAB_ENTRIES = 255;
constexpr uint32_t GTAB_POINTS = GTAB_WINDOWS * GTAB_ENTRIES;

// acc + k * G (acc = infinity by default; recover passes u2 * R, saving the final general addition)
SECP_FN Jac mul_g(const U256& k, const Aff* gtab, Jac acc = jac_inf()) {
    // window w's byte from a copy shifted right by 8 per window: u_byte(k, w) at a loop-variable w indexes the
    // limbs dynamically, which puts k in scratch memory
    U256 t = k;
    for (uint32_t w = 0; w < GTAB_WINDOWS; ++w) {
        const uint32_t j = t.v[0] & 255u;
#pragma unroll
        for (int i = 0; i < 7; ++i) t.v[i] = (t.v[i] >> 8) | (t.v[i + 1] << 24);
        t.v[7] >>= 8;
        if (j) acc = jac_add_aff(acc, gtab[w * GTAB_ENTRIES + (j - 1)]);
    }
    return acc;
}
// GLV endomorphism (secp256k1 has lambda * (x, y) = (beta * x, y)): k = k1 + k2 * lambda (mod n) with
// |k1|, |k2| < 2^128 (libsecp256k1's lattice constants; checked in tests/test_sig_cpu.py), so
// k * P = k1 * P + k2 * (lambda P) takes 128 doublings instead of 256.
SECP_FN U256 c_lambda() { return U256{{0x1B23BD72u, 0xDF02967Cu, 0x20816678u, 0x122E22EAu, 0x8812645Au, 0xA5261C02u, 0xC05C30E0u, 0x5363AD4Cu}}; }
SECP_FN U256 c_beta() { return U256{{0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u, 0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu}}; }
SECP_FN U256 c_g1() { return U256{{0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u, 0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u}}; }
SECP_FN U256 c_g2() { return U256{{0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu, 0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u}}; }
SECP_FN U256 c_mb1() { return U256{{0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u, 0u, 0u, 0u, 0u}}; }
SECP_FN U256 c_mb2() { return U256{{0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}}; }
// round(k * g / 2^384)
SECP_FN U256 mul_shift_384(const U256& k, const U256& g) {
    uint32_t t[16];
    u_mul_wide(t, k, g);
    U256 r = u_zero();
    uint64_t c = (uint64_t)(t[11] >> 31);
    for (int i = 0; i < 4; ++i) { c += t[12 + i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[4] = (uint32_t)c;
    return r;
}
SECP_FN void split_lambda(const U256& k, U256& r1, U256& r2) {
    const U256 c1 = mul_shift_384(k, c_g1()), c2 = mul_shift_384(k, c_g2());
    r2 = sc_add(sc_mul(c1, c_mb1()), sc_mul(c2, c_mb2()));
    r1 = sc_add(k, sc_neg(sc_mul(r2, c_lambda())));
}
// Radix-8 signed digits of a GLV half k (|k| < 2^128): k' = k + 4 * (8^43 - 1) / 7 < 2^130, then
// k = top * 2^129 + sum_{i < 43} d_i 8^i with d_i = ((k' >> 3i) & 7) - 4 in [-4, 3] and top = k' >> 129
SECP_FN uint32_t r8_digit(const U256& kp, uint32_t i) {        // (k' >> 3i) & 7, i < 43
    const uint32_t b = 3u * i, w = b >> 5, o = b & 31u;
    const uint32_t lo = kp.v[w] >> o;
    const uint32_t hi = (o > 29u && w < 7u) ? (kp.v[w + 1] << (32u - o)) : 0u;
    return (lo | hi) & 7u;
}
SECP_FN U256 r8_bias() {                                       // 4 * (8^43 - 1) / 7 = 0b100100...100 (43 x '100')
    U256 r = u_zero();
    for (uint32_t i = 0; i < 43; ++i) {
        const uint32_t b = 3u * i + 2u;
        r.v[b >> 5] |= 1u << (b & 31u);
    }
    return r;
}
// entry j (0..3, lane-varying) of the affine table by selects: a dynamic index into a register array
// would put the whole table in scratch memory (round 2: 944 B/lane for an 8-point Jacobian table)
SECP_FN Aff aff_select4(const Aff& t0, const Aff& t1, const Aff& t2, const Aff& t3, uint32_t j) {
    Aff r;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t x01 = (j & 1u) ? t1.x.v[k] : t0.x.v[k], x23 = (j & 1u) ? t3.x.v[k] : t2.x.v[k];
        const uint32_t y01 = (j & 1u) ? t1.y.v[k] : t0.y.v[k], y23 = (j & 1u) ? t3.y.v[k] : t2.y.v[k];
        r.x.v[k] = (j & 2u) ? x23 : x01;
        r.y.v[k] = (j & 2u) ? y23 : y01;
    }
    return r;
}
// The table 1q..4q of mul_var: in registers, selected by value (TabRegs), or in the workgroup's LDS (TabLds:
// word k of entry j of lane l at w[(16 j + k) * 64 + l], so the lanes' differing j never share a bank), which
// frees the 64 registers the table holds across the doubling chain
struct TabRegs {
    Aff t[4];
    SECP_FN void put(int j, const Aff& a) { t[j] = a; }
    SECP_FN Aff get(uint32_t j) const { return aff_select4(t[0], t[1], t[2], t[3], j); }
    SECP_FN Aff first() const { return t[0]; }
};
struct TabLds {
    uint32_t* w;                                 // the LDS array + this lane
    SECP_FN void put(int j, const Aff& a) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { w[(16 * j + k) * 64] = a.x.v[k]; w[(16 * j + 8 + k) * 64] = a.y.v[k]; }
    }
    SECP_FN Aff get(uint32_t j) const {
        Aff r;
        const uint32_t* b = w + 1024u * j;
#pragma unroll
        for (int k = 0; k < 8; ++k) { r.x.v[k] = b[k * 64]; r.y.v[k] = b[(8 + k) * 64]; }
        return r;
    }
    SECP_FN Aff first() const { return get(0); }
};
// k * P: GLV split, then radix-8 signed digits of both 128-bit halves in one doubling chain (129
// doublings, <= 86 mixed additions). The table 1q..4q is made affine with one shared inversion
// (Montgomery's trick), so every addition is mixed (7M + 4S) and the table is 64 registers selected
// by value, not a scratch-memory array; the lambda table is derived on the fly as (beta x, +-y).
template <class Tab = TabRegs>
SECP_FN Jac mul_var(const U256& k, const Aff& p, Tab tab = Tab{}) {
    U256 k1, k2;
    split_lambda(k, k1, k2);
    const bool n1 = !u_ge(c_nhalf(), k1), n2 = !u_ge(c_nhalf(), k2);
    if (n1) k1 = sc_neg(k1);
    if (n2) k2 = sc_neg(k2);
    Aff q = p;
    if (n1) q.y = fe_neg(q.y);
    const bool flip2 = n1 != n2;                 // lambda table = lambda * (i q), negated when the signs differ
    tab.put(0, q);
    {
        const Jac j1 = jac_dbl(jac_from_aff(q));                 // 2q, 3q, 4q (never infinity: prime order)
        const Jac j2 = jac_add_aff(j1, q);
        const Jac j3 = jac_dbl(j1);
        const U256 c12 = fe_mul(j1.z, j2.z), c123 = fe_mul(c12, j3.z);
        U256 inv = fe_inv(c123);
        const U256 z3 = fe_mul(inv, c12);                         // 1 / z3
        inv = fe_mul(inv, j3.z);                                  // 1 / (z1 z2)
        const U256 z2 = fe_mul(inv, j1.z);
        const U256 z1 = fe_mul(inv, j2.z);
        const U256 z1s = fe_sqr(z1), z2s = fe_sqr(z2), z3s = fe_sqr(z3);
        Aff a;
        a.x = fe_mul(j1.x, z1s); a.y = fe_mul(j1.y, fe_mul(z1s, z1)); tab.put(1, a);
        a.x = fe_mul(j2.x, z2s); a.y = fe_mul(j2.y, fe_mul(z2s, z2)); tab.put(2, a);
        a.x = fe_mul(j3.x, z3s); a.y = fe_mul(j3.y, fe_mul(z3s, z3)); tab.put(3, a);
    }
    const U256 bias = r8_bias();
    U256 k1p, k2p;
    u_add(k1p, k1, bias);
    u_add(k2p, k2, bias);
    const U256 beta = c_beta();
    Jac acc = jac_inf();
    if ((k1p.v[4] >> 1) & 1u) acc = jac_add_aff(acc, tab.first());   // bit 129: top = 1
    if ((k2p.v[4] >> 1) & 1u) {
        Aff t = tab.first();
        t.x = fe_mul(t.x, beta);
        if (flip2) t.y = fe_neg(t.y);
        acc = jac_add_aff(acc, t);
    }
    // digits from the top (w = 42 .. 0) out of copies shifted left by 3 per step: bits 126..128 of the copy are
    // digit w (r8_digit at a loop-variable w indexes the limbs dynamically: scratch memory)
    uint32_t s1[5], s2[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) { s1[i] = k1p.v[i]; s2[i] = k2p.v[i]; }
#pragma unroll 1
    for (int w = 42; w >= 0; --w) {
        if (!acc.inf) { acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc); }
        const uint32_t r1 = ((s1[3] >> 30) | (s1[4] << 2)) & 7u, r2 = ((s2[3] >> 30) | (s2[4] << 2)) & 7u;
#pragma unroll
        for (int i = 4; i > 0; --i) { s1[i] = (s1[i] << 3) | (s1[i - 1] >> 29); s2[i] = (s2[i] << 3) | (s2[i - 1] >> 29); }
        s1[0] <<= 3;
        s2[0] <<= 3;
        const int d1 = (int)r1 - 4;
        if (d1 != 0) {
            Aff t = tab.get((uint32_t)((d1 > 0 ? d1 : -d1) - 1));
            if (d1 < 0) t.y = fe_neg(t.y);
            acc = jac_add_aff(acc, t);
        }
        const int d2 = (int)r2 - 4;
        if (d2 != 0) {
            Aff t = tab.get((uint32_t)((d2 > 0 ? d2 : -d2) - 1));
            t.x = fe_mul(t.x, beta);
            if ((d2 < 0) != flip2) t.y = fe_neg(t.y);
            acc = jac_add_aff(acc, t);
        }
    }
    return acc;
}

// ------------------------------------------------------------------------------ SHA-256 / HMAC
SECP_FN uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
BFT_FN void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
    const uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = blk[i];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            uint32_t s0 = ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3);
            uint32_t s1 = ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
            w[i & 15] = wi;
        }
        uint32_t S1 = ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K[i] + wi;
        uint32_t S0 = ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
SECP_FN void sha256_init(uint32_t st[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}
// streaming SHA-256 over big-endian 32-bit words and single bytes (message lengths here < 2^16)
struct Sha256 {
    uint32_t st[8];
    uint32_t blk[16];
    uint32_t nbytes;
    SECP_FN void init() { sha256_init(st); nbytes = 0; for (int i = 0; i < 16; ++i) blk[i] = 0; }
    SECP_FN void byte(uint32_t b) {
        uint32_t pos = nbytes & 63u;
        uint32_t sh = 24u - 8u * (pos & 3u);
        blk[pos >> 2] = (pos & 3u) == 0 ? (b << sh) : (blk[pos >> 2] | (b << sh));
        ++nbytes;
        if ((nbytes & 63u) == 0) sha256_compress(st, blk);
    }
    SECP_FN void words(const uint32_t* w, int n) {       // n big-endian words (byte-aligned or not)
        for (int i = 0; i < n; ++i) {
            if ((nbytes & 3u) == 0) {
                blk[(nbytes & 63u) >> 2] = w[i];
                nbytes += 4;
                if ((nbytes & 63u) == 0) sha256_compress(st, blk);
            } else {
                byte(w[i] >> 24); byte((w[i] >> 16) & 255u); byte((w[i] >> 8) & 255u); byte(w[i] & 255u);
            }
        }
    }
    SECP_FN void final(uint32_t out[8]) {
        uint64_t bits = (uint64_t)nbytes * 8u;
        byte(0x80u);
        while ((nbytes & 63u) != 56u) byte(0);
        uint32_t hi = (uint32_t)(bits >> 32), lo = (uint32_t)bits;
        words(&hi, 1);
        words(&lo, 1);
        for (int i = 0; i < 8; ++i) out[i] = st[i];
    }
};
// HMAC-SHA256 with a 32-byte key (8 BE words) over V (8 words) || [sep byte] || [64 data bytes], the three
// shapes RFC 6979 uses (sep without data, neither, both). Blocks are laid out by compile-time positions and the
// compressions run in one loop with ONE sha256_compress site: the streaming Sha256 above indexes its block by
// the running byte count, and separate non-inlined calls pass their arrays through the stack -- both scratch
// memory on the device (sig_sign_kernel had 368 B/lane).
BFT_FN void hmac_kv(const uint32_t key[8], const uint32_t v[8], int sep, const uint32_t* data16, uint32_t out[8]) {
    uint32_t st[8], inner[8], d[16];
    const bool has_d = data16 != nullptr;
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = has_d ? data16[i] : 0u;
    const uint32_t sb = (uint32_t)sep & 0xffu;
    // steps: 0 key^ipad | 1 V... | 2 the rest of D (with data only) | 3 key^opad | 4 inner hash
#pragma unroll 1
    for (uint32_t step = 0; step < 5u; ++step) {
        if ((step == 2u) & !has_d) continue;
        if (step == 3u) {
#pragma unroll
            for (int i = 0; i < 8; ++i) inner[i] = st[i];
        }
        if ((step == 0u) | (step == 3u)) sha256_init(st);
        uint32_t blk[16];
        if ((step == 0u) | (step == 3u)) {
            const uint32_t pad = step == 0u ? 0x36363636u : 0x5c5c5c5cu;
#pragma unroll
            for (int i = 0; i < 8; ++i) { blk[i] = key[i] ^ pad; blk[8 + i] = pad; }
        } else if (step == 1u) {
#pragma unroll
            for (int i = 0; i < 8; ++i) blk[i] = v[i];
            if (has_d) {                              // V || sep || D[0..30]
                blk[8] = (sb << 24) | (d[0] >> 8);
#pragma unroll
                for (int j = 1; j < 8; ++j) blk[8 + j] = (d[j - 1] << 24) | (d[j] >> 8);
            } else {                                  // V [|| sep] + padding: the last block
                blk[8] = sep >= 0 ? (sb << 24) | 0x00800000u : 0x80000000u;
#pragma unroll
                for (int k = 9; k < 15; ++k) blk[k] = 0;
                blk[15] = (64u + 32u + (sep >= 0 ? 1u : 0u)) * 8u;
            }
        } else if (step == 2u) {                      // D[31..63] + padding (97 inner bytes after the key block)
#pragma unroll
            for (int k = 0; k < 8; ++k) blk[k] = (d[7 + k] << 24) | (d[8 + k] >> 8);
            blk[8] = (d[15] << 24) | 0x00800000u;
#pragma unroll
            for (int k = 9; k < 15; ++k) blk[k] = 0;
            blk[15] = (64u + 97u) * 8u;
        } else {                                      // the inner hash + padding
#pragma unroll
            for (int i = 0; i < 8; ++i) blk[i] = inner[i];
            blk[8] = 0x80000000u;
#pragma unroll
            for (int k = 9; k < 15; ++k) blk[k] = 0;
            blk[15] = (64u + 32u) * 8u;
        }
        sha256_compress(st, blk);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = st[i];
}
// RFC 6979 HMAC-DRBG as libsecp256k1's nonce_function_rfc6979 drives it (key32 || msg32 mod n). Each phase is a
// loop over one hmac_kv site (inlined once per phase).
struct Rfc6979 {
    uint32_t K[8], V[8];
    bool retry;
    SECP_FN void init(const U256& d, const U256& e_mod_n) {
        uint32_t kd[16];
        for (int i = 0; i < 8; ++i) { kd[i] = d.v[7 - i]; kd[8 + i] = e_mod_n.v[7 - i]; }
        for (int i = 0; i < 8; ++i) { V[i] = 0x01010101u; K[i] = 0; }
        // K = HMAC_K(V || 0x00 || kd); V = HMAC_K(V); K = HMAC_K(V || 0x01 || kd); V = HMAC_K(V)
#pragma unroll 1
        for (int s = 0; s < 4; ++s) {
            uint32_t t[8];
            const bool to_k = (s & 1) == 0;
            hmac_kv(K, V, to_k ? s >> 1 : -1, to_k ? kd : nullptr, t);
#pragma unroll
            for (int i = 0; i < 8; ++i) { K[i] = to_k ? t[i] : K[i]; V[i] = to_k ? V[i] : t[i]; }
        }
        retry = false;
    }
    SECP_FN U256 next() {
        // a retry first: K = HMAC_K(V || 0x00), V = HMAC_K(V); then V = HMAC_K(V)
#pragma unroll 1
        for (int s = retry ? 0 : 2; s < 3; ++s) {
            uint32_t t[8];
            const bool to_k = s == 0;
            hmac_kv(K, V, to_k ? 0 : -1, nullptr, t);
#pragma unroll
            for (int i = 0; i < 8; ++i) { K[i] = to_k ? t[i] : K[i]; V[i] = to_k ? V[i] : t[i]; }
        }
        retry = true;
        U256 k;
        for (int i = 0; i < 8; ++i) k.v[i] = V[7 - i];
        return k;
    }
};

// ------------------------------------------------------------------------------ Keccak address
// public_to_address: Keccak-256(X || Y)[12:32] (X, Y big-endian 32 bytes each)
SECP_FN uint32_t bswap32(uint32_t x) { return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24); }
SECP_FN void pub_address(const Aff& q, uint8_t addr[20]) {
    // little-endian 64-bit word i of X || Y (big-endian): bytes 8i..8i+7 = BE limbs 7-2i and 6-2i, byte-swapped
    uint64_t a[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) a[i] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = (uint64_t)bswap32(q.x.v[7 - 2 * i]) | ((uint64_t)bswap32(q.x.v[6 - 2 * i]) << 32);
        a[4 + i] = (uint64_t)bswap32(q.y.v[7 - 2 * i]) | ((uint64_t)bswap32(q.y.v[6 - 2 * i]) << 32);
    }
    a[8] ^= 0x01ull;                 // pad10*1 at byte 64, rate 136
    a[16] ^= 0x80ull << 56;
    keccak_f1600(a);
#pragma unroll
    for (int i = 12; i < 32; ++i) addr[i - 12] = (uint8_t)(a[i >> 3] >> (8 * (i & 7)));
}

// ------------------------------------------------------------------------------ ECDSA
// secret -> public key; false for an invalid secret (0 or >= n)
SECP_FN bool secret_to_pub(const uint8_t* sec32, const Aff* gtab, Aff& q) {
    U256 d = u_from_be(sec32);
    if (u_is_zero(d) || u_ge(d, c_n())) return false;
    return jac_to_aff(mul_g(d, gtab), q);
}
// recoverable signature r || s || recid of a 32-byte digest (libsecp256k1 ecdsa_sign_recoverable)
SECP_FN bool sign(const uint8_t* sec32, const uint8_t* msg32, const Aff* gtab, uint8_t sig[65]) {
    U256 d = u_from_be(sec32);
    if (u_is_zero(d) || u_ge(d, c_n())) return false;
    U256 e = sc_from_u256(u_from_be(msg32));
    Rfc6979 rng;
    rng.init(d, e);
    for (int tries = 0; tries < 64; ++tries) {
        U256 k = rng.next();
        if (u_is_zero(k) || u_ge(k, c_n())) continue;
        Aff R;
        if (!jac_to_aff(mul_g(k, gtab), R)) continue;
        uint32_t recid = R.y.v[0] & 1u;
        U256 r = R.x;
        if (u_ge(r, c_n())) { U256 t; u_sub(t, r, c_n()); r = t; recid |= 2u; }
        U256 s = sc_mul(sc_inv(k), sc_add(e, sc_mul(r, d)));
        if (u_is_zero(r) || u_is_zero(s)) continue;
        if (!u_ge(c_nhalf(), s)) { s = sc_neg(s); recid ^= 1u; }
        u_to_be(r, sig);
        u_to_be(s, sig + 32);
        sig[64] = (uint8_t)recid;
        return true;
    }
    return false;
}
// public key of a recoverable signature (libsecp256k1 ecdsa_recover); false if invalid
template <class Tab = TabRegs>
SECP_FN bool recover(const uint8_t* msg32, const uint8_t* sig65, const Aff* gtab, Aff& q, Tab tab = Tab{}) {
    U256 r = u_from_be(sig65), s = u_from_be(sig65 + 32);
    uint32_t recid = sig65[64];
    if (recid > 3u || u_is_zero(r) || u_is_zero(s) || u_ge(r, c_n()) || u_ge(s, c_n())) return false;
    U256 x = r;
    if (recid & 2u) {
        if (u_add(x, r, c_n())) return false;
        if (u_ge(x, c_p())) return false;
    }
    U256 y2 = fe_add(fe_mul(fe_sqr(x), x), u_small(7));
    U256 y = fe_sqrt(y2);
    if (!u_eq(fe_sqr(y), y2)) return false;
    if ((y.v[0] & 1u) != (recid & 1u)) y = fe_neg(y);
    Aff R;
    R.x = x;
    R.y = y;
    U256 e = sc_from_u256(u_from_be(msg32));
    U256 rinv = sc_inv(r);
    U256 u1 = sc_neg(sc_mul(e, rinv));
    U256 u2 = sc_mul(s, rinv);
    Jac Q = mul_g(u1, gtab, mul_var(u2, R, tab));      // u1 G + u2 R, G's additions onto u2 R
    return jac_to_aff(Q, q);
}

// host: build the fixed-base table (affine), gtab[GTAB_POINTS]
inline void build_gtab(Aff* gtab) {
    Aff base;
    base.x = c_gx();
    base.y = c_gy();
    for (uint32_t w = 0; w < GTAB_WINDOWS; ++w) {
        Jac acc = jac_from_aff(base);
        gtab[w * GTAB_ENTRIES] = base;
        for (uint32_t j = 2; j <= GTAB_ENTRIES; ++j) {
            acc = jac_add_aff(acc, base);
            jac_to_aff(acc, gtab[w * GTAB_ENTRIES + (j - 1)]);
        }
        // next window base: 256 * base
        Jac b = jac_from_aff(base);
        for (int i = 0; i < 8; ++i) b = jac_dbl(b);
        jac_to_aff(b, base);
    }
}

}  // namespace secp
}  // namespace bft
