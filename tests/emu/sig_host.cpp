// sig_host.cpp — TEST-ONLY host build of consensus-rs_amd/csrc/secp256k1.h (the exact source the
// gfx950 kernels run), so the CPU suite can check its arithmetic against oracle/secp256k1_ref.py
// without a GPU. Never linked into the product library.
#include <stdint.h>
#include <string.h>

#include <vector>

#define SECP_COUNT_OPS
#include "../../consensus-rs_amd/csrc/secp256k1.h"

uint64_t bft::secp::secp_op_count[4];

using namespace bft::secp;

static std::vector<Aff>& gtab() {
    static std::vector<Aff> t;
    if (t.empty()) {
        t.resize(GTAB_POINTS);
        build_gtab(t.data());
    }
    return t;
}

extern "C" {
// multiplications since the last call (fe_mul, fe_sqr, sc_mul, sc_sqr)
void sig_host_counts(uint64_t out[4]) {
    for (int i = 0; i < 4; ++i) { out[i] = secp_op_count[i]; secp_op_count[i] = 0; }
}
// field / scalar primitives on big-endian 32-byte operands (op: 0 fe_mul, 1 fe_sqr, 2 fe_add, 3 fe_sub,
// 4 fe_inv, 5 fe_sqrt, 6 sc_mul, 7 sc_inv, 8 sc_add, 9 sc_neg)
void sig_host_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
    U256 x = u_from_be(a), y = u_from_be(b), r = u_zero();
    switch (op) {
        case 0: r = fe_mul(x, y); break;
        case 1: r = fe_sqr(x); break;
        case 2: r = fe_add(x, y); break;
        case 3: r = fe_sub(x, y); break;
        case 4: r = fe_inv(x); break;
        case 5: r = fe_sqrt(x); break;
        case 6: r = sc_mul(x, y); break;
        case 7: r = sc_inv(x); break;
        case 8: r = sc_add(x, y); break;
        case 9: r = sc_neg(x); break;
        default: break;
    }
    u_to_be(r, out);
}
void sig_host_sha256(const uint8_t* data, uint32_t len, uint8_t out[32]) {
    Sha256 s;
    s.init();
    for (uint32_t i = 0; i < len; ++i) s.byte(data[i]);
    uint32_t o[8];
    s.final(o);
    for (int i = 0; i < 8; ++i) { out[4 * i] = o[i] >> 24; out[4 * i + 1] = o[i] >> 16; out[4 * i + 2] = o[i] >> 8; out[4 * i + 3] = o[i]; }
}
// first `count` RFC 6979 nonces (32 bytes each)
void sig_host_nonces(const uint8_t* sec, const uint8_t* msg, uint32_t count, uint8_t* out) {
    Rfc6979 g;
    g.init(u_from_be(sec), sc_from_u256(u_from_be(msg)));
    for (uint32_t i = 0; i < count; ++i) u_to_be(g.next(), out + 32 * i);
}
int sig_host_pub(const uint8_t* sec, uint8_t pub[64], uint8_t addr[20]) {
    Aff q;
    if (!secret_to_pub(sec, gtab().data(), q)) return 0;
    u_to_be(q.x, pub);
    u_to_be(q.y, pub + 32);
    pub_address(q, addr);
    return 1;
}
int sig_host_mul_var(const uint8_t* k, const uint8_t* pub, uint8_t out[64]) {
    Aff p;
    p.x = u_from_be(pub);
    p.y = u_from_be(pub + 32);
    Aff q;
    if (!jac_to_aff(mul_var(u_from_be(k), p), q)) return 0;
    u_to_be(q.x, out);
    u_to_be(q.y, out + 32);
    return 1;
}
int sig_host_sign(const uint8_t* sec, const uint8_t* msg, uint8_t sig[65]) { return sign(sec, msg, gtab().data(), sig) ? 1 : 0; }
int sig_host_recover(const uint8_t* msg, const uint8_t* sig, uint8_t pub[64], uint8_t addr[20]) {
    Aff q;
    if (!recover(msg, sig, gtab().data(), q)) return 0;
    u_to_be(q.x, pub);
    u_to_be(q.y, pub + 32);
    pub_address(q, addr);
    return 1;
}
}
