/* secp_oracle.c — plain-C CPU restatement of secp256k1 public-key derivation and recovery (SEC 1
 * v2 §4.1.6), the checker and CPU baseline of the GPU recover kernel. TEST INFRASTRUCTURE ONLY
 * (loaded by tests/ and bench.py's cpu_baseline leg, never by the product path).
 *
 * Independent of the GPU code (consensus-rs_amd/csrc/secp256k1.h) by construction: 4 x 64-bit limbs
 * with 128-bit products, a generic fold reduction for both moduli, Fermat inversions by plain
 * square-and-multiply, and textbook double-and-add scalar multiplication (no tables, no windows, no
 * signed digits). Reference call sites: `GossipMessage::address` (src/protocol/mod.rs:103-116),
 * `verify_address` (src/consensus/pbft/core/commit.rs:96-100); the validator addresses of
 * examples/c1.toml pin `orc_secp_pubkey` (tests/test_sig_cpu.py). Address hashing uses the
 * oracle's Keccak (bft_oracle.c).
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t w[4]; } num;   /* little-endian 64-bit limbs */

static const num P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const num NN = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const num GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const num GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

static int n_cmp(const num* a, const num* b) {
    for (int i = 3; i >= 0; --i) {
        if (a->w[i] != b->w[i]) return a->w[i] > b->w[i] ? 1 : -1;
    }
    return 0;
}
static int n_zero(const num* a) { return (a->w[0] | a->w[1] | a->w[2] | a->w[3]) == 0; }
static uint64_t n_add(num* r, const num* a, const num* b) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)a->w[i] + b->w[i]; r->w[i] = (uint64_t)c; c >>= 64; }
    return (uint64_t)c;
}
static uint64_t n_sub(num* r, const num* a, const num* b) {
    uint64_t br = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->w[i] - b->w[i] - br;
        r->w[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1u;
    }
    return br;
}
/* (a + b) mod m, a, b < m */
static num m_add(const num* a, const num* b, const num* m) {
    num r, s;
    uint64_t c = n_add(&r, a, b);
    if (c || n_cmp(&r, m) >= 0) { n_sub(&s, &r, m); return s; }
    return r;
}
static num m_sub(const num* a, const num* b, const num* m) {
    num r, s;
    if (n_sub(&r, a, b)) { n_add(&s, &r, m); return s; }
    return r;
}
/* a * b mod m for m = 2^256 - c (c < 2^130): fold the high half by c until it vanishes */
static num m_mul(const num* a, const num* b, const num* m) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a->w[i] * b->w[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    num cm;                                   /* 2^256 - m */
    num zero = {{0, 0, 0, 0}};
    n_sub(&cm, &zero, m);
    for (;;) {
        int hi_zero = (t[4] | t[5] | t[6] | t[7]) == 0;
        if (hi_zero) break;
        uint64_t u[8] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0};
        for (int i = 0; i < 4; ++i) {           /* u += t_hi * cm */
            u128 c = 0;
            for (int j = 0; j < 4; ++j) {
                c += (u128)t[4 + i] * cm.w[j] + u[i + j];
                u[i + j] = (uint64_t)c;
                c >>= 64;
            }
            for (int k = i + 4; k < 8 && c; ++k) { c += u[k]; u[k] = (uint64_t)c; c >>= 64; }
        }
        memcpy(t, u, sizeof(u));
    }
    num r = {{t[0], t[1], t[2], t[3]}};
    while (n_cmp(&r, m) >= 0) n_sub(&r, &r, m);
    return r;
}
static num m_pow(const num* a, const num* e, const num* m) {
    num r = {{1, 0, 0, 0}};
    for (int i = 255; i >= 0; --i) {
        r = m_mul(&r, &r, m);
        if ((e->w[i >> 6] >> (i & 63)) & 1) r = m_mul(&r, a, m);
    }
    return r;
}
static num m_inv(const num* a, const num* m) {
    num e, two = {{2, 0, 0, 0}};
    n_sub(&e, m, &two);
    return m_pow(a, &e, m);
}

typedef struct { num x, y, z; int inf; } jpt;

static jpt j_dbl(const jpt* p) {
    if (p->inf || n_zero(&p->y)) { jpt r; memset(&r, 0, sizeof r); r.inf = 1; return r; }
    num xx = m_mul(&p->x, &p->x, &P), yy = m_mul(&p->y, &p->y, &P), yyyy = m_mul(&yy, &yy, &P);
    num s = m_mul(&p->x, &yy, &P);
    s = m_add(&s, &s, &P); s = m_add(&s, &s, &P);                 /* S = 4 X Y^2 */
    num mm = m_add(&xx, &xx, &P); mm = m_add(&mm, &xx, &P);        /* M = 3 X^2 */
    jpt r;
    r.inf = 0;
    num t = m_mul(&mm, &mm, &P);
    num s2 = m_add(&s, &s, &P);
    r.x = m_sub(&t, &s2, &P);
    num y8 = m_add(&yyyy, &yyyy, &P); y8 = m_add(&y8, &y8, &P); y8 = m_add(&y8, &y8, &P);
    num d = m_sub(&s, &r.x, &P);
    d = m_mul(&mm, &d, &P);
    r.y = m_sub(&d, &y8, &P);
    num yz = m_mul(&p->y, &p->z, &P);
    r.z = m_add(&yz, &yz, &P);
    return r;
}
static jpt j_add(const jpt* p, const jpt* q) {
    if (p->inf) return *q;
    if (q->inf) return *p;
    num z1z1 = m_mul(&p->z, &p->z, &P), z2z2 = m_mul(&q->z, &q->z, &P);
    num u1 = m_mul(&p->x, &z2z2, &P), u2 = m_mul(&q->x, &z1z1, &P);
    num t1 = m_mul(&q->z, &z2z2, &P), t2 = m_mul(&p->z, &z1z1, &P);
    num s1 = m_mul(&p->y, &t1, &P), s2 = m_mul(&q->y, &t2, &P);
    num h = m_sub(&u2, &u1, &P), rr = m_sub(&s2, &s1, &P);
    if (n_zero(&h)) {
        if (n_zero(&rr)) return j_dbl(p);
        jpt r; memset(&r, 0, sizeof r); r.inf = 1; return r;
    }
    num hh = m_mul(&h, &h, &P), hhh = m_mul(&hh, &h, &P), v = m_mul(&u1, &hh, &P);
    jpt r;
    r.inf = 0;
    num x = m_mul(&rr, &rr, &P);
    x = m_sub(&x, &hhh, &P);
    num v2 = m_add(&v, &v, &P);
    r.x = m_sub(&x, &v2, &P);
    num d = m_sub(&v, &r.x, &P);
    d = m_mul(&rr, &d, &P);
    num sh = m_mul(&s1, &hhh, &P);
    r.y = m_sub(&d, &sh, &P);
    num zz = m_mul(&p->z, &q->z, &P);
    r.z = m_mul(&zz, &h, &P);
    return r;
}
static jpt j_mul(const num* k, const num* x, const num* y) {      /* double-and-add, MSB first */
    jpt acc; memset(&acc, 0, sizeof acc); acc.inf = 1;
    jpt b; b.x = *x; b.y = *y; b.z = (num){{1, 0, 0, 0}}; b.inf = 0;
    for (int i = 255; i >= 0; --i) {
        acc = j_dbl(&acc);
        if ((k->w[i >> 6] >> (i & 63)) & 1) acc = j_add(&acc, &b);
    }
    return acc;
}
static int j_affine(const jpt* p, num* x, num* y) {
    if (p->inf) return 0;
    num zi = m_inv(&p->z, &P), zi2 = m_mul(&zi, &zi, &P), zi3 = m_mul(&zi2, &zi, &P);
    *x = m_mul(&p->x, &zi2, &P);
    *y = m_mul(&p->y, &zi3, &P);
    return 1;
}
static num from_be(const uint8_t* b) {
    num r;
    for (int i = 0; i < 4; ++i) {
        uint64_t v = 0;
        for (int k = 0; k < 8; ++k) v = (v << 8) | b[8 * (3 - i) + k];
        r.w[i] = v;
    }
    return r;
}
static void to_be(const num* a, uint8_t* b) {
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 8; ++k) b[8 * (3 - i) + k] = (uint8_t)(a->w[i] >> (56 - 8 * k));
}

int orc_secp_pubkey(const uint8_t sec[32], uint8_t pub[64]) {
    num d = from_be(sec), x, y;
    if (n_zero(&d) || n_cmp(&d, &NN) >= 0) return 0;
    jpt q = j_mul(&d, &GX, &GY);
    if (!j_affine(&q, &x, &y)) return 0;
    to_be(&x, pub);
    to_be(&y, pub + 32);
    return 1;
}

int orc_secp_recover(const uint8_t msg[32], const uint8_t sig[65], uint8_t pub[64]) {
    num r = from_be(sig), s = from_be(sig + 32);
    int recid = sig[64];
    if (recid > 3 || n_zero(&r) || n_zero(&s) || n_cmp(&r, &NN) >= 0 || n_cmp(&s, &NN) >= 0) return 0;
    num x = r;
    if (recid & 2) {
        if (n_add(&x, &r, &NN) || n_cmp(&x, &P) >= 0) return 0;
    }
    num seven = {{7, 0, 0, 0}};
    num y2 = m_mul(&x, &x, &P);
    y2 = m_mul(&y2, &x, &P);
    y2 = m_add(&y2, &seven, &P);
    num e = {{0xFFFFFFFFBFFFFF0CULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0x3FFFFFFFFFFFFFFFULL}};  /* (p+1)/4 */
    num y = m_pow(&y2, &e, &P);
    num chk = m_mul(&y, &y, &P);
    if (n_cmp(&chk, &y2) != 0) return 0;
    if ((int)(y.w[0] & 1) != (recid & 1)) { num z = {{0, 0, 0, 0}}; y = m_sub(&z, &y, &P); }
    num h = from_be(msg);
    if (n_cmp(&h, &NN) >= 0) n_sub(&h, &h, &NN);
    num ri = m_inv(&r, &NN);
    num z = {{0, 0, 0, 0}};
    num u1 = m_mul(&h, &ri, &NN);
    u1 = m_sub(&z, &u1, &NN);
    num u2 = m_mul(&s, &ri, &NN);
    jpt a = j_mul(&u1, &GX, &GY), b = j_mul(&u2, &x, &y);
    jpt q = j_add(&a, &b);
    num qx, qy;
    if (!j_affine(&q, &qx, &qy)) return 0;
    to_be(&qx, pub);
    to_be(&qy, pub + 32);
    return 1;
}

typedef struct {
    const uint8_t *msgs, *sigs;
    uint8_t *pubs, *ok;
    uint64_t lo, hi;
} rjob;
static void* rwork(void* a) {
    rjob* j = (rjob*)a;
    for (uint64_t i = j->lo; i < j->hi; ++i) j->ok[i] = (uint8_t)orc_secp_recover(j->msgs + 32 * i, j->sigs + 65 * i, j->pubs + 64 * i);
    return 0;
}
/* batch recovery on `threads` POSIX threads (the CPU baseline of bench.py --workload sig) */
void orc_secp_recover_batch(const uint8_t* msgs, const uint8_t* sigs, uint64_t n, uint8_t* pubs, uint8_t* ok, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    rjob jobs[256];
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (rjob){msgs, sigs, pubs, ok, n * (uint64_t)t / threads, n * (uint64_t)(t + 1) / threads};
        pthread_create(&th[t], 0, rwork, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], 0);
}
