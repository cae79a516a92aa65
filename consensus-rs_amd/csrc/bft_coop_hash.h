// bft_coop_hash.h — one wavefront computes one Keccak-256 header hash cooperatively.
//
// Layout: state word A[x + 5y] lives in lane 8x + y (x, y < 5); the other 39 lanes hold 0.
//   theta: column parity = xor-butterfly over the 8 lanes of a column group (shfl_xor 1, 2, 4);
//   rho:   every lane rotates its own word by its own offset;
//   pi:    one gather (lane (X, Y) reads lane (3Y + X mod 5, X));
//   chi:   two gathers from (X+1, Y), (X+2, Y);
//   iota:  lane 0.
// The MessagePack header of SPEC.md §7 is assembled in an LDS byte buffer by all lanes at once:
// each of lanes 0..31 places one prev_hash byte and one tx_hash byte at offsets given by a
// ballot prefix count of the bytes >= 128 (which take two bytes, 0xcc + byte). All functions are
// collectives: every lane of the wave calls them with uniform arguments.
#pragma once
#include "bft_common.h"

namespace bft {

constexpr uint32_t COOP_BUF_BYTES = 3 * 136;   // up to 3 rate blocks (max header 274 bytes)

template <class W>
struct Coop {
    BFT_FN static uint64_t shfl64(uint64_t v, uint32_t src) {
        uint32_t lo = W::shfl((uint32_t)v, src), hi = W::shfl((uint32_t)(v >> 32), src);
        return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    BFT_FN static uint64_t xor64(uint64_t v, int m) {
        uint32_t lo = W::shfl_xor((uint32_t)v, m), hi = W::shfl_xor((uint32_t)(v >> 32), m);
        return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    BFT_FN static uint64_t rotl_var(uint64_t v, uint32_t n) {
        return n == 0 ? v : ((v << n) | (v >> (64u - n)));
    }

    // rho offsets r[x + 5y] (Keccak reference)
    BFT_FN static uint32_t rho(uint32_t i) {
        const uint8_t R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                               25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
        return i < 25 ? R[i] : 0;
    }

    BFT_FN static void keccak_f(uint64_t& a, uint32_t lane) {
        const uint64_t RC[24] = {
            0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
            0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
            0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
            0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
            0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
            0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
        const uint32_t x = lane >> 3, y = lane & 7;
        const bool valid = x < 5 && y < 5;
        const uint32_t xm = x < 5 ? x : 0, ym = y < 5 ? y : 0;
        const uint32_t src_dm1 = 8u * ((xm + 4u) % 5u), src_dp1 = 8u * ((xm + 1u) % 5u);
        const uint32_t src_pi = 8u * ((3u * ym + xm) % 5u) + xm;     // (X, Y) = (x, y) here
        const uint32_t src_c1 = 8u * ((xm + 1u) % 5u) + ym, src_c2 = 8u * ((xm + 2u) % 5u) + ym;
        // the rotation a source lane applies before pi: r of its own (x, y)
        const uint32_t my_rho = valid ? rho(xm + 5u * ym) : 0u;
        if (!valid) a = 0;
        for (int rnd = 0; rnd < 24; ++rnd) {
            uint64_t c = a;
            c ^= xor64(c, 1);
            c ^= xor64(c, 2);
            c ^= xor64(c, 4);                       // C[x] in every lane of column group x
            uint64_t cm1 = shfl64(c, src_dm1), cp1 = shfl64(c, src_dp1);
            a ^= cm1 ^ rotl_var(cp1, 1);
            uint64_t t = rotl_var(a, my_rho);
            uint64_t b = shfl64(t, src_pi);
            uint64_t b1 = shfl64(b, src_c1), b2 = shfl64(b, src_c2);
            a = b ^ (~b1 & b2);
            if (lane == 0) a ^= RC[rnd];
            if (!valid) a = 0;
        }
    }

    // Byte j (0..31) of a 32-byte hash whose little-endian 64-bit words are held by lanes
    // 0, 8, 16, 24 (the first four state words after a permutation).
    BFT_FN static uint32_t hash_byte(uint64_t a, uint32_t lane) {
        uint32_t j = lane & 31u;
        uint64_t w = shfl64(a, 8u * (j >> 3));
        return (uint32_t)(w >> (8u * (j & 7u))) & 0xffu;
    }

    // Keccak-256 of the candidate header (SPEC.md §7). `prev` = the previous hash as a state
    // (lanes 0, 8, 16, 24). Returns the new hash state in `a` (same convention).
    BFT_FN static void header_hash(uint64_t& a, uint64_t prev, uint8_t* buf, uint32_t lane,
                                   const uint8_t* addr20, uint64_t seed, uint32_t inst, uint32_t h,
                                   uint32_t prop, uint32_t var, uint64_t time) {
        // --- inputs of lanes 0..31: prev byte j and tx byte j
        uint32_t pb = hash_byte(prev, lane);
        uint32_t j = lane & 31u;
        uint32_t w4[4];
        philox(seed, inst, h, (prop << 8) | var, (j < 16) ? DOM_TX : DOM_TX2, w4);
        uint32_t wi = (j >> 2) & 3u;
        uint32_t tw = wi == 0 ? w4[0] : wi == 1 ? w4[1] : wi == 2 ? w4[2] : w4[3];
        uint32_t tb = (tw >> (8u * (j & 3u))) & 0xffu;
        bool lo32 = lane < 32;
        uint64_t bigp = W::ballot(lo32 && pb >= 128u) & 0xffffffffull;
        uint64_t bigt = W::ballot(lo32 && tb >= 128u) & 0xffffffffull;
        uint32_t np = (uint32_t)__builtin_popcountll(bigp), nt = (uint32_t)__builtin_popcountll(bigt);
        uint64_t below = (lane & 31u) ? ((1ull << (lane & 31u)) - 1ull) : 0ull;
        uint32_t offp = 4u + j + (uint32_t)__builtin_popcountll(bigp & below);
        const uint32_t Pa = 1u + 35u + np;            // address
        const uint32_t Pr = Pa + 44u;                 // root
        const uint32_t Pt = Pr + 35u;                 // tx_hash
        uint32_t offt = Pt + 3u + j + (uint32_t)__builtin_popcountll(bigt & below);
        const uint32_t Prc = Pt + 35u + nt;           // receipt
        const uint32_t Pb = Prc + 35u;                // bloom, difficulty
        const uint32_t Ph = Pb + 2u;
        const uint32_t Lh = h < 128u ? 1u : h < 256u ? 2u : h < 65536u ? 3u : 5u;
        const uint32_t Pg = Ph + Lh;
        const uint32_t Ptm = Pg + 2u;
        const uint32_t Lt = time < 128ull ? 1u : time < 256ull ? 2u : time < 65536ull ? 3u
                          : time < 4294967296ull ? 5u : 9u;
        const uint32_t Pe = Ptm + Lt;
        const uint32_t L = Pe + 12u + 1u;             // + votes nil
        const uint32_t nb = L / 136u + 1u;
        // --- zero the buffer
        uint32_t* bw = (uint32_t*)buf;
        for (uint32_t k = lane; k < COOP_BUF_BYTES / 4u; k += 64u) bw[k] = 0u;
        W::sync();
        // --- scatter bytes
        if (lo32) {
            if (pb >= 128u) { buf[offp] = 0xcc; buf[offp + 1] = (uint8_t)pb; } else buf[offp] = (uint8_t)pb;
            if (tb >= 128u) { buf[offt] = 0xcc; buf[offt + 1] = (uint8_t)tb; } else buf[offt] = (uint8_t)tb;
        }
        if (lane < 40u) {                             // address hex digits
            uint32_t ab = addr20[lane >> 1];
            uint32_t nib = (lane & 1u) ? (ab & 15u) : (ab >> 4);
            buf[Pa + 4u + lane] = (uint8_t)hexdigit(nib);
        }
        if (lane == 40) {
            buf[0] = 0x9d; buf[1] = 0xdc; buf[2] = 0x00; buf[3] = 0x20;
            buf[Pa] = 0xd9; buf[Pa + 1] = 42; buf[Pa + 2] = '0'; buf[Pa + 3] = 'x';
        }
        if (lane == 41) {
            buf[Pr] = 0xdc; buf[Pr + 1] = 0x00; buf[Pr + 2] = 0x20;
            buf[Pt] = 0xdc; buf[Pt + 1] = 0x00; buf[Pt + 2] = 0x20;
            buf[Prc] = 0xdc; buf[Prc + 1] = 0x00; buf[Prc + 2] = 0x20;
        }
        if (lane == 42) {                             // height (bloom, difficulty, gas: zeros)
            if (Lh == 1) buf[Ph] = (uint8_t)h;
            else if (Lh == 2) { buf[Ph] = 0xcc; buf[Ph + 1] = (uint8_t)h; }
            else if (Lh == 3) { buf[Ph] = 0xcd; buf[Ph + 1] = (uint8_t)(h >> 8); buf[Ph + 2] = (uint8_t)h; }
            else { buf[Ph] = 0xce; for (int i = 0; i < 4; ++i) buf[Ph + 1 + i] = (uint8_t)(h >> (24 - 8 * i)); }
        }
        if (lane == 43) {                             // time
            if (Lt == 1) buf[Ptm] = (uint8_t)time;
            else if (Lt == 2) { buf[Ptm] = 0xcc; buf[Ptm + 1] = (uint8_t)time; }
            else if (Lt == 3) { buf[Ptm] = 0xcd; buf[Ptm + 1] = (uint8_t)(time >> 8); buf[Ptm + 2] = (uint8_t)time; }
            else if (Lt == 5) { buf[Ptm] = 0xce; for (int i = 0; i < 4; ++i) buf[Ptm + 1 + i] = (uint8_t)(time >> (24 - 8 * i)); }
            else { buf[Ptm] = 0xcf; for (int i = 0; i < 8; ++i) buf[Ptm + 1 + i] = (uint8_t)(time >> (56 - 8 * i)); }
        }
        if (lane >= 48u && lane < 60u) {              // extra = "Coinse base" as an array, then votes
            const char* ex = "\x9b" "Coinse base";
            buf[Pe + (lane - 48u)] = (uint8_t)ex[lane - 48u];
        }
        if (lane == 60) buf[Pe + 12u] = 0xc0;
        W::sync();
        if (lane == 0) {                              // pad10*1, Keccak domain byte 0x01
            buf[L] ^= 0x01;
            buf[136u * nb - 1u] ^= 0x80;
        }
        W::sync();
        // --- absorb
        const uint32_t x = lane >> 3, y = lane & 7;
        const uint32_t wi2 = x + 5u * y;
        const bool rate_lane = x < 5 && y < 5 && wi2 < 17u;
        a = 0;
        for (uint32_t b = 0; b < nb; ++b) {
            if (rate_lane) {
                const uint32_t* p = (const uint32_t*)(buf + 136u * b + 8u * wi2);
                a ^= (uint64_t)p[0] | ((uint64_t)p[1] << 32);
            }
            keccak_f(a, lane);
        }
        W::sync();
    }
};

}  // namespace bft

namespace bft {

// Post-pass body: one wave hashes the committed chain of one instance, height by height,
// chaining prev_hash (power-of-two N; SPEC.md §7). Collective over the wave.
template <class W>
BFT_FN void hash_chain_wave(const Params& p, uint32_t il, uint8_t* buf) {
    const uint32_t lane = W::lane();
    if (il >= p.n_instances) return;
    const uint32_t inst = p.first_instance + il;
    const uint32_t ch = p.committed_height[il];
    uint64_t prev = 0;
    if ((lane & 7u) == 0 && lane < 32u) {
        const uint8_t* g = p.genesis_hash + 8u * (lane >> 3);
        for (int b = 0; b < 8; ++b) prev |= (uint64_t)g[b] << (8 * b);
    }
    for (uint32_t x = 1; x <= ch; ++x) {
        const uint32_t* row = p.rec + ((uint64_t)il * p.rows + x) * 4;
        uint32_t w1 = row[1];
        uint32_t prop = w1 & 0xffffu, var = (w1 >> 16) & 1u, T = row[2];
        uint64_t time = p.genesis_time + (uint64_t)p.block_period * ((uint64_t)T + 1ull);
        uint64_t a;
        Coop<W>::header_hash(a, prev, buf, lane, p.addresses + 20u * prop, p.seed, inst, x, prop, var, time);
        if ((lane & 7u) == 0 && lane < 32u) {
            uint32_t* dst = (uint32_t*)(p.hash + ((uint64_t)il * p.rows + x) * 32) + 2u * (lane >> 3);
            dst[0] = (uint32_t)a;
            dst[1] = (uint32_t)(a >> 32);
        }
        prev = a;
    }
}

}  // namespace bft
