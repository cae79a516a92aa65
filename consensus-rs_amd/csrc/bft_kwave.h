// bft_kwave.h — the block hash of one header computed by ONE wavefront, for the kernels whose proposer
// depends on the previous block hash (little-endian U128 seeds: validator.rs:33-48 `fn_selector` reads
// prev_hash[0..8]), so the hash of height x is needed before height x + 1 starts.
//
// Keccak-f[1600] over 50 lanes: lane l < 50 holds half (l & 1) of state word w = l >> 1 (w = x + 5y,
// SPEC.md §7 Keccak-256). Every VALU instruction then works on all 50 halves at once (the 25-lane form of
// bft_wave.h keccak_wave needs two per step); the 64-bit rotations take the partner half by one DPP
// quad swap (lanes 2w, 2w + 1 share a quad) and one v_alignbit_b32. Cross-word moves are ds_bpermute
// pulls with lane-constant addresses: theta's four column neighbours, its two x-neighbours, pi, and chi's
// two x-neighbours (9 per round). Lanes 50..63 compute values no valid lane reads.
//
// The header (SPEC.md §7, the byte layout of bft_common.h HdrWriter) is encoded by the lanes in parallel:
// lanes 0..31 own prev_hash byte l, lanes 32..63 tx_hash byte l - 32 (the only variable-length parts:
// a byte >= 128 is `0xcc b`); their positions are ballot prefix counts. The fixed fields are written by
// lanes from small per-lane tables, into an LDS buffer of 3 rate blocks, then read back as message words.
#pragma once
#include "bft_common.h"

namespace bft {

constexpr uint32_t KW_BUF_BYTES = LANE_HASH_BUF;     // 3 rate blocks (a header is at most 274 bytes)

// rho amount of word w (Keccak rotation offsets r[x + 5y])
BFT_FN uint32_t kw50_rho(uint32_t w) {
    const uint64_t R0 = 0ull | 1ull << 6 | 62ull << 12 | 28ull << 18 | 27ull << 24 | 36ull << 30 | 44ull << 36 |
                        6ull << 42 | 55ull << 48 | 20ull << 54;
    const uint64_t R1 = 3ull | 10ull << 6 | 43ull << 12 | 25ull << 18 | 39ull << 24 | 41ull << 30 | 45ull << 36 |
                        15ull << 42 | 21ull << 48 | 8ull << 54;
    const uint64_t R2 = 18ull | 2ull << 6 | 61ull << 12 | 56ull << 18 | 14ull << 24;
    const uint64_t v = w < 10u ? R0 : (w < 20u ? R1 : R2);
    return (uint32_t)(v >> (6u * (w % 10u))) & 63u;
}

BFT_FN uint32_t kw50_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {   // ((hi:lo) >> (s & 31)) low 32
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31u));
#endif
}

// Keccak-f[1600] over the wave (layout above): `a` = this lane's half word, in place
template <class W>
BFT_FN void kw50_permute(W& wv, uint32_t lane, uint32_t& a) {
    const uint32_t ln = lane < 50u ? lane : 0u;
    const uint32_t w = ln >> 1, hf = ln & 1u, x = w % 5u, y = w / 5u;
    // ds_bpermute byte addresses of the sources, same half
    auto at = [&](uint32_t xx, uint32_t yy) -> uint32_t { return 4u * (2u * (xx + 5u * yy) + hf); };
    const uint32_t p1 = at(x, (y + 1u) % 5u), p2 = at(x, (y + 2u) % 5u), p3 = at(x, (y + 3u) % 5u),
                   p4 = at(x, (y + 4u) % 5u);
    const uint32_t pxm = at((x + 4u) % 5u, y), pxp = at((x + 1u) % 5u, y), pxp2 = at((x + 2u) % 5u, y);
    const uint32_t ppi = at((3u * y + x) % 5u, x);   // pi: B[y][2x+3y] = A[x][y], pulled by its destination
    // rho at the source word: rotl(r) of (this half, partner half) = alignbit(first, second, s)
    const uint32_t r = kw50_rho(w);
    const bool swp = (r == 0u) | (r > 32u);
    const uint32_t s = ((r == 0u) | (r == 32u)) ? 0u : (r < 32u ? 32u - r : 64u - r);
    const bool io_lo = lane == 0u, io_hi = lane == 1u;
#pragma unroll 1
    for (int rnd = 0; rnd < 24; ++rnd) {
        // theta: C[x] (this half), E[x] = rotl1(C[x]), A ^= C[x-1] ^ E[x+1]
        const uint32_t c = a ^ wv.bperm(p1, a) ^ wv.bperm(p2, a) ^ wv.bperm(p3, a) ^ wv.bperm(p4, a);
        const uint32_t e = kw50_alignbit(c, wv.pair_swap(c), 31u);
        a ^= wv.bperm(pxm, c) ^ wv.bperm(pxp, e);
        // rho (at the source) + pi (pulled)
        const uint32_t ap = wv.pair_swap(a);
        const uint32_t rot = kw50_alignbit(swp ? ap : a, swp ? a : ap, s);
        const uint32_t b = wv.bperm(ppi, rot);
        // chi
        const uint32_t b1 = wv.bperm(pxp, b), b2 = wv.bperm(pxp2, b);
        a = b ^ (~b1 & b2);
        // iota
        a ^= (io_lo ? KECCAK_RC_LO[rnd] : 0u) | (io_hi ? KECCAK_RC_HI[rnd] : 0u);
    }
}

// compact MessagePack uint (HdrWriter::put_uint): its length and its byte i
BFT_FN uint32_t kw50_uint_len(uint64_t v) {
    return v < 128u ? 1u : v < 256u ? 2u : v < 65536u ? 3u : v < 4294967296ull ? 5u : 9u;
}
BFT_FN uint32_t kw50_uint_byte(uint64_t v, uint32_t len, uint32_t i) {
    if (len == 1u) return (uint32_t)v;
    if (i == 0u) return len == 2u ? 0xccu : len == 3u ? 0xcdu : len == 5u ? 0xceu : 0xcfu;
    return (uint32_t)(v >> (8u * (len - 1u - i))) & 0xffu;        // big-endian payload
}

// Keccak-256 of the header of block (h, prop, var) at `time` whose parent hash is `prev_w` (lane l < 8
// holds its little-endian word l), by the whole wave; `buf` = KW_BUF_BYTES of this wave's LDS, 8-aligned.
// Returns the hash the same way (lane l < 8: word l; the other lanes: unspecified).
template <class W>
BFT_FN uint32_t kw50_header_hash(W& wv, uint32_t lane, uint8_t* buf, uint32_t prev_w, const uint8_t* addr20,
                                 uint64_t seed, uint32_t inst, uint32_t h, uint32_t prop, uint32_t var,
                                 uint64_t time) {
    // the 64 variable-length elements: prev_hash byte l (l < 32) and tx_hash byte l - 32 (SPEC.md §5 TX)
    const uint32_t pw = wv.bperm(4u * ((lane & 31u) >> 2), prev_w);
    uint32_t tw[4];
    philox(seed, inst, h, (prop << 8) | var, lane >= 48u ? DOM_TX2 : DOM_TX, tw);
    const uint32_t tsel = (lane >> 2) & 3u;
    const uint32_t txw = tsel == 0u ? tw[0] : tsel == 1u ? tw[1] : tsel == 2u ? tw[2] : tw[3];
    const uint32_t eb = ((lane < 32u ? pw : txw) >> (8u * (lane & 3u))) & 0xffu;
    const bool big = eb >= 128u;
    const uint64_t bal = wv.ballot(big);
    const uint32_t prev_big = (uint32_t)__builtin_popcountll(bal & 0xffffffffull);
    const uint32_t tx_big = (uint32_t)__builtin_popcountll(bal >> 32);
    const uint32_t rank = wv.rank_below(bal) - (lane >= 32u ? prev_big : 0u);
    // field offsets (HdrWriter order, types/block.rs:16-36)
    const uint32_t o_addr = 4u + 32u + prev_big, o_root = o_addr + 44u, o_txp = o_root + 35u, o_tx = o_txp + 3u;
    const uint32_t o_rec = o_tx + 32u + tx_big, o_tail = o_rec + 35u;
    const uint32_t hl = kw50_uint_len(h), tl = kw50_uint_len(time);
    const uint32_t o_h = o_tail + 2u, o_t = o_h + hl + 2u, o_e = o_t + tl;
    const uint32_t len = o_e + 13u;                                  // "Coinse base" (11 + 1) + votes nil
    const uint32_t nb = len / 136u + 1u;
    // zero the rate blocks, then the bytes
    if (lane < KW_BUF_BYTES / 8u) ((uint64_t*)buf)[lane] = 0ull;
    wv.sync();
    {   // element bytes: 0xcc prefix for bytes >= 128
        const uint32_t off = (lane < 32u ? 4u + lane : o_tx + lane - 32u) + rank;
        buf[off] = (uint8_t)(big ? 0xccu : eb);
        if (big) buf[off + 1u] = (uint8_t)eb;
    }
    if (lane < 44u) {   // proposer: str8 "0x" + 40 lowercase hex digits
        const uint32_t j = lane - 4u;
        uint32_t v = lane == 0u ? 0xd9u : lane == 1u ? 0x2au : lane == 2u ? 0x30u : 0x78u;
        if (lane >= 4u) {
            const uint32_t ab = addr20[j >> 1];
            v = hexdigit((j & 1u) ? (ab & 15u) : (ab >> 4));
        }
        buf[o_addr + lane] = (uint8_t)v;
    }
    {   // the other non-zero fixed bytes, one per lane: array headers, height, time, extra, votes, padding
        uint32_t off = 0, v = 0;
        bool wr = true;
        const uint32_t k = lane;
        if (k == 0u) { off = 0u; v = 0x9du; }                      // array(13)
        else if (k == 1u) { off = 1u; v = 0xdcu; }                 // prev_hash: array16(32)
        else if (k == 2u) { off = 3u; v = 0x20u; }
        else if (k == 3u) { off = o_root; v = 0xdcu; }             // root = EMPTY_HASH
        else if (k == 4u) { off = o_root + 2u; v = 0x20u; }
        else if (k == 5u) { off = o_txp; v = 0xdcu; }              // tx_hash
        else if (k == 6u) { off = o_txp + 2u; v = 0x20u; }
        else if (k == 7u) { off = o_rec; v = 0xdcu; }              // receipt_hash = EMPTY_HASH
        else if (k == 8u) { off = o_rec + 2u; v = 0x20u; }
        else if (k < 14u) {                                        // height (<= 5 bytes)
            const uint32_t i = k - 9u;
            wr = i < hl; off = o_h + i; v = kw50_uint_byte(h, hl, i);
        } else if (k < 23u) {                                      // time (<= 9 bytes)
            const uint32_t i = k - 14u;
            wr = i < tl; off = o_t + i; v = kw50_uint_byte(time, tl, i);
        } else if (k < 36u) {                                      // extra "Coinse base" + votes nil
            const uint32_t i = k - 23u;
            const uint64_t E0 = 0x2065736e696f439bull, E1 = 0xc065736162ull;
            off = o_e + i; v = (uint32_t)((i < 8u ? E0 >> (8u * i) : E1 >> (8u * (i - 8u))) & 0xffu);
        } else if (k == 36u) {                                     // pad10*1, Keccak domain 0x01
            off = len; v = 0x01u | (len == 136u * nb - 1u ? 0x80u : 0u);
        } else if (k == 37u) {
            off = 136u * nb - 1u; v = 0x80u | (len == 136u * nb - 1u ? 0x01u : 0u);
        } else {
            wr = false;
        }
        if (wr) buf[off] = (uint8_t)v;
    }
    wv.sync();
    // absorb + permute: lane l < 34 takes 32-bit word l of each rate block
    uint32_t a = 0;
    for (uint32_t blk = 0; blk < nb; ++blk) {
        if (lane < 34u) a ^= ((const uint32_t*)buf)[34u * blk + lane];
        kw50_permute(wv, lane, a);
    }
    wv.sync();
    return a;
}

}  // namespace bft
