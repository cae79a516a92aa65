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

// the Keccak round constants as compile-time halves (immediates in the unrolled rounds)
constexpr uint32_t KW_RC_LO[24] = {
    0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u, 0x80008081u, 0x00008009u,
    0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au, 0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u,
    0x00008002u, 0x00000080u, 0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
constexpr uint32_t KW_RC_HI[24] = {
    0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0x80000000u, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0x80000000u,
    0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u, 0x80000000u, 0x80000000u, 0u, 0x80000000u};

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
BFT_FN __attribute__((always_inline)) void kw50_permute(W& wv, uint32_t lane, uint32_t& a) {
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
    // iota masks: the round constant goes to lanes 0 (low half) and 1 (high half) of word 0
    const uint32_t m_lo = lane == 0u ? 0xffffffffu : 0u, m_hi = lane == 1u ? 0xffffffffu : 0u;
    // fully unrolled: the round constants become immediates (no per-round table load, no loop branch)
#pragma unroll
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
        a ^= (KW_RC_LO[rnd] & m_lo) | (KW_RC_HI[rnd] & m_hi);
    }
}

// compact MessagePack uint (HdrWriter::put_uint): its length and its byte i
BFT_FN uint32_t kw50_uint_len(uint64_t v) {
    return v < 128u ? 1u : v < 256u ? 2u : v < 65536u ? 3u : v < 4294967296ull ? 5u : 9u;
}
BFT_FN uint32_t kw50_uint_byte(uint64_t v, uint32_t len, uint32_t i) {    // selects only (per-lane i)
    const uint32_t tag = len == 2u ? 0xccu : len == 3u ? 0xcdu : len == 5u ? 0xceu : 0xcfu;
    const uint32_t sh = 8u * ((len - 1u - i) & 7u);
    const uint32_t pay = (uint32_t)(v >> sh) & 0xffu;                  // big-endian payload
    return len == 1u ? (uint32_t)v & 0xffu : (i == 0u ? tag : pay);
}

// Keccak-256 of the header of block (h, prop, var) at `time` whose parent hash is `prev_w` (lane l < 8
// holds its little-endian word l), by the whole wave; `buf` = KW_BUF_BYTES of this wave's LDS, 8-aligned.
// Returns the hash the same way (lane l < 8: word l; the other lanes: unspecified).
template <class W>
BFT_FN __attribute__((always_inline)) uint32_t kw50_header_hash(W& wv, uint32_t lane, uint8_t* buf, uint32_t prev_w, const uint8_t* addr20,
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
    {   // proposer: str8 "0x" + 40 lowercase hex digits, lanes 0..43 (selects; one predicated store)
        const uint32_t j = lane >= 4u ? lane - 4u : 0u;
        const uint32_t ab = addr20[(j >> 1) < 20u ? (j >> 1) : 19u];
        const uint32_t hx = hexdigit((j & 1u) ? (ab & 15u) : (ab >> 4));
        const uint32_t v = lane == 0u ? 0xd9u : lane == 1u ? 0x2au : lane == 2u ? 0x30u : lane == 3u ? 0x78u : hx;
        if (lane < 44u) buf[o_addr + lane] = (uint8_t)v;
    }
    {   // the other non-zero fixed bytes, one per lane k (selects; one predicated store): array headers (k < 9),
        // height (9..13), time (14..22), extra + votes (23..35), padding (36, 37)
        const uint32_t k = lane;
        const uint32_t pair = (k + 1u) >> 1;
        const uint32_t hb_off = (pair == 1u ? 1u : pair == 2u ? o_root : pair == 3u ? o_txp : o_rec) + ((k & 1u) ? 0u : 2u);
        const uint32_t hb_v = (k & 1u) ? 0xdcu : 0x20u;
        const uint32_t ih = k - 9u, it = k - 14u, ie = k - 23u;
        const uint64_t E0 = 0x2065736e696f439bull, E1 = 0xc065736162ull;
        const uint32_t ev = (uint32_t)((ie < 8u ? E0 >> (8u * (ie & 7u)) : E1 >> (8u * ((ie - 8u) & 7u))) & 0xffu);
        const bool last_byte = len == 136u * nb - 1u;
        uint32_t off = k == 0u ? 0u : hb_off, v = k == 0u ? 0x9du : hb_v;
        bool wr = k < 9u;
        const bool in_h = (k >= 9u) & (k < 14u), in_t = (k >= 14u) & (k < 23u), in_e = (k >= 23u) & (k < 36u);
        off = in_h ? o_h + ih : off;  v = in_h ? kw50_uint_byte(h, hl, ih) : v;  wr = in_h ? ih < hl : wr;
        off = in_t ? o_t + it : off;  v = in_t ? kw50_uint_byte(time, tl, it) : v;  wr = in_t ? it < tl : wr;
        off = in_e ? o_e + ie : off;  v = in_e ? ev : v;  wr = in_e | wr;
        off = k == 36u ? len : off;  v = k == 36u ? (0x01u | (last_byte ? 0x80u : 0u)) : v;   // pad10*1
        off = k == 37u ? 136u * nb - 1u : off;  v = k == 37u ? (0x80u | (last_byte ? 0x01u : 0u)) : v;
        wr = wr | (k == 36u) | (k == 37u);
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

// ---- the prev_hash chain of one instance by ONE wave (small shards: bft_hash_chain_wave_kernel) ----
// The block-hash pass of a launch is a chain per instance, sequential in height (prev_hash). With few
// instances per GPU the chains run one lone wave per SIMD, and a chain's latency is the launch's: the
// lane-pair chain issues ~130 dependent VALU per Keccak round (~600 cycles for a lone wave). Here the 50
// lanes of kw50_permute take one round in ~4 dependent ds_bpermute levels instead. Per height:
//   * the suffix row (bft_hash_suffix_kernel, header bytes after prev_hash, loaded one height ahead) goes
//     into the splice buffer `sb` at dword SFX_PAD, as the lane-pair chain's splice (bft_common.h);
//   * the prefix (array header + prev_hash as MessagePack array16 of 32 uints, 36..68 bytes) is written
//     byte-wise into `pf` by lanes 0..35: lane e < 32 owns prev_hash byte e (`0xcc b` for b >= 128, at
//     4 + e + the count of such bytes below it: a ballot prefix count);
//   * lane l < 34 absorbs message dword 34 blk + l = align_bytes of the splice buffer | the prefix dword.
// `srow`: dword k of the first height's suffix row at srow[k * stride], height j at + j * rstride;
// `a_prev`: lane l < 8 holds the parent's hash dword l; `hdst`: the first height's hash row (8 dwords),
// height j at + 8 j. Same bytes as spliced_block_hash (tests/test_emu_parity.py: emu_wave_chain_check).
constexpr uint32_t KW_PFX_DW = 18;
template <class W>
BFT_FN __attribute__((always_inline)) void kw50_chain(W& wv, uint32_t lane, uint32_t* sb, uint32_t* pf,
                                                     const uint32_t* srow, uint64_t rstride, uint32_t stride,
                                                     uint32_t a_prev, uint32_t nx, uint32_t* hdst) {
    for (uint32_t i = lane; i < SFX_BUF; i += 64u) sb[i] = 0u;
    wv.sync();
    uint32_t s = lane < SFX_DEV_DW ? srow[(uint64_t)lane * stride] : 0u;
    uint8_t* pb = (uint8_t*)pf;
    const uint32_t hdr = 0x2000dc9du;                     // array(13); prev_hash: array16(32)
    for (uint32_t j = 0; j < nx; ++j) {
        if (lane < KW_PFX_DW) pf[lane] = 0u;
        if (lane < SFX_BODY_DW) sb[SFX_PAD + lane] = s;
        const uint32_t len_s = wv.readlane(s, SFX_DEV_LEN_DW);
        if ((j + 1u < nx) & (lane < SFX_DEV_DW)) s = srow[(uint64_t)(j + 1u) * rstride + (uint64_t)lane * stride];
        const uint32_t pw = wv.bperm(4u * ((lane >> 2) & 7u), a_prev);
        const uint32_t eb = (pw >> (8u * (lane & 3u))) & 0xffu;
        const bool big = (lane < 32u) & (eb >= 128u);
        const uint64_t bal = wv.ballot(big);
        const uint32_t rank = wv.rank_below(bal);
        const uint32_t nbig = (uint32_t)__builtin_popcountll(bal);
        wv.sync();                                        // pf zeroed before the byte writes
        if (lane < 32u) {
            const uint32_t off = 4u + lane + rank;
            pb[off] = (uint8_t)(big ? 0xccu : eb);
            if (big) pb[off + 1u] = (uint8_t)eb;
        } else if (lane < 36u) {
            pb[lane - 32u] = (uint8_t)(hdr >> (8u * (lane - 32u)));
        }
        wv.sync();
        const uint32_t len_p = 36u + nbig, c = 72u - len_p, r = c & 3u;
        const uint32_t nb = splice_blocks(len_p, len_s);
        const uint32_t* sx = sb + (c >> 2);
        uint32_t a = 0;
        for (uint32_t blk = 0; blk < nb; ++blk) {
            if (lane < 34u) {
                const uint32_t q = 34u * blk + lane;
                uint32_t v = align_bytes(sx[q + 1u], sx[q], r);
                if (q < KW_PFX_DW) v |= pf[q];
                if (q == 34u * nb - 1u) v ^= 0x80000000u;
                a ^= v;
            }
            kw50_permute(wv, lane, a);
        }
        if (lane < 8u) hdst[8ull * j + lane] = a;
        a_prev = a;
        wv.sync();                                        // this height's LDS reads before the next's writes
    }
}

}  // namespace bft
