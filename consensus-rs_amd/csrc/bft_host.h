// bft_host.h — host-side helpers of libbftsim shared with the CPU wave emulator used by the
// tests: Keccak-256, the genesis header hash (core/genesis.rs:44-55), launch parameters.
#pragma once
#include <string.h>
#include <vector>

#include "../../include/bftsim.h"
#include "bft_common.h"

namespace bft {


inline void host_keccak(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint64_t a[25] = {0};
    size_t off = 0;
    uint8_t blk[136];
    for (;;) {
        size_t take = len - off < 136 ? len - off : 136;
        memset(blk, 0, 136);
        memcpy(blk, data + off, take);
        bool last = take < 136;
        if (last) { blk[take] ^= 0x01; blk[135] ^= 0x80; }
        for (int i = 0; i < 17; ++i) {
            uint64_t w = 0;
            for (int b = 0; b < 8; ++b) w |= (uint64_t)blk[8 * i + b] << (8 * b);
            a[i] ^= w;
        }
        keccak_f1600(a);
        off += take;
        if (last) break;
    }
    for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(a[i] >> (8 * b));
}

// genesis header (core/genesis.rs:44-55) in the SPEC.md §7 encoding
inline void host_genesis_hash(const bftsim_config* c, uint8_t out[32]) {
    std::vector<uint8_t> o;
    auto u = [&](uint64_t v) {
        if (v < 128) { o.push_back((uint8_t)v); return; }
        if (v < 256) { o.push_back(0xcc); o.push_back((uint8_t)v); return; }
        if (v < 65536) { o.push_back(0xcd); o.push_back((uint8_t)(v >> 8)); o.push_back((uint8_t)v); return; }
        if (v < 4294967296ull) { o.push_back(0xce); for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(v >> (24 - 8 * i))); return; }
        o.push_back(0xcf);
        for (int i = 0; i < 8; ++i) o.push_back((uint8_t)(v >> (56 - 8 * i)));
    };
    auto zeros32 = [&]() { o.push_back(0xdc); o.push_back(0); o.push_back(32); for (int i = 0; i < 32; ++i) o.push_back(0); };
    static const char hx[] = "0123456789abcdef";
    o.push_back(0x9d);
    zeros32();                                        // prev_hash = EMPTY_HASH
    o.push_back(0xd9); o.push_back(42); o.push_back('0'); o.push_back('x');
    for (int i = 0; i < 20; ++i) { o.push_back((uint8_t)hx[c->genesis_proposer[i] >> 4]); o.push_back((uint8_t)hx[c->genesis_proposer[i] & 15]); }
    zeros32(); zeros32(); zeros32();                  // root, tx_hash, receipt_hash
    u(0); u(0); u(0);                                 // bloom, difficulty, height
    u(c->genesis_gas_used + 10); u(c->genesis_gas_used); u(c->genesis_time);
    const char* ex = "Hello Word!";
    o.push_back(0x9b);
    for (int i = 0; i < 11; ++i) o.push_back((uint8_t)ex[i]);
    o.push_back(0xc0);                                // votes
    host_keccak(o.data(), o.size(), out);
}


// launch parameters from a configuration (pointers are filled by the caller)
inline Params params_from_config(const bftsim_config& c, uint32_t seg, uint32_t hcap, uint32_t genesis_seed,
                                 uint64_t first, uint64_t n) {
    Params p;
    memset(&p, 0, sizeof p);
    p.n = c.n;
    p.seg = seg;
    p.heights = c.heights;
    p.hcap = hcap;
    p.rows = hcap;
    p.max_ticks = c.max_ticks;
    p.block_period = c.block_period;
    p.genesis_time = c.genesis_time;
    p.seed = c.seed;
    p.thr16 = c.drop_ppm ? (uint32_t)(((uint64_t)c.drop_ppm * 65536u + 500000u) / 1000000u) : 0;
    p.byz_count = c.byz_count;
    p.crash_thr32 = (uint32_t)(((uint64_t)c.proposer_crash_ppm << 32) / 1000000u);
    p.crash_on = c.proposer_crash_ppm ? 1u : 0u;
    p.phase_cap = c.phase_cap;
    // the next view's proposer depends on the committed block hash unless the seed is identically 0
    // (big-endian U128 and a power-of-two N, SPEC.md §1)
    p.seed_le = c.seed_byte_order == BFTSIM_SEED_LE ? 1u : 0u;
    p.need_seed = ((c.n & (c.n - 1)) != 0 || (p.seed_le && c.n > 1)) ? 1u : 0u;
    p.backlog_replay = c.backlog_mode == BFTSIM_BACKLOG_REPLAY ? 1u : 0u;
    for (int k = 0; k < 4; ++k) p.silent_mask[k] = c.silent_mask[k];
    p.first_instance = (uint32_t)first;
    p.n_instances = (uint32_t)n;
    p.genesis_seed = genesis_seed;
    p.fast = p.backlog_replay ? 0u : 1u;             // replay mode: one message at a time (SPEC.md §10)
    p.q = (2u * c.n) / 3u;
    p.nmask = (c.n & (c.n - 1)) == 0 ? c.n - 1 : 0;
    p.rcs_k = RCS_DEFAULT_K;
    return p;
}

inline uint32_t segment_size(uint32_t n) {
    uint32_t s = 1;
    while (s < n) s <<= 1;
    return s < 4 ? 4 : s;
}

}  // namespace bft
