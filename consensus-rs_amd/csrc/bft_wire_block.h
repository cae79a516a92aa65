// bft_wire_block.h — the block-carrying frames of the reference's wire format (SPEC.md §9b), as
// emitter / streaming-decoder code shared by the host and the GPU (lane per frame):
//   PrePrepare {view, proposal: Proposal(Block)}        src/consensus/types.rs:17,131-134 (newtype: transparent)
//   Block {header, transactions}, Blocks(Vec<Block>)    src/types/block.rs:16-36,146-155
//   Transaction {nonce, price, gas_limit, recipient, amount, payload, sign}  src/types/transaction.rs:16-30
//   RawMessage {Header{Block | Consensus | Sync, ttl, create_time, peer_id}, payload}  src/p2p/protocol.rs:11-70
// Emitters take a byte functor E; nested Vec<u8> levels wrap it in AsUint (each byte a MessagePack
// uint). Lengths of nested arrays come from a counting pass of the same emitter code.
#pragma once
#include "bft_common.h"
#include "bft_crypto.h"
#include "bft_wire.h"
#include "../../include/bftwire.h"

namespace bft {
namespace wire {

using crypto::mp_arr;
using crypto::mp_uint;

struct CountE {
    uint32_t* n;
    BFT_FN void operator()(uint32_t) const { *n += 1; }
};
struct BufE {                                      // bounded output buffer
    uint8_t* b;
    uint32_t* n;
    uint32_t cap;
    BFT_FN void operator()(uint32_t v) const {
        if (*n < cap) b[*n] = (uint8_t)v;
        *n += 1;
    }
};
template <class E>
struct UintE {                                     // a byte of a Vec<u8>: one MessagePack uint
    const E* in;
    BFT_FN void operator()(uint32_t b) const {
        if (b >= 128u) (*in)(0xccu);
        (*in)(b);
    }
};
struct KE {                                        // into a Keccak-256 absorber
    crypto::KSink* k;
    BFT_FN void operator()(uint32_t b) const { k->put(b); }
};

template <class E>
BFT_FN void emit_bytes(const E& e, const uint8_t* p, uint32_t n) {      // Vec<u8> / Hash / Signature
    mp_arr(e, n);
    for (uint32_t i = 0; i < n; ++i) mp_uint(e, p[i]);
}
template <class E>
BFT_FN void emit_address(const E& e, const uint8_t* a) {                // "0x" + 40 hex digits (str8)
    e(0xd9); e(42); e('0'); e('x');
    for (int i = 0; i < 20; ++i) {
        const uint32_t hi = a[i] >> 4, lo = a[i] & 15u;
        e(hi < 10 ? 48u + hi : 87u + hi);
        e(lo < 10 ? 48u + lo : 87u + lo);
    }
}
template <class E>
BFT_FN void emit_tx(const E& e, const bftwire_tx& t) {
    mp_arr(e, 7);
    mp_uint(e, t.nonce); mp_uint(e, t.price); mp_uint(e, t.gas_limit);
    if (t.has_recipient) emit_address(e, t.recipient); else e(0xc0);
    mp_uint(e, t.amount);
    emit_bytes(e, t.payload, t.payload_len);
    if (t.has_sig) emit_bytes(e, t.sig, 65); else e(0xc0);
}
template <class E>
BFT_FN void emit_header(const E& e, const bftwire_block& b) {
    mp_arr(e, 13);
    emit_bytes(e, b.prev_hash, 32);
    emit_address(e, b.proposer);
    emit_bytes(e, b.root, 32);
    emit_bytes(e, b.tx_hash, 32);
    emit_bytes(e, b.receipt_hash, 32);
    mp_uint(e, b.bloom); mp_uint(e, b.difficulty); mp_uint(e, b.height);
    mp_uint(e, b.gas_limit); mp_uint(e, b.gas_used); mp_uint(e, b.time);
    if (b.extra_len == BFTWIRE_NONE) e(0xc0); else emit_bytes(e, b.extra, b.extra_len);
    if (b.n_votes == BFTWIRE_NONE) { e(0xc0); return; }
    mp_arr(e, b.n_votes);                                   // Votes(Vec<Signature>): newtype, transparent
    for (uint32_t v = 0; v < b.n_votes; ++v) emit_bytes(e, b.votes[v], 65);
}
template <class E>
BFT_FN void emit_block(const E& e, const bftwire_block& b) {
    mp_arr(e, 2);
    emit_header(e, b);
    mp_arr(e, b.n_tx);
    for (uint32_t k = 0; k < b.n_tx; ++k) emit_tx(e, b.tx[k]);
}
BFT_FN bool block_fits(const bftwire_block& b) {
    if (b.extra_len != BFTWIRE_NONE && b.extra_len > BFTWIRE_MAX_EXTRA) return false;
    if (b.n_votes != BFTWIRE_NONE && b.n_votes > BFTWIRE_MAX_VOTES) return false;
    if (b.n_tx > BFTWIRE_MAX_TX) return false;
    for (uint32_t k = 0; k < b.n_tx; ++k)
        if (b.tx[k].payload_len > BFTWIRE_MAX_PAYLOAD) return false;
    return true;
}
template <class E>
BFT_FN void emit_pp_msg(const E& e, const bftwire_preprepare& m) {      // PrePrepare bytes
    mp_arr(e, 2);
    mp_arr(e, 2); mp_uint(e, m.round); mp_uint(e, m.height);
    emit_block(e, m.block);
}
// GossipMessage {Preprepare, create_time, msg, signature, commit_seal: None}; with_sig = false: the
// sign payload (protocol/mod.rs:133-137)
template <class E>
BFT_FN void emit_pp_gossip(const E& e, const bftwire_preprepare& m, bool with_sig) {
    uint32_t ml = 0;
    emit_pp_msg(CountE{&ml}, m);
    mp_arr(e, 5);
    mp_arr(e, 2); mp_uint(e, 0u); mp_arr(e, 0);             // MessageType::Preprepare
    mp_uint(e, m.create_time);
    mp_arr(e, ml);
    emit_pp_msg(UintE<E>{&e}, m);
    if (with_sig && m.has_sig) emit_bytes(e, m.signature, 65); else e(0xc0);
    e(0xc0);
}
// one frame: 4-byte big-endian size || RawMessage {Header{code, ttl, create_time, None}, payload}; the
// payload bytes come from `pl(emitter)`
template <class E, class PL>
BFT_FN void emit_frame(const E& e, uint32_t p2p_code, uint64_t ttl, uint64_t rtime, const PL& pl) {
    uint32_t pn = 0;
    pl(CountE{&pn});
    uint32_t body = 0;
    {
        const CountE c{&body};
        mp_arr(c, 2); mp_arr(c, 4); mp_arr(c, 2); mp_uint(c, p2p_code); mp_arr(c, 0);
        mp_uint(c, ttl); mp_uint(c, rtime); c(0xc0);
        mp_arr(c, pn);
        pl(UintE<CountE>{&c});
    }
    e(body >> 24); e((body >> 16) & 0xffu); e((body >> 8) & 0xffu); e(body & 0xffu);
    mp_arr(e, 2); mp_arr(e, 4); mp_arr(e, 2); mp_uint(e, p2p_code); mp_arr(e, 0);
    mp_uint(e, ttl); mp_uint(e, rtime); e(0xc0);
    mp_arr(e, pn);
    pl(UintE<E>{&e});
}
constexpr uint32_t P2P_BLOCK = 3, P2P_SYNC = 5;          // P2PMsgCode (p2p/protocol.rs:11-18)

// ---------------------------------------------------------------- streaming decoder
template <class S>
BFT_FN bool rd_hex(S& s, uint32_t& v) {
    uint32_t c;
    if (!s.get(c)) return false;
    if (c >= '0' && c <= '9') { v = c - '0'; return true; }
    if (c >= 'a' && c <= 'f') { v = c - 'a' + 10u; return true; }
    if (c >= 'A' && c <= 'F') { v = c - 'A' + 10u; return true; }
    return false;
}
template <class S>
BFT_FN bool rd_address_tag(S& s, uint32_t t, uint8_t* out) {     // str of "0x" + 40 hex digits
    uint32_t len;
    if (t == 0xd9) { uint64_t v; if (!rd_be(s, 1, v)) return false; len = (uint32_t)v; }
    else if ((t & 0xe0u) == 0xa0u) len = t & 31u;
    else if (t == 0xda) { uint64_t v; if (!rd_be(s, 2, v)) return false; len = (uint32_t)v; }
    else return false;
    if (len != 42) return false;
    uint32_t a, b;
    if (!s.get(a) || !s.get(b) || a != '0' || (b != 'x' && b != 'X')) return false;
    for (int i = 0; i < 20; ++i) {
        uint32_t hi, lo;
        if (!rd_hex(s, hi) || !rd_hex(s, lo)) return false;
        out[i] = (uint8_t)((hi << 4) | lo);
    }
    return true;
}
template <class S>
BFT_FN bool rd_bytes_var(S& s, uint32_t t, uint32_t max, uint8_t* out, uint32_t& len) {
    if (!rd_arr_tag(s, t, len) || len > max) return false;
    for (uint32_t i = 0; i < len; ++i) {
        uint64_t v;
        if (!rd_uint(s, v) || v > 255) return false;
        out[i] = (uint8_t)v;
    }
    return true;
}
template <class S>
BFT_FN bool rd_tx(S& s, bftwire_tx& t) {
    uint32_t n, tag;
    if (!rd_arr(s, n) || n != 7) return false;
    if (!rd_uint(s, t.nonce) || !rd_uint(s, t.price) || !rd_uint(s, t.gas_limit)) return false;
    if (!s.get(tag)) return false;
    t.has_recipient = tag != 0xc0;
    if (t.has_recipient && !rd_address_tag(s, tag, t.recipient)) return false;
    if (!rd_uint(s, t.amount)) return false;
    if (!s.get(tag) || !rd_bytes_var(s, tag, BFTWIRE_MAX_PAYLOAD, t.payload, t.payload_len)) return false;
    uint32_t present;
    if (!rd_opt_bytes(s, 65, t.sig, present)) return false;
    t.has_sig = (uint8_t)present;
    return true;
}
template <class S>
BFT_FN bool rd_block(S& s, bftwire_block& b) {
    uint32_t n, hf, tag;
    if (!rd_arr(s, n) || n != 2) return false;
    // extra and votes are #[serde(default)] (types/block.rs:30-33): 11 to 13 fields
    if (!rd_arr(s, hf) || hf < 11 || hf > 13) return false;
    if (!rd_bytes_fixed(s, 32, b.prev_hash) || !s.get(tag) || !rd_address_tag(s, tag, b.proposer)) return false;
    if (!rd_bytes_fixed(s, 32, b.root) || !rd_bytes_fixed(s, 32, b.tx_hash) || !rd_bytes_fixed(s, 32, b.receipt_hash))
        return false;
    if (!rd_uint(s, b.bloom) || !rd_uint(s, b.difficulty) || !rd_uint(s, b.height) || !rd_uint(s, b.gas_limit) ||
        !rd_uint(s, b.gas_used) || !rd_uint(s, b.time))
        return false;
    b.extra_len = BFTWIRE_NONE;
    b.n_votes = BFTWIRE_NONE;
    if (hf >= 12) {
        if (!s.get(tag)) return false;
        if (tag != 0xc0 && !rd_bytes_var(s, tag, BFTWIRE_MAX_EXTRA, b.extra, b.extra_len)) return false;
    }
    if (hf >= 13) {
        if (!s.get(tag)) return false;
        if (tag != 0xc0) {
            uint32_t nv;
            if (!rd_arr_tag(s, tag, nv) || nv > BFTWIRE_MAX_VOTES) return false;
            for (uint32_t v = 0; v < nv; ++v)
                if (!rd_bytes_fixed(s, 65, b.votes[v])) return false;
            b.n_votes = nv;
        }
    }
    if (!rd_arr(s, b.n_tx) || b.n_tx > BFTWIRE_MAX_TX) return false;
    for (uint32_t k = 0; k < b.n_tx; ++k)
        if (!rd_tx(s, b.tx[k])) return false;
    return true;
}
// the RawMessage envelope of a frame: header fields, then an Arr over the payload bytes
template <class M>
BFT_FN bool rd_envelope(M& m, uint32_t want_code, uint64_t& ttl, uint64_t& rtime, uint32_t& plen) {
    uint32_t n, idx, t;
    if (!rd_arr(m, n) || n != 2 || !rd_arr(m, n) || n != 4) return false;
    if (!rd_unit_variant(m, idx) || idx != want_code) return false;
    if (!rd_uint(m, ttl) || !rd_uint(m, rtime) || !m.get(t)) return false;
    if (t != 0xc0) {                                        // peer_id: Some (read, not returned)
        if (!rd_arr_tag(m, t, n) || n > MAX_PEER) return false;
        for (uint32_t i = 0; i < n; ++i) { uint64_t v; if (!rd_uint(m, v) || v > 255) return false; }
    }
    return rd_arr(m, plen);
}
BFT_FN bool decode_pp_frame(const uint8_t* f, uint32_t len, bftwire_preprepare& d) {
    if (len < 4 || frame_size(f) != len - 4u) return false;
    Mem m{f + 4, len - 4u, 0};
    uint32_t plen, gn, idx, mlen;
    if (!rd_envelope(m, P2P_CONSENSUS, d.ttl, d.raw_time, plen)) return false;
    Arr<Mem> g{&m, plen, false};
    if (!rd_arr(g, gn) || gn < 3 || gn > 5) return false;   // signature / commit_seal #[serde(default)]
    if (!rd_unit_variant(g, idx) || idx != 0) return false;  // MessageType::Preprepare
    if (!rd_uint(g, d.create_time) || !rd_arr(g, mlen)) return false;
    Arr<Arr<Mem>> pm{&g, mlen, false};
    uint32_t n;
    if (!rd_arr(pm, n) || n != 2 || !rd_arr(pm, n) || n != 2) return false;
    if (!rd_uint(pm, d.round) || !rd_uint(pm, d.height) || !rd_block(pm, d.block)) return false;
    if (pm.left != 0 || pm.bad) return false;
    uint32_t present = 0;
    uint8_t seal[65];
    if (gn >= 4 && !rd_opt_bytes(g, 65, d.signature, present)) return false;
    d.has_sig = (uint8_t)present;
    if (gn >= 5 && !rd_opt_bytes(g, 65, seal, present)) return false;
    if (g.left != 0 || g.bad) return false;
    return m.i == m.n;
}
BFT_FN bool decode_sync_frame(const uint8_t* f, uint32_t len, uint64_t& height) {
    if (len < 4 || frame_size(f) != len - 4u) return false;
    Mem m{f + 4, len - 4u, 0};
    uint64_t ttl, rt;
    uint32_t plen;
    if (!rd_envelope(m, P2P_SYNC, ttl, rt, plen)) return false;
    Arr<Mem> p{&m, plen, false};
    if (!rd_uint(p, height) || p.left != 0 || p.bad) return false;
    return m.i == m.n;
}

}  // namespace wire
}  // namespace bft
