// bft_wire.h — the consensus wire format of the reference, as serial encoder / streaming decoder
// code shared by the host and the GPU:
//   Subject       {view: View{round, height}, digest: Hash}             src/consensus/types.rs:60-63,101-104
//   GossipMessage {code, create_time, msg: Vec<u8>, signature, commit_seal}  src/protocol/mod.rs:44-53
//                 (address: skip_serializing); sign_payload = the same with signature = None (:133-137)
//   RawMessage    {header: Header{code: P2PMsgCode, ttl, create_time, peer_id}, payload}
//                                                                        src/p2p/protocol.rs:30-70
//   frame         |size: u32 big-endian| RawMessage bytes |              src/p2p/codec.rs:15-53
// Serialization convention (SPEC.md §9; the reference's `cryptocurrency-kit` serializer is
// unvendored, so the bytes are parity-unpinned against the reference): rmp-serde compact
// MessagePack — a struct is an array of its fields in declaration order; integers in their
// shortest MessagePack form; Vec<u8>, Hash ([u8; 32]) and Signature ([u8; 65]) as arrays of
// integers; Option None as nil, Some(v) as v; an enum unit variant as [variant index, []] (index
// 0-based in declaration order: MessageType Preprepare = 0 .. RoundChange = 3, P2PMsgCode
// Consensus = 4).
#pragma once
#include "bft_common.h"

namespace bft {
namespace wire {

constexpr uint32_t MAX_FRAME = 1028;      // 4-byte size + MAX_MSG_SIZE (codec.rs:12, 1 << 10)
constexpr uint32_t MAX_G = 512;           // GossipMessage bytes of a Subject message (<= 2*70 + 2*(3+130) + 16)
constexpr uint32_t MAX_S = 96;            // Subject bytes (<= 2 + 9 + 9 + 3 + 64)
constexpr uint32_t MAX_PEER = 64;         // peer_id bytes (libp2p PeerId multihash, 34 in practice)
constexpr uint32_t P2P_CONSENSUS = 4;     // P2PMsgCode::Consensus variant index (protocol.rs:10-17)
constexpr uint32_t DEFAULT_TTL = 10;      // p2p/server.rs:187

BFT_FN uint32_t uint_len(uint64_t v) { return v < 128 ? 1u : v < 256 ? 2u : v < 65536 ? 3u : v < (1ull << 32) ? 5u : 9u; }
BFT_FN uint32_t arr_hdr_len(uint32_t n) { return n < 16 ? 1u : n < 65536 ? 3u : 5u; }

// serial writer over a bounded byte buffer (a write past `cap` sets `ovf`)
struct Writer {
    uint8_t* b;
    uint32_t n, cap;
    bool ovf;
    BFT_FN Writer(uint8_t* buf, uint32_t c) : b(buf), n(0), cap(c), ovf(false) {}
    BFT_FN void u8(uint32_t v) {
        if (n < cap) b[n] = (uint8_t)v; else ovf = true;
        ++n;
    }
    BFT_FN void be(uint64_t v, int bytes) { for (int i = bytes - 1; i >= 0; --i) u8((uint32_t)(v >> (8 * i)) & 0xffu); }
    BFT_FN void uint(uint64_t v) {
        if (v < 128) u8((uint32_t)v);
        else if (v < 256) { u8(0xcc); u8((uint32_t)v); }
        else if (v < 65536) { u8(0xcd); be(v, 2); }
        else if (v < (1ull << 32)) { u8(0xce); be(v, 4); }
        else { u8(0xcf); be(v, 8); }
    }
    BFT_FN void arr(uint32_t len) {
        if (len < 16) u8(0x90u | len);
        else if (len < 65536) { u8(0xdc); be(len, 2); }
        else { u8(0xdd); be(len, 4); }
    }
    BFT_FN void nil() { u8(0xc0); }
    BFT_FN void unit_variant(uint32_t idx) { arr(2); uint(idx); arr(0); }
    BFT_FN void bytes_as_uints(const uint8_t* s, uint32_t len) {
        arr(len);
        for (uint32_t i = 0; i < len; ++i) uint(s[i]);
    }
};

// Subject {view: View{round, height}, digest}
BFT_FN uint32_t encode_subject(uint8_t* out, uint32_t cap, uint64_t round, uint64_t height, const uint8_t* digest) {
    Writer w(out, cap);
    w.arr(2);
    w.arr(2); w.uint(round); w.uint(height);
    w.bytes_as_uints(digest, 32);
    return w.ovf ? 0u : w.n;
}
// GossipMessage {code, create_time, msg, signature, commit_seal}; sig / seal null = None
BFT_FN uint32_t encode_gossip(uint8_t* out, uint32_t cap, uint32_t code, uint64_t ctime, const uint8_t* msg,
                              uint32_t msg_len, const uint8_t* sig, const uint8_t* seal) {
    Writer w(out, cap);
    w.arr(5);
    w.unit_variant(code - 1u);
    w.uint(ctime);
    w.bytes_as_uints(msg, msg_len);
    if (sig) w.bytes_as_uints(sig, 65); else w.nil();
    if (seal) w.bytes_as_uints(seal, 65); else w.nil();
    return w.ovf ? 0u : w.n;
}
// frame of RawMessage {Header{Consensus, ttl, create_time, peer_id}, payload}
BFT_FN uint32_t encode_frame(uint8_t* out, uint32_t cap, uint64_t ttl, uint64_t rtime, const uint8_t* peer,
                             uint32_t peer_len, const uint8_t* payload, uint32_t payload_len) {
    Writer w(out, cap);
    w.be(0, 4);                          // size, patched below
    w.arr(2);
    w.arr(4);
    w.unit_variant(P2P_CONSENSUS);
    w.uint(ttl);
    w.uint(rtime);
    if (peer) w.bytes_as_uints(peer, peer_len); else w.nil();
    w.bytes_as_uints(payload, payload_len);
    if (w.ovf) return 0u;
    uint32_t body = w.n - 4u;
    out[0] = (uint8_t)(body >> 24); out[1] = (uint8_t)(body >> 16); out[2] = (uint8_t)(body >> 8); out[3] = (uint8_t)body;
    return w.n;
}

// ---------------------------------------------------------------- streaming decoder
// byte sources: Mem (a buffer), Arr<Inner> (the integers of a MessagePack array of uint8 read from
// Inner: one source byte per element). get() returns false at the end or on malformed input.
struct Mem {
    const uint8_t* p;
    uint32_t n, i;
    BFT_FN bool get(uint32_t& b) {
        if (i >= n) return false;
        b = p[i++];
        return true;
    }
};
template <class S>
BFT_FN bool rd_be(S& s, int bytes, uint64_t& v) {
    v = 0;
    for (int k = 0; k < bytes; ++k) {
        uint32_t b;
        if (!s.get(b)) return false;
        v = (v << 8) | b;
    }
    return true;
}
template <class S>
BFT_FN bool rd_uint_tag(S& s, uint32_t t, uint64_t& v) {
    if (t < 0x80) { v = t; return true; }
    if (t == 0xcc) return rd_be(s, 1, v);
    if (t == 0xcd) return rd_be(s, 2, v);
    if (t == 0xce) return rd_be(s, 4, v);
    if (t == 0xcf) return rd_be(s, 8, v);
    return false;
}
template <class S>
BFT_FN bool rd_uint(S& s, uint64_t& v) {
    uint32_t t;
    return s.get(t) && rd_uint_tag(s, t, v);
}
template <class S>
BFT_FN bool rd_arr_tag(S& s, uint32_t t, uint32_t& len) {
    if ((t & 0xf0u) == 0x90u) { len = t & 15u; return true; }
    uint64_t v;
    if (t == 0xdc) { if (!rd_be(s, 2, v)) return false; len = (uint32_t)v; return true; }
    if (t == 0xdd) { if (!rd_be(s, 4, v)) return false; len = (uint32_t)v; return true; }
    return false;
}
template <class S>
BFT_FN bool rd_arr(S& s, uint32_t& len) {
    uint32_t t;
    return s.get(t) && rd_arr_tag(s, t, len);
}
template <class S>
BFT_FN bool rd_unit_variant(S& s, uint32_t& idx) {
    uint32_t n, z;
    uint64_t v;
    if (!rd_arr(s, n) || n != 2 || !rd_uint(s, v) || !rd_arr(s, z) || z != 0) return false;
    idx = (uint32_t)v;
    return v < 256;
}
template <class Inner>
struct Arr {
    Inner* in;
    uint32_t left;
    bool bad;
    BFT_FN bool get(uint32_t& b) {
        if (left == 0 || bad) return false;
        uint64_t v;
        if (!rd_uint(*in, v) || v > 255) { bad = true; return false; }
        --left;
        b = (uint32_t)v;
        return true;
    }
};
// a fixed-length byte array (Hash / Signature / peer_id) into out
template <class S>
BFT_FN bool rd_bytes_fixed(S& s, uint32_t len, uint8_t* out) {
    uint32_t n;
    if (!rd_arr(s, n) || n != len) return false;
    for (uint32_t i = 0; i < len; ++i) {
        uint64_t v;
        if (!rd_uint(s, v) || v > 255) return false;
        out[i] = (uint8_t)v;
    }
    return true;
}
// Option<[u8; len]>: nil -> false in *present
template <class S>
BFT_FN bool rd_opt_bytes(S& s, uint32_t len, uint8_t* out, uint32_t& present) {
    uint32_t t;
    if (!s.get(t)) return false;
    if (t == 0xc0) { present = 0; return true; }
    uint32_t n;
    if (!rd_arr_tag(s, t, n) || n != len) return false;
    for (uint32_t i = 0; i < len; ++i) {
        uint64_t v;
        if (!rd_uint(s, v) || v > 255) return false;
        out[i] = (uint8_t)v;
    }
    present = 1;
    return true;
}

struct Decoded {
    uint32_t code;                // MessageType 1..4
    uint64_t create_time, height, round;
    uint8_t digest[32];
    uint32_t has_sig, has_seal;
    uint8_t sig[65], seal[65];
    uint64_t ttl, raw_time;
    uint32_t peer_len;            // 0xffffffff = None
    uint8_t peer[MAX_PEER];
};

// a RawMessage body -> fields; false if malformed, not a Consensus RawMessage, not a
// Subject-carrying GossipMessage, or with trailing bytes
template <class M>
BFT_FN bool decode_body(M& m, Decoded& d) {
    uint32_t n, idx;
    if (!rd_arr(m, n) || n != 2 || !rd_arr(m, n) || n != 4) return false;
    if (!rd_unit_variant(m, idx) || idx != P2P_CONSENSUS) return false;
    if (!rd_uint(m, d.ttl) || !rd_uint(m, d.raw_time)) return false;
    uint32_t t;
    if (!m.get(t)) return false;
    if (t == 0xc0) {
        d.peer_len = 0xffffffffu;
    } else {
        if (!rd_arr_tag(m, t, n) || n > MAX_PEER) return false;
        for (uint32_t i = 0; i < n; ++i) {
            uint64_t v;
            if (!rd_uint(m, v) || v > 255) return false;
            d.peer[i] = (uint8_t)v;
        }
        d.peer_len = n;
    }
    // payload: the GossipMessage bytes, one array element each
    uint32_t glen;
    if (!rd_arr(m, glen)) return false;
    Arr<M> g{&m, glen, false};
    // signature and commit_seal are #[serde(default)] (protocol/mod.rs:48-51): serde's derived
    // sequence visitor accepts the array without them (3 or 4 elements) and fills None
    uint32_t gfields;
    if (!rd_arr(g, gfields) || gfields < 3 || gfields > 5) return false;
    if (!rd_unit_variant(g, idx) || idx < 1 || idx > 3) return false;     // Prepare, Commit, RoundChange
    d.code = idx + 1u;
    if (!rd_uint(g, d.create_time)) return false;
    uint32_t slen;
    if (!rd_arr(g, slen)) return false;
    Arr<Arr<M>> s{&g, slen, false};
    if (!rd_arr(s, n) || n != 2 || !rd_arr(s, n) || n != 2) return false;
    if (!rd_uint(s, d.round) || !rd_uint(s, d.height)) return false;
    if (!rd_bytes_fixed(s, 32, d.digest)) return false;
    if (s.left != 0) return false;
    d.has_sig = d.has_seal = 0;
    if (gfields >= 4 && !rd_opt_bytes(g, 65, d.sig, d.has_sig)) return false;
    if (gfields >= 5 && !rd_opt_bytes(g, 65, d.seal, d.has_seal)) return false;
    if (g.left != 0 || g.bad) return false;
    return m.i == m.n;
}
BFT_FN uint32_t frame_size(const uint8_t* f) {
    return ((uint32_t)f[0] << 24) | ((uint32_t)f[1] << 16) | ((uint32_t)f[2] << 8) | f[3];
}
// one frame (size prefix included, `len` bytes available) -> fields
BFT_FN bool decode_frame(const uint8_t* f, uint32_t len, Decoded& d) {
    if (len < 4 || frame_size(f) != len - 4u) return false;
    Mem m{f + 4, len - 4u, 0};
    return decode_body(m, d);
}

}  // namespace wire
}  // namespace bft
