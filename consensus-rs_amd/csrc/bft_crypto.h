// bft_crypto.h — real-crypto mode (SPEC.md §11): the bytes the reference signs for every consensus
// message, produced on the GPU from the simulator's broadcast log and hashed as they are emitted.
//   sign payload  = GossipMessage {code, create_time, msg, signature: None, commit_seal}
//                   (protocol/mod.rs:128-137; the serializer convention of SPEC.md §9)
//   msg           = Subject {view, digest} (Prepare / Commit / RoundChange, types.rs:60-63) or
//                   PrePrepare {view, proposal: Block {header, transactions: []}} (types.rs:131-134)
//   commit seal   = sign(keccak(0x03 || digest)) (encrypt_commit_bytes, types/votes.rs:94-101)
// The MessagePack bytes stream straight into a Keccak-256 absorber (136-byte block buffer per lane),
// so no message is ever materialised.
#pragma once
#include "bft_common.h"

namespace bft {
namespace crypto {

// Keccak-256 absorber over a 136-byte block buffer (LDS on the device)
struct KSink {
    uint64_t a[25];
    uint8_t* buf;
    uint32_t n;
    BFT_FN explicit KSink(uint8_t* b) : buf(b), n(0) {
        for (int i = 0; i < 25; ++i) a[i] = 0;
    }
    BFT_FN void absorb() {
        for (int i = 0; i < 17; ++i) {
            uint64_t w = 0;
            for (int k = 7; k >= 0; --k) w = (w << 8) | buf[8 * i + k];
            a[i] ^= w;
        }
        keccak_f1600(a);
        n = 0;
    }
    BFT_FN void put(uint32_t b) {
        buf[n++] = (uint8_t)b;
        if (n == 136u) absorb();
    }
    BFT_FN void finish(uint8_t out[32]) {
        buf[n++] = 0x01;
        while (n < 136u) buf[n++] = 0;
        buf[135] |= 0x80;
        absorb();
        for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(a[i >> 3] >> (8 * (i & 7)));
    }
};

// byte emitters: straight into the sink, or each byte as a MessagePack uint (a Vec<u8> element)
struct Direct {
    KSink* k;
    BFT_FN void operator()(uint32_t b) const { k->put(b); }
};
struct AsUint {
    KSink* k;
    BFT_FN void operator()(uint32_t b) const {
        if (b >= 128u) k->put(0xcc);
        k->put(b);
    }
};
struct Count {
    uint32_t* c;
    BFT_FN void operator()(uint32_t) const { *c += 1; }
};

template <class E>
BFT_FN void mp_uint(const E& e, uint64_t v) {
    if (v < 128u) { e((uint32_t)v); return; }
    int bytes = v < 256u ? 1 : v < 65536u ? 2 : v < 4294967296ull ? 4 : 8;
    e(bytes == 1 ? 0xccu : bytes == 2 ? 0xcdu : bytes == 4 ? 0xceu : 0xcfu);
    for (int i = bytes - 1; i >= 0; --i) e((uint32_t)(v >> (8 * i)) & 0xffu);
}
template <class E>
BFT_FN void mp_arr(const E& e, uint32_t len) {
    if (len < 16u) { e(0x90u | len); return; }
    if (len < 65536u) { e(0xdc); e(len >> 8); e(len & 0xffu); return; }
    e(0xdd); e(len >> 24); e((len >> 16) & 0xffu); e((len >> 8) & 0xffu); e(len & 0xffu);
}

// msg bytes: Subject [[round, height], digest] or PrePrepare [[round, height], [header, []]]
template <class E>
BFT_FN void emit_msg(const E& e, uint64_t round, uint64_t height, const uint8_t* digest, const uint8_t* header,
                     uint32_t hlen) {
    e(0x92);
    e(0x92); mp_uint(e, round); mp_uint(e, height);
    if (header) {
        e(0x92);
        for (uint32_t i = 0; i < hlen; ++i) e(header[i]);
        e(0x90);                                    // transactions: [] (SPEC.md §11)
    } else {
        mp_arr(e, 32);
        for (int i = 0; i < 32; ++i) mp_uint(e, digest[i]);
    }
}

// Keccak-256 of the sign payload of one message (GossipMessage with signature None)
BFT_FN void sign_digest(uint8_t* kbuf, uint32_t code, uint64_t ctime, uint64_t round, uint64_t height,
                        const uint8_t* digest, const uint8_t* header, uint32_t hlen, const uint8_t* seal,
                        uint8_t out[32]) {
    uint32_t mlen = 0;
    emit_msg(Count{&mlen}, round, height, digest, header, hlen);
    KSink k(kbuf);
    const Direct d{&k};
    const AsUint u{&k};
    d(0x95);                                        // GossipMessage: 5 fields
    d(0x92); mp_uint(d, code - 1u); d(0x90);        // MessageType unit variant
    mp_uint(d, ctime);
    mp_arr(d, mlen);
    emit_msg(u, round, height, digest, header, hlen);
    d(0xc0);                                        // signature: None
    if (seal) {
        mp_arr(d, 65);
        for (int i = 0; i < 65; ++i) mp_uint(d, seal[i]);
    } else {
        d(0xc0);
    }
    k.finish(out);
}

// keccak(0x03 || digest): what encrypt_commit_bytes signs (types/votes.rs:94-101)
BFT_FN void seal_digest(uint8_t* kbuf, const uint8_t digest[32], uint8_t out[32]) {
    KSink k(kbuf);
    k.put(MT_COMMIT);
    for (int i = 0; i < 32; ++i) k.put(digest[i]);
    k.finish(out);
}

// keccak(signature || seal or 65 zero bytes): one message's term of the per-instance checksum
BFT_FN void sig_term(uint8_t* kbuf, const uint8_t sig[65], const uint8_t* seal, uint8_t out[32]) {
    KSink k(kbuf);
    for (int i = 0; i < 65; ++i) k.put(sig[i]);
    for (int i = 0; i < 65; ++i) k.put(seal ? seal[i] : 0u);
    k.finish(out);
}

}  // namespace crypto
}  // namespace bft
