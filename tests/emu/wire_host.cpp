// wire_host.cpp — TEST-ONLY host build of consensus-rs_amd/csrc/bft_wire.h (the serial encoder and
// streaming decoder the GPU kernels share), checked against oracle/wire_ref.py on the CPU.
#include <stdint.h>
#include <string.h>

#include "../../consensus-rs_amd/csrc/bft_wire.h"

using namespace bft::wire;

extern "C" {
// frame of one Subject message; returns its length (0 on overflow); g / sp receive the
// GossipMessage and sign-payload bytes with their lengths
uint32_t wire_host_encode(uint32_t code, uint64_t round, uint64_t height, const uint8_t* digest, uint64_t ctime,
                          const uint8_t* sig, const uint8_t* seal, uint64_t ttl, uint64_t rtime, const uint8_t* peer,
                          uint32_t peer_len, uint8_t* frame, uint8_t* g, uint32_t* glen, uint8_t* sp, uint32_t* splen) {
    uint8_t s[MAX_S];
    uint32_t ls = encode_subject(s, MAX_S, round, height, digest);
    *glen = encode_gossip(g, MAX_G, code, ctime, s, ls, sig, seal);
    *splen = encode_gossip(sp, MAX_G, code, ctime, s, ls, nullptr, seal);
    return encode_frame(frame, MAX_FRAME, ttl, rtime, peer, peer_len, g, *glen);
}
int wire_host_decode(const uint8_t* f, uint32_t len, Decoded* d) { return decode_frame(f, len, *d) ? 1 : 0; }
uint32_t wire_host_decoded_size() { return (uint32_t)sizeof(Decoded); }
}

// ---- block-carrying frames (consensus-rs_amd/csrc/bft_wire_block.h), host build
#include "../../consensus-rs_amd/csrc/bft_wire_block.h"

extern "C" {
uint32_t wire_host_struct_size(int which) {
    return which == 0 ? (uint32_t)sizeof(bftwire_tx) : which == 1 ? (uint32_t)sizeof(bftwire_block)
                                                                    : (uint32_t)sizeof(bftwire_preprepare);
}
uint32_t wire_host_pp_encode(const bftwire_preprepare* m, uint8_t* out, uint32_t cap, uint8_t* sign_digest,
                             uint8_t* msg_hash) {
    if (!block_fits(m->block)) return 0;
    uint32_t n = 0;
    emit_frame(BufE{out, &n, cap}, P2P_CONSENSUS, m->ttl, m->raw_time, [&](const auto& e) { emit_pp_gossip(e, *m, true); });
    uint8_t kb[136];
    {
        bft::crypto::KSink k(kb);
        emit_pp_gossip(KE{&k}, *m, false);
        k.finish(sign_digest);
    }
    {
        bft::crypto::KSink k(kb);
        emit_pp_gossip(KE{&k}, *m, true);
        k.finish(msg_hash);
    }
    return n <= cap ? n : 0;
}
int wire_host_pp_decode(const uint8_t* f, uint32_t len, bftwire_preprepare* out) {
    memset(out, 0, sizeof *out);
    return decode_pp_frame(f, len, *out) ? 1 : 0;
}
uint32_t wire_host_blocks_encode(const bftwire_block* b, uint32_t nb, uint64_t ttl, uint64_t rt, uint8_t* out, uint32_t cap) {
    for (uint32_t j = 0; j < nb; ++j)
        if (!block_fits(b[j])) return 0;
    uint32_t n = 0;
    emit_frame(BufE{out, &n, cap}, P2P_BLOCK, ttl, rt, [&](const auto& e) {
        mp_arr(e, nb);
        for (uint32_t j = 0; j < nb; ++j) emit_block(e, b[j]);
    });
    return n <= cap ? n : 0;
}
int wire_host_blocks_decode(const uint8_t* f, uint32_t len, bftwire_block* out, uint32_t max, uint32_t* count) {
    *count = 0;
    if (len < 4 || frame_size(f) != len - 4u) return 0;
    Mem m{f + 4, len - 4u, 0};
    uint64_t t, rt;
    uint32_t plen, cnt;
    if (!rd_envelope(m, P2P_BLOCK, t, rt, plen)) return 0;
    Arr<Mem> p{&m, plen, false};
    if (!rd_arr(p, cnt) || cnt > max) return 0;
    for (uint32_t j = 0; j < cnt; ++j) {
        memset(&out[j], 0, sizeof out[j]);
        if (!rd_block(p, out[j])) return 0;
    }
    if (p.left != 0 || p.bad || m.i != m.n) return 0;
    *count = cnt;
    return 1;
}
uint32_t wire_host_sync_encode(uint64_t height, uint64_t ttl, uint64_t rt, uint8_t* out, uint32_t cap) {
    uint32_t n = 0;
    emit_frame(BufE{out, &n, cap}, P2P_SYNC, ttl, rt, [&](const auto& e) { mp_uint(e, height); });
    return n <= cap ? n : 0;
}
int wire_host_sync_decode(const uint8_t* f, uint32_t len, uint64_t* height) { return decode_sync_frame(f, len, *height) ? 1 : 0; }
}
