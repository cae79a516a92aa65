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
