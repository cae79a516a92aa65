// bftwire.hip — gfx950 kernels and the C ABI of libbftwire (include/bftwire.h): the consensus wire
// codec, batched. Encoding is wave-per-message: the nested MessagePack levels (Subject -> GossipMessage
// -> RawMessage frame) are assembled in LDS, each level's byte array expanded by all 64 lanes at once
// (a byte >= 128 becomes 0xcc b: the output position of every byte is a ballot prefix count), then
// written to a per-message slot with coalesced dword stores; a device scan gives the frame offsets and
// a pack pass copies the slots into the contiguous stream (lanes write consecutive bytes). The two
// Keccak-256 digests run lane-per-message over the GossipMessage / sign-payload slots. Decoding is
// lane-per-frame through the streaming decoder of bft_wire.h (plain byte loads: a 16-byte or 4-byte
// register window measured 1.6-1.9x slower — the per-byte window test diverges the loads).
// BFTWIRE_DECODE=wave selects a wave-per-frame decoder (frame in LDS, every nested byte array
// un-expanded by all lanes with a scanned byte automaton): bit-identical, but ~64x the instruction
// issue per message, measured 2.2x slower end to end — kept for A/B.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../../include/bftwire.h"
#include "bft_wire.h"

namespace bft {
namespace wire {

constexpr uint32_t SLOT_F = 1088;            // frame slot (>= the largest frame, multiple of 64)
constexpr uint32_t SLOT_G = 544;             // GossipMessage / sign-payload slot: 4 Keccak blocks
constexpr uint32_t LDS_S = 0, LDS_G = 96, LDS_SP = LDS_G + SLOT_G, LDS_F = LDS_SP + SLOT_G;
constexpr uint32_t LDS_WAVE = LDS_F + SLOT_F;  // 2272 bytes per wave
constexpr uint32_t WAVES = 4;                // messages per workgroup

struct EncParams {
    bftwire_batch in;
    uint64_t n;
    uint8_t *slot_f, *slot_g, *slot_sp;
    uint64_t* lens;                          // [n + 1] frame lengths (lens[n] = 0): scanned into offsets
    uint32_t *glen, *splen;
    uint8_t* ok;
    uint32_t want_hash;
};

__device__ inline void wsync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
__device__ inline uint32_t bcast0(uint32_t v) { return (uint32_t)__shfl((int)v, 0, 64); }

// bytes src[0, len) as a run of MessagePack uints into dst from `off` (no array header); all lanes
template <class P>
__device__ inline uint32_t wave_expand(P src, uint32_t len, uint8_t* dst, uint32_t off) {
    const uint32_t lane = __lane_id();
    for (uint32_t c = 0; c < len; c += 64) {
        const uint32_t i = c + lane;
        const bool act = i < len;
        const uint32_t b = act ? (uint32_t)src[i] : 0u;
        const bool two = act && b >= 128u;
        const uint64_t m = __ballot(two);
        const uint32_t pos = off + lane + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (act) {
            if (two) { dst[pos] = 0xcc; dst[pos + 1] = (uint8_t)b; }
            else dst[pos] = (uint8_t)b;
        }
        off += (len - c < 64u ? len - c : 64u) + (uint32_t)__popcll(m);
    }
    wsync();
    return off;
}

// GossipMessage {code, create_time, msg = S, signature, commit_seal} into dst; all lanes
__device__ inline uint32_t wave_gossip(uint8_t* dst, uint32_t code, uint64_t ctime, const uint8_t* s, uint32_t ls,
                                       const uint8_t* sig, const uint8_t* seal) {
    const uint32_t lane = __lane_id();
    uint32_t n0 = 0;
    if (lane == 0) {
        Writer w(dst, 32);
        w.arr(5); w.unit_variant(code - 1u); w.uint(ctime); w.arr(ls);
        n0 = w.n;
    }
    uint32_t off = bcast0(n0);
    wsync();
    off = wave_expand(s, ls, dst, off);
    const uint8_t* opt[2] = {sig, seal};
    for (int k = 0; k < 2; ++k) {
        if (opt[k]) {
            if (lane == 0) { dst[off] = 0xdc; dst[off + 1] = 0; dst[off + 2] = 65; }
            wsync();
            off = wave_expand(opt[k], 65u, dst, off + 3u);
        } else {
            if (lane == 0) dst[off] = 0xc0;
            wsync();
            off += 1u;
        }
    }
    return off;
}

__device__ inline void wave_store_slot(const uint8_t* src, uint32_t len, uint8_t* slot) {
    const uint32_t lane = __lane_id();
    for (uint32_t j = 4u * lane; j < len; j += 256u) *(uint32_t*)(slot + j) = *(const uint32_t*)(src + j);
}

__global__ __launch_bounds__(64 * WAVES) void wire_encode_kernel(EncParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * LDS_WAVE];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * WAVES + wave;
    if (i >= p.n) return;                                       // wave-uniform
    if (i == 0 && lane == 0) p.lens[p.n] = 0;
    uint8_t* S = lds + wave * LDS_WAVE + LDS_S;
    uint8_t* G = lds + wave * LDS_WAVE + LDS_G;
    uint8_t* SP = lds + wave * LDS_WAVE + LDS_SP;
    uint8_t* F = lds + wave * LDS_WAVE + LDS_F;
    const uint32_t code = p.in.code[i];
    if (code < 2u || code > 4u) {
        if (lane == 0) { p.ok[i] = 0; p.lens[i] = 0; if (p.want_hash) { p.glen[i] = 0; p.splen[i] = 0; } }
        return;
    }
    // Subject {view: [round, height], digest}
    uint32_t n0 = 0;
    if (lane == 0) {
        Writer w(S, 32);
        w.arr(2); w.arr(2); w.uint(p.in.round[i]); w.uint(p.in.height[i]); w.arr(32);
        n0 = w.n;
    }
    uint32_t ls = bcast0(n0);
    wsync();
    ls = wave_expand(p.in.digest + 32u * i, 32u, S, ls);
    // GossipMessage (signed) and its sign payload (signature None)
    const uint64_t ctime = p.in.create_time[i];
    const uint8_t* sig = p.in.signature ? p.in.signature + 65u * i : nullptr;
    const uint8_t* seal = (p.in.commit_seal && code == 3u) ? p.in.commit_seal + 65u * i : nullptr;
    const uint32_t lg = wave_gossip(G, code, ctime, S, ls, sig, seal);
    // frame: size | RawMessage {Header{Consensus, ttl, create_time, None}, payload = G}
    if (lane == 0) {
        Writer w(F, 40);
        w.be(0, 4);
        w.arr(2); w.arr(4); w.unit_variant(P2P_CONSENSUS);
        w.uint(p.in.ttl ? p.in.ttl[i] : (uint64_t)DEFAULT_TTL);
        w.uint(p.in.raw_time ? p.in.raw_time[i] : ctime);
        w.nil();
        w.arr(lg);
        n0 = w.n;
    }
    uint32_t lf = bcast0(n0);
    wsync();
    lf = wave_expand(G, lg, F, lf);
    if (lane == 0) {
        const uint32_t body = lf - 4u;
        F[0] = (uint8_t)(body >> 24); F[1] = (uint8_t)(body >> 16); F[2] = (uint8_t)(body >> 8); F[3] = (uint8_t)body;
    }
    wsync();
    wave_store_slot(F, lf, p.slot_f + i * SLOT_F);
    if (p.want_hash) {
        const uint32_t lsp = wave_gossip(SP, code, ctime, S, ls, nullptr, seal);
        wave_store_slot(G, lg, p.slot_g + i * SLOT_G);
        wave_store_slot(SP, lsp, p.slot_sp + i * SLOT_G);
        if (lane == 0) { p.glen[i] = lg; p.splen[i] = lsp; }
    }
    if (lane == 0) { p.lens[i] = lf; p.ok[i] = 1; }
}

// slots -> contiguous stream at the scanned offsets (wave per message, consecutive bytes per lane)
__global__ __launch_bounds__(64 * WAVES) void wire_pack_kernel(const uint8_t* slot_f, const uint64_t* off, uint64_t n,
                                                             uint8_t* stream, uint64_t cap, uint8_t* ok) {
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * WAVES + wave;
    if (i >= n) return;
    const uint64_t o = off[i], len = off[i + 1] - o;
    if (len == 0) return;
    if (o + len > cap) { if (lane == 0) ok[i] = 0; return; }
    const uint8_t* src = slot_f + i * SLOT_F;
    for (uint32_t j = lane; j < len; j += 64u) stream[o + j] = src[j];
}

// Keccak-256 of len bytes at an 8-byte aligned slot (reads stay inside the slot: len < SLOT_G - 136)
__device__ inline void keccak_slot(const uint8_t* slot, uint32_t len, uint8_t* out) {
    uint64_t a[25];
    for (int k = 0; k < 25; ++k) a[k] = 0;
    const uint32_t nb = len / 136u + 1u;
    for (uint32_t b = 0; b < nb; ++b) {
        for (uint32_t w = 0; w < 17; ++w) {
            const uint32_t i0 = 136u * b + 8u * w;
            uint64_t v = i0 < len ? *(const uint64_t*)(slot + i0) : 0ull;
            if (i0 < len && len < i0 + 8u) v &= (1ull << (8u * (len - i0))) - 1ull;
            if (i0 <= len && len < i0 + 8u) v ^= 1ull << (8u * (len - i0));
            if (b == nb - 1u && w == 16u) v ^= 0x80ull << 56;
            a[w] ^= v;
        }
        keccak_f1600(a);
    }
    for (int k = 0; k < 32; ++k) out[k] = (uint8_t)(a[k >> 3] >> (8 * (k & 7)));
}
__global__ __launch_bounds__(64) void wire_hash_kernel(const uint8_t* slot_g, const uint8_t* slot_sp, const uint32_t* glen,
                                                       const uint32_t* splen, uint64_t n, uint8_t* msg_hash,
                                                       uint8_t* sign_digest) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t h[32];
    if (msg_hash) {
        if (glen[i]) keccak_slot(slot_g + i * SLOT_G, glen[i], h); else for (int k = 0; k < 32; ++k) h[k] = 0;
        for (int k = 0; k < 32; ++k) msg_hash[32u * i + k] = h[k];
    }
    if (sign_digest) {
        if (splen[i]) keccak_slot(slot_sp + i * SLOT_G, splen[i], h); else for (int k = 0; k < 32; ++k) h[k] = 0;
        for (int k = 0; k < 32; ++k) sign_digest[32u * i + k] = h[k];
    }
}

__global__ __launch_bounds__(64) void wire_decode_kernel(const uint8_t* stream, const uint64_t* off, uint64_t n,
                                                         bftwire_batch out, uint8_t* has_sig, uint8_t* has_seal,
                                                         uint8_t* ok) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i], len = off[i + 1] - o;
    Decoded d;
    const bool good = len <= MAX_FRAME && decode_frame(stream + o, (uint32_t)len, d);
    out.code[i] = good ? (uint8_t)d.code : 0;
    out.round[i] = good ? d.round : 0;
    out.height[i] = good ? d.height : 0;
    out.create_time[i] = good ? d.create_time : 0;
    out.ttl[i] = good ? d.ttl : 0;
    out.raw_time[i] = good ? d.raw_time : 0;
    for (int k = 0; k < 32; ++k) out.digest[32u * i + k] = good ? d.digest[k] : 0;
    for (int k = 0; k < 65; ++k) out.signature[65u * i + k] = (good && d.has_sig) ? d.sig[k] : 0;
    for (int k = 0; k < 65; ++k) out.commit_seal[65u * i + k] = (good && d.has_seal) ? d.seal[k] : 0;
    has_sig[i] = good && d.has_sig ? 1 : 0;
    has_seal[i] = good && d.has_seal ? 1 : 0;
    ok[i] = good ? 1 : 0;
}

// BFTWIRE_DECODE=lds (A/B): one wave per 64 consecutive frames; their contiguous byte range is first
// staged in LDS with coalesced 16-byte loads, then each lane parses its frame from LDS. Bit-identical,
// but measured 1.25x slower than the global-memory lane decoder: the 40 KB buffer allows 4 waves per
// CU, too few to hide the parse's dependent-read chains. A range larger than the buffer falls back to
// global reads.
constexpr uint32_t DEC_LDS = 40960;
__global__ __launch_bounds__(64) void wire_decode_lds_kernel(const uint8_t* stream, const uint64_t* off, uint64_t n,
                                                             bftwire_batch out, uint8_t* has_sig, uint8_t* has_seal,
                                                             uint8_t* ok) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[DEC_LDS];
    const uint64_t i0 = (uint64_t)blockIdx.x * 64u;
    const uint64_t i = i0 + threadIdx.x;
    const uint64_t iend = i0 + 64u < n ? i0 + 64u : n;
    const uint64_t lo = off[i0], hi = off[iend];
    const uint64_t base = lo & ~(uint64_t)15;
    const bool staged = hi - base <= DEC_LDS;                 // block-uniform
    if (staged) {
        for (uint64_t j = 16u * threadIdx.x; base + j < hi; j += 64u * 16u)
            *(uint4*)(buf + j) = *(const uint4*)(stream + base + j);
        __syncthreads();
    }
    if (i >= n) return;
    const uint64_t o = off[i], len = off[i + 1] - o;
    Decoded d;
    const uint8_t* f = staged ? buf + (o - base) : stream + o;
    const bool good = len <= MAX_FRAME && decode_frame(f, (uint32_t)len, d);
    out.code[i] = good ? (uint8_t)d.code : 0;
    out.round[i] = good ? d.round : 0;
    out.height[i] = good ? d.height : 0;
    out.create_time[i] = good ? d.create_time : 0;
    out.ttl[i] = good ? d.ttl : 0;
    out.raw_time[i] = good ? d.raw_time : 0;
    for (int k = 0; k < 32; ++k) out.digest[32u * i + k] = good ? d.digest[k] : 0;
    for (int k = 0; k < 65; ++k) out.signature[65u * i + k] = (good && d.has_sig) ? d.sig[k] : 0;
    for (int k = 0; k < 65; ++k) out.commit_seal[65u * i + k] = (good && d.has_seal) ? d.seal[k] : 0;
    has_sig[i] = good && d.has_sig ? 1 : 0;
    has_seal[i] = good && d.has_seal ? 1 : 0;
    ok[i] = good ? 1 : 0;
}

// ---------------------------------------------------------------- wave-cooperative decode
// The elements of a MessagePack array of uint8 are 1 (fixint), 2 (0xcc), 3 (0xcd), 5 (0xce) or 9 (0xcf)
// bytes; which byte starts an element depends on every byte before it. Each lane takes one byte
// and its transition function over the states {0: at an element start, k: k bytes of the element
// left, 9: error}, packed as 10 nibbles; an inclusive Hillis-Steele scan of function composition
// (6 shuffle steps) gives every lane its entry state. A lane whose exit state is 0 ends an element
// and emits its byte (the value byte; the padding bytes of a wide encoding must be zero, as the
// serial decoder's `v > 255` check requires).
constexpr uint32_t ST_ERR = 9u;
__device__ inline uint64_t fn_of_byte(uint32_t b) {
    const uint32_t s0 = b < 0x80u ? 0u : b == 0xccu ? 1u : b == 0xcdu ? 2u : b == 0xceu ? 4u : b == 0xcfu ? 8u : ST_ERR;
    // f(0) = s0, f(k) = k - 1 (k = 1..8), f(9) = 9
    return 0x9765432100ull | s0;     // nibble k: f(k); f(1..8) = 0..7, f(9) = 9
}
__device__ inline uint32_t fn_at(uint64_t f, uint32_t s) { return (uint32_t)(f >> (4u * s)) & 15u; }
__device__ inline uint64_t fn_then(uint64_t first, uint64_t second) {      // second o first
    uint64_t r = 0;
#pragma unroll
    for (uint32_t s = 0; s < 10; ++s) r |= (uint64_t)fn_at(second, fn_at(first, s)) << (4u * s);
    return r;
}
__device__ inline uint64_t shfl_up64(uint64_t v, uint32_t d) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// `count` elements from src[pos, end) into dst; returns the position after them, or ~0u if malformed
__device__ inline uint32_t wave_unexpand(const uint8_t* src, uint32_t end, uint32_t pos, uint32_t count, uint8_t* dst) {
    const uint32_t lane = __lane_id();
    uint32_t done = 0, state = 0;
    while (done < count) {
        if (pos >= end) return ~0u;
        const uint32_t q = pos + lane;
        const bool in = q < end;
        const uint32_t b = in ? src[q] : 0u;
        uint64_t f = in ? fn_of_byte(b) : 0x9999999999ull;
        uint64_t F = f;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t o = shfl_up64(F, d);
            if (lane >= d) F = fn_then(o, F);
        }
        const uint64_t Fprev = shfl_up64(F, 1);
        const uint32_t s_in = lane == 0 ? state : fn_at(Fprev, state);
        const uint32_t s_out = fn_at(f, s_in);
        const bool emit = in && s_out == 0u;
        const bool bad = in && (s_out == ST_ERR || (s_in >= 2u && s_in <= 8u && b != 0u));
        const uint64_t em = __ballot(emit);
        const uint32_t need = count - done;
        // lanes up to the need-th emitting lane belong to this array
        uint32_t last = 63u;
        if ((uint32_t)__popcll(em) >= need) {
            uint64_t m = em;
            for (uint32_t k = 1; k < need; ++k) m &= m - 1;            // drop the first need-1 set bits
            last = (uint32_t)__ffsll((unsigned long long)m) - 1u;
        }
        const bool mine = lane <= last;
        if (__ballot(mine && bad)) return ~0u;
        if (emit && mine) dst[done + (uint32_t)__popcll(em & ((1ull << lane) - 1ull))] = (uint8_t)b;
        const uint32_t took = (uint32_t)__popcll(em & (last == 63u ? ~0ull : ((2ull << last) - 1ull)));
        state = (uint32_t)__shfl((int)s_out, (int)last, 64);
        if (last == 63u && !__shfl((int)in, 63, 64)) return ~0u;      // ran past the end of the buffer
        done += took;
        pos += last + 1u;
    }
    wsync();
    return state == 0u ? pos : ~0u;
}

struct DecScalars {
    uint32_t ok, code, peer_none;
    uint64_t ctime, round, height, ttl, rtime;
    uint32_t has_sig, has_seal;
};

__global__ __launch_bounds__(64 * WAVES) void wire_decode_wave_kernel(const uint8_t* stream, const uint64_t* off,
                                                                    uint64_t n, bftwire_batch out, uint8_t* has_sig,
                                                                    uint8_t* has_seal, uint8_t* ok) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * LDS_WAVE];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * WAVES + wave;
    if (i >= n) return;
    uint8_t* F = lds + wave * LDS_WAVE + LDS_F;
    uint8_t* G = lds + wave * LDS_WAVE + LDS_G;
    uint8_t* S = lds + wave * LDS_WAVE + LDS_S;
    uint8_t* SIG = lds + wave * LDS_WAVE + LDS_SP;          // signature, seal at +80
    uint8_t* SEAL = SIG + 80;
    const uint64_t o = off[i], len64 = off[i + 1] - o;
    bool good = len64 >= 4 && len64 <= MAX_FRAME;
    const uint32_t len = good ? (uint32_t)len64 : 0u;
    for (uint32_t j = lane; j < len; j += 64u) F[j] = stream[o + j];
    wsync();
    // RawMessage header, serially (lane 0): size, [[Consensus, ttl, time, peer], payload
    uint32_t v0 = 0, v1 = 0, v2 = 0;
    DecScalars sc{};
    if (lane == 0 && good) {
        const uint32_t body = ((uint32_t)F[0] << 24) | ((uint32_t)F[1] << 16) | ((uint32_t)F[2] << 8) | F[3];
        Mem m{F, len, 4};
        uint32_t nn, idx, t;
        bool g = body == len - 4u && rd_arr(m, nn) && nn == 2 && rd_arr(m, nn) && nn == 4 && rd_unit_variant(m, idx) &&
                 idx == P2P_CONSENSUS && rd_uint(m, sc.ttl) && rd_uint(m, sc.rtime) && m.get(t);
        if (g && t != 0xc0) {                                  // peer_id: Some (decoded, not returned)
            g = rd_arr_tag(m, t, nn) && nn <= MAX_PEER;
            for (uint32_t k = 0; g && k < nn; ++k) { uint64_t v; g = rd_uint(m, v) && v <= 255; }
        }
        uint32_t glen = 0;
        g = g && rd_arr(m, glen) && glen <= MAX_G;
        v0 = g ? 1u : 0u; v1 = m.i; v2 = glen;
    }
    good = __shfl((int)v0, 0, 64) != 0;
    uint32_t p = (uint32_t)__shfl((int)v1, 0, 64), glen = (uint32_t)__shfl((int)v2, 0, 64);
    if (good) good = wave_unexpand(F, len, p, glen, G) == len;
    // GossipMessage header: [[code, []], create_time, msg array
    if (lane == 0 && good) {
        Mem m{G, glen, 0};
        uint32_t nn = 0, idx = 0, slen = 0;
        bool g = rd_arr(m, nn) && nn == 5 && rd_unit_variant(m, idx) && idx >= 1 && idx <= 3 && rd_uint(m, sc.ctime) &&
                 rd_arr(m, slen) && slen <= MAX_S;
        sc.code = idx + 1u;
        v0 = g ? 1u : 0u; v1 = m.i; v2 = slen;
    }
    if (good) {
        good = __shfl((int)v0, 0, 64) != 0;
        p = (uint32_t)__shfl((int)v1, 0, 64);
        const uint32_t slen = (uint32_t)__shfl((int)v2, 0, 64);
        if (good) {
            p = wave_unexpand(G, glen, p, slen, S);
            good = p != ~0u;
        }
        // signature, commit_seal: nil or [65 elements]
        uint8_t* dsts[2] = {SIG, SEAL};
        uint32_t present[2] = {0, 0};
        for (int k = 0; k < 2 && good; ++k) {
            const uint32_t t = G[p < glen ? p : 0];
            if (p >= glen) { good = false; break; }
            if (t == 0xc0) { p += 1; continue; }
            uint32_t hl = (t & 0xf0u) == 0x90u ? 1u : t == 0xdcu ? 3u : t == 0xddu ? 5u : 0u;
            uint32_t nn = hl == 1u ? (t & 15u) : hl == 3u && p + 2 < glen ? ((uint32_t)G[p + 1] << 8) | G[p + 2]
                        : hl == 5u && p + 4 < glen ? ((uint32_t)G[p + 1] << 24) | ((uint32_t)G[p + 2] << 16) |
                                                      ((uint32_t)G[p + 3] << 8) | G[p + 4] : 0u;
            if (hl == 0u || nn != 65u) { good = false; break; }
            p = wave_unexpand(G, glen, p + hl, 65u, dsts[k]);
            good = p != ~0u;
            present[k] = 1;
        }
        good = good && p == glen;
        sc.has_sig = present[0];
        sc.has_seal = present[1];
        // Subject: [[round, height], digest]
        if (good) {
            if (lane == 0) {
                Mem m{S, slen, 0};
                uint32_t nn, dl = 0;
                bool g = rd_arr(m, nn) && nn == 2 && rd_arr(m, nn) && nn == 2 && rd_uint(m, sc.round) &&
                         rd_uint(m, sc.height) && rd_arr(m, dl) && dl == 32;
                v0 = g ? 1u : 0u; v1 = m.i;
            }
            good = __shfl((int)v0, 0, 64) != 0;
            if (good) good = wave_unexpand(S, slen, (uint32_t)__shfl((int)v1, 0, 64), 32u, F) == slen;   // digest -> F
        }
    }
    // outputs (F now holds the digest)
    if (lane < 32) out.digest[32u * i + lane] = good ? F[lane] : 0;
    for (uint32_t k = lane; k < 65u; k += 64u) {
        out.signature[65u * i + k] = (good && sc.has_sig) ? SIG[k] : 0;
        out.commit_seal[65u * i + k] = (good && sc.has_seal) ? SEAL[k] : 0;
    }
    if (lane == 0) {
        out.code[i] = good ? (uint8_t)sc.code : 0;
        out.round[i] = good ? sc.round : 0;
        out.height[i] = good ? sc.height : 0;
        out.create_time[i] = good ? sc.ctime : 0;
        out.ttl[i] = good ? sc.ttl : 0;
        out.raw_time[i] = good ? sc.rtime : 0;
        has_sig[i] = good && sc.has_sig ? 1 : 0;
        has_seal[i] = good && sc.has_seal ? 1 : 0;
        ok[i] = good ? 1 : 0;
    }
}

}  // namespace wire
}  // namespace bft

// ------------------------------------------------------------------------------ C ABI
struct bftwire {
    int device = 0;
    uint64_t cap = 0;
    uint8_t *slot_f = nullptr, *slot_g = nullptr, *slot_sp = nullptr;
    uint64_t* lens = nullptr;
    uint32_t *glen = nullptr, *splen = nullptr;
    void* scan_tmp = nullptr;
    size_t scan_bytes = 0;
    int decode_mode = 0;           // 0 global lanes, 1 LDS-staged lanes, 2 wave-cooperative
    std::string err;
};

static int wfail(bftwire* h, int code, const std::string& m) {
    if (h) h->err = m;
    return code;
}
#define WCHECK(h, x)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) return wfail(h, -2, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

static void wire_free(bftwire* h) {
    (void)hipFree(h->slot_f); (void)hipFree(h->slot_g); (void)hipFree(h->slot_sp); (void)hipFree(h->lens);
    (void)hipFree(h->glen); (void)hipFree(h->splen); (void)hipFree(h->scan_tmp);
    h->slot_f = h->slot_g = h->slot_sp = nullptr; h->lens = nullptr; h->glen = h->splen = nullptr; h->scan_tmp = nullptr;
    h->cap = 0; h->scan_bytes = 0;
}

static int wire_reserve(bftwire* h, uint64_t n) {
    using namespace bft::wire;
    if (n <= h->cap) return 0;
    wire_free(h);
    WCHECK(h, hipMalloc(&h->slot_f, n * SLOT_F));
    WCHECK(h, hipMalloc(&h->slot_g, n * SLOT_G));
    WCHECK(h, hipMalloc(&h->slot_sp, n * SLOT_G));
    WCHECK(h, hipMalloc(&h->lens, (n + 1) * 8));
    WCHECK(h, hipMalloc(&h->glen, n * 4));
    WCHECK(h, hipMalloc(&h->splen, n * 4));
    size_t tb = 0;
    WCHECK(h, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, h->lens, h->lens, (int)(n + 1)));
    WCHECK(h, hipMalloc(&h->scan_tmp, tb));
    h->scan_bytes = tb;
    h->cap = n;
    return 0;
}

extern "C" {

int bftwire_create(int hip_device, bftwire_t** out) {
    if (!out) return -1;
    bftwire* h = new bftwire();
    h->device = hip_device;
    const char* dm = getenv("BFTWIRE_DECODE");
    h->decode_mode = (dm && strcmp(dm, "lds") == 0) ? 1 : (dm && strcmp(dm, "wave") == 0) ? 2 : 0;
    *out = h;
    WCHECK(h, hipSetDevice(hip_device));
    return 0;
}

void bftwire_destroy(bftwire_t* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    wire_free(h);
    delete h;
}

const char* bftwire_last_error(const bftwire_t* h) { return h ? h->err.c_str() : "null handle"; }

int bftwire_encode(bftwire_t* h, const bftwire_batch* in, uint64_t n, uint8_t* stream, uint64_t cap, uint64_t* frame_off,
                   uint8_t* sign_digest, uint8_t* msg_hash, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (!in || !frame_off || !ok || (n && (!stream || !in->code || !in->round || !in->height || !in->digest ||
                                           !in->create_time)))
        return wfail(h, -1, "bftwire_encode: null buffer");
    if (n > 0x7fffffffull) return wfail(h, -1, "bftwire_encode: batch too large");
    hipStream_t s = (hipStream_t)stream_;
    WCHECK(h, hipSetDevice(h->device));
    if (n == 0) return hipMemsetAsync(frame_off, 0, 8, s) == hipSuccess ? 0 : wfail(h, -2, "memset");
    if (int rc = wire_reserve(h, n)) return rc;
    EncParams p;
    p.in = *in;
    p.n = n;
    p.slot_f = h->slot_f; p.slot_g = h->slot_g; p.slot_sp = h->slot_sp;
    p.lens = h->lens; p.glen = h->glen; p.splen = h->splen;
    p.ok = ok;
    p.want_hash = (sign_digest || msg_hash) ? 1u : 0u;
    const unsigned blocks = (unsigned)((n + WAVES - 1) / WAVES);
    hipLaunchKernelGGL(wire_encode_kernel, dim3(blocks), dim3(64 * WAVES), 0, s, p);
    WCHECK(h, hipGetLastError());
    size_t tb = h->scan_bytes;
    WCHECK(h, hipcub::DeviceScan::ExclusiveSum(h->scan_tmp, tb, h->lens, frame_off, (int)(n + 1), s));
    hipLaunchKernelGGL(wire_pack_kernel, dim3(blocks), dim3(64 * WAVES), 0, s, h->slot_f, frame_off, n, stream, cap, ok);
    WCHECK(h, hipGetLastError());
    if (p.want_hash) {
        hipLaunchKernelGGL(wire_hash_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, h->slot_g, h->slot_sp,
                           h->glen, h->splen, n, msg_hash, sign_digest);
        WCHECK(h, hipGetLastError());
    }
    return 0;
}

int bftwire_decode(bftwire_t* h, const uint8_t* stream, const uint64_t* frame_off, uint64_t n, const bftwire_batch* out,
                   uint8_t* has_sig, uint8_t* has_seal, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (n == 0) return 0;
    if (!stream || !frame_off || !out || !has_sig || !has_seal || !ok || !out->code || !out->round || !out->height ||
        !out->digest || !out->create_time || !out->signature || !out->commit_seal || !out->ttl || !out->raw_time)
        return wfail(h, -1, "bftwire_decode: null buffer");
    WCHECK(h, hipSetDevice(h->device));
    if (h->decode_mode == 0)       // product: lane per frame straight from global memory
        hipLaunchKernelGGL(wire_decode_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream_,
                           stream, frame_off, n, *out, has_sig, has_seal, ok);
    else if (h->decode_mode == 1)  // BFTWIRE_DECODE=lds: frames staged in LDS first (A/B)
        hipLaunchKernelGGL(wire_decode_lds_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream_,
                           stream, frame_off, n, *out, has_sig, has_seal, ok);
    else                           // BFTWIRE_DECODE=wave: the wave-cooperative decoder (A/B)
        hipLaunchKernelGGL(wire_decode_wave_kernel, dim3((unsigned)((n + WAVES - 1) / WAVES)), dim3(64 * WAVES), 0,
                           (hipStream_t)stream_, stream, frame_off, n, *out, has_sig, has_seal, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

uint64_t bftwire_split_frames(const uint8_t* b, uint64_t len, uint64_t* offs, uint64_t max) {
    uint64_t i = 0, k = 0;
    if (!b || !offs) return 0;
    offs[0] = 0;
    while (k < max && i + 4 <= len) {
        uint64_t sz = ((uint64_t)b[i] << 24) | ((uint64_t)b[i + 1] << 16) | ((uint64_t)b[i + 2] << 8) | b[i + 3];
        if (i + 4 + sz > len) break;                    // incomplete frame: Ok(None), wait for more bytes
        i += 4 + sz;
        offs[++k] = i;
    }
    return k;
}

}  // extern "C"
