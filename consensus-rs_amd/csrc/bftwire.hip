// bftwire.hip — gfx950 kernels and the C ABI of libbftwire (include/bftwire.h): the consensus wire
// codec, batched. Encoding is wave-per-message: the nested MessagePack levels (Subject -> GossipMessage
// -> RawMessage frame) are assembled in LDS, each level's byte array expanded by all 64 lanes at once
// (a byte >= 128 becomes 0xcc b: the output position of every byte is a ballot prefix count), then
// written to a per-message slot with coalesced dword stores; a device scan gives the frame offsets and
// a pack pass copies the slots into the contiguous stream (lanes write consecutive bytes). The two
// Keccak-256 digests run lane-per-message over the GossipMessage / sign-payload slots. Decoding is
// lane-per-frame through the streaming decoder of bft_wire.h (plain byte loads: a 16-byte or 4-byte
// register window measured 1.6-1.9x slower — the per-byte window test diverges the loads; an
// LDS-staged and a wave-per-frame decoder measured 1.25x and 2.2x slower and were removed).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../../include/bftwire.h"

// the block-frame structs are mirrored by hand-coded numpy dtypes (bftsim/wire.py TX_DTYPE, BLOCK_DTYPE,
// PP_DTYPE) and by INTEGRATION.md's Rust binding: their layout is part of the ABI
#include <stddef.h>
static_assert(sizeof(bftwire_tx) == 200, "bftwire_tx ABI");
static_assert(offsetof(bftwire_tx, payload_len) == 32 && offsetof(bftwire_tx, recipient) == 40 &&
              offsetof(bftwire_tx, payload) == 60 && offsetof(bftwire_tx, sig) == 124, "bftwire_tx ABI");
static_assert(sizeof(bftwire_block) == 1688, "bftwire_block ABI");
static_assert(offsetof(bftwire_block, extra_len) == 48 && offsetof(bftwire_block, prev_hash) == 64 &&
              offsetof(bftwire_block, proposer) == 192 && offsetof(bftwire_block, extra) == 212 &&
              offsetof(bftwire_block, votes) == 244 && offsetof(bftwire_block, tx) == 1288, "bftwire_block ABI");
static_assert(sizeof(bftwire_preprepare) == 1808, "bftwire_preprepare ABI");
static_assert(offsetof(bftwire_preprepare, has_sig) == 40 && offsetof(bftwire_preprepare, signature) == 48 &&
              offsetof(bftwire_preprepare, block) == 120, "bftwire_preprepare ABI");
#include "bft_wire.h"
#include "bft_wire_block.h"

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


// ---------------------------------------------------------------- block-carrying frames (SPEC.md §9b)
// Lane per frame: a counting pass gives every frame's length, a device scan the offsets, a writing pass
// the bytes at their offsets (and, for Preprepare, the two Keccak-256 digests streamed from the same
// emitter). These messages are O(N) per round (one Preprepare, block gossip), not the O(N^2) votes.
__global__ __launch_bounds__(64) void wire_pp_len_kernel(const bftwire_preprepare* in, uint64_t n, uint64_t* lens,
                                                         uint8_t* ok) {
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n) { if (i == n) lens[n] = 0; return; }
    const bftwire_preprepare& m = in[i];
    const bool fit = block_fits(m.block);
    uint32_t L = 0;
    if (fit) emit_frame(CountE{&L}, P2P_CONSENSUS, m.ttl, m.raw_time, [&](const auto& e) { emit_pp_gossip(e, m, true); });
    lens[i] = fit ? L : 0;
    ok[i] = fit ? 1 : 0;
}
__global__ __launch_bounds__(64) void wire_pp_write_kernel(const bftwire_preprepare* in, uint64_t n, const uint64_t* off,
                                                           uint8_t* stream, uint64_t cap, uint8_t* sign_digest,
                                                           uint8_t* msg_hash, uint8_t* ok) {
    __shared__ uint8_t kb[64 * 136];
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    const bftwire_preprepare& m = in[i];
    if (ok[i] && off[i + 1] <= cap) {
        uint32_t w = 0;
        emit_frame(BufE{stream + off[i], &w, (uint32_t)(off[i + 1] - off[i])}, P2P_CONSENSUS, m.ttl, m.raw_time,
                   [&](const auto& e) { emit_pp_gossip(e, m, true); });
    } else {
        ok[i] = 0;
    }
    uint8_t* kbuf = kb + threadIdx.x * 136;
    if (sign_digest) {
        crypto::KSink k(kbuf);
        if (ok[i]) emit_pp_gossip(KE{&k}, m, false);
        uint8_t o[32];
        k.finish(o);
        for (int j = 0; j < 32; ++j) sign_digest[32u * i + j] = ok[i] ? o[j] : 0;
    }
    if (msg_hash) {
        crypto::KSink k(kbuf);
        if (ok[i]) emit_pp_gossip(KE{&k}, m, true);
        uint8_t o[32];
        k.finish(o);
        for (int j = 0; j < 32; ++j) msg_hash[32u * i + j] = ok[i] ? o[j] : 0;
    }
}
__global__ __launch_bounds__(64) void wire_pp_decode_kernel(const uint8_t* stream, const uint64_t* off, uint64_t n,
                                                            bftwire_preprepare* out, uint8_t* ok) {
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    bftwire_preprepare d;
    memset(&d, 0, sizeof d);
    const uint64_t o = off[i], len = off[i + 1] - o;
    const bool good = len < (1u << 20) && decode_pp_frame(stream + o, (uint32_t)len, d);
    if (!good) memset(&d, 0, sizeof d);
    out[i] = d;
    ok[i] = good ? 1 : 0;
}

template <class E>
__device__ inline void emit_blocks_payload(const E& e, const bftwire_block* b, uint64_t lo, uint64_t hi) {
    mp_arr(e, (uint32_t)(hi - lo));                       // Blocks(Vec<Block>): newtype, transparent
    for (uint64_t j = lo; j < hi; ++j) emit_block(e, b[j]);
}
__global__ __launch_bounds__(64) void wire_blocks_len_kernel(const bftwire_block* b, const uint64_t* boff, uint64_t n,
                                                             const uint64_t* ttl, const uint64_t* rtime, uint64_t* lens,
                                                             uint8_t* ok) {
    const uint64_t k = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (k >= n) { if (k == n) lens[n] = 0; return; }
    bool fit = true;
    for (uint64_t j = boff[k]; j < boff[k + 1]; ++j) fit = fit && block_fits(b[j]);
    uint32_t L = 0;
    if (fit)
        emit_frame(CountE{&L}, P2P_BLOCK, ttl ? ttl[k] : DEFAULT_TTL, rtime ? rtime[k] : 0ull,
                   [&](const auto& e) { emit_blocks_payload(e, b, boff[k], boff[k + 1]); });
    lens[k] = fit ? L : 0;
    ok[k] = fit ? 1 : 0;
}
__global__ __launch_bounds__(64) void wire_blocks_write_kernel(const bftwire_block* b, const uint64_t* boff, uint64_t n,
                                                               const uint64_t* ttl, const uint64_t* rtime,
                                                               const uint64_t* off, uint8_t* stream, uint64_t cap,
                                                               uint8_t* ok) {
    const uint64_t k = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (k >= n) return;
    if (!ok[k] || off[k + 1] > cap) { ok[k] = 0; return; }
    uint32_t w = 0;
    emit_frame(BufE{stream + off[k], &w, (uint32_t)(off[k + 1] - off[k])}, P2P_BLOCK, ttl ? ttl[k] : DEFAULT_TTL,
               rtime ? rtime[k] : 0ull, [&](const auto& e) { emit_blocks_payload(e, b, boff[k], boff[k + 1]); });
}
__global__ __launch_bounds__(64) void wire_blocks_decode_kernel(const uint8_t* stream, const uint64_t* off, uint64_t n,
                                                                uint32_t maxpf, bftwire_block* out, uint32_t* count,
                                                                uint8_t* ok) {
    const uint64_t k = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (k >= n) return;
    const uint64_t o = off[k], len = off[k + 1] - o;
    const uint8_t* f = stream + o;
    bool good = len >= 4 && len < (1u << 24) && frame_size(f) == len - 4u;
    uint32_t cnt = 0;
    if (good) {
        Mem m{f + 4, (uint32_t)len - 4u, 0};
        uint64_t t, rt;
        uint32_t plen;
        good = rd_envelope(m, P2P_BLOCK, t, rt, plen);
        if (good) {
            Arr<Mem> p{&m, plen, false};
            good = rd_arr(p, cnt) && cnt <= maxpf;
            for (uint32_t j = 0; good && j < cnt; ++j) {
                bftwire_block blk;
                memset(&blk, 0, sizeof blk);
                good = rd_block(p, blk);
                out[k * maxpf + j] = blk;
            }
            good = good && p.left == 0 && !p.bad && m.i == m.n;
        }
    }
    count[k] = good ? cnt : 0;
    ok[k] = good ? 1 : 0;
}

__global__ __launch_bounds__(64) void wire_sync_len_kernel(const uint64_t* height, uint64_t n, const uint64_t* ttl,
                                                           const uint64_t* rtime, uint64_t* lens) {
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n) { if (i == n) lens[n] = 0; return; }
    uint32_t L = 0;
    const uint64_t hv = height[i];
    emit_frame(CountE{&L}, P2P_SYNC, ttl ? ttl[i] : DEFAULT_TTL, rtime ? rtime[i] : 0ull,
               [&](const auto& e) { mp_uint(e, hv); });
    lens[i] = L;
}
__global__ __launch_bounds__(64) void wire_sync_write_kernel(const uint64_t* height, uint64_t n, const uint64_t* ttl,
                                                             const uint64_t* rtime, const uint64_t* off, uint8_t* stream,
                                                             uint64_t cap, uint8_t* ok) {
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    if (off[i + 1] > cap) { ok[i] = 0; return; }
    uint32_t w = 0;
    const uint64_t hv = height[i];
    emit_frame(BufE{stream + off[i], &w, (uint32_t)(off[i + 1] - off[i])}, P2P_SYNC, ttl ? ttl[i] : DEFAULT_TTL,
               rtime ? rtime[i] : 0ull, [&](const auto& e) { mp_uint(e, hv); });
    ok[i] = 1;
}
__global__ __launch_bounds__(64) void wire_sync_decode_kernel(const uint8_t* stream, const uint64_t* off, uint64_t n,
                                                              uint64_t* height, uint8_t* ok) {
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i], len = off[i + 1] - o;
    uint64_t hv = 0;
    const bool good = len < (1u << 20) && decode_sync_frame(stream + o, (uint32_t)len, hv);
    height[i] = good ? hv : 0;
    ok[i] = good ? 1 : 0;
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
    // lane per frame straight from global memory
    hipLaunchKernelGGL(wire_decode_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream_,
                       stream, frame_off, n, *out, has_sig, has_seal, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

// the three-pass frame encoders: per-frame lengths, scan into frame_off, bytes at the offsets
static int frames_scan(bftwire* h, uint64_t n, uint64_t* frame_off, hipStream_t s) {
    size_t tb = h->scan_bytes;
    WCHECK(h, hipcub::DeviceScan::ExclusiveSum(h->scan_tmp, tb, h->lens, frame_off, (int)(n + 1), s));
    return 0;
}
static inline dim3 lanes(uint64_t n) { return dim3((unsigned)((n + 1 + 63) / 64)); }

int bftwire_encode_preprepare(bftwire_t* h, const bftwire_preprepare* in, uint64_t n, uint8_t* stream, uint64_t cap,
                              uint64_t* frame_off, uint8_t* sign_digest, uint8_t* msg_hash, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (!frame_off || !ok || (n && (!in || !stream))) return wfail(h, -1, "bftwire_encode_preprepare: null buffer");
    if (n > 0x7fffffffull) return wfail(h, -1, "bftwire_encode_preprepare: batch too large");
    hipStream_t s = (hipStream_t)stream_;
    WCHECK(h, hipSetDevice(h->device));
    if (n == 0) return hipMemsetAsync(frame_off, 0, 8, s) == hipSuccess ? 0 : wfail(h, -2, "memset");
    if (int rc = wire_reserve(h, n)) return rc;
    hipLaunchKernelGGL(wire_pp_len_kernel, lanes(n), dim3(64), 0, s, in, n, h->lens, ok);
    WCHECK(h, hipGetLastError());
    if (int rc = frames_scan(h, n, frame_off, s)) return rc;
    hipLaunchKernelGGL(wire_pp_write_kernel, lanes(n), dim3(64), 0, s, in, n, frame_off, stream, cap, sign_digest, msg_hash, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

int bftwire_decode_preprepare(bftwire_t* h, const uint8_t* stream, const uint64_t* frame_off, uint64_t n,
                              bftwire_preprepare* out, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (n == 0) return 0;
    if (!stream || !frame_off || !out || !ok) return wfail(h, -1, "bftwire_decode_preprepare: null buffer");
    WCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(wire_pp_decode_kernel, lanes(n), dim3(64), 0, (hipStream_t)stream_, stream, frame_off, n, out, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

int bftwire_encode_blocks(bftwire_t* h, const bftwire_block* blocks, const uint64_t* block_off, uint64_t n,
                          const uint64_t* ttl, const uint64_t* raw_time, uint8_t* stream, uint64_t cap,
                          uint64_t* frame_off, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (!frame_off || !ok || (n && (!blocks || !block_off || !stream))) return wfail(h, -1, "bftwire_encode_blocks: null buffer");
    if (n > 0x7fffffffull) return wfail(h, -1, "bftwire_encode_blocks: batch too large");
    hipStream_t s = (hipStream_t)stream_;
    WCHECK(h, hipSetDevice(h->device));
    if (n == 0) return hipMemsetAsync(frame_off, 0, 8, s) == hipSuccess ? 0 : wfail(h, -2, "memset");
    if (int rc = wire_reserve(h, n)) return rc;
    hipLaunchKernelGGL(wire_blocks_len_kernel, lanes(n), dim3(64), 0, s, blocks, block_off, n, ttl, raw_time, h->lens, ok);
    WCHECK(h, hipGetLastError());
    if (int rc = frames_scan(h, n, frame_off, s)) return rc;
    hipLaunchKernelGGL(wire_blocks_write_kernel, lanes(n), dim3(64), 0, s, blocks, block_off, n, ttl, raw_time, frame_off,
                       stream, cap, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

int bftwire_decode_blocks(bftwire_t* h, const uint8_t* stream, const uint64_t* frame_off, uint64_t n, uint32_t max_per_frame,
                          bftwire_block* out, uint32_t* count, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (n == 0) return 0;
    if (!stream || !frame_off || !out || !count || !ok) return wfail(h, -1, "bftwire_decode_blocks: null buffer");
    WCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(wire_blocks_decode_kernel, lanes(n), dim3(64), 0, (hipStream_t)stream_, stream, frame_off, n,
                       max_per_frame, out, count, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

int bftwire_encode_sync(bftwire_t* h, const uint64_t* height, uint64_t n, const uint64_t* ttl, const uint64_t* raw_time,
                        uint8_t* stream, uint64_t cap, uint64_t* frame_off, uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (!frame_off || !ok || (n && (!height || !stream))) return wfail(h, -1, "bftwire_encode_sync: null buffer");
    if (n > 0x7fffffffull) return wfail(h, -1, "bftwire_encode_sync: batch too large");
    hipStream_t s = (hipStream_t)stream_;
    WCHECK(h, hipSetDevice(h->device));
    if (n == 0) return hipMemsetAsync(frame_off, 0, 8, s) == hipSuccess ? 0 : wfail(h, -2, "memset");
    if (int rc = wire_reserve(h, n)) return rc;
    hipLaunchKernelGGL(wire_sync_len_kernel, lanes(n), dim3(64), 0, s, height, n, ttl, raw_time, h->lens);
    WCHECK(h, hipGetLastError());
    if (int rc = frames_scan(h, n, frame_off, s)) return rc;
    hipLaunchKernelGGL(wire_sync_write_kernel, lanes(n), dim3(64), 0, s, height, n, ttl, raw_time, frame_off, stream, cap, ok);
    WCHECK(h, hipGetLastError());
    return 0;
}

int bftwire_decode_sync(bftwire_t* h, const uint8_t* stream, const uint64_t* frame_off, uint64_t n, uint64_t* height,
                        uint8_t* ok, void* stream_) {
    using namespace bft::wire;
    if (!h) return -1;
    if (n == 0) return 0;
    if (!stream || !frame_off || !height || !ok) return wfail(h, -1, "bftwire_decode_sync: null buffer");
    WCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(wire_sync_decode_kernel, lanes(n), dim3(64), 0, (hipStream_t)stream_, stream, frame_off, n, height, ok);
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
