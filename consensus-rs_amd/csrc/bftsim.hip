// bftsim.hip — gfx950 kernels and the C ABI of libbftsim (include/bftsim.h).
//
// Kernels:
//   bft_consensus_kernel  one 64-lane wave per 64/S instances (N <= 64), or one workgroup of
//                         S = 128 / 256 lanes per instance (N <= 256); lane = validator (bft_wave.h);
//   bft_consensus_fast_kernel  N = 64 with big-endian seeds: the closed-form phases (bft_fast64.h),
//                         handing instances that need the general path to bft_consensus_resume_kernel;
//   bft_hash_pair_kernel  one lane pair per instance: Keccak-256 of every committed header, chained
//                         through prev_hash (big-endian seeds and power-of-two N, where proposer
//                         seeds are always 0 and the consensus kernel does not need hashes);
//   bft_stats_kernel      per-launch totals for the RCCL all-reduce of the benchmark.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <dlfcn.h>
#include <unistd.h>
#include <rccl/rccl.h>                 // types only: librccl is opened at bftsim_comm_init (dlopen)

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "bft_hip.h"
#include "bft_fast64.h"
#include "bft_crypto.h"

namespace bft {


// ledger export (core/ledger.rs:193-245): the Header bytes of every committed height, thread per
// (instance, height), parent hash from the hash table; into 8-aligned BFTSIM_HEADER_SLOT-byte slots
__global__ __launch_bounds__(256) void bft_export_kernel(Params p, uint8_t* out, uint32_t* lens) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t H = p.heights;
    if (t >= (uint64_t)p.n_instances * H) return;
    const uint32_t il = (uint32_t)(t / H), x = (uint32_t)(t % H) + 1u;
    if (x > p.committed_height[il]) { lens[t] = 0; return; }
    uint32_t prev[8];
    if (x == 1) {
        for (int i = 0; i < 8; ++i)
            prev[i] = (uint32_t)p.genesis_hash[4 * i] | ((uint32_t)p.genesis_hash[4 * i + 1] << 8) |
                      ((uint32_t)p.genesis_hash[4 * i + 2] << 16) | ((uint32_t)p.genesis_hash[4 * i + 3] << 24);
    } else {
        const uint32_t* ph = (const uint32_t*)(p.hash + ((uint64_t)il * p.rows + (x - 1)) * 32);
        for (int i = 0; i < 8; ++i) prev[i] = ph[i];
    }
    const uint32_t* row = p.rec + ((uint64_t)il * p.rows + x) * 4;
    const uint32_t prop = row[1] & 0xffffu, var = (row[1] >> 16) & 1u;
    const uint64_t time = p.genesis_time + (uint64_t)p.block_period * ((uint64_t)row[2] + 1ull);
    lens[t] = header_raw((uint64_t*)(out + t * BFTSIM_HEADER_SLOT), prev, p.addresses + 20u * prop, p.seed,
                         p.first_instance + il, x, prop, var, time);
}

// totals: [0] instances [1] committed [2] views [3] ticks [4..10] flag counts (the histograms are
// accumulated by the consensus kernel); block-level reduction in LDS, then one global atomic per
// counter per block
constexpr int STAT_WORDS = 11;
__global__ __launch_bounds__(256) void bft_stats_kernel(Params p, unsigned long long* st) {
    __shared__ unsigned long long acc[STAT_WORDS];
    for (uint32_t k = threadIdx.x; k < STAT_WORDS; k += 256) acc[k] = 0;
    __syncthreads();
    uint32_t il = blockIdx.x * 256u + threadIdx.x;
    if (il < p.n_instances) {
        atomicAdd(&acc[0], 1ull);
        atomicAdd(&acc[1], (unsigned long long)p.committed_height[il]);
        atomicAdd(&acc[2], (unsigned long long)p.views[il]);
        atomicAdd(&acc[3], (unsigned long long)p.ticks[il]);
        uint32_t f = p.flags[il];
        for (int b = 0; b < 7; ++b)
            if (f & (1u << b)) atomicAdd(&acc[4 + b], 1ull);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < STAT_WORDS; k += 256)
        if (acc[k]) atomicAdd(&st[k], acc[k]);
}

// hash of each instance's block at its committed height (the genesis hash at height 0): it
// commits to the whole chain, so it stands in for the per-height rows in windowed runs
__global__ __launch_bounds__(256) void bft_tip_kernel(Params p, uint8_t* tips) {
    uint32_t il = blockIdx.x * 256u + threadIdx.x;
    if (il >= p.n_instances) return;
    uint32_t ch = p.committed_height[il];
    const uint8_t* src = ch == 0 ? p.genesis_hash
                                 : p.hash + ((uint64_t)il * p.rows + (p.window_mask ? (ch & p.window_mask) : ch)) * 32;
    for (int i = 0; i < 32; ++i) tips[(uint64_t)il * 32 + i] = src[i];
}


// ------------------------------------------------------------------------------ real-crypto mode
// The batched sign / recover pass over a launch's broadcast log (SPEC.md §11; bftsim_crypto_verify).
struct CryptoArgs {
    const uint32_t* mlog;
    const uint32_t* mlog_n;
    uint32_t cap;
    uint32_t n_val;
    const uint64_t* moff;             // [n_inst] first dense message index of each instance
    uint64_t forged[4];
    // dense, per message
    uint64_t* mref;                   // instance * cap + slot
    uint8_t* raw;                     // Subject digest (block hash, zeros for RoundChange)
    uint32_t* key;                    // signing key: sender, or n_val + sender (forged key)
    uint32_t* msg_k;                  // commit seal index
    uint8_t* sign_dig;
    uint8_t* sigs;
    uint8_t* rec_addr;
    uint8_t* rec_ok;
    // dense, per commit
    uint32_t* ncm;
    uint8_t* seal_dig;
    uint8_t* seal_raw;
    uint32_t* seal_key;
    uint8_t* seals;
    uint8_t* seal_ok;
    // results
    uint32_t* inst_ck;                // [n_inst][8] XOR of keccak(signature || seal)
    unsigned long long* counts;       // [8] messages, commits, forged, recovered-as-sender, mismatches, seal errors
};

// parent hash of the block at height x as the run left it: the canonical row x-1 (genesis at 1); a
// height above the committed chain + 1 has no known parent and uses 0^32 (SPEC.md §11)
__device__ inline void crypto_parent(const Params& p, uint32_t il, uint32_t x, uint32_t prev[8]) {
    const uint32_t ch = p.committed_height[il];
    if (x <= 1) {
        for (int i = 0; i < 8; ++i)
            prev[i] = (uint32_t)p.genesis_hash[4 * i] | ((uint32_t)p.genesis_hash[4 * i + 1] << 8) |
                      ((uint32_t)p.genesis_hash[4 * i + 2] << 16) | ((uint32_t)p.genesis_hash[4 * i + 3] << 24);
    } else if (x - 1 <= ch) {
        const uint32_t* ph = (const uint32_t*)(p.hash + ((uint64_t)il * p.rows + (x - 1)) * 32);
        for (int i = 0; i < 8; ++i) prev[i] = ph[i];
    } else {
        for (int i = 0; i < 8; ++i) prev[i] = 0;
    }
}
// Subject digest of a logged block id: the canonical row's hash when the block is the committed one
// at its height, else the hash of its header over crypto_parent
__device__ inline void crypto_block_digest(const Params& p, uint32_t il, uint64_t b, uint8_t* hbuf, uint8_t out[32]) {
    const uint32_t x = blk_h(b), prop = blk_prop(b), var = blk_var(b);
    if (!blk_valid(b) || x == 0) { for (int i = 0; i < 32; ++i) out[i] = 0; return; }
    if (x <= p.committed_height[il]) {
        const uint32_t* row = p.rec + ((uint64_t)il * p.rows + x) * 4;
        if ((row[1] & 0xffffu) == prop && ((row[1] >> 16) & 1u) == var) {
            const uint8_t* hs = p.hash + ((uint64_t)il * p.rows + x) * 32;
            for (int i = 0; i < 32; ++i) out[i] = hs[i];
            return;
        }
    }
    uint32_t prev[8], w[8];
    crypto_parent(p, il, x, prev);
    const uint64_t time = p.genesis_time + (uint64_t)p.block_period * ((uint64_t)blk_T(b) + 1ull);
    lane_block_hash(hbuf, prev, p.addresses + 20u * prop, p.seed, p.first_instance + il, x, prop, var, time, w);
    for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

// pass 1 (workgroup per instance): digests, signing keys, the commits' seal digests
__global__ __launch_bounds__(64) void bft_crypto_prep_kernel(Params p, CryptoArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t hb[64 * LANE_HASH_BUF];
    __shared__ uint8_t kb[64 * 136];
    uint8_t* hbuf = hb + threadIdx.x * LANE_HASH_BUF;
    uint8_t* kbuf = kb + threadIdx.x * 136;
    const uint32_t il = blockIdx.x;
    const uint32_t cnt = a.mlog_n[il] < a.cap ? a.mlog_n[il] : a.cap;
    for (uint32_t j = threadIdx.x; j < cnt; j += 64u) {
        const uint32_t* e = a.mlog + ((uint64_t)il * a.cap + j) * MLOG_WORDS;
        const uint64_t m = a.moff[il] + j;
        const uint32_t code = (e[1] >> 8) & 0xffu, sender = e[1] >> 16;
        const bool forged = (e[6] & MLOG_FORGED) != 0;
        uint8_t d[32];
        if (code == MT_ROUND_CHANGE) { for (int i = 0; i < 32; ++i) d[i] = 0; }     // EMPTY_HASH (round_change.rs:55-58)
        else crypto_block_digest(p, il, (uint64_t)e[4] | ((uint64_t)e[5] << 32), hbuf, d);
        for (int i = 0; i < 32; ++i) a.raw[m * 32 + i] = d[i];
        const uint32_t key = sender + (forged ? a.n_val : 0u);
        a.key[m] = key;
        a.mref[m] = (uint64_t)il * a.cap + j;
        if (code == MT_COMMIT) {
            const uint32_t k = atomicAdd(a.ncm, 1u);
            a.msg_k[m] = k;
            a.seal_key[k] = key;
            uint8_t sd[32];
            crypto::seal_digest(kbuf, d, sd);
            for (int i = 0; i < 32; ++i) { a.seal_dig[(uint64_t)k * 32 + i] = sd[i]; a.seal_raw[(uint64_t)k * 32 + i] = d[i]; }
        }
    }
}

// pass 2 (lane per message): the sign digest of the GossipMessage (signature None, the seal of a Commit)
__global__ __launch_bounds__(64) void bft_crypto_digest_kernel(Params p, CryptoArgs a, uint64_t M) {
    __shared__ __attribute__((aligned(16))) uint8_t hb[64 * LANE_HASH_BUF];
    __shared__ uint8_t kb[64 * 136];
    const uint64_t m = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (m >= M) return;
    uint8_t* hbuf = hb + threadIdx.x * LANE_HASH_BUF;
    uint8_t* kbuf = kb + threadIdx.x * 136;
    const uint64_t ref = a.mref[m];
    const uint32_t il = (uint32_t)(ref / a.cap);
    const uint32_t* e = a.mlog + ref * MLOG_WORDS;
    const uint32_t code = (e[1] >> 8) & 0xffu, tick = e[0];
    const uint32_t h_ = e[2], r_ = e[3];
    // create_time: RoundChange carries the wall clock in ms (round_change.rs:61), the others 0
    const uint64_t ctime = code == MT_ROUND_CHANGE
                               ? 1000ull * (p.genesis_time + (uint64_t)p.block_period * (uint64_t)tick) : 0ull;
    const uint8_t* seal = code == MT_COMMIT ? a.seals + (uint64_t)a.msg_k[m] * 65 : nullptr;
    uint8_t out[32];
    if (code == MT_PREPREPARE) {
        const uint64_t b = (uint64_t)e[4] | ((uint64_t)e[5] << 32);
        const uint32_t x = blk_h(b), prop = blk_prop(b), var = blk_var(b);
        uint32_t prev[8];
        crypto_parent(p, il, x, prev);
        const uint64_t time = p.genesis_time + (uint64_t)p.block_period * ((uint64_t)blk_T(b) + 1ull);
        const uint32_t hlen = header_raw((uint64_t*)hbuf, prev, p.addresses + 20u * prop, p.seed, p.first_instance + il,
                                         x, prop, var, time);
        crypto::sign_digest(kbuf, code, ctime, r_, h_, nullptr, hbuf, hlen, nullptr, out);
    } else {
        crypto::sign_digest(kbuf, code, ctime, r_, h_, a.raw + m * 32, nullptr, 0, seal, out);
    }
    for (int i = 0; i < 32; ++i) a.sign_dig[m * 32 + i] = out[i];
}

// pass 3 (lane per message): the receivers' checks (handle_message, core.rs:314-322: the recovered
// address must be a validator; verify_commit, commit.rs:94-100: the seal must recover) against what the
// simulation assumed (forged senders dropped, everyone else accepted), and the per-instance checksum
__global__ __launch_bounds__(64) void bft_crypto_check_kernel(Params p, CryptoArgs a, uint64_t M) {
    __shared__ uint8_t kb[64 * 136];
    const uint64_t m = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (m >= M) return;
    uint8_t* kbuf = kb + threadIdx.x * 136;
    const uint64_t ref = a.mref[m];
    const uint32_t il = (uint32_t)(ref / a.cap);
    const uint32_t* e = a.mlog + ref * MLOG_WORDS;
    const uint32_t code = (e[1] >> 8) & 0xffu, sender = e[1] >> 16;
    const bool forged = (e[6] & MLOG_FORGED) != 0;
    const uint8_t* ra = a.rec_addr + m * 20;
    bool member = false, as_sender = false;
    if (a.rec_ok[m]) {
        for (uint32_t v = 0; v < a.n_val; ++v) {
            bool eq = true;
            for (int i = 0; i < 20 && eq; ++i) eq = ra[i] == p.addresses[20u * v + i];
            if (eq) { member = true; as_sender = as_sender || v == sender; }
        }
    }
    bool seal_err = false;
    const uint8_t* seal = nullptr;
    if (code == MT_COMMIT) {
        const uint32_t k = a.msg_k[m];
        seal = a.seals + (uint64_t)k * 65;
        seal_err = !a.seal_ok[k];
    }
    const bool mismatch = forged ? member : !as_sender;
    uint8_t t[32];
    crypto::sig_term(kbuf, a.sigs + m * 65, seal, t);
    for (int w = 0; w < 8; ++w) {
        const uint32_t v = (uint32_t)t[4 * w] | ((uint32_t)t[4 * w + 1] << 8) | ((uint32_t)t[4 * w + 2] << 16) |
                           ((uint32_t)t[4 * w + 3] << 24);
        atomicXor(a.inst_ck + (uint64_t)il * 8 + w, v);
    }
    atomicAdd(a.counts + 0, 1ull);
    if (code == MT_COMMIT) atomicAdd(a.counts + 1, 1ull);
    if (forged) atomicAdd(a.counts + 2, 1ull);
    if (as_sender) atomicAdd(a.counts + 3, 1ull);
    if (mismatch) atomicAdd(a.counts + 4, 1ull);
    if (seal_err) atomicAdd(a.counts + 5, 1ull);
}


// pass 4 (lane per message): the signatures of the canonical committer's commit set (the block's votes,
// core.rs:402-413 → backend.rs:163-174): each Commit of height x, the committed round, the committed
// block (or a wildcard), from a sender in that set
__global__ __launch_bounds__(64) void bft_crypto_votes_kernel(Params p, CryptoArgs a, uint64_t M, uint8_t* vsig,
                                                              uint8_t* vhas) {
    const uint64_t m = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (m >= M) return;
    const uint64_t ref = a.mref[m];
    const uint32_t il = (uint32_t)(ref / a.cap);
    const uint32_t* e = a.mlog + ref * MLOG_WORDS;
    const uint32_t code = (e[1] >> 8) & 0xffu, sender = e[1] >> 16, x = e[2], r = e[3];
    if (code != MT_COMMIT || (e[6] & MLOG_OLD) || x == 0 || x > p.committed_height[il]) return;
    const uint32_t* row = p.rec + ((uint64_t)il * p.rows + x) * 4;
    const uint64_t b = (uint64_t)e[4] | ((uint64_t)e[5] << 32);
    if (row[0] != r) return;
    if (!(e[6] & MLOG_WILD) && ((row[1] & 0xffffu) != blk_prop(b) || ((row[1] >> 16) & 1u) != blk_var(b))) return;
    const uint32_t* vo = p.votes + ((uint64_t)il * p.rows + x) * 8;
    if (!((vo[sender >> 5] >> (sender & 31u)) & 1u)) return;
    const uint64_t slot = ((uint64_t)il * p.heights + (x - 1)) * p.n + sender;
    for (int i = 0; i < 65; ++i) vsig[slot * 65 + i] = a.sigs[m * 65 + i];
    vhas[slot] = 1;
}

// the ledger's Header of every committed height with its votes (SPEC.md §11): the header bytes of
// bft_export_kernel with `votes: Some(Votes([signature...]))` in ascending validator order (the
// reference's order is a HashMap's, protocol/mod.rs:183); thread per (instance, height)
__global__ __launch_bounds__(64) void bft_export_votes_kernel(Params p, const uint8_t* vsig, const uint8_t* vhas,
                                                             uint8_t* out, uint64_t slot, uint32_t* lens) {
    __shared__ __attribute__((aligned(16))) uint64_t wbs[64 * HDR_WORDS];
    const uint64_t t = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    const uint64_t H = p.heights;
    if (t >= (uint64_t)p.n_instances * H) return;
    const uint32_t il = (uint32_t)(t / H), x = (uint32_t)(t % H) + 1u;
    if (x > p.committed_height[il]) { lens[t] = 0; return; }
    uint32_t prev[8];
    if (x == 1) {
        for (int i = 0; i < 8; ++i)
            prev[i] = (uint32_t)p.genesis_hash[4 * i] | ((uint32_t)p.genesis_hash[4 * i + 1] << 8) |
                      ((uint32_t)p.genesis_hash[4 * i + 2] << 16) | ((uint32_t)p.genesis_hash[4 * i + 3] << 24);
    } else {
        const uint32_t* ph = (const uint32_t*)(p.hash + ((uint64_t)il * p.rows + (x - 1)) * 32);
        for (int i = 0; i < 8; ++i) prev[i] = ph[i];
    }
    const uint32_t* row = p.rec + ((uint64_t)il * p.rows + x) * 4;
    const uint32_t prop = row[1] & 0xffffu, var = (row[1] >> 16) & 1u;
    const uint64_t time = p.genesis_time + (uint64_t)p.block_period * ((uint64_t)row[2] + 1ull);
    uint64_t* wb = wbs + threadIdx.x * HDR_WORDS;
    const uint32_t hl = header_raw(wb, prev, p.addresses + 20u * prop, p.seed, p.first_instance + il, x, prop, var, time);
    uint8_t* o = out + t * slot;
    const uint8_t* hb = (const uint8_t*)wb;
    uint64_t k = 0;
    for (uint32_t i = 0; i + 1 < hl; ++i) o[k++] = hb[i];        // all but the trailing `votes: None`
    const uint8_t* has = vhas + ((uint64_t)il * H + (x - 1)) * p.n;
    uint32_t nv = 0;
    for (uint32_t v = 0; v < p.n; ++v) nv += has[v];
    if (nv < 16u) o[k++] = (uint8_t)(0x90u | nv);
    else { o[k++] = 0xdc; o[k++] = (uint8_t)(nv >> 8); o[k++] = (uint8_t)nv; }
    for (uint32_t v = 0; v < p.n; ++v) {
        if (!has[v]) continue;
        const uint8_t* sg = vsig + (((uint64_t)il * H + (x - 1)) * p.n + v) * 65;
        o[k++] = 0xdc; o[k++] = 0x00; o[k++] = 65;
        for (int i = 0; i < 65; ++i) {
            if (sg[i] >= 128u) o[k++] = 0xcc;
            o[k++] = sg[i];
        }
    }
    lens[t] = (uint32_t)k;
}

}  // namespace bft

#include "bft_host.h"
using bft::host_keccak;
using bft::host_genesis_hash;

// Attribution pass of scripts/gpu_profile.sh only (BFTSIM_TESTING=1 + BFTSIM_PMC_EVICT=1, never the product path):
// rocprofv3 charges a kernel's dirty L2 lines to whichever later dispatch evicts them, so back-to-back kernels
// borrow each other's write-backs (a resume kernel with no hand-overs charged 30.8 MB). After
// every kernel of a launch this kernel reads 64 MiB (twice the eight XCDs' L2), evicting what the kernel left
// dirty; scripts/pmc_summary.py adds its WRITE_SIZE to the kernel before it.
// a launch's zeroed state in one dispatch (instead of one memset each): the record rows (16 B each), the
// histogram, the FAST kernel's hand-over flags and queue head (null when not a FAST launch)
__global__ __launch_bounds__(256) void bft_clear_kernel(uint4* rec, uint64_t n_rec, uint64_t* hist, uint32_t* resume,
                                                        uint32_t n_resume, uint32_t* resume_q) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x, stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = t; i < n_rec; i += stride) rec[i] = make_uint4(0u, 0u, 0u, 0u);
    if (resume)
        for (uint64_t i = t; i < n_resume; i += stride) resume[i] = 0u;
    if (t < bft::HIST_BINS) hist[t] = 0ull;
    if (resume_q && t < 2u) resume_q[t] = 0u;
}
__global__ __launch_bounds__(256) void bft_l2_evict_kernel(const uint4* buf, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256ull) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) *sink = acc;              // keeps the loads; the buffer is zero, so never taken
}

struct bftsim {
    bftsim_config cfg;
    std::vector<uint8_t> addresses;
    int device = 0;
    std::string err;
    uint8_t genesis_hash[32];
    uint32_t genesis_seed = 0;
    uint32_t seg = 64;
    uint32_t hcap = 0;
    // device buffers
    uint64_t cap_inst = 0;
    uint8_t* d_addr = nullptr;
    uint8_t* d_ghash = nullptr;
    uint32_t* d_ch = nullptr;
    uint32_t* d_flags = nullptr;
    uint32_t* d_ticks = nullptr;
    uint64_t* d_views = nullptr;
    uint32_t* d_rec = nullptr;
    uint8_t* d_hash = nullptr;
    unsigned long long* d_stats = nullptr;
    uint64_t* d_hist = nullptr;       // [HIST_BINS] of the last launch
    uint64_t* d_red = nullptr;        // bftsim_stats image reduced by bftsim_stats_allreduce
    uint4* d_evict = nullptr;         // attribution pass only (bft_l2_evict_kernel): 64 MiB of zeros
    bool pmc_evict = false;
    ncclComm_t comm = nullptr;        // bftsim_comm_init: one rank of a multi-GPU run (RCCL over xGMI)
    // real-crypto mode (bftsim_set_crypto, SPEC.md §11)
    bool crypto = false;
    uint64_t forged[4] = {0, 0, 0, 0};
    uint32_t mlog_cap = 0;
    uint32_t* d_mlog = nullptr;       // [cap_inst][mlog_cap][MLOG_WORDS]
    uint32_t* d_mlog_n = nullptr;     // [cap_inst]
    uint8_t* d_keys = nullptr;        // [2N][32]: the validators' secrets, then their forged keys
    uint32_t* d_vsnap = nullptr;      // [cap_inst][seg][8] commit set at each lane's last commit
    uint32_t* d_votes = nullptr;      // [cap_inst][rows][8] canonical committer's commit set per height
    uint8_t* d_vsig = nullptr;        // [last_n][H][N][65] the votes' signatures (bftsim_crypto_verify)
    uint8_t* d_vhas = nullptr;        // [last_n][H][N]
    uint64_t vsig_n = 0;              // instances d_vsig holds (0: no verify since the last launch)
    void* sig = nullptr;              // libbftsig handle (bftsig_t*)
    uint8_t* d_tips = nullptr;        // [cap_inst * 32]
    uint32_t* d_rcs = nullptr;        // RoundChangeSet tables, rcs_words(seg) per wave / workgroup
    uint32_t* d_backlog = nullptr;    // replay mode: backlog slots, backlog_words(seg) per wave / workgroup
    uint64_t backlog_bytes = 0;
    uint32_t* d_resume = nullptr;     // FAST launches: [cap_inst] hand-over flags
    uint32_t* d_resume_q = nullptr;   // FAST launches: [2 + cap_inst] the resume kernel's queue
    uint32_t* d_save = nullptr;       // FAST launches: [SAVE_WORDS][cap_inst * 64] saved lane state
    int fast = 1;                     // FAST kernel + resume for N = 64 (bftsim_set_fast(h, 0): full kernel)
    uint32_t window = 0;              // 0: full per-height rows; else ring of `window` rows
    uint32_t rcs_k = bft::RCS_DEFAULT_K;   // RoundChangeSet rounds per validator (bftsim_set_rcs_capacity)
    uint64_t* d_trace = nullptr;
    uint64_t* h_trace = nullptr;
    uint32_t trace_ticks = 0;
    uint64_t n_req = 0;               // instances of the next launch (bftsim_prepare); <= cap_inst
    uint64_t last_n = 0, last_first = 0;
    hipStream_t last_stream = nullptr;
    // Pipelined launches (bftsim_set_pipeline(h, D), the batch-throughput mode): a ring of D row-table sets,
    // each with the scratch of one launch, so that up to D launches are in flight at once.
    //   * the consensus kernel (+ resume + suffix rows) of each launch runs on one of `n_cs` launch streams
    //     (round-robin), after the caller's earlier work on its stream and after its set's last chain;
    //   * the prev_hash chains of `hash_batch` consecutive launches run as ONE chain kernel on one of `n_hs`
    //     hash streams (round-robin). A chain is sequential in height and a launch's chains take ~1.5 ms
    //     whatever their number, so batching B launches per kernel gives B times the chain throughput
    //     (profiles/r04). Results are complete once bftsim_sync (or any fetch) returns; those flush a
    //     partial batch first.
    static constexpr uint32_t MAX_SETS = 32, MAX_CS = 8, MAX_HS = 8, MAX_BATCH = bft::CHAIN_MAX_SETS;
    struct RowSet {
        uint32_t* ch = nullptr; uint32_t* flags = nullptr; uint32_t* ticks = nullptr; uint64_t* views = nullptr;
        uint32_t* rec = nullptr; uint8_t* hash = nullptr;
        uint32_t* sfx = nullptr;      // header suffix rows of the hash pass (sfx_rows per instance)
        uint32_t* spec = nullptr;     // little-endian seeds, N = 64: predicted blocks [H + 1][n] (seed chain)
        // big-endian seeds, N = 64: predicted chains: Byzantine masks [n], first height whose
        // recorded block differs from its prediction [n]
        uint64_t* byz = nullptr; uint32_t* bad = nullptr;
        uint32_t* pred = nullptr;     // [n][H] the predicted block of each height (bft_spec_suffix_kernel)
        // a launch's own scratch (set 0: the handle's buffers)
        uint64_t* hist = nullptr; uint32_t* rcs = nullptr; uint32_t* backlog = nullptr;
        uint32_t* resume = nullptr; uint32_t* save = nullptr; uint32_t* resume_q = nullptr;
        uint32_t* hint = nullptr;     // host-mapped: the hand-over count of the set's last launch (resume grid)
        hipEvent_t done = nullptr;    // hash pass of the last launch that used the set
        hipEvent_t batch_done = nullptr;   // or: the event of the chain batch that hashed it (flush_batch)
        hipEvent_t entry = nullptr;   // the caller's stream at the launch call
        bool busy = false;
    } sets[MAX_SETS];
    // block-hash chains: one wave per instance (bft_hash_chain_wave_kernel) up to this many instances per
    // launch, lane pairs above. 0: lane pairs at every size -- the wave chain measured slower at every
    // shard size (ds_bpermute latency and LDS issue at low occupancy), kept as an A/B arm
    // (BFTSIM_TESTING + BFTSIM_CHAIN_WAVE_MAX)
    uint64_t chain_wave_max = 0;
    // one lane per instance from this many instances per launch (kern_fast.hip bft_hash_chain_lane_kernel: fewer
    // instructions per header, longer chains; BFTSIM_TESTING + BFTSIM_CHAIN_LANE_MIN overrides)
    // predicted lanes against predicted lane pairs (r06/ab_mid, ab_lane_min): 8,192 1.69e9-1.70e9 vs 1.47e9-1.49e9;
    // 6,144 1.52e9-1.59e9 vs 1.45e9-1.46e9; 5,120 1.36e9 vs 1.41e9; 4,096 1.31e9 vs 1.41e9
    uint64_t chain_lane_min = 6144;
    // persistent lane-chain waves per dispatch, 0: a wave per 64 instances (BFTSIM_TESTING + BFTSIM_CHAIN_GRID; an A/B
    // arm: capping the chain waves so that the consensus kernels keep SIMD slots measured the same or slower)
    uint32_t chain_grid = 0;
    // lane chains encode each height's suffix themselves from the recorded rows: no suffix-row kernel on the launch
    // streams (0.3-0.45 ms per cfg3 launch beside the FAST kernels), no 400 MB of rows written and read back
    // (BFTSIM_TESTING + BFTSIM_CHAIN_INLINE=0: the suffix rows)
    uint32_t chain_inline = 1;
    uint32_t chain_prio = 0;          // s_setprio of the chain waves (BFTSIM_TESTING + BFTSIM_CHAIN_PRIO)
    // predicted chains (small shards, their latency the step's tail): above the FAST kernels' 2, with their suffix
    // rows (2,048 per GPU: 1.08e9 at 0, 1.13e9-1.22e9 at 3; profiles/r06/ab_prio; BFTSIM_CHAIN_PRIO_SPEC)
    uint32_t chain_prio_spec = 3;
    // predicted LANE chains (large shards: throughput, not latency) below the FAST kernels: 2.06e9-2.10e9 at 0 or 1
    // against 1.80e9-1.93e9 at 3 (cfg3; profiles/r06/ab_spec_lane; BFTSIM_CHAIN_PRIO_SPEC_LANE)
    uint32_t chain_prio_spec_lane = 0;
    uint32_t chain_prio_spec_early = 3;   // A/B: BFTSIM_CHAIN_PRIO_SPEC_EARLY
    uint32_t fast_lds_pad = 0;        // extra LDS per FAST wave: fewer resident FAST waves (BFTSIM_TESTING + BFTSIM_FAST_LDS_PAD)
    bool seed_spec = true;            // little-endian seeds, N = 64: predicted blocks (BFTSIM_TESTING + BFTSIM_SEED_SPEC=0: off)
    int pipeline = 0;                 // number of row-table sets (0: no pipelining)
    uint32_t sfx_rows = 0;            // heights per hash-pass chunk (0: no hash pass)
    uint32_t n_sets = 0, cur_set = 0;
    bool last_pipe = false;           // the last launch ran on the launch streams
    hipStream_t cs[MAX_CS] = {}, hstr[MAX_HS] = {};
    uint32_t n_cs = 2, n_hs = 2, cur_cs = 0, cur_hs = 0;
    // launch streams with little-endian seeds: a launch's seed chain and FAST kernel are serial on its stream
    // and there is no hash pass, so more launches run side by side (profiles/r04/ab_le_streams)
    uint32_t n_cs_seeded = 4;
    uint32_t hash_batch = 4;          // launches per chain kernel (BFTSIM_TESTING + BFTSIM_HASH_BATCH overrides)
    // big-endian seeds, N = 64, pipelined: the chains of a batch run on predicted blocks from launch time on
    // (BFTSIM_TESTING + BFTSIM_HASH_SPEC=0: off), over up to n_hs_spec hash streams so that the
    // batches of a burst of launches run side by side
    // on at every size: a small shard's chains (lane pairs) are bound by their latency, which they start ahead
    // of; a large shard's (lanes, each predicting and encoding its blocks itself) fill the issue slots the consensus
    // kernels leave from the first launch on (cfg3: 2.06e9-2.10e9 against 1.94e9-1.98e9 recorded;
    // profiles/r06/ab_spec_lane). BFTSIM_TESTING + BFTSIM_HASH_SPEC=0: recorded chains at every size; =2: predicted
    // for lossy schedules too
    uint64_t hash_spec_max = ~0ull;
    bool spec_lossy = false;          // predicted chains with drops or crashes too (BFTSIM_HASH_SPEC=2)
    uint32_t n_hs_spec = 3;
    struct Pending { uint32_t set, ev, first, cs; } pend[MAX_BATCH];   // cs: the launch stream it ran on
    // one event per chain batch (flush_batch) instead of one per set: a ring, re-recorded after BATCH_EVS batches (a set
    // still pointing at a re-recorded event waits for a later batch: later, never wrong)
    static constexpr uint32_t BATCH_EVS = 64;
    hipEvent_t batch_ev[BATCH_EVS] = {};
    uint32_t batch_ev_head = 0;
    uint32_t n_pend = 0;
    bft::Params batch_p{};            // the launch parameters of the pending batch (sizes, genesis, prio)
    bool batch_spec = false;          // the pending batch runs predicted chains
    uint32_t batch_hs = 0;            // the pending batch's hash stream (chosen at its first launch)
    // predicted suffix rows per launch at the launch, on the batch's hash stream (0: the whole batch's at the flush;
    // BFTSIM_TESTING + BFTSIM_SPEC_EARLY)
    uint32_t spec_early = 0;
    uint32_t rec_clear = 0;           // zero the record rows of FAST launches too (BFTSIM_TESTING + BFTSIM_REC_CLEAR)
    uint32_t diag_no_chain = 0;       // diagnostic: flush_batch enqueues no chain kernels (wrong hashes)
    uint32_t diag_no_clear = 0;       // diagnostic: no bft_clear_kernel (wrong statistics, hand-overs)
    uint32_t fast_prio = 0;           // FAST kernel priority + 1 (0: the kernel's default; BFTSIM_FAST_PRIO)
    uint32_t first_batch = 0;         // launches in the first chain batch after a sync (0: hash_batch; BFTSIM_FIRST_BATCH)
    uint32_t conv_stream = 0;         // a converted final batch on a hash stream of its own (A/B: BFTSIM_CONV_STREAM;
                                      // 1.70e9-1.74e9 against 1.82e9-1.85e9 on the batch's, profiles/r06/ab_conv_stream)
    uint32_t chain_on_launch = 0;     // the chain batches on the last launch's stream (BFTSIM_CHAIN_ON_LAUNCH)
    uint32_t spec_final = 1;
    uint32_t spec_first = 0;          // the first batch after a sync as predicted pair chains too (BFTSIM_SPEC_FIRST)
    bool synced = true, batch_after_sync = false;          // the flush of bftsim_sync as predicted pair chains (BFTSIM_TESTING + BFTSIM_SPEC_FINAL)   // measured: 0.99e9-1.07e9 early vs 1.09e9-1.13e9 at the flush (profiles/r06/ab_spec_early)
    // per-launch kernel timing: a ring of event quadruples, read by bftsim_kernel_ms_sum
    static constexpr uint32_t RING = 64;
    struct LaunchEv { hipEvent_t c0, c1, h0, h1, sx; bool has_hash, pending; } ring[RING] = {};
    uint32_t ring_head = 0;
    double acc_c = 0, acc_h = 0;
    uint32_t acc_n = 0;
};

static int fail(bftsim* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}
#define HIPCHECK(h, x)                                                                          \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) return fail(h, BFTSIM_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// the attribution pass's eviction after a kernel (a no-op unless BFTSIM_TESTING=1 and BFTSIM_PMC_EVICT=1)
static constexpr uint64_t EVICT_BYTES = 64ull << 20;
static hipError_t pmc_evict(bftsim* h, hipStream_t s) {
    if (!h->pmc_evict) return hipSuccess;
    if (!h->d_evict) return hipErrorNotInitialized;   // allocated and zeroed by bftsim_prepare
    hipLaunchKernelGGL(bft_l2_evict_kernel, dim3(2048), dim3(256), 0, s, (const uint4*)h->d_evict, EVICT_BYTES / 16,
                       (uint32_t*)(h->d_evict + EVICT_BYTES / 16));
    return hipGetLastError();
}

static void use_set0_scratch(bftsim* h) {
    // after a pipelined launch d_hist .. d_save point at that launch's set; set 0's are the handle's own
    if (h->n_sets == 0 || !h->sets[0].hist) return;
    bftsim::RowSet& r = h->sets[0];
    h->d_hist = r.hist; h->d_rcs = r.rcs; h->d_backlog = r.backlog; h->d_resume = r.resume; h->d_save = r.save;
    h->d_resume_q = r.resume_q;
}

static int sync_all(bftsim* h);
static void free_bufs(bftsim* h) {
    // a pending chain batch must not outlive its rows: callers sync_all first; a caller that did not (destroy)
    // runs the batch and waits for it here
    if (h->n_pend) (void)sync_all(h);
    h->n_pend = 0;
    h->last_pipe = false;
    use_set0_scratch(h);
    // the per-height row tables are owned by the sets (set 0 = the unpipelined tables); d_ch .. d_hash
    // only point at the set of the last launch
    if (h->n_sets == 0) {
        (void)hipFree(h->d_ch); (void)hipFree(h->d_flags); (void)hipFree(h->d_ticks); (void)hipFree(h->d_views);
        (void)hipFree(h->d_rec); (void)hipFree(h->d_hash);
    }
    for (uint32_t k = 0; k < h->n_sets; ++k) {
        bftsim::RowSet& r = h->sets[k];
        (void)hipFree(r.ch); (void)hipFree(r.flags); (void)hipFree(r.ticks); (void)hipFree(r.views);
        (void)hipFree(r.rec); (void)hipFree(r.hash); (void)hipFree(r.sfx); (void)hipFree(r.spec);
        (void)hipFree(r.byz); (void)hipFree(r.bad); (void)hipFree(r.pred);
        if (k > 0) {                                   // set 0's scratch is the handle's own
            (void)hipFree(r.hist); (void)hipFree(r.rcs); (void)hipFree(r.backlog); (void)hipFree(r.resume);
            (void)hipFree(r.save); (void)hipFree(r.resume_q);
        }
        r.ch = r.flags = r.ticks = nullptr; r.views = nullptr; r.rec = nullptr; r.hash = nullptr; r.sfx = nullptr;
        r.spec = nullptr; r.byz = nullptr; r.bad = nullptr; r.pred = nullptr;
        r.hist = nullptr; r.rcs = r.backlog = r.resume = r.save = r.resume_q = nullptr;
    }

    (void)hipFree(h->d_trace); (void)hipFree(h->d_tips); (void)hipFree(h->d_rcs);
    h->d_rcs = nullptr;
    (void)hipFree(h->d_backlog);
    h->d_backlog = nullptr;
    (void)hipFree(h->d_mlog); (void)hipFree(h->d_mlog_n);
    h->d_mlog = nullptr; h->d_mlog_n = nullptr;
    (void)hipFree(h->d_vsnap); (void)hipFree(h->d_votes); (void)hipFree(h->d_vsig); (void)hipFree(h->d_vhas);
    h->d_vsnap = nullptr; h->d_votes = nullptr; h->d_vsig = nullptr; h->d_vhas = nullptr; h->vsig_n = 0;
    h->backlog_bytes = 0;
    (void)hipFree(h->d_resume); (void)hipFree(h->d_save); (void)hipFree(h->d_resume_q);
    h->d_resume = nullptr; h->d_save = nullptr; h->d_resume_q = nullptr;
    for (uint32_t k = 0; k < bftsim::MAX_SETS; ++k) h->sets[k].busy = false;
    h->n_sets = 0;
    h->cur_set = 0;
    h->d_ch = h->d_flags = h->d_ticks = nullptr; h->d_views = nullptr;
    h->d_rec = nullptr; h->d_hash = nullptr; h->d_trace = nullptr; h->d_tips = nullptr;
    h->cap_inst = 0;
    h->n_req = 0;
    h->last_n = 0;                    // nothing left to fetch: the buffers of the last launch are gone
    h->last_first = 0;
}

static int flush_batch(bftsim* h, bool final = false);
static int sync_all(bftsim* h) {
    HIPCHECK(h, hipSetDevice(h->device));
    if (int rc = flush_batch(h, true)) return rc;
    h->synced = true;
    HIPCHECK(h, hipStreamSynchronize(h->last_stream));
    for (uint32_t k = 0; k < bftsim::MAX_CS; ++k)
        if (h->cs[k]) HIPCHECK(h, hipStreamSynchronize(h->cs[k]));
    for (uint32_t k = 0; k < bftsim::MAX_HS; ++k)
        if (h->hstr[k]) HIPCHECK(h, hipStreamSynchronize(h->hstr[k]));
    return BFTSIM_OK;
}

#ifdef BFT_STAMPS
static uint64_t* g_stamps = nullptr;
static uint64_t g_stamp_waves = 0;
#endif

// ------------------------------------------------------------------------------ RCCL (multi-GPU)
// The one collective of the path: the run statistics of every rank summed over RCCL.
// librccl is opened on first use (the soname torch also loads, so one copy serves the process);
// the library itself stays loadable without it.
namespace {
struct Rccl {
    ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*err)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string why;
};
Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!lib) { r.why = std::string("dlopen librccl.so.1: ") + dlerror(); return; }
        r.get_id = (decltype(r.get_id))dlsym(lib, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(lib, "ncclCommInitRank");
        r.all_reduce = (decltype(r.all_reduce))dlsym(lib, "ncclAllReduce");
        r.destroy = (decltype(r.destroy))dlsym(lib, "ncclCommDestroy");
        r.err = (decltype(r.err))dlsym(lib, "ncclGetErrorString");
        r.ok = r.get_id && r.init_rank && r.all_reduce && r.destroy && r.err;
        if (!r.ok) r.why = "librccl.so.1 lacks an entry point";
    });
    return r;
}
// RCCL prints its version banner on stdout at initialisation; the callers' stdout carries results
// (bench.py's one JSON line), so the banner goes to stderr
struct StdoutToStderr {
    int saved;
    StdoutToStderr() {
        fflush(stdout);
        saved = dup(1);
        if (saved >= 0) dup2(2, 1);
    }
    ~StdoutToStderr() {
        fflush(stdout);
        if (saved >= 0) { dup2(saved, 1); close(saved); }
    }
};
void comm_destroy(ncclComm_t c) {
    if (rccl().ok) (void)rccl().destroy(c);
}

// libbftsig (include/bftsig.h), next to this library: the batched secp256k1 of real-crypto mode
struct SigApi {
    int (*create)(int, void**) = nullptr;
    void (*destroy)(void*) = nullptr;
    const char* (*last_error)(const void*) = nullptr;
    int (*secret_to_address)(void*, const uint8_t*, uint64_t, uint8_t*, uint8_t*, uint8_t*, void*) = nullptr;
    int (*sign)(void*, const uint8_t*, const uint32_t*, const uint8_t*, uint64_t, uint8_t*, uint8_t*, void*) = nullptr;
    int (*recover)(void*, const uint8_t*, const uint8_t*, uint64_t, uint8_t*, uint8_t*, uint8_t*, void*) = nullptr;
    bool ok = false;
    std::string why;
};
void sig_api_anchor() {}
SigApi& sig_api() {
    static SigApi a;
    static std::once_flag once;
    std::call_once(once, [] {
        Dl_info di;
        std::string path = "libbftsig.so";
        if (dladdr((void*)&sig_api_anchor, &di) && di.dli_fname) {
            std::string self = di.dli_fname;
            size_t k = self.rfind('/');
            if (k != std::string::npos) path = self.substr(0, k + 1) + "libbftsig.so";
        }
        void* lib = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
        if (!lib) { a.why = std::string("dlopen ") + path + ": " + dlerror(); return; }
        a.create = (decltype(a.create))dlsym(lib, "bftsig_create");
        a.destroy = (decltype(a.destroy))dlsym(lib, "bftsig_destroy");
        a.last_error = (decltype(a.last_error))dlsym(lib, "bftsig_last_error");
        a.secret_to_address = (decltype(a.secret_to_address))dlsym(lib, "bftsig_secret_to_address");
        a.sign = (decltype(a.sign))dlsym(lib, "bftsig_sign");
        a.recover = (decltype(a.recover))dlsym(lib, "bftsig_recover");
        a.ok = a.create && a.destroy && a.last_error && a.secret_to_address && a.sign && a.recover;
        if (!a.ok) a.why = path + " lacks an entry point";
    });
    return a;
}
}  // namespace

extern "C" {

#ifdef BFT_STAMPS
// diagnostic builds only: per-section cycle sums of the last launch, summed over waves, into out[0 .. cap);
// returns the number of sections the build stamps (bft::NSTAMP), so a caller sizes its buffer from the library
// (out = nullptr, cap = 0: the count alone) instead of a copy of the constant
int bftsim_debug_stamps(uint64_t* out, uint32_t cap) {
    if (!out || cap == 0) return bft::NSTAMP;
    std::vector<uint64_t> v(g_stamp_waves * bft::NSTAMP);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpy(v.data(), g_stamps, v.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    const uint32_t m = cap < (uint32_t)bft::NSTAMP ? cap : (uint32_t)bft::NSTAMP;
    for (uint32_t k = 0; k < m; ++k) out[k] = 0;
    for (uint64_t w = 0; w < g_stamp_waves; ++w)
        for (uint32_t k = 0; k < m; ++k) out[k] += v[w * bft::NSTAMP + k];
    return bft::NSTAMP;
}
#endif

uint32_t bftsim_two_thirds_majority(uint32_t n) { return (2u * n) / 3u; }
uint32_t bftsim_seed_from_hash(const uint8_t hash[32], uint32_t n) { return n ? bft::seed_from_hash(hash, n) : 0; }
uint32_t bftsim_seed_from_hash_order(const uint8_t hash[32], uint32_t n, uint32_t order) {
    return n ? bft::seed_from_hash(hash, n, order == BFTSIM_SEED_LE) : 0;
}
uint32_t bftsim_calc_proposer(const uint8_t prev_hash[32], uint32_t n, uint64_t round) {
    if (n == 0) return 0;
    return (uint32_t)(((uint64_t)bft::seed_from_hash(prev_hash, n) + round % n) % n);
}
void bftsim_keccak256(const uint8_t* data, size_t len, uint8_t out[32]) { host_keccak(data, len, out); }
void bftsim_genesis_hash(const bftsim_config* cfg, uint8_t out[32]) { host_genesis_hash(cfg, out); }
int bftsim_check_message(uint32_t code, uint64_t msg_height, uint64_t core_height, uint32_t state) {
    if (code < 1 || code > 4 || state < 1 || state > 4 || msg_height >= (1ull << 32) || core_height >= (1ull << 32))
        return BFTSIM_EINVAL;
    return bft::check_message_class((int)code, (uint32_t)msg_height, (uint32_t)core_height, state);
}
int bftsim_view_cmp(uint64_t h1, uint64_t r1, uint64_t h2, uint64_t r2) {
    if (h1 != h2) return h1 < h2 ? -1 : 1;
    if (r1 != r2) return r1 < r2 ? -1 : 1;
    return 0;
}

const char* bftsim_last_error(bftsim_t* h) { return h ? h->err.c_str() : "null handle"; }

int bftsim_create(const bftsim_config* cfg, int hip_device, bftsim_t** out) {
    if (!cfg || !out) return BFTSIM_EINVAL;
    *out = nullptr;
    if (cfg->n < 1 || cfg->n > 256) return BFTSIM_EUNSUPPORTED;
    if (cfg->heights < 1 || cfg->heights > (1u << 20) || cfg->max_ticks < 1 || cfg->max_ticks > (1u << 28) ||
        !cfg->addresses || cfg->phase_cap < 1 || cfg->phase_cap > 255 || cfg->block_period < 1)
        return BFTSIM_EINVAL;
    for (uint32_t i = 1; i < cfg->n; ++i)
        if (memcmp(cfg->addresses + 20 * (i - 1), cfg->addresses + 20 * i, 20) >= 0) return BFTSIM_EINVAL;
    if (cfg->seed_byte_order > BFTSIM_SEED_LE || cfg->header_encoding != BFTSIM_ENC_RMP_COMPACT ||
        cfg->backlog_mode > BFTSIM_BACKLOG_REPLAY || cfg->reserved != 0)
        return BFTSIM_EINVAL;
    bftsim* h = new bftsim();
    h->cfg = *cfg;
    h->addresses.assign(cfg->addresses, cfg->addresses + 20 * cfg->n);
    h->cfg.addresses = h->addresses.data();
    h->device = hip_device;
    host_genesis_hash(&h->cfg, h->genesis_hash);
    h->genesis_seed = bft::seed_from_hash(h->genesis_hash, cfg->n, cfg->seed_byte_order == BFTSIM_SEED_LE);
    h->seg = bft::segment_size(cfg->n);
    h->hcap = cfg->heights + 64;
    *out = h;
    hipError_t e = hipSetDevice(hip_device);
    if (e != hipSuccess) return fail(h, BFTSIM_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    HIPCHECK(h, hipMalloc(&h->d_addr, 20 * cfg->n));
    HIPCHECK(h, hipMemcpy(h->d_addr, h->addresses.data(), 20 * cfg->n, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMalloc(&h->d_ghash, 32));
    HIPCHECK(h, hipMemcpy(h->d_ghash, h->genesis_hash, 32, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMalloc(&h->d_stats, 16 * sizeof(unsigned long long)));
    HIPCHECK(h, hipMalloc(&h->d_hist, bft::HIST_BINS * sizeof(uint64_t)));
    for (uint32_t i = 0; i < bftsim::RING; ++i) {
        HIPCHECK(h, hipEventCreate(&h->ring[i].c0)); HIPCHECK(h, hipEventCreate(&h->ring[i].c1));
        HIPCHECK(h, hipEventCreate(&h->ring[i].h0)); HIPCHECK(h, hipEventCreate(&h->ring[i].h1));
        HIPCHECK(h, hipEventCreateWithFlags(&h->ring[i].sx, hipEventDisableTiming));
    }
    for (uint32_t i = 0; i < bftsim::MAX_SETS; ++i)
        HIPCHECK(h, hipEventCreateWithFlags(&h->sets[i].done, hipEventDisableTiming));
    return BFTSIM_OK;
}

void bftsim_destroy(bftsim_t* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    free_bufs(h);
    (void)hipFree(h->d_addr); (void)hipFree(h->d_ghash); (void)hipFree(h->d_stats); (void)hipFree(h->d_hist);
    (void)hipFree(h->d_red);
    (void)hipFree(h->d_evict);
    (void)hipFree(h->d_keys);
    if (h->comm) comm_destroy(h->comm);
    if (h->sig) sig_api().destroy(h->sig);
    for (uint32_t i = 0; i < bftsim::RING; ++i) {
        if (h->ring[i].c0) (void)hipEventDestroy(h->ring[i].c0);
        if (h->ring[i].c1) (void)hipEventDestroy(h->ring[i].c1);
        if (h->ring[i].h0) (void)hipEventDestroy(h->ring[i].h0);
        if (h->ring[i].h1) (void)hipEventDestroy(h->ring[i].h1);
        if (h->ring[i].sx) (void)hipEventDestroy(h->ring[i].sx);
    }
    for (uint32_t i = 0; i < bftsim::MAX_SETS; ++i) {
        if (h->sets[i].done) (void)hipEventDestroy(h->sets[i].done);
        h->sets[i].batch_done = nullptr;
        if (h->sets[i].entry) (void)hipEventDestroy(h->sets[i].entry);
        if (h->sets[i].hint) (void)hipHostFree(h->sets[i].hint);
    }
    for (uint32_t i = 0; i < bftsim::BATCH_EVS; ++i)
        if (h->batch_ev[i]) (void)hipEventDestroy(h->batch_ev[i]);
    for (uint32_t i = 0; i < bftsim::MAX_CS; ++i)
        if (h->cs[i]) (void)hipStreamDestroy(h->cs[i]);
    for (uint32_t i = 0; i < bftsim::MAX_HS; ++i)
        if (h->hstr[i]) (void)hipStreamDestroy(h->hstr[i]);
    delete h;
}

static bft::Params make_params(bftsim* h, uint64_t first, uint64_t n);

int bftsim_prepare(bftsim_t* h, uint64_t n) {
    if (!h || n == 0 || n > (1ull << 31)) return fail(h, BFTSIM_EINVAL, "bad instance count");
    HIPCHECK(h, hipSetDevice(h->device));
    if (n <= h->cap_inst) { h->n_req = n; return BFTSIM_OK; }
    if (h->last_n) if (int rc = sync_all(h)) return rc;   // the last launch may still use them
    free_bufs(h);
    HIPCHECK(h, hipMalloc(&h->d_ch, n * 4));
    HIPCHECK(h, hipMalloc(&h->d_flags, n * 4));
    HIPCHECK(h, hipMalloc(&h->d_ticks, n * 4));
    HIPCHECK(h, hipMalloc(&h->d_views, n * 8));
    HIPCHECK(h, hipMalloc(&h->d_rec, n * h->hcap * 16));
    HIPCHECK(h, hipMalloc(&h->d_hash, n * h->hcap * 32));
    HIPCHECK(h, hipMalloc(&h->d_tips, n * 32));
    {
        uint64_t per_block = h->seg > 64 ? 1 : 64 / h->seg;
        uint64_t blocks = (n + per_block - 1) / per_block;
        HIPCHECK(h, hipMalloc(&h->d_rcs, blocks * bft::rcs_words(h->seg, h->rcs_k) * 4));
        if (h->crypto) {
            HIPCHECK(h, hipMalloc(&h->d_mlog, n * (uint64_t)h->mlog_cap * bft::MLOG_WORDS * 4));
            HIPCHECK(h, hipMalloc(&h->d_mlog_n, n * 4));
            HIPCHECK(h, hipMalloc(&h->d_vsnap, n * (uint64_t)h->seg * 8 * 4));
            HIPCHECK(h, hipMalloc(&h->d_votes, n * (uint64_t)h->hcap * 8 * 4));
        }
        if (h->cfg.backlog_mode == BFTSIM_BACKLOG_REPLAY) {
            h->backlog_bytes = blocks * bft::backlog_words(h->seg) * 4;
            HIPCHECK(h, hipMalloc(&h->d_backlog, h->backlog_bytes));
        }
    }
    if (h->seg == 64 && h->cfg.n == 64) {          // FAST kernel hand-over buffers
        HIPCHECK(h, hipMalloc(&h->d_resume, n * 4));
        HIPCHECK(h, hipMalloc(&h->d_resume_q, (n + 2) * 4));
        HIPCHECK(h, hipMalloc(&h->d_save, (uint64_t)bft::SAVE_WORDS * n * 64 * 4));
    }
    h->sets[0].ch = h->d_ch; h->sets[0].flags = h->d_flags; h->sets[0].ticks = h->d_ticks;
    h->sets[0].views = h->d_views; h->sets[0].rec = h->d_rec; h->sets[0].hash = h->d_hash;
    h->sets[0].hist = h->d_hist; h->sets[0].rcs = h->d_rcs; h->sets[0].backlog = h->d_backlog;
    h->sets[0].resume = h->d_resume; h->sets[0].save = h->d_save; h->sets[0].resume_q = h->d_resume_q;
    h->n_sets = 1;
    {
        const char* tst = getenv("BFTSIM_TESTING");
        const bool testing = tst && strcmp(tst, "1") == 0;
        const char* cw = getenv("BFTSIM_CHAIN_WAVE_MAX");
        if (testing && cw) h->chain_wave_max = strtoull(cw, nullptr, 10);
        const char* cl = getenv("BFTSIM_CHAIN_LANE_MIN");
        if (testing && cl) h->chain_lane_min = strtoull(cl, nullptr, 10);
        const char* cp = getenv("BFTSIM_CHAIN_PRIO");
        if (testing && cp) h->chain_prio = (uint32_t)atoi(cp);
        const char* lp = getenv("BFTSIM_FAST_LDS_PAD");
        if (testing && lp) h->fast_lds_pad = (uint32_t)atoi(lp) > 60000u ? 60000u : (uint32_t)atoi(lp);
        auto knob = [&](const char* name, uint32_t& v, uint32_t lo, uint32_t hi) {
            const char* e = getenv(name);
            if (testing && e) { const uint32_t x = (uint32_t)atoi(e); v = x < lo ? lo : x > hi ? hi : x; }
        };
        knob("BFTSIM_LAUNCH_STREAMS", h->n_cs, 1, bftsim::MAX_CS);
        knob("BFTSIM_CHAIN_GRID", h->chain_grid, 0, 1u << 20);
        knob("BFTSIM_CHAIN_PRIO_SPEC", h->chain_prio_spec, 0, 3);
        knob("BFTSIM_CHAIN_PRIO_SPEC_LANE", h->chain_prio_spec_lane, 0, 3);
        knob("BFTSIM_CHAIN_PRIO_SPEC_EARLY", h->chain_prio_spec_early, 0, 3);
        knob("BFTSIM_SPEC_EARLY", h->spec_early, 0, 1);
        knob("BFTSIM_SPEC_FINAL", h->spec_final, 0, 1);
        knob("BFTSIM_SPEC_FIRST", h->spec_first, 0, 1);
        knob("BFTSIM_REC_CLEAR", h->rec_clear, 0, 1);
        knob("BFTSIM_DIAG_NO_CHAIN", h->diag_no_chain, 0, 1);
        knob("BFTSIM_DIAG_NO_CLEAR", h->diag_no_clear, 0, 1);
        knob("BFTSIM_CONV_STREAM", h->conv_stream, 0, 1);
        knob("BFTSIM_FIRST_BATCH", h->first_batch, 0, bftsim::MAX_BATCH);
        knob("BFTSIM_FAST_PRIO", h->fast_prio, 0, 4);
        knob("BFTSIM_CHAIN_ON_LAUNCH", h->chain_on_launch, 0, 1);
        knob("BFTSIM_CHAIN_INLINE", h->chain_inline, 0, 1);
        knob("BFTSIM_LAUNCH_STREAMS_SEEDED", h->n_cs_seeded, 1, bftsim::MAX_CS);
        knob("BFTSIM_HASH_STREAMS", h->n_hs, 1, bftsim::MAX_HS);   // A/B arms
        knob("BFTSIM_HASH_BATCH", h->hash_batch, 1, bftsim::MAX_BATCH);   // A/B arms (bftsim_set_hash_batch)
        knob("BFTSIM_HASH_STREAMS_SPEC", h->n_hs_spec, 1, bftsim::MAX_HS);
        const char* ss = getenv("BFTSIM_SEED_SPEC");
        if (testing && ss) h->seed_spec = atoi(ss) != 0;
        const char* hs = getenv("BFTSIM_HASH_SPEC");   // 0: off, 1: at every size
        if (testing && hs) h->hash_spec_max = atoi(hs) != 0 ? ~0ull : 0ull;
        h->spec_lossy = testing && hs && atoi(hs) == 2;   // 2: lossy schedules too (the tests of the repairs)
        const char* pe = getenv("BFTSIM_PMC_EVICT");
        h->pmc_evict = testing && pe && atoi(pe) != 0;   // scripts/gpu_profile.sh's attribution pass
        if (h->pmc_evict && !h->d_evict) {          // before any launch, so every eviction is the same dispatch
            HIPCHECK(h, hipMalloc(&h->d_evict, EVICT_BYTES + 16));
            HIPCHECK(h, hipMemset(h->d_evict, 0, EVICT_BYTES + 16));
        }
    }
    const uint64_t per_block = h->seg > 64 ? 1 : 64 / h->seg, blocks = (n + per_block - 1) / per_block;
    for (uint32_t k = 1; k < (uint32_t)h->pipeline; ++k) {
        bftsim::RowSet& r = h->sets[k];
        HIPCHECK(h, hipMalloc(&r.ch, n * 4));
        HIPCHECK(h, hipMalloc(&r.flags, n * 4));
        HIPCHECK(h, hipMalloc(&r.ticks, n * 4));
        HIPCHECK(h, hipMalloc(&r.views, n * 8));
        HIPCHECK(h, hipMalloc(&r.rec, n * h->hcap * 16));
        HIPCHECK(h, hipMalloc(&r.hash, n * h->hcap * 32));
        h->n_sets = k + 1;
        {
            HIPCHECK(h, hipMalloc(&r.hist, bft::HIST_BINS * sizeof(uint64_t)));
            HIPCHECK(h, hipMalloc(&r.rcs, blocks * bft::rcs_words(h->seg, h->rcs_k) * 4));
            if (h->d_backlog) HIPCHECK(h, hipMalloc(&r.backlog, h->backlog_bytes));
            if (h->d_resume) {
                HIPCHECK(h, hipMalloc(&r.resume, n * 4));
                HIPCHECK(h, hipMalloc(&r.resume_q, (n + 2) * 4));
                HIPCHECK(h, hipMalloc(&r.save, (uint64_t)bft::SAVE_WORDS * n * 64 * 4));
            }
        }
    }
    // the hash pass's suffix rows (runs without in-kernel hashes): every height in one chunk up to 2 GiB
    // per set, fewer heights per chunk beyond
    h->sfx_rows = 0;
    if (!make_params(h, 0, 1).need_seed) {
        const uint64_t per_row = n * bft::SFX_DEV_DW * 4ull;
        uint64_t rows = (2ull << 30) / per_row;
        if (rows < 1) rows = 1;
        if (rows > h->cfg.heights) rows = h->cfg.heights;
        // tests only (BFTSIM_TESTING=1): fewer heights per chunk, so that small batches take the chunked path
        const char* tst = getenv("BFTSIM_TESTING");
        const char* cap = getenv("BFTSIM_SFX_ROWS");
        if (tst && cap && strcmp(tst, "1") == 0 && atoi(cap) > 0 && (uint64_t)atoi(cap) < rows) rows = (uint64_t)atoi(cap);
        if (rows * n >= (1ull << 32)) rows = ((1ull << 32) - 1) / n;
        h->sfx_rows = (uint32_t)rows;
        for (uint32_t k = 0; k < h->n_sets; ++k) HIPCHECK(h, hipMalloc(&h->sets[k].sfx, rows * per_row));
        if (h->seg == 64 && h->cfg.n == 64 && h->n_sets >= 2 && rows >= h->cfg.heights)
            for (uint32_t k = 0; k < h->n_sets; ++k) {   // predicted chains of pipelined FAST launches
                HIPCHECK(h, hipMalloc(&h->sets[k].byz, n * 8));
                HIPCHECK(h, hipMalloc(&h->sets[k].bad, n * 4));
                HIPCHECK(h, hipMalloc(&h->sets[k].pred, n * h->cfg.heights * 4ull));
            }
        // every stream of the pipelined mode now, while the HIP runtime still has hardware queues of its own to
        // give each (streams created later in a busy process can share one, which serializes their batches)
        if (h->n_sets >= 2) {
            for (uint32_t k = 0; k < h->n_cs && k < bftsim::MAX_CS; ++k)
                if (!h->cs[k]) HIPCHECK(h, hipStreamCreateWithFlags(&h->cs[k], hipStreamNonBlocking));
            const uint32_t nh = h->n_hs > h->n_hs_spec ? h->n_hs : h->n_hs_spec;
            for (uint32_t k = 0; k < nh && k < bftsim::MAX_HS; ++k)
                if (!h->hstr[k]) HIPCHECK(h, hipStreamCreateWithFlags(&h->hstr[k], hipStreamNonBlocking));
        }
    } else if (h->seg == 64 && h->cfg.n == 64 && !h->window) {
        // little-endian seeds at N = 64: the seed chain's predicted blocks
        for (uint32_t k = 0; k < h->n_sets; ++k)
            HIPCHECK(h, hipMalloc(&h->sets[k].spec, (uint64_t)(h->cfg.heights + 1u) * n * 4ull));
    }
    h->cap_inst = n;
    h->n_req = n;
    return BFTSIM_OK;
}

int bftsim_set_window(bftsim_t* h, uint32_t window) {
    if (!h) return BFTSIM_EINVAL;
    if (window != 0 && (window < 64 || (window & (window - 1)) != 0 || window > (1u << 20)))
        return fail(h, BFTSIM_EINVAL, "window must be 0 or a power of two in [64, 2^20]");
    if (window == h->window) return BFTSIM_OK;
    if (h->last_stream) if (int rc = sync_all(h)) return rc;   // pending chains use the buffers freed below
    h->window = window;
    h->hcap = window ? window : h->cfg.heights + 64;
    (void)hipSetDevice(h->device);
    free_bufs(h);                                   // row tables are re-sized by the next prepare
    return BFTSIM_OK;
}

int bftsim_set_rcs_capacity(bftsim_t* h, uint32_t rounds) {
    if (!h) return BFTSIM_EINVAL;
    if (rounds < 1 || rounds > bft::RCS_MAX_K) return fail(h, BFTSIM_EINVAL, "RoundChangeSet capacity must be 1..4096");
    if (rounds == h->rcs_k) return BFTSIM_OK;
    if (h->last_stream) if (int rc = sync_all(h)) return rc;
    h->rcs_k = rounds;
    (void)hipSetDevice(h->device);
    free_bufs(h);                                   // the tables are re-sized by the next prepare
    return BFTSIM_OK;
}

int bftsim_set_fast(bftsim_t* h, int on) {
    if (!h) return BFTSIM_EINVAL;
    h->fast = on != 0;
    return BFTSIM_OK;
}

int bftsim_set_trace(bftsim_t* h, uint64_t* host_out, uint32_t trace_ticks) {
    if (!h) return BFTSIM_EINVAL;
    h->h_trace = host_out;
    h->trace_ticks = host_out ? trace_ticks : 0;
    return BFTSIM_OK;
}

static bft::Params make_params(bftsim* h, uint64_t first, uint64_t n) {
    bft::Params p = bft::params_from_config(h->cfg, h->seg, h->hcap, h->genesis_seed, first, n);
    p.addresses = h->d_addr;
    p.genesis_hash = h->d_ghash;
    p.committed_height = h->d_ch;
    p.flags = h->d_flags;
    p.ticks = h->d_ticks;
    p.views = h->d_views;
    p.rec = h->d_rec;
    p.hash = h->d_hash;
    p.trace = h->d_trace;
    p.trace_ticks = h->trace_ticks;
    p.hist = h->d_hist;
    p.rcs = h->d_rcs;
    p.rcs_k = h->rcs_k;
    p.chain_prio = h->chain_prio;
    p.fast_prio = h->fast_prio;
    p.chain_grid = h->chain_grid;
    p.chain_inline = h->chain_inline;
    p.fast_lds_pad = h->fast_lds_pad;
    p.backlog = h->d_backlog;
    if (h->crypto && h->d_mlog) {
        p.mlog = h->d_mlog;
        p.mlog_n = h->d_mlog_n;
        p.mlog_cap = h->mlog_cap;
        for (int k = 0; k < 4; ++k) p.forged[k] = h->forged[k];
        p.vsnap = h->d_vsnap;
        p.votes = h->d_votes;
        p.fast = 0;                  // one message at a time: the commit set at the commit instant (votes)
    }
    if (h->window) {
        p.window_mask = h->window - 1;
        p.rows = h->window;
        p.hcap = h->cfg.heights + 64;               // height limit; rows live in the ring
        p.need_seed = 1;                            // hashes in-kernel: no post-pass over a ring
    }
    return p;
}

// which chain kernel hashes a batch of launches of n instances (the wave kernel has no predicted / repair mode)
static uint32_t chain_kind(const bftsim* h, uint64_t n, bool spec) {
    if (n >= h->chain_lane_min && 4ull * n < (1ull << 24)) return bft::CHAIN_KERNEL_LANE;   // its 24-bit offsets
    if (!spec && n <= h->chain_wave_max) return bft::CHAIN_KERNEL_WAVE;
    return bft::CHAIN_KERNEL_PAIR;
}

static uint32_t clear_blocks(uint64_t n_rec) {   // bft_clear_kernel's grid: grid-stride, at least one block
    const uint64_t b = (n_rec + 255u) / 256u;
    return (uint32_t)(b < 1 ? 1 : b > 4096 ? 4096 : b);
}

int bftsim_launch(bftsim_t* h, uint64_t first, void* stream) {
    if (!h || h->cap_inst == 0 || h->n_req == 0) return fail(h, BFTSIM_EINVAL, "bftsim_prepare not called");
    const uint64_t n = h->n_req;
    if (first + n > (1ull << 32)) return fail(h, BFTSIM_EINVAL, "instance ids must fit in 32 bits");
    {   // the device current already (the common case): hipGetDevice is a thread-local read, hipSetDevice is not
        int d = -1;
        if (hipGetDevice(&d) != hipSuccess || d != h->device) HIPCHECK(h, hipSetDevice(h->device));
    }
    hipStream_t s = (hipStream_t)stream;
    if (h->h_trace) {
        if (h->d_trace) (void)hipFree(h->d_trace);
        h->d_trace = nullptr;
        size_t tb = n * (size_t)h->trace_ticks * h->cfg.n * 8;
        HIPCHECK(h, hipMalloc(&h->d_trace, tb));
        HIPCHECK(h, hipMemsetAsync(h->d_trace, 0, tb, s));
    }
    bft::Params p = make_params(h, first, n);
    // pipelined: on the launch streams with the set's own scratch; not with per-launch host state (traces,
    // the crypto log, which the next calls read from the last launch alone)
    // FAST + resume for N = 64: big-endian seeds (proposer 0, hashes in the post-pass) or little-endian
    // seeds (SEEDED: the seed chain's predictions, else hashes in-kernel); not for windowed rows, traces or
    // the opt-in modes
    const bool fast = h->fast && p.fast && !p.mlog && h->d_save && !h->window && !h->h_trace && h->seg == 64 &&
                      h->cfg.n == 64;
    const bool fast_launch = fast;
    const bool spec = fast && p.need_seed && h->seed_spec && h->sets[0].spec;
    const bool pipe = h->pipeline >= 2 && (!p.need_seed || spec) && h->n_sets >= 2 && !h->h_trace && !p.mlog;
    if (h->last_pipe && !pipe) {
        // a launch on the caller's stream after pipelined ones: they may still use set 0's scratch
        if (int rc = sync_all(h)) return rc;
        h->last_pipe = false;
    }
    use_set0_scratch(h);
    p = make_params(h, first, n);
#ifdef BFT_STAMPS
    {
        static uint64_t* d_st = nullptr;
        static uint64_t cap = 0;
        uint64_t per = h->seg > 64 ? 1 : 64 / h->seg;
        uint64_t waves = (n + per - 1) / per;
        if (waves > cap) { (void)hipFree(d_st); HIPCHECK(h, hipMalloc(&d_st, waves * 8 * bft::NSTAMP)); cap = waves; }
        HIPCHECK(h, hipMemsetAsync(d_st, 0, waves * 8 * bft::NSTAMP, s));
        p.stamps = d_st;
        g_stamps = d_st;
        g_stamp_waves = waves;
    }
#endif
    if (pipe) {
        // the next row-table set in the ring, once its last launch's chains are done (a launch of it still
        // waiting in the hash batch is flushed first)
        h->cur_set = (h->cur_set + 1) % h->n_sets;
        for (uint32_t i = 0; i < h->n_pend; ++i)
            if (h->pend[i].set == h->cur_set) { if (int rc = flush_batch(h)) return rc; break; }
        bftsim::RowSet& r = h->sets[h->cur_set];
        if (!r.entry) HIPCHECK(h, hipEventCreateWithFlags(&r.entry, hipEventDisableTiming));
        HIPCHECK(h, hipEventRecord(r.entry, s));
        h->cur_cs = (h->cur_cs + 1) % (spec ? h->n_cs_seeded : h->n_cs);
        if (!h->cs[h->cur_cs]) HIPCHECK(h, hipStreamCreateWithFlags(&h->cs[h->cur_cs], hipStreamNonBlocking));
        hipStream_t ls = h->cs[h->cur_cs];
        HIPCHECK(h, hipStreamWaitEvent(ls, r.entry, 0));
        if (r.busy) HIPCHECK(h, hipStreamWaitEvent(ls, r.batch_done ? r.batch_done : r.done, 0));
        s = ls;
        h->d_hist = r.hist; h->d_rcs = r.rcs; h->d_backlog = r.backlog; h->d_resume = r.resume; h->d_save = r.save;
        h->d_resume_q = r.resume_q;
        p.hist = r.hist; p.rcs = r.rcs; p.backlog = r.backlog;
        h->d_ch = r.ch; h->d_flags = r.flags; h->d_ticks = r.ticks; h->d_views = r.views;
        h->d_rec = r.rec; h->d_hash = r.hash;
        p.committed_height = h->d_ch; p.flags = h->d_flags; p.ticks = h->d_ticks; p.views = h->d_views;
        p.rec = h->d_rec; p.hash = h->d_hash;
        h->last_pipe = true;
    }
    bftsim::LaunchEv& ev = h->ring[h->ring_head % bftsim::RING];
    if (ev.pending) {                                    // 64 launches unread: fold the oldest in
        HIPCHECK(h, hipEventSynchronize(ev.has_hash ? ev.h1 : ev.c1));
        float a = 0, b = 0;
        HIPCHECK(h, hipEventElapsedTime(&a, ev.c0, ev.c1));
        if (ev.has_hash) HIPCHECK(h, hipEventElapsedTime(&b, ev.h0, ev.h1));
        h->acc_c += a; h->acc_h += b; h->acc_n += 1;
        ev.pending = false;
    }
    h->ring_head += 1;
    // the histogram and (FAST launches) the hand-over flags and queue zeroed by one dispatch; the record rows too,
    // except for FAST launches: the FAST and resume bodies read a row only once they have recorded it (canon_blk,
    // canon_seed, refresh_tip_from_table: rows <= the canonical height), and every reader after the launch stops at
    // the committed height (fetch, export, tips, chains, the predicted chains' check) -- 43 MB of writes per cfg3
    // launch saved (BFTSIM_TESTING + BFTSIM_REC_CLEAR=1: cleared anyway)
    const bool clear_rec = !fast_launch || h->rec_clear;
    const uint64_t n_rec = clear_rec ? (uint64_t)n * h->hcap : 0;
    if (!h->diag_no_clear) {   // (diagnostic BFTSIM_DIAG_NO_CLEAR=1: the host cost of this dispatch; wrong statistics)
        hipLaunchKernelGGL(bft_clear_kernel, dim3(clear_blocks(n_rec > n ? n_rec : n)), dim3(256), 0, s, (uint4*)h->d_rec,
                           n_rec, h->d_hist, fast_launch ? h->d_resume : nullptr, (uint32_t)n,
                           fast_launch ? h->d_resume_q : nullptr);
        HIPCHECK(h, hipGetLastError());
    }
    if (h->d_backlog) HIPCHECK(h, hipMemsetAsync(h->d_backlog, 0, h->backlog_bytes, s));
    uint32_t per_block = h->seg > 64 ? 1u : 64u / h->seg;      // instances per workgroup
    uint32_t grid = (uint32_t)((n + per_block - 1) / per_block);
    size_t lds = bft::lds_bytes(h->seg, p.need_seed != 0);
    const bool ext = p.backlog_replay || p.mlog;       // the opt-in modes' kernel build (MODE_EXT)
    HIPCHECK(h, hipEventRecord(ev.c0, s));
    if (fast) {
        // FAST kernel over every instance, then the full kernel over the ones it handed over
        p.resume_flags = h->d_resume;
        p.resume_q = h->d_resume_q;
        p.save = h->d_save;
        p.save_stride = n * 64;
        {
            bftsim::RowSet& r = h->sets[pipe ? h->cur_set : 0];
            if (!r.hint) {
                HIPCHECK(h, hipHostMalloc((void**)&r.hint, 4, hipHostMallocMapped | hipHostMallocCoherent));
                *r.hint = 0xffffffffu;                    // unknown: the full grid, or another set's last count
                for (uint32_t k = 0; k < h->n_sets; ++k)  // (the grid only paces the persistent waves)
                    if (h->sets[k].hint && &h->sets[k] != &r && *h->sets[k].hint != 0xffffffffu) {
                        *r.hint = __atomic_load_n(h->sets[k].hint, __ATOMIC_RELAXED);
                        break;
                    }
            }
            p.resume_hint = r.hint;
        }
        if (spec) {                                      // the predicted blocks first (little-endian seeds)
            p.spec = h->sets[pipe ? h->cur_set : 0].spec;
            HIPCHECK(h, bft::launch_seed_chain((uint32_t)n, s, p));
            HIPCHECK(h, pmc_evict(h, s));
        }
        HIPCHECK(h, bft::launch_fast(dim3(grid), s, p));
        HIPCHECK(h, pmc_evict(h, s));
        HIPCHECK(h, bft::launch_resume(dim3(grid), lds, s, p));
        HIPCHECK(h, pmc_evict(h, s));
    } else {
        HIPCHECK(h, bft::launch_general(p.need_seed != 0, ext, h->seg, dim3(grid), lds, s, p));
        HIPCHECK(h, pmc_evict(h, s));
    }
    HIPCHECK(h, hipEventRecord(ev.c1, s));
    ev.has_hash = !p.need_seed;
    ev.pending = true;
    if (!p.need_seed) {
        uint32_t* sfx = h->sets[pipe ? h->cur_set : 0].sfx;
        const uint32_t H = h->cfg.heights, K = h->sfx_rows;
        // Where the suffix rows go depends on how long the consensus kernel runs against the chains
        // (A/B, profiles/r03/ab_sfx): the N = 64 FAST kernel is short, so a full-chip pass by a thread per
        // (instance, height) runs on the launch stream right behind it; the general kernels run far longer
        // than the chains, so a thread per instance over its heights runs on the hash stream beside them.
        const bool on_launch = fast;
        if (pipe && K >= H && on_launch) {
            bftsim::RowSet& r = h->sets[h->cur_set];
            // big-endian seeds: predicted chains, for lossless schedules (no drops, no proposer crashes),
            // where the canonical tick commits every height; with drops most instances leave it early and the
            // predicted chains would mostly be repaired (drop64: 22.6 ms of chain kernels per launch against 0.7)
            const bool hspec = r.byz && n < h->hash_spec_max && ((p.thr16 == 0 && p.crash_on == 0) || h->spec_lossy);
            if (!hspec) {
                // suffix rows now (unless the lane chains encode them); the chains in the next batch (flush_batch)
                if (!(h->chain_inline && chain_kind(h, n, false) == bft::CHAIN_KERNEL_LANE)) {
                    HIPCHECK(h, bft::launch_hash_suffix((uint32_t)n, 1, K, sfx, false, s, p));
                    HIPCHECK(h, pmc_evict(h, s));
                }
                HIPCHECK(h, hipEventRecord(ev.sx, s));
            }
            ev.has_hash = false;                          // the batch's last launch carries the chain time
            // one chain kernel runs every pending launch with the batch's sizes (suffix-row stride, grid):
            // a launch of another size starts a batch of its own
            if (h->n_pend > 0 && (h->batch_p.n_instances != p.n_instances || h->batch_spec != hspec))
                if (int rc = flush_batch(h)) return rc;
            if (h->n_pend == 0) {
                h->batch_p = p;
                h->batch_spec = hspec;
                h->batch_after_sync = h->synced;
                h->synced = false;
                h->cur_hs = (h->cur_hs + 1) % (hspec ? h->n_hs_spec : h->n_hs);   // the batch's hash stream
                if (!h->hstr[h->cur_hs]) HIPCHECK(h, hipStreamCreateWithFlags(&h->hstr[h->cur_hs], hipStreamNonBlocking));
                h->batch_hs = h->cur_hs;
            }
            if (hspec && h->spec_early) {
                // this launch's predicted suffix rows now, on the batch's hash stream, once its set is free (the
                // caller's earlier work, the set's last hash pass): at the flush only the chains are left
                hipStream_t t = h->hstr[h->batch_hs];
                HIPCHECK(h, hipStreamWaitEvent(t, r.entry, 0));
                if (r.busy) HIPCHECK(h, hipStreamWaitEvent(t, r.batch_done ? r.batch_done : r.done, 0));
                bft::ChainSets one{};
                one.count = 1;
                one.sfx[0] = r.sfx; one.byz[0] = r.byz; one.bad[0] = r.bad; one.pred[0] = r.pred;
                one.first[0] = (uint32_t)first;
                bft::Params ps = p;
                ps.chain_prio = h->chain_prio_spec;
                HIPCHECK(h, bft::launch_spec_suffix((uint32_t)n, one, t, ps));
                HIPCHECK(h, pmc_evict(h, t));
            }
            h->pend[h->n_pend++] = {h->cur_set, (h->ring_head - 1) % bftsim::RING, (uint32_t)first, h->cur_cs};
            // the burst's first batch may be shorter (its chains start sooner; A/B: BFTSIM_FIRST_BATCH)
            const uint32_t cap = h->batch_after_sync && h->first_batch ? h->first_batch : h->hash_batch;
            if (h->n_pend >= cap) if (int rc = flush_batch(h)) return rc;
        } else {
            // one launch's hash pass: on a hash stream (pipelined) or the launch stream; chunks of K heights
            // share the suffix rows (suffix and chain kernels in order on one stream)
            hipStream_t t = s;
            if (pipe) {
                h->cur_hs = (h->cur_hs + 1) % h->n_hs;
                if (!h->hstr[h->cur_hs]) HIPCHECK(h, hipStreamCreateWithFlags(&h->hstr[h->cur_hs], hipStreamNonBlocking));
                t = h->hstr[h->cur_hs];
                HIPCHECK(h, hipStreamWaitEvent(t, ev.c1, 0));
            }
            HIPCHECK(h, hipEventRecord(ev.h0, t));
            const uint32_t kind = chain_kind(h, n, false);
            for (uint32_t x0 = 1; x0 <= H; x0 += K) {
                if (!(h->chain_inline && kind == bft::CHAIN_KERNEL_LANE)) {
                    HIPCHECK(h, bft::launch_hash_suffix((uint32_t)n, x0, K, sfx, !on_launch, t, p));
                    HIPCHECK(h, pmc_evict(h, t));
                }
                HIPCHECK(h, bft::launch_hash_chain((uint32_t)n, x0, K, sfx, kind, t, p));
                HIPCHECK(h, pmc_evict(h, t));
            }
            HIPCHECK(h, hipEventRecord(ev.h1, t));
            if (pipe) {
                HIPCHECK(h, hipEventRecord(h->sets[h->cur_set].done, t));
                h->sets[h->cur_set].batch_done = nullptr;
                h->sets[h->cur_set].busy = true;
            }
        }
    }
    if (pipe && p.need_seed) {                          // no hash pass: the set is free once this launch is done
        HIPCHECK(h, hipEventRecord(h->sets[h->cur_set].done, s));
        h->sets[h->cur_set].batch_done = nullptr;
        h->sets[h->cur_set].busy = true;
    }
    h->last_n = n;
    h->vsig_n = 0;
    h->last_first = first;
    h->last_stream = s;
    return BFTSIM_OK;
}

// the chains of the pending launches as one kernel on the next hash stream, after each launch's suffix rows
// `final`: the flush of bftsim_sync (the last launches of a burst), whose chains are the burst's tail
static int flush_batch(bftsim* h, bool final) {
    if (h->n_pend == 0) return BFTSIM_OK;
    hipStream_t t = h->hstr[h->batch_hs];           // chosen at the batch's first launch
    // A final batch of recorded chains (lossless schedules with predictions off, BFTSIM_HASH_SPEC=0: lane chains that
    // start once the last launch's consensus kernel is done and take ~2 ms) runs as predicted lane-pair chains
    // instead: they start now, beside the launches' consensus kernels, and only the check and the repairs are left
    // behind them. With predictions on (the default) every batch is predicted already (§4j).
    const bool first = h->batch_after_sync && h->spec_first;   // the burst's first batch (A/B arm)
    const bool conv = ((final && h->spec_final) || first) && !h->batch_spec && h->sets[h->pend[0].set].byz != nullptr &&
                      ((h->batch_p.thr16 == 0 && h->batch_p.crash_on == 0) || h->spec_lossy);   // lossless (launch)
    const bool spec = h->batch_spec || conv;
    if (h->chain_on_launch) t = h->cs[h->pend[h->n_pend - 1].cs];   // A/B: behind the launches, no overlap
    else if (conv && h->conv_stream && h->n_hs < bftsim::MAX_HS) {
        // on a hash stream of its own: on the batch's (recorded chains' rotation) it would start only behind the
        // recorded chains of an earlier batch there, ~9 ms at 16,384 (profiles/r06/traces/r06af_timeline_t16k.txt)
        if (!h->hstr[h->n_hs]) HIPCHECK(h, hipStreamCreateWithFlags(&h->hstr[h->n_hs], hipStreamNonBlocking));
        t = h->hstr[h->n_hs];
    }
    bft::ChainSets cs{};
    cs.count = h->n_pend;
    // a launch stream runs its launches in order, so the last pending launch of each launch stream stands for the
    // others: per stream one wait on its sx (recorded after the consensus kernels and, unless the lane chains encode
    // them, the suffix rows) instead of one wait per launch
    int32_t last_on[bftsim::MAX_CS];
    for (uint32_t k = 0; k < bftsim::MAX_CS; ++k) last_on[k] = -1;
    for (uint32_t i = 0; i < h->n_pend; ++i) last_on[h->pend[i].cs] = (int32_t)i;
    if (!spec) {
        for (uint32_t k = 0; k < bftsim::MAX_CS; ++k)
            if (last_on[k] >= 0) HIPCHECK(h, hipStreamWaitEvent(t, h->ring[h->pend[last_on[k]].ev].sx, 0));
    } else if (!h->spec_early || conv) {
        // predicted chains need only their sets free, not the launch streams' earlier kernels: the caller's work
        // before the last pending launch (its entry event: the caller's stream is in order) and each distinct
        // previous hash pass of the sets
        HIPCHECK(h, hipStreamWaitEvent(t, h->sets[h->pend[h->n_pend - 1].set].entry, 0));
        hipEvent_t seen[bftsim::MAX_BATCH];
        uint32_t ns = 0;
        for (uint32_t i = 0; i < h->n_pend; ++i) {
            const bftsim::RowSet& r = h->sets[h->pend[i].set];
            if (!r.busy) continue;
            const hipEvent_t e = r.batch_done ? r.batch_done : r.done;
            bool dup = false;
            for (uint32_t j = 0; j < ns; ++j) dup |= seen[j] == e;
            if (dup) continue;
            seen[ns++] = e;
            HIPCHECK(h, hipStreamWaitEvent(t, e, 0));
        }
    }
    for (uint32_t i = 0; i < h->n_pend; ++i) {
        const bftsim::RowSet& r = h->sets[h->pend[i].set];
        cs.sfx[i] = r.sfx; cs.ch[i] = r.ch; cs.hash[i] = r.hash;
        cs.rec[i] = r.rec; cs.byz[i] = r.byz; cs.bad[i] = r.bad; cs.pred[i] = r.pred; cs.first[i] = h->pend[i].first;
    }
    bftsim::LaunchEv& last = h->ring[h->pend[h->n_pend - 1].ev];
    bft::Params p = h->batch_p;
    HIPCHECK(h, hipEventRecord(last.h0, t));
    if (h->diag_no_chain) {
        // diagnostic (BFTSIM_TESTING + BFTSIM_DIAG_NO_CHAIN=1): no chain kernels, so no block hashes; the consensus
        // kernels' pace alone
    } else if (spec) {
        // a converted final batch on lane pairs (its chains are the burst's tail: latency); the burst's first batch
        // (spec_first) has the whole burst to finish in, so it keeps the large shard's lanes (throughput)
        const uint32_t kind = conv && !(first && !final) ? bft::CHAIN_KERNEL_PAIR : chain_kind(h, p.n_instances, true);
        // lane pairs: the sync's batch (the burst's tail) at chain_prio_spec, earlier full batches (slack: they end
        // long before the burst does) at chain_prio_spec_early
        p.chain_prio = kind == bft::CHAIN_KERNEL_LANE ? h->chain_prio_spec_lane
                     : final ? h->chain_prio_spec : h->chain_prio_spec_early;
        // the predicted blocks' suffix rows and chains, which need nothing of the consensus kernels (one suffix
        // pass for the whole batch: per launch on a stream of their own they fell behind the launches); once
        // every launch's consensus kernel is done, the check of its recorded blocks against the predictions, and
        // the chains again from the first height that differs
        // (inline lane chains predict, mask and encode each block themselves: no suffix pass)
        if ((!h->spec_early || conv) && !(kind == bft::CHAIN_KERNEL_LANE && h->chain_inline)) {
            HIPCHECK(h, bft::launch_spec_suffix(p.n_instances, cs, t, p));
            HIPCHECK(h, pmc_evict(h, t));
        }
        p.chain_mode = bft::CHAIN_PREDICTED;
        HIPCHECK(h, bft::launch_hash_chain_batch(p.n_instances, cs, kind, t, p));
        HIPCHECK(h, pmc_evict(h, t));
        for (uint32_t k = 0; k < bftsim::MAX_CS; ++k)   // every launch's consensus kernels (per launch stream)
            if (last_on[k] >= 0) HIPCHECK(h, hipStreamWaitEvent(t, h->ring[h->pend[last_on[k]].ev].c1, 0));
        HIPCHECK(h, bft::launch_spec_verify(p.n_instances, cs, t, p));
        HIPCHECK(h, pmc_evict(h, t));
        p.chain_mode = bft::CHAIN_REPAIR;
        HIPCHECK(h, bft::launch_hash_chain_batch(p.n_instances, cs, kind, t, p));
    } else {
        p.chain_mode = bft::CHAIN_RECORDED;
        HIPCHECK(h, bft::launch_hash_chain_batch(p.n_instances, cs, chain_kind(h, p.n_instances, false), t, p));
    }
    HIPCHECK(h, pmc_evict(h, t));
    HIPCHECK(h, hipEventRecord(last.h1, t));
    last.has_hash = true;
    hipEvent_t& bd = h->batch_ev[h->batch_ev_head++ % bftsim::BATCH_EVS];
    if (!bd) HIPCHECK(h, hipEventCreateWithFlags(&bd, hipEventDisableTiming));
    HIPCHECK(h, hipEventRecord(bd, t));
    for (uint32_t i = 0; i < h->n_pend; ++i) {
        bftsim::RowSet& r = h->sets[h->pend[i].set];
        r.batch_done = bd;
        r.busy = true;
    }
    h->n_pend = 0;
    return BFTSIM_OK;
}

int bftsim_set_hash_batch(bftsim_t* h, uint32_t launches) {
    if (!h) return BFTSIM_EINVAL;
    if (launches < 1 || launches > bftsim::MAX_BATCH) return fail(h, BFTSIM_EINVAL, "hash batch must be 1..32 launches");
    if (int rc = flush_batch(h)) return rc;
    h->hash_batch = launches;
    return BFTSIM_OK;
}

int bftsim_set_pipeline(bftsim_t* h, int on) {
    if (!h) return BFTSIM_EINVAL;
    if (on < 0 || on > (int)bftsim::MAX_SETS) return fail(h, BFTSIM_EINVAL, "pipeline depth must be 0..32");
    const int depth = on == 0 ? 0 : on == 1 ? 2 : on;
    if (depth == h->pipeline) return BFTSIM_OK;
    int rc = h->last_stream ? sync_all(h) : BFTSIM_OK;
    if (rc) return rc;
    h->pipeline = depth;
    (void)hipSetDevice(h->device);
    free_bufs(h);                                   // re-sized (one or two sets) by the next prepare
    return BFTSIM_OK;
}

int bftsim_kernel_ms_sum(bftsim_t* h, double* consensus_ms, double* hash_ms, uint32_t* launches) {
    if (!h) return BFTSIM_EINVAL;
    if (int rc = flush_batch(h)) return rc;           // a pending batch's chain time goes to its last launch
    for (uint32_t i = 0; i < bftsim::RING; ++i) {
        bftsim::LaunchEv& ev = h->ring[i];
        if (!ev.pending) continue;
        HIPCHECK(h, hipEventSynchronize(ev.has_hash ? ev.h1 : ev.c1));
        float a = 0, b = 0;
        HIPCHECK(h, hipEventElapsedTime(&a, ev.c0, ev.c1));
        if (ev.has_hash) HIPCHECK(h, hipEventElapsedTime(&b, ev.h0, ev.h1));
        h->acc_c += a; h->acc_h += b; h->acc_n += 1;
        ev.pending = false;
    }
    if (consensus_ms) *consensus_ms = h->acc_c;
    if (hash_ms) *hash_ms = h->acc_h;
    if (launches) *launches = h->acc_n;
    h->acc_c = h->acc_h = 0;
    h->acc_n = 0;
    return BFTSIM_OK;
}

int bftsim_sync(bftsim_t* h) {
    if (!h) return BFTSIM_EINVAL;
    if (!h->last_stream) return BFTSIM_OK;
    return sync_all(h);
}

int bftsim_last_kernel_ms(bftsim_t* h, float* cms, float* hms) {
    if (!h || h->ring_head == 0) return BFTSIM_EINVAL;
    if (int rc = flush_batch(h)) return rc;           // the last launch's chains may still be pending
    bftsim::LaunchEv& ev = h->ring[(h->ring_head - 1) % bftsim::RING];
    HIPCHECK(h, hipEventSynchronize(ev.has_hash ? ev.h1 : ev.c1));
    float a = 0, b = 0;
    HIPCHECK(h, hipEventElapsedTime(&a, ev.c0, ev.c1));
    if (ev.has_hash) HIPCHECK(h, hipEventElapsedTime(&b, ev.h0, ev.h1));
    if (cms) *cms = a;
    if (hms) *hms = b;
    return BFTSIM_OK;
}

// the fetch family writes one row per launched instance into caller buffers: refuse a short buffer
// before anything is written (include/bftsim.h bftsim_launched_count)
static int check_launched(bftsim* h, uint64_t capacity, const char* what) {
    if (h->last_n == 0 || !h->d_ch) return fail(h, BFTSIM_EINVAL, std::string(what) + ": nothing launched");
    if (capacity < h->last_n)
        return fail(h, BFTSIM_EINVAL, std::string(what) + ": buffers hold " + std::to_string(capacity) +
                                          " instances, the last launch has " + std::to_string(h->last_n));
    return BFTSIM_OK;
}

int bftsim_launched_count(bftsim_t* h, uint64_t* first, uint64_t* n) {
    if (!h) return BFTSIM_EINVAL;
    if (first) *first = h->last_n ? h->last_first : 0;
    if (n) *n = h->d_ch ? h->last_n : 0;
    return BFTSIM_OK;
}

int bftsim_fetch(bftsim_t* h, bftsim_result* out) {
    if (!h || !out) return BFTSIM_EINVAL;
    if (h->window) return fail(h, BFTSIM_EINVAL, "windowed run: per-height rows are not kept (bftsim_fetch_summary)");
    if (int rc = check_launched(h, out->capacity, "bftsim_fetch")) return rc;
    if (int rc = sync_all(h)) return rc;
    uint64_t n = h->last_n;
    uint32_t H = h->cfg.heights, hc = h->hcap;
    std::vector<uint32_t> ch32(n);
    HIPCHECK(h, hipMemcpy(ch32.data(), h->d_ch, n * 4, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < n; ++i) out->committed_height[i] = ch32[i];
    HIPCHECK(h, hipMemcpy(out->flags, h->d_flags, n * 4, hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(out->ticks, h->d_ticks, n * 4, hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(out->views, h->d_views, n * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> rec(n * hc * 4);
    std::vector<uint8_t> hs(n * hc * 32);
    HIPCHECK(h, hipMemcpy(rec.data(), h->d_rec, rec.size() * 4, hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(hs.data(), h->d_hash, hs.size(), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t ch = out->committed_height[i];
        for (uint32_t x = 1; x <= H; ++x) {
            uint64_t o = i * H + (x - 1);
            const uint32_t* row = &rec[(i * hc + x) * 4];
            bool ok = x <= ch;
            out->round[o] = ok ? (uint16_t)row[0] : 0;
            out->proposer[o] = ok ? (uint16_t)(row[1] & 0xffffu) : 0;
            out->variant[o] = ok ? (uint8_t)((row[1] >> 16) & 1u) : 0;
            out->time_tick[o] = ok ? row[2] : 0;
            if (ok) memcpy(out->block_hash + o * 32, &hs[(i * hc + x) * 32], 32);
            else memset(out->block_hash + o * 32, 0, 32);
        }
    }
    if (h->h_trace && h->d_trace) {
        size_t tb = n * (size_t)h->trace_ticks * h->cfg.n * 8;
        HIPCHECK(h, hipMemcpy(h->h_trace, h->d_trace, tb, hipMemcpyDeviceToHost));
    }
    return BFTSIM_OK;
}

int bftsim_export_headers(bftsim_t* h, uint64_t capacity, uint8_t* hdr, uint32_t* hdr_len) {
    if (!h || !hdr || !hdr_len) return BFTSIM_EINVAL;
    if (h->window) return fail(h, BFTSIM_EINVAL, "windowed run: per-height rows are not kept");
    if (int rc = check_launched(h, capacity, "bftsim_export_headers")) return rc;
    if (int rc = sync_all(h)) return rc;
    const uint64_t n = h->last_n, H = h->cfg.heights, cnt = n * H;
    bft::Params p = make_params(h, h->last_first, n);
    uint8_t* d_out = nullptr;
    uint32_t* d_len = nullptr;
    HIPCHECK(h, hipMalloc(&d_out, cnt * BFTSIM_HEADER_SLOT));
    HIPCHECK(h, hipMalloc(&d_len, cnt * 4));
    hipLaunchKernelGGL(bft::bft_export_kernel, dim3((uint32_t)((cnt + 255) / 256)), dim3(256), 0, h->last_stream, p,
                       d_out, d_len);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(h->last_stream);
    if (e == hipSuccess) e = hipMemcpy(hdr, d_out, cnt * BFTSIM_HEADER_SLOT, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hdr_len, d_len, cnt * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_len);
    if (e != hipSuccess) return fail(h, BFTSIM_EHIP, std::string("bftsim_export_headers: ") + hipGetErrorString(e));
    return BFTSIM_OK;
}

int bftsim_run(bftsim_t* h, uint64_t first, uint64_t n, bftsim_result* out) {
    if (!h || !out) return BFTSIM_EINVAL;
    if (out->capacity < n)
        return fail(h, BFTSIM_EINVAL, "bftsim_run: result buffers hold " + std::to_string(out->capacity) +
                                          " instances, " + std::to_string(n) + " requested");
    for (;;) {
        int rc = bftsim_prepare(h, n);
        if (rc) return rc;
        if ((rc = bftsim_launch(h, first, nullptr))) return rc;
        if ((rc = bftsim_fetch(h, out))) return rc;
        // the RoundChangeSet is unbounded in the reference (round_change_set.rs:11-35): an overflowing
        // batch is run again at twice the capacity
        bool over = false;
        for (uint64_t i = 0; i < n && !over; ++i) over = (out->flags[i] & BFTSIM_FLAG_RCS_OVERFLOW) != 0;
        if (!over || h->rcs_k >= bft::RCS_MAX_K) return BFTSIM_OK;
        const uint32_t k = 2u * h->rcs_k < bft::RCS_MAX_K ? 2u * h->rcs_k : bft::RCS_MAX_K;
        // the larger tables must fit beside everything else, or the flagged results stand (bftsim.h)
        const uint64_t per_block = h->seg > 64 ? 1 : 64 / h->seg, blocks = (n + per_block - 1) / per_block;
        const uint64_t grow = blocks * (bft::rcs_words(h->seg, k) - bft::rcs_words(h->seg, h->rcs_k)) * 4;
        size_t free_b = 0, total_b = 0;
        HIPCHECK(h, hipMemGetInfo(&free_b, &total_b));
        if (grow > free_b / 10 * 9) return BFTSIM_OK;
        if ((rc = bftsim_set_rcs_capacity(h, k))) return rc;
    }
}

int bftsim_fetch_summary(bftsim_t* h, uint64_t capacity, uint64_t* committed_height, uint32_t* flags, uint32_t* ticks,
                         uint64_t* views, uint8_t* tip_hash) {
    if (!h) return BFTSIM_EINVAL;
    if (int rc = check_launched(h, capacity, "bftsim_fetch_summary")) return rc;
    if (int rc = sync_all(h)) return rc;                // the hash pass may run on its own stream
    uint64_t n = h->last_n;
    if (tip_hash) {
        bft::Params p = make_params(h, h->last_first, n);
        hipLaunchKernelGGL(bft::bft_tip_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, h->last_stream, p,
                           h->d_tips);
        HIPCHECK(h, hipGetLastError());
    }
    HIPCHECK(h, hipStreamSynchronize(h->last_stream));
    if (committed_height) {
        std::vector<uint32_t> ch32(n);
        HIPCHECK(h, hipMemcpy(ch32.data(), h->d_ch, n * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; ++i) committed_height[i] = ch32[i];
    }
    if (flags) HIPCHECK(h, hipMemcpy(flags, h->d_flags, n * 4, hipMemcpyDeviceToHost));
    if (ticks) HIPCHECK(h, hipMemcpy(ticks, h->d_ticks, n * 4, hipMemcpyDeviceToHost));
    if (views) HIPCHECK(h, hipMemcpy(views, h->d_views, n * 8, hipMemcpyDeviceToHost));
    if (tip_hash) HIPCHECK(h, hipMemcpy(tip_hash, h->d_tips, n * 32, hipMemcpyDeviceToHost));
    return BFTSIM_OK;
}

int bftsim_comm_available(void) {
    Rccl& r = rccl();
    return r.ok ? BFTSIM_OK : BFTSIM_EUNSUPPORTED;
}

int bftsim_comm_unique_id(uint8_t out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "NCCL_UNIQUE_ID_BYTES");
    if (!out) return BFTSIM_EINVAL;
    Rccl& r = rccl();
    if (!r.ok) return BFTSIM_EUNSUPPORTED;
    ncclUniqueId id;
    StdoutToStderr quiet;
    if (r.get_id(&id) != ncclSuccess) return BFTSIM_EHIP;
    memcpy(out, &id, 128);
    return BFTSIM_OK;
}

int bftsim_comm_init(bftsim_t* h, int world_size, int rank, const uint8_t unique_id[128]) {
    if (!h || !unique_id || world_size < 1 || rank < 0 || rank >= world_size)
        return fail(h, BFTSIM_EINVAL, "bftsim_comm_init: bad world / rank");
    Rccl& r = rccl();
    if (!r.ok) return fail(h, BFTSIM_EUNSUPPORTED, r.why);
    HIPCHECK(h, hipSetDevice(h->device));
    if (h->comm) { comm_destroy(h->comm); h->comm = nullptr; }
    ncclUniqueId id;
    memcpy(&id, unique_id, 128);
    ncclResult_t e;
    {
        StdoutToStderr quiet;
        e = r.init_rank(&h->comm, world_size, id, rank);
    }
    if (e != ncclSuccess) { h->comm = nullptr; return fail(h, BFTSIM_EHIP, std::string("ncclCommInitRank: ") + r.err(e)); }
    if (!h->d_red) HIPCHECK(h, hipMalloc(&h->d_red, sizeof(bftsim_stats)));
    return BFTSIM_OK;
}

// bftsim_stats of the last launch of every rank, summed (every field is a count): the device image of
// the local statistics, one ncclAllReduce(sum, uint64) over xGMI on the launch stream, one copy back
int bftsim_stats_allreduce(bftsim_t* h, bftsim_stats* out) {
    if (!h || !out) return BFTSIM_EINVAL;
    if (!h->comm) return fail(h, BFTSIM_EINVAL, "bftsim_comm_init not called");
    if (h->last_n == 0 || !h->d_ch) return fail(h, BFTSIM_EINVAL, "nothing launched");
    static_assert(sizeof(bftsim_stats) == (11 + bft::HIST_BINS) * 8, "bftsim_stats: a flat array of uint64 counts");
    HIPCHECK(h, hipSetDevice(h->device));
    bft::Params p = make_params(h, h->last_first, h->last_n);
    hipStream_t s = h->last_stream;
    HIPCHECK(h, hipMemsetAsync(h->d_stats, 0, 16 * 8, s));
    uint32_t g = (uint32_t)((h->last_n + 255) / 256);
    hipLaunchKernelGGL(bft::bft_stats_kernel, dim3(g), dim3(256), 0, s, p, h->d_stats);
    HIPCHECK(h, hipGetLastError());
    HIPCHECK(h, hipMemcpyAsync(h->d_red, h->d_stats, 11 * 8, hipMemcpyDeviceToDevice, s));
    HIPCHECK(h, hipMemcpyAsync(h->d_red + 11, h->d_hist, bft::HIST_BINS * 8, hipMemcpyDeviceToDevice, s));
    Rccl& r = rccl();
    ncclResult_t e;
    {
        StdoutToStderr quiet;
        e = r.all_reduce(h->d_red, h->d_red, sizeof(bftsim_stats) / 8, ncclUint64, ncclSum, h->comm, s);
    }
    if (e != ncclSuccess) return fail(h, BFTSIM_EHIP, std::string("ncclAllReduce: ") + r.err(e));
    HIPCHECK(h, hipMemcpyAsync(out, h->d_red, sizeof(bftsim_stats), hipMemcpyDeviceToHost, s));
    HIPCHECK(h, hipStreamSynchronize(s));
    return BFTSIM_OK;
}

int bftsim_set_crypto(bftsim_t* h, const uint8_t* secrets32, const uint8_t* forged, uint32_t log_cap) {
    if (!h) return BFTSIM_EINVAL;
    const uint32_t n = h->cfg.n;
    if (h->last_stream) if (int rc = sync_all(h)) return rc;   // pending chains use the buffers freed below
    if (!secrets32) {                                  // off
        h->crypto = false;
        free_bufs(h);
        return BFTSIM_OK;
    }
    if (h->window) return fail(h, BFTSIM_EINVAL, "real-crypto mode needs the per-height rows (window 0)");
    SigApi& a = sig_api();
    if (!a.ok) return fail(h, BFTSIM_EUNSUPPORTED, a.why);
    HIPCHECK(h, hipSetDevice(h->device));
    if (!h->sig && a.create(h->device, &h->sig) != 0) return fail(h, BFTSIM_EHIP, "bftsig_create failed");
    // the forged key of validator v: keccak(secret_v), a valid key that is not a validator's
    std::vector<uint8_t> keys((size_t)2 * n * 32);
    memcpy(keys.data(), secrets32, (size_t)n * 32);
    for (uint32_t v = 0; v < n; ++v) host_keccak(secrets32 + 32u * v, 32, keys.data() + (size_t)(n + v) * 32);
    if (!h->d_keys) HIPCHECK(h, hipMalloc(&h->d_keys, (size_t)2 * 256 * 32));
    HIPCHECK(h, hipMemcpy(h->d_keys, keys.data(), keys.size(), hipMemcpyHostToDevice));
    // every secret must derive the validator address of its index (the sorted validator set)
    uint8_t *d_addr = nullptr, *d_ok = nullptr;
    HIPCHECK(h, hipMalloc(&d_addr, (size_t)n * 20));
    HIPCHECK(h, hipMalloc(&d_ok, n));
    int rc = a.secret_to_address(h->sig, h->d_keys, n, nullptr, d_addr, d_ok, nullptr);
    std::vector<uint8_t> addr((size_t)n * 20), ok(n);
    hipError_t e = rc == 0 ? hipDeviceSynchronize() : hipSuccess;
    if (rc == 0 && e == hipSuccess) e = hipMemcpy(addr.data(), d_addr, addr.size(), hipMemcpyDeviceToHost);
    if (rc == 0 && e == hipSuccess) e = hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost);
    (void)hipFree(d_addr); (void)hipFree(d_ok);
    if (rc != 0) return fail(h, BFTSIM_EHIP, std::string("bftsig_secret_to_address: ") + a.last_error(h->sig));
    if (e != hipSuccess) return fail(h, BFTSIM_EHIP, hipGetErrorString(e));
    for (uint32_t v = 0; v < n; ++v)
        if (!ok[v] || memcmp(addr.data() + 20u * v, h->addresses.data() + 20u * v, 20) != 0)
            return fail(h, BFTSIM_EINVAL, "secret " + std::to_string(v) + " does not derive validator address " +
                                              std::to_string(v));
    for (int k = 0; k < 4; ++k) h->forged[k] = 0;
    if (forged)
        for (uint32_t v = 0; v < n; ++v)
            if (forged[v]) h->forged[v >> 6] |= 1ull << (v & 63u);
    h->mlog_cap = log_cap ? log_cap : h->cfg.heights * (4u * n + 8u) + 64u * n;
    h->crypto = true;
    free_bufs(h);                                      // the log is allocated by the next prepare
    return BFTSIM_OK;
}

int bftsim_crypto_verify(bftsim_t* h, bftsim_crypto_report* out, uint64_t capacity, uint8_t* inst_checksum,
                         uint32_t* inst_messages) {
    if (!h || !out) return BFTSIM_EINVAL;
    if (!h->crypto) return fail(h, BFTSIM_EINVAL, "bftsim_set_crypto not called");
    if (h->last_n == 0 || !h->d_mlog) return fail(h, BFTSIM_EINVAL, "nothing launched");
    if (inst_checksum || inst_messages)
        if (int rc = check_launched(h, capacity, "bftsim_crypto_verify")) return rc;
    if (int rc = sync_all(h)) return rc;
    SigApi& sa = sig_api();
    const uint64_t n = h->last_n;
    hipStream_t s = h->last_stream;
    std::vector<uint32_t> cnt(n);
    HIPCHECK(h, hipMemcpy(cnt.data(), h->d_mlog_n, n * 4, hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(n);
    uint64_t M = 0, over = 0;
    for (uint64_t i = 0; i < n; ++i) {
        off[i] = M;
        if (cnt[i] > h->mlog_cap) ++over;
        M += cnt[i] < h->mlog_cap ? cnt[i] : h->mlog_cap;
        if (inst_messages) inst_messages[i] = cnt[i];
    }
    memset(out, 0, sizeof *out);
    out->log_overflows = over;
    if (over) return fail(h, BFTSIM_EINVAL, "broadcast log overflow: raise log_cap (bftsim_set_crypto)");
    // device arrays of the pass (one allocation)
    const uint64_t Mx = M ? M : 1;
    const uint64_t sz_msg = 8 + 32 + 4 + 4 + 32 + 65 + 20 + 1, sz_cm = 32 + 32 + 4 + 65 + 1 + 20 + 4;
    uint8_t* pool = nullptr;
    const uint64_t bytes = n * 8 + Mx * (sz_msg + sz_cm) + n * 32 + 64 + 256;
    HIPCHECK(h, hipMalloc(&pool, bytes));
    uint8_t* q = pool;
    auto take = [&](uint64_t b) { uint8_t* r = q; q += (b + 15) & ~15ull; return r; };
    bft::CryptoArgs a{};
    a.mlog = h->d_mlog; a.mlog_n = h->d_mlog_n; a.cap = h->mlog_cap; a.n_val = h->cfg.n;
    for (int k = 0; k < 4; ++k) a.forged[k] = h->forged[k];
    uint64_t* d_off = (uint64_t*)take(n * 8); a.moff = d_off;
    a.mref = (uint64_t*)take(Mx * 8); a.raw = take(Mx * 32); a.key = (uint32_t*)take(Mx * 4);
    a.msg_k = (uint32_t*)take(Mx * 4); a.sign_dig = take(Mx * 32); a.sigs = take(Mx * 65);
    a.rec_addr = take(Mx * 20); a.rec_ok = take(Mx);
    a.seal_dig = take(Mx * 32); a.seal_raw = take(Mx * 32); a.seal_key = (uint32_t*)take(Mx * 4);
    a.seals = take(Mx * 65); a.seal_ok = take(Mx); uint8_t* seal_addr = take(Mx * 20);
    uint8_t* sig_ok = take(Mx);
    a.ncm = (uint32_t*)take(4); a.inst_ck = (uint32_t*)take(n * 32); a.counts = (unsigned long long*)take(64);
    int rc = BFTSIM_OK;
    hipError_t e = hipMemcpyAsync(d_off, off.data(), n * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(a.ncm, 0, 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(a.inst_ck, 0, n * 32, s);
    if (e == hipSuccess) e = hipMemsetAsync(a.counts, 0, 64, s);
    bft::Params p = make_params(h, h->last_first, n);
    uint32_t ncm = 0;
    if (e == hipSuccess && M) {
        hipLaunchKernelGGL(bft::bft_crypto_prep_kernel, dim3((uint32_t)n), dim3(64), 0, s, p, a);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(&ncm, a.ncm, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        // commit seals first: they are part of the Commit's sign payload
        if (e == hipSuccess && ncm && sa.sign(h->sig, h->d_keys, a.seal_key, a.seal_dig, ncm, a.seals, sig_ok, s) != 0)
            rc = fail(h, BFTSIM_EHIP, std::string("bftsig_sign (seals): ") + sa.last_error(h->sig));
        const uint32_t g = (uint32_t)((M + 63) / 64);
        if (e == hipSuccess && rc == 0) {
            hipLaunchKernelGGL(bft::bft_crypto_digest_kernel, dim3(g), dim3(64), 0, s, p, a, M);
            e = hipGetLastError();
        }
        if (e == hipSuccess && rc == 0 && sa.sign(h->sig, h->d_keys, a.key, a.sign_dig, M, a.sigs, sig_ok, s) != 0)
            rc = fail(h, BFTSIM_EHIP, std::string("bftsig_sign: ") + sa.last_error(h->sig));
        // the receivers: recover every message's signer, and every seal (verify_commit)
        if (e == hipSuccess && rc == 0 && sa.recover(h->sig, a.sign_dig, a.sigs, M, nullptr, a.rec_addr, a.rec_ok, s) != 0)
            rc = fail(h, BFTSIM_EHIP, std::string("bftsig_recover: ") + sa.last_error(h->sig));
        if (e == hipSuccess && rc == 0 && ncm &&
            sa.recover(h->sig, a.seal_raw, a.seals, ncm, nullptr, seal_addr, a.seal_ok, s) != 0)
            rc = fail(h, BFTSIM_EHIP, std::string("bftsig_recover (seals): ") + sa.last_error(h->sig));
        if (e == hipSuccess && rc == 0) {
            hipLaunchKernelGGL(bft::bft_crypto_check_kernel, dim3(g), dim3(64), 0, s, p, a, M);
            e = hipGetLastError();
        }
        // the votes of every committed block, kept for bftsim_export_ledger
        const uint64_t vs = n * (uint64_t)h->cfg.heights * h->cfg.n;
        (void)hipFree(h->d_vsig); (void)hipFree(h->d_vhas);
        h->d_vsig = nullptr; h->d_vhas = nullptr; h->vsig_n = 0;
        if (e == hipSuccess && rc == 0) e = hipMalloc(&h->d_vsig, vs * 65);
        if (e == hipSuccess && rc == 0) e = hipMalloc(&h->d_vhas, vs);
        if (e == hipSuccess && rc == 0) e = hipMemsetAsync(h->d_vhas, 0, vs, s);
        if (e == hipSuccess && rc == 0) {
            hipLaunchKernelGGL(bft::bft_crypto_votes_kernel, dim3(g), dim3(64), 0, s, p, a, M, h->d_vsig, h->d_vhas);
            e = hipGetLastError();
            if (e == hipSuccess) h->vsig_n = n;
        }
    }
    unsigned long long c[8] = {0};
    if (e == hipSuccess && rc == 0) e = hipMemcpyAsync(c, a.counts, 64, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && rc == 0 && inst_checksum) e = hipMemcpyAsync(inst_checksum, a.inst_ck, n * 32, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(pool);
    if (rc) return rc;
    if (e != hipSuccess) return fail(h, BFTSIM_EHIP, std::string("bftsim_crypto_verify: ") + hipGetErrorString(e));
    out->messages = c[0];
    out->seals = c[1];
    out->forged = c[2];
    out->recovered_as_sender = c[3];
    out->mismatches = c[4];
    out->seal_errors = c[5];
    out->signatures = c[0] + c[1];
    out->recoveries = c[0] + c[1];
    return BFTSIM_OK;
}

int bftsim_export_ledger(bftsim_t* h, uint64_t capacity, uint8_t* hdr, uint64_t slot_bytes, uint32_t* hdr_len) {
    if (!h || !hdr || !hdr_len) return BFTSIM_EINVAL;
    if (!h->crypto || h->vsig_n == 0 || h->vsig_n != h->last_n)
        return fail(h, BFTSIM_EINVAL, "no votes: bftsim_crypto_verify after the launch first");
    if (int rc = check_launched(h, capacity, "bftsim_export_ledger")) return rc;
    if (slot_bytes < bftsim_ledger_slot_bytes(h->cfg.n)) return fail(h, BFTSIM_EINVAL, "slot_bytes too small");
    if (int rc = sync_all(h)) return rc;
    const uint64_t n = h->last_n, H = h->cfg.heights, cnt = n * H;
    bft::Params p = make_params(h, h->last_first, n);
    uint8_t* d_out = nullptr;
    uint32_t* d_len = nullptr;
    HIPCHECK(h, hipMalloc(&d_out, cnt * slot_bytes));
    HIPCHECK(h, hipMalloc(&d_len, cnt * 4));
    hipLaunchKernelGGL(bft::bft_export_votes_kernel, dim3((uint32_t)((cnt + 63) / 64)), dim3(64), 0, h->last_stream, p,
                       h->d_vsig, h->d_vhas, d_out, slot_bytes, d_len);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(h->last_stream);
    if (e == hipSuccess) e = hipMemcpy(hdr, d_out, cnt * slot_bytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hdr_len, d_len, cnt * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_len);
    if (e != hipSuccess) return fail(h, BFTSIM_EHIP, std::string("bftsim_export_ledger: ") + hipGetErrorString(e));
    return BFTSIM_OK;
}

uint64_t bftsim_ledger_slot_bytes(uint32_t n) { return ((uint64_t)BFTSIM_HEADER_SLOT + 3 + (uint64_t)n * 133 + 7) & ~7ull; }

int bftsim_stats_get(bftsim_t* h, bftsim_stats* out) {
    if (!h || !out) return BFTSIM_EINVAL;
    if (h->last_n == 0 || !h->d_ch) return fail(h, BFTSIM_EINVAL, "nothing launched");
    HIPCHECK(h, hipSetDevice(h->device));
    bft::Params p = make_params(h, h->last_first, h->last_n);
    HIPCHECK(h, hipMemsetAsync(h->d_stats, 0, 16 * 8, h->last_stream));
    uint32_t g = (uint32_t)((h->last_n + 255) / 256);
    hipLaunchKernelGGL(bft::bft_stats_kernel, dim3(g), dim3(256), 0, h->last_stream, p, h->d_stats);
    HIPCHECK(h, hipGetLastError());
    unsigned long long st[16];
    uint64_t hist[bft::HIST_BINS];
    HIPCHECK(h, hipMemcpyAsync(st, h->d_stats, sizeof st, hipMemcpyDeviceToHost, h->last_stream));
    HIPCHECK(h, hipMemcpyAsync(hist, h->d_hist, sizeof hist, hipMemcpyDeviceToHost, h->last_stream));
    HIPCHECK(h, hipStreamSynchronize(h->last_stream));
    out->instances = st[0];
    out->committed_heights = st[1];
    out->views = st[2];
    out->ticks = st[3];
    for (int i = 0; i < 7; ++i) out->flagged[i] = st[4 + i];
    for (int i = 0; i < 65; ++i) out->round_hist[i] = hist[i];
    for (int i = 0; i < 65; ++i) out->latency_hist[i] = hist[65 + i];
    return BFTSIM_OK;
}

}  // extern "C"
