// wave_emu.cpp — TEST-ONLY CPU emulation of one 64-lane wavefront (or one workgroup of S = 128 /
// 256 lanes for N > 64) running the SAME kernel body (consensus-rs_amd/csrc/bft_wave.h) that the
// gfx950 kernel runs. Each lane is a ucontext fiber;
// collectives (ballot, shfl_xor, sync) are rendezvous points where every live lane must arrive at
// the same collective — a non-uniform collective aborts, which catches divergence bugs before
// they reach the GPU. Never linked into libbftsim.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ucontext.h>

#include <vector>

#include "../../consensus-rs_amd/csrc/bft_host.h"
#ifdef BFT_CENSUS_BUILD
// analysis build only (scripts/phase_census.py): a histogram of the phase shapes the general kernel sees,
// keyed by the kinds in flight, the uniformity bits and the chosen path
#include <map>
static std::map<uint32_t, uint64_t> g_census;
#define BFT_PHASE_CENSUS(ps, path, me)                                                                     \
    do {                                                                                                   \
        if ((me) == 0) {                                                                                   \
            uint32_t k_ = (S > 64 ? (ps.kinds & 127u)                                                       \
                                  : ((ps.k_pp.any() ? 1u : 0u) | (ps.k_pr.any() ? 2u : 0u) | (ps.k_cm.any() ? 4u : 0u) | \
                                     (ps.k_ocm.any() ? 8u : 0u) | (ps.k_rc.any() ? 16u : 0u) |               \
                                     (ps.k_sync.any() ? 32u : 0u) | (ps.k_blk.any() ? 64u : 0u))) |          \
                          (ps.u_pr ? 0 : 128u) | (ps.u_cm ? 0 : 256u) |                                     \
                          (ps.u_blk ? 0 : 512u) | ((uint32_t)(path) << 12);                                   \
            g_census[k_] += 1;                                                                             \
        }                                                                                                  \
    } while (0)
extern "C" int emu_census(uint32_t* keys, uint64_t* counts, int cap) {
    int i = 0;
    for (auto& kv : g_census) { if (i < cap) { keys[i] = kv.first; counts[i] = kv.second; } ++i; }
    g_census.clear();
    return i;
}
#endif
#include "../../consensus-rs_amd/csrc/bft_wave.h"
#include "../../consensus-rs_amd/csrc/bft_fast64.h"

namespace {

constexpr int MAXL = 256;
struct Sched {
    ucontext_t main_ctx;
    ucontext_t ctx[MAXL];
    std::vector<char> stack[MAXL];
    bool done[MAXL];
    int nl;           // lanes: 64, or S for a workgroup segment
    int cur;
    int op[MAXL];
    uint64_t arg[MAXL];
    uint64_t res[MAXL];
    uint64_t res4[4];  // workgroup ballot words
    uint64_t seq[MAXL];
    const bft::Params* P;
    uint8_t* lds;
    uint32_t wave;
    bool fast;  // FAST kernel (S == 64, power-of-two N)
    void (*body)(int lane);   // another wave body than the consensus kernels (emu_wave_chain_check)
};
thread_local Sched* g = nullptr;

void yield_to_sched() { swapcontext(&g->ctx[g->cur], &g->main_ctx); }

uint64_t collective(int op, uint64_t arg) {
    int l = g->cur;
    g->op[l] = op; g->arg[l] = arg; g->seq[l]++;
    yield_to_sched();
    return g->res[l];
}

struct EmuWave {
    void init(uint8_t*) {}
    static uint32_t lane() { return (uint32_t)g->cur; }
    static uint64_t ballot(bool p) {
        int l = g->cur;
        g->op[l] = 1; g->arg[l] = p ? 1 : 0; g->seq[l]++;
        yield_to_sched();
        return g->res[l];
    }
    static uint32_t shfl_xor(uint32_t v, int m) {
        int l = g->cur;
        g->op[l] = 2; g->arg[l] = (uint64_t)v | ((uint64_t)(uint32_t)m << 32); g->seq[l]++;
        yield_to_sched();
        return (uint32_t)g->res[l];
    }
    static uint32_t shfl(uint32_t v, uint32_t src) {
        int l = g->cur;
        g->op[l] = 4; g->arg[l] = (uint64_t)v | ((uint64_t)(src & 63u) << 32); g->seq[l]++;
        yield_to_sched();
        return (uint32_t)g->res[l];
    }
    static uint32_t readlane(uint32_t v, uint32_t src) { return shfl(v, src); }
    static uint32_t bperm(uint32_t addr, uint32_t v) { return shfl(v, (addr >> 2) & 63u); }   // ds_bpermute_b32
    static uint32_t pair_swap(uint32_t v) { return shfl(v, (uint32_t)g->cur ^ 1u); }           // DPP quad [1,0,3,2]
    // WaveHip::keccak_pair (lane pairs: the even lane holds the low halves, the odd lane the high halves of the
    // 25 state words) as ONE collective: the scheduler joins each pair's halves and permutes the 64-bit state
    static void keccak_pair(uint32_t X[25], uint32_t odd) {
        int l = g->cur;
        if ((uint32_t)(l & 1) != odd) { fprintf(stderr, "emu: keccak_pair parity of lane %d\n", l); abort(); }
        g->op[l] = 10; g->arg[l] = (uint64_t)(uintptr_t)X; g->seq[l]++;
        yield_to_sched();
    }
    static uint32_t rank_below(uint64_t m) {                                                   // mbcnt
        const uint32_t l = (uint32_t)g->cur;
        return (uint32_t)__builtin_popcountll(l ? (m & ((1ull << l) - 1ull)) : 0ull);
    }
    // DPP row_shl / row_shr (16-lane rows; a source outside the row reads 0)
    template <int N> static uint32_t row_shl(uint32_t v) {
        const uint32_t l = (uint32_t)g->cur, s = l + N;
        const uint32_t r = shfl(v, s & 63u);
        return (s >> 4) == (l >> 4) ? r : 0u;
    }
    template <int N> static uint32_t row_shr(uint32_t v) {
        const uint32_t l = (uint32_t)g->cur, s = l - N;
        const uint32_t r = shfl(v, s & 63u);
        return (l >= (uint32_t)N && (s >> 4) == (l >> 4)) ? r : 0u;
    }
    // readfirstlane on the GPU: here it checks that the value really is wave-uniform
    static uint32_t uni(uint32_t v) {
        uint32_t f = shfl(v, 0);
        if (f != v) { fprintf(stderr, "emu: uni() of a non-uniform value (lane %d)\n", g->cur); abort(); }
        return v;
    }
    static uint64_t clock() { return 0; }
    static void sync() {
        int l = g->cur;
        g->op[l] = 3; g->seq[l]++;
        yield_to_sched();
    }
    static uint32_t gload(const uint32_t* p) { return *p; }
    static void gstore(uint32_t* p, uint32_t v) { *p = v; }
    static void gstore4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) { p[0] = a; p[1] = b; p[2] = c; p[3] = d; }
    static void lds_add(uint32_t* p, uint32_t v) { *p += v; }
    static void gadd64(uint64_t* p, uint64_t v) { *p += v; }
};

// the workgroup flavour (S = 64*NW lanes): same collectives as GroupHip in bftsim.hip
template <int NW>
struct EmuGroup {
    uint64_t* slot = nullptr;    // the LDS group area (Layout::GRP_OFF), as GroupHip
    void init(uint8_t* p) { slot = (uint64_t*)p; }
    uint64_t* summary() const { return slot + 8 + 2 * 64; }
    static uint32_t lane() { return (uint32_t)g->cur; }
    bft::Bits<NW> ballot(bool p) {
        collective(1, p ? 1 : 0);
        bft::Bits<NW> r;
        for (int k = 0; k < NW; ++k) r.w[k] = g->res4[k];
        return r;
    }
    uint32_t bcast(uint32_t v, uint32_t j) { return (uint32_t)collective(5, (uint64_t)v | ((uint64_t)j << 32)); }
    uint32_t grp_max(uint32_t v) { return (uint32_t)collective(6, v); }
    uint32_t grp_or(uint32_t v) { return (uint32_t)collective(7, v); }
    uint64_t grp_sum64(uint32_t v) { return collective(8, v); }
    void sync() { collective(3, 0); }
    template <int K> void ballot_k(const bool (&p)[K], bft::Bits<NW> (&out)[K]) {
        for (int k = 0; k < K; ++k) out[k] = ballot(p[k]);
    }
    template <int K> void ballot_k_store(const bool (&p)[K], uint64_t* dst) {
        bft::Bits<NW> r[K];
        for (int k = 0; k < K; ++k) r[k] = ballot(p[k]);
        if (lane() == 0)
            for (int k = 0; k < K; ++k)
                for (int w = 0; w < NW; ++w) dst[k * NW + w] = r[k].w[w];
        sync();
    }
    // one gather per word: the value of the (unique) writing lane, 0 if none
    template <int K> void gather_k(const bool (&wr)[K], const uint32_t (&v)[K], uint32_t (&out)[K]) {
        for (int k = 0; k < K; ++k) out[k] = (uint32_t)collective(9, (uint64_t)v[k] | ((uint64_t)(wr[k] ? 1u : 0u) << 32));
    }
    static uint64_t clock() { return 0; }
    static uint32_t gload(const uint32_t* p) { return *p; }
    static void gstore(uint32_t* p, uint32_t v) { *p = v; }
    static void gstore4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) { p[0] = a; p[1] = b; p[2] = c; p[3] = d; }
    static void lds_add(uint32_t* p, uint32_t v) { *p += v; }
    static void gadd64(uint64_t* p, uint64_t v) { *p += v; }
};

template <bool NS, uint32_t S>
void run_sim() {
    if constexpr (S == 64) {
        if (g->fast) {                     // bft_consensus_fast_kernel (SEEDED = NS: little-endian seeds)
            if (g->P->thr16 == 0 && g->P->crash_on == 0) {   // the lossless build, as launch_fast picks
                bft::Fast64<EmuWave, false, NS> sim(*g->P, g->lds, g->wave);
                sim.run();
            } else {
                bft::Fast64<EmuWave, true, NS> sim(*g->P, g->lds, g->wave);
                sim.run();
            }
            return;
        }
        if (g->P->resume_mode) {           // bft_consensus_resume_kernel
            bft::Sim<EmuWave, NS, 64, bft::MODE_RESUME> sim(*g->P, g->lds, g->wave);
            sim.run();
            return;
        }
    }
    // as libbftsim: the opt-in modes (replay, crypto) run the MODE_EXT build of the kernel body
    const bool ext = g->P->backlog_replay || g->P->mlog;
    if constexpr (S > 64) {
        if (ext) { bft::Sim<EmuGroup<(int)(S / 64)>, NS, S, bft::MODE_EXT> sim(*g->P, g->lds, g->wave); sim.run(); }
        else { bft::Sim<EmuGroup<(int)(S / 64)>, NS, S> sim(*g->P, g->lds, g->wave); sim.run(); }
    } else {
        if (ext) { bft::Sim<EmuWave, NS, S, bft::MODE_EXT> sim(*g->P, g->lds, g->wave); sim.run(); }
        else { bft::Sim<EmuWave, NS, S> sim(*g->P, g->lds, g->wave); sim.run(); }
    }
}
template <bool NS>
void run_sim_s(uint32_t seg) {
    switch (seg) {
        case 4: run_sim<NS, 4>(); break;
        case 8: run_sim<NS, 8>(); break;
        case 16: run_sim<NS, 16>(); break;
        case 32: run_sim<NS, 32>(); break;
        case 128: run_sim<NS, 128>(); break;
        case 256: run_sim<NS, 256>(); break;
        default: run_sim<NS, 64>(); break;
    }
}
void run_sim_seg(bool ns, uint32_t seg) {
    if (ns) run_sim_s<true>(seg);
    else run_sim_s<false>(seg);
}

void lane_entry(int lane) {
    if (g->body) g->body(lane);
    else run_sim_seg(g->P->need_seed != 0, g->P->seg);
    g->done[lane] = true;
    g->op[lane] = 0;
}

int run_wave(const bft::Params& P, uint32_t wave, std::vector<uint8_t>& lds, int nl = 64, bool fast = false,
             void (*body)(int) = nullptr) {
    static thread_local Sched s;
    g = &s;
    s.fast = fast;
    s.body = body;
    s.nl = nl;
    s.P = &P;
    s.lds = lds.data();
    s.wave = wave;
    for (int l = 0; l < nl; ++l) {
        s.done[l] = false;
        s.op[l] = 0;
        s.seq[l] = 0;
        s.stack[l].resize(256 * 1024);
        getcontext(&s.ctx[l]);
        s.ctx[l].uc_stack.ss_sp = s.stack[l].data();
        s.ctx[l].uc_stack.ss_size = s.stack[l].size();
        s.ctx[l].uc_link = &s.main_ctx;
        makecontext(&s.ctx[l], (void (*)())lane_entry, 1, l);
    }
    for (;;) {
        for (int l = 0; l < nl; ++l) {
            if (s.done[l]) continue;
            s.cur = l;
            swapcontext(&s.main_ctx, &s.ctx[l]);
        }
        int nd = 0;
        for (int l = 0; l < nl; ++l) nd += s.done[l];
        if (nd == nl) break;
        if (nd != 0) { fprintf(stderr, "emu: lanes diverged at a collective (%d done)\n", nd); return -1; }
        int op = s.op[0];
        for (int l = 1; l < nl; ++l)
            if (s.op[l] != op || s.seq[l] != s.seq[0]) {
                fprintf(stderr, "emu: non-uniform collective (lane %d op %d seq %llu vs op %d seq %llu)\n", l, s.op[l],
                        (unsigned long long)s.seq[l], op, (unsigned long long)s.seq[0]);
                return -1;
            }
        if (op == 1) {
            uint64_t m4[4] = {0, 0, 0, 0};
            for (int l = 0; l < nl; ++l) m4[l >> 6] |= (s.arg[l] & 1ull) << (l & 63);
            for (int k = 0; k < 4; ++k) s.res4[k] = m4[k];
            for (int l = 0; l < nl; ++l) s.res[l] = m4[0];
        } else if (op == 5) {
            uint32_t j = (uint32_t)(s.arg[0] >> 32);
            for (int l = 1; l < nl; ++l)
                if ((uint32_t)(s.arg[l] >> 32) != j) { fprintf(stderr, "emu: non-uniform bcast source\n"); return -1; }
            for (int l = 0; l < nl; ++l) s.res[l] = (uint32_t)s.arg[j];
        } else if (op == 9) {                 // gather: the writing lane's value (more than one: abort)
            int wl = -1;
            for (int l = 0; l < nl; ++l)
                if (s.arg[l] >> 32) {
                    if (wl >= 0) { fprintf(stderr, "emu: two writers of one gathered word\n"); return -1; }
                    wl = l;
                }
            for (int l = 0; l < nl; ++l) s.res[l] = wl >= 0 ? (uint32_t)s.arg[wl] : 0u;
        } else if (op >= 6 && op <= 8) {
            uint64_t r = 0;
            for (int l = 0; l < nl; ++l) {
                uint64_t v = (uint32_t)s.arg[l];
                if (op == 6) r = v > r ? v : r;
                else if (op == 7) r |= v;
                else r += v;
            }
            for (int l = 0; l < nl; ++l) s.res[l] = r;
        } else if (op == 10) {               // keccak_pair: every lane pair's 64-bit state, permuted
            for (int l = 0; l < nl; l += 2) {
                uint32_t* lo = (uint32_t*)(uintptr_t)s.arg[l];
                uint32_t* hi = (uint32_t*)(uintptr_t)s.arg[l + 1];
                uint64_t a[25];
                for (int i = 0; i < 25; ++i) a[i] = (uint64_t)lo[i] | ((uint64_t)hi[i] << 32);
                bft::keccak_f1600_u64(a);
                for (int i = 0; i < 25; ++i) { lo[i] = (uint32_t)a[i]; hi[i] = (uint32_t)(a[i] >> 32); }
            }
        } else if (op == 4) {
            for (int l = 0; l < 64; ++l) s.res[l] = (uint32_t)s.arg[(int)(s.arg[l] >> 32)];
        } else if (op == 2) {
            for (int l = 0; l < 64; ++l) {
                int mm = (int)(s.arg[l] >> 32);
                s.res[l] = (uint32_t)s.arg[l ^ mm];
            }
        }
    }
    g = nullptr;
    return 0;
}

}  // namespace

// windowed run (bftsim_set_window): per-instance outputs, tip hashes and the histograms
extern "C" int emu_run_stream(const bftsim_config* cfg, uint64_t first, uint64_t n, uint32_t window,
                              uint32_t* committed, uint32_t* flags_out, uint32_t* ticks_out, uint64_t* views_out,
                              uint8_t* tips, uint64_t* hist) {
    if (cfg->n < 1 || cfg->n > 256 || window < 64 || (window & (window - 1))) return -4;
    uint8_t gh[32];
    bft::host_genesis_hash(cfg, gh);
    uint32_t gseed = bft::seed_from_hash(gh, cfg->n, cfg->seed_byte_order == BFTSIM_SEED_LE);
    uint32_t seg = bft::segment_size(cfg->n);
    bft::Params P = bft::params_from_config(*cfg, seg, cfg->heights + 64, gseed, first, n);
    P.window_mask = window - 1;
    P.rows = window;
    P.need_seed = 1;
    std::vector<uint32_t> rec((size_t)n * window * 4, 0);
    std::vector<uint8_t> hs((size_t)n * window * 32, 0);
    for (int b = 0; b < (int)bft::HIST_BINS; ++b) hist[b] = 0;
    P.addresses = cfg->addresses;
    P.genesis_hash = gh;
    P.committed_height = committed;
    P.flags = flags_out;
    P.ticks = ticks_out;
    P.views = views_out;
    P.rec = rec.data();
    P.hash = hs.data();
    P.hist = hist;
    uint32_t per_wave = seg > 64 ? 1 : 64 / seg;
    uint32_t waves = (uint32_t)((n + per_wave - 1) / per_wave);
    std::vector<uint8_t> lds(bft::lds_bytes(seg, true));
    if (const char* e = getenv("BFT_EMU_RCS_K")) P.rcs_k = (uint32_t)atoi(e);   // RoundChangeSet capacity
    std::vector<uint32_t> rcs((size_t)waves * bft::rcs_words(seg, P.rcs_k), 0xcdcdcdcdu);
    P.rcs = rcs.data();
    std::vector<uint32_t> backlog(P.backlog_replay ? (size_t)waves * bft::backlog_words(seg) : 0, 0);
    P.backlog = P.backlog_replay ? backlog.data() : nullptr;
    for (uint32_t w = 0; w < waves; ++w) {
        memset(lds.data(), 0xcd, lds.size());
        if (run_wave(P, w, lds, seg > 64 ? (int)seg : 64)) return -1;
    }
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t ch = committed[i];
        const uint8_t* src = ch == 0 ? gh : &hs[(i * window + (ch & (window - 1))) * 32];
        memcpy(tips + i * 32, src, 32);
    }
    return 0;
}

// real-crypto mode for the next emu_run (SPEC.md §11): forged senders + the broadcast log
static const uint64_t* g_forged = nullptr;
static uint32_t *g_mlog = nullptr, *g_mlog_n = nullptr;
static uint32_t g_mlog_cap = 0;
extern "C" void emu_set_crypto(const uint64_t* forged, uint32_t* mlog, uint32_t* mlog_n, uint32_t cap) {
    g_forged = forged; g_mlog = mlog; g_mlog_n = mlog_n; g_mlog_cap = cap;
}

extern "C" int emu_run(const bftsim_config* cfg, uint64_t first, uint64_t n, bftsim_result* out,
                       uint64_t* trace, uint32_t trace_ticks, uint64_t* hist) {
    if (cfg->n < 1 || cfg->n > 256) return -4;
    uint8_t gh[32];
    bft::host_genesis_hash(cfg, gh);
    uint32_t gseed = bft::seed_from_hash(gh, cfg->n, cfg->seed_byte_order == BFTSIM_SEED_LE);
    uint32_t seg = bft::segment_size(cfg->n);
    uint32_t hcap = cfg->heights + 64;
    bft::Params P = bft::params_from_config(*cfg, seg, hcap, gseed, first, n);
    if (getenv("BFT_EMU_SLOW")) P.fast = 0;
    if (g_mlog) {
        P.mlog = g_mlog; P.mlog_n = g_mlog_n; P.mlog_cap = g_mlog_cap;
        for (int k = 0; k < 4; ++k) P.forged[k] = g_forged[k];
        P.fast = 0;                                        // as libbftsim in real-crypto mode
        g_mlog = nullptr;                                  // one run
    }
    std::vector<uint32_t> ch(n), flags(n), ticks(n);
    std::vector<uint64_t> views(n);
    std::vector<uint32_t> rec(n * hcap * 4, 0);
    std::vector<uint8_t> hs(n * hcap * 32, 0);
    P.addresses = cfg->addresses;
    P.genesis_hash = gh;
    P.committed_height = ch.data();
    P.flags = flags.data();
    P.ticks = ticks.data();
    P.views = views.data();
    P.rec = rec.data();
    P.hash = hs.data();
    P.trace = trace;
    P.trace_ticks = trace ? trace_ticks : 0;
    P.hist = hist;
    if (hist) for (int b = 0; b < (int)bft::HIST_BINS; ++b) hist[b] = 0;
    uint32_t per_wave = seg > 64 ? 1 : 64 / seg;
    uint32_t waves = (uint32_t)((n + per_wave - 1) / per_wave);
    std::vector<uint8_t> lds(bft::lds_bytes(seg, P.need_seed != 0));
    if (const char* e = getenv("BFT_EMU_RCS_K")) P.rcs_k = (uint32_t)atoi(e);   // RoundChangeSet capacity
    std::vector<uint32_t> rcs((size_t)waves * bft::rcs_words(seg, P.rcs_k), 0xcdcdcdcdu);
    P.rcs = rcs.data();
    std::vector<uint32_t> backlog(P.backlog_replay ? (size_t)waves * bft::backlog_words(seg) : 0, 0);
    P.backlog = P.backlog_replay ? backlog.data() : nullptr;
    // as libbftsim: N = 64 runs the FAST kernel, then the full kernel resumes the instances it handed
    // over (BFT_EMU_FAST=0: the full kernel alone)
    const char* ef = getenv("BFT_EMU_FAST");
    const bool fast = seg == 64 && cfg->n == 64 && P.fast && !P.mlog && !trace && !(ef && strcmp(ef, "0") == 0);
    std::vector<uint32_t> resume, save;
    if (fast) {
        resume.assign(n, 0);
        save.assign((size_t)n * 64 * bft::SAVE_WORDS, 0xcdcdcdcdu);
        P.resume_flags = resume.data();
        P.save = save.data();
        // little-endian seeds: the seed chain's predicted blocks first (kern_fast.hip bft_seed_chain_kernel, here
        // with the one-piece header encoder; BFT_EMU_SPEC=0: none, the wave hashes every height)
        std::vector<uint32_t> spec;
        const char* es = getenv("BFT_EMU_SPEC");
        if (P.need_seed && !(es && strcmp(es, "0") == 0)) {
            spec.assign((size_t)(cfg->heights + 1) * n, 0xcdcdcdcdu);
            P.spec = spec.data();
            for (uint64_t il = 0; il < n; ++il) {
                const uint32_t inst = (uint32_t)(first + il);
                uint8_t perm[64];
                const uint64_t byz = bft::byz_mask64(P.seed, inst, P.byz_count, perm);
                uint32_t prev[8];
                for (int i = 0; i < 8; ++i)
                    prev[i] = (uint32_t)gh[4 * i] | ((uint32_t)gh[4 * i + 1] << 8) | ((uint32_t)gh[4 * i + 2] << 16) |
                              ((uint32_t)gh[4 * i + 3] << 24);
                for (uint32_t x = 1; x <= cfg->heights; ++x) {
                    uint32_t j, var;
                    if (!bft::spec_block64(P.seed, inst, x, byz, prev[0], j, var)) { spec[(size_t)x * n + il] = 0; break; }
                    alignas(8) uint8_t buf[bft::LANE_HASH_BUF];
                    uint32_t out[8];
                    bft::lane_block_hash(buf, prev, cfg->addresses + 20u * j, P.seed, inst, x, j, var,
                                         cfg->genesis_time + (uint64_t)cfg->block_period * x, out);
                    memcpy(&hs[(il * hcap + x) * 32], out, 32);
                    for (int i = 0; i < 8; ++i) prev[i] = out[i];
                    spec[(size_t)x * n + il] = bft::spec_word(j, var, bft::seed_from_words(out[0], out[1], 64, true));
                }
            }
        }
        std::vector<uint8_t> lds_fast(bft::lds_bytes_fast64(P.need_seed != 0));   // the FAST kernel's exact LDS size
        for (uint32_t w = 0; w < waves; ++w) {
            memset(lds_fast.data(), 0xcd, lds_fast.size());
            if (run_wave(P, w, lds_fast, 64, true)) return -1;
        }
        P.spec = nullptr;                                  // read by the FAST kernel only
        P.resume_mode = 1;
    }
    for (uint32_t w = 0; w < waves; ++w) {
        memset(lds.data(), 0xcd, lds.size());
        if (run_wave(P, w, lds, seg > 64 ? (int)seg : 64)) return -1;
    }
    P.resume_mode = 0;
    // invariant of the in-kernel hashes (segments of S < 64 lanes, whose canonical rows a deferred hash patches
    // after they are recorded): every recorded row's seed word is the seed of its hash row
    if (P.need_seed && seg < 64) {
        for (uint64_t i = 0; i < n; ++i)
            for (uint32_t x = 1; x <= ch[i] && x < hcap; ++x) {
                uint32_t w[2];
                memcpy(w, &hs[(i * hcap + x) * 32], 8);
                if (rec[(i * hcap + x) * 4 + 3] != bft::seed_from_words(w[0], w[1], cfg->n, cfg->seed_byte_order == BFTSIM_SEED_LE))
                    return -7;
            }
    }
    if (fast && getenv("BFT_EMU_FAST_REPORT")) {
        uint64_t nb = 0;
        for (uint64_t i = 0; i < n; ++i) nb += resume[i];
        fprintf(stderr, "emu: FAST handed over %llu of %llu instances\n", (unsigned long long)nb, (unsigned long long)n);
    }
    // the hash post-pass, as kern_fast.hip splits it: every height's header suffix first
    // (bft_hash_suffix_kernel), then the chain, splicing prev_hash in front (bft_hash_chain_kernel)
    if (!P.need_seed) {
        uint32_t sfx[bft::SFX_DWORDS];
        for (uint64_t il = 0; il < n; ++il) {
            uint32_t prev[8];
            for (int i = 0; i < 8; ++i)
                prev[i] = (uint32_t)gh[4 * i] | ((uint32_t)gh[4 * i + 1] << 8) | ((uint32_t)gh[4 * i + 2] << 16) |
                          ((uint32_t)gh[4 * i + 3] << 24);
            for (uint32_t x = 1; x <= ch[il]; ++x) {
                const uint32_t* row = &rec[(il * hcap + x) * 4];
                uint32_t prop = row[1] & 0xffffu, var = (row[1] >> 16) & 1u;
                uint64_t time = cfg->genesis_time + (uint64_t)cfg->block_period * ((uint64_t)row[2] + 1ull);
                uint32_t out[8];
                bft::header_suffix((uint64_t*)sfx, cfg->addresses + 20u * prop, cfg->seed, (uint32_t)(first + il), x,
                                   prop, var, time);
                bft::spliced_block_hash(sfx, prev, out);
                memcpy(&hs[(il * hcap + x) * 32], out, 32);
                for (int i = 0; i < 8; ++i) prev[i] = out[i];
            }
        }
    }
    uint32_t H = cfg->heights;
    for (uint64_t i = 0; i < n; ++i) {
        out->committed_height[i] = ch[i];
        out->flags[i] = flags[i];
        out->ticks[i] = ticks[i];
        out->views[i] = views[i];
        for (uint32_t x = 1; x <= H; ++x) {
            uint64_t o = i * H + (x - 1);
            const uint32_t* row = &rec[(i * hcap + x) * 4];
            bool ok = x <= ch[i];
            out->round[o] = ok ? (uint16_t)row[0] : 0;
            out->proposer[o] = ok ? (uint16_t)(row[1] & 0xffffu) : 0;
            out->variant[o] = ok ? (uint8_t)((row[1] >> 16) & 1u) : 0;
            out->time_tick[o] = ok ? row[2] : 0;
            if (ok) memcpy(out->block_hash + o * 32, &hs[(i * hcap + x) * 32], 32);
            else memset(out->block_hash + o * 32, 0, 32);
        }
    }
    return 0;
}

// philox_drop (deliver_mask's draw, products of uniform words hoisted) against philox on random counters,
// including the largest phase / receiver / block fields. Returns mismatches.
extern "C" int emu_philox_drop_check(uint32_t trials, uint64_t seed) {
    uint64_t s = seed | 1ull;
    auto nxt = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    int bad = 0;
    for (uint32_t t = 0; t < trials; ++t) {
        const uint64_t key = nxt();
        const uint32_t inst = (uint32_t)nxt(), tick = (uint32_t)nxt();
        const uint32_t phase = t < 8 ? 255u - t : (uint32_t)nxt() & 255u, recv = t < 8 ? 255u : (uint32_t)nxt() & 255u;
        const uint32_t j = t < 8 ? 31u : (uint32_t)nxt() & 31u;
        uint32_t a[4], b[4];
        bft::philox(key, inst, tick, (phase << 24) | (recv << 8) | j, bft::DOM_DROP, a);
        bft::philox_drop(key, inst, tick, bft::philox_drop_base(phase, recv), j, b);
        if (memcmp(a, b, sizeof a) != 0) ++bad;
    }
    return bad;
}

// The splice of the block-hash pass against the one-piece encoder: `trials` random headers (random parent
// hashes, proposers, variants, heights and times), including parents with every byte >= 128 or < 128 (the
// longest and shortest prefixes) and heights / times at MessagePack width boundaries. Returns mismatches.
extern "C" int emu_splice_check(uint32_t trials, uint64_t seed) {
    uint64_t s = seed | 1ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    std::vector<uint8_t> addr(64 * 20);
    for (auto& b : addr) b = (uint8_t)rnd();
    int bad = 0;
    alignas(16) uint8_t buf[bft::LANE_HASH_BUF];
    uint32_t sfx[bft::SFX_DWORDS];
    const uint64_t times[] = {0ull, 127ull, 128ull, 255ull, 256ull, 65535ull, 65536ull, 4294967295ull, 4294967296ull, ~0ull};
    const uint32_t heights[] = {1u, 127u, 128u, 255u, 256u, 65535u, 65536u, 4294967295u};
    for (uint32_t t = 0; t < trials; ++t) {
        uint32_t prev[8];
        for (int i = 0; i < 8; ++i) {
            uint32_t v = (uint32_t)rnd();
            if (t % 4 == 1) v |= 0x80808080u;
            if (t % 4 == 2) v &= 0x7f7f7f7fu;
            prev[i] = v;
        }
        const uint32_t prop = (uint32_t)(rnd() % 64), var = (uint32_t)(rnd() & 1), inst = (uint32_t)rnd();
        const uint32_t h = (t % 3 == 0) ? heights[rnd() % 8] : (uint32_t)rnd();
        const uint64_t time = (t % 3 == 1) ? times[rnd() % 10] : rnd();
        uint32_t a[8], b[8];
        bft::lane_block_hash(buf, prev, addr.data() + 20u * prop, s, inst, h, prop, var, time, a);
        bft::header_suffix((uint64_t*)sfx, addr.data() + 20u * prop, s, inst, h, prop, var, time);
        bft::spliced_block_hash(sfx, prev, b);
        if (memcmp(a, b, 32) != 0) ++bad;
        // the device layout (dword k of the row at k * stride): the same body and length
        uint32_t strided[bft::SFX_DEV_DW * 3];
        for (auto& v : strided) v = 0xdeadbeefu;
        const uint32_t ls = bft::header_suffix_strided(strided + 1, 3, addr.data() + 20u * prop, s, inst, h, prop, var, time);
        bool same = ls == sfx[bft::SFX_LEN_DW] && strided[1 + 3 * bft::SFX_DEV_LEN_DW] == ls;
        for (uint32_t k = 0; k < bft::SFX_BODY_DW; ++k) same = same && strided[1 + 3 * k] == sfx[k];
        if (!same) ++bad;
    }
    return bad;
}

// The small-shard chain kernel's body (bft_kwave.h kw50_chain: one wave per instance, the 50-lane Keccak,
// the prefix written byte-wise by the lanes) over random chains: each chain's hashes against the lane
// splice of spliced_block_hash from the same suffix rows. Returns mismatching heights.
namespace {
struct ChainJob {
    const uint32_t* srow; uint64_t rstride; uint32_t stride; uint32_t parent[8]; uint32_t nx; uint32_t* hdst;
    uint32_t* sb; uint32_t* pf;
};
thread_local ChainJob* g_chain = nullptr;
void chain_body(int lane) {
    EmuWave wv;
    ChainJob& j = *g_chain;
    bft::kw50_chain(wv, (uint32_t)lane, j.sb, j.pf, j.srow, j.rstride, j.stride, lane < 8 ? j.parent[lane] : 0u, j.nx,
                    j.hdst);
}
}  // namespace
extern "C" int emu_wave_chain_check(uint32_t chains, uint32_t heights, uint64_t seed) {
    uint64_t s = seed | 1ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    std::vector<uint8_t> addr(64 * 20);
    for (auto& b : addr) b = (uint8_t)rnd();
    const uint32_t stride = 3;                        // 3 instances per row table: dword k of the row at k * 3
    const uint64_t rstride = (uint64_t)bft::SFX_DEV_DW * stride;
    std::vector<uint32_t> rows(rstride * heights + stride, 0xdeadbeefu), host(bft::SFX_DWORDS);
    std::vector<uint32_t> hd(8ull * heights), sb(bft::SFX_BUF + 8), pf(bft::KW_PFX_DW + 2);
    const uint64_t times[] = {0ull, 127ull, 128ull, 255ull, 256ull, 65535ull, 65536ull, 4294967295ull, 4294967296ull};
    int bad = 0;
    std::vector<uint8_t> lds;
    bft::Params P{};
    for (uint32_t c = 0; c < chains; ++c) {
        ChainJob job{};
        uint32_t want[8], prev[8];
        for (int i = 0; i < 8; ++i) {                 // the parent: all-high, all-low or random bytes
            uint32_t v = (uint32_t)rnd();
            if (c % 4 == 1) v |= 0x80808080u;
            if (c % 4 == 2) v &= 0x7f7f7f7fu;
            job.parent[i] = prev[i] = v;
        }
        const uint32_t inst = (uint32_t)rnd(), h0 = (c % 3 == 0) ? 120u + (uint32_t)(rnd() % 20) : (uint32_t)rnd() % 70000u;
        for (uint32_t j = 0; j < heights; ++j) {
            const uint32_t prop = (uint32_t)(rnd() % 64), var = (uint32_t)(rnd() & 1);
            const uint64_t time = (c % 3 == 1) ? times[rnd() % 9] : rnd() >> (rnd() % 64);
            bft::header_suffix_strided(rows.data() + rstride * j + 1, stride, addr.data() + 20u * prop, s, inst, h0 + j,
                                       prop, var, time);
        }
        job.srow = rows.data() + 1; job.rstride = rstride; job.stride = stride; job.nx = heights;
        for (auto& v : hd) v = 0;
        job.hdst = hd.data(); job.sb = sb.data(); job.pf = pf.data();
        g_chain = &job;
        if (run_wave(P, 0, lds, 64, false, chain_body)) return -1;
        g_chain = nullptr;
        for (uint32_t j = 0; j < heights; ++j) {
            for (uint32_t k = 0; k < bft::SFX_BODY_DW; ++k) host[k] = rows[1 + rstride * j + (uint64_t)k * stride];
            host[bft::SFX_LEN_DW] = rows[1 + rstride * j + (uint64_t)bft::SFX_DEV_LEN_DW * stride];
            bft::spliced_block_hash(host.data(), prev, want);
            if (memcmp(want, &hd[8ull * j], 32) != 0) ++bad;
            memcpy(prev, want, 32);
        }
    }
    return bad;
}
