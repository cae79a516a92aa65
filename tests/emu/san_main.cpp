// san_main.cpp — TEST-ONLY sanitizer build of the CPU parity check (tests/test_sanitizers.py).
// One executable: the oracle (oracle/bft_oracle.c, linked from its own -fsanitize=address,undefined objects)
// and the wave emulator running the kernel bodies (this translation unit includes wave_emu.cpp), both built
// with AddressSanitizer + UndefinedBehaviorSanitizer. No Python in the process, so no sanitizer runtime has to
// be preloaded. Reads one configuration per stdin line:
//   n heights max_ticks seed drop_ppm byz crash_ppm phase_cap silent0..3 seed_order backlog first n_inst window addrhex
// window 0 compares emu_run with orc_run (every per-height row), window > 0 emu_run_stream with orc_run_stream
// (windowed rows, tip hashes, histograms). Prints "ok <line>" or "MISMATCH <line> <field>"; exit status = the
// number of mismatches (capped at 100), or 200 on a malformed line.
#include "wave_emu.cpp"
#include "../../oracle/bft_oracle.h"

#include <string>

static int hexval(char c) {
    return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
}

template <class T>
static bool same(const std::vector<T>& a, const std::vector<T>& b) { return a == b; }

int main() {
    char line[1 << 14];
    int bad = 0, k = 0;
    while (fgets(line, sizeof line, stdin)) {
        ++k;
        unsigned long long v[17];
        char hex[10320];
        int got = sscanf(line, "%llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %10300s",
                         &v[0], &v[1], &v[2], &v[3], &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12],
                         &v[13], &v[14], &v[15], &v[16], hex);
        if (got != 18) { fprintf(stderr, "san: malformed line %d\n", k); return 200; }
        const uint32_t n = (uint32_t)v[0];
        if (n < 1 || n > 256 || strlen(hex) != 40u * n) { fprintf(stderr, "san: bad validator set on line %d\n", k); return 200; }
        std::vector<uint8_t> addr(20u * n);
        for (uint32_t i = 0; i < 20u * n; ++i) addr[i] = (uint8_t)(hexval(hex[2 * i]) * 16 + hexval(hex[2 * i + 1]));
        bftsim_config c{};
        c.n = n; c.heights = (uint32_t)v[1]; c.max_ticks = (uint32_t)v[2]; c.block_period = 3;
        c.genesis_time = 1536517089ull; c.seed = v[3]; c.drop_ppm = (uint32_t)v[4]; c.byz_count = (uint32_t)v[5];
        c.proposer_crash_ppm = (uint32_t)v[6]; c.phase_cap = (uint32_t)v[7];
        for (int i = 0; i < 4; ++i) c.silent_mask[i] = v[8 + i];
        c.addresses = addr.data();
        static const uint8_t gp[20] = {0x57, 0x01, 0xfb, 0xd0, 0x5e, 0x77, 0xca, 0xc0, 0x03, 0xa6,
                                       0x89, 0x4e, 0x4b, 0x2a, 0x3c, 0x12, 0x28, 0x7e, 0xd3, 0x13};
        memcpy(c.genesis_proposer, gp, 20);
        c.genesis_gas_used = 10000;
        c.seed_byte_order = (uint32_t)v[12];
        c.backlog_mode = (uint32_t)v[13];
        orc_config o{};
        o.n = c.n; o.heights = c.heights; o.max_ticks = c.max_ticks; o.block_period = c.block_period;
        o.genesis_time = c.genesis_time; o.seed = c.seed; o.drop_ppm = c.drop_ppm; o.byz_count = c.byz_count;
        o.proposer_crash_ppm = c.proposer_crash_ppm; o.phase_cap = c.phase_cap;
        for (int i = 0; i < 4; ++i) o.silent_mask[i] = c.silent_mask[i];
        o.addresses = addr.data();
        memcpy(o.genesis_proposer, gp, 20);
        o.genesis_gas_used = c.genesis_gas_used; o.seed_byte_order = c.seed_byte_order; o.backlog_mode = c.backlog_mode;
        const uint64_t first = v[14], ni = v[15];
        const uint32_t window = (uint32_t)v[16], H = c.heights;
        std::string what;
        if (window == 0) {
            std::vector<uint64_t> ech(ni), eviews(ni), oviews(ni);
            std::vector<uint32_t> och(ni), eflags(ni), oflags(ni), eticks(ni), oticks(ni), ett(ni * H), ott(ni * H);
            std::vector<uint16_t> ern(ni * H), orn(ni * H), epr(ni * H), opr(ni * H);
            std::vector<uint8_t> eva(ni * H), ova(ni * H), eh(ni * H * 32), oh(ni * H * 32);
            bftsim_result er{ech.data(), eflags.data(), eticks.data(), eviews.data(), ern.data(), epr.data(), eva.data(),
                             ett.data(), eh.data(), ni};
            orc_result orr{och.data(), oflags.data(), oticks.data(), oviews.data(), orn.data(), opr.data(), ova.data(),
                           ott.data(), oh.data()};
            if (emu_run(&c, first, ni, &er, nullptr, 0, nullptr) != 0) what = "emu_run failed";
            else if (orc_run(&o, first, ni, &orr) != 0) what = "orc_run failed";
            else {
                for (uint64_t i = 0; i < ni && what.empty(); ++i)
                    if (ech[i] != och[i]) what = "committed_height";
                if (what.empty() && !same(eflags, oflags)) what = "flags";
                if (what.empty() && !same(eticks, oticks)) what = "ticks";
                if (what.empty() && !same(eviews, oviews)) what = "views";
                if (what.empty() && !same(ern, orn)) what = "round";
                if (what.empty() && !same(epr, opr)) what = "proposer";
                if (what.empty() && !same(eva, ova)) what = "variant";
                if (what.empty() && !same(ett, ott)) what = "time_tick";
                if (what.empty() && !same(eh, oh)) what = "block_hash";
            }
        } else {
            std::vector<uint32_t> ech(ni), och(ni), ef(ni), of(ni), et(ni), ot(ni);
            std::vector<uint64_t> ev(ni), ov(ni), ehist(130);
            std::vector<uint8_t> etip(ni * 32), otip(ni * 32);
            orc_stream os{och.data(), of.data(), ot.data(), ov.data(), otip.data(), {}};
            if (emu_run_stream(&c, first, ni, window, ech.data(), ef.data(), et.data(), ev.data(), etip.data(),
                               ehist.data()) != 0) what = "emu_run_stream failed";
            else if (orc_run_stream(&o, first, ni, &os, 1) != 0) what = "orc_run_stream failed";
            else {
                if (!same(ech, och)) what = "committed_height";
                if (what.empty() && !same(ef, of)) what = "flags";
                if (what.empty() && !same(et, ot)) what = "ticks";
                if (what.empty() && !same(ev, ov)) what = "views";
                if (what.empty() && !same(etip, otip)) what = "tip_hash";
                if (what.empty() && memcmp(ehist.data(), os.hist, sizeof os.hist) != 0) what = "histograms";
            }
        }
        if (what.empty()) printf("ok %d\n", k);
        else { printf("MISMATCH %d %s\n", k, what.c_str()); ++bad; }
        fflush(stdout);
    }
    return bad > 100 ? 100 : bad;
}
