// kern_general.hip — the general consensus kernel (bft_wave.h `Sim`), one build per
// (NEED_SEED, MODE) pair: the Makefile compiles this file with -DGEN_SEED={0,1} -DGEN_MODE={0,1}
// (MODE_FULL / MODE_EXT) into four objects.
#include "bft_hip.h"

#ifndef GEN_SEED
#error "compile with -DGEN_SEED=0|1 -DGEN_MODE=0|1"
#endif

namespace bft {

#ifndef BFT_WAVES_PER_SIMD
#define BFT_WAVES_PER_SIMD 3   // register budget of the one-wave kernels (LDS allows ~2.75 per SIMD)
#endif
// occupancy target of the segment kernels (S = 128 / 256 lanes per instance; the launch bound's second
// argument, which the compiler turns into waves per SIMD). With 1 the S = 256 body got 256 VGPRs + 46
// AGPRs, one wave per SIMD, and a CU waited on one instance's barriers; 2 runs cfg4 N = 256 1.65x
// faster. S = 128: 2 (208 VGPRs, no spills) runs 1.63x faster than 4 (128 VGPRs, 376 B/lane spills).
// (profiles/r03/ab_occupancy)
#ifndef BFT_WG_PER_CU_256
#define BFT_WG_PER_CU_256 2
#endif
#ifndef BFT_WG_PER_CU_128
#define BFT_WG_PER_CU_128 2
#endif
// several instances per wave with in-kernel hashes (S < 64, N not a power of two or little-endian seeds: cfg5):
// the header hash needs registers beside the validator state (3 waves per SIMD: 168 VGPRs + 264 B/lane of
// scratch, 207 GB of spill writes per cfg5 launch; 2: 240 VGPRs, none: cfg5 1.80e8 -> 1.93e8, profiles/r05/ab_cfg5)
#ifndef BFT_SEED_WAVES_PER_SIMD
#define BFT_SEED_WAVES_PER_SIMD 2
#endif
template <bool NS, uint32_t S>
constexpr int min_blocks_per_cu() {
    return S == 256 ? BFT_WG_PER_CU_256 : S == 128 ? BFT_WG_PER_CU_128 : (NS && S < 64) ? BFT_SEED_WAVES_PER_SIMD
                                                                                       : BFT_WAVES_PER_SIMD;
}

template <bool NEED_SEED, int MODE, uint32_t S>
__global__ __launch_bounds__(S > 64 ? S : 64, (min_blocks_per_cu<NEED_SEED, S>())) void bft_consensus_kernel(Params p) {
    extern __shared__ uint8_t lds[];
    if constexpr (S > 64) {
        Sim<GroupHip<(int)(S / 64)>, NEED_SEED, S, MODE> sim(p, lds, blockIdx.x);
        sim.run();
    } else {
        Sim<WaveHip, NEED_SEED, S, MODE> sim(p, lds, blockIdx.x);
        sim.run();
    }
}

template <bool NEED_SEED, int MODE>
static hipError_t launch_consensus(uint32_t seg, dim3 grid, size_t lds, hipStream_t s, const Params& p) {
    switch (seg) {
        case 128: {
            hipError_t e = hipFuncSetAttribute((const void*)bft_consensus_kernel<NEED_SEED, MODE, 128>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 128>), grid, dim3(128), lds, s, p);
            break;
        }
        case 256: {
            hipError_t e = hipFuncSetAttribute((const void*)bft_consensus_kernel<NEED_SEED, MODE, 256>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 256>), grid, dim3(256), lds, s, p);
            break;
        }
        case 4: hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 4>), grid, dim3(64), lds, s, p); break;
        case 8: hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 8>), grid, dim3(64), lds, s, p); break;
        case 16: hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 16>), grid, dim3(64), lds, s, p); break;
        case 32: hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 32>), grid, dim3(64), lds, s, p); break;
        default: hipLaunchKernelGGL((bft_consensus_kernel<NEED_SEED, MODE, 64>), grid, dim3(64), lds, s, p); break;
    }
    return hipGetLastError();
}

#define BFT_GEN_NAME_(a, b) launch_general_##a##_##b
#define BFT_GEN_NAME(a, b) BFT_GEN_NAME_(a, b)
hipError_t BFT_GEN_NAME(GEN_SEED, GEN_MODE)(uint32_t seg, dim3 grid, size_t lds, hipStream_t s, const Params& p) {
    return launch_consensus<GEN_SEED != 0, GEN_MODE>(seg, grid, lds, s, p);
}

}  // namespace bft
