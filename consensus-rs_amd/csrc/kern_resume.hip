// kern_resume.hip — the full kernel body (bft_wave.h `Sim`, MODE_RESUME) over the instances the
// N = 64 FAST kernel handed over, from their saved phase.
#include "bft_hip.h"

namespace bft {

#ifndef BFT_WAVES_PER_SIMD
#define BFT_WAVES_PER_SIMD 3
#endif
// the full kernel over the instances the FAST kernel handed over, from their saved phase (NEED_SEED:
// little-endian seeds, block hashes in-kernel)
template <bool NEED_SEED>
__global__ __launch_bounds__(64, BFT_WAVES_PER_SIMD) void bft_consensus_resume_kernel(Params p) {
    extern __shared__ uint8_t lds[];
    Sim<WaveHip, NEED_SEED, 64, MODE_RESUME> sim(p, lds, blockIdx.x);
    sim.run();
}
hipError_t launch_resume(dim3 grid, size_t lds, hipStream_t s, const Params& p) {
    if (p.need_seed) hipLaunchKernelGGL(bft_consensus_resume_kernel<true>, grid, dim3(64), lds, s, p);
    else hipLaunchKernelGGL(bft_consensus_resume_kernel<false>, grid, dim3(64), lds, s, p);
    return hipGetLastError();
}

}  // namespace bft
