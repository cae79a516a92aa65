// kern_resume.hip — the full kernel body (bft_wave.h `Sim`, MODE_RESUME) over the instances the
// N = 64 FAST kernel handed over, from their saved phase.
#include "bft_hip.h"

namespace bft {

#ifndef BFT_RESUME_WAVES_PER_SIMD
#define BFT_RESUME_WAVES_PER_SIMD 3
#endif
// the full kernel over the instances the FAST kernel handed over, from their saved phase (NEED_SEED:
// little-endian seeds, block hashes in-kernel)
// Persistent waves over a queue (Params::resume_q, filled by the FAST kernel: count, head, instance ids):
// each wave takes the next handed-over instance until the queue is empty. A wave per instance of the launch
// would dispatch n waves carrying the general body's LDS even when nothing was handed over, and beside the
// concurrent launches' kernels that dispatch alone took ~0.2 ms per launch (cfg3, profiles/r04).
template <bool NEED_SEED>
__global__ __launch_bounds__(64, BFT_RESUME_WAVES_PER_SIMD) void bft_consensus_resume_kernel(Params p) {
    extern __shared__ uint8_t lds[];
    const uint32_t count = __hip_atomic_load(p.resume_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x == 0 && p.resume_hint)
        __hip_atomic_store(p.resume_hint, count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        uint32_t i = 0;
        if (threadIdx.x == 0) i = atomicAdd(p.resume_q + 1, 1u);
        i = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)i, 0, 64));
        if (i >= count) break;                            // every wave gets here once the queue is empty
        Sim<WaveHip, NEED_SEED, 64, MODE_RESUME> sim(p, lds, p.resume_q[2u + i]);
        sim.run();
    }
}
hipError_t launch_resume(dim3 grid, size_t lds, hipStream_t s, const Params& p) {
    // waves that can be resident at once (3 per SIMD): more would only queue for the same slots. Fewer when
    // the host's hint (the count of an earlier launch) says few instances hand over: beside concurrent
    // launches every wave waits for a free slot, and the queue is drained by however many waves there are
    constexpr uint32_t MAXW = 256u * 4u * BFT_RESUME_WAVES_PER_SIMD;
    uint32_t g = grid.x < MAXW ? grid.x : MAXW;
    if (p.resume_hint) {
        const uint32_t hint = __atomic_load_n(p.resume_hint, __ATOMIC_RELAXED);
        const uint32_t want = hint > MAXW / 2u ? MAXW : 2u * hint + 16u;
        g = want < g ? want : g;
    }
    if (p.need_seed) hipLaunchKernelGGL(bft_consensus_resume_kernel<true>, dim3(g), dim3(64), lds, s, p);
    else hipLaunchKernelGGL(bft_consensus_resume_kernel<false>, dim3(g), dim3(64), lds, s, p);
    return hipGetLastError();
}

}  // namespace bft
