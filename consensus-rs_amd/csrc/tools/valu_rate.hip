// valu_rate.hip — wave-instruction issue rate of the chain kernels' VALU mix against the number of resident waves
// (diagnostic): v_xor_b32, v_bitop3_b32, v_alignbit_b32, v_add_u32 in 8 independent chains per lane,
// and the lane Keccak-f[1600] of the lane chain kernel, each over a grid of 1-wave workgroups. Prints one JSON
// line per (op, waves): ms, wave-instructions per second, and cycles per wave-instruction per CU and per wave.
#include "../kern_fast.hip"
#include <stdio.h>

namespace {
template <int OP>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    else if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    else if constexpr (OP == 2) asm volatile("v_alignbit_b32 %0, %1, %2, 7" : "=v"(d) : "v"(a), "v"(b));
    else asm volatile("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}

template <int OP>
__global__ __launch_bounds__(64) void rate_kernel(uint32_t* out, int iters, uint32_t seed) {
    const uint32_t t = blockIdx.x * 64u + threadIdx.x;
    uint32_t x[8];
    const uint32_t b = t * 0x9e3779b9u ^ seed, c = t + seed;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = t * (j + 3) ^ seed;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = op<OP>(x[j], b, c);
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[t] = s;
}

__global__ __launch_bounds__(64, 3) void keccak_kernel(uint32_t* out, int iters, uint32_t seed) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t t = blockIdx.x * 64u + threadIdx.x;
    uint32_t L[25], H[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) { L[i] = t * (i + 1) ^ seed; H[i] = t + i; }
    for (int it = 0; it < iters; ++it) bft::keccak_f1600_lane(L, H);
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) s ^= L[i] ^ H[i];
    out[t] = s;
#endif
}
}  // namespace

template <class F>
static void run(const char* name, F launch, int iters, double instr_per_iter, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int waves : {256, 512, 768, 1024, 1536, 2048, 3072, 4096}) {
        launch(waves, iters);                      // warm
        hipEventRecord(e0, 0);
        launch(waves, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double wi = (double)waves * iters * instr_per_iter, cyc = ms * 1e-3 * 2.4e9;
        printf("{\"op\": \"%s\", \"waves\": %d, \"ms\": %.4f, \"wave_instr_per_s\": %.4e, \"cycles_per_instr_per_cu\": %.3f, "
               "\"cycles_per_instr_per_wave\": %.2f}\n", name, waves, ms, wi / (ms * 1e-3), cyc * cus / wi,
               cyc / ((double)iters * instr_per_iter));
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    uint32_t* out;
    hipMalloc(&out, 4096 * 64 * 4);
    const int it = 20000;
    run("v_xor_b32", [&](int w, int n) { hipLaunchKernelGGL(rate_kernel<0>, dim3(w), dim3(64), 0, 0, out, n, 1u); }, it, 32, cus);
    run("v_bitop3_b32", [&](int w, int n) { hipLaunchKernelGGL(rate_kernel<1>, dim3(w), dim3(64), 0, 0, out, n, 1u); }, it, 32, cus);
    run("v_alignbit_b32", [&](int w, int n) { hipLaunchKernelGGL(rate_kernel<2>, dim3(w), dim3(64), 0, 0, out, n, 1u); }, it, 32, cus);
    run("v_add_u32", [&](int w, int n) { hipLaunchKernelGGL(rate_kernel<3>, dim3(w), dim3(64), 0, 0, out, n, 1u); }, it, 32, cus);
    // keccak: instructions per permutation from the disassembly are ~180 x 24; reported per round (180)
    run("keccak_f1600_lane_round", [&](int w, int n) { hipLaunchKernelGGL(keccak_kernel, dim3(w), dim3(64), 0, 0, out, n, 1u); },
        400, 24 * 180, cus);
    hipFree(out);
    return 0;
}
