// mad_peak.hip — measures the chip's 32x32->64 multiply-add rate (v_mad_u64_u32), the peak the
// secp256k1 kernels are priced against (the guides list no integer-multiply rate for gfx950).
// Each lane runs 8 independent accumulator chains; prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void mad_kernel(const uint32_t* in, uint64_t* out, int iters) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t b = in[i & 1023] | 1u;
    uint64_t acc[8];
    uint32_t a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = in[(i + 97 * j) & 1023]; acc[j] = a[j]; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] = (uint64_t)a[j] * b + acc[j];      // v_mad_u64_u32
            a[j] = (uint32_t)acc[j] ^ (uint32_t)(acc[j] >> 32);
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= acc[j];
    out[i] = s;
}

int main() {
    const int blocks = 256 * 8 * 4, threads = 256, iters = 4096;
    uint32_t* in;
    uint64_t* out;
    hipMalloc(&in, 4096);
    hipMalloc(&out, (size_t)blocks * threads * 8);
    hipMemset(in, 0x5a, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(mad_kernel, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(mad_kernel, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    double mads = (double)blocks * threads * iters * 8;
    printf("{\"mad_u64_u32_per_s\": %.4e, \"ms\": %.3f}\n", mads / (ms * 1e-3), ms);
    return 0;
}
