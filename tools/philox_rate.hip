// Micro-benchmark (diagnostic, not part of the library): Philox4x32-10 throughput on one MI355X, as the
// drop masks draw it (bft_common.h deliver_mask: counter (inst, tick, phase<<24 | recv<<8 | block, DOM_DROP)).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include "../consensus-rs_amd/csrc/bft_common.h"

template <int K>
__global__ __launch_bounds__(256) void philox_plain(uint64_t seed, uint32_t* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < K; ++i) {
        uint32_t w[4];
        bft::philox(seed, t >> 6, i >> 3, (i << 24) | ((t & 63u) << 8) | (i & 7u), bft::DOM_DROP, w);
        acc ^= w[0] ^ w[1] ^ w[2] ^ w[3];
    }
    out[t] = acc;
}

// the same draw with each round's two 3-input XORs as v_bitop3_b32
__device__ inline uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}
__device__ inline void philox_b3(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
        const uint32_t n0 = x3((uint32_t)(p1 >> 32), c1, k0), n2 = x3((uint32_t)(p0 >> 32), c3, k1);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
template <int K>
__global__ __launch_bounds__(256) void philox_bitop3(uint64_t seed, uint32_t* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < K; ++i) {
        uint32_t w[4];
        philox_b3(seed, t >> 6, i >> 3, (i << 24) | ((t & 63u) << 8) | (i & 7u), bft::DOM_DROP, w);
        acc ^= w[0] ^ w[1] ^ w[2] ^ w[3];
    }
    out[t] = acc;
}

// eight blocks per call, the shape of one full phase
template <int K>
__global__ __launch_bounds__(256) void philox_phase(uint64_t seed, uint32_t thr16, uint32_t* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    for (uint32_t i = 0; i < K; ++i) {
        bft::Bits<1> pr = bft::Bits<1>::low(64);
        acc ^= bft::deliver_mask<1>(seed, 64, thr16, t >> 6, i, 3, t & 63u, pr).w[0];
    }
    out[t] = (uint32_t)acc ^ (uint32_t)(acc >> 32);
}

int main() {
    uint32_t* d;
    const int blocks = 256 * 8 * 4, threads = 256;
    hipMalloc(&d, (size_t)blocks * threads * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float ms;
    philox_plain<64><<<blocks, threads>>>(0x1234, d);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) philox_plain<64><<<blocks, threads>>>(0x1234 + r, d);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    double n = 5.0 * blocks * threads * 64;
    printf("philox_plain: %.3f ms, %.3e philox/s, %.1f SIMD-cycles per wave-philox (2.4 GHz, 1024 SIMDs)\n", ms, n / (ms * 1e-3),
           1024 * 2.4e9 / (n / (ms * 1e-3) / 64));
    philox_bitop3<64><<<blocks, threads>>>(0x1234, d);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) philox_bitop3<64><<<blocks, threads>>>(0x1234 + r, d);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("philox_bitop3: %.3f ms, %.3e philox/s, %.1f SIMD-cycles per wave-philox\n", ms, n / (ms * 1e-3),
           1024 * 2.4e9 / (n / (ms * 1e-3) / 64));
    philox_phase<16><<<blocks, threads>>>(0x1234, 3277, d);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) philox_phase<16><<<blocks, threads>>>(0x1234 + r, 3277, d);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    n = 5.0 * blocks * threads * 16;
    printf("deliver_mask (8 blocks): %.3f ms, %.3e masks/s, %.1f SIMD-cycles per wave-mask\n", ms, n / (ms * 1e-3),
           1024 * 2.4e9 / (n / (ms * 1e-3) / 64));
    return 0;
}
