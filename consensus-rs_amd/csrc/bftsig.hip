// bftsig.hip — gfx950 kernels and the C ABI of libbftsig (include/bftsig.h): batched secp256k1
// recoverable ECDSA, one lane per item. The arithmetic is secp256k1.h (shared with the host tests).
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bftsig.h"
#include "secp256k1.h"

namespace bft {
namespace secp {

// byte loads of a record (items are 20/32/65-byte records; the arithmetic dwarfs the traffic)
__device__ inline void load_bytes(const uint8_t* src, uint8_t* dst, int n) {
    for (int i = 0; i < n; ++i) dst[i] = src[i];
}
__device__ inline void zero_bytes(uint8_t* dst, int n) {
    for (int i = 0; i < n; ++i) dst[i] = 0;
}

__global__ __launch_bounds__(64) void sig_address_kernel(const Aff* gtab, const uint8_t* sec, uint64_t n,
                                                         uint8_t* pub, uint8_t* addr, uint8_t* ok) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff q;
    bool good = secret_to_pub(sec + 32 * i, gtab, q);
    uint8_t a[20];
    if (good) pub_address(q, a);
    if (pub) {
        if (good) { u_to_be(q.x, pub + 64 * i); u_to_be(q.y, pub + 64 * i + 32); }
        else zero_bytes(pub + 64 * i, 64);
    }
    for (int k = 0; k < 20; ++k) addr[20 * i + k] = good ? a[k] : 0;
    ok[i] = good ? 1 : 0;
}

__global__ __launch_bounds__(64) void sig_sign_kernel(const Aff* gtab, const uint8_t* sec, const uint32_t* key_index,
                                                      const uint8_t* dig, uint64_t n, uint8_t* sig, uint8_t* ok) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t ki = key_index ? key_index[i] : i;
    // records straight from / to global memory: local byte arrays indexed in loops would live in scratch
    bool good = sign(sec + 32 * ki, dig + 32 * i, gtab, sig + 65 * i);
    if (!good) zero_bytes(sig + 65 * i, 65);
    ok[i] = good ? 1 : 0;
}

// mode 0: recover (pub nullable, addr); mode 1: verify_address against addr_in
#ifndef SIG_RECOVER_WAVES
#define SIG_RECOVER_WAVES 2
#endif
#ifndef SIG_LDS_TAB
#define SIG_LDS_TAB 1
#endif
__global__ __launch_bounds__(64, SIG_RECOVER_WAVES) void sig_recover_kernel(const Aff* gtab, const uint8_t* dig, const uint8_t* sig,
                                                         uint64_t n, uint8_t* pub, uint8_t* addr,
                                                         const uint8_t* addr_in, uint8_t* ok) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* m = dig + 32 * i;                     // read in place (no local byte copies: scratch)
    const uint8_t* sg = sig + 65 * i;
    Aff q;
#if SIG_LDS_TAB
    __shared__ uint32_t tab_lds[64 * 64];                 // mul_var's 1q..4q, 64 words per lane (TabLds)
    bool good = recover(m, sg, gtab, q, TabLds{tab_lds + threadIdx.x});
#else
    bool good = recover(m, sg, gtab, q);
#endif
    uint8_t a[20];
    if (good) pub_address(q, a);
    if (addr_in) {
        bool eq = good;
        for (int k = 0; k < 20; ++k) eq = eq && a[k] == addr_in[20 * i + k];
        ok[i] = eq ? 1 : 0;
        return;
    }
    if (pub) {
        if (good) { u_to_be(q.x, pub + 64 * i); u_to_be(q.y, pub + 64 * i + 32); }
        else zero_bytes(pub + 64 * i, 64);
    }
    for (int k = 0; k < 20; ++k) addr[20 * i + k] = good ? a[k] : 0;
    ok[i] = good ? 1 : 0;
}

}  // namespace secp
}  // namespace bft

// ------------------------------------------------------------------------------ C ABI
struct bftsig {
    int device = 0;
    bft::secp::Aff* d_gtab = nullptr;
    std::string err;
};

static int fail(bftsig* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}
#define SIGCHECK(h, x)                                                                            \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) return fail(h, -2, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

static constexpr unsigned SIG_BLOCK = 64;

extern "C" {

int bftsig_create(int hip_device, bftsig_t** out) {
    if (!out) return -1;
    *out = nullptr;
    bftsig* h = new bftsig();
    h->device = hip_device;
    *out = h;
    SIGCHECK(h, hipSetDevice(hip_device));
    std::vector<bft::secp::Aff> tab(bft::secp::GTAB_POINTS);
    bft::secp::build_gtab(tab.data());
    SIGCHECK(h, hipMalloc(&h->d_gtab, tab.size() * sizeof(bft::secp::Aff)));
    SIGCHECK(h, hipMemcpy(h->d_gtab, tab.data(), tab.size() * sizeof(bft::secp::Aff), hipMemcpyHostToDevice));
    return 0;
}

void bftsig_destroy(bftsig_t* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipFree(h->d_gtab);
    delete h;
}

const char* bftsig_last_error(const bftsig_t* h) { return h ? h->err.c_str() : "null handle"; }

static int grid_of(bftsig* h, uint64_t n, unsigned& g) {
    uint64_t blocks = (n + SIG_BLOCK - 1) / SIG_BLOCK;
    if (blocks > 0x7fffffffull) return fail(h, -1, "batch too large");
    g = (unsigned)blocks;
    return 0;
}

int bftsig_secret_to_address(bftsig_t* h, const uint8_t* sec, uint64_t n, uint8_t* pub, uint8_t* addr, uint8_t* ok,
                             void* stream) {
    if (!h || !h->d_gtab) return fail(h, -1, "bftsig_secret_to_address: no handle");
    if (n == 0) return 0;
    if (!sec || !addr || !ok) return fail(h, -1, "bftsig_secret_to_address: null buffer");
    unsigned g;
    if (grid_of(h, n, g)) return -1;
    SIGCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(bft::secp::sig_address_kernel, dim3(g), dim3(SIG_BLOCK), 0, (hipStream_t)stream, h->d_gtab, sec, n,
                       pub, addr, ok);
    SIGCHECK(h, hipGetLastError());
    return 0;
}

int bftsig_sign(bftsig_t* h, const uint8_t* sec, const uint32_t* key_index, const uint8_t* dig, uint64_t n,
                uint8_t* sig, uint8_t* ok, void* stream) {
    if (!h || !h->d_gtab) return fail(h, -1, "bftsig_sign: no handle");
    if (n == 0) return 0;
    if (!sec || !dig || !sig || !ok) return fail(h, -1, "bftsig_sign: null buffer");
    unsigned g;
    if (grid_of(h, n, g)) return -1;
    SIGCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(bft::secp::sig_sign_kernel, dim3(g), dim3(SIG_BLOCK), 0, (hipStream_t)stream, h->d_gtab, sec,
                       key_index, dig, n, sig, ok);
    SIGCHECK(h, hipGetLastError());
    return 0;
}

int bftsig_recover(bftsig_t* h, const uint8_t* dig, const uint8_t* sig, uint64_t n, uint8_t* pub, uint8_t* addr,
                   uint8_t* ok, void* stream) {
    if (!h || !h->d_gtab) return fail(h, -1, "bftsig_recover: no handle");
    if (n == 0) return 0;
    if (!dig || !sig || !addr || !ok) return fail(h, -1, "bftsig_recover: null buffer");
    unsigned g;
    if (grid_of(h, n, g)) return -1;
    SIGCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(bft::secp::sig_recover_kernel, dim3(g), dim3(SIG_BLOCK), 0, (hipStream_t)stream, h->d_gtab, dig,
                       sig, n, pub, addr, (const uint8_t*)nullptr, ok);
    SIGCHECK(h, hipGetLastError());
    return 0;
}

int bftsig_verify_address(bftsig_t* h, const uint8_t* addr, const uint8_t* dig, const uint8_t* sig, uint64_t n,
                          uint8_t* ok, void* stream) {
    if (!h || !h->d_gtab) return fail(h, -1, "bftsig_verify_address: no handle");
    if (n == 0) return 0;
    if (!addr || !dig || !sig || !ok) return fail(h, -1, "bftsig_verify_address: null buffer");
    unsigned g;
    if (grid_of(h, n, g)) return -1;
    SIGCHECK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(bft::secp::sig_recover_kernel, dim3(g), dim3(SIG_BLOCK), 0, (hipStream_t)stream, h->d_gtab, dig,
                       sig, n, (uint8_t*)nullptr, (uint8_t*)nullptr, addr, ok);
    SIGCHECK(h, hipGetLastError());
    return 0;
}

}  // extern "C"
