// valu_microbench.hip -- measures the VALU ceiling that bounds the Keccak and
// GF kernels on this MI355X: register-only loops of one instruction kind, and
// the Keccak-f[1600] permutation from device_common.hpp.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valu_microbench.hip -o tools/valu_microbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../hbbft_amd/csrc/device_common.hpp"

using namespace hbrbc;

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                     \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

// One VALU instruction kind per KIND, emitted by inline asm so the compiler
// cannot fuse or drop it; 16 independent accumulators per lane.
template <int KIND>
__global__ __launch_bounds__(256) void op_loop(uint32_t *out, int iters, uint32_t s0) {
    uint32_t a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = (KIND == 17) ? 0u : threadIdx.x * 7919u + i * 104729u + s0;
    const uint32_t b = threadIdx.x ^ 0x5a5a5a5au, c = threadIdx.x * 3u, z = s0 >> 31;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (KIND == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 1)
                    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (KIND == 2) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 3) asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(a[i]) : "s"(s0));
                if constexpr (KIND == 4) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 5) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 6) asm volatile("v_alignbit_b32 %0, %1, %0, 7" : "+v"(a[i]) : "s"(s0));
                if constexpr (KIND == 7) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (KIND == 8) asm volatile("v_pk_mov_b32 %0, %1, %0 op_sel:[0,1]" : "+v"(*(uint64_t *)&a[i & 14]) : "v"(*(uint64_t *)&a[(i + 2) & 14]));
                if constexpr (KIND == 9) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i]));
                if constexpr (KIND == 10) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 11) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                // 64-bit shifts: one instruction moves a whole (lo, hi) lane pair
                if constexpr (KIND == 12)
                    asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(*(uint64_t *)&a[i & 14]));
                if constexpr (KIND == 13)
                    asm volatile("v_lshl_add_u64 %0, %0, 7, %1" : "+v"(*(uint64_t *)&a[i & 14]) : "v"(*(uint64_t *)&a[(i + 2) & 14]));
                if constexpr (KIND == 14) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[i]));
                if constexpr (KIND == 15) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                // power probes: the same instructions on operands that never toggle
                if constexpr (KIND == 16) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(z));
                if constexpr (KIND == 17) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[i]));
                if constexpr (KIND == 18) asm volatile("v_lshrrev_b32 %0, 3, %1" : "=v"(a[i]) : "v"(b));
                if constexpr (KIND == 19) asm volatile("v_lshlrev_b32 %0, 3, %1" : "=v"(a[i]) : "v"(b));
                // left-shift candidates for the bit-plane transposes (t << d)
                if constexpr (KIND == 20) asm volatile("v_pk_lshlrev_b16 %0, 3, %0" : "+v"(a[i]));
                if constexpr (KIND == 21) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 22) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (KIND == 23) asm volatile("v_pk_add_u16 %0, %0, %0" : "+v"(a[i]));
                // multi-precision pieces of the BLS12-381 Fp product (pairing.hip)
                if constexpr (KIND == 24)
                    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(*(uint64_t *)&a[i & 14]) : "v"(b), "v"(c) : "vcc");
                if constexpr (KIND == 25) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
                if constexpr (KIND == 26) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 15]));
            }
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) x ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void keccak_loop(uint32_t *out, int iters) {
    uint32_t L[25], H[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        L[i] = threadIdx.x + i;
        H[i] = blockIdx.x + 3 * i;
    }
    for (int it = 0; it < iters; ++it) keccak_f1600(L, H);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) x ^= L[i] ^ H[i];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <class F>
static float time_ms(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("device %s, %d CUs, clock %d kHz\n", p.name, cus, p.clockRate);
    uint32_t *out;
    const int blocks = cus * 8 * 16;  // many full rounds of residency
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    const int iters = 64;
    const char *names[27] = {"v_xor_b32", "v_bitop3_b32", "v_alignbit_b32(v,v)", "v_perm_b32(s,s,v)",
                             "v_and_b32", "v_lshl_or_b32", "v_alignbit_b32(s,v)", "v_perm_b32(v,v,v)",
                             "v_pk_mov_b32", "v_lshrrev_b32", "v_alignbyte_b32", "v_add_u32",
                             "v_lshrrev_b64", "v_lshl_add_u64", "v_lshlrev_b32", "v_or3_b32",
                             "v_xor_b32 (x^0)", "v_alignbit_b32 (0)", "v_lshrrev_b32 (b)", "v_lshlrev_b32 (b)",
                             "v_pk_lshlrev_b16", "v_lshl_add_u32", "v_mul_u32_u24", "v_pk_add_u16",
                             "v_mad_u64_u32", "v_addc_co_u32 (vcc chain)", "v_mov_b32"};
#define K(n) case n: hipLaunchKernelGGL(op_loop<n>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u); break
    for (int kind = 0; kind < 27; ++kind) {
        float ms = time_ms([&] {
            switch (kind) { K(0); K(1); K(2); K(3); K(4); K(5); K(6); K(7); K(8); K(9); K(10); K(11); K(12); K(13); K(14); K(15); K(16); K(17); K(18); K(19); K(20); K(21); K(22); K(23); K(24); K(25); K(26); }
        });
        const double instr = (double)blocks * 256 * iters * 8 * 16;
        printf("%-22s %8.3f ms  %6.2f T lane-instr/s\n", names[kind], ms, instr / ms / 1e9);
    }
    // residency forced with dynamic LDS: one 256-thread block = one wave per
    // SIMD, so w blocks per CU = w waves per SIMD
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(keccak_loop),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int w : {2, 3, 4, 5}) {
        const size_t lds = (size_t)(163840 / w) / 512 * 512;
        const int nb = cus * w * 4;  // four full residency rounds
        const int kit = 64;
        float ms = time_ms([&] {
            hipLaunchKernelGGL(keccak_loop, dim3(nb), dim3(256), lds, 0, out, kit);
        });
        const double perms = (double)nb * 256 * kit;
        printf("keccak-f1600 at %d waves/SIMD: %8.3f ms  %.3f G perm/s  = %.2f T ops/s @4320 "
               "ops/perm\n", w, ms, perms / ms / 1e6, perms * 4320 / ms / 1e9);
    }
    return 0;
}
