// fp_microbench.hip -- how fast the f4 tower arithmetic can run on one lane
// (is the pairing bound by its stack traffic or by its
// instruction mix?).  Dev tooling, not product: it #includes the product's
// pairing.hip to time its own units in isolation, on register-only chains:
//
//   fp2mul      a <- a * b (fp2_mul_in, inlined), K times: the Fp2 product
//               alone, every operand in VGPRs
//   fp12sqr     f <- f^2 through the product's out-of-line fp12_sqr (its
//               Fp6 operands pass through the stack, as in the Miller loop)
//   fp12sqr_inl the same squaring with the Fp6 products inlined (one unit,
//               no call boundary inside): what a register-resident f costs
//   cyclo       f <- cyclotomic square (Granger-Scott, the final
//               exponentiation's unit, already inlined in the product)
//
// Every kernel runs 2 waves/SIMD (the pairing kernels' occupancy) over the
// whole chip and writes its result so nothing is dead code.  Rates: Fp2
// products (or squarings) per second; `rocprofv3 --pmc SQ_INSTS_VALU` of the
// same binary gives lane-ops per unit (tools/gpu_r6d.sh).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I hbbft_amd/csrc \
//          tools/fp_microbench.hip -o tools/fp_microbench
#include <chrono>
#include <cstdio>
#include <vector>

#include "pairing.hip"

namespace hbrbc {
namespace {

constexpr int kMbBlock = 64;

DEV void seed_fp(Fp &r, uint32_t s) {
    for (int i = 0; i < NL; ++i) r.l[i] = (s * 2654435761u + 97u * i) & (i == NL - 1 ? 0x0FFFFFFFu : 0xFFFFFFFFu);
}
DEV void seed12(Fp12 &f, uint32_t s) {
    Fp *p = reinterpret_cast<Fp *>(&f);
    for (int i = 0; i < 12; ++i) seed_fp(p[i], s + 31u * i);
}
DEV uint32_t fold12(const Fp12 &f) {
    const Fp *p = reinterpret_cast<const Fp *>(&f);
    uint32_t x = 0;
    for (int i = 0; i < 12; ++i)
        for (int j = 0; j < NL; ++j) x ^= p[i].l[j];
    return x;
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_fp2mul(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp2 a, b;
    seed_fp(a.c0, g);
    seed_fp(a.c1, g + 7);
    seed_fp(b.c0, g + 13);
    seed_fp(b.c1, g + 29);
    for (int it = 0; it < iters; ++it) fp2_mul_in(a, a, b);
    uint32_t x = 0;
    for (int j = 0; j < NL; ++j) x ^= a.c0.l[j] ^ a.c1.l[j];
    out[g] = x;
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_fp12sqr(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    seed12(f, g);
    for (int it = 0; it < iters; ++it) fp12_sqr(f, f);
    out[g] = fold12(f);
}

DEV void fp6_mul_inl(Fp6 &r, const Fp6 &a, const Fp6 &b) {
    Fp2 aa, bb, cc, s, t, t1, t2, t3;
    fp2_mul_in(aa, a.c0, b.c0);
    fp2_mul_in(bb, a.c1, b.c1);
    fp2_mul_in(cc, a.c2, b.c2);
    fp2_add(s, a.c1, a.c2);
    fp2_add(t, b.c1, b.c2);
    fp2_mul_in(t1, s, t);
    fp2_sub(t1, t1, bb);
    fp2_sub(t1, t1, cc);
    fp2_mul_xi(t1, t1);
    fp2_add(t1, t1, aa);
    fp2_add(s, a.c0, a.c2);
    fp2_add(t, b.c0, b.c2);
    fp2_mul_in(t3, s, t);
    fp2_sub(t3, t3, aa);
    fp2_add(t3, t3, bb);
    fp2_sub(t3, t3, cc);
    fp2_add(s, a.c0, a.c1);
    fp2_add(t, b.c0, b.c1);
    fp2_mul_in(t2, s, t);
    fp2_sub(t2, t2, aa);
    fp2_sub(t2, t2, bb);
    fp2_mul_xi(cc, cc);
    fp2_add(t2, t2, cc);
    r.c0 = t1;
    r.c1 = t2;
    r.c2 = t3;
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_fp12sqr_inl(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    seed12(f, g);
    for (int it = 0; it < iters; ++it) {
        Fp6 ab, s, t;
        fp6_mul_inl(ab, f.c0, f.c1);
        fp6_add(s, f.c0, f.c1);
        fp6_mul_v(t, f.c1);
        fp6_add(t, t, f.c0);
        fp6_mul_inl(s, s, t);
        fp6_sub(s, s, ab);
        fp6_mul_v(t, ab);
        fp6_sub(f.c0, s, t);
        fp6_dbl(f.c1, ab);
    }
    out[g] = fold12(f);
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_cyclo(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    seed12(f, g);
    for (int it = 0; it < iters; ++it) fp12_cyclo_sqr(f);
    out[g] = fold12(f);
}

// the final exponentiation's pieces: f^|x| (fp12_exp_by_x: 62 cyclotomic
// squarings + 5 products) and the whole final exponentiation
__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_expx(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    seed12(f, g);
    for (int it = 0; it < iters; ++it) fp12_exp_by_x(f, f, 0);
    out[g] = fold12(f);
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_fe(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    seed12(f, g);
    for (int it = 0; it < iters; ++it) {
        Fp12 r;
        final_exp(r, f);
        f = r;
    }
    out[g] = fold12(f);
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_fp12mul(
    int iters, uint32_t *out, const uint32_t *) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f, h;
    seed12(f, g);
    seed12(h, g + 5);
    for (int it = 0; it < iters; ++it) fp12_mul(f, f, h);
    out[g] = fold12(f);
}

// the prepared Miller loop's pieces: one line application (load 72 words,
// scale two coefficients by P, sparse product) and one whole bit step
// (squaring + two line applications, as miller_prepared_kernel runs them)
__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_apply(
    int iters, uint32_t *out, const uint32_t *line) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    Fp xp, yp;
    seed12(f, g);
    seed_fp(xp, g + 3);
    seed_fp(yp, g + 9);
    for (int it = 0; it < iters; ++it) apply_prepared_in(f, line + (it & 63) * kLineWords, xp, yp);
    out[g] = fold12(f);
}

__global__ __launch_bounds__(kMbBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mb_millerstep(
    int iters, uint32_t *out, const uint32_t *line) {
    const uint32_t g = blockIdx.x * kMbBlock + threadIdx.x;
    Fp12 f;
    Fp xa, ya, xc, yc;
    seed12(f, g);
    seed_fp(xa, g + 3);
    seed_fp(ya, g + 9);
    seed_fp(xc, g + 5);
    seed_fp(yc, g + 11);
    for (int it = 0; it < iters; ++it) {
        miller_sqr(f);
        HB_APPLY_PREPARED(f, line + (it & 63) * kLineWords, xa, ya);
        HB_APPLY_PREPARED(f, line + ((it + 7) & 63) * kLineWords, xc, yc);
    }
    out[g] = fold12(f);
}

}  // namespace
}  // namespace hbrbc

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

int main(int argc, char **argv) {
    using namespace hbrbc;
    const int lanes = argc > 1 ? atoi(argv[1]) : 256 * 4 * 2 * 64;   // 2 waves per SIMD
    const int blocks = lanes / kMbBlock;
    uint32_t *out, *line;
    CK(hipMalloc(&out, (size_t)lanes * 4));
    {   // 64 line records of arbitrary words (timing only)
        std::vector<uint32_t> h(64 * kLineWords);
        for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u) & 0x0FFFFFFFu;
        CK(hipMalloc(&line, h.size() * 4));
        CK(hipMemcpy(line, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    struct K {
        const char *name;
        void (*fn)(int, uint32_t *, const uint32_t *);
        int iters;
        int fp2_products;   // Fp2 products (or squarings) per iteration
    } ks[] = {{"fp2mul", mb_fp2mul, 2000, 1},
              {"fp12sqr", mb_fp12sqr, 200, 12},      // 2 Fp6 products x 6 Fp2 products
              {"fp12sqr_inl", mb_fp12sqr_inl, 200, 12},
              {"cyclo", mb_cyclo, 200, 9},            // 3 fp4_sqr x 3 Fp2 squarings
              {"fp12mul", mb_fp12mul, 100, 18},       // 3 Fp6 products x 6 Fp2 products
              {"expx", mb_expx, 4, 62 * 9 + 5 * 18},
              {"fe", mb_fe, 1, 0},
              {"apply", mb_apply, 100, 13},          // 13 Fp2 products (+ 2 Fp2 x Fp)
              {"millerstep", mb_millerstep, 50, 12 + 2 * 13}};
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(kMbBlock), 0, 0, 4, out, line);   // warm-up
        CK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(kMbBlock), 0, 0, k.iters, out, line);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        const double units = (double)lanes * k.iters;
        printf("{\"kernel\": \"%s\", \"lanes\": %d, \"iters\": %d, \"ms\": %.4f, \"units_per_s\": %.4e, "
               "\"fp2_products_per_s\": %.4e}\n",
               k.name, lanes, k.iters, ms, units / (ms * 1e-3), units * k.fp2_products / (ms * 1e-3));
    }
    CK(hipFree(out));
    CK(hipFree(line));
    return 0;
}
