// mfma_gf.hip -- measured evaluation of GF(2^8) Reed-Solomon coding on the
// MI355X matrix cores (SURVEY §7 "Hard parts").
//
// Formulation (bit-sliced GF(2)): multiplying by a constant c is linear over
// GF(2), an 8x8 bit matrix, so out_row[i] = sum_j c_ij * in_row[j] becomes,
// per byte position n, D[o][n] = parity( sum_K A[o][K] * B[K][n] ) with
// o = (output row i, bit q), K = (input row j, bit p), A[o][K] = bit q of
// c_ij * 2^p and B[K][n] = bit p of in_row[j][n].  An integer MFMA computes
// the sum; its lowest bit is the GF(2) result.
//   * i8 (v_mfma_i32_32x32x32_i8): B may hold the whole byte shifted right by
//     p -- A is 0/1, so only the lowest bit of B reaches the sum's parity.
//   * fp4 e2m1 (v_mfma_scale_f32_32x32x64_f8f6f4, unit e8m0 scales 127): B
//     nibbles 0x2 (= 1.0) or 0x0; the fp32 sums are exact integers <= 8k.
// 64 MFMA MACs per GF byte-MAC: cfg5 encode (k = 84, m = 166, S = 49933,
// 1024 instances) is 42 M-tiles x 1561 N-tiles x 21 (i8) / 11 (fp4) K-steps.
//
// This program (1) checks both formulations bit-exact against a host GF
// multiply on one instance of the cfg5 matrix, and (2) times MFMA-issue-bound
// kernels that execute exactly the cfg5 encode's MFMA count with register
// operands (no data movement at all): a lower bound on any MFMA encoder.
// Compare with the XOR-network encoder under rocprofv3 --stats.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_gf tools/mfma_gf.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__);       \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// ------------------------------------------------------------ host GF(2^8) --
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
        b >>= 1;
    }
    return r;
}
static uint8_t ginv(uint8_t a) {
    for (int x = 1; x < 256; ++x)
        if (gmul(a, (uint8_t)x) == 1) return (uint8_t)x;
    return 0;
}
static uint8_t gpow(uint8_t a, int n) {
    uint8_t r = 1;
    for (int i = 0; i < n; ++i) r = gmul(r, a);
    return n == 0 ? 1 : (a == 0 ? 0 : r);
}
// rse build_matrix(k, n): parity rows k..n-1 of V * inv(V[0..k])
static std::vector<uint8_t> parity_matrix(int k, int n) {
    std::vector<uint8_t> v(n * k), top(k * k), inv(k * k, 0);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) v[r * k + c] = gpow((uint8_t)r, c);
    for (int i = 0; i < k * k; ++i) top[i] = v[i];
    for (int i = 0; i < k; ++i) inv[i * k + i] = 1;
    for (int c = 0; c < k; ++c) {
        int p = c;
        while (top[p * k + c] == 0) ++p;
        for (int j = 0; j < k; ++j) {
            std::swap(top[c * k + j], top[p * k + j]);
            std::swap(inv[c * k + j], inv[p * k + j]);
        }
        const uint8_t s = ginv(top[c * k + c]);
        for (int j = 0; j < k; ++j) {
            top[c * k + j] = gmul(s, top[c * k + j]);
            inv[c * k + j] = gmul(s, inv[c * k + j]);
        }
        for (int r = 0; r < k; ++r) {
            const uint8_t f = top[r * k + c];
            if (r == c || !f) continue;
            for (int j = 0; j < k; ++j) {
                top[r * k + j] ^= gmul(f, top[c * k + j]);
                inv[r * k + j] ^= gmul(f, inv[c * k + j]);
            }
        }
    }
    const int m = n - k;
    std::vector<uint8_t> par(m * k);
    for (int r = 0; r < m; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int j = 0; j < k; ++j) acc ^= gmul(v[(k + r) * k + j], inv[j * k + c]);
            par[r * k + c] = acc;
        }
    return par;
}

// ------------------------------------------------------- exact i8 kernel ---
// One wave per (32-output-bit tile mt, 32-position tile nt).  K-step t covers
// input rows 16g..16g+15 (g = t / 4) and bits {2pp, 2pp+1} (pp = t % 4): lane
// half h supplies bit 2pp + h of the 16 rows at its column.  Operand maps
// (gfx950, checked here): A lane l = row l&31, K 16(l>>5)+j (j = byte j);
// B lane l = column l&31, same K; D reg v = row (v&3) + 8(v>>2) + 4(l>>5).
__global__ __launch_bounds__(64) void gf_mfma_i8_exact(const uint8_t *__restrict__ data, int S,
                                                      int kpad, const v4i *__restrict__ afrag,
                                                      int ksteps, uint8_t *__restrict__ out) {
    const int mt = blockIdx.y, nt = blockIdx.x, l = threadIdx.x;
    const int n = nt * 32 + (l & 31), h = l >> 5;
    v16i acc = {};
    for (int t = 0; t < ksteps; ++t) {
        const int g = t >> 2, p = 2 * (t & 3) + h;
        uint32_t w[4];
        for (int q = 0; q < 4; ++q) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) {
                const int row = 16 * g + 4 * q + b;
                const uint32_t x = (row < kpad && n < S) ? data[(size_t)row * S + n] : 0u;
                v |= ((x >> p) & 0xFFu) << (8 * b);   // high bits are don't-care
            }
            w[q] = v;
        }
        const v4i B = {(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
        const v4i A = afrag[((size_t)mt * ksteps + t) * 64 + l];
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, acc, 0, 0, 0);
    }
    // bits q = (v&3) + 4h of output row 4mt + (v>>2); the other half's nibble by shuffle
    for (int r4 = 0; r4 < 4; ++r4) {
        uint32_t nib = 0;
        for (int e = 0; e < 4; ++e) nib |= (uint32_t)(acc[4 * r4 + e] & 1) << e;
        const uint32_t other = __shfl_xor(nib, 32);
        if (h == 0 && n < S) out[(size_t)(4 * mt + r4) * S + n] = (uint8_t)(nib | (other << 4));
    }
}

// ------------------------------------------------------ exact fp4 kernel ---
// K-step t (64 K) covers rows 16g..16g+15 (g = t / 2) and bits 4pq..4pq+3
// (pq = t % 2); lane half h supplies bits 4pq + 2h + e (e = 0, 1) of its 16
// rows as K-values 16e + j.  An fp4 operand: 32 nibbles per lane, element i
// in nibble i (low nibble first); 0x2 = 1.0.
__global__ __launch_bounds__(64) void gf_mfma_fp4_exact(const uint8_t *__restrict__ data, int S,
                                                       int kpad, const v8i *__restrict__ afrag,
                                                       int ksteps, uint8_t *__restrict__ out) {
    const int mt = blockIdx.y, nt = blockIdx.x, l = threadIdx.x;
    const int n = nt * 32 + (l & 31), h = l >> 5;
    v16f acc = {};
    for (int t = 0; t < ksteps; ++t) {
        const int g = t >> 1, pq = t & 1;
        uint32_t w[4] = {0, 0, 0, 0};
        for (int e = 0; e < 2; ++e) {
            const int p = 4 * pq + 2 * h + e;
            for (int j = 0; j < 16; ++j) {
                const int row = 16 * g + j;
                const uint32_t x = (row < kpad && n < S) ? data[(size_t)row * S + n] : 0u;
                const int i = 16 * e + j;   // element index, nibble i
                w[i >> 3] |= (((x >> p) & 1u) << 1) << (4 * (i & 7));
            }
        }
        const v8i B = {(int)w[0], (int)w[1], (int)w[2], (int)w[3], 0, 0, 0, 0};
        const v8i A = afrag[((size_t)mt * ksteps + t) * 64 + l];
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, acc, 4, 4, 0, 127, 0, 127);
    }
    for (int r4 = 0; r4 < 4; ++r4) {
        uint32_t nib = 0;
        for (int e = 0; e < 4; ++e) nib |= (uint32_t)((int)acc[4 * r4 + e] & 1) << e;
        const uint32_t other = __shfl_xor(nib, 32);
        if (h == 0 && n < S) out[(size_t)(4 * mt + r4) * S + n] = (uint8_t)(nib | (other << 4));
    }
}

// ------------------------------------------------- issue-bound kernels -----
// Each wave runs `per_wave` MFMAs as 4 independent accumulator chains on
// register operands (enough to keep one SIMD's matrix core issuing).
__global__ __launch_bounds__(256) void bound_i8(int per_wave, int *__restrict__ sink) {
    v4i a = {(int)threadIdx.x, 3, 5, 7}, b = {1, (int)blockIdx.x, 2, 9};
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < per_wave; i += 4) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
    }
    int s = 0;
    for (int v = 0; v < 16; ++v) s += c0[v] ^ c1[v] ^ c2[v] ^ c3[v];
    if (s == 0x7fffffff) sink[0] = s;
}

__global__ __launch_bounds__(256) void bound_fp4(int per_wave, int *__restrict__ sink) {
    v8i a = {(int)threadIdx.x, 0x22222222, 0x20202020, 7, 0, 0, 0, 0};
    v8i b = {0x02020202, (int)blockIdx.x, 0x22002200, 9, 0, 0, 0, 0};
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < per_wave; i += 4) {
        c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 127, 0, 127);
        c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, c1, 4, 4, 0, 127, 0, 127);
        c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c2, 4, 4, 0, 127, 0, 127);
        c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, b, c3, 4, 4, 0, 127, 0, 127);
    }
    float s = 0.f;
    for (int v = 0; v < 16; ++v) s += c0[v] + c1[v] + c2[v] + c3[v];
    if (s == 123.25f) sink[0] = 1;
}

// ------------------------------------------------------------------ host ---
int main(int argc, char **argv) {
    const int k = 84, n_all = 250, m = n_all - k;   // cfg5: N = 250, f = 83
    const int inst = argc > 1 ? atoi(argv[1]) : 1024;
    const int S_full = 49933;
    const std::vector<uint8_t> par = parity_matrix(k, n_all);
    const int kpad = 96, mbits = 8 * m, mtiles = (mbits + 31) / 32;

    // ---- (1) exactness on one instance, S = 1000 positions ----
    const int S = 1000;
    std::vector<uint8_t> data((size_t)kpad * S, 0), ref((size_t)m * S, 0);
    srand(7);
    for (int r = 0; r < k; ++r)
        for (int i = 0; i < S; ++i) data[(size_t)r * S + i] = (uint8_t)(rand() >> 7);
    for (int r = 0; r < m; ++r)
        for (int i = 0; i < S; ++i) {
            uint8_t a = 0;
            for (int j = 0; j < k; ++j) a ^= gmul(par[r * k + j], data[(size_t)j * S + i]);
            ref[(size_t)r * S + i] = a;
        }
    auto abit = [&](int o, int row, int p) -> int {   // A[(i,q)][(row,p)]
        const int i = o / 8, q = o % 8;
        if (i >= m || row >= k) return 0;
        return (gmul(par[i * k + row], (uint8_t)(1u << p)) >> q) & 1;
    };
    // i8 fragments
    const int ks8 = (kpad / 16) * 4;
    std::vector<int8_t> a8((size_t)mtiles * ks8 * 64 * 16);
    for (int mt = 0; mt < mtiles; ++mt)
        for (int t = 0; t < ks8; ++t)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 16; ++j) {
                    const int g = t >> 2, p = 2 * (t & 3) + (l >> 5);
                    a8[(((size_t)mt * ks8 + t) * 64 + l) * 16 + j] =
                        (int8_t)abit(32 * mt + (l & 31), 16 * g + j, p);
                }
    // fp4 fragments (32 nibbles in the low 16 bytes of each lane's 32-byte slot)
    const int ks4 = (kpad / 16) * 2;
    std::vector<uint8_t> a4((size_t)mtiles * ks4 * 64 * 32, 0);
    for (int mt = 0; mt < mtiles; ++mt)
        for (int t = 0; t < ks4; ++t)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 2; ++e)
                    for (int j = 0; j < 16; ++j) {
                        const int g = t >> 1, p = 4 * (t & 1) + 2 * (l >> 5) + e, i = 16 * e + j;
                        if (abit(32 * mt + (l & 31), 16 * g + j, p))
                            a4[(((size_t)mt * ks4 + t) * 64 + l) * 32 + i / 2] |= (uint8_t)(0x2 << (4 * (i & 1)));
                    }
    uint8_t *d_data, *d_out, *d_a8, *d_a4;
    CK(hipMalloc(&d_data, data.size()));
    CK(hipMalloc(&d_out, (size_t)(mtiles * 4) * S));
    CK(hipMalloc(&d_a8, a8.size()));
    CK(hipMalloc(&d_a4, a4.size()));
    CK(hipMemcpy(d_data, data.data(), data.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_a8, a8.data(), a8.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_a4, a4.data(), a4.size(), hipMemcpyHostToDevice));
    std::vector<uint8_t> got((size_t)(mtiles * 4) * S);
    int bad8 = 0, bad4 = 0;
    dim3 grid((S + 31) / 32, mtiles);
    hipLaunchKernelGGL(gf_mfma_i8_exact, grid, dim3(64), 0, 0, d_data, S, kpad,
                       (const v4i *)d_a8, ks8, d_out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), d_out, got.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ref.size(); ++i) bad8 += got[i] != ref[i];
    hipLaunchKernelGGL(gf_mfma_fp4_exact, grid, dim3(64), 0, 0, d_data, S, kpad,
                       (const v8i *)d_a4, ks4, d_out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), d_out, got.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ref.size(); ++i) bad4 += got[i] != ref[i];
    printf("exact: i8 %d / %zu bytes differ, fp4 %d / %zu bytes differ (cfg5 parity block, "
           "%d positions)\n", bad8, ref.size(), bad4, ref.size(), S);

    // ---- (2) issue-bound kernels at the cfg5 encode's MFMA count ----
    const long ntiles = (S_full + 31) / 32;
    const long mf8 = (long)mtiles * ntiles * ks8 * inst;          // 32x32x32 i8
    const long mf4 = (long)mtiles * ntiles * ((8 * k + 63) / 64) * inst;  // 32x32x64 fp4
    int *sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int per_wave = 1024;
    for (int kind = 0; kind < 2; ++kind) {
        const long total = kind == 0 ? mf8 : mf4;
        const long waves = (total + per_wave - 1) / per_wave;
        const unsigned blocks = (unsigned)((waves + 3) / 4);
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            if (kind == 0)
                hipLaunchKernelGGL(bound_i8, dim3(blocks), dim3(256), 0, 0, per_wave, sink);
            else
                hipLaunchKernelGGL(bound_fp4, dim3(blocks), dim3(256), 0, 0, per_wave, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double macs = (double)blocks * 4 * per_wave * (kind == 0 ? 32.0 * 32 * 32 : 32.0 * 32 * 64);
        printf("bound %s: %ld MFMAs (cfg5 encode, %d instances) in %.2f ms = %.0f T MAC/s = %.2f T "
               "GF byte-MAC/s\n", kind == 0 ? "i8 32x32x32" : "fp4 32x32x64", total, inst, best,
               macs / best / 1e9, macs / 64.0 / best / 1e9);
    }
    printf("cfg5 encode GF byte-MACs: %.3e (k*m*S*instances)\n", (double)k * m * S_full * inst);
    return (bad8 || bad4) ? 2 : 0;
}
