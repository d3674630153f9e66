// mfma_enc.hip -- the cfg3 Reed-Solomon encoder on the matrix cores, built
// end to end to settle VERDICT r4 item 5 ("the one place MFMA could still
// pay"): loads, operand build, FP4 MFMA, parity packing, stores;
// bit-exact against libhbrbc's XOR-network encoder on the same slab, timed
// beside it, and run for the rocprofv3 SQ_INSTS_VALU pass (tools/gpu_r5f.sh).
//
// Formulation (tools/mfma_gf.hip): per byte position n, parity bit (i, q) =
// parity( sum over K = (data row r, bit p) of A[(i,q)][K] * bit p of row r ),
// A[(i,q)][(r,p)] = bit q of (c_ir * 2^p).  FP4 e2m1 32x32x64 with block
// scales: A elements 0x2 = 1.0 (scale 2^0); B elements are TWO data bits
// (x >> d) & 3 of a byte read as e2m1 0..1.5 and scaled by 2^1 -> 0, 1, 2, 3,
// whose parity is bit d: so one B dword is (X >> d) & 0x33333333 of a dword X
// holding 4 rows' bytes at one position -- two VALU per 8 K-values.  Sums are
// exact integers <= 176 * 3 in fp32.
//
// Wave = 128 consecutive positions of one instance; lane (c, h): positions
// 4c..4c+3 (4 N-subtiles of 32 columns), K-half h.  K-step t covers data rows
// 8t..8t+7 (24 rows, 2 of them zero padding); lane half h supplies rows
// 8t+4h..8t+4h+3, element e = 8d + 2i + s4 (dword d, byte i, nibble s4) is
// bit d + 4 s4 of row 8t+4h+i.  The 11 M-tiles x 3 K-steps of A fragments
// (336 parity bits x 192 K) sit in LDS (33 KB per workgroup).
//
// Packing: accumulator v of lane (c, h) is parity bit q = (v & 3) + 4h of
// row 4 mt + (v >> 2) (gfx950 32x32 D layout); adding 2^(23-e) to a count
// k < 2^(23-e) puts bit 0 of k at bit e of the float's pattern, so three
// v_bitop3 merge four counts into a nibble; the two K-halves' nibbles meet
// through one lane swap and the four subtiles' bytes of a row form one dword
// store (positions 4c..4c+3).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_enc.hip -o tools/mfma_enc \
//            -Iinclude -Lhbbft_amd -lhbrbc -Wl,-rpath,'$ORIGIN/../hbbft_amd'
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/hbrbc.h"

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__);       \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)
#define CL(x)                                                                            \
    do {                                                                                 \
        int r_ = (x);                                                                    \
        if (r_) {                                                                        \
            fprintf(stderr, "%s: status %d (%d)\n", #x, r_, __LINE__);                   \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr int K_DATA = 22, M_PAR = 42, N_ROWS = 64;
constexpr int MT = (8 * M_PAR + 31) / 32;   // 11 M-tiles of 32 parity bits
constexpr int KS = 3;                       // K-steps of 64 (8 data rows each)
constexpr int FRAGS = MT * KS;              // A fragments per lane

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
        b >>= 1;
    }
    return r;
}

__device__ __forceinline__ uint32_t pbits(float v, float magic) {
    return __float_as_uint(v + magic);
}

// grid (ceil(S / 512), count), 256 threads: wave w owns positions
// 512 * blockIdx.x + 128 w .. +127 of instance blockIdx.y
__global__ __launch_bounds__(256) void mfma_encode(uint8_t *__restrict__ slab, uint32_t S,
                                                   uint32_t stride, size_t inst_stride,
                                                   const uint4 *__restrict__ afrag) {
    __shared__ uint4 la[FRAGS * 64];
    for (int i = threadIdx.x; i < FRAGS * 64; i += 256) la[i] = afrag[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    const uint32_t p0 = blockIdx.x * 512 + wave * 128 + 4 * c;   // this lane's 4 positions
    uint8_t *ib = slab + (size_t)blockIdx.y * inst_stride;
    // rows 8t + 4h + i at positions p0..p0+3 (S % 4 == 0, checked on the host)
    uint32_t R[KS][4];
#pragma unroll
    for (int t = 0; t < KS; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 8 * t + 4 * h + i;
            R[t][i] = (r < K_DATA && p0 < S)
                          ? *reinterpret_cast<const uint32_t *>(ib + (size_t)r * stride + p0) : 0u;
        }
    // 4x4 byte transpose: X[t][s] byte i = byte s of R[t][i] (position p0 + s)
    uint32_t X[KS][4];
#pragma unroll
    for (int t = 0; t < KS; ++t) {
        const uint32_t a01 = __builtin_amdgcn_perm(R[t][1], R[t][0], 0x05010400u);  // s0,s1 of rows 0,1
        const uint32_t a23 = __builtin_amdgcn_perm(R[t][3], R[t][2], 0x05010400u);
        const uint32_t b01 = __builtin_amdgcn_perm(R[t][1], R[t][0], 0x07030602u);  // s2,s3
        const uint32_t b23 = __builtin_amdgcn_perm(R[t][3], R[t][2], 0x07030602u);
        X[t][0] = __builtin_amdgcn_perm(a23, a01, 0x05040100u);
        X[t][1] = __builtin_amdgcn_perm(a23, a01, 0x07060302u);
        X[t][2] = __builtin_amdgcn_perm(b23, b01, 0x05040100u);
        X[t][3] = __builtin_amdgcn_perm(b23, b01, 0x07060302u);
    }
    uint32_t outw[MT][4];   // [mt][j]: bytes of row 4 mt + j at positions p0..p0+3
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) outw[mt][j] = 0u;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        v8i B[KS];
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const uint32_t x = X[t][s];
            B[t] = (v8i){(int)(x & 0x33333333u), (int)((x >> 1) & 0x33333333u),
                         (int)((x >> 2) & 0x33333333u), (int)((x >> 3) & 0x33333333u), 0, 0, 0, 0};
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            v16f acc = {};
#pragma unroll
            for (int t = 0; t < KS; ++t) {
                const uint4 a = la[(mt * KS + t) * 64 + lane];
                const v8i A = {(int)a.x, (int)a.y, (int)a.z, (int)a.w, 0, 0, 0, 0};
                // fp4 (4) x fp4 (4); A scale 2^0 (127), B scale 2^1 (128)
                acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B[t], acc, 4, 4, 0, 127, 0,
                                                                      128);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // bit e of p_e = parity of the count of bit 4h + e of row 4 mt + j
                const uint32_t q0 = pbits(acc[4 * j + 0], 8388608.0f);
                const uint32_t q1 = pbits(acc[4 * j + 1], 4194304.0f);
                const uint32_t q2 = pbits(acc[4 * j + 2], 2097152.0f);
                const uint32_t q3 = pbits(acc[4 * j + 3], 1048576.0f);
                // (q0 & 1) | (q1 & ~1) ... merged with constant masks: 3 v_bitop3
                const uint32_t m01 = (q0 & 1u) | (q1 & 2u);
                const uint32_t m23 = (q2 & 4u) | (q3 & 8u);
                uint32_t nib = m01 | m23;
                // the other K-half holds bits 4..7 of the same row and position
                const uint32_t other = (uint32_t)__shfl_xor((int)nib, 32);
                const uint32_t byte = h ? ((other & 15u) | (nib << 4)) : ((nib & 15u) | (other << 4));
                outw[mt][j] |= (byte & 0xFFu) << (8 * s);
            }
        }
    }
    if (p0 >= S) return;
    // lanes of half h store rows j = 2h, 2h + 1 of every M-tile (balanced)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int i = 4 * mt + 2 * h + jj;   // (selects, not a dynamic index)
            const uint32_t v = h ? outw[mt][2 + jj] : outw[mt][jj];
            if (i < M_PAR)
                *reinterpret_cast<uint32_t *>(ib + (size_t)(K_DATA + i) * stride + p0) = v;
        }
}

// counter-PRNG fill of the data rows (device, so 8 GB do not cross PCIe)
__global__ void fill_rows(uint8_t *slab, uint32_t S, uint32_t stride, size_t inst_stride,
                          size_t count) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t per = (size_t)K_DATA * (S / 4);
    if (g >= count * per) return;
    const size_t inst = g / per, w = g - inst * per, r = w / (S / 4), o = (w - r * (S / 4)) * 4;
    uint64_t z = (g + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    *reinterpret_cast<uint32_t *>(slab + inst * inst_stride + r * stride + o) = (uint32_t)z;
}

__global__ void count_diff(const uint8_t *a, const uint8_t *b, size_t n, unsigned long long *d) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g < n / 16) {
        const uint4 x = reinterpret_cast<const uint4 *>(a)[g], y = reinterpret_cast<const uint4 *>(b)[g];
        if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) atomicAdd(d, 1ull);
    }
}

int main(int argc, char **argv) {
    const size_t count = argc > 1 ? (size_t)atol(argv[1]) : 32768;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const uint32_t S = 11916, stride = 11920;   // cfg3: 256 KiB payloads, k = 22
    const size_t inst_stride = (size_t)N_ROWS * stride;
    hbrbc_ctx *ctx = nullptr;
    CL(hbrbc_coding_new(K_DATA, M_PAR, 0, &ctx));
    std::vector<uint8_t> mat((size_t)N_ROWS * K_DATA);
    CL(hbrbc_encoding_matrix(ctx, mat.data()));
    // A fragments: lane l = (row m = l & 31 of the M-tile, K-half h = l >> 5);
    // element e = 8d + 2i + s4 <-> K (data row 8t + 4h + i, bit d + 4 s4)
    std::vector<uint8_t> af((size_t)FRAGS * 64 * 16, 0);
    for (int mt = 0; mt < MT; ++mt)
        for (int t = 0; t < KS; ++t)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 32; ++e) {
                    const int o = 32 * mt + (l & 31), i = o / 8, q = o % 8;
                    const int d = e / 8, bi = (e / 2) % 4, s4 = e % 2;
                    const int r = 8 * t + 4 * (l >> 5) + bi, p = d + 4 * s4;
                    if (i >= M_PAR || r >= K_DATA) continue;
                    const uint8_t cf = mat[(size_t)(K_DATA + i) * K_DATA + r];
                    if ((gmul(cf, (uint8_t)(1u << p)) >> q) & 1)
                        af[(((size_t)mt * KS + t) * 64 + l) * 16 + e / 2] |= (uint8_t)(0x2 << (4 * (e & 1)));
                }
    uint8_t *slab, *ref, *d_af;
    unsigned long long *d_diff;
    const size_t bytes = count * inst_stride;
    CK(hipMalloc(&slab, bytes));
    CK(hipMalloc(&ref, bytes));
    CK(hipMalloc(&d_af, af.size()));
    CK(hipMalloc(&d_diff, 8));
    CK(hipMemcpy(d_af, af.data(), af.size(), hipMemcpyHostToDevice));
    CK(hipMemset(slab, 0, bytes));
    const size_t words = count * K_DATA * (S / 4);
    hipLaunchKernelGGL(fill_rows, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, 0, slab, S,
                       stride, inst_stride, count);
    CK(hipMemcpy(ref, slab, bytes, hipMemcpyDeviceToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto xor_enc = [&] { CL(hbrbc_encode_batch(ctx, ref, S, stride, inst_stride, count, nullptr)); };
    const dim3 grid((S + 511) / 512, (unsigned)count);
    auto mfma_enc = [&] {
        hipLaunchKernelGGL(mfma_encode, grid, dim3(256), 0, 0, slab, S, stride, inst_stride,
                           (const uint4 *)d_af);
    };
    xor_enc();
    mfma_enc();
    CK(hipDeviceSynchronize());
    CK(hipMemset(d_diff, 0, 8));
    hipLaunchKernelGGL(count_diff, dim3((unsigned)((bytes / 16 + 255) / 256)), dim3(256), 0, 0, slab,
                       ref, bytes, d_diff);
    unsigned long long diff = 0;
    CK(hipMemcpy(&diff, d_diff, 8, hipMemcpyDeviceToHost));
    printf("{\"check\": \"mfma parity rows vs libhbrbc encoder\", \"instances\": %zu, "
           "\"differing_16B_chunks\": %llu}\n", count, diff);
    for (int which = 0; which < 2; ++which) {
        float best = 1e30f, sum = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            if (which == 0) xor_enc(); else mfma_enc();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        const double alg = (double)count * (K_DATA + M_PAR) * S;
        printf("{\"encoder\": \"%s\", \"instances\": %zu, \"ms_best\": %.3f, \"ms_mean\": %.3f, "
               "\"alg_GBps\": %.1f}\n", which == 0 ? hbrbc_encode_kernel(ctx) : "mfma_encode fp4",
               count, best, sum / reps, alg / best / 1e6);
    }
    // beside a leaf-hash launch on a second stream (same 64-row slab, other buffer)
    uint8_t *nodes;
    const size_t nc = hbrbc_merkle_node_count(N_ROWS);
    CK(hipMalloc(&nodes, count * nc * 32));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int which = 0; which < 3; ++which) {
        // 0: leaf hash alone; 1: leaf hash + XOR encoder; 2: leaf hash + MFMA encoder
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        CL(hbrbc_merkle_batch(ctx, ref, S, stride, inst_stride, count, nodes, nc * 32, s1));
        if (which == 1) CL(hbrbc_encode_batch(ctx, slab, S, stride, inst_stride, count, s2));
        if (which == 2)
            hipLaunchKernelGGL(mfma_encode, grid, dim3(256), 0, s2, slab, S, stride, inst_stride,
                               (const uint4 *)d_af);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"concurrent\": \"%s\", \"ms\": %.3f}\n",
               which == 0 ? "merkle alone" : which == 1 ? "merkle + xor encoder (2 streams)"
                                                        : "merkle + mfma encoder (2 streams)", ms);
    }
    hbrbc_coding_free(ctx);
    return diff ? 2 : 0;
}
