// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950
// for the access patterns of this repo's kernels.
// MI355X_MICROARCH.md documents FETCH_SIZE = 1/2 of the bytes only for a
// 16-B/lane coalesced streaming read and calls other widths uncalibrated.
// Each kernel below reads (or writes) a KNOWN byte count from a buffer far
// larger than the 256 MB Infinity Cache, in one access pattern:
//   rows8    one lane per row, 8-byte loads (uint2), 17 per 136-byte Keccak
//            block, rows `stride` bytes apart: the sponge kernels
//            (leaf_hash_kernel / validate_kernel: lane g hashes row g % n of
//            instance g / n; cfg3 rows are 11,916 B in 11,920-B slots)
//   rows16   one lane per row, 16-byte loads (the V16 sponges, cfg2 / cfg5)
//   stream16 coalesced 16 B per lane (the guide's calibrated case)
//   gf16     the GF kernels: a lane's two 16-byte pieces 1 KB apart inside
//            its wave's 2 KB chunk (gf_bitslice_kernel / the XOR networks)
//   stream4  coalesced 4 B per lane
//   write16  coalesced 16-byte stores (WRITE_SIZE)
// tools/fetch_calib.py turns the counter CSVs into raw / known factors.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                     \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

// lane = row; reads `len` bytes (multiple of 8) of its row in 8-byte loads
__global__ __launch_bounds__(256) void calib_rows8(const uint8_t *__restrict__ src, size_t stride,
                                                   uint32_t len, uint32_t rows, uint32_t *out) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const uint2 *p = reinterpret_cast<const uint2 *>(src + (size_t)r * stride);
    uint32_t a = 0, b = 0;
    const uint32_t words = len / 8;
    uint32_t w = 0;
    for (; w + 17 <= words; w += 17) {   // one 136-byte block: 17 independent loads
        uint2 v[17];
#pragma unroll
        for (int t = 0; t < 17; ++t) v[t] = p[w + t];
#pragma unroll
        for (int t = 0; t < 17; ++t) {
            a ^= v[t].x;
            b = (b ^ v[t].y) * 3u;
        }
    }
    for (; w < words; ++w) {
        const uint2 v = p[w];
        a ^= v.x;
        b = (b ^ v.y) * 3u;
    }
    out[r] = a + b;
}

// lane = row; 16-byte loads (the V16 sponge form for grids of few sponges:
// cfg2 / cfg5, leaf_hash_kernel<true> / validate_kernel<true>)
__global__ __launch_bounds__(256) void calib_rows16(const uint8_t *__restrict__ src, size_t stride,
                                                    uint32_t len, uint32_t rows, uint32_t *out) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const uint4 *p = reinterpret_cast<const uint4 *>(src + (size_t)r * stride);
    uint32_t a = 0, b = 0;
    const uint32_t words = len / 16;
    uint32_t w = 0;
    for (; w + 8 <= words; w += 8) {
        uint4 v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = p[w + t];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            a ^= v[t].x ^ v[t].z;
            b = (b ^ v[t].y ^ v[t].w) * 3u;
        }
    }
    for (; w < words; ++w) {
        const uint4 v = p[w];
        a ^= v.x ^ v.z;
        b = (b ^ v.y ^ v.w) * 3u;
    }
    out[r] = a + b;
}

__global__ __launch_bounds__(256) void calib_stream16(const uint4 *__restrict__ src, size_t n16,
                                                      uint32_t *out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = src[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

// one wave per 2 KB chunk; lane l reads bytes [16l, 16l+16) and [1024+16l, ...)
__global__ __launch_bounds__(256) void calib_gf16(const uint8_t *__restrict__ src, size_t chunks,
                                                  uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t a = 0;
    for (size_t c = (blockIdx.x * 256 + threadIdx.x) / 64; c < chunks;
         c += (size_t)gridDim.x * 4) {
        const uint4 *p = reinterpret_cast<const uint4 *>(src + c * 2048 + lane * 16);
        const uint4 v0 = p[0], v1 = p[64];
        a ^= v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

__global__ __launch_bounds__(256) void calib_stream4(const uint32_t *__restrict__ src, size_t n4,
                                                     uint32_t *out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        a ^= src[i];
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

__global__ __launch_bounds__(256) void calib_write16(uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint32_t x = (uint32_t)i;
        dst[i] = make_uint4(x, x ^ 1u, x ^ 2u, x ^ 3u);
    }
}

int main(int argc, char **argv) {
    const size_t bytes = (size_t)4 << 30;          // 16x the Infinity Cache
    uint8_t *buf;
    uint32_t *out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0x3c, bytes));
    const int grid = 256 * 16;
    CHECK(hipMalloc(&out, (size_t)8 << 20));
    // rows8 at the cfg3 row geometry: 11,916 B rows (87 blocks of 136 + 84 B;
    // the kernel reads 11,912 = whole 8-byte words) in 11,920-B slots
    const size_t stride = 11920;
    const uint32_t len = 11912;
    const uint32_t rows = (uint32_t)(bytes / stride) / 64 * 64;
    // rows16 at the cfg5 row geometry: 49,933-B rows in 49,936-B slots
    const size_t stride16 = 49936;
    const uint32_t len16 = 49920;
    const uint32_t rows16 = (uint32_t)(bytes / stride16) / 64 * 64;
    const int reps = 3;
    for (int rep = 0; rep < reps; ++rep) {
        hipLaunchKernelGGL(calib_rows8, dim3((rows + 255) / 256), dim3(256), 0, 0, buf, stride, len,
                           rows, out);
        hipLaunchKernelGGL(calib_rows16, dim3((rows16 + 255) / 256), dim3(256), 0, 0, buf, stride16,
                           len16, rows16, out);
        hipLaunchKernelGGL(calib_stream16, dim3(grid), dim3(256), 0, 0,
                           reinterpret_cast<const uint4 *>(buf), bytes / 16, out);
        hipLaunchKernelGGL(calib_gf16, dim3(grid), dim3(256), 0, 0, buf, bytes / 2048, out);
        hipLaunchKernelGGL(calib_stream4, dim3(grid), dim3(256), 0, 0,
                           reinterpret_cast<const uint32_t *>(buf), bytes / 4, out);
        hipLaunchKernelGGL(calib_write16, dim3(grid), dim3(256), 0, 0, reinterpret_cast<uint4 *>(buf),
                           bytes / 16);
    }
    CHECK(hipDeviceSynchronize());
    // known bytes per launch, read by tools/fetch_calib.py
    printf("{\"calib_rows8\": {\"read\": %zu, \"write\": %zu, \"rows\": %u, \"stride\": %zu, "
           "\"len\": %u},\n", (size_t)rows * len, (size_t)rows * 4, rows, stride, len);
    printf(" \"calib_rows16\": {\"read\": %zu, \"write\": %zu, \"rows\": %u, \"stride\": %zu, "
           "\"len\": %u},\n", (size_t)rows16 * len16, (size_t)rows16 * 4, rows16, stride16, len16);
    printf(" \"calib_stream16\": {\"read\": %zu, \"write\": %zu},\n", bytes, (size_t)grid * 256 * 4);
    printf(" \"calib_gf16\": {\"read\": %zu, \"write\": %zu},\n", bytes, (size_t)grid * 256 * 4);
    printf(" \"calib_stream4\": {\"read\": %zu, \"write\": %zu},\n", bytes, (size_t)grid * 256 * 4);
    printf(" \"calib_write16\": {\"read\": 0, \"write\": %zu}}\n", bytes);
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    (void)argc;
    (void)argv;
    return 0;
}
