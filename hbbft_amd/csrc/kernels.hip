// kernels.hip -- HIP kernels (gfx950) of the Reliable-Broadcast data path.
//
// Reference behaviour (yangl1996/hbbft, /root/reference):
//   framing            src/broadcast/broadcast.rs:174-189
//   RS encode          broadcast.rs:193 -> Coding::encode 674-679 (rse encode)
//   Merkle tree        broadcast.rs:204, merkle.rs:20-33, hash/hash_pair 137-150
//   proofs             broadcast.rs:212-222, merkle.rs:36-53
//   Proof::validate    broadcast.rs:604-606, merkle.rs:83-103
//   RS reconstruct     broadcast.rs:569 -> Coding::reconstruct_shards 682-693
//   decode tail        broadcast.rs:580-600 (re-tree, root compare, unframe)
#include "device_common.hpp"
#include "launchers.hpp"

namespace hbrbc {

namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(size_t threads, size_t cap = 256 * 32) {
    size_t b = (threads + kBlock - 1) / kBlock;
    if (b == 0) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

// ----------------------------------------------------------------- frame --
// One thread per dword of every data row (grid-stride).  Logical framed
// byte b (= BE32(len) ++ payload ++ 0s) lives in row b / S at b % S.
__global__ __launch_bounds__(kBlock) void frame_kernel(
    const uint8_t *__restrict__ payloads, size_t payload_stride, uint32_t P, size_t count,
    uint8_t *__restrict__ shards, uint32_t S, size_t shard_stride, size_t inst_stride,
    uint32_t k) {
    const size_t dw_row = shard_stride / 4;
    const size_t total = count * k * dw_row;
    for (size_t idx = blockIdx.x * (size_t)kBlock + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * kBlock) {
        const size_t w = idx % dw_row;
        const size_t row = idx / dw_row;
        const uint32_t j = (uint32_t)(row % k);
        const size_t inst = row / k;
        const uint32_t off = (uint32_t)(4 * w);
        uint32_t val = 0;
        if (off < S) {
            const uint8_t *pay = payloads + inst * payload_stride;
            const uint64_t lb = (uint64_t)j * S + off;  // logical byte of byte 0
            const int nvalid = (int)min(4u, S - off);
            if (lb >= 4) {
                const uint64_t p0 = lb - 4;
                if (p0 < P) {
                    const uint32_t *pw = reinterpret_cast<const uint32_t *>(pay);
                    const uint64_t a0 = p0 >> 2;
                    const uint32_t sh = (uint32_t)(p0 & 3) * 8;
                    uint32_t d0 = pw[a0];
                    uint32_t d1 = (sh != 0 && 4 * (a0 + 1) < P) ? pw[a0 + 1] : 0u;
                    uint32_t v = sh ? __builtin_amdgcn_alignbit(d1, d0, sh) : d0;
                    const uint64_t left = P - p0;
                    const int nb = (int)min<uint64_t>((uint64_t)nvalid, left);
                    if (nb < 4) v &= (nb == 0) ? 0u : (0xFFFFFFFFu >> (8 * (4 - nb)));
                    val = v;
                }
            } else {
                for (int q = 0; q < nvalid; ++q) {
                    const uint64_t b = lb + q;
                    uint32_t byte;
                    if (b < 4)
                        byte = (P >> (8 * (3 - b))) & 0xFFu;
                    else
                        byte = (b - 4 < P) ? pay[b - 4] : 0u;
                    val |= byte << (8 * q);
                }
            }
        }
        reinterpret_cast<uint32_t *>(shards + inst * inst_stride + (size_t)j * shard_stride)[w] =
            val;
    }
}

// -------------------------------------------------------------- GF apply --
// Split-2-bit v_perm_b32 GF(2^8) multiply-accumulate over 16-byte chunks.
// Every lane owns 16 consecutive byte positions of all rows.  Output rows
// are produced RT at a time ("passes"); the tables are pass-major
// [pass][input j][RT] so the RT entries for one input arrive as wide scalar
// loads.  Per (row, input, dword): 4 v_perm_b32 + 2 v_bitop3 (xor3) = 6 VALU
// for 4 byte-MACs.  Rows past `nout` in the last pass carry zero entries;
// only their stores are skipped.
template <int RT>
__global__ __launch_bounds__(kBlock) void gf_apply_kernel(
    uint8_t *__restrict__ base, size_t inst_stride, size_t shard_stride, int n16,
    const uint4 *__restrict__ tables, size_t tab_inst_stride,
    const uint8_t *__restrict__ in_idx, size_t in_idx_stride,
    const uint8_t *__restrict__ out_idx, size_t out_idx_stride,
    const int *__restrict__ nout_arr, int nout_uniform, int nin, int blocks_per_row) {
    const size_t inst = blockIdx.x / blocks_per_row;
    const int chunk0 = (int)(blockIdx.x % blocks_per_row) * kBlock + (int)threadIdx.x;
    const bool active = chunk0 < n16;
    const int chunk = active ? chunk0 : n16 - 1;  // clamped: loads stay in bounds
    uint8_t *ib = base + inst * inst_stride;
    const int nout = nout_arr ? nout_arr[inst] : nout_uniform;
    const int npass = (nout + RT - 1) / RT;
    const uint4 *tab = tables + inst * tab_inst_stride;
    const uint8_t *iidx = in_idx + inst * in_idx_stride;
    const uint8_t *oidx = out_idx + inst * out_idx_stride;
    const size_t off = (size_t)chunk * 16;
    for (int p = 0; p < npass; ++p) {
        uint32_t acc[RT][4];
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[t][d] = 0u;
        const uint4 *tp = tab + (size_t)p * nin * RT;
        uint4 xn = *reinterpret_cast<const uint4 *>(ib + (size_t)iidx[0] * shard_stride + off);
        for (int j = 0; j < nin; ++j) {
            const uint4 x = xn;
            if (j + 1 < nin)
                xn = *reinterpret_cast<const uint4 *>(ib + (size_t)iidx[j + 1] * shard_stride + off);
            const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
            uint32_t sel[4][4];
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int f = 0; f < 4; ++f) sel[f][d] = (xs[d] >> (2 * f)) & 0x03030303u;
            const uint4 *tj = tp + (size_t)j * RT;
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                const uint4 e = tj[t];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    acc[t][d] = xor3(acc[t][d], __builtin_amdgcn_perm(e.x, e.x, sel[0][d]),
                                     __builtin_amdgcn_perm(e.y, e.y, sel[1][d]));
                    acc[t][d] = xor3(acc[t][d], __builtin_amdgcn_perm(e.z, e.z, sel[2][d]),
                                     __builtin_amdgcn_perm(e.w, e.w, sel[3][d]));
                }
            }
        }
        if (active) {
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                if (p * RT + t < nout) {
                    const int dst = oidx[p * RT + t];
                    *reinterpret_cast<uint4 *>(ib + (size_t)dst * shard_stride + off) =
                        make_uint4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
                }
            }
        }
    }
}

// ----------------------------------------------------------- leaf hashes --
// One SHA3-256 sponge per lane: lane g hashes shard (g % n) of instance
// (g / n).  All lanes share the shard length, so every branch is uniform.
__global__ __launch_bounds__(kBlock) void leaf_hash_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, size_t shard_stride, size_t inst_stride,
    uint32_t n, size_t total, uint8_t *__restrict__ nodes, size_t node_inst_stride) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= total) return;
    const size_t inst = g / n;
    const uint32_t i = (uint32_t)(g - inst * n);
    uint32_t d[8];
    sha3_256_row(shards + inst * inst_stride + (size_t)i * shard_stride, S, d);
    store_digest(nodes + inst * node_inst_stride + (size_t)i * 32, d);
}

__global__ __launch_bounds__(kBlock) void ragged_hash_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ lens, size_t nvals, uint8_t *__restrict__ out) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= nvals) return;
    uint32_t d[8];
    sha3_256_row(base + offsets[g], lens[g], d);
    store_digest(out + g * 32, d);
}

// ------------------------------------------------------------ tree level --
__global__ __launch_bounds__(kBlock) void tree_level_kernel(
    uint8_t *__restrict__ nodes, size_t node_inst_stride, uint32_t prev_off, uint32_t prev_size,
    uint32_t cur_off, uint32_t cur_size, size_t count) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= count * cur_size) return;
    const size_t inst = g / cur_size;
    const uint32_t j = (uint32_t)(g - inst * cur_size);
    uint8_t *ns = nodes + inst * node_inst_stride;
    uint32_t a[8], d[8];
    load_digest(ns + (size_t)(prev_off + 2 * j) * 32, a);
    if (2 * j + 1 < prev_size) {
        uint32_t b[8];
        load_digest(ns + (size_t)(prev_off + 2 * j + 1) * 32, b);
        sha3_256_pair(a, b, d);
    } else {
#pragma unroll
        for (int w = 0; w < 8; ++w) d[w] = a[w];  // odd node promoted (merkle.rs:128-134)
    }
    store_digest(ns + (size_t)(cur_off + j) * 32, d);
}

// ---------------------------------------------------------------- proofs --
__global__ __launch_bounds__(kBlock) void proofs_kernel(
    const uint8_t *__restrict__ nodes, size_t node_inst_stride, uint32_t n, size_t count,
    uint8_t *__restrict__ digests, uint32_t dslots, uint8_t *__restrict__ ndig) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= count * n) return;
    const size_t inst = g / n;
    uint32_t i = (uint32_t)(g - inst * n);
    const uint8_t *ns = nodes + inst * node_inst_stride;
    uint8_t *out = digests + g * dslots * 32;
    uint32_t off = 0, sz = n, d = 0;
    while (sz > 1) {
        if ((i ^ 1u) < sz) {
            const uint4 *src = reinterpret_cast<const uint4 *>(ns + (size_t)(off + (i ^ 1u)) * 32);
            uint4 *dst = reinterpret_cast<uint4 *>(out + (size_t)d * 32);
            dst[0] = src[0];
            dst[1] = src[1];
            ++d;
        }
        i >>= 1;
        off += sz;
        sz = (sz + 1) >> 1;
    }
    ndig[g] = (uint8_t)d;
}

// -------------------------------------------------------------- validate --
__global__ __launch_bounds__(kBlock) void validate_kernel(
    const uint8_t *__restrict__ values, uint32_t value_len, size_t value_stride,
    size_t value_inst_stride, uint32_t per_inst, const uint32_t *__restrict__ indices,
    const uint8_t *__restrict__ digests, uint32_t dslots, const uint8_t *__restrict__ ndig,
    const uint8_t *__restrict__ roots, size_t root_stride, uint32_t tree_n, size_t count,
    uint8_t *__restrict__ ok_out) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= count * per_inst) return;
    const size_t inst = g / per_inst;
    const uint32_t j = (uint32_t)(g - inst * per_inst);
    uint32_t d[8];
    sha3_256_row(values + inst * value_inst_stride + (size_t)j * value_stride, value_len, d);
    uint32_t i = indices ? indices[g] : j;
    uint32_t lvl_n = tree_n, used = 0;
    const uint32_t nd = ndig[g];
    const uint8_t *dig = digests + g * dslots * 32;
    bool ok = true;
    while (lvl_n > 1) {
        if ((i ^ 1u) < lvl_n) {
            if (used >= nd) {
                ok = false;  // not enough levels in the proof
                break;
            }
            uint32_t s[8], t[8];
            load_digest(dig + (size_t)used * 32, s);
            ++used;
            if (i & 1u)
                sha3_256_pair(s, d, t);
            else
                sha3_256_pair(d, s, t);
#pragma unroll
            for (int w = 0; w < 8; ++w) d[w] = t[w];
        }
        i >>= 1;
        lvl_n = (lvl_n + 1) >> 1;
    }
    if (used != nd) ok = false;  // too many levels in the proof
    uint32_t r[8];
    load_digest(roots + inst * root_stride, r);
#pragma unroll
    for (int w = 0; w < 8; ++w) ok = ok && (r[w] == d[w]);
    ok_out[g] = ok ? 1 : 0;
}

// --------------------------------------------------------- decode matrix --
// One workgroup per instance: first-k-present selection (rse reconstruct),
// Gauss-Jordan inverse of M[valid] in LDS, recovery rows R = M[missing] *
// inv(M[valid]) (missing data rows are rows of the inverse; missing parity
// rows equal rse's parity-from-rebuilt-data by linearity over GF(2^8)),
// expanded to split-2-bit tables for gf_apply_kernel.
__global__ __launch_bounds__(kBlock) void decode_matrix_kernel(
    int n, int k, int rt, const uint8_t *__restrict__ matrix,
    const uint8_t *__restrict__ present, uint4 *__restrict__ tables,
    uint8_t *__restrict__ in_idx, uint8_t *__restrict__ out_idx, int *__restrict__ nout,
    int32_t *__restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *exp_t = smem;             // 512
    uint8_t *log_t = smem + 512;       // 256
    uint8_t *valid = smem + 768;       // 256
    uint8_t *missing = smem + 1024;    // 256
    uint8_t *fac = smem + 1280;        // 256
    int *meta = reinterpret_cast<int *>(smem + 1536);  // [0]=npresent [1]=nmiss [2]=pivot [3]=inv [4]=singular
    uint8_t *aug = smem + 1600;        // k x 2k
    const int m = n - k;
    const size_t inst = blockIdx.x;
    const int tid = threadIdx.x;
    const uint8_t *pres = present + inst * (size_t)n;

    for (int i = tid; i < 512; i += kBlock) exp_t[i] = kGf.exp[i];
    for (int i = tid; i < 256; i += kBlock) log_t[i] = kGf.log[i];
    if (tid == 0) {
        int np = 0, nm = 0, nv = 0;
        for (int i = 0; i < n; ++i) {
            if (pres[i]) {
                ++np;
                if (nv < k) valid[nv++] = (uint8_t)i;
            } else {
                missing[nm++] = (uint8_t)i;
            }
        }
        meta[0] = np;
        meta[1] = nm;
        meta[4] = 0;
    }
    __syncthreads();
    const int np = meta[0], nm = meta[1];
    if (np == n || np < k) {
        if (tid == 0) {
            nout[inst] = 0;
            status[inst] = (np < k) ? 10 /* TooFewShardsPresent */ : 0;
        }
        return;
    }
    const int w2 = 2 * k;
    for (int e = tid; e < k * w2; e += kBlock) {
        const int r = e / w2, c = e - r * w2;
        aug[e] = (c < k) ? matrix[(size_t)valid[r] * k + c] : (uint8_t)((c - k) == r);
    }
    __syncthreads();
    for (int c = 0; c < k; ++c) {
        if (tid == 0) {
            int p = -1;
            for (int r = c; r < k; ++r)
                if (aug[r * w2 + c]) {
                    p = r;
                    break;
                }
            meta[2] = p;
            if (p < 0)
                meta[4] = 1;
            else
                meta[3] = gf_inv_lds(exp_t, log_t, aug[p * w2 + c]);
        }
        __syncthreads();
        if (meta[4]) {
            if (tid == 0) {
                nout[inst] = 0;
                status[inst] = 64;  // SingularMatrix (impossible for an MDS code)
            }
            return;
        }
        const int p = meta[2];
        const uint8_t inv = (uint8_t)meta[3];
        if (p != c) {
            for (int col = tid; col < w2; col += kBlock) {
                uint8_t t = aug[c * w2 + col];
                aug[c * w2 + col] = aug[p * w2 + col];
                aug[p * w2 + col] = t;
            }
        }
        __syncthreads();
        for (int col = tid; col < w2; col += kBlock)
            aug[c * w2 + col] = gf_mul_lds(exp_t, log_t, inv, aug[c * w2 + col]);
        __syncthreads();
        for (int r = tid; r < k; r += kBlock) fac[r] = (r == c) ? 0 : aug[r * w2 + c];
        __syncthreads();
        for (int e = tid; e < k * w2; e += kBlock) {
            const int r = e / w2, col = e - r * w2;
            const uint8_t f = fac[r];
            if (f) aug[e] ^= gf_mul_lds(exp_t, log_t, f, aug[c * w2 + col]);
        }
        __syncthreads();
    }
    const int npass = (m + rt - 1) / rt;
    uint4 *tab = tables + inst * (size_t)npass * rt * k;
    const int nrows = (nm + rt - 1) / rt * rt;  // pad the last pass with zero rows
    for (int e = tid; e < nrows * k; e += kBlock) {
        const int t = e / k, c = e - t * k;
        const int row = t < nm ? missing[t] : -1;
        uint8_t coef;
        if (row < 0) {
            coef = 0;
        } else if (row < k) {
            coef = aug[row * w2 + k + c];
        } else {
            coef = 0;
            const uint8_t *mr = matrix + (size_t)row * k;
            for (int j = 0; j < k; ++j) coef ^= gf_mul_lds(exp_t, log_t, mr[j], aug[j * w2 + k + c]);
        }
        tab[((size_t)(t / rt) * k + c) * rt + (t % rt)] = gf_split2_entry(coef, exp_t, log_t);
    }
    for (int j = tid; j < k; j += kBlock) in_idx[inst * (size_t)k + j] = valid[j];
    for (int t = tid; t < nm; t += kBlock) out_idx[inst * (size_t)m + t] = missing[t];
    if (tid == 0) {
        nout[inst] = nm;
        status[inst] = 0;
    }
}

// ---------------------------------------------------------- decode check --
__device__ __forceinline__ uint8_t logical_byte(const uint8_t *ib, uint64_t b, uint32_t S,
                                                size_t shard_stride) {
    return ib[(b / S) * shard_stride + (b % S)];
}

__global__ __launch_bounds__(kBlock) void decode_check_kernel(
    const int32_t *__restrict__ recon_status, const uint8_t *__restrict__ nodes,
    size_t node_inst_stride, uint32_t root_node, const uint8_t *__restrict__ roots,
    size_t root_stride, const uint8_t *__restrict__ shards, uint32_t S, size_t shard_stride,
    size_t inst_stride, uint32_t k, size_t count, uint32_t *__restrict__ plen_out,
    int32_t *__restrict__ status_out) {
    const size_t inst = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (inst >= count) return;
    int32_t st = recon_status[inst];
    uint32_t len = 0;
    if (st == 0) {
        uint32_t a[8], b[8];
        load_digest(nodes + inst * node_inst_stride + (size_t)root_node * 32, a);
        load_digest(roots + inst * root_stride, b);
        bool same = true;
#pragma unroll
        for (int w = 0; w < 8; ++w) same = same && a[w] == b[w];
        const uint64_t total = (uint64_t)k * S;
        if (!same) {
            st = 65;  // root mismatch: the proposer is faulty
        } else if (total < 4) {
            st = 66;  // no payload length
        } else {
            const uint8_t *ib = shards + inst * inst_stride;
            uint32_t v = 0;
            for (int q = 0; q < 4; ++q) v = (v << 8) | logical_byte(ib, (uint64_t)q, S, shard_stride);
            len = (uint32_t)min<uint64_t>((uint64_t)v, total - 4);  // take() truncates
        }
    }
    plen_out[inst] = len;
    status_out[inst] = st;
}

// --------------------------------------------------------------- unframe --
// One thread per output dword: logical bytes 4 + 4w .. +3 of the
// concatenated data rows.
__global__ __launch_bounds__(kBlock) void unframe_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, size_t shard_stride, size_t inst_stride,
    uint32_t k, size_t count, const uint32_t *__restrict__ plen,
    const int32_t *__restrict__ status, uint8_t *__restrict__ payload_out,
    size_t payload_stride) {
    const uint64_t total = (uint64_t)k * S;
    const size_t dw_inst = total >= 4 ? (size_t)((total - 4 + 3) / 4) : 0;
    const size_t work = count * dw_inst;
    for (size_t idx = blockIdx.x * (size_t)kBlock + threadIdx.x; idx < work;
         idx += (size_t)gridDim.x * kBlock) {
        const size_t inst = idx / dw_inst;
        const size_t w = idx - inst * dw_inst;
        const uint32_t len = plen[inst];
        if (status[inst] != 0 || 4 * w >= len) continue;
        const uint8_t *ib = shards + inst * inst_stride;
        const uint64_t lb = 4 + 4 * (uint64_t)w;
        const uint32_t row = (uint32_t)(lb / S);
        const uint32_t off = (uint32_t)(lb - (uint64_t)row * S);
        uint32_t v;
        if (off + 4 <= S) {
            const uint32_t *rw = reinterpret_cast<const uint32_t *>(ib + (size_t)row * shard_stride);
            const uint32_t a0 = off >> 2, sh = (off & 3) * 8;
            const uint32_t d0 = rw[a0];
            v = sh ? __builtin_amdgcn_alignbit(rw[a0 + 1], d0, sh) : d0;
        } else {
            v = 0;
            for (int q = 0; q < 4; ++q) {
                const uint64_t b = lb + q;
                if (b < total) v |= (uint32_t)logical_byte(ib, b, S, shard_stride) << (8 * q);
            }
        }
        const uint32_t nb = len - 4 * (uint32_t)w;
        if (nb < 4) v &= 0xFFFFFFFFu >> (8 * (4 - nb));
        reinterpret_cast<uint32_t *>(payload_out + inst * payload_stride)[w] = v;
    }
}

}  // namespace

// ============================================================ launchers ====
hipError_t configure_kernels() {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(decode_matrix_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t launch_frame(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                        size_t count, uint8_t *shards, size_t shard_len, size_t shard_stride,
                        size_t inst_stride, size_t data_shards, hipStream_t s) {
    const size_t threads = count * data_shards * (shard_stride / 4);
    if (threads == 0) return hipSuccess;
    hipLaunchKernelGGL(frame_kernel, dim3(grid_for(threads, 256 * 64)), dim3(kBlock), 0, s,
                       payloads, payload_stride, (uint32_t)payload_len, count, shards,
                       (uint32_t)shard_len, shard_stride, inst_stride, (uint32_t)data_shards);
    return hipGetLastError();
}

hipError_t launch_gf_apply(const GfApplyArgs &a, hipStream_t s) {
    if (a.count == 0 || a.n16 == 0) return hipSuccess;
    if (!a.nout && a.nout_uniform == 0) return hipSuccess;
    const int bpr = (a.n16 + kBlock - 1) / kBlock;
    const size_t blocks = (size_t)bpr * a.count;
#define HB_GF_CASE(RT)                                                                           \
    case RT:                                                                                     \
        hipLaunchKernelGGL(gf_apply_kernel<RT>, dim3((unsigned)blocks), dim3(kBlock), 0, s,      \
                           a.base, a.inst_stride, a.shard_stride, a.n16, a.tables,               \
                           a.tab_inst_stride, a.in_idx, a.in_idx_stride, a.out_idx,              \
                           a.out_idx_stride, a.nout, a.nout_uniform, a.nin, bpr);                \
        break
    switch (a.rt) {
        HB_GF_CASE(2);
        HB_GF_CASE(4);
        HB_GF_CASE(6);
        HB_GF_CASE(8);
        HB_GF_CASE(10);
        HB_GF_CASE(12);
        HB_GF_CASE(14);
        HB_GF_CASE(16);
        default:
            return hipErrorInvalidValue;
    }
#undef HB_GF_CASE
    return hipGetLastError();
}

int gf_row_tile(int rows) {
    if (rows <= 0) return 2;
    const int passes = (rows + 15) / 16;
    int rt = (rows + passes - 1) / passes;
    rt = (rt + 1) & ~1;
    return rt < 2 ? 2 : (rt > 16 ? 16 : rt);
}

hipError_t launch_leaf_hash(const uint8_t *shards, size_t shard_len, size_t shard_stride,
                            size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
                            size_t node_inst_stride, hipStream_t s) {
    const size_t total = n * count;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(leaf_hash_kernel, dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock), 0,
                       s, shards, (uint32_t)shard_len, shard_stride, inst_stride, (uint32_t)n,
                       total, nodes, node_inst_stride);
    return hipGetLastError();
}

hipError_t launch_ragged_hash(const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
                              size_t nvals, uint8_t *out, hipStream_t s) {
    if (nvals == 0) return hipSuccess;
    hipLaunchKernelGGL(ragged_hash_kernel, dim3(grid_for(nvals, (size_t)1 << 30)), dim3(kBlock),
                       0, s, base, offsets, lens, nvals, out);
    return hipGetLastError();
}

hipError_t launch_tree_level(uint8_t *nodes, size_t node_inst_stride, size_t prev_off,
                             size_t prev_size, size_t cur_off, size_t cur_size, size_t count,
                             hipStream_t s) {
    const size_t total = count * cur_size;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(tree_level_kernel, dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock), 0,
                       s, nodes, node_inst_stride, (uint32_t)prev_off, (uint32_t)prev_size,
                       (uint32_t)cur_off, (uint32_t)cur_size, count);
    return hipGetLastError();
}

hipError_t launch_proofs(const uint8_t *nodes, size_t node_inst_stride, size_t n, size_t count,
                         uint8_t *digests, size_t dslots, uint8_t *ndig, hipStream_t s) {
    const size_t total = n * count;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(proofs_kernel, dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock), 0, s,
                       nodes, node_inst_stride, (uint32_t)n, count, digests, (uint32_t)dslots,
                       ndig);
    return hipGetLastError();
}

hipError_t launch_validate(const ValidateArgs &a, hipStream_t s) {
    const size_t total = a.count * a.per_inst;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(validate_kernel, dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock), 0,
                       s, a.values, (uint32_t)a.value_len, a.value_stride, a.value_inst_stride,
                       (uint32_t)a.per_inst, a.indices, a.digests, (uint32_t)a.dslots, a.ndig,
                       a.roots, a.root_stride, (uint32_t)a.tree_n, a.count, a.ok_out);
    return hipGetLastError();
}

hipError_t launch_decode_matrix(const DecodeMatrixArgs &a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const size_t lds = 1600 + (size_t)a.k * 2 * a.k;
    hipLaunchKernelGGL(decode_matrix_kernel, dim3((unsigned)a.count), dim3(kBlock), lds, s, a.n,
                       a.k, a.rt, a.matrix, a.present, a.tables, a.in_idx, a.out_idx, a.nout, a.status);
    return hipGetLastError();
}

hipError_t launch_decode_check(const int32_t *recon_status, const uint8_t *nodes,
                               size_t node_inst_stride, size_t root_node, const uint8_t *roots,
                               size_t root_stride, const uint8_t *shards, size_t shard_len,
                               size_t shard_stride, size_t inst_stride, size_t data_shards,
                               size_t count, uint32_t *plen_out, int32_t *status_out,
                               hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(decode_check_kernel, dim3(grid_for(count, (size_t)1 << 30)), dim3(kBlock),
                       0, s, recon_status, nodes, node_inst_stride, (uint32_t)root_node, roots,
                       root_stride, shards, (uint32_t)shard_len, shard_stride, inst_stride,
                       (uint32_t)data_shards, count, plen_out, status_out);
    return hipGetLastError();
}

hipError_t launch_unframe(const uint8_t *shards, size_t shard_len, size_t shard_stride,
                          size_t inst_stride, size_t data_shards, size_t count,
                          const uint32_t *plen, const int32_t *status, uint8_t *payload_out,
                          size_t payload_stride, hipStream_t s) {
    const uint64_t total = (uint64_t)data_shards * shard_len;
    if (count == 0 || total < 4) return hipSuccess;
    const size_t threads = count * (size_t)((total - 4 + 3) / 4);
    hipLaunchKernelGGL(unframe_kernel, dim3(grid_for(threads, 256 * 64)), dim3(kBlock), 0, s,
                       shards, (uint32_t)shard_len, shard_stride, inst_stride,
                       (uint32_t)data_shards, count, plen, status, payload_out, payload_stride);
    return hipGetLastError();
}

}  // namespace hbrbc
