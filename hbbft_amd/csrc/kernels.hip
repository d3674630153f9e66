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
#include <algorithm>
#include <cstdlib>
#include <cstring>

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
// 16 contiguous bytes (one uint4 store) of 16 consecutive bytes from five aligned dword loads:
// bytes [sh/8, sh/8 + 16) of the 20-byte little-endian window d[0..4].
__device__ __forceinline__ uint4 funnel16(const uint32_t (&d)[5], uint32_t sh) {
    if (sh == 0) return make_uint4(d[0], d[1], d[2], d[3]);
    return make_uint4(__builtin_amdgcn_alignbit(d[1], d[0], sh),
                      __builtin_amdgcn_alignbit(d[2], d[1], sh),
                      __builtin_amdgcn_alignbit(d[3], d[2], sh),
                      __builtin_amdgcn_alignbit(d[4], d[3], sh));
}

// Bytes [SH, SH + 16) of the 32-byte little-endian window (a, b): four
// v_alignbyte_b32, or plain moves when SH is a multiple of 4.
template <int SH>
__device__ __forceinline__ uint4 window16(const uint4 &a, const uint4 &b) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    constexpr int ws = SH >> 2, bs = SH & 3;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (bs == 0)
            o[i] = w[i + ws];
        else
            o[i] = __builtin_amdgcn_alignbyte(w[i + ws + 1], w[i + ws], bs);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// 16 bytes starting `sh` bytes into the 16-byte aligned `src`, from one or two
// coalesced 16-byte loads.  `sh` must be wave-uniform (the switch is scalar)
// and src + 32 readable when sh != 0.
__device__ __forceinline__ uint4 load16_shifted(const uint8_t *src, uint32_t sh) {
    const uint4 a = *reinterpret_cast<const uint4 *>(src);
    if (sh == 0) return a;
    const uint4 b = *reinterpret_cast<const uint4 *>(src + 16);
    switch (sh) {
#define HB_W16(s) \
    case s:       \
        return window16<s>(a, b);
        HB_W16(1) HB_W16(2) HB_W16(3) HB_W16(4) HB_W16(5) HB_W16(6) HB_W16(7) HB_W16(8)
        HB_W16(9) HB_W16(10) HB_W16(11) HB_W16(12) HB_W16(13) HB_W16(14)
#undef HB_W16
        default:
            return window16<15>(a, b);
    }
}

// One thread per 16-byte chunk of every data row; the (instance, row) of a
// workgroup is scalar.  Logical framed byte b (= BE32(len) ++ payload ++ 0s)
// lives in row b / S at b % S (broadcast.rs:174-189); [S, round16(S)) is zeroed.
// Ragged batches (plens != nullptr): instance i frames plens[i] bytes into
// shards of ceil((plens[i] + 4) / k) bytes, and the whole row slot up to
// row_fill is written (zeros past the shard), so one encode over the common
// row length serves every instance.
__global__ __launch_bounds__(kBlock) void frame_kernel(
    const uint8_t *__restrict__ payloads, size_t payload_stride, uint32_t P,
    uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    uint32_t k, uint32_t blocks_per_row, const uint32_t *__restrict__ plens, uint32_t row_fill) {
    const uint32_t grow = blockIdx.x / blocks_per_row;  // instance * k + j
    const uint32_t chunk = (blockIdx.x - grow * blocks_per_row) * kBlock + threadIdx.x;
    const uint32_t off = chunk * 16;
    const size_t inst = grow / k;
    if (plens) {   // P = the batch's maximum: a longer entry would read past its row
        P = min(plens[inst], P);
        S = (P + 4u + k - 1u) / k;
    }
    if (off >= (row_fill ? row_fill : ((S + 15u) & ~15u))) return;
    const uint32_t j = grow - (uint32_t)inst * k;
    uint4 *dst = reinterpret_cast<uint4 *>(shards + inst * inst_stride + rows.off(j) + off);
    if (off >= S) {
        *dst = make_uint4(0, 0, 0, 0);
        return;
    }
    const uint8_t *pay = payloads + inst * payload_stride;
    const uint64_t lb = (uint64_t)j * S + off;  // logical byte of this chunk's first byte
    const bool interior = lb >= 4 && off + 16 <= S && lb - 4 + 16 <= P;
    // Interior chunks of one row share a source misalignment.  When the whole
    // wave agrees, read the payload with aligned 16-byte loads (coalesced) and
    // shift in registers; the aligned window must stay inside the payload row.
    {
        const uintptr_t row0 = reinterpret_cast<uintptr_t>(pay);
        const uintptr_t src = row0 + (interior ? lb - 4 : 0);
        const uint32_t sh = (uint32_t)(src & 15);
        const uintptr_t a0 = src - sh;
        const bool fits = interior && a0 >= row0 && a0 + (sh ? 32 : 16) <= row0 + payload_stride;
        const uint32_t sh0 = __builtin_amdgcn_readfirstlane(sh);
        if (__all(fits && sh == sh0)) {
            *dst = load16_shifted(reinterpret_cast<const uint8_t *>(a0), sh0);
            return;
        }
    }
    if (interior) {
        // every byte is a payload byte: p0 .. p0+15 (all < P, so every dword read is in-row)
        const uint64_t p0 = lb - 4;
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(pay) + (p0 >> 2);
        const uint32_t sh = (uint32_t)(p0 & 3) * 8;
        uint32_t d[5];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = pw[q];
        d[4] = sh ? pw[4] : 0u;
        *dst = funnel16(d, sh);
        return;
    }
    uint32_t w[4] = {0, 0, 0, 0};
    for (int q = 0; q < 16; ++q) {
        if (off + q >= S) break;
        const uint64_t b = lb + q;
        uint32_t byte;
        if (b < 4)
            byte = (P >> (8 * (3 - b))) & 0xFFu;
        else
            byte = (b - 4 < P) ? pay[b - 4] : 0u;
        w[q >> 2] |= byte << (8 * (q & 3));
    }
    *dst = make_uint4(w[0], w[1], w[2], w[3]);
}

// ----------------------------------------------------------- frame fixup --
// The fused frame+encode kernel (jit.hip) reads the payload in whole dwords;
// the last P & 3 payload bytes are added here: each is written into its data
// row and, GF(2^8) being linear, c * byte is XORed into every parity row at
// the same position (c = M[k + r][row]) for parity rows r < m (the rows the
// fused launch computed).  One thread per instance.
__global__ __launch_bounds__(kBlock) void frame_fixup_kernel(
    const uint8_t *__restrict__ payloads, size_t payload_stride, uint32_t P,
    uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    uint32_t k, uint32_t m, const uint8_t *__restrict__ matrix, size_t count) {
    const size_t inst = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (inst >= count) return;
    const uint8_t *pay = payloads + inst * payload_stride;
    uint8_t *ib = shards + inst * inst_stride;
    for (uint32_t t = P & ~3u; t < P; ++t) {
        const uint8_t v = pay[t];
        const uint32_t b = t + 4, j = b / S, pos = b - j * S;
        ib[rows.off(j) + pos] = v;
        if (!v) continue;
        for (uint32_t r = 0; r < m; ++r) {
            const uint8_t c = matrix[(size_t)(k + r) * k + j];
            if (c) ib[rows.off(k + r) + pos] ^= kGf.exp[kGf.log[c] + kGf.log[v]];
        }
    }
}

// 16-byte store of a streamed output (rebuilt rows, payloads), non-temporal:
// unframe 1.82 -> 1.62 ms, reconstruct 3.10 -> 3.05 ms at cfg3 (HB_NT=0
// builds the plain store for A/B).
#ifndef HB_NT
#define HB_NT 1
#endif
typedef unsigned int hb_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_stream(void *p, uint32_t a, uint32_t b, uint32_t c,
                                               uint32_t d) {
#if HB_NT
    __builtin_nontemporal_store((hb_u32x4){a, b, c, d}, reinterpret_cast<hb_u32x4 *>(p));
#else
    *reinterpret_cast<uint4 *>(p) = make_uint4(a, b, c, d);
#endif
}

// ------------------------------------------------------- GF bit-sliced ----
// Bit-sliced GF(2^8) multiply-accumulate.  A lane owns 32 consecutive byte
// positions of every row; its 8 dwords are transposed into 8 bit-planes
// (plane b holds bit b of all 32 bytes; three delta-swap stages exchanging
// the word-index bits with position bits 0..2 -- an involution, so the same
// three stages transpose back).  c*x = XOR over set bits b of c of
// (2^b * x); doubling a bit-sliced value is three plane XORs (x^8 = 0x1D),
// and each set coefficient bit costs 8 full-rate v_xor on 32 positions.
// Coefficients are wave-uniform scalars, so "bit b of c set" is a scalar
// branch: about 1 VALU op per byte-MAC.
__device__ __forceinline__ void bs_transpose(uint32_t (&w)[8]) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int d = 1 << s;
        const uint32_t m = s == 0 ? 0x55555555u : (s == 1 ? 0x33333333u : 0x0F0F0F0Fu);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i & d) continue;
            const uint32_t x = w[i], y = w[i | d];
            const uint32_t t = ((x >> d) ^ y) & m;
            w[i | d] = y ^ t;
            w[i] = x ^ (t << d);
        }
    }
}

// Fused unframe (decode_from_shards, broadcast.rs:590-598): 16 bytes of data
// row `row` at byte `pos` are payload bytes row*S + pos - 4 .. +15.  Only the
// chunks wholly inside the payload are written here, as one 16-byte store at
// any byte alignment (the AMDGPU ABI runs global memory in unaligned mode, and
// hipcc emits global_store_dwordx4 for it).  The edge chunks -- row 0's first
// (the 4-byte length prefix) and each row's partial last chunk, whose bytes
// past S belong to the next row's writer -- are left to unframe_fixup_kernel,
// which copies them from the rebuilt shard rows: byte stores at every call
// site grew this kernel 2.5x and cost 7-20% of the reconstruct at cfg3.
typedef uint32_t hb_u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ void unframe_put(uint8_t *pb, uint32_t S, uint32_t row, uint32_t pos,
                                            uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const int64_t dst = (int64_t)row * S + pos - 4;
    if (pos + 16 <= S && dst >= 0)
        *reinterpret_cast<hb_u32x4_a1 *>(pb + dst) = (hb_u32x4_a1){a, b, c, d};
}

__device__ __forceinline__ uint32_t rfl(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

template <int RT, int MODE>
// Workgroup = up to 4 waves over the SAME 2048 positions; wave w produces
// passes w, w + nwaves, ...  The waves read identical input bytes at the
// same time, so only one copy comes from beyond L1/L2 (a lone wave running
// its passes one after another re-read every input per pass: 3x the HBM/MALL
// traffic at m = 42).  Instance i uses the coefficients and row lists of
// slot pat[i] (the decode-matrix cache) or of slot i / the shared slot 0.
#ifdef HB_GF_WPE   // A/B: waves per SIMD the register budget is cut to
#define HB_GF_ATTR __attribute__((amdgpu_waves_per_eu(HB_GF_WPE)))
#else
#define HB_GF_ATTR
#endif
__global__ __launch_bounds__(256) HB_GF_ATTR void gf_bitslice_kernel(
    uint8_t *__restrict__ base, size_t inst_stride, RowMap rows, uint32_t row_bytes,
    const uint8_t *__restrict__ coefs, size_t coef_slot_stride,
    const uint32_t *__restrict__ in_idx, size_t in_idx_stride,
    const uint32_t *__restrict__ out_idx, size_t out_idx_stride,
    const int *__restrict__ nout_arr, int nout_uniform, const int *__restrict__ pat,
    const uint64_t *__restrict__ slot_hash, uint64_t skip_hash, int hash_slots, int nin,
    uint32_t waves_per_row, uint32_t piece, uint8_t *__restrict__ uf_payload, size_t uf_stride,
    uint32_t uf_S, uint32_t uf_k, const int32_t *__restrict__ uf_status) {
    const size_t inst = blockIdx.x / waves_per_row;
    const int slot = pat ? pat[inst] : (int)inst;
    // instances of a pattern with a specialised decoder are left to it
    if (skip_hash && slot < hash_slots && slot_hash[slot] == skip_hash) return;
    const int wave = (int)(threadIdx.x >> 6), nwaves = (int)(blockDim.x >> 6);
    // a lane's 32 positions: off..off+15 and off+piece..+15.  piece = 1024:
    // every load/store instruction of the wave covers 1 KB of consecutive
    // bytes (16: 64 pieces of 16 B with 16-B gaps, two instructions per line)
    const uint32_t wchunk = blockIdx.x - (uint32_t)inst * waves_per_row, lane = threadIdx.x & 63;
    uint32_t off = piece == 16 ? (wchunk * 64 + lane) * 32 : wchunk * 2048 + lane * 16;
    const bool active = off < row_bytes;
    if (!active) off = row_bytes - 16;              // clamped, loads stay in the row
    const bool full = off + piece + 16 <= row_bytes;  // else only 16 bytes belong to this row
    const uint32_t d2 = full ? piece : 0;
    uint8_t *ib = base + inst * inst_stride;
    const int nout = nout_arr ? nout_arr[slot] : nout_uniform;
    const int npass = (nout + RT - 1) / RT;
    const uint8_t *cf = coefs + (size_t)slot * coef_slot_stride;
    // 32-bit row indices: wave-uniform, so they come through the scalar cache
    // (gfx950 has no sub-dword s_load; byte indices became vector loads whose
    // vmcnt(0) drained the prefetch pipeline)
    const uint32_t *iidx = in_idx + (size_t)slot * in_idx_stride;
    const uint32_t *oidx = out_idx + (size_t)slot * out_idx_stride;
    // fused unframe: payload bytes of the data rows this launch reads (pass 0)
    // or rebuilds; instances whose reconstruct failed are left to the fixup
    uint8_t *ufp = (uf_payload && uf_status[inst] == 0) ? uf_payload + inst * uf_stride : nullptr;
    if (ufp && npass == 0 && wave == 0 && active) {
        // nothing to rebuild: the data rows are rows 0..k-1 as they are
        for (uint32_t r = 0; r < uf_k; ++r) {
            const uint8_t *src = ib + rows.off(r) + off;
            const uint4 l = *reinterpret_cast<const uint4 *>(src);
            unframe_put(ufp, uf_S, r, off, l.x, l.y, l.z, l.w);
            if (full) {
                const uint4 h = *reinterpret_cast<const uint4 *>(src + d2);
                unframe_put(ufp, uf_S, r, off + d2, h.x, h.y, h.z, h.w);
            }
        }
    }
    for (int p = __builtin_amdgcn_readfirstlane(wave); p < npass; p += nwaves) {
        uint32_t acc[RT][8];
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[t][q] = 0u;
        // software pipeline, unrolled by two so no register ever moves: the
        // 32 input bytes of j+1 are in flight (buffer B) while input j
        // (buffer A) is consumed, and vice versa.  A loop-carried copy would
        // force s_waitcnt vmcnt(0) at the top of every iteration.
        const uint4 *cfp = reinterpret_cast<const uint4 *>(cf) + (size_t)p * nin;
        // Loads are unconditional (index clamped, a half chunk re-reads its own
        // 16 bytes) so hipcc can count vmcnt exactly instead of draining.
        auto row_of = [&](int jj) { return iidx[jj < nin ? jj : nin - 1]; };
        auto coef_of = [&](int jj) { return cfp[jj < nin ? jj : nin - 1]; };
        auto load_row = [&](uint32_t r, uint4 &l, uint4 &h) {
            const uint8_t *src = ib + rows.off(r) + off;
            l = *reinterpret_cast<const uint4 *>(src);
            h = *reinterpret_cast<const uint4 *>(src + d2);
        };
        auto consume = [&](uint32_t r, const uint4 &cw, const uint4 &lo, const uint4 &h) {
            const uint4 hi = full ? h : make_uint4(0, 0, 0, 0);
            if (ufp && p == 0) {
                if (r < uf_k && active) {
                    unframe_put(ufp, uf_S, r, off, lo.x, lo.y, lo.z, lo.w);
                    if (full) unframe_put(ufp, uf_S, r, off + d2, hi.x, hi.y, hi.z, hi.w);
                }
            }
            uint32_t x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            bs_transpose(x);
            // RT coefficient bytes of this input for this pass (16-byte padded)
            const uint32_t c4[4] = {cw.x, cw.y, cw.z, cw.w};
            if constexpr (MODE == 3) {
                // Bit pairs (b, b + 1): when both bits of a coefficient are set,
                // one v_bitop3 per plane folds 2^b x and 2^(b+1) x into the
                // accumulator at once (24 instead of 32 VALU per coefficient on
                // average).  Both multiples are live together: the doubling
                // to 2^(b+1) x rewrites only three planes, whose old values are
                // kept in o[] (3 VGPRs).
#pragma unroll
                for (int b = 0; b < 8; b += 2) {
                    const uint32_t h = x[(7 - b) & 7];
                    const uint32_t o[3] = {x[(1 - b) & 7], x[(2 - b) & 7], x[(3 - b) & 7]};
                    x[(1 - b) & 7] ^= h;
                    x[(2 - b) & 7] ^= h;
                    x[(3 - b) & 7] ^= h;
                    // logical plane q of 2^b x (before this doubling)
                    auto lo_plane = [&](int q) {
                        const int i = (q - b) & 7;
                        return i == ((1 - b) & 7) ? o[0] : i == ((2 - b) & 7) ? o[1]
                                                         : i == ((3 - b) & 7) ? o[2] : x[i];
                    };
#pragma unroll
                    for (int t = 0; t < RT; ++t) {
                        const uint32_t two = (c4[t >> 2] >> (8 * (t & 3) + b)) & 3u;
                        if (two == 3u) {
#pragma unroll
                            for (int q = 0; q < 8; ++q) acc[t][q] ^= lo_plane(q) ^ x[(q - b - 1) & 7];
                        } else if (two == 1u) {
#pragma unroll
                            for (int q = 0; q < 8; ++q) acc[t][q] ^= lo_plane(q);
                        } else if (two == 2u) {
#pragma unroll
                            for (int q = 0; q < 8; ++q) acc[t][q] ^= x[(q - b - 1) & 7];
                        }
                    }
                    if (b < 6) {   // to 2^(b+2) x for the next pair
                        const uint32_t h2 = x[(6 - b) & 7];
                        x[(0 - b) & 7] ^= h2;
                        x[(1 - b) & 7] ^= h2;
                        x[(2 - b) & 7] ^= h2;
                    }
                }
                return;
            }
            // At step b the planes of 2^b * x sit rotated: logical plane q is
            // x[(q - b) & 7], so doubling moves no registers, only XORs h into
            // logical planes 2, 3, 4 (x^8 = x^4 + x^3 + x^2 + 1).
#pragma unroll
            for (int b = 0; b < 8; ++b) {
#pragma unroll
                for (int t = 0; t < RT; ++t) {
                    const uint32_t bit = (c4[t >> 2] >> (8 * (t & 3) + b)) & 1u;
                    if constexpr (MODE == 2) {
                        // branch-free: acc ^= x & mask with a wave-uniform mask
                        const uint32_t mask = 0u - bit;
#pragma unroll
                        for (int q = 0; q < 8; ++q)
                            acc[t][q] ^= x[(q - b) & 7] & mask;  // one v_bitop3
                    } else if (MODE == 1 ? __builtin_expect(bit, 1) : bit) {
#pragma unroll
                        for (int q = 0; q < 8; ++q) acc[t][q] ^= x[(q - b) & 7];
                    }
                }
                if (b < 7) {
                    const uint32_t h = x[(7 - b) & 7];  // becomes logical plane 0
                    x[(1 - b) & 7] ^= h;                // -> logical 2
                    x[(2 - b) & 7] ^= h;                // -> logical 3
                    x[(3 - b) & 7] ^= h;                // -> logical 4
                }
            }
        };
        if constexpr (MODE == 4) {
            // Two inputs per step (j, j + 1): each keeps its own rotating
            // doubling, so plane q of 2^b x_j and of 2^b x_j+1 sit in fixed
            // registers side by side and, when bit b of both coefficients is
            // set, one v_xor3 per plane folds both into the accumulator: 6
            // instead of 8 VALU per (row, bit) on average.  (MODE 3 paired
            // two bits of ONE coefficient, whose multiples share registers:
            // copies and 3-way scalar dispatch cost more than it saved.)
            // A missing second input (odd nin) gets coefficient 0: no bit set.
            // A/B (HBRBC_GF=bitslice_x2, rejected): VALU -18 % (1.91 vs 2.32 G
            // per launch) but SALU + branches +33 % (three scalar tests per bit
            // and pair; a nested if / else went back to lane-mask flow blocks
            // and v_mov copies), 115 VGPRs = 4 waves/SIMD instead of 5, and a
            // wave issues one instruction per 4 cycles whatever its kind: the
            // same instruction count per wave, 3.50 vs 3.15 ms at cfg3.
            auto consume2 = [&](uint32_t ra, const uint4 &cwa, const uint4 &la, const uint4 &ha_,
                                uint32_t rb, const uint4 &cwb, const uint4 &lb, const uint4 &hb_,
                                bool two) {
                const uint4 ha = full ? ha_ : make_uint4(0, 0, 0, 0);
                const uint4 hb = full ? hb_ : make_uint4(0, 0, 0, 0);
                if (ufp && p == 0 && active) {
                    if (ra < uf_k) {
                        unframe_put(ufp, uf_S, ra, off, la.x, la.y, la.z, la.w);
                        if (full) unframe_put(ufp, uf_S, ra, off + d2, ha.x, ha.y, ha.z, ha.w);
                    }
                    if (two && rb < uf_k) {
                        unframe_put(ufp, uf_S, rb, off, lb.x, lb.y, lb.z, lb.w);
                        if (full) unframe_put(ufp, uf_S, rb, off + d2, hb.x, hb.y, hb.z, hb.w);
                    }
                }
                uint32_t xa[8] = {la.x, la.y, la.z, la.w, ha.x, ha.y, ha.z, ha.w};
                uint32_t xb[8] = {lb.x, lb.y, lb.z, lb.w, hb.x, hb.y, hb.z, hb.w};
                bs_transpose(xa);
                bs_transpose(xb);
                // wave-uniform: keep the bit tests on the scalar unit
                const uint32_t keep = 0u - (uint32_t)two;
                const uint32_t ca[4] = {rfl(cwa.x), rfl(cwa.y), rfl(cwa.z), rfl(cwa.w)};
                const uint32_t cb[4] = {rfl(cwb.x & keep), rfl(cwb.y & keep), rfl(cwb.z & keep),
                                        rfl(cwb.w & keep)};
                // per coefficient bit: both inputs / only the first / only the second
                uint32_t both[4], oa[4], ob[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    both[w] = ca[w] & cb[w];
                    oa[w] = ca[w] & ~cb[w];
                    ob[w] = cb[w] & ~ca[w];
                }
#pragma unroll
                for (int b = 0; b < 8; ++b) {
#pragma unroll
                    for (int t = 0; t < RT; ++t) {
                        const int sh = 8 * (t & 3) + b;
                        // three one-sided uniform branches on scalar bits (an if /
                        // else chain left the structurizer's flow blocks with v_mov
                        // copies, and && of two bits became lane-mask arithmetic)
                        if ((both[t >> 2] >> sh) & 1u) {
#pragma unroll
                            for (int q = 0; q < 8; ++q)
                                acc[t][q] = xor3(acc[t][q], xa[(q - b) & 7], xb[(q - b) & 7]);
                        }
                        if ((oa[t >> 2] >> sh) & 1u) {
#pragma unroll
                            for (int q = 0; q < 8; ++q) acc[t][q] ^= xa[(q - b) & 7];
                        }
                        if ((ob[t >> 2] >> sh) & 1u) {
#pragma unroll
                            for (int q = 0; q < 8; ++q) acc[t][q] ^= xb[(q - b) & 7];
                        }
                    }
                    if (b < 7) {
                        const uint32_t h = xa[(7 - b) & 7], g = xb[(7 - b) & 7];
                        xa[(1 - b) & 7] ^= h;
                        xa[(2 - b) & 7] ^= h;
                        xa[(3 - b) & 7] ^= h;
                        xb[(1 - b) & 7] ^= g;
                        xb[(2 - b) & 7] ^= g;
                        xb[(3 - b) & 7] ^= g;
                    }
                }
            };
            // the same software pipeline as below, one PAIR of inputs per
            // half-step: pair (j + 2, j + 3) in flight while pair j is consumed
            uint32_t ra0 = row_of(0), ra1 = row_of(1), rb0 = row_of(2), rb1 = row_of(3);
            uint4 ca0 = coef_of(0), ca1 = coef_of(1), cb0, cb1;
            uint32_t orows[RT];
#pragma unroll
            for (int t = 0; t < RT; ++t) orows[t] = oidx[p * RT + t < nout ? p * RT + t : nout - 1];
            uint4 a0l, a0h, a1l, a1h, b0l = make_uint4(0, 0, 0, 0), b0h = b0l, b1l = b0l, b1h = b0l;
            load_row(ra0, a0l, a0h);
            load_row(ra1, a1l, a1h);
            for (int j = 0; j < nin; j += 4) {
                __asm__ volatile("" ::"s"(rb0), "s"(rb1), "s"(ca0.x), "s"(ca0.y), "s"(ca0.z),
                                 "s"(ca0.w), "s"(ca1.x), "s"(ca1.y), "s"(ca1.z), "s"(ca1.w)
                                 : "memory");
                load_row(rb0, b0l, b0h);
                load_row(rb1, b1l, b1h);
                const uint32_t rn0 = row_of(j + 4), rn1 = row_of(j + 5);
                cb0 = coef_of(j + 2);
                cb1 = coef_of(j + 3);
                consume2(ra0, ca0, a0l, a0h, ra1, ca1, a1l, a1h, j + 1 < nin);
                __asm__ volatile("" ::"s"(rn0), "s"(rn1), "s"(cb0.x), "s"(cb0.y), "s"(cb0.z),
                                 "s"(cb0.w), "s"(cb1.x), "s"(cb1.y), "s"(cb1.z), "s"(cb1.w)
                                 : "memory");
                load_row(rn0, a0l, a0h);
                load_row(rn1, a1l, a1h);
                const uint32_t rn2 = row_of(j + 6), rn3 = row_of(j + 7);
                ca0 = coef_of(j + 4);
                ca1 = coef_of(j + 5);
                if (j + 2 < nin)
                    consume2(rb0, cb0, b0l, b0h, rb1, cb1, b1l, b1h, j + 3 < nin);
                ra0 = rn0;
                ra1 = rn1;
                rb0 = rn2;
                rb1 = rn3;
            }
            if (active) {
#pragma unroll
                for (int t = 0; t < RT; ++t) {
                    if (p * RT + t < nout) {
                        bs_transpose(acc[t]);
                        const uint32_t orow = orows[t];
                        uint8_t *dst = ib + rows.off(orow) + off;
                        store16_stream(dst, acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
                        if (full) store16_stream(dst + d2, acc[t][4], acc[t][5], acc[t][6], acc[t][7]);
                        if (ufp && orow < uf_k) {
                            unframe_put(ufp, uf_S, orow, off, acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
                            if (full)
                                unframe_put(ufp, uf_S, orow, off + d2, acc[t][4], acc[t][5], acc[t][6],
                                            acc[t][7]);
                        }
                    }
                }
            }
            continue;
        }
        // Software pipeline, unrolled by two so no register ever moves: the 32
        // input bytes of j+1 are in flight (buffer B) while input j (buffer A)
        // is consumed, and vice versa.  The scalar operands run one input
        // further ahead: the row index of the next load and the coefficients
        // of the next input are requested before this input's XOR work and
        // waited for after it.  (Scalar loads return out of order, so any
        // wait is lgkmcnt(0): the empty asm forces that wait at the top of a
        // half-step, before the next requests go out -- round 3 waited on
        // each index and coefficient load right where it was issued, an L2
        // round trip per input.)
        uint32_t ra = row_of(0), rb = row_of(1);
        uint4 cwa = coef_of(0), cwb;
        // the pass's output rows, requested with the first operands (the
        // stores below would otherwise wait on one scalar load per row)
        uint32_t orows[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) orows[t] = oidx[p * RT + t < nout ? p * RT + t : nout - 1];
        uint4 alo, ahi, blo = make_uint4(0, 0, 0, 0), bhi = make_uint4(0, 0, 0, 0);
        load_row(ra, alo, ahi);
        for (int j = 0; j < nin; j += 2) {
            __asm__ volatile("" ::"s"(rb), "s"(cwa.x), "s"(cwa.y), "s"(cwa.z), "s"(cwa.w) : "memory");
            load_row(rb, blo, bhi);
            const uint32_t rn = row_of(j + 2);
            cwb = coef_of(j + 1);
            consume(ra, cwa, alo, ahi);
            __asm__ volatile("" ::"s"(rn), "s"(cwb.x), "s"(cwb.y), "s"(cwb.z), "s"(cwb.w) : "memory");
            load_row(rn, alo, ahi);
            const uint32_t rn2 = row_of(j + 3);
            cwa = coef_of(j + 2);
            if (j + 1 < nin) consume(rb, cwb, blo, bhi);
            ra = rn;
            rb = rn2;
        }
        if (active) {
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                if (p * RT + t < nout) {
                    bs_transpose(acc[t]);
                    const uint32_t orow = orows[t];
                    uint8_t *dst = ib + rows.off(orow) + off;
                    store16_stream(dst, acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
                    if (full) store16_stream(dst + d2, acc[t][4], acc[t][5], acc[t][6], acc[t][7]);
                    if (ufp && orow < uf_k) {
                        unframe_put(ufp, uf_S, orow, off, acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
                        if (full)
                            unframe_put(ufp, uf_S, orow, off + d2, acc[t][4], acc[t][5], acc[t][6],
                                        acc[t][7]);
                    }
                }
            }
        }
    }
}

// ----------------------------------------------------------- leaf hashes --
// One SHA3-256 sponge per lane: lane g hashes shard (g % n) of instance
// (g / n).  All lanes share the shard length, so every branch is uniform.
// (slens != nullptr: ragged batch, instance i's shards are slens[i] bytes.)
// Sponge kernels: at most 128 VGPRs (4 waves/SIMD, the residency the
// Keccak ceiling was measured at); V16 = few-sponge grids (16-byte loads).
#ifndef HB_SPONGE_WPE
#define HB_SPONGE_WPE 4   // waves/SIMD of the 8-byte-load sponge kernels (A/B: -DHB_SPONGE_WPE)
#endif
#define HB_SPONGE_ATTR __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(V16 ? 1 : HB_SPONGE_WPE)))
template <bool V16>
__global__ HB_SPONGE_ATTR void leaf_hash_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    uint32_t n, size_t total, uint8_t *__restrict__ nodes, size_t node_inst_stride,
    const uint32_t *__restrict__ slens) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= total) return;
    const size_t inst = g / n;
    const uint32_t i = (uint32_t)(g - inst * n);
    if (slens) S = min(slens[inst], (uint32_t)rows.sst);   // never past the row slot
    uint32_t d[8];
    sha3_256_row<V16>(shards + inst * inst_stride + rows.off(i), S, d);
    store_digest(nodes + inst * node_inst_stride + (size_t)i * 32, d);
}

// Leaf hashes and every level of whole trees in one launch (north_star:
// "Merkle levels reduced in LDS"): lane = (instance li of the block, leaf);
// after the sponges the leaf digests go to level 0 of the node slab and to
// LDS, then each level is one pair hash per lane, read from one LDS buffer and
// written to the other and to the slab (merkle.rs:20-33, 128-140: an odd last
// node is promoted unchanged).  A block holds ipb = 256 / n whole instances.
template <bool V16>
__global__ HB_SPONGE_ATTR void merkle_tree_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride, uint32_t n,
    uint32_t ipb, size_t count, uint8_t *__restrict__ nodes, size_t node_inst_stride,
    const uint32_t *__restrict__ slens) {
    __shared__ uint4 lvl[2][kBlock][2];   // two levels of 256 digests: 16 KB
    const uint32_t li = threadIdx.x / n, leaf = threadIdx.x - li * n;
    const size_t inst = (size_t)blockIdx.x * ipb + li;
    const bool active = li < ipb && inst < count;   // no early exit: every lane meets every barrier
    uint8_t *ns = nodes + inst * node_inst_stride;
    if (active) {
        uint32_t d[8];
        sha3_256_row<V16>(shards + inst * inst_stride + rows.off(leaf),
                          slens ? min(slens[inst], (uint32_t)rows.sst) : S, d);
        store_digest(ns + (size_t)leaf * 32, d);
        lvl[0][threadIdx.x][0] = make_uint4(d[0], d[1], d[2], d[3]);
        lvl[0][threadIdx.x][1] = make_uint4(d[4], d[5], d[6], d[7]);
    }
    const uint32_t base = li * n;   // this instance's slots in each level buffer
    uint32_t off = 0, sz = n, cur = 0;
    while (sz > 1) {                // the same trip count in every lane
        __syncthreads();
        const uint32_t nsz = (sz + 1) >> 1;
        if (active && leaf < nsz) {
            const uint4 a0 = lvl[cur][base + 2 * leaf][0], a1 = lvl[cur][base + 2 * leaf][1];
            uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w}, o[8];
            if (2 * leaf + 1 < sz) {
                const uint4 b0 = lvl[cur][base + 2 * leaf + 1][0], b1 = lvl[cur][base + 2 * leaf + 1][1];
                const uint32_t b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                sha3_256_pair(a, b, o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; ++w) o[w] = a[w];
            }
            store_digest(ns + (size_t)(off + sz + leaf) * 32, o);
            lvl[cur ^ 1][base + leaf][0] = make_uint4(o[0], o[1], o[2], o[3]);
            lvl[cur ^ 1][base + leaf][1] = make_uint4(o[4], o[5], o[6], o[7]);
        }
        off += sz;
        sz = nsz;
        cur ^= 1u;
    }
}

// The rows a reconstruct rebuilt, compacted into one list: entry e = (instance,
// row).  One thread per instance appends its slot's out_idx rows.
__global__ __launch_bounds__(kBlock) void rebuilt_list_kernel(
    size_t count, const int *__restrict__ pat, const uint32_t *__restrict__ out_idx,
    size_t out_idx_stride, const int *__restrict__ nout, uint32_t *__restrict__ counter,
    uint2 *__restrict__ list) {
    const size_t inst = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (inst >= count) return;
    const int slot = pat[inst];
    const int no = nout[slot];
    if (no <= 0) return;
    const uint32_t at = atomicAdd(counter, (uint32_t)no);
    const uint32_t *oi = out_idx + (size_t)slot * out_idx_stride;
    for (int t = 0; t < no; ++t) list[at + t] = make_uint2((uint32_t)inst, oi[t]);
}

// SHA3 of the listed rows (a grid sized for the worst case; lanes past the
// list length exit at once, so every wave that hashes is full).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void leaf_hash_list_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    const uint2 *__restrict__ list, const uint32_t *__restrict__ counter,
    uint8_t *__restrict__ nodes, size_t node_inst_stride) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= *counter) return;
    const uint2 e = list[g];
    uint32_t d[8];
    sha3_256_row(shards + e.x * inst_stride + rows.off(e.y), S, d);
    store_digest(nodes + e.x * node_inst_stride + (size_t)e.y * 32, d);
}

// The same, two lanes per sponge (device_common.hpp keccak_f1600_pl), for
// lists far below four waves per SIMD: validator-sharded cfg3 rebuilds 21 rows
// of 4096 instances per step, 86,016 sponges = 1.3 waves per SIMD, where the
// sponge's serial permutation chain -- not issue -- sets the time.
__global__ __launch_bounds__(kBlock) void leaf_hash_list_pl_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    const uint2 *__restrict__ list, const uint32_t *__restrict__ counter,
    uint8_t *__restrict__ nodes, size_t node_inst_stride) {
    const size_t g = (blockIdx.x * (size_t)kBlock + threadIdx.x) >> 1;
    const uint32_t h = threadIdx.x & 1u;
    if (g >= *counter) return;   // both lanes of a pair leave together
    const uint2 e = list[g];
    uint32_t d[8];
    sha3_256_row_pl(shards + e.x * inst_stride + rows.off(e.y), S, h, d);
    if (!h) store_digest(nodes + e.x * node_inst_stride + (size_t)e.y * 32, d);
}

// The same list balanced over the SIMDs.  A sponge is a serial chain, so a
// list is as slow as its busiest SIMD: 86,016 sponges (validator cfg3 / cfg4)
// are 84 per SIMD -- 1.3 one-lane waves, i.e. two waves of 4,395 VALU per
// permutation back to back on a quarter of the SIMDs, or 2.6 pair-lane waves
// rounded up to three of ~2,950.  Here one 512-lane block per CU (8 waves, two
// per SIMD) takes an equal share of the list: whole rounds of 256 sponges on
// waves 0-3, one lane each, and a remainder of at most 128 on waves 4-7, two
// lanes each (a larger remainder is one more one-lane round).  At 84 per SIMD
// a SIMD then runs one wave of each form: 4,395 + 2,950 VALU per permutation.
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void leaf_hash_list_mix_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    const uint2 *__restrict__ list, const uint32_t *__restrict__ counter,
    uint8_t *__restrict__ nodes, size_t node_inst_stride) {
    const uint32_t L = *counter;
    const uint32_t lo = (uint32_t)((uint64_t)blockIdx.x * L / gridDim.x);
    const uint32_t nb = (uint32_t)((uint64_t)(blockIdx.x + 1) * L / gridDim.x) - lo;
    uint32_t d[8];
    if (nb > 384u) {
        // more than one round and a pair-lane remainder per CU (a long list:
        // ADVICE r4): every wave takes one-lane rounds of 512, so no wave
        // idles while waves 0-3 run their rounds back to back
        for (uint32_t t = threadIdx.x; t < nb; t += 512) {
            const uint2 e = list[lo + t];
            sha3_256_row(shards + e.x * inst_stride + rows.off(e.y), S, d);
            store_digest(nodes + e.x * node_inst_stride + (size_t)e.y * 32, d);
        }
        return;
    }
    const uint32_t rem = nb & 255u;
    const uint32_t np = rem <= 128u ? rem : 0u;   // pair-lane sponges of this block
    const uint32_t ns = nb - np;                  // one-lane sponges, in rounds of 256
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave < 4) {
        for (uint32_t t = threadIdx.x; t < ns; t += 256) {
            const uint2 e = list[lo + t];
            sha3_256_row(shards + e.x * inst_stride + rows.off(e.y), S, d);
            store_digest(nodes + e.x * node_inst_stride + (size_t)e.y * 32, d);
        }
        return;
    }
    const uint32_t q = (np + 3) >> 2;   // sponges per pair-lane wave (<= 32)
    const uint32_t pi = (threadIdx.x & 63u) >> 1, h = threadIdx.x & 1u;
    const uint32_t i = (wave - 4) * q + pi;
    if (pi >= q || i >= np) return;     // both lanes of a pair leave together
    const uint2 e = list[lo + ns + i];
    sha3_256_row_pl(shards + e.x * inst_stride + rows.off(e.y), S, h, d);
    if (!h) store_digest(nodes + e.x * node_inst_stride + (size_t)e.y * 32, d);
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void ragged_hash_kernel(
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

// Every level of whole trees in one launch, reduced in LDS (north_star item 4),
// after the leaf-hash kernel has written level 0: lane = (instance li of the
// block, pair t); a block holds ipb = 256 / ceil(n/2) instances.  Level 0 comes
// in from the node slab, each level is one pair hash per lane between two LDS
// buffers and goes out to the slab (odd last node promoted, merkle.rs:128-134).
__global__ __launch_bounds__(kBlock) void tree_levels_kernel(
    uint8_t *__restrict__ nodes, size_t node_inst_stride, uint32_t n, uint32_t half,
    uint32_t ipb, size_t count) {
    __shared__ uint4 lvl[2][2 * kBlock][2];   // two levels of up to 512 digests: 32 KB
    const uint32_t li = threadIdx.x / half, t = threadIdx.x - li * half;
    const size_t inst = (size_t)blockIdx.x * ipb + li;
    const bool active = li < ipb && inst < count;   // every lane meets every barrier
    uint8_t *ns = nodes + inst * node_inst_stride;
    const uint32_t base = li * 2 * half;
    if (active) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint32_t j = 2 * t + e;
            if (j < n) {
                const uint4 *src = reinterpret_cast<const uint4 *>(ns + (size_t)j * 32);
                lvl[0][base + j][0] = src[0];
                lvl[0][base + j][1] = src[1];
            }
        }
    }
    uint32_t off = 0, sz = n, cur = 0;
    while (sz > 1) {                // the same trip count in every lane
        __syncthreads();
        const uint32_t nsz = (sz + 1) >> 1;
        if (active && t < nsz) {
            const uint4 a0 = lvl[cur][base + 2 * t][0], a1 = lvl[cur][base + 2 * t][1];
            uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w}, o[8];
            if (2 * t + 1 < sz) {
                const uint4 b0 = lvl[cur][base + 2 * t + 1][0], b1 = lvl[cur][base + 2 * t + 1][1];
                const uint32_t b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                sha3_256_pair(a, b, o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; ++w) o[w] = a[w];
            }
            store_digest(ns + (size_t)(off + sz + t) * 32, o);
            lvl[cur ^ 1][base + t][0] = make_uint4(o[0], o[1], o[2], o[3]);
            lvl[cur ^ 1][base + t][1] = make_uint4(o[4], o[5], o[6], o[7]);
        }
        off += sz;
        sz = nsz;
        cur ^= 1u;
    }
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
// Proof::validate (merkle.rs:83-103) for proof (i, jj); see ValidateArgs.
template <bool V16>
__global__ HB_SPONGE_ATTR void validate_kernel(
    const uint8_t *__restrict__ values, uint32_t value_len, size_t value_inst_stride,
    RowMap vrows, uint32_t per_inst, const uint32_t *__restrict__ rows,
    const uint32_t *__restrict__ indices, const uint8_t *__restrict__ digests, uint32_t dslots,
    uint32_t dig_rows, const uint8_t *__restrict__ ndig, const uint8_t *__restrict__ roots,
    size_t root_stride, uint32_t tree_n, size_t count, uint8_t *__restrict__ ok_out,
    uint8_t *__restrict__ leaf_out, size_t leaf_inst_stride) {
    const size_t g = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (g >= count * per_inst) return;
    const size_t inst = g / per_inst;
    const uint32_t jj = (uint32_t)(g - inst * per_inst);
    const uint32_t r = rows ? rows[jj] : jj;
    uint32_t d[8];
    sha3_256_row<V16>(values + inst * value_inst_stride + vrows.off(r), value_len, d);
    if (leaf_out) store_digest(leaf_out + inst * leaf_inst_stride + (size_t)r * 32, d);
    uint32_t i = indices ? indices[g] : r;
    uint32_t lvl_n = tree_n, used = 0;
    const size_t ps = inst * dig_rows + (rows ? r : jj);   // proof slot
    const uint32_t nd = ndig[ps];
    const uint8_t *dig = digests + ps * dslots * 32;
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
    uint32_t rt[8];
    load_digest(roots + inst * root_stride, rt);
#pragma unroll
    for (int w = 0; w < 8; ++w) ok = ok && (rt[w] == d[w]);
    ok_out[g] = ok ? 1 : 0;
}

// Pair-lane forms (device_common.hpp keccak_f1600_pl): one sponge on two
// lanes, for grids too small to fill the chip and for the per-call shims
// (HBRBC_SPONGE_PAIR, launch_leaf_hash / launch_validate).
__global__ __launch_bounds__(kBlock) void leaf_hash_pl_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    uint32_t n, size_t total, uint8_t *__restrict__ nodes, size_t node_inst_stride,
    const uint32_t *__restrict__ slens) {
    const size_t g = (blockIdx.x * (size_t)kBlock + threadIdx.x) >> 1;
    const uint32_t h = threadIdx.x & 1u;
    if (g >= total) return;   // both lanes of a pair leave together
    const size_t inst = g / n;
    const uint32_t i = (uint32_t)(g - inst * n);
    if (slens) S = min(slens[inst], (uint32_t)rows.sst);
    uint32_t d[8];
    sha3_256_row_pl(shards + inst * inst_stride + rows.off(i), S, h, d);
    if (!h) store_digest(nodes + inst * node_inst_stride + (size_t)i * 32, d);
}

__global__ __launch_bounds__(kBlock) void validate_pl_kernel(
    const uint8_t *__restrict__ values, uint32_t value_len, size_t value_inst_stride,
    RowMap vrows, uint32_t per_inst, const uint32_t *__restrict__ rows,
    const uint32_t *__restrict__ indices, const uint8_t *__restrict__ digests, uint32_t dslots,
    uint32_t dig_rows, const uint8_t *__restrict__ ndig, const uint8_t *__restrict__ roots,
    size_t root_stride, uint32_t tree_n, size_t count, uint8_t *__restrict__ ok_out,
    uint8_t *__restrict__ leaf_out, size_t leaf_inst_stride) {
    const size_t g = (blockIdx.x * (size_t)kBlock + threadIdx.x) >> 1;
    const uint32_t h = threadIdx.x & 1u;
    if (g >= count * per_inst) return;
    const size_t inst = g / per_inst;
    const uint32_t jj = (uint32_t)(g - inst * per_inst);
    const uint32_t r = rows ? rows[jj] : jj;
    uint32_t d[8];
    sha3_256_row_pl(values + inst * value_inst_stride + vrows.off(r), value_len, h, d);
    if (leaf_out && !h) store_digest(leaf_out + inst * leaf_inst_stride + (size_t)r * 32, d);
    uint32_t i = indices ? indices[g] : r;
    uint32_t lvl_n = tree_n, used = 0;
    const size_t ps = inst * dig_rows + (rows ? r : jj);
    const uint32_t nd = ndig[ps];
    const uint8_t *dig = digests + ps * dslots * 32;
    bool ok = true;
    while (lvl_n > 1) {
        if ((i ^ 1u) < lvl_n) {
            if (used >= nd) {
                ok = false;
                break;
            }
            uint32_t sd[8], t[8];
            load_digest(dig + (size_t)used * 32, sd);
            ++used;
            if (i & 1u)
                sha3_256_pair_pl(sd, d, h, t);
            else
                sha3_256_pair_pl(d, sd, h, t);
#pragma unroll
            for (int w = 0; w < 8; ++w) d[w] = t[w];
        }
        i >>= 1;
        lvl_n = (lvl_n + 1) >> 1;
    }
    if (used != nd) ok = false;
    uint32_t rt[8];
    load_digest(roots + inst * root_stride, rt);
#pragma unroll
    for (int w = 0; w < 8; ++w) ok = ok && (rt[w] == d[w]);
    if (!h) ok_out[g] = ok ? 1 : 0;
}

// --------------------------------------------------- decode-matrix cache --
// Present mask of instance `inst` as 8 words (bit b of word w = present[32w+b]).
__device__ __forceinline__ uint32_t mask_word(const uint8_t *pres, int n, int w) {
    uint32_t v = 0;
    for (int b = 0; b < 32; ++b) {
        const int i = 32 * w + b;
        if (i < n && pres[i]) v |= 1u << b;
    }
    return v;
}

__host__ __device__ __forceinline__ uint64_t pat_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t pat_hash_words(const uint32_t (&w)[8], int n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    for (int i = 0; i < 8; ++i) h = pat_mix(h + ((uint64_t)w[i] << 1) + (uint64_t)i);
    return h ? h : 1ull;
}

// One thread per instance: the slot of its present pattern.  A hit (same
// 64-bit hash) joins the slot; an empty slot is claimed by CAS (this
// instance then computes it); a table at half load or 32 probes without
// success send the instance to its private slot cap + inst.
//
// spec_hash != 0: the hash of the pattern a specialised decoder serves.  The
// decoders (jit.hip guard) and the generic kernel's skip test route by slot
// hash alone, so an instance whose mask collides with that hash but differs
// from spec_mask never enters the table (private slot, generic kernel).
struct SpecKey {
    uint64_t hash;
    uint32_t mask[8];
};
__global__ __launch_bounds__(kBlock) void pattern_lookup_kernel(
    int n, const uint8_t *__restrict__ present, size_t count, PatternCache c,
    int *__restrict__ pat, uint8_t *__restrict__ own, SpecKey spec) {
    const size_t inst = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (inst >= count) return;
    const uint8_t *pres = present + inst * (size_t)n;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = mask_word(pres, n, i);
    const uint64_t h = pat_hash_words(w, n);
    bool spec_collision = false;
    if (spec.hash && h == spec.hash) {
#pragma unroll
        for (int i = 0; i < 8; ++i) spec_collision |= w[i] != spec.mask[i];
    }
    const bool may_insert = *reinterpret_cast<volatile uint32_t *>(c.fill) < (uint32_t)(c.cap / 2);
    int slot = (int)(h & (uint64_t)(c.cap - 1)), found = -1, mine = 0;
    for (int probe = spec_collision ? 32 : 0; probe < 32; ++probe) {
        unsigned long long cur = reinterpret_cast<volatile unsigned long long *>(c.hash)[slot];
        if (cur == 0 && may_insert) {
            cur = atomicCAS(reinterpret_cast<unsigned long long *>(c.hash) + slot, 0ull,
                            (unsigned long long)h);
            if (cur == 0) {
                found = slot;
                mine = 1;
                atomicAdd(c.fill, 1u);
                break;
            }
        }
        if (cur == h) {
            found = slot;
            break;
        }
        if (cur == 0) break;  // empty and full table: not cached
        slot = (slot + 1) & (c.cap - 1);
    }
    if (found < 0) {
        found = c.cap + (int)inst;
        mine = 1;
    }
    if (mine) {
#pragma unroll
        for (int i = 0; i < 8; ++i) c.keys[(size_t)found * 8 + i] = w[i];
    }
    pat[inst] = found;
    own[inst] = (uint8_t)mine;
}

// One workgroup per instance.  Instances that joined a slot verify its key
// (a 64-bit hash collision moves them to their private slot) and stop; the
// instance that owns a slot computes it: first-k-present selection (rse
// reconstruct), Gauss-Jordan inverse of M[valid] in LDS, recovery rows
// M[missing] * inv(M[valid]) (missing data rows are rows of the inverse;
// missing parity rows equal rse's parity-from-rebuilt-data by linearity over
// GF(2^8)), as coefficient bytes [pass][k][16] for gf_bitslice_kernel.
// LDS: 1600 B of tables and lists + d x 2d + d x (k - d) = 1600 + d (d + k),
// d <= min(k, n - k) (launch_decode_matrix sizes it for the largest d).
__global__ __launch_bounds__(1024) void decode_matrix_kernel(
    int n, int k, int rt, const uint8_t *__restrict__ matrix, const uint8_t *__restrict__ present,
    PatternCache c, int *__restrict__ pat, const uint8_t *__restrict__ own) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *exp_t = smem;             // 512
    uint8_t *log_t = smem + 512;       // 256
    uint8_t *valid = smem + 768;       // 256
    uint8_t *missing = smem + 1024;    // 256
    uint8_t *fac = smem + 1280;        // 256
    int *meta = reinterpret_cast<int *>(smem + 1536);  // [0]=npresent [1]=nmiss [2]=pivot [3]=inv [4]=singular [5]=slot [6]=missing data rows
    uint8_t *aug = smem + 1600;        // d x 2d [A | I], then d x (k - d) Ainv B
    const int m = n - k;
    const size_t inst = blockIdx.x;
    const int tid = threadIdx.x;
    const int nt = (int)blockDim.x;  // 64, 256 or 512 threads by k (launch_decode_matrix)
    const uint8_t *pres = present + inst * (size_t)n;
    int slot = pat[inst];
    if (!own[inst]) {
        if (tid < 64) {
            const bool diff = tid < 8 && mask_word(pres, n, tid) != c.keys[(size_t)slot * 8 + tid];
            const unsigned long long bal = __ballot(diff);
            if (tid == 0) meta[5] = bal ? 1 : 0;
        }
        __syncthreads();
        if (!meta[5]) return;          // the slot's owner computes it
        slot = c.cap + (int)inst;      // hash collision: private slot
        if (tid < 8) c.keys[(size_t)slot * 8 + tid] = mask_word(pres, n, tid);
        if (tid == 0) pat[inst] = slot;
    }

    for (int i = tid; i < 512; i += nt) exp_t[i] = kGf.exp[i];
    for (int i = tid; i < 256; i += nt) log_t[i] = kGf.log[i];
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
        int dm = 0;
        while (dm < nm && missing[dm] < k) ++dm;   // missing is ascending: data rows first
        meta[0] = np;
        meta[1] = nm;
        meta[4] = 0;
        meta[6] = dm;
    }
    __syncthreads();
    const int np = meta[0], nm = meta[1];
    if (np == n || np < k) {
        if (tid == 0) {
            c.nout[slot] = 0;
            c.status[slot] = (np < k) ? 10 /* TooFewShardsPresent */ : 0;
        }
        return;
    }
    // rse's decode rows, structured: rows 0..k-1 of the encoding matrix are the
    // identity, and first-k-present gives valid = D ++ P' (the k - d present
    // data rows, then the first d present parity rows), so the d missing data
    // rows solve A x_miss = y_P' + B y_D with A = M[P'][miss], B = M[P'][D]:
    // x_miss = Ainv y_P' + (Ainv B) y_D.  Only the d x d matrix A is inverted
    // (Gauss-Jordan in LDS, d ~ f k / n: 7 at cfg3 instead of 22); the rows are
    // those of inv(M[valid]) (unique), and a missing parity row p is M[p] times
    // them.  (Round 2 inverted all of M[valid], k x 2k.)
    const int d = meta[6], kd = k - d, w2 = 2 * d;
    uint8_t *X = aug + (size_t)d * w2;   // d x kd: Ainv B
    if (d > 0) {
        for (int e = tid; e < d * w2; e += nt) {
            const int r = e / w2, col = e - r * w2;
            aug[e] = (col < d) ? matrix[(size_t)valid[kd + r] * k + missing[col]]
                               : (uint8_t)((col - d) == r);
        }
        __syncthreads();
        for (int col0 = 0; col0 < d; ++col0) {
            if (tid < 64) {   // pivot: first nonzero row at or below col0, by ballot
                int p = -1;
                for (int r0 = col0; r0 < d && p < 0; r0 += 64) {
                    const int r = r0 + tid;
                    const unsigned long long bal = __ballot(r < d && aug[r * w2 + col0] != 0);
                    if (bal) p = r0 + __ffsll((long long)bal) - 1;
                }
                if (tid == 0) meta[2] = p;
            }
            if (tid == 0) {
                const int p = meta[2];
                if (p < 0)
                    meta[4] = 1;
                else
                    meta[3] = gf_inv_lds(exp_t, log_t, aug[p * w2 + col0]);
            }
            __syncthreads();
            if (meta[4]) {
                if (tid == 0) {
                    c.nout[slot] = 0;
                    c.status[slot] = 64;  // SingularMatrix (impossible for an MDS code)
                }
                return;
            }
            const int p = meta[2];
            const uint8_t inv = (uint8_t)meta[3];
            if (p != col0) {
                for (int col = tid; col < w2; col += nt) {
                    uint8_t t = aug[col0 * w2 + col];
                    aug[col0 * w2 + col] = aug[p * w2 + col];
                    aug[p * w2 + col] = t;
                }
            }
            __syncthreads();
            for (int col = tid; col < w2; col += nt)
                aug[col0 * w2 + col] = gf_mul_lds(exp_t, log_t, inv, aug[col0 * w2 + col]);
            __syncthreads();
            for (int r = tid; r < d; r += nt) fac[r] = (r == col0) ? 0 : aug[r * w2 + col0];
            __syncthreads();
            for (int e = tid; e < d * w2; e += nt) {
                const int r = e / w2, col = e - r * w2;
                const uint8_t f = fac[r];
                if (f) aug[e] ^= gf_mul_lds(exp_t, log_t, f, aug[col0 * w2 + col]);
            }
            __syncthreads();
        }
        for (int e = tid; e < d * kd; e += nt) {   // X = Ainv B
            const int i = e / kd, cc = e - i * kd;
            uint8_t acc = 0;
            for (int r = 0; r < d; ++r)
                acc ^= gf_mul_lds(exp_t, log_t, aug[i * w2 + d + r],
                                  matrix[(size_t)valid[kd + r] * k + valid[cc]]);
            X[e] = acc;
        }
        __syncthreads();
    }
    uint8_t *tab = c.coefs + (size_t)slot * c.coef_stride;
    const int nrows = (nm + rt - 1) / rt * rt;  // pad the last pass with zero rows
    for (int e = tid; e < nrows * k; e += nt) {
        const int t = e / k, j = e - t * k;
        const int row = t < nm ? missing[t] : -1;
        uint8_t coef = 0;
        if (row < 0) {
            coef = 0;
        } else if (row < k) {   // missing data row t (t < d)
            coef = j < kd ? X[t * kd + j] : aug[t * w2 + d + (j - kd)];
        } else {                // missing parity row: M[row] times the decode rows
            const uint8_t *mr = matrix + (size_t)row * k;
            if (j < kd) {
                coef = mr[valid[j]];
                for (int i = 0; i < d; ++i) coef ^= gf_mul_lds(exp_t, log_t, mr[missing[i]], X[i * kd + j]);
            } else {
                for (int i = 0; i < d; ++i)
                    coef ^= gf_mul_lds(exp_t, log_t, mr[missing[i]], aug[i * w2 + d + (j - kd)]);
            }
        }
        tab[((size_t)(t / rt) * k + j) * 16 + (t % rt)] = coef;  // [pass][j][16]
    }
    for (int j = tid; j < k; j += nt) c.in_idx[(size_t)slot * k + j] = valid[j];
    for (int t = tid; t < nm; t += nt) c.out_idx[(size_t)slot * m + t] = missing[t];
    if (tid == 0) {
        c.nout[slot] = nm;
        c.status[slot] = 0;
    }
}

__global__ __launch_bounds__(kBlock) void pattern_status_kernel(
    size_t count, const int *__restrict__ pat, const int32_t *__restrict__ slot_status,
    int32_t *__restrict__ status) {
    const size_t inst = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (inst < count) status[inst] = slot_status[pat[inst]];
}

// ---------------------------------------------------------- decode check --
__device__ __forceinline__ uint8_t logical_byte(const uint8_t *ib, uint64_t b, uint32_t S,
                                                const RowMap &rows) {
    // b < k * S < 2^32 at every call site: 32-bit division
    const uint32_t r = (uint32_t)b / S;
    return ib[rows.off(r) + ((uint32_t)b - r * S)];
}

__global__ __launch_bounds__(kBlock) void decode_check_kernel(
    const int32_t *__restrict__ recon_status, const uint8_t *__restrict__ nodes,
    size_t node_inst_stride, uint32_t root_node, const uint8_t *__restrict__ roots,
    size_t root_stride, const uint8_t *__restrict__ shards, uint32_t S, RowMap rows,
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
            for (int q = 0; q < 4; ++q) v = (v << 8) | logical_byte(ib, (uint64_t)q, S, rows);
            len = (uint32_t)min<uint64_t>((uint64_t)v, total - 4);  // take() truncates
        }
    }
    plen_out[inst] = len;
    status_out[inst] = st;
}

// --------------------------------------------------------------- unframe --
// One thread per 16 output bytes (payload bytes 16c..16c+15 = logical bytes
// 4+16c.. of the concatenated data rows, broadcast.rs:590-598); the instance
// of a workgroup is scalar.  Every chunk of the row is written: bytes past
// the decoded length (all of them for a failed instance) are 0.
__global__ __launch_bounds__(kBlock) void unframe_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride,
    uint32_t k, const uint32_t *__restrict__ plen, const int32_t *__restrict__ status,
    uint8_t *__restrict__ payload_out, size_t payload_stride, uint32_t chunks,
    uint32_t blocks_per_inst) {
    const size_t inst = blockIdx.x / blocks_per_inst;
    const uint32_t c = (blockIdx.x - (uint32_t)inst * blocks_per_inst) * kBlock + threadIdx.x;
    if (c >= chunks) return;
    const uint32_t len = status[inst] == 0 ? plen[inst] : 0u;
    const uint32_t o = c * 16;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (o < len) {
        const uint64_t total = (uint64_t)k * S;
        const uint8_t *ib = shards + inst * inst_stride;
        const uint64_t lb = 4 + (uint64_t)o;
        // k * S < 2^32 (checked at launch): a 32-bit division, not the
        // 64-bit software loop (cfg4 unframe 1.27 ms per 8192 instances)
        const uint32_t row = (uint32_t)lb / S;
        const uint32_t off = (uint32_t)lb - row * S;
        // Chunks inside one row share a misalignment: when the wave agrees, two
        // aligned 16-byte loads (coalesced) and a register shift.  off + 16 <= S
        // <= row slot keeps the second 16 bytes inside the row when sh != 0.
        const uint32_t sh = off & 15u;
        const uint32_t sh0 = __builtin_amdgcn_readfirstlane(sh);
        const uint8_t *rp = ib + rows.off(row);
        if (__all(off + 16 <= S && sh == sh0)) {
            const uint4 v = load16_shifted(rp + (off - sh), sh0);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if (off + 16 <= S) {
            // inside one row; the fifth dword ends at most 3 bytes past S (< slot)
            const uint32_t *rw = reinterpret_cast<const uint32_t *>(rp) + (off >> 2);
            const uint32_t s8 = (off & 3) * 8;
            uint32_t d[5];
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = rw[q];
            d[4] = s8 ? rw[4] : 0u;
            const uint4 v = funnel16(d, s8);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {
            for (int q = 0; q < 16; ++q) {
                const uint64_t b = lb + q;
                if (b < total) w[q >> 2] |= (uint32_t)logical_byte(ib, b, S, rows) << (8 * (q & 3));
            }
        }
        const uint32_t nb = len - o;  // bytes of this chunk inside the payload
        if (nb < 16) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int keep = (int)nb - 4 * q;
                if (keep <= 0) w[q] = 0;
                else if (keep < 4) w[q] &= 0xFFFFFFFFu >> (8 * (4 - keep));
            }
        }
    }
    uint32_t *dst = reinterpret_cast<uint32_t *>(payload_out + inst * payload_stride + o);
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        store16_stream(dst, w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = w[q];
    }
}

}  // namespace

// ============================================================ launchers ====
namespace {
int g_num_cus = 256;

// Residency shaping for the lane-per-sponge kernels.  A sponge cannot be
// split, so a grid of T sponges runs in ceil(T / resident) rounds and the
// last round can be mostly idle (cfg3: 524,288 sponges vs 327,680 resident
// lanes at 5 waves/SIMD = 1.6 rounds, 80 % busy).  Pick the waves/SIMD in
// [2, max_w] whose rounds are fullest and enforce it with dynamic LDS (one
// 256-thread block = one wave per SIMD, so blocks/CU = waves/SIMD).
size_t shaped_lds(size_t lanes, int max_w, size_t static_lds = 0) {
    const size_t per_w = (size_t)g_num_cus * kBlock;
    if (lanes >= per_w * (size_t)max_w * 8) return 0;  // many rounds: the tail is small
    int best_w = max_w;
    double best = -1.0;
    for (int w = max_w; w >= 2; --w) {
        const size_t cap = per_w * (size_t)w;
        const size_t rounds = (lanes + cap - 1) / cap;
        const double util = (double)lanes / (double)(rounds * cap);
        if (util > best + 1e-9) {
            best = util;
            best_w = w;
        }
    }
    if (best_w == max_w) return 0;
    return (size_t)(163840 / best_w - static_lds) / 512 * 512;
}
constexpr int kSpongeMaxWaves = 4;  // VGPR-limited residency of the sponge kernels (<= 128 VGPRs)
// Grids below 2^18 sponges (< 4 waves per SIMD) take the 16-byte-load variant.
bool few_sponges(size_t lanes) { return lanes < ((size_t)1 << 18); }
// Pair-lane sponges (two lanes each, ~33 % more VALU per sponge): for grids
// far below one wave per SIMD, where a sponge's serial permutation chain --
// not issue -- sets the time.  Per-call Proof::validate 925 -> 651 us (cfg3
// shard), 3831 -> 2361 us (cfg5); at 65536 sponges (cfg2 leaf hash, one wave
// per SIMD) 22.8 -> 31.5 ms, so only grids below 16384 sponges (r3 A/B,
// profiles/r3_percall.jsonl).  HBRBC_SPONGE_PAIR=0 never, 1 always, 2 below
// HBRBC_SPONGE_PAIR_BELOW sponges (default 2, 16384).
bool pair_sponges(size_t sponges) {
    static const int mode = [] {
        const char *e = getenv("HBRBC_SPONGE_PAIR");
        return e ? atoi(e) : 2;
    }();
    static const size_t below = [] {
        const char *e = getenv("HBRBC_SPONGE_PAIR_BELOW");
        return e ? (size_t)atoll(e) : (size_t)16384;
    }();
    return mode == 1 || (mode == 2 && sponges < below);
}
}  // namespace

void pattern_mask(const uint8_t *present, int n, uint32_t (&w)[8]) {
    for (int i = 0; i < 8; ++i) w[i] = 0;
    for (int i = 0; i < n && i < 256; ++i)
        if (present[i]) w[i / 32] |= 1u << (i % 32);
}

uint64_t pattern_hash(const uint8_t *present, int n) {
    uint32_t w[8];
    pattern_mask(present, n, w);
    return pat_hash_words(w, n);
}

hipError_t configure_kernels() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    for (const void *k : {reinterpret_cast<const void *>(decode_matrix_kernel),
                          reinterpret_cast<const void *>(leaf_hash_kernel<false>),
                          reinterpret_cast<const void *>(leaf_hash_kernel<true>),
                          reinterpret_cast<const void *>(leaf_hash_list_kernel),

                          reinterpret_cast<const void *>(validate_kernel<false>),
                          reinterpret_cast<const void *>(validate_kernel<true>)}) {
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    // (static LDS counts against the same 160 KB)
    for (const void *k : {reinterpret_cast<const void *>(merkle_tree_kernel<false>),
                          reinterpret_cast<const void *>(merkle_tree_kernel<true>)}) {
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024 - 2 * kBlock * 32);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_frame(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                        size_t count, uint8_t *shards, size_t shard_len, const RowMap &rows,
                        size_t inst_stride, size_t data_shards, hipStream_t s,
                        const uint32_t *plens, size_t row_fill) {
    const size_t chunks = ((plens ? row_fill : shard_len) + 15) / 16;
    if (count == 0 || chunks == 0) return hipSuccess;
    const size_t bpr = (chunks + kBlock - 1) / kBlock;
    const size_t blocks = bpr * count * data_shards;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(frame_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, payloads,
                       payload_stride, (uint32_t)payload_len, shards, (uint32_t)shard_len, rows,
                       inst_stride, (uint32_t)data_shards, (uint32_t)bpr, plens,
                       (uint32_t)(plens ? row_fill : 0));
    return hipGetLastError();
}

hipError_t launch_frame_fixup(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                              uint8_t *shards, size_t shard_len, const RowMap &rows,
                              size_t inst_stride, size_t k, size_t m, const uint8_t *matrix,
                              size_t count, hipStream_t s) {
    if (count == 0 || (payload_len & 3) == 0) return hipSuccess;
    hipLaunchKernelGGL(frame_fixup_kernel, dim3(grid_for(count, (size_t)1 << 30)), dim3(kBlock), 0,
                       s, payloads, payload_stride, (uint32_t)payload_len, shards,
                       (uint32_t)shard_len, rows, inst_stride, (uint32_t)k, (uint32_t)m, matrix,
                       count);
    return hipGetLastError();
}

hipError_t launch_gf_apply(const GfApplyArgs &a, hipStream_t s) {
    if (a.count == 0 || a.n16 == 0) return hipSuccess;
    if (!a.nout && a.nout_uniform == 0) return hipSuccess;
    const uint32_t row_bytes = (uint32_t)a.n16 * 16;
    const uint32_t wpr = (row_bytes + 64 * 32 - 1) / (64 * 32);
    const size_t blocks = (size_t)wpr * a.count;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const int max_rows = a.nout ? a.max_rows : a.nout_uniform;
    // waves per block: the fewest that keep the longest wave at the minimum
    // number of passes (a wave beyond an instance's passes exits at once, but
    // its slot in the block idles a SIMD: cfg3, 42 rows at most in 7-row
    // passes, 3 waves instead of 4 -> reconstruct 3.29 -> 3.11-3.17 ms)
    const int npass_max = std::max(1, (max_rows + a.rt - 1) / a.rt);
    const int path = (npass_max + 3) / 4;
    int nw = std::max(1, std::min(4, (npass_max + path - 1) / path));
    // HBRBC_GF_WAVES=1..4: waves per block (A/B; a wave beyond the passes of
    // an instance exits at once)
    if (const char *we = getenv("HBRBC_GF_WAVES")) nw = std::max(1, std::min(4, atoi(we)));
    const char *pe = getenv("HBRBC_GF_SPLIT");   // 0: 32 consecutive bytes per lane (A/B)
    const uint32_t piece = (pe && !strcmp(pe, "0")) ? 16u : 1024u;
#define HB_BS_LAUNCH(RT, MODE)                                                                   \
    hipLaunchKernelGGL((gf_bitslice_kernel<RT, MODE>), dim3((unsigned)blocks), dim3(64 * nw), 0, \
                       s, a.base, a.inst_stride, a.rows, row_bytes, a.coefs, a.coef_slot_stride, \
                       a.in_idx, a.in_idx_stride, a.out_idx, a.out_idx_stride, a.nout,          \
                       a.nout_uniform, a.pat, a.slot_hash, a.skip_hash, a.hash_slots, a.nin, wpr,   \
                       piece, a.payload, a.payload_stride, a.payload_S, a.payload_k, a.rstatus)
#define HB_BS_CASE(RT)                                                                           \
    case RT:                                                                                     \
        if (a.mode == 4)                                                                         \
            HB_BS_LAUNCH(RT, 4);                                                                 \
        else if (a.mode == 3)                                                                    \
            HB_BS_LAUNCH(RT, 3);                                                                 \
        else if (a.mode == 2)                                                                    \
            HB_BS_LAUNCH(RT, 2);                                                                 \
        else if (a.mode == 1)                                                                    \
            HB_BS_LAUNCH(RT, 1);                                                                 \
        else                                                                                     \
            HB_BS_LAUNCH(RT, 0);                                                                 \
        break
    switch (a.rt) {
        HB_BS_CASE(2);
        HB_BS_CASE(4);
        HB_BS_CASE(5);
        HB_BS_CASE(6);
        HB_BS_CASE(7);
        HB_BS_CASE(8);
        HB_BS_CASE(10);
        HB_BS_CASE(12);
        HB_BS_CASE(14);
        HB_BS_CASE(16);
        default:
            return hipErrorInvalidValue;
    }
#undef HB_BS_CASE
#undef HB_BS_LAUNCH
    return hipGetLastError();
}

int gf_row_tile(int rows) {
    if (rows <= 0) return 2;
    const int passes = (rows + 15) / 16;
    int rt = (rows + passes - 1) / passes;
    rt = (rt + 1) & ~1;
    return rt < 2 ? 2 : (rt > 16 ? 16 : rt);
}

hipError_t launch_leaf_hash(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                            size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
                            size_t node_inst_stride, hipStream_t s, const uint32_t *slens) {
    const size_t total = n * count;
    if (total == 0) return hipSuccess;
    if (pair_sponges(total)) {
        hipLaunchKernelGGL(leaf_hash_pl_kernel, dim3(grid_for(2 * total, (size_t)1 << 30)),
                           dim3(kBlock), 0, s, shards, (uint32_t)shard_len, rows, inst_stride,
                           (uint32_t)n, total, nodes, node_inst_stride, slens);
        return hipGetLastError();
    }
    const bool v16 = few_sponges(total);
    hipLaunchKernelGGL(v16 ? leaf_hash_kernel<true> : leaf_hash_kernel<false>,
                       dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock),
                       v16 ? 0 : shaped_lds(total, kSpongeMaxWaves), s, shards, (uint32_t)shard_len,
                       rows, inst_stride, (uint32_t)n, total, nodes, node_inst_stride, slens);
    return hipGetLastError();
}

bool merkle_fused_ok(size_t n) {
    // whole instances per 256-lane block, at most 1/16 of the lanes idle
    return n >= 2 && n <= (size_t)kBlock && (kBlock % n) * 16 <= (size_t)kBlock;
}

hipError_t launch_merkle_fused(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                               size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
                               size_t node_inst_stride, hipStream_t s, const uint32_t *slens) {
    if (count == 0) return hipSuccess;
    if (!merkle_fused_ok(n)) return hipErrorInvalidValue;
    const size_t ipb = kBlock / n;
    const size_t blocks = (count + ipb - 1) / ipb;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const bool v16 = few_sponges(count * n);
    const size_t dyn = v16 ? 0 : shaped_lds(blocks * kBlock, kSpongeMaxWaves, 2 * kBlock * 32);
    hipLaunchKernelGGL(v16 ? merkle_tree_kernel<true> : merkle_tree_kernel<false>, dim3((unsigned)blocks),
                       dim3(kBlock), dyn, s, shards, (uint32_t)shard_len, rows, inst_stride,
                       (uint32_t)n, (uint32_t)ipb, count, nodes, node_inst_stride, slens);
    return hipGetLastError();
}

hipError_t launch_leaf_hash_rebuilt(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                                    size_t inst_stride, size_t count, const int *pat,
                                    const uint32_t *out_idx, size_t out_idx_stride,
                                    const int *nout, int max_rows, uint8_t *nodes,
                                    size_t node_inst_stride, uint32_t *counter, uint2 *list,
                                    hipStream_t s) {
    if (count == 0 || max_rows <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rebuilt_list_kernel, dim3(grid_for(count, (size_t)1 << 30)), dim3(kBlock),
                       0, s, count, pat, out_idx, out_idx_stride, nout, counter, list);
    const size_t total = count * (size_t)max_rows;
    // pair-lane sponges below HBRBC_LIST_PAIR_BELOW rows of the worst case
    // (count x m; the list itself, count x missing rows, is known only on the
    // device -- with f random erasures about half of it).  Default 2^18: the
    // validator-sharded decodes (cfg3 4096 x 42, cfg4 2048 x 84 worst case,
    // half of it listed) pair; the instance-mode leaf reuse (16384 x 42) not.
    static const size_t pair_below = [] {
        const char *e = getenv("HBRBC_LIST_PAIR_BELOW");
        return e ? (size_t)atoll(e) : ((size_t)1 << 18);
    }();
    // below it the balanced form (one block per CU, the split decided on the
    // device from the list length); HBRBC_LIST_FORM=pair: all pair-lane (A/B)
    static const bool form_pair = [] {
        const char *e = getenv("HBRBC_LIST_FORM");
        return e && !strcmp(e, "pair");
    }();
    if (total < pair_below && !form_pair) {
        hipLaunchKernelGGL(leaf_hash_list_mix_kernel, dim3((unsigned)std::max(1, g_num_cus)),
                           dim3(512), 0, s, shards, (uint32_t)shard_len, rows, inst_stride, list,
                           counter, nodes, node_inst_stride);
        return hipGetLastError();
    }
    if (total < pair_below) {
        hipLaunchKernelGGL(leaf_hash_list_pl_kernel, dim3(grid_for(2 * total, (size_t)1 << 30)),
                           dim3(kBlock), 0, s, shards, (uint32_t)shard_len, rows, inst_stride,
                           list, counter, nodes, node_inst_stride);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(leaf_hash_list_kernel, dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock),
                       0, s, shards, (uint32_t)shard_len, rows, inst_stride, list, counter, nodes,
                       node_inst_stride);
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

hipError_t launch_tree_levels(uint8_t *nodes, size_t node_inst_stride, size_t n, size_t count,
                              hipStream_t s) {
    if (count == 0 || n < 2) return hipSuccess;
    if (n > 2 * kBlock) return hipErrorInvalidValue;
    const uint32_t half = (uint32_t)((n + 1) / 2);
    const uint32_t ipb = kBlock / half;
    const size_t blocks = (count + ipb - 1) / ipb;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tree_levels_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, nodes,
                       node_inst_stride, (uint32_t)n, half, ipb, count);
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
    if (pair_sponges(total)) {
        hipLaunchKernelGGL(validate_pl_kernel, dim3(grid_for(2 * total, (size_t)1 << 30)),
                           dim3(kBlock), 0, s, a.values, (uint32_t)a.value_len,
                           a.value_inst_stride, a.vrows, (uint32_t)a.per_inst, a.rows, a.indices,
                           a.digests, (uint32_t)a.dslots, (uint32_t)a.dig_rows, a.ndig, a.roots,
                           a.root_stride, (uint32_t)a.tree_n, a.count, a.ok_out, a.leaf_out,
                           a.leaf_inst_stride);
        return hipGetLastError();
    }
    const bool v16 = few_sponges(total);
    hipLaunchKernelGGL(v16 ? validate_kernel<true> : validate_kernel<false>,
                       dim3(grid_for(total, (size_t)1 << 30)), dim3(kBlock),
                       v16 ? 0 : shaped_lds(total, kSpongeMaxWaves), s, a.values, (uint32_t)a.value_len,
                       a.value_inst_stride, a.vrows, (uint32_t)a.per_inst, a.rows, a.indices,
                       a.digests, (uint32_t)a.dslots, (uint32_t)a.dig_rows, a.ndig, a.roots,
                       a.root_stride, (uint32_t)a.tree_n, a.count, a.ok_out, a.leaf_out,
                       a.leaf_inst_stride);
    return hipGetLastError();
}

hipError_t launch_decode_matrix(const DecodeMatrixArgs &a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    SpecKey spec;
    spec.hash = a.spec_hash;
    for (int i = 0; i < 8; ++i) spec.mask[i] = a.spec_mask[i];
    hipLaunchKernelGGL(pattern_lookup_kernel, dim3(grid_for(a.count, (size_t)1 << 30)),
                       dim3(kBlock), 0, s, a.n, a.present, a.count, a.cache, a.pat, a.own, spec);
    // d missing data rows, d <= min(k, m) (a pattern with more than m missing
    // rows stops at TooFewShardsPresent before the solve)
    const size_t dmax = (size_t)std::min(a.k, a.n - a.k);
    const size_t lds = 1600 + dmax * (dmax + (size_t)a.k);
    // threads per instance by system size (measured per step, round 2, full
    // k x 2k inversion): k = 22 one wave, 0.46 -> 0.34 ms; k = 84 eight waves
    // (four: 1.60, eight: 1.19, sixteen: 1.23 ms).  Round 3 (d x d inversion,
    // cfg4 random patterns): k = 44 two waves (one 0.48, two 0.36, four 0.39).
    // HBRBC_DM_THREADS=64..1024 forces a size.
    static const int force = [] {
        const char *e = getenv("HBRBC_DM_THREADS");
        return e ? atoi(e) : 0;
    }();
    const int threads = (force >= 64 && force <= 1024 && force % 64 == 0) ? force
                                                                         : (a.k <= 32 ? 64 : a.k <= 64 ? 128 : 512);
    hipLaunchKernelGGL(decode_matrix_kernel, dim3((unsigned)a.count), dim3(threads), lds, s, a.n,
                       a.k, a.rt, a.matrix, a.present, a.cache, a.pat, a.own);
    hipLaunchKernelGGL(pattern_status_kernel, dim3(grid_for(a.count, (size_t)1 << 30)),
                       dim3(kBlock), 0, s, a.count, a.pat, a.cache.status, a.status);
    return hipGetLastError();
}

hipError_t launch_decode_check(const int32_t *recon_status, const uint8_t *nodes,
                               size_t node_inst_stride, size_t root_node, const uint8_t *roots,
                               size_t root_stride, const uint8_t *shards, size_t shard_len,
                               const RowMap &rows, size_t inst_stride, size_t data_shards,
                               size_t count, uint32_t *plen_out, int32_t *status_out,
                               hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(decode_check_kernel, dim3(grid_for(count, (size_t)1 << 30)), dim3(kBlock),
                       0, s, recon_status, nodes, node_inst_stride, (uint32_t)root_node, roots,
                       root_stride, shards, (uint32_t)shard_len, rows, inst_stride,
                       (uint32_t)data_shards, count, plen_out, status_out);
    return hipGetLastError();
}

// Fixup after a fused-unframe reconstruct (gf_bitslice_kernel wrote the
// whole 16-byte chunks of payload bytes [0, k*S - 4) of every instance whose
// reconstruct succeeded).  Phase 1 copies the edge bytes below the decoded
// length from the shard rows: row 0's bytes 4..15 and every row's bytes past
// its last whole chunk (S & ~15 .. S-1).  Phase 2 zeroes the bytes past the
// length, or the whole slot of a failed instance, so the payload buffer ends
// exactly as unframe_kernel leaves it.  One workgroup per instance.
__global__ __launch_bounds__(kBlock) void unframe_fixup_kernel(
    const uint8_t *__restrict__ shards, uint32_t S, RowMap rows, size_t inst_stride, uint32_t k,
    uint32_t chunks, const uint32_t *__restrict__ plen, const int32_t *__restrict__ status,
    uint8_t *__restrict__ payload_out, size_t payload_stride) {
    const size_t inst = blockIdx.x;
    const uint32_t len = status[inst] == 0 ? plen[inst] : 0u;
    uint8_t *pb = payload_out + inst * payload_stride;
    if (len) {
        const uint8_t *ib = shards + inst * inst_stride;
        const uint32_t tail0 = S & ~15u;
        for (uint32_t i = threadIdx.x; i < 16 * (k + 1); i += kBlock) {
            const uint32_t r = i < 16 ? 0u : (i - 16) >> 4;
            const uint32_t pos = i < 16 ? i : tail0 + (i & 15);
            const uint32_t p = r * S + pos - 4;   // payload index (k*S < 2^32)
            if (pos < S && r * S + pos >= 4 && p < len) pb[p] = ib[rows.off(r) + pos];
        }
        __syncthreads();
    }
    for (uint32_t c = len / 16 + threadIdx.x; c < chunks; c += kBlock) {
        const uint32_t o = c * 16;
        uint4 *dst = reinterpret_cast<uint4 *>(pb + o);
        if (o >= len) {
            *dst = make_uint4(0, 0, 0, 0);
        } else {
            uint4 v = *dst;
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
            const uint32_t nb = len - o;   // 1..15 payload bytes in this chunk
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int keep = (int)nb - 4 * q;
                if (keep <= 0) w[q] = 0;
                else if (keep < 4) w[q] &= (1u << (8 * keep)) - 1u;
            }
            *dst = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

hipError_t launch_unframe_fixup(const uint8_t *shards, uint32_t S, const RowMap &rows,
                                size_t inst_stride, uint32_t k, size_t count, const uint32_t *plen,
                                const int32_t *status, uint8_t *payload_out, size_t payload_stride,
                                hipStream_t s) {
    const uint64_t total = (uint64_t)k * S;
    if (count == 0 || total <= 4) return hipSuccess;
    if (count > 0x7FFFFFFFull || total + 16 >= ((uint64_t)1 << 32)) return hipErrorInvalidValue;
    const uint32_t chunks = (uint32_t)((total - 4 + 15) / 16);
    hipLaunchKernelGGL(unframe_fixup_kernel, dim3((unsigned)count), dim3(kBlock), 0, s, shards, S,
                       rows, inst_stride, k, chunks, plen, status, payload_out, payload_stride);
    return hipGetLastError();
}

hipError_t launch_unframe(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                          size_t inst_stride, size_t data_shards, size_t count,
                          const uint32_t *plen, const int32_t *status, uint8_t *payload_out,
                          size_t payload_stride, hipStream_t s) {
    const uint64_t total = (uint64_t)data_shards * shard_len;
    if (count == 0 || total <= 4) return hipSuccess;  // nothing past the length prefix
    if (total + 16 >= ((uint64_t)1 << 32)) return hipErrorInvalidValue;   // 32-bit offsets
    const size_t chunks = (size_t)((total - 4 + 15) / 16);
    const size_t bpi = (chunks + kBlock - 1) / kBlock;
    const size_t blocks = bpi * count;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(unframe_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, shards,
                       (uint32_t)shard_len, rows, inst_stride, (uint32_t)data_shards, plen, status,
                       payload_out, payload_stride, (uint32_t)chunks, (uint32_t)bpi);
    return hipGetLastError();
}

// ------------------------------------------------------------- drop rows --
// What a receiver does not hold: every row of instance i with present == 0
// (the shards decode_from_shards gets as None, broadcast.rs:566-571) is
// overwritten with `fill` over its whole slot, so a decode that follows
// really rebuilds it.  One workgroup per instance; the row loop is uniform
// (the present flags are read once into LDS), stores are 16-byte and
// coalesced along the row.
__global__ __launch_bounds__(kBlock) void drop_rows_kernel(
    uint8_t *__restrict__ shards, uint32_t slot16, RowMap rows, size_t inst_stride,
    uint32_t n, const uint8_t *__restrict__ present, uint32_t fill) {
    __shared__ uint8_t pres[256];
    const size_t inst = blockIdx.x;
    for (uint32_t j = threadIdx.x; j < n; j += kBlock) pres[j] = present[inst * n + j];
    __syncthreads();
    const uint4 v = make_uint4(fill, fill, fill, fill);
    uint8_t *ib = shards + inst * inst_stride;
    for (uint32_t j = 0; j < n; ++j) {
        if (pres[j]) continue;
        // plain stores: non-temporal ones measured slower here (cfg3 erase
        // 1.81 -> 1.96 ms, profiles/r5d_bench.json vs r5k_cfg3_trace_bench.json)
        uint4 *row = reinterpret_cast<uint4 *>(ib + rows.off(j));
        for (uint32_t c = threadIdx.x; c < slot16; c += kBlock) row[c] = v;
    }
}

hipError_t launch_drop_rows(uint8_t *shards, size_t shard_stride, const RowMap &rows,
                            size_t inst_stride, size_t n, size_t count, const uint8_t *present,
                            uint8_t fill, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (n > 256 || count > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const uint32_t f4 = 0x01010101u * fill;
    hipLaunchKernelGGL(drop_rows_kernel, dim3((unsigned)count), dim3(kBlock), 0, s, shards,
                       (uint32_t)(shard_stride / 16), rows, inst_stride, (uint32_t)n, present, f4);
    return hipGetLastError();
}

}  // namespace hbrbc

