// device_common.hpp -- gfx950 device building blocks of the RBC data path.
//
//  * Keccak-f[1600] / SHA3-256 (tiny-keccak `Sha3::v256`, used at
//    /root/reference/src/broadcast/merkle.rs:143-150), one sponge per lane.
//    Each 64-bit lane is a (lo, hi) pair of 32-bit VGPRs: rotations are two
//    v_alignbit_b32, theta folds into v_xor3_b32 and chi into v_bitop3_b32
//    (hipcc forms both from the plain expressions below).  ~180 VALU ops per
//    round.
//  * GF(2^8) (reed-solomon-erasure galois_8: poly 0x11D, generator 2) tables
//    built at compile time for the decode-matrix kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbrbc {

// ---------------------------------------------------------------- Keccak --
__constant__ static const uint32_t kRcLo[24] = {
    0x00000001u, 0x00008082u, 0x0000808au, 0x80008000u, 0x0000808bu, 0x80000001u,
    0x80008081u, 0x00008009u, 0x0000008au, 0x00000088u, 0x80008009u, 0x8000000au,
    0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u, 0x00008002u, 0x00000080u,
    0x0000800au, 0x8000000au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ static const uint32_t kRcHi[24] = {
    0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u,
    0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u,
    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u,
    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

// rotl64 of (lo, hi) by a compile-time amount.
template <int R>
__device__ __forceinline__ void rotl64(uint32_t lo, uint32_t hi, uint32_t &ol, uint32_t &oh) {
    if constexpr (R == 0) {
        ol = lo;
        oh = hi;
    } else if constexpr (R == 32) {
        ol = hi;
        oh = lo;
    } else if constexpr (R < 32) {
        oh = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
        ol = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    } else {
        oh = __builtin_amdgcn_alignbit(lo, hi, 64 - R);
        ol = __builtin_amdgcn_alignbit(hi, lo, 64 - R);
    }
}

// rho + pi: B[dst] = rotl(A[src], r)  (FIPS-202 3.2.2 / 3.2.3)
#define HB_RHOPI(src, dst, r) rotl64<r>(L[src], H[src], BL[dst], BH[dst])
#define HB_RHOPI_ALL                                                                             \
    HB_RHOPI(0, 0, 0);                                                                           \
    HB_RHOPI(5, 16, 36);                                                                         \
    HB_RHOPI(10, 7, 3);                                                                          \
    HB_RHOPI(15, 23, 41);                                                                        \
    HB_RHOPI(20, 14, 18);                                                                        \
    HB_RHOPI(1, 10, 1);                                                                          \
    HB_RHOPI(6, 1, 44);                                                                          \
    HB_RHOPI(11, 17, 10);                                                                        \
    HB_RHOPI(16, 8, 45);                                                                         \
    HB_RHOPI(21, 24, 2);                                                                         \
    HB_RHOPI(2, 20, 62);                                                                         \
    HB_RHOPI(7, 11, 6);                                                                          \
    HB_RHOPI(12, 2, 43);                                                                         \
    HB_RHOPI(17, 18, 15);                                                                        \
    HB_RHOPI(22, 9, 61);                                                                         \
    HB_RHOPI(3, 5, 28);                                                                          \
    HB_RHOPI(8, 21, 55);                                                                         \
    HB_RHOPI(13, 12, 25);                                                                        \
    HB_RHOPI(18, 3, 21);                                                                         \
    HB_RHOPI(23, 19, 56);                                                                        \
    HB_RHOPI(4, 15, 27);                                                                         \
    HB_RHOPI(9, 6, 20);                                                                          \
    HB_RHOPI(14, 22, 39);                                                                        \
    HB_RHOPI(19, 13, 8);                                                                         \
    HB_RHOPI(24, 4, 14)

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c in one VALU op
}

// One Keccak-f[1600] permutation on a lane-private state: 180 VALU ops per
// round (theta 20 xor3 + 10 alignbit + 50 xor3, rho 48 alignbit, chi 50
// bitop3, iota 2 xor).
#ifndef HB_KECCAK_UNROLL
#define HB_KECCAK_UNROLL 4  // 4 rounds per loop trip: +4 % over a rolled loop (valu_microbench)
#endif
__device__ __forceinline__ void keccak_f1600(uint32_t (&L)[25], uint32_t (&H)[25]) {
#pragma unroll HB_KECCAK_UNROLL
    for (int round = 0; round < 24; ++round) {
        uint32_t CL[5], CH[5], RL[5], RH[5];
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            CL[x] = xor3(xor3(L[x], L[x + 5], L[x + 10]), L[x + 15], L[x + 20]);
            CH[x] = xor3(xor3(H[x], H[x + 5], H[x + 10]), H[x + 15], H[x + 20]);
        }
#pragma unroll
        for (int x = 0; x < 5; ++x) rotl64<1>(CL[(x + 1) % 5], CH[(x + 1) % 5], RL[x], RH[x]);
#pragma unroll
        for (int i = 0; i < 25; ++i) {
            L[i] = xor3(L[i], CL[(i + 4) % 5], RL[i % 5]);
            H[i] = xor3(H[i], CH[(i + 4) % 5], RH[i % 5]);
        }
        uint32_t BL[25], BH[25];
        HB_RHOPI_ALL;
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
#pragma unroll
            for (int x = 0; x < 5; ++x) {
                L[y + x] = BL[y + x] ^ (~BL[y + (x + 1) % 5] & BL[y + (x + 2) % 5]);
                H[y + x] = BH[y + x] ^ (~BH[y + (x + 1) % 5] & BH[y + (x + 2) % 5]);
            }
        }
        L[0] ^= kRcLo[round];
        H[0] ^= kRcHi[round];
    }
}

// SHA3-256 of `len` bytes at `p` (8-byte aligned; the 8-byte word holding
// the last byte must be readable).  Per-lane pointer and length; when every
// lane of a wave has the same length all branches are wave-uniform.
// V16: the 16-byte-load variant for grids of few sponges (below).  It is a
// separate instantiation: compiled into the same kernel as the 8-byte path
// its two block buffers set the kernel's VGPR count (152 -> 3 waves/SIMD for
// every grid, 130 without it).
#ifndef HB_SPONGE_PF
#define HB_SPONGE_PF 1
#endif
template <bool V16 = false>
__device__ __forceinline__ void sha3_256_row(const uint8_t *__restrict__ p, uint32_t len,
                                             uint32_t (&out)[8]) {
    uint32_t L[25], H[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) L[i] = H[i] = 0u;
    const uint2 *q = reinterpret_cast<const uint2 *>(p);
    const uint32_t nfull = len / 136u;
    // 16-byte-aligned rows (every slab row): block t starts 8*t mod 16 bytes
    // past a 16-byte boundary, so an even block is eight 16-byte loads and
    // one 8-byte load and an odd block one 8-byte load and eight 16-byte
    // loads -- 9 memory instructions per block instead of 17.  Blocks go in
    // pairs, software-pipelined like the 8-byte path below.  Taken only when
    // the grid holds fewer than 4 waves per SIMD (2^18 lanes): there it hides
    // memory latency (cfg2, 65536 rows: leaf hash 23.6 -> 22.8 ms); at full
    // occupancy (cfg3, 1 M rows) it measured 1 % slower than 8-byte loads.
    if (V16 && nfull >= 2 && (reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
        uint4 e[8], o[8];
        uint2 e8, o0;
        auto load_even = [&](const uint2 *b) {
            const uint4 *b4 = reinterpret_cast<const uint4 *>(b);
#pragma unroll
            for (int i = 0; i < 8; ++i) e[i] = b4[i];
            e8 = b[16];
        };
        auto load_odd = [&](const uint2 *b) {
            o0 = b[0];
            const uint4 *b4 = reinterpret_cast<const uint4 *>(b + 1);
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = b4[i];
        };
        load_even(q);
        uint32_t t = 0;
        for (; t + 2 <= nfull; t += 2) {
            load_odd(q + 17);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                L[2 * i] ^= e[i].x;
                H[2 * i] ^= e[i].y;
                L[2 * i + 1] ^= e[i].z;
                H[2 * i + 1] ^= e[i].w;
            }
            L[16] ^= e8.x;
            H[16] ^= e8.y;
            keccak_f1600(L, H);
            q += 34;
            if (t + 3 <= nfull) load_even(q);
            L[0] ^= o0.x;
            H[0] ^= o0.y;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                L[2 * i + 1] ^= o[i].x;
                H[2 * i + 1] ^= o[i].y;
                L[2 * i + 2] ^= o[i].z;
                H[2 * i + 2] ^= o[i].w;
            }
            keccak_f1600(L, H);
        }
        if (t < nfull) {   // one even block left, already loaded
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                L[2 * i] ^= e[i].x;
                H[2 * i] ^= e[i].y;
                L[2 * i + 1] ^= e[i].z;
                H[2 * i + 1] ^= e[i].w;
            }
            L[16] ^= e8.x;
            H[16] ^= e8.y;
            keccak_f1600(L, H);
            q += 17;
        }
    } else
    // Full blocks, software-pipelined: block t+1 is loaded while block t is
    // permuted, so the sponge never waits on memory between permutations
    // (+34 VGPRs; the sponge kernels run at 4 waves/SIMD either way).
    if (nfull) {
#if HB_SPONGE_PF
        uint2 nx[17];
#pragma unroll
        for (int w = 0; w < 17; ++w) nx[w] = q[w];
        for (uint32_t t = 0; t < nfull; ++t) {
#pragma unroll
            for (int w = 0; w < 17; ++w) {
                L[w] ^= nx[w].x;
                H[w] ^= nx[w].y;
            }
            q += 17;
            if (t + 1 < nfull) {
#pragma unroll
                for (int w = 0; w < 17; ++w) nx[w] = q[w];
            }
            keccak_f1600(L, H);
        }
#else
        // no software pipeline: 34 fewer VGPRs, more waves per SIMD hide
        // the load latency instead (HB_SPONGE_PF=0, A/B)
        for (uint32_t t = 0; t < nfull; ++t) {
#pragma unroll
            for (int w = 0; w < 17; ++w) {
                const uint2 v = q[w];
                L[w] ^= v.x;
                H[w] ^= v.y;
            }
            q += 17;
            keccak_f1600(L, H);
        }
#endif
    }
    // last (partial) block + pad10*1 with the SHA3 domain byte 0x06
    const int r = (int)(len - nfull * 136u);
    // issue every tail load before the first use: one memory wait for the
    // block instead of one per 8-byte word
    uint2 tl[17];
#pragma unroll
    for (int w = 0; w < 17; ++w) tl[w] = (r - 8 * w > 0) ? q[w] : make_uint2(0u, 0u);
#pragma unroll
    for (int w = 0; w < 17; ++w) {
        const int rem = r - 8 * w;
        uint64_t v = 0;
        if (rem > 0) {
            v = ((uint64_t)tl[w].y << 32) | tl[w].x;
            if (rem < 8) v &= ~0ull >> (64 - 8 * rem);
        }
        if (rem >= 0 && rem < 8) v ^= 0x06ull << (8 * rem);
        L[w] ^= (uint32_t)v;
        H[w] ^= (uint32_t)(v >> 32);
    }
    H[16] ^= 0x80000000u;
    keccak_f1600(L, H);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        out[2 * w] = L[w];
        out[2 * w + 1] = H[w];
    }
}

// SHA3-256(a ++ b) for two 32-byte digests: one permutation (hash_pair,
// merkle.rs:137-140).
__device__ __forceinline__ void sha3_256_pair(const uint32_t (&a)[8], const uint32_t (&b)[8],
                                              uint32_t (&out)[8]) {
    uint32_t L[25], H[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) L[i] = H[i] = 0u;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        L[w] = a[2 * w];
        H[w] = a[2 * w + 1];
        L[w + 4] = b[2 * w];
        H[w + 4] = b[2 * w + 1];
    }
    L[8] = 0x06u;
    H[16] = 0x80000000u;
    keccak_f1600(L, H);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        out[2 * w] = L[w];
        out[2 * w + 1] = H[w];
    }
}

// ------------------------------------------------ pair-lane Keccak (A/B) --
// One sponge on TWO lanes (north_star "wave-per-leaf" direction, VERDICT r2
// item 6): lane parity h = lane & 1 holds half h of every 64-bit state word
// (h = 0 the low 32 bits).  A 64-bit rotation then needs the partner's half:
// one DPP swap of adjacent lanes (quad_perm [1,0,3,2]) plus one
// v_alignbit per word, the same expression on both lanes:
//   rotl64(w, r) half h = alignbit(mine, partner, 32 - r)      r < 32
//                       = alignbit(partner, mine, 64 - r)      r > 32
// Per lane and round: theta 10 + 25 xor3, 5 + 24 DPP moves, 5 + 24 alignbit,
// chi 25 bitop3, iota 2: ~120 VALU per lane, ~240 per sponge (180 on one
// lane) -- twice the lanes per sponge for grids too small to fill the chip
// and for the latency of a lone sponge (per-call Proof::validate).
__device__ __forceinline__ uint32_t pl_partner(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // lanes 1,0,3,2
}

template <int R>
__device__ __forceinline__ uint32_t pl_rot(uint32_t mine) {
    if constexpr (R == 0) {
        return mine;
    } else {
        const uint32_t other = pl_partner(mine);
        if constexpr (R == 32) return other;
        else if constexpr (R < 32) return __builtin_amdgcn_alignbit(mine, other, 32 - R);
        else return __builtin_amdgcn_alignbit(other, mine, 64 - R);
    }
}

#define HB_PL_RHOPI(src, dst, r) B[dst] = pl_rot<r>(S[src])
__device__ __forceinline__ void keccak_f1600_pl(uint32_t (&S)[25], uint32_t h) {
#pragma unroll HB_KECCAK_UNROLL
    for (int round = 0; round < 24; ++round) {
        uint32_t C[5], D[5];
#pragma unroll
        for (int x = 0; x < 5; ++x) C[x] = xor3(xor3(S[x], S[x + 5], S[x + 10]), S[x + 15], S[x + 20]);
#pragma unroll
        for (int x = 0; x < 5; ++x) D[x] = pl_rot<1>(C[(x + 1) % 5]);
#pragma unroll
        for (int i = 0; i < 25; ++i) S[i] = xor3(S[i], C[(i + 4) % 5], D[i % 5]);
        uint32_t B[25];
        HB_PL_RHOPI(0, 0, 0);
        HB_PL_RHOPI(5, 16, 36);
        HB_PL_RHOPI(10, 7, 3);
        HB_PL_RHOPI(15, 23, 41);
        HB_PL_RHOPI(20, 14, 18);
        HB_PL_RHOPI(1, 10, 1);
        HB_PL_RHOPI(6, 1, 44);
        HB_PL_RHOPI(11, 17, 10);
        HB_PL_RHOPI(16, 8, 45);
        HB_PL_RHOPI(21, 24, 2);
        HB_PL_RHOPI(2, 20, 62);
        HB_PL_RHOPI(7, 11, 6);
        HB_PL_RHOPI(12, 2, 43);
        HB_PL_RHOPI(17, 18, 15);
        HB_PL_RHOPI(22, 9, 61);
        HB_PL_RHOPI(3, 5, 28);
        HB_PL_RHOPI(8, 21, 55);
        HB_PL_RHOPI(13, 12, 25);
        HB_PL_RHOPI(18, 3, 21);
        HB_PL_RHOPI(23, 19, 56);
        HB_PL_RHOPI(4, 15, 27);
        HB_PL_RHOPI(9, 6, 20);
        HB_PL_RHOPI(14, 22, 39);
        HB_PL_RHOPI(19, 13, 8);
        HB_PL_RHOPI(24, 4, 14);
#pragma unroll
        for (int y = 0; y < 25; y += 5)
#pragma unroll
            for (int x = 0; x < 5; ++x) S[y + x] = B[y + x] ^ (~B[y + (x + 1) % 5] & B[y + (x + 2) % 5]);
        S[0] ^= h ? kRcHi[round] : kRcLo[round];
    }
}
#undef HB_PL_RHOPI

// SHA3-256 of `len` bytes at `p` on a lane pair: this lane absorbs half h of
// every 8-byte word (the dword at 8w + 4h); the digest comes out whole on
// both lanes.  Both lanes of a pair take every branch together.
__device__ __forceinline__ void sha3_256_row_pl(const uint8_t *__restrict__ p, uint32_t len,
                                                uint32_t h, uint32_t (&out)[8]) {
    uint32_t S[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) S[i] = 0u;
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p) + h;
    const uint32_t nfull = len / 136u;
    if (nfull) {
        uint32_t nx[17];
#pragma unroll
        for (int w = 0; w < 17; ++w) nx[w] = q[2 * w];
        for (uint32_t t = 0; t < nfull; ++t) {
#pragma unroll
            for (int w = 0; w < 17; ++w) S[w] ^= nx[w];
            q += 34;
            if (t + 1 < nfull) {
#pragma unroll
                for (int w = 0; w < 17; ++w) nx[w] = q[2 * w];
            }
            keccak_f1600_pl(S, h);
        }
    }
    const int r = (int)(len - nfull * 136u);
    const uint8_t *tail = reinterpret_cast<const uint8_t *>(q - h);
#pragma unroll
    for (int w = 0; w < 17; ++w) {
        const int rem = r - 8 * w;   // bytes of this 8-byte word still in the message
        const int mine = rem - 4 * (int)h;   // ... in this lane's half
        uint32_t v = 0;
        if (mine > 0) {
            v = reinterpret_cast<const uint32_t *>(tail)[2 * w + h];
            if (mine < 4) v &= 0xFFFFFFFFu >> (8 * (4 - mine));
        }
        if (mine >= 0 && mine < 4) v ^= 0x06u << (8 * mine);   // domain byte
        S[w] ^= v;
    }
    if (h) S[16] ^= 0x80000000u;
    keccak_f1600_pl(S, h);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t other = pl_partner(S[w]);
        out[2 * w] = h ? other : S[w];
        out[2 * w + 1] = h ? S[w] : other;
    }
}

// SHA3-256(a ++ b) of two digests on a lane pair (hash_pair, merkle.rs:137-140).
__device__ __forceinline__ void sha3_256_pair_pl(const uint32_t (&a)[8], const uint32_t (&b)[8],
                                                 uint32_t h, uint32_t (&out)[8]) {
    uint32_t S[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) S[i] = 0u;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        S[w] = h ? a[2 * w + 1] : a[2 * w];
        S[w + 4] = h ? b[2 * w + 1] : b[2 * w];
    }
    S[8] = h ? 0u : 0x06u;
    S[16] = h ? 0x80000000u : 0u;
    keccak_f1600_pl(S, h);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t other = pl_partner(S[w]);
        out[2 * w] = h ? other : S[w];
        out[2 * w + 1] = h ? S[w] : other;
    }
}

__device__ __forceinline__ void load_digest(const uint8_t *p, uint32_t (&d)[8]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 a = q[0], b = q[1];
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
    d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

__device__ __forceinline__ void store_digest(uint8_t *p, const uint32_t (&d)[8]) {
    uint4 *q = reinterpret_cast<uint4 *>(p);
    q[0] = make_uint4(d[0], d[1], d[2], d[3]);
    q[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// ------------------------------------------------------------- GF(2^8) ----
struct GfTables {
    uint8_t exp[512];
    uint8_t log[256];
    constexpr GfTables() : exp(), log() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            exp[i + 255] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        exp[510] = exp[0];
        exp[511] = exp[1];
        log[0] = 0;
    }
};
__constant__ static const GfTables kGf = GfTables();

__device__ __forceinline__ uint8_t gf_mul_lds(const uint8_t *exp, const uint8_t *log, uint8_t a,
                                              uint8_t b) {
    return (a && b) ? exp[log[a] + log[b]] : (uint8_t)0;
}
__device__ __forceinline__ uint8_t gf_inv_lds(const uint8_t *exp, const uint8_t *log, uint8_t a) {
    return exp[(255 - log[a]) % 255];
}

// Split-2-bit product table entry of a GF constant c: dword f (f = 0..3),
// byte s (s = 0..3) = c * (s << 2f).  v_perm_b32 with per-byte selectors
// ((x >> 2f) & 3) then yields c * x for 4 packed bytes by linearity.
__host__ __device__ inline uint4 gf_split2_entry(uint8_t c, const uint8_t *exp, const uint8_t *log) {
    uint32_t w[4];
    for (int f = 0; f < 4; ++f) {
        uint32_t v = 0;
        for (int s = 0; s < 4; ++s) {
            uint8_t x = (uint8_t)(s << (2 * f));
            uint8_t p = (c && x) ? exp[log[c] + log[x]] : 0;
            v |= (uint32_t)p << (8 * s);
        }
        w[f] = v;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace hbrbc
