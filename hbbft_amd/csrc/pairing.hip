// pairing.hip -- batched BLS12-381 pairing checks for threshold-decrypt share
// verification.
//
// Reference: /root/reference/src/threshold_decrypt.rs:142 (`ct.verify()`) and
// :220-228 (`pk.verify_decryption_share(share, ct)`), both in `threshold_crypto`
// (git rev 624eeee, Cargo.toml:36), which evaluate
//
//     Ciphertext::verify                   e(G1::one(), W) == e(U, H)
//     PublicKeyShare::verify_decryption_share  e(share, H) == e(pk_i, W)
//
// with H = hash_g1_g2(U, V) and `PEngine::pairing` = the `pairing` crate's
// BLS12-381 optimal ate pairing.  A check here is e(a, b) == e(c, d),
// evaluated as one final exponentiation of f_a,b * f_-c,d (the two GT values
// are equal iff that product exponentiates to 1; GT has prime order r).
//
// MI355X layout.  One lane owns one Miller loop (kernel 1) or one final
// exponentiation (kernel 2): the arithmetic is serial 381-bit Montgomery
// products (12 x 32-bit limbs at rest, 14 x 29-bit limbs inside fp_mul), so a lane-per-pairing
// mapping keeps every limb in VGPRs with no cross-lane traffic.  The Miller
// values travel between the kernels in a limb-major workspace
// ([144 words][pairings]), so every store and load is one coalesced dword per
// lane.  Points arrive in the crate's uncompressed encodings (G1 96 bytes
// x || y, G2 192 bytes x.c1 || x.c0 || y.c1 || y.c0, big-endian, flag bits
// in byte 0) and are checked for canonical coordinates, curve membership and
// membership of the order-r subgroup, as the crate's deserialisation does.
//
// Tower: Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3 - (u+1)), Fp12 = Fp6[w]/(w^2 - v),
// the crate's.  Miller loop over |x| = 0xd201000000010000 with homogeneous
// projective doubling/addition on the M-type twist y^2 = x^3 + 4(u+1); each
// line is scaled into the sparse form (c0, c1, c4) and applied with
// mul_by_014; f is conjugated at the end (x < 0).  Final exponentiation: easy
// part, then the crate's hard-part chain (= f^(3 (p^4 - p^2 + 1)/r)).
#include <cstdlib>

#include "bls_consts.hpp"
#include "device_common.hpp"
#include "launchers.hpp"

namespace hbrbc {

namespace {

using namespace bls;

constexpr int NL = 12;  // 32-bit limbs per Fp element

struct Fp { uint32_t l[NL]; };
struct Fp2 { Fp c0, c1; };
struct Fp6 { Fp2 c0, c1, c2; };
struct Fp12 { Fp6 c0, c1; };

#define DEV __device__ __forceinline__
// Call boundaries: out-of-line units keep compile time bounded; everything
// below an NOINL unit is inlined into it.
#define NOINL __device__ __noinline__

// ---------------------------------------------------------------- Fp
DEV void fp_set(Fp &r, const uint32_t (&v)[NL]) {
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = v[i];
}

DEV void fp_zero(Fp &r) {
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = 0;
}

DEV bool fp_is_zero(const Fp &a) {
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) t |= a.l[i];
    return t == 0;
}

DEV bool fp_eq(const Fp &a, const Fp &b) {
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) t |= a.l[i] ^ b.l[i];
    return t == 0;
}

// 32-bit add / subtract with carry (v_add_co_ci_u32 / v_sub_co_ci_u32 chains)
DEV uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t *cout) {
    return __builtin_addc(a, b, cin, cout);
}
DEV uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t *bout) {
    return __builtin_subc(a, b, bin, bout);
}

// r = t - p if t >= p else t  (t < 2p)
DEV void fp_reduce_once(Fp &r, const uint32_t (&t)[NL]) {
    uint32_t s[NL];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) s[i] = subb(t[i], kP[i], br, &br);
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = br ? t[i] : s[i];
}

DEV void fp_add(Fp &r, const Fp &a, const Fp &b) {
    uint32_t t[NL];
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) t[i] = addc(a.l[i], b.l[i], c, &c);
    fp_reduce_once(r, t);  // a + b < 2p < 2^382: no carry out of limb 11
}

DEV void fp_sub(Fp &r, const Fp &a, const Fp &b) {
    uint32_t t[NL];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) t[i] = subb(a.l[i], b.l[i], br, &br);
    const uint32_t mask = 0u - br;  // add p back on borrow
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = addc(t[i], kP[i] & mask, c, &c);
}

DEV void fp_dbl(Fp &r, const Fp &a) { fp_add(r, a, a); }

DEV void fp_neg(Fp &r, const Fp &a) {
    Fp z;
    fp_zero(z);
    fp_sub(r, z, a);
}

// Montgomery product a*b*2^-406 mod p (R = 2^406, bls_consts.hpp), product
// scanning over 14 limbs of 29 bits: column k of a*b + M*p is a sum of at
// most 28 products < 2^58 plus the carry, so it accumulates in a 64-bit value
// fed straight by v_mad_u64_u32 (the accumulator is the 64-bit addend: no
// zero-extending moves, no carry chains, no carry-flag hazards); each of the
// first 14 columns fixes one 29-bit Montgomery digit m_k.  Two accumulators per
// column (even / odd i) halve the dependent chains.  561 VALU per product
// against 1078 for 32-bit-limb CIOS (288 mads + 248 moves + 264 add-with-carry
// + 205 hazard nops), DESIGN.md §6e.  Inputs < p in 12 x 32-bit limbs; the
// result < 2p is reduced once.
constexpr uint32_t kM29 = (1u << 29) - 1;

DEV void fp_to29(uint32_t (&o)[14], const uint32_t (&w)[NL]) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        const int bit = 29 * i, q = bit >> 5, s = bit & 31;
        const uint32_t lo = w[q], hi = (q + 1 < NL) ? w[q + 1] : 0u;
        o[i] = (s ? __builtin_amdgcn_alignbit(hi, lo, s) : lo) & kM29;
    }
}

// 14 digits (13 of 29 bits and a top one, two's complement when `neg`) to
// 12 x 32-bit limbs of the value mod p: value in (-p, 0) gets p added, value
// in [0, 2p) is reduced once.
DEV void fp_from29(Fp &r, const uint32_t (&o)[14], bool neg) {
    uint32_t t[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        const int bit = 32 * j, i = bit / 29, s = bit % 29;
        uint32_t v = o[i] >> s;
        if (i + 1 < 14) v |= o[i + 1] << (29 - s);
        if (s > 26 && i + 2 < 14) v |= o[i + 2] << (58 - s);
        t[j] = v;
    }
    const uint32_t mask = neg ? 0xFFFFFFFFu : 0u;   // value + p (mod 2^384) when negative
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) t[j] = addc(t[j], kP[j] & mask, c, &c);
    fp_reduce_once(r, t);
}

// HB_FP_CHAINS: independent 64-bit accumulators per column (the products of a
// column are split round-robin over them; each v_mad_u64_u32 depends on the
// previous one of its chain).  A/B: 2 (round 3) or 4.
#ifndef HB_FP_CHAINS
#define HB_FP_CHAINS 2
#endif
DEV void fp_mul(Fp &r, const Fp &a, const Fp &b) {
    constexpr int NC = HB_FP_CHAINS;
    uint32_t x[14], y[14], m[14], o[14];
    fp_to29(x, a.l);
    fp_to29(y, b.l);
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 14; ++k) {
        uint64_t e[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) e[c] = c ? 0 : acc;
        int q = 0;
#pragma unroll
        for (int i = 0; i <= k; ++i, ++q) e[q % NC] += (uint64_t)x[i] * y[k - i];
#pragma unroll
        for (int i = 0; i < k; ++i, ++q) e[q % NC] += (uint64_t)m[i] * kP29[k - i];
        acc = e[0];
#pragma unroll
        for (int c = 1; c < NC; ++c) acc += e[c];
        m[k] = ((uint32_t)acc * kPinv29) & kM29;
        acc += (uint64_t)m[k] * kP29[0];   // low 29 bits become 0
        acc >>= 29;
    }
#pragma unroll
    for (int k = 14; k < 27; ++k) {
        uint64_t e[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) e[c] = c ? 0 : acc;
        int q = 0;
#pragma unroll
        for (int i = k - 13; i < 14; ++i, ++q) e[q % NC] += (uint64_t)x[i] * y[k - i];
#pragma unroll
        for (int i = k - 13; i < 14; ++i, ++q) e[q % NC] += (uint64_t)m[i] * kP29[k - i];
        acc = e[0];
#pragma unroll
        for (int c = 1; c < NC; ++c) acc += e[c];
        o[k - 14] = (uint32_t)acc & kM29;
        acc >>= 29;
    }
    o[13] = (uint32_t)acc;   // < 2^5: the result is below 2p < 2^382
    fp_from29(r, o, false);
}

DEV void fp_sqr(Fp &r, const Fp &a) { fp_mul(r, a, a); }

// a^(p-2) (Fermat); once per final exponentiation.
__device__ __noinline__ void fp_inv(Fp &r, const Fp &a) {
    Fp acc, base = a;
    fp_set(acc, kOne);
    for (int w = 0; w < NL; ++w) {
        uint32_t e = kPminus2[w];
        for (int b = 0; b < 32; ++b) {
            if (e & 1u) fp_mul(acc, acc, base);
            fp_sqr(base, base);
            e >>= 1;
        }
    }
    r = acc;
}

// ---------------------------------------------------------------- Fp2
DEV void fp2_add(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp_add(r.c0, a.c0, b.c0); fp_add(r.c1, a.c1, b.c1); }
DEV void fp2_sub(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp_sub(r.c0, a.c0, b.c0); fp_sub(r.c1, a.c1, b.c1); }
DEV void fp2_dbl(Fp2 &r, const Fp2 &a) { fp_dbl(r.c0, a.c0); fp_dbl(r.c1, a.c1); }
DEV void fp2_neg(Fp2 &r, const Fp2 &a) { fp_neg(r.c0, a.c0); fp_neg(r.c1, a.c1); }
DEV void fp2_conj(Fp2 &r, const Fp2 &a) { r.c0 = a.c0; fp_neg(r.c1, a.c1); }
DEV void fp2_zero(Fp2 &r) { fp_zero(r.c0); fp_zero(r.c1); }
DEV bool fp2_is_zero(const Fp2 &a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
DEV bool fp2_eq(const Fp2 &a, const Fp2 &b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }

// Fp2 products with lazy reduction: both output coefficients of an Fp2
// product or square are column sums of 29-bit-limb products, accumulated in
// 64-bit values (c0's two's complement: a0 b0 - a1 b1) and Montgomery-reduced
// once each -- Karatsuba's three products share one pass over the columns and
// need two reductions, not three (980 instead of 1176 mads per Fp2 product),
// and the limb conversions and 12-word additions around the products go away.
// Every column stays below 2^63 in magnitude.
template <class Cols>
DEV void fp2_redc(Fp2 &r, Cols cols) {
    uint32_t m0[14], m1[14], o0[14], o1[14];
    uint64_t A0 = 0, A1 = 0;   // A0: two's complement (c0 may be negative)
#pragma unroll
    for (int k = 0; k < 27; ++k) {
        uint64_t e0 = A0, e1 = A1;
        cols(k, e0, e1);
        const int lo = k > 13 ? k - 13 : 0, hi = k < 14 ? k : 14;
#pragma unroll
        for (int i = lo; i < hi; ++i) {
            e0 += (uint64_t)m0[i] * kP29[k - i];
            e1 += (uint64_t)m1[i] * kP29[k - i];
        }
        if (k < 14) {
            m0[k] = ((uint32_t)e0 * kPinv29) & kM29;
            m1[k] = ((uint32_t)e1 * kPinv29) & kM29;
            e0 += (uint64_t)m0[k] * kP29[0];
            e1 += (uint64_t)m1[k] * kP29[0];
        } else {
            o0[k - 14] = (uint32_t)e0 & kM29;
            o1[k - 14] = (uint32_t)e1 & kM29;
        }
        A0 = (uint64_t)((int64_t)e0 >> 29);
        A1 = e1 >> 29;
    }
    o0[13] = (uint32_t)A0;   // c0 in (-p, 2p): a negative top digit
    o1[13] = (uint32_t)A1;   // c1 in [0, 2p)
    fp_from29(r.c0, o0, (int32_t)o0[13] < 0);
    fp_from29(r.c1, o1, false);
}

// HB_LAZY_MUL / HB_LAZY_SQR: the lazily reduced Fp2 product / square (1)
// or three / two Fp products (0) (A/B)
#ifndef HB_LAZY_MUL
#define HB_LAZY_MUL 0
#endif
#ifndef HB_LAZY_SQR
#define HB_LAZY_SQR 1
#endif
#if HB_LAZY_MUL
DEV void fp2_mul_in(Fp2 &r, const Fp2 &a, const Fp2 &b) {
    uint32_t x0[14], x1[14], y0[14], y1[14], s[14], t[14];
    fp_to29(x0, a.c0.l);
    fp_to29(x1, a.c1.l);
    fp_to29(y0, b.c0.l);
    fp_to29(y1, b.c1.l);
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        s[i] = x0[i] + x1[i];   // < 2^30: products < 2^60, 14 per column
        t[i] = y0[i] + y1[i];
    }
    fp2_redc(r, [&](int k, uint64_t &e0, uint64_t &e1) {
        const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
        uint64_t p0 = 0, p1 = 0, p2 = 0;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            p0 += (uint64_t)x0[i] * y0[k - i];
            p1 += (uint64_t)x1[i] * y1[k - i];
            p2 += (uint64_t)s[i] * t[k - i];
        }
        e0 += p0 - p1;        // a0 b0 - a1 b1
        e1 += p2 - p0 - p1;   // a0 b1 + a1 b0 (Karatsuba)
    });
}

#else
// HB_FP2_SERIAL (A/B): a scheduling barrier between the three Fp products, so
// the scheduler cannot interleave them (fewer live digits, less ILP)
#ifndef HB_FP2_SERIAL
#define HB_FP2_SERIAL 1   // round 6: Miller 71.1 -> 66.8, final exp 68.8 -> 66.8 ms (r6u)
#endif
template <bool SER>
DEV void fp2_mul_t(Fp2 &r, const Fp2 &a, const Fp2 &b) {
    Fp t0, t1, s0, s1;
    fp_mul(t0, a.c0, b.c0);
    if (SER) __builtin_amdgcn_sched_barrier(0);
    fp_mul(t1, a.c1, b.c1);
    if (SER) __builtin_amdgcn_sched_barrier(0);
    fp_add(s0, a.c0, a.c1);
    fp_add(s1, b.c0, b.c1);
    fp_mul(s0, s0, s1);
    if (SER) __builtin_amdgcn_sched_barrier(0);
    fp_sub(r.c0, t0, t1);
    fp_sub(s0, s0, t0);
    fp_sub(r.c1, s0, t1);
}
DEV void fp2_mul_in(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp2_mul_t<HB_FP2_SERIAL != 0>(r, a, b); }

#endif

#if HB_LAZY_SQR
DEV void fp2_sqr_in(Fp2 &r, const Fp2 &a) {
    uint32_t x0[14], x1[14], s[14], t2[14];
    int32_t d[14];
    fp_to29(x0, a.c0.l);
    fp_to29(x1, a.c1.l);
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        s[i] = x0[i] + x1[i];
        d[i] = (int32_t)x0[i] - (int32_t)x1[i];
        t2[i] = x1[i] << 1;
    }
    fp2_redc(r, [&](int k, uint64_t &e0, uint64_t &e1) {
        const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
        int64_t q0 = 0;
        uint64_t q1 = 0;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            q0 += (int64_t)(int32_t)s[i] * d[k - i];   // (a0 + a1)(a0 - a1)
            q1 += (uint64_t)x0[i] * t2[k - i];         // 2 a0 a1
        }
        e0 += (uint64_t)q0;
        e1 += q1;
    });
}

#else
DEV void fp2_sqr_in(Fp2 &r, const Fp2 &a) {
    Fp s, d, m;
    fp_add(s, a.c0, a.c1);
    fp_sub(d, a.c0, a.c1);
    fp_mul(m, a.c0, a.c1);
    fp_mul(r.c0, s, d);
    fp_dbl(r.c1, m);
}

#endif

// Out-of-line forms for cold code (inversions, Frobenius, input checks); the
// hot units (Fp6 products, the sparse line product, the cyclotomic square, the
// Miller steps) inline fp2_mul_in / fp2_sqr_in into their own bodies.
NOINL void fp2_mul(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp2_mul_in(r, a, b); }
NOINL void fp2_sqr(Fp2 &r, const Fp2 &a) { fp2_sqr_in(r, a); }

DEV void fp2_mul_fp(Fp2 &r, const Fp2 &a, const Fp &s) { fp_mul(r.c0, a.c0, s); fp_mul(r.c1, a.c1, s); }

// * xi = u + 1
DEV void fp2_mul_xi(Fp2 &r, const Fp2 &a) {
    Fp t0, t1;
    fp_sub(t0, a.c0, a.c1);
    fp_add(t1, a.c0, a.c1);
    r.c0 = t0;
    r.c1 = t1;
}

DEV void fp2_inv(Fp2 &r, const Fp2 &a) {
    Fp n0, n1;
    fp_sqr(n0, a.c0);
    fp_sqr(n1, a.c1);
    fp_add(n0, n0, n1);
    fp_inv(n0, n0);
    fp_mul(r.c0, a.c0, n0);
    fp_mul(n1, a.c1, n0);
    fp_neg(r.c1, n1);
}

DEV void fp2_frob(Fp2 &r, const Fp2 &a, int k) {
    if (k & 1) fp2_conj(r, a);
    else r = a;
}

DEV void fp2_const(Fp2 &r, const uint32_t (&v)[2][NL]) { fp_set(r.c0, v[0]); fp_set(r.c1, v[1]); }

// ---------------------------------------------------------------- Fp6
DEV void fp6_add(Fp6 &r, const Fp6 &a, const Fp6 &b) { fp2_add(r.c0, a.c0, b.c0); fp2_add(r.c1, a.c1, b.c1); fp2_add(r.c2, a.c2, b.c2); }
DEV void fp6_sub(Fp6 &r, const Fp6 &a, const Fp6 &b) { fp2_sub(r.c0, a.c0, b.c0); fp2_sub(r.c1, a.c1, b.c1); fp2_sub(r.c2, a.c2, b.c2); }
DEV void fp6_neg(Fp6 &r, const Fp6 &a) { fp2_neg(r.c0, a.c0); fp2_neg(r.c1, a.c1); fp2_neg(r.c2, a.c2); }
DEV void fp6_dbl(Fp6 &r, const Fp6 &a) { fp2_dbl(r.c0, a.c0); fp2_dbl(r.c1, a.c1); fp2_dbl(r.c2, a.c2); }

// * v: (a0, a1, a2) -> (xi a2, a0, a1)
DEV void fp6_mul_v(Fp6 &r, const Fp6 &a) {
    Fp2 t;
    fp2_mul_xi(t, a.c2);
    r.c2 = a.c1;
    r.c1 = a.c0;
    r.c0 = t;
}

DEV void fp6_mul_in(Fp6 &r, const Fp6 &a, const Fp6 &b) {
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
NOINL void fp6_mul(Fp6 &r, const Fp6 &a, const Fp6 &b) { fp6_mul_in(r, a, b); }

// (a0 + a1 v + a2 v^2)(c0 + c1 v)
DEV void fp6_mul_by_01(Fp6 &r, const Fp6 &a, const Fp2 &c0, const Fp2 &c1) {
    Fp2 aa, bb, s, t1, t2, t3;
    fp2_mul_in(aa, a.c0, c0);
    fp2_mul_in(bb, a.c1, c1);
    fp2_add(s, a.c1, a.c2);
    fp2_mul_in(t1, s, c1);
    fp2_sub(t1, t1, bb);
    fp2_mul_xi(t1, t1);
    fp2_add(t1, t1, aa);
    fp2_add(s, a.c0, a.c2);
    fp2_mul_in(t3, s, c0);
    fp2_sub(t3, t3, aa);
    fp2_add(t3, t3, bb);
    Fp2 cs;
    fp2_add(cs, c0, c1);
    fp2_add(s, a.c0, a.c1);
    fp2_mul_in(t2, s, cs);
    fp2_sub(t2, t2, aa);
    fp2_sub(t2, t2, bb);
    r.c0 = t1;
    r.c1 = t2;
    r.c2 = t3;
}

// (a0 + a1 v + a2 v^2) c1 v
DEV void fp6_mul_by_1(Fp6 &r, const Fp6 &a, const Fp2 &c1) {
    Fp2 t0, t1, t2;
    fp2_mul_in(t2, a.c1, c1);
    fp2_mul_in(t1, a.c0, c1);
    fp2_mul_in(t0, a.c2, c1);
    fp2_mul_xi(r.c0, t0);
    r.c1 = t1;
    r.c2 = t2;
}

DEV void fp6_inv(Fp6 &r, const Fp6 &a) {
    Fp2 c0, c1, c2, t, u;
    fp2_sqr(c0, a.c0);
    fp2_mul(t, a.c1, a.c2);
    fp2_mul_xi(t, t);
    fp2_sub(c0, c0, t);           // a0^2 - xi a1 a2
    fp2_sqr(c1, a.c2);
    fp2_mul_xi(c1, c1);
    fp2_mul(t, a.c0, a.c1);
    fp2_sub(c1, c1, t);           // xi a2^2 - a0 a1
    fp2_sqr(c2, a.c1);
    fp2_mul(t, a.c0, a.c2);
    fp2_sub(c2, c2, t);           // a1^2 - a0 a2
    fp2_mul(t, a.c2, c1);
    fp2_mul(u, a.c1, c2);
    fp2_add(t, t, u);
    fp2_mul_xi(t, t);
    fp2_mul(u, a.c0, c0);
    fp2_add(t, t, u);             // norm
    fp2_inv(t, t);
    fp2_mul(r.c0, c0, t);
    fp2_mul(r.c1, c1, t);
    fp2_mul(r.c2, c2, t);
}

DEV void fp6_frob(Fp6 &r, const Fp6 &a, int k) {
    Fp2 g, t;
    fp2_frob(r.c0, a.c0, k);
    fp2_frob(t, a.c1, k);
    fp2_const(g, kFrob6C1[k]);
    fp2_mul(r.c1, t, g);
    fp2_frob(t, a.c2, k);
    fp2_const(g, kFrob6C2[k]);
    fp2_mul(r.c2, t, g);
}

// ---------------------------------------------------------------- Fp12
DEV void fp12_one(Fp12 &r) {
    Fp2 z;
    fp2_zero(z);
    r.c0.c0 = z; r.c0.c1 = z; r.c0.c2 = z;
    r.c1 = r.c0;
    fp_set(r.c0.c0.c0, kOne);
}

DEV bool fp12_is_one(const Fp12 &a) {
    Fp one;
    fp_set(one, kOne);
    return fp_eq(a.c0.c0.c0, one) && fp_is_zero(a.c0.c0.c1) && fp2_is_zero(a.c0.c1) &&
           fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) && fp2_is_zero(a.c1.c1) &&
           fp2_is_zero(a.c1.c2);
}

DEV void fp12_conj(Fp12 &r, const Fp12 &a) { r.c0 = a.c0; fp6_neg(r.c1, a.c1); }

// HB_FE_INL: the Fp6 products of the full Fp12 product inlined into it (A/B)
#ifndef HB_FE_INL
#define HB_FE_INL 0
#endif
template <bool INL>
DEV void fp12_mul_t(Fp12 &r, const Fp12 &a, const Fp12 &b) {
    Fp6 aa, bb, s, t;
    if (INL) fp6_mul_in(aa, a.c0, b.c0); else fp6_mul(aa, a.c0, b.c0);
    if (INL) fp6_mul_in(bb, a.c1, b.c1); else fp6_mul(bb, a.c1, b.c1);
    fp6_add(s, a.c0, a.c1);
    fp6_add(t, b.c0, b.c1);
    if (INL) fp6_mul_in(s, s, t); else fp6_mul(s, s, t);
    fp6_sub(s, s, aa);
    fp6_sub(r.c1, s, bb);
    fp6_mul_v(bb, bb);
    fp6_add(r.c0, aa, bb);
}
NOINL void fp12_mul(Fp12 &r, const Fp12 &a, const Fp12 &b) { fp12_mul_t<HB_FE_INL != 0>(r, a, b); }

// INL: the Fp6 products inlined (no call boundary inside the unit, so no
// stack traffic for their operands; tools/fp_microbench.hip: the same 26.8 k
// lane-ops per squaring run 1.47x faster in this form)
template <bool INL>
DEV void fp12_sqr_t(Fp12 &r, const Fp12 &a) {
    Fp6 ab, s, t;
    if (INL) fp6_mul_in(ab, a.c0, a.c1); else fp6_mul(ab, a.c0, a.c1);
    fp6_add(s, a.c0, a.c1);
    fp6_mul_v(t, a.c1);
    fp6_add(t, t, a.c0);
    if (INL) fp6_mul_in(s, s, t); else fp6_mul(s, s, t);
    fp6_sub(s, s, ab);
    fp6_mul_v(t, ab);
    fp6_sub(r.c0, s, t);
    fp6_dbl(r.c1, ab);
}
NOINL void fp12_sqr(Fp12 &r, const Fp12 &a) { fp12_sqr_t<false>(r, a); }

// f * (c0 + c1 v + c4 v w): the sparse line value
DEV void fp12_mul_by_014_in(Fp12 &f, const Fp2 &c0, const Fp2 &c1, const Fp2 &c4) {
    Fp6 aa, bb, s;
    Fp2 o;
    fp6_mul_by_01(aa, f.c0, c0, c1);
    fp6_mul_by_1(bb, f.c1, c4);
    fp2_add(o, c1, c4);
    fp6_add(s, f.c1, f.c0);
    fp6_mul_by_01(s, s, c0, o);
    fp6_sub(s, s, aa);
    fp6_sub(f.c1, s, bb);
    fp6_mul_v(bb, bb);
    fp6_add(f.c0, bb, aa);
}
NOINL void fp12_mul_by_014(Fp12 &f, const Fp2 &c0, const Fp2 &c1, const Fp2 &c4) {
    fp12_mul_by_014_in(f, c0, c1, c4);
}

DEV void fp12_inv(Fp12 &r, const Fp12 &a) {
    Fp6 t0, t1;
    fp6_mul(t0, a.c0, a.c0);
    fp6_mul(t1, a.c1, a.c1);
    fp6_mul_v(t1, t1);
    fp6_sub(t0, t0, t1);          // a0^2 - v a1^2
    fp6_inv(t0, t0);
    fp6_mul(r.c0, a.c0, t0);
    fp6_mul(t1, a.c1, t0);
    fp6_neg(r.c1, t1);
}

NOINL void fp12_frob(Fp12 &r, const Fp12 &a, int k) {
    Fp6 c1;
    Fp2 g;
    fp6_frob(r.c0, a.c0, k);
    fp6_frob(c1, a.c1, k);
    fp2_const(g, kFrob12C1[k]);
    fp2_mul(r.c1.c0, c1.c0, g);
    fp2_mul(r.c1.c1, c1.c1, g);
    fp2_mul(r.c1.c2, c1.c2, g);
}

// (a + b s)^2 in Fp4 = Fp2[s]/(s^2 - xi): (a^2 + xi b^2, 2ab)
// HB_CYC_SERIAL (A/B): scheduling barriers between the Fp2 squarings of the
// cyclotomic square (fewer live digits, less ILP)
#ifndef HB_CYC_SERIAL
#define HB_CYC_SERIAL 0
#endif
DEV void fp4_sqr(Fp2 &c0, Fp2 &c1, const Fp2 &a, const Fp2 &b) {
    Fp2 t0, t1, t2;
    fp2_sqr_in(t0, a);
    if (HB_CYC_SERIAL) __builtin_amdgcn_sched_barrier(0);
    fp2_sqr_in(t1, b);
    if (HB_CYC_SERIAL) __builtin_amdgcn_sched_barrier(0);
    fp2_mul_xi(t2, t1);
    fp2_add(c0, t2, t0);
    fp2_add(t2, a, b);
    fp2_sqr_in(t2, t2);
    fp2_sub(t2, t2, t0);
    fp2_sub(c1, t2, t1);
}

// Granger-Scott squaring, valid on the cyclotomic subgroup (every value of
// the hard part): 9 Fp2 squarings instead of the 2 Fp6 products of fp12_sqr.
// HB_INL_CYC: inlined into fp12_exp_by_x's loop, so the running value stays
// in registers instead of passing through the stack 62 times per call (round
// 5, default: 262144 grouped checks 159.1 -> 157.3 ms; with 1 wave/SIMD as
// well 168.1, profiles/r5n_f4_cyclo_inline_ab.txt)
#ifndef HB_INL_CYC
#define HB_INL_CYC 1
#endif
#if HB_INL_CYC
DEV
#else
NOINL
#endif
void fp12_cyclo_sqr(Fp12 &f) {
    Fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
    Fp2 t0, t1, t2, t3;
    fp4_sqr(t0, t1, z0, z1);
    fp2_sub(z0, t0, z0);
    fp2_dbl(z0, z0);
    fp2_add(z0, z0, t0);          // 3 t0 - 2 z0
    fp2_add(z1, t1, z1);
    fp2_dbl(z1, z1);
    fp2_add(z1, z1, t1);          // 3 t1 + 2 z1
    fp4_sqr(t0, t1, z2, z3);
    fp4_sqr(t2, t3, z4, z5);
    fp2_sub(z4, t0, z4);
    fp2_dbl(z4, z4);
    fp2_add(z4, z4, t0);
    fp2_add(z5, t1, z5);
    fp2_dbl(z5, z5);
    fp2_add(z5, z5, t1);
    fp2_mul_xi(t0, t3);
    fp2_add(z2, t0, z2);
    fp2_dbl(z2, z2);
    fp2_add(z2, z2, t0);
    fp2_sub(z3, t2, z3);
    fp2_dbl(z3, z3);
    fp2_add(z3, z3, t2);
    f.c0.c0 = z0; f.c0.c1 = z4; f.c0.c2 = z3;
    f.c1.c0 = z2; f.c1.c1 = z1; f.c1.c2 = z5;
}

// f^x for the BLS parameter x < 0 (the crate's exp_by_x: pow by |x|, then
// conjugate -- the inverse on the cyclotomic subgroup).  `shift` gives |x|>>1.
// HB_EXPX_INL (A/B): 1 = the five products by `a` inlined too (Fp6 products
// inlined), so the whole f^|x| is one unit with no call inside its loop
#ifndef HB_EXPX_INL
#define HB_EXPX_INL 1   // round 6, on the serialised Fp2 base: final exp 66.9 -> 59.1 ms (r6z)
#endif
NOINL void fp12_exp_by_x(Fp12 &r, const Fp12 &a, int shift) {
    const uint64_t e = kXAbs >> shift;
    Fp12 acc = a;
    for (int b = 62 - shift; b >= 0; --b) {
        fp12_cyclo_sqr(acc);
        if ((e >> b) & 1u) {
            if (HB_EXPX_INL) fp12_mul_t<true>(acc, acc, a); else fp12_mul(acc, acc, a);
        }
    }
    fp12_conj(r, acc);
}

// ---------------------------------------------------------------- Miller loop
struct G2Proj { Fp2 x, y, z; };

// T <- 2T and the tangent line at T before it is evaluated at P, scaled by
// 2YZ^2: L0 + (L1 xp) v + (L4 yp) v w with L0 = 3X^3 - 2Y^2 Z, L1 = -3X^2 Z,
// L4 = 2 Y Z^2.
// HB_G2_SERIAL (A/B): the serialised Fp2 product in the G2 line units too
// (G2 preparation: one lane per point, latency-bound at 1/16 of the wave
// slots, where the serialisation only lengthens the chain)
#ifndef HB_G2_SERIAL
#define HB_G2_SERIAL 1
#endif
DEV void fp2_mul_g2(Fp2 &r, const Fp2 &a, const Fp2 &b) {
#if HB_LAZY_MUL
    fp2_mul_in(r, a, b);
#else
    fp2_mul_t<HB_G2_SERIAL != 0>(r, a, b);
#endif
}

NOINL void g2_dbl_line(G2Proj &T, Fp2 &l0, Fp2 &l1, Fp2 &l4) {
    Fp2 xx, w, s, ss, sss, rr, RR, B, h, t;
    fp2_sqr_in(xx, T.x);
    fp2_dbl(w, xx);
    fp2_add(w, w, xx);            // w = 3 X^2
    fp2_mul_g2(s, T.y, T.z);
    fp2_dbl(s, s);                // s = 2 Y Z
    fp2_sqr_in(ss, s);
    fp2_mul_g2(sss, s, ss);
    fp2_mul_g2(rr, T.y, s);       // R = Y s = 2 Y^2 Z
    fp2_sqr_in(RR, rr);
    fp2_add(B, T.x, rr);
    fp2_sqr_in(B, B);
    fp2_sub(B, B, xx);
    fp2_sub(B, B, RR);            // B = (X + R)^2 - X^2 - R^2
    fp2_mul_g2(l0, T.x, w);
    fp2_sub(l0, l0, rr);          // 3X^3 - 2Y^2 Z
    fp2_mul_g2(l1, w, T.z);
    fp2_neg(l1, l1);              // -3X^2 Z
    fp2_mul_g2(l4, s, T.z);       // 2 Y Z^2
    fp2_sqr_in(h, w);
    fp2_sub(h, h, B);
    fp2_sub(h, h, B);             // h = w^2 - 2B
    fp2_mul_g2(T.x, h, s);
    fp2_sub(t, B, h);
    fp2_mul_g2(t, w, t);
    fp2_dbl(RR, RR);
    fp2_sub(T.y, t, RR);          // w (B - h) - 2 R^2
    T.z = sss;
}

// T <- T + Q (Q affine) and the line through T and Q before evaluation at P,
// scaled by (xq Z - X): L0 = u xq - v yq, L1 = -u, L4 = v with u = yq Z - Y,
// v = xq Z - X.
NOINL void g2_add_line(G2Proj &T, const Fp2 &xq, const Fp2 &yq, Fp2 &l0, Fp2 &l1, Fp2 &l4) {
    Fp2 u, v, uu, vv, vvv, R, A, t;
    fp2_mul_g2(u, yq, T.z);
    fp2_sub(u, u, T.y);
    fp2_mul_g2(v, xq, T.z);
    fp2_sub(v, v, T.x);
    fp2_mul_g2(l0, u, xq);
    fp2_mul_g2(t, v, yq);
    fp2_sub(l0, l0, t);
    fp2_neg(l1, u);
    l4 = v;
    fp2_sqr_in(uu, u);
    fp2_sqr_in(vv, v);
    fp2_mul_g2(vvv, v, vv);
    fp2_mul_g2(R, vv, T.x);
    fp2_mul_g2(A, uu, T.z);
    fp2_sub(A, A, vvv);
    fp2_sub(A, A, R);
    fp2_sub(A, A, R);             // A = uu Z - vvv - 2R
    fp2_mul_g2(T.x, v, A);
    fp2_sub(t, R, A);
    fp2_mul_g2(t, u, t);
    fp2_mul_g2(vvv, vvv, T.y);
    fp2_sub(T.y, t, vvv);
    fp2_mul_g2(T.z, T.z, vv);
    fp2_mul_g2(T.z, T.z, v);      // Z vvv
}

// f <- f * line(P): the line evaluated at P = (xp, yp) (sparse (c0, c1, c4))
DEV void apply_line(Fp12 &f, const Fp2 &l0, const Fp2 &l1, const Fp2 &l4, const Fp &xp,
                    const Fp &yp) {
    Fp2 a, b;
    fp2_mul_fp(a, l1, xp);
    fp2_mul_fp(b, l4, yp);
    fp12_mul_by_014(f, l0, a, b);
}

NOINL void miller_dbl(G2Proj &T, Fp12 &f, const Fp &xp, const Fp &yp) {
    Fp2 l0, l1, l4;
    g2_dbl_line(T, l0, l1, l4);
    apply_line(f, l0, l1, l4, xp, yp);
}

NOINL void miller_add(G2Proj &T, Fp12 &f, const Fp2 &xq, const Fp2 &yq, const Fp &xp,
                      const Fp &yp) {
    Fp2 l0, l1, l4;
    g2_add_line(T, xq, yq, l0, l1, l4);
    apply_line(f, l0, l1, l4, xp, yp);
}

// ---------------------------------------------------------------- encodings
// 48 big-endian bytes -> limbs (little-endian words); returns false if the
// value is not below p.  `top_mask` clears flag bits of the first byte.
DEV bool load_be48(Fp &r, const uint8_t *src, uint32_t top_mask) {
#pragma unroll
    for (int w = 0; w < NL; ++w) {
        const uint8_t *q = src + 44 - 4 * w;
        uint32_t v = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
        r.l[w] = v;
    }
    r.l[NL - 1] &= top_mask;
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const uint64_t d = (uint64_t)r.l[i] - kP[i] - br;
        br = (d >> 32) & 1u;
    }
    return br != 0;  // r < p
}

DEV void to_mont(Fp &r, const Fp &a) {
    Fp r2;
    fp_set(r2, kR2);
    fp_mul(r, a, r2);
}

DEV void from_mont(Fp &r, const Fp &a) {
    Fp one;
    fp_zero(one);
    one.l[0] = 1;
    fp_mul(r, a, one);
}

DEV bool all_zero(const uint8_t *p, int n, uint8_t first_mask) {
    uint32_t t = p[0] & first_mask;
    for (int i = 1; i < n; ++i) t |= p[i];
    return t == 0;
}

// Status of a decoded point: 0 ok, 1 infinity, 2 invalid.
enum { PT_OK = 0, PT_INF = 1, PT_BAD = 2 };

// ------------------------------------------------------- subgroup checks
// The crate's deserialisation (`into_affine`: on-curve, then
// is_in_correct_subgroup_assuming_on_curve = [r] P == O) rejects points of
// E(Fp) / E'(Fp2) outside the order-r subgroup before any pairing.  Here the
// equivalent endomorphism tests (Scott, ePrint 2021/1130 sec. 6, proof in
// 2022/352): P in G1 iff phi(P) = (beta x, y) = -[x^2] P, and Q in G2 iff
// psi(Q) = [x] Q, i.e. a 128-bit and a 64-bit scalar multiplication instead
// of a 255-bit one.  oracle/bls_oracle.py restates the crate's [r] P test and
// tests/test_pairing.py feeds on-curve points outside the subgroup (status 2).
// Complete projective formulas for y^2 = x^3 + b (Renes-Costello-Batina 2016,
// algorithms 7 and 9 with a = 0), so no exceptional case arises mid-chain.
template <class F> struct PtProj { F x, y, z; };

DEV void fe_mul(Fp &r, const Fp &a, const Fp &b) { fp_mul(r, a, b); }
DEV void fe_mul(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp2_mul_in(r, a, b); }
DEV void fe_add(Fp &r, const Fp &a, const Fp &b) { fp_add(r, a, b); }
DEV void fe_add(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp2_add(r, a, b); }
DEV void fe_sub(Fp &r, const Fp &a, const Fp &b) { fp_sub(r, a, b); }
DEV void fe_sub(Fp2 &r, const Fp2 &a, const Fp2 &b) { fp2_sub(r, a, b); }
DEV void fe_one(Fp &r) { fp_set(r, kOne); }
DEV void fe_one(Fp2 &r) { fp_set(r.c0, kOne); fp_zero(r.c1); }
// 3b: 12 on E, 12 (u + 1) on the twist
DEV void fe_mul_b3(Fp &r, const Fp &a) {
    Fp t;
    fp_add(t, a, a);
    fp_add(t, t, a);
    fp_add(t, t, t);
    fp_add(r, t, t);
}
DEV void fe_mul_b3(Fp2 &r, const Fp2 &a) {
    Fp2 x;
    fp2_mul_xi(x, a);
    fe_mul_b3(r.c0, x.c0);
    fe_mul_b3(r.c1, x.c1);
}

template <class F>
NOINL void pt_dbl(PtProj<F> &p) {
    F t0, t1, t2, x3, y3, z3;
    fe_mul(t0, p.y, p.y);
    fe_add(z3, t0, t0);
    fe_add(z3, z3, z3);
    fe_add(z3, z3, z3);
    fe_mul(t1, p.y, p.z);
    fe_mul(t2, p.z, p.z);
    fe_mul_b3(t2, t2);
    fe_mul(x3, t2, z3);
    fe_add(y3, t0, t2);
    fe_mul(z3, t1, z3);
    fe_add(t1, t2, t2);
    fe_add(t2, t1, t2);
    fe_sub(t0, t0, t2);
    fe_mul(y3, t0, y3);
    fe_add(y3, x3, y3);
    fe_mul(t1, p.x, p.y);
    fe_mul(x3, t0, t1);
    fe_add(p.x, x3, x3);
    p.y = y3;
    p.z = z3;
}

// p <- p + (qx, qy, 1)
template <class F>
NOINL void pt_add_affine(PtProj<F> &p, const F &qx, const F &qy) {
    F t0, t1, t2, t3, t4, x3, y3, z3;
    fe_mul(t0, p.x, qx);
    fe_mul(t1, p.y, qy);
    t2 = p.z;
    fe_add(t3, p.x, p.y);
    fe_add(t4, qx, qy);
    fe_mul(t3, t3, t4);
    fe_add(t4, t0, t1);
    fe_sub(t3, t3, t4);
    fe_mul(t4, qy, p.z);
    fe_add(t4, t4, p.y);            // Y1 + Y2 Z1
    fe_mul(y3, qx, p.z);
    fe_add(y3, y3, p.x);            // X1 + X2 Z1
    fe_add(x3, t0, t0);
    fe_add(t0, x3, t0);
    fe_mul_b3(t2, t2);
    fe_add(z3, t1, t2);
    fe_sub(t1, t1, t2);
    fe_mul_b3(y3, y3);
    fe_mul(x3, t4, y3);
    fe_mul(t2, t3, t1);
    fe_sub(x3, t2, x3);
    fe_mul(y3, y3, t0);
    fe_mul(t1, t1, z3);
    fe_add(y3, t1, y3);
    fe_mul(t0, t0, t3);
    fe_mul(z3, z3, t4);
    fe_add(p.z, z3, t0);
    p.x = x3;
    p.y = y3;
}

// [k] (x, y) for the bits of k below its leading one (k's top bit at `top`)
template <class F>
DEV void pt_mul_bits(PtProj<F> &acc, const F &x, const F &y, uint64_t hi, uint64_t lo, int top) {
    acc.x = x;
    acc.y = y;
    fe_one(acc.z);
    for (int b = top - 1; b >= 0; --b) {
        pt_dbl(acc);
        const uint64_t w = b >= 64 ? hi : lo;
        if ((w >> (b & 63)) & 1u) pt_add_affine(acc, x, y);
    }
}

// (x, y) affine (Montgomery form), already on E: phi(P) == -[x^2] P, i.e.
// [x^2] P == (beta x, -y) in projective coordinates (Z != 0)
NOINL bool g1_in_subgroup(const Fp &x, const Fp &y) {
    PtProj<Fp> a;
    pt_mul_bits(a, x, y, kXSqHi, kXSqLo, 127);
    Fp bx, ny, l, r;
    fp_set(bx, kBeta);
    fp_mul(bx, bx, x);
    fp_neg(ny, y);
    fp_mul(l, bx, a.z);
    fp_mul(r, ny, a.z);
    return !fp_is_zero(a.z) && fp_eq(l, a.x) && fp_eq(r, a.y);
}

// (x, y) on E': psi(Q) == [x] Q = -[|x|] Q, i.e. [|x|] Q == (psi_x, -psi_y)
NOINL bool g2_in_subgroup(const Fp2 &x, const Fp2 &y) {
    PtProj<Fp2> a;
    pt_mul_bits(a, x, y, 0, kXAbs, 63);
    Fp2 cx, cy, px, py, l, r;
    fp2_const(cx, kPsi[0]);
    fp2_const(cy, kPsi[1]);
    fp2_conj(px, x);
    fp2_mul(px, px, cx);
    fp2_conj(py, y);
    fp2_mul(py, py, cy);
    fp2_neg(py, py);
    fp2_mul(l, px, a.z);
    fp2_mul(r, py, a.z);
    return !fp2_is_zero(a.z) && fp2_eq(l, a.x) && fp2_eq(r, a.y);
}

DEV int decode_g1(const uint8_t *src, Fp &x, Fp &y) {
    const uint8_t f = src[0];
    if (f & 0xA0) return PT_BAD;                       // compressed / sort flags
    if (f & 0x40) return all_zero(src, 96, 0x1F) ? PT_INF : PT_BAD;
    Fp xr, yr;
    if (!load_be48(xr, src, 0x1FFFFFFFu) || !load_be48(yr, src + 48, 0xFFFFFFFFu)) return PT_BAD;
    to_mont(x, xr);
    to_mont(y, yr);
    Fp l, r, b;
    fp_sqr(l, y);
    fp_sqr(r, x);
    fp_mul(r, r, x);
    fp_set(b, kB1);
    fp_add(r, r, b);
    if (!fp_eq(l, r)) return PT_BAD;                   // y^2 = x^3 + 4
    return g1_in_subgroup(x, y) ? PT_OK : PT_BAD;      // order r (the crate's into_affine)
}

// the encoding and the curve equation only (no order-r check)
DEV int decode_g2_curve(const uint8_t *src, Fp2 &x, Fp2 &y) {
    const uint8_t f = src[0];
    if (f & 0xA0) return PT_BAD;
    if (f & 0x40) return all_zero(src, 192, 0x1F) ? PT_INF : PT_BAD;
    Fp a, b, c, d;
    if (!load_be48(a, src, 0x1FFFFFFFu) || !load_be48(b, src + 48, 0xFFFFFFFFu) ||
        !load_be48(c, src + 96, 0xFFFFFFFFu) || !load_be48(d, src + 144, 0xFFFFFFFFu))
        return PT_BAD;
    to_mont(x.c1, a);
    to_mont(x.c0, b);
    to_mont(y.c1, c);
    to_mont(y.c0, d);
    Fp2 l, r, bb;
    fp2_sqr(l, y);
    fp2_sqr(r, x);
    fp2_mul(r, r, x);
    fp_set(bb.c0, kB1);
    bb.c1 = bb.c0;                                     // 4 (u + 1)
    fp2_add(r, r, bb);
    return fp2_eq(l, r) ? PT_OK : PT_BAD;
}

DEV int decode_g2(const uint8_t *src, Fp2 &x, Fp2 &y) {
    const int st = decode_g2_curve(src, x, y);
    if (st != PT_OK) return st;
    return g2_in_subgroup(x, y) ? PT_OK : PT_BAD;
}

// Limb-major workspace: word w of pairing i at ws[w * n + i].
DEV void store_f12(uint32_t *ws, size_t n, size_t i, const Fp12 &f) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&f);
#pragma unroll 4
    for (int w = 0; w < 12 * NL; ++w) ws[(size_t)w * n + i] = src[w];
}

DEV void load_f12(Fp12 &f, const uint32_t *ws, size_t n, size_t i) {
    uint32_t *dst = reinterpret_cast<uint32_t *>(&f);
#pragma unroll 4
    for (int w = 0; w < 12 * NL; ++w) dst[w] = ws[(size_t)w * n + i];
}

constexpr int kPairBlock = 64;
// waves per SIMD of every pairing kernel (512 / HB_PAIR_WPE VGPRs per lane).
// The 29-bit-limb product holds x, y, m and the output digits (56 VGPRs) on
// top of the tower operands: at 4 waves (128 VGPRs) the kernels spilled
// (1.02 M checks/s), at 2 waves (256 VGPRs) 1.57 M, at 1 wave 1.53 M (r3,
// tools/gpu_f4_wpe.sh; -DHB_PAIR_WPE=1|4 builds the A/B variants)
#ifndef HB_PAIR_WPE
#define HB_PAIR_WPE 2
#endif

// Kernel 1: one Miller loop per lane.  Pairing i takes G1 point g1[i] and G2
// point g2[i]; with `negate_odd`, odd pairings negate their G1 point (the
// c of a check a,b == c,d sits at pairing 2i+1).  status[i] gets the point
// status (max of the two); an infinity or invalid input leaves f = 1.
__global__ __launch_bounds__(kPairBlock) __attribute__((amdgpu_waves_per_eu(HB_PAIR_WPE, HB_PAIR_WPE))) void miller_kernel(
    const uint8_t *__restrict__ g1, size_t g1_stride, const uint8_t *__restrict__ g2,
    size_t g2_stride, size_t n, int pair_inputs, uint32_t *__restrict__ ws,
    uint8_t *__restrict__ status) {
    const size_t i = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    if (i >= n) return;
    // pair_inputs: pairing 2c reads (a_c, b_c) from the first halves of the
    // arrays, 2c+1 reads (c_c, d_c) from the second halves (see launcher)
    const uint8_t *p1 = g1 + i * g1_stride;
    const uint8_t *p2 = g2 + i * g2_stride;
    Fp xp, yp;
    Fp2 xq, yq;
    const int s1 = decode_g1(p1, xp, yp);
    const int s2 = decode_g2(p2, xq, yq);
    Fp12 f;
    fp12_one(f);
    const int st = s1 > s2 ? s1 : s2;
    if (st == PT_OK && s1 == PT_OK && s2 == PT_OK) {
        if (pair_inputs && (i & 1)) fp_neg(yp, yp);
        G2Proj T;
        T.x = xq;
        T.y = yq;
        fp_set(T.z.c0, kOne);
        fp_zero(T.z.c1);
        for (int b = 62; b >= 0; --b) {
            fp12_sqr(f, f);
            miller_dbl(T, f, xp, yp);
            if ((kXAbs >> b) & 1u) miller_add(T, f, xq, yq, xp, yp);
        }
        fp12_conj(f, f);
    }
    status[i] = (uint8_t)((s1 == PT_BAD || s2 == PT_BAD) ? PT_BAD : PT_OK);
    store_f12(ws, n, i, f);
}

// Kernel 1b: one lane per check e(a, b) == e(c, d) (g1 holds a, c and g2 b, d
// at rows 2i, 2i+1): the two Miller loops of f_a,b * f_-c,d share one
// squaring of f per step (a multi-Miller loop; the product is what the final
// exponentiation needs).  An infinity drops its pairing's lines (factor 1).
__global__ __launch_bounds__(kPairBlock) __attribute__((amdgpu_waves_per_eu(HB_PAIR_WPE, HB_PAIR_WPE))) void miller2_kernel(
    const uint8_t *__restrict__ g1, const uint8_t *__restrict__ g2, size_t count,
    uint32_t *__restrict__ ws, uint8_t *__restrict__ status) {
    const size_t i = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    if (i >= count) return;
    Fp xa, ya, xc, yc;
    Fp2 xb, yb, xd, yd;
    const int sa = decode_g1(g1 + (2 * i) * 96, xa, ya);
    const int sc = decode_g1(g1 + (2 * i + 1) * 96, xc, yc);
    const int sb = decode_g2(g2 + (2 * i) * 192, xb, yb);
    const int sd = decode_g2(g2 + (2 * i + 1) * 192, xd, yd);
    const bool bad = sa == PT_BAD || sb == PT_BAD || sc == PT_BAD || sd == PT_BAD;
    const bool on1 = !bad && sa == PT_OK && sb == PT_OK;
    const bool on2 = !bad && sc == PT_OK && sd == PT_OK;
    Fp12 f;
    fp12_one(f);
    if (on1 || on2) {
        fp_neg(yc, yc);   // e(-c, d) = e(c, d)^-1
        G2Proj T1, T2;
        T1.x = xb;
        T1.y = yb;
        fp_set(T1.z.c0, kOne);
        fp_zero(T1.z.c1);
        T2.x = xd;
        T2.y = yd;
        T2.z = T1.z;
        for (int b = 62; b >= 0; --b) {
            fp12_sqr(f, f);
            if (on1) miller_dbl(T1, f, xa, ya);
            if (on2) miller_dbl(T2, f, xc, yc);
            if ((kXAbs >> b) & 1u) {
                if (on1) miller_add(T1, f, xb, yb, xa, ya);
                if (on2) miller_add(T2, f, xd, yd, xc, yc);
            }
        }
        fp12_conj(f, f);
    }
    status[i] = bad ? PT_BAD : PT_OK;
    store_f12(ws, count, i, f);
}

// ---------------------------------------------------------------- prepared G2
// G2 points prepared once (the crate's G2Prepared): the 68 lines of the Miller
// loop over |x| (63 doublings, 5 additions) before evaluation at P, so every
// check against the same G2 point (hbbft: all N shares of a ciphertext share
// H and W) skips the twist arithmetic.  Table: point q, line s at
// prep + (q * kLines + s) * kLineWords words: L0, L1, L4 (Fp2, Montgomery).
constexpr int kLines = 68;
constexpr int kLineWords = 6 * NL;

DEV void store_line(uint32_t *dst, const Fp2 &l0, const Fp2 &l1, const Fp2 &l4) {
    const Fp *v[6] = {&l0.c0, &l0.c1, &l1.c0, &l1.c1, &l4.c0, &l4.c1};
#pragma unroll
    for (int e = 0; e < 6; ++e)
#pragma unroll
        for (int w = 0; w < NL; w += 4)
            *reinterpret_cast<uint4 *>(dst + e * NL + w) =
                make_uint4(v[e]->l[w], v[e]->l[w + 1], v[e]->l[w + 2], v[e]->l[w + 3]);
}

DEV void load_line(const uint32_t *src, Fp2 &l0, Fp2 &l1, Fp2 &l4) {
    Fp *v[6] = {&l0.c0, &l0.c1, &l1.c0, &l1.c1, &l4.c0, &l4.c1};
#pragma unroll
    for (int e = 0; e < 6; ++e)
#pragma unroll
        for (int w = 0; w < NL; w += 4) {
            const uint4 q = *reinterpret_cast<const uint4 *>(src + e * NL + w);
            v[e]->l[w] = q.x;
            v[e]->l[w + 1] = q.y;
            v[e]->l[w + 2] = q.z;
            v[e]->l[w + 3] = q.w;
        }
}

// HB_G2_SPLIT: the point's order-r check and its 68 lines are independent
// chains (the lines of a point that fails the check are never read: its
// status says invalid), so they run in two waves side by side -- block 2j
// checks points 64j.., block 2j + 1 computes their lines (the preparation's
// latency is the longer chain, not the sum; one ciphertext batch has only
// 8192 points, an eighth of a wave per SIMD).  0: one lane does both.
#ifndef HB_G2_SPLIT
#define HB_G2_SPLIT 1
#endif

// One lane per G2 point (per role with HB_G2_SPLIT): its 68 lines, and its
// status (0 ok, 1 infinity, 2 invalid) at pst[q].
__global__ __launch_bounds__(kPairBlock) __attribute__((amdgpu_waves_per_eu(HB_PAIR_WPE, HB_PAIR_WPE))) void g2_prepare_kernel(
    const uint8_t *__restrict__ g2, size_t count, uint32_t *__restrict__ prep,
    uint8_t *__restrict__ pst) {
    const unsigned blk = HB_G2_SPLIT ? blockIdx.x >> 1 : blockIdx.x;
    const size_t q = (size_t)blk * kPairBlock + threadIdx.x;
    if (q >= count) return;
    Fp2 xq, yq;
    if (HB_G2_SPLIT && !(blockIdx.x & 1)) {   // the status (wave-uniform role)
        pst[q] = (uint8_t)decode_g2(g2 + q * 192, xq, yq);
        return;
    }
    const int st = HB_G2_SPLIT ? decode_g2_curve(g2 + q * 192, xq, yq)
                               : decode_g2(g2 + q * 192, xq, yq);
    if (!HB_G2_SPLIT) pst[q] = (uint8_t)st;
    if (st != PT_OK) return;
    G2Proj T;
    T.x = xq;
    T.y = yq;
    fp_set(T.z.c0, kOne);
    fp_zero(T.z.c1);
    uint32_t *dst = prep + q * (size_t)kLines * kLineWords;
    Fp2 l0, l1, l4;
    for (int b = 62; b >= 0; --b) {
        g2_dbl_line(T, l0, l1, l4);
        store_line(dst, l0, l1, l4);
        dst += kLineWords;
        if ((kXAbs >> b) & 1u) {
            g2_add_line(T, xq, yq, l0, l1, l4);
            store_line(dst, l0, l1, l4);
            dst += kLineWords;
        }
    }
}

// The prepared Miller loop's per-bit work as units of their own (A/B knob
// HB_MILLER_INL): 0 = out-of-line squaring and line application (their
// Fp6 operands through the stack); 1 = the squaring's Fp6 products inlined
// into it; 2 = also the sparse product inlined into the line application.
#ifndef HB_MILLER_INL
#define HB_MILLER_INL 2   // round 6: Miller 85.97 -> 80.0-80.5 ms per 262,144 checks (r6e)
#endif
#if HB_MILLER_INL < 2
NOINL void apply_prepared(Fp12 &f, const uint32_t *line, const Fp &xp, const Fp &yp) {
    Fp2 l0, l1, l4;
    load_line(line, l0, l1, l4);
    apply_line(f, l0, l1, l4, xp, yp);
}
#endif
NOINL void miller_sqr(Fp12 &f) { fp12_sqr_t<(HB_MILLER_INL >= 1)>(f, f); }
NOINL void apply_prepared_in(Fp12 &f, const uint32_t *line, const Fp &xp, const Fp &yp) {
    Fp2 l0, l1, l4, a, b;
    load_line(line, l0, l1, l4);
    fp2_mul_fp(a, l1, xp);
    fp2_mul_fp(b, l4, yp);
    fp12_mul_by_014_in(f, l0, a, b);
}
#if HB_MILLER_INL >= 2
#define HB_APPLY_PREPARED apply_prepared_in
#else
#define HB_APPLY_PREPARED apply_prepared
#endif
// HB_MILLER_INL 3: the whole bit step -- the squaring and both line
// applications -- as one unit, so f does not pass through the stack between
// them
DEV void apply_prepared_body(Fp12 &f, const uint32_t *line, const Fp &xp, const Fp &yp) {
    Fp2 l0, l1, l4, a, b;
    load_line(line, l0, l1, l4);
    fp2_mul_fp(a, l1, xp);
    fp2_mul_fp(b, l4, yp);
    fp12_mul_by_014_in(f, l0, a, b);
}
NOINL void miller_step(Fp12 &f, const uint32_t *p1, const uint32_t *p2, const Fp &xa,
                       const Fp &ya, const Fp &xc, const Fp &yc, bool on1, bool on2) {
    fp12_sqr_t<true>(f, f);
    if (on1) apply_prepared_body(f, p1, xa, ya);
    if (on2) apply_prepared_body(f, p2, xc, yc);
}

// Prepared G1 keys: hbbft checks every decryption share against the public
// key share pk_i of its sender (threshold_decrypt.rs:220-228), and the
// validator set's N key shares are the same for every ciphertext of an epoch
// -- the crate holds them as curve points, so it decodes and checks them once,
// not per share.  One lane per key: decoded and checked like any G1 input
// (canonical coordinates, on the curve, order r), stored as Montgomery affine
// x || y (kG1KeyWords words), status at kst[q] (0 ok, 1 infinity, 2 invalid).
constexpr int kG1KeyWords = 2 * NL;

DEV void load_g1_key(const uint32_t *src, Fp &x, Fp &y) {
#pragma unroll
    for (int w = 0; w < NL; w += 4) {
        const uint4 a = *reinterpret_cast<const uint4 *>(src + w);
        const uint4 b = *reinterpret_cast<const uint4 *>(src + NL + w);
        x.l[w] = a.x; x.l[w + 1] = a.y; x.l[w + 2] = a.z; x.l[w + 3] = a.w;
        y.l[w] = b.x; y.l[w + 1] = b.y; y.l[w + 2] = b.z; y.l[w + 3] = b.w;
    }
}

// HB_G1P_WPE: waves per SIMD of the G1 preparation (affine Fp points and
// their order-r checks need far fewer registers than the tower arithmetic)
#ifndef HB_G1P_WPE
#define HB_G1P_WPE HB_PAIR_WPE
#endif
__global__ __launch_bounds__(kPairBlock) __attribute__((amdgpu_waves_per_eu(HB_G1P_WPE, HB_G1P_WPE))) void g1_prepare_kernel(
    const uint8_t *__restrict__ g1, size_t count, uint32_t *__restrict__ keys,
    uint8_t *__restrict__ kst) {
    const size_t q = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    if (q >= count) return;
    Fp x, y;
    const int st = decode_g1(g1 + q * 96, x, y);
    if (st != PT_OK) {
        fp_zero(x);
        fp_zero(y);
    }
    uint32_t *dst = keys + q * kG1KeyWords;
#pragma unroll
    for (int w = 0; w < NL; w += 4) {
        *reinterpret_cast<uint4 *>(dst + w) = make_uint4(x.l[w], x.l[w + 1], x.l[w + 2], x.l[w + 3]);
        *reinterpret_cast<uint4 *>(dst + NL + w) = make_uint4(y.l[w], y.l[w + 1], y.l[w + 2], y.l[w + 3]);
    }
    kst[q] = (uint8_t)st;
}

// One lane per check e(a, b) == e(c, d) with b, d prepared (points ib[i],
// id[i] of the table): g1 holds a, c at rows 2i, 2i+1.  Lanes of a wave
// checking against the same points read the same lines (one cache line
// serves the wave).
// KEYS: c comes from a table of prepared G1 keys (g1_prepare_kernel) by
// index ic[i] and g1 holds only a_0, a_1, ...; otherwise g1 holds a_0, c_0,
// a_1, c_1, ... and both points of a check are decoded here.
// PTS (with KEYS): a also comes decoded, from a g1_prepare table of the
// `count` shares (entry i, statuses `ast`), so the share decoding -- an
// order-r check each -- runs as its own launch beside the G2 preparation.
template <bool KEYS, bool PTS = false>
__global__ __launch_bounds__(kPairBlock) __attribute__((amdgpu_waves_per_eu(HB_PAIR_WPE, HB_PAIR_WPE))) void miller_prepared_kernel(
    const uint8_t *__restrict__ g1, const uint32_t *__restrict__ keys,
    const uint8_t *__restrict__ kst, const uint32_t *__restrict__ ic, size_t nkeys,
    const uint32_t *__restrict__ prep,
    const uint8_t *__restrict__ pst, const uint32_t *__restrict__ ib,
    const uint32_t *__restrict__ id, size_t points, size_t count, uint32_t *__restrict__ ws,
    uint8_t *__restrict__ status, const uint32_t *__restrict__ atab = nullptr,
    const uint8_t *__restrict__ ast = nullptr) {
    const size_t i = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    if (i >= count) return;
    Fp xa, ya, xc, yc;
    int sa, sc;
    if constexpr (KEYS) {
        if constexpr (PTS) {
            sa = ast[i];
            load_g1_key(atab + i * kG1KeyWords, xa, ya);   // zeros unless the point is valid
        } else {
            sa = decode_g1(g1 + i * 96, xa, ya);
        }
        const uint32_t qc = ic[i];
        // an index past the key table is an invalid input, never an out-of-bounds read
        sc = qc < nkeys ? kst[qc] : PT_BAD;
        if (sc == PT_OK) {
            load_g1_key(keys + (size_t)qc * kG1KeyWords, xc, yc);
        } else {
            fp_zero(xc);
            fp_zero(yc);
        }
    } else {
        sa = decode_g1(g1 + (2 * i) * 96, xa, ya);
        sc = decode_g1(g1 + (2 * i + 1) * 96, xc, yc);
    }
    uint32_t qb = ib[i], qd = id[i];
    // an index past the table is an invalid input, never an out-of-bounds read
    const bool range_ok = qb < points && qd < points;
    if (!range_ok) qb = qd = 0;
    const int sb = range_ok ? pst[qb] : PT_BAD, sd = range_ok ? pst[qd] : PT_BAD;
    const bool bad = sa == PT_BAD || sb == PT_BAD || sc == PT_BAD || sd == PT_BAD;
    const bool on1 = !bad && sa == PT_OK && sb == PT_OK;
    const bool on2 = !bad && sc == PT_OK && sd == PT_OK;
    Fp12 f;
    fp12_one(f);
    if (on1 || on2) {
        fp_neg(yc, yc);   // e(-c, d) = e(c, d)^-1
        const uint32_t *p1 = prep + (size_t)qb * kLines * kLineWords;
        const uint32_t *p2 = prep + (size_t)qd * kLines * kLineWords;
        for (int b = 62; b >= 0; --b) {
            if (HB_MILLER_INL >= 3) {
                miller_step(f, p1, p2, xa, ya, xc, yc, on1, on2);
            } else {
                if (HB_MILLER_INL) miller_sqr(f); else fp12_sqr(f, f);
                if (on1) HB_APPLY_PREPARED(f, p1, xa, ya);
                if (on2) HB_APPLY_PREPARED(f, p2, xc, yc);
            }
            p1 += kLineWords;
            p2 += kLineWords;
            if ((kXAbs >> b) & 1u) {
                if (on1) HB_APPLY_PREPARED(f, p1, xa, ya);
                if (on2) HB_APPLY_PREPARED(f, p2, xc, yc);
                p1 += kLineWords;
                p2 += kLineWords;
            }
        }
        fp12_conj(f, f);
    }
    status[i] = bad ? PT_BAD : PT_OK;
    store_f12(ws, count, i, f);
}

// The crate's final exponentiation (Bls12::final_exponentiation): easy part
// f^((p^6 - 1)(p^2 + 1)), then the hard-part chain.
DEV void final_exp(Fp12 &out, const Fp12 &f) {
    Fp12 r, t, y0, y1, y2, y3;
    fp12_inv(t, f);
    fp12_conj(r, f);
    fp12_mul(r, r, t);            // f^(p^6 - 1)
    fp12_frob(t, r, 2);
    fp12_mul(r, t, r);            // ^(p^2 + 1)
    fp12_sqr(y0, r);
    fp12_exp_by_x(y1, y0, 0);
    fp12_exp_by_x(y2, y1, 1);
    fp12_conj(y3, r);
    fp12_mul(y1, y1, y3);
    fp12_conj(y1, y1);
    fp12_mul(y1, y1, y2);
    fp12_exp_by_x(y2, y1, 0);
    fp12_exp_by_x(y3, y2, 0);
    fp12_conj(y1, y1);
    fp12_mul(y3, y3, y1);
    fp12_conj(y1, y1);
    fp12_frob(y1, y1, 3);
    fp12_frob(y2, y2, 2);
    fp12_mul(y1, y1, y2);
    fp12_exp_by_x(y2, y3, 0);
    fp12_mul(y2, y2, y0);
    fp12_mul(y2, y2, r);
    fp12_mul(y1, y1, y2);
    fp12_frob(y2, y3, 1);
    fp12_mul(out, y1, y2);
}

DEV void store_be48(uint8_t *dst, const Fp &a) {
    Fp c;
    from_mont(c, a);
#pragma unroll
    for (int w = 0; w < NL; ++w) {
        const uint32_t v = c.l[NL - 1 - w];
        dst[4 * w + 0] = (uint8_t)(v >> 24);
        dst[4 * w + 1] = (uint8_t)(v >> 16);
        dst[4 * w + 2] = (uint8_t)(v >> 8);
        dst[4 * w + 3] = (uint8_t)v;
    }
}

// Kernel 2: one final exponentiation per lane.  `per_out` Miller values
// (1: a pairing, 2: a check) are multiplied first.  gt_out (if set) gets the
// 576-byte GT value; ok_out (if set) gets 1 if the value is 1 (the check
// holds), 0 if not, 2 if an input point was invalid.
#ifndef HB_FE_WPE
#define HB_FE_WPE HB_PAIR_WPE   // A/B: the final exponentiation's own occupancy
#endif
__global__ __launch_bounds__(kPairBlock) __attribute__((amdgpu_waves_per_eu(HB_FE_WPE, HB_FE_WPE))) void final_exp_kernel(
    const uint32_t *__restrict__ ws, size_t n_miller, size_t n_out, int per_out,
    const uint8_t *__restrict__ status, uint8_t *__restrict__ gt_out,
    uint8_t *__restrict__ ok_out) {
    const size_t i = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    if (i >= n_out) return;
    Fp12 f;
    load_f12(f, ws, n_miller, i * per_out);
    int bad = status[i * per_out] == PT_BAD;
    for (int j = 1; j < per_out; ++j) {
        Fp12 g;
        load_f12(g, ws, n_miller, i * per_out + j);
        fp12_mul(f, f, g);
        bad |= status[i * per_out + j] == PT_BAD;
    }
    Fp12 e;
    final_exp(e, f);
    if (gt_out) {
        uint8_t *dst = gt_out + i * 576;
        const Fp2 *c = &e.c0.c0;
        const Fp2 *cs[6] = {&e.c0.c0, &e.c0.c1, &e.c0.c2, &e.c1.c0, &e.c1.c1, &e.c1.c2};
        (void)c;
        for (int k = 0; k < 6; ++k) {
            store_be48(dst + 96 * k, cs[k]->c0);
            store_be48(dst + 96 * k + 48, cs[k]->c1);
        }
    }
    if (ok_out) ok_out[i] = bad ? 2 : (fp12_is_one(e) ? 1 : 0);
}

}  // namespace

// The kernels run at 4 waves/SIMD (128 VGPRs, the rest of the tower state in
// scratch); 1 and 2 waves measured within 5 %.
hipError_t launch_pairing_miller(const uint8_t *g1, size_t g1_stride, const uint8_t *g2,
                                 size_t g2_stride, size_t n, int pair_inputs, uint32_t *ws,
                                 uint8_t *status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((n + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL(miller_kernel, dim3(blocks), dim3(kPairBlock), 0, s, g1, g1_stride, g2, g2_stride, n,
                       pair_inputs, ws, status);
    return hipGetLastError();
}

hipError_t launch_pairing_miller2(const uint8_t *g1, const uint8_t *g2, size_t count,
                                  uint32_t *ws, uint8_t *status, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((count + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL(miller2_kernel, dim3(blocks), dim3(kPairBlock), 0, s, g1, g2, count, ws,
                       status);
    return hipGetLastError();
}

size_t pairing_prepared_words(size_t points) { return points * (size_t)kLines * kLineWords; }

hipError_t launch_g2_prepare(const uint8_t *g2, size_t count, uint32_t *prep, uint8_t *pst,
                             hipStream_t s) {
    if (count == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((count + kPairBlock - 1) / kPairBlock) * (HB_G2_SPLIT ? 2 : 1);
    hipLaunchKernelGGL(g2_prepare_kernel, dim3(blocks), dim3(kPairBlock), 0, s, g2, count, prep,
                       pst);
    return hipGetLastError();
}

hipError_t launch_pairing_miller_prepared(const uint8_t *g1, const uint32_t *prep,
                                          const uint8_t *pst, const uint32_t *ib,
                                          const uint32_t *id, size_t points, size_t count,
                                          uint32_t *ws, uint8_t *status, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (points == 0) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((count + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL(miller_prepared_kernel<false>, dim3(blocks), dim3(kPairBlock), 0, s, g1,
                       nullptr, nullptr, nullptr, (size_t)0, prep, pst, ib, id, points, count, ws,
                       status);
    return hipGetLastError();
}

size_t g1_key_words(size_t points) { return points * (size_t)kG1KeyWords; }

hipError_t launch_pairing_miller_prepared_pts(const uint32_t *atab, const uint8_t *ast,
                                              const uint32_t *keys, const uint8_t *kst,
                                              const uint32_t *ic, size_t nkeys,
                                              const uint32_t *prep, const uint8_t *pst,
                                              const uint32_t *ib, const uint32_t *id,
                                              size_t points, size_t count, uint32_t *ws,
                                              uint8_t *status, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (points == 0 || nkeys == 0) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((count + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL((miller_prepared_kernel<true, true>), dim3(blocks), dim3(kPairBlock), 0, s,
                       nullptr, keys, kst, ic, nkeys, prep, pst, ib, id, points, count, ws, status,
                       atab, ast);
    return hipGetLastError();
}

hipError_t launch_g1_prepare(const uint8_t *g1, size_t count, uint32_t *keys, uint8_t *kst,
                             hipStream_t s) {
    if (count == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((count + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL(g1_prepare_kernel, dim3(blocks), dim3(kPairBlock), 0, s, g1, count, keys,
                       kst);
    return hipGetLastError();
}

hipError_t launch_pairing_miller_prepared_keys(const uint8_t *g1_a, const uint32_t *keys,
                                               const uint8_t *kst, const uint32_t *ic,
                                               size_t nkeys, const uint32_t *prep,
                                               const uint8_t *pst, const uint32_t *ib,
                                               const uint32_t *id, size_t points, size_t count,
                                               uint32_t *ws, uint8_t *status, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (points == 0 || nkeys == 0) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((count + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL(miller_prepared_kernel<true>, dim3(blocks), dim3(kPairBlock), 0, s, g1_a,
                       keys, kst, ic, nkeys, prep, pst, ib, id, points, count, ws, status);
    return hipGetLastError();
}

hipError_t launch_pairing_final(const uint32_t *ws, size_t n_miller, size_t n_out, int per_out,
                                const uint8_t *status, uint8_t *gt_out, uint8_t *ok_out,
                                hipStream_t s) {
    if (n_out == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((n_out + kPairBlock - 1) / kPairBlock);
    hipLaunchKernelGGL(final_exp_kernel, dim3(blocks), dim3(kPairBlock), 0, s, ws, n_miller, n_out, per_out,
                       status, gt_out, ok_out);
    return hipGetLastError();
}

}  // namespace hbrbc
