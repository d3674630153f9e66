// jit.hip -- matrix-specialised GF(2^8) kernels, generated per coefficient
// matrix and compiled with hiprtc for gfx950.
//
// Why: Coding::encode (broadcast.rs:193 -> rse encode) multiplies the k data
// rows by the fixed m x k parity block of rse `build_matrix(k, n)`, and a
// reconstruct of one erasure pattern (broadcast.rs:569 -> rse reconstruct,
// whose decode matrix rse caches per pattern) multiplies the first k present
// rows by a fixed recovery matrix.  The generic bit-sliced kernel (kernels.hip,
// gf_bitslice_kernel) reads every coefficient at run time and pays a
// wave-uniform branch per coefficient bit plus the doubling chain.  With the
// matrix known in advance each product c * x becomes a fixed XOR network on
// the 8 bit planes of x: output plane q of c*x is the XOR of the input planes
// p with bit q of c*2^p set.  The generated kernel is that network written
// out for every (output row, input row), accumulated with three-input XORs
// (v_bitop3): about 2.25 VALU per plane per coefficient against ~4 XORs +
// branches in the generic kernel, and no branches at all.  Passes of at most
// 8 rows use a nibble-subset network instead (one VALU per plane per
// coefficient, gen_nibble_network); at 14-row passes its longer live ranges
// cost occupancy and it measured slower (5.7 -> 9.0 ms, cfg3).
//
// Layout and lane mapping are those of gf_bitslice_kernel: a lane owns 32
// consecutive byte positions of every row; a workgroup holds one wave per
// pass (up to 8) over the same positions, wave w producing passes w, w+8, ...
// of rt output rows.  Rows are addressed through one buffer resource per row block (the
// blocked layouts of the validator-sharded simulation, launchers.hpp RowMap)
// and an SGPR row offset.  Output is bit-identical to the generic kernel
// (tests compare both with the oracle).
//
// Code objects are cached as files under <lib dir>/jit (names from
// encode_kernel_name / decode_kernel_name + "_v23.co");
// __graft_entry__.build() pre-generates the encoders of the BASELINE
// validator counts and the decoders the bench's fixed patterns need.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "jit.hpp"

namespace hbrbc {

namespace {

uint8_t gf_mul_host(uint8_t a, uint8_t b) {
    // shift-and-add with the rse generator polynomial x^8+x^4+x^3+x^2+1 (0x11D)
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        const bool hi = a & 0x80;
        a = (uint8_t)(a << 1);
        if (hi) a ^= 0x1D;
        b >>= 1;
    }
    return r;
}

// hiprtc sources get the HIP device API implicitly and no system headers.
const char *kPrelude = R"(
typedef unsigned int uint32_t;
typedef unsigned char uint8_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#ifndef HB_ST_AUX
#define HB_ST_AUX 2   // cache policy of the row stores: non-temporal (encode 5.7 -> 5.15 ms, cfg3)
#endif
// 32 bytes starting `bs` (0..3, wave-uniform) bytes into the 36 loaded bytes
// (q0, q1, q2[0]): eight v_alignbyte with a scalar shift
__device__ __forceinline__ void hb_window(const u32x4 q0, const u32x4 q1, const uint32_t q2,
                                          unsigned bs, uint32_t (&o)[8]) {
    const uint32_t w[9] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3], q2};
    _Pragma("unroll") for (int i = 0; i < 8; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], bs);
}
// split lanes: two 16-byte windows from 20 loaded bytes each (q, q2)
__device__ __forceinline__ void hb_window2(const u32x4 qa, const uint32_t qa2, const u32x4 qb,
                                           const uint32_t qb2, unsigned bs, uint32_t (&o)[8]) {
    const uint32_t w[10] = {qa[0], qa[1], qa[2], qa[3], qa2, qb[0], qb[1], qb[2], qb[3], qb2};
    _Pragma("unroll") for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], bs);
    _Pragma("unroll") for (int i = 0; i < 4; ++i) o[4 + i] = __builtin_amdgcn_alignbyte(w[i + 6], w[i + 5], bs);
}
// The window of a lane whose 32 framed bytes start at lb < 4, i.e. inside
// the 4-byte BE32 length prefix (broadcast.rs:175-177; only offset 0 of rows
// with j * S < 4): header bytes hdr[lb..3], then payload bytes 0..
// q0, q1 = payload dwords 0..7 (HB_LDF clamps that lane's load address to 0).
__device__ __forceinline__ void hb_frame_head(const u32x4 q0, const u32x4 q1, unsigned P,
                                              unsigned lb, uint32_t (&x)[8]) {
    const uint32_t w[9] = {__builtin_bswap32(P), q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
    _Pragma("unroll") for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], lb);
}
// split lanes: only the first 16-byte window starts in the prefix
__device__ __forceinline__ void hb_frame_head2(const u32x4 qa, unsigned P, unsigned lb, uint32_t (&x)[8]) {
    const uint32_t w[5] = {__builtin_bswap32(P), qa[0], qa[1], qa[2], qa[3]};
    _Pragma("unroll") for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], lb);
}
// Fused unframe (the `_uf` decoder variants only): 16 bytes of data row `row`
// at byte `pos` are payload bytes row*S + pos - 4 .. +15.  Whole chunks inside
// the payload go as one 16-byte store at any byte alignment (global memory in
// unaligned mode); the edge chunks (length prefix, each row's partial last
// chunk) are copied from the shard rows by the fixup kernel -- kernels.hip
// unframe_put.  Any payload code in a decoder slows it even when unused (a
// branch splits the straight-line program; dropped buffer stores still hold
// the load pipeline's vmcnt waits), so the plain decoders carry none and a
// call that fuses loads the _uf programs.
typedef unsigned int hb_u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ void hb_uf_put(uint8_t *pb, unsigned S, unsigned row, unsigned pos,
                                          uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const long dst = (long)row * S + pos - 4;
    if (pos + 16u <= S && dst >= 0)
        *reinterpret_cast<hb_u32x4_a1 *>(pb + dst) = (hb_u32x4_a1){a, b, c, d};
}
// 8x32 bit transpose of 8 dwords (three delta swaps; an involution)
__device__ __forceinline__ void hb_tr(uint32_t (&w)[8]) {
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
)";

// coefficient of (output t, input jj)
struct CoefView {
    const uint8_t *c;
    size_t nin;
    uint8_t at(int t, size_t jj) const { return c[(size_t)t * nin + jj]; }
};

// Nibble-subset XOR network of input jj for output rows t0..t0+rows-1:
// output plane q of c*x is the XOR of a low-nibble subset (planes 0-3) and a
// high-nibble subset (planes 4-7) of the input planes.  The subset XORs used
// by this input are built once (<= 11 + 11 ops) and shared by every row of
// the pass; each accumulator then takes exactly one op.  Fewer VALU than the
// pairwise network but more values live across the row, so it is used for
// short passes only (rt <= 8; at rt 14 it cost 2 waves/SIMD of occupancy,
// and the N = 250 programs run faster with 12-row pairwise passes).
void gen_nibble_network(std::ostringstream &o, const CoefView &cv, int t0, int rows, size_t jj) {
    std::vector<std::pair<int, int>> tgt((size_t)rows * 8, {0, 0});
    bool used[2][16] = {};
    for (int t = 0; t < rows; ++t) {
        const uint8_t c = cv.at(t0 + t, jj);
        if (!c) continue;
        uint8_t col[8];
        for (int q = 0; q < 8; ++q) col[q] = gf_mul_host(c, (uint8_t)(1u << q));
        for (int q = 0; q < 8; ++q) {
            int lo = 0, hi = 0;
            for (int pp = 0; pp < 4; ++pp) lo |= ((col[pp] >> q) & 1) << pp;
            for (int pp = 4; pp < 8; ++pp) hi |= ((col[pp] >> q) & 1) << (pp - 4);
            tgt[(size_t)t * 8 + q] = {lo, hi};
            used[0][lo] = used[1][hi] = true;
        }
    }
    // a single plane is x[] itself; 2 / 3 planes one XOR / bitop3 of planes;
    // 4 planes fold the {0,1} subset
    auto sname = [](int h, int s) {
        if (__builtin_popcount(s) == 1) return "x[" + std::to_string(4 * h + __builtin_ctz(s)) + "]";
        return std::string(h ? "h" : "l") + std::to_string(s);
    };
    for (int h = 0; h < 2; ++h) {
        if (used[h][15]) used[h][3] = true;
        for (int s = 3; s < 16; ++s) {
            if (!used[h][s] || __builtin_popcount(s) < 2) continue;
            int pl[4], np = 0;
            for (int b = 0; b < 4; ++b)
                if (s >> b & 1) pl[np++] = 4 * h + b;
            o << "        const uint32_t " << sname(h, s) << " = ";
            if (np == 2)
                o << "x[" << pl[0] << "] ^ x[" << pl[1] << "];\n";
            else if (np == 3)
                o << "__builtin_amdgcn_bitop3_b32(x[" << pl[0] << "], x[" << pl[1] << "], x[" << pl[2]
                  << "], 0x96);\n";
            else
                o << "__builtin_amdgcn_bitop3_b32(" << sname(h, 3) << ", x[" << 4 * h + 2 << "], x["
                  << 4 * h + 3 << "], 0x96);\n";
        }
    }
    for (int t = 0; t < rows; ++t)
        for (int q = 0; q < 8; ++q) {
            const auto lh = tgt[(size_t)t * 8 + q];
            const std::string acc = "a[" + std::to_string(t) + "][" + std::to_string(q) + "]";
            if (lh.first && lh.second)
                o << "        " << acc << " = __builtin_amdgcn_bitop3_b32(" << acc << ", "
                  << sname(0, lh.first) << ", " << sname(1, lh.second) << ", 0x96);\n";
            else if (lh.first || lh.second)
                o << "        " << acc << " ^= " << (lh.first ? sname(0, lh.first) : sname(1, lh.second))
                  << ";\n";
        }
}

// Pairwise network: term lists of every (row, plane); output plane q of c*x
// is the XOR of the planes p with bit q of c*2^p set.  Terms are paired in
// order ((p1,p2), (p3,p4), ...); the pair XORs are computed once per input
// and shared by all rows of the pass, and each v_bitop3 folds two pairs --
// up to four planes -- into an accumulator.
void gen_pair_network(std::ostringstream &o, const CoefView &cv, int t0, int rows, size_t jj) {
    std::vector<std::vector<int>> elems((size_t)rows * 8);
    bool used[8][8] = {};
    for (int t = 0; t < rows; ++t) {
        const uint8_t c = cv.at(t0 + t, jj);
        if (!c) continue;
        uint8_t col[8];
        for (int q = 0; q < 8; ++q) col[q] = gf_mul_host(c, (uint8_t)(1u << q));
        for (int q = 0; q < 8; ++q) {
            std::vector<int> terms;
            for (int pp = 0; pp < 8; ++pp)
                if ((col[pp] >> q) & 1) terms.push_back(pp);
            auto &el = elems[(size_t)t * 8 + q];
            for (size_t i = 0; i + 1 < terms.size(); i += 2) {
                used[terms[i]][terms[i + 1]] = true;
                el.push_back(8 + terms[i] * 8 + terms[i + 1]);  // pair id
            }
            if (terms.size() & 1) el.push_back(terms.back());   // single plane
        }
    }
    for (int a = 0; a < 8; ++a)
        for (int b = a + 1; b < 8; ++b)
            if (used[a][b])
                o << "        const uint32_t p" << a << b << " = x[" << a << "] ^ x[" << b << "];\n";
    auto name = [](int e) {
        return e < 8 ? "x[" + std::to_string(e) + "]"
                     : "p" + std::to_string((e - 8) / 8) + std::to_string((e - 8) % 8);
    };
    for (int t = 0; t < rows; ++t)
        for (int q = 0; q < 8; ++q) {
            const auto &el = elems[(size_t)t * 8 + q];
            const std::string acc = "a[" + std::to_string(t) + "][" + std::to_string(q) + "]";
            size_t i = 0;
            for (; i + 1 < el.size(); i += 2)
                o << "        " << acc << " = __builtin_amdgcn_bitop3_b32(" << acc << ", "
                  << name(el[i]) << ", " << name(el[i + 1]) << ", 0x96);\n";
            if (i < el.size()) o << "        " << acc << " ^= " << name(el[i]) << ";\n";
        }
}

// Network of input jj for output rows t0..t0+rows-1 (net: 0 auto, 1 pairwise,
// 2 nibble-subset).
void gen_network(std::ostringstream &o, const CoefView &cv, int t0, int rows, size_t jj, int rt,
                 int net) {
    if (net == 2 || (net == 0 && rt <= 8))
        gen_nibble_network(o, cv, t0, rows, jj);
    else
        gen_pair_network(o, cv, t0, rows, jj);
}

// Signature, guard, lane mapping, buffer resources and the load macros shared
// by both kernel forms.  `fused` = the frame+encode twin.
void gen_prologue(std::ostringstream &o, const XorProgram &p, bool fused, int npass,
                  const std::set<int> &blocks, const char *d2, const std::string &lds_decl) {
    auto blk = [&](int row) { return row / p.rb; };
    (void)blk;
    // one wave per pass (up to 8): the waves of a workgroup stream the same
    // input rows together, so each row comes from HBM about once per program
    // (4 waves over 6 passes fetched 4.6x the input at cfg5, PMC FETCH_SIZE)
    o << "\nextern \"C\" __global__ __launch_bounds__(" << xor_waves(npass) * 64 << ") "
      << (p.wpe > 0 ? "__attribute__((amdgpu_waves_per_eu(" + std::to_string(p.wpe) + "))) " : std::string())
      << "void "
      << p.name << (fused ? "_fe" : "")
      << "(uint8_t *__restrict__ base, unsigned long inst_stride, unsigned long shard_stride,\n"
         "    unsigned long block_stride, unsigned row_bytes, unsigned waves_per_row,\n"
         "    const uint8_t *__restrict__ payloads, unsigned long payload_stride, unsigned P, unsigned S,\n"
         "    const int *__restrict__ pat, const unsigned long *__restrict__ slot_hash, int hash_slots,\n"
         "    int p_only, uint8_t *__restrict__ uf_payload, unsigned long uf_stride,\n"
         "    const int *__restrict__ uf_status) {\n"
      << lds_decl
      << "  const unsigned long inst = blockIdx.x / waves_per_row;\n";
    if (p.guard) {
        // reconstruct of one cached erasure pattern: other patterns return
        char g[64];
        snprintf(g, sizeof g, "0x%016llxull", (unsigned long long)p.guard);
        o << "  { const int sl_ = pat[inst];\n"
             "    if (sl_ >= hash_slots || slot_hash[sl_] != "
          << g << ") return; }\n";
    }
    // a lane's 32 byte positions: off..off+15 and off2..off2+15.  Default:
    // 32 consecutive bytes (off2 = off + 16); split: two 16-byte pieces 1 KB
    // apart, so every load and store instruction of a wave covers 1 KB of
    // consecutive bytes instead of 64 pieces of 16 with 16-byte gaps
    o << "  const int wave = (int)(threadIdx.x >> 6), nw = (int)(blockDim.x >> 6);\n"
         "  const unsigned wchunk = blockIdx.x - (unsigned)inst * waves_per_row, lane = threadIdx.x & 63u;\n"
      << (p.split ? "  unsigned off = wchunk * 2048u + lane * 16u;\n" : "  unsigned off = (wchunk * 64u + lane) * 32u;\n")
      << "  const bool active = off < row_bytes;\n"
         "  if (!active) off = row_bytes - 16u;\n"
         "  const bool full = off + " << d2 << " + 16u <= row_bytes;\n"
         "  const unsigned off2 = full ? off + " << d2 << " : off;\n"
         // raw buffer ops: each row block's base lives in a scalar resource,
         // the row offset (row % rb) * shard_stride in an SGPR (soffset) and
         // the lane offset in one VGPR -- no per-lane 64-bit address per row
         "  uint8_t *const ib = base + inst * inst_stride;\n";
    if (p.uf_k > 0)
        o << "  uint8_t *const ufp = (uf_payload && uf_status[inst] == 0) ? uf_payload + inst * uf_stride"
             " : (uint8_t *)0;\n";
    for (int q : blocks)
        o << "  const __amdgpu_buffer_rsrc_t rs" << q << " = __builtin_amdgcn_make_buffer_rsrc(ib"
          << (q ? " + " + std::to_string(q) + "ul * block_stride" : std::string()) << ", (short)0, "
          << "0x7fffffff, 0x00020000);\n";
    o << "  const unsigned sst = (unsigned)shard_stride;\n"
         "#define HB_LD(L, H, Q, R) { L = __builtin_amdgcn_raw_buffer_load_b128(rs##Q, off, (R) * sst, 0); "
         "H = __builtin_amdgcn_raw_buffer_load_b128(rs##Q, off2, (R) * sst, 0); }\n";
    if (fused)
        // framing (broadcast.rs:174-189) folded into the loads: logical byte b
        // of the framed value is payload byte b - 4.  The buffer resource
        // covers the whole dwords of the payload (P & ~3 bytes; range checks
        // are per dword), so everything past them reads 0; the 0-3 bytes of a
        // partial last dword are added, with their parity, by frame_fixup.
        o << "  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(\n"
             "      (void *)(payloads + inst * payload_stride), (short)0, (int)(P & ~3u), 0x00020000);\n"
             "  const bool edge = !__all(off + " << d2 << " + 16u <= S);\n"
             // dword-aligned start: the 32 framed bytes of a lane are bytes
             // bs..bs+31 of 36 loaded bytes, bs = (j*S - 4) & 3 (uniform per row)
             // (the address add is volatile asm: LLVM would otherwise hoist every
             // row's address out of the pass loop and keep k of them live)
             "#define HB_LDF(Q0, Q1, Q2, j) { unsigned a_; "
             "__asm__ volatile(\"v_add_u32 %0, %1, %2\" : \"=v\"(a_) : \"s\"((j) * S - 4u), \"v\"(off)); "
             "a_ &= ~3u; "
             // a window starting inside the length prefix loads payload dwords 0..8
             "if ((j) < 4u && (j) * S + off < 4u) a_ = 0u; "
             "Q0 = __builtin_amdgcn_raw_buffer_load_b128(pr, a_, 0, 0); "
             "Q1 = __builtin_amdgcn_raw_buffer_load_b128(pr, a_ + 16u, 0, 0); "
             "Q2 = __builtin_amdgcn_raw_buffer_load_b32(pr, a_ + 32u, 0, 0); }\n"
             // split lanes: 20 bytes at each of the two pieces
             "#define HB_LDF2(QA, QA2, QB, QB2, j) { unsigned a_, b_; "
             "__asm__ volatile(\"v_add_u32 %0, %1, %2\" : \"=v\"(a_) : \"s\"((j) * S - 4u), \"v\"(off)); "
             "__asm__ volatile(\"v_add_u32 %0, %1, %2\" : \"=v\"(b_) : \"s\"((j) * S - 4u), \"v\"(off2)); "
             "a_ &= ~3u; b_ &= ~3u; "
             "if ((j) < 4u && (j) * S + off < 4u) a_ = 0u; "
             "QA = __builtin_amdgcn_raw_buffer_load_b128(pr, a_, 0, 0); "
             "QA2 = __builtin_amdgcn_raw_buffer_load_b32(pr, a_ + 16u, 0, 0); "
             "QB = __builtin_amdgcn_raw_buffer_load_b128(pr, b_, 0, 0); "
             "QB2 = __builtin_amdgcn_raw_buffer_load_b32(pr, b_ + 16u, 0, 0); }\n";
}

// One kernel of a program: `fused` = the frame+encode twin.
std::string gen_xor_kernel(const XorProgram &p, bool fused) {
    const size_t nin = p.in_rows.size();
    const int nout = (int)p.out_rows.size();
    // npass passes of at most rt rows, balanced (42 rows at rt 12: 11, 11,
    // 10, 10 rather than 12, 12, 12, 6 -- the longest pass sets the time)
    const int npass = (nout + p.rt - 1) / p.rt;
    auto pass_lo = [&](int ps) { return ps * (nout / npass) + std::min(ps, nout % npass); };
    const int rt = (nout + npass - 1) / npass;
    const int depth = fused ? p.fdepth : p.depth;  // 36 bytes per row in flight when fused
    const int nbuf = depth + 1;
    const int rb = p.rb;
    // every wave runs exactly one pass only when npass <= 8 waves: only then
    // do all waves reach the same barriers
    const bool lockstep = p.sync > 0 && npass <= 8 && npass > 1;
    const CoefView cv{p.coefs.data(), nin};
    auto blk = [&](int row) { return row / rb; };
    auto rin = [&](int row) { return row % rb; };
    std::set<int> blocks;
    for (int r : p.in_rows) blocks.insert(blk(r));
    for (int r : p.out_rows) blocks.insert(blk(r));
    const char *d2 = p.split ? "1024u" : "16u";
    std::ostringstream o;
    gen_prologue(o, p, fused, npass, blocks, d2, "");

    // p_only >= 0: this launch runs that one pass with one wave per workgroup
    // (the host launches the passes one after another, so every wave on a CU
    // runs the same straight-line code); p_only < 0: wave w runs passes w,
    // w + nw, ... of the same byte positions
    o << "  const int p_lo = p_only >= 0 ? p_only : __builtin_amdgcn_readfirstlane(wave);\n"
         "  const int p_hi = p_only >= 0 ? p_only + 1 : " << npass << ";\n"
         "  const int p_st = p_only >= 0 ? 1 : nw;\n"
         "  for (int p = p_lo; p < p_hi; p += p_st) {\n    switch (p) {\n";
    for (int ps = 0; ps < npass; ++ps) {
        const int t0 = pass_lo(ps);
        const int rows = pass_lo(ps + 1) - t0;
        // a distinct barrier opens every case, so no common prefix (the first
        // rows' loads) is hoisted above the switch and kept live across it
        o << "    case " << ps << ": {\n      __asm__ volatile(\"; pass " << ps
          << "\" ::: \"memory\");\n      uint32_t a[" << rows << "][8] = {};\n";
        if (fused)
            // S through an opaque SGPR copy per pass: otherwise every pass's row
            // offsets (j * S - 4 and its byte shift) are loop-invariant, get
            // hoisted above the pass loop and spill (41 SGPRs in the cfg3 encoder)
            o << "      unsigned S_; __asm__ volatile(\"s_mov_b32 %0, %1\" : \"=s\"(S_) : \"s\"(S));\n"
                 "      const unsigned S = S_;\n"
                 "      u32x4 q0[" << nbuf << "], q1[" << nbuf << "]; uint32_t q2[" << nbuf << "]"
              << (p.split ? ", q3[" + std::to_string(nbuf) + "]" : std::string()) << ";\n";
        else
            o << "      u32x4 l[" << nbuf << "], h[" << nbuf << "];\n";
        auto load = [&](size_t jj) {
            const int b = (int)(jj % nbuf);
            const int row = p.in_rows[jj];
            if (fused && p.split)
                o << "      HB_LDF2(q0[" << b << "], q2[" << b << "], q1[" << b << "], q3[" << b << "], " << row
                  << "u)";
            else if (fused)
                o << "      HB_LDF(q0[" << b << "], q1[" << b << "], q2[" << b << "], " << row << "u)";
            else
                o << "      HB_LD(l[" << b << "], h[" << b << "], " << blk(row) << ", " << rin(row) << "u)";
            // the empty asm keeps the scheduler from hoisting every row's load to
            // the top of the straight-line pass (hundreds of live VGPRs)
            o << " __asm__ volatile(\"\" ::: \"memory\");\n";
        };
        // inputs 0..depth-1 in flight before the first product; input jj + depth
        // is requested while input jj is consumed (depth rows of HBM latency hidden)
        for (int jj = 0; jj < depth && jj < (int)nin; ++jj) load((size_t)jj);
        for (size_t jj = 0; jj < nin; ++jj) {
            const int cur = (int)(jj % nbuf);
            const int row = p.in_rows[jj];
            if (jj + depth < nin) load(jj + depth);
            if (fused) {
                const std::string c = std::to_string(cur);
                o << "      { uint32_t x[8];\n";
                if (p.split)
                    o << "        hb_window2(q0[" << c << "], q2[" << c << "], q1[" << c << "], q3[" << c
                      << "], (" << row << "u * S - 4u) & 3u, x);\n";
                else
                    o << "        hb_window(q0[" << c << "], q1[" << c << "], q2[" << c << "], (" << row
                      << "u * S - 4u) & 3u, x);\n";
                // windows touching the BE32 payload length (broadcast.rs:175-177);
                // j * S < 4 needs j < 4 since S >= 1
                if (row < 4)
                    o << "        if (" << row << "u * S < 4u) { if (off == 0u) "
                      << (p.split ? "hb_frame_head2(q0[" + c + "], " : "hb_frame_head(q0[" + c + "], q1[" + c + "], ")
                      << "P, " << row << "u * S, x); }\n";
                // positions >= S of this row belong to the next shard: zero
                o << "        if (edge) {\n"
                     "          _Pragma(\"unroll\") for (int i_ = 0; i_ < 8; ++i_) {\n"
                     "            const int lim_ = (int)S - (int)(i_ < 4 ? off + 4 * i_ : off2 + 4 * (i_ - 4));\n"
                     "            x[i_] = lim_ >= 4 ? x[i_] : (lim_ <= 0 ? 0u : x[i_] & (0xFFFFFFFFu >> (8 * (4 - lim_))));\n"
                     "          }\n        }\n";
                // group 0 also writes the framed data rows, pass jj % npass row jj
                // (spread over the waves: a store ahead of a load holds that
                // load's vmcnt wait, and pass 0 storing all 22 rows at cfg3 made
                // it the workgroup's slowest wave)
                if (p.out_rows.front() == (int)nin && (p.spread ? (int)(jj % npass) == ps : ps == 0))
                    o << "        if (active) {\n"
                         "          __builtin_amdgcn_raw_buffer_store_b128((u32x4){x[0], x[1], x[2], x[3]}, rs"
                      << blk(row) << ", off, " << rin(row) << "u * sst, HB_ST_AUX);\n"
                         "          if (full) __builtin_amdgcn_raw_buffer_store_b128((u32x4){x[4], x[5], x[6], x[7]}, "
                         "rs" << blk(row) << ", off2, " << rin(row) << "u * sst, HB_ST_AUX);\n        }\n";
                o << "        hb_tr(x);\n";
            } else {
                const std::string lc = "l[" + std::to_string(cur) + "]";
                o << "      { const u32x4 hh = full ? h[" << cur << "] : (u32x4)(0u);\n"
                  << "        uint32_t x[8] = {" << lc << "[0], " << lc << "[1], " << lc << "[2], " << lc
                  << "[3], hh[0], hh[1], hh[2], hh[3]};\n";
                if (p.uf_k > 0 && p.uf_inputs && ps == 0 && row < p.uf_k)
                    o << "        if (ufp && active) { hb_uf_put(ufp, S, " << row
                      << "u, off, x[0], x[1], x[2], x[3]); if (full) hb_uf_put(ufp, S, " << row
                      << "u, off2, x[4], x[5], x[6], x[7]); }\n";
                o << "        hb_tr(x);\n";
            }
            // short passes: the nibble-subset network (net 0), or as forced
            gen_network(o, cv, t0, rows, jj, rt, p.net);
            // pin the accumulators after every input: without this the
            // reassociation pass flattens each accumulator's whole XOR chain
            // over all inputs and keeps every input's planes live at once
            o << "        for (int t_ = 0; t_ < " << rows << "; ++t_) for (int q_ = 0; q_ < 8; ++q_) "
                 "__asm__ volatile(\"\" : \"+v\"(a[t_][q_]));\n      }\n";
            // lockstep: the passes of a workgroup meet every `sync` rows, so a
            // row's bytes are fetched once and served from L1/L2 to the other
            // waves (a plain s_barrier: the prefetched rows stay in flight)
            if (lockstep && (jj + 1) % (size_t)p.sync == 0 && jj + 1 < nin)
                o << "      __builtin_amdgcn_s_barrier();\n";
        }
        o << "      if (active) {\n";
        for (int t = 0; t < rows; ++t) {
            const int row = p.out_rows[t0 + t];
            const std::string at = "a[" + std::to_string(t) + "]";
            o << "        { hb_tr(" << at << "); const unsigned so_ = " << rin(row) << "u * sst;\n"
              << "          __builtin_amdgcn_raw_buffer_store_b128((u32x4){" << at << "[0], " << at << "[1], "
              << at << "[2], " << at << "[3]}, rs" << blk(row) << ", off, so_, HB_ST_AUX);\n"
              << "          if (full) __builtin_amdgcn_raw_buffer_store_b128((u32x4){" << at << "[4], " << at
              << "[5], " << at << "[6], " << at << "[7]}, rs" << blk(row) << ", off2, so_, HB_ST_AUX); }\n";
            if (p.uf_k > 0 && row < p.uf_k)
                o << "        if (ufp) { hb_uf_put(ufp, S, " << row << "u, off, " << at << "[0], " << at
                  << "[1], " << at << "[2], " << at << "[3]); if (full) hb_uf_put(ufp, S, " << row
                  << "u, off2, " << at << "[4], " << at << "[5], " << at << "[6], " << at << "[7]); }\n";
        }
        o << "      }\n      break; }\n";
    }
    o << "    }\n  }\n}\n#undef HB_LD\n" << (fused ? "#undef HB_LDF\n#undef HB_LDF2\n" : "");
    return o.str();
}

// LDS-staged form (p.lds): every input row of a stage is loaded, framed and
// transposed ONCE per workgroup -- by wave jj % nw -- and its 8 bit planes go
// to LDS ([jj][half][lane] u32x4: conflict-free 16-byte lane slots); after one
// barrier every wave runs its pass over all inputs of the stage from LDS.  In
// the streaming form each of the npass waves loads and transposes every input
// itself (the transposes are ~25 % of a pass's VALU at cfg3) and keeps
// depth + 1 rows of load buffers live beside its accumulators (231 VGPRs, 2
// waves/SIMD); here a pass holds only its accumulators, 8 planes and the
// network's temporaries.  Stages of <= 24 inputs (48 KB of LDS) bound the
// LDS per workgroup; a barrier separates stages (the next stage's planes
// overwrite the buffer).
std::string gen_xor_kernel_lds(const XorProgram &p, bool fused) {
    const int nin = (int)p.in_rows.size();
    const int nout = (int)p.out_rows.size();
    const int npass = (nout + p.rt - 1) / p.rt;
    auto pass_lo = [&](int ps) { return ps * (nout / npass) + std::min(ps, nout % npass); };
    const int rt = (nout + npass - 1) / npass;
    const int nw = xor_waves(npass);
    const int rb = p.rb;
    const CoefView cv{p.coefs.data(), (size_t)nin};
    auto blk = [&](int row) { return row / rb; };
    auto rin = [&](int row) { return row % rb; };
    std::set<int> blocks;
    for (int r : p.in_rows) blocks.insert(blk(r));
    for (int r : p.out_rows) blocks.insert(blk(r));
    const char *d2 = p.split ? "1024u" : "16u";
    const int ss = std::min(nin, p.lds_stage > 0 ? p.lds_stage : 24);
    const int nstage = (nin + ss - 1) / ss;
    std::ostringstream o;
    gen_prologue(o, p, fused, npass, blocks, d2,
                 "  __shared__ u32x4 hb_pl[" + std::to_string(ss) + "][2][64];\n");
    if (fused)
        // S through an opaque SGPR copy: otherwise the row offsets j * S - 4
        // of every input are hoisted and kept live
        o << "  unsigned S_; __asm__ volatile(\"s_mov_b32 %0, %1\" : \"=s\"(S_) : \"s\"(S));\n"
             "  const unsigned Sx = S_;\n";
    o << "  const int w_ = __builtin_amdgcn_readfirstlane(wave);\n"
         "  switch (w_) {\n";
    // one case per wave; a wave runs pass w_ (npass <= 8 = nw here) and
    // loads the inputs jj of every stage with (jj - stage_lo) % nw == w_
    for (int w = 0; w < nw; ++w) {
        const bool has_pass = w < npass;
        const int t0 = has_pass ? pass_lo(w) : 0;
        const int rows = has_pass ? pass_lo(w + 1) - t0 : 0;
        o << "  case " << w << ": {\n    __asm__ volatile(\"; wave " << w << "\" ::: \"memory\");\n";
        if (fused) o << "    const unsigned S = Sx;\n";
        if (rows) o << "    uint32_t a[" << rows << "][8] = {};\n";
        for (int st = 0; st < nstage; ++st) {
            const int lo = st * ss, hi = std::min(nin, lo + ss);
            std::vector<int> mine;
            for (int jj = lo; jj < hi; ++jj)
                if ((jj - lo) % nw == w) mine.push_back(jj);
            // phase 1: load (all of this wave's rows of the stage at once when
            // no accumulators are live yet, else two ahead), frame, transpose
            const int depth = (st == 0) ? (int)mine.size() : std::min<int>(2, (int)mine.size());
            const int nbuf = std::max(1, depth + (st == 0 ? 0 : 1));
            if (!mine.empty()) {
                if (fused)
                    o << "    { u32x4 q0[" << nbuf << "], q1[" << nbuf << "]; uint32_t q2[" << nbuf << "]"
                      << (p.split ? ", q3[" + std::to_string(nbuf) + "]" : std::string()) << ";\n";
                else
                    o << "    { u32x4 l[" << nbuf << "], h[" << nbuf << "];\n";
            }
            auto load = [&](size_t m) {
                const int b = (int)(m % nbuf);
                const int row = p.in_rows[mine[m]];
                if (fused && p.split)
                    o << "      HB_LDF2(q0[" << b << "], q2[" << b << "], q1[" << b << "], q3[" << b << "], " << row << "u)";
                else if (fused)
                    o << "      HB_LDF(q0[" << b << "], q1[" << b << "], q2[" << b << "], " << row << "u)";
                else
                    o << "      HB_LD(l[" << b << "], h[" << b << "], " << blk(row) << ", " << rin(row) << "u)";
                o << " __asm__ volatile(\"\" ::: \"memory\");\n";
            };
            for (int m = 0; m < depth; ++m) load((size_t)m);
            for (size_t m = 0; m < mine.size(); ++m) {
                const int jj = mine[m];
                const int row = p.in_rows[jj];
                const std::string c = std::to_string(m % nbuf);
                if (m + depth < mine.size()) load(m + depth);
                if (fused) {
                    o << "      { uint32_t x[8];\n";
                    if (p.split)
                        o << "        hb_window2(q0[" << c << "], q2[" << c << "], q1[" << c << "], q3[" << c
                          << "], (" << row << "u * S - 4u) & 3u, x);\n";
                    else
                        o << "        hb_window(q0[" << c << "], q1[" << c << "], q2[" << c << "], (" << row
                          << "u * S - 4u) & 3u, x);\n";
                    if (row < 4)
                        o << "        if (" << row << "u * S < 4u) { if (off == 0u) "
                          << (p.split ? "hb_frame_head2(q0[" + c + "], " : "hb_frame_head(q0[" + c + "], q1[" + c + "], ")
                          << "P, " << row << "u * S, x); }\n";
                    o << "        if (edge) {\n"
                         "          _Pragma(\"unroll\") for (int i_ = 0; i_ < 8; ++i_) {\n"
                         "            const int lim_ = (int)S - (int)(i_ < 4 ? off + 4 * i_ : off2 + 4 * (i_ - 4));\n"
                         "            x[i_] = lim_ >= 4 ? x[i_] : (lim_ <= 0 ? 0u : x[i_] & (0xFFFFFFFFu >> (8 * (4 - lim_))));\n"
                         "          }\n        }\n";
                    // the first parity group writes the framed data rows
                    if (p.out_rows.front() == nin)
                        o << "        if (active) {\n"
                             "          __builtin_amdgcn_raw_buffer_store_b128((u32x4){x[0], x[1], x[2], x[3]}, rs"
                          << blk(row) << ", off, " << rin(row) << "u * sst, HB_ST_AUX);\n"
                             "          if (full) __builtin_amdgcn_raw_buffer_store_b128((u32x4){x[4], x[5], x[6], x[7]}, "
                             "rs" << blk(row) << ", off2, " << rin(row) << "u * sst, HB_ST_AUX);\n        }\n";
                } else {
                    o << "      { const u32x4 hh = full ? h[" << c << "] : (u32x4)(0u);\n"
                      << "        uint32_t x[8] = {l[" << c << "][0], l[" << c << "][1], l[" << c << "][2], l[" << c
                      << "][3], hh[0], hh[1], hh[2], hh[3]};\n";
                    if (p.uf_k > 0 && p.uf_inputs && row < p.uf_k)
                        o << "        if (ufp && active) { hb_uf_put(ufp, S, " << row
                          << "u, off, x[0], x[1], x[2], x[3]); if (full) hb_uf_put(ufp, S, " << row
                          << "u, off2, x[4], x[5], x[6], x[7]); }\n";
                }
                o << "        hb_tr(x);\n"
                     "        hb_pl[" << (jj - lo) << "][0][lane] = (u32x4){x[0], x[1], x[2], x[3]};\n"
                     "        hb_pl[" << (jj - lo) << "][1][lane] = (u32x4){x[4], x[5], x[6], x[7]};\n"
                     "      }\n";
            }
            if (!mine.empty()) o << "    }\n";
            o << "    __syncthreads();\n";
            // phase 2: this wave's pass over the stage's inputs
            for (int jj = lo; jj < hi && rows; ++jj) {
                o << "    { const u32x4 pa_ = hb_pl[" << (jj - lo) << "][0][lane], pb_ = hb_pl[" << (jj - lo)
                  << "][1][lane];\n"
                     "      const uint32_t x[8] = {pa_[0], pa_[1], pa_[2], pa_[3], pb_[0], pb_[1], pb_[2], pb_[3]};\n";
                gen_network(o, cv, t0, rows, (size_t)jj, rt, p.net);
                o << "      for (int t_ = 0; t_ < " << rows << "; ++t_) for (int q_ = 0; q_ < 8; ++q_) "
                     "__asm__ volatile(\"\" : \"+v\"(a[t_][q_]));\n"
                     "      __asm__ volatile(\"\" ::: \"memory\");\n    }\n";
            }
            if (st + 1 < nstage) o << "    __syncthreads();\n";
        }
        if (rows) {
            o << "    if (active) {\n";
            for (int t = 0; t < rows; ++t) {
                const int row = p.out_rows[t0 + t];
                const std::string at = "a[" + std::to_string(t) + "]";
                o << "      { hb_tr(" << at << "); const unsigned so_ = " << rin(row) << "u * sst;\n"
                  << "        __builtin_amdgcn_raw_buffer_store_b128((u32x4){" << at << "[0], " << at << "[1], "
                  << at << "[2], " << at << "[3]}, rs" << blk(row) << ", off, so_, HB_ST_AUX);\n"
                  << "        if (full) __builtin_amdgcn_raw_buffer_store_b128((u32x4){" << at << "[4], " << at
                  << "[5], " << at << "[6], " << at << "[7]}, rs" << blk(row) << ", off2, so_, HB_ST_AUX); }\n";
                if (p.uf_k > 0 && row < p.uf_k)
                    o << "      if (ufp) { hb_uf_put(ufp, S, " << row << "u, off, " << at << "[0], " << at
                      << "[1], " << at << "[2], " << at << "[3]); if (full) hb_uf_put(ufp, S, " << row
                      << "u, off2, " << at << "[4], " << at << "[5], " << at << "[6], " << at << "[7]); }\n";
            }
            o << "    }\n";
        }
        o << "    break; }\n";
    }
    o << "  }\n}\n#undef HB_LD\n" << (fused ? "#undef HB_LDF\n#undef HB_LDF2\n" : "");
    return o.str();
}

}  // namespace

int xor_waves(int npass) { return std::max(1, std::min(8, npass)); }

std::string encode_kernel_name(size_t k, size_t m, int rt, int depth, int r_lo, int r_hi, int rb,
                               int sync, int fdepth, bool spread, bool split) {
    char b[128];
    snprintf(b, sizeof b, "hbrbc_enc_k%zu_m%zu_rt%d_d%d_r%d_%d", k, m, rt, depth, r_lo, r_hi);
    std::string s = b;
    if (rb < 256) s += "_b" + std::to_string(rb);
    if (sync > 0) s += "_s" + std::to_string(sync);
    if (fdepth != 2) s += "_f" + std::to_string(fdepth);
    if (!spread) s += "_w0";
    if (!split) s += "_c";
    return s;
}

std::string decode_kernel_name(size_t n, uint64_t hash, int rt, int depth, int r_lo, int r_hi,
                               int rb, int sync, bool split) {
    char b[128];
    snprintf(b, sizeof b, "hbrbc_dec_n%zu_%016llx_rt%d_d%d_r%d_%d", n, (unsigned long long)hash,
             rt, depth, r_lo, r_hi);
    std::string s = b;
    if (rb < 256) s += "_b" + std::to_string(rb);
    if (sync > 0) s += "_s" + std::to_string(sync);
    if (!split) s += "_c";
    return s;
}

std::vector<std::pair<int, int>> xor_groups(size_t nin, size_t nout, int rt) {
    // a group = one hiprtc program; bigger ones compile superlinearly slowly
    // (HBRBC_JIT_GROUP: coefficients per program, A/B)
    const char *ge = getenv("HBRBC_JIT_GROUP");
    const size_t kMaxCoefs = ge ? std::max<size_t>(256, (size_t)atol(ge)) : (size_t)4096;
    std::vector<std::pair<int, int>> g;
    size_t per = nout;
    if (nin * nout > kMaxCoefs) per = std::max<size_t>((size_t)rt, kMaxCoefs / nin / rt * rt);
    // short passes of the LDS form (api.hip spec_lds: >= 16 inputs): at most
    // eight per program (one wave each, the form's limit), so 84 rows of 6-row
    // passes are two programs, 48 + 36
    if (nin >= 16 && rt <= 8) per = std::min(per, (size_t)(8 * rt));
    for (size_t lo = 0; lo < nout; lo += per) g.push_back({(int)lo, (int)std::min(nout, lo + per)});
    return g;
}

std::string gen_xor_source(const XorProgram &p) {
    const int npass = (int)((p.out_rows.size() + p.rt - 1) / p.rt);
    const bool lds = p.lds && npass >= 2 && npass <= 8;
    auto gen = [&](bool fused) { return lds ? gen_xor_kernel_lds(p, fused) : gen_xor_kernel(p, fused); };
    std::string s = std::string(kPrelude) + gen(false);
    if (p.fused) s += gen(true);
    return s;
}

int compile_source(const std::string &src, std::vector<char> &code, std::string &log) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "hbrbc_xor.hip", 0, nullptr, nullptr) !=
        HIPRTC_SUCCESS) {
        log = "hiprtcCreateProgram failed";
        return -1;
    }
    // HBRBC_ST_AUX (A/B): cache-policy bits of the row stores
    const char *aux = getenv("HBRBC_ST_AUX");
    const std::string aux_def = std::string("-DHB_ST_AUX=") + (aux ? aux : "2");
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", aux_def.c_str()};
    const hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
    size_t lsz = 0;
    hiprtcGetProgramLogSize(prog, &lsz);
    if (lsz > 1) {
        log.resize(lsz);
        hiprtcGetProgramLog(prog, &log[0]);
    }
    if (r != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return -2;
    }
    size_t csz = 0;
    hiprtcGetCodeSize(prog, &csz);
    code.resize(csz);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return 0;
}

}  // namespace hbrbc
