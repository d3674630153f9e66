// jit.hpp -- matrix-specialised GF(2^8) XOR-network kernels (see jit.hip).  Internal.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace hbrbc {

// One hiprtc program: out_row[t] = sum_jj coefs[t][jj] * in_row[jj] over
// GF(2^8), every coefficient compiled into the code.
//  * Coding::encode: in_rows = data rows 0..k-1, out_rows = a group of parity
//    rows; `fused` adds the frame+encode twin NAME_fe that reads the payload
//    instead of the data rows (broadcast.rs:174-193).
//  * reconstruct of one cached erasure pattern: in_rows = the first k present
//    rows, out_rows = (a group of) the missing rows, coefs = the decode rows;
//    `guard` = the pattern's hash, so instances of other patterns return.
// Row placement: row j at (j / rb) * block_stride + (j % rb) * shard_stride
// past the instance base (rb >= 256: plain shard-major).
struct XorProgram {
    std::string name;
    std::vector<int> in_rows, out_rows;
    std::vector<uint8_t> coefs;  // [out_rows.size()][in_rows.size()]
    int rt = 2, depth = 4, rb = 256;
    // > 0: a raw s_barrier after every `sync` input rows (every wave runs one
    // pass, so the waves of a workgroup stream the input rows in lockstep)
    int sync = 0;
    // prefetch depth of the frame+encode twin (its rows are 36 loaded bytes)
    int fdepth = 2;
    // frame+encode twin: the data-row stores spread over the passes (else pass 0)
    bool spread = true;
    // lane byte positions: two 16-byte pieces 1 KB apart (else 32 consecutive)
    bool split = true;
    uint64_t guard = 0;
    bool fused = false;
    // fused unframe (decoders): payload bytes of the data rows (< uf_k) this
    // program rebuilds, and of its input data rows if uf_inputs (one program
    // of a pattern writes them); 0 = none
    int uf_k = 0;
    bool uf_inputs = false;
    // LDS-staged form (gen_xor_kernel_lds): each input transposed once per
    // workgroup, planes shared through LDS; stages of lds_stage inputs
    bool lds = false;
    int lds_stage = 0;
    // network: 0 auto (nibble-subset for passes <= 8 rows, else pairwise),
    // 1 pairwise, 2 nibble-subset
    int net = 0;
    // > 0: amdgpu_waves_per_eu (the register budget the compiler targets)
    int wpe = 0;
};

// Kernel argument list shared by every generated kernel (hipModuleLaunchKernel).
struct XorArgs {
    uint8_t *base;
    unsigned long inst_stride, shard_stride, block_stride;
    unsigned row_bytes, waves_per_row;
    const uint8_t *payloads;
    unsigned long payload_stride;
    unsigned P, S;
    const int *pat;
    const unsigned long *slot_hash;
    int hash_slots;
    int p_only;
    // fused unframe: payload slab (nullptr = off), its stride, reconstruct status
    uint8_t *uf_payload;
    unsigned long uf_stride;
    const int *uf_status;
};

// Waves per workgroup of a program with npass passes (one per pass, <= 8).
int xor_waves(int npass);
std::string gen_xor_source(const XorProgram &p);
// hiprtc-compile a generated source for gfx950 (no device needed).  0 on success.
int compile_source(const std::string &src, std::vector<char> &code, std::string &log);

// Names: encoder group (k, m, rt, depth, parity rows [r_lo, r_hi), rows per
// block) and decoder group (n, pattern hash, rt, depth, output rows [r_lo,
// r_hi) of the pattern's missing-row list, rows per block).
std::string encode_kernel_name(size_t k, size_t m, int rt, int depth, int r_lo, int r_hi, int rb,
                               int sync = 0, int fdepth = 2, bool spread = true,
                               bool split = false);
std::string decode_kernel_name(size_t n, uint64_t hash, int rt, int depth, int r_lo, int r_hi,
                               int rb, int sync = 0, bool split = true);
// Output-row groups [lo, hi), one hiprtc program each (large matrices are
// split so each program stays near 4096 coefficients).
std::vector<std::pair<int, int>> xor_groups(size_t nin, size_t nout, int rt);

}  // namespace hbrbc
