// jit.hpp -- specialised RS encode kernels (see jit.hip).  Internal.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace hbrbc {

// Kernel symbol of the specialised encoder for parity rows [r_lo, ...) of
// (k, m) with tile rt and prefetch depth; `fused` names its frame+encode twin
// (which keeps min(depth, 2) rows in flight).
std::string encode_kernel_name(size_t k, size_t m, int rt, int depth, bool fused, int r_lo);
// Parity-row groups [lo, hi), one hiprtc program each (large matrices are
// split so each program stays near 4096 coefficients).
std::vector<std::pair<int, int>> encode_groups(size_t k, size_t m, int rt);
inline int fused_depth(int depth) { return depth < 2 ? depth : 2; }
// HIP source of the module: the encode kernel and the frame+encode kernel;
// parity_rows = the m x k parity block of the encoding matrix (rows k..k+m-1
// of rse build_matrix), row-major; `depth` = data rows in flight ahead of
// the one being multiplied.
std::string gen_encode_source(size_t k, size_t m, const uint8_t *parity_rows, int rt, int depth,
                              int r_lo, int r_hi);
// hiprtc-compile one group for gfx950 (no device needed).  0 on success.
int compile_encode(size_t k, size_t m, const uint8_t *parity_rows, int rt, int depth, int r_lo,
                   int r_hi, std::vector<char> &code, std::string &log);

}  // namespace hbrbc
