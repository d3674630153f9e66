// jit.hpp -- specialised RS encode kernels (see jit.hip).  Internal.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace hbrbc {

// Kernel symbol of the specialised encoder for (k, m, rt, depth); `fused`
// names its frame+encode twin (which keeps min(depth, 2) rows in flight).
std::string encode_kernel_name(size_t k, size_t m, int rt, int depth, bool fused);
inline int fused_depth(int depth) { return depth < 2 ? depth : 2; }
// HIP source of the module: the encode kernel and the frame+encode kernel;
// parity_rows = the m x k parity block of the encoding matrix (rows k..k+m-1
// of rse build_matrix), row-major; `depth` = data rows in flight ahead of
// the one being multiplied.
std::string gen_encode_source(size_t k, size_t m, const uint8_t *parity_rows, int rt, int depth);
// hiprtc-compile it for gfx950 (no device needed).  0 on success.
int compile_encode(size_t k, size_t m, const uint8_t *parity_rows, int rt, int depth,
                   std::vector<char> &code, std::string &log);

}  // namespace hbrbc
