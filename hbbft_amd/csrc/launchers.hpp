// launchers.hpp -- host-side launch wrappers for the kernels in kernels.hip.
// Internal to libhbrbc.so (the public surface is include/hbrbc.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace hbrbc {

// Frame `count` payloads into the data rows of a shard slab (zero padding).
hipError_t launch_frame(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                        size_t count, uint8_t *shards, size_t shard_len, size_t shard_stride,
                        size_t inst_stride, size_t data_shards, hipStream_t s);

// The last payload_len & 3 payload bytes of a fused frame+encode: data byte
// plus its GF(2^8) contribution to every parity row (matrix = n x k, device).
hipError_t launch_frame_fixup(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                              uint8_t *shards, size_t shard_len, size_t shard_stride,
                              size_t inst_stride, size_t k, size_t m, const uint8_t *matrix,
                              size_t count, hipStream_t s);

// out_row[r] = sum_j C[r][j] * in_row[in_idx[j]] on 16-byte chunks, for
// nout (per instance or uniform) output rows out_idx[r].
struct GfApplyArgs {
    uint8_t *base;
    size_t inst_stride, shard_stride;
    int n16;                    // 16-byte chunks per row
    const uint4 *tables;        // split-2-bit entries [inst][pass][nin][rt]
    size_t tab_inst_stride;     // in entries (0: shared)
    const uint32_t *in_idx;     // [inst][nin]
    size_t in_idx_stride;       // 0: shared
    const uint32_t *out_idx;    // [inst][max_out]
    size_t out_idx_stride;      // 0: shared
    const int *nout;            // [inst] or nullptr
    int nout_uniform;
    int max_rows;               // upper bound of nout[] (per-instance row counts)
    int nin;
    int rt;                     // rows per pass: one of 2,4,...,16
    int bitslice;               // 1: gf_bitslice_kernel, tables = coefficient bytes [pass][nin][16]
    size_t count;
};
// Row tile for `rows` output rows: fewest passes of <= 16, evened out.
int gf_row_tile(int rows);
hipError_t launch_gf_apply(const GfApplyArgs &a, hipStream_t s);

// SHA3 of every shard row -> level 0 of each instance's node slab.
hipError_t launch_leaf_hash(const uint8_t *shards, size_t shard_len, size_t shard_stride,
                            size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
                            size_t node_inst_stride, hipStream_t s);
// SHA3 of ragged values: value v at base + offsets[v], lens[v] bytes
// (offsets 8-byte aligned) -> out + 32*v.
hipError_t launch_ragged_hash(const uint8_t *base, const uint64_t *offsets,
                              const uint32_t *lens, size_t nvals, uint8_t *out, hipStream_t s);
// One Merkle level: nodes[cur_off + j] = H(prev[2j] ++ prev[2j+1]) or prev[2j].
hipError_t launch_tree_level(uint8_t *nodes, size_t node_inst_stride, size_t prev_off,
                             size_t prev_size, size_t cur_off, size_t cur_size, size_t count,
                             hipStream_t s);
hipError_t launch_proofs(const uint8_t *nodes, size_t node_inst_stride, size_t n, size_t count,
                         uint8_t *digests, size_t dslots, uint8_t *ndig, hipStream_t s);
struct ValidateArgs {
    const uint8_t *values;
    size_t value_len, value_stride, value_inst_stride, per_inst;
    const uint32_t *indices;
    const uint8_t *digests;
    size_t dslots;
    const uint8_t *ndig;
    const uint8_t *roots;
    size_t root_stride, tree_n, count;
    uint8_t *ok_out;
};
hipError_t launch_validate(const ValidateArgs &a, hipStream_t s);

// Per-instance decode matrix: inv(M[first k present]) applied to
// M[missing rows] -> split-2-bit tables + row index lists.
struct DecodeMatrixArgs {
    int n, k, rt, raw;          // raw: coefficient bytes for the bit-sliced kernel
    const uint8_t *matrix;      // n x k encoding matrix (device)
    const uint8_t *present;     // [count][n]
    size_t count;
    uint4 *tables;              // [count][ceil(m/rt)][k][rt]
    uint32_t *in_idx;           // [count][k]
    uint32_t *out_idx;          // [count][m]
    int *nout;                  // [count]
    int32_t *status;            // [count]
};
hipError_t launch_decode_matrix(const DecodeMatrixArgs &a, hipStream_t s);

// Root compare + BE32 length parse (decode_from_shards tail).
hipError_t launch_decode_check(const int32_t *recon_status, const uint8_t *nodes,
                               size_t node_inst_stride, size_t root_node, const uint8_t *roots,
                               size_t root_stride, const uint8_t *shards, size_t shard_len,
                               size_t shard_stride, size_t inst_stride, size_t data_shards,
                               size_t count, uint32_t *plen_out, int32_t *status_out,
                               hipStream_t s);
hipError_t launch_unframe(const uint8_t *shards, size_t shard_len, size_t shard_stride,
                          size_t inst_stride, size_t data_shards, size_t count,
                          const uint32_t *plen, const int32_t *status, uint8_t *payload_out,
                          size_t payload_stride, hipStream_t s);

// bincode wire format of broadcast::Message (wire.hip).
struct WireEncodeArgs {
    uint32_t variant;           // 0 Value, 1 Echo
    const uint8_t *values;
    size_t value_len, value_stride, value_inst_stride, per_inst;
    const uint32_t *indices;    // [count][per_inst] or nullptr (index = j)
    const uint8_t *digests;     // [count][per_inst][dslots][32]
    size_t dslots;
    const uint8_t *ndig;        // [count][per_inst]
    const uint8_t *roots;
    size_t root_stride, count;
    uint8_t *out;               // [count * per_inst][msg_stride]
    size_t msg_stride;
    uint32_t *msg_len;          // [count * per_inst]
};
hipError_t launch_wire_encode(const WireEncodeArgs &a, hipStream_t s);
struct WireDecodeArgs {
    const uint8_t *msgs;
    size_t msg_stride;
    const uint32_t *msg_len;
    size_t nmsg;
    uint8_t *values;            // [nmsg][value_stride]
    size_t value_stride, value_cap;  // value_cap <= value_stride (multiple of 16)
    uint32_t *value_len, *index;
    uint8_t *digests;           // [nmsg][dslots][32]
    size_t dslots;
    uint8_t *ndig, *roots;      // [nmsg], [nmsg][32]
    uint32_t *variant;
    int32_t *status;
};
hipError_t launch_wire_decode(const WireDecodeArgs &a, hipStream_t s);

hipError_t configure_kernels();

}  // namespace hbrbc
