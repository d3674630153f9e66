// launchers.hpp -- host-side launch wrappers for the kernels in kernels.hip.
// Internal to libhbrbc.so (the public surface is include/hbrbc.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/hbrbc.h"

namespace hbrbc {

// Row placement inside one instance of a shard slab: row j sits at byte
//   (j / rb) * bst + (j % rb) * sst
// past the instance base.  rb >= n is the plain shard-major layout (row j at
// j * sst, the reference's contiguous N*S buffer, broadcast.rs:184); rb < n
// groups the rows in blocks of rb, e.g. the destination-major Value/Echo
// slabs of the validator-sharded simulation ([rank][instance][rb][sst]).
struct RowMap {
    uint64_t sst = 0, bst = 0;
    uint32_t rb = 0xFFFFFFFFu;
    __host__ __device__ __forceinline__ uint64_t off(uint32_t j) const {
        if (j < rb) return (uint64_t)j * sst;
        const uint32_t q = j / rb;
        return (uint64_t)q * bst + (uint64_t)(j - q * rb) * sst;
    }
    __host__ __device__ __forceinline__ bool plain() const { return rb == 0xFFFFFFFFu; }
};
inline RowMap plain_rows(size_t sst) {
    RowMap r;
    r.sst = sst;
    return r;
}

// Frame `count` payloads into the data rows of a shard slab (zero padding).
// plens != nullptr: a ragged batch, instance i frames plens[i] bytes (its own
// shard length) and fills its row slots up to row_fill bytes.
hipError_t launch_frame(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                        size_t count, uint8_t *shards, size_t shard_len, const RowMap &rows,
                        size_t inst_stride, size_t data_shards, hipStream_t s,
                        const uint32_t *plens = nullptr, size_t row_fill = 0);

// The last payload_len & 3 payload bytes of a fused frame+encode: data byte
// plus its GF(2^8) contribution to every parity row (matrix = n x k, device).
hipError_t launch_frame_fixup(const uint8_t *payloads, size_t payload_stride, size_t payload_len,
                              uint8_t *shards, size_t shard_len, const RowMap &rows,
                              size_t inst_stride, size_t k, size_t m, const uint8_t *matrix,
                              size_t count, hipStream_t s);

// out_row[r] = sum_j C[r][j] * in_row[in_idx[j]] (bit-sliced GF(2^8)), for
// nout (per pattern or uniform) output rows out_idx[r].  With `pat` the
// coefficients, row lists and counts of instance i are those of slot pat[i]
// (the decode-matrix cache); instances whose slot hash equals `skip_hash`
// are left to a pattern-specialised kernel.
struct GfApplyArgs {
    uint8_t *base;
    size_t inst_stride;
    RowMap rows;
    int n16;                    // 16-byte chunks per row
    const uint8_t *coefs;       // coefficient bytes [slot][pass][nin][16]
    size_t coef_slot_stride;    // bytes (0: shared)
    const uint32_t *in_idx;     // [slot][nin]
    size_t in_idx_stride;       // 0: shared
    const uint32_t *out_idx;    // [slot][max_out]
    size_t out_idx_stride;      // 0: shared
    const int *nout;            // [slot] or nullptr
    int nout_uniform;
    const int *pat;             // [inst] -> slot, or nullptr (slot = inst)
    const uint64_t *slot_hash;  // [slot] (with skip_hash)
    uint64_t skip_hash;         // 0: none
    int hash_slots;             // slots < hash_slots have a slot_hash entry
    int max_rows;               // upper bound of nout[] (per-instance row counts)
    int nin;
    int rt;                     // rows per pass: one of 2,4,...,16
    int mode;                   // 0 branch per coefficient bit, 1 branch hinted, 2 masked
    size_t count;
    // fused unframe (reconstruct): payload bytes of the data rows, payload_S % 4 == 0
    uint8_t *payload = nullptr;
    size_t payload_stride = 0;
    uint32_t payload_S = 0, payload_k = 0;
    const int32_t *rstatus = nullptr;   // reconstruct status per instance (0 = ok)
};
// Row tile for `rows` output rows: fewest passes of <= 16, evened out.
int gf_row_tile(int rows);
hipError_t launch_gf_apply(const GfApplyArgs &a, hipStream_t s);

// SHA3 of every shard row -> level 0 of each instance's node slab.
hipError_t launch_leaf_hash(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                            size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
                            size_t node_inst_stride, hipStream_t s,
                            const uint32_t *slens = nullptr);
// Leaf hashes and all tree levels in one launch (LDS level reduction); only
// for validator counts with merkle_fused_ok(n).
bool merkle_fused_ok(size_t n);
hipError_t launch_merkle_fused(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                               size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
                               size_t node_inst_stride, hipStream_t s,
                               const uint32_t *slens = nullptr);
// SHA3 of only the rows a reconstruct rebuilt (out_idx of each instance's
// decode-matrix slot) -> their level-0 nodes; the other leaves are already
// there (decode with known leaves).
hipError_t launch_leaf_hash_rebuilt(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                                    size_t inst_stride, size_t count, const int *pat,
                                    const uint32_t *out_idx, size_t out_idx_stride,
                                    const int *nout, int max_rows, uint8_t *nodes,
                                    size_t node_inst_stride, uint32_t *counter, uint2 *list,
                                    hipStream_t s);
// SHA3 of ragged values: value v at base + offsets[v], lens[v] bytes
// (offsets 8-byte aligned) -> out + 32*v.
hipError_t launch_ragged_hash(const uint8_t *base, const uint64_t *offsets,
                              const uint32_t *lens, size_t nvals, uint8_t *out, hipStream_t s);
// One Merkle level: nodes[cur_off + j] = H(prev[2j] ++ prev[2j+1]) or prev[2j].
hipError_t launch_tree_level(uint8_t *nodes, size_t node_inst_stride, size_t prev_off,
                             size_t prev_size, size_t cur_off, size_t cur_size, size_t count,
                             hipStream_t s);
// Every level above level 0 in one launch, reduced in LDS (n <= 512).
hipError_t launch_tree_levels(uint8_t *nodes, size_t node_inst_stride, size_t n, size_t count,
                              hipStream_t s);
hipError_t launch_proofs(const uint8_t *nodes, size_t node_inst_stride, size_t n, size_t count,
                         uint8_t *digests, size_t dslots, uint8_t *ndig, hipStream_t s);
// Proof (i, jj): value row r = rows ? rows[jj] : jj of instance i at
// values + i*value_inst_stride + vrows.off(r); claimed index indices[i*per_inst
// + jj] (nullptr: r); digests/ndig of proof slot i*dig_rows + (rows ? r : jj);
// leaf_out (optional): SHA3(value) to leaf_out + i*leaf_inst_stride + r*32.
struct ValidateArgs {
    const uint8_t *values;
    size_t value_len, value_inst_stride, per_inst;
    RowMap vrows;
    const uint32_t *rows;
    const uint32_t *indices;
    const uint8_t *digests;
    size_t dslots, dig_rows;
    const uint8_t *ndig;
    const uint8_t *roots;
    size_t root_stride, tree_n, count;
    uint8_t *ok_out;
    uint8_t *leaf_out;
    size_t leaf_inst_stride;
};
hipError_t launch_validate(const ValidateArgs &a, hipStream_t s);

// Decode-matrix cache (rse keeps an LRU of decode matrices keyed by the
// erasure pattern, behind broadcast.rs:684).  Slot s holds the coefficient
// bytes [pass][k][16], in_idx [k], out_idx [m], nout and status of one
// present-pattern; slots [0, cap) are shared (open addressing on a 64-bit
// hash of the present mask), slot cap + i is instance i's private slot
// (table full or hash collision).
struct PatternCache {
    uint64_t *hash;             // [cap]: 0 empty
    uint32_t *keys;             // [cap + count][8]: present bitmask
    uint8_t *coefs;             // [cap + count][coef_stride]
    size_t coef_stride;
    uint32_t *in_idx;           // [cap + count][k]
    uint32_t *out_idx;          // [cap + count][m]
    int *nout;                  // [cap + count]
    int32_t *status;            // [cap + count]
    uint32_t *fill;             // shared slots claimed so far (device counter)
    int cap;                    // power of two
};
struct DecodeMatrixArgs {
    int n, k, rt;
    const uint8_t *matrix;      // n x k encoding matrix (device)
    const uint8_t *present;     // [count][n]
    size_t count;
    PatternCache cache;
    int *pat;                   // [count] -> slot
    uint8_t *own;               // [count]: this instance computes its slot
    int32_t *status;            // [count] out
    // the pattern a specialised decoder serves (spec_hash 0: none).  Its
    // decoders and the generic kernel route instances by slot hash alone, so
    // a slot with that hash may only ever hold that pattern: an instance whose
    // mask hashes to spec_hash but differs goes to its private slot
    uint64_t spec_hash = 0;
    uint32_t spec_mask[8] = {};
};
// lookup (slot per instance) -> decode matrix of new slots -> per-instance status
hipError_t launch_decode_matrix(const DecodeMatrixArgs &a, hipStream_t s);
// 64-bit hash of a present mask (as the lookup kernel computes it): lets the
// host name the slot of a pattern it specialised a decoder for.
uint64_t pattern_hash(const uint8_t *present, int n);
// the 8 mask words of a present pattern (bit i of word i / 32 = present[i])
void pattern_mask(const uint8_t *present, int n, uint32_t (&w)[8]);

// Root compare + BE32 length parse (decode_from_shards tail).
hipError_t launch_decode_check(const int32_t *recon_status, const uint8_t *nodes,
                               size_t node_inst_stride, size_t root_node, const uint8_t *roots,
                               size_t root_stride, const uint8_t *shards, size_t shard_len,
                               const RowMap &rows, size_t inst_stride, size_t data_shards,
                               size_t count, uint32_t *plen_out, int32_t *status_out,
                               hipStream_t s);
// After a fused-unframe reconstruct: zero payload bytes past the decoded
// length (all of them for a failed instance), as unframe_kernel leaves them.
hipError_t launch_unframe_fixup(const uint8_t *shards, uint32_t S, const RowMap &rows,
                                size_t inst_stride, uint32_t k, size_t count, const uint32_t *plen,
                                const int32_t *status, uint8_t *payload_out, size_t payload_stride,
                                hipStream_t s);
hipError_t launch_unframe(const uint8_t *shards, size_t shard_len, const RowMap &rows,
                          size_t inst_stride, size_t data_shards, size_t count,
                          const uint32_t *plen, const int32_t *status, uint8_t *payload_out,
                          size_t payload_stride, hipStream_t s);

// Overwrite every row with present == 0 (whole slot, 16-byte stores) with
// `fill`: the rows a receiver never got (hbrbc_drop_rows).
hipError_t launch_drop_rows(uint8_t *shards, size_t shard_stride, const RowMap &rows,
                            size_t inst_stride, size_t n, size_t count, const uint8_t *present,
                            uint8_t fill, hipStream_t s);

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

// BLS12-381 pairing checks (pairing.hip)
hipError_t launch_pairing_miller(const uint8_t *g1, size_t g1_stride, const uint8_t *g2,
                                 size_t g2_stride, size_t n, int pair_inputs, uint32_t *ws,
                                 uint8_t *status, hipStream_t s);
hipError_t launch_pairing_miller2(const uint8_t *g1, const uint8_t *g2, size_t count,
                                  uint32_t *ws, uint8_t *status, hipStream_t s);
size_t pairing_prepared_words(size_t points);
hipError_t launch_g2_prepare(const uint8_t *g2, size_t count, uint32_t *prep, uint8_t *pst,
                             hipStream_t s);
hipError_t launch_pairing_miller_prepared(const uint8_t *g1, const uint32_t *prep,
                                          const uint8_t *pst, const uint32_t *ib,
                                          const uint32_t *id, size_t points, size_t count,
                                          uint32_t *ws, uint8_t *status, hipStream_t s);
size_t g1_key_words(size_t points);
hipError_t launch_pairing_miller_prepared_pts(const uint32_t *atab, const uint8_t *ast,
                                              const uint32_t *keys, const uint8_t *kst,
                                              const uint32_t *ic, size_t nkeys,
                                              const uint32_t *prep, const uint8_t *pst,
                                              const uint32_t *ib, const uint32_t *id,
                                              size_t points, size_t count, uint32_t *ws,
                                              uint8_t *status, hipStream_t s);
hipError_t launch_g1_prepare(const uint8_t *g1, size_t count, uint32_t *keys, uint8_t *kst,
                             hipStream_t s);
hipError_t launch_pairing_miller_prepared_keys(const uint8_t *g1_a, const uint32_t *keys,
                                               const uint8_t *kst, const uint32_t *ic,
                                               size_t nkeys, const uint32_t *prep,
                                               const uint8_t *pst, const uint32_t *ib,
                                               const uint32_t *id, size_t points, size_t count,
                                               uint32_t *ws, uint8_t *status, hipStream_t s);
hipError_t launch_pairing_final(const uint32_t *ws, size_t n_miller, size_t n_out, int per_out,
                                const uint8_t *status, uint8_t *gt_out, uint8_t *ok_out,
                                hipStream_t s);

hipError_t configure_kernels();

// Broadcast state machine rounds (sim.hip).  Bytes per node: er u16[n]
// (echo | ready << 8; u8[n], echo | ready << 6, with one root), can_decodes
// u32[roots][W], full Echoes u32[W], counters u16[3][roots], flags u32, + 6 of
// alignment slack for a block, rounded to 8; an instance's block holds its
// hosted nodes' fields as structures of arrays.
// Per-node state block of sim.hip (structure of arrays over an instance's
// nodes).  Two or more roots: er u16[n] (echo entry | ready entry << 8),
// cand u32[C][W], full u32[W], counters u16[3][C], flags u32.  One root (the
// validator-sharded runs): the echo / ready entries of all senders as four
// bitmasks u32x4[W] {EchoHash, full Echo, tampered full Echo, Ready} -- the
// full-Echo mask is their .y -- then cand u32[W], counters u16[3], flags u32.
// Rounded to 16 bytes (the one-root masks are read as 16-byte words).
__host__ __device__ inline size_t sm_er_bytes(size_t n, size_t roots) {
    return roots == 1 ? 16 * ((n + 31) / 32) : 2 * n;
}
__host__ __device__ inline size_t sm_state_bytes(size_t n, size_t roots) {
    const size_t w = (n + 31) / 32;
    const size_t full = roots == 1 ? 0 : 4 * w;
    // (+ 6: the 4-byte alignment pads of cand and flags in a block)
    return (sm_er_bytes(n, roots) + 4 * roots * w + full + 6 * roots + 4 + 6 + 15) & ~(size_t)15;
}
hipError_t launch_sm_round(const hbrbc_sm_args &a, int n, int f, int k, hipStream_t s);

}  // namespace hbrbc
