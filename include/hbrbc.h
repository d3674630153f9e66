/*
 * hbrbc.h -- C ABI of the MI355X Reliable-Broadcast data path (libhbrbc.so).
 *
 * Drop-in boundary for hbbft's `broadcast` data work (reference:
 * yangl1996/hbbft, /root/reference).  The reference has no FFI of its own:
 * its seam is the private enum `Coding` (src/broadcast/broadcast.rs:639-694)
 * and the crate-private module `merkle` (src/broadcast/merkle.rs, exported at
 * src/broadcast/mod.rs:224).  Every entry point below names the reference
 * item it replaces.  INTEGRATION.md shows the Rust `extern "C"` binding that
 * `Coding`/`MerkleTree`/`Proof` delegate to.
 *
 * Two layers:
 *  1. Per-call shims on HOST memory with exactly the reference semantics
 *     (same argument meaning, same rse::Error outcomes).  They stage through
 *     the device and run the same HIP kernels as the batched layer.
 *  2. Batched entry points on DEVICE memory for thousands of independent
 *     broadcast instances per call (the hot path).  All are asynchronous on
 *     the given stream (a hipStream_t; NULL = the HIP null stream) and
 *     never allocate, free or synchronise unless documented.
 *
 * Batched layout ("shard slab"): instance `i`, shard `j`, byte `b` lives at
 *   shards + i*inst_stride + j*shard_stride + b,
 * 0 <= b < shard_len.  Requirements: shard_stride % 16 == 0,
 * shard_stride >= shard_len, inst_stride % 16 == 0,
 * inst_stride >= n_shards*shard_stride, base 16-byte aligned.  Bytes in
 * [shard_len, round_up(shard_len,16)) of a row are padding: the coding
 * kernels read and write them, hashing never covers them.
 *
 * Merkle node slab: instance `i` owns `hbrbc_merkle_node_count(n)` 32-byte
 * nodes at nodes + i*node_inst_stride: level 0 (the n leaf digests), level 1
 * (ceil(n/2)), ..., the root last.  This is `MerkleTree::levels` plus
 * `root_hash` of merkle.rs:12-16 flattened.
 *
 * Errors: every function returns an `int` status.  No exception and no
 * abort crosses this ABI.  Ownership: the caller owns every buffer passed in.
 */
#ifndef HBRBC_H
#define HBRBC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
/* 1..13 mirror reed_solomon_erasure::Error (4.0.x) in declaration order;  */
/* hbbft maps all of them to `Error::InvalidNodeCount` at construction      */
/* (broadcast.rs:101) and to `FaultKind::BroadcastDecoding` on reconstruct  */
/* (broadcast.rs:551-557, 569).                                             */
enum hbrbc_status {
    HBRBC_OK = 0,
    HBRBC_E_TOO_FEW_SHARDS = 1,
    HBRBC_E_TOO_MANY_SHARDS = 2,
    HBRBC_E_TOO_FEW_DATA_SHARDS = 3,
    HBRBC_E_TOO_MANY_DATA_SHARDS = 4,
    HBRBC_E_TOO_FEW_PARITY_SHARDS = 5,
    HBRBC_E_TOO_MANY_PARITY_SHARDS = 6,
    HBRBC_E_TOO_FEW_BUFFER_SHARDS = 7,
    HBRBC_E_TOO_MANY_BUFFER_SHARDS = 8,
    HBRBC_E_INCORRECT_SHARD_SIZE = 9,
    HBRBC_E_TOO_FEW_SHARDS_PRESENT = 10,
    HBRBC_E_EMPTY_SHARD = 11,
    HBRBC_E_INVALID_SHARD_FLAGS = 12,
    HBRBC_E_INVALID_INDEX = 13,
    /* decode outcomes of decode_from_shards (broadcast.rs:563-601) */
    HBRBC_E_SINGULAR_MATRIX = 64,
    HBRBC_E_ROOT_MISMATCH = 65,   /* mtree.root_hash() != root_hash (583-585) */
    HBRBC_E_NO_PAYLOAD_LEN = 66,  /* fewer than 4 data bytes (592-597)        */
    /* bincode deserialisation of a wire message (hbrbc_wire_decode_batch) */
    HBRBC_E_WIRE_TRUNCATED = 70,    /* bincode ErrorKind::Io(UnexpectedEof)     */
    HBRBC_E_WIRE_BAD_VARIANT = 71,  /* enum variant index > 4                   */
    HBRBC_E_WIRE_TOO_LARGE = 72,    /* value or digest list exceeds the batch's slots */
    /* library errors */
    HBRBC_E_INVALID_ARG = 100,
    HBRBC_E_DEVICE = 101,         /* a HIP call failed: see hbrbc_last_error() */
    HBRBC_E_NO_DEVICE = 102
};

typedef struct hbrbc_ctx hbrbc_ctx;

/* Message of the last failing call on this thread (static storage). */
const char *hbrbc_last_error(void);
/* Library version string ("hbrbc <semver> gfx950 src=<hash>"; the hash is
 * hbbft_amd/srchash.py over the sources the library was built from). */
const char *hbrbc_version(void);

/* ---- context = one `Coding` (broadcast.rs:639-655) --------------------- */
/* Replaces `Coding::new(data_shard_num, parity_shard_num)`
 * (broadcast.rs:648-655) -> rse `ReedSolomon::new` + `build_matrix`.
 * parity == 0 selects `Coding::Trivial`.  Errors: TOO_FEW_DATA_SHARDS
 * (data == 0), TOO_MANY_SHARDS (data + parity > 256), NO_DEVICE, DEVICE.
 * `device` < 0 uses the calling thread's current HIP device. */
int hbrbc_coding_new(size_t data_shards, size_t parity_shards, int device, hbrbc_ctx **out);
void hbrbc_coding_free(hbrbc_ctx *ctx);
/* `Coding::data_shard_count` / `parity_shard_count` (broadcast.rs:658-671). */
size_t hbrbc_data_shard_count(const hbrbc_ctx *ctx);
size_t hbrbc_parity_shard_count(const hbrbc_ctx *ctx);
/* The (data+parity) x data encoding matrix, row-major (rse `build_matrix`). */
int hbrbc_encoding_matrix(const hbrbc_ctx *ctx, uint8_t *out);
/* The context's own stream (a hipStream_t). */
void *hbrbc_stream(const hbrbc_ctx *ctx);

/* ---- layer 1: per-call shims, host memory, synchronous ------------------ */
/* `Coding::encode(&mut [&mut [u8]])` (broadcast.rs:674-679, called at 193):
 * shards[0..data) in, shards[data..n) overwritten with parity. */
int hbrbc_encode(hbrbc_ctx *ctx, uint8_t *const *shards, const size_t *lens, size_t n_shards);
/* `Coding::reconstruct_shards(&mut [Option<Box<[u8]>>])` (broadcast.rs:682-693,
 * called at 569).  present[i] != 0 marks Some(shard); absent slots must point
 * at writable buffers of the common shard length and are filled (rse
 * allocates them zeroed, then writes every byte). */
int hbrbc_reconstruct(hbrbc_ctx *ctx, uint8_t *const *shards, const size_t *lens,
                      const uint8_t *present, size_t n_shards);

/* Number of nodes in the flattened tree over n leaves (levels + root). */
size_t hbrbc_merkle_node_count(size_t n);
/* Depth bound: the largest digest count of any proof over n leaves. */
size_t hbrbc_merkle_max_proof_len(size_t n);
/* `MerkleTree::from_vec(Vec<T>)` (merkle.rs:20-33): leaf i = SHA3-256 of
 * values[i][0..lens[i]); nodes_out receives node_count(n)*32 bytes, the
 * root last.  Runs on the default device. */
int hbrbc_merkle_build(const uint8_t *const *values, const size_t *lens, size_t n,
                       uint8_t *nodes_out);
/* `MerkleTree::proof(index)` (merkle.rs:36-53): returns HBRBC_OK and fills
 * digests_out (32*ndig bytes, at most max_proof_len(n) digests), or
 * HBRBC_E_INVALID_INDEX for index >= n (`None`).  Pure data movement. */
int hbrbc_merkle_proof(const uint8_t *nodes, size_t n, size_t index, uint8_t *digests_out,
                       size_t *ndig_out);
/* `Proof::validate(n)` (merkle.rs:83-103): *valid_out = 1 iff the digests
 * form a branch from SHA3(value) at `index` to `root` in a tree of n leaves
 * (too few or too many digests -> 0). */
int hbrbc_proof_validate(const uint8_t *value, size_t len, size_t index, const uint8_t *digests,
                         size_t ndig, const uint8_t root[32], size_t n, int *valid_out);

/* ---- layer 2: batched, device memory, asynchronous on `stream` ---------- */
/* send_shards framing (broadcast.rs:174-189): payload p of instance i (bytes
 * payloads[i*payload_stride .. +payload_len)) -> data shards 0..data-1 of
 * the slab hold BE32(payload_len) ++ payload ++ zeros; padding zeroed.
 * payload_stride % 4 == 0 and >= round_up(payload_len, 4); shard_len must
 * equal hbrbc_shard_len(payload_len, data). */
size_t hbrbc_shard_len(size_t payload_len, size_t data_shards);
int hbrbc_frame_batch(hbrbc_ctx *ctx, const uint8_t *payloads, size_t payload_stride,
                      size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                      size_t shard_stride, size_t inst_stride, void *stream);
/* Coding::encode over `count` instances (broadcast.rs:193): parity rows
 * data..n-1 of every instance written in place. */
int hbrbc_encode_batch(hbrbc_ctx *ctx, uint8_t *shards, size_t shard_len, size_t shard_stride,
                       size_t inst_stride, size_t count, void *stream);
/* send_shards' framing + Coding::encode in one pass (broadcast.rs:174-193):
 * with the specialised encoder loaded and shard_stride == round_up(shard_len,
 * 16) the data rows are framed straight from the payloads inside the encode
 * kernel (one read of the payload, no re-read of the data rows); otherwise
 * hbrbc_frame_batch then hbrbc_encode_batch.  Same arguments and result. */
int hbrbc_frame_encode_batch(hbrbc_ctx *ctx, const uint8_t *payloads, size_t payload_stride,
                             size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                             size_t shard_stride, size_t inst_stride, void *stream);
/* ---- ragged batches: one launch per stage for proposals of any lengths ---- */
/* send_shards' framing + Coding::encode (broadcast.rs:174-193) for `count`
 * proposals of their own lengths, e.g. an epoch where every validator
 * proposes its contribution (honey_badger/epoch_state.rs:223-236,
 * subset/proposal_state.rs:69-113): instance i frames payload_lens[i]
 * (device uint32[count], each <= max_payload_len) bytes into shards of
 * ceil((payload_lens[i] + 4) / data) bytes; every row slot is written up to
 * shard_stride (>= round_up(shard_len(max_payload_len), 16)), zero past the
 * instance's shard, and the parity rows are encoded over that common length. */
int hbrbc_frame_encode_ragged(hbrbc_ctx *ctx, const uint8_t *payloads, size_t payload_stride,
                              const uint32_t *payload_lens, size_t max_payload_len, size_t count,
                              uint8_t *shards, size_t shard_stride, size_t inst_stride,
                              void *stream);
/* MerkleTree::from_vec of a ragged batch: leaf j of instance i hashes
 * shard_lens[i] (device uint32[count]) bytes of its row.  Each entry must be
 * <= shard_stride; the kernels clamp a larger one to shard_stride (they never
 * read past the row slot), so its digests then cover shard_stride bytes. */
int hbrbc_merkle_ragged(hbrbc_ctx *ctx, const uint8_t *shards, const uint32_t *shard_lens,
                        size_t shard_stride, size_t inst_stride, size_t count, uint8_t *nodes,
                        size_t node_inst_stride, void *stream);
/* MerkleTree::from_vec over the n = data+parity shards of every instance
 * (broadcast.rs:204, 580). */
int hbrbc_merkle_batch(hbrbc_ctx *ctx, const uint8_t *shards, size_t shard_len,
                       size_t shard_stride, size_t inst_stride, size_t count, uint8_t *nodes,
                       size_t node_inst_stride, void *stream);
/* MerkleTree::proof for every index of every instance (broadcast.rs:212-222).
 * proof (i, j): digests at digests + ((i*n + j)*max_proof_len(n))*32,
 * count in ndig[i*n + j]. */
int hbrbc_proofs_batch(hbrbc_ctx *ctx, const uint8_t *nodes, size_t node_inst_stride,
                       size_t count, uint8_t *digests, uint8_t *ndig, void *stream);
/* Proof::validate for `count` x `per_inst` proofs (broadcast.rs:254, 291,
 * 604-606).  Proof (i, j): value at values + i*value_inst_stride +
 * j*value_stride (value_len bytes, value_stride % 8 == 0), index
 * indices[i*per_inst + j] (NULL: index = j), digests/ndig laid out as
 * hbrbc_proofs_batch with digest slots = max_proof_len(tree_n), root at
 * roots + i*root_stride.  ok_out[i*per_inst + j] = 1 valid / 0 invalid. */
int hbrbc_validate_batch(hbrbc_ctx *ctx, const uint8_t *values, size_t value_len,
                         size_t value_stride, size_t value_inst_stride, size_t per_inst,
                         const uint32_t *indices, const uint8_t *digests, const uint8_t *ndig,
                         const uint8_t *roots, size_t root_stride, size_t tree_n, size_t count,
                         uint8_t *ok_out, void *stream);
/* Coding::reconstruct_shards over `count` instances (broadcast.rs:569):
 * present[i*n + j] != 0 marks shard j of instance i as received; missing
 * rows are overwritten in place (data from the first `data` present rows via
 * inv(M[valid]), parity from the rebuilt data: bit-identical to rse).
 * status_out[i] = HBRBC_OK or HBRBC_E_TOO_FEW_SHARDS_PRESENT.  Uses the
 * context's workspace (grown on demand, the only allocation on this path;
 * call hbrbc_reserve first to keep it out of a captured region). */
int hbrbc_reconstruct_batch(hbrbc_ctx *ctx, uint8_t *shards, size_t shard_len,
                            size_t shard_stride, size_t inst_stride, const uint8_t *present,
                            size_t count, int32_t *status_out, void *stream);
/* decode_from_shards (broadcast.rs:563-601): reconstruct, re-tree over all n
 * shards, compare with roots[i*root_stride..+32], unframe.  payload bytes of
 * instance i go to payload_out + i*payload_stride (payload_stride a multiple
 * of 4 and >= round_up(data*shard_len - 4, 16); every instance's row must
 * hold that many bytes, bytes past the payload are written 0), their length to payload_len_out[i] and
 * the outcome to status_out[i] (OK, TOO_FEW_SHARDS_PRESENT, ROOT_MISMATCH,
 * NO_PAYLOAD_LEN).  `nodes` (count x node_inst_stride) receives the
 * re-built trees.  Every byte of every instance's payload row up to
 * round_up(data*shard_len - 4, 16) is written: past the payload (all of it
 * for a failed instance) with 0. */
int hbrbc_decode_batch(hbrbc_ctx *ctx, uint8_t *shards, size_t shard_len, size_t shard_stride,
                       size_t inst_stride, const uint8_t *present, size_t count,
                       const uint8_t *roots, size_t root_stride, uint8_t *nodes,
                       size_t node_inst_stride, uint8_t *payload_out, size_t payload_stride,
                       uint32_t *payload_len_out, int32_t *status_out, void *stream);
/* Pre-size the reconstruct workspace (and the decode-matrix cache) for
 * `count` instances; growing it empties the cache. */
int hbrbc_reserve(hbrbc_ctx *ctx, size_t count);

/* ---- blocked row layouts (validator-sharded slabs) ----------------------- */
/* The *_rows variants take the same arguments as their *_batch forms plus a
 * row placement: row j of instance i lives at
 *   base + i*inst_stride + (j / rows_per_block)*block_stride
 *        + (j % rows_per_block)*shard_stride
 * rows_per_block == 0 or >= n is the plain layout above (row j at
 * j*shard_stride).  With rows_per_block < n (<= 255): inst_stride >=
 * rows_per_block*shard_stride and block_stride >= count*inst_stride, e.g.
 * the destination-major Value slab [rank][instance][rows_per_block][stride]
 * whose block d is the contiguous chunk an all-to-all sends to rank d, or the
 * Echo all-gather [validator rank][instance][rows_per_block][stride]. */
int hbrbc_frame_encode_rows(hbrbc_ctx *ctx, const uint8_t *payloads, size_t payload_stride,
                            size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                            size_t shard_stride, size_t rows_per_block, size_t block_stride,
                            size_t inst_stride, void *stream);
int hbrbc_merkle_rows(hbrbc_ctx *ctx, const uint8_t *shards, size_t shard_len, size_t shard_stride,
                      size_t rows_per_block, size_t block_stride, size_t inst_stride, size_t count,
                      uint8_t *nodes, size_t node_inst_stride, void *stream);
/* Proof::validate (merkle.rs:83-103) for `count` x `per_inst` proofs: proof
 * (i, jj) checks value row r = rows[jj] (rows: device uint32[per_inst], the
 * same for every instance; NULL: r = jj) of instance i in the row layout
 * above, with claimed index indices[i*per_inst + jj] (NULL: r), digests and
 * ndig of proof slot i*digest_rows + r (rows given; every r < digest_rows) or
 * i*per_inst + jj, against roots + i*root_stride.  ok_out[i*per_inst + jj].
 * leaf_out (optional): SHA3-256 of the value -- the Merkle leaf -- to
 * leaf_out + i*leaf_inst_stride + r*32, e.g. level 0 of a node slab that a
 * later hbrbc_decode_rows(known_leaves = 1) completes. */
int hbrbc_validate_rows(hbrbc_ctx *ctx, const uint8_t *values, size_t value_len,
                        size_t value_stride, size_t rows_per_block, size_t block_stride,
                        size_t value_inst_stride, size_t per_inst, const uint32_t *rows,
                        const uint32_t *indices, const uint8_t *digests, const uint8_t *ndig,
                        size_t digest_rows, const uint8_t *roots, size_t root_stride,
                        size_t tree_n, size_t count, uint8_t *ok_out, uint8_t *leaf_out,
                        size_t leaf_inst_stride, void *stream);
int hbrbc_reconstruct_rows(hbrbc_ctx *ctx, uint8_t *shards, size_t shard_len, size_t shard_stride,
                           size_t rows_per_block, size_t block_stride, size_t inst_stride,
                           const uint8_t *present, size_t count, int32_t *status_out,
                           void *stream);
/* decode_from_shards in the row layout above.  known_leaves != 0: level 0 of
 * `nodes` already holds SHA3-256 of every PRESENT row of every instance (the
 * receiver hashed them when it validated their Echo proofs, broadcast.rs:291,
 * e.g. through hbrbc_validate_rows' leaf_out); only the rows reconstruct
 * rebuilds are hashed before the levels, root compare and unframe. */
int hbrbc_decode_rows(hbrbc_ctx *ctx, uint8_t *shards, size_t shard_len, size_t shard_stride,
                      size_t rows_per_block, size_t block_stride, size_t inst_stride,
                      const uint8_t *present, size_t count, const uint8_t *roots,
                      size_t root_stride, uint8_t *nodes, size_t node_inst_stride,
                      int known_leaves, uint8_t *payload_out, size_t payload_stride,
                      uint32_t *payload_len_out, int32_t *status_out, void *stream);

/* A receiver holds only the rows it got: every row of instance i with
 * present[i*n + j] == 0 (the shards decode_from_shards gets as None,
 * broadcast.rs:566-571) is overwritten with `fill` over its whole slot
 * (shard_stride bytes), in the plain or blocked layout.  A decode after it
 * rebuilds those rows from the others; the benchmark drops the erased rows
 * of every step this way so no timed decode starts from rows that still
 * hold the right bytes.  n <= 256. */
int hbrbc_drop_rows(hbrbc_ctx *ctx, uint8_t *shards, size_t shard_stride, size_t rows_per_block,
                    size_t block_stride, size_t inst_stride, const uint8_t *present, size_t count,
                    uint8_t fill, void *stream);

/* ---- decode-matrix cache (rse's per-pattern decode-matrix LRU) ----------- */
/* Every reconstruct/decode call looks each instance's present pattern up in a
 * device hash table: the first instance of a new pattern computes inv(M[first
 * k present]) and the recovery rows into a shared slot, every other instance
 * of that pattern -- in this call or a later one -- reuses them.  Shared
 * slots are flushed after about 4 x capacity insertions.  Calls on one
 * context must be stream-ordered (the cache is context state). */
int hbrbc_decode_cache_clear(hbrbc_ctx *ctx);
/* Shared slots claimed since the last flush (synchronises the device). */
int hbrbc_decode_cache_fill(hbrbc_ctx *ctx, uint32_t *patterns_out);
/* Pattern-specialised decoder: compile (hiprtc; or load from the code-object
 * cache) an XOR network for the erasure pattern `present` (host, n bytes)
 * in layouts with this rows_per_block (0: plain).  Later reconstruct/decode
 * calls in that layout run it for every instance of the pattern and the
 * generic kernel for the rest; one pattern per layout (a new call replaces
 * the previous one).  HBRBC_JIT=0 forbids compiling (cache only). */
int hbrbc_decoder_specialise(hbrbc_ctx *ctx, const uint8_t *present, size_t rows_per_block);

/* ---- wire format: bincode of broadcast::Message -------------------------- */
/* `Message::{Value, Echo}(Proof<Vec<u8>>)` (message.rs:13-24, merkle.rs:72-78) as
 * bincode 1.x `serialize` writes it (Cargo.toml:24; examples/simulation.rs:132,
 * examples/network/commst.rs:68): u32 LE variant (0 Value, 1 Echo, 2 Ready,
 * 3 CanDecode, 4 EchoHash), then for Value/Echo u64 LE value length, the value,
 * u64 LE index, u64 LE digest count, 32 bytes per digest, 32 root bytes;
 * for the digest variants 32 bytes.  Message g lives in a slot at
 * out + g*msg_stride (16-aligned, zero-padded past its length). */
size_t hbrbc_wire_proof_message_len(size_t value_len, size_t ndig);
/* Serialise the proofs laid out as for hbrbc_validate_batch (value (i, j) at
 * values + i*value_inst_stride + j*value_stride, 16-aligned rows; index
 * indices[i*per_inst + j] or j; digests/ndig as hbrbc_proofs_batch; root at
 * roots + i*root_stride) as Value (variant 0) or Echo (1) messages, message
 * g = i*per_inst + j; msg_len_out[g] = its length.  msg_stride >=
 * round_up(proof_message_len(value_len, max_proof_len(n)), 16). */
int hbrbc_wire_encode_batch(hbrbc_ctx *ctx, uint32_t variant, const uint8_t *values,
                            size_t value_len, size_t value_stride, size_t value_inst_stride,
                            size_t per_inst, const uint32_t *indices, const uint8_t *digests,
                            const uint8_t *ndig, const uint8_t *roots, size_t root_stride,
                            size_t count, uint8_t *out, size_t msg_stride, uint32_t *msg_len_out,
                            void *stream);
/* Deserialise `nmsg` messages of msg_len[g] bytes each (bincode `deserialize`;
 * trailing bytes ignored): variant_out[g]; for Value/Echo the value into
 * values + g*value_stride (zero-padded; longer than value_stride -> WIRE_TOO_LARGE),
 * value_len_out, index_out (saturated at 2^32-1), digests + g*max_proof_len(n)*32
 * and ndig_out (more than max_proof_len(n) -> WIRE_TOO_LARGE, since no tree over
 * n leaves has that many levels), roots + g*32; for Ready/CanDecode/EchoHash the
 * digest into roots.  status_out[g] = OK or a WIRE_* code. */
int hbrbc_wire_decode_batch(hbrbc_ctx *ctx, const uint8_t *msgs, size_t msg_stride,
                            const uint32_t *msg_len, size_t nmsg, uint8_t *values,
                            size_t value_stride, uint32_t *value_len_out, uint32_t *index_out,
                            uint8_t *digests, uint8_t *ndig_out, uint8_t *roots,
                            uint32_t *variant_out, int32_t *status_out, void *stream);

/* ---- specialised encoder ------------------------------------------------ */
/* Coding::encode runs either the generic bit-sliced GF kernel or, when a code
 * object for this (data, parity) matrix is cached under <lib dir>/jit (or
 * $HBRBC_JIT_DIR), a kernel generated for the matrix: a fixed XOR network on
 * bit planes (hbbft_amd/csrc/jit.hip), bit-identical output.  Returns
 * "specialised", "bitslice", "trivial" or "jit-failed". */
const char *hbrbc_encode_kernel(const hbrbc_ctx *ctx);
/* Generate and compile (hiprtc, gfx950, no device needed) the specialised
 * encoder for rse build_matrix(data, data + parity) into `dir` (NULL: the
 * default directory).  With HBRBC_JIT=1 a context compiles a missing one
 * itself; HBRBC_JIT=0 disables the specialised path. */
int hbrbc_jit_build_encode(size_t data_shards, size_t parity_shards, const char *dir);
/* Large matrices are split into parity-row groups, one code object each (a
 * program stays near 4096 coefficients, so hiprtc time stays near a minute);
 * these build them one at a time, e.g. in parallel processes. */
size_t hbrbc_jit_encode_groups(size_t data_shards, size_t parity_shards);
int hbrbc_jit_build_encode_group(size_t data_shards, size_t parity_shards, size_t group,
                                 const char *dir);
/* Cache file name (no directory) of group `group`'s code object under the
 * current generator settings; 0 and a NUL-terminated name in buf, or an error. */
int hbrbc_jit_file_name(size_t data_shards, size_t parity_shards, size_t group, char *buf,
                        size_t buf_len);
/* The same for the encoder of a blocked row layout (rows_per_block < n). */
int hbrbc_jit_build_encode_rows(size_t data_shards, size_t parity_shards, size_t group,
                                size_t rows_per_block, const char *dir);
int hbrbc_jit_encode_file_name(size_t data_shards, size_t parity_shards, size_t group,
                               size_t rows_per_block, char *buf, size_t buf_len);
/* Pattern-specialised decoders (hbrbc_decoder_specialise) built ahead of use:
 * groups of the pattern's program, one group's code object, its file name. */
size_t hbrbc_jit_decode_groups(size_t data_shards, size_t parity_shards, const uint8_t *present);
int hbrbc_jit_build_decode(size_t data_shards, size_t parity_shards, const uint8_t *present,
                           size_t rows_per_block, size_t group, const char *dir);
/* The same for the decoder's fused-unframe variant (fused_unframe != 0: the
 * programs also write the payload bytes of the data rows; a decode that
 * unframes in the reconstruct loads them on first use). */
int hbrbc_jit_build_decode_variant(size_t data_shards, size_t parity_shards,
                                   const uint8_t *present, size_t rows_per_block, size_t group,
                                   int fused_unframe, const char *dir);
int hbrbc_jit_decode_variant_file_name(size_t data_shards, size_t parity_shards,
                                       const uint8_t *present, size_t rows_per_block,
                                       size_t group, int fused_unframe, char *buf,
                                       size_t buf_len);
int hbrbc_jit_decode_file_name(size_t data_shards, size_t parity_shards, const uint8_t *present,
                               size_t rows_per_block, size_t group, char *buf, size_t buf_len);

/* ---- measurement hooks (bench.py) --------------------------------------- */
/* Stage ids for the per-stage device timers. */
enum hbrbc_stage {
    HBRBC_STAGE_FRAME = 0,
    HBRBC_STAGE_ENCODE = 1,
    HBRBC_STAGE_LEAF_HASH = 2,
    HBRBC_STAGE_TREE_LEVELS = 3,
    HBRBC_STAGE_PROOFS = 4,
    HBRBC_STAGE_VALIDATE = 5,
    HBRBC_STAGE_DECODE_MATRIX = 6,
    HBRBC_STAGE_RECONSTRUCT = 7,
    HBRBC_STAGE_UNFRAME = 8,
    HBRBC_STAGE_COUNT = 9
};
/* When enabled, every stage's kernels are bracketed by hipEvents recorded on
 * the stream they run on.  hbrbc_profile_read synchronises those events and
 * returns total milliseconds and launch count per stage since the last
 * reset. */
int hbrbc_profile_enable(hbrbc_ctx *ctx, int enable);
int hbrbc_profile_reset(hbrbc_ctx *ctx);
int hbrbc_profile_read(hbrbc_ctx *ctx, double *ms_out, uint64_t *launches_out);
const char *hbrbc_stage_name(int stage);

/* 1 if hbrbc_decode_batch / _rows on this context (row block rows_per_block,
 * 0 = plain layout) write the payload from the reconstruct kernel (fused
 * unframe, in the generic and the pattern-specialised decoders: shard_len
 * % 4 == 0, payload_stride % 16 == 0, HBRBC_UNFRAME_FUSED != 0), else 0.
 * Outputs are identical either way; this only tells where the bytes move. */
int hbrbc_unframe_fused(const hbrbc_ctx *ctx, size_t shard_len, size_t payload_stride,
                        size_t rows_per_block);

/* ---- threshold-decrypt share verification --------------- */
/* BLS12-381 pairings of the `pairing` crate as `threshold_crypto` (rev 624eeee,
 * Cargo.toml:36) uses them behind hbbft's ThresholdDecrypt:
 *   `Ciphertext::verify`                  (threshold_decrypt.rs:142)
 *       e(G1::one(), W) == e(U, hash_g1_g2(U, V))
 *   `PublicKeyShare::verify_decryption_share` (threshold_decrypt.rs:220-228)
 *       e(share, hash_g1_g2(U, V)) == e(pk_i, W)
 * Points use the crate's uncompressed encodings: G1 = 96 bytes x || y, G2 =
 * 192 bytes x.c1 || x.c0 || y.c1 || y.c0, big-endian, infinity = flag 0x40 in
 * byte 0 with every other bit zero.  Non-canonical coordinates (>= p), set
 * compression/sort flags, points off the curve and points outside the
 * order-r subgroup are rejected per item, as the crate's deserialisation
 * (`into_affine`) rejects them.
 * hash_g1_g2 (SHA3 + ChaCha-seeded G2 sampling, once per ciphertext) stays
 * with the caller, which passes the G2 point. */
#define HBRBC_G1_BYTES 96
#define HBRBC_G2_BYTES 192
#define HBRBC_GT_BYTES 576
/* Device workspace bytes for `pairings` Miller loops. */
size_t hbrbc_pairing_workspace_size(size_t pairings);
/* `PEngine::pairing(g1[i], g2[i])` for i < count: gt_out + 576 i receives the
 * GT value (the crate's Fq12 after its final exponentiation, tower order
 * c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1, each coefficient 48 bytes
 * big-endian); status_out[i] = 0 ok, 2 invalid point (the value is then 1).
 * An infinity on either side gives 1.  Device memory, async on `stream`. */
int hbrbc_pairing_batch(const uint8_t *g1, const uint8_t *g2, size_t count, uint8_t *gt_out,
                        uint8_t *status_out, void *workspace, void *stream);
/* count checks e(a_i, b_i) == e(c_i, d_i): g1 holds a_0, c_0, a_1, c_1, ...
 * (2 count points), g2 holds b_0, d_0, b_1, d_1, ....  ok_out[i] = 1 if
 * equal, 0 if not, 2 if any of the four points is invalid.  For
 * verify_decryption_share: a = share, b = hash, c = pk_i, d = W; for
 * Ciphertext::verify: a = G1::one(), b = W, c = U, d = hash.
 * workspace >= hbrbc_pairing_workspace_size(2 count).  Device memory, async. */
int hbrbc_pairing_check_batch(const uint8_t *g1, const uint8_t *g2, size_t count,
                              uint8_t *ok_out, void *workspace, void *stream);
/* Prepared G2 points (the crate's G2Prepared): the 68 Miller-loop lines of
 * each point, computed once and shared by every check against it (hbbft:
 * the N decryption shares of a ciphertext are all checked against its H and
 * W).  `prepared` >= hbrbc_g2_prepared_size(count) bytes of device memory;
 * an invalid point is marked there and fails every check that uses it. */
size_t hbrbc_g2_prepared_size(size_t points);
int hbrbc_g2_prepare(const uint8_t *g2, size_t count, void *prepared, void *stream);
/* count checks e(a_i, P[idx_b[i]]) == e(c_i, P[idx_d[i]]) against prepared
 * points P (`points` of them in `prepared`): g1 holds a_0, c_0, a_1, c_1, ...;
 * ok_out as hbrbc_pairing_check_batch (an index >= points makes that check 2).
 * Checks that share prepared points
 * should be adjacent (a wave then reads each line once).  workspace >=
 * hbrbc_pairing_workspace_size(count).  Device memory, async on `stream`. */
int hbrbc_pairing_check_prepared(const uint8_t *g1, const void *prepared, size_t points,
                                 const uint32_t *idx_b, const uint32_t *idx_d, size_t count,
                                 uint8_t *ok_out, void *workspace, void *stream);
/* Prepared G1 keys: hbbft checks each decryption share against its sender's
 * public key share pk_i, and the validator set's key shares are the same for
 * every ciphertext; `threshold_crypto` holds them as curve points, decoded and
 * checked once.  hbrbc_g1_prepare decodes and checks `count` G1 points once
 * (as any G1 input: canonical, on the curve, order r) into `prepared` >=
 * hbrbc_g1_prepared_size(count) bytes of device memory; an invalid point is
 * marked there and fails every check that uses it.  Device memory, async. */
size_t hbrbc_g1_prepared_size(size_t points);
int hbrbc_g1_prepare(const uint8_t *g1, size_t count, void *prepared, void *stream);
/* count checks e(a_i, P[idx_b[i]]) == e(K[idx_c[i]], P[idx_d[i]]) with K the
 * `key_points` prepared G1 keys and P the `points` prepared G2 points: g1_a
 * holds a_0, a_1, ... (count points); ok_out as hbrbc_pairing_check_batch
 * (an index past either table makes that check 2).  For
 * verify_decryption_share: a = share, K = the pk_i table, b = hash, d = W.
 * workspace >= hbrbc_pairing_workspace_size(count).  Device memory, async. */
int hbrbc_pairing_check_prepared_keys(const uint8_t *g1_a, const void *keys, size_t key_points,
                                      const uint32_t *idx_c, const void *prepared, size_t points,
                                      const uint32_t *idx_b, const uint32_t *idx_d, size_t count,
                                      uint8_t *ok_out, void *workspace, void *stream);
/* The same checks with the shares decoded beforehand too: `a_prepared` is
 * hbrbc_g1_prepare of the count shares (a_i = entry i), so their decoding
 * and order-r checks run as a launch of their own (e.g. beside
 * hbrbc_g2_prepare on another stream) and the Miller loops only load them.
 * Outcomes as hbrbc_pairing_check_prepared_keys. */
int hbrbc_pairing_check_prepared_pts(const void *a_prepared, const void *keys, size_t key_points,
                                     const uint32_t *idx_c, const void *prepared, size_t points,
                                     const uint32_t *idx_b, const uint32_t *idx_d, size_t count,
                                     uint8_t *ok_out, void *workspace, void *stream);
/* Per-call shim on host memory (one check, synchronous, current device):
 * *result = 1 if e(a, b) == e(c, d), 0 if not; HBRBC_E_INVALID_ARG for an
 * invalid point. */
int hbrbc_pairing_check(const uint8_t a[96], const uint8_t b[192], const uint8_t c[96],
                        const uint8_t d[192], int *result);

/* ---- the Broadcast state machine, batched --------------- */
/* Many instances x nodes of `Broadcast` (broadcast.rs:228-558) in synchronous
 * rounds: what a node emits in round t is delivered in round t + 1, each node
 * handling its inbox in (sender index, emission order).  Round 0 is the
 * proposers' broadcast().  A message is a record of 1 + W uint32 words
 * (W = ceil(n / 32)): word 0 = kind | root << 8 | index << 16 | tampered << 24
 * (kind: 0 Value, 1 Echo, 2 Ready, 3 CanDecode, 4 EchoHash, 5 the
 * ProposeAdversary's injected broadcasts), words 1..W = recipient bits.
 * Proofs travel by reference (root c = codeword slot of the instance, index
 * j, tampered copy or not): proof_ok holds Proof::validate of each (the
 * batched validate kernel), decode_ok decode_from_shards of each root (the
 * batched decode).  Nodes [node_lo, node_lo + nodes) are hosted here; the
 * previous round's records of every sender s sit in `in` at block s / R, row
 * s % R ([G][count][R][max_out][1 + W]); this round's go to `out`
 * ([count][nodes][max_out][1 + W]); out_count bit 31 flags an overflow.
 * Fault records: blamed node << 8 | FaultKind (error.rs:28-50 order). */
#define HBRBC_SM_NONE 0xFF
enum hbrbc_sm_role {            /* per instance and node */
    HBRBC_SM_HONEST = 0,
    HBRBC_SM_SILENT = 1,        /* emits nothing when handling a message (ProposeAdversary drop) */
    HBRBC_SM_CORRUPT_ECHO = 2,  /* its Echoes carry the tampered copy of its proof */
    HBRBC_SM_WITHHOLD_ECHO = 3  /* sends no Echo at all */
};
typedef struct hbrbc_sm_args {
    size_t count;                 /* instances */
    uint32_t node_lo, nodes;      /* hosted nodes */
    uint32_t rows_per_rank;       /* R of the `in` layout (n for one rank) */
    uint32_t roots;               /* codeword slots per instance, <= 8 */
    uint32_t max_out;             /* records per node per round */
    uint32_t max_faults;          /* fault records kept per node */
    int32_t round;
    const uint8_t *proposer;      /* [count] */
    const uint8_t *role;          /* [count][n] */
    const uint8_t *value_root;    /* [count][n]: root of the proposer's Value to node j, or NONE */
    const uint8_t *value_tamper;  /* [count][n]: that Value carries the tampered copy */
    const uint8_t *proof_ok;      /* [count][roots][2][n] */
    const uint8_t *decode_ok;     /* [count][roots] */
    const uint8_t *fake_from;     /* [count]: dispatcher of the injected broadcasts, or NONE */
    const uint8_t *fake_root;     /* [count]: their codeword slot */
    const uint32_t *fake_list;    /* [count][W]: the faulty nodes whose broadcasts are injected */
    const uint32_t *in;
    const uint32_t *in_count;     /* [G][count][R] */
    uint32_t *out;
    uint32_t *out_count;          /* [count][nodes] */
    uint8_t *state;               /* [count][nodes][hbrbc_sm_state_bytes], zeroed before round 0 */
    uint8_t *output_root;         /* [count][nodes]: decided root, NONE before */
    uint16_t *faults;             /* [count][nodes][max_faults] */
    uint32_t *fault_count;        /* [count][nodes] (may exceed max_faults) */
    uint32_t *emitted;            /* [2]: [0] += records emitted this round, [1] |= 1 if a
                                     node emitted more than max_out (out_count bit 31) */
    const uint32_t *active;       /* NULL, or: the round returns at once when *active == 0
                                     (every sender's previous round emitted nothing: the
                                     network is quiescent), so a host can enqueue several
                                     rounds and read the emitted counts back once */
    uint32_t flags;               /* HBRBC_SM_NO_FAKE: no instance has a fake_from node, so no
                                     inbox holds a Fake record and those of rounds >= 2 hold only
                                     Echo, EchoHash, Ready and CanDecode records: round 1 runs a
                                     kernel without the Fake handler, rounds >= 2 one without the
                                     Value handler too (a record of a kind left out, or a
                                     fake_from node, sets emitted[1] bit 1, the caller's error) */
} hbrbc_sm_args;
#define HBRBC_SM_NO_FAKE 1u
size_t hbrbc_sm_state_bytes(size_t n, size_t roots);
/* One round for the hosted nodes of every instance (ctx gives n, f, k). */
int hbrbc_sm_round(hbrbc_ctx *ctx, const hbrbc_sm_args *args, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HBRBC_H */
