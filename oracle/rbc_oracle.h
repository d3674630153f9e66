/*
 * rbc_oracle.h -- CPU restatement of hbbft's Reliable-Broadcast data path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (hbbft_amd/libhbrbc.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  Nothing in the product path
 * links or calls it.
 *
 * What it restates (reference = /root/reference, yangl1996/hbbft):
 *   - GF(2^8) arithmetic and the Vandermonde-systematic encoding matrix of
 *     crate reed-solomon-erasure 4.0.x (dependency `reed-solomon-erasure =
 *     "4.0.1"`, Cargo.toml:34; not vendored, restated from its published
 *     algorithm: poly 0x11D, generator 2, M = V * inv(V[0..k])).
 *   - rse `encode` / `reconstruct` semantics, as used by
 *     src/broadcast/broadcast.rs:639-693 (`Coding`).
 *   - SHA3-256 (crate tiny-keccak 2.0.x `Sha3::v256`, Cargo.toml:37), FIPS-202.
 *   - MerkleTree / Proof of src/broadcast/merkle.rs:20-150.
 *   - framing / unframing of src/broadcast/broadcast.rs:170-189, 587-600.
 *
 * Parity pinning: SHA3 / Merkle roots are pinned against Python's
 * hashlib.sha3_256 (an independent FIPS-202 implementation); RS against the
 * upstream crate's published known-answer tests (tests/golden/).
 */
#ifndef RBC_ORACLE_H
#define RBC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rse::Error, in the crate's declaration order (+1 so that 0 = Ok). */
enum {
    ORC_OK = 0,
    ORC_TOO_FEW_SHARDS = 1,
    ORC_TOO_MANY_SHARDS = 2,
    ORC_TOO_FEW_DATA_SHARDS = 3,
    ORC_TOO_MANY_DATA_SHARDS = 4,
    ORC_TOO_FEW_PARITY_SHARDS = 5,
    ORC_TOO_MANY_PARITY_SHARDS = 6,
    ORC_TOO_FEW_BUFFER_SHARDS = 7,
    ORC_TOO_MANY_BUFFER_SHARDS = 8,
    ORC_INCORRECT_SHARD_SIZE = 9,
    ORC_TOO_FEW_SHARDS_PRESENT = 10,
    ORC_EMPTY_SHARD = 11,
    ORC_INVALID_SHARD_FLAGS = 12,
    ORC_INVALID_INDEX = 13,
    ORC_SINGULAR_MATRIX = 64
};

/* ---- GF(2^8), rse galois_8 ------------------------------------------- */
uint8_t orc_gf_mul(uint8_t a, uint8_t b);
uint8_t orc_gf_div(uint8_t a, uint8_t b);
uint8_t orc_gf_exp(uint8_t a, size_t n);
/* c * in[i] for every i (rse galois_8::mul_slice). */
void orc_gf_mul_slice(uint8_t c, const uint8_t *in, uint8_t *out, size_t len);

/* In-place Gauss-Jordan inverse of an n x n row-major matrix. */
int orc_gf_invert(size_t n, uint8_t *m);
/* rse build_matrix(k, total): total x k row-major, top k rows = I_k. */
int orc_build_matrix(size_t k, size_t total, uint8_t *out);

/* ---- Reed-Solomon (rse ReedSolomon<galois_8::Field>) ------------------- */
/* ReedSolomon::new(k, m) validity: ORC_OK or an rse error code. */
int orc_rs_check_new(size_t k, size_t m);
/* rse encode: shards[0..k) data, shards[k..k+m) parity (overwritten). */
int orc_rs_encode(size_t k, size_t m, uint8_t *const *shards,
                  const size_t *lens, size_t n_shards);
/* rse reconstruct: present[i] != 0 marks Some(shard); absent slots must
 * point at a writable buffer of the common length and are filled.  lens[i]
 * is only read for present shards. */
int orc_rs_reconstruct(size_t k, size_t m, uint8_t *const *shards,
                       const size_t *lens, const uint8_t *present,
                       size_t n_shards);
/* hbbft `Coding` wrapper (broadcast.rs:639-693): m == 0 -> Trivial. */
int orc_coding_reconstruct(size_t k, size_t m, uint8_t *const *shards,
                           const size_t *lens, const uint8_t *present,
                           size_t n_shards);

/* ---- SHA3-256 / Merkle (merkle.rs) ------------------------------------ */
void orc_keccak_f1600(uint64_t st[25]);
void orc_sha3_256(const uint8_t *in, size_t len, uint8_t out[32]);
/* Number of nodes of the tree over n leaves, all levels incl. the root. */
size_t orc_merkle_node_count(size_t n);
/* Level offsets (in nodes) of every level; returns the level count. */
size_t orc_merkle_levels(size_t n, size_t *offsets, size_t *sizes);
/* MerkleTree::from_vec: nodes[] = level 0 .. root (32 bytes each). */
void orc_merkle_build(size_t n, const uint8_t *const *values,
                      const size_t *lens, uint8_t *nodes);
/* MerkleTree::proof: returns 0 (None) if index >= n, else 1; fills
 * digests (32 B each) and *ndig. */
int orc_merkle_proof(size_t n, const uint8_t *nodes, size_t index,
                     uint8_t *digests, size_t *ndig);
/* Proof::validate(n). */
int orc_proof_validate(const uint8_t *value, size_t len, size_t index,
                       const uint8_t *digests, size_t ndig,
                       const uint8_t root[32], size_t n);

/* ---- framing (broadcast.rs:170-189) / unframing (587-600) -------------- */
size_t orc_shard_len(size_t payload_len, size_t k);
/* out: (k+m) * S bytes, shard-major. */
void orc_frame(const uint8_t *payload, size_t payload_len, size_t k, size_t m,
               size_t S, uint8_t *out);
/* Concatenated data shards (k*S bytes) -> payload; returns the payload
 * length or -1 when fewer than 4 bytes exist. */
long orc_unframe(const uint8_t *data, size_t k, size_t S, uint8_t *out);

/* ---- whole-path helpers ------------------------------------------------ */
/* send_shards (broadcast.rs:170-225): frame + encode + tree.  shards: N*S,
 * nodes: 32*node_count(N). */
int orc_send_shards(size_t n, size_t f, const uint8_t *payload, size_t plen,
                    uint8_t *shards, uint8_t *nodes);
/* decode_from_shards (broadcast.rs:563-601) on a contiguous N*S buffer with
 * present flags; missing slots are overwritten.  Returns payload length,
 * -1 on reconstruct error, -2 on root mismatch, -3 on missing length. */
long orc_decode_from_shards(size_t n, size_t f, uint8_t *shards, size_t S,
                            const uint8_t *present, const uint8_t root[32],
                            uint8_t *payload_out);

/* ---- synthetic workload (shared with the GPU bench) -------------------- */
uint64_t orc_mix64(uint64_t z);
/* Payload byte stream of instance `inst`: LE bytes of
 * mix64(seed*C1 + inst*C2 + word). */
void orc_gen_payload(uint64_t seed, uint64_t inst, uint8_t *out, size_t len);
/* f erasures per instance (rank selection without replacement). */
void orc_gen_present(uint64_t seed, uint64_t inst, size_t n, size_t n_erase,
                     uint8_t *present);

/* CPU baseline: the whole pipeline (frame, encode, tree, proofs, validate
 * all N, reconstruct f erasures, re-tree, root check, unframe) over `count`
 * instances on `threads` pthreads.  Returns wall seconds; *ok_out = number
 * of instances whose decoded payload matched. */
double orc_bench_pipeline(size_t n, size_t f, size_t plen, size_t count,
                          size_t n_erase, uint64_t seed, int threads,
                          size_t *ok_out);

#ifdef __cplusplus
}
#endif
#endif
