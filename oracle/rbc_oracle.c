/*
 * rbc_oracle.c -- CPU restatement of hbbft's Reliable-Broadcast data path.
 *
 * TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline); see
 * rbc_oracle.h.  The product path never links this file.
 *
 * Every function cites the reference lines it restates.  The arithmetic of
 * `reed-solomon-erasure` 4.0.x and `tiny-keccak` 2.0.x is not vendored under
 * /root/reference; it is restated from the crates' published algorithms and
 * anchored on their known-answer tests (tests/golden/rs_kat.json) and on
 * hashlib.sha3_256 (tests/golden/merkle_*.json).
 */
#include "rbc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ===================================================================== */
/* GF(2^8): rse galois_8, generating polynomial 29 (x^8+x^4+x^3+x^2+1),  */
/* generator 2.  mul(a,b) = EXP[LOG a + LOG b], 0 if either is 0.         */
/* ===================================================================== */
static uint8_t g_log[256];
static uint8_t g_exp[510];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_init_tables(void) {
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_exp[i + 255] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    g_log[0] = 0;
}
static inline void gf_init(void) { pthread_once(&g_once, gf_init_tables); }

uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

uint8_t orc_gf_div(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0) return 0;
    if (b == 0) abort(); /* rse panics on division by zero */
    int l = (int)g_log[a] - (int)g_log[b];
    if (l < 0) l += 255;
    return g_exp[l];
}

uint8_t orc_gf_exp(uint8_t a, size_t n) {
    gf_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    size_t l = ((size_t)g_log[a] * n) % 255;
    return g_exp[l];
}

void orc_gf_mul_slice(uint8_t c, const uint8_t *in, uint8_t *out, size_t len) {
    gf_init();
    uint8_t tab[256];
    for (int x = 0; x < 256; x++) tab[x] = orc_gf_mul(c, (uint8_t)x);
    for (size_t i = 0; i < len; i++) out[i] = tab[in[i]];
}

/* rse Matrix::invert -> gaussian_elim on [M | I]. */
int orc_gf_invert(size_t n, uint8_t *m) {
    gf_init();
    size_t w = 2 * n;
    uint8_t *a = (uint8_t *)calloc(n * w, 1);
    for (size_t r = 0; r < n; r++) {
        memcpy(a + r * w, m + r * n, n);
        a[r * w + n + r] = 1;
    }
    for (size_t r = 0; r < n; r++) {
        if (a[r * w + r] == 0) {
            for (size_t rb = r + 1; rb < n; rb++) {
                if (a[rb * w + r] != 0) {
                    for (size_t c = 0; c < w; c++) {
                        uint8_t t = a[r * w + c];
                        a[r * w + c] = a[rb * w + c];
                        a[rb * w + c] = t;
                    }
                    break;
                }
            }
        }
        if (a[r * w + r] == 0) {
            free(a);
            return ORC_SINGULAR_MATRIX;
        }
        if (a[r * w + r] != 1) {
            uint8_t s = orc_gf_div(1, a[r * w + r]);
            for (size_t c = 0; c < w; c++) a[r * w + c] = orc_gf_mul(s, a[r * w + c]);
        }
        for (size_t rb = r + 1; rb < n; rb++) {
            uint8_t s = a[rb * w + r];
            if (s)
                for (size_t c = 0; c < w; c++) a[rb * w + c] ^= orc_gf_mul(s, a[r * w + c]);
        }
    }
    for (size_t d = 0; d < n; d++) {
        for (size_t ra = 0; ra < d; ra++) {
            uint8_t s = a[ra * w + d];
            if (s)
                for (size_t c = 0; c < w; c++) a[ra * w + c] ^= orc_gf_mul(s, a[d * w + c]);
        }
    }
    for (size_t r = 0; r < n; r++) memcpy(m + r * n, a + r * w + n, n);
    free(a);
    return ORC_OK;
}

/* rse build_matrix(k, total): vandermonde(total, k) * inv(top k x k),
 * vandermonde[r][c] = exp(r, c). */
int orc_build_matrix(size_t k, size_t total, uint8_t *out) {
    uint8_t *v = (uint8_t *)malloc(total * k);
    uint8_t *top = (uint8_t *)malloc(k * k);
    for (size_t r = 0; r < total; r++)
        for (size_t c = 0; c < k; c++) v[r * k + c] = orc_gf_exp((uint8_t)r, c);
    memcpy(top, v, k * k);
    int st = orc_gf_invert(k, top);
    if (st == ORC_OK) {
        for (size_t r = 0; r < total; r++)
            for (size_t c = 0; c < k; c++) {
                uint8_t acc = 0;
                for (size_t j = 0; j < k; j++) acc ^= orc_gf_mul(v[r * k + j], top[j * k + c]);
                out[r * k + c] = acc;
            }
    }
    free(v);
    free(top);
    return st;
}

/* ===================================================================== */
/* Reed-Solomon (rse ReedSolomon::{new, encode, reconstruct})             */
/* ===================================================================== */
int orc_rs_check_new(size_t k, size_t m) {
    if (k == 0) return ORC_TOO_FEW_DATA_SHARDS;
    if (m == 0) return ORC_TOO_FEW_PARITY_SHARDS;
    if (k + m > 256) return ORC_TOO_MANY_SHARDS;
    return ORC_OK;
}

/* out[r] ^= / = sum_j rows[r][j] * in[j] over len bytes (rse code_some_slices). */
static void code_some_slices(size_t nrows, const uint8_t *rows, size_t row_stride,
                             size_t nin, const uint8_t *const *in, uint8_t *const *out,
                             size_t len) {
    gf_init();
    uint8_t tab[256];
    for (size_t r = 0; r < nrows; r++) {
        memset(out[r], 0, len);
        for (size_t j = 0; j < nin; j++) {
            uint8_t c = rows[r * row_stride + j];
            if (c == 0) continue;
            for (int x = 0; x < 256; x++) tab[x] = x ? g_exp[g_log[c] + g_log[x]] : 0;
            const uint8_t *src = in[j];
            uint8_t *dst = out[r];
            for (size_t b = 0; b < len; b++) dst[b] ^= tab[src[b]];
        }
    }
}

/* Per-thread cache of the last build_matrix(k, k+m). */
static __thread size_t t_mk = 0, t_mm = 0;
static __thread uint8_t *t_matrix = NULL;
static const uint8_t *matrix_for(size_t k, size_t m) {
    if (t_matrix && t_mk == k && t_mm == m) return t_matrix;
    free(t_matrix);
    t_matrix = (uint8_t *)malloc((k + m) * k);
    orc_build_matrix(k, k + m, t_matrix);
    t_mk = k;
    t_mm = m;
    return t_matrix;
}

int orc_rs_encode(size_t k, size_t m, uint8_t *const *shards, const size_t *lens,
                  size_t n_shards) {
    int st = orc_rs_check_new(k, m);
    if (st) return st;
    /* check_piece_count!(all) */
    if (n_shards < k + m) return ORC_TOO_FEW_SHARDS;
    if (n_shards > k + m) return ORC_TOO_MANY_SHARDS;
    /* check_slices!(multi) */
    size_t len = lens[0];
    if (len == 0) return ORC_EMPTY_SHARD;
    for (size_t i = 0; i < n_shards; i++)
        if (lens[i] != len) return ORC_INCORRECT_SHARD_SIZE;
    const uint8_t *mat = matrix_for(k, m);
    code_some_slices(m, mat + k * k, k, k, (const uint8_t *const *)shards, shards + k, len);
    return ORC_OK;
}

/* rse reconstruct_internal(data_only = false). */
int orc_rs_reconstruct(size_t k, size_t m, uint8_t *const *shards, const size_t *lens,
                       const uint8_t *present, size_t n_shards) {
    int st = orc_rs_check_new(k, m);
    if (st) return st;
    size_t total = k + m;
    if (n_shards < total) return ORC_TOO_FEW_SHARDS;
    if (n_shards > total) return ORC_TOO_MANY_SHARDS;
    size_t number_present = 0, shard_len = 0;
    int have_len = 0;
    for (size_t i = 0; i < total; i++) {
        if (!present[i]) continue;
        if (lens[i] == 0) return ORC_EMPTY_SHARD;
        number_present++;
        if (have_len && lens[i] != shard_len) return ORC_INCORRECT_SHARD_SIZE;
        shard_len = lens[i];
        have_len = 1;
    }
    if (number_present == total) return ORC_OK;
    if (number_present < k) return ORC_TOO_FEW_SHARDS_PRESENT;

    const uint8_t *mat = matrix_for(k, m);
    size_t valid[256], invalid[256], nvalid = 0, ninvalid = 0;
    for (size_t i = 0; i < total; i++) {
        if (present[i]) {
            if (nvalid < k) valid[nvalid++] = i;
        } else {
            invalid[ninvalid++] = i;
        }
    }
    /* data decode matrix = inv(M[valid rows]) */
    uint8_t *dm = (uint8_t *)malloc(k * k);
    for (size_t r = 0; r < k; r++) memcpy(dm + r * k, mat + valid[r] * k, k);
    st = orc_gf_invert(k, dm);
    if (st) {
        free(dm);
        return st;
    }
    const uint8_t *sub[256];
    for (size_t j = 0; j < k; j++) sub[j] = shards[valid[j]];
    /* missing data shards = dm[d] x sub */
    uint8_t *rows = (uint8_t *)calloc(total * k, 1);
    uint8_t *outs[256];
    size_t nout = 0;
    for (size_t t = 0; t < ninvalid && invalid[t] < k; t++) {
        memcpy(rows + nout * k, dm + invalid[t] * k, k);
        outs[nout++] = shards[invalid[t]];
    }
    code_some_slices(nout, rows, k, k, sub, outs, shard_len);
    /* missing parity shards = parity rows x all data shards */
    const uint8_t *data[256];
    for (size_t j = 0; j < k; j++) data[j] = shards[j];
    nout = 0;
    for (size_t t = 0; t < ninvalid; t++) {
        if (invalid[t] < k) continue;
        memcpy(rows + nout * k, mat + invalid[t] * k, k);
        outs[nout++] = shards[invalid[t]];
    }
    code_some_slices(nout, rows, k, k, data, outs, shard_len);
    free(rows);
    free(dm);
    return ORC_OK;
}

/* broadcast.rs:682-693 */
int orc_coding_reconstruct(size_t k, size_t m, uint8_t *const *shards, const size_t *lens,
                           const uint8_t *present, size_t n_shards) {
    if (m == 0) {
        for (size_t i = 0; i < n_shards; i++)
            if (!present[i]) return ORC_TOO_FEW_SHARDS_PRESENT;
        return ORC_OK;
    }
    return orc_rs_reconstruct(k, m, shards, lens, present, n_shards);
}

/* ===================================================================== */
/* SHA3-256 (tiny-keccak Sha3::v256 == FIPS-202), merkle.rs:143-150       */
/* ===================================================================== */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                             25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

static inline uint64_t rol(uint64_t x, int r) { return r ? (x << r) | (x >> (64 - r)) : x; }

void orc_keccak_f1600(uint64_t a[25]) {
    for (int round = 0; round < 24; round++) {
        uint64_t c[5], d[5], b[25];
        for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ rol(c[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
        /* rho + pi: b[y, 2x+3y] = rol(a[x,y], r[x,y]) with lane index x + 5y */
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) {
                int X = y, Y = (2 * x + 3 * y) % 5;
                b[X + 5 * Y] = rol(a[x + 5 * y], KROT[x + 5 * y]);
            }
        for (int y = 0; y < 5; y++)
            for (int x = 0; x < 5; x++)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= KRC[round];
    }
}

void orc_sha3_256(const uint8_t *in, size_t len, uint8_t out[32]) {
    uint64_t st[25];
    memset(st, 0, sizeof st);
    const size_t rate = 136;
    uint8_t blk[136];
    while (len >= rate) {
        for (int i = 0; i < 17; i++) {
            uint64_t w;
            memcpy(&w, in + 8 * i, 8); /* little-endian lanes */
            st[i] ^= w;
        }
        orc_keccak_f1600(st);
        in += rate;
        len -= rate;
    }
    memset(blk, 0, rate);
    memcpy(blk, in, len);
    blk[len] ^= 0x06;
    blk[rate - 1] ^= 0x80;
    for (int i = 0; i < 17; i++) {
        uint64_t w;
        memcpy(&w, blk + 8 * i, 8);
        st[i] ^= w;
    }
    orc_keccak_f1600(st);
    memcpy(out, st, 32);
}

/* ===================================================================== */
/* Merkle tree (merkle.rs:20-103).  Node layout: level 0 (n leaves),      */
/* level 1 (ceil(n/2)), ..., the root level (1 node), concatenated.       */
/* ===================================================================== */
size_t orc_merkle_levels(size_t n, size_t *offsets, size_t *sizes) {
    size_t lv = 0, off = 0, sz = n;
    for (;;) {
        if (offsets) offsets[lv] = off;
        if (sizes) sizes[lv] = sz;
        lv++;
        off += sz;
        if (sz <= 1) break;
        sz = (sz + 1) / 2;
    }
    return lv;
}

size_t orc_merkle_node_count(size_t n) {
    size_t off[64], sz[64];
    size_t lv = orc_merkle_levels(n, off, sz);
    return off[lv - 1] + sz[lv - 1];
}

/* hash_pair merkle.rs:137-140 */
static void hash_pair(const uint8_t *l, const uint8_t *r, uint8_t out[32]) {
    uint8_t buf[64];
    memcpy(buf, l, 32);
    memcpy(buf + 32, r, 32);
    orc_sha3_256(buf, 64, out);
}

/* MerkleTree::from_vec merkle.rs:20-33; hash_chunk 128-134 */
void orc_merkle_build(size_t n, const uint8_t *const *values, const size_t *lens,
                      uint8_t *nodes) {
    size_t off[64], sz[64];
    size_t lv = orc_merkle_levels(n, off, sz);
    for (size_t i = 0; i < n; i++) orc_sha3_256(values[i], lens[i], nodes + 32 * i);
    for (size_t l = 1; l < lv; l++) {
        const uint8_t *prev = nodes + 32 * off[l - 1];
        uint8_t *cur = nodes + 32 * off[l];
        for (size_t j = 0; j < sz[l]; j++) {
            if (2 * j + 1 < sz[l - 1])
                hash_pair(prev + 64 * j, prev + 64 * j + 32, cur + 32 * j);
            else
                memcpy(cur + 32 * j, prev + 64 * j, 32); /* odd node promoted */
        }
    }
}

/* MerkleTree::proof merkle.rs:36-53 (levels = all levels but the root) */
int orc_merkle_proof(size_t n, const uint8_t *nodes, size_t index, uint8_t *digests,
                     size_t *ndig) {
    if (index >= n) return 0;
    size_t off[64], sz[64];
    size_t lv = orc_merkle_levels(n, off, sz);
    size_t d = 0, i = index;
    for (size_t l = 0; l + 1 < lv; l++) {
        if ((i ^ 1) < sz[l]) {
            memcpy(digests + 32 * d, nodes + 32 * (off[l] + (i ^ 1)), 32);
            d++;
        }
        i /= 2;
    }
    *ndig = d;
    return 1;
}

/* Proof::validate merkle.rs:83-103 */
int orc_proof_validate(const uint8_t *value, size_t len, size_t index, const uint8_t *digests,
                       size_t ndig, const uint8_t root[32], size_t n) {
    uint8_t d[32], t[32];
    orc_sha3_256(value, len, d);
    size_t i = index, lvl_n = n, used = 0;
    while (lvl_n > 1) {
        if ((i ^ 1) < lvl_n) {
            if (used >= ndig) return 0; /* not enough levels */
            const uint8_t *s = digests + 32 * used++;
            if (i & 1)
                hash_pair(s, d, t);
            else
                hash_pair(d, s, t);
            memcpy(d, t, 32);
        }
        i /= 2;
        lvl_n = (lvl_n + 1) / 2;
    }
    if (used != ndig) return 0; /* too many levels */
    return memcmp(d, root, 32) == 0;
}

/* ===================================================================== */
/* Framing (broadcast.rs:170-189) and unframing (587-600)                 */
/* ===================================================================== */
size_t orc_shard_len(size_t payload_len, size_t k) { return (payload_len + 4 + k - 1) / k; }

void orc_frame(const uint8_t *payload, size_t plen, size_t k, size_t m, size_t S, uint8_t *out) {
    memset(out, 0, (k + m) * S);
    out[0] = (uint8_t)(plen >> 24);
    out[1] = (uint8_t)(plen >> 16);
    out[2] = (uint8_t)(plen >> 8);
    out[3] = (uint8_t)plen;
    memcpy(out + 4, payload, plen);
}

long orc_unframe(const uint8_t *data, size_t k, size_t S, uint8_t *out) {
    size_t total = k * S;
    if (total < 4) return -1;
    size_t len = ((size_t)data[0] << 24) | ((size_t)data[1] << 16) | ((size_t)data[2] << 8) |
                 (size_t)data[3];
    if (len > total - 4) len = total - 4; /* bytes.take(payload_len) truncates */
    memcpy(out, data + 4, len);
    return (long)len;
}

/* ===================================================================== */
/* Whole-path helpers                                                     */
/* ===================================================================== */
int orc_send_shards(size_t n, size_t f, const uint8_t *payload, size_t plen, uint8_t *shards,
                    uint8_t *nodes) {
    size_t m = 2 * f, k = n - m;
    size_t S = orc_shard_len(plen, k);
    orc_frame(payload, plen, k, m, S, shards);
    uint8_t *ptrs[256];
    size_t lens[256];
    for (size_t i = 0; i < n; i++) {
        ptrs[i] = shards + i * S;
        lens[i] = S;
    }
    if (m > 0) {
        int st = orc_rs_encode(k, m, ptrs, lens, n);
        if (st) return st;
    }
    orc_merkle_build(n, (const uint8_t *const *)ptrs, lens, nodes);
    return ORC_OK;
}

long orc_decode_from_shards(size_t n, size_t f, uint8_t *shards, size_t S, const uint8_t *present,
                            const uint8_t root[32], uint8_t *payload_out) {
    size_t m = 2 * f, k = n - m;
    uint8_t *ptrs[256];
    size_t lens[256];
    for (size_t i = 0; i < n; i++) {
        ptrs[i] = shards + i * S;
        lens[i] = S;
    }
    if (orc_coding_reconstruct(k, m, ptrs, lens, present, n)) return -1;
    size_t cnt = orc_merkle_node_count(n);
    uint8_t *nodes = (uint8_t *)malloc(32 * cnt);
    orc_merkle_build(n, (const uint8_t *const *)ptrs, lens, nodes);
    int same = memcmp(nodes + 32 * (cnt - 1), root, 32) == 0;
    free(nodes);
    if (!same) return -2;
    long r = orc_unframe(shards, k, S, payload_out);
    return r < 0 ? -3 : r;
}

/* ===================================================================== */
/* Synthetic workload: counter-based (SplitMix64 finaliser)               */
/* ===================================================================== */
uint64_t orc_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

#define GEN_C1 0xD6E8FEB86659FD93ULL
#define GEN_C2 0xA0761D6478BD642FULL

void orc_gen_payload(uint64_t seed, uint64_t inst, uint8_t *out, size_t len) {
    uint64_t base = seed * GEN_C1 + inst * GEN_C2;
    for (size_t q = 0; q * 8 < len; q++) {
        uint64_t v = orc_mix64(base + q);
        for (size_t b = 0; b < 8 && q * 8 + b < len; b++) out[q * 8 + b] = (uint8_t)(v >> (8 * b));
    }
}

void orc_gen_present(uint64_t seed, uint64_t inst, size_t n, size_t n_erase, uint8_t *present) {
    uint64_t base = (seed ^ 0x5EED5EED5EED5EEDULL) * GEN_C1 + inst * GEN_C2;
    for (size_t i = 0; i < n; i++) present[i] = 1;
    for (size_t t = 0; t < n_erase && t < n; t++) {
        size_t r = (size_t)(orc_mix64(base + t) % (uint64_t)(n - t));
        for (size_t i = 0; i < n; i++) {
            if (!present[i]) continue;
            if (r == 0) {
                present[i] = 0;
                break;
            }
            r--;
        }
    }
}

/* ===================================================================== */
/* CPU baseline: the whole pipeline, pthreads over independent instances. */
/* ===================================================================== */
typedef struct {
    size_t n, f, plen, count, n_erase, tid, nthreads;
    uint64_t seed;
    const uint8_t *payloads;
    size_t ok;
} bench_job;

static void *bench_worker(void *arg) {
    bench_job *j = (bench_job *)arg;
    size_t n = j->n, m = 2 * j->f, k = n - m;
    size_t S = orc_shard_len(j->plen, k);
    size_t cnt = orc_merkle_node_count(n);
    uint8_t *shards = (uint8_t *)malloc(n * S);
    uint8_t *nodes = (uint8_t *)malloc(32 * cnt);
    uint8_t *dig = (uint8_t *)malloc(32 * 64);
    uint8_t *present = (uint8_t *)malloc(n);
    uint8_t *out = (uint8_t *)malloc(k * S + 8);
    uint8_t *ptrs[256];
    for (size_t i = 0; i < n; i++) ptrs[i] = shards + i * S;
    for (size_t inst = j->tid; inst < j->count; inst += j->nthreads) {
        const uint8_t *payload = j->payloads + inst * j->plen;
        orc_send_shards(n, j->f, payload, j->plen, shards, nodes);
        const uint8_t *root = nodes + 32 * (cnt - 1);
        int all_valid = 1;
        for (size_t i = 0; i < n; i++) {
            size_t nd = 0;
            orc_merkle_proof(n, nodes, i, dig, &nd);
            all_valid &= orc_proof_validate(ptrs[i], S, i, dig, nd, root, n);
        }
        orc_gen_present(j->seed, inst, n, j->n_erase, present);
        for (size_t i = 0; i < n; i++)
            if (!present[i]) memset(ptrs[i], 0, S);
        uint8_t rootc[32];
        memcpy(rootc, root, 32);
        long r = orc_decode_from_shards(n, j->f, shards, S, present, rootc, out);
        if (all_valid && r == (long)j->plen && memcmp(out, payload, j->plen) == 0) j->ok++;
    }
    free(shards);
    free(nodes);
    free(dig);
    free(present);
    free(out);
    return NULL;
}

double orc_bench_pipeline(size_t n, size_t f, size_t plen, size_t count, size_t n_erase,
                          uint64_t seed, int threads, size_t *ok_out) {
    gf_init();
    if (threads < 1) threads = 1;
    uint8_t *payloads = (uint8_t *)malloc(count * plen + 1);
    for (size_t i = 0; i < count; i++) orc_gen_payload(seed, i, payloads + i * plen, plen);
    bench_job *jobs = (bench_job *)calloc((size_t)threads, sizeof(bench_job));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        bench_job *j = &jobs[t];
        j->n = n;
        j->f = f;
        j->plen = plen;
        j->count = count;
        j->n_erase = n_erase;
        j->tid = (size_t)t;
        j->nthreads = (size_t)threads;
        j->seed = seed;
        j->payloads = payloads;
        pthread_create(&th[t], NULL, bench_worker, j);
    }
    size_t ok = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        ok += jobs[t].ok;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (ok_out) *ok_out = ok;
    free(payloads);
    free(jobs);
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
