// api.hip -- implementation of include/hbrbc.h (the C ABI of libhbrbc.so).
//
// Host-side responsibilities only: argument checks with the reference's
// error semantics, the encoding matrix (rse `build_matrix`, computed once per
// context exactly like `ReedSolomon::new`), device workspaces (the
// decode-matrix cache among them), specialised-kernel modules, and launch
// sequencing.  Every byte of shard, digest and payload data is computed by
// the HIP kernels in kernels.hip / jit.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <dlfcn.h>
#include <sys/stat.h>

#include "../../include/hbrbc.h"
#include "device_common.hpp"
#include "jit.hpp"
#include "launchers.hpp"

using namespace hbrbc;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HB_HIP(call)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(HBRBC_E_DEVICE, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),  \
                        __FILE__, __LINE__);                                                    \
    } while (0)

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- host GF(2^8) for the encoding matrix (rse galois_8 / build_matrix) --
struct HostGf {
    uint8_t exp[512], log[256];
    HostGf() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = exp[i + 255] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        exp[510] = exp[0];
        exp[511] = exp[1];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t inv(uint8_t a) const { return exp[(255 - log[a]) % 255]; }
    uint8_t pow(uint8_t a, size_t n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(log[a] * n) % 255];
    }
};
const HostGf &gf() {
    static HostGf t;
    return t;
}

bool gf_invert(size_t n, std::vector<uint8_t> &m) {
    const HostGf &g = gf();
    std::vector<uint8_t> inv(n * n, 0);
    for (size_t i = 0; i < n; ++i) inv[i * n + i] = 1;
    for (size_t c = 0; c < n; ++c) {
        size_t p = c;
        while (p < n && m[p * n + c] == 0) ++p;
        if (p == n) return false;
        if (p != c)
            for (size_t j = 0; j < n; ++j) {
                std::swap(m[c * n + j], m[p * n + j]);
                std::swap(inv[c * n + j], inv[p * n + j]);
            }
        const uint8_t s = g.inv(m[c * n + c]);
        for (size_t j = 0; j < n; ++j) {
            m[c * n + j] = g.mul(s, m[c * n + j]);
            inv[c * n + j] = g.mul(s, inv[c * n + j]);
        }
        for (size_t r = 0; r < n; ++r) {
            const uint8_t f = m[r * n + c];
            if (r == c || f == 0) continue;
            for (size_t j = 0; j < n; ++j) {
                m[r * n + j] ^= g.mul(f, m[c * n + j]);
                inv[r * n + j] ^= g.mul(f, inv[c * n + j]);
            }
        }
    }
    m.swap(inv);
    return true;
}

// rse build_matrix(k, total) = vandermonde(total, k) * inv(vandermonde[0..k]).
bool build_matrix(size_t k, size_t total, std::vector<uint8_t> &out) {
    const HostGf &g = gf();
    std::vector<uint8_t> v(total * k), top;
    for (size_t r = 0; r < total; ++r)
        for (size_t c = 0; c < k; ++c) v[r * k + c] = g.pow((uint8_t)r, c);
    top.assign(v.begin(), v.begin() + k * k);
    if (!gf_invert(k, top)) return false;
    out.assign(total * k, 0);
    for (size_t r = 0; r < total; ++r)
        for (size_t c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (size_t j = 0; j < k; ++j) acc ^= g.mul(v[r * k + j], top[j * k + c]);
            out[r * k + c] = acc;
        }
    return true;
}

// The recovery rows of one erasure pattern, as rse reconstruct would use
// them: valid = the first k present rows, missing = every absent row;
// rows[t] = M[missing[t]] * inv(M[valid]) (a missing data row is a row of the
// inverse).  false: fewer than k present, none missing or a singular block.
bool recovery_rows(const std::vector<uint8_t> &mat, size_t k, size_t n, const uint8_t *present,
                   std::vector<int> &valid, std::vector<int> &missing,
                   std::vector<uint8_t> &rows) {
    const HostGf &g = gf();
    valid.clear();
    missing.clear();
    for (size_t i = 0; i < n; ++i) {
        if (present[i]) {
            if (valid.size() < k) valid.push_back((int)i);
        } else {
            missing.push_back((int)i);
        }
    }
    if (valid.size() < k || missing.empty()) return false;
    std::vector<uint8_t> sub(k * k);
    for (size_t r = 0; r < k; ++r)
        for (size_t c = 0; c < k; ++c) sub[r * k + c] = mat[(size_t)valid[r] * k + c];
    if (!gf_invert(k, sub)) return false;
    rows.assign(missing.size() * k, 0);
    for (size_t t = 0; t < missing.size(); ++t) {
        const size_t row = (size_t)missing[t];
        for (size_t c = 0; c < k; ++c) {
            uint8_t acc = 0;
            if (row < k) {
                acc = sub[row * k + c];
            } else {
                for (size_t j = 0; j < k; ++j) acc ^= g.mul(mat[row * k + j], sub[j * k + c]);
            }
            rows[t * k + c] = acc;
        }
    }
    return true;
}

// Grow-only device buffer.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        size_t b = round_up(bytes < 256 ? 256 : bytes, 256);
        hipError_t e = hipMalloc(&p, b);
        if (e == hipSuccess) cap = b;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

// Grow-only pinned host buffer (staging of the per-call shims: one DMA per
// direction instead of one pageable copy per shard).
struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) {
            (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
        }
        size_t b = round_up(bytes < 4096 ? 4096 : bytes, 4096);
        hipError_t e = hipHostMalloc(&p, b, hipHostMallocDefault);
        if (e == hipSuccess) cap = b;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

// rows_per_block (ABI) -> RowMap / code-object block size
RowMap make_rows(size_t n, size_t shard_stride, size_t rows_per_block, size_t block_stride) {
    RowMap r = plain_rows(shard_stride);
    if (rows_per_block && rows_per_block < n) {
        r.rb = (uint32_t)rows_per_block;
        r.bst = block_stride;
    }
    return r;
}
inline int code_rb(const RowMap &r) { return r.plain() ? 256 : (int)r.rb; }

}  // namespace

struct hbrbc_ctx {
    int device = 0;
    size_t k = 0, m = 0, n = 0;
    int rt_enc = 2, rt_rec = 2;  // GF row tiles (rows per pass) for encode / reconstruct
    int gf_mode = 0;             // generic kernel: 0 branch per bit, 1 hinted, 2 masked, 3 bit pairs, 4 input pairs
    std::vector<uint8_t> matrix;  // n x k
    hipStream_t stream = nullptr;
    // specialised XOR-network modules (jit.hip): one module per output-row group
    struct SpecGroup {
        int r_lo, r_hi;
        hipModule_t mod;
        hipFunction_t fn, fe;        // kernel / frame+encode twin (encoder only)
        // LDS-staged form (jit.hip gen_xor_kernel_lds): its waves share the
        // stage's input planes, so it cannot run pass by pass
        bool lds = false;
    };
    // encoder modules by code-object row block (256 = plain layout); an
    // empty vector records a failed load
    std::map<int, std::vector<SpecGroup>> enc_spec;
    int rt_spec = 2;              // output rows per pass of the specialised kernels
    int depth_spec = 4;           // their input-row prefetch depth
    std::string enc_kind = "none";
    // pattern-specialised decoders: at most one per code-object row block
    struct DecSpec {
        uint64_t hash;
        int rt;
        std::vector<SpecGroup> groups;
        // the fused-unframe variant of the same programs, loaded (or compiled)
        // on the first call that fuses: 0 untried, 1 loaded, -1 unavailable
        std::vector<SpecGroup> uf_groups;
        int uf_state = 0;
        std::vector<uint8_t> present;
    };
    std::map<int, DecSpec> dec_spec;
    std::string jit_missing;   // HBRBC_JIT=load: why an encoder code object is missing
    // side streams + events for the concurrent launch of a matrix's programs
    // (HBRBC_XOR_STREAMS, launch_groups)
    std::vector<hipStream_t> side;
    std::vector<hipEvent_t> side_ev;
    DevBuf d_matrix, d_enc_coefs, d_enc_in, d_enc_out;
    // reconstruct workspace: decode-matrix cache + per-call scratch
    size_t ws_count = 0;
    int pc_cap = 0;
    size_t pc_inserted = 0;       // upper bound of shared slots filled since the last clear
    DevBuf pc_hash, pc_keys, pc_coefs, pc_in, pc_out, pc_nout, pc_status, pc_fill;
    DevBuf ws_pat, ws_own, ws_status, ws_list, ws_counter;
    // per-call shim staging
    std::mutex shim_mu;
    DevBuf st_slab, st_nodes, st_aux;
    PinBuf pin;
    // profiling
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    struct Rec {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Rec> recs;

    hipEvent_t take_event() {
        if (ev_used == ev_pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            ev_pool.push_back(e);
        }
        return ev_pool[ev_used++];
    }
    size_t coef_stride() const { return (m + rt_rec - 1) / rt_rec * k * 16 + 16; }
};

namespace {

// Brackets one stage's launches with events when profiling is on.
struct StageTimer {
    hbrbc_ctx *c;
    int stage;
    hipStream_t s;
    hipEvent_t a = nullptr;
    StageTimer(hbrbc_ctx *c_, int st, hipStream_t s_) : c(c_), stage(st), s(s_) {
        if (c && c->prof) {
            a = c->take_event();
            if (a) (void)hipEventRecord(a, s);
        }
    }
    ~StageTimer() {
        if (a) {
            hipEvent_t b = c->take_event();
            if (b) {
                (void)hipEventRecord(b, s);
                c->recs.push_back({stage, a, b});
            }
        }
    }
};

// NULL selects the HIP null (default) stream, as for hipMemcpyAsync; the
// context's own stream is used only by the synchronous per-call shims.
inline hipStream_t pick(hbrbc_ctx *, void *stream) { return static_cast<hipStream_t>(stream); }

int check_slab(const void *base, size_t shard_len, size_t shard_stride, size_t inst_stride,
               size_t n, size_t count, size_t rows_per_block = 0, size_t block_stride = 0) {
    if (count == 0) return HBRBC_OK;
    if (!base) return fail(HBRBC_E_INVALID_ARG, "null shard slab");
    if (reinterpret_cast<uintptr_t>(base) % 16)
        return fail(HBRBC_E_INVALID_ARG, "shard slab base must be 16-byte aligned");
    if (shard_stride % 16 || shard_stride < shard_len)
        return fail(HBRBC_E_INVALID_ARG, "shard_stride %zu must be a multiple of 16 and >= %zu",
                    shard_stride, shard_len);
    if (shard_len > 0xFFFFFFFFull) return fail(HBRBC_E_INVALID_ARG, "shard_len too large");
    if (rows_per_block && rows_per_block < n) {
        // blocked rows: blocks of rows_per_block rows, instances interleaved inside a block
        if (rows_per_block > 255)
            return fail(HBRBC_E_INVALID_ARG, "rows_per_block %zu > 255", rows_per_block);
        if (block_stride % 16 || inst_stride % 16 || inst_stride < rows_per_block * shard_stride)
            return fail(HBRBC_E_INVALID_ARG, "blocked layout: inst_stride %zu must be a multiple "
                        "of 16 and >= rows_per_block * shard_stride", inst_stride);
        if (block_stride < count * inst_stride)
            return fail(HBRBC_E_INVALID_ARG, "blocked layout: block_stride %zu < count * "
                        "inst_stride", block_stride);
        if ((uint64_t)rows_per_block * shard_stride >= 0x7FFFFFFFull)
            return fail(HBRBC_E_INVALID_ARG, "row block larger than 2 GiB");
        return HBRBC_OK;
    }
    if (count > 1 && (inst_stride % 16 || inst_stride < n * shard_stride))
        return fail(HBRBC_E_INVALID_ARG, "inst_stride %zu must be a multiple of 16 and >= %zu",
                    inst_stride, n * shard_stride);
    return HBRBC_OK;
}

int check_nodes(const void *nodes, size_t node_inst_stride, size_t n, size_t count) {
    if (count == 0) return HBRBC_OK;
    if (!nodes || reinterpret_cast<uintptr_t>(nodes) % 16)
        return fail(HBRBC_E_INVALID_ARG, "node slab must be non-null and 16-byte aligned");
    if (node_inst_stride % 16 || (count > 1 && node_inst_stride < 32 * hbrbc_merkle_node_count(n)))
        return fail(HBRBC_E_INVALID_ARG, "node_inst_stride %zu too small or unaligned",
                    node_inst_stride);
    return HBRBC_OK;
}

// Reconstruct workspace for `count` instances: the pattern cache (cap shared
// slots, count private ones) and per-call scratch.  Growing it drops the cache.
int ensure_workspace(hbrbc_ctx *c, size_t count) {
    if (count <= c->ws_count) return HBRBC_OK;
    const size_t k = c->k, m = c->m;
    int cap = 1024;
    while ((size_t)cap < 2 * count) cap *= 2;
    const size_t slots = (size_t)cap + count;
    HB_HIP(c->pc_hash.ensure((size_t)cap * sizeof(uint64_t)));
    HB_HIP(c->pc_keys.ensure(slots * 8 * sizeof(uint32_t)));
    HB_HIP(c->pc_coefs.ensure(slots * c->coef_stride()));
    HB_HIP(c->pc_in.ensure((slots * k + 4) * sizeof(uint32_t)));
    HB_HIP(c->pc_out.ensure((slots * m + 4) * sizeof(uint32_t)));
    HB_HIP(c->pc_nout.ensure(slots * sizeof(int)));
    HB_HIP(c->pc_status.ensure(slots * sizeof(int32_t)));
    HB_HIP(c->pc_fill.ensure(sizeof(uint32_t)));
    HB_HIP(c->ws_pat.ensure(count * sizeof(int)));
    HB_HIP(c->ws_own.ensure(count));
    HB_HIP(c->ws_status.ensure(count * sizeof(int32_t)));
    HB_HIP(c->ws_list.ensure((count * std::max<size_t>(m, 1) + 1) * sizeof(uint2)));
    HB_HIP(c->ws_counter.ensure(sizeof(uint32_t)));
    HB_HIP(hipMemset(c->pc_hash.p, 0, (size_t)cap * sizeof(uint64_t)));
    HB_HIP(hipMemset(c->pc_fill.p, 0, sizeof(uint32_t)));
    c->pc_cap = cap;
    c->pc_inserted = 0;
    c->ws_count = count;
    return HBRBC_OK;
}

PatternCache cache_view(hbrbc_ctx *c) {
    PatternCache pc;
    pc.hash = c->pc_hash.as<uint64_t>();
    pc.keys = c->pc_keys.as<uint32_t>();
    pc.coefs = c->pc_coefs.as<uint8_t>();
    pc.coef_stride = c->coef_stride();
    pc.in_idx = c->pc_in.as<uint32_t>();
    pc.out_idx = c->pc_out.as<uint32_t>();
    pc.nout = c->pc_nout.as<int>();
    pc.status = c->pc_status.as<int32_t>();
    pc.fill = c->pc_fill.as<uint32_t>();
    pc.cap = c->pc_cap;
    return pc;
}

// Leaf hashes + all levels into a node slab (known_leaves: level 0 holds the
// leaves of every row but the ones the last reconstruct rebuilt).
// Leaf kernel + one launch per level (default), or leaves and levels in one
// launch with the levels reduced in LDS (HBRBC_MERKLE_FUSED=1).  The fused
// form measured slower at cfg3 (leaf hash + levels 20.95 -> 21.4 ms per step:
// each workgroup holds its four wave slots through six dependent pair-hash
// levels with at most half its lanes busy) and flat at cfg5.
bool merkle_split() {
    const char *e = getenv("HBRBC_MERKLE_FUSED");
    return !(e && !std::strcmp(e, "1"));
}

int run_merkle(hbrbc_ctx *c, const uint8_t *shards, size_t shard_len, const RowMap &rows,
               size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
               size_t node_inst_stride, bool known_leaves, hipStream_t s) {
    if (!known_leaves && merkle_fused_ok(n) && !merkle_split()) {
        // leaves and levels in one launch, attributed to the leaf-hash stage
        StageTimer t(c, HBRBC_STAGE_LEAF_HASH, s);
        HB_HIP(launch_merkle_fused(shards, shard_len, rows, inst_stride, n, count, nodes,
                                   node_inst_stride, s));
        return HBRBC_OK;
    }
    {
        StageTimer t(c, HBRBC_STAGE_LEAF_HASH, s);
        if (!known_leaves) {
            HB_HIP(launch_leaf_hash(shards, shard_len, rows, inst_stride, n, count, nodes,
                                    node_inst_stride, s));
        } else if (c->m > 0) {
            HB_HIP(launch_leaf_hash_rebuilt(shards, shard_len, rows, inst_stride, count,
                                            c->ws_pat.as<int>(), c->pc_out.as<uint32_t>(), c->m,
                                            c->pc_nout.as<int>(), (int)c->m, nodes,
                                            node_inst_stride, c->ws_counter.as<uint32_t>(),
                                            c->ws_list.as<uint2>(), s));
        }
    }
    StageTimer t(c, HBRBC_STAGE_TREE_LEVELS, s);
    // HBRBC_TREE_LEVELS_LDS=1: every level in one LDS-reduced launch (measured
    // slower at cfg3: 0.80 vs 0.31 ms per step -- the upper levels idle most
    // lanes of a block, while per-level launches keep every lane busy)
    const char *lv = getenv("HBRBC_TREE_LEVELS_LDS");
    if (n <= 512 && lv && !std::strcmp(lv, "1")) {
        HB_HIP(launch_tree_levels(nodes, node_inst_stride, n, count, s));
        return HBRBC_OK;
    }
    size_t off = 0, sz = n;
    while (sz > 1) {
        const size_t nsz = (sz + 1) / 2;
        HB_HIP(launch_tree_level(nodes, node_inst_stride, off, sz, off + sz, nsz, count, s));
        off += sz;
        sz = nsz;
    }
    return HBRBC_OK;
}

hipError_t launch_xor_group(const hbrbc_ctx::SpecGroup &g, bool fused, int rt, XorArgs a,
                            size_t count, hipStream_t s);
hipError_t launch_groups(hbrbc_ctx *c, const std::vector<hbrbc_ctx::SpecGroup> &gs, size_t first,
                         int rt, const XorArgs &x, size_t count, hipStream_t s);

// Fused unframe (decode paths): the generic reconstruct kernel writes the
// payload bytes of the data rows it reads or rebuilds, so unframe's re-read of
// k*S bytes per instance disappears (decode_check + a zero-fill fixup remain).
// Any S (byte-aligned 16-byte stores, round 3; cfg4 S % 4 = 2, cfg5 S odd),
// in the generic kernel and in the pattern-specialised decoders' _uf
// variants (v20 code objects).
// HBRBC_UNFRAME_FUSED=0 keeps the separate unframe (A/B).
bool unframe_fusable(const hbrbc_ctx *c, size_t shard_len, size_t payload_stride) {
    const char *e = getenv("HBRBC_UNFRAME_FUSED");
    if (e && !std::strcmp(e, "0")) return false;
    return c->m > 0 && payload_stride % 16 == 0 && (uint64_t)c->k * shard_len > 4;
}

// HBRBC_JIT: unset = encoders from the code-object cache when present,
// decoders compiled on a miss; "0" = no specialised encoders; "1" = compile
// any missing code object; "load" = cache only, and a missing code object is
// an error (proves build() pre-built every object a run needs).
enum JitMode { JIT_DEFAULT, JIT_OFF, JIT_COMPILE, JIT_LOAD };
JitMode jit_mode() {
    const char *e = getenv("HBRBC_JIT");
    if (!e) return JIT_DEFAULT;
    if (!std::strcmp(e, "0")) return JIT_OFF;
    if (!std::strcmp(e, "1")) return JIT_COMPILE;
    if (!std::strcmp(e, "load")) return JIT_LOAD;
    return JIT_DEFAULT;
}

bool decode_programs(const std::vector<uint8_t> &mat, size_t k, size_t n, const uint8_t *present,
                     int rb, std::vector<XorProgram> &out, uint64_t &hash, int &rt, bool uf);
int load_program(const XorProgram &p, bool compile, hbrbc_ctx::SpecGroup &g);
void drop_groups(std::vector<hbrbc_ctx::SpecGroup> &gs);

// The _uf variant of a specialised decoder, loaded (or, unless HBRBC_JIT=0,
// compiled) once; false if unavailable (the call then unframes separately).
bool uf_decoder(hbrbc_ctx *c, hbrbc_ctx::DecSpec &d, int rb) {
    if (d.uf_state == 0) {
        std::vector<XorProgram> progs;
        uint64_t hash = 0;
        int rt = 2;
        const bool compile = jit_mode() == JIT_DEFAULT || jit_mode() == JIT_COMPILE;
        const std::string saved = g_err;
        d.uf_state = -1;
        if (decode_programs(c->matrix, c->k, c->n, d.present.data(), rb, progs, hash, rt, true)) {
            d.uf_state = 1;
            for (const auto &p : progs) {
                hbrbc_ctx::SpecGroup g{0, (int)p.out_rows.size(), nullptr, nullptr, nullptr};
                if (load_program(p, compile, g)) {
                    drop_groups(d.uf_groups);
                    d.uf_state = -1;
                    break;
                }
                d.uf_groups.push_back(g);
            }
        }
        g_err = saved;   // a missing variant is not an error of the caller's call
    }
    return d.uf_state == 1;
}

int run_reconstruct(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, const RowMap &rows,
                    size_t inst_stride, const uint8_t *present, size_t count, int32_t *status,
                    hipStream_t s, uint8_t *uf_payload = nullptr, size_t uf_stride = 0,
                    bool *fused_out = nullptr) {
    if (fused_out) *fused_out = false;
    int st = ensure_workspace(c, count);
    if (st) return st;
    // rse keeps an LRU of decode matrices; here the shared slots are flushed
    // once the patterns inserted since the last flush could exceed 4x the
    // table (a repeating pattern is then recomputed once per flush)
    if (c->pc_inserted + count > 4 * (size_t)c->pc_cap) {
        HB_HIP(hipMemsetAsync(c->pc_hash.p, 0, (size_t)c->pc_cap * sizeof(uint64_t), s));
        HB_HIP(hipMemsetAsync(c->pc_fill.p, 0, sizeof(uint32_t), s));
        c->pc_inserted = 0;
    }
    c->pc_inserted += count;
    const auto ds = c->dec_spec.find(code_rb(rows));
    const bool spec = ds != c->dec_spec.end() && !ds->second.groups.empty();
    {
        StageTimer t(c, HBRBC_STAGE_DECODE_MATRIX, s);
        DecodeMatrixArgs a;
        a.n = (int)c->n;
        a.k = (int)c->k;
        a.rt = c->rt_rec;
        a.matrix = c->d_matrix.as<uint8_t>();
        a.present = present;
        a.count = count;
        a.cache = cache_view(c);
        a.pat = c->ws_pat.as<int>();
        a.own = c->ws_own.as<uint8_t>();
        a.status = status;
        if (spec) {   // slots of the specialised pattern's hash hold only that pattern
            a.spec_hash = ds->second.hash;
            pattern_mask(ds->second.present.data(), (int)c->n, a.spec_mask);
        }
        HB_HIP(launch_decode_matrix(a, s));
    }
    if (c->m == 0) return HBRBC_OK;  // Coding::Trivial: nothing to rebuild
    StageTimer t(c, HBRBC_STAGE_RECONSTRUCT, s);
    // fusing with a specialised decoder needs its _uf variant
    if (spec && uf_payload && !uf_decoder(c, ds->second, code_rb(rows))) uf_payload = nullptr;
    if (spec) {
        XorArgs x{};
        x.base = shards;
        x.inst_stride = inst_stride;
        x.shard_stride = rows.sst;
        x.block_stride = rows.bst;
        x.row_bytes = (unsigned)round_up(shard_len, 16);
        x.pat = c->ws_pat.as<int>();
        x.slot_hash = reinterpret_cast<const unsigned long *>(c->pc_hash.as<uint64_t>());
        x.hash_slots = c->pc_cap;
        x.p_only = -1;
        x.S = (unsigned)shard_len;
        if (uf_payload) {       // fused unframe in the pattern decoders too (_uf variant)
            x.uf_payload = uf_payload;
            x.uf_stride = uf_stride;
            x.uf_status = status;
        }
        HB_HIP(launch_groups(c, uf_payload ? ds->second.uf_groups : ds->second.groups, 0,
                             ds->second.rt, x, count, s));
    }
    GfApplyArgs g{};
    g.base = shards;
    g.inst_stride = inst_stride;
    g.rows = rows;
    g.n16 = (int)((shard_len + 15) / 16);
    g.coefs = c->pc_coefs.as<uint8_t>();
    g.coef_slot_stride = c->coef_stride();
    g.in_idx = c->pc_in.as<uint32_t>();
    g.in_idx_stride = c->k;
    g.out_idx = c->pc_out.as<uint32_t>();
    g.out_idx_stride = c->m;
    g.nout = c->pc_nout.as<int>();
    g.nout_uniform = 0;
    g.pat = c->ws_pat.as<int>();
    g.slot_hash = c->pc_hash.as<uint64_t>();
    g.skip_hash = spec ? ds->second.hash : 0;
    g.hash_slots = c->pc_cap;
    g.max_rows = (int)c->m;
    g.nin = (int)c->k;
    g.rt = c->rt_rec;
    g.mode = c->gf_mode;
    g.count = count;
    if (uf_payload) {
        g.payload = uf_payload;
        g.payload_stride = uf_stride;
        g.payload_S = (uint32_t)shard_len;
        g.payload_k = (uint32_t)c->k;
        g.rstatus = status;
        if (fused_out) *fused_out = true;
    }
    HB_HIP(launch_gf_apply(g, s));
    return HBRBC_OK;
}

// Directory of cached specialised code objects: $HBRBC_JIT_DIR, else
// <directory of libhbrbc.so>/jit.
std::string jit_dir() {
    if (const char *e = getenv("HBRBC_JIT_DIR")) return e;
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&hbrbc_version), &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        const size_t cut = p.find_last_of('/');
        return (cut == std::string::npos ? std::string(".") : p.substr(0, cut)) + "/jit";
    }
    return "jit";
}

std::string jit_file(const std::string &dir, const std::string &kernel) {
    const char *aux = getenv("HBRBC_ST_AUX");   // A/B builds get their own files
    return dir + "/" + kernel + (aux && std::strcmp(aux, "2") ? std::string("_a") + aux : std::string()) +
           "_v23.co";   // v23: the reconstruct programs store whole 16-byte payload chunks only
}

// Input rows in flight of the specialised kernels (HBM latency at 2 waves/SIMD).
int spec_depth() {
    if (const char *e = getenv("HBRBC_JIT_DEPTH")) return std::max(1, std::min(8, atoi(e)));
    return 4;
}

// Payload rows in flight of the frame+encode twins (36 loaded bytes per row
// and lane).  HBRBC_JIT_FDEPTH overrides (A/B).
int spec_fdepth() {
    if (const char *e = getenv("HBRBC_JIT_FDEPTH")) return std::max(1, std::min(8, atoi(e)));
    return 2;
}

// Data-row stores of the frame+encode twins spread over the passes
// (HBRBC_JIT_SPREAD=0: all in pass 0, A/B).
bool spec_spread() {
    const char *e = getenv("HBRBC_JIT_SPREAD");
    return !(e && !std::strcmp(e, "0"));
}

// Lane byte positions of the specialised kernels as two 16-byte pieces 1 KB
// apart: every load and store instruction covers 1 KB of consecutive bytes
// (cfg3 frame+encode 4.82 -> 4.36 ms against 32 consecutive bytes per lane;
// HBRBC_JIT_SPLIT=0 builds those, A/B).
bool spec_split() {
    const char *e = getenv("HBRBC_JIT_SPLIT");
    return !(e && !std::strcmp(e, "0"));
}

// Lockstep interval (input rows between workgroup barriers) of the
// specialised kernels; 0 = none.  HBRBC_JIT_SYNC overrides (A/B).
int spec_sync() {
    if (const char *e = getenv("HBRBC_JIT_SYNC")) return std::max(0, std::min(64, atoi(e)));
    return 0;
}

// LDS-staged specialised kernels (jit.hip gen_xor_kernel_lds): every input
// framed and transposed once per workgroup.  Default for 16..32 input rows
// (cfg3, k = 22: frame+encode 4.25 -> 3.70 ms on one box, r3 A/B in
// profiles/r3_enc_variants.txt); HBRBC_JIT_LDS=0/1 overrides (A/B).
bool spec_lds(size_t nin, size_t nout) {
    if (const char *e = getenv("HBRBC_JIT_LDS")) return !std::strcmp(e, "1");
    // cfg4 (k = 44): encode 4.41 -> 2.92 ms; cfg5 (k = 84, four programs):
    // encode 12.11 -> 9.89, worst-case reconstruct 11.28 -> 9.08 ms (r3 A/B)
    return nin >= 16 && nout >= 14;
}

// XOR-network form: 0 auto, 1 pairwise, 2 nibble-subset (HBRBC_JIT_NET, A/B).
int spec_net() {
    if (const char *e = getenv("HBRBC_JIT_NET")) return std::max(0, std::min(2, atoi(e)));
    return 0;
}

// LDS stage size (inputs per stage) and waves/SIMD target of the LDS form
// (HBRBC_JIT_LDS_STAGE, HBRBC_JIT_WPE; A/B).
int spec_lds_stage() {
    if (const char *e = getenv("HBRBC_JIT_LDS_STAGE")) return std::max(1, std::min(32, atoi(e)));
    return 0;
}
// waves/SIMD the LDS form targets: 7-row passes hold 56 accumulators, so
// 128 VGPRs (4 waves/SIMD) fit without spills (r3 A/B)
int spec_row_tile(size_t nin, size_t nout);
int spec_wpe(size_t nin, size_t nout) {
    if (const char *e = getenv("HBRBC_JIT_WPE")) return std::max(0, std::min(8, atoi(e)));
    if (!spec_lds(nin, nout)) return 0;
    // <= 8-row passes: 128 VGPRs (4 waves/SIMD); 9..11-row passes: 168 (3)
    return spec_row_tile(nin, nout) <= 8 ? 4 : 3;
}

// Code-object name suffix of the variant options above (only where they
// change the generated code: the LDS form needs 2..8 passes).
std::string spec_suffix(size_t nin, size_t nout, int rt) {
    const int npass = (int)((nout + rt - 1) / rt);
    std::string s;
    if (spec_lds(nin, nout) && npass >= 2 && npass <= 8) {
        s += "_L";
        if (spec_lds_stage()) s += std::to_string(spec_lds_stage());
    }
    if (spec_net()) s += "_n" + std::to_string(spec_net());
    if (spec_wpe(nin, nout)) s += "_w" + std::to_string(spec_wpe(nin, nout));
    return s;
}

void spec_variant(XorProgram &p) {
    const size_t nin = p.in_rows.size(), nout = p.out_rows.size();
    p.lds = spec_lds(nin, nout);
    p.lds_stage = spec_lds_stage();
    p.net = spec_net();
    p.wpe = spec_wpe(nin, nout);
    p.name += spec_suffix(nin, nout, p.rt);
}

bool read_file(const std::string &path, std::vector<char> &out) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n > 0 && fread(out.data(), 1, out.size(), f) == out.size();
    fclose(f);
    return ok;
}

bool write_file(const std::string &path, const std::vector<char> &code) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
    fclose(f);
    return ok;
}

// Output rows per pass of the specialised kernels: the accumulators (8 VGPRs
// per row) plus the planes, pair XORs and load buffers must stay near 200
// VGPRs (2 waves/SIMD) without spilling.
int spec_row_tile(size_t nin, size_t nout) {
    // (passes are balanced: rt is the longest pass; HBRBC_RT_SPEC overrides, A/B)
    if (const char *e = getenv("HBRBC_RT_SPEC")) return std::max(2, std::min(24, atoi(e)));
    // LDS form: passes no longer transpose their own inputs, so short passes
    // (7 rows, nibble-subset network, <= 128 VGPRs) cost no extra transposes;
    // a one-program matrix with more than 56 outputs takes longer passes so
    // that one workgroup holds them all (<= 8 waves; cfg4: 84 rows, 11 per pass)
    if (spec_lds(nin, nout)) {
        // split programs: 48-row groups in eight 6-row passes, one wave each
        // (cfg5 r3, same box: encode 10.0 -> 9.1 ms, worst-case reconstruct
        // 9.7 -> 8.8 ms against 42-row groups in six 7-row passes; 8-row
        // passes 9.9 / 9.5 ms; LDS stages of 12 / 16 / 28 inputs flat / flat /
        // 12.1 / 12.0 ms)
        // Same for a one-program matrix of more than 56 rows (xor_groups caps
        // a program at eight passes): cfg4 encode, 84 rows in 48 + 36 instead
        // of one program of 11-row passes at 3 waves/SIMD, 2.9 -> 2.57 ms
        if (nin * nout > 4096 || nout > 56) return 6;
        return (int)std::max<size_t>(7, (nout + 7) / 8);
    }
    // split matrices (N = 250): 12-row passes of the pairwise network, four
    // per 48-row program (cfg5 encode 14.7 -> 12.4 ms, worst-case
    // reconstruct 13.1 -> 11.4 ms against 8-row nibble passes; 16 rows:
    // 17.4 / 16.6 ms)
    return nin * nout > 4096 ? 12 : gf_row_tile((int)nout);
}

// The encoder program of parity-row group [r_lo, r_hi) for row block rb.
XorProgram encode_program(size_t k, size_t m, const uint8_t *parity_rows, int rt, int depth,
                          int r_lo, int r_hi, int rb) {
    XorProgram p;
    p.sync = spec_sync();
    p.fdepth = spec_fdepth();
    p.spread = spec_spread();
    p.split = spec_split();
    p.name = encode_kernel_name(k, m, rt, depth, r_lo, r_hi, rb, p.sync, p.fdepth, p.spread, p.split);
    for (size_t j = 0; j < k; ++j) p.in_rows.push_back((int)j);
    for (int r = r_lo; r < r_hi; ++r) p.out_rows.push_back((int)(k + r));
    p.coefs.assign(parity_rows + (size_t)r_lo * k, parity_rows + (size_t)r_hi * k);
    p.rt = rt;
    p.depth = depth;
    p.rb = rb;
    p.fused = true;
    spec_variant(p);
    return p;
}

// The decoder programs of one erasure pattern (output-row groups).
bool decode_programs(const std::vector<uint8_t> &mat, size_t k, size_t n, const uint8_t *present,
                     int rb, std::vector<XorProgram> &out, uint64_t &hash, int &rt,
                     bool uf = false) {
    std::vector<int> valid, missing;
    std::vector<uint8_t> rows;
    if (!recovery_rows(mat, k, n, present, valid, missing, rows)) return false;
    hash = pattern_hash(present, (int)n);
    rt = spec_row_tile(k, missing.size());
    const int depth = spec_depth();
    const auto groups = xor_groups(k, missing.size(), rt);
    out.clear();
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        XorProgram p;
        p.sync = spec_sync();
        p.split = spec_split();
        p.name = decode_kernel_name(n, hash, rt, depth, groups[gi].first, groups[gi].second, rb,
                                    p.sync, p.split) + (uf ? "_uf" : "");
        p.in_rows = valid;
        p.out_rows.assign(missing.begin() + groups[gi].first, missing.begin() + groups[gi].second);
        p.coefs.assign(rows.begin() + (size_t)groups[gi].first * k,
                       rows.begin() + (size_t)groups[gi].second * k);
        p.rt = rt;
        p.depth = depth;
        p.rb = rb;
        p.guard = hash;
        p.uf_k = uf ? (int)k : 0;       // fused unframe: rebuilt data rows, and
        p.uf_inputs = uf && gi == 0;    // the present ones from the first program
        if (uf) p.name.resize(p.name.size() - 3);   // variant suffix before "_uf"
        spec_variant(p);
        if (uf) p.name += "_uf";
        out.push_back(std::move(p));
    }
    return true;
}

// Load the module of `p` from the cache (or, if allowed, compile and cache it).
int load_program(const XorProgram &p, bool compile, hbrbc_ctx::SpecGroup &g) {
    const std::string path = jit_file(jit_dir(), p.name);
    std::vector<char> code;
    if (!read_file(path, code)) {
        if (!compile) return fail(HBRBC_E_INVALID_ARG, "no cached code object %s", path.c_str());
        std::string log;
        if (compile_source(gen_xor_source(p), code, log))
            return fail(HBRBC_E_DEVICE, "hiprtc: %s", log.substr(0, 400).c_str());
        mkdir(jit_dir().c_str(), 0755);
        (void)write_file(path, code);
    }
    g.mod = nullptr;
    g.fn = g.fe = nullptr;
    const int npass = (int)((p.out_rows.size() + p.rt - 1) / p.rt);
    g.lds = p.lds && npass >= 2 && npass <= 8;   // the test of gen_xor_source
    HB_HIP(hipModuleLoadData(&g.mod, code.data()));
    if (hipModuleGetFunction(&g.fn, g.mod, p.name.c_str()) != hipSuccess ||
        (p.fused && hipModuleGetFunction(&g.fe, g.mod, (p.name + "_fe").c_str()) != hipSuccess)) {
        (void)hipModuleUnload(g.mod);
        g.mod = nullptr;
        return fail(HBRBC_E_DEVICE, "kernel missing in %s", path.c_str());
    }
    return HBRBC_OK;
}

void drop_groups(std::vector<hbrbc_ctx::SpecGroup> &gs) {
    for (auto &g : gs)
        if (g.mod) (void)hipModuleUnload(g.mod);
    gs.clear();
}

// The specialised encoder of this context for row block rb, loaded on first
// use (or, with HBRBC_JIT=1, compiled and cached).  nullptr: use the generic
// kernel.
const std::vector<hbrbc_ctx::SpecGroup> *spec_encoder(hbrbc_ctx *c, int rb) {
    auto it = c->enc_spec.find(rb);
    if (it != c->enc_spec.end()) return it->second.empty() ? nullptr : &it->second;
    std::vector<hbrbc_ctx::SpecGroup> gs;
    const bool off = c->m == 0 || jit_mode() == JIT_OFF || c->k * c->m > 16384;
    if (!off) {
        const bool compile = jit_mode() == JIT_COMPILE;
        const std::string saved = g_err;
        for (const auto &rg : xor_groups(c->k, c->m, c->rt_spec)) {
            const XorProgram p = encode_program(c->k, c->m, c->matrix.data() + c->k * c->k,
                                                c->rt_spec, c->depth_spec, rg.first, rg.second, rb);
            hbrbc_ctx::SpecGroup g{rg.first, rg.second, nullptr, nullptr, nullptr};
            if (load_program(p, compile, g)) {
                drop_groups(gs);
                break;
            }
            gs.push_back(g);
        }
        if (gs.empty() && jit_mode() == JIT_LOAD) {
            // keep the load error: the caller fails instead of falling back
            c->jit_missing = g_err;
        } else {
            g_err = saved;  // a missing code object is not an error of the caller's call
        }
    }
    auto &slot = c->enc_spec[rb];
    slot = std::move(gs);
    return slot.empty() ? nullptr : &slot;
}

// HBRBC_SPEC_SPLIT=1: launch the specialised kernels pass by pass.
bool spec_pass_split() {
    const char *e = getenv("HBRBC_SPEC_SPLIT");
    return e && !std::strcmp(e, "1");
}

hipError_t launch_xor_group(const hbrbc_ctx::SpecGroup &g, bool fused, int rt, XorArgs a,
                            size_t count, hipStream_t s) {
    a.waves_per_row = (a.row_bytes + 64 * 32 - 1) / (64 * 32);
    const size_t blocks = (size_t)a.waves_per_row * count;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const int npass = (g.r_hi - g.r_lo + rt - 1) / rt;
    void *args[] = {&a.base,     &a.inst_stride, &a.shard_stride, &a.block_stride,
                    &a.row_bytes, &a.waves_per_row, &a.payloads,  &a.payload_stride,
                    &a.P,        &a.S,           &a.pat,          &a.slot_hash,
                    &a.hash_slots, &a.p_only,     &a.uf_payload,   &a.uf_stride,
                    &a.uf_status};
    hipFunction_t fn = fused ? g.fe : g.fn;
    // HBRBC_SPEC_SPLIT applies to the streaming form only: a wave of the LDS
    // form loads just its share of each stage's inputs
    if (!spec_pass_split() || g.lds) {
        a.p_only = -1;
        const unsigned threads = 64u * (unsigned)xor_waves(npass);
        return hipModuleLaunchKernel(fn, (unsigned)blocks, 1, 1, threads, 1, 1, 0, s, args, nullptr);
    }
    // one launch per pass, one wave per workgroup: every wave on the chip
    // runs the same pass's code (the three-pass N = 64 program is 151 KB of
    // straight-line code, more than the instruction cache a CU pair shares)
    for (a.p_only = 0; a.p_only < npass; ++a.p_only) {
        const hipError_t e = hipModuleLaunchKernel(fn, (unsigned)blocks, 1, 1, 64u, 1, 1, 0, s, args,
                                                   nullptr);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// The programs of a matrix split over several code objects (N = 250: four
// groups of output rows) read the same input rows.  Launched one after the
// other, each streams every instance's inputs from HBM again (cfg5: 1.95x /
// 2.29x the algorithmic bytes, profiles/pmc_traffic.json); launched
// concurrently on side streams they walk the instances together, so each
// input row is fetched once and served to the other programs from L2 /
// MALL -- in theory; measured flat (cfg5 encode 11.9 vs 12.1 ms, reconstruct
// 11.2 vs 11.5 ms, r3), so HBRBC_XOR_STREAMS=1 enables it for A/B only.
bool xor_streams() {   // measured no gain (cfg5 73.7 vs 73.2 GB/s, r3): off by default
    const char *e = getenv("HBRBC_XOR_STREAMS");
    return e && !std::strcmp(e, "1");
}

// HBRBC_XOR_TILE=T (A/B): the programs of a split matrix walk the instances
// T at a time (all programs over instances [i, i + T), then the next T), so
// the T instances' input rows stay in the Infinity Cache between programs.
size_t xor_tile() {
    const char *e = getenv("HBRBC_XOR_TILE");
    return e ? (size_t)atoll(e) : 0;
}

hipError_t launch_groups(hbrbc_ctx *c, const std::vector<hbrbc_ctx::SpecGroup> &gs, size_t first,
                         int rt, const XorArgs &x, size_t count, hipStream_t s) {
    const size_t ng = gs.size() - first;
    if (ng == 0) return hipSuccess;
    const size_t tile = xor_tile();
    if (ng > 1 && tile && count > tile) {
        for (size_t i0 = 0; i0 < count; i0 += tile) {
            XorArgs y = x;
            y.base = x.base + i0 * x.inst_stride;
            if (y.payloads) y.payloads = x.payloads + i0 * x.payload_stride;
            if (y.pat) y.pat = x.pat + i0;
            if (y.uf_payload) y.uf_payload = x.uf_payload + i0 * x.uf_stride;
            if (y.uf_status) y.uf_status = x.uf_status + i0;
            const size_t cnt = std::min(tile, count - i0);
            for (size_t i = first; i < gs.size(); ++i) {
                const hipError_t e = launch_xor_group(gs[i], false, rt, y, cnt, s);
                if (e != hipSuccess) return e;
            }
        }
        return hipSuccess;
    }
    if (ng == 1 || !xor_streams()) {
        for (size_t i = first; i < gs.size(); ++i) {
            const hipError_t e = launch_xor_group(gs[i], false, rt, x, count, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    while (c->side.size() < ng) {
        hipStream_t q;
        hipError_t e = hipStreamCreateWithFlags(&q, hipStreamNonBlocking);
        if (e != hipSuccess) return e;
        c->side.push_back(q);
    }
    while (c->side_ev.size() < ng + 1) {
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        c->side_ev.push_back(ev);
    }
    hipError_t e = hipEventRecord(c->side_ev[ng], s);   // inputs ready on s
    for (size_t i = 0; i < ng && e == hipSuccess; ++i) {
        e = hipStreamWaitEvent(c->side[i], c->side_ev[ng], 0);
        if (e == hipSuccess) e = launch_xor_group(gs[first + i], false, rt, x, count, c->side[i]);
        if (e == hipSuccess) e = hipEventRecord(c->side_ev[i], c->side[i]);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, c->side_ev[i], 0);
    }
    return e;
}

std::once_flag g_default_once;
hbrbc_ctx *g_default = nullptr;
int g_default_status = HBRBC_OK;

hbrbc_ctx *default_ctx(int *st) {
    std::call_once(g_default_once, [] { g_default_status = hbrbc_coding_new(1, 0, -1, &g_default); });
    *st = g_default_status;
    return g_default;
}

// Generic (bit-sliced) encode of parity rows k..n-1 in the given layout.
int generic_encode(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, const RowMap &rows,
                   size_t inst_stride, size_t count, hipStream_t s) {
    GfApplyArgs g{};
    g.base = shards;
    g.inst_stride = inst_stride;
    g.rows = rows;
    g.n16 = (int)((shard_len + 15) / 16);
    g.coefs = c->d_enc_coefs.as<uint8_t>();
    g.coef_slot_stride = 0;
    g.in_idx = c->d_enc_in.as<uint32_t>();
    g.in_idx_stride = 0;
    g.out_idx = c->d_enc_out.as<uint32_t>();
    g.out_idx_stride = 0;
    g.nout = nullptr;
    g.nout_uniform = (int)c->m;
    g.pat = nullptr;
    g.max_rows = (int)c->m;
    g.nin = (int)c->k;
    g.rt = c->rt_enc;
    g.mode = c->gf_mode;
    g.count = count;
    HB_HIP(launch_gf_apply(g, s));
    return HBRBC_OK;
}

int encode_rows(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, const RowMap &rows,
                size_t inst_stride, size_t count, hipStream_t s) {
    StageTimer t(c, HBRBC_STAGE_ENCODE, s);
    if (const auto *gs = spec_encoder(c, code_rb(rows))) {
        // specialised XOR networks (jit.hip), one launch per parity-row group
        XorArgs x{};
        x.base = shards;
        x.inst_stride = inst_stride;
        x.shard_stride = rows.sst;
        x.block_stride = rows.bst;
        x.row_bytes = (unsigned)round_up(shard_len, 16);
        x.p_only = -1;
        HB_HIP(launch_groups(c, *gs, 0, c->rt_spec, x, count, s));
        return HBRBC_OK;
    }
    if (jit_mode() == JIT_LOAD && c->k * c->m <= 16384)
        return fail(HBRBC_E_INVALID_ARG, "HBRBC_JIT=load: %s", c->jit_missing.c_str());
    return generic_encode(c, shards, shard_len, rows, inst_stride, count, s);
}

int frame_rows(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride, size_t payload_len,
               size_t count, uint8_t *shards, size_t shard_len, const RowMap &rows,
               size_t inst_stride, hipStream_t s) {
    StageTimer t(c, HBRBC_STAGE_FRAME, s);
    HB_HIP(launch_frame(payloads, payload_stride, payload_len, count, shards, shard_len, rows,
                        inst_stride, c->k, s));
    return HBRBC_OK;
}

int check_payloads(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride,
                   size_t payload_len, size_t shard_len) {
    if (shard_len != hbrbc_shard_len(payload_len, c->k))
        return fail(HBRBC_E_INVALID_ARG, "shard_len %zu != ceil((%zu+4)/%zu)", shard_len,
                    payload_len, c->k);
    if (payload_len > 0xFFFFFFFFull) return fail(HBRBC_E_INVALID_ARG, "payload too large");
    if (payload_len && (!payloads || reinterpret_cast<uintptr_t>(payloads) % 4 ||
                        payload_stride % 4 || payload_stride < round_up(payload_len, 4)))
        return fail(HBRBC_E_INVALID_ARG, "payload buffer must be 4-byte aligned with stride >= "
                                         "round_up(len, 4)");
    return HBRBC_OK;
}

int decode_rows(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, const RowMap &rows,
                size_t inst_stride, const uint8_t *present, size_t count, const uint8_t *roots,
                size_t root_stride, uint8_t *nodes, size_t node_inst_stride, bool known_leaves,
                uint8_t *payload_out, size_t payload_stride, uint32_t *payload_len_out,
                int32_t *status_out, hipStream_t s) {
    int st = ensure_workspace(c, count);
    if (st) return st;
    int32_t *rstat = c->ws_status.as<int32_t>();
    bool fused = false;
    const bool fusable = unframe_fusable(c, shard_len, payload_stride);
    st = run_reconstruct(c, shards, shard_len, rows, inst_stride, present, count, rstat, s,
                         fusable ? payload_out : nullptr, payload_stride, &fused);
    if (st) return st;
    st = run_merkle(c, shards, shard_len, rows, inst_stride, c->n, count, nodes, node_inst_stride,
                    known_leaves, s);
    if (st) return st;
    StageTimer t(c, HBRBC_STAGE_UNFRAME, s);
    HB_HIP(launch_decode_check(rstat, nodes, node_inst_stride, hbrbc_merkle_node_count(c->n) - 1,
                               roots, root_stride, shards, shard_len, rows, inst_stride, c->k,
                               count, payload_len_out, status_out, s));
    if (fused)
        HB_HIP(launch_unframe_fixup(shards, (uint32_t)shard_len, rows, inst_stride, (uint32_t)c->k,
                                    count, payload_len_out, status_out, payload_out,
                                    payload_stride, s));
    else
        HB_HIP(launch_unframe(shards, shard_len, rows, inst_stride, c->k, count, payload_len_out,
                              status_out, payload_out, payload_stride, s));
    return HBRBC_OK;
}

}  // namespace

// =========================================================================
extern "C" {

const char *hbrbc_last_error(void) { return g_err.c_str(); }
// hbrbc_version() lives in version.cpp (built with the source hash)

int hbrbc_coding_new(size_t data_shards, size_t parity_shards, int device, hbrbc_ctx **out) {
    if (!out) return fail(HBRBC_E_INVALID_ARG, "out is null");
    *out = nullptr;
    // rse ReedSolomon::new checks (Coding::new only calls it when parity > 0)
    if (data_shards == 0) return fail(HBRBC_E_TOO_FEW_DATA_SHARDS, "no data shards");
    if (data_shards + parity_shards > 256)
        return fail(HBRBC_E_TOO_MANY_SHARDS, "data + parity = %zu > 256",
                    data_shards + parity_shards);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    if (device < 0) HB_HIP(hipGetDevice(&device));
    if (device >= ndev) return fail(HBRBC_E_NO_DEVICE, "device %d of %d", device, ndev);
    HB_HIP(hipSetDevice(device));
    static std::once_flag cfg_once;
    static hipError_t cfg_err = hipSuccess;
    std::call_once(cfg_once, [] { cfg_err = configure_kernels(); });
    HB_HIP(cfg_err);

    hbrbc_ctx *c = new hbrbc_ctx();
    c->device = device;
    c->k = data_shards;
    c->m = parity_shards;
    c->n = data_shards + parity_shards;
    c->rt_enc = gf_row_tile((int)c->m);
    // reconstruct rebuilds f..2f rows per instance in hbbft (f random
    // erasures typical).  A workgroup runs up to 4 waves over the same byte
    // positions, one pass of rt rows each, so tile the typical count into ~4
    // passes (measured at N=64: rt 6 -> 3.05 ms, 8 -> 3.3, 12 -> 3.55 per
    // 16384 instances), but not below 6 rows, where the per-pass transposes
    // and doublings stop amortising.
    {
        const int h = (int)((c->m + 1) / 2);
        int rt = ((h + 3) / 4 + 1) & ~1;
        if (rt < 6) rt = (h + 1) & ~1;
        c->rt_rec = std::max(2, std::min(16, std::max(rt, std::min(6, (h + 1) & ~1))));
        // 7-row passes where they save a pass (N=64: 21 rows in 7, 7, 7 instead
        // of 6, 6, 6, 3; reconstruct 3.61 -> 3.44 ms per step, round 3)
        if (c->rt_rec == 6 && (h + 6) / 7 < (h + 5) / 6) c->rt_rec = 7;
        // and 7-row passes up to N=128 (h = 42: 12 -> 7, 3.45 -> 3.06 ms; 10: 3.17)
        if (h >= 14 && h <= 42) c->rt_rec = 7;
    }
    if (const char *e = getenv("HBRBC_GF")) {
        // bitslice (uniform branches), bitslice_likely (set-bit path inline),
        // bitslice_mask (branch-free masked xor)
        if (!std::strcmp(e, "bitslice_likely")) c->gf_mode = 1;
        else if (!std::strcmp(e, "bitslice_mask")) c->gf_mode = 2;
        else if (!std::strcmp(e, "bitslice_pair")) c->gf_mode = 3;
        else if (!std::strcmp(e, "bitslice_x2")) c->gf_mode = 4;
        else c->gf_mode = 0;
    }
    if (const char *e = getenv("HBRBC_RT_ENC")) c->rt_enc = std::max(2, std::min(16, atoi(e) & ~1));
    // (5 and 7 are instantiated too: A/B of odd tiles, e.g. 21 rows in 3 passes of 7)
    if (const char *e = getenv("HBRBC_RT_REC")) {
        const int r = atoi(e);
        c->rt_rec = (r == 5 || r == 7) ? r : std::max(2, std::min(16, r & ~1));
    }
    if (!build_matrix(c->k, c->n, c->matrix)) {
        delete c;
        return fail(HBRBC_E_SINGULAR_MATRIX, "singular Vandermonde top block");
    }
    int st = HBRBC_OK;
    auto guard = [&](hipError_t e) {
        if (e != hipSuccess && st == HBRBC_OK)
            st = fail(HBRBC_E_DEVICE, "context setup: %s", hipGetErrorString(e));
    };
    guard(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    guard(c->d_matrix.ensure(c->matrix.size()));
    if (st == HBRBC_OK)
        guard(hipMemcpy(c->d_matrix.p, c->matrix.data(), c->matrix.size(), hipMemcpyHostToDevice));
    if (c->m > 0 && st == HBRBC_OK) {
        // pass-major coefficient bytes [pass][j][16], zero-padded rows
        const size_t rt = (size_t)c->rt_enc, npass = (c->m + rt - 1) / rt;
        std::vector<uint8_t> tab(npass * c->k * 16, 0);
        for (size_t r = 0; r < c->m; ++r)
            for (size_t j = 0; j < c->k; ++j)
                tab[((r / rt) * c->k + j) * 16 + (r % rt)] = c->matrix[(c->k + r) * c->k + j];
        std::vector<uint32_t> in(c->k), outi(c->m);
        for (size_t j = 0; j < c->k; ++j) in[j] = (uint32_t)j;
        for (size_t r = 0; r < c->m; ++r) outi[r] = (uint32_t)(c->k + r);
        guard(c->d_enc_coefs.ensure(tab.size()));
        guard(c->d_enc_in.ensure(in.size() * sizeof(uint32_t)));
        guard(c->d_enc_out.ensure(outi.size() * sizeof(uint32_t)));
        if (st == HBRBC_OK) {
            guard(hipMemcpy(c->d_enc_coefs.p, tab.data(), tab.size(), hipMemcpyHostToDevice));
            guard(hipMemcpy(c->d_enc_in.p, in.data(), in.size() * sizeof(uint32_t),
                            hipMemcpyHostToDevice));
            guard(hipMemcpy(c->d_enc_out.p, outi.data(), outi.size() * sizeof(uint32_t),
                            hipMemcpyHostToDevice));
        }
    }
    if (st != HBRBC_OK) {
        hbrbc_coding_free(c);
        return st;
    }
    c->rt_spec = spec_row_tile(c->k, c->m);
    c->depth_spec = spec_depth();
    c->enc_kind = c->m == 0 ? "trivial" : (spec_encoder(c, 256) ? "specialised" : "bitslice");
    if (c->m > 0 && c->enc_kind == "bitslice") {
        if (jit_mode() == JIT_COMPILE && c->k * c->m <= 16384) c->enc_kind = "jit-failed";
        if (jit_mode() == JIT_LOAD && c->k * c->m <= 16384) {
            const std::string msg = c->jit_missing;
            hbrbc_coding_free(c);
            return fail(HBRBC_E_INVALID_ARG, "HBRBC_JIT=load: %s", msg.c_str());
        }
    }
    *out = c;
    return HBRBC_OK;
}

void hbrbc_coding_free(hbrbc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (DevBuf *b : {&c->d_matrix, &c->d_enc_coefs, &c->d_enc_in, &c->d_enc_out, &c->pc_hash,
                      &c->pc_keys, &c->pc_coefs, &c->pc_in, &c->pc_out, &c->pc_nout, &c->pc_status,
                      &c->pc_fill, &c->ws_pat, &c->ws_own, &c->ws_status, &c->ws_list,
                      &c->ws_counter, &c->st_slab, &c->st_nodes, &c->st_aux})
        b->release();
    c->pin.release();
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->side_ev) (void)hipEventDestroy(e);
    for (hipStream_t q : c->side) (void)hipStreamDestroy(q);
    for (auto &kv : c->enc_spec) drop_groups(kv.second);
    for (auto &kv : c->dec_spec) {
        drop_groups(kv.second.groups);
        drop_groups(kv.second.uf_groups);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

size_t hbrbc_data_shard_count(const hbrbc_ctx *c) { return c ? c->k : 0; }
size_t hbrbc_parity_shard_count(const hbrbc_ctx *c) { return c ? c->m : 0; }
void *hbrbc_stream(const hbrbc_ctx *c) { return c ? c->stream : nullptr; }

int hbrbc_encoding_matrix(const hbrbc_ctx *c, uint8_t *out) {
    if (!c || !out) return fail(HBRBC_E_INVALID_ARG, "null argument");
    std::memcpy(out, c->matrix.data(), c->matrix.size());
    return HBRBC_OK;
}

size_t hbrbc_shard_len(size_t payload_len, size_t data_shards) {
    return data_shards ? (payload_len + 4 + data_shards - 1) / data_shards : 0;
}

size_t hbrbc_merkle_node_count(size_t n) {
    size_t total = 0, sz = n;
    for (;;) {
        total += sz;
        if (sz <= 1) break;
        sz = (sz + 1) / 2;
    }
    return total;
}

size_t hbrbc_merkle_max_proof_len(size_t n) {
    size_t d = 0, sz = n;
    while (sz > 1) {
        ++d;
        sz = (sz + 1) / 2;
    }
    return d;
}

// ---------------------------------------------------------------- layer 2 --
int hbrbc_frame_batch(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride,
                      size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                      size_t shard_stride, size_t inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    int st = check_payloads(c, payloads, payload_stride, payload_len, shard_len);
    if (st) return st;
    st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    return frame_rows(c, payloads, payload_stride, payload_len, count, shards, shard_len,
                      plain_rows(shard_stride), inst_stride, pick(c, stream));
}

int hbrbc_encode_batch(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                       size_t inst_stride, size_t count, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (c->m == 0 || count == 0) return HBRBC_OK;  // Coding::Trivial::encode
    if (shard_len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shards");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    return encode_rows(c, shards, shard_len, plain_rows(shard_stride), inst_stride, count,
                       pick(c, stream));
}

int hbrbc_frame_encode_rows(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride,
                            size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                            size_t shard_stride, size_t rows_per_block, size_t block_stride,
                            size_t inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    int st = check_payloads(c, payloads, payload_stride, payload_len, shard_len);
    if (st) return st;
    st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count, rows_per_block,
                    block_stride);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    const RowMap rows = make_rows(c->n, shard_stride, rows_per_block, block_stride);
    const std::vector<hbrbc_ctx::SpecGroup> *gs = nullptr;
    if (c->m > 0 && shard_stride == round_up(shard_len, 16) && payload_len <= 0x7FFFFFFFull &&
        shard_len * c->k < 0x7FFFFFFFull) {
        gs = spec_encoder(c, code_rb(rows));
        // only a call the specialised encoder could serve fails on a missing
        // code object; the others take the generic encoder below
        if (!gs && jit_mode() == JIT_LOAD && c->k * c->m <= 16384)
            return fail(HBRBC_E_INVALID_ARG, "HBRBC_JIT=load: %s", c->jit_missing.c_str());
    }
    const char *fe = getenv("HBRBC_FUSE");   // 0: frame kernel + encoder (A/B)
    if (!gs || (fe && !std::strcmp(fe, "0"))) {
        st = frame_rows(c, payloads, payload_stride, payload_len, count, shards, shard_len, rows,
                        inst_stride, s);
        if (st || c->m == 0) return st;
        return encode_rows(c, shards, shard_len, rows, inst_stride, count, s);
    }
    StageTimer t(c, HBRBC_STAGE_ENCODE, s);
    // frame folded into the specialised encoder (jit.hip): group 0's twin
    // writes the framed data rows and its parity rows, the fixup adds the
    // last partial payload dword to both, and the other groups then encode
    // from the complete data rows
    XorArgs x{};
    x.base = shards;
    x.inst_stride = inst_stride;
    x.shard_stride = rows.sst;
    x.block_stride = rows.bst;
    x.row_bytes = (unsigned)shard_stride;
    x.payloads = payloads;
    x.payload_stride = payload_stride;
    x.P = (unsigned)payload_len;
    x.S = (unsigned)shard_len;
    x.p_only = -1;
    const auto &g0 = gs->front();
    HB_HIP(launch_xor_group(g0, true, c->rt_spec, x, count, s));
    HB_HIP(launch_frame_fixup(payloads, payload_stride, payload_len, shards, shard_len, rows,
                              inst_stride, c->k, (size_t)g0.r_hi, c->d_matrix.as<uint8_t>(), count,
                              s));
    HB_HIP(launch_groups(c, *gs, 1, c->rt_spec, x, count, s));
    return HBRBC_OK;
}

int hbrbc_frame_encode_batch(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride,
                             size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                             size_t shard_stride, size_t inst_stride, void *stream) {
    return hbrbc_frame_encode_rows(c, payloads, payload_stride, payload_len, count, shards,
                                   shard_len, shard_stride, 0, 0, inst_stride, stream);
}

int hbrbc_frame_encode_ragged(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride,
                              const uint32_t *payload_lens, size_t max_payload_len, size_t count,
                              uint8_t *shards, size_t shard_stride, size_t inst_stride,
                              void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!payload_lens) return fail(HBRBC_E_INVALID_ARG, "null payload_lens");
    const size_t smax = hbrbc_shard_len(max_payload_len, c->k);
    if (shard_stride < round_up(smax, 16))
        return fail(HBRBC_E_INVALID_ARG, "shard_stride %zu < round_up(%zu, 16)", shard_stride, smax);
    int st = check_payloads(c, payloads, payload_stride, max_payload_len, smax);
    if (st) return st;
    st = check_slab(shards, shard_stride, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    const RowMap rows = plain_rows(shard_stride);
    {
        StageTimer t(c, HBRBC_STAGE_FRAME, s);
        HB_HIP(launch_frame(payloads, payload_stride, max_payload_len, count, shards, smax, rows,
                            inst_stride, c->k, s, payload_lens, shard_stride));
    }
    if (c->m == 0) return HBRBC_OK;
    // rows are zero past each instance's shard: one encode over the common row length
    return encode_rows(c, shards, shard_stride, rows, inst_stride, count, s);
}

int hbrbc_merkle_ragged(hbrbc_ctx *c, const uint8_t *shards, const uint32_t *shard_lens,
                        size_t shard_stride, size_t inst_stride, size_t count, uint8_t *nodes,
                        size_t node_inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!shard_lens) return fail(HBRBC_E_INVALID_ARG, "null shard_lens");
    int st = check_slab(shards, shard_stride, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    st = check_nodes(nodes, node_inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    if (merkle_fused_ok(c->n) && !merkle_split()) {
        StageTimer t(c, HBRBC_STAGE_LEAF_HASH, s);
        HB_HIP(launch_merkle_fused(shards, shard_stride, plain_rows(shard_stride), inst_stride,
                                   c->n, count, nodes, node_inst_stride, s, shard_lens));
        return HBRBC_OK;
    }
    {
        StageTimer t(c, HBRBC_STAGE_LEAF_HASH, s);
        HB_HIP(launch_leaf_hash(shards, shard_stride, plain_rows(shard_stride), inst_stride, c->n,
                                count, nodes, node_inst_stride, s, shard_lens));
    }
    StageTimer t(c, HBRBC_STAGE_TREE_LEVELS, s);
    size_t off = 0, sz = c->n;
    while (sz > 1) {
        const size_t nsz = (sz + 1) / 2;
        HB_HIP(launch_tree_level(nodes, node_inst_stride, off, sz, off + sz, nsz, count, s));
        off += sz;
        sz = nsz;
    }
    return HBRBC_OK;
}

int hbrbc_merkle_rows(hbrbc_ctx *c, const uint8_t *shards, size_t shard_len, size_t shard_stride,
                      size_t rows_per_block, size_t block_stride, size_t inst_stride, size_t count,
                      uint8_t *nodes, size_t node_inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count, rows_per_block,
                        block_stride);
    if (st) return st;
    st = check_nodes(nodes, node_inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    return run_merkle(c, shards, shard_len,
                      make_rows(c->n, shard_stride, rows_per_block, block_stride), inst_stride,
                      c->n, count, nodes, node_inst_stride, false, pick(c, stream));
}

int hbrbc_merkle_batch(hbrbc_ctx *c, const uint8_t *shards, size_t shard_len,
                       size_t shard_stride, size_t inst_stride, size_t count, uint8_t *nodes,
                       size_t node_inst_stride, void *stream) {
    return hbrbc_merkle_rows(c, shards, shard_len, shard_stride, 0, 0, inst_stride, count, nodes,
                             node_inst_stride, stream);
}

int hbrbc_proofs_batch(hbrbc_ctx *c, const uint8_t *nodes, size_t node_inst_stride, size_t count,
                       uint8_t *digests, uint8_t *ndig, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    int st = check_nodes(nodes, node_inst_stride, c->n, count);
    if (st) return st;
    const size_t dslots = hbrbc_merkle_max_proof_len(c->n);
    if (!ndig || (dslots && (!digests || reinterpret_cast<uintptr_t>(digests) % 16)))
        return fail(HBRBC_E_INVALID_ARG, "digest buffers must be non-null, 16-byte aligned");
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    StageTimer t(c, HBRBC_STAGE_PROOFS, s);
    HB_HIP(launch_proofs(nodes, node_inst_stride, c->n, count, digests, dslots, ndig, s));
    return HBRBC_OK;
}

int hbrbc_validate_rows(hbrbc_ctx *c, const uint8_t *values, size_t value_len,
                        size_t value_stride, size_t rows_per_block, size_t block_stride,
                        size_t value_inst_stride, size_t per_inst, const uint32_t *rows,
                        const uint32_t *indices, const uint8_t *digests, const uint8_t *ndig,
                        size_t digest_rows, const uint8_t *roots, size_t root_stride,
                        size_t tree_n, size_t count, uint8_t *ok_out, uint8_t *leaf_out,
                        size_t leaf_inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0 || per_inst == 0) return HBRBC_OK;
    if (!values || reinterpret_cast<uintptr_t>(values) % 8 || value_stride % 8 ||
        value_inst_stride % 8 || block_stride % 8)
        return fail(HBRBC_E_INVALID_ARG, "values must be 8-byte aligned with 8-byte strides");
    if (!ndig || !roots || !ok_out || reinterpret_cast<uintptr_t>(roots) % 16 || root_stride % 16)
        return fail(HBRBC_E_INVALID_ARG, "roots must be 16-byte aligned; outputs non-null");
    if (tree_n == 0 || tree_n > 0xFFFFFFFFull || value_len > 0xFFFFFFFFull)
        return fail(HBRBC_E_INVALID_ARG, "bad tree_n / value_len");
    if (rows_per_block > 255 && rows_per_block < tree_n)
        return fail(HBRBC_E_INVALID_ARG, "rows_per_block %zu > 255", rows_per_block);
    if (rows && digest_rows == 0)
        return fail(HBRBC_E_INVALID_ARG, "a row list needs digest_rows > every listed row");
    if (leaf_out && (reinterpret_cast<uintptr_t>(leaf_out) % 16 || leaf_inst_stride % 16))
        return fail(HBRBC_E_INVALID_ARG, "leaf_out must be 16-byte aligned");
    const size_t dslots = hbrbc_merkle_max_proof_len(tree_n);
    if (dslots && (!digests || reinterpret_cast<uintptr_t>(digests) % 16))
        return fail(HBRBC_E_INVALID_ARG, "digests must be 16-byte aligned");
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    StageTimer t(c, HBRBC_STAGE_VALIDATE, s);
    ValidateArgs a;
    a.values = values;
    a.value_len = value_len;
    a.value_inst_stride = value_inst_stride;
    a.per_inst = per_inst;
    a.vrows = make_rows(tree_n, value_stride, rows_per_block, block_stride);
    a.rows = rows;
    a.indices = indices;
    a.digests = digests;
    a.dslots = dslots;
    a.dig_rows = rows ? digest_rows : per_inst;
    a.ndig = ndig;
    a.roots = roots;
    a.root_stride = root_stride;
    a.tree_n = tree_n;
    a.count = count;
    a.ok_out = ok_out;
    a.leaf_out = leaf_out;
    a.leaf_inst_stride = leaf_inst_stride;
    HB_HIP(launch_validate(a, s));
    return HBRBC_OK;
}

int hbrbc_validate_batch(hbrbc_ctx *c, const uint8_t *values, size_t value_len,
                         size_t value_stride, size_t value_inst_stride, size_t per_inst,
                         const uint32_t *indices, const uint8_t *digests, const uint8_t *ndig,
                         const uint8_t *roots, size_t root_stride, size_t tree_n, size_t count,
                         uint8_t *ok_out, void *stream) {
    return hbrbc_validate_rows(c, values, value_len, value_stride, 0, 0, value_inst_stride,
                               per_inst, nullptr, indices, digests, ndig, per_inst, roots,
                               root_stride, tree_n, count, ok_out, nullptr, 0, stream);
}

int hbrbc_reserve(hbrbc_ctx *c, size_t count) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    HB_HIP(hipSetDevice(c->device));
    return ensure_workspace(c, count);
}

int hbrbc_reconstruct_rows(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                           size_t rows_per_block, size_t block_stride, size_t inst_stride,
                           const uint8_t *present, size_t count, int32_t *status_out,
                           void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!present || !status_out) return fail(HBRBC_E_INVALID_ARG, "null present/status");
    if (c->m > 0 && shard_len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shards");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count, rows_per_block,
                        block_stride);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    return run_reconstruct(c, shards, shard_len,
                           make_rows(c->n, shard_stride, rows_per_block, block_stride),
                           inst_stride, present, count, status_out, pick(c, stream));
}

int hbrbc_reconstruct_batch(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                            size_t inst_stride, const uint8_t *present, size_t count,
                            int32_t *status_out, void *stream) {
    return hbrbc_reconstruct_rows(c, shards, shard_len, shard_stride, 0, 0, inst_stride, present,
                                  count, status_out, stream);
}

int hbrbc_decode_rows(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                      size_t rows_per_block, size_t block_stride, size_t inst_stride,
                      const uint8_t *present, size_t count, const uint8_t *roots,
                      size_t root_stride, uint8_t *nodes, size_t node_inst_stride,
                      int known_leaves, uint8_t *payload_out, size_t payload_stride,
                      uint32_t *payload_len_out, int32_t *status_out, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!present || !status_out || !payload_len_out || !roots)
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(roots) % 16 || root_stride % 16)
        return fail(HBRBC_E_INVALID_ARG, "roots must be 16-byte aligned");
    if (shard_len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shards");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count, rows_per_block,
                        block_stride);
    if (st) return st;
    st = check_nodes(nodes, node_inst_stride, c->n, count);
    if (st) return st;
    const size_t total = c->k * shard_len;
    const size_t need = total >= 4 ? round_up(total - 4, 16) : 0;  // 16-byte output chunks
    if (need && (!payload_out || reinterpret_cast<uintptr_t>(payload_out) % 4 ||
                 payload_stride % 4 || (count > 1 && payload_stride < need)))
        return fail(HBRBC_E_INVALID_ARG, "payload_out stride must be a multiple of 4 and >= %zu",
                    need);
    HB_HIP(hipSetDevice(c->device));
    return decode_rows(c, shards, shard_len,
                       make_rows(c->n, shard_stride, rows_per_block, block_stride), inst_stride,
                       present, count, roots, root_stride, nodes, node_inst_stride,
                       known_leaves != 0, payload_out, payload_stride, payload_len_out,
                       status_out, pick(c, stream));
}

int hbrbc_decode_batch(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                       size_t inst_stride, const uint8_t *present, size_t count,
                       const uint8_t *roots, size_t root_stride, uint8_t *nodes,
                       size_t node_inst_stride, uint8_t *payload_out, size_t payload_stride,
                       uint32_t *payload_len_out, int32_t *status_out, void *stream) {
    return hbrbc_decode_rows(c, shards, shard_len, shard_stride, 0, 0, inst_stride, present, count,
                             roots, root_stride, nodes, node_inst_stride, 0, payload_out,
                             payload_stride, payload_len_out, status_out, stream);
}

int hbrbc_drop_rows(hbrbc_ctx *c, uint8_t *shards, size_t shard_stride, size_t rows_per_block,
                    size_t block_stride, size_t inst_stride, const uint8_t *present, size_t count,
                    uint8_t fill, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!present) return fail(HBRBC_E_INVALID_ARG, "null present flags");
    int st = check_slab(shards, shard_stride, shard_stride, inst_stride, c->n, count,
                        rows_per_block, block_stride);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    HB_HIP(launch_drop_rows(shards, shard_stride,
                            make_rows(c->n, shard_stride, rows_per_block, block_stride),
                            inst_stride, c->n, count, present, fill, pick(c, stream)));
    return HBRBC_OK;
}

// ---------------------------------------------------- decode-matrix cache --
int hbrbc_decode_cache_clear(hbrbc_ctx *c) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (!c->pc_cap) return HBRBC_OK;
    HB_HIP(hipSetDevice(c->device));
    HB_HIP(hipDeviceSynchronize());
    HB_HIP(hipMemset(c->pc_hash.p, 0, (size_t)c->pc_cap * sizeof(uint64_t)));
    HB_HIP(hipMemset(c->pc_fill.p, 0, sizeof(uint32_t)));
    c->pc_inserted = 0;
    return HBRBC_OK;
}

int hbrbc_decode_cache_fill(hbrbc_ctx *c, uint32_t *patterns_out) {
    if (!c || !patterns_out) return fail(HBRBC_E_INVALID_ARG, "null argument");
    *patterns_out = 0;
    if (!c->pc_cap) return HBRBC_OK;
    HB_HIP(hipSetDevice(c->device));
    HB_HIP(hipDeviceSynchronize());
    HB_HIP(hipMemcpy(patterns_out, c->pc_fill.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return HBRBC_OK;
}

int hbrbc_decoder_specialise(hbrbc_ctx *c, const uint8_t *present, size_t rows_per_block) {
    if (!c || !present) return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (c->m == 0) return HBRBC_OK;  // Coding::Trivial rebuilds nothing
    HB_HIP(hipSetDevice(c->device));
    const int rb = (rows_per_block && rows_per_block < c->n) ? (int)rows_per_block : 256;
    if (rb > 255 && rb != 256) return fail(HBRBC_E_INVALID_ARG, "rows_per_block > 255");
    std::vector<XorProgram> progs;
    uint64_t hash = 0;
    int rt = 2;
    if (!decode_programs(c->matrix, c->k, c->n, present, rb, progs, hash, rt))
        return fail(HBRBC_E_INVALID_ARG, "pattern has nothing to rebuild or too few shards");
    const bool compile = jit_mode() == JIT_DEFAULT || jit_mode() == JIT_COMPILE;
    hbrbc_ctx::DecSpec d;
    d.hash = hash;
    d.rt = rt;
    d.present.assign(present, present + c->n);
    int ng = 0;
    for (const auto &p : progs) {
        hbrbc_ctx::SpecGroup g{0, (int)p.out_rows.size(), nullptr, nullptr, nullptr};
        (void)ng;
        const int st = load_program(p, compile, g);
        if (st) {
            drop_groups(d.groups);
            return st;
        }
        d.groups.push_back(g);
    }
    HB_HIP(hipDeviceSynchronize());  // no launch of the previous decoder is in flight
    auto it = c->dec_spec.find(rb);
    if (it != c->dec_spec.end()) {
        drop_groups(it->second.groups);
        drop_groups(it->second.uf_groups);
    }
    c->dec_spec[rb] = std::move(d);
    return HBRBC_OK;
}

size_t hbrbc_jit_decode_groups(size_t data_shards, size_t parity_shards, const uint8_t *present) {
    std::vector<uint8_t> mat;
    const size_t n = data_shards + parity_shards;
    if (!present || data_shards == 0 || n > 256 || !build_matrix(data_shards, n, mat)) return 0;
    std::vector<XorProgram> progs;
    uint64_t hash;
    int rt;
    return decode_programs(mat, data_shards, n, present, 256, progs, hash, rt) ? progs.size() : 0;
}

int hbrbc_jit_build_decode(size_t data_shards, size_t parity_shards, const uint8_t *present,
                           size_t rows_per_block, size_t group, const char *dir) {
    return hbrbc_jit_build_decode_variant(data_shards, parity_shards, present, rows_per_block,
                                          group, 0, dir);
}

int hbrbc_jit_build_decode_variant(size_t data_shards, size_t parity_shards,
                                   const uint8_t *present, size_t rows_per_block, size_t group,
                                   int fused_unframe, const char *dir) {
    std::vector<uint8_t> mat;
    const size_t n = data_shards + parity_shards;
    if (!present || data_shards == 0 || n > 256)
        return fail(HBRBC_E_INVALID_ARG, "need data >= 1, data + parity <= 256, a pattern");
    if (!build_matrix(data_shards, n, mat))
        return fail(HBRBC_E_SINGULAR_MATRIX, "singular Vandermonde top block");
    const int rb = (rows_per_block && rows_per_block < n) ? (int)rows_per_block : 256;
    std::vector<XorProgram> progs;
    uint64_t hash;
    int rt;
    if (!decode_programs(mat, data_shards, n, present, rb, progs, hash, rt, fused_unframe != 0))
        return fail(HBRBC_E_INVALID_ARG, "pattern has nothing to rebuild or too few shards");
    if (group >= progs.size()) return fail(HBRBC_E_INVALID_ARG, "group %zu of %zu", group, progs.size());
    std::vector<char> code;
    std::string log;
    if (compile_source(gen_xor_source(progs[group]), code, log))
        return fail(HBRBC_E_DEVICE, "hiprtc: %s", log.substr(0, 400).c_str());
    const std::string d = dir ? std::string(dir) : jit_dir();
    mkdir(d.c_str(), 0755);
    const std::string path = jit_file(d, progs[group].name);
    return write_file(path, code) ? HBRBC_OK
                                  : fail(HBRBC_E_INVALID_ARG, "cannot write %s", path.c_str());
}

// ---------------------------------------------------------------- layer 1 --
// The per-call shims stage through one pinned host buffer per context: one
// host-to-device DMA of everything the kernel reads, one device-to-host DMA
// of the results, one stream synchronisation (the shim mutex serialises
// calls that share the context's staging).
int hbrbc_encode(hbrbc_ctx *c, uint8_t *const *shards, const size_t *lens, size_t n_shards) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (c->m == 0) return HBRBC_OK;  // Coding::Trivial::encode -> Ok(())
    // rse check_piece_count!(all) then check_slices!(multi)
    if (n_shards < c->n) return fail(HBRBC_E_TOO_FEW_SHARDS, "%zu < %zu shards", n_shards, c->n);
    if (n_shards > c->n) return fail(HBRBC_E_TOO_MANY_SHARDS, "%zu > %zu shards", n_shards, c->n);
    if (!shards || !lens) return fail(HBRBC_E_INVALID_ARG, "null argument");
    const size_t len = lens[0];
    if (len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shard");
    for (size_t i = 0; i < n_shards; ++i)
        if (lens[i] != len) return fail(HBRBC_E_INCORRECT_SHARD_SIZE, "shard %zu length", i);
    std::lock_guard<std::mutex> lk(c->shim_mu);
    HB_HIP(hipSetDevice(c->device));
    const size_t stride = round_up(len, 16);
    HB_HIP(c->st_slab.ensure(c->n * stride));
    HB_HIP(c->pin.ensure(c->n * stride));
    uint8_t *slab = c->st_slab.as<uint8_t>(), *pin = c->pin.as<uint8_t>();
    for (size_t j = 0; j < c->k; ++j) {
        std::memcpy(pin + j * stride, shards[j], len);
        std::memset(pin + j * stride + len, 0, stride - len);
    }
    HB_HIP(hipMemcpyAsync(slab, pin, c->k * stride, hipMemcpyHostToDevice, c->stream));
    int st = encode_rows(c, slab, len, plain_rows(stride), c->n * stride, 1, c->stream);
    if (st) return st;
    HB_HIP(hipMemcpyAsync(pin + c->k * stride, slab + c->k * stride, c->m * stride,
                          hipMemcpyDeviceToHost, c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
    for (size_t r = c->k; r < c->n; ++r) std::memcpy(shards[r], pin + r * stride, len);
    return HBRBC_OK;
}

int hbrbc_reconstruct(hbrbc_ctx *c, uint8_t *const *shards, const size_t *lens,
                      const uint8_t *present, size_t n_shards) {
    if (!c || !present) return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (c->m == 0) {  // Coding::Trivial (broadcast.rs:685-690)
        for (size_t i = 0; i < n_shards; ++i)
            if (!present[i]) return fail(HBRBC_E_TOO_FEW_SHARDS_PRESENT, "trivial coding");
        return HBRBC_OK;
    }
    // rse reconstruct_internal: piece count, then lengths in index order
    if (n_shards < c->n) return fail(HBRBC_E_TOO_FEW_SHARDS, "%zu < %zu shards", n_shards, c->n);
    if (n_shards > c->n) return fail(HBRBC_E_TOO_MANY_SHARDS, "%zu > %zu shards", n_shards, c->n);
    if (!shards || !lens) return fail(HBRBC_E_INVALID_ARG, "null argument");
    size_t np = 0, len = 0;
    bool have = false;
    for (size_t i = 0; i < n_shards; ++i) {
        if (!present[i]) continue;
        if (lens[i] == 0) return fail(HBRBC_E_EMPTY_SHARD, "shard %zu empty", i);
        ++np;
        if (have && lens[i] != len) return fail(HBRBC_E_INCORRECT_SHARD_SIZE, "shard %zu", i);
        len = lens[i];
        have = true;
    }
    if (np == c->n) return HBRBC_OK;
    if (np < c->k) return fail(HBRBC_E_TOO_FEW_SHARDS_PRESENT, "%zu < %zu present", np, c->k);
    std::lock_guard<std::mutex> lk(c->shim_mu);
    HB_HIP(hipSetDevice(c->device));
    const size_t stride = round_up(len, 16);
    const size_t pres_off = c->n * stride, stat_off = round_up(pres_off + c->n, 16);
    HB_HIP(c->st_slab.ensure(stat_off + 16));
    HB_HIP(c->pin.ensure(stat_off + 16));
    uint8_t *slab = c->st_slab.as<uint8_t>(), *pin = c->pin.as<uint8_t>();
    for (size_t i = 0; i < c->n; ++i) {
        pin[pres_off + i] = present[i] ? 1 : 0;
        if (present[i]) std::memcpy(pin + i * stride, shards[i], len);
        else std::memset(pin + i * stride, 0, len);
        std::memset(pin + i * stride + len, 0, stride - len);
    }
    HB_HIP(hipMemcpyAsync(slab, pin, pres_off + c->n, hipMemcpyHostToDevice, c->stream));
    int32_t *dstat = reinterpret_cast<int32_t *>(slab + stat_off);
    int st = run_reconstruct(c, slab, len, plain_rows(stride), c->n * stride, slab + pres_off, 1,
                             dstat, c->stream);
    if (st) return st;
    HB_HIP(hipMemcpyAsync(pin + stat_off, dstat, sizeof(int32_t), hipMemcpyDeviceToHost,
                          c->stream));
    for (size_t i = 0; i < c->n; ++i)
        if (!present[i])
            HB_HIP(hipMemcpyAsync(pin + i * stride, slab + i * stride, len, hipMemcpyDeviceToHost,
                                  c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
    int32_t status = 0;
    std::memcpy(&status, pin + stat_off, sizeof status);
    if (status) return fail(status, "reconstruct status %d", status);
    for (size_t i = 0; i < c->n; ++i)
        if (!present[i]) std::memcpy(shards[i], pin + i * stride, len);
    return HBRBC_OK;
}

int hbrbc_merkle_build(const uint8_t *const *values, const size_t *lens, size_t n,
                       uint8_t *nodes_out) {
    if (n == 0) return fail(HBRBC_E_INVALID_ARG, "MerkleTree over zero values");
    if (!values || !lens || !nodes_out) return fail(HBRBC_E_INVALID_ARG, "null argument");
    int st;
    hbrbc_ctx *c = default_ctx(&st);
    if (st) return st;
    std::lock_guard<std::mutex> lk(c->shim_mu);
    HB_HIP(hipSetDevice(c->device));
    // pinned image: [offsets n x u64][lens n x u32][pad][values, 8-aligned]
    const size_t lens_off = n * sizeof(uint64_t), vals_off = round_up(lens_off + n * 4, 16);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        if (lens[i] > 0xFFFFFFFFull) return fail(HBRBC_E_INVALID_ARG, "value too long");
        total += round_up(lens[i], 8);
    }
    const size_t bytes = vals_off + total + 16;
    const size_t nodes = hbrbc_merkle_node_count(n);
    HB_HIP(c->pin.ensure(std::max(bytes, nodes * 32)));
    HB_HIP(c->st_slab.ensure(bytes));
    HB_HIP(c->st_nodes.ensure(nodes * 32));
    uint8_t *pin = c->pin.as<uint8_t>();
    uint64_t *offs = reinterpret_cast<uint64_t *>(pin);
    uint32_t *ls = reinterpret_cast<uint32_t *>(pin + lens_off);
    size_t at = 0;
    for (size_t i = 0; i < n; ++i) {
        offs[i] = vals_off + at;
        ls[i] = (uint32_t)lens[i];
        if (lens[i]) std::memcpy(pin + vals_off + at, values[i], lens[i]);
        std::memset(pin + vals_off + at + lens[i], 0, round_up(lens[i], 8) - lens[i]);
        at += round_up(lens[i], 8);
    }
    std::memset(pin + vals_off + at, 0, 16);
    uint8_t *dv = c->st_slab.as<uint8_t>();
    HB_HIP(hipMemcpyAsync(dv, pin, bytes, hipMemcpyHostToDevice, c->stream));
    uint8_t *dn = c->st_nodes.as<uint8_t>();
    HB_HIP(launch_ragged_hash(dv, reinterpret_cast<const uint64_t *>(dv),
                              reinterpret_cast<const uint32_t *>(dv + lens_off), n, dn, c->stream));
    size_t off = 0, sz = n;
    while (sz > 1) {
        const size_t nsz = (sz + 1) / 2;
        HB_HIP(launch_tree_level(dn, 0, off, sz, off + sz, nsz, 1, c->stream));
        off += sz;
        sz = nsz;
    }
    HB_HIP(hipMemcpyAsync(pin, dn, nodes * 32, hipMemcpyDeviceToHost, c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(nodes_out, pin, nodes * 32);
    return HBRBC_OK;
}

int hbrbc_merkle_proof(const uint8_t *nodes, size_t n, size_t index, uint8_t *digests_out,
                       size_t *ndig_out) {
    if (!nodes || !ndig_out) return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (index >= n) return HBRBC_E_INVALID_INDEX;  // MerkleTree::proof -> None
    size_t off = 0, sz = n, i = index, d = 0;
    while (sz > 1) {
        if ((i ^ 1) < sz) {
            if (digests_out) std::memcpy(digests_out + 32 * d, nodes + 32 * (off + (i ^ 1)), 32);
            ++d;
        }
        i >>= 1;
        off += sz;
        sz = (sz + 1) / 2;
    }
    *ndig_out = d;
    return HBRBC_OK;
}

int hbrbc_proof_validate(const uint8_t *value, size_t len, size_t index, const uint8_t *digests,
                         size_t ndig, const uint8_t root[32], size_t n, int *valid_out) {
    if (!valid_out || !root || (len && !value) || (ndig && !digests))
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    *valid_out = 0;
    if (n == 0 || n > 0xFFFFFFFFull || index > 0xFFFFFFFFull || len > 0xFFFFFFFFull)
        return fail(HBRBC_E_INVALID_ARG, "bad n / index / len");
    // A tree over n leaves has at most max_proof_len(n) levels with a sibling;
    // more digests than the device slot count can never validate, so clamp the
    // copy and let the kernel's "too many levels" rule reject it.
    const size_t dslots = hbrbc_merkle_max_proof_len(n);
    const size_t nd_dev = ndig > dslots ? dslots + 1 : ndig;
    int st;
    hbrbc_ctx *c = default_ctx(&st);
    if (st) return st;
    std::lock_guard<std::mutex> lk(c->shim_mu);
    HB_HIP(hipSetDevice(c->device));
    // pinned image: [root 32][digests (dslots+1) x 32][meta 16][value, 8-aligned, +16]
    const size_t slots = dslots + 1;
    const size_t dig_off = 32, meta_off = dig_off + 32 * slots, val_off = meta_off + 16;
    const size_t bytes = val_off + round_up(len, 8) + 16;
    HB_HIP(c->pin.ensure(bytes));
    HB_HIP(c->st_slab.ensure(bytes + 16));
    uint8_t *pin = c->pin.as<uint8_t>();
    std::memset(pin, 0, val_off);
    std::memcpy(pin, root, 32);
    if (nd_dev) std::memcpy(pin + dig_off, digests, 32 * std::min(nd_dev, ndig));
    pin[meta_off] = (uint8_t)nd_dev;
    const uint32_t idx = (uint32_t)index;
    std::memcpy(pin + meta_off + 4, &idx, 4);
    if (len) std::memcpy(pin + val_off, value, len);
    std::memset(pin + val_off + len, 0, bytes - val_off - len);
    uint8_t *d = c->st_slab.as<uint8_t>();
    HB_HIP(hipMemcpyAsync(d, pin, bytes, hipMemcpyHostToDevice, c->stream));
    ValidateArgs a;
    a.values = d + val_off;
    a.value_len = len;
    a.value_inst_stride = 0;
    a.per_inst = 1;
    a.vrows = plain_rows(0);
    a.rows = nullptr;
    a.indices = reinterpret_cast<const uint32_t *>(d + meta_off + 4);
    a.digests = d + dig_off;
    a.dslots = slots;
    a.dig_rows = 1;
    a.ndig = d + meta_off;
    a.roots = d;
    a.root_stride = 0;
    a.tree_n = n;
    a.count = 1;
    a.ok_out = d + meta_off + 8;
    a.leaf_out = nullptr;
    a.leaf_inst_stride = 0;
    HB_HIP(launch_validate(a, c->stream));
    HB_HIP(hipMemcpyAsync(pin + meta_off + 8, d + meta_off + 8, 1, hipMemcpyDeviceToHost,
                          c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
    *valid_out = pin[meta_off + 8] ? 1 : 0;
    return HBRBC_OK;
}

// ------------------------------------------------------------ wire format --
size_t hbrbc_wire_proof_message_len(size_t value_len, size_t ndig) { return 60 + value_len + 32 * ndig; }

int hbrbc_wire_encode_batch(hbrbc_ctx *c, uint32_t variant, const uint8_t *values, size_t value_len,
                            size_t value_stride, size_t value_inst_stride, size_t per_inst,
                            const uint32_t *indices, const uint8_t *digests, const uint8_t *ndig,
                            const uint8_t *roots, size_t root_stride, size_t count, uint8_t *out,
                            size_t msg_stride, uint32_t *msg_len_out, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0 || per_inst == 0) return HBRBC_OK;
    if (variant > 1) return fail(HBRBC_E_INVALID_ARG, "variant must be 0 (Value) or 1 (Echo)");
    const size_t dslots = hbrbc_merkle_max_proof_len(c->n);
    if (!values || reinterpret_cast<uintptr_t>(values) % 16 || value_stride % 16 ||
        value_inst_stride % 16 || value_stride < value_len)
        return fail(HBRBC_E_INVALID_ARG, "values must be 16-byte aligned rows of >= value_len");
    if (!ndig || !roots || !out || !msg_len_out || (dslots && !digests))
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(out) % 16 || msg_stride % 16 ||
        msg_stride < round_up(hbrbc_wire_proof_message_len(value_len, dslots), 16))
        return fail(HBRBC_E_INVALID_ARG, "msg_stride must be a multiple of 16 and >= %zu",
                    round_up(hbrbc_wire_proof_message_len(value_len, dslots), 16));
    if (value_len > 0xFFFFFFFFull - 4096) return fail(HBRBC_E_INVALID_ARG, "value too long");
    HB_HIP(hipSetDevice(c->device));
    WireEncodeArgs a;
    a.variant = variant;
    a.values = values;
    a.value_len = value_len;
    a.value_stride = value_stride;
    a.value_inst_stride = value_inst_stride;
    a.per_inst = per_inst;
    a.indices = indices;
    a.digests = digests;
    a.dslots = dslots;
    a.ndig = ndig;
    a.roots = roots;
    a.root_stride = root_stride;
    a.count = count;
    a.out = out;
    a.msg_stride = msg_stride;
    a.msg_len = msg_len_out;
    HB_HIP(launch_wire_encode(a, pick(c, stream)));
    return HBRBC_OK;
}

int hbrbc_wire_decode_batch(hbrbc_ctx *c, const uint8_t *msgs, size_t msg_stride,
                            const uint32_t *msg_len, size_t nmsg, uint8_t *values,
                            size_t value_stride, uint32_t *value_len_out, uint32_t *index_out,
                            uint8_t *digests, uint8_t *ndig_out, uint8_t *roots,
                            uint32_t *variant_out, int32_t *status_out, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (nmsg == 0) return HBRBC_OK;
    const size_t dslots = hbrbc_merkle_max_proof_len(c->n);
    if (!msgs || reinterpret_cast<uintptr_t>(msgs) % 16 || msg_stride % 16 || !msg_len)
        return fail(HBRBC_E_INVALID_ARG, "messages must be 16-byte aligned slots");
    if (!values || reinterpret_cast<uintptr_t>(values) % 16 || value_stride % 16 ||
        !value_len_out || !index_out || !ndig_out || !roots || !variant_out || !status_out ||
        (dslots && !digests))
        return fail(HBRBC_E_INVALID_ARG, "null or misaligned output");
    HB_HIP(hipSetDevice(c->device));
    WireDecodeArgs a;
    a.msgs = msgs;
    a.msg_stride = msg_stride;
    a.msg_len = msg_len;
    a.nmsg = nmsg;
    a.values = values;
    a.value_stride = value_stride;
    a.value_cap = value_stride;
    a.value_len = value_len_out;
    a.index = index_out;
    a.digests = digests;
    a.dslots = dslots;
    a.ndig = ndig_out;
    a.roots = roots;
    a.variant = variant_out;
    a.status = status_out;
    HB_HIP(launch_wire_decode(a, pick(c, stream)));
    return HBRBC_OK;
}


// ------------------------------------------------------ specialised encode --
const char *hbrbc_encode_kernel(const hbrbc_ctx *c) { return c ? c->enc_kind.c_str() : "none"; }

size_t hbrbc_jit_encode_groups(size_t data_shards, size_t parity_shards) {
    if (data_shards == 0 || parity_shards == 0) return 0;
    return xor_groups(data_shards, parity_shards, spec_row_tile(data_shards, parity_shards)).size();
}

int hbrbc_jit_build_encode_rows(size_t data_shards, size_t parity_shards, size_t group,
                                size_t rows_per_block, const char *dir) {
    if (data_shards == 0 || parity_shards == 0 || data_shards + parity_shards > 256)
        return fail(HBRBC_E_INVALID_ARG, "need data >= 1, parity >= 1, data + parity <= 256");
    const size_t n = data_shards + parity_shards;
    std::vector<uint8_t> mat;
    if (!build_matrix(data_shards, n, mat))
        return fail(HBRBC_E_SINGULAR_MATRIX, "singular Vandermonde top block");
    const int rt = spec_row_tile(data_shards, parity_shards), depth = spec_depth();
    const int rb = (rows_per_block && rows_per_block < n) ? (int)rows_per_block : 256;
    const auto groups = xor_groups(data_shards, parity_shards, rt);
    if (group >= groups.size()) return fail(HBRBC_E_INVALID_ARG, "group %zu of %zu", group,
                                            groups.size());
    const XorProgram p = encode_program(data_shards, parity_shards,
                                        mat.data() + data_shards * data_shards, rt, depth,
                                        groups[group].first, groups[group].second, rb);
    std::vector<char> code;
    std::string log;
    if (compile_source(gen_xor_source(p), code, log))
        return fail(HBRBC_E_DEVICE, "hiprtc: %s", log.substr(0, 400).c_str());
    const std::string d = dir ? std::string(dir) : jit_dir();
    mkdir(d.c_str(), 0755);
    const std::string path = jit_file(d, p.name);
    return write_file(path, code) ? HBRBC_OK
                                  : fail(HBRBC_E_INVALID_ARG, "cannot write %s", path.c_str());
}

int hbrbc_jit_build_encode_group(size_t data_shards, size_t parity_shards, size_t group,
                                 const char *dir) {
    return hbrbc_jit_build_encode_rows(data_shards, parity_shards, group, 0, dir);
}

int hbrbc_jit_encode_file_name(size_t data_shards, size_t parity_shards, size_t group,
                               size_t rows_per_block, char *buf, size_t buf_len) {
    if (data_shards == 0 || parity_shards == 0 || !buf)
        return fail(HBRBC_E_INVALID_ARG, "need data >= 1, parity >= 1, a buffer");
    const size_t n = data_shards + parity_shards;
    const int rt = spec_row_tile(data_shards, parity_shards);
    const int rb = (rows_per_block && rows_per_block < n) ? (int)rows_per_block : 256;
    const auto groups = xor_groups(data_shards, parity_shards, rt);
    if (group >= groups.size()) return fail(HBRBC_E_INVALID_ARG, "group %zu of %zu", group,
                                            groups.size());
    const std::string f =
        jit_file("", encode_kernel_name(data_shards, parity_shards, rt, spec_depth(),
                                        groups[group].first, groups[group].second, rb,
                                        spec_sync(), spec_fdepth(), spec_spread(),
                                        spec_split()) +
                     spec_suffix(data_shards, groups[group].second - groups[group].first, rt))
            .substr(1);
    if (f.size() + 1 > buf_len) return fail(HBRBC_E_INVALID_ARG, "buffer too small");
    std::memcpy(buf, f.c_str(), f.size() + 1);
    return HBRBC_OK;
}

int hbrbc_jit_file_name(size_t data_shards, size_t parity_shards, size_t group, char *buf,
                        size_t buf_len) {
    return hbrbc_jit_encode_file_name(data_shards, parity_shards, group, 0, buf, buf_len);
}

int hbrbc_jit_decode_file_name(size_t data_shards, size_t parity_shards, const uint8_t *present,
                               size_t rows_per_block, size_t group, char *buf, size_t buf_len) {
    return hbrbc_jit_decode_variant_file_name(data_shards, parity_shards, present, rows_per_block,
                                              group, 0, buf, buf_len);
}

int hbrbc_jit_decode_variant_file_name(size_t data_shards, size_t parity_shards,
                                       const uint8_t *present, size_t rows_per_block,
                                       size_t group, int fused_unframe, char *buf,
                                       size_t buf_len) {
    std::vector<uint8_t> mat;
    const size_t n = data_shards + parity_shards;
    if (!present || !buf || data_shards == 0 || n > 256 || !build_matrix(data_shards, n, mat))
        return fail(HBRBC_E_INVALID_ARG, "bad arguments");
    const int rb = (rows_per_block && rows_per_block < n) ? (int)rows_per_block : 256;
    std::vector<XorProgram> progs;
    uint64_t hash;
    int rt;
    if (!decode_programs(mat, data_shards, n, present, rb, progs, hash, rt, fused_unframe != 0) ||
        group >= progs.size())
        return fail(HBRBC_E_INVALID_ARG, "no such decoder group");
    const std::string f = jit_file("", progs[group].name).substr(1);
    if (f.size() + 1 > buf_len) return fail(HBRBC_E_INVALID_ARG, "buffer too small");
    std::memcpy(buf, f.c_str(), f.size() + 1);
    return HBRBC_OK;
}

int hbrbc_jit_build_encode(size_t data_shards, size_t parity_shards, const char *dir) {
    const size_t n = hbrbc_jit_encode_groups(data_shards, parity_shards);
    if (n == 0) return fail(HBRBC_E_INVALID_ARG, "need data >= 1, parity >= 1");
    for (size_t g = 0; g < n; ++g) {
        const int st = hbrbc_jit_build_encode_group(data_shards, parity_shards, g, dir);
        if (st) return st;
    }
    return HBRBC_OK;
}

// ------------------------------------------------------------- profiling --
int hbrbc_profile_enable(hbrbc_ctx *c, int enable) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    c->prof = enable != 0;
    return HBRBC_OK;
}

int hbrbc_profile_reset(hbrbc_ctx *c) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    HB_HIP(hipSetDevice(c->device));
    c->recs.clear();
    c->ev_used = 0;
    return HBRBC_OK;
}

int hbrbc_profile_read(hbrbc_ctx *c, double *ms_out, uint64_t *launches_out) {
    if (!c || !ms_out) return fail(HBRBC_E_INVALID_ARG, "null argument");
    HB_HIP(hipSetDevice(c->device));
    for (int i = 0; i < HBRBC_STAGE_COUNT; ++i) {
        ms_out[i] = 0.0;
        if (launches_out) launches_out[i] = 0;
    }
    for (auto &r : c->recs) {
        HB_HIP(hipEventSynchronize(r.b));
        float ms = 0.f;
        HB_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        ms_out[r.stage] += ms;
        if (launches_out) launches_out[r.stage] += 1;
    }
    return HBRBC_OK;
}

const char *hbrbc_stage_name(int stage) {
    static const char *names[HBRBC_STAGE_COUNT] = {"frame",     "encode",        "leaf_hash",
                                                   "tree_levels", "proofs",      "validate",
                                                   "decode_matrix", "reconstruct", "unframe"};
    return (stage >= 0 && stage < HBRBC_STAGE_COUNT) ? names[stage] : "?";
}

int hbrbc_unframe_fused(const hbrbc_ctx *c, size_t shard_len, size_t payload_stride,
                        size_t rows_per_block) {
    if (!c) return 0;
    RowMap rows = plain_rows(round_up(shard_len, 16));
    if (rows_per_block && rows_per_block < c->n) rows.rb = (uint32_t)rows_per_block;
    const auto ds = c->dec_spec.find(code_rb(rows));
    const bool spec = ds != c->dec_spec.end() && !ds->second.groups.empty();
    // with a specialised decoder, its _uf variant (untried: assumed loadable)
    return unframe_fusable(c, shard_len, payload_stride) && (!spec || ds->second.uf_state >= 0)
               ? 1 : 0;
}

// ---- threshold-decrypt share verification (pairing.hip) ----
size_t hbrbc_pairing_workspace_size(size_t pairings) {
    return round_up(pairings * 576, 256) + round_up(pairings, 256);
}

static int pairing_run(const uint8_t *g1, const uint8_t *g2, size_t n_pair, size_t n_out,
                       int per_out, uint8_t *gt_out, uint8_t *ok_out, uint8_t *status_out,
                       void *workspace, hipStream_t s) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    uint32_t *ws = static_cast<uint32_t *>(workspace);
    uint8_t *st = static_cast<uint8_t *>(workspace) + round_up(n_pair * 576, 256);
    const char *mm = getenv("HBRBC_PAIR_MULTI");   // 0: one lane per pairing (A/B)
    if (per_out == 2 && !(mm && !std::strcmp(mm, "0"))) {
        // checks: one lane per check, both Miller loops sharing f's squarings
        HB_HIP(launch_pairing_miller2(g1, g2, n_out, ws, st, s));
        HB_HIP(launch_pairing_final(ws, n_out, n_out, 1, st, gt_out, ok_out, s));
        return HBRBC_OK;
    }
    HB_HIP(launch_pairing_miller(g1, 96, g2, 192, n_pair, per_out == 2, ws, st, s));
    if (status_out) HB_HIP(hipMemcpyAsync(status_out, st, n_pair, hipMemcpyDeviceToDevice, s));
    HB_HIP(launch_pairing_final(ws, n_pair, n_out, per_out, st, gt_out, ok_out, s));
    return HBRBC_OK;
}

int hbrbc_pairing_batch(const uint8_t *g1, const uint8_t *g2, size_t count, uint8_t *gt_out,
                        uint8_t *status_out, void *workspace, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!g1 || !g2 || !gt_out || !workspace) return fail(HBRBC_E_INVALID_ARG, "null argument");
    return pairing_run(g1, g2, count, count, 1, gt_out, nullptr, status_out, workspace,
                       static_cast<hipStream_t>(stream));
}

int hbrbc_pairing_check_batch(const uint8_t *g1, const uint8_t *g2, size_t count,
                              uint8_t *ok_out, void *workspace, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!g1 || !g2 || !ok_out || !workspace) return fail(HBRBC_E_INVALID_ARG, "null argument");
    return pairing_run(g1, g2, 2 * count, count, 2, nullptr, ok_out, nullptr, workspace,
                       static_cast<hipStream_t>(stream));
}

size_t hbrbc_g2_prepared_size(size_t points) {
    return round_up(pairing_prepared_words(points) * 4, 256) + round_up(points, 256);
}

int hbrbc_g2_prepare(const uint8_t *g2, size_t count, void *prepared, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!g2 || !prepared) return fail(HBRBC_E_INVALID_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    uint32_t *prep = static_cast<uint32_t *>(prepared);
    uint8_t *pst = static_cast<uint8_t *>(prepared) + round_up(pairing_prepared_words(count) * 4, 256);
    HB_HIP(launch_g2_prepare(g2, count, prep, pst, static_cast<hipStream_t>(stream)));
    return HBRBC_OK;
}

int hbrbc_pairing_check_prepared(const uint8_t *g1, const void *prepared, size_t points,
                                 const uint32_t *idx_b, const uint32_t *idx_d, size_t count,
                                 uint8_t *ok_out, void *workspace, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!g1 || !prepared || !idx_b || !idx_d || !ok_out || !workspace)
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    const uint32_t *prep = static_cast<const uint32_t *>(prepared);
    const uint8_t *pst =
        static_cast<const uint8_t *>(prepared) + round_up(pairing_prepared_words(points) * 4, 256);
    uint32_t *ws = static_cast<uint32_t *>(workspace);
    uint8_t *st = static_cast<uint8_t *>(workspace) + round_up(count * 576, 256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (points == 0) return fail(HBRBC_E_INVALID_ARG, "no prepared points");
    HB_HIP(launch_pairing_miller_prepared(g1, prep, pst, idx_b, idx_d, points, count, ws, st, s));
    HB_HIP(launch_pairing_final(ws, count, count, 1, st, nullptr, ok_out, s));
    return HBRBC_OK;
}

size_t hbrbc_g1_prepared_size(size_t points) {
    return round_up(g1_key_words(points) * 4, 256) + round_up(points, 256);
}

int hbrbc_g1_prepare(const uint8_t *g1, size_t count, void *prepared, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!g1 || !prepared) return fail(HBRBC_E_INVALID_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    uint32_t *keys = static_cast<uint32_t *>(prepared);
    uint8_t *kst = static_cast<uint8_t *>(prepared) + round_up(g1_key_words(count) * 4, 256);
    HB_HIP(launch_g1_prepare(g1, count, keys, kst, static_cast<hipStream_t>(stream)));
    return HBRBC_OK;
}

int hbrbc_pairing_check_prepared_keys(const uint8_t *g1_a, const void *keys, size_t key_points,
                                      const uint32_t *idx_c, const void *prepared, size_t points,
                                      const uint32_t *idx_b, const uint32_t *idx_d, size_t count,
                                      uint8_t *ok_out, void *workspace, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!g1_a || !keys || !idx_c || !prepared || !idx_b || !idx_d || !ok_out || !workspace)
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (points == 0) return fail(HBRBC_E_INVALID_ARG, "no prepared points");
    if (key_points == 0) return fail(HBRBC_E_INVALID_ARG, "no prepared keys");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    const uint32_t *kw = static_cast<const uint32_t *>(keys);
    const uint8_t *kst =
        static_cast<const uint8_t *>(keys) + round_up(g1_key_words(key_points) * 4, 256);
    const uint32_t *prep = static_cast<const uint32_t *>(prepared);
    const uint8_t *pst =
        static_cast<const uint8_t *>(prepared) + round_up(pairing_prepared_words(points) * 4, 256);
    uint32_t *ws = static_cast<uint32_t *>(workspace);
    uint8_t *st = static_cast<uint8_t *>(workspace) + round_up(count * 576, 256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    HB_HIP(launch_pairing_miller_prepared_keys(g1_a, kw, kst, idx_c, key_points, prep, pst, idx_b,
                                               idx_d, points, count, ws, st, s));
    HB_HIP(launch_pairing_final(ws, count, count, 1, st, nullptr, ok_out, s));
    return HBRBC_OK;
}

int hbrbc_pairing_check_prepared_pts(const void *a_prepared, const void *keys, size_t key_points,
                                     const uint32_t *idx_c, const void *prepared, size_t points,
                                     const uint32_t *idx_b, const uint32_t *idx_d, size_t count,
                                     uint8_t *ok_out, void *workspace, void *stream) {
    if (count == 0) return HBRBC_OK;
    if (!a_prepared || !keys || !idx_c || !prepared || !idx_b || !idx_d || !ok_out || !workspace)
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (points == 0) return fail(HBRBC_E_INVALID_ARG, "no prepared points");
    if (key_points == 0) return fail(HBRBC_E_INVALID_ARG, "no prepared keys");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    const uint32_t *aw = static_cast<const uint32_t *>(a_prepared);
    const uint8_t *ast =
        static_cast<const uint8_t *>(a_prepared) + round_up(g1_key_words(count) * 4, 256);
    const uint32_t *kw = static_cast<const uint32_t *>(keys);
    const uint8_t *kst =
        static_cast<const uint8_t *>(keys) + round_up(g1_key_words(key_points) * 4, 256);
    const uint32_t *prep = static_cast<const uint32_t *>(prepared);
    const uint8_t *pst =
        static_cast<const uint8_t *>(prepared) + round_up(pairing_prepared_words(points) * 4, 256);
    uint32_t *ws = static_cast<uint32_t *>(workspace);
    uint8_t *st = static_cast<uint8_t *>(workspace) + round_up(count * 576, 256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    HB_HIP(launch_pairing_miller_prepared_pts(aw, ast, kw, kst, idx_c, key_points, prep, pst, idx_b,
                                              idx_d, points, count, ws, st, s));
    HB_HIP(launch_pairing_final(ws, count, count, 1, st, nullptr, ok_out, s));
    return HBRBC_OK;
}

int hbrbc_pairing_check(const uint8_t a[96], const uint8_t b[192], const uint8_t c[96],
                        const uint8_t d[192], int *result) {
    if (!a || !b || !c || !d || !result) return fail(HBRBC_E_INVALID_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(HBRBC_E_NO_DEVICE, "no HIP device visible");
    const size_t ws_bytes = hbrbc_pairing_workspace_size(2);
    const size_t total = 2 * 96 + 2 * 192 + 16 + ws_bytes;
    uint8_t *dev = nullptr;
    HB_HIP(hipMalloc(&dev, total));
    std::vector<uint8_t> host(2 * 96 + 2 * 192);
    memcpy(host.data(), a, 96);
    memcpy(host.data() + 96, c, 96);
    memcpy(host.data() + 192, b, 192);
    memcpy(host.data() + 384, d, 192);
    uint8_t ok = 0;
    int rc = HBRBC_OK;
    hipError_t e = hipMemcpy(dev, host.data(), host.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        rc = pairing_run(dev, dev + 192, 2, 1, 2, nullptr, dev + 576, nullptr, dev + 592,
                         nullptr);
        if (rc == HBRBC_OK) e = hipMemcpy(&ok, dev + 576, 1, hipMemcpyDeviceToHost);
    }
    (void)hipFree(dev);
    if (e != hipSuccess) return fail(HBRBC_E_DEVICE, "pairing check: %s", hipGetErrorString(e));
    if (rc != HBRBC_OK) return rc;
    if (ok == 2) return fail(HBRBC_E_INVALID_ARG, "invalid curve point");
    *result = ok;
    return HBRBC_OK;
}

// ---- f2: the Broadcast state machine, batched (sim.hip) -------------------
size_t hbrbc_sm_state_bytes(size_t n, size_t roots) { return sm_state_bytes(n, roots); }

int hbrbc_sm_round(hbrbc_ctx *c, const hbrbc_sm_args *a, void *stream) {
    if (!c || !a) return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (a->count == 0 || a->nodes == 0) return HBRBC_OK;
    const size_t n = c->n;
    if (n > 255) return fail(HBRBC_E_INVALID_ARG, "the state machine handles n <= 255 validators");
    if (a->roots == 0 || a->roots > 8) return fail(HBRBC_E_INVALID_ARG, "roots must be 1..8");
    if (a->max_out == 0 || a->rows_per_rank == 0 || a->node_lo >= n)
        return fail(HBRBC_E_INVALID_ARG, "bad max_out / rows_per_rank / node_lo");
    if (!a->proposer || !a->role || !a->value_root || !a->value_tamper || !a->proof_ok ||
        !a->decode_ok || !a->fake_from || !a->fake_root || !a->fake_list || !a->out ||
        !a->out_count || !a->state || !a->output_root || !a->fault_count || !a->emitted ||
        (a->max_faults && !a->faults) || (a->round > 0 && (!a->in || !a->in_count)))
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    HB_HIP(hipSetDevice(c->device));
    const int f = (int)((n - c->k) / 2);
    HB_HIP(launch_sm_round(*a, (int)n, f, (int)c->k, pick(c, stream)));
    return HBRBC_OK;
}

}  // extern "C"
