// api.hip -- implementation of include/hbrbc.h (the C ABI of libhbrbc.so).
//
// Host-side responsibilities only: argument checks with the reference's
// error semantics, the encoding matrix (rse `build_matrix`, computed once per
// context exactly like `ReedSolomon::new`), device workspaces, and launch
// sequencing.  Every byte of shard, digest and payload data is computed by
// the HIP kernels in kernels.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
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

}  // namespace

struct hbrbc_ctx {
    int device = 0;
    size_t k = 0, m = 0, n = 0;
    int rt_enc = 2, rt_rec = 2;  // GF row tiles (rows per pass) for encode / reconstruct
    int bitslice = 1;            // GF kernel: 1 bit-sliced (default), 0 split-2-bit v_perm
    std::vector<uint8_t> matrix;  // n x k
    hipStream_t stream = nullptr;
    // specialised encoder (jit.hip) for this matrix, when its code object is available
    // specialised encoder (jit.hip), one module per parity-row group
    struct SpecGroup {
        int r_lo, r_hi;
        hipModule_t mod;
        hipFunction_t enc, fe;       // encode / frame+encode twin
    };
    std::vector<SpecGroup> spec;
    int rt_spec = 2;              // parity rows per pass of the specialised encoder
    int depth_spec = 4;           // its data-row prefetch depth
    std::string enc_kind = "none";
    DevBuf d_matrix, d_enc_tables, d_enc_in, d_enc_out;
    // reconstruct workspace
    size_t ws_count = 0;
    DevBuf ws_tables, ws_in, ws_out, ws_nout, ws_status, ws_plen;
    // per-call shim staging
    std::mutex shim_mu;
    DevBuf st_slab, st_present, st_status, st_nodes, st_aux, st_aux2, st_aux3;
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
               size_t n, size_t count) {
    if (count == 0) return HBRBC_OK;
    if (!base) return fail(HBRBC_E_INVALID_ARG, "null shard slab");
    if (reinterpret_cast<uintptr_t>(base) % 16)
        return fail(HBRBC_E_INVALID_ARG, "shard slab base must be 16-byte aligned");
    if (shard_stride % 16 || shard_stride < shard_len)
        return fail(HBRBC_E_INVALID_ARG, "shard_stride %zu must be a multiple of 16 and >= %zu",
                    shard_stride, shard_len);
    if (count > 1 && (inst_stride % 16 || inst_stride < n * shard_stride))
        return fail(HBRBC_E_INVALID_ARG, "inst_stride %zu must be a multiple of 16 and >= %zu",
                    inst_stride, n * shard_stride);
    if (shard_len > 0xFFFFFFFFull) return fail(HBRBC_E_INVALID_ARG, "shard_len too large");
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

size_t rec_tab_rows(const hbrbc_ctx *c) {
    return (c->m + c->rt_rec - 1) / c->rt_rec * c->rt_rec;
}

int ensure_workspace(hbrbc_ctx *c, size_t count) {
    if (count <= c->ws_count) return HBRBC_OK;
    const size_t k = c->k, m = c->m;
    HB_HIP(c->ws_tables.ensure(count * rec_tab_rows(c) * k * sizeof(uint4) + 16));
    HB_HIP(c->ws_in.ensure((count * k + 4) * sizeof(uint32_t)));
    HB_HIP(c->ws_out.ensure((count * m + 4) * sizeof(uint32_t)));
    HB_HIP(c->ws_nout.ensure(count * sizeof(int)));
    HB_HIP(c->ws_status.ensure(count * sizeof(int32_t)));
    HB_HIP(c->ws_plen.ensure(count * sizeof(uint32_t)));
    c->ws_count = count;
    return HBRBC_OK;
}

// Leaf hashes + all levels into a node slab.
int run_merkle(hbrbc_ctx *c, const uint8_t *shards, size_t shard_len, size_t shard_stride,
               size_t inst_stride, size_t n, size_t count, uint8_t *nodes,
               size_t node_inst_stride, hipStream_t s) {
    {
        StageTimer t(c, HBRBC_STAGE_LEAF_HASH, s);
        HB_HIP(launch_leaf_hash(shards, shard_len, shard_stride, inst_stride, n, count, nodes,
                                node_inst_stride, s));
    }
    StageTimer t(c, HBRBC_STAGE_TREE_LEVELS, s);
    size_t off = 0, sz = n;
    while (sz > 1) {
        const size_t nsz = (sz + 1) / 2;
        HB_HIP(launch_tree_level(nodes, node_inst_stride, off, sz, off + sz, nsz, count, s));
        off += sz;
        sz = nsz;
    }
    return HBRBC_OK;
}

int run_reconstruct(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                    size_t inst_stride, const uint8_t *present, size_t count, int32_t *status,
                    hipStream_t s) {
    int st = ensure_workspace(c, count);
    if (st) return st;
    {
        StageTimer t(c, HBRBC_STAGE_DECODE_MATRIX, s);
        DecodeMatrixArgs a;
        a.n = (int)c->n;
        a.k = (int)c->k;
        a.rt = c->rt_rec;
        a.raw = c->bitslice;
        a.matrix = c->d_matrix.as<uint8_t>();
        a.present = present;
        a.count = count;
        a.tables = c->ws_tables.as<uint4>();
        a.in_idx = c->ws_in.as<uint32_t>();
        a.out_idx = c->ws_out.as<uint32_t>();
        a.nout = c->ws_nout.as<int>();
        a.status = status;
        HB_HIP(launch_decode_matrix(a, s));
    }
    if (c->m == 0) return HBRBC_OK;  // Coding::Trivial: nothing to rebuild
    StageTimer t(c, HBRBC_STAGE_RECONSTRUCT, s);
    GfApplyArgs g;
    g.base = shards;
    g.inst_stride = inst_stride;
    g.shard_stride = shard_stride;
    g.n16 = (int)((shard_len + 15) / 16);
    g.tables = c->ws_tables.as<uint4>();
    g.tab_inst_stride = rec_tab_rows(c) * c->k;
    g.rt = c->rt_rec;
    g.bitslice = c->bitslice;
    g.in_idx = c->ws_in.as<uint32_t>();
    g.in_idx_stride = c->k;
    g.out_idx = c->ws_out.as<uint32_t>();
    g.out_idx_stride = c->m;
    g.nout = c->ws_nout.as<int>();
    g.nout_uniform = 0;
    g.max_rows = (int)c->m;
    g.nin = (int)c->k;
    g.count = count;
    HB_HIP(launch_gf_apply(g, s));
    return HBRBC_OK;
}

// Directory of cached specialised-encoder code objects: $HBRBC_JIT_DIR, else
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

std::string jit_file(const std::string &dir, size_t k, size_t m, int rt, int depth, int r_lo) {
    const char *aux = getenv("HBRBC_ST_AUX");   // A/B builds get their own files
    return dir + "/" + encode_kernel_name(k, m, rt, depth, false, r_lo) +
           (aux && std::strcmp(aux, "2") ? std::string("_a") + aux : std::string()) + "_v10.co";
}

// Data rows the specialised encoder keeps in flight (HBM latency at 2 waves/SIMD).
int spec_depth() {
    if (const char *e = getenv("HBRBC_JIT_DEPTH")) return std::max(1, std::min(8, atoi(e)));
    return 4;
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

// Parity rows per pass of the specialised encoder: the accumulators (8 VGPRs
// per row) plus the planes, pair XORs and load buffers must stay near 200
// VGPRs (2 waves/SIMD) without spilling.
int spec_row_tile(size_t k, size_t m) {
    if (const char *e = getenv("HBRBC_RT_SPEC")) return std::max(2, std::min(16, atoi(e) & ~1));
    // split matrices: 8-row passes keep each program's straight-line passes
    // (and so its compile time) small
    return k * m > 4096 ? 8 : gf_row_tile((int)m);
}

// Load (or, with HBRBC_JIT=1, compile and cache) the specialised encoder.
// Any failure leaves the context on the generic bit-sliced kernel.
void drop_spec(hbrbc_ctx *c) {
    for (auto &g : c->spec)
        if (g.mod) (void)hipModuleUnload(g.mod);
    c->spec.clear();
}

void setup_spec_encoder(hbrbc_ctx *c) {
    const char *mode = getenv("HBRBC_JIT");
    if (c->m == 0 || (mode && !std::strcmp(mode, "0")) || c->k * c->m > 16384) return;
    c->rt_spec = spec_row_tile(c->k, c->m);
    c->depth_spec = spec_depth();
    for (const auto &rg : encode_groups(c->k, c->m, c->rt_spec)) {
        const std::string path =
            jit_file(jit_dir(), c->k, c->m, c->rt_spec, c->depth_spec, rg.first);
        std::vector<char> code;
        if (!read_file(path, code)) {
            if (!mode || std::strcmp(mode, "1")) return drop_spec(c);
            std::string log;
            if (compile_encode(c->k, c->m, c->matrix.data() + c->k * c->k, c->rt_spec,
                               c->depth_spec, rg.first, rg.second, code, log)) {
                c->enc_kind = "jit-failed";
                return drop_spec(c);
            }
            mkdir(jit_dir().c_str(), 0755);
            if (FILE *f = fopen(path.c_str(), "wb")) {
                fwrite(code.data(), 1, code.size(), f);
                fclose(f);
            }
        }
        hbrbc_ctx::SpecGroup g{rg.first, rg.second, nullptr, nullptr, nullptr};
        if (hipModuleLoadData(&g.mod, code.data()) != hipSuccess) return drop_spec(c);
        c->spec.push_back(g);
        auto &b = c->spec.back();
        if (hipModuleGetFunction(&b.enc, b.mod,
                                 encode_kernel_name(c->k, c->m, c->rt_spec, c->depth_spec, false,
                                                    rg.first)
                                     .c_str()) != hipSuccess ||
            hipModuleGetFunction(&b.fe, b.mod,
                                 encode_kernel_name(c->k, c->m, c->rt_spec,
                                                    fused_depth(c->depth_spec), true, rg.first)
                                     .c_str()) != hipSuccess)
            return drop_spec(c);
    }
    c->enc_kind = "specialised";
}

// HBRBC_SPEC_SPLIT=1: launch the specialised encoder pass by pass.
bool spec_pass_split() {
    const char *e = getenv("HBRBC_SPEC_SPLIT");
    return e && !std::strcmp(e, "1");
}

// Launch one group's encode (fused = frame+encode twin of group 0).
hipError_t launch_spec_group(hbrbc_ctx *c, const hbrbc_ctx::SpecGroup &g, bool fused,
                             uint8_t *shards, size_t shard_len, size_t shard_stride,
                             size_t inst_stride, size_t count, const uint8_t *payloads,
                             size_t payload_stride, size_t payload_len, hipStream_t s) {
    uint8_t *base = shards;
    const uint8_t *pay = payloads;
    unsigned long ist = inst_stride, sst = shard_stride, pst = payload_stride;
    unsigned row_bytes = (unsigned)(fused ? shard_stride : round_up(shard_len, 16));
    unsigned P = (unsigned)payload_len, S = (unsigned)shard_len;
    unsigned wpr = (row_bytes + 64 * 32 - 1) / (64 * 32);
    const size_t blocks = (size_t)wpr * count;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const int npass = (g.r_hi - g.r_lo + c->rt_spec - 1) / c->rt_spec;
    int p_only = -1;
    void *args_e[] = {&base, &ist, &sst, &row_bytes, &wpr, &p_only};
    void *args_f[] = {&base, &ist, &sst, &row_bytes, &wpr, &pay, &pst, &P, &S, &p_only};
    void **args = fused ? args_f : args_e;
    if (!spec_pass_split()) {
        const unsigned threads = 64u * (unsigned)std::min(4, npass);
        return hipModuleLaunchKernel(fused ? g.fe : g.enc, (unsigned)blocks, 1, 1, threads, 1, 1, 0,
                                     s, args, nullptr);
    }
    // one launch per pass, one wave per workgroup: every wave on the chip
    // runs the same pass's code (the three-pass N = 64 program is 151 KB of
    // straight-line code, more than the instruction cache a CU pair shares)
    for (p_only = 0; p_only < npass; ++p_only) {
        const hipError_t e = hipModuleLaunchKernel(fused ? g.fe : g.enc, (unsigned)blocks, 1, 1, 64u,
                                                   1, 1, 0, s, args, nullptr);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

std::once_flag g_default_once;
hbrbc_ctx *g_default = nullptr;
int g_default_status = HBRBC_OK;

hbrbc_ctx *default_ctx(int *st) {
    std::call_once(g_default_once, [] { g_default_status = hbrbc_coding_new(1, 0, -1, &g_default); });
    *st = g_default_status;
    return g_default;
}

}  // namespace

// =========================================================================
extern "C" {

const char *hbrbc_last_error(void) { return g_err.c_str(); }
const char *hbrbc_version(void) { return "hbrbc 0.1.0 gfx950"; }

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
    }
    if (const char *e = getenv("HBRBC_GF")) {
        // bitslice (uniform branches), bitslice_likely (set-bit path inline),
        // bitslice_mask (branch-free masked xor), perm (split-2-bit v_perm)
        if (!std::strcmp(e, "perm")) c->bitslice = 0;
        else if (!std::strcmp(e, "bitslice_likely")) c->bitslice = 2;
        else if (!std::strcmp(e, "bitslice_mask")) c->bitslice = 3;
        else c->bitslice = 1;
    }
    if (const char *e = getenv("HBRBC_RT_ENC")) c->rt_enc = std::max(2, std::min(16, atoi(e) & ~1));
    if (const char *e = getenv("HBRBC_RT_REC")) c->rt_rec = std::max(2, std::min(16, atoi(e) & ~1));
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
        const HostGf &g = gf();
        // pass-major tables, zero-padded rows: split-2-bit entries [pass][j][rt_enc]
        // (v_perm kernel) or coefficient bytes [pass][j][16] (bit-sliced kernel)
        const size_t rt = (size_t)c->rt_enc, npass = (c->m + rt - 1) / rt;
        std::vector<uint4> tab(npass * rt * c->k, make_uint4(0, 0, 0, 0));
        uint8_t *raw = reinterpret_cast<uint8_t *>(tab.data());
        for (size_t r = 0; r < c->m; ++r)
            for (size_t j = 0; j < c->k; ++j) {
                const uint8_t coef = c->matrix[(c->k + r) * c->k + j];
                if (c->bitslice)
                    raw[((r / rt) * c->k + j) * 16 + (r % rt)] = coef;
                else
                    tab[((r / rt) * c->k + j) * rt + (r % rt)] = gf_split2_entry(coef, g.exp, g.log);
            }
        std::vector<uint32_t> in(c->k), outi(c->m);
        for (size_t j = 0; j < c->k; ++j) in[j] = (uint32_t)j;
        for (size_t r = 0; r < c->m; ++r) outi[r] = (uint32_t)(c->k + r);
        guard(c->d_enc_tables.ensure(tab.size() * sizeof(uint4)));
        guard(c->d_enc_in.ensure(in.size() * sizeof(uint32_t)));
        guard(c->d_enc_out.ensure(outi.size() * sizeof(uint32_t)));
        if (st == HBRBC_OK) {
            guard(hipMemcpy(c->d_enc_tables.p, tab.data(), tab.size() * sizeof(uint4),
                            hipMemcpyHostToDevice));
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
    c->enc_kind = c->m == 0 ? "trivial" : (c->bitslice ? "bitslice" : "perm");
    if (c->bitslice) setup_spec_encoder(c);
    *out = c;
    return HBRBC_OK;
}

void hbrbc_coding_free(hbrbc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (DevBuf *b : {&c->d_matrix, &c->d_enc_tables, &c->d_enc_in, &c->d_enc_out, &c->ws_tables,
                      &c->ws_in, &c->ws_out, &c->ws_nout, &c->ws_status, &c->ws_plen, &c->st_slab,
                      &c->st_present, &c->st_status, &c->st_nodes, &c->st_aux, &c->st_aux2,
                      &c->st_aux3})
        b->release();
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    drop_spec(c);
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
    if (shard_len != hbrbc_shard_len(payload_len, c->k))
        return fail(HBRBC_E_INVALID_ARG, "shard_len %zu != ceil((%zu+4)/%zu)", shard_len,
                    payload_len, c->k);
    if (payload_len > 0xFFFFFFFFull) return fail(HBRBC_E_INVALID_ARG, "payload too large");
    if (payload_len && (!payloads || reinterpret_cast<uintptr_t>(payloads) % 4 ||
                        payload_stride % 4 || payload_stride < round_up(payload_len, 4)))
        return fail(HBRBC_E_INVALID_ARG, "payload buffer must be 4-byte aligned with stride >= "
                                         "round_up(len, 4)");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    StageTimer t(c, HBRBC_STAGE_FRAME, s);
    HB_HIP(launch_frame(payloads, payload_stride, payload_len, count, shards, shard_len,
                        shard_stride, inst_stride, c->k, s));
    return HBRBC_OK;
}

int hbrbc_encode_batch(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                       size_t inst_stride, size_t count, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (c->m == 0 || count == 0) return HBRBC_OK;  // Coding::Trivial::encode
    if (shard_len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shards");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    StageTimer t(c, HBRBC_STAGE_ENCODE, s);
    if (!c->spec.empty()) {
        // specialised XOR networks (jit.hip), one launch per parity-row group
        for (const auto &grp : c->spec)
            HB_HIP(launch_spec_group(c, grp, false, shards, shard_len, shard_stride, inst_stride,
                                     count, nullptr, 0, 0, s));
        return HBRBC_OK;
    }
    GfApplyArgs g;
    g.base = shards;
    g.inst_stride = inst_stride;
    g.shard_stride = shard_stride;
    g.n16 = (int)((shard_len + 15) / 16);
    g.tables = c->d_enc_tables.as<uint4>();
    g.tab_inst_stride = 0;
    g.rt = c->rt_enc;
    g.bitslice = c->bitslice;
    g.in_idx = c->d_enc_in.as<uint32_t>();
    g.in_idx_stride = 0;
    g.out_idx = c->d_enc_out.as<uint32_t>();
    g.out_idx_stride = 0;
    g.nout = nullptr;
    g.nout_uniform = (int)c->m;
    g.max_rows = (int)c->m;
    g.nin = (int)c->k;
    g.count = count;
    HB_HIP(launch_gf_apply(g, s));
    return HBRBC_OK;
}

int hbrbc_frame_encode_batch(hbrbc_ctx *c, const uint8_t *payloads, size_t payload_stride,
                             size_t payload_len, size_t count, uint8_t *shards, size_t shard_len,
                             size_t shard_stride, size_t inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    const bool fused = !c->spec.empty() && shard_stride == round_up(shard_len, 16) &&
                       shard_len == hbrbc_shard_len(payload_len, c->k) &&
                       payload_len <= 0x7FFFFFFFull && shard_len * c->k < 0x7FFFFFFFull;
    if (!fused) {
        int st = hbrbc_frame_batch(c, payloads, payload_stride, payload_len, count, shards,
                                   shard_len, shard_stride, inst_stride, stream);
        return st ? st : hbrbc_encode_batch(c, shards, shard_len, shard_stride, inst_stride, count,
                                            stream);
    }
    if (payload_len && (!payloads || reinterpret_cast<uintptr_t>(payloads) % 4 ||
                        payload_stride % 4 || payload_stride < round_up(payload_len, 4)))
        return fail(HBRBC_E_INVALID_ARG, "payload buffer must be 4-byte aligned with stride >= "
                                         "round_up(len, 4)");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    StageTimer t(c, HBRBC_STAGE_ENCODE, s);
    // frame folded into the specialised encoder (jit.hip): group 0's twin
    // writes the framed data rows and its parity rows, the fixup adds the
    // last partial payload dword to both, and the other groups then encode
    // from the complete data rows
    const auto &g0 = c->spec.front();
    HB_HIP(launch_spec_group(c, g0, true, shards, shard_len, shard_stride, inst_stride, count,
                             payloads, payload_stride, payload_len, s));
    HB_HIP(launch_frame_fixup(payloads, payload_stride, payload_len, shards, shard_len,
                              shard_stride, inst_stride, c->k, (size_t)g0.r_hi,
                              c->d_matrix.as<uint8_t>(), count, s));
    for (size_t i = 1; i < c->spec.size(); ++i)
        HB_HIP(launch_spec_group(c, c->spec[i], false, shards, shard_len, shard_stride,
                                 inst_stride, count, nullptr, 0, 0, s));
    return HBRBC_OK;
}

int hbrbc_merkle_batch(hbrbc_ctx *c, const uint8_t *shards, size_t shard_len,
                       size_t shard_stride, size_t inst_stride, size_t count, uint8_t *nodes,
                       size_t node_inst_stride, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    st = check_nodes(nodes, node_inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    return run_merkle(c, shards, shard_len, shard_stride, inst_stride, c->n, count, nodes,
                      node_inst_stride, pick(c, stream));
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

int hbrbc_validate_batch(hbrbc_ctx *c, const uint8_t *values, size_t value_len,
                         size_t value_stride, size_t value_inst_stride, size_t per_inst,
                         const uint32_t *indices, const uint8_t *digests, const uint8_t *ndig,
                         const uint8_t *roots, size_t root_stride, size_t tree_n, size_t count,
                         uint8_t *ok_out, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0 || per_inst == 0) return HBRBC_OK;
    if (!values || reinterpret_cast<uintptr_t>(values) % 8 || value_stride % 8 ||
        value_inst_stride % 8)
        return fail(HBRBC_E_INVALID_ARG, "values must be 8-byte aligned with 8-byte strides");
    if (!ndig || !roots || !ok_out || reinterpret_cast<uintptr_t>(roots) % 16 || root_stride % 16)
        return fail(HBRBC_E_INVALID_ARG, "roots must be 16-byte aligned; outputs non-null");
    if (tree_n == 0 || tree_n > 0xFFFFFFFFull || value_len > 0xFFFFFFFFull)
        return fail(HBRBC_E_INVALID_ARG, "bad tree_n / value_len");
    const size_t dslots = hbrbc_merkle_max_proof_len(tree_n);
    if (dslots && (!digests || reinterpret_cast<uintptr_t>(digests) % 16))
        return fail(HBRBC_E_INVALID_ARG, "digests must be 16-byte aligned");
    HB_HIP(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    StageTimer t(c, HBRBC_STAGE_VALIDATE, s);
    ValidateArgs a;
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
    a.tree_n = tree_n;
    a.count = count;
    a.ok_out = ok_out;
    HB_HIP(launch_validate(a, s));
    return HBRBC_OK;
}

int hbrbc_reserve(hbrbc_ctx *c, size_t count) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    HB_HIP(hipSetDevice(c->device));
    return ensure_workspace(c, count);
}

int hbrbc_reconstruct_batch(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                            size_t inst_stride, const uint8_t *present, size_t count,
                            int32_t *status_out, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!present || !status_out) return fail(HBRBC_E_INVALID_ARG, "null present/status");
    if (c->m > 0 && shard_len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shards");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
    if (st) return st;
    HB_HIP(hipSetDevice(c->device));
    return run_reconstruct(c, shards, shard_len, shard_stride, inst_stride, present, count,
                           status_out, pick(c, stream));
}

int hbrbc_decode_batch(hbrbc_ctx *c, uint8_t *shards, size_t shard_len, size_t shard_stride,
                       size_t inst_stride, const uint8_t *present, size_t count,
                       const uint8_t *roots, size_t root_stride, uint8_t *nodes,
                       size_t node_inst_stride, uint8_t *payload_out, size_t payload_stride,
                       uint32_t *payload_len_out, int32_t *status_out, void *stream) {
    if (!c) return fail(HBRBC_E_INVALID_ARG, "null context");
    if (count == 0) return HBRBC_OK;
    if (!present || !status_out || !payload_len_out || !roots)
        return fail(HBRBC_E_INVALID_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(roots) % 16 || root_stride % 16)
        return fail(HBRBC_E_INVALID_ARG, "roots must be 16-byte aligned");
    if (shard_len == 0) return fail(HBRBC_E_EMPTY_SHARD, "empty shards");
    int st = check_slab(shards, shard_len, shard_stride, inst_stride, c->n, count);
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
    hipStream_t s = pick(c, stream);
    st = ensure_workspace(c, count);
    if (st) return st;
    int32_t *rstat = c->ws_status.as<int32_t>();
    st = run_reconstruct(c, shards, shard_len, shard_stride, inst_stride, present, count, rstat, s);
    if (st) return st;
    st = run_merkle(c, shards, shard_len, shard_stride, inst_stride, c->n, count, nodes,
                    node_inst_stride, s);
    if (st) return st;
    StageTimer t(c, HBRBC_STAGE_UNFRAME, s);
    HB_HIP(launch_decode_check(rstat, nodes, node_inst_stride, hbrbc_merkle_node_count(c->n) - 1,
                               roots, root_stride, shards, shard_len, shard_stride, inst_stride,
                               c->k, count, payload_len_out, status_out, s));
    HB_HIP(launch_unframe(shards, shard_len, shard_stride, inst_stride, c->k, count,
                          payload_len_out, status_out, payload_out, payload_stride, s));
    return HBRBC_OK;
}

// ---------------------------------------------------------------- layer 1 --
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
    uint8_t *slab = c->st_slab.as<uint8_t>();
    for (size_t j = 0; j < c->k; ++j)
        HB_HIP(hipMemcpyAsync(slab + j * stride, shards[j], len, hipMemcpyHostToDevice, c->stream));
    int st = hbrbc_encode_batch(c, slab, len, stride, c->n * stride, 1, c->stream);
    if (st) return st;
    for (size_t r = c->k; r < c->n; ++r)
        HB_HIP(hipMemcpyAsync(shards[r], slab + r * stride, len, hipMemcpyDeviceToHost, c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
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
    HB_HIP(c->st_slab.ensure(c->n * stride));
    HB_HIP(c->st_present.ensure(c->n));
    HB_HIP(c->st_status.ensure(sizeof(int32_t)));
    uint8_t *slab = c->st_slab.as<uint8_t>();
    std::vector<uint8_t> pres(c->n);
    for (size_t i = 0; i < c->n; ++i) {
        pres[i] = present[i] ? 1 : 0;
        if (pres[i])
            HB_HIP(hipMemcpyAsync(slab + i * stride, shards[i], len, hipMemcpyHostToDevice,
                                  c->stream));
    }
    HB_HIP(hipMemcpyAsync(c->st_present.p, pres.data(), c->n, hipMemcpyHostToDevice, c->stream));
    int st = run_reconstruct(c, slab, len, stride, c->n * stride, c->st_present.as<uint8_t>(), 1,
                             c->st_status.as<int32_t>(), c->stream);
    if (st) return st;
    int32_t status = 0;
    HB_HIP(hipMemcpyAsync(&status, c->st_status.p, sizeof status, hipMemcpyDeviceToHost,
                          c->stream));
    for (size_t i = 0; i < c->n; ++i)
        if (!pres[i])
            HB_HIP(hipMemcpyAsync(shards[i], slab + i * stride, len, hipMemcpyDeviceToHost,
                                  c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
    if (status) return fail(status, "reconstruct status %d", status);
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
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> ls(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        if (lens[i] > 0xFFFFFFFFull) return fail(HBRBC_E_INVALID_ARG, "value too long");
        offs[i] = total;
        ls[i] = (uint32_t)lens[i];
        total += round_up(lens[i], 8);
    }
    std::vector<uint8_t> packed(total + 16, 0);
    for (size_t i = 0; i < n; ++i)
        if (lens[i]) std::memcpy(packed.data() + offs[i], values[i], lens[i]);
    const size_t nodes = hbrbc_merkle_node_count(n);
    HB_HIP(c->st_slab.ensure(packed.size()));
    HB_HIP(c->st_aux.ensure(n * sizeof(uint64_t)));
    HB_HIP(c->st_aux2.ensure(n * sizeof(uint32_t)));
    HB_HIP(c->st_nodes.ensure(nodes * 32));
    HB_HIP(hipMemcpyAsync(c->st_slab.p, packed.data(), packed.size(), hipMemcpyHostToDevice,
                          c->stream));
    HB_HIP(hipMemcpyAsync(c->st_aux.p, offs.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice,
                          c->stream));
    HB_HIP(hipMemcpyAsync(c->st_aux2.p, ls.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice,
                          c->stream));
    uint8_t *dn = c->st_nodes.as<uint8_t>();
    HB_HIP(launch_ragged_hash(c->st_slab.as<uint8_t>(), c->st_aux.as<uint64_t>(),
                              c->st_aux2.as<uint32_t>(), n, dn, c->stream));
    size_t off = 0, sz = n;
    while (sz > 1) {
        const size_t nsz = (sz + 1) / 2;
        HB_HIP(launch_tree_level(dn, 0, off, sz, off + sz, nsz, 1, c->stream));
        off += sz;
        sz = nsz;
    }
    HB_HIP(hipMemcpyAsync(nodes_out, dn, nodes * 32, hipMemcpyDeviceToHost, c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
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
    const size_t vbytes = round_up(len, 8) + 16;
    const size_t slots = dslots + 1;
    HB_HIP(c->st_slab.ensure(vbytes));
    HB_HIP(c->st_nodes.ensure(32 * slots + 32));
    HB_HIP(c->st_aux.ensure(16));
    HB_HIP(c->st_aux3.ensure(16));
    std::vector<uint8_t> v(vbytes, 0), d(32 * slots + 32, 0);
    if (len) std::memcpy(v.data(), value, len);
    std::memcpy(d.data(), root, 32);
    if (nd_dev) std::memcpy(d.data() + 32, digests, 32 * std::min(nd_dev, ndig));
    uint8_t meta[16] = {0};
    meta[0] = (uint8_t)nd_dev;
    uint32_t idx = (uint32_t)index;
    std::memcpy(meta + 4, &idx, 4);
    HB_HIP(hipMemcpyAsync(c->st_slab.p, v.data(), vbytes, hipMemcpyHostToDevice, c->stream));
    HB_HIP(hipMemcpyAsync(c->st_nodes.p, d.data(), d.size(), hipMemcpyHostToDevice, c->stream));
    HB_HIP(hipMemcpyAsync(c->st_aux.p, meta, 16, hipMemcpyHostToDevice, c->stream));
    ValidateArgs a;
    a.values = c->st_slab.as<uint8_t>();
    a.value_len = len;
    a.value_stride = 0;
    a.value_inst_stride = 0;
    a.per_inst = 1;
    a.indices = reinterpret_cast<const uint32_t *>(c->st_aux.as<uint8_t>() + 4);
    a.digests = c->st_nodes.as<uint8_t>() + 32;
    a.dslots = slots;
    a.ndig = c->st_aux.as<uint8_t>();
    a.roots = c->st_nodes.as<uint8_t>();
    a.root_stride = 0;
    a.tree_n = n;
    a.count = 1;
    a.ok_out = c->st_aux3.as<uint8_t>();
    HB_HIP(launch_validate(a, c->stream));
    uint8_t ok = 0;
    HB_HIP(hipMemcpyAsync(&ok, a.ok_out, 1, hipMemcpyDeviceToHost, c->stream));
    HB_HIP(hipStreamSynchronize(c->stream));
    *valid_out = ok ? 1 : 0;
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
    return encode_groups(data_shards, parity_shards, spec_row_tile(data_shards, parity_shards))
        .size();
}

int hbrbc_jit_build_encode_group(size_t data_shards, size_t parity_shards, size_t group,
                                 const char *dir) {
    if (data_shards == 0 || parity_shards == 0 || data_shards + parity_shards > 256)
        return fail(HBRBC_E_INVALID_ARG, "need data >= 1, parity >= 1, data + parity <= 256");
    std::vector<uint8_t> mat;
    if (!build_matrix(data_shards, data_shards + parity_shards, mat))
        return fail(HBRBC_E_SINGULAR_MATRIX, "singular Vandermonde top block");
    const int rt = spec_row_tile(data_shards, parity_shards), depth = spec_depth();
    const auto groups = encode_groups(data_shards, parity_shards, rt);
    if (group >= groups.size()) return fail(HBRBC_E_INVALID_ARG, "group %zu of %zu", group,
                                            groups.size());
    std::vector<char> code;
    std::string log;
    if (compile_encode(data_shards, parity_shards, mat.data() + data_shards * data_shards, rt,
                       depth, groups[group].first, groups[group].second, code, log))
        return fail(HBRBC_E_DEVICE, "hiprtc: %s", log.substr(0, 400).c_str());
    const std::string d = dir ? std::string(dir) : jit_dir();
    mkdir(d.c_str(), 0755);
    const std::string path =
        jit_file(d, data_shards, parity_shards, rt, depth, groups[group].first);
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return fail(HBRBC_E_INVALID_ARG, "cannot write %s", path.c_str());
    const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
    fclose(f);
    return ok ? HBRBC_OK : fail(HBRBC_E_INVALID_ARG, "short write %s", path.c_str());
}

int hbrbc_jit_file_name(size_t data_shards, size_t parity_shards, size_t group, char *buf,
                        size_t buf_len) {
    if (data_shards == 0 || parity_shards == 0 || !buf)
        return fail(HBRBC_E_INVALID_ARG, "need data >= 1, parity >= 1, a buffer");
    const int rt = spec_row_tile(data_shards, parity_shards);
    const auto groups = encode_groups(data_shards, parity_shards, rt);
    if (group >= groups.size()) return fail(HBRBC_E_INVALID_ARG, "group %zu of %zu", group,
                                            groups.size());
    const std::string f = jit_file("", data_shards, parity_shards, rt, spec_depth(),
                                   groups[group].first).substr(1);
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
    for (auto &r : c->recs) {
        (void)r;
    }
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

}  // extern "C"
