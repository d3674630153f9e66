// sim.hip -- the Reliable-Broadcast state machine of many instances and nodes
// on the GPU (GPU-resident Echo / EchoHash / Ready /
// CanDecode counters and left/right targeting for the validator-sharded
// simulation).
//
// Reference: /root/reference/src/broadcast/broadcast.rs:228-558 (handle_value,
// handle_echo, handle_echo_hash, handle_can_decode, handle_ready, the senders
// and compute_output), restated handler by handler below; the host
// restatement hbbft_amd/broadcast.py is the checker (tests/test_rbc_sim.py).
//
// Model.  Messages move in synchronous rounds: what a node emits in round t
// is delivered in round t + 1, and a node handles its inbox in (sender index,
// emission order) -- one deterministic schedule of the reference's
// asynchronous network, which tests/virtual_net.py RoundNet runs through the
// host state machine.  Round 0 is the proposer's `broadcast()`.  One thread
// per (instance, hosted node) runs the handlers sequentially; all threads of
// a workgroup scan the same message records, so the inbox loop is uniform.
//
// Data plane vs control plane.  A message carries a proof by reference:
// (root c, index j, tampered t) names row j of codeword c (or its corrupted
// copy); Proof::validate of every such proof is a pure function computed by
// the batched validate kernel (proof_ok), and decode_from_shards of root c by
// the batched decode (decode_ok) -- every stored full Echo of root c is a
// validated row of codeword c, and a codeword decodes from any k of its rows
// (MDS), so the decode outcome of root c does not depend on which rows a
// receiver holds.  Roots are small ids (codeword slots per instance).
//
// Adversaries (the scenario): a proposer that sends different codewords or
// nothing to some validators (value_root / value_tamper per recipient);
// faulty nodes that drop everything they would send (ProposeAdversary with
// drop, tests/broadcast.rs:33-98), corrupt or withhold their Echoes; and the
// ProposeAdversary's fake broadcasts: after its first delivered message,
// `fake_from` emits every listed faulty node's Broadcast of its own value
// (Values to all others, Echo to its left nodes, EchoHash to its right
// nodes) as its own messages.
#include "launchers.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

// Kernel forms (launch_sm_round picks one per round): where the state and
// records live -- global (sm_round_kernel), LDS-staged state and records
// (sm_round_staged_kernel), LDS-staged state with the records read from the
// all-gathered inbox through the scalar cache (sm_round_grec_kernel, nodes %
// 64 == 0) -- each at the default register budget or at 4 waves/SIMD (_w4);
// the handler set LV (Sm::deliver: every handler, or without the Fake / Value
// handlers for batches marked HBRBC_SM_NO_FAKE); and for the staged form WI,
// every wave one instance (the record dispatch as scalar branches).  Round 5
// (DESIGN.md 6c): the smaller handler sets, the scalar dispatch, the
// pointer-walking cursor, sender-flagged Echo / EchoHash pairs and vote-
// guarded rare steps took N=128 from 1.07 to 0.73 ms and N=64 from 0.65 to
// 0.52 ms per run of tools/sm_bench.py.

// Compile-time A/B switches of the one-root round kernel (round 4):
// HB_SM_CACHE keeps the inbox loop's 32-sender mask word in registers,
// HB_SM_MERGE takes a sender's Echo and EchoHash in one step.  Measured
// (tools/sm_bench.py, one MI355X, ms per 5 rounds of 262,144 nodes, N=64 /
// N=128): neither 0.670 / 1.368, merge 0.663 / 1.309, cache 0.690 / 1.470,
// both 0.683 / 1.460 -- the cached word costs registers (more spills at 4
// waves/SIMD) for LDS round trips the other waves were hiding.
#ifndef HB_SM_CACHE
#define HB_SM_CACHE 0
#endif
#ifndef HB_SM_MERGE
#define HB_SM_MERGE 1
#endif
// HB_SM_SELECT: the one-root Echo / EchoHash handler as predicated selects
// (handle_echo_sel; round 5, default: sm_bench N=64 0.649-0.662 -> 0.625-0.630
// ms, N=128 1.011-1.022 -> 0.993-1.001 ms, profiles/r5i_sm_select_ab.jsonl)
#ifndef HB_SM_SELECT
#define HB_SM_SELECT 1
#endif
// Global-records kernel: HB_SM_CONSTAS reads the inbox through the constant
// address space, so the wave-uniform reads (counts, record headers) are
// scalar loads; the recipient-mask word is per lane (a wave holds nodes of
// different 32-node words) and stays one vector load per record.  The typed
// pointer goes all the way into sm_node (it was cast back to a
// generic pointer there).  Checked in the ISA (hipcc -S, round 5, before and
// after that change): the inbox loop of sm_round_grec_kernel<true> reads a
// sender's count and each record header with s_load_dword and the mask word
// with one global_load_dword (offset 4 / 8: words 1.. of the record).
#ifndef HB_SM_CONSTAS
#define HB_SM_CONSTAS 1
#endif

namespace hbrbc {

namespace {

constexpr uint32_t kNone = 0xFFu;
// record header: kind | root << 8 | index << 16 | tamper << 24; bit 7 of the
// kind byte marks an Echo whose next record is the EchoHash of the same
// handle_value step (disjoint targets: the receivers merge the two, below)
constexpr uint32_t kKindMask = 0x7Fu, kPairFlag = 0x80u;

// A rare lane-divergent step behind a wave-wide test: HB_RARE(c) { if (c) ... }
// skips with one vote and a uniform branch where a plain divergent `if` costs
// an exec-mask save, a branch and a restore on every record (HB_SM_RARE=0:
// plain ifs, A/B).
#ifndef HB_SM_RARE
#define HB_SM_RARE 1
#endif
#if HB_SM_RARE
#define HB_RARE(c) if (__builtin_expect(__any(c), 0))
#else
#define HB_RARE(c) if (true)
#endif

// message kinds (broadcast::Message, message.rs:13-24) + the fake block
enum { K_VALUE = 0, K_ECHO = 1, K_READY = 2, K_CAN_DECODE = 3, K_ECHO_HASH = 4, K_FAKE = 5 };
// FaultKind (error.rs:28-50), in declaration order
enum {
    F_VALUE_FROM_NON_PROPOSER = 0,
    F_MULTIPLE_VALUES = 1,
    F_MULTIPLE_ECHOS = 2,
    F_MULTIPLE_ECHO_HASHES = 3,
    F_MULTIPLE_READYS = 4,
    F_INVALID_PROOF = 5,
    F_BROADCAST_DECODING = 6
};
enum { R_HONEST = 0, R_SILENT = 1, R_CORRUPT_ECHO = 2, R_WITHHOLD_ECHO = 3 };
// flags
enum : uint32_t {
    FL_READY_SENT = 1u,
    FL_ECHO_SENT = 2u,
    FL_ECHO_HASH_SENT = 4u,
    FL_DECIDED = 8u,
    FL_FAKE_DONE = 16u,
    FL_VALUE_SENT = 32u,
    FL_CAN_DECODE_SHIFT = 8u,   // bits 8..15: can_decode_sent per root
};

// Per sender s a node keeps one 16-bit word (er[s]): bits 0..7 the echo
// entry (EchoContent) -- 0 none, Hash: 0x10 | c, Full: 0x20 | t << 3 | c (a
// stored full Echo is always proof index s, validate_proof checks it) -- and
// bits 8..11 the Ready entry (root + 1, 0 none).  With one root (c = 0,
// Sm<true>) an entry is three bits -- hash, full, tampered -- and the Ready
// entry one: bit s of four masks {hash, full, tamper, ready} per 32 senders,
// one 16-byte LDS word (N=128: 64 bytes per node instead of 128 + a 16-byte
// full-Echo mask).
__device__ __forceinline__ uint32_t enc_full(uint32_t c, uint32_t t) {
    return 0x20u | ((t & 1u) << 3) | (c & 7u);
}
__device__ __forceinline__ uint32_t enc_hash(uint32_t c) { return 0x10u | (c & 7u); }
__device__ __forceinline__ bool is_full(uint32_t e) { return e & 0x20u; }
__device__ __forceinline__ bool is_hash(uint32_t e) { return e & 0x10u; }
__device__ __forceinline__ uint32_t root_of(uint32_t e) { return e & 7u; }
__device__ __forceinline__ uint32_t tamper_of(uint32_t e) { return (e >> 3) & 1u; }

// ONE: a single codeword slot (roots == 1, the validator-sharded runs): the
// node's Echo / full-Echo / Ready counters and its flags live in registers
// for the round (the handlers are chains of dependent read-modify-writes of
// them), written back at the end.
template <bool ONE>
struct Sm {
    const hbrbc_sm_args &a;
    int n, f, k, W, C, rec;   // rec: uint32 words per message record (1 + W)
    size_t inst;
    int me, proposer, role;
    bool drop;                // a silent node's deliveries emit nothing
    // state of (inst, me), structure of arrays over the instance's hosted
    // nodes (stride sd = nodes): the nodes of an instance are consecutive
    // threads, so every state access of a wave is one coalesced request
    // [n][sd]: echo entry | ready entry << 8 (er16); with one root (ONE:
    // every root index is 0, so ready = 1) [W][sd] masks {hash, full,
    // tamper, ready} (em): a third of the LDS image, more resident workgroups
    uint16_t *er16;
    uint4 *em;
    uint32_t *cand;           // [C][W][sd]
    uint32_t *full;           // [W][sd]: senders whose entry is a full Echo (ONE: em .y)
    uint16_t *cnt;            // [3][C][sd]: Echo+EchoHash, full Echo, Ready counts
    uint32_t *flags;          // [sd]
    size_t sd;
    const uint8_t *pok;       // this instance's proof_ok [C][2][n]
    const uint8_t *dok;       // this instance's decode_ok [C]

    // ONE: the mask word of the 32 senders the inbox loop is at lives in
    // registers (cache, word cw; the loop walks senders in order, so it moves
    // once per 32 senders): the handlers' read-modify-writes of a sender's
    // entry cost no LDS round trip.  Other words (a node's own entry, the
    // full-Echo masks of a CanDecode) go to LDS.
    uint4 cache = {0u, 0u, 0u, 0u};
    int cw = -1;
    __device__ __forceinline__ uint4 em_get(int w) const {
#if HB_SM_CACHE
        // a select of values, not of addresses (a pointer select between the
        // register copy and LDS would put the whole Sm object on the stack)
        // -- LLVM folds "if (c) v = *p else v = *q" into a load through a
        // selected pointer; the empty asm keeps the register arm a register)
        uint4 v;
        if (w == cw) {
            v = cache;
            __asm__ volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
        } else {
            v = em[(size_t)w * sd];
        }
        return v;
#else
        // (no register copy: the compiler did not fold the never-taken
        // register arm away, and its lane-mask select ran on every access)
        return em[(size_t)w * sd];
#endif
    }
    __device__ __forceinline__ void em_put(int w, const uint4 &v) {
#if HB_SM_CACHE
        if (w == cw) {
            uint4 t = v;
            __asm__ volatile("" : "+v"(t.x), "+v"(t.y), "+v"(t.z), "+v"(t.w));
            cache = t;
        } else {
            em[(size_t)w * sd] = v;
        }
#else
        em[(size_t)w * sd] = v;
#endif
    }
    __device__ __forceinline__ void em_focus(int w) {   // w uniform across the wave
        if constexpr (ONE && HB_SM_CACHE) {
            if (w == cw) return;
            if (cw >= 0) em[(size_t)cw * sd] = cache;
            cache = em[(size_t)w * sd];
            cw = w;
        }
    }
    __device__ __forceinline__ void em_flush() {
        if constexpr (ONE && HB_SM_CACHE) {
            if (cw >= 0) em[(size_t)cw * sd] = cache;
            cw = -1;
        }
    }
    __device__ __forceinline__ uint32_t ECHO(int s) const {
        if constexpr (ONE) {
            const uint4 v = em_get(s >> 5);
            const uint32_t b = 1u << (s & 31);
            return (v.y & b) ? (0x20u | ((v.z & b) ? 8u : 0u)) : ((v.x & b) ? 0x10u : 0u);
        } else {
            return er16[(size_t)s * sd] & 0xFFu;
        }
    }
    __device__ __forceinline__ void set_echo(int s, uint32_t e) {
        if constexpr (ONE) {
            const uint32_t b = 1u << (s & 31);
            uint4 t = em_get(s >> 5);
            t.x = (e & 0x10u) ? (t.x | b) : (t.x & ~b);
            t.y = (e & 0x20u) ? (t.y | b) : (t.y & ~b);
            t.z = (e & 0x28u) == 0x28u ? (t.z | b) : (t.z & ~b);
            em_put(s >> 5, t);
        } else {
            uint16_t &w = er16[(size_t)s * sd];
            w = (uint16_t)((w & 0xFF00u) | e);
        }
    }
    __device__ __forceinline__ uint32_t READY(int s) const {
        if constexpr (ONE) return (em_get(s >> 5).w >> (s & 31)) & 1u;
        else return er16[(size_t)s * sd] >> 8;
    }
    __device__ __forceinline__ void set_ready(int s, uint32_t r) {
        if constexpr (ONE) {
            const uint32_t b = 1u << (s & 31);
            uint4 t = em_get(s >> 5);
            t.w = r ? (t.w | b) : (t.w & ~b);
            em_put(s >> 5, t);
        } else {
            uint16_t &w = er16[(size_t)s * sd];
            w = (uint16_t)((w & 0xFFu) | (r << 8));
        }
    }
    __device__ __forceinline__ uint32_t &CAND(uint32_t c, int w) { return cand[((size_t)c * W + w) * sd]; }
    __device__ __forceinline__ uint32_t &FULL(int w) { return full[(size_t)w * sd]; }   // (several roots)
    __device__ __forceinline__ uint32_t full_word(int w) const {
        if constexpr (ONE) return em_get(w).y;
        else return full[(size_t)w * sd];
    }
    uint16_t r_ce = 0, r_cf = 0, r_cr = 0;
    uint32_t r_flags = 0;
    __device__ __forceinline__ uint16_t &CE(uint32_t c) {
        if constexpr (ONE) return r_ce;
        else return cnt[(size_t)c * sd];
    }
    __device__ __forceinline__ uint16_t &CF(uint32_t c) {
        if constexpr (ONE) return r_cf;
        else return cnt[((size_t)C + c) * sd];
    }
    __device__ __forceinline__ uint16_t &CR(uint32_t c) {
        if constexpr (ONE) return r_cr;
        else return cnt[((size_t)2 * C + c) * sd];
    }
    __device__ __forceinline__ uint32_t &FLAGS() {
        if constexpr (ONE) return r_flags;
        else return *flags;
    }
    __device__ __forceinline__ void cache_in() {
        if constexpr (ONE) {
            r_ce = cnt[0];
            r_cf = cnt[sd];
            r_cr = cnt[2 * sd];
            r_flags = *flags;
        }
    }
    __device__ __forceinline__ void cache_out() {
        if constexpr (ONE) {
            cnt[0] = r_ce;
            cnt[sd] = r_cf;
            cnt[2 * sd] = r_cr;
            *flags = r_flags;
        }
    }
    uint32_t *out;            // [max_out][rec]
    uint32_t nout;
    bool overflow;
    uint16_t *faults;
    uint32_t nfault;

    __device__ __forceinline__ bool bit(const uint32_t *m, int i) const { return (m[i >> 5] >> (i & 31)) & 1u; }

    __device__ __forceinline__ void fault(int node, int kind) {
        if (nfault < a.max_faults) faults[nfault] = (uint16_t)((node << 8) | kind);
        ++nfault;
    }

    // right_nodes (broadcast.rs:476-485): the f nodes before us on the circle
    __device__ __forceinline__ bool is_right_of(int j, int i) const {
        const int d = (i - j + n) % n;   // j = i - d
        return d >= 1 && d <= f;
    }

    __device__ __forceinline__ uint32_t *emit_rec(uint32_t kind, uint32_t c, uint32_t j, uint32_t t) {
        if (nout >= a.max_out) {
            overflow = true;
            return nullptr;
        }
        uint32_t *r = out + (size_t)nout * rec;
        ++nout;
        r[0] = kind | (c << 8) | (j << 16) | (t << 24);
        return r;
    }

    // Recipient masks word by word (bit operations, not a loop over n: the
    // lanes of a wave reach a send at different senders, so a per-node loop
    // would run once per distinct trigger point).  lin(w, a, b): bits [a, b)
    // of word w.
    __device__ __forceinline__ static uint32_t lin(int w, int a, int b) {
        const int lo = a > 32 * w ? a : 32 * w, hi = b < 32 * w + 32 ? b : 32 * w + 32;
        if (hi <= lo) return 0u;
        const int len = hi - lo;
        return (len >= 32 ? 0xFFFFFFFFu : ((1u << len) - 1u)) << (lo - 32 * w);
    }
    __device__ __forceinline__ uint32_t all_but_me(int w) const {
        // lin(w, 0, n): whole words, then the partial last one (a few scalar
        // ops instead of lin's clamps; it runs once per word of every send)
        const int fw = n >> 5;
        const uint32_t all = w < fw ? 0xFFFFFFFFu : (w == fw ? (1u << (n & 31)) - 1u : 0u);
        return all & ~((me >> 5) == w ? 1u << (me & 31) : 0u);
    }
    // right_nodes(me) (broadcast.rs:476-485): [me - f, me) on the circle
    __device__ __forceinline__ uint32_t right_mask(int w) const {
        const int a0 = me - f;
        return a0 >= 0 ? lin(w, a0, me) : (lin(w, 0, me) | lin(w, a0 + n, n));
    }
    template <class M>
    __device__ __forceinline__ void targets_w(uint32_t *r, M mask) {
        for (int w = 0; w < W; ++w) r[1 + w] = mask(w);
    }

    // emission as the node's own step (subject to its role)
    __device__ __forceinline__ uint32_t *emit(uint32_t kind, uint32_t c, uint32_t j = 0, uint32_t t = 0) {
        if (drop) return nullptr;
        if (kind == K_ECHO && role == R_WITHHOLD_ECHO) return nullptr;
        if (kind == K_ECHO && role == R_CORRUPT_ECHO) t = 1;
        return emit_rec(kind, c, j, t);
    }

    __device__ __forceinline__ bool validate_proof(uint32_t c, uint32_t j, uint32_t t, int sender) const {
        if ((int)j != sender || c >= (uint32_t)C || j >= (uint32_t)n) return false;
        return pok[(c * 2 + (t & 1)) * n + j] != 0;
    }

    // -- handlers (broadcast.rs) --------------------------------------------
    __device__ __forceinline__ void compute_output(uint32_t c) {   // 526-558
        const bool fire = !(FLAGS() & FL_DECIDED) && CR(c) > 2 * f && CF(c) >= k;
        HB_RARE(fire) {
            if (fire) output_now(c);
        }
    }
    __device__ __forceinline__ void output_now(uint32_t c) {
        if (dok[c]) {
            FLAGS() |= FL_DECIDED;
            a.output_root[inst * a.nodes + (me - a.node_lo)] = (uint8_t)c;
        } else {
            fault(proposer, F_BROADCAST_DECODING);
        }
    }

    __device__ __forceinline__ void send_echo_remaining(uint32_t c) {   // 428-453
        FLAGS() |= FL_ECHO_SENT;
        const uint32_t e = ECHO(me);
        if (!is_full(e) || root_of(e) != c) return;
        uint32_t *r = emit(K_ECHO, c, (uint32_t)me, tamper_of(e));
        if (!r) return;
        targets_w(r, [&](int w) { return right_mask(w) & ~CAND(c, w); });
    }

    __device__ __forceinline__ void handle_ready_core(int s, uint32_t c, bool may_send);

    __device__ __forceinline__ void send_ready(uint32_t c) {   // 513-522
        FLAGS() |= FL_READY_SENT;
        uint32_t *r = emit(K_READY, c);
        if (r) targets_w(r, [&](int w) { return all_but_me(w); });
        handle_ready_core(me, c, false);
    }

    __device__ __forceinline__ void handle_can_decode(int s, uint32_t c) {   // 358-375
        CAND(c, s >> 5) |= 1u << (s & 31);
    }

    __device__ __forceinline__ void send_can_decode(uint32_t c) {   // 488-510
        FLAGS() |= 1u << (FL_CAN_DECODE_SHIFT + c);
        uint32_t *r = emit(K_CAN_DECODE, c);
        if (r) targets_w(r, [&](int w) { return all_but_me(w) & ~full_word(w); });
        handle_can_decode(me, c);
    }

    // handle_echo (266-320, full = true) and handle_echo_hash (322-355, full =
    // false) in one body: the checks and faults differ per kind, the counter
    // updates, the entry and the thresholds are shared code, so a wave whose
    // lanes take different kinds for the same sender (Echo for the left
    // nodes, EchoHash for the right ones) runs the common part once.
    __device__ __forceinline__ void handle_echo_any(int s, uint32_t c, uint32_t j, uint32_t t,
                                                    bool full) {
#if HB_SM_SELECT
        if constexpr (ONE) {
            handle_echo_sel(s, c, j, t, full);
            return;
        }
#endif
        const uint32_t e = ECHO(s);
        int fk = -1;
        bool stop = false;
        if (full) {
            if (is_full(e)) {   // the stored proof is (root_of(e), s, tamper_of(e))
                if (e != enc_full(c, t) || (int)j != s) fk = F_MULTIPLE_ECHOS;
                stop = true;
            } else if (is_hash(e) && root_of(e) != c) {
                fk = F_MULTIPLE_ECHOS;
                stop = true;
            } else if (!validate_proof(c, j, t, s)) {
                fk = F_INVALID_PROOF;
                stop = true;
            }
        } else if (e) {
            if (root_of(e) != c) fk = F_MULTIPLE_ECHO_HASHES;
            stop = true;
        }
        if (fk >= 0) fault(s, fk);
        if (stop) return;
        if (!e) ++CE(c);   // (full: a Hash of the same root was counted already)
        if (full) {
            ++CF(c);
            if constexpr (!ONE) FULL(s >> 5) |= 1u << (s & 31);
        }
        set_echo(s, full ? enc_full(c, t) : enc_hash(c));   // (ONE: the full bit too)
        if (full && !(FLAGS() & (1u << (FL_CAN_DECODE_SHIFT + c))) && CF(c) >= k)
            send_can_decode(c);
        // Echo: send Ready at N - f, then compute_output once Ready is sent;
        // EchoHash: send Ready at N - f, else compute_output
        if (!(FLAGS() & FL_READY_SENT) && CE(c) >= n - f) {
            send_ready(c);
            if (full) compute_output(c);
        } else if (!full || (FLAGS() & FL_READY_SENT)) {
            compute_output(c);
        }
    }
    // The same handler with its common path as straight-line predicated
    // work (one root): every check and counter update is a select, the mask
    // word is read and written once, and only the rare steps -- a fault, the
    // CanDecode and Ready sends, an output -- stay behind branches (each one
    // guarded by a wave-wide test, so a wave in which no lane takes it skips
    // it with one scalar branch).  Same order of effects as handle_echo_any:
    // fault, entry and counters, CanDecode, Ready, compute_output.
    __device__ __forceinline__ void handle_echo_sel(int s, uint32_t c, uint32_t j, uint32_t t,
                                                    bool full) {
        const int w = s >> 5;
        const uint32_t b = 1u << (s & 31);
        uint4 m4 = em_get(w);
        const bool eh = m4.x & b, ef = m4.y & b, et = m4.z & b;   // entry: hash / full / tampered
        const bool any = eh || ef;
        // handle_echo (266-320): a stored full Echo of the same proof is a
        // no-op, another one a MultipleEchos; a hash of another root too; a
        // proof that does not validate an InvalidProof
        const bool same_full = ef && !(et ^ (t & 1u)) && c == 0u && (int)j == s;
        const bool bad_hash = eh && !ef && c != 0u;   // (one root: root_of(e) == 0)
        bool stop, flt;
        int fk;
        if (full) {
            const bool vp = validate_proof(c, j, t, s);
            stop = ef || bad_hash || !vp;
            flt = (ef && !same_full) || bad_hash || (!ef && !bad_hash && !vp);
            fk = (ef || bad_hash) ? F_MULTIPLE_ECHOS : F_INVALID_PROOF;
        } else {   // handle_echo_hash (322-355)
            stop = any;
            flt = any && c != 0u;
            fk = F_MULTIPLE_ECHO_HASHES;
        }
        HB_RARE(flt) {
            if (flt) fault(s, fk);
        }
        const bool go = !stop;
        r_ce += (go && !any) ? 1 : 0;
        r_cf += (go && full) ? 1 : 0;
        // the entry: full (with its tamper bit) or hash
        const uint32_t gb = go ? b : 0u;
        m4.x = full ? (m4.x & ~gb) : (m4.x | gb);
        m4.y = full ? (m4.y | gb) : m4.y;
        m4.z = (full && (t & 1u)) ? (m4.z | gb) : m4.z;
        em_put(w, m4);
        const bool cd = go && full && !(r_flags & (1u << FL_CAN_DECODE_SHIFT)) && r_cf >= (uint32_t)k;
        const bool rd_ok = go && !(r_flags & FL_READY_SENT) && r_ce >= (uint32_t)(n - f);
        const bool co = go && (rd_ok ? full : (!full || (r_flags & FL_READY_SENT)));
        HB_RARE(cd) {
            if (cd) send_can_decode(c);
        }
        HB_RARE(rd_ok) {
            if (rd_ok) send_ready(c);
        }
        if (co) compute_output(c);
    }
    __device__ __forceinline__ void handle_echo(int s, uint32_t c, uint32_t j, uint32_t t) {
        handle_echo_any(s, c, j, t, true);
    }
    __device__ __forceinline__ void handle_echo_hash(int s, uint32_t c) {
        handle_echo_any(s, c, 0, 0, false);
    }

    __device__ __forceinline__ void send_echo_hash(uint32_t c) {   // 456-468
        FLAGS() |= FL_ECHO_HASH_SENT;
        uint32_t *r = emit(K_ECHO_HASH, c);
        if (r) targets_w(r, [&](int w) { return right_mask(w); });
        handle_echo_hash(me, c);
    }

    __device__ __forceinline__ void send_echo_left(uint32_t c, uint32_t j, uint32_t t) {   // 413-425
        uint32_t *r = emit(K_ECHO, c, j, t);
        if (r) targets_w(r, [&](int w) { return all_but_me(w) & ~right_mask(w); });
        handle_echo(me, c, j, t);
    }

    // rotate out[a0, a1) behind out[a1, nout) (and the same for faults):
    // echo_steps.join(echo_hash_steps) lists the Echo step first although the
    // EchoHash step ran first (broadcast.rs:258-262)
    __device__ __forceinline__ void rotate_tail(uint32_t m0, uint32_t m1, uint32_t f0, uint32_t f1) {
        // messages: at most max_out records, rotated one record at a time
        const uint32_t nb = m1 - m0, na = nout - m1;
        for (uint32_t s = 0; s < nb; ++s) {   // move record m0 to the end, nb times
            for (int w = 0; w < rec; ++w) {
                const uint32_t first = out[(size_t)m0 * rec + w];
                for (uint32_t q = m0; q + 1 < m0 + nb + na; ++q)
                    out[(size_t)q * rec + w] = out[(size_t)(q + 1) * rec + w];
                out[(size_t)(m0 + nb + na - 1) * rec + w] = first;
            }
        }
        const uint32_t lim = nfault < a.max_faults ? nfault : a.max_faults;
        if (f1 > lim) f1 = lim;
        if (f0 > f1) f0 = f1;
        const uint32_t fb = f1 - f0, fa = lim - f1;
        for (uint32_t s = 0; s < fb; ++s) {
            const uint16_t first = faults[f0];
            for (uint32_t q = f0; q + 1 < f0 + fb + fa; ++q) faults[q] = faults[q + 1];
            faults[f0 + fb + fa - 1] = first;
        }
    }

    __device__ __forceinline__ void handle_value(int s, uint32_t c, uint32_t j, uint32_t t) {   // 228-263
        if (s != proposer) {
            fault(s, F_VALUE_FROM_NON_PROPOSER);
            return;
        }
        const uint32_t e = ECHO(me);
        if (e) {
            if (root_of(e) != c) {
                fault(s, F_MULTIPLE_VALUES);
                return;
            }
            if (is_full(e) && e == enc_full(c, t)) return;   // j == me: the stored index
        }
        if (!validate_proof(c, j, t, me)) {
            fault(s, F_INVALID_PROOF);
            return;
        }
        const uint32_t m0 = nout, f0 = nfault;
        send_echo_hash(c);
        const uint32_t m1 = nout, f1 = nfault;
        send_echo_left(c, j, t);
        const uint32_t fl = nfault < a.max_faults ? nfault : a.max_faults;
        if (!overflow && m1 == m0 + 1 && nout == m1 + 1 && (f1 == f0 || fl <= f1)) {
            // the common step -- one EchoHash record, one Echo record, no
            // fault to move: both records are read at once and written back
            // swapped, the Echo flagged (one load round trip instead of the
            // rotation's one per word, and no second pass for the flag)
            uint32_t ea[9], eb[9];
#pragma unroll
            for (int w = 0; w < 9; ++w) {
                const int ww = w < rec ? w : rec - 1;   // rec <= 9 (n <= 256)
                ea[w] = out[(size_t)m0 * rec + ww];
                eb[w] = out[(size_t)m1 * rec + ww];
            }
            if ((eb[0] & kKindMask) == K_ECHO && (ea[0] & kKindMask) == K_ECHO_HASH) eb[0] |= kPairFlag;
#pragma unroll
            for (int w = 0; w < 9; ++w) {
                if (w < rec) {
                    out[(size_t)m0 * rec + w] = eb[w];
                    out[(size_t)m1 * rec + w] = ea[w];
                }
            }
        } else if (!overflow) {
            rotate_tail(m0, m1, f0, f1);
            // After the rotation send_echo_left's records are [m0, m0 + ne),
            // the EchoHash step's follow.  Flag only send_echo_left's own Echo
            // (at m0, to all but the right nodes), and only when the step's
            // EchoHash (to the right nodes) directly follows it -- its Echo
            // step emitted one record.  Any other Echo (send_echo_remaining's,
            // to the right nodes too) is never flagged: its targets overlap
            // the EchoHash's, and the receiver's merged step assumes disjoint
            // targets.
            const uint32_t ne = nout - m1;
            if (ne == 1 && m0 + 1 < nout) {
                uint32_t &h = out[(size_t)m0 * rec];
                if ((h & kKindMask) == K_ECHO && (out[(size_t)(m0 + 1) * rec] & kKindMask) == K_ECHO_HASH)
                    h |= kPairFlag;
            }
        }
    }

    // the ProposeAdversary's injected step: per listed faulty node F (in index
    // order) its fresh Broadcast's messages -- Value(proof j) to every j != F,
    // Echo(proof F) to AllExcept(right(F)), EchoHash to right(F) -- all sent
    // by the dispatching node; a receiver handles the ones addressed to it
    __device__ __forceinline__ void handle_fake(int s, uint32_t c) {
        const uint32_t *list = a.fake_list + inst * W;
        for (int F = 0; F < n; ++F) {
            if (!bit(list, F)) continue;
            if (me != F) handle_value(s, c, (uint32_t)me, 0);
            if (!is_right_of(me, F)) handle_echo(s, c, (uint32_t)F, 0);
            else handle_echo_hash(s, c);
        }
    }

    // h0: the record's header word.  LV (handler set): 0 every handler; in a
    // batch without injected broadcasts (no Fake records: those come only
    // from a fake_from node) 1 -- round 1: no Fake handler -- and 2 -- rounds
    // >= 2, whose inboxes hold only Echo / EchoHash / Ready / CanDecode
    // records (Values go out in round 0 only): no Value handler either.  A
    // record of a kind not compiled in sets `bad` (the launch reports it,
    // emitted[1] bit 1).
    bool bad = false;
    template <int LV>
    // k0: the kind of the step's first record, which a merged Echo /
    // EchoHash step shares with its second (the class): wave-uniform in the
    // global-records kernel, so the dispatch is a scalar branch even where the
    // lanes of a merged step take different kinds (the per-lane kind is only
    // the handler's `full` operand)
    __device__ __forceinline__ void deliver(int s, uint32_t h0, uint32_t k0) {
        const uint32_t kind = h0 & kKindMask, c0 = (h0 >> 8) & 0xFFu;
        const uint32_t j = (h0 >> 16) & 0xFFu, t = (h0 >> 24) & 0xFFu;
        if constexpr (LV == 2) {
            // the round's common kinds first (a switch became a compare tree)
            if (((1u << K_ECHO) | (1u << K_ECHO_HASH)) >> k0 & 1u)
                handle_echo_any(s, c0, j, t, kind == K_ECHO);
            else if (k0 == K_READY)
                handle_ready_core(s, c0, true);
            else if (k0 == K_CAN_DECODE)
                handle_can_decode(s, c0);
            else if (k0 == K_VALUE || k0 == K_FAKE)
                bad = true;
            return;
        }
        switch (k0) {
            case K_VALUE: {
                // the proposer's Value to us: proof (value_root[me], me, value_tamper[me]);
                // an explicit root (fake Values) carries proof (c0, me, 0)
                uint32_t c = c0, tt = 0;
                if (c == kNone) {
                    c = a.value_root[inst * n + me];
                    tt = a.value_tamper[inst * n + me];
                }
                handle_value(s, c, (uint32_t)me, tt);
                break;
            }
            case K_ECHO:   // one inlined body for both kinds (lanes of a merged
            case K_ECHO_HASH:   // Echo / EchoHash step take different kinds)
                handle_echo_any(s, c0, j, t, kind == K_ECHO);
                break;
            case K_READY: handle_ready_core(s, c0, true); break;
            case K_CAN_DECODE: handle_can_decode(s, c0); break;
            case K_FAKE:
                if constexpr (LV == 0) handle_fake(s, c0);
                else bad = true;
                break;
            default: break;
        }
    }
};

template <bool ONE>
__device__ __forceinline__ void Sm<ONE>::handle_ready_core(int s, uint32_t c, bool may_send) {   // 378-410
    if constexpr (ONE) {
        // one root: the entry is bit s of the Ready mask (stored root 0), and
        // the common path -- a fresh Ready: set the bit, count it -- is
        // predicated; the fault, the sends and the output stay behind
        // branches, each condition read after the step before it ran (as in
        // the branchy form below: send_ready moves the count)
        const int w = s >> 5;
        const uint32_t b = 1u << (s & 31);
        uint4 m4 = em_get(w);
        const bool had = m4.w & b;
        HB_RARE(had && c != 0u) {
            if (had && c != 0u) fault(s, F_MULTIPLE_READYS);
        }
        const bool go = !had;
        m4.w |= go ? b : 0u;
        em_put(w, m4);
        r_cr += go ? 1 : 0;
        {
            const bool sr = go && may_send && r_cr == f + 1 && !(r_flags & FL_READY_SENT);
            HB_RARE(sr) {
                if (sr) send_ready(c);
            }
        }
        {
            const bool ser = go && r_cr == 2 * f + 1;   // (after send_ready moved the count)
            HB_RARE(ser) {
                if (ser) send_echo_remaining(c);
            }
        }
        if (go) compute_output(c);
        return;
    }
    const uint32_t old = READY(s);
    if (old) {
        if (old - 1 != c) fault(s, F_MULTIPLE_READYS);
        return;
    }
    set_ready(s, c + 1);
    ++CR(c);
    // (from send_ready, ready_sent is already set: no further send_ready)
    if (may_send && CR(c) == f + 1 && !(FLAGS() & FL_READY_SENT)) send_ready(c);
    if (CR(c) == 2 * f + 1) send_echo_remaining(c);
    compute_output(c);
}


// Byte offsets of the fields of an instance's state block holding `sd` nodes
// as structures of arrays (launchers.hpp sm_state_bytes, per node: er u16[n]
// or, with one root, masks u32x4[W]; cand u32[C][W]; full u32[W] (not with
// one root); counters u16[3][C]; flags u32).
struct SmLayout {
    size_t er, cand, full, cnt, flags;
    __device__ __forceinline__ SmLayout(int n, int C, int W, size_t sd) {
        er = 0;
        cand = (sm_er_bytes((size_t)n, (size_t)C) * sd + 3) & ~(size_t)3;
        full = cand + 4 * (size_t)C * W * sd;
        cnt = full + (C == 1 ? 0 : 4 * (size_t)W * sd);
        flags = (cnt + 6 * (size_t)C * sd + 3) & ~(size_t)3;
    }
};

// The inbox of one instance, walked sender by sender in order: sender s's
// record count and records sit at index idx(s) = ((s / R) * count + inst) * R
// + s % R of the all-gathered inbox (sm_in_block), or at s in a staged LDS
// copy (R = 0: no blocks).  The count and record pointers move incrementally
// -- one sender, and (count - 1) * R more after the last sender of a rank's
// block -- instead of the
// per-sender 32-bit division and 64-bit products of sm_in_block, which the
// ISA showed as ~50 scalar instructions per sender ahead of every record
// read (round 5: the inbox loop was bound by the CU's scalar unit,
// profiles/r5e_sm_counters.txt).  P: the pointer type (the global-records
// kernel keeps the constant address space).  WI: every lane of a wave walks
// the same instance's inbox (the LDS-staged kernel at nodes % 64 == 0), so a
// count or header read per lane is moved to a scalar register.
template <class P, bool WI = false>
struct SmInbox {
    static constexpr bool kWaveInst = WI;
    P cp, rp;          // this sender's count word and first record
    size_t jump, jumpr;  // (count - 1) * R count words, and their records
    uint32_t rr, R, MR, max_out;
    __device__ __forceinline__ uint32_t count() const {
        const uint32_t c = *cp & 0x7FFFFFFFu;
        return c < max_out ? c : max_out;
    }
    __device__ __forceinline__ P recs() const { return rp; }
    __device__ __forceinline__ void advance() {
        ++cp;
        rp += MR;
        if (R && ++rr == R) {
            rr = 0;
            cp += jump;
            rp += jumpr;
        }
    }
};
template <class P, bool WI = false>
__device__ __forceinline__ SmInbox<P, WI> sm_inbox(P cnt, P rec, size_t inst, size_t count,
                                                   uint32_t R, uint32_t MR, uint32_t max_out) {
    SmInbox<P, WI> b;
    const size_t idx = R ? inst * R : 0;   // sender 0: block 0, row 0
    b.cp = cnt + idx;
    b.rp = rec + idx * MR;
    b.jump = R ? (count - 1) * R : 0;
    b.jumpr = b.jump * MR;
    b.rr = 0;
    b.R = R;
    b.MR = MR;
    b.max_out = max_out;
    return b;
}

// Handles one node's inbox of the round (or, in round 0, the proposer's
// broadcast()).  `st` is the instance's state block (stride sd = nodes),
// `in` the instance's inbox at sender 0.
template <bool ONE, int LV, class Inbox>
__device__ __forceinline__ void sm_node(const hbrbc_sm_args &a, int n, int f, int k, size_t g, size_t inst,
                        int local, uint8_t *st, const uint8_t *pok, const uint8_t *dok,
                        Inbox in) {
    const int me = (int)a.node_lo + local;
    const int W = (n + 31) / 32, C = (int)a.roots;
    const size_t sd = a.nodes;
    const SmLayout L(n, C, W, sd);
    Sm<ONE> m{a};
    m.n = n;
    m.f = f;
    m.k = k;
    m.W = W;
    m.C = C;
    m.rec = 1 + W;
    m.inst = inst;
    m.me = me;
    m.proposer = a.proposer[inst];
    m.role = a.role[inst * n + me];
    m.sd = sd;
    m.er16 = reinterpret_cast<uint16_t *>(st + L.er) + local;
    m.em = reinterpret_cast<uint4 *>(st + L.er) + local;
    m.cand = reinterpret_cast<uint32_t *>(st + L.cand) + local;
    m.full = reinterpret_cast<uint32_t *>(st + L.full) + local;
    m.cnt = reinterpret_cast<uint16_t *>(st + L.cnt) + local;
    m.flags = reinterpret_cast<uint32_t *>(st + L.flags) + local;
    m.pok = pok;
    m.dok = dok;
    m.out = a.out + g * (size_t)a.max_out * (1 + W);
    m.nout = 0;
    m.overflow = false;
    m.faults = a.faults + g * (size_t)a.max_faults;
    m.nfault = a.fault_count[g];
    m.cache_in();
    if (LV == 0 && a.round == 0) {
        // the proposer's broadcast() (broadcast.rs:123-137, 170-225): its input
        // step goes out unfiltered (VirtualNet::send_input; only deliveries to
        // faulty nodes pass the adversary)
        m.drop = false;
        if (me == m.proposer && !(m.FLAGS() & FL_VALUE_SENT)) {
            m.FLAGS() |= FL_VALUE_SENT;
            uint32_t *r = m.emit_rec(K_VALUE, kNone, 0, 0);
            if (r) {
                // every node but me with a Value: 32 independent byte loads
                // per word (index clamped into the row), one wait, instead of
                // a load and a branch per node
                const uint8_t *vr = a.value_root + inst * n;
                for (int w = 0; w < W; ++w) {
                    uint32_t mk = 0;
#pragma unroll
                    for (int b = 0; b < 32; ++b) {
                        const int i = 32 * w + b;
                        const uint32_t v = vr[i < n ? i : n - 1];
                        mk |= (uint32_t)(i < n && i != me && v != kNone) << b;
                    }
                    r[1 + w] = mk;
                }
            }
            const uint32_t c = a.value_root[inst * n + me];
            if (c != kNone) m.handle_value(me, c, (uint32_t)me, a.value_tamper[inst * n + me]);
        }
    } else {
        m.drop = m.role == R_SILENT;
        const bool is_faker = a.fake_from[inst] == (uint8_t)me;
        const bool faker = LV == 0 && is_faker;
        // (a smaller handler set has no injection: a fake_from node means the
        // caller's HBRBC_SM_NO_FAKE was wrong, reported like a stray record)
        if (LV > 0 && is_faker) m.bad = true;
        // this node's bit in a record's recipient mask (the record pointer
        // keeps its address space: see HB_SM_CONSTAS)
        const int mw = me >> 5;
        // (a scalar load of both mask words of the wave's nodes, each lane
        // picking its own, measured slower at N=128: 0.78 vs 0.765 ms)
        auto rbit = [&](auto r) -> bool { return (r[1 + mw] >> (me & 31)) & 1u; };
        // (no lane test for s == me: no record targets its own sender, so
        // that lane's bit is clear -- a divergent `continue` cost exec-mask
        // work on every sender)
        // wave-uniform records: the global-records kernel's (scalar loads),
        // and an LDS-staged inbox whose waves each hold one instance (values
        // read per lane, equal in every lane, moved to scalar registers: the
        // kind tests and the record loop become scalar branches)
        constexpr bool UNI = Inbox::kWaveInst ||
                             !std::is_same<decltype(in.recs()), const uint32_t *>::value;
        auto uni = [](uint32_t v) {
            return UNI ? (uint32_t)__builtin_amdgcn_readfirstlane((int)v) : v;
        };
        const uint32_t rw = 1 + W;
        for (int s = 0; s < n; ++s) {
            if (HB_SM_CACHE) m.em_focus(s >> 5);
            const uint32_t cnt = uni(in.count());
            auto r = in.recs();
            in.advance();
            for (uint32_t e = 0; e < cnt; ++e, r += rw) {
                uint32_t h0 = uni(r[0]);
                const uint32_t k0 = h0 & kKindMask;
                bool hit = rbit(r);
                // An Echo flagged by its sender (kPairFlag) is followed by the
                // EchoHash of the same step, whose targets are disjoint from
                // its own (handle_value: Echo to all but the right nodes,
                // EchoHash to the right ones): a node handles at most one of
                // them, so both are taken in one step through the merged
                // handler (a sequential step is always exact).  The flag is in
                // the header, so the step is wave-uniform wherever the records
                // are (round 5: it replaced per-record kind tests and a
                // wave-wide vote on the two recipient bits).
                if (HB_SM_MERGE && (h0 & kPairFlag) && e + 1 < cnt) {
                    const uint32_t h1 = uni(r[rw]);
                    const bool hit2 = rbit(r + rw);
                    ++e;
                    r += rw;
                    if (hit2) {
                        h0 = h1;
                        hit = true;
                    }
                }
                if (!hit) continue;
                m.template deliver<LV>(s, h0, k0);
                if (faker && !(m.FLAGS() & FL_FAKE_DONE)) {
                    // after the first delivered message (tests/broadcast.rs:73-97)
                    m.FLAGS() |= FL_FAKE_DONE;
                    uint32_t *fr = m.emit_rec(K_FAKE, a.fake_root[inst], 0, 0);
                    if (fr) m.targets_w(fr, [&](int w) { return m.all_but_me(w); });
                }
            }
        }
    }
    m.em_flush();
    m.cache_out();
    a.out_count[g] = m.nout | (m.overflow ? 0x80000000u : 0u);
    a.fault_count[g] = m.nfault;
    if (m.nout) atomicAdd(a.emitted, m.nout);
    if (m.overflow) atomicOr(a.emitted + 1, 1u);
    if (LV > 0 && m.bad) atomicOr(a.emitted + 1, 2u);
}

__device__ __forceinline__ size_t sm_in_block(const hbrbc_sm_args &a, size_t inst, int s) {
    const uint32_t R = a.rows_per_rank;
    return ((size_t)(s / R) * a.count + inst) * R + (s % R);
}

// Round kernel, global form: one thread per (instance, hosted node), state,
// records and outcomes read where they lie.  For blocks whose staged copy
// does not fit the LDS budget (sm_plan).
template <bool ONE, int LV>
__global__ __launch_bounds__(256) void sm_round_kernel(hbrbc_sm_args a, int n, int f, int k) {
    if (a.active && *a.active == 0u) return;   // quiescent: nothing was sent last round
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= a.count * a.nodes) return;
    const size_t inst = g / a.nodes;
    const int local = (int)(g - inst * a.nodes);
    if ((int)a.node_lo + local >= n) return;
    const size_t MR = (size_t)a.max_out * ((n + 31) / 32 + 1);
    uint8_t *st = a.state + inst * a.nodes * sm_state_bytes(n, a.roots);
    sm_node<ONE, LV>(a, n, f, k, g, inst, local, st, a.proof_ok + inst * a.roots * 2 * n,
            a.decode_ok + inst * a.roots,
            sm_inbox<const uint32_t *>(a.in_count, a.in, inst, a.count, a.rows_per_rank,
                                       (uint32_t)MR, a.max_out));
}

// Round kernel, staged form: a workgroup owns `ipb` whole instances (ipb x
// nodes threads) and first copies into LDS, cooperatively and coalesced,
// their state blocks (contiguous in global memory), every sender's records
// and counts of the round, and their proof / decode outcomes; the handlers'
// dependent read-modify-write chains (handle_echo: entry, Echo count, full
// count, flags, outcome, ...) then cost LDS latency instead of an L2 round
// trip each.  The state goes back at the end.
// GREC (records in global memory): the state, outcomes and proofs are staged
// as above, the records and counts are NOT -- a wave holds the nodes of one
// instance (nodes a multiple of 64), so every record read is wave-uniform and
// goes through the scalar unit (s_load, the scalar cache) straight from the
// all-gathered inbox.  The LDS image shrinks to the state (N=128: 23 -> 13
// KB per instance), so the grid's blocks fit the chip in one round instead of
// 1.3 (a second, mostly idle round of blocks), and the per-thread staging
// loop over the records (a chain of dependent global loads) goes away.
template <bool ONE, bool GREC, int LV, bool WI = false>
__device__ __forceinline__ void sm_round_staged(const hbrbc_sm_args &a, int n, int f, int k,
                                                int ipb) {
    extern __shared__ uint4 sm_lds4[];
    if (a.active && *a.active == 0u) return;   // quiescent (uniform: the whole block leaves)
    uint8_t *lds = reinterpret_cast<uint8_t *>(sm_lds4);
    const int T = (int)blockDim.x, tid = (int)threadIdx.x;
    const size_t inst0 = (size_t)blockIdx.x * ipb;
    const int ni = (int)((a.count - inst0) < (size_t)ipb ? (a.count - inst0) : (size_t)ipb);
    const int W = (n + 31) / 32, C = (int)a.roots;
    const size_t sb = sm_state_bytes(n, a.roots), nodes = a.nodes;
    const size_t MR = (size_t)a.max_out * (1 + W);   // words per sender
    // LDS: state [ipb][nodes * sb] | counts u32 [ipb][n] | records u32
    // [ipb][n][MR] | proof_ok [ipb][C * 2 * n] | decode_ok [ipb][C]
    const size_t o_cnt = (size_t)ipb * nodes * sb;   // sb % 8 == 0
    const size_t o_rec = o_cnt + (GREC ? 0 : 4 * (size_t)ipb * n);
    const size_t o_pok = o_rec + (GREC ? 0 : 4 * (size_t)ipb * n * MR);
    const size_t o_dok = o_pok + (size_t)ipb * C * 2 * n;
    uint8_t *gst = a.state + inst0 * nodes * sb;
    const size_t st_words = (size_t)ni * nodes * sb / 8;
    for (size_t i = tid; i < st_words; i += T)
        reinterpret_cast<uint2 *>(lds)[i] = reinterpret_cast<const uint2 *>(gst)[i];
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(lds + o_cnt);
    uint32_t *lrec = reinterpret_cast<uint32_t *>(lds + o_rec);
    if (!GREC && a.round > 0) {
        for (int i = tid; i < ni * n; i += T) {
            const int li = i / n, s = i - li * n;
            const uint32_t c = a.in_count[sm_in_block(a, inst0 + li, s)] & 0x7FFFFFFFu;
            lcnt[i] = c < a.max_out ? c : a.max_out;
        }
        // 32-bit index arithmetic (a 64-bit division is a long software loop)
        const uint32_t mr = (uint32_t)MR, rw = (uint32_t)(ni * n) * mr;
        for (uint32_t i = tid; i < rw; i += T) {
            const uint32_t ls = i / mr, w = i - ls * mr;
            const uint32_t li = ls / (uint32_t)n, s = ls - li * (uint32_t)n;
            lrec[i] = a.in[sm_in_block(a, inst0 + li, (int)s) * MR + w];
        }
    }
    const uint32_t pw = (uint32_t)(ni * C * 2 * n);
    for (uint32_t i = tid; i < pw; i += T) lds[o_pok + i] = a.proof_ok[inst0 * C * 2 * n + i];
    for (int i = tid; i < ni * C; i += T) lds[o_dok + i] = a.decode_ok[inst0 * C + i];
    __syncthreads();
    const int li = tid / (int)nodes, local = tid - li * (int)nodes;
    if (li < ni && (int)a.node_lo + local < n) {
        const size_t inst = inst0 + li;
        if constexpr (GREC) {
            // one instance per wave: its inbox addresses are wave-uniform
            const size_t ui = (size_t)__builtin_amdgcn_readfirstlane((int)li) + inst0;
            // the constant address space: wave-uniform reads become s_load
            // (the inbox is read-only during a round)
#if HB_SM_CONSTAS
            typedef __attribute__((address_space(4))) const uint32_t cu32;
#else
            typedef const uint32_t cu32;
#endif
            cu32 *gin = (cu32 *)a.in;
            cu32 *gcnt = (cu32 *)a.in_count;
            sm_node<ONE, LV>(a, n, f, k, inst * nodes + local, inst, local,
                    lds + (size_t)li * nodes * sb, lds + o_pok + (size_t)li * C * 2 * n,
                    lds + o_dok + (size_t)li * C,
                    sm_inbox<cu32 *>(gcnt, gin, ui, a.count, a.rows_per_rank, (uint32_t)MR,
                                     a.max_out));
        } else {
            const uint32_t *cb = lcnt + (size_t)li * n;
            const uint32_t *rb = lrec + (size_t)li * n * MR;
            sm_node<ONE, LV>(a, n, f, k, inst * nodes + local, inst, local, lds + (size_t)li * nodes * sb,
                    lds + o_pok + (size_t)li * C * 2 * n, lds + o_dok + (size_t)li * C,
                    sm_inbox<const uint32_t *, WI>(cb, rb, 0, 1, 0, (uint32_t)MR, a.max_out));
        }
    }
    __syncthreads();
    for (size_t i = tid; i < st_words; i += T)
        reinterpret_cast<uint2 *>(gst)[i] = reinterpret_cast<const uint2 *>(lds)[i];
}

// WI: nodes % 64 == 0, every wave one instance (SmInbox)
template <bool ONE, int LV, bool WI>
__global__ __launch_bounds__(256) void sm_round_staged_kernel(hbrbc_sm_args a, int n, int f,
                                                              int k, int ipb) {
    sm_round_staged<ONE, false, LV, WI>(a, n, f, k, ipb);
}
// The same at 4 waves/SIMD (128 VGPRs, a few spills instead of 162 VGPRs):
// for launches whose LDS image leaves room for more than 3 waves per SIMD
// (N=64 validator-sharded object: state machine 0.82 -> 0.63 ms per step;
// at N=128 the LDS holds 2 waves per SIMD and the spills cost 1.25 -> 1.28)
#ifndef HB_SM_W4_WAVES
#define HB_SM_W4_WAVES 4   // waves/SIMD of the "w4" forms (A/B: -DHB_SM_W4_WAVES=5)
#endif
template <bool ONE, int LV, bool WI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HB_SM_W4_WAVES, HB_SM_W4_WAVES))) void
sm_round_staged_w4_kernel(hbrbc_sm_args a, int n, int f, int k, int ipb) {
    sm_round_staged<ONE, false, LV, WI>(a, n, f, k, ipb);
}
template <bool ONE, int LV>
__global__ __launch_bounds__(256) void sm_round_grec_kernel(hbrbc_sm_args a, int n, int f, int k,
                                                            int ipb) {
    sm_round_staged<ONE, true, LV>(a, n, f, k, ipb);
}
template <bool ONE, int LV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HB_SM_W4_WAVES, HB_SM_W4_WAVES))) void
sm_round_grec_w4_kernel(hbrbc_sm_args a, int n, int f, int k, int ipb) {
    sm_round_staged<ONE, true, LV>(a, n, f, k, ipb);
}

}  // namespace

// Launch plan: the staged form with ipb instances per workgroup (ipb x nodes
// <= 256 threads, at most 128 unless one instance needs more) when its LDS
// image fits 64 KiB; else the global form.
static size_t sm_lds_bytes(const hbrbc_sm_args &a, int n, int ipb, bool grec = false) {
    const size_t W = (n + 31) / 32, MR = (size_t)a.max_out * (1 + W);
    const size_t per = a.nodes * sm_state_bytes(n, a.roots) +
                       (grec ? 0 : 4 * (size_t)n + 4 * (size_t)n * MR) +
                       (size_t)a.roots * 2 * n + a.roots;
    return ((size_t)ipb * per + 15) & ~(size_t)15;
}

// One instantiation set per handler set (LV: see Sm::deliver).
template <int LV>
static hipError_t launch_sm_form(const hbrbc_sm_args &a, int n, int f, int k, hipStream_t s) {
    const size_t threads = a.count * a.nodes;
    const char *e = getenv("HBRBC_SM_STAGED");   // 0: the global form (A/B)
    const bool staged_ok = !(e && !strcmp(e, "0")) && a.nodes <= 256;
    int ipb = a.nodes >= 128 ? 1 : (int)(128 / a.nodes);
    // records through the scalar unit when every wave holds one instance's
    // nodes (HBRBC_SM_GREC=0/1 forces, A/B)
    const char *ge = getenv("HBRBC_SM_GREC");
    // (N=64, 4096 instances: 0.64 ms LDS-staged vs 0.78 global; N=128, 2048
    // instances: 1.37 vs 1.13-1.26 -- the LDS image only limits residency
    // at N >= 128, tools/sm_bench.py, profiles/r4_sm_ab.txt)
    const bool grec = (ge ? !strcmp(ge, "1") : a.nodes >= 128) && a.nodes % 64 == 0 &&
                      a.nodes >= 64;
    while (ipb > 1 && sm_lds_bytes(a, n, ipb, grec) > 65536) --ipb;
    if (staged_ok && sm_lds_bytes(a, n, ipb, grec) <= 65536) {
        const unsigned blocks = (unsigned)((a.count + ipb - 1) / ipb);
        const size_t lds = sm_lds_bytes(a, n, ipb, grec), threads_pb = (size_t)ipb * a.nodes;
        // waves per CU the LDS image allows (160 KiB per CU) above 3 per SIMD:
        // the 4-wave form (HBRBC_SM_W4=0/1 forces, A/B)
        const char *w4e = getenv("HBRBC_SM_W4");
        const bool w4 = w4e ? !strcmp(w4e, "1")
                            : (163840 / lds) * ((threads_pb + 63) / 64) > 12;
        // every wave one instance: scalar record dispatch (HBRBC_SM_WI=0: off, A/B)
        const char *wie = getenv("HBRBC_SM_WI");
        const bool wi = a.nodes % 64 == 0 && !(wie && !strcmp(wie, "0"));
        auto kern = grec ? (a.roots == 1 ? (w4 ? sm_round_grec_w4_kernel<true, LV>
                                               : sm_round_grec_kernel<true, LV>)
                                         : (w4 ? sm_round_grec_w4_kernel<false, LV>
                                               : sm_round_grec_kernel<false, LV>))
                         : wi ? (a.roots == 1 ? (w4 ? sm_round_staged_w4_kernel<true, LV, true>
                                                    : sm_round_staged_kernel<true, LV, true>)
                                              : (w4 ? sm_round_staged_w4_kernel<false, LV, true>
                                                    : sm_round_staged_kernel<false, LV, true>))
                         : (a.roots == 1 ? (w4 ? sm_round_staged_w4_kernel<true, LV, false>
                                               : sm_round_staged_kernel<true, LV, false>)
                                         : (w4 ? sm_round_staged_w4_kernel<false, LV, false>
                                               : sm_round_staged_kernel<false, LV, false>));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3((unsigned)threads_pb), lds, s, a, n, f, k, ipb);
        return hipGetLastError();
    }
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    if (a.roots == 1)
        hipLaunchKernelGGL((sm_round_kernel<true, LV>), dim3(blocks), dim3(256), 0, s, a, n, f, k);
    else
        hipLaunchKernelGGL((sm_round_kernel<false, LV>), dim3(blocks), dim3(256), 0, s, a, n, f, k);
    return hipGetLastError();
}

hipError_t launch_sm_round(const hbrbc_sm_args &a, int n, int f, int k, hipStream_t s) {
    if (a.count * a.nodes == 0) return hipSuccess;
    // the smaller handler sets for rounds >= 1 of a batch the caller marks as
    // having no injected broadcasts (HBRBC_SM_LEAN=0: never, A/B)
    const char *le = getenv("HBRBC_SM_LEAN");
    const int lv = (a.flags & HBRBC_SM_NO_FAKE) && !(le && !strcmp(le, "0"))
                       ? (a.round >= 2 ? 2 : (a.round == 1 ? 1 : 0)) : 0;
    return lv == 2 ? launch_sm_form<2>(a, n, f, k, s)
                   : (lv == 1 ? launch_sm_form<1>(a, n, f, k, s) : launch_sm_form<0>(a, n, f, k, s));
}

}  // namespace hbrbc
