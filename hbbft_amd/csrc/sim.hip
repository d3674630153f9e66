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

namespace hbrbc {

namespace {

constexpr uint32_t kNone = 0xFFu;

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

// echo entry (EchoContent): 0 none; Hash: 0x4000 | c << 8; Full: 0x8000 |
// t << 13 | c << 8 | index
__device__ __forceinline__ uint32_t enc_full(uint32_t c, uint32_t j, uint32_t t) {
    return 0x8000u | (t << 13) | (c << 8) | j;
}
__device__ __forceinline__ uint32_t enc_hash(uint32_t c) { return 0x4000u | (c << 8); }
__device__ __forceinline__ bool is_full(uint32_t e) { return e & 0x8000u; }
__device__ __forceinline__ bool is_hash(uint32_t e) { return e & 0x4000u; }
__device__ __forceinline__ uint32_t root_of(uint32_t e) { return (e >> 8) & 31u; }

struct Sm {
    const hbrbc_sm_args &a;
    int n, f, k, W, C, rec;   // rec: uint32 words per message record (1 + W)
    size_t inst;
    int me, proposer, role;
    bool drop;                // a silent node's deliveries emit nothing
    // state of (inst, me), structure of arrays over the instance's hosted
    // nodes (stride sd = nodes): the nodes of an instance are consecutive
    // threads, so every state access of a wave is one coalesced request
    uint16_t *echo;           // [n][sd]
    uint8_t *ready;           // [n][sd]
    uint32_t *cand;           // [C][W][sd]
    uint16_t *cnt;            // [3][C][sd]: Echo+EchoHash, full Echo, Ready counts
    uint32_t *flags;          // [sd]
    size_t sd;

    __device__ uint16_t &ECHO(int s) { return echo[(size_t)s * sd]; }
    __device__ uint8_t &READY(int s) { return ready[(size_t)s * sd]; }
    __device__ uint32_t &CAND(uint32_t c, int w) { return cand[((size_t)c * W + w) * sd]; }
    __device__ uint16_t &CE(uint32_t c) { return cnt[(size_t)c * sd]; }
    __device__ uint16_t &CF(uint32_t c) { return cnt[((size_t)C + c) * sd]; }
    __device__ uint16_t &CR(uint32_t c) { return cnt[((size_t)2 * C + c) * sd]; }
    __device__ uint32_t &FLAGS() { return *flags; }
    uint32_t *out;            // [max_out][rec]
    uint32_t nout;
    bool overflow;
    uint16_t *faults;
    uint32_t nfault;

    __device__ bool bit(const uint32_t *m, int i) const { return (m[i >> 5] >> (i & 31)) & 1u; }

    __device__ void fault(int node, int kind) {
        if (nfault < a.max_faults) faults[nfault] = (uint16_t)((node << 8) | kind);
        ++nfault;
    }

    // right_nodes (broadcast.rs:476-485): the f nodes before us on the circle
    __device__ bool is_right_of(int j, int i) const {
        const int d = (i - j + n) % n;   // j = i - d
        return d >= 1 && d <= f;
    }

    __device__ uint32_t *emit_rec(uint32_t kind, uint32_t c, uint32_t j, uint32_t t) {
        if (nout >= a.max_out) {
            overflow = true;
            return nullptr;
        }
        uint32_t *r = out + (size_t)nout * rec;
        ++nout;
        r[0] = kind | (c << 8) | (j << 16) | (t << 24);
        for (int w = 0; w < W; ++w) r[1 + w] = 0;
        return r;
    }

    // emission as the node's own step (subject to its role)
    __device__ uint32_t *emit(uint32_t kind, uint32_t c, uint32_t j = 0, uint32_t t = 0) {
        if (drop) return nullptr;
        if (kind == K_ECHO && role == R_WITHHOLD_ECHO) return nullptr;
        if (kind == K_ECHO && role == R_CORRUPT_ECHO) t = 1;
        return emit_rec(kind, c, j, t);
    }

    __device__ bool validate_proof(uint32_t c, uint32_t j, uint32_t t, int sender) const {
        if ((int)j != sender || c >= (uint32_t)C || j >= (uint32_t)n) return false;
        return a.proof_ok[((inst * C + c) * 2 + (t & 1)) * n + j] != 0;
    }

    // -- handlers (broadcast.rs) --------------------------------------------
    __device__ void compute_output(uint32_t c) {   // 526-558
        if ((FLAGS() & FL_DECIDED) || CR(c) <= 2 * f || CF(c) < k) return;
        if (a.decode_ok[inst * C + c]) {
            FLAGS() |= FL_DECIDED;
            a.output_root[inst * a.nodes + (me - a.node_lo)] = (uint8_t)c;
        } else {
            fault(proposer, F_BROADCAST_DECODING);
        }
    }

    __device__ void send_echo_remaining(uint32_t c) {   // 428-453
        FLAGS() |= FL_ECHO_SENT;
        const uint32_t e = ECHO(me);
        if (!is_full(e) || root_of(e) != c) return;
        uint32_t *r = emit(K_ECHO, c, e & 0xFFu, (e >> 13) & 1u);
        if (!r) return;
        for (int i = 0; i < n; ++i)
            if (is_right_of(i, me) && !((CAND(c, i >> 5) >> (i & 31)) & 1u))
                r[1 + (i >> 5)] |= 1u << (i & 31);
    }

    __device__ void handle_ready_core(int s, uint32_t c, bool may_send);

    __device__ void send_ready(uint32_t c) {   // 513-522
        FLAGS() |= FL_READY_SENT;
        uint32_t *r = emit(K_READY, c);
        if (r)
            for (int i = 0; i < n; ++i)
                if (i != me) r[1 + (i >> 5)] |= 1u << (i & 31);
        handle_ready_core(me, c, false);
    }

    __device__ void handle_can_decode(int s, uint32_t c) {   // 358-375
        CAND(c, s >> 5) |= 1u << (s & 31);
    }

    __device__ void send_can_decode(uint32_t c) {   // 488-510
        FLAGS() |= 1u << (FL_CAN_DECODE_SHIFT + c);
        uint32_t *r = emit(K_CAN_DECODE, c);
        if (r)
            for (int i = 0; i < n; ++i)
                if (i != me && !is_full(ECHO(i))) r[1 + (i >> 5)] |= 1u << (i & 31);
        handle_can_decode(me, c);
    }

    __device__ void handle_echo(int s, uint32_t c, uint32_t j, uint32_t t) {   // 266-320
        const uint32_t e = ECHO(s);
        if (is_full(e)) {
            if (e != enc_full(c, j, t)) fault(s, F_MULTIPLE_ECHOS);
            return;
        }
        if (is_hash(e) && root_of(e) != c) {
            fault(s, F_MULTIPLE_ECHOS);
            return;
        }
        if (!validate_proof(c, j, t, s)) {
            fault(s, F_INVALID_PROOF);
            return;
        }
        if (!e) ++CE(c);   // a Hash of the same root was counted already
        ++CF(c);
        ECHO(s) = (uint16_t)enc_full(c, j, t);
        if (!(FLAGS() & (1u << (FL_CAN_DECODE_SHIFT + c))) && CF(c) >= k) send_can_decode(c);
        if (!(FLAGS() & FL_READY_SENT) && CE(c) >= n - f) send_ready(c);
        if (FLAGS() & FL_READY_SENT) compute_output(c);
    }

    __device__ void handle_echo_hash(int s, uint32_t c) {   // 322-355
        const uint32_t e = ECHO(s);
        if (e) {
            if (root_of(e) != c) fault(s, F_MULTIPLE_ECHO_HASHES);
            return;
        }
        ECHO(s) = (uint16_t)enc_hash(c);
        ++CE(c);
        if ((FLAGS() & FL_READY_SENT) || CE(c) < n - f) {
            compute_output(c);
            return;
        }
        send_ready(c);
    }

    __device__ void send_echo_hash(uint32_t c) {   // 456-468
        FLAGS() |= FL_ECHO_HASH_SENT;
        uint32_t *r = emit(K_ECHO_HASH, c);
        if (r)
            for (int i = 0; i < n; ++i)
                if (is_right_of(i, me)) r[1 + (i >> 5)] |= 1u << (i & 31);
        handle_echo_hash(me, c);
    }

    __device__ void send_echo_left(uint32_t c, uint32_t j, uint32_t t) {   // 413-425
        uint32_t *r = emit(K_ECHO, c, j, t);
        if (r)
            for (int i = 0; i < n; ++i)
                if (i != me && !is_right_of(i, me)) r[1 + (i >> 5)] |= 1u << (i & 31);
        handle_echo(me, c, j, t);
    }

    // rotate out[a0, a1) behind out[a1, nout) (and the same for faults):
    // echo_steps.join(echo_hash_steps) lists the Echo step first although the
    // EchoHash step ran first (broadcast.rs:258-262)
    __device__ void rotate_tail(uint32_t m0, uint32_t m1, uint32_t f0, uint32_t f1) {
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

    __device__ void handle_value(int s, uint32_t c, uint32_t j, uint32_t t) {   // 228-263
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
            if (is_full(e) && e == enc_full(c, j, t)) return;
        }
        if (!validate_proof(c, j, t, me)) {
            fault(s, F_INVALID_PROOF);
            return;
        }
        const uint32_t m0 = nout, f0 = nfault;
        send_echo_hash(c);
        const uint32_t m1 = nout, f1 = nfault;
        send_echo_left(c, j, t);
        if (!overflow) rotate_tail(m0, m1, f0, f1);
    }

    // the ProposeAdversary's injected step: per listed faulty node F (in index
    // order) its fresh Broadcast's messages -- Value(proof j) to every j != F,
    // Echo(proof F) to AllExcept(right(F)), EchoHash to right(F) -- all sent
    // by the dispatching node; a receiver handles the ones addressed to it
    __device__ void handle_fake(int s, uint32_t c) {
        const uint32_t *list = a.fake_list + inst * W;
        for (int F = 0; F < n; ++F) {
            if (!bit(list, F)) continue;
            if (me != F) handle_value(s, c, (uint32_t)me, 0);
            if (!is_right_of(me, F)) handle_echo(s, c, (uint32_t)F, 0);
            else handle_echo_hash(s, c);
        }
    }

    __device__ void deliver(int s, const uint32_t *r) {
        const uint32_t kind = r[0] & 0xFFu, c0 = (r[0] >> 8) & 0xFFu;
        const uint32_t j = (r[0] >> 16) & 0xFFu, t = (r[0] >> 24) & 0xFFu;
        switch (kind) {
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
            case K_ECHO: handle_echo(s, c0, j, t); break;
            case K_READY: handle_ready_core(s, c0, true); break;
            case K_CAN_DECODE: handle_can_decode(s, c0); break;
            case K_ECHO_HASH: handle_echo_hash(s, c0); break;
            case K_FAKE: handle_fake(s, c0); break;
            default: break;
        }
    }
};

__device__ void Sm::handle_ready_core(int s, uint32_t c, bool may_send) {   // 378-410
    const uint32_t old = READY(s);
    if (old) {
        if (old - 1 != c) fault(s, F_MULTIPLE_READYS);
        return;
    }
    READY(s) = (uint8_t)(c + 1);
    ++CR(c);
    // (from send_ready, ready_sent is already set: no further send_ready)
    if (may_send && CR(c) == f + 1 && !(FLAGS() & FL_READY_SENT)) send_ready(c);
    if (CR(c) == 2 * f + 1) send_echo_remaining(c);
    compute_output(c);
}

__global__ __launch_bounds__(256) void sm_round_kernel(hbrbc_sm_args a, int n, int f, int k) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= a.count * a.nodes) return;
    const size_t inst = g / a.nodes;
    const int local = (int)(g - inst * a.nodes);
    const int me = (int)a.node_lo + local;
    if (me >= n) return;
    const int W = (n + 31) / 32, C = (int)a.roots;
    // this instance's state block (nodes x sm_state_bytes), structure of arrays
    const size_t sd = a.nodes;
    uint8_t *st = a.state + inst * sd * sm_state_bytes(n, a.roots);
    Sm m{a};
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
    m.echo = reinterpret_cast<uint16_t *>(st) + local;
    m.ready = st + 2 * (size_t)n * sd + local;
    const size_t o_cand = (3 * (size_t)n * sd + 3) & ~(size_t)3;
    m.cand = reinterpret_cast<uint32_t *>(st + o_cand) + local;
    const size_t o_cnt = o_cand + 4 * (size_t)C * W * sd;
    m.cnt = reinterpret_cast<uint16_t *>(st + o_cnt) + local;
    const size_t o_flags = (o_cnt + 6 * (size_t)C * sd + 3) & ~(size_t)3;
    m.flags = reinterpret_cast<uint32_t *>(st + o_flags) + local;
    m.out = a.out + g * (size_t)a.max_out * (1 + W);
    m.nout = 0;
    m.overflow = false;
    m.faults = a.faults + g * (size_t)a.max_faults;
    m.nfault = a.fault_count[g];
    if (a.round == 0) {
        // the proposer's broadcast() (broadcast.rs:123-137, 170-225): its input
        // step goes out unfiltered (VirtualNet::send_input; only deliveries to
        // faulty nodes pass the adversary)
        m.drop = false;
        if (me == m.proposer && !(*m.flags & FL_VALUE_SENT)) {
            *m.flags |= FL_VALUE_SENT;
            uint32_t *r = m.emit_rec(K_VALUE, kNone, 0, 0);
            if (r)
                for (int i = 0; i < n; ++i)
                    if (i != me && a.value_root[inst * n + i] != kNone) r[1 + (i >> 5)] |= 1u << (i & 31);
            const uint32_t c = a.value_root[inst * n + me];
            if (c != kNone) m.handle_value(me, c, (uint32_t)me, a.value_tamper[inst * n + me]);
        }
    } else {
        m.drop = m.role == R_SILENT;
        const uint32_t R = a.rows_per_rank;
        const bool faker = a.fake_from[inst] == (uint8_t)me;
        for (int s = 0; s < n; ++s) {
            if (s == me) continue;   // targets never include the sender
            const size_t blk = ((size_t)(s / R) * a.count + inst) * R + (s % R);
            const uint32_t cnt = a.in_count[blk] & 0x7FFFFFFFu;
            const uint32_t *recs = a.in + blk * (size_t)a.max_out * (1 + W);
            for (uint32_t e = 0; e < cnt && e < a.max_out; ++e) {
                const uint32_t *r = recs + (size_t)e * (1 + W);
                if (!m.bit(r + 1, me)) continue;
                m.deliver(s, r);
                if (faker && !(*m.flags & FL_FAKE_DONE)) {
                    // after the first delivered message (tests/broadcast.rs:73-97)
                    *m.flags |= FL_FAKE_DONE;
                    uint32_t *fr = m.emit_rec(K_FAKE, a.fake_root[inst], 0, 0);
                    if (fr)
                        for (int i = 0; i < n; ++i)
                            if (i != me) fr[1 + (i >> 5)] |= 1u << (i & 31);
                }
            }
        }
    }
    a.out_count[g] = m.nout | (m.overflow ? 0x80000000u : 0u);
    a.fault_count[g] = m.nfault;
    if (m.nout) atomicAdd(a.emitted, m.nout);
}

}  // namespace

hipError_t launch_sm_round(const hbrbc_sm_args &a, int n, int f, int k, hipStream_t s) {
    const size_t threads = a.count * a.nodes;
    if (threads == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    hipLaunchKernelGGL(sm_round_kernel, dim3(blocks), dim3(256), 0, s, a, n, f, k);
    return hipGetLastError();
}

}  // namespace hbrbc
