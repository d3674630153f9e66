// test_host.cpp -- the C++ host mirror (include/hbrbc.hpp, hbrbc_broadcast.hpp)
// run the way the reference's own tests run the Rust API:
//   merkle.rs:152-166 test_merkle; broadcast/mod.rs:140-220 doc-test (7 nodes,
//   proposer 3); tests/broadcast.rs test_broadcast_different_sizes with the
//   reordering / node-order schedules and silent faulty nodes; plus the rse
//   error outcomes and the golden N=4 "Foo" root (tests/golden).
// Exit 0 = all passed, 1 = a check failed, 2 = no GPU (the path has no CPU
// fallback and says so).
#include <cstdio>
#include <deque>
#include <random>

#include "hbrbc_broadcast.hpp"

using namespace hbrbc;

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

static std::string hex(const Digest &d) {
    static const char *x = "0123456789abcdef";
    std::string s;
    for (uint8_t b : d) {
        s += x[b >> 4];
        s += x[b & 15];
    }
    return s;
}

static Bytes random_bytes(std::mt19937_64 &rng, size_t n) {
    Bytes b(n);
    for (auto &v : b) v = (uint8_t)rng();
    return b;
}

// merkle.rs:152-166
static void test_merkle() {
    for (size_t n : {4, 7, 8, 9, 17}) {
        std::vector<Bytes> vals;
        for (size_t i = 0; i < n; ++i) vals.push_back(Bytes{(uint8_t)i});
        MerkleTree t = MerkleTree::from_vec(vals);
        for (size_t i = 0; i < n; ++i) {
            auto p = t.proof(i);
            CHECK(p && p->validate(n));
        }
        CHECK(!t.proof(n));
    }
}

// golden N=4 "Foo" (tests/golden/broadcast_vectors.json)
static void test_golden_foo() {
    std::optional<Coding> c;
    CHECK(Coding::create(2, 2, c) == HBRBC_OK);
    MerkleTree t = send_shards(*c, Bytes{'F', 'o', 'o'});
    CHECK(hex(t.root_hash()) == "1383678fb0dc4d90312d6ea104d5ca958d39c6dbfdc56f76667463cedb7466f1");
    CHECK(t.values()[2] == (Bytes{0x8c, 0xde, 0xde, 0x05}));
    CHECK(t.values()[3] == (Bytes{0xca, 0xb1, 0xb1, 0x06}));
}

// Coding round trips and rse outcomes (broadcast.rs:563-601, 639-694)
static void test_coding(std::mt19937_64 &rng) {
    std::optional<Coding> bad;
    CHECK(Coding::create(87, 170, bad) == HBRBC_E_TOO_MANY_SHARDS);  // N = 257
    for (size_t n : {1, 3, 4, 16, 64, 250}) {
        const size_t f = (n - 1) / 3, k = n - 2 * f;
        std::optional<Coding> c;
        CHECK(Coding::create(k, 2 * f, c) == HBRBC_OK);
        for (size_t plen : {0, 5, 1000, 30000}) {
            const Bytes payload = random_bytes(rng, plen);
            MerkleTree t = send_shards(*c, payload);
            std::vector<std::optional<Bytes>> leaves(t.values().begin(), t.values().end());
            std::vector<size_t> order(n);
            for (size_t i = 0; i < n; ++i) order[i] = i;
            std::shuffle(order.begin(), order.end(), rng);
            for (size_t i = 0; i < 2 * f; ++i) leaves[order[i]].reset();  // keep exactly k
            auto out = decode_from_shards(*c, leaves, t.root_hash());
            CHECK(out && *out == payload);
            if (f) {  // one shard too few
                std::vector<std::optional<Bytes>> few(t.values().begin(), t.values().end());
                for (size_t i = 0; i < 2 * f + 1; ++i) few[order[i]].reset();
                CHECK(c->reconstruct_shards(few) == HBRBC_E_TOO_FEW_SHARDS_PRESENT);
                // a tampered parity shard that gets used changes the root
                std::vector<std::optional<Bytes>> bent(t.values().begin(), t.values().end());
                bent[0].reset();
                (*bent[n - 1])[0] ^= 1;
                for (size_t i = 1; i < n - 1 && i < 2 * f; ++i) bent[i].reset();
                CHECK(!decode_from_shards(*c, bent, t.root_hash()));
            }
        }
        if (n > 1) {  // ragged shards -> IncorrectShardSize
            std::vector<Bytes> sh(n, Bytes(8, 1));
            sh[1].resize(7);
            CHECK(c->encode(sh) == (f != 0 ? HBRBC_E_INCORRECT_SHARD_SIZE : HBRBC_OK));
        }
    }
}

// broadcast/mod.rs:140-220
static void test_doc_example(std::mt19937_64 &rng) {
    const size_t kNodes = 7;
    const NodeId kProposer = 3;
    std::vector<NodeId> ids;
    for (NodeId i = 0; i < kNodes; ++i) ids.push_back(i);
    auto vals = std::make_shared<const ValidatorSet>(ids);
    std::map<NodeId, Broadcast> nodes;
    for (NodeId i : ids) nodes.emplace(i, Broadcast(i, vals, kProposer));
    const Bytes payload = random_bytes(rng, 128);
    std::deque<std::pair<NodeId, TargetedMessage>> queue;
    std::set<NodeId> finished;
    auto on_step = [&](NodeId id, Step step) {
        for (auto &m : step.messages) queue.emplace_back(id, std::move(m));
        if (!step.output.empty()) {
            CHECK(step.output.size() == 1 && step.output[0] == payload);
            CHECK(finished.insert(id).second);  // at most once
        }
    };
    on_step(kProposer, nodes.at(kProposer).broadcast(payload));
    while (!queue.empty()) {
        auto [src, tm] = std::move(queue.front());
        queue.pop_front();
        for (auto &[id, node] : nodes)
            if (tm.target.contains(id)) on_step(id, node.handle_message(src, tm.message));
    }
    CHECK(finished.size() == kNodes);  // and at least once
}

// tests/broadcast.rs:101-185 over a VirtualNet-style queue (hbbft_testing
// lib.rs:223-283, 908-996): schedule 0 = reordering (swap_random), 1 = node
// order (sort_ascending); the first f nodes are faulty and, with `silent`,
// send nothing (the "drop" adversary).
static void test_different_sizes(std::mt19937_64 &rng, int schedule, bool silent) {
    std::vector<size_t> sizes = {1, 2, 3, 4, 5, 6 + rng() % 14, 30 + rng() % 20};
    for (size_t size : sizes) {
        const size_t nf = (size - 1) / 3;
        const NodeId proposer = nf + rng() % (size - nf);  // a correct proposer
        std::vector<NodeId> ids;
        for (NodeId i = 0; i < size; ++i) ids.push_back(i);
        auto vals = std::make_shared<const ValidatorSet>(ids);
        std::map<NodeId, Broadcast> nodes;
        for (NodeId i : ids) nodes.emplace(i, Broadcast(i, vals, proposer));
        struct NetMsg {
            NodeId from, to;
            Message m;
        };
        std::deque<NetMsg> q;
        std::map<NodeId, std::vector<Bytes>> outputs;
        auto process = [&](NodeId id, Step step) {
            for (auto &f : step.fault_log) CHECK(f.node_id < nf || id < nf);  // no correct blamed
            auto &o = outputs[id];
            o.insert(o.end(), step.output.begin(), step.output.end());
            if (silent && id < nf) return;
            for (auto &tm : step.messages)
                for (NodeId to : ids)
                    if (to != id && tm.target.contains(to)) q.push_back({id, to, tm.message});
        };
        const Bytes value{'F', 'o', 'o'};
        process(proposer, nodes.at(proposer).broadcast(value));
        size_t cranks = 0;
        auto done = [&] {
            for (auto &[id, node] : nodes)
                if (!(silent && id < nf) && !node.terminated()) return false;
            return true;
        };
        while (!done()) {
            CHECK(!q.empty());
            if (q.empty() || ++cranks > 10000 * size) break;
            if (schedule == 0) {
                std::swap(q[0], q[rng() % q.size()]);
            } else {  // a stable sort by recipient, then the front: the oldest message to the lowest id
                size_t best = 0;
                for (size_t i = 1; i < q.size(); ++i)
                    if (q[i].to < q[best].to) best = i;
                std::rotate(q.begin(), q.begin() + best, q.begin() + best + 1);
            }
            NetMsg m = std::move(q.front());
            q.pop_front();
            process(m.to, nodes.at(m.to).handle_message(m.from, m.m));
        }
        for (NodeId id : ids)
            if (!(silent && id < nf)) CHECK(outputs[id] == std::vector<Bytes>{value});
    }
}

static void test_errors() {
    auto vals = std::make_shared<const ValidatorSet>(std::vector<NodeId>{0, 1, 2, 3});
    Broadcast b(0, vals, 1);
    try {
        b.broadcast(Bytes{1});
        CHECK(false);
    } catch (const BroadcastError &e) {
        CHECK(e.kind == ErrorKind::InstanceCannotPropose);
    }
    try {
        b.handle_message(9, Message{Message::Ready, nullptr, {}});
        CHECK(false);
    } catch (const BroadcastError &e) {
        CHECK(e.kind == ErrorKind::UnknownSender);
    }
    std::vector<NodeId> many;
    for (NodeId i = 0; i < 257; ++i) many.push_back(i);
    try {
        Broadcast big(0, std::make_shared<const ValidatorSet>(many), 0);
        CHECK(false);
    } catch (const BroadcastError &e) {
        CHECK(e.kind == ErrorKind::InvalidNodeCount);
    }
}

int main() {
    std::mt19937_64 rng(0x48424246);
    try {
        test_merkle();
        test_golden_foo();
        test_coding(rng);
        test_errors();
        test_doc_example(rng);
        for (int schedule : {0, 1})
            for (bool silent : {false, true}) test_different_sizes(rng, schedule, silent);
    } catch (const Unavailable &e) {
        std::fprintf(stderr, "HbrbcUnavailable: %s\n", e.what());
        return 2;
    }
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("test_host: all passed\n");
    return 0;
}
