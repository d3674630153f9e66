/*
 * hbrbc.hpp -- C++17 host mirror of the reference's data-path surface over
 * the C ABI (hbrbc.h), for hosts that are compiled code like the reference.
 *
 * The reference (Rust) has `Coding` (src/broadcast/broadcast.rs:639-694),
 * `MerkleTree` / `Proof` (src/broadcast/merkle.rs:12-103) and the framing of
 * `send_shards` / `decode_from_shards` (broadcast.rs:170-225, 563-601).  The
 * same names, argument meaning and outcomes here:
 *   - rse errors come back as an `int` status (HBRBC_E_*: TooManyShards,
 *     TooFewShardsPresent, IncorrectShardSize, ...), like `RseResult`;
 *   - `MerkleTree::proof` returns an empty optional for an index >= n (`None`);
 *   - `Proof::validate(n)` returns a bool;
 *   - a missing GPU or a failing HIP call throws `hbrbc::Unavailable` /
 *     `hbrbc::DeviceError`: there is no CPU fallback.
 * Every computation runs in libhbrbc.so on the MI355X.
 */
#ifndef HBRBC_HPP
#define HBRBC_HPP

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "hbrbc.h"

namespace hbrbc {

using Bytes = std::vector<uint8_t>;
using Digest = std::array<uint8_t, 32>;  // merkle.rs:6

struct Unavailable : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct DeviceError : std::runtime_error {
    int code;
    DeviceError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// Library / device failures throw; rse outcomes (codes < 100) are returned.
inline int check(int st) {
    if (st == HBRBC_E_NO_DEVICE) throw Unavailable(std::string("no HIP device: ") + hbrbc_last_error());
    if (st >= HBRBC_E_INVALID_ARG) throw DeviceError(st, hbrbc_last_error());
    return st;
}

// `Coding` (broadcast.rs:639-694): ReedSolomon(data, parity), or Trivial when parity == 0.
class Coding {
  public:
    // `Coding::new(data_shard_num, parity_shard_num) -> RseResult<Self>` (646-655).
    static int create(size_t data_shards, size_t parity_shards, std::optional<Coding> &out,
                      int device = -1) {
        hbrbc_ctx *h = nullptr;
        const int st = check(hbrbc_coding_new(data_shards, parity_shards, device, &h));
        if (st == HBRBC_OK) out = Coding(h);
        return st;
    }
    size_t data_shard_count() const { return hbrbc_data_shard_count(ctx_.get()); }
    size_t parity_shard_count() const { return hbrbc_parity_shard_count(ctx_.get()); }

    // `encode(&mut [&mut [u8]]) -> RseResult<()>` (674-679): parity overwritten in place.
    int encode(std::vector<Bytes> &shards) const {
        std::vector<uint8_t *> p(shards.size());
        std::vector<size_t> l(shards.size());
        for (size_t i = 0; i < shards.size(); ++i) {
            p[i] = shards[i].data();
            l[i] = shards[i].size();
        }
        return check(hbrbc_encode(ctx_.get(), p.data(), l.data(), shards.size()));
    }

    // `reconstruct_shards(&mut [Option<Box<[u8]>>]) -> RseResult<()>` (682-693):
    // absent entries are filled with the rebuilt shard on success.
    int reconstruct_shards(std::vector<std::optional<Bytes>> &shards) const {
        size_t len = 0;
        for (const auto &s : shards)
            if (s && s->size() > len) len = s->size();
        std::vector<Bytes> fill(shards.size());
        std::vector<uint8_t *> p(shards.size());
        std::vector<size_t> l(shards.size());
        std::vector<uint8_t> present(shards.size());
        for (size_t i = 0; i < shards.size(); ++i) {
            present[i] = shards[i].has_value();
            if (present[i]) {
                p[i] = shards[i]->data();
                l[i] = shards[i]->size();
            } else {
                fill[i].assign(len ? len : 1, 0);
                p[i] = fill[i].data();
                l[i] = 0;
            }
        }
        const int st = check(hbrbc_reconstruct(ctx_.get(), p.data(), l.data(), present.data(),
                                               shards.size()));
        if (st == HBRBC_OK)
            for (size_t i = 0; i < shards.size(); ++i)
                if (!present[i]) shards[i] = Bytes(fill[i].begin(), fill[i].begin() + len);
        return st;
    }

  private:
    explicit Coding(hbrbc_ctx *h) : ctx_(h, hbrbc_coding_free) {}
    std::shared_ptr<hbrbc_ctx> ctx_;
};

// `Proof<T>` (merkle.rs:72-78): field order value, index, digests, root_hash.
struct Proof {
    Bytes value;
    size_t index = 0;
    std::vector<Digest> digests;
    Digest root_hash{};

    // `Proof::validate(n)` (merkle.rs:83-103), on the GPU.
    bool validate(size_t n) const {
        std::vector<uint8_t> d(32 * digests.size());
        for (size_t i = 0; i < digests.size(); ++i) std::memcpy(d.data() + 32 * i, digests[i].data(), 32);
        int ok = 0;
        check(hbrbc_proof_validate(value.empty() ? nullptr : value.data(), value.size(), index,
                                   d.empty() ? nullptr : d.data(), digests.size(),
                                   root_hash.data(), n, &ok));
        return ok != 0;
    }
    bool operator==(const Proof &o) const {
        return value == o.value && index == o.index && digests == o.digests &&
               root_hash == o.root_hash;
    }
};

// `MerkleTree<T>` (merkle.rs:12-69), built on the GPU.
class MerkleTree {
  public:
    // `MerkleTree::from_vec(Vec<T>)` (merkle.rs:20-33); the reference panics on
    // an empty vector, this throws std::invalid_argument.
    static MerkleTree from_vec(std::vector<Bytes> values) {
        if (values.empty()) throw std::invalid_argument("MerkleTree::from_vec of no values");
        MerkleTree t;
        std::vector<const uint8_t *> p(values.size());
        std::vector<size_t> l(values.size());
        static const uint8_t kEmpty[8] = {0};
        for (size_t i = 0; i < values.size(); ++i) {
            p[i] = values[i].empty() ? kEmpty : values[i].data();
            l[i] = values[i].size();
        }
        t.nodes_.resize(32 * hbrbc_merkle_node_count(values.size()));
        check(hbrbc_merkle_build(p.data(), l.data(), values.size(), t.nodes_.data()));
        t.values_ = std::move(values);
        return t;
    }
    // `proof(index) -> Option<Proof<T>>` (merkle.rs:36-53).
    std::optional<Proof> proof(size_t index) const {
        const size_t n = values_.size();
        std::vector<uint8_t> d(32 * (hbrbc_merkle_max_proof_len(n) + 1));
        size_t nd = 0;
        const int st = hbrbc_merkle_proof(nodes_.data(), n, index, d.data(), &nd);
        if (st == HBRBC_E_INVALID_INDEX) return std::nullopt;
        check(st);
        Proof pr;
        pr.value = values_[index];
        pr.index = index;
        pr.digests.resize(nd);
        for (size_t i = 0; i < nd; ++i) std::memcpy(pr.digests[i].data(), d.data() + 32 * i, 32);
        pr.root_hash = root_hash();
        return pr;
    }
    Digest root_hash() const {
        Digest r;
        std::memcpy(r.data(), nodes_.data() + nodes_.size() - 32, 32);
        return r;
    }
    const std::vector<Bytes> &values() const { return values_; }
    std::vector<Bytes> into_values() && { return std::move(values_); }

  private:
    std::vector<Bytes> values_;
    std::vector<uint8_t> nodes_;  // levels + root, flattened (hbrbc.h)
};

// send_shards framing + encode + tree (broadcast.rs:170-204): BE32 length,
// shard_len = ceil((len + 4) / k), zero padding to (k + m) shards.
inline MerkleTree send_shards(const Coding &coding, const Bytes &value) {
    const size_t k = coding.data_shard_count(), m = coding.parity_shard_count();
    Bytes framed(4 + value.size());
    const uint32_t len = (uint32_t)value.size();
    framed[0] = (uint8_t)(len >> 24);
    framed[1] = (uint8_t)(len >> 16);
    framed[2] = (uint8_t)(len >> 8);
    framed[3] = (uint8_t)len;
    std::memcpy(framed.data() + 4, value.data(), value.size());
    const size_t shard_len = (framed.size() + k - 1) / k;
    framed.resize(shard_len * (k + m), 0);
    std::vector<Bytes> shards(k + m);
    for (size_t i = 0; i < k + m; ++i)
        shards[i].assign(framed.begin() + i * shard_len, framed.begin() + (i + 1) * shard_len);
    if (coding.encode(shards) != HBRBC_OK) throw std::logic_error("wrong shard size");  // 193
    return MerkleTree::from_vec(std::move(shards));
}

// decode_from_shards (broadcast.rs:563-601): reconstruct (an rse error ->
// nullopt), re-tree over all shards, root compare, BE32 length, take(len).
inline std::optional<Bytes> decode_from_shards(const Coding &coding,
                                               std::vector<std::optional<Bytes>> &leaf_values,
                                               const Digest &root_hash) {
    if (coding.reconstruct_shards(leaf_values) != HBRBC_OK) return std::nullopt;
    std::vector<Bytes> shards;
    for (auto &v : leaf_values)
        if (v) shards.push_back(*v);
    MerkleTree mtree = MerkleTree::from_vec(std::move(shards));
    if (mtree.root_hash() != root_hash) return std::nullopt;
    Bytes bytes;
    const auto values = std::move(mtree).into_values();
    for (size_t i = 0; i < coding.data_shard_count() && i < values.size(); ++i)
        bytes.insert(bytes.end(), values[i].begin(), values[i].end());
    if (bytes.size() < 4) return std::nullopt;
    const size_t len = ((size_t)bytes[0] << 24) | ((size_t)bytes[1] << 16) |
                       ((size_t)bytes[2] << 8) | (size_t)bytes[3];
    const size_t take = std::min(len, bytes.size() - 4);
    return Bytes(bytes.begin() + 4, bytes.begin() + 4 + take);
}

}  // namespace hbrbc

#endif  // HBRBC_HPP
