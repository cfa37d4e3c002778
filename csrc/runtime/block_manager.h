// Paged KV-cache block manager core (no Python dependency): used by the pybind11 module
// (block_manager.cpp) and by the sanitizer test binary (csrc/tests/test_native.cpp).
//
// Automatic prefix caching (optional): a full block of prompt tokens whose KV has been computed
// is registered under a chained hash of all tokens up to and including it (prefix_hashes).  A
// newly admitted sequence takes the longest run of registered blocks matching its own hashes
// (match_prefix, reference-counted, shared read-only) and computes only the rest.  Released
// blocks that carry a hash stay cached in an LRU list and count as free; allocation evicts
// the least recently released one only when the plain free list is empty.
//
// Cache-poisoning hardening (cf. vLLM CVE-2025-25183): the chained hash is keyed with a
// per-process random secret (optionally mixed with a per-request salt, e.g. a tenant id), and a
// hash hit alone never shares a block -- match_prefix also requires the cached block's stored
// tokens to equal the request's and its registered parent hash to equal the request's previous
// block hash, so a forged 64-bit collision cannot serve one prompt another prompt's KV.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <list>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace pk {

class BlockManagerCore {
 public:
  // hash_key 0: a random per-process key (tests pass a fixed one for reproducible hashes)
  BlockManagerCore(int64_t num_blocks, int block_size, int64_t watermark_blocks, bool prefix_caching = false,
                   uint64_t hash_key = 0)
      : num_blocks_(num_blocks), block_size_(block_size), watermark_(watermark_blocks), prefix_caching_(prefix_caching) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
    if (hash_key == 0) {
      std::random_device rd;
      hash_key = (static_cast<uint64_t>(rd()) << 32) ^ rd();
    }
    key_ = mix(hash_key ^ 0x6a09e667f3bcc908ULL);
    if (prefix_caching_) {
      tokens_.assign(static_cast<size_t>(num_blocks) * block_size, 0);
      parent_.assign(num_blocks, 0);
    }
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back(static_cast<int32_t>(b));
    ref_.assign(num_blocks, 0);
    hash_.assign(num_blocks, 0);
    lru_pos_.resize(num_blocks);
    in_lru_.assign(num_blocks, 0);
  }

  // free = never-used / unhashed blocks + cached blocks nobody references (evictable)
  int64_t num_free() const { return static_cast<int64_t>(free_.size() + lru_.size()); }
  int64_t num_cached() const { return static_cast<int64_t>(cached_.size()); }
  bool prefix_caching() const { return prefix_caching_; }
  int64_t prefix_queries() const { return queries_; }
  int64_t prefix_hits() const { return hits_; }
  int64_t prefix_collisions() const { return collisions_; }
  int64_t num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int64_t blocks_for(int64_t tokens) const { return (tokens + block_size_ - 1) / block_size_; }

  int64_t needed(int64_t seq, int64_t total_tokens) const {
    auto it = tables_.find(seq);
    const int64_t have = it == tables_.end() ? 0 : static_cast<int64_t>(it->second.size());
    return std::max<int64_t>(0, blocks_for(total_tokens) - have);
  }

  bool can_allocate(int64_t seq, int64_t total_tokens, bool admission) const {
    return needed(seq, total_tokens) + (admission ? watermark_ : 0) <= num_free();
  }

  bool allocate(int64_t seq, int64_t total_tokens) {
    const int64_t need = needed(seq, total_tokens);
    if (need > num_free()) return false;
    auto& t = tables_[seq];
    for (int64_t i = 0; i < need; ++i) t.push_back(take_block());
    return true;
  }

  void free_seq(int64_t seq) {
    auto it = tables_.find(seq);
    if (it == tables_.end()) return;
    for (auto r = it->second.rbegin(); r != it->second.rend(); ++r) release(*r);
    tables_.erase(it);
  }

  // Keyed chained hashes of the full blocks of tokens[0:n] (at most max_out): h_i covers every
  // token of blocks 0..i and the salt.  Never 0.  Lookups verify tokens (match_prefix), so the
  // hash only has to spread, not to be collision-free.
  int64_t prefix_hashes(const int32_t* tokens, int64_t n, uint64_t* out, int64_t max_out, uint64_t salt = 0) const {
    const int64_t nb = std::min<int64_t>(n / block_size_, max_out);
    uint64_t h = salt ? mix(key_ ^ mix(salt)) : key_;
    for (int64_t b = 0; b < nb; ++b) {
      for (int j = 0; j < block_size_; ++j) {
        h ^= static_cast<uint32_t>(tokens[b * block_size_ + j]);
        h *= 0x100000001b3ULL;  // FNV-1a step over each token
      }
      h = mix(h + static_cast<uint64_t>(b));
      out[b] = h ? h : 1;
    }
    return nb;
  }

  // A sequence without blocks takes the longest run of cached blocks matching hashes[0:n] whose
  // stored tokens equal tokens[i*bs:(i+1)*bs] and whose parent hash is hashes[i-1]; returns the
  // number of blocks taken (its first matched * block_size tokens are computed).
  int64_t match_prefix(int64_t seq, const uint64_t* hashes, const int32_t* tokens, int64_t n_tokens, int64_t n) {
    n = std::min<int64_t>(n, n_tokens / block_size_);
    if (!prefix_caching_ || n <= 0 || tables_.count(seq)) return 0;
    queries_ += n;
    std::vector<int32_t> t;
    for (int64_t i = 0; i < n; ++i) {
      auto it = cached_.find(hashes[i]);
      if (it == cached_.end()) break;
      const int32_t b = it->second;
      if (parent_[b] != (i ? hashes[i - 1] : 0) ||
          std::memcmp(&tokens_[static_cast<size_t>(b) * block_size_], tokens + i * block_size_,
                      sizeof(int32_t) * block_size_) != 0) {
        ++collisions_;
        break;
      }
      if (in_lru_[b]) {
        lru_.erase(lru_pos_[b]);
        in_lru_[b] = 0;
      }
      ++ref_[b];
      t.push_back(b);
    }
    hits_ += static_cast<int64_t>(t.size());
    const int64_t got = static_cast<int64_t>(t.size());
    if (got) tables_[seq] = std::move(t);
    return got;
  }

  // Registers the sequence's first n blocks (their KV computed) under hashes[0:n], keeping each
  // block's tokens and parent hash for match_prefix.  A block already registered, or a hash
  // another block already holds, is left as it is.
  void commit_prefix(int64_t seq, const uint64_t* hashes, const int32_t* tokens, int64_t n_tokens, int64_t n) {
    if (!prefix_caching_) return;
    auto it = tables_.find(seq);
    if (it == tables_.end()) return;
    const int64_t m = std::min<int64_t>({n, static_cast<int64_t>(it->second.size()), n_tokens / block_size_});
    for (int64_t i = 0; i < m; ++i) {
      const int32_t b = it->second[i];
      if (hash_[b] != 0 || hashes[i] == 0 || cached_.count(hashes[i])) continue;
      hash_[b] = hashes[i];
      parent_[b] = i ? hashes[i - 1] : 0;
      std::memcpy(&tokens_[static_cast<size_t>(b) * block_size_], tokens + i * block_size_,
                  sizeof(int32_t) * block_size_);
      cached_.emplace(hashes[i], b);
    }
  }

  // Drops every cached block nobody references (back to the plain free list).
  void reset_prefix_cache() {
    while (!lru_.empty()) evict_front(true);
  }

  bool has(int64_t seq) const { return tables_.count(seq) != 0; }
  const std::vector<int32_t>* table_ptr(int64_t seq) const {
    auto it = tables_.find(seq);
    return it == tables_.end() ? nullptr : &it->second;
  }
  std::vector<int32_t> table(int64_t seq) const {
    auto p = table_ptr(seq);
    return p ? *p : std::vector<int32_t>{};
  }
  int64_t num_seqs() const { return static_cast<int64_t>(tables_.size()); }
  int32_t ref_count(int32_t b) const { return ref_.at(b); }

  // Raw-pointer step packer (see block_manager.cpp for the layout).  Returns T.
  int64_t pack(int64_t n, const int64_t* sid, const int32_t* nc, const int32_t* nn, const int32_t* tok, int32_t* ids,
               int32_t* pos, int32_t* slot, int32_t* bt, int64_t bt_rows, int64_t bt_cols, int max_blocks,
               int32_t* cl, int32_t* cu) const {
    if (bt_rows < n || bt_cols < max_blocks) throw std::invalid_argument("block_tables too small");
    int64_t t = 0;
    cu[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
      const auto* tb = table_ptr(sid[i]);
      if (!tb) throw std::runtime_error("pack_step: sequence has no blocks: " + std::to_string(sid[i]));
      const int64_t ctx = static_cast<int64_t>(nc[i]) + nn[i];
      if (blocks_for(ctx) > static_cast<int64_t>(tb->size())) throw std::runtime_error("pack_step: block table too short");
      if (static_cast<int64_t>(tb->size()) > max_blocks) throw std::runtime_error("pack_step: max_blocks exceeded");
      for (int32_t j = 0; j < nn[i]; ++j, ++t) {
        const int64_t p = static_cast<int64_t>(nc[i]) + j;
        ids[t] = tok[t];
        pos[t] = static_cast<int32_t>(p);
        slot[t] = (*tb)[p / block_size_] * block_size_ + static_cast<int32_t>(p % block_size_);
      }
      int32_t* row = bt + i * bt_cols;
      int j = 0;
      for (; j < static_cast<int>(tb->size()); ++j) row[j] = (*tb)[j];
      for (; j < max_blocks; ++j) row[j] = 0;
      cl[i] = static_cast<int32_t>(ctx);
      cu[i + 1] = static_cast<int32_t>(t);
    }
    return t;
  }

 private:
  static uint64_t mix(uint64_t z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }

  void evict_front(bool to_free_list) {
    const int32_t b = lru_.front();
    lru_.pop_front();
    in_lru_[b] = 0;
    cached_.erase(hash_[b]);
    hash_[b] = 0;
    if (to_free_list) free_.push_back(b);
  }

  int32_t take_block() {
    int32_t b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {  // the least recently released cached block
      b = lru_.front();
      evict_front(false);
    }
    ref_[b] = 1;
    return b;
  }

  void release(int32_t b) {
    if (--ref_[b] > 0) return;
    if (hash_[b] != 0) {
      lru_.push_back(b);
      lru_pos_[b] = std::prev(lru_.end());
      in_lru_[b] = 1;
    } else {
      free_.push_back(b);
    }
  }

  int64_t num_blocks_;
  int block_size_;
  int64_t watermark_;
  bool prefix_caching_;
  uint64_t key_ = 0;
  int64_t queries_ = 0, hits_ = 0, collisions_ = 0;
  std::vector<int32_t> tokens_;   // [num_blocks, block_size] tokens of each registered block
  std::vector<uint64_t> parent_;  // hash of the block before it in its sequence (0: first block)
  std::vector<int32_t> free_;
  std::vector<int32_t> ref_;
  std::vector<uint64_t> hash_;
  std::list<int32_t> lru_;
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::vector<char> in_lru_;
  std::unordered_map<uint64_t, int32_t> cached_;
  std::unordered_map<int64_t, std::vector<int32_t>> tables_;
};

}  // namespace pk
