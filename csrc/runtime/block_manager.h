// Paged KV-cache block manager core (no Python dependency): used by the pybind11 module
// (block_manager.cpp) and by the sanitizer test binary (csrc/tests/test_native.cpp).
#pragma once
#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace pk {

class BlockManagerCore {
 public:
  BlockManagerCore(int64_t num_blocks, int block_size, int64_t watermark_blocks)
      : num_blocks_(num_blocks), block_size_(block_size), watermark_(watermark_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back(static_cast<int32_t>(b));
  }

  int64_t num_free() const { return static_cast<int64_t>(free_.size()); }
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
    for (int64_t i = 0; i < need; ++i) {
      t.push_back(free_.back());
      free_.pop_back();
    }
    return true;
  }

  void free_seq(int64_t seq) {
    auto it = tables_.find(seq);
    if (it == tables_.end()) return;
    for (auto r = it->second.rbegin(); r != it->second.rend(); ++r) free_.push_back(*r);
    tables_.erase(it);
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
  int64_t num_blocks_;
  int block_size_;
  int64_t watermark_;
  std::vector<int32_t> free_;
  std::unordered_map<int64_t, std::vector<int32_t>> tables_;
};

}  // namespace pk
