// Paged KV-cache block manager + per-step batch packer (CPU side of the engine hot loop).
//
// The reference has no engine; this is the native runtime piece behind the
// continuous-batching scheduler (SURVEY.md §3.6 "L5 Engine", §5.7 paged KV).  It owns:
//   * a free-list allocator over `num_blocks` KV blocks of `block_size` tokens,
//   * each sequence's block table (logical block i -> physical block id),
//   * `pack_step`, which writes one engine step's flattened device inputs (token ids,
//     positions, slot mapping, padded block tables, context lengths, query offsets) straight
//     into caller-provided (pinned) int32 buffers, so the Python side does no per-token work.
// Sizing: at 288 GB HBM3E an 8B model leaves ~250 GB for KV = ~1.9 M tokens = ~60k blocks of
// 32; the free list is a plain vector used as a stack (O(1) alloc/free, no fragmentation).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

class BlockManager {
 public:
  BlockManager(int64_t num_blocks, int block_size, int64_t watermark_blocks)
      : num_blocks_(num_blocks), block_size_(block_size), watermark_(watermark_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back(static_cast<int32_t>(b));
  }

  int64_t num_free() const { return static_cast<int64_t>(free_.size()); }
  int64_t num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int64_t blocks_for(int64_t tokens) const { return (tokens + block_size_ - 1) / block_size_; }

  // Blocks still needed for `seq` to hold `total_tokens` tokens.
  int64_t needed(int64_t seq, int64_t total_tokens) const {
    auto it = tables_.find(seq);
    const int64_t have = it == tables_.end() ? 0 : static_cast<int64_t>(it->second.size());
    return std::max<int64_t>(0, blocks_for(total_tokens) - have);
  }

  // Admission check for a new/preempted sequence keeps `watermark` blocks in reserve so
  // running decodes are not immediately preempted by a large prefill.
  bool can_allocate(int64_t seq, int64_t total_tokens, bool admission) const {
    const int64_t need = needed(seq, total_tokens);
    return need + (admission ? watermark_ : 0) <= num_free();
  }

  // Grow `seq`'s table to cover `total_tokens`. Returns false (and changes nothing) if short.
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
    for (auto it2 = it->second.rbegin(); it2 != it->second.rend(); ++it2) free_.push_back(*it2);
    tables_.erase(it);
  }

  bool has(int64_t seq) const { return tables_.count(seq) != 0; }

  std::vector<int32_t> table(int64_t seq) const {
    auto it = tables_.find(seq);
    return it == tables_.end() ? std::vector<int32_t>{} : it->second;
  }

  int64_t num_seqs() const { return static_cast<int64_t>(tables_.size()); }

  // Pack one step. Per scheduled sequence i:
  //   seq_ids[i], num_computed[i] (tokens already in the KV cache), num_new[i] (tokens this
  //   step), tokens = concatenated new token ids (sum num_new).
  // Outputs (int32, caller-allocated, len >= needed):
  //   input_ids[T], positions[T], slot_mapping[T], block_tables[n, max_blocks] (padded with 0),
  //   context_lens[n] (= num_computed + num_new), cu_q[n + 1]
  // Returns T (total tokens).
  int64_t pack_step(py::array_t<int64_t, py::array::c_style> seq_ids, py::array_t<int32_t, py::array::c_style> num_computed,
                    py::array_t<int32_t, py::array::c_style> num_new, py::array_t<int32_t, py::array::c_style> tokens,
                    py::array_t<int32_t, py::array::c_style> input_ids, py::array_t<int32_t, py::array::c_style> positions,
                    py::array_t<int32_t, py::array::c_style> slot_mapping,
                    py::array_t<int32_t, py::array::c_style> block_tables, int max_blocks,
                    py::array_t<int32_t, py::array::c_style> context_lens, py::array_t<int32_t, py::array::c_style> cu_q) {
    const int64_t n = seq_ids.shape(0);
    auto sid = seq_ids.unchecked<1>();
    auto nc = num_computed.unchecked<1>();
    auto nn = num_new.unchecked<1>();
    auto tok = tokens.unchecked<1>();
    auto ids = input_ids.mutable_unchecked<1>();
    auto pos = positions.mutable_unchecked<1>();
    auto slot = slot_mapping.mutable_unchecked<1>();
    auto bt = block_tables.mutable_unchecked<2>();
    auto cl = context_lens.mutable_unchecked<1>();
    auto cu = cu_q.mutable_unchecked<1>();
    if (block_tables.shape(0) < n || block_tables.shape(1) < max_blocks) throw std::invalid_argument("block_tables too small");
    int64_t t = 0;
    cu(0) = 0;
    for (int64_t i = 0; i < n; ++i) {
      auto it = tables_.find(sid(i));
      if (it == tables_.end()) throw std::runtime_error("pack_step: sequence has no blocks: " + std::to_string(sid(i)));
      const auto& tb = it->second;
      const int64_t ctx = static_cast<int64_t>(nc(i)) + nn(i);
      if (blocks_for(ctx) > static_cast<int64_t>(tb.size())) throw std::runtime_error("pack_step: block table too short");
      if (static_cast<int64_t>(tb.size()) > max_blocks) throw std::runtime_error("pack_step: max_blocks exceeded");
      for (int32_t j = 0; j < nn(i); ++j, ++t) {
        const int64_t p = static_cast<int64_t>(nc(i)) + j;
        ids(t) = tok(t);
        pos(t) = static_cast<int32_t>(p);
        slot(t) = tb[p / block_size_] * block_size_ + static_cast<int32_t>(p % block_size_);
      }
      int j = 0;
      for (; j < static_cast<int>(tb.size()); ++j) bt(i, j) = tb[j];
      for (; j < max_blocks; ++j) bt(i, j) = 0;
      cl(i) = static_cast<int32_t>(ctx);
      cu(i + 1) = static_cast<int32_t>(t);
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

PYBIND11_MODULE(_pk_runtime, m) {
  m.doc() = "polykey native runtime: paged KV block manager and step packer";
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int64_t, int, int64_t>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("watermark_blocks") = 0)
      .def_property_readonly("num_free", &BlockManager::num_free)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_seqs", &BlockManager::num_seqs)
      .def("blocks_for", &BlockManager::blocks_for)
      .def("needed", &BlockManager::needed)
      .def("can_allocate", &BlockManager::can_allocate, py::arg("seq"), py::arg("total_tokens"),
           py::arg("admission") = false)
      .def("allocate", &BlockManager::allocate)
      .def("free_seq", &BlockManager::free_seq)
      .def("has", &BlockManager::has)
      .def("table", &BlockManager::table)
      .def("pack_step", &BlockManager::pack_step);
}
