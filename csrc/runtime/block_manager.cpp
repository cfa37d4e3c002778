// pybind11 face of the native runtime (see block_manager.h for the allocator core).
//
// The reference has no engine; this is the native runtime piece behind the
// continuous-batching scheduler (SURVEY.md §3.6 "L5 Engine", §5.7 paged KV).  It owns the KV
// block free list, every sequence's block table, and `pack_step`, which writes one engine
// step's flattened device inputs (token ids, positions, slot mapping, padded block tables,
// context lengths, query offsets) straight into caller-provided pinned int32 buffers, so the
// Python side does no per-token work.  Sizing: at 288 GB HBM3E an 8B model leaves ~250 GB for
// KV = ~1.9 M tokens = ~60k blocks of 32; the free list is a vector used as a stack.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime/block_manager.h"

namespace py = pybind11;
using I32 = py::array_t<int32_t, py::array::c_style>;
using I64 = py::array_t<int64_t, py::array::c_style>;
using U64 = py::array_t<uint64_t, py::array::c_style>;

class BlockManager : public pk::BlockManagerCore {
 public:
  using pk::BlockManagerCore::BlockManagerCore;

  U64 prefix_hashes_py(I32 tokens, int64_t max_blocks, uint64_t salt) const {
    const int64_t n = tokens.shape(0);
    U64 out(std::max<int64_t>(0, std::min<int64_t>(n / block_size(), max_blocks)));
    prefix_hashes(tokens.data(), n, out.mutable_data(), out.shape(0), salt);
    return out;
  }
  int64_t match_prefix_py(int64_t seq, U64 hashes, I32 tokens, int64_t n) {
    return match_prefix(seq, hashes.data(), tokens.data(), tokens.shape(0), std::min<int64_t>(n, hashes.shape(0)));
  }
  void commit_prefix_py(int64_t seq, U64 hashes, I32 tokens, int64_t n) {
    commit_prefix(seq, hashes.data(), tokens.data(), tokens.shape(0), std::min<int64_t>(n, hashes.shape(0)));
  }

  int64_t pack_step(I64 seq_ids, I32 num_computed, I32 num_new, I32 tokens, I32 input_ids, I32 positions,
                    I32 slot_mapping, I32 block_tables, int max_blocks, I32 context_lens, I32 cu_q) {
    const int64_t n = seq_ids.shape(0);
    if (num_computed.shape(0) < n || num_new.shape(0) < n || context_lens.shape(0) < n || cu_q.shape(0) < n + 1)
      throw std::invalid_argument("pack_step: per-sequence arrays too small");
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) total += num_new.data()[i];
    if (tokens.shape(0) < total || input_ids.shape(0) < total || positions.shape(0) < total ||
        slot_mapping.shape(0) < total)
      throw std::invalid_argument("pack_step: token arrays too small");
    return pack(n, seq_ids.data(), num_computed.data(), num_new.data(), tokens.data(), input_ids.mutable_data(),
                positions.mutable_data(), slot_mapping.mutable_data(), block_tables.mutable_data(),
                block_tables.shape(0), block_tables.shape(1), max_blocks, context_lens.mutable_data(),
                cu_q.mutable_data());
  }
};

void bind_step_channel(py::module_& m);  // step_channel.cpp
void bind_vote_board(py::module_& m);    // vote_board.cpp

PYBIND11_MODULE(_pk_runtime, m) {
  m.doc() = "polykey native runtime: paged KV block manager, step packer, TP step channel";
  bind_step_channel(m);
  bind_vote_board(m);
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int64_t, int, int64_t, bool, uint64_t>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("watermark_blocks") = 0, py::arg("prefix_caching") = false, py::arg("hash_key") = 0)
      .def_property_readonly("prefix_caching", &BlockManager::prefix_caching)
      .def_property_readonly("num_cached", &BlockManager::num_cached)
      .def_property_readonly("prefix_queries", &BlockManager::prefix_queries)
      .def_property_readonly("prefix_hits", &BlockManager::prefix_hits)
      .def_property_readonly("prefix_collisions", &BlockManager::prefix_collisions)
      .def("prefix_hashes", &BlockManager::prefix_hashes_py, py::arg("tokens"), py::arg("max_blocks") = INT64_MAX,
           py::arg("salt") = 0)
      .def("match_prefix", &BlockManager::match_prefix_py, py::arg("seq"), py::arg("hashes"), py::arg("tokens"),
           py::arg("n"))
      .def("commit_prefix", &BlockManager::commit_prefix_py, py::arg("seq"), py::arg("hashes"), py::arg("tokens"),
           py::arg("n"))
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def("ref_count", &BlockManager::ref_count)
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
