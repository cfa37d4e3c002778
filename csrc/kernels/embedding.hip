// Token embedding gather with the vocab-parallel mask fused in (SURVEY.md §2.3 kernel table,
// "embedding (+vocab-parallel mask)").  Rank r of a TP group holds rows
// [vocab_start, vocab_start + vocab_local) of the table; ids outside its shard produce zero
// rows, and the TP all-reduce that follows assembles the full embedding.  With TP = 1 the
// shard is the whole vocabulary.  One workgroup per token, 16-byte copies.
#include "common.h"

using namespace pk;

namespace {

__global__ void __launch_bounds__(256) embedding_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ table,
                                                        const int* __restrict__ ids, int H, int vocab_start,
                                                        int vocab_local) {
  const int t = blockIdx.x;
  const int local = ids[t] - vocab_start;
  PK_DEVICE_ASSERT(ids[t] >= 0);
  const bool mine = local >= 0 && local < vocab_local;
  const u32x4* src = reinterpret_cast<const u32x4*>(table + static_cast<int64_t>(mine ? local : 0) * H);
  u32x4* dst = reinterpret_cast<u32x4*>(out + static_cast<int64_t>(t) * H);
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) dst[v] = mine ? src[v] : z;
}

}  // namespace

PK_EXPORT int pk_embedding(void* out, const void* table, const void* ids, int T, int H, int vocab_start,
                           int vocab_local, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return -1;
  embedding_kernel<<<T, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const bf16_t*>(table),
                                          static_cast<const int*>(ids), H, vocab_start, vocab_local);
  return PK_CHECK_LAUNCH();
}

// ----------------------------------------------------------------------------------------------
// Host → device copy done by a kernel reading pinned (hipHostMalloc'd, device-mapped) memory.
// The per-step staging buffer is small; copying it on the compute queue avoids handing the
// copy to an SDMA engine, whose cross-queue synchronisation cost ~65 us per step in the decode
// loop (rocprofv3 --memory-copy-trace, tools/trace_timeline.py).
namespace {

__global__ void __launch_bounds__(256) copy_from_host_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                             int64_t n16) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += static_cast<int64_t>(gridDim.x) * 256)
    dst[i] = src[i];
}

}  // namespace

PK_EXPORT int pk_copy_from_host(void* dst, const void* pinned_src, long long bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  if (bytes % 16) return -1;
  const int64_t n16 = bytes / 16;
  const int grid = static_cast<int>(n16 / 256 + 1 < 64 ? n16 / 256 + 1 : 64);
  copy_from_host_kernel<<<grid, 256, 0, stream>>>(static_cast<uint4*>(dst), static_cast<const uint4*>(pinned_src), n16);
  return PK_CHECK_LAUNCH();
}
