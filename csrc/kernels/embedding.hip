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
