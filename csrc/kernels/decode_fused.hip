// Fused QKV projection -> decode attention: ONE launch per decode layer instead of two.
//
// Workgroups [0, n_qkv) first run a QKV tile (the folded-norm split-K projection of
// skinny_tile.h, fp32 slabs stored write-through) and take a ticket on the kv head its head
// belongs to; then every workgroup runs one decode-attention tile (attn_decode.h decode_tile:
// seq, kv head, partition) that waits on its kv head's tickets -- 6 heads x S splits for GQA 4 --
// and reads the slabs with sc1 loads.  No fence anywhere (guide, "Hand-offs measured with sc1
// loads", first row).  The attention tiles' block-table and context loads, their launch and the
// QKV -> attention kernel boundary overlap the QKV tail.  Deadlock-free: the QKV tiles are the
// lowest workgroup indices, dispatched first, and never wait.  Every attention tile requests the
// first two K/V steps of each wave before its hand-off wait (decode_tile PRE = 2): 37.5-38 vs
// 39.5-40 us per 8B layer (tools/qa_stamps.py, profiles/r4_qa_fused_stamps.txt -- the QKV phase
// stretches from ~16 to ~22 us while the attention after the hand-off shrinks from ~20 to ~13 us).
#include "skinny_tile.h"
#include "attn_decode.h"

using namespace pk;

int pk_get_decode_z();                          // attention.hip
int decode_part(int n_seqs, int n_kv, int max_ctx);  // attention.hip: keys per partition (512 or 128)

namespace {

struct AttnArgs {
  bf16_t* out;
  bf16_t* kc;
  bf16_t* vc;
  const int* block_tables;
  const int* context_lens;
  float* part_o;
  float* part_ml;
  int n_q, n_kv, bs, max_blocks, out_stride, n_parts, n_seqs, z;
  float scale2;
  QkvIn qi;
};

template <int MT, int P>
union FusedLds {
  SkinnyLds<MT> g;
  DecodeLds<P, kDecodeWaves> a;
};

// (Removed in round 6, both measured slower on the serving chain: the TP = 1 residual update of
// the previous layer's down slabs as phase 0 of this launch, profiles/r5_phase_ab.jsonl; the
// o-projection as its phase 3 with the partitions merged in-launch, +0.4 % / 70B TP=8 7.86 vs
// 6.70 ms.)
template <int MT, int SS, int P>
__global__ void __launch_bounds__(256, 2) qkv_attn_fused_kernel(const GemmArgs qkv, const AttnArgs aa,
                                                                const Flow fq, const Flow fa, int n_qkv, int n_attn) {
  __shared__ FusedLds<MT, P> lds;
  const int b = blockIdx.x;
  if (b < n_qkv) {
    skinny_tile<MT, kPartial, true, false, false, true, 2, 1>(qkv, b, 0, n_qkv, lds.g, fq);
    __syncthreads();  // the LDS is reused by the attention tile
  }
  if (b < n_attn) {  // small batches: more QKV tiles than attention tiles
    const int x = b % aa.n_kv, y = (b / aa.n_kv) % aa.n_seqs, z = b / (aa.n_kv * aa.n_seqs);
    decode_tile<P, kDecodeWaves, true, SS, 2, 2>(
        aa.out, nullptr, aa.kc, aa.vc, aa.block_tables, aa.context_lens, aa.part_o, aa.part_ml,
        aa.n_q, aa.n_kv, aa.bs, aa.max_blocks, 0, aa.out_stride, aa.n_parts, aa.scale2,
        aa.qi, x, y, z, aa.z, lds.a, fa);
  }
}

}  // namespace

// qkv: the folded-norm QKV projection (packed W, row_scale + nrm_parts; S splits -> fp32 slabs in
// qkv.partial, M = n_seqs rows <= 64); attention over those rows as pk_paged_decode_qkv.  flow:
// int32 >= 131 * 64 words, zeroed once, left zeroed by every launch.
PK_EXPORT int pk_qkv_attn_fused(const GemmArgs* qkv_in, void* out, const void* positions, const void* cos_sin,
                                const void* slots, void* k_cache, void* v_cache, const void* block_tables,
                                const void* context_lens, void* part_o, void* part_ml, int n_q, int n_kv, int bs,
                                int max_blocks, int out_stride, float scale, int max_ctx, int* flow,
                                hipStream_t stream) {
  GemmArgs g = *qkv_in;
  const int n_seqs = g.M;
  if (n_seqs <= 0) return 0;
  // up to 128 rows (one row tile; 128 rows take the MT = 8 tile, whose row scale reads <= 16 parts)
  if (n_seqs > 128 || (n_seqs > 64 && g.nrm_nparts > 16) || g.N != (n_q + 2 * n_kv) * kHD || g.N % 128 || g.S < 1 || g.K % (kKC * g.S) || !g.row_scale ||
      g.nrm_parts == nullptr || g.nrm_nparts < 1 || g.nrm_nparts > 64 || g.partial == nullptr || g.lda % 8 ||
      g.row_offsets != nullptr || n_kv > 64 || n_q % n_kv || n_q / n_kv > 16 || bs % 32 || bs <= 0 ||
      flow == nullptr)  // n_kv <= 64: one ticket slot per kv head below the done counters
    return -1;
  if (max_ctx <= 0 || max_ctx > max_blocks * bs) max_ctx = max_blocks * bs;
  const int P = decode_part(n_seqs, n_kv, max_ctx);  // 128-key partitions when the pairs alone cannot fill the chip
  const int n_parts = (max_ctx + P - 1) / P;
  if (n_parts > 1 && (part_o == nullptr || part_ml == nullptr)) return -2;
  const int z = n_parts < pk_get_decode_z() ? n_parts : pk_get_decode_z();
  g.row_tiles = 1;
  g.tile_rows = n_seqs > 64 ? 128 : 64;
  g.max_group_rows = 0;
  const QkvIn qi{static_cast<const float*>(g.partial), static_cast<const int*>(positions),
                 static_cast<const float*>(cos_sin), static_cast<const int*>(slots), g.S, g.M};
  const AttnArgs aa{static_cast<bf16_t*>(out), static_cast<bf16_t*>(k_cache), static_cast<bf16_t*>(v_cache),
                    static_cast<const int*>(block_tables), static_cast<const int*>(context_lens),
                    static_cast<float*>(part_o), static_cast<float*>(part_ml), n_q, n_kv, bs, max_blocks, out_stride,
                    n_parts, n_seqs, z, scale * 1.4426950408889634f, qi};
  int* done = flow + 64 * kFlowPad;
  int* err = fused_err_word() != nullptr ? fused_err_word() : flow + 128 * kFlowPad;
  const int G = n_q / n_kv;
  // producer: one ticket per (head, split) tile on its kv head; consumer: (G + 2) heads x S
  const Flow fq{flow, done, err, 0, 0, 0, 1, n_q, n_kv, fused_spin_limit()};
  const Flow fa{flow, done, err, (G + 2) * g.S, n_seqs * z, 0, 2, n_q, n_kv, fused_spin_limit()};
  const int n_qkv = (g.N / 128) * g.S;
  const int n_attn = n_kv * n_seqs * z;
  const dim3 grid(n_attn > n_qkv ? n_attn : n_qkv);
  auto go = [&](auto mt, auto ss) {
    constexpr int MT = decltype(mt)::value, SS = decltype(ss)::value;
    if (P == kDecodePartSmall)
      qkv_attn_fused_kernel<MT, SS, kDecodePartSmall><<<grid, 256, 0, stream>>>(g, aa, fq, fa, n_qkv, n_attn);
    else
      qkv_attn_fused_kernel<MT, SS, 512><<<grid, 256, 0, stream>>>(g, aa, fq, fa, n_qkv, n_attn);
  };
  auto go_mt = [&](auto ss) {
    switch ((n_seqs + 15) / 16) {
      case 1: go(std::integral_constant<int, 1>{}, ss); break;
      case 2: go(std::integral_constant<int, 2>{}, ss); break;
      case 3: go(std::integral_constant<int, 3>{}, ss); break;
      case 4: go(std::integral_constant<int, 4>{}, ss); break;
      default: go(std::integral_constant<int, 8>{}, ss); break;  // 65-128 rows: one 128-row tile
    }
  };
  // the attention prologue sums the S slabs of its q / k / v columns: a compile-time S issues all
  // of them at once (a runtime loop serialised 16 sc1 round trips per column at 70B TP=8: S = 16)
  switch (g.S) {
    case 4: go_mt(std::integral_constant<int, 4>{}); break;
    case 8: go_mt(std::integral_constant<int, 8>{}); break;
    case 16: go_mt(std::integral_constant<int, 16>{}); break;
    default: go_mt(std::integral_constant<int, 0>{}); break;
  }
  int rc = PK_CHECK_LAUNCH();
  if (rc || n_parts == 1) return rc;
  if (P == kDecodePartSmall)
    paged_decode_reduce_kernel<kDecodePartSmall><<<dim3(n_q, n_seqs), 128, 0, stream>>>(
        static_cast<bf16_t*>(out), static_cast<const float*>(part_o), static_cast<const float*>(part_ml),
        static_cast<const int*>(context_lens), n_q, out_stride, n_parts, z);
  else
    paged_decode_reduce_kernel<512><<<dim3(n_q, n_seqs), 128, 0, stream>>>(
        static_cast<bf16_t*>(out), static_cast<const float*>(part_o), static_cast<const float*>(part_ml),
        static_cast<const int*>(context_lens), n_q, out_stride, n_parts, z);
  return PK_CHECK_LAUNCH();
}
