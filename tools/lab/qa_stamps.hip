// Lab build (not part of the package): the fused QKV -> decode attention launch of
// csrc/kernels/decode_fused.hip with per-workgroup wall-clock stamps (s_memrealtime, 100 MHz),
// to see where its 38 us per 8B layer go: when each QKV tile ends, when each attention tile
// starts attending (past its hand-off wait) and when it ends.
//   hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -I csrc/kernels tools/lab/qa_stamps.hip -o tools/lab/libqa_stamps.so
// Stamps: st[4 * b + 0] start, + 1 QKV tile end (0: none), + 2 attention end, + 3 XCC id.
#include "skinny_tile.h"
#include "attn_decode.h"

using namespace pk;

namespace {

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

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

template <int MT, int SS, int P, int PRE>
__global__ void __launch_bounds__(256, 2) qa_stamped(const GemmArgs qkv, const AttnArgs aa, const Flow fq,
                                                     const Flow fa, int n_qkv, int n_attn,
                                                     unsigned long long* __restrict__ st) {
  __shared__ FusedLds<MT, P> lds;
  const int b = blockIdx.x;
  const unsigned long long t0 = now();
  unsigned long long t1 = 0;
  if (b < n_qkv) {
    skinny_tile<MT, kPartial, true, false, false, true, 2, 1>(qkv, b, 0, n_qkv, lds.g, fq);
    __syncthreads();
    t1 = now();
  }
  if (b < n_attn) {
    const int x = b % aa.n_kv, y = (b / aa.n_kv) % aa.n_seqs, z = b / (aa.n_kv * aa.n_seqs);
    decode_tile<P, kDecodeWaves, true, SS, 2, PRE>(
        aa.out, nullptr, aa.kc, aa.vc, aa.block_tables, aa.context_lens, aa.part_o, aa.part_ml, nullptr, aa.n_q,
        aa.n_kv, aa.bs, aa.max_blocks, 0, aa.out_stride, aa.n_parts, aa.scale2, aa.qi, x, y, z, aa.z, lds.a, fa);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    st[4 * b + 0] = t0;
    st[4 * b + 1] = t1;
    st[4 * b + 2] = now();
    st[4 * b + 3] = __builtin_amdgcn_s_getreg((20 - 1) << 11 | 0 << 6 | 20);  // HW_REG_XCC_ID (id 20), 4 bits
  }
}

}  // namespace

int* fused_err_word() { return nullptr; }
int fused_spin_limit() { return 1 << 20; }

// same contract as pk_qkv_attn_fused for n_seqs <= 64, S in {4, 8}, 512-key partitions, one
// partition per sequence (max_ctx <= 512)
extern "C" int qa_stamped_launch(const GemmArgs* qkv_in, void* out, const void* positions, const void* cos_sin,
                                 const void* slots, void* k_cache, void* v_cache, const void* block_tables,
                                 const void* context_lens, int n_q, int n_kv, int bs, int max_blocks, int out_stride,
                                 float scale, int* flow, void* stamps, int pre, hipStream_t stream) {
  GemmArgs g = *qkv_in;
  const int n_seqs = g.M;
  if (n_seqs <= 0 || n_seqs > 64 || (g.S != 4 && g.S != 8) || g.N != (n_q + 2 * n_kv) * kHD || n_kv > 64) return -1;
  g.row_tiles = 1;
  g.tile_rows = 64;
  g.max_group_rows = 0;
  const QkvIn qi{static_cast<const float*>(g.partial), static_cast<const int*>(positions),
                 static_cast<const float*>(cos_sin), static_cast<const int*>(slots), g.S, g.M};
  const AttnArgs aa{static_cast<bf16_t*>(out), static_cast<bf16_t*>(k_cache), static_cast<bf16_t*>(v_cache),
                    static_cast<const int*>(block_tables), static_cast<const int*>(context_lens), nullptr, nullptr,
                    n_q, n_kv, bs, max_blocks, out_stride, 1, n_seqs, 1, scale * 1.4426950408889634f, qi};
  int* done = flow + 64 * kFlowPad;
  int* err = flow + 128 * kFlowPad;
  const int G = n_q / n_kv;
  const Flow fq{flow, done, err, 0, 0, 0, 1, n_q, n_kv, 1 << 20};
  const Flow fa{flow, done, err, (G + 2) * g.S, n_seqs, 0, 2, n_q, n_kv, 1 << 20};
  const int n_qkv = (g.N / 128) * g.S;
  const int n_attn = n_kv * n_seqs;
  const dim3 grid(n_attn > n_qkv ? n_attn : n_qkv);
  auto st = static_cast<unsigned long long*>(stamps);
  if (g.S != 4) return -1;
  if (pre == 2)
    qa_stamped<4, 4, 512, 2><<<grid, 256, 0, stream>>>(g, aa, fq, fa, n_qkv, n_attn, st);
  else
    qa_stamped<4, 4, 512, 0><<<grid, 256, 0, stream>>>(g, aa, fq, fa, n_qkv, n_attn, st);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---- the fused decode MLP (gemm_skinny.hip mlp_fused_kernel), stamped the same way: st[4 b + 1] =
// end of the gate_up tile, + 2 = end of the down tile (8B shape: S = 1 gate_up, 128-row down tiles)
namespace {
template <int MT, int DKR>
__global__ void __launch_bounds__(256, 2) mlp_stamped(const GemmArgs gu, const GemmArgs dn, const Flow fgu,
                                                      const Flow fdn, int n_gu, int n_dn,
                                                      unsigned long long* __restrict__ st) {
  __shared__ SkinnyLds<MT> lds;
  const int b = blockIdx.x;
  const unsigned long long t0 = now();
  unsigned long long t1 = 0;
  if (b < n_gu) {
    skinny_tile<MT, kSiluMul, true, false, true, true, 2, 1>(gu, b, 0, n_gu, lds, fgu);
    __syncthreads();
    t1 = now();
  }
  if (b < n_dn) skinny_tile<MT, kPartial, true, false, false, false, DKR, 2>(dn, b, 0, n_dn, lds, fdn);
  __syncthreads();
  if (threadIdx.x == 0) {
    st[4 * b + 0] = t0;
    st[4 * b + 1] = t1;
    st[4 * b + 2] = now();
    st[4 * b + 3] = __builtin_amdgcn_s_getreg((20 - 1) << 11 | 0 << 6 | 20);
  }
}
}  // namespace

extern "C" int mlp_stamped_launch(const GemmArgs* gu_in, const GemmArgs* dn_in, int* flow, void* stamps,
                                  hipStream_t stream) {
  GemmArgs gu = *gu_in, dn = *dn_in;
  if (gu.M != 64 || gu.S != 1 || dn.K != gu.N / 2) return -1;
  gu.row_tiles = dn.row_tiles = 1;
  gu.tile_rows = dn.tile_rows = 64;
  gu.max_group_rows = dn.max_group_rows = 0;
  int* done = flow + 64 * kFlowPad;
  int* err = flow + 128 * kFlowPad;
  const int dkr = (dn.N / 128) * dn.S < 192 ? 1 : 2;
  Flow fgu{flow, done, err, 0, 0, dn.K / dn.S, 1, 0, 0, 1 << 20};
  Flow fdn{flow, done, err, (dn.K / dn.S) / 64, dn.N / (64 * dkr), dn.K / dn.S, 2, 0, 0, 1 << 20};
  const int n_gu = gu.N / 128, n_dn = (dn.N / (64 * dkr)) * dn.S;
  const dim3 grid(n_gu > n_dn ? n_gu : n_dn);
  auto st = static_cast<unsigned long long*>(stamps);
  if (dkr == 2)
    mlp_stamped<4, 2><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn, st);
  else
    mlp_stamped<4, 1><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn, st);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
