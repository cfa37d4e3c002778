// Paged attention (decode + varlen causal prefill) for gfx950, head_dim = 128, bf16 KV.
//
// One wave computes 16 "columns" against a stream of 32-key steps with
// mfma_f32_16x16x32_bf16.  A column is (query row, head): in DECODE the 16 columns are
// the G query heads that share one KV head (GQA group, G <= 16, unused columns zero);
// in PREFILL they are 16 consecutive query tokens of one head.  Per 32-key step:
//
//   S^T (32 keys x 16 cols) = K (A operand, rows = keys) . Q^T (B operand)    8 MFMAs
//   online softmax on S^T in registers (per column: max over 8 regs + 2 xor-shuffles)
//   O^T (128 d x 16 cols) += V^T (A, rows = d) . P^T (B, k = keys)             8 MFMAs
//
// Two permutations make every operand a single 16-byte-per-lane load with no LDS
// transpose (guide §3 "accumulator tile as the next MFMA's operand"):
//   * head-dim: lane group g = lane>>4 owns dims [32g, 32g+32) across the four k-steps, so a
//     lane reads 64 contiguous bytes of its key row (K) and of its query row (Q);
//   * keys: tile t, row r holds key 8*(r>>2) + 4t + (r&3), so after QK^T lane group g holds
//     keys 8g..8g+7 of its column -- exactly the P^T B-fragment layout -- and the matching
//     V^T A-fragment is 8 consecutive tokens of one channel: one 16-byte load from the V
//     cache, stored per (block, kv head) in fragment-native 32-token tiles
//     [d / 16][key / 8][d % 16][key % 8] (common.h vcache_off: a wave's d-tile is one KiB).
// Softmax runs in base 2 with the 1/sqrt(d) scale folded into one multiply.  K/V go straight
// from global memory to VGPRs (decode is HBM-bound: guide §5 "GEMV / M <= 16" row); waves of a
// workgroup that read the same K/V tile hit the CU's L1.
// Decode splits long contexts into partitions of kPart keys (flash-decoding) and merges them
// in a second kernel; sequences that fit one partition are finished in place.
#include "attn_decode.h"

using namespace pk;

namespace {

template <int kPart, int NW, bool FROM_QKV, int SS = 0>
__global__ void __launch_bounds__(64 * NW) paged_decode_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    float* __restrict__ part_o, float* __restrict__ part_ml, int n_q, int n_kv, int bs,
    int max_blocks, int q_stride, int out_stride, int n_parts, float scale2, const QkvIn qi) {
  __shared__ DecodeLds<kPart, NW> lds;
  decode_tile<kPart, NW, FROM_QKV, SS>(out, q, kc, vc, block_tables, context_lens, part_o, part_ml, n_q, n_kv,
                                       bs, max_blocks, q_stride, out_stride, n_parts, scale2, qi, blockIdx.x, blockIdx.y,
                                       blockIdx.z, gridDim.z, lds, Flow{});
}

// ----------------------------------------------------------------------------- prefill
// grid (max_q_blocks, n_seqs, n_kv * head_groups), block 64*W with W = min(G, 8) waves:
// wave w = query head h*G + sub*W + w, 16 query tokens per workgroup.  cu_q: query offsets
// (relative to q/out), ctx: total keys per seq.  At most 8 waves keeps the VGPR cap at 256.
__global__ void __launch_bounds__(512) paged_prefill_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    const int* __restrict__ cu_q, int n_q, int n_kv, int bs, int max_blocks, int q_stride, int out_stride,
    float scale2) {
  const int qb = blockIdx.x, seq = blockIdx.y;
  const int q0 = cu_q[seq], L = cu_q[seq + 1] - q0;
  if (qb * 16 >= L) return;
  const int ctx = context_lens[seq];
  const int G = n_q / n_kv;
  const int W = blockDim.x >> 6;
  const int h = blockIdx.z / (G / W), sub = blockIdx.z % (G / W);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int hq = h * G + sub * W + w;
  const int qi = qb * 16 + r;
  const bool valid = qi < L;
  const int qpos = ctx - L + qi;
  const int last_q = min(L - 1, qb * 16 + 15);
  const int k_end = min(ctx, ctx - L + last_q + 1);
  bf16x8_t qf[4];
  load_q(qf, q + static_cast<int64_t>(q0 + (valid ? qi : 0)) * q_stride + hq * kHD, valid);
  WaveState st;
  init_state(st);
  KVFrag fa, fb;
  attend(st, qf, kc + static_cast<int64_t>(h) * bs * kHD, vc + static_cast<int64_t>(h) * kHD * bs,
         static_cast<int64_t>(n_kv) * bs * kHD, block_tables + static_cast<int64_t>(seq) * max_blocks, 0, bs, 0,
         k_end, kStep, ctx, valid ? qpos : -1, scale2, fa, fb);
  const float lsum = col_sum(st.l);
  if (!valid) return;
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  bf16_t* o = out + static_cast<int64_t>(q0 + qi) * out_stride + hq * kHD;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    uint2 v;
    v.x = pack2(st.o[dt][0] * inv, st.o[dt][1] * inv);
    v.y = pack2(st.o[dt][2] * inv, st.o[dt][3] * inv);
    *reinterpret_cast<uint2*>(o + 16 * dt + 4 * g) = v;
  }
}

// ------------------------------------------- prefill on 32x32x16 MFMAs, P kept in registers
// One wave owns 32 queries of one head against 64-key steps (guide Appendix B "Fused attention
// prefill" structure):
//   X_t = S^T (32 keys x 32 queries) = K_t . Q^T     (A = K rows, B = Q^T; 8 MFMAs per key tile t)
//   softmax per query = per lane column: 16 keys in the lane's registers x 2 tiles, the other
//   32 keys of the step in lane l ^ 32 (one permlane32_swap for the max)
//   O^T (128 d x 32 queries) += V^T . P^T           (A = V^T rows, B = X_t converted to bf16)
// The accumulator of the first product is the B operand of the second with no lane movement
// (guide §3 "An accumulator tile as the next MFMA's operand"): registers 8s..8s+7 of X_t are
// the k-step s fragment, whose element j of lane half h is X row 16s + 8(j>>2) + 4h + (j&3).
// The K rows of the QK^T A operand are read with bits 2 and 3 of the key index swapped, so
// X row rho holds key swap23(rho) and that permuted k order becomes the NATURAL key order
// 16s + 8h + j -- V^T fragments are then plain 16-byte reads of 8 consecutive keys.
// Per 64-key step and wave: 32 MFMAs of 32x32x16 against 32 KiB of LDS fragment reads and 32
// exp2 per lane.
// Workgroup: 8 waves = G heads of the kv head's GQA group x (8 / G) 32-query groups; K / V
// tiles staged through LDS (register staged, double buffered, one barrier per step).
constexpr int kKS = 64;            // keys per step
constexpr int kKRow32 = kHD + 8;   // K_s row (bf16): 272 B, 16 rows on distinct bank groups
constexpr int kVRow32 = kKS + 8;   // V_s row (bf16): 144 B

typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ int swap23(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }

template <int G, int NW>
__global__ void __launch_bounds__(64 * NW, 2) paged_prefill_mfma32_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    const int* __restrict__ cu_q, int n_kv, int bs, int max_blocks, int q_stride, int out_stride, float scale2) {
  __shared__ __attribute__((aligned(16))) bf16_t K_s[2][kKS][kKRow32];
  __shared__ __attribute__((aligned(16))) bf16_t V_s[2][kHD][kVRow32];
  static_assert(NW % G == 0, "a workgroup holds whole GQA groups");
  constexpr int kQG = NW / G;          // 32-query groups per workgroup
  constexpr int NJ = 1024 / (64 * NW); // K (and V^T) granules staged per thread per step
  constexpr int kPQ = 32 * kQG;        // queries per workgroup
  // grid (n_kv, n_seqs, q blocks) with the q block slowest: dispatch order is x fastest, so every
  // (head, sequence) pair's LAST -- heaviest, causal -- query block is launched first
  const int qb = gridDim.z - 1 - blockIdx.z, seq = blockIdx.y, h = blockIdx.x;
  const int q0 = cu_q[seq], L = cu_q[seq + 1] - q0;
  if (qb * kPQ >= L) return;
  const int ctx = context_lens[seq];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int hq = h * G + w % G;
  const int qi = qb * kPQ + (w / G) * 32 + r;  // this lane's query (column of X and O^T)
  const bool valid = qi < L;
  const int qpos = valid ? ctx - L + qi : -1;
  const int last_q = min(L - 1, qb * kPQ + kPQ - 1);
  const int k_end = min(ctx, ctx - L + last_q + 1);
  const int nsteps = (k_end + kKS - 1) / kKS;
  const int wave_last_q = min(L - 1, qb * kPQ + (w / G) * 32 + 31);
  const int wave_steps = (min(ctx, ctx - L + wave_last_q + 1) + kKS - 1) / kKS;
  const int wave_first_pos = ctx - L + qb * kPQ + (w / G) * 32;  // position of the wave's first query
  const int64_t blk_stride = static_cast<int64_t>(n_kv) * bs * kHD;
  const bf16_t* kch = kc + static_cast<int64_t>(h) * bs * kHD;
  const bf16_t* vch = vc + static_cast<int64_t>(h) * kHD * bs;
  const int* bt = block_tables + static_cast<int64_t>(seq) * max_blocks;

  // ---- staging: per step 1024 K granules (16 B = 8 dims of one key) and 1024 V^T granules
  // (8 keys of one channel); thread tid stages granules tid and tid + 512 of each
  // Which granule a lane stages is permuted inside its wave's 1 KiB (loads stay whole lines) so
  // that the LDS stores -- ds_write_b128 banks over 8 contiguous lanes, (a/4) mod 32
  // (MI355X_MICROARCH.md §LDS) -- hit 8 distinct 4-bank groups: K piece lane' takes lane bit 2 at
  // its bit 4 (dims +32: +16 banks) and lane bits 3-4 at its bits 2-3; V^T channel bit 2 comes
  // from lane bit 2 (+4 rows = +16 banks) and channel bits 0-1 / 3 from lane bits 3-4 / 5.
  const int kpl = (lane & 3) | (((lane >> 3) & 3) << 2) | (((lane >> 2) & 1) << 4) | (lane & 32);
  const int vdl = (((lane >> 2) & 1) << 2) | ((lane >> 3) & 3) | (((lane >> 5) & 1) << 3);
  const int vkg = lane & 3;
  // granule g = j * 64 NW + tid (j < NJ): 32-token tile g >> 9, wave chunk (g >> 6) & 7 of it
  u32x4 ks[NJ], vs[NJ];
  auto load_tile = [&](int step) {
    const int s0 = min(step, nsteps - 1) * kKS;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int g = j * 64 * NW + tid, i = g >> 9, ch = (g >> 6) & 7;
      const int tok = min(s0 + 32 * i, ((k_end - 1) >> 5) << 5);
      const int64_t base = static_cast<int64_t>(bt[tok / bs]) * blk_stride;
      // K: fragment-native tile of 32 tokens, piece (ch, kpl) (common.h kcache_off)
      ks[j] = *reinterpret_cast<const u32x4*>(kch + base + (tok % bs) * kHD + ((ch << 6) | kpl) * 8);
      // V: channel 16 ch + vdl, keys 8 vkg .. of the same 32-token tile (common.h vcache_off)
      vs[j] = *reinterpret_cast<const u32x4*>(vch + base + vcache_off(tok % bs + 8 * vkg, 16 * ch + vdl));
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int g = j * 64 * NW + tid, i = g >> 9, ch = (g >> 6) & 7;
      // invert kcache_off for piece (ch, kpl): lane' = kpl, (t, kk) = ch
      const int kkey = 8 * ((kpl >> 2) & 3) + 4 * (ch >> 2) + (kpl & 3);
      const int kd = 32 * (kpl >> 4) + 8 * (ch & 3);
      *reinterpret_cast<u32x4*>(&K_s[buf][32 * i + kkey][kd]) = ks[j];
      *reinterpret_cast<u32x4*>(&V_s[buf][16 * ch + vdl][32 * i + 8 * vkg]) = vs[j];
    }
  };

  // Q^T B-fragments: k-step kk (dims 16 kk + 8 hh .. +8) of query qi
  bf16x8_t qf[8];
  {
    const bf16_t* qp = q + static_cast<int64_t>(q0 + (valid ? qi : 0)) * q_stride + hq * kHD + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) qf[kk] = valid ? ld8(qp + 16 * kk) : zero8();
  }
  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m_run = kNegBig, l_run = 0.f;
  const int krow = swap23(r);

  auto compute = [&](int step, int buf) {
    if (step >= wave_steps) return;
    const int s0 = step * kKS;
    // ---- X_t = S^T for the two 32-key tiles
    f32x16 x[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) x[t][i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(&K_s[buf][32 * t + krow][16 * kk + 8 * hh]);
        x[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], x[t], 0, 0, 0);
      }
    }
    // ---- online softmax over the lane's 32 keys (+ the other half in lane ^ 32).  The max is
    // taken on raw scores (scale2 > 0) and the scale folded into the exponent's FMA; keys are
    // masked only on steps that reach past the wave's first query or the context end.
    float mx = kNegBig;
    if (s0 + kKS - 1 > wave_first_pos || s0 + kKS > ctx) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = s0 + 32 * t + (i & 7) + 8 * hh + 16 * (i >> 3);  // swap23 of X row
          const bool ok = key < ctx && key <= qpos;
          x[t][i] = ok ? x[t][i] : -INFINITY;
        }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, x[t][i]);
    {
      auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
    }
    const float m_new = fmaxf(m_run, mx * scale2);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    const bool rescale = __any(m_new != m_run);  // wave-uniform: skip the O^T scaling if no max moved
    m_run = m_new;
    float psum = 0.f;
    bf16x8_t pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          p[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(x[t][8 * s2 + j], scale2, -m_new));
          psum += p[j];
        }
        pf[t][s2] = pack_p(p);
      }
    l_run = l_run * alpha + psum;
    // ---- O^T += V^T . P^T
    if (rescale) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8_t vf =
              *reinterpret_cast<const bf16x8_t*>(&V_s[buf][32 * dt + r][32 * t + 16 * s2 + 8 * hh]);
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[t][s2], o[dt], 0, 0, 0);
        }
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    load_tile(step + 1);  // the next step's global loads fly during this step's math
    compute(step, buf);
    store_tile(buf ^ 1);  // every wave finished reading buf ^ 1 before the previous barrier
    __syncthreads();
  }
  // ---- O = O^T / l: lane holds query qi, dims dt*32 + (i&3) + 8 (i>>2) + 4 hh
  {
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
    l_run = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  }
  if (!valid) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16_t* op = out + static_cast<int64_t>(q0 + qi) * out_stride + hq * kHD + 4 * hh;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      uint2 v;
      v.x = pack2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
      v.y = pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
      *reinterpret_cast<uint2*>(op + 32 * dt + 8 * g4) = v;
    }
}


constexpr int kDecodePart = 512;  // keys per decode partition (ops/attention.py _PART must match)

}  // namespace

// Workspace for decode: part_o [n_seqs, n_q, n_parts, 128] fp32, part_ml [n_seqs, n_q, n_parts, 2] fp32,
// n_parts counted in the smallest partition (kDecodePartSmall, ops/attention.py _PART_MIN).
PK_EXPORT int pk_decode_num_parts(int max_context) { return (max_context + kDecodePartSmall - 1) / kDecodePartSmall; }

// Keys per partition of a launch: 512, or 128 when (seq, kv head) pairs x partitions would leave
// most CUs idle -- the 70B TP=8 shard has ONE kv head per rank, so 64 sequences are 64 workgroups
// at 512 keys (22.5 us for 12.6 MB of K/V, profiles/r4_solo_70b_tp8_unfused_kstats.md) and 256 at
// 128 (4 partials per sequence, merged after).
int decode_part(int n_seqs, int n_kv, int max_ctx) {
  const int big = (max_ctx + kDecodePart - 1) / kDecodePart;
  const int z = big < g_decode_z ? big : g_decode_z;
  return n_seqs * n_kv * z < g_decode_fill ? kDecodePartSmall : kDecodePart;
}

// Workgroup count below which decode takes 128-key partitions (default 64; 0: always 512 keys).
// The partition slabs must be sized for the bound (ops/attention.py decode_workspace reads the
// same POLYKEY_DECODE_FILL; kv_heads=None sizes them for any).
PK_EXPORT int pk_set_decode_fill(int n) {
  if (n < 0 || n > 65536) return -1;
  g_decode_fill = n;
  return 0;
}

template <int P>
static int decode_launch_p(void* out, const void* q, const QkvIn& qi, const void* k_cache, const void* v_cache,
                           const void* block_tables, const void* context_lens, void* part_o, void* part_ml,
                           int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int q_stride,
                           int out_stride, float scale, int max_ctx, hipStream_t stream) {
  const int n_parts = (max_ctx + P - 1) / P;
  if (n_parts > 1 && (part_o == nullptr || part_ml == nullptr)) return -2;
  // z is capped: a short context leaves the extra z-workgroups idle, and graph capture fixes
  // the grid for max_model_len, so a z of n_parts would launch mostly-empty workgroups
  dim3 grid(n_kv, n_seqs, n_parts < g_decode_z ? n_parts : g_decode_z);
#define PK_DECODE_ARGS                                                                                            \
  static_cast<bf16_t*>(out), static_cast<const bf16_t*>(q), static_cast<bf16_t*>(const_cast<void*>(k_cache)),   \
      static_cast<bf16_t*>(const_cast<void*>(v_cache)), static_cast<const int*>(block_tables),                  \
      static_cast<const int*>(context_lens), static_cast<float*>(part_o), static_cast<float*>(part_ml),          \
      n_q, n_kv, bs, max_blocks, q_stride, out_stride, n_parts, scale * kLog2e, qi
  // (the K/V prefetch across the slab reduction for launches that leave most CUs idle, PRE,
  // measured slower: profiles/r5_attn_ab4.jsonl)
  if (qi.partial != nullptr) {
    switch (qi.S) {
      case 2: paged_decode_kernel<P, kDecodeWaves, true, 2><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      case 4: paged_decode_kernel<P, kDecodeWaves, true, 4><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      case 8: paged_decode_kernel<P, kDecodeWaves, true, 8><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      case 16: paged_decode_kernel<P, kDecodeWaves, true, 16><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      default: paged_decode_kernel<P, kDecodeWaves, true, 0><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
    }
  } else
    paged_decode_kernel<P, kDecodeWaves, false><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS);
#undef PK_DECODE_ARGS
  int rc = PK_CHECK_LAUNCH();
  if (rc || n_parts == 1) return rc;
  dim3 g2(n_q, n_seqs);
  paged_decode_reduce_kernel<P><<<g2, 128, 0, stream>>>(
      static_cast<bf16_t*>(out), static_cast<const float*>(part_o), static_cast<const float*>(part_ml),
      static_cast<const int*>(context_lens), n_q, out_stride, n_parts, static_cast<int>(grid.z));
  return PK_CHECK_LAUNCH();
}

// Sequences with more than one partition are merged by a second kernel (an in-launch merge by
// the last partition measured slower, profiles/r5_tp_ab.jsonl, and was removed in round 6).
static int decode_launch(void* out, const void* q, const QkvIn& qi, const void* k_cache, const void* v_cache,
                         const void* block_tables, const void* context_lens, void* part_o, void* part_ml,
                         int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int q_stride,
                         int out_stride, float scale, int max_ctx, hipStream_t stream) {
  if (n_seqs <= 0) return 0;
  if (n_q % n_kv || n_q / n_kv > 16 || bs % 32 || bs <= 0) return -1;  // K tiles: 32 keys
  // max_ctx bounds the contexts of this launch (<= 0: the block-table capacity).  A launch
  // known to stay within one partition needs no partition grid and no merge kernel.
  if (max_ctx <= 0 || max_ctx > max_blocks * bs) max_ctx = max_blocks * bs;
  if (decode_part(n_seqs, n_kv, max_ctx) == kDecodePartSmall)
    return decode_launch_p<kDecodePartSmall>(out, q, qi, k_cache, v_cache, block_tables, context_lens, part_o, part_ml,
                                             n_seqs, n_q, n_kv, bs, max_blocks, q_stride, out_stride, scale,
                                             max_ctx, stream);
  return decode_launch_p<kDecodePart>(out, q, qi, k_cache, v_cache, block_tables, context_lens, part_o, part_ml,
                                      n_seqs, n_q, n_kv, bs, max_blocks, q_stride, out_stride, scale, max_ctx,
                                      stream);
}

// max_blocks: block-table row stride; max_ctx: bound on every context of this launch (<= 0: no bound)
PK_EXPORT int pk_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache,
                              const void* block_tables, const void* context_lens, void* part_o, void* part_ml,
                              int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int q_stride,
                              int out_stride, float scale, int max_ctx, hipStream_t stream) {
  const QkvIn none{};
  return decode_launch(out, q, none, k_cache, v_cache, block_tables, context_lens, part_o, part_ml, n_seqs,
                       n_q, n_kv, bs, max_blocks, q_stride, out_stride, scale, max_ctx, stream);
}

// Decode attention straight from the fused QKV projection's split-K slabs [S, M, (n_q+2n_kv)*128]
// (RoPE + KV-cache write folded in); rows 0..n_seqs-1 of the slabs are the decode tokens.
PK_EXPORT int pk_paged_decode_qkv(void* out, const void* partial, int S, int M, const void* positions,
                                  const void* cos_sin, const void* slots, void* k_cache, void* v_cache,
                                  const void* block_tables, const void* context_lens, void* part_o, void* part_ml,
                                  int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int out_stride, float scale,
                                  int max_ctx, hipStream_t stream) {
  if (partial == nullptr || S < 1 || M < n_seqs) return -1;
  QkvIn qi{static_cast<const float*>(partial), static_cast<const int*>(positions), static_cast<const float*>(cos_sin),
           static_cast<const int*>(slots), S, M};
  return decode_launch(out, nullptr, qi, k_cache, v_cache, block_tables, context_lens, part_o, part_ml,
                       n_seqs, n_q, n_kv, bs, max_blocks, 0, out_stride, scale, max_ctx, stream);
}

int pk_get_decode_z() { return g_decode_z; }  // the fused QKV -> attention launch (decode_fused.hip)

PK_EXPORT int pk_set_decode_z(int z) {
  if (z < 1) return -1;
  g_decode_z = z;
  return 0;
}

PK_EXPORT int pk_paged_prefill(void* out, const void* q, const void* k_cache, const void* v_cache,
                               const void* block_tables, const void* context_lens, const void* cu_q, void* unused,
                               int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int q_stride, int out_stride,
                               int max_q_len, float scale, hipStream_t stream) {
  if (n_seqs <= 0 || max_q_len <= 0) return 0;
  if (n_q % n_kv || n_q / n_kv > 16 || bs % 32 || bs <= 0) return -1;  // K tiles: 32 keys
  const int G = n_q / n_kv;
  if (G == 1 || G == 2 || G == 4 || G == 8) {
    // 4-wave workgroups (two per CU: independent barriers let one workgroup's MFMAs overlap the
    // other's softmax) where the GQA group fits; G = 8 needs all 8 waves for one query group
    // (profiles/r2_prefill_attention.txt: 4 waves >= 8 waves at every measured shape)
    const int nw = G == 8 ? 8 : 4;
    const int pq = 32 * nw / G;  // queries per workgroup (nw waves: G heads x nw/G 32-query groups)
    const dim3 grid(n_kv, n_seqs, (max_q_len + pq - 1) / pq);
#define PK_PREFILL_M32(GG, NWW)                                                                                \
  paged_prefill_mfma32_kernel<GG, NWW><<<grid, 64 * NWW, 0, stream>>>(                                         \
      static_cast<bf16_t*>(out), static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k_cache),          \
      static_cast<const bf16_t*>(v_cache), static_cast<const int*>(block_tables),                              \
      static_cast<const int*>(context_lens), static_cast<const int*>(cu_q), n_kv, bs, max_blocks, q_stride,    \
      out_stride, scale * kLog2e)
    switch (G * 16 + nw) {
      case 1 * 16 + 4: PK_PREFILL_M32(1, 4); break;
      case 2 * 16 + 4: PK_PREFILL_M32(2, 4); break;
      case 4 * 16 + 4: PK_PREFILL_M32(4, 4); break;
      default: PK_PREFILL_M32(8, 8); break;
    }
#undef PK_PREFILL_M32
    return PK_CHECK_LAUNCH();
  }
  // other GQA groups (3, 5, 6, 16, ...): one wave per query head, 16 queries per workgroup
  const int W = G > 8 ? 8 : G;
  if (G % W) return -1;
  dim3 grid((max_q_len + 15) / 16, n_seqs, n_kv * (G / W));
  paged_prefill_kernel<<<grid, 64 * W, 0, stream>>>(
      static_cast<bf16_t*>(out), static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k_cache),
      static_cast<const bf16_t*>(v_cache), static_cast<const int*>(block_tables), static_cast<const int*>(context_lens),
      static_cast<const int*>(cu_q), n_q, n_kv, bs, max_blocks, q_stride, out_stride, scale * kLog2e);
  return PK_CHECK_LAUNCH();
}
