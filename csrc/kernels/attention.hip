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
#include "common.h"

using namespace pk;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
constexpr int kHD = 128;
constexpr int kStep = 32;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1e30f;
constexpr int kDecodeWaves = 4;  // waves per (seq, kv head, partition); 8 measured ~10 % slower at 384 keys
int g_decode_z = 4;  // max partition workgroups per (seq, kv head) (pk_set_decode_z)

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }
// K/V stream loads: plain (non-temporal measured slower: in-situ decode step 4.43 vs 4.45 ms,
// tools/ab_decode.py)
__device__ __forceinline__ bf16x8_t ldkv(const bf16_t* p) { return ld8(p); }

__device__ __forceinline__ bf16x8_t zero8() {
  u32x4 z = {0u, 0u, 0u, 0u};
  return __builtin_bit_cast(bf16x8_t, z);
}

__device__ __forceinline__ bf16x8_t pack_p(const float* p) {
  u32x4 v;
  v[0] = pack2(p[0], p[1]);
  v[1] = pack2(p[2], p[3]);
  v[2] = pack2(p[4], p[5]);
  v[3] = pack2(p[6], p[7]);
  return __builtin_bit_cast(bf16x8_t, v);
}

// Reductions over the 4 lane groups of a column (lanes r, r+16, r+32, r+48) with the gfx950
// VALU lane swaps (v_permlane16/32_swap: rows 1<->0 / 3<->2, then halves) instead of
// ds_bpermute round trips through the LDS crossbar (__shfl_xor): max(x, swapped x) and
// x + swapped x are already the pairwise results in every lane (prefill attention 1-4 % faster,
// profiles/r2_prefill_attention.txt).
__device__ __forceinline__ float col_max(float x) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// Total exp-sum of the lane's column (reduce the 4 lane groups).
__device__ __forceinline__ float col_sum(float l) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(l), __float_as_uint(l), false, false);
  l = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

struct WaveState {
  float m;        // running max (base-2 scaled) of this lane's column
  float l;        // partial exp-sum of this lane's 8 keys per step (summed over lane groups at the end)
  f32x4 o[8];     // O^T: o[dt][i] = O[col = lane&15][d = 16*dt + 4*g + i]
};

// K/V fragments of one 32-key step (16 B per lane each): K as the A operand of S^T = K Q^T
// (2 key tiles x 4 head-dim k-steps), V^T as the A operand of O^T += V^T P^T (8 d-tiles).
struct KVFrag {
  bf16x8_t k[2][4];
  bf16x8_t v[8];
};

// bt[i - bt_base] = physical block of logical block i; `lim` bounds the tokens a load may touch
// (past it the address is clamped, the data never used), so the block lookups stay inside the
// caller's block-table window.  K comes from the fragment-native cache tile of step s (common.h
// kcache_off: one contiguous KiB per load instruction); V likewise (common.h vcache_off): lane
// (r, g) reads keys 8g..8g+7 of channel 16 dt + r, one contiguous KiB per d-tile (ldkv: plain loads).
__device__ __forceinline__ void load_kv(KVFrag& f, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                        int64_t blk_stride, const int* __restrict__ bt, int bt_base, int bs, int s,
                                        int lim) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int ks = min(s, lim - 1) & ~31;  // the step's 32-key tile (clamped past the end)
  const bf16_t* kt = kc + bt[ks / bs - bt_base] * blk_stride + (ks % bs) * kHD + 8 * lane;
  PK_DEVICE_ASSERT(bt[ks / bs - bt_base] >= 0);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) f.k[t][kk] = ldkv(kt + (t * 4 + kk) * 512);
  int tok0 = s + 8 * g;
  tok0 = min(tok0, ((lim - 1) >> 3) << 3);
  const int blk = bt[tok0 / bs - bt_base];
  const bf16_t* p = vc + blk * blk_stride + vcache_off(tok0 % bs, r);  // + 512 per 16-channel tile
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) f.v[dt] = ldkv(p + dt * 512);
}

__device__ __forceinline__ void attend_step(WaveState& st, const bf16x8_t (&qf)[4], const KVFrag& f, int s,
                                            int n_valid, int col_limit, float scale2) {
  const int g = (threadIdx.x & 63) >> 4;
  // ---- S^T = K . Q^T
  f32x4 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.k[t][kk], qf[kk], acc[t], 0, 0, 0);
  }
  // ---- online softmax over this step's 32 keys (8 per lane)
  float sv[8];
  float mx = kNegBig;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = s + 8 * g + 4 * t + i;
      const bool ok = key < n_valid && key <= col_limit;
      const float v = ok ? acc[t][i] * scale2 : -INFINITY;
      sv[4 * t + i] = v;
      mx = fmaxf(mx, v);
    }
  mx = col_max(mx);
  const float m_new = fmaxf(st.m, mx);
  const float alpha = exp2f(st.m - m_new);
  st.m = m_new;
  float p[8];
  float psum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    p[i] = exp2f(sv[i] - m_new);
    psum += p[i];
  }
  st.l = st.l * alpha + psum;
  const bf16x8_t pb = pack_p(p);
  // ---- O^T += V^T . P^T
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    st.o[dt] *= alpha;
    st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.v[dt], pb, st.o[dt], 0, 0, 0);
  }
}

// Process keys [k_begin, k_end) in 32-key steps (k_begin multiple of 32), stride `k_stride`
// between this wave's steps.  Keys >= n_valid or > col_limit are masked.  Software-pipelined
// over two fragment sets: the next step's K/V loads are in flight while this step computes
// (loads past the end are clamped to valid addresses and never consumed).
__device__ __forceinline__ void attend(WaveState& st, const bf16x8_t (&qf)[4], const bf16_t* __restrict__ kc,
                                       const bf16_t* __restrict__ vc, int64_t blk_stride, const int* __restrict__ bt,
                                       int bt_base, int bs, int k_begin, int k_end, int k_stride, int n_valid,
                                       int col_limit, float scale2, KVFrag& fa, bool fa_loaded = false) {
  if (k_begin >= k_end) return;
  const int lim = min(n_valid, k_end);
  KVFrag fb;
  if (!fa_loaded) load_kv(fa, kc, vc, blk_stride, bt, bt_base, bs, k_begin, lim);
  for (int s = k_begin; s < k_end; s += 2 * k_stride) {
    load_kv(fb, kc, vc, blk_stride, bt, bt_base, bs, s + k_stride, lim);
    attend_step(st, qf, fa, s, n_valid, col_limit, scale2);
    if (s + k_stride >= k_end) break;
    load_kv(fa, kc, vc, blk_stride, bt, bt_base, bs, s + 2 * k_stride, lim);
    attend_step(st, qf, fb, s + k_stride, n_valid, col_limit, scale2);
  }
}

__device__ __forceinline__ void init_state(WaveState& st) {
  st.m = kNegBig;
  st.l = 0.f;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) st.o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void load_q(bf16x8_t (&qf)[4], const bf16_t* q, bool valid) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) qf[kk] = valid ? ld8(q + 32 * g + 8 * kk) : zero8();
}



// ------------------------------------------------------------------------------ decode
// grid (n_kv, n_seqs, min(n_parts, z)), block 64*NW (NW waves).  LDS: NW waves x 16 cols x 128 d fp32.
// Decode attention fed straight from the QKV projection's split-K slabs (FROM_QKV): the
// workgroup of (seq, kv head h) sums the S fp32 slabs of its G query heads and of k/v head h,
// rounds to bf16 (the unfused GEMM output), applies RoPE, keeps q in LDS, and — the workgroup
// that owns the partition holding the new token — writes k / v into the paged cache before
// attending.  Replaces the separate QKV-reduce + RoPE + cache-write kernel of a decode layer.
struct QkvIn {
  const float* partial;    // [S, M, (n_q + 2 n_kv) * 128]
  const int* positions;    // [M]
  const float* cos_sin;    // [max_pos, 128] = cos[64] | sin[64]
  const int* slots;        // [M], < 0: nothing cached
  int S, M;
};

template <int kPart, int NW, bool FROM_QKV, int SS = 0>
__global__ void __launch_bounds__(64 * NW) paged_decode_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    float* __restrict__ part_o, float* __restrict__ part_ml, int* __restrict__ counters, int n_q, int n_kv, int bs,
    int max_blocks, int q_stride, int out_stride, int n_parts, float scale2, const QkvIn qi) {
  __shared__ float o_lds[NW][16][kHD + 4];
  __shared__ float ml_lds[NW][16][2];
  __shared__ int last;
  __shared__ int bt_s[kPart / 8 + 2];  // this partition's block-table window (LDS: lookups use lgkmcnt)
  // FROM_QKV, new token folded in (see below): its rotated k, its v and its G scores
  __shared__ __attribute__((aligned(16))) bf16_t kn_s[kHD];
  __shared__ float vn_s[kHD];
  __shared__ float sn_s[16];
  static_assert(64 * NW >= 256, "the new-token scores use 16 lanes per query head, G <= 16");
  const int h = blockIdx.x, seq = blockIdx.y;
  // the first partition's block-table window, requested before anything else so its round
  // trip overlaps the context / q preparation instead of following it (entries past the
  // sequence's blocks are in-bounds of the row and never used)
  const int pre_b0 = static_cast<int>(blockIdx.z) * (kPart / bs);
  int bt_pre = 0;
  if (static_cast<int>(threadIdx.x) <= kPart / bs && pre_b0 + static_cast<int>(threadIdx.x) < max_blocks)
    bt_pre = block_tables[static_cast<int64_t>(seq) * max_blocks + pre_b0 + threadIdx.x];
  const int ctx = context_lens[seq];
  const int G = n_q / n_kv;
  if (ctx <= 0) {
    if (blockIdx.z == 0)  // a padded (graph) row -> zeros
      for (int idx = threadIdx.x; idx < G * kHD; idx += 64 * NW)
        out[static_cast<int64_t>(seq) * out_stride + (h * G + idx / kHD) * kHD + idx % kHD] = 0;
    return;
  }
  // n_parts comes from the launch's context bound; the clamp keeps a violated bound in-bounds
  const int n_used = min((ctx + kPart - 1) / kPart, n_parts);
  PK_DEVICE_ASSERT(ctx <= n_parts * kPart);
  if (static_cast<int>(blockIdx.z) >= n_used) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t blk_stride = static_cast<int64_t>(n_kv) * bs * kHD;
  const bf16_t* kch = kc + static_cast<int64_t>(h) * bs * kHD;
  const bf16_t* vch = vc + static_cast<int64_t>(h) * kHD * bs;
  // (prefetching the first K/V step across the q preparation below was measured: it pushes
  // the kernel to 256 VGPRs + AGPRs, one wave per SIMD, and is slower overall)
  bf16x8_t qf[4];
  // fold: the workgroup holding the new token (key ctx - 1) keeps its k / v in LDS, attends to
  // keys [0, ctx - 1) from the cache and adds key ctx - 1 from LDS in the final combine; the
  // cache write goes out at the end of the kernel.  Writing the row first and reading it back
  // through the cache cost 4-5 us per launch at 384-512 keys (the scattered 2-byte V^T stores
  // and the K tile stores land on lines the waves are about to stream).
  bool fold = false;
  int slot = -1;
  if constexpr (FROM_QKV) {
    __shared__ __attribute__((aligned(16))) bf16_t q_s[16][kHD];
    const int N = (n_q + 2 * n_kv) * kHD;
    const int64_t slab = static_cast<int64_t>(qi.M) * N;
    const float* base = qi.partial + static_cast<int64_t>(seq) * N;
    const float* cs = qi.cos_sin + static_cast<int64_t>(qi.positions[seq]) * kHD;
    slot = qi.slots[seq];
    const bool writer = slot >= 0 && static_cast<int>(blockIdx.z) == (n_used - 1) % static_cast<int>(gridDim.z);
    fold = writer && qi.positions[seq] == ctx - 1;
    const int n_items = G * 64 + (writer ? 128 : 0);
    for (int it = threadIdx.x; it < n_items; it += 64 * NW) {
      int col, j;
      if (it < G * 64) {
        j = it & 63;
        col = (h * G + (it >> 6)) * kHD + j;
      } else if (it < G * 64 + 64) {
        j = it - G * 64;
        col = (n_q + h) * kHD + j;
      } else {
        j = it - G * 64 - 64;
        col = (n_q + n_kv + h) * kHD + j;
      }
      float a = 0.f, b = 0.f;
      if constexpr (SS > 0) {  // all slab loads in flight before the first add
        float va[SS], vb[SS];
#pragma unroll
        for (int sp = 0; sp < SS; ++sp) {
          va[sp] = base[sp * slab + col];
          vb[sp] = base[sp * slab + col + 64];
        }
#pragma unroll
        for (int sp = 0; sp < SS; ++sp) {
          a += va[sp];
          b += vb[sp];
        }
      } else {
        for (int sp = 0; sp < qi.S; ++sp) {
          a += base[sp * slab + col];
          b += base[sp * slab + col + 64];
        }
      }
      if (it < G * 64 + 64) {  // q or k: round (the GEMM output), rotate (neox)
        a = bf2f(f2bf(a));
        b = bf2f(f2bf(b));
        const float co = cs[j], si = cs[64 + j];
        const bf16_t ra = f2bf(a * co - b * si), rb = f2bf(b * co + a * si);
        if (it < G * 64) {
          q_s[it >> 6][j] = ra;
          q_s[it >> 6][j + 64] = rb;
        } else if (fold) {
          kn_s[j] = ra;
          kn_s[j + 64] = rb;
        } else {
          bf16_t* d = kc + (static_cast<int64_t>(slot / bs) * n_kv + h) * bs * kHD;
          d[kcache_off(slot % bs, j)] = ra;
          d[kcache_off(slot % bs, j + 64)] = rb;
        }
      } else if (fold) {
        vn_s[j] = bf2f(f2bf(a));
        vn_s[j + 64] = bf2f(f2bf(b));
      } else {
        bf16_t* d = vc + (static_cast<int64_t>(slot / bs) * n_kv + h) * kHD * bs;
        d[vcache_off(slot % bs, j)] = f2bf(a);
        d[vcache_off(slot % bs, j + 64)] = f2bf(b);
      }
    }
    if (!fold) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the new k/v rows are in L2 before any wave reads them
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      qf[kk] = r < G ? *reinterpret_cast<const bf16x8_t*>(&q_s[r][32 * g + 8 * kk]) : zero8();
    if (fold) {  // scores of the new key, 16 lanes per query head (read after the combine's barrier)
      const int c = threadIdx.x >> 4, part = threadIdx.x & 15;
      float sdot = 0.f;
      if (c < G)
#pragma unroll
        for (int e = 0; e < 8; ++e) sdot += bf2f(q_s[c][8 * part + e]) * bf2f(kn_s[8 * part + e]);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) sdot += __shfl_xor(sdot, o, 64);
      if (c < G && part == 0) sn_s[c] = sdot * scale2;
    }
  } else {
    load_q(qf, q + static_cast<int64_t>(seq) * q_stride + (h * G + r) * kHD, r < G);
  }

  // the grid's z dimension is small (<= 4); a workgroup walks partitions z, z + gridDim.z, ...
  // carrying its online-softmax state across them (the order of key blocks does not matter to
  // the softmax), so it combines its waves and writes ONE partial at the end: no LDS combine /
  // partial store between partitions and gridDim.z partials to merge instead of n_parts.
  const int n_eff = min(n_used, static_cast<int>(gridDim.z));  // partials of this sequence
  const int ctx_c = fold ? ctx - 1 : ctx;  // keys read from the cache
  WaveState st;
  init_state(st);
  for (int part = blockIdx.z; part < n_used; part += gridDim.z) {
    const int begin = part * kPart;
    const int end = min(ctx_c, begin + kPart);
    const int b0 = begin / bs, nblk = (end - 1) / bs - b0 + 1;
    __syncthreads();  // the previous partition's block-table readers are done
    if (part == static_cast<int>(blockIdx.z) && kPart % bs == 0) {  // nblk <= kPart / bs <= 64 * NW
      if (static_cast<int>(threadIdx.x) < nblk) bt_s[threadIdx.x] = bt_pre;
    } else
      for (int i = threadIdx.x; i < nblk; i += 64 * NW)
        bt_s[i] = block_tables[static_cast<int64_t>(seq) * max_blocks + b0 + i];
    __syncthreads();
    KVFrag fa;
    if (end > begin)
      attend(st, qf, kch, vch, blk_stride, bt_s, b0, bs, begin + kStep * w, end, NW * kStep, ctx_c, ctx_c - 1, scale2,
             fa);
  }
  const float lsum = col_sum(st.l);
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) o_lds[w][r][16 * dt + 4 * g + i] = st.o[dt][i];
  if (g == 0) {
    ml_lds[w][r][0] = st.m;
    ml_lds[w][r][1] = lsum;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < G * kHD; idx += 64 * NW) {
    const int c = idx / kHD, d = idx % kHD;
    float M = kNegBig;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, ml_lds[ww][c][0]);
    const float sn = fold ? sn_s[c] : kNegBig;
    M = fmaxf(M, sn);
    float O = 0.f, L = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float f = exp2f(ml_lds[ww][c][0] - M);
      O += f * o_lds[ww][c][d];
      L += f * ml_lds[ww][c][1];
    }
    if (fold) {  // key ctx - 1: P rounded to bf16 for the PV product as in attend_step
      const float f = exp2f(sn - M);
      O += bf2f(f2bf(f)) * vn_s[d];
      L += f;
    }
    const int hq = h * G + c;
    if (n_eff == 1) {
      out[static_cast<int64_t>(seq) * out_stride + hq * kHD + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const int64_t pi = (static_cast<int64_t>(seq) * n_q + hq) * n_parts + blockIdx.z;
      part_o[pi * kHD + d] = O;
      if (d == 0) {
        part_ml[2 * pi] = M;
        part_ml[2 * pi + 1] = L;
      }
    }
  }
  if (fold) {  // the new token's row into the paged cache, off the attention's critical path
    const int t = threadIdx.x;
    if (t < kHD) {
      bf16_t* d = kc + (static_cast<int64_t>(slot / bs) * n_kv + h) * bs * kHD;
      d[kcache_off(slot % bs, t)] = kn_s[t];
    } else if (t < 2 * kHD) {
      bf16_t* d = vc + (static_cast<int64_t>(slot / bs) * n_kv + h) * kHD * bs;
      d[vcache_off(slot % bs, t - kHD)] = f2bf(vn_s[t - kHD]);
    }
  }
  if (n_eff == 1 || counters == nullptr) return;
  // ---- in-launch split-K merge: the last workgroup to arrive combines the partials
  // (guide §5 "In-launch split-K reduction": plain slab stores, every wave drains, one agent
  // release + ticket; the last arriver acquires, merges and re-arms the counter).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* ctr = counters + seq * n_kv + h;
    const int t = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == n_eff - 1);
    if (last) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  for (int idx = threadIdx.x; idx < G * kHD; idx += 64 * NW) {
    const int c = idx / kHD, d = idx % kHD;
    const int hq = h * G + c;
    const int64_t base = (static_cast<int64_t>(seq) * n_q + hq) * n_parts;
    float M = kNegBig;
    for (int p = 0; p < n_eff; ++p) M = fmaxf(M, part_ml[2 * (base + p)]);
    float O = 0.f, L = 0.f;
    for (int p = 0; p < n_eff; ++p) {
      const float f = exp2f(part_ml[2 * (base + p)] - M);
      O += f * part_o[(base + p) * kHD + d];
      L += f * part_ml[2 * (base + p) + 1];
    }
    out[static_cast<int64_t>(seq) * out_stride + hq * kHD + d] = f2bf(L > 0.f ? O / L : 0.f);
  }
}

// grid (n_q, n_seqs), block 128: merge the partitions of sequences that used more than one.
template <int kPart>
__global__ void __launch_bounds__(128) paged_decode_reduce_kernel(bf16_t* __restrict__ out,
                                                                  const float* __restrict__ part_o,
                                                                  const float* __restrict__ part_ml,
                                                                  const int* __restrict__ context_lens, int n_q,
                                                                  int out_stride, int n_parts, int z) {
  const int hq = blockIdx.x, seq = blockIdx.y, d = threadIdx.x;
  const int ctx = context_lens[seq];
  const int n_used = min((ctx + kPart - 1) / kPart, z);  // one partial per partition workgroup
  bf16_t* o = out + static_cast<int64_t>(seq) * out_stride + hq * kHD;
  if (ctx <= 0) {
    o[d] = 0;
    return;
  }
  if (n_used <= 1) return;
  const int64_t base = (static_cast<int64_t>(seq) * n_q + hq) * n_parts;
  float M = kNegBig;
  for (int p = 0; p < n_used; ++p) M = fmaxf(M, part_ml[2 * (base + p)]);
  float O = 0.f, L = 0.f;
  for (int p = 0; p < n_used; ++p) {
    const float f = exp2f(part_ml[2 * (base + p)] - M);
    O += f * part_o[(base + p) * kHD + d];
    L += f * part_ml[2 * (base + p) + 1];
  }
  o[d] = f2bf(L > 0.f ? O / L : 0.f);
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
  KVFrag fa;
  attend(st, qf, kc + static_cast<int64_t>(h) * bs * kHD, vc + static_cast<int64_t>(h) * kHD * bs,
         static_cast<int64_t>(n_kv) * bs * kHD, block_tables + static_cast<int64_t>(seq) * max_blocks, 0, bs, 0,
         k_end, kStep, ctx, valid ? qpos : -1, scale2, fa);
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

// Workspace for decode: part_o [n_seqs, n_q, n_parts, 128] fp32, part_ml [n_seqs, n_q, n_parts, 2] fp32.
PK_EXPORT int pk_decode_num_parts(int max_context) { return (max_context + kDecodePart - 1) / kDecodePart; }

// counters: [n_seqs, n_kv] int32, zero-initialised once (the merging workgroup re-arms its
// counter); with counters == null the partitions are merged by a second kernel instead.
static int decode_launch(void* out, const void* q, const QkvIn& qi, const void* k_cache, const void* v_cache,
                         const void* block_tables, const void* context_lens, void* part_o, void* part_ml,
                         void* counters, int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int q_stride,
                         int out_stride, float scale, int max_ctx, hipStream_t stream) {
  if (n_seqs <= 0) return 0;
  if (n_q % n_kv || n_q / n_kv > 16 || bs % 32 || bs <= 0) return -1;  // K tiles: 32 keys
  // max_ctx bounds the contexts of this launch (<= 0: the block-table capacity).  A launch
  // known to stay within one partition needs no partition grid and no merge kernel.
  if (max_ctx <= 0 || max_ctx > max_blocks * bs) max_ctx = max_blocks * bs;
  const int n_parts = (max_ctx + kDecodePart - 1) / kDecodePart;
  if (n_parts > 1 && (part_o == nullptr || part_ml == nullptr)) return -2;
  // z is capped: a short context leaves the extra z-workgroups idle, and graph capture fixes
  // the grid for max_model_len, so a z of n_parts would launch mostly-empty workgroups
  dim3 grid(n_kv, n_seqs, n_parts < g_decode_z ? n_parts : g_decode_z);
#define PK_DECODE_ARGS                                                                                            \
  static_cast<bf16_t*>(out), static_cast<const bf16_t*>(q), static_cast<bf16_t*>(const_cast<void*>(k_cache)),   \
      static_cast<bf16_t*>(const_cast<void*>(v_cache)), static_cast<const int*>(block_tables),                  \
      static_cast<const int*>(context_lens), static_cast<float*>(part_o), static_cast<float*>(part_ml),          \
      static_cast<int*>(counters), n_q, n_kv, bs, max_blocks, q_stride, out_stride, n_parts, scale * kLog2e, qi
  if (qi.partial != nullptr) {
    switch (qi.S) {
      case 2: paged_decode_kernel<kDecodePart, kDecodeWaves, true, 2><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      case 4: paged_decode_kernel<kDecodePart, kDecodeWaves, true, 4><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      case 8: paged_decode_kernel<kDecodePart, kDecodeWaves, true, 8><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
      default: paged_decode_kernel<kDecodePart, kDecodeWaves, true, 0><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS); break;
    }
  } else
    paged_decode_kernel<kDecodePart, kDecodeWaves, false><<<grid, 64 * kDecodeWaves, 0, stream>>>(PK_DECODE_ARGS);
#undef PK_DECODE_ARGS
  int rc = PK_CHECK_LAUNCH();
  if (rc || counters != nullptr || n_parts == 1) return rc;
  dim3 g2(n_q, n_seqs);
  paged_decode_reduce_kernel<kDecodePart><<<g2, 128, 0, stream>>>(
      static_cast<bf16_t*>(out), static_cast<const float*>(part_o), static_cast<const float*>(part_ml),
      static_cast<const int*>(context_lens), n_q, out_stride, n_parts, static_cast<int>(grid.z));
  return PK_CHECK_LAUNCH();
}

// max_blocks: block-table row stride; max_ctx: bound on every context of this launch (<= 0: no bound)
PK_EXPORT int pk_paged_decode(void* out, const void* q, const void* k_cache, const void* v_cache,
                              const void* block_tables, const void* context_lens, void* part_o, void* part_ml,
                              void* counters, int n_seqs, int n_q, int n_kv, int bs, int max_blocks, int q_stride,
                              int out_stride, float scale, int max_ctx, hipStream_t stream) {
  const QkvIn none{};
  return decode_launch(out, q, none, k_cache, v_cache, block_tables, context_lens, part_o, part_ml, counters, n_seqs,
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
  return decode_launch(out, nullptr, qi, k_cache, v_cache, block_tables, context_lens, part_o, part_ml, nullptr,
                       n_seqs, n_q, n_kv, bs, max_blocks, 0, out_stride, scale, max_ctx, stream);
}

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
