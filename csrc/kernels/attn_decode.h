// Paged decode attention workgroup body (decode_tile), shared by the decode kernels
// (attention.hip) and the fused QKV -> attention launch (decode_fused.hip).
#pragma once
#include "common.h"
#include "flow.h"

using namespace pk;

namespace {

constexpr int kHD = 128;
constexpr int kStep = 32;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1e30f;
constexpr int kDecodeWaves = 4;  // waves per (seq, kv head, partition); 8 measured ~10 % slower at 384 keys
constexpr int kDecodePartSmall = 128;  // keys per partition when (seq, kv head) pairs cannot fill the chip
// ... i.e. fewer workgroups than this at the full partition (pk_set_decode_fill).  64: the 70B TP=8
// rank's 64 sequences x 1 kv head stay at 512 keys (one workgroup per sequence, no merge launch):
// per-rank step 6.52 vs 6.54 ms at 256 (128-key partitions + merge), profiles/r5_attn_ab4.jsonl
int g_decode_fill = 64;
int g_decode_z = 4;  // max partition workgroups per (seq, kv head) (pk_set_decode_z)
// (8-wave workgroups for small launches, pk_set_decode_wide: within noise at the 70B TP=8 shard,
// profiles/r5_wide_attn.jsonl -- removed in round 6)

// K/V stream loads: plain (non-temporal measured slower: in-situ decode step 4.43 vs 4.45 ms,
// tools/ab_decode.py)
__device__ __forceinline__ bf16x8_t ldkv(const bf16_t* p) { return ld8(p); }

// 16-byte load of QKV slab floats p..p+3; SC1: handed over in-launch (sc1 buffer load, base < 2 GiB)
template <bool SC1>
__device__ __forceinline__ float4 ld_slab4(const float* base, const float* p) {
  if constexpr (SC1)
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), static_cast<short>(0), 0x7ffffff0, 0x00020000),
        static_cast<int>((p - base) * 4), 0, 16));
  return *reinterpret_cast<const float4*>(p);
}

// uniform int through the vector memory path (raw buffer load), see decode_tile's prologue
__device__ __forceinline__ int ld_vmem(const int* p) {
  return __builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p), static_cast<short>(0), 0x7ffffff0, 0x00020000), 0, 0, 0);
}

__device__ __forceinline__ void add4f(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}

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
// PRE = 1 / 2: the caller already loaded the first step / two steps (fa: k_begin, fb: k_begin +
// k_stride, with the same clamp `lim`), e.g. while it waited for an in-launch hand-off.
template <int PRE = 0>
__device__ __forceinline__ void attend(WaveState& st, const bf16x8_t (&qf)[4], const bf16_t* __restrict__ kc,
                                       const bf16_t* __restrict__ vc, int64_t blk_stride, const int* __restrict__ bt,
                                       int bt_base, int bs, int k_begin, int k_end, int k_stride, int n_valid,
                                       int col_limit, float scale2, KVFrag& fa, KVFrag& fb) {
  if (k_begin >= k_end) return;
  const int lim = min(n_valid, k_end);
  int s = k_begin;
  if constexpr (PRE == 2) {  // first iteration peeled: its fb is already in flight
    attend_step(st, qf, fa, s, n_valid, col_limit, scale2);
    if (s + k_stride >= k_end) return;
    load_kv(fa, kc, vc, blk_stride, bt, bt_base, bs, s + 2 * k_stride, lim);
    attend_step(st, qf, fb, s + k_stride, n_valid, col_limit, scale2);
    s += 2 * k_stride;
  } else if constexpr (PRE == 0) {
    load_kv(fa, kc, vc, blk_stride, bt, bt_base, bs, k_begin, lim);
  }
  for (; s < k_end; s += 2 * k_stride) {
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

// LDS of one decode-attention workgroup (passed in: a fused launch shares it with its GEMM tiles)
template <int kPart, int NW>
struct DecodeLds {
  float o_lds[NW][16][kHD + 4];
  float ml_lds[NW][16][2];
  int bt_s[kPart / 8 + 2];  // this partition's block-table window (LDS: lookups use lgkmcnt)
  // FROM_QKV, new token folded in (see below): its rotated k, its v and its G scores
  bf16_t kn_s[kHD] __attribute__((aligned(16)));
  float vn_s[kHD];
  float sn_s[16];
  bf16_t q_s[16][kHD] __attribute__((aligned(16)));
};

// One decode-attention workgroup (seq = by, kv head = bx, partition = bz of gdz).  FL & 2: the
// QKV slabs are handed over in-launch (decode_fused.hip): wait on kv head bx's tickets in fin
// before reading them, and read them with sc1 loads.
// PRE = 1 / 2 (fused launch): the first partition's first one / two K/V steps per wave are
// requested before the hand-off wait, so they stream in while the QKV tiles finish.
template <int kPart, int NW, bool FROM_QKV, int SS = 0, int FL = 0, int PRE = 0>
__device__ __forceinline__ void decode_tile(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    float* __restrict__ part_o, float* __restrict__ part_ml, int n_q, int n_kv, int bs,
    int max_blocks, int q_stride, int out_stride, int n_parts, float scale2, const QkvIn qi, const int bx,
    const int by, const int bz, const int gdz, DecodeLds<kPart, NW>& L, const Flow& fin) {
  auto& o_lds = L.o_lds;
  auto& ml_lds = L.ml_lds;
  auto& bt_s = L.bt_s;
  auto& kn_s = L.kn_s;
  auto& vn_s = L.vn_s;
  auto& sn_s = L.sn_s;
  static_assert(64 * NW >= 256, "the new-token scores use 16 lanes per query head, G <= 16");
  const int h = bx, seq = by;
  // QKV slab item `it` (FROM_QKV): 4 consecutive columns j..j+3 of a head and their rotation
  // partners j+64..j+67 (16-byte slab loads); the G q heads + k + v of kv head h are 16 (G + 2) items
  auto item_col = [&](int it, int& j) {
    const int Gq = n_q / n_kv;
    if (it < Gq * 16) {
      j = (it & 15) * 4;
      return (h * Gq + (it >> 4)) * kHD + j;
    }
    if (it < Gq * 16 + 16) {
      j = (it - Gq * 16) * 4;
      return (n_q + h) * kHD + j;
    }
    j = (it - Gq * 16 - 16) * 4;
    return (n_q + n_kv + h) * kHD + j;
  };
  // Prologue loads in ONE round trip: the context / position / slot (vector loads: scalar ones
  // were waited for with lgkmcnt(0) together with the kernel-argument loads the slab addresses
  // need), the first partition's block-table window, and -- slabs complete at launch, i.e. not a
  // fused launch's in-launch hand-off -- this thread's first QKV slab item, ahead of the writer /
  // fold decision (which only selects what is stored; the first pass of the q loop consumes it).
  int ctx = ld_vmem(context_lens + seq);
  int pos_q = FROM_QKV ? ld_vmem(qi.positions + seq) : 0;
  int slot_q = FROM_QKV ? ld_vmem(qi.slots + seq) : -1;
  // (entries of the block-table window past the sequence's blocks are in-bounds of the row and
  // never used)
  const int pre_b0 = static_cast<int>(bz) * (kPart / bs);
  int bt_pre = 0;
  if (static_cast<int>(threadIdx.x) <= kPart / bs && pre_b0 + static_cast<int>(threadIdx.x) < max_blocks)
    bt_pre = block_tables[static_cast<int64_t>(seq) * max_blocks + pre_b0 + threadIdx.x];
  constexpr bool kHoist = FROM_QKV && SS > 0 && (FL & 2) == 0;
  float4 hva[kHoist ? SS : 1], hvb[kHoist ? SS : 1];
  if constexpr (kHoist) {
    const int N = (n_q + 2 * n_kv) * kHD;
    const int64_t slab = static_cast<int64_t>(qi.M) * N;
    const float* base = qi.partial + static_cast<int64_t>(seq) * N;
    int j;
    const int col = item_col(min(static_cast<int>(threadIdx.x), (n_q / n_kv) * 16 + 31), j);
#pragma unroll
    for (int sp = 0; sp < SS; ++sp) {
      hva[sp] = *reinterpret_cast<const float4*>(base + sp * slab + col);
      hvb[sp] = *reinterpret_cast<const float4*>(base + sp * slab + col + 64);
    }
  }
  // the three scalars are needed from here on: their wait (issued first) leaves the slab loads in
  // flight, and the memory clobber keeps the slab loads above it
  asm volatile("" : "+v"(ctx), "+v"(pos_q), "+v"(slot_q) :: "memory");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t blk_stride = static_cast<int64_t>(n_kv) * bs * kHD;
  const bf16_t* kch = kc + static_cast<int64_t>(h) * bs * kHD;
  const bf16_t* vch = vc + static_cast<int64_t>(h) * kHD * bs;
  KVFrag fa, fb;
  bool prefetched = false;
  if constexpr (PRE > 0) {
    static_assert(FROM_QKV && kPart % 32 == 0, "prefetch: fused launches, whole 32-key blocks");
    // the same partition range / fold decision as below (positions and slots are launch inputs,
    // not produced by the QKV tiles)
    const int n_used0 = min((ctx + kPart - 1) / kPart, n_parts);
    if (ctx > 0 && static_cast<int>(bz) < n_used0) {
      const bool writer0 = slot_q >= 0 && static_cast<int>(bz) == (n_used0 - 1) % static_cast<int>(gdz);
      const bool fold0 = writer0 && pos_q == ctx - 1;
      const int ctx_c0 = fold0 ? ctx - 1 : ctx;
      const int begin = bz * kPart, end = min(ctx_c0, begin + kPart);
      // (a writer that does not fold stores the new row into the cache before attending: no prefetch)
      prefetched = kPart % bs == 0 && end > begin && (fold0 || !writer0);
      if (prefetched && static_cast<int>(threadIdx.x) < (end - 1) / bs - begin / bs + 1) bt_s[threadIdx.x] = bt_pre;
      __syncthreads();  // uniform: ctx, bz and the fold decision are per workgroup
      if (prefetched) {
        const int lim = min(ctx_c0, end), k0 = begin + kStep * w;
        load_kv(fa, kch, vch, blk_stride, bt_s, begin / bs, bs, k0, lim);
        if constexpr (PRE == 2) load_kv(fb, kch, vch, blk_stride, bt_s, begin / bs, bs, k0 + NW * kStep, lim);
      }
    }
  }
  if constexpr ((FL & 2) != 0) flow_wait(fin, h);  // this kv head's QKV tiles (every workgroup: re-arm count)
  const int G = n_q / n_kv;
  if (ctx <= 0) {
    if (bz == 0)  // a padded (graph) row -> zeros
      for (int idx = threadIdx.x; idx < G * kHD; idx += 64 * NW)
        out[static_cast<int64_t>(seq) * out_stride + (h * G + idx / kHD) * kHD + idx % kHD] = 0;
    return;
  }
  // n_parts comes from the launch's context bound; the clamp keeps a violated bound in-bounds
  const int n_used = min((ctx + kPart - 1) / kPart, n_parts);
  PK_DEVICE_ASSERT(ctx <= n_parts * kPart);
  if (static_cast<int>(bz) >= n_used) return;
  const int r = lane & 15, g = lane >> 4;
  // (in the standalone kernel, prefetching the first K/V step across the q preparation below
  // was measured slower: 256 VGPRs + AGPRs, one wave per SIMD; the fused launch does prefetch
  // (PRE), before its hand-off wait, where the registers are otherwise idle)
  bf16x8_t qf[4];
  // fold: the workgroup holding the new token (key ctx - 1) keeps its k / v in LDS, attends to
  // keys [0, ctx - 1) from the cache and adds key ctx - 1 from LDS in the final combine; the
  // cache write goes out at the end of the kernel.  Writing the row first and reading it back
  // through the cache cost 4-5 us per launch at 384-512 keys (the scattered 2-byte V^T stores
  // and the K tile stores land on lines the waves are about to stream).
  bool fold = false;
  int slot = -1;
  if constexpr (FROM_QKV) {
    auto& q_s = L.q_s;
    const int N = (n_q + 2 * n_kv) * kHD;
    const int64_t slab = static_cast<int64_t>(qi.M) * N;
    const float* base = qi.partial + static_cast<int64_t>(seq) * N;
    const float* cs = qi.cos_sin + static_cast<int64_t>(pos_q) * kHD;
    slot = slot_q;
    const bool writer = slot >= 0 && static_cast<int>(bz) == (n_used - 1) % static_cast<int>(gdz);
    fold = writer && pos_q == ctx - 1;
    // one pass of 16-byte slab loads per thread for G <= 14 (1-column items took 3 dependent
    // rounds at G = 8)
    const int n_items = G * 16 + (writer ? 32 : 0);
    for (int it = threadIdx.x; it < n_items; it += 64 * NW) {
      int j;
      const int col = item_col(it, j);
      float4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
      if constexpr (SS > 0) {  // all slab loads in flight before the first add
        float4 va[SS], vb[SS];
        if (kHoist && it == static_cast<int>(threadIdx.x)) {
#pragma unroll
          for (int sp = 0; sp < SS; ++sp) {
            va[sp] = hva[sp];
            vb[sp] = hvb[sp];
          }
        } else {
#pragma unroll
          for (int sp = 0; sp < SS; ++sp) {
            va[sp] = ld_slab4<(FL & 2) != 0>(qi.partial, base + sp * slab + col);
            vb[sp] = ld_slab4<(FL & 2) != 0>(qi.partial, base + sp * slab + col + 64);
          }
        }
#pragma unroll
        for (int sp = 0; sp < SS; ++sp) {
          add4f(a, va[sp]);
          add4f(b, vb[sp]);
        }
      } else {
        for (int sp = 0; sp < qi.S; ++sp) {
          add4f(a, ld_slab4<(FL & 2) != 0>(qi.partial, base + sp * slab + col));
          add4f(b, ld_slab4<(FL & 2) != 0>(qi.partial, base + sp * slab + col + 64));
        }
      }
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
      if (it < G * 16 + 16) {  // q or k: round (the GEMM output), rotate (neox)
        const float4 co4 = *reinterpret_cast<const float4*>(cs + j), si4 = *reinterpret_cast<const float4*>(cs + 64 + j);
        const float co[4] = {co4.x, co4.y, co4.z, co4.w}, si[4] = {si4.x, si4.y, si4.z, si4.w};
        float ra[4], rb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = bf2f(f2bf(av[e])), y = bf2f(f2bf(bv[e]));
          ra[e] = x * co[e] - y * si[e];
          rb[e] = y * co[e] + x * si[e];
        }
        uint2 pa, pb;
        pa.x = pack2(ra[0], ra[1]);
        pa.y = pack2(ra[2], ra[3]);
        pb.x = pack2(rb[0], rb[1]);
        pb.y = pack2(rb[2], rb[3]);
        bf16_t* dst;
        if (it < G * 16) {
          dst = &q_s[it >> 4][j];
        } else if (fold) {
          dst = &kn_s[j];
        } else {  // fragment-native K tile: 4-dim groups stay contiguous (common.h kcache_off)
          bf16_t* d = kc + (static_cast<int64_t>(slot / bs) * n_kv + h) * bs * kHD;
          *reinterpret_cast<uint2*>(d + kcache_off(slot % bs, j)) = pa;
          *reinterpret_cast<uint2*>(d + kcache_off(slot % bs, j + 64)) = pb;
          continue;
        }
        *reinterpret_cast<uint2*>(dst) = pa;
        *reinterpret_cast<uint2*>(dst + 64) = pb;
      } else if (fold) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vn_s[j + e] = bf2f(f2bf(av[e]));
          vn_s[j + 64 + e] = bf2f(f2bf(bv[e]));
        }
      } else {  // transposed V tile: channels j..j+3 are 8 elements apart (common.h vcache_off)
        bf16_t* d = vc + (static_cast<int64_t>(slot / bs) * n_kv + h) * kHD * bs;
        const int va0 = vcache_off(slot % bs, j), vb0 = vcache_off(slot % bs, j + 64);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d[va0 + 8 * e] = f2bf(av[e]);
          d[vb0 + 8 * e] = f2bf(bv[e]);
        }
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

  // the grid's z dimension is small (<= 4); a workgroup walks partitions z, z + gdz, ...
  // carrying its online-softmax state across them (the order of key blocks does not matter to
  // the softmax), so it combines its waves and writes ONE partial at the end: no LDS combine /
  // partial store between partitions and gdz partials to merge instead of n_parts.
  const int n_eff = min(n_used, static_cast<int>(gdz));  // partials of this sequence
  const int ctx_c = fold ? ctx - 1 : ctx;  // keys read from the cache
  WaveState st;
  init_state(st);
  for (int part = bz; part < n_used; part += gdz) {
    const int begin = part * kPart;
    const int end = min(ctx_c, begin + kPart);
    const int b0 = begin / bs, nblk = (end - 1) / bs - b0 + 1;
    const bool pre = PRE > 0 && part == static_cast<int>(bz) && prefetched;  // window + steps loaded
    if (!pre) {
      __syncthreads();  // the previous partition's block-table readers are done
      if (part == static_cast<int>(bz) && kPart % bs == 0) {  // nblk <= kPart / bs <= 64 * NW
        if (static_cast<int>(threadIdx.x) < nblk) bt_s[threadIdx.x] = bt_pre;
      } else
        for (int i = threadIdx.x; i < nblk; i += 64 * NW)
          bt_s[i] = block_tables[static_cast<int64_t>(seq) * max_blocks + b0 + i];
      __syncthreads();
    }
    if (end > begin) {
      // ONE attend instantiation per kernel (a second, inlined next to it, made hipcc spill ~60
      // registers): with the prefetch, partitions that were not prefetched load their first step here
      if constexpr (PRE > 0) {
        if (!pre) {
          load_kv(fa, kch, vch, blk_stride, bt_s, b0, bs, begin + kStep * w, min(ctx_c, end));
          if constexpr (PRE == 2)
            load_kv(fb, kch, vch, blk_stride, bt_s, b0, bs, begin + kStep * w + NW * kStep, min(ctx_c, end));
        }
      }
      attend<PRE>(st, qf, kch, vch, blk_stride, bt_s, b0, bs, begin + kStep * w, end, NW * kStep, ctx_c, ctx_c - 1,
                  scale2, fa, fb);
    }
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
      const int64_t pi = (static_cast<int64_t>(seq) * n_q + hq) * n_parts + bz;
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


}  // namespace
