// Weight-streaming "skinny" GEMM for decode: C[M, N] = A[M, K] . W[N, K]^T, M <= 64, bf16.
//
// Decode GEMMs are HBM-bound on W (8B: 436 MB of weights per layer-step, M = batch <= 64), so
// the kernel is built around streaming W once at full rate (guide §5 "GEMV / M <= 16" row:
// operands straight to VGPRs, no LDS round trip, deep unroll):
//   * one wave owns 32 W rows (R = 2 tiles of 16) over a K-slice and computes the transposed
//     tile C^T[32 n x 16*MT m] with mfma_f32_16x16x32_bf16 (A operand = W rows, B operand =
//     activations), so every lane reads 64 contiguous bytes of a W row per 128-deep k-step;
//   * k is permuted inside each 128-step (lane group g owns k in [32g, 32g+32)) identically for
//     W and A, so all operand loads are 16-byte vectors and the dot product is unchanged;
//   * the next k-step's W fragments are issued before the current MFMAs (register double
//     buffer) so ~16 KB per wave stay in flight;
//   * split-K over workgroups when N / 32 alone cannot fill 256 CUs; partial sums are fp32
//     slabs [S, M, N] reduced by the consumer kernel (reduce / reduce+SiLU / reduce+residual+
//     RMSNorm), so a split costs no extra launch on the hot path;
//   * epilogues: bf16 store, fp32 partial store, or fused SiLU(gate)*up when W's gate/up rows
//     are interleaved in blocks of 16 (then one wave holds gate and up of the same columns);
//   * block-packed W (ops/gemm.py pack_weight): per (128-row n-block, 128-deep k-step) the 32 KiB
//     a workgroup consumes are contiguous, as 32 MFMA A-fragments of 1 KiB in lane order, so
//     every wave load instruction reads 1 KiB and a workgroup sweeps one linear stream
//     (tools/gemm_lab.hip: LM head 5.1 -> 5.9 TB/s with non-temporal loads).
#include <cstring>

#include "skinny_tile.h"

using namespace pk;

namespace {

template <int MT, int MODE, bool PK, bool NORM, bool NT, bool RS = false, int KR = 2>
__global__ void __launch_bounds__(256, 2) skinny_gemm_kernel(const GemmArgs args) {
  __shared__ SkinnyLds<MT> lds;
  skinny_tile<MT, MODE, PK, NORM, NT, RS, KR>(args, blockIdx.x, blockIdx.y, gridDim.x, lds, Flow{});
}

// Fused decode MLP (M <= 64): gate_up + SiLU (folded norm, non-temporal packed W) and the down
// projection's split-K slabs in ONE launch of max(gate_up tiles, down tiles) workgroups, one per
// CU: workgroup b runs gate_up tile b (if any), then down tile b (if any).  A down tile streams
// its first weight k-steps, then waits until the gate_up tiles of its K slice have stored h, so
// the down projection's launch boundary and weight ramp overlap the gate_up tail.  Every
// workgroup is resident at once (one per CU) and a gate_up tile never waits: no deadlock.
// (A/B, tools/gpu/mlp_ab.sh: down tiles as workgroups of their own, dispatched after the gate_up
// ones, put two down tiles on some CUs and lost 7 us per layer.)
// DKR: the down projection's n-block height (2: 128 rows; 1: 64 rows -- twice the tiles at the
// same split when 128-row tiles would leave CUs idle: 8B 32 x 4, 70B TP=8 64 x 2 -> 256).
// DNT: non-temporal down weights (A/B builds: tools/lab/build_variant.py)
// (Removed in round 6, measured slower: gate_up split over K inside this launch -- the 70B TP=8
// shard, r4_tp_solo.md -- and the o-projection's residual update as phase 0, r5_phase_ab.jsonl.)
template <int MT, int DKR, bool DNT = false>
__global__ void __launch_bounds__(256, 2) mlp_fused_kernel(const GemmArgs gu, const GemmArgs dn, const Flow fgu,
                                                           const Flow fdn, int n_gu, int n_dn) {
  __shared__ SkinnyLds<MT> lds;
  const int b = blockIdx.x;
  if (b < n_gu) {
    skinny_tile<MT, kSiluMul, true, false, true, true, 2, 1>(gu, b, 0, n_gu, lds, fgu);
    __syncthreads();  // the LDS tiles are reused by the down tile
  }
  if (b < n_dn) skinny_tile<MT, kPartial, true, false, DNT, false, DKR, 2>(dn, b, 0, n_dn, lds, fdn);
}

// x[m] = bf16(bf16(residual[m] * rinv[m]) * w), rinv from the per-row sum-of-squares parts a
// kAddResNorm epilogue wrote (the final RMSNorm of the fused decode chain).  One row per WG.
__global__ void __launch_bounds__(256) norm_apply_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ residual,
                                                         const float* __restrict__ parts, int nparts,
                                                         const bf16_t* __restrict__ w, int M, int H, float eps) {
  const int m = blockIdx.x;
  float ss = 0.f;
  for (int q = 0; q < nparts; ++q) ss += parts[q * M + m];
  const float ri = rsqrtf(ss / H + eps);
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float v[8], wv[8];
    unpack8(*reinterpret_cast<const u32x4*>(residual + static_cast<int64_t>(m) * H + c), v);
    unpack8(*reinterpret_cast<const u32x4*>(w + c), wv);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf(v[j] * ri) * wv[j];
    *reinterpret_cast<u32x4*>(x + static_cast<int64_t>(m) * H + c) = pack8(v);
  }
}

// Sum S fp32 slabs [S, M, N] -> bf16 [M, ldo]; SILU: N = 2I interleaved (16 gate | 16 up).
// One thread per 4 output columns: with SILU its 4 gate columns and the 4 up columns 16 further,
// so every thread works (SS > 0: all 2 SS slab loads issued before the first add -- one round
// trip; a runtime loop whose up loads followed the gate loads of half the threads took two).
template <bool SILU, int SS>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16_t* __restrict__ out, const float* __restrict__ partial,
                                                            int S, int M, int N, int ldo) {
  const int m = blockIdx.y;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;  // 4-column group of the output
  const int nout = SILU ? N / 2 : N;
  if (v * 4 >= nout) return;
  // SILU: output columns 4v..4v+3 = h block b, offset j; gate slab column 32 b + j, up + 16
  const int c = SILU ? ((4 * v) >> 4) * 32 + ((4 * v) & 15) : 4 * v;
  const float* src = partial + static_cast<int64_t>(m) * N + c;
  const int64_t slab = static_cast<int64_t>(M) * N;
  float4 g = slab_sum<SS>(src, slab, S);
  if (!SILU) {
    uint2 o;
    o.x = pack2(g.x, g.y);
    o.y = pack2(g.z, g.w);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * ldo + 4 * v) = o;
  } else {
    const float4 u = slab_sum<SS>(src + 16, slab, S);
    float g4[4] = {g.x, g.y, g.z, g.w}, u4[4] = {u.x, u.y, u.z, u.w}, y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = bf2f(f2bf(silu(bf2f(f2bf(g4[i]))))) * bf2f(f2bf(u4[i]));
    uint2 o;
    o.x = pack2(y[0], y[1]);
    o.y = pack2(y[2], y[3]);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * ldo + 4 * v) = o;
  }
}

// Residual update of the folded-RMSNorm decode chain: residual[m] += bf16(sum_s partial[s, m])
// (partial == null: residual unchanged) and parts[blk, m] = sum of squares of the new residual
// over columns [512 blk, 512 blk + 512).  The consumer GEMM turns the parts into rinv[m]
// (GemmArgs::row_scale) and streams the RMSNorm weight pre-multiplied into its W, so no
// normalised copy of the residual is ever written.  One wave per (512 columns, row): every lane
// issues its 2 (S + 1) loads at once and the sum of squares is a cross-lane reduction -- no LDS,
// no barrier (this kernel is latency-bound: 64 launches per 8B decode step).
template <int SS>
__global__ void __launch_bounds__(64) residual_parts_kernel(bf16_t* __restrict__ residual,
                                                            const float* __restrict__ partial, int S, int M, int H,
                                                            float* __restrict__ parts) {
  const int blk = blockIdx.x, m = blockIdx.y, lane = threadIdx.x;
  const int c = blk * kPartCols + lane * 4;  // columns c..c+3 and c+256..c+259
  bf16_t* res = residual + static_cast<int64_t>(m) * H + c;
  const uint2 r0 = *reinterpret_cast<const uint2*>(res);
  const uint2 r1 = *reinterpret_cast<const uint2*>(res + 256);
  float v[8] = {bf2f(static_cast<bf16_t>(r0.x & 0xffff)), bf2f(static_cast<bf16_t>(r0.x >> 16)),
                bf2f(static_cast<bf16_t>(r0.y & 0xffff)), bf2f(static_cast<bf16_t>(r0.y >> 16)),
                bf2f(static_cast<bf16_t>(r1.x & 0xffff)), bf2f(static_cast<bf16_t>(r1.x >> 16)),
                bf2f(static_cast<bf16_t>(r1.y & 0xffff)), bf2f(static_cast<bf16_t>(r1.y >> 16))};
  if (partial != nullptr) {
    // the projection output is rounded to bf16 first (as the unfused GEMM would store it)
    const float* src = partial + static_cast<int64_t>(m) * H + c;
    const int64_t slab = static_cast<int64_t>(M) * H;
    const float4 a = slab_sum<SS>(src, slab, S), b = slab_sum<SS>(src + 256, slab, S);
    const float av[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = rbf(rbf(av[i]) + v[i]);
    uint2 o0, o1;
    o0.x = pack2(v[0], v[1]);
    o0.y = pack2(v[2], v[3]);
    o1.x = pack2(v[4], v[5]);
    o1.y = pack2(v[6], v[7]);
    *reinterpret_cast<uint2*>(res) = o0;
    *reinterpret_cast<uint2*>(res + 256) = o1;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if (lane == 0) parts[static_cast<int64_t>(blk) * M + m] = ss;
}

// residual = bf16(residual + bf16(sum_s partial[s])); x = rmsnorm(residual) * w.
// One row per workgroup of H/4 (<= 1024) threads, PER float4 column groups per thread; the S
// slab loads of a group are independent and issued back to back (latency, not bandwidth, is
// what a 64-row reduction fights).
// Optional MoE routing of the normalised row (ROUTE): logits = bf16(x . router[e]) for the E
// experts, softmax, top-k, renormalised weights -> ids[m, k], rw[m, k].  Replaces the router
// GEMM and the top-k softmax kernel of a Mixtral decode layer.
struct RouteArgs {
  const bf16_t* router;  // [E, H]
  int* ids;              // [M, k]
  float* w;              // [M, k]
  int E, k, renorm;
};

template <int PER, int SS, bool ROUTE = false>
__global__ void __launch_bounds__(1024) splitk_add_rmsnorm_kernel(bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
                                                                  const float* __restrict__ partial,
                                                                  const bf16_t* __restrict__ w, int S, int M, int H,
                                                                  float eps, const RouteArgs ra = RouteArgs{}) {
  __shared__ float red[16];
  const int m = blockIdx.x;
  float v[PER][4];
  float ss = 0.f;
  bf16_t* res = residual + static_cast<int64_t>(m) * H;
  const int64_t slab = static_cast<int64_t>(M) * H;
  const float* base = partial + static_cast<int64_t>(m) * H;
  // the norm weight and (ROUTE) the router rows do not depend on the slabs: request them first,
  // so their round trips overlap the slab loads instead of following the row reduction
  constexpr int kRouteE = 8;  // router experts per pass (E <= 8: all of them, prefetched)
  uint2 wpre[PER];
  uint2 rpre[ROUTE ? PER : 1][ROUTE ? kRouteE : 1];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    wpre[i] = *reinterpret_cast<const uint2*>(w + c);
    if constexpr (ROUTE) {
#pragma unroll
      for (int e = 0; e < kRouteE; ++e)
        if (e < ra.E) rpre[i][e] = *reinterpret_cast<const uint2*>(ra.router + static_cast<int64_t>(e) * H + c);
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    float4 acc;
    if constexpr (SS > 0) {
      float4 p[SS];  // all slab loads in flight before the first add
#pragma unroll
      for (int q = 0; q < SS; ++q) p[q] = ld4f(base + q * slab + c);
      acc = p[0];
#pragma unroll
      for (int q = 1; q < SS; ++q) add4(acc, p[q]);
    } else {
      acc = ld4f(base + c);
      for (int q = 1; q < S; ++q) add4(acc, ld4f(base + q * slab + c));
    }
    const uint2 rr = *reinterpret_cast<const uint2*>(res + c);
    // the projection output is rounded to bf16 first (as the unfused GEMM would store it)
    v[i][0] = bf2f(f2bf(bf2f(f2bf(acc.x)) + bf2f(static_cast<bf16_t>(rr.x & 0xffff))));
    v[i][1] = bf2f(f2bf(bf2f(f2bf(acc.y)) + bf2f(static_cast<bf16_t>(rr.x >> 16))));
    v[i][2] = bf2f(f2bf(bf2f(f2bf(acc.z)) + bf2f(static_cast<bf16_t>(rr.y & 0xffff))));
    v[i][3] = bf2f(f2bf(bf2f(f2bf(acc.w)) + bf2f(static_cast<bf16_t>(rr.y >> 16))));
    uint2 o;
    o.x = pack2(v[i][0], v[i][1]);
    o.y = pack2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(res + c) = o;
    ss += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  }
  const float rinv = rsqrtf(block_sum(ss, red) / H + eps);
  bf16_t* xo = x + static_cast<int64_t>(m) * H;
  float xr[ROUTE ? PER : 1][4];  // the written (bf16-rounded) x values, kept for the router
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    const uint2 ww = wpre[i];
    float y[4];
    y[0] = bf2f(f2bf(v[i][0] * rinv)) * bf2f(static_cast<bf16_t>(ww.x & 0xffff));
    y[1] = bf2f(f2bf(v[i][1] * rinv)) * bf2f(static_cast<bf16_t>(ww.x >> 16));
    y[2] = bf2f(f2bf(v[i][2] * rinv)) * bf2f(static_cast<bf16_t>(ww.y & 0xffff));
    y[3] = bf2f(f2bf(v[i][3] * rinv)) * bf2f(static_cast<bf16_t>(ww.y >> 16));
    uint2 o;
    o.x = pack2(y[0], y[1]);
    o.y = pack2(y[2], y[3]);
    *reinterpret_cast<uint2*>(xo + c) = o;
    if constexpr (ROUTE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) xr[i][j] = bf2f(f2bf(y[j]));
    }
  }
  if constexpr (ROUTE) {
    // router logits from the x row still in registers: kRouteE experts per pass, every router
    // load of the pass issued together and the kRouteE wave reductions independent of each
    // other (one expert at a time re-derived x and serialised 8 load + reduce round trips)
    __shared__ float part_s[16][64];
    __shared__ float logit_s[64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int e0 = 0; e0 < ra.E; e0 += kRouteE) {
      float acc[kRouteE];
#pragma unroll
      for (int e = 0; e < kRouteE; ++e) acc[e] = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = 4 * (threadIdx.x + i * blockDim.x);
#pragma unroll
        for (int e = 0; e < kRouteE; ++e) {
          if (e0 + e < ra.E) {
            const uint2 rr = e0 == 0 ? rpre[i][e]
                                     : *reinterpret_cast<const uint2*>(ra.router + static_cast<int64_t>(e0 + e) * H + c);
            acc[e] += xr[i][0] * bf2f(static_cast<bf16_t>(rr.x & 0xffff)) +
                      xr[i][1] * bf2f(static_cast<bf16_t>(rr.x >> 16)) +
                      xr[i][2] * bf2f(static_cast<bf16_t>(rr.y & 0xffff)) +
                      xr[i][3] * bf2f(static_cast<bf16_t>(rr.y >> 16));
          }
        }
      }
#pragma unroll
      for (int e = 0; e < kRouteE; ++e) acc[e] = wave_sum(acc[e]);
      if (lane == 0) {
#pragma unroll
        for (int e = 0; e < kRouteE; ++e)
          if (e0 + e < ra.E) part_s[wid][e0 + e] = acc[e];
      }
    }
    __syncthreads();
    if (threadIdx.x < ra.E) {
      float t = 0.f;
      for (int q = 0; q < nw; ++q) t += part_s[q][threadIdx.x];
      logit_s[threadIdx.x] = bf2f(f2bf(t));  // the router GEMM's bf16 output
    }
    __syncthreads();
    // softmax + top-k with no serial thread: lane e reads every logit, finds its own rank (value
    // descending, lower expert first on ties -- the order a greedy arg-max scan picks) and, when
    // it ranks below k, owns output slot `rank`; the renormalisation sum adds the chosen
    // probabilities in rank order, as the scan did
    __shared__ float psel_s[64];
    const int E = ra.E, e = threadIdx.x;
    int rank = E;
    float pr = 0.f;
    if (e < E) {
      float mx = -INFINITY;
      for (int q = 0; q < E; ++q) mx = fmaxf(mx, logit_s[q]);
      float sum = 0.f;
      for (int q = 0; q < E; ++q) sum += __expf(logit_s[q] - mx);
      const float le = logit_s[e];
      rank = 0;
      for (int q = 0; q < E; ++q) {
        const float lq = logit_s[q];
        rank += (lq > le || (lq == le && q < e)) ? 1 : 0;
      }
      pr = __expf(le - mx) / sum;
      if (rank < ra.k) psel_s[rank] = pr;
    }
    __syncthreads();
    if (rank < ra.k) {
      float wsum = 0.f;
      for (int j = 0; j < ra.k; ++j) wsum += psel_s[j];
      ra.ids[m * ra.k + rank] = e;
      ra.w[m * ra.k + rank] = ra.renorm ? pr / wsum : pr;
    }
  }
}

// Split-K QKV epilogue fused with RoPE and the paged KV write: sum the S fp32 slabs of the
// fused q|k|v projection, round to bf16 (the unfused GEMM output), rotate q and k (neox, fp32
// cos|sin table), write q to q_out [M, nq*128], k to the K cache and v to the transposed V
// cache (slot < 0: padding row, nothing cached).  Replaces reduce + rope_and_cache.
// One wave per (row, head) so M * (nq + 2 nkv) waves cover the chip and every lane issues its
// 2 S slab loads back to back (a per-row workgroup walking heads serially was latency-bound).
template <int SS>
__global__ void __launch_bounds__(256) qkv_reduce_rope_cache_kernel(
    bf16_t* __restrict__ q_out, const float* __restrict__ partial, int S, int M, int nq, int nkv,
    const int* __restrict__ positions, const float* __restrict__ cos_sin, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ slots, int bs) {
  const int nh = nq + 2 * nkv;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= M * nh) return;
  const int m = item / nh, h = item % nh;
  const int lane = threadIdx.x & 63;
  const int N = nh * 128;
  const int64_t slab = static_cast<int64_t>(M) * N;
  const float* base = partial + static_cast<int64_t>(m) * N + h * 128;
  const int slot = slots[m];
  if (h >= nq && slot < 0) return;
  float a, b;
  if constexpr (SS > 0) {
    float va[SS], vb[SS];
#pragma unroll
    for (int s = 0; s < SS; ++s) {
      va[s] = base[s * slab + lane];
      vb[s] = base[s * slab + lane + 64];
    }
    a = va[0];
    b = vb[0];
#pragma unroll
    for (int s = 1; s < SS; ++s) {
      a += va[s];
      b += vb[s];
    }
  } else {
    a = 0.f;
    b = 0.f;
    for (int s = 0; s < S; ++s) {
      a += base[s * slab + lane];
      b += base[s * slab + lane + 64];
    }
  }
  if (h < nq + nkv) {
    a = rbf(a);
    b = rbf(b);
    const float* cs = cos_sin + static_cast<int64_t>(positions[m]) * 128;
    const float co = cs[lane], si = cs[64 + lane];
    if (h < nq) {
      bf16_t* d = q_out + static_cast<int64_t>(m) * nq * 128 + h * 128;
      d[lane] = f2bf(a * co - b * si);
      d[lane + 64] = f2bf(b * co + a * si);
    } else {  // fragment-native K tile (common.h kcache_off)
      bf16_t* d = kc + (static_cast<int64_t>(slot / bs) * nkv + (h - nq)) * bs * 128;
      d[kcache_off(slot % bs, lane)] = f2bf(a * co - b * si);
      d[kcache_off(slot % bs, lane + 64)] = f2bf(b * co + a * si);
    }
  } else {
    bf16_t* d = vc + (static_cast<int64_t>(slot / bs) * nkv + (h - nq - nkv)) * 128 * bs;
    d[vcache_off(slot % bs, lane)] = f2bf(a);
    d[vcache_off(slot % bs, lane + 64)] = f2bf(b);
  }
}

template <int MODE, bool PK, bool NORM, bool NT, bool RS = false, int KR = 2>
int launch(const GemmArgs& a, hipStream_t stream) {
  const dim3 grid((a.N / (64 * KR)) * a.S * a.row_tiles, a.row_offsets != nullptr ? a.groups : 1);
  if (a.tile_rows == 128) {  // row-tiled decode batches above 64 (dispatch: modes 0-2, no norm prologue)
    if constexpr (MODE <= kSiluMul && !NORM) {
      skinny_gemm_kernel<8, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a);
      return PK_CHECK_LAUNCH();
    }
    return -1;
  }
  switch ((min(min(a.M, 64), a.max_group_rows > 0 ? a.max_group_rows : 64) + 15) / 16) {
    case 1: skinny_gemm_kernel<1, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    case 2: skinny_gemm_kernel<2, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    case 3: skinny_gemm_kernel<3, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    case 4: skinny_gemm_kernel<4, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

// non-temporal weight loads are instantiated only for the large single-pass streams
// (bf16 out: LM head; SiLU: gate_up / MoE w13) on the packed layout
template <int MODE, bool NORM>
int launch_pk(const GemmArgs& a, bool packed, bool nt, hipStream_t stream) {
  // the folded-norm row scale is instantiated for the packed decode projections that take it
  // (QKV split-K slabs, gate_up SiLU)
  if constexpr ((MODE == kPartial || MODE == kSiluMul) && !NORM)
    if (a.row_scale) {
      if (!packed) return -1;
      if constexpr (MODE == kSiluMul)
        if (nt) return launch<MODE, true, NORM, true, true>(a, stream);
      return launch<MODE, true, NORM, false, true>(a, stream);
    }
  if (a.row_scale) return -1;
  if constexpr ((MODE == kBF16 || MODE == kSiluMul) && !NORM)
    if (packed && nt) return launch<MODE, true, NORM, true>(a, stream);
  return packed ? launch<MODE, true, NORM, false>(a, stream) : launch<MODE, false, NORM, false>(a, stream);
}

// kPush: one 64-row tile, split-K tickets, a TP group whose owner chunks split N evenly, and
// n-blocks (of ncol columns) that the owners' push-flag rows can index
bool push_ok(const GemmArgs& a, int ncol) {
  return a.counters != nullptr && a.partial != nullptr && a.push_peers != nullptr && a.push_world >= 2 &&
         a.push_world <= pkcomm::kMaxRanks && a.push_rank >= 0 && a.push_rank < a.push_world && a.M <= 64 &&
         a.row_tiles == 1 && !a.row_scale && a.N % (pkcomm::kRrChunk * a.push_world) == 0 &&
         a.N / ncol <= pkcomm::kMaxBlocks && static_cast<long long>(a.M) * a.N * 2 <= a.push_bytes;
}

int dispatch(const GemmArgs& args, int mode, hipStream_t stream) {
  if (args.M <= 0) return 0;
  GemmArgs a = args;
  const bool grouped = a.row_offsets != nullptr;
  if (grouped && (a.groups <= 0 || a.max_group_rows <= 0 || a.max_group_rows > kMaxRows || (mode & 7) > kSiluMul ||
                  (mode & 32)))
    return -1;
  // a group (dense: the whole M) above 64 rows: row tiles of 128 (64 when the row scale has more
  // than 16 parts per row) for the modes without an in-launch split-K reduction (its per-n-block
  // tickets would be shared by the row tiles) and without the A-staging norm prologue
  const int rows = grouped ? a.max_group_rows : a.M;
  // (bit 8: 64-row tiles regardless -- tools/bench_gemm_rows.py compares the two)
  a.tile_rows = rows > 64 && !(a.row_scale && a.nrm_nparts > 16) && !(mode & 256) ? 128 : 64;
  a.row_tiles = (rows + a.tile_rows - 1) / a.tile_rows;
  if (rows > 64 && (rows > kMaxRows || (mode & 7) > kSiluMul || (mode & 32))) return -1;
  if (a.N % 128 || a.S < 1 || a.K % (kKC * a.S) || a.lda % 8) return -1;
  const bool packed = (mode & 16) != 0;  // bit 4: W in block-packed layout
  const bool norm = (mode & 32) != 0;    // bit 5: RMSNorm prologue on A
  // bit 6: non-temporal weight loads (hint); not with several row tiles, whose workgroups of one
  // W tile read it through the XCD's L2 one after another
  const bool nt = (mode & 64) != 0 && a.row_tiles == 1;
  const bool half = (mode & 128) != 0;   // bit 7: 64-row n-blocks (KR = 1)
  if (norm && (a.nrm_parts == nullptr || a.nrm_w == nullptr)) return -1;
  if (half) {  // split-K projections (fp32 slabs, the in-launch residual update); bf16 out with too
               // few 128-row n-blocks to fill the chip (the 70B TP=8 LM-head shard: 126)
    if (grouped || norm) return -1;
    if ((mode & 7) == kBF16) {
      if (a.S != 1 || a.row_scale || a.row_tiles > 1) return -1;
      if (nt) return packed ? launch<kBF16, true, false, true, false, 1>(a, stream) : -1;
      return packed ? launch<kBF16, true, false, false, false, 1>(a, stream)
                    : launch<kBF16, false, false, false, false, 1>(a, stream);
    }
    if (nt) return -1;
    if (a.row_scale) {  // folded-norm QKV slabs (packed W only)
      if ((mode & 7) != kPartial || !packed || a.nrm_parts == nullptr || a.nrm_nparts < 1 || a.nrm_nparts > 64)
        return -1;
      return launch<kPartial, true, false, false, true, 1>(a, stream);
    }
    if ((mode & 7) == kPartial)
      return packed ? launch<kPartial, true, false, false, false, 1>(a, stream)
                    : launch<kPartial, false, false, false, false, 1>(a, stream);
    if ((mode & 7) == kAddResNorm) {
      if (a.counters == nullptr || a.residual == nullptr || a.sumsq_parts == nullptr) return -1;
      return packed ? launch<kAddResNorm, true, false, false, false, 1>(a, stream)
                    : launch<kAddResNorm, false, false, false, false, 1>(a, stream);
    }
    if ((mode & 7) == kPush) {
      if (!push_ok(a, 64)) return -1;
      return packed ? launch<kPush, true, false, false, false, 1>(a, stream)
                    : launch<kPush, false, false, false, false, 1>(a, stream);
    }
    return -1;
  }
  if (a.row_scale && (grouped || norm || a.nrm_parts == nullptr || a.nrm_nparts < 1 || a.nrm_nparts > 64))
    return -1;
  switch (mode & 7) {
    case kBF16:
      if (a.S != 1 || norm) return -1;
      return launch_pk<kBF16, false>(a, packed, nt, stream);
    case kPartial:
      if (norm) return -1;
      return launch_pk<kPartial, false>(a, packed, nt, stream);
    case kSiluMul:
      if (a.S != 1) return -1;
      return norm ? launch_pk<kSiluMul, true>(a, packed, nt, stream) : launch_pk<kSiluMul, false>(a, packed, nt, stream);
    case kAddResNorm:
      if (norm || a.counters == nullptr || a.residual == nullptr || a.sumsq_parts == nullptr) return -1;
      return launch_pk<kAddResNorm, false>(a, packed, nt, stream);
    case kQkvRope:
      if (a.counters == nullptr || a.N != (a.nq + 2 * a.nkv) * 128 || a.bs <= 0 || a.bs % 32) return -1;
      return norm ? launch_pk<kQkvRope, true>(a, packed, nt, stream) : launch_pk<kQkvRope, false>(a, packed, nt, stream);
    case kPush:
      if (norm || !push_ok(a, 128)) return -1;
      return packed ? launch<kPush, true, false, false>(a, stream) : launch<kPush, false, false, false>(a, stream);
    default: return -1;
  }
}

}  // namespace

// mode 0: out bf16 [M, ldo] (S must be 1); 1: partial fp32 [S, M, N]; 2: SiLU-mul of interleaved
// gate/up rows -> out bf16 [M, N/2] (S must be 1); bit 4: block-packed W; bit 6: non-temporal W.
// Requires M <= kMaxRows (> 64: 64-row tiles), N % 128 == 0, K % (256 S) == 0.
PK_EXPORT int pk_skinny_gemm(void* out, void* partial, const void* A, const void* W, int M, int N, int K, int lda,
                             int ldo, int S, int mode, hipStream_t stream) {
  GemmArgs a{};
  a.out = static_cast<bf16_t*>(out);
  a.partial = static_cast<float*>(partial);
  a.A = static_cast<const bf16_t*>(A);
  a.W = static_cast<const bf16_t*>(W);
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldo = ldo; a.S = S;
  if ((mode & 7) > kSiluMul || (mode & 32)) return -1;
  return dispatch(a, mode, stream);
}

// Full-featured entry: modes 0-6 (see Mode), bit 4 packed W, bit 5 RMSNorm prologue, bit 6 NT W.
PK_EXPORT int pk_skinny_gemm_ex(const GemmArgs* args, int mode, hipStream_t stream) {
  return dispatch(*args, mode, stream);
}

// Fused decode MLP (mlp_fused_kernel): gu = gate_up + SiLU (packed, non-temporal, folded norm:
// row_scale + nrm_parts; unsplit), dn = down split-K slabs (packed) reading gu's output.  flow: a
// zeroed int buffer of >= kFlowWords words (64 tickets and 64 consumer counts, 64 words apart, the
// sticky error word; ops/gemm.py FLOW_WORDS keeps 1024 spare words), left zeroed by every launch
// that completes.
constexpr int kFlowWords = 128 * kFlowPad + 64 + 1024;

// n-block height of the fused MLP's down tiles (ops/gemm.py down_kr must agree): 64 rows when
// 128-row tiles at split S would be fewer than 192 workgroups
static int down_kr(int N, int S) { return (N / 128) * S < 192 ? 1 : 2; }

PK_EXPORT int pk_mlp_fused(const GemmArgs* gu_in, const GemmArgs* dn_in, int* flow, hipStream_t stream) {
  GemmArgs gu = *gu_in, dn = *dn_in;
  if (gu.M <= 0) return 0;
  // up to 128 rows (one row tile; MT = 8 above 64 rows, whose row scale reads <= 16 parts)
  if (gu.M > 128 || (gu.M > 64 && gu.nrm_nparts > 16) || dn.M != gu.M || gu.N % 128 || gu.S != 1 || gu.K % kKC ||
      !gu.row_scale || gu.nrm_parts == nullptr || gu.nrm_nparts < 1 || gu.nrm_nparts > 64 || gu.out == nullptr ||
      dn.K != gu.N / 2 || dn.N % 128 || dn.S < 1 || dn.S > 64 || dn.K % (kKC * dn.S) || (dn.K / dn.S) % 64 ||
      dn.partial == nullptr || dn.A != gu.out || dn.lda % 8 || gu.lda % 8 || gu.row_offsets != nullptr ||
      dn.row_offsets != nullptr || flow == nullptr)
    return -1;
  gu.counters = nullptr;
  gu.row_tiles = dn.row_tiles = 1;
  gu.tile_rows = dn.tile_rows = gu.M > 64 ? 128 : 64;
  gu.max_group_rows = dn.max_group_rows = 0;
  int* done = flow + 64 * kFlowPad;
  int* err = fused_err_word() != nullptr ? fused_err_word() : flow + 128 * kFlowPad;
  const int dkr = down_kr(dn.N, dn.S);
  Flow fgu{flow, done, err, 0, 0, dn.K / dn.S, 1, 0, 0, fused_spin_limit()};
  Flow fdn{flow, done, err, (dn.K / dn.S) / 64, dn.N / (64 * dkr), dn.K / dn.S, 2, 0, 0, fused_spin_limit()};
  const int n_gu = gu.N / 128, n_dn = (dn.N / (64 * dkr)) * dn.S;
  const dim3 grid(n_gu > n_dn ? n_gu : n_dn);
  auto go = [&](auto kr) {
    constexpr int KR = decltype(kr)::value;
#define PK_MLPF(MT) mlp_fused_kernel<MT, KR><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn)
    switch ((gu.M + 15) / 16) {
      case 1: PK_MLPF(1); break;
      case 2: PK_MLPF(2); break;
      case 3: PK_MLPF(3); break;
      case 4: PK_MLPF(4); break;
      default: PK_MLPF(8); break;
    }
#undef PK_MLPF
  };
  if (dkr == 1)
    go(std::integral_constant<int, 1>{});
  else
    go(std::integral_constant<int, 2>{});
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_flow_words() { return kFlowWords; }

static int* g_fused_err = nullptr;
int* fused_err_word() { return g_fused_err; }
static int g_fused_spin_limit = 1 << 20;
int fused_spin_limit() { return g_fused_spin_limit; }

// Polls a fused launch's consumer makes before it declares its hand-off lost (default 2^20, ~0.5 s;
// n == 0 restores it).  n < 0 is a test hook: every wait reports a lost hand-off (the results are
// still computed correctly), so tests can drive the engine's fallback deterministically.
PK_EXPORT void pk_set_fused_spin_limit(int n) { g_fused_spin_limit = n != 0 ? n : (1 << 20); }

// Re-arm the sticky word after the engine has fallen back to the two-launch path.
PK_EXPORT void pk_clear_fused_err() {
  if (g_fused_err != nullptr) __atomic_store_n(g_fused_err, 0, __ATOMIC_SEQ_CST);
}

// The fused launches' sticky timeout word in host-mapped, coherent pinned memory (allocated once per
// process): returns its address (the host reads it with a plain load; 0 = no wait ever timed out).
PK_EXPORT void* pk_fused_err_word() {
  if (g_fused_err == nullptr) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    std::memset(h, 0, 64);
    g_fused_err = static_cast<int*>(h);
  }
  return g_fused_err;
}

PK_EXPORT int pk_norm_apply(void* x, const void* residual, const void* parts, int nparts, const void* w, int M,
                            int H, float eps, hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % 8) return -1;
  norm_apply_kernel<<<M, 256, 0, stream>>>(static_cast<bf16_t*>(x), static_cast<const bf16_t*>(residual),
                                           static_cast<const float*>(parts), nparts, static_cast<const bf16_t*>(w), M,
                                           H, eps);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_gemm_args_size() { return static_cast<int>(sizeof(GemmArgs)); }

PK_EXPORT int pk_splitk_reduce(void* out, const void* partial, int S, int M, int N, int ldo, int silu,
                               hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 4) return -1;
  if (silu && N % 32) return -1;
  dim3 grid(((silu ? N / 2 : N) / 4 + 255) / 256, M);
  bf16_t* o = static_cast<bf16_t*>(out);
  const float* p = static_cast<const float*>(partial);
#define PK_SKR(SI)                                                                                   \
  switch (S) {                                                                                       \
    case 2: splitk_reduce_kernel<SI, 2><<<grid, 256, 0, stream>>>(o, p, S, M, N, ldo); break;        \
    case 4: splitk_reduce_kernel<SI, 4><<<grid, 256, 0, stream>>>(o, p, S, M, N, ldo); break;        \
    case 8: splitk_reduce_kernel<SI, 8><<<grid, 256, 0, stream>>>(o, p, S, M, N, ldo); break;        \
    default: splitk_reduce_kernel<SI, 0><<<grid, 256, 0, stream>>>(o, p, S, M, N, ldo); break;       \
  }
  if (silu) {
    PK_SKR(true)
  } else {
    PK_SKR(false)
  }
#undef PK_SKR
  return PK_CHECK_LAUNCH();
}

static int add_rmsnorm_launch(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                              float eps, const RouteArgs* ra, hipStream_t stream);

PK_EXPORT int pk_splitk_add_rmsnorm(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                                    float eps, hipStream_t stream) {
  return add_rmsnorm_launch(x, residual, partial, w, S, M, H, eps, nullptr, stream);
}

// ... + MoE routing of every normalised row: ids [M, k] int32, weights [M, k] fp32 (E <= 64).
PK_EXPORT int pk_splitk_add_rmsnorm_route(void* x, void* residual, const void* partial, const void* w, int S, int M,
                                          int H, float eps, const void* router, int E, int k, int renorm, void* ids,
                                          void* rw, hipStream_t stream) {
  if (E > 64 || E < 1 || k > E) return -1;
  const RouteArgs ra{static_cast<const bf16_t*>(router), static_cast<int*>(ids), static_cast<float*>(rw), E, k, renorm};
  return add_rmsnorm_launch(x, residual, partial, w, S, M, H, eps, &ra, stream);
}

static int add_rmsnorm_launch(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                              float eps, const RouteArgs* ra, hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % 1024 || H > 8192) return -1;
  auto xx = static_cast<bf16_t*>(x);
  auto rr = static_cast<bf16_t*>(residual);
  auto pp = static_cast<const float*>(partial);
  auto ww = static_cast<const bf16_t*>(w);
  const int threads = H / 4 > 1024 ? 1024 : H / 4;
  auto go = [&](auto per, auto ss) {
    if (ra != nullptr)
      splitk_add_rmsnorm_kernel<decltype(per)::value, decltype(ss)::value, true><<<M, threads, 0, stream>>>(
          xx, rr, pp, ww, S, M, H, eps, *ra);
    else
      splitk_add_rmsnorm_kernel<decltype(per)::value, decltype(ss)::value, false><<<M, threads, 0, stream>>>(
          xx, rr, pp, ww, S, M, H, eps);
  };
  auto go_s = [&](auto per) {
    switch (S) {
      case 4: go(per, std::integral_constant<int, 4>{}); break;
      case 8: go(per, std::integral_constant<int, 8>{}); break;
      default: go(per, std::integral_constant<int, 0>{}); break;
    }
  };
  switch (H / (4 * threads)) {
    case 1: go_s(std::integral_constant<int, 1>{}); break;
    case 2: go_s(std::integral_constant<int, 2>{}); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

// residual [M, H] += sum of the S fp32 slabs [S, M, H] (partial may be null), parts [H/512, M].
PK_EXPORT int pk_residual_parts(void* residual, const void* partial, int S, int M, int H, void* parts,
                                hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % kPartCols || (partial != nullptr && S < 1)) return -1;
  const dim3 grid(H / kPartCols, M);
  auto rs = static_cast<bf16_t*>(residual);
  auto ps = static_cast<const float*>(partial);
  auto qs = static_cast<float*>(parts);
  switch (partial == nullptr ? 0 : S) {
    case 4: residual_parts_kernel<4><<<grid, 64, 0, stream>>>(rs, ps, S, M, H, qs); break;
    case 8: residual_parts_kernel<8><<<grid, 64, 0, stream>>>(rs, ps, S, M, H, qs); break;
    default: residual_parts_kernel<0><<<grid, 64, 0, stream>>>(rs, ps, S, M, H, qs); break;
  }
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_qkv_reduce_rope_cache(void* q_out, const void* partial, int S, int M, int nq, int nkv,
                                       const void* positions, const void* cos_sin, void* k_cache, void* v_cache,
                                       const void* slots, int bs, hipStream_t stream) {
  if (M <= 0) return 0;
  if (bs <= 0 || bs % 32 || S < 1) return -1;
  const int grid = (M * (nq + 2 * nkv) + 3) / 4;
  auto go = [&](auto ss) {
    qkv_reduce_rope_cache_kernel<decltype(ss)::value><<<grid, 256, 0, stream>>>(
        static_cast<bf16_t*>(q_out), static_cast<const float*>(partial), S, M, nq, nkv,
        static_cast<const int*>(positions), static_cast<const float*>(cos_sin), static_cast<bf16_t*>(k_cache),
        static_cast<bf16_t*>(v_cache), static_cast<const int*>(slots), bs);
  };
  switch (S) {
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    case 8: go(std::integral_constant<int, 8>{}); break;
    case 16: go(std::integral_constant<int, 16>{}); break;
    default: go(std::integral_constant<int, 0>{}); break;
  }
  return PK_CHECK_LAUNCH();
}
