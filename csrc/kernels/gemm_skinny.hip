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
//     are interleaved in blocks of 16 (then one wave holds gate and up of the same columns).
#include <type_traits>

#include "common.h"

using namespace pk;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

constexpr int kR = 2;        // 16-row W tiles per wave

enum Mode { kBF16 = 0, kPartial = 1, kSiluMul = 2 };

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// grid: (n_blocks * S) workgroups of 4 waves; workgroup -> (128-row n-block, k-split) with the
// split fastest.  Per 256-deep k-chunk the workgroup stages A[0:M, chunk] in LDS (double
// buffered, register-staged: loads for chunk c+1 are issued before chunk c's MFMAs and written
// after them), while each wave streams its own 32 W rows straight to VGPRs two 128-steps
// ahead (~16 KB per wave in flight).  W fragments use the natural k order (lane group g reads
// bytes [64s + 16g, +16) of a row in instruction s: 64 contiguous bytes per row).
constexpr int kKC = 256;           // k per LDS chunk
constexpr int kAStride = kKC + 8;  // bf16 elements per LDS row (+16 B pad: rows shift one 16-B slot)

template <int MT, int MODE, int D, bool PK>
__global__ void __launch_bounds__(256, D == 2 ? 2 : 1) skinny_gemm_kernel(bf16_t* __restrict__ out, float* __restrict__ partial,
                                                             const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                             int M, int N, int K, int lda, int ldo, int S, int n_blocks) {
  __shared__ __attribute__((aligned(16))) bf16_t a_lds[2][16 * MT][kAStride];
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int nb = blockIdx.x / S, split = blockIdx.x % S;
  const int kper = K / S;
  const int k0 = split * kper, k1 = k0 + kper;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = nb * 128 + w * 16 * kR;

  const bf16_t* wp[kR];
#pragma unroll
  for (int t = 0; t < kR; ++t)
    wp[t] = PK ? W + (static_cast<int64_t>((n0 >> 4) + t) * (K >> 5)) * 512 + 8 * lane   // fragment-packed
               : W + static_cast<int64_t>(n0 + 16 * t + r) * K + 8 * g;                // row-major [N, K]

  // A staging: MT*16 rows x 256 cols = MT*512 16-byte pieces over 256 threads
  constexpr int kPieces = (16 * MT * kKC / 8 + 255) / 256;
  u32x4 stage[kPieces];
  auto load_a = [&](int kc) {
#pragma unroll
    for (int p = 0; p < kPieces; ++p) {
      const int idx = tid + 256 * p;  // piece index
      const int row = idx >> 5, col = (idx & 31) * 8;
      const int src_row = min(row, M - 1);
      stage[p] = *reinterpret_cast<const u32x4*>(A + static_cast<int64_t>(src_row) * lda + kc + col);
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int p = 0; p < kPieces; ++p) {
      const int idx = tid + 256 * p;
      const int row = idx >> 5, col = (idx & 31) * 8;
      *reinterpret_cast<u32x4*>(&a_lds[buf][row][col]) = stage[p];
    }
  };

  f32x4 acc[kR][MT];
#pragma unroll
  for (int t = 0; t < kR; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // W register ring: steps k, k+128 (current chunk) loaded ahead
  bf16x8_t wa[kR][4], wb[kR][4];
  auto load_w = [&](bf16x8_t (&dst)[kR][4], int k) {
#pragma unroll
    for (int t = 0; t < kR; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) dst[t][s] = PK ? ld8(wp[t] + static_cast<int64_t>((k >> 5) + s) * 512) : ld8(wp[t] + k + 32 * s);
  };
  auto mma_step = [&](const bf16x8_t (&wf)[kR][4], int buf, int kk) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8_t af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        af[mt] = *reinterpret_cast<const bf16x8_t*>(&a_lds[buf][16 * mt + r][kk + 32 * s + 8 * g]);
#pragma unroll
      for (int t = 0; t < kR; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][s], af[mt], acc[t][mt], 0, 0, 0);
    }
  };

  // Chunk order is rotated per n-block: at any instant concurrent workgroups read different
  // column ranges of their rows, so the row-strided W stream spreads over all HBM channels
  // instead of camping on the few that one (row stride mod interleave) offset maps to.
  const int nchunks = kper / kKC;
  const int rot = (nb * 5) % nchunks;
  auto chunk_k = [&](int c) { return k0 + ((c + rot) % nchunks) * kKC; };
  // Every load in the loop is unconditional (past the last chunk the address is clamped to it
  // and the data is dropped): a load behind a branch makes the compiler's vmcnt bookkeeping
  // assume it was not issued, so it then drains ALL loads (vmcnt(0)) before the next MFMAs and
  // the W stream stalls once per chunk (measured: ~26 GB/s per workgroup).
  auto ck = [&](int c) { return chunk_k(min(c, nchunks - 1)); };
  if constexpr (D == 2) {
    // ring of 2 k-steps: W for the current chunk's two 128-steps in flight
    load_a(ck(0));
    load_w(wa, ck(0));
    load_w(wb, ck(0) + 128);
    store_a(0);
    int buf = 0;
    for (int c = 0; c < nchunks; ++c) {
      const int kn = ck(c + 1);
      load_a(kn);
      __syncthreads();  // chunk c visible in a_lds[buf]; every wave is done with a_lds[buf^1]
      mma_step(wa, buf, 0);
      load_w(wa, kn);
      mma_step(wb, buf, 128);
      load_w(wb, kn + 128);
      store_a(buf ^ 1);
      buf ^= 1;
    }
  } else {
    // ring of 4 k-steps (two chunks, ~32 KB per wave in flight); the loop is unrolled over a
    // chunk pair so every ring slot and LDS buffer index is static.
    bf16x8_t wc[kR][4], wd[kR][4];
    load_a(ck(0));
    load_w(wa, ck(0));
    load_w(wb, ck(0) + 128);
    load_w(wc, ck(1));
    load_w(wd, ck(1) + 128);
    store_a(0);
    for (int c = 0; c < nchunks; c += 2) {
      load_a(ck(c + 1));
      __syncthreads();  // chunk c visible in a_lds[0]; every wave is done with a_lds[1]
      mma_step(wa, 0, 0);
      load_w(wa, ck(c + 2));
      mma_step(wb, 0, 128);
      load_w(wb, ck(c + 2) + 128);
      store_a(1);
      if (c + 1 >= nchunks) break;  // uniform
      load_a(ck(c + 2));
      __syncthreads();  // chunk c+1 visible in a_lds[1]; every wave is done with a_lds[0]
      mma_step(wc, 1, 0);
      load_w(wc, ck(c + 3));
      mma_step(wd, 1, 128);
      load_w(wd, ck(c + 3) + 128);
      store_a(0);
    }
  }

  // C^T tile: rows = W rows (n), cols = m:  acc[t][mt][i] = C[m = 16*mt + r][n = n0 + 16*t + 4*g + i]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = 16 * mt + r;
    if (m >= M) continue;
    if (MODE == kPartial) {
      float* p = partial + (static_cast<int64_t>(split) * M + m) * N + n0 + 4 * g;
#pragma unroll
      for (int t = 0; t < kR; ++t) *reinterpret_cast<float4*>(p + 16 * t) =
          make_float4(acc[t][mt][0], acc[t][mt][1], acc[t][mt][2], acc[t][mt][3]);
    } else if (MODE == kBF16) {
      bf16_t* o = out + static_cast<int64_t>(m) * ldo + n0 + 4 * g;
#pragma unroll
      for (int t = 0; t < kR; ++t) {
        uint2 v;
        v.x = pack2(acc[t][mt][0], acc[t][mt][1]);
        v.y = pack2(acc[t][mt][2], acc[t][mt][3]);
        *reinterpret_cast<uint2*>(o + 16 * t) = v;
      }
    } else {  // kSiluMul: tile 0 = gate, tile 1 = up of the same 16 columns
      bf16_t* o = out + static_cast<int64_t>(m) * ldo + (n0 >> 1) + 4 * g;
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gt = bf2f(f2bf(acc[0][mt][i]));
        const float up = bf2f(f2bf(acc[1][mt][i]));
        y[i] = bf2f(f2bf(silu(gt))) * up;
      }
      uint2 v;
      v.x = pack2(y[0], y[1]);
      v.y = pack2(y[2], y[3]);
      *reinterpret_cast<uint2*>(o) = v;
    }
  }
}

// Sum S fp32 slabs [S, M, N] -> bf16 [M, ldo]; SILU: N = 2I interleaved (16 gate | 16 up).
template <bool SILU>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16_t* __restrict__ out, const float* __restrict__ partial,
                                                            int S, int M, int N, int ldo) {
  const int m = blockIdx.y;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;  // 4-column group
  if (v * 4 >= N) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < S; ++s) {
    const float4 p = *reinterpret_cast<const float4*>(partial + (static_cast<int64_t>(s) * M + m) * N + 4 * v);
    acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
  }
  if (!SILU) {
    uint2 o;
    o.x = pack2(acc.x, acc.y);
    o.y = pack2(acc.z, acc.w);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * ldo + 4 * v) = o;
  } else {
    // column c = 4v; block b = c / 32, within-block j = c % 32; gate if j < 16
    const int c = 4 * v, b = c >> 5, j = c & 31;
    if (j >= 16) return;
    float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) {
      const float4 p = *reinterpret_cast<const float4*>(partial + (static_cast<int64_t>(s) * M + m) * N + c + 16);
      u.x += p.x; u.y += p.y; u.z += p.z; u.w += p.w;
    }
    float g4[4] = {acc.x, acc.y, acc.z, acc.w}, u4[4] = {u.x, u.y, u.z, u.w}, y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = bf2f(f2bf(silu(bf2f(f2bf(g4[i]))))) * bf2f(f2bf(u4[i]));
    uint2 o;
    o.x = pack2(y[0], y[1]);
    o.y = pack2(y[2], y[3]);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * ldo + b * 16 + j) = o;
  }
}

// residual = bf16(residual + bf16(sum_s partial[s])); x = rmsnorm(residual) * w.
// One row per workgroup of H/4 (<= 1024) threads, PER float4 column groups per thread; the S
// slab loads of a group are independent and issued back to back (latency, not bandwidth, is
// what a 64-row reduction fights).
template <int PER>
__global__ void __launch_bounds__(1024) splitk_add_rmsnorm_kernel(bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
                                                                  const float* __restrict__ partial,
                                                                  const bf16_t* __restrict__ w, int S, int M, int H,
                                                                  float eps) {
  __shared__ float red[16];
  const int m = blockIdx.x;
  float v[PER][4];
  float ss = 0.f;
  bf16_t* res = residual + static_cast<int64_t>(m) * H;
  const int64_t slab = static_cast<int64_t>(M) * H;
  const float* base = partial + static_cast<int64_t>(m) * H;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    float4 acc = *reinterpret_cast<const float4*>(base + c);
#pragma unroll 8
    for (int s = 1; s < S; ++s) {
      const float4 p = *reinterpret_cast<const float4*>(base + s * slab + c);
      acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
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
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    const uint2 ww = *reinterpret_cast<const uint2*>(w + c);
    float y[4];
    y[0] = bf2f(f2bf(v[i][0] * rinv)) * bf2f(static_cast<bf16_t>(ww.x & 0xffff));
    y[1] = bf2f(f2bf(v[i][1] * rinv)) * bf2f(static_cast<bf16_t>(ww.x >> 16));
    y[2] = bf2f(f2bf(v[i][2] * rinv)) * bf2f(static_cast<bf16_t>(ww.y & 0xffff));
    y[3] = bf2f(f2bf(v[i][3] * rinv)) * bf2f(static_cast<bf16_t>(ww.y >> 16));
    uint2 o;
    o.x = pack2(y[0], y[1]);
    o.y = pack2(y[2], y[3]);
    *reinterpret_cast<uint2*>(xo + c) = o;
  }
}

// Split-K QKV epilogue fused with RoPE and the paged KV write: per token, sum the S fp32 slabs
// of the fused q|k|v projection, round to bf16 (the unfused GEMM output), rotate q and k
// (neox, fp32 cos|sin table), write q to q_out [M, nq*128], k to the K cache and v to the
// transposed V cache (slot < 0: padding row, nothing cached).  Replaces reduce + rope_and_cache.
__global__ void __launch_bounds__(256) qkv_reduce_rope_cache_kernel(
    bf16_t* __restrict__ q_out, const float* __restrict__ partial, int S, int M, int nq, int nkv,
    const int* __restrict__ positions, const float* __restrict__ cos_sin, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ slots, int bs) {
  const int m = blockIdx.x;
  const int N = (nq + 2 * nkv) * 128;
  const int64_t slab = static_cast<int64_t>(M) * N;
  const float* base = partial + static_cast<int64_t>(m) * N;
  const int pos = positions[m];
  const int slot = slots[m];
  const float* cs = cos_sin + static_cast<int64_t>(pos) * 128;
  const int n_rot = (nq + nkv) * 16;  // (head, 4-pair group)
  const int n_items = n_rot + nkv * 32;
  for (int it = threadIdx.x; it < n_items; it += blockDim.x) {
    if (it < n_rot) {
      const int h = it >> 4, j = (it & 15) * 4;
      const int c = h * 128 + j;
      float4 a = *reinterpret_cast<const float4*>(base + c);
      float4 b = *reinterpret_cast<const float4*>(base + c + 64);
      for (int s = 1; s < S; ++s) {
        const float4 pa = *reinterpret_cast<const float4*>(base + s * slab + c);
        const float4 pb = *reinterpret_cast<const float4*>(base + s * slab + c + 64);
        a.x += pa.x; a.y += pa.y; a.z += pa.z; a.w += pa.w;
        b.x += pb.x; b.y += pb.y; b.z += pb.z; b.w += pb.w;
      }
      const float av[4] = {bf2f(f2bf(a.x)), bf2f(f2bf(a.y)), bf2f(f2bf(a.z)), bf2f(f2bf(a.w))};
      const float bv[4] = {bf2f(f2bf(b.x)), bf2f(f2bf(b.y)), bf2f(f2bf(b.z)), bf2f(f2bf(b.w))};
      const float4 co = *reinterpret_cast<const float4*>(cs + j);
      const float4 si = *reinterpret_cast<const float4*>(cs + 64 + j);
      const float cc[4] = {co.x, co.y, co.z, co.w}, ss[4] = {si.x, si.y, si.z, si.w};
      float ra[4], rb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ra[q] = av[q] * cc[q] - bv[q] * ss[q];
        rb[q] = bv[q] * cc[q] + av[q] * ss[q];
      }
      uint2 va, vb;
      va.x = pack2(ra[0], ra[1]);
      va.y = pack2(ra[2], ra[3]);
      vb.x = pack2(rb[0], rb[1]);
      vb.y = pack2(rb[2], rb[3]);
      if (h < nq) {
        bf16_t* o = q_out + static_cast<int64_t>(m) * nq * 128 + h * 128 + j;
        *reinterpret_cast<uint2*>(o) = va;
        *reinterpret_cast<uint2*>(o + 64) = vb;
      } else if (slot >= 0) {
        bf16_t* d = kc + ((static_cast<int64_t>(slot / bs) * nkv + (h - nq)) * bs + slot % bs) * 128 + j;
        *reinterpret_cast<uint2*>(d) = va;
        *reinterpret_cast<uint2*>(d + 64) = vb;
      }
    } else if (slot >= 0) {
      const int u = it - n_rot;
      const int kh = u >> 5, d0 = (u & 31) * 4;
      const int c = (nq + nkv) * 128 + kh * 128 + d0;
      float4 a = *reinterpret_cast<const float4*>(base + c);
      for (int s = 1; s < S; ++s) {
        const float4 pa = *reinterpret_cast<const float4*>(base + s * slab + c);
        a.x += pa.x; a.y += pa.y; a.z += pa.z; a.w += pa.w;
      }
      const float av[4] = {a.x, a.y, a.z, a.w};
      bf16_t* d = vc + ((static_cast<int64_t>(slot / bs) * nkv + kh) * 128 + d0) * bs + slot % bs;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q * bs] = f2bf(av[q]);
    }
  }
}

template <int MODE, int D, bool PK>
int launch(int MT, bf16_t* out, float* partial, const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldo,
           int S, hipStream_t stream) {
  const int n_blocks = N / 128;
  const int grid = n_blocks * S;
  switch (MT) {
    case 1: skinny_gemm_kernel<1, MODE, D, PK><<<grid, 256, 0, stream>>>(out, partial, A, W, M, N, K, lda, ldo, S, n_blocks); break;
    case 2: skinny_gemm_kernel<2, MODE, D, PK><<<grid, 256, 0, stream>>>(out, partial, A, W, M, N, K, lda, ldo, S, n_blocks); break;
    case 3: skinny_gemm_kernel<3, MODE, D, PK><<<grid, 256, 0, stream>>>(out, partial, A, W, M, N, K, lda, ldo, S, n_blocks); break;
    case 4: skinny_gemm_kernel<4, MODE, D, PK><<<grid, 256, 0, stream>>>(out, partial, A, W, M, N, K, lda, ldo, S, n_blocks); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

}  // namespace

// mode 0: out bf16 [M, ldo] (S must be 1); 1: partial fp32 [S, M, N]; 2: SiLU-mul of interleaved
// gate/up rows -> out bf16 [M, N/2] (S must be 1).  Requires M <= 64, N % 32 == 0, K % (128 S) == 0.
PK_EXPORT int pk_skinny_gemm(void* out, void* partial, const void* A, const void* W, int M, int N, int K, int lda,
                             int ldo, int S, int mode, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || N % 128 || S < 1 || K % (kKC * S) || lda % 8) return -1;
  const int MT = (M + 15) / 16;
  auto o = static_cast<bf16_t*>(out);
  auto p = static_cast<float*>(partial);
  auto a = static_cast<const bf16_t*>(A);
  auto w = static_cast<const bf16_t*>(W);
  const bool deep = (mode & 8) != 0;     // bit 3: 4-step W register ring instead of 2
  const bool packed = (mode & 16) != 0;  // bit 4: W in fragment-packed layout (pk_pack_weight)
  auto go = [&](auto mode_c) -> int {
    constexpr int MD = decltype(mode_c)::value;
    const int s_ = MD == kPartial ? S : 1;
    if (packed) return deep ? launch<MD, 4, true>(MT, o, p, a, w, M, N, K, lda, ldo, s_, stream)
                            : launch<MD, 2, true>(MT, o, p, a, w, M, N, K, lda, ldo, s_, stream);
    return deep ? launch<MD, 4, false>(MT, o, p, a, w, M, N, K, lda, ldo, s_, stream)
                : launch<MD, 2, false>(MT, o, p, a, w, M, N, K, lda, ldo, s_, stream);
  };
  switch (mode & 7) {
    case kBF16:
      if (S != 1) return -1;
      return go(std::integral_constant<int, kBF16>{});
    case kPartial:
      return go(std::integral_constant<int, kPartial>{});
    case kSiluMul:
      if (S != 1) return -1;
      return go(std::integral_constant<int, kSiluMul>{});
    default: return -1;
  }
}

PK_EXPORT int pk_splitk_reduce(void* out, const void* partial, int S, int M, int N, int ldo, int silu,
                               hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 4) return -1;
  dim3 grid((N / 4 + 255) / 256, M);
  if (silu)
    splitk_reduce_kernel<true><<<grid, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const float*>(partial), S, M, N, ldo);
  else
    splitk_reduce_kernel<false><<<grid, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const float*>(partial), S, M, N, ldo);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_splitk_add_rmsnorm(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                                    float eps, hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % 1024 || H > 8192) return -1;
  auto xx = static_cast<bf16_t*>(x);
  auto rr = static_cast<bf16_t*>(residual);
  auto pp = static_cast<const float*>(partial);
  auto ww = static_cast<const bf16_t*>(w);
  const int threads = H / 4 > 1024 ? 1024 : H / 4;
  switch (H / (4 * threads)) {
    case 1: splitk_add_rmsnorm_kernel<1><<<M, threads, 0, stream>>>(xx, rr, pp, ww, S, M, H, eps); break;
    case 2: splitk_add_rmsnorm_kernel<2><<<M, threads, 0, stream>>>(xx, rr, pp, ww, S, M, H, eps); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_qkv_reduce_rope_cache(void* q_out, const void* partial, int S, int M, int nq, int nkv,
                                       const void* positions, const void* cos_sin, void* k_cache, void* v_cache,
                                       const void* slots, int bs, hipStream_t stream) {
  if (M <= 0) return 0;
  if (bs % 8) return -1;
  qkv_reduce_rope_cache_kernel<<<M, 256, 0, stream>>>(
      static_cast<bf16_t*>(q_out), static_cast<const float*>(partial), S, M, nq, nkv,
      static_cast<const int*>(positions), static_cast<const float*>(cos_sin), static_cast<bf16_t*>(k_cache),
      static_cast<bf16_t*>(v_cache), static_cast<const int*>(slots), bs);
  return PK_CHECK_LAUNCH();
}
