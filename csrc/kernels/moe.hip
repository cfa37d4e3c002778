// Mixture-of-experts kernels for gfx950 (Mixtral-8x7B: E = 8 experts, top-2).
//
//   topk_softmax   router logits [T, E] -> top-k expert ids + renormalised weights (fp32)
//   align          stable counting sort of the T*k (token, slot) pairs by expert: per-expert
//                  offsets, sorted order and its inverse (deterministic: wave ballots + prefix
//                  over waves, no atomics on positions); experts outside [e_lo, e_hi) (other
//                  EP ranks) are dropped
//   permute        gather token rows into expert-contiguous order
//   grouped GEMM   decode-sized grouped "skinny" GEMM: one wave per (expert, 32 weight rows,
//                  k-split); a wave whose expert received no tokens exits before reading a
//                  byte of that expert's weights, so a decode step streams only the experts in
//                  use (the same MFMA tiling as gemm_skinny.hip, with the fused SiLU epilogue)
//   unpermute      weighted top-k combine back to token order (fp32 accumulate)
#include "common.h"

using namespace pk;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }
__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// one thread per token, E <= 64
__global__ void topk_softmax_kernel(const bf16_t* __restrict__ logits, int stride, int T, int E, int k, int renorm,
                                    int* __restrict__ ids, float* __restrict__ w) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const bf16_t* l = logits + static_cast<int64_t>(t) * stride;
  float v[64];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    v[e] = bf2f(l[e]);
    mx = fmaxf(mx, v[e]);
  }
  float sum = 0.f;
  for (int e = 0; e < E; ++e) {
    v[e] = __expf(v[e] - mx);
    sum += v[e];
  }
  unsigned long long taken = 0ull;
  float wsum = 0.f;
  for (int j = 0; j < k; ++j) {
    int best = 0;
    float bv = -1.f;
    for (int e = 0; e < E; ++e)
      if (!((taken >> e) & 1ull) && v[e] > bv) {
        bv = v[e];
        best = e;
      }
    taken |= 1ull << best;
    ids[t * k + j] = best;
    w[t * k + j] = bv / sum;
    wsum += bv / sum;
  }
  if (renorm)
    for (int j = 0; j < k; ++j) w[t * k + j] /= wsum;
}

// Stable counting sort by expert; run by ONE workgroup of 1024 threads; n = T*k slots; E <= 64.
__device__ void align_body(const int* __restrict__ ids, int n, int E, int e_lo, int e_hi, int* __restrict__ offsets,
                           int* __restrict__ sorted, int* __restrict__ inv) {
  __shared__ int counts[64];
  __shared__ int cursor[64];
  __shared__ int wave_cnt[16][64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid < 64) counts[tid] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += 1024) {
    const int e = ids[i];
    if (e >= e_lo && e < e_hi) atomicAdd(&counts[e - e_lo], 1);
  }
  __syncthreads();
  const int El = e_hi - e_lo;
  if (tid == 0) {
    int run = 0;
    for (int e = 0; e < El; ++e) {
      offsets[e] = run;
      cursor[e] = run;
      run += counts[e];
    }
    offsets[El] = run;
  }
  __syncthreads();
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const int e = i < n ? ids[i] - e_lo : -1;
    const bool mine = i < n && e >= 0 && e < El;
    int rank = 0;
    for (int x = 0; x < El; ++x) {
      const unsigned long long m = __ballot(mine && e == x);
      if (lane == 0) wave_cnt[wid][x] = __popcll(m);
      if (mine && e == x) rank = __popcll(m & lt);
    }
    __syncthreads();
    if (tid < El) {  // exclusive prefix over waves for expert tid
      int run = cursor[tid];
      for (int w2 = 0; w2 < 16; ++w2) {
        const int c = wave_cnt[w2][tid];
        wave_cnt[w2][tid] = run;
        run += c;
      }
      cursor[tid] = run;
    }
    __syncthreads();
    if (i < n) {
      if (mine) {
        const int pos = wave_cnt[wid][e] + rank;
        sorted[pos] = i;
        inv[i] = pos;
      } else {
        inv[i] = -1;
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(1024) align_kernel(const int* __restrict__ ids, int n, int E, int e_lo, int e_hi,
                                                     int* __restrict__ offsets, int* __restrict__ sorted,
                                                     int* __restrict__ inv) {
  align_body(ids, n, E, e_lo, e_hi, offsets, sorted, inv);
}

// MoE combine fused with the residual add and the next RMSNorm (one workgroup per token):
//   y = bf16(sum_j w[t,j] * moe_out[inv[t*k+j]])   (what unpermute would store)
//   residual[t] = bf16(residual[t] + y);  x[t] = rmsnorm(residual[t]) * norm_w
template <int PER>
__global__ void __launch_bounds__(1024) combine_add_rmsnorm_kernel(bf16_t* __restrict__ xo, bf16_t* __restrict__ residual,
                                                                   const bf16_t* __restrict__ y,
                                                                   const int* __restrict__ inv,
                                                                   const float* __restrict__ w,
                                                                   const bf16_t* __restrict__ nw, int k, int H,
                                                                   float eps) {
  __shared__ float red[16];
  const int t = blockIdx.x;
  float v[PER][4];
  float ss = 0.f;
  bf16_t* res = residual + static_cast<int64_t>(t) * H;
  uint2 wpre[PER];  // the norm weight, requested before the expert rows (independent of them)
#pragma unroll
  for (int i = 0; i < PER; ++i) wpre[i] = *reinterpret_cast<const uint2*>(nw + 4 * (threadIdx.x + i * blockDim.x));
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int p = inv[t * k + j];
      if (p < 0) continue;
      const uint2 yy = *reinterpret_cast<const uint2*>(y + static_cast<int64_t>(p) * H + c);
      const float ww = w[t * k + j];
      acc[0] += ww * bf2f(static_cast<bf16_t>(yy.x & 0xffff));
      acc[1] += ww * bf2f(static_cast<bf16_t>(yy.x >> 16));
      acc[2] += ww * bf2f(static_cast<bf16_t>(yy.y & 0xffff));
      acc[3] += ww * bf2f(static_cast<bf16_t>(yy.y >> 16));
    }
    const uint2 rr = *reinterpret_cast<const uint2*>(res + c);
    v[i][0] = bf2f(f2bf(bf2f(f2bf(acc[0])) + bf2f(static_cast<bf16_t>(rr.x & 0xffff))));
    v[i][1] = bf2f(f2bf(bf2f(f2bf(acc[1])) + bf2f(static_cast<bf16_t>(rr.x >> 16))));
    v[i][2] = bf2f(f2bf(bf2f(f2bf(acc[2])) + bf2f(static_cast<bf16_t>(rr.y & 0xffff))));
    v[i][3] = bf2f(f2bf(bf2f(f2bf(acc[3])) + bf2f(static_cast<bf16_t>(rr.y >> 16))));
    uint2 o;
    o.x = pack2(v[i][0], v[i][1]);
    o.y = pack2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(res + c) = o;
    ss += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  }
  const float rinv = rsqrtf(block_sum(ss, red) / H + eps);
  bf16_t* xr = xo + static_cast<int64_t>(t) * H;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    const uint2 ww = wpre[i];
    float o4[4];
    o4[0] = bf2f(f2bf(v[i][0] * rinv)) * bf2f(static_cast<bf16_t>(ww.x & 0xffff));
    o4[1] = bf2f(f2bf(v[i][1] * rinv)) * bf2f(static_cast<bf16_t>(ww.x >> 16));
    o4[2] = bf2f(f2bf(v[i][2] * rinv)) * bf2f(static_cast<bf16_t>(ww.y & 0xffff));
    o4[3] = bf2f(f2bf(v[i][3] * rinv)) * bf2f(static_cast<bf16_t>(ww.y >> 16));
    uint2 o;
    o.x = pack2(o4[0], o4[1]);
    o.y = pack2(o4[2], o4[3]);
    *reinterpret_cast<uint2*>(xr + c) = o;
  }
}

// out[p] = x[sorted[p] / k]   (grid: n rows; H/8 vectors per row)
__global__ void permute_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x, const int* __restrict__ sorted,
                               const int* __restrict__ offsets, int E_local, int k, int H) {
  const int p = blockIdx.x;
  if (p >= offsets[E_local]) return;
  const int src = sorted[p] / k;
  const u32x4* s = reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(src) * H);
  u32x4* d = reinterpret_cast<u32x4*>(out + static_cast<int64_t>(p) * H);
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) d[v] = s[v];
}

// out[t] = sum_j w[t,j] * y[inv[t*k+j]]   (inv < 0 -> expert on another EP rank)
__global__ void unpermute_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ y, const int* __restrict__ inv,
                                 const float* __restrict__ w, int k, int H) {
  const int t = blockIdx.x;
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int p = inv[t * k + j];
      if (p < 0) continue;
      float f[8];
      unpack8(reinterpret_cast<const u32x4*>(y + static_cast<int64_t>(p) * H)[v], f);
      const float ww = w[t * k + j];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += ww * f[q];
    }
    reinterpret_cast<u32x4*>(out + static_cast<int64_t>(t) * H)[v] = pack8(acc);
  }
}

// Combine from split-K slabs of the w2 GEMM: y[p] = bf16(sum_s partial[s][p]) (the GEMM output
// the unsplit kernel would store), out[t] = sum_j w[t,j] * y[inv[t,j]].  Saves the separate
// reduce pass over [S, R, H].
__global__ void unpermute_partial_kernel(bf16_t* __restrict__ out, const float* __restrict__ partial, int S, int R,
                                         const int* __restrict__ inv, const float* __restrict__ w, int k, int H) {
  const int t = blockIdx.x;
  const int64_t slab = static_cast<int64_t>(R) * H;
  for (int v = threadIdx.x; v < H / 4; v += blockDim.x) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int p = inv[t * k + j];
      if (p < 0) continue;
      const float* src = partial + static_cast<int64_t>(p) * H + 4 * v;
      float4 y = *reinterpret_cast<const float4*>(src);
      for (int q = 1; q < S; ++q) {
        const float4 z = *reinterpret_cast<const float4*>(src + q * slab);
        y.x += z.x; y.y += z.y; y.z += z.z; y.w += z.w;
      }
      const float ww = w[t * k + j];
      acc[0] += ww * bf2f(f2bf(y.x));
      acc[1] += ww * bf2f(f2bf(y.y));
      acc[2] += ww * bf2f(f2bf(y.z));
      acc[3] += ww * bf2f(f2bf(y.w));
    }
    uint2 o;
    o.x = pack2(acc[0], acc[1]);
    o.y = pack2(acc[2], acc[3]);
    reinterpret_cast<uint2*>(out + static_cast<int64_t>(t) * H)[v] = o;
  }
}

// Grouped skinny GEMM.  Expert e's rows of A are [offsets[e], offsets[e+1]) (<= 16*MT rows);
// W is [E_local, N, K].  MODE 0: bf16 out [rows, N]; MODE 2: SiLU-mul of interleaved gate/up
// rows -> out [rows, N/2].  grid: (E_local * n_blocks * S / 4), block 256.
template <int MT, int MODE>
__global__ void __launch_bounds__(256) moe_gemm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ A,
                                                       const bf16_t* __restrict__ W, const int* __restrict__ offsets,
                                                       int N, int K, int ldo, int n_blocks, int E_local) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wave >= n_blocks * E_local) return;
  const int e = wave / n_blocks, nb = wave % n_blocks;
  const int row0 = offsets[e], cnt = offsets[e + 1] - row0;
  if (cnt <= 0) return;  // no tokens: this expert's weights are never read
  const int r = lane & 15, g = lane >> 4;
  const int n0 = nb * 32;
  const bf16_t* We = W + static_cast<int64_t>(e) * N * K;
  const bf16_t* wp[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) wp[t] = We + static_cast<int64_t>(n0 + 16 * t + r) * K + 32 * g;
  const bf16_t* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ap[mt] = A + static_cast<int64_t>(row0 + min(16 * mt + r, cnt - 1)) * K + 32 * g;
  f32x4 acc[2][MT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8_t w[2][4], wn[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) w[t][s] = ld8(wp[t] + 8 * s);
  for (int k = 0; k < K; k += 128) {
    const bool more = k + 128 < K;
    if (more) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) wn[t][s] = ld8(wp[t] + k + 128 + 8 * s);
    }
    bf16x8_t a[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int s = 0; s < 4; ++s) a[mt][s] = ld8(ap[mt] + k + 8 * s);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][s], a[mt][s], acc[t][mt], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) w[t][s] = wn[t][s];
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = 16 * mt + r;
    if (m >= cnt) continue;
    if (MODE == 0) {
      bf16_t* o = out + static_cast<int64_t>(row0 + m) * ldo + n0 + 4 * g;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        uint2 v;
        v.x = pack2(acc[t][mt][0], acc[t][mt][1]);
        v.y = pack2(acc[t][mt][2], acc[t][mt][3]);
        *reinterpret_cast<uint2*>(o + 16 * t) = v;
      }
    } else {
      bf16_t* o = out + static_cast<int64_t>(row0 + m) * ldo + (n0 >> 1) + 4 * g;
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = bf2f(f2bf(silu(bf2f(f2bf(acc[0][mt][i]))))) * bf2f(f2bf(acc[1][mt][i]));
      uint2 v;
      v.x = pack2(y[0], y[1]);
      v.y = pack2(y[2], y[3]);
      *reinterpret_cast<uint2*>(o) = v;
    }
  }
}

template <int MODE>
int launch_moe(int MT, bf16_t* out, const bf16_t* A, const bf16_t* W, const int* offsets, int N, int K, int ldo,
               int E_local, hipStream_t s) {
  const int nb = N / 32;
  const int grid = (nb * E_local + 3) / 4;
  switch (MT) {
    case 1: moe_gemm_kernel<1, MODE><<<grid, 256, 0, s>>>(out, A, W, offsets, N, K, ldo, nb, E_local); break;
    case 2: moe_gemm_kernel<2, MODE><<<grid, 256, 0, s>>>(out, A, W, offsets, N, K, ldo, nb, E_local); break;
    case 3: moe_gemm_kernel<3, MODE><<<grid, 256, 0, s>>>(out, A, W, offsets, N, K, ldo, nb, E_local); break;
    case 4: moe_gemm_kernel<4, MODE><<<grid, 256, 0, s>>>(out, A, W, offsets, N, K, ldo, nb, E_local); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

}  // namespace

PK_EXPORT int pk_moe_topk_softmax(void* ids, void* weights, const void* logits, int T, int E, int k, int stride,
                                  int renorm, hipStream_t stream) {
  if (T <= 0) return 0;
  if (E > 64 || k > E) return -1;
  topk_softmax_kernel<<<(T + 255) / 256, 256, 0, stream>>>(static_cast<const bf16_t*>(logits), stride, T, E, k, renorm,
                                                           static_cast<int*>(ids), static_cast<float*>(weights));
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_moe_align(const void* ids, void* offsets, void* sorted, void* inv, int n, int E, int e_lo, int e_hi,
                           hipStream_t stream) {
  if (e_hi - e_lo > 64 || e_hi <= e_lo) return -1;
  align_kernel<<<1, 1024, 0, stream>>>(static_cast<const int*>(ids), n, E, e_lo, e_hi, static_cast<int*>(offsets),
                                       static_cast<int*>(sorted), static_cast<int*>(inv));
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_moe_permute(void* out, const void* x, const void* sorted, const void* offsets, int n, int E_local,
                             int k, int H, hipStream_t stream) {
  if (n <= 0) return 0;
  if (H % 8) return -1;
  permute_kernel<<<n, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const bf16_t*>(x),
                                        static_cast<const int*>(sorted), static_cast<const int*>(offsets), E_local, k, H);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_moe_unpermute(void* out, const void* y, const void* inv, const void* w, int T, int k, int H,
                               hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return -1;
  unpermute_kernel<<<T, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const bf16_t*>(y),
                                          static_cast<const int*>(inv), static_cast<const float*>(w), k, H);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_moe_unpermute_partial(void* out, const void* partial, int S, int R, const void* inv, const void* w,
                                       int T, int k, int H, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 4 || S < 1) return -1;
  unpermute_partial_kernel<<<T, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const float*>(partial), S, R,
                                                  static_cast<const int*>(inv), static_cast<const float*>(w), k, H);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_moe_combine_add_rmsnorm(void* x, void* residual, const void* y, const void* inv, const void* w,
                                         const void* norm_w, int T, int k, int H, float eps, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 1024 || H > 8192) return -1;
  const int threads = H / 4 > 1024 ? 1024 : H / 4;
  auto xx = static_cast<bf16_t*>(x);
  auto rr = static_cast<bf16_t*>(residual);
  auto yy = static_cast<const bf16_t*>(y);
  auto ii = static_cast<const int*>(inv);
  auto ww = static_cast<const float*>(w);
  auto nn = static_cast<const bf16_t*>(norm_w);
  switch (H / (4 * threads)) {
    case 1: combine_add_rmsnorm_kernel<1><<<T, threads, 0, stream>>>(xx, rr, yy, ii, ww, nn, k, H, eps); break;
    case 2: combine_add_rmsnorm_kernel<2><<<T, threads, 0, stream>>>(xx, rr, yy, ii, ww, nn, k, H, eps); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

// max_rows: upper bound on rows of any expert (<= 64).  mode 0: bf16; 2: SiLU-mul interleaved.
PK_EXPORT int pk_moe_gemm(void* out, const void* A, const void* W, const void* offsets, int max_rows, int N, int K,
                          int ldo, int E_local, int mode, hipStream_t stream) {
  if (max_rows <= 0) return 0;
  if (max_rows > 64 || N % 32 || K % 128) return -1;
  const int MT = (max_rows + 15) / 16;
  auto o = static_cast<bf16_t*>(out);
  auto a = static_cast<const bf16_t*>(A);
  auto w = static_cast<const bf16_t*>(W);
  auto off = static_cast<const int*>(offsets);
  if (mode == 0) return launch_moe<0>(MT, o, a, w, off, N, K, ldo, E_local, stream);
  if (mode == 2) return launch_moe<2>(MT, o, a, w, off, N, K, ldo, E_local, stream);
  return -1;
}
