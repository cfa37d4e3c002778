// Token sampler for gfx950: greedy / temperature + top-k + top-p + min-p + seeded Gumbel-max.
//
// One 1024-thread workgroup per row (vocab up to ~256k), reading the row with 16-byte
// vectors; every pass after the first is served from L2 (a 128k-vocab bf16 row is 256 KB).
//  * greedy (temperature <= 0): one argmax pass (ties -> lowest index).
//  * top-k: exact k-th largest logit by 4-pass radix select on order-preserving uint32 keys
//    (8-bit digits, 256-bin LDS histogram; the digit is found by a 64-lane suffix scan).
//  * top-p: the same radix walk with *probability mass* per bin instead of counts, over the
//    top-k survivors: finds the smallest logit v* whose upper set holds >= p of the mass.
//  * min-p: x >= max + log(min_p) (in temperature-scaled logit space).
//  * sample: argmax over survivors of x/T + Gumbel(u), u = counter-based hash of
//    (seed, offset, token) -> bit-exact reproducible (see ops/reference.py philox_uniform).
// Ties at a threshold are kept (threshold semantics), which matches the reference mask.
#include "common.h"

using namespace pk;

namespace {

constexpr int kThreads = 1024;

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t row_hash(uint32_t seed, uint32_t offset) {
  uint32_t h = seed * 0x9E3779B1u + 0x7F4A7C15u;
  h ^= offset + 0x85EBCA6Bu + (h << 6) + (h >> 2);
  return fmix32(h);
}

__device__ __forceinline__ float uniform01(uint32_t rh, uint32_t idx) {
  const uint32_t x = fmix32(rh ^ (idx * 0xC2B2AE35u));
  return (static_cast<float>(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float from_okey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <typename T>
struct Row;

template <>
struct Row<bf16_t> {
  static __device__ __forceinline__ void load8(const bf16_t* p, int v, float* out) {
    unpack8(reinterpret_cast<const u32x4*>(p)[v], out);
  }
};

template <>
struct Row<float> {
  static __device__ __forceinline__ void load8(const float* p, int v, float* out) {
    const float4* q = reinterpret_cast<const float4*>(p) + 2 * v;
    float4 a = q[0], b = q[1];
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
    out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
  }
};

struct Smem {
  float fhist[256];
  uint32_t uhist[256];
  float red[16];
  uint32_t ured[16];
  int ired[16];
  uint32_t sel_digit;
  float sel_f;
};

// Wave 0 finds the digit d (scanning 255 -> 0) where the running total first reaches `need`;
// returns (d, total of bins above d).  Other waves wait at the barrier.
template <typename V>
__device__ __forceinline__ void select_digit(const V* hist, V need, uint32_t* out_digit, V* out_above) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    // lane handles bins 255-4*lane .. 252-4*lane (descending)
    V b[4];
    V s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      b[j] = hist[255 - 4 * lane - j];
      s += b[j];
    }
    // inclusive prefix over lanes (descending bins)
    V incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      V t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const V excl = incl - s;
    const bool hit = excl < need && incl >= need;
    const unsigned long long mask = __ballot(hit);
    const int src = mask ? __ffsll(static_cast<long long>(mask)) - 1 : 63;
    if (lane == src) {
      V acc = excl;
      int d = 252 - 4 * lane;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (acc + b[j] >= need) {
          d = 255 - 4 * lane - j;
          break;
        }
        acc += b[j];
      }
      *out_digit = static_cast<uint32_t>(d);
      *out_above = acc;
    }
  }
  __syncthreads();
}

template <typename T>
__global__ void __launch_bounds__(kThreads) sample_kernel(int* __restrict__ out, const T* __restrict__ logits,
                                                          int64_t stride, int V, const float* __restrict__ temperature,
                                                          const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                          const float* __restrict__ min_p, const int* __restrict__ seeds,
                                                          const int* __restrict__ offsets) {
  __shared__ Smem sm;
  __shared__ float above_f;
  __shared__ uint32_t above_u;
  const int row = blockIdx.x;
  const T* x = logits + row * stride;
  const int nv = V / 8;
  const float temp = temperature ? temperature[row] : 0.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  // ---- pass 1: max (and argmax for greedy)
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int v = threadIdx.x; v < nv; v += kThreads) {
    float f[8];
    Row<T>::load8(x, v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (f[j] > best) {
        best = f[j];
        besti = 8 * v + j;
      }
  }
  // block argmax: (value desc, index asc)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ov > best || (ov == best && oi < besti)) {
      best = ov;
      besti = oi;
    }
  }
  if (lane == 0) {
    sm.red[wid] = best;
    sm.ired[wid] = besti;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float b = lane < kThreads / 64 ? sm.red[lane] : -INFINITY;
    int bi = lane < kThreads / 64 ? sm.ired[lane] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(b, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > b || (ov == b && oi < bi)) {
        b = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      sm.red[0] = b;
      sm.ired[0] = bi;
    }
  }
  __syncthreads();
  const float xmax = sm.red[0];
  if (!(temp > 0.f)) {
    if (threadIdx.x == 0) out[row] = sm.ired[0];
    return;
  }
  const float inv_t = 1.f / temp;
  const float m = xmax * inv_t;
  float thr = -INFINITY;  // survivors: x*inv_t >= thr

  // ---- top-k: radix select of the k-th largest scaled logit
  const int k = top_k ? top_k[row] : 0;
  if (k > 0 && k < V) {
    uint32_t prefix = 0, pmask = 0, need = static_cast<uint32_t>(k);
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = threadIdx.x; i < 256; i += kThreads) sm.uhist[i] = 0;
      __syncthreads();
      for (int v = threadIdx.x; v < nv; v += kThreads) {
        float f[8];
        Row<T>::load8(x, v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t key = okey(f[j] * inv_t);
          if ((key & pmask) == prefix) atomicAdd(&sm.uhist[(key >> shift) & 255u], 1u);
        }
      }
      __syncthreads();
      select_digit<uint32_t>(sm.uhist, need, &sm.sel_digit, &above_u);
      prefix |= sm.sel_digit << shift;
      pmask |= 255u << shift;
      need -= above_u;
      __syncthreads();
    }
    thr = from_okey(prefix);
  }

  // ---- top-p over the top-k survivors: mass-weighted radix select
  const float p = top_p ? top_p[row] : 1.f;
  if (p > 0.f && p < 1.f) {
    float z = 0.f;
    for (int v = threadIdx.x; v < nv; v += kThreads) {
      float f[8];
      Row<T>::load8(x, v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float s = f[j] * inv_t;
        if (s >= thr) z += __expf(s - m);
      }
    }
    z = block_sum(z, sm.red);
    float need = p * z;
    uint32_t prefix = 0, pmask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = threadIdx.x; i < 256; i += kThreads) sm.fhist[i] = 0.f;
      __syncthreads();
      for (int v = threadIdx.x; v < nv; v += kThreads) {
        float f[8];
        Row<T>::load8(x, v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float s = f[j] * inv_t;
          const uint32_t key = okey(s);
          if (s >= thr && (key & pmask) == prefix) atomicAdd(&sm.fhist[(key >> shift) & 255u], __expf(s - m));
        }
      }
      __syncthreads();
      select_digit<float>(sm.fhist, need, &sm.sel_digit, &above_f);
      prefix |= sm.sel_digit << shift;
      pmask |= 255u << shift;
      need -= above_f;
      __syncthreads();
    }
    thr = fmaxf(thr, from_okey(prefix));
  }

  // ---- min-p
  const float mp = min_p ? min_p[row] : 0.f;
  if (mp > 0.f) thr = fmaxf(thr, m + __logf(mp));
  thr = fminf(thr, m);  // the max token always survives

  // ---- Gumbel-max over survivors
  const uint32_t rh = row_hash(static_cast<uint32_t>(seeds ? seeds[row] : 0), static_cast<uint32_t>(offsets ? offsets[row] : 0));
  float bs = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = threadIdx.x; v < nv; v += kThreads) {
    float f[8];
    Row<T>::load8(x, v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = f[j] * inv_t;
      if (s >= thr) {
        const int idx = 8 * v + j;
        const float u = uniform01(rh, static_cast<uint32_t>(idx));
        const float sc = s - __logf(-__logf(u));
        if (sc > bs || (sc == bs && idx < bi)) {
          bs = sc;
          bi = idx;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bs, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bs || (ov == bs && oi < bi)) {
      bs = ov;
      bi = oi;
    }
  }
  __syncthreads();
  if (lane == 0) {
    sm.red[wid] = bs;
    sm.ired[wid] = bi;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float b = lane < kThreads / 64 ? sm.red[lane] : -INFINITY;
    int bj = lane < kThreads / 64 ? sm.ired[lane] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(b, o, 64);
      const int oi = __shfl_xor(bj, o, 64);
      if (ov > b || (ov == b && oi < bj)) {
        b = ov;
        bj = oi;
      }
    }
    if (lane == 0) out[row] = bj;
  }
}

}  // namespace

// dtype: 0 = bf16 logits, 1 = fp32 logits.  Any of the parameter arrays may be null (defaults:
// temperature 0 -> greedy, top_k 0, top_p 1, min_p 0, seed 0, offset 0).
PK_EXPORT int pk_sample(void* out, const void* logits, const void* temperature, const void* top_k, const void* top_p,
                        const void* min_p, const void* seeds, const void* offsets, void* unused, int B, int V,
                        int stride, int dtype, hipStream_t stream) {
  if (B <= 0) return 0;
  if (V % 8 || stride % 8) return -1;
  if (dtype == 0) {
    sample_kernel<bf16_t><<<B, kThreads, 0, stream>>>(
        static_cast<int*>(out), static_cast<const bf16_t*>(logits), stride, V, static_cast<const float*>(temperature),
        static_cast<const int*>(top_k), static_cast<const float*>(top_p), static_cast<const float*>(min_p),
        static_cast<const int*>(seeds), static_cast<const int*>(offsets));
  } else {
    sample_kernel<float><<<B, kThreads, 0, stream>>>(
        static_cast<int*>(out), static_cast<const float*>(logits), stride, V, static_cast<const float*>(temperature),
        static_cast<const int*>(top_k), static_cast<const float*>(top_p), static_cast<const float*>(min_p),
        static_cast<const int*>(seeds), static_cast<const int*>(offsets));
  }
  return PK_CHECK_LAUNCH();
}
