// Shared device helpers for the gfx950 (CDNA4) kernels.
// Wave = 64 lanes; bf16 is moved as 16-byte vectors (8 elements) per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define PK_EXPORT extern "C" __attribute__((visibility("default")))

namespace pk {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // raw bits; converted explicitly
typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(4))) float f32x4;    // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;  // 16-byte raw vector
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;  // MFMA bf16 operand (16x16x32)

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// round-to-nearest-even f32 -> bf16: gfx950's v_cvt_pk_bf16_f32 (one VALU op per pair, no
// branches; a software RNE with a NaN test compiles to exec-mask branches per element)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, static_cast<__bf16>(f)); }

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2(f[2 * i], f[2 * i + 1]);
  return r;
}

// ---- paged K-cache layout --------------------------------------------------------------
// A K-cache block of one KV head ([bs][128] bf16, bs a multiple of 32) is stored as bs/32
// fragment-native 8 KiB tiles: inside a 32-token tile, element (token k, dim d) sits at
//     ((t * 4 + kk) * 64 + lane) * 8 + j,   t = (k >> 2) & 1, kk = (d >> 3) & 3, j = d & 7,
//     lane = 16 * (d >> 5) + 4 * (k >> 3) + (k & 3)
// -- the order in which the attention kernels' S^T = K.Q^T MFMA A-fragments (key tile t,
// k-step kk) are held by the 64 lanes (attention.hip load_kv).  Every fragment load of a wave is
// then one contiguous 1 KiB (eight full 128-B lines) instead of 16 rows x 64 B, so the decode
// stream reads whole lines (tools/attn_layout_lab.py at 384 keys: 20.9 -> 20.1 us, 17.9 us with
// non-temporal loads -- which lose in the captured decode step, so they are off).
// Writers scatter one token's 128 dims with 8-dim (16-byte) granules; RoPE halves d and d+64
// stay 16-byte aligned.
// V cache, fragment-native like K: per 32-token tile, [d / 16][key / 8][d % 16][key % 8], so the
// 8 consecutive keys of one channel (a PV MFMA operand) are 16 contiguous bytes, a wave's 64
// operand loads of one 16-channel tile are one contiguous KiB, and a decode token's 128 channels
// land in 16 cache lines (8 runs of 16 two-byte stores 16 bytes apart) instead of 128 separate
// 64-byte V^T rows (those per-token stores cost 2.6-2.9 us per decode-attention launch at 384-512
// keys, profiles/r2_decode_ab.txt).
__host__ __device__ __forceinline__ int vcache_off(int k_in_block, int d) {
  const int k = k_in_block & 31;
  return (k_in_block >> 5) * 4096 + ((((d >> 4) << 2) + (k >> 3)) * 16 + (d & 15)) * 8 + (k & 7);
}

__host__ __device__ __forceinline__ int kcache_off(int k_in_block, int d) {
  const int k = k_in_block & 31;
  const int lane = 16 * (d >> 5) + 4 * (k >> 3) + (k & 3);
  return (k_in_block >> 5) * 4096 + ((((k >> 2) & 1) * 4 + ((d >> 3) & 3)) * 64 + lane) * 8 + (d & 7);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (<= 16 waves). `red` needs 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = lane < nw ? red[lane] : 0.f;
  t = wave_sum(t);
  __syncthreads();
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = lane < nw ? red[lane] : -INFINITY;
  t = wave_max(t);
  __syncthreads();
  return t;
}

}  // namespace pk

#define PK_CHECK_LAUNCH() (static_cast<int>(hipGetLastError()))

// Device-side bounds checks, compiled in only for debug builds (POLYKEY_DEBUG_KERNELS=1 →
// -DPK_DEBUG): a failing check prints the condition and traps the kernel, so an out-of-range
// block table / slot / token id is reported at its source instead of corrupting the KV cache.
#ifdef PK_DEBUG
#include <cassert>
#define PK_DEVICE_ASSERT(c) assert(c)
#else
#define PK_DEVICE_ASSERT(c) ((void)0)
#endif
