// Fused RoPE (neox / HF rotate_half) on q and k + paged KV-cache write, gfx950.
//
// Input is the fused QKV projection output [T, (nq + 2*nkv) * 128] (row stride q_stride).
// q and k are rotated in place (fp32 math, fp32 cos/sin table [max_pos, 128] = cos | sin);
// rotated k is also written to the K cache [block][kv_head][slot][128] and v to the
// transposed V cache [block][kv_head][128][block_size].  One workgroup per 32 tokens (below).
// slot_mapping[t] < 0 marks a padding row: it is rotated but nothing is cached.
#include "common.h"

using namespace pk;

namespace {

constexpr int kHD = 128;
constexpr int kHalf = 64;

// One workgroup per 32 consecutive tokens.  q / k: each lane rotates 8 channel pairs (i, i+64)
// of one (token, head) item with two 16-byte loads and stores.  V goes to the transposed cache
// [block][kv][128][bs], where one token's 128 values are 2-byte elements bs apart: when the 32
// tokens fill one aligned 32-slot run of a block (a prefill of whole blocks, the common case),
// each lane gathers one (kv head, channel) row across the 32 tokens (coalesced 2-byte loads
// over the lanes) and writes it as 64 contiguous bytes; other groups fall back to per-token
// 2-byte stores (the per-element scatter was 85 us for an 8192-token step, 2.6x the bytes' time).
constexpr int kTokTile = 32;

__global__ void __launch_bounds__(256) rope_and_cache_kernel(bf16_t* __restrict__ qkv, const int* __restrict__ positions,
                                                             const float* __restrict__ cos_sin, bf16_t* __restrict__ kc,
                                                             bf16_t* __restrict__ vc, const int* __restrict__ slots,
                                                             int T, int nq, int nkv, int bs, int q_stride) {
  __shared__ int slot_s[kTokTile];
  __shared__ int aligned_s;
  const int t0 = blockIdx.x * kTokTile;
  const int nt = min(kTokTile, T - t0);
  if (threadIdx.x < kTokTile) slot_s[threadIdx.x] = (slots && threadIdx.x < nt) ? slots[t0 + threadIdx.x] : -1;
  __syncthreads();
  const int n_rot = (nq + nkv) * 8;  // 8 lanes x 8 pairs per head
  for (int u = threadIdx.x; u < nt * n_rot; u += blockDim.x) {
    const int tt = u / n_rot, item = u % n_rot;
    const int t = t0 + tt;
    const int head = item >> 3, c = (item & 7) * 8;
    bf16_t* x = qkv + static_cast<int64_t>(t) * q_stride + head * kHD;
    const float* cs = cos_sin + static_cast<int64_t>(positions[t]) * kHD;
    float a[8], b[8], co[8], si[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + c), a);
    unpack8(*reinterpret_cast<const u32x4*>(x + c + kHalf), b);
    const float4* cp = reinterpret_cast<const float4*>(cs + c);
    const float4* sp = reinterpret_cast<const float4*>(cs + kHalf + c);
    float4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
    co[0] = c0.x; co[1] = c0.y; co[2] = c0.z; co[3] = c0.w; co[4] = c1.x; co[5] = c1.y; co[6] = c1.z; co[7] = c1.w;
    si[0] = s0.x; si[1] = s0.y; si[2] = s0.z; si[3] = s0.w; si[4] = s1.x; si[5] = s1.y; si[6] = s1.z; si[7] = s1.w;
    float ra[8], rb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ra[j] = a[j] * co[j] - b[j] * si[j];
      rb[j] = b[j] * co[j] + a[j] * si[j];
    }
    const u32x4 va = pack8(ra), vb = pack8(rb);
    *reinterpret_cast<u32x4*>(x + c) = va;
    *reinterpret_cast<u32x4*>(x + c + kHalf) = vb;
    const int slot = slot_s[tt];
    if (head >= nq && slot >= 0) {
      const int kh = head - nq;
      bf16_t* dst = kc + (static_cast<int64_t>(slot / bs) * nkv + kh) * bs * kHD;  // fragment-native tile
      *reinterpret_cast<u32x4*>(dst + kcache_off(slot % bs, c)) = va;
      *reinterpret_cast<u32x4*>(dst + kcache_off(slot % bs, c + kHalf)) = vb;
    }
  }
  // ---- V
  if (threadIdx.x < 64) {
    const int i = threadIdx.x & 31;
    const bool ok = nt == kTokTile && slot_s[0] >= 0 && slot_s[0] % kTokTile == 0 && slot_s[i] == slot_s[0] + i;
    const unsigned long long all = __ballot(ok);
    if (threadIdx.x == 0) aligned_s = (all & 0xffffffffull) == 0xffffffffull;
  }
  __syncthreads();
  const int voff = (nq + nkv) * kHD;
  const int n_v = nkv * kHD;
  if (aligned_s) {
    const int blk = slot_s[0] / bs, k0 = slot_s[0] % bs;
    const bf16_t* v0 = qkv + static_cast<int64_t>(t0) * q_stride + voff;
    for (int u = threadIdx.x; u < n_v; u += blockDim.x) {  // u = kv head * 128 + channel
      const int kh = u / kHD, d = u % kHD;
      uint32_t w[kTokTile / 2];
#pragma unroll
      for (int j = 0; j < kTokTile / 2; ++j) {
        const uint32_t lo = v0[static_cast<int64_t>(2 * j) * q_stride + u];
        const uint32_t hi = v0[static_cast<int64_t>(2 * j + 1) * q_stride + u];
        w[j] = lo | (hi << 16);
      }
      bf16_t* vb = vc + (static_cast<int64_t>(blk) * nkv + kh) * kHD * bs;  // 8 keys per 16-byte piece
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<u32x4*>(vb + vcache_off(k0 + 8 * q, d)) = u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
    }
    return;
  }
  for (int u = threadIdx.x; u < nt * n_v; u += blockDim.x) {
    const int tt = u / n_v, e = u % n_v;
    const int slot = slot_s[tt];
    if (slot < 0) continue;
    const int kh = e / kHD, d = e % kHD;
    vc[(static_cast<int64_t>(slot / bs) * nkv + kh) * kHD * bs + vcache_off(slot % bs, d)] =
        qkv[static_cast<int64_t>(t0 + tt) * q_stride + voff + e];
  }
}

}  // namespace

PK_EXPORT int pk_rope_and_cache(void* qkv, const void* positions, const void* cos_sin, void* k_cache, void* v_cache,
                                const void* slot_mapping, int T, int nq, int nkv, int hd, int bs, int q_stride,
                                int unused, hipStream_t stream) {
  if (T <= 0) return 0;
  if (hd != kHD || (bs % 32) != 0) return -1;  // fragment-native K tiles of 32 tokens
  rope_and_cache_kernel<<<(T + kTokTile - 1) / kTokTile, 256, 0, stream>>>(
      static_cast<bf16_t*>(qkv), static_cast<const int*>(positions), static_cast<const float*>(cos_sin),
      static_cast<bf16_t*>(k_cache), static_cast<bf16_t*>(v_cache), static_cast<const int*>(slot_mapping), T, nq, nkv,
      bs, q_stride);
  return PK_CHECK_LAUNCH();
}
