// In-launch residual phase of the TP = 1 decode chain (VERDICT r4 "residual_parts: 63 launches per
// step"): the work of gemm_skinny.hip residual_parts_kernel -- residual += bf16(sum of the previous
// row-parallel projection's split-K slabs) and the per-512-column sums of squares of the new
// residual rows -- run as the FIRST phase of the launch that consumes it (the fused decode MLP
// after the o-projection, the fused QKV -> attention launch after the down projection).
//
// Producers: workgroups b < res_workgroups(), one wave per (row, 512-column part), every store
// write-through (sc1); each producer drains its stores and takes ONE ticket on slice 0 of its flow.
// Consumers: the launch's first GEMM tiles (skinny_tile FL & 4): they request their first weight
// k-steps, wait for all tickets, then read the residual (their A) and the parts (their row scale)
// with sc1 loads -- the projection's weight ramp overlaps the residual update instead of following
// a kernel boundary.  Deadlock-free: producers are the lowest workgroup indices of the grid,
// dispatched first, and never wait.
#pragma once
#include "common.h"
#include "flow.h"

// mirrored by ops/gemm.py ResArgs (ctypes)
struct ResArgs {
  uint16_t* residual;   // [M, H] bf16, updated in place
  const float* slabs;   // [S, M, H] fp32 split-K slabs of the projection (null: parts only)
  float* parts;         // [H / 512, M] sums of squares of the new residual
  int S, M, H;
  int* flow;            // zeroed hand-off buffer of its own (>= 65 * 64 words), left zeroed
};

namespace {

constexpr int kResCols = 512;  // columns per part (gemm_skinny.hip kPartCols)

__host__ __device__ inline int res_workgroups(const ResArgs& r) {
  const int items = r.M * (r.H / kResCols);
  return (items + 3) / 4;  // one wave per item, 4 waves per workgroup
}

// the residual hand-off: every producer workgroup is one ticket on slice 0; `consumers` tiles wait
inline Flow res_flow(const ResArgs& r, int consumers, int* err, int spin_limit) {
  return Flow{r.flow, r.flow + 64 * kFlowPad, err, res_workgroups(r), consumers, 0, 0, 0, 0, spin_limit};
}

template <int SS>
__device__ __forceinline__ void res_item(const ResArgs& r, int item) {
  const int lane = threadIdx.x & 63;
  const int nblk = r.H / kResCols;
  const int blk = item % nblk, m = item / nblk;
  const int c = blk * kResCols + lane * 4;  // columns c..c+3 and c+256..c+259
  uint16_t* res = r.residual + static_cast<int64_t>(m) * r.H + c;
  const uint2 r0 = *reinterpret_cast<const uint2*>(res);
  const uint2 r1 = *reinterpret_cast<const uint2*>(res + 256);
  float v[8] = {pk::bf2f(static_cast<uint16_t>(r0.x & 0xffff)), pk::bf2f(static_cast<uint16_t>(r0.x >> 16)),
                pk::bf2f(static_cast<uint16_t>(r0.y & 0xffff)), pk::bf2f(static_cast<uint16_t>(r0.y >> 16)),
                pk::bf2f(static_cast<uint16_t>(r1.x & 0xffff)), pk::bf2f(static_cast<uint16_t>(r1.x >> 16)),
                pk::bf2f(static_cast<uint16_t>(r1.y & 0xffff)), pk::bf2f(static_cast<uint16_t>(r1.y >> 16))};
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(r.residual, static_cast<short>(0), 0x7ffffff0, 0x00020000);
  if (r.slabs != nullptr) {
    // the projection output rounded to bf16 first (as the unfused GEMM would store it): the same
    // arithmetic, in the same slab order, as residual_parts_kernel -> bit-identical
    const float* src = r.slabs + static_cast<int64_t>(m) * r.H + c;
    const int64_t slab = static_cast<int64_t>(r.M) * r.H;
    float4 a, b;
    if constexpr (SS > 0) {
      float4 va[SS], vb[SS];
#pragma unroll
      for (int s = 0; s < SS; ++s) {
        va[s] = *reinterpret_cast<const float4*>(src + s * slab);
        vb[s] = *reinterpret_cast<const float4*>(src + s * slab + 256);
      }
      a = va[0];
      b = vb[0];
#pragma unroll
      for (int s = 1; s < SS; ++s) {
        a.x += va[s].x; a.y += va[s].y; a.z += va[s].z; a.w += va[s].w;
        b.x += vb[s].x; b.y += vb[s].y; b.z += vb[s].z; b.w += vb[s].w;
      }
    } else {
      a = *reinterpret_cast<const float4*>(src);
      b = *reinterpret_cast<const float4*>(src + 256);
      for (int s = 1; s < r.S; ++s) {
        const float4 x = *reinterpret_cast<const float4*>(src + s * slab);
        const float4 y = *reinterpret_cast<const float4*>(src + s * slab + 256);
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
      }
    }
    const float av[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = pk::bf2f(pk::f2bf(pk::bf2f(pk::f2bf(av[i])) + v[i]));
    typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
    const int off = static_cast<int>((res - r.residual) * 2);
    // handed off in-launch to the consumer tiles' A staging: write-through (sc1) stores
    __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk::pack2(v[0], v[1]), pk::pack2(v[2], v[3])}, rsrc, off, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk::pack2(v[4], v[5]), pk::pack2(v[6], v[7])}, rsrc, off + 512, 0,
                                          16);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
  ss = pk::wave_sum(ss);
  if (lane == 0) {
    const auto prsrc = __builtin_amdgcn_make_buffer_rsrc(r.parts, static_cast<short>(0), 0x7ffffff0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ss), prsrc,
                                          static_cast<int>((static_cast<int64_t>(blk) * r.M + m) * 4), 0, 16);
  }
}

// Workgroup b's share of the residual phase (b < res_workgroups(r)), then its ticket.
__device__ __forceinline__ void res_phase(const ResArgs& r, int b, const Flow& f) {
  const int item = b * 4 + (threadIdx.x >> 6);
  if (item < r.M * (r.H / kResCols)) {
    switch (r.slabs == nullptr ? 0 : r.S) {
      case 2: res_item<2>(r, item); break;
      case 4: res_item<4>(r, item); break;
      case 8: res_item<8>(r, item); break;
      default: res_item<0>(r, item); break;
    }
  }
  flow_signal(f, 0);
}

}  // namespace
