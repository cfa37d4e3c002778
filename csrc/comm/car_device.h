// Device side of the TP collectives over xGMI peer memory, shared by the collective kernels
// (custom_allreduce.hip, libpk_comm) and the launches that carry a collective in front of the GEMM
// that consumes its output (kernels/car_gemm.hip, libpk_kernels): the slot protocol (per-workgroup
// flags, call epochs, system-scope slot accesses, optional fences), its failure state, and the
// two-shot fused decode collective (rr2_body).  See custom_allreduce.hip for the protocol.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm/signals.h"

namespace pkcar {

using pkcomm::kMaxBlocks;
using pkcomm::kMaxRanks;
using pkcomm::kRrChunk;
using pkcomm::kSigBytes;
using pkcomm::Signals;

// per-call failure state handed to the kernels
struct Fail {
  uint32_t* host_err;      // host-mapped pinned word: polled by the engine, sticky
  long long timeout;       // wall-clock ticks a wait may take
  int fenced;              // 1: the fenced protocol (see rel_fence); 0: fence-free (default)
};

// The fenced protocol (pk_car_set_fenced): a system-scope release fence between a
// workgroup's acknowledged slot stores and its flag store, and a system-scope acquire fence after
// a flag wait.  The slot accesses stay system-scope as well, so this is strictly stronger than the
// fence-free default.  Preflight (parallel/preflight.py check_custom_ar_serving) switches a group
// to it when the fence-free form fails its serving-shape stress on the group's real devices.
// The branch is uniform (a kernel argument): fence-free calls pay one scalar compare.
__device__ __forceinline__ void rel_fence(const Fail& f) {
  if (f.fenced) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}
__device__ __forceinline__ void acq_fence(const Fail& f) {
  if (f.fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

struct PeerPtrs {
  char* base[kMaxRanks];  // every rank's IPC buffer as mapped in this process (own included)
};


// Bounded wait for flags[b][j] >= e of every peer j (one lane per peer).  ">=", not "==": a
// peer that has finished call e may already have started call e + 1 and stamped e + 1 over
// its e before this (slower, or time-sliced) rank polled -- it can never be further ahead, as
// call e + 1 needs this rank's own flag.  Serial comparison (signed difference) survives the
// 32-bit wrap.  On timeout the lane records the failure in the device copy and the
// host-mapped word and stops waiting.
__device__ __forceinline__ void spin_wait(uint32_t* flag, uint32_t e, Signals* my_sig, const Fail& f) {
  const long long t0 = wall_clock64();
  uint32_t it = 0;
  while (static_cast<int32_t>(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
    __builtin_amdgcn_s_sleep(1);
    if ((++it & 255u) == 0 && wall_clock64() - t0 > f.timeout) {
      __hip_atomic_store(&my_sig->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(f.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
  acq_fence(f);
}

// Call epilogue: workgroup b stores the call's epoch into entries b, b + nb, ... of the epoch
// array, so every entry holds the same value whatever grid the next call launches.
__device__ __forceinline__ void end_call(Signals* my_sig, uint32_t e, int b, int nb) {
  for (int i = b + static_cast<int>(threadIdx.x) * nb; i < kMaxBlocks; i += static_cast<int>(blockDim.x) * nb)
    my_sig->epoch[i] = e;
}
__device__ __forceinline__ void end_call(Signals* my_sig, uint32_t e) {
  end_call(my_sig, e, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
}

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

// System-scope (sc0 sc1) slot accesses through a buffer resource on a rank's IPC buffer (< 2 GiB:
// 32-bit byte offsets): write-through stores complete at system scope, loads bypass stale lines.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), static_cast<short>(0), 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, int64_t boff, const uint4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, static_cast<int>(boff), 0, 17);
}
__device__ __forceinline__ uint4 ld_sys(__amdgpu_buffer_rsrc_t r, int64_t boff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(boff), 0, 17));
}
__device__ __forceinline__ void stf_sys(__amdgpu_buffer_rsrc_t r, int64_t boff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, static_cast<int>(boff), 0, 17);
}
__device__ __forceinline__ float ldf_sys(__amdgpu_buffer_rsrc_t r, int64_t boff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(boff), 0, 17));
}

// Bounded relaxed poll of this rank's flag[b][j] for every peer j (the data behind a flag is read
// with system-scope loads: no acquire).
// Returns false when some peer timed out (every thread of the workgroup sees the same answer).
template <int W>
__device__ __forceinline__ bool wait_all(uint32_t (*flags)[kMaxRanks], int b, uint32_t e, Signals* my_sig,
                                         const Fail& fail) {
  __shared__ uint32_t bad_s;
  if (threadIdx.x == 0) bad_s = 0u;
  __syncthreads();
  if (threadIdx.x < W) {
    spin_wait(&flags[b][threadIdx.x], e, my_sig, fail);
    if (__hip_atomic_load(&my_sig->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) bad_s = 1u;
  }
  __syncthreads();
  return bad_s == 0u;
}

// Wait until this workgroup's (system-scope) stores are acknowledged, then stamp flags[b][rank] =
// e in every rank's signal area.
template <int W>
__device__ __forceinline__ void publish(const PeerPtrs* peers, int rank, int b, uint32_t e, bool second,
                                        const Fail& fail) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < W) {
    rel_fence(fail);
    Signals* ps = reinterpret_cast<Signals*>(peers->base[threadIdx.x]);
    __hip_atomic_store(second ? &ps->flag2[b][rank] : &ps->flag[b][rank], e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void acc8(float* acc, const uint4& v) {
  const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc[2 * q] += bf2f(static_cast<uint16_t>(w4[q] & 0xffffu));
    acc[2 * q + 1] += bf2f(static_cast<uint16_t>(w4[q] >> 16));
  }
}

__device__ __forceinline__ void unpack8f(const uint4& v, float* f) {
  const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = bf2f(static_cast<uint16_t>(w4[q] & 0xffffu));
    f[2 * q + 1] = bf2f(static_cast<uint16_t>(w4[q] >> 16));
  }
}

__device__ __forceinline__ float rbf(float x) { return bf2f(static_cast<uint16_t>(pack2(x, 0.f) & 0xffffu)); }

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}


// Everything a kernel needs of a rank's collective context (pk_car_device_ctx fills it; the
// launches of libpk_kernels that carry a collective take it by value).
struct CarDev {
  const PeerPtrs* peers;  // device copy of every rank's mapped IPC buffer
  int rank, world;
  long long data_bytes;   // bytes per slot
  Fail fail;
};

// In-launch hand-off of the collective's output to the consumer GEMM of the same launch
// (car_gemm.hip): per chunk-group tickets, the residual / parts stores write-through.
struct CarHandoff {
  int* ready;      // [ngroups] x kFlowPad: tickets of the group's finished rows
  int* all_ready;  // one counter: finished collective workgroups
  int pad;         // words between two groups' counters
};

__device__ __forceinline__ void st_wt16(void* base, int64_t boff, const uint4& v) {  // sc1 write-through
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v),
                                         __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), 0x7ffffff0,
                                                                           0x00020000),
                                         static_cast<int>(boff), 0, 16);
}
__device__ __forceinline__ void stf_wt(float* base, int64_t i, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v),
                                        __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), 0x7ffffff0,
                                                                          0x00020000),
                                        static_cast<int>(i * 4), 0, 16);
}

// Two-shot fused decode collective, workgroup b of nb (NT threads; items b, b + nb, ...): for
// W >= 4 every rank reads ~2 (W - 1) / W of the message over xGMI instead of (W - 1) x:
//   0. stage: the local split-K sum of every column (bf16 partial -> this rank's input slot);
//   1. reduce-scatter: the owner of each 256-column chunk (chunk c -> rank c % W) sums that chunk
//      of the W partials in rank order, adds it into its residual, and publishes the new residual
//      chunk and its row sums of squares in its result slot;
//   2. all-gather: every rank copies the other owners' new residual chunks and parts.
// Work item (row r, chunk group j) = chunks j W .. j W + W - 1 (one per owner); workgroup b
// synchronises only with the workgroups b of its peers (flag / flag2), so the parts are per
// 256-column chunk: [N / 256, M].  Arithmetic per element: fp32 rank-order sum of bf16 partials,
// bf16 round, bf16 residual add; every rank ends with the owner's bits.
// HO (a consumer GEMM waits in the same launch): the residual and parts stores are write-through
// and each finished item takes a ticket on its chunk group (and on the all-items counter).
template <int W, int NT, bool HO>
__device__ __forceinline__ void rr2_body(const CarDev& cd, const float* __restrict__ slabs, int S,
                                         const uint4* __restrict__ partial, uint16_t* __restrict__ residual,
                                         float* __restrict__ parts, int M, int N, int ld, int lds, int b, int nb,
                                         const CarHandoff& ho) {
  const PeerPtrs* peers = cd.peers;
  const int rank = cd.rank;
  const size_t data_bytes = static_cast<size_t>(cd.data_bytes);
  const Fail& fail = cd.fail;
  Signals* my_sig = reinterpret_cast<Signals*>(peers->base[rank]);
  const int t = threadIdx.x;
  const int nchunk = N / kRrChunk, ngroups = nchunk / W;
  const int items = M * ngroups;
  const int64_t slab = static_cast<int64_t>(M) * lds;
  // One item per workgroup (the decode shapes) and S <= 4: the item's slab operands are requested
  // before the call's epoch, so that load is not a round trip of its own on the critical path.
  constexpr int kU = (32 * W + NT - 1) / NT;  // stage-0 units per thread
  const bool pre = S >= 1 && S <= 4 && items <= nb && b < items;
  float4 pv[kU][4][2];
  if (pre) {
    const int r = b / ngroups, j = b - r * ngroups;
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int u = t + NT * k;
      if (u < 32 * W) {
        const int64_t soff = static_cast<int64_t>(r) * lds + (j * W + u / 32) * kRrChunk + (u % 32) * 8;
#pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx) {  // branch-free (slab S - 1 again past S): one load batch
          const float* sp = slabs + min(sidx, S - 1) * slab + soff;
          pv[k][sidx][0] = *reinterpret_cast<const float4*>(sp);
          pv[k][sidx][1] = *reinterpret_cast<const float4*>(sp + 4);
        }
      }
    }
  }
  __shared__ uint32_t e_s, err_s;
  if (t == 0) {
    e_s = my_sig->epoch[b] + 1;
    err_s = my_sig->error;
  }
  __syncthreads();
  if (err_s) return;  // (a consumer waiting on this workgroup's ticket times out loudly)
  const uint32_t e = e_s;
  const size_t in_slot = kSigBytes + (e & 1u) * data_bytes;
  const size_t res_slot = kSigBytes + (2 + (e & 1u)) * data_bytes;
  const int64_t parts_off = static_cast<int64_t>(M) * N * 2;  // byte offset of the parts in a result slot
  const auto mine = rsrc(peers->base[rank]);
  // 0. stage the local partial of every chunk of my items (W chunks x 256 columns = 32 W uint4)
  if (pre) {
    const int r = b / ngroups, j = b - r * ngroups;
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int u = t + NT * k;
      if (u < 32 * W) {
        const int64_t off = static_cast<int64_t>(r) * N + (j * W + u / 32) * kRrChunk + (u % 32) * 8;
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // slab order, as the loop below
#pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx)
          if (sidx < S) {
            const float4 p0 = pv[k][sidx][0], p1 = pv[k][sidx][1];
            a[0] += p0.x; a[1] += p0.y; a[2] += p0.z; a[3] += p0.w;
            a[4] += p1.x; a[5] += p1.y; a[6] += p1.z; a[7] += p1.w;
          }
        st_sys(mine, in_slot + off * 2,
               make_uint4(pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(a[4], a[5]), pack2(a[6], a[7])));
      }
    }
  }
  for (int it = pre ? items : b; it < items; it += nb) {
    const int r = it / ngroups, j = it - r * ngroups;
    for (int u = t; u < 32 * W; u += NT) {
      const int c = j * W + u / 32;
      const int64_t off = static_cast<int64_t>(r) * N + c * kRrChunk + (u % 32) * 8;  // element offset
      const int64_t goff = static_cast<int64_t>(r) * ld + c * kRrChunk + (u % 32) * 8;
      const int64_t soff = static_cast<int64_t>(r) * lds + c * kRrChunk + (u % 32) * 8;
      uint4 pk;
      if (S > 0) {
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int sidx = 0; sidx < S; ++sidx) {
          const float4 p0 = *reinterpret_cast<const float4*>(slabs + sidx * slab + soff);
          const float4 p1 = *reinterpret_cast<const float4*>(slabs + sidx * slab + soff + 4);
          a[0] += p0.x; a[1] += p0.y; a[2] += p0.z; a[3] += p0.w;
          a[4] += p1.x; a[5] += p1.y; a[6] += p1.z; a[7] += p1.w;
        }
        pk = make_uint4(pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(a[4], a[5]), pack2(a[6], a[7]));
      } else {
        pk = partial[goff >> 3];
      }
      st_sys(mine, in_slot + off * 2, pk);
    }
  }
  publish<W>(peers, rank, b, e, false, fail);
  if (!wait_all<W>(my_sig->flag, b, e, my_sig, fail)) return;
  // 1. my chunk of each item: rank-order sum over xGMI, residual add, sums of squares
  for (int it = b; it < items; it += nb) {
    const int r = it / ngroups, j = it - r * ngroups;
    const int c = j * W + rank;
    if (t < 32) {  // one wave: 32 lanes x 8 columns
      const int64_t off = static_cast<int64_t>(r) * N + c * kRrChunk + t * 8;
      const int64_t goff = static_cast<int64_t>(r) * ld + c * kRrChunk + t * 8;
      uint4 v[W];
#pragma unroll
      for (int q = 0; q < W; ++q) v[q] = ld_sys(rsrc(peers->base[q]), in_slot + off * 2);
      const uint4 rr = *reinterpret_cast<const uint4*>(residual + goff);
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) acc8(acc, v[q]);
      float res[8];
      unpack8f(rr, res);
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        res[q] = rbf(rbf(acc[q]) + res[q]);
        ss += res[q] * res[q];
      }
      const uint4 out = make_uint4(pack2(res[0], res[1]), pack2(res[2], res[3]), pack2(res[4], res[5]),
                                   pack2(res[6], res[7]));
      if constexpr (HO)
        st_wt16(residual, goff * 2, out);
      else
        *reinterpret_cast<uint4*>(residual + goff) = out;
      st_sys(mine, res_slot + off * 2, out);
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 32);
      if (t == 0) {
        if constexpr (HO)
          stf_wt(parts, static_cast<int64_t>(c) * M + r, ss);
        else
          parts[static_cast<int64_t>(c) * M + r] = ss;
        stf_sys(mine, res_slot + parts_off + (static_cast<int64_t>(c) * M + r) * 4, ss);
      }
    }
  }
  publish<W>(peers, rank, b, e, true, fail);
  if (!wait_all<W>(my_sig->flag2, b, e, my_sig, fail)) return;
  // 2. the other owners' chunks: new residual and parts
  for (int it = b; it < items; it += nb) {
    const int r = it / ngroups, j = it - r * ngroups;
    for (int u = t; u < 32 * W; u += NT) {
      const int q = u / 32;
      if (q == rank) continue;
      const int c = j * W + q;
      const int64_t off = static_cast<int64_t>(r) * N + c * kRrChunk + (u % 32) * 8;
      const int64_t goff = static_cast<int64_t>(r) * ld + c * kRrChunk + (u % 32) * 8;
      const auto rq = rsrc(peers->base[q]);
      const uint4 nv = ld_sys(rq, res_slot + off * 2);
      const float pq = u % 32 == 0 ? ldf_sys(rq, res_slot + parts_off + (static_cast<int64_t>(c) * M + r) * 4) : 0.f;
      if constexpr (HO) {
        st_wt16(residual, goff * 2, nv);
        if (u % 32 == 0) stf_wt(parts, static_cast<int64_t>(c) * M + r, pq);
      } else {
        *reinterpret_cast<uint4*>(residual + goff) = nv;
        if (u % 32 == 0) parts[static_cast<int64_t>(c) * M + r] = pq;
      }
    }
  }
  if constexpr (HO) {
    // every residual / parts store of my items acknowledged, then one ticket per item's group
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      for (int it = b; it < items; it += nb) {
        const int j = it % ngroups;
        __hip_atomic_fetch_add(ho.ready + ho.pad * j, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_fetch_add(ho.all_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  end_call(my_sig, e, b, nb);
}

}  // namespace pkcar
