// In-launch dataflow hand-off between the workgroups of one fused decode launch
// (gemm_skinny.hip mlp_fused_kernel, decode_fused.hip qkv_attn_fused_kernel).
#pragma once
#include "common.h"

// Host-mapped sticky word that a timed-out wait of any fused launch sets (pk_fused_err_word): the
// engine reads it every step without a GPU sync (the custom all-reduce's error word, the same way).
// Null: the flow buffer's own error slot.
int* fused_err_word();
// Polls a consumer makes before it gives up on its tickets (pk_set_fused_spin_limit; tests shrink
// it to force a hand-off timeout and exercise the engine's fallback to the two-launch path).
int fused_spin_limit();

namespace {

// Dataflow hand-off between the two GEMMs of one fused launch (mlp_fused_kernel): a producer
// workgroup publishes its finished output columns by a ticket on the consumer split-K slice that
// reads them; a consumer workgroup issues its first weight loads, then waits for its slice's
// tickets before staging A.  role 0: none.
constexpr int kFlowPad = 64;  // words between two slices' counters (each on 256 B of its own)
struct Flow {
  int* ready;          // [slices] producer tickets (re-armed by the slice's last consumer)
  int* done;           // [slices] consumers past the wait
  int* err;            // sticky: a wait timed out (results invalid, the grid still drains)
  int need;            // producer workgroups per slice
  int consumers;       // consumer workgroups per slice
  int cols_per_slice;  // producer output columns per slice (= the consumer's K / S)
  int role;            // 1 producer, 2 consumer
  int nq, nkv;         // > 0: producer n-blocks are the heads of a fused q | k | v projection, and
                       //   slice = the kv head a head belongs to (GQA group of q, or k / v head)
  int spin_limit = 1 << 20;  // polls before a wait gives up (~0.5 s; fused_spin_limit()); < 0: test hook
};

// slice of producer n-block nb: a QKV head's kv head, or nb's output columns / cols_per_slice
__device__ __forceinline__ int flow_slice(const Flow& fl, int nb, int ncol) {
  if (fl.nq > 0) {
    if (nb < fl.nq) return nb / (fl.nq / fl.nkv);
    return nb < fl.nq + fl.nkv ? nb - fl.nq : nb - fl.nq - fl.nkv;
  }
  return (nb * ncol) / fl.cols_per_slice;
}

// sc1 4-byte load of p inside the buffer at base (< 2 GiB): bytes handed over in-launch
__device__ __forceinline__ float ldf_sc1(const float* base, const float* p) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), static_cast<short>(0), 0x7ffffff0, 0x00020000),
      static_cast<int>((p - base) * 4), 0, 16));
}

// write-through (sc1) 4-byte store of element i of the buffer at base (< 2 GiB)
__device__ __forceinline__ void stf_sc1(float* base, int i, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(
      __builtin_bit_cast(unsigned, v),
      __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), 0x7ffffff0, 0x00020000), i * 4, 0, 16);
}

// The hand-off needs no fence (guide, "Hand-offs measured with sc1 loads", first row): the
// producer's output stores are write-through (sc1), every wave drains them (vmcnt(0)) before ONE
// lane takes the ticket; the consumer's single polling lane matches, the workgroup joins it at a
// barrier, and every load of the handed-off bytes is an sc1 load.  (Plain stores + release /
// acquire fences -- an L2 write-back per producer and an L2 invalidate per consumer -- cost
// 7-8 us per layer, tools/gpu/mlp_ab.sh.)
__device__ __forceinline__ void flow_signal(const Flow& fl, int slice) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(fl.ready + kFlowPad * slice, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Consumer: one lane polls the slice's tickets (relaxed agent-scope loads + s_sleep, bounded:
// a lost producer sets the sticky error word and the grid still drains) and the workgroup joins
// it at a barrier.  The slice's last consumer re-arms both counters, so a graph replay starts
// from zero without a memset.
__device__ __forceinline__ void flow_wait(const Flow& fl, int slice) {
  if (threadIdx.x == 0) {
    int spins = 0;
    if (fl.spin_limit < 0)  // test hook (pk_set_fused_spin_limit(-1)): report a lost hand-off
      __hip_atomic_store(fl.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    while (__hip_atomic_load(fl.ready + kFlowPad * slice, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fl.need) {
      __builtin_amdgcn_s_sleep(16);  // ~0.5 us between polls: pollers must not load the memory channel of the line
      if (++spins > fl.spin_limit) {
        __hip_atomic_store(fl.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    if (__hip_atomic_fetch_add(fl.done + kFlowPad * slice, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        fl.consumers - 1) {
      __hip_atomic_store(fl.ready + kFlowPad * slice, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(fl.done + kFlowPad * slice, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
}

}  // namespace
