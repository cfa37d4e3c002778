// One-shot all-reduce over xGMI peer memory for small TP messages (decode activations).
//
// SURVEY.md §2.3 ("C++ IPC one-shot all-reduce ... for small decode messages") and §6: a 70B TP=8
// decode step issues 160 all-reduces of ~1 MiB; at RCCL's small-message latency these cost
// as much as the weight streaming.  MI355X GPUs of a node are fully connected by xGMI
// (7 links per GPU), so every rank can read every peer's buffer directly:
//
//   1. each workgroup b copies its chunk of the input into this rank's IPC buffer (slot = call
//      parity, so a slow peer still reading the previous call is never overwritten);
//   2. once those stores are acknowledged it stamps flag[b][rank] = epoch in EVERY peer's signal
//      area (remote stores over xGMI);
//   3. it polls its own flag[b][j] == epoch for all peers j (relaxed system-scope loads, bounded
//      spin), reads chunk b from all W buffers (peer reads over xGMI), sums in fp32 in a fixed
//      rank order (bit-identical on every rank) and writes bf16 output.
// Every slot access is system-scope (sc0 sc1: st_sys / ld_sys): a store is performed at system
// scope once acknowledged (s_waitcnt vmcnt(0) before the flag) and a load is served coherently,
// so no release / acquire fence is needed -- the L2 write-back / invalidate those do per
// workgroup measured 3.8 / 3.4 us of a 14.9 us fused collective (tools/car_probe.py).
// That argument has only been exercised with every "peer" on one device; the fenced protocol
// stays available per context (pk_car_set_fenced) and the serving-shape preflight selects it when
// the fence-free form mismatches on the group's real devices.
//
// No grid-wide barrier: chunk b only depends on the W workgroups b of the W ranks.  The epoch
// lives in device memory, so the kernels replay correctly inside HIP graphs.  It is ONE call
// counter for every collective of the context (all-reduce, all-gather, fused reduce): every
// workgroup of a call advances its share of the epoch array to the same value, so workgroup b
// of the next call -- whatever its grid -- starts from the epoch every rank agrees on, and the
// data-slot parity alternates per call.  A rank can run at most one call ahead of a peer (its
// wait needs the peer's flag of that call), so a write into slot parity (e & 1) can never hit a
// region a slow peer is still reading from call e - 1.
// IPC buffers are allocated uncached (hipDeviceMallocUncached): peers' stores become visible
// to polling loads without cache maintenance, and remote data reads are never served stale.
// Failure: a peer that does not arrive within the wall-clock timeout sets the
// error word -- in host-mapped pinned memory, so the engine reads it every step without a GPU
// sync -- and from then on every call of this context (and of every peer, which in turn times
// out waiting for it) skips its waits and its output: the engine sees the word, fails loudly
// (health NOT_SERVING, non-zero exit) instead of serving tokens summed from stale peer slots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>

#define PK_EXPORT extern "C" __attribute__((visibility("default")))

#include "comm/car_device.h"
#include "comm/signals.h"

namespace {

using pkcomm::kMaxBlocks;
using pkcomm::kMaxRanks;
using pkcomm::kRrChunk;
using pkcomm::kSigBytes;
using pkcomm::Signals;
constexpr int kArBlocks = 256;    // grid cap of the one-shot / two-shot all-reduce and all-gather
constexpr int kThreads = 512;

using namespace pkcar;

struct Ctx {
  int rank = 0, world = 0;
  size_t data_bytes = 0;  // per parity slot
  char* local = nullptr;  // own IPC buffer
  PeerPtrs peers{};
  PeerPtrs* d_peers = nullptr;
  bool opened[kMaxRanks] = {};
  char* loop[kMaxRanks] = {};  // loopback context: the stand-in peer buffers it owns
  uint32_t* h_err = nullptr;   // host-mapped error word (hipHostMalloc mapped | coherent)
  uint32_t* d_err = nullptr;   // its device alias
  long long timeout_ticks = 0;
  int fenced = 0;              // pk_car_set_fenced
};

// n16: message size in 16-byte vectors (8 bf16).  Each workgroup owns a contiguous chunk.
template <int W>
__global__ void __launch_bounds__(kThreads) allreduce_1shot(const PeerPtrs* __restrict__ peers, int rank,
                                                             size_t data_bytes, const uint4* __restrict__ inp,
                                                             uint4* __restrict__ out, int64_t n16, const Fail fail) {
  const int b = blockIdx.x, nb = gridDim.x;
  Signals* my_sig = reinterpret_cast<Signals*>(peers->base[rank]);
  __shared__ uint32_t e_s, err_s;
  if (threadIdx.x == 0) {
    e_s = my_sig->epoch[b] + 1;
    err_s = my_sig->error;  // same round trip as the epoch (uncached signal area)
  }
  __syncthreads();
  if (err_s) return;  // this group already failed: fail fast, never wait again
  const uint32_t e = e_s;
  const size_t slot = kSigBytes + (e & 1u) * data_bytes;
  const int64_t per = (n16 + nb - 1) / nb;
  const int64_t lo = b * per, hi = min(n16, lo + per);

  // 1. stage my chunk into my own buffer
  const auto mine = rsrc(peers->base[rank]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) st_sys(mine, slot + i * 16, inp[i]);
  // 2. publish: every thread's stores acknowledged, then one lane stamps every peer
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < W) {
    rel_fence(fail);
    Signals* ps = reinterpret_cast<Signals*>(peers->base[threadIdx.x]);
    __hip_atomic_store(&ps->flag[b][rank], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for all peers' chunk b, then reduce
  if (threadIdx.x < W) {
    spin_wait(&my_sig->flag[b][threadIdx.x], e, my_sig, fail);
    if (__hip_atomic_load(&my_sig->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) err_s = 1u;
  }
  __syncthreads();
  if (err_s) return;  // a peer never arrived: leave the output alone (the engine fails the step)
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int j = 0; j < W; ++j) src[j] = rsrc(peers->base[j]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 v[W];
#pragma unroll
    for (int j = 0; j < W; ++j) v[j] = ld_sys(src[j], slot + i * 16);
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const uint32_t w4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += bf2f(static_cast<uint16_t>(w4[q] & 0xffffu));
        acc[2 * q + 1] += bf2f(static_cast<uint16_t>(w4[q] >> 16));
      }
    }
    out[i] = make_uint4(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]), pack2(acc[6], acc[7]));
  }
  end_call(my_sig, e);
}

// Two-shot all-reduce for larger messages: reduce-scatter (rank r sums slice r of every peer's
// staged input) then all-gather (every rank reads every reduced slice), so each rank moves
// ~2 (W-1)/W of the message over xGMI instead of (W-1) x.  Slice s is split into gridDim.x
// chunks; workgroup b owns chunk b of every slice and synchronises only with workgroups b.
template <int W>
__global__ void __launch_bounds__(kThreads) allreduce_2shot(const PeerPtrs* __restrict__ peers, int rank,
                                                             size_t data_bytes, const uint4* __restrict__ inp,
                                                             uint4* __restrict__ out, int64_t n16, const Fail fail) {
  const int b = blockIdx.x, nb = gridDim.x;
  Signals* my_sig = reinterpret_cast<Signals*>(peers->base[rank]);
  __shared__ uint32_t e_s, err_s;
  if (threadIdx.x == 0) {
    e_s = my_sig->epoch[b] + 1;
    err_s = my_sig->error;
  }
  __syncthreads();
  if (err_s) return;
  const uint32_t e = e_s;
  const size_t in_slot = kSigBytes + (e & 1u) * data_bytes;
  const size_t res_slot = kSigBytes + (2 + (e & 1u)) * data_bytes;
  const int64_t slice = (n16 + W - 1) / W;
  const int64_t per = (slice + nb - 1) / nb;
  auto range = [&](int s, int64_t& lo, int64_t& hi) {
    lo = min(n16, s * slice + b * per);
    hi = min(min(n16, (s + 1) * slice), lo + per);
  };
  // 1. stage chunk b of every slice
  const auto mine = rsrc(peers->base[rank]);
  for (int s = 0; s < W; ++s) {
    int64_t lo, hi;
    range(s, lo, hi);
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) st_sys(mine, in_slot + i * 16, inp[i]);
  }
  publish<W>(peers, rank, b, e, false, fail);
  if (!wait_all<W>(my_sig->flag, b, e, my_sig, fail)) return;
  // 2. reduce chunk b of my slice across all ranks into my result region
  {
    int64_t lo, hi;
    range(rank, lo, hi);
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      uint4 v[W];
#pragma unroll
      for (int j = 0; j < W; ++j) v[j] = ld_sys(rsrc(peers->base[j]), in_slot + i * 16);
#pragma unroll
      for (int j = 0; j < W; ++j) acc8(acc, v[j]);
      st_sys(mine, res_slot + i * 16,
             make_uint4(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]), pack2(acc[6], acc[7])));
    }
  }
  publish<W>(peers, rank, b, e, true, fail);
  if (!wait_all<W>(my_sig->flag2, b, e, my_sig, fail)) return;
  // 3. gather chunk b of every reduced slice
#pragma unroll
  for (int s = 0; s < W; ++s) {
    int64_t lo, hi;
    range(s, lo, hi);
    const auto res = rsrc(peers->base[s]);
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) out[i] = ld_sys(res, res_slot + i * 16);
  }
  end_call(my_sig, e);
}

// All-gather along the last dim: every rank contributes rows x row16 16-byte units and receives
// out[row][j * row16 + col] = rank j's inp[row][col] (the vocab-parallel LM head's logits, so
// every rank samples the same tokens from the full row without a collective library call
// inside the decode graph).  Same slot parity / per-workgroup flag protocol as the one-shot
// all-reduce; workgroup b owns a contiguous chunk of the flattened input.
template <int W>
__global__ void __launch_bounds__(kThreads) allgather_1shot(const PeerPtrs* __restrict__ peers, int rank,
                                                             size_t data_bytes, const uint4* __restrict__ inp,
                                                             uint4* __restrict__ out, int64_t rows, int64_t row16,
                                                             const Fail fail) {
  const int b = blockIdx.x, nb = gridDim.x;
  Signals* my_sig = reinterpret_cast<Signals*>(peers->base[rank]);
  __shared__ uint32_t e_s, err_s;
  if (threadIdx.x == 0) {
    e_s = my_sig->epoch[b] + 1;
    err_s = my_sig->error;
  }
  __syncthreads();
  if (err_s) return;
  const uint32_t e = e_s;
  const size_t slot = kSigBytes + (e & 1u) * data_bytes;
  const int64_t n16 = rows * row16;
  const int64_t per = (n16 + nb - 1) / nb;
  const int64_t lo = b * per, hi = min(n16, lo + per);
  const auto mine = rsrc(peers->base[rank]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) st_sys(mine, slot + i * 16, inp[i]);
  publish<W>(peers, rank, b, e, false, fail);
  if (!wait_all<W>(my_sig->flag, b, e, my_sig, fail)) return;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    const int64_t row = i / row16, col = i - row * row16;
    uint4 v[W];
#pragma unroll
    for (int j = 0; j < W; ++j) v[j] = ld_sys(rsrc(peers->base[j]), slot + i * 16);
#pragma unroll
    for (int j = 0; j < W; ++j) out[(row * W + j) * row16 + col] = v[j];
  }
  end_call(my_sig, e);
}

// Fused TP decode collective of a row-parallel projection (Llama o / down under TP; VERDICT r2
// "fused TP decode collective"): in ONE launch
//   1. sum this rank's split-K slabs [S, M, N] fp32 of the projection (or take its bf16 [M, N]
//      partial when S == 0) and write the bf16 partial straight into this rank's IPC slot,
//   2. publish, wait for the peers' flags of the same workgroup,
//   3. sum the W partials over xGMI in rank order (bit-identical on every rank), round to bf16
//      (the all-reduce's output), add it into the bf16 residual stream in place, and
//   4. write per-(1024-column chunk, row) sums of squares of the new residual: the parts the
//      NEXT projection's folded RMSNorm (RowScale) turns into rinv -- no normalised copy.
// It replaces split-K reduce + one-shot all-reduce (with its copy-in) + residual/norm kernel.
// Work items are (row, 1024-column chunk); workgroup b takes items b, b + nb, ...  A workgroup
// is 128 threads x 8 columns.  Grid size is a host choice (<= kMaxBlocks): a shared-GPU
// rehearsal keeps it small so every rank's grid is resident at once.
// ld: row stride of the residual / partial (>= N: a column chunk of a wider residual); lds: row
// stride of the slabs [S, M, lds] (a chunk's own GEMM: lds = N).
template <int W>
__global__ void __launch_bounds__(128) reduce_residual_kernel(const PeerPtrs* __restrict__ peers, int rank,
                                                               size_t data_bytes, const float* __restrict__ slabs,
                                                               int S, const uint4* __restrict__ partial,
                                                               uint16_t* __restrict__ residual,
                                                               float* __restrict__ parts, int M, int N, int ld,
                                                               int lds, const Fail fail) {
  const int b = blockIdx.x, nb = gridDim.x;
  Signals* my_sig = reinterpret_cast<Signals*>(peers->base[rank]);
  const int nchunk = N >> 10;
  const int items = M * nchunk;
  const int64_t slab = static_cast<int64_t>(M) * lds;
  // one item per workgroup and S <= 4: the slab operands are requested before the call's epoch
  // (as in reduce_residual_2shot_kernel; branch-free, slab S - 1 again past S)
  const bool pre = S >= 1 && S <= 4 && items <= nb && b < items;
  float4 pv[4][2];
  if (pre) {
    const int r = b / nchunk, c = b - r * nchunk;
    const int64_t soff = static_cast<int64_t>(r) * lds + (c << 10) + threadIdx.x * 8;
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const float* sp = slabs + min(sidx, S - 1) * slab + soff;
      pv[sidx][0] = *reinterpret_cast<const float4*>(sp);
      pv[sidx][1] = *reinterpret_cast<const float4*>(sp + 4);
    }
  }
  __shared__ uint32_t e_s, err_s;
  __shared__ float red[2];
  if (threadIdx.x == 0) {
    e_s = my_sig->epoch[b] + 1;
    err_s = my_sig->error;
  }
  __syncthreads();
  if (err_s) return;
  const uint32_t e = e_s;
  const size_t slot = kSigBytes + (e & 1u) * data_bytes;
  const auto mine = rsrc(peers->base[rank]);
  // 1. local split-K reduction -> bf16 partial in this rank's slot (slot rows of N, source rows of ld)
  if (pre) {
    const int r = b / nchunk, c = b - r * nchunk;
    const int64_t off = static_cast<int64_t>(r) * N + (c << 10) + threadIdx.x * 8;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // slab order, as the loop below
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx)
      if (sidx < S) {
        const float4 p0 = pv[sidx][0], p1 = pv[sidx][1];
        a[0] += p0.x; a[1] += p0.y; a[2] += p0.z; a[3] += p0.w;
        a[4] += p1.x; a[5] += p1.y; a[6] += p1.z; a[7] += p1.w;
      }
    st_sys(mine, slot + off * 2, make_uint4(pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(a[4], a[5]), pack2(a[6], a[7])));
  }
  for (int it = pre ? items : b; it < items; it += nb) {
    const int r = it / nchunk, c = it - r * nchunk;
    const int64_t off = static_cast<int64_t>(r) * N + (c << 10) + threadIdx.x * 8;  // element offset
    const int64_t goff = static_cast<int64_t>(r) * ld + (c << 10) + threadIdx.x * 8;
    const int64_t soff = static_cast<int64_t>(r) * lds + (c << 10) + threadIdx.x * 8;
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
    st_sys(mine, slot + off * 2, pk);
  }
  // 2. publish (same protocol as the one-shot all-reduce), wait for every peer's workgroup b
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < W) {
    rel_fence(fail);
    Signals* ps = reinterpret_cast<Signals*>(peers->base[threadIdx.x]);
    __hip_atomic_store(&ps->flag[b][rank], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < W) {
    spin_wait(&my_sig->flag[b][threadIdx.x], e, my_sig, fail);
    if (__hip_atomic_load(&my_sig->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) err_s = 1u;
  }
  __syncthreads();
  if (err_s) return;  // a peer never arrived: residual untouched, the engine fails the step
  // 3./4. rank-ordered sum over xGMI, residual add, per-chunk sums of squares
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int j = 0; j < W; ++j) src[j] = rsrc(peers->base[j]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int it = b; it < items; it += nb) {
    const int r = it / nchunk, c = it - r * nchunk;
    const int64_t off = static_cast<int64_t>(r) * N + (c << 10) + threadIdx.x * 8;
    const int64_t goff = static_cast<int64_t>(r) * ld + (c << 10) + threadIdx.x * 8;
    uint4 v[W];
#pragma unroll
    for (int j = 0; j < W; ++j) v[j] = ld_sys(src[j], slot + off * 2);
    const uint4 rr = *reinterpret_cast<const uint4*>(residual + goff);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < W; ++j) acc8(acc, v[j]);
    float res[8];
    unpack8f(rr, res);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      res[q] = rbf(rbf(acc[q]) + res[q]);
      ss += res[q] * res[q];
    }
    *reinterpret_cast<uint4*>(residual + goff) =
        make_uint4(pack2(res[0], res[1]), pack2(res[2], res[3]), pack2(res[4], res[5]), pack2(res[6], res[7]));
    ss = wave_sum64(ss);
    if (lane == 0) red[wid] = ss;
    __syncthreads();
    if (threadIdx.x == 0) parts[static_cast<int64_t>(c) * M + r] = red[0] + red[1];
    __syncthreads();
  }
  end_call(my_sig, e);
}

// Two-shot form of the fused collective (car_device.h rr2_body) for W >= 4: each rank moves
// ~2 (W - 1) / W of the message over xGMI instead of (W - 1) x; parts per 256 columns.
template <int W>
__global__ void __launch_bounds__(128) reduce_residual_2shot_kernel(const CarDev cd, const float* __restrict__ slabs,
                                                                     int S, const uint4* __restrict__ partial,
                                                                     uint16_t* __restrict__ residual,
                                                                     float* __restrict__ parts, int M, int N, int ld,
                                                                     int lds) {
  rr2_body<W, 128, false>(cd, slabs, S, partial, residual, parts, M, N, ld, lds, blockIdx.x, gridDim.x, CarHandoff{});
}

// Pushed form of the two-shot fused collective (the decode GEMM drives the
// exchange).  The projection's GEMM (kernels/skinny_tile.h kPush) has already done stage 0 of
// reduce_residual_2shot ACROSS the fabric: the last split of every n-block summed its slabs and
// stored the bf16 tile straight into the input slot of the chunk's owner -- remote stores over
// xGMI, issued while the GEMM's other tiles still stream -- then stamped the owner's
// pflag[n-block][source].  This launch therefore starts at the reduce-scatter and reads only its
// OWN slot there:
//   1. owner: wait for the push flags of the chunk's n-blocks from every source, sum the W tiles
//      in rank order, add into the residual, publish the new chunk and its parts (result slot);
//   2. all-gather: as the two-shot form.
// Bit-identical to reduce_residual_2shot over the same slabs (the same slab order into the bf16
// partial, the same rank-order sum).  nbc: columns per GEMM n-block (64 or 128).
template <int W>
__global__ void __launch_bounds__(128) reduce_residual_pushed_kernel(const PeerPtrs* __restrict__ peers, int rank,
                                                                      size_t data_bytes, uint16_t* __restrict__ residual,
                                                                      float* __restrict__ parts, int M, int N, int nbc,
                                                                      const Fail fail) {
  const int b = blockIdx.x, nb = gridDim.x;
  Signals* my_sig = reinterpret_cast<Signals*>(peers->base[rank]);
  __shared__ uint32_t e_s, err_s, bad_s;
  if (threadIdx.x == 0) {
    e_s = my_sig->epoch[b] + 1;
    err_s = my_sig->error;
  }
  __syncthreads();
  if (err_s) return;
  const uint32_t e = e_s;
  const size_t in_slot = kSigBytes + (e & 1u) * data_bytes;
  const size_t res_slot = kSigBytes + (2 + (e & 1u)) * data_bytes;
  const int nchunk = N / kRrChunk, ngroups = nchunk / W;
  const int items = M * ngroups;
  const int per = kRrChunk / nbc;  // n-blocks per chunk
  const int64_t parts_off = static_cast<int64_t>(M) * N * 2;
  const auto mine = rsrc(peers->base[rank]);
  const int t = threadIdx.x;
  int waited = -1;
  for (int it = b; it < items; it += nb) {
    const int r = it / ngroups, j = it - r * ngroups;
    const int c = j * W + rank;
    if (j != waited) {  // the chunk's W x per tiles have landed in my slot
      if (t == 0) bad_s = 0u;
      __syncthreads();
      if (t < W * per) {
        spin_wait(&my_sig->pflag[c * per + t % per][t / per], e, my_sig, fail);
        if (__hip_atomic_load(&my_sig->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) bad_s = 1u;
      }
      __syncthreads();
      if (bad_s) return;  // a peer never pushed: residual untouched, the engine fails the step
      waited = j;
    }
    if (t < 32) {
      const int64_t off = static_cast<int64_t>(r) * N + c * kRrChunk + t * 8;
      uint4 v[W];
#pragma unroll
      for (int q = 0; q < W; ++q) v[q] = ld_sys(mine, in_slot + pkcomm::push_off(q, r, j, t * 8, M, ngroups) * 2);
      const uint4 rr = *reinterpret_cast<const uint4*>(residual + off);
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
      *reinterpret_cast<uint4*>(residual + off) = out;
      st_sys(mine, res_slot + off * 2, out);
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 32);
      if (t == 0) {
        parts[static_cast<int64_t>(c) * M + r] = ss;
        stf_sys(mine, res_slot + parts_off + (static_cast<int64_t>(c) * M + r) * 4, ss);
      }
    }
  }
  publish<W>(peers, rank, b, e, true, fail);
  if (!wait_all<W>(my_sig->flag2, b, e, my_sig, fail)) return;
  for (int it = b; it < items; it += nb) {
    const int r = it / ngroups, j = it - r * ngroups;
    for (int u = t; u < 32 * W; u += 128) {
      const int q = u / 32;
      if (q == rank) continue;
      const int c = j * W + q;
      const int64_t off = static_cast<int64_t>(r) * N + c * kRrChunk + (u % 32) * 8;
      const auto rq = rsrc(peers->base[q]);
      *reinterpret_cast<uint4*>(residual + off) = ld_sys(rq, res_slot + off * 2);
      if (u % 32 == 0)
        parts[static_cast<int64_t>(c) * M + r] = ldf_sys(rq, res_slot + parts_off + (static_cast<int64_t>(c) * M + r) * 4);
    }
  }
  end_call(my_sig, e);
}

}  // namespace

// ---------------------------------------------------------------------------- host API
PK_EXPORT int pk_car_abi_version() { return 1; }

// bytes before the first data slot of an IPC buffer (tools/push_probe.py lays out stand-ins)
PK_EXPORT long long pk_car_sig_bytes() { return static_cast<long long>(kSigBytes); }

PK_EXPORT int pk_car_ipc_handle_size() { return static_cast<int>(sizeof(hipIpcMemHandle_t)); }

// Allocate this rank's IPC buffer (signals + 2 data slots of data_bytes) on the current device.
PK_EXPORT void* pk_car_create(int rank, int world, long long data_bytes) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || data_bytes <= 0 || data_bytes % 16) return nullptr;
  // every slot access is a buffer op with a 32-bit byte offset and num_records 0x7ffffff0
  // (rsrc): the whole buffer must stay below that, or offsets wrap and accesses are dropped
  if (static_cast<long long>(kSigBytes) + 4 * data_bytes > 0x7ffffff0LL) return nullptr;
  Ctx* c = new Ctx();
  c->rank = rank;
  c->world = world;
  c->data_bytes = static_cast<size_t>(data_bytes);
  const size_t total = kSigBytes + 4 * c->data_bytes;  // input slots x2 parities, result slots x2
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached) != hipSuccess) {
    delete c;
    return nullptr;
  }
  if (hipMemset(p, 0, total) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    delete c;
    return nullptr;
  }
  c->local = static_cast<char*>(p);
  c->peers.base[rank] = c->local;
  void* h = nullptr;
  if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    (void)hipFree(p);
    delete c;
    return nullptr;
  }
  c->h_err = static_cast<uint32_t*>(h);
  *c->h_err = 0u;
  void* dh = nullptr;
  if (hipHostGetDevicePointer(&dh, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    (void)hipFree(p);
    delete c;
    return nullptr;
  }
  c->d_err = static_cast<uint32_t*>(dh);
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  c->timeout_ticks = 30LL * 1000 * khz;  // 30 s default (pk_car_set_timeout_ms)
  return c;
}

// 1: every later call of this context runs the fenced protocol (rel_fence / acq_fence); 0: fence-free.
// All ranks of a group must agree (parallel/preflight.py switches them together).
PK_EXPORT int pk_car_set_fenced(void* ctx, int on) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return -1;
  c->fenced = on ? 1 : 0;
  return 0;
}

PK_EXPORT int pk_car_get_fenced(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  return c == nullptr ? -1 : c->fenced;
}

// The device view of this rank's collective context (car_device.h CarDev): what a launch of the
// kernel library that carries the two-shot collective (kernels/car_gemm.hip) needs.  bytes: the
// caller's sizeof(CarDev), checked.
PK_EXPORT int pk_car_device_ctx(void* ctx, void* out, int bytes) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr || out == nullptr || bytes != static_cast<int>(sizeof(CarDev))) return -1;
  const CarDev cd{c->d_peers, c->rank, c->world, static_cast<long long>(c->data_bytes),
                  Fail{c->d_err, c->timeout_ticks, c->fenced}};
  std::memcpy(out, &cd, sizeof(cd));
  return 0;
}

PK_EXPORT int pk_car_device_ctx_size() { return static_cast<int>(sizeof(CarDev)); }

// Wall-clock bound of every wait of this context (a peer that is this late is treated as dead).
PK_EXPORT int pk_car_set_timeout_ms(void* ctx, long long ms) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || ms <= 0) return -1;
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  c->timeout_ticks = ms * khz;
  return 0;
}

PK_EXPORT int pk_car_get_handle(void* ctx, void* out) {
  Ctx* c = static_cast<Ctx*>(ctx);
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, c->local) != hipSuccess) return -1;
  std::memcpy(out, &h, sizeof(h));
  return 0;
}

// handles: world * pk_car_ipc_handle_size() bytes, rank-major (own entry ignored).
PK_EXPORT int pk_car_open(void* ctx, const void* handles) {
  Ctx* c = static_cast<Ctx*>(ctx);
  const char* hb = static_cast<const char*>(handles);
  for (int j = 0; j < c->world; ++j) {
    if (j == c->rank) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, hb + j * sizeof(h), sizeof(h));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -1 - j;
    c->peers.base[j] = static_cast<char*>(p);
    c->opened[j] = true;
  }
  if (hipMalloc(&c->d_peers, sizeof(PeerPtrs)) != hipSuccess) return -20;
  if (hipMemcpy(c->d_peers, &c->peers, sizeof(PeerPtrs), hipMemcpyHostToDevice) != hipSuccess) return -21;
  return 0;
}

// bf16 sum over the group: out = sum_j inp_j ; bytes % 16 == 0 and bytes <= data_bytes.
// algo: 1 = one-shot, 2 = two-shot, 0 = by size (one-shot up to kOneShotMax bytes).
constexpr long long kOneShotMax = 512 << 10;

PK_EXPORT int pk_car_allreduce_bf16_algo(void* ctx, const void* inp, void* out, long long bytes, int blocks, int algo,
                                         hipStream_t stream);

PK_EXPORT int pk_car_allreduce_bf16(void* ctx, const void* inp, void* out, long long bytes, int blocks,
                                    hipStream_t stream) {
  return pk_car_allreduce_bf16_algo(ctx, inp, out, bytes, blocks, 0, stream);
}

PK_EXPORT int pk_car_allreduce_bf16_algo(void* ctx, const void* inp, void* out, long long bytes, int blocks, int algo,
                                         hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  if (bytes <= 0) return 0;
  if (bytes % 16 || static_cast<size_t>(bytes) > c->data_bytes) return -2;
  const int64_t n16 = bytes / 16;
  if (blocks <= 0) blocks = static_cast<int>(std::min<int64_t>(kArBlocks, std::max<int64_t>(1, n16 / (kThreads * 2))));
  blocks = std::min(blocks, kArBlocks);
  const uint4* in4 = static_cast<const uint4*>(inp);
  uint4* out4 = static_cast<uint4*>(out);
  if (algo == 0) algo = bytes <= kOneShotMax ? 1 : 2;
  const Fail fail{c->d_err, c->timeout_ticks, c->fenced};
  switch (c->world) {
#define PK_CAR_CASE(WW)                                                                                            \
  case WW:                                                                                                       \
    if (algo == 1)                                                                                               \
      allreduce_1shot<WW><<<blocks, kThreads, 0, stream>>>(c->d_peers, c->rank, c->data_bytes, in4, out4, n16, fail); \
    else                                                                                                         \
      allreduce_2shot<WW><<<blocks, kThreads, 0, stream>>>(c->d_peers, c->rank, c->data_bytes, in4, out4, n16, fail); \
    break;
    PK_CAR_CASE(2)
    PK_CAR_CASE(3)
    PK_CAR_CASE(4)
    PK_CAR_CASE(5)
    PK_CAR_CASE(6)
    PK_CAR_CASE(7)
    PK_CAR_CASE(8)
#undef PK_CAR_CASE
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// 1 once any wait of this rank has timed out (sticky).  A plain read of host-mapped memory:
// no GPU synchronisation, cheap enough to poll every engine step.
PK_EXPORT int pk_car_check_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->h_err == nullptr) return -1;
  return static_cast<int>(__atomic_load_n(c->h_err, __ATOMIC_ACQUIRE));
}

// Tests only: re-arm a failed context (device copy and host word).  The caller must have
// re-synchronised the group (every rank's epochs advance only on completed calls).
PK_EXPORT int pk_car_clear_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  const uint32_t z = 0;
  Signals* s = reinterpret_cast<Signals*>(c->local);
  if (hipMemcpy(&s->error, &z, sizeof(z), hipMemcpyHostToDevice) != hipSuccess) return -3;
  __atomic_store_n(c->h_err, 0u, __ATOMIC_RELEASE);
  return 0;
}

// Failure path (watchdog / peer death): set the sticky host error word, so check() raises on
// every rank's next poll.  No device call: the device may be the thing that hangs.
PK_EXPORT int pk_car_set_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return -1;
  __atomic_store_n(c->h_err, 1u, __ATOMIC_RELEASE);
  return 0;
}

PK_EXPORT void pk_car_destroy(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return;
  (void)hipDeviceSynchronize();
  for (int j = 0; j < c->world; ++j)
    if (c->opened[j]) (void)hipIpcCloseMemHandle(c->peers.base[j]);
  if (c->d_peers) (void)hipFree(c->d_peers);
  if (c->local) (void)hipFree(c->local);
  for (int j = 0; j < kMaxRanks; ++j)
    if (c->loop[j]) (void)hipFree(c->loop[j]);
  if (c->h_err) (void)hipHostFree(c->h_err);
  delete c;
}

// Loopback context for one-process timing of the real collective kernels (tools/tp_solo.py
// --car loopback): the W - 1 "peers" are stand-in buffers on this device, and every flag row of
// every buffer is pre-stamped far ahead of any epoch this run reaches, so no wait ever blocks.  The
// kernels do all their own work (slab reduction, publishes, stores, reads of the stand-ins' slots);
// what is missing is the xGMI latency and the skew between real ranks.  Results are meaningless.
PK_EXPORT void* pk_car_create_loopback(int rank, int world, long long data_bytes) {
  Ctx* c = static_cast<Ctx*>(pk_car_create(rank, world, data_bytes));
  if (c == nullptr) return nullptr;
  const size_t total = kSigBytes + 4 * c->data_bytes;
  for (int j = 0; j < world; ++j) {
    if (j != rank) {
      void* p = nullptr;
      if (hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached) != hipSuccess ||
          hipMemset(p, 0, total) != hipSuccess) {
        pk_car_destroy(c);
        return nullptr;
      }
      c->loop[j] = static_cast<char*>(p);
      c->peers.base[j] = c->loop[j];
    }
    // flag, flag2 and pflag rows: 3 x kMaxBlocks x kMaxRanks words from the start of Signals
    if (hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(c->peers.base[j]), 0x40000000,
                     3 * kMaxBlocks * kMaxRanks) != hipSuccess) {
      pk_car_destroy(c);
      return nullptr;
    }
  }
  if (hipMalloc(&c->d_peers, sizeof(PeerPtrs)) != hipSuccess ||
      hipMemcpy(c->d_peers, &c->peers, sizeof(PeerPtrs), hipMemcpyHostToDevice) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    pk_car_destroy(c);
    return nullptr;
  }
  return c;
}

// All-gather of a [rows, row_bytes] row block per rank into out [rows, world * row_bytes]
// (rank-major within each row).  row_bytes % 16 == 0, rows * row_bytes <= data_bytes.
PK_EXPORT int pk_car_allgather(void* ctx, const void* inp, void* out, long long rows, long long row_bytes, int blocks,
                               hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  if (rows <= 0 || row_bytes <= 0) return 0;
  if (row_bytes % 16 || static_cast<size_t>(rows * row_bytes) > c->data_bytes) return -2;
  const int64_t row16 = row_bytes / 16, n16 = rows * row16;
  if (blocks <= 0) blocks = static_cast<int>(std::min<int64_t>(kArBlocks, std::max<int64_t>(1, n16 / (kThreads * 2))));
  blocks = std::min(blocks, kArBlocks);
  const Fail fail{c->d_err, c->timeout_ticks, c->fenced};
  const uint4* in4 = static_cast<const uint4*>(inp);
  uint4* out4 = static_cast<uint4*>(out);
  switch (c->world) {
#define PK_CAG_CASE(WW)                                                                                         \
  case WW:                                                                                                    \
    allgather_1shot<WW><<<blocks, kThreads, 0, stream>>>(c->d_peers, c->rank, c->data_bytes, in4, out4, rows, \
                                                         row16, fail);                                        \
    break;
    PK_CAG_CASE(2)
    PK_CAG_CASE(3)
    PK_CAG_CASE(4)
    PK_CAG_CASE(5)
    PK_CAG_CASE(6)
    PK_CAG_CASE(7)
    PK_CAG_CASE(8)
#undef PK_CAG_CASE
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Fused reduce-scatter-free TP collective of a row-parallel decode projection (see
// reduce_residual_kernel): residual[M, N] (bf16, in place) += allreduce_over_ranks(bf16(sum_s
// slabs[s])) and parts[N / 1024, M] = per-chunk sums of squares of the new residual rows.
// slabs: fp32 [S, M, N] (S >= 1), or S == 0 and `partial` a bf16 [M, N] partial.
// N % 1024 == 0, M * N * 2 <= data_bytes; blocks <= 0: one workgroup per (row, chunk) item up to
// 512 workgroups.
// The two-shot form (reduce_residual_2shot_kernel) where it moves fewer bytes over xGMI: W >= 4
// and whole 256-column chunk groups per owner.  Its parts are per 256 columns ([N / 256, M]).
PK_EXPORT int pk_car_reduce_residual_nparts(void* ctx, int M, int N) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return -1;
  const bool two = c->world >= 4 && N % (kRrChunk * c->world) == 0 &&
                   static_cast<size_t>(M) * N * 2 + static_cast<size_t>(N / kRrChunk) * M * 4 <= c->data_bytes;
  return two ? N / kRrChunk : N / 1024;
}

PK_EXPORT int pk_car_reduce_residual_ex(void* ctx, const void* slabs, int S, const void* partial, void* residual,
                                        void* parts, int M, int N, int ld, int lds, int blocks, hipStream_t stream);

// Where the decode GEMM's kPush epilogue writes (kernels/skinny_tile.h GemmArgs push_*): the
// device array of every rank's IPC buffer, this rank, the group size and the slot size.
PK_EXPORT int pk_car_push_target(void* ctx, void** peers, int* rank, int* world, long long* slot_bytes) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  *peers = c->d_peers;
  *rank = c->rank;
  *world = c->world;
  *slot_bytes = static_cast<long long>(c->data_bytes);
  return 0;
}

// The fused collective after a kPush GEMM (reduce_residual_pushed_kernel): residual [M, N] bf16
// (contiguous), parts [N / 256, M]; nbc = the GEMM's n-block width (64: KR = 1, 128).
PK_EXPORT int pk_car_reduce_residual_pushed(void* ctx, void* residual, void* parts, int M, int N, int nbc, int blocks,
                                            hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  if (M <= 0) return 0;
  if (c->world < 2 || (nbc != 64 && nbc != 128) || N % (kRrChunk * c->world) || N / nbc > kMaxBlocks ||
      residual == nullptr || parts == nullptr ||
      static_cast<size_t>(M) * N * 2 + static_cast<size_t>(N / kRrChunk) * M * 4 > c->data_bytes)
    return -2;  // (the result slot holds the new residual AND its fp32 parts)
  if (c->fenced) return -5;  // the GEMM's push epilogue has no fenced form: the caller keeps the plain chain
  const Fail fail{c->d_err, c->timeout_ticks, c->fenced};
  const int items = M * (N / kRrChunk / c->world);
  int nb = blocks <= 0 ? std::min(items, 512) : blocks;
  nb = std::max(1, std::min({nb, items, kMaxBlocks}));
  uint16_t* rs = static_cast<uint16_t*>(residual);
  float* ps = static_cast<float*>(parts);
  switch (c->world) {
#define PK_CRP_CASE(WW)                                                                                         \
  case WW:                                                                                                    \
    reduce_residual_pushed_kernel<WW><<<nb, 128, 0, stream>>>(c->d_peers, c->rank, c->data_bytes, rs, ps, M, N, nbc, \
                                                              fail);                                           \
    break;
    PK_CRP_CASE(2)
    PK_CRP_CASE(3)
    PK_CRP_CASE(4)
    PK_CRP_CASE(5)
    PK_CRP_CASE(6)
    PK_CRP_CASE(7)
    PK_CRP_CASE(8)
#undef PK_CRP_CASE
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

PK_EXPORT int pk_car_reduce_residual(void* ctx, const void* slabs, int S, const void* partial, void* residual,
                                     void* parts, int M, int N, int blocks, hipStream_t stream) {
  return pk_car_reduce_residual_ex(ctx, slabs, S, partial, residual, parts, M, N, N, N, blocks, stream);
}

// The same collective over a column chunk [M, N] of a wider residual (row stride ld) -- the TP
// decode collective overlapped with its GEMM runs one per column chunk on the comm stream while
// the compute stream runs the GEMM of the next chunk (parallel/custom_ar.py reduce_residual_chunk):
// residual / partial pointers offset to the chunk's first column, parts to its first part row,
// slabs [S, M, lds] (the chunk GEMM's own, lds = N).
PK_EXPORT int pk_car_reduce_residual_ex(void* ctx, const void* slabs, int S, const void* partial, void* residual,
                                        void* parts, int M, int N, int ld, int lds, int blocks, hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  if (M <= 0) return 0;
  if (N <= 0 || N % 1024 || ld < N || ld % 8 || lds < N || lds % 8 || S < 0 || (S == 0 && partial == nullptr) ||
      (S > 0 && slabs == nullptr) || residual == nullptr || parts == nullptr)
    return -2;
  if (static_cast<size_t>(M) * N * 2 > c->data_bytes) return -2;
  const Fail fail{c->d_err, c->timeout_ticks, c->fenced};
  const float* sl = static_cast<const float*>(slabs);
  const uint4* pt = static_cast<const uint4*>(partial);
  uint16_t* rs = static_cast<uint16_t*>(residual);
  float* ps = static_cast<float*>(parts);
  if (pk_car_reduce_residual_nparts(ctx, M, N) == N / kRrChunk) {
    const CarDev cd{c->d_peers, c->rank, c->world, static_cast<long long>(c->data_bytes), fail};
    const int items = M * (N / kRrChunk / c->world);
    int nb = blocks <= 0 ? std::min(items, 512) : blocks;
    nb = std::max(1, std::min({nb, items, kMaxBlocks}));
    switch (c->world) {
#define PK_CRR2_CASE(WW)                                                                                       \
  case WW:                                                                                                   \
    reduce_residual_2shot_kernel<WW><<<nb, 128, 0, stream>>>(cd, sl, S, pt, rs, ps, M, N, ld, lds);           \
    break;
      PK_CRR2_CASE(4)
      PK_CRR2_CASE(5)
      PK_CRR2_CASE(6)
      PK_CRR2_CASE(7)
      PK_CRR2_CASE(8)
#undef PK_CRR2_CASE
      default: return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : -4;
  }
  const int items = M * (N / 1024);
  if (blocks <= 0) blocks = std::min(items, 512);
  blocks = std::max(1, std::min({blocks, items, kMaxBlocks}));
  switch (c->world) {
#define PK_CRR_CASE(WW)                                                                                          \
  case WW:                                                                                                     \
    reduce_residual_kernel<WW><<<blocks, 128, 0, stream>>>(c->d_peers, c->rank, c->data_bytes, sl, S, pt, rs, ps, M, \
                                                           N, ld, lds, fail);                                  \
    break;
    PK_CRR_CASE(2)
    PK_CRR_CASE(3)
    PK_CRR_CASE(4)
    PK_CRR_CASE(5)
    PK_CRR_CASE(6)
    PK_CRR_CASE(7)
    PK_CRR_CASE(8)
#undef PK_CRR_CASE
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
