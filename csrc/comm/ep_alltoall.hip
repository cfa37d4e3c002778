// Expert-parallel all-to-all over xGMI peer memory (DP attention + EP, SURVEY.md §2.3 "EP",
// §5.8 "the IPC path with per-peer offsets").
//
// Every rank owns one IPC buffer (hipDeviceMallocUncached, mapped into every peer):
//   Signals | recv_x [W][C][H] bf16 | recv_e [W][C] int32 | meta [W][4] int32 | ret_x [C_ret][H] bf16
// C = rows one rank may send one peer per call (decode: max_num_seqs x top-k), C_ret = rows
// one rank sends in total (the same bound).
//
// dispatch (one launch per MoE layer): the caller has sorted its T*k (token, slot) rows by
// destination rank (expert-align over ranks: offsets[W+1] ON THE DEVICE).  Workgroup b writes
// rows b, b+B, ... of every destination d straight into d's recv_x[me] / recv_e[me] region
// (remote stores over xGMI), pads recv_e[me][n_d .. C) with -1 (no expert: ignored by the
// receiver's align), workgroup 0 also stores meta[me] = {n_d, offsets[d]}; then the same
// release -> flag -> bounded poll -> acquire protocol as custom_allreduce.hip, workgroup b waiting
// only for workgroup b of every peer.
// return (one launch): workgroup b writes row i < n_src of its arrival-order expert output
// (region src of a [W*C, H] tensor) into src's ret_x[offsets_src[me] + i] -- so the source gets
// its rows back in exactly the destination-sorted order it sent them, and the ordinary MoE
// combine (inverse permutation x routing weights) applies unchanged.
// No host read-back anywhere: counts and offsets live on the device, so a decode step with its
// MoE layers is capturable in one HIP graph.  Ordering: a rank is at most one call ahead of a
// peer (every call waits for every peer), so single-buffered regions are safe: a peer writes my
// recv_* for call e + 1 only after my return of call e (after my expert GEMMs read them), and my
// ret_x for call e + 1 only after my dispatch of e + 1 (after my combine of call e).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>

#define PK_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kMaxRanks = 8;
constexpr int kBlocks = 64;  // workgroups of every call (fixed: flags pair workgroup b with b)
constexpr int kThreads = 256;

struct Signals {
  uint32_t flag_d[kBlocks][kMaxRanks];  // dispatch: peer `src`'s workgroup b has delivered
  uint32_t flag_r[kBlocks][kMaxRanks];  // return
  uint32_t epoch[kBlocks];              // call counter (all entries equal between calls)
  uint32_t error;
};
constexpr size_t kSigBytes = (sizeof(Signals) + 4095) / 4096 * 4096;

struct Layout {
  size_t recv_x, recv_e, meta, ret_x, total;
};

Layout layout(int world, int64_t C, int64_t H) {
  Layout L;
  L.recv_x = kSigBytes;
  L.recv_e = L.recv_x + static_cast<size_t>(world) * C * H * 2;
  L.meta = (L.recv_e + static_cast<size_t>(world) * C * 4 + 255) / 256 * 256;
  L.ret_x = (L.meta + kMaxRanks * 16 + 255) / 256 * 256;
  L.total = (L.ret_x + static_cast<size_t>(C) * H * 2 + 4095) / 4096 * 4096;
  return L;
}

struct Peers {
  char* base[kMaxRanks];
};

struct Ctx {
  int rank = 0, world = 0;
  int64_t C = 0, H = 0;
  Layout L{};
  char* local = nullptr;
  Peers peers{};
  Peers* d_peers = nullptr;
  bool opened[kMaxRanks] = {};
  uint32_t* h_err = nullptr;
  uint32_t* d_err = nullptr;
  long long timeout_ticks = 0;
};

struct Fail {
  uint32_t* host_err;
  long long timeout;
};

__device__ __forceinline__ void spin_ge(uint32_t* flag, uint32_t e, Signals* me, const Fail& f) {
  const long long t0 = wall_clock64();
  uint32_t it = 0;
  // ">=": a fast peer may already be one call further (see custom_allreduce.hip spin_wait)
  while (static_cast<int32_t>(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
    __builtin_amdgcn_s_sleep(1);
    if ((++it & 255u) == 0 && wall_clock64() - t0 > f.timeout) {
      __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(f.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// drain this workgroup's stores, system release, stamp flags[b][rank] = e in every peer; then wait
// for flags[b][j] >= e of every peer j and acquire.  false: some peer timed out.
template <int W>
__device__ bool exchange(const Peers* peers, int rank, uint32_t (Signals::*which)[kBlocks][kMaxRanks], uint32_t e,
                         Signals* me, const Fail& fail, uint32_t* bad) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    Signals* ps = reinterpret_cast<Signals*>(peers->base[threadIdx.x]);
    __hip_atomic_store(&(ps->*which)[blockIdx.x][rank], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < W) {
    spin_ge(&(me->*which)[blockIdx.x][threadIdx.x], e, me, fail);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (__hip_atomic_load(&me->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) *bad = 1u;
  }
  __syncthreads();
  return *bad == 0u;
}

__device__ __forceinline__ void end_call(Signals* me, uint32_t e) {
  for (int i = blockIdx.x + static_cast<int>(threadIdx.x) * static_cast<int>(gridDim.x); i < kBlocks;
       i += static_cast<int>(blockDim.x * gridDim.x))
    me->epoch[i] = e;
}

// send_x [n, H] bf16 rows sorted by destination; send_e [n] expert id local to the destination;
// offsets [W + 1] (device): rows of destination d = [offsets[d], offsets[d+1]).
template <int W>
__global__ void __launch_bounds__(kThreads) ep_dispatch_kernel(const Peers* __restrict__ peers, int rank, Layout L,
                                                               int64_t C, int64_t H, const uint4* __restrict__ send_x,
                                                               const int* __restrict__ send_e,
                                                               const int* __restrict__ offsets, Fail fail) {
  const int b = blockIdx.x;
  Signals* me = reinterpret_cast<Signals*>(peers->base[rank]);
  __shared__ uint32_t e_s, bad_s;
  if (threadIdx.x == 0) {
    e_s = me->epoch[b] + 1;
    bad_s = me->error;
  }
  __syncthreads();
  if (bad_s) return;
  const uint32_t e = e_s;
  const int64_t h16 = H / 8;  // 16-byte units per row
  for (int d = 0; d < W; ++d) {
    const int lo = offsets[d], n = min(offsets[d + 1] - lo, static_cast<int>(C));
    char* pb = peers->base[d];
    uint4* dst_x = reinterpret_cast<uint4*>(pb + L.recv_x) + static_cast<int64_t>(rank) * C * h16;
    int* dst_e = reinterpret_cast<int*>(pb + L.recv_e) + static_cast<int64_t>(rank) * C;
    for (int i = b; i < n; i += kBlocks) {
      const uint4* src = send_x + static_cast<int64_t>(lo + i) * h16;
      uint4* dr = dst_x + static_cast<int64_t>(i) * h16;
      for (int64_t c = threadIdx.x; c < h16; c += kThreads) dr[c] = src[c];
    }
    for (int i = n + b * kThreads + threadIdx.x; i < C; i += kBlocks * kThreads) dst_e[i] = -1;
    for (int i = b * kThreads + threadIdx.x; i < n; i += kBlocks * kThreads) dst_e[i] = send_e[lo + i];
    if (b == 0 && threadIdx.x == 0) {
      int* m = reinterpret_cast<int*>(pb + L.meta) + 4 * rank;
      m[0] = n;
      m[1] = lo;
    }
  }
  if (!exchange<W>(peers, rank, &Signals::flag_d, e, me, fail, &bad_s)) return;
  end_call(me, e);
}

// y [W * C, H] bf16: this rank's expert outputs for the rows it received, in arrival order
// (region src = rows [src * C, src * C + n_src)).  Writes row i of region src into src's ret_x at
// row offsets_src[rank] + i (the source's send order).
template <int W>
__global__ void __launch_bounds__(kThreads) ep_return_kernel(const Peers* __restrict__ peers, int rank, Layout L,
                                                             int64_t C, int64_t H, const uint4* __restrict__ y,
                                                             Fail fail) {
  const int b = blockIdx.x;
  Signals* me = reinterpret_cast<Signals*>(peers->base[rank]);
  __shared__ uint32_t e_s, bad_s;
  if (threadIdx.x == 0) {
    e_s = me->epoch[b];  // the dispatch of this call already advanced it
    bad_s = me->error;
  }
  __syncthreads();
  if (bad_s) return;
  const uint32_t e = e_s;
  const int64_t h16 = H / 8;
  const int* meta = reinterpret_cast<const int*>(peers->base[rank] + L.meta);
  for (int s = 0; s < W; ++s) {
    const int n = min(meta[4 * s], static_cast<int>(C)), off = meta[4 * s + 1];
    uint4* dst = reinterpret_cast<uint4*>(peers->base[s] + L.ret_x);
    for (int i = b; i < n; i += kBlocks) {
      const uint4* src = y + (static_cast<int64_t>(s) * C + i) * h16;
      uint4* dr = dst + static_cast<int64_t>(off + i) * h16;
      for (int64_t c = threadIdx.x; c < h16; c += kThreads) dr[c] = src[c];
    }
  }
  exchange<W>(peers, rank, &Signals::flag_r, e, me, fail, &bad_s);
}

}  // namespace

// ---------------------------------------------------------------------------- host API
PK_EXPORT int pk_ep_ipc_handle_size() { return static_cast<int>(sizeof(hipIpcMemHandle_t)); }

// This rank's buffer for `world` ranks, capacity C rows per (source, destination) pair, rows of
// H bf16 (H % 8 == 0).
PK_EXPORT void* pk_ep_create(int rank, int world, long long C, long long H) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || C <= 0 || H <= 0 || H % 8) return nullptr;
  Ctx* c = new Ctx();
  c->rank = rank;
  c->world = world;
  c->C = C;
  c->H = H;
  c->L = layout(world, C, H);
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, c->L.total, hipDeviceMallocUncached) != hipSuccess) {
    delete c;
    return nullptr;
  }
  if (hipMemset(p, 0, c->L.total) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
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
  (void)hipHostGetDevicePointer(&dh, h, 0);
  c->d_err = static_cast<uint32_t*>(dh);
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  c->timeout_ticks = 30LL * 1000 * khz;
  return c;
}

PK_EXPORT int pk_ep_set_timeout_ms(void* ctx, long long ms) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || ms <= 0) return -1;
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  c->timeout_ticks = ms * khz;
  return 0;
}

PK_EXPORT int pk_ep_get_handle(void* ctx, void* out) {
  Ctx* c = static_cast<Ctx*>(ctx);
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, c->local) != hipSuccess) return -1;
  std::memcpy(out, &h, sizeof(h));
  return 0;
}

PK_EXPORT int pk_ep_open(void* ctx, const void* handles) {
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
  if (hipMalloc(&c->d_peers, sizeof(Peers)) != hipSuccess) return -20;
  if (hipMemcpy(c->d_peers, &c->peers, sizeof(Peers), hipMemcpyHostToDevice) != hipSuccess) return -21;
  return 0;
}

// Device pointers of this rank's own regions (recv_x [W*C, H], recv_e [W*C], ret_x [C, H]).
PK_EXPORT void* pk_ep_recv_x(void* ctx) { Ctx* c = static_cast<Ctx*>(ctx); return c->local + c->L.recv_x; }
PK_EXPORT void* pk_ep_recv_e(void* ctx) { Ctx* c = static_cast<Ctx*>(ctx); return c->local + c->L.recv_e; }
PK_EXPORT void* pk_ep_ret_x(void* ctx) { Ctx* c = static_cast<Ctx*>(ctx); return c->local + c->L.ret_x; }

PK_EXPORT int pk_ep_dispatch(void* ctx, const void* send_x, const void* send_e, const void* offsets,
                             hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  const Fail fail{c->d_err, c->timeout_ticks};
  const uint4* sx = static_cast<const uint4*>(send_x);
  const int* se = static_cast<const int*>(send_e);
  const int* of = static_cast<const int*>(offsets);
  switch (c->world) {
#define PK_EPD(WW)                                                                                               \
  case WW:                                                                                                     \
    ep_dispatch_kernel<WW><<<kBlocks, kThreads, 0, stream>>>(c->d_peers, c->rank, c->L, c->C, c->H, sx, se, of, fail); \
    break;
    PK_EPD(2)
    PK_EPD(3)
    PK_EPD(4)
    PK_EPD(5)
    PK_EPD(6)
    PK_EPD(7)
    PK_EPD(8)
#undef PK_EPD
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

PK_EXPORT int pk_ep_return(void* ctx, const void* y, hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->d_peers == nullptr) return -1;
  const Fail fail{c->d_err, c->timeout_ticks};
  const uint4* yy = static_cast<const uint4*>(y);
  switch (c->world) {
#define PK_EPR(WW)                                                                                             \
  case WW:                                                                                                   \
    ep_return_kernel<WW><<<kBlocks, kThreads, 0, stream>>>(c->d_peers, c->rank, c->L, c->C, c->H, yy, fail); \
    break;
    PK_EPR(2)
    PK_EPR(3)
    PK_EPR(4)
    PK_EPR(5)
    PK_EPR(6)
    PK_EPR(7)
    PK_EPR(8)
#undef PK_EPR
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

PK_EXPORT int pk_ep_check_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr || c->h_err == nullptr) return -1;
  return static_cast<int>(__atomic_load_n(c->h_err, __ATOMIC_ACQUIRE));
}

PK_EXPORT int pk_ep_set_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return -1;
  __atomic_store_n(c->h_err, 1u, __ATOMIC_RELEASE);
  return 0;
}

PK_EXPORT void pk_ep_destroy(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c == nullptr) return;
  (void)hipDeviceSynchronize();
  for (int j = 0; j < c->world; ++j)
    if (c->opened[j]) (void)hipIpcCloseMemHandle(c->peers.base[j]);
  if (c->d_peers) (void)hipFree(c->d_peers);
  if (c->local) (void)hipFree(c->local);
  if (c->h_err) (void)hipHostFree(c->h_err);
  delete c;
}
