// Can the 4 M-tiles of a skinny decode GEMM share one weight stream through the XCD L2?
//
// Design question for the decode GEMMs (M = 64 = 4 MFMA row tiles): split K over 4 workgroups
// (every weight byte read once from HBM, fp32 partial slabs written and reduced later) or split
// M over 4 workgroups that each read the SAME weight rows (no slabs; 4x the weight bytes, 3/4 of
// them hopefully L2 hits when the 4 sharers sit on one XCD and run in step).  This probe streams
// a cold [N, K] bf16 weight in 16 KiB k-steps (64 rows x 128 k, block-packed) and reports the
// time of:
//   splitk  : 4 workgroups per 64-row n-block, each reads a different K quarter (unique bytes)
//   share8  : 4 workgroups per n-block read the whole block; sharers are blocks b + 8j (one XCD)
//   share1  : same, sharers are adjacent blocks (different XCDs under round-robin dispatch)
// All three move the same unique bytes from HBM; share* read 4x that through L2.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/l2_share_probe tools/l2_share_probe.hip && tools/l2_share_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// mode 0 splitk, 1 share8, 2 share1.  Block-packed: n-block nb, k-step s = 16 KiB at (nb*ksteps + s).
template <int MODE>
__global__ void __launch_bounds__(256) probe(const u32x4* __restrict__ W, int nblocks, int ksteps,
                                             unsigned* __restrict__ sink) {
  const int b = blockIdx.x;
  int nb, part;
  if (MODE == 2) {
    nb = b / 4;
    part = b % 4;
  } else {  // sharers / K quarters of one n-block are b, b+8, b+16, b+24 (same XCD)
    const int grp = b / 32, r = b % 32;
    nb = grp * 8 + (r % 8);
    part = r / 8;
  }
  int s0 = 0, s1 = ksteps;
  if (MODE == 0) {
    s0 = part * ksteps / 4;
    s1 = (part + 1) * ksteps / 4;
  }
  const u32x4* p = W + (static_cast<size_t>(nb) * ksteps) * 1024 + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  // 4 loads per lane per k-step, 3 k-steps in flight
  u32x4 v[3][4];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int q = 0; q < 4; ++q) v[d][q] = p[static_cast<size_t>(min(s0 + d, s1 - 1)) * 1024 + q * 256];
  for (int s = s0; s < s1; s += 3) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc ^= v[d][q];
      const int nx = min(s + d + 3, s1 - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[d][q] = p[static_cast<size_t>(nx) * 1024 + q * 256];
    }
  }
  const unsigned r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x12345678u) sink[b * 256 + threadIdx.x] = r;
}

int main() {
  struct Shape {
    const char* name;
    int N, K;
  };
  const Shape shapes[] = {{"o 4096x4096", 4096, 4096}, {"qkv 6144x4096", 6144, 4096},
                          {"down 4096x14336", 4096, 14336}, {"gate_up 28672x4096", 28672, 4096}};
  unsigned* sink;
  CHECK(hipMalloc(&sink, 1 << 24));
  for (const Shape& s : shapes) {
    const size_t bytes = static_cast<size_t>(s.N) * s.K * 2;
    const int copies = static_cast<int>((1ull << 30) / bytes) + 2;
    std::vector<u32x4*> W(copies);
    for (auto& w : W) {
      CHECK(hipMalloc(&w, bytes));
      CHECK(hipMemset(w, 0x11, bytes));
    }
    const int nblocks = s.N / 64, ksteps = s.K / 128;
    const int grid = nblocks * 4;
    for (int mode = 0; mode < 3; ++mode) {
      auto go = [&](int i) {
        if (mode == 0) probe<0><<<grid, 256>>>(W[i % copies], nblocks, ksteps, sink);
        if (mode == 1) probe<1><<<grid, 256>>>(W[i % copies], nblocks, ksteps, sink);
        if (mode == 2) probe<2><<<grid, 256>>>(W[i % copies], nblocks, ksteps, sink);
      };
      for (int i = 0; i < copies; ++i) go(i);
      CHECK(hipDeviceSynchronize());
      hipEvent_t a, b;
      CHECK(hipEventCreate(&a));
      CHECK(hipEventCreate(&b));
      const int iters = 40;
      CHECK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) go(i);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / iters;
      static const char* names[] = {"splitk", "share8", "share1"};
      std::printf("%-20s grid %5d  %-7s %7.2f us  %5.2f TB/s unique\n", s.name, grid, names[mode], us,
                  bytes / us / 1e6);
    }
    for (auto& w : W) CHECK(hipFree(w));
  }
  return 0;
}
