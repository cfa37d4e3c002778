// Read-bandwidth ceiling probe for MI355X: how fast can a kernel stream a cold buffer that
// does not fit in the Infinity Cache, as a function of grid size, waves per workgroup and
// 16-byte loads in flight per lane.  The decode GEMMs are pure weight streams, so this is the
// roofline they are measured against (profiles/README.md).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_read tools/hbm_read.hip && tools/hbm_read
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Each workgroup streams one contiguous chunk; every lane keeps DEPTH 16-byte loads in flight.
template <int DEPTH, bool NT>
__global__ void read_kernel(const u32x4* __restrict__ src, size_t n_vec, unsigned* __restrict__ sink) {
  const size_t per_wg = n_vec / gridDim.x;
  const u32x4* p = src + blockIdx.x * per_wg;
  const int tid = threadIdx.x, nt = blockDim.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (size_t i = tid; i + (DEPTH - 1) * nt < per_wg; i += DEPTH * nt) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) v[d] = NT ? __builtin_nontemporal_load(p + i + d * nt) : p[i + d * nt];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) acc ^= v[d];
  }
  const unsigned r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x12345678u) sink[blockIdx.x * nt + tid] = r;  // practically never: keeps the loads live
}

template <int DEPTH, bool NT>
float run(const u32x4* buf, size_t n_vec, unsigned* sink, int grid, int threads, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  // rotate over 4 quarter-GiB windows of the 4 GiB buffer so every launch reads cold data
  const size_t win = n_vec / 4;
  read_kernel<DEPTH, NT><<<grid, threads>>>(buf, win, sink);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) read_kernel<DEPTH, NT><<<grid, threads>>>(buf + (r % 4) * win, win, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = static_cast<double>(win) * 16.0 * reps;
  return static_cast<float>(bytes / (ms * 1e-3) / 1e12);
}

// Sized probe: one launch reads `mb` MiB with `grid` workgroups (cold: rotated over 4 GiB).
template <int DEPTH, bool NT>
float run_sized(const u32x4* buf, size_t total_vec, unsigned* sink, size_t mb, int grid, int threads, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const size_t win = (mb << 20) / 16;
  const int nwin = static_cast<int>(total_vec / win);
  read_kernel<DEPTH, NT><<<grid, threads>>>(buf, win, sink);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) read_kernel<DEPTH, NT><<<grid, threads>>>(buf + (r % nwin) * win, win, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;  // us per launch
}

int main(int argc, char** argv) {
  const size_t bytes = 4ull << 30;
  const size_t n_vec = bytes / 16;
  u32x4* buf;
  unsigned* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 64 << 20));
  CHECK(hipMemset(buf, 1, bytes));
  CHECK(hipDeviceSynchronize());
  if (argc > 1 && std::string(argv[1]) == "few") {
    // how fast can FEWER workgroups than CUs stream 112 MiB (a 70B TP=8 gate_up shard without
    // split-K: 56-112 n-blocks)?  us per launch, 256 / 512 threads, depth 8 / 16
    std::printf("grid | 256 thr d8 d16 | 512 thr d8 d16 (us, 112 MiB)\n");
    const int grids[] = {56, 64, 112, 128, 160, 224, 256};
    for (int g : grids)
      std::printf("%4d | %7.2f %7.2f | %7.2f %7.2f\n", g, run_sized<8, false>(buf, n_vec, sink, 112, g, 256, 40),
                  run_sized<16, false>(buf, n_vec, sink, 112, g, 256, 40), run_sized<8, false>(buf, n_vec, sink, 112, g, 512, 40),
                  run_sized<16, false>(buf, n_vec, sink, 112, g, 512, 40));
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "sized") {
    // us per launch for the decode GEMM weight sizes (MiB) over grids / depths
    const size_t sizes[] = {32, 48, 112, 224, 1002};
    const int grids[] = {192, 224, 256, 512, 1024};
    std::printf("MiB grid | d4 d8 d16 (us, default) | d8 nt  (TB/s of d8 nt)\n");
    for (size_t mb : sizes)
      for (int g : grids) {
        const float t4 = run_sized<4, false>(buf, n_vec, sink, mb, g, 256, 40);
        const float t8 = run_sized<8, false>(buf, n_vec, sink, mb, g, 256, 40);
        const float t16 = run_sized<16, false>(buf, n_vec, sink, mb, g, 256, 40);
        const float tn = run_sized<8, true>(buf, n_vec, sink, mb, g, 256, 40);
        std::printf("%5zu %5d | %7.2f %7.2f %7.2f | %7.2f (%4.2f)\n", mb, g, t4, t8, t16, tn,
                    (mb << 20) / (tn * 1e-6) / 1e12);
      }
    return 0;
  }
  std::printf("grid threads | d2 d4 d8 d16 (TB/s, default policy) | d8 nt\n");
  const int grids[] = {192, 224, 256, 512, 1024, 2048, 4096};
  const int threads[] = {256, 512};
  for (int th : threads)
    for (int g : grids) {
      std::printf("%5d %4d | %5.2f %5.2f %5.2f %5.2f | %5.2f\n", g, th, run<2, false>(buf, n_vec, sink, g, th, 20),
                  run<4, false>(buf, n_vec, sink, g, th, 20), run<8, false>(buf, n_vec, sink, g, th, 20),
                  run<16, false>(buf, n_vec, sink, g, th, 20), run<8, true>(buf, n_vec, sink, g, th, 20));
    }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
