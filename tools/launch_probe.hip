// What does a kernel boundary cost inside a HIP graph on MI355X?  A graph of 80 dependent kernel
// nodes (one stream, captured) per variant; us per node:
//   empty g         a kernel of g workgroups (256 threads) that does nothing
//   store g         each thread stores one dword (dirty lines to write back at the boundary)
//   read g MB       the grid streams `MB` MiB (rotated over 80 buffers: cold)
// The decode chain of a 70B TP=8 rank is ~9 dependent launches per layer, so the per-node floor
// bounds what launch fusion can buy (profiles/r5_launch_probe.txt).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip && tools/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void empty_kernel(int* p) {
  if (p != nullptr && threadIdx.x == 1024) p[0] = 1;  // never: keeps the argument
}

__global__ void store_kernel(int* p) { p[blockIdx.x * blockDim.x + threadIdx.x] = threadIdx.x; }

__global__ void read_kernel(const u32x4* __restrict__ src, size_t n_vec, unsigned* __restrict__ sink) {
  const size_t per_wg = n_vec / gridDim.x;
  const u32x4* p = src + blockIdx.x * per_wg;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (size_t i = threadIdx.x; i + 7 * blockDim.x < per_wg; i += 8 * blockDim.x) {
    u32x4 v[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) v[d] = p[i + d * blockDim.x];
#pragma unroll
    for (int d = 0; d < 8; ++d) acc ^= v[d];
  }
  const unsigned r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

constexpr int kNodes = 80;

template <typename F>
float graph_us(hipStream_t s, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < kNodes; ++i) launch(i);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CHECK(hipGraphLaunch(ge, s));
  CHECK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int reps = 20;
  CHECK(hipEventRecord(a, s));
  for (int r = 0; r < reps; ++r) CHECK(hipGraphLaunch(ge, s));
  CHECK(hipEventRecord(b, s));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return ms * 1e3f / reps / kNodes;
}

int main() {
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* scratch;
  CHECK(hipMalloc(&scratch, 64 << 20));
  const size_t big = 80ull * (16 << 20);  // 80 x 16 MiB
  u32x4* buf;
  CHECK(hipMalloc(&buf, big));
  CHECK(hipMemset(buf, 1, big));
  unsigned* sink;
  CHECK(hipMalloc(&sink, 16 << 20));
  CHECK(hipDeviceSynchronize());
  const int grids[] = {1, 64, 256, 1024};
  for (int g : grids)
    std::printf("empty %5d wg: %6.2f us/node\n", g,
                graph_us(s, [&](int) { empty_kernel<<<g, 256, 0, s>>>(nullptr); }));
  for (int g : grids)
    std::printf("store %5d wg: %6.2f us/node\n", g,
                graph_us(s, [&](int) { store_kernel<<<g, 256, 0, s>>>(scratch); }));
  const int mbs[] = {1, 4, 16};
  for (int mb : mbs)
    for (int g : {256, 1024}) {
      const size_t nv = (static_cast<size_t>(mb) << 20) / 16;
      std::printf("read %2d MiB %5d wg: %6.2f us/node\n", mb, g, graph_us(s, [&](int i) {
                    read_kernel<<<g, 256, 0, s>>>(buf + static_cast<size_t>(i) * ((16 << 20) / 16), nv, sink);
                  }));
    }
  // the same 80 empty launches without a graph (stream launches)
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a, s));
  for (int r = 0; r < 20 * kNodes; ++r) empty_kernel<<<256, 256, 0, s>>>(nullptr);
  CHECK(hipEventRecord(b, s));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("stream empty 256 wg: %6.2f us/launch\n", ms * 1e3f / (20 * kNodes));
  return 0;
}
