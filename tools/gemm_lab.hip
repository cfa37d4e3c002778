// Decode-GEMM lab: times the library's skinny GEMM (csrc/kernels/gemm_skinny.hip, included
// verbatim) on the Llama-3-8B decode shapes at M = 64 with cold weights (copies rotated over
// > 1 GiB, so nothing is served from the 256 MiB Infinity Cache).  Built several times with
// different PK_LAB_* knobs to attribute where the kernel loses against the HBM read ceiling
// (tools/hbm_read.hip).  Prints one line per shape: us per call and TB/s of weight bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc [-DPK_W_DEPTH=4 | -DPK_LAB_NO_MFMA=1 ...] tools/gemm_lab.hip -o tools/gemm_lab
#include "../csrc/kernels/gemm_skinny.hip"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

struct Shape {
  const char* name;
  int N, K, S, mode;
};

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 64;
  const char* tag = argc > 2 ? argv[2] : "";
  const Shape shapes[] = {{"qkv", 6144, 4096, 4, 1 | 16},   {"o", 4096, 4096, 8, 1 | 16},
                          {"gate_up", 28672, 4096, 1, 2 | 16 | 64}, {"down", 4096, 14336, 8, 1 | 16},
                          {"lm_head", 128256, 4096, 1, 0 | 16 | 64}};
  void *A, *out, *part;
  CHECK(hipMalloc(&A, 64ull * 16384 * 2));
  CHECK(hipMalloc(&out, 64ull * 131072 * 2));
  CHECK(hipMalloc(&part, 16ull * 64 * 131072 * 4));
  CHECK(hipMemset(A, 0x3c, 64ull * 16384 * 2));
  for (const Shape& s : shapes) {
    const size_t wbytes = static_cast<size_t>(s.N) * s.K * 2;
    // "hot": one copy re-read every call (served from the Infinity Cache when it fits)
    const bool hot = argc > 3 && std::string(argv[3]) == "hot";
    const int copies = hot ? 1 : static_cast<int>((1ull << 30) / wbytes) + 2;
    std::vector<void*> W(copies);
    for (auto& w : W) {
      CHECK(hipMalloc(&w, wbytes));
      CHECK(hipMemset(w, 0x11, wbytes));
    }
    auto call = [&](int i) {
      const int rc = pk_skinny_gemm(out, part, A, W[i % copies], M, s.N, s.K, s.K, (s.mode & 7) == 2 ? s.N / 2 : s.N,
                                    s.S, s.mode, nullptr);
      if (rc) {
        std::fprintf(stderr, "launch rc %d\n", rc);
        std::exit(1);
      }
    };
    for (int i = 0; i < copies; ++i) call(i);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int iters = 60;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) call(i);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    std::printf("%-10s %-8s N=%6d K=%5d S=%2d  %7.2f us  %5.2f TB/s\n", tag, s.name, s.N, s.K, s.S, us,
                wbytes / us / 1e6);
    for (auto& w : W) CHECK(hipFree(w));
  }
  return 0;
}
