// Decode-GEMM lab: times the library's skinny GEMM (csrc/kernels/gemm_skinny.hip, included
// verbatim) on the Llama-3-8B decode shapes at M = 64 with cold weights (copies rotated over
// > 1 GiB, so nothing is served from the 256 MiB Infinity Cache).  Prints one line per shape: us
// per call and TB/s of weight bytes, against the HBM read ceiling (tools/hbm_read.hip).  (The
// round-1/2 attribution knobs -- W register-ring depth, no-MFMA / no-A-staging / no-slab builds,
// slab store policies -- were retired from the library header in round 4; their results are in
// profiles/r1b_gemm_lab.txt and profiles/r2_decode_ab.txt.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc tools/gemm_lab.hip -o tools/gemm_lab
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
  // mode: bits 0-2 epilogue (0 bf16, 1 fp32 slabs, 2 SiLU, 3 in-launch residual add + row sums of
  // squares), bit 4 block-packed, bit 6 non-temporal, bit 7 64-row n-blocks (KR = 1)
  const Shape all_shapes[] = {{"qkv", 6144, 4096, 4, 1 | 16},   {"o", 4096, 4096, 8, 1 | 16},
                              {"gate_up", 28672, 4096, 1, 2 | 16 | 64}, {"down", 4096, 14336, 8, 1 | 16},
                              {"lm_head", 128256, 4096, 1, 0 | 16 | 64},
                              {"o_kr1_s4", 4096, 4096, 4, 1 | 16 | 128}, {"down_kr1_s4", 4096, 14336, 4, 1 | 16 | 128},
                              {"qkv_kr1_s4", 6144, 4096, 4, 1 | 16 | 128}, {"qkv_kr1_s2", 6144, 4096, 2, 1 | 16 | 128},
                              {"o_res_s8", 4096, 4096, 8, 3 | 16}, {"o_res_kr1_s4", 4096, 4096, 4, 3 | 16 | 128},
                              {"down_res_s8", 4096, 14336, 8, 3 | 16}, {"down_res_kr1_s4", 4096, 14336, 4, 3 | 16 | 128}};
  const char* only = argc > 4 ? argv[4] : "";
  std::vector<Shape> shapes;
  for (const Shape& s : all_shapes)
    if (!*only || std::string(only).find(std::string(",") + s.name + ",") != std::string::npos) shapes.push_back(s);
  void *A, *out, *part;
  CHECK(hipMalloc(&A, 64ull * 16384 * 2));
  CHECK(hipMalloc(&out, 64ull * 131072 * 2));
  CHECK(hipMalloc(&part, 16ull * 64 * 131072 * 4));
  CHECK(hipMemset(A, 0x3c, 64ull * 16384 * 2));
  void *res, *parts, *ctr;
  CHECK(hipMalloc(&res, 64ull * 16384 * 2));
  CHECK(hipMalloc(&parts, 64ull * 1024 * 4));
  CHECK(hipMalloc(&ctr, 4096 * 4));
  CHECK(hipMemset(res, 0, 64ull * 16384 * 2));
  CHECK(hipMemset(ctr, 0, 4096 * 4));
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
      GemmArgs g{};
      g.out = static_cast<bf16_t*>(out);
      g.partial = static_cast<float*>(part);
      g.A = static_cast<const bf16_t*>(A);
      g.W = static_cast<const bf16_t*>(W[i % copies]);
      g.M = M; g.N = s.N; g.K = s.K; g.lda = s.K; g.ldo = (s.mode & 7) == 2 ? s.N / 2 : s.N; g.S = s.S;
      g.counters = static_cast<int*>(ctr);
      g.residual = static_cast<bf16_t*>(res);
      g.sumsq_parts = static_cast<float*>(parts);
      const int rc = pk_skinny_gemm_ex(&g, s.mode, nullptr);
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
    std::printf("%-10s %-16s N=%6d K=%5d S=%2d  %7.2f us  %5.2f TB/s\n", tag, s.name, s.N, s.K, s.S, us,
                wbytes / us / 1e6);
    for (auto& w : W) CHECK(hipFree(w));
  }
  return 0;
}
