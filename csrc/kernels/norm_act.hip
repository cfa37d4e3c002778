// RMSNorm, fused residual-add + RMSNorm, and SiLU-and-mul for gfx950.
//
// All three are HBM-bound: one 16-byte (8 x bf16) vector per lane access, fp32 math,
// the row kept in registers between the reduction and the scaled write (one read, one
// write per element).  Row-per-workgroup with blockDim = H / (8 * VPT) so a 4096-wide
// row is one 512-thread workgroup holding one vector per thread (VPT = vectors/thread).
#include "common.h"

using namespace pk;

namespace {

template <int VPT>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ in,
                                                       const bf16_t* __restrict__ w, int H, int in_stride,
                                                       int out_stride, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const u32x4* x = reinterpret_cast<const u32x4*>(in + static_cast<int64_t>(row) * in_stride);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    unpack8(x[c], v[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
  }
  const float r = rsqrtf(block_sum(ss, red) / H + eps);
  const u32x4* wv = reinterpret_cast<const u32x4*>(w);
  u32x4* o = reinterpret_cast<u32x4*>(out + static_cast<int64_t>(row) * out_stride);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    float g[8];
    unpack8(wv[c], g);
    float y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(v[i][j] * r)) * g[j];
    o[c] = pack8(y);
  }
}

// residual = x + residual (bf16 stored); x = rmsnorm(residual) * w
template <int VPT>
__global__ void __launch_bounds__(1024) fused_add_rmsnorm_kernel(bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
                                                                 const bf16_t* __restrict__ w, int H, float eps) {
  __shared__ float red[16];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * H;
  u32x4* xv = reinterpret_cast<u32x4*>(x + base);
  u32x4* rv = reinterpret_cast<u32x4*>(residual + base);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    float a[8], b[8];
    unpack8(xv[c], a);
    unpack8(rv[c], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(a[j] + b[j]));  // residual is bf16
    rv[c] = pack8(v[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
  }
  const float r = rsqrtf(block_sum(ss, red) / H + eps);
  const u32x4* wv = reinterpret_cast<const u32x4*>(w);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    float g[8], y[8];
    unpack8(wv[c], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(v[i][j] * r)) * g[j];
    xv[c] = pack8(y);
  }
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// in: [T, 2*I] (gate | up), out: [T, I]
__global__ void __launch_bounds__(256) silu_and_mul_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ in,
                                                           int I) {
  const int row = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;  // vector index within the row
  if (c * 8 >= I) return;
  const u32x4* g = reinterpret_cast<const u32x4*>(in + static_cast<int64_t>(row) * 2 * I);
  const u32x4* u = reinterpret_cast<const u32x4*>(in + static_cast<int64_t>(row) * 2 * I + I);
  float a[8], b[8], y[8];
  unpack8(g[c], a);
  unpack8(u[c], b);
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(silu(a[j]))) * b[j];
  reinterpret_cast<u32x4*>(out + static_cast<int64_t>(row) * I)[c] = pack8(y);
}

// in: [T, 2*I] with gate/up interleaved in blocks of 16 columns, out: [T, I].
// Each lane handles 8 outputs (half a 16-block): gate at 32*b + h*8, up at 32*b + 16 + h*8.
__global__ void __launch_bounds__(256) silu_and_mul_il_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ in,
                                                              int I) {
  const int row = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;  // output vector index (8 columns)
  if (c * 8 >= I) return;
  const int b = c >> 1, h = c & 1;
  const bf16_t* base = in + static_cast<int64_t>(row) * 2 * I + 32 * b + 8 * h;
  float a[8], u[8], y[8];
  unpack8(*reinterpret_cast<const u32x4*>(base), a);
  unpack8(*reinterpret_cast<const u32x4*>(base + 16), u);
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(silu(a[j]))) * u[j];
  reinterpret_cast<u32x4*>(out + static_cast<int64_t>(row) * I)[c] = pack8(y);
}

int pick_vpt(int H, int* threads) {
  const int vecs = H / 8;
  for (int vpt : {1, 2, 4, 8}) {
    if (vecs % vpt == 0 && vecs / vpt <= 1024 && (vecs / vpt) % 64 == 0) {
      *threads = vecs / vpt;
      return vpt;
    }
  }
  return -1;
}

}  // namespace

// Returns 0 on success, negative on unsupported shape, hip error code otherwise.
PK_EXPORT int pk_rmsnorm(void* out, const void* in, const void* w, int T, int H, int in_stride, int out_stride,
                         float eps, hipStream_t stream) {
  if (T <= 0) return 0;
  int threads = 0;
  const int vpt = pick_vpt(H, &threads);
  auto o = static_cast<bf16_t*>(out);
  auto x = static_cast<const bf16_t*>(in);
  auto g = static_cast<const bf16_t*>(w);
  switch (vpt) {
    case 1: rmsnorm_kernel<1><<<T, threads, 0, stream>>>(o, x, g, H, in_stride, out_stride, eps); break;
    case 2: rmsnorm_kernel<2><<<T, threads, 0, stream>>>(o, x, g, H, in_stride, out_stride, eps); break;
    case 4: rmsnorm_kernel<4><<<T, threads, 0, stream>>>(o, x, g, H, in_stride, out_stride, eps); break;
    case 8: rmsnorm_kernel<8><<<T, threads, 0, stream>>>(o, x, g, H, in_stride, out_stride, eps); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_fused_add_rmsnorm(void* x, void* residual, const void* w, int T, int H, float eps,
                                   hipStream_t stream) {
  if (T <= 0) return 0;
  int threads = 0;
  const int vpt = pick_vpt(H, &threads);
  auto xx = static_cast<bf16_t*>(x);
  auto rr = static_cast<bf16_t*>(residual);
  auto g = static_cast<const bf16_t*>(w);
  switch (vpt) {
    case 1: fused_add_rmsnorm_kernel<1><<<T, threads, 0, stream>>>(xx, rr, g, H, eps); break;
    case 2: fused_add_rmsnorm_kernel<2><<<T, threads, 0, stream>>>(xx, rr, g, H, eps); break;
    case 4: fused_add_rmsnorm_kernel<4><<<T, threads, 0, stream>>>(xx, rr, g, H, eps); break;
    case 8: fused_add_rmsnorm_kernel<8><<<T, threads, 0, stream>>>(xx, rr, g, H, eps); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_silu_and_mul(void* out, const void* in, int T, int I, hipStream_t stream) {
  if (T <= 0) return 0;
  if (I % 8) return -1;
  const int vecs = I / 8;
  dim3 grid((vecs + 255) / 256, T);
  silu_and_mul_kernel<<<grid, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const bf16_t*>(in), I);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_silu_and_mul_il(void* out, const void* in, int T, int I, hipStream_t stream) {
  if (T <= 0) return 0;
  if (I % 16) return -1;
  const int vecs = I / 8;
  dim3 grid((vecs + 255) / 256, T);
  silu_and_mul_il_kernel<<<grid, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const bf16_t*>(in), I);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_kernels_abi_version() { return 1; }
