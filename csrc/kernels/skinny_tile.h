// The decode GEMM workgroup body (skinny_tile) and its argument block, shared by the plain
// decode GEMM kernels (gemm_skinny.hip) and the fused decode launches (decode_fused.hip).
#pragma once
#include <type_traits>

#include "comm/signals.h"
#include "common.h"
#include "flow.h"

using namespace pk;

// kernel arguments of the decode GEMM (mirrored by ops/gemm.py GemmArgs, ctypes)
struct GemmArgs {
  bf16_t* out;               // kBF16 / kSiluMul: [M, ldo]; kQkvRope: q [M, nq * 128]
  float* partial;            // fp32 slabs [S, M, N]
  const bf16_t* A;           // [M, lda]; with the norm prologue: the residual stream
  const bf16_t* W;           // [N, K] row-major or block-packed
  int M, N, K, lda, ldo, S;
  int* counters;             // [N / 128] zeroed once; the last arriver re-arms its counter
  const float* nrm_parts;    // norm prologue: per-row sums of squares [nrm_nparts, M]
  const bf16_t* nrm_w;       // [K]
  int nrm_nparts;
  float eps;
  bf16_t* residual;          // kAddResNorm: [M, N], updated in place
  float* sumsq_parts;        // kAddResNorm: [N / 128, M]
  const int* positions;      // kQkvRope: [M]
  const float* cos_sin;      // [max_pos, 128] = cos[64] | sin[64]
  bf16_t* k_cache;           // [blocks, nkv, bs, 128]
  bf16_t* v_cache;           // [blocks, nkv, 128, bs]
  const int* slots;          // [M]
  int nq, nkv, bs;
  const int* row_offsets;    // grouped (MoE): rows of group e = [row_offsets[e], row_offsets[e+1]) of A /
  long long w_stride;        //   out / slabs, W of group e at W + e * w_stride; group = blockIdx.y
  int groups;                // number of groups (grid.y)
  int max_group_rows;        // bound on any group's rows (<= kMaxRows): picks the M tile / row tiles
  const int* a_rows;         // grouped: A row of group row i = a_rows[i] / a_row_div (MoE permute folded
  int a_row_div;             //   into the A staging: a_rows = expert-sorted slots, a_row_div = top-k)
  int row_scale;             // output row m scaled by rinv[m] from nrm_parts (RMSNorm folded: A is the
                             //   residual stream, the norm weight is pre-multiplied into W's columns)
  int row_tiles;             // set by dispatch: row tiles of M (> 1: M > 64, see skinny_gemm_kernel)
  int tile_rows;             // set by dispatch: rows per row tile (64, or 128 for the MT = 8 variant)
  const char* const* push_peers;  // kPush: every TP rank's IPC buffer (custom_ar PeerPtrs, device)
  long long push_bytes;      // kPush: bytes of one IPC data slot
  int push_rank, push_world; // kPush: this rank, TP group size
};

namespace {


// 16-row W tiles per wave: KR = 2 (n-block of 128 rows per 4-wave workgroup; required by the
// SiLU and QKV-RoPE epilogues, whose 32 / 128 columns must sit in one wave / workgroup) or
// KR = 1 (64-row n-blocks: twice the n-blocks, so half the split-K for the same grid -- half
// the fp32 slab bytes, and a 4x smaller last-arriver reduction in kAddResNorm).

// Epilogues.  kAddResNorm / kQkvRope are split-K with an in-launch reduction: every split
// stores its fp32 slab, the last workgroup of an n-block to arrive (agent-scope release /
// ticket / acquire, guide §5 "In-launch split-K reduction") sums the slabs and applies:
//   kAddResNorm: residual[m, n] += bf16(sum)   and writes the per-(n-block, row) sum of squares
//                of the new residual, consumed by the next GEMM's RMSNorm prologue;
//   kQkvRope:    128-column n-block = one head: RoPE (neox) for q / k heads, q -> out, k -> K
//                cache, v -> transposed V cache at the token's slot (slot < 0: not cached).
//   kPush:       a row-parallel TP projection whose epilogue drives its collective: bf16(sum) of
//                the n-block is stored straight into the input slot of the rank that owns its
//                256-column chunk (remote stores over xGMI while the other tiles still stream),
//                then that rank's push flag [n-block][this rank] is stamped with the call's
//                epoch (custom_allreduce.hip reduce_residual_pushed_kernel consumes them).
// (5 was kSiluSplit, the split gate_up reduced in-launch: removed in round 6, measured slower)
enum Mode { kBF16 = 0, kPartial = 1, kSiluMul = 2, kAddResNorm = 3, kQkvRope = 4, kPush = 6 };
constexpr int kMaxRows = 1024;  // decode batch bound of the row-tiled modes
constexpr int kPartCols = 512;  // columns per sum-of-squares part (residual_parts_kernel)



// Weight loads.  NT: non-temporal (no Infinity-Cache allocation) -- measured faster for the
// large, read-once streams (gate_up 235 MB: -6 %, LM head 1 GB: -10 %) and slower for the
// small ones, which profit from whatever the Infinity Cache still holds.
template <bool NT>
__device__ __forceinline__ bf16x8_t ldw(const bf16_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(p));
  return *reinterpret_cast<const bf16x8_t*>(p);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ float4 ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void add4(float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; }
__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

// ---- split-K tile epilogues (run by the last arriving split of n-block nb) ----------------
// Sum of the SS fp32 slabs of element group (m, c..c+3) / (m, c+64..c+67); SS == 0: runtime S.
// The loads of a batch of rows are all issued before any add, so one reducer thread has
// RB * SS 16-byte loads in flight instead of paying the slab latency serially.
// sc1 (coherent past the XCD L2) 16-byte load of p, inside the buffer that starts at base (< 2 GiB)
__device__ __forceinline__ float4 ld4f_sc1(const float* base, const float* p) {
  const auto r = __builtin_amdgcn_raw_buffer_load_b128(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), static_cast<short>(0), 0x7ffffff0, 0x00020000),
      static_cast<int>((p - base) * 4), 0, 16);
  return __builtin_bit_cast(float4, r);
}

// SC1: the slabs were handed over in-launch by write-through stores: read them with sc1 loads
// (no acquire fence, i.e. no L2 invalidate; guide "Hand-offs measured with sc1 loads")
template <int SS, bool SC1 = false>
__device__ __forceinline__ float4 slab_sum(const float* src, int64_t slab, int S, const float* base = nullptr) {
  auto ld = [&](const float* p) { return SC1 ? ld4f_sc1(base, p) : ld4f(p); };
  if constexpr (SS == 0) {
    float4 a = ld(src);
    for (int s = 1; s < S; ++s) add4(a, ld(src + s * slab));
    return a;
  } else {
    float4 v[SS];
#pragma unroll
    for (int s = 0; s < SS; ++s) v[s] = ld(src + s * slab);
#pragma unroll
    for (int s = 1; s < SS; ++s) add4(v[0], v[s]);
    return v[0];
  }
}

template <int MODE, int SS, int KR>
__device__ void epilogue(const GemmArgs& args, int nb) {
  const int M = args.M, N = args.N, S = args.S, tid = threadIdx.x;
  const int64_t slab = static_cast<int64_t>(M) * N;
  constexpr int NCOL = 64 * KR;  // columns of an n-block
  const int nbase = nb * NCOL;
  constexpr int RB = (SS == 0 || SS >= 16) ? 1 : (SS == 8 ? 2 : 4);  // rows per thread per batch
  if constexpr (MODE == kAddResNorm) {
    // TPR threads per row (4 columns each), RPP rows per pass of the workgroup
    constexpr int TPR = NCOL / 4, RPP = 256 / TPR;
    const int c = nbase + (tid % TPR) * 4;
    for (int m0 = tid / TPR; m0 < M; m0 += RPP * RB) {
      float4 a[RB];
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int m = min(m0 + RPP * i, M - 1);
        a[i] = slab_sum<SS, true>(args.partial + static_cast<int64_t>(m) * N + c, slab, S, args.partial);
      }
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int m = m0 + RPP * i;
        if (m >= M) break;  // uniform per half-wave
        bf16_t* res = args.residual + static_cast<int64_t>(m) * N + c;
        const uint2 rr = *reinterpret_cast<const uint2*>(res);
        const float v0 = rbf(rbf(a[i].x) + bf2f(static_cast<bf16_t>(rr.x & 0xffff)));
        const float v1 = rbf(rbf(a[i].y) + bf2f(static_cast<bf16_t>(rr.x >> 16)));
        const float v2 = rbf(rbf(a[i].z) + bf2f(static_cast<bf16_t>(rr.y & 0xffff)));
        const float v3 = rbf(rbf(a[i].w) + bf2f(static_cast<bf16_t>(rr.y >> 16)));
        uint2 o;
        o.x = pack2(v0, v1);
        o.y = pack2(v2, v3);
        *reinterpret_cast<uint2*>(res) = o;
        float sq = v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
#pragma unroll
        for (int off = TPR / 2; off > 0; off >>= 1) sq += __shfl_xor(sq, off, TPR);
        if (tid % TPR == 0) args.sumsq_parts[static_cast<int64_t>(nb) * M + m] = sq;
      }
    }
  } else if constexpr (MODE == kPush) {
    constexpr int TPR = NCOL / 4, RPP = 256 / TPR;
    const int W = args.push_world, me = args.push_rank;
    // the call's epoch: this rank's counter + 1 (every entry is equal between calls)
    auto* mine = reinterpret_cast<pkcomm::Signals*>(const_cast<char*>(args.push_peers[me]));
    const uint32_t e = __hip_atomic_load(&mine->epoch[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
    const int chunk = nbase / pkcomm::kRrChunk, owner = chunk % W, ng = N / pkcomm::kRrChunk / W;
    char* obase = const_cast<char*>(args.push_peers[owner]);
    bf16_t* dst = reinterpret_cast<bf16_t*>(obase + pkcomm::kSigBytes + (e & 1u) * args.push_bytes);
    // system-scope write-through stores (sc0 sc1): complete once acknowledged, so the flag needs
    // no release fence -- an L2 write-back per workgroup measured 3 us of a 6 us GEMM
    // (tools/push_probe.py); slots are < 2 GiB: 32-bit buffer offsets
    const auto drs = __builtin_amdgcn_make_buffer_rsrc(dst, static_cast<short>(0), 0x7ffffff0, 0x00020000);
    typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
    const int x = nbase % pkcomm::kRrChunk + (tid % TPR) * 4;
    const int c = nbase + (tid % TPR) * 4;
    for (int m0 = tid / TPR; m0 < M; m0 += RPP * RB) {
      float4 a[RB];
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int m = min(m0 + RPP * i, M - 1);
        a[i] = slab_sum<SS, true>(args.partial + static_cast<int64_t>(m) * N + c, slab, S, args.partial);
      }
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int m = m0 + RPP * i;
        if (m >= M) break;
        const int64_t eo = pkcomm::push_off(me, m, chunk / W, x, M, ng);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pack2(a[i].x, a[i].y), pack2(a[i].z, a[i].w)}, drs,
                                              static_cast<int>(eo * 2), 0, 17);
      }
    }
    // every push acknowledged, then the owner's flag (its wait acquires)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(&reinterpret_cast<pkcomm::Signals*>(obase)->pflag[nb][me], e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  } else {  // kQkvRope: n-block nb is head nb of q | k | v
    const int nq = args.nq, nkv = args.nkv, bs = args.bs;
    if (nb < nq + nkv) {
      // 16 threads per row, 4 rotation pairs (j, j + 64) each; 16 rows per pass
      const int j = (tid & 15) * 4;
      for (int m0 = tid >> 4; m0 < M; m0 += 16 * RB) {
        float4 a[RB], b[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int m = min(m0 + 16 * i, M - 1);
          const float* src = args.partial + static_cast<int64_t>(m) * N + nbase + j;
          a[i] = slab_sum<SS>(src, slab, S);
          b[i] = slab_sum<SS>(src + 64, slab, S);
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int m = m0 + 16 * i;
          if (m >= M) break;
          const float av[4] = {rbf(a[i].x), rbf(a[i].y), rbf(a[i].z), rbf(a[i].w)};
          const float bv[4] = {rbf(b[i].x), rbf(b[i].y), rbf(b[i].z), rbf(b[i].w)};
          const float* cs = args.cos_sin + static_cast<int64_t>(args.positions[m]) * 128;
          const float4 co = ld4f(cs + j), si = ld4f(cs + 64 + j);
          const float cc[4] = {co.x, co.y, co.z, co.w}, sn[4] = {si.x, si.y, si.z, si.w};
          float ra[4], rb[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            ra[q] = av[q] * cc[q] - bv[q] * sn[q];
            rb[q] = bv[q] * cc[q] + av[q] * sn[q];
          }
          uint2 va, vb;
          va.x = pack2(ra[0], ra[1]);
          va.y = pack2(ra[2], ra[3]);
          vb.x = pack2(rb[0], rb[1]);
          vb.y = pack2(rb[2], rb[3]);
          bf16_t* d;
          if (nb < nq) {
            d = args.out + static_cast<int64_t>(m) * args.ldo + nb * 128 + j;
          } else {
            const int slot = args.slots[m];
            if (slot < 0) continue;
            // fragment-native K tile (common.h kcache_off; 4-dim groups stay contiguous)
            bf16_t* kb = args.k_cache + (static_cast<int64_t>(slot / bs) * nkv + (nb - nq)) * bs * 128;
            *reinterpret_cast<uint2*>(kb + kcache_off(slot % bs, j)) = va;
            *reinterpret_cast<uint2*>(kb + kcache_off(slot % bs, j + 64)) = vb;
            continue;
          }
          *reinterpret_cast<uint2*>(d) = va;
          *reinterpret_cast<uint2*>(d + 64) = vb;
        }
      }
    } else {
      const int kh = nb - nq - nkv;
      const int d0 = (tid & 31) * 4;
      for (int m0 = tid >> 5; m0 < M; m0 += 8 * RB) {
        float4 a[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int m = min(m0 + 8 * i, M - 1);
          a[i] = slab_sum<SS>(args.partial + static_cast<int64_t>(m) * N + nbase + d0, slab, S);
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int m = m0 + 8 * i;
          if (m >= M) break;
          const int slot = args.slots[m];
          if (slot < 0) continue;
          bf16_t* d = args.v_cache + (static_cast<int64_t>(slot / bs) * nkv + kh) * 128 * bs;
          const int vo = vcache_off(slot % bs, d0);  // channels d0 .. d0 + 3 are 8 elements apart
          d[vo] = f2bf(a[i].x);
          d[vo + 8] = f2bf(a[i].y);
          d[vo + 16] = f2bf(a[i].z);
          d[vo + 24] = f2bf(a[i].w);
        }
      }
    }
  }
}

// grid: (n_blocks * S) workgroups of 4 waves; workgroup -> (128-row n-block, k-split) with the
// split fastest.  Per 256-deep k-chunk the workgroup stages A[0:M, chunk] in LDS (double
// buffered, register-staged: loads for chunk c+1 are issued before chunk c's MFMAs and written
// after them), while each wave streams its own 32 W rows straight to VGPRs two 128-steps
// ahead.  Row-major W: lane group g reads bytes [64s + 16g, +16) of a row in instruction s
// (64 B from each of 16 rows); block-packed W (PK): one contiguous KiB per instruction.
// NORM: A is the residual stream and the RMSNorm (x = bf16(bf16(v * rinv[m]) * w[k])) is
// applied while staging A into LDS, rinv[m] from the producer's sum-of-squares parts.
constexpr int kKC = 256;           // k per LDS chunk
constexpr int kAStride = kKC + 8;  // bf16 elements per LDS row (+16 B pad: rows shift one 16-B slot)

// MT = 8 (128 A rows, decode batches above 64): A is staged per 128-deep k-step instead of per
// 256-deep chunk, so the double-buffered tile stays 68 KiB (two workgroups per CU) and the
// register staging half as wide (no spills at 2 waves / SIMD).
// (256-row tiles -- MT = 16, one workgroup per CU, accumulators in AGPRs -- measured slower than
// two XCD-grouped 128-row tiles at every 8B shape: profiles/r4_wide_tiles_probe.jsonl)
// LDS of one skinny-GEMM workgroup (passed in, so two roles of one fused launch share it)
template <int MT>
struct SkinnyLds {
  static constexpr int kKA = MT > 4 ? 128 : kKC;  // k per staged A tile
  bf16_t a[2][16 * MT][kKA + 8] __attribute__((aligned(16)));
  float rinv[MT > 4 ? 16 * MT : 64];
  int last;
};

// FL: in-launch hand-off roles (bits) --
//   1  producer: output stores write-through (sc1), one ticket per finished n-block on `fl`
//   2  consumer of per-K-slice tickets on `fl` (slice = this tile's split): weights requested first,
//      A (the producers' output) read with sc1 loads after the wait
//   4  consumer of a TP collective carried by the same launch (car_gemm.hip): `fl` slice g = the
//      collective's chunk group g (fl.cols_per_slice columns of A, the residual stream); the tile
//      waits for every group its K range overlaps after requesting its first weight k-steps, and
//      for ALL groups (`fw`, one counter) before the row scale, whose norm parts the collective
//      writes too -- A and the parts read with sc1 loads
template <int MT, int MODE, bool PK, bool NORM, bool NT, bool RS = false, int KR = 2, int FL = 0>
__device__ __forceinline__ void skinny_tile(const GemmArgs& args, const int bx_in, const int by, const int gdx,
                                            SkinnyLds<MT>& L, const Flow& fl, const Flow& fw = Flow{}) {
  constexpr bool kProd = (FL & 1) != 0;
  constexpr bool kWaitCar = (FL & 4) != 0;
  constexpr bool kWait = (FL & 2) != 0 || kWaitCar;
  constexpr int kR = KR;
  constexpr int kKA = SkinnyLds<MT>::kKA;  // k per staged A tile
  constexpr int kPPR = kKA / 8;             // 16-byte pieces per A row
  auto& a_lds = L.a;
  auto& rinv_s = L.rinv;
  int& last_s = L.last;
  const int N = args.N, K = args.K, S = args.S;
  // rows of this workgroup's group: all rows, or (grouped) expert by's
  int gbeg = 0, gend = args.M;
  const bf16_t* Wg = args.W;
  if (args.row_offsets != nullptr) {
    gbeg = args.row_offsets[by];
    gend = args.row_offsets[by + 1];
    Wg += static_cast<int64_t>(by) * args.w_stride;
  }
  // Row tiles (a group of more than 64 rows): every (n-block, split) tile runs once per 16*MT-row
  // tile.  The RT workgroups of one W tile are given consecutive dispatch slots of ONE XCD
  // (workgroups go round-robin over the 8 XCDs), so they stream the same W bytes at the same
  // time through that XCD's L2 and HBM sees each weight byte about once.
  int bx = bx_in, rt = 0;
  if (args.row_tiles > 1) {
    const int RT = args.row_tiles, T = gdx / RT;
    if ((T & 7) == 0) {
      const int q = bx >> 3;
      rt = q % RT;
      bx = (q / RT) * 8 + (bx & 7);
    } else {
      rt = bx % RT;
      bx /= RT;
    }
  }
  const int row0 = gbeg + rt * 16 * MT;
  const int M = min(gend - row0, 16 * MT);
  if (M <= 0) return;  // no tokens routed to this expert (or this row tile): its weights are never read
  const bf16_t* __restrict__ A = args.a_rows != nullptr ? args.A : args.A + static_cast<int64_t>(row0) * args.lda;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int nb = bx / S, split = bx % S;
  const int kper = K / S;
  const int k0 = split * kper;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = nb * 64 * kR + w * 16 * kR;

  if constexpr (NORM) {
    if (tid < M) {
      float ss = 0.f;
      for (int q = 0; q < args.nrm_nparts; ++q) ss += args.nrm_parts[q * M + tid];
      rinv_s[tid] = rsqrtf(ss / K + args.eps);
    }
    __syncthreads();
  }
  // RS (row scale): the sum-of-squares parts of row `tid` are requested before the weight
  // stream starts and consumed only after the main loop, so they never delay it (unconditional
  // loads from clamped addresses: a load behind a branch would make hipcc drain vmcnt)
  // (4 threads per row; up to 64 parts per row for 64 rows, 16 for 128 rows)
  constexpr int kRsRows = MT > 4 ? 2 : 1;  // 64-row groups per thread
  constexpr int kRsLoads = 16 / (kRsRows * kRsRows);
  float rs_p[RS ? kRsRows * kRsLoads : 1];
  auto load_rs = [&]() {
    const int np = min(args.nrm_nparts, 4 * kRsLoads), sub = tid & 3;
#pragma unroll
    for (int h = 0; h < kRsRows; ++h) {
      const int rr = min(64 * h + (tid >> 2), M - 1);
#pragma unroll
      for (int q = 0; q < kRsLoads; ++q) {
        const float* p = args.nrm_parts + min(sub + 4 * q, np - 1) * args.M + row0 + rr;
        rs_p[h * kRsLoads + q] = kWaitCar ? ldf_sc1(args.nrm_parts, p) : *p;  // (parts written in-launch)
      }
    }
  };
  if constexpr (RS && !kWaitCar) load_rs();
  // the consumer's wait (after its first weight k-steps are requested)
  auto wait_in = [&](int split_) {
    if constexpr (kWaitCar) {
      const int g0 = k0 / fl.cols_per_slice, g1 = (k0 + kper - 1) / fl.cols_per_slice;
      for (int g = g0; g <= g1; ++g) flow_wait(fl, g);
    } else if constexpr (kWait) {
      flow_wait(fl, split_);
    }
  };

  const bf16_t* wp[kR];
#pragma unroll
  for (int t = 0; t < kR; ++t)
    wp[t] = PK ? Wg + static_cast<int64_t>(n0 >> 7) * 128 * K + (((n0 & 127) >> 4) + t) * 4 * 512 + 8 * lane  // block-packed
               : Wg + static_cast<int64_t>(n0 + 16 * t + r) * K + 8 * g;                     // row-major [N, K]

  // A staging: MT*16 rows x kKA cols of 16-byte pieces over 256 threads
  constexpr int kPieces = (16 * MT * kPPR + 255) / 256;
  u32x4 stage[kPieces];
  u32x4 stage_w[NORM ? kPieces : 1];
  const bf16_t* arow[kPieces];  // source row of each staged piece (fixed across k-chunks)
#pragma unroll
  for (int p = 0; p < kPieces; ++p) {
    const int src_row = min((tid + 256 * p) / kPPR, M - 1);
    const int r_a = args.a_rows != nullptr ? args.a_rows[row0 + src_row] / args.a_row_div : src_row;
    arow[p] = A + static_cast<int64_t>(r_a) * args.lda;
  }
  auto load_a = [&](int kc) {
#pragma unroll
    for (int p = 0; p < kPieces; ++p) {
      const int col = ((tid + 256 * p) % kPPR) * 8;
      if constexpr (kWait)  // the producers' output, handed off in-launch: sc1 loads
        stage[p] = __builtin_amdgcn_raw_buffer_load_b128(
            __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(args.A), static_cast<short>(0), 0x7ffffff0, 0x00020000),
            static_cast<int>((arow[p] + kc + col - args.A) * 2), 0, 16);
      else
        stage[p] = *reinterpret_cast<const u32x4*>(arow[p] + kc + col);
      if constexpr (NORM) stage_w[p] = *reinterpret_cast<const u32x4*>(args.nrm_w + kc + col);
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int p = 0; p < kPieces; ++p) {
      const int idx = tid + 256 * p;
      const int row = idx / kPPR, col = (idx % kPPR) * 8;
      u32x4 v = stage[p];
      if constexpr (NORM) {
        float x[8], wv[8];
        unpack8(v, x);
        unpack8(stage_w[p], wv);
        const float ri = rinv_s[min(row, M - 1)];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = rbf(x[j] * ri) * wv[j];
        v = pack8(x);
      }
      *reinterpret_cast<u32x4*>(&a_lds[buf][row][col]) = v;
    }
  };

  f32x4 acc[kR][MT];
#pragma unroll
  for (int t = 0; t < kR; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8_t wa[kR][4], wb[kR][4];
  auto load_w = [&](bf16x8_t (&dst)[kR][4], int k) {
#pragma unroll
    for (int t = 0; t < kR; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        dst[t][s] = PK ? ldw<NT>(wp[t] + static_cast<int64_t>(k >> 7) * (32 * 512) + s * 512)
                       : ldw<NT>(wp[t] + k + 32 * s);
  };
  auto mma_step = [&](const bf16x8_t (&wf)[kR][4], int buf, int kk) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8_t af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        af[mt] = *reinterpret_cast<const bf16x8_t*>(&a_lds[buf][16 * mt + r][kk + 32 * s + 8 * g]);
#pragma unroll
      for (int t = 0; t < kR; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][s], af[mt], acc[t][mt], 0, 0, 0);
    }
  };

  // Chunk order is rotated per n-block so concurrent workgroups read different column ranges.
  // Every load in the loop is unconditional (past the last chunk the address is clamped to it
  // and the data is dropped): a load behind a branch makes the compiler's vmcnt bookkeeping
  // assume it was not issued, so it then drains ALL loads before the next MFMAs.
  const int nchunks = kper / kKC;
  const int rot = (nb * 5) % nchunks;
  auto ck = [&](int c) { return k0 + ((min(c, nchunks - 1) + rot) % nchunks) * kKC; };
  if constexpr (MT > 4) {
    // one 128-deep k-step per staged A tile: W steps alternate wa / wb, two steps in flight
    const int nsteps = 2 * nchunks;  // even
    const int rot2 = 2 * rot;
    auto ks = [&](int j) { return k0 + ((min(j, nsteps - 1) + rot2) % nsteps) * 128; };
    if constexpr (kWait) {  // consumer of an in-launch hand-off: weights first, A after the wait
      load_w(wa, ks(0));
      load_w(wb, ks(1));
      wait_in(split);
      load_a(ks(0));
    } else {
      load_a(ks(0));
      load_w(wa, ks(0));
      load_w(wb, ks(1));
    }
    store_a(0);
    int buf = 0;
    for (int j = 0; j < nsteps; j += 2) {
      load_a(ks(j + 1));
      __syncthreads();  // step j visible in a_lds[buf]; every wave is done with a_lds[buf^1]
      mma_step(wa, buf, 0);
      load_w(wa, ks(j + 2));
      store_a(buf ^ 1);
      buf ^= 1;
      load_a(ks(j + 2));
      __syncthreads();
      mma_step(wb, buf, 0);
      load_w(wb, ks(j + 3));
      store_a(buf ^ 1);
      buf ^= 1;
    }
  } else {
  if constexpr (kWait) {
    // consumer: this workgroup's first two weight k-steps are requested before the wait, so
    // they stream in while the producers finish; A (the producers' output) is read after it
    load_w(wa, ck(0));
    load_w(wb, ck(0) + 128);
    wait_in(split);
    load_a(ck(0));
  } else {
    load_a(ck(0));
    load_w(wa, ck(0));
    load_w(wb, ck(0) + 128);
  }
  store_a(0);
  int buf = 0;
  for (int c = 0; c < nchunks; ++c) {
    const int kn = ck(c + 1);
    load_a(kn);
    __syncthreads();  // chunk c visible in a_lds[buf]; every wave is done with a_lds[buf^1]
    mma_step(wa, buf, 0);
    load_w(wa, kn);
    mma_step(wb, buf, 128);
    load_w(wb, kn + 128);
    store_a(buf ^ 1);
    buf ^= 1;
  }
  }

  if constexpr (RS && kWaitCar) {  // every group's parts are final once the whole collective is
    flow_wait(fw, 0);
    load_rs();
  }
  if constexpr (RS) {
    const int np = min(args.nrm_nparts, 4 * kRsLoads), sub = tid & 3;
#pragma unroll
    for (int h = 0; h < kRsRows; ++h) {
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < kRsLoads; ++q) ss += sub + 4 * q < np ? rs_p[h * kRsLoads + q] : 0.f;
      ss += __shfl_xor(ss, 1, 4);
      ss += __shfl_xor(ss, 2, 4);
      const int row = 64 * h + (tid >> 2);
      if (sub == 0 && row < M) rinv_s[row] = rsqrtf(ss / K + args.eps);
    }
    __syncthreads();
  }

  // C^T tile: rows = W rows (n), cols = m:  acc[t][mt][i] = C[m = 16*mt + r][n = n0 + 16*t + 4*g + i]
  // (kSiluMul with 64-row n-blocks, KR = 1 -- the unsplit 70B TP=8 gate_up -- measured slower and
  // was removed in round 6: profiles/r5_kr1.jsonl)
  static_assert(MODE != kSiluMul || kR == 2, "SiLU: gate and up of the same columns in one wave");
  constexpr bool kSlab = MODE == kPartial || MODE == kAddResNorm || MODE == kQkvRope || MODE == kPush;
  // the in-launch residual update hands its slabs over write-through (measured faster than plain
  // stores + release: tools/gemm_lab.hip o_res / down_res); the plain split-K slabs are read by
  // the next kernel and stay plain (write-through made those slower)
  constexpr bool kSlabSc1 = MODE == kAddResNorm || MODE == kPush || (MODE == kPartial && kProd);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = 16 * mt + r;
    if (m >= M) continue;
    if constexpr (RS) {  // folded RMSNorm: x W^T = rinv[m] * (residual (W diag(w))^T)
      const float sc = rinv_s[m];
#pragma unroll
      for (int t = 0; t < kR; ++t) acc[t][mt] *= sc;
    }
    if constexpr (kSlab) {
      float* p = args.partial + (static_cast<int64_t>(split) * args.M + row0 + m) * N + n0 + 4 * g;
      if constexpr (kSlabSc1) {
        // write-through (sc1) stores: the slab lines leave the XCD L2 clean, so the split-K
        // hand-off needs no release fence (an L2 write-back per workgroup, guide §5 "In-launch
        // split-K reduction"); slabs are < 2 GiB: 32-bit buffer offsets
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(args.partial, static_cast<short>(0), 0x7ffffff0, 0x00020000);
        const int boff = static_cast<int>((p - args.partial) * 4);
#pragma unroll
        for (int t = 0; t < kR; ++t)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[t][mt]), rsrc, boff + 64 * t, 0, 16);
      } else {
#pragma unroll
        for (int t = 0; t < kR; ++t) *reinterpret_cast<f32x4*>(p + 16 * t) = acc[t][mt];
      }
    } else if constexpr (MODE == kBF16) {
      bf16_t* o = args.out + static_cast<int64_t>(row0 + m) * args.ldo + n0 + 4 * g;
#pragma unroll
      for (int t = 0; t < kR; ++t) {
        uint2 v;
        v.x = pack2(acc[t][mt][0], acc[t][mt][1]);
        v.y = pack2(acc[t][mt][2], acc[t][mt][3]);
        *reinterpret_cast<uint2*>(o + 16 * t) = v;
      }
    } else {  // kSiluMul: tile 0 = gate, tile 1 = up of the same 16 columns
      bf16_t* o = args.out + static_cast<int64_t>(row0 + m) * args.ldo + (n0 >> 1) + 4 * g;
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = rbf(silu(rbf(acc[0][mt][i]))) * rbf(acc[1][mt][i]);
      uint2 v;
      v.x = pack2(y[0], y[1]);
      v.y = pack2(y[2], y[3]);
      if constexpr (kProd) {  // handed off in-launch: write-through (sc1) stores
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(args.out, static_cast<short>(0), 0x7ffffff0, 0x00020000);
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{v.x, v.y}, rsrc, static_cast<int>((o - args.out) * 2), 0, 16);
      } else {
        *reinterpret_cast<uint2*>(o) = v;
      }
    }
  }
  if constexpr ((MODE == kSiluMul || MODE == kPartial) && kProd)  // output columns of n-block nb
    flow_signal(fl, flow_slice(fl, nb, MODE == kSiluMul ? 64 * kR / 2 : 64 * kR));
  if constexpr (MODE == kAddResNorm || MODE == kQkvRope || MODE == kPush) {
    // ---- in-launch split-K reduction by the last split of this n-block to arrive
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int last = 1;
      if (S > 1) {
        // write-through (sc1) slabs are already past the XCD L2: no release (L2 write-back) needed
        if constexpr (!kSlabSc1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int t = __hip_atomic_fetch_add(args.counters + nb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == S - 1;
        if (last) __hip_atomic_store(args.counters + nb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (last && !kSlabSc1) {  // write-through slabs are read back with sc1 loads: no acquire
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
    switch (S) {
      case 1: epilogue<MODE, 1, KR>(args, nb); break;
      case 2: epilogue<MODE, 2, KR>(args, nb); break;
      case 4: epilogue<MODE, 4, KR>(args, nb); break;
      case 8: epilogue<MODE, 8, KR>(args, nb); break;
      case 16: epilogue<MODE, 16, KR>(args, nb); break;
      default: epilogue<MODE, 0, KR>(args, nb); break;
    }
  }
}

}  // namespace
