// Weight-streaming "skinny" GEMM for decode: C[M, N] = A[M, K] . W[N, K]^T, M <= 64, bf16.
//
// Decode GEMMs are HBM-bound on W (8B: 436 MB of weights per layer-step, M = batch <= 64), so
// the kernel is built around streaming W once at full rate (guide §5 "GEMV / M <= 16" row:
// operands straight to VGPRs, no LDS round trip, deep unroll):
//   * one wave owns 32 W rows (R = 2 tiles of 16) over a K-slice and computes the transposed
//     tile C^T[32 n x 16*MT m] with mfma_f32_16x16x32_bf16 (A operand = W rows, B operand =
//     activations), so every lane reads 64 contiguous bytes of a W row per 128-deep k-step;
//   * k is permuted inside each 128-step (lane group g owns k in [32g, 32g+32)) identically for
//     W and A, so all operand loads are 16-byte vectors and the dot product is unchanged;
//   * the next k-step's W fragments are issued before the current MFMAs (register double
//     buffer) so ~16 KB per wave stay in flight;
//   * split-K over workgroups when N / 32 alone cannot fill 256 CUs; partial sums are fp32
//     slabs [S, M, N] reduced by the consumer kernel (reduce / reduce+SiLU / reduce+residual+
//     RMSNorm), so a split costs no extra launch on the hot path;
//   * epilogues: bf16 store, fp32 partial store, or fused SiLU(gate)*up when W's gate/up rows
//     are interleaved in blocks of 16 (then one wave holds gate and up of the same columns);
//   * block-packed W (ops/gemm.py pack_weight): per (128-row n-block, 128-deep k-step) the 32 KiB
//     a workgroup consumes are contiguous, as 32 MFMA A-fragments of 1 KiB in lane order, so
//     every wave load instruction reads 1 KiB and a workgroup sweeps one linear stream
//     (tools/gemm_lab.hip: LM head 5.1 -> 5.9 TB/s with non-temporal loads).
#include <type_traits>

#include "common.h"

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
};

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

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
enum Mode { kBF16 = 0, kPartial = 1, kSiluMul = 2, kAddResNorm = 3, kQkvRope = 4 };
constexpr int kMaxRows = 1024;  // decode batch bound of the row-tiled modes
constexpr int kPartCols = 512;  // columns per sum-of-squares part (residual_parts_kernel)


__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

// Experiment knobs for tools/gemm_lab.hip (all 0 in the library build; the NO_* ones give
// wrong results and exist only to attribute time).
#ifndef PK_W_DEPTH
#define PK_W_DEPTH 2         // k-steps of W in flight per wave (register ring; 4 measured slower)
#endif
#ifndef PK_SLAB_NT
#define PK_SLAB_NT 0         // non-temporal stores for the fp32 split-K slabs
#endif
#ifndef PK_SLAB_SC1
#define PK_SLAB_SC1 0        // write-through (sc1) buffer stores for the fp32 split-K slabs
#endif
#ifndef PK_LAB_LDS_PAD
#define PK_LAB_LDS_PAD 0     // extra LDS per workgroup (forces one workgroup per CU)
#endif
#ifndef PK_LAB_NO_MFMA
#define PK_LAB_NO_MFMA 0     // no MFMA / LDS reads: the bare W stream
#endif
#ifndef PK_LAB_NO_ASTAGE
#define PK_LAB_NO_ASTAGE 0   // stage A once, no per-chunk barrier
#endif
#ifndef PK_LAB_NO_SLAB
#define PK_LAB_NO_SLAB 0     // skip the fp32 split-K slab stores (timing only)
#endif

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
// LDS of one skinny-GEMM workgroup (passed in, so two roles of one fused launch share it)
template <int MT>
struct SkinnyLds {
  static constexpr int kKA = MT > 4 ? 128 : kKC;  // k per staged A tile
  bf16_t a[2][16 * MT][kKA + 8] __attribute__((aligned(16)));
  float rinv[MT > 4 ? 16 * MT : 64];
  int last;
};

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
};

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
    while (__hip_atomic_load(fl.ready + kFlowPad * slice, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fl.need) {
      __builtin_amdgcn_s_sleep(16);  // ~0.5 us between polls: pollers must not load the memory channel of the line
      if (++spins > (1 << 20)) {
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

template <int MT, int MODE, bool PK, bool NORM, bool NT, bool RS = false, int KR = 2, int FL = 0>
__device__ __forceinline__ void skinny_tile(const GemmArgs& args, const int bx_in, const int by, const int gdx,
                                            SkinnyLds<MT>& L, const Flow& fl) {
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
  if constexpr (RS) {
    const int np = min(args.nrm_nparts, 4 * kRsLoads), sub = tid & 3;
#pragma unroll
    for (int h = 0; h < kRsRows; ++h) {
      const int rr = min(64 * h + (tid >> 2), M - 1);
#pragma unroll
      for (int q = 0; q < kRsLoads; ++q)
        rs_p[h * kRsLoads + q] = args.nrm_parts[min(sub + 4 * q, np - 1) * args.M + row0 + rr];
    }
  }

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
      if constexpr (FL == 2)  // the producers' output, handed off in-launch: sc1 loads
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
    if constexpr (PK_LAB_NO_MFMA) {  // timing only: consume W with one VALU op per register
#pragma unroll
      for (int t = 0; t < kR; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[t][s & (MT - 1)][0] += __builtin_bit_cast(f32x4, wf[t][s])[0];
      return;
    }
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
    load_a(ks(0));
    load_w(wa, ks(0));
    load_w(wb, ks(1));
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
  } else if constexpr (PK_W_DEPTH > 2) {
    // W register ring PK_W_DEPTH k-steps deep (step j = half j&1 of chunk j>>1)
    constexpr int WD = PK_W_DEPTH;
    bf16x8_t wr[WD][kR][4];
    const int nsteps = 2 * nchunks;
    auto ks = [&](int j) { return ck(j >> 1) + (j & 1) * 128; };
    load_a(ck(0));
#pragma unroll
    for (int u = 0; u < WD; ++u) load_w(wr[u], ks(u));
    store_a(0);
    int buf = 0;
    for (int j0 = 0; j0 < nsteps; j0 += WD) {
#pragma unroll
      for (int u = 0; u < WD; ++u) {
        const int j = j0 + u;
        if ((u & 1) == 0) {
          load_a(ck((j >> 1) + 1));
          __syncthreads();
        }
        if (j < nsteps) mma_step(wr[u], buf, (u & 1) * 128);
        load_w(wr[u], ks(j + WD));
        if (u & 1) {
          store_a(buf ^ 1);
          buf ^= 1;
        }
      }
    }
  } else {
  if constexpr (FL == 2) {
    // consumer: this workgroup's first two weight k-steps are requested before the wait, so
    // they stream in while the producers finish; A (the producers' output) is read after it
    load_w(wa, ck(0));
    load_w(wb, ck(0) + 128);
    flow_wait(fl, split);
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
    if constexpr (PK_LAB_NO_ASTAGE) {
      if (c == 0) __syncthreads();
      mma_step(wa, 0, 0);
      load_w(wa, kn);
      mma_step(wb, 0, 128);
      load_w(wb, kn + 128);
      continue;
    }
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
  constexpr bool kSlab = MODE == kPartial || MODE == kAddResNorm || MODE == kQkvRope;
  // the in-launch residual update hands its slabs over write-through (measured faster than plain
  // stores + release: tools/gemm_lab.hip o_res / down_res); the plain split-K slabs are read by
  // the next kernel and stay plain (write-through made those slower)
  constexpr bool kSlabSc1 = MODE == kAddResNorm || PK_SLAB_SC1;
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
      if (PK_LAB_NO_SLAB && args.M > 0) {  // timing only: keep acc live, store nothing
#pragma unroll
        for (int t = 0; t < kR; ++t) asm volatile("" ::"v"(acc[t][mt]));
        continue;
      }
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
        for (int t = 0; t < kR; ++t) {
          const f32x4 v = acc[t][mt];
          if constexpr (PK_SLAB_NT)  // streaming store: no dirty L2 lines left for the launch-end write-back
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p + 16 * t));
          else
            *reinterpret_cast<f32x4*>(p + 16 * t) = v;
        }
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
      if constexpr (FL == 1) {  // handed off in-launch: write-through (sc1) stores
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(args.out, static_cast<short>(0), 0x7ffffff0, 0x00020000);
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{v.x, v.y}, rsrc, static_cast<int>((o - args.out) * 2), 0, 16);
      } else {
        *reinterpret_cast<uint2*>(o) = v;
      }
    }
  }
  if constexpr (MODE == kSiluMul) {
    if constexpr (FL == 1) flow_signal(fl, (nb * 64 * kR / 2) / fl.cols_per_slice);
  }
  if constexpr (MODE == kAddResNorm || MODE == kQkvRope) {
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

template <int MT, int MODE, bool PK, bool NORM, bool NT, bool RS = false, int KR = 2>
__global__ void __launch_bounds__(256, 2) skinny_gemm_kernel(const GemmArgs args) {
  __shared__ SkinnyLds<MT> lds;
#if PK_LAB_LDS_PAD
  __shared__ char lab_pad[PK_LAB_LDS_PAD];  // timing only: force one workgroup per CU
  if (args.M < 0) lab_pad[threadIdx.x] = 1;
#endif
  skinny_tile<MT, MODE, PK, NORM, NT, RS, KR>(args, blockIdx.x, blockIdx.y, gridDim.x, lds, Flow{});
}

// Fused decode MLP (M <= 64): gate_up + SiLU (folded norm, non-temporal packed W) and the down
// projection's split-K slabs in ONE launch of max(gate_up tiles, down tiles) workgroups, one per
// CU: workgroup b runs gate_up tile b (if any), then down tile b (if any).  A down tile streams
// its first weight k-steps, then waits until the gate_up tiles of its K slice have stored h, so
// the down projection's launch boundary and weight ramp overlap the gate_up tail.  Every
// workgroup is resident at once (one per CU) and a gate_up tile never waits: no deadlock.
// (A/B, tools/gpu/mlp_ab.sh: down tiles as workgroups of their own, dispatched after the gate_up
// ones, put two down tiles on some CUs and lost 7 us per layer.)
template <int MT>
__global__ void __launch_bounds__(256, 2) mlp_fused_kernel(const GemmArgs gu, const GemmArgs dn, const Flow fgu,
                                                           const Flow fdn, int n_gu, int n_dn) {
  __shared__ SkinnyLds<MT> lds;
  const int b = blockIdx.x;
  if (b < n_gu) {
    skinny_tile<MT, kSiluMul, true, false, true, true, 2, 1>(gu, b, 0, n_gu, lds, fgu);
    __syncthreads();  // the LDS tiles are reused by the down tile
  }
  if (b < n_dn) skinny_tile<MT, kPartial, true, false, false, false, 2, 2>(dn, b, 0, n_dn, lds, fdn);
}

// x[m] = bf16(bf16(residual[m] * rinv[m]) * w), rinv from the per-row sum-of-squares parts a
// kAddResNorm epilogue wrote (the final RMSNorm of the fused decode chain).  One row per WG.
__global__ void __launch_bounds__(256) norm_apply_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ residual,
                                                         const float* __restrict__ parts, int nparts,
                                                         const bf16_t* __restrict__ w, int M, int H, float eps) {
  const int m = blockIdx.x;
  float ss = 0.f;
  for (int q = 0; q < nparts; ++q) ss += parts[q * M + m];
  const float ri = rsqrtf(ss / H + eps);
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float v[8], wv[8];
    unpack8(*reinterpret_cast<const u32x4*>(residual + static_cast<int64_t>(m) * H + c), v);
    unpack8(*reinterpret_cast<const u32x4*>(w + c), wv);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf(v[j] * ri) * wv[j];
    *reinterpret_cast<u32x4*>(x + static_cast<int64_t>(m) * H + c) = pack8(v);
  }
}

// Sum S fp32 slabs [S, M, N] -> bf16 [M, ldo]; SILU: N = 2I interleaved (16 gate | 16 up).
template <bool SILU>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16_t* __restrict__ out, const float* __restrict__ partial,
                                                            int S, int M, int N, int ldo) {
  const int m = blockIdx.y;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;  // 4-column group
  if (v * 4 >= N) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < S; ++s) {
    const float4 p = *reinterpret_cast<const float4*>(partial + (static_cast<int64_t>(s) * M + m) * N + 4 * v);
    acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
  }
  if (!SILU) {
    uint2 o;
    o.x = pack2(acc.x, acc.y);
    o.y = pack2(acc.z, acc.w);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * ldo + 4 * v) = o;
  } else {
    // column c = 4v; block b = c / 32, within-block j = c % 32; gate if j < 16
    const int c = 4 * v, b = c >> 5, j = c & 31;
    if (j >= 16) return;
    float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) {
      const float4 p = *reinterpret_cast<const float4*>(partial + (static_cast<int64_t>(s) * M + m) * N + c + 16);
      u.x += p.x; u.y += p.y; u.z += p.z; u.w += p.w;
    }
    float g4[4] = {acc.x, acc.y, acc.z, acc.w}, u4[4] = {u.x, u.y, u.z, u.w}, y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = bf2f(f2bf(silu(bf2f(f2bf(g4[i]))))) * bf2f(f2bf(u4[i]));
    uint2 o;
    o.x = pack2(y[0], y[1]);
    o.y = pack2(y[2], y[3]);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * ldo + b * 16 + j) = o;
  }
}

// Residual update of the folded-RMSNorm decode chain: residual[m] += bf16(sum_s partial[s, m])
// (partial == null: residual unchanged) and parts[blk, m] = sum of squares of the new residual
// over columns [512 blk, 512 blk + 512).  The consumer GEMM turns the parts into rinv[m]
// (GemmArgs::row_scale) and streams the RMSNorm weight pre-multiplied into its W, so no
// normalised copy of the residual is ever written.  One wave per (512 columns, row): every lane
// issues its 2 (S + 1) loads at once and the sum of squares is a cross-lane reduction -- no LDS,
// no barrier (this kernel is latency-bound: 64 launches per 8B decode step).
template <int SS>
__global__ void __launch_bounds__(64) residual_parts_kernel(bf16_t* __restrict__ residual,
                                                            const float* __restrict__ partial, int S, int M, int H,
                                                            float* __restrict__ parts) {
  const int blk = blockIdx.x, m = blockIdx.y, lane = threadIdx.x;
  const int c = blk * kPartCols + lane * 4;  // columns c..c+3 and c+256..c+259
  bf16_t* res = residual + static_cast<int64_t>(m) * H + c;
  const uint2 r0 = *reinterpret_cast<const uint2*>(res);
  const uint2 r1 = *reinterpret_cast<const uint2*>(res + 256);
  float v[8] = {bf2f(static_cast<bf16_t>(r0.x & 0xffff)), bf2f(static_cast<bf16_t>(r0.x >> 16)),
                bf2f(static_cast<bf16_t>(r0.y & 0xffff)), bf2f(static_cast<bf16_t>(r0.y >> 16)),
                bf2f(static_cast<bf16_t>(r1.x & 0xffff)), bf2f(static_cast<bf16_t>(r1.x >> 16)),
                bf2f(static_cast<bf16_t>(r1.y & 0xffff)), bf2f(static_cast<bf16_t>(r1.y >> 16))};
  if (partial != nullptr) {
    // the projection output is rounded to bf16 first (as the unfused GEMM would store it)
    const float* src = partial + static_cast<int64_t>(m) * H + c;
    const int64_t slab = static_cast<int64_t>(M) * H;
    const float4 a = slab_sum<SS>(src, slab, S), b = slab_sum<SS>(src + 256, slab, S);
    const float av[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = rbf(rbf(av[i]) + v[i]);
    uint2 o0, o1;
    o0.x = pack2(v[0], v[1]);
    o0.y = pack2(v[2], v[3]);
    o1.x = pack2(v[4], v[5]);
    o1.y = pack2(v[6], v[7]);
    *reinterpret_cast<uint2*>(res) = o0;
    *reinterpret_cast<uint2*>(res + 256) = o1;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if (lane == 0) parts[static_cast<int64_t>(blk) * M + m] = ss;
}

// residual = bf16(residual + bf16(sum_s partial[s])); x = rmsnorm(residual) * w.
// One row per workgroup of H/4 (<= 1024) threads, PER float4 column groups per thread; the S
// slab loads of a group are independent and issued back to back (latency, not bandwidth, is
// what a 64-row reduction fights).
// Optional MoE routing of the normalised row (ROUTE): logits = bf16(x . router[e]) for the E
// experts, softmax, top-k, renormalised weights -> ids[m, k], rw[m, k].  Replaces the router
// GEMM and the top-k softmax kernel of a Mixtral decode layer.
struct RouteArgs {
  const bf16_t* router;  // [E, H]
  int* ids;              // [M, k]
  float* w;              // [M, k]
  int E, k, renorm;
};

template <int PER, int SS, bool ROUTE = false>
__global__ void __launch_bounds__(1024) splitk_add_rmsnorm_kernel(bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
                                                                  const float* __restrict__ partial,
                                                                  const bf16_t* __restrict__ w, int S, int M, int H,
                                                                  float eps, const RouteArgs ra = RouteArgs{}) {
  __shared__ float red[16];
  const int m = blockIdx.x;
  float v[PER][4];
  float ss = 0.f;
  bf16_t* res = residual + static_cast<int64_t>(m) * H;
  const int64_t slab = static_cast<int64_t>(M) * H;
  const float* base = partial + static_cast<int64_t>(m) * H;
  // the norm weight and (ROUTE) the router rows do not depend on the slabs: request them first,
  // so their round trips overlap the slab loads instead of following the row reduction
  constexpr int kRouteE = 8;  // router experts per pass (E <= 8: all of them, prefetched)
  uint2 wpre[PER];
  uint2 rpre[ROUTE ? PER : 1][ROUTE ? kRouteE : 1];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    wpre[i] = *reinterpret_cast<const uint2*>(w + c);
    if constexpr (ROUTE) {
#pragma unroll
      for (int e = 0; e < kRouteE; ++e)
        if (e < ra.E) rpre[i][e] = *reinterpret_cast<const uint2*>(ra.router + static_cast<int64_t>(e) * H + c);
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    float4 acc;
    if constexpr (SS > 0) {
      float4 p[SS];  // all slab loads in flight before the first add
#pragma unroll
      for (int q = 0; q < SS; ++q) p[q] = ld4f(base + q * slab + c);
      acc = p[0];
#pragma unroll
      for (int q = 1; q < SS; ++q) add4(acc, p[q]);
    } else {
      acc = ld4f(base + c);
      for (int q = 1; q < S; ++q) add4(acc, ld4f(base + q * slab + c));
    }
    const uint2 rr = *reinterpret_cast<const uint2*>(res + c);
    // the projection output is rounded to bf16 first (as the unfused GEMM would store it)
    v[i][0] = bf2f(f2bf(bf2f(f2bf(acc.x)) + bf2f(static_cast<bf16_t>(rr.x & 0xffff))));
    v[i][1] = bf2f(f2bf(bf2f(f2bf(acc.y)) + bf2f(static_cast<bf16_t>(rr.x >> 16))));
    v[i][2] = bf2f(f2bf(bf2f(f2bf(acc.z)) + bf2f(static_cast<bf16_t>(rr.y & 0xffff))));
    v[i][3] = bf2f(f2bf(bf2f(f2bf(acc.w)) + bf2f(static_cast<bf16_t>(rr.y >> 16))));
    uint2 o;
    o.x = pack2(v[i][0], v[i][1]);
    o.y = pack2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(res + c) = o;
    ss += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  }
  const float rinv = rsqrtf(block_sum(ss, red) / H + eps);
  bf16_t* xo = x + static_cast<int64_t>(m) * H;
  float xr[ROUTE ? PER : 1][4];  // the written (bf16-rounded) x values, kept for the router
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = 4 * (threadIdx.x + i * blockDim.x);
    const uint2 ww = wpre[i];
    float y[4];
    y[0] = bf2f(f2bf(v[i][0] * rinv)) * bf2f(static_cast<bf16_t>(ww.x & 0xffff));
    y[1] = bf2f(f2bf(v[i][1] * rinv)) * bf2f(static_cast<bf16_t>(ww.x >> 16));
    y[2] = bf2f(f2bf(v[i][2] * rinv)) * bf2f(static_cast<bf16_t>(ww.y & 0xffff));
    y[3] = bf2f(f2bf(v[i][3] * rinv)) * bf2f(static_cast<bf16_t>(ww.y >> 16));
    uint2 o;
    o.x = pack2(y[0], y[1]);
    o.y = pack2(y[2], y[3]);
    *reinterpret_cast<uint2*>(xo + c) = o;
    if constexpr (ROUTE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) xr[i][j] = bf2f(f2bf(y[j]));
    }
  }
  if constexpr (ROUTE) {
    // router logits from the x row still in registers: kRouteE experts per pass, every router
    // load of the pass issued together and the kRouteE wave reductions independent of each
    // other (one expert at a time re-derived x and serialised 8 load + reduce round trips)
    __shared__ float part_s[16][64];
    __shared__ float logit_s[64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int e0 = 0; e0 < ra.E; e0 += kRouteE) {
      float acc[kRouteE];
#pragma unroll
      for (int e = 0; e < kRouteE; ++e) acc[e] = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = 4 * (threadIdx.x + i * blockDim.x);
#pragma unroll
        for (int e = 0; e < kRouteE; ++e) {
          if (e0 + e < ra.E) {
            const uint2 rr = e0 == 0 ? rpre[i][e]
                                     : *reinterpret_cast<const uint2*>(ra.router + static_cast<int64_t>(e0 + e) * H + c);
            acc[e] += xr[i][0] * bf2f(static_cast<bf16_t>(rr.x & 0xffff)) +
                      xr[i][1] * bf2f(static_cast<bf16_t>(rr.x >> 16)) +
                      xr[i][2] * bf2f(static_cast<bf16_t>(rr.y & 0xffff)) +
                      xr[i][3] * bf2f(static_cast<bf16_t>(rr.y >> 16));
          }
        }
      }
#pragma unroll
      for (int e = 0; e < kRouteE; ++e) acc[e] = wave_sum(acc[e]);
      if (lane == 0) {
#pragma unroll
        for (int e = 0; e < kRouteE; ++e)
          if (e0 + e < ra.E) part_s[wid][e0 + e] = acc[e];
      }
    }
    __syncthreads();
    if (threadIdx.x < ra.E) {
      float t = 0.f;
      for (int q = 0; q < nw; ++q) t += part_s[q][threadIdx.x];
      logit_s[threadIdx.x] = bf2f(f2bf(t));  // the router GEMM's bf16 output
    }
    __syncthreads();
    // softmax + top-k with no serial thread: lane e reads every logit, finds its own rank (value
    // descending, lower expert first on ties -- the order a greedy arg-max scan picks) and, when
    // it ranks below k, owns output slot `rank`; the renormalisation sum adds the chosen
    // probabilities in rank order, as the scan did
    __shared__ float psel_s[64];
    const int E = ra.E, e = threadIdx.x;
    int rank = E;
    float pr = 0.f;
    if (e < E) {
      float mx = -INFINITY;
      for (int q = 0; q < E; ++q) mx = fmaxf(mx, logit_s[q]);
      float sum = 0.f;
      for (int q = 0; q < E; ++q) sum += __expf(logit_s[q] - mx);
      const float le = logit_s[e];
      rank = 0;
      for (int q = 0; q < E; ++q) {
        const float lq = logit_s[q];
        rank += (lq > le || (lq == le && q < e)) ? 1 : 0;
      }
      pr = __expf(le - mx) / sum;
      if (rank < ra.k) psel_s[rank] = pr;
    }
    __syncthreads();
    if (rank < ra.k) {
      float wsum = 0.f;
      for (int j = 0; j < ra.k; ++j) wsum += psel_s[j];
      ra.ids[m * ra.k + rank] = e;
      ra.w[m * ra.k + rank] = ra.renorm ? pr / wsum : pr;
    }
  }
}

// Split-K QKV epilogue fused with RoPE and the paged KV write: sum the S fp32 slabs of the
// fused q|k|v projection, round to bf16 (the unfused GEMM output), rotate q and k (neox, fp32
// cos|sin table), write q to q_out [M, nq*128], k to the K cache and v to the transposed V
// cache (slot < 0: padding row, nothing cached).  Replaces reduce + rope_and_cache.
// One wave per (row, head) so M * (nq + 2 nkv) waves cover the chip and every lane issues its
// 2 S slab loads back to back (a per-row workgroup walking heads serially was latency-bound).
template <int SS>
__global__ void __launch_bounds__(256) qkv_reduce_rope_cache_kernel(
    bf16_t* __restrict__ q_out, const float* __restrict__ partial, int S, int M, int nq, int nkv,
    const int* __restrict__ positions, const float* __restrict__ cos_sin, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ slots, int bs) {
  const int nh = nq + 2 * nkv;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= M * nh) return;
  const int m = item / nh, h = item % nh;
  const int lane = threadIdx.x & 63;
  const int N = nh * 128;
  const int64_t slab = static_cast<int64_t>(M) * N;
  const float* base = partial + static_cast<int64_t>(m) * N + h * 128;
  const int slot = slots[m];
  if (h >= nq && slot < 0) return;
  float a, b;
  if constexpr (SS > 0) {
    float va[SS], vb[SS];
#pragma unroll
    for (int s = 0; s < SS; ++s) {
      va[s] = base[s * slab + lane];
      vb[s] = base[s * slab + lane + 64];
    }
    a = va[0];
    b = vb[0];
#pragma unroll
    for (int s = 1; s < SS; ++s) {
      a += va[s];
      b += vb[s];
    }
  } else {
    a = 0.f;
    b = 0.f;
    for (int s = 0; s < S; ++s) {
      a += base[s * slab + lane];
      b += base[s * slab + lane + 64];
    }
  }
  if (h < nq + nkv) {
    a = rbf(a);
    b = rbf(b);
    const float* cs = cos_sin + static_cast<int64_t>(positions[m]) * 128;
    const float co = cs[lane], si = cs[64 + lane];
    if (h < nq) {
      bf16_t* d = q_out + static_cast<int64_t>(m) * nq * 128 + h * 128;
      d[lane] = f2bf(a * co - b * si);
      d[lane + 64] = f2bf(b * co + a * si);
    } else {  // fragment-native K tile (common.h kcache_off)
      bf16_t* d = kc + (static_cast<int64_t>(slot / bs) * nkv + (h - nq)) * bs * 128;
      d[kcache_off(slot % bs, lane)] = f2bf(a * co - b * si);
      d[kcache_off(slot % bs, lane + 64)] = f2bf(b * co + a * si);
    }
  } else {
    bf16_t* d = vc + (static_cast<int64_t>(slot / bs) * nkv + (h - nq - nkv)) * 128 * bs;
    d[vcache_off(slot % bs, lane)] = f2bf(a);
    d[vcache_off(slot % bs, lane + 64)] = f2bf(b);
  }
}

template <int MODE, bool PK, bool NORM, bool NT, bool RS = false, int KR = 2>
int launch(const GemmArgs& a, hipStream_t stream) {
  const dim3 grid((a.N / (64 * KR)) * a.S * a.row_tiles, a.row_offsets != nullptr ? a.groups : 1);
  if (a.tile_rows == 128) {  // row-tiled decode batches above 64 (dispatch: modes 0-2, no norm prologue)
    if constexpr (MODE <= kSiluMul && !NORM) {
      skinny_gemm_kernel<8, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a);
      return PK_CHECK_LAUNCH();
    }
    return -1;
  }
  switch ((min(min(a.M, 64), a.max_group_rows > 0 ? a.max_group_rows : 64) + 15) / 16) {
    case 1: skinny_gemm_kernel<1, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    case 2: skinny_gemm_kernel<2, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    case 3: skinny_gemm_kernel<3, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    case 4: skinny_gemm_kernel<4, MODE, PK, NORM, NT, RS, KR><<<grid, 256, 0, stream>>>(a); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

// non-temporal weight loads are instantiated only for the large single-pass streams
// (bf16 out: LM head; SiLU: gate_up / MoE w13) on the packed layout
template <int MODE, bool NORM>
int launch_pk(const GemmArgs& a, bool packed, bool nt, hipStream_t stream) {
  // the folded-norm row scale is instantiated for the packed decode projections that take it
  // (QKV split-K slabs, gate_up SiLU)
  if constexpr ((MODE == kPartial || MODE == kSiluMul) && !NORM)
    if (a.row_scale) {
      if (!packed) return -1;
      if constexpr (MODE == kSiluMul)
        if (nt) return launch<MODE, true, NORM, true, true>(a, stream);
      return launch<MODE, true, NORM, false, true>(a, stream);
    }
  if (a.row_scale) return -1;
  if constexpr ((MODE == kBF16 || MODE == kSiluMul) && !NORM)
    if (packed && nt) return launch<MODE, true, NORM, true>(a, stream);
  return packed ? launch<MODE, true, NORM, false>(a, stream) : launch<MODE, false, NORM, false>(a, stream);
}

int dispatch(const GemmArgs& args, int mode, hipStream_t stream) {
  if (args.M <= 0) return 0;
  GemmArgs a = args;
  const bool grouped = a.row_offsets != nullptr;
  if (grouped && (a.groups <= 0 || a.max_group_rows <= 0 || a.max_group_rows > kMaxRows || (mode & 7) > kSiluMul ||
                  (mode & 32)))
    return -1;
  // a group (dense: the whole M) above 64 rows: row tiles of 128 (64 when the row scale has more
  // than 16 parts per row) for the modes without an in-launch split-K reduction (its per-n-block
  // tickets would be shared by the row tiles) and without the A-staging norm prologue
  const int rows = grouped ? a.max_group_rows : a.M;
  // (bit 8: 64-row tiles regardless -- tools/bench_gemm_rows.py compares the two)
  a.tile_rows = rows > 64 && !(a.row_scale && a.nrm_nparts > 16) && !(mode & 256) ? 128 : 64;
  a.row_tiles = (rows + a.tile_rows - 1) / a.tile_rows;
  if (rows > 64 && (rows > kMaxRows || (mode & 7) > kSiluMul || (mode & 32))) return -1;
  if (a.N % 128 || a.S < 1 || a.K % (kKC * a.S) || a.lda % 8) return -1;
  const bool packed = (mode & 16) != 0;  // bit 4: W in block-packed layout
  const bool norm = (mode & 32) != 0;    // bit 5: RMSNorm prologue on A
  // bit 6: non-temporal weight loads (hint); not with several row tiles, whose workgroups of one
  // W tile read it through the XCD's L2 one after another
  const bool nt = (mode & 64) != 0 && a.row_tiles == 1;
  const bool half = (mode & 128) != 0;   // bit 7: 64-row n-blocks (KR = 1)
  if (norm && (a.nrm_parts == nullptr || a.nrm_w == nullptr)) return -1;
  if (half) {  // split-K projections only: fp32 slabs or the in-launch residual update
    if (grouped || norm || nt) return -1;
    if (a.row_scale) {  // folded-norm QKV slabs (packed W only)
      if ((mode & 7) != kPartial || !packed || a.nrm_parts == nullptr || a.nrm_nparts < 1 || a.nrm_nparts > 64)
        return -1;
      return launch<kPartial, true, false, false, true, 1>(a, stream);
    }
    if ((mode & 7) == kPartial)
      return packed ? launch<kPartial, true, false, false, false, 1>(a, stream)
                    : launch<kPartial, false, false, false, false, 1>(a, stream);
    if ((mode & 7) == kAddResNorm) {
      if (a.counters == nullptr || a.residual == nullptr || a.sumsq_parts == nullptr) return -1;
      return packed ? launch<kAddResNorm, true, false, false, false, 1>(a, stream)
                    : launch<kAddResNorm, false, false, false, false, 1>(a, stream);
    }
    return -1;
  }
  if (a.row_scale && (grouped || norm || a.nrm_parts == nullptr || a.nrm_nparts < 1 || a.nrm_nparts > 64))
    return -1;
  switch (mode & 7) {
    case kBF16:
      if (a.S != 1 || norm) return -1;
      return launch_pk<kBF16, false>(a, packed, nt, stream);
    case kPartial:
      if (norm) return -1;
      return launch_pk<kPartial, false>(a, packed, nt, stream);
    case kSiluMul:
      if (a.S != 1) return -1;
      return norm ? launch_pk<kSiluMul, true>(a, packed, nt, stream) : launch_pk<kSiluMul, false>(a, packed, nt, stream);
    case kAddResNorm:
      if (norm || a.counters == nullptr || a.residual == nullptr || a.sumsq_parts == nullptr) return -1;
      return launch_pk<kAddResNorm, false>(a, packed, nt, stream);
    case kQkvRope:
      if (a.counters == nullptr || a.N != (a.nq + 2 * a.nkv) * 128 || a.bs <= 0 || a.bs % 32) return -1;
      return norm ? launch_pk<kQkvRope, true>(a, packed, nt, stream) : launch_pk<kQkvRope, false>(a, packed, nt, stream);
    default: return -1;
  }
}

}  // namespace

// mode 0: out bf16 [M, ldo] (S must be 1); 1: partial fp32 [S, M, N]; 2: SiLU-mul of interleaved
// gate/up rows -> out bf16 [M, N/2] (S must be 1); bit 4: block-packed W; bit 6: non-temporal W.
// Requires M <= kMaxRows (> 64: 64-row tiles), N % 128 == 0, K % (256 S) == 0.
PK_EXPORT int pk_skinny_gemm(void* out, void* partial, const void* A, const void* W, int M, int N, int K, int lda,
                             int ldo, int S, int mode, hipStream_t stream) {
  GemmArgs a{};
  a.out = static_cast<bf16_t*>(out);
  a.partial = static_cast<float*>(partial);
  a.A = static_cast<const bf16_t*>(A);
  a.W = static_cast<const bf16_t*>(W);
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldo = ldo; a.S = S;
  if ((mode & 7) > kSiluMul || (mode & 32)) return -1;
  return dispatch(a, mode, stream);
}

// Full-featured entry: modes 0-4 (see Mode), bit 4 packed W, bit 5 RMSNorm prologue, bit 6 NT W.
PK_EXPORT int pk_skinny_gemm_ex(const GemmArgs* args, int mode, hipStream_t stream) {
  return dispatch(*args, mode, stream);
}

// Fused decode MLP (mlp_fused_kernel): gu = gate_up + SiLU (packed, non-temporal, folded norm:
// row_scale + nrm_parts), dn = down split-K slabs (packed) reading gu's output.  flow: a zeroed
// int buffer of >= 128 * 64 + 1 words (64 tickets and 64 consumer counts, 64 words apart, then
// the sticky error word),
// left zeroed by every launch that completes.
PK_EXPORT int pk_mlp_fused(const GemmArgs* gu_in, const GemmArgs* dn_in, int* flow, hipStream_t stream) {
  GemmArgs gu = *gu_in, dn = *dn_in;
  if (gu.M <= 0) return 0;
  if (gu.M > 64 || dn.M != gu.M || gu.N % 128 || gu.K % kKC || !gu.row_scale || gu.nrm_parts == nullptr ||
      gu.nrm_nparts < 1 || gu.nrm_nparts > 64 || gu.out == nullptr || dn.K != gu.N / 2 || dn.N % 128 || dn.S < 1 ||
      dn.S > 64 || dn.K % (kKC * dn.S) || (dn.K / dn.S) % 64 || dn.partial == nullptr || dn.A != gu.out ||
      dn.lda % 8 || gu.lda % 8 || gu.row_offsets != nullptr || dn.row_offsets != nullptr || flow == nullptr)
    return -1;
  gu.S = 1;
  gu.row_tiles = dn.row_tiles = 1;
  gu.tile_rows = dn.tile_rows = 64;
  gu.max_group_rows = dn.max_group_rows = 0;
  int* done = flow + 64 * kFlowPad;
  int* err = flow + 128 * kFlowPad;
  Flow fgu{flow, done, err, 0, 0, dn.K / dn.S, 1};
  Flow fdn{flow, done, err, (dn.K / dn.S) / 64, dn.N / 128, dn.K / dn.S, 2};
  const int n_gu = gu.N / 128, n_dn = (dn.N / 128) * dn.S;
  const dim3 grid(n_gu > n_dn ? n_gu : n_dn);
  switch ((gu.M + 15) / 16) {
    case 1: mlp_fused_kernel<1><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn); break;
    case 2: mlp_fused_kernel<2><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn); break;
    case 3: mlp_fused_kernel<3><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn); break;
    default: mlp_fused_kernel<4><<<grid, 256, 0, stream>>>(gu, dn, fgu, fdn, n_gu, n_dn); break;
  }
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_norm_apply(void* x, const void* residual, const void* parts, int nparts, const void* w, int M,
                            int H, float eps, hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % 8) return -1;
  norm_apply_kernel<<<M, 256, 0, stream>>>(static_cast<bf16_t*>(x), static_cast<const bf16_t*>(residual),
                                           static_cast<const float*>(parts), nparts, static_cast<const bf16_t*>(w), M,
                                           H, eps);
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_gemm_args_size() { return static_cast<int>(sizeof(GemmArgs)); }

PK_EXPORT int pk_splitk_reduce(void* out, const void* partial, int S, int M, int N, int ldo, int silu,
                               hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 4) return -1;
  dim3 grid((N / 4 + 255) / 256, M);
  if (silu)
    splitk_reduce_kernel<true><<<grid, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const float*>(partial), S, M, N, ldo);
  else
    splitk_reduce_kernel<false><<<grid, 256, 0, stream>>>(static_cast<bf16_t*>(out), static_cast<const float*>(partial), S, M, N, ldo);
  return PK_CHECK_LAUNCH();
}

static int add_rmsnorm_launch(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                              float eps, const RouteArgs* ra, hipStream_t stream);

PK_EXPORT int pk_splitk_add_rmsnorm(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                                    float eps, hipStream_t stream) {
  return add_rmsnorm_launch(x, residual, partial, w, S, M, H, eps, nullptr, stream);
}

// ... + MoE routing of every normalised row: ids [M, k] int32, weights [M, k] fp32 (E <= 64).
PK_EXPORT int pk_splitk_add_rmsnorm_route(void* x, void* residual, const void* partial, const void* w, int S, int M,
                                          int H, float eps, const void* router, int E, int k, int renorm, void* ids,
                                          void* rw, hipStream_t stream) {
  if (E > 64 || E < 1 || k > E) return -1;
  const RouteArgs ra{static_cast<const bf16_t*>(router), static_cast<int*>(ids), static_cast<float*>(rw), E, k, renorm};
  return add_rmsnorm_launch(x, residual, partial, w, S, M, H, eps, &ra, stream);
}

static int add_rmsnorm_launch(void* x, void* residual, const void* partial, const void* w, int S, int M, int H,
                              float eps, const RouteArgs* ra, hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % 1024 || H > 8192) return -1;
  auto xx = static_cast<bf16_t*>(x);
  auto rr = static_cast<bf16_t*>(residual);
  auto pp = static_cast<const float*>(partial);
  auto ww = static_cast<const bf16_t*>(w);
  const int threads = H / 4 > 1024 ? 1024 : H / 4;
  auto go = [&](auto per, auto ss) {
    if (ra != nullptr)
      splitk_add_rmsnorm_kernel<decltype(per)::value, decltype(ss)::value, true><<<M, threads, 0, stream>>>(
          xx, rr, pp, ww, S, M, H, eps, *ra);
    else
      splitk_add_rmsnorm_kernel<decltype(per)::value, decltype(ss)::value, false><<<M, threads, 0, stream>>>(
          xx, rr, pp, ww, S, M, H, eps);
  };
  auto go_s = [&](auto per) {
    switch (S) {
      case 4: go(per, std::integral_constant<int, 4>{}); break;
      case 8: go(per, std::integral_constant<int, 8>{}); break;
      default: go(per, std::integral_constant<int, 0>{}); break;
    }
  };
  switch (H / (4 * threads)) {
    case 1: go_s(std::integral_constant<int, 1>{}); break;
    case 2: go_s(std::integral_constant<int, 2>{}); break;
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

// residual [M, H] += sum of the S fp32 slabs [S, M, H] (partial may be null), parts [H/512, M].
PK_EXPORT int pk_residual_parts(void* residual, const void* partial, int S, int M, int H, void* parts,
                                hipStream_t stream) {
  if (M <= 0) return 0;
  if (H % kPartCols || (partial != nullptr && S < 1)) return -1;
  const dim3 grid(H / kPartCols, M);
  auto rs = static_cast<bf16_t*>(residual);
  auto ps = static_cast<const float*>(partial);
  auto qs = static_cast<float*>(parts);
  switch (partial == nullptr ? 0 : S) {
    case 4: residual_parts_kernel<4><<<grid, 64, 0, stream>>>(rs, ps, S, M, H, qs); break;
    case 8: residual_parts_kernel<8><<<grid, 64, 0, stream>>>(rs, ps, S, M, H, qs); break;
    default: residual_parts_kernel<0><<<grid, 64, 0, stream>>>(rs, ps, S, M, H, qs); break;
  }
  return PK_CHECK_LAUNCH();
}

PK_EXPORT int pk_qkv_reduce_rope_cache(void* q_out, const void* partial, int S, int M, int nq, int nkv,
                                       const void* positions, const void* cos_sin, void* k_cache, void* v_cache,
                                       const void* slots, int bs, hipStream_t stream) {
  if (M <= 0) return 0;
  if (bs <= 0 || bs % 32 || S < 1) return -1;
  const int grid = (M * (nq + 2 * nkv) + 3) / 4;
  auto go = [&](auto ss) {
    qkv_reduce_rope_cache_kernel<decltype(ss)::value><<<grid, 256, 0, stream>>>(
        static_cast<bf16_t*>(q_out), static_cast<const float*>(partial), S, M, nq, nkv,
        static_cast<const int*>(positions), static_cast<const float*>(cos_sin), static_cast<bf16_t*>(k_cache),
        static_cast<bf16_t*>(v_cache), static_cast<const int*>(slots), bs);
  };
  switch (S) {
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    case 8: go(std::integral_constant<int, 8>{}); break;
    case 16: go(std::integral_constant<int, 16>{}); break;
    default: go(std::integral_constant<int, 0>{}); break;
  }
  return PK_CHECK_LAUNCH();
}
