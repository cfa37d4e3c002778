// Prefill GEMM on MFMA: C[M, N] = A[M, K] . W[N, K]^T, bf16 in, fp32 accumulate, bf16 out, for
// prefill-sized M (hundreds to tens of thousands of rows), dense or grouped by expert.
//
// Why a hand-written kernel next to hipBLASLt: the Mixtral prefill runs one GEMM per expert over
// that expert's routed rows, and the row counts live on the device (ops/moe.py align).  A
// library call needs them on the host (a read-back per layer, then E launches); this kernel
// reads the group offsets itself, so the whole MoE layer is launch-count constant and
// graph-capturable (SURVEY.md §2.3 grouped_gemm: per-expert GEMM over variable row counts).
//
// Structure (guide §5 "Canonical CDNA GEMM" / "The 256² 8-phase template"):
//   * workgroup tile 256 (m) x 256 (n), 8 waves as 2 (m) x 4 (n), each wave 128 x 64 outputs
//     = 8 x 4 MFMA 16x16x32 bf16 accumulators (128 fp32 registers per lane), two waves per SIMD
//     in a ping-pong (one wave's MFMAs cover the other's LDS reads and load issue);
//   * both operands are staged HBM/L2 -> LDS with 16-byte global_load_lds (no VGPR round trip)
//     into two 64-deep k-tile buffers (128 KiB), raw s_barriers and counted vmcnt waits that keep
//     three 16 KiB pieces in flight across the phases;
//   * LDS rows are 64 bf16 (128 B); 16-byte chunks are XOR-swizzled by row (chunk ^ (row >> 1) & 7:
//     16 rows hit 16 distinct bank groups), applied to the global SOURCE address because glds
//     writes lane-linear (guide §5.4 rule 21), so the ds_read_b128 fragment reads are conflict-free;
//   * MFMA A operand = W rows, B operand = activation rows, so each lane ends with 4
//     consecutive output columns of one row (8-byte stores; the fused SiLU epilogue pairs the
//     16-row gate / up blocks of an interleaved gate_up weight inside one wave);
//   * XCD-aware tile order: consecutive workgroups of one XCD take an 8-tile-row x k-column
//     patch, so the XCD's L2 serves the shared A / W k-slices (guide §5.5 T1).
// Grouped mode: rows of group e are [off[e], off[e+1]) of A and C, W of group e at
// W + e * w_stride; the grid covers an upper bound of tile rows and surplus workgroups exit.
#include "common.h"

using namespace pk;

struct PrefillGemmArgs {
  bf16_t* C;                 // [M, ldc] (SiLU: N / 2 columns)
  const bf16_t* A;           // [M, lda]
  const bf16_t* W;           // [N, K] (grouped: [groups, N, K] with w_stride)
  int M, N, K, lda, ldc;
  const int* row_offsets;    // grouped: [groups + 1] on the device; null = dense
  long long w_stride;
  int groups;
  int tiles_m;               // tile rows covered by the grid (grouped: an upper bound)
  int silu;                  // W rows interleaved 16 gate | 16 up: C = SiLU(gate) * up
};

namespace {

constexpr int kBM = 256, kBN = 256, kThreads = 512;

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// 16-byte LDS-DMA: lane l's 16 bytes land at lds + 16 l (lds wave-uniform).  Kept in a plain
// (non-template) device function: called directly inside the kernel template, hipcc's host pass
// silently drops the kernel's launch stub (undefined symbol at load time).
__device__ __forceinline__ void glds16(const bf16_t* g, bf16_t* lds) { __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0); }

__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

// bijective round-robin-XCD -> contiguous remap (guide §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Tile of this workgroup: XCD remap, then 8-tile-row groups walked down the rows (consecutive
// workgroups of one XCD share A / W k-slices through its L2); grouped: the group owning the tile
// row (false: surplus workgroup of the tile-row bound).
struct Tile {
  int row0, rows, m0, n0;
  const bf16_t* W;
};

__device__ __forceinline__ bool tile_of(const PrefillGemmArgs& args, Tile& t) {
  const int tiles_n = args.N / kBN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = 8 * tiles_n;
  const int first = (L / per_group) * 8;
  const int gsz = min(args.tiles_m - first, 8);
  int tm = first + (L % per_group) % gsz;
  const int tn = (L % per_group) / gsz;
  t.row0 = 0;
  t.rows = args.M;
  t.W = args.W;
  if (args.row_offsets != nullptr) {
    int e = 0;
    for (; e < args.groups; ++e) {
      const int lo = args.row_offsets[e], hi = args.row_offsets[e + 1];
      const int n = (hi - lo + kBM - 1) / kBM;
      if (tm < n) {
        t.row0 = lo;
        t.rows = hi - lo;
        break;
      }
      tm -= n;
    }
    if (e == args.groups) return false;
    t.W += static_cast<long long>(e) * args.w_stride;
  }
  t.m0 = tm * kBM;
  t.n0 = tn * kBN;
  return true;
}

// ---- the k-loop: each 64-deep k-tile runs as four C-quadrant phases (A half x W half of the
// 256 x 256 tile); in a phase every wave reads its new fragments (R), stages one 16 KiB operand
// piece of a later k-tile, then runs 16 MFMAs (M); the waves of the second M-half (wr = 1) run
// one barrier behind the first, so on each SIMD (waves w and w + 4) one wave's MFMAs overlap the
// other's reads.  Three pieces stay in flight (guide §5 T3+T4: counted vmcnt letting loads span
// phases is the lever; one and a half measured 2-5 % slower, round 2).
// PW: W is block-packed (ops/gemm.py pack_weight, the decode GEMM's layout): per 128-row n-block
// and 128-deep k-step, 32 row-tile x k-block fragments of 1 KiB in MFMA lane order.  A 64-deep
// half of a k-step is 16 such fragments; they are copied linearly into the W piece (fragment
// f = 2 tile + k-block at f KiB) and every W fragment read is one lane-linear 16-byte ds_read --
// conflict-free without a swizzle.  So one weight layout serves decode and prefill.
// Measured and deleted: single-buffer-phase variants (round 2, 2-5 % slower) and a 4-wave,
// one-wave-per-SIMD kernel with AGPR accumulators (round 4, equal; profiles/r4_prefill_gemm_4wave.md).
// Every wave keeps BOTH W halves of a k-tile in registers (+16 VGPRs), so each operand half is
// read from LDS exactly once per k-tile -- quadrant order A0W0, A0W1, A1W0, A1W1 reads A0+W0,
// W1, A1, nothing -- and its LDS slot frees early: A0 / W0 after phase 0, W1 after 1, A1 after 2.
// The next tiles' pieces go into those slots as soon as the 2-phase WAR distance allows:
//   phase q0: W1(t+1)   q1: A1(t+1)   q2: A0(t+2)   q3: W0(t+2)
// (W1 / A1 of t+1 into the other buffer, last read in phases 1 / 2 of tile t-1; A0 / W0 of t+2
// into this tile's buffer, last read in phase 0).  Each piece is read 5-6 phases after it is
// issued; the R of phase p retires what phase p+1 reads, and in steady state exactly three
// younger pieces (6 loads) have been issued since the oldest one needed: vmcnt(6) everywhere
// (vmcnt(0) in the last two k-tiles, where fewer younger loads exist).  The prologue stages
// tile 0 and A0 / W0 of tile 1 and retires tile 0 (vmcnt(4)).
template <bool PW>
__global__ void __launch_bounds__(kThreads, 1) prefill_gemm_deep_kernel(const PrefillGemmArgs args) {
  constexpr int BK = 64, kChunks = 8, kPiece = 128 * BK, kStage = 4 * kPiece, kSwz = 1;
  constexpr int kRowsPerInstr = kThreads / kChunks;  // 64
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * kStage];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  Tile tl;
  if (!tile_of(args, tl)) return;
  const int K = args.K, nk = K / BK;

  // piece order in LDS: 0 = A rows 0-127, 1 = A 128-255, 2 = W 0-127, 3 = W 128-255
  const bf16_t* src[4][2];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = j * kRowsPerInstr + tid / kChunks;
      const int logical = (tid % kChunks) ^ ((row >> kSwz) & (kChunks - 1));
      if (p < 2) {
        const int m = min(tl.m0 + p * 128 + row, tl.rows - 1);
        src[p][j] = args.A + static_cast<long long>(tl.row0 + m) * args.lda + logical * 8;
      } else if constexpr (PW) {
        const int f = j * 8 + w;
        src[p][j] = tl.W + static_cast<long long>((tl.n0 >> 7) + (p - 2)) * 128 * K + ((f >> 1) * 4 + (f & 1)) * 512 +
                    lane * 8;
      } else {
        src[p][j] = tl.W + static_cast<long long>(tl.n0 + (p - 2) * 128 + row) * K + logical * 8;
      }
    }
  auto stage_piece = [&](int p, int kt) {
    bf16_t* base = lds + (kt & 1) * kStage + p * kPiece + w * 64 * 8;
    const long long off = PW && p >= 2 ? (kt >> 1) * 16384LL + (kt & 1) * 1024 : static_cast<long long>(kt) * BK;
    glds16(src[p][0] + off, base);
    glds16(src[p][1] + off, base + kRowsPerInstr * BK);
  };

  const int wr = w >> 2, wc = w & 3;
  const int r = lane & 15, g = lane >> 4;
  auto frag = [&](int piece, int row, int s) {
    return piece * kPiece + row * BK + (((4 * s + g) ^ ((row >> kSwz) & (kChunks - 1))) * 8);
  };
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
  bf16x8_t af[4][2], wf[2][2][2];  // wf[W half][n frag][k step]
  f32x4 acc[4][2][4];              // [quadrant][n frag][m frag]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < 4; ++p) stage_piece(p, 0);
  if (nk > 1) {
    stage_piece(0, 1);
    stage_piece(2, 1);
    wait_vm<4>();
  } else {
    wait_vm<0>();
  }
  barrier();
  if (wr == 1) barrier();  // the second M-half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  constexpr int kAh[4] = {0, 0, 1, 1}, kWh[4] = {0, 1, 0, 1};
  constexpr int kStagePiece[4] = {3, 1, 0, 2}, kStageAhead[4] = {1, 1, 2, 2};  // W1, A1 of t+1; A0, W0 of t+2
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* base = lds + (kt & 1) * kStage;
    const bool steady = kt + 2 < nk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // ---- R: retire what the next phase reads, read this phase's new operand halves, stage
      if (steady) wait_vm<6>();
      else wait_vm<0>();
      if (q == 0 || q == 2) {
#pragma unroll
        for (int mf = 0; mf < 4; ++mf)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[mf][s] = *reinterpret_cast<const bf16x8_t*>(base + frag(kAh[q], wr * 64 + mf * 16 + r, s));
      }
      if (q < 2) {
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            wf[q][nf][s] = *reinterpret_cast<const bf16x8_t*>(
                base + (PW ? (2 + q) * kPiece + ((wc * 2 + nf) * 2 + s) * 512 + lane * 8
                           : frag(2 + q, wc * 32 + nf * 16 + r, s)));
      }
      if (kt + kStageAhead[q] < nk) stage_piece(kStagePiece[q], kt + kStageAhead[q]);
      barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- M
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
#pragma unroll
          for (int mf = 0; mf < 4; ++mf)
            acc[q][nf][mf] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kWh[q]][nf][s], af[mf][s], acc[q][nf][mf], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (wr == 0) barrier();  // equal barrier counts for both halves

#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const int m = tl.m0 + kAh[q] * 128 + wr * 64 + mf * 16 + r;
      if (m >= tl.rows) continue;
      bf16_t* crow = args.C + static_cast<long long>(tl.row0 + m) * args.ldc;
      const int nb = tl.n0 + kWh[q] * 128 + wc * 32;
      if (args.silu) {
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = rbf(silu(rbf(acc[q][0][mf][i]))) * rbf(acc[q][1][mf][i]);
        uint2 v;
        v.x = pack2(y[0], y[1]);
        v.y = pack2(y[2], y[3]);
        *reinterpret_cast<uint2*>(crow + nb / 2 + 4 * g) = v;
      } else {
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          uint2 v;
          v.x = pack2(acc[q][nf][mf][0], acc[q][nf][mf][1]);
          v.y = pack2(acc[q][nf][mf][2], acc[q][nf][mf][3]);
          *reinterpret_cast<uint2*>(crow + nb + nf * 16 + 4 * g) = v;
        }
      }
    }
}

int launch(const PrefillGemmArgs& a, int variant, hipStream_t stream) {
  const int grid = a.tiles_m * (a.N / kBN);
  switch (variant) {
    case 4: prefill_gemm_deep_kernel<false><<<grid, kThreads, 0, stream>>>(a); break;
    case 5: prefill_gemm_deep_kernel<true><<<grid, kThreads, 0, stream>>>(a); break;  // block-packed W
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

}  // namespace

// variant: 4 = row-major W, 5 = block-packed W (K % 128 == 0); the numbers of the round-2 / round-4
// variants measured slower and deleted (0-3, 6-17) are not reused.  Requires N % 256 == 0, K % 64 == 0,
// 16-byte aligned rows (lda % 8 == 0, K % 8 == 0, ldc % 4 == 0).
PK_EXPORT int pk_prefill_gemm(const PrefillGemmArgs* a, int variant, hipStream_t stream) {
  if (a->M <= 0 || a->tiles_m <= 0) return 0;
  if (a->N % kBN || a->K % 64 || a->lda % 8 || a->ldc % 4) return -1;
  if (variant == 5 && a->K % 128) return -1;
  if (a->row_offsets != nullptr && a->groups <= 0) return -1;
  if (a->row_offsets == nullptr && a->tiles_m != (a->M + kBM - 1) / kBM) return -1;
  return launch(*a, variant, stream);
}

PK_EXPORT int pk_prefill_gemm_args_size() { return static_cast<int>(sizeof(PrefillGemmArgs)); }
