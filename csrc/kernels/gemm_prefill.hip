// Prefill GEMM on MFMA: C[M, N] = A[M, K] . W[N, K]^T, bf16 in, fp32 accumulate, bf16 out, for
// prefill-sized M (hundreds to tens of thousands of rows), dense or grouped by expert.
//
// Why a hand-written kernel next to hipBLASLt: the Mixtral prefill runs one GEMM per expert over
// that expert's routed rows, and the row counts live on the device (ops/moe.py align).  A
// library call needs them on the host (a read-back per layer, then E launches); this kernel
// reads the group offsets itself, so the whole MoE layer is launch-count constant and
// graph-capturable (SURVEY.md §2.3 grouped_gemm: per-expert GEMM over variable row counts).
//
// Structure (guide §5 "Canonical CDNA GEMM", 256x256 tile row of the glds table):
//   * workgroup tile 256 (m) x 256 (n), 8 waves as 2 (m) x 4 (n), each wave 128 x 64 outputs
//     = 8 x 4 MFMA 16x16x32 bf16 accumulators (128 fp32 registers per lane);
//   * both operands are staged HBM/L2 -> LDS with 16-byte global_load_lds (no VGPR round trip),
//     NSTAGE-deep ring of BK-deep k-tiles (BK 64 x 2 stages or BK 32 x 4 stages = 128 KiB),
//     one raw s_barrier per k-tile and a counted vmcnt that keeps the younger tiles in flight;
//   * LDS rows are 64 / 32 bf16; 16-byte chunks are XOR-swizzled by row (chunk ^ (row >> 1) & 7
//     for 128-B rows, chunk ^ (row >> 2) & 3 for 64-B rows: 16 rows hit 16 distinct bank groups), applied to the global SOURCE address because glds writes lane-linear
//     (guide §5.4 rule 21), so the ds_read_b128 fragment reads of 16 rows are conflict-free;
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
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// 16-byte LDS-DMA: lane l's 16 bytes land at lds + 16 l (lds wave-uniform).  Kept in a plain
// (non-template) device function: called directly inside the kernel template, hipcc's host pass
// silently drops the kernel's launch stub (undefined symbol at load time).
__device__ __forceinline__ void glds16(const bf16_t* g, bf16_t* lds) { __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0); }

// buffer-resource forms (same reason: plain functions, not called from the template directly)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const bf16_t* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p), static_cast<short>(0), bytes, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, bf16_t* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ bf16x8_t bld16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

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

template <int BK, int NSTAGE>
__global__ void __launch_bounds__(kThreads, 1) prefill_gemm_kernel(const PrefillGemmArgs args) {
  constexpr int kChunks = BK / 8;              // 16-byte chunks per LDS row
  constexpr int kPiece = 128 * BK;             // elements of one 128-row operand piece
  constexpr int kStage = 4 * kPiece;           // A rows 0-127 | A 128-255 | W 0-127 | W 128-255
  constexpr int kRowsPerInstr = kThreads / kChunks;           // rows one glds instruction covers
  constexpr int kInstrPerPiece = 128 / kRowsPerInstr;
  constexpr int kLoadsPerTile = 4 * kInstrPerPiece;           // glds per thread per k-tile
  constexpr int kSwz = BK == 64 ? 1 : 2;                      // log2(rows per 256-B LDS bank row)
  __shared__ __attribute__((aligned(16))) bf16_t lds[NSTAGE * kStage];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_n = args.N / kBN;

  // ---- tile of this workgroup (XCD remap, then 8-tile-row groups walked down the rows)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = 8 * tiles_n;
  const int gi = L / per_group, first = gi * 8;
  const int gsz = min(args.tiles_m - first, 8);
  int tm = first + (L % per_group) % gsz;
  const int tn = (L % per_group) / gsz;

  int row0 = 0, rows = args.M;
  const bf16_t* W = args.W;
  if (args.row_offsets != nullptr) {  // find the group that owns tile row tm
    int e = 0;
    for (; e < args.groups; ++e) {
      const int lo = args.row_offsets[e], hi = args.row_offsets[e + 1];
      const int t = (hi - lo + kBM - 1) / kBM;
      if (tm < t) {
        row0 = lo;
        rows = hi - lo;
        break;
      }
      tm -= t;
    }
    if (e == args.groups) return;  // surplus workgroup of the tile-row bound
    W += static_cast<long long>(e) * args.w_stride;
  }
  const int m0 = tm * kBM;                   // within the group
  const int n0 = tn * kBN;
  const int K = args.K, nk = K / BK;

  // ---- glds sources: thread t of instruction j covers LDS row j * kRowsPerInstr + t / kChunks,
  // physical chunk t % kChunks = logical chunk ^ swz(row)
  const bf16_t* src[4][kInstrPerPiece];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int j = 0; j < kInstrPerPiece; ++j) {
      const int row = j * kRowsPerInstr + tid / kChunks;
      const int phys = tid % kChunks;
      const int logical = phys ^ ((row >> kSwz) & (kChunks - 1));
      if (p < 2) {
        const int m = min(m0 + p * 128 + row, rows - 1);  // rows past the group: clamped, never stored
        src[p][j] = args.A + static_cast<long long>(row0 + m) * args.lda + logical * 8;
      } else {
        const int n = n0 + (p - 2) * 128 + row;
        src[p][j] = W + static_cast<long long>(n) * K + logical * 8;
      }
    }
  auto issue = [&](int kt, int stage) {
    bf16_t* base = lds + stage * kStage;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < kInstrPerPiece; ++j)
        glds16(src[p][j] + kt * BK, base + p * kPiece + j * kRowsPerInstr * BK + w * 64 * 8);
  };

  // ---- fragment reads: wave (wr, wc) = (w >> 2, w & 3) owns rows wr*128.. and cols wc*64..
  const int wr = w >> 2, wc = w & 3;
  const int r = lane & 15, g = lane >> 4;
  // element offsets inside a stage of the A / W fragment of k-sub s (32-deep), frag f
  auto a_off = [&](int mf, int s) {
    const int row = mf * 16 + r;
    return wr * kPiece + row * BK + (((4 * s + g) ^ ((row >> kSwz) & (kChunks - 1))) * 8);
  };
  auto w_off = [&](int nf, int s) {
    const int row = (wc & 1) * 64 + nf * 16 + r;
    return (2 + (wc >> 1)) * kPiece + row * BK + (((4 * s + g) ^ ((row >> kSwz) & (kChunks - 1))) * 8);
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NSTAGE - 2 < nk) wait_vm<kLoadsPerTile * (NSTAGE - 2)>();
    else wait_vm<0>();
    barrier();  // tile kt landed for every wave; every wave is done reading tile kt - 1's stage
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    const bf16_t* base = lds + (kt % NSTAGE) * kStage;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      bf16x8_t af[8], wf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) wf[f] = *reinterpret_cast<const bf16x8_t*>(base + w_off(f, s));
#pragma unroll
      for (int f = 0; f < 8; ++f) af[f] = *reinterpret_cast<const bf16x8_t*>(base + a_off(f, s));
#pragma unroll
      for (int nf = 0; nf < 4; ++nf)
#pragma unroll
        for (int mf = 0; mf < 8; ++mf)
          acc[nf][mf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nf], af[mf], acc[nf][mf], 0, 0, 0);
    }
  }

  // ---- epilogue: acc[nf][mf][i] = C[m = wr*128 + mf*16 + r][n = wc*64 + nf*16 + 4g + i]
#pragma unroll
  for (int mf = 0; mf < 8; ++mf) {
    const int m = m0 + wr * 128 + mf * 16 + r;
    if (m >= rows) continue;
    bf16_t* crow = args.C + static_cast<long long>(row0 + m) * args.ldc;
    if (args.silu) {
#pragma unroll
      for (int nf = 0; nf < 4; nf += 2) {
        const int col = (n0 + wc * 64 + nf * 16) / 2 + 4 * g;
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = rbf(silu(rbf(acc[nf][mf][i]))) * rbf(acc[nf + 1][mf][i]);
        uint2 v;
        v.x = pack2(y[0], y[1]);
        v.y = pack2(y[2], y[3]);
        *reinterpret_cast<uint2*>(crow + col) = v;
      }
    } else {
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) {
        uint2 v;
        v.x = pack2(acc[nf][mf][0], acc[nf][mf][1]);
        v.y = pack2(acc[nf][mf][2], acc[nf][mf][3]);
        *reinterpret_cast<uint2*>(crow + n0 + wc * 64 + nf * 16 + 4 * g) = v;
      }
    }
  }
}

// ---- ping-pong schedule (guide §5 "The 256² 8-phase template"): the k-tile is split into four
// C-quadrant phases (A half x W half of the 256 x 256 tile, order A0W0, A0W1, A1W1, A1W0, so
// each half's fragments are re-read only when the half changes: 28 ds_reads per k-tile).  In a
// phase every wave reads its quadrant's fragments (R), then runs 16 MFMAs on them (M); the
// waves of the second M-half (wr = 1) run one barrier behind the first, so on each SIMD (waves
// w and w + 4) one wave's MFMAs overlap the other's LDS reads.  Every phase also stages ONE
// 16 KiB operand piece of the next k-tile (A0, W0, W1, A1 in phases 0-3): a piece issued in
// phase p is retired by the vmcnt(2) at the R of phase p + 2 and read from phase p + 3 on; its
// LDS slot was last read in phase p - 2 or earlier (both checked for all four pieces), so two
// LDS buffers suffice and the loads of ~1.5 phases stay in flight across the barriers.
// PW: W is block-packed (ops/gemm.py pack_weight, the decode GEMM's layout): per 128-row
// n-block and 128-deep k-step, 32 row-tile x k-block fragments of 1 KiB in MFMA lane order.  A
// 64-deep half of a k-step is 16 such fragments; they are copied linearly into the W piece
// (fragment f = 2 tile + k-block at f KiB) and every W fragment read is one lane-linear 16-byte
// ds_read -- conflict-free without a swizzle.  So one weight layout serves decode and prefill.
template <bool PW>
__global__ void __launch_bounds__(kThreads, 1) prefill_gemm_pp_kernel(const PrefillGemmArgs args) {
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
        const int f = j * 8 + w;  // fragment of the 64-deep half: row tile f >> 1, k-block f & 1
        src[p][j] = tl.W + static_cast<long long>((tl.n0 >> 7) + (p - 2)) * 128 * K + ((f >> 1) * 4 + (f & 1)) * 512 +
                    lane * 8;
      } else {
        src[p][j] = tl.W + static_cast<long long>(tl.n0 + (p - 2) * 128 + row) * K + logical * 8;
      }
    }
  auto stage_piece = [&](int p, int kt) {
    bf16_t* base = lds + (kt & 1) * kStage + p * kPiece + w * 64 * 8;
    // packed W: k-step kt >> 1 (128 x 128 block of 16384 elements), half kt & 1 (k-blocks 2, 3)
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
  bf16x8_t af[4][2], wf[2][2];
  f32x4 acc[4][2][4];  // [quadrant][n frag][m frag]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: k-tile 0 complete in buffer 0
#pragma unroll
  for (int p = 0; p < 4; ++p) stage_piece(p, 0);
  wait_vm<0>();
  barrier();
  if (wr == 1) barrier();  // the second M-half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  constexpr int kAh[4] = {0, 0, 1, 1}, kWh[4] = {0, 1, 1, 0};
  constexpr int kStagePiece[4] = {0, 2, 3, 1};  // A0, W0, W1, A1 of the next k-tile
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* base = lds + (kt & 1) * kStage;
    const bool more = kt + 1 < nk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // ---- R: retire the piece staged two phases ago, read this quadrant's fragments, stage
      if (more) wait_vm<2>();
      else wait_vm<0>();
      if (q == 0 || q == 2) {
#pragma unroll
        for (int mf = 0; mf < 4; ++mf)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[mf][s] = *reinterpret_cast<const bf16x8_t*>(base + frag(kAh[q], wr * 64 + mf * 16 + r, s));
      }
      if (q != 2) {
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            wf[nf][s] = *reinterpret_cast<const bf16x8_t*>(
                base + (PW ? (2 + kWh[q]) * kPiece + ((wc * 2 + nf) * 2 + s) * 512 + lane * 8
                           : frag(2 + kWh[q], wc * 32 + nf * 16 + r, s)));
      }
      if (more) stage_piece(kStagePiece[q], kt + 1);
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
            acc[q][nf][mf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nf][s], af[mf][s], acc[q][nf][mf], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (wr == 0) barrier();  // equal barrier counts for both halves

  // ---- epilogue: acc[q][nf][mf][i] = C[m = ah*128 + wr*64 + mf*16 + r][n = wh*128 + wc*32 + nf*16 + 4g + i]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const int m = tl.m0 + kAh[q] * 128 + wr * 64 + mf * 16 + r;
      if (m >= tl.rows) continue;
      bf16_t* crow = args.C + static_cast<long long>(tl.row0 + m) * args.ldc;
      const int nb = tl.n0 + kWh[q] * 128 + wc * 32;
      if (args.silu) {  // n frag 0 = gate, 1 = up of the same 16 output columns
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

// ---- deep variant (4 / 5): the ping-pong phases with three 16 KiB pieces in flight instead of
// about one and a half (guide §5 T3+T4: counted vmcnt letting loads span phases is the lever).
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

// ---- 4-wave variant (6: row-major W, 7: block-packed W): one wave per SIMD, each wave owns a
// 128 x 128 quadrant of the 256 x 256 tile = 8 x 8 MFMA 16x16x32 accumulators (256 fp32 per lane),
// the structure hipBLASLt's MT256x256 kernel uses (profiles/r2_prefill_gemm_pmc.md: 0.25 LDS reads
// per MFMA instead of the 8-wave kernels' 0.38-0.44, one wave per SIMD, few barriers).  hipcc does
// not keep a 256-float accumulator in AGPRs next to the fragment registers when it sees the MFMAs
// (round 2: 528 v_accvgpr moves per k-tile), so the MFMAs are inline asm on "a" operands: the
// accumulators never leave the AGPR file.  hipcc neither counts nor pads inline asm (guide §5.7):
//   * the first k-tile's MFMAs take C = 0 (no accumulator initialisation to pad against);
//   * fragments come straight from ds_read (the compiler waits lgkmcnt for asm operands) and
//     each accumulator's next MFMA is 64 MFMAs later (no dependent-MFMA hazard);
//   * the epilogue reads the AGPRs after 32 wait states (s_nop) behind the last MFMA.
// Pipeline: BK = 32, a 4-deep LDS ring of k-tiles (A | W, 32 KiB each, 128 KiB); at k-tile kt
// each wave (1) retires its own LDS-DMA of tile kt + 1 with a counted vmcnt (tiles kt + 2 and
// kt + 3 stay in flight), (2) lgkmcnt(0) + one raw barrier: tile kt + 1 visible to every wave and
// every wave done reading tile kt's slot, (3) runs tile kt's 64 MFMAs from registers, interleaving
// the 16 ds_reads of tile kt + 1's fragments (second register set) and the 8 LDS-DMA loads of
// tile kt + 4 into tile kt's slot.  Tile kt + 4 thus has ~2.5 k-tiles (~2,500 cycles) to land.
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8_t& w, const bf16x8_t& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(a));
}
__device__ __forceinline__ void mfma_zero(f32x4& c, const bf16x8_t& w, const bf16x8_t& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(w), "v"(a));
}

constexpr int kW4Threads = 256;

template <bool PW, bool RS, bool BUF, bool STG>
__global__ void __launch_bounds__(kW4Threads, 1) prefill_gemm_w4_kernel(const PrefillGemmArgs args) {
  constexpr int BK = 32, NS = 4, kSwz = 2;
  constexpr int kPiece = 256 * BK;  // one operand of one k-tile (16 KiB)
  constexpr int kStage = 2 * kPiece;
  __shared__ __attribute__((aligned(16))) bf16_t lds[NS * kStage];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  Tile tl;
  if (!tile_of(args, tl)) return;
  const int K = args.K, nk = K / BK;

  // LDS-DMA sources: instruction j (0..3) of an operand fills LDS rows 64 j .. 64 j + 63, thread t
  // row 64 j + t / 4, physical 16-byte chunk t % 4 = logical chunk ^ (row >> 2 & 3) (64-byte rows:
  // the 16 rows of a fragment read hit 16 distinct bank groups); row-major W likewise, packed W:
  // fragment 4 j + w (128-row block h = f / 8, row tile f % 8) copied lane-linearly
  const int lrow = tid >> 2;
  const int logical = (tid & 3) ^ ((lrow >> kSwz) & 3);
  const bf16_t* asrc[4];
  const bf16_t* wsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = min(tl.m0 + 64 * j + lrow, tl.rows - 1);  // rows past the group: clamped, never stored
    asrc[j] = args.A + static_cast<long long>(tl.row0 + m) * args.lda + logical * 8;
    if constexpr (PW) {
      const int f = 4 * j + w;
      wsrc[j] = tl.W + static_cast<long long>((tl.n0 >> 7) + (f >> 3)) * 128 * K + (f & 7) * 4 * 512 + lane * 8;
    } else {
      wsrc[j] = tl.W + static_cast<long long>(tl.n0 + 64 * j + lrow) * K + logical * 8;
    }
  }
  auto src_of = [&](int j, int kt) {
    const long long wo = PW ? (kt >> 2) * 16384LL + (kt & 3) * 512 : static_cast<long long>(kt) * BK;
    return j < 4 ? asrc[j] + kt * BK : wsrc[j - 4] + wo;
  };
  auto dst_of = [&](int j, int slot) {  // wave w's 1 KiB of instruction j
    return lds + slot * kStage + w * 16 * BK + (j < 4 ? j * 64 * BK : kPiece + (j - 4) * 64 * BK);
  };
  // BUF: the same loads as buffer instructions (32-bit lane offsets, the k offset in an SGPR; A rows
  // past the group read as zeros instead of being clamped)
  const __amdgpu_buffer_rsrc_t arsrc =
      rsrc_of(args.A + static_cast<long long>(tl.row0 + tl.m0) * args.lda,
              static_cast<int>(min(static_cast<long long>(max(tl.rows - tl.m0, 0)) * args.lda * 2, 0x7fffffffLL)));
  const __amdgpu_buffer_rsrc_t wrsrc = rsrc_of(tl.W + static_cast<long long>(PW ? (tl.n0 >> 7) * 128 : tl.n0) * K, 0x7fffffff);
  int avoff[4], wvoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    avoff[j] = ((64 * j + lrow) * args.lda + logical * 8) * 2;
    const int f = 4 * j + w;
    wvoff[j] = PW ? ((f >> 3) * 128 * K + (f & 7) * 4 * 512 + lane * 8) * 2 : ((64 * j + lrow) * K + logical * 8) * 2;
  }
  auto soff_of = [&](int j, int kt) {
    return j < 4 || !PW ? kt * BK * 2 : ((kt >> 2) * 16384 + (kt & 3) * 512) * 2;
  };
  auto stage_one = [&](int j, int kt) {
    if constexpr (BUF) blds16(j < 4 ? arsrc : wrsrc, dst_of(j, kt % NS), j < 4 ? avoff[j] : wvoff[j - 4], soff_of(j, kt));
    else glds16(src_of(j, kt), dst_of(j, kt % NS));
  };
  // RS (register staging): the same LDS image written by ds_write_b128 from two register sets
  bf16x8_t S[2][8];
  auto rs_load = [&](int set, int j, int kt) {
    if constexpr (BUF) S[set][j] = bld16(j < 4 ? arsrc : wrsrc, j < 4 ? avoff[j] : wvoff[j - 4], soff_of(j, kt));
    else S[set][j] = ld8(src_of(j, kt));
  };
  auto rs_write = [&](int set, int j, int slot) { *reinterpret_cast<bf16x8_t*>(dst_of(j, slot) + lane * 8) = S[set][j]; };

  // fragment reads: wave (wr, wc) = (w >> 1, w & 1) owns rows wr*128.. and W rows wc*128..; the
  // swizzle term of row (16 f + r) is (r >> 2) & 3, so fragment f sits at a constant offset
  const int wr = w >> 1, wc = w & 1;
  const int r = lane & 15, g = lane >> 4;
  const int a_lane = (wr * 128 + r) * BK + ((g ^ ((r >> kSwz) & 3)) * 8);
  const int w_lane = PW ? kPiece + wc * 8 * 512 + lane * 8 : kPiece + (wc * 128 + r) * BK + ((g ^ ((r >> kSwz) & 3)) * 8);
  constexpr int kFragStride = PW ? 512 : 16 * BK;

  bf16x8_t fa[2][8], fw[2][8];
  f32x4 acc[8][8];  // [n frag][m frag]

  // prologue: tiles 0..3 in flight, tile 0 retired and read (RS: tiles 0, 1 in LDS, 2, 3 in the
  // register sets)
  if constexpr (RS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) rs_load(0, j, 0), rs_load(1, j, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs_write(0, j, 0), rs_write(1, j, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs_load(0, j, 2), rs_load(1, j, 3);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  } else {
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) stage_one(j, t);
    wait_vm<24>();
  }
  barrier();
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    fw[0][f] = ld8(lds + w_lane + f * kFragStride);
    fa[0][f] = ld8(lds + a_lane + f * 16 * BK);
  }

  // one k-tile from register set C.  Z: the first (C = 0); NEXT: read tile kt + 1 (after retiring
  // it: VM = its younger LDS-DMA loads still in flight); RESTAGE: load tile kt + 4 into kt's slot
  // (RS: into register set C); WR (RS): write register set C (tile kt + 2) into its slot
  // STG: the waves issue their loads at different MFMAs of a group (wave w before MFMA 2 w), so
  // the four waves' 1 KiB requests do not reach the CU's address unit in the same cycles
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto step = [&](auto Pc, auto Cc, auto Zc, auto Nc, auto Rc, auto Vc, auto Wc, int kt) {
    constexpr int C = decltype(Cc)::value, VM = decltype(Vc)::value;
    constexpr bool Z = decltype(Zc)::value, NEXT = decltype(Nc)::value, RESTAGE = decltype(Rc)::value;
    constexpr bool WR = RS && decltype(Wc)::value;
    if constexpr (NEXT) {
      if constexpr (!RS) wait_vm<VM>();
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), visible to hipcc's own waitcnt bookkeeping
      barrier();
    }
    const bf16_t* nb = lds + ((kt + 1) % NS) * kStage;
    auto load = [&](int mf) {
      if constexpr (RS) rs_load(C, mf, kt + NS);
      else stage_one(mf, kt + NS);
    };
    auto groups = [&](auto Pc) {
      constexpr int P = decltype(Pc)::value;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mf = 0; mf < 8; ++mf) {
        if constexpr (NEXT) {
          fw[C ^ 1][mf] = ld8(nb + w_lane + mf * kFragStride);
          fa[C ^ 1][mf] = ld8(nb + a_lane + mf * 16 * BK);
        }
        if constexpr (WR) rs_write(C, mf, (kt + 2) % NS);
        if constexpr (RESTAGE && P < 0) load(mf);
#pragma unroll
        for (int nf = 0; nf < 8; ++nf) {
          if constexpr (RESTAGE && P >= 0) {
            if (nf == 2 * P) {
              __builtin_amdgcn_sched_barrier(0);
              load(mf);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          if constexpr (Z) mfma_zero(acc[nf][mf], fw[C][nf], fa[C][mf]);
          else mfma_acc(acc[nf][mf], fw[C][nf], fa[C][mf]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    groups(Pc);
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using V0 = std::integral_constant<int, 0>;
  using V8 = std::integral_constant<int, 8>;
  using V16 = std::integral_constant<int, 16>;
  using T = std::true_type;
  using F = std::false_type;
  // nk = K / 32 is a multiple of 8 (launcher: K % 256 == 0)
  // the whole k-loop per load position (one code path per wave: no join inside the loop)
  auto run = [&](auto Pc) {
    step(Pc, I0{}, T{}, T{}, T{}, V16{}, T{}, 0);
    step(Pc, I1{}, F{}, T{}, T{}, V16{}, T{}, 1);
    for (int kt = 2; kt < nk - NS; kt += 2) {
      step(Pc, I0{}, F{}, T{}, T{}, V16{}, T{}, kt);
      step(Pc, I1{}, F{}, T{}, T{}, V16{}, T{}, kt + 1);
    }
    step(Pc, I0{}, F{}, T{}, F{}, V16{}, T{}, nk - 4);
    step(Pc, I1{}, F{}, T{}, F{}, V8{}, T{}, nk - 3);
    step(Pc, I0{}, F{}, T{}, F{}, V0{}, F{}, nk - 2);
    step(Pc, I1{}, F{}, F{}, F{}, V0{}, F{}, nk - 1);
  };
  if constexpr (STG) {
    if (wu == 0) run(std::integral_constant<int, 0>{});
    else if (wu == 1) run(std::integral_constant<int, 1>{});
    else if (wu == 2) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 3>{});
  } else {
    run(std::integral_constant<int, -1>{});
  }

  // the last MFMAs' results before any AGPR read (8-pass XDL: 12+ wait states)
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int nf = 0; nf < 8; ++nf)
#pragma unroll
    for (int mf = 0; mf < 8; ++mf) asm volatile("" : "+a"(acc[nf][mf]));

  // acc[nf][mf][i] = C[m = wr*128 + mf*16 + r][n = wc*128 + nf*16 + 4g + i]
#pragma unroll
  for (int mf = 0; mf < 8; ++mf) {
    const int m = tl.m0 + wr * 128 + mf * 16 + r;
    if (m >= tl.rows) continue;
    bf16_t* crow = args.C + static_cast<long long>(tl.row0 + m) * args.ldc;
    const int nb0 = tl.n0 + wc * 128;
    if (args.silu) {  // n frags 2p / 2p + 1 = gate / up of the same 16 output columns
#pragma unroll
      for (int nf = 0; nf < 8; nf += 2) {
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = rbf(silu(rbf(acc[nf][mf][i]))) * rbf(acc[nf + 1][mf][i]);
        uint2 v;
        v.x = pack2(y[0], y[1]);
        v.y = pack2(y[2], y[3]);
        *reinterpret_cast<uint2*>(crow + (nb0 + nf * 16) / 2 + 4 * g) = v;
      }
    } else {
#pragma unroll
      for (int nf = 0; nf < 8; ++nf) {
        uint2 v;
        v.x = pack2(acc[nf][mf][0], acc[nf][mf][1]);
        v.y = pack2(acc[nf][mf][2], acc[nf][mf][3]);
        *reinterpret_cast<uint2*>(crow + nb0 + nf * 16 + 4 * g) = v;
      }
    }
  }
}

int launch(const PrefillGemmArgs& a, int variant, hipStream_t stream) {
  const int grid = a.tiles_m * (a.N / kBN);
  switch (variant) {
    case 6: prefill_gemm_w4_kernel<false, false, false, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 7: prefill_gemm_w4_kernel<true, false, false, false><<<grid, kW4Threads, 0, stream>>>(a); break;  // block-packed W
    case 8: prefill_gemm_w4_kernel<false, true, false, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 9: prefill_gemm_w4_kernel<true, true, false, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 10: prefill_gemm_w4_kernel<false, false, true, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 11: prefill_gemm_w4_kernel<true, false, true, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 12: prefill_gemm_w4_kernel<false, true, true, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 13: prefill_gemm_w4_kernel<true, true, true, false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 14: prefill_gemm_w4_kernel<false, false, false, true><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 15: prefill_gemm_w4_kernel<true, false, false, true><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 16: prefill_gemm_w4_kernel<false, true, true, true><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 17: prefill_gemm_w4_kernel<true, true, true, true><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 0: prefill_gemm_kernel<64, 2><<<grid, kThreads, 0, stream>>>(a); break;
    case 1: prefill_gemm_kernel<32, 4><<<grid, kThreads, 0, stream>>>(a); break;
    case 2: prefill_gemm_pp_kernel<false><<<grid, kThreads, 0, stream>>>(a); break;
    case 3: prefill_gemm_pp_kernel<true><<<grid, kThreads, 0, stream>>>(a); break;  // block-packed W
    case 4: prefill_gemm_deep_kernel<false><<<grid, kThreads, 0, stream>>>(a); break;
    case 5: prefill_gemm_deep_kernel<true><<<grid, kThreads, 0, stream>>>(a); break;  // block-packed W
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

}  // namespace

// variant: 0 = BK 64 x 2 stages, 1 = BK 32 x 4 stages, 2 = ping-pong quadrant phases (BK 64),
// 3 = variant 2 reading block-packed W (K % 128 == 0), 4 / 5 = variants 2 / 3 with three pieces in flight.  Requires N % 256 == 0, K % 64 == 0,
// 16-byte aligned rows (lda % 8 == 0, K % 8 == 0, ldc % 4 == 0).
PK_EXPORT int pk_prefill_gemm(const PrefillGemmArgs* a, int variant, hipStream_t stream) {
  if (a->M <= 0 || a->tiles_m <= 0) return 0;
  if (a->N % kBN || a->K % 64 || a->lda % 8 || a->ldc % 4) return -1;
  if ((variant == 3 || variant == 5) && a->K % 128) return -1;
  if (variant >= 6 && a->K % 256) return -1;
  if (a->row_offsets != nullptr && a->groups <= 0) return -1;
  if (a->row_offsets == nullptr && a->tiles_m != (a->M + kBM - 1) / kBM) return -1;
  return launch(*a, variant, stream);
}

PK_EXPORT int pk_prefill_gemm_args_size() { return static_cast<int>(sizeof(PrefillGemmArgs)); }
