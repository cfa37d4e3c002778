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
//   * both operands are staged HBM/L2 -> LDS with 16-byte buffer_load ... lds (no VGPR round trip)
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
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
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
// Measured and deleted: single-buffer-phase variants (round 2, 2-5 % slower).  The 4-wave kernel
// below replaces this one where K % 128 == 0 (profiles/r4_prefill_gemm_4wave.md).
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
  // buffer_load ... lds as in the 4-wave kernel below: constant lane offsets from the tile's A / W
  // base, the k advance in an SGPR, M0 from SALU (no per-load VALU)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const bf16_t* abase = args.A + static_cast<long long>(tl.row0 + tl.m0) * args.lda;
  const bf16_t* wbase = PW ? tl.W + static_cast<long long>(tl.n0 >> 7) * 128 * K : tl.W + static_cast<long long>(tl.n0) * K;
  const auto ars = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(abase), static_cast<short>(0), 0x7ffffff0, 0x00020000);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(wbase), static_cast<short>(0), 0x7ffffff0, 0x00020000);
  unsigned vo[4][2];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int j = 0; j < 2; ++j) vo[p][j] = static_cast<unsigned>(src[p][j] - (p < 2 ? abase : wbase)) * 2u;
  auto stage_piece = [&](int p, int kt) {
    bf16_t* base = lds + (kt & 1) * kStage + p * kPiece + wu * 64 * 8;
    const unsigned off = PW && p >= 2 ? static_cast<unsigned>(kt >> 1) * 32768u + static_cast<unsigned>(kt & 1) * 2048u
                                      : static_cast<unsigned>(kt) * BK * 2u;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(p < 2 ? ars : wrs,
                                               (__attribute__((address_space(3))) void*)(base + j * kRowsPerInstr * BK), 16,
                                               vo[p][j], off, 0, 0);
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

// ---- 4-wave variant (6: row-major W, 7: block-packed W), BK = 64: one wave per SIMD, each wave
// owns a 128 x 128 quadrant of the 256 x 256 tile = 8 x 8 MFMA 16x16x32 accumulators (256 fp32 per
// lane) in AGPRs: the MFMAs are inline asm on "a" operands (hipcc does not keep such an
// accumulator in AGPRs next to the fragment registers on its own).  hipcc neither counts nor pads
// inline asm (guide §5.7): the first k-step takes C = 0, each accumulator's next MFMA is 64 MFMAs
// later, and the epilogue reads the AGPRs 32 wait states after the last MFMA.
// Pipeline: 64-deep k-tiles staged by LDS-DMA (128-byte LDS rows = whole cache lines per row --
// the BK = 32 form of this kernel doubled the L1 -> L2 requests, profiles/r4_prefill_gemm_pmc.md)
// into a 3-slot ring of A pieces and a 2-slot ring of W pieces (5 x 32 KiB = the whole LDS); the
// k-loop runs 32-deep sub-steps u: 64 MFMAs on the fragments of u (register set u & 1) while the
// 16 ds_reads of u + 1 go to the other set.  Before reading the first half of tile t (u odd) each
// wave retires all but the 8 youngest LDS-DMA loads (tile t + 1's A piece stays in flight),
// lgkmcnt(0), one raw barrier; that sub-step then stages tile t + 1's W piece and the next one
// tile t + 2's A piece, one load per 8 MFMAs: W gets two sub-steps to land, A three.  Against all
// 16 loads of tile t + 1 in the odd sub-step of a 2 x 64 KiB double buffer: down -9 %, Mixtral w2
// -14 %, the K = 4096 shapes unchanged (profiles/r6_prefill_gemm_buffer_lds.md).
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8_t& w, const bf16x8_t& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(a));
}
__device__ __forceinline__ void mfma_zero(f32x4& c, const bf16x8_t& w, const bf16x8_t& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(w), "v"(a));
}

constexpr int kW4Threads = 256;

template <bool PW>
__global__ void __launch_bounds__(kW4Threads, 1) prefill_gemm_w4_kernel(const PrefillGemmArgs args) {
  // LDS: a 3-slot ring of A pieces and a 2-slot ring of W pieces, 32 KiB each = 160 KiB (the whole
  // LDS).  The A pieces of tile t + 2 go out one sub-step after the W pieces of tile t + 1, so both
  // streams are spread over the whole tile (one load per 8 MFMAs) and the A loads get three
  // sub-steps to land instead of two.
  constexpr int BK = 64, kPiece = 256 * BK;  // 32 KiB per operand piece
  __shared__ __attribute__((aligned(16))) bf16_t lds[5 * kPiece];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  Tile tl;
  if (!tile_of(args, tl)) return;
  const int K = args.K, U = K / 32, NT = K / BK;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // provably wave-uniform: M0 from SALU

  // LDS-DMA sources: instruction j (0..7) of an operand fills rows 32 j .. 32 j + 31; thread t row
  // 32 j + t / 8, physical chunk t % 8 = logical chunk ^ ((row >> 1) & 7) = ^ ((t >> 4) & 7).
  // Packed W: slot 4 j + w of the W piece = (128-row half h, row tile t, k-block bb) with
  // slot = (8 h + t) * 2 + bb, copied lane-linearly from the packed 128 x 128 blocks.
  const int logical = (tid & 7) ^ ((tid >> 4) & 7);
  const bf16_t* abase = args.A + static_cast<long long>(tl.row0 + tl.m0) * args.lda;
  const bf16_t* wbase = PW ? tl.W + static_cast<long long>(tl.n0 >> 7) * 128 * K : tl.W + static_cast<long long>(tl.n0) * K;
  unsigned avo[8], wvo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = min(tl.m0 + 32 * j + (tid >> 3), tl.rows - 1);  // rows past the group: clamped, never stored
    avo[j] = static_cast<unsigned>((m - tl.m0) * args.lda + logical * 8) * 2u;
    if constexpr (PW) {
      const int slot = 4 * j + w, h = slot >> 4, t = (slot >> 1) & 7, bb = slot & 1;
      wvo[j] = static_cast<unsigned>(h * 128 * K + (t * 4 + bb) * 512 + lane * 8) * 2u;
    } else {
      wvo[j] = static_cast<unsigned>((32 * j + (tid >> 3)) * K + logical * 8) * 2u;
    }
  }
  // The loads are buffer_load ... lds: a per-instruction constant VGPR offset from the tile's base
  // (the resource), the k advance in an SGPR and M0 from SALU, so a load costs no VALU.  The
  // global_load_lds form (a 64-bit address add per load, a readfirstlane for M0) was 4.5-13 %
  // slower on every shape (profiles/r6_prefill_gemm_buffer_lds.md).
  const auto ars = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(abase), static_cast<short>(0), 0x7ffffff0, 0x00020000);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(wbase), static_cast<short>(0), 0x7ffffff0, 0x00020000);
  auto a_slot = [&](int t) { return lds + (t % 3) * kPiece; };
  auto w_slot = [&](int t) { return lds + (3 + (t & 1)) * kPiece; };
  auto stage_a = [&](int j, int t) {  // instruction j of tile t's A piece: wave w's 1 KiB
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        ars, (__attribute__((address_space(3))) void*)(a_slot(t) + wu * 8 * BK + j * 32 * BK), 16, avo[j],
        static_cast<unsigned>(t) * BK * 2u, 0, 0);
  };
  auto stage_w = [&](int j, int t) {
    const unsigned wo = PW ? static_cast<unsigned>(t >> 1) * 32768u + static_cast<unsigned>(t & 1) * 2048u
                           : static_cast<unsigned>(t) * BK * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        wrs, (__attribute__((address_space(3))) void*)(w_slot(t) + wu * 8 * BK + j * 32 * BK), 16, wvo[j], wo, 0, 0);
  };

  // fragment reads of sub-step u: tile u / 2, k-half s = u & 1 (chunk 4 s + g); the swizzle term of
  // row (16 f + r) is (r >> 1) & 7, so fragment f sits at a constant offset
  const int wr = w >> 1, wc = w & 1;
  const int r = lane & 15, g = lane >> 4;
  auto a_off = [&](int s) { return (wr * 128 + r) * BK + (((4 * s + g) ^ ((r >> 1) & 7)) * 8); };
  auto w_off = [&](int s) {
    if constexpr (PW) return (wc * 8 * 2 + s) * 512 + lane * 8;
    return (wc * 128 + r) * BK + (((4 * s + g) ^ ((r >> 1) & 7)) * 8);
  };
  constexpr int kWStride = PW ? 2 * 512 : 16 * BK;  // between the W fragments of one sub-step

  bf16x8_t fa[2][8], fw[2][8];
  f32x4 acc[8][8];  // [n frag][m frag]

  // prologue: tiles 0 and 1 in flight, tile 0 retired, sub-step 0's fragments read
#pragma unroll
  for (int j = 0; j < 8; ++j) stage_a(j, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) stage_w(j, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) stage_a(j, 1);
#pragma unroll
  for (int j = 0; j < 8; ++j) stage_w(j, 1);
  wait_vm<16>();
  barrier();
  {
    const bf16_t* ab = a_slot(0) + a_off(0);
    const bf16_t* wb = w_slot(0) + w_off(0);
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      fw[0][f] = ld8(wb + f * kWStride);
      fa[0][f] = ld8(ab + f * 16 * BK);
    }
  }

  // sub-step u on register set C (= u & 1).  Z: the first (C = 0); BW >= 0: u odd, the next
  // sub-step opens tile (u + 1) / 2 -- retire all but the BW youngest loads (tile t + 1's A pieces
  // may stay in flight), lgkmcnt(0), one raw barrier; NEXT: read sub-step u + 1; LOAD: u odd -> the
  // W piece of tile (u + 3) / 2, u even -> the A piece of tile u / 2 + 2, one load per 8 MFMAs
  auto step = [&](auto Cc, auto Zc, auto Bc, auto Nc, auto Lc, int u) {
    constexpr int C = decltype(Cc)::value, BW = decltype(Bc)::value;
    constexpr bool Z = decltype(Zc)::value, NEXT = decltype(Nc)::value, LOAD = decltype(Lc)::value;
    if constexpr (BW >= 0) wait_vm<BW>();
    // lgkmcnt(0) (visible to hipcc's own waitcnt bookkeeping): this sub-step's fragments, read
    // during the previous one, have long landed -- without it hipcc waits after the first new reads
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if constexpr (BW >= 0) barrier();
    const int un = u + 1;
    const bf16_t* ab = a_slot(un >> 1) + a_off(un & 1);
    const bf16_t* wb = w_slot(un >> 1) + w_off(un & 1);
    const int lt = C == 1 ? (u + 3) >> 1 : (u >> 1) + 2;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mf = 0; mf < 8; ++mf) {
      auto mm = [&](int nf) {
        if constexpr (Z) mfma_zero(acc[nf][mf], fw[C][nf], fa[C][mf]);
        else mfma_acc(acc[nf][mf], fw[C][nf], fa[C][mf]);
      };
      // one memory instruction per MFMA pair at most, pinned: ds_read W | 2 MFMA | load | 2 MFMA |
      // ds_read A | 4 MFMA
      if constexpr (NEXT) fw[C ^ 1][mf] = ld8(wb + mf * kWStride);
      mm(0);
      mm(1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (LOAD) {
        if constexpr (C == 1) stage_w(mf, lt);
        else stage_a(mf, lt);
      }
      mm(2);
      mm(3);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NEXT) fa[C ^ 1][mf] = ld8(ab + mf * 16 * BK);
      mm(4);
      mm(5);
      mm(6);
      mm(7);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using W8 = std::integral_constant<int, 8>;
  using W0 = std::integral_constant<int, 0>;
  using NB = std::integral_constant<int, -1>;
  using T = std::true_type;
  using F = std::false_type;
  // U = K / 32 is a multiple of 4 (launcher: K % 128 == 0), NT = U / 2 tiles.  Sub-step 0 stages
  // A(2); each loop pair u, u + 1 stages W((u + 3) / 2) and A((u + 1) / 2 + 2); the pair at U - 5
  // has no A left to stage, and the barrier at U - 3 retires everything.
  if (NT > 2) step(I0{}, T{}, NB{}, T{}, T{}, 0);
  else step(I0{}, T{}, NB{}, T{}, F{}, 0);
  for (int u = 1; u < U - 5; u += 2) {
    step(I1{}, F{}, W8{}, T{}, T{}, u);
    step(I0{}, F{}, NB{}, T{}, T{}, u + 1);
  }
  if (U >= 8) {
    step(I1{}, F{}, W8{}, T{}, T{}, U - 5);
    step(I0{}, F{}, NB{}, T{}, F{}, U - 4);
  }
  step(I1{}, F{}, W0{}, T{}, F{}, U - 3);
  step(I0{}, F{}, NB{}, T{}, F{}, U - 2);
  step(I1{}, F{}, NB{}, F{}, F{}, U - 1);

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
    case 4: prefill_gemm_deep_kernel<false><<<grid, kThreads, 0, stream>>>(a); break;
    case 5: prefill_gemm_deep_kernel<true><<<grid, kThreads, 0, stream>>>(a); break;  // block-packed W
    case 6: prefill_gemm_w4_kernel<false><<<grid, kW4Threads, 0, stream>>>(a); break;
    case 7: prefill_gemm_w4_kernel<true><<<grid, kW4Threads, 0, stream>>>(a); break;  // block-packed W
    default: return -1;
  }
  return PK_CHECK_LAUNCH();
}

}  // namespace

// variant: 6 / 7 = the 4-wave kernel (default; K % 128 == 0), 4 / 5 = the 8-wave kernel (K % 64 ==
// 0 fallback), row-major / block-packed W (packed: K % 128 == 0).  Requires N % 256 == 0, K % 64 == 0,
// 16-byte aligned rows (lda % 8 == 0, K % 8 == 0, ldc % 4 == 0).
PK_EXPORT int pk_prefill_gemm(const PrefillGemmArgs* a, int variant, hipStream_t stream) {
  if (a->M <= 0 || a->tiles_m <= 0) return 0;
  if (a->N % kBN || a->K % 64 || a->lda % 8 || a->ldc % 4) return -1;
  if ((variant == 5 || variant >= 6) && a->K % 128) return -1;
  if (a->row_offsets != nullptr && a->groups <= 0) return -1;
  if (a->row_offsets == nullptr && a->tiles_m != (a->M + kBM - 1) / kBM) return -1;
  return launch(*a, variant, stream);
}

PK_EXPORT int pk_prefill_gemm_args_size() { return static_cast<int>(sizeof(PrefillGemmArgs)); }
