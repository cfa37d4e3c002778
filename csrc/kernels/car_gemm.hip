// A TP decode collective and the GEMM that consumes it in ONE launch (the
// consumer side of collective / GEMM overlap).
//
// In the TP decode chain every row-parallel projection (o, down) ends in the fused two-shot
// collective (comm/car_device.h rr2_body: slab sum, xGMI reduce-scatter + all-gather, residual
// add, norm parts), and the NEXT launch -- the folded-norm gate_up after o, the next layer's QKV
// after down -- reads the residual it produced.  That consumer's weights do not depend on the
// collective, so here both run in one grid:
//   * workgroups [0, n_car): the collective, one (row, chunk group) item each, exactly as the
//     standalone kernel (bit-identical residual and parts); the residual / parts stores are
//     write-through and each item takes a ticket on its chunk group (256 W columns of the
//     residual) and on an all-items counter;
//   * workgroups [n_car, n_car + n_tiles): the consumer's split-K tiles (skinny_tile FL & 4):
//     each requests its first weight k-steps, waits only for the chunk groups its K range reads,
//     stages A (the residual) with sc1 loads, streams the rest of its weights, and waits for the
//     whole collective only before applying the row scale rinv (the norm is folded:
//     rinv * (x (W diag w)^T), so the K-chunks are consumed in arrival order).
// One launch boundary per collective less, and the xGMI exchange runs under the consumer's weight
// ramp.  Deadlock-free on a GPU of its own: the collective workgroups are the lowest indices
// (dispatched first) and wait only for their peers' collective workgroups, never for a consumer.
// Ranks sharing one GPU keep the two launches (a rank's spinning consumers could occupy the slots
// another rank's collective needs) -- models/llama.py policy.
#include <cstring>

#include "comm/car_device.h"
#include "skinny_tile.h"

using namespace pk;

namespace {

// PAIRED: workgroup b runs collective item b and then consumer tile b (grid max(n_car, n_tiles),
// about one workgroup per CU -- the fused MLP's pairing); else the two roles are workgroups of
// their own (grid n_car + n_tiles: the tiles request their weights while the collective runs, but
// two tiles can land on one CU whose neighbour holds only a finished collective item).
template <int W, int MT, int KR, bool PAIRED>
__global__ void __launch_bounds__(256, 2) car_gemm_kernel(const pkcar::CarDev cd, const float* __restrict__ slabs,
                                                          int S, uint16_t* __restrict__ residual,
                                                          float* __restrict__ parts, int M, int N,
                                                          const pkcar::CarHandoff ho, int n_car, const GemmArgs g,
                                                          const Flow fl, const Flow fw, int n_tiles) {
  __shared__ SkinnyLds<MT> lds;
  const int b = blockIdx.x;
  if constexpr (PAIRED) {
    if (b < n_car) pkcar::rr2_body<W, 256, true>(cd, slabs, S, nullptr, residual, parts, M, N, N, N, b, n_car, ho);
    if (b < n_tiles) {
      __syncthreads();
      skinny_tile<MT, kPartial, true, false, false, true, KR, 4>(g, b, 0, n_tiles, lds, fl, fw);
    }
    return;
  }
  if (b < n_car) {
    pkcar::rr2_body<W, 256, true>(cd, slabs, S, nullptr, residual, parts, M, N, N, N, b, n_car, ho);
    return;
  }
  skinny_tile<MT, kPartial, true, false, false, true, KR, 4>(g, b - n_car, 0, n_tiles, lds, fl, fw);
}

}  // namespace

PK_EXPORT int pk_car_gemm_dev_size() { return static_cast<int>(sizeof(pkcar::CarDev)); }

// car_dev: pkcar::CarDev of this rank (libpk_comm pk_car_device_ctx).  slabs: fp32 [S, M, N] of the
// row-parallel projection; residual [M, N] bf16 (in place), parts [N / 256, M] (two-shot form:
// W >= 4, N % (256 W) == 0).  cons: the folded-norm consumer projection -- kPartial split-K slabs
// into cons->partial, packed W, A = residual (lda = N), row scale from `parts`; kr: its n-block
// height in 64 rows (1: 64-row n-blocks).  flow: int32 >= 97 * 64 + 64 words, zeroed once, left
// zeroed by every launch that completes.
PK_EXPORT int pk_car_gemm(const void* car_dev, const void* slabs, int S, void* residual, void* parts, int M, int N,
                          const GemmArgs* cons, int kr, int paired, int* flow, hipStream_t stream) {
  if (car_dev == nullptr || cons == nullptr || flow == nullptr || slabs == nullptr || residual == nullptr ||
      parts == nullptr)
    return -1;
  pkcar::CarDev cd;
  std::memcpy(&cd, car_dev, sizeof(cd));
  GemmArgs g = *cons;
  const int W = cd.world;
  if (M <= 0) return 0;
  if (W < 4 || W > pkcomm::kMaxRanks || N % (pkcomm::kRrChunk * W) || S < 1 ||
      static_cast<long long>(M) * N * 2 + static_cast<long long>(N / pkcomm::kRrChunk) * M * 4 > cd.data_bytes)
    return -1;
  const int gcols = pkcomm::kRrChunk * W, ngroups = N / gcols;
  const int n_car = M * ngroups;  // one (row, chunk group) item per collective workgroup
  if (ngroups > 32 || n_car > pkcomm::kMaxBlocks) return -1;
  if ((kr != 1 && kr != 2) || g.M != M || M > 64 || g.K != N || g.lda != N || g.A != residual || !g.row_scale ||
      g.nrm_parts != parts || g.nrm_nparts != N / pkcomm::kRrChunk || g.nrm_nparts > 64 || g.partial == nullptr ||
      g.N % (64 * kr) || g.S < 1 || g.K % (kKC * g.S) || g.row_offsets != nullptr)
    return -1;
  const int kper = g.K / g.S;
  // every chunk group is read by the same number of consumer tiles (Flow.consumers)
  if (kper % gcols != 0 && gcols % kper != 0) return -1;
  const int nblocks = g.N / (64 * kr);
  const int n_tiles = nblocks * g.S;
  const int per_group = kper >= gcols ? nblocks : nblocks * (gcols / kper);
  g.row_tiles = 1;
  g.tile_rows = 64;
  g.max_group_rows = 0;
  g.counters = nullptr;
  int* done = flow + 64 * kFlowPad;
  int* err = fused_err_word() != nullptr ? fused_err_word() : flow + 128 * kFlowPad;
  // a consumer waits as long as its collective may wait for a late peer (~1.5 us per poll: ~12 s;
  // past it the sticky word reports the lost hand-off and the grid drains)
  const int spin = fused_spin_limit() < 0 ? fused_spin_limit() : (1 << 23);
  const Flow fl{flow, done, err, M, per_group, gcols, 2, 0, 0, spin};
  const Flow fw{flow + 32 * kFlowPad, done + 32 * kFlowPad, err, n_car, n_tiles, 0, 2, 0, 0, spin};
  const pkcar::CarHandoff ho{flow, flow + 32 * kFlowPad, kFlowPad};
  auto go = [&](auto w, auto mt, auto k) {
    constexpr int WW = decltype(w)::value, MT = decltype(mt)::value, KR = decltype(k)::value;
    const float* sl = static_cast<const float*>(slabs);
    uint16_t* rs = static_cast<uint16_t*>(residual);
    float* ps = static_cast<float*>(parts);
    if (paired)
      car_gemm_kernel<WW, MT, KR, true><<<dim3(n_car > n_tiles ? n_car : n_tiles), 256, 0, stream>>>(
          cd, sl, S, rs, ps, M, N, ho, n_car, g, fl, fw, n_tiles);
    else
      car_gemm_kernel<WW, MT, KR, false><<<dim3(n_car + n_tiles), 256, 0, stream>>>(
          cd, sl, S, rs, ps, M, N, ho, n_car, g, fl, fw, n_tiles);
  };
  auto go_mt = [&](auto w, auto k) {
    switch ((M + 15) / 16) {
      case 1: go(w, std::integral_constant<int, 1>{}, k); break;
      case 2: go(w, std::integral_constant<int, 2>{}, k); break;
      case 3: go(w, std::integral_constant<int, 3>{}, k); break;
      default: go(w, std::integral_constant<int, 4>{}, k); break;
    }
  };
  auto go_k = [&](auto w) {
    if (kr == 1)
      go_mt(w, std::integral_constant<int, 1>{});
    else
      go_mt(w, std::integral_constant<int, 2>{});
  };
  switch (W) {
    case 4: go_k(std::integral_constant<int, 4>{}); break;
    case 8: go_k(std::integral_constant<int, 8>{}); break;
    default: return -3;  // (TP = 5..7 keep the two launches)
  }
  return PK_CHECK_LAUNCH();
}
