// Layout of a TP rank's IPC buffer (custom_allreduce.hip), shared with the decode GEMM's push
// epilogue (kernels/skinny_tile.h kPush), which writes its finished output tiles straight into
// the owner rank's input slot and stamps that rank's push flags.
//
//   [Signals, padded to kSigBytes] [in slot, parity 0] [in slot, parity 1] [result slots x 2]
//
// every slot data_bytes long; the call counter (epoch) of a rank's collectives lives in its own
// Signals, so graph replays stay in step.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pkcomm {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 1024;  // workgroups of one call (flag rows); also the push n-block bound
constexpr int kRrChunk = 256;     // columns per owner chunk of the two-shot fused collective

struct Signals {                                 // at the start of every rank's IPC buffer
  uint32_t flag[kMaxBlocks][kMaxRanks];          // written by peers (remote stores)
  uint32_t flag2[kMaxBlocks][kMaxRanks];         // two-shot: reduce-scatter results published
  uint32_t pflag[kMaxBlocks][kMaxRanks];         // push: [n-block][source rank] tile landed here
  uint32_t epoch[kMaxBlocks];                    // this rank's call counter (all entries equal between calls)
  uint32_t error;                                // device-side copy of the sticky error word
};

constexpr size_t kSigBytes = (sizeof(Signals) + 4095) / 4096 * 4096;
// the flag rows lead the struct (pk_car_create_loopback pre-stamps them in one memset)
static_assert(offsetof(Signals, epoch) == 3 * sizeof(uint32_t) * kMaxBlocks * kMaxRanks, "flag rows first");

// Element offset (bf16) in an owner's input slot of the pushed partial of source rank `src`,
// row r, column x of the owner's local chunk lc: [src][row][local chunk][256 columns].  An owner
// holds the chunks c with c % W == owner (lc = c / W), ngroups = N / 256 / W of them.
__host__ __device__ inline int64_t push_off(int src, int r, int lc, int x, int M, int ngroups) {
  return ((static_cast<int64_t>(src) * M + r) * ngroups + lc) * kRrChunk + x;
}

}  // namespace pkcomm
