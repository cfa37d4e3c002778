// Step channel: the TP leader hands every engine step's packed inputs to the other ranks of its
// tensor-parallel group through POSIX shared memory (one node: a TP group never leaves the
// xGMI-connected node).
//
// Round 1 broadcast the device staging buffer with a collective and every worker then read the
// step header back to the host (a GPU sync per step before it could launch anything).  Here the
// header and the staging bytes travel host to host: a worker spins on the ring's sequence word,
// copies the slot into its own pinned staging buffer and launches the same graph / kernels as
// the leader without ever waiting for its GPU.  The ring has `nslots` slots; the leader waits
// only when a worker is that many steps behind on the host side.
//
// Layout (all offsets 64-byte aligned):  Header | Slot 0 | Slot 1 | ... ;  Slot = SlotHead | data.
// Memory order: the producer writes the slot, then publishes `seq` with release; a consumer
// acquires `seq`, copies, then releases its `acked` word, which the producer acquires before
// it overwrites that slot.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace pk {

constexpr int kMaxConsumers = 16;

struct alignas(64) StepChannelHeader {
  uint64_t magic;
  uint32_t nslots, nconsumers;
  uint64_t slot_bytes;
  int32_t producer_pid;                     // liveness: a rank that dies is seen by its peers
  alignas(64) std::atomic<uint64_t> seq;    // last published step (1-based; 0 = none)
  alignas(64) std::atomic<uint32_t> closed; // producer gone
  alignas(64) std::atomic<uint64_t> acked[kMaxConsumers];  // per consumer: last step copied out
  alignas(64) std::atomic<int32_t> consumer_pid[kMaxConsumers];  // 0 until that consumer attached
};

struct alignas(64) SlotHead {
  uint64_t seq;
  uint64_t nbytes;
};

class StepChannelCore {
 public:
  // producer: create (and own) the segment; consumer: attach to an existing one by name.
  StepChannelCore(const std::string& name, bool create, int nslots, int nconsumers, uint64_t slot_bytes,
                  int consumer_index);
  ~StepChannelCore();
  StepChannelCore(const StepChannelCore&) = delete;
  StepChannelCore& operator=(const StepChannelCore&) = delete;

  // Producer: copy `nbytes` into the next slot and publish it.  Waits (spinning, then sleeping)
  // while the slot is still unread by some consumer; returns false after `timeout_ms`, or at
  // once when that consumer's process has died.
  bool publish(const void* data, uint64_t nbytes, int64_t timeout_ms);
  // Consumer: wait for the next step and copy it into `dst` (capacity `cap`).  Returns the
  // byte count, -1 on timeout (call again), -2 when the producer closed the channel, -3 when
  // the producer process no longer exists (died without closing: SIGKILL, OOM, crash).
  int64_t consume(void* dst, uint64_t cap, int64_t timeout_ms);
  // Producer side: index of an attached consumer whose process no longer exists, else -1.
  int dead_consumer() const;
  bool producer_alive() const;
  void close();  // producer: wake every consumer with "closed"
  void unlink();  // producer, once every consumer attached: drop the /dev/shm name

  uint64_t published() const;
  uint64_t next_to_consume() const { return next_; }
  uint64_t slot_bytes() const { return hdr_->slot_bytes; }
  int nslots() const { return static_cast<int>(hdr_->nslots); }
  const std::string& name() const { return name_; }

 private:
  SlotHead* slot(uint64_t seq) const;
  std::string name_;
  bool owner_ = false;
  bool unlinked_ = false;
  int index_ = -1;  // consumer index (producer: -1)
  size_t bytes_ = 0;
  StepChannelHeader* hdr_ = nullptr;
  uint64_t next_ = 1;
};

}  // namespace pk
