// Vote board: the per-step lockstep vote of DP attention + EP ranks through POSIX shared memory
// ("a device-side (or step-channel) replacement for the per-step gloo vote").
//
// Every rank of an expert-parallel group runs its own scheduler, and each MoE layer is a
// collective over all of them, so before a step the ranks agree on (any rank busy, every rank
// stopping, the largest token count of the step) -- the last picks the expert all-to-all path
// (IPC slots for decode-sized steps, RCCL for prefill) uniformly.  A gloo all-reduce did this in
// ~100 us of host round trips; here each rank posts its numbers into its own cache line and spins
// until every rank has posted the same step (µs on one node), with a bounded wait and a
// liveness probe of the peers' pids, so a dead rank fails the vote instead of hanging it.
// Fields are double-buffered by step parity: a rank can be at most one vote ahead (its next vote
// waits for mine), so it never overwrites the parity I am still reading.
#include "runtime/proc.h"
#include <errno.h>
#include <fcntl.h>
#include <immintrin.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace pk {

constexpr int kVoteMaxRanks = 64;
constexpr uint64_t kVoteMagic = 0x706b766f74656264ULL;  // "pkvotebd"

struct alignas(64) VoteSlot {
  std::atomic<uint64_t> seq;  // last step this rank posted
  int32_t pid;
  int32_t busy[2], stopping[2];
  int64_t ntok[2];
};

struct alignas(64) VoteHeader {
  uint64_t magic;
  int32_t nranks;
  VoteSlot slot[kVoteMaxRanks];
};

class VoteBoard {
 public:
  VoteBoard(const std::string& name, bool create, int nranks, int rank) : name_(name), owner_(create), rank_(rank) {
    if (name.empty() || name[0] != '/') throw std::invalid_argument("vote board name must start with '/'");
    const size_t bytes = sizeof(VoteHeader);
    int fd;
    if (create) {
      if (nranks < 1 || nranks > kVoteMaxRanks) throw std::invalid_argument("vote board: bad rank count");
      shm_unlink(name.c_str());
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
      if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
        ::close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("ftruncate failed for " + name);
      }
    } else {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(attach) failed for " + name);
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed for " + name);
    h_ = static_cast<VoteHeader*>(p);
    if (create) {
      std::memset(p, 0, bytes);
      h_->nranks = nranks;
      __atomic_store_n(&h_->magic, kVoteMagic, __ATOMIC_RELEASE);
    } else if (__atomic_load_n(&h_->magic, __ATOMIC_ACQUIRE) != kVoteMagic) {
      munmap(p, bytes);
      throw std::runtime_error("vote board not initialised: " + name);
    }
    if (rank < 0 || rank >= h_->nranks) throw std::invalid_argument("vote board: rank out of range");
    n_ = h_->nranks;
    h_->slot[rank].pid = static_cast<int32_t>(getpid());
  }
  ~VoteBoard() {
    if (h_ != nullptr) munmap(h_, sizeof(VoteHeader));
    if (owner_ && !unlinked_) shm_unlink(name_.c_str());
  }
  VoteBoard(const VoteBoard&) = delete;
  VoteBoard& operator=(const VoteBoard&) = delete;

  // Owner, once every rank has attached: drop the name so a killed group leaves nothing in
  // /dev/shm (the mappings stay valid).
  void unlink() {
    if (owner_ && !unlinked_) shm_unlink(name_.c_str());
    unlinked_ = true;
  }

  // Post this rank's step numbers and wait for every rank's.  Returns (any busy, all stopping,
  // max ntok).  Throws on timeout or when a peer process has died.
  std::tuple<bool, bool, int64_t> vote(bool busy, bool stopping, int64_t ntok, int64_t timeout_ms) {
    const uint64_t s = ++step_;
    VoteSlot& mine = h_->slot[rank_];
    const int par = static_cast<int>(s & 1);
    mine.busy[par] = busy;
    mine.stopping[par] = stopping;
    mine.ntok[par] = ntok;
    mine.seq.store(s, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    bool any = false, all_stop = true;
    int64_t mx = 0;
    for (int r = 0; r < n_; ++r) {
      VoteSlot& o = h_->slot[r];
      uint64_t spins = 0;
      while (o.seq.load(std::memory_order_acquire) < s) {
        if (++spins < 2048) {
          _mm_pause();
          continue;
        }
        if ((spins & 255) == 0) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
            throw std::runtime_error("vote board: rank " + std::to_string(r) + " did not vote within the timeout");
          const int32_t pid = o.pid;
          if (pid > 0 && !pk::pid_alive(pid))
            throw std::runtime_error("vote board: rank " + std::to_string(r) + " died");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(10));
      }
      any = any || o.busy[par];
      all_stop = all_stop && o.stopping[par];
      mx = std::max<int64_t>(mx, o.ntok[par]);
    }
    return {any, all_stop, mx};
  }
  int nranks() const { return n_; }
  uint64_t step() const { return step_; }

 private:
  std::string name_;
  bool owner_;
  bool unlinked_ = false;
  int rank_;
  int n_ = 0;
  VoteHeader* h_ = nullptr;
  uint64_t step_ = 0;
};

}  // namespace pk

namespace py = pybind11;

void bind_vote_board(py::module_& m) {
  py::class_<pk::VoteBoard>(m, "VoteBoard")
      .def(py::init<const std::string&, bool, int, int>(), py::arg("name"), py::arg("create"), py::arg("nranks"),
           py::arg("rank"))
      .def("unlink", &pk::VoteBoard::unlink)
      .def(
          "vote",
          [](pk::VoteBoard& b, bool busy, bool stopping, int64_t ntok, int64_t timeout_ms) {
            py::gil_scoped_release nogil;
            return b.vote(busy, stopping, ntok, timeout_ms);
          },
          py::arg("busy"), py::arg("stopping") = false, py::arg("ntok") = 0, py::arg("timeout_ms") = 600000)
      .def_property_readonly("nranks", &pk::VoteBoard::nranks)
      .def_property_readonly("step", &pk::VoteBoard::step);
}
