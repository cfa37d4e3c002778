// Step channel implementation + pybind11 face (see step_channel.h).
#include "runtime/step_channel.h"
#include "runtime/proc.h"

#include <errno.h>
#include <fcntl.h>
#include <immintrin.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

namespace pk {

namespace {
constexpr uint64_t kMagic = 0x706b73746570636bULL;  // "pkstepck"

size_t slot_stride(uint64_t slot_bytes) { return (sizeof(SlotHead) + slot_bytes + 63) / 64 * 64; }

// Spin briefly (a decode step is a few ms; the next one is usually published within µs of the
// consumer asking), then back off to short sleeps so an idle engine costs no CPU.
class Backoff {
 public:
  explicit Backoff(int64_t timeout_ms)
      : t0_(std::chrono::steady_clock::now()), timeout_(std::chrono::milliseconds(timeout_ms)) {}
  // false once the timeout has passed
  bool wait() {
    ++n_;
    if (n_ < 4096) {
      _mm_pause();
      return true;
    }
    if (std::chrono::steady_clock::now() - t0_ > timeout_) return false;
    // the leader publishes step k+1 while the GPUs still run step k, so a ~60 µs wake-up
    // latency is hidden; sleeping (not yielding) leaves the cores to the leader's host work
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    return true;
  }
  // true every ~10 ms of sleeping: time for a (cheap, but not free) peer liveness probe
  bool probe_due() const { return n_ >= 4096 && (n_ - 4096) % 512 == 0; }

 private:
  std::chrono::steady_clock::time_point t0_;
  std::chrono::milliseconds timeout_;
  uint64_t n_ = 0;
};


}  // namespace

StepChannelCore::StepChannelCore(const std::string& name, bool create, int nslots, int nconsumers,
                                 uint64_t slot_bytes, int consumer_index)
    : name_(name), owner_(create), index_(consumer_index) {
  if (name.empty() || name[0] != '/') throw std::invalid_argument("step channel name must start with '/'");
  int fd;
  if (create) {
    if (nslots < 2 || nconsumers < 0 || nconsumers > kMaxConsumers || slot_bytes == 0)
      throw std::invalid_argument("step channel: bad geometry");
    bytes_ = sizeof(StepChannelHeader) + static_cast<size_t>(nslots) * slot_stride(slot_bytes);
    shm_unlink(name.c_str());  // a stale segment of a crashed run
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
    if (ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
      ::close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("ftruncate failed for " + name);
    }
  } else {
    fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(attach) failed for " + name);
    struct stat st {};
    if (fstat(fd, &st) != 0 || st.st_size < static_cast<off_t>(sizeof(StepChannelHeader))) {
      ::close(fd);
      throw std::runtime_error("step channel segment too small: " + name);
    }
    bytes_ = static_cast<size_t>(st.st_size);
  }
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mmap failed for " + name);
  hdr_ = static_cast<StepChannelHeader*>(p);
  if (create) {
    std::memset(p, 0, bytes_);
    hdr_->nslots = static_cast<uint32_t>(nslots);
    hdr_->nconsumers = static_cast<uint32_t>(nconsumers);
    hdr_->slot_bytes = slot_bytes;
    hdr_->producer_pid = static_cast<int32_t>(getpid());
    for (auto& c : hdr_->consumer_pid) c.store(0, std::memory_order_relaxed);
    hdr_->seq.store(0, std::memory_order_relaxed);
    hdr_->closed.store(0, std::memory_order_relaxed);
    for (auto& a : hdr_->acked) a.store(0, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    __atomic_store_n(&hdr_->magic, kMagic, __ATOMIC_RELEASE);
  } else {
    if (__atomic_load_n(&hdr_->magic, __ATOMIC_ACQUIRE) != kMagic) {
      munmap(p, bytes_);
      throw std::runtime_error("step channel not initialised: " + name);
    }
    if (consumer_index < 0 || consumer_index >= static_cast<int>(hdr_->nconsumers)) {
      munmap(p, bytes_);
      throw std::invalid_argument("step channel: consumer index out of range");
    }
    // a consumer that attaches late starts at the next step to be published
    next_ = hdr_->seq.load(std::memory_order_acquire) + 1;
    hdr_->consumer_pid[consumer_index].store(static_cast<int32_t>(getpid()), std::memory_order_release);
  }
}

StepChannelCore::~StepChannelCore() {
  if (hdr_ != nullptr) munmap(hdr_, bytes_);
  if (owner_ && !unlinked_) shm_unlink(name_.c_str());
}

SlotHead* StepChannelCore::slot(uint64_t seq) const {
  char* base = reinterpret_cast<char*>(hdr_) + sizeof(StepChannelHeader);
  return reinterpret_cast<SlotHead*>(base + (seq % hdr_->nslots) * slot_stride(hdr_->slot_bytes));
}

uint64_t StepChannelCore::published() const { return hdr_->seq.load(std::memory_order_acquire); }

bool StepChannelCore::publish(const void* data, uint64_t nbytes, int64_t timeout_ms) {
  if (!owner_) throw std::logic_error("publish on a consumer end");
  if (nbytes > hdr_->slot_bytes) throw std::invalid_argument("step larger than a channel slot");
  const uint64_t s = hdr_->seq.load(std::memory_order_relaxed) + 1;
  // the slot last held step s - nslots: every consumer must have copied it out
  if (s > hdr_->nslots) {
    const uint64_t need = s - hdr_->nslots;
    Backoff bo(timeout_ms);
    for (uint32_t c = 0; c < hdr_->nconsumers; ++c)
      while (hdr_->acked[c].load(std::memory_order_acquire) < need) {
        if (!bo.wait()) return false;
        if (bo.probe_due() && !pid_alive(hdr_->consumer_pid[c].load(std::memory_order_acquire))) return false;
      }
  }
  SlotHead* sh = slot(s);
  std::memcpy(reinterpret_cast<char*>(sh) + sizeof(SlotHead), data, nbytes);
  sh->seq = s;
  sh->nbytes = nbytes;
  hdr_->seq.store(s, std::memory_order_release);
  return true;
}

int64_t StepChannelCore::consume(void* dst, uint64_t cap, int64_t timeout_ms) {
  if (owner_) throw std::logic_error("consume on the producer end");
  Backoff bo(timeout_ms);
  while (hdr_->seq.load(std::memory_order_acquire) < next_) {
    if (hdr_->closed.load(std::memory_order_acquire)) return -2;
    if (!bo.wait()) return pid_alive(hdr_->producer_pid) ? -1 : -3;
    if (bo.probe_due() && !pid_alive(hdr_->producer_pid)) return -3;
  }
  const SlotHead* sh = slot(next_);
  if (sh->seq != next_) throw std::runtime_error("step channel overrun (consumer fell a full ring behind)");
  if (sh->nbytes > cap) throw std::invalid_argument("destination smaller than the published step");
  std::memcpy(dst, reinterpret_cast<const char*>(sh) + sizeof(SlotHead), sh->nbytes);
  const int64_t n = static_cast<int64_t>(sh->nbytes);
  hdr_->acked[index_].store(next_, std::memory_order_release);
  ++next_;
  return n;
}

int StepChannelCore::dead_consumer() const {
  for (uint32_t c = 0; c < hdr_->nconsumers; ++c) {
    const int32_t pid = hdr_->consumer_pid[c].load(std::memory_order_acquire);
    if (pid > 0 && !pid_alive(pid)) return static_cast<int>(c);
  }
  return -1;
}

bool StepChannelCore::producer_alive() const { return pid_alive(hdr_->producer_pid); }

void StepChannelCore::unlink() {
  if (owner_ && !unlinked_) shm_unlink(name_.c_str());
  unlinked_ = true;
}

void StepChannelCore::close() {
  if (owner_) hdr_->closed.store(1, std::memory_order_release);
}

}  // namespace pk

namespace py = pybind11;

void bind_step_channel(py::module_& m) {
  py::class_<pk::StepChannelCore>(m, "StepChannel")
      .def(py::init<const std::string&, bool, int, int, uint64_t, int>(), py::arg("name"), py::arg("create"),
           py::arg("nslots") = 4, py::arg("nconsumers") = 0, py::arg("slot_bytes") = 0, py::arg("consumer_index") = -1)
      .def(
          "publish",
          [](pk::StepChannelCore& c, py::buffer b, uint64_t nbytes, int64_t timeout_ms) {
            py::buffer_info bi = b.request();
            const uint64_t have = static_cast<uint64_t>(bi.size) * static_cast<uint64_t>(bi.itemsize);
            if (nbytes > have) throw std::invalid_argument("nbytes larger than the buffer");
            py::gil_scoped_release nogil;
            return c.publish(bi.ptr, nbytes, timeout_ms);
          },
          py::arg("buf"), py::arg("nbytes"), py::arg("timeout_ms") = 600000)
      .def(
          "consume",
          [](pk::StepChannelCore& c, py::buffer b, int64_t timeout_ms) {
            py::buffer_info bi = b.request(true);
            const uint64_t cap = static_cast<uint64_t>(bi.size) * static_cast<uint64_t>(bi.itemsize);
            py::gil_scoped_release nogil;
            return c.consume(bi.ptr, cap, timeout_ms);
          },
          py::arg("buf"), py::arg("timeout_ms") = 1000)
      .def("close", &pk::StepChannelCore::close)
      .def("unlink", &pk::StepChannelCore::unlink)
      .def("dead_consumer", &pk::StepChannelCore::dead_consumer)
      .def_property_readonly("producer_alive", &pk::StepChannelCore::producer_alive)
      .def_property_readonly("published", &pk::StepChannelCore::published)
      .def_property_readonly("next_to_consume", &pk::StepChannelCore::next_to_consume)
      .def_property_readonly("slot_bytes", &pk::StepChannelCore::slot_bytes)
      .def_property_readonly("nslots", &pk::StepChannelCore::nslots)
      .def_property_readonly("name", &pk::StepChannelCore::name);
}
