// Shared-memory step channel: the tensor-parallel leader publishes every engine step's inputs and
// the TP workers of the same node read them (the step-schedule broadcast).
//
// Replaces a per-step pickled broadcast_object_list over gloo TCP (two round trips through the
// loopback stack per decode step) with a POSIX shared-memory ring: the leader memcpy's the
// message into slot (seq % nslots), stores its length and releases `seq`; each worker spins on
// `seq` with acquire loads (a few microseconds after publication), copies the slot out and
// releases its own `ack`.  The leader only reuses a slot once every reader has acknowledged the
// message that occupied it, so a slow worker back-pressures the leader instead of reading a torn
// message.  All waits release the Python GIL and are bounded by a timeout (a dead peer surfaces
// as a TimeoutError in the caller, never as a hang).
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "runtime.h"

namespace py = pybind11;

namespace {

constexpr int CHAN_MAX_READERS = 63;
constexpr int CHAN_MAX_SLOTS = 64;

struct alignas(64) ChanHeader {
  uint64_t magic;
  uint64_t nslots, slot_bytes, nreaders;
  alignas(64) std::atomic<uint64_t> seq;  // messages published
  alignas(64) std::atomic<uint64_t> ack[CHAN_MAX_READERS + 1];  // per reader: messages consumed
  alignas(64) std::atomic<uint64_t> beat;  // leader liveness: bumped every second while the leader runs
  uint64_t len[CHAN_MAX_SLOTS];           // byte length of the message in each slot
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "lock-free 64-bit atomics required");
constexpr uint64_t CHAN_MAGIC = 0x6b38736c6c6d6368ull;

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

class StepChannel {
 public:
  // create=true: the leader creates (and later unlinks) the segment; readers open it by name.
  StepChannel(const std::string& name, bool create, int nslots, int64_t slot_bytes, int nreaders)
      : name_(name), owner_(create) {
    if (create) {
      if (nslots < 1 || nslots > CHAN_MAX_SLOTS || nreaders < 0 || nreaders > CHAN_MAX_READERS || slot_bytes < 64)
        throw std::invalid_argument("StepChannel: bad geometry");
      size_ = sizeof(ChanHeader) + (size_t)nslots * (size_t)slot_bytes;
      fd_ = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("shm_open(create) failed for " + name);
      if (ftruncate(fd_, (off_t)size_) != 0) {
        close(fd_);
        shm_unlink(name.c_str());
        throw std::runtime_error("ftruncate failed for " + name);
      }
    } else {
      fd_ = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("shm_open(open) failed for " + name);
      struct stat st;
      if (fstat(fd_, &st) != 0) throw std::runtime_error("fstat failed for " + name);
      size_ = (size_t)st.st_size;
    }
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) {
      close(fd_);
      if (create) shm_unlink(name.c_str());
      throw std::runtime_error("mmap failed for " + name);
    }
    base_ = (uint8_t*)p;
    hdr_ = reinterpret_cast<ChanHeader*>(base_);
    prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);  // idle back-off sleeps wake within microseconds
    if (create) {
      new (hdr_) ChanHeader();
      hdr_->nslots = (uint64_t)nslots;
      hdr_->slot_bytes = (uint64_t)slot_bytes;
      hdr_->nreaders = (uint64_t)nreaders;
      hdr_->seq.store(0, std::memory_order_relaxed);
      for (auto& a : hdr_->ack) a.store(0, std::memory_order_relaxed);
      hdr_->beat.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = CHAN_MAGIC;
    } else if (hdr_->magic != CHAN_MAGIC || size_ < sizeof(ChanHeader) + hdr_->nslots * hdr_->slot_bytes) {
      throw std::runtime_error("StepChannel: " + name + " is not an initialised channel");
    }
  }

  ~StepChannel() { close_(); }

  int64_t slot_bytes() const { return (int64_t)hdr_->slot_bytes; }
  int64_t published() const { return (int64_t)hdr_->seq.load(std::memory_order_acquire); }

  // Leader liveness without a message: an idle leader publishes no step for as long as no request
  // arrives, so its heartbeat thread bumps this word instead; a worker that cannot observe the
  // leader's process (another pid namespace) reads it to tell "idle" from "gone".
  void heartbeat() { hdr_->beat.fetch_add(1, std::memory_order_release); }
  int64_t beats() const { return (int64_t)hdr_->beat.load(std::memory_order_acquire); }

  // Leader: publish one message; waits (GIL released) while its slot still holds a message some
  // reader has not consumed.  False on timeout.
  bool publish(py::buffer data, double timeout_s) {
    py::buffer_info bi = data.request();
    const size_t n = (size_t)bi.size * (size_t)bi.itemsize;
    if (n > hdr_->slot_bytes) throw std::length_error("StepChannel: message larger than a slot");
    const uint64_t s = hdr_->seq.load(std::memory_order_relaxed);
    const uint64_t nslots = hdr_->nslots;
    {
      py::gil_scoped_release nogil;
      if (s >= nslots && !wait_acks(s + 1 - nslots, timeout_s)) return false;
      const uint64_t slot = s % nslots;
      std::memcpy(base_ + sizeof(ChanHeader) + slot * hdr_->slot_bytes, bi.ptr, n);
      hdr_->len[slot] = n;
      hdr_->seq.store(s + 1, std::memory_order_release);
    }
    return true;
  }

  // Reader `r`: the next message (bytes), or None on timeout.
  py::object recv(int r, double timeout_s) {
    if (r < 0 || (uint64_t)r >= hdr_->nreaders) throw std::out_of_range("StepChannel: bad reader index");
    const uint64_t want = hdr_->ack[r].load(std::memory_order_relaxed) + 1;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = spin_until([&] { return hdr_->seq.load(std::memory_order_acquire) >= want; }, timeout_s);
    }
    if (!ok) return py::none();
    const uint64_t slot = (want - 1) % hdr_->nslots;
    const uint8_t* src = base_ + sizeof(ChanHeader) + slot * hdr_->slot_bytes;
    py::bytes out(reinterpret_cast<const char*>(src), (size_t)hdr_->len[slot]);
    hdr_->ack[r].store(want, std::memory_order_release);
    return out;
  }

  void unlink() {
    if (owner_) shm_unlink(name_.c_str());
    owner_ = false;
  }

  void close_() {
    if (base_ != nullptr) {
      munmap(base_, size_);
      base_ = nullptr;
      hdr_ = nullptr;
    }
    if (fd_ >= 0) {
      ::close(fd_);
      fd_ = -1;
    }
    unlink();
  }

 private:
  bool wait_acks(uint64_t need, double timeout_s) {
    return spin_until(
        [&] {
          for (uint64_t r = 0; r < hdr_->nreaders; ++r)
            if (hdr_->ack[r].load(std::memory_order_acquire) < need) return false;
          return true;
        },
        timeout_s);
  }

  // Busy-poll for up to kSpinS (decode steps arrive every few ms: a sleeping reader would pay the
  // scheduler's wake-up latency, ~60 us with the default 50 us timer slack, on every step), then
  // back off to 20 us sleeps (timer slack lowered to 1 us) so an idle worker does not hold a core;
  // bounded by timeout_s (< 0: forever).
  static constexpr double kSpinS = 0.05;
  template <class F>
  static bool spin_until(F ready, double timeout_s) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (long i = 0;; ++i) {
      if (ready()) return true;
      if ((i & 255) != 0) {
        cpu_relax();
        continue;
      }
      const double el = std::chrono::duration<double>(clk::now() - t0).count();
      if (timeout_s >= 0 && el > timeout_s) return false;
      if (el < kSpinS) continue;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }

  std::string name_;
  bool owner_;
  int fd_ = -1;
  size_t size_ = 0;
  uint8_t* base_ = nullptr;
  ChanHeader* hdr_ = nullptr;
};

}  // namespace

void register_step_channel(py::module_& m) {
  py::class_<StepChannel>(m, "StepChannel")
      .def(py::init<const std::string&, bool, int, int64_t, int>(), py::arg("name"), py::arg("create"),
           py::arg("nslots") = 4, py::arg("slot_bytes") = 1 << 20, py::arg("nreaders") = 1)
      .def("publish", &StepChannel::publish, py::arg("data"), py::arg("timeout_s") = -1.0)
      .def("recv", &StepChannel::recv, py::arg("reader"), py::arg("timeout_s") = -1.0)
      .def("unlink", &StepChannel::unlink)
      .def("close", &StepChannel::close_)
      .def_property_readonly("slot_bytes", &StepChannel::slot_bytes)
      .def("heartbeat", &StepChannel::heartbeat)
      .def_property_readonly("beats", &StepChannel::beats)
      .def_property_readonly("published", &StepChannel::published);
}
