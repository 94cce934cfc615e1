// Shared-memory step-plan channel: TP leader -> followers of one replica on one node.
//
// SURVEY.md §2.7 lists the scheduler-decision broadcast (rank 0 -> TP ranks: token ids, positions, block tables,
// work items) as "CPU, gloo or shared memory". gloo pays a TCP loopback round per follower per broadcast: for
// Llama-3-70B at TP = 8 with captured decode graphs the plan carries full-width block tables, and the broadcast sits
// on the critical path of a ~4 ms step whenever plan-ahead cannot hide it. This channel is a single-producer ring
// in POSIX shared memory:
//   * header: geometry, `seq` (plans published, written only by the leader, release store) and one `ack` word per
//     follower (plans consumed, written only by that follower, release store), each on its own cache line;
//   * nslots slots of slot_bytes: [u64 hdr bytes][u64 payload bytes][hdr][payload];
//   * publish: wait until every follower has released slot seq % nslots (ack >= seq + 1 - nslots), memcpy, then
//     seq = seq + 1 (release). recv: wait for seq > ack (acquire) and hand out zero-copy views of the slot; the
//     follower acks once it has consumed the plan (uploaded it), so the leader may run up to nslots - 1 plans ahead;
//   * every wait watches its peer's PROCESS: the leader's pid sits in the header and each follower's pid next to
//     its ack word, and a waiter whose peer has exited raises at once ("peer process is gone"; the replica then
//     fails and is respawned). A follower waiting for the next plan waits as long as its leader
//     lives (timeout_s < 0: an idle replica is not a dead one — ADVICE r03); the leader's back-pressure wait for
//     acks inside a step stays bounded by timeout_s. Waits back off from pause-spinning to yielding to short
//     sleeps, so an idle follower does not burn a core;
//   * the leader unlinks the segment name once every follower has attached (``unlink``): the mappings stay valid,
//     and a group killed with SIGKILL leaves nothing behind in /dev/shm.
// Single producer / single consumer per ack word: the only atomics needed are acquire/release loads and stores.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace kafka {

constexpr uint64_t kChanMagic = 0x6b61666b61706c6eull;  // "kafkapln"
constexpr int kMaxFollowers = 63;

struct alignas(64) ChanWord {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct alignas(64) AckWord {
  std::atomic<uint64_t> v;
  std::atomic<int64_t> pid;  // the follower process (0 until it attaches)
  char pad[64 - 2 * sizeof(std::atomic<uint64_t>)];
};

struct ChanHeader {
  uint64_t magic;
  uint64_t nslots;
  uint64_t slot_bytes;
  uint64_t nfollow;
  int64_t leader_pid;
  char pad0[24];
  ChanWord seq;
  AckWord acks[kMaxFollowers];
};

static bool process_gone(int64_t pid) { return pid > 0 && kill((pid_t)pid, 0) != 0 && errno == ESRCH; }

static_assert(sizeof(ChanHeader) % 64 == 0, "header lines");

class PlanChannel {
 public:
  // leader: create (and own) the segment
  PlanChannel(const std::string& name, int nslots, int64_t slot_bytes, int nfollow)
      : name_(name), leader_(true), follower_(-1) {
    if (nslots < 2 || slot_bytes < 1024 || nfollow < 1 || nfollow > kMaxFollowers)
      throw std::invalid_argument("PlanChannel: nslots >= 2, slot_bytes >= 1024, 1 <= followers <= 63");
    bytes_ = sizeof(ChanHeader) + (size_t)nslots * (size_t)slot_bytes;
    const int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("PlanChannel: shm_open(create) failed for " + name);
    if (ftruncate(fd, (off_t)bytes_) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("PlanChannel: ftruncate failed");
    }
    map(fd);
    hdr_->nslots = (uint64_t)nslots;
    hdr_->slot_bytes = (uint64_t)slot_bytes;
    hdr_->nfollow = (uint64_t)nfollow;
    hdr_->leader_pid = (int64_t)getpid();
    hdr_->seq.v.store(0, std::memory_order_relaxed);
    for (int i = 0; i < kMaxFollowers; ++i) {
      hdr_->acks[i].v.store(0, std::memory_order_relaxed);
      hdr_->acks[i].pid.store(0, std::memory_order_relaxed);
    }
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kChanMagic;
  }

  // follower `idx` (0 .. nfollow-1): attach to the leader's segment
  PlanChannel(const std::string& name, int idx) : name_(name), leader_(false), follower_(idx) {
    const int fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("PlanChannel: shm_open(attach) failed for " + name);
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(ChanHeader)) {
      close(fd);
      throw std::runtime_error("PlanChannel: segment too small");
    }
    bytes_ = (size_t)st.st_size;
    map(fd);
    if (hdr_->magic != kChanMagic || idx < 0 || (uint64_t)idx >= hdr_->nfollow)
      throw std::runtime_error("PlanChannel: bad segment or follower index");
    hdr_->acks[idx].pid.store((int64_t)getpid(), std::memory_order_release);
  }

  // leader: drop the segment's name (every follower has attached; the mappings stay valid)
  void unlink() {
    if (leader_ && !unlinked_) {
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  ~PlanChannel() { close_(); }

  void close_() {
    if (base_ != nullptr) {
      munmap(base_, bytes_);
      base_ = nullptr;
      hdr_ = nullptr;
    }
    if (leader_ && !unlinked_) {
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  // leader: one plan = int64 header + uint8 payload
  void publish(py::array_t<int64_t, py::array::c_style> hdr, py::array_t<uint8_t, py::array::c_style> payload,
               double timeout_s) {
    if (!leader_ || hdr_ == nullptr) throw std::runtime_error("PlanChannel.publish: not an open leader channel");
    const uint64_t hb = (uint64_t)hdr.size() * 8, pb = (uint64_t)payload.size();
    if (16 + hb + pb > hdr_->slot_bytes) throw std::length_error("PlanChannel.publish: plan larger than a slot");
    const uint64_t s = hdr_->seq.v.load(std::memory_order_relaxed);
    const uint64_t need = s + 1 > hdr_->nslots ? s + 1 - hdr_->nslots : 0;  // acks that free slot s % nslots
    {
      py::gil_scoped_release nogil;
      for (uint64_t f = 0; f < hdr_->nfollow; ++f)
        wait_until([&] { return hdr_->acks[f].v.load(std::memory_order_acquire) >= need; }, timeout_s,
                   "a follower stopped consuming plans", &hdr_->acks[f].pid);
    }
    char* slot = slot_ptr(s);
    std::memcpy(slot, &hb, 8);
    std::memcpy(slot + 8, &pb, 8);
    std::memcpy(slot + 16, hdr.data(), hb);
    std::memcpy(slot + 16 + hb, payload.data(), pb);
    hdr_->seq.v.store(s + 1, std::memory_order_release);
  }

  // follower: wait for the next plan; zero-copy views (int64 header, uint8 payload) valid until ack()
  py::tuple recv(double timeout_s) {
    if (leader_ || hdr_ == nullptr) throw std::runtime_error("PlanChannel.recv: not an open follower channel");
    const uint64_t next = hdr_->acks[follower_].v.load(std::memory_order_relaxed);
    {
      py::gil_scoped_release nogil;
      wait_until([&] { return hdr_->seq.v.load(std::memory_order_acquire) > next; }, timeout_s,
                 "the leader stopped publishing plans", nullptr, hdr_->leader_pid);
    }
    char* slot = slot_ptr(next);
    uint64_t hb, pb;
    std::memcpy(&hb, slot, 8);
    std::memcpy(&pb, slot + 8, 8);
    py::object owner = py::cast(this, py::return_value_policy::reference);
    py::array h(py::dtype::of<int64_t>(), {(py::ssize_t)(hb / 8)}, {(py::ssize_t)8},
                reinterpret_cast<int64_t*>(slot + 16), owner);
    py::array p(py::dtype::of<uint8_t>(), {(py::ssize_t)pb}, {(py::ssize_t)1},
                reinterpret_cast<uint8_t*>(slot + 16 + hb), owner);
    return py::make_tuple(h, p);
  }

  // follower: the plan handed out by the last recv() has been consumed (its slot may be reused)
  void ack() {
    if (leader_ || hdr_ == nullptr) throw std::runtime_error("PlanChannel.ack: not an open follower channel");
    auto& a = hdr_->acks[follower_].v;
    a.store(a.load(std::memory_order_relaxed) + 1, std::memory_order_release);
  }

  uint64_t published() const { return hdr_->seq.v.load(std::memory_order_acquire); }
  int nslots() const { return (int)hdr_->nslots; }
  int64_t slot_bytes() const { return (int64_t)hdr_->slot_bytes; }

 private:
  void map(int fd) {
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("PlanChannel: mmap failed");
    base_ = static_cast<char*>(p);
    hdr_ = reinterpret_cast<ChanHeader*>(base_);
  }

  char* slot_ptr(uint64_t s) const {
    return base_ + sizeof(ChanHeader) + (size_t)(s % hdr_->nslots) * (size_t)hdr_->slot_bytes;
  }

  // timeout_s < 0: no time limit (only the peer's exit ends the wait); the peer is `peer_pid`, or the pid word
  // `peer_word` (a follower that has not attached yet reads 0 = unknown)
  template <class Pred>
  static void wait_until(Pred ready, double timeout_s, const char* what, const std::atomic<int64_t>* peer_word = nullptr,
                         int64_t peer_pid = 0) {
    if (ready()) return;
    const auto t0 = std::chrono::steady_clock::now();
    double next_check = 0.5;
    for (uint64_t it = 1;; ++it) {
      if (ready()) return;
      if (it < 4096) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        continue;
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (timeout_s >= 0 && el > timeout_s) throw std::runtime_error(std::string("PlanChannel timeout: ") + what);
      if (el > next_check) {  // twice a second: is the peer process still there?
        next_check = el + 0.5;
        const int64_t pid = peer_word != nullptr ? peer_word->load(std::memory_order_acquire) : peer_pid;
        if (process_gone(pid) && !ready())
          throw std::runtime_error(std::string("PlanChannel: peer process is gone: ") + what);
      }
      if (el < 1e-3) {
        sched_yield();
      } else {
        const timespec ts{0, el < 0.05 ? 20000 : 200000};  // 20 us while busy, 200 us when idle
        nanosleep(&ts, nullptr);
      }
    }
  }

  std::string name_;
  bool leader_;
  int follower_;
  bool unlinked_ = false;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  ChanHeader* hdr_ = nullptr;
};

void register_plan_channel(py::module& m) {
  py::class_<PlanChannel>(m, "PlanChannel")
      .def(py::init<const std::string&, int, int64_t, int>(), py::arg("name"), py::arg("nslots"),
           py::arg("slot_bytes"), py::arg("nfollow"))
      .def(py::init<const std::string&, int>(), py::arg("name"), py::arg("follower"))
      .def("publish", &PlanChannel::publish, py::arg("hdr"), py::arg("payload"), py::arg("timeout_s") = 300.0)
      .def("recv", &PlanChannel::recv, py::arg("timeout_s") = 300.0)
      .def("ack", &PlanChannel::ack)
      .def("close", &PlanChannel::close_)
      .def("unlink", &PlanChannel::unlink)
      .def_property_readonly("published", &PlanChannel::published)
      .def_property_readonly("nslots", &PlanChannel::nslots)
      .def_property_readonly("slot_bytes", &PlanChannel::slot_bytes);
}

}  // namespace kafka
