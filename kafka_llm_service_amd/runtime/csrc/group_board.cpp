// Shared-memory agreement board of one process group on one node (the DP-attention EP group's per-step agreement).
//
// Data-parallel attention runs the EP group in lockstep: before every forward the ranks agree on (max tokens of the
// step = the all-to-all capacity, any rank busy, any stop flag) — one tiny all-reduce-MAX per step. Over gloo that
// is a TCP loopback round trip per step on the host's critical path ("move the per-step
// agreement off gloo"); here it is a few cache lines in POSIX shared memory:
//   * one 128-byte slot per rank: an epoch word (release store) + the rank's pid + two value buffers selected by the
//     epoch's parity. exchange(): write vals into buffer e & 1, publish epoch e, wait until every slot shows >= e,
//     read every rank's buffer e & 1, max-reduce. A rank can run one exchange ahead (it writes buffer (e + 1) & 1)
//     but never two: exchange e + 1 cannot complete before every rank has published e + 1, i.e. finished reading e.
//   * a `wake` counter: a rank that receives a request while the group is idle bumps it, so idle peers (sleeping
//     in `wait_wake` with a backoff instead of polling collectives) start the group step within about a millisecond.
//   * every wait watches the peers' pids: a dead peer raises at once; a live idle one is waited for as long as the
//     caller's timeout says (< 0: no limit).
#include <errno.h>
#include <fcntl.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace kafka {

constexpr uint64_t kBoardMagic = 0x6b61666b61627264ull;  // "kafkabrd"
constexpr int kBoardMaxRanks = 64;
constexpr int kBoardVals = 6;

struct alignas(128) BoardSlot {
  std::atomic<uint64_t> epoch;
  std::atomic<int64_t> pid;
  int64_t vals[2][kBoardVals];
  char pad[128 - 16 - 2 * kBoardVals * 8];
};

struct BoardHeader {
  uint64_t magic;
  uint64_t nranks;
  char pad0[48];
  alignas(64) std::atomic<uint64_t> wake;
  char pad1[56];
  BoardSlot slots[kBoardMaxRanks];
};

static bool board_pid_gone(int64_t pid) { return pid > 0 && kill((pid_t)pid, 0) != 0 && errno == ESRCH; }

class GroupBoard {
 public:
  // rank 0 creates (create = true), the others attach
  GroupBoard(const std::string& name, int nranks, int rank, bool create) : name_(name), rank_(rank), owner_(create) {
    if (nranks < 1 || nranks > kBoardMaxRanks || rank < 0 || rank >= nranks)
      throw std::invalid_argument("GroupBoard: 1 <= nranks <= 64, 0 <= rank < nranks");
    const size_t bytes = sizeof(BoardHeader);
    const int fd = create ? shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("GroupBoard: shm_open failed for " + name);
    if (create && ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("GroupBoard: ftruncate failed");
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < bytes) {
      close(fd);
      throw std::runtime_error("GroupBoard: segment too small");
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("GroupBoard: mmap failed");
    h_ = static_cast<BoardHeader*>(p);
    if (create) {
      h_->nranks = (uint64_t)nranks;
      h_->wake.store(0, std::memory_order_relaxed);
      for (int i = 0; i < kBoardMaxRanks; ++i) {
        h_->slots[i].epoch.store(0, std::memory_order_relaxed);
        h_->slots[i].pid.store(0, std::memory_order_relaxed);
      }
      std::atomic_thread_fence(std::memory_order_release);
      h_->magic = kBoardMagic;
    } else if (h_->magic != kBoardMagic || h_->nranks != (uint64_t)nranks) {
      munmap(h_, sizeof(BoardHeader));
      h_ = nullptr;
      throw std::runtime_error("GroupBoard: bad segment");
    }
    h_->slots[rank].pid.store((int64_t)getpid(), std::memory_order_release);
  }

  ~GroupBoard() { close_(); }

  void close_() {
    if (h_ != nullptr) {
      munmap(h_, sizeof(BoardHeader));
      h_ = nullptr;
    }
    unlink();
  }

  void unlink() {
    if (owner_ && !unlinked_) {
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  // all-reduce MAX of up to kBoardVals int64 values over the group
  py::array_t<int64_t> exchange(py::array_t<int64_t, py::array::c_style> vals, double timeout_s) {
    if (h_ == nullptr) throw std::runtime_error("GroupBoard.exchange: closed");
    const int k = (int)vals.size();
    if (k < 1 || k > kBoardVals) throw std::invalid_argument("GroupBoard.exchange: 1..6 values");
    const uint64_t e = ++epoch_;
    BoardSlot& mine = h_->slots[rank_];
    std::memcpy(mine.vals[e & 1], vals.data(), (size_t)k * 8);
    mine.epoch.store(e, std::memory_order_release);
    const int n = (int)h_->nranks;
    py::array_t<int64_t> out(k);
    int64_t* o = out.mutable_data();
    std::memcpy(o, vals.data(), (size_t)k * 8);
    {
      py::gil_scoped_release nogil;
      for (int r = 0; r < n; ++r) {
        if (r == rank_) continue;
        BoardSlot& s = h_->slots[r];
        wait([&] { return s.epoch.load(std::memory_order_acquire) >= e; }, timeout_s, &s.pid,
             "a peer stopped taking part in the group agreement");
        for (int j = 0; j < k; ++j) o[j] = std::max(o[j], s.vals[e & 1][j]);
      }
    }
    return out;
  }

  void wake() { live().wake.fetch_add(1, std::memory_order_acq_rel); }
  uint64_t wake_count() const { return live().wake.load(std::memory_order_acquire); }

  // sleep until the wake counter differs from `seen` or `timeout_s` passed; returns the counter
  uint64_t wait_wake(uint64_t seen, double timeout_s) {
    live();
    py::gil_scoped_release nogil;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const uint64_t w = h_->wake.load(std::memory_order_acquire);
      if (w != seen) return w;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el >= timeout_s) return w;
      const timespec ts{0, 100000};  // 0.1 ms
      nanosleep(&ts, nullptr);
    }
  }

  int rank() const { return rank_; }
  int nranks() const { return (int)live().nranks; }

 private:
  BoardHeader& live() const {
    if (h_ == nullptr) throw std::runtime_error("GroupBoard: closed");
    return *h_;
  }

  template <class Pred>
  static void wait(Pred ready, double timeout_s, const std::atomic<int64_t>* pid, const char* what) {
    if (ready()) return;
    const auto t0 = std::chrono::steady_clock::now();
    double next_check = 0.5;
    for (uint64_t it = 1;; ++it) {
      if (ready()) return;
      if (it < 2048) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        continue;
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (timeout_s >= 0 && el > timeout_s) throw std::runtime_error(std::string("GroupBoard timeout: ") + what);
      if (el > next_check) {
        next_check = el + 0.5;
        if (board_pid_gone(pid->load(std::memory_order_acquire)) && !ready())
          throw std::runtime_error(std::string("GroupBoard: peer process is gone: ") + what);
      }
      if (el < 2e-3) {
        sched_yield();
      } else {
        const timespec ts{0, 50000};
        nanosleep(&ts, nullptr);
      }
    }
  }

  std::string name_;
  int rank_;
  bool owner_;
  bool unlinked_ = false;
  uint64_t epoch_ = 0;
  BoardHeader* h_ = nullptr;
};

void register_group_board(py::module& m) {
  py::class_<GroupBoard>(m, "GroupBoard")
      .def(py::init<const std::string&, int, int, bool>(), py::arg("name"), py::arg("nranks"), py::arg("rank"),
           py::arg("create"))
      .def("exchange", &GroupBoard::exchange, py::arg("vals"), py::arg("timeout_s") = 300.0)
      .def("wake", &GroupBoard::wake)
      .def("wake_count", &GroupBoard::wake_count)
      .def("wait_wake", &GroupBoard::wait_wake, py::arg("seen"), py::arg("timeout_s"))
      .def("unlink", &GroupBoard::unlink)
      .def("close", &GroupBoard::close_)
      .def_property_readonly("rank", &GroupBoard::rank)
      .def_property_readonly("nranks", &GroupBoard::nranks);
}

}  // namespace kafka
