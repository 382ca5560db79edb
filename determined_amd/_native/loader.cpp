// Native prefetching record loader (replaces torch DataLoader worker processes for
// fixed-size image records, reference counterpart: ``harness/determined/pytorch/_data.py`` +
// torch's multi-process DataLoader).
//
// File format (written by determined_amd.pytorch.native_loader.write_record_file):
//   header  : "DAMDREC1" | int64 num_records | int32 H | int32 W | int32 C | int32 pad
//   records : int32 label | uint8 pixels[H*W*C] (HWC)          (record_bytes = 4 + H*W*C)
//
// The file is mmap'ed read-only.  Worker threads (std::thread, no GIL, no fork) turn whole
// batches into ready-to-copy host buffers owned by Python (pinned torch tensors): random crop
// + horizontal flip + per-channel (x/255 - mean)/std, written NHWC as bf16 or fp32, plus int64
// labels.  Batches are produced into a ring of `slots` buffers in order; the consumer's
// next() blocks (GIL released) until the next batch is ready and release() hands the slot
// back once its host->device copy has finished.
//
// Determinism: the epoch permutation (Fisher-Yates) and each sample's crop/flip come from
// splitmix64 streams keyed by (seed, epoch, index), so the output is independent of the
// worker count and reproducible from Python (see sample_params / permutation).  Sharding is
// DistributedSampler-style: rank r takes positions r, r+world, ... of the permutation.

#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace damd_native {

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static inline uint16_t f2bf(float f) {  // round-to-nearest-even
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t lsb = (u >> 16) & 1u;
  u += 0x7FFFu + lsb;
  return static_cast<uint16_t>(u >> 16);
}

std::vector<int64_t> permutation(int64_t n, uint64_t seed, int64_t epoch, bool shuffle) {
  std::vector<int64_t> p(n);
  for (int64_t i = 0; i < n; ++i) p[i] = i;
  if (!shuffle) return p;
  uint64_t s = splitmix64(seed ^ (0xA5A5A5A5ull + static_cast<uint64_t>(epoch) * 0x100000001B3ull));
  for (int64_t i = n - 1; i > 0; --i) {
    s = splitmix64(s);
    const int64_t j = static_cast<int64_t>(s % static_cast<uint64_t>(i + 1));
    std::swap(p[i], p[j]);
  }
  return p;
}

struct SampleParams {
  int y0, x0;
  bool flip;
};

SampleParams sample_params(uint64_t seed, int64_t epoch, int64_t index, int H, int W, int ch, int cw, bool augment) {
  if (!augment) return {(H - ch) / 2, (W - cw) / 2, false};
  const uint64_t a = splitmix64(seed * 0x9E3779B97F4A7C15ull ^ splitmix64(static_cast<uint64_t>(epoch) << 32 ^
                                                                          static_cast<uint64_t>(index)));
  const uint64_t b = splitmix64(a);
  const uint64_t c = splitmix64(b);
  return {static_cast<int>(a % static_cast<uint64_t>(H - ch + 1)), static_cast<int>(b % static_cast<uint64_t>(W - cw + 1)),
          (c & 1ull) != 0};
}

class RecordLoader {
 public:
  RecordLoader(const std::string& path, int batch, int crop_h, int crop_w, std::vector<float> mean,
               std::vector<float> stdv, bool bf16, bool shuffle, bool augment, bool drop_last, uint64_t seed,
               int rank, int world, int workers)
      : batch_(batch), ch_(crop_h), cw_(crop_w), mean_(std::move(mean)), std_(std::move(stdv)), bf16_(bf16),
        shuffle_(shuffle), augment_(augment), drop_last_(drop_last), seed_(seed), rank_(rank), world_(world),
        workers_(std::max(1, workers)) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open record file " + path);
    struct stat st;
    fstat(fd_, &st);
    size_ = static_cast<size_t>(st.st_size);
    if (size_ < 32) throw std::runtime_error("record file too small");
    base_ = static_cast<const uint8_t*>(mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0));
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    madvise(const_cast<uint8_t*>(base_), size_, MADV_WILLNEED);
    if (std::memcmp(base_, "DAMDREC1", 8) != 0) throw std::runtime_error("not a DAMDREC1 record file");
    std::memcpy(&n_, base_ + 8, 8);
    std::memcpy(&H_, base_ + 16, 4);
    std::memcpy(&W_, base_ + 20, 4);
    std::memcpy(&C_, base_ + 24, 4);
    rec_ = 4 + static_cast<size_t>(H_) * W_ * C_;
    if (32 + n_ * rec_ > size_) throw std::runtime_error("record file truncated");
    if (ch_ > H_ || cw_ > W_) throw std::invalid_argument("crop larger than the stored image");
    if (static_cast<int>(mean_.size()) != C_ || static_cast<int>(std_.size()) != C_)
      throw std::invalid_argument("mean/std need one value per channel");
    if (world_ < 1 || rank_ < 0 || rank_ >= world_) throw std::invalid_argument("bad rank/world");
  }

  ~RecordLoader() {
    stop();
    if (base_ && base_ != MAP_FAILED) munmap(const_cast<uint8_t*>(base_), size_);
    if (fd_ >= 0) ::close(fd_);
  }

  int64_t num_records() const { return n_; }
  py::tuple image_shape() const { return py::make_tuple(H_, W_, C_); }
  int64_t samples_per_rank() const {
    return drop_last_ ? n_ / world_ : (n_ + world_ - 1 - rank_) / world_;
  }
  int64_t batches_per_epoch() const {
    const int64_t s = samples_per_rank();
    return drop_last_ ? s / batch_ : (s + batch_ - 1) / batch_;
  }

  // Host buffers (pinned torch tensors) for `slots` batches: data [B, ch, cw, C], labels int64 [B].
  void set_slots(const std::vector<uintptr_t>& data, const std::vector<uintptr_t>& labels) {
    std::lock_guard<std::mutex> g(mu_);
    if (running_) throw std::runtime_error("set_slots while an epoch is running");
    if (data.size() != labels.size() || data.empty()) throw std::invalid_argument("need >= 1 slot");
    data_ = data;
    labels_ = labels;
  }

  void start_epoch(int64_t epoch) {
    stop();
    std::lock_guard<std::mutex> g(mu_);
    if (data_.empty()) throw std::runtime_error("set_slots first");
    epoch_ = epoch;
    auto perm = permutation(n_, seed_, epoch, shuffle_);
    mine_.clear();
    const int64_t per = samples_per_rank();
    for (int64_t k = 0; k < per; ++k) mine_.push_back(perm[(rank_ + k * world_) % n_]);
    nb_ = batches_per_epoch();
    next_produce_ = 0;
    next_consume_ = 0;
    slot_batch_.assign(data_.size(), -1);
    slot_ready_.assign(data_.size(), 0);
    slot_free_.assign(data_.size(), 1);
    error_.clear();
    running_ = true;
    for (int w = 0; w < workers_; ++w) threads_.emplace_back([this] { worker(); });
  }

  // Blocks until the next batch is ready: (slot, batch size), or (-1, 0) at the end of the epoch.
  py::tuple next() {
    std::unique_lock<std::mutex> lk(mu_);
    if (next_consume_ >= nb_) return py::make_tuple(-1, 0);
    const int64_t b = next_consume_;
    const int slot = static_cast<int>(b % static_cast<int64_t>(data_.size()));
    {
      py::gil_scoped_release nogil;
      cv_.wait(lk, [&] { return (slot_ready_[slot] && slot_batch_[slot] == b) || !error_.empty(); });
    }
    if (!error_.empty()) throw std::runtime_error("loader worker failed: " + error_);
    ++next_consume_;
    return py::make_tuple(slot, batch_size_of(b));
  }

  void release(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    if (slot < 0 || slot >= static_cast<int>(data_.size())) throw std::out_of_range("bad slot");
    slot_ready_[slot] = 0;
    slot_free_[slot] = 1;
    cv_.notify_all();
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      running_ = false;
      cv_.notify_all();
    }
    for (auto& t : threads_) t.join();
    threads_.clear();
  }

 private:
  int batch_size_of(int64_t b) const {
    const int64_t left = static_cast<int64_t>(mine_.size()) - b * batch_;
    return static_cast<int>(std::min<int64_t>(batch_, left));
  }

  void worker() {
    for (;;) {
      int64_t b;
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // claim the next batch whose ring slot is free (batches are claimed in order, so
        // slot b % S is only ever reused after batch b - S was released by the consumer)
        cv_.wait(lk, [&] {
          if (!running_ || next_produce_ >= nb_) return true;
          return static_cast<bool>(slot_free_[next_produce_ % static_cast<int64_t>(data_.size())]);
        });
        if (!running_ || next_produce_ >= nb_) return;
        b = next_produce_++;
        slot = static_cast<int>(b % static_cast<int64_t>(data_.size()));
        slot_free_[slot] = 0;
        slot_batch_[slot] = b;
      }
      try {
        fill(b, slot);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu_);
        error_ = e.what();
        cv_.notify_all();
        return;
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        slot_ready_[slot] = 1;
        cv_.notify_all();
      }
    }
  }

  void fill(int64_t b, int slot) {
    const int bs = batch_size_of(b);
    int64_t* lab = reinterpret_cast<int64_t*>(labels_[slot]);
    const size_t out_px = static_cast<size_t>(ch_) * cw_ * C_;
    float inv_std[16], mean255[16];
    for (int c = 0; c < C_ && c < 16; ++c) {
      inv_std[c] = 1.f / (255.f * std_[c]);
      mean255[c] = 255.f * mean_[c];
    }
    for (int i = 0; i < bs; ++i) {
      const int64_t idx = mine_[b * batch_ + i];
      const uint8_t* rec = base_ + 32 + static_cast<size_t>(idx) * rec_;
      int32_t label;
      std::memcpy(&label, rec, 4);
      lab[i] = label;
      const uint8_t* px = rec + 4;
      const SampleParams sp = sample_params(seed_, epoch_, idx, H_, W_, ch_, cw_, augment_);
      for (int y = 0; y < ch_; ++y) {
        const uint8_t* row = px + (static_cast<size_t>(sp.y0 + y) * W_) * C_;
        const size_t obase = (static_cast<size_t>(i) * ch_ + y) * cw_ * C_;
        for (int x = 0; x < cw_; ++x) {
          const int sx = sp.flip ? (sp.x0 + cw_ - 1 - x) : (sp.x0 + x);
          const uint8_t* p = row + static_cast<size_t>(sx) * C_;
          for (int c = 0; c < C_; ++c) {
            const float v = (static_cast<float>(p[c]) - mean255[c]) * inv_std[c];
            const size_t o = obase + static_cast<size_t>(x) * C_ + c;
            if (bf16_)
              reinterpret_cast<uint16_t*>(data_[slot])[o] = f2bf(v);
            else
              reinterpret_cast<float*>(data_[slot])[o] = v;
          }
        }
      }
      (void)out_px;
    }
  }

  // configuration
  int batch_, ch_, cw_;
  std::vector<float> mean_, std_;
  bool bf16_, shuffle_, augment_, drop_last_;
  uint64_t seed_;
  int rank_, world_, workers_;
  // file
  int fd_ = -1;
  size_t size_ = 0;
  const uint8_t* base_ = nullptr;
  int64_t n_ = 0;
  int32_t H_ = 0, W_ = 0, C_ = 0;
  size_t rec_ = 0;
  // epoch state
  std::vector<uintptr_t> data_, labels_;
  std::vector<int64_t> mine_;
  int64_t epoch_ = 0, nb_ = 0, next_produce_ = 0, next_consume_ = 0;
  std::vector<int64_t> slot_batch_;
  std::vector<char> slot_ready_, slot_free_;
  std::string error_;
  bool running_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::thread> threads_;
};

void register_loader(py::module& m) {
  py::class_<RecordLoader>(m, "RecordLoader")
      .def(py::init<const std::string&, int, int, int, std::vector<float>, std::vector<float>, bool, bool, bool, bool,
                    uint64_t, int, int, int>(),
           py::arg("path"), py::arg("batch"), py::arg("crop_h"), py::arg("crop_w"), py::arg("mean"), py::arg("std"),
           py::arg("bf16"), py::arg("shuffle"), py::arg("augment"), py::arg("drop_last"), py::arg("seed"),
           py::arg("rank"), py::arg("world"), py::arg("workers"))
      .def("num_records", &RecordLoader::num_records)
      .def("image_shape", &RecordLoader::image_shape)
      .def("samples_per_rank", &RecordLoader::samples_per_rank)
      .def("batches_per_epoch", &RecordLoader::batches_per_epoch)
      .def("set_slots", &RecordLoader::set_slots)
      .def("start_epoch", &RecordLoader::start_epoch, py::call_guard<py::gil_scoped_release>())
      .def("next", &RecordLoader::next)
      .def("release", &RecordLoader::release, py::call_guard<py::gil_scoped_release>())
      .def("stop", &RecordLoader::stop, py::call_guard<py::gil_scoped_release>());
  m.def("loader_permutation", &permutation, py::arg("n"), py::arg("seed"), py::arg("epoch"), py::arg("shuffle"));
  m.def(
      "loader_sample_params",
      [](uint64_t seed, int64_t epoch, int64_t index, int H, int W, int ch, int cw, bool augment) {
        const SampleParams p = sample_params(seed, epoch, index, H, W, ch, cw, augment);
        return py::make_tuple(p.y0, p.x0, p.flip);
      },
      py::arg("seed"), py::arg("epoch"), py::arg("index"), py::arg("H"), py::arg("W"), py::arg("crop_h"),
      py::arg("crop_w"), py::arg("augment"));
}

}  // namespace damd_native
