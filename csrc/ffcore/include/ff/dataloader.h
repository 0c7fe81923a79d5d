// Native batch prefetcher: background threads gather this rank's rows of the
// next training batches from host-resident datasets into pinned staging slots.
//
// Parity: python/flexflow_dataloader.cc + flexflow_dataloader.cu (574 + 85
// LoC: the whole dataset sits in zero-copy host memory and an index launch
// copies each GPU's batch slice per iteration) and SingleDataLoader
// (flexflow_cffi.py:2449).  MI355X design: one process per GPU, so a loader
// only ever touches its own rows; gathering (optionally shuffled) rows is host
// work done by a small thread pool `depth` batches ahead, into pinned buffers
// the Python side copies to HBM with non-blocking H2D copies on a side
// stream — the training step never waits on host memory traffic.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

namespace ff {

struct LoaderArray {
  const unsigned char* data = nullptr;  // [num_samples][row_bytes], contiguous
  int64_t row_bytes = 0;
  int64_t lo = 0, hi = 0;               // rows of each global batch this rank keeps
};

class BatchPrefetcher {
 public:
  BatchPrefetcher(std::vector<LoaderArray> arrays, int64_t num_samples, int64_t batch, bool shuffle, uint64_t seed,
                  int depth, int workers);
  ~BatchPrefetcher();
  // staging pointer of array `a` in slot `s` (hi-lo rows of row_bytes), set before start()
  void set_slot(int s, int a, unsigned char* ptr);
  void start(int64_t first_batch = 0);
  // blocks (without the GIL) until the next batch in order is staged; returns its slot
  int next(int64_t* batch_index);
  void release(int slot);
  void stop();
  int64_t iters_per_epoch() const { return iters_; }
  int depth() const { return depth_; }
  // sample index of row r of batch b (the permutation of b's epoch)
  int64_t sample_of(int64_t b, int64_t r);

 private:
  void worker();
  void fill(int slot, int64_t b);
  const std::vector<int64_t>& perm(int64_t epoch);

  std::vector<LoaderArray> arrays_;
  int64_t num_samples_, batch_, iters_;
  bool shuffle_;
  uint64_t seed_;
  int depth_, nworkers_;
  std::vector<std::vector<unsigned char*>> slots_;  // [slot][array]
  std::vector<int64_t> slot_batch_;                 // batch staged in the slot (-1 free)
  std::vector<int> slot_state_;                     // 0 free, 1 filling, 2 ready, 3 consumer
  int64_t next_claim_ = 0, next_consume_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false, started_ = false;
  std::vector<std::thread> threads_;
  std::mutex perm_mu_;
  int64_t perm_epoch_[2] = {-1, -1};
  std::vector<int64_t> perm_[2];
};

}  // namespace ff
