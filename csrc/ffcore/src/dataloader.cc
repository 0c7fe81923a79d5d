#include "ff/dataloader.h"

#include <algorithm>
#include <cstring>
#include <numeric>
#include <random>
#include <stdexcept>

namespace ff {

BatchPrefetcher::BatchPrefetcher(std::vector<LoaderArray> arrays, int64_t num_samples, int64_t batch, bool shuffle,
                                 uint64_t seed, int depth, int workers)
    : arrays_(std::move(arrays)),
      num_samples_(num_samples),
      batch_(batch),
      shuffle_(shuffle),
      seed_(seed),
      depth_(std::max(2, depth)),
      nworkers_(std::max(1, workers)) {
  if (batch_ <= 0 || num_samples_ < batch_) throw std::invalid_argument("loader: need num_samples >= batch > 0");
  for (auto const& a : arrays_)
    if (!a.data || a.row_bytes <= 0 || a.lo < 0 || a.hi > batch_ || a.lo >= a.hi)
      throw std::invalid_argument("loader: bad array description");
  iters_ = num_samples_ / batch_;  // drop_last, like the reference's per-epoch iteration count
  slots_.assign(depth_, std::vector<unsigned char*>(arrays_.size(), nullptr));
  slot_batch_.assign(depth_, -1);
  slot_state_.assign(depth_, 0);
}

BatchPrefetcher::~BatchPrefetcher() { stop(); }

void BatchPrefetcher::set_slot(int s, int a, unsigned char* ptr) {
  if (started_) throw std::logic_error("loader: set_slot after start");
  if (s < 0 || s >= depth_ || a < 0 || a >= static_cast<int>(arrays_.size()))
    throw std::out_of_range("loader: slot/array index");
  slots_[s][a] = ptr;
}

const std::vector<int64_t>& BatchPrefetcher::perm(int64_t epoch) {
  std::lock_guard<std::mutex> g(perm_mu_);
  const int k = static_cast<int>(epoch & 1);
  if (perm_epoch_[k] != epoch) {
    perm_[k].resize(num_samples_);
    std::iota(perm_[k].begin(), perm_[k].end(), 0);
    if (shuffle_) {
      std::mt19937_64 rng(seed_ * 0x9E3779B97F4A7C15ull + static_cast<uint64_t>(epoch));
      std::shuffle(perm_[k].begin(), perm_[k].end(), rng);
    }
    perm_epoch_[k] = epoch;
  }
  return perm_[k];
}

int64_t BatchPrefetcher::sample_of(int64_t b, int64_t r) {
  const int64_t epoch = b / iters_, i = b % iters_;
  return perm(epoch)[i * batch_ + r];
}

void BatchPrefetcher::fill(int slot, int64_t b) {
  const int64_t epoch = b / iters_, i = b % iters_;
  const std::vector<int64_t>& p = perm(epoch);  // epochs e and e+1 stay cached (depth << iters)
  for (size_t a = 0; a < arrays_.size(); ++a) {
    const LoaderArray& A = arrays_[a];
    unsigned char* dst = slots_[slot][a];
    if (!shuffle_) {  // contiguous rows: one copy
      std::memcpy(dst, A.data + (i * batch_ + A.lo) * A.row_bytes, (A.hi - A.lo) * A.row_bytes);
      continue;
    }
    for (int64_t r = A.lo; r < A.hi; ++r)
      std::memcpy(dst + (r - A.lo) * A.row_bytes, A.data + p[i * batch_ + r] * A.row_bytes, A.row_bytes);
  }
}

void BatchPrefetcher::worker() {
  for (;;) {
    int64_t b;
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      // claim the next batch once its slot is free (slots are used round robin)
      cv_.wait(lk, [&] { return stop_ || slot_state_[next_claim_ % depth_] == 0; });
      if (stop_) return;
      b = next_claim_++;
      slot = static_cast<int>(b % depth_);
      slot_state_[slot] = 1;
      slot_batch_[slot] = b;
    }
    fill(slot, b);
    {
      std::lock_guard<std::mutex> lk(mu_);
      slot_state_[slot] = 2;
    }
    cv_.notify_all();
  }
}

void BatchPrefetcher::start(int64_t first_batch) {
  for (int s = 0; s < depth_; ++s)
    for (size_t a = 0; a < arrays_.size(); ++a)
      if (!slots_[s][a]) throw std::logic_error("loader: staging slot not set");
  stop();
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = false;
    next_claim_ = next_consume_ = first_batch;
    std::fill(slot_state_.begin(), slot_state_.end(), 0);
    std::fill(slot_batch_.begin(), slot_batch_.end(), -1);
    started_ = true;
  }
  for (int w = 0; w < nworkers_; ++w) threads_.emplace_back(&BatchPrefetcher::worker, this);
}

int BatchPrefetcher::next(int64_t* batch_index) {
  std::unique_lock<std::mutex> lk(mu_);
  if (!started_) throw std::logic_error("loader: next() before start()");
  const int slot = static_cast<int>(next_consume_ % depth_);
  cv_.wait(lk, [&] { return stop_ || (slot_state_[slot] == 2 && slot_batch_[slot] == next_consume_); });
  if (stop_) throw std::runtime_error("loader stopped");
  slot_state_[slot] = 3;
  if (batch_index) *batch_index = next_consume_;
  ++next_consume_;
  return slot;
}

void BatchPrefetcher::release(int slot) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (slot < 0 || slot >= depth_ || slot_state_[slot] != 3) throw std::logic_error("loader: release of a slot not held");
    slot_state_[slot] = 0;
    slot_batch_[slot] = -1;
  }
  cv_.notify_all();
}

void BatchPrefetcher::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
  threads_.clear();
  std::lock_guard<std::mutex> lk(mu_);
  started_ = false;
}

}  // namespace ff
