// Device memory arena of a training step (the framework-owned allocator of
// SURVEY §7.1): hipMalloc'd regions per device, sized from the liveness
// memory plan (csrc/ffcore/src/memory_plan.cc) before the first step, served
// first-fit in 2 MiB granules, free ranges coalesced; a request that does not
// fit falls back to hipMalloc and is counted as overflow.  Regions live as
// long as the process (a later, larger reservation adds one).  Tracked like the
// reference's allocator / tracked allocator (lib/local-execution/src/
// local_slots_backing.cc:20-49, tracked_allocator.cc:8-23): live bytes, high
// water mark, allocation and overflow counts.
//
// The executor hands it to PyTorch as the segment source of a MemPool
// (torch.cuda.memory.CUDAPluggableAllocator + torch.cuda.MemPool): the step's
// activations, gradients and workspaces -- eager or captured into hipGraphs
// (the graph pool IS this MemPool) -- come out of this region, with torch's
// block cache splitting segments on top.  Weights and optimizer state, which
// the plan also counts, are allocated at compile time outside it.
//
// ABI: the two entry points CUDAPluggableAllocator loads by name, plus plain C
// control / statistics calls (ctypes).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <iterator>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

constexpr size_t kGranule = size_t(2) << 20;

// one hipMalloc'd region; a device grows by adding regions when a larger
// reservation comes while the earlier ones still hold live blocks
struct Region {
  char* base = nullptr;
  size_t cap = 0;
  std::map<size_t, size_t> free_ranges;            // offset -> bytes
};

struct Block {
  int region;
  size_t bytes;                                    // rounded
};

struct DeviceArena {
  std::vector<Region> regions;
  std::unordered_map<void*, Block> in_arena;       // ptr -> region, rounded bytes
  std::unordered_map<void*, size_t> overflow;      // hipMalloc fallbacks
  size_t live = 0, high = 0, top = 0;              // top: sum over regions of the highest byte handed out
  std::vector<size_t> region_top;
  uint64_t n_alloc = 0, n_overflow = 0;
  size_t overflow_bytes = 0, overflow_high = 0;

  size_t capacity() const {
    size_t c = 0;
    for (const Region& r : regions) c += r.cap;
    return c;
  }
};

std::mutex g_mu;
std::unordered_map<int, DeviceArena> g_arenas;

size_t round_up(size_t n) { return (n + kGranule - 1) / kGranule * kGranule; }

// hipMalloc on `device` without disturbing the caller's current device
void* device_malloc(int device, size_t bytes) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, bytes);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

}  // namespace

#define FF_ARENA_API extern "C" __attribute__((visibility("default")))

// make at least `bytes` available on `device`.  With nothing live the
// existing regions are replaced by one region of that size; otherwise a region
// of the missing size is added next to them.  Returns 0 on success.
FF_ARENA_API int ff_arena_reserve(int device, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  bytes = round_up(bytes);
  const size_t have = a.capacity();
  if (have >= bytes) return 0;
  if (a.in_arena.empty()) {
    for (Region& r : a.regions) (void)hipFree(r.base);
    a.regions.clear();
    a.region_top.clear();
    a.top = 0;
  } else {
    bytes -= have;
  }
  void* p = device_malloc(device, bytes);
  if (!p) return 2;
  Region r;
  r.base = static_cast<char*>(p);
  r.cap = bytes;
  r.free_ranges[0] = bytes;
  a.regions.push_back(std::move(r));
  a.region_top.push_back(0);
  return 0;
}

FF_ARENA_API void* ff_arena_alloc(size_t size, int device, hipStream_t /*stream*/) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  const size_t need = round_up(size == 0 ? 1 : size);
  ++a.n_alloc;
  for (int ri = static_cast<int>(a.regions.size()) - 1; ri >= 0; --ri) {
    Region& r = a.regions[ri];
    for (auto it = r.free_ranges.begin(); it != r.free_ranges.end(); ++it) {
      if (it->second < need) continue;
      const size_t off = it->first, len = it->second;
      r.free_ranges.erase(it);
      if (len > need) r.free_ranges[off + need] = len - need;
      void* p = r.base + off;
      a.in_arena[p] = Block{ri, need};
      a.live += need;
      if (a.live > a.high) a.high = a.live;
      if (off + need > a.region_top[ri]) {
        a.top += off + need - a.region_top[ri];
        a.region_top[ri] = off + need;
      }
      return p;
    }
  }
  // no fit: the device allocator, counted.  (Answering "no room" instead,
  // to make torch's block cache release its free segments first, is not an
  // option: a MemPool with nothing to release raises out-of-memory.)
  void* p = device_malloc(device, size);
  if (!p) return nullptr;
  a.overflow[p] = size;
  ++a.n_overflow;
  a.overflow_bytes += size;
  if (a.overflow_bytes > a.overflow_high) a.overflow_high = a.overflow_bytes;
  return p;
}

FF_ARENA_API void ff_arena_free(void* ptr, size_t /*size*/, int device, hipStream_t /*stream*/) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  auto it = a.in_arena.find(ptr);
  if (it == a.in_arena.end()) {
    auto o = a.overflow.find(ptr);
    if (o != a.overflow.end()) {
      a.overflow_bytes -= o->second;
      a.overflow.erase(o);
      (void)hipFree(ptr);
    }
    return;
  }
  Region& r = a.regions[it->second.region];
  size_t off = static_cast<size_t>(static_cast<char*>(ptr) - r.base), len = it->second.bytes;
  a.in_arena.erase(it);
  a.live -= len;
  // coalesce with the neighbours
  auto next = r.free_ranges.lower_bound(off);
  if (next != r.free_ranges.end() && next->first == off + len) {
    len += next->second;
    next = r.free_ranges.erase(next);
  }
  if (next != r.free_ranges.begin()) {
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      off = prev->first;
      len += prev->second;
      r.free_ranges.erase(prev);
    }
  }
  r.free_ranges[off] = len;
}

// [capacity, live, high water, top offset, allocations, overflow allocations,
//  overflow bytes live, overflow high water]
FF_ARENA_API void ff_arena_stats(int device, double* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  const DeviceArena& a = g_arenas[device];
  out[0] = static_cast<double>(a.capacity());
  out[1] = static_cast<double>(a.live);
  out[2] = static_cast<double>(a.high);
  out[3] = static_cast<double>(a.top);
  out[4] = static_cast<double>(a.n_alloc);
  out[5] = static_cast<double>(a.n_overflow);
  out[6] = static_cast<double>(a.overflow_bytes);
  out[7] = static_cast<double>(a.overflow_high);
}

FF_ARENA_API void ff_arena_reset_high(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  a.high = a.live;
  a.overflow_high = a.overflow_bytes;
}

// start the counters over (a new user of the device's arena): allocation and
// overflow counts to zero, high-water marks to what is live now
FF_ARENA_API void ff_arena_reset_counts(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  a.n_alloc = 0;
  a.n_overflow = 0;
  a.high = a.live;
  a.overflow_high = a.overflow_bytes;
}
