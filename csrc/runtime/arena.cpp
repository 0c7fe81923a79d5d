// Device memory arena of a training step (the framework-owned allocator of
// SURVEY §7.1): one hipMalloc'd region per device, sized from the liveness
// memory plan (csrc/ffcore/src/memory_plan.cc) before the first step, served
// first-fit in 2 MiB granules, free ranges coalesced; a request that does not
// fit falls back to hipMalloc and is counted as overflow.  Tracked like the
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

namespace {

constexpr size_t kGranule = size_t(2) << 20;

struct DeviceArena {
  char* base = nullptr;
  size_t cap = 0;
  std::map<size_t, size_t> free_ranges;            // offset -> bytes
  std::unordered_map<void*, size_t> in_arena;      // ptr -> rounded bytes
  std::unordered_map<void*, size_t> overflow;      // hipMalloc fallbacks
  size_t live = 0, high = 0, top = 0;              // top: highest byte ever handed out
  uint64_t n_alloc = 0, n_overflow = 0;
  size_t overflow_bytes = 0, overflow_high = 0;
};

std::mutex g_mu;
std::unordered_map<int, DeviceArena> g_arenas;

size_t round_up(size_t n) { return (n + kGranule - 1) / kGranule * kGranule; }

}  // namespace

#define FF_ARENA_API extern "C" __attribute__((visibility("default")))

// reserve `bytes` on `device` (once; a second call with a larger size grows
// only if nothing is allocated yet).  Returns 0 on success.
FF_ARENA_API int ff_arena_reserve(int device, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  bytes = round_up(bytes);
  if (a.base && (bytes <= a.cap || !a.in_arena.empty())) return 0;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return 1;
  if (a.base) {
    (void)hipFree(a.base);
    a.base = nullptr;
  }
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, bytes);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    a.cap = 0;
    return 2;
  }
  a.base = static_cast<char*>(p);
  a.cap = bytes;
  a.free_ranges.clear();
  a.free_ranges[0] = bytes;
  return 0;
}

FF_ARENA_API void* ff_arena_alloc(size_t size, int device, hipStream_t /*stream*/) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& a = g_arenas[device];
  const size_t need = round_up(size == 0 ? 1 : size);
  ++a.n_alloc;
  for (auto it = a.free_ranges.begin(); it != a.free_ranges.end(); ++it) {
    if (it->second < need) continue;
    const size_t off = it->first, len = it->second;
    a.free_ranges.erase(it);
    if (len > need) a.free_ranges[off + need] = len - need;
    void* p = a.base + off;
    a.in_arena[p] = need;
    a.live += need;
    if (a.live > a.high) a.high = a.live;
    if (off + need > a.top) a.top = off + need;
    return p;
  }
  // no fit: the device allocator, counted
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, size);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
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
  size_t off = static_cast<size_t>(static_cast<char*>(ptr) - a.base), len = it->second;
  a.in_arena.erase(it);
  a.live -= len;
  // coalesce with the neighbours
  auto next = a.free_ranges.lower_bound(off);
  if (next != a.free_ranges.end() && next->first == off + len) {
    len += next->second;
    next = a.free_ranges.erase(next);
  }
  if (next != a.free_ranges.begin()) {
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      off = prev->first;
      len += prev->second;
      a.free_ranges.erase(prev);
    }
  }
  a.free_ranges[off] = len;
}

// [capacity, live, high water, top offset, allocations, overflow allocations,
//  overflow bytes live, overflow high water]
FF_ARENA_API void ff_arena_stats(int device, double* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  const DeviceArena& a = g_arenas[device];
  out[0] = static_cast<double>(a.cap);
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
