// Auto-growth best-fit device allocator (FLAGS_allocator_strategy = "auto_growth").
//
// Parity: reference `paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc` (chunks
// grown on demand, best-fit over free blocks, split + coalesce, chunks released when wholly
// free) and `stream_safe_cuda_allocator.cc` (a freed block is reused only in the stream order it
// was freed in). Plugged into PyTorch-ROCm as its CUDA(HIP) allocator through
// CUDAPluggableAllocator (`paddle_infer_amd/device/allocator.py`), so every framework tensor —
// HIP kernels, hipBLASLt workspaces, RCCL buffers — comes from here.
//
// MI355X sizing: 288 GB HBM per GPU; chunks default to 1 GiB (FLAGS-style env
// PIAMD_ALLOC_CHUNK_MB) so a 13B-parameter training state (≈220 GB) grows in ~220 hipMalloc
// calls, not tens of thousands; 512-byte block alignment (hipMalloc returns ≥ 4 KiB-aligned
// chunks, every split keeps 512 B, enough for 16-byte vector and LDS-DMA sources).
//
// Per device: blocks of a chunk form an address-ordered doubly linked list (coalescing); free
// blocks sit in a best-fit multimap keyed by (pool, stream, size). Thread-safe (one mutex per
// device).
//
// Cross-stream use (reference StreamSafeCUDAAllocator::RecordStream): `piamd_record_stream`
// (PyTorch's Tensor.record_stream, forwarded through the pluggable allocator) adds a stream to
// the block's use set; when such a block is freed an event is recorded on every other stream that
// used it and the block waits on a pending list — it returns to the free list only once all those
// events have completed (polled on every allocation), so another stream's in-flight kernels can
// never see the memory handed to new work.
//
// hipGraph capture (PyTorch private memory pools): between `piamd_begin_pool` and
// `piamd_end_pool`, allocations on streams the capture's filter accepts come from the graph's own
// pool (tagged blocks, own chunks); its freed blocks are reused only inside that pool, so a
// captured graph's addresses stay valid across replays, until `piamd_release_pool` returns them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace {

constexpr size_t kAlign = 512;
constexpr int kMaxDev = 64;

using PoolId = std::pair<unsigned long long, unsigned long long>;  // PyTorch MempoolId_t

struct Block {
  char* ptr;
  size_t size;
  bool free;
  hipStream_t stream;
  Block* prev;  // address neighbours inside the same chunk
  Block* next;
  char* chunk;  // chunk base (hipMalloc'd)
  uint64_t pool = 0;                // 0 = general pool, else a graph pool key
  std::vector<hipStream_t> uses;    // other streams recorded via record_stream
};

using FreeKey = std::tuple<uint64_t, uintptr_t, size_t>;  // (pool, stream, size)

struct Capture {
  uint64_t key;
  std::function<bool(hipStream_t)> filter;
};

struct Pending {
  Block* b;
  std::vector<hipEvent_t> events;
};

struct Pool {
  std::mutex mu;
  std::multimap<FreeKey, Block*> free_blocks;
  std::unordered_map<void*, Block*> live;
  std::unordered_map<char*, size_t> chunks;  // base -> bytes
  std::vector<Capture> captures;             // active begin_allocate_to_pool windows
  std::unordered_map<uint64_t, PoolId> pool_ids;
  std::unordered_set<uint64_t> released;     // graph pools given back
  std::vector<Pending> pending;              // freed, waiting on other streams' events
  std::vector<hipEvent_t> event_cache;
  long long allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  long long n_alloc = 0, n_free = 0, n_chunk_alloc = 0, n_chunk_free = 0;
};

// hipMalloc / hipEventQuery / hipEventRecord issued while some stream of this thread is being
// captured would invalidate the capture in the default (global) mode: the allocator's own
// bookkeeping calls run in relaxed mode, as PyTorch's caching allocator does
struct RelaxedCapture {
  hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
  RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
  ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
};

uint64_t pool_key(PoolId id) { return (id.first * 0x9E3779B97F4A7C15ull) ^ (id.second + 1); }

Pool g_pools[kMaxDev];

size_t chunk_bytes() {
  static size_t v = [] {
    const char* e = getenv("PIAMD_ALLOC_CHUNK_MB");
    long long mb = e ? atoll(e) : 1024;
    return (size_t)(mb > 0 ? mb : 1024) << 20;
  }();
  return v;
}

size_t round_up(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

void erase_free(Pool& p, Block* b) {
  auto range = p.free_blocks.equal_range(FreeKey{b->pool, (uintptr_t)b->stream, b->size});
  for (auto it = range.first; it != range.second; ++it)
    if (it->second == b) {
      p.free_blocks.erase(it);
      return;
    }
}

void insert_free(Pool& p, Block* b) {
  p.free_blocks.insert({FreeKey{b->pool, (uintptr_t)b->stream, b->size}, b});
}

// coalesce b with free neighbours of the same pool and stream, then file it (lock held)
void give_back(Pool& p, Block* b) {
  b->free = true;
  b->uses.clear();
  if (b->pool && p.released.count(b->pool)) b->pool = 0;
  auto same = [&](Block* o) { return o && o->free && o->stream == b->stream && o->pool == b->pool &&
                                     std::none_of(p.pending.begin(), p.pending.end(),
                                                  [&](const Pending& q) { return q.b == o; }); };
  if (same(b->next)) {
    Block* n = b->next;
    erase_free(p, n);
    b->size += n->size;
    b->next = n->next;
    if (n->next) n->next->prev = b;
    delete n;
  }
  if (same(b->prev)) {
    Block* q = b->prev;
    erase_free(p, q);
    q->size += b->size;
    q->next = b->next;
    if (b->next) b->next->prev = q;
    delete b;
    b = q;
  }
  insert_free(p, b);
}

// move pending blocks whose cross-stream events have all completed to the free list
void poll_pending(Pool& p) {
  for (size_t i = 0; i < p.pending.size();) {
    Pending& q = p.pending[i];
    bool done = true;
    for (hipEvent_t e : q.events)
      if (hipEventQuery(e) != hipSuccess) { done = false; break; }
    if (!done) { ++i; continue; }
    (void)hipGetLastError();
    for (hipEvent_t e : q.events) p.event_cache.push_back(e);
    Block* b = q.b;
    p.pending[i] = p.pending.back();
    p.pending.pop_back();
    give_back(p, b);
  }
}

// release chunks that are one wholly free block (caller holds the lock)
void release_free_chunks(Pool& p, int device) {
  std::vector<Block*> victims;
  for (auto& kv : p.free_blocks) {
    Block* b = kv.second;
    // a graph pool's free block may still be addressed by the captured graph: keep its chunk
    if (!b->prev && !b->next && b->pool == 0) victims.push_back(b);
  }
  if (victims.empty()) return;
  int cur = 0;
  hipGetDevice(&cur);
  if (cur != device) hipSetDevice(device);
  for (Block* b : victims) {
    erase_free(p, b);
    p.reserved -= (long long)p.chunks[b->chunk];
    p.chunks.erase(b->chunk);
    hipFree(b->chunk);
    ++p.n_chunk_free;
    delete b;
  }
  if (cur != device) hipSetDevice(cur);
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) void* piamd_alloc(ssize_t size, int device, hipStream_t stream) {
  if (size <= 0 || device < 0 || device >= kMaxDev) return nullptr;
  Pool& p = g_pools[device];
  const size_t need = round_up((size_t)size);
  RelaxedCapture rc;
  std::lock_guard<std::mutex> lk(p.mu);
  if (!p.pending.empty()) poll_pending(p);
  uint64_t pool = 0;
  for (auto& c : p.captures)
    if (c.filter(stream)) { pool = c.key; break; }
  // best fit among this (pool, stream)'s free blocks
  auto it = p.free_blocks.lower_bound(FreeKey{pool, (uintptr_t)stream, need});
  Block* b = nullptr;
  if (it != p.free_blocks.end() && std::get<0>(it->first) == pool &&
      std::get<1>(it->first) == (uintptr_t)stream) {
    b = it->second;
    p.free_blocks.erase(it);
  } else {
    size_t cb = need > chunk_bytes() ? need : chunk_bytes();
    char* base = nullptr;
    int cur = 0;
    hipGetDevice(&cur);
    if (cur != device) hipSetDevice(device);
    hipError_t e = hipMalloc((void**)&base, cb);
    if (e != hipSuccess) {  // out of memory: give back wholly free chunks, retry exact size
      (void)hipGetLastError();
      release_free_chunks(p, device);
      cb = need;
      e = hipMalloc((void**)&base, cb);
    }
    if (cur != device) hipSetDevice(cur);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    p.chunks[base] = cb;
    p.reserved += (long long)cb;
    if (p.reserved > p.peak_reserved) p.peak_reserved = p.reserved;
    ++p.n_chunk_alloc;
    b = new Block{base, cb, true, stream, nullptr, nullptr, base, pool, {}};
  }
  if (b->size - need >= kAlign) {  // split: the tail stays free
    Block* t = new Block{b->ptr + need, b->size - need, true, stream, b, b->next, b->chunk, b->pool, {}};
    if (b->next) b->next->prev = t;
    b->next = t;
    b->size = need;
    insert_free(p, t);
  }
  b->free = false;
  b->stream = stream;
  p.live[b->ptr] = b;
  p.allocated += (long long)b->size;
  if (p.allocated > p.peak_allocated) p.peak_allocated = p.allocated;
  ++p.n_alloc;
  return b->ptr;
}

__attribute__((visibility("default"))) void piamd_free(void* ptr, ssize_t size, int device,
                                                       hipStream_t stream) {
  (void)size;
  (void)stream;
  if (!ptr || device < 0 || device >= kMaxDev) return;
  Pool& p = g_pools[device];
  RelaxedCapture rc;
  std::lock_guard<std::mutex> lk(p.mu);
  auto it = p.live.find(ptr);
  if (it == p.live.end()) return;
  Block* b = it->second;
  p.live.erase(it);
  p.allocated -= (long long)b->size;
  ++p.n_free;
  // used on other streams (record_stream): wait for their work before the block is reusable
  std::vector<hipEvent_t> evs;
  for (hipStream_t us : b->uses) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (us == b->stream || hipStreamIsCapturing(us, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
      continue;
    hipEvent_t e;
    if (!p.event_cache.empty()) { e = p.event_cache.back(); p.event_cache.pop_back(); }
    else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) continue;
    if (hipEventRecord(e, us) != hipSuccess) { p.event_cache.push_back(e); continue; }
    evs.push_back(e);
  }
  (void)hipGetLastError();
  if (!evs.empty()) {
    b->free = true;
    p.pending.push_back(Pending{b, std::move(evs)});
    return;
  }
  give_back(p, b);
}

// PyTorch Tensor.record_stream → the block is also used on `stream`
__attribute__((visibility("default"))) void piamd_record_stream(void* ptr, hipStream_t stream) {
  int device = 0;
  hipGetDevice(&device);
  for (int d : {device}) {
    if (d < 0 || d >= kMaxDev) return;
    Pool& p = g_pools[d];
    std::lock_guard<std::mutex> lk(p.mu);
    auto it = p.live.find(ptr);
    if (it == p.live.end()) {  // a view into a block: find the block containing ptr
      for (auto& kv : p.live) {
        Block* b = kv.second;
        if ((char*)ptr >= b->ptr && (char*)ptr < b->ptr + b->size) { it = p.live.find(kv.first); break; }
      }
      if (it == p.live.end()) return;
    }
    Block* b = it->second;
    if (stream != b->stream && std::find(b->uses.begin(), b->uses.end(), stream) == b->uses.end())
      b->uses.push_back(stream);
  }
}

// graph capture windows (PyTorch CUDAGraph private pools)
__attribute__((visibility("default"))) void piamd_begin_pool(int device, PoolId id,
                                                             std::function<bool(hipStream_t)> filter) {
  if (device < 0 || device >= kMaxDev) return;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  const uint64_t k = pool_key(id);
  p.pool_ids[k] = id;
  p.released.erase(k);
  p.captures.push_back(Capture{k, std::move(filter)});
}

__attribute__((visibility("default"))) void piamd_end_pool(int device, PoolId id) {
  if (device < 0 || device >= kMaxDev) return;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  const uint64_t k = pool_key(id);
  p.captures.erase(std::remove_if(p.captures.begin(), p.captures.end(),
                                  [&](const Capture& c) { return c.key == k; }),
                   p.captures.end());
}

__attribute__((visibility("default"))) void piamd_release_pool(int device, PoolId id) {
  if (device < 0 || device >= kMaxDev) return;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  const uint64_t k = pool_key(id);
  p.released.insert(k);
  std::vector<Block*> mine;
  for (auto& kv : p.free_blocks)
    if (kv.second->pool == k) mine.push_back(kv.second);
  for (Block* b : mine) {
    erase_free(p, b);
    give_back(p, b);  // retagged to the general pool, coalesced there
  }
}

// stats[0..7]: allocated, reserved, peak allocated, peak reserved, #alloc, #free, #chunk alloc,
// #chunk free
__attribute__((visibility("default"))) int piamd_alloc_stats(int device, long long* stats) {
  if (device < 0 || device >= kMaxDev || !stats) return 1;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  const long long v[8] = {p.allocated, p.reserved, p.peak_allocated, p.peak_reserved,
                          p.n_alloc, p.n_free, p.n_chunk_alloc, p.n_chunk_free};
  memcpy(stats, v, sizeof(v));
  return 0;
}

__attribute__((visibility("default"))) void piamd_alloc_reset_peak(int device) {
  if (device < 0 || device >= kMaxDev) return;
  Pool& p = g_pools[device];
  std::lock_guard<std::mutex> lk(p.mu);
  p.peak_allocated = p.allocated;
  p.peak_reserved = p.reserved;
}

// hipFree every chunk that is wholly free (paddle.device.cuda.empty_cache)
__attribute__((visibility("default"))) void piamd_alloc_release(int device) {
  if (device < 0 || device >= kMaxDev) return;
  Pool& p = g_pools[device];
  hipDeviceSynchronize();
  std::lock_guard<std::mutex> lk(p.mu);
  release_free_chunks(p, device);
}

}  // extern "C"
