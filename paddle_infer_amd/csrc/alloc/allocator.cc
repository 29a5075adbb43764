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
// blocks sit in a best-fit multimap keyed by (stream, size). Thread-safe (one mutex per device).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

constexpr size_t kAlign = 512;
constexpr int kMaxDev = 64;

struct Block {
  char* ptr;
  size_t size;
  bool free;
  hipStream_t stream;
  Block* prev;  // address neighbours inside the same chunk
  Block* next;
  char* chunk;  // chunk base (hipMalloc'd)
};

using FreeKey = std::pair<uintptr_t, size_t>;  // (stream, size)

struct Pool {
  std::mutex mu;
  std::multimap<FreeKey, Block*> free_blocks;
  std::unordered_map<void*, Block*> live;
  std::unordered_map<char*, size_t> chunks;  // base -> bytes
  long long allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  long long n_alloc = 0, n_free = 0, n_chunk_alloc = 0, n_chunk_free = 0;
};

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
  auto range = p.free_blocks.equal_range({(uintptr_t)b->stream, b->size});
  for (auto it = range.first; it != range.second; ++it)
    if (it->second == b) {
      p.free_blocks.erase(it);
      return;
    }
}

void insert_free(Pool& p, Block* b) { p.free_blocks.insert({{(uintptr_t)b->stream, b->size}, b}); }

// release chunks that are one wholly free block (caller holds the lock)
void release_free_chunks(Pool& p, int device) {
  std::vector<Block*> victims;
  for (auto& kv : p.free_blocks) {
    Block* b = kv.second;
    if (!b->prev && !b->next) victims.push_back(b);
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
  std::lock_guard<std::mutex> lk(p.mu);
  // best fit among this stream's free blocks
  auto it = p.free_blocks.lower_bound({(uintptr_t)stream, need});
  Block* b = nullptr;
  if (it != p.free_blocks.end() && it->first.first == (uintptr_t)stream) {
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
    b = new Block{base, cb, true, stream, nullptr, nullptr, base};
  }
  if (b->size - need >= kAlign) {  // split: the tail stays free
    Block* t = new Block{b->ptr + need, b->size - need, true, stream, b, b->next, b->chunk};
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
  std::lock_guard<std::mutex> lk(p.mu);
  auto it = p.live.find(ptr);
  if (it == p.live.end()) return;
  Block* b = it->second;
  p.live.erase(it);
  p.allocated -= (long long)b->size;
  ++p.n_free;
  b->free = true;
  // coalesce with free neighbours of the same stream (stream-ordered reuse stays valid)
  if (b->next && b->next->free && b->next->stream == b->stream) {
    Block* n = b->next;
    erase_free(p, n);
    b->size += n->size;
    b->next = n->next;
    if (n->next) n->next->prev = b;
    delete n;
  }
  if (b->prev && b->prev->free && b->prev->stream == b->stream) {
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
