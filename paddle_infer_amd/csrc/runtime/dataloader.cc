// Native token-stream data loader for LLM pre-training (C ABI, loaded with ctypes).
//
// Parity: the reference's native data feed (`paddle/fluid/framework/data_feed.cc`,
// `data_set.cc`: C++ reader threads filling channels consumed by the trainer) and the GPT
// pre-training dataset of its benchmarks (fixed-length windows over a flat token file,
// shuffled per epoch, sharded over data-parallel ranks).
//
// Design: the token file (uint16 or int32 ids, flat) is mmap'ed read-only; `nthreads` workers
// fill a ring of `nbuf` batch slots of int64 [batch][seq_len + 1] (input + shifted label window)
// ahead of the consumer. Sample order: a per-epoch Fisher-Yates permutation of the non-overlapping
// windows (deterministic from seed + epoch), strided over ranks, so every rank reads disjoint
// samples and the stream is reproducible across restarts (`piamd_tokloader_seek`). The consumer
// copies a ready slot into caller memory (a pinned host buffer → async H2D on a side HIP stream).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#define PIAMD_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Slot {
  std::vector<int64_t> data;
  long long batch_idx = -1;  // which global batch this slot holds
  bool ready = false;
};

struct Loader {
  const uint8_t* base = nullptr;
  size_t bytes = 0;
  int fd = -1;
  int tok_bytes = 2;
  long long n_tokens = 0, n_samples = 0, per_rank = 0;
  int seq = 0, batch = 0, rank = 0, world = 1;
  uint64_t seed = 0;
  std::vector<Slot> slots;
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv_ready, cv_free;
  std::atomic<bool> stop{false};
  long long next_fill = 0;     // next global batch index to assign to a worker
  long long next_consume = 0;  // next global batch index the consumer wants
  // per-epoch permutation cache (epoch -> order)
  long long perm_epoch = -1;
  std::vector<long long> perm;
  std::mutex perm_mu;

  long long batches_per_epoch() const { return per_rank / batch; }

  long long sample_of(long long b, int i) {
    // global batch b of this rank, row i -> window index
    const long long bpe = batches_per_epoch();
    const long long epoch = b / bpe, within = b % bpe;
    const long long k = (within * batch + i) * world + rank;  // rank-strided position
    std::lock_guard<std::mutex> g(perm_mu);
    if (epoch != perm_epoch) {
      perm.resize(n_samples);
      for (long long j = 0; j < n_samples; ++j) perm[j] = j;
      std::mt19937_64 rng(seed * 1000003ull + (uint64_t)epoch);
      for (long long j = n_samples - 1; j > 0; --j) {
        std::uniform_int_distribution<long long> d(0, j);
        std::swap(perm[j], perm[d(rng)]);
      }
      perm_epoch = epoch;
    }
    return perm[k];
  }

  void fill(Slot& s, long long b) {
    s.data.resize((size_t)batch * (seq + 1));
    for (int i = 0; i < batch; ++i) {
      const long long w = sample_of(b, i);
      const long long t0 = w * (long long)seq;
      int64_t* dst = s.data.data() + (size_t)i * (seq + 1);
      for (int t = 0; t <= seq; ++t) {
        const long long idx = std::min(t0 + t, n_tokens - 1);
        if (tok_bytes == 2) {
          uint16_t v;
          std::memcpy(&v, base + idx * 2, 2);
          dst[t] = v;
        } else {
          int32_t v;
          std::memcpy(&v, base + idx * 4, 4);
          dst[t] = v;
        }
      }
    }
  }

  void worker() {
    for (;;) {
      long long b;
      size_t si;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_free.wait(lk, [&] {
          return stop.load() || next_fill < next_consume + (long long)slots.size();
        });
        if (stop.load()) return;
        b = next_fill++;
        si = (size_t)(b % (long long)slots.size());
        slots[si].ready = false;
        slots[si].batch_idx = b;
      }
      Slot tmp;
      fill(tmp, b);
      {
        std::lock_guard<std::mutex> lk(mu);
        if (slots[si].batch_idx == b) {
          slots[si].data.swap(tmp.data);
          slots[si].ready = true;
        }
      }
      cv_ready.notify_all();
    }
  }
};

}  // namespace

// Returns an opaque handle (null on error). tok_bytes: 2 (uint16) or 4 (int32).
PIAMD_EXPORT void* piamd_tokloader_create(const char* path, int tok_bytes, int seq_len, int batch,
                                         unsigned long long seed, int rank, int world, int nbuf,
                                         int nthreads) {
  if ((tok_bytes != 2 && tok_bytes != 4) || seq_len <= 0 || batch <= 0 || world <= 0 ||
      rank < 0 || rank >= world)
    return nullptr;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < (off_t)tok_bytes * (seq_len + 1)) {
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    return nullptr;
  }
  madvise(p, (size_t)st.st_size, MADV_RANDOM);
  auto* L = new Loader();
  L->base = (const uint8_t*)p;
  L->bytes = (size_t)st.st_size;
  L->fd = fd;
  L->tok_bytes = tok_bytes;
  L->n_tokens = (long long)st.st_size / tok_bytes;
  L->seq = seq_len;
  L->batch = batch;
  L->seed = seed;
  L->rank = rank;
  L->world = world;
  L->n_samples = (L->n_tokens - 1) / seq_len;
  L->per_rank = L->n_samples / world;
  if (L->per_rank < batch) {
    munmap(p, L->bytes);
    close(fd);
    delete L;
    return nullptr;
  }
  L->slots.resize((size_t)std::max(2, nbuf));
  for (int i = 0; i < std::max(1, nthreads); ++i) L->workers.emplace_back([L] { L->worker(); });
  return L;
}

// Copies the next batch ([batch][seq_len+1] int64) into `out`; returns its global batch index.
PIAMD_EXPORT long long piamd_tokloader_next(void* h, int64_t* out) {
  auto* L = (Loader*)h;
  long long b;
  size_t si;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    b = L->next_consume;
    si = (size_t)(b % (long long)L->slots.size());
    L->cv_ready.wait(lk, [&] { return L->slots[si].ready && L->slots[si].batch_idx == b; });
    std::memcpy(out, L->slots[si].data.data(), L->slots[si].data.size() * sizeof(int64_t));
    L->slots[si].ready = false;
    L->next_consume = b + 1;
  }
  L->cv_free.notify_all();
  return b;
}

// Restart the stream at global batch index `b` (resume from a checkpoint).
PIAMD_EXPORT void piamd_tokloader_seek(void* h, long long b) {
  auto* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->next_consume = b;
    L->next_fill = b;
    for (auto& s : L->slots) {
      s.ready = false;
      s.batch_idx = -1;
    }
  }
  L->cv_free.notify_all();
}

PIAMD_EXPORT long long piamd_tokloader_batches_per_epoch(void* h) {
  return ((Loader*)h)->batches_per_epoch();
}

PIAMD_EXPORT void piamd_tokloader_destroy(void* h) {
  auto* L = (Loader*)h;
  L->stop.store(true);
  L->cv_free.notify_all();
  L->cv_ready.notify_all();
  for (auto& t : L->workers) t.join();
  munmap((void*)L->base, L->bytes);
  close(L->fd);
  delete L;
}
