// Native device runtime: device properties, stream pool, events and the host/device range tracer
// behind paddle.device.cuda.{Stream, Event, get_device_properties} and paddle.profiler.
//
// Reference parity: `paddle/phi/backends/gpu/gpu_context.cc` / `gpu_info.cc` (device properties,
// stream creation with priorities), `paddle/phi/core/platform/device_event*` (events),
// `paddle/fluid/platform/profiler/host_tracer.cc` + `chrometracing_logger.cc` (RecordEvent ranges,
// chrome trace export). MI355X design: HIP streams / events straight from the runtime (the same
// runtime instance PyTorch uses: this library is loaded after torch, so a stream made here is a
// plain hipStream_t that torch.cuda.ExternalStream can adopt and that every framework kernel
// launch accepts); the tracer is a per-thread append-only range log (no lock on the hot path)
// with optional device timing through HIP event pairs recorded on the current stream, resolved
// only at export.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define PIAMD_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// ---------------------------------------------------------------------------------- properties
struct DevProps {
  char name[256];
  char arch[64];           // gcnArchName, e.g. "gfx950:sramecc+:xnack-"
  int major, minor;
  int cus;                 // compute units
  int clock_khz;
  int mem_clock_khz;
  int bus_width;
  long long total_mem;
  long long l2_bytes;
  long long lds_per_block;
  int warp;                // wavefront size
  int max_threads_per_block;
  int regs_per_block;
  int pci_bus, pci_dev, pci_domain;
  int cooperative;
  int concurrent_kernels;
};

// ---------------------------------------------------------------------------------- tracer
struct Range {
  int name;      // interned id
  int depth;
  long long t0, t1;  // host ns (steady clock, relative to the tracer epoch)
  int ev;        // index into the device-event pairs (-1: host only)
};

struct ThreadLog {
  int tid;
  std::vector<Range> ranges;
  std::vector<int> stack;
};

struct Tracer {
  std::atomic<int> on{0};
  std::atomic<int> device{0};  // also time ranges on the device (event pairs)
  std::chrono::steady_clock::time_point epoch = std::chrono::steady_clock::now();
  std::mutex mu;               // names, thread registry, event pool
  std::unordered_map<std::string, int> ids;
  std::vector<std::string> names;
  std::vector<ThreadLog*> logs;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
  hipEvent_t base = nullptr;   // device-time origin (recorded at enable)
  long long base_host = 0;
};
Tracer g_tr;
thread_local ThreadLog* t_log = nullptr;

long long now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                              g_tr.epoch).count();
}

ThreadLog* my_log() {
  if (!t_log) {
    t_log = new ThreadLog();
    std::lock_guard<std::mutex> g(g_tr.mu);
    t_log->tid = (int)g_tr.logs.size();
    g_tr.logs.push_back(t_log);
  }
  return t_log;
}

int intern(const char* name) {
  std::lock_guard<std::mutex> g(g_tr.mu);
  auto it = g_tr.ids.find(name);
  if (it != g_tr.ids.end()) return it->second;
  const int id = (int)g_tr.names.size();
  g_tr.names.emplace_back(name);
  g_tr.ids.emplace(name, id);
  return id;
}

void json_str(FILE* f, const std::string& s) {
  fputc('"', f);
  for (char c : s) {
    if (c == '"' || c == '\\') { fputc('\\', f); fputc(c, f); }
    else if ((unsigned char)c < 0x20) fprintf(f, "\\u%04x", c);
    else fputc(c, f);
  }
  fputc('"', f);
}

}  // namespace

// ---------------------------------------------------------------------------------- devices
PIAMD_EXPORT int piamd_dev_count(int* n) { return (int)hipGetDeviceCount(n); }

PIAMD_EXPORT int piamd_dev_props(int dev, DevProps* out) {
  hipDeviceProp_t p;
  const hipError_t e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) return (int)e;
  memset(out, 0, sizeof(*out));
  strncpy(out->name, p.name, sizeof(out->name) - 1);
  strncpy(out->arch, p.gcnArchName, sizeof(out->arch) - 1);
  out->major = p.major;
  out->minor = p.minor;
  out->cus = p.multiProcessorCount;
  out->clock_khz = p.clockRate;
  out->mem_clock_khz = p.memoryClockRate;
  out->bus_width = p.memoryBusWidth;
  out->total_mem = (long long)p.totalGlobalMem;
  out->l2_bytes = (long long)p.l2CacheSize;
  out->lds_per_block = (long long)p.sharedMemPerBlock;
  out->warp = p.warpSize;
  out->max_threads_per_block = p.maxThreadsPerBlock;
  out->regs_per_block = p.regsPerBlock;
  out->pci_bus = p.pciBusID;
  out->pci_dev = p.pciDeviceID;
  out->pci_domain = p.pciDomainID;
  out->cooperative = p.cooperativeLaunch;
  out->concurrent_kernels = p.concurrentKernels;
  return 0;
}

PIAMD_EXPORT int piamd_dev_synchronize(int dev) {
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess && dev != cur) e = hipSetDevice(dev);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (dev != cur) (void)hipSetDevice(cur);
  return (int)e;
}

PIAMD_EXPORT int piamd_dev_mem_info(int dev, long long* free_b, long long* total_b) {
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess && dev != cur) e = hipSetDevice(dev);
  size_t f = 0, t = 0;
  if (e == hipSuccess) e = hipMemGetInfo(&f, &t);
  if (dev != cur) (void)hipSetDevice(cur);
  *free_b = (long long)f;
  *total_b = (long long)t;
  return (int)e;
}

// ---------------------------------------------------------------------------------- streams
// priority: the HIP convention (lower = higher priority; clamped to the device's range).
PIAMD_EXPORT int piamd_stream_priority_range(int* least, int* greatest) {
  return (int)hipDeviceGetStreamPriorityRange(least, greatest);
}

PIAMD_EXPORT int piamd_stream_create(int dev, int priority, int nonblocking, void** out) {
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess && dev != cur) e = hipSetDevice(dev);
  hipStream_t s = nullptr;
  if (e == hipSuccess)
    e = hipStreamCreateWithPriority(&s, nonblocking ? hipStreamNonBlocking : hipStreamDefault, priority);
  if (dev != cur) (void)hipSetDevice(cur);
  *out = (void*)s;
  return (int)e;
}

PIAMD_EXPORT int piamd_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }
PIAMD_EXPORT int piamd_stream_sync(void* s) { return (int)hipStreamSynchronize((hipStream_t)s); }
// 1 = all work done, 0 = pending, < 0 = -error
PIAMD_EXPORT int piamd_stream_query(void* s) {
  const hipError_t e = hipStreamQuery((hipStream_t)s);
  return e == hipSuccess ? 1 : (e == hipErrorNotReady ? 0 : -(int)e);
}
PIAMD_EXPORT int piamd_stream_wait_event(void* s, void* ev) {
  return (int)hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)ev, 0);
}
PIAMD_EXPORT int piamd_stream_get_priority(void* s, int* p) {
  return (int)hipStreamGetPriority((hipStream_t)s, p);
}

// ---------------------------------------------------------------------------------- events
PIAMD_EXPORT int piamd_event_create(int timing, int blocking, void** out) {
  unsigned flags = 0;
  if (!timing) flags |= hipEventDisableTiming;
  if (blocking) flags |= hipEventBlockingSync;
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, flags);
  *out = (void*)e;
  return (int)r;
}
PIAMD_EXPORT int piamd_event_destroy(void* e) { return (int)hipEventDestroy((hipEvent_t)e); }
PIAMD_EXPORT int piamd_event_record(void* e, void* s) {
  return (int)hipEventRecord((hipEvent_t)e, (hipStream_t)s);
}
PIAMD_EXPORT int piamd_event_sync(void* e) { return (int)hipEventSynchronize((hipEvent_t)e); }
PIAMD_EXPORT int piamd_event_query(void* e) {
  const hipError_t r = hipEventQuery((hipEvent_t)e);
  return r == hipSuccess ? 1 : (r == hipErrorNotReady ? 0 : -(int)r);
}
PIAMD_EXPORT int piamd_event_elapsed(void* a, void* b, float* ms) {
  return (int)hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b);
}

// ---------------------------------------------------------------------------------- tracer
// enable: on / off; device: also time every range on the device (an event pair on `stream`,
// the stream current when the range opens — nullptr is the legacy default stream).
PIAMD_EXPORT int piamd_trace_enable(int on, int device, void* stream) {
  if (on) {
    std::lock_guard<std::mutex> g(g_tr.mu);
    for (ThreadLog* l : g_tr.logs) {
      l->ranges.clear();
      l->stack.clear();
    }
    for (auto& p : g_tr.evs) {
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
    g_tr.evs.clear();
    if (g_tr.base) (void)hipEventDestroy(g_tr.base);
    g_tr.base = nullptr;
    if (device) {
      if (hipEventCreate(&g_tr.base) != hipSuccess) return -1;
      (void)hipEventRecord(g_tr.base, (hipStream_t)stream);
    }
    g_tr.base_host = now_ns();
  }
  g_tr.device.store(on && device);
  g_tr.on.store(on);
  return 0;
}

PIAMD_EXPORT int piamd_trace_push(const char* name, void* stream) {
  if (!g_tr.on.load(std::memory_order_relaxed)) return 0;
  ThreadLog* l = my_log();
  Range r{intern(name), (int)l->stack.size(), now_ns(), -1, -1};
  if (g_tr.device.load(std::memory_order_relaxed)) {
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess) {
      (void)hipEventRecord(a, (hipStream_t)stream);
      std::lock_guard<std::mutex> g(g_tr.mu);
      r.ev = (int)g_tr.evs.size();
      g_tr.evs.emplace_back(a, b);
    }
  }
  l->stack.push_back((int)l->ranges.size());
  l->ranges.push_back(r);
  return 0;
}

PIAMD_EXPORT int piamd_trace_pop(void* stream) {
  if (!g_tr.on.load(std::memory_order_relaxed)) return 0;
  ThreadLog* l = my_log();
  if (l->stack.empty()) return -1;
  Range& r = l->ranges[l->stack.back()];
  l->stack.pop_back();
  r.t1 = now_ns();
  if (r.ev >= 0) {
    std::lock_guard<std::mutex> g(g_tr.mu);
    (void)hipEventRecord(g_tr.evs[r.ev].second, (hipStream_t)stream);
  }
  return 0;
}

// Number of closed ranges recorded so far (all threads).
PIAMD_EXPORT long long piamd_trace_count() {
  std::lock_guard<std::mutex> g(g_tr.mu);
  long long n = 0;
  for (ThreadLog* l : g_tr.logs)
    for (const Range& r : l->ranges) n += r.t1 >= 0;
  return n;
}

// Chrome trace JSON (Perfetto / chrome://tracing): host ranges as complete events on pid 0
// (one track per thread), device-timed ranges on pid 1 (synchronises on their end events).
// Returns the number of events written, < 0 on error.
PIAMD_EXPORT long long piamd_trace_dump(const char* path, int pid) {
  std::lock_guard<std::mutex> g(g_tr.mu);
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  fprintf(f, "{\"traceEvents\":[\n");
  long long n = 0;
  bool first = true;
  auto sep = [&] { if (!first) fprintf(f, ",\n"); first = false; };
  for (ThreadLog* l : g_tr.logs) {
    for (const Range& r : l->ranges) {
      if (r.t1 < 0) continue;
      sep();
      fprintf(f, "{\"ph\":\"X\",\"cat\":\"host\",\"name\":");
      json_str(f, g_tr.names[r.name]);
      fprintf(f, ",\"pid\":%d,\"tid\":%d,\"ts\":%.3f,\"dur\":%.3f,\"args\":{\"depth\":%d}}", pid, l->tid,
              (r.t0 - g_tr.base_host) / 1e3, (r.t1 - r.t0) / 1e3, r.depth);
      ++n;
      if (r.ev >= 0 && g_tr.base) {
        float a = 0.f, b = 0.f;
        const auto& p = g_tr.evs[r.ev];
        if (hipEventSynchronize(p.second) == hipSuccess &&
            hipEventElapsedTime(&a, g_tr.base, p.first) == hipSuccess &&
            hipEventElapsedTime(&b, g_tr.base, p.second) == hipSuccess) {
          sep();
          fprintf(f, "{\"ph\":\"X\",\"cat\":\"device\",\"name\":");
          json_str(f, g_tr.names[r.name]);
          fprintf(f, ",\"pid\":%d,\"tid\":%d,\"ts\":%.3f,\"dur\":%.3f}", pid + 1, l->tid, a * 1e3,
                  (b - a) * 1e3);
          ++n;
        }
      }
    }
  }
  fprintf(f, "\n],\"displayTimeUnit\":\"ms\"}\n");
  fclose(f);
  return n;
}
