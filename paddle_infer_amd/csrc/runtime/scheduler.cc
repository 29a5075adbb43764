// Native runtime for the static-graph executor and the inference predictor.
//
// Parity: reference `paddle/fluid/framework/new_executor/interpretercore.cc` +
// `interpreter/dependency_builder.cc` (op dependency analysis: RAW / WAR / WAW edges, topological
// instruction list, per-instruction GC list = variables whose last use is that instruction) and
// `paddle/fluid/framework/ir/memory_optimize_pass/` (liveness-based buffer reuse).
//
// Exposed as a C ABI (ctypes) over CSR-encoded op→var lists:
//   piamd_plan    : dependency graph, deterministic topological order (program order preferred),
//                   GC lists, dependency depth ("level") per op for multi-stream dispatch.
//   piamd_memplan : static arena planning — greedy best-fit of (size, [first,last]) lifetimes
//                   into one device arena; the inference predictor allocates ONE buffer and slices
//                   every intermediate out of it, which also makes hipGraph capture address-stable.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <queue>
#include <vector>

#define PIAMD_EXPORT extern "C" __attribute__((visibility("default")))

PIAMD_EXPORT int piamd_runtime_version() { return 1; }

PIAMD_EXPORT int piamd_plan(int num_ops, int num_vars, const int* in_ptr, const int* in_idx,
                            const int* out_ptr, const int* out_idx, const unsigned char* keep,
                            int* order, int* free_ptr, int* free_idx, int* level) {
  if (num_ops < 0 || num_vars < 0) return -1;
  std::vector<std::vector<int>> succ(num_ops);
  std::vector<int> indeg(num_ops, 0);
  std::vector<int> last_writer(num_vars, -1);
  std::vector<std::vector<int>> readers_since_write(num_vars);
  auto add_edge = [&](int a, int b) {
    if (a < 0 || a == b) return;
    succ[a].push_back(b);
  };
  for (int op = 0; op < num_ops; ++op) {
    for (int k = in_ptr[op]; k < in_ptr[op + 1]; ++k) {
      const int v = in_idx[k];
      if (v < 0 || v >= num_vars) return -2;
      add_edge(last_writer[v], op);  // RAW
    }
    for (int k = out_ptr[op]; k < out_ptr[op + 1]; ++k) {
      const int v = out_idx[k];
      if (v < 0 || v >= num_vars) return -2;
      add_edge(last_writer[v], op);                       // WAW
      for (int r : readers_since_write[v]) add_edge(r, op);  // WAR
    }
    for (int k = in_ptr[op]; k < in_ptr[op + 1]; ++k) readers_since_write[in_idx[k]].push_back(op);
    for (int k = out_ptr[op]; k < out_ptr[op + 1]; ++k) {
      last_writer[out_idx[k]] = op;
      readers_since_write[out_idx[k]].clear();
    }
  }
  for (int a = 0; a < num_ops; ++a) {
    auto& s = succ[a];
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
    for (int b : s) ++indeg[b];
  }
  // Kahn with a min-heap on the original index: the program order whenever it is legal.
  std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
  std::vector<int> depth(num_ops, 0);
  for (int i = 0; i < num_ops; ++i)
    if (indeg[i] == 0) ready.push(i);
  int n = 0;
  while (!ready.empty()) {
    const int a = ready.top();
    ready.pop();
    order[n++] = a;
    for (int b : succ[a]) {
      depth[b] = std::max(depth[b], depth[a] + 1);
      if (--indeg[b] == 0) ready.push(b);
    }
  }
  if (n != num_ops) return -3;  // cycle
  for (int i = 0; i < num_ops; ++i) level[i] = depth[i];
  // GC: last use position of every non-kept variable
  std::vector<int> pos(num_ops);
  for (int i = 0; i < num_ops; ++i) pos[order[i]] = i;
  std::vector<int> last_use(num_vars, -1);
  for (int op = 0; op < num_ops; ++op) {
    for (int k = in_ptr[op]; k < in_ptr[op + 1]; ++k)
      last_use[in_idx[k]] = std::max(last_use[in_idx[k]], pos[op]);
    for (int k = out_ptr[op]; k < out_ptr[op + 1]; ++k)
      last_use[out_idx[k]] = std::max(last_use[out_idx[k]], pos[op]);
  }
  std::vector<std::vector<int>> frees(num_ops);
  for (int v = 0; v < num_vars; ++v)
    if (last_use[v] >= 0 && !(keep && keep[v])) frees[last_use[v]].push_back(v);
  int c = 0;
  for (int i = 0; i < num_ops; ++i) {
    free_ptr[i] = c;
    for (int v : frees[i]) free_idx[c++] = v;
  }
  free_ptr[num_ops] = c;
  return 0;
}

// Greedy best-fit arena planning. Buffers sorted by size (desc); each is placed at the lowest
// aligned offset not overlapping any already-placed buffer whose [first, last] interval intersects.
PIAMD_EXPORT long long piamd_memplan(int n, const long long* sizes, const int* first,
                                     const int* last, long long align, long long* offsets) {
  if (align <= 0) align = 256;
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return sizes[a] > sizes[b]; });
  struct Placed { long long off, end; int first, last; };
  std::vector<Placed> placed;
  long long total = 0;
  for (int i : idx) {
    const long long sz = (sizes[i] + align - 1) / align * align;
    std::vector<std::pair<long long, long long>> busy;
    for (const auto& p : placed)
      if (!(p.last < first[i] || last[i] < p.first)) busy.push_back({p.off, p.end});
    std::sort(busy.begin(), busy.end());
    long long cand = 0;
    for (const auto& b : busy) {
      if (cand + sz <= b.first) break;
      cand = std::max(cand, b.second);
    }
    offsets[i] = cand;
    placed.push_back({cand, cand + sz, first[i], last[i]});
    total = std::max(total, cand + sz);
  }
  return total;
}
