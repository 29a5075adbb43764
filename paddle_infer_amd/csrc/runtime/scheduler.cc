// Native runtime for the static-graph executor and the inference predictor.
//
// Parity: reference `paddle/fluid/framework/new_executor/interpretercore.cc` +
// `interpreter/dependency_builder.cc` (op dependency analysis: RAW / WAR / WAW edges, topological
// instruction list, per-instruction GC list = variables whose last use is that instruction) and
// `paddle/fluid/framework/ir/memory_optimize_pass/` (liveness-based buffer reuse).
//
// Exposed as a C ABI (ctypes) over CSR-encoded op→var lists:
//   piamd_plan : dependency graph, deterministic topological order (program order preferred),
//                GC lists (the executor drops a variable right after its last consumer: forward
//                activations of a training program live exactly until their grad op ran), and the
//                dependency depth of every op.
//   piamd_stream_plan : stream assignment (compute stream 0, communication stream 1) and the
//                cross-stream event waits of every op (reference `new_executor/interpreter/
//                stream_analyzer.cc` + `interpretercore.cc` event insertion): an op waits only on
//                the LATEST predecessor of each other stream, and not at all when an earlier op of
//                its own stream already waited on that event or a later one (streams are in-order).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <queue>
#include <vector>

#define PIAMD_EXPORT extern "C" __attribute__((visibility("default")))

PIAMD_EXPORT int piamd_runtime_version() { return 1; }

namespace {
// RAW / WAW / WAR successor lists over the ops in program order (sorted, unique); false on a bad
// variable index
bool build_edges(int num_ops, int num_vars, const int* in_ptr, const int* in_idx, const int* out_ptr,
                 const int* out_idx, std::vector<std::vector<int>>& succ) {
  succ.assign(num_ops, {});
  std::vector<int> last_writer(num_vars, -1);
  std::vector<std::vector<int>> readers_since_write(num_vars);
  auto add_edge = [&](int a, int b) {
    if (a < 0 || a == b) return;
    succ[a].push_back(b);
  };
  for (int op = 0; op < num_ops; ++op) {
    for (int k = in_ptr[op]; k < in_ptr[op + 1]; ++k) {
      const int v = in_idx[k];
      if (v < 0 || v >= num_vars) return false;
      add_edge(last_writer[v], op);
    }
    for (int k = out_ptr[op]; k < out_ptr[op + 1]; ++k) {
      const int v = out_idx[k];
      if (v < 0 || v >= num_vars) return false;
      add_edge(last_writer[v], op);
      for (int r : readers_since_write[v]) add_edge(r, op);
    }
    for (int k = in_ptr[op]; k < in_ptr[op + 1]; ++k) readers_since_write[in_idx[k]].push_back(op);
    for (int k = out_ptr[op]; k < out_ptr[op + 1]; ++k) {
      last_writer[out_idx[k]] = op;
      readers_since_write[out_idx[k]].clear();
    }
  }
  for (auto& s : succ) {
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
  }
  return true;
}
}  // namespace

PIAMD_EXPORT int piamd_stream_plan(int num_ops, int num_vars, const int* in_ptr, const int* in_idx,
                                   const int* out_ptr, const int* out_idx, const int* order,
                                   const unsigned char* is_comm, int* stream_of, int* wait_ptr, int* wait_idx,
                                   unsigned char* record) {
  if (num_ops < 0 || num_vars < 0) return -1;
  std::vector<std::vector<int>> succ;
  if (!build_edges(num_ops, num_vars, in_ptr, in_idx, out_ptr, out_idx, succ)) return -2;
  constexpr int NS = 2;
  std::vector<int> pos(num_ops, -1);
  for (int i = 0; i < num_ops; ++i) {
    if (order[i] < 0 || order[i] >= num_ops || pos[order[i]] >= 0) return -4;
    pos[order[i]] = i;
  }
  std::vector<std::vector<int>> pred(num_ops);
  for (int a = 0; a < num_ops; ++a) {
    stream_of[a] = is_comm[a] ? 1 : 0;
    for (int b : succ[a]) pred[b].push_back(a);
    record[a] = 0;
  }
  // covered[s][t]: the latest position of a stream-t op that stream s has already waited for
  std::vector<std::vector<int>> covered(NS, std::vector<int>(NS, -1));
  int c = 0;
  for (int i = 0; i < num_ops; ++i) {
    const int b = order[i], sb = stream_of[b];
    wait_ptr[i] = c;
    int best[NS] = {-1, -1};
    for (int a : pred[b]) {
      const int sa = stream_of[a];
      if (sa == sb) continue;
      if (pos[a] > i) return -5;  // a predecessor after its successor: not a valid order
      if (best[sa] < 0 || pos[a] > pos[best[sa]]) best[sa] = a;
    }
    for (int t = 0; t < NS; ++t) {
      const int a = best[t];
      if (a < 0 || pos[a] <= covered[sb][t]) continue;
      covered[sb][t] = pos[a];
      wait_idx[c++] = a;
      record[a] = 1;
    }
  }
  wait_ptr[num_ops] = c;
  return 0;
}

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
