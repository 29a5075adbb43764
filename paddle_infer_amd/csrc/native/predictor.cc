// paddle_infer::Predictor on the native engine: load + validate the program, keep parameters
// resident on the predictor's device, run block 0 op by op, expose feed / fetch handles.
#include <algorithm>
#include <list>
#include <set>
#include <unordered_set>
#include <fstream>
#include <sstream>
#include <type_traits>

#include "engine.h"
#include "kernels.h"
#include "paddle_inference_api.h"

namespace paddle_infer {

namespace {
std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

template <typename T>
struct DtOf;
template <> struct DtOf<float> { static constexpr int v = pdn::VT_FP32; };
template <> struct DtOf<int64_t> { static constexpr int v = pdn::VT_INT64; };
template <> struct DtOf<int32_t> { static constexpr int v = pdn::VT_INT32; };
template <> struct DtOf<uint8_t> { static constexpr int v = pdn::VT_UINT8; };
template <> struct DtOf<int8_t> { static constexpr int v = pdn::VT_INT8; };
template <> struct DtOf<bool> { static constexpr int v = pdn::VT_BOOL; };

DataType to_api(int vt) {
  switch (vt) {
    case pdn::VT_FP32: return DataType::FLOAT32;
    case pdn::VT_INT64: return DataType::INT64;
    case pdn::VT_INT32: return DataType::INT32;
    case pdn::VT_UINT8: return DataType::UINT8;
    case pdn::VT_INT8: return DataType::INT8;
    case pdn::VT_FP16: return DataType::FLOAT16;  // 16-bit floats: CopyToCpu<float> converts
    case pdn::VT_BF16: return DataType::BFLOAT16;
    case pdn::VT_BOOL: return DataType::BOOL;
  }
  throw std::runtime_error("unsupported dtype " + std::to_string(vt));
}

int from_api(DataType d) {
  switch (d) {
    case DataType::FLOAT32: return pdn::VT_FP32;
    case DataType::INT64: return pdn::VT_INT64;
    case DataType::INT32: return pdn::VT_INT32;
    case DataType::UINT8: return pdn::VT_UINT8;
    case DataType::INT8: return pdn::VT_INT8;
    case DataType::FLOAT16: return pdn::VT_FP16;
    case DataType::BOOL: return pdn::VT_BOOL;
    case DataType::BFLOAT16: return pdn::VT_BF16;
  }
  throw std::runtime_error("unsupported DataType");
}
}  // namespace

class PredictorImpl {
 public:
  Config cfg;
  pdn::ProgramDesc prog;
  std::vector<std::string> feeds, fetches;
  pdn::Scope params;  // resident, on the predictor's place
  pdn::Scope scope;   // per-run (feeds, intermediates, fetches)
  pdn::Ctx ctx;

  explicit PredictorImpl(const Config& c) : cfg(c) {
    prog = pdn::parse_program(read_file(c.prog_file()));
    if (prog.blocks.empty()) throw std::runtime_error("empty program");
    const auto& reg = pdn::op_registry();
    std::vector<std::string> unknown;
    std::vector<std::pair<int64_t, std::string>> fd, ft;
    for (size_t bi = 1; bi < prog.blocks.size(); ++bi)
      if (!prog.blocks[bi].ops.empty())
        throw std::runtime_error("native engine: control-flow sub-blocks are not supported "
                                 "(use the Python Predictor)");
    for (const auto& op : prog.blocks[0].ops) {
      if (op.type == "feed") fd.emplace_back(op.ai("col", (int64_t)fd.size()), op.out("Out"));
      else if (op.type == "fetch") ft.emplace_back(op.ai("col", (int64_t)ft.size()), op.in("X"));
      else if (!reg.count(op.type) && !(c.use_gpu() && pdn::fast_knows(op.type)) &&
               std::find(unknown.begin(), unknown.end(), op.type) == unknown.end())
        unknown.push_back(op.type);
    }
    if (!unknown.empty()) {
      std::string m = "native engine: no kernel for op type(s):";
      for (auto& u : unknown) m += " " + u;
      throw std::runtime_error(m);
    }
    std::sort(fd.begin(), fd.end());
    std::sort(ft.begin(), ft.end());
    for (auto& p : fd) feeds.push_back(p.second);
    for (auto& p : ft) fetches.push_back(p.second);
    ctx.gpu = c.use_gpu();
    ctx.device = c.gpu_device_id();
    ctx.threads = std::max(1, c.cpu_math_library_num_threads());
    ctx.prec16 = c.precision() == PrecisionType::kBf16 ? pdn::VT_BF16
                 : c.precision() == PrecisionType::kHalf ? pdn::VT_FP16 : 0;
    if (ctx.gpu) pdn::dev_init(ctx);
    ctx.persist = std::make_shared<std::unordered_set<const pdn::Buffer*>>();
    ctx.consts = std::make_shared<std::map<std::string, pdn::DTensor>>();
    if (!c.params_file().empty()) {
      auto ps = pdn::load_params(prog, read_file(c.params_file()));
      for (auto& kv : ps) {
        params[kv.first] = ctx.gpu ? pdn::to_device(kv.second, ctx) : kv.second;
        ctx.persist->insert(params[kv.first].buf.get());
      }
    }
  }
  PredictorImpl(const PredictorImpl& o) : cfg(o.cfg), prog(o.prog), feeds(o.feeds), fetches(o.fetches),
                                          params(o.params) {
    ctx = o.ctx;
    ctx.stream = ctx.blas = nullptr;
    ctx.fast.reset();
    if (ctx.gpu) pdn::dev_init(ctx);  // own stream / BLAS handle, shared resident weights
  }
  ~PredictorImpl() {
    if (ctx.gpu) {
      try {
        pdn::dev_sync(ctx);
      } catch (...) {
      }
      drop_graphs();
    }
    scope.clear();
    if (ctx.gpu) {
      params.clear();
      pdn::fast_release(ctx);
      pdn::dev_release(ctx);
    }
  }

  void run_ops(pdn::Scope& s) {
    const auto& reg = pdn::op_registry();
    for (const auto& op : prog.blocks[0].ops) {
      if (op.type == "feed" || op.type == "fetch") continue;
      if (pdn::fast_run(ctx, op, s)) continue;
      auto it = reg.find(op.type);
      if (it == reg.end())
        throw std::runtime_error(op.type + ": the native engine runs this op only for bf16 / fp16 on the GPU");
      it->second(ctx, op, s);
    }
  }

  // hipGraph: one capture per feed signature (first Run: eager warm-up, then capture + launch).
  // The signature holds each feed's dtype and dims and, for caller memory shared with
  // ShareExternalData, its address: the captured kernels read and write (CacheKV) that address,
  // so a new pointer is a new capture, never a copy into the old one. A signature whose capture
  // failed (an op that reads device data back on the host) runs eagerly from then on.
  // Captures are kept in a small LRU (PIAMD_GRAPH_CACHE entries, default 4): a serving loop that
  // alternates signatures — two KV-cache buffers, prefill / decode shapes — replays each graph
  // instead of re-capturing on every switch.
  struct GraphEntry {
    std::string key;
    void* graph = nullptr;
    pdn::Scope scope;
    std::vector<std::shared_ptr<pdn::Buffer>> keep;  // every buffer the captured kernels touch
  };
  std::list<GraphEntry> graphs;  // most recently used first (list nodes: stable addresses)
  std::set<std::string> graph_failed;

  static size_t graph_capacity() {
    static const size_t cap = [] {
      const char* e = getenv("PIAMD_GRAPH_CACHE");
      const long v = e ? atol(e) : 4;
      return (size_t)(v < 1 ? 1 : v);
    }();
    return cap;
  }

  void drop_graphs() {
    for (auto& g : graphs) pdn::graph_destroy(g.graph);  // before the buffers they reference go
    graphs.clear();
  }

  bool run() {
    for (auto& kv : params) scope[kv.first] = kv.second;
    if (!(ctx.gpu && cfg.hip_graph_enabled())) {
      run_ops(scope);
      if (ctx.gpu) pdn::dev_sync(ctx);
      return true;
    }
    std::string key;
    for (auto& f : feeds) {
      const auto& t = tensor(f);
      key += f + ":" + std::to_string(t.dtype);
      for (auto d : t.dims) key += "," + std::to_string(d);
      if (t.buf && !t.buf->owned) key += "@" + std::to_string(reinterpret_cast<uintptr_t>(t.buf->p));
      key += ";";
    }
    if (graph_failed.count(key)) {
      run_ops(scope);
      pdn::dev_sync(ctx);
      return true;
    }
    auto hit = graphs.begin();
    while (hit != graphs.end() && hit->key != key) ++hit;
    if (hit == graphs.end()) {
      run_ops(scope);  // warm-up: weight copies, workspaces, code-object load
      pdn::dev_sync(ctx);
      graphs.emplace_front();
      GraphEntry& e = graphs.front();
      for (auto& kv : params) e.scope[kv.first] = kv.second;
      for (auto& f : feeds) e.scope[f] = tensor(f);
      pdn::graph_begin(ctx, &e.keep);
      bool ok = true;
      try {
        run_ops(e.scope);
      } catch (...) {
        ok = false;
      }
      void* g = nullptr;
      try {
        g = pdn::graph_end(ctx);
      } catch (...) {
        ok = false;
      }
      if (!ok) {
        // the warm-up above already produced this Run's outputs eagerly
        pdn::graph_destroy(g);
        pdn::dev_reset_capture(ctx);
        graphs.pop_front();
        graph_failed.insert(key);
        return true;
      }
      e.graph = g;
      e.key = key;
      while (graphs.size() > graph_capacity()) {
        pdn::graph_destroy(graphs.back().graph);
        graphs.pop_back();
      }
    } else {
      if (hit != graphs.begin()) graphs.splice(graphs.begin(), graphs, hit);
      GraphEntry& e = graphs.front();
      for (auto& f : feeds) {
        auto& src = tensor(f);
        auto& dst = e.scope.at(f);
        // owned buffers only: a shared external pointer is part of the key (same pointer here)
        if (src.buf != dst.buf && src.buf->owned && dst.buf->owned)
          pdn::dev_copy(dst.buf->p, src.buf->p, src.nbytes(), 2, ctx);
      }
    }
    GraphEntry& e = graphs.front();
    pdn::graph_launch(ctx, e.graph);
    for (auto& f : fetches) scope[f] = e.scope.at(f);
    pdn::dev_sync(ctx);
    return true;
  }

  size_t graph_count() const { return graphs.size(); }

  pdn::DTensor& tensor(const std::string& n) {
    auto it = scope.find(n);
    if (it == scope.end()) throw std::runtime_error("tensor '" + n + "' has no value");
    return it->second;
  }
};

// ------------------------------------------------------------------------------ Tensor
void Tensor::Reshape(const std::vector<int>& shape) { pending_shape_ = shape; }

template <typename T>
void Tensor::CopyFromCpu(const T* data) {
  if (!input_) throw std::runtime_error("CopyFromCpu on an output handle");
  pdn::DTensor t;
  t.dtype = DtOf<T>::v;
  for (int d : pending_shape_) t.dims.push_back(d);
  t.buf = pdn::alloc_buffer(t.nbytes(), p_->ctx.gpu);
  if (p_->ctx.gpu) pdn::dev_copy(t.buf->p, data, t.nbytes(), 0, p_->ctx);
  else std::memcpy(t.buf->p, data, t.nbytes());
  p_->scope[name_] = t;
}

void Tensor::ShareExternalData(void* data, const std::vector<int>& shape, PlaceType place, DataType dtype) {
  if (!input_) throw std::runtime_error("ShareExternalData on an output handle");
  if ((place == PlaceType::kGPU) != p_->ctx.gpu)
    throw std::runtime_error("ShareExternalData: the data must live on the predictor's place");
  pdn::DTensor t;
  t.dtype = from_api(dtype);
  for (int d : shape) t.dims.push_back(d);
  t.buf = std::make_shared<pdn::Buffer>();
  t.buf->p = data;
  t.buf->bytes = t.nbytes();
  t.buf->dev = p_->ctx.gpu;
  t.buf->owned = false;
  p_->scope[name_] = t;
}

template <typename T>
void Tensor::CopyToCpu(T* data) const {
  const pdn::DTensor& t = p_->tensor(name_);
  if (std::is_same<T, float>::value && pdn::is16(t.dtype)) {  // 16-bit outputs read as float
    pdn::DTensor h = t.on_dev() ? pdn::to_host(t, p_->ctx) : t;
    pdn::half_to_float(h.buf->p, t.dtype, reinterpret_cast<float*>(data), t.numel());
    return;
  }
  if (t.dtype != DtOf<T>::v) throw std::runtime_error("CopyToCpu: dtype mismatch for " + name_);
  if (t.on_dev()) pdn::dev_copy(data, t.buf->p, t.nbytes(), 1, p_->ctx);
  else std::memcpy(data, t.buf->p, t.nbytes());
}

std::vector<int> Tensor::shape() const {
  if (input_ && !p_->scope.count(name_)) return pending_shape_;
  const auto& t = p_->tensor(name_);
  return std::vector<int>(t.dims.begin(), t.dims.end());
}
DataType Tensor::type() const { return to_api(p_->tensor(name_).dtype); }
PlaceType Tensor::place() const { return p_->ctx.gpu ? PlaceType::kGPU : PlaceType::kCPU; }

template void Tensor::CopyFromCpu<float>(const float*);
template void Tensor::CopyFromCpu<int64_t>(const int64_t*);
template void Tensor::CopyFromCpu<int32_t>(const int32_t*);
template void Tensor::CopyFromCpu<uint8_t>(const uint8_t*);
template void Tensor::CopyFromCpu<int8_t>(const int8_t*);
template void Tensor::CopyToCpu<float>(float*) const;
template void Tensor::CopyToCpu<int64_t>(int64_t*) const;
template void Tensor::CopyToCpu<int32_t>(int32_t*) const;
template void Tensor::CopyToCpu<uint8_t>(uint8_t*) const;
template void Tensor::CopyToCpu<int8_t>(int8_t*) const;

// ------------------------------------------------------------------------------ Predictor
Predictor::Predictor(const Config& config) : impl_(std::make_shared<PredictorImpl>(config)) {}
Predictor::Predictor(std::shared_ptr<PredictorImpl> impl) : impl_(std::move(impl)) {}
Predictor::~Predictor() = default;
std::vector<std::string> Predictor::GetInputNames() { return impl_->feeds; }
std::vector<std::string> Predictor::GetOutputNames() { return impl_->fetches; }
std::unique_ptr<Tensor> Predictor::GetInputHandle(const std::string& name) {
  if (std::find(impl_->feeds.begin(), impl_->feeds.end(), name) == impl_->feeds.end())
    throw std::runtime_error("no input named " + name);
  return std::unique_ptr<Tensor>(new Tensor(impl_.get(), name, true));
}
std::unique_ptr<Tensor> Predictor::GetOutputHandle(const std::string& name) {
  if (std::find(impl_->fetches.begin(), impl_->fetches.end(), name) == impl_->fetches.end())
    throw std::runtime_error("no output named " + name);
  return std::unique_ptr<Tensor>(new Tensor(impl_.get(), name, false));
}
bool Predictor::Run() { return impl_->run(); }
std::unique_ptr<Predictor> Predictor::Clone() {
  return std::unique_ptr<Predictor>(new Predictor(std::make_shared<PredictorImpl>(*impl_)));
}
void Predictor::ClearIntermediateTensor() {
  pdn::Scope keep;
  for (auto& n : impl_->fetches)
    if (impl_->scope.count(n)) keep[n] = impl_->scope[n];
  impl_->scope.swap(keep);
}
std::vector<std::string> Predictor::OpTypes() const {
  std::vector<std::string> v;
  for (const auto& op : impl_->prog.blocks[0].ops) v.push_back(op.type);
  return v;
}

std::shared_ptr<Predictor> CreatePredictor(const Config& config) { return std::make_shared<Predictor>(config); }
std::string GetVersion() { return "paddle_infer_amd native 0.3 (MI355X / gfx950)"; }

}  // namespace paddle_infer
