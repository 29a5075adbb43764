// Internal structures of the native inference engine (see paddle_inference_api.h).
#pragma once

#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace pdn {

// framework.proto VarType.Type codes used by tensors
enum VT : int { VT_BOOL = 0, VT_INT16 = 1, VT_INT32 = 2, VT_INT64 = 3, VT_FP16 = 4, VT_FP32 = 5,
                VT_FP64 = 6, VT_UINT8 = 20, VT_INT8 = 21, VT_BF16 = 22,
                VT_LOD_TENSOR = 7, VT_FEED = 9, VT_FETCH = 10 };

inline size_t vt_size(int vt) {
  switch (vt) {
    case VT_BOOL: case VT_UINT8: case VT_INT8: return 1;
    case VT_INT16: case VT_FP16: case VT_BF16: return 2;
    case VT_INT32: case VT_FP32: return 4;
    case VT_INT64: case VT_FP64: return 8;
    default: throw std::runtime_error("unsupported tensor data type " + std::to_string(vt));
  }
}

// ------------------------------------------------------------------------ program description
struct Attr {
  int type = -1;  // framework.proto AttrType
  int64_t i = 0;
  float f = 0.f;
  double d = 0.0;
  bool b = false;
  std::string s;
  std::vector<int64_t> ints;
  std::vector<float> floats;
  std::vector<std::string> strings;
  std::vector<bool> bools;
};

struct OpDesc {
  std::string type;
  std::map<std::string, std::vector<std::string>> inputs, outputs;
  std::map<std::string, Attr> attrs;

  const std::string& in(const std::string& slot, size_t i = 0) const;
  bool has_in(const std::string& slot) const;
  const std::string& out(const std::string& slot, size_t i = 0) const;
  bool has_out(const std::string& slot) const;
  int64_t ai(const std::string& n, int64_t dflt) const;
  float af(const std::string& n, float dflt) const;
  bool ab(const std::string& n, bool dflt) const;
  std::string as(const std::string& n, const std::string& dflt) const;
  std::vector<int64_t> aints(const std::string& n) const;
};

struct VarDesc {
  std::string name;
  int type = VT_LOD_TENSOR;
  int dtype = VT_FP32;
  std::vector<int64_t> dims;
  bool persistable = false;
};

struct BlockDesc {
  int idx = 0, parent = -1;
  std::vector<VarDesc> vars;
  std::vector<OpDesc> ops;
};

struct ProgramDesc {
  std::vector<BlockDesc> blocks;
};

ProgramDesc parse_program(const std::string& bytes);

// ------------------------------------------------------------------------------ tensors
struct Buffer {
  void* p = nullptr;
  size_t bytes = 0;
  bool dev = false;
  bool owned = true;  // false: caller memory shared with Tensor::ShareExternalData (never freed here)
  ~Buffer();
};
std::shared_ptr<Buffer> alloc_buffer(size_t bytes, bool dev);

struct DTensor {
  int dtype = VT_FP32;
  std::vector<int64_t> dims;
  std::shared_ptr<Buffer> buf;

  int64_t numel() const {
    int64_t n = 1;
    for (auto d : dims) n *= d;
    return n;
  }
  size_t nbytes() const { return (size_t)numel() * vt_size(dtype); }
  template <typename T>
  T* data() const { return reinterpret_cast<T*>(buf->p); }
  bool on_dev() const { return buf && buf->dev; }
};

// params: persistable LoD tensors of block 0, sorted by name, read from the tensor stream
std::unordered_map<std::string, DTensor> load_params(const ProgramDesc& prog, const std::string& bytes);

// ------------------------------------------------------------------------------ execution
struct FastState;  // fast_ops.hip: weight copies and GEMM workspaces of the 16-bit GPU path

struct Ctx {
  bool gpu = false;
  void* stream = nullptr;  // hipStream_t
  void* blas = nullptr;    // rocblas_handle
  int device = 0;
  int threads = 1;
  int prec16 = 0;  // Config precision: 0 = as stored, VT_FP16 / VT_BF16 = 16-bit compute for fp32 models
  std::shared_ptr<FastState> fast;
  // buffers whose contents live as long as the predictor (loaded parameters and the weight caches
  // derived from them): the only sources the fast path's per-buffer caches may key on
  std::shared_ptr<std::unordered_set<const Buffer*>> persist;
  // load-time constants derived from parameters (e.g. folded batch-norm scale / shift), by key
  std::shared_ptr<std::map<std::string, DTensor>> consts;
};

using Scope = std::unordered_map<std::string, DTensor>;
using OpFn = std::function<void(Ctx&, const OpDesc&, Scope&)>;

// registry of op implementations (ops.cc); GPU variants dispatch inside each op
const std::unordered_map<std::string, OpFn>& op_registry();

// device helpers (gpu.hip); on a CPU-only build the GPU entry points throw
void dev_init(Ctx& c);
void dev_release(Ctx& c);
void dev_copy(void* dst, const void* src, size_t bytes, int kind /*0 h2d 1 d2h 2 d2d*/, Ctx& c);
void dev_sync(Ctx& c);
DTensor to_device(const DTensor& t, Ctx& c);
DTensor to_host(const DTensor& t, Ctx& c);
// hipGraph capture of the predictor's stream (relaxed mode: allocations stay outside the graph);
// every device buffer allocated during the capture is appended to `keep` (the graph's lifetime)
void graph_begin(Ctx& c, std::vector<std::shared_ptr<Buffer>>* keep);
void* graph_end(Ctx& c);  // instantiated executable graph
void graph_launch(Ctx& c, void* exec);
// after a failed capture: end a capture still open on the stream and clear the sticky error
void dev_reset_capture(Ctx& c);
void graph_destroy(void* exec);
// bf16 / fp16 → f32 on the host (output handles)
void half_to_float(const void* src, int dtype, float* dst, int64_t n);

}  // namespace pdn
