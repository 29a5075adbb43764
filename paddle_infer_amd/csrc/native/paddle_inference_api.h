// Native C++ inference API — no Python, no PyTorch at run time.
//
// Parity: reference `paddle/fluid/inference/api/paddle_inference_api.h:80` (namespace
// paddle_infer: Config, Predictor, Tensor, CreatePredictor, GetVersion) and
// `paddle_analysis_config.h` (SetModel, EnableUseGpu, DisableGpu, SetCpuMathLibraryNumThreads,
// SwitchIrOptim). A Predictor loads a Paddle `.pdmodel` (framework.proto ProgramDesc, decoded by
// a hand-written wire reader) and `.pdiparams` (save_combine tensor stream), and executes block 0
// op by op: plain C++ on the CPU; on the MI355X, bf16 / fp16 models run on the framework's own
// kernels (libpiamd_kernels.so + the assembly GEMM code object: fast_ops.hip) and fp32 ones on the
// engine's HIP kernels, one HIP stream per predictor, optional whole-Run hipGraph capture.
//
// Op set: feed, fetch, matmul_v2, matmul, mul, fc, elementwise_{add,sub,mul,div,max,min,pow},
// scale, relu, gelu, tanh, sigmoid, silu, swish, exp, sqrt, rsqrt, abs, softmax, layer_norm,
// lookup_table(_v2), transpose(2), reshape(2), unsqueeze(2), squeeze(2), flatten_contiguous_range,
// concat, split, slice, cast, fill_constant, assign, dropout (inference), reduce_mean, reduce_sum,
// conv2d, pool2d, batch_norm and the fused transformer ops of an IR-optimised program
// (multihead_matmul, skip_layernorm, fused_fc_elementwise_layernorm,
// fused_embedding_eltwise_layernorm, fused_multi_transformer). Anything else is rejected when the
// model is loaded (the reference predictor refuses unregistered ops the same way).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace paddle_infer {

enum class DataType { FLOAT32 = 0, INT64 = 1, INT32 = 2, UINT8 = 3, INT8 = 4, FLOAT16 = 5, BOOL = 6,
                      BFLOAT16 = 7 };
enum class PlaceType { kUNK = -1, kCPU = 0, kGPU = 1 };
// compute precision of an fp32 model on the GPU (reference `paddle_infer::PrecisionType`)
enum class PrecisionType { kFloat32 = 0, kInt8 = 1, kHalf = 2, kBf16 = 3 };

class Config {
 public:
  Config() = default;
  Config(const std::string& prog_file, const std::string& params_file)
      : prog_file_(prog_file), params_file_(params_file) {}
  void SetModel(const std::string& prog_file, const std::string& params_file) {
    prog_file_ = prog_file;
    params_file_ = params_file;
  }
  const std::string& prog_file() const { return prog_file_; }
  const std::string& params_file() const { return params_file_; }
  void EnableUseGpu(uint64_t memory_pool_init_size_mb, int device_id = 0,
                    PrecisionType precision = PrecisionType::kFloat32) {
    use_gpu_ = true;
    device_id_ = device_id;
    precision_ = precision;
    (void)memory_pool_init_size_mb;
  }
  PrecisionType precision() const { return precision_; }
  void DisableGpu() { use_gpu_ = false; }
  bool use_gpu() const { return use_gpu_; }
  int gpu_device_id() const { return device_id_; }
  void SetCpuMathLibraryNumThreads(int n) { cpu_threads_ = n; }
  int cpu_math_library_num_threads() const { return cpu_threads_; }
  void SwitchIrOptim(bool on = true) { ir_optim_ = on; }
  bool ir_optim() const { return ir_optim_; }
  void EnableMemoryOptim(bool on = true) { mem_optim_ = on; }
  bool enable_memory_optim() const { return mem_optim_; }
  // GPU: capture the whole Run() into one hipGraph per input-shape signature (replayed after)
  void EnableHipGraph(bool on = true) { hip_graph_ = on; }
  bool hip_graph_enabled() const { return hip_graph_; }

 private:
  std::string prog_file_, params_file_;
  bool use_gpu_ = false, ir_optim_ = true, mem_optim_ = true, hip_graph_ = false;
  int device_id_ = 0, cpu_threads_ = 1;
  PrecisionType precision_ = PrecisionType::kFloat32;
};

class PredictorImpl;
struct TensorSlot;

class Tensor {
 public:
  void Reshape(const std::vector<int>& shape);
  template <typename T>
  void CopyFromCpu(const T* data);
  template <typename T>
  void CopyToCpu(T* data) const;
  // zero-copy input: the predictor reads (and in-place ops such as fused_multi_transformer's
  // CacheKV write) `data` directly; the caller keeps it alive. place must be the predictor's.
  void ShareExternalData(void* data, const std::vector<int>& shape, PlaceType place, DataType dtype);
  std::vector<int> shape() const;
  DataType type() const;
  const std::string& name() const { return name_; }
  PlaceType place() const;

 private:
  friend class PredictorImpl;
  friend class Predictor;
  Tensor(PredictorImpl* p, std::string name, bool input) : p_(p), name_(std::move(name)), input_(input) {}
  PredictorImpl* p_;
  std::string name_;
  bool input_;
  std::vector<int> pending_shape_;
};

class Predictor {
 public:
  explicit Predictor(const Config& config);
  ~Predictor();
  std::vector<std::string> GetInputNames();
  std::vector<std::string> GetOutputNames();
  std::unique_ptr<Tensor> GetInputHandle(const std::string& name);
  std::unique_ptr<Tensor> GetOutputHandle(const std::string& name);
  bool Run();
  std::unique_ptr<Predictor> Clone();
  void ClearIntermediateTensor();
  // op types of the loaded program, in execution order (diagnostics)
  std::vector<std::string> OpTypes() const;

 private:
  explicit Predictor(std::shared_ptr<PredictorImpl> impl);
  std::shared_ptr<PredictorImpl> impl_;
};

std::shared_ptr<Predictor> CreatePredictor(const Config& config);
std::string GetVersion();

}  // namespace paddle_infer
