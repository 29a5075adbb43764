// The reference C API (`capi_exp` pd_inference_api.h, declared in ../capi/pd_inference_api.h)
// on the native C++ engine: libpiamd_infer.so exports the Config / Predictor / Tensor / utility
// entry points a C deployment uses, with no Python interpreter behind them.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../capi/pd_inference_api.h"
#include "paddle_inference_api.h"

struct PD_Config {
  paddle_infer::Config cfg;
  std::string prog, params;
  int mem_mb = 0;
};
struct PD_Tensor;
struct PD_Predictor {
  std::shared_ptr<paddle_infer::Predictor> p;
  std::vector<PD_Tensor*> live;  // handles whose MutableData staging is flushed by Run
};
struct PD_Tensor {
  std::unique_ptr<paddle_infer::Tensor> t;
  std::string name;
  PD_Predictor* owner = nullptr;
  std::vector<char> staged;  // PD_TensorMutableData* host staging (copied in before Run)
  int staged_dt = -1;        // PD_DATA_* of the staged data, -1 = none
  std::vector<int> shape;
};

namespace {
char* dup(const std::string& s) {
  char* c = (char*)std::malloc(s.size() + 1);
  std::memcpy(c, s.c_str(), s.size() + 1);
  return c;
}
PD_OneDimArrayCstr* cstr_array(const std::vector<std::string>& v) {
  auto* a = (PD_OneDimArrayCstr*)std::malloc(sizeof(PD_OneDimArrayCstr));
  a->size = v.size();
  a->data = (char**)std::malloc(sizeof(char*) * (v.empty() ? 1 : v.size()));
  for (size_t i = 0; i < v.size(); ++i) a->data[i] = dup(v[i]);
  return a;
}
template <typename F>
auto guarded(F&& f, decltype(f()) fail) -> decltype(f()) {
  try {
    return f();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[paddle_infer_amd native] %s\n", e.what());
    return fail;
  }
}
}  // namespace

extern "C" {

PD_Config* PD_ConfigCreate() { return new PD_Config(); }
void PD_ConfigDestroy(PD_Config* c) { delete c; }
void PD_ConfigSetModel(PD_Config* c, const char* prog, const char* params) {
  c->prog = prog ? prog : "";
  c->params = params ? params : "";
  c->cfg.SetModel(c->prog, c->params);
}
void PD_ConfigSetProgFile(PD_Config* c, const char* prog) { PD_ConfigSetModel(c, prog, c->params.c_str()); }
void PD_ConfigSetParamsFile(PD_Config* c, const char* params) { PD_ConfigSetModel(c, c->prog.c_str(), params); }
const char* PD_ConfigGetProgFile(PD_Config* c) { return c->prog.c_str(); }
const char* PD_ConfigGetParamsFile(PD_Config* c) { return c->params.c_str(); }
void PD_ConfigEnableUseGpu(PD_Config* c, uint64_t mem_mb, int32_t device_id, PD_PrecisionType prec) {
  c->mem_mb = (int)mem_mb;
  using P = paddle_infer::PrecisionType;
  c->cfg.EnableUseGpu(mem_mb, device_id,
                      prec == PD_PRECISION_BFLOAT16 ? P::kBf16 : prec == PD_PRECISION_HALF ? P::kHalf : P::kFloat32);
}
void PD_ConfigDisableGpu(PD_Config* c) { c->cfg.DisableGpu(); }
void PD_ConfigEnableHipGraph(PD_Config* c, PD_Bool x) { c->cfg.EnableHipGraph(x != 0); }
PD_Bool PD_ConfigUseGpu(PD_Config* c) { return c->cfg.use_gpu(); }
int32_t PD_ConfigGpuDeviceId(PD_Config* c) { return c->cfg.gpu_device_id(); }
int32_t PD_ConfigMemoryPoolInitSizeMb(PD_Config* c) { return c->mem_mb; }
void PD_ConfigSwitchIrOptim(PD_Config* c, PD_Bool x) { c->cfg.SwitchIrOptim(x != 0); }
PD_Bool PD_ConfigIrOptim(PD_Config* c) { return c->cfg.ir_optim(); }
void PD_ConfigSetCpuMathLibraryNumThreads(PD_Config* c, int32_t n) { c->cfg.SetCpuMathLibraryNumThreads(n); }
int32_t PD_ConfigGetCpuMathLibraryNumThreads(PD_Config* c) { return c->cfg.cpu_math_library_num_threads(); }
void PD_ConfigEnableMemoryOptim(PD_Config* c, PD_Bool x) { c->cfg.EnableMemoryOptim(x != 0); }
PD_Bool PD_ConfigMemoryOptimEnabled(PD_Config* c) { return c->cfg.enable_memory_optim(); }
PD_Bool PD_ConfigIsValid(PD_Config* c) { return !c->prog.empty(); }

PD_Predictor* PD_PredictorCreate(PD_Config* c) {
  PD_Predictor* p = guarded([&]() -> PD_Predictor* {
    auto* r = new PD_Predictor();
    r->p = paddle_infer::CreatePredictor(c->cfg);
    return r;
  }, nullptr);
  delete c;  // __pd_take
  return p;
}
PD_Predictor* PD_PredictorClone(PD_Predictor* p) {
  return guarded([&]() -> PD_Predictor* {
    auto* r = new PD_Predictor();
    r->p = std::shared_ptr<paddle_infer::Predictor>(p->p->Clone().release());
    return r;
  }, nullptr);
}
PD_OneDimArrayCstr* PD_PredictorGetInputNames(PD_Predictor* p) { return cstr_array(p->p->GetInputNames()); }
PD_OneDimArrayCstr* PD_PredictorGetOutputNames(PD_Predictor* p) { return cstr_array(p->p->GetOutputNames()); }
size_t PD_PredictorGetInputNum(PD_Predictor* p) { return p->p->GetInputNames().size(); }
size_t PD_PredictorGetOutputNum(PD_Predictor* p) { return p->p->GetOutputNames().size(); }
PD_Tensor* PD_PredictorGetInputHandle(PD_Predictor* p, const char* name) {
  return guarded([&]() -> PD_Tensor* {
    auto* t = new PD_Tensor();
    t->t = p->p->GetInputHandle(name);
    t->name = name;
    t->owner = p;
    p->live.push_back(t);
    return t;
  }, nullptr);
}
PD_Tensor* PD_PredictorGetOutputHandle(PD_Predictor* p, const char* name) {
  return guarded([&]() -> PD_Tensor* {
    auto* t = new PD_Tensor();
    t->t = p->p->GetOutputHandle(name);
    t->name = name;
    return t;
  }, nullptr);
}
namespace {
void flush(PD_Tensor* t) {
  if (t->staged_dt < 0) return;
  switch (t->staged_dt) {
    case PD_DATA_FLOAT32: t->t->CopyFromCpu(reinterpret_cast<const float*>(t->staged.data())); break;
    case PD_DATA_INT64: t->t->CopyFromCpu(reinterpret_cast<const int64_t*>(t->staged.data())); break;
    case PD_DATA_INT32: t->t->CopyFromCpu(reinterpret_cast<const int32_t*>(t->staged.data())); break;
    case PD_DATA_UINT8: t->t->CopyFromCpu(reinterpret_cast<const uint8_t*>(t->staged.data())); break;
    case PD_DATA_INT8: t->t->CopyFromCpu(reinterpret_cast<const int8_t*>(t->staged.data())); break;
  }
  t->staged_dt = -1;
}
}  // namespace

PD_Bool PD_PredictorRun(PD_Predictor* p) {
  return guarded([&]() -> PD_Bool {
    for (PD_Tensor* t : p->live) flush(t);
    return p->p->Run();
  }, (PD_Bool)0);
}
void PD_PredictorClearIntermediateTensor(PD_Predictor* p) { p->p->ClearIntermediateTensor(); }
uint64_t PD_PredictorTryShrinkMemory(PD_Predictor* p) {
  p->p->ClearIntermediateTensor();
  return 0;
}
void PD_PredictorDestroy(PD_Predictor* p) {
  for (PD_Tensor* t : p->live) t->owner = nullptr;
  delete p;
}

void PD_TensorDestroy(PD_Tensor* t) {
  if (!t) return;
  if (t->owner) {
    guarded([&]() -> int { flush(t); return 0; }, 1);
    auto& v = t->owner->live;
    v.erase(std::remove(v.begin(), v.end(), t), v.end());
  }
  delete t;
}
void PD_TensorReshape(PD_Tensor* t, size_t n, int32_t* shape) {
  t->shape.assign(shape, shape + n);
  t->t->Reshape(t->shape);
}
#define PD_MUTABLE(SUF, T, DT)                                                                 \
  T* PD_TensorMutableData##SUF(PD_Tensor* t, PD_PlaceType) {                                   \
    size_t n = 1;                                                                              \
    for (int d : t->shape) n *= (size_t)d;                                                     \
    t->staged.resize(n * sizeof(T));                                                           \
    t->staged_dt = DT;                                                                         \
    return reinterpret_cast<T*>(t->staged.data());                                             \
  }
PD_MUTABLE(Float, float, PD_DATA_FLOAT32)
PD_MUTABLE(Int64, int64_t, PD_DATA_INT64)
PD_MUTABLE(Int32, int32_t, PD_DATA_INT32)
PD_MUTABLE(Uint8, uint8_t, PD_DATA_UINT8)
PD_MUTABLE(Int8, int8_t, PD_DATA_INT8)
#undef PD_MUTABLE
PD_Bool PD_ConfigTensorRtEngineEnabled(PD_Config*) { return 0; }
#define PD_COPY(SUF, T)                                                                        \
  void PD_TensorCopyFromCpu##SUF(PD_Tensor* t, const T* d) {                                   \
    guarded([&]() -> int { t->t->CopyFromCpu(d); return 0; }, 1);                              \
  }                                                                                            \
  void PD_TensorCopyToCpu##SUF(PD_Tensor* t, T* d) {                                           \
    guarded([&]() -> int { t->t->CopyToCpu(d); return 0; }, 1);                                \
  }
PD_COPY(Float, float)
PD_COPY(Int64, int64_t)
PD_COPY(Int32, int32_t)
PD_COPY(Uint8, uint8_t)
PD_COPY(Int8, int8_t)
#undef PD_COPY
void PD_TensorShareExternalData(PD_Tensor* t, void* data, size_t n, int32_t* shape, PD_PlaceType place,
                                PD_DataType dt) {
  using D = paddle_infer::DataType;
  guarded([&]() -> int {
    D d;
    switch (dt) {
      case PD_DATA_FLOAT32: d = D::FLOAT32; break;
      case PD_DATA_INT32: d = D::INT32; break;
      case PD_DATA_INT64: d = D::INT64; break;
      case PD_DATA_UINT8: d = D::UINT8; break;
      case PD_DATA_INT8: d = D::INT8; break;
      case PD_DATA_FLOAT16: d = D::FLOAT16; break;
      case PD_DATA_BOOL: d = D::BOOL; break;
      case PD_DATA_BFLOAT16: d = D::BFLOAT16; break;
      default: throw std::runtime_error("PD_TensorShareExternalData: unknown data type");
    }
    t->shape.assign(shape, shape + n);
    t->staged.clear();
    t->staged_dt = -1;
    t->t->ShareExternalData(data, t->shape,
                            place == PD_PLACE_GPU ? paddle_infer::PlaceType::kGPU : paddle_infer::PlaceType::kCPU, d);
    return 0;
  }, 1);
}
PD_OneDimArrayInt32* PD_TensorGetShape(PD_Tensor* t) {
  const auto s = t->t->shape();
  auto* a = (PD_OneDimArrayInt32*)std::malloc(sizeof(PD_OneDimArrayInt32));
  a->size = s.size();
  a->data = (int32_t*)std::malloc(sizeof(int32_t) * (s.empty() ? 1 : s.size()));
  for (size_t i = 0; i < s.size(); ++i) a->data[i] = s[i];
  return a;
}
const char* PD_TensorGetName(PD_Tensor* t) { return t->name.c_str(); }
PD_DataType PD_TensorGetDataType(PD_Tensor* t) {
  switch (t->t->type()) {
    case paddle_infer::DataType::FLOAT32: return PD_DATA_FLOAT32;
    case paddle_infer::DataType::INT32: return PD_DATA_INT32;
    case paddle_infer::DataType::INT64: return PD_DATA_INT64;
    case paddle_infer::DataType::UINT8: return PD_DATA_UINT8;
    case paddle_infer::DataType::INT8: return PD_DATA_INT8;
    case paddle_infer::DataType::FLOAT16: return PD_DATA_FLOAT16;
    case paddle_infer::DataType::BOOL: return PD_DATA_BOOL;
    case paddle_infer::DataType::BFLOAT16: return PD_DATA_BFLOAT16;
    default: return PD_DATA_UNK;
  }
}

void PD_OneDimArrayInt32Destroy(PD_OneDimArrayInt32* a) {
  if (!a) return;
  std::free(a->data);
  std::free(a);
}
void PD_OneDimArrayCstrDestroy(PD_OneDimArrayCstr* a) {
  if (!a) return;
  for (size_t i = 0; i < a->size; ++i) std::free(a->data[i]);
  std::free(a->data);
  std::free(a);
}
void PD_OneDimArraySizeDestroy(PD_OneDimArraySize* a) {
  if (!a) return;
  std::free(a->data);
  std::free(a);
}
void PD_CstrDestroy(PD_Cstr* c) {
  if (!c) return;
  std::free(c->data);
  std::free(c);
}
PD_Cstr* PD_GetVersion() {
  auto* c = (PD_Cstr*)std::malloc(sizeof(PD_Cstr));
  const std::string v = paddle_infer::GetVersion();
  c->size = v.size() + 1;
  c->data = dup(v);
  return c;
}

}  // extern "C"
