// C inference API (pd_inference_api.h) over the framework's Python predictor.
//
// Parity: reference `paddle/fluid/inference/capi_exp/pd_{config,predictor,tensor,utils}.cc`.
// Each PD_* handle owns a reference to the matching Python object (inference.Config /
// Predictor / Tensor); every entry point takes the GIL (PyGILState) so the library works both
// inside a Python process (ctypes) and from a plain C program, where the first call initialises
// an embedded interpreter whose sys.path starts at the repository that holds this library.
// Zero-copy style accessors (PD_TensorMutableData* / PD_TensorData*) use a host staging buffer
// per handle: staged inputs are copied in when the predictor runs.
#include "pd_inference_api.h"

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

struct PD_Config {
  PyObject* obj = nullptr;
  std::string s_model_dir, s_prog, s_params, s_shape_path;
  bool valid = true;
};
struct PD_Tensor {
  PyObject* obj = nullptr;
  PD_Predictor* owner = nullptr;
  std::string name;
  std::vector<char> stage;  // host staging buffer (MutableData / Data)
  int stage_dtype = -1;
  bool stage_pending = false;
};
struct PD_Predictor {
  PyObject* obj = nullptr;
  std::vector<PD_Tensor*> staged;  // inputs with pending host data
};

namespace {

std::once_flag g_init;
PyObject* g_bridge = nullptr;

std::string repo_root() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&repo_root), &info) && info.dli_fname) {
    std::string p = info.dli_fname;  // <root>/paddle_infer_amd/_lib/libpiamd_capi.so
    for (int i = 0; i < 3; ++i) {
      const size_t k = p.find_last_of('/');
      if (k == std::string::npos) return ".";
      p = p.substr(0, k);
    }
    return p.empty() ? "/" : p;
  }
  return ".";
}

void init_python() {
  if (!Py_IsInitialized()) {
    Py_InitializeEx(0);
    PyObject* sys_path = PySys_GetObject("path");  // borrowed
    PyObject* root = PyUnicode_FromString(repo_root().c_str());
    if (sys_path && root) PyList_Insert(sys_path, 0, root);
    Py_XDECREF(root);
    PyEval_SaveThread();  // release: every entry point takes the GIL itself
  }
}

struct Gil {
  PyGILState_STATE st;
  Gil() {
    std::call_once(g_init, init_python);
    st = PyGILState_Ensure();
  }
  ~Gil() { PyGILState_Release(st); }
};

PyObject* bridge() {
  if (!g_bridge) {
    g_bridge = PyImport_ImportModule("paddle_infer_amd.inference.capi_bridge");
    if (!g_bridge) PyErr_Print();
  }
  return g_bridge;
}

// report a Python error (reference: PADDLE_ENFORCE → message + abort; here: message, continue)
bool check(PyObject* r, const char* where) {
  if (r) return true;
  fprintf(stderr, "[paddle_infer_amd C API] %s failed:\n", where);
  PyErr_Print();
  return false;
}

// Steals `args` (a new reference, e.g. from Py_BuildValue, or null): released here after the
// call on every path, so no entry point leaks its argument tuple (and the handles it pins).
PyObject* call_bridge(const char* fn, PyObject* args) {
  PyObject* b = bridge();
  PyObject* f = b ? PyObject_GetAttrString(b, fn) : nullptr;
  PyObject* r = f ? PyObject_CallObject(f, args) : nullptr;
  Py_XDECREF(f);
  Py_XDECREF(args);
  return r;
}

template <typename... A>
PyObject* meth(PyObject* obj, const char* method, const char* fmt, A... a) {
  if (!obj) return nullptr;
  PyObject* r = fmt ? PyObject_CallMethod(obj, method, fmt, a...) : PyObject_CallMethod(obj, method, nullptr);
  check(r, method);
  return r;
}
template <typename... A>
void meth0(PyObject* obj, const char* method, const char* fmt, A... a) {
  Py_XDECREF(meth(obj, method, fmt, a...));
}
PD_Bool truth(PyObject* r) {
  const int t = r ? PyObject_IsTrue(r) : 0;
  Py_XDECREF(r);
  return t > 0 ? TRUE : FALSE;
}
long long as_ll(PyObject* r, long long dflt = 0) {
  long long v = dflt;
  if (r) {
    v = PyLong_AsLongLong(r);
    if (PyErr_Occurred()) { PyErr_Clear(); v = dflt; }
  }
  Py_XDECREF(r);
  return v;
}
std::string as_str(PyObject* r) {
  std::string s;
  if (r && r != Py_None) {
    PyObject* u = PyObject_Str(r);
    if (u) {
      const char* c = PyUnicode_AsUTF8(u);
      if (c) s = c;
      Py_DECREF(u);
    }
  }
  Py_XDECREF(r);
  return s;
}
PD_OneDimArrayCstr* to_cstr_array(PyObject* list) {
  auto* a = new PD_OneDimArrayCstr{0, nullptr};
  if (!list) return a;
  PyObject* seq = PySequence_Fast(list, "expected a sequence");
  Py_DECREF(list);
  if (!seq) { PyErr_Clear(); return a; }
  a->size = (size_t)PySequence_Fast_GET_SIZE(seq);
  a->data = new char*[a->size ? a->size : 1];
  for (size_t i = 0; i < a->size; ++i) {
    const char* c = PyUnicode_AsUTF8(PySequence_Fast_GET_ITEM(seq, (Py_ssize_t)i));
    const std::string s = c ? c : "";
    a->data[i] = new char[s.size() + 1];
    memcpy(a->data[i], s.c_str(), s.size() + 1);
  }
  Py_DECREF(seq);
  return a;
}
size_t dtype_size(int code) {
  switch (code) {
    case PD_DATA_FLOAT32: case PD_DATA_INT32: return 4;
    case PD_DATA_INT64: return 8;
    case PD_DATA_UINT8: case PD_DATA_INT8: return 1;
    default: return 0;
  }
}

long long numel(PD_Tensor* t) {
  PyObject* r = call_bridge("shape", Py_BuildValue("(O)", t->obj));
  long long n = 1;
  if (!check(r, "shape")) return 0;
  const Py_ssize_t k = PyList_Size(r);
  for (Py_ssize_t i = 0; i < k; ++i) n *= PyLong_AsLongLong(PyList_GetItem(r, i));
  Py_DECREF(r);
  return n;
}

void copy_from(PD_Tensor* t, const void* data, int code) {
  const long long n = numel(t);
  PyObject* buf = PyBytes_FromStringAndSize((const char*)data, (Py_ssize_t)(n * (long long)dtype_size(code)));
  PyObject* args = Py_BuildValue("(ONi)", t->obj, buf, code);
  PyObject* r = call_bridge("copy_from", args);
  check(r, "PD_TensorCopyFromCpu");
  Py_XDECREF(r);
}

void copy_to(PD_Tensor* t, void* data, int code) {
  PyObject* args = Py_BuildValue("(Oi)", t->obj, code);
  PyObject* r = call_bridge("copy_to", args);
  if (!check(r, "PD_TensorCopyToCpu")) return;
  char* p = nullptr;
  Py_ssize_t len = 0;
  if (PyBytes_AsStringAndSize(r, &p, &len) == 0 && data) memcpy(data, p, (size_t)len);
  Py_DECREF(r);
}

template <typename T>
T* mutable_data(PD_Tensor* t, int code) {
  if (!t) return nullptr;
  Gil g;
  const long long n = numel(t);
  t->stage.assign((size_t)(n * (long long)dtype_size(code)), 0);
  t->stage_dtype = code;
  if (!t->stage_pending && t->owner) t->owner->staged.push_back(t);
  t->stage_pending = true;
  return reinterpret_cast<T*>(t->stage.data());
}

template <typename T>
T* data_of(PD_Tensor* t, int code, PD_PlaceType* place, int32_t* size) {
  if (!t) return nullptr;
  Gil g;
  const long long n = numel(t);
  t->stage.assign((size_t)(n * (long long)dtype_size(code)), 0);
  copy_to(t, t->stage.data(), code);
  if (place) *place = PD_PLACE_CPU;
  if (size) *size = (int32_t)n;
  return reinterpret_cast<T*>(t->stage.data());
}

PD_Tensor* new_tensor(PD_Predictor* p, const char* name, bool input) {
  PyObject* h = meth(p->obj, input ? "get_input_handle" : "get_output_handle", "s", name);
  if (!h) return nullptr;
  auto* t = new PD_Tensor;
  t->obj = h;
  t->owner = p;
  t->name = name;
  return t;
}

}  // namespace

// ============================================================================================ config
PD_Config* PD_ConfigCreate() {
  Gil g;
  PyObject* c = call_bridge("new_config", nullptr);
  if (!check(c, "PD_ConfigCreate")) return nullptr;
  auto* cfg = new PD_Config;
  cfg->obj = c;
  return cfg;
}
void PD_ConfigDestroy(PD_Config* c) {
  if (!c) return;
  Gil g;
  Py_XDECREF(c->obj);
  delete c;
}
void PD_ConfigSetModel(PD_Config* c, const char* prog, const char* params) { Gil g; meth0(c->obj, "set_model", "ss", prog, params); }
void PD_ConfigSetProgFile(PD_Config* c, const char* f) { Gil g; meth0(c->obj, "set_prog_file", "s", f); }
void PD_ConfigSetParamsFile(PD_Config* c, const char* f) { Gil g; meth0(c->obj, "set_params_file", "s", f); }
void PD_ConfigSetOptimCacheDir(PD_Config* c, const char* d) { (void)c; (void)d; }
void PD_ConfigSetModelDir(PD_Config* c, const char* d) { Gil g; meth0(c->obj, "set_model", "s", d); }
const char* PD_ConfigGetModelDir(PD_Config* c) { Gil g; c->s_model_dir = as_str(meth(c->obj, "model_dir", nullptr)); return c->s_model_dir.c_str(); }
const char* PD_ConfigGetProgFile(PD_Config* c) { Gil g; c->s_prog = as_str(meth(c->obj, "prog_file", nullptr)); return c->s_prog.c_str(); }
const char* PD_ConfigGetParamsFile(PD_Config* c) { Gil g; c->s_params = as_str(meth(c->obj, "params_file", nullptr)); return c->s_params.c_str(); }
void PD_ConfigDisableFCPadding(PD_Config* c) { (void)c; }
PD_Bool PD_ConfigUseFcPadding(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigEnableUseGpu(PD_Config* c, uint64_t pool_mb, int32_t dev, PD_PrecisionType prec) {
  Gil g;
  PyObject* r = call_bridge("enable_use_gpu", Py_BuildValue("(OKii)", c->obj, (unsigned long long)pool_mb, dev, prec));
  check(r, "PD_ConfigEnableUseGpu");
  Py_XDECREF(r);
}
void PD_ConfigDisableGpu(PD_Config* c) { Gil g; meth0(c->obj, "disable_gpu", nullptr); }
PD_Bool PD_ConfigUseGpu(PD_Config* c) { Gil g; return truth(meth(c->obj, "use_gpu", nullptr)); }
void PD_ConfigEnableONNXRuntime(PD_Config* c) { Gil g; meth0(c->obj, "enable_onnxruntime", nullptr); }
void PD_ConfigDisableONNXRuntime(PD_Config* c) { (void)c; }
PD_Bool PD_ConfigONNXRuntimeEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigEnableORTOptimization(PD_Config* c) { (void)c; }
void PD_ConfigEnableXpu(PD_Config* c, int32_t, PD_Bool, PD_Bool, const char*, const char*, PD_Bool) { Gil g; meth0(c->obj, "enable_xpu", nullptr); }
void PD_ConfigEnableNpu(PD_Config* c, int32_t) { Gil g; meth0(c->obj, "enable_npu", nullptr); }
PD_Bool PD_ConfigUseXpu(PD_Config* c) { (void)c; return FALSE; }
PD_Bool PD_ConfigUseNpu(PD_Config* c) { (void)c; return FALSE; }
int32_t PD_ConfigGpuDeviceId(PD_Config* c) { Gil g; return (int32_t)as_ll(meth(c->obj, "gpu_device_id", nullptr)); }
int32_t PD_ConfigXpuDeviceId(PD_Config* c) { (void)c; return 0; }
int32_t PD_ConfigNpuDeviceId(PD_Config* c) { (void)c; return 0; }
int32_t PD_ConfigMemoryPoolInitSizeMb(PD_Config* c) { Gil g; return (int32_t)as_ll(meth(c->obj, "memory_pool_init_size_mb", nullptr)); }
float PD_ConfigFractionOfGpuMemoryForPool(PD_Config* c) {
  Gil g;
  PyObject* r = meth(c->obj, "fraction_of_gpu_memory_for_pool", nullptr);
  const double v = r ? PyFloat_AsDouble(r) : 0.0;
  if (PyErr_Occurred()) PyErr_Clear();
  Py_XDECREF(r);
  return (float)v;
}
void PD_ConfigEnableCudnn(PD_Config* c) { (void)c; }  // MIOpen / own kernels are always used
PD_Bool PD_ConfigCudnnEnabled(PD_Config* c) { Gil g; return truth(meth(c->obj, "use_gpu", nullptr)); }
void PD_ConfigSwitchIrOptim(PD_Config* c, PD_Bool x) { Gil g; meth0(c->obj, "switch_ir_optim", "i", (int)x); }
PD_Bool PD_ConfigIrOptim(PD_Config* c) { Gil g; return truth(meth(c->obj, "ir_optim", nullptr)); }
void PD_ConfigEnableTensorRtEngine(PD_Config* c, int64_t, int32_t, int32_t, PD_PrecisionType, PD_Bool, PD_Bool) { Gil g; meth0(c->obj, "enable_tensorrt_engine", nullptr); }
PD_Bool PD_ConfigTensorRtEngineEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigSetTrtDynamicShapeInfo(PD_Config* c, size_t, const char**, size_t*, int32_t**, int32_t**, int32_t**, PD_Bool) { (void)c; }
PD_Bool PD_ConfigTensorRtDynamicShapeEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigEnableTunedTensorRtDynamicShape(PD_Config* c, const char*, PD_Bool) { (void)c; }
PD_Bool PD_ConfigTunedTensorRtDynamicShape(PD_Config* c) { (void)c; return FALSE; }
PD_Bool PD_ConfigTrtAllowBuildAtRuntime(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigCollectShapeRangeInfo(PD_Config* c, const char* p) { c->s_shape_path = p ? p : ""; }
const char* PD_ConfigShapeRangeInfoPath(PD_Config* c) { return c->s_shape_path.c_str(); }
PD_Bool PD_ConfigShapeRangeInfoCollected(PD_Config* c) { return c->s_shape_path.empty() ? FALSE : TRUE; }
void PD_ConfigDisableTensorRtOPs(PD_Config* c, size_t, const char**) { (void)c; }
void PD_ConfigEnableVarseqlen(PD_Config* c) { (void)c; }
PD_Bool PD_ConfigTensorRtOssEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigEnableTensorRtDla(PD_Config* c, int32_t) { (void)c; }
PD_Bool PD_ConfigTensorRtDlaEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigEnableLiteEngine(PD_Config* c, PD_PrecisionType, PD_Bool, size_t, const char**, size_t, const char**) { Gil g; meth0(c->obj, "enable_lite_engine", nullptr); }
PD_Bool PD_ConfigLiteEngineEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigSwitchIrDebug(PD_Config* c, PD_Bool x) { Gil g; meth0(c->obj, "switch_ir_debug", "i", (int)x); }
void PD_ConfigEnableMKLDNN(PD_Config* c) { Gil g; meth0(c->obj, "enable_mkldnn", nullptr); }
void PD_ConfigSetMkldnnCacheCapacity(PD_Config* c, int32_t) { (void)c; }
PD_Bool PD_ConfigMkldnnEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigSetCpuMathLibraryNumThreads(PD_Config* c, int32_t n) { Gil g; meth0(c->obj, "set_cpu_math_library_num_threads", "i", n); }
int32_t PD_ConfigGetCpuMathLibraryNumThreads(PD_Config* c) { Gil g; return (int32_t)as_ll(meth(c->obj, "cpu_math_library_num_threads", nullptr)); }
void PD_ConfigSetMkldnnOp(PD_Config* c, size_t, const char**) { (void)c; }
void PD_ConfigEnableMkldnnQuantizer(PD_Config* c) { (void)c; }
PD_Bool PD_ConfigMkldnnQuantizerEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigEnableMkldnnBfloat16(PD_Config* c) { Gil g; meth0(c->obj, "enable_mkldnn_bfloat16", nullptr); }
PD_Bool PD_ConfigMkldnnBfloat16Enabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigSetBfloat16Op(PD_Config* c, size_t, const char**) { (void)c; }
void PD_ConfigEnableGpuMultiStream(PD_Config* c) { (void)c; }
PD_Bool PD_ConfigThreadLocalStreamEnabled(PD_Config* c) { (void)c; return FALSE; }
void PD_ConfigSetModelBuffer(PD_Config* c, const char* prog, size_t prog_size, const char* params, size_t params_size) {
  Gil g;
  PyObject* pb = PyBytes_FromStringAndSize(prog, (Py_ssize_t)prog_size);
  PyObject* qb = PyBytes_FromStringAndSize(params, (Py_ssize_t)params_size);
  PyObject* r = PyObject_CallMethod(c->obj, "set_model_buffer", "OnOn", pb, (Py_ssize_t)prog_size, qb, (Py_ssize_t)params_size);
  check(r, "PD_ConfigSetModelBuffer");
  Py_XDECREF(r);
  Py_XDECREF(pb);
  Py_XDECREF(qb);
}
PD_Bool PD_ConfigModelFromMemory(PD_Config* c) { Gil g; return truth(meth(c->obj, "model_from_memory", nullptr)); }
void PD_ConfigEnableMemoryOptim(PD_Config* c, PD_Bool x) { Gil g; meth0(c->obj, "enable_memory_optim", "i", (int)x); }
PD_Bool PD_ConfigMemoryOptimEnabled(PD_Config* c) { Gil g; return truth(meth(c->obj, "enable_memory_optimize", nullptr)); }
void PD_ConfigEnableProfile(PD_Config* c) { Gil g; meth0(c->obj, "enable_profile", nullptr); }
PD_Bool PD_ConfigProfileEnabled(PD_Config* c) {
  Gil g;
  PyObject* r = PyObject_GetAttrString(c->obj, "_profile");
  if (!r) PyErr_Clear();
  return truth(r);
}
void PD_ConfigDisableGlogInfo(PD_Config* c) { Gil g; meth0(c->obj, "disable_glog_info", nullptr); }
PD_Bool PD_ConfigGlogInfoDisabled(PD_Config* c) { Gil g; return truth(meth(c->obj, "glog_info_disabled", nullptr)); }
void PD_ConfigSetInvalid(PD_Config* c) { c->valid = false; }
PD_Bool PD_ConfigIsValid(PD_Config* c) { return c && c->valid ? TRUE : FALSE; }
void PD_ConfigPartiallyRelease(PD_Config* c) { (void)c; }
void PD_ConfigDeletePass(PD_Config* c, const char* pass) { Gil g; meth0(c->obj, "delete_pass", "s", pass); }
void PD_ConfigInsertPass(PD_Config* c, size_t idx, const char* pass) {
  Gil g;
  PyObject* pb = meth(c->obj, "pass_builder", nullptr);
  meth0(pb, "insert_pass", "ns", (Py_ssize_t)idx, pass);
  Py_XDECREF(pb);
}
void PD_ConfigAppendPass(PD_Config* c, const char* pass) {
  Gil g;
  PyObject* pb = meth(c->obj, "pass_builder", nullptr);
  meth0(pb, "append_pass", "s", pass);
  Py_XDECREF(pb);
}
PD_OneDimArrayCstr* PD_ConfigAllPasses(PD_Config* c) {
  Gil g;
  return to_cstr_array(call_bridge("all_passes", Py_BuildValue("(O)", c->obj)));
}
PD_Cstr* PD_ConfigSummary(PD_Config* c) {
  Gil g;
  const std::string s = as_str(call_bridge("summary", Py_BuildValue("(O)", c->obj)));
  auto* r = new PD_Cstr{s.size() + 1, new char[s.size() + 1]};
  memcpy(r->data, s.c_str(), s.size() + 1);
  return r;
}
void PD_ConfigEnableHipGraph(PD_Config* c, PD_Bool x) { Gil g; meth0(c->obj, "enable_hip_graph", "i", (int)x); }

// ========================================================================================= predictor
PD_Predictor* PD_PredictorCreate(PD_Config* c) {
  if (!c) return nullptr;
  PD_Predictor* p = nullptr;
  {
    Gil g;
    PyObject* r = call_bridge("new_predictor", Py_BuildValue("(O)", c->obj));
    if (check(r, "PD_PredictorCreate")) {
      p = new PD_Predictor;
      p->obj = r;
    }
  }
  PD_ConfigDestroy(c);  // __pd_take: the predictor consumes the config (reference semantics)
  return p;
}
PD_Predictor* PD_PredictorClone(PD_Predictor* p) {
  Gil g;
  PyObject* r = meth(p->obj, "clone", nullptr);
  if (!r) return nullptr;
  auto* q = new PD_Predictor;
  q->obj = r;
  return q;
}
PD_OneDimArrayCstr* PD_PredictorGetInputNames(PD_Predictor* p) { Gil g; return to_cstr_array(meth(p->obj, "get_input_names", nullptr)); }
PD_OneDimArrayCstr* PD_PredictorGetOutputNames(PD_Predictor* p) { Gil g; return to_cstr_array(meth(p->obj, "get_output_names", nullptr)); }
size_t PD_PredictorGetInputNum(PD_Predictor* p) {
  Gil g;
  PyObject* r = meth(p->obj, "get_input_names", nullptr);
  const Py_ssize_t n = r ? PySequence_Size(r) : 0;
  Py_XDECREF(r);
  return n > 0 ? (size_t)n : 0;
}
size_t PD_PredictorGetOutputNum(PD_Predictor* p) {
  Gil g;
  PyObject* r = meth(p->obj, "get_output_names", nullptr);
  const Py_ssize_t n = r ? PySequence_Size(r) : 0;
  Py_XDECREF(r);
  return n > 0 ? (size_t)n : 0;
}
PD_Tensor* PD_PredictorGetInputHandle(PD_Predictor* p, const char* name) { Gil g; return new_tensor(p, name, true); }
PD_Tensor* PD_PredictorGetOutputHandle(PD_Predictor* p, const char* name) { Gil g; return new_tensor(p, name, false); }
PD_Bool PD_PredictorRun(PD_Predictor* p) {
  if (!p) return FALSE;
  Gil g;
  for (PD_Tensor* t : p->staged) {  // inputs written through PD_TensorMutableData*
    if (t->stage_pending) copy_from(t, t->stage.data(), t->stage_dtype);
    t->stage_pending = false;
  }
  p->staged.clear();
  PyObject* r = meth(p->obj, "run", nullptr);
  const bool ok = r != nullptr;
  Py_XDECREF(r);
  return ok ? TRUE : FALSE;
}
void PD_PredictorClearIntermediateTensor(PD_Predictor* p) { Gil g; meth0(p->obj, "clear_intermediate_tensor", nullptr); }
uint64_t PD_PredictorTryShrinkMemory(PD_Predictor* p) { Gil g; return (uint64_t)as_ll(meth(p->obj, "try_shrink_memory", nullptr)); }
void PD_PredictorDestroy(PD_Predictor* p) {
  if (!p) return;
  Gil g;
  Py_XDECREF(p->obj);
  delete p;
}

// ============================================================================================ tensor
void PD_TensorDestroy(PD_Tensor* t) {
  if (!t) return;
  Gil g;
  if (t->owner && t->stage_pending) {
    auto& v = t->owner->staged;
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i] == t) { v.erase(v.begin() + (long)i); break; }
  }
  Py_XDECREF(t->obj);
  delete t;
}
void PD_TensorReshape(PD_Tensor* t, size_t n, int32_t* shape) {
  Gil g;
  PyObject* l = PyList_New((Py_ssize_t)n);
  for (size_t i = 0; i < n; ++i) PyList_SET_ITEM(l, (Py_ssize_t)i, PyLong_FromLong(shape[i]));
  PyObject* r = PyObject_CallMethod(t->obj, "reshape", "O", l);
  check(r, "PD_TensorReshape");
  Py_XDECREF(r);
  Py_DECREF(l);
}
float* PD_TensorMutableDataFloat(PD_Tensor* t, PD_PlaceType) { return mutable_data<float>(t, PD_DATA_FLOAT32); }
int64_t* PD_TensorMutableDataInt64(PD_Tensor* t, PD_PlaceType) { return mutable_data<int64_t>(t, PD_DATA_INT64); }
int32_t* PD_TensorMutableDataInt32(PD_Tensor* t, PD_PlaceType) { return mutable_data<int32_t>(t, PD_DATA_INT32); }
uint8_t* PD_TensorMutableDataUint8(PD_Tensor* t, PD_PlaceType) { return mutable_data<uint8_t>(t, PD_DATA_UINT8); }
int8_t* PD_TensorMutableDataInt8(PD_Tensor* t, PD_PlaceType) { return mutable_data<int8_t>(t, PD_DATA_INT8); }
float* PD_TensorDataFloat(PD_Tensor* t, PD_PlaceType* pl, int32_t* n) { return data_of<float>(t, PD_DATA_FLOAT32, pl, n); }
int64_t* PD_TensorDataInt64(PD_Tensor* t, PD_PlaceType* pl, int32_t* n) { return data_of<int64_t>(t, PD_DATA_INT64, pl, n); }
int32_t* PD_TensorDataInt32(PD_Tensor* t, PD_PlaceType* pl, int32_t* n) { return data_of<int32_t>(t, PD_DATA_INT32, pl, n); }
uint8_t* PD_TensorDataUint8(PD_Tensor* t, PD_PlaceType* pl, int32_t* n) { return data_of<uint8_t>(t, PD_DATA_UINT8, pl, n); }
int8_t* PD_TensorDataInt8(PD_Tensor* t, PD_PlaceType* pl, int32_t* n) { return data_of<int8_t>(t, PD_DATA_INT8, pl, n); }
void PD_TensorCopyFromCpuFloat(PD_Tensor* t, const float* d) { Gil g; copy_from(t, d, PD_DATA_FLOAT32); }
void PD_TensorCopyFromCpuInt64(PD_Tensor* t, const int64_t* d) { Gil g; copy_from(t, d, PD_DATA_INT64); }
void PD_TensorCopyFromCpuInt32(PD_Tensor* t, const int32_t* d) { Gil g; copy_from(t, d, PD_DATA_INT32); }
void PD_TensorCopyFromCpuUint8(PD_Tensor* t, const uint8_t* d) { Gil g; copy_from(t, d, PD_DATA_UINT8); }
void PD_TensorCopyFromCpuInt8(PD_Tensor* t, const int8_t* d) { Gil g; copy_from(t, d, PD_DATA_INT8); }
void PD_TensorCopyToCpuFloat(PD_Tensor* t, float* d) { Gil g; copy_to(t, d, PD_DATA_FLOAT32); }
void PD_TensorCopyToCpuInt64(PD_Tensor* t, int64_t* d) { Gil g; copy_to(t, d, PD_DATA_INT64); }
void PD_TensorCopyToCpuInt32(PD_Tensor* t, int32_t* d) { Gil g; copy_to(t, d, PD_DATA_INT32); }
void PD_TensorCopyToCpuUint8(PD_Tensor* t, uint8_t* d) { Gil g; copy_to(t, d, PD_DATA_UINT8); }
void PD_TensorCopyToCpuInt8(PD_Tensor* t, int8_t* d) { Gil g; copy_to(t, d, PD_DATA_INT8); }
PD_OneDimArrayInt32* PD_TensorGetShape(PD_Tensor* t) {
  Gil g;
  auto* a = new PD_OneDimArrayInt32{0, nullptr};
  PyObject* r = call_bridge("shape", Py_BuildValue("(O)", t->obj));
  if (!check(r, "PD_TensorGetShape")) return a;
  a->size = (size_t)PyList_Size(r);
  a->data = new int32_t[a->size ? a->size : 1];
  for (size_t i = 0; i < a->size; ++i) a->data[i] = (int32_t)PyLong_AsLong(PyList_GetItem(r, (Py_ssize_t)i));
  Py_DECREF(r);
  return a;
}
void PD_TensorSetLod(PD_Tensor* t, PD_TwoDimArraySize* lod) {
  Gil g;
  PyObject* l = PyList_New(lod ? (Py_ssize_t)lod->size : 0);
  for (size_t i = 0; lod && i < lod->size; ++i) {
    PyObject* inner = PyList_New((Py_ssize_t)lod->data[i]->size);
    for (size_t j = 0; j < lod->data[i]->size; ++j)
      PyList_SET_ITEM(inner, (Py_ssize_t)j, PyLong_FromSize_t(lod->data[i]->data[j]));
    PyList_SET_ITEM(l, (Py_ssize_t)i, inner);
  }
  PyObject* r = call_bridge("set_lod", Py_BuildValue("(ON)", t->obj, l));
  check(r, "PD_TensorSetLod");
  Py_XDECREF(r);
}
PD_TwoDimArraySize* PD_TensorGetLod(PD_Tensor* t) {
  Gil g;
  auto* a = new PD_TwoDimArraySize{0, nullptr};
  PyObject* r = call_bridge("get_lod", Py_BuildValue("(O)", t->obj));
  if (!check(r, "PD_TensorGetLod")) return a;
  a->size = (size_t)PyList_Size(r);
  a->data = new PD_OneDimArraySize*[a->size ? a->size : 1];
  for (size_t i = 0; i < a->size; ++i) {
    PyObject* inner = PyList_GetItem(r, (Py_ssize_t)i);
    auto* x = new PD_OneDimArraySize{(size_t)PyList_Size(inner), nullptr};
    x->data = new size_t[x->size ? x->size : 1];
    for (size_t j = 0; j < x->size; ++j) x->data[j] = PyLong_AsSize_t(PyList_GetItem(inner, (Py_ssize_t)j));
    a->data[i] = x;
  }
  Py_DECREF(r);
  return a;
}
const char* PD_TensorGetName(PD_Tensor* t) { return t ? t->name.c_str() : ""; }
PD_DataType PD_TensorGetDataType(PD_Tensor* t) {
  Gil g;
  return (PD_DataType)as_ll(call_bridge("dtype", Py_BuildValue("(O)", t->obj)), PD_DATA_UNK);
}

// ============================================================================================= utils
void PD_OneDimArrayInt32Destroy(PD_OneDimArrayInt32* a) {
  if (!a) return;
  delete[] a->data;
  delete a;
}
void PD_OneDimArrayCstrDestroy(PD_OneDimArrayCstr* a) {
  if (!a) return;
  for (size_t i = 0; i < a->size; ++i) delete[] a->data[i];
  delete[] a->data;
  delete a;
}
void PD_OneDimArraySizeDestroy(PD_OneDimArraySize* a) {
  if (!a) return;
  delete[] a->data;
  delete a;
}
void PD_TwoDimArraySizeDestroy(PD_TwoDimArraySize* a) {
  if (!a) return;
  for (size_t i = 0; i < a->size; ++i) PD_OneDimArraySizeDestroy(a->data[i]);
  delete[] a->data;
  delete a;
}
void PD_CstrDestroy(PD_Cstr* c) {
  if (!c) return;
  delete[] c->data;
  delete c;
}
PD_Cstr* PD_GetVersion() {
  Gil g;
  const std::string s = as_str(call_bridge("version", nullptr));
  auto* r = new PD_Cstr{s.size() + 1, new char[s.size() + 1]};
  memcpy(r->data, s.c_str(), s.size() + 1);
  return r;
}
