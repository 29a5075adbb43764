// C inference API of paddle_infer_amd (libpiamd_capi.so).
//
// Parity: the reference's experimental C API `paddle/fluid/inference/capi_exp/` (pd_config.h,
// pd_predictor.h, pd_tensor.h, pd_utils.h, pd_types.h, pd_common.h): same function names,
// argument lists, enum values and array structs, so a C program written against the reference's
// `pd_inference_api.h` compiles and runs against this library unchanged.
//
// Implementation: the library embeds the Python runtime of the framework (the predictor, IR
// passes and HIP kernels live there) — it initialises CPython on first use when the host is a
// plain C program, and takes the GIL around every call when it is loaded into a Python process.
// Backends that do not exist on MI355X (TensorRT, MKLDNN, XPU, NPU, Lite, ONNXRuntime) are
// accepted and reported as disabled; the HIP path runs instead.
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#define PADDLE_CAPI_EXPORT __attribute__((visibility("default")))
#ifndef __pd_give
#define __pd_give
#endif
#ifndef __pd_take
#define __pd_take
#endif
#ifndef __pd_keep
#define __pd_keep
#endif

typedef int8_t PD_Bool;
#ifndef TRUE
#define TRUE 1
#endif
#ifndef FALSE
#define FALSE 0
#endif

typedef int32_t PD_PrecisionType;
enum { PD_PRECISION_FLOAT32 = 0, PD_PRECISION_INT8, PD_PRECISION_HALF, PD_PRECISION_BFLOAT16 };
typedef int32_t PD_PlaceType;
enum { PD_PLACE_UNK = -1, PD_PLACE_CPU, PD_PLACE_GPU, PD_PLACE_XPU };
typedef int32_t PD_DataType;
enum { PD_DATA_UNK = -1, PD_DATA_FLOAT32, PD_DATA_INT32, PD_DATA_INT64, PD_DATA_UINT8, PD_DATA_INT8,
       PD_DATA_FLOAT16, PD_DATA_BOOL, PD_DATA_BFLOAT16 };

typedef struct PD_OneDimArrayInt32 { size_t size; int32_t* data; } PD_OneDimArrayInt32;
typedef struct PD_OneDimArraySize { size_t size; size_t* data; } PD_OneDimArraySize;
typedef struct PD_OneDimArrayCstr { size_t size; char** data; } PD_OneDimArrayCstr;
typedef struct PD_Cstr { size_t size; char* data; } PD_Cstr;
typedef struct PD_TwoDimArraySize { size_t size; PD_OneDimArraySize** data; } PD_TwoDimArraySize;

typedef struct PD_Config PD_Config;
typedef struct PD_Predictor PD_Predictor;
typedef struct PD_Tensor PD_Tensor;

#ifdef __cplusplus
extern "C" {
#endif

// ---- config ----------------------------------------------------------------------------------
PADDLE_CAPI_EXPORT __pd_give PD_Config* PD_ConfigCreate();
PADDLE_CAPI_EXPORT void PD_ConfigDestroy(__pd_take PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetModel(__pd_keep PD_Config* pd_config, const char* prog_file_path,
                                          const char* params_file_path);
PADDLE_CAPI_EXPORT void PD_ConfigSetProgFile(__pd_keep PD_Config* pd_config, const char* prog_file_path);
PADDLE_CAPI_EXPORT void PD_ConfigSetParamsFile(__pd_keep PD_Config* pd_config, const char* params_file_path);
PADDLE_CAPI_EXPORT void PD_ConfigSetOptimCacheDir(__pd_keep PD_Config* pd_config, const char* opt_cache_dir);
PADDLE_CAPI_EXPORT void PD_ConfigSetModelDir(__pd_keep PD_Config* pd_config, const char* model_dir);
PADDLE_CAPI_EXPORT const char* PD_ConfigGetModelDir(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT const char* PD_ConfigGetProgFile(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT const char* PD_ConfigGetParamsFile(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigDisableFCPadding(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigUseFcPadding(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableUseGpu(__pd_keep PD_Config* pd_config, uint64_t memory_pool_init_size_mb,
                                              int32_t device_id, PD_PrecisionType precision_mode);
PADDLE_CAPI_EXPORT void PD_ConfigDisableGpu(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigUseGpu(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableONNXRuntime(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigDisableONNXRuntime(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigONNXRuntimeEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableORTOptimization(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableXpu(__pd_keep PD_Config* pd_config, int32_t l3_workspace_size,
                                           PD_Bool locked, PD_Bool autotune, const char* autotune_file,
                                           const char* precision, PD_Bool adaptive_seqlen);
PADDLE_CAPI_EXPORT void PD_ConfigEnableNpu(__pd_keep PD_Config* pd_config, int32_t device_id);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigUseXpu(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigUseNpu(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT int32_t PD_ConfigGpuDeviceId(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT int32_t PD_ConfigXpuDeviceId(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT int32_t PD_ConfigNpuDeviceId(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT int32_t PD_ConfigMemoryPoolInitSizeMb(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT float PD_ConfigFractionOfGpuMemoryForPool(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableCudnn(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigCudnnEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSwitchIrOptim(__pd_keep PD_Config* pd_config, PD_Bool x);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigIrOptim(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableTensorRtEngine(__pd_keep PD_Config* pd_config, int64_t workspace_size,
                                                      int32_t max_batch_size, int32_t min_subgraph_size,
                                                      PD_PrecisionType precision, PD_Bool use_static,
                                                      PD_Bool use_calib_mode);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigTensorRtEngineEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetTrtDynamicShapeInfo(__pd_keep PD_Config* pd_config, size_t tensor_num,
                                                        const char** tensor_name, size_t* shapes_num,
                                                        int32_t** min_shape, int32_t** max_shape,
                                                        int32_t** optim_shape, PD_Bool disable_trt_plugin_fp16);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigTensorRtDynamicShapeEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableTunedTensorRtDynamicShape(__pd_keep PD_Config* pd_config,
                                                                 const char* shape_range_info_path,
                                                                 PD_Bool allow_build_at_runtime);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigTunedTensorRtDynamicShape(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigTrtAllowBuildAtRuntime(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigCollectShapeRangeInfo(__pd_keep PD_Config* pd_config,
                                                       const char* shape_range_info_path);
PADDLE_CAPI_EXPORT const char* PD_ConfigShapeRangeInfoPath(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigShapeRangeInfoCollected(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigDisableTensorRtOPs(__pd_keep PD_Config* pd_config, size_t ops_num,
                                                    const char** ops_name);
PADDLE_CAPI_EXPORT void PD_ConfigEnableVarseqlen(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigTensorRtOssEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableTensorRtDla(__pd_keep PD_Config* pd_config, int32_t dla_core);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigTensorRtDlaEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableLiteEngine(__pd_keep PD_Config* pd_config, PD_PrecisionType precision,
                                                  PD_Bool zero_copy, size_t passes_filter_num,
                                                  const char** passes_filter, size_t ops_filter_num,
                                                  const char** ops_filter);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigLiteEngineEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSwitchIrDebug(__pd_keep PD_Config* pd_config, PD_Bool x);
PADDLE_CAPI_EXPORT void PD_ConfigEnableMKLDNN(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetMkldnnCacheCapacity(__pd_keep PD_Config* pd_config, int32_t capacity);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigMkldnnEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetCpuMathLibraryNumThreads(__pd_keep PD_Config* pd_config,
                                                             int32_t cpu_math_library_num_threads);
PADDLE_CAPI_EXPORT int32_t PD_ConfigGetCpuMathLibraryNumThreads(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetMkldnnOp(__pd_keep PD_Config* pd_config, size_t ops_num, const char** op_list);
PADDLE_CAPI_EXPORT void PD_ConfigEnableMkldnnQuantizer(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigMkldnnQuantizerEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableMkldnnBfloat16(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigMkldnnBfloat16Enabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetBfloat16Op(__pd_keep PD_Config* pd_config, size_t ops_num, const char** op_list);
PADDLE_CAPI_EXPORT void PD_ConfigEnableGpuMultiStream(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigThreadLocalStreamEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetModelBuffer(__pd_keep PD_Config* pd_config, const char* prog_buffer,
                                                size_t prog_buffer_size, const char* params_buffer,
                                                size_t params_buffer_size);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigModelFromMemory(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableMemoryOptim(__pd_keep PD_Config* pd_config, PD_Bool x);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigMemoryOptimEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigEnableProfile(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigProfileEnabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigDisableGlogInfo(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigGlogInfoDisabled(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigSetInvalid(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT PD_Bool PD_ConfigIsValid(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigPartiallyRelease(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT void PD_ConfigDeletePass(__pd_keep PD_Config* pd_config, const char* pass);
PADDLE_CAPI_EXPORT void PD_ConfigInsertPass(__pd_keep PD_Config* pd_config, size_t idx, const char* pass);
PADDLE_CAPI_EXPORT void PD_ConfigAppendPass(__pd_keep PD_Config* pd_config, const char* pass);
PADDLE_CAPI_EXPORT __pd_give PD_OneDimArrayCstr* PD_ConfigAllPasses(__pd_keep PD_Config* pd_config);
PADDLE_CAPI_EXPORT __pd_give PD_Cstr* PD_ConfigSummary(__pd_keep PD_Config* pd_config);
// MI355X extension: replay each input-shape set as one hipGraph (Config.enable_hip_graph)
PADDLE_CAPI_EXPORT void PD_ConfigEnableHipGraph(__pd_keep PD_Config* pd_config, PD_Bool x);

// ---- predictor -------------------------------------------------------------------------------
PADDLE_CAPI_EXPORT __pd_give PD_Predictor* PD_PredictorCreate(__pd_take PD_Config* pd_config);
PADDLE_CAPI_EXPORT __pd_give PD_Predictor* PD_PredictorClone(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT __pd_give PD_OneDimArrayCstr* PD_PredictorGetInputNames(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT __pd_give PD_OneDimArrayCstr* PD_PredictorGetOutputNames(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT size_t PD_PredictorGetInputNum(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT size_t PD_PredictorGetOutputNum(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT __pd_give PD_Tensor* PD_PredictorGetInputHandle(__pd_keep PD_Predictor* pd_predictor,
                                                                   const char* name);
PADDLE_CAPI_EXPORT __pd_give PD_Tensor* PD_PredictorGetOutputHandle(__pd_keep PD_Predictor* pd_predictor,
                                                                    const char* name);
PADDLE_CAPI_EXPORT PD_Bool PD_PredictorRun(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT void PD_PredictorClearIntermediateTensor(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT uint64_t PD_PredictorTryShrinkMemory(__pd_keep PD_Predictor* pd_predictor);
PADDLE_CAPI_EXPORT void PD_PredictorDestroy(__pd_take PD_Predictor* pd_predictor);

// ---- tensor ----------------------------------------------------------------------------------
PADDLE_CAPI_EXPORT void PD_TensorDestroy(__pd_take PD_Tensor* pd_tensor);
PADDLE_CAPI_EXPORT void PD_TensorReshape(__pd_keep PD_Tensor* pd_tensor, size_t shape_size, int32_t* shape);
PADDLE_CAPI_EXPORT float* PD_TensorMutableDataFloat(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType place);
PADDLE_CAPI_EXPORT int64_t* PD_TensorMutableDataInt64(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType place);
PADDLE_CAPI_EXPORT int32_t* PD_TensorMutableDataInt32(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType place);
PADDLE_CAPI_EXPORT uint8_t* PD_TensorMutableDataUint8(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType place);
PADDLE_CAPI_EXPORT int8_t* PD_TensorMutableDataInt8(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType place);
PADDLE_CAPI_EXPORT float* PD_TensorDataFloat(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType* place, int32_t* size);
PADDLE_CAPI_EXPORT int64_t* PD_TensorDataInt64(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType* place, int32_t* size);
PADDLE_CAPI_EXPORT int32_t* PD_TensorDataInt32(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType* place, int32_t* size);
PADDLE_CAPI_EXPORT uint8_t* PD_TensorDataUint8(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType* place, int32_t* size);
PADDLE_CAPI_EXPORT int8_t* PD_TensorDataInt8(__pd_keep PD_Tensor* pd_tensor, PD_PlaceType* place, int32_t* size);
PADDLE_CAPI_EXPORT void PD_TensorCopyFromCpuFloat(__pd_keep PD_Tensor* pd_tensor, const float* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyFromCpuInt64(__pd_keep PD_Tensor* pd_tensor, const int64_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyFromCpuInt32(__pd_keep PD_Tensor* pd_tensor, const int32_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyFromCpuUint8(__pd_keep PD_Tensor* pd_tensor, const uint8_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyFromCpuInt8(__pd_keep PD_Tensor* pd_tensor, const int8_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyToCpuFloat(__pd_keep PD_Tensor* pd_tensor, float* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyToCpuInt64(__pd_keep PD_Tensor* pd_tensor, int64_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyToCpuInt32(__pd_keep PD_Tensor* pd_tensor, int32_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyToCpuUint8(__pd_keep PD_Tensor* pd_tensor, uint8_t* data);
PADDLE_CAPI_EXPORT void PD_TensorCopyToCpuInt8(__pd_keep PD_Tensor* pd_tensor, int8_t* data);
/* zero-copy input on the predictor's place (extension of the native engine): the predictor reads
   and in-place ops write `data` directly; the caller keeps it alive */
PADDLE_CAPI_EXPORT void PD_TensorShareExternalData(__pd_keep PD_Tensor* pd_tensor, void* data,
                                                   size_t shape_size, int32_t* shape,
                                                   PD_PlaceType place, PD_DataType data_type);
PADDLE_CAPI_EXPORT __pd_give PD_OneDimArrayInt32* PD_TensorGetShape(__pd_keep PD_Tensor* pd_tensor);
PADDLE_CAPI_EXPORT void PD_TensorSetLod(__pd_keep PD_Tensor* pd_tensor, __pd_keep PD_TwoDimArraySize* lod);
PADDLE_CAPI_EXPORT __pd_give PD_TwoDimArraySize* PD_TensorGetLod(__pd_keep PD_Tensor* pd_tensor);
PADDLE_CAPI_EXPORT const char* PD_TensorGetName(__pd_keep PD_Tensor* pd_tensor);
PADDLE_CAPI_EXPORT PD_DataType PD_TensorGetDataType(__pd_keep PD_Tensor* pd_tensor);

// ---- utils -----------------------------------------------------------------------------------
PADDLE_CAPI_EXPORT void PD_OneDimArrayInt32Destroy(__pd_take PD_OneDimArrayInt32* array);
PADDLE_CAPI_EXPORT void PD_OneDimArrayCstrDestroy(__pd_take PD_OneDimArrayCstr* array);
PADDLE_CAPI_EXPORT void PD_OneDimArraySizeDestroy(__pd_take PD_OneDimArraySize* array);
PADDLE_CAPI_EXPORT void PD_TwoDimArraySizeDestroy(__pd_take PD_TwoDimArraySize* array);
PADDLE_CAPI_EXPORT void PD_CstrDestroy(__pd_take PD_Cstr* cstr);
PADDLE_CAPI_EXPORT __pd_give PD_Cstr* PD_GetVersion();

#ifdef __cplusplus
}  // extern "C"
#endif
