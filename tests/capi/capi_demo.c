/* Plain C client of the paddle_infer_amd C inference API (reference capi_exp usage pattern):
   config -> predictor -> input handle (reshape + copy) -> run -> output handle (shape + copy),
   then the zero-copy style MutableData path and a cloned predictor.
   usage: capi_demo <prog.pdmodel> <params.pdiparams> <batch> */
#include <stdio.h>
#include <stdlib.h>
#include "pd_inference_api.h"

static void run_once(PD_Predictor* pred, int batch, int in_dim, int mutable_path) {
  PD_OneDimArrayCstr* in_names = PD_PredictorGetInputNames(pred);
  PD_Tensor* in = PD_PredictorGetInputHandle(pred, in_names->data[0]);
  int32_t shape[2] = {batch, in_dim};
  PD_TensorReshape(in, 2, shape);
  if (mutable_path) {
    float* d = PD_TensorMutableDataFloat(in, PD_PLACE_CPU);
    for (int i = 0; i < batch * in_dim; ++i) d[i] = (float)((i * 7) % 13) / 13.0f - 0.5f;
  } else {
    float* x = (float*)malloc(sizeof(float) * batch * in_dim);
    for (int i = 0; i < batch * in_dim; ++i) x[i] = (float)((i * 7) % 13) / 13.0f - 0.5f;
    PD_TensorCopyFromCpuFloat(in, x);
    free(x);
  }
  if (!PD_PredictorRun(pred)) { fprintf(stderr, "run failed\n"); exit(2); }
  PD_OneDimArrayCstr* out_names = PD_PredictorGetOutputNames(pred);
  PD_Tensor* out = PD_PredictorGetOutputHandle(pred, out_names->data[0]);
  PD_OneDimArrayInt32* oshape = PD_TensorGetShape(out);
  int n = 1;
  for (size_t i = 0; i < oshape->size; ++i) n *= oshape->data[i];
  float* y = (float*)malloc(sizeof(float) * n);
  PD_TensorCopyToCpuFloat(out, y);
  printf("%s shape", mutable_path ? "mutable" : "copy");
  for (size_t i = 0; i < oshape->size; ++i) printf(" %d", oshape->data[i]);
  printf(" dtype %d values", (int)PD_TensorGetDataType(out));
  for (int i = 0; i < n; ++i) printf(" %.6f", y[i]);
  printf("\n");
  free(y);
  PD_OneDimArrayInt32Destroy(oshape);
  PD_TensorDestroy(out);
  PD_TensorDestroy(in);
  PD_OneDimArrayCstrDestroy(out_names);
  PD_OneDimArrayCstrDestroy(in_names);
}

int main(int argc, char** argv) {
  if (argc < 4) return 1;
  PD_Cstr* ver = PD_GetVersion();
  printf("version %s\n", ver->data);
  PD_CstrDestroy(ver);
  PD_Config* cfg = PD_ConfigCreate();
  PD_ConfigSetModel(cfg, argv[1], argv[2]);
  PD_ConfigDisableGpu(cfg);
  PD_ConfigSwitchIrOptim(cfg, TRUE);
  printf("use_gpu %d ir_optim %d trt %d prog %s\n", PD_ConfigUseGpu(cfg), PD_ConfigIrOptim(cfg),
         PD_ConfigTensorRtEngineEnabled(cfg), PD_ConfigGetProgFile(cfg));
  PD_Predictor* pred = PD_PredictorCreate(cfg); /* takes the config */
  if (!pred) return 3;
  printf("inputs %zu outputs %zu\n", PD_PredictorGetInputNum(pred), PD_PredictorGetOutputNum(pred));
  const int batch = atoi(argv[3]);
  run_once(pred, batch, 8, 0);
  run_once(pred, batch, 8, 1);
  PD_Predictor* clone = PD_PredictorClone(pred);
  run_once(clone, batch, 8, 0);
  PD_PredictorDestroy(clone);
  PD_PredictorDestroy(pred);
  return 0;
}
