// Which hipBLASLt epilogues have bf16 solutions on this GPU? Prints the heuristic count per
// (epilogue, transA/transB, aux dtype attr, bias dtype). Build: see tools/probe_blaslt.sh
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
int main() {
  hipblasLtHandle_t h; hipblasLtCreate(&h);
  const long M = 4096, N = 8192, K = 2048;
  void *A, *B, *D, *aux, *bias;
  hipMalloc(&A, 64 << 20); hipMalloc(&B, 64 << 20); hipMalloc(&D, 128 << 20);
  hipMalloc(&aux, 128 << 20); hipMalloc(&bias, 1 << 20);
  int epis[] = {1, 4, 32, 36, 160, 164, 192, 208, 256, 512};
  for (int e : epis)
    for (int tr = 0; tr < 4; ++tr)
      for (int auxdt = 0; auxdt < 2; ++auxdt)
        for (int bf = 0; bf < 2; ++bf) {
          int ta = tr & 1, tb = tr >> 1;
          hipblasLtMatmulDesc_t d; hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F);
          int32_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
          uint32_t ep = e;
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, 4);
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, 4);
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, 4);
          int32_t bt = bf ? HIP_R_32F : HIP_R_16BF;
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, 4);
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, 8);
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, 8);
          int64_t ld = N;
          hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, 8);
          if (auxdt) { int32_t at = HIP_R_16BF; hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, 4); }
          hipblasLtMatrixLayout_t la, lb, ld_;
          // D: N x M col-major
          hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ta ? K : N, ta ? N : K, ta ? K : N);
          hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, tb ? M : K, tb ? K : M, tb ? M : K);
          hipblasLtMatrixLayoutCreate(&ld_, HIP_R_16BF, N, M, N);
          hipblasLtMatmulPreference_t p; hipblasLtMatmulPreferenceCreate(&p);
          uint64_t ws = 32 << 20;
          hipblasLtMatmulPreferenceSetAttribute(p, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, 8);
          hipblasLtMatmulHeuristicResult_t r[8]; int got = 0;
          hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, ld_, ld_, p, 8, r, &got);
          float ms = -1;
          if (s == HIPBLAS_STATUS_SUCCESS && got > 0) {
            float al = 1, be = 0; hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            void* wsp; hipMalloc(&wsp, ws);
            for (int i = 0; i < 3; ++i) hipblasLtMatmul(h, d, &al, A, la, B, lb, &be, D, ld_, D, ld_, &r[0].algo, wsp, ws, 0);
            hipEventRecord(e0, 0);
            for (int i = 0; i < 10; ++i) hipblasLtMatmul(h, d, &al, A, la, B, lb, &be, D, ld_, D, ld_, &r[0].algo, wsp, ws, 0);
            hipEventRecord(e1, 0); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); ms /= 10;
            hipFree(wsp);
          }
          printf("epi=%3d ta=%d tb=%d auxdt=%d bias_f32=%d status=%d got=%d ms=%.3f\n", e, ta, tb, auxdt, bf, (int)s, got, ms);
          hipblasLtMatmulPreferenceDestroy(p); hipblasLtMatrixLayoutDestroy(la); hipblasLtMatrixLayoutDestroy(lb);
          hipblasLtMatrixLayoutDestroy(ld_); hipblasLtMatmulDescDestroy(d);
        }
  return 0;
}
