// NaN/Inf checker (FLAGS_check_nan_inf). Parity: reference
// `paddle/fluid/framework/details/nan_inf_utils_detail.cu` (CheckNanInfKernel, which prints and
// aborts inside the op). MI355X design: the check never synchronises — every op output gets one
// grid-stride pass that records the SMALLEST offending op id into a device int with atomicMin;
// the host reads that single int once per step (utils.nan_inf.check()) and maps it back to the op
// name, so the debug mode costs one extra read of each tensor and no per-op host round trip.
#include "common.h"

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }

template <typename T>
__global__ __launch_bounds__(256) void nan_inf_kernel(const T* __restrict__ x, long long n,
                                                      int* __restrict__ flag, int op_id) {
  bool bad = false;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float v = to_f<T>(x[i]);
    bad |= !isfinite(v);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicMin(flag, op_id);
}

__global__ __launch_bounds__(256) void nan_inf_f16_kernel(const _Float16* __restrict__ x,
                                                          long long n, int* __restrict__ flag,
                                                          int op_id) {
  bool bad = false;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    bad |= !isfinite((float)x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicMin(flag, op_id);
}

// dtype: 0 f32, 1 bf16, 2 f16
PIAMD_EXPORT int piamd_nan_inf_check(int dtype, const void* x, long long n, int* flag, int op_id,
                                     hipStream_t st) {
  if (n <= 0) return 0;
  dim3 grid(stride_grid(n, 256)), block(256);
  if (dtype == 0)
    hipLaunchKernelGGL(nan_inf_kernel<float>, grid, block, 0, st, (const float*)x, n, flag, op_id);
  else if (dtype == 1)
    hipLaunchKernelGGL(nan_inf_kernel<bf16_t>, grid, block, 0, st, (const bf16_t*)x, n, flag, op_id);
  else if (dtype == 2)
    hipLaunchKernelGGL(nan_inf_f16_kernel, grid, block, 0, st, (const _Float16*)x, n, flag, op_id);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
