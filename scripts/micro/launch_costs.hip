// Microbenchmark: fixed costs of short dependent kernels on MI355X (kernel-trace durations via rocprofv3).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

__global__ void k_empty(int64_t* p) {}
__global__ void k_read(const int64_t* __restrict__ c, int64_t* out) { if (threadIdx.x == 0 && *c == 12345) out[0] = 1; }
__global__ __launch_bounds__(64) void k_chain(const int64_t* __restrict__ a, int64_t* out, int n) {
  // n dependent global loads by one wave
  int64_t idx = threadIdx.x;
  for (int i = 0; i < n; ++i) idx = a[idx & 1023];
  if (idx == -7) out[0] = idx;
}
__global__ __launch_bounds__(64) void k_lds_chain(int64_t* out, int n) {
  __shared__ int64_t s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = (i * 7 + 1) & 1023;
  __syncthreads();
  int64_t idx = threadIdx.x;
  for (int i = 0; i < n; ++i) idx = s[idx & 1023];
  if (idx == -7) out[0] = idx;
}
__global__ __launch_bounds__(256) void k_blocks(const int64_t* __restrict__ c, int64_t* out) {
  __shared__ int h[256];
  h[threadIdx.x] = (int)*c;
  __syncthreads();
  for (int p = 0; p < 5; ++p) { atomicAdd(&h[(threadIdx.x * 7) & 255], 1); __syncthreads(); }
  if (h[threadIdx.x] == -1) out[0] = 1;
}

int main() {
  int64_t *a, *out;
  hipMalloc(&a, 1024 * 8); hipMalloc(&out, 64);
  int64_t h[1024]; for (int i = 0; i < 1024; ++i) h[i] = (i * 7 + 1) & 1023;
  hipMemcpy(a, h, sizeof(h), hipMemcpyHostToDevice);
  hipStream_t s; hipStreamCreate(&s);
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; ++i) {
      k_empty<<<1, 64, 0, s>>>(out);
      k_read<<<1, 64, 0, s>>>(a, out);
      k_chain<<<1, 64, 0, s>>>(a, out, 32);
      k_lds_chain<<<1, 64, 0, s>>>(out, 256);
      k_blocks<<<32, 256, 0, s>>>(a, out);
      k_empty<<<160, 256, 0, s>>>(out);
    }
    hipStreamSynchronize(s);
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("rep %d: %.2f us per 6-kernel group (wall)\n", rep, dt / 1000 * 1e6);
  }
  return 0;
}
