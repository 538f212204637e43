// Microbenchmark (r5): what it costs to start a dependent wide kernel after a one-wave producer on MI355X.
// Gap = consumer's first s_memrealtime − producer's last s_memrealtime (100 MHz clock, 10 ns), p50 over reps.
//   (a) same stream: producer → consumer (kernel boundary)
//   (b) cross stream: producer; hipEventRecord; hipStreamWaitEvent; consumer
//   (c) hipStreamWaitValue64 on signal memory written by the producer (system-scope release store)
//   (d) consumer already resident (one wave polling a device word), producer stores it (agent-scope release)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(64) void producer(uint64_t* stamps, int rep, uint64_t* sig, uint64_t* dev_word, int64_t spin_ticks,
                                               int mode) {
  const uint64_t t0 = rt();
  while (rt() - t0 < (uint64_t)spin_ticks) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t t1 = rt();
  if (threadIdx.x == 0) {
    stamps[2 * rep] = t1;
    if (mode == 2) __hip_atomic_store(sig, (uint64_t)(rep + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (mode == 3) __hip_atomic_store(dev_word, (uint64_t)(rep + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(512) void consumer(uint64_t* stamps, int rep) {
  const uint64_t t = rt();
  if (blockIdx.x == 0 && threadIdx.x == 0) stamps[2 * rep + 1] = t;
}

__global__ __launch_bounds__(64) void poller(uint64_t* stamps, int reps, const uint64_t* dev_word) {
  for (int rep = 0; rep < reps; ++rep) {
    int64_t it = 0;
    while (__hip_atomic_load(dev_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint64_t)(rep + 1)) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > (1 << 26)) return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint64_t t = rt();
    if (threadIdx.x == 0) stamps[2 * rep + 1] = t;
  }
}

int main() {
  const int reps = 200, blocks = 392;
  uint64_t *stamps, *sig, *dev_word;
  hipMalloc(&stamps, 2 * reps * 8);
  hipMalloc(&dev_word, 8);
  if (hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory) != hipSuccess) {
    printf("signal memory: unavailable\n");
    sig = nullptr;
  }
  int can = 0;
  hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("CanUseStreamWaitValue=%d\n", can);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const int64_t spin = 2000;  // 20 us of producer work
  std::vector<uint64_t> h(2 * reps);
  const char* names[] = {"same-stream boundary", "cross-stream event", "hipStreamWaitValue64", "resident poller"};
  for (int mode = 0; mode < 4; ++mode) {
    if (mode == 2 && (!sig || !can)) continue;
    hipMemset(stamps, 0, 2 * reps * 8);
    hipMemset(dev_word, 0, 8);
    if (sig) hipMemset(sig, 0, 8);
    hipDeviceSynchronize();
    if (mode == 3) poller<<<1, 64, 0, s2>>>(stamps, reps, dev_word);
    for (int rep = 0; rep < reps; ++rep) {
      if (mode == 0) {
        producer<<<1, 64, 0, s1>>>(stamps, rep, sig, dev_word, spin, mode);
        consumer<<<blocks, 512, 0, s1>>>(stamps, rep);
      } else if (mode == 1) {
        producer<<<1, 64, 0, s1>>>(stamps, rep, sig, dev_word, spin, mode);
        hipEventRecord(ev, s1);
        hipStreamWaitEvent(s2, ev, 0);
        consumer<<<blocks, 512, 0, s2>>>(stamps, rep);
      } else if (mode == 2) {
        hipStreamWaitValue64(s2, sig, (uint64_t)(rep + 1), hipStreamWaitValueGte);
        consumer<<<blocks, 512, 0, s2>>>(stamps, rep);
        producer<<<1, 64, 0, s1>>>(stamps, rep, sig, dev_word, spin, mode);
      } else {
        producer<<<1, 64, 0, s1>>>(stamps, rep, sig, dev_word, spin, mode);
      }
      hipStreamSynchronize(s1);
      hipStreamSynchronize(s2);
    }
    hipDeviceSynchronize();
    hipMemcpy(h.data(), stamps, 2 * reps * 8, hipMemcpyDeviceToHost);
    std::vector<double> g;
    for (int rep = 5; rep < reps; ++rep) g.push_back(((double)h[2 * rep + 1] - (double)h[2 * rep]) * 0.01);
    std::sort(g.begin(), g.end());
    printf("%-24s gap p10 %6.2f  p50 %6.2f  p90 %6.2f us\n", names[mode], g[g.size() / 10], g[g.size() / 2],
           g[g.size() * 9 / 10]);
  }
  return 0;
}
