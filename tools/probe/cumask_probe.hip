// Does hipExtStreamCreateWithCUMask restrict a stream's kernels on this box?  A grid of 2048
// blocks, each spinning ~20 us of wall clock, on a full-chip stream vs streams masked to 128 / 32
// CUs (evenly spread and first-n).  Prints elapsed ms per launch.  Build:
//   hipcc --offload-arch=gfx950 -O2 tools/probe/cumask_probe.hip -o tools/probe/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

__global__ void spin(unsigned long long ticks, int* out) {
  const unsigned long long t0 = wall_clock64();
  for (int n = 0; n < 200000 && wall_clock64() - t0 < ticks; ++n) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

static float run(hipStream_t s, int* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, 2000ull, d);   // warm
  hipEventRecord(a, s);
  hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, 2000ull, d);   // 20 us at 100 MHz
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int* d;
  hipMalloc(&d, 4);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  printf("CUs %d\n", ncu);
  hipStream_t full;
  hipStreamCreate(&full);
  printf("full: %.3f ms\n", run(full, d));
  for (int n : {128, 32}) {
    for (int spread = 0; spread < 2; ++spread) {
      std::vector<uint32_t> m((ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu; ++i) {
        const bool pick = spread ? ((long)(i + 1) * n / ncu != (long)i * n / ncu) : i < n;
        if (pick) m[i / 32] |= 1u << (i % 32);
      }
      hipStream_t s;
      hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data());
      printf("mask %d CUs %s: create %s, %.3f ms\n", n, spread ? "spread" : "first", hipGetErrorString(e),
             e == hipSuccess ? run(s, d) : -1.f);
      if (e == hipSuccess) hipStreamDestroy(s);
    }
  }
  return 0;
}
