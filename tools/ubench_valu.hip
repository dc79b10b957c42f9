// VALU issue-rate calibration (not part of the library): kernels of 8 independent chains per lane,
// one wave per SIMD, timed with events.  hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2v __attribute__((ext_vector_type(2)));
#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

template <int K>
__global__ __launch_bounds__(64) void k_op(float* out, int n) {
  float a[8]; f2v p[8]; double d[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x + i; p[i] = f2v{a[i], a[i] + 1}; d[i] = a[i]; }
  const float b = 1.0000001f, c = 0.5f;
  const f2v pb{b, b}, pc{c, c};
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (K == 0) a[i] = __builtin_fmaf(a[i], b, c);
      if (K == 1) p[i] = __builtin_elementwise_fma(p[i], pb, pc);
      if (K == 2) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      if (K == 3) d[i] = __builtin_fma(d[i], 1.0000001, 0.5);
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + p[i].x + p[i].y + (float)d[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int K>
double run(float* out, int waves, int n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_op<K>, dim3(waves), dim3(64), 0, 0, out, n);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_op<K>, dim3(waves), dim3(64), 0, 0, out, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e-3;
}

int main() {
  float* out; CK(hipMalloc(&out, 4 << 20));
  const int n = 20000;
  const char* names[4] = {"v_fma_f32", "v_pk_fma_f32", "v_min3_f32", "v_fma_f64"};
  for (int waves : {1024, 2048, 4096}) {
    double t[4] = {run<0>(out, waves, n), run<1>(out, waves, n), run<2>(out, waves, n), run<3>(out, waves, n)};
    for (int k = 0; k < 4; ++k) {
      const double ops = (double)waves * n * 8;            // wave-instructions
      // cycles per wave-instruction per SIMD at 2.4 GHz (1024 SIMDs)
      printf("waves %5d %-14s %.3f ms  %.2f cyc/instr/SIMD\n", waves, names[k], t[k] * 1e3,
             t[k] * 2.4e9 * 1024 / ops);
    }
  }
  return 0;
}
