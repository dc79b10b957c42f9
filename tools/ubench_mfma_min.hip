// Does gfx950 overlap v_mfma_f32_32x32x2_f32 with v_min3_f32 on one SIMD?  (not part of the
// library; the question behind k_nn_pass1's 0.50 steady state).  Per loop trip a
// wave issues 4 independent MFMAs (K & 1) and/or 32 v_min3 (K & 2) that read the previous trip's
// MFMA results (as k_nn_pass1's minimum trees do: 8 per MFMA).  Blocks of 256 threads = one wave
// per SIMD at 256 blocks; 512 blocks = two.  Timed with events; cycles at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 tools/ubench_mfma_min.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

template <int K>
__global__ __launch_bounds__(256, 2) void k_mix(float* out, int n) {
  const float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  f32x16 d[4];
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) d[j][r] = r + j;
  float m[8];
  for (int i = 0; i < 8; ++i) m[i] = 1e30f;
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (K & 2) {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(m[q]) : "v"(d[j][2 * q]), "v"(d[j][2 * q + 1]));
      }
      if (K & 1) d[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d[j], 0, 0, 0);
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += m[i];
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) s += d[j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int K>
double run(float* out, int blocks, int n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mix<K>, dim3(blocks), dim3(256), 0, 0, out, n);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_mix<K>, dim3(blocks), dim3(256), 0, 0, out, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e-3;
}

int main() {
  float* out; CK(hipMalloc(&out, 8 << 20));
  const int n = 20000;
  const char* names[4] = {"", "MFMA only", "v_min3 only", "MFMA + v_min3"};
  for (int blocks : {256, 512}) {
    double t[4] = {0, run<1>(out, blocks, n), run<2>(out, blocks, n), run<3>(out, blocks, n)};
    for (int k = 1; k < 4; ++k) {
      const double slots = (double)blocks * 4 * n * 4 / 1024;   // MFMA slots (4 per trip) per SIMD
      printf("waves/SIMD %d %-14s %.3f ms  %.1f cyc per MFMA slot per SIMD\n", blocks / 256, names[k],
             t[k] * 1e3, t[k] * 2.4e9 / slots);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
