// Micro-benchmark of the per-sample latency chain (not part of the library): s_memtime stamps
// around steer, the body rays and the arc check for one wave of samples, plus fp64 / fp32
// dependent-chain calibration.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
// -ffp-contract=off tools/ubench.hip -o tools/ubench ; run on the GPU box: tools/ubench
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../theta-rrt_amd/csrc/geom.hpp"

using namespace tr;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memtime(); }

__global__ void k_chain(double* out, int n, uint64_t* cyc) {
  double a = threadIdx.x * 1e-3, b = 1.0000001;
  float f = threadIdx.x * 1e-3f, fb = 1.0001f;
  uint64_t t0 = now();
  for (int i = 0; i < n; ++i) a = fma(a, b, 0.5);
  __builtin_amdgcn_s_waitcnt(0);
  out[threadIdx.x] = a;
  uint64_t t1 = now();
  for (int i = 0; i < n; ++i) f = fmaf(f, fb, 0.5f);
  out[64 + threadIdx.x] = f;
  uint64_t t2 = now();
  double s = 0, c = 0, x = a;
  for (int i = 0; i < 16; ++i) { sincos(x, &s, &c); x = s + c; }
  out[128 + threadIdx.x] = x;
  uint64_t t3 = now();
  for (int i = 0; i < 16; ++i) { x = atan2(x, 1.5); }
  out[192 + threadIdx.x] = x;
  uint64_t t4 = now();
  for (int i = 0; i < 16; ++i) { x = 1.0 / (x + 2.0); }
  out[256 + threadIdx.x] = x;
  uint64_t t5 = now();
  for (int i = 0; i < 16; ++i) { x = sqrt(x + 2.0); }
  out[320 + threadIdx.x] = x;
  uint64_t t6 = now();
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4;
    cyc[5] = t6 - t5;
  }
}

struct In { double ox, oy, oth, gx, gy, gth; };

// phases per wave: [0] input load, [1] steer, [2] body rays, [3] arc window + plan + pixels
__global__ __launch_bounds__(64) void k_phases(Params P, Grid g, const In* in, int n,
                                               double* sink, uint64_t* cyc) {
  const int lane = threadIdx.x;
  const int j = blockIdx.x * 64 + lane;
  uint64_t t0 = now();
  In q = in[j < n ? j : 0];
  __builtin_amdgcn_s_waitcnt(0);
  double acc = q.ox + q.gth;
  uint64_t t1 = now();
  double nx, ny, nth;
  Ctrl u;
  steer(P, q.ox, q.oy, q.oth, q.gx, q.gy, q.gth, nx, ny, nth, u);
  acc += nx + ny + nth;
  uint64_t t2 = now();
  int ierr = 0;
  bool ok = body_rays_clear(g, P, nx, ny, nth, &ierr);
  acc += ok ? 1 : 0;
  uint64_t t3 = now();
  // arc check of every lane's arc by the whole wave, one after another (k_arc's wave per record)
  uint64_t arc = 0;
  int nb = 0;
  for (int l = 0; l < 4; ++l) {
    Ctrl v;
    v.steer = __shfl(u.steer, l); v.iccx = __shfl(u.iccx, l); v.iccy = __shfl(u.iccy, l);
    v.rad = __shfl(u.rad, l); v.dist = __shfl(u.dist, l); v.straight = __shfl(u.straight, l);
    double bx = __shfl(q.ox, l), by = __shfl(q.oy, l), lx = __shfl(nx, l), ly = __shfl(ny, l);
    uint64_t a0 = now();
    ArcWin w = arc_window(bx, by, lx, ly, v);
    acc += w.diff;
    int e = 0;
    // the pixel loop of arc_blocked_wave (kernels.hip) restated inline would duplicate it; time the
    // window + circle decomposition, the part every record pays
    int64_t r = trunc_i(v.rad), K = circle_octant_len(r), R2;
    bool dm = circle_drawmore(g, trunc_i(v.iccx), trunc_i(v.iccy), r, K, R2);
    acc += (double)K + (dm ? 1 : 0) + e;
    uint64_t a1 = now();
    arc += a1 - a0;
    nb++;
  }
  uint64_t t4 = now();
  sink[j] = acc;
  if (lane == 0) {
    cyc[4 * blockIdx.x + 0] = t1 - t0;
    cyc[4 * blockIdx.x + 1] = t2 - t1;
    cyc[4 * blockIdx.x + 2] = t3 - t2;
    cyc[4 * blockIdx.x + 3] = arc / nb;
  }
}

int main() {
  const int H = 512, W = 512;
  std::vector<uint8_t> grid(H * W, 1);
  srand(1);
  for (int i = 0; i < H * W; ++i) grid[i] = (rand() % 100) < 8 ? 0 : 1;
  uint8_t* dg;
  CK(hipMalloc(&dg, H * W));
  CK(hipMemcpy(dg, grid.data(), H * W, hipMemcpyHostToDevice));
  Params P{5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 0};
  const int NW = 64, n = NW * 64;
  std::vector<In> in(n);
  for (int j = 0; j < n; ++j) {
    In& q = in[j];
    q.ox = 50 + (rand() % 40000) / 100.0;
    q.oy = 50 + (rand() % 40000) / 100.0;
    q.oth = (rand() % 36000) / 100.0 - 180;
    q.gx = (int)(q.ox + (rand() % 121) - 60);
    q.gy = (int)(q.oy + (rand() % 121) - 60);
    q.gth = (rand() % 36000) / 100.0 - 180;
  }
  In* din;
  double* sink;
  uint64_t* cyc;
  CK(hipMalloc(&din, sizeof(In) * n));
  CK(hipMalloc(&sink, sizeof(double) * 4096));
  CK(hipMalloc(&cyc, sizeof(uint64_t) * 4 * NW));
  CK(hipMemcpy(din, in.data(), sizeof(In) * n, hipMemcpyHostToDevice));
  uint64_t hc[4 * NW];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, sink, 1000, cyc);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc, cyc, sizeof(uint64_t) * 6, hipMemcpyDeviceToHost));
    printf("chain: fp64 fma %.1f cyc/op, fp32 fma %.1f, sincos %.0f cyc, atan2 %.0f, div %.0f, sqrt %.0f\n",
           hc[0] / 1000.0, hc[1] / 1000.0, hc[2] / 16.0, hc[3] / 16.0, hc[4] / 16.0, hc[5] / 16.0);
  }
  Grid g{dg, H, W};
  for (int nw : {1, 64}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_phases, dim3(nw), dim3(64), 0, 0, P, g, din, n, sink, cyc);
      CK(hipEventRecord(e1, 0));
      CK(hipDeviceSynchronize());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(hc, cyc, sizeof(uint64_t) * 4 * nw, hipMemcpyDeviceToHost));
      double m[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0};
      for (int b = 0; b < nw; ++b)
        for (int k = 0; k < 4; ++k) {
          m[k] += hc[4 * b + k] / (double)nw;
          mx[k] = std::max(mx[k], (double)hc[4 * b + k]);
        }
      printf("waves %d: kernel %.1f us | load %.0f steer %.0f rays %.0f arcprep %.0f cyc (mean) | max %.0f %.0f %.0f %.0f\n",
             nw, ms * 1e3, m[0], m[1], m[2], m[3], mx[0], mx[1], mx[2], mx[3]);
    }
  }
  return 0;
}
