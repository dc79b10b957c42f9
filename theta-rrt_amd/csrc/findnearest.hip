// findnearest (rrt.py:117-128): for a goal pose g, the first child in the reference's traversal
//   for parent in G.keys(): for child in G[parent]:  d = weightxy * L2norm(child[0], g[0])
//                                                       + (1 - weightxy) * |anglediff(child[1], g[1])|
// with the smallest d (strict <: the first of equal distances wins).  main.py:79 calls it when an
// RRT segment misses its goal.
//
// Edges arrive as (parent index, child index) pairs in any order that lists each parent's children
// in append order (the session's append log, or the traversal itself): the traversal position of an
// edge is then the lexicographic (parent, edge position) key, so the reference's choice is the
// minimum of (d, parent, position) -- a plain associative reduction.
//
// k_fn_partial  grid (blocks, goals): every thread keeps the minimum over a strided slice of the
//               edges (increasing positions), the block reduces it (wave shuffles, then LDS) and
//               writes one partial per (goal, block).  Per edge: two node loads (x, y and theta),
//               one sqrt, one sincos and two atan2 of the exact scipy anglediff restatement (fp64):
//               the kernel is fp64-VALU/latency bound, edges are streamed once (16 B per edge).
// k_fn_final    one wave per goal reduces its partials.
#pragma clang fp contract(off)
#include "thetarrt_internal.hpp"

namespace tr {

struct FnKey {
  double d;
  int64_t par, pos;   // pos = -1: no edge
};

__device__ __forceinline__ bool fn_less(const FnKey& a, const FnKey& b) {
  if (a.pos < 0) return false;
  if (b.pos < 0) return true;
  if (a.d != b.d) return a.d < b.d;
  if (a.par != b.par) return a.par < b.par;
  return a.pos < b.pos;
}

__device__ __forceinline__ FnKey fn_shfl_xor(const FnKey& k, int off) {
  FnKey o;
  o.d = __shfl_xor(k.d, off);
  o.par = __shfl_xor(k.par, off);
  o.pos = __shfl_xor(k.pos, off);
  return o;
}

__device__ __forceinline__ FnKey fn_wave_min(FnKey k) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const FnKey o = fn_shfl_xor(k, off);
    if (fn_less(o, k)) k = o;
  }
  return k;
}

// rrt.py:122 for one child pose against goal (gx, gy, gth); w = builtins.weightxy.
__device__ __forceinline__ double fn_distance(double x, double y, double th, double gx, double gy,
                                              double gth, double w) {
  const double a = gx - x, b = gy - y;                 // L2norm(child[0], goal[0]), search.py:13-15
  const double l2 = sqrt(a * a + b * b);
  return w * l2 + (1 - w) * fabs(angle_diff_exact(th, gth));
}

constexpr int FN_T = 256;

__global__ __launch_bounds__(FN_T) void k_fn_partial(const double* __restrict__ xs, int sx,
                                                     const double* __restrict__ ys, int sy,
                                                     const double* __restrict__ ths, int sth,
                                                     const int64_t* __restrict__ e_par,
                                                     const int64_t* __restrict__ e_child,
                                                     int64_t E, const double* __restrict__ goals3,
                                                     double w, FnKey* __restrict__ part) {
  __shared__ FnKey red[FN_T / 64];
  const int g = blockIdx.y;
  const double gx = goals3[3 * g], gy = goals3[3 * g + 1], gth = goals3[3 * g + 2];
  FnKey best{INFINITY, 0, -1};
  const int64_t stride = (int64_t)gridDim.x * FN_T;
  for (int64_t e = (int64_t)blockIdx.x * FN_T + threadIdx.x; e < E; e += stride) {
    const int64_t c = e_child[e];
    const double d = fn_distance(xs[c * sx], ys[c * sy], ths[c * sth], gx, gy, gth, w);
    const FnKey k{d, e_par[e], e};
    if (fn_less(k, best)) best = k;
  }
  best = fn_wave_min(best);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 1; k < FN_T / 64; ++k)
      if (fn_less(red[k], best)) best = red[k];
    part[(int64_t)g * gridDim.x + blockIdx.x] = best;
  }
}

__global__ __launch_bounds__(64) void k_fn_final(const FnKey* __restrict__ part, int nblk,
                                                 const int64_t* __restrict__ e_child,
                                                 int64_t* __restrict__ out_child,
                                                 double* __restrict__ out_d) {
  const int g = blockIdx.x;
  FnKey best{INFINITY, 0, -1};
  for (int k = threadIdx.x; k < nblk; k += 64) {
    const FnKey o = part[(int64_t)g * nblk + k];
    if (fn_less(o, best)) best = o;
  }
  best = fn_wave_min(best);
  if (threadIdx.x == 0) {
    out_child[g] = best.pos >= 0 ? e_child[best.pos] : -1;
    out_d[g] = best.pos >= 0 ? best.d : NAN;
  }
}

int64_t fn_blocks(int64_t E, int64_t G) {
  // about 4 edges per thread; the grid of all goals stays within a few blocks per CU
  const int64_t want = (E + 4 * FN_T - 1) / (4 * FN_T);
  const int64_t cap = std::max<int64_t>(1, 2048 / std::max<int64_t>(1, G));
  return std::max<int64_t>(1, std::min(want, cap));
}

int64_t fn_scratch(int64_t E, int64_t G) {   // bytes of partials
  return (int64_t)sizeof(FnKey) * fn_blocks(E, G) * G;
}

void launch_findnearest(hipStream_t st, const double* xs, int sx, const double* ys, int sy,
                        const double* ths, int sth, const int64_t* e_par, const int64_t* e_child,
                        int64_t E, const double* goals3, int64_t G, double w, void* scratch,
                        int64_t* out_child, double* out_d) {
  const int64_t nb = fn_blocks(E, G);
  FnKey* part = static_cast<FnKey*>(scratch);
  hipLaunchKernelGGL(k_fn_partial, dim3((unsigned)nb, (unsigned)G), dim3(FN_T), 0, st, xs, sx, ys,
                     sy, ths, sth, e_par, e_child, E, goals3, w, part);
  hipLaunchKernelGGL(k_fn_final, dim3((unsigned)G), dim3(64), 0, st, part, (int)nb, e_child,
                     out_child, out_d);
}

}  // namespace tr
