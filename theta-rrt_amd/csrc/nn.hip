// Nearest-node argmin (rrt.py:155-158 + search.py:13-15): for every sample j,
//   first index of min_i sqrt(fl(fl((qx - x_i)^2) + fl((qy - y_i)^2)))   in fp64, as np.argmin.
//
// Two sweeps over the node chunks (node = one (x, y) pair; chunk = a contiguous index range):
//   pass 1  packed-fp32 screen: m32[c][j] = min over chunk c of d32 (4 VALU ops per pair, no index)
//   merge 1 per sample: m = min_c m32, thr = m + 2E(m) + m*2^-48 with E a rigorous bound on
//           |d32 - d| (below), so every node of the winning sqrt class has d32 <= thr
//   pass 2  only chunks with m32[c][j] <= thr: exact fp64 distance for nodes with d32 <= thr and
//           the exact (sqrt class, first index) order; every other chunk is skipped per wave
//   merge 2 per sample: exact order over the surviving chunks -> index
// Bound: x32 = fl32(x), q exact; |d32 - d| <= u(2.83 D X + 4 D^2) + O(u^2 X^2) with u = 2^-24,
// D = sqrt(d), X = max |coordinate|.  E uses u' = 4u and 2x the coefficients.
#pragma clang fp contract(off)
#include <stdlib.h>

#include "thetarrt_internal.hpp"

namespace tr {

typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int S1 = 4;      // samples per lane, pass 1
constexpr int S2 = 2;      // samples per lane, pass 2

__device__ __forceinline__ double sqrt_class_lo2(double s) {   // smallest x with sqrt(x)==sqrt(s)
  double r = sqrt(s), x = s;
  for (int it = 0; it < 8; ++it) {
    double p = nextafter(x, -1.0);
    if (!(p >= 0.0) || sqrt(p) != r) break;
    x = p;
  }
  return x;
}

// fp32 screen distance: fma(dx, dx, dy * dy).  Pass 1 and the resolve use this one expression, and
// the bound E below covers it (two roundings of the differences, one product, one fma).
__device__ __forceinline__ float d32of(f2v q, f2v n) {
  const float dx = q.x - n.x, dy = q.y - n.y;
  return __builtin_fmaf(dx, dx, dy * dy);
}

// ------------------------------------------------------------------ pass 1
// grid (ceil(B / 256 S1), Cgrid); the node count N is read on the device (the tree grows on the
// device between launches); chunks past N exit.  m32[j * Cs + c] = chunk minimum of d32.
// A chunk is swept 256 nodes at a time: each lane loads 4 nodes (coalesced, the next sub-chunk in
// flight while this one is used) and v_readlane broadcasts every node to the wave as a scalar
// operand, so the inner loop has no memory access and no wait.
constexpr int SUB = 256;          // nodes per sub-chunk = 64 lanes x 4

__device__ __forceinline__ float bcast(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__global__ __launch_bounds__(256) void k_nn_pass1(const int2* __restrict__ qxy, int64_t B,
                                                  const float2* __restrict__ t32,
                                                  const int64_t* __restrict__ count, int64_t chunk,
                                                  int64_t Cs, float* __restrict__ m32) {
  const int64_t N = count[0];
  const int64_t c = blockIdx.y;
  const int64_t i0 = c * chunk;
  if (i0 >= N) return;
  const int64_t i1 = min(N, i0 + chunk);
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)blockIdx.x * (256 * S1) + threadIdx.x;
  f2v q[S1];
  float m[S1];
#pragma unroll
  for (int s = 0; s < S1; ++s) {
    const int64_t j = base + s * 256;
    const int2 v = j < B ? qxy[j] : make_int2(0, 0);
    q[s] = f2v{(float)v.x, (float)v.y};
    m[s] = INFINITY;
  }
  auto load = [&](int64_t at, float2 (&nd)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t k = at + r * 64 + lane;
      nd[r] = k < i1 ? t32[k] : make_float2(INFINITY, INFINITY);   // inf: d32 = inf, no effect
    }
  };
  float2 cur[4], nxt[4];
  load(i0, cur);
  for (int64_t at = i0; at < i1; at += SUB) {
    load(at + SUB, nxt);                       // next sub-chunk in flight
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int l = 0; l < 64; l += 8) {          // 16 readlanes ahead of their uses (no hazards)
        f2v n[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) n[k] = f2v{bcast(cur[r].x, l + k), bcast(cur[r].y, l + k)};
#pragma unroll
        for (int k = 0; k < 8; k += 2)
#pragma unroll
          for (int s = 0; s < S1; ++s)
            m[s] = fminf(m[s], fminf(d32of(q[s], n[k]), d32of(q[s], n[k + 1])));
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) cur[r] = nxt[r];
  }
#pragma unroll
  for (int s = 0; s < S1; ++s) {
    const int64_t j = base + s * 256;
    if (j < B) m32[j * Cs + c] = m[s];
  }
}

// ------------------------------------------------------------------ resolve
__device__ __forceinline__ float screen_threshold(float m32min, double X) {
  if (!(m32min < INFINITY)) return INFINITY;
  const double u = 2.384185791015625e-07;             // 2^-22 = 4 * 2^-24
  const double m = (double)m32min;
  const double a = 1.0 - 8.0 * u;
  const double Dm = (4.0 * u * X + sqrt(16.0 * u * u * X * X + 4.0 * a * m)) / (2.0 * a) + 1e-12;
  const double E = u * (4.0 * Dm * X + 8.0 * Dm * Dm) + (u * X) * (u * X);
  const double thr = m + 2.01 * E + m * 3.552713678800501e-15 + 1e-30;   // + m * 2^-48
  return nextafterf((float)thr, INFINITY);
}

__device__ __forceinline__ bool exact_better(double sa, int64_t ia, double sb, int64_t ib) {
  if (ia < 0) return false;
  if (ib < 0) return true;
  if (sa == sb) return ia < ib;
  const double ra = sqrt(sa), rb = sqrt(sb);
  return ra < rb || (ra == rb && ia < ib);
}

// One wave per sample: threshold from the chunk minima, then an exact fp64 scan (lanes over
// nodes, coalesced) of only the chunks whose minimum is under it, then the exact wave argmin.
__global__ __launch_bounds__(256) void k_nn_resolve(const int2* __restrict__ qxy, int64_t B,
                                                    const double2* __restrict__ txy,
                                                    const float2* __restrict__ t32,
                                                    const int64_t* __restrict__ count,
                                                    int64_t chunk, int64_t Cs,
                                                    const unsigned long long* __restrict__ maxabs,
                                                    double qmax, const float* __restrict__ m32,
                                                    int64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= B) return;
  const int64_t N = count[0];
  const int64_t C = (N + chunk - 1) / chunk;
  const float* row = m32 + j * Cs;
  float m = INFINITY;
#pragma unroll 8
  for (int64_t c = lane; c < C; c += 64) m = fminf(m, row[c]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fminf(m, __shfl_xor(m, off));
  const double X = fmax(__longlong_as_double((long long)maxabs[0]), qmax) + 1.0;
  const float thr = screen_threshold(m, X);
  const int2 qi = qxy[j];
  const f2v q{(float)qi.x, (float)qi.y};
  const double qx = (double)qi.x, qy = (double)qi.y;
  double sb = INFINITY, lob = INFINITY;
  int64_t ib = -1;
  for (int64_t cb = 0; cb < C; cb += 64) {
    const int64_t cl = cb + lane;
    unsigned long long mask = __ballot(cl < C && row[cl] <= thr);
    while (mask) {
      const int64_t c = cb + __builtin_ctzll(mask);
      mask &= mask - 1;
      const int64_t i1 = min(N, (c + 1) * chunk);
#pragma unroll 4
      for (int64_t i = c * chunk + lane; i < i1; i += 64) {
        const float2 n = t32[i];
        if (d32of(q, f2v{n.x, n.y}) <= thr) {            // candidate: exact fp64 and order
          const double2 e = txy[i];
          const double a = qx - e.x, b = qy - e.y;
          const double d = a * a + b * b;
          if (d < lob) {                                 // this lane visits increasing i
            sb = d;
            ib = i;
            lob = sqrt_class_lo2(d);
          }
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double so = __shfl_xor(sb, off);
    const int64_t io = __shfl_xor(ib, off);
    if (exact_better(so, io, sb, ib)) { sb = so; ib = io; }
  }
  if (lane == 0) out[j] = ib;
}

// ------------------------------------------------------------------ host side
static int64_t env_or(const char* name, int64_t dflt) {   // tuning knobs (TR_NN_BLOCKS ...)
  const char* v = getenv(name);
  return v ? atoll(v) : dflt;
}

int64_t nn_chunks(int64_t B, int64_t N, int64_t* chunk) {
  static const int64_t target = env_or("TR_NN_BLOCKS", 2048), minch = env_or("TR_NN_MINCHUNK", 256);
  const int64_t bx = (B + 256 * S1 - 1) / (256 * S1);
  int64_t C = std::max<int64_t>(1, target / bx);
  C = std::min<int64_t>(C, std::max<int64_t>(1, N / minch));
  // whole sub-chunks, rounded down so that the grid keeps at least the target chunk count
  const int64_t ch = std::max<int64_t>(1, N / (C * SUB)) * SUB;
  *chunk = ch;
  return std::max<int64_t>(1, (N + ch - 1) / ch);
}

void nn_launch(hipStream_t st, const int2* qxy, int64_t B, const double2* txy, const float2* t32,
               const int64_t* count, int64_t n_ub, const unsigned long long* maxabs, double qmax,
               float* m32, int64_t* out) {
  int64_t chunk;
  const int64_t C = nn_chunks(B, n_ub, &chunk);
  dim3 g1((unsigned)((B + 256 * S1 - 1) / (256 * S1)), (unsigned)C);
  hipLaunchKernelGGL(k_nn_pass1, g1, dim3(256), 0, st, qxy, B, t32, count, chunk, C, m32);
  hipLaunchKernelGGL(k_nn_resolve, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, qxy, B, txy, t32,
                     count, chunk, C, maxabs, qmax, m32, out);
}

int64_t nn_scratch(int64_t B, int64_t n_ub) {    // floats of m32 needed
  int64_t chunk;
  return nn_chunks(B, n_ub, &chunk) * B;
}

}  // namespace tr
