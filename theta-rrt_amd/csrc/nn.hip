// Nearest-node argmin (rrt.py:155-158 + search.py:13-15): for every sample j,
//   first index of min_i sqrt(fl(fl((qx - x_i)^2) + fl((qy - y_i)^2)))   in fp64, as np.argmin.
//
// Two kernels over node chunks (chunk = a contiguous index range of the tree):
//   k_nn_pass1   fp32 screen.  A node is screened as s_i = fma(ax, x^, fma(by, y^, w^)) with
//                (x^, y^) = fp32 of the node relative to the tree centre, w^ = fp32(x^2 + y^2),
//                (ax, by) = -2 (q - centre): s_i = |q - n_i|^2 - |q - centre|^2 up to rounding.
//                Two packed FMAs per two samples and one v_min3 per two nodes; a wave streams its
//                chunk's nodes through the scalar cache (wave-uniform SGPR operands).  Output:
//                the minimum of s over every (chunk, sample), m32[c * B + j] (coalesced stores).
//   k_nn_resolve one wave per sample (chunk minima staged through LDS): m = min_c m32, threshold thr = m + 2E + slack with E a rigorous
//                bound on |s_i - (d_i - |q^|^2)| (below); only chunks with a minimum <= thr are
//                rescanned (exact fp64 distance over all their nodes, 8 independent 64-node pieces
//                in flight per lane) with the exact (sqrt class, first index) order of the reference.
// Bound (u = 2^-24, X = max |centred coordinate| over nodes and queries): representation 8uX^2,
// w^ 2uX^2, inner fma 4uX^2, outer fma 6uX^2: |s_i - (d_i - |q^|^2)| <= 20uX^2 (1 + O(u)); E uses
// 24uX^2.  Every node of the winning sqrt class then has s <= m + 2E + (|m| + |q^|^2 + E) 2^-48.
#pragma clang fp contract(off)
#include <stdlib.h>

#include "thetarrt_internal.hpp"

namespace tr {

typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int S = 8;          // samples per lane in pass 1 (4 packed pairs)
constexpr int CH_ALIGN = 64;  // chunk sizes are multiples of this

__device__ __forceinline__ f2v pkfma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// ------------------------------------------------------------------ pass 1
// Work unit (g, c): sample group g = [g*GS, +GS) (S samples per lane, four waves) against chunk c
// of the node range [lo, hi) (both read on the device: the tree grows there between launches).
// The block stages the chunk (tiles of CHMAX nodes) into LDS; each wave then reads the nodes
// back as wave-wide broadcasts, four at a time with the next four in flight, and screens them
// against its 64 x S samples.  A grid of a few blocks per CU loops over the units.
constexpr int GS = 256 * S;      // samples per unit
constexpr int CHMAX = 1024;      // max chunk (nodes staged in LDS: 16 KB)

__device__ __forceinline__ float min3f(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__global__ __launch_bounds__(256) void k_nn_pass1_valu(const int2* __restrict__ qxy, int64_t B,
                                                       int32_t cx, int32_t cy,
                                                       const float4* __restrict__ t4,
                                                       const int64_t* __restrict__ lo_p,
                                                       const int64_t* __restrict__ hi_p,
                                                       int64_t chunk, int32_t ngrp,
                                                       float* __restrict__ m32) {
  __shared__ float4 tile[CHMAX];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t lo = lo_p ? lo_p[0] : 0;
  const int64_t hi = hi_p[0];
  const int C = (int)((hi - lo + chunk - 1) / chunk);
  const int units = ngrp * C;
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int c = u / ngrp, gsel = u - c * ngrp;
    const int64_t i0 = lo + (int64_t)c * chunk;
    const int64_t nu = min(hi, i0 + chunk) - i0;         // 1 .. chunk
    const int64_t jb = (int64_t)gsel * GS + w * (64 * S) + lane;
    f2v ax[S / 2], by[S / 2];
    float mx[S / 2], my[S / 2];
#pragma unroll
    for (int p = 0; p < S / 2; ++p) {
      const int64_t j0 = jb + (2 * p) * 64, j1 = j0 + 64;
      const int2 a = qxy[j0 < B ? j0 : B - 1];
      const int2 b = qxy[j1 < B ? j1 : B - 1];
      ax[p] = f2v{-2.0f * (float)(a.x - cx), -2.0f * (float)(b.x - cx)};
      by[p] = f2v{-2.0f * (float)(a.y - cy), -2.0f * (float)(b.y - cy)};
      mx[p] = my[p] = INFINITY;
    }
    for (int64_t t0 = 0; t0 < nu; t0 += CHMAX) {          // one tile unless chunk > CHMAX
      const int n = (int)min<int64_t>(CHMAX, nu - t0);
      __syncthreads();                                    // the previous tile is consumed
      for (int k = t; k < n; k += 256) tile[k] = t4[i0 + t0 + k];
      __syncthreads();
      // node k >= n reads node n - 1 again (a repeated node leaves a minimum unchanged)
      float4 A[4], Q[4];
      auto load4 = [&](float4* v, int k) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tile[min(k + r, n - 1)];
      };
      auto screen4 = [&](const float4* v) {
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f2v xa{v[r].x, v[r].x}, ya{v[r].y, v[r].y}, wa{v[r].z, v[r].z};
          const f2v xb{v[r + 1].x, v[r + 1].x}, yb{v[r + 1].y, v[r + 1].y};
          const f2v wb{v[r + 1].z, v[r + 1].z};
#pragma unroll
          for (int p = 0; p < S / 2; ++p) {
            const f2v da = pkfma(ax[p], xa, pkfma(by[p], ya, wa));
            const f2v db = pkfma(ax[p], xb, pkfma(by[p], yb, wb));
            mx[p] = min3f(mx[p], da.x, db.x);
            my[p] = min3f(my[p], da.y, db.y);
          }
        }
      };
      load4(A, 0);
      for (int k = 0; k < n; k += 8) {
        load4(Q, k + 4);
        screen4(A);
        load4(A, k + 8);
        screen4(Q);
      }
    }
    float* out = m32 + (int64_t)c * B;
#pragma unroll
    for (int p = 0; p < S / 2; ++p) {
      const int64_t j0 = jb + (2 * p) * 64, j1 = j0 + 64;
      if (j0 < B) out[j0] = mx[p];
      if (j1 < B) out[j1] = my[p];
    }
  }
}

// ------------------------------------------------------------------ pass 1 on the matrix cores
// The screen of a 32-node x 32-sample tile is ONE v_mfma_f32_32x32x2_f32:
//   A = nodes   (row i = node, k0 = y^, k1 = x^),   lane l holds A[l & 31][l >> 5]
//   B = samples (col j = sample, k0 = by, k1 = ax),  lane l holds B[l >> 5][l & 31]
//   C = w^ of the row's node.
// gfx950's f32 MFMA is bit-for-bit the k-ordered fmaf chain D = fma(a1, b1, fma(a0, b0, C))
// (cdna_hip_programming.md, "FP32-input MFMA"), i.e. s = fma(ax, x^, fma(by, y^, w^)) exactly as the
// VALU screen (k_nn_pass1_valu) rounds it: same m32, same error bound.  D's column is the lane
// (j = l & 31) and its 16 registers are node rows (r & 3) + 8 (r >> 2) + 4 (l >> 5), so the minimum
// over nodes is a per-lane v_min3 tree; lanes l and l ^ 32 (the other 16 rows) merge once per unit.
// Per tile and wave: 64 MFMA cycles for 1024 pairs (the f32 matrix peak, 16 pairs/clk/SIMD) beside
// 8 v_min3 on the VALU (about 40 issue cycles, hidden in the MFMA's shadow).  The chunk is staged
// in LDS as three planes (y^, x^, w^): one ds_read_b32 for A and four ds_read_b128 for C per tile,
// shared by the wave's MT sample tiles.
constexpr int MT = 16;           // sample tiles (32 samples each) per wave: 4 waves x 16 x 32 = GS
static_assert(4 * 32 * MT == GS, "a unit's samples are the four waves' tiles");
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float fmin3(float a, float b, float c) {
  return __builtin_fminf(__builtin_fminf(a, b), c);      // v_min3_f32 (operands never NaN)
}

__device__ __forceinline__ float min16(const f32x16& d, float m) {
  const float a = fmin3(d[0], d[1], d[2]), b = fmin3(d[3], d[4], d[5]);
  const float c = fmin3(d[6], d[7], d[8]), e = fmin3(d[9], d[10], d[11]);
  const float f = fmin3(d[12], d[13], d[14]);
  return fmin3(fmin3(a, b, c), fmin3(e, f, d[15]), m);
}

__global__ __launch_bounds__(256, 2) void k_nn_pass1(const int2* __restrict__ qxy, int64_t B,
                                                  int32_t cx, int32_t cy,
                                                  const float4* __restrict__ t4,
                                                  const int64_t* __restrict__ lo_p,
                                                  const int64_t* __restrict__ hi_p, int64_t chunk,
                                                  int32_t ngrp, float* __restrict__ m32) {
  __shared__ float py[CHMAX], px[CHMAX];
  __shared__ __attribute__((aligned(16))) float pw[CHMAX];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, col = lane & 31, h = lane >> 5;
  const int64_t lo = lo_p ? lo_p[0] : 0;
  const int64_t hi = hi_p[0];
  const int C = (int)((hi - lo + chunk - 1) / chunk);
  const int units = ngrp * C;
  const float* pa = h ? px : py;                          // A's k = lane half: y^ then x^
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int c = u / ngrp, gsel = u - c * ngrp;
    const int64_t i0 = lo + (int64_t)c * chunk;
    const int64_t nu = min(hi, i0 + chunk) - i0;         // 1 .. chunk
    const int64_t jb = (int64_t)gsel * GS + w * (32 * MT) + col;   // sample of tile s: jb + 32 s
    // every load of the unit's samples is in flight at once (both components, then a select)
    int2 qa[MT];
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      const int64_t j = jb + 32 * s;
      qa[s] = qxy[j < B ? j : B - 1];
    }
    float bq[MT], m[MT];
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      const float fx = -2.0f * (float)(qa[s].x - cx), fy = -2.0f * (float)(qa[s].y - cy);
      bq[s] = h ? fx : fy;                                // B's k = lane half
      m[s] = INFINITY;
    }
    for (int64_t t0 = 0; t0 < nu; t0 += CHMAX) {          // one tile unless chunk > CHMAX
      const int n = (int)min<int64_t>(CHMAX, nu - t0);
      const int n32 = (n + 31) & ~31;                     // rows >= n repeat node n - 1
      float4 v[CHMAX / 256];
#pragma unroll
      for (int r = 0; r < CHMAX / 256; ++r) {             // all staging loads in flight
        const int k = t + 256 * r;
        if (k < n32) v[r] = t4[i0 + t0 + min(k, n - 1)];
      }
      __syncthreads();                                    // the previous tile is consumed
#pragma unroll
      for (int r = 0; r < CHMAX / 256; ++r) {
        const int k = t + 256 * r;
        if (k < n32) {
          px[k] = v[r].x;
          py[k] = v[r].y;
          pw[k] = v[r].z;
        }
      }
      __syncthreads();
      for (int k = 0; k < n32; k += 32) {
        const float a = pa[k + col];
        f32x16 cw;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(&pw[k + 8 * q + 4 * h]);
          cw[4 * q] = v.x;
          cw[4 * q + 1] = v.y;
          cw[4 * q + 2] = v.z;
          cw[4 * q + 3] = v.w;
        }
        // PD accumulators in flight: tile s + PD - 1's MFMA issues before tile s's minimum reads D
        constexpr int PD = 4;
        f32x16 d[PD];
#pragma unroll
        for (int s = 0; s < PD - 1; ++s)
          d[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bq[s], cw, 0, 0, 0);
#pragma unroll
        for (int s = 0; s < MT; ++s) {
          if (s + PD - 1 < MT)
            d[(s + PD - 1) % PD] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bq[s + PD - 1], cw, 0, 0, 0);
          m[s] = min16(d[s % PD], m[s]);
        }
      }
    }
    float* out = m32 + (int64_t)c * B;
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      const float o = fminf(m[s], __shfl_xor(m[s], 32));
      const int64_t j = jb + 32 * s;
      if (h == 0 && j < B) out[j] = o;
    }
  }
}

// ------------------------------------------------------------------ resolve
// Threshold on s for sample p = q - centre (exact integers), from the minimum m of s over the tree.
// Eg = 24 u X^2 bounds |s_i - (d_i - |p|^2)| for every node.  The winner w and the node k that
// attains m both have d <= Dup = m + |p|^2 + Eg, i.e. lie within R = sqrt(Dup) of q, so their
// rounding errors obey a bound in terms of |p| and R only (much tighter for samples near the
// centre):  w^ rounding u1 Wp, inner fma u T, outer fma u Sm, fp32 coordinates rep.
__device__ __forceinline__ double screen_E(double px, double py, double R, double Eg) {
  const double u = 5.9604644775390625e-08, u1 = u + 2.220446049250313e-16;   // 2^-24, + 2^-52
  const double p2 = px * px + py * py;
  const double Ax = (fabs(px) + R) * (1.0 + 2.0 * u1), Ay = (fabs(py) + R) * (1.0 + 2.0 * u1);
  const double R1 = R + u1 * fmax(Ax, Ay);                       // |fp32 coordinate - p| bound
  const double Wp = (Ax * Ax + Ay * Ay) * (1.0 + 4.0 * u1);      // >= |w^|
  const double T = fmax(Ax * Ax + R1 * R1, py * py) + u1 * Wp;   // >= |inner fma before rounding|
  const double Sm = p2 + 2.0 * R1 * R1 + u1 * Wp + u * T + 1.0;   // >= |outer fma before rounding|
  const double rep = 2.0 * u1 * (Ax * (2.0 * R1 + u1 * Ax) + Ay * (2.0 * R1 + u1 * Ay));
  return fmin(Eg, 1.25 * (u1 * Wp + u * T + u * Sm + rep));
}

__device__ __forceinline__ double screen_Eg(double X) {
  return 24.0 * 5.9604644775390625e-08 * X * X;                  // 24 u X^2: every node
}

__device__ __forceinline__ float screen_threshold(float mmin, double px, double py, double X) {
  if (!(mmin < INFINITY)) return INFINITY;
  const double m = (double)mmin, p2 = px * px + py * py;
  const double Eg = screen_Eg(X);
  const double Dup = fmax(0.0, m + p2 + Eg) * (1.0 + 1e-12);
  const double R = sqrt(Dup) * (1.0 + 1e-12) + 1e-9;
  const double E = screen_E(px, py, R, Eg);
  const double thr = m + 2.0 * E + (fabs(m) + p2 + E + 1.0) * 5.684341886080802e-14;   // 2^-44
  return nextafterf((float)thr, INFINITY);
}

// Block of RS waves = RS consecutive samples, one wave each.  The block first stages the chunk
// minima of its samples (m32[c][j0 .. j0 + RS), 64 B row pieces, coalesced) into LDS, so every
// wave reads its column from LDS.  Per sample: threshold from the minimum, then an exact fp64 scan
// (lanes over nodes, coalesced) of only the chunks whose minimum is under it, then the exact wave
// argmin.
#ifndef TR_RS
#define TR_RS 16                 // build-time A/B knob (tools/build_variants.py)
#endif
constexpr int RS = TR_RS;
#ifdef TR_DIAG_RESOLVE
__device__ unsigned long long g_diag_res[6];
#endif        // samples (waves) per resolve block
constexpr int RSP = RS + 1;      // padded LDS row (column reads hit distinct banks)
constexpr int64_t CMAX = 2048;   // chunk count cap (LDS: CMAX * RSP * 4 B)

// Nearest node over the chunks of [0, *count) swept into m32 -> out[j] (its exact d -> dout[j]).
__global__ __launch_bounds__(64 * RS) void k_nn_resolve(const int2* __restrict__ qxy, int64_t B,
                                                        int32_t cx, int32_t cy,
                                                        const double2* __restrict__ txy,
                                                        const int64_t* __restrict__ count,
                                                        int64_t chunk,
                                                        const unsigned long long* __restrict__ maxabs,
                                                        double qmax, const float* __restrict__ m32,
                                                        int64_t* __restrict__ out,
                                                        double* __restrict__ dout) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * RS;
  const int64_t N = count[0];
  const int64_t C = (N + chunk - 1) / chunk;
  const int64_t j = j0 + w;
  const int2 qi = qxy[min(j, B - 1)];
  const double X = fmax(__longlong_as_double((long long)maxabs[0]), qmax) + 1.0;
  {
    // thread t stages column t % RS of rows t / RS + 64 k: all loads of a thread in flight at once
    constexpr int SU = 8;
    const int k = threadIdx.x % RS;
    const bool ok = j0 + k < B;
    for (int64_t c0 = threadIdx.x / RS; c0 < C; c0 += SU * 64) {
      float v[SU];
#pragma unroll
      for (int r = 0; r < SU; ++r) {
        const int64_t c = c0 + r * 64;
        v[r] = INFINITY;
        if (ok && c < C) v[r] = m32[c * B + j0 + k];
      }
#pragma unroll
      for (int r = 0; r < SU; ++r) {
        const int64_t c = c0 + r * 64;
        if (c < C) sm[c * RSP + k] = v[r];
      }
    }
  }
  __syncthreads();
  if (j >= B) return;                      // no barrier below
  const float* col = sm + w;
  const int nc = (int)C;
  const double hx = (double)(qi.x - cx), hy = (double)(qi.y - cy);
  float m = INFINITY;
#pragma unroll 4
  for (int c = lane; c < nc; c += 64) m = fminf(m, col[c * RSP]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fminf(m, __shfl_xor(m, off));
  const float thr = screen_threshold(m, hx, hy, X);
  const double qx = (double)qi.x, qy = (double)qi.y;
  // per lane: the smallest sqrt(d) (the reference's key, math.sqrt of the fp64 sum) and its first
  // index -- lanes visit increasing indices, so a strict < keeps the first of equal keys
  double rb = INFINITY, db = INFINITY;
  int64_t ib = -1;
#ifndef TR_RU
#define TR_RU 8                  // build-time A/B knob (tools/build_variants.py)
#endif
  constexpr int U = TR_RU;                 // pieces in flight per lane
#ifdef TR_DIAG_RESOLVE
  unsigned long long diag_chunks = 0;
#endif
  for (int cb = 0; cb < nc; cb += 64) {
    const int cl = cb + lane;
    unsigned long long mk = __ballot(cl < nc && col[cl * RSP] <= thr);
#ifdef TR_DIAG_RESOLVE
    diag_chunks += (unsigned long long)__builtin_popcountll(mk);
#endif
    // every 64-node piece of every chunk under the threshold, in increasing node order
    int64_t at = 0, end = 0;
    if (mk) { at = (cb + __builtin_ctzll(mk)) * chunk; end = min(N, at + chunk); }
    while (mk) {
      int64_t ii[U];
#pragma unroll
      for (int r = 0; r < U; ++r) {
        ii[r] = -1;
        if (mk) {
          const int64_t i = at + lane;
          if (i < end) ii[r] = i;
          at += 64;
          if (at >= end) {
            mk &= mk - 1;
            if (mk) { at = (cb + __builtin_ctzll(mk)) * chunk; end = min(N, at + chunk); }
          }
        }
      }
      double2 e[U];
#pragma unroll
      for (int r = 0; r < U; ++r) {
        e[r] = make_double2(INFINITY, INFINITY);
        if (ii[r] >= 0) e[r] = txy[ii[r]];
      }
#pragma unroll
      for (int r = 0; r < U; ++r) {
        const double a = qx - e[r].x, b = qy - e[r].y;
        const double d = a * a + b * b;
        if (ii[r] >= 0 && d < db) {          // d >= db: sqrt(d) >= rb at a later index
          const double rt = sqrt(d);
          if (rt < rb) { rb = rt; db = d; ib = ii[r]; }
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ro = __shfl_xor(rb, off), dq = __shfl_xor(db, off);
    const int64_t io = __shfl_xor(ib, off);
    if (io >= 0 && (ib < 0 || ro < rb || (ro == rb && io < ib))) { rb = ro; db = dq; ib = io; }
  }
  if (lane == 0) {
    out[j] = ib;
#ifdef TR_DIAG_RESOLVE                       // diagnosis builds only: rescanned chunks per sample
    atomicAdd(&g_diag_res[0], diag_chunks);
    atomicAdd(&g_diag_res[1], 1ull);
    if (diag_chunks > 8) atomicAdd(&g_diag_res[3], 1ull);
    atomicMax(&g_diag_res[4], diag_chunks);
    if (diag_chunks > 8 && atomicAdd(&g_diag_res[5], 1ull) < 3)
      printf("TR_DIAG_RESOLVE heavy: q=(%d,%d) chunks=%llu m=%g thr=%g d=%g near=%ld\n", qi.x, qi.y,
             diag_chunks, (double)m, (double)thr, db, (long)ib);
    __threadfence();
    if (atomicAdd(&g_diag_res[2], 1ull) == (unsigned long long)B - 1) {
      printf("TR_DIAG_RESOLVE B=%ld C=%ld chunk=%ld rescanned chunks/sample=%.3f samples>8=%llu\n",
             (long)B, (long)C, (long)chunk, (double)g_diag_res[0] / (double)g_diag_res[1],
             g_diag_res[3]);
      printf("TR_DIAG_RESOLVE max chunks=%llu\n", g_diag_res[4]);
      g_diag_res[0] = g_diag_res[1] = g_diag_res[2] = g_diag_res[3] = g_diag_res[4] = g_diag_res[5] = 0;
    }
#endif
    if (dout) dout[j] = db;
  }
}

// ------------------------------------------------------------------ delta (look-ahead correction)
// The nodes appended since a look-ahead resolve, [snap, count), against each live sample's known
// nearest node (near[j], dnear[j] = its exact d).  Exact fp64 over all of them.  A block takes DS
// samples (their coordinates uniform: scalar registers) and its DWV waves split the delta nodes: a
// lane loads one node (coalesced, L2-resident) and tests it against every sample of the block, so
// each node is read once per block and no LDS tile or large workgroup is needed (the main stream's
// kernels share the chip with the look-ahead sweep).  A node wins only with a strictly smaller key
// sqrt(d) (its index is larger than every snapshot index), the first of equal keys among the delta
// nodes; winners replace near / dnear and the sample is appended to changed[].
constexpr int DS = 8;                     // samples per block
constexpr int DWV = 4;                    // waves per block (node split)
__global__ __launch_bounds__(64 * DWV) void k_nn_delta(const int2* __restrict__ qxy, int64_t B,
                                                       const double2* __restrict__ txy,
                                                       const int64_t* __restrict__ snap_p,
                                                       const int64_t* __restrict__ count,
                                                       const int32_t* __restrict__ live,
                                                       int64_t* __restrict__ near,
                                                       double* __restrict__ dnear,
                                                       int32_t* __restrict__ changed,
                                                       int32_t* __restrict__ n_changed) {
  __shared__ double s_rb[DWV][DS], s_dl[DWV][DS];
  __shared__ int64_t s_ib[DWV][DS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t lo = snap_p[0], hi = count[0];
  if (hi <= lo) return;                      // uniform: nothing appended
  const int64_t j0 = (int64_t)blockIdx.x * DS;
  double qx[DS], qy[DS], db[DS], rb[DS], dl[DS];
  int64_t ib[DS];
#pragma unroll
  for (int s = 0; s < DS; ++s) {
    const int64_t j = j0 + s;
    const bool act = j < B && live[j] == 1;
    const int2 q = act ? qxy[j] : make_int2(0, 0);
    qx[s] = (double)q.x;
    qy[s] = (double)q.y;
    db[s] = act ? dnear[j] : -1.0;           // inactive: no node can beat it
    rb[s] = INFINITY;
    dl[s] = INFINITY;
    ib[s] = -1;
  }
#pragma unroll 2
  for (int64_t i = lo + w * 64 + lane; i < hi; i += 64 * DWV) {   // each lane: increasing indices
    const double2 e = txy[i];
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      const double a = qx[s] - e.x, b = qy[s] - e.y;
      const double d = a * a + b * b;
      if (d < db[s] && d < dl[s]) {          // d >= db: sqrt(d) >= the known key
        const double rt = sqrt(d);
        if (rt < rb[s]) { rb[s] = rt; dl[s] = d; ib[s] = i; }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < DS; ++s) {
    if (__ballot(ib[s] >= 0)) {              // rare: some lane has a candidate for sample s
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const double ro = __shfl_xor(rb[s], off), dq = __shfl_xor(dl[s], off);
        const int64_t io = __shfl_xor(ib[s], off);
        if (io >= 0 && (ib[s] < 0 || ro < rb[s] || (ro == rb[s] && io < ib[s]))) {
          rb[s] = ro; dl[s] = dq; ib[s] = io;
        }
      }
    }
    if (lane == 0) {
      s_rb[w][s] = rb[s];
      s_dl[w][s] = dl[s];
      s_ib[w][s] = ib[s];
    }
  }
  __syncthreads();
  if (threadIdx.x < DS) {                    // one thread per sample combines the waves
    const int s = threadIdx.x;
    const int64_t j = j0 + s;
    double r = INFINITY, d = INFINITY;
    int64_t k = -1;
    for (int q = 0; q < DWV; ++q) {
      const int64_t io = s_ib[q][s];
      if (io >= 0 && (k < 0 || s_rb[q][s] < r || (s_rb[q][s] == r && io < k))) {
        r = s_rb[q][s]; d = s_dl[q][s]; k = io;
      }
    }
    if (k >= 0 && j < B && r < sqrt(dnear[j])) {
      near[j] = k;
      dnear[j] = d;
      changed[atomicAdd(n_changed, 1)] = (int32_t)j;
    }
  }
}

// ------------------------------------------------------------------ host side
static int64_t env_or(const char* name, int64_t dflt) {   // tuning knobs (TR_NN_BLOCKS ...)
  const char* v = getenv(name);
  return v ? atoll(v) : dflt;
}

// Chunking of a sweep over up to N nodes for B samples: about `target` pass-1 units (sample
// groups x chunks) when the tree is large enough; chunks of at most maxch <= CHMAX nodes (staged in
// LDS in one tile; the resolve rescans whole chunks), a multiple of CH_ALIGN.
static int64_t nn_chunk_size(int64_t B, int64_t N, int64_t cmax) {
  static const int64_t target = env_or("TR_NN_UNITS", 512);
  static const int64_t maxch = std::min<int64_t>(env_or("TR_NN_MAXCHUNK", 1024), CHMAX);
  const int64_t groups = (B + GS - 1) / GS;
  int64_t C = std::max<int64_t>(1, target / groups);
  C = std::max<int64_t>(C, (N + maxch - 1) / maxch);
  C = std::min<int64_t>(C, cmax);
  const int64_t ch = (std::max<int64_t>(N, 1) + C - 1) / C;
  return std::max<int64_t>(1, (ch + CH_ALIGN - 1) / CH_ALIGN) * CH_ALIGN;
}

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

NNPlan nn_plan(int64_t B, int64_t n_ub) {
  NNPlan p;
  p.chunk = nn_chunk_size(B, n_ub, CMAX);
  p.cmax = std::max<int64_t>(1, ceil_div(n_ub, p.chunk));
  return p;
}

int64_t nn_scratch(int64_t B, const NNPlan& p) { return p.cmax * B; }

void nn_sweep(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy, const float4* t4,
              const int64_t* hi_p, const NNPlan& p, float* m32) {
  // a few blocks per CU loop over the (sample group, chunk) units; the kernel reads the actual
  // node count (the tree may have grown past the plan's bound: more units, same grid)
  static const int64_t cap = env_or("TR_NN_GRID", 512);
  const int64_t groups = ceil_div(B, GS);
  const int64_t g = std::max<int64_t>(1, std::min(groups * p.cmax, cap));
  static const bool valu = env_or("TR_NN_VALU", 0) != 0;   // the VALU screen (same m32), A/B runs
  if (valu)
    hipLaunchKernelGGL(k_nn_pass1_valu, dim3((unsigned)g), dim3(256), 0, st, qxy, B, cx, cy, t4,
                       (const int64_t*)nullptr, hi_p, p.chunk, (int32_t)groups, m32);
  else
    hipLaunchKernelGGL(k_nn_pass1, dim3((unsigned)g), dim3(256), 0, st, qxy, B, cx, cy, t4,
                       (const int64_t*)nullptr, hi_p, p.chunk, (int32_t)groups, m32);
}

void nn_resolve(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy,
                const double2* txy, const int64_t* count, const NNPlan& p,
                const unsigned long long* maxabs, double qmax, const float* m32, int64_t* out,
                double* dout) {
  const size_t lds = (size_t)(p.cmax * RSP * sizeof(float));
  static const bool big_lds = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nn_resolve),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  (int)(CMAX * RSP * sizeof(float))) == hipSuccess;
  (void)big_lds;                     // > 64 KB of chunk minima per block (C > 963 chunks)
  hipLaunchKernelGGL(k_nn_resolve, dim3((unsigned)ceil_div(B, RS)), dim3(64 * RS), lds, st, qxy, B,
                     cx, cy, txy, count, p.chunk, maxabs, qmax, m32, out, dout);
}

void nn_delta(hipStream_t st, const int2* qxy, int64_t B, const double2* txy, const int64_t* snap_p,
              const int64_t* count, const int32_t* live, int64_t* near, double* dnear,
              int32_t* changed, int32_t* n_changed) {
  hipLaunchKernelGGL(k_nn_delta, dim3((unsigned)ceil_div(B, DS)), dim3(64 * DWV), 0, st, qxy, B, txy,
                     snap_p, count, live, near, dnear, changed, n_changed);
}

void nn_launch(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy,
               const double2* txy, const float4* t4, const int64_t* count, int64_t n_ub,
               const unsigned long long* maxabs, double qmax, float* m32, int64_t* out) {
  const NNPlan p = nn_plan(B, n_ub);
  nn_sweep(st, qxy, B, cx, cy, t4, count, p, m32);
  nn_resolve(st, qxy, B, cx, cy, txy, count, p, maxabs, qmax, m32, out, nullptr);
}

}  // namespace tr
