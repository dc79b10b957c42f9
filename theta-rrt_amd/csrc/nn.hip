// Nearest-node argmin (rrt.py:155-158 + search.py:13-15): for every sample j,
//   first index of min_i sqrt(fl(fl((qx - x_i)^2) + fl((qy - y_i)^2)))   in fp64, as np.argmin.
//
// Two kernels over node chunks (chunk = a contiguous index range of the tree):
//   k_nn_pass1   fp32 screen.  A node is screened as s_i = fma(ax, x^, fma(by, y^, w^)) with
//                (x^, y^) = fp32 of the node relative to the tree centre, w^ = fp32(x^2 + y^2),
//                (ax, by) = -2 (q - centre): s_i = |q - n_i|^2 - |q - centre|^2 up to rounding,
//                32 nodes x 32 samples per v_mfma_f32_32x32x2_f32.  Output: the minimum of s over
//                every (chunk, sample), m32[c * B + j] (coalesced stores).
//   k_nn_resolve RS samples per block (chunk minima staged through LDS): m = min_c m32, threshold thr = m + 2E + slack with E a rigorous
//                bound on |s_i - (d_i - |q^|^2)| (below); only chunks with a minimum <= thr are
//                rescanned, as (sample, chunk) pairs shared by the block's waves (exact fp64
//                distance over all their nodes, 8 independent 64-node pieces in flight per lane)
//                with the exact (sqrt class, first index) order of the reference.
// Bound (u = 2^-24, X = max |centred coordinate| over nodes and queries): representation 8uX^2,
// w^ 2uX^2, inner fma 4uX^2, outer fma 6uX^2: |s_i - (d_i - |q^|^2)| <= 20uX^2 (1 + O(u)); E uses
// 24uX^2.  Every node of the winning sqrt class then has s <= m + 2E + (|m| + |q^|^2 + E) 2^-48.
#pragma clang fp contract(off)
#include <stdlib.h>

#include "thetarrt_internal.hpp"
#include "diaglog.hpp"
TR_DLOG_EXPORT(tr_diag_log_nn)

namespace tr {

constexpr int CH_ALIGN = 64;  // chunk sizes are multiples of this

// Work unit (g, c): sample group g = [g*GS, +GS) against chunk c of the node range [lo, hi) (both
// read on the device: the tree grows there between launches).  The block stages the chunk (tiles
// of CHMAX nodes) into LDS; a grid of a few blocks per CU loops over the units.
constexpr int GS = 2048;         // samples per unit
constexpr int CHMAX = 1024;      // max chunk (nodes staged in LDS: 12 KB)

// ------------------------------------------------------------------ pass 1 on the matrix cores
// The screen of a 32-node x 32-sample tile is ONE v_mfma_f32_32x32x2_f32:
//   A = nodes   (row i = node, k0 = y^, k1 = x^),   lane l holds A[l & 31][l >> 5]
//   B = samples (col j = sample, k0 = by, k1 = ax),  lane l holds B[l >> 5][l & 31]
//   C = w^ of the row's node.
// gfx950's f32 MFMA is bit-for-bit the k-ordered fmaf chain D = fma(a1, b1, fma(a0, b0, C))
// (cdna_hip_programming.md, "FP32-input MFMA"), i.e. s = fma(ax, x^, fma(by, y^, w^)) exactly as the
// two-fmaf chain rounds it, which is what the error bound below is stated for.  D's column is the lane
// (j = l & 31) and its 16 registers are node rows (r & 3) + 8 (r >> 2) + 4 (l >> 5), so the minimum
// over nodes is a per-lane v_min3 tree; lanes l and l ^ 32 (the other 16 rows) merge once per unit.
// Per tile and wave: 64 MFMA cycles for 1024 pairs (the f32 matrix peak, 16 pairs/clk/SIMD) beside
// 8 v_min3 on the VALU (about 40 issue cycles, hidden in the MFMA's shadow).  The chunk is staged
// in LDS as three planes (y^, x^, w^): one ds_read_b32 for A and four ds_read_b128 for C per tile,
// shared by the wave's MT sample tiles.
constexpr int MT = 16;           // sample tiles (32 samples each) per wave: 4 waves x 16 x 32 = GS
constexpr int NW1 = GS / (32 * MT), NT1 = 64 * NW1;    // waves / threads per pass-1 block
static_assert(NW1 * 32 * MT == GS, "a unit's samples are the waves' tiles");
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

__global__ __launch_bounds__(NT1, NW1 / 2) void k_nn_pass1(const int2* __restrict__ qxy, int64_t B,
                                                  int32_t cx, int32_t cy,
                                                  const float4* __restrict__ t4,
                                                  const int64_t* __restrict__ lo_p,
                                                  const int64_t* __restrict__ hi_p, int64_t chunk,
                                                  const int32_t* __restrict__ nq_p,
                                                  float* __restrict__ m32) {
  __shared__ float py[CHMAX], px[CHMAX];
  __shared__ __attribute__((aligned(16))) float pw[CHMAX];
  TR_DLOG_T0;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, col = lane & 31, h = lane >> 5;
  // (the node counts are read past this XCD's L2, like every count a dedupe leaves behind)
  const int64_t lo = lo_p ? ld_sc1(lo_p) : 0;
  const int64_t hi = ld_sc1(hi_p);
  const int C = (int)((hi - lo + chunk - 1) / chunk);
  // the samples screened: all B, or the first *nq_p of them (a list filled on the device; m32
  // keeps its row stride B)
  const int64_t Bq = nq_p ? min(B, (int64_t)nq_p[0]) : B;
  const int ngrp = (int)((Bq + GS - 1) / GS);
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
      qa[s] = qxy[j < Bq ? j : Bq - 1];
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
      float4 v[CHMAX / NT1];
#pragma unroll
      for (int r = 0; r < CHMAX / NT1; ++r) {             // all staging loads in flight
        const int k = t + NT1 * r;
        if (k < n32) v[r] = t4[i0 + t0 + min(k, n - 1)];
      }
      __syncthreads();                                    // the previous tile is consumed
#pragma unroll
      for (int r = 0; r < CHMAX / NT1; ++r) {
        const int k = t + NT1 * r;
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
      if (h == 0 && j < Bq) out[j] = o;
    }
  }
  TR_DLOG(1);
}

// ------------------------------------------------------------------ resolve
// screen_E / screen_Eg: thetarrt_internal.hpp (the look-ahead correction uses them too).
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

// Block of RS waves = RS consecutive samples.  (1) The block stages the chunk minima of its samples
// (m32[c][j0 .. j0 + RS), 64 B row pieces, coalesced) into LDS; every wave takes its sample's
// minimum m and threshold and lists the chunks under it, in chunk order, in a block-wide list of
// (sample, chunk) pairs.  (2) All RS waves rescan the listed pairs round-robin: exact fp64 distance
// over the chunk's nodes (lanes over nodes, coalesced), the exact (sqrt class, first index) order.
// A sample with many candidate chunks (the clipped map-corner samples, where nodes pile up within
// 1e-6 px and the fp32 screen cannot separate them) is thus spread over the block
// instead of one wave setting the kernel's tail.  (3) Each wave reduces its own sample's pair
// results.  A block whose list exceeds the pair capacity rescans one wave per sample instead.
#ifndef TR_RS
#define TR_RS 8                  // samples (waves) per resolve block; build-time A/B knob
#endif
constexpr int RS = TR_RS;
constexpr int RSP = RS + 1;      // padded LDS row (column reads hit distinct banks)
constexpr int64_t CMAX = 2048;   // chunk count cap (LDS: CMAX * RSP * 4 B)
constexpr int RPAIR = 1024;      // (sample, chunk) pairs per block (LDS: 24 B results + 4 B entry)
#ifndef TR_RU
#define TR_RU 8                  // 64-node pieces in flight per lane; build-time A/B knob
#endif
constexpr int RU = TR_RU;

static size_t resolve_list_offset(int64_t cmax) {   // bytes: columns / pair results overlay, then list
  const size_t a = (size_t)cmax * RSP * sizeof(float), b = (size_t)RPAIR * 24;
  return ((a > b ? a : b) + 15) & ~(size_t)15;
}

// Exact scan of nodes [at, end) for query (qx, qy): per lane the smallest sqrt(d) (the reference's
// key, math.sqrt of the fp64 sum), its d and its first index -- lanes visit increasing indices, so a
// strict < keeps the first of equal keys.
__device__ __forceinline__ void scan_nodes(int64_t at, int64_t end, double qx, double qy,
                                           const double2* __restrict__ txy, double& rb, double& db,
                                           int64_t& ib) {
  const int lane = threadIdx.x & 63;
  for (int64_t b = at; b < end; b += 64 * RU) {
    int64_t ii[RU];
    double2 e[RU];
#pragma unroll
    for (int r = 0; r < RU; ++r) {
      const int64_t i = b + r * 64 + lane;
      ii[r] = i < end ? i : -1;
    }
#pragma unroll
    for (int r = 0; r < RU; ++r) e[r] = ii[r] >= 0 ? txy[ii[r]] : make_double2(INFINITY, INFINITY);
#pragma unroll
    for (int r = 0; r < RU; ++r) {
      const double a = qx - e[r].x, c = qy - e[r].y;
      const double d = a * a + c * c;
      if (ii[r] >= 0 && d < db) {          // d >= db: sqrt(d) >= rb at a later index
        const double rt = sqrt(d);
        if (rt < rb) { rb = rt; db = d; ib = ii[r]; }
      }
    }
  }
}

// Wave argmin of (key, index) with its d.
__device__ __forceinline__ void wave_best(double& rb, double& db, int64_t& ib) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ro = __shfl_xor(rb, off), dq = __shfl_xor(db, off);
    const int64_t io = __shfl_xor(ib, off);
    if (io >= 0 && (ib < 0 || ro < rb || (ro == rb && io < ib))) { rb = ro; db = dq; ib = io; }
  }
}

// Nearest node over the chunks of [0, *count) swept into m32 -> out[j] (its exact d -> dout[j]).
__global__ __launch_bounds__(64 * RS) void k_nn_resolve(const int2* __restrict__ qxy, int64_t B,
                                                        int32_t cx, int32_t cy,
                                                        const double2* __restrict__ txy,
                                                        const int64_t* __restrict__ count,
                                                        int64_t chunk,
                                                        const unsigned long long* __restrict__ maxabs,
                                                        double qmax, const float* __restrict__ m32,
                                                        int32_t list_off,
                                                        const int32_t* __restrict__ nq_p,
                                                        const int32_t* __restrict__ map,
                                                        int64_t* __restrict__ out,
                                                        double* __restrict__ dout, ResolvePub pub) {
  extern __shared__ __align__(16) unsigned char smraw[];
  __shared__ int s_cnt[RS];
  __shared__ int2 s_q[RS];
  float* sm = reinterpret_cast<float*>(smraw);
  int* plist = reinterpret_cast<int*>(smraw + list_off);
  TR_DLOG_T0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * RS;
  const int64_t N = ld_sc1(count);
  const int64_t C = (N + chunk - 1) / chunk;
  const int64_t j = j0 + w;
  // the samples resolved: all B, or the first *nq_p of them, sample j's result going to map[j]
  const int64_t Bq = nq_p ? min(B, (int64_t)nq_p[0]) : B;
  const bool act = j < Bq;
  const int64_t jq = j < Bq ? j : Bq - 1;
  const int2 qi = qxy[jq > 0 ? jq : 0];
  const double X = fmax(__longlong_as_double((long long)maxabs[0]), qmax) + 1.0;
  {
    // thread t stages column t % RS of rows t / RS + 64 k: all loads of a thread in flight at once
    constexpr int SU = 8;
    const int k = threadIdx.x % RS;
    const bool ok = j0 + k < Bq;
    for (int64_t c0 = threadIdx.x / RS; j0 < Bq && c0 < C; c0 += SU * 64) {   // (no sample: no work)
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
  const float* col = sm + w;
  const int nc = (int)C;
  float m = INFINITY;
#pragma unroll 4
  for (int c = lane; c < nc; c += 64) m = fminf(m, col[c * RSP]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fminf(m, __shfl_xor(m, off));
  const float thr = act ? screen_threshold(m, (double)(qi.x - cx), (double)(qi.y - cy), X) : -INFINITY;
  int n = 0;
  for (int cb = 0; cb < nc; cb += 64) {
    const int cl = cb + lane;
    n += __builtin_popcountll(__ballot(cl < nc && col[cl * RSP] <= thr));
  }
  if (lane == 0) { s_cnt[w] = n; s_q[w] = qi; }
  __syncthreads();
  int off = 0, total = 0;
#pragma unroll
  for (int q = 0; q < RS; ++q) {
    const int v = s_cnt[q];
    off += q < w ? v : 0;
    total += v;
  }
  double rb = INFINITY, db = INFINITY;
  int64_t ib = -1;
  if (total <= RPAIR) {                      // block-uniform
    int o = off;
    const unsigned long long lt = (1ull << lane) - 1;
    for (int cb = 0; cb < nc; cb += 64) {
      const int cl = cb + lane;
      const bool in = cl < nc && col[cl * RSP] <= thr;
      const unsigned long long mk = __ballot(in);
      if (in) plist[o + __builtin_popcountll(mk & lt)] = cl * RS + w;
      o += __builtin_popcountll(mk);
    }
    __syncthreads();                         // the columns are dead: results overlay them
    double* res_rt = reinterpret_cast<double*>(smraw);
    double* res_d = res_rt + RPAIR;
    int64_t* res_i = reinterpret_cast<int64_t*>(res_d + RPAIR);
    for (int p = w; p < total; p += RS) {
      const int e = plist[p], s = e % RS;
      const int64_t at = (int64_t)(e / RS) * chunk;
      const int2 q = s_q[s];
      double r1 = INFINITY, d1 = INFINITY;
      int64_t i1 = -1;
      scan_nodes(at, min(N, at + chunk), (double)q.x, (double)q.y, txy, r1, d1, i1);
      wave_best(r1, d1, i1);
      if (lane == 0) { res_rt[p] = r1; res_d[p] = d1; res_i[p] = i1; }
    }
    __syncthreads();
    for (int p = off + lane; p < off + n; p += 64) {
      const int64_t io = res_i[p];
      const double ro = res_rt[p];
      if (io >= 0 && (ib < 0 || ro < rb || (ro == rb && io < ib))) { rb = ro; db = res_d[p]; ib = io; }
    }
  } else {                                   // one wave per sample, its chunks in order
    for (int cb = 0; cb < nc; cb += 64) {
      const int cl = cb + lane;
      unsigned long long mk = __ballot(cl < nc && col[cl * RSP] <= thr);
      while (mk) {
        const int64_t at = (int64_t)(cb + __builtin_ctzll(mk)) * chunk;
        scan_nodes(at, min(N, at + chunk), (double)qi.x, (double)qi.y, txy, rb, db, ib);
        mk &= mk - 1;
      }
    }
  }
  wave_best(rb, db, ib);
  const int64_t jo = act && map ? (int64_t)map[j] : j;
  if (!pub.flag) {
    if (act && lane == 0) {
      out[jo] = ib;
      if (dout) dout[jo] = db;
    }
    TR_DLOG(2);
    return;
  }
  // publishing the look-ahead from here: the results travel in sc1 stores (read by another
  // stream's kernel before this one ends), every wave waits for them, the last block stores the
  // flag (thetarrt_internal.hpp: st_sc1)
  if (act && lane == 0) {
    st_sc1(out + jo, ib);
    if (dout) st_sc1(dout + jo, db);
  }
  wave_stores_done();
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(pub.blocks, 1) == (int32_t)gridDim.x - 1;
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    st_sc1(pub.blocks, 0);
    st_sc1(pub.flag, pub.v);
  }
  TR_DLOG(2);
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
constexpr int DU = 12;                    // delta nodes in flight per lane
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
  const int64_t lo = ld_sc1(snap_p), hi = ld_sc1(count);
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
    db[s] = act ? ld_sc1(dnear + j) : -1.0;  // inactive: no node can beat it (sc1: the resolve's)
    rb[s] = INFINITY;
    dl[s] = INFINITY;
    ib[s] = -1;
  }
  // each lane: indices i0 + u * 64 DWV, increasing; DU loads in flight per round (the delta of a
  // cfg2 batch, ~2.6k nodes, is one or two rounds: a serial load per node made it L2-latency bound)
  for (int64_t i0 = lo + w * 64 + lane; i0 < hi; i0 += 64 * DWV * DU) {
    double2 e[DU];
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * 64 * DWV;
      e[u] = i < hi ? txy[i] : make_double2(INFINITY, INFINITY);
    }
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * 64 * DWV;
#pragma unroll
      for (int s = 0; s < DS; ++s) {
        const double a = qx[s] - e[u].x, b = qy[s] - e[u].y;
        const double d = a * a + b * b;
        if (i < hi && d < db[s] && d < dl[s]) {   // d >= db: sqrt(d) >= the known key
          const double rt = sqrt(d);
          if (rt < rb[s]) { rb[s] = rt; dl[s] = d; ib[s] = i; }
        }
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
    if (k >= 0 && j < B && r < sqrt(ld_sc1(dnear + j))) {
      near[j] = k;
      dnear[j] = d;
      changed[atomicAdd(n_changed, 1)] = (int32_t)j;
    }
  }
}

// ------------------------------------------------------------------ host side
// Chunking of a sweep over up to N nodes for B samples: about `target` pass-1 units (sample
// groups x chunks) when the tree is large enough; chunks of at most maxch <= CHMAX nodes (staged in
// LDS in one tile; the resolve rescans whole chunks), a multiple of CH_ALIGN.
static int64_t nn_chunk_size(int64_t B, int64_t N, int64_t cmax) {
  constexpr int64_t target = 512, maxch = CHMAX;
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

// The largest nn_scratch of any plan for up to n_ub nodes: a plan has at most as many chunks as
// nn_chunk_size aimed for, and that number is not monotonic in the node count (the chunk size is
// rounded up to CH_ALIGN), so a buffer sized by the plan of the largest tree can be too small for a
// smaller one.
int64_t nn_scratch_ub(int64_t B, int64_t n_ub) {
  const int64_t groups = (B + GS - 1) / GS;
  const int64_t c = std::max<int64_t>(std::max<int64_t>(1, 512 / groups), ceil_div(std::max<int64_t>(n_ub, 1), CHMAX));
  return std::min<int64_t>(c, CMAX) * B;
}

void nn_sweep(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy, const float4* t4,
              const int64_t* hi_p, const NNPlan& p, float* m32, const int32_t* nq_p) {
  // a few blocks per CU loop over the (sample group, chunk) units; the kernel reads the actual
  // node count (the tree may have grown past the plan's bound: more units, same grid)
#ifndef TR_P1_CAP
#define TR_P1_CAP 512
#endif
  constexpr int64_t cap = TR_P1_CAP;
  const int64_t groups = ceil_div(B, GS);
  const int64_t g = std::max<int64_t>(1, std::min(groups * p.cmax, cap));
  hipLaunchKernelGGL(k_nn_pass1, dim3((unsigned)g), dim3(NT1), 0, st, qxy, B, cx, cy, t4,
                     (const int64_t*)nullptr, hi_p, p.chunk, nq_p, m32);
}

void nn_resolve(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy,
                const double2* txy, const int64_t* count, const NNPlan& p,
                const unsigned long long* maxabs, double qmax, const float* m32, int64_t* out,
                double* dout, ResolvePub pub, const int32_t* nq_p, const int32_t* map) {
  const size_t lo = resolve_list_offset(p.cmax), lds = lo + RPAIR * sizeof(int);
  static const bool big_lds = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nn_resolve),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  (int)(resolve_list_offset(CMAX) + RPAIR * sizeof(int))) == hipSuccess;
  (void)big_lds;                     // > 64 KB of chunk minima per block (C > 963 chunks)
  hipLaunchKernelGGL(k_nn_resolve, dim3((unsigned)ceil_div(B, RS)), dim3(64 * RS), lds, st, qxy, B,
                     cx, cy, txy, count, p.chunk, maxabs, qmax, m32, (int32_t)lo, nq_p, map, out, dout,
                     pub);
}

void nn_delta(hipStream_t st, const int2* qxy, int64_t B, const double2* txy, const int64_t* snap_p,
              const int64_t* count, const int32_t* live, int64_t* near, double* dnear,
              int32_t* changed, int32_t* n_changed) {
  hipLaunchKernelGGL(k_nn_delta, dim3((unsigned)ceil_div(B, DS)), dim3(64 * DWV), 0, st, qxy, B, txy,
                     snap_p, count, live, near, dnear, changed, n_changed);
}

void nn_launch(hipStream_t st, const int2* qxy, int64_t B, int32_t cx, int32_t cy,
               const double2* txy, const float4* t4, const int64_t* count, int64_t n_ub,
               const unsigned long long* maxabs, double qmax, float* m32, int64_t* out,
               double* dout) {
  const NNPlan p = nn_plan(B, n_ub);
  nn_sweep(st, qxy, B, cx, cy, t4, count, p, m32);
  nn_resolve(st, qxy, B, cx, cy, txy, count, p, maxabs, qmax, m32, out, dout);
}

}  // namespace tr
