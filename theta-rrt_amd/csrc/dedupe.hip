// Device side of the tree bookkeeping (rrt.py:151,179-188): exact-value pose dedupe and node-index
// assignment for a batch of records, and the append of the new nodes to the device tree.
//
// The reference appends records one by one:  qrand in G -> skip (rrt.py:151);  qnew not in G ->
// new vertex (rrt.py:179-180).  For a batch in sample order the same result is:
//   member[j] = sample pose j is a node of the snapshot            (device pose table lookup)
//   e[j]      = index of the snapshot node equal to qnew_j, or -1    (same table)
//   first[j]  = smallest record index with the same new pose        (batch table, atomicMin)
//   idx[j]    = e[j] >= 0 ? e[j] : N + rank(first[j]),  rank = prefix count of first occurrences
// New nodes are written to the device tree at N + rank and inserted into the pose table; the host
// replays the records in order (parents, edges, controls) without hashing (capi.hip).
#pragma clang fp contract(off)
#include "thetarrt_internal.hpp"

namespace tr {

__device__ __forceinline__ uint64_t pbits(double v) {
  return v == 0.0 ? 0ull : (uint64_t)__double_as_longlong(v);   // -0.0 == 0.0 (Python keys)
}
__device__ __forceinline__ uint64_t fmix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}
__device__ __forceinline__ uint64_t pose_hash(double x, double y, double t) {
  return fmix(pbits(x) ^ fmix(pbits(y) + 0x9E3779B97F4A7C15ull) ^ fmix(pbits(t) + 0x632BE59BD9B4E019ull));
}
__device__ __forceinline__ bool pose_eq(double ax, double ay, double at, double bx, double by,
                                        double bt) {
  return pbits(ax) == pbits(bx) && pbits(ay) == pbits(by) && pbits(at) == pbits(bt);
}

// Node table lookup: slot -> node index (-1 empty); keys are the device tree's poses.
__device__ __forceinline__ int32_t node_lookup(const int32_t* __restrict__ tab, uint64_t mask,
                                               const double2* __restrict__ txy,
                                               const double* __restrict__ tth, double x, double y,
                                               double t) {
  for (uint64_t p = pose_hash(x, y, t) & mask;; p = (p + 1) & mask) {
    const int32_t v = tab[p];
    if (v < 0) return -1;
    const double2 n = txy[v];
    if (pose_eq(n.x, n.y, tth[v], x, y, t)) return v;
  }
}

__device__ __forceinline__ void node_insert(int32_t* tab, uint64_t mask, double x, double y,
                                            double t, int32_t v) {
  for (uint64_t p = pose_hash(x, y, t) & mask;; p = (p + 1) & mask)
    if (atomicCAS(&tab[p], -1, v) == -1) return;
}

__device__ __forceinline__ bool accepted(const tr_record& r) { return r.status == TR_ST_OK; }

// Batch table: 64-bit slots (epoch << 32 | record index); a slot of another epoch is empty, so the
// table never needs clearing between batches (epoch = batch counter, never 0).
__device__ __forceinline__ bool slot_live(unsigned long long v, unsigned long long ep) {
  return (v >> 32) == ep;
}

// 1: membership of the sample, snapshot lookup of qnew, batch-table claim of new poses.
__global__ __launch_bounds__(256) void k_dd_lookup(const tr_sample* __restrict__ smp,
                                                   const tr_record* __restrict__ rec, int64_t n,
                                                   const int32_t* __restrict__ htab, uint64_t hmask,
                                                   const double2* __restrict__ txy,
                                                   const double* __restrict__ tth,
                                                   unsigned long long* __restrict__ btab,
                                                   uint64_t bmask, unsigned long long ep,
                                                   int32_t* __restrict__ e,
                                                   int32_t* __restrict__ fl) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const tr_record r = rec[j];
  int32_t f = 0, ex = -1;
  if (r.status != TR_ST_SKIP && r.status != TR_ST_INDEX) {
    const tr_sample s = smp[j];
    if (node_lookup(htab, hmask, txy, tth, (double)s.x, (double)s.y, s.th) >= 0) f |= TR_CI_MEMBER;
  }
  if (!(f & TR_CI_MEMBER) && accepted(r)) {
    const double2 q = txy[r.near];
    if (pose_eq(r.x, r.y, r.th, q.x, q.y, tth[r.near])) f |= TR_CI_SAME_NEAR;
    ex = node_lookup(htab, hmask, txy, tth, r.x, r.y, r.th);
    if (ex < 0) {                                // claim the pose in the batch table
      const unsigned long long mine = (ep << 32) | (unsigned long long)j;
      for (uint64_t p = pose_hash(r.x, r.y, r.th) & bmask;; p = (p + 1) & bmask) {
        unsigned long long v = btab[p];
        if (!slot_live(v, ep)) {
          const unsigned long long old = atomicCAS(&btab[p], v, mine);
          if (old == v) break;                   // claimed
          v = old;
          if (!slot_live(v, ep)) { p = (p - 1) & bmask; continue; }   // raced to a stale value: retry
        }
        const tr_record o = rec[(int64_t)(v & 0xffffffffull)];
        if (pose_eq(o.x, o.y, o.th, r.x, r.y, r.th)) {
          atomicMin(&btab[p], mine);
          break;
        }
      }
    }
  }
  e[j] = ex;
  fl[j] = f;
}

// 2: first occurrence of each new pose in the batch.
__global__ __launch_bounds__(256) void k_dd_first(const tr_record* __restrict__ rec, int64_t n,
                                                  const unsigned long long* __restrict__ btab,
                                                  uint64_t bmask, unsigned long long ep,
                                                  const int32_t* __restrict__ e,
                                                  int32_t* __restrict__ fl,
                                                  int32_t* __restrict__ first,
                                                  int32_t* __restrict__ isfirst) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const tr_record r = rec[j];
  int32_t f0 = -1, is = 0;
  if (!(fl[j] & TR_CI_MEMBER) && accepted(r) && e[j] < 0) {
    for (uint64_t p = pose_hash(r.x, r.y, r.th) & bmask;; p = (p + 1) & bmask) {
      const unsigned long long v = btab[p];
      const int32_t k = (int32_t)(v & 0xffffffffull);
      const tr_record o = rec[k];
      if (slot_live(v, ep) && pose_eq(o.x, o.y, o.th, r.x, r.y, r.th)) {
        f0 = k;
        break;
      }
    }
    is = f0 == (int32_t)j;
    if (is) fl[j] |= TR_CI_FIRST;
  }
  first[j] = f0;
  isfirst[j] = is;
}

// 3: exclusive prefix count of first occurrences (one block), then count += total (and a copy of
// the new count in this batch's snapshot slot).
constexpr int SCAN_T = 1024, SCAN_I = 4;
__global__ __launch_bounds__(SCAN_T) void k_dd_scan(const int32_t* __restrict__ a, int64_t n,
                                                    int32_t* __restrict__ rank,
                                                    int64_t* __restrict__ count,
                                                    int64_t* __restrict__ base,
                                                    int64_t* __restrict__ snap) {
  __shared__ int32_t sh[SCAN_T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t carry = 0;
  for (int64_t t0 = 0; t0 < n; t0 += SCAN_T * SCAN_I) {
    const int64_t b0 = t0 + (int64_t)threadIdx.x * SCAN_I;
    int32_t v[SCAN_I], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
      v[k] = b0 + k < n ? a[b0 + k] : 0;
      s += v[k];
    }
    int32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int32_t off = 0, tot = 0;
    for (int k = 0; k < SCAN_T / 64; ++k) {
      if (k < w) off += sh[k];
      tot += sh[k];
    }
    __syncthreads();
    int32_t run = carry + off + x - s;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
      if (b0 + k < n) rank[b0 + k] = run;
      run += v[k];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) {
    const int64_t N = count[0];
    base[0] = N;
    count[0] = N + carry;
    snap[0] = N + carry;     // the tree a staged NN sweep of a later batch covers
  }
}

// 4: final node index per record, append of the first occurrences to the device tree, and the
// commit record written straight into pinned host memory (zero-copy) for the host replay.
__global__ __launch_bounds__(256) void k_dd_assign(const tr_record* __restrict__ rec, int64_t n,
                                                   const int32_t* __restrict__ e,
                                                   const int32_t* __restrict__ fl,
                                                   const int32_t* __restrict__ first,
                                                   const int32_t* __restrict__ rank,
                                                   const int64_t* __restrict__ base,
                                                   double2* __restrict__ txy, float4* __restrict__ t4,
                                                   double* __restrict__ tth, int32_t* htab,
                                                   uint64_t hmask, unsigned long long* maxabs,
                                                   int32_t cx, int32_t cy,
                                                   tr_commit_rec* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int64_t N = base[0];
  const int32_t f = fl[j];
  int64_t idx = -1;
  const tr_record r = rec[j];
  if (!(f & TR_CI_MEMBER) && accepted(r)) {
    idx = e[j] >= 0 ? (int64_t)e[j] : N + rank[first[j]];
    if (f & TR_CI_FIRST) {
      txy[idx] = make_double2(r.x, r.y);
      t4[idx] = screen_node(r.x, r.y, cx, cy);
      tth[idx] = r.th;
      node_insert(htab, hmask, r.x, r.y, r.th, (int32_t)idx);
      const double m = centred_abs(r.x, r.y, cx, cy);
      atomicMax(maxabs, (unsigned long long)__double_as_longlong(m));   // m >= 0: bits order
    }
  }
  tr_commit_rec o;
  o.r = r;
  o.idx = idx;
  o.flags = f;
  o.pad = 0;
  out[j] = o;
}

// Insert nodes [0, N) into a fresh table (tree reset / table growth); poses are unique.
__global__ __launch_bounds__(256) void k_dd_rebuild(const double2* __restrict__ txy,
                                                    const double* __restrict__ tth, int64_t N,
                                                    int32_t* htab, uint64_t hmask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const double2 p = txy[i];
  node_insert(htab, hmask, p.x, p.y, tth[i], (int32_t)i);
}

// ------------------------------------------------------------------ host side
void dd_batch(hipStream_t st, const DDState& d, const tr_sample* smp, const tr_record* rec, int64_t n,
              double2* txy, float4* t4, double* tth, tr_commit_rec* out) {
  const unsigned g = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_dd_lookup, dim3(g), dim3(256), 0, st, smp, rec, n, d.htab, d.hmask, txy, tth,
                     d.btab, d.bmask, d.epoch, d.e, d.fl);
  hipLaunchKernelGGL(k_dd_first, dim3(g), dim3(256), 0, st, rec, n, d.btab, d.bmask, d.epoch, d.e,
                     d.fl, d.first, d.isfirst);
  hipLaunchKernelGGL(k_dd_scan, dim3(1), dim3(SCAN_T), 0, st, d.isfirst, n, d.rank, d.count, d.base,
                     d.snap);
  hipLaunchKernelGGL(k_dd_assign, dim3(g), dim3(256), 0, st, rec, n, d.e, d.fl, d.first, d.rank,
                     d.base, txy, t4, tth, d.htab, d.hmask, d.maxabs, d.cx, d.cy, out);
}

void dd_rebuild(hipStream_t st, const DDState& d, const double2* txy, const double* tth, int64_t N) {
  (void)hipMemsetAsync(d.htab, 0xff, sizeof(int32_t) * (d.hmask + 1), st);
  if (N > 0)
    hipLaunchKernelGGL(k_dd_rebuild, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, txy, tth, N,
                       d.htab, d.hmask);
}

}  // namespace tr
