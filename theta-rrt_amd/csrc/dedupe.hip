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

__device__ __forceinline__ void node_insert(PoseSlot* tab, uint64_t mask, double x, double y,
                                            double t, int32_t v, int32_t* err) {
  uint64_t p = pose_hash(x, y, t) & mask;
  for (uint64_t it = 0; it <= mask; ++it, p = (p + 1) & mask)
    if (atomicCAS(&tab[p].idx, -1, v) == -1) {
      tab[p].x = x;
      tab[p].y = y;
      tab[p].th = t;
      return;
    }
  atomicOr(err, TR_DDE_INSERT);
}


// Batch table: 64-bit slots (epoch << 32 | record index); a slot of another epoch is empty, so the
// table never needs clearing between batches (epoch = batch counter, never 0).
__device__ __forceinline__ bool slot_live(unsigned long long v, unsigned long long ep) {
  return (v >> 32) == ep;
}

// 1: membership of the sample, snapshot lookup of qnew, batch-table claim of new poses.
__device__ __forceinline__ void dd_lookup_one(const tr_sample* __restrict__ smp,
                                              const tr_record* __restrict__ rec, int64_t j,
                                              const PoseSlot* __restrict__ htab, uint64_t hmask,
                                              const double2* __restrict__ txy,
                                              const double* __restrict__ tth,
                                              unsigned long long* __restrict__ btab, uint64_t bmask,
                                              unsigned long long ep, int32_t& ex_out,
                                              int32_t& f_out, int32_t* err) {
  const tr_record r = rec[j];
  int32_t f = 0, ex = -1;
  snapshot_lookup(smp[j], r, htab, hmask, txy, tth, ex, f, err);
  if (!(f & TR_CI_MEMBER) && accepted(r)) {
    if (ex < 0) {                                // claim the pose in the batch table
      const unsigned long long mine = (ep << 32) | (unsigned long long)j;
      uint64_t p = pose_hash(r.x, r.y, r.th) & bmask;
      uint64_t it = 0;
      for (; it <= 2 * bmask + 1; ++it) {
        unsigned long long v = btab[p];
        if (!slot_live(v, ep)) {
          const unsigned long long old = atomicCAS(&btab[p], v, mine);
          if (old == v) break;                   // claimed
          v = old;
          if (!slot_live(v, ep)) continue;       // raced to a stale value: retry the slot
        }
        const tr_record o = rec[(int64_t)(v & 0xffffffffull)];
        if (pose_eq(o.x, o.y, o.th, r.x, r.y, r.th)) {
          atomicMin(&btab[p], mine);
          break;
        }
        p = (p + 1) & bmask;
      }
      if (it > 2 * bmask + 1) atomicOr(err, TR_DDE_CLAIM);
    }
  }
  ex_out = ex;
  f_out = f;
}

__global__ __launch_bounds__(256) void k_dd_lookup(const tr_sample* __restrict__ smp,
                                                   const tr_record* __restrict__ rec, int64_t n,
                                                   const PoseSlot* __restrict__ htab, uint64_t hmask,
                                                   const double2* __restrict__ txy,
                                                   const double* __restrict__ tth,
                                                   unsigned long long* __restrict__ btab,
                                                   uint64_t bmask, unsigned long long ep,
                                                   int32_t* __restrict__ e,
                                                   int32_t* __restrict__ fl,
                                                   int32_t* __restrict__ err) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  int32_t ex, f;
  dd_lookup_one(smp, rec, j, htab, hmask, txy, tth, btab, bmask, ep, ex, f, err);
  e[j] = ex;
  fl[j] = f;
}

// 2: first occurrence of each new pose (the batch-table claim of step 1 holds the smallest record
// index), its rank among the block's first occurrences, and the block's count.  Block 0 also
// keeps the node count before the batch.  No block waits for another: the ranks across blocks
// are resolved in step 3, after this kernel.
constexpr int FT = 256;
__global__ __launch_bounds__(FT) void k_dd_first(const tr_record* __restrict__ rec, int64_t n,
                                                 const unsigned long long* __restrict__ btab,
                                                 uint64_t bmask, unsigned long long ep,
                                                 const int32_t* __restrict__ e,
                                                 int32_t* __restrict__ fl,
                                                 int32_t* __restrict__ first,
                                                 int32_t* __restrict__ lrank,
                                                 int32_t* __restrict__ bcount,
                                                 const int64_t* __restrict__ count,
                                                 int64_t* __restrict__ base,
                                                 int32_t* __restrict__ err) {
  __shared__ int32_t s_wsum[FT / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t j = (int64_t)blockIdx.x * FT + t;
  if (j == 0) base[0] = count[0];
  int32_t f0 = -1, is = 0;
  if (j < n) {
    const tr_record& r = rec[j];
    const int32_t f = fl[j];
    if (!(f & TR_CI_MEMBER) && accepted(r) && e[j] < 0) {
      uint64_t p = pose_hash(r.x, r.y, r.th) & bmask;
      for (uint64_t it = 0; it <= bmask; ++it, p = (p + 1) & bmask) {
        const unsigned long long v = btab[p];
        const int32_t k = (int32_t)(v & 0xffffffffull);
        if (slot_live(v, ep)) {
          const tr_record& o = rec[k];
          if (pose_eq(o.x, o.y, o.th, r.x, r.y, r.th)) { f0 = k; break; }
        }
      }
      if (f0 < 0) atomicOr(err, TR_DDE_FIRST);
      is = f0 == (int32_t)j;
      if (is) fl[j] = f | TR_CI_FIRST;
    }
    first[j] = f0;
  }
  int32_t x = is;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wsum[w] = x;
  __syncthreads();
  int32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < FT / 64; ++k) {
    if (k < w) off += s_wsum[k];
    tot += s_wsum[k];
  }
  if (is) lrank[j] = off + x - 1;
  if (t == 0) bcount[blockIdx.x] = tot;
}

// 3: node index (N + first occurrences of earlier blocks + rank in the block), the append of the
// first occurrences to the device tree and the pose table, and the commit record written straight
// into pinned host memory (zero-copy) for the host replay.  Block 0 updates the node count.
__global__ __launch_bounds__(FT) void k_dd_assign(const tr_record* __restrict__ rec, int64_t n,
                                                  const int32_t* __restrict__ e,
                                                  const int32_t* __restrict__ fl,
                                                  const int32_t* __restrict__ first,
                                                  const int32_t* __restrict__ lrank,
                                                  const int32_t* __restrict__ bcount,
                                                  const int64_t* __restrict__ base,
                                                  int64_t* __restrict__ count,
                                                  int64_t* __restrict__ snap,
                                                  double2* __restrict__ txy, float4* __restrict__ t4,
                                                  double* __restrict__ tth, PoseSlot* htab,
                                                  uint64_t hmask, unsigned long long* maxabs,
                                                  int32_t cx, int32_t cy,
                                                  int32_t* __restrict__ err,
                                                  tr_commit_rec* __restrict__ out) {
  __shared__ int32_t s_pre[2];
  const int t = threadIdx.x, lane = t & 63;
  const int nblk = (int)((n + FT - 1) / FT);
  const int bid = (int)blockIdx.x;
  // prefix of the block counts before this block, and the total (block 0 updates the count)
  int32_t pre = 0, tot = 0;
  for (int q = t; q < nblk; q += FT) {
    const int32_t v = bcount[q];
    if (q < bid) pre += v;
    tot += v;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    pre += __shfl_xor(pre, o);
    tot += __shfl_xor(tot, o);
  }
  if (t == 0) s_pre[0] = s_pre[1] = 0;
  __syncthreads();
  if (lane == 0) {
    atomicAdd(&s_pre[0], pre);
    atomicAdd(&s_pre[1], tot);
  }
  __syncthreads();
  const int64_t N = base[0];
  if (bid == 0 && t == 0) {
    count[0] = N + s_pre[1];
    snap[0] = N + s_pre[1];     // the tree a look-ahead of a later batch covers
  }
  const int64_t j = (int64_t)bid * FT + t;
  double mx = 0.0;
  if (j < n) {
    const int32_t f = fl[j];
    int64_t idx = -1;
    const tr_record r = rec[j];
    if (!(f & TR_CI_MEMBER) && accepted(r)) {
      if (e[j] >= 0) {
        idx = e[j];
      } else {
        const int32_t f0 = first[j];
        int64_t pf = s_pre[0];                   // first occurrence in this block ...
        if (f0 / FT != bid) {                    // ... or an earlier one: its block's prefix
          pf = 0;
          for (int q = 0; q < f0 / FT; ++q) pf += bcount[q];
        }
        idx = N + pf + lrank[f0];
      }
      if (f & TR_CI_FIRST) {
        txy[idx] = make_double2(r.x, r.y);
        t4[idx] = screen_node(r.x, r.y, cx, cy);
        tth[idx] = r.th;
        node_insert(htab, hmask, r.x, r.y, r.th, (int32_t)idx, err);
        mx = centred_abs(r.x, r.y, cx, cy);
      }
    }
    tr_commit_rec o;
    o.r = r;
    o.idx = idx;
    o.flags = f;
    o.pad = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // TR_DDE_*
    out[j] = o;
  }
  // one atomic per wave (m >= 0: the bits order like the values)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if (lane == 0 && mx > 0.0) atomicMax(maxabs, (unsigned long long)__double_as_longlong(mx));
}

// Insert nodes [0, N) into a fresh table (tree reset / table growth); poses are unique.
__global__ __launch_bounds__(256) void k_dd_rebuild(const double2* __restrict__ txy,
                                                    const double* __restrict__ tth, int64_t N,
                                                    PoseSlot* htab, uint64_t hmask,
                                                    int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const double2 p = txy[i];
  node_insert(htab, hmask, p.x, p.y, tth[i], (int32_t)i, err);
}

// ------------------------------------------------------------------ host side
void dd_batch(hipStream_t st, const DDState& d, const tr_sample* smp, const tr_record* rec, int64_t n,
              double2* txy, float4* t4, double* tth, tr_commit_rec* out) {
  const unsigned g = (unsigned)((n + FT - 1) / FT);
  hipLaunchKernelGGL(k_dd_lookup, dim3(g), dim3(256), 0, st, smp, rec, n, d.htab, d.hmask, txy, tth,
                     d.btab, d.bmask, d.epoch, d.e, d.fl, d.err);
  hipLaunchKernelGGL(k_dd_first, dim3(g), dim3(FT), 0, st, rec, n, d.btab, d.bmask, d.epoch, d.e,
                     d.fl, d.first, d.lrank, d.bcount, d.count, d.base, d.err);
  hipLaunchKernelGGL(k_dd_assign, dim3(g), dim3(FT), 0, st, rec, n, d.e, d.fl, d.first, d.lrank,
                     d.bcount, d.base, d.count, d.snap, txy, t4, tth, d.htab, d.hmask, d.maxabs,
                     d.cx, d.cy, d.err, out);
}

void dd_rebuild(hipStream_t st, const DDState& d, const double2* txy, const double* tth, int64_t N) {
  (void)hipMemsetAsync(d.htab, 0xff, sizeof(PoseSlot) * (d.hmask + 1), st);
  if (N > 0)
    hipLaunchKernelGGL(k_dd_rebuild, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, txy, tth, N,
                       d.htab, d.hmask, d.err);
}

}  // namespace tr
