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

// Pose table: open addressing over PoseSlot {x, y, th, idx} (idx -1 = empty), keys in the slot so
// a probe is one 32-byte load.  Inserts claim a slot by CAS on idx, then write the key: lookups and
// inserts run in different kernels (the tree grows only in k_dd_assign / k_dd_tail).
__device__ __forceinline__ int32_t node_lookup(const PoseSlot* __restrict__ tab, uint64_t mask,
                                               double x, double y, double t) {
  for (uint64_t p = pose_hash(x, y, t) & mask;; p = (p + 1) & mask) {
    const PoseSlot v = tab[p];
    if (v.idx < 0) return -1;
    if (pose_eq(v.x, v.y, v.th, x, y, t)) return v.idx;
  }
}

// Lookup continuing from an already loaded first slot (the first probes of independent lookups
// are issued together).
__device__ __forceinline__ int32_t node_lookup_from(const PoseSlot* __restrict__ tab, uint64_t mask,
                                                    uint64_t p, PoseSlot v, double x, double y,
                                                    double t) {
  for (;;) {
    if (v.idx < 0) return -1;
    if (pose_eq(v.x, v.y, v.th, x, y, t)) return v.idx;
    p = (p + 1) & mask;
    v = tab[p];
  }
}

__device__ __forceinline__ void node_insert(PoseSlot* tab, uint64_t mask, double x, double y,
                                            double t, int32_t v) {
  for (uint64_t p = pose_hash(x, y, t) & mask;; p = (p + 1) & mask)
    if (atomicCAS(&tab[p].idx, -1, v) == -1) {
      tab[p].x = x;
      tab[p].y = y;
      tab[p].th = t;
      return;
    }
}

__device__ __forceinline__ bool accepted(const tr_record& r) { return r.status == TR_ST_OK; }

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
                                              int32_t& f_out) {
  const tr_record r = rec[j];
  const tr_sample s = smp[j];
  const bool look_s = r.status != TR_ST_SKIP && r.status != TR_ST_INDEX;
  const bool acc = accepted(r);
  // first probes of both lookups and qnear's pose, all in flight together
  const double sx = (double)s.x, sy = (double)s.y;
  const uint64_t ps = pose_hash(sx, sy, s.th) & hmask, pq = pose_hash(r.x, r.y, r.th) & hmask;
  PoseSlot vs, vq;
  vs.idx = vq.idx = -1;
  double2 q = make_double2(0.0, 0.0);
  double qt = 0.0;
  if (look_s) vs = htab[ps];
  if (acc) {
    vq = htab[pq];
    q = txy[r.near];
    qt = tth[r.near];
  }
  int32_t f = 0, ex = -1;
  if (look_s && node_lookup_from(htab, hmask, ps, vs, sx, sy, s.th) >= 0) f |= TR_CI_MEMBER;
  if (!(f & TR_CI_MEMBER) && acc) {
    if (pose_eq(r.x, r.y, r.th, q.x, q.y, qt)) f |= TR_CI_SAME_NEAR;
    ex = node_lookup_from(htab, hmask, pq, vq, r.x, r.y, r.th);
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
                                                   unsigned int* __restrict__ ticket) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j == 0) ticket[0] = 0;                   // block tickets of k_dd_final
  if (j >= n) return;
  int32_t ex, f;
  dd_lookup_one(smp, rec, j, htab, hmask, txy, tth, btab, bmask, ep, ex, f);
  e[j] = ex;
  fl[j] = f;
}

// 2: one pass over the batch in blocks of 256 records taken in ticket order: first occurrence of
// each new pose (the batch-table claim of step 1 holds the smallest record index), the block's
// prefix count of first occurrences chained across blocks (decoupled look-back: every block
// publishes its count tagged with the batch epoch, a block sums the counts of the blocks before
// it), node index, append of the first occurrences to the device tree and the pose table, and the
// commit record written straight into pinned host memory (zero-copy) for the host replay.
constexpr int FT = 256;
__global__ __launch_bounds__(FT) void k_dd_final(const tr_record* __restrict__ rec, int64_t n,
                                                 const unsigned long long* __restrict__ btab,
                                                 uint64_t bmask, unsigned long long ep,
                                                 const int32_t* __restrict__ e,
                                                 const int32_t* __restrict__ fl_in,
                                                 unsigned int* __restrict__ ticket,
                                                 unsigned long long* __restrict__ agg,
                                                 unsigned long long* __restrict__ fidx,
                                                 int64_t* __restrict__ count,
                                                 int64_t* __restrict__ base,
                                                 int64_t* __restrict__ snap,
                                                 double2* __restrict__ txy, float4* __restrict__ t4,
                                                 double* __restrict__ tth, PoseSlot* htab,
                                                 uint64_t hmask, unsigned long long* maxabs,
                                                 int32_t cx, int32_t cy,
                                                 tr_commit_rec* __restrict__ out) {
  __shared__ unsigned int s_bid;
  __shared__ int32_t s_wsum[FT / 64];
  __shared__ int64_t s_prefix;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t N = count[0];                  // read before the ticket: the last block updates it
  if (t == 0) s_bid = atomicAdd(ticket, 1u);
  __syncthreads();
  const unsigned int bid = s_bid;
  const unsigned int nblk = (unsigned int)((n + FT - 1) / FT);
  const int64_t j = (int64_t)bid * FT + t;
  // first occurrence
  int32_t f = 0, f0 = -1;
  tr_record r;
  if (j < n) {
    r = rec[j];
    f = fl_in[j];
    if (!(f & TR_CI_MEMBER) && accepted(r) && e[j] < 0) {
      for (uint64_t p = pose_hash(r.x, r.y, r.th) & bmask;; p = (p + 1) & bmask) {
        const unsigned long long v = btab[p];
        const int32_t k = (int32_t)(v & 0xffffffffull);
        if (slot_live(v, ep)) {
          const tr_record& o = rec[k];
          if (pose_eq(o.x, o.y, o.th, r.x, r.y, r.th)) { f0 = k; break; }
        }
      }
      if (f0 == (int32_t)j) f |= TR_CI_FIRST;
    }
  }
  const int32_t is = (f & TR_CI_FIRST) ? 1 : 0;
  // block scan
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
  // publish this block's count, then sum the counts of the blocks before it
  if (t == 0)
    __hip_atomic_store(&agg[bid], (ep << 32) | (unsigned long long)(uint32_t)tot, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
  // Waits are bounded: a block only waits for blocks with earlier tickets, which are running and
  // publish before they wait themselves, so the bound is never reached in a correct run; if it is,
  // the records are flagged and the host replay fails instead of the GPU hanging.
  constexpr int SPIN = 1 << 22;
  bool stuck = false;
  int64_t pre = 0;
  for (unsigned int q = t; q < bid; q += FT) {
    unsigned long long v;
    int it = 0;
    do {
      v = __hip_atomic_load(&agg[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    } while ((v >> 32) != ep && ++it < SPIN);
    stuck |= it >= SPIN;
    pre += (int64_t)(v & 0xffffffffull);
  }
  stuck = __any(stuck);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o);
  if (t == 0) s_prefix = 0;
  __syncthreads();
  if (lane == 0 && pre) atomicAdd((unsigned long long*)&s_prefix, (unsigned long long)pre);
  __syncthreads();
  const int64_t prefix = s_prefix;
  double mx = 0.0;
  int64_t idx = -1;
  if (j < n && !(f & TR_CI_MEMBER) && accepted(r)) {
    if (e[j] >= 0) {
      idx = e[j];
    } else if (f & TR_CI_FIRST) {
      const int64_t rank = prefix + (off + x - is);
      idx = N + rank;
      __hip_atomic_store(&fidx[j], (ep << 32) | (unsigned long long)rank, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
      txy[idx] = make_double2(r.x, r.y);
      t4[idx] = screen_node(r.x, r.y, cx, cy);
      tth[idx] = r.th;
      node_insert(htab, hmask, r.x, r.y, r.th, (int32_t)idx);
      mx = centred_abs(r.x, r.y, cx, cy);
    }
  }
  __syncthreads();
  // a later duplicate of a new pose: the node its first record got (that record is in this block
  // or an earlier one, whose rank depends only on blocks before it)
  if (j < n && idx < 0 && f0 >= 0) {
    unsigned long long v;
    int it = 0;
    do {
      v = __hip_atomic_load(&fidx[f0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    } while ((v >> 32) != ep && ++it < SPIN);
    stuck |= it >= SPIN;
    idx = N + (int64_t)(v & 0xffffffffull);
  }
  if (j < n) {
    tr_commit_rec o;
    o.r = r;
    o.idx = idx;
    o.flags = f | (stuck ? TR_CI_FAILED : 0);
    o.pad = 0;
    out[j] = o;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if (lane == 0 && mx > 0.0) atomicMax(maxabs, (unsigned long long)__double_as_longlong(mx));
  if (bid == nblk - 1 && t == 0) {             // every earlier block has published: total known
    base[0] = N;
    count[0] = N + prefix + tot;
    snap[0] = N + prefix + tot;
  }
}

// Insert nodes [0, N) into a fresh table (tree reset / table growth); poses are unique.
__global__ __launch_bounds__(256) void k_dd_rebuild(const double2* __restrict__ txy,
                                                    const double* __restrict__ tth, int64_t N,
                                                    PoseSlot* htab, uint64_t hmask) {
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
                     d.btab, d.bmask, d.epoch, d.e, d.fl, d.ticket);
  hipLaunchKernelGGL(k_dd_final, dim3((unsigned)((n + FT - 1) / FT)), dim3(FT), 0, st, rec, n, d.btab,
                     d.bmask, d.epoch, d.e, d.fl, d.ticket, d.agg, d.fidx, d.count, d.base, d.snap,
                     txy, t4, tth, d.htab, d.hmask, d.maxabs, d.cx, d.cy, out);
}

void dd_rebuild(hipStream_t st, const DDState& d, const double2* txy, const double* tth, int64_t N) {
  (void)hipMemsetAsync(d.htab, 0xff, sizeof(PoseSlot) * (d.hmask + 1), st);
  if (N > 0)
    hipLaunchKernelGGL(k_dd_rebuild, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, txy, tth, N,
                       d.htab, d.hmask);
}

}  // namespace tr
