// Device side of the tree bookkeeping (rrt.py:151,179-188): exact-value pose dedupe, node-index
// assignment and the append of the new nodes to the device tree, for one batch of records in
// sample order, plus the compact delta the host book replays.
//
// The reference appends records one by one:  qrand in G -> skip (rrt.py:151);  qnew not in G ->
// new vertex (rrt.py:179-180);  G[qnear].append(qnew) (rrt.py:181-185);  cameFrom[qnew] =
// (qnear, u) unless qnew == qnear (rrt.py:187-188).  For a batch in sample order the result is:
//   member[j], same_near[j], ex[j] = the snapshot lookups, done by the expansion (k_expand_arc)
//   accepted[j] = status OK and not member
//   first[j] / last[j] = smallest / largest record index with the same new pose (ex < 0)
//   idx[j]    = ex[j] >= 0 ? ex[j] : N + rank(first[j]),  rank = prefix count of first occurrences
//   edges     = (near, idx) of every accepted record, in order
//   new node  = pose of its first record, cameFrom from its LAST record (later ones overwrite)
//   updates   = (idx, near, u) of accepted records re-reaching a snapshot node, qnew != qnear
// A batch with a goal, an error or a record the reference raises on (TR_ST_INDEX / TR_ST_STRAIGHT)
// is `special`: the host replays its full resolved records in order instead (it stops there).
//
// Three kernels: k_dd_claim (the new poses in an epoch-tagged batch table, first record by
// atomicMin, last by atomicMax), k_dd_count (first occurrences, block-local ranks) and k_dd_emit
// (indices, tree append, the delta), written straight into pinned host memory by every block.
// (Claiming at the tail of k_expand_arc instead was measured slower: +31 us there against 16 us
// for the separate kernel, profiles/r02/.)
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

__device__ __forceinline__ bool rec_upd(const tr_record& r) {
  return rec_accepted(r) && r.ex >= 0 && !(r.flags & TR_FL_SAME_NEAR);
}

// cameFrom control u6 (steer, iccx, iccy, rad, dist; straight: ICC and rad unset -> 0)
__device__ __forceinline__ void rec_u(const tr_record& r, double* u, int32_t& straight) {
  straight = (r.flags & TR_FL_STRAIGHT) ? 1 : 0;
  u[0] = r.steer;
  u[1] = straight ? 0.0 : r.iccx;
  u[2] = straight ? 0.0 : r.iccy;
  u[3] = straight ? 0.0 : r.rad;
  u[4] = r.dist;
}

// Outputs of one record once its index and ranks are known (both paths).
__device__ __forceinline__ void dd_emit(const DDArgs& a, int64_t j, const tr_record& r, int64_t idx,
                                        bool first, int64_t node_rank, int64_t edge_rank,
                                        int64_t upd_rank, bool special, double& mx) {
  if (rec_accepted(r)) {
    a.out.edges[edge_rank] = DEdge{(int32_t)r.near, (int32_t)idx};
    if (rec_upd(r)) {
      DUpd u;
      rec_u(r, u.u, u.straight);
      u.idx = (int32_t)idx;
      u.parent = (int32_t)r.near;
      u.pad = 0;
      a.out.upd[upd_rank] = u;
    }
    if (first) {
      a.txy[idx] = make_double2(r.x, r.y);
      a.t4[idx] = screen_node(r.x, r.y, a.cx, a.cy);
      a.tth[idx] = r.th;
      node_insert(a.htab, a.hmask, r.x, r.y, r.th, (int32_t)idx, a.err);
      mx = centred_abs(r.x, r.y, a.cx, a.cy);
    }
  }
  if (special) {
    tr_resolved o;
    o.r = r;
    o.idx = idx;
    o.flags = ((r.flags & TR_FL_MEMBER) ? TR_RS_MEMBER : 0) |
              ((r.flags & TR_FL_SAME_NEAR) ? TR_RS_SAME_NEAR : 0) | (first ? TR_RS_FIRST : 0);
    o.pad = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // TR_DDE_*
    a.out.res[j] = o;
  }
}

// A new node's entry: its pose, cameFrom from the last record with that pose.
__device__ __forceinline__ void dd_node(const DDArgs& a, int64_t rank, const tr_record& r,
                                        int64_t last) {
  const tr_record& L = a.rec[last];
  DNode d;
  d.x = r.x;
  d.y = r.y;
  d.th = r.th;
  rec_u(L, d.u, d.straight);
  d.parent = (int32_t)L.near;
  a.out.nodes[rank] = d;
}

__device__ __forceinline__ void dd_max(double mx, unsigned long long* maxabs) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0 && mx > 0.0) atomicMax(maxabs, (unsigned long long)__double_as_longlong(mx));
}

// ------------------------------------------------------------------ claim / count / emit
constexpr int DK_T = 256;

// 1: the claims of the batch's new poses (first by atomicMin, last by atomicMax), special records.
__global__ __launch_bounds__(DK_T) void k_dd_claim(DDArgs a) {
  const int64_t j = (int64_t)blockIdx.x * DK_T + threadIdx.x;
  if (j >= a.n) return;
  const tr_record r = a.rec[j];
  a.slot[j] = dd_claim_one(a.claim, a.rec, j, r, a.err);
}

// 2: first occurrences and the block-local ranks (node, edge, update) and counts.
__global__ __launch_bounds__(DK_T) void k_dd_count(DDArgs a) {
  __shared__ int32_t s_w[3][DK_T / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t j = (int64_t)blockIdx.x * DK_T + t;
  if (j == 0) a.base[0] = a.count[0];
  bool f = false, acc = false, up = false;
  if (j < a.n) {
    const tr_record& r = a.rec[j];
    acc = rec_accepted(r);
    up = rec_upd(r);
    const int32_t sl = a.slot[j];
    f = sl >= 0 && (int64_t)(a.claim.btab[sl] & 0xffffffffull) == j;
  }
  const uint64_t m[3] = {__ballot(f), __ballot(acc), __ballot(up)};
  if (lane == 0)
    for (int i = 0; i < 3; ++i) s_w[i][wv] = __popcll(m[i]);
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int i = 0; i < 3; ++i) {
    int32_t off = 0, tot = 0;
    for (int q = 0; q < DK_T / 64; ++q) {
      off += q < wv ? s_w[i][q] : 0;
      tot += s_w[i][q];
    }
    if (j < a.n) a.lr[3 * j + i] = off + __popcll(m[i] & lt);
    if (t == 0) a.bc[3 * blockIdx.x + i] = tot;
  }
}

// prefix of counter i over blocks [0, nb) (every thread of the block gets it)
__device__ __forceinline__ int64_t dd_block_prefix(const int32_t* bc, int i, int64_t nb, int64_t* s) {
  int64_t v = 0;
  for (int64_t q = threadIdx.x; q < nb; q += DK_T) v += bc[3 * q + i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (threadIdx.x == 0) *s = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long*)s, (unsigned long long)v);
  __syncthreads();
  return *s;
}

// 3: indices, tree append, outputs; block 0 writes the totals.
__global__ __launch_bounds__(DK_T) void k_dd_emit(DDArgs a) {
  __shared__ int64_t s_p;
  const int t = threadIdx.x;
  const int64_t bid = blockIdx.x, nblk = (a.n + DK_T - 1) / DK_T;
  int64_t pre[3];
  for (int i = 0; i < 3; ++i) pre[i] = dd_block_prefix(a.bc, i, bid, &s_p);
  const int64_t N = a.base[0];
  const bool special = *a.claim.special == a.claim.epoch;
  const int64_t j = bid * DK_T + t;
  double mx = 0.0;
  if (j < a.n) {
    const tr_record r = a.rec[j];
    const int32_t sl = a.slot[j];
    const bool f = sl >= 0 && (int64_t)(a.claim.btab[sl] & 0xffffffffull) == j;
    int64_t idx = -1;
    if (rec_accepted(r)) {
      if (r.ex >= 0) {
        idx = r.ex;
      } else if (sl >= 0) {
        const int64_t f0 = (int64_t)(a.claim.btab[sl] & 0xffffffffull);
        int64_t pf = pre[0];                 // node rank: the first occurrence's block prefix ...
        if (f0 / DK_T != bid) {
          pf = 0;
          for (int64_t q = 0; q < f0 / DK_T; ++q) pf += a.bc[3 * q];
        }
        idx = N + pf + a.lr[3 * f0];         // ... + its rank in its block
      }
    }
    const int64_t nr = pre[0] + a.lr[3 * j], er = pre[1] + a.lr[3 * j + 1], ur = pre[2] + a.lr[3 * j + 2];
    dd_emit(a, j, r, idx, f, nr, er, ur, special, mx);
    if (f) dd_node(a, nr, r, (int64_t)(a.claim.blast[sl] & 0xffffffffull));
  }
  dd_max(mx, a.maxabs);
  if (bid == 0) {
    int64_t tot[3];
    for (int i = 0; i < 3; ++i) tot[i] = dd_block_prefix(a.bc, i, nblk, &s_p);
    if (t == 0) {
      a.count[0] = N + tot[0];
      a.snap[0] = N + tot[0];
      DHead hd;
      hd.n_new = tot[0];
      hd.n_edge = tot[1];
      hd.n_upd = tot[2];
      hd.special = special ? 1 : 0;
      hd.n = a.n;
      hd.base = N;
      hd.err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      hd.pad = 0;
      *a.out.head = hd;
    }
  }
  // the last block to finish publishes the batch: `done` (device) for a stream gated on the tree
  // after this dedupe, `ready` (pinned host) for the replay worker polling the commit slot.  Every
  // thread releases its own writes first (system scope when the host reads them), the counter
  // orders the blocks, and the last one acquires before it stores the flags.
  if (a.done || a.ready) {
    if (a.ready) __threadfence_system(); else __threadfence();
    __syncthreads();
    if (t == 0 && atomicAdd(a.blocks, 1) == (int32_t)nblk - 1) {
      __threadfence();
      __hip_atomic_store(a.blocks, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.done) __hip_atomic_store(a.done, a.claim.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (a.ready) __hip_atomic_store(a.ready, a.claim.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
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

// ------------------------------------------------------------------ stream gates
// A stream that must wait for a point of another stream (the look-ahead for the tree after a
// dedupe, the batch for its look-ahead) launches k_gate instead of waiting on an event: one wave
// polls a device flag in L2 that the producer's last kernel (k_dd_emit's last block, or k_publish)
// stores.  An event edge costs ~10-15 us of GPU time per batch between the producer's end and the
// consumer's start (marker packet with a cache release, barrier packet, CP re-evaluation); a gate
// costs one kernel's dispatch.  Bounded: after ~1 s of wall clock (100 MHz counter) it sets
// TR_DDE_GATE and lets the stream go on, so a producer that never comes cannot hang the device
// (the run then fails with that error; later gates of the session pass at once).
__global__ __launch_bounds__(64) void k_gate(const unsigned long long* __restrict__ flag,
                                            unsigned long long target, int32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & TR_DDE_GATE) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (wall_clock64() - t0 > 100000000ull) {
      atomicOr(err, TR_DDE_GATE);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__global__ __launch_bounds__(64) void k_publish(unsigned long long* __restrict__ flag,
                                               unsigned long long v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------ host side
void launch_gate(hipStream_t st, const unsigned long long* flag, unsigned long long target, int32_t* err) {
  hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, st, flag, target, err);
}

void launch_publish(hipStream_t st, unsigned long long* flag, unsigned long long v) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, flag, v);
}

void dd_batch(hipStream_t st, const DDArgs& a) {
  const unsigned g = (unsigned)((a.n + DK_T - 1) / DK_T);
  hipLaunchKernelGGL(k_dd_claim, dim3(g), dim3(DK_T), 0, st, a);
  hipLaunchKernelGGL(k_dd_count, dim3(g), dim3(DK_T), 0, st, a);
  hipLaunchKernelGGL(k_dd_emit, dim3(g), dim3(DK_T), 0, st, a);
}

void dd_rebuild(hipStream_t st, PoseSlot* htab, uint64_t hmask, int32_t* err, const double2* txy,
                const double* tth, int64_t N) {
  (void)hipMemsetAsync(htab, 0xff, sizeof(PoseSlot) * (hmask + 1), st);
  if (N > 0)
    hipLaunchKernelGGL(k_dd_rebuild, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, txy, tth, N,
                       htab, hmask, err);
}

}  // namespace tr
