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
#include "diaglog.hpp"
TR_DLOG_EXPORT(tr_diag_log_dd)

namespace tr {

__device__ __forceinline__ void node_insert(PoseSlot* tab, uint64_t mask, double x, double y,
                                            double t, int32_t v, int32_t* err) {
  // the first empty slot from the home bucket on (thetarrt_internal.hpp: pose table)
  uint64_t p = (pose_hash(x, y, t) & (mask / POSE_BUCKET)) * POSE_BUCKET;
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

// A new node into its bin of this epoch's set (thetarrt_internal.hpp: DeltaBins), in two steps so
// that the slot's atomic is in flight together with the pose table's (node_insert): bins_slot
// before it, bins_store after.
__device__ __forceinline__ int64_t bins_bin(const DeltaBins& b, double x, double y) {
  return (int64_t)(db_coord(y, b.ymax) >> b.shift) * b.nbx + (db_coord(x, b.xmax) >> b.shift);
}
__device__ __forceinline__ uint32_t bins_slot(const DeltaBins& b, unsigned long long epoch, int64_t bin) {
  const int64_t nb = (int64_t)b.nbx * b.nby, set = (int64_t)(epoch & 3);
  return atomicAdd(b.cnt + set * (nb + 1) + bin, 1u);
}
__device__ __forceinline__ void bins_store(const DeltaBins& b, unsigned long long epoch, int64_t bin,
                                           uint32_t slot, double x, double y, int32_t idx) {
  const int64_t nb = (int64_t)b.nbx * b.nby, set = (int64_t)(epoch & 3);
  if (slot < (uint32_t)DB_CAP) {
    b.items[(set * nb + bin) * DB_CAP + slot] = DBItem{x, y, idx, 0};
  } else {                                   // a full bin: the set's overflow list
    const uint32_t o = atomicAdd(b.cnt + set * (nb + 1) + nb, 1u);
    if (o < (uint32_t)b.ovf_cap) b.ovf[set * b.ovf_cap + o] = DBItem{x, y, idx, 0};
  }
}

// The next dedupe's bin counts (its set is idle while this dedupe runs), by every thread of a launch.
__device__ __forceinline__ void bins_zero_next(const DeltaBins& b, unsigned long long epoch,
                                               int64_t tid, int64_t nthreads) {
  const int64_t nb = (int64_t)b.nbx * b.nby + 1;             // + the overflow list's count
  uint32_t* z = b.cnt + ((epoch + 1) & 3) * nb;
  for (int64_t q = tid; q < nb; q += nthreads) z[q] = 0;
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
      int64_t bin = 0;
      uint32_t bslot = 0;
      if (a.bins.cnt) {
        bin = bins_bin(a.bins, r.x, r.y);
        bslot = bins_slot(a.bins, a.claim.epoch, bin);
      }
      a.txy[idx] = make_double2(r.x, r.y);
      a.t4[idx] = screen_node(r.x, r.y, a.cx, a.cy);
      a.tth[idx] = r.th;
      node_insert(a.htab, a.hmask, r.x, r.y, r.th, (int32_t)idx, a.err);
      mx = centred_abs(r.x, r.y, a.cx, a.cy);
      if (a.bins.cnt) bins_store(a.bins, a.claim.epoch, bin, bslot, r.x, r.y, (int32_t)idx);
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
constexpr int DK_T = DD_BLOCK;      // threads (= records) per dedupe block
// k_dd's status word packs each block's node / edge / update counts into 10-bit fields
static_assert(DK_T <= 512 && DK_T % 64 == 0, "a block's counts must fit k_dd's 10-bit fields");

// 1: the claims of the batch's new poses (first by atomicMin, last by atomicMax), special records.
__global__ __launch_bounds__(DK_T) void k_dd_claim(DDArgs a) {
  const int64_t j = (int64_t)blockIdx.x * DK_T + threadIdx.x;
  if (a.bins.cnt) bins_zero_next(a.bins, a.claim.epoch, j, (int64_t)gridDim.x * DK_T);
  if (j >= a.n) return;
  const tr_record r = a.rec[j];
  a.slot[j] = dd_claim_one(a.claim, a.rec, j, r, a.err);
}

// 2: first occurrences and the block-local ranks (node, edge, update) and counts.
__global__ __launch_bounds__(DK_T) void k_dd_count(DDArgs a) {
  __shared__ int32_t s_w[3][DK_T / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t j = (int64_t)blockIdx.x * DK_T + t;
  if (j == 0) a.base[0] = ld_sc1(a.count);
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
      hd.pad = head_tag(a.claim.epoch);
      *a.out.head = hd;
    }
  }
  // the last block to finish publishes the batch: `done` (device) for a stream gated on the tree
  // after this dedupe, `ready` (pinned host) for the replay worker polling the commit slot.  Every
  // wave waits for its stores, one thread per block writes the L2 back (system scope when the host
  // reads the slot), the counter orders the blocks (thetarrt_internal.hpp: st_sc1).
  if (a.done || a.ready) {
    wave_stores_done();
    __syncthreads();
    if (t == 0) {
      if (a.ready) release_sys(); else release_l2();   // this block's stores, once
      if (atomicAdd(a.blocks, 1) == (int32_t)nblk - 1) {
        __hip_atomic_store(a.blocks, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.done) __hip_atomic_store(a.done, a.claim.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a.ready) __hip_atomic_store(a.ready, a.claim.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
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

// ------------------------------------------------------------------ one-kernel dedupe
// k_dd does claim / count / emit in one launch.  Blocks take tickets in dispatch order, so every
// lower ticket belongs to a block that is running or done and a block may wait for its
// predecessors: (1) claim its records' new poses, publish "claimed"; (2) wait until every earlier
// block has claimed (a record is the first occurrence of its pose iff the batch table holds its
// index once every lower record has claimed: higher ones cannot lower the minimum), rank the
// first occurrences / edges / updates in the block, publish the counts; (3) look back over the
// earlier blocks' counts (the exclusive prefix, and per block the node-count prefix for a
// duplicate whose first occurrence is in an earlier block); (4) emit.  A new node's cameFrom is its
// first record's; later records of the same pose overwrite it through the update list, in record
// order, as the reference's cameFrom[qnew] = ... does (rrt.py:187-188), so no "last record" claim is
// needed.  The last block to finish writes the head and totals, the node count, the resolved
// records of a special batch, and the done / ready flags.
// Status word per block: (epoch & 0xffffffff) << 32 | stage << 30 | nodes << 20 | edges << 10 | upd.
constexpr unsigned long long DD_CLAIMED = 1, DD_COUNTED = 2;

__device__ __forceinline__ unsigned long long dd_tag(unsigned long long epoch) {
  return (epoch & 0xffffffffull) << 32;
}

// Spins until block q's status has reached `stage` in this epoch (bounded like k_gate: tickets
// are taken in dispatch order, so the block waited for is running or done).
__device__ __forceinline__ unsigned long long dd_wait(const unsigned long long* bst, int64_t q,
                                                      unsigned long long tag,
                                                      unsigned long long stage, int32_t* err) {
  uint64_t t0 = 0;
  for (int it = 0;; ++it) {
    const unsigned long long v = __hip_atomic_load(bst + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((v & 0xffffffff00000000ull) == tag && ((v >> 30) & 3) >= stage) return v;
    if (it == 0) {
      t0 = wall_clock64();
    } else if (wall_clock64() - t0 > GATE_TICKS) {
      atomicOr(err, TR_DDE_GATE);
      return tag | (stage << 30);
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ bool rec_upd_fused(const tr_record& r, bool first) {
  return rec_accepted(r) && (r.ex >= 0 ? !(r.flags & TR_FL_SAME_NEAR) : !first);
}

#ifdef TR_DIAG_DD
__device__ unsigned long long g_dd[8];
#endif
#ifdef TR_DIAG_PHASES
// diagnosis builds only: first block start / last block end / gate passed of the latest 8 k_dd
// launches (100 MHz wall clock, slot = epoch % 8), read back through tr_diag_dd
__device__ unsigned long long g_dds[8 * 4];
extern "C" int tr_diag_dd(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dds), sizeof(g_dds));
}
#endif
__global__ __launch_bounds__(DK_T) void k_dd(DDArgs a) {
  extern __shared__ int32_t s_c0[];        // node counts of the earlier blocks
  __shared__ int32_t s_w[3][DK_T / 64];
  __shared__ unsigned long long s_sum[3];
  __shared__ int s_bid, s_last;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t nblk = (a.n + DK_T - 1) / DK_T;
  const unsigned long long tag = dd_tag(a.claim.epoch);
  TR_DLOG_T0;
#ifdef TR_DIAG_DD
  uint64_t tdd[8];
  tdd[0] = wall_clock64();
#define TR_DD(i) if (t == 0) tdd[i] = wall_clock64()
#else
#define TR_DD(i)
#endif
#ifdef TR_DIAG_PHASES
  if (t == 0) {
    unsigned long long* d = g_dds + (a.claim.epoch & 7) * 4;
    if (atomicAdd(a.ticket, 0) == 0) { d[0] = wall_clock64(); d[1] = 0; d[2] = 0; d[3] = a.claim.epoch; }
  }
#endif
  if (t == 0) s_bid = atomicAdd(a.ticket, 1);
  if (t < 3) s_sum[t] = 0;
  if (a.bins.cnt) bins_zero_next(a.bins, a.claim.epoch, (int64_t)blockIdx.x * DK_T + t, (int64_t)gridDim.x * DK_T);
  __syncthreads();
  const int64_t bid = s_bid;
  const int64_t j = bid * DK_T + t;
  const bool act = j < a.n;
  // (read past this XCD's L2: a count one dedupe old would put this batch's nodes over the last one's)
  const int64_t N = ld_sc1(a.count);       // updated only by the last block to finish
  tr_record r{};
  int32_t sl = -1;
  if (act) {
    r = a.rec[j];
    sl = dd_claim_one(a.claim, a.rec, j, r, a.err);
    st_sc1(a.slot + j, sl);
  }
  TR_DD(1);
  // (1) claimed (the claims are atomics: coherent once each wave has waited for them)
  wave_stores_done();
  __syncthreads();
  if (t == 0) st_sc1(a.bst + bid, tag | (DD_CLAIMED << 30));
  TR_DD(2);
  // (2) every earlier block has claimed: first occurrences, block-local ranks
  for (int64_t q = t; q < bid; q += DK_T) (void)dd_wait(a.bst, q, tag, DD_CLAIMED, a.err);
  __syncthreads();
  const bool f = sl >= 0 && (int64_t)(__hip_atomic_load(a.claim.btab + sl, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffull) == j;
  const bool acc = act && rec_accepted(r), up = act && rec_upd_fused(r, f);
  const uint64_t m[3] = {__ballot(f), __ballot(acc), __ballot(up)};
  if (lane == 0)
    for (int i = 0; i < 3; ++i) s_w[i][wv] = __popcll(m[i]);
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  int32_t rk[3], cnt[3];
  for (int i = 0; i < 3; ++i) {
    int32_t off = 0, tot = 0;
    for (int q = 0; q < DK_T / 64; ++q) {
      off += q < wv ? s_w[i][q] : 0;
      tot += s_w[i][q];
    }
    rk[i] = off + __popcll(m[i] & lt);
    cnt[i] = tot;
  }
  if (f) st_sc1(a.lr + j, rk[0]);          // a later duplicate's node index needs it
  wave_stores_done();
  __syncthreads();
  if (t == 0)
    st_sc1(a.bst + bid, tag | (DD_COUNTED << 30) | ((unsigned long long)cnt[0] << 20) |
                            ((unsigned long long)cnt[1] << 10) | (unsigned long long)cnt[2]);
  TR_DD(3);
  // (3) look back: the exclusive prefix over the earlier blocks
  unsigned long long p0 = 0, p1 = 0, p2 = 0;
  for (int64_t q = t; q < bid; q += DK_T) {
    const unsigned long long v = dd_wait(a.bst, q, tag, DD_COUNTED, a.err);
    const int32_t c0 = (int32_t)((v >> 20) & 1023);
    s_c0[q] = c0;
    p0 += c0;
    p1 += (v >> 10) & 1023;
    p2 += v & 1023;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    p0 += __shfl_xor(p0, o);
    p1 += __shfl_xor(p1, o);
    p2 += __shfl_xor(p2, o);
  }
  if (lane == 0) {
    atomicAdd(&s_sum[0], p0);
    atomicAdd(&s_sum[1], p1);
    atomicAdd(&s_sum[2], p2);
  }
  __syncthreads();
  const int64_t pre0 = (int64_t)s_sum[0], pre1 = (int64_t)s_sum[1], pre2 = (int64_t)s_sum[2];
  TR_DD(4);
  // (4) emit
  double mx = 0.0;
  if (act) {
    int64_t idx = -1;
    if (acc) {
      if (r.ex >= 0) {
        idx = r.ex;
      } else if (f) {
        idx = N + pre0 + rk[0];
      } else if (sl >= 0) {                  // a duplicate: its first occurrence's index
        const int64_t f0 = (int64_t)(__hip_atomic_load(a.claim.btab + sl, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffull);
        const int64_t b0 = f0 / DK_T;
        int64_t pf = pre0;
        if (b0 != bid) {
          pf = 0;
          for (int64_t q = 0; q < b0; ++q) pf += s_c0[q];
        }
        idx = N + pf + ld_sc1(a.lr + f0);
      }
    }
    st_sc1(a.idxs + j, idx);
    if (acc) {
#ifndef TR_DIAG_NOHOSTDELTA                  /* diagnosis builds only: the host's delta not written */
      a.out.edges[pre1 + rk[1]] = DEdge{(int32_t)r.near, (int32_t)idx};
      if (up) {
        DUpd u;
        rec_u(r, u.u, u.straight);
        u.idx = (int32_t)idx;
        u.parent = (int32_t)r.near;
        u.pad = 0;
        a.out.upd[pre2 + rk[2]] = u;
      }
#endif
      if (f) {
        int64_t bin = 0;
        uint32_t bslot = 0;
        if (a.bins.cnt) {                      // (its atomic in flight with the pose table's)
          bin = bins_bin(a.bins, r.x, r.y);
          bslot = bins_slot(a.bins, a.claim.epoch, bin);
        }
        a.txy[idx] = make_double2(r.x, r.y);
        a.t4[idx] = screen_node(r.x, r.y, a.cx, a.cy);
        a.tth[idx] = r.th;
        node_insert(a.htab, a.hmask, r.x, r.y, r.th, (int32_t)idx, a.err);
        mx = centred_abs(r.x, r.y, a.cx, a.cy);
#ifndef TR_DIAG_NOHOSTDELTA
        dd_node(a, pre0 + rk[0], r, j);
#endif
        if (a.bins.cnt) bins_store(a.bins, a.claim.epoch, bin, bslot, r.x, r.y, (int32_t)idx);
      }
    }
  }
  dd_max(mx, a.maxabs);
  // the last block to finish: totals, head, special records, flags.  Every block writes its L2
  // back once (the tree and pose-table stores are read by the look-ahead's kernels, gated on
  // `done`, before this kernel ends).
  wave_stores_done();
  __syncthreads();
  if (t == 0) {
    release_l2();
    s_last = atomicAdd(a.blocks, 1) == (int32_t)nblk - 1;
  }
  __syncthreads();
#ifdef TR_DIAG_DD                          // diagnosis builds only: block phases (us), wall clock
  TR_DD(5);
  if (t == 0) {
    for (int q = 0; q < 5; ++q) atomicAdd(&g_dd[q], tdd[q + 1] - tdd[q]);
    atomicMax(&g_dd[5], tdd[5] - tdd[0]);
    atomicAdd(&g_dd[6], 1ull);
  }
  if (s_last && t == 0) {
    const unsigned long long L = atomicAdd(&g_dd[7], 1ull);
    const double nb = (double)g_dd[6];
    if (L % 40 == 39)
      printf("TR_DIAG_DD blocks %.0f mean us: claim %.2f wait-claimed %.2f count %.2f look-back %.2f "
             "emit %.2f | max block %.2f\n", nb, g_dd[0] * 0.01 / nb, g_dd[1] * 0.01 / nb,
             g_dd[2] * 0.01 / nb, g_dd[3] * 0.01 / nb, g_dd[4] * 0.01 / nb, g_dd[5] * 0.01);
    for (int q = 0; q < 7; ++q) g_dd[q] = 0;
  }
#endif
#undef TR_DD
  if (!s_last) {
    TR_DLOG(4);
    return;
  }
  if (t < 3) s_sum[t] = 0;
  __syncthreads();
  unsigned long long q0 = 0, q1 = 0, q2 = 0;
  for (int64_t q = t; q < nblk; q += DK_T) {
    const unsigned long long v = __hip_atomic_load(a.bst + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    q0 += (v >> 20) & 1023;
    q1 += (v >> 10) & 1023;
    q2 += v & 1023;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    q0 += __shfl_xor(q0, o);
    q1 += __shfl_xor(q1, o);
    q2 += __shfl_xor(q2, o);
  }
  if (lane == 0) {
    atomicAdd(&s_sum[0], q0);
    atomicAdd(&s_sum[1], q1);
    atomicAdd(&s_sum[2], q2);
  }
  __syncthreads();
  const bool special = __hip_atomic_load(a.claim.special, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                       a.claim.epoch;
  if (special) {                             // every record in order, for the sequential replay
    const int32_t e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int64_t i = t; i < a.n; i += DK_T) {
      const tr_record ri = a.rec[i];
      const int32_t si = ld_sc1(a.slot + i);
      const bool fi = si >= 0 && (int64_t)(ld_sc1(a.claim.btab + si) & 0xffffffffull) == i;
      tr_resolved o;
      o.r = ri;
      o.idx = ld_sc1(a.idxs + i);
      o.flags = ((ri.flags & TR_FL_MEMBER) ? TR_RS_MEMBER : 0) |
                ((ri.flags & TR_FL_SAME_NEAR) ? TR_RS_SAME_NEAR : 0) | (fi ? TR_RS_FIRST : 0);
      o.pad = e;
      a.out.res[i] = o;
    }
  }
  if (t == 0) {
    const int64_t tot0 = (int64_t)s_sum[0];
    a.count[0] = N + tot0;
    a.snap[0] = N + tot0;
    DHead hd;
    hd.n_new = tot0;
    hd.n_edge = (int64_t)s_sum[1];
    hd.n_upd = (int64_t)s_sum[2];
    hd.special = special ? 1 : 0;
    hd.n = a.n;
    hd.base = N;
    hd.err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    hd.pad = head_tag(a.claim.epoch);
    *a.out.head = hd;
    __hip_atomic_store(a.blocks, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  wave_stores_done();
  __syncthreads();
  if (t == 0) {
    if (a.ready) release_sys(); else release_l2();
    if (a.done) __hip_atomic_store(a.done, a.claim.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (a.ready) __hip_atomic_store(a.ready, a.claim.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#ifdef TR_DIAG_PHASES
    g_dds[(a.claim.epoch & 7) * 4 + 1] = wall_clock64();
#endif
    // the next batch's gate (its look-ahead was enqueued before this dedupe and waits only for
    // the `done` just stored): this kernel ends once it has passed, bounded like k_gate
    if (a.gate && !(__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & TR_DDE_GATE)) {
      const uint64_t t0 = wall_clock64();
      while (ld_sc1(a.gate) < a.gate_v) {
        if (wall_clock64() - t0 > GATE_TICKS) {
          atomicOr(a.err, TR_DDE_GATE);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
#ifdef TR_DIAG_PHASES
    g_dds[(a.claim.epoch & 7) * 4 + 2] = wall_clock64();
#endif
  }
  TR_DLOG(4);
}

// ------------------------------------------------------------------ stream gates
// A stream that must wait for a point of another stream (the look-ahead for the tree after a
// dedupe, the batch for its look-ahead) launches k_gate instead of waiting on an event: one wave
// polls a device flag in L2 that the producer's last kernel (k_dd_emit's last block, or k_publish)
// stores.  An event edge costs ~10-15 us of GPU time per batch between the producer's end and the
// consumer's start (marker packet with a cache release, barrier packet, CP re-evaluation); a gate
// costs one kernel's dispatch.  Bounded (GATE_TICKS): after ~30 s of wall clock (100 MHz counter) it sets
// TR_DDE_GATE and lets the stream go on, so a producer that never comes cannot hang the device
// (the run then fails with that error; later gates of the session pass at once).
__global__ __launch_bounds__(64) void k_gate(const unsigned long long* __restrict__ flag,
                                            unsigned long long target, int32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & TR_DDE_GATE) return;
  TR_DLOG_T0;
  const uint64_t t0 = wall_clock64();
  while (ld_sc1(flag) < target) {           // relaxed: the next kernel's dispatch acquires
    // 30 s: in a sharded run the look-ahead's gate waits for a dedupe behind the all-gather,
    // i.e. for the slowest rank (the first RCCL collective sets up its connections)
    if (wall_clock64() - t0 > GATE_TICKS) {
      atomicOr(err, TR_DDE_GATE);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  TR_DLOG(5);
}

__global__ __launch_bounds__(64) void k_publish(unsigned long long* __restrict__ flag,
                                               unsigned long long v) {
  // the stream's earlier kernels have ended (their end-of-kernel release is done)
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One side of the concurrency probe (capi.hip gate_probe): store `mine`, wait up to `ticks` of the
// 100 MHz wall clock for `other`, report whether it came.
__global__ __launch_bounds__(64) void k_handshake(unsigned long long* __restrict__ mine,
                                                 const unsigned long long* __restrict__ other,
                                                 unsigned long long ticks,
                                                 unsigned long long* __restrict__ ok) {
  if (threadIdx.x != 0) return;
  __hip_atomic_store(mine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  unsigned long long seen = 0;
  while (!(seen = ld_sc1(other)) && wall_clock64() - t0 <= ticks) __builtin_amdgcn_s_sleep(2);
  *ok = seen ? 1ull : 0ull;
}

// ------------------------------------------------------------------ host side
void launch_handshake(hipStream_t st, unsigned long long* mine, const unsigned long long* other,
                      unsigned long long ticks, unsigned long long* ok) {
  hipLaunchKernelGGL(k_handshake, dim3(1), dim3(64), 0, st, mine, other, ticks, ok);
}

void launch_gate(hipStream_t st, const unsigned long long* flag, unsigned long long target, int32_t* err) {
  hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, st, flag, target, err);
}

void launch_publish(hipStream_t st, unsigned long long* flag, unsigned long long v) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, flag, v);
}

void dd_batch(hipStream_t st, const DDArgs& a, bool fused) {
  const unsigned g = (unsigned)((a.n + DK_T - 1) / DK_T);
  if (fused) {
    hipLaunchKernelGGL(k_dd, dim3(g), dim3(DK_T), sizeof(int32_t) * g, st, a);
    return;
  }
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
