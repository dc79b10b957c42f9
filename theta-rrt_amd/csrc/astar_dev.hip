// A* / lazy Theta* (search.py:221-307) resident on the device: one wave per (start, goal) query, a
// batch of queries per launch, no host round trip until the paths come back.
//
// The search is the reference's, pop for pop: the open queue holds (f, (x, y)) tuples and hands them
// out in tuple order (Python's PriorityQueue), stale copies of closed nodes are skipped
// (search.py:250-255), lazy Theta* tests lineofsight(current, cameFrom[current]) at the pop and
// re-parents to the best closed neighbour when it fails (search.py:258-263), neighbours come in
// itertools.product([-1, 0, 1], repeat=2) order (search.py:184-194) and are relaxed through the
// current node and through its parent (search.py:274-304).  So path and len(closedSet) equal the
// reference's.  What the wave parallelises is inside one pop: the Bresenham pixels of the
// line-of-sight test (lanegroup.hpp), the 8 neighbours (a lane each: they are distinct nodes, so
// their relaxations commute), and the queue operations.
//
// The queue.  f = g + h >= h(start) for every entry (g is a sum of straight segment lengths from the
// start, h the straight distance to the goal), so entries go into NBK buckets of width 1/64 above
// f0 = h(start) (512 units of detour): byte counts in LDS, CAP entry slots per bucket in global
// memory.  A pop scans the counts
// from the lowest bucket that can be non-empty, loads that bucket's entries (one per lane) and takes
// their exact minimum in (f, x, y) order by a wave reduction; a push is an LDS atomic for the slot
// and one store, all of a pop's pushes at once.  Each lane also loads the state word and gScore of
// its entry's node: copies of closed nodes (which the reference pops and skips, search.py:250-255,
// to no effect) are dropped from the bucket there and then, and the winner's state arrives with it.  An entry beyond the buckets' range, or for a full
// bucket, goes to a `far` list in global memory; while that list is not empty its exact minimum
// (cached, rescanned after it has been popped) competes with the bucket's minimum, so the order
// stays exact in every case and only the speed depends on the bucket geometry.
//
// Per-cell state (global): word = state << 30 | (cameFrom id + 1), and gScore.  A query lives in one
// wave, so its memory needs no more than workgroup scope: relaxed workgroup-scope atomics are plain
// loads and stores served by the CU's own L1 / the XCD's L2 (agent scope would send every access
// past the per-XCD L2 to the fabric, ~1.5 us each: measured 3x the search time), kept in program
// order against each other by one wait for outstanding stores at the top of every pop.
#pragma clang fp contract(off)
#include "lanegroup.hpp"
#include "thetarrt_internal.hpp"

namespace tr {

namespace {

constexpr int A_NBK = 32768;       // buckets (LDS byte counts: 32 KB per query in flight)
constexpr int A_CAP = 64;          // entries per bucket: one per lane
constexpr double A_BW = 64.0;      // buckets per unit of f.  Measured on map2, main.py:57's query:
                                   // 8 per unit 0.25 s (buckets overflow into the far list, whose
                                   // pops rescan it), 32 per unit 0.135 s, 64 per unit 0.128 s
constexpr uint32_t A_OPEN = 1u << 30, A_CLOSED = 2u << 30, A_IDMASK = (1u << 30) - 1;

template <class T>
__device__ __forceinline__ void st_wg(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <class T>
__device__ __forceinline__ T ld_wg(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct AEntry {                    // 16 bytes
  double f;
  uint32_t key, pad;               // key = x << 16 | y: tuple order of (x, y)
};

__device__ __forceinline__ bool key_less(double fa, uint32_t ka, double fb, uint32_t kb) {
  return fa < fb || (fa == fb && ka < kb);
}

// Wave minimum of (f, key) with the lane that holds it (lanes without an entry pass f = +inf).
__device__ __forceinline__ void wave_min_entry(double& f, uint32_t& k, int& who) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const double fo = __shfl_xor(f, o);
    const uint32_t ko = __shfl_xor(k, o);
    const int wo = __shfl_xor(who, o);
    if (key_less(fo, ko, f, k) || (fo == f && ko == k && wo < who)) { f = fo; k = ko; who = wo; }
  }
}

__device__ __forceinline__ double l2i(int64_t x0, int64_t y0, int64_t x1, int64_t y1) {
  const int64_t dx = x1 - x0, dy = y1 - y0;      // search.py:13-15 on ints
  return sqrt((double)(dx * dx + dy * dy));
}

struct AQueue {                    // wave-uniform copies in every lane
  uint32_t* cnt;                   // LDS: entries per bucket, a byte each (four to a word)
  AEntry* bk;                      // global: A_NBK x A_CAP
  AEntry* far;                     // global: far_cap
  int64_t far_cap;
  double f0;
  int cur;                         // no bucket below it holds an entry
  int64_t nfar;
  bool far_valid;                  // the cached minimum below is the far list's
  double far_f;
  uint32_t far_k;
  int64_t far_slot;
  int overflow;                    // far list full: the search stops with status 6
  int64_t far_pushes;
};

__device__ __forceinline__ void st_entry(AEntry* p, double f, uint32_t k) {
  st_wg(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(f));
  st_wg(reinterpret_cast<unsigned long long*>(p) + 1, (unsigned long long)k);
}
__device__ __forceinline__ void ld_entry(const AEntry* p, double& f, uint32_t& k) {
  f = __longlong_as_double((long long)ld_wg(reinterpret_cast<const unsigned long long*>(p)));
  k = (uint32_t)ld_wg(reinterpret_cast<const unsigned long long*>(p) + 1);
}

// Every lane with `on` pushes its (f, key); only lanes 0 .. 7 (one per neighbour) ever do.
__device__ __forceinline__ void aq_push(AQueue& q, bool on, double f, uint32_t key) {
  const int lane = threadIdx.x & 63;
  bool to_far = false;
  int b = 0;
  if (on) {
    const double rel = (f - q.f0) * A_BW;
    b = rel <= 0.0 ? 0 : (rel >= (double)A_NBK ? A_NBK : (int)rel);
    if (b >= A_NBK) {
      to_far = true;
    } else {
      const int sh = 8 * (b & 3);    // counts stay <= CAP + 8 < 256: no carry between bytes
      const uint32_t slot = (atomicAdd(&q.cnt[b >> 2], 1u << sh) >> sh) & 0xffu;
      if (slot >= (uint32_t)A_CAP) {
        atomicSub(&q.cnt[b >> 2], 1u << sh);
        to_far = true;
      } else {
        st_entry(q.bk + (int64_t)b * A_CAP + slot, f, key);
      }
    }
  }
  int bmin = on && !to_far ? b : A_NBK;
#pragma unroll
  for (int o = 4; o >= 1; o >>= 1) bmin = min(bmin, __shfl_xor(bmin, o));
  q.cur = min(q.cur, __shfl(bmin, 0));
  const uint64_t fm = __ballot(to_far);
  if (fm) {
    const int64_t slot = q.nfar + __popcll(fm & ((1ull << lane) - 1ull));
    const bool fits = slot < q.far_cap;
    if (to_far && fits) st_entry(q.far + slot, f, key);
    if (__ballot(to_far && !fits)) q.overflow = 1;
    // the cached minimum takes the new entries in
    double mf = to_far && fits ? f : INFINITY;
    uint32_t mk = key;
    int who = lane;
    wave_min_entry(mf, mk, who);
    if (q.far_valid && mf < INFINITY && (q.nfar == 0 || key_less(mf, mk, q.far_f, q.far_k))) {
      q.far_f = mf;
      q.far_k = mk;
      q.far_slot = q.nfar + __popcll(fm & ((1ull << who) - 1ull));
    }
    q.nfar = min(q.nfar + (int64_t)__popcll(fm), q.far_cap);
    q.far_pushes += __popcll(fm);
  }
}

// The far list's exact minimum (f, key, slot), by a scan.
__device__ __forceinline__ void aq_far_rescan(AQueue& q) {
  const int lane = threadIdx.x & 63;
  double bf = INFINITY;
  uint32_t bkey = 0;
  int64_t bs = -1;
  for (int64_t i = lane; i < q.nfar; i += 64) {
    double f;
    uint32_t k;
    ld_entry(q.far + i, f, k);
    if (bs < 0 || key_less(f, k, bf, bkey)) { bf = f; bkey = k; bs = i; }
  }
  int who = lane;
  double mf = bf;
  uint32_t mk = bkey;
  wave_min_entry(mf, mk, who);
  q.far_f = mf;
  q.far_k = mk;
  q.far_slot = __shfl(bs, who);
  q.far_valid = true;
}

// Pops the smallest live (f, key): false when the queue is empty.  cw / gc = the node's state
// word and gScore.  Copies of closed nodes are discarded on the way, as the reference's pops of
// them are no-ops.
__device__ __forceinline__ bool aq_pop(AQueue& q, const uint32_t* cell, const double* gsc, int64_t W,
                                       double& f, uint32_t& key, uint32_t& cw, double& gc,
                                       int64_t& pops) {
  const int lane = threadIdx.x & 63;
  wave_stores_done();                      // the stores of the last pop / expansion have landed
  for (;;) {
    // first non-empty bucket at or above cur
    int b = A_NBK;
    for (int base = q.cur & ~3; base < A_NBK; base += 256) {      // a word of 4 counts per lane
      const int i = base + 4 * lane;
      uint32_t wd = i < A_NBK ? q.cnt[i >> 2] : 0u;
      const int skip = q.cur - i;                      // buckets of this word below cur
      if (skip >= 4) wd = 0u;
      else if (skip > 0) wd &= ~0u << (8 * skip);
      const uint64_t m = __ballot(wd != 0);
      if (m) {
        const int l = __ffsll((unsigned long long)m) - 1;
        const uint32_t w0 = __shfl(wd, l);
        b = base + 4 * l + (__ffs((int)w0) - 1) / 8;
        break;
      }
    }
    q.cur = b;
    double bf = INFINITY, mg = 0.0;
    uint32_t bkey = 0, mw = 0;
    int who = lane;
    uint64_t live = 0;
    int n = 0;
    if (b < A_NBK) {
      n = (int)((q.cnt[b >> 2] >> (8 * (b & 3))) & 0xffu);
      AEntry* e = q.bk + (int64_t)b * A_CAP;
      double f0 = INFINITY;
      uint32_t k0 = 0;
      if (lane < n) {
        ld_entry(e + lane, f0, k0);
        const int64_t c0 = (int64_t)(k0 >> 16) * W + (k0 & 0xffff);
        mw = ld_wg(cell + c0);
        mg = ld_wg(gsc + c0);
      }
      const bool alive = lane < n && !(mw & A_CLOSED);
      live = __ballot(alive);
      pops += n - __popcll(live);                     // the closed copies the reference would pop
      if (!live) {
        if (lane == 0) q.cnt[b >> 2] &= ~(0xffu << (8 * (b & 3)));
        q.cur = b + 1;
        continue;
      }
      bf = alive ? f0 : INFINITY;
      bkey = k0;
      wave_min_entry(bf, bkey, who);
      // the bucket keeps its live entries but the winner, packed to the front
      bool far_wins = false;
      if (q.nfar > 0) {
        if (!q.far_valid) aq_far_rescan(q);
        far_wins = key_less(q.far_f, q.far_k, bf, bkey);
      }
      const uint64_t keep = far_wins ? live : live & ~(1ull << who);
      if ((keep >> lane) & 1) {
        const int slot = __popcll(keep & ((1ull << lane) - 1ull));
        if (slot != lane) st_entry(e + slot, f0, k0);
      }
      if (lane == 0)
        q.cnt[b >> 2] = (q.cnt[b >> 2] & ~(0xffu << (8 * (b & 3)))) | ((uint32_t)__popcll(keep) << (8 * (b & 3)));
      if (!far_wins) {
        f = bf;
        key = bkey;
        cw = __shfl(mw, who);
        gc = __shfl(mg, who);
        ++pops;
        return true;
      }
      wave_stores_done();
    } else if (q.nfar > 0) {
      if (!q.far_valid) aq_far_rescan(q);
    } else {
      return false;
    }
    // the far list's minimum goes first
    f = q.far_f;
    key = q.far_k;
    const int64_t last = q.nfar - 1;
    if (q.far_slot != last && lane == 0) {
      double lf;
      uint32_t lk;
      ld_entry(q.far + last, lf, lk);
      st_entry(q.far + q.far_slot, lf, lk);
    }
    q.nfar = last;
    q.far_valid = false;
    ++pops;
    const int64_t c = (int64_t)(key >> 16) * W + (key & 0xffff);
    cw = ld_wg(cell + c);
    gc = ld_wg(gsc + c);
    wave_stores_done();
    if (!(cw & A_CLOSED)) return true;                // else a closed copy: next
  }
}

}  // namespace

// out per query: path_xy[q * cap ..] (x, y) pairs start .. goal, path_len[q], stats[q * 4 ..] =
// (expanded, queue entries consumed, pushes that went to the far list, status): 0 found, 1 start/goal not valid, 2 inside an obstacle, 3 no
// path, 4 IndexError, 5 ValueError (search.py:262), 6 queue capacity, 7 path longer than cap.
__global__ __launch_bounds__(64) void k_astar(Grid g, const int32_t* __restrict__ sg4, int64_t nq,
                                              int theta, uint32_t* __restrict__ cells,
                                              double* __restrict__ gs, AEntry* __restrict__ bks,
                                              AEntry* __restrict__ fars, int64_t far_cap,
                                              int64_t* __restrict__ path_xy, int64_t cap,
                                              int64_t* __restrict__ path_len,
                                              int64_t* __restrict__ stats) {
  __shared__ uint32_t s_cnt[A_NBK / 4];
  const int lane = threadIdx.x & 63;
  const int64_t qi = blockIdx.x;
  if (qi >= nq) return;
  const int64_t H = g.H, W = g.W, NC = H * W;
  uint32_t* cell = cells + qi * NC;
  double* gsc = gs + qi * NC;
  const int64_t sx = sg4[4 * qi], sy = sg4[4 * qi + 1], gx = sg4[4 * qi + 2], gy = sg4[4 * qi + 3];
  int64_t expanded = 0, pops = 0;
  int status = -1;
  AQueue q;
  q.far_pushes = 0;
  auto finish = [&](int st, int64_t plen) {
    if (lane == 0) {
      path_len[qi] = plen;
      stats[4 * qi] = expanded;
      stats[4 * qi + 1] = pops;
      stats[4 * qi + 2] = q.far_pushes;
      stats[4 * qi + 3] = st;
    }
  };
  for (int i = lane; i < A_NBK / 4; i += 64) s_cnt[i] = 0;
  __syncthreads();
  if (!valid_i(g, sx, sy) || !valid_i(g, gx, gy)) { finish(1, 0); return; }
  {
    int ierr = 0;
    const bool fs = free_i(g, sx, sy, &ierr), fg = free_i(g, gx, gy, &ierr);
    if (ierr) { finish(4, 0); return; }
    if (!fs || !fg) { finish(2, 0); return; }
  }
  auto id = [&](int64_t x, int64_t y) { return x * W + y; };
  q.cnt = s_cnt;
  q.bk = bks + qi * (int64_t)A_NBK * A_CAP;
  q.far = fars + qi * far_cap;
  q.far_cap = far_cap;
  q.f0 = l2i(sx, sy, gx, gy) - 1e-6;
  q.cur = A_NBK;
  q.nfar = 0;
  q.far_valid = true;
  q.far_f = INFINITY;
  q.far_k = 0;
  q.far_slot = -1;
  q.overflow = 0;
  q.far_pushes = 0;
  // neighbour k of (x, y) in the reference's order: deltas (a, b) over product([-1, 0, 1]) without
  // (0, 0), candidate = node - delta
  const int kk = lane < 8 ? (lane < 4 ? lane : lane + 1) : 0;
  const int da = kk / 3 - 1, db = kk % 3 - 1;
  const int64_t s = id(sx, sy);
  // the start node: closed, its neighbours opened (search.py:236-244)
  if (lane == 0) {
    st_wg(gsc + s, 0.0);
    st_wg(cell + s, A_CLOSED);
  }
  {
    const int64_t vx = sx - da, vy = sy - db;
    int ierr = 0;
    const bool ok = lane < 8 && valid_i(g, vx, vy) && free_i(g, vx, vy, &ierr);
    if (__ballot(lane < 8 && ierr)) { finish(4, 0); return; }
    double f = 0;
    if (ok) {
      const double gv = l2i(sx, sy, vx, vy);
      st_wg(gsc + id(vx, vy), gv);
      st_wg(cell + id(vx, vy), A_OPEN | (uint32_t)(s + 1));
      f = gv + l2i(vx, vy, gx, gy);
    }
    aq_push(q, ok, f, (uint32_t)(vx << 16 | vy));
  }
  expanded = 1;
  const Grp<64> gr(lane);
  int64_t goal_id = -1;
  for (;;) {
    if (q.overflow) { status = 6; break; }
    double f, gc;
    uint32_t key, cw;
    if (!aq_pop(q, cell, gsc, W, f, key, cw, gc, pops)) { status = 3; break; }
    const int64_t cx = key >> 16, cy = key & 0xffff, c = id(cx, cy);
    int64_t p = (int64_t)(cw & A_IDMASK) - 1;
    // the neighbours' state and the parent's gScore: loads in flight while the line of sight runs
    const int64_t vx = cx - da, vy = cy - db, v = id(vx, vy);
    int nerr = 0;
    const bool nb = lane < 8 && valid_i(g, vx, vy) && free_i(g, vx, vy, &nerr);
    const uint32_t vw = nb ? ld_wg(cell + v) : A_CLOSED;
    double gv = nb ? ld_wg(gsc + v) : 0.0;             // (garbage for a node never opened: not used)
    double gp = ld_wg(gsc + p);
    if (theta) {
      int ierr = 0;
      const bool clear = los_group<64>(g, gr, cx, cy, p / W, p % W, &ierr);
      if (gr.any(ierr != 0)) { status = 4; break; }
      if (!clear) {                                    // search.py:260-263
        if (__ballot(lane < 8 && nerr)) { status = 4; break; }
        double val = INFINITY;
        if (nb && (vw & A_CLOSED)) val = gv + l2i(vx, vy, cx, cy);
        const uint64_t have = __ballot(val < INFINITY);
        if (!have) { status = 5; break; }
        // np.argmin: the first minimum in neighbour order = the lowest lane among equal values
        double mv = val;
        int who = lane;
#pragma unroll
        for (int o = 4; o >= 1; o >>= 1) {
          const double vo = __shfl_xor(mv, o);
          const int wo = __shfl_xor(who, o);
          if (vo < mv || (vo == mv && wo < who)) { mv = vo; who = wo; }
        }
        mv = __shfl(mv, 0);
        who = __shfl(who, 0);
        const int wk = who < 4 ? who : who + 1;
        p = id(cx - (wk / 3 - 1), cy - (wk % 3 - 1));
        gc = mv;
        if (lane == 0) st_wg(gsc + c, gc);
        gp = ld_wg(gsc + p);
      }
    }
    if (lane == 0) st_wg(cell + c, A_CLOSED | (uint32_t)(p + 1));
    ++expanded;
    if (cx == gx && cy == gy) { status = 0; goal_id = c; wave_stores_done(); break; }
    // the neighbours, a lane each (search.py:274-304)
    {
      if (__ballot(lane < 8 && nerr)) { status = 4; break; }
      const bool live = nb && !(vw & A_CLOSED);
      uint32_t came = vw & A_IDMASK;
      bool push1 = false, push2 = false;
      double f1 = 0, f2 = 0;
      if (live) {
        const double h = l2i(vx, vy, gx, gy);
        double gg = gc + l2i(vx, vy, cx, cy);
        if (!(vw & A_OPEN) || gg < gv) {
          gv = gg;
          came = (uint32_t)(c + 1);
          push1 = true;
          f1 = gg + h;
        }
        if (theta) {
          gg = gp + l2i(p / W, p % W, vx, vy);
          if (gg < gv) {
            gv = gg;
            came = (uint32_t)(p + 1);
            push2 = true;
            f2 = gg + h;
          }
        }
        if (push1 || push2) {
          st_wg(gsc + v, gv);
          st_wg(cell + v, A_OPEN | came);
        }
      }
      const uint32_t vkey = (uint32_t)(vx << 16 | vy);
      aq_push(q, push1, f1, vkey);
      aq_push(q, push2, f2, vkey);
    }
  }
  if (status != 0) { finish(status, 0); return; }
  // reconstruct (search.py:196-204): follow cameFrom from the goal; written start .. goal
  int64_t n = 0;
  if (lane == 0) {
    for (int64_t v = goal_id; v >= 0; v = (v == s ? -1 : (int64_t)(ld_wg(cell + v) & A_IDMASK) - 1)) ++n;
    if (n <= cap) {
      int64_t k = n - 1;
      for (int64_t v = goal_id; v >= 0; v = (v == s ? -1 : (int64_t)(ld_wg(cell + v) & A_IDMASK) - 1), --k) {
        path_xy[(qi * cap + k) * 2] = v / W;
        path_xy[(qi * cap + k) * 2 + 1] = v % W;
      }
    }
  }
  n = __shfl(n, 0);
  finish(n <= cap ? 0 : 7, n);
}

int64_t astar_dev_bytes_per_query(int64_t H, int64_t W, int64_t far_cap) {
  return H * W * (int64_t)(sizeof(uint32_t) + sizeof(double)) +
         (int64_t)sizeof(AEntry) * ((int64_t)A_NBK * A_CAP + far_cap);
}

// Carves the per-query state out of `work` (astar_dev_bytes_per_query(H, W, far_cap) * nq bytes,
// 16-byte aligned; the cell words zeroed by the caller) and launches the batch.
void launch_astar_dev(hipStream_t st, const Grid& g, const int32_t* sg4, int64_t nq, int theta,
                      void* work, int64_t far_cap, int64_t* path_xy, int64_t cap,
                      int64_t* path_len, int64_t* stats) {
  const int64_t NC = g.H * g.W;
  unsigned char* p = static_cast<unsigned char*>(work);
  AEntry* bks = reinterpret_cast<AEntry*>(p);
  p += sizeof(AEntry) * (size_t)A_NBK * A_CAP * (size_t)nq;
  AEntry* fars = reinterpret_cast<AEntry*>(p);
  p += sizeof(AEntry) * (size_t)far_cap * (size_t)nq;
  double* gs = reinterpret_cast<double*>(p);
  p += sizeof(double) * (size_t)NC * (size_t)nq;
  uint32_t* cells = reinterpret_cast<uint32_t*>(p);
  hipLaunchKernelGGL(k_astar, dim3((unsigned)nq), dim3(64), 0, st, g, sg4, nq, theta, cells, gs, bks,
                     fars, far_cap, path_xy, cap, path_len, stats);
}

// byte offset of the cell words inside `work` (what the caller zeroes), and their size
void astar_dev_cells(int64_t H, int64_t W, int64_t far_cap, int64_t nq, int64_t* off, int64_t* bytes) {
  *off = (int64_t)sizeof(AEntry) * ((int64_t)A_NBK * A_CAP + far_cap) * nq +
         (int64_t)sizeof(double) * H * W * nq;
  *bytes = (int64_t)sizeof(uint32_t) * H * W * nq;
}

}  // namespace tr
