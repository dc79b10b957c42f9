// Nearest node through a cell grid (rrt.py:155-158 + search.py:13-15): the same answer as nn.hip's
// sweep -- first index of min_i sqrt(fl(fl((qx - x_i)^2) + fl((qy - y_i)^2))) in fp64 -- from the
// few cells around each sample instead of every node.
//
// A tree that covers the map holds a node within a pixel or two of most samples (75k nodes on
// 512 x 512), so the sweep's B x N pairs are almost all wasted: 3e8 pairs per cfg2 batch, 7e10 at
// cfg3, against a few hundred per sample here.
//
// Structure: the nodes as {x, y, index, cell} items grouped by cell, start[c] = first item of
// cell c.  Cells are squares of 2^cs pixels over the map (coordinates clamped into it, which is
// monotone: a node's cell lies on the node's side of every cell boundary); they are numbered along
// the Morton curve of a padded P x P grid, so the 4^L cells of an aligned level-L block (side
// 2^(cs + L)) are one contiguous item range.
//
// The tree only grows, so a build merges the nodes appended since the last one, [built, *hi), into
// the grouped items instead of regrouping all of them (which costs one atomic per node on its
// cell's counter: the few cells where the tree piles up thousands of nodes serialize them, 30 us
// per pass at 90k nodes, and slow every other kernel's atomics meanwhile).  Three launches:
// k_cell_new counts the new nodes by cell (rank within the cell from the atomic), k_cell_scan
// turns the counts into shift[c] = new nodes in cells before c and the new starts, k_cell_move
// copies every old item shift[its cell] places up into the other item array and drops the new
// nodes behind their cells' old items.  Item and start arrays alternate between two buffers; the
// first build after a tree reset, a map change or a new cell size takes every node as new.
//
// Query, sixteen lanes per sample: the 3 x 3 blocks around the sample's block at the lowest level
// that holds a node there; nine lanes load the blocks' item ranges, the group takes the items 64
// at a time (exact fp64, key sqrt(d), lowest index among equal keys: items come in no particular
// order).  The search ends when the best squared distance is safely below the squared distance
// from the sample to the nearest searched side that is not the map's edge (every node beyond such
// a side is farther than the side).  Else every node that can still win lies within the
// candidate's distance R: a second pass takes the blocks that reach into that disc (8 x 8 over its
// box, pruned by their distance).  Where the 3 x 3 blocks are coarse and full (a sample far from
// the tree) they are not searched at all: a descent into the nearest non-empty block finds a
// candidate, and the second pass does the exact work.
#pragma clang fp contract(off)
#include "thetarrt_internal.hpp"
#include "lanegroup.hpp"
#include "diaglog.hpp"
TR_DLOG_EXPORT(tr_diag_log_nng)

namespace tr {

__host__ __device__ inline uint32_t morton_spread(uint32_t v) {   // 16 bits -> even bit positions
  v &= 0xffffu;
  v = (v | (v << 8)) & 0x00ff00ffu;
  v = (v | (v << 4)) & 0x0f0f0f0fu;
  v = (v | (v << 2)) & 0x33333333u;
  v = (v | (v << 1)) & 0x55555555u;
  return v;
}
__host__ __device__ inline uint32_t morton(uint32_t cx, uint32_t cy) {
  return morton_spread(cx) | (morton_spread(cy) << 1);
}

__device__ __forceinline__ uint32_t node_cell(const NNGrid& g, double x, double y) {
  return morton((uint32_t)(db_coord(x, g.xmax) >> g.cs), (uint32_t)(db_coord(y, g.ymax) >> g.cs));
}

// b0 = nodes already grouped (none on a full build), hi = nodes to group
__device__ __forceinline__ void build_range(const NNGrid& g, const int64_t* hi_p, int64_t& b0, int64_t& hi) {
  hi = ld_sc1(hi_p);
  b0 = g.full ? 0 : g.built_old[0];
  if (b0 > hi) b0 = hi;                       // (a tree never shrinks without a full build)
}

__global__ __launch_bounds__(256) void k_cell_new(NNGrid g, const double2* __restrict__ txy,
                                                  const int64_t* __restrict__ hi_p) {
  TR_DLOG_T0;
  int64_t b0, hi;
  build_range(g, hi_p, b0, hi);
  for (int64_t i = b0 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < hi; i += (int64_t)gridDim.x * 256) {
    const double2 p = txy[i];
    g.rank[i - b0] = atomicAdd(g.cnt + node_cell(g, p.x, p.y), 1u);
  }
  TR_DLOG(12);
}

// shift[c] = exclusive prefix of cnt (the new nodes per cell), shift[cells] = their number;
// start[c] = start_old[c] + shift[c] (start_old = 0 on a full build); cnt is zeroed for the next
// build.  Blocks of SCAN_T threads take SCAN_T * SCAN_U consecutive cells each (small blocks: a
// 1024-thread block waited 12 to 19 us for a compute unit beside the expansion kernel); block i
// publishes its cells' sum in part[i], tagged with the build's serial number, and adds up the
// sums of the blocks before it (dispatched before it, so they publish whatever else runs; the
// wait is bounded all the same and reports through *err).
static constexpr int SCAN_T = 256, SCAN_U = 16;
__global__ __launch_bounds__(SCAN_T) void k_cell_scan(NNGrid g) {
  __shared__ uint32_t s_w[SCAN_T / 64];
  __shared__ uint32_t s_b[SCAN_T / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t nc = (int64_t)g.P * g.P;                 // a power of four >= 1
  TR_DLOG_T0;
  const int64_t c = ((int64_t)blockIdx.x * SCAN_T + t) * SCAN_U;
  uint32_t v[SCAN_U], so[SCAN_U];
  if (c + SCAN_U <= nc) {                                // (whole vectors: nc and c are multiples of 4)
#pragma unroll
    for (int u = 0; u < SCAN_U; u += 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(g.cnt + c + u);
      v[u] = q.x; v[u + 1] = q.y; v[u + 2] = q.z; v[u + 3] = q.w;
    }
#pragma unroll
    for (int u = 0; u < SCAN_U; u += 4) {
      uint4 q = make_uint4(0, 0, 0, 0);
      if (!g.full) q = *reinterpret_cast<const uint4*>(g.start_old + c + u);
      so[u] = q.x; so[u + 1] = q.y; so[u + 2] = q.z; so[u + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int u = 0; u < SCAN_U; ++u) {
      v[u] = c + u < nc ? g.cnt[c + u] : 0;
      so[u] = c + u < nc && !g.full ? g.start_old[c + u] : 0;
    }
  }
  uint32_t sum = 0;
#pragma unroll
  for (int u = 0; u < SCAN_U; ++u) sum += v[u];
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t w = __shfl_up(inc, o);
    if (lane >= o) inc += w;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  uint32_t off = inc - sum, tile = 0;
#pragma unroll
  for (int q = 0; q < SCAN_T / 64; ++q) {
    const uint32_t w = s_w[q];
    off += q < wv ? w : 0;
    tile += w;
  }
  const unsigned long long tag = (unsigned long long)g.serial << 32;
  if (t == 0) st_sc1(g.part + blockIdx.x, tag | tile);
  // the sums of the blocks before this one
  uint32_t before = 0;
  const unsigned long long t0 = wall_clock64();
  for (int64_t j = t; j < (int64_t)blockIdx.x; j += SCAN_T) {
    unsigned long long pv = ld_sc1(g.part + j);
    while ((pv >> 32) != g.serial) {
      if (wall_clock64() - t0 > GATE_TICKS) {
        atomicOr(g.err, TR_DDE_GATE);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      pv = ld_sc1(g.part + j);
    }
    before += (uint32_t)pv;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) before += __shfl_xor(before, o);
  if (lane == 0) s_b[wv] = before;
  __syncthreads();
  uint32_t base = 0;
#pragma unroll
  for (int q = 0; q < SCAN_T / 64; ++q) base += s_b[q];
  off += base;
  uint32_t sh[SCAN_U];
#pragma unroll
  for (int u = 0; u < SCAN_U; ++u) {
    sh[u] = off;
    off += v[u];
  }
  if (c + SCAN_U <= nc) {
#pragma unroll
    for (int u = 0; u < SCAN_U; u += 4) {
      *reinterpret_cast<uint4*>(g.shift + c + u) = make_uint4(sh[u], sh[u + 1], sh[u + 2], sh[u + 3]);
      *reinterpret_cast<uint4*>(g.start + c + u) =
          make_uint4(so[u] + sh[u], so[u + 1] + sh[u + 1], so[u + 2] + sh[u + 2], so[u + 3] + sh[u + 3]);
      *reinterpret_cast<uint4*>(g.cnt + c + u) = make_uint4(0, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int u = 0; u < SCAN_U; ++u)
      if (c + u < nc) {
        g.shift[c + u] = sh[u];
        g.start[c + u] = so[u] + sh[u];
        g.cnt[c + u] = 0;
      }
  }
  if (blockIdx.x == 0 && t == 0 && g.far_n) g.far_n[0] = 0;
  if (blockIdx.x == gridDim.x - 1 && t == 0) {
    g.shift[nc] = base + tile;
    g.start[nc] = (g.full ? 0u : g.start_old[nc]) + base + tile;
  }
  TR_DLOG(13);
}

__global__ __launch_bounds__(256) void k_cell_move(NNGrid g, const double2* __restrict__ txy,
                                                   const int64_t* __restrict__ hi_p) {
  TR_DLOG_T0;
  int64_t b0, hi;
  build_range(g, hi_p, b0, hi);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < hi; i += (int64_t)gridDim.x * 256) {
    if (i < b0) {                              // an old item: up by the new nodes of the cells before
      const DBItem it = g.items_old[i];
      g.items[i + g.shift[it.pad]] = it;
    } else {                                   // a new node: behind its cell's old items
      const double2 p = txy[i];
      const uint32_t m = node_cell(g, p.x, p.y);
      const uint32_t at = g.start[m + 1] - (g.shift[m + 1] - g.shift[m]) + g.rank[i - b0];
      g.items[at] = DBItem{p.x, p.y, (int32_t)i, (int32_t)m};
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) g.built_new[0] = hi;
  TR_DLOG(14);
}

constexpr int QG = 16;           // lanes per sample
constexpr int QU = 4;            // items in flight per lane

// The group scans the item ranges its lanes hold (NR per lane: s, n; n = 0: none), flattened:
// slot t belongs to the first lane whose inclusive count passes t (binary search over the group's
// lanes by shuffle), and to the first of that lane's ranges whose end passes it.
template <int G, int NR>
__device__ __forceinline__ void scan_ranges(const Grp<G>& gr, const DBItem* __restrict__ items,
                                            const uint32_t* s, const uint32_t* n, double qx, double qy,
                                            double& rb, double& db, int64_t& ib) {
  uint32_t tot = 0;
#pragma unroll
  for (int r = 0; r < NR; ++r) tot += n[r];
  uint32_t inc = tot;
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const uint32_t w = (uint32_t)__shfl_up((int)inc, o, G);
    if (gr.li >= o) inc += w;
  }
  const uint32_t T = (uint32_t)__shfl((int)inc, G - 1, G);
  // range r of this lane holds slots [end[r] - n[r], end[r]); slot t of it is item base[r] + t
  uint32_t end[NR], base[NR];
  uint32_t e = inc - tot;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    base[r] = s[r] - e;
    e += n[r];
    end[r] = e;
  }
  for (uint32_t t0 = 0; t0 < T; t0 += G * QU) {
    DBItem v[QU];
    bool ok[QU];
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      const uint32_t t = t0 + gr.li + G * u;
      ok[u] = t < T;
      int lo = 0;
#pragma unroll
      for (int step = G / 2; step >= 1; step >>= 1)
        if ((uint32_t)__shfl((int)inc, lo + step - 1, G) <= t) lo += step;
      uint32_t at = (uint32_t)__shfl((int)base[NR - 1], lo, G);
#pragma unroll
      for (int r = NR - 2; r >= 0; --r) {
        const uint32_t er = (uint32_t)__shfl((int)end[r], lo, G), br = (uint32_t)__shfl((int)base[r], lo, G);
        if (t < er) at = br;
      }
      v[u] = items[ok[u] ? at + t : 0];
    }
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      const double a = qx - v[u].x, c = qy - v[u].y;
      const double d = a * a + c * c;
      const double rt = sqrt(d);
      if (ok[u] && (rt < rb || (rt == rb && (int64_t)v[u].idx < ib))) { rb = rt; db = d; ib = v[u].idx; }
    }
  }
  // group argmin of (key, index)
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) {
    const double ro = __shfl_xor(rb, o, G), dq = __shfl_xor(db, o, G);
    const int64_t io = __shfl_xor(ib, o, G);
    if (io >= 0 && (ib < 0 || ro < rb || (ro == rb && io < ib))) { rb = ro; db = dq; ib = io; }
  }
}

// lane of the group holding the least v (the lowest such lane)
template <int G>
__device__ __forceinline__ int group_argmin(const Grp<G>& gr, double v) {
  int w = gr.li;
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) {
    const double vo = __shfl_xor(v, o, G);
    const int wo = __shfl_xor(w, o, G);
    if (vo < v || (vo == v && wo < w)) { v = vo; w = wo; }
  }
  return w;
}

constexpr uint32_t DESCEND = 256;   // nodes in the 3 x 3 blocks past which they are not all searched
constexpr uint32_t HEAVY = 256;     // nodes of a second pass past which the whole block scans them

// A second pass too long for sixteen lanes (a sample far from every node, or one whose disc reaches
// a cell where the tree piles up thousands of nodes): parked in LDS for the block's 256 threads,
// once its other samples are done.  blk = the pass's non-empty blocks within reach (level K, x |
// y << 16), R2 = the squared reach, rb / db / ib = the sample's best so far.  The block refines
// the blocks two levels at a time (sixteen children each, kept when they hold a node within
// reach: what survives is the ring around the disc at ever finer grain, the disc itself being
// empty) until few enough nodes are left, then scans them, or hands the sample to the far list.
struct HeavyJob {
  double qx, qy, rb, db, R2;
  int64_t ib, j;
  int32_t K, nblk;
  uint32_t blk[64];
};
constexpr int LCAP = 1024;          // blocks of a refined pass
constexpr uint32_t REFINED = 1024;  // nodes below which a pass is scanned as it stands

// One group of QG lanes per sample (most samples settle on the few dozen nodes of the nine cells
// around them: a whole wave per sample spent four times the instructions on the same loads, and
// the expansion kernel running beside this one pays for every instruction issued here).
__global__ __launch_bounds__(256) void k_nn_grid(NNGrid g, const int2* __restrict__ qxy,
                                                 const int32_t* __restrict__ live, int64_t B,
                                                 int64_t* __restrict__ out, double* __restrict__ dout,
                                                 ResolvePub pub, int32_t sc1) {
  constexpr int G = QG;
  __shared__ HeavyJob s_job[256 / G];
  __shared__ int s_nj;
  const Grp<G> gr(threadIdx.x & 63);
  const int li = gr.li;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const bool act = j < B;
  TR_DLOG_T0;
  if (threadIdx.x == 0) s_nj = 0;
  __syncthreads();
  double rb = INFINITY, db = INFINITY;
  int64_t ib = -1;
  bool parked = false;                           // the sample's result comes from the block scan
  if (act && (!live || live[j] == 1)) {          // uniform in the group (other samples never expand)
    const int2 q = qxy[j];
    const double qx = (double)q.x, qy = (double)q.y;
    // the sample's cell (clamped like the nodes'); levels count up from single cells
    const int32_t fx = (q.x < 0 ? 0 : (q.x > g.xmax ? g.xmax : q.x)) >> g.cs;
    const int32_t fy = (q.y < 0 ? 0 : (q.y > g.ymax ? g.ymax : q.y)) >> g.cs;
    const int Lmax = 31 - __clz(g.P);            // P = 2^Lmax: one block at level Lmax
    // squared distance to the nearest point a node of block (X, Y) of level lev can be at:
    // x >= its low side unless the block touches the low edge of the map, x < its high side
    // unless it reaches the high edge (clamped nodes lie beyond those)
    auto block_d2 = [&](int32_t X, int32_t Y, int lev) {
      const int shk = g.cs + lev;
      const double lox = (double)((int64_t)X << shk), hix = (double)((int64_t)(X + 1) << shk);
      const double loy = (double)((int64_t)Y << shk), hiy = (double)((int64_t)(Y + 1) << shk);
      double dx = 0.0, dy = 0.0;
      if (X > 0 && qx < lox) dx = lox - qx;
      if (hix <= (double)g.xmax && qx > hix) dx = qx - hix;
      if (Y > 0 && qy < loy) dy = loy - qy;
      if (hiy <= (double)g.ymax && qy > hiy) dy = qy - hiy;
      return dx * dx + dy * dy;
    };
    for (int L = 0;;) {
      const int32_t PL = g.P >> L, bx = fx >> L, by = fy >> L;     // blocks per side, the sample's
      uint32_t s = 0, n = 0;                     // lanes 0-8: the 3 x 3 blocks' item ranges
      if (li < 9) {
        const int32_t cx = bx + li % 3 - 1, cy = by + li / 3 - 1;
        if (cx >= 0 && cy >= 0 && cx < PL && cy < PL) {
          const uint32_t m = morton((uint32_t)cx, (uint32_t)cy) << (2 * L);
          s = g.start[m];
          n = g.start[m + (1u << (2 * L))] - s;
        }
      }
      uint32_t TL = n;                           // nodes in the level's 3 x 3 blocks
#pragma unroll
      for (int o = G / 2; o >= 1; o >>= 1) TL += (uint32_t)__shfl_xor((int)TL, o, G);
      if (TL == 0 && L < Lmax) {                 // nothing around: two levels up (any level serves)
        L = L + 2 < Lmax ? L + 2 : Lmax;
        continue;
      }
      bool square = true;                        // the 3 x 3 blocks were searched
      double dcand;                              // squared distance of a node near the sample
      if (TL > DESCEND) {
        // Blocks full of nodes, nearly all of them far away (coarse blocks around a sample far
        // from the tree), or a cell where the tree piles up: not searched here.  A node near the
        // sample is found by descending into the nearest block that holds one, two levels (4 x 4
        // blocks, one per lane) at a time, down to a cell; its first node bounds the search.
        square = false;
        double v = INFINITY;
        if (n > 0) v = block_d2(bx + li % 3 - 1, by + li / 3 - 1, L);
        int w = group_argmin(gr, v);
        int32_t X = bx + w % 3 - 1, Y = by + w / 3 - 1;
        uint32_t sw = (uint32_t)__shfl((int)s, w, G);
        for (int Lc = L; Lc > 0;) {
          const int Ld = Lc > 2 ? Lc - 2 : 0, sb = Lc - Ld;
          uint32_t s2 = 0, n2 = 0;
          int32_t X2 = 0, Y2 = 0;
          v = INFINITY;
          if (li < (1 << (2 * sb))) {
            X2 = (X << sb) + (li & ((1 << sb) - 1));
            Y2 = (Y << sb) + (li >> sb);
            const uint32_t m = morton((uint32_t)X2, (uint32_t)Y2) << (2 * Ld);
            s2 = g.start[m];
            n2 = g.start[m + (1u << (2 * Ld))] - s2;
            if (n2 > 0) v = block_d2(X2, Y2, Ld);
          }
          w = group_argmin(gr, v);
          X = __shfl(X2, w, G);
          Y = __shfl(Y2, w, G);
          sw = (uint32_t)__shfl((int)s2, w, G);
          Lc = Ld;
        }
        const DBItem it = g.items[sw];
        const double a = qx - it.x, c = qy - it.y;
        dcand = a * a + c * c;
      } else {
        scan_ranges<G, 1>(gr, g.items, &s, &n, qx, qy, rb, db, ib);
        // the searched square [x0, x1) x [y0, y1) in pixels; a side at or beyond the map's edge is
        // open (clamping put every node beyond it into the edge cells, which were searched)
        const int sh = g.cs + L;
        const int64_t x0 = (int64_t)(bx - 1) << sh, x1 = (int64_t)(bx + 2) << sh;
        const int64_t y0 = (int64_t)(by - 1) << sh, y1 = (int64_t)(by + 2) << sh;
        double rho = INFINITY;
        if (x0 > 0) rho = fmin(rho, qx - (double)x0);
        if (x1 <= g.xmax) rho = fmin(rho, (double)x1 - qx);
        if (y0 > 0) rho = fmin(rho, qy - (double)y0);
        if (y1 <= g.ymax) rho = fmin(rho, (double)y1 - qy);
        // A node not searched has its clamped floor(coordinate) beyond a closed side: below x0
        // means x < x0 <= qx - rho, at or above x1 means x >= x1 >= qx + rho (the sample's own
        // clamped coordinate lies a whole block inside the square, and clamping moved it towards
        // the map), so its d >= rho^2 in the same rounded arithmetic (rho is an integer).  The
        // margin keeps the two keys sqrt(d) apart, where a tie would go to the lower index.
        if (!(rho < INFINITY) || ib < 0) break;  // the whole map was searched (or holds no node)
        if (db * (1.0 + 1e-12) < rho * rho) break;
        dcand = db;
      }
      // Every node that can beat or tie the candidate lies within R of the sample, i.e. has its
      // clamped floor(coordinates) between those of q - R and q + R.  The blocks of the coarsest
      // level that covers that box with 8 x 8, four per lane; blocks inside a searched square and
      // blocks farther than R are dropped.
      const double R = sqrt(dcand) * (1.0 + 1e-12) + 1e-9;
      const int32_t cx0 = db_coord(qx - R, g.xmax) >> g.cs, cx1 = db_coord(qx + R, g.xmax) >> g.cs;
      const int32_t cy0 = db_coord(qy - R, g.ymax) >> g.cs, cy1 = db_coord(qy + R, g.ymax) >> g.cs;
      int K = 0;
      while ((cx1 >> K) - (cx0 >> K) >= 8 || (cy1 >> K) - (cy0 >> K) >= 8) ++K;
      const int32_t X0 = cx0 >> K, nbx = (cx1 >> K) - X0 + 1;
      const int32_t Y0 = cy0 >> K, nby = (cy1 >> K) - Y0 + 1;
      constexpr int NR = 64 / G;
      uint32_t s4[NR], n4[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int bq = li + G * r;
        s4[r] = n4[r] = 0;
        if (bq < nbx * nby) {
          const int32_t X = X0 + bq % nbx, Y = Y0 + bq / nbx;
          const int64_t ax0 = (int64_t)(bx - 1) << L, ax1 = (int64_t)(bx + 2) << L;   // the square, in cells
          const int64_t ay0 = (int64_t)(by - 1) << L, ay1 = (int64_t)(by + 2) << L;
          const bool inside = square && ((int64_t)X << K) >= ax0 && ((int64_t)(X + 1) << K) <= ax1 &&
                              ((int64_t)Y << K) >= ay0 && ((int64_t)(Y + 1) << K) <= ay1;
          if (!inside && block_d2(X, Y, K) <= R * R * (1.0 + 1e-12)) {
            const uint32_t m = morton((uint32_t)X, (uint32_t)Y) << (2 * K);
            s4[r] = g.start[m];
            n4[r] = g.start[m + (1u << (2 * K))] - s4[r];
          }
        }
      }
      uint32_t tot = 0;
#pragma unroll
      for (int r = 0; r < NR; ++r) tot += n4[r];
      uint32_t TB = tot;
#pragma unroll
      for (int o = G / 2; o >= 1; o >>= 1) TB += (uint32_t)__shfl_xor((int)TB, o, G);
      if (TB <= HEAVY) {
        scan_ranges<G, NR>(gr, g.items, s4, n4, qx, qy, rb, db, ib);
      } else {                                   // parked for the block: its non-empty blocks
        int slot = 0;
        if (li == 0) slot = atomicAdd(&s_nj, 1);
        slot = __shfl(slot, 0, G);
        HeavyJob& hj = s_job[slot];
        uint32_t kept = 0;
#pragma unroll
        for (int r = 0; r < NR; ++r) kept += n4[r] > 0;
        uint32_t inc = kept;
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
          const uint32_t w = (uint32_t)__shfl_up((int)inc, o, G);
          if (li >= o) inc += w;
        }
        uint32_t at = inc - kept;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int bq = li + G * r;
          if (n4[r] > 0) hj.blk[at++] = (uint32_t)(X0 + bq % nbx) | ((uint32_t)(Y0 + bq / nbx) << 16);
        }
        if (li == G - 1) hj.nblk = (int32_t)inc;
        if (li == 0) {
          hj.qx = qx; hj.qy = qy; hj.rb = rb; hj.db = db; hj.ib = ib; hj.j = j;
          hj.R2 = R * R * (1.0 + 1e-12);
          hj.K = K;
        }
        parked = true;
      }
      break;
    }
  }
  __syncthreads();
  const int nj = s_nj;                           // block-uniform
  if (nj > 0) {
    __shared__ uint32_t s_list[2][LCAP], s_inc[LCAP], s_base[LCAP];
    __shared__ uint32_t s_len, s_tot;
    __shared__ uint32_t s_ws[4];
    __shared__ double s_rr[4], s_rd[4];
    __shared__ int64_t s_ri[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, t = threadIdx.x;
    for (int q = 0; q < nj; ++q) {
      const HeavyJob& hj = s_job[q];
      const double qx = hj.qx, qy = hj.qy, R2 = hj.R2;
      auto block_d2 = [&](int32_t X, int32_t Y, int lev) {          // (as in the groups' passes)
        const int shk = g.cs + lev;
        const double lox = (double)((int64_t)X << shk), hix = (double)((int64_t)(X + 1) << shk);
        const double loy = (double)((int64_t)Y << shk), hiy = (double)((int64_t)(Y + 1) << shk);
        double dx = 0.0, dy = 0.0;
        if (X > 0 && qx < lox) dx = lox - qx;
        if (hix <= (double)g.xmax && qx > hix) dx = qx - hix;
        if (Y > 0 && qy < loy) dy = loy - qy;
        if (hiy <= (double)g.ymax && qy > hiy) dy = qy - hiy;
        return dx * dx + dy * dy;
      };
      int level = hj.K, cur = 0;
      uint32_t len = (uint32_t)hj.nblk;
      for (uint32_t i = t; i < len; i += 256) s_list[0][i] = hj.blk[i];
      uint32_t total = 0;
      for (;;) {
        // the blocks' item ranges and the nodes they hold
        if (t == 0) { s_tot = 0; s_len = 0; }
        __syncthreads();
        uint32_t mine = 0;
        for (uint32_t i = t; i < len; i += 256) {
          const uint32_t b = s_list[cur][i];
          const uint32_t m = morton(b & 0xffffu, b >> 16) << (2 * level);
          const uint32_t s0 = g.start[m], n0 = g.start[m + (1u << (2 * level))] - s0;
          s_base[i] = s0;
          s_inc[i] = n0;
          mine += n0;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) mine += (uint32_t)__shfl_xor((int)mine, o);
        if (lane == 0 && mine) atomicAdd(&s_tot, mine);
        __syncthreads();
        total = s_tot;
        if (level == 0 || total <= REFINED) break;
        // the children that hold a node within reach
        const int sb = level >= 2 ? 2 : 1, nl = level - sb, nch = 1 << (2 * sb);
        for (uint32_t i = t; i < len * nch; i += 256) {
          const uint32_t b = s_list[cur][i >> (2 * sb)], ch = i & (nch - 1);
          const int32_t X2 = (int32_t)((b & 0xffffu) << sb) + (int32_t)(ch & ((1u << sb) - 1));
          const int32_t Y2 = (int32_t)((b >> 16) << sb) + (int32_t)(ch >> sb);
          const uint32_t m = morton((uint32_t)X2, (uint32_t)Y2) << (2 * nl);
          const uint32_t n2 = g.start[m + (1u << (2 * nl))] - g.start[m];
          if (n2 > 0 && block_d2(X2, Y2, nl) <= R2) {
            const uint32_t pos = atomicAdd(&s_len, 1u);
            if (pos < LCAP) s_list[cur ^ 1][pos] = (uint32_t)X2 | ((uint32_t)Y2 << 16);
          }
        }
        __syncthreads();
        const uint32_t nlen = s_len;
        __syncthreads();                         // (s_len is reset at the top of the loop)
        if (nlen > LCAP) break;                  // too many to list: scanned at this level
        cur ^= 1;
        len = nlen;
        level = nl;
      }
      if (g.far_n && total > g.far_min) {        // left to the sweep over the far list
        if (t == 0) {
          const int32_t hq = atomicAdd(g.far_n, 1);
          g.far_j[hq] = (int32_t)hj.j;
          g.far_q[hq] = make_int2((int)qx, (int)qy);
        }
        __syncthreads();
        continue;
      }
      // inclusive counts over the list (four entries per thread), then slot t of the pass is item
      // s_base[i] + t of the first entry i whose count passes t
      {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t i = 4 * t + u;
          v[u] = i < len ? s_inc[i] : 0;
          sum += v[u];
        }
        uint32_t inc = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t w = (uint32_t)__shfl_up((int)inc, o);
          if (lane >= o) inc += w;
        }
        if (lane == 63) s_ws[wv] = inc;
        __syncthreads();
        uint32_t e = inc - sum;
        for (int w = 0; w < wv; ++w) e += s_ws[w];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t i = 4 * t + u;
          if (i < len) {
            s_base[i] -= e;
            e += v[u];
            s_inc[i] = e;
          }
        }
        __syncthreads();
      }
      const uint32_t T = total;
      double r1 = INFINITY, d1 = INFINITY;
      int64_t i1 = -1;
      for (uint32_t t0 = 0; t0 < T; t0 += 256 * QU) {
        DBItem v[QU];
        bool ok[QU];
#pragma unroll
        for (int u = 0; u < QU; ++u) {
          const uint32_t ts = t0 + t + 256 * u;
          ok[u] = ts < T;
          uint32_t lo = 0;
#pragma unroll
          for (uint32_t step = LCAP / 2; step >= 1; step >>= 1)
            if (lo + step - 1 < len && s_inc[lo + step - 1] <= ts) lo += step;
          v[u] = g.items[ok[u] ? s_base[lo < len ? lo : 0] + ts : 0];
        }
#pragma unroll
        for (int u = 0; u < QU; ++u) {
          const double a = qx - v[u].x, c = qy - v[u].y;
          const double d = a * a + c * c;
          const double rt = sqrt(d);
          if (ok[u] && (rt < r1 || (rt == r1 && (int64_t)v[u].idx < i1))) { r1 = rt; d1 = d; i1 = v[u].idx; }
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const double ro = __shfl_xor(r1, o), dq = __shfl_xor(d1, o);
        const int64_t io = __shfl_xor(i1, o);
        if (io >= 0 && (i1 < 0 || ro < r1 || (ro == r1 && io < i1))) { r1 = ro; d1 = dq; i1 = io; }
      }
      if (lane == 0) { s_rr[wv] = r1; s_rd[wv] = d1; s_ri[wv] = i1; }
      __syncthreads();
      if (t == 0) {
        double r0 = hj.rb, d0 = hj.db;
        int64_t i0 = hj.ib;
        for (int w = 0; w < 4; ++w) {
          const double ro = s_rr[w];
          const int64_t io = s_ri[w];
          if (io >= 0 && (i0 < 0 || ro < r0 || (ro == r0 && io < i0))) { r0 = ro; d0 = s_rd[w]; i0 = io; }
        }
        if (pub.flag || sc1) {
          st_sc1(out + hj.j, i0);
          if (dout) st_sc1(dout + hj.j, d0);
        } else {
          out[hj.j] = i0;
          if (dout) dout[hj.j] = d0;
        }
      }
      __syncthreads();
    }
  }
  if (!pub.flag) {
    if (act && li == 0 && !parked) {
      if (sc1) {
        st_sc1(out + j, ib);
        if (dout) st_sc1(dout + j, db);
      } else {
        out[j] = ib;
        if (dout) dout[j] = db;
      }
    }
    TR_DLOG(11);
    return;
  }
  // published for another stream's kernel before this one ends: sc1 stores, every wave waits for
  // its own, the last block stores the flag (thetarrt_internal.hpp: st_sc1)
  if (act && li == 0 && !parked) {
    st_sc1(out + j, ib);
    if (dout) st_sc1(dout + j, db);
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
  TR_DLOG(11);
}


// Cell side for about 12 nodes per cell (1 .. 2^8 pixels), the padded grid and the buffer sizes.
void nn_grid_plan(NNGrid& g, int64_t H, int64_t W, int64_t n_ub) {
  const double side = std::sqrt(12.0 * (double)H * (double)W / (double)std::max<int64_t>(n_ub, 1));
  int cs = 0;
  while (cs < 8 && (double)(2 << cs) <= side) ++cs;
  const int64_t ncx = ((H - 1) >> cs) + 1, ncy = ((W - 1) >> cs) + 1;
  int64_t P = 1;
  while (P < ncx || P < ncy) P <<= 1;
  g.cs = cs;
  g.P = (int32_t)P;
  g.xmax = (int32_t)H - 1;
  g.ymax = (int32_t)W - 1;
}

int64_t nn_grid_scan_blocks(const NNGrid& g) {
  const int64_t per = (int64_t)SCAN_T * SCAN_U, nc = (int64_t)g.P * g.P;
  return (nc + per - 1) / per;
}

void nn_grid_build(hipStream_t st, const NNGrid& g, const double2* txy, const int64_t* hi_p,
                   int64_t n_ub) {
  const unsigned blocks = (unsigned)std::min<int64_t>(std::max<int64_t>((n_ub + 255) / 256, 1), 2048);
  hipLaunchKernelGGL(k_cell_new, dim3(blocks), dim3(256), 0, st, g, txy, hi_p);
  const int64_t per = (int64_t)SCAN_T * SCAN_U, nc = (int64_t)g.P * g.P;
  hipLaunchKernelGGL(k_cell_scan, dim3((unsigned)((nc + per - 1) / per)), dim3(SCAN_T), 0, st, g);
  hipLaunchKernelGGL(k_cell_move, dim3(blocks), dim3(256), 0, st, g, txy, hi_p);
}

void nn_grid_query(hipStream_t st, const NNGrid& g, const int2* qxy, const int32_t* live, int64_t B,
                   int64_t* out, double* dout, ResolvePub pub, bool sc1) {
  if (B <= 0) return;
  const int64_t per = 256 / QG;                  // samples per block
  hipLaunchKernelGGL(k_nn_grid, dim3((unsigned)((B + per - 1) / per)), dim3(256), 0, st, g, qxy, live,
                     B, out, dout, pub, sc1 ? 1 : 0);
}

}  // namespace tr
