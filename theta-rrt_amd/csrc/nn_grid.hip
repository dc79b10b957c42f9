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
// Query, one wave per sample: level L = 0, 1, ...: the 3 x 3 level-L blocks around the sample's
// block; nine lanes load the blocks' item ranges, the wave takes the items 64 at a time (exact
// fp64, key sqrt(d), lowest index among equal keys: items come in no particular order); the search
// ends when the best squared distance is safely below the squared distance from the sample to the
// nearest searched side that is not the map's edge (every node beyond such a side is farther than
// the side), else the next level doubles the blocks.  Far samples climb levels: the last level is
// the whole map.  Corner cells of clipped samples hold thousands of nodes: a wave reads them 256
// items per round.
#pragma clang fp contract(off)
#include "thetarrt_internal.hpp"
#include "diaglog.hpp"
TR_DLOG_EXPORT(tr_diag_log_nng)

namespace tr {

namespace {

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
constexpr int SCAN_T = 256, SCAN_U = 16;
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

constexpr int QW = 4;            // samples (waves) per query block
constexpr int QU = 4;            // items in flight per lane

// The wave scans the item ranges its lanes hold (s, n; n = 0: none), flattened: slot t belongs to
// the first lane whose inclusive count passes t (binary search over the lanes by shuffle).
__device__ __forceinline__ void scan_ranges(const DBItem* __restrict__ items, uint32_t s, uint32_t n,
                                            int lane, double qx, double qy, double& rb, double& db,
                                            int64_t& ib) {
  uint32_t inc = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t w = __shfl_up(inc, o);
    if (lane >= o) inc += w;
  }
  const uint32_t T = (uint32_t)__shfl((int)inc, 63);
  const uint32_t base = s - (inc - n);           // the lane's range holds slots [inc - n, inc)
  for (uint32_t t0 = 0; t0 < T; t0 += 64 * QU) {
    DBItem v[QU];
    bool ok[QU];
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      const uint32_t t = t0 + lane + 64 * u;
      ok[u] = t < T;
      int lo = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1)
        if ((uint32_t)__shfl((int)inc, lo + step - 1) <= t) lo += step;
      const uint32_t at = (uint32_t)__shfl((int)base, lo) + t;
      v[u] = items[ok[u] ? at : 0];
    }
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      const double a = qx - v[u].x, c = qy - v[u].y;
      const double d = a * a + c * c;
      const double rt = sqrt(d);
      if (ok[u] && (rt < rb || (rt == rb && (int64_t)v[u].idx < ib))) { rb = rt; db = d; ib = v[u].idx; }
    }
  }
  // wave argmin of (key, index)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const double ro = __shfl_xor(rb, o), dq = __shfl_xor(db, o);
    const int64_t io = __shfl_xor(ib, o);
    if (io >= 0 && (ib < 0 || ro < rb || (ro == rb && io < ib))) { rb = ro; db = dq; ib = io; }
  }
}

__global__ __launch_bounds__(64 * QW) void k_nn_grid(NNGrid g, const int2* __restrict__ qxy,
                                                     const int32_t* __restrict__ live, int64_t B,
                                                     int64_t* __restrict__ out,
                                                     double* __restrict__ dout, ResolvePub pub) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * QW + (threadIdx.x >> 6);
  const bool act = j < B;
  TR_DLOG_T0;
  double rb = INFINITY, db = INFINITY;
  int64_t ib = -1;
  if (act && (!live || live[j] == 1)) {          // uniform in the wave (other samples never expand)
    const int2 q = qxy[j];
    const double qx = (double)q.x, qy = (double)q.y;
    // the sample's cell (clamped like the nodes'); levels count up from single cells
    const int32_t fx = (q.x < 0 ? 0 : (q.x > g.xmax ? g.xmax : q.x)) >> g.cs;
    const int32_t fy = (q.y < 0 ? 0 : (q.y > g.ymax ? g.ymax : q.y)) >> g.cs;
    for (int L = 0;; ++L) {
      const int32_t PL = g.P >> L, bx = fx >> L, by = fy >> L;     // blocks per side, the sample's
      uint32_t s = 0, n = 0;                     // lanes 0-8: the 3 x 3 blocks' item ranges
      if (lane < 9) {
        const int32_t cx = bx + lane % 3 - 1, cy = by + lane / 3 - 1;
        if (cx >= 0 && cy >= 0 && cx < PL && cy < PL) {
          const uint32_t m = morton((uint32_t)cx, (uint32_t)cy) << (2 * L);
          s = g.start[m];
          n = g.start[m + (1u << (2 * L))] - s;
        }
      }
      scan_ranges(g.items, s, n, lane, qx, qy, rb, db, ib);
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
      // A node not searched has its clamped floor(coordinate) beyond a closed side: below x0 means
      // x < x0 <= qx - rho, at or above x1 means x >= x1 >= qx + rho (the sample's own clamped
      // coordinate lies a whole block inside the square, and clamping moved it towards the map), so
      // its d >= rho^2 in the same rounded arithmetic (rho is an integer).  The margin keeps the
      // two keys sqrt(d) apart, where a tie would go to the lower index.
      if (!(rho < INFINITY)) break;              // the whole map was searched
      if (ib < 0) continue;                      // nothing yet: the next level (it ends at the map)
      if (db * (1.0 + 1e-12) < rho * rho) break;
      // A candidate that the square does not settle: every node that can beat or tie it lies
      // within R of the sample, i.e. has its clamped floor(coordinates) between those of q - R and
      // q + R.  The blocks of the coarsest level that covers that box with 8 x 8, one per lane;
      // blocks inside the square (searched) and blocks farther than R are dropped.
      const double R = sqrt(db) * (1.0 + 1e-12) + 1e-9;
      const int32_t cx0 = db_coord(qx - R, g.xmax) >> g.cs, cx1 = db_coord(qx + R, g.xmax) >> g.cs;
      const int32_t cy0 = db_coord(qy - R, g.ymax) >> g.cs, cy1 = db_coord(qy + R, g.ymax) >> g.cs;
      int K = 0;
      while ((cx1 >> K) - (cx0 >> K) >= 8 || (cy1 >> K) - (cy0 >> K) >= 8) ++K;
      const int32_t X0 = cx0 >> K, nbx = (cx1 >> K) - X0 + 1;
      const int32_t Y0 = cy0 >> K, nby = (cy1 >> K) - Y0 + 1;
      s = n = 0;
      if (lane < nbx * nby) {
        const int32_t X = X0 + lane % nbx, Y = Y0 + lane / nbx;
        const int64_t ax0 = (int64_t)(bx - 1) << L, ax1 = (int64_t)(bx + 2) << L;   // the square, in cells
        const int64_t ay0 = (int64_t)(by - 1) << L, ay1 = (int64_t)(by + 2) << L;
        const bool inside = ((int64_t)X << K) >= ax0 && ((int64_t)(X + 1) << K) <= ax1 &&
                            ((int64_t)Y << K) >= ay0 && ((int64_t)(Y + 1) << K) <= ay1;
        // the nearest a node of the block can be: x >= lox unless the block touches the low edge
        // of the map, x < hix unless it reaches the high edge (clamped nodes lie beyond those)
        const int shk = g.cs + K;
        const double lox = (double)((int64_t)X << shk), hix = (double)((int64_t)(X + 1) << shk);
        const double loy = (double)((int64_t)Y << shk), hiy = (double)((int64_t)(Y + 1) << shk);
        double dx = 0.0, dy = 0.0;
        if (X > 0 && qx < lox) dx = lox - qx;
        if (hix <= (double)g.xmax && qx > hix) dx = qx - hix;
        if (Y > 0 && qy < loy) dy = loy - qy;
        if (hiy <= (double)g.ymax && qy > hiy) dy = qy - hiy;
        if (!inside && dx * dx + dy * dy <= R * R * (1.0 + 1e-12)) {
          const uint32_t m = morton((uint32_t)X, (uint32_t)Y) << (2 * K);
          s = g.start[m];
          n = g.start[m + (1u << (2 * K))] - s;
        }
      }
      scan_ranges(g.items, s, n, lane, qx, qy, rb, db, ib);
      break;
    }
  }
  if (!pub.flag) {
    if (act && lane == 0) {
      out[j] = ib;
      if (dout) dout[j] = db;
    }
    TR_DLOG(11);
    return;
  }
  // published for another stream's kernel before this one ends: sc1 stores, every wave waits for
  // its own, the last block stores the flag (thetarrt_internal.hpp: st_sc1)
  if (act && lane == 0) {
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

}  // namespace

// Cell side for about 12 nodes per cell (2^2 .. 2^8 pixels), the padded grid and the buffer sizes.
void nn_grid_plan(NNGrid& g, int64_t H, int64_t W, int64_t n_ub) {
  const double side = std::sqrt(12.0 * (double)H * (double)W / (double)std::max<int64_t>(n_ub, 1));
  int cs = 2;
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
                   int64_t* out, double* dout, ResolvePub pub) {
  if (B <= 0) return;
  hipLaunchKernelGGL(k_nn_grid, dim3((unsigned)((B + QW - 1) / QW)), dim3(64 * QW), 0, st, g, qxy,
                     live, B, out, dout, pub);
}

}  // namespace tr
