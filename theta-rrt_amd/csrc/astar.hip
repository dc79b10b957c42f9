// A* / lazy Theta* (search.py:221-307) on the host: the call for ONE search (astar_dev.hip runs
// batches of searches resident on the GPU).
//
// The search itself is the reference's, step for step: 8-connected neighbours in
// itertools.product([-1, 0, 1], repeat=2) order (search.py:184-194), a priority queue of (f, node)
// tuples popped in tuple order (Python's PriorityQueue = heapq: f, then x, then y), stale entries
// skipped when their node is closed, gScore / cameFrom updates and the Theta* parent shortcut
// (search.py:294-304) in the same order, fp64 sums of math.sqrt of exact integer squares.
//
// Lazy Theta* tests lineofsight(current, cameFrom[current]) when a node is popped (search.py:258-263):
// through `los` (the host grid's closed-form Bresenham), one pair at a time: a map2 ray is ~100
// pixels, a fraction of a microsecond on the host against tens of microseconds for a GPU round trip.
#include <stdint.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>
#include <math.h>

#include "thetarrt_internal.hpp"

namespace tr {

namespace {

struct PQItem {
  double f;
  int32_t x, y;
};

// heap "less" for a min-queue on (f, x, y): std heaps keep the largest on top, so invert.
struct PQAfter {
  bool operator()(const PQItem& a, const PQItem& b) const {
    if (a.f != b.f) return a.f > b.f;
    if (a.x != b.x) return a.x > b.x;
    return a.y > b.y;
  }
};

inline double l2i(int64_t x0, int64_t y0, int64_t x1, int64_t y1) {   // search.py:13-15, ints
  const int64_t dx = x1 - x0, dy = y1 - y0;
  return sqrt((double)(dx * dx + dy * dy));
}

}  // namespace

int astar_run(const uint8_t* free_yx, int64_t H, int64_t W, int64_t sx, int64_t sy, int64_t gx,
              int64_t gy, bool theta, const LosFn& los,
              std::vector<int64_t>& path, AStarStats& st, std::string& msg) {
  path.clear();
  st = AStarStats{};
  // valid: 0 <= x < shape[0], 0 <= y < shape[1] (search.py:17-24); freespace reads imarray[y][x]
  auto valid = [&](int64_t x, int64_t y) { return x >= 0 && y >= 0 && x < H && y < W; };
  int index_err = 0;
  auto freeat = [&](int64_t x, int64_t y) -> bool {
    if (!valid(x, y)) return false;
    if (y >= H || x >= W) {            // imarray[y][x] past the array: the reference's IndexError
      index_err = 1;
      return false;
    }
    return free_yx[y * W + x] != 0;
  };
  if (!valid(sx, sy) || !valid(gx, gy)) {
    st.status = 1;                     // "Start or goal is not valid. Error."
    return TR_OK;
  }
  const bool fs = freeat(sx, sy), fg = freeat(gx, gy);
  if (index_err) { msg = "IndexError: index out of bounds (imarray[y][x])"; return TR_E_INDEX; }
  if (!fs || !fg) {
    st.status = 2;                     // "Start or goal is inside an obstacle. Error."
    return TR_OK;
  }
  // node id = x * W + y over the valid box [0, H) x [0, W)
  const int64_t NN = H * W;
  auto id = [&](int64_t x, int64_t y) { return x * W + y; };
  std::vector<double> g((size_t)NN, 0.0);
  std::vector<int64_t> came((size_t)NN, -1);
  std::vector<uint8_t> state((size_t)NN, 0);   // bit 0 open, bit 1 closed, bit 2 has g
  std::vector<PQItem> heap;
  heap.reserve(1 << 16);
  PQAfter after;
  auto push = [&](double f, int64_t x, int64_t y) {
    heap.push_back(PQItem{f, (int32_t)x, (int32_t)y});
    std::push_heap(heap.begin(), heap.end(), after);
  };
  int64_t nb[8][2];
  auto neighbors = [&](int64_t x, int64_t y) -> int {   // search.py:184-194 order
    int n = 0;
    for (int a = -1; a <= 1; ++a)
      for (int b = -1; b <= 1; ++b) {
        if (a == 0 && b == 0) continue;
        const int64_t cx = x - a, cy = y - b;
        if (valid(cx, cy) && freeat(cx, cy)) { nb[n][0] = cx; nb[n][1] = cy; ++n; }
      }
    return n;
  };
  auto h = [&](int64_t x, int64_t y) { return l2i(x, y, gx, gy); };

  const int64_t s = id(sx, sy);
  g[s] = 0.0;
  state[s] |= 4;
  int n0 = neighbors(sx, sy);
  for (int k = 0; k < n0; ++k) {
    const int64_t v = id(nb[k][0], nb[k][1]);
    g[v] = l2i(sx, sy, nb[k][0], nb[k][1]);
    state[v] |= 4 | 1;
    came[v] = s;
    push(g[v] + h(nb[k][0], nb[k][1]), nb[k][0], nb[k][1]);
  }
  state[s] |= 2;
  int64_t closed = 1;
  if (index_err) { msg = "IndexError: index out of bounds (imarray[y][x])"; return TR_E_INDEX; }

  while (!heap.empty()) {
    std::pop_heap(heap.begin(), heap.end(), after);
    const PQItem it = heap.back();
    heap.pop_back();
    const int64_t cx = it.x, cy = it.y, c = id(cx, cy);
    if (state[c] & 2) continue;         // stale copy (search.py:250-255)
    if (theta) {
      const int64_t p = came[c];
      bool clear = false;
      if (int e = los(cx, cy, p / W, p % W, &clear)) return e;
      st.los_segments++;
      if (!clear) {                    // re-parent to the best closed neighbour (search.py:260-263)
        const int n = neighbors(cx, cy);
        int best = -1;
        double bv = 0.0;
        for (int k = 0; k < n; ++k) {
          const int64_t v = id(nb[k][0], nb[k][1]);
          if (!(state[v] & 2)) continue;
          const double val = g[v] + l2i(nb[k][0], nb[k][1], cx, cy);
          if (best < 0 || val < bv) { best = k; bv = val; }   // np.argmin: first minimum
        }
        if (best < 0) {
          msg = "ValueError: attempt to get argmin of an empty sequence (search.py:262)";
          return TR_E_VALUE;
        }
        came[c] = id(nb[best][0], nb[best][1]);
        g[c] = bv;
      }
    }
    state[c] = (uint8_t)((state[c] & ~1) | 2);
    ++closed;
    if (cx == gx && cy == gy) {
      st.expanded = closed;
      for (int64_t v = c; v >= 0; v = (v == s ? -1 : came[v])) {
        path.push_back(v / W);
        path.push_back(v % W);
      }
      // reverse pairs: start .. goal
      const size_t m = path.size() / 2;
      for (size_t a = 0, b = m - 1; a < b; ++a, --b) {
        std::swap(path[2 * a], path[2 * b]);
        std::swap(path[2 * a + 1], path[2 * b + 1]);
      }
      return TR_OK;
    }
    const int n = neighbors(cx, cy);
    if (index_err) { msg = "IndexError: index out of bounds (imarray[y][x])"; return TR_E_INDEX; }
    for (int k = 0; k < n; ++k) {
      const int64_t nx = nb[k][0], ny = nb[k][1], v = id(nx, ny);
      if (state[v] & 2) continue;
      double gg = g[c] + l2i(nx, ny, cx, cy);
      if (!(state[v] & 1)) {
        g[v] = gg;
        state[v] |= 4 | 1;
        push(gg + h(nx, ny), nx, ny);
        came[v] = c;
      } else if (gg < g[v]) {
        g[v] = gg;
        came[v] = c;
        push(gg + h(nx, ny), nx, ny);
      }
      if (theta) {                     // search.py:294-304 (line of sight deferred: lazy)
        const int64_t p = came[c];
        const int64_t px = p / W, py = p % W;
        gg = g[p] + l2i(px, py, nx, ny);
        if (gg < g[v]) {
          came[v] = p;
          g[v] = gg;
          push(gg + h(nx, ny), nx, ny);
        }
      }
    }
  }
  st.status = 3;                       // queue exhausted: the reference returns False
  st.expanded = closed;
  return TR_OK;
}

}  // namespace tr
