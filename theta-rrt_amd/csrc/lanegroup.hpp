// Lane groups and the lane-parallel Bresenham line of sight (search.py:35-94) shared by the
// expansion kernels (kernels.hip) and the device Theta* search (astar_dev.hip).
#pragma once
#pragma clang fp contract(off)
#include "geom.hpp"

namespace tr {

// ------------------------------------------------------------------ lane groups
// A group of G lanes (G | 64) works on one sample: every lane computes the sample's scalar chain
// (steer, drive: the same instructions, so no extra latency) and the group splits the pixel work
// (body rays, arc candidates, LOS).  Group-wide votes come from one wave ballot.
template <int G>
struct Grp {
  int li, base;
  __device__ __forceinline__ explicit Grp(int lane) : li(lane & (G - 1)), base(lane & ~(G - 1)) {}
  __device__ __forceinline__ uint64_t bits(bool p) const {
    const uint64_t b = __ballot(p);
    return G == 64 ? b : (b >> base) & ((1ull << (G & 63)) - 1);
  }
  __device__ __forceinline__ bool any(bool p) const { return bits(p) != 0; }
  template <class T>
  __device__ __forceinline__ T bcast(T v, int src) const { return __shfl(v, base + src); }
};

// floor(num / den) for 0 <= num < 2^53, den > 0, without a 64-bit integer division.
__device__ __forceinline__ int64_t floordiv_nn(int64_t num, int64_t den) {
  int64_t q = (int64_t)floor((double)num / (double)den);
  if (q * den > num) --q;
  else if ((q + 1) * den <= num) ++q;
  return q;
}

// A Bresenham line of search.py:35-94 in its normalised octant (steep swap, then x0 <= x1).  Pixel
// k's y-step count is floor((2 dy k + dx - 1) / (2 dx)): the err recurrence of search.py:71-92 in
// closed form (checked exhaustively for dx < 300 in tests/test_host.py), so lanes take pixels
// independently, in the reference's order k = 0 .. dx.
struct BLine {
  int64_t x0, y0, dx, dy, step;
  bool steep;
};
__device__ __forceinline__ BLine bline(int64_t x0, int64_t y0, int64_t x1, int64_t y1) {
  BLine L;
  L.steep = !(llabs(y1 - y0) < llabs(x1 - x0));
  if (L.steep) { int64_t t = x0; x0 = y0; y0 = t; t = x1; x1 = y1; y1 = t; }
  if (x0 > x1) { int64_t t = x0; x0 = x1; x1 = t; t = y0; y0 = y1; y1 = t; }
  L.x0 = x0;
  L.y0 = y0;
  L.dx = x1 - x0;
  L.dy = y1 - y0;
  L.step = 1;
  if (L.dy < 0) { L.step = -1; L.dy = -L.dy; }
  return L;
}
// Pixel k of the line: class 0 = its grid byte decides, 1 blocked (outside: freespace False),
// 2 IndexError (outside a non-square array), 3 past the end; the cell's word is loaded
// unconditionally (word 0 for classes 1-3) so a lane's loads issue back to back.
__device__ __forceinline__ void bline_pixel(const Grid& g, const BLine& L, int64_t k, uint8_t& cls,
                                            uint8_t& v) {
  const int64_t n = k == 0 ? 0 : floordiv_nn(2 * L.dy * k + L.dx - 1, 2 * L.dx);
  const int64_t x = L.x0 + k, y = L.y0 + L.step * n;
  const int64_t px = L.steep ? y : x, py = L.steep ? x : y;
  cls = k > L.dx ? 3 : (!valid_i(g, px, py) ? 1 : ((py >= g.H || px >= g.W) ? 2 : 0));
  v = (uint8_t)grid_bit_if(g, cls == 0, px, py);
}
__device__ __forceinline__ int pixel_state(uint8_t cls, uint8_t v) {   // 0 free, 1 blocked, 2 raise
  return cls == 0 ? (v != 0 ? 0 : 1) : (cls == 3 ? 0 : cls);
}

// First non-free state (0 free, 1 blocked, 2 IndexError) of the lines L[0..NL), in each line's
// Bresenham order, by a lane group; all lines' loads of a chunk in flight together.
template <int G, int NL, int LU>
__device__ __forceinline__ void group_line_states(const Grid& g, const Grp<G>& gr, const BLine* L,
                                                  int* st) {
  int64_t len = 0;
  bool done[NL];
#pragma unroll
  for (int r = 0; r < NL; ++r) {
    st[r] = 0;
    done[r] = false;
    len = L[r].dx + 1 > len ? L[r].dx + 1 : len;
  }
  for (int64_t base = 0; base < len; base += G * LU) {
    uint8_t cls[NL][LU], v[NL][LU];
#pragma unroll
    for (int u = 0; u < LU; ++u)
#pragma unroll
      for (int r = 0; r < NL; ++r) bline_pixel(g, L[r], base + gr.li + G * u, cls[r][u], v[r][u]);
    bool all = true;
#pragma unroll
    for (int r = 0; r < NL; ++r) {
#pragma unroll
      for (int u = 0; u < LU; ++u) {
        const int s = pixel_state(cls[r][u], v[r][u]);
        const uint64_t m = gr.bits(s != 0);
        if (!done[r] && m) {
          st[r] = gr.bcast(s, __ffsll((unsigned long long)m) - 1);
          done[r] = true;
        }
      }
      all = all && done[r];
    }
    if (all) break;
  }
}

// Every pixel of a line by a lane group, no early exit: any blocked, any IndexError (the eager
// `False in [freespace(px) for px in pixels]` of rrt.py:173-174).
template <int G>
__device__ __forceinline__ void line_all_states(const Grid& g, const Grp<G>& gr, const BLine& L,
                                                bool& blocked, bool& raises) {
  bool b = false, r = false;
  for (int64_t base = 0; base <= L.dx; base += G * 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint8_t cls, v;
      bline_pixel(g, L, base + gr.li + G * u, cls, v);
      const int s = pixel_state(cls, v);
      b = b || s == 1;
      r = r || s == 2;
    }
  }
  blocked = gr.any(b);
  raises = gr.any(r);
}

// lineofsight (search.py:35-41) by a lane group; true = clear, *ierr on IndexError.
template <int G>
__device__ __forceinline__ bool los_group(const Grid& g, const Grp<G>& gr, int64_t x0, int64_t y0,
                                          int64_t x1, int64_t y1, int* ierr) {
  const BLine L = bline(x0, y0, x1, y1);
  int st;
  group_line_states<G, 1, 4>(g, gr, &L, &st);
  if (st == 2) *ierr = 1;
  return st == 0;
}

}  // namespace tr
