// HIP kernels of the batched RRT expansion + LOS engine (gfx950 / CDNA4).
//
// Per batch of B samples against a tree snapshot of N nodes:
//   k_samples     thread per sample: rand_conf from the gaussian stream + freespace.
//   nn.hip        nearest node (fp32 screen + exact fp64 resolve).
//   k_expand_arc  16 lanes per sample: steer + drive (every lane), body rays and the arc-pixel
//                 collision test split across the lanes; one record per sample.
//   k_los         wave per ray: Bresenham line of sight (Theta* batches, RRT straight arcs).
#pragma clang fp contract(off)
#include "geom.hpp"
#include "lanegroup.hpp"
#include "thetarrt_internal.hpp"
#include "diaglog.hpp"
TR_DLOG_EXPORT(tr_diag_log_k)

namespace tr {

// Diagnosis builds only (build.py --variant phases): wall-clock stamps (100 MHz) between the
// phases of k_expand_arc, one row per sample of the latest launch, stored with plain stores and
// read back through tr_diag_phases (no atomics or printf: those stretched what they measured).
#ifdef TR_DIAG_PHASES
constexpr int PH_N = 10, PH_ROWS = 4096, PH_RING = 8;   // the latest PH_RING launches, by dedupe epoch
__device__ unsigned long long g_ph[PH_RING * PH_ROWS * PH_N];
#define TR_PH(i) tp[i] = wall_clock64()
#define TR_PH_ARG , unsigned long long* tp
#define TR_PH_PASS , tp
#else
#define TR_PH(i)
#define TR_PH_ARG
#define TR_PH_PASS
#endif

// ------------------------------------------------------------------ samples (rrt.py:53-68, 144-150)
__device__ __forceinline__ void make_sample(const Params& P, const Grid& g, const double* gauss,
                                            int64_t j, double gx, double gy, double gth,
                                            tr_sample& s, bool& live, int& ierr) {
  double g0 = gauss[3 * j], g1 = gauss[3 * j + 1], g2 = gauss[3 * j + 2];
  double sx = P.xystdv * (double)g.H, sy = P.xystdv * (double)g.W;
  double x = gx + sx * g0, y = gy + sy * g1;
  x = fmin(fmax(x, 0.0), (double)(g.H - 1));     // np.clip
  y = fmin(fmax(y, 0.0), (double)(g.W - 1));
  double th = wrap180(wrap180(wrap180(gth) + P.anglestdv * g2));
  s.x = (int32_t)x;
  s.y = (int32_t)y;
  s.th = th;
  live = free_i(g, s.x, s.y, &ierr);
}

// ------------------------------------------------------------------ samples
// rand_conf for B samples (rrt.py:53-68) + the freespace test (rrt.py:148).  live: 1 = free,
// 0 = on an obstacle, 2 = IndexError in the reference (non-square map).
__global__ __launch_bounds__(256) void k_samples(Params P, Grid g, const double* __restrict__ gauss,
                                                 int64_t B, double gx, double gy, double gth,
                                                 tr_sample* __restrict__ samples,
                                                 int2* __restrict__ qxy, int32_t* __restrict__ live,
                                                 int32_t* __restrict__ zero) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  TR_DLOG_T0;
  if (zero && j == 0) zero[0] = 0;       // the batch's fix-up list counter
  TR_DLOG(0);
  if (j >= B) return;
  tr_sample s;
  bool ok;
  int ierr = 0;
  make_sample(P, g, gauss, j, gx, gy, gth, s, ok, ierr);
  samples[j] = s;
  qxy[j] = make_int2(s.x, s.y);
  live[j] = ok ? 1 : (ierr ? 2 : 0);
}

// rrt.py:169 `valid(qnew) and bike_clear(qnew) and front_of_bike_clear(qnew)` (rrt.py:208-222):
// one rotation for both rays (body_rays_clear, geom.hpp), both rays' pixels tested by the group.
template <int G>
__device__ __forceinline__ bool body_rays_group(const Grid& g, const Grp<G>& gr, const Params& P,
                                                double x, double y, double th, int* ierr) {
  const int64_t x0 = trunc_i(x), y0 = trunc_i(y);
  if (!valid_i(g, x0, y0)) return false;
  double z, w;
  zquat(th, z, w);
  const double x2 = 0.0, y2 = 0.0, z2 = z * z, w2 = w * w, xy = 0.0, zw = z * w;
  const double m00 = x2 - y2 - z2 + w2, m01 = 2 * (xy - zw), m02 = 2 * (0.0 * z + 0.0 * w);
  const double m10 = 2 * (xy + zw), m11 = -x2 + y2 - z2 + w2, m12 = 2 * (0.0 * z - 0.0 * w);
  const double len[2] = {P.bikelength * 1.0, P.bikelength * P.frontclearance};
  BLine L[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const double ex = (m00 * len[r] + m01 * 0.0 + m02 * 0.0) + x;
    const double ey = (m10 * len[r] + m11 * 0.0 + m12 * 0.0) + y;
    L[r] = bline(x0, y0, trunc_i(ex), trunc_i(ey));
  }
  int s[2];
  group_line_states<G, 2, 1>(g, gr, L, s);
  if (s[0] == 2 || (s[0] == 0 && s[1] == 2)) { *ierr = 1; return false; }
  return s[0] == 0 && s[1] == 0;
}

// ------------------------------------------------------------------ expand (rrt.py:155-171)
// One sample's steer / body rays / drive against its nearest node nn, by a lane group: the
// record, with status TR_ST_PENDING when the arc check (rrt.py:173-176) is still to do.
template <int G>
__device__ __forceinline__ tr_record expand_group(const Params& P, const Grid& g, const Grp<G>& gr,
                                                  int64_t nn, const tr_sample& s, int32_t lv,
                                                  const double2* __restrict__ txy,
                                                  const double* __restrict__ tth TR_PH_ARG) {
  tr_record r;
  r.x = r.y = r.th = 0;
  r.steer = r.iccx = r.iccy = r.rad = r.dist = 0;
  r.near = -1;
  r.flags = 0;
  r.ex = -1;
  if (lv != 1) {
    r.status = lv == 2 ? TR_ST_INDEX : TR_ST_SKIP;
    if (lv == 2) r.flags |= TR_FL_INDEX_SAMPLE;
    return r;
  }
  const double2 o = txy[nn];
  const double ox = o.x, oy = o.y, oth = tth[nn];
  double nx, ny, nth;
  Ctrl u;
  steer(P, ox, oy, oth, (double)s.x, (double)s.y, s.th, nx, ny, nth, u);
  TR_PH(3);
  r.near = nn;
  int ierr = 0;
  if (wrap180(u.steer) < P.leftc || wrap180(u.steer) > P.rightc) {
    r.status = TR_ST_CONSTRAINT;
    return r;
  }
#ifdef TR_DIAG_NORAYS             // diagnosis builds only: body rays taken as clear
  bool ok = true;
#else
  bool ok = body_rays_group<G>(g, gr, P, nx, ny, nth, &ierr);
#endif
  TR_PH(4);
  if (!ok) {
    u.dist = u.dist / 3;
    r.flags |= TR_FL_DROVE;
    if (!drive(P, ox, oy, oth, u, nx, ny, nth)) {
      r.status = TR_ST_STRAIGHT;
      return r;
    }
  }
  r.x = nx;
  r.y = ny;
  r.th = nth;
  r.steer = u.steer;
  r.iccx = u.iccx;
  r.iccy = u.iccy;
  r.rad = u.rad;
  r.dist = u.dist;
  if (u.straight) r.flags |= TR_FL_STRAIGHT;
  r.status = ierr ? TR_ST_INDEX : TR_ST_PENDING;
  return r;
}

// ------------------------------------------------------------------ arc check (search.py:144-182)
// getCircle's pixels are the 8 images of the octant points (x_k, k), k < K (geom.hpp).  A lane takes
// one k per round and all 8 images of its point: one circle_x per 8 candidates, the images' grid
// words loaded together.  Small circles (K <= 16, or K <= 32 under a wide window) are walked whole;
// otherwise only the k whose images can fall inside a box: the arc's bounding box grown by the
// sagitta + 4 px (kept pixels lie within 3 px of the arc), or, for a circle too big to walk whole
// under a wide window, the grid itself (the only pixels getCircle can emit, valid_i).  The plan is
// made by the group: the lanes split the octant-length search, the diagonal-patch test and the
// images' k-ranges, and the set-up's two headings.
struct ArcPlan {
  int64_t xc, yc, r, K, R2;
  bool drawmore, boxed, split;
  int64_t bx0, bx1, by0, by1;       // offsets relative to (xc, yc), inclusive (boxed)
  int64_t kmin, kmax;               // union of the images' k-ranges (all of [0, K) when not boxed)
  int64_t my_lo, my_hi;             // the k-range of image li & 7 (boxed)
};

// k-range of the octant points whose x_k = circle_x(r, k) can lie in [a0, a1] (a superset: x_k is
// non-increasing in k, x_k <= a1 implies k^2 >= r^2 - a1 (a1 + 1), x_k >= a0 > 0 implies
// k^2 < r^2 - a0 (a0 - 1); one unit of slack each side for the rounding of sqrt).
__device__ __forceinline__ void circle_k_for_x(int64_t r, int64_t a0, int64_t a1, int64_t& klo,
                                               int64_t& khi) {
  const double r2 = (double)r * (double)r;
  const double t1 = r2 - (double)a1 * (double)(a1 + 1);
  klo = t1 > 0 ? (int64_t)floor(sqrt(t1)) - 1 : 0;
  const double t0 = a0 > 0 ? r2 - (double)a0 * (double)(a0 - 1) : r2;
  khi = t0 > 0 ? (int64_t)ceil(sqrt(t0)) + 1 : 0;
}

// circle_octant_len by a group: K = first k with x_k <= k, and x_k - k falls strictly with k, so
// with one k per lane from just below r / sqrt(2) K is the window's start plus the lanes still
// above the diagonal (the sequential search if the window misses K).
template <int G>
__device__ __forceinline__ int64_t circle_octant_len_group(const Grp<G>& gr, int64_t r) {
  if (r <= 0) return 0;
  int64_t k0 = (int64_t)((double)r * 0.70710678118654752) - 4;
  if (k0 < 0) k0 = 0;
  const int64_t k = k0 + gr.li;
  const uint64_t above = gr.bits(circle_x(r, k) > k);
  const bool first = above & 1, last = (above >> (G - 1)) & 1;
  if ((k0 > 0 && !first) || last) return circle_octant_len(r);
  return k0 + __popcll((unsigned long long)above);
}

// circle_drawmore (search.py:124-138) with one neighbour of the diagonal pixel per lane.
template <int G>
__device__ __forceinline__ bool circle_drawmore_group(const Grid& g, const Grp<G>& gr, int64_t xc,
                                                      int64_t yc, int64_t r, int64_t K, int64_t& R2) {
  R2 = (int64_t)rint((double)r * 0.5 * kSqrt2);
  const int i = gr.li & 3;
  const int64_t nx = xc + R2 + (i == 0 ? 1 : (i == 1 ? -1 : 0));
  const int64_t ny = yc + R2 + (i == 2 ? 1 : (i == 3 ? -1 : 0));
  const int64_t a = nx - xc, b = ny - yc;
  const bool diag = (a < 0 ? -a : a) == (b < 0 ? -b : b);     // never emitted (|v1| == |v2|)
  return !gr.any(!diag && valid_i(g, nx, ny) && circle_member(r, K, a, b));
}

template <int G>
__device__ __forceinline__ void arc_plan_group(const Grid& g, const Grp<G>& gr, double bx, double by,
                                               double lx, double ly, const Ctrl& u, const ArcWin& w,
                                               ArcPlan& pl) {
  pl.xc = trunc_i(u.iccx);
  pl.yc = trunc_i(u.iccy);
  pl.r = trunc_i(u.rad);
  pl.K = circle_octant_len_group<G>(gr, pl.r);
  pl.drawmore = circle_drawmore_group<G>(g, gr, pl.xc, pl.yc, pl.r, pl.K, pl.R2);
  const bool arcbox = pl.K > 16 && w.diff < 90 && u.steer != 0;
  pl.boxed = arcbox || pl.K > 32;
  pl.split = false;
  pl.kmin = 0;
  pl.kmax = pl.K - 1;
  if (!pl.boxed) return;
  // valid region x in [0, H), y in [0, W) (search.py:17-24), as offsets from the centre
  pl.bx0 = -pl.xc;
  pl.bx1 = g.H - 1 - pl.xc;
  pl.by0 = -pl.yc;
  pl.by1 = g.W - 1 - pl.yc;
  if (arcbox) {                              // the arc's box grown by the sagitta + 4 px
    double sag = u.rad * (1 - cos(w.diff * kDeg * 0.5));
    double m = sag + 4;
    pl.bx0 = max(pl.bx0, (int64_t)floor(fmin(bx, lx) - m) - pl.xc);
    pl.bx1 = min(pl.bx1, (int64_t)ceil(fmax(bx, lx) + m) - pl.xc);
    pl.by0 = max(pl.by0, (int64_t)floor(fmin(by, ly) - m) - pl.yc);
    pl.by1 = min(pl.by1, (int64_t)ceil(fmax(by, ly) + m) - pl.yc);
  }
  // image li & 7: images 0-3 carry k on the y offset and x_k on x, 4-7 the other way; bit0 / bit1
  // negate the x / y offset.  Its k-range is cut by both box sides.
  const int im = gr.li & 7;
  const bool on_y = !(im & 4);
  const bool negk = on_y ? (im & 2) : (im & 1), negx = on_y ? (im & 1) : (im & 2);
  const int64_t a0 = on_y ? pl.by0 : pl.bx0, a1 = on_y ? pl.by1 : pl.bx1;
  const int64_t c0 = on_y ? pl.bx0 : pl.by0, c1 = on_y ? pl.bx1 : pl.by1;
  int64_t klo = negk ? -a1 : a0, khi = negk ? -a0 : a1;
  int64_t x0 = negx ? -c1 : c0, x1 = negx ? -c0 : c1;     // range of x_k itself
  if (x0 < 0) x0 = 0;
  if (x1 < x0) {
    klo = 1;
    khi = 0;
  } else {
    int64_t k0, k1;
    circle_k_for_x(pl.r, x0, x1, k0, k1);
    if (k0 > klo) klo = k0;
    if (k1 < khi) khi = k1;
  }
  if (klo < 0) klo = 0;
  if (khi > pl.K - 1) khi = pl.K - 1;
  pl.my_lo = klo;
  pl.my_hi = khi;
  // union and total over the 8 images (every aligned 8 lanes hold all of them)
  const bool some = khi >= klo;
  int64_t lo = some ? klo : INT64_MAX, hi = some ? khi : -1, tot = some ? khi - klo + 1 : 0;
#pragma unroll
  for (int off = 1; off <= 4; off <<= 1) {
    const int64_t lo2 = __shfl_xor(lo, off), hi2 = __shfl_xor(hi, off), t2 = __shfl_xor(tot, off);
    lo = lo2 < lo ? lo2 : lo;
    hi = hi2 > hi ? hi2 : hi;
    tot += t2;
  }
  pl.kmin = lo;
  pl.kmax = hi;
  // pieces of the circle far apart in k (a circle crossing the grid twice): image by image
  pl.split = hi >= lo && (hi - lo + 1) > 2 * tot + 4 * G;
}

// Returns true if pixel (kept by the arc window) is blocked.  The grid byte is read first: only a
// pixel that is not free (or raises) can matter, so the angle test (fp64 atan2) runs for those only.
__device__ __forceinline__ bool arc_pixel_blocked(const Grid& g, const ArcWin& w, int64_t px,
                                                  int64_t py, int* ierr) {
  if (!valid_i(g, px, py)) return false;
  int perr = 0;
  if (free_i(g, px, py, &perr)) return false;
  if (!arc_keeps(w, px, py)) return false;
  if (perr) *ierr = 1;
  return !perr;
}

// The window of getArc with its two headings taken by two lanes at once (geom.hpp arc_window).
template <int G>
__device__ __forceinline__ ArcWin arc_window_group(const Grp<G>& gr, double bx, double by, double lx,
                                                   double ly, const Ctrl& u) {
  ArcWin w;
  w.iccx = u.iccx;
  w.iccy = u.iccy;
  w.steer = u.steer;
  w.bvx = bx - u.iccx;
  w.bvy = by - u.iccy;
  w.evx = lx - u.iccx;
  w.evy = ly - u.iccy;
  w.bn2 = w.bvx * w.bvx + w.bvy * w.bvy;
  w.en2 = w.evx * w.evx + w.evy * w.evy;
  const bool odd = gr.li & 1;
  const double ang = heading(odd ? w.evx : w.bvx, odd ? w.evy : w.bvy);
  w.b_ang = gr.bcast(ang, 0);
  w.e_ang = gr.bcast(ang, 1);
  double d = u.steer < 0 ? angle_diff_fast(w.b_ang, w.e_ang) : angle_diff_fast(w.e_ang, w.b_ang);
  if (d < 0) d = 360 + d;
  w.diff = d;
  return w;
}

// Arc (or, for a straight control, segment) collision test of rrt.py:173-176 by a lane group.
template <int G>
__device__ bool arc_blocked_group(const Grid& g, const Grp<G>& gr, double bx, double by, double lx,
                                  double ly, const Ctrl& u, int* ierr TR_PH_ARG) {
  if (u.straight) {
    if (g.H != g.W) {            // a pixel after a blocked one can still raise: test them all
      bool b, r;
      line_all_states<G>(g, gr, bline(trunc_i(bx), trunc_i(by), trunc_i(lx), trunc_i(ly)), b, r);
      if (r) *ierr = 1;
      return b;
    }
    int e = 0;
    const bool clear = los_group<G>(g, gr, trunc_i(bx), trunc_i(by), trunc_i(lx), trunc_i(ly), &e);
    if (e) *ierr = 1;
    return !clear;
  }
  const ArcWin w = arc_window_group<G>(gr, bx, by, lx, ly, u);
  ArcPlan pl;
  arc_plan_group<G>(g, gr, bx, by, lx, ly, u, w, pl);
  TR_PH(6);
  // rrt.py:174 evaluates freespace on every kept pixel, so on a non-square map a later pixel can
  // still raise: stop at the first blocked pixel only when no pixel can raise.
  const bool can_raise = g.H != g.W;
  bool blocked = false;
  const int npass = pl.split ? 8 : 1;
  for (int pass = 0; pass < npass; ++pass) {         // uniform in the group
    int64_t klo = pl.kmin, khi = pl.kmax;
    uint32_t ims = 0xffu;
    if (pl.split) {
      klo = gr.bcast(pl.my_lo, pass);
      khi = gr.bcast(pl.my_hi, pass);
      ims = 1u << pass;
    }
    for (int64_t kb = klo; kb <= khi; kb += G) {
      const int64_t k = kb + gr.li;
      const bool live = k <= khi;
      const int64_t x = live ? circle_x(pl.r, k) : 0;
      // per image: its grid bit loaded unconditionally (masked after) so the 8 loads are in flight
      // together; decide = the bit decides, raise = outside a non-square array (raises if kept)
      uint32_t decide = 0, raise = 0, v[8];
#pragma unroll
      for (int im = 0; im < 8; ++im) {
        int64_t dx, dy;
        circle_image(im, x, k, dx, dy);
        const bool in = live && ((ims >> im) & 1) &&
                        !(pl.boxed && (dx < pl.bx0 || dx > pl.bx1 || dy < pl.by0 || dy > pl.by1));
        const int64_t px = pl.xc + dx, py = pl.yc + dy;
        const bool ok = in && valid_i(g, px, py);
        const bool inside = ok && !(py >= g.H || px >= g.W);
        if (ok) (inside ? decide : raise) |= 1u << im;
        v[im] = grid_bit_if(g, inside, px, py);
      }
      uint32_t look = raise;                          // candidates that are not free
#pragma unroll
      for (int im = 0; im < 8; ++im)
        if (((decide >> im) & 1) && v[im] == 0) look |= 1u << im;
      while (look) {                                  // the keep test only for those
        const int im = __ffs(look) - 1;
        look &= look - 1;
        int64_t dx, dy;
        circle_image(im, x, k, dx, dy);
        if (!arc_keeps(w, pl.xc + dx, pl.yc + dy)) continue;
        if ((raise >> im) & 1) *ierr = 1;
        else blocked = true;
      }
      if (!can_raise && gr.any(blocked)) break;
    }
    if (!can_raise && gr.any(blocked)) break;
  }
  if (pl.drawmore && gr.li < 4) {
    int64_t sx = (gr.li == 0 || gr.li == 2) ? pl.R2 : -pl.R2;
    int64_t sy = (gr.li == 0 || gr.li == 3) ? pl.R2 : -pl.R2;
    if (arc_pixel_blocked(g, w, pl.xc + sx, pl.yc + sy, ierr)) blocked = true;
  }
  return gr.any(blocked);
}

// Arc check of a pending record by a lane group: final status and the goal flag (rrt.py:190-201).
template <int G>
__device__ __forceinline__ void arc_finish(const Params& P, const Grid& g, const Grp<G>& gr,
                                           const double2* __restrict__ txy, double gx, double gy,
                                           double gth, tr_record& r TR_PH_ARG) {
  Ctrl u{r.steer, r.iccx, r.iccy, r.rad, r.dist, (r.flags & TR_FL_STRAIGHT) ? 1 : 0};
  int ierr = 0;
  const double2 o = txy[r.near];
  bool blocked = arc_blocked_group<G>(g, gr, o.x, o.y, r.x, r.y, u, &ierr TR_PH_PASS);
  bool anyerr = gr.any(ierr != 0);
  int32_t st = anyerr ? TR_ST_INDEX : (blocked ? TR_ST_COLLISION : TR_ST_OK);
  if (st == TR_ST_OK) {
    double dx = gx - r.x, dy = gy - r.y;
    double d = sqrt(dx * dx + dy * dy);
    if (d < P.tol_xy && fabs(angle_diff_exact(r.th, gth)) < P.tol_ang) r.flags |= TR_FL_GOAL;
  }
  r.status = st;
}

// ------------------------------------------------------------------ fused expansion
// rrt.py:151-188 for one sample per group of EG lanes: steer / body rays / drive, the arc check,
// and the snapshot lookups of the bookkeeping (sample membership, qnew's node, qnew == qnear);
// record written once.
constexpr int EG = 16;           // lanes per sample
// Pose-table lookup by a lane group (thetarrt_internal.hpp: buckets of POSE_BUCKET slots): the
// group's first POSE_BUCKET lanes hold the slots of bucket b (loaded by the caller, v); the pose
// or an empty slot in the bucket decides, else the next bucket (rare at the table's load).
template <int G>
__device__ __forceinline__ int32_t group_lookup(const Grp<G>& gr, const PoseSlot* __restrict__ tab,
                                                uint64_t mask, uint64_t b, PoseSlot v, double x,
                                                double y, double t, int32_t* err) {
  const uint64_t bmask = mask / POSE_BUCKET;
  const bool mine = gr.li < POSE_BUCKET;
  for (uint64_t it = 0; it <= bmask; ++it) {
    const bool empty = mine && v.idx < 0, hit = mine && !empty && pose_eq(v.x, v.y, v.th, x, y, t);
    const uint64_t h = gr.bits(hit);
    if (h) return gr.bcast(v.idx, __ffsll((unsigned long long)h) - 1);
    if (gr.any(empty)) return -1;
    b = (b + 1) & bmask;
    if (mine) v = tab[b * POSE_BUCKET + gr.li];
  }
  if (gr.li == 0) atomicOr(err, TR_DDE_LOOKUP);
  return -1;
}

constexpr int XU = 8;                        // t4 operands in flight per lane

// The correction screened in fp32: node n can beat the known key only with d_n < sd, i.e.
// s_n = d_n - |p|^2 < sd - |p|^2 where s_n is the NN screen's fma(ax, x^, fma(by, y^, w^)) on the
// node's t4 operands; such a node lies within R = sqrt(sd) of the sample, so the screen's error
// is at most screen_E(p, R) (nn.hip) and every node passing s <= thr gets the exact fp64 test in
// increasing index order per lane, as the unscreened version does.  Each lane loads XU 16-byte
// t4 operands per round; txy only for the few candidates.
template <int G>
__device__ __forceinline__ int64_t delta_near_screen(const DeltaArgs& da, const double2* __restrict__ txy,
                                                     double qx, double qy, bool act, int64_t nn) {
  constexpr int NW = 64 / G;
  const int lane = threadIdx.x & 63;
  const int64_t lo = ld_sc1(da.snap), hi = ld_sc1(da.count);
  if (hi <= lo) return nn;                   // uniform: nothing appended
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const double dmine = act ? ld_sc1(da.dnear + j) : -1.0;
  const double X = fmax(__longlong_as_double((long long)da.maxabs[0]), da.qmax) + 1.0;
  const double Eg = screen_Eg(X);
  float thr_mine = -INFINITY;
  if (act) {
    const double px = qx - (double)da.cx, py = qy - (double)da.cy, p2 = px * px + py * py;
    const double R = sqrt(fmax(dmine, 0.0)) * (1.0 + 1e-12) + 1e-9;
    const double E = screen_E(px, py, R, Eg);
    const double t = (dmine - p2) + E + (fabs(dmine - p2) + p2 + E + 1.0) * 5.684341886080802e-14;
    thr_mine = nextafterf((float)t, INFINITY);
  }
  double sx[NW], sy[NW], sd[NW], rb[NW], dl[NW];
  float ax[NW], by[NW], th[NW];
  int64_t ib[NW];
#pragma unroll
  for (int s = 0; s < NW; ++s) {
    sx[s] = __shfl(qx, s * G);
    sy[s] = __shfl(qy, s * G);
    sd[s] = __shfl(dmine, s * G);
    th[s] = __shfl(thr_mine, s * G);
    ax[s] = -2.0f * (float)(sx[s] - (double)da.cx);
    by[s] = -2.0f * (float)(sy[s] - (double)da.cy);
    rb[s] = dl[s] = INFINITY;
    ib[s] = -1;
  }
  for (int64_t i0 = lo + lane; i0 < hi; i0 += 64 * XU) {
    float4 f[XU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int64_t i = i0 + u * 64;
      f[u] = i < hi ? da.t4[i] : make_float4(0.0f, 0.0f, INFINITY, 0.0f);
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int64_t i = i0 + u * 64;
      bool cand = false;
#pragma unroll
      for (int s = 0; s < NW; ++s) cand = cand || fmaf(ax[s], f[u].x, fmaf(by[s], f[u].y, f[u].z)) <= th[s];
      if (cand && i < hi) {                   // rare: the exact test for every sample
        const double2 e = txy[i];
#pragma unroll
        for (int s = 0; s < NW; ++s) {
          const double a = sx[s] - e.x, b = sy[s] - e.y;
          const double d = a * a + b * b;
          if (d < sd[s] && d < dl[s]) {
            const double rt = sqrt(d);
            if (rt < rb[s]) { rb[s] = rt; dl[s] = d; ib[s] = i; }
          }
        }
      }
    }
  }
  int64_t out = nn;
#pragma unroll
  for (int s = 0; s < NW; ++s) {
    if (!__ballot(ib[s] >= 0)) continue;     // uniform
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ro = __shfl_xor(rb[s], off), dq = __shfl_xor(dl[s], off);
      const int64_t io = __shfl_xor(ib[s], off);
      if (io >= 0 && (ib[s] < 0 || ro < rb[s] || (ro == rb[s] && io < ib[s]))) {
        rb[s] = ro; dl[s] = dq; ib[s] = io;
      }
    }
    if (lane / G == s && ib[s] >= 0 && rb[s] < sqrt(sd[s])) out = ib[s];
  }
  return out;
}

// The same correction through the appended nodes' bins (thetarrt_internal.hpp: DeltaBins): a node
// beats the known key sqrt(dmine) only from inside the disc of that radius around the sample, so
// the group's 16 lanes share the bins the disc's box covers (up to DB_LANE each).  Round one loads
// every bin's count, and with it the first DB_LIGHT items of the lane's first bin (a near sample's
// box is a few bins: its whole correction is this one round).  A lane then reads its other light
// bins (<= DB_LIGHT items, few non-empty: far from the tree little is appended), and the heavy
// bins (map corners and borders, where clipped samples pile nodes up) are taken one by one by the
// whole group, DB_CAP / 16 items per lane in flight.  Items are tested in exact fp64 (the rule of
// k_nn_delta: a strictly smaller sqrt(d), the lowest index among equal ones).  full = the sample
// needs the scan of the appended nodes instead (a box of more than 16 DB_LANE bins, or a bin past
// its capacity).
__device__ __forceinline__ int64_t delta_near_bins(const DeltaArgs& da, const Grp<16>& gr, double qx,
                                                   double qy, bool act, double dmine, int64_t nn,
                                                   bool& full TR_PH_ARG) {
  constexpr int G = 16;
  static_assert(DB_CAP == 4 * G && DB_LIGHT <= 7 && DB_LANE <= 16, "heavy bins: 4 items per lane");
  const DeltaBins& B = da.bins;
  double rb = INFINITY;
  int32_t ib = -1;
  bool over = false;
  if (act && dmine > 0.0) {                  // uniform in the group
    const double R = sqrt(dmine) * (1.0 + 1e-12) + 1e-9;
    const int32_t bx0 = db_coord(qx - R, B.xmax) >> B.shift, bx1 = db_coord(qx + R, B.xmax) >> B.shift;
    const int32_t by0 = db_coord(qy - R, B.ymax) >> B.shift, by1 = db_coord(qy + R, B.ymax) >> B.shift;
    const int32_t w = bx1 - bx0 + 1, nbins = w * (by1 - by0 + 1);
    if (nbins > G * DB_LANE) {
      over = true;
#ifdef TR_DIAG_PHASES
      tp[PH_N - 1] |= 1;                     // why the sample scans: its box covers too many bins
#endif
    } else {
      const int64_t nb = (int64_t)B.nbx * B.nby;
      auto test = [&](const DBItem& v) {
        const double a = qx - v.x, b = qy - v.y;
        const double d = a * a + b * b;
        if (d < dmine) {
          const double rt = sqrt(d);
          if (ib < 0 || rt < rb || (rt == rb && v.idx < ib)) { rb = rt; ib = v.idx; }
        }
      };
      auto bin_at = [&](int32_t b) {         // the box's b-th bin, row-major
        const int32_t row = b / w;
        return (int64_t)(by0 + row) * B.nbx + bx0 + (b - row * w);
      };
      for (unsigned long long e = da.e_lo; e <= da.e_hi; ++e) {
        const uint32_t* cn = B.cnt + (int64_t)(e & 3) * (nb + 1);
        const DBItem* items = B.items + (int64_t)(e & 3) * nb * DB_CAP;
        bool spill = false;                  // a bin of the box sent nodes to the overflow list
        // counts of the lane's bins: light ones 3 bits each, heavy ones a bit in hv
        unsigned long long pk = 0;
        uint32_t hv = 0;
        const DBItem* it0 = items + (gr.li < nbins ? bin_at(gr.li) : 0) * DB_CAP;
        DBItem v[DB_LIGHT];
#pragma unroll
        for (int q = 0; q < DB_LANE; ++q) {
          const int32_t b = gr.li + G * q;
          const uint32_t c = b < nbins ? ld_sc1(cn + bin_at(b)) : 0u;
          if (c > (uint32_t)DB_LIGHT) hv |= 1u << q;
          else pk |= (unsigned long long)c << (3 * q);
        }
#pragma unroll
        for (int q = 0; q < DB_LIGHT; ++q) v[q] = it0[q];
#pragma unroll
        for (int q = 0; q < DB_LIGHT; ++q)
          if ((uint32_t)q < (uint32_t)(pk & 7)) test(v[q]);
        pk >>= 3;
        for (int q = 1; pk; ++q, pk >>= 3) {   // the lane's other light bins
          const uint32_t c = (uint32_t)(pk & 7);
          if (!c) continue;
          const DBItem* it = items + bin_at(gr.li + G * q) * DB_CAP;
#pragma unroll
          for (int r = 0; r < DB_LIGHT; ++r) v[r] = it[r];
#pragma unroll
          for (int r = 0; r < DB_LIGHT; ++r)
            if ((uint32_t)r < c) test(v[r]);
        }
        for (;;) {                             // heavy bins: the whole group on one at a time
          const uint64_t m = gr.bits(hv != 0);
          if (!m) break;
          const int L = __ffsll((unsigned long long)m) - 1;
          const uint32_t hl = gr.bcast(hv, L);
          const int q = __ffs(hl) - 1;
          if (gr.li == L) hv &= hv - 1;
          const int64_t at = bin_at(L + G * q);
          const DBItem* it = items + at * DB_CAP;
          const uint32_t c = ld_sc1(cn + at);
#pragma unroll
          for (int r = 0; r < DB_CAP / G; ++r) v[r] = it[gr.li + G * r];
          if (c > (uint32_t)DB_CAP) spill = true;
#pragma unroll
          for (int r = 0; r < DB_CAP / G; ++r)
            if ((uint32_t)(gr.li + G * r) < c) test(v[r]);
        }
        if (spill) {                           // uniform in the group: the whole list, as a heavy bin
          const uint32_t c = ld_sc1(cn + nb);
          if (c > (uint32_t)B.ovf_cap) over = true;
          const DBItem* it = B.ovf + (int64_t)(e & 3) * B.ovf_cap;
          for (uint32_t s0 = 0; s0 < c && s0 < (uint32_t)B.ovf_cap; s0 += DB_CAP) {
#pragma unroll
            for (int r = 0; r < DB_CAP / G; ++r) {
              const uint32_t s1 = s0 + gr.li + G * r;
              v[r] = it[s1 < (uint32_t)B.ovf_cap ? s1 : 0];
            }
#pragma unroll
            for (int r = 0; r < DB_CAP / G; ++r)
              if (s0 + gr.li + G * r < c) test(v[r]);
          }
#ifdef TR_DIAG_PHASES
          tp[PH_N - 1] |= 4;                 // (diagnosis: the sample read the overflow list)
#endif
        }
#ifdef TR_DIAG_PHASES
        if (over) tp[PH_N - 1] |= 2;         // ... or a bin is past its capacity
#endif
      }
    }
  }
  full = gr.any(over);
  if (full || !gr.any(ib >= 0)) return nn;
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) {
    const double ro = __shfl_xor(rb, off);
    const int32_t io = __shfl_xor(ib, off);
    if (io >= 0 && (ib < 0 || ro < rb || (ro == rb && io < ib))) { rb = ro; ib = io; }
  }
  return (ib >= 0 && rb < sqrt(dmine)) ? (int64_t)ib : nn;
}

__global__ __launch_bounds__(256) void k_expand_arc(Params P, Grid g, const int64_t* __restrict__ nnidx,
                                                    int64_t B, const tr_sample* __restrict__ samples,
                                                    const int32_t* __restrict__ live,
                                                    const double2* __restrict__ txy,
                                                    const double* __restrict__ tth, double gx,
                                                    double gy, double gth,
                                                    const PoseSlot* __restrict__ htab, uint64_t hmask,
                                                    int32_t* __restrict__ err,
                                                    tr_record* __restrict__ rec, DeltaArgs da) {
  const Grp<EG> gr(threadIdx.x & 63);
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) / EG;
  const bool in = j < B;
  TR_DLOG_T0;
#ifdef TR_DIAG_PHASES
  unsigned long long tp[PH_N];
  for (int q = 0; q < PH_N; ++q) tp[q] = 0;
#endif
  TR_PH(0);
  const int32_t lv = in ? live[j] : 0;
  tr_sample sm{};
  if (in) sm = samples[j];
  // the look-ahead resolve may publish from inside its kernel with sc1 stores: read them sc1
  // (thetarrt_internal.hpp: an sc1 store is only coherent with sc1 loads)
  // (every input of the correction is loaded here, with the sample: one round trip, not three)
  int64_t nn = in ? ld_sc1(nnidx + j) : -1;
  const bool binned = da.snap && da.bins.cnt;
  const double dm = binned && in ? ld_sc1(da.dnear + j) : -1.0;
  const bool appended = binned && ld_sc1(da.count) > ld_sc1(da.snap);      // uniform
  if (lv != 1) nn = -1;
  TR_PH(1);
#ifdef TR_DIAG_NODELTA                       // diagnosis builds only: correction skipped
  da.snap = nullptr;
#endif
  if (da.snap) {
    if (binned) {
      if (appended) {
        bool full;
        nn = delta_near_bins(da, gr, (double)sm.x, (double)sm.y, lv == 1, dm, nn, full TR_PH_PASS);
        if (__any(full)) nn = delta_near_screen<EG>(da, txy, (double)sm.x, (double)sm.y, full, nn);
      }
    } else {
      nn = delta_near_screen<EG>(da, txy, (double)sm.x, (double)sm.y, lv == 1, nn);
    }
  }
  if (!in) return;
  TR_PH(2);
  // rrt.py:151 `qrand in G.keys()` against the snapshot: the first probe is issued now and
  // resolved after the expansion (its latency hides behind steer)
  // The group's first lanes load the slots of the pose's home bucket (group_lookup).
  const bool look = htab != nullptr && lv == 1;
  const double sx = (double)sm.x, sy = (double)sm.y;
  uint64_t ps = 0, pq = 0;
  PoseSlot vs, vq;
  vs.idx = vq.idx = -1;
  if (look) {
    ps = pose_hash(sx, sy, sm.th) & (hmask / POSE_BUCKET);
    if (gr.li < POSE_BUCKET) vs = htab[ps * POSE_BUCKET + gr.li];
  }
  tr_record r = expand_group<EG>(P, g, gr, nn, sm, lv, txy, tth TR_PH_PASS);
  TR_PH(5);
  if (look && r.status == TR_ST_PENDING) {   // rrt.py:179 `qnew in G`: first probe, before the arc
    pq = pose_hash(r.x, r.y, r.th) & (hmask / POSE_BUCKET);
    if (gr.li < POSE_BUCKET) vq = htab[pq * POSE_BUCKET + gr.li];
  }
#ifdef TR_DIAG_NOARC              // diagnosis builds only (tools/build_variants.py): arc skipped
  if (r.status == TR_ST_PENDING) r.status = TR_ST_OK;
#else
  if (r.status == TR_ST_PENDING) arc_finish<EG>(P, g, gr, txy, gx, gy, gth, r TR_PH_PASS);
#endif
  TR_PH(7);
  if (look) {
    if (group_lookup<EG>(gr, htab, hmask, ps, vs, sx, sy, sm.th, err) >= 0) {
      r.flags |= TR_FL_MEMBER;                 // skipped whatever it would have done
    } else if (r.status == TR_ST_OK) {
      const double2 o = txy[r.near];
      if (pose_eq(r.x, r.y, r.th, o.x, o.y, tth[r.near])) r.flags |= TR_FL_SAME_NEAR;   // rrt.py:187
      r.ex = group_lookup<EG>(gr, htab, hmask, pq, vq, r.x, r.y, r.th, err);
    }
  }
  if (gr.li == 0) rec[j] = r;
#ifdef TR_DIAG_PHASES
  TR_PH(8);
  if (gr.li == 0 && j < PH_ROWS) {
    unsigned long long* row = g_ph + ((da.e_hi % PH_RING) * PH_ROWS + j) * PH_N;
    for (int q = 0; q < PH_N - 1; ++q) row[q] = tp[q];
    row[PH_N - 1] = (unsigned long long)r.status | (tp[PH_N - 1] << 8) | (da.e_hi << 16);
  }
#endif
  TR_DLOG(3);                                // (thread 0's end: a lower bound of the block's)
}

// Stand-alone arc batch (API / parity): in10 rows, one wave each.
__global__ __launch_bounds__(256) void k_arc_batch(Grid g, const double* __restrict__ in10,
                                                   int64_t n, uint8_t* __restrict__ out,
                                                   int32_t* __restrict__ err) {
  const Grp<64> gr(threadIdx.x & 63);
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const double* a = in10 + 10 * j;
  Ctrl u{a[4], a[5], a[6], a[7], a[8], a[9] != 0 ? 1 : 0};
  int ierr = 0;
#ifdef TR_DIAG_PHASES
  unsigned long long tp[PH_N];
#endif
  bool blocked = arc_blocked_group<64>(g, gr, a[0], a[1], a[2], a[3], u, &ierr TR_PH_PASS);
  bool anyerr = gr.any(ierr != 0);
  if (gr.li == 0) {
    out[j] = blocked ? 0 : 1;
    if (anyerr) atomicOr(err, 1);
  }
}

// ------------------------------------------------------------------ LOS (search.py:35-41)
// One wave per ray (los_group): the pixels of a ray are tested in parallel, so a Theta* batch of
// long rays costs a few grid-load round trips per ray instead of one per pixel.
__global__ __launch_bounds__(256) void k_los_i32(Grid g, const int32_t* __restrict__ seg, int64_t n,
                                                 uint8_t* __restrict__ out, int32_t* err) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const int4 s = reinterpret_cast<const int4*>(seg)[j];
  int ierr = 0;
  const bool clear = los_group<64>(g, Grp<64>(lane), s.x, s.y, s.z, s.w, &ierr);
  if (lane == 0) {
    out[j] = clear ? 1 : 0;
    if (ierr) atomicOr(err, 1);
  }
}

__global__ __launch_bounds__(256) void k_los_f64(Grid g, const double* __restrict__ seg, int64_t n,
                                                 uint8_t* __restrict__ out, int32_t* err) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const double* s = seg + 4 * j;
  int ierr = 0;
  const bool clear = los_group<64>(g, Grp<64>(lane), trunc_i(s[0]), trunc_i(s[1]), trunc_i(s[2]),
                                   trunc_i(s[3]), &ierr);
  if (lane == 0) {
    out[j] = clear ? 1 : 0;
    if (ierr) atomicOr(err, 1);
  }
}

// ------------------------------------------------------------------ per-function batches (API)
__global__ void k_steer_batch(Params P, const double* __restrict__ in6, int64_t n,
                              double* __restrict__ out9) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double* a = in6 + 6 * j;
  double nx, ny, nth;
  Ctrl u;
  steer(P, a[0], a[1], a[2], a[3], a[4], a[5], nx, ny, nth, u);
  double* o = out9 + 9 * j;
  o[0] = nx; o[1] = ny; o[2] = nth;
  o[3] = u.steer; o[4] = u.iccx; o[5] = u.iccy; o[6] = u.rad; o[7] = u.dist;
  o[8] = u.straight ? 1.0 : 0.0;
}

__global__ void k_drive_batch(Params P, const double* __restrict__ in9, int64_t n,
                              double* __restrict__ out3, int32_t* __restrict__ ok) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double* a = in9 + 9 * j;
  Ctrl u{a[3], a[4], a[5], a[6], a[7], a[8] != 0 ? 1 : 0};
  double nx = 0, ny = 0, nth = 0;
  ok[j] = drive(P, a[0], a[1], a[2], u, nx, ny, nth) ? 1 : 0;
  out3[3 * j] = nx; out3[3 * j + 1] = ny; out3[3 * j + 2] = nth;
}

__global__ void k_body_batch(Params P, Grid g, const double* __restrict__ xyt, int64_t n,
                             double mult, uint8_t* __restrict__ out, int32_t* err) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  int ierr = 0;
  out[j] = body_clear(g, P, xyt[3 * j], xyt[3 * j + 1], xyt[3 * j + 2], mult, &ierr) ? 1 : 0;
  if (ierr) atomicOr(err, 1);
}

// ------------------------------------------------------------------ pixel lists, reference order
__global__ void k_bresenham_list(const double* seg, int64_t* out, int64_t cap, int64_t* count) {
  int64_t x0 = trunc_i(seg[0]), y0 = trunc_i(seg[1]), x1 = trunc_i(seg[2]), y1 = trunc_i(seg[3]);
  bool steep = !(llabs(y1 - y0) < llabs(x1 - x0));
  if (steep) { int64_t t = x0; x0 = y0; y0 = t; t = x1; x1 = y1; y1 = t; }
  if (x0 > x1) { int64_t t = x0; x0 = x1; x1 = t; t = y0; y0 = y1; y1 = t; }
  int64_t dx = x1 - x0, dy = y1 - y0, step = 1;
  if (dy < 0) { step = -1; dy = -dy; }
  int64_t e = 2 * dy - dx, y = y0, n = 0;
  for (int64_t x = x0; x <= x1; ++x, ++n) {
    if (n < cap) {
      out[2 * n] = steep ? y : x;
      out[2 * n + 1] = steep ? x : y;
    }
    if (e > 0) { y += step; e -= 2 * dx; }
    e += 2 * dy;
  }
  *count = n;
}

__device__ void emit(int64_t* out, int64_t cap, int64_t& n, int64_t x, int64_t y) {
  if (n < cap) { out[2 * n] = x; out[2 * n + 1] = y; }
  ++n;
}

// getCircle (search.py:107-142) then, for arcs, getArc's filter (search.py:161-181), in order.
__global__ void k_circle_list(Grid g, double cx, double cy, double rr, const double* arc10,
                              int64_t* out, int64_t cap, int64_t* count) {
  const int64_t xc = trunc_i(cx), yc = trunc_i(cy), r = trunc_i(rr);
  const int64_t K = circle_octant_len(r);
  ArcWin w;
  if (arc10) {
    Ctrl u{arc10[4], arc10[5], arc10[6], arc10[7], arc10[8], 0};
    w = arc_window(arc10[0], arc10[1], arc10[2], arc10[3], u);
  }
  int64_t n = 0;
  for (int64_t k = 0; k < K; ++k) {
    const int64_t x = circle_x(r, k);
    const int64_t vals[4] = {-x, x, -k, k};
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) {
        int64_t v1 = vals[a], v2 = vals[b];
        if ((v1 < 0 ? -v1 : v1) == (v2 < 0 ? -v2 : v2)) continue;
        int64_t px = xc + v1, py = yc + v2;
        if (!valid_i(g, px, py)) continue;
        if (arc10 && !arc_keeps(w, px, py)) continue;
        emit(out, cap, n, px, py);
      }
  }
  int64_t R2;
  if (circle_drawmore(g, xc, yc, r, K, R2)) {
    const int64_t dd[4][2] = {{R2, R2}, {-R2, -R2}, {R2, -R2}, {-R2, R2}};
    for (int i = 0; i < 4; ++i) {
      int64_t px = xc + dd[i][0], py = yc + dd[i][1];
      if (!valid_i(g, px, py)) continue;
      if (arc10 && !arc_keeps(w, px, py)) continue;
      emit(out, cap, n, px, py);
    }
  }
  *count = n;
}

#ifdef TR_DIAG_PHASES
// rows x PH_N stamps of the latest k_expand_arc launch (diagnosis builds only)
extern "C" int tr_diag_phases(unsigned long long* out) {   // PH_RING x PH_ROWS x PH_N
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph), sizeof(g_ph));
}
#endif

// ------------------------------------------------------------------ launchers
void launch_samples(hipStream_t st, const Params& P, const Grid& g, const double* gauss, int64_t B,
                    double gx, double gy, double gth, tr_sample* samples, int2* qxy, int32_t* live,
                    int32_t* zero) {
  hipLaunchKernelGGL(k_samples, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, P, g, gauss, B,
                     gx, gy, gth, samples, qxy, live, zero);
}
void launch_expand_arc(hipStream_t st, const Params& P, const Grid& g, const int64_t* nnidx,
                       int64_t B, const tr_sample* samples, const int32_t* live, const double2* txy,
                       const double* tth, double gx, double gy, double gth, const PoseSlot* htab,
                       uint64_t hmask, int32_t* err, tr_record* rec, DeltaArgs delta) {
  if (B <= 0) return;
  hipLaunchKernelGGL(k_expand_arc, dim3((unsigned)((B * EG + 255) / 256)), dim3(256), 0, st, P, g,
                     nnidx, B, samples, live, txy, tth, gx, gy, gth, htab, hmask, err, rec, delta);
}
void launch_arc_batch(hipStream_t st, const Grid& g, const double* in10, int64_t n, uint8_t* out,
                      int32_t* err) {
  hipLaunchKernelGGL(k_arc_batch, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, g, in10, n, out,
                     err);
}
void launch_los_i32(hipStream_t st, const Grid& g, const int32_t* seg, int64_t n, uint8_t* out,
                    int32_t* err) {
  hipLaunchKernelGGL(k_los_i32, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, g, seg, n, out,
                     err);
}
void launch_los_f64(hipStream_t st, const Grid& g, const double* seg, int64_t n, uint8_t* out,
                    int32_t* err) {
  hipLaunchKernelGGL(k_los_f64, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, g, seg, n, out,
                     err);
}
void launch_steer(hipStream_t st, const Params& P, const double* in6, int64_t n, double* out9) {
  hipLaunchKernelGGL(k_steer_batch, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, P, in6, n,
                     out9);
}
void launch_drive(hipStream_t st, const Params& P, const double* in9, int64_t n, double* out3,
                  int32_t* ok) {
  hipLaunchKernelGGL(k_drive_batch, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, P, in9, n,
                     out3, ok);
}
void launch_body(hipStream_t st, const Params& P, const Grid& g, const double* xyt, int64_t n,
                 double mult, uint8_t* out, int32_t* err) {
  hipLaunchKernelGGL(k_body_batch, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, P, g, xyt, n,
                     mult, out, err);
}
void launch_bresenham_list(hipStream_t st, const double* seg, int64_t* out, int64_t cap,
                           int64_t* count) {
  hipLaunchKernelGGL(k_bresenham_list, dim3(1), dim3(1), 0, st, seg, out, cap, count);
}
void launch_circle_list(hipStream_t st, const Grid& g, double cx, double cy, double r,
                        const double* arc10, int64_t* out, int64_t cap, int64_t* count) {
  hipLaunchKernelGGL(k_circle_list, dim3(1), dim3(1), 0, st, g, cx, cy, r, arc10, out, cap, count);
}

}  // namespace tr
