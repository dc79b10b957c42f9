// Device-side restatement of the theta-rrt per-sample geometry (freespace, steer, drive, body rays, circle / arc pixels).
//
// Every numeric step mirrors the reference expression it replaces, in the same operation order,
// because node coordinates feed exact-value dedupe (rrt.py:179) and branch decisions
// (rrt.py:348,368,375; search.py:170-179).  Compiled with contraction OFF (pragma below and
// -ffp-contract=off): an FMA appears only where the reference's own numpy/OpenBLAS call is an FMA
// on the reference host (np.dot / np.linalg.norm of 2-vectors, the 2x2 dgesv update steps).
//
// scipy Rotation (compiled, no source in the image) is restated from its published algorithm:
// from_euler('z') quaternion, as_matrix apply, quaternion compose + normalise, as_euler('xyz')
// (Bernardes & Viollet form used by scipy >= 1.11).  Oracle twin: oracle/thetarrt_oracle.py.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define TR_HD __host__ __device__ __forceinline__

namespace tr {

constexpr double kDeg = 0.017453292519943295;   // np.deg2rad multiplier  (pi/180)
constexpr double kRad = 57.29577951308232;      // np.rad2deg multiplier  (180/pi)
constexpr double kPi = 3.141592653589793;
constexpr double kSqrt2 = 1.4142135623730951;   // math.sqrt(2)

struct Params {           // builtins block, main.py:14-32
  double bikelength, leftc, rightc, frontclearance, maxdrivedist, weightxy, xystdv, anglestdv;
  double tol_xy, tol_ang;
  int32_t forwardonly, pad;
};

// builtins.imarray: bool [H][W], True = free (main.py:42), one bit per cell: row y is `wpr` 32-bit
// words, cell (x, y) is bit x & 31 of word y * wpr + (x >> 5) (1 = free; the padding bits of a
// row's last word are 0).  512^2 is 32 KB, 2048^2 512 KB: the whole map stays in every cache
// level that a byte map 8 times its size would fall out of.
struct Grid {
  const uint32_t* bits;
  int64_t H, W;           // shape[0], shape[1]
  int64_t wpr;            // words per row = ceil(W / 32)
};

// The occupancy bit of a cell inside the array (callers have checked 0 <= x < W, 0 <= y < H).
TR_HD uint32_t grid_bit(const Grid& g, int64_t x, int64_t y) {
  return (g.bits[y * g.wpr + (x >> 5)] >> (x & 31)) & 1u;
}
// The same as an unconditional load: `inside` false reads word 0 (the caller masks the result), so
// a lane's loads of a round issue back to back whatever their classes.
TR_HD uint32_t grid_bit_if(const Grid& g, bool inside, int64_t x, int64_t y) {
  const int64_t w = inside ? y * g.wpr + (x >> 5) : 0;
  return (g.bits[w] >> (inside ? (x & 31) : 0)) & 1u;
}
TR_HD int64_t grid_words(int64_t H, int64_t W) { return H * ((W + 31) / 32); }

struct V2 { double x, y; };
struct V3 { double x, y, z; };

// Control u = (steerangle, ICC, rad, traveldist); straight = the (0, None, None, d) form.
struct Ctrl { double steer, iccx, iccy, rad, dist; int32_t straight; };

// ------------------------------------------------------------------ angles (rrt.py:9-14,73-77,108-115)
TR_HD double wrap180(double a) {                 // standardangle
  while (a > 180) a = a - 360;
  while (a <= -180) a = a + 360;
  return a;
}

// sin / cos of h = deg * (pi/180) / 2 for the right angles steer and drive rotate by (rrt.py:
// 313-333, 373, 407, 285): the host libm values (math.sin / math.cos), no range reduction.
constexpr double kS45 = 0x1.6a09e667f3bccp-1, kC45 = 0x1.6a09e667f3bcdp-1;   // h = +-pi/4
constexpr double kC90 = 0x1.1a62633145c07p-54;                                // cos(+-pi/2)

TR_HD void zquat(double deg, double& z, double& w) {   // from_euler('z', deg, degrees=True)
  if (deg == 90.0 || deg == -90.0) { z = deg > 0 ? kS45 : -kS45; w = kC45; return; }
  if (deg == 180.0 || deg == -180.0) { z = deg > 0 ? 1.0 : -1.0; w = kC90; return; }
  double h = deg * kDeg / 2;
  sincos(h, &z, &w);                                    // one range reduction, same values
}

// Rotation.from_euler('z', deg).apply(v): scipy as_matrix() then row-wise dot, left to right.
// Matrix of the (0, 0, z, w) quaternion applied to v, as scipy does it (zrot below).
TR_HD V3 zrot_q(double z, double w, V3 v) {
  const double x = 0.0, y = 0.0;
  double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
  double xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
  double m00 = x2 - y2 - z2 + w2, m01 = 2 * (xy - zw), m02 = 2 * (xz + yw);
  double m10 = 2 * (xy + zw), m11 = -x2 + y2 - z2 + w2, m12 = 2 * (yz - xw);
  double m20 = 2 * (xz - yw), m21 = 2 * (yz + xw), m22 = -x2 - y2 + z2 + w2;
  V3 r;
  r.x = m00 * v.x + m01 * v.y + m02 * v.z;
  r.y = m10 * v.x + m11 * v.y + m12 * v.z;
  r.z = m20 * v.x + m21 * v.y + m22 * v.z;
  return r;
}

TR_HD V3 zrot(double deg, V3 v) {
  double z, w;
  zquat(deg, z, w);
  return zrot_q(z, w, v);
}

// anglediff(a1, a2) = degrees(as_euler('xyz')[2] of Rz(a1).inv() * Rz(a2)), exact scipy arithmetic.
TR_HD double angle_diff_exact(double a1, double a2) {
  double pz, pw, qz, qw;
  zquat(a1, pz, pw);
  zquat(a2, qz, qw);
  const double px = -0.0, py = -0.0;  // inv() negates the vector part
  pz = -pz;
  const double qx = 0.0, qy = 0.0;
  double c0 = py * qz - pz * qy, c1 = pz * qx - px * qz, c2 = px * qy - py * qx;
  double r0 = pw * qx + qw * px + c0;
  double r1 = pw * qy + qw * py + c1;
  double r2 = pw * qz + qw * pz + c2;
  double r3 = pw * qw - (px * qx + py * qy + pz * qz);
  double n = sqrt(r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3);
  double x = r0 / n, y = r1 / n, z = r2 / n, w = r3 / n;
  double ang = atan2(x + z, w - y) + atan2(z - x, y + w);
  if (ang < -kPi) ang += 2 * kPi;
  else if (ang > kPi) ang -= 2 * kPi;
  return ang * kRad;
}

// Same value outside a 1e-9 deg band around the 0 / +-180 branch points, where only the sign or a
// `< 180` comparison of the result is consumed (search.py:170-179).  Closed form error < 1e-11 deg.
TR_HD double angle_diff_fast(double a1, double a2) {
  double d = a2 - a1;
  if (d > 180) d -= 360;
  else if (d <= -180) d += 360;
  double ad = fabs(d);
  if (ad < 1e-9 || ad > 180 - 1e-9) return angle_diff_exact(a1, a2);
  return d;
}

// anglebetween(v1, v2): np.dot of two float 2-vectors is fma(v1.y, v2.y, v1.x*v2.x) on the host.
TR_HD double angle_between(V2 a, V2 b) {
  double dot = fma(a.y, b.y, a.x * b.x);
  double det = b.x * a.y - a.x * b.y;
  return wrap180(atan2(det, dot) * kRad);
}

// anglebetween([1,0], v)
TR_HD double heading(double vx, double vy) {
  double dot = fma(0.0, vy, 1.0 * vx);
  double det = vx * 0.0 - 1.0 * vy;
  return wrap180(atan2(det, dot) * kRad);
}

TR_HD double norm2(double x, double y) { return sqrt(fma(y, y, x * x)); }   // np.linalg.norm

TR_HD double arc_len(double radius, double angle) {          // angle_to_arclength, rrt.py:48-51
  while (angle < 0) angle = angle + 360;
  return (kPi * 2 * radius) * angle / 360;
}
TR_HD double arc_angle(double radius, double len) {          // arclength_to_angle, rrt.py:70-71
  return len * 360 / (kPi * 2 * radius);
}

// ------------------------------------------------------------------ 2x2 solve (np.linalg.solve / cond)
// OpenBLAS dgesv on the reference host: partial pivoting, l = a10 * (1/a00), u11 = a11 - l*a01,
// forward step fma(-l, b0, b1), back substitution x1 = y1/u11, x0 = fma(-x1, a01, b0)/a00.
// Returns false where numpy raises LinAlgError or cond(a) > 1e6 (rrt.py:347-350, 388-391).
TR_HD bool solve_icc(double a00, double a01, double a10, double a11, double b0, double b1, V2& out) {
  // cond_2(A) = smax / smin = smax^2 / |det|
  double w = a01 * a10;
  double det = fma(a00, a11, -w) + fma(-a01, a10, w);
  double S = a00 * a00 + a01 * a01 + a10 * a10 + a11 * a11;
  double ad = fabs(det);
  double disc = sqrt(fmax(0.0, (S - 2 * ad) * (S + 2 * ad)));
  double smax2 = (S + disc) / 2;
  if (fabs(a10) > fabs(a00)) {
    double t;
    t = a00; a00 = a10; a10 = t;
    t = a01; a01 = a11; a11 = t;
    t = b0; b0 = b1; b1 = t;
  }
  if (a00 == 0.0) return false;
  double l = a10 * (1.0 / a00);
  double u11 = a11 - l * a01;
  if (u11 == 0.0) return false;
  if (!(smax2 <= 1000000.0 * ad)) return false;   // cond > 1e6 (inf when det == 0)
  double y1 = fma(-l, b0, b1);
  double x1 = y1 / u11;
  double x0 = fma(-x1, a01, b0) / a00;
  out.x = x0;
  out.y = x1;
  return true;
}

// linefrompoints(p, p + d), rrt.py:42-46
TR_HD void line_coefs(V2 p, V2 q, double& a, double& b, double& c) {
  a = q.y - p.y;
  b = p.x - q.x;
  c = a * p.x + b * p.y;
}

// ------------------------------------------------------------------ grid queries (search.py:13-41)
TR_HD int64_t trunc_i(double v) { return (int64_t)v; }     // Python int(): toward zero

TR_HD bool valid_i(const Grid& g, int64_t x, int64_t y) {   // search.py:17-24 (x vs shape[0]!)
  return x >= 0 && y >= 0 && x < g.H && y < g.W;
}

// freespace for an integer pixel; *ierr set where numpy would raise IndexError (non-square maps).
TR_HD bool free_i(const Grid& g, int64_t x, int64_t y, int* ierr) {
  if (!valid_i(g, x, y)) return false;
  if (y >= g.H || x >= g.W) { *ierr = 1; return false; }
  return grid_bit(g, x, y) != 0;
}

// lineofsight(n1, n2) on already-truncated endpoints: every Bresenham pixel free (search.py:35-94).
TR_HD bool los_i(const Grid& g, int64_t x0, int64_t y0, int64_t x1, int64_t y1, int* ierr) {
  bool steep = !(llabs(y1 - y0) < llabs(x1 - x0));
  if (steep) { int64_t t = x0; x0 = y0; y0 = t; t = x1; x1 = y1; y1 = t; }
  if (x0 > x1) { int64_t t = x0; x0 = x1; x1 = t; t = y0; y0 = y1; y1 = t; }
  int64_t dx = x1 - x0, dy = y1 - y0, step = 1;
  if (dy < 0) { step = -1; dy = -dy; }
  int64_t err = 2 * dy - dx, y = y0;
  for (int64_t x = x0; x <= x1; ++x) {
    bool f = steep ? free_i(g, y, x, ierr) : free_i(g, x, y, ierr);
    if (!f) return false;
    if (err > 0) { y += step; err -= 2 * dx; }
    err += 2 * dy;
  }
  return true;
}

TR_HD bool los(const Grid& g, V2 a, V2 b, int* ierr) {
  return los_i(g, trunc_i(a.x), trunc_i(a.y), trunc_i(b.x), trunc_i(b.y), ierr);
}

// bike_clear (mult = 1) / front_of_bike_clear (mult = frontclearance), rrt.py:208-222
// The same test with every pixel's grid byte loaded at once (no dependent chain of loads): pixel
// states in Bresenham order, then the first non-free one decides (blocked, or the reference's
// IndexError when it is outside a non-square array).  Lines of more than MAXP pixels fall back.
template <int MAXP>
TR_HD bool los_i_par(const Grid& g, int64_t x0, int64_t y0, int64_t x1, int64_t y1, int* ierr) {
  bool steep = !(llabs(y1 - y0) < llabs(x1 - x0));
  if (steep) { int64_t t = x0; x0 = y0; y0 = t; t = x1; x1 = y1; y1 = t; }
  if (x0 > x1) { int64_t t = x0; x0 = x1; x1 = t; t = y0; y0 = y1; y1 = t; }
  int64_t dx = x1 - x0, dy = y1 - y0, step = 1;
  if (dy < 0) { step = -1; dy = -dy; }
  if (dx + 1 > MAXP) return steep ? los_i(g, y0, x0, y1, x1, ierr) : los_i(g, x0, y0, x1, y1, ierr);
  int64_t err = 2 * dy - dx, y = y0;
  uint8_t st[MAXP];                     // 0 free, 1 blocked, 2 index error
#pragma unroll
  for (int k = 0; k < MAXP; ++k) {
    const int64_t x = x0 + k;
    const int64_t px = steep ? y : x, py = steep ? x : y;
    st[k] = 0;
    if (k <= dx) {
      if (!valid_i(g, px, py)) st[k] = 1;
      else if (py >= g.H || px >= g.W) st[k] = 2;
      else st[k] = grid_bit(g, px, py) != 0 ? 0 : 1;
    }
    if (err > 0) { y += step; err -= 2 * dx; }
    err += 2 * dy;
  }
#pragma unroll
  for (int k = 0; k < MAXP; ++k) {
    if (st[k] == 2) { *ierr = 1; return false; }
    if (st[k] == 1) return false;
  }
  return true;
}

TR_HD bool body_clear(const Grid& g, const Params& P, double x, double y, double th, double mult,
                      int* ierr) {
  V3 f = zrot(th, V3{P.bikelength * mult, 0, 0});
  double px = f.x + x, py = f.y + y;
  return los_i_par<16>(g, trunc_i(x), trunc_i(y), trunc_i(px), trunc_i(py), ierr);
}

// Pixel states of a Bresenham line of at most MAXP pixels (los_i_par's first half): returns the
// first non-free state (0 free, 1 blocked, 2 index error), or -1 when the line is longer.  Every
// pixel's byte is loaded unconditionally (out-of-range pixels read byte 0 and are masked after),
// so the MAXP loads issue back to back and the wave waits once instead of once per pixel.
template <int MAXP>
TR_HD int line_state(const Grid& g, int64_t x0, int64_t y0, int64_t x1, int64_t y1) {
  bool steep = !(llabs(y1 - y0) < llabs(x1 - x0));
  if (steep) { int64_t t = x0; x0 = y0; y0 = t; t = x1; x1 = y1; y1 = t; }
  if (x0 > x1) { int64_t t = x0; x0 = x1; x1 = t; t = y0; y0 = y1; y1 = t; }
  int64_t dx = x1 - x0, dy = y1 - y0, step = 1;
  if (dy < 0) { step = -1; dy = -dy; }
  if (dx + 1 > MAXP) return -1;
  int64_t err = 2 * dy - dx, y = y0;
  uint8_t cls[MAXP], v[MAXP];          // cls: 0 load decides, 1 blocked, 2 index error, 3 past end
#pragma unroll
  for (int k = 0; k < MAXP; ++k) {
    const int64_t x = x0 + k;
    const int64_t px = steep ? y : x, py = steep ? x : y;
    const bool ok = valid_i(g, px, py), inb = py < g.H && px < g.W;
    cls[k] = k > dx ? 3 : (!ok ? 1 : (!inb ? 2 : 0));
    v[k] = (uint8_t)grid_bit_if(g, cls[k] == 0, px, py);
    if (err > 0) { y += step; err -= 2 * dx; }
    err += 2 * dy;
  }
#pragma unroll
  for (int k = 0; k < MAXP; ++k) {
    const int st = cls[k] == 0 ? (v[k] != 0 ? 0 : 1) : (cls[k] == 3 ? 0 : cls[k]);
    if (st) return st;
  }
  return 0;
}

// rrt.py:169: valid(qnew) and bike_clear(qnew) and front_of_bike_clear(qnew), short-circuit and
// IndexError semantics kept, with one rotation for both rays and both rays' pixels loaded at once.
TR_HD bool body_rays_clear(const Grid& g, const Params& P, double x, double y, double th, int* ierr) {
  const int64_t x0 = trunc_i(x), y0 = trunc_i(y);
  if (!valid_i(g, x0, y0)) return false;
  double z, w;
  zquat(th, z, w);
  // zrot's matrix for a (0, 0, z, w) quaternion; rows applied to (L, 0, 0) left to right
  const double x2 = 0.0, y2 = 0.0, z2 = z * z, w2 = w * w, xy = 0.0, zw = z * w;
  const double m00 = x2 - y2 - z2 + w2, m01 = 2 * (xy - zw), m02 = 2 * (0.0 * z + 0.0 * w);
  const double m10 = 2 * (xy + zw), m11 = -x2 + y2 - z2 + w2, m12 = 2 * (0.0 * z - 0.0 * w);
  double ex[2], ey[2];
  const double len[2] = {P.bikelength * 1.0, P.bikelength * P.frontclearance};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    ex[r] = (m00 * len[r] + m01 * 0.0 + m02 * 0.0) + x;
    ey[r] = (m10 * len[r] + m11 * 0.0 + m12 * 0.0) + y;
  }
  const int s1 = line_state<16>(g, x0, y0, trunc_i(ex[0]), trunc_i(ey[0]));
  const int s2 = line_state<16>(g, x0, y0, trunc_i(ex[1]), trunc_i(ey[1]));
  if (s1 < 0 || s2 < 0)         // long rays (large bikelength): the sequential test
    return body_clear(g, P, x, y, th, 1.0, ierr) && body_clear(g, P, x, y, th, P.frontclearance, ierr);
  if (s1 == 2 || (s1 == 0 && s2 == 2)) { *ierr = 1; return false; }
  return s1 == 0 && s2 == 0;
}

// ------------------------------------------------------------------ drive (rrt.py:272-304)
// Returns false for a straight control: the reference raises TypeError there (rrt.py:275 -> :71).
TR_HD bool drive(const Params& P, double ox, double oy, double oth, const Ctrl& u, double& nx,
                 double& ny, double& nth) {
  if (u.straight) return false;
  double ang = arc_angle(u.rad, u.dist);
  V3 front = zrot(oth, V3{P.bikelength, 0, 0});
  V3 back = zrot(180, front);
  double dx = ox - u.iccx, dy = oy - u.iccy, dz = 0.0 - 0.0;
  front = V3{dx + front.x, dy + front.y, dz + front.z};
  back = V3{dx + back.x, dy + back.y, dz + back.z};
  double rot = u.steer < 0 ? -ang : ang;
  double rz, rw;
  zquat(rot, rz, rw);                  // one rotation for both points
  front = zrot_q(rz, rw, front);
  back = zrot_q(rz, rw, back);
  double fx = u.iccx + front.x, fy = u.iccy + front.y;
  double bx = u.iccx + back.x, by = u.iccy + back.y;
  double mx = 0.5 * (bx + fx), my = 0.5 * (by + fy);
  nx = mx;
  ny = my;
  nth = -heading(fx - mx, fy - my);
  return true;
}

// ------------------------------------------------------------------ steer (rrt.py:306-541)
// Sample goal (gx, gy) is integral (rand_conf truncates, rrt.py:68).
TR_HD void steer(const Params& P, double ox, double oy, double th, double gx, double gy, double tg,
                 double& nx, double& ny, double& nth, Ctrl& u) {
  V2 mid{0.5 * (ox + gx), 0.5 * (oy + gy)};
  double bisx = ox - gx, bisy = oy - gy;
  V3 frame = zrot(th, V3{P.bikelength, 0, 0});
  V3 normal = zrot(90, frame);
  V3 perp = zrot(90, V3{bisx, bisy, 0});
  double a1, b1, c1, a2, b2, c2;
  line_coefs(mid, V2{mid.x + perp.x, mid.y + perp.y}, a1, b1, c1);
  line_coefs(V2{ox, oy}, V2{ox + normal.x, oy + normal.y}, a2, b2, c2);
  V2 icc;
  bool ok = solve_icc(a1, b1, a2, b2, c1, c2, icc);
  double steer_a = 0, rad = 0;
  bool limited = false;
  V2 pivot{frame.x + ox, frame.y + oy};
  if (ok) {
    rad = norm2(ox - icc.x, oy - icc.y);
    V3 sv = zrot(90, V3{pivot.x - icc.x, pivot.y - icc.y, 0});
    steer_a = wrap180(-angle_between(V2{frame.x, frame.y}, V2{sv.x, sv.y}));
    if (P.forwardonly && (steer_a > 90 || steer_a < -90)) steer_a = wrap180(steer_a + 180);
    if (steer_a < P.leftc || steer_a > P.rightc) {
      steer_a = steer_a < P.leftc ? P.leftc : P.rightc;
      V3 fn = zrot(steer_a, normal);
      line_coefs(pivot, V2{pivot.x + fn.x, pivot.y + fn.y}, a1, b1, c1);
      line_coefs(V2{ox, oy}, V2{ox + normal.x, oy + normal.y}, a2, b2, c2);
      ok = solve_icc(a1, b1, a2, b2, c1, c2, icc);
      if (ok) rad = norm2(ox - icc.x, oy - icc.y);
      limited = true;
    }
  }
  if (!ok) {                       // straight branch, rrt.py:526-541
    double vx = gx - ox, vy = gy - oy;
    nx = gx;
    ny = gy;
    double n = norm2(vx, vy);
    if (n > 0.000001) {
      double sx = P.maxdrivedist * vx / norm2(vx, vy), sy = P.maxdrivedist * vy / norm2(vx, vy);
      if (!(norm2(sx, sy) > norm2(vx, vy))) { nx = ox + sx; ny = oy + sy; }
    }
    nth = th;
    u = Ctrl{0, 0, 0, 0, 1, 1};
    return;
  }
  double ccw = ((steer_a >= 0 && steer_a < 90) || (steer_a <= -90 && steer_a > -180)) ? -90 : 90;
  auto tangent_heading = [&](double px, double py) {
    V3 f = zrot(-ccw, V3{px - icc.x, py - icc.y, 0});
    return -heading(f.x, f.y);
  };
  double fin = tangent_heading(gx, gy);
  double mix = P.weightxy * wrap180(fin) + (1 - P.weightxy) * wrap180(tg);
  if (limited) mix = heading(gx - ox, gy - oy);
  double t2 = mix + ccw;
  double goal_ang = heading(gx - icc.x, gy - icc.y);
  V2 mp[2];
  double dd[2];
  for (int k = 0; k < 2; ++k) {
    V3 m = zrot(k == 0 ? t2 : t2 + 180, V3{1, 0, 0});
    double n = norm2(m.x, m.y);
    V2 q{icc.x + rad * m.x / n, icc.y + rad * m.y / n};
    mp[k] = q;
    dd[k] = angle_diff_fast(heading(q.x - icc.x, q.y - icc.y), goal_ang);
  }
  // only the order of |dd| is used: the closed form decides unless the two are within its error
  if (fabs(fabs(dd[0]) - fabs(dd[1])) < 1e-9)
    for (int k = 0; k < 2; ++k)
      dd[k] = angle_diff_exact(heading(mp[k].x - icc.x, mp[k].y - icc.y), goal_ang);
  fin = mix;
  V2 gp;
  if (fabs(dd[0]) < fabs(dd[1])) {
    gp = mp[0];
  } else {
    gp = mp[1];
    fin = wrap180(fin - 180);
  }
  if (limited) {
    gp = mp[0];
    fin = tangent_heading(gp.x, gp.y);
  }
  double tox = ox - icc.x, toy = oy - icc.y;
  double arc = angle_diff_exact(heading(gp.x - icc.x, gp.y - icc.y), heading(tox, toy));
  if (steer_a > 0) {
    if (arc < 0) arc = 360 + arc;
  } else if (arc > 0) {
    arc = 360 - arc;
  }
  double dist = arc_len(rad, fabs(arc));
  if (dist > P.maxdrivedist) {
    dist = P.maxdrivedist;
    double turn = arc_angle(rad, P.maxdrivedist);
    V3 q = zrot(steer_a < 0 ? -turn : turn, V3{tox, toy, 0});
    gp = V2{q.x + icc.x, q.y + icc.y};
    fin = tangent_heading(gp.x, gp.y);
  }
  nx = gp.x;
  ny = gp.y;
  nth = fin;
  u = Ctrl{steer_a, icc.x, icc.y, rad, dist, 0};
}

// ------------------------------------------------------------------ midpoint circle (search.py:96-142)
// The octant walk of getCircle emits (x_k, k) for k = 0..K-1 with
//   x_k = min{ x >= 0 : x(x+1) >= r^2 - k^2 }   and K = first k with x_k <= k
// (d = x^2 - x + (k+1)^2 - r^2 is the walk's decision variable).  Closed form lets a
// wave test only the pixels near the arc instead of walking a circle of up to 10^5 pixels.
TR_HD int64_t circle_x(int64_t r, int64_t k) {
  int64_t T = r * r - k * k;
  if (T <= 0) return 0;
  int64_t x = (int64_t)((sqrt(4.0 * (double)T + 1.0) - 1.0) * 0.5);
  if (x < 0) x = 0;
  while (x * (x + 1) < T) ++x;
  while (x > 0 && (x - 1) * x >= T) --x;
  return x;
}

TR_HD int64_t circle_octant_len(int64_t r) {
  if (r <= 0) return 0;
  int64_t k = (int64_t)((double)r * 0.70710678118654752) - 2;
  if (k < 0) k = 0;
  while (k > 0 && circle_x(r, k - 1) <= k - 1) --k;
  while (circle_x(r, k) > k) ++k;
  return k;
}

TR_HD bool circle_member(int64_t r, int64_t K, int64_t a, int64_t b) {   // |a| != |b| offsets
  a = a < 0 ? -a : a;
  b = b < 0 ? -b : b;
  return (b < K && circle_x(r, b) == a) || (a < K && circle_x(r, a) == b);
}

// Image m (0..7) of octant point (x, k): offsets (dx, dy).
TR_HD void circle_image(int m, int64_t x, int64_t k, int64_t& dx, int64_t& dy) {
  int64_t p = (m & 4) ? k : x, q = (m & 4) ? x : k;
  dx = (m & 1) ? -p : p;
  dy = (m & 2) ? -q : q;
}

// getCircle's diagonal patch decision (search.py:124-138).
TR_HD bool circle_drawmore(const Grid& g, int64_t xc, int64_t yc, int64_t r, int64_t K, int64_t& R2) {
  R2 = (int64_t)rint((double)r * 0.5 * kSqrt2);
  const int64_t tx = xc + R2, ty = yc + R2;
  const int64_t nb[4][2] = {{tx + 1, ty}, {tx - 1, ty}, {tx, ty + 1}, {tx, ty - 1}};
  for (int i = 0; i < 4; ++i) {
    int64_t a = nb[i][0] - xc, b = nb[i][1] - yc;
    if ((a < 0 ? -a : a) == (b < 0 ? -b : b)) continue;     // never emitted (|v1| == |v2|)
    if (valid_i(g, nb[i][0], nb[i][1]) && circle_member(r, K, a, b)) return false;
  }
  return true;
}

// The arc window of getArc (search.py:150-160).
struct ArcWin {
  double iccx, iccy, b_ang, e_ang, diff, steer;
  double bvx, bvy, evx, evy, bn2, en2;   // begin / land directions from the ICC, their squared norms
};

TR_HD ArcWin arc_window(double bx, double by, double lx, double ly, const Ctrl& u) {
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
  w.b_ang = heading(w.bvx, w.bvy);
  w.e_ang = heading(w.evx, w.evy);
  // consumed as a sign, `< 180` (angle_diff_fast is exact around both) and a box margin
  double d = u.steer < 0 ? angle_diff_fast(w.b_ang, w.e_ang) : angle_diff_fast(w.e_ang, w.b_ang);
  if (d < 0) d = 360 + d;
  w.diff = d;
  return w;
}

// Keep test for one circle pixel (search.py:161-181), through the angles as the reference takes it.
TR_HD bool arc_keeps_angles(const ArcWin& w, int64_t px, int64_t py) {
  double a = heading((double)px - w.iccx, (double)py - w.iccy);
  double fwd, bwd;
  if (w.steer > 0) {
    fwd = angle_diff_fast(a, w.b_ang);
    bwd = angle_diff_fast(w.e_ang, a);
  } else {
    fwd = angle_diff_fast(w.b_ang, a);
    bwd = angle_diff_fast(a, w.e_ang);
  }
  if (w.diff < 180) return fwd >= 0 && bwd >= 0;
  return fwd >= 0 || bwd >= 0;
}

// The same decision from cross products.  Only the signs of fwd and bwd are consumed, and with
// image-frame angles (heading = -atan2(vy, vx) in degrees) the wrapped difference b_ang - a has the
// sign of sin(phi(v) - phi(b)) = cross(b, v) / (|b| |v|), likewise a - e_ang that of cross(v, e).
// The angles carry rounding errors near 1e-13 deg and angle_diff_fast switches to the quaternion
// form inside 1e-9 deg of 0 and 180, so a sine above 1e-8 in magnitude (5.7e-7 deg) fixes the sign
// for both; anything closer takes the angle path.
TR_HD bool arc_keeps(const ArcWin& w, int64_t px, int64_t py) {
  const double vx = (double)px - w.iccx, vy = (double)py - w.iccy;
  const double vn2 = vx * vx + vy * vy;
  double s1 = w.bvx * vy - w.bvy * vx;      // sign of b_ang - a
  double s2 = vx * w.evy - vy * w.evx;      // sign of a - e_ang
  const double t1 = 1e-16 * (vn2 * w.bn2), t2 = 1e-16 * (vn2 * w.en2);
  if (!(s1 * s1 > t1) || !(s2 * s2 > t2)) return arc_keeps_angles(w, px, py);
  if (!(w.steer > 0)) { s1 = -s1; s2 = -s2; }
  if (w.diff < 180) return s1 > 0 && s2 > 0;
  return s1 > 0 || s2 > 0;
}

}  // namespace tr
