// Host program (no kernel launch): arc_keeps (cross products, geom.hpp) against arc_keeps_angles (the
// reference's angle comparisons, search.py:161-181) over random arcs, integral centres with pixels on
// the begin / land rays, large radii and wide windows.  Built and run by tests/test_host.py.
#include "geom.hpp"
#include <cstdio>
#include <random>
using namespace tr;
int main() {
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(0, 1);
  long bad = 0, n = 0, amb = 0;
  for (int it = 0; it < 400000; ++it) {
    Ctrl u;
    const int mode = it % 4;
    u.iccx = mode == 1 ? floor(U(g) * 300) : U(g) * 600 - 150;
    u.iccy = mode == 1 ? floor(U(g) * 300) : U(g) * 600 - 150;
    u.rad = mode == 2 ? U(g) * 20000 : 2.3 + U(g) * 60;
    u.steer = U(g) < 0.5 ? -(U(g) * 65) : U(g) * 65;
    if (it % 97 == 0) u.steer = 0;
    u.dist = 30; u.straight = 0;
    double ab = U(g) * 2 * kPi, sweep = mode == 3 ? U(g) * 2 * kPi : U(g) * 1.2;
    double bx = u.iccx + u.rad * cos(ab), by = u.iccy + u.rad * sin(ab);
    double ae = ab + (U(g) < 0.5 ? sweep : -sweep);
    double lx = u.iccx + u.rad * cos(ae), ly = u.iccy + u.rad * sin(ae);
    if (mode == 1) { bx = rint(bx); by = rint(by); lx = rint(lx); ly = rint(ly); }   // integral: pixels on the rays
    ArcWin w = arc_window(bx, by, lx, ly, u);
    for (int k = 0; k < 24; ++k) {
      int64_t px, py;
      if (k < 12) {
        double a = U(g) * 2 * kPi, r = u.rad + U(g) * 4 - 2;
        px = (int64_t)(u.iccx + r * cos(a)); py = (int64_t)(u.iccy + r * sin(a));
      } else {          // multiples of the begin / land direction from an integral centre
        double f = (k - 11) * (U(g) < 0.5 ? 1.0 : -1.0);
        const bool useb = k & 1;
        px = (int64_t)rint(u.iccx + f * (useb ? w.bvx : w.evx)); py = (int64_t)rint(u.iccy + f * (useb ? w.bvy : w.evy));
      }
      const bool a1 = arc_keeps(w, px, py), a2 = arc_keeps_angles(w, px, py);
      const double vx = px - w.iccx, vy = py - w.iccy, s1 = w.bvx * vy - w.bvy * vx;
      if (!(s1 * s1 > 1e-16 * (vx * vx + vy * vy) * w.bn2)) ++amb;
      ++n;
      if (a1 != a2) { if (bad++ < 10) printf("MISMATCH it %d px %ld %ld steer %g diff %g\n", it, (long)px, (long)py, u.steer, w.diff); }
    }
  }
  printf("checked %ld, ambiguous(begin) %ld, mismatches %ld\n", n, amb, bad);
  return bad != 0;
}
