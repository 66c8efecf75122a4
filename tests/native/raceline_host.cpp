// Host harness for csrc/raceline.hpp (test infrastructure): runs the device ConstantSpeed
// walker on the CPU over tables and starts written by tests/test_raceline_native.py and
// prints the per-model references, so the Python test compares them with the oracle —
// built with AddressSanitizer (host code only) to catch any out-of-bounds table access.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "raceline.hpp"

static std::vector<double> read_all(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) { std::perror(path); std::exit(2); }
  std::vector<double> v;
  double x;
  while (std::fread(&x, sizeof x, 1, f) == 1) v.push_back(x);
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  // tables.bin: n, M, knots[n], xy[8(n-1)], speed[4(n-1)M], mus[M]
  // cases.bin:  H, then per case (mu, s0, v0, scale, Ts)
  // argv[3] = "win": the speed profiles through the window of the kernel's prologue
  // (seg0 by bisect-right on s0, window_need segments from the table's bounds)
  if (argc < 3) return 2;
  const bool win = argc > 3 && argv[3][0] == 'w';
  const std::vector<double> t = read_all(argv[1]), c = read_all(argv[2]);
  const int n = (int)t[0], M = (int)t[1];
  const size_t m = n - 1;
  std::vector<double> knots(t.begin() + 2, t.begin() + 2 + n);
  std::vector<double> xy(t.begin() + 2 + n, t.begin() + 2 + n + 8 * m);
  std::vector<double> speed(t.begin() + 2 + n + 8 * m, t.begin() + 2 + n + 8 * m + 4 * m * M);
  std::vector<double> mus(t.begin() + 2 + n + 8 * m + 4 * m * M, t.end());
  knots.resize(n + llampc::kKnotPad, INFINITY);   // the walker's +inf pad (raceline.hpp)
  double hmin = knots[1] - knots[0];
  for (int i = 2; i < n; ++i) hmin = std::min(hmin, knots[i] - knots[i - 1]);
  const double vmax = llampc::speed_bound(knots.data(), speed.data(), n, M);
  llampc::RacelineK r{knots.data(), xy.data(), speed.data(), mus.data(), n, M, (int)m, hmin, vmax};
  const int H = (int)c[0];
  std::vector<double> wbuf;
  for (size_t i = 1; i + 5 <= c.size(); i += 5) {
    llampc::SpeedWin sw{nullptr, 0, 0};
    if (win) {                           // the kernel prologue's window (kernels.hip)
      int lo = 0, hi = (int)m;
      while (hi - lo > 1) {
        const int md = (lo + hi) >> 1;
        if (knots[md] <= c[i + 1]) lo = md;
        else hi = md;
      }
      const double L = knots[m];
      const double adv = llampc::window_adv(c[i + 2], c[i + 3], c[i + 4], H, vmax);
      double need = 1e300;
      if (adv < L && c[i + 1] >= 0.0 && c[i + 1] < L) {
        double te = c[i + 1] + adv;
        if (te >= L) te -= L;
        int l2 = 0, h2 = (int)m;
        while (h2 - l2 > 1) {
          const int md = (l2 + h2) >> 1;
          if (knots[md] <= te) l2 = md;
          else h2 = md;
        }
        need = (double)(l2 >= lo ? l2 - lo : l2 + (int)m - lo) + 2.0;
      }
      if (need <= (double)m) {
        const int W = (int)need;
        wbuf.assign((size_t)M * 4 * W, 0.0);
        for (size_t e = 0; e < wbuf.size(); ++e) {
          const int row = (int)(e / W), j = (int)(e % W);
          int sg = lo + j;
          if (sg >= (int)m) sg -= (int)m;
          wbuf[e] = speed[(size_t)row * m + sg];
        }
        sw = llampc::SpeedWin{wbuf.data(), lo, W};
      }
    }
    llampc::RaceRef rr;
    rr.init(r, knots.data(), mus.data(), c[i], c[i + 1], c[i + 2], c[i + 3], c[i + 4]);
    for (int k = 0; k < H; ++k) {
      double xr, yr;
      rr.step(r, knots.data(), xy.data(), sw, xr, yr);
      std::printf("%.17g %.17g\n", xr, yr);
    }
  }
  return 0;
}
