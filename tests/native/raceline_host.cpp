// Host harness for csrc/raceline.hpp (test infrastructure): runs the device ConstantSpeed
// walker on the CPU over tables and starts written by tests/test_raceline_native.py and
// prints the per-model references, so the Python test compares them with the oracle —
// built with AddressSanitizer (host code only) to catch any out-of-bounds table access.
#include <cstdio>
#include <cstdlib>
#include <vector>
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
  if (argc != 3) return 2;
  const std::vector<double> t = read_all(argv[1]), c = read_all(argv[2]);
  const int n = (int)t[0], M = (int)t[1];
  const size_t m = n - 1;
  std::vector<double> knots(t.begin() + 2, t.begin() + 2 + n);
  std::vector<double> xy(t.begin() + 2 + n, t.begin() + 2 + n + 8 * m);
  std::vector<double> speed(t.begin() + 2 + n + 8 * m, t.begin() + 2 + n + 8 * m + 4 * m * M);
  std::vector<double> mus(t.begin() + 2 + n + 8 * m + 4 * m * M, t.end());
  llampc::RacelineK r{knots.data(), xy.data(), speed.data(), mus.data(), n, M};
  const int H = (int)c[0];
  for (size_t i = 1; i + 5 <= c.size(); i += 5) {
    llampc::RaceRef rr;
    rr.init(r, knots.data(), c[i], c[i + 1], c[i + 2], c[i + 3], c[i + 4]);
    for (int k = 0; k < H; ++k) {
      double xr, yr;
      rr.step(r, knots.data(), xy.data(), xr, yr);
      std::printf("%.17g %.17g\n", xr, yr);
    }
  }
  return 0;
}
