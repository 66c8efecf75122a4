// Host harness for csrc/ctl.hpp (test infrastructure): runs the controller tick's pure
// functions — Philox4x32-10, the candidate sampler with its clip / rate chains, the
// reference projection and NumPy's pairwise mean — on the CPU and prints the results, so
// tests/test_ctl_native.py compares them bitwise with the NumPy restatement.  Built with
// AddressSanitizer (host code only).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ctl.hpp"

using namespace llampc;

static std::vector<double> read_all(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    std::perror(path);
    std::exit(2);
  }
  std::vector<double> v;
  double x;
  while (std::fread(&x, sizeof x, 1, f) == 1) v.push_back(x);
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::vector<double> in = read_all(argv[2]);
  if (!std::strcmp(argv[1], "philox")) {
    // in: per case c0 c1 c2 c3 k0 k1 (as doubles); out: four words
    for (size_t i = 0; i + 6 <= in.size(); i += 6) {
      const Philox4 r = philox4x32_10(Philox4{(uint32_t)in[i], (uint32_t)in[i + 1], (uint32_t)in[i + 2], (uint32_t)in[i + 3]},
                                      (uint32_t)in[i + 4], (uint32_t)in[i + 5]);
      std::printf("%u %u %u %u\n", r.x, r.y, r.z, r.w);
    }
  } else if (!std::strcmp(argv[1], "cands")) {
    // in: C H has_prev tick seed up0 up1 ns0 ns1 lo0 lo1 hi0 hi1 r0 r1 prev[H][2]
    const int C = (int)in[0], H = (int)in[1], has_prev = (int)in[2];
    const uint64_t tick = (uint64_t)in[3], seed = (uint64_t)in[4];
    const double up[2] = {in[5], in[6]}, ns[2] = {in[7], in[8]}, lo[2] = {in[9], in[10]}, hi[2] = {in[11], in[12]},
                 r[2] = {in[13], in[14]};
    const double* prev = has_prev ? in.data() + 15 : nullptr;
    std::vector<double> U((size_t)C * H * 2);
    for (int c = 0; c < C; ++c)
      for (int k = 0; k < H; ++k) ctl_cand_pair(c, k, H, prev, up, ns, lo, hi, tick, seed, 0, &U[((size_t)c * H + k) * 2]);
    for (int c = 0; c < C; ++c)
      for (int j = 0; j < 2; ++j) ctl_rate_chain(U.data() + (size_t)c * H * 2 + j, H, up[j], r[j]);
    for (double v : U) std::printf("%.17g\n", v);
  } else if (!std::strcmp(argv[1], "project")) {
    // in: np, points [2][np], then per case px py p0; out: the argmin index and the distances
    const int np_ = (int)in[0];
    const double* pts = in.data() + 1;
    for (size_t i = 1 + 2 * (size_t)np_; i + 3 <= in.size(); i += 3) {
      const double px = in[i], py = in[i + 1];
      const int p0 = (int)in[i + 2];
      const int segs = ctl_segments(p0, np_);
      double d[kCtlSegs];
      for (int s = 0; s < segs; ++s)
        d[s] = ref_project_dist(px, py, pts[p0 + s], pts[np_ + p0 + s], pts[p0 + s + 1], pts[np_ + p0 + s + 1]);
      std::printf("%d", np_argmin(d, segs));
      for (int s = 0; s < segs; ++s) std::printf(" %.17g", d[s]);
      std::printf("\n");
    }
  } else if (!std::strcmp(argv[1], "mean")) {
    // in: per case n cap first v[cap]; out: the pairwise sum / n
    size_t i = 0;
    while (i + 3 <= in.size()) {
      const int n = (int)in[i], cap = (int)in[i + 1], first = (int)in[i + 2];
      std::printf("%.17g\n", np_pairwise_ring(in.data() + i + 3, first, n, cap) / n);
      i += 3 + cap;
    }
  } else {
    return 2;
  }
  return 0;
}
