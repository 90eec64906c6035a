// tests/test_host_cpu.py::test_lazy_longterm_bound: the device VADMachine's
// lazy long-term test (fvad_staged.hip vadm_stream, through fvad_exact.h's
// lt_bound / lt_decide / lt_estimate -- the same header the kernel includes)
// against the reference's exact decision, st_avg > RN(avg * f) with avg the
// RollingAverage fold (RollingAverage.zig:45-56: avg += data[i] * scalar in
// array order; VADMachine.zig:150-167).
//
// A long-term buffer of n entries (full, optionally from an initial average)
// takes long pushes from adversarial value streams (log-uniform over 70
// binades, huge/tiny alternation, rare spikes over zeros, powers of two +-
// an ulp, constants); the walk keeps the estimate exactly as the kernel does
// (an open test folds and restarts it, an owed run folds at a random defer
// limit up to kLtDeferMax = 4096).  At each test point st_avg is placed at the
// exact threshold RN(fold * f) and +-1, +-2 ulps of it, at both edges of the
// bound's window +-1, +-2 ulps, and at random points around it.  Every
// decision the bound settles must equal the exact one; |approx - fold| must
// stay within E.  Prints the counts; exit status 1 on any mismatch.
//
//   lt_bound_harness [n_decisions] [scale]   scale: E times this (a scale
//   well below 1 must produce mismatches -- the harness's own sensitivity check)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "fvad_exact.h"

namespace {
std::mt19937_64 rng(0x5EEDF1AD);
double U() { return std::uniform_real_distribution<double>(0, 1)(rng); }
int I(int n) { return (int)(U() * n); }

// one pushed band value (an f32, >= 0) of value stream `kind`
float value(int kind, long step) {
  switch (kind) {
    case 0: return (float)(U() * 1e-2);
    case 1: return (float)std::ldexp(U(), I(70) - 60);
    case 2: return (step & 1) ? (float)std::ldexp(1.0 + U(), 8) : (float)std::ldexp(U(), -40);
    case 3: return U() < 0.01 ? (float)(U() * 1e4) : 0.0f;
    case 4: {
      const float p = std::ldexp(1.0f, I(40) - 30);
      const int d = I(5) - 2;
      return d < 0 ? std::nextafter(p, 0.0f) : (d > 0 ? std::nextafter(p, 1e30f) : p);
    }
    case 5: return 0.1f;
    default: return (float)(U() < 0.5 ? 999.0 : U() * 1e-6);  // a window's min is at most 999
  }
}
}  // namespace

int main(int argc, char **argv) {
  const long want = argc > 1 ? atol(argv[1]) : 1000000;
  const double scale = argc > 2 ? atof(argv[2]) : 1.0;
  const unsigned ns[] = {2, 3, 17, 64, 421, 4218, 4218, 4218};
  const float fs[] = {18.0f, 18.0f, 0.5f, 1.0f, 1000.0f, 3.0f};
  long decisions = 0, settled = 0, open = 0, bad = 0, tests = 0, folds = 0, pushes = 0;
  double worst = 0.0;  // max |approx - fold| / E
  for (int run = 0; decisions < want; run++) {
    const unsigned n = ns[run % 8];
    const float f32 = (run % 7 == 6) ? (float)(U() * 50) : fs[run % 6];
    const double f = (double)f32, scalar = 1.0 / (double)n;
    const int kind = run % 7;
    const bool has_init = run % 3 == 0;
    const unsigned defer_max = 1 + (unsigned)I(4096);
    std::vector<double> data(n);
    for (unsigned i = 0; i < n; i++) data[i] = has_init ? 0.005 : (double)value(kind, i);
    unsigned widx = has_init ? 0 : 0;
    auto fold = [&]() {  // RollingAverage.avg of the full buffer
      double acc = 0.0;
      for (unsigned i = 0; i < n; i++) acc += data[i] * scalar;
      return acc;
    };
    double lt_last = fold(), approx = lt_last, amax = std::fabs(lt_last);
    unsigned pending = 0;
    auto refold = [&]() {
      lt_last = fold();
      approx = lt_last;
      amax = std::fabs(lt_last);
      pending = 0;
      folds++;
    };
    const long steps = 2000 + I(20000);
    for (long step = 0; step < steps && decisions < want; step++) {
      // a long push (the window did not meet the speech condition)
      const float v = value(kind, step);
      const double t_old = data[widx] * scalar;
      data[widx] = (double)v;
      widx = (widx + 1) % n;
      fvad::lt_estimate(approx, amax, (double)v * scalar, t_old);
      pending++;
      pushes++;
      if (pending >= defer_max) refold();  // the owed fold at the defer limit
      if (pending == 0 || U() > 0.05) continue;
      // a test point: the reference's decision at each candidate st_avg
      tests++;
      const double F = fold(), thr = F * f;
      const double E = fvad::lt_bound(n, pending, amax, scale);
      if (E > 0) worst = std::fmax(worst, std::fabs(approx - F) / (E / scale));
      const double lo = (approx - 2.0 * E) * f, hi = (approx + 2.0 * E) * f;
      double cand[24];
      int k = 0;
      for (double c : {thr, lo, hi}) {
        double up = c, dn = c;
        cand[k++] = c;
        for (int d = 0; d < 2; d++) {
          up = std::nextafter(up, INFINITY);
          dn = std::nextafter(dn, -INFINITY);
          cand[k++] = up;
          cand[k++] = dn;
        }
      }
      for (int r = 0; r < 9; r++) cand[k++] = lo + (hi - lo) * (U() * 3 - 1);
      bool opened = false;
      for (int c = 0; c < k; c++) {
        const bool ref = cand[c] > thr;
        const int d = fvad::lt_decide(cand[c], approx, E, f);
        decisions++;
        if (d < 0) {
          open++;
          opened = true;  // the kernel folds here (its decision is then exact)
          continue;
        }
        settled++;
        if ((d == 1) != ref) {
          if (bad < 5)
            printf("MISMATCH n=%u f=%a pending=%u st_avg=%a fold=%a approx=%a E=%a d=%d\n", n, f, pending, cand[c],
                   F, approx, E, d);
          bad++;
        }
      }
      if (opened && U() < 0.5) refold();  // an open test's fold restarts the estimate
    }
  }
  printf("decisions %ld settled %ld open %ld mismatches %ld | tests %ld pushes %ld folds %ld | max |approx-fold|/E %.3e\n",
         decisions, settled, open, bad, tests, pushes, folds, worst);
  return bad != 0;
}
