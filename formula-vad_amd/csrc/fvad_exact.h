// Exact shortcuts for serial floating-point chains whose every step is known
// in advance (host and device).  Each returns the bits the plain C loop gives.
#pragma once
#include <cstdint>

#if defined(__HIP__)
#define FVAD_HD __host__ __device__
#else
#define FVAD_HD  // plain C++ (the CPU test harness, tests/test_host_cpu.py)
#endif

namespace fvad {

// acc = fl(acc + c), n times, in IEEE double round-to-nearest-even: the
// RollingAverage recompute over entries that still hold the initial average
// (RollingAverage.zig:45-56: `avg += data[i] * scalar`, every term the same
// double), done per binade instead of per step.  With acc > 0 in
// [2^e, 2^(e+1)) and u = ulp(acc) = 2^(e-52), write acc = M u (2^52 <= M <
// 2^53) and c = (q + f) u, q integer, 0 <= f < 1 (exact: a power-of-two
// scaling).  While the exact sum stays below 2^(e+1) every step rounds to M +
// q + [f > 1/2] -- the same integer d each time unless f = 1/2 (a tie, whose
// outcome depends on M's parity) -- so k steps add k d exactly.  The step that
// leaves the binade runs as a plain add and the next binade starts over.
// Anything outside that case (acc or c not a positive normal number, c not
// small against acc, a tie) takes plain adds, so the result is the loop's
// bits in every case.
FVAD_HD inline double add_const_n(double acc, double c, unsigned n) {
  constexpr double kTwo52 = 4503599627370496.0;  // 2^52
  constexpr double kTiny = 2.2250738585072014e-308 * kTwo52;  // acc / 2^52 stays normal above this
  while (n > 0) {
    if (!(acc >= kTiny && acc < 1e300 && c > 0 && c < 1e300)) {
      acc = acc + c;
      n--;
      continue;
    }
    // u = ulp(acc): the power of two of acc's exponent, times 2^-52
    // and its inverse 2^(52-e) (both powers of two in range: scaling by them is exact)
    const uint64_t eb = __builtin_bit_cast(uint64_t, acc) & 0x7ff0000000000000ull;
    const uint64_t ub = eb - (52ull << 52), ib = (2046ull << 52) - ub;
    const double u = __builtin_bit_cast(double, ub), iu = __builtin_bit_cast(double, ib);
    const double r = c * iu;  // c / u, exact (inf on overflow: the plain-add branch)
    if (r >= kTwo52) {  // c at least half of acc: the binade changes within a step or two
      acc = acc + c;
      n--;
      continue;
    }
    const double qf = __builtin_floor(r), f = r - qf;  // both exact
    if (f == 0.5) {  // a tie: rounds to even, the parity of M alternates
      acc = acc + c;
      n--;
      continue;
    }
    const uint64_t d = (uint64_t)qf + (f > 0.5 ? 1u : 0u);
    if (d == 0) return acc;  // c < u / 2: every remaining step rounds back to acc
    const uint64_t M = (uint64_t)(acc * iu);  // exact integer, 2^52 <= M < 2^53
    const uint64_t room = ((1ull << 53) - 1 - M) / d;  // steps that keep M + k d in the binade
    const uint64_t k = room < n ? room : n;
    acc = (double)(M + k * d) * u;  // exact: < 2^53 units of u
    n -= (unsigned)k;
    if (n > 0) {  // the step that leaves the binade
      acc = acc + c;
      n--;
    }
  }
  return acc;
}

// The lazy long-term test of the device VADMachine (fvad_staged.hip
// vadm_stream).  VADMachine.zig:150-167 tests st_avg > RN(lt_avg * f), lt_avg
// the long-term RollingAverage's fold of its n terms t_i = RN(e_i / n)
// (RollingAverage.zig:45-56, C order).  Between exact folds the walk carries
// an estimate `approx` of that fold, updated per long push as
// RN(RN(approx + t_new) - t_old) (lt_estimate), and the largest |approx| seen
// since the last exact fold (amax).  With every entry >= 0:
//  * a fold of n nonnegative terms is within (n - 1) u of their exact sum
//    (u = 2^-53), and that sum is <= the fold (1 + (n - 1) u) <= ~amax;
//  * the estimate starts at an exact fold, and each update adds at most
//    u |approx + t_new| + u |result| <= 2u (2 amax) to its distance from the
//    exact sum of the current terms;
// so |approx - fold| <= (n - 1) u (S_then + S_now) + 4 u pending amax, and
// lt_bound's E = (2n + 4 pending + 64) u amax * 2 covers it twice over (the
// +64 and the factor 2 absorb the higher-order terms).  `scale` is the test
// hook FVAD_DEBUG_VADM_BOUND_SCALE (1 in production; +inf: no test settled).
FVAD_HD inline double lt_bound(unsigned n, unsigned pending, double amax, double scale) {
  return (2.0 * n + 4.0 * pending + 64.0) * 0x1p-53 * amax * 2.0 * scale;
}
// The test from the estimate: 1 if st_avg > RN(fold * f) for every fold within
// E of approx, 0 if for none, -1 if the bound leaves it open (the caller then
// folds exactly).  f >= 0: RN is monotone, and RN(approx +- 2E) lies beyond
// approx +- E, so hi >= RN(fold * f) >= lo.
FVAD_HD inline int lt_decide(double st_avg, double approx, double E, double f) {
  const double lo = (approx - 2.0 * E) * f, hi = (approx + 2.0 * E) * f;
  if (st_avg > hi) return 1;
  if (st_avg <= lo) return 0;
  return -1;
}
// One long push into the estimate: t_new = RN(pushed * 1/n) replaces t_old
// (the overwritten entry's term).
FVAD_HD inline void lt_estimate(double &approx, double &amax, double t_new, double t_old) {
  approx = (approx + t_new) - t_old;
  amax = __builtin_fmax(amax, __builtin_fabs(approx));
}

}  // namespace fvad
