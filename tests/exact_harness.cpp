// tests/test_host_cpu.py::test_add_const_n_exact: fvad_exact.h add_const_n against the plain loop
// (acc = fl(acc + c), n times) over random and edge cases, bit for bit.
#include <cmath>
#include "fvad_exact.h"
#include <cstdio>
#include <random>
#include <cstring>
int main() {
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(0, 1);
  long bad = 0, tot = 0;
  for (int it = 0; it < 200000; it++) {
    double acc, c; unsigned n;
    int kind = it % 6;
    double e1 = std::pow(2.0, (int)(U(g) * 40) - 30), e2 = std::pow(2.0, (int)(U(g) * 40) - 40);
    acc = (kind == 0) ? 0.0 : (kind == 1 ? -U(g) * e1 : U(g) * e1);
    c = (kind == 2) ? 0.005 / 4218 : U(g) * e2;
    if (kind == 3) c = std::ldexp(std::floor(U(g) * 1e6) + 0.5, -20) ; // ties likely
    if (kind == 4) { acc = std::ldexp(1.0, -8) - std::ldexp(3.0, -60); }
    n = (unsigned)(U(g) * 5000);
    double ref = acc;
    for (unsigned i = 0; i < n; i++) ref = ref + c;
    double got = fvad::add_const_n(acc, c, n);
    tot++;
    if (std::memcmp(&ref, &got, 8)) { if (bad < 5) printf("MISMATCH acc=%a c=%a n=%u ref=%a got=%a\n", acc, c, n, ref, got); bad++; }
  }
  printf("%ld / %ld mismatches\n", bad, tot);
  return bad != 0;
}
