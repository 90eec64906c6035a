// Host-side plan construction: every read-only table the HIP kernels consume.
// Built once per engine on the host (double-precision libm, then rounded to
// f32 exactly as the reference's initialisers do) and uploaded to HBM.
//
//  * rnnoise tables (denoise.c check_init, [upstream, recalled]): analysis /
//    synthesis half window, 22x22 DCT, tansig_table;
//  * celt kiss_fft plan for the 960-point FFT A (factors 5,3,4,4,4): twiddles
//    (float)cos/sin((-2*pi/960)*i) and the digit-reversal table;
//  * kissfft plan for FFT B (FFT.zig:179-191 -> kiss_fftr_alloc): substate
//    twiddles (float)cos/sin(-2*pi*i/ncfft), super twiddles, and the kf_work
//    leaf permutation;
//  * hannWindowPeriodic (window_fn.zig:22-28,51-68) and FFT.zig's
//    normalisation factor (FFT.zig:94,162-166).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fvad_internal.h"

namespace fvad {
namespace {

const int kEband5ms[kBands] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 34, 40, 48, 60, 78, 100};

// celt kf_factor for 960 -> reversed stage list {5,192, 3,64, 4,16, 4,4, 4,1}.
void celt_digit_reverse(int fout, int *f, int fstride, const int *factors) {
  const int p = factors[0], m = factors[1];
  if (m == 1) {
    for (int j = 0; j < p; j++) {
      *f = fout + j;
      f += fstride;
    }
  } else {
    for (int j = 0; j < p; j++) {
      celt_digit_reverse(fout, f, fstride * p, factors + 2);
      f += fstride;
      fout += m;
    }
  }
}

// kissfft kf_work leaf placement: Fout[k] = fin[perm[k]].
// kf_factor (kissfft): powers of 4 first, then 2, then odd primes; one (p, m)
// pair per stage with m = the remaining length
void kiss_factor(int n, int *fac, int *nf) {
  int p = 4, k = 0;
  const double floor_sqrt = std::floor(std::sqrt((double)n));
  do {
    while (n % p) {
      switch (p) {
        case 4: p = 2; break;
        case 2: p = 3; break;
        default: p += 2; break;
      }
      if (p > floor_sqrt) p = n;
    }
    n /= p;
    fac[2 * k] = p;
    fac[2 * k + 1] = n;
    k++;
  } while (n > 1);
  *nf = k;
}

void kiss_leaf_perm(int *perm, int out_base, int in_base, int fstride, const int *factors) {
  const int p = factors[0], m = factors[1];
  if (m == 1) {
    for (int j = 0; j < p; j++) perm[out_base + j] = in_base + j * fstride;
  } else {
    for (int j = 0; j < p; j++) kiss_leaf_perm(perm, out_base + j * m, in_base + j * fstride, fstride * p, factors + 2);
  }
}

}  // namespace

void build_plan(Plan *p, int nfft_b) {
  std::memset(p, 0, sizeof(Plan));
  const double pi = 3.14159265358979323846;
  for (int i = 0; i < kFrame; i++) {
    const double s = std::sin(.5 * pi * (i + .5) / kFrame);
    p->half_window[i] = (float)std::sin(.5 * pi * s * s);
  }
  for (int i = 0; i < kBands; i++)
    for (int j = 0; j < kBands; j++) {
      float v = (float)std::cos((i + .5) * j * pi / kBands);
      if (j == 0) v = (float)(v * std::sqrt(.5));
      p->dct[i * kBands + j] = v;
    }
  for (int i = 0; i < 201; i++) {  // tansig_table literals: "%f" of tanh(0.04 i), parsed as float
    char buf[64];
    std::snprintf(buf, sizeof buf, "%f", std::tanh(0.04 * i));
    p->tansig[i] = std::strtof(buf, nullptr);
  }
  for (int b = 0; b < kBands; b++) p->eband4[b] = kEband5ms[b] << 2;
  for (int b = 0; b < kBands - 1; b++) {
    const int size = (kEband5ms[b + 1] - kEband5ms[b]) << 2;
    for (int j = 0; j < size; j++) {
      p->band_of[(kEband5ms[b] << 2) + j] = b;
      p->band_frac[(kEband5ms[b] << 2) + j] = (float)j / size;
    }
  }
  // celt FFT 960
  for (int i = 0; i < kWin; i++) {
    const double cpi = 3.14159265358979323846264338327;
    const double phase = (-2 * cpi / kWin) * i;
    p->tw960[2 * i] = (float)std::cos(phase);
    p->tw960[2 * i + 1] = (float)std::sin(phase);
  }
  const int celt_factors[10] = {5, 192, 3, 64, 4, 16, 4, 4, 4, 1};
  celt_digit_reverse(0, p->bitrev960, 1, celt_factors);
  for (int i = 0; i < kWin; i++) p->ibitrev960[p->bitrev960[i]] = i;
  // kissfft real FFT B
  p->nfft_b = nfft_b;
  p->ncfft_b = nfft_b / 2;
  const int nc = p->ncfft_b;
  kiss_factor(nc, p->fac_b, &p->nfac_b);
  int st = 0;
  for (int i = 0; i < p->nfac_b; i++) {
    st = (p->fac_b[2 * i] == 4 && st == i) ? st + 1 : st;
    if (p->fac_b[2 * i] > 5) p->generic_b = 1;
  }
  p->stages_b = st == p->nfac_b ? st : 0;
  if (nfft_b <= kMaxFftB) p->norm_b = build_fftb_tables(nfft_b, p->fac_b, p->twb, p->superb, p->permb, p->hannb);
}

float build_fftb_tables(int nfft_b, const int *fac, float *twb, float *superb, int *permb, float *hannb) {
  const double pi = 3.14159265358979323846;
  const int nc = nfft_b / 2;
  for (int i = 0; i < nc; i++) {
    const double kpi = 3.141592653589793238462643383279502884197169399375105820974944;
    const double phase = -2 * kpi * i / nc;
    twb[2 * i] = (float)std::cos(phase);
    twb[2 * i + 1] = (float)std::sin(phase);
  }
  for (int i = 0; i < nc / 2; i++) {
    const double phase = -3.14159265358979323846264338327 * ((double)(i + 1) / nc + .5);
    superb[2 * i] = (float)std::cos(phase);
    superb[2 * i + 1] = (float)std::sin(phase);
  }
  kiss_leaf_perm(permb, 0, 0, 1, fac);
  // hannWindowPeriodic in f32 (2*pi coerced to f32, (2*pi*k*n)/N in f32, f32 cos)
  const float N = (float)nfft_b;
  const float two_pi = (float)(2.0 * pi);
  for (int i = 0; i < nfft_b; i++) {
    const float nn = (float)i;
    float acc = 0;
    for (int k = 0; k <= 1; k++) {
      const float kk = (float)k;
      const float sgn = k == 0 ? 1.0f : -1.0f;
      const float arg = ((two_pi * kk) * nn) / N;
      acc += (sgn * 0.5f) * (float)std::cos((double)arg);
    }
    hannb[i] = acc;
  }
  float sum = 0;
  for (int i = 0; i < nfft_b; i++) sum += hannb[i];
  const float window_norm = (float)nfft_b / sum;
  return window_norm / (float)(nfft_b / 2);
}

}  // namespace fvad
