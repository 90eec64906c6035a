/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of mborgerding/kissfft (complex kf_work recursion + kiss_fftr
 * real-input post-processing, kiss_fft_scalar=float per build.zig:145-147) as
 * used by /root/reference/src/FFT.zig:70-98,179-208 (FFT B).  The kissfft
 * submodule is EMPTY in /root/reference (.gitmodules:1-3); the only version
 * hint is commit 8f47a67f cited at FFT.zig:203.  [upstream, recalled]
 *
 * Also restates FFT.zig's wrapper semantics (window multiply FFT.zig:147-159,
 * normalisation FFT.zig:162-177), window_fn.zig and audio_utils.rmsVolume.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

typedef struct { float r, i; } kcpx;

#define MAXFACTORS 32
typedef struct {
  int nfft;
  int inverse;
  int factors[2 * MAXFACTORS];
  kcpx twiddles[1];
} kstate;

typedef struct {
  kstate *substate;
  kcpx *tmpbuf;
  kcpx *super_twiddles;
} krstate;

#define ALIGN_UP(x) (((x) + 15) & ~(size_t)15)

static void kf_factor(int n, int *facbuf) {
  int p = 4;
  double floor_sqrt = floor(sqrt((double)n));
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
    *facbuf++ = p;
    *facbuf++ = n;
  } while (n > 1);
}

static kstate *kiss_fft_alloc(int nfft, int inverse, void *mem, size_t *lenmem) {
  kstate *st = NULL;
  size_t memneeded = ALIGN_UP(sizeof(kstate) + sizeof(kcpx) * (nfft - 1));
  if (lenmem == NULL) {
    st = (kstate *)malloc(memneeded);
  } else {
    if (mem != NULL && *lenmem >= memneeded) st = (kstate *)mem;
    *lenmem = memneeded;
  }
  if (st) {
    int i;
    st->nfft = nfft;
    st->inverse = inverse;
    for (i = 0; i < nfft; ++i) {
      const double pi = 3.141592653589793238462643383279502884197169399375105820974944;
      double phase = -2 * pi * i / nfft;
      if (st->inverse) phase *= -1;
      st->twiddles[i].r = (float)cos(phase);
      st->twiddles[i].i = (float)sin(phase);
    }
    kf_factor(nfft, st->factors);
  }
  return st;
}

#define KC_MUL(m, a, b)                    \
  do {                                     \
    (m).r = (a).r * (b).r - (a).i * (b).i; \
    (m).i = (a).r * (b).i + (a).i * (b).r; \
  } while (0)
#define KC_ADD(res, a, b)    \
  do {                       \
    (res).r = (a).r + (b).r; \
    (res).i = (a).i + (b).i; \
  } while (0)
#define KC_SUB(res, a, b)    \
  do {                       \
    (res).r = (a).r - (b).r; \
    (res).i = (a).i - (b).i; \
  } while (0)
#define KC_ADDTO(res, a) \
  do {                   \
    (res).r += (a).r;    \
    (res).i += (a).i;    \
  } while (0)
#define HALF_OF(x) ((x) * ((float).5))

static void kf_bfly2(kcpx *Fout, size_t fstride, const kstate *st, int m) {
  kcpx *Fout2 = Fout + m;
  const kcpx *tw1 = st->twiddles;
  kcpx t;
  do {
    KC_MUL(t, *Fout2, *tw1);
    tw1 += fstride;
    KC_SUB(*Fout2, *Fout, t);
    KC_ADDTO(*Fout, t);
    ++Fout2;
    ++Fout;
  } while (--m);
}

static void kf_bfly4(kcpx *Fout, size_t fstride, const kstate *st, size_t m) {
  const kcpx *tw1, *tw2, *tw3;
  kcpx s[6];
  size_t k = m;
  const size_t m2 = 2 * m, m3 = 3 * m;
  tw3 = tw2 = tw1 = st->twiddles;
  do {
    KC_MUL(s[0], Fout[m], *tw1);
    KC_MUL(s[1], Fout[m2], *tw2);
    KC_MUL(s[2], Fout[m3], *tw3);
    KC_SUB(s[5], *Fout, s[1]);
    KC_ADDTO(*Fout, s[1]);
    KC_ADD(s[3], s[0], s[2]);
    KC_SUB(s[4], s[0], s[2]);
    KC_SUB(Fout[m2], *Fout, s[3]);
    tw1 += fstride;
    tw2 += fstride * 2;
    tw3 += fstride * 3;
    KC_ADDTO(*Fout, s[3]);
    if (st->inverse) {
      Fout[m].r = s[5].r - s[4].i;
      Fout[m].i = s[5].i + s[4].r;
      Fout[m3].r = s[5].r + s[4].i;
      Fout[m3].i = s[5].i - s[4].r;
    } else {
      Fout[m].r = s[5].r + s[4].i;
      Fout[m].i = s[5].i - s[4].r;
      Fout[m3].r = s[5].r - s[4].i;
      Fout[m3].i = s[5].i + s[4].r;
    }
    ++Fout;
  } while (--k);
}

static void kf_bfly3(kcpx *Fout, size_t fstride, const kstate *st, size_t m) {
  size_t k = m;
  const size_t m2 = 2 * m;
  const kcpx *tw1, *tw2;
  kcpx s[5];
  kcpx epi3 = st->twiddles[fstride * m];
  tw1 = tw2 = st->twiddles;
  do {
    KC_MUL(s[1], Fout[m], *tw1);
    KC_MUL(s[2], Fout[m2], *tw2);
    KC_ADD(s[3], s[1], s[2]);
    KC_SUB(s[0], s[1], s[2]);
    tw1 += fstride;
    tw2 += fstride * 2;
    Fout[m].r = Fout->r - HALF_OF(s[3].r);
    Fout[m].i = Fout->i - HALF_OF(s[3].i);
    s[0].r *= epi3.i;
    s[0].i *= epi3.i;
    KC_ADDTO(*Fout, s[3]);
    Fout[m2].r = Fout[m].r + s[0].i;
    Fout[m2].i = Fout[m].i - s[0].r;
    Fout[m].r -= s[0].i;
    Fout[m].i += s[0].r;
    ++Fout;
  } while (--k);
}

static void kf_bfly5(kcpx *Fout, size_t fstride, const kstate *st, int m) {
  kcpx *F0, *F1, *F2, *F3, *F4;
  int u;
  kcpx s[13];
  const kcpx *tw = st->twiddles;
  kcpx ya = st->twiddles[fstride * m], yb = st->twiddles[fstride * 2 * m];
  F0 = Fout;
  F1 = F0 + m;
  F2 = F0 + 2 * m;
  F3 = F0 + 3 * m;
  F4 = F0 + 4 * m;
  for (u = 0; u < m; ++u) {
    s[0] = *F0;
    KC_MUL(s[1], *F1, tw[u * fstride]);
    KC_MUL(s[2], *F2, tw[2 * u * fstride]);
    KC_MUL(s[3], *F3, tw[3 * u * fstride]);
    KC_MUL(s[4], *F4, tw[4 * u * fstride]);
    KC_ADD(s[7], s[1], s[4]);
    KC_SUB(s[10], s[1], s[4]);
    KC_ADD(s[8], s[2], s[3]);
    KC_SUB(s[9], s[2], s[3]);
    F0->r += s[7].r + s[8].r;
    F0->i += s[7].i + s[8].i;
    s[5].r = s[0].r + s[7].r * ya.r + s[8].r * yb.r;
    s[5].i = s[0].i + s[7].i * ya.r + s[8].i * yb.r;
    s[6].r = s[10].i * ya.i + s[9].i * yb.i;
    s[6].i = -(s[10].r * ya.i) - s[9].r * yb.i;
    KC_SUB(*F1, s[5], s[6]);
    KC_ADD(*F4, s[5], s[6]);
    s[11].r = s[0].r + s[7].r * yb.r + s[8].r * ya.r;
    s[11].i = s[0].i + s[7].i * yb.r + s[8].i * ya.r;
    s[12].r = -(s[10].i * yb.i) + s[9].i * ya.i;
    s[12].i = s[10].r * yb.i - s[9].r * ya.i;
    KC_ADD(*F2, s[11], s[12]);
    KC_SUB(*F3, s[11], s[12]);
    ++F0;
    ++F1;
    ++F2;
    ++F3;
    ++F4;
  }
}

static void kf_bfly_generic(kcpx *Fout, size_t fstride, const kstate *st, int m, int p) {
  int u, k, q1, q;
  const kcpx *twiddles = st->twiddles;
  kcpx t;
  int Norig = st->nfft;
  kcpx *scratch = (kcpx *)malloc(sizeof(kcpx) * p);
  for (u = 0; u < m; ++u) {
    k = u;
    for (q1 = 0; q1 < p; ++q1) {
      scratch[q1] = Fout[k];
      k += m;
    }
    k = u;
    for (q1 = 0; q1 < p; ++q1) {
      int twidx = 0;
      Fout[k] = scratch[0];
      for (q = 1; q < p; ++q) {
        twidx += (int)fstride * k;
        if (twidx >= Norig) twidx -= Norig;
        KC_MUL(t, scratch[q], twiddles[twidx]);
        KC_ADDTO(Fout[k], t);
      }
      k += m;
    }
  }
  free(scratch);
}

static void kf_work(kcpx *Fout, const kcpx *f, size_t fstride, int in_stride, const int *factors,
                    const kstate *st) {
  kcpx *Fout_beg = Fout;
  const int p = *factors++;
  const int m = *factors++;
  const kcpx *Fout_end = Fout + p * m;
  if (m == 1) {
    do {
      *Fout = *f;
      f += fstride * in_stride;
    } while (++Fout != Fout_end);
  } else {
    do {
      kf_work(Fout, f, fstride * p, in_stride, factors, st);
      f += fstride * in_stride;
    } while ((Fout += m) != Fout_end);
  }
  Fout = Fout_beg;
  switch (p) {
    case 2: kf_bfly2(Fout, fstride, st, m); break;
    case 3: kf_bfly3(Fout, fstride, st, m); break;
    case 4: kf_bfly4(Fout, fstride, st, m); break;
    case 5: kf_bfly5(Fout, fstride, st, m); break;
    default: kf_bfly_generic(Fout, fstride, st, m, p); break;
  }
}

static void kiss_fft(const kstate *st, const kcpx *fin, kcpx *fout) { kf_work(fout, fin, 1, 1, st->factors, st); }

void *ora_kiss_fftr_alloc(int nfft, int inverse, void *mem, size_t *lenmem) {
  int i;
  krstate *st = NULL;
  size_t subsize = 0, memneeded;
  if (nfft & 1) return NULL;
  nfft >>= 1;
  kiss_fft_alloc(nfft, inverse, NULL, &subsize);
  memneeded = sizeof(krstate) + subsize + sizeof(kcpx) * (nfft * 3 / 2);
  if (lenmem == NULL) {
    st = (krstate *)malloc(memneeded);
  } else {
    if (*lenmem >= memneeded) st = (krstate *)mem;
    *lenmem = memneeded;
  }
  if (!st) return NULL;
  st->substate = (kstate *)(st + 1);
  st->tmpbuf = (kcpx *)(((char *)st->substate) + subsize);
  st->super_twiddles = st->tmpbuf + nfft;
  kiss_fft_alloc(nfft, inverse, st->substate, &subsize);
  for (i = 0; i < nfft / 2; ++i) {
    double phase = -3.14159265358979323846264338327 * ((double)(i + 1) / nfft + .5);
    if (inverse) phase *= -1;
    st->super_twiddles[i].r = (float)cos(phase);
    st->super_twiddles[i].i = (float)sin(phase);
  }
  return st;
}

void ora_kiss_fftr(void *cfg, const float *timedata, float *freqdata_ri) {
  krstate *st = (krstate *)cfg;
  int k, ncfft = st->substate->nfft;
  kcpx fpnk, fpk, f1k, f2k, tw, tdc;
  kcpx *freqdata = (kcpx *)freqdata_ri;
  kiss_fft(st->substate, (const kcpx *)timedata, st->tmpbuf);
  tdc.r = st->tmpbuf[0].r;
  tdc.i = st->tmpbuf[0].i;
  freqdata[0].r = tdc.r + tdc.i;
  freqdata[ncfft].r = tdc.r - tdc.i;
  freqdata[ncfft].i = freqdata[0].i = 0;
  for (k = 1; k <= ncfft / 2; ++k) {
    fpk = st->tmpbuf[k];
    fpnk.r = st->tmpbuf[ncfft - k].r;
    fpnk.i = -st->tmpbuf[ncfft - k].i;
    KC_ADD(f1k, fpk, fpnk);
    KC_SUB(f2k, fpk, fpnk);
    KC_MUL(tw, f2k, st->super_twiddles[k - 1]);
    freqdata[k].r = HALF_OF(f1k.r + tw.r);
    freqdata[k].i = HALF_OF(f1k.i + tw.i);
    freqdata[ncfft - k].r = HALF_OF(f1k.r - tw.r);
    freqdata[ncfft - k].i = HALF_OF(tw.i - f1k.i);
  }
}

/* ---------------- window_fn.zig ---------------- */
/* hannWindowPeriodic -> cosineSumWindowPeriodic(K=1, {0.5, 0.5}) (window_fn.zig:22-28,51-68).
 * Zig evaluates (2*pi*k*n)/N in f32 (2*pi coerced to f32) and @cos in f32; f32 cos
 * is modelled as the correctly rounded value (float)cos((double)arg). */
void ora_hann_periodic(float *w, int n) {
  const float N = (float)n;
  const float two_pi = (float)(2.0 * 3.14159265358979323846);
  int i;
  for (i = 0; i < n; i++) {
    const float nn = (float)i;
    float acc = 0;
    int k;
    for (k = 0; k <= 1; k++) {
      const float kk = (float)k;
      const float alpha = 0.5f;
      const float sgn = (k == 0) ? 1.0f : -1.0f; /* std.math.pow(f32, -1, k) */
      const float arg = ((two_pi * kk) * nn) / N;
      const float c = (float)cos((double)arg);
      acc += (sgn * alpha) * c;
    }
    w[i] = acc;
  }
}

float ora_window_norm_factor(const float *w, int n) {
  float sum = 0;
  int i;
  for (i = 0; i < n; i++) sum += w[i];
  return (float)n / sum;
}

/* FFT.fft (FFT.zig:70-98): returns 0 ok, <0 on the Zig error conditions. */
int ora_fftzig(int nfft, const float *samples, const float *window, float *mag) {
  size_t lenmem = 1;
  void *cfg;
  float *fin, *fout;
  float window_norm, norm_factor;
  int i, bins = nfft / 2 + 1;
  if (nfft == 0 || (nfft % 2) != 0) return -1;
  ora_kiss_fftr_alloc(nfft, 0, NULL, &lenmem); /* size probe, FFT.zig:193-208 */
  cfg = malloc(lenmem);
  if (!ora_kiss_fftr_alloc(nfft, 0, cfg, &lenmem)) {
    free(cfg);
    return -2;
  }
  fin = (float *)malloc(sizeof(float) * nfft);
  fout = (float *)malloc(sizeof(float) * 2 * nfft);
  for (i = 0; i < nfft; i++) fin[i] = samples[i] * window[i];
  ora_kiss_fftr(cfg, fin, fout);
  window_norm = ora_window_norm_factor(window, nfft);
  norm_factor = window_norm / (float)(nfft / 2);
  for (i = 0; i < bins; i++) {
    const float r = fout[2 * i], im = fout[2 * i + 1];
    const float r2 = r * r, i2 = im * im; /* std.math.pow(f32, x, 2) == x*x for normal x */
    mag[i] = sqrtf(r2 + i2) * norm_factor;
  }
  free(fin);
  free(fout);
  free(cfg);
  return 0;
}

/* audio_utils.rmsVolume (audio_utils.zig:14-24) */
float ora_rms_volume(const float *x, int n) {
  float sum = 0;
  int i;
  for (i = 0; i < n; i++) sum += x[i] * x[i];
  return sqrtf(sum / (float)n);
}

/* Recorder.findBestChannel (Recorder.zig:95-110): the lowest rmsVolume, first
 * on ties (strict <, starting from 9999) */
int ora_recording_channel(const float *const *ch, int n_channels, int n) {
  int best = 0, c;
  float best_vol = 9999;
  for (c = 0; c < n_channels; c++) {
    const float vol = ora_rms_volume(ch[c], n);
    if (vol < best_vol) {
      best = c;
      best_vol = vol;
    }
  }
  return best;
}
