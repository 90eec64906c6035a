/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar C restatement of the classic rnnoise per-frame algorithm as called by
 * /root/reference/src/Denoiser.zig:60 (rnnoise_process_frame) and
 * Denoiser.zig:23,36,69 (create / destroy / get_frame_size).  The rnnoise
 * sources are NOT in /root/reference (lib/rnnoise is an empty submodule,
 * .gitmodules:4-6, built from denoise.c celt_lpc.c kiss_fft.c pitch.c rnn.c
 * rnn_data.c rnn_reader.c per build.zig:182-191), so every function below
 * restates the published algorithm [upstream, recalled] — SURVEY.md Appendix A.
 * Float-mode opus macro semantics are used literally (MULT16_16 = a*b,
 * MAC16_16 = c + a*b, HALF32 = .5f*x, QCONST16(x,b) = x, celt_sqrt = (float)sqrt).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define FRAME_SIZE 480
#define WINDOW_SIZE 960
#define FREQ_SIZE 481
#define NB_BANDS 22
#define CEPS_MEM 8
#define NB_DELTA_CEPS 6
#define NB_FEATURES 42
#define PITCH_MIN_PERIOD 60
#define PITCH_MAX_PERIOD 768
#define PITCH_FRAME_SIZE 960
#define PITCH_BUF_SIZE (PITCH_MAX_PERIOD + PITCH_FRAME_SIZE)
#define MAX_NEURONS 128
#define WEIGHTS_SCALE (1.f / 256)

static const short eband5ms[NB_BANDS] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  10, 12,
                                         14, 16, 20, 24, 28, 34, 40, 48, 60, 78, 100};

typedef struct { float r, i; } cpx;

/* ------------------------------------------------------------------ */
/* celt / opus kiss_fft (float), forward only, nfft = 960             */
/* ------------------------------------------------------------------ */
typedef struct {
  int nfft;
  float scale;
  short factors[16];
  short bitrev[WINDOW_SIZE];
  cpx twiddles[WINDOW_SIZE];
} celt_fft_state;

static int celt_kf_factor(int n, short *facbuf) {
  int p = 4, i, stages = 0, nbak = n;
  do {
    while (n % p) {
      switch (p) {
        case 4: p = 2; break;
        case 2: p = 3; break;
        default: p += 2; break;
      }
      if (p > 32000 || p * p > n) p = n;
    }
    n /= p;
    if (p > 5) return 0;
    facbuf[2 * stages] = (short)p;
    if (p == 2 && stages > 1) {
      facbuf[2 * stages] = 4;
      facbuf[2] = 2;
    }
    stages++;
  } while (n > 1);
  n = nbak;
  for (i = 0; i < stages / 2; i++) {
    short tmp = facbuf[2 * i];
    facbuf[2 * i] = facbuf[2 * (stages - i - 1)];
    facbuf[2 * (stages - i - 1)] = tmp;
  }
  for (i = 0; i < stages; i++) {
    n /= facbuf[2 * i];
    facbuf[2 * i + 1] = (short)n;
  }
  return 1;
}

static void celt_bitrev(int Fout, short *f, size_t fstride, int in_stride, const short *factors) {
  const int p = *factors++;
  const int m = *factors++;
  int j;
  if (m == 1) {
    for (j = 0; j < p; j++) {
      *f = (short)(Fout + j);
      f += fstride * in_stride;
    }
  } else {
    for (j = 0; j < p; j++) {
      celt_bitrev(Fout, f, fstride * p, in_stride, factors);
      f += fstride * in_stride;
      Fout += m;
    }
  }
}

static void celt_fft_init(celt_fft_state *st, int nfft) {
  int i;
  st->nfft = nfft;
  st->scale = 1.f / nfft;
  for (i = 0; i < nfft; i++) {
    const double pi = 3.14159265358979323846264338327;
    double phase = (-2 * pi / nfft) * i;
    st->twiddles[i].r = (float)cos(phase);
    st->twiddles[i].i = (float)sin(phase);
  }
  celt_kf_factor(nfft, st->factors);
  celt_bitrev(0, st->bitrev, 1, 1, st->factors);
}

#define C_MUL(m, a, b)                  \
  do {                                  \
    (m).r = (a).r * (b).r - (a).i * (b).i; \
    (m).i = (a).r * (b).i + (a).i * (b).r; \
  } while (0)
#define C_ADD(res, a, b)     \
  do {                       \
    (res).r = (a).r + (b).r; \
    (res).i = (a).i + (b).i; \
  } while (0)
#define C_SUB(res, a, b)     \
  do {                       \
    (res).r = (a).r - (b).r; \
    (res).i = (a).i - (b).i; \
  } while (0)
#define C_ADDTO(res, a) \
  do {                  \
    (res).r += (a).r;   \
    (res).i += (a).i;   \
  } while (0)

static void celt_bfly4(cpx *Fout, size_t fstride, const celt_fft_state *st, int m, int N, int mm) {
  int i;
  if (m == 1) {
    for (i = 0; i < N; i++) {
      cpx s0, s1;
      C_SUB(s0, *Fout, Fout[2]);
      C_ADDTO(*Fout, Fout[2]);
      C_ADD(s1, Fout[1], Fout[3]);
      C_SUB(Fout[2], *Fout, s1);
      C_ADDTO(*Fout, s1);
      C_SUB(s1, Fout[1], Fout[3]);
      Fout[1].r = s0.r + s1.i;
      Fout[1].i = s0.i - s1.r;
      Fout[3].r = s0.r - s1.i;
      Fout[3].i = s0.i + s1.r;
      Fout += 4;
    }
  } else {
    int j;
    cpx s[6];
    const cpx *tw1, *tw2, *tw3;
    const int m2 = 2 * m, m3 = 3 * m;
    cpx *Fout_beg = Fout;
    for (i = 0; i < N; i++) {
      Fout = Fout_beg + i * mm;
      tw3 = tw2 = tw1 = st->twiddles;
      for (j = 0; j < m; j++) {
        C_MUL(s[0], Fout[m], *tw1);
        C_MUL(s[1], Fout[m2], *tw2);
        C_MUL(s[2], Fout[m3], *tw3);
        C_SUB(s[5], *Fout, s[1]);
        C_ADDTO(*Fout, s[1]);
        C_ADD(s[3], s[0], s[2]);
        C_SUB(s[4], s[0], s[2]);
        C_SUB(Fout[m2], *Fout, s[3]);
        tw1 += fstride;
        tw2 += fstride * 2;
        tw3 += fstride * 3;
        C_ADDTO(*Fout, s[3]);
        Fout[m].r = s[5].r + s[4].i;
        Fout[m].i = s[5].i - s[4].r;
        Fout[m3].r = s[5].r - s[4].i;
        Fout[m3].i = s[5].i + s[4].r;
        ++Fout;
      }
    }
  }
}

static void celt_bfly3(cpx *Fout, size_t fstride, const celt_fft_state *st, int m, int N, int mm) {
  int i;
  size_t k;
  const size_t m2 = 2 * m;
  const cpx *tw1, *tw2;
  cpx s[5];
  cpx epi3 = st->twiddles[fstride * m];
  cpx *Fout_beg = Fout;
  for (i = 0; i < N; i++) {
    Fout = Fout_beg + i * mm;
    tw1 = tw2 = st->twiddles;
    k = m;
    do {
      C_MUL(s[1], Fout[m], *tw1);
      C_MUL(s[2], Fout[m2], *tw2);
      C_ADD(s[3], s[1], s[2]);
      C_SUB(s[0], s[1], s[2]);
      tw1 += fstride;
      tw2 += fstride * 2;
      Fout[m].r = Fout->r - s[3].r * .5f;
      Fout[m].i = Fout->i - s[3].i * .5f;
      s[0].r *= epi3.i;
      s[0].i *= epi3.i;
      C_ADDTO(*Fout, s[3]);
      Fout[m2].r = Fout[m].r + s[0].i;
      Fout[m2].i = Fout[m].i - s[0].r;
      Fout[m].r = Fout[m].r - s[0].i;
      Fout[m].i = Fout[m].i + s[0].r;
      ++Fout;
    } while (--k);
  }
}

static void celt_bfly5(cpx *Fout, size_t fstride, const celt_fft_state *st, int m, int N, int mm) {
  cpx *F0, *F1, *F2, *F3, *F4;
  int i, u;
  cpx s[13];
  const cpx *tw = st->twiddles;
  cpx ya = st->twiddles[fstride * m];
  cpx yb = st->twiddles[fstride * 2 * m];
  cpx *Fout_beg = Fout;
  for (i = 0; i < N; i++) {
    Fout = Fout_beg + i * mm;
    F0 = Fout;
    F1 = F0 + m;
    F2 = F0 + 2 * m;
    F3 = F0 + 3 * m;
    F4 = F0 + 4 * m;
    for (u = 0; u < m; ++u) {
      s[0] = *F0;
      C_MUL(s[1], *F1, tw[u * fstride]);
      C_MUL(s[2], *F2, tw[2 * u * fstride]);
      C_MUL(s[3], *F3, tw[3 * u * fstride]);
      C_MUL(s[4], *F4, tw[4 * u * fstride]);
      C_ADD(s[7], s[1], s[4]);
      C_SUB(s[10], s[1], s[4]);
      C_ADD(s[8], s[2], s[3]);
      C_SUB(s[9], s[2], s[3]);
      /* Opus 1.2-era (2017) expression forms: left-associative sums */
      F0->r += s[7].r + s[8].r;
      F0->i += s[7].i + s[8].i;
      s[5].r = s[0].r + s[7].r * ya.r + s[8].r * yb.r;
      s[5].i = s[0].i + s[7].i * ya.r + s[8].i * yb.r;
      s[6].r = s[10].i * ya.i + s[9].i * yb.i;
      s[6].i = -(s[10].r * ya.i) - s[9].r * yb.i;
      C_SUB(*F1, s[5], s[6]);
      C_ADD(*F4, s[5], s[6]);
      s[11].r = s[0].r + s[7].r * yb.r + s[8].r * ya.r;
      s[11].i = s[0].i + s[7].i * yb.r + s[8].i * ya.r;
      s[12].r = -(s[10].i * yb.i) + s[9].i * ya.i;
      s[12].i = s[10].r * yb.i - s[9].r * ya.i;
      C_ADD(*F2, s[11], s[12]);
      C_SUB(*F3, s[11], s[12]);
      ++F0;
      ++F1;
      ++F2;
      ++F3;
      ++F4;
    }
  }
}

static void celt_fft(const celt_fft_state *st, const cpx *fin, cpx *fout) {
  int i, L = 0, m, m2, p;
  int fstride[8];
  for (i = 0; i < st->nfft; i++) {
    cpx x = fin[i];
    fout[st->bitrev[i]].r = st->scale * x.r;
    fout[st->bitrev[i]].i = st->scale * x.i;
  }
  fstride[0] = 1;
  do {
    p = st->factors[2 * L];
    m = st->factors[2 * L + 1];
    fstride[L + 1] = fstride[L] * p;
    L++;
  } while (m != 1);
  m = st->factors[2 * L - 1];
  for (i = L - 1; i >= 0; i--) {
    m2 = (i != 0) ? st->factors[2 * i - 1] : 1;
    switch (st->factors[2 * i]) {
      case 4: celt_bfly4(fout, fstride[i], st, m, fstride[i], m2); break;
      case 3: celt_bfly3(fout, fstride[i], st, m, fstride[i], m2); break;
      case 5: celt_bfly5(fout, fstride[i], st, m, fstride[i], m2); break;
      default: abort(); /* radix 2 never occurs for 960 */
    }
    m = m2;
  }
}

/* ------------------------------------------------------------------ */
/* common tables (denoise.c check_init)                               */
/* ------------------------------------------------------------------ */
static struct {
  int init;
  celt_fft_state fft;
  float half_window[FRAME_SIZE];
  float dct_table[NB_BANDS * NB_BANDS];
} common;

static const double ORA_PI = 3.14159265358979323846;

static void check_init(void) {
  int i, j;
  if (common.init) return;
  celt_fft_init(&common.fft, WINDOW_SIZE);
  for (i = 0; i < FRAME_SIZE; i++) {
    double s = sin(.5 * ORA_PI * (i + .5) / FRAME_SIZE);
    common.half_window[i] = (float)sin(.5 * ORA_PI * s * s);
  }
  for (i = 0; i < NB_BANDS; i++) {
    for (j = 0; j < NB_BANDS; j++) {
      common.dct_table[i * NB_BANDS + j] = (float)cos((i + .5) * j * ORA_PI / NB_BANDS);
      if (j == 0) common.dct_table[i * NB_BANDS + j] = (float)(common.dct_table[i * NB_BANDS + j] * sqrt(.5));
    }
  }
  common.init = 1;
}

/* tansig table: tanh(0.04 i) printed with 6 decimals (rnnoise tansig_table.h) */
static float tansig_table[201];
static int tansig_init = 0;
static void init_tansig(void) {
  int i;
  if (tansig_init) return;
  for (i = 0; i < 201; i++) {
    /* the upstream table holds tanh(.04 i) printed "%f"; a float literal parses
       to the nearest float of that decimal string */
    char buf[64];
    snprintf(buf, sizeof buf, "%f", tanh(0.04 * i));
    tansig_table[i] = strtof(buf, NULL);
  }
  tansig_init = 1;
}

void ora_tables(float *hw, float *dct, float *tt) {
  check_init();
  init_tansig();
  if (hw) memcpy(hw, common.half_window, sizeof(common.half_window));
  if (dct) memcpy(dct, common.dct_table, sizeof(common.dct_table));
  if (tt) memcpy(tt, tansig_table, sizeof(tansig_table));
}

void ora_fft960(const float *in_ri, float *out_ri) {
  cpx x[WINDOW_SIZE], y[WINDOW_SIZE];
  int i;
  check_init();
  for (i = 0; i < WINDOW_SIZE; i++) {
    x[i].r = in_ri[2 * i];
    x[i].i = in_ri[2 * i + 1];
  }
  celt_fft(&common.fft, x, y);
  for (i = 0; i < WINDOW_SIZE; i++) {
    out_ri[2 * i] = y[i].r;
    out_ri[2 * i + 1] = y[i].i;
  }
}

/* ------------------------------------------------------------------ */
/* band energy / correlation / interpolation (denoise.c)              */
/* ------------------------------------------------------------------ */
static void compute_band_energy(float *bandE, const cpx *X) {
  int i;
  float sum[NB_BANDS] = {0};
  for (i = 0; i < NB_BANDS - 1; i++) {
    int j, band_size = (eband5ms[i + 1] - eband5ms[i]) << 2;
    for (j = 0; j < band_size; j++) {
      float tmp, frac = (float)j / band_size;
      int b = (eband5ms[i] << 2) + j;
      tmp = X[b].r * X[b].r;
      tmp += X[b].i * X[b].i;
      sum[i] += (1 - frac) * tmp;
      sum[i + 1] += frac * tmp;
    }
  }
  sum[0] *= 2;
  sum[NB_BANDS - 1] *= 2;
  for (i = 0; i < NB_BANDS; i++) bandE[i] = sum[i];
}

static void compute_band_corr(float *bandE, const cpx *X, const cpx *P) {
  int i;
  float sum[NB_BANDS] = {0};
  for (i = 0; i < NB_BANDS - 1; i++) {
    int j, band_size = (eband5ms[i + 1] - eband5ms[i]) << 2;
    for (j = 0; j < band_size; j++) {
      float tmp, frac = (float)j / band_size;
      int b = (eband5ms[i] << 2) + j;
      tmp = X[b].r * P[b].r;
      tmp += X[b].i * P[b].i;
      sum[i] += (1 - frac) * tmp;
      sum[i + 1] += frac * tmp;
    }
  }
  sum[0] *= 2;
  sum[NB_BANDS - 1] *= 2;
  for (i = 0; i < NB_BANDS; i++) bandE[i] = sum[i];
}

/* NB: upstream memsets FREQ_SIZE *bytes*; callers pass zero-initialised arrays,
 * so bins >= 400 stay at their initial values (0, or gf[0]=1 untouched). */
static void interp_band_gain(float *g, const float *bandE) {
  int i;
  memset(g, 0, FREQ_SIZE);
  for (i = 0; i < NB_BANDS - 1; i++) {
    int j, band_size = (eband5ms[i + 1] - eband5ms[i]) << 2;
    for (j = 0; j < band_size; j++) {
      float frac = (float)j / band_size;
      g[(eband5ms[i] << 2) + j] = (1 - frac) * bandE[i] + frac * bandE[i + 1];
    }
  }
}

static void dct(float *out, const float *in) {
  int i;
  check_init();
  for (i = 0; i < NB_BANDS; i++) {
    int j;
    float sum = 0;
    for (j = 0; j < NB_BANDS; j++) sum += in[j] * common.dct_table[j * NB_BANDS + i];
    out[i] = (float)(sum * sqrt(2. / 22));
  }
}

static void forward_transform(cpx *out, const float *in) {
  int i;
  cpx x[WINDOW_SIZE], y[WINDOW_SIZE];
  check_init();
  for (i = 0; i < WINDOW_SIZE; i++) {
    x[i].r = in[i];
    x[i].i = 0;
  }
  celt_fft(&common.fft, x, y);
  for (i = 0; i < FREQ_SIZE; i++) out[i] = y[i];
}

static void inverse_transform(float *out, const cpx *in) {
  int i;
  cpx x[WINDOW_SIZE], y[WINDOW_SIZE];
  check_init();
  for (i = 0; i < FREQ_SIZE; i++) x[i] = in[i];
  for (; i < WINDOW_SIZE; i++) {
    x[i].r = x[WINDOW_SIZE - i].r;
    x[i].i = -x[WINDOW_SIZE - i].i;
  }
  celt_fft(&common.fft, x, y);
  out[0] = WINDOW_SIZE * y[0].r;
  for (i = 1; i < WINDOW_SIZE; i++) out[i] = WINDOW_SIZE * y[WINDOW_SIZE - i].r;
}

static void apply_window(float *x) {
  int i;
  check_init();
  for (i = 0; i < FRAME_SIZE; i++) {
    x[i] *= common.half_window[i];
    x[WINDOW_SIZE - 1 - i] *= common.half_window[i];
  }
}

/* ------------------------------------------------------------------ */
/* pitch.c / celt_lpc.c (float)                                        */
/* ------------------------------------------------------------------ */
static float inner_prod(const float *x, const float *y, int N) {
  int i;
  float xy = 0;
  for (i = 0; i < N; i++) xy = xy + x[i] * y[i];
  return xy;
}

static void dual_inner_prod(const float *x, const float *y01, const float *y02, int N, float *xy1,
                            float *xy2) {
  int i;
  float a = 0, b = 0;
  for (i = 0; i < N; i++) {
    a = a + x[i] * y01[i];
    b = b + x[i] * y02[i];
  }
  *xy1 = a;
  *xy2 = b;
}

/* celt_pitch_xcorr: xcorr[k] = sequential sum_j x[j]*y[j+k] (xcorr_kernel order) */
static void pitch_xcorr(const float *x, const float *y, float *xcorr, int len, int max_pitch) {
  int k;
  for (k = 0; k < max_pitch; k++) xcorr[k] = inner_prod(x, y + k, len);
}

static void celt_autocorr(const float *x, float *ac, int lag, int n) {
  int i, k;
  int fastN = n - lag;
  float d;
  pitch_xcorr(x, x, ac, fastN, lag + 1);
  for (k = 0; k <= lag; k++) {
    for (i = k + fastN, d = 0; i < n; i++) d = d + x[i] * x[i - k];
    ac[k] += d;
  }
}

static void celt_lpc(float *lpc, const float *ac, int p) {
  int i, j;
  float r;
  float error = ac[0];
  memset(lpc, 0, sizeof(float) * p);
  if (ac[0] != 0) {
    for (i = 0; i < p; i++) {
      float rr = 0;
      for (j = 0; j < i; j++) rr += lpc[j] * ac[i - j];
      rr += ac[i + 1];
      r = -rr / error;
      lpc[i] = r;
      for (j = 0; j < (i + 1) >> 1; j++) {
        float tmp1 = lpc[j], tmp2 = lpc[i - 1 - j];
        lpc[j] = tmp1 + r * tmp2;
        lpc[i - 1 - j] = tmp2 + r * tmp1;
      }
      error = error - (r * r) * error;
      if (error < .001f * ac[0]) break;
    }
  }
}

static void celt_fir5(const float *x, const float *num, float *y, int N) {
  int i;
  float num0 = num[0], num1 = num[1], num2 = num[2], num3 = num[3], num4 = num[4];
  float mem0 = 0, mem1 = 0, mem2 = 0, mem3 = 0, mem4 = 0;
  for (i = 0; i < N; i++) {
    float sum = x[i];
    sum = sum + num0 * mem0;
    sum = sum + num1 * mem1;
    sum = sum + num2 * mem2;
    sum = sum + num3 * mem3;
    sum = sum + num4 * mem4;
    mem4 = mem3;
    mem3 = mem2;
    mem2 = mem1;
    mem1 = mem0;
    mem0 = x[i];
    y[i] = sum;
  }
}

static void pitch_downsample(const float *x, float *x_lp, int len) {
  int i;
  float ac[5];
  float tmp = 1.0f;
  float lpc[4], lpc2[5];
  float c1 = .8f;
  for (i = 1; i < len >> 1; i++) x_lp[i] = .5f * (.5f * (x[2 * i - 1] + x[2 * i + 1]) + x[2 * i]);
  x_lp[0] = .5f * (.5f * (x[1]) + x[0]);
  celt_autocorr(x_lp, ac, 4, len >> 1);
  ac[0] *= 1.0001f;
  for (i = 1; i <= 4; i++) ac[i] -= ac[i] * (.008f * i) * (.008f * i);
  celt_lpc(lpc, ac, 4);
  for (i = 0; i < 4; i++) {
    tmp = .9f * tmp;
    lpc[i] = lpc[i] * tmp;
  }
  lpc2[0] = lpc[0] + .8f;
  lpc2[1] = lpc[1] + c1 * lpc[0];
  lpc2[2] = lpc[2] + c1 * lpc[1];
  lpc2[3] = lpc[3] + c1 * lpc[2];
  lpc2[4] = c1 * lpc[3];
  celt_fir5(x_lp, lpc2, x_lp, len >> 1);
}

static void find_best_pitch(const float *xcorr, const float *y, int len, int max_pitch,
                            int *best_pitch) {
  int i, j;
  float Syy = 1;
  float best_num[2] = {-1, -1};
  float best_den[2] = {0, 0};
  best_pitch[0] = 0;
  best_pitch[1] = 1;
  for (j = 0; j < len; j++) Syy = Syy + y[j] * y[j];
  for (i = 0; i < max_pitch; i++) {
    if (xcorr[i] > 0) {
      float num, xcorr16 = xcorr[i];
      xcorr16 *= 1e-12f;
      num = xcorr16 * xcorr16;
      if (num * best_den[1] > best_num[1] * Syy) {
        if (num * best_den[0] > best_num[0] * Syy) {
          best_num[1] = best_num[0];
          best_den[1] = best_den[0];
          best_pitch[1] = best_pitch[0];
          best_num[0] = num;
          best_den[0] = Syy;
          best_pitch[0] = i;
        } else {
          best_num[1] = num;
          best_den[1] = Syy;
          best_pitch[1] = i;
        }
      }
    }
    Syy += y[i + len] * y[i + len] - y[i] * y[i];
    Syy = (1 > Syy) ? 1 : Syy;
  }
}

static void pitch_search(const float *x_lp, const float *y, int len, int max_pitch, int *pitch, int *n_fine) {
  int i, j, lag, offset;
  int best_pitch[2] = {0, 0};
  float x_lp4[PITCH_FRAME_SIZE >> 2];
  float y_lp4[(PITCH_FRAME_SIZE + PITCH_MAX_PERIOD) >> 2];
  float xcorr[PITCH_MAX_PERIOD >> 1];
  lag = len + max_pitch;
  for (j = 0; j < len >> 2; j++) x_lp4[j] = x_lp[2 * j];
  for (j = 0; j < lag >> 2; j++) y_lp4[j] = y[2 * j];
  pitch_xcorr(x_lp4, y_lp4, xcorr, len >> 2, max_pitch >> 2);
  find_best_pitch(xcorr, y_lp4, len >> 2, max_pitch >> 2, best_pitch);
  for (i = 0; i < max_pitch >> 1; i++) {
    float sum;
    xcorr[i] = 0;
    if (abs(i - 2 * best_pitch[0]) > 2 && abs(i - 2 * best_pitch[1]) > 2) continue;
    sum = inner_prod(x_lp, y + i, len >> 1);
    (*n_fine)++;
    xcorr[i] = (-1 > sum) ? -1 : sum;
  }
  find_best_pitch(xcorr, y, len >> 1, max_pitch >> 1, best_pitch);
  if (best_pitch[0] > 0 && best_pitch[0] < (max_pitch >> 1) - 1) {
    float a = xcorr[best_pitch[0] - 1], b = xcorr[best_pitch[0]], c = xcorr[best_pitch[0] + 1];
    if ((c - a) > .7f * (b - a))
      offset = 1;
    else if ((a - c) > .7f * (b - c))
      offset = -1;
    else
      offset = 0;
  } else {
    offset = 0;
  }
  *pitch = 2 * best_pitch[0] - offset;
}

static float compute_pitch_gain(float xy, float xx, float yy) {
  return xy / (float)sqrt(1 + xx * yy);
}

static const int second_check[16] = {0, 0, 3, 2, 3, 2, 5, 2, 3, 2, 3, 2, 5, 2, 3, 2};

static float remove_doubling(const float *x, int maxperiod, int minperiod, int N, int *T0_,
                             int prev_period, float prev_gain, int *n_cand) {
  int k, i, T, T0, offset, minperiod0 = minperiod;
  float g, g0, pg, xy, xx, yy, xy2, best_xy, best_yy;
  float xcorr[3];
  float yy_lookup[(PITCH_MAX_PERIOD >> 1) + 1];
  maxperiod /= 2;
  minperiod /= 2;
  *T0_ /= 2;
  prev_period /= 2;
  N /= 2;
  x += maxperiod;
  if (*T0_ >= maxperiod) *T0_ = maxperiod - 1;
  T = T0 = *T0_;
  dual_inner_prod(x, x, x - T0, N, &xx, &xy);
  yy_lookup[0] = xx;
  yy = xx;
  for (i = 1; i <= maxperiod; i++) {
    yy = yy + x[-i] * x[-i] - x[N - i] * x[N - i];
    yy_lookup[i] = (0 > yy) ? 0 : yy;
  }
  yy = yy_lookup[T0];
  best_xy = xy;
  best_yy = yy;
  g = g0 = compute_pitch_gain(xy, xx, yy);
  for (k = 2; k <= 15; k++) {
    int T1, T1b;
    float g1, cont = 0, thresh;
    T1 = (int)((unsigned)(2 * T0 + k) / (unsigned)(2 * k));
    if (T1 < minperiod) break;
    (*n_cand)++;
    if (k == 2) {
      if (T1 + T0 > maxperiod)
        T1b = T0;
      else
        T1b = T0 + T1;
    } else {
      T1b = (int)((unsigned)(2 * second_check[k] * T0 + k) / (unsigned)(2 * k));
    }
    dual_inner_prod(x, &x[-T1], &x[-T1b], N, &xy, &xy2);
    xy = .5f * (xy + xy2);
    yy = .5f * (yy_lookup[T1] + yy_lookup[T1b]);
    g1 = compute_pitch_gain(xy, xx, yy);
    if (abs(T1 - prev_period) <= 1)
      cont = prev_gain;
    else if (abs(T1 - prev_period) <= 2 && 5 * k * k < T0)
      cont = .5f * prev_gain;
    else
      cont = 0;
    {
      float a = .7f * g0 - cont;
      thresh = (.3f > a) ? .3f : a;
    }
    if (T1 < 3 * minperiod) {
      float a = .85f * g0 - cont;
      thresh = (.4f > a) ? .4f : a;
    } else if (T1 < 2 * minperiod) {
      float a = .9f * g0 - cont;
      thresh = (.5f > a) ? .5f : a;
    }
    if (g1 > thresh) {
      best_xy = xy;
      best_yy = yy;
      T = T1;
      g = g1;
    }
  }
  best_xy = (0 > best_xy) ? 0 : best_xy;
  if (best_yy <= best_xy)
    pg = 1.0f;
  else
    pg = best_xy / (best_yy + 1);
  for (k = 0; k < 3; k++) xcorr[k] = inner_prod(x, x - (T + k - 1), N);
  if ((xcorr[2] - xcorr[0]) > .7f * (xcorr[1] - xcorr[0]))
    offset = 1;
  else if ((xcorr[0] - xcorr[2]) > .7f * (xcorr[1] - xcorr[2]))
    offset = -1;
  else
    offset = 0;
  if (pg > g) pg = g;
  *T0_ = 2 * T + offset;
  if (*T0_ < minperiod0) *T0_ = minperiod0;
  return pg;
}

/* ------------------------------------------------------------------ */
/* rnn.c                                                               */
/* ------------------------------------------------------------------ */
static float tansig_approx(float x) {
  int i;
  float y, dy, sign = 1;
  if (!(x < 8)) return 1;
  if (!(x > -8)) return -1;
  if (x != x) return 0;
  if (x < 0) {
    x = -x;
    sign = -1;
  }
  i = (int)floor(.5f + 25 * x);
  x -= .04f * i;
  y = tansig_table[i];
  dy = 1 - y * y;
  y = y + x * dy * (1 - y * x);
  return sign * y;
}

static float sigmoid_approx(float x) { return (float)(.5 + .5 * tansig_approx((float)(.5 * x))); }

static float relu(float x) { return x < 0 ? 0 : x; }

static float activate(int act, float x) {
  if (act == ORA_ACT_SIGMOID) return sigmoid_approx(x);
  if (act == ORA_ACT_TANH) return tansig_approx(x);
  return relu(x);
}

static void compute_dense(const ora_dense *layer, float *output, const float *input) {
  int i, j;
  const int M = layer->nb_inputs, N = layer->nb_neurons, stride = N;
  for (i = 0; i < N; i++) {
    float sum = layer->bias[i];
    for (j = 0; j < M; j++) sum += layer->input_weights[j * stride + i] * input[j];
    output[i] = WEIGHTS_SCALE * sum;
  }
  for (i = 0; i < N; i++) output[i] = activate(layer->activation, output[i]);
}

static void compute_gru(const ora_gru *gru, float *state, const float *input) {
  int i, j;
  const int M = gru->nb_inputs, N = gru->nb_neurons, stride = 3 * N;
  float z[MAX_NEURONS], r[MAX_NEURONS], h[MAX_NEURONS];
  for (i = 0; i < N; i++) {
    float sum = gru->bias[i];
    for (j = 0; j < M; j++) sum += gru->input_weights[j * stride + i] * input[j];
    for (j = 0; j < N; j++) sum += gru->recurrent_weights[j * stride + i] * state[j];
    z[i] = sigmoid_approx(WEIGHTS_SCALE * sum);
  }
  for (i = 0; i < N; i++) {
    float sum = gru->bias[N + i];
    for (j = 0; j < M; j++) sum += gru->input_weights[N + j * stride + i] * input[j];
    for (j = 0; j < N; j++) sum += gru->recurrent_weights[N + j * stride + i] * state[j];
    r[i] = sigmoid_approx(WEIGHTS_SCALE * sum);
  }
  for (i = 0; i < N; i++) {
    float sum = gru->bias[2 * N + i];
    for (j = 0; j < M; j++) sum += gru->input_weights[2 * N + j * stride + i] * input[j];
    for (j = 0; j < N; j++) sum += gru->recurrent_weights[2 * N + j * stride + i] * state[j] * r[j];
    sum = activate(gru->activation, WEIGHTS_SCALE * sum);
    h[i] = z[i] * state[i] + (1 - z[i]) * sum;
  }
  for (i = 0; i < N; i++) state[i] = h[i];
}

/* ------------------------------------------------------------------ */
/* denoise.c                                                            */
/* ------------------------------------------------------------------ */
struct ora_denoise {
  float analysis_mem[FRAME_SIZE];
  float cepstral_mem[CEPS_MEM][NB_BANDS];
  int memid;
  float synthesis_mem[FRAME_SIZE];
  float pitch_buf[PITCH_BUF_SIZE];
  float last_gain;
  int last_period;
  float mem_hp_x[2];
  float lastg[NB_BANDS];
  float vad_gru_state[MAX_NEURONS];
  float noise_gru_state[MAX_NEURONS];
  float denoise_gru_state[MAX_NEURONS];
  const ora_model *model;
  int bypass;
  /* debug */
  int dbg_pitch, dbg_silence;
  float dbg_gain, dbg_features[NB_FEATURES];
  /* work counters (instrumented op count, ora_rnnoise_counts) */
  uint64_t n_frames, n_silent, n_fine_lags, n_rd_cands;
};

ora_denoise *ora_rnnoise_create(const ora_model *m) {
  ora_denoise *st = (ora_denoise *)calloc(1, sizeof(ora_denoise));
  check_init();
  init_tansig();
  st->model = m;
  return st;
}
void ora_rnnoise_destroy(ora_denoise *st) { free(st); }
int ora_rnnoise_get_frame_size(void) { return FRAME_SIZE; }
void ora_rnnoise_set_bypass(ora_denoise *st, int bypass) { st->bypass = bypass; }
void ora_rnnoise_counts(const ora_denoise *st, uint64_t *counts) {
  counts[0] += st->n_frames;
  counts[1] += st->n_silent;
  counts[2] += st->n_fine_lags;
  counts[3] += st->n_rd_cands;
}
void ora_rnnoise_debug(const ora_denoise *st, int *pitch, float *gain, int *silence, float *f) {
  if (pitch) *pitch = st->dbg_pitch;
  if (gain) *gain = st->dbg_gain;
  if (silence) *silence = st->dbg_silence;
  if (f) memcpy(f, st->dbg_features, sizeof(st->dbg_features));
}

static void frame_analysis(ora_denoise *st, cpx *X, float *Ex, const float *in) {
  int i;
  float x[WINDOW_SIZE];
  memcpy(x, st->analysis_mem, FRAME_SIZE * sizeof(float));
  for (i = 0; i < FRAME_SIZE; i++) x[FRAME_SIZE + i] = in[i];
  memcpy(st->analysis_mem, in, FRAME_SIZE * sizeof(float));
  apply_window(x);
  forward_transform(X, x);
  compute_band_energy(Ex, X);
}

static int compute_frame_features(ora_denoise *st, cpx *X, cpx *P, float *Ex, float *Ep, float *Exp,
                                  float *features, const float *in) {
  int i;
  float E = 0;
  float *ceps_0, *ceps_1, *ceps_2;
  float spec_variability = 0;
  float Ly[NB_BANDS];
  float p[WINDOW_SIZE];
  float pitch_buf[PITCH_BUF_SIZE >> 1];
  int pitch_index;
  float gain;
  float tmp[NB_BANDS];
  float follow, logMax;
  frame_analysis(st, X, Ex, in);
  memmove(st->pitch_buf, &st->pitch_buf[FRAME_SIZE], (PITCH_BUF_SIZE - FRAME_SIZE) * sizeof(float));
  memcpy(&st->pitch_buf[PITCH_BUF_SIZE - FRAME_SIZE], in, FRAME_SIZE * sizeof(float));
  pitch_downsample(st->pitch_buf, pitch_buf, PITCH_BUF_SIZE);
  {
    int n_fine = 0;
    pitch_search(pitch_buf + (PITCH_MAX_PERIOD >> 1), pitch_buf, PITCH_FRAME_SIZE,
                 PITCH_MAX_PERIOD - 3 * PITCH_MIN_PERIOD, &pitch_index, &n_fine);
    st->n_fine_lags += (uint64_t)n_fine;
  }
  pitch_index = PITCH_MAX_PERIOD - pitch_index;
  {
    int n_cand = 0;
    gain = remove_doubling(pitch_buf, PITCH_MAX_PERIOD, PITCH_MIN_PERIOD, PITCH_FRAME_SIZE,
                           &pitch_index, st->last_period, st->last_gain, &n_cand);
    st->n_rd_cands += (uint64_t)n_cand;
  }
  st->last_period = pitch_index;
  st->last_gain = gain;
  st->dbg_pitch = pitch_index;
  st->dbg_gain = gain;
  for (i = 0; i < WINDOW_SIZE; i++) p[i] = st->pitch_buf[PITCH_BUF_SIZE - WINDOW_SIZE - pitch_index + i];
  apply_window(p);
  forward_transform(P, p);
  compute_band_energy(Ep, P);
  compute_band_corr(Exp, X, P);
  for (i = 0; i < NB_BANDS; i++) Exp[i] = (float)(Exp[i] / sqrt(.001 + Ex[i] * Ep[i]));
  dct(tmp, Exp);
  for (i = 0; i < NB_DELTA_CEPS; i++) features[NB_BANDS + 2 * NB_DELTA_CEPS + i] = tmp[i];
  features[NB_BANDS + 2 * NB_DELTA_CEPS] = (float)(features[NB_BANDS + 2 * NB_DELTA_CEPS] - 1.3);
  features[NB_BANDS + 2 * NB_DELTA_CEPS + 1] = (float)(features[NB_BANDS + 2 * NB_DELTA_CEPS + 1] - 0.9);
  features[NB_BANDS + 3 * NB_DELTA_CEPS] = (float)(.01 * (pitch_index - 300));
  logMax = -2;
  follow = -2;
  for (i = 0; i < NB_BANDS; i++) {
    double a, b;
    Ly[i] = (float)log10(1e-2 + Ex[i]);
    /* MAX16(logMax-7, MAX16(follow-1.5, Ly[i])) with double promotion of follow-1.5 */
    b = (follow - 1.5 > (double)Ly[i]) ? follow - 1.5 : (double)Ly[i];
    a = ((double)(logMax - 7) > b) ? (double)(logMax - 7) : b;
    Ly[i] = (float)a;
    logMax = (logMax > Ly[i]) ? logMax : Ly[i];
    follow = (float)((follow - 1.5 > (double)Ly[i]) ? follow - 1.5 : (double)Ly[i]);
    E += Ex[i];
  }
  if (E < 0.04) {
    memset(features, 0, NB_FEATURES * sizeof(float));
    return 1;
  }
  dct(features, Ly);
  features[0] -= 12;
  features[1] -= 4;
  ceps_0 = st->cepstral_mem[st->memid];
  ceps_1 = (st->memid < 1) ? st->cepstral_mem[CEPS_MEM + st->memid - 1] : st->cepstral_mem[st->memid - 1];
  ceps_2 = (st->memid < 2) ? st->cepstral_mem[CEPS_MEM + st->memid - 2] : st->cepstral_mem[st->memid - 2];
  for (i = 0; i < NB_BANDS; i++) ceps_0[i] = features[i];
  st->memid++;
  for (i = 0; i < NB_DELTA_CEPS; i++) {
    features[i] = ceps_0[i] + ceps_1[i] + ceps_2[i];
    features[NB_BANDS + i] = ceps_0[i] - ceps_2[i];
    features[NB_BANDS + NB_DELTA_CEPS + i] = ceps_0[i] - 2 * ceps_1[i] + ceps_2[i];
  }
  if (st->memid == CEPS_MEM) st->memid = 0;
  for (i = 0; i < CEPS_MEM; i++) {
    int j;
    float mindist = 1e15f;
    for (j = 0; j < CEPS_MEM; j++) {
      int k;
      float dist = 0;
      for (k = 0; k < NB_BANDS; k++) {
        float t = st->cepstral_mem[i][k] - st->cepstral_mem[j][k];
        dist += t * t;
      }
      if (j != i) mindist = (mindist < dist) ? mindist : dist;
    }
    spec_variability += mindist;
  }
  features[NB_BANDS + 3 * NB_DELTA_CEPS + 1] = (float)(spec_variability / CEPS_MEM - 2.1);
  return 0;
}

static void frame_synthesis(ora_denoise *st, float *out, const cpx *y) {
  float x[WINDOW_SIZE];
  int i;
  inverse_transform(x, y);
  apply_window(x);
  for (i = 0; i < FRAME_SIZE; i++) out[i] = x[i] + st->synthesis_mem[i];
  memcpy(st->synthesis_mem, &x[FRAME_SIZE], FRAME_SIZE * sizeof(float));
}

static void biquad(float *y, float mem[2], const float *x, const float *b, const float *a, int N) {
  int i;
  for (i = 0; i < N; i++) {
    float xi = x[i], yi;
    yi = x[i] + mem[0];
    mem[0] = (float)(mem[1] + (b[0] * (double)xi - a[0] * (double)yi));
    mem[1] = (float)(b[1] * (double)xi - a[1] * (double)yi);
    y[i] = yi;
  }
}

static void pitch_filter(cpx *X, const cpx *P, const float *Ex, const float *Ep, const float *Exp,
                         const float *g) {
  int i;
  float r[NB_BANDS];
  float rf[FREQ_SIZE] = {0};
  float newE[NB_BANDS], norm[NB_BANDS];
  float normf[FREQ_SIZE] = {0};
  for (i = 0; i < NB_BANDS; i++) {
    if (Exp[i] > g[i])
      r[i] = 1;
    else
      r[i] = (float)((Exp[i] * Exp[i]) * (1 - (g[i] * g[i])) / (.001 + (g[i] * g[i]) * (1 - (Exp[i] * Exp[i]))));
    {
      float c = (0 > r[i]) ? 0 : r[i];
      c = (1 < c) ? 1 : c;
      r[i] = (float)sqrt(c);
    }
    r[i] = (float)(r[i] * sqrt(Ex[i] / (1e-8 + Ep[i])));
  }
  interp_band_gain(rf, r);
  for (i = 0; i < FREQ_SIZE; i++) {
    X[i].r += rf[i] * P[i].r;
    X[i].i += rf[i] * P[i].i;
  }
  compute_band_energy(newE, X);
  for (i = 0; i < NB_BANDS; i++) norm[i] = (float)sqrt(Ex[i] / (1e-8 + newE[i]));
  interp_band_gain(normf, norm);
  for (i = 0; i < FREQ_SIZE; i++) {
    X[i].r *= normf[i];
    X[i].i *= normf[i];
  }
}

static void compute_rnn(ora_denoise *st, float *gains, float *vad, const float *input) {
  const ora_model *m = st->model;
  int i;
  float dense_out[MAX_NEURONS];
  float noise_input[MAX_NEURONS * 3];
  float denoise_input[MAX_NEURONS * 3];
  const int nd = m->input_dense.nb_neurons, nv = m->vad_gru.nb_neurons, nn = m->noise_gru.nb_neurons;
  compute_dense(&m->input_dense, dense_out, input);
  compute_gru(&m->vad_gru, st->vad_gru_state, dense_out);
  compute_dense(&m->vad_output, vad, st->vad_gru_state);
  for (i = 0; i < nd; i++) noise_input[i] = dense_out[i];
  for (i = 0; i < nv; i++) noise_input[i + nd] = st->vad_gru_state[i];
  for (i = 0; i < NB_FEATURES; i++) noise_input[i + nd + nv] = input[i];
  compute_gru(&m->noise_gru, st->noise_gru_state, noise_input);
  for (i = 0; i < nv; i++) denoise_input[i] = st->vad_gru_state[i];
  for (i = 0; i < nn; i++) denoise_input[i + nv] = st->noise_gru_state[i];
  for (i = 0; i < NB_FEATURES; i++) denoise_input[i + nv + nn] = input[i];
  compute_gru(&m->denoise_gru, st->denoise_gru_state, denoise_input);
  compute_dense(&m->denoise_output, gains, st->denoise_gru_state);
}

float ora_rnnoise_process_frame(ora_denoise *st, float *out, const float *in) {
  int i;
  cpx X[FREQ_SIZE];
  cpx P[WINDOW_SIZE];
  float x[FRAME_SIZE];
  float Ex[NB_BANDS], Ep[NB_BANDS], Exp[NB_BANDS];
  float features[NB_FEATURES];
  float g[NB_BANDS];
  float gf[FREQ_SIZE] = {1};
  float vad_prob = 0;
  int silence;
  static const float a_hp[2] = {-1.99599f, 0.99600f};
  static const float b_hp[2] = {-2, 1};
  biquad(x, st->mem_hp_x, in, b_hp, a_hp, FRAME_SIZE);
  silence = compute_frame_features(st, X, P, Ex, Ep, Exp, features, x);
  st->dbg_silence = silence;
  st->n_frames++;
  st->n_silent += (uint64_t)silence;
  memcpy(st->dbg_features, features, sizeof(features));
  if (st->bypass) {
    /* weight-free KAT hook: unit gains, no pitch filter */
    frame_synthesis(st, out, X);
    return 0;
  }
  if (!silence) {
    compute_rnn(st, g, &vad_prob, features);
    pitch_filter(X, P, Ex, Ep, Exp, g);
    for (i = 0; i < NB_BANDS; i++) {
      float alpha = .6f;
      g[i] = (g[i] > alpha * st->lastg[i]) ? g[i] : alpha * st->lastg[i];
      st->lastg[i] = g[i];
    }
    interp_band_gain(gf, g);
    for (i = 0; i < FREQ_SIZE; i++) {
      X[i].r *= gf[i];
      X[i].i *= gf[i];
    }
  }
  frame_synthesis(st, out, X);
  return vad_prob;
}
