// Device-side building blocks shared by the fused (k_frame) and the staged
// kernels.  Every function reproduces the C evaluation order of the restated
// rnnoise / kissfft sources (see fvad_kernels.hip header on numerics).
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cmath>

#include "fvad_internal.h"

namespace fvad {

constexpr float kWs = 1.f / 256;  // WEIGHTS_SCALE (rnn.c)

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  float2 m;
  m.x = a.x * b.x - a.y * b.y;
  m.y = a.x * b.y + a.y * b.x;
  return m;
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// tansig_approx / sigmoid_approx / relu (rnn.c, [upstream, recalled])
__device__ __forceinline__ float tansig(const float *__restrict__ table, float x) {
  if (!(x < 8)) return 1;
  if (!(x > -8)) return -1;
  if (x != x) return 0;
  float sign = 1;
  if (x < 0) {
    x = -x;
    sign = -1;
  }
  const int i = (int)floorf(.5f + 25 * x);
  x -= .04f * i;
  float y = table[i];
  const float dy = 1 - y * y;
  y = y + x * dy * (1 - y * x);
  return sign * y;
}
__device__ __forceinline__ float sigmoid(const float *__restrict__ table, float x) {
  return (float)(.5 + .5 * (double)tansig(table, (float)(.5 * (double)x)));
}
__device__ __forceinline__ float activate(const float *__restrict__ table, int act, float x) {
  if (act == kActSigmoid) return sigmoid(table, x);
  if (act == kActTanh) return tansig(table, x);
  return x < 0 ? 0 : x;
}

// --- celt kiss_fft (960 = 5*3*4*4*4), forward, in place on W after the
//     digit-reversed scaled copy.  Stage order and butterfly expressions
//     follow opus_fft_impl / kf_bfly{4,3,5} (Opus 1.2-era float forms).
__device__ __forceinline__ void bfly4(float2 *F, int m, float2 tw1, float2 tw2, float2 tw3) {
  float2 a0 = F[0];
  const float2 s0 = cmul(F[m], tw1), s1 = cmul(F[2 * m], tw2), s2 = cmul(F[3 * m], tw3);
  const float2 s5 = csub(a0, s1);
  a0 = cadd(a0, s1);
  const float2 s3 = cadd(s0, s2), s4 = csub(s0, s2);
  F[2 * m] = csub(a0, s3);
  a0 = cadd(a0, s3);
  F[0] = a0;
  F[m] = make_float2(s5.x + s4.y, s5.y - s4.x);
  F[3 * m] = make_float2(s5.x - s4.y, s5.y + s4.x);
}

__device__ __forceinline__ void bfly3(float2 *F, int m, float2 tw1, float2 tw2, float2 epi3) {
  float2 a0 = F[0];
  const float2 s1 = cmul(F[m], tw1), s2 = cmul(F[2 * m], tw2);
  const float2 s3 = cadd(s1, s2);
  float2 s0 = csub(s1, s2);
  const float2 b1 = make_float2(a0.x - s3.x * .5f, a0.y - s3.y * .5f);
  s0.x *= epi3.y;
  s0.y *= epi3.y;
  a0 = cadd(a0, s3);
  F[0] = a0;
  F[2 * m] = make_float2(b1.x + s0.y, b1.y - s0.x);
  F[m] = make_float2(b1.x - s0.y, b1.y + s0.x);
}

// --- mborgerding kissfft (FFT B: kiss_fftr at FFT.zig:90), forward, any size.
// kf_work's recursion in iterative form: W holds the leaf-permuted input
// (Plan::permb / the compat cfg), then stage k = nf-1 .. 0 runs fstride_k =
// nc / (p_k m_k) groups of radix-p_k butterflies over m_k, each butterfly the
// expression of kf_bfly{2,3,4,5,generic} (oracle/ora_kissfft.c) on its own
// elements.  Generic radices (p > 5, kf_factor's remaining primes) are computed
// out of place into S (nc complex) and copied back, the order of every
// output's sum as in kf_bfly_generic.
__device__ __forceinline__ void kbfly5(float2 *F, int m, float2 t1, float2 t2, float2 t3, float2 t4, float2 ya,
                                       float2 yb) {
  const float2 s0 = F[0];
  const float2 s1 = cmul(F[m], t1), s2 = cmul(F[2 * m], t2), s3 = cmul(F[3 * m], t3), s4 = cmul(F[4 * m], t4);
  const float2 s7 = cadd(s1, s4), s10 = csub(s1, s4), s8 = cadd(s2, s3), s9 = csub(s2, s3);
  F[0] = make_float2(s0.x + (s7.x + s8.x), s0.y + (s7.y + s8.y));
  const float2 s5 = make_float2(s0.x + s7.x * ya.x + s8.x * yb.x, s0.y + s7.y * ya.x + s8.y * yb.x);
  const float2 s6 = make_float2(s10.y * ya.y + s9.y * yb.y, -(s10.x * ya.y) - s9.x * yb.y);
  F[m] = csub(s5, s6);
  F[4 * m] = cadd(s5, s6);
  const float2 s11 = make_float2(s0.x + s7.x * yb.x + s8.x * ya.x, s0.y + s7.y * yb.x + s8.y * ya.x);
  const float2 s12 = make_float2(-(s10.y * yb.y) + s9.y * ya.y, s10.x * yb.y - s9.x * ya.y);
  F[2 * m] = cadd(s11, s12);
  F[3 * m] = csub(s11, s12);
}

// one stage: (p, m), fstride = nc / (p m); threads tid, tid + nt, ... take
// butterflies (group g, u); returns after its own writes (the caller syncs)
__device__ __forceinline__ void kiss_stage(float2 *W, float2 *S, int p, int m, int nc,
                                           const float2 *__restrict__ tw, int tid, int nt) {
  if (p == 1) return;  // nc = 1 (fft_size 2): kf_bfly_generic with p = 1 copies in place
  const int fstride = nc / (p * m);
  if (p <= 5) {
    const int nb = fstride * m;
    for (int idx = tid; idx < nb; idx += nt) {
      const int g = idx / m, u = idx - g * m;
      float2 *F = W + g * p * m + u;
      if (p == 4) {
        bfly4(F, m, tw[u * fstride], tw[2 * u * fstride], tw[3 * u * fstride]);
      } else if (p == 2) {
        const float2 t = cmul(F[m], tw[u * fstride]);
        F[m] = csub(F[0], t);
        F[0] = cadd(F[0], t);
      } else if (p == 3) {
        bfly3(F, m, tw[u * fstride], tw[2 * u * fstride], tw[fstride * m]);
      } else {
        kbfly5(F, m, tw[u * fstride], tw[2 * u * fstride], tw[3 * u * fstride], tw[4 * u * fstride],
               tw[fstride * m], tw[fstride * 2 * m]);
      }
    }
    return;
  }
  // generic: output (g, u, q1) = scratch[0] + sum_q scratch[q] * tw[q * fstride * k mod nc], k = u + q1 m
  const int no = fstride * m * p;
  for (int idx = tid; idx < no; idx += nt) {
    const int g = idx / (p * m), r = idx - g * (p * m), q1 = r / m, u = r - q1 * m;
    const float2 *F = W + g * p * m + u;
    const int k = u + q1 * m;
    float2 acc = F[0];
    int twidx = 0;
    for (int q = 1; q < p; q++) {
      twidx += fstride * k;
      if (twidx >= nc) twidx -= nc;
      acc = cadd(acc, cmul(F[q * m], tw[twidx]));
    }
    S[g * p * m + k] = acc;
  }
}

// all stages of one transform; fac = kf_factor's (p, m) pairs, nf of them
__device__ __forceinline__ void kiss_stages(float2 *W, float2 *S, const int *__restrict__ fac, int nf, int nc,
                                            const float2 *__restrict__ tw, int tid, int nt) {
  for (int k = nf - 1; k >= 0; k--) {
    const int p = fac[2 * k], m = fac[2 * k + 1];
    kiss_stage(W, S, p, m, nc, tw, tid, nt);
    __syncthreads();
    if (p > 5) {
      for (int i = tid; i < nc; i += nt) W[i] = S[i];
      __syncthreads();
    }
  }
}


__device__ __forceinline__ void bfly5(float2 *F, int m, float2 t1, float2 t2, float2 t3, float2 t4, float2 ya,
                                      float2 yb) {
  const float2 s0 = F[0];
  const float2 s1 = cmul(F[m], t1), s2 = cmul(F[2 * m], t2), s3 = cmul(F[3 * m], t3), s4 = cmul(F[4 * m], t4);
  const float2 s7 = cadd(s1, s4), s10 = csub(s1, s4), s8 = cadd(s2, s3), s9 = csub(s2, s3);
  float2 f0;
  f0.x = s0.x + (s7.x + s8.x);
  f0.y = s0.y + (s7.y + s8.y);
  float2 s5, s6, s11, s12;
  s5.x = s0.x + s7.x * ya.x + s8.x * yb.x;
  s5.y = s0.y + s7.y * ya.x + s8.y * yb.x;
  s6.x = s10.y * ya.y + s9.y * yb.y;
  s6.y = -(s10.x * ya.y) - s9.x * yb.y;
  s11.x = s0.x + s7.x * yb.x + s8.x * ya.x;
  s11.y = s0.y + s7.y * yb.x + s8.y * ya.x;
  s12.x = -(s10.y * yb.y) + s9.y * ya.y;
  s12.y = s10.x * yb.y - s9.x * ya.y;
  F[0] = f0;
  F[m] = csub(s5, s6);
  F[4 * m] = cadd(s5, s6);
  F[2 * m] = cadd(s11, s12);
  F[3 * m] = csub(s11, s12);
}

template <int NT>
__device__ void fft960_stages(float2 *W, const float2 *__restrict__ tw, int tid) {
  for (int b = tid; b < 240; b += NT) {  // radix 4, m = 1 (degenerate: no twiddles)
    float2 *F = W + 4 * b;
    float2 f0 = F[0];
    const float2 f1 = F[1], f2 = F[2], f3 = F[3];
    const float2 s0 = csub(f0, f2);
    f0 = cadd(f0, f2);
    float2 s1 = cadd(f1, f3);
    F[2] = csub(f0, s1);
    F[0] = cadd(f0, s1);
    s1 = csub(f1, f3);
    F[1] = make_float2(s0.x + s1.y, s0.y - s1.x);
    F[3] = make_float2(s0.x - s1.y, s0.y + s1.x);
  }
  __syncthreads();
  for (int q = tid; q < 240; q += NT) {  // radix 4, m = 4, fstride 60
    const int i = q >> 2, j = q & 3;
    bfly4(W + i * 16 + j, 4, tw[j * 60], tw[j * 120], tw[j * 180]);
  }
  __syncthreads();
  for (int q = tid; q < 240; q += NT) {  // radix 4, m = 16, fstride 15
    const int i = q >> 4, j = q & 15;
    bfly4(W + i * 64 + j, 16, tw[j * 15], tw[j * 30], tw[j * 45]);
  }
  __syncthreads();
  {
    const float2 epi3 = tw[320];
    for (int q = tid; q < 320; q += NT) {  // radix 3, m = 64, fstride 5
      const int i = q >> 6, k = q & 63;
      bfly3(W + i * 192 + k, 64, tw[k * 5], tw[k * 10], epi3);
    }
  }
  __syncthreads();
  {
    const float2 ya = tw[192], yb = tw[384];
    for (int u = tid; u < 192; u += NT) bfly5(W + u, 192, tw[u], tw[2 * u], tw[3 * u], tw[4 * u], ya, yb);
  }
  __syncthreads();
}

// The same transform for persistent 256-thread workgroups: every twiddle a
// thread needs in the five stages is loaded once into registers (Fft960Tw)
// and reused for every frame the workgroup processes.  Butterfly assignment
// and arithmetic are exactly fft960_stages<256>'s.
struct Fft960Tw {
  float2 s2[3], s3[3], s4a[2], s4b[2], s5[4];
  float2 epi3, ya, yb;
};
__device__ __forceinline__ void fft960_load(Fft960Tw &t, const float2 *__restrict__ tw, int tid) {
  const int j2 = tid & 3, j3 = tid & 15, k4 = tid & 63;
  t.s2[0] = tw[j2 * 60];
  t.s2[1] = tw[j2 * 120];
  t.s2[2] = tw[j2 * 180];
  t.s3[0] = tw[j3 * 15];
  t.s3[1] = tw[j3 * 30];
  t.s3[2] = tw[j3 * 45];
  t.s4a[0] = tw[k4 * 5];  // q = tid and q = tid + 256 share k = q & 63
  t.s4a[1] = tw[k4 * 10];
  t.s4b[0] = t.s4a[0];
  t.s4b[1] = t.s4a[1];
  const int u = tid < 192 ? tid : 0;
  t.s5[0] = tw[u];
  t.s5[1] = tw[2 * u];
  t.s5[2] = tw[3 * u];
  t.s5[3] = tw[4 * u];
  t.epi3 = tw[320];
  t.ya = tw[192];
  t.yb = tw[384];
}
// F independent 960-point transforms W[fr][960], fr < F, by one 256-thread
// workgroup: a thread owns the same butterfly index in every frame, so its
// twiddles stay in registers and each stage costs one barrier for F frames.
template <int F, int P>
__device__ __forceinline__ void fft960_run(const Fft960Tw &t, float2 (*W)[P], int tid) {
  if (tid < 240) {  // radix 4, m = 1
#pragma unroll
    for (int fr = 0; fr < F; fr++) {
      float2 *Fp = W[fr] + 4 * tid;
      float2 f0 = Fp[0];
      const float2 f1 = Fp[1], f2 = Fp[2], f3 = Fp[3];
      const float2 s0 = csub(f0, f2);
      f0 = cadd(f0, f2);
      float2 s1 = cadd(f1, f3);
      Fp[2] = csub(f0, s1);
      Fp[0] = cadd(f0, s1);
      s1 = csub(f1, f3);
      Fp[1] = make_float2(s0.x + s1.y, s0.y - s1.x);
      Fp[3] = make_float2(s0.x - s1.y, s0.y + s1.x);
    }
  }
  __syncthreads();
  if (tid < 240) {
#pragma unroll
    for (int fr = 0; fr < F; fr++) bfly4(W[fr] + (tid >> 2) * 16 + (tid & 3), 4, t.s2[0], t.s2[1], t.s2[2]);
  }
  __syncthreads();
  if (tid < 240) {
#pragma unroll
    for (int fr = 0; fr < F; fr++) bfly4(W[fr] + (tid >> 4) * 64 + (tid & 15), 16, t.s3[0], t.s3[1], t.s3[2]);
  }
  __syncthreads();
#pragma unroll
  for (int fr = 0; fr < F; fr++) {
    bfly3(W[fr] + (tid >> 6) * 192 + (tid & 63), 64, t.s4a[0], t.s4a[1], t.epi3);
    if (tid < 64) bfly3(W[fr] + ((tid + 256) >> 6) * 192 + (tid & 63), 64, t.s4b[0], t.s4b[1], t.epi3);
  }
  __syncthreads();
  if (tid < 192) {
#pragma unroll
    for (int fr = 0; fr < F; fr++) bfly5(W[fr] + tid, 192, t.s5[0], t.s5[1], t.s5[2], t.s5[3], t.ya, t.yb);
  }
  __syncthreads();
}

// Band tables of one persistent workgroup, staged in LDS: the band edges and
// interpolation weights (every band sum and gain interpolation), plus the DCT
// matrix for the kernels that compute cepstra (k_synthw keeps only the edges).
struct BandEdges {
  float frac[400];
  int of[400];
  int e4[kBands + 2];
};
struct BandTab : BandEdges {
  float dct[kBands * kBands];
};
__device__ __forceinline__ void bandedges_load(BandEdges &b, const Plan *__restrict__ P, int tid, int nt) {
  for (int i = tid; i < 400; i += nt) {
    b.frac[i] = P->band_frac[i];
    b.of[i] = P->band_of[i];
  }
  for (int i = tid; i < kBands; i += nt) b.e4[i] = P->eband4[i];
}
__device__ __forceinline__ void bandtab_load(BandTab &b, const Plan *__restrict__ P, int tid, int nt) {
  bandedges_load(b, P, tid, nt);
  for (int i = tid; i < kBands * kBands; i += nt) b.dct[i] = P->dct[i];
}
__device__ __forceinline__ float band_sum_t(const float2 *A, const float2 *B, const BandEdges &T, int b) {
  float acc = 0;
  if (b >= 1) {
#pragma unroll 4
    for (int k = T.e4[b - 1]; k < T.e4[b]; k++) {
      float tmp = A[k].x * B[k].x;
      tmp += A[k].y * B[k].y;
      acc += T.frac[k] * tmp;
    }
  }
  if (b <= kBands - 2) {
#pragma unroll 4
    for (int k = T.e4[b]; k < T.e4[b + 1]; k++) {
      float tmp = A[k].x * B[k].x;
      tmp += A[k].y * B[k].y;
      acc += (1 - T.frac[k]) * tmp;
    }
  }
  if (b == 0 || b == kBands - 1) acc *= 2;
  return acc;
}
// compute_band_energy / compute_band_corr split in two: the per-bin terms of
// bin k < 400 (band i = of[k]) are computed by any lane,
//   lo[k] = (1 - frac[k]) * tmp  (summed into band i)
//   hi[k] = frac[k] * tmp        (summed into band i + 1),  tmp = A.x*B.x + A.y*B.y,
// with exactly band_sum_t's roundings; band_chain() then adds them in band_sum_t's
// order.  Band edges are multiples of 4, so the chain reads 4 terms per load.
__device__ __forceinline__ void band_terms(float2 A, float2 B, const BandEdges &T, int k, float &lo, float &hi) {
  float tmp = A.x * B.x;
  tmp += A.y * B.y;
  hi = T.frac[k] * tmp;
  lo = (1 - T.frac[k]) * tmp;
}
__device__ __forceinline__ float band_chain(const float *lo, const float *hi, const BandEdges &T, int b) {
  float acc = 0;
  if (b >= 1) {
    const float4 *h4 = reinterpret_cast<const float4 *>(hi);
    for (int q = T.e4[b - 1] >> 2; q < T.e4[b] >> 2; q++) {
      const float4 v = h4[q];
      acc += v.x;
      acc += v.y;
      acc += v.z;
      acc += v.w;
    }
  }
  if (b <= kBands - 2) {
    const float4 *l4 = reinterpret_cast<const float4 *>(lo);
    for (int q = T.e4[b] >> 2; q < T.e4[b + 1] >> 2; q++) {
      const float4 v = l4[q];
      acc += v.x;
      acc += v.y;
      acc += v.z;
      acc += v.w;
    }
  }
  if (b == 0 || b == kBands - 1) acc *= 2;
  return acc;
}

__device__ __forceinline__ float interp_gain_t(const float *bandE, const BandEdges &T, int k) {
  if (k >= 400) return 0.0f;
  const int b = T.of[k];
  const float frac = T.frac[k];
  return (1 - frac) * bandE[b] + frac * bandE[b + 1];
}

// compute_band_energy / compute_band_corr: one lane per band, C summation order.
__device__ __forceinline__ float band_sum(const float2 *A, const float2 *B, const Plan *__restrict__ P, int b) {
  float acc = 0;
  if (b >= 1) {
#pragma unroll 4
    for (int k = P->eband4[b - 1]; k < P->eband4[b]; k++) {
      float tmp = A[k].x * B[k].x;
      tmp += A[k].y * B[k].y;
      acc += P->band_frac[k] * tmp;
    }
  }
  if (b <= kBands - 2) {
#pragma unroll 4
    for (int k = P->eband4[b]; k < P->eband4[b + 1]; k++) {
      float tmp = A[k].x * B[k].x;
      tmp += A[k].y * B[k].y;
      acc += (1 - P->band_frac[k]) * tmp;
    }
  }
  if (b == 0 || b == kBands - 1) acc *= 2;
  return acc;
}

// interp_band_gain value at bin k (bins >= 400 keep their zero initialiser)
__device__ __forceinline__ float interp_gain(const float *bandE, const Plan *__restrict__ P, int k) {
  if (k >= 400) return 0.0f;
  const int b = P->band_of[k];
  const float frac = P->band_frac[k];
  return (1 - frac) * bandE[b] + frac * bandE[b + 1];
}

// Sequential dot product acc = ((acc + a[0]*b[0]) + a[1]*b[1]) + ... in C
// order over LDS operands (strides sa / sb, n a multiple of 4, n >= 8), with
// the loads of the next two 4-term blocks issued before the current block's
// arithmetic: the serial add chain no longer waits on LDS latency per block.
__device__ __forceinline__ float dot_seq(float acc, const float *a, int sa, const float *b, int sb, int n) {
  float a0[4], b0[4], a1[4], b1[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    a0[u] = a[u * sa];
    b0[u] = b[u * sb];
    a1[u] = a[(4 + u) * sa];
    b1[u] = b[(4 + u) * sb];
  }
  int i = 0;
  for (; i + 8 < n; i += 4) {
    float a2[4], b2[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      a2[u] = a[(i + 8 + u) * sa];
      b2[u] = b[(i + 8 + u) * sb];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc = acc + a0[u] * b0[u];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      a0[u] = a1[u];
      b0[u] = b1[u];
      a1[u] = a2[u];
      b1[u] = b2[u];
    }
  }
#pragma unroll
  for (int u = 0; u < 4; u++) acc = acc + a0[u] * b0[u];
#pragma unroll
  for (int u = 0; u < 4; u++) acc = acc + a1[u] * b1[u];
  return acc;
}

// find_best_pitch (pitch.c) split in two: the Syy energy recurrence depends
// only on y, so syy_sequence() produces the value Syy holds at every lag i
// (before its update), and best_pitch_visit() replays the selection for one
// lag.  Visiting the lags in increasing order reproduces find_best_pitch
// exactly; lags with xcorr <= 0 only advance Syy and may be skipped.
__device__ void syy_sequence(const float *y, int ys, int len, int max_pitch, float *syy) {
  float Syy = dot_seq(1.0f, y, ys, y, ys, len);
#pragma unroll 4
  for (int i = 0; i < max_pitch; i++) {
    syy[i] = Syy;
    const float ya = y[(i + len) * ys], yb = y[i * ys];
    Syy += ya * ya - yb * yb;
    Syy = (1 > Syy) ? 1 : Syy;
  }
}

__device__ __forceinline__ void best_pitch_visit(float xc, float Syy, int i, float &bn0, float &bn1, float &bd0,
                                                 float &bd1, int *best) {
  // branch-free form of find_best_pitch's update: same comparisons, same values
  float xcorr16 = xc;
  xcorr16 *= 1e-12f;
  const float num = xcorr16 * xcorr16;
  const bool c1 = (xc > 0) && (num * bd1 > bn1 * Syy);
  const bool c2 = c1 && (num * bd0 > bn0 * Syy);
  bn1 = c2 ? bn0 : (c1 ? num : bn1);
  bd1 = c2 ? bd0 : (c1 ? Syy : bd1);
  best[1] = c2 ? best[0] : (c1 ? i : best[1]);
  bn0 = c2 ? num : bn0;
  bd0 = c2 ? Syy : bd0;
  best[0] = c2 ? i : best[0];
}

__device__ __forceinline__ float pitch_gain(float xy, float xx, float yy) { return xy / sqrtf(1 + xx * yy); }

// pitch.c second_check[16] = {0,0,3,2,3,2,5,2,3,2,3,2,5,2,3,2}, packed 3 bits per entry
__device__ __forceinline__ int second_check(int k) { return (int)((0x4d54d35534c0ull >> (3 * k)) & 7); }

template <int NT>
__device__ void dense_layer(const DevDense &d, const float *in, float *out, const float *tansig_tab, int tid) {
  for (int i = tid; i < d.nout; i += NT) {
    float sum = d.b[i];
#pragma unroll 8
    for (int j = 0; j < d.nin; j++) sum += d.w[j * d.nout + i] * in[j];
    out[i] = activate(tansig_tab, d.act, kWs * sum);
  }
}

// compute_gru (rnn.c): z/r gates on 2N lanes, then h on N lanes.  Each
// neuron's sum runs in C order on its own lane.
template <int NT>
__device__ void gru_gates(const DevGru &g, const float *in, const float *state, float *zr, const float *tab,
                          int tid) {
  const int N = g.nout, M = g.nin, S3 = 3 * N;
  for (int t = tid; t < 2 * N; t += NT) {
    const int col = t;  // z: col = i, r: col = N + i
    float sum = g.b[col];
#pragma unroll 8
    for (int j = 0; j < M; j++) sum += g.win[j * S3 + col] * in[j];
#pragma unroll 8
    for (int j = 0; j < N; j++) sum += g.wrec[j * S3 + col] * state[j];
    zr[t] = sigmoid(tab, kWs * sum);
  }
}
template <int NT>
__device__ void gru_out(const DevGru &g, const float *in, const float *state, const float *zr, float *h,
                        const float *tab, int tid) {
  const int N = g.nout, M = g.nin, S3 = 3 * N;
  for (int i = tid; i < N; i += NT) {
    float sum = g.b[2 * N + i];
#pragma unroll 8
    for (int j = 0; j < M; j++) sum += g.win[j * S3 + 2 * N + i] * in[j];
#pragma unroll 8
    for (int j = 0; j < N; j++) sum += g.wrec[j * S3 + 2 * N + i] * state[j] * zr[N + j];
    sum = activate(tab, g.act, kWs * sum);
    h[i] = zr[i] * state[i] + (1 - zr[i]) * sum;
  }
}


}  // namespace fvad
