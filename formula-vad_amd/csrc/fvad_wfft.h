// Wave-per-frame 960-point celt FFT (opus_fft_impl order: radix 4 (m = 1),
// 4 (m = 4), 4 (m = 16), 3 (m = 64), 5 (m = 192)) in registers, with two
// wave-private LDS exchanges and no workgroup barrier.
//
// Write the in-place transform index as n = 192a + 64b + 16c + 4d + e
// (a < 5, b < 3, c, d, e < 4).  The digit-reversed copy of opus_fft_impl puts
// input sample i = a + 5b + 15c + 60d + 240e at W[n] (checked against
// celt_bitrev for all 960 indices), and the five stages mix e, d, c, b, a in
// that order.  Three lane layouts keep each stage's butterfly in one lane:
//
//   A  lane = 4q + c, q = a + 5b (60 lanes), registers k = d + 4e: input
//      samples 60k + q + 15c (one 240-byte run per register); stages 1 and 2
//   C  lane = 4q + d, registers c + 4e: stage 3 (twiddles per lane: j = 4d + e)
//   B  lane = 16c + 4d + e, registers R = 3a + b: stages 4 and 5; register R
//      of lane l then holds bin 64R + l of the output (natural order)
//
// A -> C and C -> B go through the wave's own 1024-slot LDS region (8 KB):
//   exchange 1 slot = 68q + 17c + d + 4e,   exchange 2 slot = 65q + 16c + 4d + e.
// In each of the four accesses the lane part is one base address and the
// register part a compile-time offset, and every access is bank-conflict free
// (ds_write_b64: (slot mod 16) distinct in each 16-lane group; ds_read_b64:
// (slot mod 32) distinct in each 32-lane group).  Idle lanes (q = 15) neither
// write nor read out of the region.
// Butterflies are fvad_device.h's bfly4 / bfly3 / bfly5 on a register array
// (m = 1), i.e. the same expressions in the same order as the restated
// kiss_fft, so results are bit-identical to fft960_run.
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "fvad_device.h"

namespace fvad {
namespace wfft {

constexpr int kSlots = 1024;  // float2 slots of a wave's exchange region

// LDS written and read back by lanes of the same wave only: a wave's LDS
// operations execute in order, so a compiler-level fence is all it needs.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Twiddles.  Per lane in registers: stage 2 (wave-uniform) and stage 4; in a
// per-workgroup LDS table (TwTab): stage 3 (j = 4d + e) and stage 5
// (u = 64b + lane), read once per transform (conflict-free / broadcast).
struct Tw {
  float2 s2[4][3];  // stage 2, j = e: tw[60j], tw[120j], tw[180j]
  float2 s4[2];     // stage 4, k = lane: tw[5k], tw[10k]
  float2 epi3, ya, yb;
};
struct TwTab {
  float2 s3[4][3][4];   // [e][r][d]: tw[15 (r + 1) (4d + e)]
  float2 s5[3][4][64];  // [b][r][lane]: tw[(r + 1) (64b + lane)]
};
__device__ __forceinline__ void load_tw(Tw &t, const float2 *__restrict__ tw, int lane) {
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int r = 0; r < 3; r++) t.s2[j][r] = tw[60 * (r + 1) * j];
  t.s4[0] = tw[5 * lane];
  t.s4[1] = tw[10 * lane];
  t.epi3 = tw[320];
  t.ya = tw[192];
  t.yb = tw[384];
}
__device__ __forceinline__ void load_twtab(TwTab &T, const float2 *__restrict__ tw, int tid, int nt) {
  for (int i = tid; i < 48; i += nt) {
    const int e = i / 12, r = (i / 4) % 3, d = i % 4;
    T.s3[e][r][d] = tw[15 * (r + 1) * (4 * d + e)];
  }
  for (int i = tid; i < 768; i += nt) {
    const int b = i / 256, r = (i / 64) % 4, l = i % 64;
    T.s5[b][r][l] = tw[(r + 1) * (64 * b + l)];
  }
}

// Input index of register k of a layout-A lane (q = lane >> 2, c = lane & 3);
// lanes 60..63 (q = 15) carry no data.
__device__ __forceinline__ int in_index(int lane, int k) { return (lane >> 2) + 15 * (lane & 3) + 60 * k; }

// v: layout A on entry (v[k] = scaled input sample in_index(lane, k), zero
// for lanes >= 60); on return v[R] = X[64R + lane] for R < 15.  R: this wave's
// exchange region.
__device__ __forceinline__ void run(float2 (&v)[16], const Tw &t, const TwTab &TT, float2 *R, int lane) {
  // stage 1: radix 4, m = 1 (degenerate, no twiddles) over e
#pragma unroll
  for (int d = 0; d < 4; d++) {
    float2 f0 = v[d];
    const float2 f1 = v[d + 4], f2 = v[d + 8], f3 = v[d + 12];
    const float2 s0 = csub(f0, f2);
    f0 = cadd(f0, f2);
    float2 s1 = cadd(f1, f3);
    v[d + 8] = csub(f0, s1);
    v[d] = cadd(f0, s1);
    s1 = csub(f1, f3);
    v[d + 4] = make_float2(s0.x + s1.y, s0.y - s1.x);
    v[d + 12] = make_float2(s0.x - s1.y, s0.y + s1.x);
  }
  // stage 2: radix 4, m = 4 over d (j = e)
#pragma unroll
  for (int e = 0; e < 4; e++) {
    float2 F[4] = {v[4 * e], v[4 * e + 1], v[4 * e + 2], v[4 * e + 3]};
    bfly4(F, 1, t.s2[e][0], t.s2[e][1], t.s2[e][2]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[4 * e + u] = F[u];
  }
  // A -> C
  const int q = lane >> 2, lo = lane & 3;  // A: lo = c; C: lo = d
  const bool live = q < 15;
  const int qc = live ? q : 14;  // idle lanes read (and ignore) lane 56's slots
  {
    float2 *w = R + 68 * q + 17 * lo;  // + d + 4e = k
    if (live) {
#pragma unroll
      for (int k = 0; k < 16; k++) w[k] = v[k];
    }
  }
  wsync();
  {
    const float2 *r = R + 68 * qc + lo;  // + 17c + 4e
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = r[17 * (i & 3) + 4 * (i >> 2)];  // v[c + 4e]
  }
  // stage 3: radix 4, m = 16 over c (j = 4d + e)
#pragma unroll
  for (int e = 0; e < 4; e++) {
    float2 F[4] = {v[4 * e], v[4 * e + 1], v[4 * e + 2], v[4 * e + 3]};
    bfly4(F, 1, TT.s3[e][0][lo], TT.s3[e][1][lo], TT.s3[e][2][lo]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[4 * e + u] = F[u];
  }
  wsync();
  // C -> B
  {
    float2 *w = R + 65 * q + 4 * lo;  // + 16c + e
    if (live) {
#pragma unroll
      for (int i = 0; i < 16; i++) w[16 * (i & 3) + (i >> 2)] = v[i];
    }
  }
  wsync();
  {
    const float2 *r = R + lane;  // lane = 16c + 4d + e; + 65q
#pragma unroll
    for (int Rg = 0; Rg < 15; Rg++) v[Rg] = r[65 * (Rg / 3 + 5 * (Rg % 3))];
  }
  wsync();
  // stage 4: radix 3, m = 64 over b (k = lane)
#pragma unroll
  for (int a = 0; a < 5; a++) {
    float2 F[3] = {v[3 * a], v[3 * a + 1], v[3 * a + 2]};
    bfly3(F, 1, t.s4[0], t.s4[1], t.epi3);
#pragma unroll
    for (int u = 0; u < 3; u++) v[3 * a + u] = F[u];
  }
  // stage 5: radix 5, m = 192 over a (u = 64b + lane)
#pragma unroll
  for (int b = 0; b < 3; b++) {
    float2 F[5] = {v[b], v[3 + b], v[6 + b], v[9 + b], v[12 + b]};
    bfly5(F, 1, TT.s5[b][0][lane], TT.s5[b][1][lane], TT.s5[b][2][lane], TT.s5[b][3][lane], t.ya, t.yb);
#pragma unroll
    for (int u = 0; u < 5; u++) v[3 * u + b] = F[u];
  }
}

}  // namespace wfft
}  // namespace fvad
