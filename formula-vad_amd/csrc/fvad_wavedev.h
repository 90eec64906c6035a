// Per-wave frame helpers shared by the wave-per-frame kernels (fvad_wave.hip)
// and the fused pitch-spectrum + GRU kernel (fvad_gru16.hip, k_fused16): the
// tables a workgroup keeps in LDS, a frame's window loads, and one frame's
// pitch spectrum (k_pspecw's per-frame work), so both kernels run the same
// expressions in the same order.
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "fvad_device.h"
#include "fvad_internal.h"
#include "fvad_staged.h"
#include "fvad_staged_dev.h"
#include "fvad_wfft.h"

namespace fvad {

// A per-iteration zero the compiler cannot see through: table reads indexed
// with it stay inside the frame loop instead of being hoisted into registers
// for the whole kernel (which would cost occupancy).
__device__ __forceinline__ int opaque0() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

struct WaveTabs {
  BandTab T;
  wfft::TwTab tw;
  float hw[kFrame];
};
__device__ __forceinline__ void wave_tabs_load(WaveTabs &w, const Plan *__restrict__ P, int tid, int nt) {
  bandtab_load(w.T, P, tid, nt);
  wfft::load_twtab(w.tw, reinterpret_cast<const float2 *>(P->tw960), tid, nt);
  for (int i = tid; i < kFrame; i += nt) w.hw[i] = P->half_window[i];
}

// A frame's raw window samples.  (Loading them one frame ahead saved k_pspecw
// 0.07 ms at 3 waves per SIMD; its 16 registers kept it there.  Without the
// prefetch it fits 128 VGPRs and runs 4 waves per SIMD, which hide that
// latency better: 0.531 -> 0.497 ms.)
struct WinRaw {
  float x[16];
};
__device__ __forceinline__ void win_load(WinRaw &w, const float *__restrict__ pb, int lane) {
#pragma unroll
  for (int k = 0; k < 16; k++) w.x[k] = lane < 60 ? pb[wfft::in_index(lane, k)] : 0.0f;
}
// layout-A input of a 960-sample analysis window from its prefetched samples
// (x * w / 960, imag 0)
__device__ __forceinline__ void win_apply(const WinRaw &w, const float *hw, int lane, float2 (&v)[16]) {
  hw += opaque0();
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int i = wfft::in_index(lane, k);
    float val = w.x[k];
    val *= lane < 60 ? win960(hw, i) : 0.0f;
    v[k] = make_float2(kScale960 * val, kScale960 * 0.0f);
  }
}

// One frame's pitch spectrum, one wave (rnnoise compute_frame_features after
// pitch_search / remove_doubling, called from rnnoise_process_frame at
// Denoiser.zig:60), in two halves.  pspec_transform: the pitch window at lag
// pit -> FFT -> P (HBM), the Ep and Exp band terms into the wave's exchange
// region R (its inputs from pspec_load; the frame's Ex of band `lane` goes on
// to the second half).  pspec_features: the band energies Ep and the normalised
// correlations Exp (HBM, k_synthw reads them), DCT(Exp); returns, on lanes
// 0..6, the frame's features 34..40 (lane 6: .01 (pit - 300)), which the
// caller stores.  k_pspecw runs the halves back to back (pspec_frame),
// k_fused16 one per phase.
// A frame's inputs to pspec_transform: the raw pitch window, X of bins < 400
// (Exp terms) and the band's Ex (k_fused16 loads them a phase ahead)
struct PspecIn {
  WinRaw w;
  float2 xr[7];
  float exl;
};
__device__ __forceinline__ void pspec_load(PspecIn &in, const StagedArgs &a, int f, int pit, int lane) {
  win_load(in.w, frame_pb(a, f) + (kPitchBuf - kWin - pit), lane);
  const float2 *X = a.X + (size_t)f * kFreq;
#pragma unroll
  // (unconditional loads, lanes past the bins read bin 480 and are never
  // used: a masked load's block would take its consumers, and their wait,
  // right after it)
  for (int r = 0; r < 7; r++) in.xr[r] = X[min(64 * r + lane, kFreq - 1)];
  in.exl = a.Ex[(size_t)f * kBands + min(lane, kBands - 1)];
}
__device__ __forceinline__ void pspec_transform(const StagedArgs &a, int f, const PspecIn &in, const WaveTabs &tb,
                                                const wfft::Tw &tw, float2 *R, int lane) {
  const BandTab &T = tb.T;
  float *tr = reinterpret_cast<float *>(R);
  const float2 *xr = in.xr;
  float2 v[16];
  win_apply(in.w, tb.hw, lane, v);
  wfft::run(v, tw, tb.tw, R, lane);
  float2 *P = a.P + (size_t)f * kFreq;
#pragma unroll
  for (int r = 0; r < 8; r++)
    if (64 * r + lane < kFreq) P[64 * r + lane] = v[r];
#pragma unroll
  for (int r = 0; r < 7; r++) {
    const int n = 64 * r + lane;
    if (n < 400) {
      band_terms(v[r], v[r], T, n, tr[n], tr[400 + n]);
      band_terms(xr[r], v[r], T, n, tr[800 + n], tr[1200 + n]);
    }
  }
  wfft::wsync();
}
__device__ __forceinline__ float pspec_features(const StagedArgs &a, int f, int pit, const WaveTabs &tb,
                                                const float2 *R, int lane, float exl) {
  const BandTab &T = tb.T;
  const float *tr = reinterpret_cast<const float *>(R);
  // Ep chains on lanes 0..21, Exp chains on lanes 32..53
  const int h = lane >> 5, b = lane & 31;
  float cv = 0;
  if (b < kBands) cv = band_chain(tr + 800 * h, tr + 800 * h + 400, T, b);
  const float expv = __shfl(cv, lane + 32);
  float e = 0;
  if (lane < kBands) {
    const size_t o = (size_t)f * kBands + lane;
    e = (float)((double)expv / sqrt(.001 + (double)(exl * cv)));
    a.Ep[o] = cv;
    a.Exp[o] = e;
  }
  float sum = 0;
#pragma unroll
  for (int j = 0; j < kBands; j++)
    sum += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), j)) * T.dct[j * kBands + (lane < 6 ? lane : 0)];
  float val = (float)(sum * sqrt(2. / 22));
  if (lane == 0) val = (float)(val - 1.3);
  if (lane == 1) val = (float)(val - 0.9);
  if (lane == 6) val = (float)(.01 * (pit - 300));
  wfft::wsync();
  return val;
}
__device__ __forceinline__ float pspec_frame(const StagedArgs &a, int f, int pit, const WaveTabs &tb,
                                             const wfft::Tw &tw, float2 *R, int lane) {
  // (inputs loaded before the transform: Ex loaded after the P stores waited for them)
  PspecIn in;
  pspec_load(in, a, f, pit, lane);
  pspec_transform(a, f, in, tb, tw, R, lane);
  return pspec_features(a, f, pit, tb, R, lane, in.exl);
}

}  // namespace fvad
