// Wave-per-frame FFT kernels of the staged pipeline (k_fftAw, k_pspecw,
// k_synthw).  A translation unit of their own: they are built without SLP
// vectorisation (Makefile), which keeps their f32 arithmetic in single
// (non-packed) VALU instructions -- measured faster for these kernels, while
// the GRU kernel in fvad_staged.hip prefers the packed form.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "fvad_device.h"
#include "fvad_internal.h"
#include "fvad_staged.h"
#include "fvad_staged_dev.h"
#include "fvad_wavedev.h"
#include "fvad_wfft.h"

namespace fvad {

// ---------------------------------------------------------------------------
// Wave-per-frame frame kernels (k_fftAw, k_pspecw, k_synthw): one wave owns a
// frame at a time and runs its 960-point transform in registers (fvad_wfft.h)
// with its own LDS region, so a workgroup never waits at a barrier between
// FFT stages; band terms go to the same region once the transform is done and
// the 22 band chains run on lanes 0..21 (k_pspecw: Ep on 0..21 beside Exp on
// 32..53).  Same arithmetic as the fused k_frame.  Frames are taken
// in batches of kWB consecutive frames per wave (dynamic, per-XCD queues as
// take_group); k_fftAw runs each batch's serial Ly chains lane per frame.
// ---------------------------------------------------------------------------
constexpr int kWB = 8;   // frames per wave batch
constexpr int kWNW = 4;  // waves per workgroup
constexpr int kWOcc = 3;  // waves per SIMD (<= 168 VGPRs; 3 workgroups per CU at <= 53 KB LDS)

// Batches of a wave: dynamic (per-XCD queues, wave_take) or static striding
// over the grid's waves, per kernel (bit 1 << kind of kWaveStatic).  k_fftAw
// runs beside the next push's k_prep3 and balances better dynamically; the
// others run alone, where static striding saves the queue atomics.
constexpr int kWaveStatic = (1 << kWavePspec) | (1 << kWaveSynth);
__device__ __forceinline__ bool wave_is_static(const StagedArgs &, WaveKernel k) { return (kWaveStatic >> k) & 1; }
template <int NW = kWNW>
__device__ __forceinline__ long long wave_first(const StagedArgs &a, WaveKernel k, int slot, int lane) {
  return wave_is_static(a, k) ? (long long)blockIdx.x * NW + (threadIdx.x >> 6) : wave_take(a, slot, lane);
}
template <int NW = kWNW>
__device__ __forceinline__ long long wave_next(const StagedArgs &a, WaveKernel k, int slot, int lane, long long g) {
  return wave_is_static(a, k) ? g + (long long)gridDim.x * NW : wave_take(a, slot, lane);
}

// A batch's frame indices, lane fr < kWB holding slot fr's frame (or -1),
// computed once per batch: the frame loop reads them with readlane instead of
// a per-frame ticks_valid load, whose wait also waited for every store the
// wave still had in flight (gfx9 counts loads and stores in one vmcnt)
__device__ __forceinline__ int batch_frames(const StagedArgs &a, long long g, int lane) {
  return lane < kWB ? frame_of(a, g, kWB, lane) : -1;
}
__device__ __forceinline__ int lane_val(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// wait for v's load here, once per batch (a readlane of it inside the frame
// loop would otherwise get a conservative wait that also drains the stores of
// the frames before)
__device__ __forceinline__ void settle(int v) { asm volatile("" ::"v"(v)); }

__global__ void __launch_bounds__(64 * kWNW, kWOcc) k_fftAw(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 Rg[kWNW][wfft::kSlots];
  __shared__ WaveTabs tb;
  __shared__ float exb[kWNW][kWB][kBands + 2], lyb[kWNW][kWB][kBands + 2];
  __shared__ int silb[kWNW][kWB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  wave_tabs_load(tb, a.plan, tid, 64 * kWNW);
  wfft::Tw tw;
  wfft::load_tw(tw, reinterpret_cast<const float2 *>(a.plan->tw960), lane);
  __syncthreads();
  const BandTab &T = tb.T;
  float2 *R = Rg[wv];
  float *tr = reinterpret_cast<float *>(R);
  const long long nb = ((long long)a.n_streams * a.V + kWB - 1) / kWB;
  for (long long g = wave_first(a, kWaveFftA, kWorkFftA, lane); g < nb; g = wave_next(a, kWaveFftA, kWorkFftA, lane, g)) {
    const int fl = batch_frames(a, g, lane);
    for (int fr = 0; fr < kWB; fr++) {
      const int f = lane_val(fl, fr);
      if (f < 0) continue;
      float2 v[16];
      const float *pb = frame_pb(a, f);
      // the frame's new x_lp values n = 624..863 (pitch buffer samples
      // 1247..1727, inside the window), 4 per lane (lanes 0..59): samples
      // 1247 + 8 * lane .. 1255 + 8 * lane load before the transform
      static_assert(kXlp - kXlpHist == 4 * 60 && kHist % 4 == 0, "x_lp lanes");
      float xm = 0;
      float4 qa = make_float4(0, 0, 0, 0), qb = qa;
      if (lane < 60) {
        const float *q = pb + kHist + 8 * lane;
        xm = q[-1];
        qa = *reinterpret_cast<const float4 *>(q);
        qb = *reinterpret_cast<const float4 *>(q + 4);
      }
      WinRaw w;
      win_load(w, pb + (kPitchBuf - kWin), lane);
      win_apply(w, tb.hw, lane, v);
      wfft::run(v, tw, tb.tw, R, lane);
      float2 *X = a.X + (size_t)f * kFreq;
#pragma unroll
      for (int r = 0; r < 8; r++)
        if (64 * r + lane < kFreq) X[64 * r + lane] = v[r];
      if (lane < 60) {
        // x_lp[n] = f(x[2n-1], x[2n], x[2n+1]), n = 624 + 4 * lane + t
        float4 o;
        o.x = xlp_value(xm, qa.x, qa.y);
        o.y = xlp_value(qa.y, qa.z, qa.w);
        o.z = xlp_value(qa.w, qb.x, qb.y);
        o.w = xlp_value(qb.y, qb.z, qb.w);
        *reinterpret_cast<float4 *>(frame_xlp(a, f) + kXlpHist + 4 * lane) = o;
      }
#pragma unroll
      for (int r = 0; r < 7; r++) {
        const int n = 64 * r + lane;
        if (n < 400) band_terms(v[r], v[r], T, n, tr[n], tr[400 + n]);
      }
      wfft::wsync();
      if (lane < kBands) {
        const float ex = band_chain(tr, tr + 400, T, lane);
        a.Ex[(size_t)f * kBands + lane] = ex;
        exb[wv][fr][lane] = ex;
        lyb[wv][fr][lane] = (float)log10(1e-2 + (double)ex);
      }
      wfft::wsync();
    }
    // the Ly floor chain and the silence gate, lane per frame
    if (lane < kWB) {
      const int f = fl;
      if (f >= 0) {
        float *Ly = lyb[wv][lane];
        const float *Exl = exb[wv][lane];
        float logMax = -2, follow = -2, E = 0;
        for (int i = 0; i < kBands; i++) {
          const float ly0 = Ly[i];
          const double bb = (follow - 1.5 > (double)ly0) ? follow - 1.5 : (double)ly0;
          const double aa = ((double)(logMax - 7) > bb) ? (double)(logMax - 7) : bb;
          const float ly = (float)aa;
          Ly[i] = ly;
          logMax = (logMax > ly) ? logMax : ly;
          follow = (float)((follow - 1.5 > (double)ly) ? follow - 1.5 : (double)ly);
          E += Exl[i];
        }
        const int sil = ((double)E < 0.04) ? 1 : 0;
        silb[wv][lane] = sil;
        a.silence[f] = sil;
      }
    }
    wfft::wsync();
    for (int idx = lane; idx < kWB * kBands; idx += 64) {
      const int fr = idx / kBands, b = idx - fr * kBands;
      const int f = __shfl(fl, fr);
      if (f >= 0 && !silb[wv][fr]) {
        const float *Ly = lyb[wv][fr];
        float sum = 0;
#pragma unroll
        for (int j = 0; j < kBands; j++) sum += Ly[j] * T.dct[j * kBands + b];
        float val = (float)(sum * sqrt(2. / 22));
        if (b == 0) val -= 12;
        if (b == 1) val -= 4;
        a.Lyf[(size_t)f * kBands + b] = val;
      }
    }
    wfft::wsync();
  }
}

// k_pspecw: as k_synthw, kPNW waves per workgroup on one table copy, 2
// workgroups per CU = 4 waves per SIMD (<= 128 VGPRs, 79 KB of LDS)
constexpr int kPNW = 8;
__global__ void __launch_bounds__(64 * kPNW, 4) k_pspecw(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 Rg[kPNW][wfft::kSlots];
  __shared__ WaveTabs tb;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  wave_tabs_load(tb, a.plan, tid, 64 * kPNW);
  wfft::Tw tw;
  wfft::load_tw(tw, reinterpret_cast<const float2 *>(a.plan->tw960), lane);
  __syncthreads();
  float2 *R = Rg[wv];
  const long long nb = ((long long)a.n_streams * a.V + kWB - 1) / kWB;
  for (long long g = wave_first<kPNW>(a, kWavePspec, kWorkPspec, lane); g < nb;
       g = wave_next<kPNW>(a, kWavePspec, kWorkPspec, lane, g)) {
    // the batch's frames and their pitches, lane per frame
    const int fl = batch_frames(a, g, lane);
    const int pl = fl >= 0 ? a.pitch[fl] : 0;
    settle(pl);
#pragma unroll 1
    for (int fr = 0; fr < kWB; fr++) {
      const int f = lane_val(fl, fr);
      if (f < 0) continue;
      const float v34 = pspec_frame(a, f, lane_val(pl, fr), tb, tw, R, lane);
      if (lane < 7) a.f34[(size_t)f * 8 + lane] = v34;
    }
  }
}

// k_synthw: kSNW waves per workgroup sharing one copy of the tables (band
// edges without the DCT, twiddles, window): 2 workgroups = 16 waves per CU,
// 4 per SIMD, within 160 KB of LDS and 128 VGPRs (the other wave kernels hold
// 3 per SIMD: their VGPRs exceed 128)
constexpr int kSNW = 8;
constexpr int kSOcc = 4;  // waves per SIMD
struct SynthTabs {
  BandEdges T;
  wfft::TwTab tw;
  float hw[kFrame];
};
__global__ void __launch_bounds__(64 * kSNW, kSOcc) k_synthw(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 Rg[kSNW][wfft::kSlots];
  __shared__ SynthTabs tb;
  __shared__ float bp[kSNW][3][kBands + 2];  // r, nrm, smoothed gains of the wave's frame
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  bandedges_load(tb.T, a.plan, tid, 64 * kSNW);
  wfft::load_twtab(tb.tw, reinterpret_cast<const float2 *>(a.plan->tw960), tid, 64 * kSNW);
  for (int i = tid; i < kFrame; i += 64 * kSNW) tb.hw[i] = a.plan->half_window[i];
  wfft::Tw tw;
  wfft::load_tw(tw, reinterpret_cast<const float2 *>(a.plan->tw960), lane);
  __syncthreads();
  const BandEdges &T = tb.T;
  float2 *R = Rg[wv];
  float *tr = reinterpret_cast<float *>(R);
  float *rr = bp[wv][0], *nrm = bp[wv][1], *gsm = bp[wv][2];
  const long long nb = ((long long)a.n_streams * a.V + kWB - 1) / kWB;
  for (long long g = wave_first<kSNW>(a, kWaveSynth, kWorkSynth, lane); g < nb;
       g = wave_next<kSNW>(a, kWaveSynth, kWorkSynth, lane, g)) {
    // the batch's frames and silence flags, lane per frame
    const int fl = batch_frames(a, g, lane);
    const int sl = fl >= 0 ? a.silence[fl] : 0;
    settle(sl);
    for (int fr = 0; fr < kWB; fr++) {
      const int f = lane_val(fl, fr);
      if (f < 0) continue;
      const bool fil = !lane_val(sl, fr);  // silent frames: X passes through
      // every input of the frame in one batch of loads (each later load
      // would also wait for the stores still in flight)
      const float2 *X = a.X + (size_t)f * kFreq;
      const float2 *P = a.P + (size_t)f * kFreq;
      // (unconditional: lanes past the 481 bins / 22 bands read the last
      // one and are never used; a masked load's block would take its
      // consumers, and their wait, right after it)
      float2 xv[8], pv[8];
#pragma unroll
      for (int r = 0; r < 8; r++) xv[r] = X[min(64 * r + lane, kFreq - 1)];
#pragma unroll
      for (int r = 0; r < 8; r++) pv[r] = P[min(64 * r + lane, kFreq - 1)];
      const size_t o = (size_t)f * kBands + min(lane, kBands - 1);
      const float Exp = a.Exp[o], Ex = a.Ex[o], Ep = a.Ep[o];
      const float gg = a.gr[o], gs = a.gs[o];
      if (fil) {
        if (lane < kBands) {
          float r;
          if (Exp > gg)
            r = 1;
          else
            r = (float)((double)((Exp * Exp) * (1 - (gg * gg))) / (.001 + (double)((gg * gg) * (1 - (Exp * Exp)))));
          float cl = (0 > r) ? 0 : r;
          cl = (1 < cl) ? 1 : cl;
          r = (float)sqrt((double)cl);
          r = (float)((double)r * sqrt((double)Ex / (1e-8 + (double)Ep)));
          rr[lane] = r;
          gsm[lane] = gs;
        }
        wfft::wsync();
        // pitch filter X += r P; band terms of the filtered X
#pragma unroll
        for (int r = 0; r < 8; r++) {
          const int n = 64 * r + lane;
          if (n < kFreq) {
            const float rf = interp_gain_t(rr, T, n);
            xv[r].x += rf * pv[r].x;
            xv[r].y += rf * pv[r].y;
            if (n < 400) band_terms(xv[r], xv[r], T, n, tr[n], tr[400 + n]);
          }
        }
        wfft::wsync();
        if (lane < kBands) {
          const float newE = band_chain(tr, tr + 400, T, lane);
          nrm[lane] = (float)sqrt((double)Ex / (1e-8 + (double)newE));
        }
        wfft::wsync();
#pragma unroll
        for (int r = 0; r < 8; r++) {
          const int n = 64 * r + lane;
          if (n < kFreq) {
            const float nf = interp_gain_t(nrm, T, n);
            xv[r].x *= nf;
            xv[r].y *= nf;
            const float gf = interp_gain_t(gsm, T, n);
            xv[r].x *= gf;
            xv[r].y *= gf;
          }
        }
      }
      // Hermitian extension, gathered into layout A through the region
#pragma unroll
      for (int r = 0; r < 8; r++)
        if (64 * r + lane < kFreq) R[64 * r + lane] = xv[r];
      wfft::wsync();
      float2 v[16];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int i = wfft::in_index(lane, k);
        float2 val = make_float2(0, 0);
        if (lane < 60) {
          if (i < kFreq) {
            val = R[i];
          } else {
            const float2 c = R[kWin - i];
            val = make_float2(c.x, -c.y);
          }
        }
        v[k] = make_float2(kScale960 * val.x, kScale960 * val.y);
      }
      wfft::wsync();
      wfft::run(v, tw, tb.tw, R, lane);
      float *y = a.ys + (size_t)f * kWin;
#pragma unroll
      for (int r = 0; r < 15; r++) {
        const int n = 64 * r + lane;
        const int i = (n == 0) ? 0 : kWin - n;
        const float yv = kWin * v[r].x;
        y[i] = yv * win960(tb.hw, i);
      }
      wfft::wsync();
    }
  }
}

// ---------------------------------------------------------------------------
// k_fftbw: FFT B (kiss_fftr, nfft 2048 = a 1024-point complex kissfft, radix
// 4 x 5) of one (stream, completed window, channel) per wave, in registers.
// Transform index n = d0 + 4 d1 + 16 d2 + 64 d3 + 256 d4; kf_work's leaf
// copy puts packed input k = rev4(n) at n, and stage s (m = 4^(s-1)) mixes
// digit d(s-1) with twiddles twb[u fstride], u = n mod m.  Lane layouts:
//   X  lane = d4 + 4 d3 + 16 d2, registers d1 + 4 d0: input k = lane + 64 r
//      (coalesced); stages 1, 2
//   Y  lane = d4 + 4 d0 + 16 d1, registers d2 + 4 d3: stages 3, 4
//   Z  lane = d0 + 4 d1 + 16 d2, registers d3 + 4 d4: stage 5; register r of
//      lane l = bin 64 r + l
// Exchanges through the wave's LDS region (bank-conflict free, bijective):
//   X -> Y  slot = d4 + 4 d0 + 16 d1 + 64 d2 + 260 d3
//   Y -> Z  slot = d0 + 4 d1 + 16 d2 + 64 d3 + 260 d4
// Butterflies are bfly4 (the kissfft kf_bfly4 expressions), twiddles at every
// stage (kissfft has no degenerate m = 1 case), so results equal k_fftb's.
// ---------------------------------------------------------------------------
constexpr int kFbSlots = 1040;  // float2 slots of a wave's region (1036 used)
constexpr int kFbMag = 256;     // magnitude slots (bin_hi_all - bin_lo_all < 256, host-checked)

struct FbTabs {
  float2 t4[4][3][16];  // stage 4: [d2][r][u16]: twb[4 (r + 1) (u16 + 16 d2)]
  float2 t5[4][3][64];  // stage 5: [d3][r][lane]: twb[(r + 1) (lane + 64 d3)]
};

// Per-workgroup stage-4/5 twiddle tables; stage-2/3 twiddles come per
// transform from the plan (FbTw, cached loads) so they do not hold registers
// between transforms.
struct FbTw {
  float2 s2[4][3], s3[3], tw0;
};
__device__ __forceinline__ void fftb_tabs_load(FbTabs &tb, const Plan *__restrict__ P, int tid, int nt) {
  const float2 *__restrict__ twb = reinterpret_cast<const float2 *>(P->twb);
  for (int i = tid; i < 4 * 3 * 16; i += nt) {
    const int d2 = i / 48, r = (i / 16) % 3, u = i % 16;
    tb.t4[d2][r][u] = twb[4 * (r + 1) * (u + 16 * d2)];
  }
  for (int i = tid; i < 4 * 3 * 64; i += nt) {
    const int d3 = i / 192, r = (i / 64) % 3, l = i % 64;
    tb.t5[d3][r][l] = twb[(r + 1) * (l + 64 * d3)];
  }
}
__device__ __forceinline__ void fftb_tw_load(FbTw &w, const Plan *__restrict__ P, int lane) {
  // opaque offset: the loads stay at the transform instead of being hoisted
  const float2 *__restrict__ twb = reinterpret_cast<const float2 *>(P->twb) + opaque0();
#pragma unroll
  for (int d0 = 0; d0 < 4; d0++)
#pragma unroll
    for (int r = 0; r < 3; r++) w.s2[d0][r] = twb[64 * (r + 1) * d0];
#pragma unroll
  for (int r = 0; r < 3; r++) w.s3[r] = twb[16 * (r + 1) * (lane >> 2)];
  w.tw0 = twb[0];
}

// FFT B of one windowed 2048-sample frame given in layout X (register r of
// lane l = packed input k = l + 64 r), then kiss_fftr's split for the
// reported bins, magnitudes and the band sums in bin order; lane b < n_bands
// returns band b's sum.  R: the wave's exchange region (kFbSlots float2; the
// caller's input may live there until v is loaded); mag: kFbMag floats.
__device__ __forceinline__ float fftb_bands(float2 (&v)[16], float2 *R, float *mag, const FbTabs &tb,
                                            const StagedArgs &a, int lane) {
  const Plan *__restrict__ P = a.plan;
  FbTw w;
  fftb_tw_load(w, P, lane);
  const float2 *__restrict__ sup = reinterpret_cast<const float2 *>(P->superb);
  const int nb = a.n_bands, lo = a.bin_lo_all, hi = a.bin_hi_all;
  // stage 1 (m = 1, over d0), stage 2 (m = 4, over d1, u = d0)
#pragma unroll
  for (int d1 = 0; d1 < 4; d1++) {
    float2 F[4] = {v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12]};
    bfly4(F, 1, w.tw0, w.tw0, w.tw0);
#pragma unroll
    for (int u = 0; u < 4; u++) v[d1 + 4 * u] = F[u];
  }
#pragma unroll
  for (int d0 = 0; d0 < 4; d0++) {
    float2 F[4] = {v[4 * d0], v[4 * d0 + 1], v[4 * d0 + 2], v[4 * d0 + 3]};
    bfly4(F, 1, w.s2[d0][0], w.s2[d0][1], w.s2[d0][2]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[4 * d0 + u] = F[u];
  }
  // X -> Y
  wfft::wsync();
  {
    float2 *wr = R + (lane & 3) + 260 * ((lane >> 2) & 3) + 64 * (lane >> 4);  // + 4 d0 + 16 d1
#pragma unroll
    for (int r = 0; r < 16; r++) wr[4 * (r >> 2) + 16 * (r & 3)] = v[r];
  }
  wfft::wsync();
  {
    const float2 *rd = R + lane;  // + 64 d2 + 260 d3
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = rd[64 * (r & 3) + 260 * (r >> 2)];
  }
  // stage 3 (m = 16, over d2, u = lane >> 2), stage 4 (m = 64, over d3, u = (lane >> 2) + 16 d2)
#pragma unroll
  for (int d3 = 0; d3 < 4; d3++) {
    float2 F[4] = {v[4 * d3], v[4 * d3 + 1], v[4 * d3 + 2], v[4 * d3 + 3]};
    bfly4(F, 1, w.s3[0], w.s3[1], w.s3[2]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[4 * d3 + u] = F[u];
  }
#pragma unroll
  for (int d2 = 0; d2 < 4; d2++) {
    float2 F[4] = {v[d2], v[d2 + 4], v[d2 + 8], v[d2 + 12]};
    const int u16 = lane >> 2;
    bfly4(F, 1, tb.t4[d2][0][u16], tb.t4[d2][1][u16], tb.t4[d2][2][u16]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[d2 + 4 * u] = F[u];
  }
  wfft::wsync();
  // Y -> Z
  {
    float2 *wr = R + (lane >> 2) + 260 * (lane & 3);  // + 16 d2 + 64 d3
#pragma unroll
    for (int r = 0; r < 16; r++) wr[16 * (r & 3) + 64 * (r >> 2)] = v[r];
  }
  wfft::wsync();
  {
    const float2 *rd = R + lane;  // + 64 d3 + 260 d4
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = rd[64 * (r & 3) + 260 * (r >> 2)];
  }
  // stage 5 (m = 256, over d4, u = lane + 64 d3)
#pragma unroll
  for (int d3 = 0; d3 < 4; d3++) {
    float2 F[4] = {v[d3], v[d3 + 4], v[d3 + 8], v[d3 + 12]};
    bfly4(F, 1, tb.t5[d3][0][lane], tb.t5[d3][1][lane], tb.t5[d3][2][lane]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[d3 + 4 * u] = F[u];
  }
  wfft::wsync();
  // natural order into the region (bins 64 r + lane), then kiss_fftr's
  // split for the bins the bands use, magnitudes, band sums in bin order
#pragma unroll
  for (int r = 0; r < 16; r++) R[64 * r + lane] = v[r];
  wfft::wsync();
  const int nc = 1024;
  for (int k = lo + lane; k <= hi; k += 64) {
    float re, imv;
    if (k == 0) {
      re = R[0].x + R[0].y;
      imv = 0;
    } else if (k == nc) {
      re = R[0].x - R[0].y;
      imv = 0;
    } else {
      const int kk = (k < nc / 2) ? k : nc - k;
      const float2 fpk = R[kk];
      const float2 fpnk = make_float2(R[nc - kk].x, -R[nc - kk].y);
      const float2 f1k = cadd(fpk, fpnk), f2k = csub(fpk, fpnk);
      const float2 tw2 = cmul(f2k, sup[kk - 1]);
      if (k < nc / 2) {
        re = (f1k.x + tw2.x) * ((float).5);
        imv = (f1k.y + tw2.y) * ((float).5);
      } else {
        re = (f1k.x - tw2.x) * ((float).5);
        imv = (tw2.y - f1k.y) * ((float).5);
      }
    }
    const float r2 = re * re, i2 = imv * imv;
    mag[k - lo] = sqrtf(r2 + i2) * P->norm_b;
  }
  wfft::wsync();
  float acc = 0.0f;
  if (lane < nb)
    for (int k = a.band_lo[lane]; k <= a.band_hi[lane]; k++) acc += mag[k - lo];
  wfft::wsync();
  return acc;
}

__global__ void __launch_bounds__(64 * kWNW, kWOcc) k_fftbw(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 Rg[kWNW][kFbSlots];
  __shared__ float mg[kWNW][kFbMag];
  __shared__ FbTabs tb;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const Plan *__restrict__ P = a.plan;
  fftb_tabs_load(tb, P, tid, 64 * kWNW);
  __syncthreads();
  float2 *R = Rg[wv];
  float *mag = mg[wv];
  const int C = a.n_channels, nb = a.n_bands;
  const long long items = (long long)a.n_streams * a.wmax * C;
  // static assignment: most (stream, slot) items are empty slots, and a queue
  // atomic per item costs more than the skip
  const long long nw = (long long)gridDim.x * kWNW;
  for (long long it = (long long)blockIdx.x * kWNW + wv; it < items; it += nw) {
    const int c = (int)(it % C);
    const long long sj = it / C;
    const int s = (int)(sj / a.wmax), j = (int)(sj - (long long)s * a.wmax);
    const int t = a.win_tick[(size_t)s * a.wmax + j];
    if (t < 0) continue;
    const long long wstart = a.win_start[(size_t)s * a.wmax + j];
    const float *ring = a.ring + ((size_t)s * C + c) * a.ring_len;
    // layout X: register r = d1 + 4 d0 holds packed input k = lane + 64 r;
    // ring positions: one 64-bit remainder per item, then 2k + 1 < 2048 <=
    // ring_len needs at most one wrap
    const int rl = a.ring_len, w0 = (int)(wstart % rl);
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int k = lane + 64 * r;
      int i0 = w0 + 2 * k;
      i0 -= (i0 >= rl) ? rl : 0;
      int i1 = i0 + 1;
      i1 -= (i1 >= rl) ? rl : 0;
      const float t0 = ring[i0] * P->hannb[2 * k];
      const float t1 = ring[i1] * P->hannb[2 * k + 1];
      v[r] = make_float2(t0, t1);
    }
    const float band = fftb_bands(v, R, mag, tb, a, lane);
    if (lane < nb) a.out_band[(((size_t)t * a.n_streams + s) * C + c) * nb + lane] = band;
  }
}

// ---------------------------------------------------------------------------
// k_olafb (fft_size 2048, C <= 4): k_ola + k_winmeta + k_fftbw in one kernel
// (BASELINE configs[4]'s fusion of the synthesis tail: overlap-add ->
// 480 -> 2048 re-block -> FFT B -> band sums, VAD.zig:298-348,
// PipelineFFT.zig:88-112).  A workgroup takes 4 / C streams, wave = (stream,
// channel).  The wave walks its channel's ticks: overlap-add of the ys rows
// (the next tick's rows load during this tick), the denoised samples go
// straight into the wave's LDS window (the current FFT-B window, VAD.zig's
// fft_input_buffer), and when a tick completes the window the wave runs FFT B
// on it in place (fftb_bands) -- the re-block ring in HBM only carries the
// partial window from one push to the next (<= 2047 samples per channel
// instead of every sample written and read back).  The window bookkeeping of
// k_winmeta (completion, share-weighted volume ratio, window vad) runs on
// every wave of the stream identically; channel 0 writes it.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64 * kWNW, kWOcc) k_olafb(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 Rg[kWNW][kFbSlots];  // window samples, then the FFT exchanges
  __shared__ float mg[kWNW][kFbMag];
  __shared__ float ovg[kWNW][kFrame];  // a completing tick's samples past the window
  __shared__ FbTabs tb;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const Plan *__restrict__ P = a.plan;
  fftb_tabs_load(tb, P, tid, 64 * kWNW);
  __syncthreads();
  constexpr int FB = 2048;
  float *ov = ovg[wv];
  static_assert(kFbSlots * 2 >= FB, "window fits the exchange region");
  float2 *R = Rg[wv];
  float *W = reinterpret_cast<float *>(R);
  float *mag = mg[wv];
  const int C = a.n_channels, nb = a.n_bands, B = a.n_streams, V = a.V;
  const int G = kWNW / C;  // streams per workgroup item
  // wave-uniform bookkeeping in scalar registers (the transform needs the VGPRs)
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int sw = wvu / C, c = wvu - sw * C;
  const float kInv = a.raw_s16 ? 1.0f : 1.0f / (float)32767;
  const int rl = a.ring_len;
  for (int sb = blockIdx.x * G; sb < B; sb += gridDim.x * G) {
    const int s = sb + sw;
    const bool on = sw < G && s < B;
    const int nt = __builtin_amdgcn_readfirstlane(on ? ticks_of(a, s) : 0);
    float *stp = a.state + (size_t)(on ? s : 0) * st::kWords;
    int fd0 = 0;
    float vol = 0;
    if (nt > 0) {
      fd0 = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int *>(stp)[st::kFramesDone]);
      vol = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(stp[st::kVolAcc])));
    }
    // the partial window carried from the previous push: samples [ws, fd0 * 480)
    long long ws = (long long)fd0 * kFrame / FB * FB;
    const float *ring = a.ring + ((size_t)(on ? s : 0) * C + c) * rl;
    if (nt > 0) {
      const int ncarry = (int)((long long)fd0 * kFrame - ws);
      const int r0 = (int)(ws % rl);
      for (int i = lane; i < ncarry; i += 64) {
        int ri = r0 + i;
        ri -= ri >= rl ? rl : 0;
        W[i] = ring[ri];
      }
    }
    // the stream's synthesis memory is read (tick 0, channel 0) before the
    // last channel's wave replaces it
    __syncthreads();
    if (nt > 0) {
      const float *ysr = a.ys + (size_t)s * V * kWin;
      // lane l < 60 owns samples 8 l .. 8 l + 7 of each tick
      const bool sl = lane < 60;
      const int q = 8 * lane;
      auto load = [&](int t, float4 (&cur)[2], float4 (&prv)[2]) {
        const int v = t * C + c;
        const float *cp = ysr + (size_t)v * kWin + q;
        const float *pp = v == 0 ? stp + st::kSyn + q : ysr + (size_t)(v - 1) * kWin + kFrame + q;
        if (sl) {
          cur[0] = *reinterpret_cast<const float4 *>(cp);
          cur[1] = *reinterpret_cast<const float4 *>(cp + 4);
          prv[0] = *reinterpret_cast<const float4 *>(pp);
          prv[1] = *reinterpret_cast<const float4 *>(pp + 4);
        }
      };
      float4 cn[2] = {}, pn[2] = {};
      load(0, cn, pn);
      // per-tick inputs of the window bookkeeping, 64 ticks at a time: lane l
      // holds tick t0 + l's volume ratio and vad_low (VAD.zig:284-293), read
      // per tick with a wave-uniform readlane (no global load waits per tick)
      float tk_ratio = 0, tk_vad = 1;
      for (int t = 0; t < nt; t++) {
        if ((t & 63) == 0) {
          const int tl = t + lane;
          tk_ratio = 0;
          tk_vad = 1;
          if (tl < nt) {
            tk_ratio = a.ratio[(size_t)tl * B + s];
            for (int cc = 0; cc < C; cc++) {
              const float vv = a.vadf[(size_t)s * V + tl * C + cc];
              if (vv < tk_vad) tk_vad = vv;
            }
          }
        }
        float4 cur[2] = {cn[0], cn[1]}, prv[2] = {pn[0], pn[1]};
        const long long p0 = (long long)(fd0 + t) * kFrame;
        const int off = (int)(p0 - ws);  // window position of the tick's first sample
        const bool complete = off + kFrame >= FB;
        // the next tick's rows load now, or after this tick's FFT B (the
        // transform needs the registers)
        if (!complete && t + 1 < nt) load(t + 1, cn, pn);
        float o[8];
        o[0] = (cur[0].x + prv[0].x) * kInv;
        o[1] = (cur[0].y + prv[0].y) * kInv;
        o[2] = (cur[0].z + prv[0].z) * kInv;
        o[3] = (cur[0].w + prv[0].w) * kInv;
        o[4] = (cur[1].x + prv[1].x) * kInv;
        o[5] = (cur[1].y + prv[1].y) * kInv;
        o[6] = (cur[1].z + prv[1].z) * kInv;
        o[7] = (cur[1].w + prv[1].w) * kInv;
        const size_t ot = (size_t)t * B + s;
        if (a.out_den && sl) {
          float4 *dp = reinterpret_cast<float4 *>(a.out_den + (ot * C + c) * kFrame + q);
          dp[0] = make_float4(o[0], o[1], o[2], o[3]);
          dp[1] = make_float4(o[4], o[5], o[6], o[7]);
        }
        // samples inside the current window
        if (sl) {
#pragma unroll
          for (int e = 0; e < 8; e++)
            if (off + q + e < FB) W[off + q + e] = o[e];
        }
        // vad_low and the window bookkeeping (VAD.zig:298-348)
        const float vad_low = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tk_vad), t & 63));
        const float ratio = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tk_ratio), t & 63));
        if (complete) {
          const int r = FB - off;
          vol += ratio * ((float)r / (float)FB);
          if (c == 0 && lane == 0) {
            a.out_win_ratio[ot] = vol;
            a.out_win_vad[ot] = vad_low;
          }
          vol = 0;
          if (kFrame - r > 0) vol += ratio * ((float)(kFrame - r) / (float)FB);
          // the tick's samples past the window wait in ov during FFT B
          if (sl) {
#pragma unroll
            for (int e = 0; e < 8; e++)
              if (off + q + e >= FB) ov[off + q + e - FB] = o[e];
          }
          // FFT B of the completed window, in place
          wfft::wsync();
          float2 v[16];
#pragma unroll
          for (int rr = 0; rr < 16; rr++) {
            const int k = lane + 64 * rr;
            const float2 x = *reinterpret_cast<const float2 *>(W + 2 * k);
            v[rr] = make_float2(x.x * P->hannb[2 * k], x.y * P->hannb[2 * k + 1]);
          }
          const float band = fftb_bands(v, R, mag, tb, a, lane);
          if (lane < nb) a.out_band[(ot * C + c) * nb + lane] = band;
          // they start the next window
          for (int i = lane; i < off + kFrame - FB; i += 64) W[i] = ov[i];
          ws += FB;
          if (t + 1 < nt) load(t + 1, cn, pn);
        } else {
          vol += ratio * ((float)kFrame / (float)FB);
          if (c == 0 && lane == 0) {
            a.out_win_ratio[ot] = 0.0f;
            a.out_win_vad[ot] = 0.0f;
          }
          if (lane < nb) a.out_band[(ot * C + c) * nb + lane] = 0.0f;
        }
        if (c == 0 && lane == 0) {
          a.out_vad[ot] = vad_low;
          a.out_win_flag[ot] = complete ? 1 : 0;
        }
      }
      // the partial window goes back to the ring for the next push
      wfft::wsync();
      const int ncarry = (int)((long long)(fd0 + nt) * kFrame - ws);
      const int r0 = (int)(ws % rl);
      float *rw = a.ring + ((size_t)s * C + c) * rl;
      for (int i = lane; i < ncarry; i += 64) {
        int ri = r0 + i;
        ri -= ri >= rl ? rl : 0;
        rw[ri] = W[i];
      }
    }
    __syncthreads();  // every wave of the stream has read its state
    if (nt > 0) {
      if (c == 0 && lane == 0) {
        reinterpret_cast<int *>(stp)[st::kFramesDone] = fd0 + nt;
        stp[st::kVolAcc] = vol;
      }
      if (c == C - 1) {  // synthesis memory = second half of the stream's last frame
        const float4 *yl =
            reinterpret_cast<const float4 *>(a.ys + ((size_t)s * V + (size_t)nt * C - 1) * kWin + kFrame);
        float4 *dst = reinterpret_cast<float4 *>(stp + st::kSyn);
        for (int i = lane; i < kFrame / 4; i += 64) dst[i] = yl[i];
      }
    }
  }
}

namespace {
// workgroups of a kernel one CU holds (occupancy calculator, once per kernel)
template <typename K>
int wave_per_cu(K kernel, int nw = kWNW) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 64 * nw, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  return per_cu;
}
}  // namespace

// n_cu: the CUs the engine's stream may use (all, or its CU mask's)
hipError_t launch_wave(WaveKernel which, const StagedArgs &a, int n_cu, hipStream_t stream) {
  static const int p_fftA = wave_per_cu(k_fftAw), p_pspec = wave_per_cu(k_pspecw, kPNW), p_synth = wave_per_cu(k_synthw, kSNW),
                   p_fftb = wave_per_cu(k_fftbw), p_olafb = wave_per_cu(k_olafb);
  // k_olafb: at most 2 of its 3 resident workgroups per CU.  Beside the next
  // push's k_fftAw (which starts ~10 us after it) it then leaves that kernel
  // a workgroup slot per CU from the start, and its 1 024 items (2 048 stereo
  // streams) run as two even rounds instead of 1.33: k_olafb 0.44 -> 0.40 ms,
  // k_fftAw 0.75 -> 0.72, push 4.759 -> 4.745 ms (three interleaved pairs;
  // measured with the timed pushes' dispatch race gone, §8 r5)
  const int g_fftA = p_fftA * n_cu, g_pspec = p_pspec * n_cu, g_synth = p_synth * n_cu, g_fftb = p_fftb * n_cu,
            g_olafb = std::min(p_olafb, 2) * n_cu;
  if (which == kWaveOlaFb) {
    const int G = kWNW / a.n_channels;
    hipLaunchKernelGGL(k_olafb, dim3((unsigned)std::min<long long>((a.n_streams + G - 1) / G, g_olafb)), dim3(64 * kWNW),
                       0, stream, a);
    return hipGetLastError();
  }
  if (which == kWaveFftB) {
    const long long items = (long long)a.n_streams * a.wmax * a.n_channels;
    hipLaunchKernelGGL(k_fftbw, dim3((unsigned)std::min<long long>(std::max<long long>((items + kWNW - 1) / kWNW, 1), g_fftb)),
                       dim3(64 * kWNW), 0, stream, a);
    return hipGetLastError();
  }
  const long long batches = ((long long)a.n_streams * a.V + kWB - 1) / kWB;
  // dynamic mode: queue x is served by the blocks with blockIdx % 8 == x, so
  // the grid covers min(batches, 8) blocks at least; static mode: batches /
  // kWNW blocks suffice
  auto grid = [&](int resident, int nw = kWNW) {
    const long long want = ((kWaveStatic >> which) & 1) ? (batches + nw - 1) / nw : batches;
    return dim3((unsigned)std::min<long long>(std::max<long long>(want, 1), resident));
  };
  if (which == kWaveFftA)
    hipLaunchKernelGGL(k_fftAw, grid(g_fftA), dim3(64 * kWNW), 0, stream, a);
  else if (which == kWavePspec)
    hipLaunchKernelGGL(k_pspecw, grid(g_pspec, kPNW), dim3(64 * kPNW), 0, stream, a);
  else
    hipLaunchKernelGGL(k_synthw, grid(g_synth, kSNW), dim3(64 * kSNW), 0, stream, a);
  return hipGetLastError();
}

}  // namespace fvad
