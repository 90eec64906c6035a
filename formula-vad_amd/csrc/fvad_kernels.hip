// MI355X (gfx950) HIP kernels for Formula-VAD's per-frame hot path.
//
//   k_prep   lane-per-stream: Denoiser.zig s16 scaling, the rnnoise high-pass
//            biquad (serial IIR with double intermediates), and
//            VAD.preAnalyzeSegment's per-channel RMS / volume ratio
//            (VAD.zig:253-272, audio_utils.zig:14-24).  One lane owns one
//            stream, so every serial recurrence runs on all 64 lanes.
//   k_frame  workgroup-per-stream (NT threads): the rest of
//            rnnoise_process_frame (FFT A analysis, band energies, pitch
//            downsample/LPC/xcorr/remove_doubling, pitch spectrum, features,
//            GRU stack, pitch filter, gains, inverse FFT + overlap-add) for
//            every channel of every tick in stream order on ONE shared state
//            (VAD.zig:274-296), then the 480 -> fft_size re-block with the
//            share-weighted volume ratio (VAD.zig:298-348) and, when a window
//            completes, FFT B (kissfft real FFT), magnitude and band sums
//            (FFT.zig:70-98, PipelineFFT.zig:88-112).
//
// Numerics: compiled with -ffp-contract=off and correctly rounded f32
// divide/sqrt; every expression reproduces the C promotion rules and the
// evaluation order of the restated sources so results are bit-identical to
// the CPU oracle.  Per-element parallel work (FFT
// butterflies, windowing, interpolation, xcorr lags, GRU neurons) is spread
// over lanes; every sequential sum keeps its C order on one lane.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cmath>

#include "fvad_internal.h"
#include "fvad_kernels.h"
#include "fvad_device.h"

namespace fvad {

// ---------------------------------------------------------------------------
// k_prep
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_prep(PrepArgs a) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= a.n_streams) return;
  const int nt = a.ticks_valid ? a.ticks_valid[s] : a.n_ticks;
  float *stp = a.state + (size_t)s * st::kWords;
  float mem0 = stp[st::kHp], mem1 = stp[st::kHp + 1];
  const float b0 = -2.0f, b1 = 1.0f, a0 = -1.99599f, a1 = 0.99600f;  // denoise.c b_hp / a_hp
  const float scalar = (float)32767;                                 // Denoiser.zig:72
  const int C = a.n_channels;
  for (int t = 0; t < nt; t++) {
    float vmin = 1, vmax = 0;
    for (int c = 0; c < C; c++) {
      const size_t base = (((size_t)t * a.n_streams + s) * C + c) * kFrame;
      const float4 *in4 = reinterpret_cast<const float4 *>(a.pcm + base);
      float4 *out4 = reinterpret_cast<float4 *>(a.xbuf + base);
      float sum = 0;
      for (int i4 = 0; i4 < kFrame / 4; i4++) {
        const float4 v = in4[i4];
        float vv[4] = {v.x, v.y, v.z, v.w};
        float yy[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const float v0 = vv[k];
          sum += v0 * v0;                    // rmsVolume: sequential f32 sum
          const float xi = a.raw_s16 ? v0 : v0 * scalar;  // normalizedPcmToRnnoise
          const float yi = xi + mem0;        // biquad (denoise.c)
          mem0 = (float)(mem1 + (b0 * (double)xi - a0 * (double)yi));
          mem1 = (float)(b1 * (double)xi - a1 * (double)yi);
          yy[k] = yi;
        }
        out4[i4] = make_float4(yy[0], yy[1], yy[2], yy[3]);
      }
      const float vol = sqrtf(sum / (float)kFrame);
      if (vol < vmin) vmin = vol;
      if (vol > vmax) vmax = vol;
    }
    a.ratio[(size_t)t * a.n_streams + s] = (vmax == 0) ? 0 : vmin / vmax;
  }
  stp[st::kHp] = mem0;
  stp[st::kHp + 1] = mem1;
}

// ---------------------------------------------------------------------------
// k_frame helpers
// ---------------------------------------------------------------------------
// LDS layout (floats).  Work area doubles as the 960/1024-point complex FFT
// buffer, the pitch-analysis scratch and the pitch spectrum P.
namespace lds {
constexpr int kPb = 0;                                   // pitch_buf[1728]
constexpr int kSyn = kPb + fvad::kPitchBuf;              // synthesis_mem[480]
constexpr int kWork = kSyn + fvad::kFrame;               // 2048 floats (1024 complex)
constexpr int kX = kWork + 2048;                         // X[481] complex
constexpr int kEx = kX + 2 * fvad::kFreq + 2;            // Ex[22]
constexpr int kEp = kEx + 24;
constexpr int kExp = kEp + 24;
constexpr int kLy = kExp + 24;
constexpr int kFeat = kLy + 24;                          // features[42]
constexpr int kG = kFeat + 44;                           // gains[22]
constexpr int kR = kG + 24;                              // pitch-filter r[22]
constexpr int kNorm = kR + 24;
constexpr int kNewE = kNorm + 24;
constexpr int kLastG = kNewE + 24;
constexpr int kCepsMem = kLastG + 24;                    // cepstral_mem[8][22]
constexpr int kGv = kCepsMem + fvad::kCeps * fvad::kBands;  // vad_gru_state[128]
constexpr int kGn = kGv + 128;
constexpr int kGd = kGn + 128;
constexpr int kDout = kGd + 128;                         // dense_out[128]
constexpr int kRin = kDout + 128;                        // concatenated GRU input[384]
constexpr int kZr = kRin + 384;                          // z,r gates[256]
constexpr int kH = kZr + 256;                            // h[128]
constexpr int kMisc = kH + 128;                          // float scratch[64]
constexpr int kIMisc = kMisc + 64;                       // int scratch[32]
constexpr int kRd = kIMisc + 32;                         // remove_doubling partials [64]
constexpr int kMag = kRd + 64;                           // FFT-B magnitudes of reported bins [256]
constexpr int kTotal = kMag + 256;
// work-area sub-buffers during pitch analysis
constexpr int kXlpBuf = kWork;                           // raw x_lp[864]
constexpr int kXf = kWork + fvad::kXlp;                  // FIR-filtered x_lp[864]
constexpr int kXc = kWork + 2 * fvad::kXlp;              // xcorr[294]
constexpr int kYy = kWork;                               // yy_lookup[385] (reuses raw x_lp)
constexpr int kSyyC = kWork;                             // coarse Syy sequence[147] (raw x_lp is dead)
constexpr int kSyyF = kWork + 160;                       // fine Syy sequence[294]
static_assert(kXc + 294 <= kWork + 2048, "pitch scratch exceeds the work area");
static_assert(kTotal * 4 <= 32768, "LDS budget");
}  // namespace lds

// misc slots
namespace ms {
constexpr int kAc = 0;      // ac[5]
constexpr int kLpc2 = 8;    // lpc2[5]
constexpr int kXx = 16;     // remove_doubling xx
constexpr int kXy = 17;     // xy at T0
constexpr int kPg = 18;     // last_gain; [19] holds the tentative gain
constexpr int kMind = 24;   // mindist[8]
constexpr int kXc3 = 32;    // remove_doubling final xcorr[3]
constexpr int kVadCh = 40;  // per-channel vad[8]
constexpr int kFine = 48;   // fine-search xcorr of the 10 candidate lags
}  // namespace ms
namespace is {
constexpr int kBest0 = 0, kBest1 = 1, kPitch = 2, kT0 = 3, kT = 4, kSilence = 5, kMemId = 6, kLastPeriod = 7,
              kFineBase = 8;  // [8..17] candidate-lane valid flags
}


// Diagnostic build only (-DFVAD_STAMPS): per-phase s_memtime accounting on
// thread 0, written to a debug buffer that no other code reads.
#ifdef FVAD_STAMPS
#define STAMP(id)                                          \
  do {                                                     \
    if (tid == 0) {                                        \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
      stamp_acc[id] += t_ - stamp_last;                    \
      stamp_last = t_;                                     \
    }                                                      \
  } while (0)
#else
#define STAMP(id) \
  do {            \
  } while (0)
#endif
#ifdef FVAD_STAMPS
constexpr int kStamps = 24;
#endif

// ---------------------------------------------------------------------------
// k_frame
// ---------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(NT) k_frame(FrameArgs a) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  const int tid = threadIdx.x;
  const int s = blockIdx.x;
  if (s >= a.n_streams) return;
  const int nt = a.ticks_valid ? a.ticks_valid[s] : a.n_ticks;
  if (nt <= 0) return;
#ifdef FVAD_STAMPS
  unsigned long long stamp_acc[kStamps];
  for (int i = 0; i < kStamps; i++) stamp_acc[i] = 0;
  unsigned long long stamp_last = __builtin_amdgcn_s_memtime();
#endif
  const Plan *__restrict__ P = a.plan;
  const float2 *__restrict__ tw = reinterpret_cast<const float2 *>(P->tw960);
  const float *__restrict__ hw = P->half_window;
  const float *__restrict__ tt = P->tansig;
  const DevModel &M = *a.model;
  const int C = a.n_channels;
  float *stp = a.state + (size_t)s * st::kWords;
  int *istp = reinterpret_cast<int *>(stp);
  float *pb = L + lds::kPb;
  float *syn = L + lds::kSyn;
  float2 *W = reinterpret_cast<float2 *>(L + lds::kWork);
  float2 *X = reinterpret_cast<float2 *>(L + lds::kX);
  float *Ex = L + lds::kEx, *Ep = L + lds::kEp, *Exp = L + lds::kExp, *Ly = L + lds::kLy;
  float *feat = L + lds::kFeat, *g = L + lds::kG, *rr = L + lds::kR, *nrm = L + lds::kNorm;
  float *newE = L + lds::kNewE, *lastg = L + lds::kLastG, *ceps = L + lds::kCepsMem;
  float *gv = L + lds::kGv, *gn = L + lds::kGn, *gd = L + lds::kGd;
  float *dout = L + lds::kDout, *rin = L + lds::kRin, *zr = L + lds::kZr, *hb = L + lds::kH;
  float *misc = L + lds::kMisc;
  int *im = reinterpret_cast<int *>(L + lds::kIMisc);
  float *rd = L + lds::kRd;
  float *mag = L + lds::kMag;
  float *xlp = L + lds::kXlpBuf, *xf = L + lds::kXf, *xc = L + lds::kXc, *yyl = L + lds::kYy;

  // ---- load persistent state into LDS
  for (int i = tid; i < kPitchBuf; i += NT) pb[i] = stp[st::kPitch + i];
  for (int i = tid; i < kFrame; i += NT) syn[i] = stp[st::kSyn + i];
  for (int i = tid; i < kCeps * kBands; i += NT) ceps[i] = stp[st::kCepsMem + i];
  for (int i = tid; i < kBands; i += NT) lastg[i] = stp[st::kLastG + i];
  for (int i = tid; i < kMaxNeurons; i += NT) {
    gv[i] = stp[st::kVadGru + i];
    gn[i] = stp[st::kNoiseGru + i];
    gd[i] = stp[st::kDenGru + i];
  }
  if (tid == 0) {
    im[is::kMemId] = istp[st::kMemId];
    im[is::kLastPeriod] = istp[st::kLastPeriod];
    misc[ms::kPg] = stp[st::kLastGain];
  }
  int frames_done = istp[st::kFramesDone];
  float vol_acc = stp[st::kVolAcc];
  const float scale = 1.f / 960;
  const int FB = P->nfft_b, ring_len = a.ring_len;
  __syncthreads();
      STAMP(0);

  for (int t = 0; t < nt; t++) {
    for (int c = 0; c < C; c++) {
      const float *xin = a.xbuf + (((size_t)t * a.n_streams + s) * C + c) * kFrame;
      // ---- pitch_buf shift by 480, append x (RNN_MOVE + RNN_COPY)
      {
        float tmp[(kPitchBuf - kFrame + NT - 1) / NT];
#pragma unroll
        for (int r = 0; r < (kPitchBuf - kFrame + NT - 1) / NT; r++) {
          const int k = tid + r * NT;
          if (k < kPitchBuf - kFrame) tmp[r] = pb[kFrame + k];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < (kPitchBuf - kFrame + NT - 1) / NT; r++) {
          const int k = tid + r * NT;
          if (k < kPitchBuf - kFrame) pb[k] = tmp[r];
        }
        for (int i = tid; i < kFrame; i += NT) pb[kPitchBuf - kFrame + i] = xin[i];
      }
      __syncthreads();
      STAMP(1);
      // ---- frame_analysis: [analysis_mem | x] = pb[768..1728), window, FFT, Ex
      for (int i = tid; i < kWin; i += NT) {
        float v = pb[kPitchBuf - kWin + i];
        v *= (i < kFrame) ? hw[i] : hw[kWin - 1 - i];
        const int d = P->bitrev960[i];
        W[d] = make_float2(scale * v, scale * 0.0f);
      }
      __syncthreads();
      STAMP(1);
      fft960_stages<NT>(W, tw, tid);
      for (int k = tid; k < kFreq; k += NT) X[k] = W[k];
      __syncthreads();
      STAMP(2);
      if (tid < kBands) Ex[tid] = band_sum(X, X, P, tid);
      // ---- pitch_downsample: x_lp, autocorr, LPC, FIR5
      for (int i = tid; i < kXlp; i += NT) {
        xlp[i] = (i == 0) ? .5f * (.5f * (pb[1]) + pb[0]) : .5f * (.5f * (pb[2 * i - 1] + pb[2 * i + 1]) + pb[2 * i]);
      }
      __syncthreads();
      STAMP(3);
      if (tid < 5) {
        const int k = tid;
        const int fastN = kXlp - 4;
        float acc = 0;
#pragma unroll 8
        for (int i = 0; i < fastN; i++) acc = acc + xlp[i] * xlp[i + k];
        float d = 0;
        for (int i = k + fastN; i < kXlp; i++) d = d + xlp[i] * xlp[i - k];
        misc[ms::kAc + k] = acc + d;
      }
      __syncthreads();
      STAMP(4);
      if (tid == 0) {
        float ac[5];
        for (int i = 0; i < 5; i++) ac[i] = misc[ms::kAc + i];
        ac[0] *= 1.0001f;
        for (int i = 1; i <= 4; i++) ac[i] -= ac[i] * (.008f * i) * (.008f * i);
        float lpc[4] = {0, 0, 0, 0};
        float error = ac[0];
        if (ac[0] != 0) {
          for (int i = 0; i < 4; i++) {
            float r_acc = 0;
            for (int j = 0; j < i; j++) r_acc += lpc[j] * ac[i - j];
            r_acc += ac[i + 1];
            const float r = -r_acc / error;
            lpc[i] = r;
            for (int j = 0; j < (i + 1) >> 1; j++) {
              const float tmp1 = lpc[j], tmp2 = lpc[i - 1 - j];
              lpc[j] = tmp1 + r * tmp2;
              lpc[i - 1 - j] = tmp2 + r * tmp1;
            }
            error = error - (r * r) * error;
            if (error < .001f * ac[0]) break;
          }
        }
        float tmp = 1.0f;
        for (int i = 0; i < 4; i++) {
          tmp = .9f * tmp;
          lpc[i] = lpc[i] * tmp;
        }
        const float c1 = .8f;
        misc[ms::kLpc2 + 0] = lpc[0] + .8f;
        misc[ms::kLpc2 + 1] = lpc[1] + c1 * lpc[0];
        misc[ms::kLpc2 + 2] = lpc[2] + c1 * lpc[1];
        misc[ms::kLpc2 + 3] = lpc[3] + c1 * lpc[2];
        misc[ms::kLpc2 + 4] = c1 * lpc[3];
      }
      __syncthreads();
      STAMP(5);
      {
        const float n0 = misc[ms::kLpc2 + 0], n1 = misc[ms::kLpc2 + 1], n2 = misc[ms::kLpc2 + 2],
                    n3 = misc[ms::kLpc2 + 3], n4 = misc[ms::kLpc2 + 4];
        for (int i = tid; i < kXlp; i += NT) {
          const float m0 = i >= 1 ? xlp[i - 1] : 0.0f, m1 = i >= 2 ? xlp[i - 2] : 0.0f,
                      m2 = i >= 3 ? xlp[i - 3] : 0.0f, m3 = i >= 4 ? xlp[i - 4] : 0.0f,
                      m4 = i >= 5 ? xlp[i - 5] : 0.0f;
          float sum = xlp[i];
          sum = sum + n0 * m0;
          sum = sum + n1 * m1;
          sum = sum + n2 * m2;
          sum = sum + n3 * m3;
          sum = sum + n4 * m4;
          xf[i] = sum;
        }
      }
      __syncthreads();
      STAMP(6);
      // ---- pitch_search: coarse xcorr (4x decimation) on 147 lanes.  The
      //      find_best_pitch energy recurrences (Syy) depend only on y, so
      //      two more lanes produce the per-lag Syy sequences meanwhile.
      const float *xl = xf + (kPitchMax >> 1);  // x_lp = pitch_buf_lp + 384
      float *syy_c = L + lds::kSyyC, *syy_f = L + lds::kSyyF;
      if (tid < 147) {
        const int k = tid;
        float acc = 0;
#pragma unroll 8
        for (int j = 0; j < 240; j++) acc = acc + xl[2 * j] * xf[2 * (j + k)];
        xc[k] = acc;
      } else if (tid == 160) {
        syy_sequence(xf, 2, 240, 147, syy_c);
      } else if (tid == 192) {
        syy_sequence(xf, 1, 480, 294, syy_f);
      }
      __syncthreads();
      STAMP(7);
      if (tid == 0) {
        int best[2] = {0, 1};
        float bn0 = -1, bn1 = -1, bd0 = 0, bd1 = 0;
#pragma unroll 4
        for (int i = 0; i < 147; i++) best_pitch_visit(xc[i], syy_c[i], i, bn0, bn1, bd0, bd1, best);
        im[is::kBest0] = best[0];
        im[is::kBest1] = best[1];
      }
      __syncthreads();
      STAMP(8);
      {
        // fine search: only lags within +-2 of 2*best[0] or 2*best[1] are non-zero
        const int bp0 = im[is::kBest0], bp1 = im[is::kBest1];
        for (int i = tid; i < 294; i += NT) xc[i] = 0;
        const int lane = tid;
        if (lane < 10) {
          const int i = (lane < 5 ? 2 * bp0 : 2 * bp1) - 2 + (lane % 5);
          const bool dup = lane >= 5 && abs(i - 2 * bp0) <= 2;  // also in the first window
          if (i >= 0 && i < 294 && !dup) {
            float sum = 0;
#pragma unroll 8
            for (int j = 0; j < 480; j++) sum = sum + xl[j] * xf[i + j];
            im[is::kFineBase + lane] = 1;
            misc[ms::kFine + lane] = (-1 > sum) ? -1 : sum;
          } else {
            im[is::kFineBase + lane] = 0;
          }
        }
      }
      __syncthreads();
      STAMP(9);
      if (tid < 10 && im[is::kFineBase + tid]) {
        const int bp0 = im[is::kBest0], bp1 = im[is::kBest1];
        const int i = (tid < 5 ? 2 * bp0 : 2 * bp1) - 2 + (tid % 5);
        xc[i] = misc[ms::kFine + tid];
      }
      __syncthreads();
      if (tid == 0) {
        const int bp0 = im[is::kBest0], bp1 = im[is::kBest1];
        int best[2] = {0, 1};
        float bn0 = -1, bn1 = -1, bd0 = 0, bd1 = 0;
        // visit the union of the two candidate windows in increasing lag order
        int w0lo = 2 * bp0 - 2, w0hi = 2 * bp0 + 2, w1lo = 2 * bp1 - 2, w1hi = 2 * bp1 + 2;
        if (w1lo < w0lo) {
          int t0 = w0lo, t1 = w0hi;
          w0lo = w1lo;
          w0hi = w1hi;
          w1lo = t0;
          w1hi = t1;
        }
        for (int i = max(0, w0lo); i <= min(293, w0hi); i++)
          best_pitch_visit(xc[i], syy_f[i], i, bn0, bn1, bd0, bd1, best);
        for (int i = max(max(0, w1lo), w0hi + 1); i <= min(293, w1hi); i++)
          best_pitch_visit(xc[i], syy_f[i], i, bn0, bn1, bd0, bd1, best);
        int offset;
        if (best[0] > 0 && best[0] < 294 - 1) {
          const float aa = xc[best[0] - 1], bb = xc[best[0]], cc = xc[best[0] + 1];
          if ((cc - aa) > .7f * (bb - aa))
            offset = 1;
          else if ((aa - cc) > .7f * (bb - cc))
            offset = -1;
          else
            offset = 0;
        } else {
          offset = 0;
        }
        const int pitch = 2 * best[0] - offset;
        int T0 = (kPitchMax - pitch) / 2;  // remove_doubling: *T0_ /= 2
        if (T0 >= 384) T0 = 383;
        im[is::kT0] = T0;
      }
      __syncthreads();
      STAMP(10);
      // ---- remove_doubling: independent inner products in parallel
      //   lane 0: xx, xy(T0); lane 1: xx then yy_lookup chain; lanes 2..15: k candidates
      {
        const float *x = xl;  // x += maxperiod (384)
        const int T0 = im[is::kT0];
        if (tid == 0) {
          float xx = 0, xy = 0;
#pragma unroll 8
          for (int i = 0; i < 480; i++) {
            xx = xx + x[i] * x[i];
            xy = xy + x[i] * x[i - T0];
          }
          misc[ms::kXx] = xx;
          misc[ms::kXy] = xy;
        } else if (tid == 1) {
          float xx = 0;
#pragma unroll 8
          for (int i = 0; i < 480; i++) xx = xx + x[i] * x[i];
          float yy = xx;
          yyl[0] = xx;
#pragma unroll 8
          for (int i = 1; i <= 384; i++) {
            yy = yy + x[-i] * x[-i] - x[480 - i] * x[480 - i];
            yyl[i] = (0 > yy) ? 0 : yy;
          }
        } else if (tid >= 2 && tid <= 15) {
          const int k = tid;
          const int T1 = (int)((unsigned)(2 * T0 + k) / (unsigned)(2 * k));
          if (T1 >= 30) {
            int T1b;
            if (k == 2)
              T1b = (T1 + T0 > 384) ? T0 : T0 + T1;
            else
              T1b = (int)((unsigned)(2 * second_check(k) * T0 + k) / (unsigned)(2 * k));
            float s1 = 0, s2 = 0;
#pragma unroll 8
            for (int i = 0; i < 480; i++) {
              s1 = s1 + x[i] * x[i - T1];
              s2 = s2 + x[i] * x[i - T1b];
            }
            rd[2 * k] = s1;
            rd[2 * k + 1] = s2;
          }
        }
      }
      __syncthreads();
      STAMP(11);
      if (tid == 0) {
        const int T0 = im[is::kT0];
        const int prev_period = im[is::kLastPeriod] / 2;
        const float prev_gain = misc[ms::kPg];
        const float xx = misc[ms::kXx];
        float xy = misc[ms::kXy];
        float yy = yyl[T0];
        float best_xy = xy, best_yy = yy;
        float g0 = pitch_gain(xy, xx, yy);
        float gg = g0;
        int T = T0;
        for (int k = 2; k <= 15; k++) {
          const int T1 = (int)((unsigned)(2 * T0 + k) / (unsigned)(2 * k));
          if (T1 < 30) break;
          int T1b;
          if (k == 2)
            T1b = (T1 + T0 > 384) ? T0 : T0 + T1;
          else
            T1b = (int)((unsigned)(2 * second_check(k) * T0 + k) / (unsigned)(2 * k));
          xy = .5f * (rd[2 * k] + rd[2 * k + 1]);
          yy = .5f * (yyl[T1] + yyl[T1b]);
          const float g1 = pitch_gain(xy, xx, yy);
          float cont;
          if (abs(T1 - prev_period) <= 1)
            cont = prev_gain;
          else if (abs(T1 - prev_period) <= 2 && 5 * k * k < T0)
            cont = .5f * prev_gain;
          else
            cont = 0;
          float thresh;
          {
            const float v = .7f * g0 - cont;
            thresh = (.3f > v) ? .3f : v;
          }
          if (T1 < 3 * 30) {
            const float v = .85f * g0 - cont;
            thresh = (.4f > v) ? .4f : v;
          } else if (T1 < 2 * 30) {
            const float v = .9f * g0 - cont;
            thresh = (.5f > v) ? .5f : v;
          }
          if (g1 > thresh) {
            best_xy = xy;
            best_yy = yy;
            T = T1;
            gg = g1;
          }
        }
        best_xy = (0 > best_xy) ? 0 : best_xy;
        float pg;
        if (best_yy <= best_xy)
          pg = 1.0f;
        else
          pg = best_xy / (best_yy + 1);
        if (pg > gg) pg = gg;
        im[is::kT] = T;
        misc[ms::kPg + 1] = pg;  // tentative gain (final after offset)
      }
      __syncthreads();
      STAMP(12);
      if (tid < 3) {
        const float *x = xl;
        const int T = im[is::kT];
        float acc = 0;
#pragma unroll 8
        for (int i = 0; i < 480; i++) acc = acc + x[i] * x[i - (T + tid - 1)];
        misc[ms::kXc3 + tid] = acc;
      }
      __syncthreads();
      if (tid == 0) {
        const float x0 = misc[ms::kXc3], x1 = misc[ms::kXc3 + 1], x2 = misc[ms::kXc3 + 2];
        int offset;
        if ((x2 - x0) > .7f * (x1 - x0))
          offset = 1;
        else if ((x0 - x2) > .7f * (x1 - x2))
          offset = -1;
        else
          offset = 0;
        int pi = 2 * im[is::kT] + offset;
        if (pi < kPitchMin) pi = kPitchMin;
        im[is::kPitch] = pi;
        im[is::kLastPeriod] = pi;
        misc[ms::kPg] = misc[ms::kPg + 1];  // last_gain
      }
      __syncthreads();
      STAMP(13);
      // ---- pitch spectrum P (in W), Ep, Exp
      {
        const int pitch = im[is::kPitch];
        for (int i = tid; i < kWin; i += NT) {
          float v = pb[kPitchBuf - kWin - pitch + i];
          v *= (i < kFrame) ? hw[i] : hw[kWin - 1 - i];
          W[P->bitrev960[i]] = make_float2(scale * v, scale * 0.0f);
        }
      }
      __syncthreads();
      fft960_stages<NT>(W, tw, tid);
      if (tid < kBands)
        Ep[tid] = band_sum(W, W, P, tid);
      else if (tid >= 32 && tid < 32 + kBands)
        Exp[tid - 32] = band_sum(X, W, P, tid - 32);
      __syncthreads();
      STAMP(14);
      if (tid < kBands) {
        Exp[tid] = (float)((double)Exp[tid] / sqrt(.001 + (double)(Ex[tid] * Ep[tid])));
        Ly[tid] = (float)log10(1e-2 + (double)Ex[tid]);
      }
      __syncthreads();
      if (tid < 6) {  // dct(tmp, Exp) -> features[34..39]
        float sum = 0;
#pragma unroll
        for (int j = 0; j < kBands; j++) sum += Exp[j] * P->dct[j * kBands + tid];
        float v = (float)(sum * sqrt(2. / 22));
        if (tid == 0) v = (float)(v - 1.3);
        if (tid == 1) v = (float)(v - 0.9);
        feat[34 + tid] = v;
      } else if (tid == 32) {
        // Ly floor chain and E (sequential over bands)
        float logMax = -2, follow = -2, E = 0;
        for (int i = 0; i < kBands; i++) {
          const float ly0 = Ly[i];
          const double bb = (follow - 1.5 > (double)ly0) ? follow - 1.5 : (double)ly0;
          const double aa = ((double)(logMax - 7) > bb) ? (double)(logMax - 7) : bb;
          const float ly = (float)aa;
          Ly[i] = ly;
          logMax = (logMax > ly) ? logMax : ly;
          follow = (float)((follow - 1.5 > (double)ly) ? follow - 1.5 : (double)ly);
          E += Ex[i];
        }
        im[is::kSilence] = ((double)E < 0.04) ? 1 : 0;
      }
      __syncthreads();
      STAMP(15);
      const bool silence = im[is::kSilence] != 0;
      if (!silence) {
        // ---- features: DCT(Ly), cepstral memory, deltas, spectral variability
        const int memid = im[is::kMemId];
        if (tid < kBands) {
          float sum = 0;
#pragma unroll
          for (int j = 0; j < kBands; j++) sum += Ly[j] * P->dct[j * kBands + tid];
          float v = (float)(sum * sqrt(2. / 22));
          if (tid == 0) v -= 12;
          if (tid == 1) v -= 4;
          ceps[memid * kBands + tid] = v;  // ceps_0[i] = features[i]
          feat[tid] = v;
        } else if (tid == 32) {
          feat[40] = (float)(.01 * (im[is::kPitch] - 300));
        }
        __syncthreads();
        if (tid < 6) {
          const float *c0 = ceps + memid * kBands;
          const float *c1 = ceps + ((memid < 1) ? kCeps + memid - 1 : memid - 1) * kBands;
          const float *c2 = ceps + ((memid < 2) ? kCeps + memid - 2 : memid - 2) * kBands;
          const int i = tid;
          feat[i] = c0[i] + c1[i] + c2[i];
          feat[kBands + i] = c0[i] - c2[i];
          feat[kBands + 6 + i] = c0[i] - 2 * c1[i] + c2[i];
        } else if (tid >= 32 && tid < 32 + kCeps) {
          const int i = tid - 32;
          float mindist = 1e15f;
          for (int j = 0; j < kCeps; j++) {
            float dist = 0;
#pragma unroll
            for (int k = 0; k < kBands; k++) {
              const float tmp = ceps[i * kBands + k] - ceps[j * kBands + k];
              dist += tmp * tmp;
            }
            if (j != i) mindist = (mindist < dist) ? mindist : dist;
          }
          misc[ms::kMind + i] = mindist;
        }
        __syncthreads();
        if (tid == 0) {
          float sv = 0;
          for (int i = 0; i < kCeps; i++) sv += misc[ms::kMind + i];
          feat[41] = (float)(sv / kCeps - 2.1);
          int mid = memid + 1;
          if (mid == kCeps) mid = 0;
          im[is::kMemId] = mid;
        }
        __syncthreads();
      STAMP(16);
        // ---- compute_rnn
        dense_layer<NT>(M.in_dense, feat, dout, tt, tid);
        __syncthreads();
        gru_gates<NT>(M.vad, dout, gv, zr, tt, tid);
        __syncthreads();
        gru_out<NT>(M.vad, dout, gv, zr, hb, tt, tid);
        __syncthreads();
      STAMP(17);
        {
          const int nd = M.in_dense.nout, nv = M.vad.nout;
          for (int i = tid; i < nv; i += NT) gv[i] = hb[i];
          __syncthreads();
          // noise_input = [dense_out, vad_state, features]
          for (int i = tid; i < nd + nv + kFeat; i += NT)
            rin[i] = (i < nd) ? dout[i] : (i < nd + nv) ? gv[i - nd] : feat[i - nd - nv];
          if (tid == NT - 1) {  // vad_output on the updated vad state
            const DevDense &d = M.vad_out;
            float sum = d.b[0];
            for (int j = 0; j < d.nin; j++) sum += d.w[j * d.nout] * gv[j];
            misc[ms::kVadCh + c] = activate(tt, d.act, kWs * sum);
          }
        }
        __syncthreads();
        gru_gates<NT>(M.noise, rin, gn, zr, tt, tid);
        __syncthreads();
        gru_out<NT>(M.noise, rin, gn, zr, hb, tt, tid);
        __syncthreads();
      STAMP(18);
        {
          const int nv = M.vad.nout, nn = M.noise.nout;
          for (int i = tid; i < nn; i += NT) gn[i] = hb[i];
          __syncthreads();
          for (int i = tid; i < nv + nn + kFeat; i += NT)
            rin[i] = (i < nv) ? gv[i] : (i < nv + nn) ? gn[i - nv] : feat[i - nv - nn];
        }
        __syncthreads();
        gru_gates<NT>(M.den, rin, gd, zr, tt, tid);
        __syncthreads();
        gru_out<NT>(M.den, rin, gd, zr, hb, tt, tid);
        __syncthreads();
        for (int i = tid; i < M.den.nout; i += NT) gd[i] = hb[i];
        __syncthreads();
        dense_layer<NT>(M.den_out, gd, g, tt, tid);
        __syncthreads();
      STAMP(19);
        // ---- pitch_filter
        if (tid < kBands) {
          const int i = tid;
          float r;
          if (Exp[i] > g[i])
            r = 1;
          else
            r = (float)((double)((Exp[i] * Exp[i]) * (1 - (g[i] * g[i]))) /
                        (.001 + (double)((g[i] * g[i]) * (1 - (Exp[i] * Exp[i])))));
          float cl = (0 > r) ? 0 : r;
          cl = (1 < cl) ? 1 : cl;
          r = (float)sqrt((double)cl);
          r = (float)((double)r * sqrt((double)Ex[i] / (1e-8 + (double)Ep[i])));
          rr[i] = r;
        }
        __syncthreads();
        for (int k = tid; k < kFreq; k += NT) {
          const float rf = interp_gain(rr, P, k);
          X[k].x += rf * W[k].x;
          X[k].y += rf * W[k].y;
        }
        __syncthreads();
        if (tid < kBands) newE[tid] = band_sum(X, X, P, tid);
        __syncthreads();
        if (tid < kBands) {
          const int i = tid;
          nrm[i] = (float)sqrt((double)Ex[i] / (1e-8 + (double)newE[i]));
          const float al = .6f * lastg[i];
          const float gi = (g[i] > al) ? g[i] : al;
          g[i] = gi;
          lastg[i] = gi;
        }
        __syncthreads();
        for (int k = tid; k < kFreq; k += NT) {
          const float nf = interp_gain(nrm, P, k);
          float2 v = X[k];
          v.x *= nf;
          v.y *= nf;
          const float gf = interp_gain(g, P, k);
          v.x *= gf;
          v.y *= gf;
          X[k] = v;
        }
        __syncthreads();
      STAMP(20);
      } else {
        if (tid == 0) misc[ms::kVadCh + c] = 0;
      }
      // ---- frame_synthesis: inverse via forward FFT of the Hermitian extension
      for (int i = tid; i < kWin; i += NT) {
        float2 v;
        if (i < kFreq)
          v = X[i];
        else
          v = make_float2(X[kWin - i].x, -X[kWin - i].y);
        W[P->bitrev960[i]] = make_float2(scale * v.x, scale * v.y);
      }
      __syncthreads();
      fft960_stages<NT>(W, tw, tid);
      {
        const float inv = 1.0f / (float)32767;  // Denoiser.zig:73
        float *ring = a.ring + ((size_t)s * C + c) * ring_len;
        float *dout_g = a.out_den ? a.out_den + (((size_t)t * a.n_streams + s) * C + c) * kFrame : nullptr;
        const long long base = (long long)frames_done * kFrame;
        for (int i = tid; i < kFrame; i += NT) {
          const float y0 = (i == 0) ? kWin * W[0].x : kWin * W[kWin - i].x;
          const float y1 = kWin * W[kWin - (i + kFrame)].x;
          const float a0 = y0 * hw[i];
          const float a1 = y1 * hw[kFrame - 1 - i];
          const float o = a0 + syn[i];
          syn[i] = a1;
          const float dn = a.raw_s16 ? o : o * inv;
          ring[(base + i) % ring_len] = dn;
          if (dout_g) dout_g[i] = dn;
        }
      }
      __syncthreads();
      STAMP(21);
    }  // channels
    // ---- per tick: vad_low, re-blocking, window completion (VAD.zig:284-348)
    {
      float vad_low = 1;
      for (int c = 0; c < C; c++) {
        const float v = misc[ms::kVadCh + c];
        if (v < vad_low) vad_low = v;
      }
      const float ratio = a.ratio[(size_t)t * a.n_streams + s];
      const long long a0 = (long long)frames_done * kFrame;
      const long long wdone = a0 / FB;
      const long long next_end = (wdone + 1) * FB;
      const bool complete = a0 + kFrame >= next_end;
      float win_ratio = 0;
      if (complete) {
        const int r = (int)(next_end - a0);
        vol_acc += ratio * ((float)r / (float)FB);
        win_ratio = vol_acc;
        vol_acc = 0;
        if (kFrame - r > 0) vol_acc += ratio * ((float)(kFrame - r) / (float)FB);
      } else {
        vol_acc += ratio * ((float)kFrame / (float)FB);
      }
      const size_t o = (size_t)t * a.n_streams + s;
      if (tid == 0) {
        a.out_vad[o] = vad_low;
        a.out_win_flag[o] = complete ? 1 : 0;
        a.out_win_ratio[o] = complete ? win_ratio : 0.0f;
        a.out_win_vad[o] = complete ? vad_low : 0.0f;
      }
      if (!complete && tid < C * a.n_bands) a.out_band[o * C * a.n_bands + tid] = 0.0f;  // defined: no window
      if (complete) {
        // FFT B per channel: window, kissfft (mixed radix), kiss_fftr post-pass, |X|*norm, band sums
        const int nc = P->ncfft_b;
        const float2 *__restrict__ twb = reinterpret_cast<const float2 *>(P->twb);
        const float2 *__restrict__ sup = reinterpret_cast<const float2 *>(P->superb);
        const long long wstart = wdone * FB;
        for (int c = 0; c < C; c++) {
          const float *ring = a.ring + ((size_t)s * C + c) * ring_len;
          for (int k = tid; k < nc; k += NT) {
            const int n = P->permb[k];
            const float t0 = ring[(wstart + 2 * n) % ring_len] * P->hannb[2 * n];
            const float t1 = ring[(wstart + 2 * n + 1) % ring_len] * P->hannb[2 * n + 1];
            W[k] = make_float2(t0, t1);
          }
          __syncthreads();
          // fused mode: fft_size <= 2048 and radices 2..5 (no out-of-place stage)
          kiss_stages(W, nullptr, P->fac_b, P->nfac_b, nc, twb, tid, NT);
          // magnitudes of the union of reported bins
          const int lo = a.bin_lo_all, hi = a.bin_hi_all;
          for (int k = lo + tid; k <= hi; k += NT) {
            float re, imv;
            if (k == 0) {
              re = W[0].x + W[0].y;
              imv = 0;
            } else if (k == nc) {
              re = W[0].x - W[0].y;
              imv = 0;
            } else {
              const int kk = (2 * k < nc) ? k : nc - k;
              const float2 fpk = W[kk];
              const float2 fpnk = make_float2(W[nc - kk].x, -W[nc - kk].y);
              const float2 f1k = cadd(fpk, fpnk), f2k = csub(fpk, fpnk);
              const float2 tw2 = cmul(f2k, sup[kk - 1]);
              if (2 * k < nc) {
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
          __syncthreads();
          if (tid < a.n_bands) {
            float acc = 0.0f;
            for (int k = a.band_lo[tid]; k <= a.band_hi[tid]; k++) acc += mag[k - lo];
            a.out_band[(o * C + c) * a.n_bands + tid] = acc;
          }
          __syncthreads();
        }
      }
      frames_done++;
    }
      STAMP(22);
  }  // ticks

  // ---- store persistent state
  __syncthreads();
  for (int i = tid; i < kPitchBuf; i += NT) stp[st::kPitch + i] = pb[i];
  for (int i = tid; i < kFrame; i += NT) stp[st::kSyn + i] = syn[i];
  for (int i = tid; i < kCeps * kBands; i += NT) stp[st::kCepsMem + i] = ceps[i];
  for (int i = tid; i < kBands; i += NT) stp[st::kLastG + i] = lastg[i];
  for (int i = tid; i < kMaxNeurons; i += NT) {
    stp[st::kVadGru + i] = gv[i];
    stp[st::kNoiseGru + i] = gn[i];
    stp[st::kDenGru + i] = gd[i];
  }
  if (tid == 0) {
    istp[st::kMemId] = im[is::kMemId];
    istp[st::kLastPeriod] = im[is::kLastPeriod];
    stp[st::kLastGain] = misc[ms::kPg];
    istp[st::kFramesDone] = frames_done;
    stp[st::kVolAcc] = vol_acc;
  }
#ifdef FVAD_STAMPS
  STAMP(23);
  if (tid == 0 && a.stamps)
    for (int i = 0; i < kStamps; i++) atomicAdd(&a.stamps[i], stamp_acc[i]);
#endif
}

// ---------------------------------------------------------------------------
// k_kiss_fftr: one workgroup computes the complete kissfft real FFT of one
// nfft-point frame (kiss_fftr, FFT.zig:90) -- used by the kiss_fftr compat
// shim, any even nfft.  Tables (twiddles, super twiddles, factors, leaf
// permutation) come from the caller's cfg memory (kiss_fftr_alloc lenmem
// protocol).  The work arrays W / S are in LDS when they fit, else in the
// shim's device scratch (work).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_kiss_fftr(int ncfft, const int *__restrict__ fac, int nf,
                                                   const float2 *__restrict__ twb, const float2 *__restrict__ sup,
                                                   const int *__restrict__ perm, const float *__restrict__ in,
                                                   float2 *__restrict__ out, float2 *work, int in_lds) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  float2 *W = in_lds ? reinterpret_cast<float2 *>(L) : work;
  float2 *S = W + ncfft;
  const int tid = threadIdx.x;
  const float2 *in2 = reinterpret_cast<const float2 *>(in);
  for (int k = tid; k < ncfft; k += 256) W[k] = in2[perm[k]];
  __syncthreads();
  kiss_stages(W, S, fac, nf, ncfft, twb, tid, 256);
  for (int k = tid; k <= ncfft; k += 256) {
    float2 r;
    if (k == 0) {
      r = make_float2(W[0].x + W[0].y, 0.0f);
    } else if (k == ncfft) {
      r = make_float2(W[0].x - W[0].y, 0.0f);
    } else {
      // kiss_fftr's loop kk = 1 .. ncfft/2 writes bin kk, then bin ncfft - kk
      // (the later write wins at kk = ncfft/2)
      const bool lower = 2 * k < ncfft;
      const int kk = lower ? k : ncfft - k;
      const float2 fpk = W[kk];
      const float2 fpnk = make_float2(W[ncfft - kk].x, -W[ncfft - kk].y);
      const float2 f1k = cadd(fpk, fpnk), f2k = csub(fpk, fpnk);
      const float2 tw2 = cmul(f2k, sup[kk - 1]);
      if (lower)
        r = make_float2((f1k.x + tw2.x) * ((float).5), (f1k.y + tw2.y) * ((float).5));
      else
        r = make_float2((f1k.x - tw2.x) * ((float).5), (tw2.y - f1k.y) * ((float).5));
    }
    out[k] = r;
  }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
constexpr int kFrameThreads = 256;

size_t frame_lds_bytes() { return sizeof(float) * lds::kTotal; }

hipError_t launch_prep(const PrepArgs &a, hipStream_t stream) {
  const int blocks = (a.n_streams + 63) / 64;
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_prep, dim3(blocks), dim3(64), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_kiss_fftr(int ncfft, const int *fac, int nf, const float *twb, const float *sup, const int *perm,
                            const float *in, float *out, float *work, hipStream_t stream) {
  const size_t lds = sizeof(float) * 4 * (size_t)ncfft;  // W + S
  const bool in_lds = lds <= 64 * 1024;
  hipLaunchKernelGGL(k_kiss_fftr, dim3(1), dim3(256), in_lds ? lds : 0, stream, ncfft, fac, nf,
                     reinterpret_cast<const float2 *>(twb), reinterpret_cast<const float2 *>(sup), perm, in,
                     reinterpret_cast<float2 *>(out), reinterpret_cast<float2 *>(work), in_lds ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_frame(const FrameArgs &a, hipStream_t stream) {
  (void)hipGetLastError();  // clear stale errors from earlier calls
  hipLaunchKernelGGL(k_frame<kFrameThreads>, dim3(a.n_streams), dim3(kFrameThreads), frame_lds_bytes(), stream, a);
  return hipGetLastError();
}

}  // namespace fvad
