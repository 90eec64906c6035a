// Staged (time-parallel) MI355X pipeline for the Formula-VAD hot path.
//
// rnnoise_process_frame splits into work that depends only on the input
// samples of the (virtual, channel-interleaved) stream and a thin recurrence:
//
//   k_prep2   lane/stream   HP biquad (serial IIR), s16 scaling, RMS volume
//                           ratio; x written stream-contiguous with 1248 samples
//                           of pitch history in front of the launch's frames
//   k_fftA    wg/frame      analysis window + FFT A, band energies Ex, the
//                           log/floor chain (Ly, E, silence gate), DCT(Ly)
//   k_pitch   wg/frame      pitch_downsample (autocorr, LPC, FIR5), coarse and
//                           fine xcorr + find_best_pitch, every remove_doubling
//                           inner product for every candidate period (the
//                           final 3-lag xcorr speculatively for all 15)
//   k_select  lane/stream   remove_doubling's sequential candidate selection
//                           (needs last_period / last_gain) -> pitch index
//   k_pspec   wg/frame      pitch window + FFT A -> P, Ep, Exp, DCT(Exp)
//   k_rnn     wg/stream     the true recurrence: cepstral memory, spectral
//                           variability, GRU stack, pitch filter, gain smoothing
//   k_synth   wg/frame      Hermitian extension + FFT A + synthesis window
//   k_ola     per sample    overlap-add, 1/32767, re-block ring, per-tick vad
//   k_winmeta lane/stream   window completion, share-weighted ratio, state
//   k_fftb    wg/window     FFT B (kissfft radix-4), magnitudes, band sums
//
// Each wg/frame kernel is persistent (grid-stride over frames) so per-thread
// table values stay in registers across frames.  All arithmetic reproduces the
// oracle's operation order (see fvad_kernels.hip), so results are
// bit-identical to the fused kernel and the CPU oracle.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "fvad_device.h"
#include "fvad_internal.h"
#include "fvad_staged.h"

namespace fvad {

// Diagnostic build only (-DFVAD_STAMPS): per-phase s_memtime totals of
// thread 0 (it joins every barrier, so a phase's stamp is its critical path),
// accumulated into a.stamps[base + id]; no other code reads them.
#ifdef FVAD_STAMPS
#define STAMP_INIT()                \
  unsigned long long st_acc[16] = {}; \
  unsigned long long st_last = __builtin_amdgcn_s_memtime()
#define RSTAMP(id)                                                \
  do {                                                            \
    if (tid == 0) {                                               \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
      st_acc[id] += t_ - st_last;                                 \
      st_last = t_;                                               \
    }                                                             \
  } while (0)
#define STAMP_FLUSH(base, n)                                                  \
  do {                                                                        \
    if (tid == 0 && a.stamps)                                                 \
      for (int i_ = 0; i_ < (n); i_++) atomicAdd(&a.stamps[(base) + i_], st_acc[i_]); \
  } while (0)
#else
#define STAMP_INIT() \
  do {               \
  } while (0)
#define RSTAMP(id) \
  do {             \
  } while (0)
#define STAMP_FLUSH(base, n) \
  do {                       \
  } while (0)
#endif

namespace {
constexpr int kHist = kPitchBuf - kFrame;  // 1248
#ifndef FVAD_PITCH_FRAMES
#define FVAD_PITCH_FRAMES 4
#endif
constexpr int kPitchFrames = FVAD_PITCH_FRAMES;  // frames per k_pitch workgroup
constexpr float kScale960 = 1.f / 960;

__device__ __forceinline__ int ticks_of(const StagedArgs &a, int s) {
  return a.ticks_valid ? a.ticks_valid[s] : a.n_ticks;
}

// analysis / synthesis window value for index i of the 960-sample window
__device__ __forceinline__ float win960(const float *__restrict__ hw, int i) {
  return (i < kFrame) ? hw[i] : hw[kWin - 1 - i];
}
}  // namespace

// ---------------------------------------------------------------------------
// k_prep2: high-pass biquad (a serial IIR with f64 intermediates: no exact
// parallel form exists, so one lane walks one stream), s16 scaling, RMS
// volume ratio.  A 256-thread workgroup owns S = 16 / C streams: wave 0 runs
// the S serial biquad chains out of LDS while waves 2-3 stream the next
// tick's input in and the previous tick's output out with coalesced 16-byte
// accesses (the input of S consecutive streams of one tick is contiguous),
// and wave 1 computes the per-channel RMS sums.
// ---------------------------------------------------------------------------
constexpr int kPrepSlots = 16;  // channel-frames per tick per workgroup

__global__ void __launch_bounds__(256) k_prep2(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float inb[2][kPrepSlots * kFrame];
  __shared__ __attribute__((aligned(16))) float outb[2][kPrepSlots * kFrame];
  __shared__ float vol[2][kPrepSlots];
  __shared__ int nts[kPrepSlots];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int C = a.n_channels, S = kPrepSlots / C, sb = blockIdx.x * S;
  const int ns = min(S, a.n_streams - sb);  // streams in this workgroup
  if (ns <= 0) return;
  const int slots = ns * C;
  if (tid < S) nts[tid] = (tid < ns) ? ticks_of(a, sb + tid) : 0;
  __syncthreads();
  int T = 0;
  for (int s = 0; s < ns; s++) T = max(T, nts[s]);
  // pitch history of every stream -> xs[s][0..1248)
  for (int idx = tid; idx < ns * kHist; idx += 256) {
    const int s = idx / kHist, i = idx - s * kHist;
    if (nts[s] > 0)
      a.xs[(size_t)(sb + s) * a.L + i] = a.state[(size_t)(sb + s) * st::kWords + st::kPitch + kFrame + i];
  }
  auto load_tick = [&](int t, int buf) {  // waves 2-3
    const float4 *src = reinterpret_cast<const float4 *>(a.pcm + ((size_t)t * a.n_streams + sb) * C * kFrame);
    float4 *dst = reinterpret_cast<float4 *>(inb[buf]);
    for (int i = tid - 128; i < slots * kFrame / 4; i += 128) dst[i] = src[i];
  };
  auto store_tick = [&](int t, int buf) {  // waves 2-3
    for (int i = tid - 128; i < slots * kFrame / 4; i += 128) {
      const int slot = i / (kFrame / 4), s = slot / C, c = slot - s * C, k = i - slot * (kFrame / 4);
      if (t < nts[s])
        reinterpret_cast<float4 *>(a.xs + (size_t)(sb + s) * a.L + kHist + (size_t)(t * C + c) * kFrame)[k] =
            reinterpret_cast<const float4 *>(outb[buf] + slot * kFrame)[k];
    }
  };
  float mem0 = 0, mem1 = 0;
  if (wave == 0 && lane < ns) {
    mem0 = a.state[(size_t)(sb + lane) * st::kWords + st::kHp];
    mem1 = a.state[(size_t)(sb + lane) * st::kWords + st::kHp + 1];
  }
  if (wave >= 2 && T > 0) load_tick(0, 0);
  __syncthreads();
  const float b0 = -2.0f, b1 = 1.0f, a0 = -1.99599f, a1 = 0.99600f;
  const float scalar = (float)32767;
  for (int t = 0; t <= T; t++) {
    const int cur = t & 1;
    if (t < T) {
      if (wave == 0) {
        if (lane < ns && t < nts[lane]) {
          for (int c = 0; c < C; c++) {
            const float *x = inb[cur] + (lane * C + c) * kFrame;
            float *y = outb[cur] + (lane * C + c) * kFrame;
#pragma unroll 8
            for (int i = 0; i < kFrame; i++) {
              const float v0 = x[i];
              const float xi = a.raw_s16 ? v0 : v0 * scalar;
              const float yi = xi + mem0;
              // b*x and a*y are exact in double (24-bit x 24-bit significands), so
              // one fma rounds b*x - a*y exactly once, as the C expression does;
              // it shortens the serial chain by one dependent f64 operation
              const double yd = (double)yi;
              mem0 = (float)((double)mem1 + __builtin_fma(-(double)a0, yd, b0 * (double)xi));
              mem1 = (float)__builtin_fma(-(double)a1, yd, b1 * (double)xi);
              y[i] = yi;
            }
          }
        }
      } else if (wave == 1) {
        if (lane < slots) {
          const float *x = inb[cur] + lane * kFrame;
          float sum = 0;
#pragma unroll 8
          for (int i = 0; i < kFrame; i++) sum += x[i] * x[i];
          vol[cur][lane] = sqrtf(sum / (float)kFrame);
        }
        if (t > 0 && lane < ns && t - 1 < nts[lane]) {
          float vmin = 1, vmax = 0;
          for (int c = 0; c < C; c++) {
            const float vl = vol[cur ^ 1][lane * C + c];
            if (vl < vmin) vmin = vl;
            if (vl > vmax) vmax = vl;
          }
          a.ratio[(size_t)(t - 1) * a.n_streams + sb + lane] = (vmax == 0) ? 0 : vmin / vmax;
        }
      } else {
        if (t + 1 < T) load_tick(t + 1, cur ^ 1);
        if (t > 0) store_tick(t - 1, cur ^ 1);
      }
    } else {
      if (wave >= 2 && t > 0) store_tick(t - 1, cur ^ 1);
      if (wave == 1 && t > 0 && lane < ns && t - 1 < nts[lane]) {
        float vmin = 1, vmax = 0;
        for (int c = 0; c < C; c++) {
          const float vl = vol[cur ^ 1][lane * C + c];
          if (vl < vmin) vmin = vl;
          if (vl > vmax) vmax = vl;
        }
        a.ratio[(size_t)(t - 1) * a.n_streams + sb + lane] = (vmax == 0) ? 0 : vmin / vmax;
      }
    }
    __syncthreads();
  }
  if (wave == 0 && lane < ns && nts[lane] > 0) {
    a.state[(size_t)(sb + lane) * st::kWords + st::kHp] = mem0;
    a.state[(size_t)(sb + lane) * st::kWords + st::kHp + 1] = mem1;
  }
  // pitch_buf after the last frame = the last 1728 samples of the row
  for (int idx = tid; idx < ns * kPitchBuf; idx += 256) {
    const int s = idx / kPitchBuf, i = idx - s * kPitchBuf;
    if (nts[s] > 0)
      a.state[(size_t)(sb + s) * st::kWords + st::kPitch + i] =
          a.xs[(size_t)(sb + s) * a.L + (size_t)(nts[s] * C - 1) * kFrame + i];
  }
}

// ---------------------------------------------------------------------------
// Persistent 256-thread frame kernels (k_fftA, k_pspec, k_synth) work on F
// frames per workgroup iteration: each phase covers all F frames, so the
// per-band serial sums (band energies, the Ly chain, DCTs) of F frames share
// wave instructions and every barrier is amortised over F frames.  Per-thread
// setup, loaded once: the element indices a thread owns in the 960-point
// windowed scatter (i = tid + 256 r), their digit-reversed destinations and
// window values, and the FFT twiddles.
// ---------------------------------------------------------------------------
constexpr int kFftFrames = 4;

struct FrameCtx {
  Fft960Tw tw;
  int dst[4];      // scatter form: W[dst[r]] <- element tid + 256 r
  float win[4];    //   and its window value
  int src[4];      // gather form: W[tid + 256 r] <- element src[r]
  float wsrc[4];   //   and its window value
};
__device__ __forceinline__ void frame_ctx_load(FrameCtx &c, const Plan *__restrict__ P, int tid) {
  fft960_load(c.tw, reinterpret_cast<const float2 *>(P->tw960), tid);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int i = tid + 256 * r;
    c.dst[r] = i < kWin ? P->bitrev960[i] : 0;
    c.win[r] = i < kWin ? win960(P->half_window, i) : 0.0f;
    c.src[r] = i < kWin ? P->ibitrev960[i] : 0;
    c.wsrc[r] = i < kWin ? win960(P->half_window, c.src[r]) : 0.0f;
  }
}

// frame indices of group g (-1: past the end or beyond the stream's valid ticks)
template <int F>
__device__ __forceinline__ void group_frames(const StagedArgs &a, long long g, int tid, int *fidx) {
  if (tid < F) {
    const long long f = g * F + tid;
    int ok = -1;
    if (f < (long long)a.n_streams * a.V) {
      const int s = (int)(f / a.V), v = (int)(f - (long long)s * a.V);
      if (v < ticks_of(a, s) * a.n_channels) ok = (int)f;
    }
    fidx[tid] = ok;
  }
}
__device__ __forceinline__ const float *frame_pb(const StagedArgs &a, int f) {
  const int s = f / a.V, v = f - s * a.V;
  return a.xs + (size_t)s * a.L + (size_t)v * kFrame;
}
// frame index of slot fr of group g, or -1 (same rule as group_frames)
__device__ __forceinline__ int frame_of(const StagedArgs &a, long long g, int F, int fr) {
  const long long f = g * F + fr;
  if (f >= (long long)a.n_streams * a.V) return -1;
  const int s = (int)(f / a.V), v = (int)(f - (long long)s * a.V);
  return v < ticks_of(a, s) * a.n_channels ? (int)f : -1;
}
// This thread's 4 samples of the 960-sample analysis window of every frame of
// group g (issued one group ahead so the HBM latency hides behind the work)
// (gathered in digit-reversed order: sample src[r] lands in W[tid + 256 r])
template <int F>
__device__ __forceinline__ void load_window(const StagedArgs &a, long long g, int tid, const FrameCtx &cx,
                                            float (&buf)[F][4]) {
#pragma unroll
  for (int fr = 0; fr < F; fr++) {
    const int f = frame_of(a, g, F, fr);
    const float *pb = f >= 0 ? frame_pb(a, f) + (kPitchBuf - kWin) : nullptr;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = tid + 256 * r;
      buf[fr][r] = (pb && i < kWin) ? pb[cx.src[r]] : 0.0f;
    }
  }
}

// ---------------------------------------------------------------------------
// k_fftA: X, Ex, Ly chain, silence, DCT(Ly)
// ---------------------------------------------------------------------------
template <int F>
__global__ void __launch_bounds__(256) k_fftA(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 W[F][kWin];
  __shared__ BandTab T;
  __shared__ float Ly[F][kBands + 2], Exl[F][kBands + 2];
  __shared__ int sil[F], fidx[F];
  const int tid = threadIdx.x;
  FrameCtx cx;
  frame_ctx_load(cx, a.plan, tid);
  bandtab_load(T, a.plan, tid, 256);
  const long long ngroups = ((long long)a.n_streams * a.V + F - 1) / F;
  STAMP_INIT();
  float win_cur[F][4];
  if (blockIdx.x < ngroups) load_window<F>(a, blockIdx.x, tid, cx, win_cur);
  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    group_frames<F>(a, g, tid, fidx);
    float win_nxt[F][4];
    if (g + gridDim.x < ngroups) load_window<F>(a, g + gridDim.x, tid, cx, win_nxt);
    __syncthreads();
    RSTAMP(0);
#pragma unroll
    for (int fr = 0; fr < F; fr++) {
      if (fidx[fr] < 0) continue;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = tid + 256 * r;
        if (i < kWin) {
          float val = win_cur[fr][r];
          val *= cx.wsrc[r];
          W[fr][i] = make_float2(kScale960 * val, kScale960 * 0.0f);
        }
      }
    }
#pragma unroll
    for (int fr = 0; fr < F; fr++)
#pragma unroll
      for (int r = 0; r < 4; r++) win_cur[fr][r] = win_nxt[fr][r];
    __syncthreads();
    RSTAMP(1);
    fft960_run<F>(cx.tw, W, tid);
    RSTAMP(2);
    for (int idx = tid; idx < F * kFreq; idx += 256) {
      const int fr = idx / kFreq, k = idx - fr * kFreq;
      if (fidx[fr] >= 0) a.X[(size_t)fidx[fr] * kFreq + k] = W[fr][k];
    }
    if (tid < F * kBands) {
      const int fr = tid / kBands, b = tid - fr * kBands;
      const float ex = band_sum_t(W[fr], W[fr], T, b);
      Exl[fr][b] = ex;
      if (fidx[fr] >= 0) a.Ex[(size_t)fidx[fr] * kBands + b] = ex;
      Ly[fr][b] = (float)log10(1e-2 + (double)ex);
    }
    __syncthreads();
    RSTAMP(3);
    if (tid < F) {
      const int fr = tid;
      float logMax = -2, follow = -2, E = 0;
      for (int i = 0; i < kBands; i++) {
        const float ly0 = Ly[fr][i];
        const double bb = (follow - 1.5 > (double)ly0) ? follow - 1.5 : (double)ly0;
        const double aa = ((double)(logMax - 7) > bb) ? (double)(logMax - 7) : bb;
        const float ly = (float)aa;
        Ly[fr][i] = ly;
        logMax = (logMax > ly) ? logMax : ly;
        follow = (float)((follow - 1.5 > (double)ly) ? follow - 1.5 : (double)ly);
        E += Exl[fr][i];
      }
      sil[fr] = ((double)E < 0.04) ? 1 : 0;
      if (fidx[fr] >= 0) a.silence[fidx[fr]] = sil[fr];
    }
    __syncthreads();
    RSTAMP(4);
    if (tid < F * kBands) {
      const int fr = tid / kBands, b = tid - fr * kBands;
      if (fidx[fr] >= 0 && !sil[fr]) {
        float sum = 0;
#pragma unroll
        for (int j = 0; j < kBands; j++) sum += Ly[fr][j] * T.dct[j * kBands + b];
        float val = (float)(sum * sqrt(2. / 22));
        if (b == 0) val -= 12;
        if (b == 1) val -= 4;
        a.Lyf[(size_t)fidx[fr] * kBands + b] = val;
      }
    }
    __syncthreads();
    RSTAMP(5);
  }
  STAMP_FLUSH(16, 6);
}

// ---------------------------------------------------------------------------
// k_pitch: everything of pitch_search / remove_doubling that does not depend
// on the previous frame, for F frames per workgroup.  Every C-order sum stays
// on one lane; lanes are assigned (frame, task) pairs so the serial chains of
// F different frames (autocorr lags, Syy / yy recurrences, find_best_pitch
// scans) share wave instructions instead of running on 1-5 lanes each.
//   P0 x_lp (pitch_downsample)        all lanes
//   P1 _celt_autocorr, 5 lags x F     wave 0
//   P2 LPC + lag window + FIR coeffs  F lanes
//   P3 5-tap FIR in place             all lanes (via registers)
//   P4 wave 0: coarse / fine Syy sequences; wave 1: xx + yy_lookup chain;
//      waves 2-3: coarse xcorr, R consecutive lags per lane
//   P5 coarse find_best_pitch scan    F lanes
//   P6 fine xcorr at the <= 10 candidate lags
//   P7 fine scan -> T0, candidate periods and energies
//   P8 remove_doubling inner products + speculative final xcorr (T-1, T+1)
// ---------------------------------------------------------------------------
namespace rec {
constexpr int kT0 = 0, kXx = 1, kXy = 2, kYyT0 = 3, kNValid = 4;
constexpr int kK = 8;       // per k=2..15: T1, T1b, s1 = xcorr(T1), s2 = xcorr(T1b), yyT1, yyT1b
constexpr int kSpec = 96;   // candidate c (0 = T0, k-1 = T1_k): xcorr at T-1 [+0] and T+1 [+2]
constexpr int kSize = 144;  // (the xcorr at T itself is kXy / s1)
}  // namespace rec
static_assert(rec::kSize == kPitchRecord, "pitch record size");

template <int F>
struct PitchGeom {
  static constexpr int kXS = 868;                    // padded x row (floats)
  static constexpr int kR = 2 * ((F * 147 + 255) / 256);  // coarse lags per lane (pairs)
  static constexpr int kTPF = (147 + kR - 1) / kR;   // coarse lanes per frame
  static constexpr int kG3 = 59;                     // remove_doubling dots per frame
  static_assert(F * kTPF <= 128, "coarse xcorr lanes exceed waves 2-3");
  static_assert(5 * F <= 64 && 2 * F <= 64, "serial lanes exceed one wave");
};

__device__ __forceinline__ int rd_T1(int T0, int k) { return (int)((unsigned)(2 * T0 + k) / (unsigned)(2 * k)); }
__device__ __forceinline__ int rd_T1b(int T0, int T1, int k) {
  if (k == 2) return (T1 + T0 > 384) ? T0 : T0 + T1;
  return (int)((unsigned)(2 * second_check(k) * T0 + k) / (unsigned)(2 * k));
}

template <int F>
__global__ void __launch_bounds__(256) k_pitch(StagedArgs a) {
  using G = PitchGeom<F>;
  constexpr int NT = 256, XS = G::kXS, R = G::kR, TPF = G::kTPF;
  __shared__ __attribute__((aligned(16))) float xf[F][XS];  // FIR output (x_lp filtered)
  // per-frame scratch: x_lp during P0-P3, then xcorr / Syy / yy sequences
  __shared__ __attribute__((aligned(16))) float scr[F][980];
  constexpr int oXc = 0, oSyc = 148, oSyf = 296, oYy = 592;
  __shared__ float ac[F][5], lpc2[F][5], xxs[F], fine[F][10];
  __shared__ int best[F][2], T0s[F], nvs[F], fval[F];
  __shared__ long long pbo[F];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int V = a.V;
  const long long total = (long long)a.n_streams * V;
  const long long ngroups = (total + F - 1) / F;
  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    if (tid < F) {
      const long long f = g * F + tid;
      int ok = 0;
      long long off = 0;
      if (f < total) {
        const int s = (int)(f / V), v = (int)(f - (long long)s * V);
        ok = v < ticks_of(a, s) * a.n_channels;
        off = (long long)s * a.L + (long long)v * kFrame;
      }
      fval[tid] = ok;
      pbo[tid] = off;
    }
    __syncthreads();
    // P0: x_lp[i] = .5*(.5*(pb[2i-1] + pb[2i+1]) + pb[2i])
    for (int idx = tid; idx < F * kXlp; idx += NT) {
      const int fr = idx / kXlp, i = idx - fr * kXlp;
      const float *pb = a.xs + pbo[fr];
      scr[fr][i] = (i == 0) ? .5f * (.5f * (pb[1]) + pb[0]) : .5f * (.5f * (pb[2 * i - 1] + pb[2 * i + 1]) + pb[2 * i]);
    }
    __syncthreads();
    // P1: _celt_autocorr, lag k of frame fr
    if (tid < 5 * F) {
      const int fr = tid / 5, k = tid - 5 * fr;
      const float *x = scr[fr];
      const int fastN = kXlp - 4;
      const float acc = dot_seq(0.0f, x, 1, x + k, 1, fastN);
      float d = 0;
      for (int i = k + fastN; i < kXlp; i++) d = d + x[i] * x[i - k];
      ac[fr][k] = acc + d;
    }
    __syncthreads();
    // P2: lag window, _celt_lpc (order 4), bandwidth expansion, FIR coefficients
    if (tid < F) {
      float acv[5];
      for (int i = 0; i < 5; i++) acv[i] = ac[tid][i];
      acv[0] *= 1.0001f;
      for (int i = 1; i <= 4; i++) acv[i] -= acv[i] * (.008f * i) * (.008f * i);
      float lpc[4] = {0, 0, 0, 0};
      float error = acv[0];
      if (acv[0] != 0) {
        for (int i = 0; i < 4; i++) {
          float r_acc = 0;
          for (int j = 0; j < i; j++) r_acc += lpc[j] * acv[i - j];
          r_acc += acv[i + 1];
          const float r = -r_acc / error;
          lpc[i] = r;
          for (int j = 0; j < (i + 1) >> 1; j++) {
            const float tmp1 = lpc[j], tmp2 = lpc[i - 1 - j];
            lpc[j] = tmp1 + r * tmp2;
            lpc[i - 1 - j] = tmp2 + r * tmp1;
          }
          error = error - (r * r) * error;
          if (error < .001f * acv[0]) break;
        }
      }
      float tmp = 1.0f;
      for (int i = 0; i < 4; i++) {
        tmp = .9f * tmp;
        lpc[i] = lpc[i] * tmp;
      }
      const float c1 = .8f;
      lpc2[tid][0] = lpc[0] + .8f;
      lpc2[tid][1] = lpc[1] + c1 * lpc[0];
      lpc2[tid][2] = lpc[2] + c1 * lpc[1];
      lpc2[tid][3] = lpc[3] + c1 * lpc[2];
      lpc2[tid][4] = c1 * lpc[3];
    }
    __syncthreads();
    // P3: celt_fir5, x_lp (scratch) -> xf
    for (int idx = tid; idx < F * kXlp; idx += NT) {
      const int fr = idx / kXlp, i = idx - fr * kXlp;
      const float *x = scr[fr];
      const float m0 = i >= 1 ? x[i - 1] : 0.0f, m1 = i >= 2 ? x[i - 2] : 0.0f, m2 = i >= 3 ? x[i - 3] : 0.0f,
                  m3 = i >= 4 ? x[i - 4] : 0.0f, m4 = i >= 5 ? x[i - 5] : 0.0f;
      float sum = x[i];
      sum = sum + lpc2[fr][0] * m0;
      sum = sum + lpc2[fr][1] * m1;
      sum = sum + lpc2[fr][2] * m2;
      sum = sum + lpc2[fr][3] * m3;
      sum = sum + lpc2[fr][4] * m4;
      xf[fr][i] = sum;
    }
    __syncthreads();
    // P4: energy sequences (waves 0-1) concurrently with the coarse xcorr (waves 2-3)
    if (wave == 0) {
      if (lane < 2 * F) {
        const int fr = lane % F;
        const bool fs = lane >= F;
        syy_sequence(xf[fr], fs ? 1 : 2, fs ? 480 : 240, fs ? 294 : 147, scr[fr] + (fs ? oSyf : oSyc));
      }
    } else if (wave == 1) {
      if (lane < F) {
        const float *x = xf[lane] + (kPitchMax >> 1);
        const float xx = dot_seq(0.0f, x, 1, x, 1, 480);
        xxs[lane] = xx;
        float yy = xx;
        float *yo = scr[lane] + oYy;
        yo[0] = xx;
#pragma unroll 4
        for (int i = 1; i <= 384; i++) {
          yy = yy + x[-i] * x[-i] - x[480 - i] * x[480 - i];
          yo[i] = (0 > yy) ? 0 : yy;
        }
      }
    } else {
      const int l = tid - 128;
      const int fr = l / TPF, blk = l - fr * TPF;
      if (fr < F) {
        const int k0 = blk * R;
        const float *xr = xf[fr] + (kPitchMax >> 1);
        const float *yr = xf[fr] + 2 * k0;
        // two lags per packed f32 multiply / add (v_pk_mul_f32, v_pk_add_f32)
        typedef float f2v __attribute__((ext_vector_type(2)));
        f2v acc[R / 2];
#pragma unroll
        for (int p = 0; p < R / 2; p++) acc[p] = f2v{0.0f, 0.0f};
#pragma unroll 4
        for (int j = 0; j < 240; j++) {
          const float xv = xr[2 * j];
          const f2v xb = f2v{xv, xv};
#pragma unroll
          for (int p = 0; p < R / 2; p++) acc[p] = acc[p] + xb * f2v{yr[2 * (j + 2 * p)], yr[2 * (j + 2 * p + 1)]};
        }
#pragma unroll
        for (int p = 0; p < R / 2; p++) {
          if (k0 + 2 * p < 147) scr[fr][oXc + k0 + 2 * p] = acc[p].x;
          if (k0 + 2 * p + 1 < 147) scr[fr][oXc + k0 + 2 * p + 1] = acc[p].y;
        }
      }
    }
    __syncthreads();
    // P5: coarse find_best_pitch
    if (tid < F) {
      int bst[2] = {0, 1};
      float bn0 = -1, bn1 = -1, bd0 = 0, bd1 = 0;
#pragma unroll 4
      for (int i = 0; i < 147; i++) best_pitch_visit(scr[tid][oXc + i], scr[tid][oSyc + i], i, bn0, bn1, bd0, bd1, bst);
      best[tid][0] = bst[0];
      best[tid][1] = bst[1];
    }
    __syncthreads();
    // P6: fine xcorr, only the lags within +-2 of 2*best0 / 2*best1 are non-zero
    if (tid < 10 * F) {
      const int fr = tid / 10, t = tid - 10 * fr;
      const int bp0 = best[fr][0], bp1 = best[fr][1];
      const int i = (t < 5 ? 2 * bp0 : 2 * bp1) - 2 + (t % 5);
      const bool dup = t >= 5 && abs(i - 2 * bp0) <= 2;
      if (i >= 0 && i < 294 && !dup) {
        const float *xl = xf[fr] + (kPitchMax >> 1), *y = xf[fr] + i;
        const float sum = dot_seq(0.0f, xl, 1, y, 1, 480);
        fine[fr][t] = (-1 > sum) ? -1 : sum;
      }
    }
    __syncthreads();
    // P7: fine find_best_pitch + pseudo-interpolation -> T0 (remove_doubling input)
    if (tid < F) {
      const int fr = tid;
      const int bp0 = best[fr][0], bp1 = best[fr][1];
      const int w0 = 2 * bp0 - 2, w1 = 2 * bp1 - 2;
      auto xcf = [&](int i) -> float {
        if (i >= w0 && i <= w0 + 4) return fine[fr][i - w0];
        if (i >= w1 && i <= w1 + 4) return fine[fr][5 + i - w1];
        return 0.0f;
      };
      int bst[2] = {0, 1};
      float bn0 = -1, bn1 = -1, bd0 = 0, bd1 = 0;
      int lo0 = w0, hi0 = w0 + 4, lo1 = w1, hi1 = w1 + 4;
      if (lo1 < lo0) {
        const int t0 = lo0, t1 = hi0;
        lo0 = lo1;
        hi0 = hi1;
        lo1 = t0;
        hi1 = t1;
      }
      for (int i = max(0, lo0); i <= min(293, hi0); i++) best_pitch_visit(xcf(i), scr[fr][oSyf + i], i, bn0, bn1, bd0, bd1, bst);
      for (int i = max(max(0, lo1), hi0 + 1); i <= min(293, hi1); i++)
        best_pitch_visit(xcf(i), scr[fr][oSyf + i], i, bn0, bn1, bd0, bd1, bst);
      int offset;
      if (bst[0] > 0 && bst[0] < 294 - 1) {
        const float aa = xcf(bst[0] - 1), bb = xcf(bst[0]), cc = xcf(bst[0] + 1);
        if ((cc - aa) > .7f * (bb - aa))
          offset = 1;
        else if ((aa - cc) > .7f * (bb - cc))
          offset = -1;
        else
          offset = 0;
      } else {
        offset = 0;
      }
      const int pitch = 2 * bst[0] - offset;
      int T0 = (kPitchMax - pitch) / 2;
      if (T0 >= 384) T0 = 383;
      int nv = 0;
      for (int k = 2; k <= 15; k++) {
        if (rd_T1(T0, k) < 30) break;
        nv++;
      }
      T0s[fr] = T0;
      nvs[fr] = nv;
      if (fval[fr]) {
        float *rg = a.rec + (g * F + fr) * rec::kSize;
        rg[rec::kT0] = __int_as_float(T0);
        rg[rec::kXx] = xxs[fr];
        rg[rec::kYyT0] = scr[fr][oYy + T0];
        rg[rec::kNValid] = __int_as_float(nv);
      }
    }
    __syncthreads();
    // P8: candidate metadata + remove_doubling dots (C order, one per lane)
    if (tid < 14 * F) {
      const int fr = tid / 14, kk = tid - 14 * fr, k = kk + 2;
      if (fval[fr] && kk < nvs[fr]) {
        const int T0 = T0s[fr], T1 = rd_T1(T0, k), T1b = rd_T1b(T0, T1, k);
        float *q = a.rec + (g * F + fr) * rec::kSize + rec::kK + kk * 6;
        q[0] = __int_as_float(T1);
        q[1] = __int_as_float(T1b);
        q[4] = scr[fr][oYy + T1];
        q[5] = scr[fr][oYy + T1b];
      }
    }
    for (int idx = tid; idx < F * G::kG3; idx += NT) {
      const int fr = idx / G::kG3, q = idx - fr * G::kG3;
      if (!fval[fr]) continue;
      const int T0 = T0s[fr], nv = nvs[fr];
      int lag = -1, slot = 0;
      if (q == 0) {
        lag = T0;
        slot = rec::kXy;
      } else if (q < 29) {
        const int kk = (q - 1) >> 1, k = kk + 2;
        if (kk < nv) {
          const int T1 = rd_T1(T0, k);
          lag = ((q - 1) & 1) ? rd_T1b(T0, T1, k) : T1;
          slot = rec::kK + kk * 6 + 2 + ((q - 1) & 1);
        }
      } else {
        const int c = (q - 29) >> 1, side = (q - 29) & 1;
        if (c == 0 || c - 1 < nv) {
          const int T = (c == 0) ? T0 : rd_T1(T0, c + 1);
          lag = side ? T + 1 : T - 1;
          slot = rec::kSpec + c * 3 + (side ? 2 : 0);
        }
      }
      if (lag >= 0) {
        const float *xl = xf[fr] + (kPitchMax >> 1);
        const float acc = dot_seq(0.0f, xl, 1, xl - lag, 1, 480);
        a.rec[(g * F + fr) * rec::kSize + slot] = acc;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_select: remove_doubling's sequential selection (one lane per stream).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_select(StagedArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_streams) return;
  const int nf = ticks_of(a, s) * a.n_channels;
  if (nf <= 0) return;
  float *stp = a.state + (size_t)s * st::kWords;
  int *istp = reinterpret_cast<int *>(stp);
  int last_period = istp[st::kLastPeriod];
  float last_gain = stp[st::kLastGain];
  for (int v = 0; v < nf; v++) {
    const size_t f = (size_t)s * a.V + v;
    const float *r = a.rec + f * rec::kSize;
    const int T0 = __float_as_int(r[rec::kT0]);
    const int nv = __float_as_int(r[rec::kNValid]);
    const int prev_period = last_period / 2;
    const float prev_gain = last_gain;
    const float xx = r[rec::kXx];
    float xy = r[rec::kXy];
    float yy = r[rec::kYyT0];
    float best_xy = xy, best_yy = yy;
    const float g0 = pitch_gain(xy, xx, yy);
    float gg = g0;
    int T = T0, cand = 0;
    for (int k = 2; k <= 15; k++) {
      const int kk = k - 2;
      if (kk >= nv) break;
      const float *q = r + rec::kK + kk * 6;
      const int T1 = __float_as_int(q[0]);
      xy = .5f * (q[2] + q[3]);
      yy = .5f * (q[4] + q[5]);
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
        const float vv = .7f * g0 - cont;
        thresh = (.3f > vv) ? .3f : vv;
      }
      if (T1 < 3 * 30) {
        const float vv = .85f * g0 - cont;
        thresh = (.4f > vv) ? .4f : vv;
      } else if (T1 < 2 * 30) {
        const float vv = .9f * g0 - cont;
        thresh = (.5f > vv) ? .5f : vv;
      }
      if (g1 > thresh) {
        best_xy = xy;
        best_yy = yy;
        T = T1;
        gg = g1;
        cand = k - 1;
      }
    }
    best_xy = (0 > best_xy) ? 0 : best_xy;
    float pg;
    if (best_yy <= best_xy)
      pg = 1.0f;
    else
      pg = best_xy / (best_yy + 1);
    const float x0 = r[rec::kSpec + cand * 3], x2 = r[rec::kSpec + cand * 3 + 2];
    const float x1 = cand == 0 ? r[rec::kXy] : r[rec::kK + (cand - 1) * 6 + 2];  // xcorr at T itself
    int offset;
    if ((x2 - x0) > .7f * (x1 - x0))
      offset = 1;
    else if ((x0 - x2) > .7f * (x1 - x2))
      offset = -1;
    else
      offset = 0;
    if (pg > gg) pg = gg;
    int pi = 2 * T + offset;
    if (pi < kPitchMin) pi = kPitchMin;
    a.pitch[f] = pi;
    last_period = pi;
    last_gain = pg;
  }
  istp[st::kLastPeriod] = last_period;
  stp[st::kLastGain] = last_gain;
}

// ---------------------------------------------------------------------------
// k_pspec: pitch spectrum P, Ep, normalised Exp, DCT(Exp)[0..5], feature 40
// ---------------------------------------------------------------------------
template <int F>
__global__ void __launch_bounds__(256) k_pspec(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 W[F][kWin];
  __shared__ __attribute__((aligned(16))) float2 Xl[F][kFreq + 1];
  __shared__ BandTab T;
  __shared__ float Ep[F][kBands + 2], Exp[F][kBands + 2];
  __shared__ int fidx[F], pit[F];
  const int tid = threadIdx.x;
  FrameCtx cx;
  frame_ctx_load(cx, a.plan, tid);
  bandtab_load(T, a.plan, tid, 256);
  const long long ngroups = ((long long)a.n_streams * a.V + F - 1) / F;
  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    group_frames<F>(a, g, tid, fidx);
    __syncthreads();
    if (tid < F) pit[tid] = fidx[tid] >= 0 ? a.pitch[fidx[tid]] : 0;
    __syncthreads();
#pragma unroll
    for (int fr = 0; fr < F; fr++) {
      const int f = fidx[fr];
      if (f < 0) continue;
      const float *pb = frame_pb(a, f) + (kPitchBuf - kWin - pit[fr]);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = tid + 256 * r;
        if (i < kWin) {
          float val = pb[cx.src[r]];
          val *= cx.wsrc[r];
          W[fr][i] = make_float2(kScale960 * val, kScale960 * 0.0f);
        }
      }
    }
    for (int idx = tid; idx < F * kFreq; idx += 256) {
      const int fr = idx / kFreq, k = idx - fr * kFreq;
      if (fidx[fr] >= 0) Xl[fr][k] = a.X[(size_t)fidx[fr] * kFreq + k];
    }
    __syncthreads();
    fft960_run<F>(cx.tw, W, tid);
    for (int idx = tid; idx < F * kFreq; idx += 256) {
      const int fr = idx / kFreq, k = idx - fr * kFreq;
      if (fidx[fr] >= 0) a.P[(size_t)fidx[fr] * kFreq + k] = W[fr][k];
    }
    if (tid < 2 * F * kBands) {
      const int h = tid / (F * kBands), r = tid - h * (F * kBands), fr = r / kBands, b = r - fr * kBands;
      if (h == 0)
        Ep[fr][b] = band_sum_t(W[fr], W[fr], T, b);
      else
        Exp[fr][b] = band_sum_t(Xl[fr], W[fr], T, b);
    }
    __syncthreads();
    if (tid < F * kBands) {
      const int fr = tid / kBands, b = tid - fr * kBands;
      const int f = fidx[fr];
      if (f >= 0) {
        const float ex = a.Ex[(size_t)f * kBands + b];
        const float e = (float)((double)Exp[fr][b] / sqrt(.001 + (double)(ex * Ep[fr][b])));
        Exp[fr][b] = e;
        a.Ep[(size_t)f * kBands + b] = Ep[fr][b];
        a.Exp[(size_t)f * kBands + b] = e;
      }
    }
    __syncthreads();
    if (tid < F * 8) {
      const int fr = tid >> 3, i = tid & 7;
      const int f = fidx[fr];
      if (f >= 0 && i < 6) {
        float sum = 0;
#pragma unroll
        for (int j = 0; j < kBands; j++) sum += Exp[fr][j] * T.dct[j * kBands + i];
        float val = (float)(sum * sqrt(2. / 22));
        if (i == 0) val = (float)(val - 1.3);
        if (i == 1) val = (float)(val - 0.9);
        a.f34[(size_t)f * 8 + i] = val;
      } else if (f >= 0 && i == 6) {
        a.f34[(size_t)f * 8 + 6] = (float)(.01 * (pit[fr] - 300));
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_rnn: the recurrence.  One workgroup owns S streams and walks their frames
// in lockstep (frame v of every stream, then v+1 ...).  The whole GRU stack is
// resident in LDS as an int8 image (rnnimg, 88 KB; int8 -> f32 is exact), so
// weights never come from L2 per frame.  A matrix column = one neuron's C-order
// sum: lane (column, stream group) accumulates SL streams of that column with
// one weight fetch per term; per-stream vectors are stored [j][S] so the SL
// inputs of a term are one LDS read.  GRU inputs are read in place from their
// segments (no concatenation copies), GRU states ping-pong between two
// buffers (no copy-back phase), and the next frame's features are prefetched
// into registers while the current frame runs.  Per frame and stream:
// cepstral memory + deltas, spectral variability (distance matrix kept in the
// state, only the new row recomputed), compute_rnn, and the gain recurrence
// lastg; the pitch filter and gain application are in k_synth (nothing
// recurrent is left in them once g and the smoothed gains are known).
// ---------------------------------------------------------------------------
constexpr int kRnnS = 8;   // streams per workgroup
constexpr int kRnnG = 4;   // lanes per column (stream groups of S/G = 2)
constexpr int kRnnNT = 1024;
constexpr int kRnnPf = 30; // prefetched words per stream and frame: Lyf[22], f34[7], silence


// acc[q] += w[j] * v[j][s0 + q] for the n terms of one segment, C order.  The
// segment's weights start 8-byte aligned: 8 terms = one 64-bit LDS read plus
// eight SL-float input reads, all issued before the arithmetic.
template <int SL>
struct VecT;
template <>
struct VecT<2> {
  typedef float2 T;
};
template <>
struct VecT<4> {
  typedef float4 T;
};
__device__ __forceinline__ float wbyte(uint2 w8, int u) {
  return (float)(signed char)((u < 4 ? w8.x : w8.y) >> (8 * (u & 3)));
}
template <int SL>
__device__ __forceinline__ void mac(float (&acc)[SL], float w, const typename VecT<SL>::T &v) {
  acc[0] = acc[0] + w * v.x;
  acc[1] = acc[1] + w * v.y;
  if constexpr (SL == 4) {
    acc[2] = acc[2] + w * v.z;
    acc[3] = acc[3] + w * v.w;
  }
}
template <int SL>
__device__ __forceinline__ void mac_r(float (&acc)[SL], float w, const typename VecT<SL>::T &sv,
                                      const typename VecT<SL>::T &rv) {
  acc[0] = acc[0] + w * sv.x * rv.x;
  acc[1] = acc[1] + w * sv.y * rv.y;
  if constexpr (SL == 4) {
    acc[2] = acc[2] + w * sv.z * rv.z;
    acc[3] = acc[3] + w * sv.w * rv.w;
  }
}

template <int n, int S, int SL>
__device__ __forceinline__ void mv_seg(const int8_t *__restrict__ wc, const float *vT, int s0, float (&acc)[SL]) {
  typedef typename VecT<SL>::T V;
  constexpr int nb = n / 8, r = n % 8;
#pragma unroll 1
  for (int jb = 0; jb < nb; jb++) {
    const uint2 w8 = *reinterpret_cast<const uint2 *>(wc + jb * 8);
    V v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = *reinterpret_cast<const V *>(vT + (jb * 8 + u) * S + s0);
#pragma unroll
    for (int u = 0; u < 8; u++) mac<SL>(acc, wbyte(w8, u), v[u]);
  }
  if (r) {
    const uint2 w8 = *reinterpret_cast<const uint2 *>(wc + nb * 8);
#pragma unroll
    for (int u = 0; u < r; u++) mac<SL>(acc, wbyte(w8, u), *reinterpret_cast<const V *>(vT + (nb * 8 + u) * S + s0));
  }
}

// GRU candidate recurrent segment: acc[q] += (w[j] * state[j][q]) * r[j][q]
template <int n, int S, int SL>
__device__ __forceinline__ void mv_seg_r(const int8_t *__restrict__ wc, const float *sT, const float *rT, int s0,
                                         float (&acc)[SL]) {
  typedef typename VecT<SL>::T V;
  static_assert(n % 8 == 0, "recurrent segment shape");
#pragma unroll 1
  for (int jb = 0; jb < n / 8; jb++) {
    const uint2 w8 = *reinterpret_cast<const uint2 *>(wc + jb * 8);
    V sv[8], rv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      sv[u] = *reinterpret_cast<const V *>(sT + (jb * 8 + u) * S + s0);
      rv[u] = *reinterpret_cast<const V *>(rT + (jb * 8 + u) * S + s0);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) mac_r<SL>(acc, wbyte(w8, u), sv[u], rv[u]);
  }
}

// Input of one matrix: its input-vector segments in concatenation order.
struct RnnIn {
  const float *v0, *v1, *v2;
};

template <int m, int S, int SL>
__device__ __forceinline__ void rnn_inputs(const int8_t *wc, const RnnIn &in, int s0, float (&acc)[SL]) {
  constexpr int n0 = rnnimg::kSegs[m][0];
  mv_seg<n0, S, SL>(wc, in.v0, s0, acc);
  if constexpr (m == 3 || m == 4 || m == 5 || m == 6) {
    constexpr int n1 = rnnimg::kSegs[m][1], n2 = rnnimg::kSegs[m][2];
    mv_seg<n1, S, SL>(wc + rnnimg::seg_off(m, 1), in.v1, s0, acc);
    mv_seg<n2, S, SL>(wc + rnnimg::seg_off(m, 2), in.v2, s0, acc);
  }
}

// dense layer / GRU z|r gates of image matrix m:
//   out[c][s] = act(kWs * (b[c] + sum_j w[c][j] * [in ; state][j][s]))
template <int m, int S, int G, int NT>
__device__ __forceinline__ void rnn_gates(const int8_t *W, const RnnIn &in, const float *stT, float *outT, int act,
                                          const float *tt, int tid) {
  constexpr int SL = S / G, cols = rnnimg::kCols[m];
  constexpr int ob = rnnimg::off_b(m), ow = rnnimg::off_w(m), ws = rnnimg::stride(m);
  constexpr int gst = (m == 1) ? 1 : (m == 3 || m == 5) ? 3 : -1;  // state segment of z|r matrices
  for (int t = tid; t < cols * G; t += NT) {
    const int c = t / G, s0 = (t - c * G) * SL;
    const int8_t *wc = W + ow + c * ws;
    float acc[SL];
    const float b = (float)W[ob + c];
#pragma unroll
    for (int q = 0; q < SL; q++) acc[q] = b;
    rnn_inputs<m, S, SL>(wc, in, s0, acc);
    if constexpr (gst >= 0) mv_seg<rnnimg::kSegs[m][gst], S, SL>(wc + rnnimg::seg_off(m, gst), stT, s0, acc);
#pragma unroll
    for (int q = 0; q < SL; q++) outT[c * S + s0 + q] = activate(tt, act, kWs * acc[q]);
  }
}

// GRU candidate of image matrix m: sum = b + sum_j w*in[j] + sum_j (w*state[j])*r[j];
// new[c][s] = z*state + (1-z)*act(kWs*sum) for active streams, state otherwise
template <int m, int S, int G, int NT>
__device__ __forceinline__ void rnn_cand(const int8_t *W, const RnnIn &in, const float *stT, const float *zrT,
                                         float *newT, const int *actv, int act, const float *tt, int tid) {
  constexpr int SL = S / G, cols = rnnimg::kCols[m], N = cols;
  constexpr int ob = rnnimg::off_b(m), ow = rnnimg::off_w(m), ws = rnnimg::stride(m);
  constexpr int gst = (m == 2) ? 1 : 3;
  for (int t = tid; t < cols * G; t += NT) {
    const int c = t / G, s0 = (t - c * G) * SL;
    const int8_t *wc = W + ow + c * ws;
    float acc[SL];
    const float b = (float)W[ob + c];
#pragma unroll
    for (int q = 0; q < SL; q++) acc[q] = b;
    rnn_inputs<m, S, SL>(wc, in, s0, acc);
    mv_seg_r<rnnimg::kSegs[m][gst], S, SL>(wc + rnnimg::seg_off(m, gst), stT, zrT + N * S, s0, acc);
#pragma unroll
    for (int q = 0; q < SL; q++) {
      const int o = c * S + s0 + q;
      const float sum = activate(tt, act, kWs * acc[q]);
      const float z = zrT[o];
      newT[o] = actv[s0 + q] ? z * stT[o] + (1 - z) * sum : stT[o];
    }
  }
}

template <int S, int G, int NT>
__global__ void __launch_bounds__(NT) k_rnn(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) int8_t W[rnnimg::kBytes];
  __shared__ float tt[204];
  __shared__ __attribute__((aligned(16))) float featT[44 * S];
  __shared__ float ceps[S][kCeps * kBands];
  __shared__ float dist[S][kCeps * kCeps];
  __shared__ __attribute__((aligned(16))) float doutT[24 * S], gvT[2][24 * S], gnT[2][48 * S], gdT[2][96 * S];
  __shared__ __attribute__((aligned(16))) float zrT[192 * S];
  __shared__ float lastg[S][kBands];
  __shared__ float pf[S][kRnnPf];  // features of the current frame (prefetched)
  __shared__ int memid[S], act[S], nfs[S];
  __shared__ long long fbase[S];
  __shared__ float vad_s[S];
  const int tid = threadIdx.x;
  const int sb = blockIdx.x * S;
  {
    const int4 *src = reinterpret_cast<const int4 *>(a.rnn_img);
    int4 *dst = reinterpret_cast<int4 *>(W);
    for (int i = tid; i < rnnimg::kBytes / 16; i += NT) dst[i] = src[i];
    for (int i = tid; i < 201; i += NT) tt[i] = a.plan->tansig[i];
  }
  for (int idx = tid; idx < S * kCeps * kBands; idx += NT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    ceps[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += NT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    dist[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kBands; idx += NT) {
    const int s = idx / kBands, i = idx - s * kBands;
    lastg[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] : 0.0f;
  }
  for (int idx = tid; idx < S * 96; idx += NT) {
    const int s = idx / 96, i = idx - s * 96;
    const bool ok = sb + s < a.n_streams;
    const float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) gvT[0][i * S + s] = ok ? stp[st::kVadGru + i] : 0.0f;
    if (i < 48) gnT[0][i * S + s] = ok ? stp[st::kNoiseGru + i] : 0.0f;
    gdT[0][i * S + s] = ok ? stp[st::kDenGru + i] : 0.0f;
  }
  if (tid < S) {
    const int s = sb + tid;
    const bool ok = s < a.n_streams;
    memid[tid] = ok ? reinterpret_cast<const int *>(a.state)[(size_t)s * st::kWords + st::kMemId] : 0;
    nfs[tid] = ok ? ticks_of(a, s) * a.n_channels : 0;
    fbase[tid] = (long long)s * a.V;
  }
  __syncthreads();
  int maxnf = 0;
#pragma unroll
  for (int s = 0; s < S; s++) maxnf = max(maxnf, nfs[s]);
  // prefetch lane (s, i): i < 22 Lyf, 22..28 f34, 29 silence (as 1.0 / 0.0)
  const int pfs = tid / kRnnPf, pfi = tid - pfs * kRnnPf;
  const bool pf_lane = tid < S * kRnnPf;
  auto fetch = [&](int v) -> float {
    if (!pf_lane || v >= nfs[pfs]) return 1.0f;  // past the end: treated as silent (inactive)
    const long long f = fbase[pfs] + v;
    if (pfi < kBands) return a.Lyf[f * kBands + pfi];
    if (pfi < kBands + 7) return a.f34[f * 8 + (pfi - kBands)];
    return a.silence[f] ? 1.0f : 0.0f;
  };
  // frame 0's silence must be known before its Lyf (which k_fftA leaves unwritten for silent frames) is used
  if (pf_lane) pf[pfs][pfi] = fetch(0);
  __syncthreads();
  if (tid < S) {
    act[tid] = (0 < nfs[tid]) && pf[tid][kRnnPf - 1] == 0.0f;
    if (0 < nfs[tid] && !act[tid]) a.vadf[fbase[tid]] = 0;
  }
  float pf_next = fetch(1);
  const int *ra = a.rnn_act;
  __syncthreads();
  STAMP_INIT();
  for (int v = 0; v < maxnf; v++) {
    const int cur = v & 1, nxt = cur ^ 1;
    // C: features 0..21 = DCT(Ly) (k_fftA) -> cepstral memory, deltas, the new
    //    row of the distance matrix, features 34..40 (k_pspec)
    for (int idx = tid; idx < S * (kBands + 7 + kCeps); idx += NT) {
      const int s = idx / (kBands + 7 + kCeps), i = idx - s * (kBands + 7 + kCeps);
      if (!act[s]) continue;
      const int mi = memid[s];
      const float *c0 = pf[s];  // ceps_0 (the row being written at memid)
      if (i < kBands) {
        ceps[s][mi * kBands + i] = c0[i];
        if (i < 6) {
          const float *c1 = ceps[s] + ((mi < 1) ? kCeps + mi - 1 : mi - 1) * kBands;
          const float *c2 = ceps[s] + ((mi < 2) ? kCeps + mi - 2 : mi - 2) * kBands;
          featT[i * S + s] = c0[i] + c1[i] + c2[i];
          featT[(kBands + i) * S + s] = c0[i] - c2[i];
          featT[(kBands + 6 + i) * S + s] = c0[i] - 2 * c1[i] + c2[i];
        } else {
          featT[i * S + s] = c0[i];
        }
      } else if (i < kBands + 7) {
        featT[(34 + i - kBands) * S + s] = c0[i];
      } else {
        const int j = i - kBands - 7;
        if (j != mi) {
          const float *cj = ceps[s] + j * kBands;
          float d = 0;
#pragma unroll
          for (int k = 0; k < kBands; k++) {
            const float tmp = c0[k] - cj[k];
            d += tmp * tmp;
          }
          dist[s][mi * kCeps + j] = d;
          dist[s][j * kCeps + mi] = d;
        }
      }
    }
    __syncthreads();
    RSTAMP(0);
    // D: spectral variability
    if (tid < S && act[tid]) {
      const int s = tid;
      float sv = 0;
      for (int i = 0; i < kCeps; i++) {
        float mindist = 1e15f;
        for (int j = 0; j < kCeps; j++)
          if (j != i) mindist = (mindist < dist[s][i * kCeps + j]) ? mindist : dist[s][i * kCeps + j];
        sv += mindist;
      }
      featT[41 * S + s] = (float)(sv / kCeps - 2.1);
      int mid = memid[s] + 1;
      if (mid == kCeps) mid = 0;
      memid[s] = mid;
    }
    __syncthreads();
    RSTAMP(1);
    // compute_rnn
    rnn_gates<0, S, G, NT>(W, RnnIn{featT, nullptr, nullptr}, nullptr, doutT, ra[0], tt, tid);
    __syncthreads();
    RSTAMP(2);
    rnn_gates<1, S, G, NT>(W, RnnIn{doutT, nullptr, nullptr}, gvT[cur], zrT, kActSigmoid, tt, tid);
    __syncthreads();
    RSTAMP(3);
    rnn_cand<2, S, G, NT>(W, RnnIn{doutT, nullptr, nullptr}, gvT[cur], zrT, gvT[nxt], act, ra[2], tt,
                          tid);
    __syncthreads();
    RSTAMP(4);
    // noise_input = [dense_out, vad_state, features]; vad_output alongside
    rnn_gates<3, S, G, NT>(W, RnnIn{doutT, gvT[nxt], featT}, gnT[cur], zrT, kActSigmoid, tt, tid);
    if (tid >= NT - S) {
      const int s = tid - (NT - S);
      constexpr int ob = rnnimg::off_b(8), ow = rnnimg::off_w(8);
      float sum = (float)W[ob];
      for (int j = 0; j < 24; j++) sum += (float)W[ow + j] * gvT[nxt][j * S + s];
      vad_s[s] = activate(tt, ra[8], kWs * sum);
    }
    __syncthreads();
    RSTAMP(5);
    rnn_cand<4, S, G, NT>(W, RnnIn{doutT, gvT[nxt], featT}, gnT[cur], zrT, gnT[nxt], act, ra[4],
                          tt, tid);
    __syncthreads();
    RSTAMP(6);
    // denoise_input = [vad_state, noise_state, features]
    rnn_gates<5, S, G, NT>(W, RnnIn{gvT[nxt], gnT[nxt], featT}, gdT[cur], zrT, kActSigmoid, tt,
                           tid);
    __syncthreads();
    RSTAMP(7);
    rnn_cand<6, S, G, NT>(W, RnnIn{gvT[nxt], gnT[nxt], featT}, gdT[cur], zrT, gdT[nxt], act, ra[6],
                          tt, tid);
    __syncthreads();
    RSTAMP(8);
    rnn_gates<7, S, G, NT>(W, RnnIn{gdT[nxt], nullptr, nullptr}, nullptr, zrT, ra[7], tt, tid);
    __syncthreads();
    RSTAMP(9);
    // gain smoothing g = max(g, .6*lastg) (denoise.c) and outputs of frame v;
    // the prefetched features of frame v+1 land in LDS
    for (int idx = tid; idx < S * kBands; idx += NT) {
      const int s = idx / kBands, i = idx - s * kBands;
      if (!act[s]) continue;
      const long long f = fbase[s] + v;
      const float gi = zrT[i * S + s];
      const float al = .6f * lastg[s][i];
      const float gsm = (gi > al) ? gi : al;
      lastg[s][i] = gsm;
      a.gr[f * kBands + i] = gi;
      a.gs[f * kBands + i] = gsm;
      if (i == 0) a.vadf[f] = vad_s[s];
    }
    if (pf_lane) pf[pfs][pfi] = pf_next;
    pf_next = fetch(v + 2);
    __syncthreads();
    RSTAMP(10);
    if (tid < S) {
      const bool valid = v + 1 < nfs[tid];
      act[tid] = valid && pf[tid][kRnnPf - 1] == 0.0f;
      if (valid && !act[tid]) a.vadf[fbase[tid] + v + 1] = 0;  // silent: X passes through, state untouched
    }
    __syncthreads();
    RSTAMP(11);
  }
  STAMP_FLUSH(0, 12);
  const int fin = maxnf & 1;  // buffer holding the latest GRU states
  for (int idx = tid; idx < S * kCeps * kBands; idx += NT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    if (sb + s < a.n_streams && nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] = ceps[s][i];
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += NT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    if (sb + s < a.n_streams && nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] = dist[s][i];
  }
  for (int idx = tid; idx < S * kBands; idx += NT) {
    const int s = idx / kBands, i = idx - s * kBands;
    if (sb + s < a.n_streams && nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] = lastg[s][i];
  }
  for (int idx = tid; idx < S * 96; idx += NT) {
    const int s = idx / 96, i = idx - s * 96;
    if (sb + s >= a.n_streams || nfs[s] <= 0) continue;
    float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) stp[st::kVadGru + i] = gvT[fin][i * S + s];
    if (i < 48) stp[st::kNoiseGru + i] = gnT[fin][i * S + s];
    stp[st::kDenGru + i] = gdT[fin][i * S + s];
  }
  if (tid < S && sb + tid < a.n_streams && nfs[tid] > 0)
    reinterpret_cast<int *>(a.state)[(size_t)(sb + tid) * st::kWords + st::kMemId] = memid[tid];
}

// ---------------------------------------------------------------------------
// k_synth: pitch_filter + gain application (no recurrence left once g / the
// smoothed gains are known), then the inverse transform (forward FFT of the
// Hermitian extension) and the synthesis window
// ---------------------------------------------------------------------------
template <int F>
__global__ void __launch_bounds__(256) k_synth(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 W[F][kWin];
  __shared__ __attribute__((aligned(16))) float2 Xl[F][kFreq + 1];
  __shared__ BandTab T;
  __shared__ float rr[F][kBands + 2], nrm[F][kBands + 2], gs[F][kBands + 2], newE[F][kBands + 2];
  __shared__ int fidx[F], fil[F];
  const int tid = threadIdx.x;
  FrameCtx cx;
  frame_ctx_load(cx, a.plan, tid);
  bandtab_load(T, a.plan, tid, 256);
  const long long ngroups = ((long long)a.n_streams * a.V + F - 1) / F;
  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    group_frames<F>(a, g, tid, fidx);
    __syncthreads();
    if (tid < F) fil[tid] = fidx[tid] >= 0 && !a.silence[fidx[tid]];  // silent frames: X passes through
    for (int idx = tid; idx < F * kFreq; idx += 256) {
      const int fr = idx / kFreq, k = idx - fr * kFreq;
      if (fidx[fr] >= 0) Xl[fr][k] = a.X[(size_t)fidx[fr] * kFreq + k];
    }
    __syncthreads();
    if (tid < F * kBands) {
      const int fr = tid / kBands, i = tid - fr * kBands;
      if (fil[fr]) {
        const size_t o = (size_t)fidx[fr] * kBands + i;
        const float Exp = a.Exp[o], gg = a.gr[o], Ex = a.Ex[o], Ep = a.Ep[o];
        float r;
        if (Exp > gg)
          r = 1;
        else
          r = (float)((double)((Exp * Exp) * (1 - (gg * gg))) / (.001 + (double)((gg * gg) * (1 - (Exp * Exp)))));
        float cl = (0 > r) ? 0 : r;
        cl = (1 < cl) ? 1 : cl;
        r = (float)sqrt((double)cl);
        r = (float)((double)r * sqrt((double)Ex / (1e-8 + (double)Ep)));
        rr[fr][i] = r;
        gs[fr][i] = a.gs[o];
      }
    }
    __syncthreads();
    for (int idx = tid; idx < F * kFreq; idx += 256) {
      const int fr = idx / kFreq, k = idx - fr * kFreq;
      if (fil[fr]) {
        const float rf = interp_gain_t(rr[fr], T, k);
        const float2 pk = a.P[(size_t)fidx[fr] * kFreq + k];
        Xl[fr][k].x += rf * pk.x;
        Xl[fr][k].y += rf * pk.y;
      }
    }
    __syncthreads();
    if (tid < F * kBands) {
      const int fr = tid / kBands, i = tid - fr * kBands;
      if (fil[fr]) {
        newE[fr][i] = band_sum_t(Xl[fr], Xl[fr], T, i);
        nrm[fr][i] = (float)sqrt((double)a.Ex[(size_t)fidx[fr] * kBands + i] / (1e-8 + (double)newE[fr][i]));
      }
    }
    __syncthreads();
    for (int idx = tid; idx < F * kFreq; idx += 256) {
      const int fr = idx / kFreq, k = idx - fr * kFreq;
      if (fil[fr]) {
        const float nf = interp_gain_t(nrm[fr], T, k);
        float2 val = Xl[fr][k];
        val.x *= nf;
        val.y *= nf;
        const float gf = interp_gain_t(gs[fr], T, k);
        val.x *= gf;
        val.y *= gf;
        Xl[fr][k] = val;
      }
    }
    __syncthreads();
#pragma unroll
    for (int fr = 0; fr < F; fr++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = tid + 256 * r;
        if (i < kWin) {
          float2 val;
          if (i < kFreq) {
            val = Xl[fr][i];
          } else {
            const float2 c = Xl[fr][kWin - i];
            val = make_float2(c.x, -c.y);
          }
          W[fr][cx.dst[r]] = make_float2(kScale960 * val.x, kScale960 * val.y);
        }
      }
    }
    __syncthreads();
    fft960_run<F>(cx.tw, W, tid);
#pragma unroll
    for (int fr = 0; fr < F; fr++) {
      const int f = fidx[fr];
      if (f < 0) continue;
      float *y = a.ys + (size_t)f * kWin;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = tid + 256 * r;
        if (i < kWin) {
          const float yv = (i == 0) ? kWin * W[fr][0].x : kWin * W[fr][kWin - i].x;
          y[i] = yv * cx.win[r];
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_ola: out = x[0..479] + synthesis_mem; denoised * 1/32767; re-block ring;
// per-tick vad_low (min over channels in channel order)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ola(StagedArgs a) {
  const int C = a.n_channels, V = a.V;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)a.n_streams * V * kFrame;
  if (gid >= total) return;
  const int i = (int)(gid % kFrame);
  const long long fv = gid / kFrame;
  const int s = (int)(fv / V), v = (int)(fv - (long long)s * V);
  const int nt = ticks_of(a, s);
  if (v >= nt * C) return;
  const int t = v / C, c = v - t * C;
  const float *stp = a.state + (size_t)s * st::kWords;
  const size_t f = (size_t)s * V + v;
  const float prev = (v == 0) ? stp[st::kSyn + i] : a.ys[(f - 1) * kWin + kFrame + i];
  const float o = a.ys[f * kWin + i] + prev;
  const float dn = a.raw_s16 ? o : o * (1.0f / (float)32767);
  const int frames_done = reinterpret_cast<const int *>(stp)[st::kFramesDone];
  const long long absi = (long long)(frames_done + t) * kFrame + i;
  a.ring[((size_t)s * C + c) * a.ring_len + (size_t)(absi % a.ring_len)] = dn;
  if (a.out_den) a.out_den[(((size_t)t * a.n_streams + s) * C + c) * kFrame + i] = dn;
  if (i == 0 && c == 0) {
    float vad_low = 1;
    for (int cc = 0; cc < C; cc++) {
      const float vv = a.vadf[(size_t)s * V + t * C + cc];
      if (vv < vad_low) vad_low = vv;
    }
    a.out_vad[(size_t)t * a.n_streams + s] = vad_low;
  }
}

// ---------------------------------------------------------------------------
// k_winmeta: window completion bookkeeping (VAD.zig:298-348), lane per stream
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_winmeta(StagedArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_streams) return;
  const int nt = ticks_of(a, s);
  int *wt = a.win_tick + (size_t)s * a.wmax;
  long long *wsx = a.win_start + (size_t)s * a.wmax;
  int j = 0;
  if (nt > 0) {
    float *stp = a.state + (size_t)s * st::kWords;
    int *istp = reinterpret_cast<int *>(stp);
    int fd = istp[st::kFramesDone];
    float vol = stp[st::kVolAcc];
    const int FB = a.plan->nfft_b;
    for (int t = 0; t < nt; t++) {
      const size_t o = (size_t)t * a.n_streams + s;
      const float ratio = a.ratio[o];
      const long long a0 = (long long)fd * kFrame;
      const long long wdone = a0 / FB;
      const long long next_end = (wdone + 1) * FB;
      const bool complete = a0 + kFrame >= next_end;
      if (complete) {
        const int r = (int)(next_end - a0);
        vol += ratio * ((float)r / (float)FB);
        a.out_win_ratio[o] = vol;
        a.out_win_vad[o] = a.out_vad[o];
        vol = 0;
        if (kFrame - r > 0) vol += ratio * ((float)(kFrame - r) / (float)FB);
        wt[j] = t;
        wsx[j] = wdone * FB;
        j++;
      } else {
        vol += ratio * ((float)kFrame / (float)FB);
        a.out_win_ratio[o] = 0.0f;
        a.out_win_vad[o] = 0.0f;
      }
      a.out_win_flag[o] = complete ? 1 : 0;
      fd++;
    }
    istp[st::kFramesDone] = fd;
    stp[st::kVolAcc] = vol;
    // synthesis_mem for the next launch = second half of the last frame's window
    const float *yl = a.ys + ((size_t)s * a.V + (size_t)nt * a.n_channels - 1) * kWin + kFrame;
    for (int i = 0; i < kFrame; i++) stp[st::kSyn + i] = yl[i];
  }
  for (; j < a.wmax; j++) wt[j] = -1;
}

// ---------------------------------------------------------------------------
// k_fftb: one workgroup per (stream, completed window): FFT B per channel
// ---------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(NT) k_fftb(StagedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 W[kMaxFftB / 2];
  __shared__ float mag[256];
  const int tid = threadIdx.x;
  const int s = blockIdx.x / a.wmax, j = blockIdx.x - s * a.wmax;
  if (s >= a.n_streams) return;
  const int t = a.win_tick[(size_t)s * a.wmax + j];
  if (t < 0) return;
  const long long wstart = a.win_start[(size_t)s * a.wmax + j];
  const Plan *__restrict__ P = a.plan;
  const int nc = P->ncfft_b, C = a.n_channels;
  const float2 *__restrict__ twb = reinterpret_cast<const float2 *>(P->twb);
  const float2 *__restrict__ sup = reinterpret_cast<const float2 *>(P->superb);
  const size_t o = (size_t)t * a.n_streams + s;
  for (int c = 0; c < C; c++) {
    const float *ring = a.ring + ((size_t)s * C + c) * a.ring_len;
    for (int k = tid; k < nc; k += NT) {
      const int n = P->permb[k];
      const float t0 = ring[(wstart + 2 * n) % a.ring_len] * P->hannb[2 * n];
      const float t1 = ring[(wstart + 2 * n + 1) % a.ring_len] * P->hannb[2 * n + 1];
      W[k] = make_float2(t0, t1);
    }
    __syncthreads();
    for (int stg = 0, m = 1; stg < P->stages_b; stg++, m *= 4) {
      const int fstride = nc / (4 * m);
      for (int q = tid; q < nc / 4; q += NT) {
        const int blk = q / m, u = q - blk * m;
        bfly4(W + blk * 4 * m + u, m, twb[u * fstride], twb[2 * u * fstride], twb[3 * u * fstride]);
      }
      __syncthreads();
    }
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
        const int kk = (k < nc / 2) ? k : nc - k;
        const float2 fpk = W[kk];
        const float2 fpnk = make_float2(W[nc - kk].x, -W[nc - kk].y);
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
    __syncthreads();
    if (tid < a.n_bands) {
      float acc = 0.0f;
      for (int k = a.band_lo[tid]; k <= a.band_hi[tid]; k++) acc += mag[k - lo];
      a.out_band[(o * C + c) * a.n_bands + tid] = acc;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_vadm: VADMachine.run (VADMachine.zig:126-230) for every completed FFT-B
// window of the push, one lane per stream, every attached machine.
// RollingAverage.avg (RollingAverage.zig:34-56) recomputes the mean over the
// whole buffer in array order on every push, in f64 - reproduced as is (an
// incremental mean would round differently).  Buffers are stored [i][stream]
// so the lanes of a wave read one contiguous line per term.
// ---------------------------------------------------------------------------
// Short rolling averages: the plain recompute.
__device__ __forceinline__ double ra_push(float *buf, int B, int n, unsigned &widx, unsigned &count, double &last,
                                          int &has, float sample) {
  buf[(size_t)widx * B] = sample;  // stored as f32: (double)f32 is exact
  widx = (widx + 1) % (unsigned)n;
  if (count < (unsigned)n) count++;
  double acc = 0.0;
  const double scalar = 1.0 / (double)count;
  for (unsigned i = 0; i < count; i++) acc += (double)buf[(size_t)i * B] * scalar;
  last = acc;
  has = 1;
  return acc;
}

// The long-term average (4218 entries by default).  Same operation sequence as
// the full recompute, two savings that keep it bit-identical:
//  * once the buffer is full the scalar 1/n no longer changes, so the running
//    sum over the entries before the write position is exactly what the
//    previous pass had accumulated there (those entries have not changed) -
//    the pass starts from that cached prefix;
//  * entries are read 32 ahead of the f64 add chain (register double buffer),
//    so the chain does not wait on memory per term.
// acc += entry[i] * scalar for i in [i0, i1), C order; entries are pushed f32
// values (read 8 ahead of the add chain) or, for never-written entries, the
// initial average (a double).
__device__ __forceinline__ double lt_sum(double acc, const float *buf, size_t bs, unsigned i0, unsigned i1,
                                         double scalar) {
  unsigned i = i0;
  for (; i + 8 <= i1; i += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = buf[(size_t)(i + u) * bs];
    double p[8];
#pragma unroll
    for (int u = 0; u < 8; u++) p[u] = (double)v[u] * scalar;
#pragma unroll
    for (int u = 0; u < 8; u++) acc += p[u];
  }
  for (; i < i1; i++) acc += (double)buf[(size_t)i * bs] * scalar;
  return acc;
}
__device__ __forceinline__ double lt_sum_init(double acc, double term, unsigned n) {
  for (unsigned i = 0; i < n; i++) acc += term;
  return acc;
}
__device__ __forceinline__ double lt_range(double acc, const float *buf, size_t bs, unsigned p, unsigned q,
                                           unsigned nw, double init, double scalar) {
  const unsigned mid = min(max(nw, p), q);  // [p, mid) written, [mid, q) initial
  acc = lt_sum(acc, buf, bs, p, mid, scalar);
  return lt_sum_init(acc, init * scalar, q - mid);
}

// The long-term average (4218 entries by default).  Same operation sequence as
// the full recompute, with one exact saving: once the buffer is full the
// scalar 1/n no longer changes, so the running sum over the entries before the
// write position is exactly what the previous pass had accumulated there
// (those entries have not changed) - the pass starts from that cached prefix.
// Entries never written since the machine started hold the initial average
// (a double, RollingAverage.zig init): entry i is a pushed f32 iff i < nw.
__device__ __forceinline__ double ra_push_long(float *buf, size_t bs, int n, unsigned &widx, unsigned &count,
                                               unsigned &nw, double init, double &last, int &has, double &pre,
                                               int &pre_ok, float sample) {
  const unsigned w = widx;
  buf[(size_t)w * bs] = sample;
  widx = (w + 1) % (unsigned)n;
  if (count < (unsigned)n) count++;
  if (nw < (unsigned)n) nw++;
  const double scalar = 1.0 / (double)count;
  const unsigned start = pre_ok ? w : 0u;
  double acc = pre_ok ? pre : 0.0;
  const unsigned save_at = widx;  // the next pass starts at the next write position
  double save = 0.0;              // (save_at == 0: it starts from 0.0)
  if (save_at > start && save_at < count) {
    acc = lt_range(acc, buf, bs, start, save_at, nw, init, scalar);
    save = acc;
    acc = lt_range(acc, buf, bs, save_at, count, nw, init, scalar);
  } else {
    if (save_at == start) save = acc;
    acc = lt_range(acc, buf, bs, start, count, nw, init, scalar);
  }
  pre = save;
  pre_ok = count == (unsigned)n;
  last = acc;
  has = 1;
  return acc;
}

constexpr int kVadmS = 8;        // streams per workgroup
constexpr int kVadmLds = 4225;   // LDS-resident long-term buffer length (odd: no bank conflicts)

// One machine over all completed windows of the push for one stream; `lt`
// points at entry 0 of the stream's long-term buffer, `lts` is its stride.
__device__ void vadm_stream(const StagedArgs &a, int m, int s, float *lt, size_t lts) {
  const int B = a.n_streams, C = a.n_channels, nb = a.n_bands;
  const int nt = ticks_of(a, s);
  const unsigned long long fft = (unsigned long long)a.plan->nfft_b;
  enum { kClosed = 0, kOpening = 1, kOpen = 2, kClosing = 3 };
  const VadmConst &K = a.vadm.c[m];
  VadmState S = a.vadm.st[(size_t)m * B + s];
  float *st = a.vadm.buf + K.st_off + s, *rb = a.vadm.buf + K.r_off + s;
  VadmSeg *seg = a.vadm.seg + ((size_t)m * B + s) * a.vadm.seg_cap;
  for (int t = 0; t < nt; t++) {
    const size_t o = (size_t)t * B + s;
    if (!a.out_win_flag[o]) continue;
    const unsigned long long index = S.windows_done * fft;
    S.windows_done++;
    float min_v = 999, max_v = 0;
    for (int c = 0; c < C; c++) {
      const float v = a.out_band[(o * C + c) * nb + K.slot];
      if (v < min_v) min_v = v;
      if (v > max_v) max_v = v;
    }
    const float vad = a.out_win_vad[o], vr = a.out_win_ratio[o];
    const double st_avg = ra_push(st, B, K.n_st, S.st_widx, S.st_count, S.st_last, S.st_has, min_v);
    const double r_avg = ra_push(rb, B, K.n_r, S.r_widx, S.r_count, S.r_last, S.r_has, vr);
    double base;
    if (S.lt_has)
      base = S.lt_last;
    else if (K.has_init)
      base = K.init;
    else
      base = st_avg;
    const double threshold = base * (double)K.thr_factor;
    const bool met = st_avg > threshold && r_avg > (double)K.ratio_thr;
    if (!met)
      ra_push_long(lt, lts, K.n_lt, S.lt_widx, S.lt_count, S.lt_nw, K.init, S.lt_last, S.lt_has, S.lt_pre,
                   S.lt_pre_ok, min_v);
    const int from = S.state;
    bool ended = false;
    switch (from) {
      case kClosed:
        if (met) {
          S.state = kOpening;
          S.speech_start = index;
        }
        break;
      case kOpening:
        if (met && index - S.speech_start >= K.min_open)
          S.state = kOpen;
        else if (!met)
          S.state = kClosed;
        break;
      case kOpen:
        if (!met) {
          S.state = kClosing;
          S.speech_end = index;
        }
        break;
      default:  // kClosing
        if (met) {
          S.state = kOpen;
        } else if (index - S.speech_end >= K.max_gap) {
          S.state = kClosed;
          ended = true;
        }
        break;
    }
    if (ended) {  // onSpeechEnd (before the tracking update of this window, as in VADMachine.zig)
      const unsigned long long len = S.speech_end - S.speech_start;
      const float len_rt = (float)len / K.sr;
      if (len_rt >= K.min_dur) {
        if (S.n_segs < (unsigned)a.vadm.seg_cap) {
          VadmSeg g;
          g.sample_from = K.rec_pad > S.speech_start ? 0ull : S.speech_start - K.rec_pad;
          g.sample_to = S.speech_end + K.rec_pad;
          g.debug_rnn_vad = S.rnn_vad / (float)S.rnn_vad_count;
          g.debug_avg_speech_vol_ratio = S.vol_ratio / (float)S.vol_ratio_count;
          seg[S.n_segs] = g;
        }
        S.n_segs++;
      }
    }
    // track(vad, vr, from, to)
    if (from == kClosed && S.state == kOpening) {
      S.rnn_vad = vad;
      S.rnn_vad_count = 1;
      S.vol_ratio = vr;
      S.vol_ratio_count = 1;
    } else if (from == kOpening || from == kOpen) {
      S.rnn_vad += vad;
      S.rnn_vad_count += 1;
      S.vol_ratio += vr;
      S.vol_ratio_count += 1;
    }
  }
  a.vadm.st[(size_t)m * B + s] = S;
}

// One 64-thread workgroup per 8 streams.  Default-length long-term buffers
// (4218 entries) of the 8 streams live in LDS for the whole push: loaded once
// with all lanes, walked by the 8 stream lanes window after window, stored
// back once.  Longer configurations walk them in HBM.  (The engine normally
// runs k_vadm_hbm instead, on a side stream overlapped with the next push.)
__global__ void __launch_bounds__(64) k_vadm(StagedArgs a) {
  __shared__ float ltl[kVadmS][kVadmLds];
  const int tid = threadIdx.x, sb = blockIdx.x * kVadmS;
  const int B = a.n_streams, ns = min(kVadmS, B - sb);
  if (ns <= 0) return;
  for (int m = 0; m < a.vadm.n; m++) {
    const VadmConst &K = a.vadm.c[m];
    if (K.n_lt <= kVadmLds) {
      for (int idx = tid; idx < ns * K.n_lt; idx += 64) {
        const int i = idx / ns, j = idx - i * ns;
        ltl[j][i] = a.vadm.buf[K.lt_off + (size_t)i * B + sb + j];
      }
      __syncthreads();
      if (tid < ns && ticks_of(a, sb + tid) > 0) vadm_stream(a, m, sb + tid, ltl[tid], 1);
      __syncthreads();
      for (int idx = tid; idx < ns * K.n_lt; idx += 64) {
        const int i = idx / ns, j = idx - i * ns;
        a.vadm.buf[K.lt_off + (size_t)i * B + sb + j] = ltl[j][i];
      }
      __syncthreads();
    } else if (tid < ns && ticks_of(a, sb + tid) > 0) {
      vadm_stream(a, m, sb + tid, a.vadm.buf + K.lt_off + sb + tid, (size_t)B);
    }
  }
}

// ---------------------------------------------------------------------------
// launcher
// ---------------------------------------------------------------------------
const char *staged_kernel_name(int i) {
  static const char *const names[kStagedKernels] = {"k_prep2", "k_fftA",  "k_pitch", "k_select", "k_pspec",
                                                     "k_rnn",   "k_synth", "k_ola",   "k_winmeta", "k_fftb"};
  return (i >= 0 && i < kStagedKernels) ? names[i] : nullptr;
}

namespace {
// persistent grids: exactly the resident capacity (blocks per CU from the
// occupancy calculator x CUs), so no workgroup starts late and leaves a tail
template <typename K>
int resident_blocks(K kernel, int threads, int n_cu) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  return per_cu * n_cu;
}
}  // namespace

hipError_t launch_staged(const StagedArgs &a, int n_cu, hipStream_t stream, hipEvent_t *ev) {
  constexpr int NT = 256;
  constexpr int FF = kFftFrames;
  static const int g_fftA = resident_blocks(k_fftA<FF>, 256, n_cu);
  static const int g_pspec = resident_blocks(k_pspec<FF>, 256, n_cu);
  static const int g_synth = resident_blocks(k_synth<FF>, 256, n_cu);
  static const int g_pitch4 = resident_blocks(k_pitch<4>, 256, n_cu);
  static const int g_pitch8 = resident_blocks(k_pitch<8>, 256, n_cu);
  // lane-per-stream kernels: 16 streams per workgroup spreads the serial
  // chains over more CUs (each chain is latency-bound, not lane-bound)
  const int lane_blocks = (a.n_streams + 15) / 16;
  const long long frames = (long long)a.n_streams * a.V;
  auto grid = [&](long long units, int resident) { return dim3((unsigned)std::min<long long>(units, resident)); };
  (void)hipGetLastError();
  auto rec = [&](int k) {
    if (ev) (void)hipEventRecord(ev[k], stream);
  };
  rec(0);
  {
    const int S = kPrepSlots / a.n_channels;
    hipLaunchKernelGGL(k_prep2, dim3((a.n_streams + S - 1) / S), dim3(256), 0, stream, a);
  }
  rec(1);
  const long long fgroups = (frames + FF - 1) / FF;
  hipLaunchKernelGGL(k_fftA<FF>, grid(fgroups, g_fftA), dim3(NT), 0, stream, a);
  rec(2);
  {
    // frames per k_pitch workgroup: 4 (default) or 8 (FVAD_PITCH_FRAMES=8, tuning only)
    static const int fp = [] {
      const char *e = getenv("FVAD_PITCH_FRAMES");
      return (e && atoi(e) == 8) ? 8 : kPitchFrames;
    }();
    const long long groups = (frames + fp - 1) / fp;
    if (fp == 8)
      hipLaunchKernelGGL(k_pitch<8>, grid(groups, g_pitch8), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL(k_pitch<4>, grid(groups, g_pitch4), dim3(256), 0, stream, a);
  }
  rec(3);
  hipLaunchKernelGGL(k_select, dim3(lane_blocks), dim3(16), 0, stream, a);
  rec(4);
  hipLaunchKernelGGL(k_pspec<FF>, grid(fgroups, g_pspec), dim3(NT), 0, stream, a);
  rec(5);
  hipLaunchKernelGGL((k_rnn<kRnnS, kRnnG, kRnnNT>), dim3((a.n_streams + kRnnS - 1) / kRnnS), dim3(kRnnNT), 0,
                     stream, a);
  rec(6);
  hipLaunchKernelGGL(k_synth<FF>, grid(fgroups, g_synth), dim3(NT), 0, stream, a);
  rec(7);
  const long long ola_threads = frames * kFrame;
  hipLaunchKernelGGL(k_ola, dim3((unsigned)((ola_threads + 255) / 256)), dim3(256), 0, stream, a);
  rec(8);
  hipLaunchKernelGGL(k_winmeta, dim3(lane_blocks), dim3(16), 0, stream, a);
  rec(9);
  hipLaunchKernelGGL(k_fftb<NT>, dim3(a.n_streams * a.wmax), dim3(NT), 0, stream, a);
  rec(10);
  return hipGetLastError();
}

// k_vadm_hbm: the same machine, long-term buffers walked in HBM, no LDS, 16
// lanes per workgroup: a light kernel that co-runs with the next push's
// pipeline on the engine's side stream.
__global__ void __launch_bounds__(64) k_vadm_hbm(StagedArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_streams || ticks_of(a, s) <= 0) return;
  for (int m = 0; m < a.vadm.n; m++)
    vadm_stream(a, m, s, a.vadm.buf + a.vadm.c[m].lt_off + s, (size_t)a.n_streams);
}

hipError_t launch_vadm(const StagedArgs &a, bool overlap, hipStream_t stream) {
  (void)hipGetLastError();
  if (overlap)
    hipLaunchKernelGGL(k_vadm_hbm, dim3((a.n_streams + 15) / 16), dim3(16), 0, stream, a);
  else
    hipLaunchKernelGGL(k_vadm, dim3((a.n_streams + kVadmS - 1) / kVadmS), dim3(64), 0, stream, a);
  return hipGetLastError();
}

}  // namespace fvad
