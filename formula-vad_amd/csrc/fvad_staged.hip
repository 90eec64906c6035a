// Staged (time-parallel) MI355X pipeline for the Formula-VAD hot path.
//
// rnnoise_process_frame splits into work that depends only on the input
// samples of the (virtual, channel-interleaved) stream and a thin recurrence:
//
//   k_prep3   lane/stream   HP biquad (serial IIR), s16 scaling, RMS volume
//                           ratio; x written stream-contiguous with 1248 samples
//                           of pitch history in front of the launch's frames
//   k_fftAw   wave/frame    analysis window + FFT A, band energies Ex, the
//                           log/floor chain (Ly, E, silence gate), DCT(Ly)
//                           (fvad_wave.hip)
//   k_plpc    lane/frame    pitch_downsample (x_lp, autocorr, LPC, FIR5) and
//                           the serial energy recurrences Syy and xx
//   k_pcorr   wg/8 frames   coarse and fine xcorr + find_best_pitch, every
//                           remove_doubling inner product for every candidate
//                           period (fvad_pitch.hip)
//   k_select  lane/(stream, candidate)  remove_doubling's sequential candidate
//                           selection (needs last_period / last_gain) -> pitch
//   k_pspecw  wave/frame    pitch window + FFT A -> P, Ep, Exp, DCT(Exp)
//   k_rnn3    wg/8 streams  the true recurrence: cepstral memory, spectral
//                           variability, GRU stack, gain smoothing
//   k_synthw  wave/frame    pitch filter, gains, Hermitian extension + FFT A +
//                           synthesis window
//   k_ola     per sample    overlap-add, 1/32767, re-block ring, per-tick vad
//   k_winmeta lane/stream   window completion, share-weighted ratio, state
//   k_fftbw   wave/window   FFT B (kissfft radix-4), magnitudes, band sums
//                           (k_fftb, workgroup per window, for fft_size 512)
//   k_vadm_hbm lane/stream  VADMachine.run per completed window (side stream)
//
// The wave kernels are persistent (batches of frames from per-XCD queues) so
// per-lane table values stay in registers across frames.  All arithmetic
// reproduces the oracle's operation order (see fvad_kernels.hip), so results
// are bit-identical to the fused kernel and the CPU oracle.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fvad_device.h"
#include "fvad_exact.h"
#include "fvad_internal.h"
#include "fvad_staged.h"
#include "fvad_staged_dev.h"

namespace fvad {

namespace {
// LDS row pitch of the 960-point transforms (float2): frames 16 banks apart,
// so band-sum lanes of different frames reading the same bin do not conflict
constexpr int kWinP = kWin + 8;
// after a forward transform, bins >= 481 of a row are dead: band terms go there
constexpr int kTermOff = 964;  // float offset in a W row (16-byte aligned; + 800 <= 2 * kWinP)
static_assert(kTermOff >= 2 * kFreq && kTermOff % 4 == 0 && kTermOff + 800 <= 2 * kWinP, "band term area");

}  // namespace

// ---------------------------------------------------------------------------
// k_prep3: high-pass biquad (a serial IIR with f64 intermediates: no exact
// parallel form exists, so one lane walks one stream), s16 scaling, RMS volume
// ratio, pitch history.  It uses no LDS and one wave per 64 channel-slots:
// the engine runs it on its own stream beside the previous push's kernels
// (xs, ratio and ticks are double-buffered), where it must not take the LDS
// or the wave slots those kernels are sized for.  Lane = stream: the biquad
// chain straight from the input rows (16-byte loads through an 8-deep
// prefetch ring, 16-byte stores into the stream's xs row), and beside it, off
// the chain's dependency path, each channel's RMS sum and per tick the volume
// ratio.  (A second wave that re-read the input for the RMS sums cost the
// co-running kernels 0.17 ms per push.)
// ---------------------------------------------------------------------------
#ifndef FVAD_PREP_SLOTS
#define FVAD_PREP_SLOTS 64
#endif
constexpr int kPrepSlots = FVAD_PREP_SLOTS;  // channel-slots per workgroup (32 stereo streams)
__host__ __device__ constexpr int prep_streams(int C) { return kPrepSlots / C < 64 ? kPrepSlots / C : 64; }
#ifndef FVAD_PREP_RING
#define FVAD_PREP_RING 8
#endif
constexpr int kPrepRing = FVAD_PREP_RING;  // float4 loads in flight per lane
// blocks per trip of the chain loop: the compiler's wait at the loop header
// drains every load and store in flight, so it is paid once per trip
#ifndef FVAD_PREP_UNROLL
#define FVAD_PREP_UNROLL 4
#endif
static_assert((kFrame / 4) % kPrepRing == 0, "prep ring must divide a frame");

// One lane walks its stream's input in blocks of kPrepRing float4 chunks: per
// tick the C * 480 samples of stream s are contiguous, ticks B * C * 480
// floats apart, and a tick holds a whole number of blocks, so a block is one
// base pointer and kPrepRing immediate offsets.  The next block's chunks load
// while this block's are filtered (the last block reloads itself).
// A chunk is 4 samples: a float4 of the float input, or a uint2 of 16-bit
// samples k (fvad_engine_submit_i16), read as k / 32768.0f -- k_pcm16's
// conversion, exact in f32, done here so the 16-bit push needs no float copy
// of its input (half k_prep3's input bytes, and no conversion kernel).
__device__ __forceinline__ float4 chunk4(float4 v) { return v; }
__device__ __forceinline__ float4 chunk4(uint2 v) {
  constexpr float k = 1.0f / 32768.0f;
  return make_float4((float)(short)(v.x & 0xffffu) * k, (float)(short)(v.x >> 16) * k,
                     (float)(short)(v.y & 0xffffu) * k, (float)(short)(v.y >> 16) * k);
}
template <bool Scaled, typename In>
__device__ __forceinline__ void prep_chain(const StagedArgs &a, const void *src, int s, int nt, float &mem0,
                                           float &mem1) {
  constexpr int kChunksCh = kFrame / 4;  // chunks of one channel's frame
  static_assert(kChunksCh % kPrepRing == 0, "ring blocks end at channel boundaries");
  const int C = a.n_channels;
  const int per_tick = C * kChunksCh;
  const int bpt = per_tick / kPrepRing;  // blocks per tick
  const int nb = nt * bpt;
  const size_t tick_stride = (size_t)a.n_streams * per_tick;  // in chunks
  const In *tick_row = reinterpret_cast<const In *>(src) + (size_t)s * per_tick;
  float4 *dst = reinterpret_cast<float4 *>(a.xs + (size_t)s * a.L + kHist);
  In ring[kPrepRing];
#pragma unroll
  for (int u = 0; u < kPrepRing; u++) ring[u] = tick_row[u];
  int rn = 1;  // block within the tick of the next block
  const float b0 = -2.0f, b1 = 1.0f, a0 = -1.99599f, a1 = 0.99600f;
  const float scalar = (float)32767;
  // b*x and a*y are exact in double (24-bit x 24-bit significands), so one
  // fma rounds b*x - a*y exactly once, as the C expression does
  auto step = [&](float v) -> float {
    const float xi = Scaled ? v * scalar : v;
    const float yi = xi + mem0;
    const double yd = (double)yi;
    mem0 = (float)((double)mem1 + __builtin_fma(-(double)a0, yd, b0 * (double)xi));
    mem1 = (float)__builtin_fma(-(double)a1, yd, b1 * (double)xi);
    return yi;
  };
  // RMS volume (VAD.zig:253-272): sum of squares of the raw samples of each
  // channel's frame in sample order, vol = sqrt(sum / 480), ratio = min / max
  // over the stream's channels in channel order
  float sum = 0, vmin = 1, vmax = 0;
  int jt = 0, t = 0;  // chunk within the tick, tick
#pragma unroll FVAD_PREP_UNROLL
  for (int b = 0; b < nb; b++) {
    if (rn == bpt && b + 1 < nb) {
      rn = 0;
      tick_row += tick_stride;
    }
    const In *q = tick_row + (b + 1 < nb ? rn : rn - 1) * kPrepRing;
    rn++;
#pragma unroll
    for (int u = 0; u < kPrepRing; u++) {
      const float4 x = chunk4(ring[u]);
      ring[u] = q[u];
      float4 y;
      y.x = step(x.x);
      y.y = step(x.y);
      y.z = step(x.z);
      y.w = step(x.w);
      dst[b * kPrepRing + u] = y;
      sum += x.x * x.x;
      sum += x.y * x.y;
      sum += x.z * x.z;
      sum += x.w * x.w;
    }
    jt += kPrepRing;
    if (jt % kChunksCh == 0) {
      const float vol = sqrtf(sum / (float)kFrame);
      sum = 0;
      if (vol < vmin) vmin = vol;
      if (vol > vmax) vmax = vol;
      if (jt == per_tick) {
        a.ratio[(size_t)t * a.n_streams + s] = (vmax == 0) ? 0 : vmin / vmax;
        vmin = 1;
        vmax = 0;
        jt = 0;
        t++;
      }
    }
  }
}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(64) k_prep3(StagedArgs a) {
  const int tid = threadIdx.x, lane = tid;
  const int C = a.n_channels, S = prep_streams(C), sb = blockIdx.x * S;
  const int ns = min(S, a.n_streams - sb);  // streams in this workgroup
  if (ns <= 0) return;
  // pitch history of every stream -> xs[s][0..1248), and its x_lp values
  // (the first frame's x_lp[1..623]; k_fftAw writes the rest): flat over the
  // workgroup's streams, each lane's loads in batches of 8 before their
  // stores (a stream with no ticks gets a copy nobody reads)
  {
    constexpr int kH4 = kHist / 4, B = 8;
    f4 v[B];  // (a native vector: arrays of float4 structs stayed in scratch)
    float w[B];
    for (int i0 = 0; i0 < ns * kH4; i0 += 64 * B) {
#pragma unroll
      for (int u = 0; u < B; u++) {  // (clamped: every load unconditional)
        const int i = min(i0 + lane + 64 * u, ns * kH4 - 1), s = i / kH4, j = i - s * kH4;
        v[u] = reinterpret_cast<const f4 *>(a.state + (size_t)(sb + s) * st::kWords + st::kPitch + kFrame)[j];
      }
#pragma unroll
      for (int u = 0; u < B; u++) {
        const int i = i0 + lane + 64 * u, s = i / kH4, j = i - s * kH4;
        if (i < ns * kH4) reinterpret_cast<f4 *>(a.xs + (size_t)(sb + s) * a.L)[j] = v[u];
      }
    }
    for (int i0 = 0; i0 < ns * kXlpHist; i0 += 64 * B) {
#pragma unroll
      for (int u = 0; u < B; u++) {
        const int i = min(i0 + lane + 64 * u, ns * kXlpHist - 1), s = i / kXlpHist, m = max(i - s * kXlpHist, 1);
        const float *h = a.state + (size_t)(sb + s) * st::kWords + st::kPitch + kFrame;
        w[u] = xlp_value(h[2 * m - 1], h[2 * m], h[2 * m + 1]);
      }
#pragma unroll
      for (int u = 0; u < B; u++) {
        const int i = i0 + lane + 64 * u, s = i / kXlpHist, m = i - s * kXlpHist;
        if (i < ns * kXlpHist && m > 0) a.xlp[(size_t)(sb + s) * a.LX + m] = w[u];
      }
    }
  }
  {
    // the chain wave shares its SIMD with the previous push's kernels: its
    // latency-bound instruction stream goes first
    __builtin_amdgcn_s_setprio(3);
    if (lane < ns) {
      const int s = sb + lane, nt = ticks_of(a, s);
      if (nt > 0) {
        float *hp = a.state + (size_t)s * st::kWords + st::kHp;
        float mem0 = hp[0], mem1 = hp[1];
        if (a.raw_s16)
          prep_chain<false, float4>(a, a.pcm, s, nt, mem0, mem1);
        else if (a.pcm16)
          prep_chain<true, uint2>(a, a.pcm16, s, nt, mem0, mem1);
        else
          prep_chain<true, float4>(a, a.pcm, s, nt, mem0, mem1);
        hp[0] = mem0;
        hp[1] = mem1;
      }
    }
  }
  __syncthreads();
  // pitch_buf after the last frame = the last 1728 samples of the row (flat
  // over the workgroup's streams, as the history copies)
  {
    constexpr int kP4 = kPitchBuf / 4, B = 8;
    f4 v[B];
    for (int i0 = 0; i0 < ns * kP4; i0 += 64 * B) {
#pragma unroll
      for (int u = 0; u < B; u++) {
        const int i = min(i0 + lane + 64 * u, ns * kP4 - 1), s = i / kP4, j = i - s * kP4;
        const int nt = max(ticks_of(a, sb + s), 1);
        v[u] = reinterpret_cast<const f4 *>(a.xs + (size_t)(sb + s) * a.L + (size_t)(nt * C - 1) * kFrame)[j];
      }
#pragma unroll
      for (int u = 0; u < B; u++) {
        const int i = i0 + lane + 64 * u, s = i / kP4, j = i - s * kP4;
        const int nt = i < ns * kP4 ? ticks_of(a, sb + s) : 0;
        if (nt > 0) reinterpret_cast<f4 *>(a.state + (size_t)(sb + s) * st::kWords + st::kPitch)[j] = v[u];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pitch analysis (pitch.c: pitch_downsample, pitch_search, remove_doubling up
// to its sequential selection), split by how each part parallelises:
//
//   k_plpc   lane per frame.  Every serial chain that depends only on the
//            frame itself and streams its pitch buffer: x_lp, the 5 autocorr
//            sums (860 terms each), LPC, the 5-tap FIR, the Syy recurrences of
//            both find_best_pitch calls and xx.  A wave owns a tile of 64
//            streams at one frame position (lane = stream), so all 64 lanes
//            walk a chain.  Writes xf and the sequences to the tile buffer.
//   k_pcorr  8 frames per workgroup, xf resident in LDS.  The inner products
//            (coarse xcorr: 147 lags x 240, fine xcorr at <= 10 lags, the
//            remove_doubling products), both find_best_pitch scans and the
//            yy_lookup recurrence (lane per frame) and the pitch record for
//            k_select (fvad_pitch.hip).
// Every C-order sum stays on one lane in its original order.
// ---------------------------------------------------------------------------
// Pitch record of a frame (k_pcorr -> k_select): everything of

// LDS written and read back by lanes of the same wave only: LDS operations of
// a wave execute in order, so a compiler-level fence is all that is needed.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// pitch_downsample's LPC part (celt_lpc.c _celt_lpc, order 4) and the FIR
// coefficients lpc2 of celt_fir5, from the 5 autocorrelation values.
__device__ __forceinline__ void lpc_fir5_coeffs(float (&acv)[5], float (&lpc2)[5]) {
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
  lpc2[0] = lpc[0] + .8f;
  lpc2[1] = lpc[1] + c1 * lpc[0];
  lpc2[2] = lpc[2] + c1 * lpc[1];
  lpc2[3] = lpc[3] + c1 * lpc[2];
  lpc2[4] = c1 * lpc[3];
}

// ---------------------------------------------------------------------------
// k_plpc.  Both passes walk the frame's x_lp (pitch_downsample's 2:1
// decimation of the pitch buffer), read from the x_lp rows: every x_lp value
// of the push is computed once (k_prep3 for the history, k_fftAw for each
// frame's 240 new values) instead of from 1728 pitch-buffer samples per frame
// and pass, which halves this kernel's input bytes (0.88 -> 0.7x ms).  A
// tile's 64 rows are staged through LDS in chunks of 8 values: 16-byte
// coalesced loads of each stream's row, transposed to [value][stream] (row
// pitch 68: conflict-free for both the transposing writes and the column
// reads), the next chunk loading while one is summed.  x_lp[0] is the frame's
// own edge value (.5 * (.5 * x[1] + x[0])), from two pitch-buffer samples.
// Tile t = sb * Vr + v (Vr = frame positions of this push); the four waves of
// a workgroup take consecutive v of the same streams.
// ---------------------------------------------------------------------------
constexpr int kLpStep = 8;                // x_lp steps per chunk
constexpr int kLpRows = kLpStep;          // x_lp values of a stream per chunk (32 bytes)
constexpr int kLpPR = kLpRows / 4;        // float4 per stream row of a chunk (= loads per lane)
constexpr int kLpSPI = 64 / kLpPR;        // streams per load instruction
constexpr int kLpCols = 68;               // 4 * 68 = 16 (mod 32): the two float4 columns of a
                                          // half-wave's ds_write_b32 land on disjoint bank halves
constexpr int kLpChunks = kXlp / kLpStep;  // 108
static_assert(kXlp % kLpStep == 0 && kLpPR == 2, "x_lp chunking");

struct LpSrc {
  const float *p[kLpPR];  // per load slot: stream's x_lp row + 4 * (lane % kLpPR)
};

__device__ __forceinline__ void lp_fetch(const LpSrc &s, int c, float4 (&r)[kLpPR]) {
#pragma unroll
  for (int i = 0; i < kLpPR; i++) r[i] = *reinterpret_cast<const float4 *>(s.p[i] + kLpRows * c);
}

// chunk registers -> LDS [value][stream]
__device__ __forceinline__ void lp_stage(float *stg, int lane, const float4 (&r)[kLpPR]) {
  wave_sync();
  const int p = lane % kLpPR, s0 = lane / kLpPR;
#pragma unroll
  for (int i = 0; i < kLpPR; i++) {
    float *d = stg + (4 * p) * kLpCols + s0 + kLpSPI * i;
    d[0] = r[i].x;
    d[kLpCols] = r[i].y;
    d[2 * kLpCols] = r[i].z;
    d[3 * kLpCols] = r[i].w;
  }
  wave_sync();
}

// x_lp[n] for n = kLpStep * c + u from the staged column; the frame's x_lp[0]
// (pitch_downsample's edge value, .5 * (.5 * x[1] + x[0])) is not in the
// shared row and comes from the lane (x0)
template <bool First>
__device__ __forceinline__ float lp_value(const float *col, int u, float x0) {
  return (First && u == 0) ? x0 : col[u * kLpCols];
}

// pass-2 state of one lane (k_plpc)
struct Fir5State {
  float l[5];
  float m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0;  // x_lp[n-1..n-5]
  float b1 = 0, b2 = 0, b3 = 0, b4 = 0, b5 = 0;  // x_lp[n-481..n-485]: the lagged filter (xf[n - 480])
  float x0 = 0;                                  // x_lp[0]
  float Sc = 1.0f, Sf = 1.0f, xx = 0.0f;
};

// celt_fir5 step: y = x + l0 x[n-1] + ... + l4 x[n-5] in C order, history shifted
__device__ __forceinline__ float fir5_step(const float (&l)[5], float x, float &m1, float &m2, float &m3, float &m4,
                                           float &m5) {
  float y = x;
  y = y + l[0] * m1;
  y = y + l[1] * m2;
  y = y + l[2] * m3;
  y = y + l[3] * m4;
  y = y + l[4] * m5;
  m5 = m4, m4 = m3, m3 = m2, m2 = m1, m1 = x;
  return y;
}

// Row stores of the tile buffer go through a per-wave LDS stage: a chunk's
// rows (one value per lane each) are written to LDS [row][lane], then each
// lane stores two float4 of its quarter's [row][16] block, so one store
// instruction writes 1 KB in four 256-byte runs instead of 256 bytes in four
// 64-byte pieces (measured: the per-step dword row stores cost k_plpc ~0.4 ms).
// xf itself is not stored (k_pcorr rebuilds it from x_lp and the coefficients):
// the Syy recurrences' xf[n - 480] comes from a second filter over the x_lp
// chunk 480 values back, staged like the current one.
struct OutStage {
  float sf[1][64];            // the fine Syy checkpoint of the chunk (i = n0 - 480, a multiple of 8)
  float sc[kLpStep / 2][64];  // coarse Syy rows
};
// rows row0 .. row0 + NR - 1 of the lane's quarter (qbase = its [row][16] block)
template <int NR>
__device__ __forceinline__ void flush_rows(float *qbase, int row0, const float (*ob)[64], int lane) {
  const int q = lane >> 4;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int j = (lane & 15) + 16 * k, u = j >> 2, c4 = j & 3;
    if (u < NR)
      *reinterpret_cast<float4 *>(qbase + (row0 + u) * ptile::kQuarter + 4 * c4) =
          *reinterpret_cast<const float4 *>(&ob[u][16 * q + 4 * c4]);
  }
}

// One chunk of pass 2.  Region R of n = n0 .. n0+7:
//   1 [0, 384)    Syy initial sums      2 [384, 480)  + xx
//   3 [480, 774)  xx + Syy recurrences  4 the chunk holding n = 773 (guarded)
//   5 [774, 864)  xx only
// bcol: the staged x_lp column of chunk n0 - 480 (regions 3, 4; LagFirst: it
// is chunk 0, whose x_lp[0] is the lane's x0)
template <bool First, int R, bool LagFirst>
__device__ __forceinline__ void fir5_chunk(Fir5State &f, const float *col, const float *bcol, float *qbase, int n0,
                                           OutStage &ob, int lane) {
  constexpr int kR4 = (480 + 294) % kLpStep;  // region 4 starts at a chunk boundary
#pragma unroll
  for (int u = 0; u < kLpStep; u++) {
    const float y = fir5_step(f.l, lp_value<First>(col, u, f.x0), f.m1, f.m2, f.m3, f.m4, f.m5);
    if (R <= 2) {
      if ((u & 1) == 0) f.Sc = f.Sc + y * y;  // n0 is a multiple of 8: n even <=> u even
      f.Sf = f.Sf + y * y;
    }
    if (R == 3 || (R == 4 && u < kR4)) {
      const float yb = fir5_step(f.l, lp_value<LagFirst>(bcol, u, f.x0), f.b1, f.b2, f.b3, f.b4, f.b5);
      if (u == 0) ob.sf[0][lane] = f.Sf;  // k_pcorr walks from here to the lags it needs
      f.Sf += y * y - yb * yb;
      f.Sf = (1 > f.Sf) ? 1 : f.Sf;
      if ((u & 1) == 0) {
        ob.sc[u >> 1][lane] = f.Sc;
        f.Sc += y * y - yb * yb;
        f.Sc = (1 > f.Sc) ? 1 : f.Sc;
      }
    }
    if (R >= 2) f.xx = f.xx + y * y;
  }
  if (R == 3 || R == 4) {
    wave_sync();
    flush_rows<1>(qbase, ptile::kSf + (n0 - 480) / kLpStep, ob.sf, lane);
    if (R == 3)
      flush_rows<kLpStep / 2>(qbase, ptile::kSc + (n0 - 480) / 2, ob.sc, lane);
    else
      flush_rows<(kR4 + 1) / 2>(qbase, ptile::kSc + (n0 - 480) / 2, ob.sc, lane);
    wave_sync();
  }
}
static_assert(384 % kLpStep == 0 && 480 % kLpStep == 0 && kLpStep % 2 == 0, "pass-2 regions");
static_assert(480 % kLpStep == 0, "the lagged chunk is a whole chunk");
static_assert(kLpStep == 8 && (294 + kLpStep - 1) / kLpStep == ptile::kSfCk, "fine Syy checkpoints every 8 lags");

// x_lp chunks in flight per pass (the ring depth)
#ifndef FVAD_PLPC_OCC
#define FVAD_PLPC_OCC 2
#endif
#ifndef FVAD_LP_PF
#define FVAD_LP_PF 4
#endif
constexpr int kLpPf = FVAD_LP_PF;
static_assert(kLpChunks % kLpPf == 0, "prefetch ring must divide the passes");

// pass-1 state of one lane (k_plpc): _celt_autocorr's 5 lag sums, the tail
// sums of lags 1..3 and the last 4 x_lp values
struct AcState {
  float acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0, acc4 = 0;
  float d0 = 0, d1 = 0, d2 = 0, d3 = 0;
  float h1 = 0, h2 = 0, h3 = 0, h4 = 0;
};
// One chunk of pass 1 (lag k: sum_{i<860} x[i] x[i+k], then the tail).
// Kind 0: the first chunk (x_lp[0] = x0, lags start at their first term),
// 1: a middle chunk, 2: the last (n = 856..863: term i = n - k belongs to the
// 860-term sum while i < 860, else (n >= 860 + k) to the tail sum of x[n] x[n-k])
template <int Kind>
__device__ __forceinline__ void ac_chunk(AcState &s, const float *col, float x0, int c) {
#pragma unroll
  for (int u = 0; u < kLpStep; u++) {
    const float x = lp_value<Kind == 0>(col, u, x0);
    if (Kind == 2) {
      const int n = c * kLpStep + u;
      if (n < 860) s.acc0 = s.acc0 + x * x; else s.d0 = s.d0 + x * x;
      if (n - 1 < 860) s.acc1 = s.acc1 + s.h1 * x; else s.d1 = s.d1 + x * s.h1;
      if (n - 2 < 860) s.acc2 = s.acc2 + s.h2 * x; else s.d2 = s.d2 + x * s.h2;
      if (n - 3 < 860) s.acc3 = s.acc3 + s.h3 * x; else s.d3 = s.d3 + x * s.h3;
      s.acc4 = s.acc4 + s.h4 * x;  // n - 4 <= 859
    } else {
      s.acc0 = s.acc0 + x * x;
      if (Kind == 1 || u >= 1) s.acc1 = s.acc1 + s.h1 * x;
      if (Kind == 1 || u >= 2) s.acc2 = s.acc2 + s.h2 * x;
      if (Kind == 1 || u >= 3) s.acc3 = s.acc3 + s.h3 * x;
      if (Kind == 1 || u >= 4) s.acc4 = s.acc4 + s.h4 * x;
    }
    s.h4 = s.h3, s.h3 = s.h2, s.h2 = s.h1, s.h1 = x;
  }
}
static_assert(kLpChunks * kLpStep == 864 && (kLpChunks - 1) * kLpStep == 856, "pass-1 tail chunk");

__global__ void __launch_bounds__(256, FVAD_PLPC_OCC) k_plpc(StagedArgs a) {
  __shared__ float stg_all[4][2][kLpRows * kLpCols];
  __shared__ __attribute__((aligned(16))) OutStage ost_all[4];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  float *stg = stg_all[w][0], *stgb = stg_all[w][1];
  OutStage &ob = ost_all[w];
  const float *col = stg + lane;
  const int Vr = a.n_ticks * a.n_channels;
  const int n_sb = (a.n_streams + 63) >> 6;
  const long long n_tiles = (long long)n_sb * Vr;
  // a workgroup takes 4 consecutive tiles (one per wave: neighbouring frame
  // positions of the same streams share pitch-buffer samples in L2)
  const long long n_quads = (n_tiles + 3) / 4;
  __shared__ long long gq;
  STAMP_INIT();
  if (tid == 0) gq = take_group(a, kWorkPlpc);
  __syncthreads();
  long long q = gq;
  while (q < n_quads) {
    const long long t = q * 4 + w;
    if (t >= n_tiles) {
      __syncthreads();
      if (tid == 0) gq = take_group(a, kWorkPlpc);
      __syncthreads();
      q = gq;
      continue;
    }
    const int sb = (int)(t / Vr), v = (int)(t - (long long)sb * Vr);
    LpSrc src;
#pragma unroll
    for (int i = 0; i < kLpPR; i++) {
      const int s = min(sb * 64 + lane / kLpPR + kLpSPI * i, a.n_streams - 1);
      src.p[i] = a.xlp + (size_t)s * a.LX + (size_t)v * (kFrame / 2) + 4 * (lane % kLpPR);
    }
    float x0;
    {
      const float *pb = a.xs + (size_t)min(sb * 64 + lane, a.n_streams - 1) * a.L + (size_t)v * kFrame;
      x0 = .5f * (.5f * (pb[1]) + pb[0]);
    }
    // lane's output column: quarter (lane >> 4) of tile t, [row][16]
    float *out = a.ptile + ((size_t)(t * 4 + (lane >> 4)) * ptile::kRows) * ptile::kQuarter + (lane & 15);
    float *qbase = out - (lane & 15);
    RSTAMP(3);

    // Both passes walk the x_lp chunks through a register ring: chunk c is
    // staged while the loads of chunks c + 1 .. c + kLpPf are in flight (the
    // chunk loops unrolled by the ring depth, so slots are static registers)
    float4 pf[kLpPf][kLpPR];
    // pass 1: x_lp -> _celt_autocorr
    AcState as;
#pragma unroll
    for (int d = 0; d < kLpPf; d++) lp_fetch(src, d, pf[d]);
    for (int c0 = 0; c0 < kLpChunks; c0 += kLpPf) {
#pragma unroll
      for (int dd = 0; dd < kLpPf; dd++) {
        const int c = c0 + dd;
        lp_stage(stg, lane, pf[dd]);
        if (c + kLpPf < kLpChunks) lp_fetch(src, c + kLpPf, pf[dd]);
        if (c == 0)
          ac_chunk<0>(as, col, x0, c);
        else if (c + 1 < kLpChunks)
          ac_chunk<1>(as, col, x0, c);
        else
          ac_chunk<2>(as, col, x0, c);
      }
    }
    RSTAMP(0);
    float acv[5] = {as.acc0 + as.d0, as.acc1 + as.d1, as.acc2 + as.d2, as.acc3 + as.d3, as.acc4 + 0.0f};
    float l[5];
    lpc_fir5_coeffs(acv, l);

    // pass 2: x_lp again -> celt_fir5 -> xf; Syy initial sums, xx; from
    // n = 480 on, the Syy recurrences with xf[n - 480] from a second filter
    // over the x_lp chunk 480 values back (a second ring, staged in the
    // wave's second column).  The chunk body is specialised per region of n,
    // so it has no branches.
    Fir5State fs;
    fs.x0 = x0;
#pragma unroll
    for (int i = 0; i < 5; i++) fs.l[i] = l[i];
    const float *bcol = stgb + lane;
    constexpr int kLag = 480 / kLpStep;  // chunks between a value and its lagged partner
    auto lagged = [](int c) { return c * kLpStep >= 480 && c * kLpStep < 480 + 294; };
    float4 bk[kLpPf][kLpPR];
#pragma unroll
    for (int d = 0; d < kLpPf; d++) lp_fetch(src, d, pf[d]);
    for (int c0 = 0; c0 < kLpChunks; c0 += kLpPf) {
#pragma unroll
      for (int dd = 0; dd < kLpPf; dd++) {
        const int c = c0 + dd, n0 = c * kLpStep;
        lp_stage(stg, lane, pf[dd]);
        if (c + kLpPf < kLpChunks) lp_fetch(src, c + kLpPf, pf[dd]);
        if (lagged(c)) lp_stage(stgb, lane, bk[dd]);
        if (lagged(c + kLpPf)) lp_fetch(src, c + kLpPf - kLag, bk[dd]);
        if (c == 0)
          fir5_chunk<true, 1, false>(fs, col, bcol, qbase, n0, ob, lane);
        else if (n0 < 384)
          fir5_chunk<false, 1, false>(fs, col, bcol, qbase, n0, ob, lane);
        else if (n0 < 480)
          fir5_chunk<false, 2, false>(fs, col, bcol, qbase, n0, ob, lane);
        else if (n0 == 480)
          fir5_chunk<false, 3, true>(fs, col, bcol, qbase, n0, ob, lane);
        else if (n0 + kLpStep <= 480 + 294)
          fir5_chunk<false, 3, false>(fs, col, bcol, qbase, n0, ob, lane);
        else if (n0 < 480 + 294)
          fir5_chunk<false, 4, false>(fs, col, bcol, qbase, n0, ob, lane);
        else
          fir5_chunk<false, 5, false>(fs, col, bcol, qbase, n0, ob, lane);
      }
    }
    RSTAMP(1);
    out[ptile::kXx * ptile::kQuarter] = fs.xx;
    // k_pcorr's xf: the FIR coefficients and x_lp[0]
#pragma unroll
    for (int i = 0; i < 5; i++) out[(ptile::kFir + i) * ptile::kQuarter] = l[i];
    out[(ptile::kFir + 5) * ptile::kQuarter] = x0;

    // yy_lookup (remove_doubling's energy recurrence from xx) is k_pcorr's:
    // it walks it on a wave its product phase leaves idle, from xf in LDS
    RSTAMP(2);
    __syncthreads();
    if (tid == 0) gq = take_group(a, kWorkPlpc);
    __syncthreads();
    q = gq;
  }
  STAMP_FLUSH(56, 4);
}

// ---------------------------------------------------------------------------
// k_select: remove_doubling's sequential selection.  The frames of a stream
// stay sequential (prev_period / prev_gain), but a frame's 14 candidate tests
// are independent given them: 16 lanes per stream (4 streams per wave), lane
// k tests candidate k (T1 of k + 2), a ballot finds the last passing one (the
// reference loop keeps overwriting, so the highest k wins) and its values are
// read from its lane.  Every comparison and value is the reference's.  A
// frame's record loads kSelRing - 1 frames ahead through a register ring.
// ---------------------------------------------------------------------------
constexpr int kSelStreams = 4;  // streams per 64-thread workgroup
#ifndef FVAD_SEL_RING
#define FVAD_SEL_RING 8
#endif
constexpr int kSelRing = FVAD_SEL_RING;  // frames of records in flight
struct SelRec {
  int T0, nv, Tk, offk, off0;
  float g0, xy0, yy0, gk, xyk, yyk;
};
__device__ __forceinline__ void sel_load(SelRec &r, const float *__restrict__ row, int k, bool on) {
  if (!on) return;
  r.T0 = __float_as_int(row[rec::kT0]);
  r.nv = __float_as_int(row[rec::kNValid]);
  r.g0 = row[rec::kG0];
  r.xy0 = row[rec::kXy0];
  r.yy0 = row[rec::kYy0];
  r.off0 = __float_as_int(row[rec::kOff0]);
  const float *q = row + rec::kK + min(k, 13) * rec::kKStride;
  r.Tk = __float_as_int(q[0]);
  r.gk = q[1];
  r.xyk = q[2];
  r.yyk = q[3];
  r.offk = __float_as_int(q[4]);
}

__global__ void __launch_bounds__(64) k_select(StagedArgs a) {
  const int lane = threadIdx.x, sl = lane >> 4, k = lane & 15;
  // the persistent kernels' group counters: those of this push's k_fftAw /
  // k_plpc / k_pcorr are done with (they ran before), the rest are used after
  // this kernel; zeroed here instead of by a memset node of their own
  static_assert(kWorkSlots * kQueues <= 64, "one lane per counter");
  if (blockIdx.x == 0 && lane < kWorkSlots * kQueues) a.work[lane] = 0;
  const int s = blockIdx.x * kSelStreams + sl;
  const bool sok = s < a.n_streams;
  const int nf = sok ? ticks_of(a, s) * a.n_channels : 0;
  int nfw = nf;  // frames of the wave's longest stream (shuffles need every lane)
#pragma unroll
  for (int d = 16; d < 64; d <<= 1) nfw = max(nfw, __shfl_xor(nfw, d));
  if (nfw <= 0) return;
  float *stp = a.state + (size_t)(sok ? s : 0) * st::kWords;
  int *istp = reinterpret_cast<int *>(stp);
  int last_period = sok ? istp[st::kLastPeriod] : 0;
  float last_gain = sok ? stp[st::kLastGain] : 0.0f;
  const float *rows = a.rec + (size_t)(sok ? s : 0) * a.V * rec::kSize;
  const int K = k + 2;  // remove_doubling's k for this lane's candidate
  auto step = [&](const SelRec &r, int v) {
    const bool on = v < nf;
    const int prev_period = last_period / 2;
    const float prev_gain = last_gain;
    bool pass = false;
    if (on && k < 14 && k < r.nv) {
      const int T1 = r.Tk;
      float cont;
      if (abs(T1 - prev_period) <= 1)
        cont = prev_gain;
      else if (abs(T1 - prev_period) <= 2 && 5 * K * K < r.T0)
        cont = .5f * prev_gain;
      else
        cont = 0;
      float thresh;
      {
        const float vv = .7f * r.g0 - cont;
        thresh = (.3f > vv) ? .3f : vv;
      }
      if (T1 < 3 * 30) {
        const float vv = .85f * r.g0 - cont;
        thresh = (.4f > vv) ? .4f : vv;
      } else if (T1 < 2 * 30) {
        const float vv = .9f * r.g0 - cont;
        thresh = (.5f > vv) ? .5f : vv;
      }
      pass = r.gk > thresh;
    }
    const unsigned seg = (unsigned)(__ballot(pass) >> (16 * sl)) & 0x3fffu;
    const int win = seg ? 31 - __clz(seg) : 0;
    const int src = 16 * sl + win;
    const float wxy = __shfl(r.xyk, src), wyy = __shfl(r.yyk, src), wg = __shfl(r.gk, src);
    const int wT = __shfl(r.Tk, src), woff = __shfl(r.offk, src);
    float best_xy = seg ? wxy : r.xy0, best_yy = seg ? wyy : r.yy0, gg = seg ? wg : r.g0;
    const int T = seg ? wT : r.T0, offset = seg ? woff : r.off0;
    if (!on) return;
    best_xy = (0 > best_xy) ? 0 : best_xy;
    float pg;
    if (best_yy <= best_xy)
      pg = 1.0f;
    else
      pg = best_xy / (best_yy + 1);
    if (pg > gg) pg = gg;
    int pi = 2 * T + offset;
    if (pi < kPitchMin) pi = kPitchMin;
    if (k == 0) a.pitch[(size_t)s * a.V + v] = pi;
    last_period = pi;
    last_gain = pg;
  };
  // records kSelRing frames ahead through a register ring (static slots: the
  // loop over a ring turn is unrolled)
  SelRec r[kSelRing];
#pragma unroll
  for (int u = 0; u < kSelRing - 1; u++) {
    r[u] = SelRec{};
    sel_load(r[u], rows + (size_t)u * rec::kSize, k, u < nf);
  }
  r[kSelRing - 1] = SelRec{};
  for (int v = 0; v < nfw; v += kSelRing) {
#pragma unroll
    for (int u = 0; u < kSelRing; u++) {
      if (v + u >= nfw) break;
      // slot (u - 1) mod R was consumed last step: frame v + u + R - 1 goes there
      const int ls = (u + kSelRing - 1) % kSelRing;
      sel_load(r[ls], rows + (size_t)(v + u + kSelRing - 1) * rec::kSize, k, v + u + kSelRing - 1 < nf);
      step(r[u], v + u);
    }
  }
  if (sok && nf > 0 && k == 0) {
    istp[st::kLastPeriod] = last_period;
    stp[st::kLastGain] = last_gain;
  }
}

// ---------------------------------------------------------------------------
// GRU helpers of k_rnn3.  The whole GRU stack is resident in LDS as an int8
// image (rnnimg, 88 KB; int8 -> f32 is exact), so weights never come from L2
// per frame.  A matrix column = one neuron's C-order sum: lane (column, stream
// group) accumulates SL streams of that column with one weight fetch per term;
// per-stream vectors are stored [j][S] so the SL inputs of a term are one LDS
// read.  GRU inputs are read in place from their segments (no concatenation
// copies) and GRU states live in rings indexed by frame (no copy-back phase).
// ---------------------------------------------------------------------------
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

// input segments [G0, G1) of matrix m (a sum split across phases continues
// where the stored partial sum stopped: the same adds in the same order)
template <int m, int S, int SL, int G0, int G1>
__device__ __forceinline__ void rnn_segs(const int8_t *wc, const RnnIn &in, int s0, float (&acc)[SL]) {
  if constexpr (G0 <= 0 && G1 > 0) mv_seg<rnnimg::kSegs[m][0], S, SL>(wc, in.v0, s0, acc);
  if constexpr (m == 3 || m == 4 || m == 5 || m == 6) {
    if constexpr (G0 <= 1 && G1 > 1) mv_seg<rnnimg::kSegs[m][1], S, SL>(wc + rnnimg::seg_off(m, 1), in.v1, s0, acc);
    if constexpr (G0 <= 2 && G1 > 2) mv_seg<rnnimg::kSegs[m][2], S, SL>(wc + rnnimg::seg_off(m, 2), in.v2, s0, acc);
  }
}
template <int SL>
__device__ __forceinline__ void acc_load(float (&acc)[SL], const float *p) {
  const typename VecT<SL>::T v = *reinterpret_cast<const typename VecT<SL>::T *>(p);
  acc[0] = v.x;
  acc[1] = v.y;
  if constexpr (SL == 4) {
    acc[2] = v.z;
    acc[3] = v.w;
  }
}
template <int SL>
__device__ __forceinline__ void acc_store(const float (&acc)[SL], float *p) {
  typename VecT<SL>::T v;
  v.x = acc[0];
  v.y = acc[1];
  if constexpr (SL == 4) {
    v.z = acc[2];
    v.w = acc[3];
  }
  *reinterpret_cast<typename VecT<SL>::T *>(p) = v;
}

// dense layer / GRU z|r gates of image matrix m:
//   out[c][s] = act(kWs * (b[c] + sum_j w[c][j] * [in ; state][j][s]))
// (tasks t = tid, tid + NT, ...; NT = 0: the single task tid)
// (PART 3: b + input segment 0 only, stored to preT [c][S]; PART 5: from
// preT, the remaining input segments and the state)
template <int m, int S, int G, int NT, int PART = 0>
__device__ __forceinline__ void rnn_gates(const int8_t *W, const RnnIn &in, const float *stT, float *outT, int act,
                                          const float *tt, int tid, float *preT = nullptr) {
  constexpr int SL = S / G, cols = rnnimg::kCols[m];
  constexpr int ob = rnnimg::off_b(m), ow = rnnimg::off_w(m), ws = rnnimg::stride(m);
  constexpr int gst = (m == 1) ? 1 : (m == 3 || m == 5) ? 3 : -1;  // state segment of z|r matrices
  for (int t = tid; t < cols * G; t += (NT ? NT : cols * G)) {
    const int c = t / G, s0 = (t - c * G) * SL;
    const int8_t *wc = W + ow + c * ws;
    float acc[SL];
    if constexpr (PART == 5) {
      acc_load<SL>(acc, preT + c * S + s0);
      rnn_segs<m, S, SL, 1, 3>(wc, in, s0, acc);
    } else {
      const float b = (float)W[ob + c];
#pragma unroll
      for (int q = 0; q < SL; q++) acc[q] = b;
      if constexpr (PART == 3) {
        rnn_segs<m, S, SL, 0, 1>(wc, in, s0, acc);
        acc_store<SL>(acc, preT + c * S + s0);
        continue;
      } else {
        rnn_inputs<m, S, SL>(wc, in, s0, acc);
      }
    }
    if constexpr (gst >= 0) mv_seg<rnnimg::kSegs[m][gst], S, SL>(wc + rnnimg::seg_off(m, gst), stT, s0, acc);
#pragma unroll
    for (int q = 0; q < SL; q++) outT[c * S + s0 + q] = activate(tt, act, kWs * acc[q]);
  }
}

// GRU candidate of image matrix m: sum = b + sum_j w*in[j] + sum_j (w*state[j])*r[j];
// new[c][s] = z*state + (1-z)*act(kWs*sum) for active streams, state otherwise.
// The sum's input prefix (b + the input terms) does not depend on the reset
// gate, so it can run one phase early: PART 1 stores the prefix to preT
// ([c][S]) and returns, PART 2 starts from preT and adds the recurrent terms
// -- the same sequence of f32 adds as PART 0, split at a store.
template <int m, int S, int G, int NT, int PART = 0>
__device__ __forceinline__ void rnn_cand(const int8_t *W, const RnnIn &in, const float *stT, const float *zrT,
                                         float *newT, const int *actv, int act, const float *tt, int tid,
                                         float *preT = nullptr) {
  constexpr int SL = S / G, cols = rnnimg::kCols[m], N = cols;
  constexpr int ob = rnnimg::off_b(m), ow = rnnimg::off_w(m), ws = rnnimg::stride(m);
  constexpr int gst = (m == 2) ? 1 : 3;
  for (int t = tid; t < cols * G; t += (NT ? NT : cols * G)) {
    const int c = t / G, s0 = (t - c * G) * SL;
    const int8_t *wc = W + ow + c * ws;
    float acc[SL];
    if constexpr (PART == 2 || PART == 4) {
      acc_load<SL>(acc, preT + c * S + s0);
      if constexpr (PART == 4) rnn_segs<m, S, SL, 1, 3>(wc, in, s0, acc);
    } else {
      const float b = (float)W[ob + c];
#pragma unroll
      for (int q = 0; q < SL; q++) acc[q] = b;
      if constexpr (PART == 3)
        rnn_segs<m, S, SL, 0, 1>(wc, in, s0, acc);
      else
        rnn_inputs<m, S, SL>(wc, in, s0, acc);
    }
    if constexpr (PART == 1 || PART == 3 || PART == 4) {
      acc_store<SL>(acc, preT + c * S + s0);
      continue;
    }
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

// ---------------------------------------------------------------------------
// k_rnn3: the recurrence.  One workgroup owns 8 streams and walks their
// frames in lockstep, 4 streams per lane (G = 2: one column's 8 streams on two
// lanes), as a two-phase layer pipeline over frames: compute_rnn's GRUs
// depend on each other only within a frame (vad -> noise -> denoise) and on
// their own previous state, so one step runs different layers of different
// frames side by side.  A lane's inputs
// for one term are one 16-byte LDS read (ds_read_b128, full LDS rate; the
// float2 reads of G = 4 were paired into half-rate ds_read2_b64) and one
// int8 -> f32 conversion serves 4 streams.  Step t:
//   P1  z|r gates of vad(t-1), noise(t-2), denoise(t-3); the denoise
//       candidates' input prefixes of t-3; spectral variability of t; gain
//       smoothing of t-5
//   P2  candidates of vad(t-1), noise(t-2), denoise(t-3) (denoise: its 96
//       recurrent terms after the P1 prefix); dense(t); denoise_output(t-4);
//       vad_output(t-2); features of t+1 (cepstral memory, deltas, distance
//       row) -> LDS; the denoise z|r gates' and candidates' first segment
//       (b + the 24 vad-state terms) of frame t-2, continued by the next P1
// Two barriers per step.  Every term keeps its C order; buffers are rings
// indexed by frame (features 8, dense/vad state 4, noise/denoise state 2).
// ---------------------------------------------------------------------------

// P2 wave priorities (s_setprio while the role runs): bit 2 the noise h
// waves, bit 4 denoise_output (kept: k_rnn3 1.19 -> 1.16 ms; both are young
// waves that set P2's end), bit 128 the denoise candidates' vad-state
// segment wave 15 (kept: 1.141 -> 1.128 ms; the z|r segment waves 12-14
// raised lost, 1.17), bit 8 vad h + dense (no gain; nor vad_output or
// the feature waves raised: 1.17 -> 1.18 ms).  Raising P1's
// noise or vad z|r waves above the denoise waves lost (1.16 -> 1.19 / 1.21 ms),
// as did the denoise prefix waves (1.23 ms).
#ifndef FVAD_PRIO
#define FVAD_PRIO 134
#endif
constexpr int kR3S = 8, kR3G = 2, kR3NT = 1024;
__global__ void __launch_bounds__(kR3NT) k_rnn3(StagedArgs a) {
  constexpr int S = kR3S, G = kR3G, NT = kR3NT;
  struct Lds {
    alignas(16) float featT[8][44 * S];  // frame f in slot f & 7
    alignas(16) float doutT[4][24 * S];
    alignas(16) float gvT[4][24 * S];
    alignas(16) float gnT[2][48 * S];
    alignas(16) float gdT[2][96 * S];
    alignas(16) float zrv[48 * S], zrn[96 * S], zrd[192 * S];
    alignas(16) float dhp[2][96 * S];  // denoise candidate input prefixes of frame f in slot f & 1
    alignas(16) float zpre[192 * S];  // denoise z|r: b + the vad-state segment of the frame P1 continues
    alignas(16) float gout[2][22 * S];  // denoise_output of frame f in slot f & 1
    alignas(16) float vo[S];  // vad_output of the frame P2 computed last
    float tt[204];
    float ceps[S][kCeps * kBands];
    float dist[S][kCeps * kCeps];
    float lastg[S][kBands];
    float pf[S][kRnnPf];  // features of the frame the next F-C stage reads
    int act[8][S];        // frame f in slot f & 7: valid and not silent
    int memid[S], nfs[S];
    long long fbase[S];
    alignas(16) int8_t W[rnnimg::kBytes];
  };
  __shared__ Lds L;
  const int tid = threadIdx.x;
  const int sb = blockIdx.x * S;
  const int *ra = a.rnn_act;
  {
    const int4 *src = reinterpret_cast<const int4 *>(a.rnn_img);
    int4 *dst = reinterpret_cast<int4 *>(L.W);
    for (int i = tid; i < rnnimg::kBytes / 16; i += NT) dst[i] = src[i];
    for (int i = tid; i < 201; i += NT) L.tt[i] = a.plan->tansig[i];
  }
  for (int idx = tid; idx < S * kCeps * kBands; idx += NT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    L.ceps[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += NT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    L.dist[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kBands; idx += NT) {
    const int s = idx / kBands, i = idx - s * kBands;
    L.lastg[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] : 0.0f;
  }
  // states before frame 0 = "frame -1": gv slot 3, gn / gd slot 1
  for (int idx = tid; idx < S * 96; idx += NT) {
    const int s = idx / 96, i = idx - s * 96;
    const bool ok = sb + s < a.n_streams;
    const float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) L.gvT[3][i * S + s] = ok ? stp[st::kVadGru + i] : 0.0f;
    if (i < 48) L.gnT[1][i * S + s] = ok ? stp[st::kNoiseGru + i] : 0.0f;
    L.gdT[1][i * S + s] = ok ? stp[st::kDenGru + i] : 0.0f;
  }
  if (tid < 8 * S) L.act[tid / S][tid % S] = 0;
  if (tid < S) {
    const int s = sb + tid;
    const bool ok = s < a.n_streams;
    L.memid[tid] = ok ? reinterpret_cast<const int *>(a.state)[(size_t)s * st::kWords + st::kMemId] : 0;
    L.nfs[tid] = ok ? ticks_of(a, s) * a.n_channels : 0;
    L.fbase[tid] = (long long)s * a.V;
  }
  __syncthreads();
  int maxnf = 0;
#pragma unroll
  for (int s = 0; s < S; s++) maxnf = max(maxnf, L.nfs[s]);
  // prefetch lane (s, i): i < 22 Lyf, 22..28 f34, 29 silence (the flag's bits,
  // nonzero = silent: converting it here would wait for the load at the top of
  // every step, before the lane's P1 role)
  const int pfs = tid / kRnnPf, pfi = tid - pfs * kRnnPf;
  const bool pf_lane = tid < S * kRnnPf;
  auto fetch = [&](int v) -> float {
    if (!pf_lane || v >= L.nfs[pfs]) return 1.0f;  // past the end: treated as silent (inactive)
    const long long f = L.fbase[pfs] + v;
    if (pfi < kBands) return a.Lyf[f * kBands + pfi];
    if (pfi < kBands + 7) return a.f34[f * 8 + (pfi - kBands)];
    return __int_as_float(a.silence[f]);
  };
  // F-C: frame f's features from L.pf (cepstral memory, deltas, 34..40, the
  // new distance row); item (s, i), i < 37; item i == 0 records act(f)
  auto feat_c = [&](int f, int idx) {
    const int s = idx / (kBands + 7 + kCeps), i = idx - s * (kBands + 7 + kCeps);
    const bool valid = f < L.nfs[s];
    const bool on = valid && __float_as_int(L.pf[s][kRnnPf - 1]) == 0;
    if (i == 0) {
      L.act[f & 7][s] = on;
      if (valid && !on) a.vadf[L.fbase[s] + f] = 0;  // silent: X passes through, state untouched
    }
    if (!on) return;
    float *featT = L.featT[f & 7];
    const int mi = L.memid[s];
    const float *c0 = L.pf[s];  // ceps_0 (the row being written at memid)
    if (i < kBands) {
      L.ceps[s][mi * kBands + i] = c0[i];
      if (i < 6) {
        const float *c1 = L.ceps[s] + ((mi < 1) ? kCeps + mi - 1 : mi - 1) * kBands;
        const float *c2 = L.ceps[s] + ((mi < 2) ? kCeps + mi - 2 : mi - 2) * kBands;
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
        const float *cj = L.ceps[s] + j * kBands;
        float d = 0;
#pragma unroll
        for (int k = 0; k < kBands; k++) {
          const float tmp = c0[k] - cj[k];
          d += tmp * tmp;
        }
        L.dist[s][mi * kCeps + j] = d;
        L.dist[s][j * kCeps + mi] = d;
      }
    }
  };
  // F-D: spectral variability of frame f, stream s
  auto feat_d = [&](int f, int s) {
    if (!L.act[f & 7][s]) return;
    float sv = 0;
    for (int i = 0; i < kCeps; i++) {
      float mindist = 1e15f;
      for (int j = 0; j < kCeps; j++)
        if (j != i) mindist = (mindist < L.dist[s][i * kCeps + j]) ? mindist : L.dist[s][i * kCeps + j];
      sv += mindist;
    }
    L.featT[f & 7][41 * S + s] = (float)(sv / kCeps - 2.1);
    int mid = L.memid[s] + 1;
    if (mid == kCeps) mid = 0;
    L.memid[s] = mid;
  };
  // prologue: features of frame 0 (its spectral variability: P1 of step 0)
  if (pf_lane) L.pf[pfs][pfi] = fetch(0);
  __syncthreads();
  for (int idx = tid; idx < S * (kBands + 7 + kCeps); idx += NT) feat_c(0, idx);
  __syncthreads();
  // P1 wave plan (w = tid >> 6).  Waves w, w+4, w+8, w+12 share a SIMD under
  // the cyclic wave placement, so the heavy roles are spread over the four
  // residue classes -- {den, den, pre}, {den, den, pre}, {den, noise, noise,
  // vad}, {den, noise, vad, pre} -- and no wave holds lanes of two roles (it
  // would run both branches one after the other): denoise z|r waves 0..5 (384
  // tasks), noise z|r waves 6, 7, 10 (192), vad z|r waves 11, 14 (96), the
  // denoise candidates' input prefixes (b + the 114 input terms, which do not
  // need the reset gate) waves 12, 13, 15 (192), gain smoothing + vad_output
  // store wave 8, spectral variability of frame t wave 9.  (The constants
  // name each role's first thread, for the stamps build.)  Measured and lost
  // (DESIGN §8 r3): the noise candidates' prefixes here too (on waves 8 / 9,
  // gains moved to P2: P1 16.0 -> 17.7 k cycles, P2 12.6 -> 10.9 k), and the
  // heavy roles on the oldest waves of each SIMD (the young vad waves starve).
  [[maybe_unused]] constexpr int kP1Den = 0, kP1Noise = 384, kP1Vad = 704, kP1Var = 576, kP1Gain = 512;
  // P2 wave plan, balanced over the residue classes the same way (a wave
  // holding lanes of two roles set the phase at 19.6 k cycles before): denoise
  // h waves 0..2 (192 tasks; the 96 recurrent terms from the P1 prefix),
  // noise h waves 3, 6 (96), denoise_output wave 4 (44), vad h wave 5 (48),
  // dense of frame t wave 7 (48), vad_output wave 8 (2 lanes), features of
  // frame t+1 waves 9..11 (296 items, two per lane on the first 104), the
  // denoise z|r first segments of frame t-2 waves 12..14 (384 tasks, two per
  // lane), the denoise candidates' wave 15 (192, three per lane).  (Denoise h with 2 streams per lane on
  // 6 waves shortened its chain to 11.1 k cycles but the extra waves
  // stretched the other roles: 15.3 vs 14.6 k per phase.)
  [[maybe_unused]] constexpr int kP2Den = 0, kP2Noise = 192, kP2Vad = 320, kP2Dense = 448, kP2Out = 256, kP2VadOut = 512,
                kP2Feat = 576;
  constexpr int kFeatItems = S * (kBands + 7 + kCeps);
  static_assert(kP2Feat + kFeatItems <= 14 * 64 && 96 * kR3G == 192 && 48 * kR3G <= 128 && 22 * kR3G <= 64 &&
                    24 * kR3G <= 64,
                "P2 wave plan");
  STAMP_INIT();
#ifdef FVAD_STAMPS
  // role finish times: the first thread of each role adds (its role's end -
  // its phase start) to stamps[2 + role]
  unsigned long long ph0 = 0, racc = 0;
  int rslot = -1;
  {
    const int l1[5] = {kP1Den, kP1Noise, kP1Vad, kP1Var, kP1Gain};
    const int l2[7] = {kP2Den, kP2Noise, kP2Vad, kP2Dense, kP2Out, kP2VadOut, kP2Feat};
    for (int i = 0; i < 5; i++)
      if (tid == l1[i]) rslot = i;
    for (int i = 0; i < 7; i++)
      if (tid == l2[i]) rslot = (rslot < 0) ? 16 + i : rslot;  // tid 0 / 384 lead in both phases
  }
  unsigned long long racc2[2] = {0, 0};
#define ROLE_BEGIN() ph0 = __builtin_amdgcn_s_memtime()
#define ROLE_END(ph) racc2[ph] += __builtin_amdgcn_s_memtime() - ph0
#else
#define ROLE_BEGIN() \
  do {               \
  } while (0)
#define ROLE_END(ph) \
  do {               \
  } while (0)
#endif
  // gain smoothing g = max(g, .6*lastg) (denoise.c) of frame f5 on lanes
  // i0, i0 + n, ...; reads denoise_output slot f5 & 1
  auto gains = [&](int f5, int i0, int n) {
    for (int idx = i0; f5 >= 0 && idx < S * kBands; idx += n) {
      const int s = idx / kBands, i = idx - s * kBands;
      if (!L.act[f5 & 7][s]) continue;
      const long long f = L.fbase[s] + f5;
      const float gi = L.gout[f5 & 1][i * S + s];
      const float al = .6f * L.lastg[s][i];
      const float gsm = (gi > al) ? gi : al;
      L.lastg[s][i] = gsm;
      a.gr[f * kBands + i] = gi;
      a.gs[f * kBands + i] = gsm;
    }
  };
  for (int t = 0; t <= maxnf + 4; t++) {
    // per-step opaque thread id: the roles' per-thread offsets are recomputed
    // each step instead of hoisted out of the frame loop, where they spilled
    // (128 VGPRs + 34 spilled -> 112, no scratch: 1.27 -> 1.23-1.24 ms)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int fv = t - 1, fn = t - 2, fd = t - 3;
    ROLE_BEGIN();
    // frame t+1's raw features, staged at the end of P1 for P2's feat_c:
    // issued here, so no load is outstanding across a step boundary (a
    // loop-carried register would make the step's last barrier wait for it)
    const float pf_now = fetch(t + 1);
    // ---- P1
    // (the wave index as a scalar, readfirstlane: measured neutral here,
    // 1.135-1.154 vs 1.126-1.155 ms interleaved; k_gru16 gains from it)
    const int wv = tq >> 6, ln = tq & 63;
    if (wv < 6) {
      if (fd >= 0 && fd < maxnf)
        rnn_gates<5, S, G, 0, 5>(L.W, RnnIn{L.gvT[fd & 3], L.gnT[fd & 1], L.featT[fd & 7]}, L.gdT[(fd + 1) & 1],
                                 L.zrd, kActSigmoid, L.tt, tq, L.zpre);
    } else if (wv == 6 || wv == 7 || wv == 10) {
      if (fn >= 0 && fn < maxnf)
        rnn_gates<3, S, G, 0>(L.W, RnnIn{L.doutT[fn & 3], L.gvT[fn & 3], L.featT[fn & 7]}, L.gnT[(fn + 1) & 1], L.zrn,
                              kActSigmoid, L.tt, (wv == 10 ? 128 : 64 * (wv - 6)) + ln);
    } else if (wv == 11 || wv == 14) {
      if (fv >= 0 && fv < maxnf)
        rnn_gates<1, S, G, 0>(L.W, RnnIn{L.doutT[fv & 3], nullptr, nullptr}, L.gvT[(fv + 3) & 3], L.zrv, kActSigmoid,
                              L.tt, (wv == 14 ? 64 : 0) + ln);
    } else if (wv == 12 || wv == 13 || wv == 15) {
      // denoise candidate input prefixes of frame t-3
      if (fd >= 0 && fd < maxnf)
        rnn_cand<6, S, G, 0, 4>(L.W, RnnIn{L.gvT[fd & 3], L.gnT[fd & 1], L.featT[fd & 7]}, nullptr, nullptr, nullptr,
                                nullptr, 0, nullptr, (wv == 15 ? 128 : 64 * (wv - 12)) + ln, L.dhp[fd & 1]);
    } else if (wv == 8 && ln < 48) {  // gain smoothing of frame t-5
      gains(t - 5, ln, 48);
    } else if (wv == 9 && ln < S) {  // spectral variability of frame t (features: P2 of step t-1)
      if (t < maxnf) feat_d(t, ln);
    } else if (wv == 8 && ln >= 48 && ln < 48 + S) {  // vad_output of frame t-3 (P2 of step t-1)
      const int s = ln - 48, fw = t - 3;
      if (fw >= 0 && fw < maxnf && L.act[fw & 7][s]) a.vadf[L.fbase[s] + fw] = L.vo[s];
    }
    ROLE_END(0);
    if (pf_lane) L.pf[pfs][pfi] = pf_now;
    lds_sync();
    RSTAMP(0);
    ROLE_BEGIN();
    // ---- P2
    const int fo = t - 4;
    if (wv < 3) {
      if (fd >= 0 && fd < maxnf)
        rnn_cand<6, S, G, 0, 2>(L.W, RnnIn{nullptr, nullptr, nullptr}, L.gdT[(fd + 1) & 1], L.zrd, L.gdT[fd & 1],
                                L.act[fd & 7], ra[6], L.tt, tq, L.dhp[fd & 1]);
    } else if (wv == 3 || wv == 6) {
      if (FVAD_PRIO & 2) __builtin_amdgcn_s_setprio(3);
      if (fn >= 0 && fn < maxnf)
        rnn_cand<4, S, G, 0>(L.W, RnnIn{L.doutT[fn & 3], L.gvT[fn & 3], L.featT[fn & 7]}, L.gnT[(fn + 1) & 1], L.zrn,
                             L.gnT[fn & 1], L.act[fn & 7], ra[4], L.tt, (wv == 6 ? 64 : 0) + ln);
      if (FVAD_PRIO & 2) __builtin_amdgcn_s_setprio(0);
    } else if (wv == 5) {
      if (FVAD_PRIO & 8) __builtin_amdgcn_s_setprio(2);
      if (fv >= 0 && fv < maxnf)
        rnn_cand<2, S, G, 0>(L.W, RnnIn{L.doutT[fv & 3], nullptr, nullptr}, L.gvT[(fv + 3) & 3], L.zrv, L.gvT[fv & 3],
                             L.act[fv & 7], ra[2], L.tt, ln);
      if (FVAD_PRIO & 8) __builtin_amdgcn_s_setprio(0);
    } else if (wv == 7) {
      if (FVAD_PRIO & 8) __builtin_amdgcn_s_setprio(2);
      if (t < maxnf)
        rnn_gates<0, S, G, 0>(L.W, RnnIn{L.featT[t & 7], nullptr, nullptr}, nullptr, L.doutT[t & 3], ra[0], L.tt, ln);
      if (FVAD_PRIO & 8) __builtin_amdgcn_s_setprio(0);
    } else if (wv == 4) {
      if (FVAD_PRIO & 4) __builtin_amdgcn_s_setprio(2);
      if (fo >= 0 && fo < maxnf)
        rnn_gates<7, S, G, 0>(L.W, RnnIn{L.gdT[fo & 1], nullptr, nullptr}, nullptr, L.gout[fo & 1], ra[7], L.tt, ln);
      if (FVAD_PRIO & 4) __builtin_amdgcn_s_setprio(0);
    } else if (wv == 8 && ln < G) {
      // vad_output(t-2) -> L.vo, stored by the next step's P1
      if (fn >= 0 && fn < maxnf)
        rnn_gates<8, S, G, 0>(L.W, RnnIn{L.gvT[fn & 3], nullptr, nullptr}, nullptr, L.vo, ra[8], L.tt, ln);
    } else if (tq >= kP2Feat && tq < kP2Feat + 192) {  // features of t+1 on waves 9..11
      for (int idx = tq - kP2Feat; t + 1 < maxnf && idx < kFeatItems; idx += 192) feat_c(t + 1, idx);
    } else if (wv >= 12 && wv <= 14) {  // denoise z|r of frame t-2: b + the vad-state segment
      const int fz = t - 2;
      if (fz >= 0 && fz < maxnf)
        rnn_gates<5, S, G, 192, 3>(L.W, RnnIn{L.gvT[fz & 3], nullptr, nullptr}, nullptr, nullptr, kActSigmoid, L.tt,
                                   tq - 768, L.zpre);
    } else if (wv == 15) {  // denoise candidates of frame t-2: b + the vad-state segment
      const int fz = t - 2;
      if (FVAD_PRIO & 128) __builtin_amdgcn_s_setprio(2);
      if (fz >= 0 && fz < maxnf)
        rnn_cand<6, S, G, 64, 3>(L.W, RnnIn{L.gvT[fz & 3], nullptr, nullptr}, nullptr, nullptr, nullptr, nullptr, 0,
                                 nullptr, ln, L.dhp[fz & 1]);
      if (FVAD_PRIO & 128) __builtin_amdgcn_s_setprio(0);
    }
    ROLE_END(1);
    lds_sync();
    RSTAMP(1);
  }
  STAMP_FLUSH(0, 2);
#ifdef FVAD_STAMPS
  // P1 roles -> stamps[2..6], P2 roles -> stamps[8..14] (tid 0 and 384 lead a
  // role in both phases)
  if (a.stamps) {
    const int p1[5] = {kP1Den, kP1Noise, kP1Vad, kP1Var, kP1Gain};
    const int p2[7] = {kP2Den, kP2Noise, kP2Vad, kP2Dense, kP2Out, kP2VadOut, kP2Feat};
    for (int i = 0; i < 5; i++)
      if (tid == p1[i]) atomicAdd(&a.stamps[2 + i], racc2[0]);
    for (int i = 0; i < 7; i++)
      if (tid == p2[i]) atomicAdd(&a.stamps[8 + i], racc2[1]);
  }
  // every wave's busy cycles per phase (lane 0): stamps[64 + w] P1, [80 + w] P2
  if (a.stamps && (tid & 63) == 0) {
    atomicAdd(&a.stamps[64 + (tid >> 6)], racc2[0]);
    atomicAdd(&a.stamps[80 + (tid >> 6)], racc2[1]);
  }
  (void)racc;
  (void)rslot;
#endif
#undef ROLE_BEGIN
#undef ROLE_END
  const int fin = maxnf - 1;  // the slots of the latest states ("frame -1" if there were none)
  for (int idx = tid; idx < S * kCeps * kBands; idx += NT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    if (sb + s < a.n_streams && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] = L.ceps[s][i];
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += NT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    if (sb + s < a.n_streams && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] = L.dist[s][i];
  }
  for (int idx = tid; idx < S * kBands; idx += NT) {
    const int s = idx / kBands, i = idx - s * kBands;
    if (sb + s < a.n_streams && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] = L.lastg[s][i];
  }
  for (int idx = tid; idx < S * 96; idx += NT) {
    const int s = idx / 96, i = idx - s * 96;
    if (sb + s >= a.n_streams || L.nfs[s] <= 0) continue;
    float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) stp[st::kVadGru + i] = L.gvT[fin & 3][i * S + s];
    if (i < 48) stp[st::kNoiseGru + i] = L.gnT[fin & 1][i * S + s];
    stp[st::kDenGru + i] = L.gdT[fin & 1][i * S + s];
  }
  if (tid < S && sb + tid < a.n_streams && L.nfs[tid] > 0)
    reinterpret_cast<int *>(a.state)[(size_t)(sb + tid) * st::kWords + st::kMemId] = L.memid[tid];
}

// ---------------------------------------------------------------------------
// k_ola: out = x[0..479] + synthesis_mem; denoised * 1/32767; re-block ring;
// per-tick vad_low (min over channels in channel order).  Two frames per
// 256-thread workgroup, a float4 of samples per thread (32-bit frame
// arithmetic; the ring position of a frame is reduced once per thread).
// ---------------------------------------------------------------------------
static_assert(st::kSyn % 4 == 0 && kFrame % 4 == 0, "k_ola float4 rows");
__global__ void __launch_bounds__(256) k_ola(StagedArgs a) {
  const int C = a.n_channels, V = a.V;
  const int q = threadIdx.x & 127;
  const long long fl = (long long)blockIdx.x * 2 + (threadIdx.x >> 7);
  if (fl >= (long long)a.n_streams * V || q >= kFrame / 4) return;
  const int s = (int)(fl / V), v = (int)(fl - (long long)s * V);
  const int nt = ticks_of(a, s);
  if (v >= nt * C) return;
  const int t = v / C, c = v - t * C, i = 4 * q;
  const float *stp = a.state + (size_t)s * st::kWords;
  const size_t f = (size_t)s * V + v;
  const float4 prev = (v == 0) ? *reinterpret_cast<const float4 *>(stp + st::kSyn + i)
                               : *reinterpret_cast<const float4 *>(a.ys + (f - 1) * kWin + kFrame + i);
  const float4 cur = *reinterpret_cast<const float4 *>(a.ys + f * kWin + i);
  float4 o = make_float4(cur.x + prev.x, cur.y + prev.y, cur.z + prev.z, cur.w + prev.w);
  if (!a.raw_s16) {
    const float k = 1.0f / (float)32767;
    o = make_float4(o.x * k, o.y * k, o.z * k, o.w * k);
  }
  const int frames_done = reinterpret_cast<const int *>(stp)[st::kFramesDone];
  long long ri = (long long)(frames_done + t) * kFrame % a.ring_len + i;  // ring_len % 4 == 0: no float4 wraps
  if (ri >= a.ring_len) ri -= a.ring_len;
  *reinterpret_cast<float4 *>(a.ring + ((size_t)s * C + c) * a.ring_len + ri) = o;
  if (a.out_den) *reinterpret_cast<float4 *>(a.out_den + (((size_t)t * a.n_streams + s) * C + c) * kFrame + i) = o;
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
// k_winmeta: window completion bookkeeping (VAD.zig:298-348): lane per stream
// for the serial tick walk (16 streams per 64-thread workgroup), then the
// whole workgroup copies the streams' synthesis memory (second half of each
// stream's last frame) into the state.
// ---------------------------------------------------------------------------
constexpr int kWmS = 16;
__global__ void __launch_bounds__(64) k_winmeta(StagedArgs a) {
  const int sb = blockIdx.x * kWmS, tid = threadIdx.x;
  if (tid < kWmS && sb + tid < a.n_streams) {
    const int s = sb + tid;
    const int nt = ticks_of(a, s);
    int *wt = a.win_tick + (size_t)s * a.wmax;
    long long *wsx = a.win_start + (size_t)s * a.wmax;
    int j = 0;
    if (nt > 0) {
      float *stp = a.state + (size_t)s * st::kWords;
      int *istp = reinterpret_cast<int *>(stp);
      int fd = istp[st::kFramesDone];
      float vol = stp[st::kVolAcc];
      const int FB = a.plan->nfft_b, wpt = a.wpt;
      // the per-tick inputs (ratio, vad) of 8 ticks load before any of their
      // outputs is stored (stores between the loads would serialise them)
      constexpr int kWmT = 8;
      for (int t0 = 0; t0 < nt; t0 += kWmT) {
        float rr[kWmT], vv[kWmT];
#pragma unroll
        for (int u = 0; u < kWmT; u++) {
          const size_t o = (size_t)(t0 + u) * a.n_streams + s;
          rr[u] = t0 + u < nt ? a.ratio[o] : 0.0f;
          vv[u] = t0 + u < nt ? a.out_vad[o] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kWmT; u++) {
          const int t = t0 + u;
          if (t < nt) {
            const size_t o = (size_t)t * a.n_streams + s, ow = o * wpt;
            const float ratio = rr[u];
            // fftBufferStep (VAD.zig:307-347): the frame goes into the FFT
            // buffer in pieces of min(room left, samples left); each piece
            // adds ratio * written / fft_size, a full buffer is a window
            // (vad = this frame's); fft_size < 480 completes several per tick
            const long long a0 = (long long)fd * kFrame;
            int off = 0, nw = 0;
            while (off < kFrame) {
              const long long pos = a0 + off, wdone = pos / FB, next_end = (wdone + 1) * FB;
              const int written = (int)min((long long)(kFrame - off), next_end - pos);
              vol += ratio * ((float)written / (float)FB);
              off += written;
              if (pos + written == next_end) {
                a.out_win_ratio[ow + nw] = vol;
                a.out_win_vad[ow + nw] = vv[u];
                vol = 0;
                wt[j] = t * wpt + nw;
                wsx[j] = wdone * FB;
                j++;
                nw++;
              }
            }
            // slots without a window: band sums, ratio and vad defined as 0
            for (int w = nw; w < wpt; w++) {
              a.out_win_ratio[ow + w] = 0.0f;
              a.out_win_vad[ow + w] = 0.0f;
              for (int i = 0; i < a.n_channels * a.n_bands; i++)
                a.out_band[(ow + w) * a.n_channels * a.n_bands + i] = 0.0f;
            }
            a.out_win_flag[o] = nw;
            fd++;
          }
        }
      }
      istp[st::kFramesDone] = fd;
      stp[st::kVolAcc] = vol;
    }
    for (; j < a.wmax; j++) wt[j] = -1;
  }
  // synthesis_mem for the next launch = second half of the last frame's
  // window; each lane's float4 loads go out before its stores (a store
  // between them would make every load wait for the one before)
  // (4 streams per pass: lane = float4 q and q + 64 of each stream's 120)
  constexpr int kSynQ = kFrame / 4, kSynS = 4;
  static_assert(kSynQ <= 128 && kWmS % kSynS == 0, "synthesis copy");
  for (int s0 = 0; s0 < kWmS; s0 += kSynS) {
    float4 v[kSynS][2];
    bool ok[kSynS][2];
#pragma unroll
    for (int k = 0; k < kSynS; k++) {
      const int s = sb + s0 + k;
      const int nt = s < a.n_streams ? ticks_of(a, s) : 0;
      const float4 *yl = reinterpret_cast<const float4 *>(
          a.ys + ((size_t)s * a.V + (size_t)max(nt, 1) * a.n_channels - 1) * kWin + kFrame);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int q = tid + 64 * h;
        ok[k][h] = nt > 0 && q < kSynQ;
        v[k][h] = ok[k][h] ? yl[q] : make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < kSynS; k++)
#pragma unroll
      for (int h = 0; h < 2; h++)
        if (ok[k][h])
          reinterpret_cast<float4 *>(a.state + (size_t)(sb + s0 + k) * st::kWords + st::kSyn)[tid + 64 * h] = v[k][h];
  }
}

// ---------------------------------------------------------------------------
// k_fftb: one workgroup per (stream, completed window): FFT B per channel.
// kLds: the transform's work arrays in dynamic LDS (fft_size <= kMaxFftB);
// otherwise each of the grid's workgroups owns a slice of device scratch and
// walks the (stream, window) units grid-stride.  Output index of a window:
// its slot (tick * wpt + rank in the tick, k_winmeta / k_ndmeta).
// ---------------------------------------------------------------------------
__device__ __forceinline__ size_t win_out(const StagedArgs &a, int s, int slot) {
  const int t = slot / a.wpt;
  return ((size_t)t * a.n_streams + s) * a.wpt + (slot - t * a.wpt);
}

template <int NT, bool kLds>
__global__ void __launch_bounds__(NT) k_fftb(StagedArgs a) {
  // W[nc] (+ S[nc] with a radix > 5), then the magnitudes of the reported bins
  extern __shared__ __attribute__((aligned(16))) float2 Wl[];
  const Plan *__restrict__ P = a.plan;
  const int nc = P->ncfft_b, C = a.n_channels;
  float2 *W = kLds ? Wl : a.fb_work + (size_t)blockIdx.x * a.fb_work_stride;
  float2 *S = W + nc;
  float *mag = reinterpret_cast<float *>(W + (P->generic_b ? 2 * nc : nc));
  const int tid = threadIdx.x;
  const float2 *__restrict__ twb = a.fb_tw;
  const float2 *__restrict__ sup = a.fb_sup;
  const int *__restrict__ perm = a.fb_perm;
  const float *__restrict__ hann = a.fb_hann;
  const long long units = (long long)a.n_streams * a.wmax;
  for (long long unit = blockIdx.x; unit < units; unit += gridDim.x) {
    const int s = (int)(unit / a.wmax), j = (int)(unit - (long long)s * a.wmax);
    const int slot = a.win_tick[(size_t)s * a.wmax + j];
    if (slot < 0) continue;  // uniform over the workgroup
    const long long wstart = a.win_start[(size_t)s * a.wmax + j];
    const size_t o = win_out(a, s, slot);
    for (int c = 0; c < C; c++) {
      const float *ring = a.ring + ((size_t)s * C + c) * a.ring_len;
      for (int k = tid; k < nc; k += NT) {
        const int n = perm[k];
        const float t0 = ring[(wstart + 2 * n) % a.ring_len] * hann[2 * n];
        const float t1 = ring[(wstart + 2 * n + 1) % a.ring_len] * hann[2 * n + 1];
        W[k] = make_float2(t0, t1);
      }
      __syncthreads();
      kiss_stages(W, S, P->fac_b, P->nfac_b, nc, twb, tid, NT);
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
#ifndef FVAD_LT_BLOCK
#define FVAD_LT_BLOCK 16
#endif
template <int kL = FVAD_LT_BLOCK>
__device__ __forceinline__ double lt_sum(double acc, const float *buf, size_t bs, unsigned i0, unsigned i1,
                                         double scalar) {
  // blocks of kL entries, the next block's loads issued before this block's
  // adds (two blocks in flight: the chain waits a memory latency per kL
  // entries at most, not per block of its own)
  unsigned i = i0;
  if (i + kL <= i1) {
    float cur[kL];
#pragma unroll
    for (int u = 0; u < kL; u++) cur[u] = buf[(size_t)(i + u) * bs];
    for (; i + 2 * kL <= i1; i += kL) {
      float nxt[kL];
#pragma unroll
      for (int u = 0; u < kL; u++) nxt[u] = buf[(size_t)(i + kL + u) * bs];
#pragma unroll
      for (int u = 0; u < kL; u++) acc += (double)cur[u] * scalar;
#pragma unroll
      for (int u = 0; u < kL; u++) cur[u] = nxt[u];
    }
#pragma unroll
    for (int u = 0; u < kL; u++) acc += (double)cur[u] * scalar;
    i += kL;
  }
  for (; i < i1; i++) acc += (double)buf[(size_t)i * bs] * scalar;
  return acc;
}
// The same over a stream's own contiguous row (the long-term buffers'
// layout, bs == 1): 16-byte loads, blocks of kV of them double-buffered.
template <int kV = FVAD_LT_BLOCK / 4>
__device__ __forceinline__ double lt_sum_row(double acc, const float *row, unsigned i0, unsigned i1, double scalar) {
  unsigned i = i0;
  for (; i < i1 && (i & 3u); i++) acc += (double)row[i] * scalar;  // to a 16-byte boundary
  const float4 *r4 = reinterpret_cast<const float4 *>(row);
  unsigned q = i >> 2;
  const unsigned qe = i < i1 ? i1 >> 2 : q;  // whole float4 in [i, i1)
  if (q + kV <= qe) {
    float4 cur[kV];
#pragma unroll
    for (int u = 0; u < kV; u++) cur[u] = r4[q + u];
    for (; q + 2 * kV <= qe; q += kV) {
      float4 nxt[kV];
#pragma unroll
      for (int u = 0; u < kV; u++) nxt[u] = r4[q + kV + u];
#pragma unroll
      for (int u = 0; u < kV; u++) {
        acc += (double)cur[u].x * scalar;
        acc += (double)cur[u].y * scalar;
        acc += (double)cur[u].z * scalar;
        acc += (double)cur[u].w * scalar;
      }
#pragma unroll
      for (int u = 0; u < kV; u++) cur[u] = nxt[u];
    }
#pragma unroll
    for (int u = 0; u < kV; u++) {
      acc += (double)cur[u].x * scalar;
      acc += (double)cur[u].y * scalar;
      acc += (double)cur[u].z * scalar;
      acc += (double)cur[u].w * scalar;
    }
    q += kV;
  }
  for (; q < qe; q++) {
    const float4 v = r4[q];
    acc += (double)v.x * scalar;
    acc += (double)v.y * scalar;
    acc += (double)v.z * scalar;
    acc += (double)v.w * scalar;
  }
  for (i = i < i1 ? (qe << 2 > i ? qe << 2 : i) : i1; i < i1; i++) acc += (double)row[i] * scalar;  // the tail
  return acc;
}
// entries never written hold the initial average: n adds of one term, done
// per binade (fvad_exact.h: the loop's bits)
__device__ __forceinline__ double lt_sum_init(double acc, double term, unsigned n) {
  return add_const_n(acc, term, n);
}
template <int kL = FVAD_LT_BLOCK>
__device__ __forceinline__ double lt_range(double acc, const float *buf, size_t bs, unsigned p, unsigned q,
                                           unsigned nw, double init, double scalar) {
  const unsigned mid = min(max(nw, p), q);  // [p, mid) written, [mid, q) initial
  acc = bs == 1 ? lt_sum_row<(kL >= 8 ? kL / 4 : 2)>(acc, buf, p, mid, scalar) : lt_sum<kL>(acc, buf, bs, p, mid, scalar);
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

// VADMachine.run's per-window steps (VADMachine.zig:126-230), shared by the
// serial walk (vadm_stream) and the window-parallel kernel (k_vadm_par).
enum { kVmClosed = 0, kVmOpening = 1, kVmOpen = 2, kVmClosing = 3 };
// short-term and channel-ratio averages (pushed every window); `met`: the
// speech condition against the long-term average of the last long push
__device__ __forceinline__ bool vadm_short(VadmState &S, const VadmConst &K, float *st, float *rb, int B, float min_v,
                                           float vr) {
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
  return st_avg > threshold && r_avg > (double)K.ratio_thr;
}
// the speech-state transition, segment output and tracking of one window
__device__ __forceinline__ void vadm_fsm(VadmState &S, const VadmConst &K, unsigned long long index, bool met,
                                         float vad, float vr, VadmSeg *seg, int seg_cap) {
  const int from = S.state;
  bool ended = false;
  switch (from) {
    case kVmClosed:
      if (met) {
        S.state = kVmOpening;
        S.speech_start = index;
      }
      break;
    case kVmOpening:
      if (met && index - S.speech_start >= K.min_open)
        S.state = kVmOpen;
      else if (!met)
        S.state = kVmClosed;
      break;
    case kVmOpen:
      if (!met) {
        S.state = kVmClosing;
        S.speech_end = index;
      }
      break;
    default:  // kVmClosing
      if (met) {
        S.state = kVmOpen;
      } else if (index - S.speech_end >= K.max_gap) {
        S.state = kVmClosed;
        ended = true;
      }
      break;
  }
  if (ended) {  // onSpeechEnd (before the tracking update of this window, as in VADMachine.zig)
    const unsigned long long len = S.speech_end - S.speech_start;
    const float len_rt = (float)len / K.sr;
    if (len_rt >= K.min_dur) {
      if (S.n_segs < (unsigned)seg_cap) {
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
  if (from == kVmClosed && S.state == kVmOpening) {
    S.rnn_vad = vad;
    S.rnn_vad_count = 1;
    S.vol_ratio = vr;
    S.vol_ratio_count = 1;
  } else if (from == kVmOpening || from == kVmOpen) {
    S.rnn_vad += vad;
    S.rnn_vad_count += 1;
    S.vol_ratio += vr;
    S.vol_ratio_count += 1;
  }
}

// Deferred folds.  Between sync points (k_vadm_hbm, final = false) the exact
// fold a push would end with is owed instead of done: the estimate, its
// bound's magnitude and the exact prefix ride in the state (lt_defer long
// pushes since the last exact fold) and the next push's walk continues from
// them, so a machine folds only for a test the bound does not settle, after
// kLtDeferMax long pushes, or at a sync point (final: k_vadm_par's drain, or
// k_vadm_hbm when the push cannot take k_vadm_par), where every machine is
// resolved -- states and segments read after a sync are the reference's.
// (One fold per stream and push was ~4 000 f64 adds in the full-buffer
// regime: k_vadm_hbm 0.44-0.65 ms beside the next push, which stretched the
// co-running k_prep3 and, through it, k_pspecw.)
#ifndef FVAD_LT_DEFER_MAX
#define FVAD_LT_DEFER_MAX 4096
#endif
constexpr unsigned kLtDeferMax = FVAD_LT_DEFER_MAX;
// the fold a deferred machine owes: vadm_stream's fold, the same adds in the
// same order (the exact prefix through the last pushed index, then the
// entries after it)
// lt_neg's bookkeeping for one long push of v
__device__ __forceinline__ void lt_neg_push(VadmState &S, unsigned n, float v) {
  if (S.lt_neg > 0) S.lt_neg--;
  if (!(v >= 0.0f)) S.lt_neg = (int)n;
}
__device__ __forceinline__ void lt_resolve(VadmState &S, const VadmConst &K, const float *lt, size_t lts) {
  if (!S.lt_defer) return;
  const unsigned n = (unsigned)K.n_lt;
  double acc = S.lt_fpre;
  if (S.lt_widx != 0) acc = lt_range(acc, lt, lts, S.lt_widx, n, S.lt_nw, K.init, 1.0 / (double)n);
  S.lt_last = acc;
  S.lt_defer = 0;
}

// One machine over all completed windows of the push for one stream; `lt`
// points at entry 0 of the stream's long-term buffer, `lts` is its stride.
//
// Lazy long-term folds.  Once the long-term buffer is full (from the start
// with an initial average) every window that pushes re-folds ~n - w entries
// (RollingAverage.zig:45-56), ~12 folds per push: 7 ms per push at 2048
// streams once a stream is past its first long_term_speech_avg_sec (a full
// buffer of pushed values, measured with FVAD_DEBUG_VADM_LT_FULL).  But a
// window's average is only *observed* through the next window's test
// st_avg > RN(lt_last * factor), and the last one through the state.  So the
// walk keeps a running estimate of the average (approx += t_new - t_old per
// push, t = RN(entry * 1/n)) with a rigorous bound E on its distance to the
// fold's result -- the fold of nonnegative terms is within (n-1) u of their
// exact sum (u = 2^-53), each estimate update adds <= 2u -- decides every test
// whose outcome the bound settles, runs the exact fold (the same adds in the
// same order as the reference) only for a test it does not settle, and folds
// once at the end of the push for the state.  The cached prefix P_w advances
// by one add per push, as in k_vadm_par.  Every decision and every stored value
// is the reference's; typically one fold per push instead of one per window.
// Used when the buffer is full, the terms are nonnegative (band energies,
// a nonnegative initial average) and the threshold factor is nonnegative;
// otherwise each pushing window folds at once (ra_push_long).
__device__ void vadm_stream(const StagedArgs &a, int m, int s, float *lt, size_t lts, bool final) {
  const int B = a.n_streams, C = a.n_channels, nb = a.n_bands;
  const int nt = ticks_of(a, s);
  const unsigned long long fft = (unsigned long long)a.plan->nfft_b;
  const VadmConst &K = a.vadm.c[m];
  VadmState S = a.vadm.st[(size_t)m * B + s];
  float *st = a.vadm.buf + K.st_off + s, *rb = a.vadm.buf + K.r_off + s;
  VadmSeg *seg = a.vadm.seg + ((size_t)m * B + s) * a.vadm.seg_cap;
  const unsigned n = (unsigned)K.n_lt;
  const double f = (double)K.thr_factor, scalar = 1.0 / (double)n;
  const bool lazy = S.lt_count == n && S.lt_pre_ok && S.lt_has && n > 1 && f >= 0.0 &&
                    !(K.has_init && !(K.init >= 0.0)) && S.lt_neg == 0;
  if (!lazy) lt_resolve(S, K, lt, lts);  // (a deferring machine is lazy; kept for safety)
  unsigned long long *cnt = a.vadm.count;
  // the bound's scale: the test hook's, +inf once a negative entry is pushed
  // (no bound holds then: every later test of the push folds)
  double bscale = a.vadm.bound_scale;
  double approx = S.lt_last, amax = fabs(S.lt_last), fpre = 0.0;
  int pending = 0;  // pushes since lt_last was last folded exactly
  if (S.lt_defer) {  // owed from earlier pushes (deferred folds)
    approx = S.lt_approx;
    amax = S.lt_amax;
    fpre = S.lt_fpre;
    pending = (int)S.lt_defer;
  }
  // the exact average of the current buffer: the fold through the last pushed
  // index (fpre) continued over the entries after it, C order
  auto fold = [&]() {
    double acc = fpre;
    if (S.lt_widx != 0) acc = lt_range(acc, lt, lts, S.lt_widx, n, S.lt_nw, K.init, scalar);
    S.lt_last = acc;
    approx = acc;
    amax = fabs(acc);
    pending = 0;
  };
  // every window of the push in order: ticks, then a tick's slots (several
  // when fft_size < 480)
  for (int t = 0; t < nt; t++)
    for (int w = 0, nw = a.out_win_flag[(size_t)t * B + s]; w < nw; w++) {
      const size_t o = ((size_t)t * B + s) * a.wpt + w;
      const unsigned long long index = S.windows_done * fft;
      float min_v = 999, max_v = 0;
      for (int c = 0; c < C; c++) {
        const float v = a.out_band[(o * C + c) * nb + K.slot];
        if (v < min_v) min_v = v;
        if (v > max_v) max_v = v;
      }
      if ((long long)S.windows_done == a.vadm.negate_at) min_v = -min_v;  // test hook
      S.windows_done++;
      // fft_input.vad orelse 0 (VADMachine.zig:240-246): no vad without the denoiser
      const float vad = a.use_denoiser ? a.out_win_vad[o] : 0.0f, vr = a.out_win_ratio[o];
      bool met;
      if (!lazy) {
        met = vadm_short(S, K, st, rb, B, min_v, vr);
        if (!met) {
          ra_push_long(lt, lts, K.n_lt, S.lt_widx, S.lt_count, S.lt_nw, K.init, S.lt_last, S.lt_has, S.lt_pre,
                       S.lt_pre_ok, min_v);
          lt_neg_push(S, n, min_v);
        }
      } else {
        const double st_avg = ra_push(st, B, K.n_st, S.st_widx, S.st_count, S.st_last, S.st_has, min_v);
        const double r_avg = ra_push(rb, B, K.n_r, S.r_widx, S.r_count, S.r_last, S.r_has, vr);
        met = false;
        if (r_avg > (double)K.ratio_thr) {  // else met is false whatever the long-term average
          if (pending == 0) {
            met = st_avg > S.lt_last * f;
            if (cnt) atomicAdd(cnt + kVcExact, 1ull);
          } else {
            // |approx - fold| <= E (fvad_exact.h lt_bound: the fold's (n-1) u,
            // twice, and 2u per estimate update, on the largest estimate)
            const int d = lt_decide(st_avg, approx, lt_bound(n, (unsigned)pending, amax, bscale), f);
            if (d >= 0) {
              met = d == 1;
              if (cnt) atomicAdd(cnt + kVcSettled, 1ull);
            } else {  // not settled by the bound: the exact fold
              fold();
              met = st_avg > S.lt_last * f;
              if (cnt) atomicAdd(cnt + kVcOpen, 1ull);
            }
          }
        }
        if (!met) {  // push min_v into the long-term buffer (ra_push_long's state, the fold deferred)
          const unsigned wi = S.lt_widx;
          const double t_old = (wi < S.lt_nw ? (double)lt[(size_t)wi * lts] : K.init) * scalar;
          lt[(size_t)wi * lts] = min_v;
          const double t_new = (double)min_v * scalar;
          fpre = S.lt_pre + t_new;  // the fold through index wi
          S.lt_widx = (wi + 1) % n;
          if (S.lt_nw < n) S.lt_nw++;
          S.lt_pre = S.lt_widx == 0 ? 0.0 : fpre;
          lt_estimate(approx, amax, t_new, t_old);
          pending++;
          lt_neg_push(S, n, min_v);
          if (S.lt_neg) bscale = __builtin_inf();
        }
      }
      vadm_fsm(S, K, index, met, vad, vr, seg, a.vadm.seg_cap);
    }
  if (pending && (final || (unsigned)pending >= (a.vadm.defer_max ? a.vadm.defer_max : kLtDeferMax))) {
    fold();
    if (cnt) atomicAdd(cnt + kVcEndFold, 1ull);
  }
  S.lt_defer = (unsigned)pending;
  S.lt_approx = approx;
  S.lt_amax = amax;
  S.lt_fpre = fpre;
  a.vadm.st[(size_t)m * B + s] = S;
}

// ---------------------------------------------------------------------------
// k_vadm_par: the same machine with the long-term averages of a push's
// windows computed side by side.  Once the long-term buffer is full (from
// the start with an initial average) a push at write index w averages
//   acc = P_w + v * s, then acc += e_i * s for i = w + 1 .. n - 1 (C order),
// P_w the cached prefix, a chain of one add per push; the suffix entries are
// the old buffer's, or values pushed earlier in this push (a wrap).  So given
// which windows push, the ~12 averages of a push are independent serial
// chains.  Whether a window pushes (`met` false) depends on the average of the
// last push, so 16 lanes per stream fold the hypothesis "the next 16 windows
// all push" in one round; the stream's leader lane then replays the windows
// in order with the exact averages -- each `met` decided exactly as the
// serial walk does -- and commits every push up to the first window that
// does not push (speech); the next round starts after it.  A round costs one
// suffix chain instead of one per window; windows with no push cost none.
// Bit-identical to vadm_stream (same adds, same order); streams whose buffer
// is not full yet (no initial average) or with more than kVpMaxW windows in
// the push take the serial walk.
// ---------------------------------------------------------------------------
// (48 windows: 4.2 KB of LDS, which fits beside three k_fftAw or four
// k_pcorr workgroups on a CU; the machine state lives in LDS, not in VGPRs)
#ifndef FVAD_VP_BLOCK
#define FVAD_VP_BLOCK 8  // long-term entries per prefetched block
#endif
constexpr int kVpG = 16, kVpS = 4, kVpMaxW = 48;  // lanes per stream, streams per workgroup, windows per push
// acc += e_i * s over old entries [i0, i1): pushed f32 below nw, the initial
// average above (entry i of the stream at lt[i * lts])
__device__ __forceinline__ double lt_fold(double acc, const float *lt, size_t lts, unsigned i0, unsigned i1, unsigned nw,
                                          double init, double scalar) {
  if (i0 >= i1) return acc;
  return lt_range<FVAD_VP_BLOCK>(acc, lt, lts, i0, i1, nw, init, scalar);
}
__global__ void __launch_bounds__(64) k_vadm_par(StagedArgs a) {
  __shared__ float wmin[kVpS][kVpMaxW], wvad[kVpS][kVpMaxW], wvr[kVpS][kVpMaxW];
  __shared__ float pv[kVpS][kVpMaxW];  // values pushed in this push, in push order (committed + the round's hypotheses)
  __shared__ double favg[kVpS][kVpG];
  __shared__ double rpre[kVpS];  // the cached prefix before the round's first push
  __shared__ int rnd[kVpS][4];  // round: first window, pushes committed so far, state (0 run, 1 done, 2 serial)
  __shared__ VadmState Ss[kVpS];
  const int B = a.n_streams, C = a.n_channels, nb = a.n_bands;
  const int g = threadIdx.x / kVpG, r = threadIdx.x % kVpG;
  const int s = blockIdx.x * kVpS + g;
  const bool sok = s < B && ticks_of(a, s) > 0;
  const int nt = sok ? ticks_of(a, s) : 0;
  const unsigned long long fft = (unsigned long long)a.plan->nfft_b;
  const int self = threadIdx.x;
  for (int m = 0; m < a.vadm.n; m++) {
    const VadmConst &K = a.vadm.c[m];
    float *lt = a.vadm.buf + K.lt_off + (size_t)(sok ? s : 0) * K.lt_pitch;  // the stream's row
    const size_t lts = 1;
    // the push's windows in order -> LDS (16 ticks at a time, positions by a
    // prefix count over the group's lanes)
    int Kw = 0;
    for (int t0 = 0; t0 < nt; t0 += kVpG) {
      const int t = t0 + r;
      const int nwt = t < nt ? a.out_win_flag[(size_t)t * B + s] : 0;
      int pos = nwt;
#pragma unroll
      for (int d = 1; d < kVpG; d <<= 1) {
        const int up = __shfl(pos, self - d);
        if (r >= d) pos += up;
      }
      const int tot = __shfl(pos, g * kVpG + kVpG - 1);
      for (int w = 0; w < nwt; w++) {
        const int k = Kw + pos - nwt + w;
        if (k < kVpMaxW) {
          const size_t o = ((size_t)t * B + s) * a.wpt + w;
          float min_v = 999;
          for (int c = 0; c < C; c++) {
            const float v = a.out_band[(o * C + c) * nb + K.slot];
            if (v < min_v) min_v = v;
          }
          wmin[g][k] = min_v;
          wvad[g][k] = a.use_denoiser ? a.out_win_vad[o] : 0.0f;
          wvr[g][k] = a.out_win_ratio[o];
        }
      }
      Kw += tot;
    }
    if (r == 0) {
      Ss[g] = a.vadm.st[(size_t)m * B + (sok ? s : 0)];
      // k_vadm_par runs at sync points only: a fold owed from earlier pushes
      // first (the walk below needs the exact average), also for a stream
      // with no ticks in this push
      if (sok) {
        lt_resolve(Ss[g], K, lt, lts);
      } else if (s < B) {
        VadmState S2 = a.vadm.st[(size_t)m * B + s];
        if (S2.lt_defer) {
          lt_resolve(S2, K, a.vadm.buf + K.lt_off + (size_t)s * K.lt_pitch, 1);
          a.vadm.st[(size_t)m * B + s] = S2;
        }
      }
    }
    wave_sync();
    if (r == 0 && sok && a.vadm.negate_at >= 0) {  // test hook FVAD_DEBUG_VADM_NEGATE_AT
      const long long k = a.vadm.negate_at - (long long)Ss[g].windows_done;
      if (k >= 0 && k < Kw && k < kVpMaxW) wmin[g][k] = -wmin[g][k];
      wave_sync();
    }
    VadmState &S = Ss[g];
    float *st = a.vadm.buf + K.st_off + (sok ? s : 0), *rb = a.vadm.buf + K.r_off + (sok ? s : 0);
    VadmSeg *seg = a.vadm.seg + ((size_t)m * B + (sok ? s : 0)) * a.vadm.seg_cap;
    // (n > kVpMaxW: a push wraps around the buffer at most once)
    const bool forced = a.vadm.par_serial_every > 0 && s % a.vadm.par_serial_every == 0;
    const bool fast = sok && !forced && Kw <= kVpMaxW && K.n_lt > kVpMaxW && S.lt_count == (unsigned)K.n_lt &&
                      S.lt_pre_ok;
    const unsigned n = (unsigned)K.n_lt, wbase = S.lt_widx, nw0 = S.lt_nw;
    const double scalar = 1.0 / (double)n;  // the full buffer's
    if (r == 0) {
      rnd[g][0] = 0;
      rnd[g][1] = 0;
      rnd[g][2] = !sok ? 1 : (fast ? 0 : 2);
    }
    wave_sync();
    // leader state across rounds (lane 0 of the group)
    int j = 0, npush = 0;
    double pre = S.lt_pre;
    for (;;) {
      if (r == 0 && rnd[g][2] == 0) {
        // windows that do not push need no fold: replay them up to the next
        // one that does (its short-term pushes done, its long push pending)
        while (j < Kw) {
          const unsigned long long index = S.windows_done * fft;
          const bool met = vadm_short(S, K, st, rb, B, wmin[g][j], wvr[g][j]);
          if (!met) break;  // window j pushes: its short-term pushes are done, its long push waits for the folds
          S.windows_done++;
          vadm_fsm(S, K, index, met, wvad[g][j], wvr[g][j], seg, a.vadm.seg_cap);
          j++;
        }
        if (j >= Kw) rnd[g][2] = 1;
        rnd[g][0] = j;
        rnd[g][1] = npush;
        // the round's hypotheses: windows j, j + 1, ... push in order
        for (int q = 0; q < kVpG && j + q < Kw; q++) pv[g][npush + q] = wmin[g][j + q];
        rpre[g] = pre;
      }
      wave_sync();
      const int state = rnd[g][2];
      if (__ballot(state == 0) == 0) break;  // every group of the wave is done with its fast walk
      if (state == 0) {
        // lane r: the push of window j0 + r after the r pushes before it
        const int j0 = rnd[g][0], np = rnd[g][1];
        if (j0 + r < Kw) {
          const unsigned k = (unsigned)(np + r);  // pushes of this push before it
          const unsigned nw = min(n, nw0 + k + 1);
          // its prefix P_w: the chain of one add per push since the cached
          // one; w: its write index
          double P = rpre[g];
          unsigned w = (wbase + (unsigned)np) % n;
#pragma unroll 1
          for (int q = 0; q < r; q++) {
            P = (w + 1 == n) ? 0.0 : P + (double)pv[g][np + q] * scalar;
            w = (w + 1 == n) ? 0u : w + 1;
          }
          double acc = P + (double)pv[g][np + r] * scalar;
          if (wbase + k < n) {
            // no wrap in this push: every entry past w is the old buffer's
            acc = lt_fold(acc, lt, lts, w + 1, n, nw, K.init, scalar);
          } else {
            // wrapped: (w, wbase) old entries (all pushed by now), [wbase, n) pushed in this push
            acc = lt_fold(acc, lt, lts, w + 1, wbase, nw, K.init, scalar);
            for (unsigned i = wbase; i < n; i++) acc += (double)pv[g][i - wbase] * scalar;
          }
          favg[g][r] = acc;
        }
      }
      wave_sync();
      if (r == 0 && state == 0) {
        // replay in order with the exact averages; commit up to the first
        // window that does not push
        const int j0 = j;
        for (int q = 0; q < kVpG && j0 + q < Kw; q++) {
          const int jj = j0 + q;
          const unsigned long long index = S.windows_done * fft;
          bool met = false;
          if (q > 0) met = vadm_short(S, K, st, rb, B, wmin[g][jj], wvr[g][jj]);
          if (!met) {
            // the long push (ra_push_long's state updates, the average folded above)
            const unsigned w = S.lt_widx;
            S.lt_widx = (w + 1) % n;
            if (S.lt_nw < n) S.lt_nw++;
            pre = (w + 1 == n) ? 0.0 : pre + (double)wmin[g][jj] * scalar;
            S.lt_pre = pre;
            S.lt_last = favg[g][q];
            S.lt_has = 1;
            lt_neg_push(S, n, wmin[g][jj]);
            npush++;
          }
          S.windows_done++;
          vadm_fsm(S, K, index, met, wvad[g][jj], wvr[g][jj], seg, a.vadm.seg_cap);
          j = jj + 1;
          if (met) break;
        }
      }
      wave_sync();
    }
    if (r == 0 && sok) {
      if (rnd[g][2] == 2) {
        // a machine outside the window-parallel case (launch_vadm sends
        // engines whose machines can get here to k_vadm_hbm; the test hook
        // par_serial_every forces it): the serial walk on the leader lane,
        // from the untouched state in HBM
        vadm_stream(a, m, s, lt, lts, true);
      } else {
        // the push's long-term values into the buffer (read above as the old entries)
        unsigned w = wbase;
#pragma unroll 1
        for (int q = 0; q < npush; q++) {
          lt[(size_t)w * lts] = pv[g][q];
          w = (w + 1 == n) ? 0u : w + 1;
        }
        a.vadm.st[(size_t)m * B + s] = S;
      }
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------
// launcher
// ---------------------------------------------------------------------------
const char *staged_kernel_name(int i) {
  static const char *const names[kStagedKernels] = {"k_prep3", "k_fftAw",  "k_plpc",  "k_pcorr",   "k_select", "k_pspecw",
                                                    "k_rnn3",  "k_synthw", "k_ola",   "k_winmeta", "k_fftbw"};
  return (i >= 0 && i < kStagedKernels) ? names[i] : nullptr;
}

namespace {
// persistent grids: exactly the resident capacity (blocks per CU from the
// occupancy calculator x CUs), so no workgroup starts late and leaves a tail
template <typename K>
int blocks_per_cu(K kernel, int threads) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  return per_cu;
}
}  // namespace

// ---------------------------------------------------------------------------
// use_denoiser = false (VAD.zig:206-212,239-249): the pipeline reads fft_size
// frames of raw input straight into FFT B; no rnnoise, no per-frame vad.  The
// reference takes a window as soon as fft_size samples are in, whatever the
// size of the pushes, so this path counts samples, not ticks: a stream's last
// valid tick may hold only a.tail[s] real samples (the end of a stream, or the
// remainder of an AudioPipeline push), and st::kNdSamples (u64) is the
// stream's absolute sample count.
// k_ndring: the real input samples -> the stream's re-block ring, per-tick vad
// / ratio set to -1 (not produced by the reference on this path), the raw
// input as the "denoised" output.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int nd_real(const StagedArgs &a, int s, int t, int nt) {
  return (a.tail && t == nt - 1) ? a.tail[s] : kFrame;
}
__device__ __forceinline__ unsigned long long *nd_count(const StagedArgs &a, int s) {
  return reinterpret_cast<unsigned long long *>(a.state + (size_t)s * st::kWords + st::kNdSamples);
}

__global__ void __launch_bounds__(256) k_ndring(StagedArgs a) {
  const int C = a.n_channels, V = a.V;
  const int q = threadIdx.x & 127;
  const long long fl = (long long)blockIdx.x * 2 + (threadIdx.x >> 7);
  if (fl >= (long long)a.n_streams * V || q >= kFrame / 4) return;
  const int s = (int)(fl / V), v = (int)(fl - (long long)s * V);
  const int nt = ticks_of(a, s);
  if (v >= nt * C) return;
  const int t = v / C, c = v - t * C, i = 4 * q;
  const size_t o = (size_t)t * a.n_streams + s;
  const float4 x = *reinterpret_cast<const float4 *>(a.pcm + (o * C + c) * kFrame + i);
  const int n = nd_real(a, s, t, nt);
  const unsigned long long p0 = *nd_count(a, s) + (unsigned long long)t * kFrame + i;
  float *ring = a.ring + ((size_t)s * C + c) * a.ring_len;
  const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int e = 0; e < 4; e++)
    if (i + e < n) ring[(p0 + e) % (unsigned long long)a.ring_len] = xv[e];
  if (a.out_den) *reinterpret_cast<float4 *>(a.out_den + (o * C + c) * kFrame + i) = x;
  if (i == 0 && c == 0) {
    a.out_vad[o] = -1.0f;
    a.ratio[o] = -1.0f;
  }
}

// k_ndmeta: window completion per tick (a window completes in the tick that
// brings its last sample; fft_size < 480: several per tick), lane per stream;
// the completed windows' volume ratios are k_ndvol's.
__global__ void __launch_bounds__(64) k_ndmeta(StagedArgs a) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= a.n_streams) return;
  const int nt = ticks_of(a, s), C = a.n_channels, FB = a.nfft_b;
  int *wt = a.win_tick + (size_t)s * a.wmax;
  long long *wsx = a.win_start + (size_t)s * a.wmax;
  int j = 0;
  if (nt > 0) {
    unsigned long long *cnt = nd_count(a, s);
    const unsigned long long sd0 = *cnt;
    for (int t = 0; t < nt; t++) {
      const size_t o = (size_t)t * a.n_streams + s, ow = o * a.wpt;
      // the tick's samples [a0, end) complete every window ending in (a0, end]
      // (fft_size < 480: several)
      const unsigned long long a0 = sd0 + (unsigned long long)t * kFrame;
      const unsigned long long end = a0 + (unsigned)nd_real(a, s, t, nt);
      unsigned long long next_end = (a0 / (unsigned)FB + 1) * (unsigned)FB;
      int nw = 0;
      for (; next_end <= end; next_end += (unsigned)FB, nw++) {
        a.out_win_vad[ow + nw] = -1.0f;
        wt[j] = t * a.wpt + nw;
        wsx[j] = (long long)(next_end - (unsigned)FB);
        j++;
      }
      for (int w = nw; w < a.wpt; w++) {
        a.out_win_ratio[ow + w] = 0.0f;
        a.out_win_vad[ow + w] = 0.0f;
        for (int i = 0; i < C * a.n_bands; i++) a.out_band[(ow + w) * C * a.n_bands + i] = 0.0f;
      }
      a.out_win_flag[o] = nw;
    }
    *cnt = sd0 + (unsigned long long)(nt - 1) * kFrame + (unsigned)nd_real(a, s, nt - 1, nt);
  }
  for (; j < a.wmax; j++) wt[j] = -1;
}

// k_ndvol: a completed window's volume ratio, preAnalyzeSegment over its
// fft_size input samples (VAD.zig:253-272: rmsVolume per channel =
// sqrt(sum x^2 / n) with the sum in sample order, audio_utils.zig:14-24; min /
// max over channels in channel order).  The sum is one serial f32 chain per
// channel, so the parallelism is across windows: lane per (stream, window of
// this push) -- ~fft_size / 480 times k_ndmeta's lanes.
__global__ void __launch_bounds__(64) k_ndvol(StagedArgs a) {
  const long long item = (long long)blockIdx.x * 64 + threadIdx.x;
  if (item >= (long long)a.n_streams * a.wmax) return;
  const int s = (int)(item / a.wmax), j = (int)(item - (long long)s * a.wmax);
  const int t = a.win_tick[(size_t)s * a.wmax + j];
  if (t < 0) return;
  const int C = a.n_channels, FB = a.nfft_b;
  const unsigned long long ws = (unsigned long long)a.win_start[(size_t)s * a.wmax + j];
  float vol_min = 1, vol_max = 0;
  for (int c = 0; c < C; c++) {
    const float *ring = a.ring + ((size_t)s * C + c) * a.ring_len;
    long long ri = (long long)(ws % (unsigned long long)a.ring_len);
    float sum = 0.0f;
    for (int n = 0; n < FB; n++) {
      const float x = ring[ri];
      sum += x * x;
      if (++ri == a.ring_len) ri = 0;
    }
    const float vol = sqrtf(sum / (float)FB);
    if (vol < vol_min) vol_min = vol;
    if (vol > vol_max) vol_max = vol;
  }
  a.out_win_ratio[win_out(a, s, t)] = vol_max == 0 ? 0.0f : vol_min / vol_max;
}

// every launch is checked where it is issued: a failed launch in the middle of
// the pipeline returns its own error instead of surfacing at the end
#define FVAD_LAUNCH_TRY(x)            \
  do {                                \
    const hipError_t e_ = (x);        \
    if (e_ != hipSuccess) return e_;  \
  } while (0)
#define FVAD_KERNEL_TRY(...)                   \
  do {                                         \
    hipLaunchKernelGGL(__VA_ARGS__);           \
    FVAD_LAUNCH_TRY(hipGetLastError());        \
  } while (0)

// FFT B of every completed window: the wave-per-window kernel for 2048 points
// (one window per tick at most), the block kernel k_fftb (mixed radix) for
// every other size -- work arrays in LDS up to kMaxFftB and 160 KB, else in
// device scratch (the engine sizes a.fb_work by fftb_work_stride)
bool fftb_generic(int nc) {  // kf_factor(nc) has a radix > 5
  int n = nc;
  for (int p : {4, 2, 3, 5})
    while (n % p == 0) n /= p;
  return n > 1;
}

long long fftb_work_stride(int nfft_b, int bin_lo_all, int bin_hi_all, int generic) {
  const long long nc = nfft_b / 2, bins = bin_hi_all - bin_lo_all + 1;
  const long long lds = (long long)sizeof(float2) * nc * (generic ? 2 : 1) + (long long)sizeof(float) * bins;
  if (nfft_b <= kMaxFftB && lds <= 160 * 1024) return 0;
  return (nc * (generic ? 2 : 1) + (bins + 1) / 2 + 1) & ~1LL;  // float2 units, 16-byte aligned slices
}

hipError_t launch_fftb(const StagedArgs &a, int n_cu, hipStream_t stream) {
  if (a.nfft_b == 2048) return launch_wave(kWaveFftB, a, n_cu, stream);
  static const bool attr = [] {
    bool ok = true;
    for (const void *k : {reinterpret_cast<const void *>(&k_fftb<256, true>),
                          reinterpret_cast<const void *>(&k_fftb<64, true>)})
      ok &= hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
  }();
  (void)attr;
  const long long units = (long long)a.n_streams * a.wmax;
  if (a.fb_work) {
    const unsigned grid = (unsigned)std::min<long long>(units, a.fb_work_blocks);
    FVAD_KERNEL_TRY((k_fftb<256, false>), dim3(grid), dim3(256), 0, stream, a);
    return hipSuccess;
  }
  const int nc = a.nfft_b / 2;
  const size_t lds = sizeof(float2) * (size_t)nc * (fftb_generic(nc) ? 2 : 1) +
                     sizeof(float) * (size_t)(a.bin_hi_all - a.bin_lo_all + 1);
  const unsigned grid = (unsigned)std::min<long long>(units, 1 << 16);
  if (nc <= 64)  // fft_size <= 128: a wave per window
    FVAD_KERNEL_TRY((k_fftb<64, true>), dim3(grid), dim3(64), lds, stream, a);
  else
    FVAD_KERNEL_TRY((k_fftb<256, true>), dim3(grid), dim3(256), lds, stream, a);
  return hipSuccess;
}

// the fused synthesis tail (k_olafb) serves fft_size 2048 with <= 4 channels;
// FVAD_OLAFB=0 selects k_ola + k_winmeta + k_fftbw (A/B)
bool olafb_fused(const StagedArgs &a) {
  static const bool off = [] {
    const char *v = getenv("FVAD_OLAFB");
    return v && atoi(v) == 0;
  }();
  return !off && a.nfft_b == 2048 && a.n_channels <= 4;
}

hipError_t launch_prep(const StagedArgs &a, hipStream_t stream, hipEvent_t *ev) {
  (void)hipGetLastError();
  if (ev) FVAD_LAUNCH_TRY(hipEventRecord(ev[0], stream));
  const int S = prep_streams(a.n_channels);
  FVAD_KERNEL_TRY(k_prep3, dim3((a.n_streams + S - 1) / S), dim3(64), 0, stream, a);
  if (ev) FVAD_LAUNCH_TRY(hipEventRecord(ev[1], stream));
  return hipSuccess;
}

hipError_t launch_staged(const StagedArgs &a, int n_cu, hipStream_t stream, hipEvent_t *ev, hipEvent_t fft_a_done,
                         hipStream_t fa_stream, hipEvent_t fa_after, hipEvent_t synth_done) {
  static const int p_plpc = blocks_per_cu(k_plpc, 256);
  const int g_plpc = p_plpc * n_cu;
  const long long frames = (long long)a.n_streams * a.V;
  auto grid = [&](long long units, int resident) { return dim3((unsigned)std::min<long long>(units, resident)); };
  (void)hipGetLastError();
  // a.work: zero when the engine is created, then reset by every push's
  // k_select for the next (the kernels before it) and this push (after it)
  static_assert(kWorkSlots * kQueues <= kWorkCounters, "work counters");
#define REC(k) \
  if (ev) FVAD_LAUNCH_TRY(hipEventRecord(ev[k], stream))
  // k_fftAw and the pitch branch (k_plpc -> k_pcorr -> k_select) run in
  // order (side by side on two streams they stretch each other: 15.0 vs 14.1
  // ms per push in r1); k_fftAw itself may run on fa_stream beside the
  // previous push's k_olafb (fvad_staged.h)
  if (fa_stream && fft_a_done) {
    // k_fftAw on fa_stream beside the previous push's k_olafb: it writes
    // nothing that kernel reads, only what the previous push's k_synthw read
    if (fa_after) FVAD_LAUNCH_TRY(hipStreamWaitEvent(fa_stream, fa_after, 0));
    if (ev) FVAD_LAUNCH_TRY(hipEventRecord(ev[2], fa_stream));
    FVAD_LAUNCH_TRY(launch_wave(kWaveFftA, a, n_cu, fa_stream));
    if (ev) FVAD_LAUNCH_TRY(hipEventRecord(ev[3], fa_stream));
    FVAD_LAUNCH_TRY(hipEventRecord(fft_a_done, fa_stream));
    FVAD_LAUNCH_TRY(hipStreamWaitEvent(stream, fft_a_done, 0));
  } else {
    REC(2);
    FVAD_LAUNCH_TRY(launch_wave(kWaveFftA, a, n_cu, stream));
    if (fft_a_done) FVAD_LAUNCH_TRY(hipEventRecord(fft_a_done, stream));
    REC(3);
  }
  {
    const long long tiles = (long long)((a.n_streams + 63) / 64) * a.n_ticks * a.n_channels;
    REC(14);
    // as many workgroups as give every one the same number of quads: 3 200
    // tiles on 2 048 wave slots run as 2 even rounds on 400 workgroups rather
    // than a full round and a 56 % one (0.90 -> 0.88 ms)
    const long long quads = (tiles + 3) / 4, rounds = (quads + g_plpc - 1) / g_plpc;
    FVAD_KERNEL_TRY(k_plpc, grid((quads + rounds - 1) / rounds, g_plpc), dim3(256), 0, stream, a);
    REC(4);
    FVAD_LAUNCH_TRY(launch_pcorr(a, tiles, n_cu, stream));
  }
  REC(5);
  FVAD_KERNEL_TRY(k_select, dim3((a.n_streams + kSelStreams - 1) / kSelStreams), dim3(64), 0, stream, a);
  REC(6);
  REC(7);
  if (!(a.gru16_frags && a.fuse16))  // FVAD_MODE_FP16_FUSED: k_fused16 computes the pitch spectra
    FVAD_LAUNCH_TRY(launch_wave(kWavePspec, a, n_cu, stream));
  REC(8);
  if (a.gru16_frags)  // FVAD_MODE_FP16: the GRU stack on the matrix cores (configs[4])
    FVAD_LAUNCH_TRY(launch_gru16(a, stream));
  else
    FVAD_KERNEL_TRY(k_rnn3, dim3((a.n_streams + kR3S - 1) / kR3S), dim3(kR3NT), 0, stream, a);
  REC(9);
  FVAD_LAUNCH_TRY(launch_wave(kWaveSynth, a, n_cu, stream));
  if (ev && synth_done) {
    // a timed push: its timing event ev[10] (k_synthw's end, the tail's start)
    // is also the one the next push's k_fftAw waits for, so every push has
    // one event record between k_synthw and the tail.  (With a second one in
    // the timed pushes the tail's dispatch fell behind the next k_fftAw's,
    // whose persistent grid then took the CUs first: k_plpc ~130 us late in
    // every timed push.)
    FVAD_LAUNCH_TRY(hipEventRecord(ev[10], stream));
  } else {
    if (synth_done) FVAD_LAUNCH_TRY(hipEventRecord(synth_done, stream));
    REC(10);
  }
  if (olafb_fused(a)) {
    // overlap-add, window bookkeeping and FFT B in one kernel (k_olafb);
    // the k_winmeta / k_fftbw events bracket nothing
    FVAD_LAUNCH_TRY(launch_wave(kWaveOlaFb, a, n_cu, stream));
    REC(11);
    REC(12);
    REC(13);
  } else {
    FVAD_KERNEL_TRY(k_ola, dim3((unsigned)((frames + 1) / 2)), dim3(256), 0, stream, a);
    REC(11);
    FVAD_KERNEL_TRY(k_winmeta, dim3((a.n_streams + kWmS - 1) / kWmS), dim3(64), 0, stream, a);
    REC(12);
    FVAD_LAUNCH_TRY(launch_fftb(a, n_cu, stream));
    REC(13);
  }
#undef REC
  return hipSuccess;
}

// k_vadm_hbm: the same machine, long-term buffers walked in HBM, no LDS, 16
// lanes per workgroup: a light kernel that co-runs with the next push's
// pipeline on the engine's side stream.
#ifndef FVAD_VADM_LANES
#define FVAD_VADM_LANES 64
#endif
constexpr int kVadmHbmLanes = FVAD_VADM_LANES;  // streams per workgroup (one wave); 16 / 32 / 64 measured within noise, 64 takes fewest wave slots
__global__ void __launch_bounds__(64) k_vadm_hbm(StagedArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_streams) return;
  const bool final = a.vadm.vfinal != 0;
  if (ticks_of(a, s) <= 0) {  // no windows; at a sync point its owed fold is still due
    if (final)
      for (int m = 0; m < a.vadm.n; m++) {
        VadmState *p = a.vadm.st + (size_t)m * a.n_streams + s;
        if (p->lt_defer) {
          VadmState S = *p;
          lt_resolve(S, a.vadm.c[m], a.vadm.buf + a.vadm.c[m].lt_off + (size_t)s * a.vadm.c[m].lt_pitch, 1);
          *p = S;
        }
      }
    return;
  }
  for (int m = 0; m < a.vadm.n; m++)
    vadm_stream(a, m, s, a.vadm.buf + a.vadm.c[m].lt_off + (size_t)s * a.vadm.c[m].lt_pitch, 1, final);
}

hipError_t launch_nodenoise(const StagedArgs &a, int n_cu, hipStream_t stream) {
  (void)hipGetLastError();
  const long long frames = (long long)a.n_streams * a.V;
  FVAD_KERNEL_TRY(k_ndring, dim3((unsigned)((frames + 1) / 2)), dim3(256), 0, stream, a);
  FVAD_KERNEL_TRY(k_ndmeta, dim3((a.n_streams + 63) / 64), dim3(64), 0, stream, a);
  FVAD_KERNEL_TRY(k_ndvol, dim3((unsigned)(((long long)a.n_streams * a.wmax + 63) / 64)), dim3(64), 0, stream, a);
  return launch_fftb(a, n_cu, stream);
}

hipError_t launch_vadm(const StagedArgs &a, hipStream_t stream, bool fast, bool *ran_par) {
  (void)hipGetLastError();
  // k_vadm_par's case: every machine's long-term buffer full from the start
  // (an initial average) and longer than a push's windows, at most kVpMaxW
  // windows per push (wmax bounds them)
  bool par = fast && a.wmax <= kVpMaxW;
  for (int m = 0; m < a.vadm.n; m++) par = par && a.vadm.c[m].has_init && a.vadm.c[m].n_lt > kVpMaxW;
  if (ran_par) *ran_par = par;
  if (!par)
    FVAD_KERNEL_TRY(k_vadm_hbm, dim3((a.n_streams + kVadmHbmLanes - 1) / kVadmHbmLanes), dim3(kVadmHbmLanes), 0,
                    stream, a);
  else
    FVAD_KERNEL_TRY(k_vadm_par, dim3((a.n_streams + kVpS - 1) / kVpS), dim3(kVpS * kVpG), 0, stream, a);
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// k_pcm16: the 16-bit ingest's conversion (fvad_engine_submit_i16), samples
// k -> k / 32768.0f, libsndfile's short -> float normalisation (the simulator's
// WAV reader does the same), exact in f32.  HBM-bound streaming: 16 B in and
// 32 B out per thread and step, grid-stride over the push.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pcm16(const int4 *__restrict__ src, float4 *__restrict__ dst, size_t n8) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    const int4 v = src[i];
    const int w[4] = {v.x, v.y, v.z, v.w};
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o[2 * k] = (float)(short)(w[k] & 0xffff) * (1.0f / 32768.0f);
      o[2 * k + 1] = (float)(short)(w[k] >> 16) * (1.0f / 32768.0f);
    }
    dst[2 * i] = make_float4(o[0], o[1], o[2], o[3]);
    dst[2 * i + 1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}

hipError_t launch_pcm16(const int16_t *src, float *dst, size_t n, hipStream_t stream) {
  if (n % 8) return hipErrorInvalidValue;
  const size_t n8 = n / 8;
  const unsigned grid = (unsigned)std::min<size_t>((n8 + 255) / 256, 256 * 16);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pcm16, dim3(grid), dim3(256), 0, stream, reinterpret_cast<const int4 *>(src),
                     reinterpret_cast<float4 *>(dst), n8);
  return hipGetLastError();
}

}  // namespace fvad
