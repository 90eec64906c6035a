// k_gru16: the staged pipeline's recurrence with the GRU stack on the matrix
// cores -- BASELINE.json configs[4]'s "fp16 GRU weights" variant (engine mode
// FVAD_MODE_FP16), replacing k_rnn3 (fvad_staged.hip) and nothing else.
//
// What it computes is rnnoise's compute_rnn (rnn.c, called from
// rnnoise_process_frame at Denoiser.zig:60) plus the recurrent feature work
// k_rnn3 does (cepstral memory, deltas, spectral variability, gain smoothing).
// The features, activations, state updates and gain smoothing are the same f32
// expressions as k_rnn3; only the gate sums change: every neuron's sum
// b + sum_j W[j] in[j] is a v_mfma_f32_16x16x32_f16 chain with the int8 weights
// as exact f16 values and the inputs rounded to f16 (f32 accumulation).  That
// is the stated tolerance of configs[4] (vad |d| <= 2e-2,
// segments identical or reported), not bit-exactness.
//
// Layout.  A workgroup owns S <= 16 streams = the 16 columns (N) of every
// MFMA; rows (M) are neurons, 16 per tile; K runs over the layer's input
// vector in the rnnimg term order (inputs in concatenation order, then the
// state or r*state), 8-element chunks of a per-stream f16 operand row in LDS.
// Each wave keeps the A fragments (weights) of its tiles in registers for the
// whole kernel (24 slots = 96 VGPRs); the denoise z|r matrix (84 of the 192
// fragments) sits in LDS.  A tile costs per frame one ds_read_b128
// of B (and of A from LDS) per K-block plus the MFMA chain.
//
// Frame t is seven phases (one barrier each) on 8 waves; features of t+1 and
// the gains of t-1 run on waves the phase leaves idle:
//   P0  dense(t) [w0,1]                den_out(t-1) [w2,3]
//   P1  vad z|r(t) [w4..6]             features(t+1) [w0..3]   gains(t-1) [w7]
//   P2  vad h(t) [w4,5]                spectral variability(t+1) [w0,1]
//   P3  noise z|r(t) [w0..5]           vad_out(t) [w6]         fetch raw features(t+2)
//   P4  noise h(t) [w5..7]
//   P5  denoise z|r(t) [w0..7, w0..3 a second tile]
//   P6  denoise h(t) [w2..7]           stage raw features(t+2)
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "fvad_device.h"
#include "fvad_internal.h"
#include "fvad_staged.h"
#include "fvad_staged_dev.h"

namespace fvad {
namespace g16 {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

// operand row of one stream, in 8-element chunks
enum OpSeg { kFeat = 0, kDense, kSv, kRsv, kSn, kRsn, kSd, kRsd, kNSeg };
constexpr int kSegBase[kNSeg] = {0, 12, 15, 18, 21, 27, 33, 45};  // feature slot 1 at chunk 6
constexpr int kZeroChunk = 57;
constexpr int kRowChunks = 59;  // 944 B: rows of 16 streams fall on distinct 4-bank groups
constexpr int kRowHalf = kRowChunks * 8;
// image matrix -> operand segment of each of its rnnimg segments (fvad_internal.h)
constexpr int kMatSeg[rnnimg::kMats][4] = {{kFeat, -1, -1, -1}, {kDense, kSv, -1, -1},   {kDense, kRsv, -1, -1},
                                           {kDense, kSv, kFeat, kSn}, {kDense, kSv, kFeat, kRsn},
                                           {kSv, kSn, kFeat, kSd},    {kSv, kSn, kFeat, kRsd},
                                           {kSd, -1, -1, -1},         {kSv, -1, -1, -1}};
constexpr int kTiles[rnnimg::kMats] = {2, 3, 2, 6, 3, 12, 6, 2, 1};
constexpr int nkb(int m) { return (rnnimg::stride(m) + 31) / 32; }
constexpr int frag_base(int m) {
  int o = 0;
  for (int i = 0; i < m; i++) o += kTiles[i] * nkb(i);
  return o;
}
constexpr int kFrags = frag_base(rnnimg::kMats);
constexpr int bias_base(int m) {
  int o = 0;
  for (int i = 0; i < m; i++) o += kTiles[i] * 16;
  return o;
}
constexpr int kBiasRows = bias_base(rnnimg::kMats);
static_assert(nkb(5) == 7 && nkb(3) == 5 && nkb(0) == 2 && nkb(7) == 3 && nkb(8) == 1, "K blocks");

// chunk q of matrix m -> operand chunk (feature chunks: slot 0; bit 0x100 marks them)
constexpr int op_chunk(int m, int q) {
  int c0 = 0;
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const int n = rnnimg::pad8(rnnimg::kSegs[m][g]) / 8;
    if (q < c0 + n) {
      const int seg = kMatSeg[m][g];
      return kSegBase[seg] + (q - c0) + (seg == kFeat ? 0x100 : 0);
    }
    c0 += n;
  }
  return kZeroChunk;
}

}  // namespace g16

// Host side: the MFMA images from the int8 rnnimg image (fvad_engine.cpp).
// frags: [kFrags][64 lanes][8] f16 bits, lane l of fragment (m, tile, kb) holds
// A[row tile*16 + (l & 15)][k = 32 kb + 8 (l >> 4) + j]; bias: [kBiasRows] f32.
int gru16_frag_count() { return g16::kFrags; }
int gru16_bias_rows() { return g16::kBiasRows; }
void gru16_build(const int8_t *img, uint16_t *frags, float *bias) {
  namespace R = rnnimg;
  auto f16bits = [](int v) -> uint16_t {  // int8 -> binary16, exact
    const _Float16 h = (_Float16)v;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    return u;
  };
  for (int m = 0; m < R::kMats; m++) {
    const int K = R::stride(m), nk = g16::nkb(m);
    for (int t = 0; t < g16::kTiles[m]; t++) {
      for (int r = 0; r < 16; r++) {
        const int c = t * 16 + r;
        bias[g16::bias_base(m) + c] = c < R::kCols[m] ? (float)img[R::off_b(m) + c] : 0.0f;
      }
      for (int kb = 0; kb < nk; kb++) {
        uint16_t *f = frags + (size_t)(g16::frag_base(m) + t * nk + kb) * 64 * 8;
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 8; j++) {
            const int c = t * 16 + (l & 15), k = 32 * kb + 8 * (l >> 4) + j;
            f[l * 8 + j] = f16bits(c < R::kCols[m] && k < K ? img[R::off_w(m) + c * K + k] : 0);
          }
      }
    }
  }
}

namespace {
using namespace g16;

constexpr int kGS = 16;      // streams per workgroup (MFMA N)
constexpr int kGNT = 512;    // 8 waves, 2 per SIMD (fragments + operands need > 128 VGPRs)
constexpr int kPfW = 30;     // raw feature words per stream and frame: Lyf[22], f34[7], silence
constexpr int kFeatItems = kGS * (kBands + 7 + kCeps);

struct Job {
  int m = -1, tile = 0;
};

constexpr int kDzrFrags = 12 * 7;
constexpr int kFr = 24;  // register fragment slots (see the wave plan)  // denoise z|r: the largest matrix lives in LDS (84 KB)

struct Lds {
  alignas(16) half8 dzr[kDzrFrags][64];
  alignas(16) _Float16 op[kGS][kRowHalf];
  alignas(16) float sv[kGS][28], sn[kGS][52], sd[kGS][100];  // f32 GRU states (row pitch: distinct bank groups)
  alignas(16) float zv[kGS][28], zn[kGS][52], zd[kGS][100];  // update gates z of the frame
  alignas(16) float gout[kGS][24];
  alignas(16) float bias[kBiasRows];
  float tt[204];
  float ceps[kGS][kCeps * kBands];
  float dist[kGS][kCeps * kCeps];
  float lastg[kGS][kBands];
  float pf[kGS][kPfW];
  int act[8][kGS];
  int memid[kGS], nfs[kGS];
  long long fbase[kGS];
};

__device__ __forceinline__ void job_init(Job &J, int m, int tile) {
  J.m = m;
  J.tile = tile;
}

template <int F0, int NK>
__device__ __forceinline__ void load_frags(half8 (&fr)[kFr], const half8 *__restrict__ img, const Job &J, int lane) {
  if (J.m < 0) return;
  int nk = 0, base = 0;
#pragma unroll
  for (int m = 0; m < rnnimg::kMats; m++)
    if (m == J.m) {
      nk = nkb(m);
      base = frag_base(m);
    }
  const half8 *src = img + (size_t)(base + J.tile * nk) * 64 + lane;
#pragma unroll
  for (int kb = 0; kb < NK; kb++)
    if (kb < nk) fr[F0 + kb] = src[kb * 64];
}

// acc = bias + sum over matrix M's K blocks of A . B (C-in and C-out of one
// chain); M is known at every call site, so this lane's operand chunk of
// block kb is a select over the four lane groups of compile-time offsets
template <int M>
__device__ __forceinline__ half8 b_operand(const Lds &L, int lane, int kb, int fslot) {
  const int s = lane & 15, g = lane >> 4;
  const char *row = reinterpret_cast<const char *>(L.op[s]);
  const int c0 = op_chunk(M, 4 * kb), c1 = op_chunk(M, 4 * kb + 1), c2 = op_chunk(M, 4 * kb + 2),
            c3 = op_chunk(M, 4 * kb + 3);
  const int c = g == 0 ? c0 : g == 1 ? c1 : g == 2 ? c2 : c3;
  return *reinterpret_cast<const half8 *>(row + (c & 0xff) * 16 + ((c & 0x100) ? fslot * 6 * 16 : 0));
}

// acc = bias + sum over matrix M's K blocks of A . B (C-in and C-out of one
// chain); M is known at every call site, so this lane's operand chunk of
// block kb is a select over the four lane groups of compile-time offsets.
// A from registers fr[F0 + kb] (F0 >= 0) or from LDS (denoise z|r, F0 < 0).
template <int F0, int M>
__device__ __forceinline__ f4 mma_job(const half8 (&fr)[kFr], int tile, const Lds &L, int lane, int fslot) {
  constexpr int NK = nkb(M);
  f4 acc = *reinterpret_cast<const f4 *>(&L.bias[bias_base(M) + tile * 16 + 4 * (lane >> 4)]);
#pragma unroll
  for (int kb = 0; kb < NK; kb++) {
    const half8 b = b_operand<M>(L, lane, kb, fslot);
    half8 w;
    if constexpr (F0 >= 0)
      w = fr[F0 + kb];
    else
      w = L.dzr[tile * NK + kb][lane];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w, b, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ void put_h4(_Float16 *dst, float a, float b, float c, float d) {
  half4 h;
  h[0] = (_Float16)a;
  h[1] = (_Float16)b;
  h[2] = (_Float16)c;
  h[3] = (_Float16)d;
  *reinterpret_cast<half4 *>(dst) = h;
}

// z|r tile epilogue of a GRU with N neurons: z -> Z, r * state -> operand segment rs
template <int N, int PZ, int PS>
__device__ __forceinline__ void epi_zr(Lds &L, const f4 &acc, int tile, int lane, float (*Z)[PZ], float (*S)[PS],
                                       int rs_seg) {
  const int s = lane & 15, r0 = tile * 16 + 4 * (lane >> 4);
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = sigmoid(L.tt, kWs * acc[i]);
  if (r0 < N) {
    *reinterpret_cast<f4 *>(&Z[s][r0]) = f4{v[0], v[1], v[2], v[3]};
  } else {
    const int j = r0 - N;
    const f4 st = *reinterpret_cast<const f4 *>(&S[s][j]);
    put_h4(&L.op[s][kSegBase[rs_seg] * 8 + j], v[0] * st[0], v[1] * st[1], v[2] * st[2], v[3] * st[3]);
  }
}

// candidate tile epilogue: s' = z s + (1 - z) act(sum) for active streams
template <int N, int PZ, int PS>
__device__ __forceinline__ void epi_h(Lds &L, const f4 &acc, int tile, int lane, int act, float (*Z)[PZ],
                                      float (*S)[PS], int st_seg, bool on) {
  const int s = lane & 15, r0 = tile * 16 + 4 * (lane >> 4);
  if (r0 >= N || !on) return;
  const f4 z = *reinterpret_cast<const f4 *>(&Z[s][r0]);
  const f4 st = *reinterpret_cast<const f4 *>(&S[s][r0]);
  float n[4];
#pragma unroll
  for (int i = 0; i < 4; i++) n[i] = z[i] * st[i] + (1 - z[i]) * activate(L.tt, act, kWs * acc[i]);
  *reinterpret_cast<f4 *>(&S[s][r0]) = f4{n[0], n[1], n[2], n[3]};
  put_h4(&L.op[s][kSegBase[st_seg] * 8 + r0], n[0], n[1], n[2], n[3]);
}

}  // namespace

__global__ void __launch_bounds__(kGNT) k_gru16(StagedArgs a) {
  constexpr int S = kGS;
  __shared__ Lds L;
  const int tid = threadIdx.x, lane = tid & 63, W = tid >> 6;
  const int sb = blockIdx.x * S;
  const int *ra = a.rnn_act;
  // ---- jobs of this wave (register slots: A = fr[0..4] noise z|r, E = fr[5..9]
  // noise h, F = fr[10..16] denoise h, B = fr[17..19] dense / den_out /
  // vad_out, C = fr[20..21] vad z|r, D = fr[22..23] vad h)
  Job JA, JE, JF, JB, JC, JD;
  if (W < 6) job_init(JA, 3, W);
  if (W >= 5) job_init(JE, 4, W - 5);
  if (W >= 2) job_init(JF, 6, W - 2);
  if (W < 2) job_init(JB, 0, W);
  else if (W < 4) job_init(JB, 7, W - 2);
  else if (W == 6) job_init(JB, 8, 0);
  if (W >= 4 && W < 7) job_init(JC, 1, W - 4);
  if (W == 4 || W == 5) job_init(JD, 2, W - 4);
  half8 fr[kFr];
  {
    const half8 *img = reinterpret_cast<const half8 *>(a.gru16_frags);
    load_frags<0, 5>(fr, img, JA, lane);
    load_frags<5, 5>(fr, img, JE, lane);
    load_frags<10, 7>(fr, img, JF, lane);
    load_frags<17, 3>(fr, img, JB, lane);
    load_frags<20, 2>(fr, img, JC, lane);
    load_frags<22, 2>(fr, img, JD, lane);
    const half8 *dz = img + (size_t)frag_base(5) * 64;
    for (int i = tid; i < kDzrFrags * 64; i += kGNT) (&L.dzr[0][0])[i] = dz[i];
  }
  // ---- LDS: operand rows, states, tables
  for (int i = tid; i < S * kRowHalf; i += kGNT) (&L.op[0][0])[i] = (_Float16)0;
  for (int i = tid; i < kBiasRows; i += kGNT) L.bias[i] = a.gru16_bias[i];
  for (int i = tid; i < 201; i += kGNT) L.tt[i] = a.plan->tansig[i];
  for (int idx = tid; idx < S * kCeps * kBands; idx += kGNT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    L.ceps[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += kGNT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    L.dist[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kBands; idx += kGNT) {
    const int s = idx / kBands, i = idx - s * kBands;
    L.lastg[s][i] = (sb + s < a.n_streams) ? a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] : 0.0f;
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
  for (int idx = tid; idx < S * 96; idx += kGNT) {
    const int s = idx / 96, i = idx - s * 96;
    const bool ok = sb + s < a.n_streams;
    const float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) {
      L.sv[s][i] = ok ? stp[st::kVadGru + i] : 0.0f;
      L.op[s][kSegBase[kSv] * 8 + i] = (_Float16)L.sv[s][i];
    }
    if (i < 48) {
      L.sn[s][i] = ok ? stp[st::kNoiseGru + i] : 0.0f;
      L.op[s][kSegBase[kSn] * 8 + i] = (_Float16)L.sn[s][i];
    }
    L.sd[s][i] = ok ? stp[st::kDenGru + i] : 0.0f;
    L.op[s][kSegBase[kSd] * 8 + i] = (_Float16)L.sd[s][i];
  }
  int maxnf = 0;
#pragma unroll
  for (int s = 0; s < S; s++) maxnf = max(maxnf, L.nfs[s]);
  // raw feature lane (s, i): i < 22 Lyf, 22..28 f34, 29 silence (as 1.0 / 0.0)
  const int pfs = tid / kPfW, pfi = tid - pfs * kPfW;
  const bool pf_lane = tid < S * kPfW;
  auto fetch = [&](int v) -> float {
    if (!pf_lane || v >= L.nfs[pfs]) return 1.0f;  // past the end: treated as silent (inactive)
    const long long f = L.fbase[pfs] + v;
    if (pfi < kBands) return a.Lyf[f * kBands + pfi];
    if (pfi < kBands + 7) return a.f34[f * 8 + (pfi - kBands)];
    return a.silence[f] ? 1.0f : 0.0f;
  };
  // features of frame f from L.pf (k_rnn3's F-C: cepstral memory, deltas,
  // 34..40, the new distance row) into feature slot f & 1; item (s, i)
  auto feat_c = [&](int f, int idx) {
    const int s = idx / (kBands + 7 + kCeps), i = idx - s * (kBands + 7 + kCeps);
    const bool valid = f < L.nfs[s];
    const bool on = valid && L.pf[s][kPfW - 1] == 0.0f;
    if (i == 0) {
      L.act[f & 7][s] = on;
      if (valid && !on) a.vadf[L.fbase[s] + f] = 0;  // silent: X passes through, state untouched
    }
    if (!on) return;
    _Float16 *feat = &L.op[s][(f & 1) * 6 * 8];
    const int mi = L.memid[s];
    const float *c0 = L.pf[s];
    if (i < kBands) {
      L.ceps[s][mi * kBands + i] = c0[i];
      if (i < 6) {
        const float *c1 = L.ceps[s] + ((mi < 1) ? kCeps + mi - 1 : mi - 1) * kBands;
        const float *c2 = L.ceps[s] + ((mi < 2) ? kCeps + mi - 2 : mi - 2) * kBands;
        feat[i] = (_Float16)(c0[i] + c1[i] + c2[i]);
        feat[kBands + i] = (_Float16)(c0[i] - c2[i]);
        feat[kBands + 6 + i] = (_Float16)(c0[i] - 2 * c1[i] + c2[i]);
      } else {
        feat[i] = (_Float16)c0[i];
      }
    } else if (i < kBands + 7) {
      feat[34 + i - kBands] = (_Float16)c0[i];
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
  // spectral variability of frame f (feature 41): lane (s, i) = (tid >> 3,
  // tid & 7) takes row i's minimum distance, lane i == 0 adds the 8 minima in
  // row order (the C loop's sum) and advances memid; 128 lanes (w0, w1)
  auto feat_d = [&](int f) {
    const int s = tid >> 3, i = tid & 7;
    float mindist = 1e15f;
#pragma unroll
    for (int j = 0; j < kCeps; j++)
      if (j != i) mindist = (mindist < L.dist[s][i * kCeps + j]) ? mindist : L.dist[s][i * kCeps + j];
    float m[kCeps];
#pragma unroll
    for (int k = 0; k < kCeps; k++) m[k] = __shfl(mindist, (lane & ~7) + k);
    if (i != 0 || !L.act[f & 7][s]) return;
    float sv = 0;
#pragma unroll
    for (int k = 0; k < kCeps; k++) sv += m[k];
    L.op[s][(f & 1) * 6 * 8 + 41] = (_Float16)(float)(sv / kCeps - 2.1);
    int mid = L.memid[s] + 1;
    if (mid == kCeps) mid = 0;
    L.memid[s] = mid;
  };
  // prologue: features of frame 0, raw features of frame 1 staged
  if (pf_lane) L.pf[pfs][pfi] = fetch(0);
  __syncthreads();
  for (int idx = tid; idx < kFeatItems; idx += kGNT) feat_c(0, idx);
  __syncthreads();
  if (tid < S * kCeps && 0 < maxnf) feat_d(0);
  const float pf1 = fetch(1);
  __syncthreads();
  if (pf_lane) L.pf[pfs][pfi] = pf1;
  __syncthreads();
  const int col = lane & 15;
  STAMP_INIT();
  for (int t = 0; t <= maxnf; t++) {
    const int fs = t & 1;
    const bool fr_t = t < maxnf;
    const bool on_t = fr_t && L.act[t & 7][col];
    // ---- P0: dense(t) [w0, w1], denoise_output(t-1) [w2, w3]
    if (W < 2) {
      if (fr_t) {
        const f4 acc = mma_job<17, 0>(fr, JB.tile, L, lane, fs);
        const int r0 = JB.tile * 16 + 4 * (lane >> 4);
        if (r0 < 24) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; i++) v[i] = activate(L.tt, ra[0], kWs * acc[i]);
          put_h4(&L.op[col][kSegBase[kDense] * 8 + r0], v[0], v[1], v[2], v[3]);
        }
      }
    } else if (W < 4) {
      if (t >= 1) {
        const f4 acc = mma_job<17, 7>(fr, JB.tile, L, lane, fs);
        const int r0 = JB.tile * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (r0 + i < kBands) L.gout[col][r0 + i] = activate(L.tt, ra[7], kWs * acc[i]);
      }
    }
    __syncthreads();
    RSTAMP(0);
    // ---- P1: vad z|r(t) [w4..6], features(t+1) [w0..3], gains(t-1) [w7]
    if (W >= 4 && W < 7) {
      if (fr_t) epi_zr<24>(L, mma_job<20, 1>(fr, JC.tile, L, lane, fs), JC.tile, lane, L.zv, L.sv, kRsv);
    } else if (W < 4) {
      // distance rows (the 22-term sums) one per lane on w0, w1; the rest on w2, w3
      if (t + 1 < maxnf) {
        constexpr int kIt = kBands + 7 + kCeps, kLight = kBands + 7;
        if (tid < S * kCeps)
          feat_c(t + 1, (tid >> 3) * kIt + kLight + (tid & 7));
        else
          for (int k = tid - S * kCeps; k < S * kLight; k += 4 * 64 - S * kCeps)
            feat_c(t + 1, (k / kLight) * kIt + k % kLight);
      }
    } else if (t >= 1) {  // gain smoothing g = max(g, .6*lastg) (denoise.c), frame t-1
      const int f1 = t - 1;
      for (int idx = lane; idx < S * kBands; idx += 64) {
        const int s = idx / kBands, i = idx - s * kBands;
        if (!L.act[f1 & 7][s]) continue;
        const long long f = L.fbase[s] + f1;
        const float gi = L.gout[s][i];
        const float al = .6f * L.lastg[s][i];
        const float gsm = (gi > al) ? gi : al;
        L.lastg[s][i] = gsm;
        a.gr[f * kBands + i] = gi;
        a.gs[f * kBands + i] = gsm;
      }
    }
    __syncthreads();
    RSTAMP(1);
    if (!fr_t) break;
    // ---- P2: vad h(t) [w4, w5], spectral variability(t+1) [w0]
    if (W == 4 || W == 5)
      epi_h<24>(L, mma_job<22, 2>(fr, JD.tile, L, lane, fs), JD.tile, lane, ra[2], L.zv, L.sv, kSv, on_t);
    else if (W < 2 && t + 1 < maxnf)
      feat_d(t + 1);
    __syncthreads();
    RSTAMP(2);
    // ---- P3: noise z|r(t) [w0..5], vad_output(t) [w6]; raw features of t+2 requested
    const float pf_next = fetch(t + 2);
    if (W < 6) {
      epi_zr<48>(L, mma_job<0, 3>(fr, JA.tile, L, lane, fs), JA.tile, lane, L.zn, L.sn, kRsn);
    } else if (W == 6) {
      const f4 acc = mma_job<17, 8>(fr, JB.tile, L, lane, fs);
      if (lane < 16 && on_t) a.vadf[L.fbase[col] + t] = activate(L.tt, ra[8], kWs * acc[0]);
    }
    __syncthreads();
    RSTAMP(3);
    // ---- P4: noise h(t) [w5..7]
    if (W >= 5) epi_h<48>(L, mma_job<5, 4>(fr, JE.tile, L, lane, fs), JE.tile, lane, ra[4], L.zn, L.sn, kSn, on_t);
    __syncthreads();
    RSTAMP(4);
    // ---- P5: denoise z|r(t), A from LDS: tile w [w0..7] and w + 8 [w0..3]
    epi_zr<96>(L, mma_job<-1, 5>(fr, W, L, lane, fs), W, lane, L.zd, L.sd, kRsd);
    if (W < 4) epi_zr<96>(L, mma_job<-1, 5>(fr, W + 8, L, lane, fs), W + 8, lane, L.zd, L.sd, kRsd);
    __syncthreads();
    RSTAMP(5);
    // ---- P6: denoise h(t) [w2..7]; raw features of t+2 staged
    if (W >= 2) epi_h<96>(L, mma_job<10, 6>(fr, JF.tile, L, lane, fs), JF.tile, lane, ra[6], L.zd, L.sd, kSd, on_t);
    if (pf_lane) L.pf[pfs][pfi] = pf_next;
    __syncthreads();
    RSTAMP(6);
  }
  STAMP_FLUSH(48, 7);
  // ---- state write-back (streams that ran at least one frame)
  for (int idx = tid; idx < S * kCeps * kBands; idx += kGNT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    if (sb + s < a.n_streams && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] = L.ceps[s][i];
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += kGNT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    if (sb + s < a.n_streams && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] = L.dist[s][i];
  }
  for (int idx = tid; idx < S * kBands; idx += kGNT) {
    const int s = idx / kBands, i = idx - s * kBands;
    if (sb + s < a.n_streams && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] = L.lastg[s][i];
  }
  for (int idx = tid; idx < S * 96; idx += kGNT) {
    const int s = idx / 96, i = idx - s * 96;
    if (sb + s >= a.n_streams || L.nfs[s] <= 0) continue;
    float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) stp[st::kVadGru + i] = L.sv[s][i];
    if (i < 48) stp[st::kNoiseGru + i] = L.sn[s][i];
    stp[st::kDenGru + i] = L.sd[s][i];
  }
  if (tid < S && sb + tid < a.n_streams && L.nfs[tid] > 0)
    reinterpret_cast<int *>(a.state)[(size_t)(sb + tid) * st::kWords + st::kMemId] = L.memid[tid];
}

hipError_t launch_gru16(const StagedArgs &a, hipStream_t stream) {
  hipLaunchKernelGGL(k_gru16, dim3((a.n_streams + kGS - 1) / kGS), dim3(kGNT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace fvad
