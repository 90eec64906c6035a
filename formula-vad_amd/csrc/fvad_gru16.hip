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
// whole kernel (kFr = 20 slots of 8 f16); the denoise z|r matrix (84 of the
// 192 fragments) sits in LDS.  A tile costs per frame one ds_read_b128 of B
// (and of A from LDS) per K-block plus the MFMA chain.
//
// Schedule: a superstep pipeline over frames (details above k_gru16).  Layer
// L of frame t waits only for layer L - 1 of t and layer L of t - 1, so
// superstep u runs dense(u), vad(u - 1), noise(u - 2), denoise(u - 3) and the
// outputs of u - 2 / u - 4 side by side in two phases -- A: every z|r gate,
// B: every candidate -- two barriers per frame; the features of u + 1 and the
// gain smoothing of u - 4 fill the waves a phase leaves idle.  Operand
// segments read by layers of different frames in one phase are versioned by
// frame (OpSeg).
//
// k_fused16 (engine mode FVAD_MODE_FP16_FUSED, configs[4]'s "fused FFT ->
// feature -> GRU kernel") is the same body with k_pspecw's per-frame work on
// 8 more waves; see above gru16_body.  Its outputs equal k_gru16's bit for bit.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fvad_device.h"
#include "fvad_internal.h"
#include "fvad_staged.h"
#include "fvad_staged_dev.h"
#include "fvad_wavedev.h"

namespace fvad {
namespace g16 {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

// operand row of one stream, in 8-element chunks.  The layers run a frame
// apart (see the superstep plan), so the segments that layers of different
// frames read are versioned by frame: features (5 versions, f % 5), dense
// output (3, f % 3), vad state (3, f % 3), noise state (2, f & 1).
enum OpSeg { kFeat = 0, kDense, kSv, kRsv, kSn, kRsn, kSd, kRsd, kNSeg };
constexpr int kSegLen[kNSeg] = {6, 3, 3, 3, 6, 6, 12, 12};   // chunks of one version
constexpr int kSegVer[kNSeg] = {5, 3, 3, 1, 2, 1, 1, 1};      // versions
constexpr int seg_base(int g) {
  int o = 0;
  for (int i = 0; i < g; i++) o += kSegLen[i] * kSegVer[i];
  return o;
}
constexpr int kSegBase[kNSeg] = {seg_base(0), seg_base(1), seg_base(2), seg_base(3),
                                 seg_base(4), seg_base(5), seg_base(6), seg_base(7)};
constexpr int kZeroChunk = seg_base(kNSeg);
constexpr int kRowChunks = kZeroChunk + 2;  // odd: rows of 16 streams fall on distinct 4-bank groups
static_assert(kRowChunks % 2 == 1, "operand row pitch");
constexpr int kRowHalf = kRowChunks * 8;
// versioned segment tags (op_chunk bits 8..10): 1 feat, 2 dense, 3 vad state, 4 noise state
constexpr int seg_tag(int seg) { return seg == kFeat ? 1 : seg == kDense ? 2 : seg == kSv ? 3 : seg == kSn ? 4 : 0; }
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

// chunk q of matrix m -> operand chunk of version 0, its versioned-segment tag in bits 8..10
constexpr int op_chunk(int m, int q) {
  int c0 = 0;
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const int n = rnnimg::pad8(rnnimg::kSegs[m][g]) / 8;
    if (q < c0 + n) {
      const int seg = kMatSeg[m][g];
      return kSegBase[seg] + (q - c0) + (seg_tag(seg) << 8);
    }
    c0 += n;
  }
  return kZeroChunk;
}

// versions of the operand segments matrix M reads for its frame f:
// the vad z|r gates read the vad state of frame f - 1, the noise z|r gates the
// noise state of f - 1; everything else reads frame f's values
struct Ver {
  int f, d, v, n;  // byte offsets of the feature, dense, vad-state and noise-state versions
  __device__ __forceinline__ int of(int tag) const { return tag == 1 ? f : tag == 2 ? d : tag == 3 ? v : tag == 4 ? n : 0; }
};
template <int M>
__device__ __forceinline__ Ver versions(int f) {
  Ver v;
  const int fv = (M == 1) ? f - 1 : f;  // vad state version
  const int fn = (M == 3) ? f - 1 : f;  // noise state version
  v.f = ((f + 5) % 5) * kSegLen[kFeat] * 16;
  v.d = ((f + 3) % 3) * kSegLen[kDense] * 16;
  v.v = ((fv + 3) % 3) * kSegLen[kSv] * 16;
  v.n = ((fn + 2) & 1) * kSegLen[kSn] * 16;
  return v;
}
// chunk offset (in halfs) of version `ver` of segment seg
__device__ __forceinline__ int seg_half(int seg, int ver) { return (kSegBase[seg] + ver * kSegLen[seg]) * 8; }

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

constexpr int kGS = 16;      // stream columns per workgroup (MFMA N)
constexpr int kGNT = 512;    // 8 waves, 2 per SIMD (fragments + operands need > 128 VGPRs)
constexpr int kPfW = 30;     // raw feature words per stream and frame: Lyf[22], f34[7], silence
constexpr int kFeatItems = kGS * (kBands + 7 + kCeps);

constexpr int kDzrFrags = 12 * 7;  // denoise z|r: the largest matrix lives in LDS (84 KB)
constexpr int kFr = 20;            // register fragment slots (see the wave plan)

struct LdsCore {
  alignas(16) _Float16 op[kGS][kRowHalf];
  alignas(16) float sv[kGS][28], sn[kGS][52], sd[kGS][100];  // f32 GRU states (row pitch: distinct bank groups)
  alignas(16) float zv[kGS][28], zn[kGS][52], zd[kGS][100];  // update gates z of the frame
  alignas(16) float gout[kGS][24];
  alignas(16) float bias[kBiasRows];
  float tt[204];
  float ceps[kGS][kCeps * kBands];
  float dist[kGS][kCeps * kCeps];
  float lastg[kGS][kBands];
  float pf[2][kGS][kPfW];  // raw features of frame f in pf[f & 1]
  int act[8][kGS];
  int memid[kGS], nfs[kGS];
  long long fbase[kGS];
};
// k_gru16: the denoise z|r fragments in LDS
struct LdsSplit : LdsCore {
  alignas(16) half8 dzr[kDzrFrags][64];
};
// k_fused16: the pitch-spectrum waves' exchange regions (one per wave) and
// FFT tables take that LDS; every A fragment is read from L2 instead
constexpr int kFW = 8;             // k_fused16: pitch-spectrum waves (one per stream), after the 8 GRU waves
constexpr int kFNT = kGNT + 64 * kFW;
struct LdsFused : LdsCore {
  alignas(16) float2 Rg[kFW][wfft::kSlots];
  WaveTabs tb;
};

// A fragments of tile `tile` of matrix M into fr[F0 .. F0 + nkb(M))
template <int F0, int M>
__device__ __forceinline__ void load_frags(half8 (&fr)[kFr], const half8 *__restrict__ img, int tile, int lane) {
  constexpr int NK = nkb(M);
  static_assert(F0 + NK <= kFr, "fragment slots");
  const half8 *src = img + (size_t)(frag_base(M) + tile * NK) * 64 + lane;
#pragma unroll
  for (int kb = 0; kb < NK; kb++) fr[F0 + kb] = src[kb * 64];
}

// this lane's B chunk of K block kb of matrix M (frame versions in V): a
// select over the four lane groups of compile-time chunks, plus the version
// offset of the segment the chunk belongs to
template <int M, class LT>
__device__ __forceinline__ half8 b_operand(const LT &L, int lane, int kb, const Ver &V) {
  const int s = lane & 15, g = lane >> 4;
  const char *row = reinterpret_cast<const char *>(L.op[s]);
  const int c0 = op_chunk(M, 4 * kb), c1 = op_chunk(M, 4 * kb + 1), c2 = op_chunk(M, 4 * kb + 2),
            c3 = op_chunk(M, 4 * kb + 3);
  const int c = g == 0 ? c0 : g == 1 ? c1 : g == 2 ? c2 : c3;
  return *reinterpret_cast<const half8 *>(row + (c & 0xff) * 16 + V.of(c >> 8));
}

// acc = bias + sum over matrix M's K blocks of A . B for frame f (one MFMA
// chain).  k_gru16: A from registers fr[F0 + kb] (F0 >= 0) or, for the
// denoise z|r matrix (F0 < 0), from its LDS copy dz.  k_fused16 (LdsFused):
// every A fragment from the global image dz (L2), the registers are the FFT's.
template <int F0, int M, class LT>
__device__ __forceinline__ f4 mma_job(const half8 (&fr)[kFr], int tile, const LT &L, const half8 *__restrict__ dz,
                                      int lane, int f) {
  constexpr int NK = nkb(M);
  const Ver V = versions<M>(f);
  f4 acc = *reinterpret_cast<const f4 *>(&L.bias[bias_base(M) + tile * 16 + 4 * (lane >> 4)]);
#pragma unroll
  for (int kb = 0; kb < NK; kb++) {
    const half8 b = b_operand<M>(L, lane, kb, V);
    half8 w;
    if constexpr (std::is_same_v<LT, LdsFused>)
      w = dz[(frag_base(M) + tile * NK + kb) * 64 + lane];
    else if constexpr (F0 >= 0)
      w = fr[F0 + kb];
    else
      w = dz[(tile * NK + kb) * 64 + lane];
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
template <int N, int PZ, int PS, class LT>
__device__ __forceinline__ void epi_zr(LT &L, const f4 &acc, int tile, int lane, float (*Z)[PZ], float (*S)[PS],
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

// candidate tile epilogue: s' = z s + (1 - z) act(sum) for active streams, the
// new state into operand half offset `dst` (the frame's version); an inactive
// stream keeps its state and still fills the frame's version with it
template <int N, int PZ, int PS, class LT>
__device__ __forceinline__ void epi_h(LT &L, const f4 &acc, int tile, int lane, int act, float (*Z)[PZ],
                                      float (*S)[PS], int dst, bool on) {
  const int s = lane & 15, r0 = tile * 16 + 4 * (lane >> 4);
  if (r0 >= N) return;
  const f4 st = *reinterpret_cast<const f4 *>(&S[s][r0]);
  if (!on) {
    put_h4(&L.op[s][dst + r0], st[0], st[1], st[2], st[3]);
    return;
  }
  const f4 z = *reinterpret_cast<const f4 *>(&Z[s][r0]);
  float n[4];
#pragma unroll
  for (int i = 0; i < 4; i++) n[i] = z[i] * st[i] + (1 - z[i]) * activate(L.tt, act, kWs * acc[i]);
  *reinterpret_cast<f4 *>(&S[s][r0]) = f4{n[0], n[1], n[2], n[3]};
  put_h4(&L.op[s][dst + r0], n[0], n[1], n[2], n[3]);
}

}  // namespace

// The layers of one frame form a chain (dense -> vad -> noise -> denoise ->
// denoise_output), but layer L of frame t only waits for layer L - 1 of t and
// layer L of t - 1.  So superstep u runs dense(u), vad(u - 1), noise(u - 2),
// denoise(u - 3), outputs(u - 2 / u - 4) side by side in two phases (all z|r
// gates, then all candidates): two barriers per frame instead of seven.
// Operands that layers of different frames read at once are versioned
// (OpSeg).  Wave plan (waves w and w + 4 share a SIMD; balanced by per-wave
// stamps, tools/stamps.py fp16):
//   A  every wave denoise z|r(u-3) tile w (w0..3 also w+8, A from LDS);
//      w0,1 dense(u) t w + the distance rows of the features of u+1 |
//      w2,3 vad z|r(u-1) t w-2 | w4 vad z|r t2, noise z|r(u-2) t0, vad_out(u-2) |
//      w5,6 noise z|r t 2w-9, 2w-8 | w5 den_out(u-4) t1 | w7 noise z|r t5,
//      den_out t0; w2,3,6,7 the rest of the features of u+1
//   B  w0..5 denoise h(u-3) t w; w4 noise h(u-2) t1; w6 noise h t0, vad h(u-1)
//      t1; w7 noise h t2, vad h t0; w0,1 spectral variability(u+1); w2,3,5
//      gains(u-4)
// Register fragments (kFr = 20 slots of 8 f16): w0,1 dense 0-1, denoise h 2-8;
// w2,3 vad z|r 0-1, denoise h 2-8; w4 vad z|r 0-1, noise z|r 2-6, vad_out 7,
// denoise h 8-14, noise h 15-19; w5 noise z|r 0-4, 5-9, denoise h 10-16,
// den_out 17-19; w6 noise z|r 0-4, 5-9, noise h 10-14, vad h 15-16;
// w7 noise z|r 0-4, den_out 5-7, noise h 11-15, vad h 16-17.
// kSpw = the streams a workgroup owns (<= kGS; the MFMA columns past it stay
// inactive).  8 puts 256 workgroups on the 256 CUs at 2048 streams instead of
// 128: k_gru16 0.554 -> 0.530 ms (latency-bound supersteps, the same per
// workgroup).
//
// kFuse (k_fused16, BASELINE configs[4]'s "fused FFT -> feature -> GRU
// kernel"): the pitch-spectrum FFT and its features 34..40 (k_pspecw's
// per-frame work, fvad_wavedev.h) run inside the recurrence on 8 more waves,
// wave 8 + j on stream j: at superstep u it transforms frame u + 2 in phase A
// (pspec_transform) and finishes its features in phase B (pspec_features),
// handing them to the GRU waves in LDS (pf) instead of through HBM; P, Ep and
// Exp still go to HBM for k_synthw.  16 waves = 4 per SIMD leave 128 VGPRs a
// wave, so the GRU waves hold no A fragments (every fragment is read from L2
// each frame step: 192 KB per workgroup, the same 192 KB for every workgroup
// of an XCD), and the exchange regions take the LDS of the denoise z|r copy.
template <int kSpw, bool kFuse>
__device__ __forceinline__ void gru16_body(const StagedArgs &a) {
  static_assert(kSpw > 0 && kSpw <= kGS, "streams per k_gru16 workgroup");
  static_assert(!kFuse || kSpw == kFW, "k_fused16: one pitch-spectrum wave per stream");
  constexpr int S = kGS;
  constexpr int NT = kFuse ? kFNT : kGNT;  // threads of the workgroup
  using LT = std::conditional_t<kFuse, LdsFused, LdsSplit>;
  __shared__ LT L;
  // (tid / lane / col: renewed opaquely every k_fused16 step, see the loop)
  int tid = threadIdx.x, lane = tid & 63;
  // the wave index as a scalar: the wave plan's branches are scalar and the
  // tile offsets derived from it stay out of the VGPRs (k_fused16's 128
  // would not hold them; k_gru16 0.532 -> 0.514 ms, interleaved A/B)
  const int W = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sb = blockIdx.x * kSpw;
  auto sok = [&](int s) { return s < kSpw && sb + s < a.n_streams; };
  const int *ra = a.rnn_act;
  half8 fr[kFr];
  {
    const half8 *img = reinterpret_cast<const half8 *>(a.gru16_frags);
    if constexpr (!kFuse) {  // (k_fused16 reads every fragment from L2)
      if (W < 2) {
        load_frags<0, 0>(fr, img, W, lane);
        load_frags<2, 6>(fr, img, W, lane);
      } else if (W < 4) {
        load_frags<0, 1>(fr, img, W - 2, lane);
        load_frags<2, 6>(fr, img, W, lane);
      } else if (W == 4) {
        load_frags<0, 1>(fr, img, 2, lane);
        load_frags<2, 3>(fr, img, 0, lane);
        load_frags<7, 8>(fr, img, 0, lane);
        load_frags<8, 6>(fr, img, 4, lane);
        load_frags<15, 4>(fr, img, 1, lane);
      } else if (W == 5) {
        load_frags<0, 3>(fr, img, 1, lane);
        load_frags<5, 3>(fr, img, 2, lane);
        load_frags<10, 6>(fr, img, 5, lane);
        load_frags<17, 7>(fr, img, 1, lane);
      } else if (W == 6) {
        load_frags<0, 3>(fr, img, 3, lane);
        load_frags<5, 3>(fr, img, 4, lane);
        load_frags<10, 4>(fr, img, 0, lane);
        load_frags<15, 2>(fr, img, 1, lane);
      } else {
        load_frags<0, 3>(fr, img, 5, lane);
        load_frags<5, 7>(fr, img, 0, lane);
        load_frags<11, 4>(fr, img, 2, lane);
        load_frags<16, 2>(fr, img, 0, lane);
      }
    }
    if constexpr (!kFuse) {
      const half8 *dzg = img + (size_t)frag_base(5) * 64;
      for (int i = tid; i < kDzrFrags * 64; i += kGNT) (&L.dzr[0][0])[i] = dzg[i];
    } else {
      wave_tabs_load(L.tb, a.plan, tid, NT);
    }
  }
  const half8 *__restrict__ dz;
  if constexpr (!kFuse)
    dz = &L.dzr[0][0];
  else
    dz = reinterpret_cast<const half8 *>(a.gru16_frags);
  // ---- LDS: operand rows, states, tables
  for (int i = tid; i < S * kRowHalf; i += NT) (&L.op[0][0])[i] = (_Float16)0;
  for (int i = tid; i < kBiasRows; i += NT) L.bias[i] = a.gru16_bias[i];
  for (int i = tid; i < 201; i += NT) L.tt[i] = a.plan->tansig[i];
  for (int idx = tid; idx < S * kCeps * kBands; idx += NT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    L.ceps[s][i] = sok(s) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += NT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    L.dist[s][i] = sok(s) ? a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] : 0.0f;
  }
  for (int idx = tid; idx < S * kBands; idx += NT) {
    const int s = idx / kBands, i = idx - s * kBands;
    L.lastg[s][i] = sok(s) ? a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] : 0.0f;
  }
  if (tid < 8 * S) L.act[tid / S][tid % S] = 0;
  if (tid < S) {
    const int s = sb + tid;
    const bool ok = sok(tid);
    L.memid[tid] = ok ? reinterpret_cast<const int *>(a.state)[(size_t)s * st::kWords + st::kMemId] : 0;
    L.nfs[tid] = ok ? ticks_of(a, s) * a.n_channels : 0;
    L.fbase[tid] = (long long)s * a.V;
  }
  __syncthreads();
  // states before frame 0 = the versions of frame -1 (vad 2, noise 1)
  for (int idx = tid; idx < S * 96; idx += NT) {
    const int s = idx / 96, i = idx - s * 96;
    const bool ok = sok(s);
    const float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) {
      L.sv[s][i] = ok ? stp[st::kVadGru + i] : 0.0f;
      L.op[s][seg_half(kSv, 2) + i] = (_Float16)L.sv[s][i];
    }
    if (i < 48) {
      L.sn[s][i] = ok ? stp[st::kNoiseGru + i] : 0.0f;
      L.op[s][seg_half(kSn, 1) + i] = (_Float16)L.sn[s][i];
    }
    L.sd[s][i] = ok ? stp[st::kDenGru + i] : 0.0f;
    L.op[s][seg_half(kSd, 0) + i] = (_Float16)L.sd[s][i];
  }
  int maxnf = 0;
#pragma unroll
  for (int s = 0; s < S; s++) maxnf = max(maxnf, L.nfs[s]);
  // raw feature lane (s, i): i < 22 Lyf, 22..28 f34, 29 silence (the flag's
  // bits, nonzero = silent: no wait for the load where it is issued)
  // (k_fused16: the f34 words come from pspec below, not from HBM)
  const int pfs = tid / kPfW, pfi = tid - pfs * kPfW;
  const bool pf_lane = tid < S * kPfW && !(kFuse && pfi >= kBands && pfi < kBands + 7);
  auto fetch = [&](int v) -> float {
    if (!pf_lane || v >= L.nfs[pfs]) return 1.0f;  // past the end: treated as silent (inactive)
    const long long f = L.fbase[pfs] + v;
    if (pfi < kBands) return a.Lyf[f * kBands + pfi];
    if (pfi < kBands + 7) return a.f34[f * 8 + (pfi - kBands)];
    return __int_as_float(a.silence[f]);
  };
  // features of frame f from L.pf (k_rnn3's F-C: cepstral memory, deltas,
  // 34..40, the new distance row) into feature version f % 5; item (s, i)
  auto feat_c = [&](int f, int idx) {
    const int s = idx / (kBands + 7 + kCeps), i = idx - s * (kBands + 7 + kCeps);
    const bool valid = f < L.nfs[s];
    const bool on = valid && __float_as_int(L.pf[f & 1][s][kPfW - 1]) == 0;
    if (i == 0) {
      L.act[f & 7][s] = on;
      if (valid && !on) a.vadf[L.fbase[s] + f] = 0;  // silent: X passes through, state untouched
    }
    if (!on) return;
    _Float16 *feat = &L.op[s][seg_half(g16::kFeat, f % 5)];
    const int mi = L.memid[s];
    const float *c0 = L.pf[f & 1][s];
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
    L.op[s][seg_half(g16::kFeat, f % 5) + 41] = (_Float16)(float)(sv / kCeps - 2.1);
    int mid = L.memid[s] + 1;
    if (mid == kCeps) mid = 0;
    L.memid[s] = mid;
  };
  // k_fused16: waves kGNT / 64 + j are stream j's pitch-spectrum waves (their
  // loop is below the GRU's); pframe(v): stream j's frame v, or -1
  const bool fft_wave = kFuse && W >= kGNT / 64;
  const int fj = W - kGNT / 64;
  auto pframe = [&](int v) { return (kFuse && sok(fj) && v < L.nfs[fj]) ? (int)(L.fbase[fj] + v) : -1; };
  // prologue: features of frame 0, raw features of frame 1 staged
  if (pf_lane) L.pf[0][pfs][pfi] = fetch(0);
  if constexpr (kFuse) {
#ifndef FVAD_DIAG_NO_PSPEC  // (diagnostic build: k_fused16's GRU alone, wrong features)
    if (fft_wave) {
      wfft::Tw tw;
      wfft::load_tw(tw, reinterpret_cast<const float2 *>(a.plan->tw960), lane);
      for (int v = 0; v < 2; v++) {
        const int f = pframe(v);
        if (f < 0) continue;
        const float v34 = pspec_frame(a, f, a.pitch[f], L.tb, tw, L.Rg[fj], lane);
        if (lane < 7) L.pf[v & 1][fj][kBands + lane] = v34;
      }
    }
#endif
  }
  __syncthreads();
  for (int idx = tid; idx < kFeatItems; idx += NT) feat_c(0, idx);
  __syncthreads();
  if (tid < S * kCeps && 0 < maxnf) feat_d(0);
  const float pf1 = fetch(1);
  __syncthreads();
  if (pf_lane) L.pf[1][pfs][pfi] = pf1;
  __syncthreads();
  int col = lane & 15;
  auto live = [&](int f) { return f >= 0 && f < maxnf; };
  auto den_out = [&](const f4 &acc, int tile) {  // denoise_output tile -> the frame's gains
    const int r0 = tile * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (r0 + i < kBands) L.gout[col][r0 + i] = activate(L.tt, ra[7], kWs * acc[i]);
  };
  auto on_of = [&](int f) { return L.act[f & 7][col] != 0; };
  STAMP_INIT();
#ifdef FVAD_STAMPS
  // per-wave busy cycles of each phase (lane 0 of every wave): stamps[0..7] A, [8..15] B
  unsigned long long wacc[2] = {0, 0}, wt0 = 0;
#define WSTAMP_BEGIN() wt0 = __builtin_amdgcn_s_memtime()
#define WSTAMP_END(p) wacc[p] += __builtin_amdgcn_s_memtime() - wt0
#else
#define WSTAMP_BEGIN() \
  do {                 \
  } while (0)
#define WSTAMP_END(p) \
  do {                \
  } while (0)
#endif
  if (fft_wave) {
    // k_fused16's pitch-spectrum waves, in step with the GRU waves' barriers
    // (two per superstep): at superstep u the transform of frame u + 2 in
    // phase A, its features in phase B; a frame's pitch loads one superstep
    // ahead.  (Its window, X and Ex loaded a phase ahead as well measured
    // slower: 1.65 vs 1.39 ms.)
    if constexpr (kFuse) {
      int f2 = pframe(2), f3 = pframe(3);
      int pit2 = f2 >= 0 ? a.pitch[f2] : 0, pit3 = f3 >= 0 ? a.pitch[f3] : 0;
#ifdef FVAD_DIAG_NO_PSPEC
      f2 = f3 = -1;
#endif
      for (int u = 0; u < maxnf + 4; u++) {
        const int f = f2, pit = pit2;  // frame u + 2
        asm volatile("" : "+v"(lane));  // lane-derived table addresses: per step, not held (as the GRU loop)
        WSTAMP_BEGIN();
        float exl = 0.0f;
        if (f >= 0) {
          PspecIn in;
          pspec_load(in, a, f, pit, lane);
          wfft::Tw tw;
          wfft::load_tw(tw, reinterpret_cast<const float2 *>(a.plan->tw960 + opaque0()), lane);
          pspec_transform(a, f, in, L.tb, tw, L.Rg[fj], lane);
          exl = in.exl;
        }
        f2 = f3;
        pit2 = pit3;
        f3 = pframe(u + 4);
#ifdef FVAD_DIAG_NO_PSPEC
        f3 = -1;
#endif
        pit3 = f3 >= 0 ? a.pitch[f3] : 0;
        WSTAMP_END(0);
        lds_sync();
        WSTAMP_BEGIN();
        if (f >= 0) {
          const float v34 = pspec_features(a, f, pit, L.tb, L.Rg[fj], lane, exl);
          if (lane < 7) L.pf[u & 1][fj][kBands + lane] = v34;
        }
        WSTAMP_END(1);
        lds_sync();
      }
    }
  } else {
  for (int u = 0; u < maxnf + 4; u++) {
    const int fV = u - 1, fN = u - 2, fD = u - 3, fO = u - 4;
    // k_fused16: the fragment loads stay in the step (hoisted out of the loop
    // they would be the resident fragments again, in more registers than exist)
    const half8 *__restrict__ dzs = kFuse ? dz + opaque0() : dz;
    // ... and so do the lane-derived LDS and HBM addresses: as loop invariants
    // they would all be held (or spilled) in the 128 VGPRs
    if constexpr (kFuse) {
      asm volatile("" : "+v"(tid));
      asm volatile("" : "+v"(lane));
      asm volatile("" : "+v"(col));
    }
    const float pf_next = fetch(u + 2);  // raw features of u + 2, staged at the end of phase B
    // ---- phase A: z|r gates of vad(u-1), noise(u-2), denoise(u-3); dense(u),
    // vad_out(u-2), den_out(u-4); features(u+1)
    WSTAMP_BEGIN();
    // waves 5..7 carry the longest phase-A chains (stamps): they issue first
    // (k_gru16 0.512 -> 0.505 ms interleaved; w5 and w7 only 0.512, phase B's
    // longest waves raised as well 0.514-0.523)
    if (W >= 5) __builtin_amdgcn_s_setprio(2);
    if (live(fD)) {
      epi_zr<96>(L, mma_job<-1, 5>(fr, W, L, dzs, lane, fD), W, lane, L.zd, L.sd, kRsd);
      if (W < 4) epi_zr<96>(L, mma_job<-1, 5>(fr, W + 8, L, dzs, lane, fD), W + 8, lane, L.zd, L.sd, kRsd);
    }
    if (W < 2) {
      if (u < maxnf) {
        const f4 acc = mma_job<0, 0>(fr, W, L, dzs, lane, u);
        const int r0 = W * 16 + 4 * (lane >> 4);
        if (r0 < 24) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; i++) v[i] = activate(L.tt, ra[0], kWs * acc[i]);
          put_h4(&L.op[col][seg_half(kDense, u % 3) + r0], v[0], v[1], v[2], v[3]);
        }
      }
    } else if (W < 4) {
      if (live(fV)) epi_zr<24>(L, mma_job<0, 1>(fr, W - 2, L, dzs, lane, fV), W - 2, lane, L.zv, L.sv, kRsv);
    } else if (W == 4) {
      if (live(fV)) epi_zr<24>(L, mma_job<0, 1>(fr, 2, L, dzs, lane, fV), 2, lane, L.zv, L.sv, kRsv);
      if (live(fN)) {
        epi_zr<48>(L, mma_job<2, 3>(fr, 0, L, dzs, lane, fN), 0, lane, L.zn, L.sn, kRsn);
        const f4 acc = mma_job<7, 8>(fr, 0, L, dzs, lane, fN);
        if (lane < 16 && on_of(fN)) a.vadf[L.fbase[col] + fN] = activate(L.tt, ra[8], kWs * acc[0]);
      }
    } else if (W < 7) {
      if (live(fN)) {
        epi_zr<48>(L, mma_job<0, 3>(fr, 2 * W - 9, L, dzs, lane, fN), 2 * W - 9, lane, L.zn, L.sn, kRsn);
        epi_zr<48>(L, mma_job<5, 3>(fr, 2 * W - 8, L, dzs, lane, fN), 2 * W - 8, lane, L.zn, L.sn, kRsn);
      }
      if (W == 5 && live(fO)) den_out(mma_job<17, 7>(fr, 1, L, dzs, lane, fO), 1);
    } else {
      if (live(fN)) epi_zr<48>(L, mma_job<0, 3>(fr, 5, L, dzs, lane, fN), 5, lane, L.zn, L.sn, kRsn);
      if (live(fO)) den_out(mma_job<5, 7>(fr, 0, L, dzs, lane, fO), 0);
    }
    if (u + 1 < maxnf) {
      // distance rows (the 22-term sums) one per lane on w0, w1; the rest on w2, w3, w6, w7
      constexpr int kIt = kBands + 7 + kCeps, kLight = kBands + 7;
      if (tid < S * kCeps)
        feat_c(u + 1, (tid >> 3) * kIt + kLight + (tid & 7));
      else if ((W & 3) >= 2)
        for (int k = lane + 64 * ((W & 1) + (W >> 2) * 2); k < S * kLight; k += 4 * 64)
          feat_c(u + 1, (k / kLight) * kIt + k % kLight);
    }
    if (W >= 5) __builtin_amdgcn_s_setprio(0);
    WSTAMP_END(0);
    lds_sync();
    RSTAMP(0);
    WSTAMP_BEGIN();
    // ---- phase B: candidates of vad(u-1), noise(u-2), denoise(u-3); gains(u-4);
    // spectral variability(u+1); raw features of u+2 staged
    if (W < 6) {
      if (live(fD)) {
        const int dst = seg_half(kSd, 0);
        const bool on = on_of(fD);
        if (W < 4)
          epi_h<96>(L, mma_job<2, 6>(fr, W, L, dzs, lane, fD), W, lane, ra[6], L.zd, L.sd, dst, on);
        else if (W == 4)
          epi_h<96>(L, mma_job<8, 6>(fr, 4, L, dzs, lane, fD), 4, lane, ra[6], L.zd, L.sd, dst, on);
        else
          epi_h<96>(L, mma_job<10, 6>(fr, 5, L, dzs, lane, fD), 5, lane, ra[6], L.zd, L.sd, dst, on);
      }
      if (W == 4 && live(fN))
        epi_h<48>(L, mma_job<15, 4>(fr, 1, L, dzs, lane, fN), 1, lane, ra[4], L.zn, L.sn, seg_half(kSn, fN & 1), on_of(fN));
      if (W < 2 && u + 1 < maxnf) feat_d(u + 1);
      // gain smoothing g = max(g, .6*lastg) (denoise.c), frame u-4, on w2, w3, w5
      if ((W == 2 || W == 3 || W == 5) && live(fO)) {
        const int gl = lane + 64 * (W == 5 ? 2 : W - 2);
        for (int idx = gl; idx < S * kBands; idx += 3 * 64) {
          const int s = idx / kBands, i = idx - s * kBands;
          if (!L.act[fO & 7][s]) continue;
          const long long f = L.fbase[s] + fO;
          const float gi = L.gout[s][i];
          const float al = .6f * L.lastg[s][i];
          const float gsm = (gi > al) ? gi : al;
          L.lastg[s][i] = gsm;
          a.gr[f * kBands + i] = gi;
          a.gs[f * kBands + i] = gsm;
        }
      }
    } else {
      if (live(fN)) {
        const int t = W == 6 ? 0 : 2;
        const f4 acc = W == 6 ? mma_job<10, 4>(fr, 0, L, dzs, lane, fN) : mma_job<11, 4>(fr, 2, L, dzs, lane, fN);
        epi_h<48>(L, acc, t, lane, ra[4], L.zn, L.sn, seg_half(kSn, fN & 1), on_of(fN));
      }
      if (live(fV)) {
        const int t = W == 6 ? 1 : 0;
        const f4 acc = W == 6 ? mma_job<15, 2>(fr, 1, L, dzs, lane, fV) : mma_job<16, 2>(fr, 0, L, dzs, lane, fV);
        epi_h<24>(L, acc, t, lane, ra[2], L.zv, L.sv, seg_half(kSv, fV % 3), on_of(fV));
      }
    }
    if (pf_lane) L.pf[u & 1][pfs][pfi] = pf_next;  // frame u + 2: read from the next phase A on
    WSTAMP_END(1);
    lds_sync();
    RSTAMP(1);
  }
  }  // GRU waves
#ifdef FVAD_STAMPS
  if (lane == 0 && a.stamps) {  // k_fused16's pitch-spectrum waves: [16..23] A, [24..31] B
    atomicAdd(&a.stamps[W < 8 ? W : W + 8], wacc[0]);
    atomicAdd(&a.stamps[W < 8 ? 8 + W : W + 16], wacc[1]);
  }
#endif
#undef WSTAMP_BEGIN
#undef WSTAMP_END
  STAMP_FLUSH(48, 2);
  // ---- state write-back (streams that ran at least one frame)
  for (int idx = tid; idx < S * kCeps * kBands; idx += NT) {
    const int s = idx / (kCeps * kBands), i = idx - s * (kCeps * kBands);
    if (sok(s) && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsMem + i] = L.ceps[s][i];
  }
  for (int idx = tid; idx < S * kCeps * kCeps; idx += NT) {
    const int s = idx / (kCeps * kCeps), i = idx - s * (kCeps * kCeps);
    if (sok(s) && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kCepsDist + i] = L.dist[s][i];
  }
  for (int idx = tid; idx < S * kBands; idx += NT) {
    const int s = idx / kBands, i = idx - s * kBands;
    if (sok(s) && L.nfs[s] > 0) a.state[(size_t)(sb + s) * st::kWords + st::kLastG + i] = L.lastg[s][i];
  }
  for (int idx = tid; idx < S * 96; idx += NT) {
    const int s = idx / 96, i = idx - s * 96;
    if (!sok(s) || L.nfs[s] <= 0) continue;
    float *stp = a.state + (size_t)(sb + s) * st::kWords;
    if (i < 24) stp[st::kVadGru + i] = L.sv[s][i];
    if (i < 48) stp[st::kNoiseGru + i] = L.sn[s][i];
    stp[st::kDenGru + i] = L.sd[s][i];
  }
  if (tid < S && sok(tid) && L.nfs[tid] > 0)
    reinterpret_cast<int *>(a.state)[(size_t)(sb + tid) * st::kWords + st::kMemId] = L.memid[tid];
}

__global__ void __launch_bounds__(kGNT) k_gru16(StagedArgs a) { gru16_body<8, false>(a); }
__global__ void __launch_bounds__(kFNT) k_fused16(StagedArgs a) { gru16_body<8, true>(a); }

hipError_t launch_gru16(const StagedArgs &a, hipStream_t stream) {
  if (a.fuse16)
    hipLaunchKernelGGL(k_fused16, dim3((a.n_streams + 7) / 8), dim3(kFNT), 0, stream, a);
  else
    hipLaunchKernelGGL(k_gru16, dim3((a.n_streams + 7) / 8), dim3(kGNT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace fvad
