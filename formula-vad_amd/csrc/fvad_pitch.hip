// k_pcorr in a translation unit of its own: built without SLP vectorisation
// (Makefile), which keeps its f32 sums in single VALU instructions -- measured
// faster for this kernel (1.60 -> 1.46 ms), while k_plpc and the GRU kernel
// in fvad_staged.hip prefer the packed form.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "fvad_device.h"
#include "fvad_internal.h"
#include "fvad_staged.h"
#include "fvad_staged_dev.h"

#include <algorithm>

namespace fvad {

// ---------------------------------------------------------------------------
// k_pcorr: one 256-thread workgroup per half quarter tile (8 streams at one
// frame position; 39.8 KB of LDS, so 4 workgroups share a CU).
//   Q0 the frames' x_lp windows (from the x_lp rows) and the coarse Syy
//      sequence -> LDS; xf = celt_fir5(x_lp) with k_plpc's coefficients, in
//      place
//   Q1 coarse xcorr: lane = (frame, 5 consecutive lags), a register window of
//      5 y values slides one sample per step (2 LDS reads per 5 MACs); then
//      the coarse scan's survivors: a prefix top-2 of the lags' xcorr^2/Syy
//      ratios over the frame's 32 lanes drops every lag that provably cannot
//      change find_best_pitch's state, and the rest are listed in lag order
//   Q2 coarse find_best_pitch over the survivors (exact, lane per frame; ~3 k
//      instead of ~23 k cycles for all 147 lags)
//   Q3 fine xcorr at the <= 10 lags within +-2 of 2*best (others are 0), on
//      lanes split by lag parity; each lane also walks the fine Syy
//      recurrence from k_plpc's checkpoint below its lag (<= 7 steps)
//   Q4 fine find_best_pitch + pseudo-interpolation -> T0, candidate count
//   Q5 remove_doubling products: lane = (frame, candidate c); candidate c's
//      xcorr at T-1, T, T+1 share a sliding window of 3, plus xcorr(T1b);
//      operands are read as aligned pairs (ds_read_b64: 64 banks, 2 steps
//      per read), the lane's window parity resolved by selects
//   Beside Q2..Q4, wave 2 (idle there) walks remove_doubling's yy_lookup
//   recurrence (lane per frame, 384 serial steps), keeping every 8th state in
//   LDS; Q5 rebuilds the values it needs from those checkpoints.
// ---------------------------------------------------------------------------
#ifndef FVAD_WALK_Q2
#define FVAD_WALK_Q2 6
#endif
#ifndef FVAD_WALK_Q3
#define FVAD_WALK_Q3 36
#endif
// Q5's walking waves at s_setprio 2 (the group ends with them; 1.20 -> 1.19
// ms); the yy walker at priority 2 beside Q2..Q4 measured no better
#ifndef FVAD_PC_PRIO
#define FVAD_PC_PRIO 1
#endif
#ifndef FVAD_Q5_UNROLL
#define FVAD_Q5_UNROLL 4  // Q5 walk unroll (2 / 8 measured no better)
#endif
#define FVAD_PRAGMA_(x) _Pragma(#x)
#define FVAD_UNROLL(n) FVAD_PRAGMA_(unroll n)
constexpr int kWalkQ2 = FVAD_WALK_Q2, kWalkQ3 = FVAD_WALK_Q3;  // yy walk checkpoint blocks done by the end of Q2 / Q3 (of 49)
constexpr int kYyCk = 49;  // checkpoints yy_{8k}, 8k <= 384
static_assert(FVAD_WALK_Q2 <= 6, "the checkpoints walked during Q2 live in the spare floats of the xf rows");
constexpr int kPcF = 8;                // frames per workgroup (a quarter tile holds 16)
constexpr int kPcL = 32;               // lanes per frame in Q1 (16: 188 VGPRs, 2 waves per SIMD, 3 % slower)
constexpr int kPcNT = kPcL * kPcF;
static_assert(ptile::kQuarter % kPcF == 0 && kPcF % 4 == 0, "k_pcorr groups");
// FVAD_DIAG_SKIP (bit 1 Q1, 2 Q3, 4 Q5): diagnostic flavours without that
// phase's sums, for the per-phase LDS attribution (`make diag`,
// tools/lds_attr.sh); bit 8: Q1's y reads at a lane stride of 5 words instead
// of 10 (wrong values, the same instructions; 32 distinct banks per 32-lane
// group instead of 16): the upper bound of a conflict-free Q1 layout.  Never
// set in the product build
#ifndef FVAD_DIAG_SKIP
#define FVAD_DIAG_SKIP 0
#endif
constexpr int kPcXS = 870;  // xf row pitch: even (8-byte aligned pairs in Q5), = 6 mod 8 (conflict-free Q0 stores)
constexpr int kPcSP = 153;  // coarse xcorr / Syy row pitch (odd; >= 147 rounded up to the scan block)

// __shfl_up within 32-lane halves from an explicit lane id (`self`, made
// opaque per group by the caller, so the bpermute addresses are not hoisted
// out of the persistent loop into registers held for the whole kernel)
__device__ __forceinline__ int shfl_up32(int v, int d, int self) {
  const int idx = (self & 31) >= d ? self - d : self;
  return __builtin_amdgcn_ds_bpermute(idx << 2, v);
}
__device__ __forceinline__ float shfl_up32(float v, int d, int self) {
  return __int_as_float(shfl_up32(__float_as_int(v), d, self));
}

__global__ void __launch_bounds__(kPcNT) k_pcorr(StagedArgs a) {
  constexpr int NT = kPcNT;
  constexpr int kHalves = ptile::kQuarter / kPcF;
  __shared__ __attribute__((aligned(16))) float xf[kPcF][kPcXS];
  __shared__ float scl[kPcF][kPcSP], xc[kPcF][kPcSP];
  __shared__ float sfl[kPcF][10], fine[kPcF][10];
  __shared__ unsigned char lst[kPcF][kPcSP - 1];  // lags of the coarse scan's survivors (Q1 -> Q2)
  __shared__ int ncand[kPcF];
  __shared__ int best[kPcF][2], T0s[kPcF], nvs[kPcF], fval[kPcF];
  __shared__ long long fidx[kPcF];
  // yy_lookup checkpoints yy_{8k}, k = 0..48: k < 6 (walked during Q2, while
  // xc is still read) in the 6 spare floats of each xf row, the rest in xc
  // rows (dead after Q2; Q5 uses only xc[fr][0..14])
  auto yy_ck = [&](int fr, int k) -> float * { return k < 6 ? &xf[fr][kXlp + k] : &xc[fr][16 + k]; };
  const int tid = threadIdx.x;
  const int Vr = a.n_ticks * a.n_channels;
  const int n_sb = (a.n_streams + 63) >> 6;
  const long long nquarters = (long long)n_sb * Vr * 4;
  const long long ngroups = (nquarters + 7) / 8 * 16;  // whole blocks of 16 units; units past the quarters skip
  STAMP_INIT();
#ifdef FVAD_STAMPS
  unsigned long long st_scan = 0, st_walk = 0;  // lane 0 of waves 0 / 1: the coarse scan / the yy walk alone
#endif
  __shared__ long long gq;
  if (threadIdx.x == 0) gq = take_group(a, kWorkPcorr);
  __syncthreads();
  long long g = gq;
  while (g < ngroups) {
    // per-group opaque copy of tid: keeps the compiler from hoisting the
    // phases' per-thread offsets out of the persistent loop into registers
    // held for the whole kernel (124 -> 86 VGPRs)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    // group g -> (quarter tile, frame columns h*kPcF ..): T is the group's
    // first column, rows keep the quarter's 16-column pitch.  The halves of a
    // quarter are units x + 16 b and x + 16 b + 8, both from queue x (one
    // XCD), so the second half's 64-byte row reads find the first half's
    // 128-byte lines in that XCD's L2.
    static_assert(kHalves == 2 && kQueues == 8, "k_pcorr unit map");
    const long long gq4 = (g >> 4) * 8 + (g & 7);
    const int h = (int)((g >> 3) & 1);
    if (gq4 >= nquarters) {  // padding unit of the last block (uniform branch)
      __syncthreads();
      if (tq == 0) gq = take_group(a, kWorkPcorr);
      __syncthreads();
      g = gq;
      continue;
    }
    float *Tq = a.ptile + (size_t)gq4 * ptile::kRows * ptile::kQuarter;  // the quarter's block
    const float *T = Tq + h * kPcF;
    const long long gt = gq4 >> 2;
    const int gqq = (int)(gq4 & 3);
    const int gsb = (int)(gt / Vr), gv = (int)(gt - (long long)gsb * Vr);
    const int s_first = gsb * 64 + gqq * 16 + h * kPcF;  // stream of the group's frame 0
    if (tq < kPcF) {
      const int s = s_first + tq;
      fval[tq] = s < a.n_streams && gv < ticks_of(a, s) * a.n_channels;
      fidx[tq] = (long long)s * a.V + gv;
    }
    // Q0: xf = celt_fir5(x_lp) rebuilt here (k_plpc stores only the filter's
    // coefficients): the frames' x_lp rows (864 values each, contiguous in
    // the x_lp row of the stream) -> LDS, and the coarse Syy sequence; loads
    // go out in batches of kQ0B before their LDS stores
    {
      constexpr int kRow4 = kXlp / 4;                    // float4 per frame's x_lp window
      constexpr int P4 = kPcF / 4;                       // float4 per Syy row and group
      constexpr int kN1 = kRow4 * kPcF, kQ0N = kN1 + 147 * P4, kQ0B = 4;
      for (int u0 = 0; u0 < kQ0N; u0 += NT * kQ0B) {
        float4 w4[kQ0B];
#pragma unroll
        for (int u = 0; u < kQ0B; u++) {
          const int idx = u0 + tq + NT * u;
          if (idx < kN1) {
            const int fr = idx / kRow4, j = idx - fr * kRow4;
            const int s = min(s_first + fr, a.n_streams - 1);
            w4[u] = *reinterpret_cast<const float4 *>(a.xlp + (size_t)s * a.LX + (size_t)gv * (kFrame / 2) + 4 * j);
          } else if (idx < kQ0N) {
            const int r = (idx - kN1) / P4, p = (idx - kN1) % P4;
            w4[u] = *reinterpret_cast<const float4 *>(T + (ptile::kSc + r) * ptile::kQuarter + 4 * p);
          }
        }
#pragma unroll
        for (int u = 0; u < kQ0B; u++) {
          const int idx = u0 + tq + NT * u;
          if (idx < kN1) {
            const int fr = idx / kRow4, j = idx - fr * kRow4;
            float2 *d = reinterpret_cast<float2 *>(&xf[fr][4 * j]);  // rows are 8-byte aligned
            d[0] = make_float2(w4[u].x, w4[u].y);
            d[1] = make_float2(w4[u].z, w4[u].w);
          } else if (idx < kQ0N) {
            const int r = (idx - kN1) / P4, p = (idx - kN1) % P4;
            float *d = &scl[4 * p][r];
            d[0] = w4[u].x;
            d[kPcSP] = w4[u].y;
            d[2 * kPcSP] = w4[u].z;
            d[3 * kPcSP] = w4[u].w;
          }
        }
      }
    }
    {
      // celt_fir5 in place: lane (frame, l) filters x_lp[27 l .. 27 l + 26]
      // (history x[n-1..n-5] = 0 before n = 0; x_lp[0] = the frame's edge
      // value), the outputs held until every lane has read its inputs
      constexpr int kRun = kXlp / kPcL;
      static_assert(kRun * kPcL == kXlp, "FIR runs");
      const int fr = tq / kPcL, n0 = kRun * (tq % kPcL);
      const float *ft = T + ptile::kFir * ptile::kQuarter + fr;
      float l[5];
#pragma unroll
      for (int i = 0; i < 5; i++) l[i] = ft[i * ptile::kQuarter];
      const float x0 = ft[5 * ptile::kQuarter];
      __syncthreads();
      const float *xr = xf[fr];
      float m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0;
      if (n0 > 0) {
        m1 = xr[n0 - 1];
        m2 = xr[n0 - 2];
        m3 = xr[n0 - 3];
        m4 = xr[n0 - 4];
        m5 = xr[n0 - 5];
      }
      float y[kRun];
#pragma unroll
      for (int k = 0; k < kRun; k++) {
        const float x = (k == 0 && n0 == 0) ? x0 : xr[n0 + k];
        float v = x;
        v = v + l[0] * m1;
        v = v + l[1] * m2;
        v = v + l[2] * m3;
        v = v + l[3] * m4;
        v = v + l[4] * m5;
        m5 = m4, m4 = m3, m3 = m2, m2 = m1, m1 = x;
        y[k] = v;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kRun; k++) xf[fr][n0 + k] = y[k];
    }
    __syncthreads();
    RSTAMP(0);
    // Q1: xcorr[k] = sum_j x_lp4[j] y_lp4[j+k], x_lp4[j] = xf[384+2j], y_lp4[m] = xf[2m]
    {
      constexpr int R = 5;
      static_assert(R * (kPcL - 1) >= 147 && 240 % R == 0 && kPcL == 32, "Q1 lag blocks");
      const int fr = tq / kPcL, l = tq % kPcL, k0 = R * l;
      float acc[R];
#pragma unroll
      for (int r = 0; r < R; r++) acc[r] = 0.0f;
      if (k0 < 147) {
        const float *X = xf[fr] + (kPitchMax >> 1);
        const float *Y = xf[fr] + ((FVAD_DIAG_SKIP & 8) ? k0 : 2 * k0);
        float win[R];
        auto yld = [&](int m) -> float { return Y[2 * m]; };
#pragma unroll
        for (int r = 0; r < R; r++) win[r] = yld(r);
        for (int jb = 0; jb < ((FVAD_DIAG_SKIP & 1) ? 0 : 240); jb += R) {
#pragma unroll
          for (int u = 0; u < R; u++) {
            const float xv = X[2 * (jb + u)];
#pragma unroll
            for (int r = 0; r < R; r++) acc[r] = acc[r] + xv * win[(r + u) % R];
            win[u] = yld(jb + u + R);  // lag k0+R-1 at step jb+u+1
          }
        }
#pragma unroll
        for (int r = 0; r < R; r++)
          if (k0 + r < 147) xc[fr][k0 + r] = acc[r];
      } else if (k0 < kPcSP) {
        // lags 147.. pad the scan's last block: xcorr <= 0 never updates the best pair
        for (int k = 147; k < kPcSP; k++) xc[fr][k] = -1.0f;
      }
      // Survivors of the coarse find_best_pitch.  A lag j changes the scan's
      // state only if num_j * bd1 > bn1 * Syy_j against the second-best pair
      // at j, whose ratio bn1 / bd1 is (up to float rounding) at least the
      // second largest ratio num / Syy among the positive lags before j.  A
      // lag whose ratio is below that by more than 0.1 % fails its test for
      // certain and is dropped; the exact scan (Q2) then visits only the
      // survivors, in order, and ends in the same state.  Ratios here are only
      // a filter (rounded reciprocal); lags with xcorr <= 0 never update.
      constexpr float kNoRatio = -__builtin_inff();
      float rho[R];
      float m1 = kNoRatio, m2 = kNoRatio;
#pragma unroll
      for (int r = 0; r < R; r++) {
        float v = kNoRatio;
        if (k0 + r < 147 && acc[r] > 0) {
          float x16 = acc[r];
          x16 *= 1e-12f;
          v = (x16 * x16) * __builtin_amdgcn_rcpf(scl[fr][k0 + r]);
        }
        rho[r] = v;
        m2 = fmaxf(m2, fminf(m1, v));
        m1 = fmaxf(m1, v);
      }
      int self = tq & 63;
      asm volatile("" : "+v"(self));
      // inclusive prefix top-2 over the frame's 32 lanes, then exclusive
#pragma unroll
      for (int d = 1; d < kPcL; d <<= 1) {
        const float p1 = shfl_up32(m1, d, self), p2 = shfl_up32(m2, d, self);
        if (l >= d) {
          const float n2 = fmaxf(fminf(m1, p1), fmaxf(m2, p2));
          m1 = fmaxf(m1, p1);
          m2 = n2;
        }
      }
      float e1 = shfl_up32(m1, 1, self), e2 = shfl_up32(m2, 1, self);
      if (l == 0) e1 = e2 = kNoRatio;
      unsigned mask = 0;
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (rho[r] != kNoRatio && !(e2 > rho[r] * 1.001f)) mask |= 1u << r;
        e2 = fmaxf(e2, fminf(e1, rho[r]));
        e1 = fmaxf(e1, rho[r]);
      }
      // the survivors' lags in order
      const int c = __builtin_popcount(mask);
      int pos = c;
#pragma unroll
      for (int d = 1; d < kPcL; d <<= 1) {
        const int t = shfl_up32(pos, d, self);
        if (l >= d) pos += t;
      }
      int o = pos - c;
#pragma unroll
      for (int r = 0; r < R; r++)
        if (mask & (1u << r)) lst[fr][o++] = (unsigned char)(k0 + r);
      if (l == kPcL - 1) {
        ncand[fr] = pos;
        // pad entries: the scan runs whole blocks of 4 (lag 147: xcorr -1, no update)
#pragma unroll
        for (int u = 0; u < 4; u++) lst[fr][pos + u] = 147;
      }
    }
    __syncthreads();
    RSTAMP(1);
    // remove_doubling's yy_lookup recurrence, lane per frame on wave 2 (idle
    // from Q2 to Q4), in three pieces beside Q2, Q3 and Q4:
    // yy_lookup[i] = max(0, yy_i), yy_i = (yy_{i-1} + x[-i]^2) - x[480-i]^2
    // from yy_0 = xx, x = xf + 384.  Only every 8th state yy_{8k} (unclamped)
    // is kept, in LDS (yy_ck): Q5 rebuilds the two values an item needs from
    // the checkpoint below them in at most 7 steps of the same recurrence.
    const bool walker = tq >= 128 && tq < 128 + kPcF && fval[tq - 128];
    float wyy = 0;
    const float *wxr = nullptr;
    int wfr = 0;
    if (walker) {
      wfr = tq - 128;
      wxr = xf[wfr];
      wyy = Tq[ptile::kXx * ptile::kQuarter + h * kPcF + wfr];
    }
    // walk checkpoint blocks [k0, k1): block k > 0 runs steps 8k-7 .. 8k
    auto walk = [&](int k0, int k1) {
#ifdef FVAD_STAMPS
      const unsigned long long w0_ = __builtin_amdgcn_s_memtime();
#endif
      int k = k0;
      if (k == 0) {
        *yy_ck(wfr, 0) = wyy;
        k = 1;
      }
#pragma unroll 2
      for (; k < k1; k++) {
#pragma unroll
        for (int i = 8 * k - 7; i <= 8 * k; i++) {
          const float va = wxr[384 - i], vb = wxr[864 - i];
          wyy = wyy + va * va - vb * vb;
        }
        *yy_ck(wfr, k) = wyy;
      }
#ifdef FVAD_STAMPS
      if (tq == 128) st_walk += __builtin_amdgcn_s_memtime() - w0_;
#endif
    };
    // Q2
    if (tq < kPcF) {
      const int fr = tq;
#ifdef FVAD_STAMPS
      const unsigned long long s0_ = __builtin_amdgcn_s_memtime();
#endif
      int bst[2] = {0, 1};
      float bn0 = -1, bn1 = -1, bd0 = 0, bd1 = 0;
      // operands of the next 4 lags load while these 4 are visited (8 ahead:
      // 112 VGPRs, and 4 x 112 + k_prep3's 96 no longer fit one SIMD's 512,
      // so the CUs that host k_prep3 lose a workgroup: 1.45 vs 1.39 ms)
      constexpr int B = 4;
      int jb[B];
#pragma unroll
      for (int u = 0; u < B; u++) jb[u] = lst[fr][u];
      const int n = ncand[fr];
      for (int i0 = 0; i0 < n; i0 += B) {
        int jn[B];
#pragma unroll
        for (int u = 0; u < B; u++) jn[u] = lst[fr][min(i0 + B + u, kPcSP - 2)];
        float xb[B], yb[B];
#pragma unroll
        for (int u = 0; u < B; u++) {
          xb[u] = xc[fr][jb[u]];
          yb[u] = scl[fr][jb[u]];
        }
#pragma unroll
        for (int u = 0; u < B; u++) best_pitch_visit(xb[u], yb[u], jb[u], bn0, bn1, bd0, bd1, bst);
#pragma unroll
        for (int u = 0; u < B; u++) jb[u] = jn[u];
      }
      best[fr][0] = bst[0];
      best[fr][1] = bst[1];
#ifdef FVAD_STAMPS
      if (fr == 0) st_scan += __builtin_amdgcn_s_memtime() - s0_;
#endif
    } else if (walker) {
      walk(0, kWalkQ2);
    }
    __syncthreads();
    RSTAMP(2);
    // Q3
    if (walker) walk(kWalkQ2, kWalkQ3);
    // lanes by lag parity: wave 0 = the 6 even lags of each frame (u % 5 in
    // {0, 2, 4}), wave 1 = the 4 odd ones, so each wave reads its y operands
    // as aligned pairs (ds_read_b64) without per-lane parity selects; x is
    // the frame's aligned pair row (broadcast to its lanes)
    if (tq < 6 * kPcF || (tq >= 64 && tq < 64 + 4 * kPcF)) {
      const bool odd = tq >= 64;
      const int e = odd ? tq - 64 : tq, per = odd ? 4 : 6;
      const int fr = e / per, k = e - per * fr;
      // u: window (k / (per / 2)), position within the window by parity
      const int win = k / (per / 2), kk = k - win * (per / 2);
      const int u = 5 * win + (odd ? 1 + 2 * kk : 2 * kk);
      const int bp0 = best[fr][0], bp1 = best[fr][1];
      const int i = (u < 5 ? 2 * bp0 : 2 * bp1) - 2 + (u % 5);
      const bool dup = u >= 5 && abs(i - 2 * bp0) <= 2;
      if (i >= 0 && i < 294 && !dup) {
        // the fine Syy of lag i (Q4): k_plpc's checkpoint before step 8 (i / 8),
        // loaded now, walked to i after the product
        const int ck = i >> 3;
        float syy = T[(ptile::kSf + ck) * ptile::kQuarter + fr];
        typedef float v2f __attribute__((ext_vector_type(2)));
        const v2f *xp = reinterpret_cast<const v2f *>(xf[fr] + (kPitchMax >> 1));
        float sum = 0.0f;
        constexpr int kQ3N = (FVAD_DIAG_SKIP & 2) ? 0 : 240;
        if (!odd) {
          const v2f *yp = reinterpret_cast<const v2f *>(xf[fr] + i);
#pragma unroll 8
          for (int j = 0; j < kQ3N; j++) {
            const v2f xv = xp[j], yv = yp[j];
            sum = sum + xv.x * yv.x;
            sum = sum + xv.y * yv.y;
          }
        } else {
          // y[2j] = pair(i - 1 + 2j).y, y[2j + 1] = pair(i + 1 + 2j).x
          const v2f *yp = reinterpret_cast<const v2f *>(xf[fr] + i - 1);
          v2f prev = yp[0];
#pragma unroll 8
          for (int j = 0; j < kQ3N; j++) {
            const v2f xv = xp[j], nx = yp[j + 1];
            sum = sum + xv.x * prev.y;
            sum = sum + xv.y * nx.x;
            prev = nx;
          }
        }
        fine[fr][u] = (-1 > sum) ? -1 : sum;
        for (int j = 8 * ck; j < i; j++) {
          const float y = xf[fr][j + 480], yb = xf[fr][j];
          syy += y * y - yb * yb;
          syy = (1 > syy) ? 1 : syy;
        }
        sfl[fr][u] = syy;
      }
    }
    __syncthreads();
    RSTAMP(3);
    // Q4
    if (walker) walk(kWalkQ3, kYyCk);
    if (tq < kPcF) {
      const int fr = tq;
      const int bp0 = best[fr][0], bp1 = best[fr][1];
      const int w0 = 2 * bp0 - 2, w1 = 2 * bp1 - 2;
      // lags of the first window take its values (a duplicate lag of the
      // second window was not computed in Q3)
      auto slot = [&](int i) -> int { return (i >= w0 && i <= w0 + 4) ? i - w0 : ((i >= w1 && i <= w1 + 4) ? 5 + i - w1 : -1); };
      auto xcf = [&](int i) -> float {
        const int s = slot(i);
        return s < 0 ? 0.0f : fine[fr][s];
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
      for (int i = max(0, lo0); i <= min(293, hi0); i++) best_pitch_visit(xcf(i), sfl[fr][slot(i)], i, bn0, bn1, bd0, bd1, bst);
      for (int i = max(max(0, lo1), hi0 + 1); i <= min(293, hi1); i++)
        best_pitch_visit(xcf(i), sfl[fr][slot(i)], i, bn0, bn1, bd0, bd1, bst);
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
    }
    __syncthreads();
    RSTAMP(4);
    // Q5
    // Item (frame, candidate c) = lane fr * 15 + c of waves 0-1 for the
    // sliding-window sums (T-1, T, T+1) and the same lane of waves 2-3 for the
    // T1b sum, which goes through xc (dead since Q2) to the window lane: each
    // wave's serial walk carries 3 or 1 chains instead of 4.
    const bool q5b = tq >= 128;
    const int q5i = q5b ? tq - 128 : tq;
    // the next group is taken here, so the atomic's round trip hides under
    // the walks; published through LDS at the group's end, whose barrier then
    // waits for LDS only (not for this group's record stores)
    long long g_next = 0;
    if (tq == 0) g_next = take_group(a, kWorkPcorr);
    // items packed in frame order from lane 0 (window items c = 0..nv on
    // waves 0-1, T1b items c = 1..nv on waves 2-3): ~7.6 items per frame fill
    // one wave of each pair, the other usually has none and skips the walk
    int q5f = 0, q5c = 0;
    bool q5on = false;
    {
      int base = 0;
#pragma unroll
      for (int f = 0; f < kPcF; f++) {
        const int n = fval[f] ? (q5b ? nvs[f] : 1 + nvs[f]) : 0;
        if (!q5on && q5i >= base && q5i < base + n) {
          q5on = true;
          q5f = f;
          q5c = q5i - base + (q5b ? 1 : 0);
        }
        base += n;
      }
    }
    float aM = 0, a0 = 0, aP = 0;
    int q5T0 = 0, q5Tc = 0, q5Tb = 0;
    if ((FVAD_PC_PRIO & 1) && q5on) __builtin_amdgcn_s_setprio(2);
    if (q5on) {
      const int fr = q5f, c = q5c;
      q5T0 = T0s[fr];
      q5Tc = c == 0 ? q5T0 : rd_T1(q5T0, c + 1);
      q5Tb = c == 0 ? q5T0 : rd_T1b(q5T0, q5Tc, c + 1);
      const float *X = xf[fr] + (kPitchMax >> 1);
      typedef float v2f __attribute__((ext_vector_type(2)));
      const char *xb0 = reinterpret_cast<const char *>(&xf[0][0]);
      const v2f *Xp = reinterpret_cast<const v2f *>(X);
      int oX = (int)(reinterpret_cast<const char *>(Xp) - xb0);
      if (q5b) {
        // xcorr(T1b): X[j - Tb] in aligned pairs, the lane's parity by selects
        const int mb = -q5Tb, ob = mb & 1;
        const v2f *Bq = reinterpret_cast<const v2f *>(X + (mb - ob));
        v2f r0 = Bq[0], rp = Bq[1];
        float b0 = ob ? r0.y : r0.x, b1 = ob ? rp.x : r0.y;
        int oB = (int)(reinterpret_cast<const char *>(Bq) - xb0);
        float aB = 0;
        FVAD_UNROLL(FVAD_Q5_UNROLL)
        for (int i = 0; i < ((FVAD_DIAG_SKIP & 4) ? 0 : 240); i++) {
          const v2f xp = *reinterpret_cast<const v2f *>(xb0 + oX);
          const v2f rn = *reinterpret_cast<const v2f *>(xb0 + oB + 16);
          oX += 8;
          oB += 8;
          asm volatile("" : "+v"(oX), "+v"(oB));
          aB = aB + xp.x * b0;
          aB = aB + xp.y * b1;
          b0 = ob ? rp.y : rp.x;
          b1 = ob ? rn.x : rp.y;
          rp = rn;
        }
        xc[fr][c] = aB;
      } else {
        // xcorr at T+1, T, T-1 from one sliding window X[j - Tc - 1 + t]
        const int m0 = -q5Tc - 1, ow = m0 & 1;
        const v2f *W = reinterpret_cast<const v2f *>(X + (m0 - ow));
        v2f q0 = W[0], q1 = W[1], qp = W[2];
        float w0 = ow ? q0.y : q0.x, w1 = ow ? q1.x : q0.y;
        float w2 = ow ? q1.y : q1.x, w3 = ow ? qp.x : q1.y;
        int oW = (int)(reinterpret_cast<const char *>(W) - xb0);
        FVAD_UNROLL(FVAD_Q5_UNROLL)
        for (int i = 0; i < ((FVAD_DIAG_SKIP & 4) ? 0 : 240); i++) {  // j = 2i, 2i + 1
          const v2f xp = *reinterpret_cast<const v2f *>(xb0 + oX);
          const v2f qn = *reinterpret_cast<const v2f *>(xb0 + oW + 24);
          oX += 8;
          oW += 8;
          asm volatile("" : "+v"(oX), "+v"(oW));
          aM = aM + xp.x * w0;
          a0 = a0 + xp.x * w1;
          aP = aP + xp.x * w2;
          aM = aM + xp.y * w1;
          a0 = a0 + xp.y * w2;
          aP = aP + xp.y * w3;
          w0 = w2;
          w1 = w3;
          w2 = ow ? qp.y : qp.x;
          w3 = ow ? qn.x : qp.y;
          qp = qn;
        }
      }
    }
    if (FVAD_PC_PRIO & 1) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    if (q5on && !q5b) {
      const int fr = q5f, c = q5c;
      // yy_lookup[T] from the checkpoint yy_{8 (T / 8)}: the walker's steps
      // to T, then its clamp
      auto yy_at = [&](int Tl) -> float {
        const int k = Tl >> 3;
        float w = *yy_ck(fr, k);
        for (int i = 8 * k + 1; i <= Tl; i++) {
          const float va = xf[fr][384 - i], vb = xf[fr][864 - i];
          w = w + va * va - vb * vb;
        }
        return (0 > w) ? 0 : w;
      };
      const float yyA = yy_at(q5Tc);
      const float xx = T[ptile::kXx * ptile::kQuarter + fr];
      float *rg = a.rec + fidx[fr] * rec::kSize;
      const int off = pitch_offset(aP, a0, aM);
      if (c == 0) {
        rg[rec::kT0] = __int_as_float(q5T0);
        rg[rec::kNValid] = __int_as_float(nvs[fr]);
        rg[rec::kG0] = pitch_gain(a0, xx, yyA);
        rg[rec::kXy0] = a0;
        rg[rec::kYy0] = yyA;
        rg[rec::kOff0] = __int_as_float(off);
      } else {
        const float yyB = yy_at(q5Tb);
        float *qk = rg + rec::kK + (c - 1) * rec::kKStride;
        const float xy = .5f * (a0 + xc[fr][c]), yy = .5f * (yyA + yyB);
        qk[0] = __int_as_float(q5Tc);
        qk[1] = pitch_gain(xy, xx, yy);
        qk[2] = xy;
        qk[3] = yy;
        qk[4] = __int_as_float(off);
      }
    }
    if (tq == 0) gq = g_next;
    lds_sync();
    RSTAMP(5);
    g = gq;
  }
  STAMP_FLUSH(32, 6);
#ifdef FVAD_STAMPS
  if (a.stamps && tid == 0) atomicAdd(&a.stamps[38], st_scan);
  if (a.stamps && tid == 128) atomicAdd(&a.stamps[39], st_walk);
#endif
}

hipError_t launch_pcorr(const StagedArgs &a, long long tiles, int n_cu, hipStream_t stream) {
  static const int per_cu = [] {
    int p = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, k_pcorr, kPcNT, 0) != hipSuccess || p < 1) p = 1;
    return p;
  }();
  const int resident = per_cu * n_cu;
  const long long groups = tiles * 4 * (ptile::kQuarter / kPcF);
  hipLaunchKernelGGL(k_pcorr, dim3((unsigned)std::min<long long>(groups, resident)), dim3(kPcNT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace fvad
