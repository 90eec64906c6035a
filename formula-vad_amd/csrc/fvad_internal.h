// Internal definitions shared by the host-side plan/model code and the HIP
// kernels of the MI355X-native Formula-VAD hot path.  Not part of the C ABI
// (that is include/fvad.h).
#pragma once
#include <cstddef>
#include <cstdint>

namespace fvad {

// rnnoise frame geometry (Denoiser.zig:68-70 -> rnnoise_get_frame_size()).
constexpr int kFrame = 480;
constexpr int kWin = 960;
constexpr int kFreq = 481;
constexpr int kBands = 22;
constexpr int kFeat = 42;
constexpr int kCeps = 8;
constexpr int kPitchBuf = 1728;  // PITCH_MAX_PERIOD + PITCH_FRAME_SIZE
constexpr int kPitchMax = 768;
constexpr int kPitchMin = 60;
constexpr int kXlp = kPitchBuf / 2;  // 864
constexpr int kMaxNeurons = 128;
constexpr int kMaxCh = 8;
constexpr int kMaxBandCfg = 4;

// FFT B (FFT.zig) is a real FFT of fft_size: any even fft_size (FFT.zig:29-31)
// from 2 up to kMaxFftSize on the device (kissfft's mixed-radix
// factorisation).  Up to kMaxFftB the tables live in the Plan and one
// transform's work array (twice that with a radix > 5) stays in LDS; above it
// the tables are separate device arrays and the work arrays device scratch.
// kMaxFftSize keeps every per-window index in 32 bits (a 87 s window); the
// real limit is memory: the re-block ring holds B * C * (fft_size + T * 480)
// floats.
constexpr int kMaxFftB = 16384;
constexpr int kMaxFftSize = 1 << 22;
constexpr int kMaxFactors = 32;

// FFT-B windows that can complete in one 480-sample tick: one for fft_size >=
// 480, else up to floor((fft_size - 1 + 480) / fft_size) -- the reference
// splits one denoiser frame over several FFT-buffer writes (VAD.zig:307-347).
// The engine's window outputs hold that many slots per (tick, stream).
constexpr int windows_per_tick(int fft_size) { return fft_size >= kFrame ? 1 : (fft_size - 1 + kFrame) / fft_size; }

// ---------------------------------------------------------------------------
// Per-stream persistent state, one contiguous record per stream (the kernels
// run one workgroup per stream, so a record is read/written coalesced).
// Offsets are in 32-bit words.
// ---------------------------------------------------------------------------
namespace st {
constexpr int kPitch = 0;                       // pitch_buf[1728] (last 480 = analysis_mem source)
constexpr int kNdSamples = kPitch;              // use_denoiser = 0 (no pitch buffer): u64 samples consumed
constexpr int kSyn = kPitch + kPitchBuf;        // synthesis_mem[480]
constexpr int kCepsMem = kSyn + kFrame;         // cepstral_mem[8][22]
constexpr int kLastG = kCepsMem + kCeps * kBands;  // lastg[22]
constexpr int kVadGru = kLastG + kBands;        // vad_gru_state[128]
constexpr int kNoiseGru = kVadGru + kMaxNeurons;    // noise_gru_state[128]
constexpr int kDenGru = kNoiseGru + kMaxNeurons;    // denoise_gru_state[128]
constexpr int kHp = kDenGru + kMaxNeurons;      // mem_hp_x[2] (float)
constexpr int kMemId = kHp + 2;                 // int
constexpr int kLastPeriod = kMemId + 1;         // int
constexpr int kLastGain = kLastPeriod + 1;      // float
constexpr int kFramesDone = kLastGain + 1;      // int: ticks processed (480-sample frames per channel)
constexpr int kVolAcc = kFramesDone + 1;        // float: temp_fft_buffer_vol_ratio
constexpr int kCepsDist = kVolAcc + 1;          // staged mode: cepstral distance matrix [8][8]
constexpr int kWords = ((kCepsDist + kCeps * kCeps + 63) / 64) * 64;
}  // namespace st

// ---------------------------------------------------------------------------
// int8 image of the GRU stack for the staged recurrence kernel (k_rnn3 keeps it
// in LDS).  Nine column-major matrices; column c of matrix m holds the K
// weights of one output neuron in summation order (input part, then the
// recurrent part for GRU gates), so one lane walks one column.
//   0 input_dense   1 vad z|r   2 vad h   3 noise z|r   4 noise h
//   5 denoise z|r   6 denoise h 7 denoise_output        8 vad_output
// Shapes are the classic rnnoise model's (the only ones the loaders accept).
// ---------------------------------------------------------------------------
namespace rnnimg {
constexpr int kMats = 9;
constexpr int kCols[kMats] = {24, 48, 24, 96, 48, 192, 96, 22, 1};
constexpr int kKin[kMats] = {42, 24, 24, 90, 90, 114, 114, 96, 24};  // input-vector part of K
constexpr int kK[kMats] = {42, 48, 48, 138, 138, 210, 210, 96, 24};
// Summation segments of a column (inputs in concatenation order, then the
// GRU state); each starts 8-byte aligned so 8 weights are one 64-bit LDS read.
constexpr int kSegs[kMats][4] = {{42, 0, 0, 0},   {24, 24, 0, 0},  {24, 24, 0, 0},
                                 {24, 24, 42, 48}, {24, 24, 42, 48}, {24, 48, 42, 96},
                                 {24, 48, 42, 96}, {96, 0, 0, 0},   {24, 0, 0, 0}};
constexpr int pad8(int x) { return (x + 7) & ~7; }
constexpr int pad16(int x) { return (x + 15) & ~15; }
constexpr int seg_off(int m, int g) {  // byte offset of segment g inside a column
  int o = 0;
  for (int i = 0; i < g; i++) o += pad8(kSegs[m][i]);
  return o;
}
constexpr int stride(int m) { return seg_off(m, 4); }  // bytes per column
constexpr int off_b(int m) {
  int o = 0;
  for (int i = 0; i < m; i++) o += pad16(kCols[i]) + pad16(kCols[i] * stride(i));
  return o;
}
constexpr int off_w(int m) { return off_b(m) + pad16(kCols[m]); }
constexpr int kBytes = off_b(kMats);
}  // namespace rnnimg

// ---------------------------------------------------------------------------
// Read-only plan tables (built on the host by fvad_plan.cpp, uploaded once).
// ---------------------------------------------------------------------------
struct Plan {
  float half_window[kFrame];     // rnnoise analysis/synthesis half window
  float dct[kBands * kBands];    // dct_table[i*22+j]
  float tansig[201];             // tansig_table
  float band_frac[400];          // (float)j/band_size of bin k inside its band
  int band_of[400];              // band index i of bin k (k < 400)
  int eband4[kBands];            // eband5ms[i] << 2
  float tw960[2 * kWin];         // celt twiddles (r,i)
  int bitrev960[kWin];           // celt bit-reverse table
  int ibitrev960[kWin];          // its inverse: ibitrev960[bitrev960[i]] = i
  // FFT B (kissfft real FFT of size nfft_b)
  int nfft_b;                    // real size (2048)
  int ncfft_b;                   // nfft_b / 2
  int stages_b;                  // log4(ncfft_b) when ncfft_b = 4^k (k_fftbw), else 0
  int nfac_b;                    // kf_factor(ncfft_b): (p, m) pairs
  int fac_b[2 * kMaxFactors];
  int generic_b;                 // a radix > 5 occurs (out-of-place stage scratch needed)
  float norm_b;                  // windowNormFactor / (nfft/2)
  float twb[2 * kMaxFftB / 2];   // kissfft substate twiddles (r,i)
  float superb[2 * kMaxFftB / 4];  // super twiddles (r,i)
  int permb[kMaxFftB / 2];       // kf_work leaf permutation
  float hannb[kMaxFftB];         // hannWindowPeriodic(nfft_b)
};

// Device-side model: int8 weights stored as float (int8->float is exact).
struct DevDense {
  int nin, nout, act;
  const float *w;  // [nin][nout]
  const float *b;  // [nout]
};
struct DevGru {
  int nin, nout, act;
  const float *win;   // [nin][3*nout]
  const float *wrec;  // [nout][3*nout]
  const float *b;     // [3*nout]
};
struct DevModel {
  DevDense in_dense, den_out, vad_out;
  DevGru vad, noise, den;
};

constexpr int kActTanh = 0, kActSigmoid = 1, kActRelu = 2;

// Host-side model (int8, text-file order).
struct HostLayer {
  int nin = 0, nout = 0, act = 0;
  bool gru = false;
  std::size_t off_w = 0, off_r = 0, off_b = 0;  // offsets into blob
};
struct HostModel {
  HostLayer layers[6];  // input_dense, vad_gru, noise_gru, denoise_gru, denoise_output, vad_output
  int8_t *blob = nullptr;
  std::size_t blob_size = 0;
};

// Every table of the plan; for nfft_b > kMaxFftB only FFT B's metadata
// (sizes, factors, norm_b), the tables then come from build_fftb_tables.
void build_plan(Plan *p, int nfft_b);
// FFT B's tables for any even nfft_b into caller arrays: twb[nfft_b]
// (nfft_b / 2 complex), superb[nfft_b / 2], permb[nfft_b / 2], hannb[nfft_b];
// fac = kf_factor(nfft_b / 2) pairs.  Returns norm_b.
float build_fftb_tables(int nfft_b, const int *fac, float *twb, float *superb, int *permb, float *hannb);

}  // namespace fvad

// Synthetic streams base + s0 .. base + s0 + ns - 1 (each generated with length
// total_ticks * 480) in push layout: ticks [tick0, tick0 + n_ticks) to
// out[t][s][c][480] with out_streams streams per tick row (fvad_synth.cpp)
int fvad_synth_group(uint32_t base, int s0, int ns, int n_channels, int total_ticks, int tick0, int n_ticks,
                     float *out, std::size_t out_streams);
