// Batched multi-stream engine (C ABI in include/fvad.h).
//
// One engine owns one GPU and a partition of streams.  Device memory layout
// (all HBM, sized for thousands of streams; 288 GB per MI355X leaves room for
// hundreds of ticks of input per push):
//   state   [streams][st::kWords]        persistent rnnoise + re-block state
//   ring    [streams][channels][ring]    denoised samples awaiting FFT B
//   pcm     [max_ticks][streams][ch][480] input staging (or resident synthetic)
//   xbuf    [max_ticks][streams][ch][480] high-passed s16-scale frames (k_prep)
//   ratio / outputs [max_ticks][streams] (+ channels, bands)
// staged mode (default, fvad_staged.hip) adds per-frame intermediates,
// frame f = s * V + tick * C + c with V = max_ticks * C:
//   xs [streams][1248 + V*480]  high-passed samples with pitch history
//   X, P [f][481] complex; Ex/Ep/Exp/Lyf [f][22]; f34 [f][8]; rec [f][144];
//   ys [f][960]; silence / pitch / vad [f]
// fused mode (fvad_kernels.hip): xbuf [max_ticks][streams][ch][480] and one
// k_frame workgroup per stream.  Both run on the engine's HIP stream and give
// identical results.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <algorithm>
#include <vector>

#include "../../include/fvad.h"
#include "fvad_internal.h"
#include "fvad_kernels.h"
#include "fvad_staged.h"

const fvad::HostModel *fvad_model_host(const fvad_model *m);

namespace {
thread_local std::string g_err;
int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}
// the GRU stack on the matrix cores (configs[4]): split (k_pspecw + k_gru16) or fused (k_fused16)
bool fp16_mode(int mode) { return mode == FVAD_MODE_FP16 || mode == FVAD_MODE_FP16_FUSED; }
}  // namespace

extern "C" const char *fvad_last_error(void) { return g_err.c_str(); }
extern "C" const char *fvad_version(void) { return "fvad-mi355x 0.1 (gfx950)"; }

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail(FVAD_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct fvad_engine {
  fvad_engine_config cfg{};
  int ring_len = 0;
  hipStream_t stream = nullptr;
  fvad::Plan *d_plan = nullptr;
  float *d_weights = nullptr;
  fvad::DevModel dmodel{};
  fvad::DevModel *d_model = nullptr;
  float *d_state = nullptr, *d_ring = nullptr;
  float *d_pcm = nullptr, *d_xbuf = nullptr, *d_ratio = nullptr;
  float *d_vad = nullptr, *d_wratio = nullptr, *d_wvad = nullptr, *d_band = nullptr, *d_den = nullptr;
  int *d_wflag = nullptr, *d_ticks = nullptr;
  // staged-mode intermediates
  float *d_xs = nullptr, *d_X = nullptr, *d_P = nullptr, *d_Ex = nullptr, *d_Ep = nullptr, *d_Exp = nullptr,
        *d_Lyf = nullptr, *d_f34 = nullptr, *d_rec = nullptr, *d_ptile = nullptr, *d_vadf = nullptr, *d_ys = nullptr;
  int *d_sil = nullptr, *d_pitch = nullptr, *d_wtick = nullptr;
  float *d_gr = nullptr, *d_gs = nullptr;
  int8_t *d_rnn_img = nullptr;
  uint16_t *d_gru16 = nullptr;  // FVAD_MODE_FP16: MFMA weight fragments (f16 bits)
  float *d_gru16_bias = nullptr;
  // device VADMachines (fvad_engine_attach_vadm)
  fvad::VadmArgs vadm{};
  // k_vadm_hbm runs on a side stream over copies of one push's window outputs,
  // overlapped with the next push (it only depends on its own state)
  hipStream_t side = nullptr;
  // staged mode: k_prep3 runs on pstream, so push k's prep overlaps push k-1's
  // kernels; xs / ratio / ticks are double-buffered (d_xs, d_ratio, d_ticks
  // alias the buffer of the latest push), buffer b is reused once the push that
  // used it last has finished (ev_buf_free[b])
  hipStream_t pstream = nullptr;
  // owners of pstream / side: engines of one GPU may share them
  // (fvad_engine_share_streams), the last one destroys the stream
  std::shared_ptr<ihipStream_t> pstream_ref, side_ref;
  float *d_xs_b[2] = {}, *d_ratio_b[2] = {}, *d_xlp_b[2] = {};
  int *d_ticks_b[2] = {};
  hipEvent_t ev_prep_done[2] = {}, ev_buf_free[2] = {};
  // the last push's k_fftAw done: push k's k_prep3 starts once push k-1's
  // k_fftAw has finished, so it runs beside k_plpc / k_pcorr instead (measured:
  // k_fftAw 0.64 -> 0.57, k_plpc 0.48 -> 0.40, k_pcorr 1.18 -> 1.24 ms, push
  // 5.00 -> 4.90 ms; started after k_plpc it overruns into k_rnn3: 5.93 ms)
  hipEvent_t ev_fft_a = nullptr;
  bool fft_a_rec = false;
  // push k's k_fftAw runs on pstream (after its k_prep3) once push k-1's
  // k_synthw, the last reader of what it writes, is done (ev_synth): beside
  // push k-1's k_olafb instead of after it (push 4.87 -> 4.78 ms)
  hipEvent_t ev_synth = nullptr;
  bool synth_rec = false;
  hipEvent_t synth_wait = nullptr;  // the last push's k_synthw-end event: ev_synth, or ev[10] in a timed push
  bool buf_busy[2] = {false, false};
  int next_buf = 0;
  int n_events = 0;           // timing events per launch
  int last_event = 0;         // the one recorded last (the launch's end)
  hipEvent_t ev_copy = nullptr, ev_vadm = nullptr, ev_vt[2][2] = {};  // [slot][begin/end] timing pairs
  // window outputs of push k in set k & 1 (the second set exists with VADMachines):
  // k_vadm_hbm of push k reads them in place, push k + 2 rewrites them after it
  int *wflag_b[2] = {};
  float *wratio_b[2] = {}, *wvad_b[2] = {}, *band_b[2] = {};
  hipEvent_t ev_vadm_b[2] = {};
  int32_t *d_vflag = nullptr, *d_vticks = nullptr, *d_vticks_b[2] = {};
  // The VADMachine of push k is enqueued when the next push is launched, as
  // k_vadm_hbm (32 waves, overlapping that push quietly: the 512-wave burst of
  // k_vadm_par beside the next push's k_fftAw cost more than it saved,
  // measured), or at a sync point with nothing else queued as k_vadm_par
  // (0.25 ms instead of 1.45: the drain of a job's last push).
  bool vpend = false, vpend_timed = false;
  int vpend_b = 0;
  fvad::StagedArgs vpend_args{};
  // a non-final k_vadm_hbm was queued last (its machines may owe their
  // long-term fold): a sync point with no push pending resolves it with a
  // resolve-only pass (vowed_args: that launch's argument block)
  bool vowed = false;
  fvad::StagedArgs vowed_args{};
  float *d_vwratio = nullptr, *d_vwvad = nullptr, *d_vband = nullptr;
  // VADMachine timing, by kernel: [0] k_vadm_hbm (steady state), [1] k_vadm_par
  // (a push flushed at a sync point); vadm_kind[slot]: the kernel a pending
  // event pair brackets
  double vadm_ms_sum[2] = {};
  int vadm_timed[2] = {};
  bool vadm_pending[2] = {false, false};
  int vadm_kind[2] = {};
  int vadm_slot = 0;
  bool dbg_always_par = false;  // test hook FVAD_DEBUG_VADM_ALWAYS_PAR
  bool dbg_lt_full = false;     // test hook FVAD_DEBUG_VADM_LT_FULL
  // test hook (fvad_engine_output_log): the per-tick outputs of the next
  // log_cap pushes, copied on the engine stream as each push ends
  float *d_log = nullptr;
  int log_cap = 0, log_n = 0;
  size_t log_stride = 0;
  std::vector<int> log_ticks;
  std::vector<fvad::VadmState> vadm_init;  // [m][stream] initial states
  size_t vadm_buf_len = 0;
  int rnn_act[fvad::rnnimg::kMats] = {};
  long long *d_wstart = nullptr;
  int V = 0, L = 0, LX = 0, wmax = 0, grid_frames = 0;
  int wpt = 1;  // window slots per (tick, stream): windows_per_tick(fft_size)
  // FFT B above kMaxFftB: tables [tw | sup | hann | perm] and k_fftb's scratch
  float *d_fbtab = nullptr;
  float2 *d_fbwork = nullptr;
  int fb_work_blocks = 0;
  long long fb_work_stride = 0;
  int resident_ticks = 0;
  int n_kernels = 0;
  bool olafb = false;  // staged: k_olafb in place of k_ola, k_winmeta, k_fftbw (kernel 8)
  // per-kernel timing events, two sets used alternately so the host reads
  // push k's events while push k+1 is already queued (no launch gap)
  hipEvent_t evs[2][FVAD_MAX_TIMES] = {};
  hipEvent_t *ev = evs[0];
  int ev_slot = 0;
  bool slot_pending[2] = {false, false};
  double ms_sum[FVAD_MAX_TIMES] = {};
  int n_timed = 0;
  int res_count = 0;  // run_resident calls since the last clear_times (event sampling)
  int raw_s16 = 0;  // rnnoise compat mode (s16-scaled I/O)
  unsigned long long *d_stamps = nullptr;
  unsigned *d_work = nullptr;  // staged: persistent-kernel group counters  // diagnostic stamp buffer (FVAD_STAMPS builds)
  // Device inputs alternate by push (d_pcm aliases the current one): the
  // input of push k+1 may be copied in while push k's k_prep3 still reads
  // its own.  ev_in_free[i]: buffer i's last reader (k_prep3 / k_prep) done.
  // run_resident reads d_pcm_b[0] (fvad_engine_load_synthetic).
  float *d_pcm_b[2] = {};
  // fvad_engine_load_synthetic_ex with n_pushes > 1: [push][tick][stream][ch][480]
  float *d_res = nullptr;
  int res_pushes = 0, res_next = 0;
  hipEvent_t ev_in_free[2] = {};
  bool in_busy[2] = {false, false};
  int in_next = 0;
  // Streaming ingest (fvad_engine_submit / collect): pinned host input slots
  // and output slots per in-flight push (kSlots = FVAD_MAX_IN_FLIGHT), H2D
  // copies on their own stream.  Allocated on first use.  With three pushes in
  // flight the H2D of push k + 2 waits only for its device input buffer, free
  // once push k's k_prep3 has read it -- not for push k's outputs.
  hipStream_t cstream = nullptr;
  struct Slot {
    float *in = nullptr;                 // pinned [max_ticks][B][C][480]
    int16_t *in16 = nullptr;             // pinned 16-bit input slot (fvad_engine_input_slot_i16; on first use)
    int32_t *ticks = nullptr;            // pinned [B]
    float *vad = nullptr, *ratio = nullptr, *wratio = nullptr, *wvad = nullptr, *band = nullptr, *den = nullptr;
    int32_t *wflag = nullptr;            // pinned outputs of the push that used this slot
    hipEvent_t h2d = nullptr, done = nullptr;
    bool h2d_busy = false, pending = false;
    int n_ticks = 0;
  } slots[FVAD_MAX_IN_FLIGHT];
  bool slots_ready = false;
  int sub_next = 0, col_next = 0;
  int16_t *d_pcm16 = nullptr;  // device staging of a 16-bit submit (converted into d_pcm by k_pcm16)
  // this push's input is 16-bit samples in d_pcm's buffer, read by k_prep3
  // itself (staged engines with the denoiser: no d_pcm16, no k_pcm16)
  bool pcm16_push = false;

};

// Diagnostic builds: per-phase cycle totals of k_frame (thread 0 of every workgroup).
extern "C" int fvad_engine_stamps(fvad_engine *e, unsigned long long *out, int n) {
  if (!e) return FVAD_EINVAL;
  if (!e->d_stamps) {
    HIP_TRY(hipMalloc(&e->d_stamps, 128 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(e->d_stamps, 0, 128 * sizeof(unsigned long long)));
    return FVAD_OK;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (out) HIP_TRY(hipMemcpy(out, e->d_stamps, std::min(n, 128) * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return FVAD_OK;
}

void fvad_engine_set_raw_s16(fvad_engine *e, int raw) { e->raw_s16 = raw; }

extern "C" void fvad_engine_config_default(fvad_engine_config *c, int n_streams, int n_channels) {
  std::memset(c, 0, sizeof(*c));
  c->n_streams = n_streams;
  c->n_channels = n_channels;
  c->device = 0;
  c->sample_rate = 48000;
  c->fft_size = 2048;
  c->max_ticks = 100;
  c->n_bands = 1;
  // VADMachine defaults: freqToBin(100) .. freqToBin(1500) at 48 kHz / 2048 (FFT.zig:120-131)
  c->band_lo[0] = 4;
  c->band_hi[0] = 64;
  c->want_denoised = 0;
  c->use_denoiser = 1;
}

namespace {

template <typename T>
int dalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), count * sizeof(T));
  if (e != hipSuccess) return fail(FVAD_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return FVAD_OK;
}

// int8 GRU-stack image for k_rnn3 (layout: fvad_internal.h rnnimg).  Term j of
// a column's C-order sum lives in segment g at seg_off(g) + (j - start of g).
void build_rnn_image(const fvad::HostModel &hm, std::vector<int8_t> &img, int *act) {
  namespace R = fvad::rnnimg;
  img.assign(R::kBytes, 0);
  const int8_t *b = hm.blob;
  auto put = [&](int m, int c, int j, int8_t v) {
    int g = 0, base = 0;
    while (j >= base + R::kSegs[m][g]) base += R::kSegs[m][g++];
    img[R::off_w(m) + c * R::stride(m) + R::seg_off(m, g) + (j - base)] = v;
  };
  auto dense = [&](int m, int l) {
    const fvad::HostLayer &L = hm.layers[l];
    for (int c = 0; c < L.nout; c++) {
      img[R::off_b(m) + c] = b[L.off_b + c];
      for (int j = 0; j < L.nin; j++) put(m, c, j, b[L.off_w + (size_t)j * L.nout + c]);
    }
    act[m] = L.act;
  };
  auto gru = [&](int mg, int mh, int l) {
    const fvad::HostLayer &L = hm.layers[l];
    const int N = L.nout, M = L.nin, S3 = 3 * N;
    for (int col = 0; col < S3; col++) {
      const int m = col < 2 * N ? mg : mh, c = col < 2 * N ? col : col - 2 * N;
      img[R::off_b(m) + c] = b[L.off_b + col];
      for (int j = 0; j < M; j++) put(m, c, j, b[L.off_w + (size_t)j * S3 + col]);
      for (int j = 0; j < N; j++) put(m, c, M + j, b[L.off_r + (size_t)j * S3 + col]);
    }
    act[mg] = fvad::kActSigmoid;
    act[mh] = L.act;
  };
  dense(0, 0);
  gru(1, 2, 1);
  gru(3, 4, 2);
  gru(5, 6, 3);
  dense(7, 4);
  dense(8, 5);
}

int upload_model(fvad_engine *e, const fvad::HostModel &hm) {
  std::vector<float> w(hm.blob_size);
  for (size_t i = 0; i < hm.blob_size; i++) w[i] = (float)hm.blob[i];
  int rc = dalloc(&e->d_weights, w.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpy(e->d_weights, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice));
  auto dense = [&](int l) {
    const fvad::HostLayer &L = hm.layers[l];
    fvad::DevDense d;
    d.nin = L.nin;
    d.nout = L.nout;
    d.act = L.act;
    d.w = e->d_weights + L.off_w;
    d.b = e->d_weights + L.off_b;
    return d;
  };
  auto gru = [&](int l) {
    const fvad::HostLayer &L = hm.layers[l];
    fvad::DevGru g;
    g.nin = L.nin;
    g.nout = L.nout;
    g.act = L.act;
    g.win = e->d_weights + L.off_w;
    g.wrec = e->d_weights + L.off_r;
    g.b = e->d_weights + L.off_b;
    return g;
  };
  for (int l = 0; l < 6; l++) {
    const fvad::HostLayer &L = hm.layers[l];
    const int m = l == 0 ? 0 : l == 1 ? 1 : l == 2 ? 3 : l == 3 ? 5 : l == 4 ? 7 : 8;
    if (L.nin != fvad::rnnimg::kKin[m] || (l >= 1 && l <= 3 ? 2 * L.nout : L.nout) != fvad::rnnimg::kCols[m])
      return fail(FVAD_EFORMAT, "model layer shapes differ from the rnnoise classic model");
  }
  {
    std::vector<int8_t> img;
    build_rnn_image(hm, img, e->rnn_act);
    rc = dalloc(&e->d_rnn_img, img.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(e->d_rnn_img, img.data(), img.size(), hipMemcpyHostToDevice));
    if (fp16_mode(e->cfg.mode)) {  // MFMA fragments of the same image (fvad_gru16.hip)
      std::vector<uint16_t> frags((size_t)fvad::gru16_frag_count() * 64 * 8);
      std::vector<float> bias(fvad::gru16_bias_rows());
      fvad::gru16_build(img.data(), frags.data(), bias.data());
      if ((rc = dalloc(&e->d_gru16, frags.size())) || (rc = dalloc(&e->d_gru16_bias, bias.size()))) return rc;
      HIP_TRY(hipMemcpy(e->d_gru16, frags.data(), frags.size() * 2, hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(e->d_gru16_bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    }
  }
  e->dmodel.in_dense = dense(0);
  e->dmodel.vad = gru(1);
  e->dmodel.noise = gru(2);
  e->dmodel.den = gru(3);
  e->dmodel.den_out = dense(4);
  e->dmodel.vad_out = dense(5);
  rc = dalloc(&e->d_model, 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(e->d_model, &e->dmodel, sizeof(fvad::DevModel), hipMemcpyHostToDevice));
  return FVAD_OK;
}

void free_all(fvad_engine *e) {
  void *ptrs[] = {e->d_plan, e->d_weights, e->d_state, e->d_ring, e->d_pcm_b[0], e->d_pcm_b[1], e->d_xbuf, e->d_ratio_b[0],
                  e->d_ratio_b[1], e->d_ticks_b[0], e->d_ticks_b[1], e->d_xs_b[0], e->d_xs_b[1], e->d_xlp_b[0], e->d_xlp_b[1],
                  e->d_vad,  e->wratio_b[0] ? e->wratio_b[0] : e->d_wratio,  e->wvad_b[0] ? e->wvad_b[0] : e->d_wvad,
                  e->band_b[0] ? e->band_b[0] : e->d_band, e->d_den,   e->wflag_b[0] ? e->wflag_b[0] : e->d_wflag,
                  e->d_model, e->d_stamps, e->d_X,    e->d_P,     e->d_Ex,    e->d_Ep,
                  e->d_Exp,  e->d_Lyf,     e->d_f34,   e->d_rec,  e->d_ptile, e->d_work, e->d_vadf,  e->d_ys,    e->d_sil,
                  e->d_pitch, e->d_wtick,  e->d_wstart, e->d_gr, e->d_gs, e->d_rnn_img, e->d_gru16, e->d_gru16_bias, e->vadm.st, e->vadm.buf,
                  e->vadm.seg, e->vadm.count, e->d_res, e->d_vflag, e->d_vticks, e->d_vticks_b[1], e->d_vwratio, e->d_vwvad, e->d_vband,
                  e->d_fbtab, e->d_fbwork, e->d_log};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  for (auto &set : e->evs)
    for (auto &ev : set)
      if (ev) (void)hipEventDestroy(ev);
  hipEvent_t evs[] = {e->ev_copy,     e->ev_vadm,     e->ev_vt[0][0],    e->ev_vt[0][1],
                      e->ev_vt[1][0], e->ev_vt[1][1], e->ev_vadm_b[0], e->ev_vadm_b[1]};
  for (hipEvent_t ev : evs)
    if (ev) (void)hipEventDestroy(ev);
  if (e->d_pcm16) (void)hipFree(e->d_pcm16);

  if (e->side && !e->side_ref) (void)hipStreamDestroy(e->side);  // created, not yet owned (a failed attach)
  if (e->pstream && !e->pstream_ref) (void)hipStreamDestroy(e->pstream);
  e->side_ref.reset();
  e->pstream_ref.reset();
  if (e->cstream) (void)hipStreamDestroy(e->cstream);
  for (auto &sl : e->slots) {
    void *hp[] = {sl.in, sl.in16, sl.ticks, sl.vad, sl.ratio, sl.wratio, sl.wvad, sl.band, sl.den, sl.wflag};
    for (void *q : hp)
      if (q) (void)hipHostFree(q);
    if (sl.h2d) (void)hipEventDestroy(sl.h2d);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  for (auto &ev : e->ev_in_free)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : e->ev_prep_done)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : e->ev_buf_free)
    if (ev) (void)hipEventDestroy(ev);
  if (e->ev_fft_a) (void)hipEventDestroy(e->ev_fft_a);
  if (e->ev_synth) (void)hipEventDestroy(e->ev_synth);
  if (e->stream) (void)hipStreamDestroy(e->stream);
}

}  // namespace

int vadm_reset(fvad_engine *e);
int vadm_flush(fvad_engine *e, bool fast);

extern "C" int fvad_engine_reset(fvad_engine *e) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (e->cstream) HIP_TRY(hipStreamSynchronize(e->cstream));
  if (e->pstream) HIP_TRY(hipStreamSynchronize(e->pstream));
  if (e->vadm.n > 0) {
    e->vpend = false;  // the pending push's machine state is wiped below: not run
    e->vowed = false;
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipStreamSynchronize(e->side));
    const int rc = vadm_reset(e);
    if (rc) return rc;
  }
  HIP_TRY(hipMemsetAsync(e->d_state, 0, sizeof(float) * fvad::st::kWords * (size_t)e->cfg.n_streams, e->stream));
  e->res_next = 0;  // fresh streams start at the resident cycle's first push (t = 0)
  if (e->d_work) HIP_TRY(hipMemsetAsync(e->d_work, 0, sizeof(unsigned) * fvad::kWorkCounters, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_ring, 0,
                         sizeof(float) * (size_t)e->ring_len * e->cfg.n_channels * e->cfg.n_streams, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return FVAD_OK;
}

namespace {
void fill_bands(const fvad_engine_config &c, int *band_lo, int *band_hi, int *lo_all, int *hi_all) {
  int lo = 1 << 30, hi = -1;
  for (int b = 0; b < fvad::kMaxBandCfg; b++) {
    band_lo[b] = b < c.n_bands ? c.band_lo[b] : 0;
    band_hi[b] = b < c.n_bands ? c.band_hi[b] : -1;
    if (b < c.n_bands) {
      lo = std::min(lo, c.band_lo[b]);
      hi = std::max(hi, c.band_hi[b]);
    }
  }
  *lo_all = lo;
  *hi_all = hi;
}

}  // namespace

namespace {
// an engine stream: non-blocking, so the synchronous null-stream copies of the
// setup calls never wait for queued pushes
hipError_t make_stream(hipStream_t *s) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking); }
void destroy_stream(ihipStream_t *s) { (void)hipStreamDestroy(s); }
}  // namespace

extern "C" int fvad_engine_create(const fvad_engine_config *cfg, const fvad_model *model, fvad_engine **out) {
  if (!cfg || !model || !out) return fail(FVAD_EINVAL, "null argument");
  const fvad_engine_config &c = *cfg;
  if (c.sample_rate != 48000) return fail(FVAD_ERATE, "only 48 kHz is supported (VAD.zig:101-104)");
  if (c.n_streams < 1 || c.n_channels < 1 || c.n_channels > FVAD_MAX_CHANNELS)
    return fail(FVAD_EINVAL, "n_streams >= 1 and 1 <= n_channels <= 8 required");
  // FFT.zig:29-31: any even, non-zero size.  fft_size < 480 completes several
  // windows per tick (VAD.zig:307-347; fvad_engine_windows_per_tick slots per
  // tick in the window outputs); kMaxFftSize keeps window indices in 32 bits
  if (c.fft_size < 2 || (c.fft_size & 1) || c.fft_size > fvad::kMaxFftSize)
    return fail(FVAD_EINVAL, "fft_size must be even, 2 <= fft_size <= 4194304 (FFT.zig:29-31)");
  if (c.mode == FVAD_MODE_FUSED) {
    int n = c.fft_size / 2;
    for (int p : {4, 2, 3, 5})
      while (n % p == 0) n /= p;
    if (n != 1 || c.fft_size > 2048 || c.fft_size < fvad::kFrame)
      return fail(FVAD_EINVAL, "fused mode: 480 <= fft_size <= 2048 with radices 2, 3, 4, 5 (use the staged mode)");
  }
  if (!c.use_denoiser && c.mode == FVAD_MODE_FUSED)
    return fail(FVAD_EINVAL, "use_denoiser = 0 runs on the staged engine");
  if (c.max_ticks < 1) return fail(FVAD_EINVAL, "max_ticks must be >= 1");
  if (c.n_bands < 1 || c.n_bands > FVAD_MAX_BANDS) return fail(FVAD_EINVAL, "1 <= n_bands <= 4");
  int lo = 1 << 30, hi = -1;
  for (int b = 0; b < c.n_bands; b++) {
    if (c.band_lo[b] < 0 || c.band_hi[b] < c.band_lo[b] || c.band_hi[b] > c.fft_size / 2)
      return fail(FVAD_EINVAL, "invalid band range");
    lo = std::min(lo, c.band_lo[b]);
    hi = std::max(hi, c.band_hi[b]);
  }
  if (hi - lo + 1 > 256 && (c.mode == FVAD_MODE_FUSED || c.fft_size == 2048))
    return fail(FVAD_EINVAL, "reported bins must span <= 256");
  if (c.mode != FVAD_MODE_STAGED && c.mode != FVAD_MODE_FUSED && !fp16_mode(c.mode))
    return fail(FVAD_EINVAL, "unknown engine mode");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(FVAD_EDEVICE, "no HIP device available");
  if (c.device < 0 || c.device >= ndev) return fail(FVAD_EDEVICE, "device ordinal out of range");

  fvad_engine *e = new fvad_engine();
  e->cfg = c;
  // the staged path writes every tick of a push before FFT B reads its
  // windows, so the ring holds one window plus a whole push
  // the re-block ring holds a window plus a push; a multiple of 4 so a
  // frame's float4 writes never straddle its end (k_ola, k_ndring)
  e->ring_len = (c.fft_size + c.max_ticks * fvad::kFrame + 3) & ~3;
  e->n_kernels = c.mode != FVAD_MODE_FUSED ? fvad::kStagedKernels : 2;
  if (c.mode != FVAD_MODE_FUSED && c.use_denoiser) {
    fvad::StagedArgs probe{};
    probe.nfft_b = c.fft_size;
    probe.n_channels = c.n_channels;
    e->olafb = fvad::olafb_fused(probe);
    if (e->olafb) e->n_kernels = fvad::kStagedKernels - 2;  // k_olafb's events span k_ola's pair
  }
  e->n_events = c.mode != FVAD_MODE_FUSED ? fvad::kStagedEvents : 3;
  e->last_event = c.mode != FVAD_MODE_FUSED ? fvad::kStagedLast : 2;
  static_assert(fvad::kStagedEvents <= FVAD_MAX_TIMES, "timing events");
  auto bail = [&](int rc) {
    free_all(e);
    delete e;
    return rc;
  };
  if (hipSetDevice(c.device) != hipSuccess) return bail(fail(FVAD_EDEVICE, "hipSetDevice failed"));
  if (make_stream(&e->stream) != hipSuccess) return bail(fail(FVAD_EDEVICE, "hipStreamCreate failed"));
  if (c.mode != FVAD_MODE_FUSED &&
      (make_stream(&e->pstream) != hipSuccess ||
       hipEventCreateWithFlags(&e->ev_prep_done[0], hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&e->ev_prep_done[1], hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&e->ev_buf_free[0], hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&e->ev_buf_free[1], hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&e->ev_fft_a, hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&e->ev_synth, hipEventDisableTiming) != hipSuccess))
    return bail(fail(FVAD_EDEVICE, "hipStreamCreate failed"));
  if (e->pstream) e->pstream_ref.reset(e->pstream, destroy_stream);
  for (int i = 0; i < e->n_events; i++)
    if (hipEventCreate(&e->evs[0][i]) != hipSuccess || hipEventCreate(&e->evs[1][i]) != hipSuccess)
      return bail(fail(FVAD_EDEVICE, "hipEventCreate failed"));
  fvad::Plan *plan = new fvad::Plan();
  fvad::build_plan(plan, c.fft_size);
  e->wpt = fvad::windows_per_tick(c.fft_size);
  int rc = FVAD_OK;
  if (c.fft_size > fvad::kMaxFftB) {  // FFT B's tables outside the plan: [tw | sup | hann | perm]
    const size_t n = c.fft_size;
    std::vector<float> tab(n + n / 2 + n + n / 2);
    int *perm = reinterpret_cast<int *>(tab.data() + n + n / 2 + n);
    plan->norm_b = fvad::build_fftb_tables(c.fft_size, plan->fac_b, tab.data(), tab.data() + n, perm,
                                           tab.data() + n + n / 2);
    rc = dalloc(&e->d_fbtab, tab.size());
    if (!rc && hipMemcpy(e->d_fbtab, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      rc = fail(FVAD_EDEVICE, "FFT-B table upload failed");
  }
  if (!rc) rc = dalloc(&e->d_plan, 1);
  if (!rc && hipMemcpy(e->d_plan, plan, sizeof(fvad::Plan), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(FVAD_EDEVICE, "plan upload failed");
  delete plan;
  if (rc) return bail(rc);
  if ((rc = upload_model(e, *fvad_model_host(model)))) return bail(rc);
  const size_t B = c.n_streams, C = c.n_channels, T = c.max_ticks;
  const size_t frames = T * B * C * fvad::kFrame;
  const size_t TBW = T * B * e->wpt;  // window slots
  if ((rc = dalloc(&e->d_state, B * fvad::st::kWords)) || (rc = dalloc(&e->d_ring, B * C * e->ring_len)) ||
      (rc = dalloc(&e->d_pcm_b[0], frames)) || (rc = dalloc(&e->d_pcm_b[1], frames)) ||
      (rc = dalloc(&e->d_ratio_b[0], T * B)) ||
      (rc = dalloc(&e->d_vad, T * B)) || (rc = dalloc(&e->d_wratio, TBW)) || (rc = dalloc(&e->d_wvad, TBW)) ||
      (rc = dalloc(&e->d_wflag, T * B)) || (rc = dalloc(&e->d_band, TBW * C * c.n_bands)) ||
      (rc = dalloc(&e->d_ticks_b[0], 2 * B)) || (c.want_denoised && (rc = dalloc(&e->d_den, frames))))
    return bail(rc);
  e->d_pcm = e->d_pcm_b[0];
  if (hipEventCreateWithFlags(&e->ev_in_free[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_in_free[1], hipEventDisableTiming) != hipSuccess)
    return bail(fail(FVAD_EDEVICE, "hipEventCreate failed"));
  e->d_ratio = e->d_ratio_b[0];
  e->d_ticks = e->d_ticks_b[0];
  e->wflag_b[0] = e->wflag_b[1] = e->d_wflag;
  e->wratio_b[0] = e->wratio_b[1] = e->d_wratio;
  e->wvad_b[0] = e->wvad_b[1] = e->d_wvad;
  e->band_b[0] = e->band_b[1] = e->d_band;
  if (c.mode == FVAD_MODE_FUSED) {
    if ((rc = dalloc(&e->d_xbuf, frames))) return bail(rc);
  } else {
    e->V = (int)(T * C);
    e->L = (fvad::kPitchBuf - fvad::kFrame) + e->V * fvad::kFrame;
    e->LX = e->L / 2;
    e->wmax = (int)(T * fvad::kFrame / c.fft_size) + 2;
    const size_t F = B * e->V;
    if ((rc = dalloc(&e->d_xs_b[0], B * e->L)) || (rc = dalloc(&e->d_xs_b[1], B * e->L)) ||
        (rc = dalloc(&e->d_xlp_b[0], B * e->LX)) || (rc = dalloc(&e->d_xlp_b[1], B * e->LX)) ||
        (rc = dalloc(&e->d_ratio_b[1], T * B)) || (rc = dalloc(&e->d_ticks_b[1], 2 * B)) || (rc = dalloc(&e->d_X, F * fvad::kFreq * 2)) ||
        (rc = dalloc(&e->d_P, F * fvad::kFreq * 2)) || (rc = dalloc(&e->d_Ex, F * fvad::kBands)) ||
        (rc = dalloc(&e->d_Ep, F * fvad::kBands)) || (rc = dalloc(&e->d_Exp, F * fvad::kBands)) ||
        (rc = dalloc(&e->d_Lyf, F * fvad::kBands)) || (rc = dalloc(&e->d_f34, F * 8)) ||
        (rc = dalloc(&e->d_rec, F * fvad::kPitchRecord)) || (rc = dalloc(&e->d_work, (size_t)fvad::kWorkCounters)) ||
        (rc = dalloc(&e->d_ptile, (B + fvad::ptile::kTile - 1) / fvad::ptile::kTile * e->V * fvad::ptile::kTile *
                                      fvad::ptile::kRows)) || (rc = dalloc(&e->d_vadf, F)) ||
        (rc = dalloc(&e->d_ys, F * fvad::kWin)) || (rc = dalloc(&e->d_sil, F)) || (rc = dalloc(&e->d_pitch, F)) ||
        (rc = dalloc(&e->d_wtick, B * e->wmax)) || (rc = dalloc(&e->d_wstart, B * e->wmax)) ||
        (rc = dalloc(&e->d_gr, F * fvad::kBands)) || (rc = dalloc(&e->d_gs, F * fvad::kBands)))
      return bail(rc);
    e->d_xs = e->d_xs_b[0];
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c.device) != hipSuccess) return bail(fail(FVAD_EDEVICE, "device query failed"));
    // CUs; persistent grids are sized per kernel
    e->grid_frames = prop.multiProcessorCount;
    // k_fftb's device scratch when a transform does not fit in LDS: a slice per
    // workgroup, at most two per CU and 1 GiB
    int lo = 0, hi = 0, band_lo[fvad::kMaxBandCfg], band_hi[fvad::kMaxBandCfg];
    fill_bands(c, band_lo, band_hi, &lo, &hi);
    e->fb_work_stride = fvad::fftb_work_stride(c.fft_size, lo, hi, fvad::fftb_generic(c.fft_size / 2));
    if (e->fb_work_stride > 0) {
      const long long per = e->fb_work_stride * (long long)sizeof(float2);
      const long long units = (long long)B * e->wmax;
      e->fb_work_blocks = (int)std::max<long long>(
          1, std::min<long long>({units, 2LL * e->grid_frames, (1LL << 30) / per}));
      if ((rc = dalloc(&e->d_fbwork, (size_t)e->fb_work_blocks * e->fb_work_stride))) return bail(rc);
    }
  }
  if ((rc = fvad_engine_reset(e))) return bail(rc);
  *out = e;
  return FVAD_OK;
}

extern "C" void fvad_engine_destroy(fvad_engine *e) {
  if (!e) return;
  (void)hipSetDevice(e->cfg.device);
  if (e->cstream) (void)hipStreamSynchronize(e->cstream);
  if (e->pstream) (void)hipStreamSynchronize(e->pstream);
  e->vpend = false;  // the last push's machine would only update state that is freed
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->side) (void)hipStreamSynchronize(e->side);
  free_all(e);
  delete e;
}

// e runs its k_prep3 (which & FVAD_SHARE_PREP) and / or its VADMachine
// kernels (which & FVAD_SHARE_SIDE) on other's streams from now on.  Both
// engines idle (synchronised here); every dependency stays an event, so
// sharing only adds order between the engines' side work.  An engine whose
// prep stream is shared runs k_fftAw on its own stream (launch_staged), so
// the main pipelines stay independent.
extern "C" int fvad_engine_share_streams(fvad_engine *e, fvad_engine *other, int which) {
  if (!e || !other || e == other || (which & ~(FVAD_SHARE_PREP | FVAD_SHARE_SIDE)) || !which)
    return fail(FVAD_EINVAL, "invalid argument");
  if (e->cfg.device != other->cfg.device) return fail(FVAD_EINVAL, "engines on different devices");
  if ((which & FVAD_SHARE_PREP) && (!e->pstream || !other->pstream))
    return fail(FVAD_EINVAL, "FVAD_SHARE_PREP needs two staged engines");
  if ((which & FVAD_SHARE_SIDE) && (!e->side || !other->side))
    return fail(FVAD_EINVAL, "FVAD_SHARE_SIDE needs device VADMachines attached to both engines");
  int rc;
  if ((rc = fvad_engine_sync(e)) || (rc = fvad_engine_sync(other))) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (which & FVAD_SHARE_PREP) {
    e->pstream_ref = other->pstream_ref;
    e->pstream = other->pstream;
  }
  if (which & FVAD_SHARE_SIDE) {
    e->side_ref = other->side_ref;
    e->side = other->side;
  }
  return FVAD_OK;
}

namespace {

int launch_fused(fvad_engine *e, int n_ticks, bool use_ticks, bool timed) {
  const fvad_engine_config &c = e->cfg;
  fvad::PrepArgs pa;
  pa.n_streams = c.n_streams;
  pa.n_channels = c.n_channels;
  pa.n_ticks = n_ticks;
  pa.ticks_valid = use_ticks ? e->d_ticks : nullptr;
  pa.pcm = e->d_pcm;
  pa.xbuf = e->d_xbuf;
  pa.ratio = e->d_ratio;
  pa.state = e->d_state;
  pa.raw_s16 = e->raw_s16;
  fvad::FrameArgs fa;
  fa.n_streams = c.n_streams;
  fa.n_channels = c.n_channels;
  fa.n_ticks = n_ticks;
  fa.ticks_valid = pa.ticks_valid;
  fa.xbuf = e->d_xbuf;
  fa.ratio = e->d_ratio;
  fa.state = e->d_state;
  fa.ring = e->d_ring;
  fa.ring_len = e->ring_len;
  fa.plan = e->d_plan;
  fa.model = e->d_model;
  fa.n_bands = c.n_bands;
  fill_bands(c, fa.band_lo, fa.band_hi, &fa.bin_lo_all, &fa.bin_hi_all);
  fa.out_vad = e->d_vad;
  fa.out_win_ratio = e->d_wratio;
  fa.out_win_vad = e->d_wvad;
  fa.out_band = e->d_band;
  fa.out_den = e->d_den;
  fa.out_win_flag = e->d_wflag;
  fa.raw_s16 = e->raw_s16;
  fa.stamps = e->d_stamps;
  if (timed) HIP_TRY(hipEventRecord(e->ev[0], e->stream));
  HIP_TRY(fvad::launch_prep(pa, e->stream));
  if (timed) HIP_TRY(hipEventRecord(e->ev[1], e->stream));
  HIP_TRY(fvad::launch_frame(fa, e->stream));
  if (timed) HIP_TRY(hipEventRecord(e->ev[2], e->stream));
  return FVAD_OK;
}

}  // namespace

// a cross-stream wait (skipping the ones already complete measured no gain:
// DESIGN §8 r4)
hipError_t wait_event(hipStream_t stream, hipEvent_t ev) { return hipStreamWaitEvent(stream, ev, 0); }

// k_vadm of one push on the side stream (its waits already queued), with
// its timing pair and the events later pushes wait for
int enqueue_vadm(fvad_engine *e, const fvad::StagedArgs &v, int b, bool timed, bool fast) {
  // k_vadm timing never blocks the host (it would serialise the overlap):
  // two event pairs alternate and are read once complete
  const int slot = e->vadm_slot ^= 1;
  if (timed) {
    e->vadm_pending[slot] = false;  // an unread older sample in this slot is dropped
    HIP_TRY(hipEventRecord(e->ev_vt[slot][0], e->side));
  }
  bool par = false;
  // a sync point's flush (or the test hook's every push) leaves every machine
  // exact; between sync points k_vadm_hbm may owe its long-term fold
  fvad::StagedArgs vf = v;
  vf.vadm.vfinal = (fast || e->dbg_always_par) ? 1 : 0;
  e->vowed = false;  // (a final pass resolves every machine, those without ticks included)
  HIP_TRY(fvad::launch_vadm(vf, e->side, fast || e->dbg_always_par, &par));
  if (!vf.vadm.vfinal) {
    e->vowed = true;
    e->vowed_args = vf;
  }
  if (timed) {
    HIP_TRY(hipEventRecord(e->ev_vt[slot][1], e->side));
    e->vadm_pending[slot] = true;
    e->vadm_kind[slot] = par ? 1 : 0;
  }
  HIP_TRY(hipEventRecord(e->ev_vadm, e->side));
  HIP_TRY(hipEventRecord(e->ev_vadm_b[b], e->side));
  return FVAD_OK;
}

// the last push's VADMachine, enqueued now (after its push's kernels);
// fast: nothing else is queued behind it (a sync point)
int vadm_flush(fvad_engine *e, bool fast = true) {
  if (!e->vpend) {
    if (fast && e->vowed) {
      // folds owed with no push pending (a push whose launch failed after
      // the previous push's non-final pass was queued): k_vadm_hbm with no
      // ticks and vfinal = 1 only resolves them
      fvad::StagedArgs r = e->vowed_args;
      r.n_ticks = 0;
      r.ticks_valid = nullptr;
      r.vadm = e->vadm;
      r.vadm.vfinal = 1;
      e->vowed = false;
      HIP_TRY(fvad::launch_vadm(r, e->side, false, nullptr));
      HIP_TRY(hipEventRecord(e->ev_vadm, e->side));
    }
    return FVAD_OK;
  }
  e->vpend = false;
  // the push's end: ev_buf_free of its parity (recorded after its kernels and
  // ticks copy; re-recorded only by the push after next)
  HIP_TRY(hipStreamWaitEvent(e->side, e->ev_buf_free[e->vpend_b], 0));
  // a flush at a sync point (k_vadm_par, the job's drain) is always timed:
  // its event pair sits on the side stream, after everything else
  return enqueue_vadm(e, e->vpend_args, e->vpend_b, e->vpend_timed || fast, fast);
}

namespace {

int launch_staged(fvad_engine *e, int n_ticks, bool use_ticks, bool use_tail, bool timed) {
  const fvad_engine_config &c = e->cfg;
  fvad::StagedArgs a{};
  a.n_streams = c.n_streams;
  a.n_channels = c.n_channels;
  a.n_ticks = n_ticks;
  a.V = e->V;
  a.L = e->L;
  // the previous push's VADMachine (after that push's ev_buf_free)
  if (e->vpend)
    if (const int rf = vadm_flush(e, false)) return rf;
  // push k uses buffer b = k & 1 of xs / ratio / ticks; its k_prep3 waits
  // (on pstream) until push k-2 released b, then runs beside push k-1
  const int b = e->next_buf;
  if (e->buf_busy[b]) HIP_TRY(wait_event(e->pstream, e->ev_buf_free[b]));
  if (e->fft_a_rec) HIP_TRY(wait_event(e->pstream, e->ev_fft_a));
  e->d_xs = e->d_xs_b[b];
  e->d_ratio = e->d_ratio_b[b];
  e->d_ticks = e->d_ticks_b[b];
  e->d_wflag = e->wflag_b[b];
  e->d_wratio = e->wratio_b[b];
  e->d_wvad = e->wvad_b[b];
  e->d_band = e->band_b[b];
  a.ticks_valid = use_ticks ? e->d_ticks : nullptr;
  a.tail = use_tail ? e->d_ticks + c.n_streams : nullptr;  // [B..2B) of the ticks buffer
  a.pcm = e->d_pcm;
  a.pcm16 = e->pcm16_push ? reinterpret_cast<const int16_t *>(e->d_pcm) : nullptr;
  a.xs = e->d_xs;
  a.xlp = e->d_xlp_b[b];
  a.LX = e->LX;
  a.ratio = e->d_ratio;
  a.state = e->d_state;
  a.X = reinterpret_cast<float2 *>(e->d_X);
  a.P = reinterpret_cast<float2 *>(e->d_P);
  a.Ex = e->d_Ex;
  a.Ep = e->d_Ep;
  a.Exp = e->d_Exp;
  a.Lyf = e->d_Lyf;
  a.f34 = e->d_f34;
  a.silence = e->d_sil;
  a.rec = e->d_rec;
  a.ptile = e->d_ptile;
  a.work = e->d_work;
  a.pitch = e->d_pitch;
  a.vadf = e->d_vadf;
  a.gr = e->d_gr;
  a.gs = e->d_gs;
  a.rnn_img = e->d_rnn_img;
  a.gru16_frags = e->d_gru16;
  a.gru16_bias = e->d_gru16_bias;
  a.fuse16 = e->cfg.mode == FVAD_MODE_FP16_FUSED;
  for (int m = 0; m < fvad::rnnimg::kMats; m++) a.rnn_act[m] = e->rnn_act[m];
  a.ys = e->d_ys;
  a.ring = e->d_ring;
  a.ring_len = e->ring_len;
  a.win_tick = e->d_wtick;
  a.win_start = e->d_wstart;
  a.wmax = e->wmax;
  a.wpt = e->wpt;
  if (e->d_fbtab) {  // fft_size > kMaxFftB: [tw | sup | hann | perm] (fvad_engine_create)
    const size_t n = c.fft_size;
    a.fb_tw = reinterpret_cast<const float2 *>(e->d_fbtab);
    a.fb_sup = reinterpret_cast<const float2 *>(e->d_fbtab + n);
    a.fb_hann = e->d_fbtab + n + n / 2;
    a.fb_perm = reinterpret_cast<const int *>(e->d_fbtab + n + n / 2 + n);
  } else {  // the plan's own tables (device addresses inside d_plan)
    const char *pb = reinterpret_cast<const char *>(e->d_plan);
    a.fb_tw = reinterpret_cast<const float2 *>(pb + offsetof(fvad::Plan, twb));
    a.fb_sup = reinterpret_cast<const float2 *>(pb + offsetof(fvad::Plan, superb));
    a.fb_hann = reinterpret_cast<const float *>(pb + offsetof(fvad::Plan, hannb));
    a.fb_perm = reinterpret_cast<const int *>(pb + offsetof(fvad::Plan, permb));
  }
  a.fb_work = e->d_fbwork;
  a.fb_work_blocks = e->fb_work_blocks;
  a.fb_work_stride = e->fb_work_stride;
  a.plan = e->d_plan;
  a.model = e->d_model;
  a.n_bands = c.n_bands;
  fill_bands(c, a.band_lo, a.band_hi, &a.bin_lo_all, &a.bin_hi_all);
  a.nfft_b = c.fft_size;
  a.use_denoiser = c.use_denoiser;
  a.out_vad = e->d_vad;
  a.out_win_ratio = e->d_wratio;
  a.out_win_vad = e->d_wvad;
  a.out_band = e->d_band;
  a.out_den = e->d_den;
  a.out_win_flag = e->d_wflag;
  a.raw_s16 = e->raw_s16;
  a.vadm = e->vadm;
  a.stamps = e->d_stamps;
  if (c.use_denoiser) {
    HIP_TRY(fvad::launch_prep(a, e->pstream, timed ? e->ev : nullptr));
    HIP_TRY(hipEventRecord(e->ev_prep_done[b], e->pstream));
    HIP_TRY(wait_event(e->stream, e->ev_prep_done[b]));
    // window output set b is free once push k-2's k_vadm_hbm has read it
    if (e->vadm.n > 0) HIP_TRY(wait_event(e->stream, e->ev_vadm_b[b]));
    // k_fftAw runs on the prep stream only while this engine owns it: on a
    // shared one (FVAD_SHARE_PREP) it would queue behind the other engine's
    // waits and couple the two pipelines, so it stays on the engine stream
    const bool own_prep = e->pstream_ref.use_count() <= 1;
    HIP_TRY(fvad::launch_staged(a, e->grid_frames, e->stream, timed ? e->ev : nullptr, e->ev_fft_a,
                                own_prep ? e->pstream : nullptr, e->synth_rec ? e->synth_wait : nullptr,
                                e->ev_synth));
    e->synth_wait = timed ? e->ev[10] : e->ev_synth;  // (launch_staged records ev[10] in its place when timed)
    e->synth_rec = true;
    e->fft_a_rec = true;
  } else {
    // no denoiser: raw input frames to the ring, windows, FFT B, all on the
    // engine stream after the input copy (queued on the prep stream)
    HIP_TRY(hipEventRecord(e->ev_prep_done[b], e->pstream));
    HIP_TRY(wait_event(e->stream, e->ev_prep_done[b]));
    if (e->vadm.n > 0) HIP_TRY(wait_event(e->stream, e->ev_vadm_b[b]));
    HIP_TRY(fvad::launch_nodenoise(a, e->grid_frames, e->stream));
  }
  if (e->vadm.n > 0) {
    // the ticks copy of parity b may be overwritten once push k - 2's
    // VADMachine has read it (ev_vadm_b[b], waited for above)
    if (use_ticks)
      HIP_TRY(hipMemcpyAsync(e->d_vticks_b[b], e->d_ticks, (size_t)c.n_streams * 4, hipMemcpyDeviceToDevice, e->stream));
    fvad::StagedArgs v = a;
    v.ticks_valid = use_ticks ? e->d_vticks_b[b] : nullptr;
    e->vpend = true;
    e->vpend_args = v;
    e->vpend_b = b;
    e->vpend_timed = timed;
  }
  if (e->log_n < e->log_cap) {  // test hook: this push's outputs into the log (read after a sync)
    const size_t B = c.n_streams, TB = (size_t)n_ticks * B, TBW = TB * e->wpt, MT = (size_t)c.max_ticks * B,
                 MW = MT * e->wpt;
    float *L = e->d_log + e->log_stride * (size_t)e->log_n;
    const void *src[6] = {e->d_vad, e->d_ratio, e->d_wflag, e->d_wratio, e->d_wvad, e->d_band};
    const size_t off[6] = {0, MT, 2 * MT, 3 * MT, 3 * MT + MW, 3 * MT + 2 * MW};
    const size_t n[6] = {TB, TB, TB, TBW, TBW, TBW * c.n_channels * c.n_bands};
    for (int i = 0; i < 6; i++)
      HIP_TRY(hipMemcpyAsync(L + off[i], src[i], n[i] * 4, hipMemcpyDeviceToDevice, e->stream));
    e->log_ticks[e->log_n++] = n_ticks;
  }
  // every reader of buffer b (incl. the copy of ticks for k_vadm_hbm) is queued
  HIP_TRY(hipEventRecord(e->ev_buf_free[b], e->stream));
  e->buf_busy[b] = true;
  e->next_buf = b ^ 1;
  return FVAD_OK;
}

int launch(fvad_engine *e, int n_ticks, bool use_ticks, bool timed, bool use_tail = false) {
  if (!e->cfg.use_denoiser) timed = false;  // the no-denoiser pipeline records no kernel events
  const int rc = e->cfg.mode == FVAD_MODE_FUSED ? launch_fused(e, n_ticks, use_ticks, timed)
                                                 : launch_staged(e, n_ticks, use_ticks, use_tail, timed);
  if (!rc && timed) e->slot_pending[e->ev_slot] = true;
  return rc;
}

int collect_slot(fvad_engine *e, int slot) {
  if (!e->slot_pending[slot]) return FVAD_OK;
  hipEvent_t *ev = e->evs[slot];
  const bool staged = e->cfg.mode != FVAD_MODE_FUSED;
  HIP_TRY(hipEventSynchronize(ev[e->last_event]));
  for (int i = 0; i < e->n_kernels; i++) {
    float ms = 0;
    const int b = staged ? fvad::kStagedTime[i][0] : i, en = staged ? fvad::kStagedTime[i][1] : i + 1;
    HIP_TRY(hipEventElapsedTime(&ms, ev[b], ev[en]));
    e->ms_sum[1 + i] += ms;
  }
  float total = 0;  // GPU time of the launch (kernels may overlap)
  HIP_TRY(hipEventElapsedTime(&total, ev[0], ev[e->last_event]));
  e->ms_sum[0] += total;
  e->n_timed++;
  e->slot_pending[slot] = false;
  return FVAD_OK;
}

int collect_timing(fvad_engine *e) {
  int rc = collect_slot(e, e->ev_slot ^ 1);
  if (!rc) rc = collect_slot(e, e->ev_slot);
  return rc;
}

// VADMachine samples whose end event has completed (non-blocking), by kernel
int collect_vadm_timing(fvad_engine *e) {
  for (int k = 0; k < 2; k++) {
    if (!e->vadm_pending[k] || hipEventQuery(e->ev_vt[k][1]) != hipSuccess) continue;
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e->ev_vt[k][0], e->ev_vt[k][1]));
    e->vadm_ms_sum[e->vadm_kind[k]] += ms;
    e->vadm_timed[e->vadm_kind[k]]++;
    e->vadm_pending[k] = false;
  }
  return FVAD_OK;
}

int fetch(fvad_engine *e, int n_ticks, fvad_outputs *o) {
  if (!o) return FVAD_OK;
  const fvad_engine_config &c = e->cfg;
  const size_t TB = (size_t)n_ticks * c.n_streams, TBW = TB * e->wpt;
  auto cp = [&](void *dst, const void *src, size_t bytes) -> int {
    if (!dst) return FVAD_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream));
    return FVAD_OK;
  };
  int rc;
  if ((rc = cp(o->vad, e->d_vad, TB * 4)) || (rc = cp(o->ratio, e->d_ratio, TB * 4)) ||
      (rc = cp(o->win_flag, e->d_wflag, TB * 4)) || (rc = cp(o->win_ratio, e->d_wratio, TBW * 4)) ||
      (rc = cp(o->win_vad, e->d_wvad, TBW * 4)) || (rc = cp(o->band, e->d_band, TBW * c.n_channels * c.n_bands * 4)))
    return rc;
  if (o->denoised) {
    if (!e->d_den) return fail(FVAD_EINVAL, "engine created without want_denoised");
    if ((rc = cp(o->denoised, e->d_den, TB * c.n_channels * fvad::kFrame * 4))) return rc;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  return FVAD_OK;
}

}  // namespace

namespace {

// the stream whose kernel reads the device input: k_prep3 on the prep stream
// (staged), k_prep / k_ndring on the engine stream (fused, no denoiser)
hipStream_t input_reader(const fvad_engine *e) {
  return (e->cfg.mode != FVAD_MODE_FUSED && e->cfg.use_denoiser) ? e->pstream : e->stream;
}

// the input of the push about to launch goes to device buffer in_next; its
// previous reader (the k_prep3 of the push two before) must be done
int input_buffer(fvad_engine *e, hipStream_t cs) {
  const int ib = e->in_next;
  if (e->in_busy[ib]) HIP_TRY(hipStreamWaitEvent(cs, e->ev_in_free[ib], 0));
  e->d_pcm = e->d_pcm_b[ib];
  return FVAD_OK;
}

// after the launch: the buffer is free again once this push's prep read it
int release_input(fvad_engine *e) {
  const int ib = e->in_next;
  HIP_TRY(hipEventRecord(e->ev_in_free[ib], input_reader(e)));
  e->in_busy[ib] = true;
  e->in_next = ib ^ 1;
  e->resident_ticks = 0;
  return FVAD_OK;
}

int check_ticks(const fvad_engine *e, const int32_t *ticks_valid, int n_ticks) {
  if (ticks_valid)
    for (int s = 0; s < e->cfg.n_streams; s++)
      if (ticks_valid[s] < 0 || ticks_valid[s] > n_ticks) return fail(FVAD_EINVAL, "ticks_valid out of range");
  return FVAD_OK;
}

// last_tick_samples (nullable): real samples in each stream's last valid tick.
// Only the no-denoiser path consumes a partial tick (it reads fft_size frames,
// VAD.zig:206-220); with the denoiser a frame needs all 480 samples.  Fills
// tt = [ticks_valid (n_ticks where NULL) | tails] when tails are in use.
int tail_ticks(const fvad_engine *e, const int32_t *ticks_valid, const int32_t *last, int n_ticks,
               std::vector<int32_t> &tt) {
  tt.clear();
  if (!last) return FVAD_OK;
  const int B = e->cfg.n_streams;
  bool partial = false;
  for (int s = 0; s < B; s++) {
    if (last[s] < 1 || last[s] > fvad::kFrame) return fail(FVAD_EINVAL, "last_tick_samples out of range [1, 480]");
    partial |= last[s] != fvad::kFrame;
  }
  if (!partial) return FVAD_OK;
  if (e->cfg.use_denoiser || e->cfg.mode == FVAD_MODE_FUSED)
    return fail(FVAD_EINVAL, "a partial tick is only consumed with use_denoiser = 0 (VAD.zig:206-220)");
  tt.resize(2 * (size_t)B);
  for (int s = 0; s < B; s++) {
    tt[s] = ticks_valid ? ticks_valid[s] : n_ticks;
    tt[B + s] = last[s];
  }
  return FVAD_OK;
}

// host copy into a pinned slot, split over threads for large inputs
void par_copy(void *dst, const void *src, size_t bytes) {
  constexpr size_t kChunk = 8u << 20;
  unsigned nthr = std::thread::hardware_concurrency();
  nthr = std::max(1u, std::min(nthr, 16u));
  const size_t parts = std::min<size_t>(nthr, (bytes + kChunk - 1) / kChunk);
  if (parts <= 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> pool;
  for (size_t i = 0; i < parts; i++) {
    const size_t a = bytes * i / parts, b = bytes * (i + 1) / parts;
    pool.emplace_back([=]() { std::memcpy((char *)dst + a, (const char *)src + a, b - a); });
  }
  for (auto &t : pool) t.join();
}

// The copy stream, and slot i's pinned buffers on first use: a caller that
// keeps k pushes in flight pins k slots, not FVAD_MAX_IN_FLIGHT
int ensure_slots(fvad_engine *e, int i) {
  const fvad_engine_config &c = e->cfg;
  const size_t B = c.n_streams, C = c.n_channels, T = c.max_ticks;
  const size_t TB = T * B, TBW = TB * e->wpt, frames = TB * C * fvad::kFrame;
  {
    // a streaming slot pins one push of input and outputs (fvad_engine_submit,
    // up to FVAD_MAX_IN_FLIGHT of them); the window outputs grow with W =
    // windows_per_tick (up to 240 at fft_size 2): refuse configurations whose
    // slot would not be a sane pinned allocation (the streaming API only:
    // resident and push-from-host engines never allocate a slot)
    const double slot = 4.0 * ((double)frames * (c.want_denoised ? 2 : 1) + 3.0 * TB + 2.0 * TBW +
                               (double)TBW * C * c.n_bands);
    if (slot > 16.0 * (1ull << 30))
      return fail(FVAD_ENOMEM, "a push of max_ticks x n_streams needs > 16 GiB of pinned slot memory "
                               "(outputs scale with windows_per_tick): lower max_ticks or n_streams");
  }
  if (!e->slots_ready) {
    // the copy stream at the highest priority: its own hardware queue, so the
    // 16-bit ingest's k_pcm16 does not queue behind a long kernel of a stream
    // sharing its queue (it waited for k_vadm_hbm at the default priority)
    int lo_prio = 0, hi_prio = 0;
    if (!e->cstream && (hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) != hipSuccess ||
                        hipStreamCreateWithPriority(&e->cstream, hipStreamNonBlocking, hi_prio) != hipSuccess))
      return fail(FVAD_EDEVICE, "copy stream creation failed");
    e->slots_ready = true;
  }
  auto &sl = e->slots[i];
  if (sl.done) return FVAD_OK;  // allocated (the events come last)
  auto host = [&](auto **p, size_t count) -> int {
    if (*p) return FVAD_OK;  // kept from an earlier, partly failed call
    if (hipHostMalloc(reinterpret_cast<void **>(p), std::max<size_t>(count, 1) * 4, 0) != hipSuccess) {
      *p = nullptr;
      return fail(FVAD_ENOMEM, "hipHostMalloc failed (pinned input / output slots)");
    }
    return FVAD_OK;
  };
  int rc;
  if ((rc = host(&sl.in, frames)) || (rc = host(&sl.ticks, 2 * B)) || (rc = host(&sl.vad, TB)) ||
      (rc = host(&sl.ratio, TB)) || (rc = host(&sl.wflag, TB)) || (rc = host(&sl.wratio, TBW)) ||
      (rc = host(&sl.wvad, TBW)) || (rc = host(&sl.band, TBW * C * c.n_bands)) ||
      (c.want_denoised && (rc = host(&sl.den, frames))))
    return rc;
  if ((!sl.h2d && hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming) != hipSuccess) ||
      hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) {
    sl.done = nullptr;
    return fail(FVAD_EDEVICE, "hipEventCreate failed");
  }
  return FVAD_OK;
}

// slot i's pinned 16-bit input and the device staging buffer, on first use
int ensure_slots16(fvad_engine *e, int i) {
  const fvad_engine_config &c = e->cfg;
  const size_t n = (size_t)c.max_ticks * c.n_streams * c.n_channels * fvad::kFrame;
  auto &sl = e->slots[i];
  if (!sl.in16 && hipHostMalloc(reinterpret_cast<void **>(&sl.in16), n * sizeof(int16_t), 0) != hipSuccess) {
    sl.in16 = nullptr;
    return fail(FVAD_ENOMEM, "hipHostMalloc failed (16-bit input slot)");
  }
  if (!e->d_pcm16 && hipMalloc(reinterpret_cast<void **>(&e->d_pcm16), n * sizeof(int16_t)) != hipSuccess) {
    e->d_pcm16 = nullptr;
    return fail(FVAD_ENOMEM, "hipMalloc failed (16-bit input staging)");
  }
  return FVAD_OK;
}

}  // namespace

extern "C" int fvad_engine_push(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid,
                                fvad_outputs *out) {
  return fvad_engine_push_ex(e, pcm, n_ticks, ticks_valid, nullptr, out);
}

extern "C" int fvad_engine_push_ex(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid,
                                   const int32_t *last_tick_samples, fvad_outputs *out) {
  if (!e || !pcm) return fail(FVAD_EINVAL, "null argument");
  const fvad_engine_config &c = e->cfg;
  if (n_ticks < 0 || n_ticks > c.max_ticks) return fail(FVAD_EINVAL, "n_ticks out of range [0, max_ticks]");
  if (n_ticks == 0) return FVAD_OK;
  int rc = check_ticks(e, ticks_valid, n_ticks);
  if (rc) return rc;
  std::vector<int32_t> tt;
  if ((rc = tail_ticks(e, ticks_valid, last_tick_samples, n_ticks, tt))) return rc;
  HIP_TRY(hipSetDevice(c.device));
  const size_t bytes = (size_t)n_ticks * c.n_streams * c.n_channels * fvad::kFrame * sizeof(float);
  // staged: the inputs go through the prep stream (ticks buffer b is free
  // once push k-2 finished)
  hipStream_t cs = e->stream;
  int *dticks = e->d_ticks;
  if (e->cfg.mode != FVAD_MODE_FUSED) {
    const int b = e->next_buf;
    if (e->buf_busy[b]) HIP_TRY(hipStreamWaitEvent(e->pstream, e->ev_buf_free[b], 0));
    cs = e->pstream;
    dticks = e->d_ticks_b[b];
  }
  if ((rc = input_buffer(e, cs))) return rc;
  HIP_TRY(hipMemcpyAsync(e->d_pcm, pcm, bytes, hipMemcpyHostToDevice, cs));
  if (!tt.empty()) {  // ticks and tails, [2 * B] (synchronous copy: tt is a local)
    HIP_TRY(hipMemcpyAsync(dticks, tt.data(), sizeof(int32_t) * tt.size(), hipMemcpyHostToDevice, cs));
    HIP_TRY(hipStreamSynchronize(cs));
  } else if (ticks_valid) {
    HIP_TRY(hipMemcpyAsync(dticks, ticks_valid, sizeof(int32_t) * c.n_streams, hipMemcpyHostToDevice, cs));
  }
  if ((rc = launch(e, n_ticks, ticks_valid != nullptr || !tt.empty(), false, !tt.empty()))) return rc;
  if ((rc = release_input(e))) return rc;
  return fetch(e, n_ticks, out);
}

extern "C" float *fvad_engine_input_slot(fvad_engine *e) {
  if (!e) {
    fail(FVAD_EINVAL, "null engine");
    return nullptr;
  }
  if (hipSetDevice(e->cfg.device) != hipSuccess || ensure_slots(e, e->sub_next)) return nullptr;
  auto &sl = e->slots[e->sub_next];
  if (sl.h2d_busy) {
    if (hipEventSynchronize(sl.h2d) != hipSuccess) {
      fail(FVAD_EDEVICE, "hipEventSynchronize failed");
      return nullptr;
    }
    sl.h2d_busy = false;
  }
  return sl.in;
}

extern "C" int fvad_engine_submit(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid) {
  return fvad_engine_submit_ex(e, pcm, n_ticks, ticks_valid, nullptr);
}

namespace {

// fvad_engine_submit_ex / fvad_engine_submit_i16: pcm is float or int16_t
// (16-bit samples k, pushed as k / 32768.0f -- libsndfile's short -> float
// normalisation, exact in f32: half the host-to-device bytes, converted by
// k_pcm16 on the copy stream right after the copy)
template <typename Sample>
int submit_any(fvad_engine *e, const Sample *pcm, int n_ticks, const int32_t *ticks_valid,
               const int32_t *last_tick_samples) {
  constexpr bool k16 = sizeof(Sample) == 2;
  if (!e || !pcm) return fail(FVAD_EINVAL, "null argument");
  const fvad_engine_config &c = e->cfg;
  if (n_ticks < 1 || n_ticks > c.max_ticks) return fail(FVAD_EINVAL, "n_ticks out of range [1, max_ticks]");
  int rc = check_ticks(e, ticks_valid, n_ticks);
  if (rc) return rc;
  std::vector<int32_t> tt;
  if ((rc = tail_ticks(e, ticks_valid, last_tick_samples, n_ticks, tt))) return rc;
  HIP_TRY(hipSetDevice(c.device));
  const int si = e->sub_next;
  if ((rc = ensure_slots(e, si))) return rc;
  if constexpr (k16)
    if ((rc = ensure_slots16(e, si))) return rc;
  auto &sl = e->slots[si];
  if (sl.pending) return fail(FVAD_EINVAL, "FVAD_MAX_IN_FLIGHT pushes in flight: collect the oldest one first");
  const size_t B = c.n_streams, TB = (size_t)n_ticks * B, TBW = TB * e->wpt;
  const size_t n_samples = TB * c.n_channels * fvad::kFrame, bytes = n_samples * sizeof(float);
  Sample *slot_in;
  if constexpr (k16)
    slot_in = sl.in16;
  else
    slot_in = sl.in;
  if (pcm != slot_in) {  // otherwise the producer wrote into the slot (fvad_engine_input_slot[_i16])
    if (sl.h2d_busy) HIP_TRY(hipEventSynchronize(sl.h2d));
    par_copy(slot_in, pcm, n_samples * sizeof(Sample));
  }
  if (!tt.empty())
    std::memcpy(sl.ticks, tt.data(), tt.size() * sizeof(int32_t));
  else if (ticks_valid)
    std::memcpy(sl.ticks, ticks_valid, B * sizeof(int32_t));
  const bool use_ticks = ticks_valid != nullptr || !tt.empty();
  // staged: copies on the copy stream, overlapping the previous push's
  // kernels; the prep stream waits for them.  Fused: everything in order on
  // the engine stream (its kernels read d_ticks in place).
  const bool staged = c.mode != FVAD_MODE_FUSED;
  hipStream_t cs = staged ? e->cstream : e->stream;
  if ((rc = input_buffer(e, cs))) return rc;
  // staged with the denoiser: k_prep3 reads the 16-bit samples straight from
  // the input buffer (half its input bytes; the copy stream carries only the
  // H2D copy, and no conversion kernel takes a slot beside the pushes)
  const bool direct16 = k16 && staged && c.use_denoiser && !e->raw_s16;
  if constexpr (k16) {
    if (direct16) {
      HIP_TRY(hipMemcpyAsync(e->d_pcm, sl.in16, n_samples * sizeof(int16_t), hipMemcpyHostToDevice, cs));
    } else {
      // d_pcm16 is overwritten by the next 16-bit submit only after this
      // conversion read it (both on cs, in order)
      HIP_TRY(hipMemcpyAsync(e->d_pcm16, sl.in16, n_samples * sizeof(int16_t), hipMemcpyHostToDevice, cs));
      HIP_TRY(fvad::launch_pcm16(e->d_pcm16, e->d_pcm, n_samples, cs));
    }
  } else {
    HIP_TRY(hipMemcpyAsync(e->d_pcm, sl.in, bytes, hipMemcpyHostToDevice, cs));
  }
  if (use_ticks) {
    int *dticks = e->d_ticks;
    if (staged) {
      const int b = e->next_buf;
      if (e->buf_busy[b]) HIP_TRY(hipStreamWaitEvent(cs, e->ev_buf_free[b], 0));
      dticks = e->d_ticks_b[b];
    }
    HIP_TRY(hipMemcpyAsync(dticks, sl.ticks, (tt.empty() ? B : 2 * B) * sizeof(int32_t), hipMemcpyHostToDevice, cs));
  }
  HIP_TRY(hipEventRecord(sl.h2d, cs));
  sl.h2d_busy = true;
  if (staged) HIP_TRY(hipStreamWaitEvent(e->pstream, sl.h2d, 0));
  e->pcm16_push = direct16;
  rc = launch(e, n_ticks, use_ticks, false, !tt.empty());
  e->pcm16_push = false;
  if (rc) return rc;
  if ((rc = release_input(e))) return rc;
  // outputs into the slot's pinned buffers, after the kernels on the engine
  // stream (the next push's kernels queue behind these copies)
  auto d2h = [&](void *dst, const void *src, size_t n) -> int {
    HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, e->stream));
    return FVAD_OK;
  };
  if ((rc = d2h(sl.vad, e->d_vad, TB * 4)) || (rc = d2h(sl.ratio, e->d_ratio, TB * 4)) ||
      (rc = d2h(sl.wflag, e->d_wflag, TB * 4)) || (rc = d2h(sl.wratio, e->d_wratio, TBW * 4)) ||
      (rc = d2h(sl.wvad, e->d_wvad, TBW * 4)) || (rc = d2h(sl.band, e->d_band, TBW * c.n_channels * c.n_bands * 4)) ||
      (c.want_denoised && (rc = d2h(sl.den, e->d_den, bytes))))
    return rc;
  HIP_TRY(hipEventRecord(sl.done, e->stream));
  sl.pending = true;
  sl.n_ticks = n_ticks;
  e->sub_next = (si + 1) % FVAD_MAX_IN_FLIGHT;
  return FVAD_OK;
}

}  // namespace

extern "C" int fvad_engine_submit_ex(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid,
                                     const int32_t *last_tick_samples) {
  return submit_any(e, pcm, n_ticks, ticks_valid, last_tick_samples);
}

extern "C" int16_t *fvad_engine_input_slot_i16(fvad_engine *e) {
  if (!e) {
    fail(FVAD_EINVAL, "null engine");
    return nullptr;
  }
  if (hipSetDevice(e->cfg.device) != hipSuccess || ensure_slots(e, e->sub_next) || ensure_slots16(e, e->sub_next))
    return nullptr;
  auto &sl = e->slots[e->sub_next];
  if (sl.h2d_busy) {
    if (hipEventSynchronize(sl.h2d) != hipSuccess) {
      fail(FVAD_EDEVICE, "hipEventSynchronize failed");
      return nullptr;
    }
    sl.h2d_busy = false;
  }
  return sl.in16;
}

extern "C" int fvad_engine_submit_i16(fvad_engine *e, const int16_t *pcm, int n_ticks, const int32_t *ticks_valid,
                                      const int32_t *last_tick_samples) {
  return submit_any(e, pcm, n_ticks, ticks_valid, last_tick_samples);
}

extern "C" int fvad_engine_collect(fvad_engine *e, fvad_outputs *out, int *n_ticks) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  auto &sl = e->slots[e->col_next];
  if (!e->slots_ready || !sl.pending) return fail(FVAD_EINVAL, "no submitted push to collect");
  const fvad_engine_config &c = e->cfg;
  HIP_TRY(hipSetDevice(c.device));
  HIP_TRY(hipEventSynchronize(sl.done));
  const size_t TB = (size_t)sl.n_ticks * c.n_streams, TBW = TB * e->wpt;
  if (out) {
    if (out->denoised && !c.want_denoised) return fail(FVAD_EINVAL, "engine created without want_denoised");
    auto cp = [](void *dst, const void *src, size_t n) {
      if (dst) std::memcpy(dst, src, n);
    };
    cp(out->vad, sl.vad, TB * 4);
    cp(out->ratio, sl.ratio, TB * 4);
    cp(out->win_flag, sl.wflag, TB * 4);
    cp(out->win_ratio, sl.wratio, TBW * 4);
    cp(out->win_vad, sl.wvad, TBW * 4);
    cp(out->band, sl.band, TBW * c.n_channels * c.n_bands * 4);
    if (out->denoised) par_copy(out->denoised, sl.den, TB * c.n_channels * fvad::kFrame * 4);
  }
  if (n_ticks) *n_ticks = sl.n_ticks;
  sl.pending = false;
  e->col_next = (e->col_next + 1) % FVAD_MAX_IN_FLIGHT;
  return FVAD_OK;
}

extern "C" int fvad_engine_load_synthetic(fvad_engine *e, int n_ticks, uint32_t base) {
  return fvad_engine_load_synthetic_ex(e, n_ticks, 1, base);
}

// n_pushes distinct pushes of n_ticks resident in HBM: stream s's first
// n_pushes * n_ticks ticks of fvad_synth_stream(base + s) (generated at that
// length).  One push lives in the input buffer d_pcm_b[0]; more get their own
// [push][tick][stream][ch][480] buffer, and run_resident cycles through them.
// Host memory stays bounded: groups of kGroup streams are generated and copied
// (one strided copy per group: a group's rows of every tick), never the whole
// block.
extern "C" int fvad_engine_load_synthetic_ex(fvad_engine *e, int n_ticks, int n_pushes, uint32_t base) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  const fvad_engine_config &c = e->cfg;
  if (n_ticks < 1 || n_ticks > c.max_ticks) return fail(FVAD_EINVAL, "n_ticks out of range");
  if (n_pushes < 1 || (long long)n_ticks * n_pushes > (1LL << 30))
    return fail(FVAD_EINVAL, "1 <= n_pushes and n_ticks * n_pushes <= 2^30 required");
  HIP_TRY(hipSetDevice(c.device));
  const size_t row = (size_t)c.n_channels * fvad::kFrame;  // floats of one (tick, stream)
  const size_t per_push = (size_t)n_ticks * c.n_streams * row;
  const int total = n_ticks * n_pushes;
  constexpr int kGroup = 64;
  const int gs = std::min(kGroup, c.n_streams);
  std::vector<float> host;
  try {
    host.resize((size_t)total * gs * row);
  } catch (...) {
    return fail(FVAD_ENOMEM, "host buffer for the synthetic input");
  }
  // buffer 0 (or the resident set) may still be read by an in-flight push
  int rc = fvad_engine_sync(e);
  if (rc) return rc;
  if (e->d_res) {
    HIP_TRY(hipFree(e->d_res));
    e->d_res = nullptr;
  }
  e->res_pushes = 0;
  if (n_pushes > 1 && (rc = dalloc(&e->d_res, per_push * n_pushes))) return rc;
  // [push][tick][stream] rows are [global tick][stream] rows: tick g = k * n_ticks + t
  float *dst = n_pushes == 1 ? e->d_pcm_b[0] : e->d_res;
  for (int s0 = 0; s0 < c.n_streams; s0 += gs) {
    const int ns = std::min(gs, c.n_streams - s0);
    if ((rc = fvad_synth_group(base, s0, ns, c.n_channels, total, 0, total, host.data(), (size_t)ns)))
      return fail(rc, "synthetic input generation failed");
    HIP_TRY(hipMemcpy2D(dst + (size_t)s0 * row, (size_t)c.n_streams * row * sizeof(float), host.data(),
                        (size_t)ns * row * sizeof(float), (size_t)ns * row * sizeof(float), (size_t)total,
                        hipMemcpyHostToDevice));
  }
  if (n_pushes > 1) e->res_pushes = n_pushes;
  e->res_next = 0;
  e->resident_ticks = n_ticks;
  return FVAD_OK;
}

extern "C" int fvad_engine_resident_seek(fvad_engine *e, int push) {
  if (!e || e->resident_ticks < 1) return fail(FVAD_EINVAL, "no resident input");
  if (push < 0 || push >= std::max(1, e->res_pushes)) return fail(FVAD_EINVAL, "push index out of range");
  e->res_next = push;
  return FVAD_OK;
}

extern "C" int fvad_engine_run_resident(fvad_engine *e, int n_ticks) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  if (n_ticks < 1 || n_ticks > e->resident_ticks) return fail(FVAD_EINVAL, "n_ticks exceeds resident input");
  HIP_TRY(hipSetDevice(e->cfg.device));
  // the set this push will record into was used two pushes ago: read it (it
  // is long finished) before reusing it; the previous push keeps running
  e->ev_slot ^= 1;
  e->ev = e->evs[e->ev_slot];
  int rc = collect_slot(e, e->ev_slot);
  if (rc) return rc;
  if (e->res_pushes > 1) {  // the next of the resident pushes, cyclically
    const size_t per_push = (size_t)e->resident_ticks * e->cfg.n_streams * e->cfg.n_channels * fvad::kFrame;
    e->d_pcm = e->d_res + per_push * (size_t)e->res_next;
    e->res_next = (e->res_next + 1) % e->res_pushes;
  } else {
    e->d_pcm = e->d_pcm_b[0];
  }
  // Timing events on every FVAD_EVENT_EVERY-th push (default 4: the 15
  // event markers of a push cost it ~1 %, measured); FVAD_NO_EVENTS=1: none
  static const bool no_events = [] {
    const char *v = getenv("FVAD_NO_EVENTS");
    return v && atoi(v) == 1;
  }();
  static const int every = [] {
    const char *v = getenv("FVAD_EVENT_EVERY");
    const int n = v ? atoi(v) : 4;
    return n < 1 ? 1 : n;
  }();
  const bool timed = !no_events && e->res_count++ % every == 0;
  if ((rc = launch(e, n_ticks, false, timed))) return rc;
  // a later submit / push must not overwrite buffer 0 under this run's prep
  if (e->res_pushes <= 1) {
    HIP_TRY(hipEventRecord(e->ev_in_free[0], input_reader(e)));
    e->in_busy[0] = true;
  }
  return FVAD_OK;
}

extern "C" int fvad_engine_sync(fvad_engine *e) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (e->cstream) HIP_TRY(hipStreamSynchronize(e->cstream));
  if (e->pstream) HIP_TRY(hipStreamSynchronize(e->pstream));
  if (e->side)
    if (const int rf = vadm_flush(e, true)) return rf;
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->side) {
    HIP_TRY(hipStreamSynchronize(e->side));
    const int rc = collect_vadm_timing(e);
    if (rc) return rc;
  }
  return collect_timing(e);
}

extern "C" int fvad_engine_kernel_times(fvad_engine *e, double *ms_avg, int *n_runs) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  int rc = fvad_engine_sync(e);
  if (rc) return rc;
  for (int i = 0; i < FVAD_MAX_TIMES; i++)
    ms_avg[i] = (e->n_timed && i <= e->n_kernels) ? e->ms_sum[i] / e->n_timed : 0.0;
  // the VADMachine (side stream, overlapped with the next push): reported after
  // the pipeline kernels, not part of [0]; k_vadm_hbm (steady state) and
  // k_vadm_par (the push flushed at a sync point) separately
  for (int k = 0; k < 2; k++)
    if (e->vadm.n > 0 && e->n_kernels + 1 + k < FVAD_MAX_TIMES)
      ms_avg[e->n_kernels + 1 + k] = e->vadm_timed[k] ? e->vadm_ms_sum[k] / e->vadm_timed[k] : 0.0;
  if (n_runs) *n_runs = e->n_timed;
  return FVAD_OK;
}

extern "C" int fvad_engine_clear_times(fvad_engine *e) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  int rc = fvad_engine_sync(e);
  if (rc) return rc;
  for (double &v : e->ms_sum) v = 0;
  for (int k = 0; k < 2; k++) {
    e->vadm_ms_sum[k] = 0;
    e->vadm_timed[k] = 0;
  }
  e->n_timed = 0;
  e->res_count = 0;
  return FVAD_OK;
}

extern "C" int fvad_engine_fetch(fvad_engine *e, int n_ticks, fvad_outputs *out) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  if (n_ticks < 1 || n_ticks > e->cfg.max_ticks) return fail(FVAD_EINVAL, "n_ticks out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return fetch(e, n_ticks, out);
}

extern "C" int fvad_engine_windows_per_tick(const fvad_engine *e) { return e ? e->wpt : FVAD_EINVAL; }

extern "C" const char *fvad_engine_kernel_name(const fvad_engine *e, int i) {
  if (e && i == e->n_kernels && e->vadm.n > 0) return "k_vadm_hbm";
  if (e && i == e->n_kernels + 1 && e->vadm.n > 0) return "k_vadm_par";
  if (!e || i < 0 || i >= e->n_kernels) return nullptr;
  if (e->cfg.mode == FVAD_MODE_FUSED) return i == 0 ? "k_prep" : "k_frame";
  if (fp16_mode(e->cfg.mode) && i == 6) return e->cfg.mode == FVAD_MODE_FP16_FUSED ? "k_fused16" : "k_gru16";
  if (e->olafb && i == 8) return "k_olafb";
  return fvad::staged_kernel_name(i);
}

// ---------------------------------------------------------------------------
// Device VADMachines (VADMachine.zig:126-230 on the GPU)
// ---------------------------------------------------------------------------
namespace {
// RollingAverage(count, init) initial state (RollingAverage.zig:16-32)
double initial_avg(size_t n, double init) {
  double a = 0.0;
  const double scalar = 1.0 / (double)n;
  for (size_t i = 0; i < n; i++) a += init * scalar;
  return a;
}
}  // namespace

int vadm_reset(fvad_engine *e) {
  std::vector<fvad::VadmState> st = e->vadm_init;
  if (!e->dbg_lt_full) {
    // every entry 0.0f (initial entries are K.init, tracked by lt_nw): a device
    // memset, no host image of the buffers (hundreds of MB at 2048 streams)
    HIP_TRY(hipMemset(e->vadm.buf, 0, e->vadm_buf_len * sizeof(float)));
  } else {
    std::vector<float> buf(e->vadm_buf_len, 0.0f);
    // test hook FVAD_DEBUG_VADM_LT_FULL: every long-term entry counts as pushed
    // (holding (float)init), the state of a stream past its first
    // long_term_speech_avg_sec -- timing only, not the reference's values
    const int B = e->cfg.n_streams;
    for (int m = 0; m < e->vadm.n; m++) {
      const fvad::VadmConst &K = e->vadm.c[m];
      for (int s = 0; s < B; s++)
        for (int i = 0; i < K.n_lt; i++) buf[K.lt_off + (size_t)s * K.lt_pitch + i] = (float)K.init;
      for (int s = 0; s < B; s++) st[(size_t)m * B + s].lt_nw = (unsigned)K.n_lt;
    }
    HIP_TRY(hipMemcpy(e->vadm.buf, buf.data(), buf.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(e->vadm.st, st.data(), st.size() * sizeof(fvad::VadmState), hipMemcpyHostToDevice));
  return FVAD_OK;
}

extern "C" int fvad_engine_attach_vadm(fvad_engine *e, const fvad_vadm_config *cfgs, int n, int seg_capacity) {
  if (!e || !cfgs || n < 1 || n > FVAD_MAX_BANDS || seg_capacity < 1) return fail(FVAD_EINVAL, "invalid argument");
  if (e->cfg.mode == FVAD_MODE_FUSED) return fail(FVAD_EINVAL, "device VADMachines need the staged engine");
  if (e->vadm.n > 0) return fail(FVAD_EINVAL, "VADMachines already attached");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int B = e->cfg.n_streams;
  const float sr = (float)e->cfg.sample_rate;
  const float eval_per_sec = sr / (float)e->cfg.fft_size;
  auto len_of = [&](float sec) { return std::max<size_t>(1, (size_t)(eval_per_sec * sec)); };
  auto freq_to_bin = [&](float f) { return (int)std::round(f / (sr / (float)e->cfg.fft_size)); };
  fvad::VadmArgs v{};
  v.n = n;
  v.seg_cap = seg_capacity;
  v.bound_scale = 1.0;
  v.negate_at = -1;
  long long off = 0;
  std::vector<fvad::VadmState> init((size_t)n * B);
  for (int m = 0; m < n; m++) {
    const fvad_vadm_config &c = cfgs[m];
    fvad::VadmConst &K = v.c[m];
    const int lo = freq_to_bin(c.speech_min_freq), hi = freq_to_bin(c.speech_max_freq);
    K.slot = -1;
    for (int b = 0; b < e->cfg.n_bands; b++)
      if (e->cfg.band_lo[b] == lo && e->cfg.band_hi[b] == hi) K.slot = b;
    if (K.slot < 0) return fail(FVAD_EINVAL, "no engine band matches the machine's speech band");
    K.n_lt = (int)len_of(c.long_term_speech_avg_sec);
    K.n_st = (int)len_of(c.short_term_speech_avg_sec);
    K.n_r = (int)len_of(c.channel_vol_ratio_avg_sec);
    K.lt_pitch = (K.n_lt + 3) & ~3;  // 16-byte rows
    off = (off + 3) & ~3LL;
    K.lt_off = off;
    off += (long long)K.lt_pitch * B;
    K.st_off = off;
    off += (long long)K.n_st * B;
    K.r_off = off;
    off += (long long)K.n_r * B;
    K.min_open = (unsigned long long)(size_t)(sr * c.min_consecutive_sec_to_open);
    K.max_gap = (unsigned long long)(size_t)(sr * c.max_speech_gap_sec);
    K.rec_pad = (unsigned long long)(sr * 2);
    K.thr_factor = c.speech_threshold_factor;
    K.ratio_thr = c.channel_vol_ratio_threshold;
    K.min_dur = c.min_vad_duration_sec;
    K.sr = sr;
    K.has_init = c.has_initial_long_term_avg != 0;
    K.init = c.initial_long_term_avg;
    fvad::VadmState s0{};
    if (K.has_init) {
      // RollingAverage(initial_avg): data = init (a double, VADMachine.zig:89-94)
      s0.lt_count = (unsigned)K.n_lt;
      s0.lt_last = initial_avg((size_t)K.n_lt, K.init);
      s0.lt_has = 1;
      s0.lt_pre_ok = 1;  // next write is at 0: the next pass starts from 0.0
      s0.lt_pre = 0.0;
    }
    for (int s = 0; s < B; s++) init[(size_t)m * B + s] = s0;
  }
  int rc;
  if ((rc = dalloc(&v.st, init.size())) || (rc = dalloc(&v.buf, (size_t)off)) ||
      (rc = dalloc(&v.seg, (size_t)n * B * seg_capacity))) {
    void *ptrs[] = {v.st, v.buf, v.seg};
    for (void *p : ptrs)
      if (p) (void)hipFree(p);
    return rc;
  }
  e->vadm = v;
  e->vadm_init = std::move(init);
  e->vadm_buf_len = (size_t)off;
  const size_t TB = (size_t)e->cfg.max_ticks * B, TBW = TB * e->wpt;
  if ((rc = dalloc(&e->d_vflag, TB)) || (rc = dalloc(&e->d_vwratio, TBW)) || (rc = dalloc(&e->d_vwvad, TBW)) ||
      (rc = dalloc(&e->d_vband, TBW * e->cfg.n_channels * e->cfg.n_bands)) || (rc = dalloc(&e->d_vticks, (size_t)B)) ||
      (rc = dalloc(&e->d_vticks_b[1], (size_t)B)))
    return rc;
  if (make_stream(&e->side) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_copy, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_vadm, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&e->ev_vt[0][0]) != hipSuccess || hipEventCreate(&e->ev_vt[0][1]) != hipSuccess ||
      hipEventCreate(&e->ev_vt[1][0]) != hipSuccess || hipEventCreate(&e->ev_vt[1][1]) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_vadm_b[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_vadm_b[1], hipEventDisableTiming) != hipSuccess)
    return fail(FVAD_EDEVICE, "side stream / event creation failed");
  e->side_ref.reset(e->side, destroy_stream);
  e->d_vticks_b[0] = e->d_vticks;
  HIP_TRY(hipEventRecord(e->ev_vadm, e->side));
  HIP_TRY(hipEventRecord(e->ev_vadm_b[0], e->side));
  HIP_TRY(hipEventRecord(e->ev_vadm_b[1], e->side));
  // the second window-output set (push parity 1); set 0 is the engine's own
  e->wflag_b[1] = e->d_vflag;
  e->wratio_b[1] = e->d_vwratio;
  e->wvad_b[1] = e->d_vwvad;
  e->band_b[1] = e->d_vband;
  return vadm_reset(e);
}

extern "C" size_t fvad_engine_segments(fvad_engine *e, int stream, int machine, fvad_segment *out, size_t cap) {
  return fvad_engine_segments_range(e, stream, machine, 0, out, cap);
}

extern "C" int fvad_engine_vadm_state(fvad_engine *e, int stream, int machine, int *speech_state,
                                      uint64_t *speech_start, uint64_t *speech_end) {
  if (!e || e->vadm.n == 0 || stream < 0 || stream >= e->cfg.n_streams || machine < 0 || machine >= e->vadm.n)
    return fail(FVAD_EINVAL, "no such attached machine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (const int rf = vadm_flush(e, true)) return rf;
  HIP_TRY(hipStreamSynchronize(e->side));
  fvad::VadmState st;
  HIP_TRY(hipMemcpy(&st, e->vadm.st + (size_t)machine * e->cfg.n_streams + stream, sizeof(st),
                    hipMemcpyDeviceToHost));
  if (speech_state) *speech_state = st.state;
  if (speech_start) *speech_start = st.speech_start;
  if (speech_end) *speech_end = st.speech_end;
  return FVAD_OK;
}

extern "C" size_t fvad_engine_segments_range(fvad_engine *e, int stream, int machine, size_t first,
                                             fvad_segment *out, size_t cap) {
  if (!e || e->vadm.n == 0 || stream < 0 || stream >= e->cfg.n_streams || machine < 0 || machine >= e->vadm.n)
    return 0;
  if (hipSetDevice(e->cfg.device) != hipSuccess || vadm_flush(e, true) != FVAD_OK ||
      hipStreamSynchronize(e->stream) != hipSuccess || hipStreamSynchronize(e->side) != hipSuccess)
    return 0;
  const size_t idx = (size_t)machine * e->cfg.n_streams + stream;
  fvad::VadmState st;
  if (hipMemcpy(&st, e->vadm.st + idx, sizeof(st), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  const size_t n = std::min<size_t>(st.n_segs, (size_t)e->vadm.seg_cap);
  const size_t k = first < n ? std::min(n - first, cap) : 0;
  if (out && k) {
    std::vector<fvad::VadmSeg> tmp(k);
    if (hipMemcpy(tmp.data(), e->vadm.seg + idx * e->vadm.seg_cap + first, k * sizeof(fvad::VadmSeg),
                  hipMemcpyDeviceToHost) != hipSuccess)
      return 0;
    for (size_t i = 0; i < k; i++) {
      out[i].sample_from = tmp[i].sample_from;
      out[i].sample_to = tmp[i].sample_to;
      out[i].debug_rnn_vad = tmp[i].debug_rnn_vad;
      out[i].debug_avg_speech_vol_ratio = tmp[i].debug_avg_speech_vol_ratio;
    }
  }
  return st.n_segs;
}

// ---------------------------------------------------------------------------
// Checker access: the whole device machine state and the test hooks
// ---------------------------------------------------------------------------
namespace {
int vadm_read_state(fvad_engine *e, int stream, int machine, fvad::VadmState *st) {
  if (!e || e->vadm.n == 0 || stream < 0 || stream >= e->cfg.n_streams || machine < 0 || machine >= e->vadm.n)
    return fail(FVAD_EINVAL, "no such attached machine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (const int rc = fvad_engine_sync(e)) return rc;
  HIP_TRY(hipMemcpy(st, e->vadm.st + (size_t)machine * e->cfg.n_streams + stream, sizeof(*st),
                    hipMemcpyDeviceToHost));
  return FVAD_OK;
}
}  // namespace

extern "C" int fvad_engine_vadm_snapshot(fvad_engine *e, int stream, int machine, fvad_vadm_snapshot *out) {
  if (!out) return fail(FVAD_EINVAL, "null argument");
  fvad::VadmState st;
  if (const int rc = vadm_read_state(e, stream, machine, &st)) return rc;
  std::memset(out, 0, sizeof(*out));
  out->speech_state = st.state;
  out->speech_start = st.speech_start;
  out->speech_end = st.speech_end;
  out->windows = st.windows_done;
  out->avg[0] = st.lt_last;
  out->avg[1] = st.st_last;
  out->avg[2] = st.r_last;
  out->write_idx[0] = st.lt_widx;
  out->write_idx[1] = st.st_widx;
  out->write_idx[2] = st.r_widx;
  out->written[0] = st.lt_count;
  out->written[1] = st.st_count;
  out->written[2] = st.r_count;
  out->speech_rnn_vad = st.rnn_vad;
  out->speech_vol_ratio = st.vol_ratio;
  out->speech_rnn_vad_count = st.rnn_vad_count;
  out->speech_vol_ratio_count = st.vol_ratio_count;
  out->n_segments = st.n_segs;
  return FVAD_OK;
}

extern "C" long fvad_engine_vadm_rolling(fvad_engine *e, int stream, int machine, int which, double *out, size_t cap) {
  if (which < 0 || which > 2) return fail(FVAD_EINVAL, "which: 0 long-term, 1 short-term, 2 volume ratio");
  fvad::VadmState st;
  if (const int rc = vadm_read_state(e, stream, machine, &st)) return rc;
  const fvad::VadmConst &K = e->vadm.c[machine];
  const int n = which == 0 ? K.n_lt : which == 1 ? K.n_st : K.n_r;
  const long long off = which == 0 ? K.lt_off : which == 1 ? K.st_off : K.r_off;
  const size_t B = e->cfg.n_streams, k = std::min<size_t>((size_t)n, cap);
  if (out && k) {
    // long-term entries: the stream's row; the others [i][stream]: a strided 2D copy of its column
    std::vector<float> col(k);
    if (which == 0)
      HIP_TRY(hipMemcpy(col.data(), e->vadm.buf + off + (size_t)stream * K.lt_pitch, k * sizeof(float),
                        hipMemcpyDeviceToHost));
    else
      HIP_TRY(hipMemcpy2D(col.data(), sizeof(float), e->vadm.buf + off + stream, B * sizeof(float), sizeof(float), k,
                          hipMemcpyDeviceToHost));
    for (size_t i = 0; i < k; i++)
      // long-term entries never written since the machine started hold the
      // initial average, a double (RollingAverage.zig:16-32; lt_nw counts the written)
      out[i] = (which == 0 && K.has_init && i >= st.lt_nw) ? K.init : (double)col[i];
  }
  return n;
}

extern "C" int fvad_engine_set_debug(fvad_engine *e, int key, int value) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  switch (key) {
    case FVAD_DEBUG_VADM_PAR_SERIAL_EVERY:
      if (value < 0) return fail(FVAD_EINVAL, "value >= 0 required");
      e->vadm.par_serial_every = value;
      return FVAD_OK;
    case FVAD_DEBUG_VADM_ALWAYS_PAR:
      e->dbg_always_par = value != 0;
      return FVAD_OK;
    case FVAD_DEBUG_VADM_DEFER_MAX:
      if (value < 0) return fail(FVAD_EINVAL, "value >= 0 required");
      e->vadm.defer_max = (unsigned)value;
      return FVAD_OK;
    case FVAD_DEBUG_VADM_BOUND_SCALE:
      if (e->vadm.n == 0) return fail(FVAD_EINVAL, "no VADMachines attached");
      if (value < -1) return fail(FVAD_EINVAL, "value >= -1 required");
      if (const int rc = fvad_engine_sync(e)) return rc;  // a queued k_vadm_hbm reads the argument block's copy
      e->vadm.bound_scale = value == -1 ? HUGE_VAL : (value == 0 ? 1.0 : (double)value);
      return FVAD_OK;
    case FVAD_DEBUG_VADM_NEGATE_AT:
      if (e->vadm.n == 0) return fail(FVAD_EINVAL, "no VADMachines attached");
      if (value < -1) return fail(FVAD_EINVAL, "value >= -1 required");
      if (const int rc = fvad_engine_sync(e)) return rc;
      e->vadm.negate_at = value;
      return FVAD_OK;
    case FVAD_DEBUG_VADM_COUNT:
      if (e->vadm.n == 0) return fail(FVAD_EINVAL, "no VADMachines attached");
      if (const int rc = fvad_engine_sync(e)) return rc;
      if (value && !e->vadm.count) {
        if (const int rc = dalloc(&e->vadm.count, fvad::kVadmCounts)) return rc;
      }
      if (!value && e->vadm.count) {
        HIP_TRY(hipFree(e->vadm.count));
        e->vadm.count = nullptr;
      }
      if (e->vadm.count) HIP_TRY(hipMemset(e->vadm.count, 0, fvad::kVadmCounts * sizeof(unsigned long long)));
      return FVAD_OK;
    case FVAD_DEBUG_VADM_LT_FULL:
      if (e->vadm.n == 0) return fail(FVAD_EINVAL, "no VADMachines attached");
      e->dbg_lt_full = value != 0;
      if (const int rc = fvad_engine_sync(e)) return rc;
      return vadm_reset(e);
    default:
      return fail(FVAD_EINVAL, "unknown debug key");
  }
}

extern "C" int fvad_engine_debug_counts(fvad_engine *e, unsigned long long *out, int n) {
  if (!e || !out || n < 1) return fail(FVAD_EINVAL, "invalid argument");
  if (!e->vadm.count) return fail(FVAD_EINVAL, "FVAD_DEBUG_VADM_COUNT is not set");
  if (const int rc = fvad_engine_sync(e)) return rc;
  unsigned long long c[fvad::kVadmCounts];
  HIP_TRY(hipMemcpy(c, e->vadm.count, sizeof(c), hipMemcpyDeviceToHost));
  const int k = std::min(n, (int)fvad::kVadmCounts);
  for (int i = 0; i < k; i++) out[i] = c[i];
  return k;
}

extern "C" int fvad_engine_output_log(fvad_engine *e, int n_pushes) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  if (e->cfg.mode == FVAD_MODE_FUSED || !e->cfg.use_denoiser)
    return fail(FVAD_EINVAL, "the output log records staged / fp16 engines with the denoiser");
  if (n_pushes < 0) return fail(FVAD_EINVAL, "n_pushes >= 0 required");
  if (const int rc = fvad_engine_sync(e)) return rc;
  if (e->d_log) {
    HIP_TRY(hipFree(e->d_log));
    e->d_log = nullptr;
  }
  const fvad_engine_config &c = e->cfg;
  const size_t MT = (size_t)c.max_ticks * c.n_streams, MW = MT * e->wpt;
  e->log_stride = 3 * MT + 2 * MW + MW * c.n_channels * c.n_bands;
  e->log_cap = e->log_n = 0;
  e->log_ticks.assign((size_t)n_pushes, 0);
  if (n_pushes > 0) {
    if (const int rc = dalloc(&e->d_log, e->log_stride * (size_t)n_pushes)) return rc;
    e->log_cap = n_pushes;
  }
  return FVAD_OK;
}

extern "C" int fvad_engine_output_log_read(fvad_engine *e, int push, fvad_outputs *out, int *n_ticks) {
  if (!e) return fail(FVAD_EINVAL, "null engine");
  if (push < 0 || push >= e->log_n) return fail(FVAD_EINVAL, "push not in the log");
  if (const int rc = fvad_engine_sync(e)) return rc;
  const fvad_engine_config &c = e->cfg;
  const int T = e->log_ticks[push];
  const size_t MT = (size_t)c.max_ticks * c.n_streams, MW = MT * e->wpt;
  const size_t TB = (size_t)T * c.n_streams, TBW = TB * e->wpt;
  const float *L = e->d_log + e->log_stride * (size_t)push;
  if (n_ticks) *n_ticks = T;
  if (!out) return FVAD_OK;
  void *dst[6] = {out->vad, out->ratio, out->win_flag, out->win_ratio, out->win_vad, out->band};
  const size_t off[6] = {0, MT, 2 * MT, 3 * MT, 3 * MT + MW, 3 * MT + 2 * MW};
  const size_t n[6] = {TB, TB, TB, TBW, TBW, TBW * c.n_channels * c.n_bands};
  for (int i = 0; i < 6; i++)
    if (dst[i]) HIP_TRY(hipMemcpy(dst[i], L + off[i], n[i] * 4, hipMemcpyDeviceToHost));
  return FVAD_OK;
}
