"""Python bindings (ctypes) for libfvad.so — the MI355X-native Formula-VAD hot path.

Mirrors the reference's API surface for this path:
  * Denoiser        (src/Denoiser.zig)        -> rnnoise_* C ABI on the GPU
  * KissFFTR        (src/FFT.zig kissfft use) -> kiss_fftr_* C ABI on the GPU
  * Engine          batched multi-stream hot path (fvad_engine_*)
  * AudioPipeline   (src/AudioPipeline.zig pushSamples + VAD + VADMachine)
  * Multi           multi-stream simulator core (simulator.zig runAll)
  * evaluate/aggregate/parse_audacity (src/Evaluator/*)

All compute goes through the HIP kernels in libfvad.so; there is no CPU
fallback — operations raise FvadError when the library or the GPU is missing.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("FVAD_LIB", os.path.join(PKG_ROOT, "lib", "libfvad.so"))

FVAD_OK = 0
F32P = C.POINTER(C.c_float)
I32P = C.POINTER(C.c_int32)
MAX_BANDS = 4
FRAME = 480


class FvadError(RuntimeError):
    pass


class EngineConfig(C.Structure):
    _fields_ = [("n_streams", C.c_int), ("n_channels", C.c_int), ("device", C.c_int), ("sample_rate", C.c_int),
                ("fft_size", C.c_int), ("max_ticks", C.c_int), ("n_bands", C.c_int),
                ("band_lo", C.c_int * MAX_BANDS), ("band_hi", C.c_int * MAX_BANDS), ("want_denoised", C.c_int),
                ("mode", C.c_int), ("use_denoiser", C.c_int)]


MODE_STAGED, MODE_FUSED, MODE_FP16, MODE_FP16_FUSED = 0, 1, 2, 3
MAX_TIMES = 16


class Outputs(C.Structure):
    _fields_ = [("vad", F32P), ("ratio", F32P), ("win_flag", I32P), ("win_ratio", F32P), ("win_vad", F32P),
                ("band", F32P), ("denoised", F32P)]


class VadmConfig(C.Structure):
    _fields_ = [("speech_min_freq", C.c_float), ("speech_max_freq", C.c_float),
                ("long_term_speech_avg_sec", C.c_float), ("has_initial_long_term_avg", C.c_int),
                ("initial_long_term_avg", C.c_double), ("short_term_speech_avg_sec", C.c_float),
                ("speech_threshold_factor", C.c_float), ("channel_vol_ratio_avg_sec", C.c_float),
                ("channel_vol_ratio_threshold", C.c_float), ("min_consecutive_sec_to_open", C.c_float),
                ("max_speech_gap_sec", C.c_float), ("min_vad_duration_sec", C.c_float)]

    @classmethod
    def default(cls):
        c = cls()
        lib().fvad_vadm_config_default(C.byref(c))
        return c


class VadConfig(C.Structure):
    """VAD.Config (VAD.zig:17-23)."""
    _fields_ = [("fft_size", C.c_int), ("use_denoiser", C.c_int), ("vad_machine_config", VadmConfig),
                ("alt_vad_machine_configs", C.c_void_p), ("n_alt", C.c_int)]

    @classmethod
    def make(cls, fft_size=2048, use_denoiser=True, main_cfg=None, alt_cfgs=()):
        c = cls()
        lib().fvad_vad_config_default(C.byref(c))
        c.fft_size = fft_size
        c.use_denoiser = int(use_denoiser)
        if main_cfg is not None:
            c.vad_machine_config = main_cfg
        arr = (VadmConfig * max(1, len(alt_cfgs)))(*alt_cfgs)
        c._alts = arr
        c.alt_vad_machine_configs = C.cast(arr, C.c_void_p) if alt_cfgs else None
        c.n_alt = len(alt_cfgs)
        return c


class VadmSnapshot(C.Structure):
    """fvad_vadm_snapshot (include/fvad.h): a device machine's whole state."""
    _fields_ = [("speech_state", C.c_int), ("speech_start", C.c_uint64), ("speech_end", C.c_uint64),
                ("windows", C.c_uint64), ("avg", C.c_double * 3), ("write_idx", C.c_uint64 * 3),
                ("written", C.c_uint64 * 3), ("speech_rnn_vad", C.c_float), ("speech_vol_ratio", C.c_float),
                ("speech_rnn_vad_count", C.c_uint64), ("speech_vol_ratio_count", C.c_uint64),
                ("n_segments", C.c_uint64)]

    def as_dict(self):
        return {n: (list(getattr(self, n)) if n in ("avg", "write_idx", "written") else getattr(self, n))
                for n, _ in self._fields_}


DEBUG_VADM_PAR_SERIAL_EVERY, DEBUG_VADM_ALWAYS_PAR, DEBUG_VADM_LT_FULL, DEBUG_VADM_DEFER_MAX = 1, 2, 3, 4
DEBUG_VADM_BOUND_SCALE, DEBUG_VADM_COUNT, DEBUG_VADM_NEGATE_AT = 5, 6, 7
SHARE_PREP, SHARE_SIDE = 1, 2  # fvad_engine_share_streams

READ_FN = C.CFUNCTYPE(C.c_size_t, C.c_void_p, C.c_int, C.POINTER(F32P), C.c_size_t)


class Segment(C.Structure):
    _fields_ = [("sample_from", C.c_uint64), ("sample_to", C.c_uint64), ("debug_rnn_vad", C.c_float),
                ("debug_avg_speech_vol_ratio", C.c_float)]


class StatConfig(C.Structure):
    _fields_ = [("ignore_shorter_than_sec", C.c_float), ("extrude_start", C.c_float), ("extrude_end", C.c_float),
                ("fill_gaps", C.c_float)]


_STAT_FIELDS = ("total_positives_sec", "true_positives_sec", "false_positives_sec", "false_negatives_sec",
                "true_positive_rate", "false_negative_rate", "false_discovery_rate", "precision", "fm_index",
                "f_score", "f_score_beta")


class SingleStats(C.Structure):
    _fields_ = [(n, C.c_float) for n in _STAT_FIELDS]


class AggStat(C.Structure):
    _fields_ = [("overall", C.c_float), ("min", C.c_float), ("max", C.c_float), ("avg", C.c_float)]


class AggregateStats(C.Structure):
    _fields_ = [("total_positives_sec", C.c_float), ("true_positives_sec", C.c_float),
                ("false_positives_sec", C.c_float), ("false_negatives_sec", C.c_float),
                ("true_positive_rate", AggStat), ("false_negative_rate", AggStat),
                ("false_discovery_rate", AggStat), ("precision", AggStat), ("fm_index", C.c_float),
                ("f_score", C.c_float), ("f_score_beta", C.c_float)]


class KissCpx(C.Structure):
    _fields_ = [("r", C.c_float), ("i", C.c_float)]


# Every symbol include/fvad.h declares: (name, restype, argtypes)
SYMBOLS = [
    ("fvad_last_error", C.c_char_p, []),
    ("fvad_version", C.c_char_p, []),
    ("rnnoise_create", C.c_void_p, [C.c_void_p]),
    ("rnnoise_destroy", None, [C.c_void_p]),
    ("rnnoise_process_frame", C.c_float, [C.c_void_p, F32P, F32P]),
    ("rnnoise_get_frame_size", C.c_int, []),
    ("fvad_set_default_model", None, [C.c_void_p]),
    ("kiss_fftr_alloc", C.c_void_p, [C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_size_t)]),
    ("kiss_fftr", None, [C.c_void_p, F32P, C.c_void_p]),
    ("fvad_model_synthetic", C.c_int, [C.c_uint64, C.POINTER(C.c_void_p)]),
    ("fvad_model_load_text", C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    ("fvad_model_free", None, [C.c_void_p]),
    ("fvad_model_blob", C.c_size_t, [C.c_void_p, C.c_void_p]),
    ("fvad_engine_config_default", None, [C.c_void_p, C.c_int, C.c_int]),
    ("fvad_engine_create", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fvad_engine_destroy", None, [C.c_void_p]),
    ("fvad_engine_reset", C.c_int, [C.c_void_p]),
    ("fvad_engine_push", C.c_int, [C.c_void_p, F32P, C.c_int, I32P, C.c_void_p]),
    ("fvad_engine_push_ex", C.c_int, [C.c_void_p, F32P, C.c_int, I32P, I32P, C.c_void_p]),
    ("fvad_engine_submit_ex", C.c_int, [C.c_void_p, F32P, C.c_int, I32P, I32P]),
    ("fvad_engine_input_slot", C.c_void_p, [C.c_void_p]),
    ("fvad_engine_submit", C.c_int, [C.c_void_p, F32P, C.c_int, I32P]),
    ("fvad_engine_collect", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]),
    ("fvad_engine_input_slot_i16", C.c_void_p, [C.c_void_p]),
    ("fvad_engine_submit_i16", C.c_int, [C.c_void_p, C.POINTER(C.c_int16), C.c_int, I32P, I32P]),
    ("fvad_engine_load_synthetic", C.c_int, [C.c_void_p, C.c_int, C.c_uint32]),
    ("fvad_engine_load_synthetic_ex", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_uint32]),
    ("fvad_engine_resident_seek", C.c_int, [C.c_void_p, C.c_int]),
    ("fvad_engine_run_resident", C.c_int, [C.c_void_p, C.c_int]),
    ("fvad_engine_sync", C.c_int, [C.c_void_p]),
    ("fvad_engine_kernel_times", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    ("fvad_engine_kernel_name", C.c_char_p, [C.c_void_p, C.c_int]),
    ("fvad_engine_windows_per_tick", C.c_int, [C.c_void_p]),
    ("fvad_engine_attach_vadm", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    ("fvad_engine_segments", C.c_size_t, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t]),
    ("fvad_engine_segments_range", C.c_size_t, [C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_size_t]),
    ("fvad_engine_vadm_state", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint64)]),
    ("fvad_engine_vadm_snapshot", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    ("fvad_engine_vadm_rolling", C.c_long, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_size_t]),
    ("fvad_engine_set_debug", C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    ("fvad_engine_debug_counts", C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    ("fvad_engine_share_streams", C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    ("fvad_engine_output_log", C.c_int, [C.c_void_p, C.c_int]),
    ("fvad_engine_output_log_read", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_int)]),
    ("fvad_engine_clear_times", C.c_int, [C.c_void_p]),
    ("fvad_engine_fetch", C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    ("fvad_vadm_config_default", None, [C.c_void_p]),
    ("fvad_vadm_create", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("fvad_vadm_destroy", None, [C.c_void_p]),
    ("fvad_vadm_bins", None, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("fvad_vadm_run", C.c_int, [C.c_void_p, C.c_uint64, F32P, C.c_float, C.c_float]),
    ("fvad_vadm_segments", C.c_size_t, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("fvad_pipeline_create", C.c_int, [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                       C.POINTER(C.c_void_p)]),
    ("fvad_pipeline_destroy", None, [C.c_void_p]),
    ("fvad_pipeline_push", C.c_int, [C.c_void_p, C.POINTER(F32P), C.c_size_t, C.POINTER(C.c_uint64)]),
    ("fvad_pipeline_segments", C.c_size_t, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    ("fvad_recording_channel", C.c_int, [C.POINTER(F32P), C.c_int, C.c_size_t]),
    ("fvad_pipeline_set_recorder", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fvad_multi_create", C.c_int, [C.c_int, C.c_int, C.c_void_p, I32P, C.c_int, C.c_void_p, C.c_int,
                                    C.POINTER(C.c_void_p)]),
    ("fvad_multi_create_ex", C.c_int, [C.c_int, I32P, C.c_void_p, I32P, C.c_int, C.c_void_p, C.c_int,
                                       C.POINTER(C.c_void_p)]),
    ("fvad_multi_run_stream", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fvad_multi_segments_alt", C.c_size_t, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t]),
    ("fvad_vad_config_default", None, [C.c_void_p]),
    ("fvad_pipeline_create_ex", C.c_int, [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("fvad_multi_destroy", None, [C.c_void_p]),
    ("fvad_multi_run", C.c_int, [C.c_void_p, C.POINTER(F32P), C.POINTER(C.c_size_t)]),
    ("fvad_multi_segments", C.c_size_t, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    ("fvad_eval_stats", C.c_int, [F32P, C.c_size_t, F32P, C.c_size_t, C.c_void_p, C.c_void_p]),
    ("fvad_eval_aggregate", None, [C.c_void_p, C.c_size_t, C.c_void_p]),
    ("fvad_parse_audacity", C.c_long, [C.c_char_p, C.c_size_t, F32P, C.c_size_t]),
    ("fvad_synth_stream", C.c_long, [C.c_uint32, C.c_size_t, C.c_int, F32P, F32P, C.c_size_t]),
    ("fvad_synth_ticks", C.c_int, [C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, F32P]),
    ("fvad_synth_cache_clear", None, []),
    ("fvad_simulator_main", C.c_int, [C.c_int, C.POINTER(C.c_char_p)]),
]

_lib = None


def lib():
    """Load libfvad.so (built in-tree by `make -C formula-vad_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FvadError("libfvad.so not built: run `make -C formula-vad_amd` (%s)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error():
    return lib().fvad_last_error().decode()


def _check(rc, what):
    if rc != FVAD_OK:
        raise FvadError("%s failed (%d): %s" % (what, rc, last_error()))


def fptr(a):
    return a.ctypes.data_as(F32P)


class Model:
    def __init__(self, seed=None, path=None):
        h = C.c_void_p()
        if path is not None:
            _check(lib().fvad_model_load_text(path.encode(), C.byref(h)), "fvad_model_load_text")
        else:
            _check(lib().fvad_model_synthetic(0 if seed is None else seed, C.byref(h)), "fvad_model_synthetic")
        self.h = h

    def blob(self):
        n = lib().fvad_model_blob(self.h, None)
        b = np.zeros(n, np.int8)
        lib().fvad_model_blob(self.h, b.ctypes.data_as(C.c_void_p))
        return b

    def __del__(self):
        try:
            lib().fvad_model_free(self.h)
        except Exception:
            pass


def synth_stream(stream_id, n_samples, n_channels=2, label_cap=4096):
    """Synthetic 48 kHz onboard audio (planar [ch][n]) and its speech labels (seconds)."""
    out = np.zeros((n_channels, n_samples), np.float32)
    lab = np.zeros(2 * label_cap, np.float32)
    n = lib().fvad_synth_stream(stream_id, n_samples, n_channels, fptr(out), fptr(lab), label_cap)
    return out, lab[: 2 * min(n, label_cap)].reshape(-1, 2).copy()


def synth_ticks(base, n_streams, n_channels, total_ticks, tick0=0, n_ticks=None, out=None):
    """fvad_synth_ticks: [n_ticks][n_streams][n_channels][480] of the streams
    base.. generated at total_ticks * 480 samples (nothing cached); into `out`
    (a C-contiguous float32 array of that shape, e.g. a pinned input slot) if given."""
    n_ticks = total_ticks - tick0 if n_ticks is None else n_ticks
    shape = (n_ticks, n_streams, n_channels, FRAME)
    if out is None:
        out = np.zeros(shape, np.float32)
    elif out.shape != shape or out.dtype != np.float32 or not out.flags.c_contiguous:
        raise ValueError("synth_ticks: out must be C-contiguous float32 %s" % (shape,))
    _check(lib().fvad_synth_ticks(base, n_streams, n_channels, total_ticks, tick0, n_ticks, fptr(out)),
           "fvad_synth_ticks")
    return out


def synth_cache_clear():
    lib().fvad_synth_cache_clear()


class Engine:
    """Batched hot path for a partition of streams on one GPU."""

    def __init__(self, model, n_streams, n_channels=2, device=0, max_ticks=100, fft_size=2048, bands=((4, 64),),
                 want_denoised=False, mode="staged", use_denoiser=True):
        cfg = EngineConfig()
        lib().fvad_engine_config_default(C.byref(cfg), n_streams, n_channels)
        cfg.device = device
        cfg.max_ticks = max_ticks
        cfg.fft_size = fft_size
        cfg.n_bands = len(bands)
        for i, (lo, hi) in enumerate(bands):
            cfg.band_lo[i] = lo
            cfg.band_hi[i] = hi
        cfg.want_denoised = int(want_denoised)
        cfg.mode = {"staged": MODE_STAGED, "fused": MODE_FUSED, "fp16": MODE_FP16, "fp16_fused": MODE_FP16_FUSED}[mode]
        cfg.use_denoiser = int(use_denoiser)
        self.cfg = cfg
        self.model = model
        h = C.c_void_p()
        _check(lib().fvad_engine_create(C.byref(cfg), model.h, C.byref(h)), "fvad_engine_create")
        self.h = h
        self.B, self.C, self.nb = n_streams, n_channels, len(bands)
        self.max_ticks = max_ticks
        # window slots per (tick, stream): 1 for fft_size >= 480, else several
        # (VAD.zig:307-347); with W > 1 the window outputs get a slot axis
        self.wpt = lib().fvad_engine_windows_per_tick(h)

    def _alloc_out(self, n_ticks, denoised):
        T, B, Ch, nb, W = n_ticks, self.B, self.C, self.nb, self.wpt
        ws = (T, B) if W == 1 else (T, B, W)
        o = {"vad": np.zeros((T, B), np.float32), "ratio": np.zeros((T, B), np.float32),
             "win_flag": np.zeros((T, B), np.int32), "win_ratio": np.zeros(ws, np.float32),
             "win_vad": np.zeros(ws, np.float32), "band": np.zeros(ws + (Ch, nb), np.float32)}
        if denoised:
            o["denoised"] = np.zeros((T, B, Ch, FRAME), np.float32)
        s = Outputs(fptr(o["vad"]), fptr(o["ratio"]), o["win_flag"].ctypes.data_as(I32P), fptr(o["win_ratio"]),
                    fptr(o["win_vad"]), fptr(o["band"]), fptr(o["denoised"]) if denoised else None)
        return o, s

    def push(self, pcm, ticks_valid=None, denoised=False, last_tick_samples=None):
        """pcm: [ticks][streams][channels][480] normalised f32; last_tick_samples
        (no-denoiser engines): real samples in each stream's last valid tick."""
        pcm = np.ascontiguousarray(pcm, np.float32)
        T = pcm.shape[0]
        assert pcm.shape[1:] == (self.B, self.C, FRAME), pcm.shape
        o, s = self._alloc_out(T, denoised)
        tv = None
        if ticks_valid is not None:
            tv = np.ascontiguousarray(ticks_valid, np.int32)
        lt = np.ascontiguousarray(last_tick_samples, np.int32) if last_tick_samples is not None else None
        _check(lib().fvad_engine_push_ex(self.h, fptr(pcm), T, tv.ctypes.data_as(I32P) if tv is not None else None,
                                         lt.ctypes.data_as(I32P) if lt is not None else None, C.byref(s)),
               "fvad_engine_push_ex")
        return o

    def input_slot(self):
        """The engine's pinned input slot for the next submit, as a
        [max_ticks][streams][channels][480] float32 view (fill it in place
        and pass it to submit: no host copy)."""
        p = lib().fvad_engine_input_slot(self.h)
        if not p:
            raise FvadError("fvad_engine_input_slot: %s" % last_error())
        n = self.max_ticks * self.B * self.C * FRAME
        arr = np.ctypeslib.as_array(C.cast(p, F32P), shape=(n,))
        return arr.reshape(self.max_ticks, self.B, self.C, FRAME)

    def submit(self, pcm, ticks_valid=None):
        """Asynchronous push (fvad_engine_submit): returns once queued."""
        pcm = np.ascontiguousarray(pcm, np.float32)
        assert pcm.shape[1:] == (self.B, self.C, FRAME), pcm.shape
        tv = np.ascontiguousarray(ticks_valid, np.int32) if ticks_valid is not None else None
        self._sub_keep = tv
        _check(lib().fvad_engine_submit(self.h, fptr(pcm), pcm.shape[0],
                                        tv.ctypes.data_as(I32P) if tv is not None else None), "fvad_engine_submit")

    def input_slot_i16(self):
        """The pinned 16-bit input slot for the next submit_i16, as a
        [max_ticks][streams][channels][480] int16 view."""
        p = lib().fvad_engine_input_slot_i16(self.h)
        if not p:
            raise FvadError("fvad_engine_input_slot_i16: %s" % last_error())
        n = self.max_ticks * self.B * self.C * FRAME
        arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int16)), shape=(n,))
        return arr.reshape(self.max_ticks, self.B, self.C, FRAME)

    def submit_i16(self, pcm, ticks_valid=None, last_tick_samples=None):
        """Asynchronous push of 16-bit samples k (fvad_engine_submit_i16): the
        same outputs as submit() of k / 32768.0f, half the PCIe bytes."""
        pcm = np.ascontiguousarray(pcm, np.int16)
        assert pcm.shape[1:] == (self.B, self.C, FRAME), pcm.shape
        tv = np.ascontiguousarray(ticks_valid, np.int32) if ticks_valid is not None else None
        lt = np.ascontiguousarray(last_tick_samples, np.int32) if last_tick_samples is not None else None
        self._sub_keep = (tv, lt)
        _check(lib().fvad_engine_submit_i16(self.h, pcm.ctypes.data_as(C.POINTER(C.c_int16)), pcm.shape[0],
                                            tv.ctypes.data_as(I32P) if tv is not None else None,
                                            lt.ctypes.data_as(I32P) if lt is not None else None),
               "fvad_engine_submit_i16")

    def collect(self, denoised=False, want=True):
        """Outputs of the oldest submitted push (fvad_engine_collect)."""
        if not want:
            _check(lib().fvad_engine_collect(self.h, None, None), "fvad_engine_collect")
            return None
        o, s = self._alloc_out(self.max_ticks, denoised)
        n = C.c_int()
        _check(lib().fvad_engine_collect(self.h, C.byref(s), C.byref(n)), "fvad_engine_collect")
        return {k: v[: n.value] for k, v in o.items()}

    def reset(self):
        _check(lib().fvad_engine_reset(self.h), "fvad_engine_reset")

    def load_synthetic(self, n_ticks, base=0, pushes=1):
        """pushes distinct resident pushes of n_ticks (run_resident cycles through them)."""
        _check(lib().fvad_engine_load_synthetic_ex(self.h, n_ticks, pushes, base), "fvad_engine_load_synthetic_ex")

    def resident_seek(self, push):
        _check(lib().fvad_engine_resident_seek(self.h, push), "fvad_engine_resident_seek")

    def run_resident(self, n_ticks):
        _check(lib().fvad_engine_run_resident(self.h, n_ticks), "fvad_engine_run_resident")

    def sync(self):
        _check(lib().fvad_engine_sync(self.h), "fvad_engine_sync")

    def kernel_times(self):
        """{"total_ms": push average, "kernels": {name: ms average}, "runs": n}"""
        ms = (C.c_double * MAX_TIMES)()
        n = C.c_int()
        _check(lib().fvad_engine_kernel_times(self.h, ms, C.byref(n)), "fvad_engine_kernel_times")
        names = []
        while len(names) < MAX_TIMES - 1:
            nm = lib().fvad_engine_kernel_name(self.h, len(names))
            if nm is None:
                break
            names.append(nm.decode())
        return {"total_ms": ms[0], "kernels": {nm: ms[1 + i] for i, nm in enumerate(names)}, "runs": n.value}

    def clear_times(self):
        _check(lib().fvad_engine_clear_times(self.h), "fvad_engine_clear_times")

    def attach_vadm(self, cfgs=None, seg_capacity=256):
        """Run VADMachines on the device after every push (default config if None)."""
        cfgs = list(cfgs) if cfgs else [VadmConfig.default()]
        arr = (VadmConfig * len(cfgs))(*cfgs)
        self._vadm_keep = arr
        _check(lib().fvad_engine_attach_vadm(self.h, arr, len(cfgs), seg_capacity), "fvad_engine_attach_vadm")

    def segments(self, stream, machine=0):
        n = lib().fvad_engine_segments(self.h, stream, machine, None, 0)
        buf = (Segment * max(1, n))()
        lib().fvad_engine_segments(self.h, stream, machine, buf, n)
        return [(s.sample_from, s.sample_to, s.debug_rnn_vad, s.debug_avg_speech_vol_ratio) for s in buf[:n]]

    def vadm_snapshot(self, stream, machine=0):
        """The device machine's whole state (fvad_engine_vadm_snapshot) as a dict."""
        s = VadmSnapshot()
        _check(lib().fvad_engine_vadm_snapshot(self.h, stream, machine, C.byref(s)), "fvad_engine_vadm_snapshot")
        return s.as_dict()

    def vadm_rolling(self, stream, which, machine=0):
        """RollingAverage.data (which 0 long-term, 1 short-term, 2 volume ratio) as float64."""
        n = lib().fvad_engine_vadm_rolling(self.h, stream, machine, which, None, 0)
        if n < 0:
            raise FvadError("fvad_engine_vadm_rolling failed (%d): %s" % (n, last_error()))
        out = np.zeros(n, np.float64)
        lib().fvad_engine_vadm_rolling(self.h, stream, machine, which, out.ctypes.data_as(C.c_void_p), n)
        return out

    def share_streams(self, other, which=SHARE_PREP | SHARE_SIDE):
        """Run this engine's k_prep3 / VADMachine kernels on other's streams
        (fvad_engine_share_streams); either engine may be destroyed first:
        the last one using a stream destroys it."""
        _check(lib().fvad_engine_share_streams(self.h, other.h, which), "fvad_engine_share_streams")

    def set_debug(self, key, value):
        """Test hooks (fvad_engine_set_debug): DEBUG_VADM_PAR_SERIAL_EVERY, DEBUG_VADM_ALWAYS_PAR,
        DEBUG_VADM_LT_FULL, DEBUG_VADM_DEFER_MAX, DEBUG_VADM_BOUND_SCALE, DEBUG_VADM_COUNT."""
        _check(lib().fvad_engine_set_debug(self.h, key, value), "fvad_engine_set_debug")

    def debug_counts(self):
        """DEBUG_VADM_COUNT's counters (fvad_engine_debug_counts): long-term tests
        decided exactly / settled by the bound / left open by it (folded), and
        end-of-push folds."""
        out = np.zeros(4, np.uint64)
        n = lib().fvad_engine_debug_counts(self.h, out.ctypes.data_as(C.c_void_p), 4)
        _check(n if n < 0 else 0, "fvad_engine_debug_counts")
        return dict(zip(("exact", "settled", "open", "end_fold"), (int(v) for v in out[:n])))

    def output_log(self, n_pushes):
        """Record the per-tick outputs of the next n_pushes pushes on the device (no host sync)."""
        _check(lib().fvad_engine_output_log(self.h, n_pushes), "fvad_engine_output_log")

    def output_log_read(self, push):
        o, s = self._alloc_out(self.max_ticks, False)
        n = C.c_int()
        _check(lib().fvad_engine_output_log_read(self.h, push, C.byref(s), C.byref(n)), "fvad_engine_output_log_read")
        return {k: v[: n.value] for k, v in o.items()}

    def fetch(self, n_ticks, denoised=False):
        o, s = self._alloc_out(n_ticks, denoised)
        _check(lib().fvad_engine_fetch(self.h, n_ticks, C.byref(s)), "fvad_engine_fetch")
        return o

    def __del__(self):
        try:
            lib().fvad_engine_destroy(self.h)
        except Exception:
            pass



class EngineGroup:
    """One GPU's streams as `groups` engines of about n_streams / groups each,
    pushing concurrently: each engine its own main stream, k_prep3 and the
    VADMachines of all of them on engine 0's two side streams
    (fvad_engine_share_streams), so a group of two takes 4 streams where two
    separate engines would take 6 (the runtime shares its 4 hardware queues
    round the streams).  Results are each engine's own, bit-identical to one
    engine over all the streams (tests/test_gpu_groups.py).  Throughput
    (DESIGN.md section 8, r5): +2-3 % over one engine when it is the first
    group a process creates, down to -35 % when the runtime's queue placement
    puts a main stream beside the side work -- so bench.py runs one engine per
    GPU unless asked (--groups).  Engine g owns streams
    [first[g], first[g] + sizes[g])."""

    def __init__(self, model, n_streams, n_channels=2, groups=2, vadm=False, **kw):
        if not 1 <= groups <= n_streams:
            raise ValueError("groups must be in [1, n_streams]")
        q, r = divmod(n_streams, groups)
        self.sizes = [q + (1 if g < r else 0) for g in range(groups)]
        self.first = [sum(self.sizes[:g]) for g in range(groups)]
        self.B, self.C = n_streams, n_channels
        self.engines = []
        for g, n in enumerate(self.sizes):
            # engine g's streams exist before engine g + 1's: the runtime hands
            # out hardware queues in creation order
            e = Engine(model, n, n_channels, **kw)
            if vadm:
                e.attach_vadm()
            if g and kw.get("mode", "staged") != "fused":  # the fused engine has no side streams
                e.share_streams(self.engines[0], SHARE_PREP | (SHARE_SIDE if vadm else 0))
            self.engines.append(e)

    def set_debug(self, key, value):
        for e in self.engines:
            e.set_debug(key, value)

    def load_synthetic(self, n_ticks, base=0, pushes=1):
        for e, f in zip(self.engines, self.first):
            e.load_synthetic(n_ticks, base=base + f, pushes=pushes)

    def run_resident(self, n_ticks):
        for e in self.engines:
            e.run_resident(n_ticks)

    def sync(self):
        for e in self.engines:
            e.sync()

    def clear_times(self):
        for e in self.engines:
            e.clear_times()

    def kernel_times(self):
        """Per kernel the mean over the engines of their launch averages (each
        launch covers one engine's streams, co-running with the others')."""
        ts = [e.kernel_times() for e in self.engines]
        names = ts[0]["kernels"].keys()
        return {"total_ms": sum(t["total_ms"] for t in ts) / len(ts),
                "kernels": {n: sum(t["kernels"].get(n, 0.0) for t in ts) / len(ts) for n in names},
                "runs": min(t["runs"] for t in ts)}

    def segments(self, stream, machine=0):
        g = max(i for i, f in enumerate(self.first) if f <= stream)
        return self.engines[g].segments(stream - self.first[g], machine)

class Denoiser:
    """src/Denoiser.zig over the rnnoise_* C ABI (GPU, batch of one)."""

    def __init__(self, model=None):
        self.model = model
        self.h = lib().rnnoise_create(model.h if model is not None else None)
        if not self.h:
            raise FvadError("rnnoise_create failed: %s" % last_error())

    @staticmethod
    def get_frame_size():
        return lib().rnnoise_get_frame_size()

    def process_s16(self, frame):
        frame = np.ascontiguousarray(frame, np.float32)
        if frame.shape != (FRAME,):
            raise ValueError("InvalidFrameSize")
        out = np.zeros(FRAME, np.float32)
        vad = lib().rnnoise_process_frame(self.h, fptr(out), fptr(frame))
        return out, vad

    def denoise(self, samples):
        """Denoiser.denoise: normalised [-1,1] in, normalised out, returns (out, vad)."""
        samples = np.asarray(samples, np.float32)
        if samples.shape != (FRAME,):
            raise ValueError("InvalidFrameSize")
        scaled = samples * np.float32(32767)
        out, vad = self.process_s16(scaled)
        return out * (np.float32(1.0) / np.float32(32767)), vad

    def __del__(self):
        try:
            lib().rnnoise_destroy(self.h)
        except Exception:
            pass


def kiss_fftr(x):
    """kiss_fftr over the GPU compat shim; returns complex64[n/2+1]."""
    x = np.ascontiguousarray(x, np.float32)
    n = len(x)
    lenmem = C.c_size_t(1)
    if lib().kiss_fftr_alloc(n, 0, None, C.byref(lenmem)) is not None:
        raise FvadError("size probe must fail")
    if lenmem.value == 0:
        raise ValueError("unsupported nfft %d" % n)
    mem = C.create_string_buffer(lenmem.value)
    cfg = lib().kiss_fftr_alloc(n, 0, mem, C.byref(lenmem))
    if not cfg:
        raise FvadError("kiss_fftr_alloc failed")
    out = np.zeros(2 * (n // 2 + 1), np.float32)
    lib().kiss_fftr(cfg, fptr(x), out.ctypes.data_as(C.c_void_p))
    return out[0::2] + 1j * out[1::2]


class VADMachine:
    """src/AudioPipeline/VADMachine.zig (host decision logic)."""

    def __init__(self, cfg=None, n_channels=2, sample_rate=48000, fft_size=2048):
        c = cfg if cfg is not None else VadmConfig.default()
        self._cfg = c
        self.n_channels = n_channels
        h = C.c_void_p()
        _check(lib().fvad_vadm_create(C.byref(c), sample_rate, fft_size, n_channels, C.byref(h)), "fvad_vadm_create")
        self.h = h

    def bins(self):
        lo, hi = C.c_int(), C.c_int()
        lib().fvad_vadm_bins(self.h, C.byref(lo), C.byref(hi))
        return lo.value, hi.value

    def run(self, index, band_per_channel, vad, vol_ratio):
        b = np.ascontiguousarray(band_per_channel, np.float32)
        _check(lib().fvad_vadm_run(self.h, index, fptr(b), vad, vol_ratio), "fvad_vadm_run")

    def segments(self):
        n = lib().fvad_vadm_segments(self.h, None, 0)
        buf = (Segment * max(1, n))()
        lib().fvad_vadm_segments(self.h, buf, n)
        return [(s.sample_from, s.sample_to, s.debug_rnn_vad, s.debug_avg_speech_vol_ratio) for s in buf[:n]]

    def __del__(self):
        try:
            lib().fvad_vadm_destroy(self.h)
        except Exception:
            pass


# on_recording callback (fvad_recording_fn)
RECORDING_FN = C.CFUNCTYPE(None, C.c_void_p, F32P, C.c_size_t, C.c_uint64, C.c_int)


def recording_channel(channel_pcm):
    """Recorder.findBestChannel: index of the lowest-rmsVolume channel."""
    chans = [np.ascontiguousarray(c, np.float32) for c in channel_pcm]
    arr = (F32P * len(chans))(*[fptr(c) for c in chans])
    return lib().fvad_recording_channel(arr, len(chans), len(chans[0]))


class AudioPipeline:
    """src/AudioPipeline.zig for one stream (pushSamples -> VAD -> VADMachine)."""

    def __init__(self, model, n_channels=2, sample_rate=48000, device=0, main_cfg=None, alt_cfgs=(),
                 fft_size=2048, use_denoiser=True):
        self.model = model
        vc = VadConfig.make(fft_size, use_denoiser, main_cfg, tuple(alt_cfgs))
        self._keep = (vc,)
        self.n_alt = len(alt_cfgs)
        h = C.c_void_p()
        _check(lib().fvad_pipeline_create_ex(sample_rate, n_channels, model.h, device, C.byref(vc), C.byref(h)),
               "fvad_pipeline_create_ex")
        self.h = h

    def push_samples(self, channel_pcm):
        chans = [np.ascontiguousarray(c, np.float32) for c in channel_pcm]
        arr = (F32P * len(chans))(*[fptr(c) for c in chans])
        first = C.c_uint64()
        _check(lib().fvad_pipeline_push(self.h, arr, len(chans[0]), C.byref(first)), "fvad_pipeline_push")
        return first.value

    def record(self):
        """Attach the Recorder: completed main-machine segments are captured
        into self.recordings as (start_sample, channel, pcm) (on_recording)."""
        self.recordings = []

        def on_rec(ctx, pcm, n, start, channel):
            self.recordings.append((int(start), int(channel), np.ctypeslib.as_array(pcm, shape=(n,)).copy()))

        self._rec_cb = RECORDING_FN(on_rec)
        _check(lib().fvad_pipeline_set_recorder(self.h, C.cast(self._rec_cb, C.c_void_p), None),
               "fvad_pipeline_set_recorder")

    def segments(self, alt=-1):
        n = lib().fvad_pipeline_segments(self.h, alt, None, 0)
        buf = (Segment * max(1, n))()
        lib().fvad_pipeline_segments(self.h, alt, buf, n)
        return [(s.sample_from, s.sample_to, s.debug_rnn_vad, s.debug_avg_speech_vol_ratio) for s in buf[:n]]

    def __del__(self):
        try:
            lib().fvad_pipeline_destroy(self.h)
        except Exception:
            pass


class Multi:
    """Multi-stream simulator core: lock-step ticks, streams grouped by channel
    count and partitioned over devices (fvad_multi_create_ex)."""

    def __init__(self, model, n_streams, n_channels=2, devices=(0,), cfg=None, ticks_per_push=50, fft_size=2048,
                 use_denoiser=True, alt_cfgs=()):
        self.model = model
        self.n = n_streams
        d = np.ascontiguousarray(devices, np.int32)
        ch = np.ascontiguousarray([n_channels] * n_streams if np.isscalar(n_channels) else n_channels, np.int32)
        vc = VadConfig.make(fft_size, use_denoiser, cfg, tuple(alt_cfgs))
        self._keep = (d, ch, vc)
        h = C.c_void_p()
        _check(lib().fvad_multi_create_ex(n_streams, ch.ctypes.data_as(I32P), model.h, d.ctypes.data_as(I32P), len(d),
                                          C.byref(vc), ticks_per_push, C.byref(h)), "fvad_multi_create_ex")
        self.h = h

    def run_stream(self, streams, chunk=48000):
        """Pull each stream through fvad_multi_run_stream in reads of at most
        `chunk` frames (the simulator's streaming read loop)."""
        arrs = [np.ascontiguousarray(s, np.float32) for s in streams]
        pos = [0] * len(arrs)

        def read(ctx, s, dst, max_frames):
            a = arrs[s]
            k = min(max_frames, chunk, a.shape[1] - pos[s])
            for c in range(a.shape[0]):
                C.memmove(dst[c], a[c, pos[s]:].ctypes.data, k * 4)
            pos[s] += k
            return k

        cb = READ_FN(read)
        _check(lib().fvad_multi_run_stream(self.h, C.cast(cb, C.c_void_p), None), "fvad_multi_run_stream")

    def run(self, streams):
        """streams: list of planar float32 arrays [ch][len]."""
        arrs = [np.ascontiguousarray(s, np.float32) for s in streams]
        ptrs = (F32P * len(arrs))(*[fptr(a) for a in arrs])
        lens = (C.c_size_t * len(arrs))(*[a.shape[1] for a in arrs])
        _check(lib().fvad_multi_run(self.h, ptrs, lens), "fvad_multi_run")

    def segments(self, stream, machine=0):
        n = lib().fvad_multi_segments_alt(self.h, stream, machine, None, 0)
        buf = (Segment * max(1, n))()
        lib().fvad_multi_segments_alt(self.h, stream, machine, buf, n)
        return [(s.sample_from, s.sample_to, s.debug_rnn_vad, s.debug_avg_speech_vol_ratio) for s in buf[:n]]

    def __del__(self):
        try:
            lib().fvad_multi_destroy(self.h)
        except Exception:
            pass


def evaluate(vad_segs, ref_segs, ignore_shorter_than_sec=0.0, extrude_start=0.0, extrude_end=0.0, fill_gaps=0.0):
    v = np.ascontiguousarray(np.asarray(vad_segs, np.float32).reshape(-1, 2))
    r = np.ascontiguousarray(np.asarray(ref_segs, np.float32).reshape(-1, 2))
    cfg = StatConfig(ignore_shorter_than_sec, extrude_start, extrude_end, fill_gaps)
    out = SingleStats()
    _check(lib().fvad_eval_stats(fptr(v), len(v), fptr(r), len(r), C.byref(cfg), C.byref(out)), "fvad_eval_stats")
    return {n: getattr(out, n) for n in _STAT_FIELDS}


def aggregate(stats_list):
    arr = (SingleStats * max(1, len(stats_list)))()
    for i, s in enumerate(stats_list):
        for n in _STAT_FIELDS:
            setattr(arr[i], n, s[n])
    out = AggregateStats()
    lib().fvad_eval_aggregate(arr, len(stats_list), C.byref(out))
    return out


def parse_audacity(txt):
    b = txt.encode() if isinstance(txt, str) else txt
    n = lib().fvad_parse_audacity(b, len(b), None, 0)
    if n < 0:
        raise ValueError("malformed Audacity label text")
    out = np.zeros(2 * max(1, n), np.float32)
    lib().fvad_parse_audacity(b, len(b), fptr(out), n)
    return out[: 2 * n].reshape(-1, 2)
