"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end for the C restatement in this directory (see oracle.h for the
citation map and parity status).  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import this module; the product
(formula-vad_amd/) never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

F32P = C.POINTER(C.c_float)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.ora_model_synthetic.restype = C.c_void_p
        L.ora_model_synthetic.argtypes = [C.c_uint64]
        L.ora_model_from_text.restype = C.c_void_p
        L.ora_model_from_text.argtypes = [C.c_char_p]
        L.ora_model_free.argtypes = [C.c_void_p]
        L.ora_model_blob.restype = C.c_size_t
        L.ora_model_blob.argtypes = [C.c_void_p, C.c_void_p]
        L.ora_rnnoise_create.restype = C.c_void_p
        L.ora_rnnoise_create.argtypes = [C.c_void_p]
        L.ora_rnnoise_destroy.argtypes = [C.c_void_p]
        L.ora_rnnoise_process_frame.restype = C.c_float
        L.ora_rnnoise_process_frame.argtypes = [C.c_void_p, F32P, F32P]
        L.ora_rnnoise_set_bypass.argtypes = [C.c_void_p, C.c_int]
        L.ora_rnnoise_debug.argtypes = [C.c_void_p, C.POINTER(C.c_int), F32P, C.POINTER(C.c_int), F32P]
        L.ora_tables.argtypes = [F32P, F32P, F32P]
        L.ora_fft960.argtypes = [F32P, F32P]
        L.ora_kiss_fftr_alloc.restype = C.c_void_p
        L.ora_kiss_fftr_alloc.argtypes = [C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_size_t)]
        L.ora_kiss_fftr.argtypes = [C.c_void_p, F32P, F32P]
        L.ora_hann_periodic.argtypes = [F32P, C.c_int]
        L.ora_window_norm_factor.restype = C.c_float
        L.ora_window_norm_factor.argtypes = [F32P, C.c_int]
        L.ora_fftzig.restype = C.c_int
        L.ora_fftzig.argtypes = [C.c_int, F32P, F32P, F32P]
        L.ora_rms_volume.restype = C.c_float
        L.ora_rms_volume.argtypes = [F32P, C.c_int]
        L.ora_recording_channel.restype = C.c_int
        L.ora_recording_channel.argtypes = [C.POINTER(F32P), C.c_int, C.c_int]
        L.ora_segwriter_write.restype = C.c_size_t
        L.ora_segwriter_write.argtypes = [C.c_void_p, F32P, C.c_size_t, F32P, C.c_size_t, C.c_size_t, C.c_long]
        L.ora_ring_write.restype = C.c_size_t
        L.ora_ring_write.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_size_t, C.c_size_t, C.c_size_t]
        L.ora_vadm_config_default.argtypes = [C.c_void_p]
        L.ora_pipeline_create.restype = C.c_void_p
        L.ora_pipeline_create.argtypes = [C.c_int, C.c_int, C.c_size_t, C.c_int, C.c_int, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_int]
        L.ora_pipeline_destroy.argtypes = [C.c_void_p]
        L.ora_pipeline_push.restype = C.c_uint64
        L.ora_pipeline_push.argtypes = [C.c_void_p, C.POINTER(F32P), C.c_size_t]
        L.ora_pipeline_segments.restype = C.c_size_t
        L.ora_pipeline_segments.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
        L.ora_pipeline_vadm_snapshot.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.ora_pipeline_vadm_rolling.restype = C.c_size_t
        L.ora_pipeline_vadm_rolling.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t]
        L.ora_pipeline_enable_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                                F32P, C.c_size_t]
        L.ora_pipeline_trace_counts.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.ora_evaluate.restype = C.c_int
        L.ora_evaluate.argtypes = [F32P, C.c_size_t, F32P, C.c_size_t, C.c_void_p, C.c_void_p]
        L.ora_aggregate.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.ora_calc_false_positive_sec.restype = C.c_float
        L.ora_calc_false_positive_sec.argtypes = [C.c_float, C.c_float, F32P, C.c_size_t, C.c_void_p]
        L.ora_parse_audacity.restype = C.c_long
        L.ora_parse_audacity.argtypes = [C.c_char_p, C.c_size_t, F32P, C.c_size_t]
        L.ora_bench_denoise.restype = C.c_double
        L.ora_bench_denoise.argtypes = [C.c_void_p, F32P, C.c_int, C.c_int, C.c_int, C.c_int, F32P]
        _lib = L
    return _lib


def fptr(a):
    return a.ctypes.data_as(F32P)


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
        lib().ora_vadm_config_default(C.byref(c))
        return c


class Segment(C.Structure):
    _fields_ = [("sample_from", C.c_uint64), ("sample_to", C.c_uint64),
                ("debug_rnn_vad", C.c_float), ("debug_avg_speech_vol_ratio", C.c_float)]


class VadmSnapshot(C.Structure):
    """ora_vadm_snapshot (oracle.h): the machine's whole state."""
    _fields_ = [("speech_state", C.c_int), ("speech_start", C.c_uint64), ("speech_end", C.c_uint64),
                ("windows", C.c_uint64), ("avg", C.c_double * 3), ("write_idx", C.c_uint64 * 3),
                ("written", C.c_uint64 * 3), ("speech_rnn_vad", C.c_float), ("speech_vol_ratio", C.c_float),
                ("speech_rnn_vad_count", C.c_uint64), ("speech_vol_ratio_count", C.c_uint64),
                ("n_segments", C.c_uint64)]

    def as_dict(self):
        return {n: (list(getattr(self, n)) if n in ("avg", "write_idx", "written") else getattr(self, n))
                for n, _ in self._fields_}


class FrameTrace(C.Structure):
    _fields_ = [("frame_index", C.c_uint64), ("vad_low", C.c_float), ("vol_ratio", C.c_float)]


class WindowTrace(C.Structure):
    _fields_ = [("index", C.c_uint64), ("band", C.c_float * 8), ("vol_ratio", C.c_float), ("vad", C.c_float)]


class StatConfig(C.Structure):
    _fields_ = [("ignore_shorter_than_sec", C.c_float), ("extrude_start", C.c_float),
                ("extrude_end", C.c_float), ("fill_gaps", C.c_float)]


class SingleStats(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "total_positives_sec", "true_positives_sec", "false_positives_sec", "false_negatives_sec",
        "true_positive_rate", "false_negative_rate", "false_discovery_rate", "precision",
        "fm_index", "f_score", "f_score_beta")]


class AggStat(C.Structure):
    _fields_ = [("overall", C.c_float), ("min", C.c_float), ("max", C.c_float), ("avg", C.c_float)]


class AggregateStats(C.Structure):
    _fields_ = [("total_positives_sec", C.c_float), ("true_positives_sec", C.c_float),
                ("false_positives_sec", C.c_float), ("false_negatives_sec", C.c_float),
                ("true_positive_rate", AggStat), ("false_negative_rate", AggStat),
                ("false_discovery_rate", AggStat), ("precision", AggStat),
                ("fm_index", C.c_float), ("f_score", C.c_float), ("f_score_beta", C.c_float)]


class Model:
    def __init__(self, seed=None, path=None):
        L = lib()
        if path is not None:
            self.h = L.ora_model_from_text(path.encode())
        else:
            self.h = L.ora_model_synthetic(seed if seed is not None else 0)
        if not self.h:
            raise RuntimeError("oracle: model load failed")

    def blob(self):
        n = lib().ora_model_blob(self.h, None)
        b = np.zeros(n, dtype=np.int8)
        lib().ora_model_blob(self.h, b.ctypes.data_as(C.c_void_p))
        return b

    def __del__(self):
        try:
            lib().ora_model_free(self.h)
        except Exception:
            pass


class Denoiser:
    """rnnoise state (s16-scaled frames of 480)."""

    def __init__(self, model):
        self.model = model
        self.h = lib().ora_rnnoise_create(model.h)

    def process(self, frame):
        frame = np.ascontiguousarray(frame, dtype=np.float32)
        out = np.zeros(480, dtype=np.float32)
        vad = lib().ora_rnnoise_process_frame(self.h, fptr(out), fptr(frame))
        return out, vad

    def set_bypass(self, b):
        lib().ora_rnnoise_set_bypass(self.h, int(b))

    def debug(self):
        p = C.c_int()
        g = C.c_float()
        s = C.c_int()
        f = np.zeros(42, dtype=np.float32)
        lib().ora_rnnoise_debug(self.h, C.byref(p), C.byref(g), C.byref(s), fptr(f))
        return p.value, g.value, s.value, f

    def __del__(self):
        try:
            lib().ora_rnnoise_destroy(self.h)
        except Exception:
            pass


def tables():
    hw = np.zeros(480, np.float32)
    dct = np.zeros(484, np.float32)
    tt = np.zeros(201, np.float32)
    lib().ora_tables(fptr(hw), fptr(dct), fptr(tt))
    return hw, dct.reshape(22, 22), tt


def fft960(x):
    x = np.ascontiguousarray(x, dtype=np.complex64)
    inp = np.zeros(1920, np.float32)
    inp[0::2] = x.real
    inp[1::2] = x.imag
    out = np.zeros(1920, np.float32)
    lib().ora_fft960(fptr(inp), fptr(out))
    return out[0::2] + 1j * out[1::2]


def kiss_fftr(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = len(x)
    lenmem = C.c_size_t(1)
    assert lib().ora_kiss_fftr_alloc(n, 0, None, C.byref(lenmem)) is None
    mem = C.create_string_buffer(lenmem.value)
    cfg = lib().ora_kiss_fftr_alloc(n, 0, mem, C.byref(lenmem))
    assert cfg
    out = np.zeros(2 * (n // 2 + 1), np.float32)
    lib().ora_kiss_fftr(cfg, fptr(x), fptr(out))
    return out[0::2] + 1j * out[1::2], out


def hann_periodic(n):
    w = np.zeros(n, np.float32)
    lib().ora_hann_periodic(fptr(w), n)
    return w


def fftzig(samples, window):
    samples = np.ascontiguousarray(samples, np.float32)
    window = np.ascontiguousarray(window, np.float32)
    mag = np.zeros(len(samples) // 2 + 1, np.float32)
    rc = lib().ora_fftzig(len(samples), fptr(samples), fptr(window), fptr(mag))
    if rc != 0:
        raise ValueError("FFT.fft error %d" % rc)
    return mag


def rms_volume(x):
    x = np.ascontiguousarray(x, np.float32)
    return lib().ora_rms_volume(fptr(x), len(x))


def recording_channel(channel_pcm):
    """Recorder.findBestChannel (Recorder.zig:95-110)."""
    chans = [np.ascontiguousarray(c, np.float32) for c in channel_pcm]
    arr = (F32P * len(chans))(*[fptr(c) for c in chans])
    return lib().ora_recording_channel(arr, len(chans), len(chans[0]))


def recordings(channel_pcm, segments):
    """What AudioPipeline's Recorder hands to on_recording (AudioPipeline.zig:
    134-195, Recorder.zig:52-146): for each completed main-machine segment
    (sample_from, sample_to, ...) -- whose bounds are VADMachine's
    getOffsetRecordingStart/End, the capture's start and finalize sample -- the
    pushed input of [sample_from, sample_to) on its lowest-RMS channel, as
    (start_sample, channel, pcm)."""
    out = []
    for seg in segments:
        a, b = int(seg[0]), int(seg[1])
        sl = [np.ascontiguousarray(c[a:b], np.float32) for c in channel_pcm]
        ch = recording_channel(sl)
        out.append((a, ch, sl[ch].copy()))
    return out


class Pipeline:
    """AudioPipeline + VAD + VADMachine restatement with an optional trace."""

    def __init__(self, n_channels, model, fft_size=2048, use_denoiser=True, buffer_length=0,
                 main_cfg=None, alt_cfgs=(), trace_frames=0, trace_windows=0, trace_denoised=0):
        self.model = model
        self.n_channels = n_channels
        main = main_cfg if main_cfg is not None else VadmConfig.default()
        self._main = main
        alts = (VadmConfig * max(1, len(alt_cfgs)))(*alt_cfgs) if alt_cfgs else None
        self._alts = alts
        self.n_alt = len(alt_cfgs)
        self.h = lib().ora_pipeline_create(n_channels, 48000, buffer_length, fft_size, int(use_denoiser),
                                           model.h if model is not None else None, C.byref(main),
                                           alts, self.n_alt)
        if not self.h:
            raise ValueError("oracle: pipeline init failed")
        self.tf = (FrameTrace * max(1, trace_frames))()
        self.tw = (WindowTrace * max(1, trace_windows))()
        self.tden = np.zeros((n_channels, max(1, trace_denoised)), np.float32)
        lib().ora_pipeline_enable_trace(self.h, self.tf if trace_frames else None, trace_frames,
                                        self.tw if trace_windows else None, trace_windows,
                                        fptr(self.tden) if trace_denoised else None, trace_denoised)

    def push(self, pcm):
        pcm = [np.ascontiguousarray(c, np.float32) for c in pcm]
        arr = (F32P * len(pcm))(*[fptr(c) for c in pcm])
        return lib().ora_pipeline_push(self.h, arr, len(pcm[0]))

    def segments(self, alt=-1):
        n = lib().ora_pipeline_segments(self.h, alt, None, 0)
        buf = (Segment * max(1, n))()
        lib().ora_pipeline_segments(self.h, alt, buf, n)
        return [(s.sample_from, s.sample_to, s.debug_rnn_vad, s.debug_avg_speech_vol_ratio) for s in buf[:n]]

    def vadm_snapshot(self, alt=-1):
        s = VadmSnapshot()
        lib().ora_pipeline_vadm_snapshot(self.h, alt, C.byref(s))
        return s.as_dict()

    def vadm_rolling(self, which, alt=-1):
        """RollingAverage.data of the machine: which 0 long_term, 1 short_term, 2 ratio."""
        n = lib().ora_pipeline_vadm_rolling(self.h, alt, which, None, 0)
        out = np.zeros(n, np.float64)
        lib().ora_pipeline_vadm_rolling(self.h, alt, which, out.ctypes.data_as(C.c_void_p), n)
        return out

    def trace(self):
        nf = C.c_size_t()
        nw = C.c_size_t()
        lib().ora_pipeline_trace_counts(self.h, C.byref(nf), C.byref(nw))
        # the trace structs read in place (same field layout: 16 and 48 bytes)
        fdt = np.dtype([("index", np.uint64), ("vad", np.float32), ("ratio", np.float32)])
        wdt = np.dtype([("index", np.uint64), ("band", np.float32, 8), ("ratio", np.float32), ("vad", np.float32)])
        assert fdt.itemsize == C.sizeof(FrameTrace) and wdt.itemsize == C.sizeof(WindowTrace)
        frames = np.frombuffer(self.tf, dtype=fdt, count=nf.value).copy()
        wins = np.frombuffer(self.tw, dtype=wdt, count=nw.value).copy()
        return frames, wins

    def __del__(self):
        try:
            lib().ora_pipeline_destroy(self.h)
        except Exception:
            pass


def evaluate(vad_segs, ref_segs, ignore_shorter_than_sec=0.0, extrude_start=0.0, extrude_end=0.0,
             fill_gaps=0.0):
    v = np.ascontiguousarray(np.asarray(vad_segs, np.float32).reshape(-1, 2))
    r = np.ascontiguousarray(np.asarray(ref_segs, np.float32).reshape(-1, 2))
    cfg = StatConfig(ignore_shorter_than_sec, extrude_start, extrude_end, fill_gaps)
    out = SingleStats()
    lib().ora_evaluate(fptr(v), len(v), fptr(r), len(r), C.byref(cfg), C.byref(out))
    return {n: getattr(out, n) for n, _ in SingleStats._fields_}


def aggregate(stats_list):
    arr = (SingleStats * len(stats_list))()
    for i, s in enumerate(stats_list):
        for n, _ in SingleStats._fields_:
            setattr(arr[i], n, s[n])
    out = AggregateStats()
    lib().ora_aggregate(arr, len(stats_list), C.byref(out))
    return out


def calc_false_positive_sec(vad_from, vad_to, refs, extrude_start=0, extrude_end=0, fill_gaps=0):
    r = np.ascontiguousarray(np.asarray(refs, np.float32).reshape(-1, 2))
    cfg = StatConfig(0, extrude_start, extrude_end, fill_gaps)
    return lib().ora_calc_false_positive_sec(vad_from, vad_to, fptr(r), len(r), C.byref(cfg))


def parse_audacity(txt):
    b = txt.encode() if isinstance(txt, str) else txt
    n = lib().ora_parse_audacity(b, len(b), None, 0)
    if n < 0:
        raise ValueError("parse error")
    out = np.zeros(2 * max(1, n), np.float32)
    lib().ora_parse_audacity(b, len(b), fptr(out), n)
    return out[: 2 * n].reshape(-1, 2)


def bench_denoise(model, pcm, n_threads=1, want_vad=False):
    """pcm: [frames][streams][ch][480] s16-scaled float32. Returns (seconds, vad[frames][streams])."""
    pcm = np.ascontiguousarray(pcm, np.float32)
    T, S, Ch, _ = pcm.shape
    vad = np.zeros((T, S), np.float32) if want_vad else None
    secs = lib().ora_bench_denoise(model.h, fptr(pcm), S, Ch, T, n_threads,
                                   fptr(vad) if want_vad else None)
    return secs, vad


def _bench_lib(path):
    L = C.CDLL(path)
    L.ora_bench_pipeline.restype = C.c_double
    L.ora_bench_pipeline.argtypes = [C.c_void_p, F32P, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_int,
                                     C.POINTER(C.c_uint64)]
    L.ora_model_synthetic.restype = C.c_void_p
    L.ora_model_synthetic.argtypes = [C.c_uint64]
    L.ora_model_free.argtypes = [C.c_void_p]
    return L


def native_lib():
    """The -O3 -march=native flavour of the restatement for the CPU baseline,
    built on the host that runs it (tag = this host's CPU model)."""
    import hashlib
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    tag = hashlib.sha1(model.encode()).hexdigest()[:10]
    out = os.path.join(_HERE, "_build", "liboracle_native_%s.so" % tag)
    subprocess.check_call(["make", "-s", "-C", _HERE, "native", "NATIVE_OUT=_build/" + os.path.basename(out)])
    return _bench_lib(out), model


def bench_pipeline(pcm, chunk=24000, n_threads=1, seed=1, L=None):
    """pcm: [streams][ch][n] float32 in [-1, 1].  Runs the whole per-stream path
    (ora_bench_pipeline).  Returns (seconds, counts{frames, silent, fine_lags,
    rd_cands})."""
    L = L or _bench_lib(_LIB_PATH)
    pcm = np.ascontiguousarray(pcm, np.float32)
    S, Ch, n = pcm.shape
    m = L.ora_model_synthetic(seed)
    cnt = (C.c_uint64 * 4)()
    try:
        secs = L.ora_bench_pipeline(m, fptr(pcm), S, Ch, n, chunk, n_threads, cnt)
    finally:
        L.ora_model_free(m)
    if secs < 0:
        raise ValueError("ora_bench_pipeline: bad arguments")
    return secs, dict(zip(("frames", "silent", "fine_lags", "rd_cands"), [int(c) for c in cnt]))
