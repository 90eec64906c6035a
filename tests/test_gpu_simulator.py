"""`fvad-simulator -i plan.json` end to end (simulator.zig:74-139): WAV +
Audacity labels in, report / Audacity txt out; segments and TP/FP/FN equal
the oracle's on the same inputs."""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, "formula-vad_amd", "lib", "fvad-simulator")


def write_wav(path, planar, pcm16=False):
    ch, n = planar.shape
    inter = planar.T.reshape(-1)
    if pcm16:
        data = np.clip(np.round(inter * 32767), -32768, 32767).astype("<i2").tobytes()
        fmt, bits = 1, 16
    else:
        data = inter.astype("<f4").tobytes()
        fmt, bits = 3, 32
    bps = bits // 8
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, fmt, ch, 48000, 48000 * ch * bps, ch * bps, bits)
    hdr += b"data" + struct.pack("<I", len(data))
    with open(path, "wb") as f:
        f.write(hdr + data)


def read_back(planar, pcm16):
    if not pcm16:
        return planar
    q = np.clip(np.round(planar * 32767), -32768, 32767).astype(np.int16)
    return (q.astype(np.float32) / np.float32(32768.0)).astype(np.float32)


def test_simulator_plan(fvad_mod, oracle_mod, tmp_path):
    ids, secs = [0, 4, 19], [40.0, 33.3, 25.0]
    plan = {"instances": [], "config": {"vad_config": {}, "output_dir": "sim-out", "preload_audio": False,
                                          "audio_read_frame_count": 48000, "unknown_field": 1}}
    truth = {}
    for k, (i, s) in enumerate(zip(ids, secs)):
        x, lab = fvad_mod.synth_stream(i, int(48000 * s), 2)
        pcm16 = k == 1
        write_wav(tmp_path / ("s%d.wav" % i), x, pcm16=pcm16)
        (tmp_path / ("s%d.txt" % i)).write_text("".join("%f\t%f\tspeech\n" % (a, b) for a, b in lab))
        plan["instances"].append({"name": "drv%d" % i, "audio_path": "s%d.wav" % i, "ref_path": "s%d.txt" % i})
        truth["drv%d" % i] = (read_back(x, pcm16), oracle_mod.parse_audacity(
            (tmp_path / ("s%d.txt" % i)).read_text()))
    (tmp_path / "plan.json").write_text(json.dumps(plan))
    js = tmp_path / "summary.json"
    env = dict(os.environ, FVAD_SIM_JSON=str(js))
    r = subprocess.run([SIM, "-i", str(tmp_path / "plan.json")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "=> Performance Report" in r.stdout and "Fowlkes-Mallows" in r.stdout
    out = json.loads(js.read_text())
    om = oracle_mod.Model(seed=1)
    for inst in out["instances"]:
        x, refs = truth[inst["name"]]
        p = oracle_mod.Pipeline(2, om)
        p.push([x[0], x[1]])
        ref_segs = [(a, b) for a, b, _, _ in p.segments()]
        assert [tuple(s) for s in inst["segments"]] == ref_segs, inst["name"]
        st = oracle_mod.evaluate([(a / 48000.0, b / 48000.0) for a, b in ref_segs], refs, 0.7, 5, 10, 5)
        assert np.float32(inst["tp"]) == np.float32(st["true_positives_sec"])
        assert np.float32(inst["fp"]) == np.float32(st["false_positives_sec"])
        assert np.float32(inst["fn"]) == np.float32(st["false_negatives_sec"])
    outdirs = list((tmp_path / "sim-out").iterdir())
    assert len(outdirs) == 1
    files = sorted(f.name for f in outdirs[0].iterdir())
    assert "report.txt" in files and "plan.json" in files and "drv0-audacity.txt" in files
    # Recorder: one mono float WAV per completed segment, NNN-<name>.wav, equal
    # to the oracle's capture (raw input of the segment on its lowest-RMS channel)
    n_rec = 0
    for inst in out["instances"]:
        x, _ = truth[inst["name"]]
        exp = oracle_mod.recordings([x[0], x[1]], [tuple(sg) for sg in inst["segments"]])
        for k, (start, ch, pcm) in enumerate(exp):
            got = read_wav_f32(outdirs[0] / ("%03d-%s.wav" % (k, inst["name"])))
            assert np.array_equal(got, pcm), (inst["name"], k)
            n_rec += 1
        assert not (outdirs[0] / ("%03d-%s.wav" % (len(exp), inst["name"]))).exists()
    assert n_rec > 0


def read_wav_f32(path):
    b = open(path, "rb").read()
    assert b[:4] == b"RIFF" and b[8:12] == b"WAVE"
    pos, fmt, data = 12, None, None
    while pos + 8 <= len(b):
        cid, sz = b[pos:pos + 4], struct.unpack("<I", b[pos + 4:pos + 8])[0]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", b[pos + 8:pos + 24])
        elif cid == b"data":
            data = b[pos + 8:pos + 8 + sz]
        pos += 8 + sz
    assert fmt[0] == 3 and fmt[1] == 1 and fmt[2] == 48000 and fmt[5] == 32
    return np.frombuffer(data, "<f4")


def test_simulator_bad_plan(tmp_path):
    (tmp_path / "plan.json").write_text('{"instances": [{"name": "a", "audio_path": "missing.wav", '
                                        '"ref_path": "missing.txt"}]}')
    r = subprocess.run([SIM, "-i", str(tmp_path / "plan.json")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Failed to initialize simulation" in r.stdout


@pytest.mark.parametrize("fft_size,use_denoiser,preload", [(1000, True, False), (2048, False, True),
                                                           (3000, False, False), (256, True, False),
                                                           (256, False, True)])
def test_simulator_vad_config(fvad_mod, oracle_mod, tmp_path, fft_size, use_denoiser, preload):
    """plan.json with a non-default VAD.Config (VAD.zig:17-23): fft_size,
    use_denoiser, alternative machines; instances of different channel counts
    (mono and stereo), streamed or preloaded.  Segments and TP/FP/FN equal the
    oracle's AudioPipeline with the same config."""
    alt = {"speech_threshold_factor": 9.0, "min_vad_duration_sec": 0.5}
    main = {"speech_threshold_factor": 15.0}
    plan = {"instances": [], "config": {"vad_config": {"fft_size": fft_size, "use_denoiser": use_denoiser,
                                                       "vad_machine_config": main,
                                                       "alt_vad_machine_configs": [alt]},
                                        "preload_audio": preload}}
    truth = {}
    for i, secs, ch in ((0, 41.0, 2), (7, 33.7, 1), (19, 28.0, 2)):
        x, lab = fvad_mod.synth_stream(i, int(48000 * secs), ch)
        write_wav(tmp_path / ("s%d.wav" % i), x)
        (tmp_path / ("s%d.txt" % i)).write_text("".join("%f\t%f\tspeech\n" % (a, b) for a, b in lab))
        plan["instances"].append({"name": "i%d" % i, "audio_path": "s%d.wav" % i, "ref_path": "s%d.txt" % i})
        truth["i%d" % i] = (x, oracle_mod.parse_audacity((tmp_path / ("s%d.txt" % i)).read_text()))
    (tmp_path / "plan.json").write_text(json.dumps(plan))
    js = tmp_path / "summary.json"
    r = subprocess.run([SIM, "-i", str(tmp_path / "plan.json")], capture_output=True, text=True,
                       env=dict(os.environ, FVAD_SIM_JSON=str(js)), timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(js.read_text())
    om = oracle_mod.Model(seed=1)
    mcfg = oracle_mod.VadmConfig.default()
    mcfg.speech_threshold_factor = 15.0
    acfg = oracle_mod.VadmConfig.default()
    acfg.speech_threshold_factor, acfg.min_vad_duration_sec = 9.0, 0.5
    for inst in out["instances"]:
        x, refs = truth[inst["name"]]
        p = oracle_mod.Pipeline(x.shape[0], om, fft_size=fft_size, use_denoiser=use_denoiser, main_cfg=mcfg,
                                alt_cfgs=(acfg,))
        for k in range(0, x.shape[1], 48000):
            p.push([x[c, k:k + 48000] for c in range(x.shape[0])])
        ref_segs = [(a, b) for a, b, _, _ in p.segments()]
        assert [tuple(s) for s in inst["segments"]] == ref_segs, inst["name"]
        st = oracle_mod.evaluate([(a / 48000.0, b / 48000.0) for a, b in ref_segs], refs, 0.7, 5, 10, 5)
        for k in ("tp", "fp", "fn"):
            key = {"tp": "true_positives_sec", "fp": "false_positives_sec", "fn": "false_negatives_sec"}[k]
            assert np.float32(inst[k]) == np.float32(st[key])


def test_multi_stream_reader_alt_machines(fvad_mod, oracle_mod):
    """fvad_multi_run_stream (the streaming read loop) with mono and stereo
    streams in one multi (two channel groups) and an alternative machine:
    main and alternative segments equal the oracle's."""
    m, om = fvad_mod.Model(seed=1), oracle_mod.Model(seed=1)
    specs = [(0, 30.0, 2), (1, 21.3, 1), (2, 30.0, 2), (19, 17.1, 1), (5, 26.0, 2)]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), c)[0] for i, s, c in specs]
    alt_f = fvad_mod.VadmConfig.default()
    alt_f.speech_threshold_factor = 9.0
    alt_o = oracle_mod.VadmConfig.default()
    alt_o.speech_threshold_factor = 9.0
    multi = fvad_mod.Multi(m, len(streams), [c for _, _, c in specs], devices=(0, 0), ticks_per_push=40,
                           alt_cfgs=(alt_f,))
    multi.run_stream(streams, chunk=48000 - 17)
    n = 0
    for s, x in enumerate(streams):
        p = oracle_mod.Pipeline(x.shape[0], om, alt_cfgs=(alt_o,))
        p.push([x[c] for c in range(x.shape[0])])
        assert multi.segments(s) == p.segments(), s
        assert multi.segments(s, 1) == p.segments(0), s
        n += len(p.segments()) + len(p.segments(0))
    assert n > 3
