#!/usr/bin/env python3
"""Regenerate tests/golden/oracle_seed1.npz + oracle_seed1.json.

Golden vectors of the hot path produced by the CPU oracle (oracle/, the C
restatement of rnnoise + FFT.zig + VAD.zig, see oracle/oracle.h) with the
deterministic synthetic model (seed 1) on deterministic synthetic streams
(fvad_synth_stream).  Inputs are not stored: each case records the stream id,
length and the SHA-256 of the generated input so drift in the generator is
detected.  Outputs stored per case:
  vad[T], ratio[T]                      per tick (VAD.zig:253-296)
  win_band[W][C], win_ratio[W], win_vad[W]  per completed 2048-window
  den_head[C][960], den_sha256          denoised PCM (normalised)
  segments                              VADMachine segments (VADMachine.zig)
Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))

CASES = [  # name, stream id, seconds, channels
    ("stereo_id0_6s", 0, 6.0, 2),
    ("stereo_id19_7s_digital_silence", 19, 7.0, 2),
    ("mono_id3_4s", 3, 4.0, 1),
    ("stereo_id42_40s_segments", 42, 40.0, 2),
]
MODEL_SEED = 1


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_case(oracle, om, fvad, sid, secs, ch):
    x, _ = fvad.synth_stream(sid, int(48000 * secs), ch)
    frames = x.shape[1] // 480
    p = oracle.Pipeline(ch, om, trace_frames=frames + 1, trace_windows=frames // 4 + 2,
                        trace_denoised=frames * 480)
    for k in range(0, x.shape[1], 48000):
        p.push([x[c, k:k + 48000] for c in range(ch)])
    fr, wi = p.trace()
    den = p.tden[:, :frames * 480].copy()
    return x, {
        "vad": np.asarray(fr["vad"], np.float32), "ratio": np.asarray(fr["ratio"], np.float32),
        "win_band": np.asarray(wi["band"][:, :ch], np.float32), "win_ratio": np.asarray(wi["ratio"], np.float32),
        "win_vad": np.asarray(wi["vad"], np.float32), "den_head": den[:, :960].astype(np.float32),
        "den_sha256": sha(den.astype(np.float32)),
        "segments": [[int(a), int(b)] for a, b, _, _ in p.segments()],
    }


def main():
    import oracle
    import fvad
    om = oracle.Model(seed=MODEL_SEED)
    arrays, meta = {}, {"model_seed": MODEL_SEED, "model_blob_sha256": sha(om.blob()), "cases": {}}
    for name, sid, secs, ch in CASES:
        x, r = run_case(oracle, om, fvad, sid, secs, ch)
        for k in ("vad", "ratio", "win_band", "win_ratio", "win_vad", "den_head"):
            arrays["%s__%s" % (name, k)] = r[k]
        meta["cases"][name] = {"stream_id": sid, "seconds": secs, "channels": ch, "input_sha256": sha(x),
                               "den_sha256": r["den_sha256"], "segments": r["segments"],
                               "ticks": int(len(r["vad"])), "windows": int(len(r["win_vad"]))}
    np.savez_compressed(os.path.join(HERE, "oracle_seed1.npz"), **arrays)
    with open(os.path.join(HERE, "oracle_seed1.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps({k: (v["ticks"], v["windows"], len(v["segments"])) for k, v in meta["cases"].items()}))


if __name__ == "__main__":
    main()
