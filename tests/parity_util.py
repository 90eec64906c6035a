"""Helpers shared by the parity tests: run the same synthetic streams through
the CPU oracle (checker) and through the HIP engine (product)."""
import numpy as np

FRAME = 480


def make_streams(fvad, ids, seconds, n_channels=2):
    out, labels = [], []
    for sid in ids:
        x, lab = fvad.synth_stream(sid, int(48000 * seconds), n_channels)
        out.append(x)
        labels.append(lab)
    return out, labels


def oracle_run(oracle, om, streams, denoised=True):
    res = []
    for x in streams:
        Ch, n = x.shape
        frames = n // FRAME
        p = oracle.Pipeline(Ch, om, trace_frames=frames + 1, trace_windows=frames // 4 + 2,
                            trace_denoised=(frames * FRAME if denoised else 0))
        for k in range(0, n, 48000):
            p.push([x[c, k:k + 48000] for c in range(Ch)])
        fr, wi = p.trace()
        res.append({"frames": fr, "windows": wi, "segments": p.segments(),
                    "denoised": p.tden[:, : frames * FRAME].copy() if denoised else None})
    return res


def engine_run(fvad, engine, streams, chunk_ticks, denoised=True):
    B = len(streams)
    Ch = streams[0].shape[0]
    lens = [x.shape[1] // FRAME for x in streams]
    T = max(lens)
    outs = []
    for t0 in range(0, T, chunk_ticks):
        nt = min(chunk_ticks, T - t0)
        pcm = np.zeros((nt, B, Ch, FRAME), np.float32)
        valid = np.zeros(B, np.int32)
        for s, x in enumerate(streams):
            v = max(0, min(nt, lens[s] - t0))
            valid[s] = v
            if v:
                seg = x[:, t0 * FRAME:(t0 + v) * FRAME].reshape(Ch, v, FRAME)
                pcm[:v, s] = seg.transpose(1, 0, 2)
        outs.append((engine.push(pcm, ticks_valid=valid, denoised=denoised), valid))
    W = getattr(engine, "wpt", 1)
    per = []
    for s in range(B):
        vad, ratio, wf, wr, wv, band, den = [], [], [], [], [], [], []
        for o, valid in outs:
            v = valid[s]
            cnt = o["win_flag"][:v, s]
            vad.append(o["vad"][:v, s])
            ratio.append(o["ratio"][:v, s])
            wf.append(cnt)
            wr.append(tick_windows(o["win_ratio"][:v, s], cnt, W))
            wv.append(tick_windows(o["win_vad"][:v, s], cnt, W))
            band.append(tick_windows(o["band"][:v, s], cnt, W))
            if denoised:
                den.append(o["denoised"][:v, s])
        r = {"vad": np.concatenate(vad), "ratio": np.concatenate(ratio), "win_flag": np.concatenate(wf),
             "win_ratio": np.concatenate(wr), "win_vad": np.concatenate(wv), "band": np.concatenate(band)}
        if denoised:
            d = np.concatenate(den)  # [T][Ch][480]
            r["denoised"] = d.transpose(1, 0, 2).reshape(Ch, -1)
        per.append(r)
    return per


def tick_windows(x, counts, W):
    """The completed windows of one stream's ticks, in sample order: x is
    [ticks]... (W == 1) or [ticks][W]... (window slots), counts the ticks'
    win_flag (windows completed per tick)."""
    counts = np.asarray(counts)
    if W == 1:
        return x[counts.astype(bool)]
    return x[np.arange(W)[None, :] < counts[:, None]]


def first_mismatch(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    ne = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
    return int(ne[0]) if len(ne) else -1
