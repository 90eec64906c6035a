"""How many coarse-pitch lags must k_pcorr compute exactly?  (CPU study, not
part of the product.)

Reproduces rnnoise's coarse pitch search input (pitch_downsample of the
biquad-filtered pitch buffer, in float64 -- close enough for counting) on a
sample of the bench's synthetic streams and counts per frame:
  exact     lags surviving k_pcorr's current filter (prefix top-2 of the exact
            ratios, 0.1 % margin)
  approx_c  lags surviving an interval filter built from an approximate
            xcorr with |xcorr_approx - xcorr| <= c * sqrt(xx * Syy_k)
            (the Cauchy-Schwarz bound of any summation order's error)
  updates   lags that change find_best_pitch's state (the floor)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))


def frames_xlp(pcm, n_frames):
    # biquad (rnnoise: b_hp = {-2, 1}, a_hp = {-1.99599, .99600}) on x * 32767
    x = pcm.astype(np.float64) * 32767.0
    b0, b1 = -2.0, 1.0
    a0, a1 = -1.99599, 0.99600
    m0 = m1 = 0.0
    y = np.empty_like(x)
    for i, xi in enumerate(x):
        yi = xi + m0
        m0 = m1 + (b0 * xi - a0 * yi)
        m1 = b1 * xi - a1 * yi
        y[i] = yi
    buf = np.zeros(1728)
    out = []
    for f in range(n_frames):
        buf[:-480] = buf[480:]
        buf[-480:] = y[480 * f: 480 * (f + 1)]
        xl = np.empty(864)
        xl[1:] = .5 * (.5 * (buf[1:-1:2][:863] + buf[3::2][:863]) + buf[2::2][:863])
        xl[0] = .5 * (.5 * buf[1] + buf[0])
        out.append(xl)  # (the 5-tap LPC FIR is omitted: it does not change the counts' order)
    return out


def study(xl, cs=(2.0 ** -20, 2.0 ** -14, 2.0 ** -11, 2.0 ** -8)):
    x4 = xl[384::2][:240]
    y4 = xl[0::2][:432]
    xc = np.array([np.dot(x4, y4[k:k + 240]) for k in range(147)])
    syy = np.empty(147)
    s = 1 + np.dot(y4[:240], y4[:240])
    for k in range(147):
        syy[k] = s
        s = max(1.0, s + y4[k + 240] ** 2 - y4[k] ** 2)
    xx = np.dot(x4, x4)
    # exact scan: updates
    bn = [-1.0, -1.0]
    bd = [0.0, 0.0]
    upd = 0
    for k in range(147):
        if xc[k] > 0:
            num = (xc[k] * 1e-12) ** 2
            if num * bd[1] > bn[1] * syy[k]:
                upd += 1
                if num * bd[0] > bn[0] * syy[k]:
                    bn[1], bd[1] = bn[0], bd[0]
                    bn[0], bd[0] = num, syy[k]
                else:
                    bn[1], bd[1] = num, syy[k]
    rho = np.where(xc > 0, xc * xc / syy, -np.inf)

    def survivors(lo, hi):
        # keep k unless hi[k] < (second best lower bound before k) / 1.001
        m1 = m2 = -np.inf
        n = 0
        for k in range(147):
            if hi[k] != -np.inf and not (m2 > hi[k] * 1.001):
                n += 1
            v = lo[k]
            m2 = max(m2, min(m1, v))
            m1 = max(m1, v)
        return n

    res = {"exact": survivors(rho, rho), "updates": upd}
    for c in cs:
        e = c * np.sqrt(xx * syy)
        hi = np.where(xc + e > 0, (np.abs(xc) + e) ** 2 / syy, -np.inf)
        lo = np.where(xc - e > 0, (xc - e) ** 2 / syy, -np.inf)
        res["approx_2^%d" % round(np.log2(c))] = survivors(lo, hi)
    return res


def main(n_streams=6, n_frames=200):
    import fvad
    tot = {}
    nf = 0
    for sid in range(n_streams):
        pcm, _ = fvad.synth_stream(sid * 7 + 1, 480 * n_frames, 1)
        for xl in frames_xlp(pcm[0], n_frames)[4:]:
            r = study(xl)
            nf += 1
            for k, v in r.items():
                tot[k] = tot.get(k, 0) + v
    print({k: round(v / nf, 2) for k, v in tot.items()}, "frames", nf)


if __name__ == "__main__":
    main()
