"""Several engines on one GPU sharing their side streams
(fvad_engine_share_streams): a GPU's streams split into sub-partitions that
push concurrently must give exactly the outputs, segments and VADMachine
state of one engine over all of them, whatever the order the
engines are destroyed in."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FRAME = 480
OUT_KEYS = ("vad", "ratio", "win_flag", "win_ratio", "win_vad", "band")


def _pushes(fvad_mod, ids, secs, nt_push):
    streams = [fvad_mod.synth_stream(i, int(48000 * secs), 2)[0] for i in ids]
    n = streams[0].shape[1] // FRAME
    out = []
    for t0 in range(0, n, nt_push):
        nt = min(nt_push, n - t0)
        pcm = np.zeros((nt, len(streams), 2, FRAME), np.float32)
        for s, x in enumerate(streams):
            pcm[:, s] = x[:, t0 * FRAME:(t0 + nt) * FRAME].reshape(2, nt, FRAME).transpose(1, 0, 2)
        out.append(pcm)
    return out


@pytest.mark.parametrize("which", [3, 1])
def test_shared_streams_equal_one_engine(fvad_mod, which):
    m = fvad_mod.Model(seed=1)
    ids = list(range(40, 52))
    nA = 5  # sub-partitions of unequal size
    pushes = _pushes(fvad_mod, ids, 5.0, 50)
    ref = fvad_mod.Engine(m, len(ids), 2, max_ticks=50)
    ref.attach_vadm()
    want = [ref.push(p) for p in pushes]
    a = fvad_mod.Engine(m, nA, 2, max_ticks=50)
    a.attach_vadm()
    b = fvad_mod.Engine(m, len(ids) - nA, 2, max_ticks=50)
    b.attach_vadm()
    b.share_streams(a, which)
    # interleaved, up to two pushes in flight per engine (no synchronisation
    # between the engines' pushes)
    got_a, got_b, depth = [], [], 0
    for p in pushes:
        if depth == 2:
            got_a.append(a.collect())
            got_b.append(b.collect())
            depth -= 1
        a.submit(np.ascontiguousarray(p[:, :nA]))
        b.submit(np.ascontiguousarray(p[:, nA:]))
        depth += 1
    while depth:
        got_a.append(a.collect())
        got_b.append(b.collect())
        depth -= 1
    for w, ga, gb in zip(want, got_a, got_b):
        for k in OUT_KEYS:
            np.testing.assert_array_equal(np.concatenate([ga[k], gb[k]], axis=1), w[k], err_msg=k)
    for s in range(len(ids)):
        e, j = (a, s) if s < nA else (b, s - nA)
        assert e.segments(j) == ref.segments(s), s
        assert repr(e.vadm_snapshot(j)) == repr(ref.vadm_snapshot(s)), s  # bitwise (nan-safe)
    # the engine that created the shared streams goes first; b keeps them
    del a
    more = _pushes(fvad_mod, ids, 1.0, 50)
    for p in more:
        w = ref.push(p)
        g = b.push(np.ascontiguousarray(p[:, nA:]))
        for k in OUT_KEYS:
            np.testing.assert_array_equal(g[k], w[k][:, nA:], err_msg=k)
    for s in range(nA, len(ids)):
        assert b.segments(s - nA) == ref.segments(s), s


def test_share_streams_rejects_bad_arguments(fvad_mod):
    m = fvad_mod.Model(seed=1)
    a = fvad_mod.Engine(m, 2, 2, max_ticks=4)
    b = fvad_mod.Engine(m, 2, 2, max_ticks=4)
    with pytest.raises(fvad_mod.FvadError):
        b.share_streams(a, 2)  # no VADMachines attached
    with pytest.raises(fvad_mod.FvadError):
        b.share_streams(b, 1)
    with pytest.raises(fvad_mod.FvadError):
        b.share_streams(a, 4)
    b.share_streams(a, 1)
