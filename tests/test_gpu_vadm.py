"""Device VADMachine (k_vadm, VADMachine.zig:126-230 on the GPU) against the
host restatement (fvad_vadm_*, itself checked against the oracle in
test_host_cpu.py) fed the same engine outputs: segments and their debug
averages must be identical, for the default and an alternative config, over
ragged pushes of several streams.  Machines that all start from an initial
long-term average run on k_vadm_par (the push's long-term averages folded
side by side); an alternative machine without one sends the push through the
serial k_vadm_hbm walk; a 10 s long-term buffer (234 windows) wraps around
several times within the streams (the wrap branch of k_vadm_par), with a
sync point after every push so each push's machines take k_vadm_par (between
pushes the engine runs k_vadm_hbm; a sync point flushes the last push as
k_vadm_par) -- and once more without the syncs, so k_vadm_hbm's lazy folds
run over a buffer of pushed values that wraps (the production regime of a
stream past its first long_term_speech_avg_sec)."""
import numpy as np
import pytest

import parity_util as pu

pytestmark = pytest.mark.gpu


def host_segments(fvad_mod, outs, cfg, C, slot, stream):
    vm = fvad_mod.VADMachine(cfg, n_channels=C)
    wd = 0
    for o, valid in outs:
        for t in range(valid[stream]):
            if not o["win_flag"][t, stream]:
                continue
            vm.run(wd * 2048, o["band"][t, stream, :, slot], float(o["win_vad"][t, stream]),
                   float(o["win_ratio"][t, stream]))
            wd += 1
    return vm.segments()


@pytest.mark.parametrize("alt_init,alt_lt_sec,sync_each,defer_max,bound",
                         [(True, 180.0, False, 0, 0), (False, 180.0, False, 0, 0), (True, 10.0, True, 0, 0),
                          (True, 10.0, False, 0, 0), (True, 10.0, False, 1, 0), (True, 10.0, False, 7, 0),
                          (True, 10.0, False, 0, -1), (True, 180.0, False, 0, -1)])
def test_device_vadm_matches_host(fvad_mod, alt_init, alt_lt_sec, sync_each, defer_max, bound):
    """bound -1: FVAD_DEBUG_VADM_BOUND_SCALE infinite -- every long-term test
    the lazy walk's estimate would settle takes the exact fold instead (the
    branch the bound leaves open, fvad_staged.hip vadm_stream), counted with
    FVAD_DEBUG_VADM_COUNT."""
    m = fvad_mod.Model(seed=1)
    alt = fvad_mod.VadmConfig.default()
    alt.speech_min_freq, alt.speech_max_freq = 300.0, 3000.0
    alt.min_vad_duration_sec = 0.3
    alt.long_term_speech_avg_sec = alt_lt_sec
    if not alt_init:
        alt.has_initial_long_term_avg = 0
    ids, secs = [0, 4, 19, 42, 7], [70.0, 55.5, 40.0, 66.0, 12.0]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=64, bands=((4, 64), (13, 128)))
    eng.attach_vadm([fvad_mod.VadmConfig.default(), alt])
    if defer_max:  # the long-term fold owed across at most defer_max long pushes (1: every push)
        eng.set_debug(fvad_mod.DEBUG_VADM_DEFER_MAX, defer_max)
    if bound:
        eng.set_debug(fvad_mod.DEBUG_VADM_BOUND_SCALE, bound)
        eng.set_debug(fvad_mod.DEBUG_VADM_COUNT, 1)
    B, C = len(streams), 2
    lens = [x.shape[1] // 480 for x in streams]
    outs = []
    for t0 in range(0, max(lens), 64):
        nt = min(64, max(lens) - t0)
        pcm = np.zeros((nt, B, C, 480), np.float32)
        valid = np.zeros(B, np.int32)
        for s, x in enumerate(streams):
            v = max(0, min(nt, lens[s] - t0))
            valid[s] = v
            if v:
                pcm[:v, s] = x[:, t0 * 480:(t0 + v) * 480].reshape(C, v, 480).transpose(1, 0, 2)
        outs.append((eng.push(pcm, ticks_valid=valid), valid))
        if sync_each:
            eng.sync()  # a sync point per push: every push's machines run as k_vadm_par
    total = 0
    for s in range(B):
        for mi, (cfg, slot) in enumerate(((fvad_mod.VadmConfig.default(), 0), (alt, 1))):
            ref = host_segments(fvad_mod, outs, cfg, C, slot, s)
            got = eng.segments(s, mi)
            assert got == ref, (s, mi, got[:3], ref[:3])
            total += len(ref)
    assert total > 0
    if bound:  # the open branch ran, and nothing was settled from the estimate
        cnt = eng.debug_counts()
        assert cnt["open"] > 0 and cnt["settled"] == 0, cnt


@pytest.mark.parametrize("flavour", ["default", "always_par", "par_serial_fallback", "defer_max_5", "ragged",
                                     "bound_open", "bound_open_defer_max_5"])
def test_device_vadm_state_matches_oracle(fvad_mod, oracle_mod, flavour):
    """The whole device machine state (fvad_engine_vadm_snapshot: speech state
    and indices, RollingAverage last averages / write indices / counts, the
    tracked speech sums, segment count) and its RollingAverage buffers equal
    the oracle's VADMachine after the same windows.  default: k_vadm_hbm
    between pushes, k_vadm_par for the last one; always_par: every push's
    machine on k_vadm_par (FVAD_DEBUG_VADM_ALWAYS_PAR); par_serial_fallback:
    the same with every second stream forced through k_vadm_par's in-kernel
    serial walk (FVAD_DEBUG_VADM_PAR_SERIAL_EVERY = 2); defer_max_5: k_vadm_hbm
    folds once 5 long pushes are owed (FVAD_DEBUG_VADM_DEFER_MAX), so owed folds
    are resolved in the middle of pushes as well as by the sync point; ragged:
    three streams end early (3, 6 and 9.5 s of 14), so their machines owe a
    fold from their last pushes and have no ticks when the sync point's
    k_vadm_par resolves it; bound_open (also with defer_max_5): the lazy
    walk's bound made infinite (FVAD_DEBUG_VADM_BOUND_SCALE = -1), so every
    long-term test it would settle from the estimate runs the exact fold
    (vadm_stream's open branch), counted (FVAD_DEBUG_VADM_COUNT); default
    counts how its tests were decided and needs some settled by the bound."""
    m = fvad_mod.Model(seed=1)
    om = oracle_mod.Model(seed=1)
    ids = [0, 3, 19, 39, 7, 12, 59, 8]
    streams, _ = pu.make_streams(fvad_mod, ids, 14.0)
    if flavour == "ragged":
        for s, sec in ((1, 6.0), (4, 9.5), (6, 3.0)):
            streams[s] = np.ascontiguousarray(streams[s][:, :int(48000 * sec)])
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=50)
    eng.attach_vadm()
    if flavour in ("always_par", "par_serial_fallback"):
        eng.set_debug(fvad_mod.DEBUG_VADM_ALWAYS_PAR, 1)
    if flavour == "par_serial_fallback":
        eng.set_debug(fvad_mod.DEBUG_VADM_PAR_SERIAL_EVERY, 2)
    if flavour.endswith("defer_max_5"):
        eng.set_debug(fvad_mod.DEBUG_VADM_DEFER_MAX, 5)
    if flavour.startswith("bound_open"):
        eng.set_debug(fvad_mod.DEBUG_VADM_BOUND_SCALE, -1)
    eng.set_debug(fvad_mod.DEBUG_VADM_COUNT, 1)
    pu.engine_run(fvad_mod, eng, streams, 50, denoised=False)
    cnt = eng.debug_counts()
    print(flavour, cnt)
    if flavour.startswith("bound_open"):
        assert cnt["open"] > 0 and cnt["settled"] == 0, cnt
    elif flavour == "default":
        assert cnt["settled"] > 0, cnt
    for s, x in enumerate(streams):
        p = oracle_mod.Pipeline(2, om)
        for k in range(0, x.shape[1], 24000):
            p.push([x[0, k:k + 24000], x[1, k:k + 24000]])
        assert eng.vadm_snapshot(s) == p.vadm_snapshot(), s
        for which in range(3):
            assert np.array_equal(eng.vadm_rolling(s, which), p.vadm_rolling(which)), (s, which)
        assert eng.segments(s) == p.segments(), s


@pytest.mark.parametrize("negate_at", [60, 700])
def test_device_vadm_negative_entry_matches_host(fvad_mod, negate_at):
    """A band minimum the pipeline never produces -- window `negate_at` of every
    stream enters the machines negated (FVAD_DEBUG_VADM_NEGATE_AT) -- voids the
    lazy walk's bound (it holds for nonnegative terms), so the device machine
    folds exactly until that entry has left the long-term buffer (lt_neg) and
    then goes back to the lazy walk: the 10 s alternative machine (234
    entries) does both within these 40-70 s streams, the default 180 s one
    stays on the exact path.  Segments and their debug averages equal the
    host VADMachine's fed the same values (VADMachine.zig:126-230)."""
    m = fvad_mod.Model(seed=1)
    alt = fvad_mod.VadmConfig.default()
    alt.speech_min_freq, alt.speech_max_freq = 300.0, 3000.0
    alt.min_vad_duration_sec = 0.3
    alt.long_term_speech_avg_sec = 10.0
    ids, secs = [0, 4, 19, 42], [70.0, 55.5, 40.0, 66.0]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=64, bands=((4, 64), (13, 128)))
    eng.attach_vadm([fvad_mod.VadmConfig.default(), alt])
    eng.set_debug(fvad_mod.DEBUG_VADM_NEGATE_AT, negate_at)
    B, C = len(streams), 2
    lens = [x.shape[1] // 480 for x in streams]
    outs = []
    for t0 in range(0, max(lens), 64):
        nt = min(64, max(lens) - t0)
        pcm = np.zeros((nt, B, C, 480), np.float32)
        valid = np.zeros(B, np.int32)
        for s, x in enumerate(streams):
            v = max(0, min(nt, lens[s] - t0))
            valid[s] = v
            if v:
                pcm[:v, s] = x[:, t0 * 480:(t0 + v) * 480].reshape(C, v, 480).transpose(1, 0, 2)
        outs.append((eng.push(pcm, ticks_valid=valid), valid))
    total = 0
    for s in range(B):
        for mi, (cfg, slot) in enumerate(((fvad_mod.VadmConfig.default(), 0), (alt, 1))):
            vm = fvad_mod.VADMachine(cfg, n_channels=C)
            wd = 0
            for o, valid in outs:
                for t in range(valid[s]):
                    if not o["win_flag"][t, s]:
                        continue
                    band = np.array(o["band"][t, s, :, slot], np.float32)
                    if wd == negate_at:  # the machine sees -min over the channels
                        band = np.full(C, -band.min(), np.float32)
                    vm.run(wd * 2048, band, float(o["win_vad"][t, s]), float(o["win_ratio"][t, s]))
                    wd += 1
            assert wd > negate_at + 234, (s, wd)
            ref = vm.segments()
            got = eng.segments(s, mi)
            assert got == ref, (s, mi, got[:3], ref[:3])
            total += len(ref)
    assert total > 0
