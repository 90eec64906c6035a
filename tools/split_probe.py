#!/usr/bin/env python3
"""Split-GPU probe: the bench workload (2048 stereo streams x 50 ticks per
push) on one engine over every CU, against two engines of 1024 streams each
on disjoint CU masks (fvad_engine_config.cu_mask) running side by side, and
two unmasked engines.  Prints ms per push (all 2048 streams) per layout.
  python3 tools/split_probe.py [staged|fp16] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))


def half_masks(n_cu, parts=2, group=8):
    """CU i goes to part (i // group) % parts: every XCD keeps a share whether
    the mask's CU numbering runs XCD-major or interleaves the XCDs"""
    return [[i for i in range(n_cu) if (i // group) % parts == p] for p in range(parts)]


def run(layout, mode, steps, B=2048, T=50, P=4, group=8):
    import fvad
    import torch
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    m = fvad.Model(seed=1)
    if layout == "one":
        engs = [fvad.Engine(m, B, 2, max_ticks=T, mode=mode)]
        bases = [0]
    else:
        masks = half_masks(n_cu, 2, group) if layout.startswith("masked") else [None, None]
        engs = [fvad.Engine(m, B // 2, 2, max_ticks=T, mode=mode, cu_mask=mk) for mk in masks]
        bases = [0, B // 2]
    for e, b in zip(engs, bases):
        e.attach_vadm()
        e.load_synthetic(T, base=b, pushes=P)
    for _ in range(3):
        for e in engs:
            e.run_resident(T)
    for e in engs:
        e.sync()
        e.clear_times()
    t0 = time.perf_counter()
    for _ in range(steps):
        for e in engs:
            e.run_resident(T)
    for e in engs:
        e.sync()
    ms = 1000 * (time.perf_counter() - t0) / steps
    kt = engs[0].kernel_times()
    print("%-10s %-6s %7.3f ms/push  %.2f M frames/s  engine0 kernels %s" % (
        layout, mode, ms, B * 2 * T / ms / 1e3, {k: round(v, 3) for k, v in kt["kernels"].items()}), flush=True)
    del engs
    fvad.synth_cache_clear()


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "staged"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    for layout in ("one", "masked8", "unmasked", "one", "masked8"):
        run(layout, mode, steps, group=8)
