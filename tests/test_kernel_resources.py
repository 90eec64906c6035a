"""The kernels' register / LDS budgets as DESIGN.md states them, checked on
the CPU from hipcc's resource remarks (device-only compiles for gfx950 with
the Makefile's flags): the occupancy each kernel's grid and co-residency plan
relies on, and no scratch spills except k_fused16's few (its 16 waves leave
128 VGPRs a wave).  A change that pushes a kernel over a
register boundary fails here before it costs a GPU run."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "formula-vad_amd")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "--offload-arch=gfx950", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"]
NO_SLP = {"fvad_wave.hip", "fvad_pitch.hip"}  # Makefile: built without SLP vectorisation

# kernel -> (waves per SIMD, max scratch-spilled VGPRs)
EXPECT = {
    "k_prep3": (4, 0), "k_plpc": (2, 0), "k_pcorr": (4, 0), "k_select": (4, 0), "k_rnn3": (4, 0),
    "k_fftAw": (3, 0), "k_pspecw": (4, 0), "k_synthw": (4, 0), "k_olafb": (3, 0), "k_vadm_hbm": (3, 0),
    "k_vadm_par": (2, 0), "k_gru16": (2, 0), "k_fused16": (4, 64),
}


def resources(src):
    cmd = [HIPCC] + FLAGS + (["-fno-slp-vectorize"] if src in NO_SLP else []) + \
          ["-c", os.path.join(PKG, "csrc", src), "-o", os.devnull]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600).stderr
    res, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: _ZN4fvad\d+(k_\w+?)E", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1).split(" ")[0] + ("_spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
    return res


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_kernel_register_budgets():
    got = {}
    for src in ("fvad_staged.hip", "fvad_pitch.hip", "fvad_wave.hip", "fvad_gru16.hip"):
        got.update(resources(src))
    for k, (occ, spill) in EXPECT.items():
        assert k in got, (k, sorted(got))
        r = got[k]
        assert r["Occupancy"] >= occ, (k, r)
        assert r["VGPRs_spill"] <= spill, (k, r)
        assert r["LDS"] <= 160 * 1024, (k, r)
    print({k: (got[k]["VGPRs"], got[k]["Occupancy"], got[k]["VGPRs_spill"], got[k]["LDS"]) for k in EXPECT})
