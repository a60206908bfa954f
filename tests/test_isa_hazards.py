"""The fused-DPP fmacs of the diagonal-tile pivot (inline asm) keep the DPP read wait states in the
compiled gfx950 ISA (tools/dpp_hazards.py).  CPU only: hipcc cross-compiles to assembly."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_fused_dpp_fmacs_have_their_wait_states(tmp_path):
    import dpp_hazards
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "linalg.s"
    subprocess.check_call([hipcc, "-w", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "--cuda-device-only", "-S", os.path.join(CSRC, "mk_linalg.hip"), "-o", str(out)])
    n, n_dpp, bad = dpp_hazards.check(out.read_text())
    assert n >= 150, n          # 120 factor updates + 36 inverse updates (four row groups) per pivot block
    assert n_dpp > n            # the compiler's own DPP moves (wave reductions) are checked too
    assert not bad, bad[:3]
