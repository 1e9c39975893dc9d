"""Host check of the f64-FFT PBS level-1 digit (csrc/fft64_decomp.hpp) against the reference's native
decomposition restated in C (tests/cpp/fft_decomp_check.cpp): every base_log 1..31, rounding corners and random
words.  No GPU: hipcc builds host code only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_level1_digit_matches_reference(tmp_path):
    exe = str(tmp_path / "fft_decomp_check")
    subprocess.run([HIPCC, "-O2", "-x", "hip", os.path.join(ROOT, "tests", "cpp", "fft_decomp_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert " 0 mismatches" in out.stdout
