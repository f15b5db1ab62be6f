"""The OneBlob forward skips the wrap-around quartic CDF terms that clamp (csrc/encodings.hip
wrapped_cdf). Its exactness rests on quartic_cdf (common_device.h:905-912, the kernel's explicit-FMA
op sequence) being exactly 1 for every fp32 u >= 1.0625 and exactly 0 for every u <= -1.0625; the
checker enumerates every float in [1, 2^20] (larger |u| only grows the polynomial)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_quartic_cdf_clamps_exactly_beyond_threshold(tmp_path):
    exe = str(tmp_path / "qc")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(REPO, "tools", "quartic_clamp_check.c"), "-lm"],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
