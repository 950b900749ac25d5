"""Table mode's narrow keys (k <= 21): the key code, hash and 32-bit form
round trip on the host (tests/native/narrow_keys_check.hip, built with hipcc
from the library's own header; no GPU needed)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_narrow_key_round_trip(tmp_path):
    exe = tmp_path / "narrow_keys_check"
    src = os.path.join(HERE, "native", "narrow_keys_check.hip")
    inc = os.path.join(HERE, "..", "kmerjs_amd", "csrc")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I", inc, "-o", str(exe), src], check=True,
                   capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 of " in r.stdout
