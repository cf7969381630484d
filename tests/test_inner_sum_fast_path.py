"""aten_inner_sum's fast path for 8..15 elements (csrc/dfq_common.h: the CLE stop
rule's per-layer means over 8 thread slots, the sweep's 3x3 error sums) equals the
generic ATen-order walk bit for bit, on 200,000 random inputs with signed zeros,
infinities, NaN, denormals and huge values -- a host build of the same header, no GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_inner_sum_fast_path_bit_exact(tmp_path):
    exe = tmp_path / "inner_sum_check"
    src = os.path.join(ROOT, "tests", "native", "inner_sum_check.hip")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "data_free_quantization_amd", "csrc"),
                    src, "-o", str(exe)], check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout, r.stdout
