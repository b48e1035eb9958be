"""Host-side sanitizer runs of the native runtime: the CSV parser built with
AddressSanitizer + UndefinedBehaviorSanitizer and, separately, ThreadSanitizer (its parse is
multi-threaded), driven by a standalone C++ program over edge-case inputs.  GPU sanitizers are
not available on the MI355X pool; device kernels are covered by host-side shape checks in every
C entry point and the numerics tests."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "shifu_amd", "runtime", "csrc", "csv_parser.cpp")
DRV = os.path.join(ROOT, "tests", "native", "csv_parser_sanitize.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_csv_parser_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "drv")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           SRC, DRV, "-o", exe, "-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "sanitizer" in (r.stderr or "").lower() and "not" in r.stderr.lower():
        pytest.skip(f"sanitizer {san} unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
