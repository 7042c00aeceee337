"""SURVEY §5.2 (race detection / sanitizers) for the native runtime's host code: the parts that parse
peer-supplied bytes or carve memory by hand (csrc/runtime/host_logic.h - engine workspace layout,
xGMI IPC record decoding, residency grid fitting) built with -fsanitize=address,undefined and run
on the CPU (tools/sanitize_host.sh)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                    reason="needs g++ and the ROCm headers")
def test_host_logic_under_asan_ubsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "HOST_LOGIC_TEST PASS" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
