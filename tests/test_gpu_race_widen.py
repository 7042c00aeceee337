"""T3 race-window widening: every overlapped schedule - OVERLAP (bf16,
eager and split graphs, B = 200 and 1500), the fp32 OVERLAP step, the world-1 XGMI and RCCL
schedules (bf16 and fp32) - runs once under the debug build ``_C_rw`` (random 0..20 us sleeps before
each kernel's first global read and before each stream hand-off signal, csrc/include/device_utils.h)
and must stay bitwise equal to its one-stream reference.  ``broken_w1t`` switches off the w1t
ping-pong (the race round 5 found by luck) and must be caught: the widened run differs."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(200)
@pytest.mark.parametrize("case", ["overlap", "overlap_eager", "overlap_large", "fp32", "xgmi", "xgmi_fp32", "rccl",
                                  "rccl_fp32", "broken_w1t"])
def test_schedule_bitwise_under_race_widening(gpu_box, case):
    env = dict(os.environ, PYTHONPATH=ROOT, MNIST_AMD_RACE_WIDEN="1", MNIST_AMD_NO_BUILD="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "race_widen_check.py"), "--case", case],
                       capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "RACE_WIDEN PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
    assert "widened (_C_rw)" in r.stdout
