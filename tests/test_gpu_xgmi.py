"""T3 on one GPU: the direct xGMI all-reduce (csrc/runtime/xgmi_comm.h, kernels/xgmi_allreduce.hip)
with 2 and 4 ranks sharing GPU 0 (IPC mappings, stage hand-offs, shard index sets, graph replay,
engine schedule 3 with rank-identical parameters).  Drives tools/xgmi_check.py in a subprocess."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,engine_steps", [(2, 30), (4, 0)])
def test_xgmi_allreduce_multiprocess_one_gpu(cuda_device, world, engine_steps):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "xgmi_check.py"), "--world", str(world),
           "--same-device", "--iters", "20", "--engine-steps", str(engine_steps), "--timeout", "100"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=dict(os.environ, PYTHONPATH=ROOT))
    print(r.stdout[-3000:])
    assert r.returncode == 0 and "XGMI_CHECK PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
