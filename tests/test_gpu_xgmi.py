"""T3 on one GPU: the direct xGMI all-reduce (csrc/runtime/xgmi_comm.h, kernels/xgmi_allreduce.hip)
with 2 and 4 ranks sharing GPU 0 (IPC mappings, stage hand-offs, shard index sets, graph replay,
engine schedule 3 with rank-identical parameters).  Drives tools/xgmi_check.py in a subprocess."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(260)
@pytest.mark.parametrize("world,engine_steps,fault", [(2, 30, False), (3, 20, False), (4, 30, False), (8, 30, False),
                                                       (4, 0, True)])
def test_xgmi_allreduce_multiprocess_one_gpu(cuda_device, world, engine_steps, fault):
    """With engine steps the FUSED schedule (the production default) runs with W ranks' spinning
    grids on one GPU: the residency planner must shrink them so all are resident.  W = 3 and 8
    execute those template instantiations of every xGMI kernel (8 = the headline config)."""
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "xgmi_check.py"), "--world", str(world),
           "--same-device", "--iters", "20", "--engine-steps", str(engine_steps), "--timeout", "230"]
    if fault:
        cmd.append("--fault-test")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=245, env=dict(os.environ, PYTHONPATH=ROOT))
    print(r.stdout[-3000:])
    assert r.returncode == 0 and "XGMI_CHECK PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])


def test_allreduce_auto_choice_plumbing_world1(cuda_device):
    """choose_allreduce at world 1 (RCCL comms + the xGMI communicator's copy path): both launch
    sequences run, the timings come back and the buffers are left zeroed."""
    import torch
    import torch.distributed as dist
    from conftest import init_world1_pg
    from pytorch_mnist_ddp_amd.parallel.distributed import choose_allreduce, create_rccl_comms, create_xgmi_comm
    init_world1_pg("nccl", cuda_device)
    try:
        c0, c1 = create_rccl_comms(1, 0, 0, n=2)
        n, split = 1200000, 1181120
        g = torch.randn(n, device=cuda_device)
        x = create_xgmi_comm(1, 0, cuda_device, n)
        assert x is not None
        gin, gout = x.grad_in, x.grad_out
        assert gin.shape == (n,) and gin.is_cuda and gin.data_ptr() != gout.data_ptr()
        gin.normal_()
        gout.normal_()
        pick, t = choose_allreduce(c1, c0, x, g, (0, split), (split, n - split), cuda_device)
        assert pick in ("rccl", "xgmi") and t["rccl_us"] > 0 and t["xgmi_us"] > 0
        for b in (g, gin, gout):
            assert int(b.abs().sum().item()) == 0
    finally:
        dist.destroy_process_group()


def test_trainer_auto_probe_path_world1(tmp_path):
    """The trainer's --allreduce auto path (probe of both implementations on scratch optimizer
    state, forced at world 1) runs and leaves training bit-identical to a plain RCCL run."""
    outs = {}
    for name, env in (("auto", {"MNIST_AMD_PROBE_ALWAYS": "1"}), ("rccl", {"MNIST_AMD_ALLREDUCE": "rccl"})):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "1", "--standalone",
               "--local-addr", "127.0.0.1", os.path.join(ROOT, "bench.py"),
               "--force-comm", "--no-full-run", "--steps", "40", "--warmup", "10"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=tmp_path,
                           env=dict(os.environ, PYTHONPATH=ROOT, **env))
        assert r.returncode == 0, r.stderr[-3000:]
        import json
        outs[name] = json.loads(r.stdout.strip().splitlines()[-1])
    assert outs["auto"]["config"]["allreduce_probe_us"]["rccl_us"] > 0
    assert outs["auto"]["last_train_loss"] == outs["rccl"]["last_train_loss"]


@pytest.mark.timeout(200)
@pytest.mark.parametrize("mode", ["1", "comm"])
def test_conv_bucket_split_bitwise_at_two_ranks(cuda_device, mode):
    """Opt-in conv bucket split (MNIST_AMD_CONV_SPLIT=1: a third stream, =comm: queued on the comm
    stream after the fc bucket, inside the side graph): the startup validation inside the engine
    check compares it bitwise with the separate launches, at 2 ranks on one GPU (4 HW queues per
    process: the split's third stream needs its own queue)."""
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "xgmi_check.py"), "--world", "2", "--same-device",
           "--iters", "10", "--engine-steps", "20", "--timeout", "170"]
    env = dict(os.environ, PYTHONPATH=ROOT, MNIST_AMD_CONV_SPLIT=mode, GPU_MAX_HW_QUEUES="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=185, env=env)
    print(r.stdout[-3000:])
    assert r.returncode == 0 and "XGMI_CHECK PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
    assert ("conv split True" if mode == "1" else "conv split comm") in r.stdout


def test_rccl_single_communicator_schedule_world1(tmp_path):
    """DDP schedule 3 on ONE RCCL communicator (the default: fc all-reduce on the comm stream, the
    conv all-reduce on the compute stream ordered after it by a device counter) trains bitwise like
    the opt-in two-communicator schedule and like the plain single-GPU step (world 1, --force-comm)."""
    import json
    outs = {}
    runs = (("one", ["--force-comm"], {}), ("two", ["--force-comm"], {"MNIST_AMD_RCCL_COMMS": "2"}),
            ("plain", [], {}))
    for name, extra, env in runs:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "1", "--standalone",
               "--local-addr", "127.0.0.1", os.path.join(ROOT, "bench.py"), "--allreduce", "rccl",
               "--no-full-run", "--steps", "60", "--warmup", "10", *extra]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=tmp_path,
                           env=dict(os.environ, PYTHONPATH=ROOT, **env))
        assert r.returncode == 0, (name, r.stderr[-3000:])
        outs[name] = json.loads(r.stdout.strip().splitlines()[-1])
    assert outs["one"]["config"]["rccl_comms"] == 1 and outs["two"]["config"]["rccl_comms"] == 2
    assert outs["plain"]["config"]["rccl_comms"] == 0
    assert outs["one"]["last_train_loss"] == outs["two"]["last_train_loss"] == outs["plain"]["last_train_loss"]


def test_world_gt1_without_transport_refuses(cuda_device, monkeypatch):
    """world > 1 with neither an RCCL communicator nor a working xGMI one must raise instead of
    training every rank alone on a gradient 1/world too small."""
    import torch
    import pytorch_mnist_ddp_amd.parallel.distributed as D
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.models.net import Net
    monkeypatch.setattr(D, "create_xgmi_comm", lambda *a, **k: None)
    torch.manual_seed(1)
    ms = ModelState(Net(), cuda_device)
    train = load_mnist(train=True, synthetic_data=True, synthetic_size=512, verbose=False)
    with pytest.raises(RuntimeError, match="no RCCL communicator"):
        FusedTrainer(ms, train, None, 64, 128, num_samples=512, world_size=2, rank=0, allreduce="xgmi")
