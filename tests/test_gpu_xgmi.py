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
def test_xgmi_allreduce_multiprocess_one_gpu(gpu_box, world, engine_steps, fault):
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


def _world1_trainer(dev, comm, **kw):
    import torch
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.models.net import Net
    torch.manual_seed(1)
    ms = ModelState(Net(), dev, lr=1.0)
    train = load_mnist(train=True, synthetic_data=True, synthetic_size=2000, verbose=False)
    t = FusedTrainer(ms, train, None, 200, 1000, num_samples=2000, comm=comm, seed=1, graph_steps=4, **kw)
    return ms, t


def test_fp32_xgmi_schedule_world1_matches_single_gpu(cuda_device):
    """The fp32 step's XGMI schedule - the fc bucket's two-shot all-reduce with the Adadelta step
    fused on the comm stream beside the conv backward, the conv bucket's one-shot at the step tail,
    split side / compute graphs - at world 1 trains bitwise like the single-GPU fp32 OVERLAP step."""
    import torch
    import torch.distributed as dist
    from conftest import init_world1_pg
    init_world1_pg("gloo")
    try:
        idx = torch.randperm(2000, generator=torch.Generator().manual_seed(6))
        res = {}
        for name, kw in (("xgmi", dict(allreduce="xgmi", fp32=True)), ("single", dict(fp32=True))):
            ms, t = _world1_trainer(cuda_device, None, **kw)
            assert (t.allreduce == "xgmi") if name == "xgmi" else t.overlap
            for ep in (1, 2):
                t.train_epoch(ep, idx)
            t.synchronize()
            res[name] = (ms.param.clone(), t.loss_log.clone())
        assert torch.equal(res["xgmi"][0], res["single"][0])
        assert torch.equal(res["xgmi"][1], res["single"][1])
    finally:
        dist.destroy_process_group()


def test_transport_choice_by_schedule_replay_world1(cuda_device):
    """--allreduce fastest picks the transport by replaying each candidate's PRODUCTION schedule: at
    world 1 with an RCCL communicator and the xGMI candidate forced in (probe_world1), both captured
    chunk graphs are validated and timed (us per step in transport_report), the faster is kept, and
    training on it is bitwise the single-transport runs (RCCL schedule; xGMI schedule) - the
    validation replays leave no trace in the model, the optimizer state or the step counter."""
    import torch
    import torch.distributed as dist
    from conftest import init_world1_pg
    from pytorch_mnist_ddp_amd.parallel.distributed import create_rccl_comm
    init_world1_pg("nccl", cuda_device)
    try:
        comm = create_rccl_comm(1, 0, 0)
        idx = torch.randperm(2000, generator=torch.Generator().manual_seed(4))
        res = {}
        for name, kw in (("fastest", dict(allreduce="fastest", probe_world1=True)), ("rccl", dict(allreduce="rccl")),
                         ("xgmi", dict(allreduce="xgmi"))):
            ms, t = _world1_trainer(cuda_device, comm, **kw)
            if name == "fastest":
                rep = t.transport_report
                assert set(rep) == {"xgmi", "rccl"}, rep
                assert all(r["ok"] and r["us_per_step"] > 0 for r in rep.values()), rep
                assert rep["xgmi"]["validation"].startswith("ok (graph replay of the 4-step")
                fast = min(rep, key=lambda k: rep[k]["us_per_step"])
                assert t.allreduce == fast
                assert set(t.setup.s) >= {"validate.xgmi", "validate.rccl", "xgmi_comm", "stream_probe"}
            else:
                assert t.allreduce == name and set(t.transport_report) == {name}
            assert ms.get_step() == 0
            t.train_epoch(1, idx)
            t.synchronize()
            res[name] = (ms.param.clone(), t.loss_log.clone())
        for name in ("rccl", "xgmi"):
            assert torch.equal(res[name][0], res["fastest"][0]) and torch.equal(res[name][1], res["fastest"][1]), name
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_rccl_schedule_world1_matches_single_gpu(tmp_path, dtype):
    """The RCCL DDP schedule (fc bucket forked onto the comm stream, conv bucket after the join, one
    communicator, one graph per chunk in step order) at world 1 (--force-comm) trains bitwise like the
    plain single-GPU step, and the bench JSON names one communicator and the startup validation
    (fp32: the fp32 step's chains, the fc bucket's all-reduce on the comm stream)."""
    import json
    outs = {}
    runs = (("rccl", ["--force-comm"]), ("plain", []))
    for name, extra in runs:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "1", "--standalone",
               "--local-addr", "127.0.0.1", os.path.join(ROOT, "bench.py"), "--allreduce", "rccl",
               "--no-full-run", "--steps", "60", "--warmup", "10", "--dtype", dtype, *extra]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=tmp_path,
                           env=dict(os.environ, PYTHONPATH=ROOT))
        assert r.returncode == 0, (name, r.stderr[-3000:])
        outs[name] = json.loads(r.stdout.strip().splitlines()[-1])
    c = outs["rccl"]["config"]
    assert c["rccl_comms"] == 1 and c["rccl_world"] == 1 and c["allreduce"] == "rccl" and c["schedule"] == "rccl"
    assert c["transport_report"]["rccl"]["ok"] and c["allreduce_schedule_us"]["rccl"] > 0
    assert outs["plain"]["config"]["rccl_comms"] == 0 and outs["plain"]["config"]["schedule"] == "overlap"
    assert outs["rccl"]["last_train_loss"] == outs["plain"]["last_train_loss"]


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


def test_stuck_rccl_candidate_is_aborted_and_xgmi_kept(cuda_device, monkeypatch):
    """--allreduce fastest where the RCCL candidate's validation replay never completes (an injected
    device-side stall in front of it, MNIST_AMD_FAULT=rccl_stall): the host watchdog fires, the RCCL
    communicator is aborted (ncclCommAbort) and dropped, the streams drain, and training continues on
    the already-validated xGMI schedule - bitwise equal to --allreduce xgmi, no fatal exit."""
    import torch
    import torch.distributed as dist
    from conftest import init_world1_pg
    from pytorch_mnist_ddp_amd.parallel.distributed import create_rccl_comm
    init_world1_pg("nccl", cuda_device)
    try:
        idx = torch.randperm(2000, generator=torch.Generator().manual_seed(4))
        monkeypatch.setenv("MNIST_AMD_FAULT", "rccl_stall:0:60")
        monkeypatch.setenv("MNIST_AMD_RCCL_WATCHDOG", "3")
        comm = create_rccl_comm(1, 0, 0)
        assert comm.nonblocking                      # ncclCommInitRankConfig(blocking = 0)
        ms, t = _world1_trainer(cuda_device, comm, allreduce="fastest", probe_world1=True)
        rep = t.transport_report
        assert rep["xgmi"]["ok"] and not rep["rccl"]["ok"], rep
        assert "communicator aborted after" in rep["rccl"]["validation"], rep
        assert comm.aborted and t.comm is None and t.allreduce == "xgmi"
        assert ms.get_step() == 0
        t.train_epoch(1, idx)
        t.synchronize()
        got = (ms.param.clone(), t.loss_log.clone())
        monkeypatch.delenv("MNIST_AMD_FAULT")
        ms2, t2 = _world1_trainer(cuda_device, None, allreduce="xgmi")
        t2.train_epoch(1, idx)
        t2.synchronize()
        assert torch.equal(got[0], ms2.param) and torch.equal(got[1], t2.loss_log)
    finally:
        dist.destroy_process_group()
