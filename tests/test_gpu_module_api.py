"""GPU: the reference programming model on the fused kernels (Net + autograd + Adadelta + DDP)."""
import copy
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.optim import Adadelta, StepLR

from refmodel import rel_err

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(B, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    from pytorch_mnist_ddp_amd.data.synthetic import generate
    from pytorch_mnist_ddp_amd.data.datasets import normalize_u8
    imgs, lab = generate(B, seed=seed + 3)
    return normalize_u8(imgs).to(dev), lab.to(dev)


def test_module_forward_backward_matches_cpu_reference(cuda_device):
    torch.manual_seed(1)
    net = Net()
    ref = copy.deepcopy(net)
    net = net.to(cuda_device)
    for m in (net, ref):
        m.dropout1.p = m.dropout2.p = 0.0
    x, y = _data(64, cuda_device)
    net.eval()
    with torch.no_grad():
        lp = net(x)
    ref.eval()
    lp_ref = ref(x.cpu())
    assert rel_err(lp.cpu(), lp_ref) < 1e-2
    net.train(), ref.train()
    F.nll_loss(net(x), y).backward()
    F.nll_loss(ref(x.cpu()), y.cpu()).backward()
    for (n, a), b in zip(net.named_parameters(), ref.parameters()):
        assert rel_err(a.grad.cpu(), b.grad) < 0.1, n


def test_module_training_loop_converges_and_checkpoints(cuda_device, tmp_path):
    torch.manual_seed(1)
    net = Net().to(cuda_device)
    opt = Adadelta(net.parameters(), lr=1.0)
    sched = StepLR(opt, step_size=1, gamma=0.7)
    x, y = _data(512, cuda_device, seed=1)
    losses = []
    for epoch in range(3):
        for i in range(0, 512, 64):
            opt.zero_grad()
            loss = F.nll_loss(net(x[i:i + 64]), y[i:i + 64])
            loss.backward()
            opt.step()
            losses.append(loss.item())
        sched.step()
    assert losses[-1] < 0.5 * losses[0]
    sd = opt.state_dict()
    assert len(sd["state"]) == 8 and "square_avg" in sd["state"][0]
    torch.save(net.state_dict(), tmp_path / "m.pt")
    cpu = Net()
    cpu.load_state_dict(torch.load(tmp_path / "m.pt", weights_only=True, map_location="cpu"))
    net.eval(), cpu.eval()
    with torch.no_grad():
        assert rel_err(net(x[:32]).cpu(), cpu(x[:32].cpu())) < 2e-2


def test_module_path_with_stock_torch_optimizer(cuda_device):
    torch.manual_seed(2)
    net = Net().to(cuda_device)
    opt = torch.optim.SGD(net.parameters(), lr=0.05)
    x, y = _data(128, cuda_device, seed=2)
    first = None
    for _ in range(20):
        opt.zero_grad()
        loss = F.nll_loss(net(x), y)
        loss.backward()
        opt.step()                       # in-place param update: fused shadows refresh lazily
        first = first if first is not None else loss.item()
    assert loss.item() < first


def test_ddp_wrapper_and_engine_ddp_schedule_on_one_gpu(cuda_device):
    """world_size=1 process group: DDP wrapper hooks (nccl) + engine's RCCL-overlapped schedule."""
    import torch.distributed as dist
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.ops import native
    from pytorch_mnist_ddp_amd.parallel.ddp import DistributedDataParallel
    from conftest import init_world1_pg
    init_world1_pg("nccl", cuda_device)
    try:
        torch.manual_seed(3)
        net = Net().to(cuda_device)
        ddp = DistributedDataParallel(net, device_ids=[0])
        x, y = _data(64, cuda_device, seed=4)
        F.nll_loss(ddp(x), y).backward()
        assert [c[0] for c in ddp.reducer.calls] == [0, 1]
        assert list(ddp.state_dict())[0] == "module.conv1.weight"
        # native C++ reducer (RCCL comm from the c10d store) == python reducer == no DDP
        from pytorch_mnist_ddp_amd.parallel.ddp import NativeBucketReducer
        from pytorch_mnist_ddp_amd.parallel.distributed import create_rccl_comm
        ncomm = create_rccl_comm(1, 0, 0, tag="native-reducer-test")
        grads = []
        for mode in ("plain", "python", "native"):
            torch.manual_seed(7)
            m = Net().to(cuda_device)
            m.dropout1.p = m.dropout2.p = 0.0
            w = m if mode == "plain" else DistributedDataParallel(m, device_ids=[0],
                                                                  comm=ncomm if mode == "native" else None)
            if mode == "native":
                assert isinstance(w.reducer, NativeBucketReducer)
            for _ in range(2):                       # two iterations: reducer state resets cleanly
                for p_ in m.parameters():
                    p_.grad = None
                F.nll_loss(w(x), y).backward()
            if mode == "native":
                assert [c[0] for c in w.reducer.calls] == [0, 1, 0, 1]
            torch.cuda.synchronize()
            grads.append([p_.grad.detach().clone() for p_ in m.parameters()])
        for a_, b_, c_ in zip(*grads):
            assert torch.equal(a_, b_) and torch.equal(a_, c_)
        # engine with an attached RCCL communicator: fc bucket all-reduce + Adadelta on the comm
        # stream overlapped with the conv backward, captured into graphs; must equal no-comm runs
        C = native.load()
        comm = C.RcclComm(C.RcclComm.unique_id(), 1, 0, 0)
        tr = load_mnist(synthetic_data=True, train=True, synthetic_size=1024, verbose=False)
        idx = torch.randperm(1024, generator=torch.Generator().manual_seed(0))
        res = []
        # RCCL schedule (graphs / eager / one bucket), xGMI schedule (world 1: its output buffer path;
        # fused and separate launches, graphs / eager), single GPU OVERLAP and SERIAL
        for c, gs, ar, kw, sched in ((comm, 4, "rccl", {}, C.SCHED_RCCL), (comm, 0, "rccl", {}, C.SCHED_RCCL),
                                     (comm, 4, "rccl", {"two_buckets": False}, C.SCHED_RCCL),
                                     (comm, 4, "xgmi", {}, C.SCHED_XGMI), (comm, 0, "xgmi", {}, C.SCHED_XGMI),
                                     (comm, 4, "xgmi", {"xgmi_fuse": False}, C.SCHED_XGMI),
                                     (None, 4, None, {"overlap": False}, C.SCHED_SERIAL),
                                     (None, 4, None, {}, C.SCHED_OVERLAP)):
            torch.manual_seed(5)
            ms = ModelState(Net(), cuda_device)
            t = FusedTrainer(ms, tr, None, 128, 1, num_samples=1024, comm=c, graph_steps=gs,
                             allreduce=ar or "auto", **kw)
            assert t.allreduce == ar and t.engine.schedule == sched, (ar, kw)
            t.train_epoch(1, idx)
            t.synchronize()
            res.append(ms.param.clone())
        diffs = [(r - res[-1]).abs().max().item() for r in res]
        assert all(d == 0 for d in diffs), diffs
    finally:
        dist.destroy_process_group()


def test_fc_bucket_hooks_fire_before_conv_backward(cuda_device, monkeypatch):
    """Module path: autograd finalises the fc gradients (DDP bucket 0) and runs their hooks before
    conv_bwd is enqueued, so DDP's bucket-0 all-reduce overlaps the conv backward as in torch DDP
    (reference mnist_ddp.py:72); the conv gradients' hooks fire after it."""
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load()
    events = []

    class Spy:
        def __getattr__(self, name):
            fn = getattr(C, name)
            if name in ("conv_bwd", "fc_bwd"):
                def wrapped(*a, **k):
                    events.append(name)
                    return fn(*a, **k)
                return wrapped
            return fn
    monkeypatch.setattr(native, "load", lambda *a, **k: Spy())
    torch.manual_seed(3)
    net = Net().to(cuda_device)
    for n, p_ in net.named_parameters():
        p_.register_post_accumulate_grad_hook(lambda _p, n=n: events.append(n))
    x, y = _data(64, cuda_device, seed=4)
    F.nll_loss(net(x), y).backward()
    torch.cuda.synchronize()
    i = events.index("conv_bwd")
    assert events.index("fc_bwd") < i
    assert set(events[:i]) >= {"fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"}
    assert set(events[i + 1:]) == {"conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"}


def test_scripts_on_gpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    common = ["--epochs", "2", "--batch-size", "200", "--synthetic", "--synthetic-train-size", "4000",
              "--synthetic-test-size", "1000", "--save-model"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "mnist_ddp.py"), *common], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout
    assert "Not using distributed mode" in out and out.count("Test set: Average loss:") == 2
    assert "Train Epoch: 2 [2000/4000 (50%)]" in out and "Total cost time:" in out
    # epoch pipelining (driver.py): every epoch's test line after its train lines, before the next's
    kinds = [ln.split(":")[0].split(" [")[0] for ln in out.splitlines()
             if ln.startswith(("Train Epoch", "Test set"))]
    assert kinds == ["Train Epoch"] * 2 + ["Test set"] + ["Train Epoch"] * 2 + ["Test set"], kinds
    sd = torch.load(os.path.join(tmp_path, "mnist_cnn_.pt"), weights_only=True)
    assert sd["fc1.weight"].is_cuda and sd["fc1.weight"].dtype == torch.float32
    r = subprocess.run([sys.executable, os.path.join(ROOT, "mnist.py"), *common, "--engine", "module", "--dry-run"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("Train Epoch:") == 2 and os.path.exists(os.path.join(tmp_path, "mnist_cnn.pt"))


def test_torchrun_ddp_paths_on_one_gpu(tmp_path):
    """torchrun world_size=1: env rendezvous, c10d-store RCCL unique-id exchange, engine broadcast,
    comm-attached graphs (fused engine) and hook-driven buckets (module engine)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    for engine in ("fused", "module"):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--standalone", "--local-addr=127.0.0.1", os.path.join(ROOT, "mnist_ddp.py"),
               "--epochs", "1", "--batch-size", "200", "--synthetic", "--synthetic-train-size", "2000",
               "--synthetic-test-size", "1000", "--save-model", "--engine", engine]
        r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "| distributed init (rank 0): env://, local rank:0, world size:1" in r.stdout
        assert "Test set: Average loss:" in r.stdout
        sd = torch.load(os.path.join(tmp_path, "mnist_cnn.pt"), weights_only=True)
        assert list(sd)[0] == "module.conv1.weight"
        os.remove(os.path.join(tmp_path, "mnist_cnn.pt"))


def test_fp32_parity_mode_uses_torch_ops(cuda_device):
    """--dtype fp32: Net.compute_dtype = float32 runs stock torch fp32 ops on the GPU."""
    torch.manual_seed(4)
    net = Net()
    ref = copy.deepcopy(net)
    net = net.to(cuda_device)
    net.compute_dtype = torch.float32
    net.eval(), ref.eval()
    x, _ = _data(32, cuda_device, seed=5)
    with torch.no_grad():
        assert rel_err(net(x).cpu(), ref(x.cpu())) < 1e-4
    assert not hasattr(net, "_amd_fused_state")
