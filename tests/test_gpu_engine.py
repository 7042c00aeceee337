"""Engine-level GPU tests: captured graphs vs eager, convergence on synthetic data."""
import copy

import pytest
import torch

from pytorch_mnist_ddp_amd.data.datasets import load_mnist
from pytorch_mnist_ddp_amd.data.samplers import RandomIndexStream
from pytorch_mnist_ddp_amd.engine.state import ModelState
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
from pytorch_mnist_ddp_amd.models.net import Net

pytestmark = pytest.mark.gpu


def _trainer(dev, graph_steps, n_train=2000, n_test=1000, B=200, seed=1, **kw):
    torch.manual_seed(seed)
    net = Net()
    tr = load_mnist(synthetic_data=True, train=True, synthetic_size=n_train, verbose=False)
    te = load_mnist(synthetic_data=True, train=False, synthetic_size=n_test, verbose=False)
    ms = ModelState(net, dev, lr=1.0)
    t = FusedTrainer(ms, tr, te, B, 1000, num_samples=n_train, seed=seed, graph_steps=graph_steps, **kw)
    return net, ms, t


def test_graph_replay_bitwise_equals_eager(cuda_device):
    idx = torch.randperm(2000, generator=torch.Generator().manual_seed(3))
    _, ms_g, tg = _trainer(cuda_device, graph_steps=4)
    _, ms_e, te = _trainer(cuda_device, graph_steps=0)
    tg.train_epoch(1, idx)
    te.train_epoch(1, idx)
    torch.cuda.synchronize()
    assert torch.equal(ms_g.param, ms_e.param)
    assert torch.equal(tg.loss_log, te.loss_log)
    assert ms_g.get_step() == 10


def test_multi_round_warm_replay_restores_state_bitwise(cuda_device):
    """bench.py's warm replays (FusedTrainer.warm_graphs with a step budget): the timed chunk graphs
    replayed for several rounds, the step counter restored after every round (it indexes the
    gathered rows and the loss log: a run past them faulted the GPU once) and the whole state after
    the last; the steps that follow are bitwise those of a trainer that never replayed."""
    n, steps = 6, 4
    idx = torch.randperm(n * 200, generator=torch.Generator().manual_seed(11))   # the dataset's rows
    runs = []
    for warm in (0, 5 * steps):
        _, ms, t = _trainer(cuda_device, graph_steps=steps, n_train=n * 200)
        t.start_stream(idx, gather=True)
        t.precapture(steps)
        if warm:
            assert t.warm_graphs(steps, warm) == warm
        t.run_steps(n)
        t.synchronize()
        runs.append((ms.param.clone(), t.loss_log[:n].clone(), ms.get_step()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])
    assert runs[0][2] == runs[1][2] == n


def test_training_converges_on_synthetic(cuda_device):
    net, ms, t = _trainer(cuda_device, graph_steps=10, n_train=6000)
    stream = RandomIndexStream(6000)
    l0, c0, n = t.evaluate()
    for ep in range(1, 4):
        st = t.train_epoch(ep, stream.epoch_indices())
        assert st.steps == 30
    l1, c1, _ = t.evaluate()
    assert l1 / n < 0.5 * (l0 / n)
    assert c1 / n > 0.9, c1 / n
    assert torch.isfinite(ms.param).all()


def test_partial_last_batch_and_dry_run(cuda_device):
    _, ms, t = _trainer(cuda_device, graph_steps=10, n_train=2000, B=64)   # 31 full + 1 of 16
    idx = torch.randperm(2000)
    logs = []
    st = t.train_epoch(1, idx, log_interval=10, log_fn=lambda b, n, l: logs.append((b, n, l)))
    assert st.steps == 32
    assert [b for b, _, _ in logs] == [0, 10, 20, 30]
    st = t.train_epoch(2, idx, dry_run=True, log_fn=lambda b, n, l: logs.append((b, n, l)))
    assert st.steps == 1
    assert torch.isfinite(ms.param).all()


@pytest.mark.parametrize("graph_steps", [0, 3, 4])
def test_overlap_schedule_bitwise_equals_serial(cuda_device, graph_steps):
    """The OVERLAP schedule (fc update and conv2's reduce + update on the comm stream with device-
    counter hand-offs, w2d ping-pong across odd and even chunk lengths, split side / compute graphs
    launched from two threads, or eager) == the SERIAL one-stream schedule, bit for bit, including
    every bf16 shadow and the evaluation after training (the side-stream schedules had
    only manual A/B evidence)."""
    idx = torch.randperm(2000, generator=torch.Generator().manual_seed(5))
    _, ms_o, to = _trainer(cuda_device, graph_steps=graph_steps, overlap=True)
    _, ms_s, ts = _trainer(cuda_device, graph_steps=graph_steps, overlap=False)
    assert to.overlap and not ts.overlap
    C = to.C
    assert to.engine.schedule == C.SCHED_OVERLAP and ts.engine.schedule == C.SCHED_SERIAL
    for ep in (1, 2):
        to.train_epoch(ep, idx)
        ts.train_epoch(ep, idx)
    torch.cuda.synchronize()
    for name in ("param", "square_avg", "acc_delta", "w1", "w1t", "w2f", "w2d"):
        assert torch.equal(getattr(ms_o, name), getattr(ms_s, name)), name
    assert torch.equal(to.loss_log, ts.loss_log)
    w1 = ms_o.views(ms_o.param)["fc1.weight"]
    assert torch.equal(ms_o.w1t.view(9216, 128), w1.t().contiguous().to(torch.bfloat16))
    lo, co, _ = to.evaluate()
    ls, cs, _ = ts.evaluate()
    assert lo == ls and co == cs


@pytest.mark.parametrize("B", [200, 1500])
def test_one_wave_conv1_tail_bitwise_equals_reduce_parts(cuda_device, B):
    """The OVERLAP step tail's conv1 reduce + update on 80 one-wave workgroups (adadelta_c1_kernel,
    the slice tree on cross-lane moves; B = 1500 reads the group sums c1red) == the same work as the
    20 conv1 parts of the 256-thread reduce launch (hook c1_lanes=0), bit for bit, gradients included."""
    n = 2000 if B == 200 else 3000
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(13))
    _, ms_a, ta = _trainer(cuda_device, graph_steps=3, n_train=n, B=B, overlap=True)
    _, ms_b, tb = _trainer(cuda_device, graph_steps=3, n_train=n, B=B, overlap=True, hooks={"c1_lanes": 0})
    assert ta.engine.c1_lanes and not tb.engine.c1_lanes
    for ep in (1, 2):
        ta.train_epoch(ep, idx)
        tb.train_epoch(ep, idx)
    torch.cuda.synchronize()
    for name in ("param", "square_avg", "acc_delta", "grad"):
        assert torch.equal(getattr(ms_a, name), getattr(ms_b, name)), name
    assert torch.equal(ta.loss_log, tb.loss_log)


@pytest.mark.parametrize("graph_steps", [0, 2])
def test_overlap_schedule_large_batch_bitwise_equals_serial(cuda_device, graph_steps):
    """B > 1024: fc_bwd's split partials are summed on the comm stream (ahead of the fc update) in
    the OVERLAP schedule, on the compute stream in SERIAL - same bits, same logged losses."""
    idx = torch.randperm(3000, generator=torch.Generator().manual_seed(9))
    _, ms_o, to = _trainer(cuda_device, graph_steps=graph_steps, n_train=3000, B=1500, overlap=True)
    _, ms_s, ts = _trainer(cuda_device, graph_steps=graph_steps, n_train=3000, B=1500, overlap=False)
    assert to.overlap and not ts.overlap
    for ep in (1, 2):
        to.train_epoch(ep, idx)
        ts.train_epoch(ep, idx)
    torch.cuda.synchronize()
    for name in ("param", "square_avg", "acc_delta", "grad", "w1", "w1t", "w2f", "w2d"):
        assert torch.equal(getattr(ms_o, name), getattr(ms_s, name)), name
    assert torch.equal(to.loss_log, ts.loss_log)


def test_whole_split_eval_bitwise_equals_test_batch_chunks(cuda_device):
    """evaluate() runs the test split as one batch; per-row losses / hits must be bitwise the
    chunked (--test-batch-size 1000) ones."""
    _, ms, t = _trainer(cuda_device, graph_steps=4, n_train=2000, n_test=4000)
    assert t.eval_batch == 4000
    t.train_epoch(1, torch.randperm(2000, generator=torch.Generator().manual_seed(1)))
    rows = []
    for batch in (1000, 4000, 1000):
        t.engine.eval(4000, batch)
        torch.cuda.synchronize()
        rows.append((t.test_loss_rows.clone(), t.test_correct.clone()))
    for l_, c_ in rows[1:]:
        assert torch.equal(l_, rows[0][0]) and torch.equal(c_, rows[0][1])
    loss, correct, n = t.evaluate()
    assert n == 4000 and correct == int(rows[0][1].sum())


def test_torch_profiler_sees_native_kernels(cuda_device):
    """the hand-written kernels launched by the C++ engine on torch streams show up
    in torch.profiler (kineto/roctracer) traces by name."""
    from torch.profiler import ProfilerActivity, profile
    _, ms, t = _trainer(cuda_device, graph_steps=0, n_train=400, n_test=100)
    t.train_epoch(1, torch.randperm(400, generator=torch.Generator().manual_seed(2)))   # warm
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        t.train_epoch(2, torch.randperm(400, generator=torch.Generator().manual_seed(3)))
        torch.cuda.synchronize()
    names = " ".join({e.name for e in prof.events()})
    for k in ("trunk_fwd", "fc1_fwd", "head_train", "fc_bwd", "conv2_wgrad", "conv2_dgrad", "adadelta"):
        assert k in names, k


def test_stream_handoff_probe(cuda_device):
    """The OVERLAP / XGMI precondition check: compute and comm streams progress independently (each
    waits on a device counter the other signals afterwards) and the probe is repeatable."""
    _, ms, t = _trainer(cuda_device, graph_steps=0)
    assert t.engine.probe_stream_handoff(2.0)
    assert t.engine.probe_stream_handoff(2.0)


def test_profile_window_bitwise_equals_graph_and_reports_device_time(cuda_device):
    """--profile runs the first steps eagerly with one roctx range per phase (Engine.profile_steps,
    every phase drained before its range closes); the results must be those of the graph path, and
    the epoch reports its HIP-event device time."""
    idx = torch.randperm(2000, generator=torch.Generator().manual_seed(5))
    _, ms_g, tg = _trainer(cuda_device, graph_steps=4)
    _, ms_p, tp = _trainer(cuda_device, graph_steps=4)
    tp.profile_left = 6
    sg = tg.train_epoch(1, idx)
    sp = tp.train_epoch(1, idx)
    torch.cuda.synchronize()
    assert tp.profile_left == 0
    assert torch.equal(ms_g.param, ms_p.param) and torch.equal(tg.loss_log, tp.loss_log)
    assert sg.device_seconds is not None and 0 < sg.device_seconds <= sg.train_seconds + 1e-3


def test_module_path_reuses_step_buffers(cuda_device):
    """Net.forward on GPU takes its activation set from a per-(batch, stream) pool: no per-step
    allocation once warm, and results identical to a fresh allocation."""
    from pytorch_mnist_ddp_amd.ops.fused_net import fused_state
    import torch.nn.functional as F
    torch.manual_seed(1)
    net = Net().to(cuda_device)
    x = torch.randn(32, 1, 28, 28, device=cuda_device)
    y = torch.randint(0, 10, (32,), device=cuda_device)
    net.eval()
    with torch.no_grad():
        o1 = net(x)
        o2 = net(x)
    assert torch.equal(o1, o2)
    st = fused_state(net)
    ids = {id(b) for v in st.pool.values() for b in v}
    net.train()
    for _ in range(3):
        net.zero_grad(set_to_none=True)
        F.nll_loss(net(x), y).backward()
    torch.cuda.synchronize()
    assert {id(b) for v in st.pool.values() for b in v} >= ids      # sets recycled, not replaced
    assert sum(len(v) for v in st.pool.values()) == 1


def test_large_batch_conv1_prereduce_matches_functional(cuda_device):
    """B = 512 (4B > C1_PRE_MIN_SLABS): the engine pre-reduces the 4B conv1 partial rows in 256
    fixed-order groups before the conv reduce; its gradients equal the functional path's (one pass
    over the 4B rows) up to fp32 summation order, and a repeated run gives the same bits."""
    from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT
    from pytorch_mnist_ddp_amd.ops import functional as Fk
    B = 512

    def fresh_net():
        torch.manual_seed(1)
        return Net()

    tr = load_mnist(synthetic_data=True, train=True, synthetic_size=B, verbose=False)
    idx = torch.arange(B)
    grads = []
    for _ in range(2):
        ms = ModelState(fresh_net(), cuda_device, lr=1.0)
        t = FusedTrainer(ms, tr, None, B, 1, num_samples=B, seed=1, graph_steps=0, dropout=False)
        t.train_epoch(1, idx)
        t.synchronize()
        torch.cuda.synchronize()
        grads.append(ms.grad.clone())
    assert torch.equal(grads[0], grads[1])
    ms2 = ModelState(fresh_net(), cuda_device, lr=1.0)
    u8 = tr.images.reshape(B, -1).contiguous().to(cuda_device)
    lab = tr.targets.to(torch.int32).to(cuda_device)
    buf = Fk.StepBuffers.allocate(B, cuda_device)
    ms2.set_state(0, seed=1, rng_base=0, flags=FLAG_NO_DROPOUT)
    Fk.train_step(ms2, u8, lab, torch.arange(B, dtype=torch.int32, device=cuda_device), buf, update=False)
    torch.cuda.synchronize()
    g_eng, g_fn = ms.views(grads[0]), ms2.views(ms2.grad)
    for name in g_fn:
        err = ((g_eng[name] - g_fn[name]).norm() / g_fn[name].norm().clamp_min(1e-30)).item()
        assert err < 1e-4, (name, err)


@pytest.mark.parametrize("B,grid", [(200, 800), (200, 37), (512, 512)])
def test_dgrad_persistent_grid_independent(cuda_device, B, grid):
    """Persistent conv2_dgrad (conv2 weights staged once per workgroup, items it, it+G, ... with the
    next item's loads in flight under the MFMA loop): any grid gives the bits of the default one -
    one item per workgroup (4B), a small odd grid (37 workgroups: ~22 items each, ragged last round)."""
    idx = torch.randperm(B * 4, generator=torch.Generator().manual_seed(23))
    out = {}
    C = None
    try:
        for g in (0, grid):
            from pytorch_mnist_ddp_amd.ops import native
            C = native.load()
            C.set_dgrad_grid(g)
            _, ms, t = _trainer(cuda_device, graph_steps=2, n_train=B * 4, B=B)
            t.train_epoch(1, idx)
            t.synchronize()
            torch.cuda.synchronize()
            out[g] = (ms.param.clone(), t.loss_log.clone(), ms.grad.clone())
    finally:
        if C is not None:
            C.set_dgrad_grid(0)
    a, b = out[0], out[grid]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


@pytest.mark.parametrize("B", [200, 512])
def test_wgrad_staggered_halves_agree(cuda_device, B):
    """conv2_wgrad with two staggered 4-wave halves (alternate chunks, accumulators summed half 0 +
    half 1; the large-batch default) vs the 8-wave lean kernel: the same conv gradients up to fp32
    summation order, and each form repeats bit for bit."""
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load()
    idx = torch.randperm(B, generator=torch.Generator().manual_seed(29))
    grads = {}
    try:
        for form in (0, 1, 1):
            C.set_wgrad_form(form)
            _, ms, t = _trainer(cuda_device, graph_steps=0, n_train=B, B=B, dropout=False, overlap=False)
            t.train_epoch(1, idx)
            t.synchronize()
            torch.cuda.synchronize()
            g = ms.grad.clone()
            if form in grads:
                assert torch.equal(grads[form], g)
            grads[form] = g
    finally:
        C.set_wgrad_form(-1)
    g0, g1 = grads[0], grads[1]
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 1e-5, rel
