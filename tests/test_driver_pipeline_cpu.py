"""CPU test of the fused driver's pipelined epoch loop (driver._run_fused) with a stand-in trainer:
the printed lines come out in the reference's order (each epoch's train lines, then its test line)
and the global-RNG draws happen in the reference's order (train base seed, sampler permutation,
test base seed[, test permutation], next epoch ...; mnist_ddp.py:186-190, mnist.py:127-131), although
the evaluation of epoch e is only read back while epoch e+1 runs and e+1's sampler order is drawn
before that read-back."""
import types

import pytest

import torch

from pytorch_mnist_ddp_amd import driver
from pytorch_mnist_ddp_amd.data.samplers import RandomIndexStream, SequentialIndexStream
from pytorch_mnist_ddp_amd.engine.trainer import EpochStats
from pytorch_mnist_ddp_amd.utils.profiling import PhaseTimes


class _Handle:
    def __init__(self, log, epoch):
        self.log, self.epoch = log, epoch

    def result(self):
        self.log.append(("eval_read", self.epoch))
        return 1.0 * self.epoch, 7, 10


class _FakeTrainer:
    def __init__(self, log, steps):
        self.log, self.steps = log, steps
        self.setup = PhaseTimes()
        self.allreduce, self.transport_report, self.allreduce_timings = None, {}, {}
        self.profile_left = 0

    def set_lr(self, lr):
        self.log.append(("lr", round(lr, 6)))

    def train_epoch(self, epoch, idx, log_interval=10, dry_run=False, log_fn=None, sync=True, before_log=None):
        self.log.append(("train_enqueue", epoch, int(idx[0])))
        for b in range(0, self.steps, log_interval):
            if before_log is not None:
                before_log()
                before_log = None
            log_fn(b, 2, 0.5)
        if before_log is not None:
            before_log()
        return EpochStats(epoch, self.steps, 2 * self.steps, 0.01, {}, 0.01 if sync else None, None)

    def evaluate_async(self):
        self.log.append(("eval_enqueue",))
        return _Handle(self.log, len([e for e in self.log if e[0] == "eval_enqueue"]))

    def synchronize(self):
        self.log.append(("sync",))

    def check_errors(self):
        self.log.append(("check",))


def test_pipelined_epochs_keep_reference_print_and_rng_order(monkeypatch, capsys):
    log = []
    real_consume = driver.consume_loader_base_seed

    def consume():
        log.append(("seed", real_consume()))

    class Stream(RandomIndexStream):
        def epoch_indices(self):
            idx = super().epoch_indices()
            log.append(("perm", int(idx[0])))
            return idx

    monkeypatch.setattr(driver, "consume_loader_base_seed", consume)
    fake = _FakeTrainer(log, steps=20)
    monkeypatch.setattr("pytorch_mnist_ddp_amd.engine.trainer.FusedTrainer", lambda *a, **k: fake)
    monkeypatch.setattr("pytorch_mnist_ddp_amd.engine.state.ModelState",
                        lambda model, device, lr=1.0: types.SimpleNamespace(param=torch.zeros(1)))
    args = types.SimpleNamespace(_setup=PhaseTimes(), _prewarm=types.SimpleNamespace(join=lambda: None, seconds=0.0, steps={},
                                                                                    error=None),
                                 lr=1.0, gamma=0.7, allreduce="auto", graph_steps=None, log_interval=10,
                                 batch_size=2, test_batch_size=10, profile=False, profile_steps=0, epochs=3,
                                 dry_run=False, check_sync=False, json_log=None, save_model=False, dtype="bf16",
                                 _pending_comm=None, seed=1)
    net = driver.Net()
    torch.manual_seed(3)
    train = [0] * 40
    test = [0] * 10
    driver._run_fused(args, net, torch.device("cpu"), train, test, Stream(40), SequentialIndexStream(10),
                      False, 1, 0, 0, True)
    out = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith(("Train Epoch", "Test set"))]
    kinds = [ln.split(":")[0].split(" [")[0] for ln in out]
    assert kinds == (["Train Epoch"] * 2 + ["Test set"]) * 3, out
    # RNG draws: the same values, in the same order, as the sequential reference loop
    torch.manual_seed(3)
    ref = []
    for _ in range(3):
        ref.append(("seed", real_consume()))
        ref.append(("perm", int(RandomIndexStream(40).epoch_indices()[0])))
        ref.append(("seed", real_consume()))
    assert [e for e in log if e[0] in ("seed", "perm")] == ref
    # pipelining: epoch e's evaluation is read back after epoch e+1 was enqueued
    ev = [e for e in log if e[0] in ("train_enqueue", "eval_read")]
    assert [e[0] for e in ev] == ["train_enqueue", "train_enqueue", "eval_read", "train_enqueue", "eval_read",
                                  "eval_read"]
    assert [e[1] for e in log if e[0] == "lr"] == [1.0, 0.7, 0.49]
    # fail fast: the device error flags are read at every epoch boundary, after that epoch's work
    # (pipelined epochs used to surface a hand-off timeout only after the last epoch)
    reads = [e[0] for e in log if e[0] in ("eval_read", "check")]
    assert reads == ["eval_read", "check"] * 3


def test_fatal_transport_hang_exits_without_teardown(monkeypatch, capsys):
    """A TransportHang (a collective stuck on the device) in the real entry point leaves through
    os._exit - the interpreter's teardown of RCCL / HIP objects would wait for the stuck kernel."""
    from pytorch_mnist_ddp_amd.engine.trainer import TransportHang

    def boom(*a, **k):
        raise TransportHang("rank 0: RCCL schedule validation did not complete within 1 s")

    exits = []

    def fake_exit(code):
        exits.append(code)
        raise SystemExit(code)

    monkeypatch.setattr(driver, "run", boom)
    monkeypatch.setattr(driver.os, "_exit", fake_exit)
    for entry in (driver.main_mnist_ddp, driver.main_mnist):
        with pytest.raises(SystemExit):
            entry([])
    assert exits == [3, 3]
    assert "FATAL: TransportHang" in capsys.readouterr().err
    # an ordinary error still propagates (normal teardown)
    monkeypatch.setattr(driver, "run", lambda *a, **k: (_ for _ in ()).throw(ValueError("x")))
    with pytest.raises(ValueError):
        driver.main_mnist_ddp([])
