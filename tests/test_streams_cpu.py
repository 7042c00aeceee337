"""Engine stream selection on the host (no GPU): one process-wide pair of non-blocking streams per
device (engine/trainer.py make_streams), created once and reused by every trainer."""
import torch

from pytorch_mnist_ddp_amd.engine import trainer


def test_make_streams_creates_one_non_blocking_pair_per_device(monkeypatch):
    calls = []

    class FakeC:
        @staticmethod
        def create_stream(device, dedicated, priority):
            calls.append((device, dedicated, priority))
            return 1000 + len(calls)

        @staticmethod
        def probe_streams(x, y, timeout_s=0.5):
            return True

    monkeypatch.setattr(trainer.native, "load", lambda: FakeC)
    monkeypatch.setattr(torch.cuda, "ExternalStream", lambda ptr, device=None: ("stream", ptr, str(device)))
    monkeypatch.setattr(trainer, "_ENGINE_STREAMS", {})
    monkeypatch.setattr(trainer, "_STREAM_KIND", {})
    a = trainer.make_streams("cuda:3")
    b = trainer.make_streams(torch.device("cuda", 3))
    assert a is b and len(a) == 2 and a[0] != a[1]
    assert calls == [(3, False, 0), (3, False, 0)]      # plain non-blocking streams, created once
    assert trainer.stream_kind(3).startswith("non-blocking")


def test_make_streams_falls_back_to_dedicated_queues_when_the_pair_shares_one(monkeypatch):
    calls, destroyed = [], []

    class FakeC:
        @staticmethod
        def create_stream(device, dedicated, priority):
            calls.append(dedicated)
            return 2000 + len(calls)

        @staticmethod
        def probe_streams(x, y, timeout_s=0.5):
            return False                                 # the non-blocking pair shares a queue

        @staticmethod
        def destroy_stream(s):
            destroyed.append(s)

    monkeypatch.setattr(trainer.native, "load", lambda: FakeC)
    monkeypatch.setattr(torch.cuda, "ExternalStream", lambda ptr, device=None: ("stream", ptr))
    monkeypatch.setattr(trainer, "_ENGINE_STREAMS", {})
    monkeypatch.setattr(trainer, "_STREAM_KIND", {})
    for k in [k for k in list(__import__("os").environ) if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    pair = trainer.make_streams("cuda:0")
    assert calls == [False, False, True, True] and destroyed == [2001, 2002]
    assert [p[1] for p in pair] == [2003, 2004] and trainer.stream_kind(0).startswith("cu_masked")


def test_make_streams_keeps_the_plain_pair_under_rocprofv3(monkeypatch):
    calls = []

    class FakeC:
        @staticmethod
        def create_stream(device, dedicated, priority):
            calls.append(dedicated)
            return 3000 + len(calls)

        @staticmethod
        def probe_streams(x, y, timeout_s=0.5):
            return False

    monkeypatch.setattr(trainer.native, "load", lambda: FakeC)
    monkeypatch.setattr(torch.cuda, "ExternalStream", lambda ptr, device=None: ("stream", ptr))
    monkeypatch.setattr(trainer, "_ENGINE_STREAMS", {})
    monkeypatch.setattr(trainer, "_STREAM_KIND", {})
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    trainer.make_streams("cuda:0")
    assert calls == [False, False]                   # no CU-masked streams under the profiler
