"""Engine stream selection on the host (no GPU): plain streams under rocprofv3, reported by stream_kind."""
from pytorch_mnist_ddp_amd.engine import trainer


def test_profiler_detection_and_stream_kind(monkeypatch):
    for k in [k for k in list(__import__("os").environ) if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    monkeypatch.setattr(trainer, "_STREAM_FALLBACK", [])
    assert not trainer.under_profiler()
    assert trainer.stream_kind() == "cu_masked"
    monkeypatch.setattr(trainer, "_STREAM_FALLBACK", ["hipExtStreamCreateWithCUMask failed"])
    assert trainer.stream_kind().startswith("plain (CU-masked stream failed")
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    assert trainer.under_profiler()
    assert trainer.stream_kind() == "plain (rocprofv3)"
