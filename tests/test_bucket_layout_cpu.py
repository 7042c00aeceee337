"""--bucket-cap-mb / --first-bucket-mb on the fused engine: the DDP bucket
assignment (torch DDP semantics, parallel/ddp.py) is mapped onto the engine's schedules - the two
buckets {fc},{conv} at the default caps, one bucket when the first cap swallows everything - and any
other layout is refused with a clear error instead of being silently ignored."""
import pytest

from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.parallel.ddp import compute_bucket_assignment, engine_bucket_layout

MIB = 1024 * 1024


def _buckets(first_mb, cap_mb):
    params = list(Net().parameters())
    ready = list(reversed(range(len(params))))
    sizes = [params[i].numel() * 4 for i in ready]
    return [[ready[j] for j in b] for b in compute_bucket_assignment(sizes, [int(first_mb * MIB), int(cap_mb * MIB)])]


def test_default_caps_give_torch_rebuilt_layout():
    b = _buckets(1.0, 25.0)
    assert b == [[7, 6, 5, 4], [3, 2, 1, 0]]
    assert engine_bucket_layout(b) is True


@pytest.mark.parametrize("first,cap", [(5.0, 25.0), (25.0, 25.0), (100.0, 1.0)])
def test_single_bucket_layouts(first, cap):
    b = _buckets(first, cap)
    assert len(b) == 1
    assert engine_bucket_layout(b) is False


@pytest.mark.parametrize("first,cap", [(1.0, 0.01), (0.001, 25.0), (0.001, 0.001)])
def test_unsupported_layouts_are_refused(first, cap):
    b = _buckets(first, cap)
    assert len(b) > 2 or b[0] != [7, 6, 5, 4]
    with pytest.raises(ValueError, match="--engine module"):
        engine_bucket_layout(b)


def test_dist_backend_flag():
    from pytorch_mnist_ddp_amd import cli
    a = cli.parse_args(ddp=True, argv=["--dist-backend", "gloo", "--allreduce", "xgmi"])
    assert a.pg_backend == "gloo" and a.allreduce == "xgmi"
    assert cli.parse_args(ddp=True, argv=[]).pg_backend is None
