"""T0: CLI parity with the reference (mnist.py:75-96, mnist_ddp.py:110-135)."""
from pytorch_mnist_ddp_amd import cli

REF_DEFAULTS = {"batch_size": 64, "test_batch_size": 1000, "epochs": 14, "lr": 1.0, "gamma": 0.7,
                "no_cuda": False, "dry_run": False, "seed": 1, "log_interval": 10, "save_model": False}


def test_reference_defaults_both_scripts():
    for ddp in (False, True):
        a = cli.parse_args(ddp=ddp, argv=[])
        for k, v in REF_DEFAULTS.items():
            assert getattr(a, k) == v, k


def test_ddp_extra_flags_and_local_rank_aliases():
    a = cli.parse_args(ddp=True, argv=[])
    assert a.local_rank is None and a.world_size == 1 and a.dist_url == "env://"
    assert cli.parse_args(ddp=True, argv=["--local_rank", "3"]).local_rank == 3
    # torch>=2.0 torch.distributed.launch passes --local-rank=<i> (reference rejects it)
    assert cli.parse_args(ddp=True, argv=["--local-rank=5"]).local_rank == 5


def test_reference_readme_command_parses():
    a = cli.parse_args(ddp=True, argv="--batch-size 200 --epochs 20".split())
    assert a.batch_size == 200 and a.epochs == 20


def test_framework_flags_default_to_reference_behaviour():
    a = cli.parse_args(ddp=True, argv=[])
    assert a.resume is None and a.profile is False and a.bucket_cap_mb == 25.0 and a.first_bucket_mb == 1.0
    assert a.synthetic is None and a.data_root == "./data"
    assert a.dtype == "bf16" and a.check_sync is False
    b = cli.parse_args(ddp=False, argv=["--dtype", "fp32", "--synthetic-size", "123", "--check-sync"])
    assert b.dtype == "fp32" and b.synthetic_train_size == 123 and b.check_sync


def test_fail_fast_on_non_finite_loss():
    import pytest
    from pytorch_mnist_ddp_amd.driver import _check_finite
    _check_finite(0.5, 1, 0)
    for bad in (float("nan"), float("inf")):
        with pytest.raises(FloatingPointError):
            _check_finite(bad, 1, 10)
