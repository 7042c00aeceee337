"""T0: IDX reader/writer, synthetic data, torchvision-equivalent normalisation."""
import numpy as np
import torch

from pytorch_mnist_ddp_amd.data import idx, synthetic
from pytorch_mnist_ddp_amd.data.datasets import MNIST_MEAN, MNIST_STD, load_mnist, normalize_u8


def test_idx_roundtrip_plain_and_gzip(tmp_path):
    imgs = np.random.default_rng(0).integers(0, 256, size=(5, 28, 28), dtype=np.uint8)
    labels = np.arange(5, dtype=np.uint8)
    raw = tmp_path / "MNIST" / "raw"
    idx.write_idx(str(raw / "train-images-idx3-ubyte.gz"), imgs)
    idx.write_idx(str(raw / "train-labels-idx1-ubyte"), labels)
    assert (idx.read_idx(str(raw / "train-images-idx3-ubyte.gz")) == imgs).all()
    d = load_mnist(str(tmp_path), train=True, synthetic_data=False)
    assert d.images.shape == (5, 28, 28) and d.images.dtype == torch.uint8
    assert d.targets.tolist() == list(range(5)) and d.source.startswith("idx:")


def test_idx_header_magic():
    import struct
    hdr = struct.pack(">HBB", 0, 8, 3) + struct.pack(">iii", 1, 2, 2) + bytes(range(4))
    import tempfile, os
    with tempfile.NamedTemporaryFile(delete=False) as f:
        f.write(hdr)
    try:
        a = idx.read_idx(f.name)
        assert a.shape == (1, 2, 2) and a.dtype == np.uint8 and a.reshape(-1).tolist() == [0, 1, 2, 3]
    finally:
        os.unlink(f.name)


def test_missing_files_fall_back_to_synthetic_or_raise(tmp_path):
    d = load_mnist(str(tmp_path), train=False, synthetic_data=None, synthetic_size=100, verbose=False)
    assert d.source == "synthetic" and len(d) == 100
    try:
        load_mnist(str(tmp_path), train=False, synthetic_data=False)
        raise AssertionError("expected FileNotFoundError")
    except FileNotFoundError:
        pass


def test_synthetic_shapes_determinism_and_balance():
    a_img, a_lab = synthetic.generate(3000, seed=11)
    b_img, b_lab = synthetic.generate(3000, seed=11)
    assert a_img.shape == (3000, 28, 28) and a_img.dtype == torch.uint8 and a_lab.dtype == torch.int64
    assert torch.equal(a_img, b_img) and torch.equal(a_lab, b_lab)
    counts = torch.bincount(a_lab, minlength=10)
    assert counts.min() > 200
    # non-trivial but learnable: a nearest-class-mean classifier gets well above chance
    x = a_img.float().reshape(3000, -1)
    means = torch.stack([x[a_lab == c].mean(0) for c in range(10)])
    t_img, t_lab = synthetic.generate(1000, seed=12)
    pred = torch.cdist(t_img.float().reshape(1000, -1), means).argmin(1)
    acc = (pred == t_lab).float().mean().item()
    assert 0.3 < acc < 1.0


def test_normalize_matches_torchvision_formula():
    u8 = torch.arange(256, dtype=torch.uint8).reshape(1, 16, 16)
    x = normalize_u8(u8)
    ref = (u8.float().div(255) - MNIST_MEAN) / MNIST_STD
    assert x.shape == (1, 1, 16, 16)
    assert torch.equal(x[0, 0], ref[0])


def test_split_sizes_match_mnist():
    assert synthetic.TRAIN_SIZE == 60000 and synthetic.TEST_SIZE == 10000


def test_native_generator_v3_thread_invariant_and_balanced(monkeypatch):
    """Generator v3 (csrc/data/synthetic_gen.cpp): every sample is a pure function of (seed, index),
    so 1 and 7 threads give the same bytes, a prefix of a larger split equals the smaller split, the
    classes are balanced, ~1 % of the train labels are flipped, and train / test streams differ."""
    import torch
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    a_img, a_lab = synthetic.generate_native(3000, seed=11, label_noise=0.0)
    monkeypatch.setenv("OMP_NUM_THREADS", "7")
    b_img, b_lab = synthetic.generate_native(3000, seed=11, label_noise=0.0)
    assert a_img.dtype == torch.uint8 and a_img.shape == (3000, 28, 28) and a_lab.dtype == torch.int64
    assert torch.equal(a_img, b_img) and torch.equal(a_lab, b_lab)
    c_img, c_lab = synthetic.generate_native(1000, seed=11, label_noise=0.0)
    assert torch.equal(c_img, a_img[:1000]) and torch.equal(c_lab, a_lab[:1000])
    counts = torch.bincount(a_lab, minlength=10)
    assert counts.min() > 240 and counts.max() < 360
    n_img, n_lab = synthetic.generate_native(20000, seed=11, label_noise=0.01)
    assert torch.equal(n_img[:3000], a_img)                     # label noise leaves the images alone
    flipped = (n_lab[:3000] != a_lab).float().mean().item()
    assert flipped < 0.02
    assert 0.003 < (n_lab != synthetic.generate_native(20000, seed=11)[1]).float().mean().item() < 0.02
    d_img, _ = synthetic.generate_native(1000, seed=12)
    assert not torch.equal(d_img, c_img)
    assert 30 < a_img.float().mean().item() < 80                # strokes + speckle, not blank / saturated


def test_synthetic_split_is_generated_not_cached(tmp_path):
    """load_mnist(synthetic) builds the split in-process every run (no disk cache, so no cold / warm
    difference inside the reference's timer) and gives the same bytes each time."""
    import os
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    a = load_mnist(str(tmp_path), train=False, synthetic_data=True, synthetic_size=500, verbose=False)
    b = load_mnist(str(tmp_path), train=False, synthetic_data=True, synthetic_size=500, verbose=False)
    assert torch_equal(a.images, b.images) and torch_equal(a.targets, b.targets)
    assert not os.path.exists(os.path.join(str(tmp_path), "synthetic_cache"))


def torch_equal(x, y):
    import torch
    return torch.equal(x, y)
