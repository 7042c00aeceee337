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
