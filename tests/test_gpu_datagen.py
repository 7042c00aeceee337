"""T1: the synthetic generator's device render (csrc/kernels/datagen.hip) gives the host render's bytes
(csrc/data/synthetic_gen.cpp; the per-pixel math of both is csrc/data/synth_render.h, contraction off),
so the fused engine's HBM-rendered split and the module / CPU path train on identical data."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,params", [(3000, None), (777, {"overlay": 1.3, "rot_deg": 25.0, "namp": 0.4})])
def test_device_render_equals_host_render(cuda_device, n, params):
    from pytorch_mnist_ddp_amd.data import synthetic as S
    pl = S.SynthPlan(n, seed=12345, label_noise=0.01, params=params)
    host = pl.render_cpu().reshape(n, -1)
    dev = pl.render_device(cuda_device).cpu()
    bad = (host != dev).sum().item()
    assert bad == 0, f"{bad} of {host.numel()} pixels differ"


def test_fused_trainer_uses_device_rendered_split(cuda_device):
    """load_mnist(synthetic) renders nothing on the host until asked; the trainer's HBM copy equals
    the host render of the same split."""
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    d = load_mnist(train=False, synthetic_data=True, synthetic_size=1000, verbose=False)
    assert d._images is None
    on_dev = d.device_images(cuda_device).cpu()
    assert d._images is None
    assert torch.equal(on_dev, d.images.reshape(1000, -1))
