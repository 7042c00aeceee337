"""Per-kernel device timing with HIP events over the functional entry points (1 GPU).

usage: python tools/kernel_bench.py [B]
Times every stage of one training step, and fc_bwd's three workgroup roles on their own.
"""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_mnist_ddp_amd.data.datasets import load_mnist  # noqa: E402
from pytorch_mnist_ddp_amd.engine.state import ModelState  # noqa: E402
from pytorch_mnist_ddp_amd.models.net import Net  # noqa: E402
from pytorch_mnist_ddp_amd.ops import functional as Fk  # noqa: E402
from pytorch_mnist_ddp_amd.ops import native  # noqa: E402
from pytorch_mnist_ddp_amd.ops.functional import round_up  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    C = native.load()
    tr = load_mnist(synthetic_data=True, train=True, synthetic_size=max(B, 1024), verbose=False)
    torch.manual_seed(0)
    ms = ModelState(Net(), dev)
    u8 = tr.images.reshape(len(tr), -1).contiguous().to(dev)
    lab = tr.targets.to(torch.int32).to(dev)
    idx = torch.arange(B, dtype=torch.int32, device=dev)
    buf = Fk.StepBuffers.allocate(B, dev)
    ms.set_state(0, seed=1, rng_base=0)
    Fk.train_step(ms, u8, lab, idx, buf, update=False)
    torch.cuda.synchronize()
    p = native.ptr
    s = torch.cuda.current_stream().cuda_stream

    def fcb(role):
        return lambda: C.fc_bwd(p(buf.dz1), p(buf.p), p(buf.pmask), p(ms.w1t), p(buf.h_bf), p(buf.dl_bf),
                                p(buf.loss_rows), p(ms.state), p(ms.grad), p(buf.dyc), 0, 1.0, 1.0 / B, B,
                                round_up(B, 32), s, role=role, part=p(buf.fcpart))
    rows = [("fc_bwd (all roles)", fcb(-1)), ("fc_bwd role C (dW2, loss)", fcb(0)),
            ("fc_bwd role A (dW1, 145 WGs)", fcb(1)), ("fc_bwd role B (dy)", fcb(2)),
            *([("fc_bwd_dw1 (role A, lean kernel)", fcb(3)), ("fc_bwd roles C+B", fcb(4))] if B > 1024 else []),
            ("fc1_fwd", lambda: Fk.fc1_fwd(ms, buf)),
            ("conv_bwd (dgrad+wgrad+reduce)", lambda: Fk.conv_bwd(ms, u8, idx, buf))]
    for name, fn in rows:
        print(f"{name:34s} {timeit(fn):8.2f} us")


if __name__ == "__main__":
    main()
