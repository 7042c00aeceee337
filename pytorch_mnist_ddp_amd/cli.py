"""Command-line flags for ``mnist.py`` / ``mnist_ddp.py``.

Reference flags and defaults are reproduced verbatim (``mnist.py:75-96``,
``mnist_ddp.py:110-135``).  Deliberate additions (all default to reference
behaviour):

* ``--local-rank`` accepted as an alias of ``--local_rank``: torch>=2.0's
  ``torch.distributed.launch`` appends ``--local-rank=<i>`` which the reference's
  underscore-only flag rejects.
* ``--synthetic`` / ``--data-root`` / ``--synthetic-train-size`` /
  ``--synthetic-test-size``: offline data selection.
* ``--bucket-cap-mb`` / ``--first-bucket-mb``: DDP gradient bucket sizing.
* ``--engine {fused,module}``: native step engine vs the reference's module-level loop.
* ``--dtype {bf16,fp32}``: bf16 = the MI355X kernels (bf16 MFMA operands, fp32 accumulation,
  fp32 master weights / optimizer state / gradient all-reduce); fp32 = the reference's precision:
  the fused engine's fp32 step (csrc/kernels/f32_net.hip, f32-input MFMA GEMMs; RCCL or xGMI at N > 1),
  or stock torch fp32 ops with ``--engine module``.
* ``--dist-backend``: process-group backend override (``gloo`` + ``--allreduce xgmi`` needs no
  RCCL at all, e.g. several ranks on one GPU).
* ``--check-sync``: all-gather a parameter checksum after every epoch (DDP desync detector).
* ``--graph-steps``: training steps captured per HIP graph (0 = eager launches).
* ``--profile``: roctx ranges + per-epoch device timing; ``--json-log``: machine
  readable per-epoch metrics.
* ``--resume``: optional checkpoint to load before training (off by default).
"""
from __future__ import annotations

import argparse


def _reference_flags(parser: argparse.ArgumentParser) -> None:
    parser.add_argument('--batch-size', type=int, default=64, metavar='N',
                        help='input batch size for training (default: 64)')
    parser.add_argument('--test-batch-size', type=int, default=1000, metavar='N',
                        help='input batch size for testing (default: 1000)')
    parser.add_argument('--epochs', type=int, default=14, metavar='N',
                        help='number of epochs to train (default: 14)')
    parser.add_argument('--lr', type=float, default=1.0, metavar='LR',
                        help='learning rate (default: 1.0)')
    parser.add_argument('--gamma', type=float, default=0.7, metavar='M',
                        help='Learning rate step gamma (default: 0.7)')
    parser.add_argument('--no-cuda', action='store_true', default=False,
                        help='disables GPU training')
    parser.add_argument('--dry-run', action='store_true', default=False,
                        help='quickly check a single pass')
    parser.add_argument('--seed', type=int, default=1, metavar='S',
                        help='random seed (default: 1)')
    parser.add_argument('--log-interval', type=int, default=10, metavar='N',
                        help='how many batches to wait before logging training status')
    parser.add_argument('--save-model', action='store_true', default=False,
                        help='For Saving the current Model')


def _framework_flags(parser: argparse.ArgumentParser) -> None:
    g = parser.add_argument_group("mi355x framework options")
    g.add_argument('--data-root', default='./data', help='MNIST root (torchvision layout)')
    g.add_argument('--synthetic', action='store_true', default=None,
                   help='use deterministic synthetic 28x28 data (auto when MNIST files are absent)')
    g.add_argument('--synthetic-train-size', type=int, default=None)
    g.add_argument('--synthetic-test-size', type=int, default=None)
    g.add_argument('--synthetic-size', dest='synthetic_train_size', type=int, default=None,
                   help='alias of --synthetic-train-size')
    g.add_argument('--dtype', choices=['bf16', 'fp32'], default='bf16',
                   help='bf16: MI355X bf16-MFMA kernels (default); fp32: the fp32 step (f32-input MFMA kernels; '
                        'torch fp32 ops with --engine module)')
    g.add_argument('--check-sync', action='store_true', default=False,
                   help='verify parameters are identical on every rank after each epoch')
    g.add_argument('--engine', choices=['fused', 'module'], default=None,
                   help='fused: native step engine (GPU default); module: the reference loop over '
                        'Net/DDP/Adadelta (always used with --no-cuda)')
    g.add_argument('--graph-steps', type=int, default=None,
                   help='training steps per captured HIP graph (default 50; 0 = eager)')
    g.add_argument('--bucket-cap-mb', type=float, default=25.0,
                   help='DDP gradient bucket cap in MiB (default 25, as torch DDP)')
    g.add_argument('--first-bucket-mb', type=float, default=1.0,
                   help='DDP first-bucket cap in MiB (default 1, as torch DDP)')
    g.add_argument('--allreduce', choices=['auto', 'rccl', 'xgmi', 'fastest'], default=None,
                   help='DDP gradient all-reduce of the fused engine: RCCL, the direct xGMI kernels, auto '
                        '(default: xGMI when it validates at startup on one node, RCCL only as the fallback - '
                        'never waited for otherwise), or fastest (validate and time both, keep the faster)')
    g.add_argument('--dist-backend', dest='pg_backend', choices=['nccl', 'gloo'], default=None,
                   help='torch.distributed backend for bootstrap / construction collectives (default: nccl = '
                        'RCCL on GPU, gloo with --no-cuda); gloo + --allreduce xgmi runs DDP without RCCL')
    g.add_argument('--profile', action='store_true', default=False,
                   help='roctx ranges per epoch (train / eval) and, on the fused engine, a window of '
                        '--profile-steps eager steps with one range per phase (fwd, bwd, all-reduce, update)')
    g.add_argument('--profile-steps', type=int, default=20,
                   help='steps in the --profile window at the start of training (default 20)')
    g.add_argument('--json-log', default=None, help='append per-epoch JSON metrics to this file')
    g.add_argument('--resume', default=None, help='load a state_dict checkpoint before training')


def build_parser(ddp: bool) -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description='PyTorch MNIST Example')
    _reference_flags(parser)
    if ddp:
        parser.add_argument('--local_rank', '--local-rank', dest='local_rank', type=int,
                            help='local rank, will passed by ddp')
        parser.add_argument("--world-size", default=1, type=int,
                            help="number of distributed processes")
        parser.add_argument("--dist-url", default="env://", type=str,
                            help="url used to set up distributed training")
    _framework_flags(parser)
    return parser


def parse_args(ddp: bool, argv=None) -> argparse.Namespace:
    return build_parser(ddp).parse_args(argv)
