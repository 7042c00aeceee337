"""The reference's stdout formats, verbatim."""
from __future__ import annotations


def train_line(epoch: int, seen: int, total: int, batch_idx: int, n_batches: int, loss: float) -> str:
    # mnist.py:47-49 / mnist_ddp.py:77-79, 82-84
    return 'Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f}'.format(
        epoch, seen, total, 100. * batch_idx / n_batches, loss)


def test_line(test_loss: float, correct: int, total: int) -> str:
    # mnist.py:68-70 = mnist_ddp.py:103-105
    return '\nTest set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n'.format(
        test_loss, correct, total, 100. * correct / total)


def total_time_line(seconds: float) -> str:
    # mnist_ddp.py:203 (value is seconds although labelled "ms"; preserved)
    return f'Total cost time:{seconds} ms'


def print_line(line: str) -> None:
    """One whole line in ONE write: lines every rank prints (the distributed-init and Total-cost-time
    lines) stay whole in a shared pipe even with an unbuffered stdout, where ``print`` writes the text
    and the newline separately and two ranks' lines can interleave."""
    import sys
    sys.stdout.write(line + "\n")
    sys.stdout.flush()
