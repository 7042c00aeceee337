"""Diagnostic: do IPC handles of different processes' buffers collide byte for byte?

    python tools/ipc_handles.py [--procs 4] [--comms 3]

Each process creates ``--comms`` world-1 xGMI communicators (the allocation sequence a trainer does)
and prints the hex of the four exported handles (input, output, flags, staging) of each.  Identical
bytes across processes mean an importer cannot tell a peer's buffer from its own."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(r, comms, q):
    import torch
    from pytorch_mnist_ddp_amd.ops import native
    torch.cuda.set_device(0)
    C = native.load()
    keep, out = [], []
    for c in range(comms):
        x = C.XgmiComm(1, 0, 0, 1200000, 2, 32768, 1)
        keep.append(x)
        rec = bytes(x.record())
        out.append([rec[64 * h:64 * h + 64].hex() for h in range(4)])
    q.put((r, os.getpid(), out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--comms", type=int, default=3)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.comms, q)) for r in range(a.procs)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    seen = {}
    for r, pid, out in res:
        for c, hs in enumerate(out):
            for h, hx in enumerate(hs):
                print(f"proc {r} pid {pid} comm {c} buf {'in out flags stage'.split()[h]:5s} {hx[:48]}...")
                seen.setdefault(hx, []).append((r, c, h))
    dup = {k: v for k, v in seen.items() if len(v) > 1}
    print(f"IPC_HANDLES distinct={len(seen)} duplicated={len(dup)}")
    for k, v in dup.items():
        print("  same bytes:", v)


if __name__ == "__main__":
    main()
