"""CPU tests of the launch / bootstrap plumbing that the multi-GPU driver run depends on:

* ``bench.py --gpus N`` without a launcher fails fast, with one JSON line and a clear message, when
  the node shows fewer than N GPUs (the driver's plain command on the wrong box);
* the store-based host collectives (``parallel/hostcomm.py``) that replace torch collectives on the
  default process group during startup: results in rank order, key garbage collection, and a peer's
  abort reaching ranks blocked in a collective within seconds instead of the 300 s timeout.
"""
import datetime
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_gpus_n_fails_fast_without_enough_gpus():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = ROOT
    env.pop("MNIST_AMD_ONE_GPU", None)
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "5"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 3, (r.stdout, r.stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["value"] is None and j["n_gpus"] == 8 and "needs 8 visible GPUs" in j["error"]
    assert "needs 8 visible GPUs" in r.stderr
    assert time.perf_counter() - t0 < 60


def _hc_worker(rank, world, port, q, mode):
    import torch.distributed as dist
    from pytorch_mnist_ddp_amd.parallel.hostcomm import get_hostcomm, reset_hostcomm
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank,
                            timeout=datetime.timedelta(seconds=60))
    try:
        hc = get_hostcomm()
        if mode == "ops":
            out = [hc.gather_strings(f"r{rank}"), hc.all_ok(True), hc.all_ok(rank != 2), hc.max(0.5 * rank),
                   hc.all_equal(b"x"), hc.all_equal(bytes([rank]))]
            for _ in range(10):                       # keys of old operations are deleted as we go
                hc.barrier()
            store = dist.distributed_c10d._get_default_store()
            live = sum(store.check([hc._key(s, rank)]) for s in range(hc.seq))
            out.append(live)
            q.put((rank, out))
        elif mode == "channels":
            # a helper thread's channel and the main thread interleave their collectives differently
            # on every rank (random sleeps): each sequence still pairs up with its peers'
            import random
            import threading
            from pytorch_mnist_ddp_amd.parallel.hostcomm import channel, use_channel
            rnd = random.Random(rank)
            side = {}

            def helper():
                with use_channel(channel("helper")):
                    got = []
                    for i in range(8):
                        time.sleep(rnd.random() * 0.02)
                        got.append(get_hostcomm().gather_strings(f"h{i}r{rank}"))
                    side["h"] = got

            t = threading.Thread(target=helper)
            t.start()
            main = []
            for i in range(8):
                time.sleep(rnd.random() * 0.02)
                main.append(hc.gather_strings(f"m{i}r{rank}"))
            t.join(60)
            q.put((rank, (main, side.get("h"))))
            time.sleep(2.0)
        elif mode == "clone":
            # helper-thread clients are clones of the default store (same key namespace); two channels
            # of one name never see each other's keys; a default-store abort reaches a clone-channel wait
            from pytorch_mnist_ddp_amd.parallel.hostcomm import channel, own_store_client
            c1 = own_store_client()
            assert c1 is not None
            a = channel("setup", c1)
            first = a.gather_strings(f"a{rank}")
            b = channel("setup", own_store_client())   # a later channel of the same name
            second = b.gather_strings(f"b{rank}")
            assert a.prefix != b.prefix
            if rank == 1:
                time.sleep(1.0)
                hc.abort("rank 1 failed in xgmi setup")
                q.put((rank, (first, second, "aborted")))
            else:
                t0 = time.perf_counter()
                try:
                    b.barrier(timeout_s=120)
                    q.put((rank, (first, second, "no error")))
                except RuntimeError as e:
                    q.put((rank, (first, second, f"{time.perf_counter() - t0:.1f}|{e}")))
            time.sleep(3.0)
        else:                                         # rank 1 fails, the others wait in a collective
            if rank == 1:
                time.sleep(1.0)
                hc.abort("rank 1 failed in trainer: boom")
                q.put((rank, "aborted"))
            else:
                t0 = time.perf_counter()
                try:
                    hc.barrier(timeout_s=120)
                    q.put((rank, "no error"))
                except RuntimeError as e:
                    q.put((rank, f"{time.perf_counter() - t0:.1f}|{e}"))
            time.sleep(3.0)                           # keep rank 0's store up until every rank has read it
        reset_hostcomm()
    finally:
        dist.destroy_process_group()


def _run(world, mode):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hc_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    return res


def test_host_collectives_gloo():
    res = _run(3, "ops")
    for r in range(3):
        strings, ok_all, ok_some, mx, eq, neq, live = res[r]
        assert strings == ["r0", "r1", "r2"]
        assert ok_all is True and ok_some is False and mx == 1.0 and eq is True and neq is False
        assert live <= 2                              # only the last two operations' keys remain


def test_host_collective_abort_reaches_waiting_ranks():
    res = _run(3, "abort")
    assert res[1] == "aborted"
    for r in (0, 2):
        dt, msg = res[r].split("|", 1)
        assert "job aborted by a peer: rank 1 failed in trainer: boom" in msg
        assert float(dt) < 20.0                       # not the 120 s timeout


def test_host_collective_channels_are_independent():
    res = _run(3, "channels")
    for r in range(3):
        main, helper = res[r]
        assert main == [[f"m{i}r{q}" for q in range(3)] for i in range(8)]
        assert helper == [[f"h{i}r{q}" for q in range(3)] for i in range(8)]


def test_helper_channels_share_the_default_namespace_and_abort():
    """helper-thread store clients are clones of the default store, so their keys
    and the abort key live in the default store's namespace; every channel instance has its own key
    prefix (a later channel of the same name never reads an earlier one's leftovers)."""
    res = _run(3, "clone")
    for r in range(3):
        first, second, tail = res[r]
        assert first == ["a0", "a1", "a2"] and second == ["b0", "b1", "b2"]
    assert res[1][2] == "aborted"
    for r in (0, 2):
        dt, msg = res[r][2].split("|", 1)
        assert "job aborted by a peer: rank 1 failed in xgmi setup" in msg and float(dt) < 20.0
