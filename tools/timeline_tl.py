"""Unperturbed per-queue timeline of the training step from in-kernel timestamps.

    python -m pytorch_mnist_ddp_amd._build --timeline        # once: the _C_tl debug extension
    python tools/timeline_tl.py [--batch 200] [--steps 20] [--graph-steps 25] [--out profiles/.../timeline.md]

rocprofv3 intercepts every dispatch and stretches the overlapped B = 200 step from ~68 to ~412 us,
so the overlap of the comm-stream work (the fc Adadelta step, conv2's slab reduce + update) with
the conv backward cannot be read from a kernel trace.  Here every wave of every kernel records its
start and end (s_memrealtime, the device-wide 100 MHz clock) into a device ring
(csrc/include/timeline.h, compiled in only with -DMNIST_TIMELINE); this script trains the bench
workload (single GPU, OVERLAP schedule, captured chunks replayed exactly as bench.py does), clusters
the wave records into launches, assigns them to steps by the trunk_fwd launches, and prints:

* per kernel: mean start / end offset inside the step and mean duration (stream, us);
* the step period (trunk_fwd start to start) next to the period of the SAME command with the
  product build (bench-style host timing; the debug build adds one atomic + store per wave);
* overlap checks: the comm-stream fc update and conv2 update run inside the conv backward window.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["trunk_fwd", "fc1_fwd", "head_train", "fc_bwd", "conv2_wgrad", "conv2_dgrad", "ada_fc", "ada_conv",
         "ada_all", "reduce+update(all)", "conv2 reduce+update", "conv1 reduce+update", "stream_wait",
         "stream_signal", "gather_rows", "xgmi_fc_fused", "xgmi_conv1_fused", "xgmi_conv2_fused", "conv_grad_reduce",
         "xgmi_twoshot", "xgmi_oneshot", "c1_prereduce"]
COMM = {"ada_fc", "conv2 reduce+update", "stream_wait", "stream_signal", "xgmi_fc_fused", "xgmi_conv2_fused"}


def clusters(recs):
    """Wave records [(kid, t0, t1)] -> per kid a list of launches (start, end, waves, wave durations,
    wave start offsets)."""
    by = {}
    for kid, t0, t1 in recs:
        by.setdefault(kid, []).append((t0, t1))
    out = {}
    for kid, v in by.items():
        v.sort()
        cur = None
        res = []
        for t0, t1 in v:
            if cur is None or t0 > cur[1]:
                if cur is not None:
                    res.append(cur)
                cur = [t0, t1, 1, [], []]
            else:
                cur[1] = max(cur[1], t1)
                cur[2] += 1
            cur[3].append(t1 - t0)                       # wave durations
            cur[4].append(t0 - cur[0])                   # wave start offsets in the launch
        res.append(cur)
        out[kid] = res
    return out


def measure(args):
    os.environ["MNIST_AMD_TIMELINE"] = "1"
    import torch
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.data.samplers import DistributedIndexStream
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.models.net import Net
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load()
    assert C.TIMELINE, "the timeline build was not loaded"
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    B = args.batch
    train = load_mnist(train=True, synthetic_data=True, verbose=False)
    ms = ModelState(Net(), dev, lr=1.0)
    total = args.warmup + args.steps
    sampler = DistributedIndexStream(len(train), 1, 0, shuffle=True, seed=0)
    parts, ep = [], 1
    while sum(p.numel() for p in parts) < total * B:
        sampler.set_epoch(ep)
        idx = sampler.epoch_indices()
        parts.append(idx[: (idx.numel() // B) * B])
        ep += 1
    stream = torch.cat(parts)[: total * B]
    comm, kw = None, {}
    if args.sched != "overlap":
        # world-1 DDP production schedule: a one-rank process group (its store carries the RCCL uid)
        # and the selected transport attached, exactly as bench.py --force-comm under torchrun
        import socket
        import torch.distributed as dist
        from pytorch_mnist_ddp_amd.parallel.distributed import create_rccl_comm
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("gloo", init_method="env://", world_size=1, rank=0)
        if args.sched == "rccl":
            comm = create_rccl_comm(1, 0, 0)
        kw = dict(comm=comm, allreduce=args.sched)
    hooks = dict(h.split("=", 1) for h in args.hook)
    tr = FusedTrainer(ms, train, None, B, 1000, num_samples=max(total * B, 60000), seed=1,
                      graph_steps=args.graph_steps, hooks=hooks, **kw)
    tr.start_stream(stream, gather=True)
    tr.precapture(args.warmup)
    tr.precapture(args.steps)
    tr.warm_graphs(args.steps)                           # as bench.py: every timed graph has run once
    tr.run_steps(args.warmup)
    tr.synchronize()
    C.timeline_dump()                                    # discard the warmup's records
    tr.run_steps(args.steps)
    tr.synchronize()
    raw = C.timeline_dump()
    import numpy as np
    a = np.frombuffer(raw, dtype=np.uint64).reshape(-1, 3)
    recs = [(int(k), int(t0), int(t1)) for k, t0, t1 in a]
    return recs, tr.engine.schedule


def analyse(recs, steps):
    cl = clusters(recs)
    trunk = sorted(cl.get(0, []))
    if len(trunk) < 2:
        raise SystemExit(f"expected {steps} trunk_fwd launches, got {len(trunk)}")
    starts = [c[0] for c in trunk]
    period = (starts[-1] - starts[0]) / (len(starts) - 1) / 100.0      # ticks of 10 ns -> us
    rows, wstat = {}, {}
    for kid, launches in cl.items():
        for s, e, w, wd, ws in launches:
            i = max(j for j in range(len(starts)) if starts[j] <= s) if s >= starts[0] else -1
            if i < 1:                                    # skip the first step (ramp from idle)
                continue
            rows.setdefault(kid, []).append(((s - starts[i]) / 100.0, (e - starts[i]) / 100.0, w))
            d = wstat.setdefault(kid, ([], []))
            d[0].extend(wd)
            d[1].append(sorted(ws)[int(0.9 * (len(ws) - 1))])
    table = []
    for kid, v in sorted(rows.items(), key=lambda kv: sum(x[0] for x in kv[1]) / len(kv[1])):
        n = len(v)
        st = sum(x[0] for x in v) / n
        en = sum(x[1] for x in v) / n
        wd, ws = wstat[kid]
        wd = sorted(wd)
        table.append({"kernel": NAMES[kid] if kid < len(NAMES) else str(kid), "launches": n,
                      "start_us": round(st, 2), "end_us": round(en, 2), "dur_us": round(en - st, 2),
                      "waves": round(sum(x[2] for x in v) / n, 1),
                      "wave_p50_us": round(wd[len(wd) // 2] / 100.0, 2),
                      "wave_p90_us": round(wd[int(0.9 * (len(wd) - 1))] / 100.0, 2),
                      "start_p90_us": round(sum(ws) / len(ws) / 100.0, 2)})
    span = {"period_us": round(period, 2), "steps": len(starts),
            "step_periods_us": [round((b - a) / 100.0, 1) for a, b in zip(starts, starts[1:])]}
    ends = [c[1] for launches in cl.values() for c in launches]
    span["window_us"] = round((max(ends) - starts[0]) / 100.0, 1)       # first trunk start -> last end
    # the first replayed step (from an idle GPU, right after the graph launches): every launch that
    # starts before the second trunk_fwd, relative to the first trunk_fwd start
    first = []
    for kid, launches in cl.items():
        for s, e, w, _, _ in launches:
            if s < starts[1]:
                first.append((round((s - starts[0]) / 100.0, 2), round((e - starts[0]) / 100.0, 2),
                              NAMES[kid] if kid < len(NAMES) else str(kid)))
    span["first_step"] = sorted(first)
    return table, span


def overlap_checks(table):
    t = {r["kernel"]: r for r in table}
    out = []
    fc = "ada_fc" if "ada_fc" in t else "xgmi_fc_fused"
    c2 = "conv2 reduce+update" if "conv2 reduce+update" in t else "xgmi_conv2_fused"
    if fc in t and "conv2_wgrad" in t and "conv2_dgrad" in t:
        r = t[fc]
        out.append(f"fc update {fc} (comm stream) {r['start_us']:.1f}-{r['end_us']:.1f} us inside the conv backward "
                   f"{t['conv2_wgrad']['start_us']:.1f}-{t['conv2_dgrad']['end_us']:.1f} us: "
                   f"{t['conv2_wgrad']['start_us'] <= r['start_us'] and r['end_us'] <= t['conv2_dgrad']['end_us']}")
    if c2 in t and "conv2_dgrad" in t:
        r = t[c2]
        out.append(f"conv2 part {c2} (comm stream) {r['start_us']:.1f}-{r['end_us']:.1f} us under conv2_dgrad "
                   f"{t['conv2_dgrad']['start_us']:.1f}-{t['conv2_dgrad']['end_us']:.1f} us: "
                   f"{r['start_us'] >= t['conv2_dgrad']['start_us'] and r['end_us'] <= t['conv2_dgrad']['end_us'] + 1.0}")
    return out


def product_period(args) -> float | None:
    """The same command's period with the product build (bench.py, host-timed)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--batch-size", str(args.batch), "--graph-steps", str(args.graph_steps), "--no-full-run"]
    for h in args.hook:
        cmd += ["--hook", h]
    if args.sched != "overlap":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes",
               "1", "--nproc-per-node", "1"] + cmd[1:] + ["--force-comm", "--allreduce", args.sched]
    env = {k: v for k, v in os.environ.items() if k != "MNIST_AMD_TIMELINE"}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    for ln in r.stdout.splitlines():
        if ln.startswith("{"):
            return 1000.0 * json.loads(ln)["ms_per_step"]
    return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=200)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph-steps", type=int, default=25)
    ap.add_argument("--out", default=None)
    ap.add_argument("--sched", choices=["overlap", "xgmi", "rccl"], default="overlap",
                    help="overlap: single GPU; xgmi / rccl: the world-1 DDP production schedule")
    ap.add_argument("--no-product", action="store_true")
    ap.add_argument("--hook", action="append", default=[], metavar="NAME=VALUE",
                    help="engine variant (FusedTrainer.HOOKS), for the timeline and the product run")
    args = ap.parse_args()
    recs, sched = measure(args)
    table, span = analyse(recs, args.steps)
    prod = None if args.no_product else product_period(args)
    lines = [f"# In-kernel timeline, B = {args.batch}, {args.steps} replayed steps (graph chunks of "
             f"{args.graph_steps}), schedule {['serial', 'overlap', 'rccl', 'xgmi'][sched]}", "",
             f"period (trunk_fwd start to start, steps 2..{span['steps']}): {span['period_us']} us/step "
             f"(timeline build); product build, same command: {round(prod, 2) if prod else 'n/a'} us/step", "",
             f"device window (first trunk_fwd start to last kernel end): {span['window_us']} us for "
             f"{span['steps']} steps; step periods: {span['step_periods_us']}", "",
             "| kernel | stream | launches | start us | end us | duration us | waves | wave p50 / p90 us | "
             "90 % of waves started by us |", "|---|---|---|---|---|---|---|---|---|"]
    for r in table:
        lines.append(f"| {r['kernel']} | {'comm' if r['kernel'] in COMM else 'compute'} | {r['launches']} | "
                     f"{r['start_us']} | {r['end_us']} | {r['dur_us']} | {r['waves']} | "
                     f"{r['wave_p50_us']} / {r['wave_p90_us']} | {r['start_p90_us']} |")
    lines += ["", "Offsets are relative to the step's trunk_fwd start (first step excluded); every wave records"
              " its start / end with s_memrealtime (10 ns), a launch = the union of its waves.", ""]
    lines += ["First replayed step (launches starting before the second trunk_fwd; us from the first trunk_fwd start):",
              "", "| kernel | start us | end us |", "|---|---|---|"]
    lines += [f"| {n} | {a} | {b} |" for a, b, n in span["first_step"]]
    lines += [""]
    lines += ["- " + c for c in overlap_checks(table)]
    text = "\n".join(lines) + "\n"
    print(text)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
