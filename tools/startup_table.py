"""Per-phase startup table of the reference script at N ranks (the part of ``Total cost time`` before
the first epoch).

    python tools/startup_table.py --world 2 4 [--reps 2] [--one-gpu] [--out profiles/.../startup.md]

Runs ``mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --json-log`` under torch.distributed.run
(``--one-gpu``: every rank on GPU 0 - gloo process group + the xGMI kernels, 2 hardware queues per
process, as the one-GPU rehearsals; ``--production``: every rank on GPU 0 but the driver's production
command - default ``nccl`` process group, ``--allreduce auto``, no transport flag - where RCCL cannot
initialise, two ranks sharing a GPU).  Every run generates its synthetic data in-process (native
generator, no cache), so each row is a cold start. and prints, per run, every rank's setup phases (host seconds on
its main thread, in order), their sum (``setup_total_s`` is the max of these over ranks), the xGMI
communicator's sub-steps and the helper-thread timings, plus the script's ``Total cost time``.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(world: int, one_gpu: bool, extra: list[str], production: bool = False) -> tuple[list[dict], float | None, str]:
    jlog = tempfile.NamedTemporaryFile(prefix="startup_", suffix=".jsonl", delete=False).name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes",
           "1", "--nproc-per-node", str(world), os.path.join(ROOT, "mnist_ddp.py"), "--batch-size", "200",
           "--epochs", "20", "--synthetic", "--json-log", jlog] + extra
    env = dict(os.environ, PYTHONPATH=ROOT)
    if one_gpu or production:
        env.update(MNIST_AMD_ONE_GPU="1", GPU_MAX_HW_QUEUES="2")
    if one_gpu and not production:
        cmd += ["--dist-backend", "gloo", "--allreduce", "xgmi"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    if r.returncode != 0:
        raise SystemExit(f"world {world}: rc {r.returncode}\n{r.stderr[-3000:]}")
    times = [float(x) for x in re.findall(r"Total cost time:([0-9.eE+-]+) ms", r.stdout)]
    recs = [json.loads(ln) for ln in open(jlog) if ln.strip()]
    os.unlink(jlog)
    return [x for x in recs if "setup_s" in x], max(times) if times else None, " ".join(cmd[3:])


def critical(setups: list[dict]) -> tuple[float | None, float | None]:
    """(launch skew = last rank's timer start - first rank's, startup critical path = last rank ready -
    last rank's start): the first collective makes every earlier-started rank wait out the skew, which
    the launcher (process start, `import torch`), not the startup, decides."""
    if not all("t_start_unix" in x and "trainer_ready_unix" in x for x in setups):
        return None, None
    t0 = [x["t_start_unix"] for x in setups]
    t1 = [x["trainer_ready_unix"] for x in setups]
    return max(t0) - min(t0), max(t1) - max(t0)


def table(world: int, setups: list[dict], total: float | None) -> list[str]:
    keys = list(dict.fromkeys(k for x in setups for k in x["setup_s"]))
    skew, crit = critical(setups)
    extra = (f"; launch skew {skew:.3f} s, critical path from the last rank's start {crit:.3f} s"
             if skew is not None else "")
    out = [f"### world {world}: Total cost time {total:.3f} s, setup_total_s (max over ranks) "
           f"{max(sum(x['setup_s'].values()) for x in setups):.3f} s{extra}", "",
           "| phase | " + " | ".join(f"rank {i}" for i in range(len(setups))) + " |",
           "|---|" + "---|" * len(setups)]
    for k in keys:
        out.append(f"| {k} | " + " | ".join(f"{x['setup_s'].get(k, 0.0):.3f}" for x in setups) + " |")
    out.append("| **sum** | " + " | ".join(f"**{sum(x['setup_s'].values()):.3f}**" for x in setups) + " |")
    out.append("")
    for i, x in enumerate(setups):
        info = x.get("setup_info") or {}
        out.append(f"- rank {i} helper threads / sub-steps: `{json.dumps(info)}`")
    out.append("")
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--one-gpu", action="store_true")
    ap.add_argument("--production", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("extra", nargs="*")
    args = ap.parse_args()
    lines = ["# Startup inside the reference timer, per phase and rank", ""]
    for w in args.world:
        for rep in range(args.reps):
            setups, total, cmd = run(w, args.one_gpu, args.extra, args.production)
            lines.append(f"`{cmd}` (rep {rep + 1})")
            lines.append("")
            lines += table(w, setups, total)
            print("\n".join(lines[-(len(setups) + 12):]), flush=True)
    text = "\n".join(lines) + "\n"
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
