"""Per-kernel roofline table from a rocprofv3 --kernel-trace --stats dir + tools/pmc.sh passes.

usage: python tools/roofline.py --stats DIR --pmc DIR1 [DIR2 ...] --batch B [--md]

Per kernel: average duration, analytic FLOPs at batch B (SURVEY §2.4 GEMM views), HBM bytes
(FETCH_SIZE + WRITE_SIZE, KB per dispatch), achieved TFLOP/s and TB/s, raw MFMA-busy / SQ-busy
cycles and LDS bank-conflict cycles per dispatch (summed over the chip's counter instances).
Peaks priced: 2.5 PFLOP/s dense bf16, 8 TB/s HBM3E.
"""
import argparse
import collections
import csv
import glob

PEAK_TF, PEAK_TBS = 2500.0, 8.0


def flops(name: str, B: int) -> float:
    n = name
    if n.startswith("trunk_fwd"):
        return (2 * 676 * 32 * 9 + 2 * 576 * 64 * 288) * B
    if n.startswith("fc1_fwd"):
        return 2 * 9216 * 128 * B
    if n.startswith("fc_bwd"):
        return 4 * 9216 * 128 * B + 4 * 128 * 10 * B
    if n.startswith("conv2_wgrad"):
        return 2 * 64 * 288 * 576 * B
    if n.startswith("conv2_dgrad"):
        return 2 * 676 * 32 * 576 * B + 2 * 32 * 9 * 676 * B
    if n.startswith("head_train"):
        return 3 * 2 * 128 * 10 * B
    return 0.0


def short(k: str) -> str:
    return k.split("(")[0].replace("void ", "").replace("mnist::", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--pmc", nargs="+", default=[])
    ap.add_argument("--batch", type=int, required=True)
    a = ap.parse_args()
    dur, calls = {}, {}
    for f in glob.glob(f"{a.stats}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mnist::" not in r["Name"]:
                continue
            k = short(r["Name"])
            dur[k], calls[k] = float(r["AverageNs"]) / 1000.0, int(r["Calls"])
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.pmc:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "mnist::" not in r["Kernel_Name"]:
                    continue
                pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in pmc.items()}
    print(f"| kernel (B={a.batch}) | calls | us | GFLOP | TFLOP/s | % bf16 peak | HBM KB | TB/s | % HBM peak "
          f"| SQ_VALU_MFMA_BUSY_CYCLES | SQ_BUSY_CYCLES | LDS bank-conflict cyc |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    tot = 0.0
    for k in sorted(dur, key=lambda k: -dur[k] * (calls[k] > 10)):
        if calls[k] < 10:
            continue
        us = dur[k]
        tot += us
        fl = flops(k, a.batch)
        p = avg.get(k, {})
        kb = p.get("FETCH_SIZE", float("nan")) + p.get("WRITE_SIZE", float("nan"))
        tf = fl / us / 1e6 if fl else 0.0
        tbs = kb * 1024 / us / 1e6
        busy = p.get("SQ_BUSY_CYCLES")
        mf = p.get("SQ_VALU_MFMA_BUSY_CYCLES")
        lds = p.get("SQ_LDS_BANK_CONFLICT")
        f0 = lambda v: "-" if v is None else f"{v:.0f}"
        print(f"| {k} | {calls[k]} | {us:.2f} | {fl / 1e9:.3f} | {tf:.1f} | {100 * tf / PEAK_TF:.1f} % | {kb:.0f} | "
              f"{tbs:.2f} | {100 * tbs / PEAK_TBS:.1f} % | {f0(mf)} | {f0(busy)} | {f0(lds)} |")
    print(f"\nsum of per-step kernel time: {tot:.2f} us")


if __name__ == "__main__":
    main()
