"""Per-phase device time of a --profile window from a rocprofv3 --marker-trace --kernel-trace run.

usage: python tools/marker_summary.py DIR   (DIR holds run_marker_api_trace.csv + run_kernel_trace.csv)

Engine.profile_steps wraps every phase of a training step in a roctx range and drains the streams
before the range closes, so every kernel of a phase starts and ends inside it.  For each range name:
calls, mean host-side range length (launch + drain), mean summed device time of the kernels that
ran inside, and which kernels those were.
"""
import collections
import csv
import glob
import sys


def main(d: str) -> None:
    mk = glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True)[0]
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    ranges = [(r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mk))]
    kern = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mnist::", ""))
                  for r in csv.DictReader(open(kt)))
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, collections.Counter()])
    for name, t0, t1 in ranges:
        a = agg[name]
        a[0] += 1
        a[1] += (t1 - t0) / 1e3
        for k0, k1, kn in kern:
            if k0 >= t0 and k1 <= t1:
                a[2] += (k1 - k0) / 1e3
                a[3][kn] += 1
    print("| range | calls | host range us (launch + drain) | device kernel us | kernels per call |")
    print("|---|---|---|---|---|")
    for name, (n, host, dev, ks) in sorted(agg.items(), key=lambda kv: -kv[1][2] / max(1, kv[1][0])):
        kinds = ", ".join(f"{k} x{c / n:g}" for k, c in ks.most_common(6))
        print(f"| {name} | {n} | {host / n:.1f} | {dev / n:.2f} | {kinds} |")


if __name__ == "__main__":
    main(sys.argv[1])
