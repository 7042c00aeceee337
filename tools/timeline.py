"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv.

usage: python tools/timeline.py <kernel_trace.csv> [first_kernel_substr]
Steps are delimited by launches of the first kernel (default trunk_fwd); prints, for the median
step of the last half of the trace, every kernel's start/end offset (us) from step start and its
queue/stream, plus the median step period.
"""
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "trunk_fwd"
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                  r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows))
    starts = [i for i, k in enumerate(ks) if first in k[2]]
    steps = [ks[a:b] for a, b in zip(starts, starts[1:])]
    steps = steps[len(steps) // 2:]
    periods = [s[0][0] - p[0][0] for p, s in zip(steps, steps[1:])]
    if not periods:
        print("not enough steps")
        return
    med = statistics.median(periods)
    print(f"steps analysed: {len(steps)}  median period: {med / 1000:.2f} us")
    sig = {}
    for s in steps:
        key = tuple(k[2] for k in s)
        sig.setdefault(key, []).append(s)
    key = max(sig, key=lambda k: len(sig[k]))
    group = sig[key]
    for j, name in enumerate(key):
        st = statistics.median((s[j][0] - s[0][0]) / 1000 for s in group)
        en = statistics.median((s[j][1] - s[0][0]) / 1000 for s in group)
        print(f"  {name[:48]:48s} q={group[0][j][3]:>3s} start {st:8.2f}  end {en:8.2f}  dur {en - st:7.2f}")


if __name__ == "__main__":
    main()
