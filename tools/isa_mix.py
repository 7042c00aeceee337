"""Static instruction mix of each kernel in a hipcc --save-temps .s file, with loop bodies marked.

usage: python tools/isa_mix.py file.s [kernel_substr]
"""
import collections
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", lines[i])
        if m and want in m.group(1):
            name = m.group(1)
            j = i + 1
            body = []
            while j < len(lines) and "s_endpgm" not in lines[j]:
                body.append(lines[j])
                j += 1
            labels = {}
            for k, ln in enumerate(body):
                lm = re.match(r"^(\.LBB\S+):", ln)
                if lm:
                    labels[lm.group(1)] = k
            loops = []
            for k, ln in enumerate(body):
                bm = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", ln)
                if bm:
                    tgt = bm.group(1) or bm.group(2)
                    if tgt in labels and labels[tgt] < k:
                        loops.append((labels[tgt], k))
            cat = collections.Counter()
            for ln in body:
                t = ln.strip().split(" ")[0].split("\t")[0]
                if not t or t.startswith((".", ";")) or t.endswith(":"):
                    continue
                key = ("mfma" if "mfma" in t else "valu" if t.startswith("v_") else "salu" if t.startswith("s_")
                       and not t.startswith(("s_waitcnt", "s_barrier", "s_load", "s_buffer")) else
                       "smem" if t.startswith(("s_load", "s_buffer")) else "lds" if t.startswith("ds_") else
                       "vmem" if t.startswith(("global_", "buffer_", "flat_")) else "sync" if t.startswith(
                           ("s_waitcnt", "s_barrier")) else "other")
                cat[key] += 1
            print(name[:70], dict(cat), "loops:", [(a, b, b - a) for a, b in loops])
            i = j
        i += 1


if __name__ == "__main__":
    main()
