"""One line per bench.py log: step time, the reference timer (``Total cost time`` of the
mnist_ddp.py child job), its startup phases and the prewarm thread's sub-steps.

    python tools/bench_exact_summary.py gpurun_out/bench_exact_*.log
"""
import json
import sys


def main(paths):
    for f in paths:
        js = [ln for ln in open(f) if ln.startswith("{")]
        if not js:
            print(f"{f}: no JSON line")
            continue
        d = json.loads(js[-1])
        r = d.get("reference_script") or {}
        info = r.get("setup_info") or {}
        print(f"{f}: {1000 * d['ms_per_step']:.2f} us/step, total_cost_time_s {r.get('total_cost_time_s')}, "
              f"setup_total_s {r.get('setup_total_s')}")
        print(f"  phases {json.dumps(r.get('setup_phases_s'))}")
        print(f"  prewarm {json.dumps(info.get('prewarm_steps_s'))}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
