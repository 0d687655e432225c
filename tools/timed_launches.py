#!/usr/bin/env python
"""Per-dispatch durations of k_bake and k_bucket_fold from a rocprofv3 --kernel-trace CSV of
`bench.py --steps K --warmup W`, and their mean over the timed (non-warm-up) dispatches.

  python tools/timed_launches.py <session>/prof/run_kernel_trace.csv <out.json> [--warmup 1]"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rec = {"source": f"{a.trace} (rocprofv3 --kernel-trace of python bench.py; the first {a.warmup} "
                     "dispatch(es) of each kernel are the warm-up steps)"}
    for k in ("k_bake", "k_bucket_fold"):
        sel = [r for r in rows if k in r["Kernel_Name"]]
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
        # a bake launch of the launch-tail pair is two dispatches of two instances, back to back: one figure
        # per launch (bench.py's HIP events bracket the pair)
        n = len({r["Kernel_Name"] for r in sel}) or 1
        if n > 1:
            rec[f"{k}_instances"] = sorted({r["Kernel_Name"] for r in sel}, key=lambda x: [r["Kernel_Name"] for r in sel].index(x))
            ms = [sum(ms[i:i + n]) for i in range(0, len(ms) - n + 1, n)]
        rec[f"{k}_ms_per_dispatch"] = ms
        timed = ms[a.warmup:]
        rec[f"{k}_timed_mean_ms"] = sum(timed) / len(timed) if timed else None
    rec["note"] = "the bench's HIP-event kernel_ms averages the timed steps"
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
