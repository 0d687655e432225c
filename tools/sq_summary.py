#!/usr/bin/env python
"""Summarise a gpu_session.sh `sq` step (two rocprofv3 --pmc passes of SQ counters) into per-dispatch
instruction counts of the bake kernel, recorded in profiles/sq_issue.json under the bench config name
(bench.py reads SQ_INSTS_VALU per launch for its issue roofline).

  python tools/sq_summary.py gpurun_out/s47 box200 [--out profiles/sq_issue.json]

The SQ_*_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* counters are in units of 4 cycles on gfx9 (quad-cycles);
they are kept as reported. SQ_INSTS_* are wave-instruction counts."""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("config")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "sq_issue.json"))
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    ids = collections.defaultdict(set)
    kernel = None
    for step in ("sq1", "sq2"):
        for p in glob.glob(os.path.join(a.session, step, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if "k_bake" not in r["Kernel_Name"]:
                    continue
                kernel = r["Kernel_Name"]
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                ids[r["Counter_Name"]].add(r["Dispatch_Id"])
    if not tot:
        raise SystemExit("no k_bake dispatch in the SQ files")
    per = {k: tot[k] / max(len(ids[k]), 1) for k in sorted(tot)}
    data = json.load(open(a.out)) if os.path.exists(a.out) else {}
    data[a.config] = {
        "kernel": kernel,
        "source": f"{a.session}: rocprofv3 --pmc SQ counters in two passes (tools/gpu_session.sh step sq), per dispatch",
        "per_launch": per,
    }
    with open(a.out, "w") as fh:
        json.dump(data, fh, indent=1)
    for k, v in per.items():
        print(f"{k:28s} {v:.4e}")


if __name__ == "__main__":
    main()
