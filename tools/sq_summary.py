#!/usr/bin/env python
"""Summarise the counter passes of one gpu_session.sh session (steps sq, sq3, grbm, tcp, clock) into
per-dispatch counters of the bake kernel, recorded in profiles/sq_issue.json under the bench config name.
bench.py derives its `roofline.issue` block from this file (clock, SIMD cycles, wave-cycle split,
vector-memory path busy fractions).

  python tools/sq_summary.py profiles/r03/final box200 [--out profiles/sq_issue.json]

<session>/<pass>/**/*counter_collection.csv are rocprofv3 --pmc outputs (one pass per directory);
<session>/bench_clock.json, if present, is the FMGI_CLOCK_STAMP build's bench line (in-kernel
s_memtime / s_memrealtime clock). SQ_*_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* are kept as reported (units of 4
cycles on gfx9; only their ratios are used); SQ_INSTS_* are wave-instruction counts; GRBM_GUI_ACTIVE is
summed over the 8 XCDs; TA_/TD_/TCP_ *_sum are summed over the 256 CUs."""
import argparse
import collections
import csv
import glob
import json
import os

PASSES = ("sq1", "sq2", "sq3", "grbm", "tcp")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("config")
    ap.add_argument("--kernel", default="k_bake")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "sq_issue.json"))
    a = ap.parse_args()
    # per (instance, counter): the sum over its dispatches and the dispatch ids. A bake launch of the
    # launch-tail pair runs two k_bake instances: its per-launch figure is the sum of their per-dispatch means
    tot = collections.defaultdict(float)
    ids = collections.defaultdict(set)
    first = {}
    src = {}
    for step in PASSES:
        for p in glob.glob(os.path.join(a.session, step, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                k = r["Kernel_Name"]
                if a.kernel not in k:
                    continue
                c = r["Counter_Name"]
                if c in src and src[c] != step:
                    continue  # a counter collected in several passes: keep the first pass's value
                src[c] = step
                tot[k, c] += float(r["Counter_Value"])
                d = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
                ids[k, c].add(d)
                first[k] = min(first.get(k, float("inf")), float(d or 0))
    if not tot:
        raise SystemExit(f"no {a.kernel} dispatch in the counter files of {a.session}")
    names = sorted(first, key=first.get)  # launch order: the saving instance before the resuming one
    per = collections.defaultdict(float)
    for (k, c), v in tot.items():
        per[c] += v / max(len(ids[k, c]), 1)
    per = dict(sorted(per.items()))
    rec = {
        "kernel": " + ".join(names),
        "source": f"{a.session}/{{{','.join(PASSES)}}}: rocprofv3 --pmc passes (tools/gpu_session.sh steps sq, sq3, "
                  "grbm, tcp), per dispatch",
        "pass_of": src,
        "per_launch": per,
    }
    clk = os.path.join(a.session, "bench_clock.json")
    if os.path.exists(clk):
        d = json.load(open(clk))
        rec["clock_ghz"] = d["in_kernel_clock_ghz"]
        rec["clock_source"] = f"{clk}: FMGI_CLOCK_STAMP build, s_memtime / s_memrealtime (100 MHz) per wave"
    if per.get("GRBM_GUI_ACTIVE"):
        rec["grbm_cycles_per_xcd"] = per["GRBM_GUI_ACTIVE"] / 8.0
    data = json.load(open(a.out)) if os.path.exists(a.out) else {}
    data[a.config] = rec
    with open(a.out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    for k, v in per.items():
        print(f"{k:40s} {v:.4e}  ({src[k]})")


if __name__ == "__main__":
    main()
