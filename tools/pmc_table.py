#!/usr/bin/env python
"""Per-dispatch means of every rocprofv3 --pmc counter of a gpu_session.sh session, per kernel.

  python tools/pmc_table.py gpurun_out/r3s1 [--out profiles/r03/s1/pmc_table.json] [--kernels k_bake,k_tile]

Reads every <session>/<pass>/run_counter_collection.csv (one pass per directory), groups rows by
kernel (the name up to its template arguments) and counter, and writes the mean over the dispatches of
that kernel in that pass. Values are as rocprofv3 reports them: SQ_*CYCLES / SQ_WAIT_* / SQ_ACTIVE_* in
quad-cycles, GRBM_GUI_ACTIVE summed over the 8 XCDs, FETCH_SIZE / WRITE_SIZE in KiB (uncorrected)."""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    """kernel name without its argument list and template arguments ("void (anonymous namespace)::k_bake<...>(...)"
    -> "k_bake")"""
    n = name.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("<")[0].split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("--out")
    ap.add_argument("--kernels", default="k_bake,k_tile_runs,k_slice_sort")
    a = ap.parse_args()
    want = [k for k in a.kernels.split(",") if k]
    table = collections.defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(a.session, "*", "**", "*counter_collection.csv"), recursive=True)):
        pas = os.path.relpath(p, a.session).split(os.sep)[0]
        tot = collections.defaultdict(float)
        ids = collections.defaultdict(set)
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            if want and not any(w in k for w in want):
                continue
            key = (k, r["Counter_Name"])
            tot[key] += float(r["Counter_Value"])
            ids[key].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        for (k, c), v in tot.items():
            table[k][c] = {"per_dispatch": v / max(len(ids[(k, c)]), 1), "dispatches": len(ids[(k, c)]), "pass": pas}
    out = {"session": a.session, "kernels": table}
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)
    for k, cs in table.items():
        print(k)
        for c, d in sorted(cs.items()):
            print(f"   {c:40s} {d['per_dispatch']:.4e}  ({d['dispatches']} dispatches, {d['pass']})")


if __name__ == "__main__":
    main()
