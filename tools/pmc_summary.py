#!/usr/bin/env python
"""Summarise a gpu_session.sh `pmc` step (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes) into
per-dispatch HBM bytes per kernel, and record the bake kernel's figure in profiles/pmc_traffic.json
under the bench config name (bench.py reads it as roofline.traffic).

  python tools/pmc_summary.py gpurun_out/s17 box200 [--out profiles/pmc_traffic.json]

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) is reported at half the bytes of wide
coalesced streaming reads on gfx950 and is doubled here; WRITE_SIZE (KiB) is taken as is. Both count
Infinity-Cache hits as traffic. Values are per dispatch (the mean over the profiled dispatches)."""
import argparse
import collections
import csv
import json
import os


def per_dispatch(path, counter, order=None):
    """per kernel: the counter's mean over its dispatches (order: each kernel's first dispatch id)"""
    tot = collections.defaultdict(float)
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        d = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
        tot[k] += float(r["Counter_Value"])
        ids[k].add(d)
        if order is not None:
            order[k] = min(order.get(k, float("inf")), float(d or 0))
    return {k: tot[k] / max(len(ids[k]), 1) for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("config")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    order = {}
    fetch = per_dispatch(os.path.join(a.session, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE", order)
    write = per_dispatch(os.path.join(a.session, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = sorted(set(fetch) | set(write))
    table = {}
    for k in kernels:
        f = 2.0 * 1024 * fetch.get(k, 0.0)
        w = 1024 * write.get(k, 0.0)
        table[k] = {"fetch_bytes": f, "write_bytes": w, "hbm_bytes": f + w}
    bake = [k for k in kernels if "k_bake" in k]
    if not bake:
        raise SystemExit("no k_bake dispatch in the PMC files")
    # a bake launch of the launch-tail pair runs two k_bake instances: its figure is their sum, and its
    # name theirs joined in launch order (as fmgi_last_bake_kernel reports it)
    bake.sort(key=lambda k: order.get(k, float("inf")))
    kb = " + ".join(bake)
    per_launch = {f: sum(table[k][f] for k in bake) for f in ("fetch_bytes", "write_bytes", "hbm_bytes")}
    data = json.load(open(a.out)) if os.path.exists(a.out) else {}
    data[a.config] = {
        "kernel": kb,
        "source": f"{a.session}: rocprofv3 --pmc FETCH_SIZE, then a separate --pmc WRITE_SIZE pass "
                  "(tools/gpu_session.sh step pmc), per dispatch",
        "fetch_bytes_per_launch": per_launch["fetch_bytes"],
        "write_bytes_per_launch": per_launch["write_bytes"],
        "hbm_bytes_per_launch": per_launch["hbm_bytes"],
        "all_kernels": table,
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 reports 1/2 of wide streaming reads); "
                "WRITE_SIZE as reported",
    }
    with open(a.out, "w") as fh:
        json.dump(data, fh, indent=1)
    for k in kernels:
        t = table[k]
        print(f"{t['fetch_bytes'] / 1e9:10.3f} GB read {t['write_bytes'] / 1e9:10.3f} GB written  {k[:90]}")


if __name__ == "__main__":
    main()
