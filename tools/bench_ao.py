#!/usr/bin/env python
"""Ambient-occlusion backend measurement (not the BASELINE metric).

Times fmgi_ambient_occlusion on a scene: the whole call (BSP build on the host, uploads, the k_ao
kernel, download) and, with --kernel-trace under rocprofv3, the kernel alone. Unit of work = one AO
ray (a BSP query): level-0 texels x 481 directions. The CPU baseline is the oracle restatement
(oracle/ao_oracle.c, OpenMP) on the same scene, checked bit-identical to the GPU output here.

  python tools/bench_ao.py [--scene example|box200|box2000] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="example", choices=["example", "box200", "box2000", "box8"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import fmgi
    from fmgi import scene

    sc = (scene.load_geometry(os.path.join(REPO, "tests", "golden", "example_geometry.bin"), "example")
          if a.scene == "example" else scene.box_scene(int(a.scene[3:])))
    texels = int(sum(int(w["lm"][1]) * int(w["lm"][2]) for w in sc.walls))
    rays = texels * len(fmgi.geosphere(4))
    out = fmgi.ambient_occlusion(sc)  # warm-up (code object load, first allocations)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = fmgi.ambient_occlusion(sc)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    res = {"metric": "ambient-occlusion rays/s (whole fmgi_ambient_occlusion call)", "value": rays / t,
           "unit": "rays/s", "scene": a.scene, "walls": int(len(sc.walls)), "texels_level0": texels,
           "rays": rays, "call_s": t, "n_gpus": 1}
    if not a.no_cpu_baseline:
        import fm_oracle as O

        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        t0 = time.perf_counter()
        ref = O.ambient_occlusion(sc, nthreads=threads)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": rays / dt, "unit": "rays/s", "cores": threads, "kind": "port",
                               "sample": f"oracle/ao_oracle.c on the full scene, {dt:.2f} s"}
        res["bitwise_equal_to_oracle"] = bool(np.array_equal(out.view(np.uint32), ref.view(np.uint32)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
