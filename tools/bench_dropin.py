#!/usr/bin/env python
"""End-to-end time of the drop-in boundary (not the BASELINE metric): what the reference's main.c sees
when it calls performGlobalIlluminationCl (global_illumination_cl.c:275-321) linked against
libflatmatch_gi.so. Each call plans the reference launch schedule (consuming libc rand() once per
launch), bakes, reduces the GPU shards, adds the sums to the caller's texels and copies them back; the
device contexts, scene tables and buffers are cached across calls per geometry (fmgi_dropin_release;
--no-cache frees them after every call, as the reference re-creates its OpenCL context and recompiles
photonmap.cl on every call).

  python tools/bench_dropin.py [--reps 3]

Reports, per BASELINE config on one process: the first call (includes the HIP runtime's start-up and
code-object load) and the best of the following calls, as photons per second of wall time.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402

CASES = [  # (BASELINE config, scene, numSamplesPerArea)
    ("1: example.png, 1e6 photons", "example", 65_000),
    ("2: example.png, 1e8 photons", "example", 6_500_000),
    ("3: box200, 1e9 photons", "box200", 172_413_793),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-cache", action="store_true", help="FMGI_DROPIN_CACHE=0: no device state kept between calls")
    a = ap.parse_args()
    if a.no_cache:
        os.environ["FMGI_DROPIN_CACHE"] = "0"
    os.environ.setdefault("FMGI_QUIET", "1")
    import fmgi
    from fmgi import scene

    libc = ctypes.CDLL(None)
    for desc, name, spa in CASES:
        sc = (scene.load_geometry(os.path.join(REPO, "tests", "golden", f"{name}_geometry.bin"), name)
              if name == "example" else scene.box_scene(200))
        _, items = fmgi.plan_count(sc, spa)
        photons = 100 * items
        ts = []
        for _ in range(1 + a.reps):
            libc.srand(1)
            tex = np.zeros((sc.num_texels, 4), np.float32)
            t0 = time.perf_counter()
            out = fmgi.bake_geometry(sc, spa, tex)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"metric": "drop-in photons/s (wall time of one performGlobalIlluminationCl-equivalent call)",
                          "config": desc, "spa": spa, "photons": photons, "gpus": fmgi.device_count(),
                          "cache": not a.no_cache,
                          "first_call_s": ts[0], "warm_call_s": min(ts[1:]),
                          "warm_photons_per_s": photons / min(ts[1:]),
                          "texel_sum": float(out[:, :3].astype(np.float64).sum())}), flush=True)


if __name__ == "__main__":
    main()
