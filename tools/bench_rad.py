#!/usr/bin/env python
"""Radiosity backend measurement (not the BASELINE metric).

Times fmgi_radiosity on a scene: the whole call (host setup, uploads, the device rand() replay, the
candidate lists and ray casts, 7 bounces, download) and its device phases (fmgi_radiosity_stats, HIP
events). Unit of work = one form-factor ray (10000 per level-0 wall texel), as SURVEY §6 quotes the
reference (3.7e6 gather-rays/s on one core). The CPU baseline is the oracle restatement
(oracle/rad_oracle.c, OpenMP) on --cpu-scene (default: the same scene when it is small), checked
bit-identical to the GPU there. With a reference fixture for the scene (tests/golden/rad_ref.json)
the GPU result is checked against it too.

  python tools/bench_rad.py [--scene example|box200|box200_t2_lit|box2000] [--reps 3]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402


def load_scene(name):
    from fmgi import scene

    if name == "example":
        return scene.load_geometry(os.path.join(REPO, "tests", "golden", "example_geometry.bin"), "example")
    if name.endswith("_t2_lit"):
        return scene.box_scene(int(name[3:].split("_")[0]), tile_size=2.0, with_light=True)
    return scene.box_scene(int(name[3:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="example")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--cpu-scene", default="box200_t2_lit")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import fmgi

    libc = ctypes.CDLL(None)
    libc.srand.argtypes = [ctypes.c_uint]
    sc = load_scene(a.scene)
    fixtures = json.load(open(os.path.join(REPO, "tests", "golden", "rad_ref.json")))
    fx = fixtures.get(a.scene)
    seed = fx["seed"] if fx else 1
    libc.srand(seed)
    out = fmgi.radiosity(sc)  # warm-up (code objects, first allocations) + fixture check
    res = {"metric": "radiosity form-factor rays/s (whole fmgi_radiosity call)", "scene": a.scene,
           "walls": int(len(sc.walls)), "n_gpus": 1}
    if fx:
        res["equal_to_reference_fixture"] = hashlib.sha256(out.tobytes()).hexdigest() == fx["sha256_f32"]
        res["next_rand_ok"] = libc.rand() == fx["next_rand"]
    ts, st = [], None
    for _ in range(a.reps):
        libc.srand(seed)
        t0 = time.perf_counter()
        fmgi.radiosity(sc)
        ts.append(time.perf_counter() - t0)
        st = fmgi.radiosity_stats()
    t = min(ts)
    res.update({"value": st["rays"] / t, "unit": "rays/s", "call_s": t, "stats": st,
                "device_rays_per_s": st["rays"] / ((st["rand_ms"] + st["rays_ms"]) / 1e3),
                "bounce_ms_per_iteration": st["bounce_ms"] / 7})
    if not a.no_cpu_baseline:
        import fm_oracle as O

        cs = load_scene(a.cpu_scene)
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        libc.srand(1)
        t0 = time.perf_counter()
        ref = O.radiosity(cs, nthreads=threads)
        dt = time.perf_counter() - t0
        libc.srand(1)
        got = fmgi.radiosity(cs)
        rays = fmgi.radiosity_stats()["rays"]
        res["cpu_baseline"] = {"value": rays / dt, "unit": "rays/s", "cores": threads, "kind": "port",
                               "sample": f"oracle/rad_oracle.c on {a.cpu_scene} ({rays} rays), {dt:.2f} s"}
        res["cpu_scene_bitwise_equal"] = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
