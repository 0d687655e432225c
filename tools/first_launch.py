#!/usr/bin/env python
"""First-launch probe: device time of each of the first bakes of a process (box200, config 3).

The rocprof trace of bench.py shows the first k_bake of a process at ~242 ms and the later ones at
~126 ms. This separates the candidate causes: with --spin S the GPU runs S seconds of fp32 GEMMs
before the first bake (clocks ramped, nothing of the bake's memory touched); without it the first
bake starts from an idle GPU. Prints one JSON line per run.

  python tools/first_launch.py [--spin 0|2] [--bakes 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd")]

import torch  # noqa: E402
import fmgi  # noqa: E402
from fmgi import scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", type=float, default=0.0)
    ap.add_argument("--bakes", type=int, default=3)
    args = ap.parse_args()

    sc = scene.box_scene(200)
    ctx = fmgi.Context(0)
    ctx.set_scene(sc)
    ctypes.CDLL(None).srand(1)
    items = ctx.plan(172_413_793)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    lm = torch.zeros((sc.num_texels, 4), dtype=torch.int64, device=dev)
    if args.spin > 0:
        a = torch.randn(4096, 4096, device=dev)
        t0 = time.time()
        while time.time() - t0 < args.spin:
            for _ in range(20):
                a = torch.tanh(a @ a * 1e-3)
            torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.timing()
    out = []
    for _ in range(args.bakes):
        lm.zero_()
        t0 = time.perf_counter()
        ctx.bake_items(0, items, lm.data_ptr(), fmgi.KERNEL_AUTO, stream.cuda_stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        t = ctx.timing()
        out.append({"wall_ms": round(wall, 2), **{k: (round(v, 2) if isinstance(v, float) else v) for k, v in t.items()}})
    print(json.dumps({"spin_s": args.spin, "bakes": out}))
    ctx.close()


if __name__ == "__main__":
    main()
