#!/usr/bin/env python
"""A/B of environment settings that the library reads per call (e.g. FMGI_FOLD_CARRY), in one process:
every setting bakes the same configuration `--reps` times; the first setting's int64 lightmap is the
reference and every other setting must equal it bit for bit. Prints one JSON line per setting with the
mean k_bake and fold times (HIP events, fmgi_set_timing) and whether the lightmap matched.

  python tools/ab_exact.py --config box200 --set "" --set FMGI_FOLD_CARRY=1 --set FMGI_FOLD_CARRY=2
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd"), REPO]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="box200")
    ap.add_argument("--set", action="append", default=[], help="space-separated K=V assignments ('' = defaults)")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import bench
    import fmgi

    cfg = bench.CONFIGS[args.config]
    sc = bench.load_scene(cfg["scene"])
    ctx = fmgi.Context(0)
    ctx.set_scene(sc)
    ctypes.CDLL(None).srand(1)
    items = ctx.plan(cfg["spa"])
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    lm = torch.zeros((sc.num_texels, 4), dtype=torch.int64, device=dev)
    ref = None
    base_env = dict(os.environ)
    ctx.set_timing(True)
    for setting in args.set or [""]:
        os.environ.clear()
        os.environ.update(base_env)
        for kv in setting.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        lm.zero_()  # warm-up bake (first use of this setting's kernels)
        ctx.bake_items(0, items, lm.data_ptr(), fmgi.KERNEL_AUTO, stream.cuda_stream)
        torch.cuda.synchronize()
        ctx.timing()
        same = True
        for _ in range(args.reps):
            lm.zero_()
            ctx.bake_items(0, items, lm.data_ptr(), fmgi.KERNEL_AUTO, stream.cuda_stream)
            torch.cuda.synchronize()
            got = lm.cpu().numpy()
            if ref is None:
                ref = got.copy()
            same = same and bool(np.array_equal(got, ref))
        t = ctx.timing()
        print(json.dumps({"config": args.config, "set": setting, "k_bake_ms": t["bake_ms"] / max(t["bake_launches"], 1),
                          "fold_ms": t["fold_ms"] / args.reps, "bake_launches_per_step": t["bake_launches"] / args.reps,
                          "bit_identical_to_first": same}), flush=True)
        if not same:
            raise SystemExit(f"setting {setting!r}: lightmap differs from the first setting's")
    ctx.close()


if __name__ == "__main__":
    main()
