#!/usr/bin/env python
"""The launch the planner chooses for a configuration: one bake of each (scene, spa) on cuda:0, printing the
experiment build's launch line (FMGI_SHOW_LAUNCH: kernel instance, accumulation, block, grid, LDS, staged
table offsets) and the k_bake instance the bake ran (fmgi_last_bake_kernel).

  FMGI_LIB=exp FMGI_SHOW_LAUNCH=1 python tools/show_launch.py box200 example:65000 example box2000 apartment30
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd"), REPO]


def main():
    import torch

    import bench
    import fmgi

    for arg in sys.argv[1:] or ["box200"]:
        name, _, spa = arg.partition(":")
        cfg = bench.CONFIGS[name]
        sc = bench.load_scene(cfg["scene"])
        ctx = fmgi.Context(0)
        ctx.set_scene(sc)
        items = ctx.plan(int(spa) if spa else cfg["spa"])
        lm = torch.zeros((sc.num_texels, 4), dtype=torch.int64, device="cuda")
        s = torch.cuda.Stream()
        print(f"== {arg}: {items} items", flush=True)
        ctx.bake_items(0, items, lm.data_ptr(), fmgi.KERNEL_AUTO, s.cuda_stream)
        s.synchronize()
        print(f"   {ctx.last_bake_kernel}", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
