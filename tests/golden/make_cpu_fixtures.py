"""Regenerate the CPU-side golden fixtures (run in the build container; outputs are committed).

  glibc_rand_4096.npy   first 4096 values of unseeded glibc rand() -- the reference's per-launch
                        rng_offset source (global_illumination_cl.c:251); lets the GPU box detect a
                        different libc.
  oracle_config1.json   oracle result for BASELINE config 1 (example.png, spa=65,000, WG 256):
                        schedule, counters, sha256 of the int64 fixed-point lightmap, per-wall sums.
                        A regression pin of the oracle itself; the oracle's faithfulness to the
                        reference is pinned separately by ref_items_*.npz (make_ref_fixtures.py).
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "flatmatch-global-illumination_amd")]

import fm_oracle as O  # noqa: E402
from fmgi import scene as S  # noqa: E402


def main():
    libc = ctypes.CDLL(None)
    libc.srand(1)
    vals = np.array([libc.rand() for _ in range(4096)], np.int32)
    np.save(os.path.join(HERE, "glibc_rand_4096.npy"), vals)

    ex = S.load_geometry(os.path.join(HERE, "example_geometry.bin"), "example")
    libc.srand(1)
    L = O.schedule(ex, 65000)
    lm, st = O.bake(ex, L)
    per_wall = []
    for w in ex.walls:
        b, s1, s2 = int(w["lm"][0]), int(w["lm"][1]), int(w["lm"][2])
        per_wall.append([int(x) for x in lm[b : b + s1 * s2].sum(axis=0)])
    out = {
        "config": "example.png, spa=65000, wg=256",
        "launches": L.tolist(),
        "stats": st,
        "lightmap_sha256": hashlib.sha256(np.ascontiguousarray(lm).tobytes()).hexdigest(),
        "per_wall_fx_sums": per_wall,
        "total_fx": [int(x) for x in lm.sum(axis=0)],
    }
    with open(os.path.join(HERE, "oracle_config1.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("ok", st)


if __name__ == "__main__":
    main()
