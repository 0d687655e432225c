"""How far the reference kernel's DEPLOYED arithmetic moves a whole lightmap (run on the GPU box; the
outputs are committed and checked by tests/test_tolerance.py on the CPU).

The reference builds photonmap.cl with -cl-fast-relaxed-math (global_illumination_cl.c:196). That exact
build faults on the MI355X (finite-math-only drops photonmap.cl:208's INFINITY test; oracle/build_ref.sh),
so the nearest well-defined build, -cl-unsafe-math-optimizations ("relaxed"), stands for it; "strict" is
the oracle's contract (IEEE div/sqrt, no contraction). For each case every work item of a reference
launch range is run alone on a zeroed lightColors buffer (oracle/ref_runner.cpp ref_run_sum: the race-free
sum of the reference's own per-item fp32 lightmaps, exact in int64 units of 2^-25) and compared with the
exact sum the product computes (== the oracle, bit for bit: tests/test_gpu_*.py):

  ref_launch_<case>.npz : items [begin, end) of the schedule (spa, glibc rand() offsets), the oracle's
                          lightmap digest (sha256 of its int64 [numTexels, 3] bytes), and
                          d_strict / d_relaxed = reference sum - oracle sum (int64, units of 2^-25)

  case config1 : example.png, spa 65,000 -- all 11,008 items of BASELINE config 1 (10 launches)
  case box200  : box200, spa 172,413,793 -- launch 0 of BASELINE config 3 (25,600 items, 2.56e6 photons)

  python tests/golden/make_tolerance_fixtures.py [out_dir]    (GPU box; GPU_MAX_HW_QUEUES=16 speeds it up)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "flatmatch-global-illumination_amd")]

import fm_oracle as O  # noqa: E402
from fmgi import scene as S  # noqa: E402


def metrics(ours_fx, ref_fx, counts, level0):
    """max relative difference over level-0 texels with >= 100 deposits (max over the 3 channels) and the
    L1 relative difference over all texels and channels"""
    a = ours_fx.astype(np.float64)
    d = np.abs(ref_fx.astype(np.float64) - a)
    sel = level0 & (counts >= 100)
    rel = (d[sel] / np.maximum(a[sel], 1.0)).max() if sel.any() else 0.0
    return {"max_rel_ge100": float(rel), "l1_rel": float(d.sum() / max(a.sum(), 1.0)),
            "texels_ge100": int(sel.sum()), "texels_differing": int((d.sum(axis=1) > 0).sum())}


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else HERE
    offs = np.load(os.path.join(HERE, "glibc_rand_4096.npy"))
    example = S.load_geometry(os.path.join(HERE, "example_geometry.bin"), "example")
    cases = [("config1", example, 65_000, 0, None), ("box200", S.box_scene(200), 172_413_793, 0, 25_600)]
    summary = {}
    for name, sc, spa, b, e in cases:
        L = O.schedule_with_offsets(sc, spa, offs)
        if e is None:
            e = int(L["item_begin"][-1] + L["count"][-1])
        t0 = time.time()
        ours, _, counts = O.bake(sc, L, b, e, counts=True)
        print(f"{name}: oracle {e - b} items in {time.time() - t0:.1f} s", flush=True)
        res = {"items": [b, e], "spa": spa, "oracle_sha256": hashlib.sha256(ours.tobytes()).hexdigest()}
        arrays = {}
        level0 = sc.level0_mask()
        for variant in ("strict", "relaxed"):
            t0 = time.time()
            ref = O.ref_run_sum(sc, L, b, e, variant)
            print(f"{name}/{variant}: reference {e - b} items in {time.time() - t0:.1f} s", flush=True)
            arrays[f"d_{variant}"] = ref - ours
            res[variant] = metrics(ours, ref, counts, level0)
            print(json.dumps({f"{name}/{variant}": res[variant]}), flush=True)
        np.savez_compressed(os.path.join(out_dir, f"ref_launch_{name}.npz"), items=np.array([b, e], np.int64),
                            spa=np.int64(spa), oracle_sha256=np.array(res["oracle_sha256"]), **arrays)
        summary[name] = res
    with open(os.path.join(out_dir, "ref_launch_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
