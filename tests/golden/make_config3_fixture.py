"""Regenerate tests/golden/oracle_config3.npz: the oracle's whole BASELINE config 3 lightmap (box200, spa =
172,413,793: 10,000,128 work items, 1,000,012,800 photons, 391 launches), so the GPU suite compares the HIP
bake with it without re-running ~200 s of host oracle.

Generated in the build container from oracle/liboracle_port.so (the oracle's restatement of photonmap.cl with
the per-rect values hoisted, bit-identical to liboracle.so: tests/test_oracle.py) over the schedule of the
committed glibc rand() prefix, in 16 item ranges. Stored: the int64 [numTexels, 3] lightmap (units of 2^-25),
the per-range photon / scan / deposit / escape counters, a SHA-256 digest of each range's own int64 lightmap
(so the live range is checked against the fixture's lightmap, not only its counters) and the range
cuts. test_config3_full_lightmap_exact compares the GPU's whole lightmap with it and re-runs one of the 16
ranges live, so the fixture itself stays checked against the oracle of the commit.

  python tests/golden/make_config3_fixture.py [nthreads]
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "flatmatch-global-illumination_amd")]

import fm_oracle as O  # noqa: E402
from fmgi import scene as S  # noqa: E402

SPA = 172_413_793
RANGES = 16
KEYS = ("photons", "scans", "deposits", "escapes")


def main():
    nthreads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    box = S.box_scene(200)
    offsets = np.load(os.path.join(HERE, "glibc_rand_4096.npy"))
    L = O.schedule_with_offsets(box, SPA, offsets)
    n = int(L["item_begin"][-1] + L["count"][-1])
    cuts = np.array([n * k // RANGES for k in range(RANGES + 1)], np.int64)
    lm = np.zeros((box.num_texels, 3), np.int64)
    stats = np.zeros((RANGES, len(KEYS)), np.int64)
    digests = np.zeros((RANGES, 32), np.uint8)
    t0 = time.time()
    for k in range(RANGES):
        part, st = O.bake_port(box, L, int(cuts[k]), int(cuts[k + 1]), nthreads=nthreads)
        lm += part
        digests[k] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(part, np.int64).tobytes()).digest(), np.uint8)
        stats[k] = [st[key] for key in KEYS]
        print(f"range {k + 1}/{RANGES}: items {cuts[k + 1]:,} of {n:,} ({time.time() - t0:.0f} s)", flush=True)
    np.savez_compressed(os.path.join(HERE, "oracle_config3.npz"), lightmap=lm, cuts=cuts, stats=stats, range_sha256=digests,
                        stat_keys=np.array(KEYS), spa=np.int64(SPA), launches=np.int64(len(L)))


if __name__ == "__main__":
    main()
