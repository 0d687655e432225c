#!/usr/bin/env python
"""oracle/geosphere_check.py -- one-off check, run in the container that holds /root/reference:
oracle/geosphere.py's tables equal the reference's geoSphere.c tables (parsed as text; values are
the double literals rounded to float, as the C compiler does) for levels 3, 4 and 5, in order.
Writes the SHA-256 of each float32 table to tests/golden/geosphere.json (no reference data)."""
import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import geosphere  # noqa: E402


def reference_table(src, name):
    i = src.index("const Vector3 %s[]" % name)
    j = src.index("};", i)
    rows = re.findall(r"\{ *([-0-9.e]+) *, *([-0-9.e]+) *, *([-0-9.e]+) *\}", src[i:j])
    return np.array([[float(x) for x in r] for r in rows], dtype=np.float64).astype(np.float32)


def main():
    ref = os.environ.get("FMGI_REFERENCE", "/root/reference")
    src = open(os.path.join(ref, "geoSphere.c")).read()
    out = {}
    for level in (3, 4, 5):
        r = reference_table(src, "geoSphere%d" % level)
        g = geosphere.generate(level)
        assert r.shape == g.shape and np.array_equal(r.view(np.uint32), g.view(np.uint32)), level
        out[str(level)] = {"count": int(len(g)), "sha256_f32": hashlib.sha256(g.tobytes()).hexdigest()}
        print("level %d: %d directions identical to geoSphere%d" % (level, len(g), level))
    path = os.path.join(HERE, "..", "tests", "golden", "geosphere.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", os.path.normpath(path))


if __name__ == "__main__":
    main()
