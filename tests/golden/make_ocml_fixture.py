"""Record the device library's sin/cos (ROCm ocml __ocml_sin_f32 / __ocml_cos_f32 on the MI355X) on every
reachable sampler phi as a SHA-256 (run on the GPU box; the JSON is committed as
tests/golden/ocml_sincos.json). tests/test_math.py checks the CPU restatements against it.

  python tests/golden/make_ocml_fixture.py [out_dir]
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "flatmatch-global-illumination_amd")]

import fm_oracle as O  # noqa: E402
import fmgi  # noqa: E402


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else HERE
    phi = O.reachable_phi()
    ctx = fmgi.Context(0)
    s, c = ctx.device_sincosf(phi, library=True)
    ctx.close()
    d = {"inputs": int(len(phi)),
         "sha256_sin_cos_bits": hashlib.sha256(s.view(np.uint32).tobytes() + c.view(np.uint32).tobytes()).hexdigest(),
         "source": "fmgi_device_sincosf_library (HIP sinf/cosf = ROCm ocml) on an MI355X, phi in O.reachable_phi() order"}
    print(json.dumps(d))
    with open(os.path.join(out_dir, "ocml_sincos.json"), "w") as f:
        json.dump(d, f, indent=1)


if __name__ == "__main__":
    main()
