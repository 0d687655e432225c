"""Pack the gfx950 v_sqrt_f32 / v_rsq_f32 truth tables into tests/golden/gfx950_sqrt_rsq.npz.

Input: the raw output of tools/hw_sqrt_rsq_table.hip run on an MI355X (int8 delta_sqrt[2^24], then int8
delta_rsq[2^24]; each entry = the hardware result minus the once-rounded double value, in ulps, for the
input x in [1, 4) with index exponent-parity << 23 | mantissa). Both ops depend only on that class
(tools/hw_sqrt_table.hip checks it over 40 binades) and are within 1 ulp, so each entry packs into 2 bits.
The CPU oracle (oracle/fm_oracle.py hw_tables) unpacks them to reproduce ROCm's length()/normalize().

  python tests/golden/make_hw_tables.py gpurun_out/hw/sqrt_rsq_delta.bin
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main(path):
    d = np.fromfile(path, np.int8)
    assert d.size == 2 << 24, d.size
    d = d.reshape(2, -1)
    assert d.min() >= -1 and d.max() <= 1
    packed = {}
    for k, name in enumerate(("sqrt", "rsq")):
        v = (d[k] + 1).astype(np.uint8)
        packed[name] = (v[0::4] | (v[1::4] << 2) | (v[2::4] << 4) | (v[3::4] << 6)).astype(np.uint8)
    np.savez_compressed(os.path.join(HERE, "gfx950_sqrt_rsq.npz"), **packed)
    print({k: int((d[i] != 0).sum()) for i, k in enumerate(("sqrt", "rsq"))})


if __name__ == "__main__":
    main(sys.argv[1])
