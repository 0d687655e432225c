#!/usr/bin/env python
"""One line per bench JSON in a gpu_session.sh session directory: config, photons/s, ms/step, k_bake ms, fold ms."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            if not isinstance(d.get("config"), dict):
                continue
            r = d.get("roofline", {})
            print(f"{os.path.basename(f)[:-4]:14s} {d['config'].get('scene', '?'):12s} {d['value']:.4g} "
                  f"ms/step {d['ms_per_step']:.2f} bake {r.get('kernel_ms', 0):.2f} fold {r.get('fold_ms_per_step', 0):.2f} "
                  f"kernel {d['config'].get('kernel')}")
