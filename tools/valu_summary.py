#!/usr/bin/env python
"""profiles/valu_peak.json from the JSON lines of tools/valu_peak (one case per line): the v_fma_f32 case's
wave64 VALU instructions per SIMD-cycle at its own in-kernel clock, by resident waves per SIMD (bench.py
valu_peak() reads f32_per_simd_per_clk_by_waves).

  python tools/valu_summary.py profiles/r03/<session>/valu_peak.jsonl [--out profiles/valu_peak.json]"""
import argparse
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jsonl")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "valu_peak.json"))
    a = ap.parse_args()
    cases = [json.loads(l) for l in open(a.jsonl) if l.startswith("{") and '"case"' in l]
    by = {str(c["waves_per_simd"]): c["per_simd_per_clk_at_measured_clock"] for c in cases if c["case"] == "v_fma_f32"}
    rec = {"source": f"{a.jsonl}: tools/valu_peak.hip on one MI355X, >= 50 ms launches, 8 independent v_fma_f32 "
                     "chains per lane (three VGPR sources, as compiled code reads them), in-kernel clock "
                     "(s_memtime / s_memrealtime) per case",
           "f32_per_simd_per_clk_by_waves": by, "cases": cases,
           "note": "the ceiling bench.py prices the bake's VALU rate against, at the bake's resident waves per SIMD"}
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(by))


if __name__ == "__main__":
    main()
