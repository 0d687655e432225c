#!/usr/bin/env python
"""profiles/valu_peak.json from one session of tools/valu_peak (steps `valu`, `valupmc` of tools/gpu_session.sh):
the vector-instruction issue ceilings of one MI355X SIMD, by instruction and resident waves per SIMD, measured
per SIMD (each wave's s_memtime stamps and HW_ID/XCC_ID: rate = instructions of a SIMD's waves / its first-in
to last-out shader cycles), with the rocprofv3 counters of the same cases beside them (SQ_INSTS_VALU per
SIMD-cycle from GRBM_GUI_ACTIVE, the method bench.py applies to the bake).

bench.py valu_peak() reads f32_per_simd_per_clk_by_waves (the v_fma_f32 ceiling at the bake's occupancy).

  python tools/valu_summary.py profiles/r04/s1 [--out profiles/valu_peak.json]"""
import argparse
import collections
import csv
import glob
import json
import os

SPEC_TFLOPS = 157.3  # MI355X FP32 vector peak (spec): 256 CUs x 4 SIMDs x 2.4 GHz x 64 lanes x 2 flops x 0.5


def counters(session):
    """per case: the measured launch of each wave count (the last dispatch of its group of five:
    calibration, calibration, 2 x sustained load, measured) -> VALU and SALU per SIMD-cycle"""
    out = {}
    for p in sorted(glob.glob(os.path.join(session, "valupmc_*", "**", "*counter_collection.csv"), recursive=True)):
        case = os.path.relpath(p, session).split(os.sep)[0][len("valupmc_"):]
        by = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(p)):
            by[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        ids = sorted(by)
        rows = {}
        for k in ids[4::5]:
            d = by[k]
            simd_cycles = d["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0
            w = int(round(d["SQ_WAVES"] / 1024.0))
            rows[str(w)] = {"valu_per_simd_cycle": d["SQ_INSTS_VALU"] / simd_cycles,
                            "salu_per_simd_cycle": d["SQ_INSTS_SALU"] / simd_cycles,
                            "active_inst_valu_cycles_per_valu": 4.0 * d["SQ_ACTIVE_INST_VALU"] / d["SQ_INSTS_VALU"],
                            "wave_cycles_issuing": d["SQ_ACTIVE_INST_ANY"] / d["SQ_WAVE_CYCLES"]}
        out[case] = rows
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "valu_peak.json"))
    a = ap.parse_args()
    cases = [json.loads(l) for l in open(os.path.join(a.session, "valu.log")) if l.startswith("{") and '"case"' in l]
    by = collections.defaultdict(dict)
    for c in cases:
        by[c["case"]][str(c["waves_per_simd"])] = c["per_simd_cycle_median_exact_w"]
    one = {c["case"]: c["cycles_per_inst_per_wave"] for c in cases if c["waves_per_simd"] == 1}
    sat = {k: max(v.values()) for k, v in by.items()}
    spec = SPEC_TFLOPS * 1e12 / (256 * 4 * 2.4e9 * 128)  # wave64 v_fma_f32 per SIMD-cycle at the spec peak
    rec = {
        "source": f"{a.session}/valu.log (tools/valu_peak.hip: per-SIMD s_memtime stamps, HW_ID placement, >= 50 ms "
                  f"launches, 64 independent instructions per loop iteration over 16 chains) and "
                  f"{a.session}/valupmc_*/ (rocprofv3 --pmc of the same cases)",
        "f32_per_simd_per_clk_by_waves": by["fma64"],
        "by_case": by,
        "one_wave_cycles_per_instruction": one,
        "saturated_per_simd_cycle": sat,
        "spec_fma_per_simd_cycle": spec,
        "saturated_fma_frac_of_spec": sat["fma64"] / spec,
        "counters": counters(a.session),
        "reading": [
            "v_fma_f32: one wave alone issues one every 5.4 cycles (MI355X_MICROARCH.md's table: 4); two waves double "
            "it; the SIMD saturates at 0.39 per cycle with 3-4 waves and 0.45 with 8 (the spec's 157.3 TF is 0.5: "
            "wave64 over the 32-lane SIMD in 2 cycles)",
            "v_pk_fma_f32, v_fma_f64 and v_mul_u32_u24 occupy the SIMD for 4 cycles: 0.24-0.25 per cycle at any "
            "occupancy, so packed fp32 gives no more flops than v_fma_f32 and the 24-bit multiply is half rate",
            "v_add_u32: 4.4 cycles for one wave, 0.45-0.47 per cycle from 2 waves",
            "SALU: the CU's scalar unit serves its 4 SIMDs; at one s_mul_i32 per v_fma_f32 both settle at 0.235 "
            "per SIMD-cycle (0.94 scalar instructions per CU-cycle)",
            "the round-3 microbenchmark (8 FMAs per loop iteration, case fma8): 8.5 cycles per VALU for one wave = "
            "8 x 5.4 + the loop's s_add/s_cmp/s_cbranch; its 0.27 at 4 waves was a chip-average over an uneven "
            "placement; this tool measures per SIMD and reports the placement (every SIMD held exactly the "
            "requested waves in this session)",
        ],
        "note": "bench.py prices the bake's VALU rate against f32_per_simd_per_clk_by_waves at the bake's resident "
                "waves per SIMD",
    }
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps({"fma64": by["fma64"], "saturated": sat}))


if __name__ == "__main__":
    main()
