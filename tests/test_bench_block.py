"""CPU test of bench.py's roofline block over the committed measurement set (profiles/): every figure
the BENCH line derives from counters can be recomputed from the files of this commit, and is bounded."""
import importlib.util
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_issue_block_from_committed_counters_is_bounded():
    b = _bench()
    rec = b.sq_record("box200")
    assert rec is not None, "profiles/sq_issue.json has no box200 record"
    # the counters' own source directory is committed
    src = rec["source"].split("/{")[0]
    assert os.path.isdir(os.path.join(REPO, src)), src
    kernel_s = json.load(open(os.path.join(REPO, src, "kernel_timed_launches.json")))["k_bake_timed_mean_ms"] / 1e3
    scans = 8.0e9  # box200: scans per launch (bench per_photon.scans x photons)
    iss = b.issue_block(rec, kernel_s, scans, 256)
    assert iss is not None
    for k in ("valu_frac_of_peak", "valu_frac_of_saturated", "valu_frac_of_spec"):
        assert 0 < iss[k] <= 1.05, (k, iss[k])
    assert iss["valu_peak_per_simd_cycle"] <= iss["valu_saturated_per_simd_cycle"] <= iss["valu_spec_per_simd_cycle"]
    w = iss["wave_cycles"]
    assert abs(w["issuing"] + w["issue_stalled"] + w["waiting"] - 1.0) < 0.02, w
    for k, v in iss["vmem_path"].items():
        if k.endswith("busy") or k.startswith("td_stalled"):
            assert 0 <= v <= 1.0, (k, v)
    assert 0 < iss["valu_per_simd_cycle"] <= 1.0
    # the profiled launch (GRBM busy cycles at the in-kernel clock) agrees with the live HIP-event time
    assert iss["profiled_launch_ms"] == pytest.approx(kernel_s * 1e3, rel=0.03)
    bound, why = b.binding_of(iss, 0.0)
    assert bound in ("valu", "vmem", "latency", "atomics") and why


def test_traffic_summary_is_committed():
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    d = json.load(open(p))["box200"]
    assert "k_bake" in d["kernel"]
    assert d["hbm_bytes_per_launch"] == pytest.approx(d["fetch_bytes_per_launch"] + d["write_bytes_per_launch"])
    src = d["source"].split(":")[0]
    assert os.path.isdir(os.path.join(REPO, src)), src


def test_valu_ceiling_summary_is_committed_and_consistent():
    """profiles/valu_peak.json: its session is committed; the per-SIMD v_fma_f32 rates grow with occupancy
    up to at most the spec's 0.5 per SIMD-cycle; the counter-derived rate of each measured launch (GRBM
    cycles, the method bench.py applies to the bake) agrees with the per-SIMD stamps"""
    d = json.load(open(os.path.join(REPO, "profiles", "valu_peak.json")))
    src = d["source"].split("/valu.log")[0]
    assert os.path.isdir(os.path.join(REPO, src)), src
    by = {int(k): v for k, v in d["f32_per_simd_per_clk_by_waves"].items()}
    assert by[1] < by[2] <= max(by.values()) <= d["spec_fma_per_simd_cycle"] == pytest.approx(0.5, rel=0.01)
    for w, c in d["counters"]["fma64"].items():
        assert c["valu_per_simd_cycle"] == pytest.approx(by[int(w)], rel=0.05), (w, c)


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "rad_ref")),
                    reason="oracle/_ref not built (needs /root/reference at build time)")
def test_radiosity_cpu_leg_runs():
    """bench.py's cpu_baseline_radiosity: the reference's performRadiosityNative on the lit 2-m-tile box,
    labelled not photon-comparable (north_star: radiosityNative.c timed on the host cores in the same run)."""
    b = _bench()
    r = b.cpu_baseline_radiosity(procs=1)
    assert r["kind"] == "reference" and r["comparable"] is False and r["cores"] == 1
    assert r["unit"] == "form-factor rays/s" and r["value"] > 0


def test_weak_scaling_spa_fits_the_reference_int_at_8_gpus():
    """bench.py's weak configs run spa x N photons per area at N GPUs; numSamplesPerArea is an int in the
    reference's interface (global_illumination_cl.h:10), so spa x 8 must stay <= INT_MAX for every config, and
    a clamp (never hit by these configs) is reported instead of silently changing the workload."""
    b = _bench()
    for name, cfg in b.CONFIGS.items():
        for n in (1, 2, 4, 8):
            spa, clamped = b.weak_spa(cfg, n)
            assert spa <= 2**31 - 1
            if cfg["weak"]:
                assert not clamped, (name, n)
                assert spa == cfg["spa"] * n
            else:
                assert spa == cfg["spa"]
    huge = {"spa": 2**30, "weak": True}
    assert b.weak_spa(huge, 4) == (2**31 - 1, True)
