#!/usr/bin/env python
"""bench.py -- photons/s of the MI355X photon-mapping lightmap baker (BASELINE.json metric).

A step = one full bake of the configuration's reference launch schedule (global_illumination_cl.c:
215-272 flattened) over the synthetic scene resident in HBM: zero the int64 lightmap, trace every
photon of this rank's shard, RCCL-reduce the per-GPU lightmaps to rank 0 (N > 1), finalise the float
texels on rank 0. Host<->device copies of the geometry and texels are outside the timed region.

  python bench.py [--gpus N --steps K --warmup W --config box200|box2000|example|box200-1e10]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Default (N=1): BASELINE config 3 -- synthetic 200-rectangle box, spa=172,413,793 = 1,000,012,800
photons per step. Multi-GPU is weak scaling: spa x N photons per step, sharded evenly by work item.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "flatmatch-global-illumination_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402

CONFIGS = {
    "box200": dict(scene="box200", spa=172_413_793, weak=True,
                   desc="synthetic 200-rectangle box scene, 1e9 photons per GPU (BASELINE config 3)"),
    "box200-1e10": dict(scene="box200", spa=1_724_137_931, weak=False,
                        desc="synthetic 200-rectangle box scene, 1e10 photons sharded over N GPUs (BASELINE config 4)"),
    "box2000": dict(scene="box2000", spa=172_413_793, weak=True,
                    desc="synthetic 2000-rectangle box scene, 1e9 photons per GPU (BASELINE config 5)"),
    "example": dict(scene="example", spa=6_500_000, weak=True,
                    desc="example.png layout, 1e8 photons per GPU (BASELINE config 2)"),
    "apartment30": dict(scene="apartment30", spa=3_000_000, weak=True,
                        desc="generated 30-room layout (654 walls, 34 light sources), 1.8e8 photons per GPU "
                             "(not a BASELINE config: the acceleration structure on a large layout)"),
}
METRIC = "photons/sec + achieved HBM GB/s (% of peak), 200-rect scene, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak (spec) = 0.5 wave64 v_fma_f32 per SIMD-cycle at 2.4 GHz


def valu_peak():
    """Measured wave64 v_fma_f32 issue ceiling of one MI355X SIMD per shader cycle, by resident waves per
    SIMD (tools/valu_peak.hip: per-SIMD s_memtime stamps with HW_ID placement, >= 50 ms launches ->
    profiles/valu_peak.json), its saturated value (8 waves) and the spec's 0.5."""
    p = os.path.join(REPO, "profiles", "valu_peak.json")
    try:
        d = json.load(open(p))
        by = {int(k): float(v) for k, v in d["f32_per_simd_per_clk_by_waves"].items()}
        return by, d.get("source", p), max(by.values()), d.get("spec_fma_per_simd_cycle", 0.5)
    except (OSError, ValueError, KeyError):
        return None, None, None, 0.5


def load_scene(name):
    from fmgi import scene

    if name in ("example", "apartment30"):
        return scene.load_geometry(os.path.join(REPO, "tests", "golden", f"{name}_geometry.bin"), name)
    return scene.box_scene(int(name[3:]))


def cpu_threads():
    """host threads for the CPU legs: OMP_NUM_THREADS (16 on the GPU box: its share of the host), else
    every CPU this process may run on"""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env or len(os.sched_getaffinity(0))


def cpu_baseline(sc, spa, target_s=10.0):
    """The reference kernel's algorithm on the host: oracle/liboracle_port.so (the plain-C restatement of
    photonmap.cl -- the linear scan over every rect, photonmap.cl:189-206 -- with the per-rect builtin
    values hoisted and FMA instructions, bit-identical to the oracle), OpenMP over work items on all the
    host threads, timed on a bounded prefix of the same schedule. Reported next to the GPU number, never
    used as the GPU result."""
    import fm_oracle as O

    threads = cpu_threads()
    offs = np.load(os.path.join(REPO, "tests", "golden", "glibc_rand_4096.npy"))
    L = O.schedule_with_offsets(sc, spa, offs)
    n = 64
    while True:
        t0 = time.perf_counter()
        _, st = O.bake_port(sc, L, 0, n, nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= target_s or n >= 10_000_000:
            break
        n = int(n * min(8.0, max(1.5, 1.2 * target_s / max(dt, 1e-3))))
    return {
        "value": st["photons"] / dt,
        "unit": "photons/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle/liboracle_port.so (photonmap.cl restated: linear scan, hoisted per-rect values, FMA) "
                  f"on the first {n} work items ({st['photons']} photons) of the same schedule, {dt:.1f} s, "
                  f"{threads} OpenMP threads",
    }


def cpu_baseline_reference(sc, target_s=10.0, procs=1):
    """The reference's own CPU photon mapper, performPhotonMappingNative (photonmap.c:408-435: BSP-tree scan,
    one photon per sample, single-threaded), built from /root/reference by oracle/build_ref.sh into
    oracle/_ref/photon_ref and timed on this host on a bounded sample of the same scene: `procs`
    independent processes at once (one per host thread: the reference's CPU path on all the cores), value =
    their photons / the slowest one's time. Its RNG is libc rand(), so it is a timing baseline, not a
    parity reference. None if the build is absent."""
    import subprocess
    import tempfile

    from fmgi import scene as S

    exe = os.path.join(REPO, "oracle", "_ref", "photon_ref")
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory() as d:
        g = os.path.join(d, "geometry.bin")
        S.save_geometry(sc, g)

        def run(spa, k):
            ps = [subprocess.Popen([exe, g, str(spa)], stdout=subprocess.PIPE, text=True) for _ in range(k)]
            outs = [p.communicate(timeout=300)[0] for p in ps]
            if any(p.returncode for p in ps):
                raise RuntimeError("photon_ref failed")
            return [json.loads(o.strip().splitlines()[-1]) for o in outs]

        area = sum(float(S._len(x["width"][:3]) * S._len(x["height"][:3])) for x in sc.sources)
        r = run(max(1, int(2e4 / max(area, 1e-6))), 1)[0]  # ~2e4 photons: calibration
        rate = r["photons"] / max(r["seconds"], 1e-6)
        rs = run(max(1, int(target_s * rate / max(area, 1e-6))), procs)
    photons = sum(x["photons"] for x in rs)
    secs = max(x["seconds"] for x in rs)
    return {
        "value": photons / secs,
        "unit": "photons/s",
        "cores": procs,
        "kind": "reference",
        "sample": f"the reference's performPhotonMappingNative (oracle/_ref/photon_ref, built from /root/reference): "
                  f"{procs} concurrent process(es) x {rs[0]['photons']} photons of the same scene, slowest "
                  f"{secs:.1f} s (a different algorithm: BSP scan, libc rand(), one photon per sample)",
    }


def cpu_baseline_radiosity(target_s=10.0, procs=1):
    """The reference's radiosityNative path (performRadiosityNative, radiosityNative.c:92-268), built from
    /root/reference by oracle/build_ref.sh into oracle/_ref/rad_ref, timed on this host on the tiny lit box
    (box200 with 2-m tiles and a ceiling light: 830 wall texels, 8.3e6 form-factor rays, ~10 s on one core):
    `procs` concurrent single-threaded processes (one per host thread), value = their rays / the slowest
    one's time. A different algorithm and unit (form-factor rays, not photons): reported beside the photon
    numbers as north_star asks, not comparable with them. None if the build is absent."""
    import subprocess
    import tempfile

    from fmgi import scene as S

    exe = os.path.join(REPO, "oracle", "_ref", "rad_ref")
    if not os.path.exists(exe):
        return None
    sc = S.box_scene(200, tile_size=2.0, with_light=True)
    rays = 10_000 * int(sum(int(w["lm"][1]) * int(w["lm"][2]) for w in sc.walls))
    with tempfile.TemporaryDirectory() as d:
        g = os.path.join(d, "geometry.bin")
        S.save_geometry(sc, g)
        t0 = time.perf_counter()
        ps = [subprocess.Popen([exe, g, os.path.join(d, f"tex{k}.bin"), "1"], stdout=subprocess.DEVNULL)
              for k in range(procs)]
        ends = []
        for p in ps:
            p.wait(timeout=max(300.0, 30 * target_s))
            ends.append(time.perf_counter() - t0)
        if any(p.returncode for p in ps):
            raise RuntimeError("rad_ref failed")
    secs = max(ends)
    return {
        "value": procs * rays / secs,
        "unit": "form-factor rays/s",
        "cores": procs,
        "kind": "reference",
        "comparable": False,
        "sample": f"the reference's performRadiosityNative (oracle/_ref/rad_ref, built from /root/reference): "
                  f"{procs} concurrent process(es) x {rays} rays (box200, 2-m tiles, ceiling light; 7 bounces), "
                  f"slowest {secs:.1f} s. Not photon-comparable: a different algorithm and unit",
    }


def pmc_record(config_name):
    """The committed rocprofv3 PMC summary of the bake (HBM bytes per launch, profiles/pmc_traffic.json)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(config_name)
    except (OSError, ValueError):
        return None


def sq_record(config_name):
    """Per-launch counters of the bake (SQ, GRBM, TA/TD/TCP) and its measured clock, from the committed
    summary of one session's rocprofv3 --pmc passes (profiles/sq_issue.json, tools/sq_summary.py)."""
    p = os.path.join(REPO, "profiles", "sq_issue.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(config_name)
    except (OSError, ValueError):
        return None


def issue_block(rec, ks, per_launch_scans, cus):
    """The bake's bounded issue and memory-path figures. Every fraction is <= 1 by construction:
      SIMD cycles   = GRBM_GUI_ACTIVE / 8 XCDs x 4 SIMDs x CUs (the profiled launch's own busy cycles;
                      the live launch time x the in-kernel clock is given beside it)
      VALU / total instructions per SIMD-cycle, against the measured VALU ceiling at the same occupancy
      wave-cycle split: SQ_ACTIVE_INST_ANY (issuing) + SQ_WAIT_INST_ANY (ready, issue-stalled) +
                      SQ_WAIT_ANY (parked on s_waitcnt / barrier) = SQ_WAVE_CYCLES (MI355X_MICROARCH.md)
      TA / TD busy  = TA_TA_BUSY_sum, TD_TD_BUSY_sum over (CUs x the per-XCD busy cycles)"""
    per = rec.get("per_launch", {})
    need = ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
            "GRBM_GUI_ACTIVE", "SQ_WAVES")
    if not all(per.get(k) for k in need):
        return None
    cyc = per["GRBM_GUI_ACTIVE"] / 8.0
    simd_cycles = cyc * 4.0 * cus
    insts = {k: per.get(f"SQ_INSTS_{k}", 0.0) for k in ("VALU", "SALU", "SMEM", "BRANCH", "VMEM", "LDS")}
    total = sum(insts.values())
    waves_per_simd = per["SQ_WAVES"] / (4.0 * cus)
    peaks, peak_src, vsat, vspec = valu_peak()
    vpeak = None
    if peaks:
        w = max(1, int(round(waves_per_simd)))
        vpeak = peaks.get(w) or peaks[min(peaks, key=lambda k: abs(k - w))]
    wc = per["SQ_WAVE_CYCLES"]
    clock = rec.get("clock_ghz")
    vpc = insts["VALU"] / simd_cycles
    out = {
        "clock_ghz": clock,
        "clock_source": rec.get("clock_source"),
        "profiled_launch_ms": cyc / (clock * 1e6) if clock else None,
        "simd_cycles_per_launch": simd_cycles,
        "live_simd_cycles_per_launch": ks * clock * 1e9 * 4.0 * cus if clock else None,
        "waves_per_simd": waves_per_simd,
        "valu_per_simd_cycle": vpc,
        "insts_per_simd_cycle": total / simd_cycles,
        "valu_peak_per_simd_cycle": vpeak,
        "valu_frac_of_peak": vpc / vpeak if vpeak else None,
        "valu_saturated_per_simd_cycle": vsat,
        "valu_frac_of_saturated": vpc / vsat if vsat else None,
        "valu_spec_per_simd_cycle": vspec,
        "valu_frac_of_spec": vpc / vspec,
        "wave_cycles": {"issuing": per["SQ_ACTIVE_INST_ANY"] / wc, "issue_stalled": per["SQ_WAIT_INST_ANY"] / wc,
                        "waiting": per["SQ_WAIT_ANY"] / wc},
        "insts_per_launch": insts,
        "insts_per_scan_wave": {k: 64.0 * v / per_launch_scans for k, v in insts.items()},
        "source": f"{rec.get('source')}; VALU ceiling {peak_src}",
    }
    if per.get("TA_TA_BUSY_sum"):
        out["vmem_path"] = {
            "ta_busy": per["TA_TA_BUSY_sum"] / (cus * cyc),
            "td_busy": per.get("TD_TD_BUSY_sum", 0.0) / (cus * cyc),
            "td_stalled_on_tc": per.get("TD_TC_STALL_sum", 0.0) / (cus * cyc),
            "tcp_accesses_per_scan_wave": 64.0 * per.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / per_launch_scans,
        }
    return out


def binding_of(issue, atomic_rate):
    """(roofline.bound, binding) from the measured figures: the resource closest to saturation"""
    if atomic_rate > 0.8 * 2.0e10:
        return "atomics", "memory-side atomic rate"
    if not issue:
        return "latency", "unmeasured for this config (no committed counter summary): see DESIGN.md §4.1"
    vm = issue.get("vmem_path", {})
    fr = {"vmem": max(vm.get("ta_busy", 0.0), vm.get("td_busy", 0.0)),
          "valu": issue.get("valu_frac_of_peak") or 0.0}
    res = max(fr, key=fr.get)
    w = issue["wave_cycles"]
    if fr[res] >= 0.8:  # (box200's VALU issue: 84 % of the ceiling 6 waves per SIMD reach, profiles/r05/s23)
        what = {"vmem": "vector-memory path (TA/TD busy %.0f %% of cycles)" % (100 * fr["vmem"]),
                "valu": "VALU issue (%.0f %% of the measured ceiling)" % (100 * fr["valu"])}[res]
        return res, what + "; waves parked on s_waitcnt %.0f %% of wave cycles" % (100 * w["waiting"])
    return "latency", ("dependent-load latency: waves parked on s_waitcnt %.0f %% of wave cycles, issuing %.0f %%; "
                       "VALU %.0f %% of its ceiling, TA/TD busy %.0f %%"
                       % (100 * w["waiting"], 100 * w["issuing"], 100 * fr["valu"], 100 * fr["vmem"]))


def weak_spa(cfg, world):
    """numSamplesPerArea of a step on `world` GPUs: weak configs take spa x world (the reference's int
    argument, global_illumination_cl.h:10), clamped to INT_MAX; the photons actually planned are what the
    BENCH line reports (config.photons_per_step), and config.spa_clamped says when the clamp bit."""
    spa = cfg["spa"] * world if (cfg["weak"] and world > 1) else cfg["spa"]
    return min(spa, 2**31 - 1), spa > 2**31 - 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="box200", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", default="auto", choices=["auto", "grid", "fast", "exact", "hybrid"])
    ap.add_argument("--accum", default="auto", choices=["auto", "fx3", "state", "stream", "none"],
                    help="none = PROFILING ONLY (deposits discarded; lightmap wrong)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--spa", type=int, default=0, help="override numSamplesPerArea of the config (per GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import fmgi
    from fmgi import parallel

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # FMGI_BENCH_BACKEND=gloo rehearses the N-rank path on fewer GPUs (ranks share devices, reductions go
    # through host memory); the default is RCCL, one rank per GPU
    backend = os.environ.get("FMGI_BENCH_BACKEND", "nccl")
    device_index = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
    torch.cuda.set_device(device_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    # what the job ran on: torch.distributed's world, and the ranks RCCL itself counts (an all-reduce of
    # ones over the process group's communicator)
    dist_info = {"world_size": dist.get_world_size() if world > 1 else 1, "backend": backend if world > 1 else None,
                 "rccl_ranks": None}
    if world > 1 and backend == "nccl":
        one = torch.ones(1, dtype=torch.int32, device=torch.device("cuda", device_index))
        dist.all_reduce(one)
        dist_info["rccl_ranks"] = int(one.item())

    cfg = dict(CONFIGS[args.config])
    if args.spa:
        cfg["spa"] = args.spa
        cfg["desc"] += f" [spa overridden: {args.spa}]"
    sc = load_scene(cfg["scene"])
    spa, spa_clamped = weak_spa(cfg, world)
    kernel = {"auto": fmgi.KERNEL_AUTO, "grid": fmgi.KERNEL_GRID, "fast": fmgi.KERNEL_FAST,
              "exact": fmgi.KERNEL_EXACT, "hybrid": fmgi.KERNEL_HYBRID}[args.kernel]

    ctx = fmgi.Context(device_index)
    ctx.set_accumulation({"auto": fmgi.ACCUM_AUTO, "fx3": fmgi.ACCUM_FX3, "state": fmgi.ACCUM_STATE,
                          "stream": fmgi.ACCUM_STREAM, "none": fmgi.ACCUM_NONE}[args.accum])
    ctx.set_scene(sc)
    libc = ctypes.CDLL(None)
    libc.srand(1)  # the unseeded state main.c runs with; every rank builds the same schedule
    total_items = ctx.plan(spa)  # consumes rand() once per reference launch
    b, e = parallel.shard_range(total_items, rank, world)
    photons_per_step = 100 * total_items

    dev = torch.device("cuda", device_index)
    # one non-default stream for every device op of the step: the lightmap zero-fill, the bake kernel,
    # the RCCL reduce (ordered after it by torch) and the finalisation; HIP events time the bake on it
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    lm = torch.zeros((sc.num_texels, 4), dtype=torch.int64, device=dev)
    tex_in = torch.zeros((sc.num_texels, 4), dtype=torch.float32, device=dev)
    tex_out = torch.empty_like(tex_in)

    k_ms, r_ms = [], []

    def step(timed):
        lm.zero_()
        if timed:
            s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_ev.record(stream)
        ctx.bake_items(b, e, lm.data_ptr(), kernel, sptr)
        if timed:
            e_ev.record(stream)
            k_ms.append((s_ev, e_ev))
        if world > 1:
            parallel.reduce_lightmap(lm, dst=0)  # RCCL over xGMI
            if timed:  # the reduce as this rank's stream sees it: from the bake's end to the reduce's end
                r_ev = torch.cuda.Event(enable_timing=True)
                r_ev.record(stream)
                r_ms.append((e_ev, r_ev))
        if rank == 0:
            ctx.finalize(lm.data_ptr(), tex_in.data_ptr(), tex_out.data_ptr(), sptr)

    ctx.set_timing(True)  # HIP events around every k_bake / fold launch, on the bake's stream
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    ctx.timing()  # drop the warm-up launches
    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    # every rank's photon counter must cover exactly its shard (no work skipped or repeated), and no stream
    # may have overflowed; a failed check ends every rank together (a lone exit would leave the others
    # waiting in the next collective until the launcher's timeout)
    shard_photons = 100 * (e - b) * args.steps
    err = None
    if st["stream_overflow"]:
        err = f"rank {rank}: stream accumulation overflowed ({st['stream_overflow']} blocks dropped): lightmap invalid"
    elif int(st["photons"]) != shard_photons:
        err = f"rank {rank}: photon counter {st['photons']} != its shard's {shard_photons}"
    if world > 1:
        bad = torch.tensor([1 if err else 0], dtype=torch.int32, device=dev)
        parallel.all_reduce(bad, dist.ReduceOp.MAX)
        if int(bad.item()) and not err:
            err = f"rank {rank}: another rank failed its photon / overflow check"
        if err:
            dist.destroy_process_group()
    if err:
        raise SystemExit(err)
    span_ms = float(np.mean([s.elapsed_time(x) for s, x in k_ms]))  # whole fmgi_bake_items per step
    tim = ctx.timing()
    bake_launch_ms = tim["bake_ms"] / max(tim["bake_launches"], 1)  # the dominant kernel, per launch
    bake_launches = tim["bake_launches"]
    if world > 1:  # per-rank breakdown, gathered to every rank (diagnoses the driver's multi-GPU runs)
        row = [float(rank), float(device_index), float(b), float(e), float(st["photons"]), bake_launch_ms,
               float(bake_launches) / args.steps, tim["fold_ms"] / args.steps, span_ms,
               float(np.mean([s0.elapsed_time(s1) for s0, s1 in r_ms])), elapsed * 1e3 / args.steps]
        keys = ("rank", "device", "item_begin", "item_end", "photons", "k_bake_ms_per_launch", "k_bake_launches_per_step",
                "fold_ms_per_step", "bake_path_ms_per_step", "reduce_ms_per_step", "wall_ms_per_step")
        rows = parallel.gather_rows(row, dev)
        dist_info["per_rank"] = [{k: (int(v) if k in ("rank", "device", "item_begin", "item_end", "photons") else v)
                                  for k, v in zip(keys, r)} for r in rows]
        dist_info["reduce_ms_per_step_max"] = max(r[9] for r in rows)
        dist_info["k_bake_ms_per_launch_spread"] = [min(r[5] for r in rows), max(r[5] for r in rows)]

    vals = torch.tensor([elapsed, st["scans"], st["deposits"], st["photons"]], dtype=torch.float64, device=dev)
    if world > 1:
        t_max = vals[:1].clone()
        parallel.all_reduce(t_max, dist.ReduceOp.MAX)
        sums = vals[1:].clone()
        parallel.all_reduce(sums, dist.ReduceOp.SUM)
        elapsed = float(t_max.item())
        scans, deposits, photons_done = (float(x) for x in sums.tolist())
    else:
        scans, deposits, photons_done = float(st["scans"]), float(st["deposits"]), float(st["photons"])

    if rank == 0:
        assert int(photons_done) == photons_per_step * args.steps, (photons_done, photons_per_step)
        value = photons_per_step * args.steps / elapsed
        # rank 0's dominant kernel (k_bake) per launch: SURVEY.md §8d algorithmic work of the photons that
        # launch traced (12 B per deposit; the 16 B/texel write-back belongs to fmgi_finalize)
        per_launch_scans = st["scans"] / bake_launches
        per_launch_deps = st["deposits"] / bake_launches
        hbm_bytes = 12.0 * per_launch_deps
        ks = bake_launch_ms / 1e3
        achieved_gbs = hbm_bytes / ks / 1e9
        # memory-side atomic adds issued per second by the bake (1 per deposit for the colour-state
        # counters, 3 for int64 RGB); ~20e9/s is the chip's rate for lane-scattered atomics
        # (MI355X_MICROARCH.md §Global float atomics: ~0.08 TB/s of 4-B adds)
        per_dep = {1: 3, 2: 1, 3: 0, 4: 0}[ctx.accumulation]
        atomic_rate = per_dep * per_launch_deps / ks
        atomics = {"per_deposit": per_dep, "achieved_per_s": atomic_rate, "ceiling_per_s": 2.0e10,
                   "frac": atomic_rate / 2.0e10}
        # what binds the bake: counters of this config and build (profiles/sq_issue.json) against the
        # measured clock and VALU ceiling; bounded fractions only (issue_block)
        # (only counters of the k_bake instance(s) this run launched: a summary of another instance, e.g. one
        # taken before a kept kernel change renamed it, is reported as stale and not used)
        instance = ctx.last_bake_kernel
        rec = sq_record(args.config)
        pmc = pmc_record(args.config)
        counters = {"kernel": instance,
                    "issue_source": rec.get("source") if rec else None,
                    "issue_matches_kernel": bool(rec) and rec.get("kernel") == instance,
                    "traffic_source": pmc.get("source") if pmc else None,
                    "traffic_matches_kernel": bool(pmc) and pmc.get("kernel") == instance}
        issue = issue_block(rec, ks, per_launch_scans, torch.cuda.get_device_properties(dev).multi_processor_count) \
            if counters["issue_matches_kernel"] else None
        traffic = pmc.get("hbm_bytes_per_launch") if counters["traffic_matches_kernel"] else None
        bound, binding = binding_of(issue, atomic_rate)
        if rec and not counters["issue_matches_kernel"]:
            binding = "unmeasured for this build (the committed counter summary names another kernel instance)"
        # SURVEY.md §8d FLOP roofline of the same launches: F = 40 x T + 150 x S per photon (40 = one
        # branch-free intersects(), 150 = sampling, tile index and colour per bounce), S = scans per photon,
        # T = rect tests per photon -- the tests this bake evaluates (its scans test a few records each), and
        # the reference's linear scan (every rect per scan, T = rects x S) as the algorithmic equivalent
        ph_launch = st["photons"] / bake_launches
        s_bar = per_launch_scans / ph_launch
        t_eval = st["tests"] / bake_launches / ph_launch
        f_eval = 40.0 * t_eval + 150.0 * s_bar
        f_lin = 40.0 * len(sc.walls) * s_bar + 150.0 * s_bar
        flops = {
            "bound_unit": "TFLOP/s", "peak": VALU_PEAK_TFLOPS,
            "scans_per_photon": s_bar, "rect_tests_per_photon": t_eval,
            "flops_per_photon": f_eval,
            "achieved": f_eval * ph_launch / ks / 1e12,
            "frac": f_eval * ph_launch / ks / 1e12 / VALU_PEAK_TFLOPS,
            "linear_scan_flops_per_photon": f_lin,
            "linear_scan_equivalent": f_lin * ph_launch / ks / 1e12,
            "linear_scan_equivalent_frac": f_lin * ph_launch / ks / 1e12 / VALU_PEAK_TFLOPS,
            "note": "achieved/frac count the rect tests the bake evaluates; linear_scan_* the reference's "
                    "rects x scans (SURVEY.md §8d), which the acceleration structure does not execute",
        }
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "photons/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if cfg["weak"] else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic scene generator; seeds = unseeded glibc rand() as the reference)",
            "config": {
                "workload": cfg["desc"],
                "scene": sc.name,
                "rects": int(len(sc.walls)),
                "texels": int(sc.num_texels),
                "spa": spa,
                "photons_per_step": photons_per_step,
                "spa_clamped": spa_clamped,
                "kernel": {0: "exact", 1: "fast", 2: "grid", 4: "hybrid"}[kernel if kernel != fmgi.KERNEL_AUTO else ctx.auto_kernel]
                + (" (auto)" if kernel == fmgi.KERNEL_AUTO else ""),
                "accumulation": {1: "fx3", 2: "state", 3: "none (PROFILING: deposits discarded)",
                                 4: "stream"}[ctx.accumulation],
                "parallelism": f"dp{world} (work-item shards, RCCL reduce of int64 lightmaps)" if backend == "nccl"
                else f"dp{world} REHEARSAL ({backend}: ranks share {torch.cuda.device_count()} GPU(s), host reduce)",
            },
            "distributed": dist_info,
            "roofline": {
                # BASELINE metric: achieved HBM GB/s of the dominant kernel (the bake) as a fraction of the
                # HBM peak, algorithmic bytes per SURVEY.md §8d (12 B per deposit) / HIP-event kernel time.
                # The bake is not HBM-bound (it writes 4 B per deposit): `bound` names the resource the
                # counters show closest to saturation, `binding` and `issue` the figures.
                "bound": bound,
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "k_bake",
                "counters": counters,
                "kernel_ms": bake_launch_ms,
                "launches_per_step": bake_launches / args.steps,
                "bake_path_ms_per_step": span_ms,
                "fold_ms_per_step": tim["fold_ms"] / args.steps,
                "algorithmic_bytes_per_launch": hbm_bytes,
                "binding": binding,
                "atomics": atomics,
                "issue": issue,
                "ops": {"scans_per_launch": per_launch_scans, "rect_tests_per_launch": st["tests"] / bake_launches,
                        "rect_tests_per_s": st["tests"] / bake_launches / ks,
                        "note": "rect tests = phase-1 record tests + exact tests the scans evaluated "
                                "(the reference's linear scan would do rects x scans)"},
            },
            "flops": flops,
            "per_photon": {
                "scans": scans / photons_done,
                "deposits": deposits / photons_done,
                "rect_tests_evaluated": st["tests"] / max(st["photons"], 1),
                "exact_rescans_per_scan": st["exact_rescans"] / max(st["scans"], 1),
                "rescans_tie_per_scan": st["rescans_tie"] / max(st["scans"], 1),
                "rescans_invalid_per_scan": st["rescans_invalid"] / max(st["scans"], 1),
            },
        }
        if os.environ.get("FMGI_LIB") == "timing":  # profiling build: where the bake's wave time goes
            import ctypes as C

            cyc = (C.c_uint64 * 16)()
            ctx.lib.fmgi_get_stage_cycles(ctx.h, cyc)
            names = ["start", "sample", "scan_phase1", "scan_phase2", "fallback", "hit", "append"]
            tot = sum(cyc[k] for k in range(len(names))) or 1
            out["stage_cycles_frac"] = {n: cyc[k] / tot for k, n in enumerate(names)}
            out["note"] = "PROFILING BUILD (s_memtime per stage): value is not a valid bench number"
        if os.environ.get("FMGI_LIB") == "clock":  # diagnostic build: s_memtime / s_memrealtime per wave
            import ctypes as C

            cyc = (C.c_uint64 * 16)()
            ctx.lib.fmgi_get_stage_cycles(ctx.h, cyc)
            out["in_kernel_clock_ghz"] = 0.1 * cyc[8] / max(cyc[9], 1)
            out["note"] = "CLOCK BUILD (FMGI_CLOCK_STAMP): in-kernel clock of k_bake, median-free wave-time weighted"
        if world == 1 and not args.no_cpu_baseline:
            # the reference kernel's algorithm on every host thread (the CL_DEVICE_TYPE_CPU analogue; the
            # reference photonmap.cl itself cannot be built for the host here: DESIGN.md §5)
            out["cpu_baseline"] = cpu_baseline(sc, cfg["spa"], args.cpu_seconds)
            ref = cpu_baseline_reference(sc, args.cpu_seconds, procs=cpu_threads())
            if ref is not None:
                out["cpu_baseline_reference_native"] = ref
            rad = cpu_baseline_radiosity(args.cpu_seconds, procs=cpu_threads())
            if rad is not None:  # north_star: radiosityNative.c timed on the host cores in the same run
                out["cpu_baseline_radiosity"] = rad
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
