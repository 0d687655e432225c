#!/usr/bin/env bash
# A/B of experiment builds (make -C <pkg> variant VNAME=...): one short bench per (variant, config).
#   VARIANTS="base b3s1 ..." CONFIGS="box200 example" FMGI_SESSION=sX bash tools/variants.sh
# "base" = the product library. A crash/timeout (rc > 1) stops the run.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${FMGI_SESSION:-v1}
mkdir -p "$OUT"
for v in ${VARIANTS:-base}; do
  for c in ${CONFIGS:-box200}; do
    if [ "$v" = base ]; then unset FMGI_LIB; else export FMGI_LIB=$v; fi
    timeout -k 10 300 python bench.py --config "$c" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${VARGS:-} > "$OUT/v_${v}_$c.log" 2>&1
    rc=$?
    python - "$OUT/v_${v}_$c.log" "$v" "$c" "$rc" <<'PY'
import json, sys
p, v, c, rc = sys.argv[1:]
line = [l for l in open(p) if l.startswith("{")]
if not line:
    print(f"{v:10s} {c:8s} rc={rc} (no result)")
else:
    d = json.loads(line[0])
    print(f"{v:10s} {c:8s} {d['value']:.4e} photons/s  k_bake {d['roofline']['kernel_ms']:.1f} ms x{d['roofline'].get('launches_per_step',0):.0f}  path {d['roofline'].get('bake_path_ms_per_step',0):.1f} ms  fold {d['roofline'].get('fold_ms_per_step',0):.1f} ms  [{d['config']['kernel']}]")
PY
    if [ $rc -gt 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
  done
done
