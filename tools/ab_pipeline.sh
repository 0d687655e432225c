#!/usr/bin/env bash
# A/B of the STREAM fold pipeline knobs: PB="pipeline:foldblock:wg_per_cu ..." (0 = default)
set -u
cd "$(dirname "$0")/.."
for pb in ${PB:-1:1024:0 4:1024:0}; do
  IFS=: read -r p b w <<< "$pb"
  echo "pipeline=$p foldblock=$b wg_per_cu=$w"
  FMGI_PIPELINE=$p FMGI_FOLD_BLOCK=$b FMGI_BAKE_WG_PER_CU=$w VARIANTS=base CONFIGS="${CONFIGS:-box200}" \
    FMGI_SESSION=${FMGI_SESSION}_p${p}b${b}w${w} bash tools/variants.sh || exit $?
done
