#!/usr/bin/env bash
# A/B of environment knobs on the product library: ENVS="A=1:B=2 C=3 ..." (one set per run, ':'-joined)
set -u
cd "$(dirname "$0")/.."
for e in ${ENVS:-none}; do
  echo "env: $e"
  ( [ "$e" != none ] && for kv in ${e//:/ }; do export "$kv"; done
    VARIANTS=base CONFIGS="${CONFIGS:-box200}" FMGI_SESSION=${FMGI_SESSION}_$(echo "$e" | tr -c 'A-Za-z0-9\n' '_') bash tools/variants.sh ) || exit $?
done
