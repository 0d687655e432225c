set -o pipefail
# A/B of the fold's colour-table variants (FMGI_FOLD_CARRY, experiment build) in one process per config, each
# setting twice; tools/ab_exact.py checks every setting's lightmap bit for bit against the first one.
#   AB_CARRY="2 4 5" AB_OUT=gpurun_out/r6f1 bash tools/ab_colour.sh
export TMPDIR=/tmp
O=${AB_OUT:-gpurun_out/r6f1}; mkdir -p $O
S=""
for r in 1 2; do for k in ${AB_CARRY:-2 4 5}; do S="$S --set FMGI_FOLD_CARRY=$k"; done; done
for c in ${AB_CONFIGS:-box200 box2000 example}; do
  echo "== $c $(date +%T)"
  FMGI_LIB=exp timeout -k 10 300 python tools/ab_exact.py --config $c --reps 3 $S > $O/ab_$c.log 2>&1 || { echo "rc=$? on $c"; tail -5 $O/ab_$c.log; exit 1; }
  cat $O/ab_$c.log | grep '^{'
done
