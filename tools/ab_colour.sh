set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6f1; mkdir -p $O
S="--set FMGI_FOLD_CARRY=2 --set FMGI_FOLD_CARRY=4 --set FMGI_FOLD_CARRY=5 --set FMGI_FOLD_CARRY=2 --set FMGI_FOLD_CARRY=4 --set FMGI_FOLD_CARRY=5"
for c in box200 box2000 example; do
  echo "== $c $(date +%T)"
  FMGI_LIB=exp timeout -k 10 300 python tools/ab_exact.py --config $c --reps 3 $S > $O/ab_$c.log 2>&1 || { echo "rc=$? on $c"; tail -5 $O/ab_$c.log; exit 1; }
  cat $O/ab_$c.log | grep '^{'
done
