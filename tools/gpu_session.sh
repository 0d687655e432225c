#!/usr/bin/env bash
# One gpurun session: GPU tests -> reference-kernel pin -> bench -> rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout (rc > 1) stops the session.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${FMGI_SESSION:-s1}
mkdir -p "$OUT"
step() {  # step <name> <timeout-seconds> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name"; date +%T
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
    if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
python -c "import __graft_entry__ as g; g.build()" || exit 3
for s in ${FMGI_STEPS:-tests ref bench prof}; do
  case $s in
    tests) step tests 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    ref)   step ref 600 python tests/golden/make_ref_fixtures.py "$OUT" ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)  export TMPDIR=/tmp; step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} ;;
  esac
done
echo "session done"
