#!/bin/bash
# Round-4 GPU pass: CR A/B (deep back-substitution launch), full -m gpu suite,
# smoke, default bench line. usage: gpurun --timeout 1200 -- 'bash scripts/gpu_r4_round.sh TAG'
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
out=gpurun_out/cr_${tag}.log
: > $out
for shape in "278 112" "9 112" "4 112"; do
  for v in "" "SQLM_CR_DEEP_BACK=1"; do
    echo "-- $shape $v" >> $out
    env $v CRB_NO_LEVELS=1 timeout -k 5 60 ./tools/cr_bench $shape 20 2>&1 | grep '"p"' >> $out || exit 1
  done
done
cat $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_${tag}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_${tag}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${tag}.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err
rc=$?
tail -c 600 gpurun_out/bench_${tag}.json
exit $rc
