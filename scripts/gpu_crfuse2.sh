# CR fusion threshold sweep (SQLM_CR_FUSE_MIN) against the unfused launches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crf_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/crf_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in unfused m128 m64 m32 m16 unfused2 m128b m64b; do
  unset SQLM_CR_UNFUSED SQLM_CR_FUSE_MIN
  case $v in unfused*) export SQLM_CR_UNFUSED=1;; m128*) export SQLM_CR_FUSE_MIN=128;; m64*) export SQLM_CR_FUSE_MIN=64;; m32) export SQLM_CR_FUSE_MIN=32;; m16) export SQLM_CR_FUSE_MIN=16;; esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/crf_$v.json 2> gpurun_out/crf_$v.err || { tail -5 gpurun_out/crf_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/crf_$v.json')); k=d['kernel_ms_per_step']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), d['chi2_last'], round(k['k_solve'],4))"
done
