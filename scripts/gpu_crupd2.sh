# 2x2-grouped E update (k_cr_update_gemm2): parity tests, then A/B by SQLM_CR_UPD2_MIN (chi2_last must match bit for bit).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cr_fuse.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cru_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/cru_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in off m64 m1 off2 m64b m1b; do
  unset SQLM_CR_UPD2_MIN
  case $v in off*) export SQLM_CR_UPD2_MIN=1000000;; m64*) export SQLM_CR_UPD2_MIN=64;; m1*) export SQLM_CR_UPD2_MIN=1;; esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/cru_$v.json 2> gpurun_out/cru_$v.err || { tail -5 gpurun_out/cru_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/cru_$v.json')); k=d['kernel_ms_per_step']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), repr(d['chi2_last']), round(k['k_solve'],4))"
done
