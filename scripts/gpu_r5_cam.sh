#!/bin/bash
# CR A/Bs (update waves: gpu_r5_upd.sh; LDS-staged TRSM: cr_bench_t1 vs
# cr_bench_u1), then the camera-pass / landmark-update variants: bitwise check
# against the committed library and interleaved bench A/B.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5h}
out=gpurun_out/trsm_$tag.log
: > $out
for rep in 1 2; do
for shape in "278 112" "9 112" "140 112" "17 96"; do
  for b in cr_bench_u1 cr_bench_t1 cr_bench_t4 cr_bench_ts; do
    echo -n "$b $shape " >> $out
    CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/$b $shape 30 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep '"x_hash"' gpurun_out/crb_tmp.log >> $out
    [ $rc -eq 0 ] || { echo "rc=$rc" >> $out; tail -5 gpurun_out/crb_tmp.log >> $out; exit 1; }
  done
done
done
bash scripts/gpu_r5_upd.sh $tag || exit 1
out=gpurun_out/cam_$tag.log
: > $out
for v in libsqrtlm_cam4.so libsqrtlm_lmh.so libsqrtlm_new.so; do
  echo "bits $v" >> $out
  timeout -k 10 240 python -u scripts/ab_bits.py $v 0.2 >> $out 2>&1 || { echo "rc=$?" >> $out; exit 1; }
done
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm_base.so libsqrtlm_cam4.so libsqrtlm_cam5n.so libsqrtlm_lmh.so \
  libsqrtlm_new.so libsqrtlm_base.so libsqrtlm_cam4.so libsqrtlm_cam5n.so libsqrtlm_lmh.so libsqrtlm_new.so >> $out 2>&1 || exit 1
echo done
