# EG bench line, then a 2-rank RCCL rehearsal with both ranks on GPU 0 (small GBA).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config eg > gpurun_out/bench_eg.json 2> gpurun_out/bench_eg.err; rc=$?
cat gpurun_out/bench_eg.json; tail -3 gpurun_out/bench_eg.err; [ $rc -eq 0 ] || exit $rc
SQLM_BENCH_ONE_GPU=1 NCCL_DEBUG=WARN timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --scale 0.05 --no-cpu-baseline \
  > gpurun_out/rccl2.json 2> gpurun_out/rccl2.err; rc=$?
cat gpurun_out/rccl2.json; tail -15 gpurun_out/rccl2.err; exit $rc
