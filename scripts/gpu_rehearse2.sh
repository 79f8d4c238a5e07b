# 2-rank host-transport rehearsal of the sharded bench on one GPU (the driver's N>1 path minus RCCL).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 2 --comm host --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_host2.json 2> gpurun_out/bench_host2.err; rc=$?
tail -2 gpurun_out/bench_host2.err; cut -c1-700 gpurun_out/bench_host2.json; exit $rc
