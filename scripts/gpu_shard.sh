# GPU tests (incl. sharded ranks over the host transport), a 2-rank bench
# rehearsal on one GPU, then the default N=1 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --comm host --scale 0.1 --steps 3 --warmup 1 > gpurun_out/bench_n2_host.json 2> gpurun_out/bench_n2_host.err; rc=$?; cat gpurun_out/bench_n2_host.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_n2_host.err; exit $rc; }
timeout -k 10 900 python bench.py --no-cpu-baseline > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err; rc=$?; cat gpurun_out/bench_n1.json; exit $rc
