# GPU suite (sharded tests included), N=1 bench, then a 2-rank host-transport rehearsal of the sharded bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_n1.json')); print('N1', d['value'], d['ms_per_step'])"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 2 --comm host --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_host2.json 2> gpurun_out/bench_host2.err; rc=$?
tail -2 gpurun_out/bench_host2.err; cat gpurun_out/bench_host2.json; exit $rc
