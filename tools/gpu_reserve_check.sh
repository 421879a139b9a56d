# CU-split (sod_set_cu_reserve) parity tests + default bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/res
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v --timeout 120 --timeout-method thread -k "overlap" > gpurun_out/res/pytest.log 2>&1 || { tail -30 gpurun_out/res/pytest.log; exit 1; }
tail -3 gpurun_out/res/pytest.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/res/bench$i.log 2>&1 || { tail -20 gpurun_out/res/bench$i.log; exit 1; }
  grep '^{' gpurun_out/res/bench$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d['config'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --comm host --no-extras > gpurun_out/res/host2.log 2>&1 || { tail -20 gpurun_out/res/host2.log; exit 1; }
grep '^{' gpurun_out/res/host2.log | cut -c1-300
