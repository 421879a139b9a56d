# C2 bench step: default library vs tools/variants/${VAR}_libsod.so, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2 3; do
  for v in new $VAR; do
    if [ $v = new ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=$PWD/tools/variants/${v}_libsod.so; fi
    timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras > gpurun_out/c2l.log 2>&1 || { tail -5 gpurun_out/c2l.log; exit 1; }
    grep "^{" gpurun_out/c2l.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-8s' % '$v', round(d['ms_per_step'],4), round(d['host_enqueue_ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
