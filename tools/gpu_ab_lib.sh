# interleaved A/B of two libsod builds on the default bench (A = tools/variants/old_libsod.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ablib
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export SOD_LIB_PATH=$PWD/tools/variants/old_libsod.so; else unset SOD_LIB_PATH; fi
    timeout -k 10 150 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/ablib/o.log 2>&1 || { tail -5 gpurun_out/ablib/o.log; exit 1; }
    grep '^{' gpurun_out/ablib/o.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4), d['surviving_bins'])"
  done
done
