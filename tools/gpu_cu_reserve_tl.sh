# kernel timeline of the CU-split bench (sod_set_cu_reserve) and of the 2-context default
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tl
timeout -k 10 180 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/tl" -o res1 --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras --cu-reserve 1 > gpurun_out/tl/res1.log 2>&1 || exit 1
for v in "--cu-reserve 1" "--contexts 2" "--cu-reserve 1" "--contexts 2"; do
  timeout -k 10 120 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras $v > gpurun_out/tl/o.log 2>&1 || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/tl/o.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4), d['good_matches'], d['surviving_bins'])"
done
