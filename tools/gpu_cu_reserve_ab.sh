cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cur
for i in 1 2; do
for v in "--contexts 2" "--overlap 1 --cu-reserve 1" "--overlap 1 --cu-reserve 2" "--overlap 1"; do
  timeout -k 10 120 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras $v > gpurun_out/cur/o.log 2>&1 || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/cur/o.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4), d['good_matches'], d['surviving_bins'])"
done; done
