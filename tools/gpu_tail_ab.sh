# step time of the small configs against the tail's placement: CU reserve per XCD (0 = tail
# beside the matcher on any free CU) and contexts (query streams).  usage: tools/gpu_tail_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-tail}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "c2 1 1" "c2 2 1" "c2 0 2" "c2 3 1" "img1 0 2" "img1 1 1" "img1 2 1" "img1 0 3"; do
    set -- $cfg
    f=$O/${1}_r${2}_c${3}_$r.log
    if [ $2 = 0 ]; then ov=0; else ov=1; fi
    timeout -k 10 200 python3 bench.py --config $1 --cu-reserve $2 --overlap $ov --contexts $3 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    grep '^{' $f | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']
print('$1 reserve $2 ctx $3 r$r step %.4f match %.4f iso %.4f host %.4f' % (d['ms_per_step'], s['match_kernel'], s.get('match_kernel_isolated') or 0, d['host_enqueue_ms_per_step']))"
  done
done
