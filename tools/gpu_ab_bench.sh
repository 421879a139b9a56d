# interleaved bench A/B of library variants on one box: TAG ROUNDS "CONFIGS" LIB...
# (LIB "default" = sift-based-od_amd/libsod.so, else tools/variants/lib<LIB>.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=$1; R=$2; CFGS=$3; shift 3; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -c "import torch" > /dev/null 2>&1
for r in $(seq 1 $R); do
  for CFG in $CFGS; do
    for L in "$@"; do
      if [ "$L" = default ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=tools/variants/lib$L.so; fi
      timeout -k 10 300 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/b_${L}_${CFG}_$r.log 2>&1 || { tail -20 $O/b_${L}_${CFG}_$r.log; exit 1; }
      grep '^{' $O/b_${L}_${CFG}_$r.log > $O/b_${L}_${CFG}_$r.json
      python3 -c "
import json; d=json.load(open('$O/b_${L}_${CFG}_$r.json'))
print('round $r $CFG %-8s' % '$L', 'step %.4f ms' % d['ms_per_step'], 'matcher %.4f ms' % d['stage_ms']['match_kernel'], 'frac %.4f' % d['roofline']['frac'], 'good', d['good_matches'], 'valid', d['valid_bins'], 'surv', d['surviving_bins'])"
    done
  done
done
