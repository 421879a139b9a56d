# A/B: untimed matcher-stream launches signal the context stream by a dispatch-recorded end
# event (SOD_END_EVENT=1) instead of a marker after the kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-endev}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
for rep in 1 2 3; do
  for CFG in img1 c2; do
    for E in 0 1; do
      if [ $E = 1 ]; then export SOD_END_EVENT=1; else unset SOD_END_EVENT; fi
      timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/b_${CFG}_${E}_$rep.log 2>&1 || { tail -20 $O/b_${CFG}_${E}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/b_${CFG}_${E}_$rep.log') if l.startswith('{')][0]); print('$CFG endev=$E rep $rep ms/step %.5f match %.5f' % (d['ms_per_step'], d['stage_ms']['match_kernel']))"
    done
  done
done
