# two matcher streams (default) vs one (SOD_MSTREAMS=1): split/overlap parity tests, then
# c3 / c2 / img1 step A/B, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-mstreams}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "overlap or untimed_split or cu_reserve or query_batch or sharded or threshold_slots or one_query_image" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for CFG in img1 c2 c3; do
    for M in 2 1; do
      timeout -k 10 200 env SOD_MSTREAMS=$M python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/b_${CFG}_${M}_$rep.log 2>&1 || { tail -20 $O/b_${CFG}_${M}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/b_${CFG}_${M}_$rep.log') if l.startswith('{')][0]); print('$CFG mstreams=$M rep $rep ms/step %.5f match %.5f' % (d['ms_per_step'], d['stage_ms']['match_kernel']))"
    done
  done
done
