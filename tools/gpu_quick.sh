# GPU suite + short bench lines (c3, c2, img1; no CPU baseline / extras). usage: TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-quick}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -c "import torch; print('torch', torch.__version__)" > $O/torch_warm.log 2>&1 || { tail -5 $O/torch_warm.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for CFG in c3 c2 img1; do
  timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  grep '^{' $O/bench_$CFG.log > $O/bench_$CFG.json
  python3 -c "import json; d=json.load(open('$O/bench_$CFG.json')); print('$CFG ms/step %.5f match %.5f lat %.4f' % (d['ms_per_step'], d['stage_ms']['match_kernel'], d['single_image_latency_ms']), {k: round(v, 4) for k, v in (d['stage_ms_whole_chip'] or {}).items()})"
done
