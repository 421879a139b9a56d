# LDS prefetch distance A/B (SOD_MATCH_PF 1 / 2): parity of the matcher tests with PF 2, the
# small-query configs, one image at QT 4, and C3.  usage: tools/gpu_r03g.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r03g}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
SOD_MATCH_PF=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or c2 or one_query" --timeout 300 --timeout-method thread > $O/pytest_pf2.log 2>&1 || { tail -30 $O/pytest_pf2.log; exit 1; }
tail -2 $O/pytest_pf2.log
VAR=SOD_MATCH_PF MODES=1,2 timeout -k 10 400 python3 -u tools/small_q.py > $O/pf_small.log 2> $O/pf_small.err || { tail -20 $O/pf_small.err; exit 1; }
head -3 $O/pf_small.log | cut -c1-600
SOD_MATCH_QT=4 CONFIGS=img500x1M VAR=SOD_MATCH_PF MODES=1,2 timeout -k 10 200 python3 -u tools/small_q.py > $O/pf_img_qt4.log 2> $O/pf_img_qt4.err || { tail -20 $O/pf_img_qt4.err; exit 1; }
head -1 $O/pf_img_qt4.log | cut -c1-600
for r in 1 2; do for pf in 1 2; do
  SOD_MATCH_PF=$pf timeout -k 10 200 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $O/c3_pf${pf}_r$r.log 2>&1 || { tail -5 $O/c3_pf${pf}_r$r.log; exit 1; }
  grep '^{' $O/c3_pf${pf}_r$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('C3 pf $pf r$r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
done; done
