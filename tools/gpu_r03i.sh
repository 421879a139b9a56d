# shared best-row slots (SOD_I8_SLOTS) and the tree slow-path update (SOD_I8_TREE): matcher
# parity with the in-tree build, then interleaved A/B against tools/variants/libsod_<v>.so on
# the small-query configs and C3.  usage: tools/gpu_r03i.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r03i}; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab_small.sh $T "$@" || exit 1
for r in 1 2; do for v in base "$@"; do
  if [ $v = base ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=$PWD/tools/variants/libsod_$v.so; fi
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $O/c3_${v}_r$r.log 2>&1 || { tail -5 $O/c3_${v}_r$r.log; exit 1; }
  grep '^{' $O/c3_${v}_r$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('C3 $v r$r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
done; done
