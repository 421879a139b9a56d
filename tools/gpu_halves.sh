# one query image as 4 query tiles per wave in two subtile halves (option match_halves):
# parity with it on, then interleaved bench lines against 2 tiles per wave and against the
# previous library (tools/variants/libold.so), one image and C3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/halves; mkdir -p $O
SOD_MATCH_HALVES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges or pipeline" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in new halves old; do
    L=""; E=0
    [ $v = old ] && L=tools/variants/libold.so
    [ $v = halves ] && E=1
    SOD_LIB_PATH=$L SOD_MATCH_HALVES=$E timeout -k 10 200 python3 bench.py --config img1 --steps 300 --warmup 100 --no-cpu-baseline --no-extras > $O/img1_${v}_$r.log 2>&1 || { tail -5 $O/img1_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/img1_${v}_$r.log') if l.startswith('{')][0]); print('img1 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
for r in 1 2 3; do
  for v in new old; do
    L=""; [ $v = old ] && L=tools/variants/libold.so
    SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][0]); print('c3 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
