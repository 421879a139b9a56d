# one-image seed length at 2 query tiles per wave: 8 / 12 subtiles against the default 16
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/seedqt2; mkdir -p $O
SOD_LIB_PATH=tools/variants/libseed8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "one_query or query_tiles" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base seed8 seed12; do
    L=""; [ $v != base ] && L=tools/variants/lib$v.so
    f=$O/img1_${v}_$r.log
    SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config img1 --steps 300 --warmup 50 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('img1 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
