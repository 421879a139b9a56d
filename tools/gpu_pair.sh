# paired waves (option match_pair = 2: the two waves of a SIMD share a query slice and take
# the even / odd subtiles of every stage): parity, then interleaved bench lines for one image
# (pair at 4 tiles vs the default 2) and C2 (pair at 8 vs the default 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pair; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges or c2_full" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in 0:0:img1 4:2:img1 0:0:c2 8:2:c2; do
    IFS=: read -r qt pair cfg <<< "$v"
    f=$O/${cfg}_q${qt}r${pair}_$r.log
    SOD_MATCH_QT=$qt SOD_MATCH_PAIR=$pair timeout -k 10 200 python3 bench.py --config $cfg --steps 300 --warmup 100 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
