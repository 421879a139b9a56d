# one query image (500 x 1M): ring kernel with 4 waves per work-group (one wave per SIMD,
# half the LDS fragment reads per MFMA) at 2 / 4 / 8 query tiles per wave and LDS prefetch
# 1 / 2, against the default 8-wave build; parity of the 4-wave build first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/nw4_img1; mkdir -p $O
SOD_LIB_PATH=tools/variants/libnw4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in base:2:1 nw4:2:1 nw4:4:1 nw4:4:2 nw4:8:1 nw4:8:2; do
    IFS=: read -r lib qt pf <<< "$v"
    L=""; [ $lib != base ] && L=tools/variants/lib$lib.so
    f=$O/${lib}_q${qt}p${pf}_$r.log
    SOD_LIB_PATH=$L SOD_MATCH_QT=$qt SOD_MATCH_PF=$pf timeout -k 10 200 python3 bench.py --config img1 --steps 300 --warmup 100 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('img1 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
