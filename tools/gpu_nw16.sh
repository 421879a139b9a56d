# one query image (500 x 1M) and C2: ring kernel with 16 waves per work-group (4 per SIMD, one
# work-group holds the whole one-image query set, so each DB chunk crosses L2 once) against the
# default 8-wave build; parity of the 16-wave build first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/nw16_img1; mkdir -p $O
SOD_LIB_PATH=tools/variants/libnw16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in base:2:1:img1 nw16:2:1:img1 nw16:2:2:img1 base:4:1:c2 nw16:2:1:c2 nw16:4:1:c2; do
    IFS=: read -r lib qt pf cfg <<< "$v"
    L=""; [ $lib != base ] && L=tools/variants/lib$lib.so
    f=$O/${cfg}_${lib}_q${qt}p${pf}_$r.log
    SOD_LIB_PATH=$L SOD_MATCH_QT=$qt SOD_MATCH_PF=$pf timeout -k 10 200 python3 bench.py --config $cfg --steps 300 --warmup 100 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
