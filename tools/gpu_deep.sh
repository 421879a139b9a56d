# prefilter two subtiles behind the MFMAs (variants deep2 / deep4: SOD_I8_DEEPQT = 2 / 4)
# against the default one-behind pipeline: parity of deep4, then interleaved bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/deep; mkdir -p $O
SOD_LIB_PATH=tools/variants/libdeep4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges or c2_full" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base:img1 deep2:img1 base:c2 deep4:c2; do
    IFS=: read -r lib cfg <<< "$v"
    L=""; [ $lib != base ] && L=tools/variants/lib$lib.so
    f=$O/${cfg}_${lib}_$r.log
    SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config $cfg --steps 300 --warmup 50 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
