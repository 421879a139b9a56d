# shared-threshold apply without the vmcnt(0) wait (variant xw0, SOD_I8_XWAIT=0): parity,
# then interleaved bench lines (one image, C2, C3) against the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/xwait; mkdir -p $O
SOD_LIB_PATH=tools/variants/libxw0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges or c2_full" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base:img1:300 xw0:img1:300 base:c2:300 xw0:c2:300 base:c3:30 xw0:c3:30; do
    IFS=: read -r lib cfg n <<< "$v"
    L=""; [ $lib != base ] && L=tools/variants/lib$lib.so
    f=$O/${cfg}_${lib}_$r.log
    SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config $cfg --steps $n --warmup 20 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
