# one query image: 16-subtile stages with one or two work-groups per CU (4 waves per SIMD)
# against the default 32-subtile stage, bench img1 lines, interleaved; parity with the
# two-work-group variant first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/occ_img1; mkdir -p $O
SOD_LIB_PATH=tools/variants/libsps16x2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base sps16 sps16x2; do
    L=""; [ $v != base ] && L=tools/variants/lib$v.so
    SOD_LIB_PATH=$L timeout -k 10 200 python3 bench.py --config img1 --steps 300 --warmup 100 --no-cpu-baseline --no-extras > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/${v}_$r.log') if l.startswith('{')][0]); print('img1 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
