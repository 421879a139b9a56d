# paired waves WITH the counted asm LDS waits (now at <= 2 tiles per wave and phase) and
# two-ahead prefetch: one image (pair 4) and C2 (pair 8 / plain 4, variant asm1 = asm reads
# at every tile count) against the defaults; parity of both libraries first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pair_asm; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "vs_oracle_options or query_tiles" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
SOD_LIB_PATH=tools/variants/libasm1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "vs_oracle or query_tiles or c2_full" --timeout 200 --timeout-method thread > $O/pytest_asm1.log 2>&1 || { tail -30 $O/pytest_asm1.log; exit 1; }
tail -1 $O/pytest_asm1.log
for r in 1 2 3; do
  for v in base:0:0:0:img1 base:4:2:1:img1 base:4:2:2:img1 base:0:0:0:c2 asm1:4:1:2:c2 asm1:8:2:2:c2 base:8:2:2:c2; do
    IFS=: read -r lib qt pair pf cfg <<< "$v"
    L=""; [ $lib != base ] && L=tools/variants/lib$lib.so
    f=$O/${cfg}_${lib}_${qt}_${pair}_${pf}_$r.log
    SOD_LIB_PATH=$L SOD_MATCH_QT=$qt SOD_MATCH_PAIR=$pair SOD_MATCH_PF=$pf timeout -k 10 300 python3 bench.py --config $cfg --steps 300 --warmup 50 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
