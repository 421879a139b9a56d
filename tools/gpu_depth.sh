# DB prefetch depth for one image: burst refill at the stage barrier (DMA=0) with 32-subtile
# stages in 2 slots (b32), 16-subtile stages in 2 (b16r2) or 4 slots (b16r4: 3 stages = 96 KiB
# ahead) against the default spread refill; parity of b16r4 first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/depth; mkdir -p $O
SOD_LIB_PATH=tools/variants/libb16r4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base b32 b16r2 b16r4; do
    L=""; [ $v != base ] && L=tools/variants/lib$v.so
    f=$O/img1_${v}_$r.log
    SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config img1 --steps 300 --warmup 50 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('img1 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
