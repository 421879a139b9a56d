# ring fragment reads as inline-asm ds_read_b128 with counted lgkmcnt waits (variant asm,
# SOD_I8_ASMLDS=1) at LDS prefetch 1 / 2 against the default build: parity (both prefetch
# distances), then interleaved bench lines for one image, C2 and C3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/asmlds; mkdir -p $O
for pf in 2 1; do
  SOD_MATCH_PF=$pf SOD_LIB_PATH=tools/variants/libasm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "matcher or one_query or golden or edges or c2_full" --timeout 200 --timeout-method thread > $O/pytest_pf$pf.log 2>&1 || { tail -30 $O/pytest_pf$pf.log; exit 1; }
  tail -1 $O/pytest_pf$pf.log
done
for r in 1 2; do
  for v in base:1:img1:300 asm:1:img1:300 asm:2:img1:300 base:1:c2:300 asm:1:c2:300 asm:2:c2:300 base:1:c3:30 asm:1:c3:30 asm:2:c3:30; do
    IFS=: read -r lib pf cfg n <<< "$v"
    L=""; [ $lib != base ] && L=tools/variants/lib$lib.so
    f=$O/${cfg}_${lib}_pf${pf}_$r.log
    SOD_MATCH_PF=$pf SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config $cfg --steps $n --warmup 20 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
