# C3: threshold exchange every 8th / 16th stage (after the dense first 8) against every 4th
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/xevery; mkdir -p $O
for r in 1 2 3; do
  for v in base xe8 xe16; do
    L=""; [ $v != base ] && L=tools/variants/lib$v.so
    f=$O/c3_${v}_$r.log
    SOD_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][0]); print('c3 $v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
