# one query image: ring-kernel exchange / seed knobs against the default, bench img1 lines,
# interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/knob_img1; mkdir -p $O
for r in 1 2 3; do
  for v in new xdense16 xevery1 seedq8 dense16; do
    if [ $v = new ]; then L=""; else L=tools/variants/lib$v.so; fi
    SOD_LIB_PATH=$L timeout -k 10 200 python3 bench.py --config img1 --steps 300 --warmup 100 --no-cpu-baseline --no-extras > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/${v}_$r.log') if l.startswith('{')][0]); print('$v round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
