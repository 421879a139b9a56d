# one query image (500 x 1M): ring-kernel query tiles per wave 2 / 4 / 8 (option match_qt
# seeded from SOD_MATCH_QT), interleaved rounds of the img1 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/qt_img1; mkdir -p $O
for r in 1 2 3; do
  for qt in 2 4 8; do
    SOD_MATCH_QT=$qt timeout -k 10 200 python3 bench.py --config img1 --steps 200 --warmup 100 --no-cpu-baseline --no-extras > $O/qt${qt}_$r.log 2>&1 || { tail -5 $O/qt${qt}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/qt${qt}_$r.log') if l.startswith('{')][0]); print('qt $qt round $r', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4))"
  done
done
