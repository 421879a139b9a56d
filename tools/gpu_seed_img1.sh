# one query image (500 x 1M) and C2: the ring kernel's seed-pass extent per query-tile count,
# interleaved rounds, one process per (variant, QT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/seed_img1; mkdir -p $O
for r in 1 2; do
  for v in base seed16 seed8 noseed; do
    if [ $v = base ]; then L=""; else L=tools/variants/lib$v.so; fi
    for qt in 2 4; do
      SOD_LIB_PATH=$L SOD_MATCH_QT=$qt timeout -k 10 120 python3 tools/ab_i8.py 500 1000 64 0 > $O/${v}_qt${qt}_$r.log 2>&1 || { tail -5 $O/${v}_qt${qt}_$r.log; exit 1; }
      echo "$v qt$qt r$r $(tail -1 $O/${v}_qt${qt}_$r.log)"
    done
  done
done
