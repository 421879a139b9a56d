# upper bound of what the stage barrier costs: a diagnostic build without it (SOD_I8_NOBAR,
# waves race on the ring: WRONG results, timing only) against the default, matcher only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for a in "50000 1000" "500 1000" "10000 100"; do
    for v in base nobar; do
      L=""; [ $v != base ] && L=tools/variants/lib$v.so
      SOD_LIB_PATH=$L timeout -k 10 200 python3 tools/ab_match.py $a i8 2>&1 | grep match | sed "s/^/$v /"
    done
  done
done
