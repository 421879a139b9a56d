# the ring kernel without shared thresholds (and without seeds) against the default, one image
# and C2, matcher only: what the threshold machinery is worth at these sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for a in "500 1000" "10000 100"; do
    for v in base noxs nox; do
      L=""; [ $v != base ] && L=tools/variants/lib$v.so
      SOD_LIB_PATH=$L timeout -k 10 200 python3 tools/ab_match.py $a i8 2>&1 | grep match | sed "s/^/$v /"
    done
  done
done
