# L2->fabric read / write bytes (FETCH_SIZE, WRITE_SIZE passes) of the matcher for each
# variant in tools/variants/*.so, C3 launches from tools/ab_i8.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT="$GRAFT_REPO_ROOT/gpurun_out/pmcab"; mkdir -p "$OUT"
for v in tools/variants/*.so; do
  n=$(basename $v .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex match_i8_kernel -d "$OUT/$n/$c" -o pmc --output-format csv -- python3 tools/ab_i8.py 50000 1000 8 1 > "$OUT/$n.$c.log" 2>&1 || { tail -5 "$OUT/$n.$c.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/$n" "$OUT/$n.json" - match_i8_kernel | grep hbm
done
