# interleaved matcher A/B of the default library against tools/variants/${VAR}_libsod.so
# at AB_SIZES (ab_i8.py args, comma-separated), no test suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  for a in ${AB_SIZES:-"500,1000,200,0"}; do
    for v in new $VAR; do
      if [ $v = new ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=$PWD/tools/variants/${v}_libsod.so; fi
      echo -n "$v " ; timeout -k 10 120 python3 tools/ab_i8.py ${a//,/ } || exit 1
    done
  done
done
