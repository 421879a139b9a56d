set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02g
SOD_LIB_PATH=$PWD/tools/variants/libsod_stamp.so timeout -k 10 120 python3 tools/ab_match.py 50000 1000 i8 > gpurun_out/r02g/stamp_c3.log 2>&1 || { tail -5 gpurun_out/r02g/stamp_c3.log; exit 1; }
SOD_LIB_PATH=$PWD/tools/variants/libsod_stamp.so timeout -k 10 120 python3 tools/ab_match.py 10000 100 i8 > gpurun_out/r02g/stamp_c2.log 2>&1 || { tail -5 gpurun_out/r02g/stamp_c2.log; exit 1; }
cat gpurun_out/r02g/stamp_c3.log gpurun_out/r02g/stamp_c2.log
