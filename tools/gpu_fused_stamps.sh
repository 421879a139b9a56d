# phase stamps of hough_small_kernel (variant build with SOD_SEL_STAMP)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-fst}; mkdir -p $O; export TMPDIR=/tmp
SOD_LIB_PATH=$PWD/tools/stampvar/libsod.so timeout -k 10 120 python3 tools/fused_stamps.py img1 > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
