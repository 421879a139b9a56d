# SIFT lone-image stream split A/B: the SIFT parity suite, then tools/sift_prof.py wall clock
# per image with SOD_SIFT_LAYER_SPLIT / SOD_SIFT_EAGER_RANK interleaved, then the kernel timeline of the
# default.  usage: tools/gpu_sift_split_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-siftab}; O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sift.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
# v: <octaves split (9 = all)><eager rank>
for r in 1 2 3 4 5; do for v in ${VARIANTS:-01 91 90}; do
  SOD_SIFT_LAYER_SPLIT=${v:0:1} SOD_SIFT_EAGER_RANK=${v:1:1} timeout -k 10 120 python3 tools/sift_prof.py 500 > $O/ab_${v}_$r.log 2>&1 || { tail -5 $O/ab_${v}_$r.log; exit 1; }
  echo "split,eager=$v r$r $(tail -1 $O/ab_${v}_$r.log)"
done; done
bash tools/gpu_sift_timeline.sh $T > /dev/null || exit 1
head -22 $O/timeline.txt
