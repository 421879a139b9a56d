# SIFT one-image A/B over environment settings: the SIFT parity suite, then
# tools/sift_prof.py wall clock per image for each setting, 5 interleaved rounds, then the
# kernel timeline of the default.  usage: tools/gpu_sift_env_ab.sh TAG "A=1" "A=0 B=2" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-siftenv}; shift; O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sift.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3 4 5; do k=0; for v in "$@"; do k=$((k+1))
  env $v timeout -k 10 120 python3 tools/sift_prof.py 500 > $O/ab_${k}_$r.log 2>&1 || { tail -5 $O/ab_${k}_$r.log; exit 1; }
  echo "[$v] r$r $(tail -1 $O/ab_${k}_$r.log)"
done; done
bash tools/gpu_sift_timeline.sh $T > /dev/null || exit 1
head -18 $O/timeline.txt; tail -16 $O/timeline.txt
