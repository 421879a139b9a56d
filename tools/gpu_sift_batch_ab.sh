# SIFT batch of 16 and one image in bench.py's process layout under SOD_SIFT_STREAM_MASK
# settings (1 = slot 0 only, the default; 2 = all slots; 0 = none), SIFT parity suite first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-siftbab}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sift.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for v in 1 2 0; do
  SOD_SIFT_STREAM_MASK=$v timeout -k 10 200 python3 bench.py --config c2 --steps 5 --warmup 5 --no-cpu-baseline > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
  grep '^{' $O/b_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['extras']['sift']; print('mask=$v r$r one %.3f batch %.3f e2e %.3f' % (d['single_image_ms'], d['batch_ms'], d['image_to_pose_batch_ms']))"
done; done
