# tools/sift_ctx_probe.py under SIFT stream settings, then the SIFT parity suite.
# usage: tools/gpu_sift_ctx_probe.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-siftctx}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for v in "X=0" "PROBE_SPLIT=0" "PROBE_SECOND=0" "SOD_SIFT_STREAM_MASK=0" "X=0" "PROBE_SPLIT=0"; do
  env $v PROBE_TAG="[$v]" timeout -k 10 120 python3 tools/sift_ctx_probe.py 10 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
done
cat $O/probe.log
timeout -k 10 300 python -u -m pytest tests/test_sift.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d['extras']['sift']))"
