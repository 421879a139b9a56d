# SIFT stream CU-mask settings (SOD_SIFT_STREAM_MASK 0 none / 1 slot 0 / 2 all) in a bench-like
# process (matcher context split, then unsplit as bench.py's extras): one image and a batch
# of 16, 3 interleaved rounds.  usage: tools/gpu_sift_mask_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-siftmask}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
for v in "SOD_SIFT_STREAM_MASK=0" "SOD_SIFT_STREAM_MASK=1" "SOD_SIFT_STREAM_MASK=2"; do
  env $v PROBE_UNSPLIT=1 PROBE_TAG="[$v r$r]" timeout -k 10 120 python3 tools/sift_ctx_probe.py 10 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
  tail -1 $O/probe.log
done; done
