# A/B: matcher timing events on every S-th launch of the timed region (img1, c2), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-strideab}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
for rep in 1 2; do
  for CFG in img1 c2; do
    for S in 1 4 1000; do
      timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --no-extras --match-timing-stride $S > $O/b_${CFG}_${S}_$rep.log 2>&1 || { tail -20 $O/b_${CFG}_${S}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/b_${CFG}_${S}_$rep.log') if l.startswith('{')][0]); print('$CFG S=$S rep $rep ms/step %.5f match %.5f lat %.4f' % (d['ms_per_step'], d['stage_ms']['match_kernel'], d['single_image_latency_ms']))"
    done
  done
done
