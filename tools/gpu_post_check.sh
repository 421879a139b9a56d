# exact post-processing: GPU tests + the C3 post-processing time
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-postcheck}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_quick_tests.sh ${1:-postcheck} "postprocess or fullsize or main or pipeline" || exit 1
timeout -k 10 200 python3 bench.py --config c3 --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][0]); print('c3 post', d['stage_ms']['post_process'], 'step', d['ms_per_step'])"
