# round-3 check: GPU parity suite (+ smoke).  usage: tools/gpu_r03.sh TAG [pytest-args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r03}; shift; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 "$@" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -20 gpurun_out/$TAG/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
echo smoke ok
