# round-3 check: GPU parity suite + smoke, then C3 / C2 bench lines.  usage: tools/gpu_r03b.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r03b}; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=20 > gpurun_out/$TAG/pytest.log 2>&1 || { tail -60 gpurun_out/$TAG/pytest.log; exit 1; }
tail -25 gpurun_out/$TAG/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python3 bench.py > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.err || { tail -30 gpurun_out/$TAG/bench_c3.err; exit 1; }
echo c3 ok
timeout -k 10 200 python3 bench.py --config c2 --no-extras > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.err || { tail -30 gpurun_out/$TAG/bench_c2.err; exit 1; }
echo c2 ok
