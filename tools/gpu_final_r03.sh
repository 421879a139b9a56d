# round-3 final evidence: full GPU parity suite, smoke, then tools/gpu_r03d.sh (bench lines,
# rocprofv3 kernel stats, PMC passes).  usage: tools/gpu_final_r03.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r03zf}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_r03d.sh $T || exit 1
