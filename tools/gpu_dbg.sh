cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dbg; export TMPDIR=/tmp
timeout -k 10 100 python -u -X faulthandler -m pytest tests/test_gpu_api.py -m gpu -x -v -s -k "single_train_row" --timeout 60 --timeout-method thread > gpurun_out/dbg/t.log 2>&1; echo rc=$? >> gpurun_out/dbg/t.log; tail -60 gpurun_out/dbg/t.log
