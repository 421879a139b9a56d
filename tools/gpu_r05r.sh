# affine outlier-test rounding (option affine_fma) and the affine / pipeline parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "outlier or affine or pipeline or main or c3 or golden" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
# the N > 1 bench path (FileStore bootstrap, barriers, max over ranks, host-staged exchange)
# with two ranks on the box's one GPU
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --comm host --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log | cut -c1-400
