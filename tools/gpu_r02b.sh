cd "$GRAFT_REPO_ROOT" && timeout -k 10 60 ./tools/cu_mask_probe > gpurun_out/cu_probe.log 2>&1 && AB_ROUNDS=3 bash tools/gpu_ab_i8.sh
