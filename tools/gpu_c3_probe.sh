set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/main_c3_probe.py > gpurun_out/c3_probe.log 2>&1 || { tail -20 gpurun_out/c3_probe.log; exit 1; }
cat gpurun_out/c3_probe.log
