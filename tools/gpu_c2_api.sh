# C2: HIP API trace beside the kernel trace (where does the host wait?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c2a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace -d "$GRAFT_REPO_ROOT/$O" -o tr --output-format csv -- python3 bench.py --config c2 --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
ls -la $O
