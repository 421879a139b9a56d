# PMC counter passes for one matcher kernel (one counter group per rocprofv3 run, no
# tracing domains combined with --pmc).  Usage on the GPU box:
#     bash tools/gpu_pmc.sh [config] [impl]        (impl: i8 | i8w | bf16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CFG=${1:-c3}
IMPL=${2:-i8}
case $IMPL in i8) K=match_i8_kernel ;; i8w) K=match_i8w_kernel ;; bf16) K=match_kernel ;; esac
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_${K}_$CFG"
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$OUT/$name" -o pmc \
    --output-format csv -- python3 bench.py --config "$CFG" --impl "$IMPL" --steps 2 --warmup 1 --no-cpu-baseline --no-extras --contexts 1 \
    > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU || exit $?
run sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS || exit $?
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
exit 0
