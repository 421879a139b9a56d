set -o pipefail
mkdir -p gpurun_out/r06i
for S in 128 62 0; do
  python3 tools/probes/sift_operand_bytes.py /tmp/sift_s$S.bin $S || exit 1
  timeout -k 10 100 ./tools/probes/mfma_power /tmp/sift_s$S.bin x >> gpurun_out/r06i/shift.log 2>&1 || exit 1
done
cat gpurun_out/r06i/shift.log
