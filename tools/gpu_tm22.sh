# stage-top waits split (SOD_I8_TIME2=2 build): the wave's own refill (vmcnt) vs the barrier
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tm22; mkdir -p $O
for a in "500 1000" "10000 100" "50000 1000"; do
  TIME2=1 SOD_LIB_PATH=tools/variants/libtm22.so timeout -k 10 300 python3 tools/ab_match.py $a i8 > $O/tm22_${a// /_}.log 2>&1 || { tail -5 $O/tm22_${a// /_}.log; exit 1; }
  grep -E "match|per wave" $O/tm22_${a// /_}.log
done
