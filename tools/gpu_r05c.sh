set -o pipefail
export ROUNDS=2
timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05c_default.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libscount.so timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05c_count.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libscount2.so timeout -k 10 200 python -u tools/ab_small.py img1,c2 > gpurun_out/r05c_count2.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libsd4.so timeout -k 10 200 python -u tools/ab_small.py img1,c2 > gpurun_out/r05c_d4.log 2>&1
