set -o pipefail
export ROUNDS=2
timeout -k 10 200 python -u tools/ab_small.py tiny,img1,c2,q5k > gpurun_out/r05b_default.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libscount.so timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05b_count.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libsnox.so timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05b_nox.log 2>&1
