set -o pipefail
export ROUNDS=2
timeout -k 10 200 python -u tools/ab_small.py tiny,odd,img1,c2,q2k,q5k > gpurun_out/r05d_default.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libscount.so timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05d_count.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libsd8.so timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05d_d8.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libsn4.so timeout -k 10 200 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05d_n4.log 2>&1
