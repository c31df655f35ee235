# Round-3 closing GPU call: full check (default library), then the k_msm_bucket phase-timing probe
# and the quad-distributed k_msm_final variant (uncached-key tests + msm leg) from build_exp/.
set -o pipefail
bash tools/sha_and_check.sh r03z || exit 1
mkdir -p gpurun_out/r03y
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_msmtiming.so timeout -k 10 120 python3 -u tools/msm_probe.py > gpurun_out/r03y/timing.log 2>&1 || exit 1
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_quadd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_keys.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03y/quadd_tests.log 2>&1 || { tail -20 gpurun_out/r03y/quadd_tests.log; exit 1; }
tail -1 gpurun_out/r03y/quadd_tests.log
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_quadd.so timeout -k 10 180 python3 -u tools/msm_ab.py > gpurun_out/r03y/quadd_msm.jsonl 2>&1 || exit 1
timeout -k 10 180 python3 -u tools/msm_ab.py > gpurun_out/r03y/default_msm.jsonl 2>&1 || exit 1
cat gpurun_out/r03y/quadd_msm.jsonl gpurun_out/r03y/default_msm.jsonl
