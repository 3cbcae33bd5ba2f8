set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
timeout -k 10 120 tools/wide_lab gcross > gpurun_out/r4h/gcross.txt 2>&1 || { cat gpurun_out/r4h/gcross.txt; exit 1; }
cat gpurun_out/r4h/gcross.txt
TESTS="tests/test_gpu_wide.py tests/test_gpu_eig.py tests/test_gpu_configs.py" CFGS="c5" STEPS=20 tools/ab_round.sh r4h "RSVD_GSPLIT_X=1" "" "RSVD_GSPLIT_X=1" ""
