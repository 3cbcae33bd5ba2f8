set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
for v in 0 1 2; do
  RSVD_GSPLIT_LG=$v timeout -k 10 120 tools/wide_lab gsplit > gpurun_out/r4i/gsplit_$v.txt 2>&1 || { cat gpurun_out/r4i/gsplit_$v.txt; exit 1; }
  echo "LG=$v"; grep "LP=128\|LP 128\|128" gpurun_out/r4i/gsplit_$v.txt | head -3
done
TESTS="tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py" CFGS="c3" STEPS=20 tools/ab_round.sh r4i "RSVD_GSPLIT_LG=0" "" "RSVD_GSPLIT_LG=2" "RSVD_GSPLIT_LG=0" ""
