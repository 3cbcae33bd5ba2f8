#!/bin/bash
# round 5, call g: R^-1 fused into chol_reg_kernel (RSVD_CHOL_RINV A/B): digest bit-identity, lab,
# Cholesky-path tests, bench A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5g
for v in 0 1; do
  RSVD_CHOL_RINV=$v timeout -k 10 120 python tools/digest_run.py > $R/gpurun_out/r5g/digest_$v.txt 2>&1 || { cat $R/gpurun_out/r5g/digest_$v.txt; exit 1; }
  echo "rinv fused=$v"; grep -v amdgpu.ids $R/gpurun_out/r5g/digest_$v.txt
done
timeout -k 10 180 ./tools/wide_lab_cprof chol > $R/gpurun_out/r5g/chol.txt 2>&1 || { cat $R/gpurun_out/r5g/chol.txt; exit 1; }
grep -E "chol|diagonal" $R/gpurun_out/r5g/chol.txt
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_eig.py tests/test_gpu_big_l.py > $R/gpurun_out/r5g/tests.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r5g/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CFGS="c4 c5 c3" STEPS=10 tools/ab_round.sh r5g "RSVD_CHOL_RINV=0" "RSVD_CHOL_RINV=1"
