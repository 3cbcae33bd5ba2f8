#!/bin/bash
# round 5, call e: new shard / limit / long-n tests, C2 PMC passes (no cooperative launches at C2),
# then ONE PMC pass on the default cooperative path (C4 MFMA busy) LAST: does --pmc also hit the
# rocprofv3 7.2 exit-time fault that --kernel-trace hits after a cooperative launch?
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5e
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread \
  "tests/test_gpu_distributed.py::test_row_sharded_world2_shard_smaller_than_l" \
  "tests/test_gpu_big_l.py::test_big_l_range_finder_and_limits" \
  "tests/test_gpu_configs.py::test_split_cross_gram_long_n" > $R/gpurun_out/r5e/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $R/gpurun_out/r5e/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
out=$R/gpurun_out/prof_r05_c2
mkdir -p $out
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 $R/bench.py --config c2 --steps 3 --warmup 1 --cpu-budget 0 > $out/fetch.log 2>&1) || { tail -5 $out/fetch.log; exit 1; }
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 $R/bench.py --config c2 --steps 3 --warmup 1 --cpu-budget 0 > $out/write.log 2>&1) || { tail -5 $out/write.log; exit 1; }
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $out/mfma -o run -- python3 $R/bench.py --config c2 --steps 1 --warmup 1 --cpu-budget 0 > $out/mfma.log 2>&1) || { tail -5 $out/mfma.log; exit 1; }
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $R/bench.py --config c2 --steps 20 --warmup 3 --cpu-budget 0 > $out/trace.log 2>&1) || { tail -5 $out/trace.log; exit 1; }
echo "c2 passes ok"
out=$R/gpurun_out/prof_r05_c4coop
mkdir -p $out
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $out/mfma -o run -- python3 $R/bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 > $out/mfma.log 2>&1
echo "c4 MFMA PMC pass on the cooperative path: rc=$?"
ls $out/mfma
