#!/bin/bash
# round 5, call f: the padded Sturm count (digest + eigensolver tests), C3 stall / LDS / cache counter
# passes and traffic (RSVD_COOP=0: clean exits), then the C4 kernel trace on the cooperative path LAST
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5f
timeout -k 10 120 python tools/digest_run.py > $R/gpurun_out/r5f/digest.txt 2>&1 || { cat $R/gpurun_out/r5f/digest.txt; exit 1; }
grep -v amdgpu.ids $R/gpurun_out/r5f/digest.txt
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_eig.py tests/test_gpu_bench_pin.py > $R/gpurun_out/r5f/tests.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r5f/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
out=$R/gpurun_out/prof_r05f_c3
mkdir -p $out
B="python3 $R/bench.py --config c3 --steps 2 --warmup 1 --cpu-budget 0"
cd /tmp
RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/p1 -o run -- $B > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_MFMA --output-format csv -d $out/p2 -o run -- $B > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $out/p3 -o run -- $B > $out/p3.log 2>&1 || { tail -5 $out/p3.log; echo "p3 failed (continuing)"; }
RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- $B > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- $B > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
echo "c3 counter passes ok"
out=$R/gpurun_out/prof_r05f_c4
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $R/bench.py --config c4 --steps 3 --warmup 1 --cpu-budget 0 > $out/trace.log 2>&1
echo "c4 kernel trace (cooperative path) rc=$? (139: the known exit-time fault after the trace is written)"
ls $out/trace
