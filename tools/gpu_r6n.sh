#!/bin/bash
# round 5: factor levels in place + assembly fused into the Rinv12 GEMM -- digests, tests, bench, C5 sequence
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6n/digest.txt 2>&1 || { cat gpurun_out/r6n/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6n/digest.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_bench_pin.py tests/test_gpu_knob_identity.py tests/test_gpu_dense.py > gpurun_out/r6n/tests.log 2>&1 || { tail -30 gpurun_out/r6n/tests.log; exit 1; }
tail -2 gpurun_out/r6n/tests.log
CFGS="c5 c4" STEPS=10 tools/ab_round.sh r6n "" "" || exit 1
RSVD_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6n/c5 -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/r6n/c5.log 2>&1 || { echo "rocprof failed"; exit 1; }
f=$(find gpurun_out/r6n/c5 -name "*.db" | head -1)
python3 tools/rocpd_seq.py "$f" > gpurun_out/r6n/c5_seq.txt && rm -f "$f"
tail -1 gpurun_out/r6n/c5_seq.txt
