set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
timeout -k 10 120 tools/wide_lab_cprof chol > gpurun_out/r4c/chol_prof.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c/cholk -o run -- tools/wide_lab chol > gpurun_out/r4c/chol_k.log 2>&1 || exit 1
timeout -k 10 120 tools/wide_lab gsplit > gpurun_out/r4c/gsplit.txt 2>&1 || exit 1
timeout -k 10 60 tools/eig_lab 256 256 3 > gpurun_out/r4c/eig.txt 2>&1 || exit 1
timeout -k 10 60 tools/eig_lab 512 512 3 >> gpurun_out/r4c/eig.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_eig.py > gpurun_out/r4c/eigtest.txt 2>&1 || { tail -30 gpurun_out/r4c/eigtest.txt; exit 1; }
cat gpurun_out/r4c/chol_prof.txt gpurun_out/r4c/gsplit.txt gpurun_out/r4c/eig.txt; tail -3 gpurun_out/r4c/eigtest.txt
