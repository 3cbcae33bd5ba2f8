set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
timeout -k 10 120 tools/wide_lab_cprof chol > gpurun_out/r4d/chol_prof.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eig.py tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_dense.py > gpurun_out/r4d/tests.txt 2>&1 || { tail -30 gpurun_out/r4d/tests.txt; exit 1; }
cat gpurun_out/r4d/chol_prof.txt; tail -3 gpurun_out/r4d/tests.txt
