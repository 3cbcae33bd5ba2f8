set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
timeout -k 10 300 python -u bench.py --config c5 --cpu-budget 0 > gpurun_out/r4f/b_c5.json 2> gpurun_out/r4f/b_c5.err || { tail gpurun_out/r4f/b_c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-budget 0 > gpurun_out/r4f/b_c4.json 2> gpurun_out/r4f/b_c4.err || { tail gpurun_out/r4f/b_c4.err; exit 1; }
python3 - <<'PY'
import json
for c in ("c4","c5"):
    d=json.load(open(f"gpurun_out/r4f/b_{c}.json")); print(c, round(d["ms_per_step"],3), d["engine_info"], d["check"])
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_eig.py tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_dense.py > gpurun_out/r4f/tests.txt 2>&1 || { tail -30 gpurun_out/r4f/tests.txt; exit 1; }
tail -3 gpurun_out/r4f/tests.txt
