set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
timeout -k 10 120 tools/wide_lab gsplit > gpurun_out/r4g/gsplit.txt 2>&1 || { cat gpurun_out/r4g/gsplit.txt; exit 1; }
cat gpurun_out/r4g/gsplit.txt
timeout -k 10 300 python -u bench.py --config c3 --cpu-budget 0 > gpurun_out/r4g/b_c3.json 2> gpurun_out/r4g/b_c3.err || { tail gpurun_out/r4g/b_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-budget 0 > gpurun_out/r4g/b_c4.json 2> gpurun_out/r4g/b_c4.err || { tail gpurun_out/r4g/b_c4.err; exit 1; }
python3 - <<'PY'
import json
for c in ("c3","c4"):
    d=json.load(open(f"gpurun_out/r4g/b_{c}.json")); print(c, round(d["ms_per_step"],3), d["engine_info"]["cholqr_fallbacks"], d["check"]["ok"])
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_wide.py tests/test_gpu_eig.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/r4g/tests.txt 2>&1 || { tail -30 gpurun_out/r4g/tests.txt; exit 1; }
tail -3 gpurun_out/r4g/tests.txt
