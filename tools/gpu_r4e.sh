set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
timeout -k 10 300 python -u bench.py --cpu-budget 0 > gpurun_out/r4e/b_c4.json 2> gpurun_out/r4e/b_c4.err || { tail gpurun_out/r4e/b_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --cpu-budget 0 > gpurun_out/r4e/b_c5.json 2> gpurun_out/r4e/b_c5.err || { tail gpurun_out/r4e/b_c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --cpu-budget 0 > gpurun_out/r4e/b_c3.json 2> gpurun_out/r4e/b_c3.err || { tail gpurun_out/r4e/b_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --cpu-budget 0 > gpurun_out/r4e/b_c2.json 2> gpurun_out/r4e/b_c2.err || { tail gpurun_out/r4e/b_c2.err; exit 1; }
python3 - <<'PY'
import json
for c in ("c2","c3","c4","c5"):
    d=json.load(open(f"gpurun_out/r4e/b_{c}.json")); print(c, round(d["ms_per_step"],3), d["engine_info"], d["check"]["ok"])
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r4e/tests.txt 2>&1 || { tail -30 gpurun_out/r4e/tests.txt; exit 1; }
tail -3 gpurun_out/r4e/tests.txt
