"""MFMA pipe occupancy per kernel from a tools/pmc_mfma.sh pass.

SQ_VALU_MFMA_BUSY_CYCLES sums the MFMA-busy cycles of all SIMDs (calibrated on C4's TN kernel:
2.68e8 v_mfma_f32_16x16x32_bf16 x 16 cycles = 4.295e9, the counter reads 4.295e9); GRBM_GUI_ACTIVE
sums the 8 XCDs.  mfma_busy_frac = busy / (1024 SIMDs x GUI_ACTIVE / 8); clock_GHz_est =
(GUI_ACTIVE / 8) / dispatch duration (Start/End timestamps of the PMC run).

usage: python tools/mfma_busy.py gpurun_out/pmc_mfma_<c> <workload-key> > profiles/<tag>_mfma_busy.json
"""
import collections
import csv
import json
import os
import sys


def main():
    root, key = sys.argv[1], sys.argv[2]
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(root, "run_counter_collection.csv"))):
        k = r["Kernel_Name"].replace("void ", "").replace("rsvd::(anonymous namespace)::", "").split("(")[0]
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {"workload": key, "source": root, "method": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": {}}
    for k, v in d.items():
        if not any(s in k for s in ("proj", "gram", "jacobi", "chol", "panel", "svd")):
            continue
        busy = sum(v["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(v["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(v["GRBM_GUI_ACTIVE"]) / len(v["GRBM_GUI_ACTIVE"])
        t = sum(dur[k]) / len(dur[k]) if dur[k] else 0.0
        out["kernels"][k] = {
            "dispatches": len(v["GRBM_GUI_ACTIVE"]),
            "mfma_busy_cycles": busy,
            "gui_active_cycles_sum_xcd": gui,
            "mfma_busy_frac": busy / (1024 * gui / 8) if gui > 0 else None,
            "clock_GHz_est": (gui / 8 / t * 1e-9) if t > 0 else None,
        }
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
