"""Per-kernel HBM traffic from rocprofv3 PMC passes (tools/profile.sh output).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane) coalesced streaming read, so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  profiles/r02_fetch_calibration.json
(tools/fetch_calib.hip) measured the factor for the projection kernels' own access shapes -- 32-,
64- and 128-B column runs and contiguous streaming read by global_load_lds_dwordx4 all report
0.50-0.52 of the bytes -- so the doubled figure applies to every projection kernel.

usage: python tools/traffic.py gpurun_out/prof_<tag> <workload-key> > profiles/traffic_<key>.json
"""
import collections
import csv
import json
import os
import sys


def short(name):
    return name.replace("void ", "").replace("rsvd::(anonymous namespace)::", "").split("(")[0]


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}, {k: len(v) for k, v in d.items()}


def main():
    root, key = sys.argv[1], sys.argv[2]
    fetch, nf = per_kernel(os.path.join(root, "fetch", "run_counter_collection.csv"))
    write, _ = per_kernel(os.path.join(root, "write", "run_counter_collection.csv"))
    out = {"workload": key, "source": root,
           "correction": "FETCH_SIZE x2 for every kernel (calibrated for 32/64/128-B column runs and streaming: "
                         "profiles/r02_fetch_calibration.json); WRITE_SIZE x1",
           "kernels": {}}
    for k in fetch:
        if not (k.startswith("rsvd::") or "proj" in k or "gram" in k or "svd" in k or "panel" in k):
            continue
        f = 2 * fetch[k] * 1024
        w = write.get(k, 0.0) * 1024
        out["kernels"][k] = {"dispatches": nf[k], "fetch_bytes": f, "write_bytes": w, "hbm_bytes": f + w}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
