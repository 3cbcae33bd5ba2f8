"""Sum rocprofv3 counter_collection.csv files per (kernel, counter) and print the means over dispatches."""
import csv, glob, os, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        k = k.replace("(anonymous namespace)::", "").replace("void rsvd::", "").split("(")[0][:110]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"    {c:32s} mean {sum(v)/len(v):.4g}  (n={len(v)})")
