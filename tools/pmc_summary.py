"""Aggregate rocprofv3 --pmc CSV output per kernel (sum over dispatches and per-dispatch mean).

    python tools/pmc_summary.py gpurun_out/pmc1 [gpurun_out/pmc2 ...] [--kernel conv_pipe]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs):
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "?")
                name = r.get("Counter_Name")
                agg[k][name] += float(r.get("Counter_Value", 0) or 0)
                cnt[k][name] += 1
    return agg, cnt


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = None
    if "--kernel" in sys.argv:
        filt = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != filt]
    agg, cnt = load(args)
    for k in sorted(agg, key=lambda k: -max(agg[k].values())):
        if filt and filt not in k:
            continue
        print(k[:100])
        for name in sorted(agg[k]):
            n = cnt[k][name]
            print(f"   {name:32s} sum {agg[k][name]:16.4g}   per-dispatch {agg[k][name] / max(n, 1):14.4g}  (n={n})")


if __name__ == "__main__":
    main()
