"""HBM traffic per launch of a kernel family from the PMC passes of tools/pmc_passes.sh.

Bytes = FETCH_SIZE x 2 (gfx950 reports half of the bytes of 16-B/lane streaming reads,
MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KiB in rocprofv3's derived counters;
Infinity-Cache hits are included in these memory-side counts.

    python tools/pmc_traffic.py gpurun_out/pmc convgn [out.json]
    python tools/pmc_traffic.py gpurun_out/pmc "conv3x3_gn_pws_kernel<32>" [out.json]
"""
import csv
import glob
import re
import json
import os
import sys
from collections import defaultdict

FAMILIES = {  # census op classes; any other argument is taken as a kernel-name substring
    "convgn": ("conv3x3_gn_kernel",),
    "convgnw": ("conv3x3_gn_p4_kernel<32>", "conv3x3_gn_p4_kernel<16>"),
    "convgnw4": ("conv3x3_gn_p4_kernel<8>",),
    "conv": ("conv_pipe", "conv_small", "splitk_epilogue_kernel", "splitk_wide_epilogue_kernel"),
}


def main():
    d, fam = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    pats = FAMILIES.get(fam, (fam,))
    per = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            # the census names drop the default trailing template arguments: "<32, 0, false>" is the
            # shipped "<32>", "<16, 128, false>" the sub-pixel "<16, 128>"
            kn = re.sub(r", 0>", ">", re.sub(r", false>", ">", r["Kernel_Name"]))
            if not any(p in kn for p in pats):
                continue
            k = int(r["Dispatch_Id"])
            c = r["Counter_Name"]
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                per[k][c] = per[k].get(c, 0.0) + float(r["Counter_Value"])
                names[k] = r["Kernel_Name"]
    rows = [v for v in per.values() if "FETCH_SIZE" in v and "WRITE_SIZE" in v]
    if not rows:
        sys.exit(f"no dispatches with both counters for {pats}")
    fetch = sum(v["FETCH_SIZE"] for v in rows) * 2 * 1024 / len(rows)
    write = sum(v["WRITE_SIZE"] for v in rows) * 1024 / len(rows)
    res = {"family": fam, "kernels": sorted({n.split("(")[0] for n in names.values()}), "launches": len(rows),
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE in separate passes over one "
                     "census forward (tools/pmc_passes.sh); KiB -> bytes"}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
