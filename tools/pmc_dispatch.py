"""Per-dispatch table from the rocprofv3 --pmc passes of tools/pmc_passes.sh.

Passes run the same census forward, so dispatch ids line up across passes.

    python tools/pmc_dispatch.py gpurun_out/pmc2 [--filter conv]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    filt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    vals = defaultdict(dict)
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            name = r["Counter_Name"]
            vals[k][name] = vals[k].get(name, 0.0) + float(r["Counter_Value"])
            if k not in meta:
                meta[k] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]),
                           (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'id':>4} {'kernel':28} {'blocks':>6} {'us':>7} {'mfma%':>6} {'waitAny%':>8} {'waitInst%':>9} "
          f"{'ldsConf':>8} {'L2hit%':>6} {'fetchMB':>8} {'writeMB':>8}")
    for k in sorted(vals):
        name, grid, wg, us = meta[k]
        if filt not in name:
            continue
        v = vals[k]
        blocks = grid // max(wg, 1)
        wave = v.get("SQ_WAVE_CYCLES", 0.0)
        busy = v.get("SQ_BUSY_CYCLES", 0.0)
        mfma = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gui = v.get("GRBM_GUI_ACTIVE", 0.0)
        # gfx950 (MI355X_MICROARCH.md): SQ_VALU_MFMA_BUSY_CYCLES = 32 x MFMAs (32x32x16 bf16) summed
        # over the chip's 1024 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs -> kernel cycles =
        # GUI / 8. (The gfx94x MfmaUtil formula rocprofv3 falls back to does not apply.)
        mf = 100.0 * mfma / (gui / 8.0 * 1024) if gui else 0.0
        wa = 100.0 * v.get("SQ_WAIT_ANY", 0.0) / wave if wave else 0.0
        wi = 100.0 * v.get("SQ_WAIT_INST_ANY", 0.0) / wave if wave else 0.0
        hit, miss = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else 0.0
        fetch = v.get("FETCH_SIZE", 0.0) * 2 / 1e3  # KB -> MB with the gfx950 x2 correction
        write = v.get("WRITE_SIZE", 0.0) / 1e3
        short = name.split("(")[0].replace("void itsd::", "")[:28]
        print(f"{k:4d} {short:28} {blocks:6d} {us:7.1f} {mf:6.1f} {wa:8.1f} {wi:9.1f} "
              f"{v.get('SQ_LDS_BANK_CONFLICT', 0.0):8.3g} {l2:6.1f} {fetch:8.1f} {write:8.1f}")


if __name__ == "__main__":
    main()
