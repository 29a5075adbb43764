"""Summarise rocprofv3 ``--pmc ... --output-format csv`` passes: mean value of every counter per
kernel (averaged over that kernel's dispatches), with a few derived ratios.

  python tools/pmc_summary.py OUTDIR [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if sub and sub not in name:
                    continue
                short = name.split("(")[0][:70]
                vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
                vals[short]["_vgpr"] = [float(row.get("VGPR_Count", 0) or 0)]
                vals[short]["_agpr"] = [float(row.get("Accum_VGPR_Count", 0) or 0)]
                vals[short]["_lds"] = [float(row.get("LDS_Block_Size", 0) or 0)]
    for k, cs in sorted(vals.items()):
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}")
        for c in sorted(mean):
            print(f"   {c:28s} {mean[c]:16.1f}")
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in mean:
                    print(f"   {c + ' / wave_cycles':40s} {mean[c] / wc:6.3f}")
        bc = mean.get("SQ_BUSY_CYCLES")
        if bc and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            print(f"   {'MFMA_BUSY / (BUSY*4 SIMD*CUs)':40s} (see raw; per-SE normalisation differs)")
        if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   {'LDS bank conflict / LDS active':40s} {mean['SQ_LDS_BANK_CONFLICT'] / mean['SQ_LDS_IDX_ACTIVE']:6.3f}")


if __name__ == "__main__":
    main()
