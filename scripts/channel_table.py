"""Per-channel TCC read requests from scripts/r02_channels.sh runs: one line
per run, the 16 channels' share of the kernel's read requests (volume_kernel /
cascade_kernel dispatches, all launches averaged) and max/mean."""
import csv
import glob
import os
import sys

out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "ch_*"))):
    if not os.path.isdir(d):
        continue
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    per = {}
    for r in csv.DictReader(open(files[0])):
        k = r["Kernel_Name"]
        if "volume_kernel" in k or "cascade_kernel" in k:
            per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    ch = [sum(per.get(f"AQZ_RDREQ_CH{k}", [0])) for k in range(16)]
    tot = sum(ch) or 1
    if len([c for c in ch if c]) < 3:
        print(os.path.basename(d), {k: v for k, v in per.items()})
        continue
    share = [c / tot * 16 for c in ch]
    print(f"{os.path.basename(d):14s} max/mean {max(share):.2f} min/mean {min(share):.2f} | "
          + " ".join(f"{s:.2f}" for s in share))
