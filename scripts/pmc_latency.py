"""Summaries of scripts/r06_vdec_pmc.sh (measurement aid, not product code).

ch_* runs: the 16 TCC channels' share of the kernel's read requests
(1.00 = even).  lat_* runs, per kernel and grid (dispatches averaged): read
requests leaving the L2, requests in flight summed over cycles
(TCC_EA0_RDREQ_LEVEL), their ratio — the mean number of TCC cycles a read
waits for its data (Little's law) — and the DRAM credit stall cycles per
request."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    return list(csv.DictReader(open(files[0]))) if files else []


def short(k):
    for tag in ("volume_kernel", "cascade_band_kernel", "cascade_kernel", "rows_kernel", "mix_kernel"):
        if tag in k:
            return tag
    return k.split("(")[0][-40:]


for d in sorted(glob.glob(os.path.join(out, "*"))):
    if not os.path.isdir(d):
        continue
    name = os.path.basename(d)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows(d):
        key = (short(r["Kernel_Name"]), r.get("Grid_Size", "?"))
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if name.startswith("ch_"):
        for key, c in per.items():
            if not key[0].startswith(("volume", "cascade")):
                continue
            ch = [sum(c.get(f"AQZ_RDREQ_CH{k}", [0])) for k in range(16)]
            tot = sum(ch) or 1
            share = [x / tot * 16 for x in ch]
            print(f"{name:14s} {key[0]:20s} max/mean {max(share):.3f} min/mean {min(share):.3f} | "
                  + " ".join(f"{s:.2f}" for s in share))
    else:
        for key, c in sorted(per.items()):
            n = len(c.get("TCC_EA0_RDREQ_sum", []))
            if not n:
                continue
            req = sum(c["TCC_EA0_RDREQ_sum"]) / n
            lvl = sum(c.get("TCC_EA0_RDREQ_LEVEL_sum", [0])) / n
            stall = sum(c.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", [0])) / n
            cyc = sum(c.get("TCC_CYCLE_sum", [0])) / n
            if req < 1e5:
                continue
            print(f"{name:14s} {key[0]:20s} grid {key[1]:>10s} x{n:<3d} rdreq {req:12.0f} "
                  f"wait/req {lvl / req:7.1f} cyc  stall/req {stall / req:6.3f}  "
                  f"in-flight/chan {lvl / cyc * 1.0 if cyc else 0:6.2f}  cyc {cyc:.3g}")


def probe_cases(d):
    """lat_probe: tools/pitch_probe.py --set volume runs, per case in
    volume_cases() order, nt x (16:5 mix, read-only) x (3 warm + reps)
    dispatches; the per-case means (both mixes) of the counters above."""
    import csv as _csv
    names = [f"plane{w}_{k}" for w in (512, 1024, 2048, 4096) for k in ("all_rows", "decimate")]
    per = collections.OrderedDict()
    for r in rows(d):
        if "rows_kernel" not in r["Kernel_Name"]:
            continue
        per.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = list(per.values())
    n = len(disp) // len(names)
    for i, name in enumerate(names):
        for half, load in ((0, "nt"), (1, "plain")):
            g = disp[i * n + half * n // 2: i * n + (half + 1) * n // 2]
            req = sum(x["TCC_EA0_RDREQ_sum"] for x in g) / len(g)
            lvl = sum(x["TCC_EA0_RDREQ_LEVEL_sum"] for x in g) / len(g)
            st = sum(x["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] for x in g) / len(g)
            print(f"probe {name:20s} {load:5s} rdreq {req:10.0f} wait/req {lvl / req:7.1f} cyc  "
                  f"stall/req {st / req:6.3f}")


if len(sys.argv) > 2 and sys.argv[2] == "--probe-cases":
    probe_cases(os.path.join(out, "lat_probe"))
