"""Group a rocprofv3 --kernel-trace CSV by (kernel, grid): calls and average
kernel-only duration.  Usage: python scripts/kernel_by_grid.py TRACE.csv"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"aqz::\(anonymous namespace\)::|\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*$", "", name)          # drop the argument list
    return name


def main(path):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            n = short(r["Kernel_Name"])
            if n.startswith("at::"):
                continue
            key = (n, int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))
            acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("kernel\tgrid_x\tgrid_y\tcalls\tavg_us")
    for (n, gx, gy), v in sorted(acc.items()):
        print(f"{n}\t{gx}\t{gy}\t{len(v)}\t{sum(v) / len(v):.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
