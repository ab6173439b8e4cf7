"""Markdown table of every BASELINE config x method from a closing sweep's
bench lines (scripts/r06_final.sh writes <dir>/m_<workload>_<method>.json):
µs per launch, frames per launch, GPix/s, fraction of the 8 TB/s spec,
fraction of the same-mix ceiling, PMC traffic / algorithmic bytes, and the
buffer sets the launch rotated over.  DESIGN.md §0 carries its output."""
import json
import os
import sys

WORKLOADS = [("4096x4096_u16", "H 4096² u16, 5 levels (headline)"),
             ("4096x4096_f32", "F 4096² f32, 5 levels"),
             ("1024x1024x256_u16", "V 1024²×256 u16, 3 levels, 4 volumes"),
             ("v1", "V, one volume per launch"),
             ("2048x2048_u16", "C2 2048² u16, 4 levels"),
             ("512x512_u8", "C1b 512² u8, 3 levels")]
METHODS = ["decimate", "mean", "min", "max"]


def row(d):
    r = d["roofline"]
    ceil = (r.get("same_mix_ceiling") or {}).get("frac_of_ceiling")
    traffic = r.get("traffic")
    alg = r.get("alg_bytes_per_launch")
    tr = f"{traffic / alg:.4f}" if traffic and alg else "—"
    sets = r.get("buffer_sets", 1)
    return (f"{r['avg_launch_us']:.1f}", str(d["config"].get("frames_per_step_per_gpu", "?")),
            f"{d['value']:.0f}", f"{r['frac']:.3f}",
            f"{ceil:.2f}" if ceil else "—", tr, str(sets), d["config"].get("check", "?"))


def main():
    out = sys.argv[1]
    print("| Config | Method | µs per launch | frames | GPix/s | of spec | of ceiling | traffic | buffer sets | check |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for w, label in WORKLOADS:
        for i, m in enumerate(METHODS):
            p = os.path.join(out, f"v1_{m}.json" if w == "v1" else f"m_{w}_{m}.json")
            if not os.path.exists(p):
                continue
            try:
                d = json.load(open(p))
            except ValueError:
                continue
            cells = row(d)
            print(f"| {label if i == 0 else ''} | {m.capitalize()} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
