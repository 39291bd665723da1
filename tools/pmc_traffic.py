"""Per-launch HBM traffic of the libfmx kernels from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py --fetch DIR_FETCH --write DIR_WRITE --dims D,A,F --out FILE.json

Inputs are the ``run_counter_collection.csv`` files of a FETCH_SIZE pass and a WRITE_SIZE
pass over tools/kbench.py (run separately: the two counters do not fit one pass).
FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE under-reads wide streaming
loads (MI355X_MICROARCH.md, HBM section), so the read side is calibrated in the same run
on a kernel with a known read volume: the register-ring ts_mean kernel reads the panel
exactly once (D*A*F*8 bytes) with the same 8-B-per-lane coalesced pattern as the other
kernels.  traffic = fetch * scale + write, per launch.
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            per[name][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in per.items()}   # KiB per dispatch


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--fetch", required=True)
    p.add_argument("--write", required=True)
    p.add_argument("--dims", required=True, help="D,A,F of the profiled panel")
    p.add_argument("--out", required=True)
    a = p.parse_args()
    D, A, F = (int(x) for x in a.dims.split(","))
    fetch = load(a.fetch, "FETCH_SIZE")
    write = load(a.write, "WRITE_SIZE")
    panel = D * A * F * 8.0
    cal = [k for k in fetch if k.startswith("fmx::k_ts_reg<1,")]
    scale = panel / (fetch[cal[0]] * 1024.0) if cal else 2.0
    out = {"dims": [D, A, F], "panel_bytes": panel, "fetch_scale": scale,
           "fetch_scale_source": cal[0] if cal else "guide default (x2)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 1024.0
        wb = write.get(k, 0.0) * 1024.0
        out["kernels"][k] = {"fetch_bytes_raw": fb, "write_bytes": wb, "traffic_bytes": fb * scale + wb,
                             "traffic_per_unit": (fb * scale + wb) / (D * A * F)}
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in out["kernels"].items():
        print(f"{k:45s} {v['traffic_bytes'] / 1e9:9.2f} GB/launch  {v['traffic_per_unit']:6.2f} B/unit")
    print("fetch scale", scale)


if __name__ == "__main__":
    main()
