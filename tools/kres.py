"""Per-kernel register / scratch table from hipcc's resource-usage remarks.

    python tools/kres.py factormodeling_amd/csrc/ts_ops.hip [name-filter ...]

Compiles one source with the Makefile's flags plus -Rpass-analysis=kernel-resource-usage
and prints VGPRs, AGPRs, spilled VGPRs, scratch bytes/lane, LDS and occupancy per kernel
(demangled).  Used to check "0 scratch for every launched instantiation" (VERDICT r3).
"""
from __future__ import annotations

import re
import subprocess
import sys

FLAGS = [*__import__("os").environ.get("KRES_DEFS", "").split(), "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
         "-Wno-unused-function", "-munsafe-fp-atomics"]


def main():
    src = sys.argv[1]
    filt = sys.argv[2:]
    p = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-c", src, "-o", "/tmp/_kres.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    if p.returncode:
        sys.stderr.write(p.stderr)
        sys.exit(p.returncode)
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        txt = m.group(1).strip()
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*\)$", "", n)
        if filt and not any(f in n for f in filt):
            continue
        print(f"{n:70s} vgpr={r.get('VGPRs', '?'):>4s} agpr={r.get('AGPRs', '?'):>3s} "
              f"spillV={r.get('VGPRs Spill', '?'):>3s} scratch={r.get('ScratchSize [bytes/lane]', '?'):>4s} "
              f"lds={r.get('LDS Size [bytes/block]', '?'):>6s} occ={r.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
