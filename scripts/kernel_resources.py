#!/usr/bin/env python3
"""Per-kernel resource table from the compiler's own accounting (CPU only).

Compiles a .hip source for gfx950 with -Rpass-analysis=kernel-resource-usage
and tabulates, per kernel instantiation: VGPRs, AGPRs, SGPRs, LDS bytes per
workgroup, scratch, and the occupancy the compiler computes (waves per SIMD,
from registers alone), plus the occupancy LDS allows at the kernel's
workgroup size (160 KB per CU).  VERDICT r5 weak #1 asked for these figures
next to the PMC wait breakdown of the flagship families.

    python scripts/kernel_resources.py native/kernels/conv_gemm.hip --match conv_pro,conv23,conv_glds
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
LDS_PER_CU = 160 * 1024


def demangle(names: list[str]) -> dict[str, str]:
    try:
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return dict(zip(names, out))
    except (OSError, subprocess.CalledProcessError):
        return {n: n for n in names}


def resources(src: Path) -> list[dict]:
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           f"-I{REPO / 'native' / 'include'}", "-c", str(src), "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    names = demangle([r["name"] for r in rows])
    for r in rows:
        r["pretty"] = names[r["name"]]
    return rows


def threads_of(pretty: str) -> int:
    # launch bounds are not in the remarks; the families' block sizes
    if "conv23_kernel" in pretty or "conv_big" in pretty or "conv_halo" in pretty:
        m = re.search(r"conv23_kernel<(\d+), (\d+)", pretty)
        if m and int(m.group(1)) * int(m.group(2)) >= 128 * 128:
            return 512
        return 512 if ("conv_big" in pretty or "conv_halo" in pretty) else 256
    return 256


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="+")
    ap.add_argument("--match", default="", help="comma list of substrings of kernel names to keep")
    a = ap.parse_args(argv)
    keep = [s for s in a.match.split(",") if s]
    print("| kernel | VGPR | AGPR | SGPR | LDS B/WG | scratch | waves/SIMD (regs) | WG/CU by LDS |")
    print("|---|---|---|---|---|---|---|---|")
    for s in a.src:
        for r in resources(Path(s)):
            p = r["pretty"]
            if keep and not any(k in p for k in keep):
                continue
            lds = int(r.get("LDS Size [bytes/block]", 0))
            by_lds = LDS_PER_CU // lds if lds else "-"
            short = re.sub(r"\(anonymous namespace\)::", "", p)
            short = short.split("(")[0][:70]
            print(f"| `{short}` | {r.get('VGPRs')} | {r.get('AGPRs')} | {r.get('TotalSGPRs')} | {lds} | "
                  f"{r.get('ScratchSize [bytes/lane]')} | {r.get('Occupancy [waves/SIMD]')} | {by_lds} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
