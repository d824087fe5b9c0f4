#!/usr/bin/env python3
"""Per-kernel register / spill / LDS / occupancy table of a HIP translation unit
for gfx950, from the compiler's kernel-resource-usage remarks (no GPU needed).

  python tools/resource_usage.py [toymeshpathtracer_amd/csrc/tmpt_render.hip] [filter]

Compiles with the library's own flags (csrc/Makefile) into /tmp, so a code
change can be checked for register pressure and spills before a GPU run."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "toymeshpathtracer_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
         f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}", "-O2", "-fno-slp-vectorize"]
KEYS = ("VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
        "Occupancy [waves/SIMD]", "LDS Size [bytes/block]")


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.splitlines()
        return [o.split("(")[0] for o in out]
    except Exception:
        return names


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(CSRC, "tmpt_render.hip")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    extra = os.environ.get("EXTRA", "").split()
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-x", "hip", "-c", src, "-o", "/tmp/_ru.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        sys.exit(r.returncode)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass-analysis", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None and k in KEYS:
            cur[k] = v
    names = demangle([x["name"] for x in rows])
    print(f"{'kernel':<100} {'VGPR':>5} {'SGPR':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'occ':>4} {'LDS':>6}")
    for x, n in zip(rows, names):
        if filt and filt not in n:
            continue
        print(f"{n[:100]:<100} {x.get('VGPRs', '?'):>5} {x.get('SGPRs', '?'):>5} {x.get('VGPRs Spill', '?'):>6} "
              f"{x.get('SGPRs Spill', '?'):>6} {x.get('ScratchSize [bytes/lane]', '?'):>7} "
              f"{x.get('Occupancy [waves/SIMD]', '?'):>4} {x.get('LDS Size [bytes/block]', '?'):>6}")


if __name__ == "__main__":
    main()
