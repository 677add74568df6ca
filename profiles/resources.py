"""Per-kernel VGPR / scratch / LDS / occupancy from hipcc -Rpass-analysis=kernel-resource-usage.
Usage: python profiles/resources.py [regex]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "chameleon-rag-acceleration_amd", "csrc", "ivfpq_kernels.hip")


def main(rx=".*"):
    out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                          "-I" + os.path.join(REPO, "include"), "-c", SRC, "-o", "/tmp/_res.o",
                          "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split()[0]] = int(m.group(2))
    for r in rows:
        n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        n = n.replace("chivf::(anonymous namespace)::", "")
        if re.search(rx, n):
            print(f"{n[:70]:70s} vgpr={r.get('VGPRs')} scratch={r.get('ScratchSize')} lds={r.get('LDS')} occ={r.get('Occupancy')}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else ".*")
