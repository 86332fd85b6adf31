"""Per-kernel register / scratch / occupancy table of a HIP source (hipcc
-Rpass-analysis=kernel-resource-usage), optionally diffed against another tree.

    python scripts/kernel_resources.py imagent_amd/csrc/kernels/conv_igemm.hip [--old OLD.hip] [--grep igemm]
"""
import argparse
import re
import subprocess


def resources(src):
    r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/dev/null",
                        "-munsafe-fp-atomics", "-Rpass-analysis=kernel-resource-usage"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    out, cur = {}, None
    for line in r.stdout.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]"
                      r"|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = v
            out[cur] = {}
        elif cur:
            out[cur][k if k.endswith("Spill") else k.split(" ")[0]] = v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--old")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    new = resources(a.src)
    old = resources(a.old) if a.old else {}
    for k, v in sorted(new.items()):
        if a.grep not in k:
            continue
        o = old.get(k)
        f = lambda d: f"vgpr {d.get('VGPRs')} scratch {d.get('ScratchSize')} occ {d.get('Occupancy')}"  # noqa
        print(f"{f(o) + '  ->  ' if o else ''}{f(v)}  {k[:110]}")


if __name__ == "__main__":
    main()
