"""Per-kernel register / occupancy / spill table of the HIP sources, from the
compiler's kernel-resource-usage remarks (gfx950, the release flags).
usage: python tools/resources.py [SRC ...] [-D...]   (default: the pair walkers)
Prints one line per kernel; with two define sets separated by '--vs' prints both
side by side (e.g. -DCRLOT_PDFT16_CLASSIC --vs) so a change's register cost shows."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "crlot-dsp_amd", "csrc")
FLAGS = ["-std=c++17", "-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-slp-vectorize",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-c", "-o", "/dev/null",
         "-Rpass-analysis=kernel-resource-usage"]
ILP = {"pair1k", "pair_any", "pair30"}


def usage(src, defs):
    cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + defs + [os.path.join(CSRC, src + ".hip")]
    if src in ILP:
        cmd += ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    res, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"remark: +([A-Za-z][\w \[\]/]*?): (\S+) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2)
        if key == "Function Name":
            cur = res.setdefault(val, {})
        elif cur is not None:
            cur[key] = val
    return res


def short(name):
    m = re.match(r"_ZN5crlot2fk\d+(\w+?)I(.*)EEvNS0_9FusedArgsE", name)
    return (m.group(1) + "<" + m.group(2) + ">") if m else name


def main():
    args = sys.argv[1:]
    sets, cur, srcs = [], [], []
    for a in args:
        if a == "--vs":
            sets.append(cur)
            cur = []
        elif a.startswith("-D"):
            cur.append(a)
        else:
            srcs.append(a)
    sets.append(cur)
    srcs = srcs or ["pair1k", "pair_hot", "pair_any"]
    for src in srcs:
        tabs = [usage(src, d) for d in sets]
        for k in sorted(tabs[0]):
            cols = []
            for t in tabs:
                u = t.get(k, {})
                cols.append("v%-3s s%-3s occ%s sp%s/%s" % (u.get("VGPRs"), u.get("TotalSGPRs"),
                                                         u.get("Occupancy [waves/SIMD]"),
                                                         u.get("VGPRs Spill"), u.get("SGPRs Spill")))
            print("%-9s %-58s %s" % (src, short(k)[:58], " | ".join(cols)))


if __name__ == "__main__":
    main()
