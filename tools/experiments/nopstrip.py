"""Experiment (not part of the release build): drop the `s_nop 0` hipcc pads
between two plain VALU instructions in a device .s (LLVM's gfx950 dst-sel
forwarding hazard model treats every inline-asm VOP3P as a producer that needs
one wait state).  Pads next to permlane / readlane / DPP / SALU / memory
instructions, and every `s_nop N` with N > 0, stay.
usage: python nopstrip.py in.s out.s  -> prints the count removed"""
import re
import sys

PLAIN = re.compile(r"^\s*v_(pk_fma_f32|pk_add_f32|pk_mul_f32|fma_f32|fmac_f32_e32|add_f32_e32|sub_f32_e32|"
                   r"mul_f32_e32|min3_f32|max3_f32|min_f32_e32|max_f32_e32)\b")
BAD = re.compile(r"dpp|row_|quad_perm|permlane|readlane|readfirstlane|writelane")


def real(lines, i, step):
    while 0 <= i < len(lines):
        s = lines[i].strip()
        if s and not s.startswith(";") and not s.startswith(".") and not s.endswith(":"):
            return s
        i += step
    return ""


def main(src, dst):
    lines = open(src).read().split("\n")
    out, n = [], 0
    for i, l in enumerate(lines):
        if l.strip() == "s_nop 0":
            p, q = real(lines, i - 1, -1), real(lines, i + 1, 1)
            if PLAIN.match(p) and PLAIN.match(q) and not BAD.search(p) and not BAD.search(q):
                n += 1
                continue
        out.append(l)
    open(dst, "w").write("\n".join(out))
    print(n)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
