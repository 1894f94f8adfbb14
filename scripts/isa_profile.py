"""ISA histogram of the main loops of the round-trip kernels (gfx950 device
assembly compiled here): profiles/<tag>_isa_hist.json.  Per kernel: the loop's
instruction classes and the VALU count per frame pair, the figure the headline
kernel's VALU-issue bound is priced in.
usage: python scripts/isa_profile.py rNN"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "crlot-dsp_amd", "csrc")
FLAGS = ["-std=c++17", "-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-slp-vectorize",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-S"]

# (source, mangled-name substring, frame pairs per loop iteration, label)
KERNELS = [
    ("pair1k.hip", "k_stft_ola_pairILi4ELi4ELi4ELb0ELb0EEE", 4, "K_pair 1024/256 (headline)"),
    ("pair_hot.hip", "k_pair_wg_hotINS0_12_GLOBAL__N_15Geo4kELi4ELi4ELb0EEE", 4, "K_pair4k hot 4096/1024 (config 3)"),
    ("pair_hot.hip", "k_pair512_hotILi2ELi4ELi4EEE", None, "K_pair512 hot 512/128"),
    ("pair_any.hip", "k_pair15_hotILi64ELi4ELb0E", None, "K_pair15 960/240"),
    ("pair_any.hip", "k_pair15_hotILi32ELi2ELb0E", None, "K_pair15 480/120"),
]


def loop_hist(asm, pat):
    m = re.search(r"^(_Z\w*" + re.escape(pat) + r"\w*):.*?\n(.*?)\n\s*s_endpgm", asm, re.S | re.M)
    if not m:
        return None, None
    body = m.group(2).split("\n")
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
    loops = []
    for i, l in enumerate(body):
        mm = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            loops.append((labels[mm.group(1)], i))
    a, b = max(loops, key=lambda t: t[1] - t[0])
    c = collections.Counter()
    skip = False  # inside a frexp_min_if fallback: skipped unless the output screen fails
    for l in body[a:b + 1]:
        t = l.strip().split()
        if not t:
            continue
        if t[0] == "s_cbranch_vccz" and ".Lfx_skip" in l:
            skip = True
        elif t[0].startswith(".Lfx_skip"):
            skip = False
        if t and not t[0].startswith((".", ";")):
            c[("fallback:" if skip and t[0] != "s_cbranch_vccz" else "") + t[0]] += 1
    return m.group(1), c


def src_hash() -> str:
    """bench.py's src_hash: the kernel sources and the Makefile (the histogram
    describes that build only)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                    [os.path.join(CSRC, "Makefile")]):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    out = {"tag": tag, "src_hash": src_hash(), "note": "main loop = the longest backward branch span of the kernel; "
           "counts are static instructions in it (every one issues once per iteration), except the "
           "exact sanitize test inside the frexp_min_if asm blocks, which runs only when the output "
           "screen fails (loop_valu_fallback_skipped, not in loop_valu)", "kernels": []}
    asm_cache = {}
    with tempfile.TemporaryDirectory() as td:
        for src, pat, pairs, label in KERNELS:
            if src not in asm_cache:
                s_path = os.path.join(td, src + ".s")
                extra = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"] if src == "pair1k.hip" else []  # as the Makefile
                subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, os.path.join(CSRC, src), "-o", s_path],
                               check=True, capture_output=True)
                asm_cache[src] = open(s_path).read()
            name, c = loop_hist(asm_cache[src], pat)
            if c is None:
                print("not found:", pat, file=sys.stderr)
                continue
            fb = sum(v for k, v in c.items() if k.startswith("fallback:v_"))
            c = collections.Counter({k: v for k, v in c.items() if not k.startswith("fallback:")})
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            pk = sum(v for k, v in c.items() if k.startswith("v_pk_"))
            perm = sum(v for k, v in c.items() if "permlane" in k)
            rec = {"label": label, "symbol": name, "loop_valu": valu, "loop_packed": pk,
                   "loop_permlane": perm,
                   "loop_lds": sum(v for k, v in c.items() if k.startswith("ds_")),
                   "loop_barriers": c.get("s_barrier", 0),
                   "loop_salu": sum(v for k, v in c.items() if k.startswith("s_")),
                   "loop_vmem": sum(v for k, v in c.items() if k.startswith(("buffer_", "global_"))),
                   "loop_valu_fallback_skipped": fb,
                   "top": dict(c.most_common(30))}
            if pairs:
                rec["pairs_per_iteration"] = pairs
                rec["valu_per_pair"] = round(valu / pairs, 1)
            out["kernels"].append(rec)
            print(f"{label:40s} VALU {valu:5d} packed {pk:5d} permlane {perm:4d}"
                  + (f"  per pair {valu / pairs:.1f}" if pairs else ""))
    path = os.path.join(ROOT, "profiles", f"{tag}_isa_hist.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
