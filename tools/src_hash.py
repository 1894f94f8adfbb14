"""Source hashes of the library (test / measurement infrastructure and build step).

lib_hash(): every file libcrlot_dsp.so is built from -- crlot-dsp_amd/csrc/*.hip,
*.h, *.cpp, its Makefile and include/crlot_dsp.h.  The Makefile bakes it into
the library (crlot_build_info()); bench.py and smoke() compare the loaded
library's value with the tree's, so a stale prebuilt .so is caught.
kernel_hash(): the device sources and the Makefile only (bench.py src_hash()):
the key of the PMC summaries in profiles/ (host-only changes keep it).
Run as a script: prints lib_hash() (the Makefile's use)."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "crlot-dsp_amd", "csrc")


def _digest(files) -> str:
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def kernel_hash() -> str:
    return _digest(sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                          [os.path.join(CSRC, "Makefile")]))


def lib_hash() -> str:
    return _digest(sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                          glob.glob(os.path.join(CSRC, "*.cpp")) + [os.path.join(CSRC, "Makefile")]) +
                   [os.path.join(ROOT, "include", "crlot_dsp.h")])


if __name__ == "__main__":
    print(lib_hash())
