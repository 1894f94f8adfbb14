"""The reference's own harness and test sources type-check against the drop-in.

VERDICT r04 item 4: `g++ -std=c++17 -fsyntax-only -I include/ref -I tests/stubs`
over /root/reference/bench/*_benchmark.cc and the reference's gtest files, so that
every dsp:: name, signature and include path they use exists in include/ref +
include/crlot_dsp.hpp.  tests/stubs holds minimal syntax stubs of the two test
frameworks (benchmark/benchmark.h, gtest/gtest.h) -- not of the reference.  The
reference files are read where they lie and never copied; the test is skipped
where /root/reference is absent (the GPU box).
"""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
BENCH = ["e2e", "performance", "ola", "micro_fft", "kernels", "micro_kernels"]
TESTS = ["framer", "ola_accumulator", "fft", "kernels", "window_lut", "norm_builder", "frame_queue",
         "wav_io", "window", "ring_buffer", "base"]
FILES = [f"bench/{b}_benchmark.cc" for b in BENCH] + [f"tests/{t}_test.cc" for t in TESTS]


def _syntax(rel):
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-I" + os.path.join(ROOT, "include", "ref"), "-I" + os.path.join(ROOT, "tests", "stubs"),
           os.path.join(REF, rel)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    return rel, r.returncode, r.stderr


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "bench")), reason="reference sources absent")
def test_reference_bench_and_test_sources_typecheck_against_dropin():
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        results = list(ex.map(_syntax, FILES))
    bad = [(rel, err) for rel, rc, err in results if rc != 0]
    msg = "\n\n".join(f"{rel}:\n" + "\n".join(l for l in err.splitlines() if "error" in l)[:3000] for rel, err in bad)
    assert not bad, msg
