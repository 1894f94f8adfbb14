"""The INTEGRATION.md IFftPlan backend compiles against the reference's own
interface header (dsp/fft/api/fft_api.h), i.e. it is a drop-in for MakeFftPlan.
Build container only (the reference tree is not on the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "dsp/fft/api/fft_api.h")),
                    reason="reference tree not present")
def test_hip_adapter_compiles_against_reference_interface():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
                        "-I/opt/rocm/include", f"-I{REF}", f"-I{ROOT}/include",
                        os.path.join(ROOT, "integration", "hip_adapter.cc")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
