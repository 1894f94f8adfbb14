"""The reference's own gtest suites of its device-backed components -- IFftPlan
(fft_test.cc), OLAAccumulator (ola_accumulator_test.cc, 1290 lines), the OLA
kernels (kernels_test.cc, dispatch_debug_test.cc) and FrameQueue
(frame_queue_test.cc) -- compiled unchanged against the drop-in headers and run
against the MI355X library on the GPU (tests/reftests/Makefile builds them in
the build container from /root/reference; the binaries travel with the tree)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_reference_sources import BIN, run_suite  # noqa: E402

DEVICE_SUITES = ["fft", "ola_accumulator", "kernels", "frame_queue", "dispatch_debug"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", DEVICE_SUITES)
def test_reference_device_suite_passes_against_dropin(torch_cuda, name):
    if not os.path.exists(os.path.join(BIN, name)):
        pytest.skip("reference suites not built")
    s = run_suite(name)
    print(f"\n{name}: {s}")
    assert s["rc"] == 0 and s["failed"] == 0 and s["tests"] > 0, s
