"""Source checks that need no GPU.

The bit-cast rule (tools/bitcast_lint.py): ROCm 7.2 clang miscompiles
__builtin_bit_cast applied directly to an element of a vector value; it bit the
project twice (commit 8b3b77b, NaN samples unflagged by the
hop check).  The tree must be clean, and the linter must catch the pattern that
shipped before 8b3b77b (a macro expanding to a subscript of a register-pair array).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bitcast_lint as BL  # noqa: E402


def test_no_bit_cast_of_vector_elements_in_tree():
    hits = BL.lint_files(BL.default_paths())
    assert not hits, "\n".join(f"{p}:{l}: {w}" for p, l, w in hits)


# The shape of the round-4 regression (pair1k.hip before 8b3b77b), restated.
PRE_8B3B77B = """
typedef float pc __attribute__((ext_vector_type(2)));
#if CRLOT_PAIR_PKX
    dev::pc xr2[R / 2][SH];
#define XR(s, q) xr2[(s) / 2][q][(s) % 2]
#else
    float xr[R][SH];
#define XR(s, q) xr[s][q]
#endif
    auto slot_ok = [&](auto sc, int at) {
        for (int q = 0; q < SH; ++q) {
            const uint32_t u = __builtin_bit_cast(uint32_t, XR(s, q)) & 0x7fffffffu;
        }
    };
"""


@pytest.mark.parametrize("snippet,bad", [
    (PRE_8B3B77B, True),
    ("float2 v; unsigned a = __builtin_bit_cast(unsigned, v.x);", True),
    ("auto v = __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0); float f = __builtin_bit_cast(float, v[1]);", True),
    ("pc v[16]; float f = __builtin_bit_cast(float, v[3][1]);", True),
    ("float h[4]; unsigned u = __builtin_bit_cast(unsigned, h[2]);", False),
    ("float2 v; const float lo = v.x; unsigned u = __builtin_bit_cast(unsigned, lo);", False),
    ("pc v[16]; pc w = __builtin_bit_cast(pc, v[3]);", False),
])
def test_linter_classifies(snippet, bad):
    assert bool(BL.lint_text(snippet)) == bad


def test_linter_flags_the_pre_fix_source_from_history():
    """The real pre-8b3b77b pair1k.hip, when the git history is at hand."""
    try:
        src = subprocess.run(["git", "-C", ROOT, "show", "8b3b77b^:crlot-dsp_amd/csrc/pair1k.hip"],
                             capture_output=True, text=True, timeout=30)
    except (OSError, subprocess.TimeoutExpired):
        pytest.skip("git unavailable")
    if src.returncode != 0:
        pytest.skip("history not available")
    hits = BL.lint_text(src.stdout, "pair1k.hip@8b3b77b^")
    assert any("XR(s, q)" in w for _, _, w in hits), hits
