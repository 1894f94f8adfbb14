"""Flags __builtin_bit_cast applied directly to an element of a vector value.

ROCm 7.2 clang miscompiles __builtin_bit_cast(T, v.x) / (T, v[i]) when v is an
ext_vector_type (HIP float2/float4, our `pc`, the b64/b128 buffer-load results):
it read a single dword of a b64 load and, in round 4, the
wrong element of a register pair (commit 8b3b77b, NaN samples went unflagged).
Copying the element to a scalar first is correct, so the rule is mechanical:
the operand of a bit cast must not be a vector element.

What counts as a vector element (on the source text, every #if branch at once):
  * NAME.x / .y / .z / .w (vector swizzles; our structs have no such fields);
  * NAME[i]...[j] with one subscript more than NAME's array rank, where NAME is
    declared with a vector type (pc, float2/3/4, int2/4, uint2/4, u2, or a typedef
    with ext_vector_type in the same file);
  * a subscript applied to a call's result (f(...)[i]).
Function-like macros defined in the file are expanded (every definition of the
name, so both sides of an #if are checked) before the operand is classified.

usage: python tools/bitcast_lint.py [FILE ...]   (default: crlot-dsp_amd/csrc/**)
exit status 1 when anything is flagged."""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VEC_TYPES = {"pc", "float2", "float3", "float4", "int2", "int4", "uint2", "uint4", "u2", "u4", "double2"}


def _balanced(s, i):
    """index just past the parenthesis group opening at s[i] == '('"""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j + 1
    return len(s)


def _split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return [a.strip() for a in out]


def _macros(text):
    macs = {}
    for m in re.finditer(r"^[ \t]*#\s*define\s+(\w+)\(([^)]*)\)[ \t]+(.*?)$", text, re.M):
        params = [p.strip() for p in m.group(2).split(",") if p.strip()]
        macs.setdefault(m.group(1), []).append((params, m.group(3).strip()))
    return macs


def _decls(text):
    """name -> [(offset, rank or None)]: every declaration of the name, vector ones
    with their array rank, scalar ones (float, int, ...) as None; a use takes the
    nearest declaration before it (a crude scope)."""
    types = set(VEC_TYPES)
    for m in re.finditer(r"typedef\s+[\w\s]+?\b(\w+)\s*__attribute__\s*\(\(\s*ext_vector_type", text):
        types.add(m.group(1))
    decls = {}
    tpat = "|".join(sorted(map(re.escape, types)))
    for m in re.finditer(r"\b(?:" + tpat + r")\b\s*[&*]?\s*(\w+)\s*((?:\[[^\]]*\])*)\s*(?=[;=,){])", text):
        decls.setdefault(m.group(1), []).append((m.start(), m.group(2).count("[")))
    for m in re.finditer(r"\bauto\s+(\w+)\s*=\s*__builtin_amdgcn_raw_buffer_load_b(?:64|96|128)\b", text):
        decls.setdefault(m.group(1), []).append((m.start(), 0))
    spat = r"\b(?:float|double|int|unsigned|uint32_t|int32_t|uint64_t|int64_t|bool|half)\b"
    for m in re.finditer(spat + r"\s+(\w+)\s*((?:\[[^\]]*\])*)\s*(?=[;=,){])", text):
        decls.setdefault(m.group(1), []).append((m.start(), None))
    for v in decls.values():
        v.sort()
    return decls


def _rank_at(decls, name, pos):
    best = None
    for off, rank in decls.get(name, []):
        if off < pos:
            best = (rank,)
    return None if best is None else best[0]


def _expand(arg, macs, depth=0):
    m = re.match(r"^(\w+)\s*\((.*)\)$", arg, re.S)
    if depth > 4 or not m or m.group(1) not in macs:
        return [arg]
    args = _split_args(m.group(2))
    outs = []
    for params, body in macs[m.group(1)]:
        if len(params) != len(args):
            continue
        b = body
        for p, a in zip(params, args):
            b = re.sub(r"\b" + re.escape(p) + r"\b", "(" + a + ")", b)
        outs += _expand(b.strip(), macs, depth + 1)
    return outs or [arg]


def _is_vector_element(expr, decls, pos):
    e = re.sub(r"\s+", "", expr)
    while e.startswith("(") and _balanced(e, 0) == len(e):
        e = e[1:-1]
    if re.search(r"\.(x|y|z|w)$", e):
        return True
    m = re.match(r"^(\w+)((?:\[.+\])+)$", e)
    if m:
        n_sub, depth = 0, 0
        for ch in m.group(2):
            if ch == "[":
                if depth == 0:
                    n_sub += 1
                depth += 1
            elif ch == "]":
                depth -= 1
        rank = _rank_at(decls, m.group(1), pos)
        return rank is not None and n_sub > rank
    return bool(re.match(r"^[\w:]+\(.*\)\[[^\]]+\]$", e))


def lint_text(text, path="<text>"):
    macs, decls = _macros(text), _decls(text)
    found = []
    for m in re.finditer(r"__builtin_bit_cast\s*\(", text):
        end = _balanced(text, m.end() - 1)
        args = _split_args(text[m.end():end - 1])
        if len(args) != 2:
            continue
        for e in _expand(args[1], macs):
            if _is_vector_element(e, decls, m.start()):
                line = text.count("\n", 0, m.start()) + 1
                found.append((path, line, args[1] if e == args[1] else f"{args[1]} -> {e}"))
                break
    return found


def lint_files(paths):
    found = []
    for p in paths:
        with open(p) as f:
            found += lint_text(f.read(), os.path.relpath(p, ROOT))
    return found


def default_paths():
    c = os.path.join(ROOT, "crlot-dsp_amd", "csrc")
    pats = ["*.h", "*.hip", "experiments/*.h", "experiments/*.hip", "experiments/*.inc"]
    return sorted(p for pat in pats for p in glob.glob(os.path.join(c, pat)))


if __name__ == "__main__":
    hits = lint_files(sys.argv[1:] or default_paths())
    for path, line, what in hits:
        print(f"{path}:{line}: __builtin_bit_cast on a vector element: {what}")
    sys.exit(1 if hits else 0)
